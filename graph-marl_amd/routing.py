"""Batched routing environment with the reference's NetworkEnv API.

Mirrors `Network` + `Routing` (reference src/env/network.py:42-389,
src/env/routing.py:43-552) for `n_env` independent graph instances resident in
HBM. Every method returns torch tensors on the GPU with a leading env dimension;
the arithmetic runs in the HIP kernels of libgraphmarl_amd.so (gm_env_*).
Per-env behaviour is bit-identical to the reference given the same numpy seed.
"""
import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import _lib as L

# the fused DQN reads the GEMM-ready copy of the agent rows (K = 6N+8) instead of the env obs (K = 6N+10)
GEMM_OBS = True

EVAL_SEEDS = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "eval_seeds.npy"))


class Discrete:
    """Stand-in for gymnasium.spaces.Discrete as the reference uses it (.n only)."""

    def __init__(self, n, start=0):
        self.n, self.start = n, start


@dataclass
class Network:
    """Topology configuration (reference Network.__init__, src/env/network.py:47-98).

    Seeds are resolved exactly like the reference: a fixed topology seed, a list of
    `n_random_seeds` valid seeds built from `topology_init_seed` (device
    build_seed_list), provided seeds, or a fresh random seed per reset."""

    n_nodes: int = 20
    random_topology: bool = False
    n_random_seeds: Optional[int] = None
    sequential_topology_seeds: bool = False
    topology_init_seed: int = 476
    excluded_seeds: Optional[List[int]] = None
    provided_seeds: Optional[List[int]] = None
    device: int = 0
    seeds: List[int] = field(default_factory=list)

    def __post_init__(self):
        if self.n_nodes % 2:
            raise ValueError("n_nodes must be even (random 3-regular topologies)")
        if self.provided_seeds is not None and len(self.provided_seeds) > 0:
            self.seeds = list(self.provided_seeds)
        elif not self.random_topology:
            self.seeds = [self.topology_init_seed]
        elif self.n_random_seeds is None or self.n_random_seeds <= 0:
            self.seeds = []
        else:
            self.seeds = build_seed_list(self.n_nodes, self.topology_init_seed, self.n_random_seeds,
                                         self.excluded_seeds, self.device)
        if self.excluded_seeds is not None:
            ex = set(int(s) for s in self.excluded_seeds)
            assert all(int(s) not in ex for s in self.seeds)

    def mode(self):
        if not self.random_topology and not (self.provided_seeds and len(self.provided_seeds) > 0):
            return L.TOPO_FIXED, self.topology_init_seed, None
        if len(self.seeds) == 0:
            return L.TOPO_RANDOM, self.topology_init_seed, None
        if self.sequential_topology_seeds and len(self.seeds) > 1:
            return L.TOPO_SEQUENTIAL, self.topology_init_seed, self.seeds
        return L.TOPO_LIST, self.topology_init_seed, self.seeds


def build_seed_list(n_nodes, init_seed, count, excluded=None, device=0):
    """Network.build_seed_list (src/env/network.py:100-120), computed on the GPU."""
    L.require_gpu()
    out = np.zeros(count, dtype=np.int64)
    ex = None if excluded is None else np.ascontiguousarray(np.sort(np.asarray(excluded, np.int64)))
    L.check(L.lib().gm_build_seed_list(n_nodes, init_seed, count, None if ex is None else ex.ctypes.data,
                                       0 if ex is None else len(ex), device, out.ctypes.data))
    return [int(s) for s in out]


class Routing:
    """n_env routing environments (reference Routing, src/env/routing.py:43).

    :param network: topology configuration (`Network`)
    :param n_data: packets (agents) per env
    :param env_var: environment variant: 1 INDEPENDENT, 2 WITH_K_NEIGHBORS (+5k columns),
        3 GLOBAL (+ flattened I+A and node observations)
    :param k: neighbour slots of variant 2 (reference default 3)
    :param n_env: number of parallel graph instances
    :param seeds: per-env numpy-legacy seeds (default: seed + env index)
    :param obs_extra: extra zero columns reserved after each agent observation (the
        NetMon wrapper writes its 4H graph features there, fusing the reference's concat)
    :param agent_adjacency: compute the agent adjacency every step (the reference
        returns it from step(); the DQN ignores it, the hot path turns it off)
    """

    def __init__(self, network: Network, n_data=20, env_var=1, k=3, enable_congestion=True,
                 enable_action_mask=False, ttl=0, n_env=1, seeds=None, seed=0, obs_extra=0,
                 agent_adjacency=True, device=None):
        L.require_gpu()
        self.network = network
        self.n_data = n_data
        self.n_env = n_env
        self.env_var = env_var
        self.k = k
        self.enable_congestion = enable_congestion
        self.enable_action_mask = enable_action_mask
        self.ttl = ttl
        self.action_space = Discrete(4, start=0)
        self.agent_adjacency = agent_adjacency
        self.device = torch.device("cuda", network.device if device is None else device)
        self.eval_info_enabled = False
        mode, tseed, lst = network.mode()
        cfg = L.EnvConfig()
        cfg.n_env, cfg.n_nodes, cfg.n_data, cfg.env_var = n_env, network.n_nodes, n_data, int(env_var)
        cfg.k = int(k)
        cfg.congestion, cfg.action_mask, cfg.ttl = int(enable_congestion), int(enable_action_mask), int(ttl)
        cfg.topo_mode, cfg.topo_seed = mode, int(tseed)
        self._keep = []
        if lst is not None:
            arr = np.ascontiguousarray(np.asarray(lst, np.int64))
            self._keep.append(arr)
            cfg.seed_list, cfg.n_seed_list = arr.ctypes.data_as(C.POINTER(C.c_int64)), len(arr)
        if network.excluded_seeds is not None:
            ex = np.ascontiguousarray(np.sort(np.asarray(network.excluded_seeds, np.int64)))
            self._keep.append(ex)
            cfg.excluded, cfg.n_excluded = ex.ctypes.data_as(C.POINTER(C.c_int64)), len(ex)
        cfg.device = self.device.index or 0
        if seeds is None:
            seeds = [(seed + i) & 0xFFFFFFFF for i in range(n_env)]
        seeds_arr = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        assert len(seeds_arr) == n_env
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            L.check(L.lib().gm_env_create(C.byref(cfg), seeds_arr.ctypes.data, C.byref(h)))
        self._h = h
        N, A = network.n_nodes, n_data
        self.n_nodes = N
        dims = [C.c_int32() for _ in range(5)]
        L.check(L.lib().gm_env_dims(h, *[C.byref(x) for x in dims]))
        self.obs_dim = dims[3].value  # 6N+10 (+5k variant 2, +N^2+N(4N+8) variant 3)
        self.node_obs_dim = 4 * N + 8
        self.obs_stride = ((self.obs_dim + obs_extra + 3) // 4) * 4
        dev = self.device
        # persistent device buffers (filled in place by the kernels; no allocation per step)
        self.obs_buf = torch.zeros(n_env, A, self.obs_stride, device=dev)
        self.node_obs = torch.zeros(n_env, N, self.node_obs_dim, device=dev)
        self.agent_node = torch.zeros(n_env, A, dtype=torch.int32, device=dev)
        self.agent_adj = torch.zeros(n_env, A, A, dtype=torch.int8, device=dev)
        self.reward = torch.zeros(n_env, A, device=dev)
        self.done = torch.zeros(n_env, A, dtype=torch.uint8, device=dev)
        self.info = torch.zeros(n_env, L.GM_INFO_FIELDS, dtype=torch.float64, device=dev)
        self.nbr = torch.zeros(n_env, N, 3, dtype=torch.int32, device=dev)
        self._actions = torch.zeros(n_env, A, dtype=torch.int32, device=dev)
        self.obs_gemm = None  # GEMM-ready env obs copy (enable_gemm_obs)
        self._lazy_obs = False  # kernels write only obs_gemm; obs rows rebuilt on demand (set_lazy_obs)
        self._obs_stale = False
        self._has_state = False
        self._obsbufs = self._make_obsbufs(self.agent_adjacency)

    # -- plumbing ---------------------------------------------------------------
    def _make_obsbufs(self, adj):
        o = L.ObsBuffers()
        o.obs = None if (self._lazy_obs and self.obs_gemm is not None) else self.obs_buf.data_ptr()
        o.obs_row_stride = self.obs_stride
        o.node_obs = self.node_obs.data_ptr()
        o.agent_node = self.agent_node.data_ptr()
        o.agent_adj = self.agent_adj.data_ptr() if adj else None
        if self.obs_gemm is not None:
            o.obs_gemm = self.obs_gemm.data_ptr()
            o.obs_gemm_stride = self.obs_gemm.stride(1)
        return o

    def enable_gemm_obs(self):
        """Have every reset / step / observe also write the GEMM-ready copy of the agent rows
        (gm_obs_buffers.obs_gemm: 6N+8 columns, the two linearly dependent ones dropped) that the
        fused DQN's first layer reads with K = 6N+8. Variant 1 only."""
        if self.obs_gemm is not None or self.env_var != 1 or not GEMM_OBS:
            return self.obs_gemm
        self.obs_gemm = torch.zeros(self.n_env, self.n_data, 6 * self.n_nodes + 8, device=self.device)
        self._obsbufs = self._make_obsbufs(self.agent_adjacency)
        if self._has_state:  # fill it for the current state
            L.check(L.lib().gm_env_observe(self._h, C.byref(self._obsbufs), self._stream()))
        return self.obs_gemm

    def set_lazy_obs(self, on=True):
        """on: every reset / step writes only the GEMM-ready copy (one HBM copy of the agent rows per
        step instead of two), and reading .obs rebuilds the reference rows from it
        (gm_obs_from_gemm, bit-identical). For rollouts whose DQN reads obs_gemm and that do not
        store every step's obs (benchmarks, evaluation). Needs enable_gemm_obs(); returns whether
        the mode is on."""
        if on and self.obs_gemm is None:
            return False
        if self._lazy_obs and not on:
            self.sync_obs()
        self._lazy_obs = bool(on)
        self._obsbufs = self._make_obsbufs(self.agent_adjacency)
        return self._lazy_obs

    def mark_obs_stale(self):
        """The env kernels that just ran (step_ / reset_, or a replayed HIP graph) wrote only the GEMM-ready
        rows: in lazy mode the obs rows are rebuilt on the next read. Call it on the stream those kernels
        ran on: it records an event there, and sync_obs orders the rebuild after it (the reader's stream
        may differ, e.g. StreamedRollout's group streams)."""
        if self._lazy_obs:
            self._obs_stale = True
            if not torch.cuda.is_current_stream_capturing():
                ev = self._obs_ev = getattr(self, "_obs_ev", None) or torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))

    def sync_obs(self):
        """Rebuild the agent obs rows from the GEMM-ready copy if the last kernels wrote only that."""
        if self._obs_stale:
            ev = getattr(self, "_obs_ev", None)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
            L.check(L.lib().gm_obs_from_gemm(self.obs_gemm.data_ptr(), self.obs_gemm.stride(1),
                                             self.n_env * self.n_data, self.n_nodes, self.obs_buf.data_ptr(),
                                             self.obs_stride, self._stream()))
            self._obs_stale = False

    def _stream(self):
        return L.stream_ptr(self.device)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().gm_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def obs(self):
        """agent observations [n_env, A, 6N+10] (view of the persistent buffer)."""
        self.sync_obs()
        return self.obs_buf[..., : self.obs_dim]

    def __str__(self):
        return (f"Routing environment (graph-marl_amd, {self.n_env} parallel envs)\n"
                f"> Network: {self.n_nodes} nodes\n> Number of packets: {self.n_data}\n"
                f"> Congestion: {self.enable_congestion}\n> Action mask: {self.enable_action_mask}\n"
                f"> TTL: {self.ttl if self.ttl > 0 else 'disabled'}")

    # -- NetworkEnv API -----------------------------------------------------------
    def set_eval_info(self, val):
        """Enable the eval-only step statistics (routing.py:414-441) in step()'s info."""
        self.eval_info_enabled = bool(val)
        if self.eval_info_enabled and not hasattr(self, "eval_stats"):
            self.eval_stats = torch.zeros(self.n_env, L.GM_EVAL_FIELDS, dtype=torch.float64, device=self.device)

    def set_topology_seeds(self, seeds, sequential=True, interleave=False):
        """network.seeds = seeds; network.sequential_topology_seeds = sequential (the reference's
        switch to EVAL_SEEDS before evaluation, src/main.py:553-560). interleave: env b starts at
        seeds[b] and advances by n_env (n_env envs walk the list like consecutive episodes)."""
        seeds = [int(x) for x in seeds]
        self.network.seeds = seeds
        self.network.sequential_topology_seeds = sequential
        mode, tseed, lst = self.network.mode()
        arr = None if lst is None else np.ascontiguousarray(np.asarray(lst, np.int64))
        L.check(L.lib().gm_env_set_topology(self._h, mode, int(tseed), None if arr is None else arr.ctypes.data,
                                            0 if arr is None else len(arr), int(interleave)))

    def reset_(self, mask=None):
        """Reset envs in place (mask: bool/uint8 [n_env] on device, None = all)."""
        m = None if mask is None else mask.to(torch.uint8)
        with L.timed("env_reset"):
            L.check(L.lib().gm_env_reset(self._h, L.ptr(m), C.byref(self._obsbufs), self._stream()))
        self._has_state = True
        self.mark_obs_stale()
        L.check(L.lib().gm_env_topology(self._h, L.ptr(self.nbr), None, None, None, self._stream()))

    def reset(self):
        """Routing.reset (routing.py:160-178) for every env -> (obs, agent adjacency)."""
        self.reset_()
        return self.obs, self.agent_adj

    def step_(self, actions, detail=None):
        """Routing.step in place; results in self.obs/reward/done/info."""
        a = actions
        if a.dtype != torch.int32 or not a.is_contiguous():
            self._actions.copy_(a)
            a = self._actions
        det = self._detail(detail)
        with L.timed("env_step"):
            L.check(L.lib().gm_env_step(self._h, L.ptr(a), L.ptr(self.reward), L.ptr(self.done), L.ptr(self.info),
                                        None if det is None else C.byref(det), C.byref(self._obsbufs),
                                        self._stream()))
        self.mark_obs_stale()

    def policy_step_(self, q, epsilon, actions, detail=None):
        """egreedy(q, epsilon, actions) then step_(actions) as one kernel (gm_env_policy_step):
        identical draws, actions and results; q [n_env, A, 4] contiguous, actions int32 [n_env, A]."""
        assert q.is_contiguous() and actions.dtype == torch.int32 and actions.is_contiguous()
        det = self._detail(detail)
        with L.timed("env_step"):
            L.check(L.lib().gm_env_policy_step(self._h, L.ptr(q), float(epsilon), L.ptr(actions), L.ptr(self.reward),
                                               L.ptr(self.done), L.ptr(self.info),
                                               None if det is None else C.byref(det), C.byref(self._obsbufs),
                                               self._stream()))
        self.mark_obs_stale()
        return actions

    def _detail(self, detail):
        det = None
        if detail is not None or self.eval_info_enabled:
            det = L.StepDetail()
            if detail is not None:
                det.done_steps, det.done_opt, det.success = (detail["done_steps"].data_ptr(),
                                                             detail["done_opt"].data_ptr(),
                                                             detail["success"].data_ptr())
            if self.eval_info_enabled:
                det.eval = self.eval_stats.data_ptr()
        return det

    def step(self, act):
        """Routing.step (routing.py:360-520) -> (obs, adj, reward, done, info) with a
        leading env dim; info holds per-env sums (see _lib.INFO_KEYS)."""
        if not torch.is_tensor(act):
            act = torch.as_tensor(np.asarray(act), device=self.device)
        self.step_(act.to(self.device))
        info = {k: self.info[:, i] for i, k in enumerate(L.INFO_KEYS)}
        if self.eval_info_enabled:
            info.update({k: self.eval_stats[:, i] for i, k in enumerate(L.EVAL_KEYS)})
        return self.obs, self.agent_adj, self.reward, self.done.bool(), info

    def egreedy(self, q, epsilon, actions):
        """EpsilonGreedy draws (src/policy.py:44-50) from each env's stream; q [n_env, A, 4]."""
        with L.timed("egreedy"):
            L.check(L.lib().gm_policy_egreedy(self._h, L.ptr(q), float(epsilon), L.ptr(actions),
                                              L.stream_ptr(self.device)))
        return actions

    def shortest_path_actions(self, actions):
        """ShortestPath policy (src/policy.py:90-139) for every packet of every env."""
        with L.timed("shortest_path"):
            L.check(L.lib().gm_policy_shortest_path(self._h, L.ptr(actions), L.stream_ptr(self.device)))
        return actions

    def get_nodes_adjacency(self):
        out = torch.empty(self.n_env, self.n_nodes, self.n_nodes, dtype=torch.int8, device=self.device)
        L.check(L.lib().gm_env_topology(self._h, None, L.ptr(out), None, None, self._stream()))
        return out

    def get_node_observation(self):
        return self.node_obs

    def get_node_aux(self):
        out = torch.empty(self.n_env, self.n_nodes, self.n_nodes, device=self.device)
        L.check(L.lib().gm_env_topology(self._h, None, None, L.ptr(out), None, self._stream()))
        return out

    def get_node_agent_matrix(self):
        m = torch.zeros(self.n_env, self.n_nodes, self.n_data, dtype=torch.int8, device=self.device)
        m.scatter_(1, self.agent_node.long().unsqueeze(1), 1)
        return m

    def get_topology_seeds(self):
        out = torch.empty(self.n_env, dtype=torch.int64, device=self.device)
        L.check(L.lib().gm_env_topology(self._h, None, None, None, L.ptr(out), self._stream()))
        return out

    def final_info(self):
        """[n_env, 2] float64: sum and count of the non-zero agent steps (get_final_info)."""
        out = torch.empty(self.n_env, 2, dtype=torch.float64, device=self.device)
        L.check(L.lib().gm_env_final_info(self._h, L.ptr(out), self._stream()))
        return out

    def get_final_info(self, info):
        """Routing.get_final_info: adds the still-running packets' steps to the delays."""
        out = self.final_info()
        info = dict(info)
        info["sum_delays"] = info["sum_delays"] + out[:, 0]
        info["n_delays"] = info["n_delays"] + out[:, 1]
        return info

    def observe(self):
        lazy, self._lazy_obs = self._lazy_obs, False
        try:  # every buffer, the obs rows included
            L.check(L.lib().gm_env_observe(self._h, C.byref(self._make_obsbufs(True)), self._stream()))
        finally:
            self._lazy_obs = lazy
        self._obs_stale = False

    def get_num_agents(self):
        return self.n_data

    def get_num_nodes(self):
        return self.n_nodes

    def get(self):
        return self

    # -- parity / debugging ---------------------------------------------------------
    def get_state(self):
        """Copy the full env state to host numpy arrays (synchronous)."""
        B, A, N, E = self.n_env, self.n_data, self.n_nodes, 3 * self.n_nodes // 2
        arrs = dict(
            now=np.zeros((B, A), np.int32), target=np.zeros((B, A), np.int32), edge=np.zeros((B, A), np.int32),
            time=np.zeros((B, A), np.int32), ttl=np.zeros((B, A), np.int32), start=np.zeros((B, A), np.int32),
            spw=np.zeros((B, A), np.int32), agent_steps=np.zeros((B, A), np.int32),
            size=np.zeros((B, A), np.float64), visited=np.zeros((B, A, 2), np.uint64),
            amask=np.zeros((B, A, 4), np.uint8), loads=np.zeros((B, E), np.float64),
            topo_seed=np.zeros(B, np.int64), topo_reps=np.zeros(B, np.int32), edge_a=np.zeros((B, E), np.int32),
            edge_b=np.zeros((B, E), np.int32), edge_len=np.zeros((B, E), np.int32),
            nbr_edge=np.zeros((B, N, 3), np.int32), apsp=np.zeros((B, N, N), np.int32),
            rng_key=np.zeros((B, 624), np.uint32), rng_pos=np.zeros(B, np.int32), seq_index=np.zeros(B, np.int32),
        )
        st = L.EnvState()
        for k, v in arrs.items():
            setattr(st, k, v.ctypes.data)
        torch.cuda.synchronize(self.device)
        L.check(L.lib().gm_env_get_state(self._h, C.byref(st)))
        return arrs

    def set_state(self, arrs):
        """Restore a get_state() dump (gm_env_set_state) and re-emit the observations; keys
        missing from `arrs` keep their current device values."""
        B, A, N, E = self.n_env, self.n_data, self.n_nodes, 3 * self.n_nodes // 2
        shapes = dict(now=(B, A), target=(B, A), edge=(B, A), time=(B, A), ttl=(B, A), start=(B, A), spw=(B, A),
                      agent_steps=(B, A), size=(B, A), visited=(B, A, 2), amask=(B, A, 4), loads=(B, E),
                      topo_seed=(B,), topo_reps=(B,), edge_a=(B, E), edge_b=(B, E), edge_len=(B, E),
                      nbr_edge=(B, N, 3), apsp=(B, N, N), rng_key=(B, 624), rng_pos=(B,), seq_index=(B,))
        dtypes = dict(size=np.float64, loads=np.float64, visited=np.uint64, amask=np.uint8, topo_seed=np.int64,
                      rng_key=np.uint32)
        st = L.EnvState()
        keep = []
        for k, shp in shapes.items():
            if k not in arrs:
                continue
            a = np.ascontiguousarray(np.asarray(arrs[k], dtype=dtypes.get(k, np.int32)).reshape(shp))
            keep.append(a)
            setattr(st, k, a.ctypes.data)
        torch.cuda.synchronize(self.device)
        L.check(L.lib().gm_env_set_state(self._h, C.byref(st)))
        self._has_state = True
        self.observe()
        L.check(L.lib().gm_env_topology(self._h, L.ptr(self.nbr), None, None, None, self._stream()))
        torch.cuda.synchronize(self.device)

    @property
    def action_mask(self):
        return torch.as_tensor(self.get_state()["amask"].astype(bool), device=self.device)
