"""Batched SimpleEnvironment on the device (reference src/env/simple_environment.py:45-334).

Three routers on a line, one packet at the middle router choosing one of its two edges;
reward = score (-1/+1) of the router reached, done every step. n_env independent
instances, each with its own numpy-legacy stream (seeds[env]) that reproduces the
reference's global-stream draws (reset: scores, positions, edge order; ε-greedy:
randint(2) + rand(1)). Same NetworkEnv surface as `Routing`, with a leading env dim.
"""
import ctypes as C

import numpy as np
import torch

from . import _lib as L
from .routing import Discrete


class SimpleObs(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("obs_row_stride", C.c_int64), ("node_obs", C.c_void_p),
                ("node_adj", C.c_void_p), ("nbr", C.c_void_p), ("agent_node", C.c_void_p)]


class SimpleState(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("score", "router_edge", "edge_end", "start", "now")]


def _bind():
    lib = L.lib()
    if not getattr(lib, "_simple_ready", False):
        vp, i32 = C.c_void_p, C.c_int32
        lib.gm_simple_create.argtypes = [i32, i32, i32, vp, i32, C.POINTER(vp)]
        lib.gm_simple_destroy.argtypes = [vp]
        lib.gm_simple_reset.argtypes = [vp, vp, C.POINTER(SimpleObs), vp]
        lib.gm_simple_step.argtypes = [vp, vp, vp, vp, C.POINTER(SimpleObs), vp]
        lib.gm_simple_observe.argtypes = [vp, C.POINTER(SimpleObs), vp]
        lib.gm_simple_policy_egreedy.argtypes = [vp, vp, C.c_double, vp, vp]
        lib.gm_simple_get_state.argtypes = [vp, C.POINTER(SimpleState)]
        lib._simple_ready = True
    return lib


class SimpleEnvironment:
    """:param env_var: 1 = INDEPENDENT (obs [now]); 2/3 add the adjacency and scores
    :param random_topology: randomise node ids and edge order (simple_environment.py:129-190)
    :param seeds: per-env numpy-legacy seeds (default seed + env index)
    :param obs_extra: zero columns reserved after the observation (NetMon graph features)"""

    n_router = 3
    n_data = 1

    def __init__(self, env_var=1, random_topology=True, n_env=1, seeds=None, seed=0, obs_extra=0, device=None):
        L.require_gpu()
        self.env_var = int(env_var)
        self.random_topology = bool(random_topology)
        self.n_env = n_env
        self.n_nodes = 3
        self.action_space = Discrete(2, start=0)
        self.enable_action_mask = False
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        if seeds is None:
            seeds = [(seed + i) & 0xFFFFFFFF for i in range(n_env)]
        s = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        assert len(s) == n_env
        lib = _bind()
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            L.check(lib.gm_simple_create(n_env, self.env_var, int(self.random_topology), s.ctypes.data,
                                         self.device.index or 0, C.byref(h)))
        self._h = h
        self.obs_dim = 1 if self.env_var == 1 else 1 + 9 + 3
        self.node_obs_dim = 1
        self.obs_stride = ((self.obs_dim + obs_extra + 3) // 4) * 4
        dev = self.device
        self.obs_buf = torch.zeros(n_env, 1, self.obs_stride, device=dev)
        self.node_obs = torch.zeros(n_env, 3, 1, device=dev)
        self.node_adj = torch.zeros(n_env, 3, 3, dtype=torch.int8, device=dev)
        self.nbr = torch.zeros(n_env, 3, 2, dtype=torch.int32, device=dev)
        self.agent_node = torch.zeros(n_env, 1, dtype=torch.int32, device=dev)
        self.agent_adj = torch.ones(n_env, 1, 1, dtype=torch.int8, device=dev)
        self.reward = torch.zeros(n_env, 1, device=dev)
        self.done = torch.zeros(n_env, 1, dtype=torch.uint8, device=dev)
        self._actions = torch.zeros(n_env, 1, dtype=torch.int32, device=dev)
        o = SimpleObs()
        o.obs, o.obs_row_stride = self.obs_buf.data_ptr(), self.obs_stride
        o.node_obs, o.node_adj = self.node_obs.data_ptr(), self.node_adj.data_ptr()
        o.nbr, o.agent_node = self.nbr.data_ptr(), self.agent_node.data_ptr()
        self._o = o

    def close(self):
        if getattr(self, "_h", None):
            _bind().gm_simple_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __str__(self):
        return (f"SimpleEnvironment (graph-marl_amd, {self.n_env} parallel envs) with parameters\n"
                f"> Environment variant: {self.env_var}\n> Random topology: {self.random_topology}")

    @property
    def obs(self):
        return self.obs_buf[..., : self.obs_dim]

    # -- NetworkEnv API ---------------------------------------------------------------
    def reset_(self, mask=None):
        m = None if mask is None else mask.to(torch.uint8)
        with L.timed("env_reset"):
            L.check(_bind().gm_simple_reset(self._h, L.ptr(m), C.byref(self._o), L.stream_ptr(self.device)))

    def reset(self):
        self.reset_()
        return self.obs, self.agent_adj

    def step_(self, actions, detail=None):
        a = actions
        if a.dtype != torch.int32 or not a.is_contiguous() or a.dim() != 2:
            self._actions.copy_(a.reshape(self.n_env, 1))
            a = self._actions
        with L.timed("env_step"):
            L.check(_bind().gm_simple_step(self._h, L.ptr(a), L.ptr(self.reward), L.ptr(self.done),
                                           C.byref(self._o), L.stream_ptr(self.device)))

    def step(self, act):
        if not torch.is_tensor(act):
            act = torch.as_tensor(np.asarray(act), device=self.device)
        self.step_(act.to(self.device))
        return self.obs, self.agent_adj, self.reward, self.done.bool(), {}

    def egreedy(self, q, epsilon, actions):
        """EpsilonGreedy draws (src/policy.py:44-50) from each env's stream; q [n_env, 1, 2]."""
        assert q.shape[-1] == 2 and q.is_contiguous()
        L.check(_bind().gm_simple_policy_egreedy(self._h, L.ptr(q), float(epsilon), L.ptr(actions),
                                                 L.stream_ptr(self.device)))
        return actions

    def get_nodes_adjacency(self):
        return self.node_adj

    def get_node_observation(self):
        return self.node_obs

    def get_node_aux(self):
        return None

    def get_node_agent_matrix(self):
        m = torch.zeros(self.n_env, 3, 1, dtype=torch.int8, device=self.device)
        m.scatter_(1, self.agent_node.long().unsqueeze(1), 1)
        return m

    def get_final_info(self, info):
        return info

    def set_eval_info(self, val):
        pass

    def get_num_agents(self):
        return 1

    def get_num_nodes(self):
        return 3

    def get(self):
        return self

    def get_state(self):
        """Host copy of the env state (synchronous): score, router_edge, edge_end, start, now."""
        B = self.n_env
        arrs = dict(score=np.zeros((B, 3), np.int32), router_edge=np.zeros((B, 3, 2), np.int32),
                    edge_end=np.zeros((B, 2, 2), np.int32), start=np.zeros(B, np.int32), now=np.zeros(B, np.int32))
        st = SimpleState()
        for k, v in arrs.items():
            setattr(st, k, v.ctypes.data)
        torch.cuda.synchronize(self.device)
        L.check(_bind().gm_simple_get_state(self._h, C.byref(st)))
        return arrs
