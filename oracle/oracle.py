"""ctypes wrapper around the C oracle (gm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the parity checker / CPU baseline. The product
path (graph-marl_amd) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libgm_oracle.so")

MAXN, MAXA = 128, 256
MAXE = MAXN * 3 // 2
TOPO_FIXED, TOPO_RANDOM, TOPO_LIST, TOPO_SEQUENTIAL = 0, 1, 2, 3


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class MT(C.Structure):
    _fields_ = [("key", C.c_uint32 * 624), ("pos", C.c_int32)]


class Topo(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("n_edges", C.c_int32),
        ("x", C.c_double * MAXN), ("y", C.c_double * MAXN),
        ("deg", C.c_int32 * MAXN),
        ("neighbors", (C.c_int32 * 3) * MAXN),
        ("node_edges", (C.c_int32 * 3) * MAXN),
        ("nbr", (C.c_int32 * 3) * MAXN),
        ("edge_a", C.c_int32 * MAXE), ("edge_b", C.c_int32 * MAXE), ("edge_len", C.c_int32 * MAXE),
        ("apsp", (C.c_int32 * MAXN) * MAXN),
        ("seed", C.c_int64), ("repetitions", C.c_int32),
    ]

    def arrays(self):
        n, E = self.n, self.n_edges
        return dict(
            n=n, E=E, seed=int(self.seed), repetitions=int(self.repetitions),
            pos=np.stack([np.ctypeslib.as_array(self.x)[:n], np.ctypeslib.as_array(self.y)[:n]], -1),
            edges=np.stack([np.ctypeslib.as_array(self.edge_a)[:E], np.ctypeslib.as_array(self.edge_b)[:E],
                            np.ctypeslib.as_array(self.edge_len)[:E]], -1).astype(np.int64),
            neighbors=np.ctypeslib.as_array(self.neighbors)[:n].astype(np.int64),
            node_edges=np.ctypeslib.as_array(self.node_edges)[:n].astype(np.int64),
            nbr=np.ctypeslib.as_array(self.nbr)[:n].astype(np.int64),
            apsp=np.ctypeslib.as_array(self.apsp)[:n, :n].astype(np.int64),
        )


class Config(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int32), ("n_data", C.c_int32),
        ("congestion", C.c_int32), ("action_mask", C.c_int32), ("ttl", C.c_int32),
        ("topo_mode", C.c_int32), ("topo_seed", C.c_int64),
        ("seed_list", C.POINTER(C.c_int64)), ("n_seed_list", C.c_int32),
        ("excluded", C.POINTER(C.c_int64)), ("n_excluded", C.c_int32),
        ("env_var", C.c_int32), ("k", C.c_int32),
    ]


class Env(C.Structure):
    _fields_ = [
        ("cfg", Config), ("rng", MT), ("topo", Topo), ("seq_index", C.c_int32),
        ("now", C.c_int32 * MAXA), ("target", C.c_int32 * MAXA), ("edge", C.c_int32 * MAXA),
        ("time", C.c_int32 * MAXA), ("ttl", C.c_int32 * MAXA), ("start", C.c_int32 * MAXA),
        ("spw", C.c_int32 * MAXA), ("size", C.c_double * MAXA),
        ("visited", (C.c_uint64 * 2) * MAXA), ("agent_steps", C.c_double * MAXA),
        ("load", C.c_double * MAXE), ("amask", (C.c_uint8 * 4) * MAXA),
        ("neigh_cnt", C.c_int32 * MAXA), ("neigh", (C.c_int16 * MAXA) * MAXA),
    ]


class Info(C.Structure):
    _fields_ = [
        ("looped", C.c_double), ("throughput", C.c_int32), ("dropped", C.c_int32), ("blocked", C.c_int32),
        ("n_delays", C.c_int32), ("n_arrived", C.c_int32),
        ("delays", C.c_double * MAXA), ("delays_arrived", C.c_double * MAXA), ("spr", C.c_double * MAXA),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.gmo_mt_seed.argtypes = [C.POINTER(MT), C.c_uint32]
        L.gmo_mt_next32.argtypes = [C.POINTER(MT)]
        L.gmo_mt_next32.restype = C.c_uint32
        L.gmo_mt_random.argtypes = [C.POINTER(MT)]
        L.gmo_mt_random.restype = C.c_double
        L.gmo_mt_randint.argtypes = [C.POINTER(MT), C.c_int64]
        L.gmo_mt_randint.restype = C.c_int64
        L.gmo_obs_dim_cfg.argtypes = [C.POINTER(Config)]
        L.gmo_create_valid.argtypes = [C.POINTER(Topo), C.POINTER(Config), C.POINTER(MT), C.c_int32]
        L.gmo_create_valid.restype = C.c_int64
        L.gmo_build_seed_list.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.POINTER(C.c_int64), C.c_int32,
                                          C.POINTER(C.c_int64)]
        L.gmo_env_sizeof.restype = C.c_size_t
        L.gmo_env_init.argtypes = [C.POINTER(Env), C.POINTER(Config), C.c_uint32]
        L.gmo_env_reset.argtypes = [C.POINTER(Env)]
        L.gmo_env_step.argtypes = [C.POINTER(Env), C.POINTER(C.c_int32), C.POINTER(C.c_float),
                                   C.POINTER(C.c_uint8), C.POINTER(Info)]
        L.gmo_env_observe.argtypes = [C.POINTER(Env), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.gmo_env_final_delays.argtypes = [C.POINTER(Env), C.POINTER(C.c_double), C.POINTER(C.c_int32)]
        L.gmo_bench_rollout.argtypes = [C.POINTER(Config), C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                        C.c_void_p, C.c_void_p]
        L.gmo_bench_rollout.restype = C.c_double
        assert L.gmo_env_sizeof() == C.sizeof(Env), "oracle struct layout mismatch"
        _lib = L
    return _lib


class MTStream:
    """numpy legacy RandomState restated in C."""

    def __init__(self, seed):
        self.s = MT()
        lib().gmo_mt_seed(C.byref(self.s), C.c_uint32(seed & 0xFFFFFFFF))

    def next32(self):
        return lib().gmo_mt_next32(C.byref(self.s))

    def random(self):
        return lib().gmo_mt_random(C.byref(self.s))

    def randint(self, high):
        return lib().gmo_mt_randint(C.byref(self.s), high)

    @property
    def key(self):
        return np.ctypeslib.as_array(self.s.key).copy()


def make_config(n_nodes, n_data, congestion=True, action_mask=False, ttl=0, topo_mode=TOPO_FIXED,
                topo_seed=476, seed_list=None, excluded=None, env_var=1, k=3):
    cfg = Config()
    cfg.n_nodes, cfg.n_data = n_nodes, n_data
    cfg.env_var, cfg.k = int(env_var), int(k)
    cfg.congestion, cfg.action_mask, cfg.ttl = int(congestion), int(action_mask), int(ttl)
    cfg.topo_mode, cfg.topo_seed = topo_mode, topo_seed
    keep = []
    if seed_list is not None:
        arr = np.ascontiguousarray(np.asarray(seed_list, dtype=np.int64))
        keep.append(arr)
        cfg.seed_list = arr.ctypes.data_as(C.POINTER(C.c_int64))
        cfg.n_seed_list = len(arr)
    if excluded is not None:
        arr = np.ascontiguousarray(np.sort(np.asarray(excluded, dtype=np.int64)))
        keep.append(arr)
        cfg.excluded = arr.ctypes.data_as(C.POINTER(C.c_int64))
        cfg.n_excluded = len(arr)
    cfg._keep = keep
    return cfg


def create_valid(cfg, main_stream, seed_index=-1):
    t = Topo()
    s = lib().gmo_create_valid(C.byref(t), C.byref(cfg), C.byref(main_stream.s), seed_index)
    return s, t


def build_seed_list(n, init_seed, count, excluded=None):
    out = np.zeros(count, dtype=np.int64)
    if excluded is not None:
        ex = np.ascontiguousarray(np.sort(np.asarray(excluded, dtype=np.int64)))
        exp, nex = ex.ctypes.data_as(C.POINTER(C.c_int64)), len(ex)
    else:
        ex, exp, nex = None, None, 0
    lib().gmo_build_seed_list(n, init_seed, count, exp, nex, out.ctypes.data_as(C.POINTER(C.c_int64)))
    return out


class OracleEnv:
    """Single routing env instance restated in C (mirrors src/env/routing.py Routing)."""

    def __init__(self, cfg, seed):
        self.cfg = cfg
        self.e = Env()
        lib().gmo_env_init(C.byref(self.e), C.byref(cfg), C.c_uint32(seed & 0xFFFFFFFF))
        self.n, self.A = cfg.n_nodes, cfg.n_data

    @property
    def rng(self):
        s = MTStream.__new__(MTStream)
        s.s = self.e.rng
        return s

    def draw_egreedy(self, q, eps):
        """EpsilonGreedy.__call__ draws (src/policy.py:46-51) from this env's stream."""
        A = self.A
        ra = np.array([lib().gmo_mt_randint(C.byref(self.e.rng), 4) for _ in range(A)], dtype=np.int64)
        rf = np.array([lib().gmo_mt_random(C.byref(self.e.rng)) for _ in range(A)]) < eps
        return np.argmax(q, axis=-1) * ~rf + rf * ra

    def reset(self):
        lib().gmo_env_reset(C.byref(self.e))

    def step(self, actions):
        act = np.ascontiguousarray(np.asarray(actions, dtype=np.int32))
        rew = np.zeros(self.A, np.float32)
        done = np.zeros(self.A, np.uint8)
        info = Info()
        lib().gmo_env_step(C.byref(self.e), act.ctypes.data_as(C.POINTER(C.c_int32)),
                           rew.ctypes.data_as(C.POINTER(C.c_float)), done.ctypes.data_as(C.POINTER(C.c_uint8)),
                           C.byref(info))
        inf = dict(
            looped=info.looped, throughput=info.throughput, dropped=info.dropped, blocked=info.blocked,
            delays=list(np.ctypeslib.as_array(info.delays)[: info.n_delays]),
            delays_arrived=list(np.ctypeslib.as_array(info.delays_arrived)[: info.n_arrived]),
            spr=list(np.ctypeslib.as_array(info.spr)[: info.n_arrived]),
        )
        return rew, done.astype(bool), inf

    def obs_dim(self):
        return lib().gmo_obs_dim_cfg(C.byref(self.cfg))

    def observe(self):
        n, A = self.n, self.A
        obs = np.zeros((A, self.obs_dim()), np.float32)
        nobs = np.zeros((n, 4 * n + 8), np.float32)
        adj = np.zeros((A, A), np.int8)
        na = np.zeros((n, A), np.int8)
        aux = np.zeros((n, n), np.float32)
        lib().gmo_env_observe(C.byref(self.e), obs.ctypes.data, nobs.ctypes.data, adj.ctypes.data,
                              na.ctypes.data, aux.ctypes.data)
        return dict(obs=obs, node_obs=nobs, adj=adj, node_agent=na, aux=aux)

    def final_delays(self):
        out = np.zeros(self.A, np.float64)
        k = C.c_int32(0)
        lib().gmo_env_final_delays(C.byref(self.e), out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(k))
        return list(out[: k.value])

    def state(self):
        e, A = self.e, self.A
        E = e.topo.n_edges
        g = np.ctypeslib.as_array
        return dict(
            now=g(e.now)[:A].astype(np.int64), target=g(e.target)[:A].astype(np.int64),
            edge=g(e.edge)[:A].astype(np.int64), time=g(e.time)[:A].astype(np.int64),
            ttl=g(e.ttl)[:A].astype(np.int64), start=g(e.start)[:A].astype(np.int64),
            spw=g(e.spw)[:A].astype(np.int64), size=g(e.size)[:A].copy(),
            visited=g(e.visited)[:A].copy(), agent_steps=g(e.agent_steps)[:A].copy(),
            loads=g(e.load)[:E].copy(), amask=g(e.amask)[:A].copy(),
            topo_seed=int(e.topo.seed), rng_key=g(e.rng.key).copy(), rng_pos=int(e.rng.pos),
        )

    def topology(self):
        return self.e.topo.arrays()


def bench_rollout(cfg, n_env, steps, episode_steps, n_threads, write_obs=True):
    n, A = cfg.n_nodes, cfg.n_data
    obs = np.zeros((n_env, A, 6 * n + 10), np.float32) if write_obs else None
    nobs = np.zeros((n_env, n, 4 * n + 8), np.float32) if write_obs else None
    sec = lib().gmo_bench_rollout(C.byref(cfg), n_env, steps, episode_steps, n_threads,
                                  None if obs is None else obs.ctypes.data,
                                  None if nobs is None else nobs.ctypes.data)
    return sec, obs, nobs
