"""CPU baseline ("port") for bench.py: the oracle's C env (OpenMP over envs) plus a
NumPy fp32 restatement of NetMon + DQN ε-greedy, batched over envs — the same
workload as the GPU rollout step (env step + NetMon K iterations + DQN policy).

TEST/BASELINE INFRASTRUCTURE ONLY: used by bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import time

import numpy as np

import oracle as O


def _setup():
    L = O.lib()
    if not hasattr(L, "_batch_ready"):
        L.gmo_batch_create.argtypes = [C.POINTER(O.Config), C.c_int32, C.c_uint32]
        L.gmo_batch_create.restype = C.c_void_p
        L.gmo_batch_free.argtypes = [C.c_void_p]
        L.gmo_batch_run.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L._batch_ready = True
    return L


def _lrelu(x):
    return np.where(x >= 0, x, np.float32(0.01) * x)


def _sig(x):
    return np.float32(1) / (np.float32(1) + np.exp(-x))


class NumpyRollout:
    def __init__(self, n_env, n_nodes=20, n_data=20, H=128, enc=(512, 256), hidden=(512, 256), K=1,
                 episode_steps=50, eps=0.5, seed=0):
        self.L = _setup()
        self.B, self.N, self.A, self.H, self.K, self.ep = n_env, n_nodes, n_data, H, K, episode_steps
        ev = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                                  "eval_seeds.npy"))
        self.cfg = O.make_config(n_nodes, n_data, topo_mode=O.TOPO_RANDOM, excluded=ev)
        self.envs = self.L.gmo_batch_create(C.byref(self.cfg), n_env, 1000)
        rng = np.random.default_rng(seed)
        D, ND = 6 * n_nodes + 10, 4 * n_nodes + 8
        self.D = D
        self.stride = D + 4 * H

        def lin(i, o):
            s = 1 / np.sqrt(i)
            return (rng.uniform(-s, s, (o, i)).astype(np.float32), rng.uniform(-s, s, o).astype(np.float32))

        dims = [ND, *enc, H]
        self.enc = [lin(dims[i], dims[i + 1]) for i in range(len(dims) - 1)]
        self.lstm = [lin(2 * H, 4 * H) for _ in range(2)]
        qd = [self.stride, *hidden]
        self.dqn = [lin(qd[i], qd[i + 1]) for i in range(len(qd) - 1)] + [lin(hidden[-1], 4)]
        self.obs = np.zeros((n_env, n_data, self.stride), np.float32)
        self.nobs = np.zeros((n_env, n_nodes, ND), np.float32)
        self.an = np.zeros((n_env, n_data), np.int32)
        self.nbr = np.zeros((n_env, n_nodes, 3), np.int32)
        self.rew = np.zeros((n_env, n_data), np.float32)
        self.done = np.zeros((n_env, n_data), np.uint8)
        self.state = np.zeros((n_env * n_nodes, 2 * H), np.float32)
        self.eps = eps
        self.rng = np.random.default_rng(seed + 1)
        self.t = 0

    def _env(self, reset, act):
        self.L.gmo_batch_run(self.envs, self.B, int(reset), None if act is None else act.ctypes.data,
                             self.rew.ctypes.data, self.done.ctypes.data, self.obs.ctypes.data, self.stride,
                             self.nobs.ctypes.data, self.an.ctypes.data, self.nbr.ctypes.data)

    def _lstm(self, w, x, h, c):
        g = np.concatenate([x, h], -1) @ w[0].T + w[1]
        H = self.H
        i, f, gg, o = _sig(g[:, :H]), _sig(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), _sig(g[:, 3 * H:])
        c1 = f * c + i * gg
        return o * np.tanh(c1), c1

    def _netmon(self):
        B, N, H = self.B, self.N, self.H
        x = self.nobs.reshape(B * N, -1)
        for w, b in self.enc:
            x = _lrelu(x @ w.T + b)
        h, c = self._lstm(self.lstm[0], x, self.state[:, :H], self.state[:, H:])
        base = (np.arange(B)[:, None, None] * N + self.nbr).reshape(B * N, 3)
        last = h
        for _ in range(self.K):
            last = h
            M = h + h[base[:, 0]] + h[base[:, 1]] + h[base[:, 2]]
            h, c = self._lstm(self.lstm[1], M, h, c)
        self.state = np.concatenate([h, c], -1)
        rows = (np.arange(B)[:, None] * N + self.an).reshape(-1)
        nb = base[rows]
        out = self.obs.reshape(B * self.A, -1)
        out[:, self.D:self.D + H] = h[rows]
        for k in range(3):
            out[:, self.D + (k + 1) * H:self.D + (k + 2) * H] = last[nb[:, k]]

    def _policy(self):
        x = self.obs.reshape(self.B * self.A, -1)
        for w, b in self.dqn[:-1]:
            x = _lrelu(x @ w.T + b)
        q = x @ self.dqn[-1][0].T + self.dqn[-1][1]
        a = q.argmax(-1)
        r = self.rng.integers(0, 4, a.shape)
        f = self.rng.random(a.shape) < self.eps
        return np.where(f, r, a).astype(np.int32).reshape(self.B, self.A)

    def reset(self):
        self._env(True, None)
        self.state[:] = 0
        self._netmon()
        self.t = 0

    def step(self):
        act = self._policy()
        self._env(False, act)
        self._netmon()
        self.t += 1
        if self.t % self.ep == 0:
            self.reset()

    def close(self):
        self.L.gmo_batch_free(self.envs)


def measure(n_env=256, steps=20, threads=16, K=1, episode_steps=50):
    """env-steps/s of the CPU port over a bounded sample (n_env x steps)."""
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    r = NumpyRollout(n_env, K=K, episode_steps=episode_steps)
    r.reset()
    r.step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        r.step()
    dt = time.perf_counter() - t0
    r.close()
    return n_env * steps / dt, dt
