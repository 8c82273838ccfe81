"""CPU restatement of SimpleEnvironment (reference src/env/simple_environment.py:45-334)
and of EpsilonGreedy's draws for it (src/policy.py:44-50) — TEST INFRASTRUCTURE ONLY.

Used by tests/ as the checker of the HIP SimpleEnvironment (graph-marl_amd/csrc/
gm_simple.hip); pinned against tests/golden/simple.npz, which was produced by importing
the reference itself (tests/golden/make_golden.py::gen_simple). Every env draws from its
own numpy legacy RandomState, exactly as the reference draws from the global stream.
"""
import numpy as np


class SimpleRef:
    def __init__(self, seed, env_var=1, random_topology=True):
        self.rs = np.random.RandomState(seed)
        self.env_var = env_var
        self.rt = bool(random_topology)
        self.score = np.zeros(3, np.int32)
        self.redge = np.full((3, 2), -1, np.int32)
        self.ends = np.zeros((2, 2), np.int32)
        self.start = 0
        self.now = 0

    def _shuffle(self, x):
        # legacy RandomState.shuffle: i = n-1..1, j = random_interval(i) (masked rejection)
        for i in range(len(x) - 1, 0, -1):
            j = int(self.rs.randint(i + 1))
            x[i], x[j] = x[j], x[i]

    def reset(self):
        """_build_network (simple_environment.py:123-209)."""
        border = [-1, 1]
        self._shuffle(border)
        sc = [border[0], 0, border[1]]
        if self.rt:
            self._shuffle(sc)
        n0 = sc.index(0)
        n1 = (n0 + 1) % 3
        n2 = (n1 + 1) % 3
        self.rs.random_sample(6)  # router positions x, y (plot only)
        dest = [n1, n2]
        if self.rt:
            self._shuffle(dest)
        e0 = [n0, dest[0]]
        if self.rt:
            self._shuffle(e0)
        e1 = [n0, dest[1]]
        if self.rt:
            self._shuffle(e1)
        order = [0, 1]
        if self.rt and dest[1] < dest[0]:
            order = [1, 0]
        self.score = np.array(sc, np.int32)
        self.redge = np.full((3, 2), -1, np.int32)
        self.redge[n0] = order
        self.redge[dest[0], 0] = 0
        self.redge[dest[1], 0] = 1
        self.ends = np.array([e0, e1], np.int32)
        self.start = self.now = n0
        return self.observe()

    def adjacency(self):
        adj = np.eye(3, dtype=np.int8)
        for i in range(3):
            for t in self.redge[i]:
                if t >= 0:
                    a, b = self.ends[t]
                    adj[i, b if a == i else a] = 1
        return adj

    def observe(self):
        ob = [float(self.now)]
        if self.env_var != 1:
            ob += list(self.adjacency().reshape(-1).astype(np.float32)) + list(self.score.astype(np.float32))
        return np.array([ob], np.float32)

    def egreedy(self, q, eps):
        ra = self.rs.randint(2, size=1)
        rf = self.rs.rand(1) < eps
        return np.argmax(q, axis=-1) * ~rf + rf * ra

    def step(self, act):
        """simple_environment.py:283-315 -> (obs, reward)."""
        t = self.redge[self.now][int(act)]
        a, b = self.ends[t]
        reached = b if a == self.now else a
        reward = float(self.score[reached])
        self.now = self.start
        return self.observe(), reward
