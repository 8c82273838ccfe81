"""Vectorised rollout driver: the reference's act -> step -> NetMon loop
(src/main.py:667-748 with src/env/wrapper.py:66-109) over many envs per GPU, split into
`groups` independent env groups that run on their own HIP streams.

Each group owns a Routing env batch (its own seeds, topology, packets and NetMon state)
and an ε-greedy policy; the NetMon and DQN modules (and their packed weights) are shared.
One call to step() enqueues every group's step on that group's stream, so the GPU
overlaps one group's latency-bound kernels (env step, ε-greedy draws, routing encoder)
and GEMM tails with another group's GEMMs. Results are identical to running the groups
one after another: the groups share no mutable state.

capture() records an even number of vector steps as HIP graphs (the NetMon state and h_prev
alternate between two fixed buffer pairs, so a graph reads and writes the same addresses on
every replay): by default one graph per group, captured on and replayed on that group's own
stream, so the groups keep the cross-group slack of eager launching (a single graph forks the
groups from the capturing stream and joins them at its end, which re-synchronises them on every
replay); run() then replays them, which removes the per-kernel launch gaps and most of the host
launch cost (one replay call per group per captured length). Graph replay bakes the kernel
arguments in: it is for fixed-ε rollouts (ε decay 1.0: benchmarks, evaluation); episode resets
stay eager between replays.
"""

import torch

from . import _lib as L
from . import fused as FU  # noqa: F401  (packed-weight caches shared by the groups)
from .policy import EpsilonGreedy
from .routing import Routing
from .wrapper import NetMonWrapper


# the rollout's envs write only the GEMM-ready obs copy that the fused DQN reads; reading .obs
# rebuilds the reference rows from it (Routing.set_lazy_obs); tests set it False to compare with envs that
# write both copies every step
LAZY_OBS = True


class _PlainEnv:
    """The no-NetMon counterpart of NetMonWrapper (reference: the env used directly,
    src/main.py without --netmon): same reset / step_ / obs surface."""

    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        return getattr(self.env, name)

    def get(self):
        return self.env

    @property
    def obs(self):
        return self.env.obs

    def reset(self):
        self.env.reset_()

    def reset_(self):
        self.env.reset_()

    def step_(self, actions, detail=None):
        self.env.step_(actions, detail)


class StreamedRollout:
    def __init__(self, network, n_data, n_env, netmon, model, groups=1, seed=0, epsilon=0.5, episode_steps=50,
                 obs_extra=None, device=None, stagger=False, stagger_quantum=1, **env_kw):
        """netmon None: DQN on the env observation alone (the reference without --netmon).
        stagger: group g's episodes start about g * episode_steps / groups steps into the first one
        (rounded down to a multiple of stagger_quantum: the graph length for graph replay), so the
        groups' resets (latency-bound, low occupancy) overlap another group's GEMMs instead of all
        groups resetting on the same step; every env still runs fixed-length episodes."""
        assert n_env % groups == 0, "n_env must be divisible by groups"
        self.groups = groups
        self.n_env = n_env
        self.episode_steps = episode_steps
        per = n_env // groups
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        extra = (netmon.get_out_features() if netmon is not None else 0) if obs_extra is None else obs_extra
        self.envs, self.wenvs, self.policies, self.streams = [], [], [], []
        for g in range(groups):
            env = Routing(network, n_data, n_env=per, seed=seed + g * per, obs_extra=extra, agent_adjacency=False,
                          device=dev.index, **env_kw)
            wenv = NetMonWrapper(env, netmon, 1) if netmon is not None else _PlainEnv(env)
            pol = EpsilonGreedy(wenv, model, epsilon=epsilon, epsilon_decay=1.0, epsilon_update_freq=100,
                                step_before_train=0)
            if LAZY_OBS:
                env.set_lazy_obs(True)  # the fused DQN reads obs_gemm: the reference rows are rebuilt on read
            self.envs.append(env)
            self.wenvs.append(wenv)
            self.policies.append(pol)
            self.streams.append(torch.cuda.Stream(dev))
        self.ep = 0
        self.stagger = stagger and groups > 1
        q = max(1, int(stagger_quantum))
        self._offs = [((g * episode_steps) // groups) // q * q if self.stagger else 0 for g in range(groups)]
        self._graph = None
        self._graphs = None
        self._gsteps = 0

    def _on(self, g):
        return torch.cuda.stream(self.streams[g])

    @torch.no_grad()
    def reset(self):
        """Reset every group (new topologies + NetMon start-up step). The first call also
        builds the packed weights on the caller's stream before the group streams use them."""
        cur = torch.cuda.current_stream()
        for g in range(self.groups):
            self.streams[g].wait_stream(cur)
            with self._on(g):
                self.wenvs[g].reset_()
        self.ep = 0

    def _after_caller(self):
        """Order every group stream after what the caller's stream holds (weight copies, edits): one
        event recorded, one wait per group."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        for s in self.streams:
            s.wait_event(ev)

    def _enqueue_step(self):
        self._after_caller()
        for g in range(self.groups):
            with self._on(g):
                self.policies[g].act_step(self.wenvs[g])

    @torch.no_grad()
    def step(self):
        """One vector step of every env (act, env step, NetMon step), a reset of every group
        after episode_steps steps like the reference's fixed-length episodes (per group when
        staggered)."""
        self._enqueue_step()
        self.ep += 1
        if self.ep >= self.episode_steps:
            L.check_range()  # split-f16 range guard of the finished launches (no sync)
        for g in range(self.groups):
            if (self.ep + self._offs[g]) % self.episode_steps == 0:
                with self._on(g):
                    self.wenvs[g].reset_()
        if self.ep >= self.episode_steps:
            self.ep = 0

    @torch.no_grad()
    def capture(self, steps=2, per_group=True):
        """Record `steps` (even, dividing episode_steps) vector steps: per_group, one graph per
        group on its own stream; else every group in one graph. Call after reset() and a few
        eager steps (packed weights and scratch exist)."""
        assert steps % 2 == 0 and self.episode_steps % steps == 0, "steps must be even and divide episode_steps"
        if any(o % steps for o in self._offs):
            raise ValueError("graph replay needs group episode offsets that are multiples of the captured length "
                             "(StreamedRollout(stagger_quantum=steps))")
        if any(w._eps_changes() for w in self.policies):
            raise ValueError("graph replay needs a fixed epsilon (epsilon_decay = 1.0)")
        torch.cuda.synchronize()
        if per_group:
            graphs = []
            for g in range(self.groups):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=self.streams[g]):
                    for _ in range(steps):
                        self.policies[g].act_step(self.wenvs[g])
                graphs.append(gr)
            self._graph, self._graphs, self._gsteps = None, graphs, steps
            return
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cap = torch.cuda.current_stream()
            for s in self.streams:
                s.wait_stream(cap)
            for _ in range(steps):
                self._enqueue_step()
            for s in self.streams:
                cap.wait_stream(s)
        self._graph, self._graphs, self._gsteps = graph, None, steps
        # the capture only recorded: the env / NetMon state is where it was before it; the
        # ping-pong buffer parity advanced by `steps` (even): unchanged

    @torch.no_grad()
    def run(self, n):
        """n vector steps (graph replays of capture()'s length when captured, else eager)."""
        if self._graph is None and self._graphs is None:
            for _ in range(n):
                self.step()
            return
        assert n % self._gsteps == 0
        for _ in range(n // self._gsteps):
            if self.ep % self._gsteps:
                raise RuntimeError("graph replay must start at a multiple of the captured length")
            if self._graphs is not None:
                self._after_caller()
                for g, gr in enumerate(self._graphs):
                    with self._on(g):
                        gr.replay()
                        self.envs[g].mark_obs_stale()  # on the group stream: sync_obs waits for it
                self.ep += self._gsteps
                if self.ep >= self.episode_steps:
                    L.check_range()
                for g in range(self.groups):
                    if (self.ep + self._offs[g]) % self.episode_steps == 0:
                        with self._on(g):
                            self.wenvs[g].reset_()
                if self.ep >= self.episode_steps:
                    self.ep = 0
                continue
            self._graph.replay()
            for e in self.envs:
                e.mark_obs_stale()
            self.ep += self._gsteps
            if self.ep >= self.episode_steps:
                L.check_range()
            due = [g for g in range(self.groups) if (self.ep + self._offs[g]) % self.episode_steps == 0]
            if due:
                cur = torch.cuda.current_stream()  # the replay's stream
                for g in due:
                    self.streams[g].wait_stream(cur)
                    with self._on(g):
                        self.wenvs[g].reset_()
                for g in due:
                    cur.wait_stream(self.streams[g])
            if self.ep >= self.episode_steps:
                self.ep = 0

    def join(self):
        """Make the caller's stream wait for every group's work."""
        cur = torch.cuda.current_stream()
        for s in self.streams:
            cur.wait_stream(s)
