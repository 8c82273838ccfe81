"""Device-resident replay memory for n_env parallel envs (reference
src/replaybuffer.py:34-287 ReplayBuffer).

Differences from the reference, by design:
  * one ring slot = one vector step = n_env transitions, all tensors stay in HBM
    (the reference copies 17 host arrays to the device per sampled step);
  * the 4H NetMon part of the agent observation is not stored: the update re-runs
    NetMon over the sampled sequence and overwrites it anyway (src/main.py:865-880,
    909-915); the graph is stored as its neighbour table and the node-agent matrix
    as the agent -> node index, the NetMon input state as in the reference
    (the state *before* the NetMon call that produced obs, wrapper.py:99-104);
  * sampling: the reference's stream itself, np.random.default_rng(seed).choice(n, size,
    replace=True), generated on the device (gm_pcg64_choice: numpy's PCG64 + Lemire bounded
    draws, state kept in HBM). The ring is (slot, env): a uniform batch draws
    f = choice(count * n_env) -> (slot f // n_env, env f % n_env); a sequence batch draws
    f = choice(n_env * (count - L)) -> env f // (count - L), start = (index % count +
    f % (count - L)) % count. With n_env = 1 both are the reference's indices exactly
    (src/replaybuffer.py:107-130; tests/test_replay_rng.py against its golden).
"""
import ctypes as C
from collections import namedtuple

import torch

from . import _lib as L

TransitionBatch = namedtuple(
    "TransitionBatch",
    ["idx", "obs", "action", "reward", "next_obs", "done", "episode_done", "node_obs", "nbr", "node_state",
     "agent_node", "next_node_obs", "next_agent_node", "adj", "next_adj", "agent_state", "node_aux"],
    defaults=(None, None, None, None),
)


class LazyRows:
    """A field of a sampled batch gathered on demand: [r] gathers the rows r of the batch,
    full() all of them (ReplayBuffer.get_batch(lazy_next=True): the update's target pass needs
    the next observations only at the last step of a sequence and at episode ends)."""

    def __init__(self, src, slot, env, conv):
        self.src, self.slot, self.env, self.conv = src, slot, env, conv

    def __getitem__(self, r):
        return self.conv(self.src[self.slot[r], self.env[r]])

    def full(self):
        return self.conv(self.src[self.slot, self.env])


def materialize(x):
    return x.full() if isinstance(x, LazyRows) else x


class ReplayBuffer:
    def __init__(self, seed, capacity, n_env, n_agents, obs_dim, n_nodes, node_obs_dim, node_state_size,
                 device, half_precision=False, nbr_width=3, agent_state_size=0, store_adj=False, node_aux_size=0):
        """capacity: transitions (env-steps) like the reference; the ring holds
        ceil(capacity / n_env) vector steps. agent_state_size > 0 stores the recurrent
        models' agent state (DQNR / CommNet), store_adj the agent adjacency (DGN / CommNet),
        src/replaybuffer.py:64-99; node_aux_size > 0 stores the env's node aux targets
        (get_node_aux, [N][node_aux_size]) for the NetMon aux loss (--aux-loss-coeff)."""
        self.n_env, self.A, self.N = n_env, n_agents, n_nodes
        self.slots = max(1, -(-int(capacity) // n_env))
        self.capacity = self.slots * n_env
        self.count = 0  # filled slots
        self.index = 0  # next slot
        self.device = device
        ft = torch.float16 if half_precision else torch.float32
        S, B, A, N = self.slots, n_env, n_agents, n_nodes

        def z(*shape, dtype=ft):
            return torch.zeros(*shape, dtype=dtype, device=device)

        # observation rows padded to a multiple of 4 floats: a sampled batch is a view whose rows the
        # GEMM kernels read in place (16-byte rows), no padded copy per update step
        self.obs_dim = obs_dim
        odp = (obs_dim + 3) // 4 * 4
        self.obs = z(S, B, A, odp)
        self.next_obs = z(S, B, A, odp)
        self.action = z(S, B, A, dtype=torch.int8)
        self.reward = z(S, B, A)
        self.done = z(S, B, A, dtype=torch.bool)
        self.episode_done = z(S, dtype=torch.bool)
        self.graph = node_state_size > 0  # NetMon transitions carry the graph inputs
        if self.graph:
            self.node_obs = z(S, B, N, node_obs_dim)
            self.next_node_obs = z(S, B, N, node_obs_dim)
            self.nbr = z(S, B, N, nbr_width, dtype=torch.int8)
            self.agent_node = z(S, B, A, dtype=torch.int8)
            self.next_agent_node = z(S, B, A, dtype=torch.int8)
            self.node_state = z(S, B, N, node_state_size)
        self.agent_state = z(S, B, A, agent_state_size) if agent_state_size > 0 else None
        self.node_aux = z(S, B, N, node_aux_size) if node_aux_size > 0 else None
        self.adj = z(S, B, A, A, dtype=torch.bool) if store_adj else None
        self.next_adj = z(S, B, A, A, dtype=torch.bool) if store_adj else None
        st = L.PCG64()
        L.check(L.lib().gm_pcg64_seed(C.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), C.byref(st)))
        self.rng = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(device)  # gm_pcg64 in HBM

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.__dict__.values() if torch.is_tensor(t))

    def add_pre(self, obs, node_state=None, node_obs=None, nbr=None, agent_node=None, adj=None, agent_state=None,
                node_aux=None):
        """First half of a transition, recorded before the env step: the observation and the
        NetMon inputs that produced it (node_state = the NetMon state before that call), the
        agent adjacency, the agent state the model starts the step from (None = zeros) and the
        node aux targets (src/main.py:697-699)."""
        i = self.index
        self.obs[i, ..., : self.obs_dim].copy_(obs)
        if self.node_aux is not None:
            self.node_aux[i].copy_(node_aux)
        if self.adj is not None:
            self.adj[i].copy_(adj != 0)
        if self.agent_state is not None:
            if agent_state is None:
                self.agent_state[i].zero_()
            else:
                self.agent_state[i].copy_(agent_state)
        if self.graph:
            if node_state is None:
                self.node_state[i].zero_()
            else:
                self.node_state[i].copy_(node_state)
            self.node_obs[i].copy_(node_obs)
            self.nbr[i].copy_(nbr)
            self.agent_node[i].copy_(agent_node)

    def add_post(self, action, reward, next_obs, done, episode_done, next_node_obs=None, next_agent_node=None,
                 next_adj=None):
        """Second half, after the step; commits the slot."""
        i = self.index
        if self.next_adj is not None:
            self.next_adj[i].copy_(next_adj != 0)
        self.action[i].copy_(action)
        self.reward[i].copy_(reward)
        self.next_obs[i, ..., : self.obs_dim].copy_(next_obs)
        self.done[i].copy_(done)
        self.episode_done[i] = bool(episode_done)
        if self.graph:
            self.next_node_obs[i].copy_(next_node_obs)
            self.next_agent_node[i].copy_(next_agent_node)
        if self.count < self.slots:
            self.count += 1
        self.index = (self.index + 1) % self.slots

    def add(self, obs, action, reward, next_obs, done, episode_done, node_state, node_obs, nbr, agent_node,
            next_node_obs, next_agent_node):
        """One vector step (every argument has a leading n_env dim; node_state may be None = zeros)."""
        self.add_pre(obs, node_state, node_obs, nbr, agent_node)
        self.add_post(action, reward, next_obs, done, episode_done, next_node_obs, next_agent_node)

    def _gather(self, slot, env, first=True, lazy_next=False):
        """One TransitionBatch of the (slot, env) pairs. The stored start states (NetMon node state,
        agent state) are read by the update at the first step of a sequence only
        (src/main.py:846-851, 858-859), so later steps leave them out (None)."""
        f = torch.float32
        g = self.graph
        if lazy_next:
            od = self.obs_dim
            return TransitionBatch(
                (slot, env), self.obs[slot, env].to(f)[..., :od], self.action[slot, env].long(),
                self.reward[slot, env].to(f), LazyRows(self.next_obs, slot, env, lambda t: t.to(f)[..., :od]),
                self.done[slot, env], self.episode_done[slot], self.node_obs[slot, env].to(f) if g else None,
                self.nbr[slot, env].int().contiguous() if g else None,
                self.node_state[slot, env].to(f) if g and first else None,
                self.agent_node[slot, env].int().contiguous() if g else None,
                LazyRows(self.next_node_obs, slot, env, lambda t: t.to(f)) if g else None,
                LazyRows(self.next_agent_node, slot, env, lambda t: t.int().contiguous()) if g else None,
                self.adj[slot, env].to(f) if self.adj is not None else None,
                LazyRows(self.next_adj, slot, env, lambda t: t.to(f)) if self.next_adj is not None else None,
                self.agent_state[slot, env].to(f) if self.agent_state is not None and first else None,
                self.node_aux[slot, env].to(f) if self.node_aux is not None else None,
            )
        return TransitionBatch(
            (slot, env), self.obs[slot, env].to(f)[..., : self.obs_dim], self.action[slot, env].long(),
            self.reward[slot, env].to(f), self.next_obs[slot, env].to(f)[..., : self.obs_dim], self.done[slot, env],
            self.episode_done[slot],
            self.node_obs[slot, env].to(f) if g else None, self.nbr[slot, env].int().contiguous() if g else None,
            self.node_state[slot, env].to(f) if g and first else None,
            self.agent_node[slot, env].int().contiguous() if g else None,
            self.next_node_obs[slot, env].to(f) if g else None,
            self.next_agent_node[slot, env].int().contiguous() if g else None,
            self.adj[slot, env].to(f) if self.adj is not None else None,
            self.next_adj[slot, env].to(f) if self.next_adj is not None else None,
            self.agent_state[slot, env].to(f) if self.agent_state is not None and first else None,
            self.node_aux[slot, env].to(f) if self.node_aux is not None else None,
        )

    def choice(self, n, size):
        """np.random.default_rng(seed).choice(n, size, replace=True) continuing this buffer's
        stream, as a device int64 tensor (gm_pcg64_choice)."""
        out = torch.empty(size, dtype=torch.int64, device=self.device)
        L.check(L.lib().gm_pcg64_choice(L.ptr(self.rng), int(n), int(size), L.ptr(out), L.stream_ptr(self.device)))
        return out

    def rng_state(self):
        """The sampling stream's numpy bit_generator.state fields (synchronous)."""
        st = L.PCG64.from_buffer_copy(self.rng.cpu().numpy().tobytes())
        return {"state": (st.state_hi << 64) | st.state_lo, "inc": (st.inc_hi << 64) | st.inc_lo,
                "has_uint32": st.has_uint32, "uinteger": st.uinteger}

    def get_sequences(self, batch_size, sequence_length):
        """The sequences get_batch(batch_size, sequence_length) draws (same stream, same indices), as
        one train_seq.SeqBatch with every step's fields stacked ([L, B, ...], one gather per field);
        the next-step fields are gathered on demand (next_fields(t, rows))."""
        from .train_seq import SeqBatch

        if not self.graph:
            raise ValueError("get_sequences: NetMon transitions only")
        if self.count <= sequence_length:
            raise ValueError("not enough transitions for the requested sequence length")
        Lq = sequence_length
        span = self.count - Lq
        f = self.choice(self.n_env * span, batch_size)
        env = f // span
        first = (self.index % self.count + f % span) % self.count
        slots = (first.unsqueeze(0) + torch.arange(Lq, device=f.device).unsqueeze(1)) % self.count  # [L, B]
        envs = env.unsqueeze(0).expand(Lq, -1)
        fl = torch.float32
        od = self.obs_dim

        def next_fields(t, rows):
            s, e = (slots[t], env) if rows is None else (slots[t][rows], env[rows])
            return (self._records(self.next_obs, s, e), self._records(self.next_node_obs, s, e),
                    self.next_agent_node[s, e].int().contiguous())

        return SeqBatch(self._records(self.obs, slots, env), od, self.action[slots, envs].long(),
                        self.reward[slots, envs].to(fl), self.done[slots, envs], self.episode_done[slots],
                        self._records(self.node_obs, slots, env), self.nbr[slots, envs].int().contiguous(),
                        self.agent_node[slots, envs].int().contiguous(), self._records(self.node_state, first, env),
                        next_fields, (slots, env))

    @staticmethod
    def _records(src, slots, env):
        """src[slots, env] as float32 (slots [..., B'] int64 slot indices, env [B'] env indices): one
        gm_gather_records launch for float32 ring fields with 16-byte records, torch indexing otherwise."""
        rec = src.shape[2:]
        nbytes = src[0, 0].numel() * src.element_size()
        if not src.is_cuda or src.dtype != torch.float32 or nbytes % 16 or not src.is_contiguous():
            return src[slots, env.expand_as(slots)].to(torch.float32)
        sl = slots.contiguous()
        ev = env.contiguous()
        out = torch.empty(*sl.shape, *rec, dtype=torch.float32, device=src.device)
        if out.numel() == 0:
            return out
        L.check(L.lib().gm_gather_records(src.data_ptr(), src.stride(0) * 4, src.stride(1) * 4, sl.data_ptr(),
                                          ev.data_ptr(), ev.numel(), sl.numel(), nbytes, out.data_ptr(),
                                          L.stream_ptr()))
        return out

    def get_batch(self, batch_size, sequence_length=1, lazy_next=False):
        """Yields sequence_length TransitionBatches of batch_size transitions
        (src/replaybuffer.py:103-130): uniform (slot, env); sequences are consecutive slots of
        one env, starting from the oldest slot and wrapping. lazy_next: the next-step fields of
        every step but the last are LazyRows (gathered on demand)."""
        if self.count == 0:
            raise ValueError("empty replay buffer")
        if sequence_length <= 1:
            f = self.choice(self.count * self.n_env, batch_size)
            yield self._gather(f // self.n_env, f % self.n_env)
            return
        if self.count <= sequence_length:
            raise ValueError("not enough transitions for the requested sequence length")
        span = self.count - sequence_length
        f = self.choice(self.n_env * span, batch_size)
        env = f // span
        first = (self.index % self.count + f % span) % self.count
        for o in range(sequence_length):
            yield self._gather((first + o) % self.count, env, first=o == 0,
                               lazy_next=lazy_next and o < sequence_length - 1)
