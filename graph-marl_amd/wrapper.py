"""NetMon graph observations for the batched routing env (reference
src/env/wrapper.py:7-109 NetMonWrapper).

After every env step one NetMon step runs on the device over all n_env graphs.
Fused mode (lstm / lnlstm / gru NetMon with carry-over, default): the step is three encoder
GEMMs plus the RNN cells on the HIP kernels (fused.netmon_step: lstm / gru one gate-tile GEMM
with the gate math in its epilogue, lnlstm two GEMMs + the LayerNorm-LSTM pointwise kernel); the graph part of the joint
observation is NOT materialised — the DQN gathers it inside its first GEMM
(policy.EpsilonGreedy.act). Reading `.obs` (the reference API) materialises the joint
observation [env obs | readout] on demand. Unfused mode runs NetMon.forward_graph and writes
the readout into the joint observation buffer after every step.
"""
import torch

from . import _lib as L
from . import fused as FU
from .model import NetMon, netmon_readout


class NetMonWrapper:
    def __init__(self, env, netmon: NetMon, startup_iterations=1, fused=None):
        assert startup_iterations >= 1, "Number of startup iterations must be >= 1"
        # the readout is [h, h_prev of deg neighbours] with deg = the graph's max degree
        # (src/model.py:582-589), so the graph part is (deg + 1) H wide (4H on routing graphs)
        H = netmon.hidden_features
        self.graph_features = H * (1 + (env.nbr.shape[-1] if netmon.output_neighbor_hidden else 0) +
                                   (1 if netmon.output_global_hidden else 0))
        need = env.obs_dim + self.graph_features
        if env.obs_stride < need:
            raise ValueError(f"env obs buffer too narrow: create the env with obs_extra={self.graph_features}")
        self.env = env
        self.netmon = netmon
        self.startup_iterations = startup_iterations
        self.last_netmon_state = None
        self.current_netmon_state = None
        self.h_prev = None
        self.obs_dim = need
        if fused is None:
            fused = FU.fused_ok(netmon)
        self.fused = fused
        if fused and hasattr(env, "enable_gemm_obs"):
            env.enable_gemm_obs()  # the fused DQN reads the GEMM-ready env obs copy
        self._dirty = False
        # fused mode: the state and h_prev alternate between two fixed buffer pairs, so a
        # captured 2-step HIP graph (rollout.StreamedRollout.capture) reads and writes the
        # same addresses on every replay
        self._bufs = None
        self._cur = 0

    def __getattr__(self, name):
        return getattr(self.env, name)

    def __str__(self):
        return str(self.env) + "\n▲ environment is wrapped with NetMon (graph obs)"

    @property
    def obs(self):
        """joint observation [n_env, A, obs_dim + (deg+1)H] (reference: concat of obs and graph obs)."""
        if self._dirty:
            self._materialize()
        if hasattr(self.env, "sync_obs"):
            self.env.sync_obs()  # env columns rebuilt when the env wrote only its GEMM-ready copy
        return self.env.obs_buf[..., : self.obs_dim]

    def _materialize(self):
        e, H = self.env, self.netmon.hidden_features
        B, N = e.n_env, e.n_nodes
        hf = self.current_netmon_state.reshape(B * N, -1)[:, :H].contiguous()
        hp = self.h_prev[:, :H].contiguous()
        with torch.no_grad():
            netmon_readout(hf, hp, e.nbr, e.agent_node, out=e.obs_buf, col0=e.obs_dim)
        self._dirty = False

    def _netmon_step(self):
        e = self.env
        with torch.no_grad():
            self.last_netmon_state = self.current_netmon_state
            if self.fused:
                B, N, H2 = e.n_env, e.n_nodes, self.netmon.get_state_size()
                if self._bufs is None:
                    self._bufs = [(torch.empty(B, N, H2, device=e.device), torch.empty(B * N, H2, device=e.device))
                                  for _ in range(2)]
                nxt = 1 - self._cur
                st, hp = self._bufs[nxt]
                state, self.h_prev = FU.netmon_step(self.netmon, e.node_obs, e.nbr, self.current_netmon_state,
                                                    out=st, last_out=hp)
                self._cur = nxt
                self.current_netmon_state = state
                self._dirty = True
            else:
                self.netmon.state = self.current_netmon_state
                self.netmon.forward_graph(e.node_obs, e.nbr, e.agent_node, out=e.obs_buf, out_col=e.obs_dim)
                self.current_netmon_state = self.netmon.state

    def reset_(self):
        """reset() without materialising the joint observation (the rollout driver's form)."""
        self.current_netmon_state = None
        self.last_netmon_state = None
        self._cur = 1  # the start-up step writes buffer pair 0
        self.env.reset_()
        for _ in range(self.startup_iterations):
            self._netmon_step()

    def reset(self):
        self.reset_()
        return self.obs, self.env.agent_adj

    def step(self, actions):
        _, adj, reward, done, info = self.env.step(actions)
        self._netmon_step()
        return self.obs, adj, reward, done, info

    def step_(self, actions, detail=None):
        self.env.step_(actions, detail)
        self._netmon_step()

    def policy_step_(self, q, epsilon, actions, detail=None):
        """ε-greedy on q + env step in one launch (Routing.policy_step_), then the NetMon step."""
        self.env.policy_step_(q, epsilon, actions, detail)
        self._netmon_step()

    def get_netmon_info(self):
        return self.env.node_obs, self.env.nbr, self.env.agent_node

    def get(self):
        return self.env
