"""ε-greedy action selection on the device (reference src/policy.py:7-87 EpsilonGreedy).

Q-values come from the agent model (DQN, DGN, DQNR, CommNet) on the HIP kernels; the random draws
(randint(n_actions, size=A) then rand(A), every call, from each env's numpy-legacy
stream) and the argmax/mix run in the env's egreedy kernel (gm_policy_egreedy /
gm_simple_policy_egreedy).
"""

import torch

# ε-greedy runs as the env step kernel's prologue (gm_env_policy_step); tests compare it with the two launches
FUSED_POLICY_STEP = True


class EpsilonGreedy:
    def __init__(self, env, model, action_space=4, args=None, epsilon=None, epsilon_decay=None,
                 epsilon_update_freq=None, step_before_train=None):
        self._env = env.get() if hasattr(env, "get") else env
        self._model = model
        self._action_space = action_space
        self._epsilon = epsilon if epsilon is not None else getattr(args, "epsilon", 0.6)
        self._decay = epsilon_decay if epsilon_decay is not None else getattr(args, "epsilon_decay", 0.996)
        self._freq = epsilon_update_freq if epsilon_update_freq is not None else getattr(args, "epsilon_update_freq",
                                                                                          100)
        self._before = step_before_train if step_before_train is not None else getattr(args, "step_before_train",
                                                                                        2000)
        self._step = 0
        self._eps_tmp = None
        e = self._env
        self.actions = torch.zeros(e.n_env, e.n_data, dtype=torch.int32, device=e.device)
        self._scratch = {}

    def _buf(self, i, m, n):
        key = (i, m, n)
        b = self._scratch.get(key)
        if b is None:
            b = torch.empty(m, n, device=self._env.device)
            self._scratch[key] = b
        return b

    def q_values(self, obs, adj=None):
        """q [n_env, A, 4] for a joint observation view [n_env, A, D] (strided rows ok); adj:
        agent adjacency [n_env, A, A] for DGN / CommNet (default: the env's)."""
        e = self._env
        with torch.no_grad():
            x2 = obs.reshape(-1, obs.shape[-1])
            if adj is None:
                adj = getattr(e, "agent_adj", None)
            if adj is not None and adj.dtype != torch.int8:
                adj = (adj != 0).to(torch.int8)
            # rows are spaced by the agent-dim stride (reshape may renormalise size-1 dims)
            q = self._model.forward_rows(x2, obs.stride(-2), obs.shape[-1], self._buf, adj=adj, B=e.n_env,
                                         A=e.n_data)
        return q.view(e.n_env, e.n_data, -1)

    def select(self, q):
        """ε-greedy mix of argmax(q) and uniform actions, drawn from each env's stream."""
        return self._env.egreedy(q.contiguous(), self._epsilon, self.actions)

    def _decay_step(self):
        self._step += 1
        if self._epsilon > 0 and self._step > self._before and self._step % self._freq == 0:
            self._epsilon = max(self._epsilon * self._decay, 0.01)

    def __call__(self, obs, adj=None):
        actions = self.select(self.q_values(obs, adj))
        self._decay_step()
        return actions

    def act(self, wenv):
        """Fast path for a fused NetMonWrapper: the DQN's first GEMM gathers the NetMon
        readout from the node state tables instead of reading a materialised joint obs."""
        from . import fused as FU
        from .model import DQN

        if not getattr(wenv, "fused", False) or not isinstance(self._model, DQN):
            return self(wenv.obs)
        e = wenv.env
        q = FU.dqn_q(self._model, e.obs_buf, e.obs_dim, wenv.current_netmon_state, wenv.h_prev, e.nbr,
                     e.agent_node, self._buf, hidden=wenv.netmon.hidden_features, obs_gemm=e.obs_gemm)
        actions = self.select(q.view(e.n_env, e.n_data, -1))
        self._decay_step()
        return actions

    def act_step(self, wenv, detail=None):
        """act(wenv) then wenv.step_(actions). On the fused NetMon path the ε-greedy draws run
        as the env step kernel's prologue (gm_env_policy_step: one launch instead of two, the
        same draws and actions)."""
        from . import fused as FU
        from .model import DQN

        if not (getattr(wenv, "fused", False) and isinstance(self._model, DQN) and FUSED_POLICY_STEP):
            actions = self.act(wenv)
            if detail is None:
                wenv.step_(actions)
            else:
                wenv.step_(actions, detail)
            return actions
        e = wenv.env
        q = FU.dqn_q(self._model, e.obs_buf, e.obs_dim, wenv.current_netmon_state, wenv.h_prev, e.nbr,
                     e.agent_node, self._buf, hidden=wenv.netmon.hidden_features, obs_gemm=e.obs_gemm)
        wenv.policy_step_(q.view(e.n_env, e.n_data, -1).contiguous(), self._epsilon, self.actions, detail)
        self._decay_step()
        return self.actions

    def _eps_changes(self):
        """True when ε still decays (its value is a kernel argument)."""
        return self._epsilon > 0.01 and self._decay != 1.0

    def reset(self, agents_to_reset):
        """src/policy.py:72-82: zero the recurrent agent state of the given agents
        ([n_env, A] bool, or True for all)."""
        st = getattr(self._model, "state", None)
        if st is not None:
            m = torch.as_tensor(agents_to_reset, device=st.device).bool()
            self._model.state = st * ~(m.unsqueeze(-1) if m.dim() else m)

    def eval(self):
        self._eps_tmp = self._epsilon
        self._epsilon = 0

    def train(self):
        if self._eps_tmp is not None:
            self._epsilon = self._eps_tmp
            self._eps_tmp = None
