"""NetMon graph observations for the batched routing env (reference
src/env/wrapper.py:7-109 NetMonWrapper).

After every env step one NetMon step runs on the device over all n_env graphs;
its readout is written straight into columns [6N+10, 6N+10+4H) of the env's
joint observation buffer (the reference's np.concatenate of obs and graph obs).
"""
import torch

from .model import NetMon


class NetMonWrapper:
    def __init__(self, env, netmon: NetMon, startup_iterations=1):
        assert startup_iterations >= 1, "Number of startup iterations must be >= 1"
        need = env.obs_dim + netmon.get_out_features()
        if env.obs_stride < need:
            raise ValueError(f"env obs buffer too narrow: create Routing with obs_extra={netmon.get_out_features()}")
        self.env = env
        self.netmon = netmon
        self.startup_iterations = startup_iterations
        self.last_netmon_state = None
        self.current_netmon_state = None
        self.obs_dim = need

    def __getattr__(self, name):
        return getattr(self.env, name)

    def __str__(self):
        return str(self.env) + "\n▲ environment is wrapped with NetMon (graph obs)"

    @property
    def obs(self):
        return self.env.obs_buf[..., : self.obs_dim]

    def _netmon_step(self):
        with torch.no_grad():
            self.last_netmon_state = self.current_netmon_state
            self.netmon.state = self.current_netmon_state
            self.netmon.forward_graph(self.env.node_obs, self.env.nbr, self.env.agent_node,
                                      out=self.env.obs_buf, out_col=self.env.obs_dim)
            self.current_netmon_state = self.netmon.state

    def reset(self):
        self.current_netmon_state = None
        self.last_netmon_state = None
        self.env.reset_()
        for _ in range(self.startup_iterations):
            self._netmon_step()
        return self.obs, self.env.agent_adj

    def step(self, actions):
        _, adj, reward, done, info = self.env.step(actions)
        self._netmon_step()
        return self.obs, adj, reward, done, info

    def step_(self, actions, detail=None):
        self.env.step_(actions, detail)
        self._netmon_step()

    def get_netmon_info(self):
        return self.env.node_obs, self.env.nbr, self.env.agent_node

    def get(self):
        return self.env
