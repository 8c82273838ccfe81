"""Non-learned policies of the reference (src/policy.py:90-189) on the device.

ShortestPath (routing): first hop of networkx's weighted shortest path (Dijkstra with
networkx's tie-breaking, src/env/network.py:279) from each packet's node to its target,
computed per env by gm_policy_shortest_path.
RandomPolicy: uniform actions. The reference samples gymnasium's Discrete.sample(), an
unseeded generator of its own, so its draws are not reproducible there either; here they
come from a seeded torch device generator.
SimplePolicy (simple env): the reference compares a node id with a Router object
(src/policy.py:177-186), so the comparison never matches and it always returns action 0;
that behaviour is kept.
"""
import torch


class ShortestPath:
    def __init__(self, env, model=None, action_space=4, args=None):
        self._env = env.get() if hasattr(env, "get") else env
        if not hasattr(self._env, "shortest_path_actions"):
            raise ValueError("ShortestPath needs the routing environment")
        e = self._env
        self.actions = torch.zeros(e.n_env, e.n_data, dtype=torch.int32, device=e.device)

    def reset_episode(self):
        pass

    def act(self, env):
        return self._env.shortest_path_actions(self.actions)

    def __call__(self, obs=None, adj=None):
        return self.act(self._env)


class RandomPolicy:
    def __init__(self, env, model=None, action_space=4, args=None, seed=0):
        self._env = env.get() if hasattr(env, "get") else env
        self._n = action_space
        e = self._env
        self.gen = torch.Generator(device=e.device)
        self.gen.manual_seed(seed)
        self.actions = torch.zeros(e.n_env, e.n_data, dtype=torch.int32, device=e.device)

    def act(self, env):
        e = self._env
        self.actions.copy_(torch.randint(0, self._n, (e.n_env, e.n_data), device=e.device, generator=self.gen))
        return self.actions

    def __call__(self, obs=None, adj=None):
        return self.act(self._env)


class SimplePolicy:
    def __init__(self, env, model=None, action_space=2, args=None):
        self._env = env.get() if hasattr(env, "get") else env
        e = self._env
        self.actions = torch.zeros(e.n_env, e.n_data, dtype=torch.int32, device=e.device)

    def act(self, env):
        return self.actions

    def __call__(self, obs=None, adj=None):
        return self.actions

