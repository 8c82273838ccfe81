"""SimpleEnvironment (BASELINE config 1): the CPU restatement against the reference's
golden traces (CPU), and the HIP env against both (GPU). Traces interleave resets,
EpsilonGreedy draws (src/policy.py:44-50) and steps on one stream per env."""
import importlib
import os

import numpy as np
import pytest
import torch

from simple_ref import SimpleRef

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "simple.npz")


def _configs(g):
    return [tuple(int(v) for v in c) for c in g["configs"]]


def _replay_oracle(g, ci, seed, env_var, rt):
    o = SimpleRef(seed, env_var, rt)
    T = len(g[f"c{ci}_reset"])
    for t in range(T):
        if g[f"c{ci}_reset"][t]:
            o.reset()
        np.testing.assert_array_equal(o.score, g[f"c{ci}_score"][t])
        np.testing.assert_array_equal(o.redge, g[f"c{ci}_redge"][t])
        np.testing.assert_array_equal(o.ends, g[f"c{ci}_ends"][t])
        assert o.start == g[f"c{ci}_start"][t]
        np.testing.assert_array_equal(o.adjacency(), g[f"c{ci}_node_adj"][t])
        act = o.egreedy(g[f"c{ci}_q"][t], 0.5)
        np.testing.assert_array_equal(act, g[f"c{ci}_act"][t])
        obs, rw = o.step(act[0])
        np.testing.assert_array_equal(obs, g[f"c{ci}_obs"][t])
        assert rw == g[f"c{ci}_reward"][t][0]


def test_oracle_matches_reference_golden():
    g = np.load(GOLDEN)
    for ci, (seed, env_var, rt) in enumerate(_configs(g)):
        _replay_oracle(g, ci, seed, env_var, rt)


@pytest.mark.gpu
def test_device_matches_reference_golden():
    S = importlib.import_module("graph-marl_amd.simple")
    g = np.load(GOLDEN)
    for ci, (seed, env_var, rt) in enumerate(_configs(g)):
        env = S.SimpleEnvironment(env_var, bool(rt), n_env=1, seeds=[seed])
        act = torch.zeros(1, 1, dtype=torch.int32, device="cuda")
        for t in range(len(g[f"c{ci}_reset"])):
            if g[f"c{ci}_reset"][t]:
                env.reset()
            st = env.get_state()
            np.testing.assert_array_equal(st["score"][0], g[f"c{ci}_score"][t], err_msg=f"cfg {ci} step {t}")
            np.testing.assert_array_equal(st["router_edge"][0], g[f"c{ci}_redge"][t])
            np.testing.assert_array_equal(st["edge_end"][0], g[f"c{ci}_ends"][t])
            assert st["start"][0] == g[f"c{ci}_start"][t]
            np.testing.assert_array_equal(env.node_adj[0].cpu().numpy(), g[f"c{ci}_node_adj"][t])
            np.testing.assert_array_equal(env.node_obs[0].cpu().numpy(), g[f"c{ci}_node_obs"][t])
            np.testing.assert_array_equal(env.get_node_agent_matrix()[0].cpu().numpy(), g[f"c{ci}_node_agent"][t])
            q = torch.as_tensor(g[f"c{ci}_q"][t], device="cuda").reshape(1, 1, 2).contiguous()
            env.egreedy(q, 0.5, act)
            assert act.item() == g[f"c{ci}_act"][t][0], f"cfg {ci} step {t} action"
            obs, _, rw, done, _ = env.step(act)
            np.testing.assert_array_equal(obs[0].cpu().numpy(), g[f"c{ci}_obs"][t])
            assert rw.item() == g[f"c{ci}_reward"][t][0]
            assert bool(done.all())
        env.get_state()  # no invalid action was reported


@pytest.mark.gpu
def test_device_batch_matches_oracle():
    """256 envs with distinct seeds, masked resets, random q: every env equals its own
    CPU restatement."""
    S = importlib.import_module("graph-marl_amd.simple")
    B = 256
    seeds = [1000 + 7 * i for i in range(B)]
    for env_var, rt in ((1, True), (3, True), (1, False)):
        env = S.SimpleEnvironment(env_var, rt, n_env=B, seeds=seeds)
        orc = [SimpleRef(s, env_var, rt) for s in seeds]
        rng = np.random.RandomState(5)
        env.reset()
        for o in orc:
            o.reset()
        act = torch.zeros(B, 1, dtype=torch.int32, device="cuda")
        for t in range(12):
            mask = rng.rand(B) < 0.4
            env.reset_(torch.as_tensor(mask, device="cuda"))
            for b in np.nonzero(mask)[0]:
                orc[b].reset()
            q = rng.standard_normal((B, 1, 2)).astype(np.float32)
            env.egreedy(torch.as_tensor(q, device="cuda"), 0.3, act)
            a = act.cpu().numpy()
            exp_obs = []
            exp_rw = []
            for b, o in enumerate(orc):
                ea = o.egreedy(q[b], 0.3)
                assert ea[0] == a[b, 0], f"env {b} step {t}"
                ob, rw = o.step(ea[0])
                exp_obs.append(ob)
                exp_rw.append(rw)
            env.step_(act)
            np.testing.assert_array_equal(env.obs.cpu().numpy(), np.stack(exp_obs))
            np.testing.assert_array_equal(env.reward[:, 0].cpu().numpy(), np.array(exp_rw, np.float32))


@pytest.mark.gpu
def test_invalid_action_is_reported():
    S = importlib.import_module("graph-marl_amd.simple")
    L = importlib.import_module("graph-marl_amd._lib")
    env = S.SimpleEnvironment(1, True, n_env=2, seeds=[0, 1])
    env.reset()
    env.step_(torch.tensor([[0], [2]], dtype=torch.int32, device="cuda"))
    with pytest.raises(L.GMError):
        env.get_state()
    env.get_state()  # the error was consumed
