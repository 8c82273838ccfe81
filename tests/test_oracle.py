"""CPU tests: pin the oracle against the reference's golden vectors.

The golden files were produced by importing the reference (tests/golden/make_golden.py).
"""
import numpy as np
import pytest

import os

import golden_replay as R
import netmon_ref


def test_mt19937_streams(oracle_mod):
    g = np.load(f"{R.GOLDEN}/rng.npz")
    for s in g["seeds"]:
        s = int(s)
        m = oracle_mod.MTStream(s)
        np.testing.assert_array_equal(m.key, g[f"key_{s}"])
        raw = np.array([m.next32() for _ in range(1500)], dtype=np.uint32)
        np.testing.assert_array_equal(raw, g[f"raw_{s}"])
        m = oracle_mod.MTStream(s)
        mix = []
        for _ in range(100):
            mix += [m.randint(20), m.randint(20), m.random()]
        np.testing.assert_array_equal(np.array(mix), g[f"packet20_{s}"])
        m = oracle_mod.MTStream(s)
        np.testing.assert_array_equal([m.randint(2**31 - 1) for _ in range(64)], g[f"randint31_{s}"])
        m = oracle_mod.MTStream(s)
        ns = [1, 2, 3, 5, 7, 10, 13, 20, 33, 50, 64, 100, 1000] * 20
        np.testing.assert_array_equal([m.randint(n) for n in ns], g[f"randint_n_{s}"])
        m = oracle_mod.MTStream(s)
        eg = []
        for _ in range(40):
            eg.append([m.randint(4) for _ in range(20)])
            eg.append([m.random() for _ in range(20)])
        np.testing.assert_array_equal(np.array(eg, dtype=np.float64), g[f"egreedy_{s}"])


def test_eval_seeds_are_the_generator_output(oracle_mod):
    """EVAL_SEEDS (src/env/constants.py) = first 1000 valid seeds from init seed 476."""
    ev = np.load(f"{R.GOLDEN}/eval_seeds.npy")
    np.testing.assert_array_equal(oracle_mod.build_seed_list(20, 476, 1000), ev)


def test_product_eval_seed_table_matches_reference():
    import os

    prod = np.load(os.path.join(R.GOLDEN, "..", "..", "graph-marl_amd", "data", "eval_seeds.npy"))
    np.testing.assert_array_equal(prod, np.load(f"{R.GOLDEN}/eval_seeds.npy"))


@pytest.mark.parametrize("n", [10, 20, 30, 40, 50, 100])
def test_random_topologies(oracle_mod, n):
    t = np.load(f"{R.GOLDEN}/topology.npz")
    k = f"rand_n{n}"
    cfg = oracle_mod.make_config(n, 1, topo_mode=oracle_mod.TOPO_RANDOM, excluded=R.EVAL_SEEDS)
    m = oracle_mod.MTStream(int(t[k + "_main_seed"]))
    for r in range(len(t[k + "_seed"])):
        s, tp = oracle_mod.create_valid(cfg, m)
        a = tp.arrays()
        assert s == t[k + "_seed"][r]
        assert a["repetitions"] == t[k + "_repetitions"][r]
        for f in ["pos", "edges", "node_edges", "neighbors", "apsp"]:
            np.testing.assert_array_equal(a[f], t[k + "_" + f][r], err_msg=f)
    np.testing.assert_array_equal([m.next32() for _ in range(4)], t[k + "_post_raw"])


def test_fixed_topologies_and_seed_lists(oracle_mod):
    t = np.load(f"{R.GOLDEN}/topology.npz")
    for s in t["fixed_seeds"]:
        cfg = oracle_mod.make_config(20, 1, topo_mode=oracle_mod.TOPO_FIXED, topo_seed=int(s))
        seed, tp = oracle_mod.create_valid(cfg, oracle_mod.MTStream(0))
        a = tp.arrays()
        assert seed == s
        np.testing.assert_array_equal(a["edges"], t[f"fixed_{s}_edges"])
        np.testing.assert_array_equal(a["apsp"], t[f"fixed_{s}_apsp"])
    for key in [k for k in t.files if k.startswith("seedlist_")]:
        _, n, i = key.split("_")
        got = oracle_mod.build_seed_list(int(n[1:]), int(i[1:]), len(t[key]))
        np.testing.assert_array_equal(got, t[key])


class OracleAdapter:
    def __init__(self, oracle_mod, cfg, spec):
        O = oracle_mod
        mode, seed, lst = spec
        m = {"fixed": O.TOPO_FIXED, "random": O.TOPO_RANDOM, "list": O.TOPO_LIST,
             "sequential": O.TOPO_SEQUENTIAL}[mode]
        self.c = O.make_config(int(cfg["n"]), int(cfg["a"]), bool(cfg["cong"]), bool(cfg["mask"]), int(cfg["ttl"]),
                               m, seed, seed_list=lst,
                               excluded=R.EVAL_SEEDS if mode in ("random", "list") else None,
                               env_var=int(cfg.get("var", 1)))
        self.env = O.OracleEnv(self.c, int(cfg["seed"]))

    def reset(self):
        self.env.reset()

    def egreedy(self, q, eps):
        return self.env.draw_egreedy(q, eps)

    def step(self, a):
        return self.env.step(a)

    def state(self):
        return self.env.state()

    def observe(self):
        return self.env.observe()

    def final_delays(self):
        return self.env.final_delays()


@pytest.mark.parametrize("path", R.env_golden_files(), ids=lambda p: p.split("/")[-1])
def test_env_trace_bit_exact(oracle_mod, path):
    n = R.replay(path, lambda cfg, spec: OracleAdapter(oracle_mod, cfg, spec))
    assert n > 10


def test_netmon_restatement_matches_reference():
    g = np.load(f"{R.GOLDEN}/netmon.npz")
    for vi, v in enumerate(g["variants"]):
        rnn, agg, K = v.split("|")[:3]
        W = netmon_ref.weights_from_npz(g, f"v{vi}_w_")
        state = None
        for t in range(3):
            out, state = netmon_ref.netmon_forward(W, g["node_obs"][t], g["node_adj"][t], state, rnn, agg, int(K))
            np.testing.assert_allclose(out, g[f"v{vi}_h_{t}"], atol=1e-5, rtol=0)
            np.testing.assert_allclose(state, g[f"v{vi}_state_{t}"], atol=1e-5, rtol=0)
            mapped = netmon_ref.to_network_obs(out, g["node_agent"][t])
            np.testing.assert_allclose(mapped, g[f"v{vi}_mapped_{t}"], atol=1e-5, rtol=0)
    W = netmon_ref.weights_from_npz(g, "dqn_w_")
    np.testing.assert_allclose(netmon_ref.dqn_forward(W, g["dqn_obs"]), g["dqn_q"], atol=1e-5, rtol=0)


def test_oracle_bench_driver_runs(oracle_mod):
    cfg = oracle_mod.make_config(20, 20, topo_mode=oracle_mod.TOPO_RANDOM, excluded=R.EVAL_SEEDS)
    sec, obs, nobs = oracle_mod.bench_rollout(cfg, 16, 60, 50, 2)
    assert sec > 0 and obs.shape == (16, 20, 130) and nobs.shape == (16, 20, 88)
    # every agent observation has exactly one "now" and one "target" one-hot
    assert (obs[..., :20].sum(-1) == 1).all() and (obs[..., 20:40].sum(-1) == 1).all()


@pytest.mark.parametrize("name", ["train.npz", "train_big.npz", "train_prod.npz", "train_lnlstm.npz", "train_gru.npz", "train_relu.npz",
                                  "train_elu.npz", "train_tanh.npz", "train_sigmoid.npz",
                                  "train_softplus.npz", "train_gelu.npz", "train_silu.npz", "train_mish.npz"])
def test_train_golden_forward_matches_restatement(name):
    """The golden DQN+NetMon updates' Q / Q-target / loss follow from their weights (stored, or for
    the compact production-size golden regenerated by tests/golden/detparams.py) through the fp64
    restatement — pins the fixtures and the detparams regeneration itself."""
    import golden_update as GU

    g = np.load(f"{R.GOLDEN}/{name}")
    Wn, Wm, Wt, state = GU.weights_np(g)
    rnn, agg, K, H, enc, dq = GU.arch(g)
    act = GU.activation(g)
    tot, L = 0.0, g["actions"].shape[0]
    gamma = float(g["gamma"])
    for t in range(L):
        out, ns = netmon_ref.netmon_forward(Wn, g["node_obs"][t], g["node_adj"][t], state, rnn, agg, K, act=act)
        obs = np.concatenate([g["agent_obs"][t], netmon_ref.to_network_obs(out, g["node_agent"][t])], -1)
        q = netmon_ref.dqn_forward(Wm, obs, act=act)
        out2, _ = netmon_ref.netmon_forward(Wn, g["node_obs"][t + 1], g["node_adj"][t + 1], ns, rnn, agg, K, act=act)
        nobs = np.concatenate([g["agent_obs"][t + 1], netmon_ref.to_network_obs(out2, g["node_agent"][t + 1])], -1)
        nq = netmon_ref.dqn_forward(Wt, nobs, act=act).max(-1)
        qt = q.copy()
        tgt = g["reward"][t] + (1 - g["done"][t]) * gamma * nq
        np.put_along_axis(qt, g["actions"][t][..., None].astype(np.int64), tgt[..., None], -1)
        np.testing.assert_allclose(q, g[f"q_{t}"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(qt, g[f"qtarget_{t}"], atol=1e-5, rtol=0)
        tot += ((q - qt) ** 2).mean() / L
        state = ns * (1 - g["episode_done"][t])[:, None, None]
    np.testing.assert_allclose(tot, g["loss"].item(), rtol=1e-6)


@pytest.mark.parametrize("name", ["dgn", "dgn_small", "dqnr", "commnet"])
def test_agent_model_restatement_matches_reference(name):
    """oracle/models_ref.py (fp64) vs the reference's DGN / DQNR / CommNet forwards."""
    import models_ref as MR

    g = np.load(os.path.join(R.GOLDEN, "models.npz"))
    W = {k[len(name) + 3:]: g[k].astype(np.float64) for k in g.files if k.startswith(name + "_w_")}
    state = None
    for t in range(3):
        x, adj = g["obs"][t].astype(np.float64), g["adj"][t].astype(np.float64)
        if name.startswith("dgn"):
            heads = g[f"{name}_att0_{t}"].shape[1]
            q, atts = MR.dgn(W, x, adj, heads)
            for li, w in enumerate(atts):
                np.testing.assert_allclose(w, g[f"{name}_att{li}_{t}"], atol=5e-6, rtol=0)
        else:
            if t > 0:
                np.testing.assert_allclose(state, g[f"{name}_statein_{t}"], atol=5e-6, rtol=0)
            f = MR.dqnr if name == "dqnr" else (lambda W, x, s: MR.commnet(W, x, adj, s))
            q, st = f(W, x, state)
            np.testing.assert_allclose(st, g[f"{name}_state_{t}"], atol=5e-6, rtol=0)
            state = st * (1 - g["done"][t][..., None])
        np.testing.assert_allclose(q, g[f"{name}_q_{t}"], atol=5e-6, rtol=0)


def _log_softmax(x):
    m = x.max(-1, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(-1, keepdims=True))


@pytest.mark.parametrize("name", ["dgn", "dqnr", "commnet"])
def test_model_update_golden_reproduced_by_fp64_restatement(name):
    """Pins tests/golden/train_{dgn,dqnr,commnet}.npz (make_golden.py gen_train_models):
    the fp64 restatement (oracle/models_ref.py) replays the reference's update loop (src/main.py:840-964
    with netmon None) on the fixture's inputs: q, q_target, the TD loss and DGN's attention KL (KL(softmax
    target || softmax online) per source agent, summed over layers / heads / destinations, averaged over the
    agents that are not done)."""
    import models_ref as MR

    g = np.load(os.path.join(R.GOLDEN, f"train_{name}.npz"))
    W = lambda p: {k[len(p):]: g[k].astype(np.float64) for k in g.files  # noqa: E731
                   if k.startswith(p) and not k.startswith(p + "after_")}
    Wm, Wt = W("model_"), W("target_")
    L, gamma = g["actions"].shape[0], float(g["gamma"])
    state = g["agent_state0"].astype(np.float64) if "agent_state0" in g.files else None
    loss_q = loss_att = 0.0
    for t in range(L):
        x, adj = g["agent_obs"][t].astype(np.float64), g["agent_adj"][t].astype(np.float64)
        xn, adjn = g["agent_obs"][t + 1].astype(np.float64), g["agent_adj"][t + 1].astype(np.float64)
        done = g["done"][t].astype(bool)
        if name == "dgn":
            q, att = MR.dgn(Wm, x, adj, 4)
            qn, att_t = MR.dgn(Wt, xn, adjn, 4)
            lp = _log_softmax(np.stack(att))
            pt = np.exp(_log_softmax(np.stack(att_t)))
            kl = (pt * (np.log(np.maximum(pt, 1e-300)) - lp)).sum(-1).sum(axis=(0, 2))  # (B, A)
            loss_att += (kl * ~done).sum() / max(int((~done).sum()), 1) / L
        else:
            f = MR.dqnr if name == "dqnr" else MR.commnet
            q, st = f(Wm, x, state) if name == "dqnr" else f(Wm, x, adj, state)
            qn, _ = f(Wt, xn, st) if name == "dqnr" else f(Wt, xn, adjn, st)
            state = st * (~done * ~g["episode_done"][t].astype(bool)[:, None])[..., None]
        tgt = g["reward"][t] + (~done) * gamma * qn.max(-1)
        qt = q.copy()
        np.put_along_axis(qt, g["actions"][t].astype(np.int64)[..., None], tgt[..., None], -1)
        np.testing.assert_allclose(q, g[f"q_{t}"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(qt, g[f"qtarget_{t}"], atol=1e-5, rtol=0)
        loss_q += ((q - qt) ** 2).mean() / L
    np.testing.assert_allclose(loss_q, g["loss_q"].item(), rtol=1e-5)
    np.testing.assert_allclose(loss_att, g["loss_att"].item(), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(loss_q + float(g["att_coeff"]) * loss_att, g["loss"].item(), rtol=1e-5)
    if name == "dgn":
        assert loss_att > 1e-3  # the fixture exercises the regulariser (perturbed target attention)


def test_netmon_global_restatement_matches_reference():
    """--netmon-global readout of the fp64 restatement vs the reference (netmon_global.npz)."""
    g = np.load(os.path.join(R.GOLDEN, "netmon_global.npz"))
    for vi, K in enumerate((1, 2)):
        W = {k[len(f"v{vi}_w_"):]: g[k].astype(np.float64) for k in g.files if k.startswith(f"v{vi}_w_")}
        state = None
        for t in range(3):
            out, state = netmon_ref.netmon_forward(W, g["node_obs"][t], g["node_adj"][t], state, "lstm", "sum", K,
                                                   global_h=True)
            mapped = netmon_ref.to_network_obs(out, g["node_agent"][t])
            np.testing.assert_allclose(mapped, g[f"v{vi}_mapped_{t}"], atol=5e-6, rtol=0)
            np.testing.assert_allclose(state, g[f"v{vi}_state_{t}"], atol=5e-6, rtol=0)


def test_netmon_nocarry_restatement_matches_reference():
    """--netmon-rnn-carryover 0 (lstm / lnlstm / gru) of the fp64 restatement vs the reference
    (netmon_nocarry.npz): agent-mapped readout and the 2x state over 3 carried steps."""
    g = np.load(os.path.join(R.GOLDEN, "netmon_nocarry.npz"))
    for vi, v in enumerate(g["variants"]):
        rnn, K = str(v).split(":")
        W = {k[len(f"v{vi}_w_"):]: g[k].astype(np.float64) for k in g.files if k.startswith(f"v{vi}_w_")}
        state = None
        for t in range(3):
            out, state = netmon_ref.netmon_forward(W, g["node_obs"][t], g["node_adj"][t], state, rnn, "sum", int(K),
                                                   carryover=False)
            assert state.shape[-1] == int(g[f"v{vi}_state_size"])
            mapped = netmon_ref.to_network_obs(out, g["node_agent"][t])
            np.testing.assert_allclose(mapped, g[f"v{vi}_mapped_{t}"], atol=5e-6, rtol=0)
            np.testing.assert_allclose(state, g[f"v{vi}_state_{t}"], atol=5e-6, rtol=0)
