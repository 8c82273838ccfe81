"""GPU parity: the HIP routing env vs the reference (golden traces) and vs the C
oracle on many envs at once. Bar: bit-exact for every integer, fp64 load and fp32
observation."""
import numpy as np
import pytest
import torch

import golden_replay as R

pytestmark = pytest.mark.gpu


class DeviceAdapter:
    """Drives one env of a graph-marl_amd Routing batch through the replay interface."""

    def __init__(self, gm, cfg, spec, n_env=1):
        mode, seed, lst = spec
        n, a = int(cfg["n"]), int(cfg["a"])
        if mode == "fixed":
            net = gm.Network(n, random_topology=False, topology_init_seed=seed)
        elif mode == "random":
            net = gm.Network(n, random_topology=True, topology_init_seed=seed, excluded_seeds=gm.EVAL_SEEDS)
        elif mode == "list":  # built on the device by build_seed_list, like the reference
            net = gm.Network(n, random_topology=True, n_random_seeds=5, topology_init_seed=seed,
                             excluded_seeds=gm.EVAL_SEEDS)
            assert list(net.seeds) == [int(s) for s in lst]
        else:
            net = gm.Network(n, random_topology=True, provided_seeds=[int(s) for s in lst],
                             sequential_topology_seeds=True)
        self.env = gm.Routing(net, a, int(cfg.get("var", 1)), enable_congestion=bool(cfg["cong"]),
                              enable_action_mask=bool(cfg["mask"]),
                              ttl=int(cfg["ttl"]), n_env=n_env, seed=int(cfg["seed"]))
        self.gm = gm
        self.A = a
        dev = self.env.device
        self.detail = dict(done_steps=torch.zeros(n_env, a, dtype=torch.int32, device=dev),
                           done_opt=torch.zeros(n_env, a, dtype=torch.int32, device=dev),
                           success=torch.zeros(n_env, a, dtype=torch.uint8, device=dev))

    def reset(self):
        self.env.reset_()

    def egreedy(self, q, eps):
        from importlib import import_module

        L = import_module("graph-marl_amd._lib")
        qt = torch.as_tensor(np.asarray(q, np.float32), device=self.env.device).reshape(1, self.A, 4).contiguous()
        act = torch.zeros(1, self.A, dtype=torch.int32, device=self.env.device)
        L.check(L.lib().gm_policy_egreedy(self.env._h, L.ptr(qt), float(eps), L.ptr(act), L.stream_ptr()))
        return act[0].cpu().numpy().astype(np.int64)

    def step(self, a):
        act = torch.as_tensor(np.asarray(a, np.int32), device=self.env.device).reshape(1, self.A)
        self.env.step_(act, self.detail)
        rew = self.env.reward[0].cpu().numpy()
        done = self.env.done[0].cpu().numpy().astype(bool)
        inf = self.env.info[0].cpu().numpy()
        ds = self.detail["done_steps"][0].cpu().numpy()
        dop = self.detail["done_opt"][0].cpu().numpy()
        suc = self.detail["success"][0].cpu().numpy().astype(bool)
        delays = [float(ds[i]) for i in range(self.A) if done[i]]
        arrived = [float(ds[i]) for i in range(self.A) if done[i] and suc[i]]
        spr = [float(ds[i]) / float(dop[i]) for i in range(self.A) if done[i] and suc[i]]
        info = dict(looped=inf[0], throughput=int(inf[1]), dropped=int(inf[2]), blocked=int(inf[3]),
                    delays=delays, delays_arrived=arrived, spr=spr)
        assert inf[4] == len(delays) and inf[5] == sum(delays) and inf[6] == len(arrived)
        assert inf[7] == sum(arrived)
        return rew, done, info

    def state(self, b=0):
        s = self.env.get_state()
        out = {k: s[k][b] for k in ["now", "target", "edge", "time", "ttl", "start", "spw", "size", "visited",
                                    "loads", "amask"]}
        out = {k: (v.astype(np.int64) if v.dtype == np.int32 else v) for k, v in out.items()}
        out["agent_steps"] = s["agent_steps"][b].astype(np.float64)
        out["topo_seed"] = int(s["topo_seed"][b])
        return out

    def observe(self, b=0):
        e = self.env
        torch.cuda.synchronize()
        return dict(obs=e.obs[b].cpu().numpy(), node_obs=e.node_obs[b].cpu().numpy(),
                    adj=e.agent_adj[b].cpu().numpy(), node_agent=e.get_node_agent_matrix()[b].cpu().numpy())

    def final_delays(self, b=0):
        st = self.env.get_state()["agent_steps"][b]
        return [float(x) for x in st if x != 0]


@pytest.mark.parametrize("path", R.env_golden_files(), ids=lambda p: p.split("/")[-1])
def test_golden_trace_on_device(gm, path):
    n = R.replay(path, lambda cfg, spec: DeviceAdapter(gm, cfg, spec))
    assert n > 10


def test_build_seed_list_reproduces_eval_seeds(gm):
    got = gm.build_seed_list(20, 476, 1000)
    np.testing.assert_array_equal(np.array(got), np.load(f"{R.GOLDEN}/eval_seeds.npy"))


def _oracle_env(oracle_mod, n, a, mode, topo_seed, seed, cong=True, mask=False, ttl=0, lst=None, var=1, k=3):
    O = oracle_mod
    m = {"fixed": O.TOPO_FIXED, "random": O.TOPO_RANDOM, "list": O.TOPO_LIST, "sequential": O.TOPO_SEQUENTIAL}[mode]
    c = O.make_config(n, a, cong, mask, ttl, m, topo_seed, seed_list=lst,
                      excluded=R.EVAL_SEEDS if mode in ("random", "list") else None, env_var=var, k=k)
    e = O.OracleEnv(c, seed)
    e._cfg_keep = c
    return e


BATCH_CASES = [
    # n, a, mode, congestion, mask, ttl, n_env, steps, episode
    (20, 20, "random", True, False, 0, 48, 120, 50),
    (20, 20, "fixed", True, False, 0, 32, 150, 300),
    (10, 30, "random", False, False, 0, 24, 80, 40),
    (64, 64, "random", True, False, 0, 8, 60, 30),
    (50, 20, "random", True, True, 12, 16, 90, 45),
    (4, 1, "random", True, False, 0, 16, 40, 20),
    # config-4 node counts around the 32-node LDS image of the reset (k_env_reset<32>)
    (30, 20, "random", True, False, 0, 24, 110, 50),
    (32, 20, "random", True, False, 0, 16, 80, 40),
    (34, 20, "random", True, False, 0, 8, 60, 30),
    (40, 20, "random", True, False, 0, 16, 110, 50),
    (100, 20, "random", True, False, 0, 8, 60, 30),
    (128, 64, "random", True, True, 16, 4, 40, 20),
    # observation variants: (env_var, k) as an optional 10th element
    (20, 20, "random", True, False, 0, 16, 60, 30, (2, 3)),
    (12, 40, "random", True, False, 0, 8, 40, 20, (2, 8)),
    (20, 20, "fixed", True, False, 0, 8, 40, 20, (2, 0)),
    (10, 12, "random", True, False, 0, 8, 40, 20, (3, 3)),
    (64, 8, "random", True, False, 0, 4, 20, 10, (3, 3)),
]


@pytest.mark.parametrize("case", BATCH_CASES,
                         ids=lambda c: f"n{c[0]}a{c[1]}{c[2]}e{c[6]}" + (f"v{c[9][0]}k{c[9][1]}" if len(c) > 9 else ""))
def test_batch_vs_oracle(gm, oracle_mod, case):
    n, a, mode, cong, mask, ttl, B, T, ep = case[:9]
    var, k = case[9] if len(case) > 9 else (1, 3)
    if mode == "fixed":
        net = gm.Network(n, random_topology=False, topology_init_seed=476)
    else:
        net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    seeds = [(7919 * b + 17) & 0xFFFFFFFF for b in range(B)]
    env = gm.Routing(net, a, var, k=k, enable_congestion=cong, enable_action_mask=mask, ttl=ttl, n_env=B, seeds=seeds)
    orc = [_oracle_env(oracle_mod, n, a, mode, 476, s, cong, mask, ttl, var=var, k=k) for s in seeds]
    assert env.obs_dim == orc[0].obs_dim()
    rng = np.random.RandomState(123)
    env.reset_()
    for o in orc:
        o.reset()

    def compare(tag):
        st = env.get_state()
        torch.cuda.synchronize()
        obs = env.obs.cpu().numpy()
        nobs = env.node_obs.cpu().numpy()
        adj = env.agent_adj.cpu().numpy()
        for b, o in enumerate(orc):
            s = o.state()
            for k in ["now", "target", "edge", "time", "ttl", "start", "spw"]:
                np.testing.assert_array_equal(st[k][b], s[k], err_msg=f"{tag} env {b} {k}")
            np.testing.assert_array_equal(st["size"][b].view(np.uint64), s["size"].view(np.uint64))
            np.testing.assert_array_equal(st["loads"][b].view(np.uint64), s["loads"].view(np.uint64),
                                          err_msg=f"{tag} env {b} loads")
            np.testing.assert_array_equal(st["agent_steps"][b], s["agent_steps"])
            np.testing.assert_array_equal(st["visited"][b], s["visited"], err_msg=f"{tag} env {b} visited")
            assert st["topo_seed"][b] == s["topo_seed"]
            np.testing.assert_array_equal(st["rng_key"][b], s["rng_key"], err_msg=f"{tag} env {b} rng")
            assert st["rng_pos"][b] == s["rng_pos"]
            ob = o.observe()
            np.testing.assert_array_equal(obs[b], ob["obs"], err_msg=f"{tag} env {b} obs")
            np.testing.assert_array_equal(nobs[b], ob["node_obs"], err_msg=f"{tag} env {b} node obs")
            np.testing.assert_array_equal(adj[b], ob["adj"], err_msg=f"{tag} env {b} adj")

    compare("reset")
    for t in range(1, T + 1):
        act = rng.randint(4, size=(B, a)).astype(np.int32)
        env.step_(torch.as_tensor(act, device=env.device))
        rew = env.reward.cpu().numpy()
        done = env.done.cpu().numpy()
        for b, o in enumerate(orc):
            r, d, _ = o.step(act[b])
            np.testing.assert_array_equal(rew[b].view(np.uint32), r.view(np.uint32), err_msg=f"step {t} env {b}")
            np.testing.assert_array_equal(done[b].astype(bool), d)
        if t % 10 == 0 or t < 4:
            compare(f"step {t}")
        if t % ep == 0:
            env.reset_()
            for o in orc:
                o.reset()
            compare(f"reset at {t}")


def test_egreedy_batch_vs_oracle(gm, oracle_mod):
    B, n, a = 64, 20, 20
    net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    seeds = list(range(100, 100 + B))
    env = gm.Routing(net, a, 1, n_env=B, seeds=seeds)
    orc = [_oracle_env(oracle_mod, n, a, "random", 476, s) for s in seeds]
    env.reset_()
    for o in orc:
        o.reset()
    from importlib import import_module

    L = import_module("graph-marl_amd._lib")
    rng = np.random.RandomState(9)
    act = torch.zeros(B, a, dtype=torch.int32, device=env.device)
    for t in range(40):  # 40 x 60 draws: crosses several MT blocks
        q = rng.standard_normal((B, a, 4)).astype(np.float32)
        eps = [0.0, 0.3, 1.0][t % 3]
        qt = torch.as_tensor(q, device=env.device)
        L.check(L.lib().gm_policy_egreedy(env._h, L.ptr(qt), eps, L.ptr(act), L.stream_ptr()))
        got = act.cpu().numpy()
        for b, o in enumerate(orc):
            np.testing.assert_array_equal(got[b], o.draw_egreedy(q[b], eps), err_msg=f"t {t} env {b}")
        env.step_(act)
        for b, o in enumerate(orc):
            o.step(got[b])
    st = env.get_state()
    for b, o in enumerate(orc):
        np.testing.assert_array_equal(st["rng_key"][b], o.state()["rng_key"])


@pytest.mark.parametrize("mask,ttl", [(False, 0), (True, 9)])
def test_policy_step_fused_matches_split(gm, oracle_mod, mask, ttl):
    """gm_env_policy_step (ε-greedy as the env step kernel's prologue) == gm_policy_egreedy +
    gm_env_step, bit for bit: actions, rewards, done, info, observations and the whole env state
    incl. the MT streams, over 120 steps with resets every 50 (respawn draws after the policy's
    draws in one kernel); the actions also match the oracle's draws on a sample of envs."""
    B, n, a = 256, 20, 20
    net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    seeds = list(range(300, 300 + B))
    kw = dict(enable_action_mask=mask, ttl=ttl, n_env=B, seeds=seeds)
    ea, eb = gm.Routing(net, a, 1, **kw), gm.Routing(net, a, 1, **kw)
    sample = [0, 5, 255]
    orc = [_oracle_env(oracle_mod, n, a, "random", 476, seeds[b], mask=mask, ttl=ttl) for b in sample]
    from importlib import import_module

    L = import_module("graph-marl_amd._lib")
    rng = np.random.RandomState(17)
    act_a = torch.zeros(B, a, dtype=torch.int32, device=ea.device)
    act_b = torch.zeros_like(act_a)
    for t in range(120):
        if t % 50 == 0:
            ea.reset_()
            eb.reset_()
            for o in orc:
                o.reset()
        q = rng.standard_normal((B, a, 4)).astype(np.float32)
        eps = [0.0, 0.3, 1.0][t % 3]
        qt = torch.as_tensor(q, device=ea.device)
        L.check(L.lib().gm_policy_egreedy(ea._h, L.ptr(qt), eps, L.ptr(act_a), L.stream_ptr()))
        ea.step_(act_a)
        eb.policy_step_(qt, eps, act_b)
        got = act_b.cpu().numpy()
        np.testing.assert_array_equal(got, act_a.cpu().numpy(), err_msg=f"actions t {t}")
        for name in ("reward", "done", "info", "obs_buf", "node_obs", "nbr", "agent_node"):
            x, y = getattr(ea, name), getattr(eb, name)
            assert torch.equal(x, y), f"{name} differs at t {t}"
        for i, o in zip(sample, orc):
            want = o.draw_egreedy(q[i], eps)  # the oracle's draws ignore the action mask
            if not mask:
                np.testing.assert_array_equal(got[i], want, err_msg=f"oracle t {t} env {i}")
            o.step(got[i])
    sa, sb = ea.get_state(), eb.get_state()
    for k in sa:
        np.testing.assert_array_equal(np.asarray(sa[k]), np.asarray(sb[k]), err_msg=f"state {k}")
    for i, o in zip(sample, orc):
        np.testing.assert_array_equal(sb["rng_key"][i], o.state()["rng_key"])


@pytest.mark.parametrize("n", [20, 30])
def test_obs_gemm_copy(gm, n):
    """gm_obs_buffers.obs_gemm (the fused DQN's env operand) == the agent obs without columns N-1
    and 2N, after reset, steps and a late enable_gemm_obs (filled from the current state)."""
    B, a = 64, 20
    net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    env = gm.Routing(net, a, 1, n_env=B, seed=11)
    keep = [c for c in range(6 * n + 10) if c not in (n - 1, 2 * n)]
    rng = np.random.RandomState(5)
    env.reset_()
    env.step_(torch.as_tensor(rng.randint(0, 4, (B, a)), dtype=torch.int32, device=env.device))
    g = env.enable_gemm_obs()
    assert torch.equal(g, env.obs[..., keep])
    for t in range(60):
        if t == 30:
            env.reset_()
        env.step_(torch.as_tensor(rng.randint(0, 4, (B, a)), dtype=torch.int32, device=env.device))
        assert torch.equal(env.obs_gemm, env.obs[..., keep]), f"step {t}"


def test_large_batch_invariants(gm, oracle_mod):
    """4096 envs (the benchmark size): conservation laws every step, and a sample of
    envs replayed bit-exactly on the oracle."""
    B, n, a, T = 4096, 20, 20, 150
    net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    env = gm.Routing(net, a, 1, n_env=B, seed=1, agent_adjacency=False)
    sample = [0, 1, 777, 2048, 4095]
    orc = [_oracle_env(oracle_mod, n, a, "random", 476, 1 + b) for b in sample]
    env.reset_()
    for o in orc:
        o.reset()
    g = torch.Generator(device=env.device)
    g.manual_seed(5)
    for t in range(1, T + 1):
        act = torch.randint(0, 4, (B, a), device=env.device, dtype=torch.int32, generator=g)
        env.step_(act)
        actn = act[sample].cpu().numpy()
        for i, o in enumerate(orc):
            o.step(actn[i])
        if t % 50 == 0:
            env.reset_()
            for o in orc:
                o.reset()
        if t % 25 == 0:
            st = env.get_state()
            # load of every edge = sizes of the packets on it (up to fp64 rounding of +/- sequences)
            E = 3 * n // 2
            ref = np.zeros((B, E))
            on = st["edge"] >= 0
            bi, ai = np.nonzero(on)
            np.add.at(ref, (bi, st["edge"][bi, ai]), st["size"][bi, ai])
            assert np.abs(ref - st["loads"]).max() < 1e-9
            assert (st["loads"] <= 1.0 + 1e-12).all()
            obs = env.obs.cpu().numpy()
            assert (obs[..., :n].sum(-1) == 1).all() and (obs[..., n:2 * n].sum(-1) == 1).all()
            nobs = env.node_obs.cpu().numpy()
            assert (nobs[..., n] .sum(-1) == (st["edge"] < 0).sum(-1)).all()
            for i, (b, o) in enumerate(zip(sample, orc)):
                s = o.state()
                np.testing.assert_array_equal(st["now"][b], s["now"])
                np.testing.assert_array_equal(st["loads"][b].view(np.uint64), s["loads"].view(np.uint64))
                np.testing.assert_array_equal(obs[b], o.observe()["obs"])


@pytest.mark.parametrize("n", [10, 20, 30, 40, 50, 100])
def test_topology_from_seed_matches_reference_golden(gm, n):
    """Topologies generated on the device from the reference's recorded (valid) seeds:
    edges in creation order, lengths, APSP and the I+A adjacency (get_nodes_adjacency,
    src/env/network.py:385-389) equal the reference's networkx output
    (tests/golden/topology.npz, rand_n*), N = 10..50 (BASELINE config 4) and 100 (config 5)."""
    g = np.load(f"{R.GOLDEN}/topology.npz")
    seeds = g[f"rand_n{n}_seed"]
    B = len(seeds)
    env = gm.Routing(gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 4, n_env=B, seed=1)
    env.set_topology_seeds(seeds, sequential=True, interleave=True)
    env.reset_()
    st = env.get_state()
    E = 3 * n // 2
    for b in range(B):
        ge = g[f"rand_n{n}_edges"][b]
        np.testing.assert_array_equal(st["edge_a"][b, :E], ge[:, 0], err_msg=f"n={n} topology {b}")
        np.testing.assert_array_equal(st["edge_b"][b, :E], ge[:, 1])
        np.testing.assert_array_equal(st["edge_len"][b, :E], ge[:, 2])
        np.testing.assert_array_equal(st["apsp"][b], g[f"rand_n{n}_apsp"][b])
        assert st["topo_seed"][b] == seeds[b]
    adj = env.get_nodes_adjacency().cpu().numpy()
    np.testing.assert_array_equal(adj, g[f"rand_n{n}_adj"].astype(np.int8))


def test_set_state_restores_a_dump(gm, oracle_mod):
    """gm_env_set_state (Routing.set_state) restores a get_state() dump into an env created with
    other seeds: observations are re-emitted identically and the next 40 steps (with resets of
    done packets drawing from the restored numpy streams) match the original env bit for bit;
    a dump taken from the C oracle (same state layout) restores into the device env too."""
    n, a, B = 20, 20, 12
    net = gm.Network(n, random_topology=True, excluded_seeds=R.EVAL_SEEDS)
    e1 = gm.Routing(net, a, n_env=B, seed=5)
    e2 = gm.Routing(net, a, n_env=B, seed=900)
    e1.reset_()
    e2.reset_()
    rng = np.random.RandomState(0)
    for _ in range(25):
        e1.step_(torch.as_tensor(rng.randint(4, size=(B, a)), dtype=torch.int32, device="cuda"))
    dump = e1.get_state()
    e2.set_state(dump)
    np.testing.assert_array_equal(e2.obs_buf.cpu().numpy(), e1.obs_buf.cpu().numpy())
    np.testing.assert_array_equal(e2.node_obs.cpu().numpy(), e1.node_obs.cpu().numpy())
    np.testing.assert_array_equal(e2.nbr.cpu().numpy(), e1.nbr.cpu().numpy())
    for _ in range(40):
        act = torch.as_tensor(rng.randint(4, size=(B, a)), dtype=torch.int32, device="cuda")
        e1.step_(act)
        e2.step_(act)
    s1, s2 = e1.get_state(), e2.get_state()
    for k in s1:
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)
    np.testing.assert_array_equal(e2.obs_buf.cpu().numpy(), e1.obs_buf.cpu().numpy())
    # oracle -> device: one oracle env advanced 30 steps, its packet/load/stream state written
    # into env 0 of e2 (topology taken from the oracle as well)
    cfg = oracle_mod.make_config(n, a, topo_mode=oracle_mod.TOPO_RANDOM, excluded=R.EVAL_SEEDS)
    o = oracle_mod.OracleEnv(cfg, 77)
    o.reset()
    for _ in range(30):
        o.step(rng.randint(4, size=a))
    os_, ot = o.state(), o.topology()
    d = e2.get_state()
    for k in ("now", "target", "edge", "time", "ttl", "start", "spw", "agent_steps", "size", "visited", "amask"):
        d[k][0] = os_[k]
    E = 3 * n // 2
    d["loads"][0] = os_["loads"]
    d["topo_seed"][0] = os_["topo_seed"]
    d["edge_a"][0], d["edge_b"][0], d["edge_len"][0] = ot["edges"][:E, 0], ot["edges"][:E, 1], ot["edges"][:E, 2]
    d["nbr_edge"][0] = ot["node_edges"]
    d["apsp"][0] = ot["apsp"]
    d["rng_key"][0], d["rng_pos"][0] = os_["rng_key"], os_["rng_pos"]
    e2.set_state(d)
    for t in range(30):
        act = rng.randint(4, size=(B, a))
        o.step(act[0])
        e2.step_(torch.as_tensor(act, dtype=torch.int32, device="cuda"))
        np.testing.assert_array_equal(e2.obs_buf[0, :, : 6 * n + 10].cpu().numpy(), o.observe()["obs"],
                                      err_msg=f"step {t}")


def test_set_state_restores_the_topology_seed_list_position(gm):
    """gm_env_state.seq_index: the position in a sequential topology-seed list
    (Network.sequential_topology_index, src/env/network.py:356-371) survives a dump/restore, so a
    restored env walks the list from the same place (the EVAL_SEEDS walk of evaluation)."""
    n, a, B = 20, 20, 4
    seeds = [int(s) for s in R.EVAL_SEEDS[:9]]

    def make(seed):
        e = gm.Routing(gm.Network(n, random_topology=True, excluded_seeds=None), a, n_env=B, seed=seed)
        e.set_topology_seeds(seeds, sequential=True)
        return e

    e1, e2 = make(5), make(6)
    for _ in range(4):
        e1.reset_()
    d = e1.get_state()
    assert (d["seq_index"] == 4 % len(seeds)).all()
    e2.reset_()
    e2.set_state(d)
    assert (e2.get_state()["seq_index"] == d["seq_index"]).all()
    for k in range(7):  # both walk on from position 4 (wrapping past the list end)
        e1.reset_()
        e2.reset_()
        s1, s2 = e1.get_state(), e2.get_state()
        assert (s1["topo_seed"] == seeds[(4 + k) % len(seeds)]).all()
        np.testing.assert_array_equal(s1["topo_seed"], s2["topo_seed"])
        np.testing.assert_array_equal(s1["edge_a"], s2["edge_a"])
        np.testing.assert_array_equal(s1["seq_index"], s2["seq_index"])
