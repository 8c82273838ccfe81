"""GPU tests of the vectorised rollout driver (graph-marl_amd/rollout.py): env groups on
separate HIP streams give the same trajectories as each group run alone, and the HIP-graph
replay gives the same trajectories as eager launches (bit-exact: same kernels, same
inputs, only the launch mechanism differs)."""
import importlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, A, B = 20, 20, 8


def build(groups, seed=0, episode_steps=10, n_env=B, K=2, epsilon=0.3, netmon=True, **kw):
    """netmon False: BASELINE config 2 (no NetMon, the DQN on the env obs, fixed topology)."""
    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    RO = importlib.import_module("graph-marl_amd.rollout")
    net = gm.Network(N, random_topology=netmon, excluded_seeds=gm.EVAL_SEEDS, device=0)
    torch.manual_seed(3)
    netmon = M.NetMon(4 * N + 8, 128, [512, 256], K).cuda() if netmon else None
    dqn = M.DQN(6 * N + 10 + (netmon.get_out_features() if netmon is not None else 0), [512, 256], 4).cuda()
    return RO.StreamedRollout(net, A, n_env, netmon, dqn, groups=groups, seed=seed, epsilon=epsilon,
                              episode_steps=episode_steps, device=0, **kw)


def snapshot(ro):
    torch.cuda.synchronize()
    out = []
    for env, wenv in zip(ro.envs, ro.wenvs):
        st = env.get_state()
        out.append({"now": st["now"], "target": st["target"], "loads": st["loads"], "rng": st["rng_key"],
                    "obs": env.obs.cpu().numpy(), "reward": env.reward.cpu().numpy(),
                    "netmon": wenv.current_netmon_state.cpu().numpy() if hasattr(wenv, "netmon") else np.zeros(1)})
    return out


def cat(snaps):
    return {k: np.concatenate([s[k] for s in snaps]) for k in snaps[0]}


def assert_same(a, b):
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_groups_match_serial():
    """Two stream groups == the same envs as two separately-run single-group rollouts."""
    ro = build(2)
    ro.reset()
    ro.run(25)  # crosses two episode resets
    got = cat(snapshot(ro))
    parts = []
    # single-group rollouts over B/2 envs each, seeds as the group split assigns them
    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    RO = importlib.import_module("graph-marl_amd.rollout")
    net = gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS, device=0)
    for g in range(2):
        r1 = RO.StreamedRollout(net, A, B // 2, ro.wenvs[0].netmon, ro.policies[0]._model, groups=1,
                                seed=g * (B // 2), epsilon=0.3, episode_steps=10, device=0)
        r1.reset()
        r1.run(25)
        parts.append(cat(snapshot(r1)))
    assert_same(got, cat(parts))


def test_staggered_groups_match_serial():
    """stagger=True: group g resets g * episode_steps / groups steps out of phase; each group ==
    a single-group rollout that resets on the same steps."""
    gm = importlib.import_module("graph-marl_amd")
    RO = importlib.import_module("graph-marl_amd.rollout")
    base = build(2)
    net = gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS, device=0)
    ro = RO.StreamedRollout(net, A, B, base.wenvs[0].netmon, base.policies[0]._model, groups=2, seed=0,
                            epsilon=0.3, episode_steps=10, device=0, stagger=True)
    assert ro._offs == [0, 5]
    ro.reset()
    ro.run(27)
    got = cat(snapshot(ro))
    parts = []
    for g, off in enumerate(ro._offs):
        r1 = RO.StreamedRollout(net, A, B // 2, ro.wenvs[0].netmon, ro.policies[0]._model, groups=1,
                                seed=g * (B // 2), epsilon=0.3, episode_steps=10, device=0)
        r1.reset()
        for t in range(1, 28):
            r1._enqueue_step()
            if (t + off) % 10 == 0:
                with r1._on(0):
                    r1.wenvs[0].reset()
        parts.append(cat(snapshot(r1)))
    assert_same(got, cat(parts))


def test_stagger_refuses_graph_off_quantum():
    ro = build(2, stagger=True)  # offsets 0, 5: not multiples of a 2-step graph
    assert ro._offs == [0, 5]
    ro.reset()
    ro.step()
    ro.step()
    with pytest.raises(ValueError):
        ro.capture(2)


@pytest.mark.parametrize("per_group", [True, False])
def test_staggered_graph_replay_matches_eager(per_group):
    """Staggered episodes (group 1 resets 4 steps after group 0: offsets quantised to the 2-step graph)
    under graph replay == the same staggered rollout stepped eagerly, across several resets of each group."""
    eager = build(2, stagger=True, stagger_quantum=2)
    assert eager._offs == [0, 4]
    eager.reset()
    eager.run(4 + 40)
    ref = snapshot(eager)
    ro = build(2, stagger=True, stagger_quantum=2)
    ro.reset()
    for _ in range(4):
        ro.step()
    ro.capture(2, per_group=per_group)
    ro.run(40)
    for a, b in zip(snapshot(ro), ref):
        assert_same(a, b)


@pytest.mark.parametrize("per_group", [True, False])
@pytest.mark.parametrize("groups,gsteps,warm", [(1, 2, 4), (2, 2, 4), (2, 10, 10)])
def test_graph_replay_matches_eager(groups, gsteps, warm, per_group):
    """Replays cross episode resets (episode 10 steps), which run eagerly in between; one graph
    per group on its own stream (default) or every group in one graph."""
    eager = build(groups)
    eager.reset()
    eager.run(warm + 40)
    ref = snapshot(eager)

    ro = build(groups)
    ro.reset()
    for _ in range(warm):
        ro.step()
    ro.capture(gsteps, per_group=per_group)
    ro.run(40)
    assert (ro._graphs is not None and len(ro._graphs) == groups) if per_group else ro._graph is not None
    for a, b in zip(snapshot(ro), ref):
        assert_same(a, b)


def test_graph_replay_matches_eager_config2():
    """BASELINE config 2 (no NetMon: EpsilonGreedy.act on the env obs, the DQN as torch modules over the
    HIP GEMMs, fixed topology) under per-group graph replay, as bench.py times it: bit-identical to eager."""
    kw = dict(n_env=1024, epsilon=0.5, episode_steps=50, netmon=False)
    eager = build(2, **kw)
    eager.reset()
    eager.run(10 + 120)
    ref = snapshot(eager)
    ro = build(2, **kw)
    ro.reset()
    for _ in range(10):
        ro.step()
    ro.capture(10, per_group=True)
    ro.run(120)
    for a, b in zip(snapshot(ro), ref):
        assert_same(a, b)


def test_graph_replay_matches_eager_benched_size():
    """The headline's launch mode at the headline's size (bench.py defaults): 4096 envs in 2 stream
    groups, NetMon K = 1, ε = 0.5, 50-step episodes, one graph of 10 vector steps per group, 120
    replayed steps (two resets between replays). At 40 960 rows per group every GEMM runs the tiles
    the bench replays (LDS-DMA k_gemm3g forms), not the small-batch register-staged ones. Bit-identical
    to eager launches: env state, RNG keys, joint observations, rewards and NetMon states."""
    kw = dict(n_env=4096, K=1, epsilon=0.5, episode_steps=50)
    eager = build(2, **kw)
    eager.reset()
    eager.run(10 + 120)
    ref = snapshot(eager)
    del eager
    torch.cuda.empty_cache()

    ro = build(2, **kw)
    ro.reset()
    for _ in range(10):
        ro.step()
    ro.capture(10, per_group=True)
    ro.run(120)
    assert ro._graphs is not None and len(ro._graphs) == 2
    for a, b in zip(snapshot(ro), ref):
        assert_same(a, b)


def test_rollout_orders_after_caller_stream():
    """Replays (and eager steps) wait for work the caller enqueued on its own stream before run(): a
    NetMon state edit made on the current stream behind a busy kernel is seen by every group's next
    step (graph replay == eager with the same edit, and both differ from no edit)."""
    def go(graph, edit=True):
        ro = build(2)
        ro.reset()
        for _ in range(2):
            ro.step()
        if graph:
            ro.capture(2)
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)  # keep the caller's stream busy: an unordered step would race the edit
        if edit:
            for w in ro.wenvs:
                w.current_netmon_state.mul_(0.5)
        ro.run(2)
        return snapshot(ro)

    g = go(True)
    for a, b in zip(g, go(False)):
        assert_same(a, b)
    assert any(not np.array_equal(a["netmon"], b["netmon"]) for a, b in zip(g, go(False, edit=False)))


@pytest.mark.parametrize("graph", [False, True])
def test_lazy_obs_rows_match_written_rows(graph):
    """The rollout's envs write only the GEMM-ready obs copy (Routing.set_lazy_obs); reading .obs
    rebuilds the reference rows (gm_obs_from_gemm). They equal, bit for bit, the rows the env kernels
    write when asked to, at every step, across episode resets, eager and under graph replay; and the
    two modes give the same trajectories."""
    RO = importlib.import_module("graph-marl_amd.rollout")
    ros = []
    for lazy in (True, False):
        RO.LAZY_OBS = lazy
        try:
            ro = build(groups=2, n_env=64, episode_steps=10)
        finally:
            RO.LAZY_OBS = True
        assert all(e._lazy_obs == lazy for e in ro.envs)
        ro.reset()
        ro.run(2)
        if graph:
            ro.capture(2)
        ros.append(ro)
    for step in range(12):
        for ro in ros:
            ro.run(2)
        torch.cuda.synchronize()
        for el, ew in zip(ros[0].envs, ros[1].envs):
            assert el._obs_stale and not ew._obs_stale
            assert torch.equal(el.obs_gemm, ew.obs_gemm), step
            assert torch.equal(el.obs, ew.obs), step  # rebuilt vs written
            assert torch.equal(el.reward, ew.reward) and torch.equal(el.node_obs, ew.node_obs)
            assert not el._obs_stale
    # a masked reset on a lazy env, then the obs rows of every env (reset or not)
    el, ew = ros[0].envs[0], ros[1].envs[0]
    mask = (torch.arange(el.n_env, device="cuda") % 3 == 0).to(torch.uint8)
    el.reset_(mask)
    ew.reset_(mask)
    assert torch.equal(el.obs, ew.obs)


def test_graph_needs_fixed_epsilon():
    ro = build(1)
    ro.policies[0]._decay = 0.99
    ro.reset()
    ro.step()
    ro.step()
    with pytest.raises(ValueError):
        ro.capture(2)


def test_packed_caches_across_streams_and_deepcopy():
    """The packed-weight caches are shared by the stream groups (each later stream waits for the
    builder's event, L.Published) and a module copied after packing (the training's target
    network, copy.deepcopy) gets empty caches and computes the same Q as the original."""
    import copy

    ro = build(2)
    ro.reset()
    ro.run(3)
    pol = ro.policies[1]
    dqn = pol._model
    lin0 = dqn.encoder.linear_layers[0]
    assert lin0._packed_first.pub is not None and len(lin0._packed_first.pub.seen) >= 2  # both groups read it
    tar = copy.deepcopy(dqn)
    assert tar.encoder.linear_layers[0]._packed_first.key is None
    FU = importlib.import_module("graph-marl_amd.fused")
    env, wenv = ro.envs[0], ro.wenvs[0]
    with torch.no_grad():
        def q(m):
            bufs = {}
            return FU.dqn_q(m, env.obs_buf, env.obs_dim, wenv.current_netmon_state, wenv.h_prev, env.nbr,
                            env.agent_node, lambda i, mm, nn: bufs.setdefault(i, torch.empty(mm, nn, device="cuda")),
                            hidden=wenv.netmon.hidden_features, obs_gemm=env.obs_gemm).clone()
        np.testing.assert_array_equal(q(dqn).cpu().numpy(), q(tar).cpu().numpy())
