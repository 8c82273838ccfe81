"""Full-size, long-horizon parity of the benched rollout (bench.py's default workload) and of
config 4's other node counts.

StreamedRollout exactly as bench.py runs it: 4096 envs in 2 stream groups, N = 20 random
topologies (EVAL_SEEDS excluded), A = 20 packets, NetMon K = 1 (lstm, sum) + DQN 512,256,
ε = 0.5, 50-step episodes, 120 vector steps (two topology resets + NetMon start-ups inside).
Config 4 (random 10-50-node topologies) at N = 10, 30, 40, 50: 512 envs in 2 groups, 30-step
episodes, 70 steps (two resets) — this covers the N-dependent rows per block of the routing
encoder, DQN layer 1 on the folded GEMM-ready obs (K = 512 + 6N + 8, not a whole number of k
tiles off N = 20), the aggregate and the readout at those sizes. The LayerNorm-LSTM and GRU NetMon
cells (--netmon-rnn-type lnlstm / gru, src/layernormlstm.py, src/model.py:387-393): 1024 envs,
N = 20, the same 120 steps. Other --activation-function values (elu, tanh: the GEMM epilogues,
the routing encoder and the fused Q head): 512 envs, N = 20, 70 steps. The LN-LSTM bound is the fp32
envelope described at netmon_check (the 1e-5 contract is out of reach for any fp32 evaluation of that
cell over carried steps).
BASELINE config 3 (NetMon K = 1 on the fixed 20-node graph, seed 476) at its own 4096 envs, and
config 2 (no NetMon: the DQN reads the 130-wide env obs, K = 130, on the fixed graph) at its 1024
envs, both 120 steps (reference src/main.py:667-748, src/model.py:187-203).
Eight envs spread over both groups are shadowed every step by
  * the C oracle env (oracle/gm_oracle.c) fed the GPU's Q-values, which must take the same
    ε-greedy actions and give bit-identical rewards, done flags, agent and node observations
    and I+A adjacency (reference src/env/routing.py:160-539, src/policy.py:20-64);
  * the NumPy fp64 restatement of NetMon (oracle/netmon_ref.py, reference src/model.py:451-631)
    carried over the whole horizon from its own fp64 state (reset to the start-up step at each
    episode), against which the GPU NetMon state, the readout part of the joint observation and
    the Q-values must stay within 1e-5 (BASELINE.json north_star tolerance) at every step.
Run once per GEMM form: the split-f16 form the headline is measured with, and GM_GEMM=f32.
"""
import importlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

A, G, EPS = 20, 2, 0.5
TOL = 1e-5
# (N, envs, episode steps, vector steps, NetMon cell (None: no NetMon), --activation-function, random topology
#  [, --netmon-iterations K, default 1 [, --netmon-agg-type, default sum]])
CASES = [(20, 4096, 50, 120, "lstm", "leaky_relu", True), (10, 512, 30, 70, "lstm", "leaky_relu", True),
         (30, 512, 30, 70, "lstm", "leaky_relu", True), (40, 512, 30, 70, "lstm", "leaky_relu", True),
         (50, 512, 30, 70, "lstm", "leaky_relu", True), (20, 1024, 50, 120, "lnlstm", "leaky_relu", True),
         (20, 1024, 50, 120, "gru", "leaky_relu", True), (20, 512, 30, 70, "lstm", "elu", True),
         (20, 512, 30, 70, "lstm", "tanh", True),
         (20, 4096, 50, 120, "lstm", "leaky_relu", False),  # config 3: NetMon on the fixed graph
         (20, 1024, 50, 120, None, "leaky_relu", False),    # config 2: no NetMon, fixed graph
         (20, 1024, 50, 120, "lstm", "leaky_relu", True, 3),  # the CLI default --netmon-iterations 3
         (20, 512, 30, 70, "lstm", "leaky_relu", True, 2, "mean")]  # --netmon-agg-type mean
# LN-LSTM: the GPU must stay within ENVELOPE_X times the fp32 restatement's own drift from fp64 so far
# (floor ENVELOPE_FLOOR), never above ENVELOPE_CAP (measured 1.9e-3 state / 1.4e-3 readout for the fp32 restatement
# over 120 steps, GPU 1.6e-3 / 6.2e-4). Round 6: 2x and 3e-3 instead
# of 4x and 8e-3, which a 4x regression would have passed. 1.5x was tried: the GPU is a second fp32
# evaluation whose error vs fp64 reached 0.96x (split form) and 1.6x (f32 form, step 22: readout 3.1e-5
# against a restatement drift of 1.9e-5) of the restatement's own drift
ENVELOPE_X = 2.0
ENVELOPE_CAP = 3e-3
# floor of the envelope: in the first steps the fp32 restatement's own drift is ~1e-5 and the GPU's error is another
# draw of the same size (a first 1.5x run failed at step 7 with 1.76e-5 against 1.5 x 1.0e-5)
ENVELOPE_FLOOR = 2e-5


def case_id(c):
    return f"N{c[0]}-{c[4] or 'no_netmon'}-{c[5]}" + ("" if c[6] else "-fixed") + (f"-K{c[7]}" if len(c) > 7 else "") + (f"-{c[8]}" if len(c) > 8 else "")


def adjacency(topo, N):
    m = np.eye(N, dtype=np.int8)
    for i, row in enumerate(topo["nbr"]):
        for j in row:
            if j >= 0:
                m[i, j] = 1
    return m


@pytest.mark.parametrize("case", CASES, ids=[case_id(c) for c in CASES])
@pytest.mark.parametrize("form", ["x3", "f32"])
def test_benched_rollout_long_horizon(form, case, monkeypatch, oracle_mod):
    import netmon_ref

    N, B, EP, STEPS, RNN, ACT, RANDOM = case[:7]
    K = case[7] if len(case) > 7 else 1
    AGG = case[8] if len(case) > 8 else "sum"
    SAMPLE = sorted({0, 1, B // 5, B // 2 - 1, B // 2, B // 2 + 1, (4 * B) // 5, B - 1})

    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    RO = importlib.import_module("graph-marl_amd.rollout")
    monkeypatch.setattr(gm._lib, "GEMM_MODE", form)
    gm._lib.range_status(clear=True)
    net = gm.Network(N, random_topology=RANDOM, excluded_seeds=gm.EVAL_SEEDS, device=0)
    torch.manual_seed(0)
    netmon = M.NetMon(4 * N + 8, 128, [512, 256], K, rnn_type=RNN, activation=ACT, agg_type=AGG).cuda() if RNN else None
    dqn = M.DQN(6 * N + 10 + (netmon.get_out_features() if RNN else 0), [512, 256], 4, activation=ACT).cuda()
    ro = RO.StreamedRollout(net, A, B, netmon, dqn, groups=G, seed=0, epsilon=EPS, episode_steps=EP, device=0)
    per = B // G
    Wn = {k: v.detach().double().cpu().numpy() for k, v in netmon.state_dict().items()} if RNN else {}
    Wd = {k: v.detach().double().cpu().numpy() for k, v in dqn.state_dict().items()}
    od = 6 * N + 10

    qrec = {}
    for g, pol in enumerate(ro.policies):
        orig = pol.select

        def select(q, g=g, orig=orig):
            qrec[g] = q
            return orig(q)

        pol.select = select
        wenv = ro.wenvs[g]
        if not RNN:  # no NetMon: act() -> select(), then the env step
            continue
        orig_ps = wenv.policy_step_

        def policy_step_(q, eps, actions, detail=None, g=g, orig_ps=orig_ps):  # fused ε-greedy + env step
            qrec[g] = q.clone()
            return orig_ps(q, eps, actions, detail)

        wenv.policy_step_ = policy_step_

    cfg = oracle_mod.make_config(N, A, topo_mode=oracle_mod.TOPO_RANDOM if RANDOM else oracle_mod.TOPO_FIXED,
                                 excluded=gm.EVAL_SEEDS)
    orc = {e: oracle_mod.OracleEnv(cfg, e) for e in SAMPLE}
    loc = {e: (e // per, e % per) for e in SAMPLE}

    def gpu_view():
        torch.cuda.synchronize()
        out = {}
        for e, (g, i) in loc.items():
            env, wenv = ro.envs[g], ro.wenvs[g]
            out[e] = dict(obs=env.obs[i, :, :od].cpu().numpy(), node_obs=env.node_obs[i].cpu().numpy(),
                          state=wenv.current_netmon_state[i].cpu().numpy() if RNN else None,
                          readout=wenv.obs[i, :, od:].cpu().numpy() if RNN else None, reward=env.reward[i].cpu().numpy(),
                          done=env.done[i].cpu().numpy().astype(bool),
                          adj=env.get_nodes_adjacency()[i].cpu().numpy())
        return out

    state64, worst = {}, {"state": 0.0, "readout": 0.0, "q": 0.0}
    # LN-LSTM: the carried state is ill-conditioned (the cell LayerNorm divides by the spread of
    # c), so an fp32 evaluation of the reference's own formula drifts from fp64 far beyond 1e-5
    # (tests/test_long_horizon_gpu.py history: 7.5e-4 over 50 steps on the C-oracle env). The
    # same formulas in fp32 (netmon_ref, dtype float32, carried from their own fp32 state) run
    # beside the fp64 ones, and the GPU must stay within max(1e-5, 4 x the worst fp32 drift so far)
    fp32_envelope = RNN == "lnlstm"
    Wn32 = {k: v.astype(np.float32) for k, v in Wn.items()}
    state32, worst32 = {}, {"state": 0.0, "readout": 0.0}
    ratio = {"worst": 0.0}  # LN-LSTM: worst GPU error / envelope (printed: a creep shows between runs)

    def netmon_check(e, o, v, t):
        ob = o.observe()
        assert (v["obs"] == ob["obs"]).all(), f"step {t} env {e}: agent obs"
        assert (v["node_obs"] == ob["node_obs"]).all(), f"step {t} env {e}: node obs"
        adj = adjacency(o.topology(), N)
        assert (v["adj"] == adj).all(), f"step {t} env {e}: I+A adjacency"
        if not RNN:  # config 2: the DQN reads the env obs alone
            return ob["obs"].astype(np.float64)
        out, st = netmon_ref.netmon_forward(Wn, ob["node_obs"][None], adj[None], state64.get(e), RNN, AGG, K, act=ACT)
        state64[e] = st
        ro_ = netmon_ref.to_network_obs(out, ob["node_agent"][None])[0]
        tol_s = tol_r = TOL
        if fp32_envelope:
            out32, st32 = netmon_ref.netmon_forward(Wn32, ob["node_obs"][None].astype(np.float32),
                                                    adj[None].astype(np.float32), state32.get(e), RNN, AGG, K,
                                                    act=ACT, dtype=np.float32)
            state32[e] = st32
            ro32 = netmon_ref.to_network_obs(out32, ob["node_agent"][None])[0]
            worst32["state"] = max(worst32["state"], np.abs(st32 - st).max())
            worst32["readout"] = max(worst32["readout"], np.abs(ro32 - ro_).max())
            tol_s = min(ENVELOPE_CAP, max(ENVELOPE_FLOOR, ENVELOPE_X * worst32["state"]))
            tol_r = min(ENVELOPE_CAP, max(ENVELOPE_FLOOR, ENVELOPE_X * worst32["readout"]))
        es = np.abs(v["state"] - st[0]).max()
        er = np.abs(v["readout"] - ro_).max()
        ratio["worst"] = max(ratio["worst"], es / tol_s, er / tol_r)
        worst["state"], worst["readout"] = max(worst["state"], es), max(worst["readout"], er)
        assert es < tol_s and er < tol_r, f"step {t} env {e}: NetMon state err {es}, readout err {er} (tol {tol_s}, {tol_r})"
        return np.concatenate([ob["obs"].astype(np.float64), ro_], -1)

    ro.reset()
    for o in orc.values():
        o.reset()
    joint = {e: netmon_check(e, orc[e], v, 0) for e, v in gpu_view().items()}
    resets = 0
    for t in range(1, STEPS + 1):
        ro.step()
        v = gpu_view()
        acts = {g: ro.policies[g].actions.cpu().numpy() for g in range(G)}
        for e, o in orc.items():
            g, i = loc[e]
            q = qrec[g][i].cpu().numpy()
            q64 = netmon_ref.dqn_forward(Wd, joint[e], act=ACT)
            eq = np.abs(q - q64).max()
            worst["q"] = max(worst["q"], eq)
            tol_q = min(ENVELOPE_CAP, max(ENVELOPE_FLOOR, ENVELOPE_X * worst32["readout"])) if fp32_envelope else TOL
            ratio["worst"] = max(ratio["worst"], eq / tol_q)
            assert eq < tol_q, f"step {t} env {e}: Q err {eq}"
            exp = o.draw_egreedy(q, EPS)
            assert (exp == acts[g][i]).all(), f"step {t} env {e}: ε-greedy actions"
            rew, done, _ = o.step(acts[g][i])
            assert (rew == v[e]["reward"]).all() and (done == v[e]["done"]).all(), f"step {t} env {e}: reward/done"
            if t % EP == 0:  # the rollout reset the episode after this step: new topology, NetMon start-up
                o.reset()
                state64.pop(e, None)
                state32.pop(e, None)
            joint[e] = netmon_check(e, o, v[e], t)
        resets += t % EP == 0
    assert resets == STEPS // EP >= 2
    gm._lib.check_range()
    print(f"N={N} K={K} {AGG} {RNN} {ACT} {'random' if RANDOM else 'fixed'} form {form}: worst |err| over {STEPS} steps x "
          f"{len(SAMPLE)} envs: {worst}; worst err / tolerance {ratio['worst']:.3g}"
          + (f"; fp32 restatement of the reference formula vs fp64: {worst32}" if fp32_envelope else ""))
