"""GPU parity of the fused GEMM path (gm_gemm_f32): dense/ragged GEMMs and the LSTM
epilogue vs torch fp32, the fused NetMon step and DQN readout-gather vs the unfused
(golden-validated) path, and the reference goldens through the fused path."""
import ctypes as C
import importlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_replay as R

pytestmark = pytest.mark.gpu


def mods():
    return (importlib.import_module("graph-marl_amd"), importlib.import_module("graph-marl_amd.model"),
            importlib.import_module("graph-marl_amd.fused"), importlib.import_module("graph-marl_amd.wrapper"))


@pytest.mark.parametrize("m,n,k,ldx", [(81920, 512, 642, 644), (1000, 256, 512, 512), (777, 130, 90, 92),
                                       (5, 3, 7, 8), (4097, 33, 129, 132), (64, 4, 256, 256), (300, 64, 16, 16)])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("form", ["f32", "x3"])
def test_gemm_dense_vs_torch(m, n, k, ldx, epi, form):
    """Both arithmetic forms within the rollout tolerance (1e-5, scaled for K > 64) of fp64."""
    gm, M, FU, W = mods()
    torch.manual_seed(m + n + k)
    buf = torch.randn(m, ldx, device="cuda")
    x = buf[:, :k]
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda")
    wp, ldw = FU._pad_cols(w)
    x3 = FU.X3(wp, ldw, n, k) if form == "x3" else None
    y = torch.empty(m, n, device="cuda")
    FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, epi, y.data_ptr(), n,
            x3=x3)
    ref = F.linear(x.double(), w.double(), b.double())
    if epi == 1:
        ref = F.leaky_relu(ref)
    assert (y.double() - ref).abs().max().item() < 1e-5 * max(1.0, k ** 0.5 / 8)


def test_gemm_x3_error_is_fp32_order():
    """Split-f16 error vs fp64 stays within a small factor of the exact-fp32 GEMM's own
    error, on activations spanning 2^-9..2^3 (rows of very different scale) and weights
    spanning 2^-12..2^0 — i.e. x3 is an fp32-accuracy GEMM, not a reduced-precision one."""
    gm, M, FU, W = mods()
    torch.manual_seed(7)
    m, n, k = 8192, 256, 512
    x = torch.randn(m, k, device="cuda") * torch.exp2(torch.randint(-9, 4, (m, 1), device="cuda").float())
    w = torch.randn(n, k, device="cuda") * torch.exp2(torch.randint(-12, 1, (n, 1), device="cuda").float())
    b = torch.zeros(n, device="cuda")
    wp, ldw = FU._pad_cols(w)
    ref = F.linear(x.double(), w.double())
    mag = F.linear(x.abs().double(), w.abs().double())  # sum |a*w| per output
    errs = {}
    for form in ("f32", "x3"):
        y = torch.empty(m, n, device="cuda")
        FU.gemm(FU.dense(x.data_ptr(), k, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 0, y.data_ptr(), n,
                x3=FU.X3(wp, ldw, n, k) if form == "x3" else None)
        errs[form] = ((y.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    assert errs["f32"] < 1e-6
    assert errs["x3"] < 4e-6, errs


@pytest.mark.parametrize("form", ["f32", "x3"])
def test_gemm_two_sources_and_lstm_epilogue(form, monkeypatch):
    gm, M, FU, W = mods()
    monkeypatch.setattr(FU.L, "GEMM_MODE", form)
    torch.manual_seed(0)
    Mr, H = 5000, 128
    cell = M.LSTMCell(H, H).cuda()
    x = torch.randn(Mr, H, device="cuda")
    st = torch.randn(Mr, 2 * H, device="cuda")
    h, c = st[:, :H], st[:, H:]
    wp, ldw, bp, x3 = FU.pack_lstm(cell)
    assert (x3 is not None) == (form == "x3")
    S = torch.empty(Mr, 2 * H, device="cuda")
    FU.gemm(FU.dense(x.data_ptr(), H, H), FU.dense(st.data_ptr(), 2 * H, H), wp.data_ptr(), ldw, bp.data_ptr(), Mr,
            4 * H, FU.GM_EPI_LSTM, S.data_ptr(), 2 * H, S[:, H:].data_ptr(), 2 * H, c.data_ptr(), 2 * H, x3=x3)
    ref = torch.nn.LSTMCell(H, H).cuda()
    ref.load_state_dict(cell.state_dict())
    rh, rc = ref(x, (h.contiguous(), c.contiguous()))
    torch.testing.assert_close(S[:, :H], rh, atol=1e-5, rtol=0)
    torch.testing.assert_close(S[:, H:], rc, atol=1e-5, rtol=0)


def _setup_env(gm, W, M, B=64, seed=5, fused=True, rnn="lstm", K=1):
    N, A = 20, 20
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), A, n_env=B, seed=seed,
                     obs_extra=512, agent_adjacency=False)
    torch.manual_seed(1)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], K, rnn_type=rnn).cuda()
    return env, nm, W.NetMonWrapper(env, nm, 1, fused=fused)


@pytest.mark.parametrize("rnn,K", [("lstm", 1), ("lnlstm", 1), ("gru", 2)])
def test_fused_rollout_matches_unfused_path(rnn, K):
    """Fused rollout (readout gathered in the DQN GEMM; lstm / gru gate math in the GEMM epilogue;
    lnlstm GEMMs + the LayerNorm-LSTM pointwise kernel) == NetMon.forward_graph + joint obs."""
    gm, M, FU, W = mods()
    P = importlib.import_module("graph-marl_amd.policy")
    e1, nm1, w1 = _setup_env(gm, W, M, fused=True, rnn=rnn, K=K)
    e2, nm2, w2 = _setup_env(gm, W, M, fused=False, rnn=rnn, K=K)
    assert w1.fused
    # lnlstm: the cell LayerNorm divides by the spread of c, so both fp32 paths sit ~4e-6 from an
    # fp64 evaluation per step already with exact f32 GEMMs (tools/diag_lnlstm.py); after 6
    # carried steps they differ by up to ~1.2e-5 from each other. The 1e-5 contract against the
    # reference holds per step (test_fused_netmon_vs_reference_golden, lnlstm variants).
    tol = 3e-5 if rnn == "lnlstm" else 1e-5
    torch.manual_seed(2)
    dqn = M.DQN(e1.obs_dim + 512, [512, 256], 4).cuda()
    p1 = P.EpsilonGreedy(w1, dqn, epsilon=0.5, epsilon_decay=1.0, step_before_train=0)
    p2 = P.EpsilonGreedy(w2, dqn, epsilon=0.5, epsilon_decay=1.0, step_before_train=0)
    w1.reset()
    w2.reset()
    for t in range(6):
        q1 = FU.dqn_q(dqn, e1.obs_buf, e1.obs_dim, w1.current_netmon_state, w1.h_prev, e1.nbr, e1.agent_node,
                      p1._buf, hidden=128).view(e1.n_env, e1.n_data, -1).clone()
        q2 = p2.q_values(w2.obs)
        torch.testing.assert_close(q1, q2, atol=tol, rtol=0)
        a1 = p1.select(q1).clone()
        a2 = p2.select(q2).clone()
        # identical draws; argmax may only differ on exact near-ties
        assert (a1 != a2).float().mean().item() < 1e-3
        w1.step_(a2)
        w2.step_(a2)
        torch.testing.assert_close(w1.current_netmon_state, w2.current_netmon_state, atol=tol, rtol=0)
        torch.testing.assert_close(w1.obs, w2.obs, atol=tol, rtol=0)


@pytest.mark.parametrize("vi", [0, 1, 2, 3, 4, 5])
def test_fused_netmon_vs_reference_golden(vi):
    """Every carry-over variant of tests/golden/netmon.npz (lstm sum/mean K=1..3, lnlstm sum/mean,
    gru) through the fused step vs the reference's states and readouts over 3 carried steps."""
    gm, M, FU, W = mods()
    g = np.load(f"{R.GOLDEN}/netmon.npz")
    rnn, agg, K, H, enc = g["variants"][vi].split("|")
    nm = M.NetMon(g["node_obs"].shape[-1], int(H), [int(e) for e in enc.split(",")], int(K), rnn_type=rnn,
                  agg_type=agg).cuda()
    nm.load_state_dict({k[len(f"v{vi}_w_"):]: torch.as_tensor(g[k]) for k in g.files if k.startswith(f"v{vi}_w_")})
    state = None
    for t in range(3):
        x = torch.as_tensor(g["node_obs"][t], device="cuda")
        nbr = M.dense_to_nbr(torch.as_tensor(g["node_adj"][t], device="cuda"))
        na = torch.as_tensor(g["node_agent"][t], device="cuda")
        an = M.node_agent_to_index(na)
        state, hprev = FU.netmon_step(nm, x, nbr, state)
        np.testing.assert_allclose(state.cpu().numpy(), g[f"v{vi}_state_{t}"], atol=1e-5, rtol=0)
        B, N = x.shape[:2]
        Hh = int(H)
        hprev = hprev.reshape(B * N, -1)
        out = M.netmon_readout(state.reshape(B * N, -1)[:, :Hh].contiguous(), hprev[:, :Hh].contiguous(), nbr, an)
        np.testing.assert_allclose(out.view(B, -1, 4 * Hh).cpu().numpy(), g[f"v{vi}_mapped_{t}"], atol=1e-5, rtol=0)


@pytest.mark.parametrize("n,out", [(20, 512), (50, 512), (10, 64), (20, 192), (30, 512), (40, 256)])
def test_routing_node_encoder_vs_torch(n, out):
    """Sparse first encoder layer on real routing node observations vs the dense fp32 product."""
    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    FU = importlib.import_module("graph-marl_amd.fused")
    B, A = 64, 20
    env = gm.Routing(gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), A, n_env=B, seed=5)
    env.reset()
    rng = np.random.RandomState(0)
    for _ in range(5):
        env.step_(torch.as_tensor(rng.randint(0, 4, (B, A)), dtype=torch.int32, device="cuda"))
    x = env.node_obs.reshape(-1, 4 * n + 8)
    torch.manual_seed(1)
    lin = M.Linear(4 * n + 8, out, act=1).cuda()
    assert FU.routing_encoder_ok(lin, n, 4 * n + 8, env.nbr)
    y = FU.routing_encoder(lin, x, env.nbr, B, n, torch.empty(B * n, out, device="cuda"))
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.linear(x.double(), lin.weight.double(),
                                                                    lin.bias.double()), 0.01)
    err = (y.double() - ref).abs().max().item()
    assert err < 1e-5, err


@pytest.mark.parametrize("mfma", [1, 0])
@pytest.mark.parametrize("tile", [8, 9, 10, 11, 12, 13, 14])
def test_gemm_lds_dma_tiles(tile, mfma):
    """The LDS-DMA x3 kernel (tiles 8..14, 16x16x32 and 32x32x16 MFMA forms): dense (ragged M/N/K,
    padded rows), two sources with the LSTM epilogue, and the DQN readout gather of the fused
    rollout, vs fp64 / torch."""
    gm, M, FU, W = mods()
    lib = FU._setup()
    lib.gm_gemm_set_tile(tile)
    FU.L.check(lib.gm_gemm_set_mfma(mfma))
    try:
        for (m, n, k, ldx) in [(81920, 512, 642, 644), (1000, 256, 512, 512), (777, 130, 90, 92),
                               (4097, 33, 129, 132), (300, 64, 16, 16)]:
            for epi in (0, 1):
                test_gemm_dense_vs_torch(m, n, k, ldx, epi, "x3")
        test_gemm_x3_error_is_fp32_order()

        class MP:
            def setattr(self, obj, name, val):
                setattr(obj, name, val)
        old = FU.L.GEMM_MODE
        try:
            test_gemm_two_sources_and_lstm_epilogue("x3", MP())
            FU.L.GEMM_MODE = "x3"
            test_fused_rollout_matches_unfused_path("lstm", 1)
            test_fused_rollout_matches_unfused_path("gru", 2)
        finally:
            FU.L.GEMM_MODE = old
    finally:
        lib.gm_gemm_set_tile(-1)
        lib.gm_gemm_set_mfma(2)


@pytest.mark.parametrize("m,n,k,ldx,nq", [(81920, 256, 512, 512, 4), (1000, 256, 512, 516, 4), (777, 100, 90, 92, 2),
                                          (33, 256, 256, 256, 3), (5, 64, 16, 16, 1)])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("mfma", [1, 2])
def test_gemm_x3_head_vs_torch(m, n, k, ldx, nq, act, mfma):
    """gm_gemm_x3_head (last DQN layer + Q head in one kernel; 32x32x16 and 16x16x32 MFMA forms)
    vs fp64: q within the rollout tolerance, and the optional hidden output equal to the plain
    split-f16 GEMM's."""
    gm, M, FU, W = mods()
    FU.L.check(FU._setup().gm_gemm_set_mfma(mfma))
    try:
        _head_case(M, FU, m, n, k, ldx, nq, act)
    finally:
        FU._setup().gm_gemm_set_mfma(2)


def _head_case(M, FU, m, n, k, ldx, nq, act):
    torch.manual_seed(m + n + k + nq)
    buf = torch.randn(m, ldx, device="cuda")
    x = buf[:, :k]
    lin = M.Linear(k, n, act=act).cuda()
    fc = M.Linear(n, nq, act=0).cuda()
    assert FU.head_ok(lin, fc) == (FU.L.GEMM_MODE == "x3")
    if FU.L.GEMM_MODE != "x3":
        pytest.skip("split-f16 form disabled (GM_GEMM=f32)")
    q = torch.full((m, nq), float("nan"), device="cuda")
    y = torch.empty(m, n, device="cuda")
    FU.linear_head(lin, fc, buf, ldx, k, q, y=y)
    hid = F.linear(x.double(), lin.weight.double(), lin.bias.double())
    if act == 1:
        hid = F.leaky_relu(hid)
    ref = F.linear(hid, fc.weight.double(), fc.bias.double())
    tol = 1e-5 * max(1.0, k ** 0.5 / 8)
    assert (y.double() - hid).abs().max().item() < tol
    assert (q.double() - ref).abs().max().item() < tol * max(1.0, n ** 0.5 / 8)
    q2 = torch.full((m, nq), float("nan"), device="cuda")
    FU.linear_head(lin, fc, buf, ldx, k, q2)  # without the hidden output: same q
    assert torch.equal(q, q2)


@pytest.mark.parametrize("mag", [1e-9, 1e-6, 1.0, 3e3])
def test_input_gradient_x3_scaled(mag):
    """gx = gy @ w in the split-f16 form with the device power-of-two A scale
    (gm_absmax_scale): fp32-order error relative to sum |gy*w| at any gradient magnitude,
    including far below the f16 normal range, where the unscaled split would lose precision."""
    gm, M, FU, W = mods()
    if FU.L.GEMM_MODE != "x3":
        pytest.skip("split-f16 form disabled (GM_GEMM=f32)")
    torch.manual_seed(11)
    m, n, k = 4096, 512, 642
    gy = torch.randn(m, n, device="cuda") * mag * torch.exp2(torch.randint(-6, 1, (m, 1), device="cuda").float())
    w = torch.randn(n, k, device="cuda") / n ** 0.5
    gx = M._dgrad(gy, w)
    ref = gy.double() @ w.double()
    mag_ref = gy.abs().double() @ w.abs().double()
    rel = ((gx.double() - ref).abs() / mag_ref.clamp_min(1e-300)).max().item()
    assert rel < 4e-6, rel
    f32 = gy @ w
    rel32 = ((f32.double() - ref).abs() / mag_ref.clamp_min(1e-300)).max().item()
    assert rel < 8 * max(rel32, 5e-7), (rel, rel32)


@pytest.mark.parametrize("Mb,o,k,ldx,mag", [(20001, 512, 642, 644, 1e-7), (65536, 256, 512, 512, 1.0),
                                            (9000, 4, 256, 256, 1e-4), (131072, 512, 130, 132, 1e-6)])
def test_weight_gradient_kmajor(Mb, o, k, ldx, mag):
    """gW = gy^T x by the split-K split-f16 GEMM on K-major operands (gm_gemm_x3_wgrad; ragged
    batch, ragged k with padded rows, 4-wide heads, tiny gradients): fp32-order error relative
    to sum |gy*x|."""
    gm, M_, FU, W = mods()
    if FU.L.GEMM_MODE != "x3":
        pytest.skip("split-f16 form disabled (GM_GEMM=f32)")
    torch.manual_seed(Mb + o)
    gy = torch.randn(Mb, o, device="cuda") * mag
    xb = torch.randn(Mb, ldx, device="cuda")
    x = xb[:, :k]
    ref = gy.double().t() @ x.double()
    mag_ref = gy.abs().double().t() @ x.abs().double()
    lib = FU._setup()
    try:
        for form in (-1, 3, 2, 0):  # transposed reads 128x128 (default), 16x16x32 MFMA, 128x256, dword form
            lib.gm_gemm_set_wgrad(form)
            gw = M_._wgrad(gy, x, k)
            assert gw.shape == (o, k)
            rel = ((gw.double() - ref).abs() / mag_ref.clamp_min(1e-300)).max().item()
            assert rel < 4e-6, (form, rel)
    finally:
        lib.gm_gemm_set_wgrad(-1)


@pytest.mark.parametrize("Mb,o,k1,ld1,k2,ld2", [(131072, 512, 128, 128, 128, 256), (65536, 512, 512, 512, 130, 132),
                                               (20001, 256, 128, 256, 256, 256)])
def test_weight_gradient_two_sources(Mb, o, k1, ld1, k2, ld2):
    """gm_gemm_x3_wgrad2 (round 6): the two weight gradients that share a gradient operand (LSTM W_ih / W_hh on
    [x] and the h half of the [h | c] state rows, DQN layer 1 on [readout | env obs]) from ONE launch, each with
    its own operand scale: fp32-order error vs fp64 like gm_gemm_x3_wgrad, on both 128-column forms."""
    gm, M_, FU, W = mods()
    torch.manual_seed(Mb + k2)
    gy = torch.randn(Mb, o, device="cuda") * 1e-5
    x1 = torch.randn(Mb, ld1, device="cuda")
    x2 = torch.randn(Mb, ld2, device="cuda") * 3e-3
    s = [torch.empty(1, device="cuda") for _ in range(3)]
    lib = FU._setup()
    L = FU.L
    L.check(lib.gm_absmax_scale(gy.data_ptr(), gy.numel(), s[0].data_ptr(), L.stream_ptr()))
    L.check(lib.gm_absmax_scale_rows(x1.data_ptr(), Mb, k1, ld1, s[1].data_ptr(), L.stream_ptr()))
    L.check(lib.gm_absmax_scale_rows(x2.data_ptr(), Mb, k2, ld2, s[2].data_ptr(), L.stream_ptr()))
    try:
        for form in (-1, 3):
            lib.gm_gemm_set_wgrad(form)
            r = M_._wgrad2(gy, [(x1, k1, s[1], 0, 0), (x2, k2, s[2], 0, 0)], s[0])
            assert r is not None
            for got, x, k in zip(r, (x1, x2), (k1, k2)):
                assert got.shape == (o, k)
                ref = gy.double().t() @ x[:, :k].double()
                mag = gy.abs().double().t() @ x[:, :k].abs().double()
                rel = ((got.double() - ref).abs() / mag.clamp_min(1e-300)).max().item()
                assert rel < 4e-6, (form, k, rel)
    finally:
        lib.gm_gemm_set_wgrad(-1)
    bad = L.WgradSrc(x1.data_ptr(), ld1, s[1].data_ptr(), 0, 0, Mb)  # n1 = 100: a column tile would straddle
    assert lib.gm_gemm_x3_wgrad2(gy.data_ptr(), o, C.byref(bad), 100, C.byref(bad), 4, o, Mb, 4096, s[0].data_ptr(),
                                 gy.data_ptr(), 104, None) != 0


def test_weight_gradient_row_maps():
    """gm_wgrad_src row maps (round 6, config 5): the obs cell's x is the same encoder output E [M][H] at every one
    of L steps, so W_ih's gradient over all L steps' gate gradients reads E with period M in ONE launch; W_hh's
    reads step t-1's state (shift -M, zero at t = 0). Both against fp64 sums over the steps."""
    gm, M_, FU, W = mods()
    Ls, M, H, o = 4, 20480, 128, 512
    torch.manual_seed(3)
    dG = torch.randn(Ls * M, o, device="cuda") * 1e-4
    E = torch.randn(M, H, device="cuda")
    Sprev = torch.randn((Ls - 1) * M, 2 * H, device="cuda")  # states of steps 0..L-2, [h | c] rows
    s = [torch.empty(1, device="cuda") for _ in range(3)]
    lib = FU._setup()
    L = FU.L
    L.check(lib.gm_absmax_scale(dG.data_ptr(), dG.numel(), s[0].data_ptr(), L.stream_ptr()))
    L.check(lib.gm_absmax_scale_rows(E.data_ptr(), M, H, H, s[1].data_ptr(), L.stream_ptr()))
    L.check(lib.gm_absmax_scale_rows(Sprev.data_ptr(), (Ls - 1) * M, H, 2 * H, s[2].data_ptr(), L.stream_ptr()))
    r = M_._wgrad2(dG, [(E, H, s[1], M, 0), (Sprev, H, s[2], 0, -M)], s[0])
    assert r is not None
    d64 = dG.double().view(Ls, M, o)
    ref_ih = sum(d64[t].t() @ E.double() for t in range(Ls))
    mag_ih = sum(d64[t].abs().t() @ E.abs().double() for t in range(Ls))
    hp = Sprev[:, :H].double().view(Ls - 1, M, H)
    ref_hh = sum(d64[t].t() @ hp[t - 1] for t in range(1, Ls))
    mag_hh = sum(d64[t].abs().t() @ hp[t - 1].abs() for t in range(1, Ls))
    for got, ref, mag in ((r[0], ref_ih, mag_ih), (r[1], ref_hh, mag_hh)):
        rel = ((got.double() - ref).abs() / mag.clamp_min(1e-300)).max().item()
        assert rel < 4e-6, rel


@pytest.mark.parametrize("rows,k,n,act", [(8192, 642, 512, 1), (5000, 256, 128, 1), (4096, 512, 4, 0),
                                          (100000, 512, 640, 1), (131072, 256, 512, 0)])
def test_linear_backward_large_batch(rows, k, n, act):
    """LinearFn backward at training batch sizes — fused leaky-ReLU backward + bias partials
    (gm_leaky_bwd), scaled split-f16 input and weight gradients — vs fp64, relative to the
    magnitude of each gradient's terms. The reference takes the leaky-ReLU mask from the
    kernel's own forward output: at 1e5 rows a few pre-activations within the forward's 5e-6
    error of zero flip sign, which is a forward property, not a backward one."""
    gm, M, FU, W = mods()
    torch.manual_seed(rows + n)
    lin = M.Linear(k, n, act=act).cuda()
    x = torch.randn(rows, k, device="cuda", requires_grad=True)
    y = lin(x)
    g = torch.randn_like(y) * 1e-5
    y.backward(g)
    xd, wd = x.detach().double(), lin.weight.detach().double()
    gyd = g.double() * torch.where(y.detach() >= 0, 1.0, 0.01 if act == 1 else 1.0)
    refs = ((x.grad, gyd @ wd, gyd.abs() @ wd.abs()), (lin.weight.grad, gyd.t() @ xd, gyd.abs().t() @ xd.abs()),
            (lin.bias.grad, gyd.sum(0), gyd.abs().sum(0)))
    for got, ref, mag in refs:
        rel = ((got.double() - ref).abs() / mag.clamp_min(1e-300)).max().item()
        assert rel < 1e-5, rel


@pytest.mark.parametrize("rows,k,n", [(8192, 642, 512), (4096, 256, 512), (100000, 642, 512), (131072, 256, 512)])
def test_forward_amax_publishes_max(rows, k, n):
    """gm_gemm_x3's src0 amax: the forward GEMM publishes max|x| (exact float bits) and
    gm_absmax_finish turns it into the same scale gm_absmax_scale_rows computes."""
    gm, M, FU, W = mods()
    if FU.L.GEMM_MODE != "x3":
        pytest.skip("split-f16 form disabled (GM_GEMM=f32)")
    torch.manual_seed(rows + k)
    ld = (k + 3) // 4 * 4 + 4
    xb = torch.randn(rows, ld, device="cuda") * 3.0
    xb[:, k:] = 1e6  # padding columns past k must not count
    x = xb[:, :k]
    w = torch.randn(n, k, device="cuda") * 0.05
    slot = M._amax_slot(xb, ld, n, True)
    assert slot is not None
    y = M.linear_raw(xb, ld, k, w, None, 0, amax=slot)
    torch.cuda.synchronize()
    assert slot.view(torch.int32).item() == x.abs().max().view(torch.int32).item()
    M._finish_scale(slot)
    ref = torch.empty(1, device="cuda")
    FU.L.check(FU._setup().gm_absmax_scale_rows(xb.data_ptr(), rows, k, ld, ref.data_ptr(), FU.L.stream_ptr()))
    assert slot.item() == ref.item()
    torch.testing.assert_close(y, x @ w.t(), rtol=1e-5, atol=1e-4)


def test_backward_kernels_publish_scale():
    """gm_leaky_bwd / gm_lstm_pointwise_bwd g_scale == gm_absmax_scale of their output."""
    gm, M, FU, W = mods()
    lib = FU._setup()
    torch.manual_seed(11)
    rows, cols = 5000, 256
    gy = torch.randn(rows, cols, device="cuda") * 1e-4
    y = torch.randn(rows, cols, device="cuda")
    g = torch.empty_like(gy)
    part = torch.empty((rows + 63) // 64, cols, device="cuda")
    sc = torch.empty(1, device="cuda")
    FU.L.check(lib.gm_leaky_bwd(gy.data_ptr(), y.data_ptr(), rows, cols, 0.01, g.data_ptr(), part.data_ptr(), 64,
                                sc.data_ptr(), FU.L.stream_ptr()))
    ref = M._gy_scale(g)
    assert sc.item() == ref.item()
    torch.testing.assert_close(g, torch.where(y >= 0, gy, 0.01 * gy), rtol=0, atol=0)
    Mr, H = 9000, 128
    act = torch.rand(Mr, 4 * H, device="cuda")
    c = torch.randn(Mr, H, device="cuda")
    c1 = torch.randn(Mr, H, device="cuda")
    dh = torch.randn(Mr, H, device="cuda") * 1e-3
    dg = torch.empty(Mr, 4 * H, device="cuda")
    dc = torch.empty(Mr, H, device="cuda")
    sc2 = torch.empty(1, device="cuda")
    FU.L.check(lib.gm_lstm_pointwise_bwd(dh.data_ptr(), None, act.data_ptr(), c.data_ptr(), c1.data_ptr(), Mr, H,
                                         dg.data_ptr(), dc.data_ptr(), sc2.data_ptr(), FU.L.stream_ptr()))
    dg0 = torch.empty_like(dg)
    dc0 = torch.empty_like(dc)
    FU.L.check(lib.gm_lstm_pointwise_bwd(dh.data_ptr(), None, act.data_ptr(), c.data_ptr(), c1.data_ptr(), Mr, H,
                                         dg0.data_ptr(), dc0.data_ptr(), None, FU.L.stream_ptr()))
    assert torch.equal(dg, dg0) and torch.equal(dc, dc0)
    assert sc2.item() == M._gy_scale(dg).item()


@pytest.mark.parametrize("rows", [8192, 1000])
def test_lstm_cell_backward_large_batch(rows):
    """LSTMCell step at training batch sizes (one autograd node: gates GEMM + gate math, scales
    published by the producers) vs fp64 autograd of nn.LSTMCell semantics."""
    gm, M, FU, W = mods()
    torch.manual_seed(rows)
    H = 128
    cell = M.LSTMCell(H, H).cuda()
    x = torch.randn(rows, H, device="cuda", requires_grad=True)
    h = torch.randn(rows, H, device="cuda", requires_grad=True)
    c = torch.randn(rows, H, device="cuda", requires_grad=True)
    h1, c1 = cell(x, (h, c))
    gh = torch.randn_like(h1) * 1e-4
    gc = torch.randn_like(c1) * 1e-4
    torch.autograd.backward((h1, c1), (gh, gc))
    ref = torch.nn.LSTMCell(H, H).double().cuda()
    with torch.no_grad():
        for name in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
            getattr(ref, name).copy_(getattr(cell, name).double())
    xd, hd, cd = (t.detach().double().requires_grad_(True) for t in (x, h, c))
    h1d, c1d = ref(xd, (hd, cd))
    torch.testing.assert_close(h1.double(), h1d, rtol=0, atol=2e-5)
    torch.testing.assert_close(c1.double(), c1d, rtol=0, atol=2e-5)
    torch.autograd.backward((h1d, c1d), (gh.double(), gc.double()))
    for got, want in ((x.grad, xd.grad), (h.grad, hd.grad), (c.grad, cd.grad), (cell.weight_ih.grad, ref.weight_ih.grad),
                      (cell.weight_hh.grad, ref.weight_hh.grad), (cell.bias_ih.grad, ref.bias_ih.grad)):
        scale = want.abs().max().item()
        err = (got.double() - want).abs().max().item()
        assert err <= 1e-5 * scale + 1e-12, (err, scale)


@pytest.mark.parametrize("m,n,k,epi", [(4096, 128, 128, 0), (32768, 256, 256, 1), (4096, 512, 256, 2)])
def test_gemm_x3_range_guard(m, n, k, epi):
    """Split-f16 operands in [2^15, 65504): values whose low piece stays in the f16 range give
    fp32-order results and leave the guard clear; one value whose low piece overflows
    (32784 = f16 32768 + 16: 16 * 2^12 = 65536 -> inf) sets the host-mapped status word, the
    next x3 call raises GMError, and clearing the word re-enables the form. Covers the
    register-staged kernel (n = 128), the LDS-DMA kernel (n >= 256, K >= 256, m >= 32768) and
    the LSTM epilogue (which would squash the inf to a finite h)."""
    gm, M, FU, W = mods()
    L = gm._lib
    L.range_status(clear=True)
    torch.manual_seed(11)
    x = torch.empty(m, k, device="cuda").uniform_(32768.0, 60000.0) * torch.where(
        torch.rand(m, k, device="cuda") < 0.5, -1.0, 1.0)
    r = (x - x.half().float()).abs()
    x = torch.where(r < 15.9, x, x.half().float())  # keep every low piece inside the f16 range
    w = torch.randn(n, k, device="cuda") * 0.05
    b = torch.zeros(n, device="cuda")
    wp, ldw = FU._pad_cols(w)
    xp = FU.X3(wp, ldw, n, k)
    y = torch.empty(m, n if epi != 2 else n // 4, device="cuda")

    def run(xx):
        if epi == 2:  # LSTM epilogue on [x | h] halves of K
            c_in = torch.zeros(m, n // 4, device="cuda")
            y2 = torch.empty(m, n // 4, device="cuda")
            FU.gemm(FU.dense(xx.data_ptr(), k, k // 2), FU.dense(xx[:, k // 2:].data_ptr(), k, k // 2), wp.data_ptr(),
                    ldw, b.data_ptr(), m, n, FU.GM_EPI_LSTM, y.data_ptr(), n // 4, y2.data_ptr(), n // 4,
                    c_in.data_ptr(), n // 4, x3=xp)
        else:
            FU.gemm(FU.dense(xx.data_ptr(), k, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, epi, y.data_ptr(), n,
                    x3=xp)
        torch.cuda.synchronize()

    run(x)
    assert L.range_status() == 0
    if epi == 0:
        ref = F.linear(x.double(), w.double())
        mag = F.linear(x.abs().double(), w.abs().double())
        assert ((y.double() - ref).abs() / mag).max().item() < 4e-6
    bad = x.clone()
    # the register-staged forms (n = 128; the LSTM case at m = 4096) scale the low piece by 2^12, so 32784 is
    # the first value that overflows it; the LDS-DMA form on rollout operands (the epi 1 case) keeps the low
    # piece unscaled (no overflow below the f16 range), so there the guard trips at 65520 (f16(65520) = inf)
    bad[m // 3, 5] = 65520.0 if epi == 1 else 32784.0
    run(bad)
    assert L.range_status() == 1
    with pytest.raises(gm._lib.GMError):
        L.check_range()
    with pytest.raises(gm._lib.GMError):
        run(x)  # every later x3 call fails until the word is cleared
    assert L.range_status(clear=True) == 1
    run(x)
    assert L.range_status() == 0


@pytest.mark.parametrize("rows,H", [(4096, 128), (1000, 32), (333, 96), (2048, 256)])
def test_lnlstm_pointwise_vs_torch(rows, H):
    """gm_lnlstm_pointwise == the reference's LayerNormLSTMCell arithmetic after its two GEMMs
    (src/layernormlstm.py:24-42) in fp64 torch, on strided c / h' / c' rows."""
    gm, M, FU, W = mods()
    L = gm._lib
    torch.manual_seed(H)
    G = torch.randn(rows, 8 * H, device="cuda") * 3 + 0.5
    st = torch.randn(rows, 3 * H, device="cuda")
    c = st[:, H:2 * H]
    p = [torch.randn(4 * H, device="cuda") * s + o for s, o in ((0.2, 1), (0.1, 0), (0.2, 1), (0.1, 0), (0.3, 0))]
    lc = [torch.randn(H, device="cuda") * 0.2 + 1, torch.randn(H, device="cuda") * 0.1]
    out = torch.zeros(rows, 3 * H, device="cuda")
    L.check(L.lib().gm_lnlstm_pointwise(G.data_ptr(), 8 * H, c.data_ptr(), 3 * H, *[t.data_ptr() for t in p],
                                        lc[0].data_ptr(), lc[1].data_ptr(), rows, H, 1e-5, out.data_ptr(), 3 * H,
                                        out[:, H:].data_ptr(), 3 * H, L.stream_ptr()))
    d = lambda t: t.double()  # noqa: E731
    gi = F.layer_norm(d(G[:, :4 * H]), (4 * H,), d(p[0]), d(p[1]))
    gh = F.layer_norm(d(G[:, 4 * H:]), (4 * H,), d(p[2]), d(p[3]))
    g = gi + gh + d(p[4])
    i, f, gg, o = torch.sigmoid(g[:, :H]), torch.sigmoid(g[:, H:2 * H]), torch.tanh(g[:, 2 * H:3 * H]), \
        torch.sigmoid(g[:, 3 * H:])
    cy = F.layer_norm(f * d(c) + i * gg, (H,), d(lc[0]), d(lc[1]))
    hy = o * torch.tanh(cy)
    torch.testing.assert_close(out[:, :H].double(), hy, atol=2e-6, rtol=0)
    torch.testing.assert_close(out[:, H:2 * H].double(), cy, atol=4e-6, rtol=0)
    assert (out[:, 2 * H:] == 0).all()


@pytest.mark.parametrize("rows", [4096, 65540])
def test_joint_first_layer_split_vs_fp64(rows):
    """DQN first layer on [env obs | graph obs] as two GEMM sources (_JointLinearFn, training): the
    output, the graph-obs input gradient and the weight / bias gradients vs fp64, relative to the
    magnitude of each gradient's terms (the leaky mask from the kernel's own forward, as in
    test_linear_backward_large_batch); the env observation is a padded-row view like replay
    batches (130 of 132 columns)."""
    gm, M, FU, W = mods()
    torch.manual_seed(rows)
    A = 20
    B = (rows + A - 1) // A
    dqn = M.DQN(130 + 512, [512, 256], 4).cuda()
    envp = torch.randn(B, A, 132, device="cuda")
    env = envp[..., :130]
    graph = (torch.randn(B, A, 512, device="cuda") * 0.3).requires_grad_(True)
    lin = dqn.encoder.linear_layers[0]
    g2, e2 = graph.reshape(-1, 512), env.reshape(-1, 130)
    assert M.joint_first_layer_ok(g2, e2)
    y = M._JointLinearFn.apply(g2, e2, lin.weight, lin.bias, lin)
    xd = torch.cat([e2, g2.detach()], 1).double()
    wd = lin.weight.detach().double()
    pre = xd @ wd.t() + lin.bias.detach().double()
    yd = torch.where(pre >= 0, pre, 0.01 * pre)
    mag = xd.abs() @ wd.abs().t()
    assert ((y.detach().double() - yd).abs() / mag).max().item() < 4e-6
    gy = torch.randn_like(y) * 1e-4
    y.backward(gy)
    gyd = gy.double() * torch.where(y.detach() >= 0, 1.0, 0.01)
    refs = ((graph.grad.reshape(-1, 512), gyd @ wd[:, 130:], gyd.abs() @ wd[:, 130:].abs()),
            (lin.weight.grad, gyd.t() @ xd, gyd.abs().t() @ xd.abs()), (lin.bias.grad, gyd.sum(0), gyd.abs().sum(0)))
    for got, ref, mg in refs:
        rel = ((got.double() - ref).abs() / mg.clamp_min(1e-300)).max().item()
        assert rel < 1e-5, rel
    # the whole DQN: forward_split == forward on the joint observation
    with torch.no_grad():
        T = importlib.import_module("graph-marl_amd.train")
        q1 = dqn.forward_split(env, graph.detach())
        q0 = dqn(T.joint_obs(env, graph.detach()))
        torch.testing.assert_close(q1, q0, atol=1e-5, rtol=0)


@pytest.mark.parametrize("N,B", [(20, 4096), (10, 333), (30, 700), (40, 512), (50, 1024)])
def test_routing_encoder_fold_matches_two_kernels(N, B):
    """Round 5: the rollout computes NetMon encoder layer 1 inside layer 2's A-tile load (GM_A_ROUTING_ENC,
    the m x 512 layer-1 output never written) — layer 2's output equals gm_routing_node_encoder + the
    dense layer-2 GEMM on real routing node observations (random topologies, packets in flight), and the
    fp64 evaluation of the two layers within the split-f16 rollout tolerance."""
    gm, M, FU, W = mods()
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3,
                     agent_adjacency=False)
    env.reset_()
    for _ in range(3):  # packets on edges: nonzero load / count features
        env.step_(torch.randint(0, 4, (B, 20), device="cuda", dtype=torch.int32))
    torch.manual_seed(N)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    l0, l1 = list(nm.encode.linear_layers)[:2]
    x = env.node_obs.reshape(B * N, -1)
    nbr = env.nbr
    assert FU.renc_fold_ok(list(nm.encode.linear_layers), N, x.shape[1], nbr)
    y_fold = torch.empty(B * N, 256, device="cuda")
    FU.gemm(FU.routing_enc_src(l0, x, nbr, N), None, None, 0, l1.bias.data_ptr(), B * N, 256, FU._epi(l1.act),
            y_fold.data_ptr(), 256, x3=FU.pack_x3(l1))
    h1 = FU.routing_encoder(l0, x, nbr, B, N, torch.empty(B * N, 512, device="cuda"))
    y_two = FU._linear(h1, h1.stride(0), 512, l1, torch.empty(B * N, 256, device="cuda"))
    ref = F.leaky_relu(F.linear(F.leaky_relu(F.linear(x.double(), l0.weight.double(), l0.bias.double())),
                                l1.weight.double(), l1.bias.double()))
    d = (y_fold - y_two).abs().max().item()
    assert d < 2e-6, d  # same A values up to the encoder's fma contraction, same split-f16 GEMM
    assert (y_fold.double() - ref).abs().max().item() < 1e-5


def test_routing_encoder_fold_refuses_unsupported_cases():
    """gm_gemm_x3 only (not gm_gemm_f32) and 4N + 8 <= 208 (N <= 50)."""
    gm, M, FU, W = mods()
    N, B = 52, 8
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=1,
                     agent_adjacency=False)
    env.reset_()
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    l0, l1 = list(nm.encode.linear_layers)[:2]
    x = env.node_obs.reshape(B * N, -1)
    assert not FU.renc_fold_ok(list(nm.encode.linear_layers), N, x.shape[1], env.nbr)
    y = torch.empty(B * N, 256, device="cuda")
    with pytest.raises(gm._lib.GMError, match="4N"):
        FU.gemm(FU.routing_enc_src(l0, x, env.nbr, N), None, None, 0, l1.bias.data_ptr(), B * N, 256, 1,
                y.data_ptr(), 256, x3=FU.pack_x3(l1))


@pytest.mark.parametrize("N,B", [(20, 4096), (10, 333), (30, 700), (40, 512), (50, 1024)])
def test_encoder_chain_matches_layer_by_layer(N, B):
    """gm_encoder_x3 (round 5: NetMon encoder layers 1-3 of the rollout in one launch, layer 2's output kept
    on chip as split-f16 images) == the fold (layers 1 + 2) + the dense layer-3 GEMM, and fp64 within the
    rollout tolerance, on real routing node observations."""
    gm, M, FU, W = mods()
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=5,
                     agent_adjacency=False)
    env.reset_()
    for _ in range(3):
        env.step_(torch.randint(0, 4, (B, 20), device="cuda", dtype=torch.int32))
    torch.manual_seed(N + 1)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    l0, l1, l2 = list(nm.encode.linear_layers)
    x = env.node_obs.reshape(B * N, -1)
    nbr = env.nbr
    assert FU.encoder_chain_ok(list(nm.encode.linear_layers), N, x.shape[1], nbr)
    y = FU.encoder_chain(l0, l1, l2, x, nbr, N, torch.empty(B * N, 128, device="cuda"))
    y2 = torch.empty(B * N, 256, device="cuda")
    FU.gemm(FU.routing_enc_src(l0, x, nbr, N), None, None, 0, l1.bias.data_ptr(), B * N, 256, FU._epi(l1.act),
            y2.data_ptr(), 256, x3=FU.pack_x3(l1))
    y3 = FU._linear(y2, 256, 256, l2, torch.empty(B * N, 128, device="cuda"))
    ref = x.double()
    for lin in (l0, l1, l2):
        ref = F.leaky_relu(F.linear(ref, lin.weight.double(), lin.bias.double()))
    assert (y - y3).abs().max().item() < 1e-6
    assert (y.double() - ref).abs().max().item() < 1e-5
    assert FU.L.range_status() == 0
