"""GPU parity of the sequence-batched update (graph-marl_amd/train_seq.py): its kernels against
torch autograd, the whole update against the reference's golden update (src/main.py:832-1022),
and against the autograd path (train.dqn_update) on replayed rollout data at training size."""
import ctypes as C
import importlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_replay as R

pytestmark = pytest.mark.gpu


def mods():
    return (importlib.import_module("graph-marl_amd.model"), importlib.import_module("graph-marl_amd.train"),
            importlib.import_module("graph-marl_amd.train_seq"), importlib.import_module("graph-marl_amd.fused"),
            importlib.import_module("graph-marl_amd._lib"))


def _rel(a, b):
    return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)


def _pack_bits(b):
    """bool [rows][cols] -> int32 words [rows][ceil(cols / 32)], bit c % 32 of word c / 32."""
    rows, cols = b.shape
    W = (cols + 31) // 32
    x = torch.zeros(rows, W * 32, dtype=torch.int64, device=b.device)
    x[:, :cols] = b.long()
    w = (x.view(rows, W, 32) << torch.arange(32, device=b.device)).sum(-1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32).contiguous()


@pytest.mark.parametrize("n,mfma", [(512, 1), (256, 0), (96, 1), (40, 1)])
def test_forward_sign_bits(n, mfma):
    """Sign bits written by the forward epilogues (k_gemm3g 16x16 / 32x32, k_gemm3, routing encoder)
    equal the activation's y > 0."""
    M, T, S, FU, L = mods()
    gm = importlib.import_module("graph-marl_amd")
    torch.manual_seed(n)
    m, k = 40000, 256
    x = torch.randn(m, k, device="cuda")
    lin = M.Linear(k, n, act=1).cuda()
    y = torch.empty(m, n, device="cuda")
    bits = S._sign_bits(m, n, "cuda")
    slot = torch.zeros(1, device="cuda")
    FU.L.check(FU._setup().gm_gemm_set_mfma(mfma))
    try:
        for tile in (-1, 0):
            FU._setup().gm_gemm_set_tile(tile)
            bits.fill_(-7)
            S._gemm_amax(x, k, k, S._lin_x3(lin), lin.bias, m, n, FU.GM_EPI_BIAS_LEAKY, y, n, slot, sbits=bits)
            assert torch.equal(bits, _pack_bits(y > 0)), tile
    finally:
        FU._setup().gm_gemm_set_tile(-1)
        FU._setup().gm_gemm_set_mfma(2)
    B, N = 64, 20
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3)
    env.reset()
    for out in (512, 64):
        lin0 = M.Linear(4 * N + 8, out, act=1).cuda()
        x0 = env.node_obs.reshape(-1, 4 * N + 8)
        y0 = torch.empty(B * N, out, device="cuda")
        b0 = S._sign_bits(B * N, out, "cuda")
        FU.routing_encoder(lin0, x0, env.nbr, B, N, y0, sbits=b0)
        assert torch.equal(b0, _pack_bits(y0 > 0)), out


def _fro(a, b):
    return (a.double() - b.double()).norm().item() / max(b.double().norm().item(), 1e-30)


@pytest.mark.parametrize("form,mfma", [(-1, 1), (0, 1), (1, 1), (1, 0), (2, 1), (2, 0)])
@pytest.mark.parametrize("m,n,k,split", [(70000, 512, 256, 512), (4099, 256, 512, 128), (300, 64, 48, 40)])
def test_dgrad_epilogue_vs_torch(m, n, k, split, form, mfma):
    """gm_gemm_x3_dgrad: D = g W (scaled split-f16 A), leaky derivative of the mask on columns < split,
    bias partials, max |g|; columns >= split unchanged into y2. Every kernel form (gm_gemm_set_dgrad)
    and MFMA shape of the LDS-DMA forms."""
    M, T, S, FU, L = mods()
    lib = FU._setup()
    L.check(lib.gm_gemm_set_dgrad(form))
    L.check(lib.gm_gemm_set_mfma(mfma))
    try:
        _dgrad_case(M, T, S, FU, L, m, n, k, split)
    finally:
        lib.gm_gemm_set_dgrad(-1)
        lib.gm_gemm_set_mfma(2)


def _dgrad_case(M, T, S, FU, L, m, n, k, split):
    torch.manual_seed(m)
    g = torch.randn(m, k, device="cuda") * 1e-4
    w = torch.randn(k, n, device="cuda") / k ** 0.5  # gx = g @ w, w = W of a Linear [k out][n in]
    mask = torch.randn(m, split, device="cuda")
    mask[0, :7] = 0.0  # exact zeros take the slope (torch: input > 0)
    sc = torch.empty(1, device="cuda")
    L.check(FU._setup().gm_absmax_scale(g.data_ptr(), g.numel(), sc.data_ptr(), L.stream_ptr()))
    x3 = S._x3(w.t().contiguous())
    y = torch.empty(m, split, device="cuda")
    y2 = torch.empty(m, max(n - split, 1), device="cuda")
    part = torch.empty((m + 127) // 128, split, device="cuda")
    gmax = torch.zeros(1, device="cuda")
    bits = _pack_bits(mask > 0)
    S._dgrad(g, k, k, sc, x3, m, n, split, bits, bits.stride(0), y, split, y2 if split < n else None, n - split, part,
             gmax)
    ref = g.double() @ w.double()
    lo = torch.where(mask.double() > 0, ref[:, :split], 0.01 * ref[:, :split])
    assert _rel(y, lo) < 1e-5
    if split < n:
        assert _rel(y2, ref[:, split:]) < 1e-5
    assert _rel(part.sum(0), lo.sum(0)) < 1e-5
    assert gmax.item() == y.abs().max().item()  # the slot holds the max's float bits


@pytest.mark.parametrize("rows,cols,nq", [(100000, 256, 4), (777, 32, 3), (5, 64, 1), (300, 100, 2)])
def test_qhead_bwd_vs_torch(rows, cols, nq):
    M, T, S, FU, L = mods()
    torch.manual_seed(rows)
    z = torch.randn(rows, cols, device="cuda", requires_grad=True)
    y = F.leaky_relu(z, 0.01)
    y.retain_grad()
    wq = torch.randn(nq, cols, device="cuda", requires_grad=True)
    bq = torch.randn(nq, device="cuda", requires_grad=True)
    q = F.linear(y, wq, bq)
    dq = torch.randn(rows, nq, device="cuda")
    q.backward(dq)
    rpb = 512
    nb = (rows + rpb - 1) // rpb
    g = torch.empty(rows, cols, device="cuda")
    pb, pw, pq = (torch.empty(nb, cols, device="cuda"), torch.empty(nb, nq, cols, device="cuda"),
                  torch.empty(nb, nq, device="cuda"))
    sc = torch.empty(1, device="cuda")
    yd = y.detach().contiguous()
    L.check(L.lib().gm_qhead_bwd(dq.data_ptr(), nq, nq, wq.data_ptr(), cols, yd.data_ptr(), cols, rows, cols, 1,
                                 g.data_ptr(), cols, pb.data_ptr(), pw.data_ptr(), pq.data_ptr(), rpb, sc.data_ptr(),
                                 L.stream_ptr()))
    assert _rel(g, z.grad) < 1e-6
    assert _rel(pb.sum(0), z.grad.sum(0)) < 1e-5
    assert _rel(pw.sum(0), wq.grad) < 1e-5
    assert _rel(pq.sum(0), bq.grad) < 1e-5


@pytest.mark.parametrize("mean", [0, 1])
@pytest.mark.parametrize("H", [128, 32, 30])
def test_lstm_cell_bwd_vs_autograd(mean, H):
    """gm_lstm_cell_bwd with every gradient source (two plain dh, the transposed aggregate of dm,
    masked external dh / dc, plain dc) against torch autograd of nn.LSTMCell gate math."""
    M, T, S, FU, L = mods()
    gm = importlib.import_module("graph-marl_amd")
    torch.manual_seed(H + mean)
    B, N = 48, 20
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=1)
    env.reset()
    nbr = env.nbr.contiguous()
    m = B * N
    pre = torch.randn(m, 4 * H, device="cuda", requires_grad=True)
    c = torch.randn(m, H, device="cuda", requires_grad=True)
    i, f, gg, o = torch.sigmoid(pre[:, :H]), torch.sigmoid(pre[:, H:2 * H]), torch.tanh(pre[:, 2 * H:3 * H]), \
        torch.sigmoid(pre[:, 3 * H:])
    c1 = f * c + i * gg
    h1 = o * torch.tanh(c1)
    act = torch.cat([i, f, gg, o], 1).detach().contiguous()
    dh0, dh1 = torch.randn(m, H, device="cuda"), torch.randn(m, H, device="cuda")
    dm = torch.randn(m, H, device="cuda")
    dhe, dce, dcp = torch.randn(m, H, device="cuda"), torch.randn(m, H, device="cuda"), torch.randn(m, H, device="cuda")
    emask = (torch.rand(B, device="cuda") < 0.3)
    keep = (~emask).float().repeat_interleave(N).unsqueeze(1)
    aggT = M.mp_aggregate(dm, nbr, mean) if mean == 0 else None
    if mean:  # transpose of the mean aggregate: dh[j] = sum_{n in {j} U nbr(j)} dm[n] / cnt(n)
        cnt = (nbr >= 0).sum(-1).reshape(-1, 1).float() + 1
        aggT = M.mp_aggregate((dm / cnt).contiguous(), nbr, 0)
    dh = dh0 + dh1 + aggT + keep * dhe
    dc = dcp + keep * dce
    torch.autograd.backward([h1, c1], [dh, dc])
    a = L.LSTMBwdArgs()
    a.act, a.ld_act = act.data_ptr(), 4 * H
    cd, c1d = c.detach().contiguous(), c1.detach().contiguous()
    a.c_in, a.ld_cin, a.c_out, a.ld_cout = cd.data_ptr(), H, c1d.data_ptr(), H
    a.dh0, a.ld_dh0, a.dh1, a.ld_dh1 = dh0.data_ptr(), H, dh1.data_ptr(), H
    a.dm, a.ld_dm, a.nbr, a.n_nodes, a.deg, a.mean = dm.data_ptr(), H, nbr.data_ptr(), N, 3, mean
    a.dh_ext, a.ld_ext, a.dc_ext, a.ld_dcext = dhe.data_ptr(), H, dce.data_ptr(), H
    em = emask.to(torch.uint8)
    a.ext_mask, a.rows_per_sample = em.data_ptr(), N
    a.dc, a.ld_dc = dcp.data_ptr(), H
    a.m, a.hidden = m, H
    dg = torch.empty(m, 4 * H, device="cuda")
    dco = torch.empty(m, H, device="cuda")
    part = torch.empty((m + 63) // 64, 4 * H, device="cuda")
    sc = torch.empty(1, device="cuda")
    mx = torch.zeros(1, device="cuda")
    a.dgates, a.ld_dg, a.dc_out, a.ld_dco = dg.data_ptr(), 4 * H, dco.data_ptr(), H
    a.bias_part, a.rows_per_block, a.dg_scale, a.dg_max = part.data_ptr(), 64, sc.data_ptr(), mx.data_ptr()
    L.check(L.lib().gm_lstm_cell_bwd(C.byref(a), L.stream_ptr()))
    assert _rel(dg, pre.grad) < 2e-6
    assert _rel(dco, c.grad) < 2e-6
    assert _rel(part.sum(0), pre.grad.sum(0)) < 1e-5
    assert mx.item() == dg.abs().max().item()


def _golden_seq(g, dev, netmon, RBm, state0=None):
    """SeqBatch of the reference's golden update (L steps of B sequences; next obs = obs of t + 1)."""
    M, T, S, FU, L = mods()
    f = lambda a: torch.as_tensor(a, device=dev)  # noqa: E731
    Lq = g["actions"].shape[0]
    od = g["agent_obs"].shape[-1]
    odp = (od + 3) // 4 * 4
    obs = F.pad(f(g["agent_obs"]), (0, odp - od))  # [L + 1, B, A, odp]
    nbr = torch.stack([M.dense_to_nbr(f(g["node_adj"][t]).float()) for t in range(Lq + 1)])
    an = torch.stack([M.node_agent_to_index(f(g["node_agent"][t]).float()) for t in range(Lq + 1)])
    node_obs = f(g["node_obs"])

    def next_fields(t, rows):
        r = slice(None) if rows is None else rows
        return obs[t + 1][r], node_obs[t + 1][r], an[t + 1][r].contiguous()

    return S.SeqBatch(obs[:Lq].contiguous(), od, f(g["actions"]).long(), f(g["reward"]), f(g["done"]).bool(),
                      f(g["episode_done"]).bool(), node_obs[:Lq].contiguous(), nbr[:Lq].contiguous(),
                      an[:Lq].contiguous(), f(g["node_state0"]) if state0 is None else state0, next_fields)


@pytest.mark.parametrize("name", ["train.npz", "train_big.npz", "train_prod.npz"])
def test_seq_update_matches_reference_golden(name):
    """The sequence-batched update on the reference's golden updates at the autograd path's
    tolerances: q, targets, loss, raw and clipped gradients, AdamW step, soft target update.
    train.npz: NetMon H = 32, encoder [64, 48], DQN [64, 32], L = 3 with episode ends;
    train_big.npz: the CLI-default sizes with 256 graphs x 4 steps (20 480 node and agent rows per
    batched layer, every kernel in its HIP form); train_prod.npz: 512 graphs x 4 steps (40 960 rows
    per batched layer: the production LDS-DMA forward / input-gradient tiles, >= 32 768 rows)."""
    M, T, S, FU, L = mods()
    RBm = importlib.import_module("graph-marl_amd.replaybuffer")
    import golden_update as GU
    from test_train_gpu import check_update
    g = np.load(f"{R.GOLDEN}/{name}")
    dev = torch.device("cuda")
    netmon, model, target, state0 = GU.build(g, M, dev)
    assert S.seq_ok(netmon, model, target)
    seq = _golden_seq(g, dev, netmon, RBm, state0)
    params = list(model.parameters()) + list(netmon.parameters())
    names = [f"model_{k}" for k, _ in model.named_parameters()] + [f"netmon_{k}" for k, _ in netmon.named_parameters()]
    opt = torch.optim.AdamW(params, lr=float(g["lr"]))
    loss, q, qt = S.seq_loss(netmon, model, target, seq, float(g["gamma"]), params)
    for t in range(q.shape[0]):
        np.testing.assert_allclose(q[t].detach().cpu().numpy(), g[f"q_{t}"], atol=1e-5, rtol=0, err_msg=f"q_{t}")
        np.testing.assert_allclose(qt[t].cpu().numpy(), g[f"qtarget_{t}"], atol=1e-5, rtol=0, err_msg=f"qt_{t}")
    np.testing.assert_allclose(loss.item(), g["loss"].item(), rtol=1e-5, atol=1e-6)
    opt.zero_grad()
    loss.backward()
    check_update(g, names, params, opt, model, target, T)


@pytest.mark.parametrize("K,agg,tiles", [(1, "sum", "common"), (2, "mean", "common"), (1, "sum", "default")])
def test_seq_update_matches_autograd_path_on_rollout(K, agg, tiles):
    """Replayed rollout data (64 envs x 30 steps, episodes of 10 steps), the CLI-default model sizes:
    the same sampled sequences through train.dqn_loss (autograd, consecutive target reuse) and the
    sequence-batched path give the same q, targets, loss and gradients (fp32 order). tiles "common":
    both paths on one GEMM tile (identical forward bits); "default": each path on the tiles it picks
    in production (the batched path's 40 960-row layers on the LDS-DMA forms), compared kink-tolerantly."""
    gm = importlib.import_module("graph-marl_amd")
    M, T, S, FU, L = mods()
    RB = importlib.import_module("graph-marl_amd.replaybuffer")
    W = importlib.import_module("graph-marl_amd.wrapper")
    P = importlib.import_module("graph-marl_amd.policy")
    B, N, A = 64, 20, 20
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), A, n_env=B, seed=7,
                     obs_extra=512, agent_adjacency=False)
    torch.manual_seed(K)
    netmon = M.NetMon(4 * N + 8, 128, [512, 256], K, agg_type=agg).cuda()
    model = M.DQN(6 * N + 10 + 512, [512, 256], 4).cuda()
    target = M.DQN(6 * N + 10 + 512, [512, 256], 4).cuda()
    target.load_state_dict(model.state_dict())
    with torch.no_grad():
        for p in target.parameters():
            p.add_(0.01 * torch.randn_like(p))
    wenv = W.NetMonWrapper(env, netmon, 1)
    pol = P.EpsilonGreedy(wenv, model, epsilon=0.5, epsilon_decay=1.0, epsilon_update_freq=100, step_before_train=0)
    rb = RB.ReplayBuffer(0, 40 * B, B, A, env.obs_dim, N, 4 * N + 8, netmon.get_state_size(), "cuda")
    wenv.reset()
    for t in range(30):
        obs = env.obs.clone()
        node_obs, agent_node = env.node_obs.clone(), env.agent_node.clone()
        state_in = wenv.last_netmon_state
        act = pol(wenv.obs)
        wenv.step_(act)
        rb.add(obs, act, env.reward, env.obs, env.done.bool(), (t + 1) % 10 == 0, state_in, node_obs, env.nbr,
               agent_node, env.node_obs, env.agent_node)
        if (t + 1) % 10 == 0:
            wenv.reset()
    params = list(model.parameters()) + list(netmon.parameters())
    rng0 = rb.rng.clone()
    batches = list(rb.get_batch(512, sequence_length=8, lazy_next=True))
    rb.rng.copy_(rng0)
    seq = rb.get_sequences(512, 8)
    assert all(torch.equal(b.idx[0], seq.idx[0][t]) for t, b in enumerate(batches))
    assert seq.episode_done[:-1].any()
    netmon.train()
    model.train()
    # both paths on the same GEMM tile (k_gemm3, 128x128), so every forward pre-activation has the
    # same bits and leaky_relu's kink cannot flip between them (see below)
    if tiles == "default":
        _compare_paths(M, T, S, L, netmon, model, target, batches, seq, params, kink_tolerant=True)
        return
    lib = FU._setup()
    lib.gm_gemm_set_tile(0)
    try:
        _compare_paths(M, T, S, L, netmon, model, target, batches, seq, params)
    finally:
        lib.gm_gemm_set_tile(-1)


def _compare_paths(M, T, S, L, netmon, model, target, batches, seq, params, kink_tolerant=False):
    l0, q0, t0 = T.dqn_loss(netmon, model, target, batches, 0.98, consecutive=True)
    for p in params:
        p.grad = None
    l0.backward()
    g0 = [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    netmon.state = None
    l1, q1, t1 = S.seq_loss(netmon, model, target, seq, 0.98, params)
    l1.backward()
    g1 = [p.grad.clone() for p in params]
    # exact-fp32 reference: the autograd path with every GEMM in fp32 (GM_GEMM=f32 semantics)
    for p in params:
        p.grad = None
    netmon.state = None
    old = L.GEMM_MODE
    L.GEMM_MODE = "f32"
    try:
        lf, _, _ = T.dqn_loss(netmon, model, target, batches, 0.98, consecutive=True)
        lf.backward()
    finally:
        L.GEMM_MODE = old
    gf = [p.grad.clone() for p in params]
    for t in range(8):
        torch.testing.assert_close(q1[t], q0[t].detach(), rtol=0, atol=2e-5)
        torch.testing.assert_close(t1[t], t0[t], rtol=0, atol=2e-5)
    torch.testing.assert_close(l1, l0.detach(), rtol=1e-5, atol=1e-8)
    # Frobenius-relative errors vs exact fp32. On their default tiles the two paths run the encoder /
    # DQN layers at different batch sizes, i.e. on different GEMM kernels whose summation orders differ
    # in the last bits; a pre-activation within rounding of 0 then takes the other side of leaky_relu's
    # kink (derivative 1 vs 0.01; tools/seq_debug.py found 5 of 21 M elements, exact 0.0 in one order,
    # 2^-27 in the other), which moves the encoder gradients by ~1e-4 — hence the common tile above
    errs = {}
    for (n, _), a, b, c in zip(list(model.named_parameters()) + list(netmon.named_parameters()), g0, g1, gf):
        errs[n] = (_fro(a, c), _fro(b, c))
    print("Frobenius-relative gradient error vs exact fp32 (autograd x3, sequence-batched x3):", errs)
    for n, (e_old, e_new) in errs.items():
        # default tiles: a kink flip moves a few gradient elements by ~1e-4 (see above); the bound
        # still fails any systematic error (a wrong tile gives O(1) relative errors)
        assert e_new < (max(1e-3, 4 * e_old) if kink_tolerant else max(2e-5, 2 * e_old)), (n, e_old, e_new)


def test_operands_beyond_2gb():
    """Dense GEMM sources and weight-gradient operands past 2 GB (the kernels address rows relative
    to their block / k chunk with 32-bit offsets): split-f16 forward GEMM and weight gradient vs
    fp64 on a 1.1 M x 512 operand (2.25 GB)."""
    M, T, S, FU, L = mods()
    torch.manual_seed(5)
    m, k, n = 1_100_000, 512, 64
    x = torch.randn(m, k, device="cuda")
    assert x.numel() * 4 > 2 ** 31
    lin = M.Linear(k, n, act=1).cuda()
    y = torch.empty(m, n, device="cuda")
    slot = torch.zeros(1, device="cuda")
    S._gemm_amax(x, k, k, S._lin_x3(lin), lin.bias, m, n, FU.GM_EPI_BIAS_LEAKY, y, n, slot)
    rows = torch.cat([torch.arange(0, 256, device="cuda"), torch.arange(m - 256, m, device="cuda"),
                      torch.randint(0, m, (4096,), device="cuda")])
    ref = F.leaky_relu(F.linear(x[rows].double(), lin.weight.double(), lin.bias.double()), 0.01)
    assert (y[rows].double() - ref).abs().max().item() < 1e-4
    assert slot.item() == x.abs().max().item()
    gy = torch.randn(m, n, device="cuda") * 1e-3
    gw = M._wgrad(gy, x, k)
    refw = gy.double().t() @ x.double()
    assert _rel(gw, refw) < 1e-5


@pytest.mark.parametrize("rec", [(20, 132), (20, 88), (20, 256), (4,)])
def test_gather_records_matches_indexing(rec):
    """gm_gather_records (replaybuffer.get_sequences' field gather) == torch advanced indexing
    src[slots, env], bit for bit: [L, B] slots with per-column envs, a 1-D row subset, no rows."""
    RB = importlib.import_module("graph-marl_amd.replaybuffer")
    torch.manual_seed(len(rec))
    S_, B_ = 37, 64
    src = torch.randn(S_, B_, *rec, device="cuda")
    slots = torch.randint(0, S_, (8, 300), device="cuda")
    env = torch.randint(0, B_, (300,), device="cuda")
    assert torch.equal(RB.ReplayBuffer._records(src, slots, env), src[slots, env.expand_as(slots)])
    rows = torch.randint(0, 300, (77,), device="cuda")
    assert torch.equal(RB.ReplayBuffer._records(src, slots[3][rows], env[rows]), src[slots[3][rows], env[rows]])
    e = torch.empty(0, dtype=torch.long, device="cuda")
    assert RB.ReplayBuffer._records(src, e, e).shape == (0, *rec)
