"""Arithmetic of the split-f16 GEMMs at the PRODUCTION tiles.

The rollout's GEMMs run >= 32 768 rows with plain operands (AX = 0 in gm_gemm.hip) on the LDS-DMA
kernel k_gemm3g: tile 12 (128x128, 2 blocks / CU) for the dense layers, tile 9 (128x256, 3 stages,
ping-pong k loop) for DQN layer 1 on its READOUT source, and the fused DQN layer 2 + Q head kernel. The
smaller-M tests in test_fused_gpu.py run the register-staged k_gemm3 instead, so they do not pin these.

Each case draws activation ROWS whose scales span 2^-12 .. 2^3 (one power of two per row: a row of
small activations is what a denormal low split piece would hurt) and weight rows spanning 2^-12 .. 2^0,
and bounds the error of every output against fp64, relative to sum |a * w| of that output (the error
measure of an fp32 dot product), for both the split-f16 form and the exact-f32 form on the same inputs.

Stated bound (round 6): split-f16 <= max(1e-6, 2 x the exact-f32 GEMM's own error);
measured 2.5-6.4e-7 against 3.5-10.2e-7 for the exact-f32 form (round 5: max(4e-6, 4x), which a 6-15x
regression would have passed). Every case prints its error / tolerance ratio. The dropped a_lo * w_lo term
and the 22-bit pieces put the split form at ~2^-22 of sum |a * w|; the exact f32 MFMA chain at ~2^-24 * a
small K-dependent factor. A low piece that rounds to an f16 denormal (|a| < 2^-3 without the 2^12 scale)
has an absolute error up to 2^-25 per element and fails this bound on the 2^-12 rows."""
import importlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BOUND_ABS = 1e-6
BOUND_X_F32 = 2.0


def _check(name, e_x3, e_f32):
    tol = max(BOUND_ABS, BOUND_X_F32 * e_f32)
    print(f"{name}: split {e_x3:.3g}, exact-f32 {e_f32:.3g}, tolerance {tol:.3g}, worst/tolerance {e_x3 / tol:.3f}")
    assert e_x3 <= tol, (name, e_x3, e_f32)


def mods():
    return importlib.import_module("graph-marl_amd.model"), importlib.import_module("graph-marl_amd.fused")


def _operands(m, k, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(m, k, device="cuda", generator=g)
    x *= torch.exp2(torch.randint(-12, 4, (m, 1), device="cuda", generator=g).float())
    w = torch.randn(n, k, device="cuda", generator=g)
    w *= torch.exp2(torch.randint(-12, 1, (n, 1), device="cuda", generator=g).float())
    return x, w


def _rel(y, ref, mag):
    return ((y.double() - ref).abs() / mag.clamp_min(1e-300)).max().item()


def _gemm(FU, x, wp, ldw, n, k, form):
    m = x.shape[0]
    y = torch.empty(m, n, device="cuda")
    b = torch.zeros(n, device="cuda")
    FU.gemm(FU.dense(x.data_ptr(), x.stride(0), k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 0, y.data_ptr(), n,
            x3=FU.X3(wp, ldw, n, k) if form == "x3" else None)
    return y


@pytest.mark.parametrize("name,m,n,k,tile", [
    ("dqn_layer1_dense_tile12", 81920, 512, 640, -1),
    ("dqn_layer1_tile9", 81920, 512, 640, 9),
    ("cell_k256", 81920, 512, 256, -1),
    ("encoder3_k256", 81920, 128, 256, -1),
    ("encoder2_k512", 40960, 256, 512, -1),
])
def test_split_gemm_error_at_production_tile(name, m, n, k, tile):
    M, FU = mods()
    lib = FU._setup()
    x, w = _operands(m, k, n, seed=m + n + k + tile)
    wp, ldw = FU._pad_cols(w)
    ref = F.linear(x.double(), w.double())
    mag = F.linear(x.abs().double(), w.abs().double())
    lib.gm_gemm_set_tile(tile)
    try:
        errs = {form: _rel(_gemm(FU, x, wp, ldw, n, k, form), ref, mag) for form in ("f32", "x3")}
    finally:
        lib.gm_gemm_set_tile(-1)
    print(f"{name}: relative error vs fp64 (of sum |a w|): {errs}")
    assert errs["f32"] < 2e-6, errs  # the exact-f32 MFMA chain itself, K <= 640
    _check(name, errs["x3"], errs["f32"])


def test_split_readout_layer_error_at_production_tile():
    """DQN layer 1 as the rollout runs it: READOUT source [h_final(v) | h_prev(nbr 0..2 of v)] gathered
    per agent row ‖ the GEMM-ready env rows, 4096 graphs x 20 agents = 81 920 rows, K = 512 + 128,
    on its default tile (9). Node rows carry one power-of-two scale each (2^-12 .. 2^3)."""
    M, FU = mods()
    G, N, A, H, od = 4096, 20, 20, 128, 128
    g = torch.Generator(device="cuda").manual_seed(3)
    node_scale = torch.exp2(torch.randint(-12, 4, (G * N, 1), device="cuda", generator=g).float())
    hf = torch.randn(G * N, 2 * H, device="cuda", generator=g) * node_scale
    hp = torch.randn(G * N, 2 * H, device="cuda", generator=g) * node_scale.roll(7, 0)
    # 3-regular-ish neighbour table (ascending ids, some missing = -1 like odd-degree leftovers)
    nbr = torch.stack([(torch.arange(N, device="cuda") + d) % N for d in (1, 5, 9)], 1).sort(1).values
    nbr = nbr.expand(G, N, 3).contiguous().int()
    nbr[::3, 0, 2] = -1
    agent_node = torch.randint(0, N, (G, A), device="cuda", generator=g).int()
    env = torch.randn(G * A, od, device="cuda", generator=g) * torch.exp2(
        torch.randint(-12, 4, (G * A, 1), device="cuda", generator=g).float())
    K0 = 4 * H
    w = torch.randn(512, K0 + od, device="cuda", generator=g) * torch.exp2(
        torch.randint(-12, 1, (512, 1), device="cuda", generator=g).float())
    # the A operand the kernel gathers, in fp64
    rows = (torch.arange(G, device="cuda")[:, None] * N + agent_node.long()).reshape(-1)
    gi = torch.arange(G, device="cuda").repeat_interleave(A)
    parts = [hf[rows, :H].double()]
    for s in range(3):
        nb = nbr[gi, agent_node.reshape(-1).long(), s].long()
        v = hp[(gi * N + nb.clamp_min(0)), :H].double()
        parts.append(torch.where((nb >= 0)[:, None], v, torch.zeros_like(v)))
    a = torch.cat(parts + [env.double()], 1)
    ref = a @ w.double().t()
    mag = a.abs() @ w.abs().double().t()
    wp, ldw = FU._pad_cols(w)
    b = torch.zeros(512, device="cuda")
    errs = {}
    for form in ("f32", "x3"):
        y = torch.empty(G * A, 512, device="cuda")
        FU.gemm(FU.readout(hf.data_ptr(), 2 * H, hp.data_ptr(), 2 * H, nbr, agent_node, N, H),
                FU.dense(env.data_ptr(), od, od), wp.data_ptr(), ldw, b.data_ptr(), G * A, 512, 0, y.data_ptr(), 512,
                x3=FU.X3(wp, ldw, 512, K0 + od) if form == "x3" else None)
        errs[form] = _rel(y, ref, mag)
    print(f"dqn_layer1_readout_tile9: relative error vs fp64 (of sum |a w|): {errs}")
    assert errs["f32"] < 2e-6, errs  # the exact-f32 MFMA chain itself, K <= 640
    _check("dqn_layer1_readout_tile9", errs["x3"], errs["f32"])


def test_split_head_error_at_production_tile():
    """The fused DQN layer 2 + Q head (gm_gemm_x3_head, 128x128 blocks with partial Q per column block)
    at 81 920 x 256 x 512: hidden output (no activation) and Q, both against fp64 relative to their
    sum |a w| magnitudes."""
    M, FU = mods()
    m, n, k, nq = 81920, 256, 512, 4
    x, w = _operands(m, k, n, seed=11)
    lin = M.Linear(k, n, act=0).cuda()
    fc = M.Linear(n, nq, act=0).cuda()
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.zero_()
        fc.bias.zero_()
    q = torch.empty(m, nq, device="cuda")
    y = torch.empty(m, n, device="cuda")
    FU.linear_head(lin, fc, x, k, k, q, y=y)
    hid = F.linear(x.double(), w.double())
    mag = F.linear(x.abs().double(), w.abs().double())
    e_hid = _rel(y, hid, mag)
    qref = F.linear(hid, fc.weight.double())
    qmag = F.linear(mag, fc.weight.abs().double())
    e_q = _rel(q, qref, qmag)
    y32 = _gemm(FU, x, *FU._pad_cols(w), n, k, "f32")
    e32 = _rel(y32, hid, mag)
    print(f"head: hidden {e_hid:.3g}, q {e_q:.3g}, exact-f32 hidden {e32:.3g}")
    _check("head hidden", e_hid, e32)
    _check("head q", e_q, e32)
