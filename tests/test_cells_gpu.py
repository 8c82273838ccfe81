"""The hand-written LayerNorm-LSTM and GRU training cells (model._LNLSTMFn / model._GRUFn on
gm_lnlstm_fwd / gm_lnlstm_bwd / gm_gru_pointwise / gm_gru_bwd) against torch fp64 autograd of the
reference arithmetic (src/layernormlstm.py:24-42, torch.nn.GRUCell): outputs and every gradient
(raw gate rows, state, LayerNorm weights and biases, gate bias), at training row counts and with
either output gradient absent."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _ref_lnlstm(gi, gh, c, wi, bi, wh, bh, bias, wc, bc, eps=1e-5):
    """src/layernormlstm.py:24-42 after its two GEMMs (fp64 torch)."""
    H = c.shape[1]
    ln = torch.nn.functional.layer_norm
    g = ln(gi, (4 * H,), wi, bi, eps) + ln(gh, (4 * H,), wh, bh, eps) + bias
    i, f, gg, o = g.chunk(4, 1)
    cy = ln(torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg), (H,), wc, bc, eps)
    return torch.sigmoid(o) * torch.tanh(cy), cy


@pytest.mark.parametrize("M,H", [(5000, 128), (777, 32), (300, 200)])
@pytest.mark.parametrize("grads", ["both", "h", "c"])
def test_lnlstm_cell_fwd_bwd(M, H, grads):
    Mo = importlib.import_module("graph-marl_amd.model")
    torch.manual_seed(M + H)
    dev = "cuda"
    gi = (torch.randn(M, 4 * H, device=dev) * 0.7 + 0.1).requires_grad_()
    gh = (torch.randn(M, 4 * H, device=dev) * 0.5 - 0.2).requires_grad_()
    c = torch.randn(M, H, device=dev).requires_grad_()
    ps = [(1 + 0.1 * torch.randn(4 * H, device=dev)).requires_grad_(), (0.1 * torch.randn(4 * H, device=dev)).requires_grad_(),
          (1 + 0.1 * torch.randn(4 * H, device=dev)).requires_grad_(), (0.1 * torch.randn(4 * H, device=dev)).requires_grad_(),
          (0.1 * torch.randn(4 * H, device=dev)).requires_grad_(), (1 + 0.1 * torch.randn(H, device=dev)).requires_grad_(),
          (0.1 * torch.randn(H, device=dev)).requires_grad_()]
    h1, c1 = Mo._LNLSTMFn.apply(gi, gh, c, *ps, 1e-5)
    leaves = [gi, gh, c] + ps
    r64 = [t.detach().double().requires_grad_() for t in leaves]
    rh, rc = _ref_lnlstm(*r64)
    assert _rel(h1, rh) < 2e-6 and _rel(c1, rc) < 2e-6
    assert (h1.double() - rh).abs().max() < 1e-5 and (c1.double() - rc).abs().max() < 2e-5
    dh = torch.randn(M, H, device=dev)
    dc = torch.randn(M, H, device=dev)
    outs, routs, gs = [], [], []
    if grads in ("both", "h"):
        outs.append(h1), routs.append(rh), gs.append(dh)
    if grads in ("both", "c"):
        outs.append(c1), routs.append(rc), gs.append(dc)
    got = torch.autograd.grad(outs, leaves, gs)
    ref = torch.autograd.grad(routs, r64, [g.double() for g in gs])
    names = ["gi", "gh", "c", "ln_in_w", "ln_in_b", "ln_hid_w", "ln_hid_b", "bias", "ln_cell_w", "ln_cell_b"]
    for n, a, b in zip(names, got, ref):
        assert _rel(a, b) < 1e-5, f"{n}: rel err {_rel(a, b)}"


@pytest.mark.parametrize("M,H", [(5000, 128), (777, 32)])
def test_gru_cell_fwd_bwd(M, H):
    Mo = importlib.import_module("graph-marl_amd.model")
    torch.manual_seed(M + H)
    dev = "cuda"
    gi = torch.randn(M, 3 * H, device=dev).requires_grad_()
    gh = torch.randn(M, 3 * H, device=dev).requires_grad_()
    h = torch.randn(M, H, device=dev).requires_grad_()
    h1 = Mo._GRUFn.apply(gi, gh, h)
    a, b, hh = (t.detach().double().requires_grad_() for t in (gi, gh, h))
    r = torch.sigmoid(a[:, :H] + b[:, :H])
    z = torch.sigmoid(a[:, H:2 * H] + b[:, H:2 * H])
    n = torch.tanh(a[:, 2 * H:] + r * b[:, 2 * H:])
    ref = (1 - z) * n + z * hh
    assert (h1.double() - ref).abs().max() < 1e-6
    g = torch.randn(M, H, device=dev)
    got = torch.autograd.grad(h1, (gi, gh, h), g)
    exp = torch.autograd.grad(ref, (a, b, hh), g.double())
    for nm, x, y in zip(("gi", "gh", "h"), got, exp):
        assert _rel(x, y) < 1e-6, nm


@pytest.mark.parametrize("rnn", ["lnlstm", "gru"])
def test_cell_modules_match_reference_cells(rnn):
    """LayerNormLSTMCell / GRUCell modules (GEMMs + the HIP cell) vs fp64 torch of the reference
    cell with the same parameters, forward and parameter gradients, at 5120 rows (HIP GEMM forms)."""
    Mo = importlib.import_module("graph-marl_amd.model")
    torch.manual_seed(3)
    H, M = 128, 5120
    cell = (Mo.LayerNormLSTMCell(H, H) if rnn == "lnlstm" else Mo.GRUCell(H, H)).cuda()
    with torch.no_grad():
        for name, p in cell.named_parameters():
            if "ln_" in name and name.endswith("weight"):
                p.add_(0.1 * torch.randn_like(p))
            elif "ln_" in name:
                p.copy_(0.1 * torch.randn_like(p))
    x = torch.randn(M, H, device="cuda")
    h = torch.randn(M, H, device="cuda") * 0.5
    c = torch.randn(M, H, device="cuda")
    P64 = {n: p.detach().double().requires_grad_() for n, p in cell.named_parameters()}
    x64, h64, c64 = x.double(), h.double(), c.double()
    if rnn == "lnlstm":
        hy, cy = cell(x, (h, c))
        rh, rc = _ref_lnlstm(x64 @ P64["weight_ih"].t(), h64 @ P64["weight_hh"].t(), c64, P64["ln_input.weight"],
                             P64["ln_input.bias"], P64["ln_hidden.weight"], P64["ln_hidden.bias"], P64["bias_ih"],
                             P64["ln_cell.weight"], P64["ln_cell.bias"])
        outs, routs = [hy, cy], [rh, rc]
    else:
        ref = torch.nn.GRUCell(H, H).cuda().double()
        with torch.no_grad():
            for n, p in ref.named_parameters():
                p.copy_(P64[n])
        P64 = dict(ref.named_parameters())
        outs, routs = [cell(x, h)], [ref(x64, h64)]
    for a, b in zip(outs, routs):
        assert (a.double() - b).abs().max() < 2e-5
    gs = [torch.randn_like(o) for o in outs]
    names = [n for n, _ in cell.named_parameters()]
    got = torch.autograd.grad(outs, list(cell.parameters()), gs)
    exp = torch.autograd.grad(routs, [P64[n] for n in names], [g.double() for g in gs])
    for n, a, b in zip(names, got, exp):
        assert _rel(a, b) < 2e-5, f"{n}: rel err {_rel(a, b)}"
