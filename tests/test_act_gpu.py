"""Layer activations (--activation-function = any elementwise torch.nn.functional name with its defaults,
reference src/main.py:194-197, 440-441; MLP src/model.py:13-42) on the device: the forward kernels
(gm_act_fwd, the GEMM epilogues' fast forms), the backward from the layer output (gm_act_bwd) or from the
pre-activation (gm_act_bwd_z), and a Linear layer with each activation under grad and under no_grad,
all against torch's own functional and autograd in fp64."""
import importlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

M = importlib.import_module("graph-marl_amd.model")
L = importlib.import_module("graph-marl_amd._lib")
NAMES = sorted(M.ACTIVATIONS, key=M.ACTIVATIONS.get)


def z_values(n=4096 * 64, seed=0):
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(n, generator=g) * 4.0
    z[:64] = torch.tensor([-25., -20.5, -20., -6., -3.5, -3., -2.5, -1., -0.5, -1e-3, 0., 1e-3, 0.5, 1., 2.5, 3.,
                           3.5, 6., 6.5, 19.5, 20., 20.5, 25., -7., 7., -0.25, 0.25, -4., 4., -10., 10., 1e-6] * 2)
    return z.view(4096, 64)


@pytest.mark.parametrize("name", NAMES)
def test_act_forward_and_backward_kernels(name):
    act = M.ACTIVATIONS[name]
    z = z_values().cuda()
    fn = getattr(F, name)
    y = M.act_fwd(z, act)
    ref = fn(z.double())
    assert (y.double() - ref).abs().max().item() < 2e-6 * max(1.0, ref.abs().max().item() / 8), name
    # backward: from y (codes up to softplus) and from z (every code), vs torch autograd in fp64
    gy = torch.randn_like(z)
    zd = z.double().requires_grad_(True)
    fn(zd).backward(gy.double())
    want = zd.grad
    rows, cols = z.shape
    for use_z in ([False, True] if act not in M.Z_ACTS else [True]):
        g = torch.empty_like(z)
        part = torch.empty((rows + 63) // 64, cols, device="cuda")
        f = L.lib().gm_act_bwd_z if use_z else L.lib().gm_act_bwd
        src = z if use_z else M.act_fwd(z, act)
        L.check(f(gy.data_ptr(), src.data_ptr(), rows, cols, act, g.data_ptr(), part.data_ptr(), 64, None, None))
        torch.cuda.synchronize()
        err = (g.double() - want).abs()
        # a kink exactly at an input point: torch and the kernel may take either side; skip those
        kink = torch.zeros_like(z, dtype=torch.bool)
        for k in (0.0, -3.0, 3.0, 6.0, -1.0, 1.0, 20.0, -20.0):
            kink |= (z == k)
        assert err[~kink].max().item() < 1e-5 * max(1.0, want.abs().max().item()), (name, use_z)
        np.testing.assert_allclose(part.sum(0).cpu().numpy(), g.sum(0).cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", ["gelu", "silu", "mish", "softplus", "selu", "hardswish", "logsigmoid"])
@pytest.mark.parametrize("rows", [300, 8192])
def test_linear_with_activation_matches_torch(name, rows):
    """M.Linear with the activation: no_grad (the GEMM epilogue's form) and grad (Z_ACTS: pre-activation
    kept, gm_act_fwd + gm_act_bwd_z; the rest: gm_act_bwd from the output), both GEMM sizes (the
    register-staged and the split-f16 LDS-DMA forms), vs torch in fp64."""
    torch.manual_seed(1)
    lin = M.Linear(256, 128, act=M.act_code(name)).cuda()
    x = torch.randn(rows, 256, device="cuda")
    fn = getattr(F, name)
    w, b = lin.weight.detach().double(), lin.bias.detach().double()
    with torch.no_grad():
        y0 = lin(x)
    xd = x.double().requires_grad_(True)
    wd, bd = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = fn(xd @ wd.t() + bd)
    assert (y0.double() - ref.detach()).abs().max().item() < 1e-4
    xg = x.clone().requires_grad_(True)
    y = lin(xg)
    assert (y.double() - ref.detach()).abs().max().item() < 1e-4
    gy = torch.randn_like(y)
    y.backward(gy)
    ref.backward(gy.double())
    for got, want in ((xg.grad, xd.grad), (lin.weight.grad, wd.grad), (lin.bias.grad, bd.grad)):
        err = (got.double() - want).abs().max().item()
        assert err < 1e-4 * max(1.0, want.abs().max().item()), (name, rows, err)
