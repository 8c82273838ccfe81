"""Host-side pieces of the SL driver's sequence-batched loss (graph-marl_amd/sl.py): the per-step
MSE and the two-stage bias-gradient column sum against torch's own ops (no GPU)."""
import importlib

import torch


def test_step_mse_matches_per_step_mse_loss():
    SL = importlib.import_module("graph-marl_amd.sl")
    torch.manual_seed(0)
    for shape in ((3, 4, 5, 6), (2, 7, 3, 1), (1, 8, 8, 8)):
        pred = torch.randn(*shape, dtype=torch.float64, requires_grad=True)
        tgt = torch.randn(*shape[1:], dtype=torch.float64)
        per = SL._StepMSE.apply(pred, tgt)
        ref = torch.stack([torch.nn.functional.mse_loss(pred[t], tgt) for t in range(shape[0])])
        torch.testing.assert_close(per, ref)
        w = torch.randn(shape[0], dtype=torch.float64)
        g1, = torch.autograd.grad((per * w).sum(), pred)
        g2, = torch.autograd.grad((ref * w).sum(), pred)
        torch.testing.assert_close(g1, g2)


def test_colsum_two_stage():
    M = importlib.import_module("graph-marl_amd.model")
    torch.manual_seed(1)
    for rows in (1000, 65536, 70001):
        g = torch.randn(rows, 7, dtype=torch.float64)
        torch.testing.assert_close(M._colsum(g), g.sum(0))
