#!/usr/bin/env python3
"""Per-k-tile error map of one k_gemm3g tile form: A nonzero in one 32-deep k tile only.
python tools/tile_diag2.py tile mfma K"""
import importlib
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")

tile, mf, K = (int(a) for a in sys.argv[1:4])
lib = FU._setup()
lib.gm_gemm_set_tile(tile)
FU.L.check(lib.gm_gemm_set_mfma(mf))
m, n = 8192, 512
torch.manual_seed(0)
w = torch.randn(n, K, device="cuda") / K ** 0.5
b = torch.zeros(n, device="cuda")
wp, ldw = FU._pad_cols(w)
x3 = FU.X3(wp, ldw, n, K)
for t in range((K + 31) // 32):
    for part in ("full", "hi_only"):
        x = torch.zeros(m, K, device="cuda")
        x[:, 32 * t:32 * t + 32] = torch.randn(m, min(32, K - 32 * t), device="cuda")
        if part == "hi_only":  # values exact in f16: a_lo = 0, only a_hi terms
            x = x.half().float()
        y = torch.empty(m, n, device="cuda")
        FU.gemm(FU.dense(x.data_ptr(), K, K), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 0, y.data_ptr(), n, x3=x3)
        torch.cuda.synchronize()
        ref = F.linear(x.double(), w.double())
        err = (y.double() - ref).abs()
        bad = err > 2e-5
        cb = bad.view(m, n // 32, 32).any(2).any(0).nonzero().flatten().tolist()
        rb = bad.view(m // 32, 32, n).any(2).any(1).view(-1, 4).any(0).nonzero().flatten().tolist()
        print(f"tile={tile} mf={mf} K={K} ktile={t} {part}: max_err={err.max().item():.2e} bad={int(bad.sum())} "
              f"bad 32-col blocks={cb} bad 32-row blocks (mod 4)={rb}", flush=True)
