#!/usr/bin/env python3
"""Debug of the routing-encoder fold (GM_A_ROUTING_ENC): layer-2 output of the fold vs the two-kernel path."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
FU = importlib.import_module("graph-marl_amd.fused")
for N, B in ((20, 64), (20, 4096), (10, 64)):
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3,
                     agent_adjacency=False)
    env.reset_()
    torch.manual_seed(N)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    l0, l1 = list(nm.encode.linear_layers)[:2]
    x = env.node_obs.reshape(B * N, -1)
    gm._lib.range_status(clear=True)
    y_fold = torch.full((B * N, 256), float("nan"), device="cuda")
    FU.gemm(FU.routing_enc_src(l0, x, env.nbr, N), None, None, 0, l1.bias.data_ptr(), B * N, 256, FU._epi(l1.act),
            y_fold.data_ptr(), 256, x3=FU.pack_x3(l1))
    torch.cuda.synchronize()
    flag = gm._lib.range_status(clear=True)
    h1 = FU.routing_encoder(l0, x, env.nbr, B, N, torch.empty(B * N, 512, device="cuda"))
    y_two = FU._linear(h1, h1.stride(0), 512, l1, torch.empty(B * N, 256, device="cuda"))
    d = (y_fold - y_two).abs()
    bad = ~torch.isfinite(y_fold) | (d > 1e-5)
    print(f"N={N} B={B} range_flag={flag} bad={int(bad.sum())}/{bad.numel()} maxdiff={d[torch.isfinite(d)].max().item() if torch.isfinite(d).any() else None}")
    if bad.any():
        rows = bad.any(1).nonzero().flatten()
        cols = bad.any(0).nonzero().flatten()
        print("  bad rows", rows[:20].tolist(), "n", len(rows), "rows%128 hist", torch.bincount(rows % 128, minlength=128)[:16].tolist())
        print("  bad cols", cols[:20].tolist(), "n", len(cols))
        r = int(rows[0])
        print("  row", r, "fold", y_fold[r, :8].tolist(), "two", y_two[r, :8].tolist())
