#!/usr/bin/env python3
"""NetMon encoder forms at the rollout's size (4096 graphs x 20 nodes, layers 88 -> 512 -> 256 -> 128,
leaky): the chained launch (gm_encoder_x3), the fold alone (layers 1 + 2, routing-encoder A source),
layer 3 alone, and layer 2 on a dense A (the layer-1 output read from HBM) for the A-source cost.
  python tools/chain_bench.py        (G=2048 for one stream group's launch)"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
FU = importlib.import_module("graph-marl_amd.fused")

B, N = int(os.environ.get("G", "4096")), 20
env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3)
env.reset()
torch.manual_seed(0)
nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
l0, l1, l2 = list(nm.encode.linear_layers)
x = env.node_obs.reshape(B * N, -1)
nbr = env.nbr
rows = B * N
y3 = torch.empty(rows, 128, device="cuda")
y2 = torch.empty(rows, 256, device="cuda")
y1 = torch.empty(rows, 512, device="cuda")
FU.routing_encoder(l0, x, nbr, B, N, y1)


def chain():
    FU.encoder_chain(l0, l1, l2, x, nbr, N, y3)


def fold():
    FU.gemm(FU.routing_enc_src(l0, x, nbr, N), None, None, 0, l1.bias.data_ptr(), rows, 256, FU._epi(l1.act),
            y2.data_ptr(), 256, x3=FU.pack_x3(l1))


def layer3():
    FU._linear(y2, 256, 256, l2, y3)


def dense2():
    FU._linear(y1, 512, 512, l1, y2)


def timeit(f, reps=20, rounds=5):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(rounds):
        s.record()
        for _ in range(reps):
            f()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e3)
    return best


res = {name: timeit(f) for name, f in (("chain", chain), ("fold", fold), ("layer3", layer3), ("dense2", dense2))}
mf = 3 * 2 * rows * (256 * 512 + 128 * 256) / 2516.8e12 * 1e6
print(f"rows {rows}: " + ", ".join(f"{k} {v:.1f} us" for k, v in res.items()) +
      f"; chain MFMA floor {mf:.1f} us (frac {mf / res['chain']:.3f})")
