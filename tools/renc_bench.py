#!/usr/bin/env python3
"""gm_routing_node_encoder timing at the rollout's size (4096 graphs x 20 nodes -> 512 columns, leaky,
sign bits): python tools/renc_bench.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
FU = importlib.import_module("graph-marl_amd.fused")
TS = importlib.import_module("graph-marl_amd.train_seq")

B, N = int(os.environ.get("G", "4096")), 20
env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3)
env.reset()
lin = M.Linear(4 * N + 8, 512, act=1).cuda()
x = env.node_obs.reshape(-1, 4 * N + 8)
y = torch.empty(B * N, 512, device="cuda")
bits = TS._sign_bits(B * N, 512, "cuda") if os.environ.get("BITS", "1") == "1" else None


def run():
    FU.routing_encoder(lin, x, env.nbr, B, N, y, sbits=bits)


run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(5):
    s.record()
    for _ in range(20):
        run()
    e.record()
    torch.cuda.synchronize()
    best = min(best, s.elapsed_time(e) / 20 * 1e3)
print(f"routing encoder {B * N} rows: {best:.1f} us, {y.numel() * 4 / best / 1e3:.2f} TB/s of output")
