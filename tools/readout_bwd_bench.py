#!/usr/bin/env python3
"""gm_netmon_readout_bwd timing at the sequence-batched update's size (G graphs of N nodes, R agents,
H = 128): python tools/readout_bwd_bench.py."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = importlib.import_module("graph-marl_amd._lib")

G, N, R, H, deg = int(os.environ.get("G", "104864")), 20, 20, 128, 3
torch.manual_seed(0)
dout = torch.randn(G * R, 4 * H, device="cuda")
nbr = torch.randint(-1, N, (G, N, deg), dtype=torch.int32, device="cuda")
an = torch.randint(0, N, (G, R), dtype=torch.int32, device="cuda")
dhf = torch.empty(G * N, H, device="cuda")
dhp = torch.empty(G * N, H, device="cuda")
lib = L.lib()


def run():
    L.check(lib.gm_netmon_readout_bwd(dout.data_ptr(), 4 * H, nbr.data_ptr(), an.data_ptr(), G, N, R, deg, H,
                                      dhf.data_ptr(), dhp.data_ptr(), L.stream_ptr()))


run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(3):
    s.record()
    for _ in range(5):
        run()
    e.record()
    torch.cuda.synchronize()
    best = min(best, s.elapsed_time(e) / 5 * 1e3)
gb = (dout.numel() + dhf.numel() + dhp.numel()) * 4 / 1e9
print(f"cs: {best:.1f} us, {gb / best * 1e6 / 1e3:.2f} TB/s "
      f"checksum {dhf.double().sum().item():.6e} {dhp.double().sum().item():.6e}")
