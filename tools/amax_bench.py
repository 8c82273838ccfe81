"""Cost of the forward GEMM's max|x| publication (gm_gemm_x3 src0 amax): the same
linear_raw with and without the amax slot, HIP events on the current stream."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
M = importlib.import_module("graph-marl_amd.model")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


out = {}
for rows, k, n in ((131072, 642, 512), (131072, 512, 256), (131072, 256, 512)):
    x = torch.randn(rows, (k + 3) // 4 * 4, device="cuda")
    w = torch.randn(n, k, device="cuda") * 0.05
    wc = M._WeightCache()
    slot = torch.zeros(1, device="cuda")
    t0 = timeit(lambda: M.linear_raw(x, x.stride(0), k, w, None, 1, wcache=wc))
    t1 = timeit(lambda: M.linear_raw(x, x.stride(0), k, w, None, 1, wcache=wc, amax=slot.zero_()))
    out[f"{rows}x{n}x{k}"] = {"plain_us": round(t0, 1), "amax_us": round(t1, 1)}
print(json.dumps(out))
