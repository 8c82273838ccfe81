#!/usr/bin/env python3
"""Fixed vs per-k cost of the input-gradient GEMM (gm_gemm_x3_dgrad, no mask / partials) at the training
update's row count: time over K at N = 512, next to a plain 4.3 GB write (torch fill) and copy, to split a
launch into its k loop and its prologue + epilogue. python tools/gemm_k_sweep.py  (ROWS, KS, N env)"""
import ctypes as C
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")
S = importlib.import_module("graph-marl_amd.train_seq")
L = importlib.import_module("graph-marl_amd._lib")


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e3)
    return best


m = int(os.environ.get("ROWS", "2097152"))
n = int(os.environ.get("N", "512"))
lib = FU._setup()
out = {"rows": m, "n": n, "lib": os.environ.get("GM_LIB", "default")}
y = torch.empty(m, n, device="cuda")
out["fill_us"] = round(timeit(lambda: y.fill_(1.0)), 1)
y2 = torch.empty_like(y)
out["copy_us"] = round(timeit(lambda: y2.copy_(y)), 1)
del y2
for k in [int(v) for v in os.environ.get("KS", "32,64,128,256,512").split(",")]:
    g = torch.randn(m, k, device="cuda") * 1e-3
    w = torch.randn(k, n, device="cuda") / k ** 0.5
    x3 = S._x3(w.t().contiguous())
    a = FU.dense(g.data_ptr(), k, k)

    def run():
        L.check(lib.gm_gemm_x3_dgrad(C.byref(a), x3.wp.data_ptr(), x3.sinv.data_ptr(), m, n, n, None, 0, y.data_ptr(), n,
                                     None, 0, None, None, L.stream_ptr()))
    out[f"k{k}_us"] = round(timeit(run), 1)
    out[f"k{k}_sum"] = float(y.double().sum())  # the same bits across library builds
    del g
print(json.dumps(out), flush=True)
