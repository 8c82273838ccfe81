#!/usr/bin/env python3
"""gm_gemm_x3_dgrad timing on the sequence-batched update's shapes: with / without the leaky mask
and the bias partials, and the plain scaled-A GEMM (gm_gemm_x3). python tools/dgrad_bench.py"""
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
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


m = int(os.environ.get("ROWS", "1040384"))
out = {}
SH = ((512, 256), (512, 512), (256, 128), (256, 512))
if os.environ.get("DSHAPES"):  # n:k,... (output columns : gradient columns; e.g. 512:100, config 5's head)
    SH = tuple(tuple(int(v) for v in x.split(":")) for x in os.environ["DSHAPES"].split(","))
for n, k in SH:
    g = torch.randn(m, k, device="cuda") * 1e-6
    w = torch.randn(k, n, device="cuda") / k ** 0.5
    mask = torch.randint(-2 ** 31, 2 ** 31 - 1, (m, (n + 31) // 32), dtype=torch.int32, device="cuda")  # sign words
    sc = torch.empty(1, device="cuda")
    L.check(FU._setup().gm_absmax_scale(g.data_ptr(), g.numel(), sc.data_ptr(), L.stream_ptr()))
    x3 = S._x3(w.t().contiguous())
    y = torch.empty(m, n, device="cuda")
    part = torch.empty((m + 127) // 128, n, device="cuda")
    gmax = torch.zeros(1, device="cuda")
    r = {}
    lib = FU._setup()
    import ctypes as C

    def raw(msk, ldm, prt, gm):  # one launch (no row blocks): ldm = 0 re-reads one mask row (cache hits)
        a = FU.dense(g.data_ptr(), k, k, scale=sc.data_ptr())
        L.check(lib.gm_gemm_x3_dgrad(C.byref(a), x3.wp.data_ptr(), x3.sinv.data_ptr(), m, n, n,
                                     None if msk is None else msk.data_ptr(), ldm, y.data_ptr(), n, None, 0,
                                     None if prt is None else prt.data_ptr(), None if gm is None else gm.data_ptr(),
                                     L.stream_ptr()))
    forms = [(int(f.split(":")[0]), int(f.split(":")[1])) for f in os.environ.get("FORMS", "0:1").split(",")]
    y0 = None
    for form, mf in forms:  # gm_gemm_set_dgrad form : gm_gemm_set_mfma shape
        L.check(lib.gm_gemm_set_dgrad(form))
        L.check(lib.gm_gemm_set_mfma(mf))
        tag = f"f{form}m{mf}:"
        for name, msk, ldm, prt, gm in (("mask+part+max", mask, (n + 31) // 32, part, gmax),
                                        ("part+max", None, 0, part, gmax), ("bare", None, 0, None, None)):
            us = min(timeit(lambda: raw(msk, ldm, prt, gm)) for _ in range(3))
            r[tag + name] = round(us, 1)
        r[tag + "tflops_bare"] = round(6.0 * m * n * k / (r[tag + "bare"] * 1e-6) / 1e12, 1)
        raw(mask, (n + 31) // 32, part, gmax)
        torch.cuda.synchronize()
        if y0 is None:
            y0 = y.clone()
        else:
            r[tag + "rel_vs_first"] = float((y - y0).abs().max() / y0.abs().max())
    lib.gm_gemm_set_dgrad(-1)
    lib.gm_gemm_set_mfma(2)
    out[f"{n}x{k}"] = r
    print(n, k, r, flush=True)
print(json.dumps(out))
