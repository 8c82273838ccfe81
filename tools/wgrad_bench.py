#!/usr/bin/env python3
"""Weight-gradient GEMM timing on the training shapes (131072 batch rows): split-f16 K-major
kernel (model._wgrad) vs the library fp32 GEMM. python tools/wgrad_bench.py"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
M = importlib.import_module("graph-marl_amd.model")


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    torch.manual_seed(0)
    Mb = int(os.environ.get("ROWS", "262160"))
    lib = M.L.lib()
    out = {}
    for o, k, ldx in ((512, 642, 644), (512, 512, 512), (256, 512, 512), (512, 256, 256), (128, 256, 256),
                      (512, 128, 128), (512, 88, 88)):
        gy = torch.randn(Mb, o, device="cuda") * 1e-6
        x = torch.randn(Mb, ldx, device="cuda")[:, :k]
        r = {}
        sa = M._gy_scale(gy)
        sb = torch.empty(1, device="cuda")
        M.L.check(lib.gm_absmax_scale_rows(x.data_ptr(), Mb, k, ldx, sb.data_ptr(), M.L.stream_ptr()))
        flop = 6.0 * Mb * o * k
        res = {}
        for form, name in ((9, "tr128_noxcd"), (1, "tr128"), (3, "tr128_mfma16"), (2, "tr256")):
            lib.gm_gemm_set_wgrad(form)
            us = timeit(lambda: M._wgrad(gy, x, k, sa, sb))
            r[name + "_us"] = round(us, 1)
            r[name + "_TF"] = round(flop / us / 1e6, 1)
            res[name] = M._wgrad(gy, x, k, sa, sb)
        r["xcd_bitwise_equal"] = bool(torch.equal(res["tr128"], res["tr128_noxcd"]))
        lib.gm_gemm_set_wgrad(-1)
        lib.gm_gemm_set_wgrad(1)
        g1 = M._wgrad(gy, x, k)
        lib.gm_gemm_set_wgrad(3)
        g3 = M._wgrad(gy, x, k)
        lib.gm_gemm_set_wgrad(-1)
        r["rel_16_vs_32"] = float((g3 - g1).abs().max() / g1.abs().max())
        print(o, k, r, flush=True)
        out[f"{o}x{k}"] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
