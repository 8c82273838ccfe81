#!/usr/bin/env python3
"""DQN layer 2 + fused Q head (gm_gemm_x3_head, 81920 x 256 x 512 + 4 heads) per tile form: default
(128 x 128 blocks, 2 per CU, partial Q per column block onto a zeroed q), tile 10 (128 x 256, 1 block / CU);
Q and hidden output compared with the default form; against the same GEMM with a plain bias + act store
(gm_gemm_x3) and the q zeroing alone. python tools/head_bench.py"""
import ctypes as C
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")


def timeit(fn, reps=20):
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
    lib = FU._setup()
    m, k, n, nq = int(os.environ.get("ROWS", "81920")), 512, 256, 4
    x = torch.randn(m, k, device="cuda").abs() * 0.5
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda") * 0.1
    wq = torch.randn(nq, n, device="cuda") / n ** 0.5
    bq = torch.randn(nq, device="cuda")
    wp, ldw = FU._pad_cols(w)
    x3 = FU.X3(wp, ldw, n, k)
    q = torch.empty(m, nq, device="cuda")
    y = torch.empty(m, n, device="cuda")
    out = {}
    for with_y in (False, True):
        def run():
            FU.L.check(lib.gm_gemm_x3_head(C.byref(FU.dense(x.data_ptr(), k, k)), x3.wp.data_ptr(), x3.sinv.data_ptr(),
                                           b.data_ptr(), m, n, 1, wq.data_ptr(), n, bq.data_ptr(), nq, q.data_ptr(), nq,
                                           y.data_ptr() if with_y else None, n, FU.L.stream_ptr()))
        ref = None
        r = {}
        for t in (-1, 10):
            lib.gm_gemm_set_tile(t)
            run()
            torch.cuda.synchronize()
            o = (q.clone(), y.clone() if with_y else None)
            if ref is None:
                ref = o
            else:
                r[f"t{t}_qdiff"] = float((o[0] - ref[0]).abs().max())
                if with_y:
                    r[f"t{t}_ydiff"] = float((o[1] - ref[1]).abs().max())
        ts = {t: [] for t in (-1, 10)}
        for _ in range(3):
            for t in ts:
                lib.gm_gemm_set_tile(t)
                ts[t].append(timeit(run))
        lib.gm_gemm_set_tile(-1)
        r.update({f"t{t}_us": round(min(v), 1) for t, v in ts.items()})
        out["with_y" if with_y else "q_only"] = r
    x3b = FU.X3(wp, ldw, n, k)
    out["plain_gemm_us"] = round(min(timeit(lambda: FU.gemm(FU.dense(x.data_ptr(), k, k), None, wp.data_ptr(), ldw,
                                                                 b.data_ptr(), m, n, 1, y.data_ptr(), n, x3=x3b))
                                     for _ in range(3)), 1)
    out["q_zero_us"] = round(min(timeit(lambda: q.zero_()) for _ in range(3)), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
