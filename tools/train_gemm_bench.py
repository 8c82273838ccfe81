#!/usr/bin/env python3
"""Training-operand GEMMs (forward publishing max|A|, input gradient on a power-of-two scaled A,
LSTM gate epilogue publishing max|[x | h]|) at update batch sizes: k_gemm3 (gm_gemm_set_tile(0))
vs the LDS-DMA kernel k_gemm3g (tiles 12, 13). Checks that every form gives the same outputs and
the same published max as k_gemm3. python tools/train_gemm_bench.py"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")
MD = importlib.import_module("graph-marl_amd.model")

M = int(os.environ.get("ROWS", "262160"))
# name, N, K, kind: fwd = bias+leaky with amax, dgrad = no bias with a scaled A, lstm = gate epilogue
SHAPES = [("fwd.dqn1", 256, 512, "fwd"), ("fwd.enc2", 128, 256, "fwd"), ("fwd.dqn0", 512, 642, "fwd"),
          ("dgrad.dqn1", 512, 256, "dgrad"), ("dgrad.enc2", 256, 128, "dgrad"), ("dgrad.lstm", 256, 512, "dgrad"),
          ("dgrad.dqn0", 512, 512, "dgrad"), ("lstm", 512, 256, "lstm")]
if os.environ.get("SHAPES"):  # name:N:K:kind,... (e.g. fwd.slhead:100:512:fwd, config 5's output head)
    SHAPES = [(f[0], int(f[1]), int(f[2]), f[3]) for f in (x.split(":") for x in os.environ["SHAPES"].split(","))]


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
    lib = FU._setup()
    out = {}
    tiles = [int(t) for t in os.environ.get("TILES", "0,12,13").split(",")]
    for name, n, k, kind in SHAPES:
        ldx = (k + 3) // 4 * 4
        buf = torch.randn(M, ldx, device="cuda")
        if kind == "dgrad":
            buf *= 1e-5
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        slot = torch.zeros(1, device="cuda")
        sc = torch.empty(1, device="cuda")
        if kind == "dgrad":
            MD.L.check(lib.gm_absmax_scale(buf.data_ptr(), buf.numel(), sc.data_ptr(), MD.L.stream_ptr()))
        if kind == "lstm":
            cell = MD.LSTMCell(k // 2, n // 4).cuda()
            wp, ldw, bp, x3 = FU.pack_lstm(cell)
            H = n // 4
            h1 = torch.empty(M, H, device="cuda")
            c1 = torch.empty(M, H, device="cuda")
            c0 = torch.randn(M, H, device="cuda")
            act = torch.empty(M, n, device="cuda")

            def run():
                slot.zero_()
                FU.gemm(FU.dense(buf.data_ptr(), ldx, k, amax=slot.data_ptr()), None, wp.data_ptr(), ldw,
                        bp.data_ptr(), M, n, FU.GM_EPI_LSTM, h1.data_ptr(), H, c1.data_ptr(), H, c0.data_ptr(), H,
                        act.data_ptr(), x3=x3)

            outs = lambda: (h1.clone(), c1.clone(), act.clone(), slot.clone())
        else:
            wp, ldw = FU._pad_cols(w)
            x3 = FU.X3(wp, ldw, n, k)
            y = torch.empty(M, n, device="cuda")
            if kind == "fwd":
                def run():
                    slot.zero_()
                    FU.gemm(FU.dense(buf.data_ptr(), ldx, k, amax=slot.data_ptr()), None, wp.data_ptr(), ldw,
                            b.data_ptr(), M, n, 1, y.data_ptr(), n, x3=x3)
            else:
                def run():
                    FU.gemm(FU.dense(buf.data_ptr(), ldx, k, scale=sc.data_ptr()), None, wp.data_ptr(), ldw, None, M,
                            n, 0, y.data_ptr(), n, x3=x3)
            outs = lambda: (y.clone(), slot.clone())
        r = {}
        ref = None
        for t in tiles:
            lib.gm_gemm_set_tile(t)
            run()
            torch.cuda.synchronize()
            o = outs()
            if ref is None:
                ref = o
            else:
                r[f"t{t}_maxdiff"] = max(float((a - b_).abs().max()) for a, b_ in zip(o, ref))
        times = {t: [] for t in tiles}
        for _ in range(3):
            for t in tiles:
                lib.gm_gemm_set_tile(t)
                times[t].append(timeit(run))
        lib.gm_gemm_set_tile(-1)
        fl = 3 * 2.0 * M * n * k
        for t in tiles:
            us = min(times[t])
            r[f"t{t}_us"] = round(us, 1)
            r[f"t{t}_tf"] = round(fl / (us * 1e-6) / 1e12, 1)
        out[name] = r
        print(name, json.dumps(r), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
