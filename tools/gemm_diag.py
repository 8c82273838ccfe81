#!/usr/bin/env python3
"""x3 GEMM timings on the rollout shapes for the library named by GM_LIB (diagnostic
builds: csrc GM_DIAG=1/2/3) over the x3 tile table. Prints one JSON line per shape."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")
M_ = importlib.import_module("graph-marl_amd.model")
TILES = [int(t) for t in os.environ.get("X3_TILES", "-1,1,2,3").split(",")]


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
    m = 81920
    shapes = []
    for name, n, k in (("enc.l1", 256, 512), ("dqn.l1.dense", 512, 642), ("enc.l2", 128, 256)):
        ldx = (k + 3) // 4 * 4
        buf = torch.randn(m, ldx, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        wp, ldw = FU._pad_cols(w)
        x3 = FU.X3(wp, ldw, n, k)
        y = torch.empty(m, n, device="cuda")
        shapes.append((name, 2.0 * m * n * k, lambda buf=buf, ldx=ldx, k=k, wp=wp, ldw=ldw, b=b, n=n, y=y, x3=x3:
                       FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 1,
                               y.data_ptr(), n, x3=x3)))
    H = 128
    cell = M_.LSTMCell(H, H).cuda()
    st = torch.randn(m, 2 * H, device="cuda")
    x = torch.randn(m, H, device="cuda")
    wp, ldw, bp, _ = FU.pack_lstm(cell)
    x3l = FU.X3(wp, ldw, 4 * H, 2 * H)
    S = torch.empty(m, 2 * H, device="cuda")
    nbr = torch.randint(0, 20, (m // 20, 20, 3), device="cuda", dtype=torch.int32)
    shapes.append(("lstm", 2.0 * m * 512 * 256, lambda: FU.gemm(
        FU.dense(x.data_ptr(), H, H), FU.dense(st.data_ptr(), 2 * H, H), wp.data_ptr(), ldw, bp.data_ptr(), m, 4 * H,
        FU.GM_EPI_LSTM, S.data_ptr(), 2 * H, S[:, H:].data_ptr(), 2 * H, st[:, H:].data_ptr(), 2 * H, x3=x3l)))
    shapes.append(("lstm_agg", 2.0 * m * 512 * 256, lambda: FU.gemm(
        FU.aggregate(st.data_ptr(), 2 * H, H, nbr, 20), FU.dense(st.data_ptr(), 2 * H, H), wp.data_ptr(), ldw,
        bp.data_ptr(), m, 4 * H, FU.GM_EPI_LSTM, S.data_ptr(), 2 * H, S[:, H:].data_ptr(), 2 * H,
        st[:, H:].data_ptr(), 2 * H, x3=x3l)))
    for name, fl, fn in shapes:
        r = {}
        for t in TILES:
            lib.gm_gemm_set_tile(t)
            us = min(timeit(fn) for _ in range(3))
            r[f"t{t}"] = {"us": round(us, 1), "tf32eq": round(fl / us / 1e6, 1)}
        lib.gm_gemm_set_tile(-1)
        print(os.environ.get("GM_LIB", "default"), name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
