#!/usr/bin/env python3
"""One GEMM shape in a loop (for rocprofv3 PMC passes): python tools/gemm_one.py [name] [form] [reps]
name in enc.l1 / dqn.l1 / lstm_agg; form x3 / f32."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")
M_ = importlib.import_module("graph-marl_amd.model")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "enc.l1"
    form = sys.argv[2] if len(sys.argv) > 2 else "x3"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    torch.manual_seed(0)
    FU._setup().gm_gemm_set_tile(int(os.environ.get("GM_TILE", "-1")))
    m = 81920
    if name == "lstm_agg":
        H = 128
        cell = M_.LSTMCell(H, H).cuda()
        st = torch.randn(m, 2 * H, device="cuda")
        wp, ldw, bp, _ = FU.pack_lstm(cell)
        x3 = FU.X3(wp, ldw, 4 * H, 2 * H) if form == "x3" else None
        S = torch.empty(m, 2 * H, device="cuda")
        nbr = torch.randint(0, 20, (m // 20, 20, 3), device="cuda", dtype=torch.int32)

        def fn():
            FU.gemm(FU.aggregate(st.data_ptr(), 2 * H, H, nbr, 20), FU.dense(st.data_ptr(), 2 * H, H),
                    wp.data_ptr(), ldw, bp.data_ptr(), m, 4 * H, FU.GM_EPI_LSTM, S.data_ptr(), 2 * H,
                    S[:, H:].data_ptr(), 2 * H, st[:, H:].data_ptr(), 2 * H, x3=x3)
    else:
        n, k = {"enc.l1": (256, 512), "dqn.l1": (512, 642), "enc.l2": (128, 256)}[name]
        ldx = (k + 3) // 4 * 4
        buf = torch.randn(m, ldx, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        wp, ldw = FU._pad_cols(w)
        x3 = FU.X3(wp, ldw, n, k) if form == "x3" else None
        y = torch.empty(m, n, device="cuda")

        def fn():
            FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 1, y.data_ptr(),
                    n, x3=x3)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
