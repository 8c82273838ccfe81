#!/usr/bin/env python3
"""GEMM microbenchmark on the rollout's layer shapes: gm_gemm_f32 vs hipBLASLt fp32
(torch.nn.functional.linear), interleaved rounds in one process (cdna guide rule 24)."""
import importlib
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")

SHAPES = [  # name, M, N, K
    ("dqn.l1", 81920, 512, 642), ("dqn.l2", 81920, 256, 512), ("enc.l0", 81920, 512, 88),
    ("enc.l1", 81920, 256, 512), ("enc.l2", 81920, 128, 256), ("lstm", 81920, 512, 256),
]


if os.environ.get("SHAPES") == "train":  # the update's dense layers at 131072 rows (8 x 819 sequences x 20)
    SHAPES = [("dqn.l1", 131072, 512, 642), ("dqn.l2", 131072, 256, 512), ("enc.l1", 131072, 256, 512),
              ("enc.l2", 131072, 128, 256), ("lstm", 131072, 512, 256)]

if os.environ.get("ROWS"):  # e.g. one stream group of the rollout (40960 rows)
    SHAPES = [(nm, int(os.environ["ROWS"]), n, k) for nm, _, n, k in SHAPES]
TILES = [int(t) for t in os.environ.get("TILES", "-1").split(",") if t]
X3_TILES = [int(t) for t in os.environ.get("X3_TILES", "-1,1,2").split(",")]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    torch.manual_seed(0)
    out = {}
    for name, m, n, k in SHAPES:
        ldx = (k + 3) // 4 * 4
        buf = torch.randn(m, ldx, device="cuda")
        x = buf[:, :k]
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        wp, ldw = FU._pad_cols(w)
        y = torch.empty(m, n, device="cuda")
        xc = x.contiguous()

        x3 = FU.X3(wp, ldw, n, k)

        def mine():
            FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 1, y.data_ptr(), n)

        def mine3():
            FU.gemm(FU.dense(buf.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, b.data_ptr(), m, n, 1, y.data_ptr(), n,
                    x3=x3)

        def blas():
            F.linear(xc, w, b)

        lib = FU._setup()
        r = {f"tile{t}": [] for t in TILES}
        r.update({f"x3tile{t}": [] for t in X3_TILES})
        r["hipblaslt"] = []
        for _ in range(3):
            for t in TILES:
                lib.gm_gemm_set_tile(t)
                r[f"tile{t}"].append(timeit(mine))
            for t in X3_TILES:
                lib.gm_gemm_set_tile(t)
                r[f"x3tile{t}"].append(timeit(mine3))
            r["hipblaslt"].append(timeit(blas))
        lib.gm_gemm_set_tile(-1)
        fl = 2.0 * m * n * k
        out[name] = {k2: {"us": round(min(v), 1), "tflops": round(fl / (min(v) * 1e-6) / 1e12, 1)} for k2, v in r.items()}
        print(name, json.dumps(out[name]), flush=True)
    # DQN first layer as run in the rollout: A = [NetMon readout gathered per agent | env obs]
    B_, N_, A_, H_ = 4096, 20, 20, 128
    m = B_ * A_
    state = torch.randn(B_ * N_, 2 * H_, device="cuda")
    hprev = torch.randn(B_ * N_, 2 * H_, device="cuda")
    nbr = torch.randint(0, N_, (B_, N_, 3), device="cuda", dtype=torch.int32)
    agent_node = torch.randint(0, N_, (B_, A_), device="cuda", dtype=torch.int32)
    obs = torch.randn(B_, A_, 644, device="cuda")
    w = torch.randn(512, 642, device="cuda") / 642 ** 0.5
    b = torch.randn(512, device="cuda")
    wp, ldw = FU._pad_cols(w)
    y = torch.empty(m, 512, device="cuda")

    x3r = FU.X3(wp, ldw, 512, 642)

    def ro(x3=None):
        a0 = FU.readout(state.data_ptr(), 2 * H_, hprev.data_ptr(), 2 * H_, nbr, agent_node, N_, H_)
        FU.gemm(a0, FU.dense(obs.data_ptr(), 644, 130), wp.data_ptr(), ldw, b.data_ptr(), m, 512, 1, y.data_ptr(), 512,
                x3=x3)

    lib = FU._setup()
    r = {f"tile{t}": [] for t in TILES}
    r.update({f"x3tile{t}": [] for t in X3_TILES})
    for _ in range(3):
        for t in TILES:
            lib.gm_gemm_set_tile(t)
            r[f"tile{t}"].append(timeit(ro))
        for t in X3_TILES:
            lib.gm_gemm_set_tile(t)
            r[f"x3tile{t}"].append(timeit(lambda: ro(x3r)))
    lib.gm_gemm_set_tile(-1)
    fl = 2.0 * m * 512 * 642
    print("dqn.l1.readout", json.dumps({t: {"us": round(min(v), 1), "tflops": round(fl / (min(v) * 1e-6) / 1e12, 1)}
                                        for t, v in r.items()}), flush=True)
    # fused LSTM cell GEMM (dense [x|h] source, gate epilogue)
    M_ = importlib.import_module("graph-marl_amd.model")
    H, m = 128, 81920
    cell = M_.LSTMCell(H, H).cuda()
    x = torch.randn(m, H, device="cuda")
    st = torch.randn(m, 2 * H, device="cuda")
    wp, ldw, bp, _ = FU.pack_lstm(cell)
    x3l = FU.X3(wp, ldw, 4 * H, 2 * H)
    S = torch.empty(m, 2 * H, device="cuda")
    nbr = torch.randint(0, 20, (m // 20, 20, 3), device="cuda", dtype=torch.int32)

    def lstm_dense(x3=None):
        FU.gemm(FU.dense(x.data_ptr(), H, H), FU.dense(st.data_ptr(), 2 * H, H), wp.data_ptr(), ldw, bp.data_ptr(),
                m, 4 * H, FU.GM_EPI_LSTM, S.data_ptr(), 2 * H, S[:, H:].data_ptr(), 2 * H, st[:, H:].data_ptr(), 2 * H,
                x3=x3)

    def lstm_agg(x3=None):
        FU.gemm(FU.aggregate(st.data_ptr(), 2 * H, H, nbr, 20), FU.dense(st.data_ptr(), 2 * H, H), wp.data_ptr(),
                ldw, bp.data_ptr(), m, 4 * H, FU.GM_EPI_LSTM, S.data_ptr(), 2 * H, S[:, H:].data_ptr(), 2 * H,
                st[:, H:].data_ptr(), 2 * H, x3=x3)

    lib = FU._setup()
    for name, fn in (("lstm_fused", lstm_dense), ("lstm_agg_fused", lstm_agg)):
        r = {f"tile{t}": [] for t in TILES}
        r.update({f"x3tile{t}": [] for t in X3_TILES})
        for _ in range(3):
            for t in TILES:
                lib.gm_gemm_set_tile(t)
                r[f"tile{t}"].append(timeit(fn))
            for t in X3_TILES:
                lib.gm_gemm_set_tile(t)
                r[f"x3tile{t}"].append(timeit(lambda: fn(x3l)))
        lib.gm_gemm_set_tile(-1)
        fl = 2.0 * m * 4 * H * 2 * H
        print(name, json.dumps({t: {"us": round(min(v), 1), "tflops": round(fl / (min(v) * 1e-6) / 1e12, 1)}
                                for t, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
