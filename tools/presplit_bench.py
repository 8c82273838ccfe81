#!/usr/bin/env python3
"""DQN layer 1 as run in the rollout (readout-gathered A, 81920 x 512 x 640) timed on operands whose
fp32 words are also two valid random f16 values, so that a diagnostic build reading A as pre-split
f16 pairs (GM_LIB=.../diag11) multiplies realistic data. Prints one JSON line (min over 3 x 20)."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")


def f16pairs(*shape):
    """fp32 tensor whose words are pairs of random f16 values of magnitude O(1)."""
    n = 1
    for s in shape:
        n *= s
    return (torch.randn(2 * n, device="cuda") * 0.5).half().view(torch.float32).view(*shape)


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
    B_, N_, A_, H_ = 4096, 20, 20, 128
    m = B_ * A_
    state, hprev = f16pairs(B_ * N_, 2 * H_), f16pairs(B_ * N_, 2 * H_)
    nbr = torch.randint(0, N_, (B_, N_, 3), device="cuda", dtype=torch.int32)
    agent_node = torch.randint(0, N_, (B_, A_), device="cuda", dtype=torch.int32)
    obs = f16pairs(B_, A_, 128)
    w = torch.randn(512, 640, device="cuda") / 640 ** 0.5
    b = torch.randn(512, device="cuda")
    wp, ldw = FU._pad_cols(w)
    y = torch.empty(m, 512, device="cuda")
    x3 = FU.X3(wp, ldw, 512, 640)

    def ro():
        a0 = FU.readout(state.data_ptr(), 2 * H_, hprev.data_ptr(), 2 * H_, nbr, agent_node, N_, H_)
        FU.gemm(a0, FU.dense(obs.data_ptr(), 128, 128), wp.data_ptr(), ldw, b.data_ptr(), m, 512, 1, y.data_ptr(), 512,
                x3=x3)

    if os.environ.get("TILE"):  # tile override (gm_gemm_set_tile), e.g. 9 = 3-stage 128x256
        FU._setup().gm_gemm_set_tile(int(os.environ["TILE"]))
    for _ in range(10):  # ~2 s of back-to-back launches before timing (clock settles)
        timeit(ro, 20)
    us = min(timeit(ro) for _ in range(3))
    print(json.dumps({"lib": os.environ.get("GM_LIB", "default"), "tile": os.environ.get("TILE", "-1"), "dqn_l1_us": round(us, 1),
                      "tflops_f16": round(3 * 2.0 * m * 512 * 640 / (us * 1e-6) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
