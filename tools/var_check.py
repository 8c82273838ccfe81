#!/usr/bin/env python3
"""Outputs of the rollout GEMM forms for one library build (GM_LIB) on fixed seeded inputs, recorded as
SHA-256 digests in gpurun_out/varcheck_<tag>.json; `var_check.py --compare a b` asserts two builds agree
bit for bit (a k-loop schedule change must not change any output bit)."""
import hashlib
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(tag):
    FU = importlib.import_module("graph-marl_amd.fused")
    M = importlib.import_module("graph-marl_amd.model")
    torch.manual_seed(0)
    out = {}
    B_, N_, A_, H_ = 1024, 20, 20, 128
    m = B_ * A_
    state, hprev = torch.randn(B_ * N_, 2 * H_, device="cuda"), torch.randn(B_ * N_, 2 * H_, device="cuda")
    nbr = torch.randint(0, N_, (B_, N_, 3), device="cuda", dtype=torch.int32)
    agent_node = torch.randint(0, N_, (B_, A_), device="cuda", dtype=torch.int32)
    obs = torch.randn(B_, A_, 128, device="cuda")
    w = torch.randn(512, 640, device="cuda") / 640 ** 0.5
    b = torch.randn(512, device="cuda")
    wp, ldw = FU._pad_cols(w)
    y = torch.empty(m, 512, device="cuda")
    x3 = FU.X3(wp, ldw, 512, 640)
    a0 = FU.readout(state.data_ptr(), 2 * H_, hprev.data_ptr(), 2 * H_, nbr, agent_node, N_, H_)
    FU.gemm(a0, FU.dense(obs.data_ptr(), 128, 128), wp.data_ptr(), ldw, b.data_ptr(), m, 512, 1, y.data_ptr(), 512, x3=x3)
    out["readout_l1"] = y.cpu().numpy()
    for name, mm, n, k in (("dense_256x512", 40960, 256, 512), ("dense_128x256", 40960, 128, 256),
                           ("dense_512x88", 4096, 512, 88)):
        x = torch.randn(mm, k, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        wp, ldw = FU._pad_cols(w)
        y = torch.empty(mm, n, device="cuda")
        FU.gemm(FU.dense(x.data_ptr(), k, k), None, wp.data_ptr(), ldw, b.data_ptr(), mm, n, 1, y.data_ptr(), n,
                x3=FU.X3(wp, ldw, n, k))
        out[name] = y.cpu().numpy()
    # LSTM cells ([x | h] two sources, gate epilogue) on the LDS-DMA and the register-staged forms
    for rows in (40960, 2048):
        cell = M.LSTMCell(H_, H_).cuda()
        x, h, c = (torch.randn(rows, H_, device="cuda") for _ in range(3))
        with torch.no_grad():
            h1, c1 = cell(x, (h, c))
        out[f"lstm_{rows}_h"], out[f"lstm_{rows}_c"] = h1.cpu().numpy(), c1.cpu().numpy()
    torch.cuda.synchronize()
    os.makedirs("gpurun_out", exist_ok=True)
    dig = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()[:24] for k, v in out.items()}
    with open(f"gpurun_out/varcheck_{tag}.json", "w") as f:
        json.dump(dig, f)
    print("varcheck", tag, {k: float(np.abs(v).sum()) for k, v in out.items()}, flush=True)


def compare(a, b):
    with open(f"gpurun_out/varcheck_{a}.json") as f:
        A = json.load(f)
    with open(f"gpurun_out/varcheck_{b}.json") as f:
        B = json.load(f)
    bad = [k for k in A if A[k] != B.get(k)]
    print("varcheck compare", a, b, "identical" if not bad else f"DIFFERENT {bad}", flush=True)
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        ok = all(compare(sys.argv[2], t) for t in sys.argv[3:])
        sys.exit(0 if ok else 1)
    run(sys.argv[1])
