#!/usr/bin/env python3
"""Where a k step of the LDS-DMA GEMM spends its cycles (diagnostic build 30: s_memtime stamps by waves
0 and 4 of every block = the two waves of one SIMD, k steps 4..11). GM_LIB=graph-marl_amd/lib/vstamp/...
Segments: 0-1 fragment read + first-half MFMAs (incl. the A split), 1-2 the DMA wait, 2-3 lgkmcnt +
barrier, 3-4 DMA issue, 4-5 zero tail + next reads, 5-6 second-half MFMAs. Median cycles per segment."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FU = importlib.import_module("graph-marl_amd.fused")
L = importlib.import_module("graph-marl_amd._lib")


def main():
    lib = L.lib()
    buf = torch.zeros(4096 * 2 * 64, dtype=torch.int64, device="cuda")
    lib.gm_diag_stamps.argtypes = [ctypes.c_void_p]
    assert lib.gm_diag_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    torch.manual_seed(0)
    B_, N_, A_, H_ = 4096, 20, 20, 128
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
    xd = torch.randn(m, 512, device="cuda")
    w2 = torch.randn(256, 512, device="cuda") / 512 ** 0.5
    wp2, ldw2 = FU._pad_cols(w2)
    x32 = FU.X3(wp2, ldw2, 256, 512)
    y2 = torch.empty(m, 256, device="cuda")
    shapes = {
        "dqn_l1_readout": lambda: FU.gemm(FU.readout(state.data_ptr(), 2 * H_, hprev.data_ptr(), 2 * H_, nbr, agent_node,
                                                     N_, H_), FU.dense(obs.data_ptr(), 128, 128), wp.data_ptr(), ldw,
                                          b.data_ptr(), m, 512, 1, y.data_ptr(), 512, x3=x3),
        "enc_l1_dense_256x512": lambda: FU.gemm(FU.dense(xd.data_ptr(), 512, 512), None, wp2.data_ptr(), ldw2,
                                                b.data_ptr(), m, 256, 1, y2.data_ptr(), 256, x3=x32),
    }
    for name, fn in shapes.items():
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        buf.zero_()
        fn()
        torch.cuda.synchronize()
        st = buf.view(4096, 2, 8, 8).cpu().numpy().astype(np.int64)
        ok = st[:, :, :, 0] > 0
        out = {}
        for wv in range(2):
            segs = []
            for a, bb in ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (0, 6)):
                d = (st[:, wv, :, bb] - st[:, wv, :, a])[ok[:, wv, :] & (st[:, wv, :, bb] > 0)]
                segs.append(int(np.median(d)) if d.size else None)
            out[f"wave{4 * wv}"] = dict(zip(["read+mfma0", "dma_wait", "barrier", "dma_issue", "reads", "mfma1",
                                             "step"], segs))
        print(json.dumps({"shape": name, **out}), flush=True)


if __name__ == "__main__":
    main()
