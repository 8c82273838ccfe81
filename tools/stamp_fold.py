#!/usr/bin/env python3
"""Where a k step of the fold (routing-encoder A source, NetMon encoder layer 2 at 81 920 x 256 x 512) and of
the readout-source DQN layer 1 (tile 9) goes in the ping-pong loop (diagnostic build 30: s_memtime stamps of waves 0
(early) and 4 (late) of every block, one SIMD, k steps 4..11):
  GM_LIB=graph-marl_amd/lib/vstamp/libgraphmarl_amd.so python tools/stamp_fold.py
Stamp points of a step: 0 after the barrier, 1 after the late wave's MFMAs of the previous tile, 2 after the
issue (DMA; fold: + the A tile computed), 3 after the fragment reads (+ split), 4 after the early wave's
MFMAs. Segments per wave, median cycles: late_mfma 0-1, issue 1-2, reads 2-3, early_mfma 3-4, to_next_barrier
(4 -> next step's 0: the wait at the barrier), step (0 -> next 0)."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
FU = importlib.import_module("graph-marl_amd.fused")
L = importlib.import_module("graph-marl_amd._lib")


def main():
    lib = L.lib()
    buf = torch.zeros(4096 * 2 * 64, dtype=torch.int64, device="cuda")
    lib.gm_diag_stamps.argtypes = [ctypes.c_void_p]
    assert lib.gm_diag_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    B, N = 4096, 20
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), 20, n_env=B, seed=3)
    env.reset()
    torch.manual_seed(0)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    l0, l1, l2 = list(nm.encode.linear_layers)
    x = env.node_obs.reshape(B * N, -1)
    rows = B * N
    y2 = torch.empty(rows, 256, device="cuda")
    y3 = torch.empty(rows, 128, device="cuda")
    # DQN layer 1 on its READOUT source (as tools/stamp_bench.py): 4096 graphs x 20 agents, K = 512 + 128
    state, hprev = torch.randn(rows, 256, device="cuda"), torch.randn(rows, 256, device="cuda")
    nbr = torch.randint(0, N, (B, N, 3), device="cuda", dtype=torch.int32)
    agent_node = torch.randint(0, N, (B, 20), device="cuda", dtype=torch.int32)
    obs = torch.randn(B, 20, 128, device="cuda")
    w = torch.randn(512, 640, device="cuda") / 640 ** 0.5
    b = torch.randn(512, device="cuda")
    wp, ldw = FU._pad_cols(w)
    y = torch.empty(rows, 512, device="cuda")
    shapes = {
        "fold_81920x256x512": lambda: FU.gemm(FU.routing_enc_src(l0, x, env.nbr, N), None, None, 0, l1.bias.data_ptr(),
                                              rows, 256, FU._epi(l1.act), y2.data_ptr(), 256, x3=FU.pack_x3(l1)),
        "chain": lambda: FU.encoder_chain(l0, l1, l2, x, env.nbr, N, y3),
        "dqn_l1_readout_81920x512x640": lambda: FU.gemm(
            FU.readout(state.data_ptr(), 256, hprev.data_ptr(), 256, nbr, agent_node, N, 128),
            FU.dense(obs.data_ptr(), 128, 128), wp.data_ptr(), ldw, b.data_ptr(), rows, 512, 1, y.data_ptr(), 512,
            x3=FU.X3(wp, ldw, 512, 640)),
    }
    for name, fn in shapes.items():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        buf.zero_()
        fn()
        torch.cuda.synchronize()
        st = buf.view(4096, 2, 8, 8).cpu().numpy().astype(np.int64)  # block, wave (0 early / 1 late), step, point
        out = {}
        for wv, tag in ((0, "early"), (1, "late")):
            s = st[:, wv]
            ok = (s[:, :-1, 0] > 0) & (s[:, 1:, 0] > 0)
            segs = {}
            for nm_, (p0, p1) in {"late_mfma": (0, 1), "issue": (1, 2), "reads": (2, 3), "early_mfma": (3, 4)}.items():
                d = (s[:, :-1, p1] - s[:, :-1, p0])[ok]
                segs[nm_] = int(np.median(d)) if d.size else None
            d = (s[:, 1:, 0] - s[:, :-1, 4])[ok]
            segs["to_next_barrier"] = int(np.median(d)) if d.size else None
            d = (s[:, 1:, 0] - s[:, :-1, 0])[ok]
            segs["step"] = int(np.median(d)) if d.size else None
            out[tag] = segs
        print(json.dumps({"shape": name, **out}), flush=True)


if __name__ == "__main__":
    main()
