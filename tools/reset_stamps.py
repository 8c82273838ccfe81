#!/usr/bin/env python3
"""Diagnostic (a stamp build of gm_env.hip exporting gm_diag_reset_stamps, via GM_LIB): per env the
cycles of MT seeding, twist, attempt bodies and the finish (APSP), and the worst env's split."""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
L = gm._lib.lib()
for N in [int(a) for a in sys.argv[1:]] or [20]:
    net = gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    env = gm.Routing(net, 20, n_env=4096, seed=0, agent_adjacency=False)
    buf = torch.zeros(4096 * 6, dtype=torch.int64, device="cuda")
    L.gm_diag_reset_stamps(C.c_void_p(buf.data_ptr()))
    env.reset_()
    for it in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.reset_()
        e.record()
        torch.cuda.synchronize()
        st = buf.view(4096, 6).cpu().numpy().astype(np.float64)
        reps = env.get_state()["topo_reps"]
        w = int(np.argmax(st[:, 5] - st[:, 4]))
        t0 = st[:, 4].min()
        print(f"N={N} reset {s.elapsed_time(e) * 1e3:.0f} us; cycles/attempt mean: seed {st[:, 0].sum() / reps.sum():.0f} "
              f"twist {st[:, 1].sum() / reps.sum():.0f} body {st[:, 2].sum() / reps.sum():.0f}; finish {st[:, 3].mean():.0f}; "
              f"worst env {w}: reps {reps[w]} start {st[w, 4] - t0:.0f} span {st[w, 5] - st[w, 4]:.0f} "
              f"seed {st[w, 0]:.0f} twist {st[w, 1]:.0f} body {st[w, 2]:.0f}; last end {st[:, 5].max() - t0:.0f}; "
              f"start spread p50 {np.median(st[:, 4] - t0):.0f} max {(st[:, 4] - t0).max():.0f}", flush=True)
