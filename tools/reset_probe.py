#!/usr/bin/env python3
"""k_env_reset at the bench's sizes: launch time (HIP events on the launch stream) and the topology
attempts per env (topo_reps), to split the reset into per-attempt cost x worst env. Usage:
python tools/reset_probe.py [N ...]"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")

for N in [int(a) for a in sys.argv[1:]] or [20]:
    net = gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    env = gm.Routing(net, 20, n_env=4096, seed=0, agent_adjacency=False)
    env.reset_()
    ts, reps = [], []
    for it in range(6):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.reset_()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
        reps.append(env.get_state()["topo_reps"].copy())
    r = np.concatenate(reps)
    per_env_max = [int(x.max()) for x in reps]
    print(f"N={N} reset us {[round(t) for t in ts]} reps mean {r.mean():.2f} max per reset {per_env_max} "
          f"p99 {np.percentile(r, 99):.0f}; us per worst-env attempt {np.median(ts) / np.median(per_env_max):.1f}",
          flush=True)
