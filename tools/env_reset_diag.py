#!/usr/bin/env python3
"""k_env_reset time (4096 envs, A=20) for random vs fixed topologies and N = 20 / 50:
python tools/env_reset_diag.py"""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")


def timed(env, reps=5):
    env.reset_()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        env.reset_()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    out = {}
    for N in (20, 50):
        for rnd in (True, False):
            net = gm.Network(N, random_topology=rnd, excluded_seeds=gm.EVAL_SEEDS)
            env = gm.Routing(net, 20, n_env=4096, seeds=list(range(4096)), obs_extra=512)
            out[f"N{N}_{'random' if rnd else 'fixed'}_us"] = round(timed(env), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
