#!/usr/bin/env python3
"""k_env_step time split (4096 envs, N=20, A=20, random topologies): full step, without the
observation emission (null obs buffers), without the info sums; HIP events over 50 steps of
random actions. python tools/env_step_diag.py"""
import ctypes as C
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gm = importlib.import_module("graph-marl_amd")
L = gm._lib


def run(env, bufs, info, steps=50):
    lib = L.lib()
    acts = [torch.randint(0, 4, (env.n_env, env.n_data), device="cuda", dtype=torch.int32) for _ in range(steps)]
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for a in acts:
        L.check(lib.gm_env_step(env._h, L.ptr(a), L.ptr(env.reward), L.ptr(env.done), L.ptr(env.info) if info else None,
                                None, C.byref(bufs), env._stream()))
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps * 1e3


def main():
    net = gm.Network(20, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
    env = gm.Routing(net, 20, n_env=4096, seeds=list(range(4096)), obs_extra=512)
    env.reset()
    full = env._obsbufs
    none = L.gm_obs_buffers() if hasattr(L, "gm_obs_buffers") else type(full)()
    r = {"full_us": run(env, full, True), "no_obs_us": run(env, none, True), "no_obs_no_info_us": run(env, none, False),
         "full2_us": run(env, full, True)}
    print(json.dumps({k: round(v, 1) for k, v in r.items()}))


if __name__ == "__main__":
    main()
