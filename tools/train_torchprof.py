#!/usr/bin/env python3
"""torch.profiler attribution of one training update (device time per torch op, incl. the
glue kernels between the HIP library calls): runs bench.py's rollout + training leg and
profiles the third dqn_update call. python tools/train_torchprof.py [rows]"""
import importlib
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
T = importlib.import_module("graph-marl_amd.train")
import bench  # noqa: E402

_orig = T.dqn_update
calls = {"n": 0}
ROWS = int(sys.argv[1]) if len(sys.argv) > 1 else 60


def wrapped(*a, **k):
    calls["n"] += 1
    if calls["n"] != 3:
        return _orig(*a, **k)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        r = _orig(*a, **k)
        torch.cuda.synchronize()
    rows = ROWS
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=rows, max_name_column_width=60),
          flush=True)
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=rows,
                                                             max_name_column_width=50, max_shapes_column_width=70),
          flush=True)
    return r


T.dqn_update = wrapped
sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-f32-compare", "--steps", "10", "--warmup", "2", "--train-steps",
            "3", "--no-kernel-timers"]
bench.main()
