#!/usr/bin/env python3
"""torch.profiler attribution of one config-5 SL iteration (device time per torch op, incl. the glue
kernels between the HIP library calls): sl.py --bench at N = 100, batch 8192, L = 8, K = 1; profiles
the third train_step call. python tools/sl_torchprof.py [rows]"""
import importlib
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SL = importlib.import_module("graph-marl_amd.sl")

_orig = SL.train_step
calls = {"n": 0}
ROWS = int(sys.argv[1]) if len(sys.argv) > 1 else 40


def wrapped(*a, **k):
    calls["n"] += 1
    if calls["n"] != 3:
        return _orig(*a, **k)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        r = _orig(*a, **k)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=ROWS, max_name_column_width=60),
          flush=True)
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=ROWS,
                                                             max_name_column_width=40, max_shapes_column_width=90),
          flush=True)
    return r


SL.train_step = wrapped
print(SL.main(["--bench", "--n-nodes", "100", "--batch-size", "8192", "--sequence-length", "8",
               "--netmon-iterations", "1", "--iterations", "2", "--warmup", "1"], quiet=True), flush=True)
