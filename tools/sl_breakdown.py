#!/usr/bin/env python3
"""Per-kernel time of the LAST SL iteration in a rocprofv3 kernel trace of tools/prof_sl_train.sh
(iterations split at AdamW's multi_tensor_apply launches). python tools/sl_breakdown.py [trace] [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/slprof/sl_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"]]
ends = [adam[i] for i in range(len(adam)) if i + 1 == len(adam) or adam[i + 1] - adam[i] > 20]
seq = rows[ends[-2] + 1:ends[-1] + 1]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"last iteration: {len(seq)} kernels, {sum(map(dur, seq)):.0f} us busy, span {span:.0f} us")
agg, cnt = collections.Counter(), collections.Counter()
for r in seq:
    k = (r["Kernel_Name"].replace("_ZN12_GLOBAL__N_1", "")[:50], r.get("Grid_Size_X") or r.get("Grid_Size"))
    agg[k] += dur(r)
    cnt[k] += 1
for k, v in agg.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    print(f"{v:9.1f} us {cnt[k]:4d}x  grid {k[1]:>10}  {k[0]}")
