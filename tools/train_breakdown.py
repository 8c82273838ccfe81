#!/usr/bin/env python3
"""Per-kernel breakdown of the LAST training update in a rocprofv3 kernel trace of
tools/train_prof.sh (split at the first weight-gradient kernel: forward + target | backward)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tprof/t_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "pcg64" in r["Kernel_Name"]]
seq = rows[idx[-1]:]
b = [i for i, r in enumerate(seq) if "kmajor" in r["Kernel_Name"] or "wgrad" in r["Kernel_Name"]][0]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


print(f"forward+target {sum(map(dur, seq[:b])):.0f} us, backward+optimizer {sum(map(dur, seq[b:])):.0f} us, "
      f"span {(int(seq[-1]['End_Timestamp']) - int(seq[0]['Start_Timestamp'])) / 1e3:.0f} us")
for part, s in (("forward+target", seq[:b]), ("backward", seq[b:])):
    agg = collections.Counter()
    cnt = collections.Counter()
    for r in s:
        k = (r["Kernel_Name"].replace("_ZN12_GLOBAL__N_1", "")[:44], r["Grid_Size_X"] + "x" + r.get("Grid_Size_Y", "1"))
        agg[k] += dur(r)
        cnt[k] += 1
    print(part)
    for k, v in agg.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 24):
        print(f"{v:9.1f} us {cnt[k]:4d}x  grid {k[1]:>9}  {k[0]}")

if len(sys.argv) > 3 and sys.argv[3] == "order":  # every backward launch above 50 us, in launch order
    print("backward launches in order")
    for r in seq[b:]:
        if dur(r) > 50:
            print(f"{dur(r):9.1f} us  grid {r['Grid_Size_X']:>9}x{r.get('Grid_Size_Y', '1'):<5} {r['Kernel_Name'][:60]}")
