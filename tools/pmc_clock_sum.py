#!/usr/bin/env python3
"""Summarise tools/pmc_clock.sh passes: per GEMM dispatch average of each counter, the kernel
duration from the kernel trace, effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration and the
MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcc"
for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gemm" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    kt = f.replace("counter_collection", "kernel_trace")
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt))
           if "gemm" in r["Kernel_Name"]] if glob.glob(kt) else []
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    us = sum(dur[2:]) / max(1, len(dur[2:])) / 1e3 if dur else float("nan")
    g = avg.get("GRBM_GUI_ACTIVE", 0) / 8
    print(f.split("/")[-1].replace("_counter_collection.csv", ""), f"dur {us:.1f} us",
          f"clock {g / us / 1e3:.2f} GHz" if dur else "",
          f"mfma busy {avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / max(g, 1):.3f}",
          {k: round(v / 1e6, 2) for k, v in avg.items()})
