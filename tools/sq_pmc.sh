#!/bin/bash
# SQ counters (one rocprofv3 pass of 8) over a short rollout bench, summarised per kernel:
# tools/sq_pmc.sh  ->  gpurun_out/sq/summary.txt
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -T --output-format csv -d gpurun_out/sq -o sq -- python bench.py --steps 10 \
    --warmup 3 --groups 1 --no-cpu-baseline --no-pmc --no-extras --no-kernel-timers --no-train --no-f32-compare \
    > gpurun_out/sq/bench.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/sq/summary.txt
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/sq/sq_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    n = max(len(v) for v in d.values())
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    w = avg.get("SQ_WAVES", 1) or 1
    wc = avg.get("SQ_WAVE_CYCLES", 0)
    print(f"{k:60s} launches {n:4d} waves {w:8.0f} wave-qcycles/wave {wc / w:9.0f} "
          f"active {avg.get('SQ_ACTIVE_INST_ANY', 0) / max(wc, 1):.2f} wait {avg.get('SQ_WAIT_ANY', 0) / max(wc, 1):.2f} "
          f"stall {avg.get('SQ_WAIT_INST_ANY', 0) / max(wc, 1):.2f} valu/wave {avg.get('SQ_INSTS_VALU', 0) / w:7.0f} "
          f"salu/wave {avg.get('SQ_INSTS_SALU', 0) / w:7.0f} lds/wave {avg.get('SQ_INSTS_LDS', 0) / w:6.0f}")
PY
