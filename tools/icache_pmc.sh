#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ic
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -T --output-format csv -d gpurun_out/ic -o ic -- python bench.py --steps 10 --warmup 3 --groups 1 --no-cpu-baseline --no-pmc --no-extras --no-kernel-timers --no-train --no-f32-compare --graph 0 > gpurun_out/ic/bench.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/ic/summary.txt
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/ic/ic_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQC_ICACHE_MISSES", [0]))):
    h = sum(d.get("SQC_ICACHE_HITS", [0])) / max(1, len(d.get("SQC_ICACHE_HITS", [1])))
    m = sum(d.get("SQC_ICACHE_MISSES", [0])) / max(1, len(d.get("SQC_ICACHE_MISSES", [1])))
    print(f"{k:70s} hits {h:12.0f} misses {m:10.0f} miss-rate {m / max(h + m, 1):.4f}")
PY
