#!/bin/bash
# SQ counters (LDS / MFMA / wait split) of the training kernels: one rocprofv3 pass over a short
# rollout + 2 sequence-batched updates -> gpurun_out/tsq/summary.txt
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tsq
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -T --output-format csv -d gpurun_out/tsq -o sq \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timers --no-f32-compare --train-steps 2 --graph 0 --no-pmc --no-extras \
    > gpurun_out/tsq/bench.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/tsq/summary.txt
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/tsq/sq_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:25]:
    wc = max(d.get("SQ_WAVE_CYCLES", 0), 1)
    lds = max(d.get("SQ_LDS_IDX_ACTIVE", 0), 1)
    print(f"{k:70s} wavecyc {wc:12.0f} active {d.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait {d.get('SQ_WAIT_ANY', 0) / wc:.2f} "
          f"stall {d.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} ldsstall {d.get('SQ_WAIT_INST_LDS', 0) / wc:.2f} "
          f"bankconf/ldsactive {d.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.3f} mfma_busy {d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.3e}")
PY
