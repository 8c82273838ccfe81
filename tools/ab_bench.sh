#!/bin/bash
# Interleaved bench.py A/B of library builds (GM_LIB; "default" = graph-marl_amd/lib): rollout + training line
# without the extra legs, kernel timers on. tools/ab_bench.sh <reps> <lib dir> [<lib dir> ...]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
reps=$1; shift
for i in $(seq "$reps"); do
  for name in "$@"; do
    lib=""; [ "$name" != default ] && lib=graph-marl_amd/lib/$name/libgraphmarl_amd.so
    GM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --no-f32-compare --no-extras --no-pmc \
        --train-steps 4 > gpurun_out/ab_bench.tmp 2>&1 || exit $?
    python - "$name" >> gpurun_out/ab_bench.log <<'PY'
import json, sys
s = open("gpurun_out/ab_bench.tmp").read()
i = s.index('{"metric"')
d = json.loads(s[i:s.index("\n", i)])
k = {t[:40]: round(v["avg_us"], 1) for t, v in d["kernels"].items()}
print(sys.argv[1], "rollout", d["value"], "train", (d.get("rollout_train") or {}).get("value"), k)
PY
  done
done
