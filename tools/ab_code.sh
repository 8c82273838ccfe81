#!/bin/bash
# Interleaved A/B of two code trees on one box (round 6): ab_old/ (an earlier commit's bench.py + package +
# headers, library built in place, git-ignored) against the working tree: rollout + training line without
# the extra legs. tools/ab_code.sh <reps>
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in $(seq "$1"); do
  for tree in ab_old .; do
    timeout -k 10 300 python $tree/bench.py --no-cpu-baseline --steps 100 --no-f32-compare --no-extras --no-pmc \
        --train-steps 4 > gpurun_out/ab_code.tmp 2>&1 || exit $?
    python - "$tree" >> gpurun_out/ab_code.log <<'PY'
import json, sys
s = open("gpurun_out/ab_code.tmp").read()
i = s.index('{"metric"')
d = json.loads(s[i:s.index("\n", i)])
k = {t[:40]: round(v["avg_us"], 1) for t, v in d["kernels"].items()}
print(sys.argv[1], "rollout", d["value"], "train", (d.get("rollout_train") or {}).get("value"),
      (d.get("rollout_train") or {}).get("ms_per_step"), k)
PY
  done
done
