#!/bin/bash
# A/B of bench.py flag sets, interleaved (ROUNDS, default 2): tools/bench_ab_flags.sh "<flags A>" "<flags B>" ..
# -> gpurun_out/abf.log, one JSON line per run {flags, rollout value, ms per step, DQN layer-1 frac}
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do
  for f in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-extras --steps ${STEPS:-200} --no-train \
        --no-f32-compare $f > gpurun_out/abf.tmp 2>&1 || exit $?
    python - "$f" >> gpurun_out/abf.log <<'PY'
import json, sys
s = open("gpurun_out/abf.tmp").read()
i = s.index('{"metric"')
d = json.loads(s[i:s.index("\n", i)])
print(json.dumps({"flags": sys.argv[1], "rollout": d["value"], "ms": d["ms_per_step"], "frac": (d.get("roofline") or {}).get("frac")}))
PY
  done
done
