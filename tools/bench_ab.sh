#!/bin/bash
# Interleaved bench.py A/B of variant libraries (rollout + training leg, no extras / CPU baseline / PMC),
# ROUNDS rounds (default 2; EXTRAS=1 also times the other configs, incl. config 5 SL):   tools/bench_ab.sh <lib dir> ...   ("default" = lib/)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    lib=graph-marl_amd/lib/$v/libgraphmarl_amd.so
    [ "$v" = default ] && lib=
    GM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $([ -n "$EXTRAS" ] || echo --no-extras) --no-pmc --no-f32-compare \
        ${BENCH_ARGS:---steps 100 --train-steps 5} > gpurun_out/bench_ab.tmp 2>&1 || exit $?
    python - "$v" >> gpurun_out/bench_ab.log <<'PY'
import json, sys
s = open("gpurun_out/bench_ab.tmp").read()
i = s.index('{"metric"')
d = json.loads(s[i:s.index("\n", i)])
k = {t: round(v["avg_us"], 1) for t, v in (d.get("kernels") or {}).items()}
print(json.dumps({"lib": sys.argv[1], "rollout": d["value"], "ms": d["ms_per_step"], "frac": (d.get("roofline") or {}).get("frac"),
                  "train": (d.get("rollout_train") or {}).get("value"),
                  "other": {c: v.get("value") for c, v in (d.get("other_configs") or {}).items()}, "kernels": k}))
PY
  done
done
