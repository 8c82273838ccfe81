#!/bin/bash
# A/B of bench.py flag sets, interleaved: tools/bench_ab_flags.sh "<flags A>" "<flags B>"
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-train --no-f32-compare $1 > gpurun_out/abf_a$i.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-train --no-f32-compare $2 > gpurun_out/abf_b$i.log 2>&1 || exit $?
done
