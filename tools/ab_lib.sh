#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-train --no-f32-compare > gpurun_out/ab_new$i.log 2>&1 || exit $?
  GM_LIB=$PWD/ab_old/libgraphmarl_amd.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-train --no-f32-compare > gpurun_out/ab_old$i.log 2>&1 || exit $?
done
