#!/bin/bash
# Interleaved config-5 (sl.py --bench, N = 100, 8192 graphs, 8 steps) A/B of library builds (GM_LIB; "default" =
# graph-marl_amd/lib). tools/sl_ab.sh <reps> <lib dir> [<lib dir> ...]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
reps=$1; shift
for i in $(seq "$reps"); do
  for name in "$@"; do
    lib=""; [ "$name" != default ] && lib=graph-marl_amd/lib/$name/libgraphmarl_amd.so
    echo -n "$name " >> gpurun_out/sl_ab.log
    GM_LIB=$lib timeout -k 10 200 python graph-marl_amd/sl.py --bench --n-nodes 100 --batch-size 8192 --sequence-length 8 \
        --netmon-iterations 1 --iterations 5 --warmup 2 2>/dev/null | grep '"metric"' | cut -c1-200 >> gpurun_out/sl_ab.log || exit $?
  done
done
