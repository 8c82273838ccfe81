#!/bin/bash
# A/B of DQN layer 1 against the pre-split diagnostic builds (tools/build_diag.sh with DIAGS="11 12")
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for d in "" diag11 diag12; do
    if [ -n "$d" ]; then lib=graph-marl_amd/lib/$d/libgraphmarl_amd.so; else lib=; fi
    GM_LIB=$lib timeout -k 10 120 python tools/presplit_bench.py >> gpurun_out/presplit_ab.log 2>&1 || exit $?
  done
done
cat gpurun_out/presplit_ab.log
