#!/bin/bash
# Default vs diagnostic builds (graph-marl_amd/lib/diagN, tools/build_diag.sh) on the rollout GEMM shapes
# (tools/gemm_bench.py, default x3 tiles): tools/diag_ab.sh 7 10  [ROWS=40960]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in "" "$@"; do
  lib=${d:+graph-marl_amd/lib/diag$d/libgraphmarl_amd.so}
  echo "== ${lib:-default}" >> gpurun_out/diag_ab.log
  GM_LIB=$lib X3_TILES=-1 TILES= timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/diag_ab.log || exit $?
done
cat gpurun_out/diag_ab.log
