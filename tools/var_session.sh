#!/bin/bash
# One GPU session of GEMM-variant work: bit checks of every build vs the default, k-step stamps of
# the stamp builds (STAMPS="vstamp ..."), then interleaved timing (tools/var_ab.sh).
#   tools/var_session.sh <lib dir> ...     (STAMPS env: diagnostic-30 builds)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in $STAMPS; do
  GM_LIB=graph-marl_amd/lib/$v/libgraphmarl_amd.so timeout -k 10 120 python tools/stamp_bench.py 2>&1 | grep -v amdgpu.ids \
      | sed "s/^/$v /" >> gpurun_out/stamps.log || exit $?
done
timeout -k 10 900 tools/var_ab.sh "$@"
