#!/bin/bash
# Interleaved A/B of variant libraries (tools/build_var.sh) on DQN layer 1 (tools/presplit_bench.py) and the
# rollout GEMM shapes (tools/gemm_bench.py):   tools/var_ab.sh <lib dir> [<lib dir> ...]   ("default" = lib/)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in "$@"; do  # outputs of every build on the same inputs: a schedule change must not change a bit
  lib=graph-marl_amd/lib/$v/libgraphmarl_amd.so
  [ "$v" = default ] && lib=
  GM_LIB=$lib timeout -k 10 120 python tools/var_check.py $v >> gpurun_out/var_ab.log 2>&1 || exit $?
done
python tools/var_check.py --compare "$@" >> gpurun_out/var_ab.log 2>&1
for i in 1 2 3; do
  for v in "$@"; do
    lib=graph-marl_amd/lib/$v/libgraphmarl_amd.so
    [ "$v" = default ] && lib=
    GM_LIB=$lib timeout -k 10 120 python tools/presplit_bench.py >> gpurun_out/var_ab.log 2>&1 || exit $?
    [ -n "$TILE9" ] && { GM_LIB=$lib TILE=9 timeout -k 10 120 python tools/presplit_bench.py >> gpurun_out/var_ab.log 2>&1 || exit $?; }
    if [ "$i" = 1 ]; then
      echo "== $v gemm_bench" >> gpurun_out/var_ab.log
      GM_LIB=$lib X3_TILES=${X3_TILES:--1} TILES= timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/var_ab.log || exit $?
    fi
  done
done
