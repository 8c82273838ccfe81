#!/bin/bash
# k_gemm3g timings: default build, then diag5 (no DMA in the loop) and diag6 (no compute).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in "" ${GDIAGS:-diag5 diag6}; do
  if [ -n "$d" ]; then export GM_LIB=$PWD/graph-marl_amd/lib/$d/libgraphmarl_amd.so; fi
  X3_TILES=${X3_TILES:--1,8,9,10,11} timeout -k 10 200 python tools/gemm_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
done
