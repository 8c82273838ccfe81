#!/bin/bash
# LDS-DMA GEMM tiles: parity test, then timings over the x3 tile table.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --tb=short --timeout=240 -k "lds_dma" -p no:cacheprovider > gpurun_out/glds_test.log 2>&1
rc=$?; tail -15 gpurun_out/glds_test.log; [ $rc -eq 0 ] || exit $rc
X3_TILES=${X3_TILES:--1,8,9,10,11} timeout -k 10 300 python tools/gemm_diag.py > gpurun_out/glds_diag.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/glds_diag.log; exit $rc
