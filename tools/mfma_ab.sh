#!/bin/bash
# MFMA shape of k_gemm3g (GM_MFMA=16 vs 32): correctness tests on the default form, the training
# GEMM shapes under both, then the rollout and rollout + training numbers interleaved (two rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_netmon_gpu.py tests/test_long_horizon_gpu.py tests/test_train_gpu.py \
  > gpurun_out/mab_tests.log 2>&1 || exit $?
for m in 16 32; do
  GM_MFMA=$m TILES=0,12 timeout -k 10 300 python tools/train_gemm_bench.py > gpurun_out/mab_tgb_$m.log 2>&1 || exit $?
done
for i in 1 2; do
  for m in 16 32; do
    GM_MFMA=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-f32-compare --train-steps 4 \
      > gpurun_out/mab_${m}_$i.log 2>&1 || exit $?
  done
done
