#!/bin/bash
# GEMM-ready env obs copy (K = 640 DQN layer 1): parity tests, then the rollout A/B (GM_GEMM_OBS=0 / 1)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_env_gpu.py tests/test_fused_gpu.py tests/test_long_horizon_gpu.py tests/test_rollout_gpu.py \
  tests/test_cli_train_gpu.py tests/test_distributed_gpu.py > gpurun_out/r2m.log 2>&1 && \
for v in 0 1 0 1; do
  GM_GEMM_OBS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 200 \
    > gpurun_out/bench_gobs_$v.log 2>&1 || exit $?
  echo "gemm_obs=$v $(python tools/ab_show.py gpurun_out/bench_gobs_$v.log)" >> gpurun_out/gobs_ab.txt 2>&1
done
