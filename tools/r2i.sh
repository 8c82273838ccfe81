#!/bin/bash
# fused ε-greedy + env step: parity tests, then the rollout bench A/B (GM_POLICY_STEP=split / fused)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_fused_gpu.py tests/test_long_horizon_gpu.py \
  tests/test_cli_train_gpu.py > gpurun_out/r2i.log 2>&1 && \
for v in split fused split fused; do
  GM_POLICY_STEP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 200 \
    > gpurun_out/bench_pol_$v.log 2>&1 || exit $?
  python tools/ab_show.py gpurun_out/bench_pol_$v.log >> gpurun_out/pol_ab.txt 2>&1
done
