#!/bin/bash
# routing encoder rows rule: parity tests, then the rollout at N = 20 / 30 / 40
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_train_seq_gpu.py tests/test_sl_gpu.py tests/test_netmon_gpu.py > gpurun_out/r2l.log 2>&1 && \
for n in 20 30 40; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --steps 50 --train-steps 2 --n-router $n \
    > gpurun_out/bench_rule_n$n.log 2>&1 || exit $?
  echo "n=$n $(python tools/ab_show.py gpurun_out/bench_rule_n$n.log)" >> gpurun_out/rule_ab.txt 2>&1
done
