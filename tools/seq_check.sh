#!/bin/bash
# train_seq: kernel + golden + autograd-parity tests, then rollout+train with the sequence-batched
# and the autograd update (interleaved)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_train_seq_gpu.py -k "rollout or golden" > gpurun_out/seq_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers \
    > gpurun_out/seq_b$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers --train-autograd \
    > gpurun_out/seq_a$i.log 2>&1 || exit $?
done
