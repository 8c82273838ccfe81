#!/bin/bash
# train_seq: kernel + golden + autograd-parity tests, the rollout+train number, and a kernel profile
# of the update (gpurun_out/tprof, tools/train_breakdown.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tprof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_train_seq_gpu.py tests/test_netmon_gpu.py tests/test_fused_gpu.py > gpurun_out/seq_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers \
    > gpurun_out/seq_b1.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/tprof -o t \
    -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-f32-compare --no-kernel-timers --train-steps 4 \
    > gpurun_out/tprof/b.log 2>&1 || exit $?
python tools/train_breakdown.py gpurun_out/tprof/t_kernel_trace.csv 30 > gpurun_out/tprof/breakdown.txt
