#!/bin/bash
# rocprofv3 kernel stats of a short rollout + training bench (training kernels dominate)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tprof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/tprof -o t \
    -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-f32-compare --no-kernel-timers --graph 0 --no-extras --train-steps 4 \
    > gpurun_out/tprof/b.log 2>&1
