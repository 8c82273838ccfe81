#!/bin/bash
# rocprofv3 kernel stats of the config-5 SL bench and of the rollout + training leg (bench.py
# --train-steps), one profile each: gpurun_out/slprof/sl_kernel_stats.csv, gpurun_out/tprof/t_kernel_stats.csv
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/slprof gpurun_out/tprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/slprof -o sl \
    -- python graph-marl_amd/sl.py --bench --n-nodes 100 --batch-size 8192 --sequence-length 8 --netmon-iterations 1 \
    --iterations 3 --warmup 1 > gpurun_out/slprof/run.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/tprof -o t \
    -- python bench.py --steps 4 --warmup 2 --graph 0 --no-extras --no-cpu-baseline --no-f32-compare --no-kernel-timers \
    --no-pmc --train-steps 4 > gpurun_out/tprof/b.log 2>&1
