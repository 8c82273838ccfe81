#!/bin/bash
# config-4 node counts: rollout kernel times at N = 30 / 40 (one group for the per-kernel timers)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for n in 30 40 20; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 50 --n-router $n \
    > gpurun_out/bench_n$n.log 2>&1 || exit $?
  python tools/ab_show.py gpurun_out/bench_n$n.log >> gpurun_out/n_ab.txt 2>&1
done
