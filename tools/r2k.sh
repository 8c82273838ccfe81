#!/bin/bash
# routing encoder rows per block at N = 20 / 30 / 40 (GM_RENC_ROWS = 256 / 512 / 1024)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for n in 40 30 20; do
  for r in 256 512 1024; do
    GM_RENC_ROWS=$r timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 50 \
      --n-router $n > gpurun_out/bench_renc_n${n}_r$r.log 2>&1 || exit $?
    echo "n=$n rows=$r $(python tools/ab_show.py gpurun_out/bench_renc_n${n}_r$r.log)" >> gpurun_out/renc_ab.txt 2>&1
  done
done
