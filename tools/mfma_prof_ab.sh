#!/bin/bash
# rocprofv3 kernel trace of a one-group rollout under two MFMA settings (GM_MFMA), same box
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for m in 16 16all; do
  GM_MFMA=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/mprof_$m -o bench \
      -- python bench.py --steps 100 --groups 1 --no-cpu-baseline --no-train --no-f32-compare > gpurun_out/mprof_$m.log 2>&1 || exit $?
done
