#!/bin/bash
# SQ counters of the routing encoder micro-benchmark (one rocprofv3 pass, 8 SQ counters)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/renc
export TMPDIR=/tmp
timeout -k 10 120 python tools/renc_bench.py > gpurun_out/renc/time.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -T --output-format csv -d gpurun_out/renc -o sq -- python tools/renc_bench.py \
    > gpurun_out/renc/pmc.log 2>&1 || exit $?
