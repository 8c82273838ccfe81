#!/bin/bash
# Config-5 checks through gpurun: the SL GPU tests, the SL bench (N = 100, batch 8192, L = 8, K = 1) and the
# output head's forward GEMM per tile (tools/train_gemm_bench.py). Each step under its own time limit, chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sl_seq_gpu.py tests/test_sl_gpu.py -p no:cacheprovider > gpurun_out/sl_tests.log 2>&1 &&
timeout -k 10 300 python graph-marl_amd/sl.py --bench --n-nodes 100 --batch-size 8192 --sequence-length 8 --netmon-iterations 1 --iterations 5 --warmup 2 > gpurun_out/sl_bench.log 2>&1 &&
ROWS=6553600 SHAPES=fwd.slhead:100:512:fwd TILES=0,12,13,9,10 timeout -k 10 300 python tools/train_gemm_bench.py > gpurun_out/slhead_tiles.log 2>&1
