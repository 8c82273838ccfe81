#!/bin/bash
# Effective clock and MFMA busy of one GEMM shape / tile (one PMC pass + kernel trace):
#   tools/pmc_clock.sh <shape> <tile> [lib]   -> gpurun_out/pmcc/<shape>_t<tile>*
cd "$(dirname "$0")/.." || exit 1
shape=$1; t=$2; tag=${3:-default}
[ -n "$3" ] && export GM_LIB=$PWD/graph-marl_amd/lib/$3/libgraphmarl_amd.so
mkdir -p gpurun_out/pmcc
GM_TILE=$t timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-trace -T --output-format csv -d gpurun_out/pmcc -o ${shape}_t${t}_$tag \
    -- python tools/gemm_one.py $shape x3 20 > gpurun_out/pmcc/${shape}_t${t}_$tag.log 2>&1
