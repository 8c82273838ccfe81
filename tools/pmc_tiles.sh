#!/bin/bash
# PMC passes (one counter group per run) of one GEMM shape for several x3 tiles:
#   tools/pmc_tiles.sh <shape> <tile> [<tile> ...]
cd "$(dirname "$0")/.." || exit 1
shape=$1; shift
mkdir -p gpurun_out/pmct
for t in "$@"; do
  for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    tag=$(echo $c | cut -d' ' -f1)
    GM_TILE=$t timeout -s KILL 90 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/pmct -o ${shape}_t${t}_$tag \
        -- python tools/gemm_one.py $shape x3 5 > gpurun_out/pmct/${shape}_t${t}_$tag.log 2>&1 || { echo "fail $t $c"; exit 1; }
  done
done
