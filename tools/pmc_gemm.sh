cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmcg
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmcg/avail.txt 2>&1 || true
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/pmcg -o $tag -- python tools/gemm_one.py enc.l1 x3 5 > gpurun_out/pmcg/$tag.log 2>&1 || echo "fail $c"
done
