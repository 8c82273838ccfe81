#!/bin/bash
# GPU validation chain (run through gpurun). Each step has its own time limit and
# the chain stops at the first failure, so a fault/timeout never starts more GPU work.
#   tools/gpu_check.sh [smoke] [tests] [bench] [prof]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))" | tee -a gpurun_out/chain.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/chain.log
    tail -5 "gpurun_out/$name.log"
    return $rc
}
rc=0
for s in "$@"; do
    case $s in
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        tests) step gpu_tests 900 python -m pytest tests -m gpu -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        envtests) step env_tests 600 python -m pytest tests/test_env_gpu.py -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        clitests) step cli_tests 900 python -m pytest tests/test_cli_train_gpu.py -x -q --tb=short --timeout=600 -p no:cacheprovider || exit $? ;;
        nettests) step net_tests 600 python -m pytest tests/test_netmon_gpu.py tests/test_train_gpu.py -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        sl) step sl_bench 600 python graph-marl_amd/sl.py --bench --n-nodes 100 --batch-size 8192 --sequence-length 8 \
                --netmon-iterations 1 --iterations 5 --warmup 2 || exit $? ;;
        sl20) step sl20_bench 600 python graph-marl_amd/sl.py --bench --n-nodes 20 --batch-size 1024 --sequence-length 4 \
                --netmon-iterations 3 --iterations 20 --warmup 3 || exit $? ;;
        dist2) GM_BENCH_SHARE_GPU=1 step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 \
                --no-cpu-baseline || exit $? ;;
        gemm) X3_TILES=${X3_TILES:--1,1,2,3,4,5} step gemm 300 python tools/gemm_bench.py || exit $? ;;
        models) step models_tests 600 python -m pytest tests/test_models_gpu.py -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        fused) step fused_tests 600 python -m pytest tests/test_fused_gpu.py -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        rollout) step rollout_tests 600 python -m pytest tests/test_rollout_gpu.py -x -q --tb=short --timeout=300 -p no:cacheprovider || exit $? ;;
        benchg) step bench_graph 300 python bench.py --no-cpu-baseline --steps 100 --graph ${GRAPH:-2} --no-train || exit $? ;;
        benchg0) step bench_eager 300 python bench.py --no-cpu-baseline --steps 100 --no-train || exit $? ;;
        benchf32) GM_GEMM=f32 step bench_f32 300 python bench.py --no-cpu-baseline --steps 100 || exit $? ;;
        bench) step bench 600 python bench.py || exit $? ;;
        benchst) step bench_stagger 300 python bench.py --no-cpu-baseline --steps 100 --stagger || exit $? ;;
        benchq) step bench 300 python bench.py --no-cpu-baseline --steps 100 || exit $? ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o bench \
                  -- python bench.py --steps 100 --groups 1 --no-cpu-baseline --no-pmc --no-train --no-f32-compare --no-extras --graph 0 || exit $? ;;
        pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc -o fetch \
                 -- python bench.py --steps 20 --warmup 5 --groups 1 --no-cpu-baseline --no-pmc --no-kernel-timers --no-train --no-f32-compare --no-extras --graph 0 || exit $?
             step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/pmc -o write \
                 -- python bench.py --steps 20 --warmup 5 --groups 1 --no-cpu-baseline --no-pmc --no-kernel-timers --no-train --no-f32-compare --no-extras --graph 0 || exit $? ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
exit $rc
