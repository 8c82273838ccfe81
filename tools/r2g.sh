cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_netmon_gpu.py tests/test_fused_gpu.py -k "aggregate or fused or netmon" > gpurun_out/r2g.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 100 > gpurun_out/bench_g.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmcg -o fetch \
  -- python bench.py --steps 20 --warmup 5 --groups 1 --no-cpu-baseline --no-kernel-timers --no-train --no-f32-compare > gpurun_out/pmcg.log 2>&1
