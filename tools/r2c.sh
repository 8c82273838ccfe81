cd /root/repo && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_netmon_gpu.py tests/test_rollout_gpu.py > gpurun_out/r2c.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 100 --netmon-rnn-type lnlstm > gpurun_out/bench_lnlstm.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-compare --no-train --steps 100 --netmon-rnn-type gru > gpurun_out/bench_gru.log 2>&1
