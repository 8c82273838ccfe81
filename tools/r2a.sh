cd /root/repo && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py::test_gemm_x3_range_guard tests/test_long_horizon_gpu.py tests/test_distributed_gpu.py \
  tests/test_sl_gpu.py "tests/test_env_gpu.py" > gpurun_out/r2a.log 2>&1
