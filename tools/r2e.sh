cd /root/repo && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py::test_joint_first_layer_split_vs_fp64 tests/test_train_gpu.py tests/test_replay_rng.py \
  tests/test_cli_train_gpu.py tests/test_distributed_gpu.py tests/test_models_gpu.py > gpurun_out/r2e.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu-baseline --no-f32-compare --steps 20 --warmup 5 --train-steps 5 > gpurun_out/bench_train.log 2>&1
