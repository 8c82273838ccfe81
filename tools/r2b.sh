cd /root/repo && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_replay_rng.py tests/test_checkpoint.py tests/test_train_gpu.py \
  "tests/test_env_gpu.py::test_set_state_restores_a_dump" \
  "tests/test_cli_train_gpu.py::test_routing_netmon_aux_loss_train" > gpurun_out/r2b.log 2>&1
