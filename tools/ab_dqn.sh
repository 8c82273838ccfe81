#!/bin/bash
# fused-DQN parity tests, the benched long horizon, then GM_DQN_FUSED A/B (two interleaved pairs)
cd "$(dirname "$0")/.." || exit 1
B="python bench.py --no-extras --no-cpu-baseline --no-train --no-f32-compare --steps 200"
tools/gpu_steps.sh "t:400:python -u -m pytest tests/test_fused_gpu.py -v --timeout 120 --timeout-method thread -k 'dqn_fused or rollout_matches'" \
  "lh:300:python -u -m pytest tests/test_long_horizon_gpu.py -v -s --timeout 200 --timeout-method thread -k 'x3 and N20 and lstm and leaky'" \
  "f1:200:GM_DQN_FUSED=1 $B" "f0:200:$B" "f1b:200:GM_DQN_FUSED=1 $B" "f0b:200:$B"
