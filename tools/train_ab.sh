#!/bin/bash
# A/B of the rollout + training number: tools/train_ab.sh "<env A>" "<env B>" (e.g. "" "GM_JOINT_CAT=1")
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers --no-extras > gpurun_out/tab_a$i.log 2>&1 || exit $?
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers --no-extras > gpurun_out/tab_b$i.log 2>&1 || exit $?
done
