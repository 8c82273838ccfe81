#!/bin/bash
# A/B of rollout + training throughput between environment settings, interleaved in one box
# (box-to-box spread is ~4 %): tools/env_ab.sh "GM_DGRAD=0" "GM_DGRAD=-1" [reps]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
A=$1 B=$2 REPS=${3:-2}
for i in $(seq 1 "$REPS"); do
    for v in A B; do
        spec=${!v}
        env $spec timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-f32-compare \
            --no-kernel-timers --train-steps 5 > "gpurun_out/envab_$v$i.log" 2>&1 || exit $?
        python -c "
import json,sys; d=json.loads(open('gpurun_out/envab_$v$i.log').read().strip().splitlines()[-1])
print('$v', '$spec', d['value'], d['rollout_train']['value'], d['rollout_train']['ms_per_step'])"
    done
done
