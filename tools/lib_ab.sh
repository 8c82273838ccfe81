#!/bin/bash
# A/B of two builds of libgraphmarl_amd.so (GM_LIB) in one box, interleaved: DQN layer 1
# (tools/presplit_bench.py), the rollout GEMM shapes (tools/gemm_bench.py, default tiles) and the
# rollout bench line without the training / extra legs.   tools/lib_ab.sh <lib dir B> [<lib dir A>]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
B=graph-marl_amd/lib/$1/libgraphmarl_amd.so
A=${2:+graph-marl_amd/lib/$2/libgraphmarl_amd.so}
for i in 1 2; do
  for lib in "$A" "$B"; do
    tag=${lib:-default}
    echo "== $tag" >> gpurun_out/lib_ab.log
    GM_LIB=$lib timeout -k 10 120 python tools/presplit_bench.py >> gpurun_out/lib_ab.log 2>&1 || exit $?
    GM_LIB=$lib X3_TILES=-1 TILES= timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/lib_ab.log || exit $?
    GM_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --no-train --no-f32-compare --no-extras \
        > gpurun_out/lib_ab_bench.tmp 2>&1 || exit $?
    python -c "import json,sys; s=open('gpurun_out/lib_ab_bench.tmp').read(); i=s.index('{\"metric\"'); d=json.loads(s[i:s.index(chr(10),i)]); print('rollout', d['value'], d['ms_per_step'], {k: v.get('avg_us') for k, v in (d.get('kernels') or {}).items()} if isinstance(d.get('kernels'), dict) else '')" >> gpurun_out/lib_ab.log
    if [ -n "$TRAIN" ]; then
      GM_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --no-f32-compare --no-kernel-timers \
          --no-extras > gpurun_out/lib_ab_bench.tmp 2>&1 || exit $?
      python -c "import json; s=open('gpurun_out/lib_ab_bench.tmp').read(); i=s.index('{\"metric\"'); d=json.loads(s[i:s.index(chr(10),i)]); print('train', d['rollout_train'])" >> gpurun_out/lib_ab.log
    fi
  done
done
