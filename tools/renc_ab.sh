#!/bin/bash
# A/B of the routing encoder block size (GM_RENC_TPB=256 vs the default 512) in the rollout at several
# node counts, interleaved: tools/renc_ab.sh "20 40 50"
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in ${1:-20 40 50}; do
  for t in 256 512 256 512; do
    GM_RENC_TPB=$t timeout -k 10 240 python bench.py --n-router $n --steps 50 --no-train --no-cpu-baseline --no-extras \
        --no-f32-compare > gpurun_out/renc_ab.log 2>&1 || exit 1
    python -c "import json; s=open('gpurun_out/renc_ab.log').read(); i=s.index('{\"metric\"'); d=json.loads(s[i:s.index(chr(10),i)]); print('N=$n tpb=$t', d['value'], [round(v['avg_us'],1) for k, v in d['kernels'].items() if k.startswith('routing_enc')])"
  done
done
