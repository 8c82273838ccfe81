#!/bin/bash
# A/B of the routing encoder's columns per lane above N = 30 (GM_RENC_CPL=2: the W^T slice up to 160 KB of
# LDS, one block per CU, vs the default 1 column per lane), rollout at several node counts, interleaved:
# tools/renc_cpl_ab.sh "40 50" -> gpurun_out/renc_cpl_ab.log
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for n in ${1:-40 50}; do
  for c in 0 2 0 2; do
    GM_RENC_CPL=$c timeout -k 10 240 python bench.py --n-router $n --steps 50 --no-train --no-cpu-baseline --no-extras \
        --no-pmc --no-f32-compare > gpurun_out/renc_cpl.tmp 2>&1 || exit 1
    python -c "import json; s=open('gpurun_out/renc_cpl.tmp').read(); i=s.index('{\"metric\"'); d=json.loads(s[i:s.index(chr(10),i)]); print('N=$n cpl=$c', d['value'], [round(v['avg_us'],1) for k, v in d['kernels'].items() if k.startswith('routing_enc')])" >> gpurun_out/renc_cpl_ab.log
  done
done
