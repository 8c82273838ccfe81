#!/bin/bash
# A/B: round-2 library (lib/old, before the activation generalisation) vs the current one, then the
# whole GPU suite
cd "$(dirname "$0")/.." || exit 1
O="GM_LIB=/root/repo/graph-marl_amd/lib/old/libgraphmarl_amd.so"
tools/gpu_steps.sh "o1:200:$O python bench.py --no-extras --no-cpu-baseline --no-train --no-f32-compare --steps 200" "n1:200:python bench.py --no-extras --no-cpu-baseline --no-train --no-f32-compare --steps 200" "o2:200:$O python bench.py --no-extras --no-cpu-baseline --no-train --no-f32-compare --steps 200" "n2:200:python bench.py --no-extras --no-cpu-baseline --no-train --no-f32-compare --steps 200"   "gputests:1200:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
