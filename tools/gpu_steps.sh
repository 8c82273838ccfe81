#!/bin/bash
# Generic GPU session runner (run through gpurun): each argument is one step "name:seconds:command".
# Every step runs under its own time limit with its output in gpurun_out/<name>.log. A step that
# passes (0) or only has failing tests (pytest exit 1) lets the next one start; anything else
# (fault, abort, segfault, time limit) ends the session there, so no GPU work follows a fault.
#   tools/gpu_steps.sh "cells:300:python -u -m pytest tests/test_cells_gpu.py -v" "bench:400:python bench.py"
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
done
