cd $GRAFT_REPO_ROOT
for g in 1 2 4; do
  timeout -k 10 300 python bench.py --groups $g --no-cpu-baseline --no-train --no-f32-compare --steps 100 > gpurun_out/grp$g.log 2>&1 || exit 1
done
