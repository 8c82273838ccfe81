cd $GRAFT_REPO_ROOT
for d in "" diag1 diag2 diag3; do
  if [ -n "$d" ]; then export GM_LIB=$PWD/graph-marl_amd/lib/$d/libgraphmarl_amd.so; fi
  timeout -k 10 200 python tools/gemm_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
done
