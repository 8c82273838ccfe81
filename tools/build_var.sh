#!/bin/bash
# Variant builds of gm_gemm.hip into graph-marl_amd/lib/<name>/ for GM_LIB A/B runs (tools/lib_ab.sh,
# tools/l1_ab.py):   tools/build_var.sh <name> "<extra hipcc flags>"   (run `make` first: links the other objects)
cd "$(dirname "$0")/../graph-marl_amd/csrc" || exit 1
d=../lib/$1
mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include $2 -c gm_gemm.hip -o $d/gm_gemm.o || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libgraphmarl_amd.so ../lib/obj/gm_env.o \
    ../lib/obj/gm_netmon.o ../lib/obj/gm_simple.o ../lib/obj/gm_agents.o ../lib/obj/gm_replay.o ../lib/obj/gm_build_info.o \
    $d/gm_gemm.o || exit 1
rm -f $d/gm_gemm.o
