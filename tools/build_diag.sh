#!/bin/bash
# Diagnostic builds of the GEMM into graph-marl_amd/lib/diagN/ (timing only, wrong results).
# k_gemm3 (GM_DIAG 1: no A split, 2: no operand traffic in the k loop, 3: as 2 without barriers);
# k_gemm3g (7: prologue + epilogue only, 10: MFMAs only in the k loop). Results of the removed
# variants (no split / no DMA / no fragment reads / no barrier, 16x16x32 MFMAs): DESIGN.md 4a.
cd "$(dirname "$0")/../graph-marl_amd/csrc" || exit 1
make -s || exit 1
for d in ${DIAGS:-1 2 3}; do
  mkdir -p ../lib/diag$d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -DGM_DIAG=$d -c gm_gemm.hip -o ../lib/diag$d/gm_gemm.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/diag$d/libgraphmarl_amd.so ../lib/obj/gm_env.o \
      ../lib/obj/gm_netmon.o ../lib/obj/gm_simple.o ../lib/obj/gm_agents.o ../lib/obj/gm_replay.o ../lib/diag$d/gm_gemm.o || exit 1
  rm -f ../lib/diag$d/gm_gemm.o
done
