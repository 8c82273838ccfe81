/* Tuning and diagnostic switches of libgraphmarl_amd (not part of the reference-facing interface:
 * a binding of the reference's call sites never needs them; tools/ and the A/B benches do). Every
 * switch selects among kernel forms with the same arithmetic contract; the defaults are the
 * measured-best forms. */
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Tuning knob: tile configuration of gm_gemm_f32 (-1 = per-shape default; 0 = 128x128x32;
 * 1 = 128x256x16; 2 = 256x128x16 (LSTM: 256x128x16); 3 = 128x128x16; 4 = 128x128x16 at 4
 * blocks/CU); of gm_gemm_x3 (-1/0 = 128x128x16; 1 = 128x256x16 (LSTM: 128x128x32);
 * 2 = 128x128x32 (LSTM: 256x128x16)); 8..14 the LDS-DMA tiles of gm_gemm_x3's dense / readout
 * sources (8 = 256x256, 9 = 128x256 3 stages, 10 = 128x256, 12 = 128x128 2 blocks/CU, 13 = 128x128
 * of 64x64 waves, 14 = 128x256 of 64x128 waves). Process-wide. */
/* Weight-gradient kernel of gm_gemm_x3_wgrad (same arithmetic, diagnostics / A-B timing):
 * -1 (default) or 1 = transposed LDS reads (ds_read_b64_tr_b16) with 128 x 128 tiles, 2 = the same
 * with 128 x 256 tiles, 3 = 128 x 128 tiles on v_mfma_f32_16x16x32_f16, 0 = the dword-load
 * register-transpose form (tools/wgrad_bench.py). + 8: the same form with the blocks in dispatch order
 * (default: the tiles of a k chunk grouped on one XCD). */
int gm_gemm_set_wgrad(int32_t form);
int gm_gemm_set_tile(int32_t tile);
/* MFMA shape of the LDS-DMA split-f16 kernel (gm_gemm_x3's dense / readout tiles, gm_gemm_x3_head):
 * 2 (default) = v_mfma_f32_16x16x32_f16 everywhere, 1 = 16x16x32 except gm_gemm_x3_head (32x32x16),
 * 0 = v_mfma_f32_32x32x16_f16 everywhere. Same tiles and operand images; the summation order inside
 * an MFMA differs (fp32-order results either way). */
int gm_gemm_set_mfma(int32_t shape);
/* Input-gradient kernel of gm_gemm_x3_dgrad (same arithmetic and epilogue contract; A-B timing):
 * -1 (default) = per-shape choice, 0 = register-staged 128 x 128 tile (k_gemm3), 1 = LDS-DMA
 * 128 x 128 tile (4 waves, 2 blocks/CU), 2 = LDS-DMA 128 x 256 tile (8 waves). Process-wide. */
int gm_gemm_set_dgrad(int32_t form);
/* Arithmetic form the GEMM kernels were compiled with, e.g. "x3=lo12 diag=0": x3=lo12 = split-f16
 * with the A operand's low piece scaled by 2^12 in every kernel (the only form since round 5);
 * diag = 0 for the product build, 30 for the k-step stamp build (tools/stamp_bench.py). */
const char* gm_gemm_form(void);

#ifdef __cplusplus
}
#endif
