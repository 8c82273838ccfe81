// gm_gemm.hip — fp32 MFMA GEMM with gathered A operands and fused epilogues for the
// NetMon / DQN layers (reference src/model.py:13-42 MLP, 119-125 Q_Net, 187-203 DQN,
// 206-229 SimpleAggregation, 379-382/491/543 LSTMCell, 582-631 readout).
//
//   y = epi( A @ W^T + b ),  A = [ src0 (k0 cols) | src1 (k1 cols) ]   (K concatenation)
//
// A sources (per row of A):
//   DENSE     row-major rows (any stride) — plain layer input, [x | h] of the LSTM, env obs
//   AGGREGATE Σ_{m ∈ {n} ∪ nbr(n)} h[m] (ascending node id; /count for mean) — the
//             message-passing aggregate is computed while the tile is loaded
//   READOUT   [h_final[v], h_prev[nbr(v,0)], h_prev[nbr(v,1)], h_prev[nbr(v,2)]] with
//             v = agent_node[row] — NetMon readout + agent gather (output_to_network_obs)
// Epilogues: bias (+ leaky_relu), or LSTM gates (weights packed so one 128-wide tile holds
// i,f,g,o of 32 hidden units): c' = σ(f)c + σ(i)tanh(g), h' = σ(o)tanh(c').
//
// Two arithmetic forms of the same kernel:
//   F32  exact fp32 (v_mfma_f32_32x32x2_f32 = fmaf chain per k), W as given (fp32 rows);
//   X3   split-f16 (v_mfma_f32_32x32x16_f16, 1/5.3 of the f32 MFMA cycles per k): every
//        operand is a sum of two f16 pieces, a = a_hi + a_lo (a_hi = f16(a), 22 significant
//        bits together), and a·w = a_hi·w_hi + a_hi·w_lo + a_lo·w_hi accumulated in fp32
//        (the dropped a_lo·w_lo term is ~2^-22 |a·w|). W is split once (gm_gemm_pack_x3)
//        after a power-of-two scale S keeps its pieces normal; A (fp32 in HBM) is split
//        while its tile is stored to LDS, its low piece scaled by 2^12 (a_lo' = f16((a -
//        a_hi)·2^12), normal down to |a| ~ 2^-15) and paired with w_hi·2^-12 (formed in
//        registers, exact), so all three products share one accumulator; the epilogue
//        multiplies by 1/S (exact). Operand tiles are prefetched two k steps ahead.
// All operand loads are
// unconditional buffer_load_dwordx4 (hardware bounds check returns 0: missing
// neighbours use an out-of-range offset, rows are clamped), so the load stream has
// no per-lane branches; the ragged K tail is zeroed in the LDS store of the last tile
// (wave-uniform branch). LDS is double-buffered: one barrier per 32-deep K tile while
// the next tile's loads are in flight in registers. Blocks are remapped so that tiles
// sharing A rows run on one XCD.
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>

// Arithmetic form (one form, no compile-time alternatives since round 5): the A operand's low split
// piece is scaled by 2^GM_LO_E (a_lo' = f16((a - a_hi) * 2^12): a normal f16 down to |a| ~ 2^-15) and
// paired with w_hi * 2^-12, in every kernel incl. the rollout's. Round 4's unscaled low piece on rollout
// operands (a denormal f16 below |a| = 2^-3, absolute error up to 2^-25 per element) measured 2.1e-5 of
// sum |a w| on rows of 2^-12 activations at the production tile vs 2.5e-7 scaled and 5e-7 for the exact
// f32 GEMM (tests/test_gemm_precision_gpu.py); it was removed with the other round-4 variant knobs.
#define GM_LO_E 12
#ifndef GM_DIAG
#define GM_DIAG 0  // 30: per-segment s_memtime stamps of the LDS-DMA k loop (diagnostic build, tools/stamp_bench.py)
#endif
#if GM_DIAG != 0 && GM_DIAG != 30
#error "GM_DIAG must be 0 or 30"
#endif
#include <string>

#include "../../include/graph_marl_amd.h"
#include "gm_amax.hpp"
#include "gm_act.hpp"

int gm_fail(int code, const std::string& msg);

#if GM_DIAG == 30
// diagnostic build 30: per-segment s_memtime stamps of the LDS-DMA k loop (tools/stamp_bench.py)
__device__ unsigned long long* g_stamps;
extern "C" int gm_diag_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BKMAX = 32;            // largest K tile of any configuration (host-side checks)
constexpr int OOB = 0x7ff00000;       // byte offset beyond any buffer: load returns 0
enum { EPI_BIAS = 0, EPI_LSTM = 1, EPI_HEAD = 2, EPI_DGRAD = 3, EPI_CHAIN = 5 };

struct ASrc {
    int mode;                 // GM_A_DENSE / GM_A_AGGREGATE / GM_A_READOUT
    const float* p0;          // dense rows | node rows h | h_final rows
    const float* p1;          // READOUT: h_prev rows
    long long ld0, ld1;       // row strides (floats)
    const int* nbr;           // [G][N][deg]
    const int* agent_node;    // READOUT: [G*R]
    int n_nodes, deg, mean, rows_per_graph, k, hidden;
    long long bytes0, bytes1; // buffer extents for the bounds check (DENSE: of the whole operand; the
                              // kernels address its rows relative to their block's first row)
    const float* scale;       // k_gemm3 DENSE source: power-of-two A scale (nullable)
    unsigned* amax;           // k_gemm3: max |A| float bits published here (nullable)
    const float* bias0;       // ROUTING_ENC: the folded encoder layer's bias (nullable) and activation
    int act0;
};

struct Epi {
    const float* bias;
    int act;                  // EPI_BIAS / EPI_HEAD: GM_ACT_* (gm_act.hpp)
    float* y;
    long long ldy;
    float* y2;                // EPI_LSTM: c' out
    long long ldy2;
    const float* c_in;        // EPI_LSTM: c in
    long long ldc;
    float* act_out;           // EPI_LSTM: [M][4H] activations i,f,g,o (optional)
    int hidden;
    const float* wq;          // EPI_HEAD: head weights [nq][ldwq], bias bq, out q [M][ldq]
    long long ldwq;
    const float* bq;
    int nq;
    float* q;
    int q_atomic;             // EPI_HEAD over several column blocks: each adds its partial Q (block 0 with bq) to q (zeroed)
    long long ldq;
    unsigned* range_flag;     // X3: set to 1 when an accumulator is not finite (host-mapped; nullable)
    int cell;                 // EPI_LSTM tiles: 0 LSTM (i, f, g, o), 1 GRU (r, z, n_x, n_h; c_in = h)
    // EPI_DGRAD (input gradient of a layer whose input went through leaky_relu): columns < split get
    // the leaky derivative of mask[row][col] (the layer's input, nullable = none), go to y, their
    // per-128-row-tile column sums to part[tile][col] (nullable) and their max |.| to gmax
    // (nullable); columns >= split go unchanged to y2[row][col - split]
    const unsigned* mbits;    // sign bits of the layer input: bit c % 32 of word [row][c / 32] = input > 0
    long long ldmb;           // words per row (0: one row for all)
    int split;
    float* part;
    unsigned* gmax;
    // EPI_BIAS: sign bits of y (> 0) out, one uint32 per 32 columns, ldsb words per row (nullable):
    // the leaky_relu derivative of the layer's output for the training backward, 1/32 of its bytes
    unsigned* sbits;
    long long ldsb;
    // EPI_CHAIN (the next MLP layer after this one, in the same block): packed split-f16 weights of that
    // layer (gm_gemm_pack_x3 layout, rows of ldw2 bytes), their 1/S, bias, act
    const _Float16* w2;
    long long ldw2;
    unsigned w2bytes;
    const float* wsi2;
    const float* b2;
    int act2;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
// buffer resource over the rows [r0, ..) of a row-major operand of `bytes` bytes: 32-bit offsets stay
// small whatever the operand's size; the extent is clamped below the OOB sentinel
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_rows(const float* p, long long ld, long long r0,
                                                           long long bytes) {
    long long rem = bytes - r0 * ld * 4;
    rem = rem < 0 ? 0 : (rem > 0x7fe00000LL ? 0x7fe00000LL : rem);
    return rsrc(p + r0 * ld, (unsigned)rem);
}
__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, int byte_off) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
// 16 B per lane from a buffer straight into LDS (lane-linear from the wave-uniform base);
// voff per lane, soff wave-uniform
// (kept out of the kernel bodies: with the builtin inside a __global__ template, hipcc's host
// pass silently drops the kernel's launch stub)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_base, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, soff, 0,
                                             0);
}
__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// LSTM gate nonlinearities on the hardware transcendentals (v_exp_f32 / v_rcp_f32, ~1 ulp
// each): sigma(x) = 1 / (1 + 2^(-x log2 e)), tanh(x) = 2 sigma(2x) - 1; absolute error
// < 1e-6, against the 1e-5 tolerance of the NetMon outputs (expf/divide/tanhf cost ~4x)
__device__ __forceinline__ float sigm(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigm(2.0f * x) - 1.0f; }

// (up ? b : a, up ? a : b) as a bitwise blend of the two values: written as selects of two elements of a
// local array, LLVM turns them into one dynamically indexed access, and the array is then lowered to
// 16-way v_cmp / v_cndmask chains per element (the Q-head reduction cost ~29 us per 81 920-row launch)
__device__ __forceinline__ void swap_if(bool up, float a, float b, float& mine, float& other) {
    const unsigned m = up ? ~0u : 0u, ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    mine = __builtin_bit_cast(float, (ua & ~m) | (ub & m));
    other = __builtin_bit_cast(float, (ub & ~m) | (ua & m));
}

// Layer activation in the epilogues with the common cases resolved at compile time: A = 0 none,
// 1 leaky_relu, -1 any GM_ACT_* at run time (a per-element branch tree: relu / elu / tanh / sigmoid
// only). act_dispatch calls f with A chosen from the wave-uniform act, so the default epilogues carry
// no activation branches per element.
template <int A>
__device__ __forceinline__ float act_t(float v, int act) {
    if constexpr (A == 0)
        return v;
    else if constexpr (A == 1)
        return v >= 0.f ? v : 0.01f * v;
    else
        return gm_act_fast(v, act);
}
template <typename F>
__device__ __forceinline__ void act_dispatch(int act, F&& f) {
    if (act == 1)
        f(std::integral_constant<int, 1>{});
    else if (act == 0)
        f(std::integral_constant<int, 0>{});
    else
        f(std::integral_constant<int, -1>{});
}

// Range guard of the split-f16 form: an A element whose pieces leave the f16 range (|a| >=
// 65520, or a low piece (a - a_hi) * 2^12 >= 65520, possible from |a| >= 2^15 where the low piece
// is scaled: training operands and the register-staged kernels) makes every
// accumulator of its row inf or NaN, whatever the epilogue does with it afterwards (the LSTM
// gates would squash inf to a finite h). One wave-wide vote per tile; lane 0 of a wave that saw
// a non-finite accumulator stores 1 into the host-mapped status word (gm_gemm_range_status).
template <int TM, int TN>
__device__ __forceinline__ void range_guard(const floatx16 (&acc)[TM][TN], unsigned* flag, int lane) {
    if (!flag) return;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) bad |= !__builtin_isfinite(acc[i][j][r]);
    if (__ballot(bad) != 0ull && lane == 0) *reinterpret_cast<volatile unsigned*>(flag) = 1u;
}
// GM_LO_E: the low piece of the split is scaled by 2^12 (a normal f16 down to |a| ~ 2^-15); the w_hi
// factor 2^-12 restores it
constexpr float LO_S = (float)(1 << GM_LO_E);
// routing-encoder (ROUTING_ENC) source: node-obs rows 4N + 8 up to N = 50 (BASELINE config 4's largest graphs)
#define GM_RENC_ROWS 208
// a = hi + 2^-12 lo with hi = f16(a) (RNE), lo = f16((a - hi) * 2^12)
__device__ __forceinline__ void split4(float4 v, half4& hi, half4& lo) {
    const floatx4 a = {v.x, v.y, v.z, v.w};
    hi = __builtin_convertvector(a, half4);
    lo = __builtin_convertvector((a - __builtin_convertvector(hi, floatx4)) * LO_S, half4);
}

// lo = f16(fma(hi, -4096, X)) of a pair (hp = the two f16 hi, X = 4096 x): exact in f32, one rounding
// (compiler-visible f32: the round-3 inline-asm v_fma_mix form raced an MFMA's read of the lo register,
// DESIGN.md §4a "Hazard")
__device__ __forceinline__ unsigned split_lo_pair(unsigned hp, float X0, float X1) {
    constexpr float m4096 = -(float)(1 << GM_LO_E);
    typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
    const half2_t h = __builtin_bit_cast(half2_t, hp);
    const half2_t l = {(_Float16)__builtin_fmaf((float)h[0], m4096, X0), (_Float16)__builtin_fmaf((float)h[1], m4096, X1)};
    return __builtin_bit_cast(unsigned, l);
}

// The same split for 8 floats: hi = cvt_pk (RNE), X = 4096 x (exact), lo = f16(fma(hi, -4096, X)) =
// f16(4096 (x - hi)) (the fma is exact in f32, so one rounding, RNE: the same bits as split4;
// split_lo_pair).
// The split of x * 2^e (e = 0, or a device power-of-two operand scale) with 4096 x by v_ldexp_f32 instead
// of v_pk_mul_f32 (packed f32 VALU beside MFMAs costs extra issue cycles: rollout +0.9 %)
__device__ __forceinline__ void split8(floatx4 x0, floatx4 x1, half8& hi, half8& lo, int e = 0) {
    typedef float floatx2 __attribute__((ext_vector_type(2)));
    typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
    unsigned hp[4], lp[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        floatx2 x = q < 2 ? floatx2{x0[2 * q], x0[2 * q + 1]} : floatx2{x1[2 * q - 4], x1[2 * q - 3]};
        const floatx2 X = {__builtin_ldexpf(x[0], e + GM_LO_E), __builtin_ldexpf(x[1], e + GM_LO_E)};
        if (e != 0) x = floatx2{__builtin_ldexpf(x[0], e), __builtin_ldexpf(x[1], e)};
        hp[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(x, half2_t));
        lp[q] = split_lo_pair(hp[q], X[0], X[1]);
    }
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    hi = __builtin_bit_cast(half8, u32x4_t{hp[0], hp[1], hp[2], hp[3]});
    lo = __builtin_bit_cast(half8, u32x4_t{lp[0], lp[1], lp[2], lp[3]});
}

// split4 of v * 2^e (a device power-of-two operand scale) without packed f32 VALU: hi = f16(ldexp(v, e))
// (cvt_pk), lo = f16(fma(hi, -4096, ldexp(v, e + 12))) by v_fma_mix{lo,hi}_f16; the same bits as
// split4(v * 2^e) while v * 2^e is finite and normal
__device__ __forceinline__ void split4e(float4 v, int e, half4& hi, half4& lo) {
    typedef float floatx2 __attribute__((ext_vector_type(2)));
    typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
    const float x[4] = {v.x, v.y, v.z, v.w};
    unsigned hp[2], lp[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const floatx2 xs = {__builtin_ldexpf(x[2 * q], e), __builtin_ldexpf(x[2 * q + 1], e)};
        hp[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(xs, half2_t));
        const float X0 = __builtin_ldexpf(x[2 * q], e + GM_LO_E), X1 = __builtin_ldexpf(x[2 * q + 1], e + GM_LO_E);
        lp[q] = split_lo_pair(hp[q], X0, X1);
    }
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    hi = __builtin_bit_cast(half4, u32x2_t{hp[0], hp[1]});
    lo = __builtin_bit_cast(half4, u32x2_t{lp[0], lp[1]});
}

// LSTM epilogue input c, loaded into registers before the k loop (the loads retire behind
// the MFMAs instead of one dependent HBM round trip per output row in the epilogue)
template <int TM, int EPI>
struct CIn {};
template <int TM>
struct CIn<TM, EPI_LSTM> {
    float v[TM][16];
};
template <int TM, int EPI>
__device__ __forceinline__ void cin_load(CIn<TM, EPI>& c, const Epi& ep, int wm0, int wn0, int M, int lane) {
    if constexpr (EPI == EPI_LSTM) {
        const int h = lane >> 5, unit = (wn0 >> 2) + (lane & 31);
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = wm0 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
                c.v[i][r] = (row < M && unit < ep.hidden) ? ep.c_in[(long long)row * ep.ldc + unit] : 0.f;
            }
    }
}

// Epilogue of both forms. C/D map of the 32x32 MFMA tiles: col = lane & 31, row =
// (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); wave tile origin (wm0, wn0).
template <int TM, int TN, int EPI, int A = -1>
__device__ __forceinline__ void epilogue(floatx16 (&acc)[TM][TN], const Epi& ep, int wm0, int wn0, int M, int N,
                                         int lane, const CIn<TM, EPI>& cin) {
    const int h = lane >> 5, l32 = lane & 31;
    if constexpr (EPI == EPI_BIAS) {
        // buffer stores on a resource over the wave's rows [wm0, M) (rows past M dropped by its extent), columns
        // past N at the OOB offset: no per-element branches or 64-bit addresses
        const __amdgpu_buffer_rsrc_t rs = rsrc_rows(ep.y + wn0, ep.ldy, wm0, (long long)M * ep.ldy * 4);
        const unsigned ld4 = (unsigned)ep.ldy * 4u;
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int col = wn0 + j * 32 + l32;
            const float bv = (ep.bias && col < N) ? ep.bias[col] : 0.f;
            const unsigned vb = col < N ? 4u * h * ld4 + 4u * (j * 32 + l32) : (unsigned)OOB;
#pragma unroll
            for (int i = 0; i < TM; i++) {
                const int rb0 = wm0 + i * 32 + 4 * h;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int row = rb0 + (r & 3) + 8 * (r >> 2);
                    float v = acc[i][j][r] + bv;
                    v = act_t<A>(v, ep.act);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs,
                                                          (int)(vb + (unsigned)(i * 32 + (r & 3) + 8 * (r >> 2)) * ld4), 0, 0);
                    if (ep.sbits) {  // lanes 0-31 / 32-63: 32 columns of rows row(h = 0) / row(h = 1)
                        const unsigned long long b = __ballot(v > 0.f && col < N);
                        if (l32 == 0 && row < M && wn0 + j * 32 < N)
                            ep.sbits[(long long)row * ep.ldsb + ((wn0 + j * 32) >> 5)] = (unsigned)(b >> (32 * h));
                    }
                }
            }
        }
    } else {  // EPI_LSTM: TN == 4 gate tiles (i, f, g, o) of 32 hidden units
        const int H = ep.hidden;
        const int unit = (wn0 >> 2) + l32;
        float bgate[4];
#pragma unroll
        for (int g = 0; g < 4; g++) bgate[g] = ep.bias ? ep.bias[wn0 + g * 32 + l32] : 0.f;
        // buffer stores on resources over the wave's rows [wm0, M) (rows past M dropped by their extent), units
        // past H at the OOB offset: no per-element branches or 64-bit addresses
        const bool in = unit < H;
        const unsigned ly = (unsigned)ep.ldy * 4u, lc = (unsigned)ep.ldy2 * 4u, la = (unsigned)H * 16u;
        const __amdgpu_buffer_rsrc_t ry = rsrc_rows(ep.y + (wn0 >> 2), ep.ldy, wm0, (long long)M * ep.ldy * 4);
        const __amdgpu_buffer_rsrc_t rc =
            rsrc_rows(ep.y2 ? ep.y2 + (wn0 >> 2) : ep.y, ep.ldy2, wm0, ep.y2 ? (long long)M * ep.ldy2 * 4 : 0);
        const __amdgpu_buffer_rsrc_t ra =
            rsrc_rows(ep.act_out ? ep.act_out + (wn0 >> 2) : ep.y, 4LL * H, wm0, ep.act_out ? (long long)M * H * 16 : 0);
        const unsigned vy = in ? 4u * h * ly + 4u * l32 : (unsigned)OOB, vc = in ? 4u * h * lc + 4u * l32 : (unsigned)OOB;
        const unsigned va = in ? 4u * h * la + 4u * l32 : (unsigned)OOB;
        auto st = [](float v, __amdgpu_buffer_rsrc_t rr, unsigned off) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rr, (int)off, 0, 0);
        };
#pragma unroll
        for (int i = 0; i < TM; i++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const unsigned rl = (unsigned)(i * 32 + (r & 3) + 8 * (r >> 2));  // row - wm0 - 4 h
                if (ep.cell == 1) {  // GRU (torch.nn.GRUCell): the 4th tile is W_hn h, kept apart for r * (.)
                    const float rg = sigm(acc[i][0][r] + bgate[0]);
                    const float zg = sigm(acc[i][1][r] + bgate[1]);
                    const float ng = tanh_fast(acc[i][2][r] + bgate[2] + rg * (acc[i][3][r] + bgate[3]));
                    st((1.f - zg) * ng + zg * cin.v[i][r], ry, vy + rl * ly);
                    continue;
                }
                float gi = sigm(acc[i][0][r] + bgate[0]);
                float gf = sigm(acc[i][1][r] + bgate[1]);
                float gg = tanh_fast(acc[i][2][r] + bgate[2]);
                float go = sigm(acc[i][3][r] + bgate[3]);
                float cn = gf * cin.v[i][r] + gi * gg;
                float hn = go * tanh_fast(cn);
                st(hn, ry, vy + rl * ly);
                st(cn, rc, vc + rl * lc);
                if (ep.act_out) {
                    const unsigned ao = va + rl * la;
                    st(gi, ra, ao);
                    st(gf, ra, ao + 4u * H);
                    st(gg, ra, ao + 8u * H);
                    st(go, ra, ao + 12u * H);
                }
            }
        }
    }
}

// EPI_HEAD (block spans all N columns, n0 = 0): y = act(acc + b) stays in registers and
// q[row][a] = bq[a] + sum_col y[row][col] wq[a][col] (a < nq <= 4). Per lane, the partial
// dot products of its TN columns for its 16 rows x 4 heads (64 values) are reduce-scattered
// over the 32 lanes of its half (xor 16..1: 62 shuffles, lane l ends with entries 2l, 2l+1
// of row r = l >> 1, heads 2 (l & 1) + t); the WGN column waves are summed through LDS.
template <int TM, int TN, int WGN, int BM, int A = -1>
__device__ __forceinline__ void head_epilogue(floatx16 (&acc)[TM][TN], const Epi& ep, char* lds, int m0, int wr,
                                              int wc, int M, int N, int lane, int tid) {
    const int h = lane >> 5, l32 = lane & 31;
    float bv[TN], wqv[TN][4];
#pragma unroll
    for (int j = 0; j < TN; j++) {
        const int col = wc * TN * 32 + j * 32 + l32;
        bv[j] = (ep.bias && col < N) ? ep.bias[col] : 0.f;
#pragma unroll
        for (int a = 0; a < 4; a++) wqv[j][a] = (col < N && a < ep.nq) ? ep.wq[a * ep.ldwq + col] : 0.f;
    }
    float* qp = reinterpret_cast<float*>(lds);  // [WGN][BM][4]
    float red[TM][2];
#pragma unroll
    for (int i = 0; i < TM; i++) {
        float x[64];
#pragma unroll
        for (int e = 0; e < 64; e++) x[e] = 0.f;
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int col = wc * TN * 32 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                float y = acc[i][j][r] + bv[j];
                y = act_t<A>(y, ep.act);
                if (ep.y) {
                    const int row = m0 + wr * TM * 32 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
                    if (row < M && col < N) ep.y[(long long)row * ep.ldy + col] = y;
                }
#pragma unroll
                for (int a = 0; a < 4; a++) x[r * 4 + a] = fmaf(y, wqv[j][a], x[r * 4 + a]);
            }
        }
#pragma unroll
        for (int mask = 16, n = 32; mask >= 1; mask >>= 1, n >>= 1) {
            const bool up = (l32 & mask) != 0;
#pragma unroll
            for (int k = 0; k < n; k++) {
                float mine, other;
                swap_if(up, x[k], x[n + k], mine, other);
                x[k] = mine + __shfl_xor(other, mask);
            }
        }
        red[i][0] = x[0];
        red[i][1] = x[1];
    }
    __syncthreads();  // every wave is done with the operand stages
#pragma unroll
    for (int i = 0; i < TM; i++) {
        const int r = l32 >> 1;
        const int rl = wr * TM * 32 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
        const int a = 2 * (l32 & 1);
        qp[(wc * BM + rl) * 4 + a] = red[i][0];
        qp[(wc * BM + rl) * 4 + a + 1] = red[i][1];
    }
    __syncthreads();
    for (int e = tid; e < BM * 4; e += WGN * (BM / TM / 32) * 64) {
        const int rl = e >> 2, a = e & 3, row = m0 + rl;
        if (a >= ep.nq || row >= M) continue;
        float v = ep.bq ? ep.bq[a] : 0.f;
#pragma unroll
        for (int w = 0; w < WGN; w++) v += qp[(w * BM + rl) * 4 + a];
        ep.q[(long long)row * ep.ldq + a] = v;
    }
}

// XCD-aware tile order: consecutive tiles (sharing A rows) land on one XCD
__device__ __forceinline__ int xcd_remap(int bid, int T) {
    const int q = T / 8, r = T % 8, xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int WGM, int WGN, int TM, int TN, int BK_>
struct Cfg {
    static constexpr int BK = BK_;
    static constexpr int LDP = BK + 4;  // padded LDS row (floats): conflict-free ds_read_b128
    static constexpr int KH = BK / 2;   // k per lane half: MFMA k pair {s, KH + s}
    static constexpr int BM = WGM * TM * 32;
    static constexpr int BN = WGN * TN * 32;
    static constexpr int THREADS = WGM * WGN * 64;
    static constexpr int AQ = BM * BK / 4 / THREADS;  // float4 per thread per A tile
    static constexpr int BQ = BN * BK / 4 / THREADS;
    static constexpr int RSTEP = THREADS / (BK / 4);   // rows between a thread's A rows
};

template <int WGM, int WGN, int TM, int TN, int BK_, int AMODE, int EPI, int OCC>
__global__ __launch_bounds__(WGM* WGN * 64, OCC) void k_gemm(ASrc a0, ASrc a1, const float* __restrict__ w,
                                                            long long ldw, unsigned wbytes, int M, int N, int K,
                                                            Epi ep) {
    using C = Cfg<WGM, WGN, TM, TN, BK_>;
    constexpr int BK = C::BK, LDP = C::LDP, KH = C::KH;
    __shared__ __attribute__((aligned(16))) float As[2][C::BM * LDP];
    __shared__ __attribute__((aligned(16))) float Bs[2][C::BN * LDP];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WGN, wc = wave % WGN;
    const int nM = (M + C::BM - 1) / C::BM, nN = (N + C::BN - 1) / C::BN;
    const int T = nM * nN;
    const int bid = xcd_remap(blockIdx.x, T);
    const int m0 = (bid / nN) * C::BM, n0 = (bid % nN) * C::BN;

    // ---- per-thread A rows (fixed over K) and their source rows ----
    const int c4 = tid % (BK / 4);
    const int rbase = tid / (BK / 4);
    int rowoff0[C::AQ], rowoff1[C::AQ];
    int src[C::AQ][4];  // AGGREGATE: member rows; READOUT: segment source rows (-1 = none)
    // READOUT: byte offsets of the 4 segment rows in separate register arrays (one array
    // indexed by the runtime segment would be demoted to scratch)
    int ro0[C::AQ], ro1[C::AQ], ro2[C::AQ], ro3[C::AQ];
    float scale[C::AQ];
#pragma unroll
    for (int q = 0; q < C::AQ; q++) {
        int row = min(m0 + rbase + q * C::RSTEP, M - 1);
        rowoff0[q] = AMODE == GM_A_DENSE ? (int)((row - m0) * a0.ld0) : (int)(row * a0.ld0);
        rowoff1[q] = (int)((row - m0) * a1.ld0);
        scale[q] = 1.0f;
        if (AMODE == GM_A_AGGREGATE) {
            const int g = row / a0.n_nodes, n = row - g * a0.n_nodes;
            const int* nb = a0.nbr + (size_t)row * a0.deg;
            int cnt = 0, self_done = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) src[q][j] = -1;
            for (int j = 0; j < a0.deg; j++) {
                int v = nb[j];
                if (v < 0) continue;
                if (!self_done && n < v) { src[q][cnt++] = g * a0.n_nodes + n; self_done = 1; }
                src[q][cnt++] = g * a0.n_nodes + v;
            }
            if (!self_done) src[q][cnt++] = g * a0.n_nodes + n;
            if (a0.mean) scale[q] = 1.0f / (float)cnt;
        } else if (AMODE == GM_A_READOUT) {
            const int g = row / a0.rows_per_graph;
            const int v = a0.agent_node[row];
            const int* nb = a0.nbr + ((size_t)g * a0.n_nodes + v) * a0.deg;
            src[q][0] = g * a0.n_nodes + v;
#pragma unroll
            for (int j = 1; j < 4; j++) {
                int m = j - 1 < a0.deg ? nb[j - 1] : -1;
                src[q][j] = m >= 0 ? g * a0.n_nodes + m : -1;
            }
            ro0[q] = (int)(src[q][0] * a0.ld0) * 4;
            ro1[q] = src[q][1] >= 0 ? (int)(src[q][1] * a0.ld1) * 4 : OOB;
            ro2[q] = src[q][2] >= 0 ? (int)(src[q][2] * a0.ld1) * 4 : OOB;
            ro3[q] = src[q][3] >= 0 ? (int)(src[q][3] * a0.ld1) * 4 : OOB;
        }
    }
    int woff[C::BQ];
#pragma unroll
    for (int q = 0; q < C::BQ; q++) woff[q] = (int)(min(n0 + rbase + q * C::RSTEP, N - 1) * ldw);

    const __amdgpu_buffer_rsrc_t r0a =
        AMODE == GM_A_DENSE ? rsrc_rows(a0.p0, a0.ld0, m0, a0.bytes0) : rsrc(a0.p0, (unsigned)a0.bytes0);
    const __amdgpu_buffer_rsrc_t r0b = rsrc(a0.p1 ? a0.p1 : a0.p0, (unsigned)(a0.p1 ? a0.bytes1 : a0.bytes0));
    const __amdgpu_buffer_rsrc_t r1 = a1.p0 ? rsrc_rows(a1.p0, a1.ld0, m0, a1.bytes0) : rsrc(a0.p0, 0u);
    const __amdgpu_buffer_rsrc_t rw = rsrc(w, wbytes);

    float4 ra[C::AQ], rb[C::BQ];
    auto gload = [&](int k0) {
        if (k0 < a0.k) {
            const int kl = k0 + 4 * c4;
            if (AMODE == GM_A_DENSE) {
#pragma unroll
                for (int q = 0; q < C::AQ; q++) ra[q] = bload(r0a, (rowoff0[q] + kl) * 4);
            } else if (AMODE == GM_A_AGGREGATE) {
                const long long ld = a0.ld0;
#pragma unroll
                for (int q = 0; q < C::AQ; q++) {
                    float4 v = bload(r0a, src[q][0] >= 0 ? (int)(src[q][0] * ld + kl) * 4 : OOB);
#pragma unroll
                    for (int j = 1; j < 4; j++)
                        v = f4add(v, bload(r0a, src[q][j] >= 0 ? (int)(src[q][j] * ld + kl) * 4 : OOB));
                    ra[q] = make_float4(v.x * scale[q], v.y * scale[q], v.z * scale[q], v.w * scale[q]);
                }
            } else {  // READOUT: the K tile lies inside one H-wide segment
                const int seg = k0 / a0.hidden, ko4 = (kl - seg * a0.hidden) * 4;
                if (seg == 0) {
#pragma unroll
                    for (int q = 0; q < C::AQ; q++) ra[q] = bload(r0a, ro0[q] + ko4);
                } else if (seg == 1) {
#pragma unroll
                    for (int q = 0; q < C::AQ; q++) ra[q] = bload(r0b, ro1[q] == OOB ? OOB : ro1[q] + ko4);
                } else if (seg == 2) {
#pragma unroll
                    for (int q = 0; q < C::AQ; q++) ra[q] = bload(r0b, ro2[q] == OOB ? OOB : ro2[q] + ko4);
                } else {
#pragma unroll
                    for (int q = 0; q < C::AQ; q++) ra[q] = bload(r0b, ro3[q] == OOB ? OOB : ro3[q] + ko4);
                }
            }
        } else {
            const int kl = k0 - a0.k + 4 * c4;
#pragma unroll
            for (int q = 0; q < C::AQ; q++) ra[q] = bload(r1, (rowoff1[q] + kl) * 4);
        }
#pragma unroll
        for (int q = 0; q < C::BQ; q++) rb[q] = bload(rw, (woff[q] + k0 + 4 * c4) * 4);
    };
    auto lstore = [&](int buf, int k0) {
        // zero the columns past the end of the current source on its last (ragged) tile
        const int kend = k0 < a0.k ? a0.k : K;
        if (k0 + BK > kend) {
            const int kk = k0 + 4 * c4;
#pragma unroll
            for (int q = 0; q < C::AQ; q++) {
                if (kk + 0 >= kend) ra[q].x = 0.f;
                if (kk + 1 >= kend) ra[q].y = 0.f;
                if (kk + 2 >= kend) ra[q].z = 0.f;
                if (kk + 3 >= kend) ra[q].w = 0.f;
            }
#pragma unroll
            for (int q = 0; q < C::BQ; q++) {
                if (kk + 0 >= K) rb[q].x = 0.f;
                if (kk + 1 >= K) rb[q].y = 0.f;
                if (kk + 2 >= K) rb[q].z = 0.f;
                if (kk + 3 >= K) rb[q].w = 0.f;
            }
        }
#pragma unroll
        for (int q = 0; q < C::AQ; q++)
            *reinterpret_cast<float4*>(&As[buf][(rbase + q * C::RSTEP) * LDP + 4 * c4]) = ra[q];
#pragma unroll
        for (int q = 0; q < C::BQ; q++)
            *reinterpret_cast<float4*>(&Bs[buf][(rbase + q * C::RSTEP) * LDP + 4 * c4]) = rb[q];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

    const int h = lane >> 5, l32 = lane & 31;
    const int nk = (K + BK - 1) / BK;
    gload(0);
    lstore(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * BK);
        const float* as = As[cur];
        const float* bs = Bs[cur];
#pragma unroll
        for (int s4 = 0; s4 < KH / 4; s4++) {
            float4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; i++)
                af[i] = *reinterpret_cast<const float4*>(&as[(wr * TM * 32 + i * 32 + l32) * LDP + h * KH + 4 * s4]);
#pragma unroll
            for (int j = 0; j < TN; j++)
                bf[j] = *reinterpret_cast<const float4*>(&bs[(wc * TN * 32 + j * 32 + l32) * LDP + h * KH + 4 * s4]);
#pragma unroll
            for (int e = 0; e < 4; e++)
#pragma unroll
                for (int i = 0; i < TM; i++)
#pragma unroll
                    for (int j = 0; j < TN; j++) {
                        float a = e == 0 ? af[i].x : e == 1 ? af[i].y : e == 2 ? af[i].z : af[i].w;
                        float b = e == 0 ? bf[j].x : e == 1 ? bf[j].y : e == 2 ? bf[j].z : bf[j].w;
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i][j], 0, 0, 0);
                    }
        }
        if (kt + 1 < nk) lstore(cur ^ 1, (kt + 1) * BK);
        __syncthreads();
    }

    CIn<TM, EPI> cin;
    cin_load<TM, EPI>(cin, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, lane);
    if constexpr (EPI == EPI_BIAS)
        act_dispatch(ep.act, [&](auto A) {
            epilogue<TM, TN, EPI, decltype(A)::value>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane,
                                                      cin);
        });
    else
        epilogue<TM, TN, EPI>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane, cin);
}

// EPI_DGRAD epilogue of k_gemm3 (32x32 C layout): the leaky_relu derivative of the layer input
// (sign bit set ? 1 : 0.01, the reference MLP's F.leaky_relu) applied to the input gradient, per
// 128-row tile column sums (bias gradient partials: lane sums of its rows, the two lane halves,
// then the WGM row waves through LDS, a fixed order) and max |g| (the next gradient GEMMs' operand
// scale). red: >= WGM * WGN * TN * 32 floats of LDS no longer used by the k loop.
template <int WGM, int WGN, int TM, int TN, bool STAGED = false>
__device__ __forceinline__ void dgrad_epilogue(floatx16 (&acc)[TM][TN], const Epi& ep, float* red, int m0, int n0,
                                               int wr, int wc, int M, int N, int lane) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = m0 + wr * TM * 32, wn0 = n0 + wc * TN * 32;
    constexpr int BM = WGM * TM * 32, BN = WGN * TN * 32, WPR = BN / 32;
    // the tile's sign words (BM rows x BN / 32) staged in LDS with coalesced loads (all ones = no
    // derivative where there is no mask or the column lies past split)
    unsigned* smb = reinterpret_cast<unsigned*>(red + WGM * BN);
    if (ep.mbits && !STAGED) {
        for (int e = threadIdx.x; e < BM * WPR; e += WGM * WGN * 64) {
            const int r = e / WPR, w = e - r * WPR;
            const int row = m0 + r, col0 = n0 + 32 * w;
            smb[e] = (row < M && col0 < ep.split) ? ep.mbits[(long long)row * ep.ldmb + (col0 >> 5)] : ~0u;
        }
        __syncthreads();
    }
    float mx = 0.f;
    float cs[TN];
#pragma unroll
    for (int j = 0; j < TN; j++) {
        const int col = wn0 + j * 32 + l32;
        const bool lo = col < ep.split;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = wm0 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
                if (row >= M || col >= N) continue;
                float v = acc[i][j][r];
                if (lo) {
                    // torch's leaky_relu backward: input > 0 ? g : 0.01 g (leaky(z) > 0 iff z > 0); the
                    // 32 lanes of a half read one sign word (a broadcast load)
                    if (ep.mbits && !((smb[(row - m0) * WPR + ((col - n0) >> 5)] >> l32) & 1u)) v *= 0.01f;
                    ep.y[(long long)row * ep.ldy + col] = v;
                    s += v;
                    mx = fmaxf(mx, fabsf(v));
                } else {
                    ep.y2[(long long)row * ep.ldy2 + col - ep.split] = v;
                }
            }
        cs[j] = s + __shfl_xor(s, 32);
    }
    if (ep.gmax) {
        mx = gm_wave_max(mx);
        if (lane == 0) gm_amax_publish(ep.gmax, mx);
    }
    if (ep.part) {
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; j++) red[wr * BN + wc * TN * 32 + j * 32 + l32] = cs[j];
        }
        __syncthreads();
        if (wr == 0 && h == 0) {
#pragma unroll
            for (int j = 0; j < TN; j++) {
                const int c = wc * TN * 32 + j * 32 + l32, col = n0 + c;
                float s = red[c];
#pragma unroll
                for (int w = 1; w < WGM; w++) s += red[w * BN + c];
                if (col < ep.split && col < N) ep.part[(long long)(m0 / (WGM * TM * 32)) * ep.split + col] = s;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// X3 (split-f16) kernel. LDS row image of A and B tiles (4*BK + 16 bytes, conflict-free
// ds_read_b128 on the 32 rows of an MFMA operand): per 16-deep k block s, bytes
// [64s, 64s+32) = 16 hi halves, [64s+32, 64s+64) = 16 lo halves. Packed weights
// (gm_gemm_pack_x3) have this block layout in HBM, so B tiles are plain copies; A tiles
// are split while stored. Operand tiles are loaded two k steps ahead into two register
// sets (the loop is unrolled by two so each set has fixed registers and the waits stay
// counted); AGGREGATE keeps its 4 member rows raw until the store, so no load result is
// consumed before the step that stores it.
template <int WGM, int WGN, int TM, int TN, int BK, int AMODE, int EPI, int OCC>
__global__ __launch_bounds__(WGM* WGN * 64, OCC) void k_gemm3(ASrc a0, ASrc a1, const _Float16* __restrict__ w,
                                                             long long ldw, unsigned wbytes, int M, int N, int K,
                                                             Epi ep, const float* __restrict__ wscale_inv) {
    constexpr int BM = WGM * TM * 32, BN = WGN * TN * 32, THREADS = WGM * WGN * 64;
    constexpr int ROWB = 4 * BK + 16;          // LDS row bytes (A and B)
    constexpr int CPR = BK / 4;                // 16-byte chunks per tile row (A: float4; B: 8 halves)
    constexpr int RSTEP = THREADS / CPR;       // rows between a thread's rows
    constexpr int AQ = BM / RSTEP, BQ = BN / RSTEP;
    constexpr int NR = AMODE == GM_A_AGGREGATE ? 4 : 1;  // raw float4 per A chunk
    static_assert(BK % 16 == 0 && BM % RSTEP == 0 && BN % RSTEP == 0, "tile shape");
    __shared__ __attribute__((aligned(16))) char As[2][BM * ROWB];
    __shared__ __attribute__((aligned(16))) char Bs[2][BN * ROWB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WGN, wc = wave % WGN;
    const int nM = (M + BM - 1) / BM, nN = (N + BN - 1) / BN;
    const int bid = xcd_remap(blockIdx.x, nM * nN);
    const int m0 = (bid / nN) * BM, n0 = (bid % nN) * BN;

    // ---- per-thread source byte offsets (fixed over K) ----
    const int c4 = tid % CPR, rbase = tid / CPR;
    // rows permuted inside aligned 8-row blocks (a row's CPR chunks stay on consecutive
    // lanes, so every load instruction touches the same lines) so that the LDS stores meet distinct banks
    // at the 4 BK + 16 byte row stride: A (ds_write_b64, 16-lane groups, CPR 4) rows {0,2,4,6} / {1,3,5,7}
    // per group, (CPR 8: 2 rows per group, offset 2); B (ds_write_b128, 8-lane groups, CPR 4) rows {r, r+4}
    const int j8 = rbase & 7;
    const int rba = (rbase & ~7) | (CPR == 4 ? ((j8 & 3) << 1) | (j8 >> 2) : CPR == 8 ? (j8 & 4) | ((j8 & 1) << 1) | ((j8 >> 1) & 1) : j8);
    const int rbb = CPR != 4 ? rbase : (rbase & ~7) | ((j8 & 1) << 2) | (j8 >> 1);
    int off1[AQ];       // src1 row
    int so[AQ][4];      // DENSE: so[q][0] row; AGGREGATE: member rows; READOUT: segment rows (OOB = none)
    float scale[AQ];
#pragma unroll
    for (int q = 0; q < AQ; q++) {
        const int row = min(m0 + rba + q * RSTEP, M - 1);
        off1[q] = (int)((row - m0) * a1.ld0) * 4;
        scale[q] = 1.0f;
#pragma unroll
        for (int j = 0; j < 4; j++) so[q][j] = OOB;
        if (AMODE == GM_A_DENSE) {
            so[q][0] = (int)((row - m0) * a0.ld0) * 4;
        } else if (AMODE == GM_A_AGGREGATE) {
            // members of (I + A) row n in ascending node id (SimpleAggregation's bmm order)
            const int g = row / a0.n_nodes, n = row - g * a0.n_nodes;
            const int* nb = a0.nbr + (size_t)row * a0.deg;
            int mem[4] = {-1, -1, -1, -1};
            int cnt = 0, self_done = 0;
            for (int j = 0; j < a0.deg; j++) {
                const int v = nb[j];
                if (v < 0) continue;
                if (!self_done && n < v) { mem[cnt++] = n; self_done = 1; }
                mem[cnt++] = v;
            }
            if (!self_done) mem[cnt++] = n;
#pragma unroll
            for (int j = 0; j < 4; j++) so[q][j] = mem[j] >= 0 ? (int)((g * a0.n_nodes + mem[j]) * a0.ld0) * 4 : OOB;
            if (a0.mean) scale[q] = 1.0f / (float)cnt;
        } else {  // READOUT: [h_final[v] | h_prev[nbr(v, 0..2)]], v = agent_node[row]
            const int g = row / a0.rows_per_graph;
            const int v = a0.agent_node[row];
            const int* nb = a0.nbr + ((size_t)g * a0.n_nodes + v) * a0.deg;
            so[q][0] = (int)((g * a0.n_nodes + v) * a0.ld0) * 4;
#pragma unroll
            for (int j = 1; j < 4; j++) {
                const int m = j - 1 < a0.deg ? nb[j - 1] : -1;
                so[q][j] = m >= 0 ? (int)((g * a0.n_nodes + m) * a0.ld1) * 4 : OOB;
            }
        }
    }
    int woff[BQ];
#pragma unroll
    for (int q = 0; q < BQ; q++) woff[q] = (int)(min(n0 + rbb + q * RSTEP, N - 1) * ldw) + 16 * c4;

    const __amdgpu_buffer_rsrc_t r0a =
        AMODE == GM_A_DENSE ? rsrc_rows(a0.p0, a0.ld0, m0, a0.bytes0) : rsrc(a0.p0, (unsigned)a0.bytes0);
    const __amdgpu_buffer_rsrc_t r0b = rsrc(a0.p1 ? a0.p1 : a0.p0, (unsigned)(a0.p1 ? a0.bytes1 : a0.bytes0));
    const __amdgpu_buffer_rsrc_t r1 = a1.p0 ? rsrc_rows(a1.p0, a1.ld0, m0, a1.bytes0) : rsrc(a0.p0, 0u);
    const __amdgpu_buffer_rsrc_t rw = rsrc(reinterpret_cast<const float*>(w), wbytes);

    float4 ra[2][AQ][NR], rb[2][BQ];
    auto gload = [&](auto SET, int k0) {
        constexpr int S = decltype(SET)::value;
        if (k0 < a0.k) {
            const int kb = (k0 + 4 * c4) * 4;
            if (AMODE == GM_A_DENSE) {
#pragma unroll
                for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r0a, so[q][0] + kb);
            } else if (AMODE == GM_A_AGGREGATE) {
#pragma unroll
                for (int q = 0; q < AQ; q++)
#pragma unroll
                    for (int j = 0; j < NR; j++) ra[S][q][j] = bload(r0a, so[q][j] == OOB ? OOB : so[q][j] + kb);
            } else {  // READOUT: the k tile lies inside one H-wide segment
                const int seg = k0 / a0.hidden, ko = kb - seg * a0.hidden * 4;
                if (seg == 0) {
#pragma unroll
                    for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r0a, so[q][0] + ko);
                } else if (seg == 1) {
#pragma unroll
                    for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r0b, so[q][1] == OOB ? OOB : so[q][1] + ko);
                } else if (seg == 2) {
#pragma unroll
                    for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r0b, so[q][2] == OOB ? OOB : so[q][2] + ko);
                } else {
#pragma unroll
                    for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r0b, so[q][3] == OOB ? OOB : so[q][3] + ko);
                }
            }
        } else {
            const int kb = (k0 - a0.k + 4 * c4) * 4;
#pragma unroll
            for (int q = 0; q < AQ; q++) ra[S][q][0] = bload(r1, off1[q] + kb);
        }
#pragma unroll
        for (int q = 0; q < BQ; q++) rb[S][q] = bload(rw, woff[q] + k0 * 4);
    };
    const bool ascaled = a0.scale != nullptr;  // uniform
    const float ascale = ascaled ? *a0.scale : 1.0f;
    const int aexp = __builtin_amdgcn_frexp_expf(ascale) - 1;  // ascale = 2^aexp
    unsigned* const amax = a0.amax;  // uniform
    float amx = 0.f;
    auto lstore = [&](auto SET, int buf, int k0) {
        constexpr int S = decltype(SET)::value;
        const bool agg = AMODE == GM_A_AGGREGATE && k0 < a0.k;
        const int kend = k0 < a0.k ? a0.k : K;  // zero the columns past the current source
        const int kk = k0 + 4 * c4;
        char* as = As[buf] + (c4 >> 2) * 64 + (c4 & 3) * 8;
#pragma unroll
        for (int q = 0; q < AQ; q++) {
            float4 v = ra[S][q][0];
            if (agg) {
#pragma unroll
                for (int j = 1; j < NR; j++) v = f4add(v, ra[S][q][j]);
                v = make_float4(v.x * scale[q], v.y * scale[q], v.z * scale[q], v.w * scale[q]);
            }
            if (k0 + BK > kend) {
                if (kk + 0 >= kend) v.x = 0.f;
                if (kk + 1 >= kend) v.y = 0.f;
                if (kk + 2 >= kend) v.z = 0.f;
                if (kk + 3 >= kend) v.w = 0.f;
            }
            if (amax) amx = fmaxf(amx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            half4 hi, lo;
            split4e(v, aexp, hi, lo);
            char* row = as + (rba + q * RSTEP) * ROWB;
            *reinterpret_cast<half4*>(row) = hi;
            *reinterpret_cast<half4*>(row + 32) = lo;
        }
#pragma unroll
        for (int q = 0; q < BQ; q++) *reinterpret_cast<float4*>(Bs[buf] + (rbb + q * RSTEP) * ROWB + 16 * c4) = rb[S][q];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

    const int h = lane >> 5, l32 = lane & 31;
    const _Float16 s12 = (_Float16)(1.0f / LO_S);
    auto compute = [&](int buf) {
        const char* ac = As[buf] + (wr * TM * 32 + l32) * ROWB + 16 * h;
        const char* bc = Bs[buf] + (wc * TN * 32 + l32) * ROWB + 16 * h;
#pragma unroll
        for (int sb = 0; sb < BK / 16; sb++) {
            half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; i++) {
                ah[i] = *reinterpret_cast<const half8*>(ac + i * 32 * ROWB + sb * 64);
                al[i] = *reinterpret_cast<const half8*>(ac + i * 32 * ROWB + sb * 64 + 32);
            }
#pragma unroll
            for (int j = 0; j < TN; j++) {
                bh[j] = *reinterpret_cast<const half8*>(bc + j * 32 * ROWB + sb * 64);
                bl[j] = *reinterpret_cast<const half8*>(bc + j * 32 * ROWB + sb * 64 + 32);
            }
#pragma unroll
            for (int i = 0; i < TM; i++)
#pragma unroll
                for (int j = 0; j < TN; j++) {
                    const half8 bs = bh[j] * s12;  // w_hi * 2^-12, exact
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bs, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
    };

    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    const int nk = (K + BK - 1) / BK;
    gload(S0{}, 0);
    if (nk > 1) gload(S1{}, BK);
    lstore(S0{}, 0, 0);
    __syncthreads();
    // step kt computes LDS buffer kt&1, loads tile kt+2 into register set kt&1 (its tile kt
    // is already in LDS) and stores tile kt+1 (set (kt+1)&1) into the other buffer
    auto step = [&](auto SET, int kt) {
        constexpr int S = decltype(SET)::value;
        if (kt + 2 < nk) gload(SET, (kt + 2) * BK);
        compute(S);
        if (kt + 1 < nk) lstore(std::integral_constant<int, S ^ 1>{}, S ^ 1, (kt + 1) * BK);
        __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
        step(S0{}, kt);
        if (kt + 1 < nk) step(S1{}, kt + 1);
    }

    if (amax) {
        amx = gm_wave_max(amx);
        if (lane == 0) gm_amax_publish(amax, amx);
    }
    const float si = *wscale_inv / ascale;  // undo the weight and A scales (powers of two: exact)
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] *= si;
    range_guard<TM, TN>(acc, ep.range_flag, lane);
    if constexpr (EPI == EPI_DGRAD) {
        dgrad_epilogue<WGM, WGN, TM, TN>(acc, ep, reinterpret_cast<float*>(As), m0, n0, wr, wc, M, N, lane);
    } else {
        CIn<TM, EPI> cin;
        cin_load<TM, EPI>(cin, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, lane);
        if constexpr (EPI == EPI_BIAS)
            act_dispatch(ep.act, [&](auto A) {
                epilogue<TM, TN, EPI, decltype(A)::value>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane,
                                                          cin);
            });
        else
            epilogue<TM, TN, EPI>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane, cin);
    }
}

// ---- 16x16x32 MFMA form of the LDS-DMA kernel (k_gemm3g MF = 1) ----
// v_mfma_f32_16x16x32_f16: lane l holds A[row l & 15][k 8 (l >> 4) .. +7], B[k same][col l & 15];
// C/D: col = l & 15, row = 4 (l >> 4) + r (r < 4). The chip holds a higher clock on this shape
// than on 32x32x16 for the same FLOPs on random data (MI355X_MICROARCH 'DVFS give-back' item 7).
// Wave tile (TM x 32) x (TN x 32) = (2 TM) x (2 TN) blocks of 16 x 16; LSTM / GRU gate tiles keep
// the 32-unit interleave: block j = 2 gate + b holds unit 16 b + (l & 15).
template <int T2, int EPI>
struct CIn16 {};
template <int T2>
struct CIn16<T2, EPI_LSTM> {
    float v[T2][2][4];
};
template <int T2, int EPI>
__device__ __forceinline__ void cin_load16(CIn16<T2, EPI>& c, const Epi& ep, int wm0, int wn0, int M, int lane) {
    if constexpr (EPI == EPI_LSTM) {
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int unit = (wn0 >> 2) + 16 * b + (lane & 15);
#pragma unroll
            for (int i = 0; i < T2; i++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = wm0 + 16 * i + 4 * (lane >> 4) + r;
                    c.v[i][b][r] = (row < M && unit < ep.hidden) ? ep.c_in[(long long)row * ep.ldc + unit] : 0.f;
                }
        }
    }
}
template <int T2, int N2>
__device__ __forceinline__ void range_guard16(const floatx4 (&acc)[T2][N2], unsigned* flag, int lane) {
    if (!flag) return;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < T2; i++)
#pragma unroll
        for (int j = 0; j < N2; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) bad |= !__builtin_isfinite(acc[i][j][r]);
    if (__ballot(bad) != 0ull && lane == 0) *reinterpret_cast<volatile unsigned*>(flag) = 1u;
}
template <int T2, int N2, int EPI, int A = -1>
__device__ __forceinline__ void epilogue16(floatx4 (&acc)[T2][N2], const Epi& ep, int wm0, int wn0, int M, int N,
                                           int lane, const CIn16<T2, EPI>& cin, const float* bl = nullptr) {
    const int l16 = lane & 15, rq = 4 * (lane >> 4);
    if constexpr (EPI == EPI_BIAS) {
        static_assert(N2 % 2 == 0, "column blocks in pairs (32-column sign words)");
        // buffer stores on a resource over the wave's rows [wm0, M) (rows past M dropped by its extent), columns
        // past N at the OOB offset: no per-element branches or 64-bit addresses
        const __amdgpu_buffer_rsrc_t rs = rsrc_rows(ep.y + wn0, ep.ldy, wm0, (long long)M * ep.ldy * 4);
        const unsigned ld4 = (unsigned)ep.ldy * 4u;
        unsigned vb[N2];
#pragma unroll
        for (int j = 0; j < N2; j++) vb[j] = wn0 + 16 * j + l16 < N ? (unsigned)rq * ld4 + 4u * (16 * j + l16) : (unsigned)OOB;
#pragma unroll
        for (int jp = 0; jp < N2 / 2; jp++) {
            float bv[2];
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const int col = wn0 + (2 * jp + b) * 16 + l16;
                bv[b] = bl ? bl[(2 * jp + b) * 16 + l16] : (ep.bias && col < N) ? ep.bias[col] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < T2; i++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = wm0 + i * 16 + rq + r;
                    unsigned long long bb[2];
#pragma unroll
                    for (int b = 0; b < 2; b++) {
                        const int col = wn0 + (2 * jp + b) * 16 + l16;
                        float v = acc[i][2 * jp + b][r] + bv[b];
                        v = act_t<A>(v, ep.act);
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs,
                                                              (int)(vb[2 * jp + b] + (unsigned)(i * 16 + r) * ld4), 0, 0);
                        bb[b] = ep.sbits ? __ballot(v > 0.f && col < N) : 0ull;
                    }
                    if (ep.sbits && l16 == 0 && row < M && wn0 + jp * 32 < N) {  // group q: 16 columns of row 4q + r
                        const int q = lane >> 4;
                        ep.sbits[(long long)row * ep.ldsb + ((wn0 + jp * 32) >> 5)] =
                            (unsigned)((bb[0] >> (16 * q)) & 0xFFFFull) | ((unsigned)((bb[1] >> (16 * q)) & 0xFFFFull) << 16);
                    }
                }
        }
    } else {  // EPI_LSTM: N2 == 8 blocks, gate g of unit 16 b + l16 in block 2 g + b
        const int H = ep.hidden;
        // buffer stores on resources over the wave's rows [wm0, M) (rows past M dropped by their extent), units
        // past H at the OOB offset: no per-element branches or 64-bit addresses
        const unsigned ly = (unsigned)ep.ldy * 4u, lc = (unsigned)ep.ldy2 * 4u, la = (unsigned)H * 16u;
        const __amdgpu_buffer_rsrc_t ry = rsrc_rows(ep.y + (wn0 >> 2), ep.ldy, wm0, (long long)M * ep.ldy * 4);
        const __amdgpu_buffer_rsrc_t rc =
            rsrc_rows(ep.y2 ? ep.y2 + (wn0 >> 2) : ep.y, ep.ldy2, wm0, ep.y2 ? (long long)M * ep.ldy2 * 4 : 0);
        const __amdgpu_buffer_rsrc_t ra =
            rsrc_rows(ep.act_out ? ep.act_out + (wn0 >> 2) : ep.y, 4LL * H, wm0, ep.act_out ? (long long)M * H * 16 : 0);
        auto st = [](float v, __amdgpu_buffer_rsrc_t rr, unsigned off) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rr, (int)off, 0, 0);
        };
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const int unit = (wn0 >> 2) + 16 * b + l16;
            const bool in = unit < H;
            const unsigned u4 = 4u * (16 * b + l16);
            const unsigned vy = in ? rq * ly + u4 : (unsigned)OOB, vc = in ? rq * lc + u4 : (unsigned)OOB;
            const unsigned va = in ? rq * la + u4 : (unsigned)OOB;
            float bgate[4];
#pragma unroll
            for (int g = 0; g < 4; g++)  // bl: the block's gate biases staged in LDS (k_gemm3g, EPI_LSTM)
                bgate[g] = bl ? bl[g * 32 + 16 * b + l16]  // (bl at this wave's first column)
                              : ep.bias ? ep.bias[wn0 + g * 32 + 16 * b + l16] : 0.f;
#pragma unroll
            for (int i = 0; i < T2; i++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const unsigned rl = (unsigned)(i * 16 + r);  // row - wm0 - rq
                    const float a0 = acc[i][b][r] + bgate[0], a1 = acc[i][2 + b][r] + bgate[1];
                    const float a2 = acc[i][4 + b][r] + bgate[2], a3 = acc[i][6 + b][r] + bgate[3];
                    if (ep.cell == 1) {  // GRU: r, z, n_x, n_h tiles
                        const float rg = sigm(a0), zg = sigm(a1);
                        const float ng = tanh_fast(a2 + rg * a3);
                        st((1.f - zg) * ng + zg * cin.v[i][b][r], ry, vy + rl * ly);
                        continue;
                    }
                    const float gi = sigm(a0), gf = sigm(a1), gg = tanh_fast(a2), go = sigm(a3);
                    const float cn = gf * cin.v[i][b][r] + gi * gg;
                    const float hn = go * tanh_fast(cn);
                    st(hn, ry, vy + rl * ly);
                    st(cn, rc, vc + rl * lc);
                    if (ep.act_out) {
                        const unsigned ao = va + rl * la;
                        st(gi, ra, ao);
                        st(gf, ra, ao + 4u * H);
                        st(gg, ra, ao + 8u * H);
                        st(go, ra, ao + 12u * H);
                    }
                }
        }
    }
}
// EPI_DGRAD on the 16x16 layout (dgrad_epilogue's contract): block j covers columns wn0 + 16 j +
// (l & 15), so a 32-column sign word spans block pair (2p, 2p + 1); column sums over the lane's 4
// rows, its 4 row groups (xor 16, 32), then the WGM row waves through LDS.
template <int WGM, int WGN, int T2, int N2, bool STAGED = false>
__device__ __forceinline__ void dgrad_epilogue16(floatx4 (&acc)[T2][N2], const Epi& ep, float* red, int m0, int n0,
                                                 int wr, int wc, int M, int N, int lane) {
    const int l16 = lane & 15, rq = 4 * (lane >> 4);
    const int wm0 = m0 + wr * T2 * 16, wn0 = n0 + wc * N2 * 16;
    constexpr int BM = WGM * T2 * 16, BN = WGN * N2 * 16, WPR = BN / 32;
    static_assert(N2 % 2 == 0, "column blocks in pairs (32-column sign words)");
    unsigned* smb = reinterpret_cast<unsigned*>(red + WGM * BN);
    if (ep.mbits && !STAGED) {
        for (int e = threadIdx.x; e < BM * WPR; e += WGM * WGN * 64) {
            const int r = e / WPR, w = e - r * WPR;
            const int row = m0 + r, col0 = n0 + 32 * w;
            smb[e] = (row < M && col0 < ep.split) ? ep.mbits[(long long)row * ep.ldmb + (col0 >> 5)] : ~0u;
        }
        __syncthreads();
    }
    float mx = 0.f;
    float cs[N2];
    const int sp = ep.split;
    const bool blk_lo = n0 + BN <= sp, blk_hi = n0 >= sp;  // block-uniform
    if (n0 + BN <= N && (blk_lo || blk_hi)) {
        // the block's columns all on one side of the split and inside N: buffer stores on a resource over
        // the wave's rows [wm0, M) (rows past M dropped by its extent), the row offset in the VGPR and the
        // column block in the instruction's offset; no per-element bounds branches or 64-bit addresses
        const long long ld = blk_lo ? ep.ldy : ep.ldy2;
        float* yb = blk_lo ? ep.y + wn0 : ep.y2 + (wn0 - sp);
        const __amdgpu_buffer_rsrc_t rs = rsrc_rows(yb, ld, wm0, (long long)M * ld * 4);
        const int voff = (rq * (int)ld + l16) * 4, ld4 = (int)ld * 4;
        if (blk_lo) {
#pragma unroll
            for (int j = 0; j < N2; j++) {
                const int bit = (j & 1) * 16 + l16, wofs = (wn0 - n0 + 16 * j) >> 5;
                float s = 0.f;
#pragma unroll
                for (int i = 0; i < T2; i++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = wm0 + i * 16 + rq + r;
                        float v = acc[i][j][r];
                        if (ep.mbits && !((smb[(row - m0) * WPR + wofs] >> bit) & 1u)) v *= 0.01f;
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff + (i * 16 + r) * ld4 + j * 64,
                                                              0, 0);
                        const bool in = row < M;
                        s += in ? v : 0.f;
                        mx = in ? fmaxf(mx, fabsf(v)) : mx;
                    }
                s += __shfl_xor(s, 16);
                cs[j] = s + __shfl_xor(s, 32);
            }
        } else {
#pragma unroll
            for (int j = 0; j < N2; j++) {
#pragma unroll
                for (int i = 0; i < T2; i++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rs,
                                                              voff + (i * 16 + r) * ld4 + j * 64, 0, 0);
                cs[j] = 0.f;
            }
        }
    } else {
#pragma unroll
    for (int j = 0; j < N2; j++) {
        const int col = wn0 + j * 16 + l16;
        const int bit = (j & 1) * 16 + l16, wofs = (col - n0) >> 5;
        const bool lo = col < ep.split;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < T2; i++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = wm0 + i * 16 + rq + r;
                if (row >= M || col >= N) continue;
                float v = acc[i][j][r];
                if (lo) {
                    if (ep.mbits && !((smb[(row - m0) * WPR + wofs] >> bit) & 1u)) v *= 0.01f;
                    ep.y[(long long)row * ep.ldy + col] = v;
                    s += v;
                    mx = fmaxf(mx, fabsf(v));
                } else {
                    ep.y2[(long long)row * ep.ldy2 + col - ep.split] = v;
                }
            }
        s += __shfl_xor(s, 16);
        cs[j] = s + __shfl_xor(s, 32);
    }
    }
    if (ep.gmax) {
        mx = gm_wave_max(mx);
        if (lane == 0) gm_amax_publish(ep.gmax, mx);
    }
    if (ep.part) {
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < N2; j++) red[wr * BN + wc * N2 * 16 + j * 16 + l16] = cs[j];
        }
        __syncthreads();
        if (wr == 0 && lane < 16) {
#pragma unroll
            for (int j = 0; j < N2; j++) {
                const int c = wc * N2 * 16 + j * 16 + l16, col = n0 + c;
                float s = red[c];
#pragma unroll
                for (int w = 1; w < WGM; w++) s += red[w * BN + c];
                if (col < ep.split && col < N) ep.part[(long long)(m0 / BM) * ep.split + col] = s;
            }
        }
    }
}

// EPI_HEAD on the 16x16 layout: per row block i, a lane's partial dot products (4 rows x 4 heads)
// are reduce-scattered over its 16-lane group (xor 8..1: 15 shuffles; lane ends with entry l & 15
// = row 4 (l >> 4) + (e >> 2), head e & 3), the WGN column waves summed through LDS.
// hl (optional): the block's bias and Q-head weight columns staged in LDS before the k loop ([5][block
// width]: bias, wq rows 0..3, zero past N / nq; k_gemm3g head_load / head_store), instead of global loads here
template <int T2, int N2, int WGN, int BM, int A = -1>
__device__ __forceinline__ void head_epilogue16(floatx4 (&acc)[T2][N2], const Epi& ep, char* lds, int m0, int wr,
                                                int wc, int M, int N, int lane, int tid, int n0 = 0,
                                                const float* hl = nullptr) {
    constexpr int BNH = WGN * N2 * 16;  // the block's columns
    const int l16 = lane & 15, rq = 4 * (lane >> 4);
    float bv[N2], wqv[N2][4];
#pragma unroll
    for (int j = 0; j < N2; j++) {
        const int cl = wc * N2 * 16 + j * 16 + l16, col = n0 + cl;
        if (hl) {
            bv[j] = hl[cl];
#pragma unroll
            for (int a = 0; a < 4; a++) wqv[j][a] = hl[(1 + a) * BNH + cl];
        } else {
            bv[j] = (ep.bias && col < N) ? ep.bias[col] : 0.f;
#pragma unroll
            for (int a = 0; a < 4; a++) wqv[j][a] = (col < N && a < ep.nq) ? ep.wq[a * ep.ldwq + col] : 0.f;
        }
    }
    float* qp = reinterpret_cast<float*>(lds);  // [WGN][BM][4]
    float red[T2];
#pragma unroll
    for (int i = 0; i < T2; i++) {
        float x[16];
#pragma unroll
        for (int e = 0; e < 16; e++) x[e] = 0.f;
#pragma unroll
        for (int j = 0; j < N2; j++) {
            const int col = n0 + wc * N2 * 16 + j * 16 + l16;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float y = acc[i][j][r] + bv[j];
                y = act_t<A>(y, ep.act);
                if (ep.y) {
                    const int row = m0 + wr * T2 * 16 + i * 16 + rq + r;
                    if (row < M && col < N) ep.y[(long long)row * ep.ldy + col] = y;
                }
#pragma unroll
                for (int a = 0; a < 4; a++) x[r * 4 + a] = fmaf(y, wqv[j][a], x[r * 4 + a]);
            }
        }
#pragma unroll
        for (int mask = 8, n = 8; mask >= 1; mask >>= 1, n >>= 1) {
            const bool up = (l16 & mask) != 0;
#pragma unroll
            for (int k = 0; k < n; k++) {
                float mine, other;
                swap_if(up, x[k], x[n + k], mine, other);
                x[k] = mine + __shfl_xor(other, mask);
            }
        }
        red[i] = x[0];
    }
    __syncthreads();  // every wave is done with the operand stages
#pragma unroll
    for (int i = 0; i < T2; i++) {
        const int rl = wr * T2 * 16 + i * 16 + rq + (l16 >> 2);
        qp[(wc * BM + rl) * 4 + (l16 & 3)] = red[i];
    }
    __syncthreads();
    for (int e = tid; e < BM * 4; e += WGN * (BM / T2 / 16) * 64) {
        const int rl = e >> 2, a = e & 3, row = m0 + rl;
        if (a >= ep.nq || row >= M) continue;
        float v = (ep.bq && n0 == 0) ? ep.bq[a] : 0.f;
#pragma unroll
        for (int w = 0; w < WGN; w++) v += qp[(w * BM + rl) * 4 + a];
        if (ep.q_atomic)  // two column blocks onto a zeroed q: 0 + x is exact, so x + y is order-free
            atomicAdd(&ep.q[(long long)row * ep.ldq + a], v);
        else
            ep.q[(long long)row * ep.ldq + a] = v;
    }
}

// K-major split-f16 LDS image swizzle (EPI_CHAIN): the 8-byte slot of row k is XOR'd with dqn_swz(k) =
// k & 15 with bits 1 and 2 swapped, so the epilogue's 16 consecutive-k writes and the transposed reads
// (rows 8g + q, 4 lanes per row) both hit distinct banks.
__device__ __forceinline__ int dqn_swz(int k) {
    return (k & 9) | ((k & 2) << 1) | ((k & 4) >> 1);
}

// ---- EPI_CHAIN: the next MLP layer in the block that computed this one (the rollout's NetMon encoder
// layers 2 -> 3, src/model.py:13-42) ----
// The block (BM rows x the layer's whole width K2 = WGN * N2 * 16) sends its activations through bias +
// activation and the split (split4: the bits a dense A tile of the next layer would get) into two
// K-major LDS images ([k][BM rows] f16, dqn_swz slots, BM * 2-byte rows), which
// alias the finished operand stages. The next layer (N3 columns) has its own wave grid: NW / W3N waves over
// the rows (T3 16-row blocks each) x W3N over the columns (J3 16-column blocks each), so each weight
// fragment is fetched by NW / W3N waves (2, not WGM = 4: half the tail's L2 traffic). Each wave reads its A
// fragments transposed from the images (ds_read_b64_tr_b16) and its packed weight fragments straight from
// L2, two k tiles ahead, and stores act3(. + b3) with epilogue16. The m x K2 activation of the first layer
// never reaches HBM.
template <int WGM, int WGN, int T2, int N2, int BM, int N3, int W3N, int A = -1>
__device__ __forceinline__ void chain_tail(floatx4 (&acc)[T2][N2], const Epi& ep, char* lds, int m0, int wr, int wc,
                                           int M, int lane, const float* bl, float si3) {
    static_assert(WGM * T2 * 16 == BM, "the wave rows hold the block's rows");
    constexpr int NW = WGM * WGN, W3M = NW / W3N;
    constexpr int T3 = BM / 16 / W3M, J3 = N3 / 16 / W3N;
    static_assert(NW % W3N == 0 && T3 * 16 * W3M == BM && J3 * 16 * W3N == N3 && J3 % 2 == 0, "layer-3 wave grid");
    constexpr int K2 = WGN * N2 * 16;  // next layer's K = this layer's width
    constexpr int RS = BM * 2;         // image row bytes
    constexpr int NK = K2 / 32;        // next layer's k tiles
    char* ih = lds;
    char* il = lds + K2 * RS;
    const int l16 = lane & 15, rq = 4 * (lane >> 4);
    __syncthreads();  // every wave is past its last reads of the operand stages
#pragma unroll
    for (int j = 0; j < N2; j++) {
        const int n = wc * N2 * 16 + j * 16 + l16;  // this layer's column = the next layer's k
        const float bj = bl[n];  // staged before the k loop (k_gemm3g head_load / head_store)
        const int sw = dqn_swz(n) << 3;
#pragma unroll
        for (int i = 0; i < T2; i++) {
            const int m = wr * T2 * 16 + i * 16 + rq;
            float4 v;
            v.x = act_t<A>(acc[i][j][0] + bj, ep.act);
            v.y = act_t<A>(acc[i][j][1] + bj, ep.act);
            v.z = act_t<A>(acc[i][j][2] + bj, ep.act);
            v.w = act_t<A>(acc[i][j][3] + bj, ep.act);
            half4 hi, lo;
            split4(v, hi, lo);
            const int off = n * RS + ((2 * m) ^ sw);
            *reinterpret_cast<half4*>(ih + off) = hi;
            *reinterpret_cast<half4*>(il + off) = lo;
        }
    }
    const int w3 = wr * WGN + wc, w3r = w3 / W3N, w3c = w3 % W3N;  // this wave's layer-3 block
    // weight fragments of this wave's 16 J3 columns: row n3 = 16 J3 w3c + 16 jb + l16, k 8 q .. 8 q + 7 of
    // each 32-deep tile (16-k block (q >> 1), halves (q & 1) x 8; hi at +0, lo at +32 of a block's 64 bytes)
    const int q = lane >> 4;
    const __amdgpu_buffer_rsrc_t rw = rsrc(reinterpret_cast<const float*>(ep.w2), ep.w2bytes);
    int wo[J3];
#pragma unroll
    for (int jb = 0; jb < J3; jb++)
        wo[jb] = (int)((w3c * J3 * 16 + jb * 16 + l16) * ep.ldw2) + (q >> 1) * 64 + (q & 1) * 16;
    constexpr int NB3 = 2;  // weight tiles in flight
    u32x4 pbh[NB3][J3], pbl[NB3][J3];
    auto bfetch = [&](int slot, int kt) {
#pragma unroll
        for (int jb = 0; jb < J3; jb++) {
            pbh[slot][jb] = __builtin_amdgcn_raw_buffer_load_b128(rw, wo[jb] + kt * 128, 0, 0);
            pbl[slot][jb] = __builtin_amdgcn_raw_buffer_load_b128(rw, wo[jb] + kt * 128 + 32, 0, 0);
        }
    };
#pragma unroll
    for (int t = 0; t < NB3; t++) bfetch(t, t);
    __syncthreads();  // the images are complete
    floatx4 acc3[T3][J3];
#pragma unroll
    for (int i = 0; i < T3; i++)
#pragma unroll
        for (int j = 0; j < J3; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc3[i][j][r] = 0.f;
    const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
    typedef __fp16 v4fp16 __attribute__((__vector_size__(8)));
    auto frag = [&](const char* img, int k0, int col0) {  // 8 consecutive k of one row
        const int r0 = k0 + 8 * g + qq, r1 = r0 + 4;
        const char* a0 = img + r0 * RS + ((2 * (col0 + 4 * p)) ^ (dqn_swz(r0) << 3));
        const char* a1 = img + r1 * RS + ((2 * (col0 + 4 * p)) ^ (dqn_swz(r1) << 3));
        const half4 x0 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a0)));
        const half4 x1 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a1)));
        return half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    };
    const _Float16 s12 = (_Float16)(1.0f / LO_S);
    const int row0 = w3r * T3 * 16;
    half8 fah[2][T3], fal[2][T3];
#pragma unroll
    for (int i = 0; i < T3; i++) {
        fah[0][i] = frag(ih, 0, row0 + 16 * i);
        fal[0][i] = frag(il, 0, row0 + 16 * i);
    }
#pragma unroll
    for (int kt = 0; kt < NK; kt++) {
        const int cur = kt & 1, slot = kt % NB3;
        if (kt + 1 < NK) {
#pragma unroll
            for (int i = 0; i < T3; i++) {
                fah[cur ^ 1][i] = frag(ih, (kt + 1) * 32, row0 + 16 * i);
                fal[cur ^ 1][i] = frag(il, (kt + 1) * 32, row0 + 16 * i);
            }
        }
        half8 bh[J3], bl[J3];
#pragma unroll
        for (int jb = 0; jb < J3; jb++) {
            bh[jb] = __builtin_bit_cast(half8, pbh[slot][jb]);
            bl[jb] = __builtin_bit_cast(half8, pbl[slot][jb]);
        }
        if (kt + NB3 < NK) bfetch(slot, kt + NB3);
#pragma unroll
        for (int jb = 0; jb < J3; jb++) {
            const half8 bs = bh[jb] * s12;
#pragma unroll
            for (int i = 0; i < T3; i++) {
                floatx4& c = acc3[i][jb];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[cur][i], bs, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[cur][i], bl[jb], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[cur][i], bh[jb], c, 0, 0, 0);
            }
        }
    }
    const float si = si3;  // *ep.wsi2, loaded at kernel start
#pragma unroll
    for (int i = 0; i < T3; i++)
#pragma unroll
        for (int j = 0; j < J3; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc3[i][j][r] *= si;
    range_guard16<T3, J3>(acc3, ep.range_flag, lane);
    Epi e3 = ep;
    e3.bias = ep.b2;
    e3.act = ep.act2;
    e3.sbits = nullptr;
    CIn16<T3, EPI_BIAS> none;
    act_dispatch(e3.act, [&](auto A3) {
        epilogue16<T3, J3, EPI_BIAS, decltype(A3)::value>(acc3, e3, m0 + row0, w3c * J3 * 16, M, N3, lane, none,
                                                          bl + WGN * N2 * 16 + w3c * J3 * 16);
    });
}

// ---------------------------------------------------------------------------------------
// X3 kernel with LDS-DMA staging (buffer_load ... lds): both operands go HBM/L2 -> LDS with
// no VGPR round trip and no ds_write pass. A stays fp32 in LDS (32-deep k tiles = one 128-B
// line per row) and is split into its f16 hi / 2^12-scaled lo pieces per MFMA fragment, in
// registers, between the MFMAs; B tiles are the packed weight rows (same 128-B line per row).
// LDS image per stage: [BM rows of A | BN rows of B] x 128 B, 16-B chunks XOR-swizzled by
// row (pos = chunk ^ ((row >> 1) & 7): conflict-free ds_read_b128 on the 32-row fragments);
// the DMA writes lane-linear (8 rows per wave-instruction), so the swizzle is applied to the
// per-lane SOURCE address. The k loop is unrolled by STAGES so every LDS stage offset is a
// compile-time immediate; the per-lane DMA offsets are fixed over K (the k position goes in
// the scalar offset) and the fragment addresses are fixed per lane, so the loop's vector ALU
// work is the A split and the w_hi * 2^-12 scaling only. Tile kt+STAGES-1 is issued at the
// top of step kt, and a counted vmcnt + raw s_barrier at the bottom retires tile kt+1 only.
// A sources: DENSE, READOUT (the 32-deep tile lies inside one H-wide segment; missing
// neighbours read an out-of-range offset = zeros), then the optional dense second source.
// AX (training operands): 0 plain; 1 publish max|A| into a0.amax (the weight gradient's
// operand scale, as k_gemm3 does while splitting its A tiles); 2 A scaled by the device power
// of two *a0.scale before the split (gradient operands), undone with the weight scale.
// MF: 0 v_mfma_f32_32x32x16_f16 fragments, 1 v_mfma_f32_16x16x32_f16 (same tiles, LDS image and
// pipeline; the 16x16 form splits a k tile's MFMAs into two column halves and keeps the split A
// of the tile in registers for the second half).
// Row swizzle of the LDS-DMA images: 16-B chunk c of row R sits at position c ^ swz(R >> 1 & 7).
// 32x32x16 reads: the identity. 16x16x32 reads: a row's 16-lane ds_read_b128 group holds rows 0..15
// with two k groups (q) split by (R >> 1) in {2..5}, and the identity puts two of its lanes on one
// bank quadruple (2-way for the A fragments, MI355X_MICROARCH §LDS lane groups); this permutation
// keeps both the A chunks (2q + p) and the B chunks (2p + q) of every group on distinct banks
template <int MF>
__device__ __forceinline__ int gswz(int k) {
    return MF == 1 ? (int)((0x32765410u >> (4 * k)) & 7u) : k;
}

template <int WGM, int WGN, int TM, int TN, int STAGES, int AMODE, int EPI, int OCC, int AX = 0, int MF = 0>
__global__ __launch_bounds__(WGM* WGN * 64, OCC) void k_gemm3g(ASrc a0, ASrc a1, const _Float16* __restrict__ w,
                                                              long long ldw, unsigned wbytes, int M, int N, int K,
                                                              Epi ep, const float* __restrict__ wscale_inv) {
    constexpr int BK = 32, NW = WGM * WGN;
    constexpr int BM = WGM * TM * 32, BN = WGN * TN * 32;
    // ROUTING_ENC (RENC): the A tile is computed in the block from the routing node observations and the
    // folded encoder layer's W0^T, whose 32-column slice per k tile is DMA'd (RW pieces of 8 rows per wave)
    constexpr bool RENC = AMODE == GM_A_ROUTING_ENC;
    // W0^T slice: 4N + 8 <= GM_RENC_ROWS rows (N <= 50) in pieces of 8 rows, piece j NW + wave DMA'd by wave
    constexpr int W0P = RENC ? (GM_RENC_ROWS + 7) / 8 : 0;  // pieces per slice stage
    constexpr int RW = RENC ? (W0P + NW - 1) / NW : 0;       // pieces per wave (the last ones skipped past 4N + 8)
    constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;  // DMA instructions per wave per tile
    constexpr int NAD = RENC ? 0 : NA;                   // A pieces actually DMA'd
    constexpr int NL = NAD + NB + RW;
    constexpr int STAGE_B = (BM + BN) * 128;
    constexpr int W0S_B = W0P * 1024;                     // one W0^T slice stage
    constexpr int RENC_B = RENC ? 2 * W0S_B + 4 * 1024 : 0;  // two slice stages + the bias (<= 1024 columns)
    static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows per wave");
    static_assert(AMODE != GM_A_AGGREGATE, "aggregate source uses k_gemm3");
    static_assert(STAGES >= 2 && STAGES <= 4, "stages");
    static_assert(!RENC || (STAGES == 2 && BM * 4 == NW * 64 && MF == 1 && NW == 8),
                  "routing-encoder source: 2-stage ping-pong tile, 8 threads x 2 rows per 128 A rows");
    static_assert(EPI != EPI_CHAIN || (MF == 1 && STAGES * STAGE_B + RENC_B >= 2 * BN * BM * 2),
                  "chain epilogue: the next layer's split A images alias the operand stages");
    // EPI_HEAD: the block's bias and Q-head weight columns, staged once (head_load / head_store) so that the
    // epilogue does not start with 40 dependent global loads per lane
    constexpr int HEAD_N = EPI == EPI_HEAD    ? 5 * BN
                           : EPI == EPI_CHAIN ? BN + 128  // + the layer-3 biases
                           : (EPI == EPI_LSTM || EPI == EPI_BIAS) ? BN
                                                                   : 0;
    constexpr int HEAD_B = HEAD_N * 4;
#if GM_DIAG == 30
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE_B + RENC_B + HEAD_B + 1024];
#else
    __shared__ __attribute__((aligned(16))) char lds[STAGES * STAGE_B + RENC_B + HEAD_B];
#endif

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases in SGPRs
#if GM_DIAG == 30
    // stamps of k steps 4..11 x 8 points by waves 0 and NW / 2 (one SIMD), kept in LDS until the end
    unsigned long long* stl = reinterpret_cast<unsigned long long*>(lds + STAGES * STAGE_B + RENC_B + HEAD_B);
    const bool stw = lane == 0 && (wave == 0 || wave == NW / 2);
    auto stamp = [&](int kt, int pt) {
        if (stw && kt >= 4 && kt < 12) stl[((wave != 0) * 8 + (kt - 4)) * 8 + pt] = __builtin_amdgcn_s_memtime();
    };
#define GM_STAMP(kt, pt)                  \
    __builtin_amdgcn_sched_barrier(0); \
    stamp(kt, pt);                     \
    __builtin_amdgcn_sched_barrier(0);
#else
#define GM_STAMP(kt, pt)
#endif
    const int wr = wave / WGN, wc = wave % WGN;
    const int nM = (M + BM - 1) / BM, nN = (N + BN - 1) / BN;
    const int bid = xcd_remap(blockIdx.x, nM * nN);
    const int m0 = (bid / nN) * BM, n0 = (bid % nN) * BN;

    // ---- per-lane DMA source offsets (fixed over K): row (lane >> 3) of each 8-row piece,
    // logical chunk c = (lane & 7) ^ swizzle(row) ----
    const int sub = lane >> 3;
    int so[NA][4];  // DENSE: [0]; READOUT: segment rows (OOB = none)
    int o1[NA];     // second (dense) source
#pragma unroll
    for (int j = 0; j < NAD; j++) {
        const int R = (wave * NA + j) * 8 + sub;
        const int c = (lane & 7) ^ gswz<MF>((R >> 1) & 7);
        const int row = min(m0 + R, M - 1);
        o1[j] = (int)((row - m0) * a1.ld0) * 4 + 16 * c;
#pragma unroll
        for (int s = 0; s < 4; s++) so[j][s] = OOB;
        if (AMODE == GM_A_DENSE) {
            so[j][0] = (int)((row - m0) * a0.ld0) * 4 + 16 * c;
        } else if constexpr (AMODE == GM_A_READOUT) {  // [h_final[v] | h_prev[nbr(v, 0..2)]], v = agent_node[row]
            const int g = row / a0.rows_per_graph;
            const int v = a0.agent_node[row];
            const int* nb = a0.nbr + ((size_t)g * a0.n_nodes + v) * a0.deg;
            so[j][0] = (int)((g * a0.n_nodes + v) * a0.ld0) * 4 + 16 * c;
#pragma unroll
            for (int s = 1; s < 4; s++) {
                const int mm = s - 1 < a0.deg ? nb[s - 1] : -1;
                so[j][s] = mm >= 0 ? (int)((g * a0.n_nodes + mm) * a0.ld1) * 4 + 16 * c : OOB;
            }
        }
    }
    int wo[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const int R = (wave * NB + j) * 8 + sub;
        const int c = (lane & 7) ^ gswz<MF>((R >> 1) & 7);
        wo[j] = (int)(min(n0 + R, N - 1) * ldw) + 16 * c;
    }

    const __amdgpu_buffer_rsrc_t r0a =
        AMODE == GM_A_DENSE ? rsrc_rows(a0.p0, a0.ld0, m0, a0.bytes0) : rsrc(a0.p0, (unsigned)a0.bytes0);
    const __amdgpu_buffer_rsrc_t r0b = rsrc(a0.p1 ? a0.p1 : a0.p0, (unsigned)(a0.p1 ? a0.bytes1 : a0.bytes0));
    const __amdgpu_buffer_rsrc_t r1 = a1.p0 ? rsrc_rows(a1.p0, a1.ld0, m0, a1.bytes0) : rsrc(a0.p0, 0u);
    const __amdgpu_buffer_rsrc_t rw = rsrc(reinterpret_cast<const float*>(w), wbytes);

    // ---- ROUTING_ENC: this thread's 16-byte chunk rq (k = 4 rq .. 4 rq + 3 of every tile) of A rows rr and
    // rr + BM / 2, and their node-obs features: A[r][k] = act0(b0[k] + W0^T[v][k] + cnt W0^T[N][k] + load
    // W0^T[N + 1][k] + sum over the 3 neighbour blocks (W0^T[off + u][k] + len W0^T[off + N][k] + load
    // W0^T[off + N + 1][k])), the 12 nonzero columns of the node observation [onehot(n) | cnt | load | 3 x
    // (onehot(nbr) | len | load)] (src/env/routing.py:187-235), in k_routing_enc's order of operations. The
    // 9 row-independent W0^T / bias chunks are read once for both rows ----
    const int rr = tid >> 3, rq = tid & 7;
    int r_oh[2][4] = {};
    float r_sv[2][8] = {};
    int wso[RW > 0 ? RW : 1];
    if constexpr (RENC) {
        const int Nn = a0.n_nodes;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int row = min(m0 + rr + h * (BM / 2), M - 1);
            const int g = row / Nn, v = row - g * Nn;
            const float* xr = a0.p0 + (long long)row * a0.ld0;
            const int* nb = a0.nbr + ((long long)g * Nn + v) * 3;
            r_oh[h][0] = v;
            r_sv[h][0] = xr[Nn];
            r_sv[h][1] = xr[Nn + 1];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const int off = Nn + 2 + k * (Nn + 2);
                r_oh[h][k + 1] = off + nb[k];
                r_sv[h][2 + 2 * k] = xr[off + Nn];
                r_sv[h][3 + 2 * k] = xr[off + Nn + 1];
            }
        }
        const int K0 = 4 * Nn + 8;
#pragma unroll
        for (int j = 0; j < RW; j++) {  // piece j NW + wave: 8 rows of W0^T (see issue_w0)
            const int R = (j * NW + wave) * 8 + sub;
            wso[j] = R < K0 ? (int)(R * a0.ld1) * 4 + 16 * (lane & 7) : OOB;
        }
        // the folded layer's bias for all k, once (plain loads: retired before the k loop's counted waits)
        float* b0s = reinterpret_cast<float*>(lds + STAGES * STAGE_B + 2 * W0S_B);
        for (int k = tid; k < a0.k; k += NW * 64) b0s[k] = a0.bias0 ? a0.bias0[k] : 0.f;
    }
    const __amdgpu_buffer_rsrc_t rw0 = rsrc(RENC ? a0.p1 : a0.p0, RENC ? (unsigned)a0.bytes1 : 0u);
    // EPI_HEAD staging: loaded into registers before the prologue DMAs, stored to LDS after them (the store's
    // wait then covers these loads only: they were issued first); published by the k loop's barriers
    constexpr int HPT = HEAD_N ? (HEAD_N + NW * 64 - 1) / (NW * 64) : 1;
    float hv[HPT];
    float* const hlds = reinterpret_cast<float*>(lds + STAGES * STAGE_B + RENC_B);
    auto head_load = [&]() {
        if constexpr (EPI == EPI_LSTM || EPI == EPI_BIAS) {  // the block's biases
#pragma unroll
            for (int i = 0; i < HPT; i++) {
                const int e = tid + i * NW * 64, col = n0 + e;
                hv[i] = (e < HEAD_N && col < N && ep.bias) ? ep.bias[col] : 0.f;
            }
        }
        if constexpr (EPI == EPI_CHAIN) {  // layer-2 biases (one column block: n0 = 0), then layer 3's
#pragma unroll
            for (int i = 0; i < HPT; i++) {
                const int e = tid + i * NW * 64;
                hv[i] = 0.f;
                if (e < BN) {
                    if (e < N && ep.bias) hv[i] = ep.bias[e];
                } else if (e < HEAD_N && ep.b2)
                    hv[i] = ep.b2[e - BN];
            }
        }
        if constexpr (EPI == EPI_HEAD) {
#pragma unroll
            for (int i = 0; i < HPT; i++) {
                const int e = tid + i * NW * 64, r = e / BN, col = n0 + (e - r * BN);
                hv[i] = 0.f;
                if (e < HEAD_N && col < N) {
                    if (r == 0)
                        hv[i] = ep.bias ? ep.bias[col] : 0.f;
                    else if (r - 1 < ep.nq)
                        hv[i] = ep.wq[(r - 1) * ep.ldwq + col];
                }
            }
        }
    };
    auto head_store = [&]() {
        if constexpr (HEAD_N > 0) {
#pragma unroll
            for (int i = 0; i < HPT; i++)
                if (tid + i * NW * 64 < HEAD_N) hlds[tid + i * NW * 64] = hv[i];
        }
    };
    // DMA of the W0^T slice of k tile kt (32 columns of every input row) into slice stage kt & 1 = WS (2-stage
    // tile: compile-time, like every LDS base of the loop). Wave w issues pieces j NW + w (j < RW) and skips
    // the pieces past the 4N + 8 input rows (wave-uniform): at N = 20 the 11 pieces put at most 3 of a SIMD's
    // two waves' DMA issues in a step (the 2-stage loop waits vmcnt(0), so the count may vary per wave)
    const int w0rows = RENC ? 4 * a0.n_nodes + 8 : 0;
    auto issue_w0 = [&](auto WS, int kt) {
        char* base = lds + STAGES * STAGE_B + decltype(WS)::value * W0S_B;
#pragma unroll
        for (int j = 0; j < RW; j++)
            if ((j * NW + wave) * 8 < w0rows) dma16(rw0, base + (j * NW + wave) * 1024, wso[j], kt * BK * 4);
    };
    // split-f16 A tile kt into stage ST from slice stage kt & 1 (landed and published by a barrier)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    auto lo2 = [](const float4& v, int p) { return p == 0 ? f32x2{v.x, v.y} : f32x2{v.z, v.w}; };
    auto renc_a = [&](auto ST, int kt) {  // (tile kt's slice stage kt & 1 = its operand stage ST)
        const float* wsl = reinterpret_cast<const float*>(lds + STAGES * STAGE_B + decltype(ST)::value * W0S_B);
        const float* b0s = reinterpret_cast<const float*>(lds + STAGES * STAGE_B + 2 * W0S_B) + kt * BK;
        char* adst = lds + decltype(ST)::value * STAGE_B;
        const int Nn = a0.n_nodes;
        auto wrow = [&](int r) { return *reinterpret_cast<const float4*>(wsl + r * BK + 4 * rq); };
        const float4 bz = *reinterpret_cast<const float4*>(b0s + 4 * rq);
        const float4 wa = wrow(Nn), wb = wrow(Nn + 1);
        float4 wl[3], wd[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int off = Nn + 2 + k * (Nn + 2);
            wl[k] = wrow(off + Nn);
            wd[k] = wrow(off + Nn + 1);
        }
        // the folded layer's activation resolved once per tile (act_dispatch), not per element
        act_dispatch(a0.act0, [&](auto ACT) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int* oh = r_oh[h];
            const float* sv = r_sv[h];
            // element pairs on packed f32 (v_pk_fma_f32 / v_pk_add_f32): the same operations, half the issues
            const float4 e0 = wrow(oh[0]);
            const f32x2 s0 = {sv[0], sv[0]}, s1 = {sv[1], sv[1]};
            f32x2 ap[2];
#pragma unroll
            for (int p = 0; p < 2; p++)
                ap[p] = lo2(bz, p) + lo2(e0, p) + s0 * lo2(wa, p) + s1 * lo2(wb, p);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const float4 ek = wrow(oh[k + 1]);
                const f32x2 ln = {sv[2 + 2 * k], sv[2 + 2 * k]}, ld = {sv[3 + 2 * k], sv[3 + 2 * k]};
#pragma unroll
                for (int p = 0; p < 2; p++) ap[p] += lo2(ek, p) + ln * lo2(wl[k], p) + ld * lo2(wd[k], p);
            }
            float a[4] = {ap[0][0], ap[0][1], ap[1][0], ap[1][1]};
#pragma unroll
            for (int e = 0; e < 4; e++) a[e] = act_t<decltype(ACT)::value>(a[e], a0.act0);
            // split once here (the bits of the k loop's split8), stored where the 16x16 read takes its A
            // chunks: hi of k 8q .. 8q + 7 at logical chunk 2q, lo at 2q + 1 (q = rq / 2, this thread's 4 k
            // at byte 8 (rq & 1)); even rows store hi first, odd rows lo first, so the two rows of a
            // 16-lane store group hit disjoint banks
            half4 hi, lo;
            split4e(make_float4(a[0], a[1], a[2], a[3]), 0, hi, lo);
            const int R = rr + h * (BM / 2);
            const int sw = gswz<MF>((R >> 1) & 7), odd = R & 1;
            char* rowp = adst + R * 128 + 8 * (rq & 1);
            const half4 first = odd ? lo : hi, second = odd ? hi : lo;
            *reinterpret_cast<half4*>(rowp + (((2 * (rq >> 1) + odd) ^ sw) << 4)) = first;
            *reinterpret_cast<half4*>(rowp + (((2 * (rq >> 1) + 1 - odd) ^ sw) << 4)) = second;
        }
        });
    };

    // DMA of k tile kt into stage ST (all LDS bases wave-uniform); ROUTING_ENC: the A tile computed from
    // this tile's slice, then the B tile and the next W0^T slice. In that order: LDS reads after an LDS-DMA
    // whose destination the compiler cannot tell apart wait for it (s_waitcnt vmcnt(0)), which put the DMA
    // latency in front of the A computation (2.2-3.1 k of a 4.7 k-cycle step, tools/stamp_fold.py)
    auto issue = [&](auto ST, int kt) {
        char* base = lds + decltype(ST)::value * STAGE_B + wave * NA * 1024;
        const int k0 = kt * BK;
        if constexpr (RENC) {
            renc_a(ST, kt);
            char* bbase = lds + decltype(ST)::value * STAGE_B + BM * 128 + wave * NB * 1024;
#pragma unroll
            for (int j = 0; j < NB; j++) dma16(rw, bbase + j * 1024, wo[j], k0 * 4);
            if ((kt + 1) * BK < K) issue_w0(std::integral_constant<int, 1 - decltype(ST)::value>{}, kt + 1);
            return;
        }
        if (k0 < a0.k) {
            if (AMODE == GM_A_DENSE) {
#pragma unroll
                for (int j = 0; j < NA; j++) dma16(r0a, base + j * 1024, so[j][0], k0 * 4);
            } else if constexpr (AMODE == GM_A_READOUT) {
                const int seg = k0 / a0.hidden, ko = (k0 - seg * a0.hidden) * 4;
                // OOB + ko stays out of range, so missing neighbours need no select
                switch (seg) {
                    case 0:
#pragma unroll
                        for (int j = 0; j < NA; j++) dma16(r0a, base + j * 1024, so[j][0], ko);
                        break;
                    case 1:
#pragma unroll
                        for (int j = 0; j < NA; j++) dma16(r0b, base + j * 1024, so[j][1], ko);
                        break;
                    case 2:
#pragma unroll
                        for (int j = 0; j < NA; j++) dma16(r0b, base + j * 1024, so[j][2], ko);
                        break;
                    default:
#pragma unroll
                        for (int j = 0; j < NA; j++) dma16(r0b, base + j * 1024, so[j][3], ko);
                        break;
                }
            }
        } else {
            const int kk = k0 - a0.k;
#pragma unroll
            for (int j = 0; j < NA; j++) dma16(r1, base + j * 1024, o1[j], kk * 4);
        }
        char* bbase = lds + decltype(ST)::value * STAGE_B + BM * 128 + wave * NB * 1024;
#pragma unroll
        for (int j = 0; j < NB; j++) dma16(rw, bbase + j * 1024, wo[j], k0 * 4);
    };

    // EPI_DGRAD: the tile's sign words are loaded before the k loop (their latency hides under it)
    // and staged in LDS after it; MW words per thread
    constexpr int MW = EPI == EPI_DGRAD ? BM * (BN / 32) / (NW * 64) : 0;
    static_assert(EPI != EPI_DGRAD || MW * NW * 64 == BM * (BN / 32), "sign words per thread");
    unsigned mw[MW > 0 ? MW : 1];
    if constexpr (EPI == EPI_DGRAD) {
        if (ep.mbits) {
#pragma unroll
            for (int q = 0; q < MW; q++) {
                const int e = tid + q * NW * 64, r = e / (BN / 32), wd = e - r * (BN / 32);
                const int row = m0 + r, col0 = n0 + 32 * wd;
                mw[q] = (row < M && col0 < ep.split) ? ep.mbits[(long long)row * ep.ldmb + (col0 >> 5)] : ~0u;
            }
        }
    }
    std::conditional_t<MF == 1, CIn16<2 * TM, EPI>, CIn<TM, EPI>> cin;
    if constexpr (MF == 1)
        cin_load16<2 * TM, EPI>(cin, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, lane);
    else
        cin_load<TM, EPI>(cin, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, lane);
    floatx16 acc[TM][TN];
    floatx4 acc4[2 * TM][2 * TN];
    // LOACC (ping-pong loop, not the chain: it would spill): the a_lo' w_hi products in their own accumulators
    constexpr bool LOACC = MF == 1 && NW == 8 && STAGES <= 3 && EPI != EPI_CHAIN;
    floatx4 acc4l[LOACC ? 2 * TM : 1][LOACC ? 2 * TN : 1];
#pragma unroll
    for (int i = 0; i < (LOACC ? 2 * TM : 1); i++)
#pragma unroll
        for (int j = 0; j < (LOACC ? 2 * TN : 1); j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc4l[i][j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * TM; i++)
#pragma unroll
        for (int j = 0; j < 2 * TN; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc4[i][j][r] = 0.f;

    const int h = lane >> 5, l32 = lane & 31;
    const int gsw = (l32 >> 1) & 7;  // swizzle of every fragment row this lane reads
    // per-lane fragment byte offsets inside a stage: A chunks (4 sb + 2 h + p), B hi/lo chunks
    // (4 sb + 2 p + h); the stage and fragment-row offsets are immediates
    int aoff[2][2], boff[2][2];
#pragma unroll
    for (int sb = 0; sb < 2; sb++)
#pragma unroll
        for (int p = 0; p < 2; p++) {
            aoff[sb][p] = (wr * TM * 32 + l32) * 128 + (((4 * sb + 2 * h + p) ^ gsw) << 4);
            boff[sb][p] = BM * 128 + (wc * TN * 32 + l32) * 128 + (((4 * sb + 2 * p + h) ^ gsw) << 4);
        }
    // 16x16 form: A chunks 2q + p (q = l >> 4: k 8q..8q+7), B hi / lo chunks 4 (q >> 1) + 2 hl + (q & 1)
    // of rows (l & 15) + 16 x block; the row swizzle ((row >> 1) & 7) is the same for every block
    int aoff16[2], boff16[2];
    {
        const int q = lane >> 4, r16 = lane & 15, sw = gswz<MF>((r16 >> 1) & 7);
#pragma unroll
        for (int p = 0; p < 2; p++) {
            aoff16[p] = (wr * TM * 32 + r16) * 128 + (((2 * q + p) ^ sw) << 4);
            boff16[p] = BM * 128 + (wc * TN * 32 + r16) * 128 + (((4 * (q >> 1) + 2 * p + (q & 1)) ^ sw) << 4);
        }
    }
    half8 sah[2 * TM], sal[2 * TM];  // 16x16 form: split A of the current k tile (both column halves)
    constexpr bool PINGPONG = MF == 1 && NW == 8 && STAGES <= 3;
    const bool late = wave >= NW / 2;  // wave-uniform (readfirstlane)
    const _Float16 s12 = (_Float16)(1.0f / LO_S);
    const float ascale = AX == 2 ? *a0.scale : 1.0f;
    const int aexp = __builtin_amdgcn_frexp_expf(ascale) - 1;  // ascale = 2^aexp
    // epilogue scales read here, not after the k loop, so their latency hides under it
    const float wsi0 = *wscale_inv;
    const float wsi3 = EPI == EPI_CHAIN ? *ep.wsi2 : 1.0f;
    float amx = 0.f;  // AX 1: max |A| over the fragments this lane reads (all A elements of the tile
                      // are read by some lane of every column wave; ragged columns zeroed first)
    // fragments of one 16-deep half (SB) of a k tile: A raw fp32 (split at use), B hi / lo
    struct Frag {
        floatx4 xa[MF == 1 ? 2 * TM : TM][2];
        half8 bh[TN], bl[TN];
    };
    auto read = [&](auto ST, auto SB, Frag& f) {
        constexpr int sb = decltype(SB)::value;
        const char* sbase = lds + decltype(ST)::value * STAGE_B;
        if constexpr (MF == 1) {  // half sb: A (half 0 only) and B blocks sb TN .. sb TN + TN - 1
            if constexpr (sb == 0) {
#pragma unroll
                for (int i = 0; i < 2 * TM; i++) {
                    f.xa[i][0] = *reinterpret_cast<const floatx4*>(sbase + aoff16[0] + i * 16 * 128);
                    f.xa[i][1] = *reinterpret_cast<const floatx4*>(sbase + aoff16[1] + i * 16 * 128);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; j++) {
                f.bh[j] = *reinterpret_cast<const half8*>(sbase + boff16[0] + (sb * TN + j) * 16 * 128);
                f.bl[j] = *reinterpret_cast<const half8*>(sbase + boff16[1] + (sb * TN + j) * 16 * 128);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < TM; i++) {
            f.xa[i][0] = *reinterpret_cast<const floatx4*>(sbase + aoff[sb][0] + i * 32 * 128);
            f.xa[i][1] = *reinterpret_cast<const floatx4*>(sbase + aoff[sb][1] + i * 32 * 128);
        }
#pragma unroll
        for (int j = 0; j < TN; j++) {
            f.bh[j] = *reinterpret_cast<const half8*>(sbase + boff[sb][0] + j * 32 * 128);
            f.bl[j] = *reinterpret_cast<const half8*>(sbase + boff[sb][1] + j * 32 * 128);
        }
    };
    // split row block i of f's raw A into (h, l) (the same bits as the in-segment split)
    auto split_blk = [&](const Frag& f, int i, half8& h, half8& l) {
        floatx4 x0 = f.xa[i][0], x1 = f.xa[i][1];
        if constexpr (AX == 1) {
#pragma unroll
            for (int e = 0; e < 4; e++) amx = fmaxf(amx, fmaxf(fabsf(x0[e]), fabsf(x1[e])));
        }
        split8(x0, x1, h, l, AX == 2 ? aexp : 0);
    };
    // the MFMAs of column half sb of the current tile on a split A held in (ch, cl) (ping-pong loop)
    auto mfma16s = [&](const Frag& f, auto SB, half8 (&ch)[2 * TM], half8 (&cl)[2 * TM]) {
        constexpr int sb = decltype(SB)::value;
#pragma unroll
        for (int j = 0; j < TN; j++) {
            if constexpr (LOACC) {
            // a_lo' w_hi (scaled 2^12 by the split) into its own accumulators, scaled once after the k loop:
            // no per-tile w_hi * 2^-12 VALU
#pragma unroll
            for (int i = 0; i < 2 * TM; i++) {
                floatx4& c = acc4[i][sb * TN + j];
                floatx4& cl4 = acc4l[i][sb * TN + j];
                cl4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(cl[i], f.bh[j], cl4, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch[i], f.bl[j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch[i], f.bh[j], c, 0, 0, 0);
            }
            } else {
            const half8 bs = f.bh[j] * s12;  // w_hi * 2^-12, exact
#pragma unroll
            for (int i = 0; i < 2 * TM; i++) {
                floatx4& c = acc4[i][sb * TN + j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(cl[i], bs, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch[i], f.bl[j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch[i], f.bh[j], c, 0, 0, 0);
            }
            }
        }
    };
    auto mfma16 = [&](const Frag& f, auto SB, auto J0, auto J1) {
        constexpr int sb = decltype(SB)::value;
        constexpr int j0 = decltype(J0)::value, j1 = decltype(J1)::value;
        if constexpr (sb == 0 && j0 == 0) {
#pragma unroll
            for (int i = 0; i < 2 * TM; i++) {
                floatx4 x0 = f.xa[i][0], x1 = f.xa[i][1];
                if constexpr (AX == 1) {
#pragma unroll
                    for (int e = 0; e < 4; e++) amx = fmaxf(amx, fmaxf(fabsf(x0[e]), fabsf(x1[e])));
                }
                split8(x0, x1, sah[i], sal[i], AX == 2 ? aexp : 0);
            }
        }
#pragma unroll
        for (int j = j0; j < j1; j++) {
            const half8 bs = f.bh[j] * s12;  // w_hi * 2^-12, exact
#pragma unroll
            for (int i = 0; i < 2 * TM; i++) {
                floatx4& c = acc4[i][sb * TN + j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(sal[i], bs, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(sah[i], f.bl[j], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(sah[i], f.bh[j], c, 0, 0, 0);
            }
        }
    };
    auto mfma = [&](const Frag& f) {
        half8 ah[TM], al[TM];
#pragma unroll
        for (int i = 0; i < TM; i++) {
            floatx4 x0 = f.xa[i][0], x1 = f.xa[i][1];
            if constexpr (AX == 1) {
#pragma unroll
                for (int e = 0; e < 4; e++) amx = fmaxf(amx, fmaxf(fabsf(x0[e]), fabsf(x1[e])));
            }
            split8(x0, x1, ah[i], al[i], AX == 2 ? aexp : 0);
        }
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const half8 bs = f.bh[j] * s12;  // w_hi * 2^-12, exact
#pragma unroll
            for (int i = 0; i < TM; i++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bs, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], f.bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], f.bh[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    const int nk = (K + BK - 1) / BK;
    // the DMA reads whatever lies past a ragged source end (in-buffer data, or zeros out of
    // range); once the last tile has landed, those A columns are zeroed in LDS (all waves,
    // then a barrier) before its first fragment read
    const int kend_last = (nk - 1) * BK < a0.k ? a0.k : K;
    const bool ragged = kend_last < nk * BK;
    auto zero_tail = [&](auto ST) {
        char* sa = lds + decltype(ST)::value * STAGE_B;
        for (int e = tid; e < BM * BK; e += NW * 64) {
            const int r = e / BK, c = e % BK;
            if ((nk - 1) * BK + c >= kend_last)
                *reinterpret_cast<float*>(sa + r * 128 + ((((c >> 2) ^ gswz<MF>((r >> 1) & 7))) << 4) + (c & 3) * 4) = 0.f;
        }
        __syncthreads();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    // Pipeline, one barrier per k tile placed MID-step: tile t lives in stage t % STAGES.
    //   step k: read half 1 of tile k | MFMAs half 0 of tile k | wait own DMA of tile k+1,
    //   lgkmcnt(0), barrier B_k | DMA tile k+STAGES into stage k (every wave is past its reads
    //   of tile k) | read half 0 of tile k+1 | MFMAs half 1 of tile k
    // so every fragment read overlaps the MFMAs of the other half, and a DMA has STAGES-1
    // steps to land.
    if constexpr (PINGPONG) {
        // one tile read, split and multiplied per barrier; STAGES - 1 tiles in flight
        Frag fa, fb;
        auto mfma_all = [&]() {
            mfma16s(fa, I0{}, sah, sal);
            mfma16s(fb, I1{}, sah, sal);
        };
        head_load();
        if constexpr (RENC) {  // the first slice lands and is published before tile 0's A is computed
            issue_w0(std::integral_constant<int, 0>{}, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        issue(I0{}, 0);
        if constexpr (STAGES == 3)
            if (nk > 1) issue(I1{}, 1);
        head_store();
        auto pp_step = [&](auto ST, int kt) {
            constexpr int S = decltype(ST)::value;
            using SI = std::integral_constant<int, (S + STAGES - 1) % STAGES>;  // stage of tile kt + STAGES - 1
            // own DMA of tile kt landed (with 3 stages tile kt + 1 may stay in flight); own reads done
            if (STAGES == 3 && kt + 1 < nk)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");  // no LDS access moves across the barrier
            GM_STAMP(kt, 0);
            if (ragged && kt == nk - 1) zero_tail(ST);
            if (late && kt > 0) {  // the previous tile, from registers
                __builtin_amdgcn_sched_barrier(0);
                mfma_all();
            }
            __builtin_amdgcn_sched_barrier(0);
            GM_STAMP(kt, 1);
            if (RENC && kt + STAGES - 1 < nk) issue(SI{}, kt + STAGES - 1);  // into the stage of tile kt - 1
            GM_STAMP(kt, 2);
            read(ST, I0{}, fa);
            read(ST, I1{}, fb);
            if (!RENC && kt + STAGES - 1 < nk) issue(SI{}, kt + STAGES - 1);  // behind the reads (guide: cheaper)
#pragma unroll
            for (int i = 0; i < 2 * TM; i++) {
                if constexpr (RENC) {  // stored split (renc_a): hi / lo chunks as read
                    sah[i] = __builtin_bit_cast(half8, fa.xa[i][0]);
                    sal[i] = __builtin_bit_cast(half8, fa.xa[i][1]);
                } else {
                    split_blk(fa, i, sah[i], sal[i]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            GM_STAMP(kt, 3);
            if (!late) {
                mfma_all();
                __builtin_amdgcn_sched_barrier(0);
            }
            GM_STAMP(kt, 4);
        };
        for (int kt = 0; kt < nk; kt += STAGES) {
            pp_step(I0{}, kt);
            if (kt + 1 < nk) pp_step(I1{}, kt + 1);
            if constexpr (STAGES == 3)
                if (kt + 2 < nk) pp_step(I2{}, kt + 2);
        }
        if (late) mfma_all();  // the last tile
    } else {
    head_load();
    issue(I0{}, 0);
    if (nk > 1) issue(I1{}, 1);
    if constexpr (STAGES >= 3)
        if (nk > 2) issue(I2{}, 2);
    if constexpr (STAGES >= 4)
        if (nk > 3) issue(I3{}, 3);
    head_store();
    // wait until this wave's DMA of the oldest tile landed, n younger tiles left in flight
    auto wait_landed = [&](int n) {
        if (n >= 3)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NL) : "memory");
        else if (n == 2)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL) : "memory");
        else if (n == 1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    wait_landed(min(STAGES - 1, nk - 1));  // tiles issued after tile 0
    // head_store's LDS writes are read by other waves in the epilogue: publish them here too (with
    // nk == 1 no later barrier of the k loop would)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ragged && nk == 1) zero_tail(I0{});
    Frag f0, f1;
    read(I0{}, I0{}, f0);
    auto step = [&](auto ST, int kt) {
        constexpr int S = decltype(ST)::value;
        using SN = std::integral_constant<int, (S + 1) % STAGES>;
        GM_STAMP(kt, 0);
        read(ST, I1{}, f1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MF == 1)
            mfma16(f0, I0{}, I0{}, std::integral_constant<int, TN>{});
        else
            mfma(f0);
        __builtin_amdgcn_sched_barrier(0);
        GM_STAMP(kt, 1);
        if (kt + 1 < nk) {
            // own DMA of tile kt+1 landed (tiles kt+2 .. kt+STAGES-1 may stay in flight)
            wait_landed(min(STAGES - 2, nk - 2 - kt));
            GM_STAMP(kt, 2);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of tile kt done
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");  // no LDS access moves across the barrier
            GM_STAMP(kt, 3);
            if (kt + STAGES < nk) issue(ST, kt + STAGES);
            GM_STAMP(kt, 4);
            if (ragged && kt + 1 == nk - 1) zero_tail(SN{});
            read(SN{}, I0{}, f0);
        }
        GM_STAMP(kt, 5);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MF == 1)
            mfma16(f1, I1{}, I0{}, std::integral_constant<int, TN>{});
        else
            mfma(f1);
        GM_STAMP(kt, 6);
    };
    for (int kt = 0; kt < nk; kt += STAGES) {
        step(I0{}, kt);
        if (kt + 1 < nk) step(I1{}, kt + 1);
        if constexpr (STAGES >= 3)
            if (kt + 2 < nk) step(I2{}, kt + 2);
        if constexpr (STAGES >= 4)
            if (kt + 3 < nk) step(I3{}, kt + 3);
    }
    }  // !PINGPONG

#if GM_DIAG == 30
    if (stw && g_stamps && blockIdx.x < 4096)
        for (int i = 0; i < 64; i++) g_stamps[((size_t)blockIdx.x * 2 + (wave != 0)) * 64 + i] = stl[(wave != 0) * 64 + i];
#endif
    if constexpr (AX == 1) {
        amx = gm_wave_max(amx);
        if (lane == 0) gm_amax_publish(a0.amax, amx);
    }
    const float si = wsi0 / ascale;  // undo the weight and A scales (powers of two: exact)
    if constexpr (LOACC) {
#pragma unroll
        for (int i = 0; i < 2 * TM; i++)
#pragma unroll
            for (int j = 0; j < 2 * TN; j++)
#pragma unroll
                for (int r = 0; r < 4; r++) acc4[i][j][r] += acc4l[i][j][r] * (1.0f / LO_S);
    }
    if constexpr (MF == 1) {
#pragma unroll
        for (int i = 0; i < 2 * TM; i++)
#pragma unroll
            for (int j = 0; j < 2 * TN; j++)
#pragma unroll
                for (int r = 0; r < 4; r++) acc4[i][j][r] *= si;
        range_guard16<2 * TM, 2 * TN>(acc4, ep.range_flag, lane);
        if constexpr (EPI == EPI_DGRAD) {
            __syncthreads();  // every wave is past its last fragment reads: LDS is scratch from here
            if (ep.mbits) {
                unsigned* smb = reinterpret_cast<unsigned*>(lds) + WGM * BN;
#pragma unroll
                for (int q = 0; q < MW; q++) smb[tid + q * NW * 64] = mw[q];
                __syncthreads();
            }
            dgrad_epilogue16<WGM, WGN, 2 * TM, 2 * TN, true>(acc4, ep, reinterpret_cast<float*>(lds), m0, n0, wr, wc, M,
                                                             N, lane);
        } else if constexpr (EPI == EPI_HEAD)
            act_dispatch(ep.act, [&](auto A) {
                head_epilogue16<2 * TM, 2 * TN, WGN, BM, decltype(A)::value>(acc4, ep, lds, m0, wr, wc, M, N, lane, tid, n0,
                                                                             hlds);
            });
        else if constexpr (EPI == EPI_CHAIN)
            act_dispatch(ep.act, [&](auto A) {
                chain_tail<WGM, WGN, 2 * TM, 2 * TN, BM, 128, 4, decltype(A)::value>(acc4, ep, lds, m0, wr, wc, M, lane, hlds,
                                                                                       wsi3);
            });
        else
            if constexpr (EPI == EPI_BIAS)
                act_dispatch(ep.act, [&](auto A) {
                    epilogue16<2 * TM, 2 * TN, EPI, decltype(A)::value>(acc4, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M,
                                                                        N, lane, cin, hlds + wc * TN * 32);
                });
            else
                epilogue16<2 * TM, 2 * TN, EPI>(acc4, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane, cin,
                                                EPI == EPI_LSTM ? hlds + wc * TN * 32 : nullptr);
    } else {
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
            for (int j = 0; j < TN; j++)
#pragma unroll
                for (int r = 0; r < 16; r++) acc[i][j][r] *= si;
        range_guard<TM, TN>(acc, ep.range_flag, lane);
        if constexpr (EPI == EPI_DGRAD) {
            __syncthreads();
            if (ep.mbits) {
                unsigned* smb = reinterpret_cast<unsigned*>(lds) + WGM * BN;
#pragma unroll
                for (int q = 0; q < MW; q++) smb[tid + q * NW * 64] = mw[q];
                __syncthreads();
            }
            dgrad_epilogue<WGM, WGN, TM, TN, true>(acc, ep, reinterpret_cast<float*>(lds), m0, n0, wr, wc, M, N, lane);
        } else if constexpr (EPI == EPI_HEAD)
            act_dispatch(ep.act, [&](auto A) {
                head_epilogue<TM, TN, WGN, BM, decltype(A)::value>(acc, ep, lds, m0, wr, wc, M, N, lane, tid);
            });
        else if constexpr (EPI == EPI_BIAS)
            act_dispatch(ep.act, [&](auto A) {
                epilogue<TM, TN, EPI, decltype(A)::value>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane, cin);
            });
        else if constexpr (EPI != EPI_CHAIN)  // EPI_CHAIN: the 16x16x32 form only
            epilogue<TM, TN, EPI>(acc, ep, m0 + wr * TM * 32, n0 + wc * TN * 32, M, N, lane, cin);
    }
}

// k_gemm3g MFMA shape (gm_gemm_set_mfma): 2 16x16x32 everywhere (default), 1 16x16x32 except the
// fused Q head (32x32x16), 0 32x32x16 everywhere. The head on 16x16x32 measured 89.5 -> 105 us per
// 81920 rows before the 16x16 row swizzle (gswz) removed its 2-way ds_read_b128 conflicts; since
// then it runs as fast as on 32x32x16 and the whole rollout gains 0.6 % with every GEMM on one shape
// (5.54-5.55 -> 5.57-5.59 M env-steps/s, three interleaved pairs on one box)
int g_mfma16 = 2;
// input-gradient kernel (gm_gemm_set_dgrad): -1 per-shape default, 0 k_gemm3 128x128, 1 k_gemm3g
// 128x128 (4 waves), 2 k_gemm3g 128x256 (8 waves)
int g_dgrad = -1;

template <int WGM, int WGN, int TM, int TN, int STAGES, int AMODE, int EPI, int OCC, int AX = 0>
int launch_g(const ASrc& a0, const ASrc& a1, const float* w, long long ldw, unsigned wbytes, int M, int N, int K,
             const Epi& ep, hipStream_t st, const float* wscale_inv, int mf = -1) {
    constexpr int BM = WGM * TM * 32, BN = WGN * TN * 32;
    const int T = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if constexpr (AMODE == GM_A_ROUTING_ENC)  // 16x16x32 only
        hipLaunchKernelGGL((k_gemm3g<WGM, WGN, TM, TN, STAGES, AMODE, EPI, OCC, AX, 1>), dim3(T), dim3(WGM * WGN * 64), 0,
                           st, a0, a1, reinterpret_cast<const _Float16*>(w), ldw, wbytes, M, N, K, ep, wscale_inv);
    else if (mf < 0 ? g_mfma16 : mf)
        hipLaunchKernelGGL((k_gemm3g<WGM, WGN, TM, TN, STAGES, AMODE, EPI, OCC, AX, 1>), dim3(T), dim3(WGM * WGN * 64), 0,
                           st, a0, a1, reinterpret_cast<const _Float16*>(w), ldw, wbytes, M, N, K, ep, wscale_inv);
    else
        hipLaunchKernelGGL((k_gemm3g<WGM, WGN, TM, TN, STAGES, AMODE, EPI, OCC, AX, 0>), dim3(T), dim3(WGM * WGN * 64), 0,
                           st, a0, a1, reinterpret_cast<const _Float16*>(w), ldw, wbytes, M, N, K, ep, wscale_inv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gemm launch: ") + hipGetErrorString(e));
    return GM_OK;
}

template <int WGM, int WGN, int TM, int TN, int BK_, int AMODE, int EPI, int OCC = 2, bool X3 = false>
int launch(const ASrc& a0, const ASrc& a1, const float* w, long long ldw, unsigned wbytes, int M, int N, int K,
           const Epi& ep, hipStream_t st, const float* wscale_inv = nullptr) {
    using C = Cfg<WGM, WGN, TM, TN, BK_>;
    const int T = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
    if constexpr (X3)
        hipLaunchKernelGGL((k_gemm3<WGM, WGN, TM, TN, BK_, AMODE, EPI, OCC>), dim3(T), dim3(C::THREADS), 0, st, a0, a1,
                           reinterpret_cast<const _Float16*>(w), ldw, wbytes, M, N, K, ep, wscale_inv);
    else
        hipLaunchKernelGGL((k_gemm<WGM, WGN, TM, TN, BK_, AMODE, EPI, OCC>), dim3(T), dim3(C::THREADS), 0, st, a0, a1, w,
                           ldw, wbytes, M, N, K, ep);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gemm launch: ") + hipGetErrorString(e));
    return GM_OK;
}

// activation of a bias epilogue code: GM_EPI_BIAS none, GM_EPI_BIAS_LEAKY leaky_relu, GM_EPI_BIAS_RELU ..
// GM_EPI_BIAS_SIGMOID -> GM_ACT_RELU .. GM_ACT_SIGMOID
int epi_act(int epilogue) {
    if (epilogue == GM_EPI_BIAS_LEAKY) return GM_ACT_LEAKY_RELU;
    if (epilogue >= GM_EPI_BIAS_RELU && epilogue <= GM_EPI_BIAS_SIGMOID) return GM_ACT_RELU + (epilogue - GM_EPI_BIAS_RELU);
    if (epilogue >= GM_EPI_BIAS_ACT && epilogue <= GM_EPI_BIAS_ACT + GM_ACT_LAST) return epilogue - GM_EPI_BIAS_ACT;
    return GM_ACT_NONE;
}
bool is_bias_epi(int e) {
    return e == GM_EPI_BIAS || e == GM_EPI_BIAS_LEAKY || (e >= GM_EPI_BIAS_RELU && e <= GM_EPI_BIAS_SIGMOID) ||
           (e >= GM_EPI_BIAS_ACT && e <= GM_EPI_BIAS_ACT + GM_ACT_LAST);
}

int g_tile = -1;  // tile configuration override (gm_gemm_set_tile), -1 = per-shape default

bool fits(long long bytes) { return bytes >= 0 && bytes < (1ll << 31) - (1 << 24); }

int to_asrc_any(const gm_a_src* s, int M, ASrc& o) {
    memset(&o, 0, sizeof(o));
    if (!s) return GM_OK;
    o.mode = s->mode;
    o.p0 = s->p0;
    o.p1 = s->p1;
    o.ld0 = s->ld0;
    o.ld1 = s->ld1;
    o.nbr = s->nbr;
    o.agent_node = s->agent_node;
    o.n_nodes = s->n_nodes;
    o.deg = s->deg;
    o.mean = s->mean;
    o.rows_per_graph = s->rows_per_graph;
    o.k = s->k;
    o.hidden = s->hidden;
    o.scale = s->scale;
    o.amax = reinterpret_cast<unsigned*>(s->amax);
    o.bias0 = s->bias0;
    o.act0 = s->act0;
    if (s->scale && s->mode != GM_A_DENSE)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm: an A scale needs a DENSE source");
    if (s->mode == GM_A_ROUTING_ENC) {
        const long long K0 = 4ll * s->n_nodes + 8;
        if (!s->p0 || !s->p1 || !s->nbr || s->deg != 3 || s->n_nodes < 4 || K0 > GM_RENC_ROWS || s->k <= 0 || (s->k % BKMAX) ||
            s->k > 1024 || s->ld0 < K0 || s->ld1 < s->k || (s->ld1 & 3) || (reinterpret_cast<uintptr_t>(s->p1) & 15) ||
            (M % s->n_nodes) || s->act0 < GM_ACT_NONE || s->act0 > GM_ACT_LAST || s->amax)
            return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm: routing-encoder source needs deg 3, 4N + 8 <= 208, k % 32 == 0, "
                                               "k <= 1024, ld1 >= k (16-byte W0^T rows), M = G * N");
        o.bytes0 = ((long long)(M - 1) * s->ld0 + K0) * 4;
        o.bytes1 = ((K0 - 1) * s->ld1 + s->k) * 4;
        if (!fits(o.bytes0) || !fits(o.bytes1)) return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm: routing-encoder source > 2 GB");
        return GM_OK;
    }
    if (!s->p0 || s->k <= 0 || (s->ld0 & 3) || (reinterpret_cast<uintptr_t>(s->p0) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: A source needs p0, k > 0, ld0 % 4 == 0, 16-byte base");
    long long rows0 = M;
    if (s->mode == GM_A_DENSE) {
        if (s->ld0 < s->k) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: dense ld0 < k");
    } else {
        if (!s->nbr || s->n_nodes <= 0 || s->deg < 0 || s->deg > 3)
            return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: gather source needs nbr, n_nodes, deg <= 3");
        if (s->mode == GM_A_AGGREGATE) {
            if (s->ld0 < s->k) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: aggregate ld0 < k");
        } else if (s->mode == GM_A_READOUT) {
            if (!s->p1 || !s->agent_node || s->rows_per_graph <= 0 || s->hidden <= 0 || (s->hidden % BKMAX) ||
                s->k != (s->deg + 1) * s->hidden || (s->ld1 & 3) || (reinterpret_cast<uintptr_t>(s->p1) & 15) ||
                (M % s->rows_per_graph))
                return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: readout source: hidden % 32 == 0, k = (deg+1)*hidden");
            rows0 = (long long)(M / s->rows_per_graph) * s->n_nodes;
            long long b1 = ((rows0 - 1) * s->ld1 + s->hidden) * 4;
            if (!fits(b1)) return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm_f32: source larger than 2 GB");
            o.bytes1 = b1;
        } else {
            return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: unknown A source mode");
        }
    }
    long long width = s->mode == GM_A_READOUT ? s->hidden : s->k;
    long long b0 = ((rows0 - 1) * s->ld0 + width) * 4;
    // dense rows are addressed from the block's first row (any size); gathered sources are not
    if (s->mode != GM_A_DENSE && !fits(b0))
        return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm_f32: gathered source larger than 2 GB (split M)");
    o.bytes0 = b0;
    return GM_OK;
}

// the A sources of every entry but gm_gemm_x3: no ROUTING_ENC
int to_asrc(const gm_a_src* s, int M, ASrc& o, bool renc_ok = false) {
    if (s && s->mode == GM_A_ROUTING_ENC && !renc_ok)
        return gm_fail(GM_ERR_UNSUPPORTED, "routing-encoder A source: gm_gemm_x3 only");
    return to_asrc_any(s, M, o);
}

// Tile tables. F32: per-shape default from tools/gemm_bench.py on MI355X (BK=16 for short
// K, narrow N and the readout layer; BK=32 for K=512, N>=256). X3: 128x128x16 tiles
// (49 KB of LDS: 3 blocks/CU), LSTM 128 rows x 4 gate tiles.
template <bool X3>
int dispatch(const ASrc& s0, const ASrc& s1, const float* w, long long ldw, unsigned wb, int m, int n, int K,
             int epilogue, Epi& ep, hipStream_t st, const float* wsi) {
    const int tile = g_tile;
#define GM_L(WGM, WGN, TM, TN, BK_, AM, EP) \
    launch<WGM, WGN, TM, TN, BK_, AM, EP, 2, X3>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
#define GM_L4(WGM, WGN, TM, TN, BK_, AM, EP) \
    launch<WGM, WGN, TM, TN, BK_, AM, EP, 4, X3>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
    if constexpr (X3) {
        // LDS-DMA kernel (tiles 8..14) for dense / readout sources
#define GM_G(WGM, WGN, TM, TN, S, AM, EP, OC) \
    launch_g<WGM, WGN, TM, TN, S, AM, EP, OC>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
        // defaults (tools/gemm_bench.py on MI355X): the readout-sourced DQN layer (the rollout's
        // largest GEMM) on tile 10; wide dense layers with K >= 256 at rollout batch sizes (incl.
        // the LSTM gate GEMMs on [x | h]) on tile 12 (128x128, 2 blocks/CU: 7-11 % faster than
        // k_gemm3 at 81920 rows); narrow or short-K layers on k_gemm3
        // training operands (forward GEMMs publishing max|A|, input-gradient GEMMs on a scaled A):
        // the LDS-DMA kernel's 128x128 tile at 2 blocks/CU for large dense GEMMs, k_gemm3 otherwise
        const int ax = s0.amax ? 1 : (s0.scale ? 2 : 0);
        if (s0.mode == GM_A_ROUTING_ENC) {  // the A tile computed in the block: 128 x 256 ping-pong tile, 2 stages,
                                            // always on 16x16x32 (whatever gm_gemm_set_mfma selects elsewhere)
            if (!is_bias_epi(epilogue) || s1.p0)
                return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm_x3: routing-encoder source needs a bias epilogue and no "
                                                   "second source");
            ep.act = epi_act(epilogue);
            return launch_g<4, 2, 1, 4, 2, GM_A_ROUTING_ENC, EPI_BIAS, 1>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi, 1);
        }
        int gt = 0;
        if (ax) {
            // tools/train_gemm_bench.py at 262 160 rows: wide forward layers (N >= 256, K >= 512) gain
            // 3-5 % on the 128x128 LDS-DMA tile, short-K and input-gradient GEMMs do not
            // round 6: wide bias layers on the 8-wave ping-pong tile 9 (second accumulator set), tools/gemm_bench.py
            // SHAPES=train at 1 M rows: DQN layer 1 (K = 642) 2 397 vs 2 630 us, K = 512 layers -4 %
            if (s0.mode == GM_A_DENSE && epilogue != GM_EPI_LSTM &&
                (tile == 9 || tile == 10 || (tile == -1 && m >= 32768 && n >= 256 && K >= 512)))
                gt = tile == 10 ? 10 : 9;
            // round 6 (row-bounded epilogue stores): the LSTM cells at K = 256 too, 437.5 vs 453.3 us at 262 160 rows
            // config 5's output head (N = 100, K = 512, 6.55 M rows): 4242 -> 3620 us on tile 12 (tools/train_gemm_bench.py)
            else if (s0.mode == GM_A_DENSE &&
                     (tile == 12 || tile == 13 ||
                      (tile == -1 && ax == 1 && m >= 32768 &&
                       ((n >= 256 && (K >= 512 || (epilogue == GM_EPI_LSTM && K >= 256))) ||
                        (n > 64 && K >= 512 && epilogue != GM_EPI_LSTM)))))
                gt = tile == 13 && epilogue != GM_EPI_LSTM ? 13 : 12;
        } else if (tile >= 8)
            gt = tile;
        else if (tile == -1 && s0.mode == GM_A_READOUT && n > 128)
            gt = 9;  // ping-pong: 3 stages (two tiles in flight) 177 -> 172 us for DQN layer 1
        else if (tile == -1 && s0.mode == GM_A_DENSE && n >= 256 && K >= 512 && m >= 32768 && is_bias_epi(epilogue))
            gt = 9;  // wide bias layers (the update's target DQN layer 1, config 5's encoder): as above
        else if (tile == -1 && s0.mode == GM_A_DENSE && n >= 128 && K >= 256 && m >= 32768)
            gt = 12;  // N = 128 (the encoder's last layer): 25.9 -> 21.4 us at 40 960 rows
#define GM_GX(WGM, WGN, TM, TN, EP, AXV) \
    launch_g<WGM, WGN, TM, TN, 2, GM_A_DENSE, EP, 2, AXV>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
        if (gt >= 8 && ax) {
            if (epilogue == GM_EPI_LSTM) {
                ep.hidden = n / 4;
                return ax == 1 ? GM_GX(4, 1, 1, 4, EPI_LSTM, 1) : GM_GX(4, 1, 1, 4, EPI_LSTM, 2);
            }
            ep.act = epi_act(epilogue);
            if (gt == 9)
                return ax == 1 ? launch_g<4, 2, 1, 4, 3, GM_A_DENSE, EPI_BIAS, 1, 1>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
                               : launch_g<4, 2, 1, 4, 3, GM_A_DENSE, EPI_BIAS, 1, 2>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi);
            if (gt == 10)
                return ax == 1 ? launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_BIAS, 1, 1>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi)
                               : launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_BIAS, 1, 2>(s0, s1, w, ldw, wb, m, n, K, ep, st, wsi);
            if (gt == 13) return ax == 1 ? GM_GX(2, 2, 2, 2, EPI_BIAS, 1) : GM_GX(2, 2, 2, 2, EPI_BIAS, 2);
            return ax == 1 ? GM_GX(4, 1, 1, 4, EPI_BIAS, 1) : GM_GX(4, 1, 1, 4, EPI_BIAS, 2);
        }
#undef GM_GX
        if (gt >= 8 && s0.mode != GM_A_AGGREGATE) {
            if (epilogue == GM_EPI_LSTM) {
                ep.hidden = n / 4;
                if (s0.mode != GM_A_DENSE) return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm: LSTM epilogue with readout source");
                switch (gt) {  // 8 waves each
                    case 8: return GM_G(4, 2, 2, 4, 2, GM_A_DENSE, EPI_LSTM, 1);   // 256x256
                    case 9: return GM_G(4, 2, 1, 4, 3, GM_A_DENSE, EPI_LSTM, 1);   // 128x256, 3 stages
                    case 10: return GM_G(4, 2, 1, 4, 2, GM_A_DENSE, EPI_LSTM, 1);  // 128x256, 2 stages
                    case 12:  // 128x128, 4 waves, 2 blocks/CU (tile 13's 64x64 waves cannot hold a gate group)
                    case 13: return GM_G(4, 1, 1, 4, 2, GM_A_DENSE, EPI_LSTM, 2);
                    case 14: return GM_G(2, 2, 2, 4, 2, GM_A_DENSE, EPI_LSTM, 1);  // 128x256, 64x128 waves
                    default: return GM_G(8, 1, 1, 4, 2, GM_A_DENSE, EPI_LSTM, 1);  // 256x128
                }
            }
            ep.act = epi_act(epilogue);
#define GM_GB(AM)                                                \
    switch (gt) {                                              \
        case 8: return GM_G(4, 2, 2, 4, 2, AM, EPI_BIAS, 1);     \
        case 9: return GM_G(4, 2, 1, 4, 3, AM, EPI_BIAS, 1);     \
        case 10: return GM_G(4, 2, 1, 4, 2, AM, EPI_BIAS, 1);    \
        case 12: return GM_G(4, 1, 1, 4, 2, AM, EPI_BIAS, 2);    \
        case 13: return GM_G(2, 2, 2, 2, 2, AM, EPI_BIAS, 2);    \
        case 14: return GM_G(2, 2, 2, 4, 2, AM, EPI_BIAS, 1);    \
        default: return GM_G(8, 1, 1, 4, 2, AM, EPI_BIAS, 1);    \
    }
            if (n > 32) {
                if (s0.mode == GM_A_READOUT) GM_GB(GM_A_READOUT)
                GM_GB(GM_A_DENSE)
            }
#undef GM_GB
        }
#undef GM_G
    }
    if (epilogue == GM_EPI_LSTM) {
        ep.hidden = n / 4;
        if constexpr (X3) {
            // 0: 128 rows x 4 gate tiles (4 waves of 32 rows); 1: 256 rows, 8 waves; 2: BK = 32
#define GM_LSTM3(AM)                                          \
    switch (tile) {                                           \
        case 1: return GM_L(8, 1, 1, 4, 16, AM, EPI_LSTM);    \
        case 2: return GM_L(4, 1, 1, 4, 32, AM, EPI_LSTM);    \
        default: return GM_L(4, 1, 1, 4, 16, AM, EPI_LSTM);   \
    }
            if (s0.mode == GM_A_DENSE) GM_LSTM3(GM_A_DENSE)
            if (s0.mode == GM_A_AGGREGATE) GM_LSTM3(GM_A_AGGREGATE)
#undef GM_LSTM3
        } else {
            // default: 128x128x16 at 4 blocks/CU (<= 128 VGPRs, 40 KB LDS): +20 % over 2 blocks/CU
            if (s0.mode == GM_A_DENSE) {
                if (tile == 0) return GM_L(4, 1, 1, 4, 32, GM_A_DENSE, EPI_LSTM);
                if (tile == 2) return GM_L(4, 1, 2, 4, 16, GM_A_DENSE, EPI_LSTM);
                return GM_L4(4, 1, 1, 4, 16, GM_A_DENSE, EPI_LSTM);
            }
            if (s0.mode == GM_A_AGGREGATE) {
                if (tile == 0) return GM_L(4, 1, 1, 4, 32, GM_A_AGGREGATE, EPI_LSTM);
                if (tile == 2) return GM_L(4, 1, 2, 4, 16, GM_A_AGGREGATE, EPI_LSTM);
                return GM_L4(4, 1, 1, 4, 16, GM_A_AGGREGATE, EPI_LSTM);
            }
        }
        return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm: LSTM epilogue with readout source");
    }
    ep.act = epi_act(epilogue);
    if constexpr (X3) {
        // 0: 128x128 (4 waves of 64x64); 1: 128x256, 8 waves; 2: 256x128, 8 waves; 3: BK = 32
#define GM_BIAS3(AM)                                          \
    switch (tile) {                                           \
        case 1: return GM_L(2, 4, 2, 2, 16, AM, EPI_BIAS);    \
        case 2: return GM_L(4, 2, 2, 2, 16, AM, EPI_BIAS);    \
        case 3: return GM_L(2, 2, 2, 2, 32, AM, EPI_BIAS);    \
        default: return GM_L(2, 2, 2, 2, 16, AM, EPI_BIAS);   \
    }
        if (s0.mode == GM_A_READOUT) GM_BIAS3(GM_A_READOUT)
        if (s0.mode == GM_A_AGGREGATE) GM_BIAS3(GM_A_AGGREGATE)
        if (n <= 32) return GM_L(1, 1, 1, 1, 16, GM_A_DENSE, EPI_BIAS);
        GM_BIAS3(GM_A_DENSE)
#undef GM_BIAS3
    } else {
    const int t = tile >= 0 ? tile : ((s0.mode == GM_A_READOUT || K <= 128 || n <= 128) ? 3 : 0);
    if (s0.mode == GM_A_READOUT) {
        if (t == 1) return GM_L(2, 2, 2, 4, 16, GM_A_READOUT, EPI_BIAS);
        if (t == 2) return GM_L(2, 2, 4, 2, 16, GM_A_READOUT, EPI_BIAS);
        if (t == 3) return GM_L(2, 2, 2, 2, 16, GM_A_READOUT, EPI_BIAS);
        if (t == 4) return GM_L4(2, 2, 2, 2, 16, GM_A_READOUT, EPI_BIAS);
        return GM_L(2, 2, 2, 2, 32, GM_A_READOUT, EPI_BIAS);
    }
    if (s0.mode == GM_A_AGGREGATE) return GM_L(2, 2, 2, 2, 32, GM_A_AGGREGATE, EPI_BIAS);
    if (n <= 32) return GM_L(4, 1, 1, 1, 32, GM_A_DENSE, EPI_BIAS);
    if (t == 1) return GM_L(2, 2, 2, 4, 16, GM_A_DENSE, EPI_BIAS);
    if (t == 2) return GM_L(2, 2, 4, 2, 16, GM_A_DENSE, EPI_BIAS);
    if (t == 3) return GM_L(2, 2, 2, 2, 16, GM_A_DENSE, EPI_BIAS);
    if (t == 4) return GM_L4(2, 2, 2, 2, 16, GM_A_DENSE, EPI_BIAS);
    return GM_L(2, 2, 2, 2, 32, GM_A_DENSE, EPI_BIAS);
    }
#undef GM_L
#undef GM_L4
}

// Status word of the split-f16 range guard: host memory mapped into the device address space
// (fine-grained, coherent), so the host reads what a finished kernel stored without a copy or a
// stream synchronisation. Allocated on the first x3 call.
unsigned* g_range_host = nullptr;
unsigned* g_range_dev = nullptr;

int range_flag(unsigned** dev) {
    if (!g_range_host) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return gm_fail(GM_ERR_HIP, "gm_gemm_x3: hipHostMalloc of the range status word failed");
        memset(p, 0, 64);
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess)
            return gm_fail(GM_ERR_HIP, "gm_gemm_x3: hipHostGetDevicePointer of the range status word failed");
        g_range_host = static_cast<unsigned*>(p);
        g_range_dev = static_cast<unsigned*>(d);
    }
    if (*reinterpret_cast<volatile unsigned*>(g_range_host))
        return gm_fail(GM_ERR_RANGE,
                       "gm_gemm_x3: an earlier split-f16 GEMM produced a non-finite accumulator (an A operand "
                       "outside the f16 range, |a| >= 2^15 possible); its outputs are invalid: rerun with the exact "
                       "form (GM_GEMM=f32) or clear with gm_gemm_range_status(.., 1)");
    *dev = g_range_dev;
    return GM_OK;
}

// shared argument checks of gm_gemm_f32 / gm_gemm_x3; x3: w = packed weights
int gemm_entry(bool x3, const gm_a_src* a0, const gm_a_src* a1, const void* w, int64_t ldw, const float* wsi,
               const float* b, int32_t m, int32_t n, int32_t epilogue, float* y, int64_t ldy, float* y2,
               int64_t ldy2, const float* c_in, int64_t ldc, float* act_out, void* stream) {
    const char* fn = x3 ? "gm_gemm_x3" : "gm_gemm_f32";
    if (!a0 || !w || !y || m <= 0 || n <= 0 || (reinterpret_cast<uintptr_t>(w) & 15) || (!x3 && (ldw & 3)) ||
        (x3 && !wsi))
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": bad arguments");
    ASrc s0, s1;
    int rc = to_asrc(a0, m, s0, x3);
    if (rc) return rc;
    rc = to_asrc(a1, m, s1);
    if (rc) return rc;
    if (s0.scale && (!x3 || a1 || s1.scale))
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": an A scale needs the x3 form and a single source");
    if ((s0.amax && !x3) || s1.amax)
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": amax needs the x3 form and goes on src0");
    if (a1 && (a1->mode != GM_A_DENSE || (s0.k % BKMAX)))
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": second A source must be dense and the first k % 32 == 0");
    const int K = s0.k + (a1 ? s1.k : 0);
    long long wb;
    if (x3) {
        ldw = (long long)((K + BKMAX - 1) / BKMAX * BKMAX) / 16 * 64;  // packed row bytes
        wb = (long long)n * ldw;
    } else {
        if (ldw < K) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_f32: ldw < K");
        wb = ((long long)(n - 1) * ldw + ((K + 3) & ~3)) * 4;
    }
    if (!fits(wb)) return gm_fail(GM_ERR_UNSUPPORTED, std::string(fn) + ": weights larger than 2 GB");
    Epi ep;
    memset(&ep, 0, sizeof(ep));
    ep.bias = b;
    ep.y = y;
    ep.ldy = ldy;
    ep.y2 = y2;
    ep.ldy2 = ldy2;
    ep.c_in = c_in;
    ep.ldc = ldc;
    ep.act_out = act_out;
    if (is_bias_epi(epilogue)) {  // act_out: sign bits of y (x3 form)
        if (act_out && (!x3 || ldc < (n + 31) / 32))
            return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": sign bits need the x3 form and ldc >= ceil(n / 32)");
        ep.sbits = reinterpret_cast<unsigned*>(act_out);
        ep.ldsb = ldc;
        ep.act_out = nullptr;
        ep.c_in = nullptr;
    }
    if (x3 && (rc = range_flag(&ep.range_flag))) return rc;
    if (epilogue == GM_EPI_GRU) {  // the LSTM gate-tile kernels with the GRU gate math
        if (n % 128 || !c_in || act_out)
            return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": GRU epilogue needs 4H % 128 == 0, c_in = h, no act_out");
        ep.cell = 1;
        epilogue = GM_EPI_LSTM;
    } else if (epilogue == GM_EPI_LSTM) {
        if (n % 128 || !y2 || !c_in) return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": LSTM epilogue needs 4H % 128 == 0");
    } else if (!is_bias_epi(epilogue)) {
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": unknown epilogue");
    } else if (ldy < n) {
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": ldy < n");
    }
    const float* wf = static_cast<const float*>(w);
    hipStream_t st = (hipStream_t)stream;
    return x3 ? dispatch<true>(s0, s1, wf, ldw, (unsigned)wb, m, n, K, epilogue, ep, st, wsi)
              : dispatch<false>(s0, s1, wf, ldw, (unsigned)wb, m, n, K, epilogue, ep, st, nullptr);
}

// ---- weight split for X3: S = 2^(15 - e) with max|w| = f * 2^e (f in [0.5, 1)), so
// S*max|w| in [2^14, 2^15) (< f16 max 65504) and both pieces of every weight stay normal
// down to ~2^-24 of the largest ----
// max |W| over the [n][k] block (row stride ldw) as float bits into *acc (zeroed first): one
// row per wave at a time, lanes over columns (coalesced), rows spread over the grid
__global__ void k_absmax(const float* __restrict__ w, long long ldw, int n, int k, unsigned* __restrict__ acc) {
    __shared__ float red[16];
    float m = 0.f;
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int r = blockIdx.x * nw + wave; r < n; r += gridDim.x * nw)
        for (int c = threadIdx.x & 63; c < k; c += 64) m = fmaxf(m, fabsf(w[(long long)r * ldw + c]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < nw; i++) m = fmaxf(m, red[i]);
        m = fmaxf(m, red[0]);
        atomicMax(acc, __float_as_uint(m));
    }
}

// 1/S from the max: S * max|W| in [2^14, 2^15)
__global__ void k_wscale_from_max(float* __restrict__ wsi) {
    const float m = __uint_as_float(*reinterpret_cast<const unsigned*>(wsi));
    int e = 0;
    if (m > 0.f && isfinite(m)) frexpf(m, &e);
    e = max(-100, min(100, e));
    wsi[0] = ldexpf(1.0f, e - 15);
}

// one thread per (row, 16-deep k block, element): packed[row][blk] = hi[16] | lo[16]
__global__ void k_split_w(const float* __restrict__ w, long long ldw, int n, int k, int nblk,
                          _Float16* __restrict__ wp, const float* __restrict__ wsi) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n * nblk * 16) return;
    const int e = (int)(i & 15);
    const long long rb = i >> 4;
    const int r = (int)(rb / nblk), blk = (int)(rb - (long long)r * nblk);
    const int c = blk * 16 + e;
    const float S = 1.0f / wsi[0];
    const float v = c < k ? w[(long long)r * ldw + c] * S : 0.f;
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    _Float16* o = wp + rb * 32;
    o[e] = hi;
    o[16 + e] = lo;
}

}  // namespace

extern "C" int gm_gemm_f32(const gm_a_src* a0, const gm_a_src* a1, const float* w, int64_t ldw, const float* b,
                           int32_t m, int32_t n, int32_t epilogue, float* y, int64_t ldy, float* y2, int64_t ldy2,
                           const float* c_in, int64_t ldc, float* act_out, void* stream) {
    return gemm_entry(false, a0, a1, w, ldw, nullptr, b, m, n, epilogue, y, ldy, y2, ldy2, c_in, ldc, act_out, stream);
}

extern "C" int gm_gemm_x3(const gm_a_src* a0, const gm_a_src* a1, const void* wp, const float* wscale_inv,
                          const float* b, int32_t m, int32_t n, int32_t epilogue, float* y, int64_t ldy, float* y2,
                          int64_t ldy2, const float* c_in, int64_t ldc, float* act_out, void* stream) {
    return gemm_entry(true, a0, a1, wp, 0, wscale_inv, b, m, n, epilogue, y, ldy, y2, ldy2, c_in, ldc, act_out,
                      stream);
}

extern "C" int gm_gemm_x3_dgrad(const gm_a_src* a0, const void* wp, const float* wscale_inv, int32_t m, int32_t n,
                                int32_t split, const uint32_t* mask_bits, int64_t ldm, float* y, int64_t ldy, float* y2,
                                int64_t ldy2, float* part, float* gmax, void* stream) {
    if (!a0 || a0->mode != GM_A_DENSE || !wp || !wscale_inv || !y || m <= 0 || n <= 0 || split <= 0 || split > n ||
        ldy < split || (split < n && (!y2 || ldy2 < n - split)) ||
        (mask_bits && ldm != 0 && ldm < (split + 31) / 32) || (reinterpret_cast<uintptr_t>(wp) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_x3_dgrad: bad arguments (dense source, 0 < split <= n)");
    ASrc s0, s1;
    int rc = to_asrc(a0, m, s0);
    if (rc) return rc;
    if (s0.amax) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_x3_dgrad: no amax on the A source");
    memset(&s1, 0, sizeof(s1));
    const int K = s0.k;
    const long long ldw = (long long)((K + BKMAX - 1) / BKMAX * BKMAX) / 16 * 64, wb = (long long)n * ldw;
    if (!fits(wb)) return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm_x3_dgrad: weights larger than 2 GB");
    Epi ep;
    memset(&ep, 0, sizeof(ep));
    ep.y = y;
    ep.ldy = ldy;
    ep.y2 = y2;
    ep.ldy2 = ldy2;
    ep.mbits = mask_bits;
    ep.ldmb = ldm;
    ep.split = split;
    ep.part = part;
    ep.gmax = reinterpret_cast<unsigned*>(gmax);
    if ((rc = range_flag(&ep.range_flag))) return rc;
    const float* w = static_cast<const float*>(wp);
    hipStream_t st = (hipStream_t)stream;
    // tools/dgrad_bench.py at 1.04 M rows: the LDS-DMA tile gains 13-15 % at K = 512 and 2-3 % at
    // K = 256; since the row-bounded epilogue stores (round 6) also at K = 128: 256 x 128 with mask, bias partials
    // and max 615 -> 517 us (128x128), 512 x 128 1070 -> 1010 us (128x256), config 5's head (512 x 100 at
    // 6.55 M rows, bare) 6179 -> 5193 us (128x256)
    const int form = g_dgrad >= 0 ? g_dgrad : (m >= 32768 && K >= 64 ? (K < 256 && n >= 512 ? 2 : 1) : 0);
    if (form == 1)  // LDS-DMA 128x128, 4 waves, 2 blocks/CU
        return s0.scale ? launch_g<4, 1, 1, 4, 2, GM_A_DENSE, EPI_DGRAD, 2, 2>(s0, s1, w, ldw, (unsigned)wb, m, n, K, ep,
                                                                               st, wscale_inv)
                        : launch_g<4, 1, 1, 4, 2, GM_A_DENSE, EPI_DGRAD, 2, 0>(s0, s1, w, ldw, (unsigned)wb, m, n, K, ep,
                                                                               st, wscale_inv);
    if (form == 2)  // LDS-DMA 128x256, 8 waves, 1 block/CU
        return s0.scale ? launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_DGRAD, 1, 2>(s0, s1, w, ldw, (unsigned)wb, m, n, K, ep,
                                                                               st, wscale_inv)
                        : launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_DGRAD, 1, 0>(s0, s1, w, ldw, (unsigned)wb, m, n, K, ep,
                                                                               st, wscale_inv);
    return launch<2, 2, 2, 2, 16, GM_A_DENSE, EPI_DGRAD, 2, true>(s0, s1, w, ldw, (unsigned)wb, m, n, K, ep, st,
                                                                 wscale_inv);
}

extern "C" int gm_gemm_range_status(int32_t* status, int32_t clear) {
    if (!status) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_range_status: null status");
    *status = g_range_host ? (int32_t)*reinterpret_cast<volatile unsigned*>(g_range_host) : 0;
    if (clear && g_range_host) *reinterpret_cast<volatile unsigned*>(g_range_host) = 0u;
    return GM_OK;
}

// NetMon encoder layers 1-3 of the rollout in one launch (src/model.py:13-42, 489): layer 1 in layer 2's
// A-tile load (a0: GM_A_ROUTING_ENC), layer 2 (128 x 256 block tiles: the whole width) kept on chip as split
// f16 images, layer 3 from them (EPI_CHAIN); only y = layer 3's output is written
extern "C" int gm_encoder_x3(const gm_a_src* a0, const void* w2p, const float* w2sinv, const float* b2, int32_t act2,
                             const void* w3p, const float* w3sinv, const float* b3, int32_t act3, int32_t m, int32_t n2,
                             int32_t n3, float* y, int64_t ldy, void* stream) {
    if (!a0 || a0->mode != GM_A_ROUTING_ENC || !w2p || !w2sinv || !w3p || !w3sinv || !y || m <= 0 || n2 != 256 ||
        n3 != 128 || ldy < n3 || act2 < GM_ACT_NONE || act2 > GM_ACT_LAST || act3 < GM_ACT_NONE || act3 > GM_ACT_LAST ||
        (reinterpret_cast<uintptr_t>(w2p) & 15) || (reinterpret_cast<uintptr_t>(w3p) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_encoder_x3: bad arguments (routing-encoder source, layers 256, 128 wide)");
    ASrc s0, s1;
    int rc = to_asrc(a0, m, s0, true);
    if (rc) return rc;
    memset(&s1, 0, sizeof(s1));
    const int K = s0.k;
    const long long ldw2 = (long long)K / 16 * 64, wb2 = (long long)n2 * ldw2;
    const long long ldw3 = (long long)n2 / 16 * 64, wb3 = (long long)n3 * ldw3;  // layer-3 K = n2
    Epi ep;
    memset(&ep, 0, sizeof(ep));
    ep.bias = b2;
    ep.act = act2;
    ep.w2 = static_cast<const _Float16*>(w3p);
    ep.ldw2 = ldw3;
    ep.w2bytes = (unsigned)wb3;
    ep.wsi2 = w3sinv;
    ep.b2 = b3;
    ep.act2 = act3;
    ep.y = y;
    ep.ldy = ldy;
    if ((rc = range_flag(&ep.range_flag))) return rc;
    return launch_g<4, 2, 1, 4, 2, GM_A_ROUTING_ENC, EPI_CHAIN, 1>(s0, s1, static_cast<const float*>(w2p), ldw2,
                                                                  (unsigned)wb2, m, n2, K, ep, (hipStream_t)stream,
                                                                  w2sinv, 1);
}

extern "C" int gm_gemm_x3_head(const gm_a_src* a0, const void* wp, const float* wscale_inv, const float* b,
                               int32_t m, int32_t n, int32_t act, const float* wq, int64_t ldwq, const float* bq,
                               int32_t nq, float* q, int64_t ldq, float* y, int64_t ldy, void* stream) {
    if (!a0 || a0->mode != GM_A_DENSE || !wp || !wscale_inv || !wq || !q || m <= 0 || n <= 0 || n > 256 ||
        nq <= 0 || nq > 4 || ldwq < n || ldq < nq || (y && ldy < n) || act < GM_ACT_NONE || act > GM_ACT_LAST ||
        (reinterpret_cast<uintptr_t>(wp) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_x3_head: bad arguments (dense source, n <= 256, nq <= 4)");
    ASrc s0, s1;
    int rc = to_asrc(a0, m, s0);
    if (rc) return rc;
    if (s0.scale) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_x3_head: no A scale");
    memset(&s1, 0, sizeof(s1));
    const int K = s0.k;
    const long long ldw = (long long)((K + BKMAX - 1) / BKMAX * BKMAX) / 16 * 64, wb = (long long)n * ldw;
    if (!fits(wb)) return gm_fail(GM_ERR_UNSUPPORTED, "gm_gemm_x3_head: weights larger than 2 GB");
    Epi ep;
    memset(&ep, 0, sizeof(ep));
    ep.bias = b;
    ep.act = act;
    ep.y = y;
    ep.ldy = ldy;
    ep.wq = wq;
    ep.ldwq = ldwq;
    ep.bq = bq;
    ep.nq = nq;
    ep.q = q;
    ep.ldq = ldq;
    if ((rc = range_flag(&ep.range_flag))) return rc;
    if (!s0.amax && n > 128 && g_mfma16 == 2) {  // (the 16x16 epilogue adds partials)
        // rollout: 128x128 blocks at 2 per CU (the plain layer's faster tile); each of the two column
        // blocks adds its partial Q to a zeroed q (column block 0 with bq)
        const hipError_t me = hipMemset2DAsync(q, (size_t)ldq * 4, 0, (size_t)nq * 4, (size_t)m, (hipStream_t)stream);
        if (me != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gemm_x3_head: ") + hipGetErrorString(me));
        ep.q_atomic = 1;
        return launch_g<4, 1, 1, 4, 2, GM_A_DENSE, EPI_HEAD, 2>(s0, s1, static_cast<const float*>(wp), ldw, (unsigned)wb, m, n,
                                                                K, ep, (hipStream_t)stream, wscale_inv, g_mfma16 == 2);
    }
    if (s0.amax)  // training forward: max |A| for the layer's weight gradient
        return launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_HEAD, 1, 1>(s0, s1, static_cast<const float*>(wp), ldw,
                                                                  (unsigned)wb, m, n, K, ep, (hipStream_t)stream,
                                                                  wscale_inv, g_mfma16 == 2);
    return launch_g<4, 2, 1, 4, 2, GM_A_DENSE, EPI_HEAD, 1>(s0, s1, static_cast<const float*>(wp), ldw, (unsigned)wb, m,
                                                          n, K, ep, (hipStream_t)stream, wscale_inv, g_mfma16 == 2);
}

// max |x| as float bits (non-negative floats order as unsigned ints) into *acc (zeroed first)
__global__ void k_absmax_atomic(const float* __restrict__ x, long long n, unsigned* __restrict__ acc) {
    __shared__ float red[4];
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(x[i]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); i++) m = fmaxf(m, red[i]);
        m = fmaxf(m, red[0]);
        atomicMax(acc, __float_as_uint(m));
    }
}

__global__ void k_scale_from_max(float* __restrict__ scale) {
    const float m = __uint_as_float(*reinterpret_cast<const unsigned*>(scale));
    int e = 0;
    if (m > 0.f && isfinite(m)) frexpf(m, &e);  // m in [2^(e-1), 2^e)
    e = max(-100, min(100, e));
    scale[0] = (m > 0.f && isfinite(m)) ? ldexpf(1.0f, 14 - e) : 1.0f;  // s * max in [2^13, 2^14)
}

// max |x| over a [rows][cols] block with row stride ld: one row per wave at a time, lanes over
// columns, rows spread over the grid; float bits into *acc (zeroed first)
__global__ void k_absmax_rows(const float* __restrict__ x, long long rows, int cols, long long ld,
                              unsigned* __restrict__ acc) {
    __shared__ float red[4];
    float m = 0.f;
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (long long r = (long long)blockIdx.x * nw + wave; r < rows; r += (long long)gridDim.x * nw)
        for (int c = threadIdx.x & 63; c < cols; c += 64) m = fmaxf(m, fabsf(x[r * ld + c]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < nw; i++) m = fmaxf(m, red[i]);
        m = fmaxf(m, red[0]);
        atomicMax(acc, __float_as_uint(m));
    }
}

extern "C" int gm_absmax_scale_rows(const float* x, int64_t rows, int32_t cols, int64_t ld, float* scale,
                                    void* stream) {
    if (!x || !scale || rows <= 0 || cols <= 0 || ld < cols)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_absmax_scale_rows: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(scale, 0, sizeof(float), st);
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_absmax_scale_rows: ") + hipGetErrorString(e));
    if (ld == cols) {  // contiguous rows: one flat grid-stride pass
        const long long n = rows * (long long)cols;
        hipLaunchKernelGGL(k_absmax_atomic, dim3((unsigned)std::min<long long>(2048, (n + 255) / 256)), dim3(256), 0, st,
                           x, n, reinterpret_cast<unsigned*>(scale));
    } else {
        const long long blocks = std::min<long long>(1024, (rows + 3) / 4);
        hipLaunchKernelGGL(k_absmax_rows, dim3((unsigned)blocks), dim3(256), 0, st, x, (long long)rows, (int)cols,
                           (long long)ld, reinterpret_cast<unsigned*>(scale));
    }
    hipLaunchKernelGGL(k_scale_from_max, dim3(1), dim3(1), 0, st, scale);
    e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_absmax_scale_rows: ") + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_absmax_finish(float* scale, void* stream) {
    if (!scale) return gm_fail(GM_ERR_INVALID_ARG, "gm_absmax_finish: bad arguments");
    hipLaunchKernelGGL(k_scale_from_max, dim3(1), dim3(1), 0, (hipStream_t)stream, scale);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_absmax_finish: ") + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_absmax_scale(const float* x, int64_t n, float* scale, void* stream) {
    if (!x || !scale || n <= 0) return gm_fail(GM_ERR_INVALID_ARG, "gm_absmax_scale: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(scale, 0, sizeof(float), st);
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_absmax_scale: ") + hipGetErrorString(e));
    const long long blocks = std::min<long long>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_absmax_atomic, dim3((unsigned)blocks), dim3(256), 0, st, x, (long long)n,
                       reinterpret_cast<unsigned*>(scale));
    hipLaunchKernelGGL(k_scale_from_max, dim3(1), dim3(1), 0, st, scale);
    e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_absmax_scale: ") + hipGetErrorString(e));
    return GM_OK;
}

// ---------------------------------------------------------------------------------------
// Weight-gradient GEMM (training): C_z[m][n] = sum over k of split z of A[k][m] * B[k][n],
// A = dY [K][lda], B = X [K][ldb], both K-major fp32 (K = batch rows) — the transposes are done
// on the way into LDS. Both operands are scaled by device powers of two (sa, sb) and split as
// a = a_hi + 2^-12 a_lo' (both pieces normal f16), a*b ~ a_hi b_hi + 2^-12 (a_lo' b_hi + a_hi b_lo')
// with the 2^-12 terms in a second accumulator. 128x128x32 tiles, 4 waves of 64x64; each
// thread moves two 4(k) x 4(m|n) sub-blocks per k step (32 coalesced dword loads, a register
// transpose, 2 x 8-B LDS stores per column and block). Split-K over blockIdx.y, partial sums
// written to C + z * cz (the caller reduces them).
__global__ __launch_bounds__(256, 2) void k_gemm3_kmajor(const float* __restrict__ A, long long lda,
                                                        const float* __restrict__ B, long long ldb, int M, int N,
                                                        int K, int kchunk, const float* __restrict__ sa,
                                                        const float* __restrict__ sb, float* __restrict__ C,
                                                        long long ldc, long long cz) {
    // 32-deep k tiles: per LDS row two 16-deep blocks of [16 hi | 16 lo] halves (64 B each) + 16 B
    // pad (conflict-free ds_read_b128 over the 32 rows of a fragment, as k_gemm3's BK=32 tiles)
    constexpr int BM = 128, BN = 128, BK = 32, ROWB = 4 * BK + 16, TM = 2, TN = 2;
    __shared__ __attribute__((aligned(16))) char As[2][BM * ROWB];
    __shared__ __attribute__((aligned(16))) char Bs[2][BN * ROWB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int nN = (N + BN - 1) / BN;
    const int m0 = (blockIdx.x / nN) * BM, n0 = (blockIdx.x % nN) * BN;
    const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
    const int nk = (ke - kb + BK - 1) / BK;
    // this thread: operand (A for tid < 128), 4-deep k groups k4 and k4 + 4 (one per 16-deep
    // block), columns c4 + 32 c (c = 0..3): dword loads (coalesced over c4) and LDS rows
    // c4 + 32 c (consecutive rows per store instruction: conflict-free 8-B stores)
    const bool isA = tid < 128;
    const int t = tid & 127, k4 = t >> 5, c4 = t & 31;
    const float* src = isA ? A : B;
    const long long ld = isA ? lda : ldb;
    const int col0 = (isA ? m0 : n0) + c4, lim = isA ? M : N;
    const float s = isA ? *sa : *sb;
    char* dstb[2] = {(isA ? As[0] : Bs[0]) + c4 * ROWB + 8 * k4, (isA ? As[1] : Bs[1]) + c4 * ROWB + 8 * k4};
    float rv[2][4][4];  // [16-deep block g][column c][k row r]
    auto load = [&](int kt) {
#pragma unroll
        for (int g = 0; g < 2; g++) {
            const int k = kb + kt * BK + 16 * g + 4 * k4;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float* rowp = src + (long long)(k + r) * ld + col0;
                const bool kok = k + r < ke;
#pragma unroll
                for (int c = 0; c < 4; c++) rv[g][c][r] = (kok && col0 + 32 * c < lim) ? rowp[32 * c] : 0.f;
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int g = 0; g < 2; g++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                half4 hi, lo;
                split4(make_float4(rv[g][c][0] * s, rv[g][c][1] * s, rv[g][c][2] * s, rv[g][c][3] * s), hi, lo);
                char* row = dstb[buf] + 32 * c * ROWB + 64 * g;
                *reinterpret_cast<half4*>(row) = hi;
                *reinterpret_cast<half4*>(row + 32) = lo;
            }
    };
    floatx16 acc[TM][TN], acc2[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = acc2[i][j][r] = 0.f;
    const int h = lane >> 5, l32 = lane & 31;
    auto compute = [&](int buf) {
        const char* ac = As[buf] + (wr * TM * 32 + l32) * ROWB + 16 * h;
        const char* bc = Bs[buf] + (wc * TN * 32 + l32) * ROWB + 16 * h;
#pragma unroll
        for (int sb = 0; sb < BK / 16; sb++) {
            half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; i++) {
                ah[i] = *reinterpret_cast<const half8*>(ac + i * 32 * ROWB + 64 * sb);
                al[i] = *reinterpret_cast<const half8*>(ac + i * 32 * ROWB + 64 * sb + 32);
            }
#pragma unroll
            for (int j = 0; j < TN; j++) {
                bh[j] = *reinterpret_cast<const half8*>(bc + j * 32 * ROWB + 64 * sb);
                bl[j] = *reinterpret_cast<const half8*>(bc + j * 32 * ROWB + 64 * sb + 32);
            }
#pragma unroll
            for (int i = 0; i < TM; i++)
#pragma unroll
                for (int j = 0; j < TN; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc2[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc2[i][j], 0, 0, 0);
                }
        }
    };
    // (loading two steps ahead into alternating register sets measured no faster)
    if (nk > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        if (kt + 1 < nk) load(kt + 1);
        compute(kt & 1);
        if (kt + 1 < nk) store((kt + 1) & 1);
        __syncthreads();
    }
    const float inv = 1.0f / (*sa * *sb);  // powers of two: exact
    float* Cz = C + (size_t)blockIdx.y * cz;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int n = n0 + wc * TN * 32 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int m = m0 + wr * TM * 32 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
                if (m < M && n < N) Cz[(long long)m * ldc + n] = (acc[i][j][r] + acc2[i][j][r] * (1.0f / LO_S)) * inv;
            }
        }
}

// Weight-gradient GEMM, transposed-read form (default): the same arithmetic as k_gemm3_kmajor
// (both operands scaled by device powers of two and split into f16 pieces, hi*hi in one
// accumulator and the two 2^-12 cross terms in a second), but the K-major operands are staged in
// their natural layout: 16-byte loads of 4 consecutive m (n) columns of one k row, split in
// registers, stored as 8-byte [k][column] f16 rows (hi and lo images), and the MFMA fragments
// (8 consecutive k of one column) are read with ds_read_b64_tr_b16, which transposes 4 k rows x 16
// columns per 16-lane group. No register transpose, 4x fewer global load instructions than the
// dword form, and a 64 x (BN/2) wave tile. Row stride of an image = columns * 2 + 64 B: the four
// k rows of a 32-lane half then start 16 banks apart (conflict-free transposed reads).
// MF = 1: v_mfma_f32_16x16x32_f16 (16-lane group g reads k rows 8 g .. 8 g + 7 of its 16 columns; the
// images' 32-byte column segments are XOR-swizzled by bit 3 of the k row so that the two groups of a
// 32-lane half (rows 8 g + q, 8 (g + 1) + q) hit disjoint banks)
// XCD = 1: the (tile, k chunk) of a block comes from a permutation of the dispatch order that puts
// every tile of a k chunk on one XCD (workgroups go to the 8 XCDs round-robin by linear id), so the
// chunk's A and B rows are fetched into that XCD's L2 once and reused by all its tiles there
// (identity order: the tiles of a chunk spread over the 8 XCDs and each L2 fetches its own copy)
struct WgB {  // one K-major B source of k_wgrad_tr (gm_wgrad_src): batch row r reads source row
                // (period ? r % period : r) + shift, zero outside [0, rows); a k chunk maps to one run of rows
    const float* p;
    long long ld;
    const float* s;
    long long period, shift, rows;
};

template <int BN, int MF = 0>
__global__ __launch_bounds__(256, BN == 128 ? 2 : 1) void k_wgrad_tr(const float* __restrict__ A, long long lda,
                                                                   unsigned abytes, WgB b1, WgB b2, int nsplit, int M,
                                                                   int N, int K, int kchunk, const float* __restrict__ sa,
                                                                   float* __restrict__ C, long long ldc, long long cz,
                                                                   int xcd) {
    constexpr int BM = 128, BK = 32, TM = 2, TN = BN / 64;
    constexpr int RA = BM * 2 + 64, RB = BN * 2 + 64;  // image row strides (bytes)
    constexpr int LA = BM / 4 * BK / 256, LB = BN / 4 * BK / 256;  // float4 loads per thread
    __shared__ __attribute__((aligned(16))) char smem[2][2 * BK * RA + 2 * BK * RB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int nN = (N + BN - 1) / BN;
    int tile = blockIdx.x, chunk = blockIdx.y;
    if (xcd) {  // host guarantees gridDim.x * gridDim.y % 8 == 0
        const int T = gridDim.x, nb = T * gridDim.y, b = blockIdx.x + blockIdx.y * T;
        const int l = (b & 7) * (nb >> 3) + (b >> 3);
        tile = l % T;
        chunk = l / T;
    }
    const int m0 = (tile / nN) * BM, n0 = (tile % nN) * BN;
    const int kb = chunk * kchunk, ke = min(K, kb + kchunk);
    const int nk = (ke - kb + BK - 1) / BK;
    // B source of this tile: output columns [0, nsplit) from b1, [nsplit, N) from b2 (nsplit % BN == 0, so a tile
    // lies in one source); nb0 / nlim: the tile's first column and the column count inside its source. The k
    // chunk's batch rows map to source rows brow0 .. brow0 + kchunk - 1 (host: kchunk divides every period and
    // shift), zero where they fall outside the source
    const bool sec = n0 >= nsplit;
    const WgB& bs = sec ? b2 : b1;
    const int nb0 = sec ? n0 - nsplit : n0, nlim = sec ? N - nsplit : min(N, nsplit);
    const long long brow0 = (bs.period ? kb % bs.period : kb) + bs.shift;
    const long long bav = (brow0 < 0 || brow0 >= bs.rows) ? 0 : min((long long)kchunk, bs.rows - brow0);
    const long long ldb = bs.ld;
    const float s_a = *sa, s_b = *bs.s;
    const int e_a = __builtin_amdgcn_frexp_expf(s_a) - 1, e_b = __builtin_amdgcn_frexp_expf(s_b) - 1;  // 2^e = scale
    // buffer resources over this block's k chunk only: 32-bit offsets stay small whatever the batch
    // (abytes / bbytes: the bytes of one chunk of rows, host-checked)
    const __amdgpu_buffer_rsrc_t ra = rsrc(A + (long long)kb * lda, abytes),
                                 rb = rsrc(bs.p + (bav ? brow0 : 0) * ldb, (unsigned)(bav * ldb * 4));
    // loader map: A tile 32 k x 128 m = 32 float4 per k row -> lane q = tid & 31 (m = 4q), rows
    // (tid >> 5) + 8 j; B tile 32 x BN: BN / 4 float4 per row
    constexpr int QB = BN / 4, RB_STEP = 256 / QB;
    const int qa = tid & 31, ka0 = tid >> 5, qb = tid % QB, kb0 = tid / QB;
    // NS register sets of staged operands: 2 (128-wide 32x32x16 form) loads tile kt + 2 while
    // tile kt + 1 waits in the other set for its store, so a load has a whole k step plus the MFMAs to land
    constexpr int NS = (MF == 0 && BN == 128) ? 2 : 1;
    float4 va[NS][LA], vb[NS][LB];
    auto load = [&](auto SET, int kt) {
        constexpr int S = decltype(SET)::value;
        const int k0 = kb + kt * BK;
#pragma unroll
        for (int j = 0; j < LA; j++) {
            const int k = k0 + ka0 + 8 * j, m = m0 + 4 * qa;
            const int off = (k < ke && m < M) ? (int)(((long long)(k - kb) * lda + m) * 4) : OOB;
            va[S][j] = bload(ra, off);
        }
#pragma unroll
        for (int j = 0; j < LB; j++) {
            const int k = k0 + kb0 + RB_STEP * j, n = nb0 + 4 * qb;
            const int off = (k < ke && n < nlim) ? (int)(((long long)(k - kb) * ldb + n) * 4) : OOB;
            vb[S][j] = bload(rb, off);
        }
    };
    auto store = [&](auto SET, int buf) {
        constexpr int S = decltype(SET)::value;
        char* ah = smem[buf];
        char* al = ah + BK * RA;
        char* bh = al + BK * RA;
        char* bl = bh + BK * RB;
#pragma unroll
        for (int j = 0; j < LA; j++) {
            half4 hi, lo;
            split4e(va[S][j], e_a, hi, lo);
            const int o = (ka0 + 8 * j) * RA + ((8 * qa) ^ (MF ? (((ka0 + 8 * j) >> 3) & 1) << 5 : 0));
            *reinterpret_cast<half4*>(ah + o) = hi;
            *reinterpret_cast<half4*>(al + o) = lo;
        }
#pragma unroll
        for (int j = 0; j < LB; j++) {
            half4 hi, lo;
            split4e(vb[S][j], e_b, hi, lo);
            const int o = (kb0 + RB_STEP * j) * RB + ((8 * qb) ^ (MF ? (((kb0 + RB_STEP * j) >> 3) & 1) << 5 : 0));
            *reinterpret_cast<half4*>(bh + o) = hi;
            *reinterpret_cast<half4*>(bl + o) = lo;
        }
    };
    floatx4 c4[2 * TM][2 * TN], c4b[2 * TM][2 * TN];  // MF = 1: 16 x 16 blocks (hi*hi, cross terms)
#pragma unroll
    for (int i = 0; i < 2 * TM; i++)
#pragma unroll
        for (int j = 0; j < 2 * TN; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) c4[i][j][r] = c4b[i][j][r] = 0.f;
    floatx16 acc[TM][TN], acc2[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = acc2[i][j][r] = 0.f;
    // transposed-read address of this lane inside a 32-column fragment (T10): 16-lane group g reads
    // k rows 8 (g >> 1) + 4 h + q (h = 0, 1: the two reads of 4 rows), columns 16 (g & 1) + 4 p
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int trk = 8 * (g >> 1) + q, trc = 16 * (g & 1) + 4 * p;
    typedef __fp16 v4fp16 __attribute__((__vector_size__(8)));
    auto frag = [&](const char* img, int rs, int col0, int k0) {
        const char* a0 = img + (k0 + trk) * rs + 2 * (col0 + trc);
        const half4 x0 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a0)));
        const half4 x1 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a0 + 4 * rs)));
        return half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    };
    // 16x16x32 form: group g = lane >> 4 reads rows 8 g + q (+ 4), columns 4 p of its 16-column block,
    // segment swizzle g & 1 (bit 3 of the row)
    const int swz16 = ((lane >> 4) & 1) << 5;
    auto frag16 = [&](const char* img, int rs, int col0) {
        const char* a0 = img + (8 * g + q) * rs + ((2 * col0 + 8 * p) ^ swz16);
        const half4 x0 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a0)));
        const half4 x1 = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) v4fp16*)(a0 + 4 * rs)));
        return half8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    };
    auto compute16 = [&](int buf) {
        const char* ah = smem[buf];
        const char* al = ah + BK * RA;
        const char* bh = al + BK * RA;
        const char* bl = bh + BK * RB;
        half8 fah[2 * TM], fal[2 * TM], fbh[2 * TN], fbl[2 * TN];
#pragma unroll
        for (int i = 0; i < 2 * TM; i++) {
            fah[i] = frag16(ah, RA, wr * TM * 32 + 16 * i);
            fal[i] = frag16(al, RA, wr * TM * 32 + 16 * i);
        }
#pragma unroll
        for (int j = 0; j < 2 * TN; j++) {
            fbh[j] = frag16(bh, RB, wc * TN * 32 + 16 * j);
            fbl[j] = frag16(bl, RB, wc * TN * 32 + 16 * j);
        }
#pragma unroll
        for (int i = 0; i < 2 * TM; i++)
#pragma unroll
            for (int j = 0; j < 2 * TN; j++) {
                c4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[i], fbh[j], c4[i][j], 0, 0, 0);
                c4b[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[i], fbh[j], c4b[i][j], 0, 0, 0);
                c4b[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[i], fbl[j], c4b[i][j], 0, 0, 0);
            }
    };
    auto compute = [&](int buf) {
        if constexpr (MF == 1) {
            compute16(buf);
            return;
        }
        const char* ah = smem[buf];
        const char* al = ah + BK * RA;
        const char* bh = al + BK * RA;
        const char* bl = bh + BK * RB;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 16) {
            half8 fah[TM], fal[TM], fbh[TN], fbl[TN];
#pragma unroll
            for (int i = 0; i < TM; i++) {
                fah[i] = frag(ah, RA, wr * TM * 32 + 32 * i, kk);
                fal[i] = frag(al, RA, wr * TM * 32 + 32 * i, kk);
            }
#pragma unroll
            for (int j = 0; j < TN; j++) {
                fbh[j] = frag(bh, RB, wc * TN * 32 + 32 * j, kk);
                fbl[j] = frag(bl, RB, wc * TN * 32 + 32 * j, kk);
            }
#pragma unroll
            for (int i = 0; i < TM; i++)
#pragma unroll
                for (int j = 0; j < TN; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbh[j], acc[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[i], fbh[j], acc2[i][j], 0, 0, 0);
                    acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbl[j], acc2[i][j], 0, 0, 0);
                }
        }
    };
    using W0 = std::integral_constant<int, 0>;
    using W1 = std::integral_constant<int, NS - 1>;
    if constexpr (NS == 1) {
        if (nk > 0) {
            load(W0{}, 0);
            store(W0{}, 0);
        }
        __syncthreads();
        for (int kt = 0; kt < nk; kt++) {
            if (kt + 1 < nk) load(W0{}, kt + 1);
            compute(kt & 1);
            if (kt + 1 < nk) store(W0{}, (kt + 1) & 1);
            __syncthreads();
        }
    } else {
        // step kt: load tile kt + 2 into set kt & 1 (its tile kt is in LDS buffer kt & 1), compute buffer
        // kt & 1, store tile kt + 1 (set (kt + 1) & 1, loaded one step earlier) into the other buffer
        if (nk > 0) {
            load(W0{}, 0);
            if (nk > 1) load(W1{}, 1);
            store(W0{}, 0);
        }
        __syncthreads();
        auto step = [&](auto SET, int kt) {
            constexpr int S = decltype(SET)::value;
            if (kt + 2 < nk) load(SET, kt + 2);
            compute(S);
            if (kt + 1 < nk) store(std::integral_constant<int, S ^ 1>{}, S ^ 1);
            __syncthreads();
        };
        for (int kt = 0; kt < nk; kt += 2) {
            step(W0{}, kt);
            if (kt + 1 < nk) step(W1{}, kt + 1);
        }
    }
    const float inv = 1.0f / (s_a * s_b);  // powers of two: exact
    float* Cz = C + (size_t)chunk * cz;
    if constexpr (MF == 1) {
#pragma unroll
        for (int i = 0; i < 2 * TM; i++)
#pragma unroll
            for (int j = 0; j < 2 * TN; j++) {
                const int n = n0 + wc * TN * 32 + j * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int m = m0 + wr * TM * 32 + i * 16 + 4 * (lane >> 4) + r;
                    if (m < M && n < N) Cz[(long long)m * ldc + n] = (c4[i][j][r] + c4b[i][j][r] * (1.0f / LO_S)) * inv;
                }
            }
        return;
    }
    const int hh = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int n = n0 + wc * TN * 32 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int m = m0 + wr * TM * 32 + i * 32 + 4 * hh + (r & 3) + 8 * (r >> 2);
                if (m < M && n < N) Cz[(long long)m * ldc + n] = (acc[i][j][r] + acc2[i][j][r] * (1.0f / LO_S)) * inv;
            }
        }
}

int g_wgrad = -1;  // weight-gradient kernel: -1 / 1 transposed reads 128 x 128 (default), 2 the same 128 x 256, 0 dword form
int g_wgrad_xcd = 1;  // XCD-grouped k chunks (k_wgrad_tr xcd), when the grid is a multiple of 8

// launcher of both entry points: n1 columns from source 1, n2 from source 2 (n2 = 0: none)
static int wgrad_launch(const float* a, int64_t lda, const gm_wgrad_src& s1, int32_t n1, const gm_wgrad_src* s2,
                        int32_t n2, int32_t m, int32_t k, int32_t kchunk, const float* sa, float* c, int64_t ldc,
                        void* stream, const char* what) {
    const int n = n1 + n2;
    auto src_ok = [&](const gm_wgrad_src& b, int nb) {
        return b.p && b.scale && nb > 0 && (nb % 4) == 0 && b.ld >= nb && (b.ld % 4) == 0 &&
               !(reinterpret_cast<uintptr_t>(b.p) & 15) && b.period >= 0 && b.rows > 0 &&
               (b.period == 0 || b.period % kchunk == 0) && (b.shift % kchunk) == 0;
    };
    if (!a || !sa || !c || m <= 0 || n1 <= 0 || n2 < 0 || k <= 0 || kchunk <= 0 || (kchunk % 16) || (m % 4) ||
        lda < m || (lda % 4) || ldc < n || (reinterpret_cast<uintptr_t>(a) & 15) || !src_ok(s1, n1) ||
        (n2 > 0 && (!s2 || !src_ok(*s2, n2))))
        return gm_fail(GM_ERR_INVALID_ARG, std::string(what) + ": bad arguments (m, n, ld multiples of 4, 16-B bases, "
                                                               "kchunk % 16 == 0 and dividing every period / shift)");
    const int S = (k + kchunk - 1) / kchunk;
    const bool plain = n2 == 0 && s1.period == 0 && s1.shift == 0;
    if (!plain && (g_wgrad == 0 || g_wgrad == 2 || (n2 > 0 && n1 % 128)))
        return gm_fail(GM_ERR_UNSUPPORTED, std::string(what) + ": two sources / row maps need the 128-column "
                                                               "transposed-read forms and n1 % 128 == 0");
    if (g_wgrad == 0) {
        const int T = ((m + 127) / 128) * ((n + 127) / 128);
        hipLaunchKernelGGL(k_gemm3_kmajor, dim3(T, S), dim3(256), 0, (hipStream_t)stream, a, (long long)lda, s1.p,
                           (long long)s1.ld, m, n, k, kchunk, sa, s1.scale, c, (long long)ldc, (long long)m * ldc);
    } else {
        // per-block buffer resources cover one k chunk (any batch size; a chunk below 2 GB)
        const long long kc = std::min<long long>(kchunk, k);
        const long long ab = kc * lda * 4;
        if (ab >= 0x7ff00000LL || kc * s1.ld * 4 >= 0x7ff00000LL || (n2 > 0 && kc * s2->ld * 4 >= 0x7ff00000LL))
            return gm_fail(GM_ERR_UNSUPPORTED, std::string(what) + ": one k chunk of an operand larger than 2 GB");
        const WgB w1{s1.p, s1.ld, s1.scale, s1.period, s1.shift, s1.rows};
        const WgB w2 = n2 > 0 ? WgB{s2->p, s2->ld, s2->scale, s2->period, s2->shift, s2->rows} : w1;
        const int T128 = ((m + 127) / 128) * ((n + 127) / 128);
        const int xcd = g_wgrad_xcd && (T128 * S) % 8 == 0;
        if (g_wgrad == 3) {  // 16x16x32 MFMA
            hipLaunchKernelGGL((k_wgrad_tr<128, 1>), dim3(T128, S), dim3(256), 0, (hipStream_t)stream, a,
                               (long long)lda, (unsigned)ab, w1, w2, n1, m, n, k, kchunk, sa, c, (long long)ldc,
                               (long long)m * ldc, xcd);
        } else if (g_wgrad != 2) {  // 128 x 128 tiles at 2 blocks/CU: 8-24 % faster than 128 x 256 at 1 block/CU
            hipLaunchKernelGGL(k_wgrad_tr<128>, dim3(T128, S), dim3(256), 0, (hipStream_t)stream, a, (long long)lda,
                               (unsigned)ab, w1, w2, n1, m, n, k, kchunk, sa, c, (long long)ldc, (long long)m * ldc,
                               xcd);
        } else {
            const int T = ((m + 127) / 128) * ((n + 255) / 256);
            hipLaunchKernelGGL(k_wgrad_tr<256>, dim3(T, S), dim3(256), 0, (hipStream_t)stream, a, (long long)lda,
                               (unsigned)ab, w1, w2, n1, m, n, k, kchunk, sa, c, (long long)ldc, (long long)m * ldc,
                               (int)(g_wgrad_xcd && (T * S) % 8 == 0));
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_gemm_x3_wgrad(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t m, int32_t n, int32_t k,
                                int32_t kchunk, const float* sa, const float* sb, float* c, int64_t ldc, void* stream) {
    const gm_wgrad_src s1{b, ldb, sb, 0, 0, k};
    return wgrad_launch(a, lda, s1, n, nullptr, 0, m, k, kchunk, sa, c, ldc, stream, "gm_gemm_x3_wgrad");
}

extern "C" int gm_gemm_x3_wgrad2(const float* a, int64_t lda, const gm_wgrad_src* b1, int32_t n1, const gm_wgrad_src* b2,
                                 int32_t n2, int32_t m, int32_t k, int32_t kchunk, const float* sa, float* c, int64_t ldc,
                                 void* stream) {
    if (!b1) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_x3_wgrad2: no first source");
    return wgrad_launch(a, lda, *b1, n1, b2, b2 ? n2 : 0, m, k, kchunk, sa, c, ldc, stream, "gm_gemm_x3_wgrad2");
}

extern "C" int64_t gm_gemm_pack_x3_bytes(int32_t n, int32_t k) {
    if (n <= 0 || k <= 0) return 0;
    return (int64_t)n * ((k + BKMAX - 1) / BKMAX * BKMAX / 16) * 64;
}

extern "C" int gm_gemm_pack_x3(const float* w, int64_t ldw, int32_t n, int32_t k, void* wp, float* wscale_inv,
                               void* stream) {
    if (!w || !wp || !wscale_inv || n <= 0 || k <= 0 || ldw < k || (reinterpret_cast<uintptr_t>(wp) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_pack_x3: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    const int nblk = (k + BKMAX - 1) / BKMAX * BKMAX / 16;
    hipError_t e0 = hipMemsetAsync(wscale_inv, 0, sizeof(float), st);
    if (e0 != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gemm_pack_x3: ") + hipGetErrorString(e0));
    hipLaunchKernelGGL(k_absmax, dim3((unsigned)std::min(64, (n + 3) / 4)), dim3(256), 0, st, w, (long long)ldw, n, k,
                       reinterpret_cast<unsigned*>(wscale_inv));
    hipLaunchKernelGGL(k_wscale_from_max, dim3(1), dim3(1), 0, st, wscale_inv);
    const long long tot = (long long)n * nblk * 16;
    hipLaunchKernelGGL(k_split_w, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, w, (long long)ldw, n, k, nblk,
                       static_cast<_Float16*>(wp), wscale_inv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gemm_pack_x3: ") + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_gemm_set_wgrad(int32_t form) {
    if (form < -1 || (form >= 0 && ((form & 7) > 3 || form > 11))) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_set_wgrad: form in [-1, 3] (+8)");
    g_wgrad_xcd = form < 0 || !(form & 8);
    g_wgrad = form < 0 ? form : (form & 7);
    return GM_OK;
}

extern "C" int gm_gemm_set_dgrad(int32_t form) {
    if (form < -1 || form > 2) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_set_dgrad: form -1..2");
    g_dgrad = form;
    return GM_OK;
}

extern "C" int gm_gemm_set_mfma(int32_t shape) {
    if (shape < 0 || shape > 2)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_set_mfma: 0 (32x32x16), 1 (16x16x32, head 32x32x16), 2 (16x16x32)");
    g_mfma16 = shape;
    return GM_OK;
}

#define GM_STR2(x) #x
#define GM_STR(x) GM_STR2(x)
extern "C" const char* gm_gemm_form(void) { return "x3=lo" GM_STR(GM_LO_E) " diag=" GM_STR(GM_DIAG); }
#undef GM_STR
#undef GM_STR2

extern "C" int gm_gemm_set_tile(int32_t tile) {
    if (tile < -1 || tile > 14) return gm_fail(GM_ERR_INVALID_ARG, "gm_gemm_set_tile: tile in [-1, 14]");
    g_tile = tile;
    return GM_OK;
}

extern "C" int gm_linear_f32(const float* x, int64_t ldx, const float* w, int64_t ldw, const float* b, int32_t m,
                             int32_t n, int32_t k, int32_t act, float* y, int64_t ldy, void* stream) {
    if (!x || !w || !y || act < GM_ACT_NONE || act > GM_ACT_LAST)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_linear_f32: bad arguments");
    gm_a_src a;
    memset(&a, 0, sizeof(a));
    a.mode = GM_A_DENSE;
    a.p0 = x;
    a.ld0 = ldx;
    a.k = k;
    return gm_gemm_f32(&a, nullptr, w, ldw, b, m, n, act == GM_ACT_NONE ? GM_EPI_BIAS : act == GM_ACT_LEAKY_RELU ? GM_EPI_BIAS_LEAKY : GM_EPI_BIAS_ACT + act, y, ldy, nullptr, 0,
                       nullptr, 0, nullptr, stream);
}
