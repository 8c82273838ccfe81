// gm_linear.hip — fused fp32 linear layer on the gfx950 f32 MFMA
// (v_mfma_f32_32x32x2_f32): y = act(x @ w^T + b), the nn.Linear (+ MLP
// leaky_relu) of the reference (src/model.py:13-42, 119-125). Exact fp32
// products/accumulation (an fmaf chain per k), so results stay within the 1e-5
// contract of the reference's fp32 torch layers; no reduced-precision path.
//
// Block tile BM x BN x BK(32) staged in LDS with a 4-float row pad (conflict-free
// ds_read_b128); each wave owns TM x TN 32x32 accumulator tiles. The k pairing
// per MFMA is {s, 16+s}: lane half h reads 16 contiguous k of its row, so every
// fragment load is a ds_read_b128. Next K tile is prefetched into registers
// while the current one is multiplied. Blocks are remapped so that tiles sharing
// x rows run on one XCD (shared L2).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/graph_marl_amd.h"

int gm_fail(int code, const std::string& msg);

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDP = BK + 4;  // padded LDS row (floats)

template <int WGM, int WGN, int TM, int TN>
struct Cfg {
    static constexpr int BM = WGM * TM * 32;
    static constexpr int BN = WGN * TN * 32;
    static constexpr int THREADS = WGM * WGN * 64;
    static constexpr int A_F4 = BM * BK / 4 / THREADS;  // float4 loads per thread
    static constexpr int B_F4 = BN * BK / 4 / THREADS;
};

// 4 consecutive k of one row: vector load when the whole quad is inside K,
// element-masked scalar loads on the ragged K tail, zeros outside.
__device__ __forceinline__ float4 ld4(const float* p, bool row_ok, int gk, int K) {
    if (!row_ok || gk >= K) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (gk + 4 <= K) return *reinterpret_cast<const float4*>(p);
    float4 v = make_float4(p[0], 0.f, 0.f, 0.f);
    if (gk + 1 < K) v.y = p[1];
    if (gk + 2 < K) v.z = p[2];
    return v;
}

template <int WGM, int WGN, int TM, int TN>
__global__ __launch_bounds__(WGM* WGN * 64) void k_linear_f32(const float* __restrict__ x, long long ldx,
                                                               const float* __restrict__ w, long long ldw,
                                                               const float* __restrict__ bias, int M, int N, int K,
                                                               int act, float* __restrict__ y, long long ldy) {
    using C = Cfg<WGM, WGN, TM, TN>;
    __shared__ __attribute__((aligned(16))) float As[C::BM * LDP];
    __shared__ __attribute__((aligned(16))) float Bs[C::BN * LDP];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WGN, wc = wave % WGN;

    // XCD-aware bijective remap: blocks b and b+8 share an XCD; give one XCD a
    // contiguous run of tiles (same m-tile => same x rows in that XCD's L2).
    const int nM = (M + C::BM - 1) / C::BM, nN = (N + C::BN - 1) / C::BN;
    const int T = nM * nN;
    int bid = blockIdx.x;
    {
        const int q = T / 8, r = T % 8, xcd = bid % 8, loc = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    }
    const int m0 = (bid / nN) * C::BM, n0 = (bid % nN) * C::BN;

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

    float4 ra[C::A_F4], rb[C::B_F4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int q = 0; q < C::A_F4; q++) {
            int idx = tid + q * C::THREADS, row = idx / (BK / 4), c4 = idx % (BK / 4);
            int gm = m0 + row, gk = k0 + 4 * c4;
            ra[q] = ld4(x + (long long)gm * ldx + gk, gm < M, gk, K);
        }
#pragma unroll
        for (int q = 0; q < C::B_F4; q++) {
            int idx = tid + q * C::THREADS, row = idx / (BK / 4), c4 = idx % (BK / 4);
            int gn = n0 + row, gk = k0 + 4 * c4;
            rb[q] = ld4(w + (long long)gn * ldw + gk, gn < N, gk, K);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int q = 0; q < C::A_F4; q++) {
            int idx = tid + q * C::THREADS, row = idx / (BK / 4), c4 = idx % (BK / 4);
            *reinterpret_cast<float4*>(&As[row * LDP + 4 * c4]) = ra[q];
        }
#pragma unroll
        for (int q = 0; q < C::B_F4; q++) {
            int idx = tid + q * C::THREADS, row = idx / (BK / 4), c4 = idx % (BK / 4);
            *reinterpret_cast<float4*>(&Bs[row * LDP + 4 * c4]) = rb[q];
        }
    };

    const int h = lane >> 5, l32 = lane & 31;
    gload(0);
    for (int k0 = 0; k0 < K; k0 += BK) {
        __syncthreads();
        lstore();
        __syncthreads();
        if (k0 + BK < K) gload(k0 + BK);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            float4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; i++)
                af[i] = *reinterpret_cast<const float4*>(
                    &As[(wr * TM * 32 + i * 32 + l32) * LDP + h * 16 + 4 * s4]);
#pragma unroll
            for (int j = 0; j < TN; j++)
                bf[j] = *reinterpret_cast<const float4*>(
                    &Bs[(wc * TN * 32 + j * 32 + l32) * LDP + h * 16 + 4 * s4]);
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
    }

    // epilogue: C/D map col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
    for (int j = 0; j < TN; j++) {
        const int col = n0 + wc * TN * 32 + j * 32 + l32;
        const float bv = (bias && col < N) ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; i++) {
            const int rbase = m0 + wr * TM * 32 + i * 32 + 4 * h;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = rbase + (r & 3) + 8 * (r >> 2);
                float v = acc[i][j][r] + bv;
                if (act == 1) v = v >= 0.f ? v : 0.01f * v;
                if (row < M && col < N) y[(long long)row * ldy + col] = v;
            }
        }
    }
}

template <int WGM, int WGN, int TM, int TN>
int launch(const float* x, long long ldx, const float* w, long long ldw, const float* b, int M, int N, int K, int act,
           float* y, long long ldy, hipStream_t st) {
    using C = Cfg<WGM, WGN, TM, TN>;
    const int T = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
    hipLaunchKernelGGL((k_linear_f32<WGM, WGN, TM, TN>), dim3(T), dim3(C::THREADS), 0, st, x, ldx, w, ldw, b, M, N, K, act,
                       y, ldy);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_linear_f32 launch: ") + hipGetErrorString(e));
    return GM_OK;
}

}  // namespace

extern "C" int gm_linear_f32(const float* x, int64_t ldx, const float* w, int64_t ldw, const float* b, int32_t m,
                             int32_t n, int32_t k, int32_t act, float* y, int64_t ldy, void* stream) {
    if (!x || !w || !y || m <= 0 || n <= 0 || k <= 0 || (ldx & 3) || (ldw & 3) || ldx < k || ldw < k || ldy < n ||
        (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) || act < 0 || act > 1)
        return gm_fail(GM_ERR_INVALID_ARG,
                       "gm_linear_f32: bad arguments (ldx, ldw multiples of 4; 16-byte aligned x and w)");
    hipStream_t st = (hipStream_t)stream;
    if (n <= 32) return launch<4, 1, 1, 1>(x, ldx, w, ldw, b, m, n, k, act, y, ldy, st);
    return launch<2, 2, 2, 2>(x, ldx, w, ldw, b, m, n, k, act, y, ldy, st);
}
