// gm_netmon.hip — NetMon message passing (reference src/model.py:206-229,
// 476-631) as HBM-bound HIP kernels for gfx950.
//
// Graph layout: node rows h[G*N][H] (fp32, row-major; float4 lanes when H % 4 == 0), neighbour
// table nbr[G][N][deg] (ELL, ascending ids, -1 = none). The reference multiplies a
// dense (I+A) mask with h (bmm); with deg 3 that reads 4 rows per output row, so
// the aggregate is a gather of 4 contiguous 512-byte rows per node with float4
// lanes: 32 lanes per row, a wave covers 2 rows, consecutive rows share the same
// graph's 10 KB working set in L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/graph_marl_amd.h"
#include "gm_amax.hpp"
#include "gm_act.hpp"

int gm_fail(int code, const std::string& msg);

namespace {

constexpr int MAXDEG = 8;

// V-wide fp32 vectors (V = 4, 2 or 1 chosen from H's alignment on the host)
template <int V> struct Vec { float v[V]; };
template <int V> __device__ __forceinline__ Vec<V> ldv(const float* p) {
    Vec<V> r;
    if constexpr (V == 4) {
        float4 t = *reinterpret_cast<const float4*>(p);
        r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
    } else if constexpr (V == 2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        r.v[0] = t.x; r.v[1] = t.y;
    } else {
        r.v[0] = *p;
    }
    return r;
}
template <int V> __device__ __forceinline__ void stv(float* p, const Vec<V>& a) {
    if constexpr (V == 4) *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
    else if constexpr (V == 2) *reinterpret_cast<float2*>(p) = make_float2(a.v[0], a.v[1]);
    else *p = a.v[0];
}
template <int V> __device__ __forceinline__ Vec<V> zerov() {
    Vec<V> r;
#pragma unroll
    for (int i = 0; i < V; i++) r.v[i] = 0.f;
    return r;
}

// sorted member list {n} ∪ nbr(n) (ascending node id) — the summation order of a
// sequential dense row product (I+A)[n,:] · h
__device__ __forceinline__ int members(const int32_t* nb, int deg, int n, int* out) {
    int cnt = 0;
    bool self_done = false;
    for (int k = 0; k < deg; k++) {
        int v = nb[k];
        if (v < 0) continue;
        if (!self_done && n < v) {
            out[cnt++] = n;
            self_done = true;
        }
        out[cnt++] = v;
    }
    if (!self_done) out[cnt++] = n;
    return cnt;
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// XCD-aware block order: the hardware deals block b to XCD b % 8; logical block numbers are
// handed out so that each XCD gets one contiguous run of rows, and the 4 rows every node reads
// (itself + 3 neighbours of the same graph) sit in that XCD's L2 instead of being fetched once per
// XCD that touches the graph (a graph's 20 rows span 3 consecutive 8-row blocks)
__device__ __forceinline__ unsigned xcd_block(unsigned bid, unsigned T) {
    const unsigned q = T / 8, r = T % 8, x = bid % 8, loc = bid / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + loc;
}

// forward: out[n] = Σ_{m ∈ {n} ∪ nbr(n)} h[m]  (/ count for mean)
// backward (symmetric adjacency): dh[j] = Σ_{n ∈ {j} ∪ nbr(j)} dout[n] * scale(n)
template <bool BWD, int V>
__global__ __launch_bounds__(256) void k_mp_aggregate(const float* __restrict__ h, const int32_t* __restrict__ nbr,
                                                      int G, int N, int deg, int H, int mode, float* __restrict__ out,
                                                      long long ldh, long long ldo) {
    const int HV = H / V;
    const long long gid = (long long)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    const long long total = (long long)G * N * HV;
    if (gid >= total) return;
    const int cv = (int)(gid % HV);
    const long long row = gid / HV;
    const int g = (int)(row / N), n = (int)(row % N);
    const int32_t* nb = nbr + ((size_t)g * N + n) * deg;
    int mem[MAXDEG + 1];
    const int cnt = members(nb, deg, n, mem);
    const float* src = h + (size_t)g * N * ldh + (size_t)cv * V;
    Vec<V> acc = zerov<V>();
    if (!BWD && deg <= 3) {
        // routing graphs (degree 3): the up to 4 member rows are loaded back to back (independent
        // loads in flight together), then summed in ascending id order like the general loop
        Vec<V> x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = q < cnt ? ldv<V>(src + (size_t)mem[q] * ldh) : zerov<V>();
        acc = x[0];
#pragma unroll
        for (int q = 1; q < 4; q++)
            if (q < cnt) {
#pragma unroll
                for (int i = 0; i < V; i++) acc.v[i] = acc.v[i] + x[q].v[i];
            }
        if (mode == 1) {
#pragma unroll
            for (int i = 0; i < V; i++) acc.v[i] = acc.v[i] / cnt;
        }
        stv<V>(out + row * ldo + (size_t)cv * V, acc);
        return;
    }
    for (int q = 0; q < cnt; q++) {
        Vec<V> x = ldv<V>(src + (size_t)mem[q] * ldh);
        if (BWD && mode == 1) {
            const int32_t* nbm = nbr + ((size_t)g * N + mem[q]) * deg;
            int cm = 1;
            for (int k = 0; k < deg; k++) cm += nbm[k] >= 0;
#pragma unroll
            for (int i = 0; i < V; i++) x.v[i] = x.v[i] * (1.0f / (float)cm);
        }
#pragma unroll
        for (int i = 0; i < V; i++) acc.v[i] = q == 0 ? x.v[i] : acc.v[i] + x.v[i];
    }
    if (!BWD && mode == 1) {
#pragma unroll
        for (int i = 0; i < V; i++) acc.v[i] = acc.v[i] / cnt;
    }
    stv<V>(out + row * ldo + (size_t)cv * V, acc);
}

// forward of k_mp_aggregate for degree-3 graphs with fewer than 2^31 (row, vector) items: 32-bit index
// math (the 64-bit divisions of the general kernel were most of its instructions) and the members
// {n} u nbr(n) put in ascending id order by a 4-input sorting network (missing neighbours last) instead of
// members()'s dynamically indexed local array; the same members, the same summation order
template <int V>
__global__ __launch_bounds__(256) void k_mp_aggregate3(const float* __restrict__ h, const int32_t* __restrict__ nbr,
                                                       unsigned N, unsigned HV, int mode, float* __restrict__ out,
                                                       long long ldh, long long ldo, unsigned total) {
    const unsigned gid = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const unsigned row = gid / HV, cv = gid - row * HV;
    const unsigned g = row / N;
    const int32_t* nb = nbr + (size_t)row * 3;
    constexpr int MISSING = 0x7fffffff;
    int m[4] = {(int)(row - g * N), nb[0] < 0 ? MISSING : nb[0], nb[1] < 0 ? MISSING : nb[1],
                nb[2] < 0 ? MISSING : nb[2]};
    const int cnt = 1 + (m[1] != MISSING) + (m[2] != MISSING) + (m[3] != MISSING);
    auto cswap = [](int& a, int& b) {
        const int lo = min(a, b), hi = max(a, b);
        a = lo;
        b = hi;
    };
    cswap(m[0], m[1]);
    cswap(m[2], m[3]);
    cswap(m[0], m[2]);
    cswap(m[1], m[3]);
    cswap(m[1], m[2]);
    const float* src = h + (size_t)g * N * ldh + (size_t)cv * V;
    Vec<V> x[4];
#pragma unroll
    for (int q = 0; q < 4; q++) x[q] = q < cnt ? ldv<V>(src + (size_t)m[q] * ldh) : zerov<V>();
    Vec<V> acc = x[0];
#pragma unroll
    for (int q = 1; q < 4; q++)
        if (q < cnt) {
#pragma unroll
            for (int i = 0; i < V; i++) acc.v[i] = acc.v[i] + x[q].v[i];
        }
    if (mode == 1) {
#pragma unroll
        for (int i = 0; i < V; i++) acc.v[i] = acc.v[i] / cnt;
    }
    stv<V>(out + (size_t)row * ldo + (size_t)cv * V, acc);
}

// readout: out row r of graph g = [h_final[v], h_prev[nbr(v,0..deg-1)]], v = agent_node or r.
// Output rows may sit inside a wider joint observation (stride); V-wide stores.
template <int V>
__global__ __launch_bounds__(256) void k_readout(const float* __restrict__ hf, const float* __restrict__ hp,
                                                 const int32_t* __restrict__ nbr, const int32_t* __restrict__ agent_node,
                                                 int G, int N, int R, int deg, int H, float* __restrict__ out,
                                                 long long stride, long long ldf, long long ldp) {
    const int HV = H / V;
    const int WV = (deg + 1) * HV;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)G * R * WV;
    if (gid >= total) return;
    const int cv = (int)(gid % WV);
    const long long row = gid / WV;
    const int g = (int)(row / R), r = (int)(row % R);
    const int v = agent_node ? agent_node[(size_t)g * R + r] : r;
    const int seg = cv / HV, off = (cv - seg * HV) * V;
    Vec<V> val;
    if (seg == 0) {
        val = ldv<V>(hf + ((size_t)g * N + v) * ldf + off);
    } else {
        int m = nbr[((size_t)g * N + v) * deg + seg - 1];
        val = m >= 0 ? ldv<V>(hp + ((size_t)g * N + m) * ldp + off) : zerov<V>();
    }
    stv<V>(out + row * stride + (size_t)cv * V, val);
}

// readout backward, deterministic (no atomics): node v of graph g gathers the
// gradient of every row that read it, rows in ascending order.
template <int V>
__global__ __launch_bounds__(256) void k_readout_bwd(const float* __restrict__ dout, long long stride,
                                                     const int32_t* __restrict__ nbr,
                                                     const int32_t* __restrict__ agent_node, int G, int N, int R,
                                                     int deg, int H, float* __restrict__ dhf, float* __restrict__ dhp) {
    const int HV = H / V;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)G * N * HV;
    if (gid >= total) return;
    const int off = (int)(gid % HV) * V;
    const long long node = gid / HV;
    const int g = (int)(node / N), v = (int)(node % N);
    Vec<V> af = zerov<V>(), ap = zerov<V>();
    for (int r = 0; r < R; r++) {
        const int u = agent_node ? agent_node[(size_t)g * R + r] : r;
        const float* drow = dout + ((size_t)g * R + r) * stride;
        if (u == v) {
            Vec<V> x = ldv<V>(drow + off);
#pragma unroll
            for (int i = 0; i < V; i++) af.v[i] += x.v[i];
        }
        const int32_t* nb = nbr + ((size_t)g * N + u) * deg;
        for (int k = 0; k < deg; k++) {
            if (nb[k] == v) {
                Vec<V> x = ldv<V>(drow + (size_t)(k + 1) * H + off);
#pragma unroll
                for (int i = 0; i < V; i++) ap.v[i] += x.v[i];
            }
        }
    }
    if (dhf) stv<V>(dhf + node * H + off, af);
    if (dhp) stv<V>(dhp + node * H + off, ap);
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// nn.LSTMCell gate math (i, f, g, o): c' = σ(f)c + σ(i)tanh(g), h' = σ(o)tanh(c')
__global__ __launch_bounds__(256) void k_lstm_pw(const float* __restrict__ gates, const float* __restrict__ c,
                                                 int M, int H, float* __restrict__ h1, float* __restrict__ c1,
                                                 float* __restrict__ act) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)M * H) return;
    const long long m = gid / H;
    const int j = (int)(gid % H);
    const float* g = gates + m * 4 * H;
    float i = sigm(g[j]), f = sigm(g[H + j]), gg = tanhf(g[2 * H + j]), o = sigm(g[3 * H + j]);
    float cn = f * c[gid] + i * gg;
    float hn = o * tanhf(cn);
    c1[gid] = cn;
    h1[gid] = hn;
    if (act) {
        float* a = act + m * 4 * H;
        a[j] = i;
        a[H + j] = f;
        a[2 * H + j] = gg;
        a[3 * H + j] = o;
    }
}

__global__ __launch_bounds__(256) void k_lstm_pw_bwd(const float* __restrict__ dh1, const float* __restrict__ dc1,
                                                     const float* __restrict__ act, const float* __restrict__ c,
                                                     const float* __restrict__ c1, int M, int H,
                                                     float* __restrict__ dgates, float* __restrict__ dc,
                                                     unsigned* __restrict__ amax) {
    float mx = 0.f;
    const long long total = (long long)M * H;
    for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
         gid += (long long)gridDim.x * blockDim.x) {
        const long long m = gid / H;
        const int j = (int)(gid % H);
        const float* a = act + m * 4 * H;
        float i = a[j], f = a[H + j], gg = a[2 * H + j], o = a[3 * H + j];
        float tc = tanhf(c1[gid]);
        float dh = dh1 ? dh1[gid] : 0.f;
        float dct = (dc1 ? dc1[gid] : 0.f) + dh * o * (1.f - tc * tc);
        float* dg = dgates + m * 4 * H;
        const float d0 = dct * gg * i * (1.f - i), d1 = dct * c[gid] * f * (1.f - f);
        const float d2 = dct * i * (1.f - gg * gg), d3 = dh * tc * o * (1.f - o);
        dg[j] = d0;
        dg[H + j] = d1;
        dg[2 * H + j] = d2;
        dg[3 * H + j] = d3;
        dc[gid] = dct * f;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(d0), fabsf(d1)), fmaxf(fabsf(d2), fabsf(d3))));
    }
    if (amax) gm_block_amax(amax, mx);
}


// bits 0..15 of x to the even bit positions 0, 2, .., 30
__device__ __forceinline__ unsigned spread16(unsigned x) {
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// First NetMon encoder layer on routing node observations (src/model.py:272-276 on the
// node obs of src/env/routing.py:187-235). Row n of graph g is
//   [onehot(n) | cnt | load | 3 x (onehot(nbr_k) | len_k | load_k)]
// so W x touches 12 of the 4N+8 weight columns: the dense GEMM's K = 4N+8 collapses to a
// 12-term gather over W^T staged in LDS (BN output columns per block, 64 lanes x BN/64
// columns). HBM-bound on the output rows (n floats per node).
template <int AC>
__device__ __forceinline__ float renc_act(float v, int act) {
    if constexpr (AC == 0)
        return v;
    else if constexpr (AC == 1)
        return v >= 0.f ? v : 0.01f * v;
    else
        return gm_act_fast(v, act);
}

// AC: the activation at compile time (0 none, 1 leaky_relu) or -1 = GM_ACT_* `act` at run time (a per
// element branch tree: kept out of the default kernels, it cost 65 -> 76 us per 81 920 rows)
template <int CPL, int AC, int TPB = 256>  // output columns per lane (BN = 64 * CPL), threads per block
__global__ __launch_bounds__(TPB) void k_routing_enc(const float* __restrict__ x, long long ldx,
                                                     const int32_t* __restrict__ nbr, int G, int N,
                                                     const float* __restrict__ wt, const float* __restrict__ b,
                                                     int n, int act, float* __restrict__ y, long long ldy,
                                                     int rows_per_block, unsigned* __restrict__ sbits,
                                                     long long ldsb) {
    constexpr int BN = 64 * CPL;
    extern __shared__ __attribute__((aligned(16))) float sw[];  // [K][BN]
    const int K = 4 * N + 8;
    const int c0 = blockIdx.y * BN;
    for (int i = threadIdx.x; i < K * (BN / 4); i += blockDim.x) {
        const int r = i / (BN / 4), c4 = i - r * (BN / 4);
        reinterpret_cast<float4*>(sw)[i] = *reinterpret_cast<const float4*>(wt + (size_t)r * n + c0 + 4 * c4);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = CPL * lane;
    float bias[CPL];
#pragma unroll
    for (int j = 0; j < CPL; j++) bias[j] = b ? b[c0 + col + j] : 0.f;
    const long long M = (long long)G * N;
    // each wave owns groups of 64 consecutive rows: lane l gathers the 11 nonzero features of
    // row base + l up front (coalesced, one latency), the row loop broadcasts them by readlane;
    // the block's W^T slice is staged once for rows_per_block rows
    const long long bend = min(M, (long long)(blockIdx.x + 1) * rows_per_block);
    for (long long base = (long long)blockIdx.x * rows_per_block + (long long)wv * 64; base < bend;
         base += (blockDim.x >> 6) * 64) {
    const int nrows = bend - base < 64 ? (int)(bend - base) : 64;
    int fv = 0, f_nb[3] = {0, 0, 0};
    float f_cnt = 0.f, f_tl = 0.f, f_len[3] = {0.f, 0.f, 0.f}, f_ld[3] = {0.f, 0.f, 0.f};
    if (lane < nrows) {
        const long long r = base + lane;
        const int g = (int)(r / N);
        fv = (int)(r - (long long)g * N);
        const float* xr = x + r * ldx;
        f_cnt = xr[N];
        f_tl = xr[N + 1];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int off = N + 2 + k * (N + 2);
            f_len[k] = xr[off + N];
            f_ld[k] = xr[off + N + 1];
            f_nb[k] = nbr[((size_t)g * N + fv) * 3 + k];
        }
    }
    // weight columns of the 8 scalar features (cnt, load, 3 x (len, load)) stay in registers;
    // only the 4 one-hot columns (node, 3 neighbours) are looked up in LDS per row
    float wc[4][2][CPL];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int off = k == 0 ? N : N + 2 + (k - 1) * (N + 2) + N;
#pragma unroll
        for (int j = 0; j < CPL; j++) {
            wc[k][0][j] = sw[off * BN + col + j];
            wc[k][1][j] = sw[(off + 1) * BN + col + j];
        }
    }
    for (int i = 0; i < nrows; i++) {
        const int v = __builtin_amdgcn_readlane(fv, i);
        const float cnt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f_cnt), i));
        const float tl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f_tl), i));
        float acc[CPL];
        // one-hot weight rows as 8-byte LDS reads (CPL = 2: ds_read_b64 is conflict-free; the
        // ds_read2_b32 the compiler made of two float reads spent 54 % of its LDS cycles in bank
        // conflicts, though the kernel time did not change: 57.5 vs 57.7 us per 81 920 rows)
        auto wrow = [&](int r, float (&e)[CPL]) {
            if constexpr (CPL == 2) {
                const float2 t = *reinterpret_cast<const float2*>(sw + r * BN + col);
                e[0] = t.x;
                e[CPL - 1] = t.y;
            } else {
#pragma unroll
                for (int j = 0; j < CPL; j++) e[j] = sw[r * BN + col + j];
            }
        };
        float e0[CPL];
        wrow(v, e0);
#pragma unroll
        for (int j = 0; j < CPL; j++) acc[j] = bias[j] + e0[j] + cnt * wc[0][0][j] + tl * wc[0][1][j];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int off = N + 2 + k * (N + 2);
            const int u = __builtin_amdgcn_readlane(f_nb[k], i);
            const float ln = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f_len[k]), i));
            const float ld = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f_ld[k]), i));
            float ek[CPL];
            wrow(off + u, ek);
#pragma unroll
            for (int j = 0; j < CPL; j++) acc[j] += ek[j] + ln * wc[k + 1][0][j] + ld * wc[k + 1][1][j];
        }
        float* yr = y + (base + i) * ldy + c0 + col;
        if (CPL == 2) {
            float a0 = acc[0], a1 = acc[CPL - 1];
            a0 = renc_act<AC>(a0, act);
            a1 = renc_act<AC>(a1, act);
            *reinterpret_cast<float2*>(yr) = make_float2(a0, a1);
            if (sbits) {  // 32-column sign words: lanes 16k..16k+15 hold columns 32k..32k+31, two each
                const unsigned long long b0 = __ballot(a0 > 0.f), b1 = __ballot(a1 > 0.f);
                if ((lane & 15) == 0) {
                    const int k = lane >> 4;
                    sbits[(base + i) * ldsb + (c0 >> 5) + k] =
                        spread16((unsigned)(b0 >> (16 * k)) & 0xFFFFu) | (spread16((unsigned)(b1 >> (16 * k)) & 0xFFFFu) << 1);
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < CPL; j++) yr[j] = renc_act<AC>(acc[j], act);
            if (sbits) {
                const float a0 = renc_act<AC>(acc[0], act);
                const unsigned long long b0 = __ballot(a0 > 0.f);
                if ((lane & 31) == 0) sbits[(base + i) * ldsb + (c0 >> 5) + (lane >> 5)] = (unsigned)(b0 >> lane);
            }
        }
    }
    }
}

inline unsigned nblocks(long long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

int launched() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return GM_OK;
}

}  // namespace

// widest vector that divides H and keeps every access aligned (base pointers are
// torch allocations; strides are checked)
static int vec_width(int H, long long stride, const void* p) {
    if (H % 4 == 0 && stride % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0) return 4;
    if (H % 2 == 0 && stride % 2 == 0 && (reinterpret_cast<uintptr_t>(p) & 7) == 0) return 2;
    return 1;
}

#define GM_VLAUNCH(KER, V, GRID, ...)                                                                  \
    do {                                                                                               \
        if ((V) == 4) hipLaunchKernelGGL(KER<4>, GRID, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
        else if ((V) == 2) hipLaunchKernelGGL(KER<2>, GRID, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__); \
        else hipLaunchKernelGGL(KER<1>, GRID, dim3(256), 0, (hipStream_t)stream, __VA_ARGS__);        \
    } while (0)

template <bool BWD>
static int launch_agg(const float* h, const int32_t* nbr, int32_t G, int32_t N, int32_t deg, int32_t H, int32_t mode,
                      float* out, void* stream, long long ldh = 0, long long ldo = 0) {
    if (!ldh) ldh = H;
    if (!ldo) ldo = H;
    const int V = vec_width(H, ldh, h) < vec_width(H, ldo, out) ? vec_width(H, ldh, h) : vec_width(H, ldo, out);
    long long total = (long long)G * N * (H / V);
    dim3 grid(nblocks(total, 256));
    if (!BWD && deg == 3 && total < (1ll << 31)) {
        GM_VLAUNCH(k_mp_aggregate3, V, grid, h, nbr, (unsigned)N, (unsigned)(H / V), mode, out, ldh, ldo, (unsigned)total);
        return launched();
    }
    if (V == 4) hipLaunchKernelGGL((k_mp_aggregate<BWD, 4>), grid, dim3(256), 0, (hipStream_t)stream, h, nbr, G, N, deg, H, mode, out, ldh, ldo);
    else if (V == 2) hipLaunchKernelGGL((k_mp_aggregate<BWD, 2>), grid, dim3(256), 0, (hipStream_t)stream, h, nbr, G, N, deg, H, mode, out, ldh, ldo);
    else hipLaunchKernelGGL((k_mp_aggregate<BWD, 1>), grid, dim3(256), 0, (hipStream_t)stream, h, nbr, G, N, deg, H, mode, out, ldh, ldo);
    return launched();
}

// Backward of act(x W^T + b) with leaky_relu(0.01) after the Linear (reference MLP,
// src/model.py:13-42): g = dY * (Y >= 0 ? 1 : slope), and per-block column sums of g for the
// bias gradient (partial[block][col]; the caller sums the blocks: a fixed summation order).
// Threads own columns, blocks own row chunks; loads and stores are row-contiguous.
// act < 0: leaky_relu with the given slope; else GM_ACT_* (derivative from the output, gm_act.hpp)
__global__ __launch_bounds__(256) void k_leaky_bwd(const float* __restrict__ gy, const float* __restrict__ y,
                                                   long long rows, int cols, int rows_per_block, float slope,
                                                   int act, int fromz, float* __restrict__ g,
                                                   float* __restrict__ part, unsigned* __restrict__ amax) {
    const long long r0 = (long long)blockIdx.x * rows_per_block;
    const long long r1 = min(rows, r0 + rows_per_block);
    float m = 0.f;
    for (int c = threadIdx.x; c < cols; c += blockDim.x) {
        float acc = 0.f;
        for (long long r = r0; r < r1; r++) {
            const long long i = r * cols + c;
            // torch: input > 0 ? g : slope g; fromz: y holds the pre-activation z (gm_act_bwd_z)
            const float v = act < 0 ? (y[i] > 0.f ? gy[i] : slope * gy[i])
                                    : gy[i] * (fromz ? gm_act_dz(y[i], act) : gm_act_dy(y[i], act));
            g[i] = v;
            acc += v;
            m = fmaxf(m, fabsf(v));
        }
        part[(long long)blockIdx.x * cols + c] = acc;
    }
    if (amax) gm_block_amax(amax, m);
}

static int act_bwd(const char* fn, const float* gy, const float* y, int64_t rows, int32_t cols, float slope, int act,
                   float* g, float* part, int32_t rows_per_block, float* g_scale, void* stream, int fromz = 0) {
    if (!gy || !y || !g || !part || rows <= 0 || cols <= 0 || rows_per_block <= 0)
        return gm_fail(GM_ERR_INVALID_ARG, std::string(fn) + ": bad arguments");
    hipStream_t st = (hipStream_t)stream;
    if (g_scale && hipMemsetAsync(g_scale, 0, sizeof(float), st) != hipSuccess)
        return gm_fail(GM_ERR_HIP, std::string(fn) + ": memset");
    const long long nb = (rows + rows_per_block - 1) / rows_per_block;
    hipLaunchKernelGGL(k_leaky_bwd, dim3((unsigned)nb), dim3(256), 0, st, gy, y, (long long)rows, (int)cols,
                       (int)rows_per_block, slope, act, fromz, g, part, reinterpret_cast<unsigned*>(g_scale));
    int rc = launched();
    if (rc == GM_OK && g_scale) rc = gm_absmax_finish(g_scale, stream);
    return rc;
}

extern "C" int gm_leaky_bwd(const float* gy, const float* y, int64_t rows, int32_t cols, float slope, float* g,
                            float* part, int32_t rows_per_block, float* g_scale, void* stream) {
    return act_bwd("gm_leaky_bwd", gy, y, rows, cols, slope, -1, g, part, rows_per_block, g_scale, stream);
}

extern "C" int gm_act_bwd(const float* gy, const float* y, int64_t rows, int32_t cols, int32_t act, float* g,
                          float* part, int32_t rows_per_block, float* g_scale, void* stream) {
    if (act < GM_ACT_NONE || act > GM_ACT_SOFTPLUS)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_act_bwd: unknown act (codes >= GM_ACT_GELU: gm_act_bwd_z)");
    return act_bwd("gm_act_bwd", gy, y, rows, cols, 0.f, act, g, part, rows_per_block, g_scale, stream);
}

extern "C" int gm_act_bwd_z(const float* gy, const float* z, int64_t rows, int32_t cols, int32_t act, float* g,
                            float* part, int32_t rows_per_block, float* g_scale, void* stream) {
    if (act < GM_ACT_NONE || act > GM_ACT_LAST) return gm_fail(GM_ERR_INVALID_ARG, "gm_act_bwd_z: unknown act");
    return act_bwd("gm_act_bwd_z", gy, z, rows, cols, 0.f, act, g, part, rows_per_block, g_scale, stream, 1);
}

// y = act(z) elementwise (the training forward of the activations whose derivative needs z)
__global__ __launch_bounds__(256) void k_act_fwd(const float* __restrict__ z, long long n, int act, float* __restrict__ y) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        y[i] = gm_act(z[i], act);
}

extern "C" int gm_act_fwd(const float* z, int64_t rows, int32_t cols, int32_t act, float* y, void* stream) {
    if (!z || !y || rows <= 0 || cols <= 0 || act < GM_ACT_NONE || act > GM_ACT_LAST)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_act_fwd: bad arguments");
    const long long n = (long long)rows * cols;
    long long nb = (n + 255) / 256;
    if (nb > 65536) nb = 65536;
    hipLaunchKernelGGL(k_act_fwd, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, z, n, (int)act, y);
    return launched();
}

extern "C" int gm_mp_aggregate(const float* h, const int32_t* nbr, int32_t G, int32_t N, int32_t deg, int32_t H,
                               int32_t mode, float* out, void* stream) {
    if (!h || !nbr || !out || G <= 0 || N <= 0 || deg < 0 || deg > MAXDEG || H <= 0 || mode < 0 || mode > 1)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_mp_aggregate: bad arguments (deg <= 8)");
    return launch_agg<false>(h, nbr, G, N, deg, H, mode, out, stream);
}

extern "C" int gm_mp_aggregate_rows(const float* h, int64_t ldh, const int32_t* nbr, int32_t G, int32_t N, int32_t deg,
                                    int32_t H, int32_t mode, float* out, int64_t ldo, void* stream) {
    if (!h || !nbr || !out || G <= 0 || N <= 0 || deg < 0 || deg > MAXDEG || H <= 0 || mode < 0 || mode > 1 ||
        ldh < H || ldo < H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_mp_aggregate_rows: bad arguments (deg <= 8, ld >= H)");
    return launch_agg<false>(h, nbr, G, N, deg, H, mode, out, stream, ldh, ldo);
}

extern "C" int gm_mp_aggregate_bwd(const float* dout, const int32_t* nbr, int32_t G, int32_t N, int32_t deg,
                                   int32_t H, int32_t mode, float* dh, void* stream) {
    if (!dout || !nbr || !dh || G <= 0 || N <= 0 || deg < 0 || deg > MAXDEG || H <= 0 || mode < 0 || mode > 1)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_mp_aggregate_bwd: bad arguments");
    return launch_agg<true>(dout, nbr, G, N, deg, H, mode, dh, stream);
}

// readout, one wave per output row (the row's node and neighbour ids read once, as wave-uniform
// loads), 16-byte lanes over the (deg + 1) * H columns; two rows per iteration keep 4 independent
// loads in flight per lane. Requires H % 4 == 0 and 16-byte aligned rows (host-checked).
__global__ __launch_bounds__(256) void k_readout_rows(const float* __restrict__ hf, const float* __restrict__ hp,
                                                      const int32_t* __restrict__ nbr,
                                                      const int32_t* __restrict__ agent_node, long long rows, int N,
                                                      int R, int deg, int H, float* __restrict__ out,
                                                      long long stride, long long ldf, long long ldp) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const int H4 = H >> 2, W4 = (deg + 1) * H4;
    // U rows per iteration: their node ids first, then every row's loads, then the stores
    constexpr int U = 4, C = 2;  // C float4 per lane and row cover W4 <= 128 (larger W4: the loop below)
    for (long long rb = wave * U; rb < rows; rb += nw * U) {
        long long src[U][C];
        float* dst[U];
        bool okc[U][C];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const long long row = min(rb + k, rows - 1);
            const long long g = row / R;
            const int r = (int)(row - g * R);
            const int v = agent_node ? agent_node[row] : r;
            dst[k] = (rb + k < rows) ? out + row * stride : nullptr;
#pragma unroll
            for (int cc = 0; cc < C; cc++) {
                const int c = lane + 64 * cc;
                const int seg = c / H4, off = (c - seg * H4) * 4;
                okc[k][cc] = c < W4;
                const int m = seg == 0 ? v : (c < W4 ? nbr[(g * N + v) * deg + seg - 1] : -1);
                src[k][cc] = m < 0 ? -1 : (seg == 0 ? (g * N + m) * ldf + off : -(2 + (g * N + m) * ldp + off));
            }
        }
        float4 val[U][C];
#pragma unroll
        for (int k = 0; k < U; k++)
#pragma unroll
            for (int cc = 0; cc < C; cc++) {
                const long long o = src[k][cc];
                val[k][cc] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (okc[k][cc] && o != -1) val[k][cc] = o >= 0 ? *reinterpret_cast<const float4*>(hf + o)
                                                                : *reinterpret_cast<const float4*>(hp + (-o - 2));
            }
#pragma unroll
        for (int k = 0; k < U; k++)
#pragma unroll
            for (int cc = 0; cc < C; cc++)
                if (dst[k] && okc[k][cc]) *reinterpret_cast<float4*>(dst[k] + 4 * (lane + 64 * cc)) = val[k][cc];
        for (int k = 0; k < U && W4 > 64 * C; k++) {  // columns past 64 C float4 (wide readouts)
            const long long row = rb + k;
            if (row >= rows) break;
            const long long g = row / R;
            const int r = (int)(row - g * R);
            const int v = agent_node ? agent_node[row] : r;
            for (int c = lane + 64 * C; c < W4; c += 64) {
                const int seg = c / H4, off = (c - seg * H4) * 4;
                float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
                if (seg == 0) {
                    x = *reinterpret_cast<const float4*>(hf + (g * N + v) * ldf + off);
                } else {
                    const int m = nbr[(g * N + v) * deg + seg - 1];
                    if (m >= 0) x = *reinterpret_cast<const float4*>(hp + (g * N + m) * ldp + off);
                }
                *reinterpret_cast<float4*>(out + row * stride + 4 * c) = x;
            }
        }
    }
}

// readout backward, one block per graph: the graph's R output rows ((deg + 1) H floats each) are
// staged in LDS with coalesced 16-byte loads, then thread (node, 4 columns) sums the rows that read
// it in the same (row, segment) order as k_readout_bwd (identical results)
__global__ __launch_bounds__(1024) void k_readout_bwd_lds(const float* __restrict__ dout, long long stride,
                                                          const int32_t* __restrict__ nbr,
                                                          const int32_t* __restrict__ agent_node, int N, int R,
                                                          int deg, int H, float* __restrict__ dhf,
                                                          float* __restrict__ dhp) {
    extern __shared__ float sd[];  // [R][(deg + 1) H]
    __shared__ int su[64];
    __shared__ int snb[64 * MAXDEG];
    const long long g = blockIdx.x;
    const int W = (deg + 1) * H, W4 = W >> 2;
    for (int i = threadIdx.x; i < R; i += blockDim.x) su[i] = agent_node ? agent_node[g * R + i] : i;
    for (int i = threadIdx.x; i < R * W4; i += blockDim.x) {
        const int r = i / W4, c = i - r * W4;
        reinterpret_cast<float4*>(sd)[i] = *reinterpret_cast<const float4*>(dout + (g * R + r) * stride + 4 * c);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R * deg; i += blockDim.x) {
        const int r = i / deg, k = i - r * deg;
        snb[i] = nbr[(g * N + su[r]) * deg + k];
    }
    __syncthreads();
    const int H4 = H >> 2;
    for (int t = threadIdx.x; t < N * H4; t += blockDim.x) {
        const int v = t / H4, off = (t - v * H4) * 4;
        float4 af = make_float4(0.f, 0.f, 0.f, 0.f), ap = af;
        for (int r = 0; r < R; r++) {
            const float* drow = sd + r * W;
            if (su[r] == v) af = f4add(af, *reinterpret_cast<const float4*>(drow + off));
            for (int k = 0; k < deg; k++)
                if (snb[r * deg + k] == v) ap = f4add(ap, *reinterpret_cast<const float4*>(drow + (k + 1) * H + off));
        }
        const long long node = g * N + v;
        if (dhf) *reinterpret_cast<float4*>(dhf + node * H + off) = af;
        if (dhp) *reinterpret_cast<float4*>(dhp + node * H + off) = ap;
    }
}

// k_readout_bwd_lds over S column chunks per graph (block = (graph, chunk)): 1/S of the LDS per
// block, so S times as many blocks stay resident. The (row, segment) -> node map is inverted once per
// block into per-node row bitmasks (LDS atomic OR: order-free; MW 64-bit words per mask, rows up to
// 64 MW: every node of a 100-node graph without agent map), so a (node, column) thread visits only the
// rows that read its node, in ascending (row, segment) order: the same summation order as
// k_readout_bwd (identical results).
template <int MW>
__global__ __launch_bounds__(256) void k_readout_bwd_cs(const float* __restrict__ dout, long long stride,
                                                        const int32_t* __restrict__ nbr,
                                                        const int32_t* __restrict__ agent_node, int N, int R, int deg,
                                                        int H, int S, float* __restrict__ dhf, float* __restrict__ dhp) {
    extern __shared__ float4 sq[];  // [R][deg + 1][C4]
    __shared__ int su[64 * MW];
    __shared__ unsigned long long smask[128][4][MW];  // node -> rows reading it, per segment (deg <= 3)
    const long long g = blockIdx.x / S;
    const int cs = blockIdx.x - (int)(g * S);
    const int C4 = (H >> 2) / S, SEG = deg + 1;
    for (int i = threadIdx.x; i < R; i += blockDim.x) su[i] = agent_node ? agent_node[g * R + i] : i;
    for (int i = threadIdx.x; i < N * SEG * MW; i += blockDim.x) smask[i / (SEG * MW)][(i / MW) % SEG][i % MW] = 0ull;
    for (int i = threadIdx.x; i < R * SEG * C4; i += blockDim.x) {
        const int r = i / (SEG * C4), rem = i - r * SEG * C4, sg = rem / C4, c = rem - sg * C4;
        sq[i] = *reinterpret_cast<const float4*>(dout + (g * R + r) * stride + sg * H + (cs * C4 + c) * 4);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < R * SEG; e += blockDim.x) {
        const int r = e / SEG, sg = e - r * SEG;
        const int v = sg == 0 ? su[r] : nbr[(g * N + su[r]) * deg + sg - 1];
        if (v >= 0 && v < N) atomicOr(&smask[v][sg][r >> 6], 1ull << (r & 63));
    }
    __syncthreads();
    for (int t = threadIdx.x; t < N * C4; t += blockDim.x) {
        const int v = t / C4, c = t - v * C4;
        float4 af = make_float4(0.f, 0.f, 0.f, 0.f), ap = af;
#pragma unroll
        for (int w = 0; w < MW; w++)
            for (unsigned long long m = smask[v][0][w]; m; m &= m - 1)
                af = f4add(af, sq[(64 * w + __ffsll(m) - 1) * SEG * C4 + c]);
#pragma unroll
        for (int w = 0; w < MW; w++) {
            unsigned long long mk[3], any = 0ull;
            for (int k = 0; k < deg; k++) any |= (mk[k] = smask[v][k + 1][w]);
            for (; any; any &= any - 1) {
                const int rb = __ffsll(any) - 1, r = 64 * w + rb;
                for (int k = 0; k < deg; k++)
                    if ((mk[k] >> rb) & 1ull) ap = f4add(ap, sq[(r * SEG + k + 1) * C4 + c]);
            }
        }
        const long long o = (g * N + v) * H + (cs * C4 + c) * 4;
        if (dhf) *reinterpret_cast<float4*>(dhf + o) = af;
        if (dhp) *reinterpret_cast<float4*>(dhp + o) = ap;
    }
}

// Readout backward without an agent map (every node reads itself out: config 5's all-nodes readout,
// src/sl.py:132-168): row v of dout is [dh_final(v) | dh_prev(nbr(v, 0)) | ... ], so dhf(u) is row u's
// segment 0 and dhp(u) = sum over the neighbours v of u, ascending, of row v's segment 1 + (slot of u in v's
// ascending list) (symmetric adjacency: u is in v's list once). A gather per (node, 16-B chunk) instead of the
// per-graph LDS staging of k_readout_bwd_cs; the same ascending-row order, so the same fp32 sums
template <typename I>
__global__ __launch_bounds__(256) void k_readout_bwd_nodes(const float* __restrict__ dout, long long stride,
                                                           const int32_t* __restrict__ nbr, long long nodes, int N,
                                                           int deg, int H, float* __restrict__ dhf,
                                                           float* __restrict__ dhp) {
    // I: the index type of the (node, chunk) decomposition, 32-bit when nodes * H / 4 fits (no 64-bit division)
    const I C4 = (I)(H >> 2);
    const I t = (I)blockIdx.x * (I)blockDim.x + (I)threadIdx.x;
    if ((long long)t >= nodes * C4) return;
    const I u = t / C4;
    const int c = (int)(t - u * C4);
    const I g0 = (u / (I)N) * (I)N;
    const int ul = (int)(u - g0);
    const long long U = (long long)u, G0 = (long long)g0;
    if (dhf) *reinterpret_cast<float4*>(dhf + U * H + 4 * c) = *reinterpret_cast<const float4*>(dout + U * stride + 4 * c);
    if (!dhp) return;
    // all neighbour ids, then all their lists, then all gradient loads in flight together; summed in ascending k
    // as before (the same fp32 sums)
    int v[MAXDEG], slot[MAXDEG];
#pragma unroll
    for (int k = 0; k < MAXDEG; k++) v[k] = k < deg ? nbr[U * deg + k] : -1;
#pragma unroll
    for (int k = 0; k < MAXDEG; k++) {
        slot[k] = -1;
        if (v[k] >= 0 && v[k] < N)
            for (int j = 0; j < deg; j++)
                if (nbr[(G0 + v[k]) * deg + j] == ul) slot[k] = j;
    }
    float4 x[MAXDEG];
#pragma unroll
    for (int k = 0; k < MAXDEG; k++)
        x[k] = slot[k] >= 0 ? *reinterpret_cast<const float4*>(dout + (G0 + v[k]) * stride + (1 + slot[k]) * H + 4 * c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 ap = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < MAXDEG; k++)
        if (slot[k] >= 0) ap = f4add(ap, x[k]);
    *reinterpret_cast<float4*>(dhp + U * H + 4 * c) = ap;
}

extern "C" int gm_netmon_readout_ld(const float* hf, int64_t ldf, const float* hp, int64_t ldp, const int32_t* nbr,
                                    const int32_t* agent_node, int32_t G, int32_t N, int32_t R, int32_t deg, int32_t H,
                                    float* out, int64_t stride, void* stream) {
    if (!hf || !hp || !nbr || !out || G <= 0 || N <= 0 || R <= 0 || deg < 0 || H <= 0 ||
        stride < (int64_t)(deg + 1) * H || ldf < H || ldp < H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout: bad arguments");
    if (!agent_node && R != N) return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout: R must equal N without agent map");
    int V = vec_width(H, stride, out);
    int v2 = vec_width(H, ldf, hf), v3 = vec_width(H, ldp, hp);
    V = V < v2 ? V : v2;
    V = V < v3 ? V : v3;
    if (V == 4) {
        const long long rows = (long long)G * R;
        const long long blocks = std::min<long long>((rows + 3) / 4, 65536);
        hipLaunchKernelGGL(k_readout_rows, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, hf, hp, nbr,
                           agent_node, rows, N, R, deg, H, out, (long long)stride, (long long)ldf, (long long)ldp);
        return launched();
    }
    long long total = (long long)G * R * (deg + 1) * (H / V);
    GM_VLAUNCH(k_readout, V, dim3(nblocks(total, 256)), hf, hp, nbr, agent_node, G, N, R, deg, H, out,
               (long long)stride, (long long)ldf, (long long)ldp);
    return launched();
}

extern "C" int gm_netmon_readout(const float* hf, const float* hp, const int32_t* nbr, const int32_t* agent_node,
                                 int32_t G, int32_t N, int32_t R, int32_t deg, int32_t H, float* out, int64_t stride,
                                 void* stream) {
    return gm_netmon_readout_ld(hf, H, hp, H, nbr, agent_node, G, N, R, deg, H, out, stride, stream);
}

// Same gather, one block per graph: the graph's agent nodes and their neighbour lists are
// staged in LDS once (the per-thread version re-read them from L1/L2 for every node and column
// chunk), then every (node, column chunk) thread sums its contributions in the same (agent,
// segment) order as k_readout_bwd, so the results are identical.
template <int V>
__global__ __launch_bounds__(1024) void k_readout_bwd_g(const float* __restrict__ dout, long long stride,
                                                        const int32_t* __restrict__ nbr,
                                                        const int32_t* __restrict__ agent_node, int N, int R, int deg,
                                                        int H, float* __restrict__ dhf, float* __restrict__ dhp) {
    __shared__ int su[64];
    __shared__ int snb[64 * MAXDEG];
    const long long g = blockIdx.x;
    for (int i = threadIdx.x; i < R; i += blockDim.x) su[i] = agent_node ? agent_node[g * R + i] : i;
    __syncthreads();
    for (int i = threadIdx.x; i < R * deg; i += blockDim.x) {
        const int r = i / deg, k = i - r * deg;
        snb[i] = nbr[(g * N + su[r]) * deg + k];
    }
    __syncthreads();
    const int HV = H / V;
    if ((int)threadIdx.x >= N * HV) return;
    const int v = threadIdx.x / HV, off = (threadIdx.x % HV) * V;
    Vec<V> af = zerov<V>(), ap = zerov<V>();
    for (int r = 0; r < R; r++) {
        const float* drow = dout + (g * R + r) * stride;
        if (su[r] == v) {
            Vec<V> x = ldv<V>(drow + off);
#pragma unroll
            for (int i = 0; i < V; i++) af.v[i] += x.v[i];
        }
        for (int k = 0; k < deg; k++) {
            if (snb[r * deg + k] == v) {
                Vec<V> x = ldv<V>(drow + (size_t)(k + 1) * H + off);
#pragma unroll
                for (int i = 0; i < V; i++) ap.v[i] += x.v[i];
            }
        }
    }
    const long long node = g * N + v;
    if (dhf) stv<V>(dhf + node * H + off, af);
    if (dhp) stv<V>(dhp + node * H + off, ap);
}

extern "C" int gm_netmon_readout_bwd(const float* dout, int64_t stride, const int32_t* nbr, const int32_t* agent_node,
                                     int32_t G, int32_t N, int32_t R, int32_t deg, int32_t H, float* dhf, float* dhp,
                                     void* stream) {
    if (!dout || !nbr || G <= 0 || N <= 0 || R <= 0 || deg < 0 || H <= 0)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout_bwd: bad arguments");
    int V = vec_width(H, stride, dout);
    if (dhf) { int v = vec_width(H, H, dhf); V = V < v ? V : v; }
    if (dhp) { int v = vec_width(H, H, dhp); V = V < v ? V : v; }
    if (!agent_node && R == N && V == 4 && deg <= MAXDEG) {  // every node read out: a gather per node
        const long long total = (long long)G * N * (H / 4);
        if (total + 256 < (1ll << 31))
            hipLaunchKernelGGL(k_readout_bwd_nodes<unsigned>, dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, dout, (long long)stride, nbr, (long long)G * N, N, deg, H, dhf, dhp);
        else
            hipLaunchKernelGGL(k_readout_bwd_nodes<long long>, dim3(nblocks(total, 256)), dim3(256), 0,
                               (hipStream_t)stream, dout, (long long)stride, nbr, (long long)G * N, N, deg, H, dhf, dhp);
        return launched();
    }
    const size_t lds = (size_t)R * (deg + 1) * H * 4;
    // column chunks per graph: 4, or 8 when a quarter of the graph's rows exceeds 48 KB of LDS
    const int S = (lds / 4 <= 48 * 1024 || (H / 4) % 8) ? 4 : 8;
    if (V == 4 && R <= 128 && N <= 128 && deg <= 3 && (H / 4) % S == 0 && lds / S <= 48 * 1024) {
        const int threads = std::min(256, (N * (H / (4 * S)) + 63) / 64 * 64);
        if (R <= 64)
            hipLaunchKernelGGL(k_readout_bwd_cs<1>, dim3((unsigned)((long long)G * S)), dim3(threads), lds / S,
                               (hipStream_t)stream, dout, (long long)stride, nbr, agent_node, N, R, deg, H, S, dhf, dhp);
        else  // up to 128 rows per graph (e.g. every node of a 100-node graph, no agent map)
            hipLaunchKernelGGL(k_readout_bwd_cs<2>, dim3((unsigned)((long long)G * S)), dim3(threads), lds / S,
                               (hipStream_t)stream, dout, (long long)stride, nbr, agent_node, N, R, deg, H, S, dhf, dhp);
        return launched();
    }
    if (V == 4 && R <= 64 && deg <= MAXDEG && lds <= 48 * 1024) {
        const int threads = std::min(1024, (N * (H / 4) + 63) / 64 * 64);
        hipLaunchKernelGGL(k_readout_bwd_lds, dim3(G), dim3(threads), lds, (hipStream_t)stream, dout, (long long)stride,
                           nbr, agent_node, N, R, deg, H, dhf, dhp);
        return launched();
    }
    if (R <= 64 && deg <= MAXDEG && N * (H / V) <= 1024) {
        const int threads = (N * (H / V) + 63) / 64 * 64;
        hipStream_t st = (hipStream_t)stream;
        if (V == 4)
            hipLaunchKernelGGL(k_readout_bwd_g<4>, dim3(G), dim3(threads), 0, st, dout, (long long)stride, nbr,
                               agent_node, N, R, deg, H, dhf, dhp);
        else if (V == 2)
            hipLaunchKernelGGL(k_readout_bwd_g<2>, dim3(G), dim3(threads), 0, st, dout, (long long)stride, nbr,
                               agent_node, N, R, deg, H, dhf, dhp);
        else
            hipLaunchKernelGGL(k_readout_bwd_g<1>, dim3(G), dim3(threads), 0, st, dout, (long long)stride, nbr,
                               agent_node, N, R, deg, H, dhf, dhp);
        return launched();
    }
    long long total = (long long)G * N * (H / V);
    GM_VLAUNCH(k_readout_bwd, V, dim3(nblocks(total, 256)), dout, (long long)stride, nbr, agent_node, G, N, R, deg, H,
               dhf, dhp);
    return launched();
}

extern "C" int gm_lstm_pointwise(const float* gates, const float* c, int32_t m, int32_t H, float* h1, float* c1,
                                 float* act, void* stream) {
    if (!gates || !c || !h1 || !c1 || m <= 0 || H <= 0) return gm_fail(GM_ERR_INVALID_ARG, "gm_lstm_pointwise: bad args");
    long long total = (long long)m * H;
    hipLaunchKernelGGL(k_lstm_pw, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, gates, c, m, H, h1, c1,
                       act);
    return launched();
}

extern "C" int gm_lstm_pointwise_bwd(const float* dh1, const float* dc1, const float* act, const float* c,
                                     const float* c1, int32_t m, int32_t H, float* dgates, float* dc,
                                     float* dgates_scale, void* stream) {
    if (!act || !c || !c1 || !dgates || !dc || m <= 0 || H <= 0)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_lstm_pointwise_bwd: bad args");
    hipStream_t st = (hipStream_t)stream;
    if (dgates_scale && hipMemsetAsync(dgates_scale, 0, sizeof(float), st) != hipSuccess)
        return gm_fail(GM_ERR_HIP, "gm_lstm_pointwise_bwd: memset");
    long long total = (long long)m * H;
    // grid-stride over at most 4096 blocks: one published max per block
    const long long nb = std::min<long long>(nblocks(total, 256), 4096);
    hipLaunchKernelGGL(k_lstm_pw_bwd, dim3((unsigned)nb), dim3(256), 0, st, dh1, dc1, act, c, c1, m, H, dgates, dc,
                       reinterpret_cast<unsigned*>(dgates_scale));
    int rc = launched();
    if (rc == GM_OK && dgates_scale) rc = gm_absmax_finish(dgates_scale, stream);
    return rc;
}

// ---------------------------------------------------------------------------
// Sequence-batched training backward (graph-marl_amd/train_seq.py)
// ---------------------------------------------------------------------------
namespace {

// max over the block through LDS (any block size <= 1024), published once per block
__device__ void block_max_publish(float m, unsigned* slot) {
    __shared__ float red[1024];
    red[threadIdx.x] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)blockDim.x; i++) m = fmaxf(m, red[i]);
        gm_amax_publish(slot, m);
    }
}

// LSTM cell backward with its gradient sources summed on the fly (gm_lstm_cell_bwd). Thread
// (rl, u) of a block of RL x H threads owns unit u of the rows r0 + rl, r0 + rl + RL, ... of the
// block's rows_per_block rows: loads and stores are unit-contiguous; the per-block bias sums are
// the RL row lanes combined in LDS in a fixed order.
__global__ __launch_bounds__(1024) void k_lstm_cell_bwd(gm_lstm_bwd_args a, unsigned* sc_slot, unsigned* max_slot) {
    __shared__ float red[4][1024];
    const int H = a.hidden, RL = blockDim.x / H;
    const int u = threadIdx.x % H, rl = threadIdx.x / H;
    const long long r0 = (long long)blockIdx.x * a.rows_per_block;
    const long long r1 = min((long long)a.m, r0 + a.rows_per_block);
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f, mx = 0.f;
    for (long long r = r0 + rl; r < r1; r += RL) {
        const float* ar = a.act + r * a.ld_act + u;
        const float gi = ar[0], gf = ar[H], gg = ar[2 * H], go = ar[3 * H];
        const float c = a.c_in[r * a.ld_cin + u];
        const float tc = tanhf(a.c_out[r * a.ld_cout + u]);
        float dh = 0.f;
        if (a.dh0) dh += a.dh0[r * a.ld_dh0 + u];
        if (a.dh1) dh += a.dh1[r * a.ld_dh1 + u];
        if (a.dm) {  // transpose of the (I + A) aggregate: members of row r's node, ascending id
            const int N = a.n_nodes;
            const long long g = r / N;
            const int n = (int)(r - g * N);
            int mem[MAXDEG + 1];
            const int cnt = members(a.nbr + r * a.deg, a.deg, n, mem);
            for (int q = 0; q < cnt; q++) {
                float v = a.dm[(g * N + mem[q]) * a.ld_dm + u];
                if (a.mean) {
                    const int32_t* nbm = a.nbr + (g * N + mem[q]) * a.deg;
                    int cm = 1;
                    for (int k = 0; k < a.deg; k++) cm += nbm[k] >= 0;
                    v = v * (1.0f / (float)cm);
                }
                dh += v;
            }
        }
        float dcn = a.dc ? a.dc[r * a.ld_dc + u] : 0.f;
        const bool ext = !a.ext_mask || !a.ext_mask[r / a.rows_per_sample];
        if (ext) {
            if (a.dh_ext) dh += a.dh_ext[r * a.ld_ext + u];
            if (a.dc_ext) dcn += a.dc_ext[r * a.ld_dcext + u];
        }
        const float dct = dcn + dh * go * (1.f - tc * tc);
        const float d0 = dct * gg * gi * (1.f - gi), d1 = dct * c * gf * (1.f - gf);
        const float d2 = dct * gi * (1.f - gg * gg), d3 = dh * tc * go * (1.f - go);
        float* dg = a.dgates + r * a.ld_dg + u;
        dg[0] = d0;
        dg[H] = d1;
        dg[2 * H] = d2;
        dg[3 * H] = d3;
        if (a.dc_out) a.dc_out[r * a.ld_dco + u] = dct * gf;
        p0 += d0;
        p1 += d1;
        p2 += d2;
        p3 += d3;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(d0), fabsf(d1)), fmaxf(fabsf(d2), fabsf(d3))));
    }
    if (a.bias_part) {
        red[0][threadIdx.x] = p0;
        red[1][threadIdx.x] = p1;
        red[2][threadIdx.x] = p2;
        red[3][threadIdx.x] = p3;
        __syncthreads();
        if (rl == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                float s = red[k][u];
                for (int l = 1; l < RL; l++) s += red[k][l * H + u];
                a.bias_part[(long long)blockIdx.x * 4 * H + k * H + u] = s;
            }
        }
        __syncthreads();
    }
    if (sc_slot || max_slot) {
        __shared__ float mred[1024];
        mred[threadIdx.x] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < (int)blockDim.x; i++) mx = fmaxf(mx, mred[i]);
            if (sc_slot) gm_amax_publish(sc_slot, mx);
            if (max_slot) gm_amax_publish(max_slot, mx);
        }
    }
}

// k_lstm_cell_bwd with 4 consecutive units per thread (16-byte loads and stores; every ld and base
// 16-byte aligned, H % 4 == 0): thread (rl, u4) of RL x H/4 threads; per element the same arithmetic
// in the same order as k_lstm_cell_bwd. Bias partials: the RL row lanes combined in LDS in a fixed
// order; max |dgates| per wave, then over the block's waves.
__global__ __launch_bounds__(256) void k_lstm_cell_bwd4(gm_lstm_bwd_args a, unsigned* sc_slot, unsigned* max_slot) {
    __shared__ float4 red[4][256];
    __shared__ float wmx[4];
    const int H = a.hidden, H4 = H >> 2, RL = blockDim.x / H4;
    const int u = (threadIdx.x % H4) * 4, rl = threadIdx.x / H4;
    const long long r0 = (long long)blockIdx.x * a.rows_per_block;
    const long long r1 = min((long long)a.m, r0 + a.rows_per_block);
    auto ld4 = [](const float* p) { return *reinterpret_cast<const float4*>(p); };
    auto add4 = [](float4& x, float4 y) {
        x.x += y.x;
        x.y += y.y;
        x.z += y.z;
        x.w += y.w;
    };
    float4 p[4];
#pragma unroll
    for (int k = 0; k < 4; k++) p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    float mx = 0.f;
    for (long long r = r0 + rl; r < r1; r += RL) {
        const float* ar = a.act + r * a.ld_act + u;
        const float4 gi4 = ld4(ar), gf4 = ld4(ar + H), gg4 = ld4(ar + 2 * H), go4 = ld4(ar + 3 * H);
        const float4 c4 = ld4(a.c_in + r * a.ld_cin + u), co4 = ld4(a.c_out + r * a.ld_cout + u);
        float4 dh4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.dh0) add4(dh4, ld4(a.dh0 + r * a.ld_dh0 + u));
        if (a.dh1) add4(dh4, ld4(a.dh1 + r * a.ld_dh1 + u));
        if (a.dm) {
            const int N = a.n_nodes;
            const long long g = r / N;
            const int n = (int)(r - g * N);
            int mem[MAXDEG + 1];
            const int cnt = members(a.nbr + r * a.deg, a.deg, n, mem);
            for (int q = 0; q < cnt; q++) {
                float4 v = ld4(a.dm + (g * N + mem[q]) * a.ld_dm + u);
                if (a.mean) {
                    const int32_t* nbm = a.nbr + (g * N + mem[q]) * a.deg;
                    int cm = 1;
                    for (int k = 0; k < a.deg; k++) cm += nbm[k] >= 0;
                    const float f = 1.0f / (float)cm;
                    v = make_float4(v.x * f, v.y * f, v.z * f, v.w * f);
                }
                add4(dh4, v);
            }
        }
        float4 dc4 = a.dc ? ld4(a.dc + r * a.ld_dc + u) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool ext = !a.ext_mask || !a.ext_mask[r / a.rows_per_sample];
        if (ext) {
            if (a.dh_ext) add4(dh4, ld4(a.dh_ext + r * a.ld_ext + u));
            if (a.dc_ext) add4(dc4, ld4(a.dc_ext + r * a.ld_dcext + u));
        }
        const float* gi = &gi4.x;
        const float* gf = &gf4.x;
        const float* gg = &gg4.x;
        const float* go = &go4.x;
        const float* c = &c4.x;
        const float* co = &co4.x;
        const float* dh = &dh4.x;
        const float* dcn = &dc4.x;
        float4 o0, o1, o2, o3, oc;
        float* d0 = &o0.x;
        float* d1 = &o1.x;
        float* d2 = &o2.x;
        float* d3 = &o3.x;
        float* dco = &oc.x;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float tc = tanhf(co[e]);
            const float dct = dcn[e] + dh[e] * go[e] * (1.f - tc * tc);
            d0[e] = dct * gg[e] * gi[e] * (1.f - gi[e]);
            d1[e] = dct * c[e] * gf[e] * (1.f - gf[e]);
            d2[e] = dct * gi[e] * (1.f - gg[e] * gg[e]);
            d3[e] = dh[e] * tc * go[e] * (1.f - go[e]);
            dco[e] = dct * gf[e];
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(d0[e]), fabsf(d1[e])), fmaxf(fabsf(d2[e]), fabsf(d3[e]))));
        }
        float* dg = a.dgates + r * a.ld_dg + u;
        *reinterpret_cast<float4*>(dg) = o0;
        *reinterpret_cast<float4*>(dg + H) = o1;
        *reinterpret_cast<float4*>(dg + 2 * H) = o2;
        *reinterpret_cast<float4*>(dg + 3 * H) = o3;
        if (a.dc_out) *reinterpret_cast<float4*>(a.dc_out + r * a.ld_dco + u) = oc;
        add4(p[0], o0);
        add4(p[1], o1);
        add4(p[2], o2);
        add4(p[3], o3);
    }
    if (a.bias_part) {
#pragma unroll
        for (int k = 0; k < 4; k++) red[k][threadIdx.x] = p[k];
        __syncthreads();
        if (rl == 0) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                float4 s = red[k][threadIdx.x];
                for (int l = 1; l < RL; l++) add4(s, red[k][l * H4 + threadIdx.x]);
                *reinterpret_cast<float4*>(a.bias_part + (long long)blockIdx.x * 4 * H + k * H + u) = s;
            }
        }
    }
    if (sc_slot || max_slot) {
        mx = gm_wave_max(mx);
        if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < (int)(blockDim.x >> 6); w++) mx = fmaxf(mx, wmx[w]);
            if (sc_slot) gm_amax_publish(sc_slot, mx);
            if (max_slot) gm_amax_publish(max_slot, mx);
        }
    }
}

// Q head + leaky hidden layer backward (gm_qhead_bwd): thread c owns column c of the block's rows
__global__ __launch_bounds__(1024) void k_qhead_bwd(const float* __restrict__ dq, long long ldq, int nq,
                                                   const float* __restrict__ wq, long long ldwq,
                                                   const float* __restrict__ y, long long ldy, long long rows, int cols,
                                                   int act, float* __restrict__ g, long long ldg,
                                                   float* __restrict__ part_b, float* __restrict__ part_wq,
                                                   float* __restrict__ part_bq, int rpb, unsigned* __restrict__ amax) {
    const int c = threadIdx.x;
    const bool ok = c < cols;
    float w[4] = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < nq; q++) w[q] = ok ? wq[q * ldwq + c] : 0.f;
    const long long r0 = (long long)blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
    float pb = 0.f, mx = 0.f, pw[4] = {0.f, 0.f, 0.f, 0.f}, pq[4] = {0.f, 0.f, 0.f, 0.f};
    // U rows per iteration with their loads issued together (independent HBM round trips in flight)
    constexpr int U = 8;
    for (long long rb = r0; rb < r1; rb += U) {
        float d[U][4], yv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long r = min(rb + u, r1 - 1);
#pragma unroll
            for (int q = 0; q < 4; q++) d[u][q] = q < nq ? dq[r * ldq + q] : 0.f;
            yv[u] = ok ? y[r * ldy + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (rb + u >= r1) break;
            const long long r = rb + u;
#pragma unroll
            for (int q = 0; q < 4; q++) pq[q] += d[u][q];
            if (ok) {
                float gv = 0.f;
#pragma unroll
                for (int q = 0; q < 4; q++) gv = fmaf(d[u][q], w[q], gv);
                if (act) gv *= gm_act_dy(yv[u], act);
                g[r * ldg + c] = gv;
                pb += gv;
                mx = fmaxf(mx, fabsf(gv));
#pragma unroll
                for (int q = 0; q < 4; q++) pw[q] = fmaf(d[u][q], yv[u], pw[q]);
            }
        }
    }
    if (ok) {
        part_b[(long long)blockIdx.x * cols + c] = pb;
        for (int q = 0; q < nq; q++) part_wq[((long long)blockIdx.x * nq + q) * cols + c] = pw[q];
    }
    if (c == 0)
        for (int q = 0; q < nq; q++) part_bq[(long long)blockIdx.x * nq + q] = pq[q];
    if (amax) block_max_publish(mx, amax);
}

// k_qhead_bwd with 4 columns per thread (16-byte loads / stores; cols % 4 == 0, 16-byte bases and
// strides): RL row lanes x cols/4 threads, U rows per lane in flight; per element the arithmetic of
// k_qhead_bwd; the row lanes' partial sums combined in LDS in a fixed order.
__global__ __launch_bounds__(256) void k_qhead_bwd4(const float* __restrict__ dq, long long ldq, int nq,
                                                   const float* __restrict__ wq, long long ldwq,
                                                   const float* __restrict__ y, long long ldy, long long rows, int cols,
                                                   int act, float* __restrict__ g, long long ldg,
                                                   float* __restrict__ part_b, float* __restrict__ part_wq,
                                                   float* __restrict__ part_bq, int rpb, unsigned* __restrict__ amax) {
    __shared__ float4 red[5][256];
    __shared__ float rq[4][256];
    __shared__ float wmx[4];
    const int C4 = cols >> 2, RL = blockDim.x / C4;
    const int c4 = threadIdx.x % C4, rl = threadIdx.x / C4, c = 4 * c4;
    float4 w[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
        w[q] = q < nq ? *reinterpret_cast<const float4*>(wq + q * ldwq + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const long long r0 = (long long)blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
    float4 pb = make_float4(0.f, 0.f, 0.f, 0.f), pw[4];
    float pq[4] = {0.f, 0.f, 0.f, 0.f}, mx = 0.f;
#pragma unroll
    for (int q = 0; q < 4; q++) pw[q] = pb;
    constexpr int U = 4;
    for (long long rb = r0 + rl; rb < r1; rb += (long long)U * RL) {
        float d[U][4];
        float4 yv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long r = min(rb + (long long)u * RL, r1 - 1);
#pragma unroll
            for (int q = 0; q < 4; q++) d[u][q] = q < nq ? dq[r * ldq + q] : 0.f;
            yv[u] = *reinterpret_cast<const float4*>(y + r * ldy + c);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long r = rb + (long long)u * RL;
            if (r >= r1) break;
            if (c4 == 0)
#pragma unroll
                for (int q = 0; q < 4; q++) pq[q] += d[u][q];
            const float* ye = &yv[u].x;
            float4 gv4;
            float* gv = &gv4.x;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                float v = 0.f;
#pragma unroll
                for (int q = 0; q < 4; q++) v = fmaf(d[u][q], (&w[q].x)[e], v);
                if (act) v *= gm_act_dy(ye[e], act);
                gv[e] = v;
                mx = fmaxf(mx, fabsf(v));
            }
            *reinterpret_cast<float4*>(g + r * ldg + c) = gv4;
            pb.x += gv4.x;
            pb.y += gv4.y;
            pb.z += gv4.z;
            pb.w += gv4.w;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                pw[q].x = fmaf(d[u][q], ye[0], pw[q].x);
                pw[q].y = fmaf(d[u][q], ye[1], pw[q].y);
                pw[q].z = fmaf(d[u][q], ye[2], pw[q].z);
                pw[q].w = fmaf(d[u][q], ye[3], pw[q].w);
            }
        }
    }
    red[0][threadIdx.x] = pb;
#pragma unroll
    for (int q = 0; q < 4; q++) red[1 + q][threadIdx.x] = pw[q];
    if (c4 == 0)
#pragma unroll
        for (int q = 0; q < 4; q++) rq[q][rl] = pq[q];
    __syncthreads();
    if (rl == 0) {
        for (int k = 0; k <= nq; k++) {
            float4 sm = red[k][c4];
            for (int l = 1; l < RL; l++) {
                const float4 o = red[k][l * C4 + c4];
                sm.x += o.x;
                sm.y += o.y;
                sm.z += o.z;
                sm.w += o.w;
            }
            float* dst = k == 0 ? part_b + (long long)blockIdx.x * cols : part_wq + ((long long)blockIdx.x * nq + k - 1) * cols;
            *reinterpret_cast<float4*>(dst + c) = sm;
        }
        if (c4 == 0)
            for (int q = 0; q < nq; q++) {
                float sm = rq[q][0];
                for (int l = 1; l < RL; l++) sm += rq[q][l];
                part_bq[(long long)blockIdx.x * nq + q] = sm;
            }
    }
    if (amax) {
        mx = gm_wave_max(mx);
        if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < (int)(blockDim.x >> 6); k++) mx = fmaxf(mx, wmx[k]);
            gm_amax_publish(amax, mx);
        }
    }
}

}  // namespace

extern "C" int gm_lstm_cell_bwd(const gm_lstm_bwd_args* a, void* stream) {
    if (!a || !a->act || !a->c_in || !a->c_out || !a->dgates || a->m <= 0 || a->hidden <= 0 || a->hidden > 1024 ||
        (a->hidden > 256 && a->hidden % 64) || (a->dm && (!a->nbr || a->n_nodes <= 0 || a->deg < 0 || a->deg > MAXDEG)) ||
        (a->ext_mask && a->rows_per_sample <= 0) || (a->bias_part && a->rows_per_block <= 0))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_lstm_cell_bwd: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    const int H = a->hidden;
    const int RL = H >= 256 ? 1 : 256 / H;
    const int threads = H * RL;
    gm_lstm_bwd_args b = *a;
    if (b.rows_per_block <= 0) b.rows_per_block = 64;
    if (b.dg_scale && hipMemsetAsync(b.dg_scale, 0, sizeof(float), st) != hipSuccess)
        return gm_fail(GM_ERR_HIP, "gm_lstm_cell_bwd: memset");
    const long long nb = (b.m + b.rows_per_block - 1) / b.rows_per_block;
    auto a16 = [](const void* p, long long ld) { return !p || ((reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0); };
    const bool vec = H % 4 == 0 && H / 4 <= 256 && ((256 / (H / 4)) * (H / 4)) % 64 == 0 &&
                     a16(b.act, b.ld_act) && a16(b.c_in, b.ld_cin) && a16(b.c_out, b.ld_cout) &&
                     a16(b.dh0, b.ld_dh0) && a16(b.dh1, b.ld_dh1) && a16(b.dm, b.ld_dm) && a16(b.dh_ext, b.ld_ext) &&
                     a16(b.dc_ext, b.ld_dcext) && a16(b.dc, b.ld_dc) && a16(b.dgates, b.ld_dg) &&
                     a16(b.dc_out, b.ld_dco) && a16(b.bias_part, 4);
    if (vec) {
        const int rl4 = 256 / (H / 4);
        hipLaunchKernelGGL(k_lstm_cell_bwd4, dim3((unsigned)nb), dim3(rl4 * (H / 4)), 0, st, b,
                           reinterpret_cast<unsigned*>(b.dg_scale), reinterpret_cast<unsigned*>(b.dg_max));
    } else {
        hipLaunchKernelGGL(k_lstm_cell_bwd, dim3((unsigned)nb), dim3(threads), 0, st, b,
                           reinterpret_cast<unsigned*>(b.dg_scale), reinterpret_cast<unsigned*>(b.dg_max));
    }
    int rc = launched();
    if (rc == GM_OK && b.dg_scale) rc = gm_absmax_finish(b.dg_scale, stream);
    return rc;
}

extern "C" int gm_qhead_bwd(const float* dq, int64_t ldq, int32_t nq, const float* wq, int64_t ldwq, const float* y,
                            int64_t ldy, int64_t rows, int32_t cols, int32_t act, float* g, int64_t ldg, float* part_b,
                            float* part_wq, float* part_bq, int32_t rows_per_block, float* g_scale, void* stream) {
    if (!dq || !wq || !y || !g || !part_b || !part_wq || !part_bq || nq <= 0 || nq > 4 || rows <= 0 || cols <= 0 ||
        cols > 1024 || ldq < nq || ldwq < cols || ldy < cols || ldg < cols || rows_per_block <= 0)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_qhead_bwd: bad arguments (nq <= 4, cols <= 1024)");
    hipStream_t st = (hipStream_t)stream;
    if (g_scale && hipMemsetAsync(g_scale, 0, sizeof(float), st) != hipSuccess)
        return gm_fail(GM_ERR_HIP, "gm_qhead_bwd: memset");
    const long long nb = (rows + rows_per_block - 1) / rows_per_block;
    auto a16 = [](const void* p, long long ld) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0; };
    if (cols % 4 == 0 && cols <= 1024 && ((256 / (cols / 4)) * (cols / 4)) % 64 == 0 && a16(wq, ldwq) &&
        a16(y, ldy) && a16(g, ldg) && a16(part_b, cols) && a16(part_wq, cols)) {
        const int rl = 256 / (cols / 4);
        hipLaunchKernelGGL(k_qhead_bwd4, dim3((unsigned)nb), dim3(rl * (cols / 4)), 0, st, dq, (long long)ldq, nq, wq,
                           (long long)ldwq, y, (long long)ldy, (long long)rows, cols, act, g, (long long)ldg, part_b,
                           part_wq, part_bq, rows_per_block, reinterpret_cast<unsigned*>(g_scale));
        int rc = launched();
        if (rc == GM_OK && g_scale) rc = gm_absmax_finish(g_scale, stream);
        return rc;
    }
    const int threads = (cols + 63) / 64 * 64;
    hipLaunchKernelGGL(k_qhead_bwd, dim3((unsigned)nb), dim3(threads), 0, st, dq, (long long)ldq, nq, wq,
                       (long long)ldwq, y, (long long)ldy, (long long)rows, cols, act, g, (long long)ldg, part_b,
                       part_wq, part_bq, rows_per_block, reinterpret_cast<unsigned*>(g_scale));
    int rc = launched();
    if (rc == GM_OK && g_scale) rc = gm_absmax_finish(g_scale, stream);
    return rc;
}

extern "C" int gm_routing_node_encoder(const float* x, int64_t ldx, const int32_t* nbr, int32_t G, int32_t N,
                                       const float* wt, const float* b, int32_t n, int32_t act, float* y, int64_t ldy,
                                       void* stream) {
    return gm_routing_node_encoder_bits(x, ldx, nbr, G, N, wt, b, n, act, y, ldy, nullptr, 0, stream);
}

extern "C" int gm_routing_node_encoder_bits(const float* x, int64_t ldx, const int32_t* nbr, int32_t G, int32_t N,
                                            const float* wt, const float* b, int32_t n, int32_t act, float* y,
                                            int64_t ldy, uint32_t* sbits, int64_t ldsb, void* stream) {
    if (!x || !nbr || !wt || !y || G <= 0 || N < 4 || n <= 0 || (n % 64) || act < GM_ACT_NONE || act > GM_ACT_LAST ||
        ldx < 4 * N + 8 || ldy < n || (ldy % 2) || (reinterpret_cast<uintptr_t>(wt) & 15) ||
        (sbits && ldsb < n / 32))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_routing_node_encoder: bad arguments (n % 64 == 0, 16-byte W^T)");
    const int K = 4 * N + 8;
    // columns per lane: 2 while the block's W^T slice (K x 128 floats) fits 64 KB (N <= 30), else 1 (2 above
    // N = 30 with a slice of up to 160 KB at one block per CU measured within noise, round 4)
    const int cpl = (n % 128 == 0 && (size_t)K * 128 * 4 <= 65536) ? 2 : 1;
    const size_t lds = (size_t)K * 64 * cpl * 4;
    if (lds > 160 * 1024) return gm_fail(GM_ERR_UNSUPPORTED, "gm_routing_node_encoder: 4N+8 too large for the LDS slice");
    const long long M = (long long)G * N;
    // 8 waves per block share the staged W^T slice; rows per block grow with the graph size (the slice is
    // staged once for them). Round 3, interleaved rollout A/B, per-launch times at 4096 envs: N = 20 512
    // rows 54.9 vs 63.8 us (256 rows, 4 waves), N = 30 1024 rows 88.9 vs 111.7 us, N = 40 157.5 vs 170.5
    // us, N = 50 222 vs 240 us
    const int rows = (K <= 88 ? 256 : (K <= 128 ? 512 : 1024)) * (K <= 128 ? 2 : 1);
    dim3 grid((unsigned)((M + rows - 1) / rows), (unsigned)(n / (64 * cpl)));
#define GM_RENC(C, A)                                                                                               \
    do {                                                                                                            \
        if (lds > 65536)                                                                                            \
            (void)hipFuncSetAttribute((const void*)(k_routing_enc<C, A, 512>),                                      \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                        \
        hipLaunchKernelGGL((k_routing_enc<C, A, 512>), grid, dim3(512), lds, (hipStream_t)stream, x, (long long)ldx, \
                           nbr, G, N, wt, b, n, act, y, (long long)ldy, rows, reinterpret_cast<unsigned*>(sbits),    \
                           (long long)ldsb);                                                                        \
    } while (0)
    if (cpl == 2) {
        if (act == GM_ACT_LEAKY_RELU) GM_RENC(2, 1);
        else if (act == GM_ACT_NONE) GM_RENC(2, 0);
        else GM_RENC(2, -1);
    } else {
        if (act == GM_ACT_LEAKY_RELU) GM_RENC(1, 1);
        else if (act == GM_ACT_NONE) GM_RENC(1, 0);
        else GM_RENC(1, -1);
    }
#undef GM_RENC
    return launched();
}

// ---------------------------------------------------------------------------
// LayerNorm-LSTM cell after its two gate GEMMs (reference src/layernormlstm.py:24-42):
//   g  = LN_in(x W_ih^T) + LN_hid(h W_hh^T) + b_ih      (LN over the 4H gate pre-activations)
//   c' = LN_cell(sigma(f) c + sigma(i) tanh(g_c)),  h' = sigma(o) tanh(c')   (LN over H)
// One wave per row, the row's 8H raw products (gi | gh, columns in the original gate order)
// held in registers: lane l owns units u = l + 64 q (q < UPL) of all four gates, so every load
// and store is a 64-wide coalesced run and the three LayerNorm statistics are two-pass wave
// reductions over registers (mean, then the sum of squared deviations, like torch's fp32
// LayerNorm, eps 1e-5). HBM-bound: 8H floats in, c in, h' and c' out per row.
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// precise expf / tanhf (not the GEMM epilogues' 1e-6 hardware approximations): the cell LayerNorm
// divides by the spread of c, which would amplify gate errors; the kernel is HBM-bound anyway
__device__ __forceinline__ float sig_f(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return tanhf(x); }

struct LnLstmP {
    const float *gi_w, *gi_b, *gh_w, *gh_b, *bias, *lc_w, *lc_b;
};

template <int UPL>
__global__ __launch_bounds__(256) void k_lnlstm_pw(const float* __restrict__ Gi, long long ldgi,
                                                   const float* __restrict__ Gh, long long ldgh,
                                                   const float* __restrict__ c_in, long long ldc, LnLstmP p, int M,
                                                   int H, float eps, float* __restrict__ y, long long ldy,
                                                   float* __restrict__ y2, long long ldy2, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;  // wave-uniform
    const float* gi = Gi + row * ldgi;
    const float* gh = Gh + row * ldgh;
    float a[UPL][4], b[UPL][4];
    float si = 0.f, sh = 0.f;
#pragma unroll
    for (int q = 0; q < UPL; q++) {
        const int u = lane + 64 * q;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool ok = u < H;
            a[q][k] = ok ? gi[k * H + u] : 0.f;
            b[q][k] = ok ? gh[k * H + u] : 0.f;
            si += a[q][k];
            sh += b[q][k];
        }
    }
    const float inv4h = 1.0f / (float)(4 * H);
    const float mi = wsum(si) * inv4h, mh = wsum(sh) * inv4h;
    float vi = 0.f, vh = 0.f;
#pragma unroll
    for (int q = 0; q < UPL; q++)
        if (lane + 64 * q < H)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float di = a[q][k] - mi, dh = b[q][k] - mh;
                vi += di * di;
                vh += dh * dh;
            }
    const float ri = 1.0f / sqrtf(wsum(vi) * inv4h + eps), rh = 1.0f / sqrtf(wsum(vh) * inv4h + eps);
    float cp[UPL], og[UPL], sc = 0.f;
#pragma unroll
    for (int q = 0; q < UPL; q++) {
        const int u = lane + 64 * q;
        cp[q] = og[q] = 0.f;
        if (u >= H) continue;
        float g[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int col = k * H + u;
            g[k] = ((a[q][k] - mi) * ri * p.gi_w[col] + p.gi_b[col]) + ((b[q][k] - mh) * rh * p.gh_w[col] + p.gh_b[col]) +
                   p.bias[col];
        }
        cp[q] = sig_f(g[1]) * c_in[row * ldc + u] + sig_f(g[0]) * tanh_f(g[2]);
        og[q] = sig_f(g[3]);
        sc += cp[q];
    }
    const float invh = 1.0f / (float)H;
    const float mc = wsum(sc) * invh;
    float vc = 0.f;
#pragma unroll
    for (int q = 0; q < UPL; q++)
        if (lane + 64 * q < H) {
            const float d = cp[q] - mc;
            vc += d * d;
        }
    const float rc = 1.0f / sqrtf(wsum(vc) * invh + eps);
#pragma unroll
    for (int q = 0; q < UPL; q++) {
        const int u = lane + 64 * q;
        if (u >= H) continue;
        const float cn = (cp[q] - mc) * rc * p.lc_w[u] + p.lc_b[u];
        y[row * ldy + u] = og[q] * tanh_f(cn);
        y2[row * ldy2 + u] = cn;
    }
    if (stats && lane < 6) {  // the row's LayerNorm statistics for the backward pass
        const float v = lane == 0 ? mi : lane == 1 ? ri : lane == 2 ? mh : lane == 3 ? rh : lane == 4 ? mc : rc;
        stats[row * 8 + lane] = v;
    }
}

// Backward of k_lnlstm_pw (src/layernormlstm.py:24-42 differentiated by hand). One wave per row, the
// same unit ownership as the forward; the forward quantities are recomputed from the raw gate GEMM
// outputs, c and the saved statistics (no activation tensor in HBM). Per row:
//   dcy = dc1 + dh1 o (1 - tanh^2 cy), do = dh1 tanh cy
//   LN_cell^T: dn = dcy w_c, du = r_c (dn - mean dn - n_c mean(dn n_c))
//   di = du g, dg = du i, df = du c, dc = du f; gate pre-activations dG through sigma' / tanh'
//   LN_in^T / LN_hid^T: dni = dG w_i, d gi = r_i (dni - mean dni - n_i mean(dni n_i)) (same for h)
// Parameter gradients are accumulated per wave in registers and written as one partial row per wave:
// part[wave][14H] = [d w_i (4H) | d w_h (4H) | d bias (4H; also d b_i and d b_h) | d w_c (H) | d b_c (H)].
template <int UPL>
__global__ __launch_bounds__(256) void k_lnlstm_bwd(const float* __restrict__ Gi, long long ldgi,
                                                    const float* __restrict__ Gh, long long ldgh,
                                                    const float* __restrict__ c_in, long long ldc, LnLstmP p,
                                                    const float* __restrict__ stats, const float* __restrict__ dh1,
                                                    long long lddh, const float* __restrict__ dc1, long long lddc,
                                                    int M, int H, int rpw, float* __restrict__ dgi, long long lddgi,
                                                    float* __restrict__ dgh, long long lddgh, float* __restrict__ dc,
                                                    long long lddco, float* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long r0 = wave * rpw;
    if (r0 >= M) return;  // wave-uniform
    const long long r1 = r0 + rpw < M ? r0 + rpw : M;
    float pwi[UPL][4], pwh[UPL][4], pb[UPL][4], pwc[UPL], pbc[UPL];
#pragma unroll
    for (int q = 0; q < UPL; q++) {
        pwc[q] = pbc[q] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; k++) pwi[q][k] = pwh[q][k] = pb[q][k] = 0.f;
    }
    const float inv4h = 1.0f / (float)(4 * H), invh = 1.0f / (float)H;
    for (long long row = r0; row < r1; row++) {
        const float mi = stats[row * 8 + 0], ri = stats[row * 8 + 1], mh = stats[row * 8 + 2],
                    rh = stats[row * 8 + 3], mc = stats[row * 8 + 4], rc = stats[row * 8 + 5];
        const float* gi = Gi + row * ldgi;
        const float* gh = Gh + row * ldgh;
        float ni[UPL][4], nh[UPL][4], act[UPL][4], cx[UPL], nc[UPL], dcy[UPL], dO[UPL];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int q = 0; q < UPL; q++) {
            const int u = lane + 64 * q;
            cx[q] = nc[q] = dcy[q] = dO[q] = 0.f;
#pragma unroll
            for (int k = 0; k < 4; k++) ni[q][k] = nh[q][k] = act[q][k] = 0.f;
            if (u >= H) continue;
            float g[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int col = k * H + u;
                ni[q][k] = (gi[col] - mi) * ri;
                nh[q][k] = (gh[col] - mh) * rh;
                g[k] = (ni[q][k] * p.gi_w[col] + p.gi_b[col]) + (nh[q][k] * p.gh_w[col] + p.gh_b[col]) + p.bias[col];
            }
            act[q][0] = sig_f(g[0]);
            act[q][1] = sig_f(g[1]);
            act[q][2] = tanh_f(g[2]);
            act[q][3] = sig_f(g[3]);
            cx[q] = c_in[row * ldc + u];
            const float cp = act[q][1] * cx[q] + act[q][0] * act[q][2];
            nc[q] = (cp - mc) * rc;
            const float cy = nc[q] * p.lc_w[u] + p.lc_b[u];
            const float th = tanh_f(cy);
            const float gh1 = dh1 ? dh1[row * lddh + u] : 0.f;
            dcy[q] = (dc1 ? dc1[row * lddc + u] : 0.f) + gh1 * act[q][3] * (1.f - th * th);
            dO[q] = gh1 * th;
            pwc[q] += dcy[q] * nc[q];
            pbc[q] += dcy[q];
            const float dn = dcy[q] * p.lc_w[u];
            s1 += dn;
            s2 += dn * nc[q];
        }
        const float m1 = wsum(s1) * invh, m2 = wsum(s2) * invh;
        float dG[UPL][4];
        float ti1 = 0.f, ti2 = 0.f, th1 = 0.f, th2 = 0.f;
#pragma unroll
        for (int q = 0; q < UPL; q++) {
            const int u = lane + 64 * q;
#pragma unroll
            for (int k = 0; k < 4; k++) dG[q][k] = 0.f;
            if (u >= H) continue;
            const float du = rc * (dcy[q] * p.lc_w[u] - m1 - nc[q] * m2);
            const float i = act[q][0], f = act[q][1], gg = act[q][2], o = act[q][3];
            dc[row * lddco + u] = du * f;
            dG[q][0] = du * gg * i * (1.f - i);
            dG[q][1] = du * cx[q] * f * (1.f - f);
            dG[q][2] = du * i * (1.f - gg * gg);
            dG[q][3] = dO[q] * o * (1.f - o);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int col = k * H + u;
                pb[q][k] += dG[q][k];
                pwi[q][k] += dG[q][k] * ni[q][k];
                pwh[q][k] += dG[q][k] * nh[q][k];
                const float a = dG[q][k] * p.gi_w[col], b = dG[q][k] * p.gh_w[col];
                ti1 += a;
                ti2 += a * ni[q][k];
                th1 += b;
                th2 += b * nh[q][k];
            }
        }
        const float mi1 = wsum(ti1) * inv4h, mi2 = wsum(ti2) * inv4h;
        const float mh1 = wsum(th1) * inv4h, mh2 = wsum(th2) * inv4h;
#pragma unroll
        for (int q = 0; q < UPL; q++) {
            const int u = lane + 64 * q;
            if (u >= H) continue;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int col = k * H + u;
                dgi[row * lddgi + col] = ri * (dG[q][k] * p.gi_w[col] - mi1 - ni[q][k] * mi2);
                dgh[row * lddgh + col] = rh * (dG[q][k] * p.gh_w[col] - mh1 - nh[q][k] * mh2);
            }
        }
    }
    float* pr = part + wave * 14LL * H;
#pragma unroll
    for (int q = 0; q < UPL; q++) {
        const int u = lane + 64 * q;
        if (u >= H) continue;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            pr[k * H + u] = pwi[q][k];
            pr[4 * H + k * H + u] = pwh[q][k];
            pr[8 * H + k * H + u] = pb[q][k];
        }
        pr[12 * H + u] = pwc[q];
        pr[13 * H + u] = pbc[q];
    }
}

// GRU cell gate math (torch.nn.GRUCell, gate order r, z, n): gi = x W_ih^T + b_ih, gh = h W_hh^T + b_hh
// ([m][3H] each, strided), r = sigma(gi_r + gh_r), z = sigma(gi_z + gh_z), n = tanh(gi_n + r gh_n),
// h' = (1 - z) n + z h. One thread per (row, unit).
__global__ __launch_bounds__(256) void k_gru_pw(const float* __restrict__ gi, long long ldgi,
                                                const float* __restrict__ gh, long long ldgh,
                                                const float* __restrict__ h, long long ldh, int M, int H,
                                                float* __restrict__ y, long long ldy) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)M * H) return;
    const long long row = t / H;
    const int u = (int)(t - row * H);
    const float* a = gi + row * ldgi;
    const float* b = gh + row * ldgh;
    const float r = sig_f(a[u] + b[u]), z = sig_f(a[H + u] + b[H + u]);
    const float n = tanh_f(a[2 * H + u] + r * b[2 * H + u]);
    y[row * ldy + u] = (1.f - z) * n + z * h[row * ldh + u];
}

// Backward of k_gru_pw: dn = dh' (1 - z), dz = dh' (h - n), dh = dh' z; dn_pre = dn (1 - n^2);
// d gi = [dr_pre, dz_pre, dn_pre], d gh = [dr_pre, dz_pre, dn_pre r], dr_pre = dn_pre gh_n r (1 - r),
// dz_pre = dz z (1 - z).
__global__ __launch_bounds__(256) void k_gru_bwd(const float* __restrict__ gi, long long ldgi,
                                                 const float* __restrict__ gh, long long ldgh,
                                                 const float* __restrict__ h, long long ldh,
                                                 const float* __restrict__ dy, long long lddy, int M, int H,
                                                 float* __restrict__ dgi, long long lddgi, float* __restrict__ dgh,
                                                 long long lddgh, float* __restrict__ dh, long long lddh) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)M * H) return;
    const long long row = t / H;
    const int u = (int)(t - row * H);
    const float* a = gi + row * ldgi;
    const float* b = gh + row * ldgh;
    const float r = sig_f(a[u] + b[u]), z = sig_f(a[H + u] + b[H + u]);
    const float ghn = b[2 * H + u];
    const float n = tanh_f(a[2 * H + u] + r * ghn);
    const float g = dy[row * lddy + u], hv = h[row * ldh + u];
    const float dnp = g * (1.f - z) * (1.f - n * n);
    const float drp = dnp * ghn * r * (1.f - r);
    const float dzp = g * (hv - n) * z * (1.f - z);
    dgi[row * lddgi + u] = drp;
    dgi[row * lddgi + H + u] = dzp;
    dgi[row * lddgi + 2 * H + u] = dnp;
    dgh[row * lddgh + u] = drp;
    dgh[row * lddgh + H + u] = dzp;
    dgh[row * lddgh + 2 * H + u] = dnp * r;
    dh[row * lddh + u] = g * z;
}
}  // namespace

static int lnlstm_fwd(const char* name, const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* c,
                      int64_t ldc, const LnLstmP& p, int32_t m, int32_t H, float eps, float* h1, int64_t ldh, float* c1,
                      int64_t ldc1, float* stats, void* stream) {
    if (!gi || !gh || !c || !h1 || !c1 || !p.gi_w || !p.gi_b || !p.gh_w || !p.gh_b || !p.bias || !p.lc_w || !p.lc_b ||
        m <= 0 || H <= 0 || H > 512 || ldgi < 4 * (int64_t)H || ldgh < 4 * (int64_t)H || ldc < H || ldh < H || ldc1 < H)
        return gm_fail(GM_ERR_INVALID_ARG, std::string(name) + ": bad arguments (H <= 512, gate rows >= 4H)");
    const dim3 grid((m + 3) / 4), blk(256);
    hipStream_t st = (hipStream_t)stream;
#define GM_LN(U)                                                                                                    \
    hipLaunchKernelGGL(k_lnlstm_pw<U>, grid, blk, 0, st, gi, (long long)ldgi, gh, (long long)ldgh, c, (long long)ldc, \
                       p, m, H, eps, h1, (long long)ldh, c1, (long long)ldc1, stats)
    if (H <= 64)
        GM_LN(1);
    else if (H <= 128)
        GM_LN(2);
    else if (H <= 256)
        GM_LN(4);
    else
        GM_LN(8);
#undef GM_LN
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string(name) + ": " + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_lnlstm_pointwise(const float* g, int64_t ldg, const float* c, int64_t ldc, const float* ln_in_w,
                                   const float* ln_in_b, const float* ln_hid_w, const float* ln_hid_b,
                                   const float* bias, const float* ln_cell_w, const float* ln_cell_b, int32_t m,
                                   int32_t H, float eps, float* h1, int64_t ldh, float* c1, int64_t ldc1,
                                   void* stream) {
    if (!g || ldg < 8 * (int64_t)H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_lnlstm_pointwise: bad arguments (H <= 512, ldg >= 8H)");
    LnLstmP p{ln_in_w, ln_in_b, ln_hid_w, ln_hid_b, bias, ln_cell_w, ln_cell_b};
    return lnlstm_fwd("gm_lnlstm_pointwise", g, ldg, g + 4 * (int64_t)H, ldg, c, ldc, p, m, H, eps, h1, ldh, c1, ldc1,
                      nullptr, stream);
}

extern "C" int gm_lnlstm_fwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* c,
                             int64_t ldc, const float* ln_in_w, const float* ln_in_b, const float* ln_hid_w,
                             const float* ln_hid_b, const float* bias, const float* ln_cell_w, const float* ln_cell_b,
                             int32_t m, int32_t H, float eps, float* h1, int64_t ldh, float* c1, int64_t ldc1,
                             float* stats, void* stream) {
    if (!stats) return gm_fail(GM_ERR_INVALID_ARG, "gm_lnlstm_fwd: stats is required");
    LnLstmP p{ln_in_w, ln_in_b, ln_hid_w, ln_hid_b, bias, ln_cell_w, ln_cell_b};
    return lnlstm_fwd("gm_lnlstm_fwd", gi, ldgi, gh, ldgh, c, ldc, p, m, H, eps, h1, ldh, c1, ldc1, stats, stream);
}

extern "C" int gm_lnlstm_bwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* c,
                             int64_t ldc, const float* ln_in_w, const float* ln_in_b, const float* ln_hid_w,
                             const float* ln_hid_b, const float* bias, const float* ln_cell_w, const float* ln_cell_b,
                             const float* stats, const float* dh1, int64_t lddh, const float* dc1, int64_t lddc,
                             int32_t m, int32_t H, int32_t rows_per_wave, float* dgi, int64_t lddgi, float* dgh,
                             int64_t lddgh, float* dc, int64_t lddco, float* part, void* stream) {
    if (!gi || !gh || !c || !stats || !dgi || !dgh || !dc || !part || !ln_in_w || !ln_in_b || !ln_hid_w || !ln_hid_b ||
        !bias || !ln_cell_w || !ln_cell_b || (!dh1 && !dc1) || m <= 0 || H <= 0 || H > 512 || rows_per_wave <= 0 ||
        ldgi < 4 * (int64_t)H || ldgh < 4 * (int64_t)H || lddgi < 4 * (int64_t)H || lddgh < 4 * (int64_t)H ||
        ldc < H || lddco < H || (dh1 && lddh < H) || (dc1 && lddc < H))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_lnlstm_bwd: bad arguments (H <= 512, gate rows >= 4H)");
    LnLstmP p{ln_in_w, ln_in_b, ln_hid_w, ln_hid_b, bias, ln_cell_w, ln_cell_b};
    const long long waves = ((long long)m + rows_per_wave - 1) / rows_per_wave;
    const dim3 grid((unsigned)((waves + 3) / 4)), blk(256);
    hipStream_t st = (hipStream_t)stream;
#define GM_LNB(U)                                                                                                     \
    hipLaunchKernelGGL(k_lnlstm_bwd<U>, grid, blk, 0, st, gi, (long long)ldgi, gh, (long long)ldgh, c, (long long)ldc, \
                       p, stats, dh1, (long long)lddh, dc1, (long long)lddc, m, H, rows_per_wave, dgi,                 \
                       (long long)lddgi, dgh, (long long)lddgh, dc, (long long)lddco, part)
    if (H <= 64)
        GM_LNB(1);
    else if (H <= 128)
        GM_LNB(2);
    else if (H <= 256)
        GM_LNB(4);
    else
        GM_LNB(8);
#undef GM_LNB
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_lnlstm_bwd: ") + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_gru_pointwise(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* h,
                                int64_t ldh, int32_t m, int32_t H, float* h1, int64_t ldh1, void* stream) {
    if (!gi || !gh || !h || !h1 || m <= 0 || H <= 0 || ldgi < 3 * (int64_t)H || ldgh < 3 * (int64_t)H || ldh < H ||
        ldh1 < H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gru_pointwise: bad arguments (gate rows >= 3H)");
    const long long n = (long long)m * H;
    hipLaunchKernelGGL(k_gru_pw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, gi,
                       (long long)ldgi, gh, (long long)ldgh, h, (long long)ldh, m, H, h1, (long long)ldh1);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gru_pointwise: ") + hipGetErrorString(e));
    return GM_OK;
}

extern "C" int gm_gru_bwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* h, int64_t ldh,
                          const float* dh1, int64_t lddh1, int32_t m, int32_t H, float* dgi, int64_t lddgi, float* dgh,
                          int64_t lddgh, float* dh, int64_t lddh, void* stream) {
    if (!gi || !gh || !h || !dh1 || !dgi || !dgh || !dh || m <= 0 || H <= 0 || ldgi < 3 * (int64_t)H ||
        ldgh < 3 * (int64_t)H || ldh < H || lddh1 < H || lddgi < 3 * (int64_t)H || lddgh < 3 * (int64_t)H || lddh < H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gru_bwd: bad arguments (gate rows >= 3H)");
    const long long n = (long long)m * H;
    hipLaunchKernelGGL(k_gru_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, gi,
                       (long long)ldgi, gh, (long long)ldgh, h, (long long)ldh, dh1, (long long)lddh1, m, H, dgi,
                       (long long)lddgi, dgh, (long long)lddgh, dh, (long long)lddh);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gru_bwd: ") + hipGetErrorString(e));
    return GM_OK;
}

// ---- per-step mean squared error of the SL unroll (src/sl.py:396-400: mse_loss(pred_all, targets_all) after
// every unroll step, averaged over the steps) ----
// pred [L][n] (every step's prediction), tgt [n] (the same target at every step), n % 4 == 0, 16-byte
// bases. Block b owns float4 indices [b * 256 * V, (b + 1) * 256 * V) of a step; its target elements are loaded
// once and stay in registers while the block walks the L steps (the target is not re-read per step).
namespace {
constexpr int MSE_V = 4;

__global__ __launch_bounds__(256) void k_step_mse_fwd(const float4* __restrict__ pred, const float4* __restrict__ tgt,
                                                      long long n4, int L, float* __restrict__ part) {
    __shared__ float wsum[4];
    const long long base = (long long)blockIdx.x * (256 * MSE_V) + threadIdx.x;
    float4 t[MSE_V];
#pragma unroll
    for (int v = 0; v < MSE_V; v++) {
        const long long i = base + (long long)v * 256;
        t[v] = i < n4 ? tgt[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int l = 0; l < L; l++) {
        const float4* pl = pred + (long long)l * n4;
        float4 p[MSE_V];
#pragma unroll
        for (int v = 0; v < MSE_V; v++) {
            const long long i = base + (long long)v * 256;
            p[v] = i < n4 ? pl[i] : t[v];  // past the end: d = 0
        }
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < MSE_V; v++) {
            const float dx = p[v].x - t[v].x, dy = p[v].y - t[v].y, dz = p[v].z - t[v].z, dw = p[v].w - t[v].w;
            s = fmaf(dx, dx, s);
            s = fmaf(dy, dy, s);
            s = fmaf(dz, dz, s);
            s = fmaf(dw, dw, s);
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) part[(long long)l * gridDim.x + blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
        __syncthreads();
    }
}

// grad[l][i] = (pred[l][i] - tgt[i]) * (g[l] * two_over_n): torch's d * (g * (2 / n)) in fp32, element for element
__global__ __launch_bounds__(256) void k_step_mse_bwd(const float4* __restrict__ pred, const float4* __restrict__ tgt,
                                                      long long n4, int L, const float* __restrict__ g,
                                                      float two_over_n, float4* __restrict__ grad) {
    const long long base = (long long)blockIdx.x * (256 * MSE_V) + threadIdx.x;
    float4 t[MSE_V];
#pragma unroll
    for (int v = 0; v < MSE_V; v++) {
        const long long i = base + (long long)v * 256;
        t[v] = i < n4 ? tgt[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int l = 0; l < L; l++) {
        const float s = g[l] * two_over_n;
        const float4* pl = pred + (long long)l * n4;
        float4* gl = grad + (long long)l * n4;
        float4 p[MSE_V];
#pragma unroll
        for (int v = 0; v < MSE_V; v++) {
            const long long i = base + (long long)v * 256;
            p[v] = i < n4 ? pl[i] : t[v];
        }
#pragma unroll
        for (int v = 0; v < MSE_V; v++) {
            const long long i = base + (long long)v * 256;
            if (i < n4)
                gl[i] = make_float4((p[v].x - t[v].x) * s, (p[v].y - t[v].y) * s, (p[v].z - t[v].z) * s,
                                    (p[v].w - t[v].w) * s);
        }
    }
}

bool mse_args_ok(const float* pred, const float* tgt, int64_t n, int32_t L) {
    auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return pred && tgt && n > 0 && n % 4 == 0 && L > 0 && a16(pred) && a16(tgt) && n / 4 <= (1ll << 40);
}
}  // namespace

extern "C" int32_t gm_step_mse_blocks(int64_t n) {
    return n > 0 ? (int32_t)((n / 4 + 256 * MSE_V - 1) / (256 * MSE_V)) : 0;
}

extern "C" int gm_step_mse(const float* pred, const float* tgt, int64_t n, int32_t L, float* part, void* stream) {
    if (!mse_args_ok(pred, tgt, n, L) || !part)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_step_mse: bad arguments (n % 4 == 0, 16-byte pred / tgt)");
    const int nb = gm_step_mse_blocks(n);
    hipLaunchKernelGGL(k_step_mse_fwd, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(pred), reinterpret_cast<const float4*>(tgt), (long long)(n / 4),
                       L, part);
    return launched();
}

extern "C" int gm_step_mse_bwd(const float* pred, const float* tgt, int64_t n, int32_t L, const float* g,
                               float two_over_n, float* grad, void* stream) {
    if (!mse_args_ok(pred, tgt, n, L) || !g || !grad || (reinterpret_cast<uintptr_t>(grad) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_step_mse_bwd: bad arguments (n % 4 == 0, 16-byte pred / tgt / grad)");
    const int nb = gm_step_mse_blocks(n);
    hipLaunchKernelGGL(k_step_mse_bwd, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(pred), reinterpret_cast<const float4*>(tgt), (long long)(n / 4),
                       L, g, two_over_n, reinterpret_cast<float4*>(grad));
    return launched();
}
