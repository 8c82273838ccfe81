// gm_netmon.hip — NetMon message passing (reference src/model.py:206-229,
// 476-631) as HBM-bound HIP kernels for gfx950.
//
// Graph layout: node rows h[G*N][H] (fp32, row-major, H % 4 == 0), neighbour
// table nbr[G][N][deg] (ELL, ascending ids, -1 = none). The reference multiplies a
// dense (I+A) mask with h (bmm); with deg 3 that reads 4 rows per output row, so
// the aggregate is a gather of 4 contiguous 512-byte rows per node with float4
// lanes: 32 lanes per row, a wave covers 2 rows, consecutive rows share the same
// graph's 10 KB working set in L2.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/graph_marl_amd.h"

int gm_fail(int code, const std::string& msg);

namespace {

constexpr int MAXDEG = 8;

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4scale(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }

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

// forward: out[n] = Σ_{m ∈ {n} ∪ nbr(n)} h[m]  (/ count for mean)
// backward (symmetric adjacency): dh[j] = Σ_{n ∈ {j} ∪ nbr(j)} dout[n] * scale(n)
template <bool BWD>
__global__ __launch_bounds__(256) void k_mp_aggregate(const float* __restrict__ h, const int32_t* __restrict__ nbr,
                                                      int G, int N, int deg, int H, int mode, float* __restrict__ out) {
    const int H4 = H >> 2;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)G * N * H4;
    if (gid >= total) return;
    const int c4 = (int)(gid % H4);
    const long long row = gid / H4;
    const int g = (int)(row / N), n = (int)(row % N);
    const int32_t* nb = nbr + ((size_t)g * N + n) * deg;
    int mem[MAXDEG + 1];
    const int cnt = members(nb, deg, n, mem);
    const float4* src = reinterpret_cast<const float4*>(h) + (size_t)g * N * H4 + c4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < cnt; q++) {
        float4 v = src[(size_t)mem[q] * H4];
        if (BWD && mode == 1) {
            const int32_t* nbm = nbr + ((size_t)g * N + mem[q]) * deg;
            int cm = 1;
            for (int k = 0; k < deg; k++) cm += nbm[k] >= 0;
            v = f4scale(v, 1.0f / (float)cm);
        }
        acc = q == 0 ? v : f4add(acc, v);
    }
    if (!BWD && mode == 1) acc = make_float4(acc.x / cnt, acc.y / cnt, acc.z / cnt, acc.w / cnt);
    reinterpret_cast<float4*>(out)[row * H4 + c4] = acc;
}

// readout: out row r of graph g = [h_final[v], h_prev[nbr(v,0..deg-1)]], v = agent_node or r.
// Output rows may sit inside a wider joint observation (stride, 8-byte aligned) so
// stores are float2.
__global__ __launch_bounds__(256) void k_readout(const float* __restrict__ hf, const float* __restrict__ hp,
                                                 const int32_t* __restrict__ nbr, const int32_t* __restrict__ agent_node,
                                                 int G, int N, int R, int deg, int H, float* __restrict__ out,
                                                 long long stride) {
    const int H2 = H >> 1;
    const int W2 = (deg + 1) * H2;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)G * R * W2;
    if (gid >= total) return;
    const int c2 = (int)(gid % W2);
    const long long row = gid / W2;
    const int g = (int)(row / R), r = (int)(row % R);
    const int v = agent_node ? agent_node[(size_t)g * R + r] : r;
    const int seg = c2 / H2, off = c2 - seg * H2;
    float2 val;
    if (seg == 0) {
        val = reinterpret_cast<const float2*>(hf)[((size_t)g * N + v) * H2 + off];
    } else {
        int m = nbr[((size_t)g * N + v) * deg + seg - 1];
        val = m >= 0 ? reinterpret_cast<const float2*>(hp)[((size_t)g * N + m) * H2 + off] : make_float2(0.f, 0.f);
    }
    *reinterpret_cast<float2*>(out + row * stride + 2 * c2) = val;
}

// readout backward, deterministic (no atomics): node v of graph g gathers the
// gradient of every row that read it, rows in ascending order.
__global__ __launch_bounds__(256) void k_readout_bwd(const float* __restrict__ dout, long long stride,
                                                     const int32_t* __restrict__ nbr,
                                                     const int32_t* __restrict__ agent_node, int G, int N, int R,
                                                     int deg, int H, float* __restrict__ dhf, float* __restrict__ dhp) {
    const int H2 = H >> 1;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)G * N * H2;
    if (gid >= total) return;
    const int off = (int)(gid % H2);
    const long long node = gid / H2;
    const int g = (int)(node / N), v = (int)(node % N);
    float2 af = make_float2(0.f, 0.f), ap = make_float2(0.f, 0.f);
    for (int r = 0; r < R; r++) {
        const int u = agent_node ? agent_node[(size_t)g * R + r] : r;
        const float* drow = dout + ((size_t)g * R + r) * stride;
        if (u == v) {
            float2 x = *reinterpret_cast<const float2*>(drow + 2 * off);
            af.x += x.x;
            af.y += x.y;
        }
        const int32_t* nb = nbr + ((size_t)g * N + u) * deg;
        for (int k = 0; k < deg; k++) {
            if (nb[k] == v) {
                float2 x = *reinterpret_cast<const float2*>(drow + (size_t)(k + 1) * H + 2 * off);
                ap.x += x.x;
                ap.y += x.y;
            }
        }
    }
    if (dhf) reinterpret_cast<float2*>(dhf)[node * H2 + off] = af;
    if (dhp) reinterpret_cast<float2*>(dhp)[node * H2 + off] = ap;
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
                                                     float* __restrict__ dgates, float* __restrict__ dc) {
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)M * H) return;
    const long long m = gid / H;
    const int j = (int)(gid % H);
    const float* a = act + m * 4 * H;
    float i = a[j], f = a[H + j], gg = a[2 * H + j], o = a[3 * H + j];
    float tc = tanhf(c1[gid]);
    float dh = dh1 ? dh1[gid] : 0.f;
    float dct = (dc1 ? dc1[gid] : 0.f) + dh * o * (1.f - tc * tc);
    float* dg = dgates + m * 4 * H;
    dg[j] = dct * gg * i * (1.f - i);
    dg[H + j] = dct * c[gid] * f * (1.f - f);
    dg[2 * H + j] = dct * i * (1.f - gg * gg);
    dg[3 * H + j] = dh * tc * o * (1.f - o);
    dc[gid] = dct * f;
}

inline unsigned nblocks(long long total, int bs) { return (unsigned)((total + bs - 1) / bs); }

int launched() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return GM_OK;
}

}  // namespace

extern "C" int gm_mp_aggregate(const float* h, const int32_t* nbr, int32_t G, int32_t N, int32_t deg, int32_t H,
                               int32_t mode, float* out, void* stream) {
    if (!h || !nbr || !out || G <= 0 || N <= 0 || deg < 0 || deg > MAXDEG || H <= 0 || (H & 3) || mode < 0 || mode > 1)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_mp_aggregate: bad arguments (H % 4 == 0, deg <= 8)");
    long long total = (long long)G * N * (H / 4);
    hipLaunchKernelGGL(k_mp_aggregate<false>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, h, nbr, G,
                       N, deg, H, mode, out);
    return launched();
}

extern "C" int gm_mp_aggregate_bwd(const float* dout, const int32_t* nbr, int32_t G, int32_t N, int32_t deg,
                                   int32_t H, int32_t mode, float* dh, void* stream) {
    if (!dout || !nbr || !dh || G <= 0 || N <= 0 || deg < 0 || deg > MAXDEG || H <= 0 || (H & 3) || mode < 0 ||
        mode > 1)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_mp_aggregate_bwd: bad arguments");
    long long total = (long long)G * N * (H / 4);
    hipLaunchKernelGGL(k_mp_aggregate<true>, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, dout, nbr, G,
                       N, deg, H, mode, dh);
    return launched();
}

extern "C" int gm_netmon_readout(const float* hf, const float* hp, const int32_t* nbr, const int32_t* agent_node,
                                 int32_t G, int32_t N, int32_t R, int32_t deg, int32_t H, float* out, int64_t stride,
                                 void* stream) {
    if (!hf || !hp || !nbr || !out || G <= 0 || N <= 0 || R <= 0 || deg < 0 || H <= 0 || (H & 1) || (stride & 1) ||
        (reinterpret_cast<uintptr_t>(out) & 7) || stride < (int64_t)(deg + 1) * H)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout: bad arguments (even H/stride, 8-byte aligned out)");
    if (!agent_node && R != N) return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout: R must equal N without agent map");
    long long total = (long long)G * R * (deg + 1) * (H / 2);
    hipLaunchKernelGGL(k_readout, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, hf, hp, nbr, agent_node,
                       G, N, R, deg, H, out, (long long)stride);
    return launched();
}

extern "C" int gm_netmon_readout_bwd(const float* dout, int64_t stride, const int32_t* nbr, const int32_t* agent_node,
                                     int32_t G, int32_t N, int32_t R, int32_t deg, int32_t H, float* dhf, float* dhp,
                                     void* stream) {
    if (!dout || !nbr || G <= 0 || N <= 0 || R <= 0 || deg < 0 || H <= 0 || (H & 1) || (stride & 1))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_netmon_readout_bwd: bad arguments");
    long long total = (long long)G * N * (H / 2);
    hipLaunchKernelGGL(k_readout_bwd, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, dout,
                       (long long)stride, nbr, agent_node, G, N, R, deg, H, dhf, dhp);
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
                                     const float* c1, int32_t m, int32_t H, float* dgates, float* dc, void* stream) {
    if (!act || !c || !c1 || !dgates || !dc || m <= 0 || H <= 0)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_lstm_pointwise_bwd: bad args");
    long long total = (long long)m * H;
    hipLaunchKernelGGL(k_lstm_pw_bwd, dim3(nblocks(total, 256)), dim3(256), 0, (hipStream_t)stream, dh1, dc1, act, c,
                       c1, m, H, dgates, dc);
    return launched();
}
