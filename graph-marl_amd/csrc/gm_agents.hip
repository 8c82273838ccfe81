// gm_agents.hip — agent-communication ops of the DGN and CommNet agent models
// (reference src/model.py:45-117 AttModel, 747-794 CommNet) for the batched envs.
//
// Both are per-env A x A contractions with A <= 64 agents: far too small for MFMA tiles,
// so one workgroup per env stages the env's key/value (or hidden) rows in LDS and each
// thread owns (agent, head) or (agent, column) outputs. The projections around them
// (q/k/v, fc_out, LSTM) run on the GEMM kernels.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/graph_marl_amd.h"

int gm_fail(int code, const std::string& msg);

namespace {

constexpr int MAXA = 64;
constexpr int MAXD = 64;  // per-head key / value width

// AttModel core for one env per block: for agent i and head h,
//   w_ij = <q_i, k_j> / sqrt(dk)          (att_weights, returned before masking)
//   p_ij = softmax_j(adj_ij ? w_ij : -1e9)
//   out_i = sum_j p_ij v_j + v_i          (skip connection), heads concatenated
// q/k/v rows: [B*A][ld], head h at columns [h*d, (h+1)*d) of each.
// D > 0: dk == dv == D at compile time (the reference's 16: registers, unrolled);
// D == 0: runtime widths up to MAXD.
template <int D>
__global__ void k_agent_attention(const float* __restrict__ q, const float* __restrict__ k,
                                  const float* __restrict__ v, long long ld, const int8_t* __restrict__ adj, int A,
                                  int heads, int dk_, int dv_, float scale, float* __restrict__ out, long long ldo,
                                  float* __restrict__ wout) {
    constexpr int RD = D > 0 ? D : MAXD;
    const int dk = D > 0 ? D : dk_, dv = D > 0 ? D : dv_;
    extern __shared__ float sm[];
    const int b = blockIdx.x;
    float* ks = sm;                    // [A][heads*dk]
    float* vs = sm + A * heads * dk;   // [A][heads*dv]
    const int KD = heads * dk, VD = heads * dv;
    for (int idx = threadIdx.x; idx < A * KD; idx += blockDim.x) {
        const int j = idx / KD, c = idx - j * KD;
        ks[idx] = k[((long long)b * A + j) * ld + c];
    }
    for (int idx = threadIdx.x; idx < A * VD; idx += blockDim.x) {
        const int j = idx / VD, c = idx - j * VD;
        vs[idx] = v[((long long)b * A + j) * ld + c];
    }
    __syncthreads();
    const int8_t* ad = adj + (long long)b * A * A;
    for (int p = threadIdx.x; p < A * heads; p += blockDim.x) {
        const int i = p / heads, h = p - i * heads;
        float qi[RD];
        const float* qr = q + ((long long)b * A + i) * ld + h * dk;
#pragma unroll
        for (int d = 0; d < RD; d++)
            if (d < dk) qi[d] = qr[d];
        float mx = -INFINITY;
        for (int j = 0; j < A; j++) {
            const float* kj = ks + j * KD + h * dk;
            float s = 0.f;
#pragma unroll
            for (int d = 0; d < RD; d++)
                if (d < dk) s = fmaf(qi[d], kj[d], s);
            s *= scale;
            if (wout) wout[(((long long)b * heads + h) * A + i) * A + j] = s;
            mx = fmaxf(mx, ad[i * A + j] ? s : -1e9f);
        }
        float acc[RD];
#pragma unroll
        for (int d = 0; d < RD; d++) acc[d] = 0.f;
        float sum = 0.f;
        for (int j = 0; j < A; j++) {
            const float* kj = ks + j * KD + h * dk;
            float s = 0.f;
#pragma unroll
            for (int d = 0; d < RD; d++)
                if (d < dk) s = fmaf(qi[d], kj[d], s);
            s *= scale;
            const float e = expf((ad[i * A + j] ? s : -1e9f) - mx);
            sum += e;
            const float* vj = vs + j * VD + h * dv;
#pragma unroll
            for (int d = 0; d < RD; d++)
                if (d < dv) acc[d] = fmaf(e, vj[d], acc[d]);
        }
        const float inv = 1.0f / sum;
        const float* vi = vs + i * VD + h * dv;
        float* o = out + ((long long)b * A + i) * ldo + h * dv;
#pragma unroll
        for (int d = 0; d < RD; d++)
            if (d < dv) o[d] = acc[d] * inv + vi[d];
    }
}

// CommNet communication step for one env per block: out_i = h_i + mean_{j != i, adj_ij} h_j
// (count clamped to 1), src/model.py:780-787.
__global__ void k_agent_comm(const float* __restrict__ h, long long ldh, const int8_t* __restrict__ adj, int A, int H,
                             float* __restrict__ out, long long ldo) {
    __shared__ float inv[MAXA];
    const int b = blockIdx.x;
    const int8_t* ad = adj + (long long)b * A * A;
    for (int i = threadIdx.x; i < A; i += blockDim.x) {
        int cnt = 0;
        for (int j = 0; j < A; j++) cnt += (j != i && ad[i * A + j]) ? 1 : 0;
        inv[i] = 1.0f / (float)max(cnt, 1);
    }
    __syncthreads();
    const float* hb = h + (long long)b * A * ldh;
    for (int idx = threadIdx.x; idx < A * H; idx += blockDim.x) {
        const int i = idx / H, c = idx - i * H;
        float s = 0.f;
        for (int j = 0; j < A; j++)
            if (j != i && ad[i * A + j]) s += hb[(long long)j * ldh + c];
        out[((long long)b * A + i) * ldo + c] = hb[(long long)i * ldh + c] + s * inv[i];
    }
}

int launched(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return GM_OK;
}

}  // namespace

extern "C" int gm_agent_attention(const float* q, const float* k, const float* v, int64_t ld, const int8_t* adj,
                                  int32_t B, int32_t A, int32_t heads, int32_t dk, int32_t dv, float* out,
                                  int64_t ldo, float* att_weights, void* stream) {
    if (!q || !k || !v || !adj || !out || B <= 0 || A <= 0 || A > MAXA || heads <= 0 || dk <= 0 || dk > MAXD ||
        dv <= 0 || dv > MAXD || ld < (int64_t)heads * (dk > dv ? dk : dv) || ldo < (int64_t)heads * dv)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_agent_attention: bad arguments (A <= 64, dk, dv <= 64)");
    const size_t lds = (size_t)A * heads * (dk + dv) * sizeof(float);
    if (lds > 160 * 1024) return gm_fail(GM_ERR_UNSUPPORTED, "gm_agent_attention: A * heads * (dk + dv) too large");
    const float scale = 1.0f / sqrtf((float)dk);
    if (dk == 16 && dv == 16)
        hipLaunchKernelGGL(k_agent_attention<16>, dim3(B), dim3(256), lds, (hipStream_t)stream, q, k, v,
                           (long long)ld, adj, A, heads, dk, dv, scale, out, (long long)ldo, att_weights);
    else
        hipLaunchKernelGGL(k_agent_attention<0>, dim3(B), dim3(256), lds, (hipStream_t)stream, q, k, v,
                           (long long)ld, adj, A, heads, dk, dv, scale, out, (long long)ldo, att_weights);
    return launched("gm_agent_attention");
}

extern "C" int gm_agent_comm(const float* h, int64_t ldh, const int8_t* adj, int32_t B, int32_t A, int32_t H,
                             float* out, int64_t ldo, void* stream) {
    if (!h || !adj || !out || B <= 0 || A <= 0 || A > MAXA || H <= 0 || ldh < H || ldo < H || h == out)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_agent_comm: bad arguments (A <= 64, out must not alias h)");
    hipLaunchKernelGGL(k_agent_comm, dim3(B), dim3(256), 0, (hipStream_t)stream, h, (long long)ldh, adj, A, H, out,
                       (long long)ldo);
    return launched("gm_agent_comm");
}
