// Layer activations of the MLPs (reference --activation-function: any elementwise torch.nn.functional
// name with its default arguments, src/main.py:194-197, 440-441, applied by MLP / AttModel,
// src/model.py:13-42, 86-117). GM_ACT_* in include/graph_marl_amd.h:
//   0 none, 1 leaky_relu (slope 0.01), 2 relu, 3 elu (alpha 1), 4 tanh, 5 sigmoid, 6 relu6, 7 hardtanh
//   (-1, 1), 8 hardsigmoid, 9 selu, 10 celu (alpha 1), 11 softsign, 12 logsigmoid, 13 softplus (beta 1,
//   threshold 20) -- derivative from the layer OUTPUT; 14 gelu (exact erf form), 15 silu, 16 mish,
//   17 hardswish, 18 tanhshrink -- derivative from the PRE-activation (gm_act_dz).
// Precise libm forms (expm1f / tanhf / expf / erff / log1pf), like torch's CPU kernels.
#pragma once
#include <hip/hip_runtime.h>

constexpr float GM_SELU_SCALE = 1.0507009873554804934193349852946f;
constexpr float GM_SELU_ALPHA = 1.6732632423543772848170429916717f;

// softplus(v) with torch's threshold (beta 1: v > 20 -> v), log1p(exp(v)) else
__device__ __forceinline__ float gm_softplus(float v) { return v > 20.f ? v : log1pf(expf(v)); }

__device__ __forceinline__ float gm_act(float v, int act) {
    switch (act) {
        case 1: return v >= 0.f ? v : 0.01f * v;
        case 2: return v > 0.f ? v : 0.f;
        case 3: return v > 0.f ? v : expm1f(v);
        case 4: return tanhf(v);
        case 5: return 1.0f / (1.0f + expf(-v));
        case 6: return fminf(fmaxf(v, 0.f), 6.f);
        case 7: return fminf(fmaxf(v, -1.f), 1.f);
        case 8: return fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
        case 9: return GM_SELU_SCALE * (v > 0.f ? v : GM_SELU_ALPHA * expm1f(v));
        case 10: return v > 0.f ? v : expm1f(v);
        case 11: return v / (1.f + fabsf(v));
        case 12: return fminf(v, 0.f) - log1pf(expf(-fabsf(v)));  // torch's log_sigmoid form
        case 13: return gm_softplus(v);
        case 14: return 0.5f * v * (1.f + erff(v * 0.70710678118654752440f));
        case 15: return v / (1.0f + expf(-v));
        case 16: return v * tanhf(gm_softplus(v));
        case 17: return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
        case 18: return v - tanhf(v);
        default: return v;
    }
}

// the precise forms of the rarer activations as ONE out-of-line function per code object: inlined into
// every GEMM epilogue instantiation they quadrupled the library (7.9 -> 30.9 MB); static: internal linkage,
// one copy per translation unit (no duplicate symbol under relocatable device code)
static __device__ __noinline__ float gm_act_rare(float v, int act) { return gm_act(v, act); }

// GEMM epilogues (every tile instantiation carries one): leaky_relu / identity stay a select, the rest
// branch (wave-uniform act) to short hardware-transcendental forms (v_exp_f32 / v_rcp_f32, absolute
// error ~1e-7 against the 1e-5 tolerance; the libm forms in every instantiation double the library)
__device__ __forceinline__ float gm_act_fast(float v, int act) {
    if (act == 1) return v >= 0.f ? v : 0.01f * v;
    if (act == 0) return v;
    if (act == 2) return v > 0.f ? v : 0.f;
    constexpr float L2E = 1.44269504088896341f;
    if (act == 3) return v > 0.f ? v : __builtin_amdgcn_exp2f(v * L2E) - 1.0f;
    if (act <= 5) {
        const float x = act == 4 ? 2.0f * v : v;
        const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-L2E * x));
        return act == 4 ? 2.0f * s - 1.0f : s;
    }
    return gm_act_rare(v, act);  // the rarer names: the precise forms (one branch per wave, uniform act)
}

// d act / d x from the output y = act(x) (torch's backward conventions: leaky_relu / relu
// compare the input with 0, i.e. y > 0; elu / celu: x > 0 ? 1 : y + 1; selu: x > 0 ? scale :
// y + scale alpha; hardtanh / relu6 / hardsigmoid: inside the open interval; softsign (1 - |y|)^2;
// logsigmoid 1 - e^y; softplus y > 20 ? 1 : 1 - e^-y). Codes >= GM_ACT_GELU: gm_act_dz
__device__ __forceinline__ float gm_act_dy(float y, int act) {
    switch (act) {
        case 1: return y > 0.f ? 1.f : 0.01f;
        case 2: return y > 0.f ? 1.f : 0.f;
        case 3: return y > 0.f ? 1.f : y + 1.f;
        case 4: return 1.f - y * y;
        case 5: return y * (1.f - y);
        case 6: return (y > 0.f && y < 6.f) ? 1.f : 0.f;
        case 7: return (y > -1.f && y < 1.f) ? 1.f : 0.f;
        case 8: return (y > 0.f && y < 1.f) ? 1.f / 6.f : 0.f;
        case 9: return y > 0.f ? GM_SELU_SCALE : y + GM_SELU_SCALE * GM_SELU_ALPHA;
        case 10: return y > 0.f ? 1.f : y + 1.f;
        case 11: {
            const float t = 1.f - fabsf(y);
            return t * t;
        }
        case 12: return -expm1f(y);
        case 13: return y > 20.f ? 1.f : -expm1f(-y);
        default: return 1.f;
    }
}

// d act / d z from the pre-activation z (every code; torch's formulas: gelu Phi(z) + z phi(z), silu
// s (1 + z (1 - s)), mish tanh(sp) + z sech^2(sp) sigmoid(z), hardswish z < -3 ? 0 : z <= 3 ? z / 3 + 0.5 : 1,
// tanhshrink tanh^2)
__device__ __forceinline__ float gm_act_dz(float z, int act) {
    switch (act) {
        case 14: {
            const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752440f));
            const float pdf = expf(-0.5f * z * z) * 0.39894228040143267794f;
            return cdf + z * pdf;
        }
        case 15: {
            const float s = 1.0f / (1.0f + expf(-z));
            return s * (1.f + z * (1.f - s));
        }
        case 16: {
            const float t = tanhf(gm_softplus(z));
            const float s = 1.0f / (1.0f + expf(-z));
            return t + z * (1.f - t * t) * s;
        }
        case 17: return z < -3.f ? 0.f : (z <= 3.f ? z / 3.f + 0.5f : 1.f);
        case 18: {
            const float t = tanhf(z);
            return t * t;
        }
        default: return act == 0 ? 1.f : gm_act_dy(gm_act(z, act), act);
    }
}
