// Layer activations of the MLPs (reference --activation-function: any torch.nn.functional name,
// src/main.py:194-197, 440-441, applied by MLP / AttModel, src/model.py:13-42, 86-117). The
// built set is the one whose derivative follows from the layer OUTPUT alone, so the backward
// passes need no pre-activation tensor (GM_ACT_* in include/graph_marl_amd.h):
//   0 none, 1 leaky_relu (slope 0.01), 2 relu, 3 elu (alpha 1), 4 tanh, 5 sigmoid.
// Precise libm forms (expm1f / tanhf / expf), like torch's CPU kernels.
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ float gm_act(float v, int act) {
    switch (act) {
        case 1: return v >= 0.f ? v : 0.01f * v;
        case 2: return v > 0.f ? v : 0.f;
        case 3: return v > 0.f ? v : expm1f(v);
        case 4: return tanhf(v);
        case 5: return 1.0f / (1.0f + expf(-v));
        default: return v;
    }
}

// GEMM epilogues (every tile instantiation carries one): leaky_relu / identity stay a select, the rest
// branch (wave-uniform act) to short hardware-transcendental forms (v_exp_f32 / v_rcp_f32, absolute
// error ~1e-7 against the 1e-5 tolerance; the libm forms in every instantiation double the library)
__device__ __forceinline__ float gm_act_fast(float v, int act) {
    if (act == 1) return v >= 0.f ? v : 0.01f * v;
    if (act == 0) return v;
    if (act == 2) return v > 0.f ? v : 0.f;
    constexpr float L2E = 1.44269504088896341f;
    if (act == 3) return v > 0.f ? v : __builtin_amdgcn_exp2f(v * L2E) - 1.0f;
    const float x = act == 4 ? 2.0f * v : v;
    const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-L2E * x));
    return act == 4 ? 2.0f * s - 1.0f : s;
}

// d act / d x from the output y = act(x) (torch's backward conventions: leaky_relu / relu
// compare the input with 0, i.e. y > 0; elu: x > 0 ? 1 : y + 1)
__device__ __forceinline__ float gm_act_dy(float y, int act) {
    switch (act) {
        case 1: return y > 0.f ? 1.f : 0.01f;
        case 2: return y > 0.f ? 1.f : 0.f;
        case 3: return y > 0.f ? 1.f : y + 1.f;
        case 4: return 1.f - y * y;
        case 5: return y * (1.f - y);
        default: return 1.f;
    }
}
