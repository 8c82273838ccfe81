// Device-wide max |x| for the power-of-two operand scales of the split-f16 gradient GEMMs
// (gm_absmax_finish turns the max into the scale). Non-negative floats order like their bit
// patterns, so the max is an unsigned atomicMax on the float bits (the slot zeroed first);
// an agent-scope load skips the atomic when the slot already holds a larger value, so
// producers with thousands of blocks do not serialise on the one address.
#pragma once
#include <hip/hip_runtime.h>

__device__ inline float gm_wave_max(float m) {
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    return m;
}

__device__ inline void gm_amax_publish(unsigned* slot, float m) {
    const unsigned b = __float_as_uint(m);
    if (b > __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(slot, b);
}

// block-wide max (blockDim.x a multiple of 64, at most 1024) published once per block
__device__ inline void gm_block_amax(unsigned* slot, float m) {
    __shared__ float red[16];
    m = gm_wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); i++) m = fmaxf(m, red[i]);
        gm_amax_publish(slot, m);
    }
}
