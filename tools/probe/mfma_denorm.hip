// Does v_mfma_f32_16x16x32_f16 keep f16 denormal inputs? (DESIGN §9.0 lever (d)). One wave multiplies
// A = 2^-20 (f16 denormal; min normal 2^-14) by B = 1 over k = 32: exact result 32 * 2^-20 = 2^-15.
// Prints the result and the same product with A = 2^-10 (normal) for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, float a) {
    half8 va, vb;
    for (int i = 0; i < 8; i++) { va[i] = (_Float16)a; vb[i] = (_Float16)1.0f; }
    floatx4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, vb, c, 0, 0, 0);
    if (threadIdx.x == 0) out[0] = c[0];
}
int main() {
    float* d;
    float h[2];
    if (hipMalloc(&d, 8) != hipSuccess) return 1;
    const float as[2] = {0x1p-20f, 0x1p-10f};
    for (int t = 0; t < 2; t++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, as[t]);
        if (hipMemcpy(&h[t], d, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    }
    printf("denormal A 2^-20: got %a (exact 0x1p-15)\nnormal A 2^-10: got %a (exact 0x1p-5)\n", h[0], h[1]);
    (void)hipFree(d);
    return 0;
}
