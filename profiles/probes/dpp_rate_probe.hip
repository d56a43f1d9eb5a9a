// DPP VALU rate probe: a loop of v_fmac_f32 with / without row_newbcast, 3 independent chains, many waves
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void k(float* out, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, c0 = a0 * 0.5f, c1 = a0 * 0.25f, c2 = a0 * 0.125f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                asm volatile("v_fmac_f32 %0, %3, %6\n\tv_fmac_f32 %1, %4, %6\n\tv_fmac_f32 %2, %5, %6"
                             : "+v"(a0), "+v"(a1), "+v"(a2) : "v"(c0), "v"(c1), "v"(c2), "v"(b));
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                asm volatile("v_fmac_f32_dpp %0, %3, %6 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                             "v_fmac_f32_dpp %1, %4, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                             "v_fmac_f32_dpp %2, %5, %6 row_newbcast:7 row_mask:0xf bank_mask:0xf"
                             : "+v"(a0), "+v"(a1), "+v"(a2) : "v"(c0), "v"(c1), "v"(c2), "v"(b));
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2;
}
int main() {
    float* o;
    (void)hipMalloc(&o, 4 << 20);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int blocks = 256 * 4 * 6, iters = 2000;
    for (int m = 0; m < 2; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, o, iters);
            else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, o, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * iters * 48;  // wave-instructions
            printf("%s rep %d: %.3f ms, %.2f wave-instr per CU-cycle (2.4 GHz)\n", m ? "fmac_dpp" : "fmac    ", rep, ms,
                   ops / (ms * 1e-3) / 256 / 2.4e9);
        }
    }
    return 0;
}
