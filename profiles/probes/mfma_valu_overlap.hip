// Probe: do MFMA instructions of one wave and VALU FMAs of another wave on the SAME SIMD run concurrently?
// One workgroup of 8 waves per CU: wave w runs on SIMD w % 4 (two waves per SIMD). Mode 0: waves 0-3 issue a
// chain-free MFMA stream (8 independent accumulators), waves 4-7 idle; mode 1: waves 4-7 issue independent
// v_fma_f32 streams, waves 0-3 idle; mode 2: both. Concurrent pipes give t2 ~ max(t0, t1); a shared issue
// port gives t2 ~ t0 + t1. MFMA kinds: 0 = v_mfma_f32_16x16x4_f32, 1 = v_mfma_f32_16x16x32_bf16,
// 2 = v_mfma_f32_32x32x2_f32.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_valu_overlap.hip -o profiles/probes/mfma_valu_overlap_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ __launch_bounds__(512) void k_overlap(float* out, int mfma_iters, int valu_iters, int mode) {
    const int w = threadIdx.x / 64;
    float sink = 0.0f;
    if (w < 4 && mode != 1) {
        if constexpr (KIND == 2) {
            f16v acc[2];
            for (int j = 0; j < 2; ++j) acc[j] = f16v{};
            float a = threadIdx.x * 1e-3f, b = 1.0f;
            for (int i = 0; i < mfma_iters; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
            }
            for (int j = 0; j < 2; ++j) sink += acc[j][0];
        } else {
            f4 acc[8];
            for (int j = 0; j < 8; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
            float a = threadIdx.x * 1e-3f, b = 1.0f;
            bf8 ab, bb;
            for (int j = 0; j < 8; ++j) { ab[j] = (__bf16)(a + j); bb[j] = (__bf16)1.0f; }
            for (int i = 0; i < mfma_iters; ++i) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if constexpr (KIND == 0) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
                    else acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc[j], 0, 0, 0);
                }
            }
            for (int j = 0; j < 8; ++j) sink += acc[j][0];
        }
    }
    if (w >= 4 && mode != 0) {
        float x[8];
        for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3f + j;
        const float m = 0.999f, c = 1e-3f;
        for (int i = 0; i < valu_iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = fmaf(x[j], m, c);
        }
        for (int j = 0; j < 8; ++j) sink += x[j];
    }
    if (sink == 12345.678f) out[threadIdx.x] = sink;  // keep the work
}

template <int KIND>
static float run(int mfma_iters, int valu_iters, int mode, int cus) {
    float* out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_overlap<KIND>, dim3(cus), dim3(512), 0, 0, out, mfma_iters, valu_iters, mode);
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(k_overlap<KIND>, dim3(cus), dim3(512), 0, 0, out, mfma_iters, valu_iters, mode);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipFree(out);
    return ms / 5;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const char* names[3] = {"16x16x4_f32", "16x16x32_bf16", "32x32x2_f32"};
    for (int kind = 0; kind < 3; ++kind) {
        const int mi = 4000, vi = 16000;
        float t0, t1, t2;
        if (kind == 0) { t0 = run<0>(mi, vi, 0, cus); t1 = run<0>(mi, vi, 1, cus); t2 = run<0>(mi, vi, 2, cus); }
        else if (kind == 1) { t0 = run<1>(mi, vi, 0, cus); t1 = run<1>(mi, vi, 1, cus); t2 = run<1>(mi, vi, 2, cus); }
        else { t0 = run<2>(mi, vi, 0, cus); t1 = run<2>(mi, vi, 1, cus); t2 = run<2>(mi, vi, 2, cus); }
        const double mfma_n = (kind == 2 ? 2.0 : 8.0) * mi;  // MFMAs per wave
        const double valu_n = 8.0 * vi;                       // FMAs per wave
        std::printf("%-14s mfma-only %.3f ms (%.1f cyc/MFMA at 2.4 GHz)  valu-only %.3f ms (%.2f cyc/FMA)  both %.3f ms"
                    "  -> both / (mfma + valu) = %.2f, both / max = %.2f\n",
                    names[kind], t0, t0 * 1e-3 * 2.4e9 / mfma_n, t1, t1 * 1e-3 * 2.4e9 / valu_n, t2, t2 / (t0 + t1),
                    t2 / (t0 > t1 ? t0 : t1));
    }
    return 0;
}
