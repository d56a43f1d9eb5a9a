// Probe: what a broadcast SH-row read and its FMAs cost on gfx950 (the k_render_cor blend step).
//   hipcc -O3 --offload-arch=gfx950 -o lds_bcast_probe lds_bcast_probe.hip
//   rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES --kernel-trace -- ./lds_bcast_probe
// Kernels (one-wave workgroups, 24 waves per CU, as k_render_cor):
//   k_bcast<M>  12 broadcast ds_read_b128 per iteration (every lane the same address) + 48 FMAs, with EXEC
//               restricted to lane mask M (tests whether b128 lane groups without an active lane cost LDS cycles)
//   k_dpp       48 v_fmac_f32_dpp row_newbcast per iteration (coefficients from 3 ds_read_b32)
//   k_fma       48 plain v_fmac per iteration (no LDS): the VALU issue rate reference
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 2048;

template <uint64_t M>
__global__ __launch_bounds__(64) void k_bcast(float* out, float seed) {
    __shared__ float4 sh[64 * 12];
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    for (int i = lane; i < 64 * 12; i += 64) sh[i] = make_float4(seed + i, seed - i, seed * i, 1.0f);
    __syncthreads();
    float bs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) bs[q] = seed * (q + lane);
    float acc = 0.0f;
    if ((M >> lane) & 1) {
        for (int it = 0; it < kIters; ++it) {
            const float4* s4 = sh + (it & 63) * 12;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const float4 q0 = s4[ch * 4 + 0], q1 = s4[ch * 4 + 1], q2 = s4[ch * 4 + 2], q3 = s4[ch * 4 + 3];
                const float s[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                     q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
                float a = s[0];
#pragma unroll
                for (int q = 1; q < 16; ++q) a = fmaf(bs[q], s[q], a);
                acc += a;
            }
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

__global__ __launch_bounds__(64) void k_fma(float* out, float seed) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    float bs[16], c[3];
#pragma unroll
    for (int q = 0; q < 16; ++q) bs[q] = seed * (q + lane);
    for (int k = 0; k < 3; ++k) c[k] = seed + k + lane;
    float acc = 0.0f;
    for (int it = 0; it < kIters; ++it) {
        float a0 = c[0] * bs[0], a1 = c[1] * bs[0], a2 = c[2] * bs[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            asm volatile("v_fmac_f32 %0, %3, %4\n\tv_fmac_f32 %1, %3, %5\n\tv_fmac_f32 %2, %3, %6"
                         : "+v"(a0), "+v"(a1), "+v"(a2) : "v"(bs[q]), "v"(c[0]), "v"(c[1]), "v"(c[2]));
        }
        acc += a0 + a1 + a2;
        c[0] += 1.0f;
    }
    out[blockIdx.x * 64 + lane] = acc;
}

#define DPP3(k)                                                                                          \
    "v_fmac_f32_dpp %0, %4, %3 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n\t"                    \
    "v_fmac_f32_dpp %1, %5, %3 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n\t"                    \
    "v_fmac_f32_dpp %2, %6, %3 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n\t"

__global__ __launch_bounds__(64) void k_dpp(float* out, float seed) {
    __shared__ float shc[64 * 48];
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    for (int i = lane; i < 64 * 48; i += 64) shc[i] = seed + i;
    __syncthreads();
    float bs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) bs[q] = seed * (q + lane);
    float acc = 0.0f;
    for (int it = 0; it < kIters; ++it) {
        const float* row = shc + (it & 63) * 48 + (lane & 15);
        float c0 = row[0], c1 = row[16], c2 = row[32];
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
        asm volatile("s_nop 1\n\t" DPP3(0) DPP3(1) DPP3(2) DPP3(3) DPP3(4) DPP3(5) DPP3(6) DPP3(7)
                         : "+v"(a0), "+v"(a1), "+v"(a2)
                         : "v"(bs[0]), "v"(c0), "v"(c1), "v"(c2));
        asm volatile(DPP3(8) DPP3(9) DPP3(10) DPP3(11) DPP3(12) DPP3(13) DPP3(14) DPP3(15)
                         : "+v"(a0), "+v"(a1), "+v"(a2)
                         : "v"(bs[1]), "v"(c0), "v"(c1), "v"(c2));
        acc += a0 + a1 + a2;
    }
    out[blockIdx.x * 64 + lane] = acc;
}

template <class F>
static float time_it(const char* name, F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.3f ms\n", name, ms);
    return ms;
}

int main() {
    const int blocks = 256 * 24 * 2;
    float* out;
    hipMalloc(&out, blocks * 64 * sizeof(float));
    constexpr uint64_t ALL = ~0ull;
    constexpr uint64_t G0 = 0x0ff0f00full;                                  // b128 lane group {0-3,12-15,20-27}
    constexpr uint64_t ROW0 = 0xffffull;                                    // lanes 0-15
    constexpr uint64_t HALF = 0xffffffffull;                                // lanes 0-31
    constexpr uint64_t G0G2 = G0 | (G0 << 32);                              // two groups, one per half
    constexpr uint64_t ONE = 1ull;
    time_it("bcast all lanes", [&] { hipLaunchKernelGGL(k_bcast<ALL>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("bcast group0 only", [&] { hipLaunchKernelGGL(k_bcast<G0>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("bcast lanes 0-15", [&] { hipLaunchKernelGGL(k_bcast<ROW0>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("bcast lanes 0-31", [&] { hipLaunchKernelGGL(k_bcast<HALF>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("bcast group0+group2", [&] { hipLaunchKernelGGL(k_bcast<G0G2>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("bcast lane 0", [&] { hipLaunchKernelGGL(k_bcast<ONE>, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("fma plain (48/iter)", [&] { hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    time_it("fma dpp newbcast (48/iter)", [&] { hipLaunchKernelGGL(k_dpp, dim3(blocks), dim3(64), 0, 0, out, 1.0f); });
    hipFree(out);
    return 0;
}
