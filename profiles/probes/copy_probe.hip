// Probe: device-to-device copy rates of copy-kernel shapes on the MI355X (the scene-update copies, C5: 240 MB params,
// 120 MB AABBs). hipcc -O3 --offload-arch=gfx950 -o copy_probe copy_probe.hip && ./copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// the library's k_copy_rows: one-wave workgroups, grid-stride, U loads of 16 B per lane in flight
template <int U>
__global__ __launch_bounds__(64) void k_rows(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    const size_t row = 64 * U, stride = (size_t)gridDim.x * row;
    for (size_t i = (size_t)blockIdx.x * row + threadIdx.x; i < n16; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 64 * u < n16) v[u] = src[i + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 64 * u < n16) dst[i + 64 * u] = v[u];
    }
}
// one pass: every workgroup copies one block of B threads x U x 16 B (no loop), 32-bit indices
template <int B, int U>
__global__ __launch_bounds__(B) void k_block(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t n16) {
    const uint32_t base = blockIdx.x * (B * U) + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + B * u < n16) v[u] = __builtin_nontemporal_load(&src[base + B * u].x) == 0 ? src[base + B * u] : src[base + B * u];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + B * u < n16) dst[base + B * u] = v[u];
}
template <int B, int U>
__global__ __launch_bounds__(B) void k_block2(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t n16) {
    const uint32_t base = blockIdx.x * (B * U) + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + B * u < n16) v[u] = src[base + B * u];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + B * u < n16) dst[base + B * u] = v[u];
}

int main() {
    const size_t bytes = 240ull << 20;  // C5's params
    const size_t n16 = bytes / 16;
    uint4 *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-34s %8.1f us  %6.2f TB/s (read + write)\n", name, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e12);
    };
    run("k_rows<4> x1024", [&] { hipLaunchKernelGGL(k_rows<4>, dim3(1024), dim3(64), 0, 0, b, a, n16); });
    run("k_rows<8> x2048", [&] { hipLaunchKernelGGL(k_rows<8>, dim3(2048), dim3(64), 0, 0, b, a, n16); });
    run("k_rows<8> x8192", [&] { hipLaunchKernelGGL(k_rows<8>, dim3(8192), dim3(64), 0, 0, b, a, n16); });
    run("k_rows<4> x16384", [&] { hipLaunchKernelGGL(k_rows<4>, dim3(16384), dim3(64), 0, 0, b, a, n16); });
    run("k_block2<64,8> (1 pass)", [&] { hipLaunchKernelGGL((k_block2<64, 8>), dim3((n16 + 511) / 512), dim3(64), 0, 0, b, a, (uint32_t)n16); });
    run("k_block2<64,4> (1 pass)", [&] { hipLaunchKernelGGL((k_block2<64, 4>), dim3((n16 + 255) / 256), dim3(64), 0, 0, b, a, (uint32_t)n16); });
    run("k_block2<256,4> (1 pass)", [&] { hipLaunchKernelGGL((k_block2<256, 4>), dim3((n16 + 1023) / 1024), dim3(256), 0, 0, b, a, (uint32_t)n16); });
    run("k_block2<256,8> (1 pass)", [&] { hipLaunchKernelGGL((k_block2<256, 8>), dim3((n16 + 2047) / 2048), dim3(256), 0, 0, b, a, (uint32_t)n16); });
    run("k_block<256,4> (nt load)", [&] { hipLaunchKernelGGL((k_block<256, 4>), dim3((n16 + 1023) / 1024), dim3(256), 0, 0, b, a, (uint32_t)n16); });
    run("hipMemcpyAsync D2D", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
