// Dispatch-rate probe: how long does a grid of one-wave workgroups that do (almost) nothing take on one MI355X?
// Build: hipcc --offload-arch=gfx950 -O3 -o profiles/probes/dispatch_probe profiles/probes/dispatch_probe.hip
// Run under rocprofv3 --kernel-trace --stats; the kernel names carry the workgroup size.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_empty(unsigned* out, unsigned n) {
    const unsigned i = blockIdx.x * THREADS + threadIdx.x;
    if (i == 0xFFFFFFFFu) out[0] = n;  // never true: keeps the kernel from being empty
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_touch(const uint4* __restrict__ in, uint4* out, unsigned n) {
    const unsigned i = blockIdx.x * THREADS + threadIdx.x;
    uint4 v = i < n ? in[i] : make_uint4(0, 0, 0, 0);
    if (v.x == 0x12345678u && v.y == 0x9abcdef0u) out[0] = v;  // (never, for the zero-filled input)
}

int main() {
    unsigned* out = nullptr;
    uint4* in = nullptr;
    const unsigned n = 1u << 24;
    hipMalloc(&out, 64);
    hipMalloc(&in, sizeof(uint4) * n);
    hipMemset(in, 0, sizeof(uint4) * n);
    for (int rep = 0; rep < 20; ++rep) {
        for (unsigned blocks : {1024u, 4096u, 15625u, 62500u}) {
            hipLaunchKernelGGL(k_empty<64>, dim3(blocks), dim3(64), 0, 0, out, blocks);
            hipLaunchKernelGGL(k_empty<256>, dim3((blocks + 3) / 4), dim3(256), 0, 0, out, blocks);
            hipLaunchKernelGGL(k_touch<64>, dim3(blocks), dim3(64), 0, 0, in, reinterpret_cast<uint4*>(out), blocks * 64);
        }
    }
    hipDeviceSynchronize();
    std::printf("done\n");
    return 0;
}
