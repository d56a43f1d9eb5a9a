// Probe: which HIP streams share a hardware queue, for the streams a gsrt context + communicator creates, in their
// creation order. A spin kernel (one wave, ~2 ms of s_memrealtime) goes on stream i, then a one-wave stamp kernel on
// stream j: when j shares i's hardware queue the stamp waits behind the spin (queues are FIFOs), otherwise it runs at
// once. Prints the matrix ('X' = j waited for i).
//   hipcc -O3 --offload-arch=gfx950 -o queue_map_probe queue_map_probe.hip -lrccl
//   ./queue_map_probe [order]    order: a string of stream kinds in creation order (default "NHLHLcC":
//                                N normal, H highest priority, L lowest, c = ncclCommInitRank (1 rank), C normal)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

__global__ void k_spin(uint32_t ticks) {
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    while ((uint32_t)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_stamp(uint32_t* out) {
    if (threadIdx.x == 0) out[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
}
__global__ void k_now(uint32_t* out) {
    if (threadIdx.x == 0) out[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
}

int main(int argc, char** argv) {
    const std::string order = argc > 1 ? argv[1] : "NHLHLcC";
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    std::vector<hipStream_t> s;
    std::vector<char> kind;
    ncclComm_t comm = nullptr;
    for (char k : order) {
        if (k == 'c') {
            ncclUniqueId id;
            ncclGetUniqueId(&id);
            if (ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) { printf("nccl init failed\n"); return 1; }
            continue;
        }
        hipStream_t x;
        const int prio = k == 'H' ? hi : (k == 'L' ? lo : 0);
        if (hipStreamCreateWithPriority(&x, hipStreamNonBlocking, prio) != hipSuccess) return 1;
        s.push_back(x);
        kind.push_back(k);
    }
    uint32_t *d, h[2];
    hipMalloc(&d, 8);
    const uint32_t ticks = 200000;  // 2 ms at 100 MHz
    // warm up every stream
    for (auto x : s) hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, x, d);
    hipDeviceSynchronize();
    printf("streams in creation order: %s (ncclCommInitRank at 'c')\n     ", order.c_str());
    for (size_t j = 0; j < s.size(); ++j) printf(" %c%zu", kind[j], j);
    printf("\n");
    for (size_t i = 0; i < s.size(); ++i) {
        printf("%c%zu:  ", kind[i], i);
        for (size_t j = 0; j < s.size(); ++j) {
            if (i == j) { printf("  -"); continue; }
            hipLaunchKernelGGL(k_now, dim3(1), dim3(64), 0, s[i], d + 1);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[i], ticks);
            hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s[j], d);
            hipDeviceSynchronize();
            hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
            const int32_t dt = (int32_t)(h[0] - h[1]);  // stamp time - spin start, 10 ns ticks
            printf("  %c", dt > (int32_t)(ticks * 9 / 10) ? 'X' : '.');
        }
        printf("\n");
    }
    if (comm) ncclCommDestroy(comm);
    return 0;
}
