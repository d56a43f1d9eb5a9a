// gsrt_scene.hip -- per-Gaussian kernels: scene build (a1) and per-frame projection (rint:62-102).
//
// Both are one thread per Gaussian, HBM-bound streaming kernels: 40 B in / 72 B out for the scene
// build, 72 B in / 64 B out per frame for the projection.
#include <algorithm>
#include <cstdint>

#include "gsrt_internal.hpp"
#include "gsrt_project.hpp"

namespace gsrt {

// Gauss::init_cov3d / init_radius / BoundingBox (RayTracingInVulkan/src/Assets/Sphere.hpp:108-165),
// packed as Scene.cpp:125-136 does. glm mat3 products are summed left to right.
__global__ __launch_bounds__(256) void k_cov3d(uint32_t n, const float* __restrict__ center,
                                               const float* __restrict__ rot, const float* __restrict__ scale,
                                               const float* __restrict__ opacity, gsrt_gauss_param* __restrict__ params,
                                               gsrt_aabb* __restrict__ aabbs) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float r = rot[4 * i + 0], x = rot[4 * i + 1], y = rot[4 * i + 2], z = rot[4 * i + 3];
    const float s0 = scale[3 * i + 0], s1 = scale[3 * i + 1], s2 = scale[3 * i + 2];
    // R[c][row], glm::mat3 column-major constructor (Sphere.hpp:143-147)
    float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                  2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                  2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
    const float S[9] = {s0, 0.f, 0.f, 0.f, s1, 0.f, 0.f, 0.f, s2};
    float M[9];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            M[c * 3 + k] = (S[0 * 3 + k] * R[c * 3 + 0] + S[1 * 3 + k] * R[c * 3 + 1]) + S[2 * 3 + k] * R[c * 3 + 2];
    // Sigma = transpose(M) * M: Sigma[c][k] = (Mt[0][k]*M[c][0] + Mt[1][k]*M[c][1]) + Mt[2][k]*M[c][2], Mt[a][k] = M[k][a]
    float Sig[9];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            Sig[c * 3 + k] = (M[k * 3 + 0] * M[c * 3 + 0] + M[k * 3 + 1] * M[c * 3 + 1]) + M[k * 3 + 2] * M[c * 3 + 2];
    gsrt_gauss_param g;
    g.center_opacity[0] = center[3 * i + 0];
    g.center_opacity[1] = center[3 * i + 1];
    g.center_opacity[2] = center[3 * i + 2];
    g.center_opacity[3] = opacity[i];
    g.cov3d[0] = Sig[0]; g.cov3d[1] = Sig[1]; g.cov3d[2] = Sig[2];
    g.cov3d[3] = Sig[4]; g.cov3d[4] = Sig[5]; g.cov3d[5] = Sig[8];
    g.pad[0] = 0.f; g.pad[1] = 0.f;
    params[i] = g;
    float mx = s0;
    if (s1 > mx) mx = s1;
    if (s2 > mx) mx = s2;
    const float rad = (float)(3.0 * (double)mx);  // Sphere.hpp:164, double product stored as float
    gsrt_aabb a;
    a.min_x = g.center_opacity[0] - rad; a.min_y = g.center_opacity[1] - rad; a.min_z = g.center_opacity[2] - rad;
    a.max_x = g.center_opacity[0] + rad; a.max_y = g.center_opacity[1] + rad; a.max_z = g.center_opacity[2] + rad;
    aabbs[i] = a;
}

void launch_cov3d(hipStream_t s, uint32_t n, const float* center, const float* rot, const float* scale,
                  const float* opacity, gsrt_gauss_param* params, gsrt_aabb* aabbs) {
    if (!n) return;
    hipLaunchKernelGGL(k_cov3d, dim3((n + 255) / 256), dim3(256), 0, s, n, center, rot, scale, opacity, params, aabbs);
}

// keyed (per frame slot, one bit per splat, nullable): bit 0 = the splat's record depth and node key in this slot
// are +inf (it was outside the rank's tiles when the slot was last projected), so while it stays outside, nothing
// needs writing. Bits are rewritten here every projection; all ones (unknown) after a build, a buffer allocation,
// or a frame that wrote the slot without this kernel's bookkeeping (launch_render).
template <int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void k_project(uint32_t n, const gsrt_ubo ubo,
                                                 const gsrt_gauss_param* __restrict__ params,
                                                 const gsrt_aabb* __restrict__ aabbs, SplatRec* __restrict__ recs,
                                                 BvhNode* __restrict__ nodes, const uint32_t* __restrict__ gid_slot,
                                                 float4* __restrict__ footprint,
                                                 unsigned long long* __restrict__ counters, const RankTiles own,
                                                 uint32_t* __restrict__ keyed, uint32_t leaf_fp,
                                                 uint32_t* __restrict__ depth_unsafe) {
    __builtin_amdgcn_s_setprio(kPrepSetprio);  // see gsrt_render.hip: ahead of the render kernel's waves
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    // the frame's stats words (ordered before every kernel that adds to them); the error word stays: a pipelined
    // frame's projection runs while the previous frame's render may still set it
    if (i < kCounters && i != kErrWord) counters[i] = 0;
    bool k = true;
    if (i < n) {
        const bool prev = keyed ? ((keyed[i >> 5] >> (i & 31u)) & 1u) != 0 : true;
        k = project_one<MODE>(i, n, ubo, params, aabbs, recs, nodes, gid_slot, footprint, own, prev, leaf_fp != 0,
                              depth_unsafe);
    }
    if (keyed) {  // one-wave workgroups: lanes 0 and 32 write the wave's two bitmap words
        const uint64_t m = __ballot(k);
        if ((threadIdx.x & 31u) == 0 && i < n) keyed[i >> 5] = (uint32_t)(m >> (threadIdx.x & 32u));
    }
}

void launch_project(hipStream_t st, uint32_t n, uint32_t mode, const gsrt_ubo& ubo, const gsrt_gauss_param* params,
                    const gsrt_aabb* aabbs, SplatRec* recs, BvhNode* nodes, const uint32_t* gid_slot, float4* footprint,
                    unsigned long long* counters, const RankTiles* own, uint32_t* keyed, bool leaf_fp,
                    uint32_t* depth_unsafe) {
    const RankTiles all{};  // active = 0: every splat kept
    if (!n) {
        (void)hipMemsetAsync(counters, 0, sizeof(unsigned long long) * kErrWord, st);
        (void)hipMemsetAsync(counters + kErrWord + 1, 0, sizeof(unsigned long long) * (kCounters - kErrWord - 1), st);
        return;
    }
    dim3 grid((n + 63) / 64), block(64);
    if (n < 2) nodes = nullptr;  // a single Gaussian is the root leaf: no parent node to hold its key
    if ((mode & 0xff) == GSRT_MODE_REF)
        hipLaunchKernelGGL(k_project<GSRT_MODE_REF>, grid, block, 0, st, n, ubo, params, aabbs, recs, nullptr, nullptr,
                           nullptr, counters, all, nullptr, 0u, nullptr);
    else hipLaunchKernelGGL(k_project<GSRT_MODE_COR>, grid, block, 0, st, n, ubo, params, aabbs, recs, nodes, gid_slot,
                            footprint, counters, own && footprint ? *own : all, keyed, leaf_fp && nodes ? 1u : 0u,
                            depth_unsafe);
}

// Scene-update copies (gsrt_scene_update / refit / stream_pages from device sources) beside the previous frames'
// kernels: 1024 one-wave workgroups looping over the rows, each copying 4 x 1 KB per step (16 B per lane in flight 4
// times). Few short workgroups of few VGPRs take the slots render waves free without crowding them out. Measured alone
// on 240 MB (profiles/probes/copy_probe.hip): 2.51 TB/s read + write; one pass with a workgroup per 4 KB reached 4.99
// and 16384 looping workgroups 4.71, but both were slower beside the render kernel on the C5 share; the
// runtime's blit (5.32 alone) took 2.9 ms for C5's 360 MB beside a running render kernel (starved of dispatch slots)
constexpr uint32_t kCopyUnroll = 4;
constexpr size_t kCopyGroups = 1024;
__global__ __launch_bounds__(64) void k_copy_rows(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
    __builtin_amdgcn_s_setprio(kPrepSetprio);
    const size_t stride = (size_t)gridDim.x * (64 * kCopyUnroll);
    for (size_t base = (size_t)blockIdx.x * (64 * kCopyUnroll) + threadIdx.x; base < n16; base += stride) {
        uint4 v[kCopyUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kCopyUnroll; ++u)
            if (base + 64 * u < n16) v[u] = src[base + 64 * u];
#pragma unroll
        for (uint32_t u = 0; u < kCopyUnroll; ++u)
            if (base + 64 * u < n16) dst[base + 64 * u] = v[u];
    }
}

void launch_copy_d2d(hipStream_t s, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    if (((uintptr_t)dst | (uintptr_t)src | bytes) & 15u) {
        (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
        return;
    }
    const size_t n16 = bytes / 16;
    const size_t blocks = std::min(kCopyGroups, (n16 + 64 * kCopyUnroll - 1) / (64 * kCopyUnroll));
    hipLaunchKernelGGL(k_copy_rows, dim3((uint32_t)blocks), dim3(64), 0, s, reinterpret_cast<uint4*>(dst),
                       reinterpret_cast<const uint4*>(src), n16);
}

}  // namespace gsrt
