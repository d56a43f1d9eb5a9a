// gsrt_mesh_trace.hip -- closest triangle hit per primary ray of a REF frame.
//
// Reference: inside VulkanRayTracing::traceRay every triangle of a hit BLAS leaf is tested with
// mt_ray_triangle_test (vulkan-sim/src/cuda-sim/vulkan_ray_tracing.cc:1184-1206) against the object ray of the
// identity instance (origin o, direction d/|d|, :148-160); a hit counts when Tmin <= t/|d| <= Tmax (:925-931)
// and min_thit keeps the smallest (:929-931). The REF rays of a pixel are the same every round and sample
// (GaussTracing.rgen:37-43, no jitter, origin never advanced), so gsrt computes min_thit once per pixel here,
// before k_render_ref, which uses it for the Gaussian cull (:806-807), the report rule (instructions.cc:7050)
// and the triangle closest-hit (Trans = 0, RayTracing.rchit + Scatter.glsl).
//
// One lane per pixel, 8x8-pixel tiles per 64-lane workgroup (k_render_ref's tile shape), a per-lane DFS over
// the host-built mesh BVH with the stack in LDS (lane-interleaved: no bank conflicts). The minimum over the
// triangles a ray hits does not depend on the visiting order; a child box is skipped when the ray misses it or
// enters it farther than the best hit so far by a margin (1e-3 relative) that covers the rounding of the
// Moller-Trumbore t against the slab bound of the same triangle, so the result equals the brute-force minimum
// the oracle computes.
#include "gsrt_internal.hpp"

namespace gsrt {

// mt_ray_triangle_test (vulkan_ray_tracing.cc:1184-1206) with vector-math.cc's cross / dot (:41-50), left to
// right; e1 = v0v1, e2 = v0v2 (precomputed with the same fp32 subtractions). Returns the object-space t, or NaN
// when the test rejects (NaN fails the caller's Tmin <= t test, as a rejection does).
__device__ inline float mt_thit(const float o[3], const float dir[3], const float4 p0, const float4 e1,
                                const float4 e2) {
    const float px = dir[1] * e2.z - dir[2] * e2.y;  // pvec = cross(dir, v0v2)
    const float py = dir[2] * e2.x - dir[0] * e2.z;
    const float pz = dir[0] * e2.y - dir[1] * e2.x;
    const float det = (e1.x * px + e1.y * py) + e1.z * pz;
    const float idet = 1.0f / det;
    const float tx = o[0] - p0.x, ty = o[1] - p0.y, tz = o[2] - p0.z;  // tvec
    const float u = ((tx * px + ty * py) + tz * pz) * idet;
    if (u < 0.0f || u > 1.0f) return __builtin_nanf("");
    const float qx = ty * e1.z - tz * e1.y;  // qvec = cross(tvec, v0v1)
    const float qy = tz * e1.x - tx * e1.z;
    const float qz = tx * e1.y - ty * e1.x;
    const float v = ((dir[0] * qx + dir[1] * qy) + dir[2] * qz) * idet;
    if (v < 0.0f || u + v > 1.0f) return __builtin_nanf("");
    return ((e2.x * qx + e2.y * qy) + e2.z * qz) * idet;
}

// entry t of the object ray into a box (ray_box_test, :217-237), +inf when it misses
__device__ inline float box_entry(const float o[3], const float idir[3], float tmin, float tmax, const float lo[3],
                                  const float hi[3]) {
    float l0 = (lo[0] - o[0]) * idir[0], h0 = (hi[0] - o[0]) * idir[0];
    float l1 = (lo[1] - o[1]) * idir[1], h1 = (hi[1] - o[1]) * idir[1];
    float l2 = (lo[2] - o[2]) * idir[2], h2 = (hi[2] - o[2]) * idir[2];
    float t = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(l0, h0), tmin),
                              __builtin_fmaxf(__builtin_fminf(l1, h1), __builtin_fminf(l2, h2)));
    float u = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(l0, h0), tmax),
                              __builtin_fminf(__builtin_fmaxf(l1, h1), __builtin_fmaxf(l2, h2)));
    return t <= u ? t : __builtin_inff();
}

__global__ __launch_bounds__(64) void k_mesh_thit(const gsrt_ubo ubo, const BvhNode* __restrict__ nodes,
                                                  const float4* __restrict__ tris, float* __restrict__ tri_t,
                                                  uint32_t tiles_x) {
    __shared__ uint32_t stack[kMeshStack][64];
    const uint32_t lane = threadIdx.x;
    const uint32_t px = (blockIdx.x % tiles_x) * 8 + (lane & 7u), py = (blockIdx.x / tiles_x) * 8 + (lane >> 3);
    if (px >= ubo.width || py >= ubo.height) return;
    float o[3], d[3];
    gen_ray(ubo, (float)px, (float)py, o, d);  // rgen:39-43 at the integer launch id
    // object ray of the identity instance (make_transformed_ray, :148-160; calculate_idir, :200-215)
    const float norm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    float dn[3], idir[3];
    const float ooeps = 8.27180613e-25f;  // exp2f(-80)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        dn[k] = d[k] / norm;
        idir[k] = 1.0f / (fabsf(dn[k]) > ooeps ? dn[k] : copysignf(ooeps, dn[k]));
    }
    const float tmin = kTMin * norm, tmax = kTMax * norm;
    float best = kTMax;  // min_thit starts at Tmax (:534); world units
    float bound = __builtin_inff();  // object-space entry beyond which no box can hold a closer hit
    uint32_t sp = 0;
    stack[sp++][lane] = 0u;
    while (sp) {
        const BvhNode& n = nodes[stack[--sp][lane]];
        const uint32_t refs[2] = {n.l_ref, n.r_ref}, cnt[2] = {n.l_key, n.r_key};
        const float* los[2] = {n.l_lo, n.r_lo};
        const float* his[2] = {n.l_hi, n.r_hi};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t ref = refs[c];
            if (ref == 0xFFFFFFFFu) continue;  // empty child of a one-leaf mesh
            if (box_entry(o, idir, tmin, tmax, los[c], his[c]) > bound) continue;
            if (ref & kLeafBit) {
                const uint32_t first = ref & ~kLeafBit;
                for (uint32_t i = first; i < first + cnt[c]; ++i) {
                    const float t = mt_thit(o, dn, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2]);
                    const float w = t / norm;  // world_thit (:925)
                    if (kTMin <= w && w <= kTMax && w < best) {
                        best = w;
                        bound = (best * norm) * 1.001f;
                    }
                }
            } else {
                stack[sp++][lane] = ref;
            }
        }
    }
    tri_t[(size_t)py * ubo.width + px] = best;
}

void launch_mesh_thit(hipStream_t s, const gsrt_ubo& ubo, const gsrt_scene* sc, float* tri_t) {
    const uint32_t tiles_x = (ubo.width + 7) / 8, tiles_y = (ubo.height + 7) / 8;
    hipLaunchKernelGGL(k_mesh_thit, dim3(tiles_x * tiles_y), dim3(64), 0, s, ubo, sc->d_mesh_nodes, sc->d_tris, tri_t,
                       tiles_x);
}

}  // namespace gsrt
