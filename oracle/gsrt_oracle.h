/*
 * gsrt_oracle.h -- CPU restatement of the reference's ray-traced 3DGS hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This header and gsrt_oracle.c are the checker used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing in the
 * product (3dgs-raytrace_amd/) includes, links or calls it.
 *
 * Parity pinning: the reference (RayTracingInVulkan + mesa-vulkan-sim + vulkan-sim +
 * Embree) cannot be built or run here. The only
 * reference-derived known answer is KAT-1 (scene 33 @16x16, hand-derived from
 * GaussTracing.rgen / RayTracing.ProceduralGauss.rint / .rchit and SceneList.cpp:108-128),
 * which tests/test_oracle.py checks. Everything else is "parity unpinned" against
 * the reference binary; it is pinned against this restatement only.
 *
 * Types here are declared independently of include/gsrt.h; tests check that the
 * byte layouts agree.
 */
#ifndef GSRT_ORACLE_H
#define GSRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GaussParam (RayTracingInVulkan/assets/shaders/Gauss.glsl:1-6, Sphere.hpp:10-19), 48 B std430 */
typedef struct { float center_opacity[4]; float cov3d[6]; float pad[2]; } or_gauss_param;
/* VkAabbPositionsKHR (Scene.cpp:129-130), 24 B */
typedef struct { float lo[3]; float hi[3]; } or_aabb;
/* UniformBufferObject (Assets/UniformBuffer.hpp:15-36), 320 B; matrices column-major */
typedef struct {
    float model_view[16], projection[16], model_view_inverse[16], projection_inverse[16];
    float light_position[3], light_radius, aperture, focus_distance, heatmap_scale;
    uint32_t total_samples, samples, bounces, shadows, random_seed, width, height, has_sky, show_heatmap;
} or_ubo;
/* per-ray state dump: RayInfo (RayPayload.glsl:11-16) + Ray.Trans + NextK[8] (Gauss.glsl:8-12) */
typedef struct {
    float trans; float depth; int32_t gauss_num; int32_t gauss_num_raw;
    float k[8][2];               /* {depth, alpha} */
} or_raystate;

enum { OR_MODE_REF = 0, OR_MODE_COR = 1 };
enum { OR_FLAG_LUT = 0x100 };    /* COR: use LinearExp LUT instead of the exp restatement */
enum { OR_SYNTH_COR = 0, OR_SYNTH_REF = 1, OR_SYNTH_NEEDLE = 2 };

/* glm restatements (glm 2022.05.10 via vcpkg, RTV/vcpkg_linux.sh:8) */
void or_perspective_rh_zo(float fovy_rad, float aspect, float znear, float zfar, float out[16]);
void or_inverse4(const float m[16], float out[16]);
void or_lookat_rh(const float eye[3], const float center[3], const float up[3], float out[16]);
void or_mul4(const float a[16], const float b[16], float out[16]);

/* RayTracer::GetUniformBufferObject (RayTracer.cpp:38-65) with ModelViewController::Reset +
 * ModelView (ModelViewController.cpp:4-34) applied to an initial modelview. */
void or_make_ubo(const float init_mv[16], float fovy_deg, uint32_t width, uint32_t height,
                 float focus_distance, uint32_t samples, uint32_t bounces, or_ubo* out);

/* Gauss::init_cov3d/init_radius + BoundingBox (Sphere.hpp:108-165) and Scene.cpp:125-136 packing */
void or_gauss_from_model(uint32_t n, const float* center, const float* rot_rxyz, const float* scale,
                         const float* opacity, or_gauss_param* out_params, or_aabb* out_aabbs);

/* generateExpLUT(256, 0, 8) (Utilities/ExpLUT.hpp:10-24, Scene.cpp:47): out[2*i] = k, out[2*i+1] = b */
void or_exp_lut(float out[512]);
/* LinearExp (RayTracing.ProceduralGauss.rint:45-54) */
float or_linear_exp(const float* lut, float x);
/* COR exponential: exp(x) for x<=0 built only from IEEE-exact ops (shared definition with the HIP kernel) */
float or_exp_neg(float x);

/* synthetic clouds: std::mt19937(seed) + std::uniform_real_distribution<float> */
void or_synth_cloud(uint32_t kind, uint32_t n, uint32_t seed, int with_sh,
                    float* center, float* rot_rxyz, float* scale, float* opacity, float* sh);

/* CPU BVH over AABBs (median split); candidate sets are BVH-independent (exact slab test on leaves). */
typedef struct or_bvh or_bvh;
or_bvh* or_bvh_build(const or_aabb* aabbs, uint32_t n);
void or_bvh_free(or_bvh* b);

/* Render rows [row_begin, row_end) of the frame. mode = OR_MODE_REF | OR_MODE_COR (| OR_FLAG_LUT).
 * sh: NULL or n*48 floats ([gauss][coef 16][rgb]). rgba: W*H*4 floats (full frame indexing).
 * raystate: W*H or NULL. stats: W*H*4 u32 {candidates, blended, rounds, terminated} or NULL.
 * bvh may be NULL (brute force). Returns 0 on success. */
int or_render(const or_gauss_param* params, const or_aabb* aabbs, const float* sh, uint32_t n,
              const or_bvh* bvh, const or_ubo* ubo, uint32_t mode, uint32_t threads,
              uint32_t row_begin, uint32_t row_end,
              float* rgba, or_raystate* raystate, uint32_t* stats);

/* or_render with triangle meshes co-traced (REF mode only): tris = ntri * 9 floats
 * (p0 p1 p2 per triangle, world space, identity instance). Per ray the closest Moller-Trumbore hit over all
 * triangles (vulkan_ray_tracing.cc:1184-1206, :925-931) sets min_thit: Gaussian boxes entered at or beyond it are
 * culled (:806-807), Gaussian reports must lie below it (instructions.cc:7050), and a round whose closest hit
 * is the triangle sets Trans = 0 (RayTracing.rchit -> Scatter.glsl). Returns -1 for COR with ntri > 0. */
int or_render_mesh(const or_gauss_param* params, const or_aabb* aabbs, const float* sh, uint32_t n,
                   const or_bvh* bvh, const float* tris, uint32_t ntri, const or_ubo* ubo, uint32_t mode,
                   uint32_t threads, uint32_t row_begin, uint32_t row_end,
                   float* rgba, or_raystate* raystate, uint32_t* stats);
/* Model::CreateSphere (RayTracingInVulkan/src/Assets/Model.cpp:566-629): 561 vertices (3 floats), 1024
 * triangles (3 u32) */
void or_sphere_mesh(const float center[3], float radius, float* vertices, uint32_t* indices);

uint32_t or_sizeof_ubo(void);
uint32_t or_sizeof_raystate(void);

#ifdef __cplusplus
}
#endif
#endif
