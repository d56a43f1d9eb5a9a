// gsrt_device.hpp -- device data layouts and per-ray arithmetic shared by the gsrt HIP kernels.
//
// All device code is compiled with -ffp-contract=off and correctly rounded f32 divide/sqrt, so every
// a*b+c below is two roundings unless written as fmaf(). The REF-mode formulas follow the reference
// GLSL left to right (RayTracing.ProceduralGauss.rint:56-117); the COR-mode formulas are this
// project's definitions ("COR flags") and are restated independently by the
// CPU oracle (oracle/gsrt_oracle.c), which the parity tests compare against bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsrt.h"

namespace gsrt {

// Every device function is inlined into its kernel: the kernels re-read their arguments through the kernarg
// segment pointer (kargs() in gsrt_render.hip), which is only defined inside a kernel, and a called function would
// also pay the call ABI (stack, saved registers). The build checks the code objects for call instructions
// (tools/check_isa.py, run by the Makefile), so a function the compiler outlines anyway fails the build.
#define GSRT_INLINE __attribute__((always_inline)) inline

constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kCounters = 32;              // per-frame counter block: [0..7] stats, [8] error, rest diagnostics
constexpr uint32_t kErrWord = 8;                // sticky error word of the counter block: not zeroed per frame, cleared
                                                // when the host reads it (gsrt_render, gsrt_synchronize)
constexpr float kGMax = 5.6f;                 // rint:102 `g > 5.6`
constexpr float kAlphaMin = 1.0f / 255.0f;    // rint:107
constexpr float kTMin = 0.001f;               // rgen:50
constexpr float kTMax = 10000.0f;             // rgen:51
constexpr float kKEmpty = 10000.0f;           // rgen:56, Scene.cpp:40
constexpr uint32_t kMeshStack = 48;           // per-lane node stack of the mesh BVH walk (k_mesh_thit)

// Per-frame splat record: one 64-B line per Gaussian, read with one wave-uniform 64-B load per
// candidate. AABB (world, static) + the view-dependent 2D projection of the frame.
// lo/hi are the world AABB minus the camera origin o (every primary ray starts at o = MV^-1 (0,0,0,1),
// GaussTracing.rgen:41), computed with the same fp32 subtraction the slab test would do per ray, so the
// per-ray test multiplies only (slab_hit_rel) and stays bit-identical to ray_box_test.
struct alignas(64) SplatRec {
    float lo[3];      // AABB min - o
    float depth;      // REF: view z (rint:67); COR: -view z
    float hi[3];      // AABB max - o
    float opacity;
    float ppx, ppy;   // projected centre in pixels (rint:71-74)
    float a, b;       // REF: V00, V01 of V = T Sigma T^T (rint:93-95); COR: conic (A, B, C) of (V + 0.3 I)
                      // stored as (A/2, B): g = fma(C/2 dy, dy, fma(B dx, dy, (A/2 dx) dx)) equals
                      // 0.5 fma(C dy, dy, fma(2B dx, dy, (A dx) dx)) (power-of-two scaling is exact)
    float c;          // REF: V11; COR: C/2
    float gcut;       // COR: max(0, min(kGMax, ln(255 opacity) + 0.01)): alpha > 1/255 needs g <= gcut (REF: 0)
                      // (next to c: the shading loop's g test reads both with one ds_read_b64)
    uint32_t valid;   // COR: depth > 0 && det > 0
    uint32_t pad1;
};
static_assert(sizeof(SplatRec) == 64, "SplatRec is one 64-B line");

// Binary LBVH node (Karras 2012), 64 B: both child boxes live in the parent so a visit tests two
// boxes and pushes only the hit children. ref: internal node index, or kLeafBit | gaussian id.
// l_key / r_key: for a leaf child, its per-frame sort key (COR: float bits of the view depth, +inf when
// the splat is invalid), written by the projection kernel, so the traversal reads a leaf's key from the
// node it already has instead of issuing a dependent load of the record.
struct alignas(64) BvhNode {
    float l_lo[3]; uint32_t l_ref;
    float l_hi[3]; uint32_t r_ref;
    float r_lo[3]; uint32_t l_key;
    float r_hi[3]; uint32_t r_key;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode is one 64-B line");

__host__ __device__ GSRT_INLINE float cm(const float* m, int c, int r) { return m[c * 4 + r]; }

// GLSL mat4 * vec4 summed left to right
__host__ __device__ GSRT_INLINE void mul4v(const float* m, const float v[4], float out[4]) {
    float r0 = ((cm(m, 0, 0) * v[0] + cm(m, 1, 0) * v[1]) + cm(m, 2, 0) * v[2]) + cm(m, 3, 0) * v[3];
    float r1 = ((cm(m, 0, 1) * v[0] + cm(m, 1, 1) * v[1]) + cm(m, 2, 1) * v[2]) + cm(m, 3, 1) * v[3];
    float r2 = ((cm(m, 0, 2) * v[0] + cm(m, 1, 2) * v[1]) + cm(m, 2, 2) * v[2]) + cm(m, 3, 2) * v[3];
    float r3 = ((cm(m, 0, 3) * v[0] + cm(m, 1, 3) * v[1]) + cm(m, 2, 3) * v[2]) + cm(m, 3, 3) * v[3];
    out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3;
}

// The view-z row of a modelview (column-major): COR depth = -(((z0 x + z1 y) + z2 z) + z3), mul4v's third row
struct ZRow { float z0, z1, z2, z3; };
__host__ __device__ GSRT_INLINE ZRow zrow_of(const float* mv) { return ZRow{cm(mv, 0, 2), cm(mv, 1, 2), cm(mv, 2, 2), cm(mv, 3, 2)}; }
// A lower bound of the COR sort-key depth (project_cor: -view z of the centre, mul4v in f32) of any centre inside the
// box [lo, hi]: minus the largest view z over the box, less 1e-6 of the magnitudes summed (mul4v's f32 sums and this
// one round at most 6 times by 2^-24 of them). Monotone in the box: each max / abs term only grows with the box and
// f32 rounding is monotone, so a box inside another gets a bound >= the other's. k_project checks every centre it
// keys against its own AABB's bound (a centre outside its AABB turns the depth cull off, RenderArgs::depth_unsafe),
// so a node box's bound is <= the depth of every key below it.
__host__ __device__ GSRT_INLINE float depth_lo(const ZRow& z, const float lo[3], const float hi[3]) {
    const float t0 = fmaxf(z.z0 * lo[0], z.z0 * hi[0]);
    const float t1 = fmaxf(z.z1 * lo[1], z.z1 * hi[1]);
    const float t2 = fmaxf(z.z2 * lo[2], z.z2 * hi[2]);
    const float u = ((t0 + t1) + t2) + z.z3;
    const float m = ((fabsf(z.z0) * fmaxf(fabsf(lo[0]), fabsf(hi[0])) + fabsf(z.z1) * fmaxf(fabsf(lo[1]), fabsf(hi[1]))) +
                     fabsf(z.z2) * fmaxf(fabsf(lo[2]), fabsf(hi[2]))) + fabsf(z.z3);
    return -u - 1e-6f * m;
}
// An internal node slot of a band-restricted fit (lbvh_fit_band) whose subtree no tile of the rank can see: an inverted
// box every frustum test rejects (each side plane's positive vertex lies ~1e30 behind it), and whose union with a real
// box is that box
constexpr float kEmptyLo = 1e30f, kEmptyHi = -1e30f;

// GaussTracing.rgen:41 -- ray origin (the same for every primary ray)
__host__ __device__ GSRT_INLINE void ray_origin(const gsrt_ubo& u, float o[3]) {
    const float o4[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    float org[4];
    mul4v(u.model_view_inverse, o4, org);
    o[0] = org[0]; o[1] = org[1]; o[2] = org[2];
}

// GaussTracing.rgen:39-43 -- origin and direction of the ray through pixel coordinate (px, py)
__device__ GSRT_INLINE void gen_ray(const gsrt_ubo& u, float px, float py, float o[3], float d[3]) {
    float uvx = (px / (float)u.width) * 2.0f - 1.0f;
    float uvy = (py / (float)u.height) * 2.0f - 1.0f;
    const float o4[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    float org[4], tg[4], dir[4];
    mul4v(u.model_view_inverse, o4, org);
    const float t4[4] = {uvx, uvy, 1.0f, 1.0f};
    mul4v(u.projection_inverse, t4, tg);
    float v0 = tg[0] * u.focus_distance, v1 = tg[1] * u.focus_distance, v2 = tg[2] * u.focus_distance;
    float len = sqrtf((v0 * v0 + v1 * v1) + v2 * v2);
    const float dv[4] = {v0 / len, v1 / len, v2 / len, 0.0f};
    mul4v(u.model_view_inverse, dv, dir);
    o[0] = org[0]; o[1] = org[1]; o[2] = org[2];
    d[0] = dir[0]; d[1] = dir[1]; d[2] = dir[2];
}

// Object-space ray of the BLAS test: identity instance transform, direction renormalised and the
// t range scaled by its norm (vulkan_ray_tracing.cc:148-160); calculate_idir (:200-215).
struct ObjRay { float idir[3]; float tmin, tmax, norm; };

__device__ GSRT_INLINE ObjRay make_obj_ray(const float d[3]) {
    ObjRay r;
    float norm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    const float ooeps = 8.27180613e-25f;  // exp2f(-80)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float dn = d[k] / norm;
        r.idir[k] = 1.0f / (fabsf(dn) > ooeps ? dn : copysignf(ooeps, dn));
    }
    r.tmin = kTMin * norm;
    r.tmax = kTMax * norm;
    r.norm = norm;
    return r;
}

// ray_box_test (vulkan_ray_tracing.cc:217-237): exact fp32 slab test. The reference's MIN/MAX macros are
// compare-selects; here they are v_min/v_max(3). Every operand is finite and never NaN (idir is clamped to
// |idir| <= 2^80, the box and origin are finite), so the two differ at most in the sign of a zero, and a
// zero's sign cannot change the final `tmin <= tmax` (tmin > 0 is always one of the max operands).
__device__ GSRT_INLINE bool slab_hit(const ObjRay& r, const float o[3], const float lo[3], const float hi[3]) {
    float l0 = (lo[0] - o[0]) * r.idir[0], h0 = (hi[0] - o[0]) * r.idir[0];
    float l1 = (lo[1] - o[1]) * r.idir[1], h1 = (hi[1] - o[1]) * r.idir[1];
    float l2 = (lo[2] - o[2]) * r.idir[2], h2 = (hi[2] - o[2]) * r.idir[2];
    float t = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(l0, h0), r.tmin),
                              __builtin_fmaxf(__builtin_fminf(l1, h1), __builtin_fminf(l2, h2)));
    float u = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(l0, h0), r.tmax),
                              __builtin_fminf(__builtin_fmaxf(l1, h1), __builtin_fmaxf(l2, h2)));
    return t <= u;
}

// slab_hit with the box already relative to the ray origin (SplatRec lo/hi): the same products, same result
__device__ GSRT_INLINE bool slab_hit_rel(const ObjRay& r, const float rlo[3], const float rhi[3]) {
    float l0 = rlo[0] * r.idir[0], h0 = rhi[0] * r.idir[0];
    float l1 = rlo[1] * r.idir[1], h1 = rhi[1] * r.idir[1];
    float l2 = rlo[2] * r.idir[2], h2 = rhi[2] * r.idir[2];
    float t = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(l0, h0), r.tmin),
                              __builtin_fmaxf(__builtin_fminf(l1, h1), __builtin_fminf(l2, h2)));
    float u = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(l0, h0), r.tmax),
                              __builtin_fminf(__builtin_fmaxf(l1, h1), __builtin_fmaxf(l2, h2)));
    return t <= u;
}

// slab_hit_rel for a REF ray after the triangles: the box also must be entered below tcut = min_thit * |d|
// (vulkan_ray_tracing.cc:806-807 culls thit >= min_thit * worldToObject_tMultiplier)
__device__ GSRT_INLINE bool slab_hit_rel_cut(const ObjRay& r, const float rlo[3], const float rhi[3], float tcut) {
    float l0 = rlo[0] * r.idir[0], h0 = rhi[0] * r.idir[0];
    float l1 = rlo[1] * r.idir[1], h1 = rhi[1] * r.idir[1];
    float l2 = rlo[2] * r.idir[2], h2 = rhi[2] * r.idir[2];
    float t = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(l0, h0), r.tmin),
                              __builtin_fmaxf(__builtin_fminf(l1, h1), __builtin_fminf(l2, h2)));
    float u = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(l0, h0), r.tmax),
                              __builtin_fminf(__builtin_fmaxf(l1, h1), __builtin_fmaxf(l2, h2)));
    return t <= u && t < tcut;
}

// slab_hit_rel for a COR record whose box lies strictly on one side of the origin on every axis (k_project
// stores it as (near, far) per axis for the rays that can reach it, and flags it by a positive opacity word):
// a ray whose direction has the matching sign on every axis gets near * idir = min(l, h) and far * idir =
// max(l, h) exactly (all products are non-zero and finite), so t and u equal ray_box_test's; any other ray
// cannot reach the box and gets u < 0 < tmin <= t, a miss, as in ray_box_test
// v_max3 / v_min3 of four values without the compiler's per-use canonicalisation (v_max x, x) of loop-invariant
// operands such as the ray's tmin / tmax: no signalling NaN ever reaches the slab test (products of finite
// record values and the ray's finite idir, or constants), so the result is fmaxf / fminf's
__device__ GSRT_INLINE float max4_nc(float a, float b, float c, float d) {
    float m, o;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
    asm("v_max_f32 %0, %1, %2" : "=v"(o) : "v"(m), "v"(d));
    return o;
}
__device__ GSRT_INLINE float min4_nc(float a, float b, float c, float d) {
    float m, o;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
    asm("v_min_f32 %0, %1, %2" : "=v"(o) : "v"(m), "v"(d));
    return o;
}
__device__ GSRT_INLINE bool slab_hit_ordered(const ObjRay& r, const float nr[3], const float fr[3]) {
    const float t = max4_nc(nr[0] * r.idir[0], nr[1] * r.idir[1], nr[2] * r.idir[2], r.tmin);
    const float u = min4_nc(fr[0] * r.idir[0], fr[1] * r.idir[1], fr[2] * r.idir[2], r.tmax);
    return t <= u;
}

// LinearExp (rint:45-54) over the 256-segment LUT (ExpLUT.hpp:10-24); 0 <= x <= 5.6
__device__ GSRT_INLINE float linear_exp(const float* lut, float x) {
    float tx = x * 32.0f;
    uint32_t qx = (uint32_t)tx;
    float dqx = (float)qx / 32.0f;
    float dx = x - dqx;
    return lut[2 * qx] * dx + lut[2 * qx + 1];
}

// COR exponential for x <= 0 from IEEE-exact operations only (rint, fma, ldexp), so the CPU oracle
// reproduces it bit for bit: reduction by one fp32 ln2 (n <= 8 on the shading range, so n (ln2 - ln2_f32) stays
// below 2e-8) and a degree-5 polynomial with near-minimax coefficients (Lawson-weighted least squares on
// [-ln2/2, ln2/2], relative error 9e-8 before rounding). Measured over every float in [-5.6, 0] (g <= 5.6, the
// shading range): at most 2.0 ulp from exp; over [-87, 0]: 4.8 ulp.
// exp_neg for x >= -87 (no underflow branch: the same arithmetic, so the same result there)
__device__ GSRT_INLINE float exp_neg_nocheck(float x) {
    float n = rintf(x * 1.44269504088896341f);
    float r = fmaf(-n, 0.693147182464599609375f, x);
    float p = fmaf(r, 8.290272206e-03f, 4.189816117e-02f);
    p = fmaf(r, p, 1.666763872e-01f);
    p = fmaf(r, p, 4.999914765e-01f);
    p = fmaf(r, p, 9.999997020e-01f);
    p = fmaf(r, p, 1.0f);
    return ldexpf(p, (int)n);
}
__device__ GSRT_INLINE float exp_neg(float x) {
    if (x < -87.0f) return 0.0f;
    return exp_neg_nocheck(x);
}

// 3DGS real spherical-harmonics basis (degree 3) at the world ray direction; bs[0] = kShY0 is constant (the
// DC term is folded into the stored coefficients, see gsrt_api.cpp upload_common)
constexpr float kShY0 = 0.28209479177387814f;
__device__ GSRT_INLINE void sh_basis(const float d[3], float bs[16]) {
    float x = d[0], y = d[1], z = d[2];
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    bs[0] = kShY0;
    bs[1] = -0.4886025119029199f * y;
    bs[2] = 0.4886025119029199f * z;
    bs[3] = -0.4886025119029199f * x;
    bs[4] = 1.0925484305920792f * xy;
    bs[5] = -1.0925484305920792f * yz;
    bs[6] = 0.31539156525252005f * ((2.0f * zz - xx) - yy);
    bs[7] = -1.0925484305920792f * xz;
    bs[8] = 0.5462742152960396f * (xx - yy);
    bs[9] = (-0.5900435899266435f * y) * (3.0f * xx - yy);
    bs[10] = (2.890611442640554f * xy) * z;
    bs[11] = (-0.4570457994644658f * y) * ((4.0f * zz - xx) - yy);
    bs[12] = (0.3731763325901154f * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
    bs[13] = (-0.4570457994644658f * x) * ((4.0f * zz - xx) - yy);
    bs[14] = (1.445305721320277f * z) * (xx - yy);
    bs[15] = (-0.5900435899266435f * x) * (xx - 3.0f * yy);
}

// ---- tile order -------------------------------------------------------------------------------
// Spatial order of a grid of tiles: super-tiles of kSuper x kSuper tiles, row-major over super-tiles and row-major
// inside each (edge super-tiles are partial). A rank's tiles (its band, below) are numbered in this order over the
// band's own grid; inside a rank, xcd_local_tile() hands the workgroups of one XCD runs of kRun consecutive tiles.
// The mapping is a bijection whatever the dispatcher does; placement only changes the cache hit rate.
constexpr uint32_t kSuper = 16;
constexpr uint32_t kRun = kSuper * kSuper;

__host__ __device__ GSRT_INLINE void spatial_tile(uint32_t k, uint32_t tiles_x, uint32_t tiles_y, uint32_t& tx,
                                             uint32_t& ty) {
    const uint32_t R = k / (kSuper * tiles_x);
    const uint32_t hR = tiles_y - R * kSuper < kSuper ? tiles_y - R * kSuper : kSuper;
    const uint32_t k1 = k - R * kSuper * tiles_x;
    const uint32_t C = k1 / (hR * kSuper);
    const uint32_t wC = tiles_x - C * kSuper < kSuper ? tiles_x - C * kSuper : kSuper;
    const uint32_t k2 = k1 - C * hR * kSuper;
    ty = R * kSuper + k2 / wC;
    tx = C * kSuper + k2 % wC;
}

__host__ __device__ GSRT_INLINE uint32_t spatial_index(uint32_t tx, uint32_t ty, uint32_t tiles_x, uint32_t tiles_y) {
    const uint32_t R = ty / kSuper, C = tx / kSuper;
    const uint32_t hR = tiles_y - R * kSuper < kSuper ? tiles_y - R * kSuper : kSuper;
    const uint32_t wC = tiles_x - C * kSuper < kSuper ? tiles_x - C * kSuper : kSuper;
    return R * kSuper * tiles_x + C * hR * kSuper + (ty - R * kSuper) * wC + (tx - C * kSuper);
}

// The partition of a sharded frame: contiguous bands of whole tile rows, rank r owning rows
// [bands[r], bands[r + 1]) of every column. The boundaries balance the ranks' measured shading cost (gsrt_comm.cpp:
// per-row costs of an earlier frame, all-reduced over the ranks); rank 0, the gather's root, gets a lighter weight.
// A rank's local tile lt is tile spatial_tile(lt) of its band's own tiles_x x (row1 - row0) grid, rows offset by
// row0; k_unpack inverts it (band_of). One rank: a single band of every row.
constexpr uint32_t kMaxRanks = 64;
struct Bands {
    uint32_t n;                     // ranks
    uint32_t row[kMaxRanks + 1];    // boundaries: row[0] = 0 <= row[1] <= ... <= row[n] = tiles_y
};
__host__ __device__ GSRT_INLINE uint32_t band_of(const Bands& b, uint32_t ty) {
    uint32_t r = 0;
    while (r + 1 < b.n && ty >= b.row[r + 1]) ++r;
    return r;
}
// local tile lt of the band [row0, row1) of a frame tiles_x wide -> tile (tx, ty)
__host__ __device__ GSRT_INLINE void band_tile(uint32_t lt, uint32_t row0, uint32_t row1, uint32_t tiles_x, uint32_t& tx,
                                          uint32_t& ty) {
    spatial_tile(lt, tiles_x, row1 - row0, tx, ty);
    ty += row0;
}
__host__ __device__ GSRT_INLINE uint32_t band_index(uint32_t tx, uint32_t ty, uint32_t row0, uint32_t row1,
                                               uint32_t tiles_x) {
    return spatial_index(tx, ty - row0, tiles_x, row1 - row0);
}

// Multi-GPU: the pixel rows of this rank's band. The projection and the BVH frontier skip work none of its tiles
// needs: a splat whose pixel box misses the band (or the frame) is not projected for this rank.
struct RankTiles {
    uint32_t active;            // 0: every tile is this rank's (one rank)
    float y0, y1;               // the band's sample rows [y0, y1) in pixels (row0 * th, row1 * th)
    float width;                // frame width in pixels
};
// may a tile of the rank see the pixel box [x0, x1] x [y0, y1]? Conservative by one pixel on every side (the
// footprint boxes carry their own rounding margins; a wrong "yes" only costs work)
__host__ __device__ GSRT_INLINE bool rank_owns_box(float x0, float x1, float y0, float y1, const RankTiles& o) {
    if (!o.active) return true;
    if (!(x0 <= x1 && y0 <= y1)) return false;  // empty box (and NaN): the splat reaches no pixel
    return y1 >= o.y0 - 1.0f && y0 <= o.y1 + 1.0f && x1 >= -1.0f && x0 <= o.width + 1.0f;
}

// GSRT_FLAG_OUT_DUMP8: a pixel as the integers the frame dump prints (gsrt_dump_ppm, vulkan_ray_tracing.cc:2245-2246:
// "%3.0f" of channel * 255 for r, g, b): 10 bits per channel, the value rint(v * 255) (round half to even, as printf
// rounds the float's exact value) when it is a finite non-negative number (not -0) of at most 1022; otherwise the
// pixel carries kDump8Escape and its exact channel values travel in an escape list. 4 bytes per pixel instead of
// RGBA32F's 16, and the dump of the codes is byte-identical to the dump of the floats.
constexpr uint32_t kDump8Escape = 1u << 30;
constexpr uint32_t kDump8Max = 1022u;
__host__ __device__ GSRT_INLINE uint32_t dump8_code(const float4 v) {
    const float ch[3] = {v.x, v.y, v.z};
    uint32_t code = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float x = ch[k] * 255.0f;  // the dump's own float product
        const float c = rintf(x);
        if (!(x >= 0.0f) || (__builtin_bit_cast(uint32_t, x) >> 31) || c > (float)kDump8Max) return kDump8Escape;
        code |= (uint32_t)c << (10 * k);
    }
    return code;
}

// Random.glsl:24-37 -- LCG + 24-bit float (host side builds the per-sample jitter table)
__host__ __device__ GSRT_INLINE float random_float(uint32_t* seed) {
    *seed = 1664525u * *seed + 1013904223u;
    return (float)(*seed & 0x00FFFFFFu) / (float)0x01000000;
}

}  // namespace gsrt
