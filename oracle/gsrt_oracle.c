/*
 * gsrt_oracle.c -- CPU restatement of the reference's ray-traced 3DGS hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gsrt_oracle.h). Built by oracle/Makefile into
 * oracle/_build/libgsrt_oracle.so; loaded by tests/, smoke() and bench.py's
 * cpu_baseline leg, never by the product.
 *
 * Compiled with -ffp-contract=off: every a*b+c below is two roundings unless the
 * code calls fmaf() explicitly. The REF-mode arithmetic follows the GLSL source
 * left to right (the reference's PTX contraction is unknown: SURVEY.md §8c).
 *
 * Reference files restated (paths relative to /root/reference):
 *   RayTracingInVulkan/assets/shaders/GaussTracing.rgen:22-76            (raygen, round loop)
 *   RayTracingInVulkan/assets/shaders/RayTracing.ProceduralGauss.rint:24-117 (EWA, LinearExp, K=8 insert)
 *   RayTracingInVulkan/assets/shaders/RayTracing.ProceduralGauss.rchit:15-33 (transmittance, depth advance)
 *   RayTracingInVulkan/src/Utilities/ExpLUT.hpp:10-24, src/Assets/Scene.cpp:38-47
 *   RayTracingInVulkan/src/Assets/Sphere.hpp:108-165                       (cov3d, radius, AABB)
 *   RayTracingInVulkan/src/RayTracer.cpp:38-65, src/ModelViewController.cpp:4-34 (camera UBO)
 *   vulkan-sim/src/cuda-sim/vulkan_ray_tracing.cc:148-237                   (object ray, slab test)
 *   vulkan-sim/src/cuda-sim/instructions.cc:7018-7082                       (report rule)
 *   RayTracingInVulkan/assets/shaders/Random.glsl:7-37                      (COR spp jitter)
 *
 * Pinning. The reference ships no test, fixture or golden output for this path, and it cannot be
 * built or run here (Embree runtime and lavapipe binaries missing, no Vulkan SDK/glslang, meson or
 * CUDA: SURVEY.md §8c), so there is no oracle/_ref. REF mode is pinned by KAT-1, the known answer
 * for scene 33 derived by hand from the reference shaders (pixel (8,8): Trans 0.100000024, Depth 1;
 * every other pixel Trans 1, Depth 0; image all zeros; tests/test_oracle.py). Beyond KAT-1 the REF
 * restatement is unpinned by reference outputs. COR mode is this project's definition (the reference
 * has no colour path): parity unpinned against the reference by construction; the GPU is held
 * bit-exact to this file.
 */
#include "gsrt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define CM(m, c, r) ((m)[(c) * 4 + (r)]) /* glm column-major: m[col][row] */

uint32_t or_sizeof_ubo(void) { return (uint32_t)sizeof(or_ubo); }
uint32_t or_sizeof_raystate(void) { return (uint32_t)sizeof(or_raystate); }

/* ------------------------------------------------------------------ glm restatements */

/* glm::perspectiveRH_ZO (GLM_FORCE_DEPTH_ZERO_TO_ONE + GLM_FORCE_RIGHT_HANDED, Utilities/Glm.hpp:3-4) */
void or_perspective_rh_zo(float fovy, float aspect, float zn, float zf, float out[16]) {
    memset(out, 0, 16 * sizeof(float));
    float tan_half = tanf(fovy / 2.0f);
    CM(out, 0, 0) = 1.0f / (aspect * tan_half);
    CM(out, 1, 1) = 1.0f / tan_half;
    CM(out, 2, 2) = zf / (zn - zf);
    CM(out, 2, 3) = -1.0f;
    CM(out, 3, 2) = -(zf * zn) / (zf - zn);
}

/* glm mat4 * mat4: Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3] */
void or_mul4(const float a[16], const float b[16], float out[16]) {
    float r[16];
    for (int c = 0; c < 4; ++c)
        for (int i = 0; i < 4; ++i)
            r[c * 4 + i] = ((CM(a, 0, i) * CM(b, c, 0) + CM(a, 1, i) * CM(b, c, 1)) + CM(a, 2, i) * CM(b, c, 2)) +
                           CM(a, 3, i) * CM(b, c, 3);
    memcpy(out, r, sizeof r);
}

/* glm mat4 * vec4 (non-SIMD detail/type_mat4x4.inl): (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
static void mul4v_glm(const float m[16], const float v[4], float out[4]) {
    float r[4];
    for (int i = 0; i < 4; ++i)
        r[i] = (CM(m, 0, i) * v[0] + CM(m, 1, i) * v[1]) + (CM(m, 2, i) * v[2] + CM(m, 3, i) * v[3]);
    memcpy(out, r, sizeof r);
}

/* glm::inverse for mat4 (detail/func_matrix.inl compute_inverse<4,4>) */
void or_inverse4(const float m[16], float out[16]) {
#define Mx(c, r) CM(m, c, r)
    float c00 = Mx(2, 2) * Mx(3, 3) - Mx(3, 2) * Mx(2, 3);
    float c02 = Mx(1, 2) * Mx(3, 3) - Mx(3, 2) * Mx(1, 3);
    float c03 = Mx(1, 2) * Mx(2, 3) - Mx(2, 2) * Mx(1, 3);
    float c04 = Mx(2, 1) * Mx(3, 3) - Mx(3, 1) * Mx(2, 3);
    float c06 = Mx(1, 1) * Mx(3, 3) - Mx(3, 1) * Mx(1, 3);
    float c07 = Mx(1, 1) * Mx(2, 3) - Mx(2, 1) * Mx(1, 3);
    float c08 = Mx(2, 1) * Mx(3, 2) - Mx(3, 1) * Mx(2, 2);
    float c10 = Mx(1, 1) * Mx(3, 2) - Mx(3, 1) * Mx(1, 2);
    float c11 = Mx(1, 1) * Mx(2, 2) - Mx(2, 1) * Mx(1, 2);
    float c12 = Mx(2, 0) * Mx(3, 3) - Mx(3, 0) * Mx(2, 3);
    float c14 = Mx(1, 0) * Mx(3, 3) - Mx(3, 0) * Mx(1, 3);
    float c15 = Mx(1, 0) * Mx(2, 3) - Mx(2, 0) * Mx(1, 3);
    float c16 = Mx(2, 0) * Mx(3, 2) - Mx(3, 0) * Mx(2, 2);
    float c18 = Mx(1, 0) * Mx(3, 2) - Mx(3, 0) * Mx(1, 2);
    float c19 = Mx(1, 0) * Mx(2, 2) - Mx(2, 0) * Mx(1, 2);
    float c20 = Mx(2, 0) * Mx(3, 1) - Mx(3, 0) * Mx(2, 1);
    float c22 = Mx(1, 0) * Mx(3, 1) - Mx(3, 0) * Mx(1, 1);
    float c23 = Mx(1, 0) * Mx(2, 1) - Mx(2, 0) * Mx(1, 1);
    float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    float v0[4] = {Mx(1, 0), Mx(0, 0), Mx(0, 0), Mx(0, 0)};
    float v1[4] = {Mx(1, 1), Mx(0, 1), Mx(0, 1), Mx(0, 1)};
    float v2[4] = {Mx(1, 2), Mx(0, 2), Mx(0, 2), Mx(0, 2)};
    float v3[4] = {Mx(1, 3), Mx(0, 3), Mx(0, 3), Mx(0, 3)};
    float inv[16];
    const float sa[4] = {+1, -1, +1, -1}, sb[4] = {-1, +1, -1, +1};
    for (int i = 0; i < 4; ++i) {
        inv[0 * 4 + i] = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3[i] * f2[i]) * sa[i];
        inv[1 * 4 + i] = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3[i] * f4[i]) * sb[i];
        inv[2 * 4 + i] = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3[i] * f5[i]) * sa[i];
        inv[3 * 4 + i] = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb[i];
    }
    float row0[4] = {inv[0], inv[4], inv[8], inv[12]};
    float d0[4];
    for (int i = 0; i < 4; ++i) d0[i] = Mx(0, i) * row0[i];
    float d1 = (d0[0] + d0[1]) + (d0[2] + d0[3]);
    float one_over = 1.0f / d1;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * one_over;
#undef Mx
}

static float dot3_glm(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static void cross3(const float x[3], const float y[3], float o[3]) {
    float r0 = x[1] * y[2] - y[1] * x[2], r1 = x[2] * y[0] - y[2] * x[0], r2 = x[0] * y[1] - y[0] * x[1];
    o[0] = r0; o[1] = r1; o[2] = r2;
}
static void normalize3_glm(float v[3]) { /* v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt */
    float is = 1.0f / sqrtf(dot3_glm(v, v));
    v[0] *= is; v[1] *= is; v[2] *= is;
}

/* glm::lookAtRH (SceneList.cpp:705-712 applies it to .camera files) */
void or_lookat_rh(const float eye[3], const float center[3], const float up[3], float out[16]) {
    float f[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
    normalize3_glm(f);
    float s[3]; cross3(f, up, s); normalize3_glm(s);
    float u[3]; cross3(s, f, u);
    memset(out, 0, 16 * sizeof(float));
    CM(out, 0, 0) = s[0]; CM(out, 1, 0) = s[1]; CM(out, 2, 0) = s[2];
    CM(out, 0, 1) = u[0]; CM(out, 1, 1) = u[1]; CM(out, 2, 1) = u[2];
    CM(out, 0, 2) = -f[0]; CM(out, 1, 2) = -f[1]; CM(out, 2, 2) = -f[2];
    CM(out, 3, 0) = -dot3_glm(s, eye);
    CM(out, 3, 1) = -dot3_glm(u, eye);
    CM(out, 3, 2) = dot3_glm(f, eye);
    CM(out, 3, 3) = 1.0f;
}

void or_make_ubo(const float init_mv[16], float fovy_deg, uint32_t width, uint32_t height, float focus_distance,
                 uint32_t samples, uint32_t bounces, or_ubo* u) {
    memset(u, 0, sizeof *u);
    /* ModelViewController::Reset: position = inverse(mv)*(0,0,0,1); orientation = mat4(mat3(mv)) */
    float inv[16], pos[4];
    const float o4[4] = {0, 0, 0, 1};
    or_inverse4(init_mv, inv);
    mul4v_glm(inv, o4, pos);
    float orient[16];
    memset(orient, 0, sizeof orient);
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) CM(orient, c, r) = CM(init_mv, c, r);
    CM(orient, 3, 3) = 1.0f;
    /* ModelView(): orientation * translate(I, -position) * model(identity at rest) */
    float tr[16];
    memset(tr, 0, sizeof tr);
    tr[0] = tr[5] = tr[10] = tr[15] = 1.0f;
    CM(tr, 3, 0) = -pos[0]; CM(tr, 3, 1) = -pos[1]; CM(tr, 3, 2) = -pos[2];
    or_mul4(orient, tr, u->model_view);
    /* glm::radians: degrees * 0.01745329251994329576923690768489 (as float) */
    float fovy = fovy_deg * 0.01745329251994329576923690768489f;
    or_perspective_rh_zo(fovy, (float)width / (float)height, 0.1f, 10000.0f, u->projection);
    CM(u->projection, 1, 1) *= -1.0f;
    or_inverse4(u->model_view, u->model_view_inverse);
    or_inverse4(u->projection, u->projection_inverse);
    u->focus_distance = focus_distance;
    u->total_samples = samples;
    u->samples = samples;
    u->bounces = bounces;
    u->random_seed = 1; /* RayTracer.cpp:59 */
    u->width = width;
    u->height = height;
    u->has_sky = 1;
}

/* ------------------------------------------------------------------ scene assets */

void or_gauss_from_model(uint32_t n, const float* center, const float* rot, const float* scale, const float* opacity,
                         or_gauss_param* out, or_aabb* aabb) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* C = center + 3 * i;
        const float* Q = rot + 4 * i;
        const float* S = scale + 3 * i;
        float r = Q[0], x = Q[1], y = Q[2], z = Q[3];
        /* glm::mat3 R(...) column-major constructor (Sphere.hpp:143-147): R[c][r] */
        float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                      2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                      2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)};
        float Sm[9] = {S[0], 0, 0, 0, S[1], 0, 0, 0, S[2]};
        /* M = S * R (glm mat3 mul: Result[c][i] = (A[0][i]*B[c][0] + A[1][i]*B[c][1]) + A[2][i]*B[c][2]) */
        float M[9], Mt[9], Sig[9];
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k)
                M[c * 3 + k] = (Sm[0 * 3 + k] * R[c * 3 + 0] + Sm[1 * 3 + k] * R[c * 3 + 1]) + Sm[2 * 3 + k] * R[c * 3 + 2];
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k) Mt[c * 3 + k] = M[k * 3 + c];
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k)
                Sig[c * 3 + k] = (Mt[0 * 3 + k] * M[c * 3 + 0] + Mt[1 * 3 + k] * M[c * 3 + 1]) + Mt[2 * 3 + k] * M[c * 3 + 2];
        or_gauss_param* g = out + i;
        memset(g, 0, sizeof *g);
        g->center_opacity[0] = C[0]; g->center_opacity[1] = C[1]; g->center_opacity[2] = C[2];
        g->center_opacity[3] = opacity[i];
        g->cov3d[0] = Sig[0 * 3 + 0]; g->cov3d[1] = Sig[0 * 3 + 1]; g->cov3d[2] = Sig[0 * 3 + 2];
        g->cov3d[3] = Sig[1 * 3 + 1]; g->cov3d[4] = Sig[1 * 3 + 2]; g->cov3d[5] = Sig[2 * 3 + 2];
        /* Radius = 3.0 * max(scale) in double, stored float (Sphere.hpp:164) */
        float mx = S[0];
        if (S[1] > mx) mx = S[1];
        if (S[2] > mx) mx = S[2];
        float rad = (float)(3.0 * (double)mx);
        for (int a = 0; a < 3; ++a) { aabb[i].lo[a] = C[a] - rad; aabb[i].hi[a] = C[a] + rad; }
    }
}

void or_exp_lut(float out[512]) {
    float step = (8.0f - 0.0f) / 256; /* ExpLUT.hpp:12 */
    for (int i = 0; i < 256; ++i) {
        float x = 0.0f + i * step;
        out[2 * i] = -expf(-x);
        out[2 * i + 1] = expf(-x);
    }
}

float or_linear_exp(const float* lut, float x) {
    float tx = x * 32;
    uint32_t qx = (uint32_t)tx; /* callers guarantee 0 <= x <= 5.6 */
    float dqx = (float)qx / 32.0f;
    float dx = x - dqx;
    float k = lut[2 * qx], b = lut[2 * qx + 1];
    return k * dx + b;
}

float or_exp_neg(float x) {
    if (x < -87.0f) return 0.0f;
    float n = rintf(x * 1.44269504088896341f);
    float r = fmaf(-n, 0.693147182464599609375f, x);
    float p = fmaf(r, 8.290272206e-03f, 4.189816117e-02f);
    p = fmaf(r, p, 1.666763872e-01f);
    p = fmaf(r, p, 4.999914765e-01f);
    p = fmaf(r, p, 9.999997020e-01f);
    p = fmaf(r, p, 1.0f);
    return ldexpf(p, (int)n);
}

/* ------------------------------------------------------------------ synthetic clouds */

typedef struct { uint32_t mt[624]; int idx; } mt19937;
static void mt_seed(mt19937* g, uint32_t s) {
    g->mt[0] = s;
    for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}
static uint32_t mt_next(mt19937* g) {
    if (g->idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
            g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        g->idx = 0;
    }
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
/* libstdc++ uniform_real_distribution<float>: generate_canonical<float,24> * (b-a) + a */
static float mt_uniform(mt19937* g, float a, float b) {
    float sum = (float)mt_next(g) * 1.0f;
    float ret = sum / 4294967296.0f;
    if (ret >= 1.0f) ret = nextafterf(1.0f, 0.0f);
    return ret * (b - a) + a;
}

void or_synth_cloud(uint32_t kind, uint32_t n, uint32_t seed, int with_sh, float* center, float* rot, float* scale,
                    float* opacity, float* sh) {
    mt19937 g;
    mt_seed(&g, seed);
    float sigma0 = 0.0107f * sqrtf(1e6f / (float)n);
    for (uint32_t i = 0; i < n; ++i) {
        float* C = center + 3 * i;
        float* Q = rot + 4 * i;
        float* S = scale + 3 * i;
        if (kind == OR_SYNTH_NEEDLE) {
            C[0] = mt_uniform(&g, -0.05f, 0.05f);
            C[1] = mt_uniform(&g, -0.05f, 0.05f);
            C[2] = mt_uniform(&g, 0.05f, 1.0f);
            S[0] = mt_uniform(&g, 0.0005f, 0.002f);
            S[1] = mt_uniform(&g, 0.0005f, 0.002f);
            S[2] = mt_uniform(&g, 0.4f, 1.0f);
            Q[0] = 1.0f; Q[1] = Q[2] = Q[3] = 0.0f;
        } else {
            C[0] = mt_uniform(&g, -4.0f, 4.0f);
            C[1] = mt_uniform(&g, -4.0f, 4.0f);
            C[2] = kind == OR_SYNTH_REF ? mt_uniform(&g, -4.0f, 4.0f) : mt_uniform(&g, -12.0f, -4.0f);
            for (int a = 0; a < 3; ++a) S[a] = sigma0 * expf(mt_uniform(&g, -0.5f, 0.5f));
            float q[4], qq = 0.0f;
            for (int a = 0; a < 4; ++a) { q[a] = mt_uniform(&g, -1.0f, 1.0f); qq += q[a] * q[a]; }
            float inv = 1.0f / sqrtf(qq);
            for (int a = 0; a < 4; ++a) Q[a] = q[a] * inv;
        }
        opacity[i] = mt_uniform(&g, 0.05f, 0.95f);
        if (with_sh) {
            float* s = sh + 48 * (size_t)i;
            for (int k = 0; k < 16; ++k)
                for (int c = 0; c < 3; ++c) {
                    float u = mt_uniform(&g, 0.0f, 1.0f);
                    s[k * 3 + c] = k == 0 ? u - 0.5f : 0.2f * (u - 0.5f);
                }
        }
    }
}

/* ------------------------------------------------------------------ CPU BVH (candidate enumeration only) */

struct or_bvh {
    uint32_t n, nnodes;
    float* box;      /* nnodes * 6 */
    uint32_t* info;  /* nnodes * 2: internal {left, right}; leaf {0x80000000|first, count} */
    uint32_t* ids;
};
typedef struct { const or_aabb* a; float* cen; uint32_t* ids; or_bvh* b; } bvh_build_ctx;

static int cmp_axis;
static const float* cmp_cen;
static int cmp_ids(const void* x, const void* y) {
    float a = cmp_cen[3 * *(const uint32_t*)x + cmp_axis], b = cmp_cen[3 * *(const uint32_t*)y + cmp_axis];
    if (a < b) return -1;
    if (a > b) return 1;
    return (*(const uint32_t*)x < *(const uint32_t*)y) ? -1 : (*(const uint32_t*)x > *(const uint32_t*)y);
}
/* partial order ids[0..n): ids[0..k) hold the k smallest keys (cmp_ids), ids[k..n) the rest */
static void select_kth(uint32_t* ids, uint32_t n, uint32_t k) {
    uint32_t lo = 0, hi = n;  /* the k-th smallest lies in [lo, hi) */
    while (hi - lo > 16) {
        uint32_t m = lo + (hi - lo) / 2;
        /* median of three as the pivot, moved to hi - 1 */
        uint32_t a = lo, b = m, c = hi - 1, t;
        if (cmp_ids(&ids[b], &ids[a]) < 0) { t = a; a = b; b = t; }
        if (cmp_ids(&ids[c], &ids[b]) < 0) { t = b; b = c; c = t; if (cmp_ids(&ids[b], &ids[a]) < 0) { t = a; a = b; b = t; } }
        t = ids[b]; ids[b] = ids[hi - 1]; ids[hi - 1] = t;
        const uint32_t piv = ids[hi - 1];
        uint32_t st = lo;
        for (uint32_t i = lo; i < hi - 1; ++i)
            if (cmp_ids(&ids[i], &piv) < 0) { t = ids[i]; ids[i] = ids[st]; ids[st] = t; ++st; }
        t = ids[st]; ids[st] = ids[hi - 1]; ids[hi - 1] = t;  /* pivot at its final rank st */
        if (st == k) return;
        if (st < k) lo = st + 1; else hi = st;
    }
    if (hi > lo) qsort(ids + lo, hi - lo, sizeof(uint32_t), cmp_ids);
}

static uint32_t bvh_rec(bvh_build_ctx* c, uint32_t first, uint32_t count) {
    uint32_t node = c->b->nnodes++;
    float* bx = c->b->box + 6 * node;
    bx[0] = bx[1] = bx[2] = INFINITY;
    bx[3] = bx[4] = bx[5] = -INFINITY;
    float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = first; i < first + count; ++i) {
        const or_aabb* a = c->a + c->ids[i];
        for (int k = 0; k < 3; ++k) {
            if (a->lo[k] < bx[k]) bx[k] = a->lo[k];
            if (a->hi[k] > bx[3 + k]) bx[3 + k] = a->hi[k];
            float ce = c->cen[3 * c->ids[i] + k];
            if (ce < cl[k]) cl[k] = ce;
            if (ce > ch[k]) ch[k] = ce;
        }
    }
    if (count <= 4) {
        c->b->info[2 * node] = 0x80000000u | first;
        c->b->info[2 * node + 1] = count;
        return node;
    }
    int axis = 0;
    for (int k = 1; k < 3; ++k)
        if (ch[k] - cl[k] > ch[axis] - cl[axis]) axis = k;
    cmp_axis = axis;
    cmp_cen = c->cen;
    uint32_t half = count / 2;
    /* median split: the `half` smallest (centroid, id) keys go left. Only the sets matter (candidates are
     * sorted after collection), so a quickselect replaces the full sort (O(N log N) build) */
    select_kth(c->ids + first, count, half);
    uint32_t l = bvh_rec(c, first, half);
    uint32_t r = bvh_rec(c, first + half, count - half);
    c->b->info[2 * node] = l;
    c->b->info[2 * node + 1] = r;
    return node;
}

or_bvh* or_bvh_build(const or_aabb* aabbs, uint32_t n) {
    or_bvh* b = (or_bvh*)calloc(1, sizeof *b);
    b->n = n;
    uint32_t maxn = n ? 2 * n : 1;
    b->box = (float*)malloc(sizeof(float) * 6 * maxn);
    b->info = (uint32_t*)malloc(sizeof(uint32_t) * 2 * maxn);
    b->ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    float* cen = (float*)malloc(sizeof(float) * 3 * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) {
        b->ids[i] = i;
        for (int k = 0; k < 3; ++k) cen[3 * i + k] = 0.5f * (aabbs[i].lo[k] + aabbs[i].hi[k]);
    }
    if (n) {
        bvh_build_ctx c = {aabbs, cen, b->ids, b};
        bvh_rec(&c, 0, n);
    }
    free(cen);
    return b;
}
void or_bvh_free(or_bvh* b) {
    if (!b) return;
    free(b->box); free(b->info); free(b->ids); free(b);
}

/* ------------------------------------------------------------------ per-ray semantics */

typedef struct { float o[3], idir[3], tmin, tmax, dn[3], norm; } obj_ray;

/* VulkanRayTracing::make_transformed_ray with the identity instance transform (Application.cpp:361-362):
 * direction renormalised, t range scaled by the norm (vulkan_ray_tracing.cc:128-160); calculate_idir (:200-215) */
static void make_obj_ray(const float o[3], const float d[3], obj_ray* r) {
    float norm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    const float ooeps = 8.27180613e-25f; /* exp2f(-80) */
    for (int k = 0; k < 3; ++k) {
        float dn = d[k] / norm;
        r->o[k] = o[k];
        r->dn[k] = dn;
        r->idir[k] = 1.0f / (fabsf(dn) > ooeps ? dn : copysignf(ooeps, dn));
    }
    r->tmin = 0.001f * norm;
    r->tmax = 10000.0f * norm;
    r->norm = norm;
}

/* VulkanRayTracing::mt_ray_triangle_test (vulkan_ray_tracing.cc:1184-1206) on the object ray, with
 * vector-math.cc's operator-, cross and dot (:13-50); returns 1 and the object-space t on a hit */
static int mt_ray_triangle(const float* p /* p0 p1 p2 */, const obj_ray* r, float* thit) {
    float v0v1[3], v0v2[3], pvec[3], tvec[3], qvec[3];
    for (int k = 0; k < 3; ++k) {
        v0v1[k] = p[3 + k] - p[k];
        v0v2[k] = p[6 + k] - p[k];
    }
    const float* d = r->dn;
    pvec[0] = d[1] * v0v2[2] - d[2] * v0v2[1];
    pvec[1] = d[2] * v0v2[0] - d[0] * v0v2[2];
    pvec[2] = d[0] * v0v2[1] - d[1] * v0v2[0];
    float det = v0v1[0] * pvec[0] + v0v1[1] * pvec[1] + v0v1[2] * pvec[2];
    float idet = 1 / det;
    for (int k = 0; k < 3; ++k) tvec[k] = r->o[k] - p[k];
    float u = (tvec[0] * pvec[0] + tvec[1] * pvec[1] + tvec[2] * pvec[2]) * idet;
    if (u < 0 || u > 1) return 0;
    qvec[0] = tvec[1] * v0v1[2] - tvec[2] * v0v1[1];
    qvec[1] = tvec[2] * v0v1[0] - tvec[0] * v0v1[2];
    qvec[2] = tvec[0] * v0v1[1] - tvec[1] * v0v1[0];
    float v = (d[0] * qvec[0] + d[1] * qvec[1] + d[2] * qvec[2]) * idet;
    if (v < 0 || (u + v) > 1) return 0;
    *thit = (v0v2[0] * qvec[0] + v0v2[1] * qvec[1] + v0v2[2] * qvec[2]) * idet;
    return 1;
}

/* the triangle part of traceRay for one ray: min_thit starts at Tmax (:534) and keeps the smallest world t with
 * Tmin <= t <= Tmax (:925-931); the minimum over all triangles is what any visiting order leaves */
static float closest_triangle(const float* tris, uint32_t ntri, const obj_ray* r) {
    float min_thit = 10000.0f;
    for (uint32_t i = 0; i < ntri; ++i) {
        float t;
        if (!mt_ray_triangle(tris + 9ull * i, r, &t)) continue;
        float w = t / r->norm;
        if (0.001f <= w && w <= 10000.0f && w < min_thit) min_thit = w;
    }
    return min_thit;
}
#define VS_MAX(a, b) (((a) > (b)) ? (a) : (b))
#define VS_MIN(a, b) (((a) < (b)) ? (a) : (b))
/* ray_box_test (vulkan_ray_tracing.cc:217-237) with get_t_bound (:179-195) and magic_max7/min7 (:163-177);
 * *thit = the entry t (the `min` the caller compares with min_thit, :806-807) */
static int slab_hit_t(const obj_ray* r, const or_aabb* a, float* thit) {
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = (a->lo[k] - r->o[k]) * r->idir[k];
        hi[k] = (a->hi[k] - r->o[k]) * r->idir[k];
    }
    float t1 = VS_MAX(VS_MIN(lo[0], hi[0]), r->tmin);
    float t2 = VS_MAX(VS_MIN(lo[1], hi[1]), t1);
    float t3 = VS_MAX(VS_MIN(lo[2], hi[2]), t2);
    float u1 = VS_MIN(VS_MAX(lo[0], hi[0]), r->tmax);
    float u2 = VS_MIN(VS_MAX(lo[1], hi[1]), u1);
    float u3 = VS_MIN(VS_MAX(lo[2], hi[2]), u2);
    *thit = t3;
    return t3 <= u3;
}
static int slab_hit(const obj_ray* r, const or_aabb* a) {
    float t;
    return slab_hit_t(r, a, &t);
}

/* GLSL mat4 * vec4, summed left to right */
static void mul4v(const float m[16], const float v[4], float out[4]) {
    float r[4];
    for (int i = 0; i < 4; ++i) r[i] = ((CM(m, 0, i) * v[0] + CM(m, 1, i) * v[1]) + CM(m, 2, i) * v[2]) + CM(m, 3, i) * v[3];
    memcpy(out, r, sizeof r);
}

/* GaussTracing.rgen:39-43: uv from (launch id [+ jitter]); origin, direction */
static void gen_ray(const or_ubo* u, float px, float py, float o[3], float d[3]) {
    float uvx = (px / (float)u->width) * 2.0f - 1.0f;
    float uvy = (py / (float)u->height) * 2.0f - 1.0f;
    const float o4[4] = {0, 0, 0, 1};
    float org[4], tg[4], dir[4];
    mul4v(u->model_view_inverse, o4, org);
    const float t4[4] = {uvx, uvy, 1, 1};
    mul4v(u->projection_inverse, t4, tg);
    float v[3] = {tg[0] * u->focus_distance, tg[1] * u->focus_distance, tg[2] * u->focus_distance};
    float len = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    float dv[4] = {v[0] / len, v[1] / len, v[2] / len, 0.0f};
    mul4v(u->model_view_inverse, dv, dir);
    for (int k = 0; k < 3; ++k) { o[k] = org[k]; d[k] = dir[k]; }
}

/* Per-Gaussian projection shared by every ray (rint:62-102), REF convention. */
typedef struct { float depth, ppx, ppy, a, b, c, opacity; int valid; } splat2d;

static void project_ref(const or_ubo* u, const or_gauss_param* g, splat2d* s) {
    const float* MV = u->model_view;
    const float* P = u->projection;
    float c4[4] = {g->center_opacity[0], g->center_opacity[1], g->center_opacity[2], 1.0f};
    float t[4];
    mul4v(MV, c4, t);
    s->depth = t[2];
    s->opacity = g->center_opacity[3];
    float ph[4];
    mul4v(P, t, ph);
    float ndcx = ph[0] / ph[3], ndcy = ph[1] / ph[3];
    s->ppx = ((ndcx + 1.0f) * (float)u->width) * 0.5f;
    s->ppy = ((ndcy + 1.0f) * (float)u->height) * 0.5f;
    float fx = (CM(P, 0, 0) * (float)u->height) * 0.5f; /* rint:76-77: both use Height */
    float fy = (CM(P, 1, 1) * (float)u->height) * 0.5f;
    float zz = t[2] * t[2];
    float J[9] = {fx / t[2], 0.0f, 0.0f, 0.0f, fy / t[2], 0.0f, (-fx * t[0]) / zz, (-fy * t[1]) / zz, 0.0f};
    float W[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) W[c * 3 + r] = CM(MV, c, r);
    const float* cv = g->cov3d;
    float S[9] = {cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]};
    /* T = J*W; V = (T*Cov3D)*transpose(T); GLSL mat3 products summed left to right */
    float T[9], TS[9], Tt[9], V[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) T[c * 3 + r] = (J[0 * 3 + r] * W[c * 3 + 0] + J[1 * 3 + r] * W[c * 3 + 1]) + J[2 * 3 + r] * W[c * 3 + 2];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) TS[c * 3 + r] = (T[0 * 3 + r] * S[c * 3 + 0] + T[1 * 3 + r] * S[c * 3 + 1]) + T[2 * 3 + r] * S[c * 3 + 2];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) Tt[c * 3 + r] = T[r * 3 + c];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) V[c * 3 + r] = (TS[0 * 3 + r] * Tt[c * 3 + 0] + TS[1 * 3 + r] * Tt[c * 3 + 1]) + TS[2 * 3 + r] * Tt[c * 3 + 2];
    s->a = V[0 * 3 + 0];
    s->b = V[0 * 3 + 1];
    s->c = V[1 * 3 + 1];
    s->valid = 1;
}

/* COR convention (SURVEY.md Appendix A "COR flags"): depth = -view z, true Jacobian with
 * fx = P00*W/2, fy = P11*H/2, V += 0.3 I, conic = V^-1. Invalid: depth <= 0 or det <= 0. */
static void project_cor(const or_ubo* u, const or_gauss_param* g, splat2d* s) {
    const float* MV = u->model_view;
    const float* P = u->projection;
    float c4[4] = {g->center_opacity[0], g->center_opacity[1], g->center_opacity[2], 1.0f};
    float t[4];
    mul4v(MV, c4, t);
    s->valid = 0;
    s->depth = -t[2];
    s->opacity = g->center_opacity[3];
    if (!(s->depth > 0.0f)) return;
    float ph[4];
    mul4v(P, t, ph);
    float ndcx = ph[0] / ph[3], ndcy = ph[1] / ph[3];
    s->ppx = ((ndcx + 1.0f) * (float)u->width) * 0.5f;
    s->ppy = ((ndcy + 1.0f) * (float)u->height) * 0.5f;
    float fx = (CM(P, 0, 0) * (float)u->width) * 0.5f;
    float fy = (CM(P, 1, 1) * (float)u->height) * 0.5f;
    float id = 1.0f / s->depth;
    float id2 = id * id;
    /* J rows: (fx/d, 0, fx*x/d^2), (0, fy/d, fy*y/d^2) */
    float j00 = fx * id, j02 = (fx * t[0]) * id2, j11 = fy * id, j12 = (fy * t[1]) * id2;
    /* T = J * W, W[r][k] = MV[k][r] (rows of the view rotation) */
    float T0[3], T1[3];
    for (int k = 0; k < 3; ++k) {
        T0[k] = fmaf(j02, CM(MV, k, 2), j00 * CM(MV, k, 0));
        T1[k] = fmaf(j12, CM(MV, k, 2), j11 * CM(MV, k, 1));
    }
    const float* cv = g->cov3d;
    float S[9] = {cv[0], cv[1], cv[2], cv[1], cv[3], cv[4], cv[2], cv[4], cv[5]};
    float u0[3], u1[3]; /* Sigma * T0, Sigma * T1 */
    for (int r = 0; r < 3; ++r) {
        u0[r] = fmaf(S[r * 3 + 2], T0[2], fmaf(S[r * 3 + 1], T0[1], S[r * 3 + 0] * T0[0]));
        u1[r] = fmaf(S[r * 3 + 2], T1[2], fmaf(S[r * 3 + 1], T1[1], S[r * 3 + 0] * T1[0]));
    }
    float v00 = fmaf(T0[2], u0[2], fmaf(T0[1], u0[1], T0[0] * u0[0])) + 0.3f;
    float v01 = fmaf(T0[2], u1[2], fmaf(T0[1], u1[1], T0[0] * u1[0]));
    float v11 = fmaf(T1[2], u1[2], fmaf(T1[1], u1[1], T1[0] * u1[0])) + 0.3f;
    float det = fmaf(v00, v11, -(v01 * v01));
    if (!(det > 0.0f)) return;
    float idet = 1.0f / det;
    s->a = v11 * idet;
    s->b = -v01 * idet;
    s->c = v00 * idet;
    s->valid = 1;
}

/* 3DGS real SH basis, degree 3, evaluated at the (world) ray direction. */
static void sh_basis(const float d[3], float bs[16]) {
    float x = d[0], y = d[1], z = d[2];
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    bs[0] = 0.28209479177387814f;
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
/* COR colour: max(0, 0.5 + sum_k s_k Y_k(dir)) in this order: the ray-independent DC term with the 0.5 offset
 * first, (s_0 Y_0) + 0.5, then the fma chain over k = 1..15 (the device stores the DC term precomputed). */
static void sh_color(const float* s, const float bs[16], float col[3]) {
    for (int c = 0; c < 3; ++c) {
        float acc = s[c] * bs[0] + 0.5f;
        for (int k = 1; k < 16; ++k) acc = fmaf(bs[k], s[k * 3 + c], acc);
        col[c] = acc > 0.0f ? acc : 0.0f;
    }
}

/* Random.glsl:24-37 (RandomInt LCG + RandomFloat) */
static float random_float(uint32_t* seed) {
    *seed = 1664525u * *seed + 1013904223u;
    return (float)(*seed & 0x00FFFFFFu) / (float)0x01000000;
}

/* ------------------------------------------------------------------ render */

typedef struct {
    const or_gauss_param* params; const or_aabb* aabbs; const float* sh; uint32_t n;
    const float* tris; uint32_t ntri;
    const or_bvh* bvh; const or_ubo* ubo; uint32_t mode;
    float* rgba; or_raystate* rs; uint32_t* stats;
    splat2d* proj; float lut[512];
    uint32_t next_row, row_end;
    pthread_mutex_t mu;
} render_ctx;

typedef struct { uint32_t* ids; uint32_t cnt, cap; } cand_list;

static void cand_push(cand_list* l, uint32_t id) {
    if (l->cnt == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 256;
        l->ids = (uint32_t*)realloc(l->ids, sizeof(uint32_t) * l->cap);
    }
    l->ids[l->cnt++] = id;
}

static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* every Gaussian whose exact AABB passes the slab test with an entry t below tcut (the triangle cull, :806-807;
 * +inf: none), ascending id */
static int cand_hit(const obj_ray* r, const or_aabb* a, float tcut) {
    float t;
    return slab_hit_t(r, a, &t) && t < tcut;
}
static void gather_candidates(const render_ctx* c, const obj_ray* r, float tcut, cand_list* out) {
    out->cnt = 0;
    if (!c->bvh) {
        for (uint32_t i = 0; i < c->n; ++i)
            if (cand_hit(r, c->aabbs + i, tcut)) cand_push(out, i);
        return;
    }
    uint32_t stack[128];
    int sp = 0;
    if (c->bvh->nnodes) stack[sp++] = 0;
    while (sp) {
        uint32_t nd = stack[--sp];
        const float* bx = c->bvh->box + 6 * nd;
        or_aabb nb = {{bx[0], bx[1], bx[2]}, {bx[3], bx[4], bx[5]}};
        /* conservative node test: an exact-hit leaf box is inside its ancestors' boxes; min/max are exact,
         * so the node test can only be looser than the leaf test. */
        if (!slab_hit(r, &nb)) continue;
        uint32_t a = c->bvh->info[2 * nd], b = c->bvh->info[2 * nd + 1];
        if (a & 0x80000000u) {
            for (uint32_t i = a & 0x7fffffffu; i < (a & 0x7fffffffu) + b; ++i) {
                uint32_t id = c->bvh->ids[i];
                if (cand_hit(r, c->aabbs + id, tcut)) cand_push(out, id);
            }
        } else {
            stack[sp++] = b;
            stack[sp++] = a;
        }
    }
    qsort(out->ids, out->cnt, sizeof(uint32_t), cmp_u32);
}

static void render_ref_pixel(render_ctx* c, uint32_t px, uint32_t py, cand_list* cl) {
    const or_ubo* u = c->ubo;
    const float thr_g = 5.6f, thr_a = 1.0f / 255.0f;
    float o[3], d[3];
    gen_ray(u, (float)px, (float)py, o, d);
    obj_ray r;
    make_obj_ray(o, d, &r);
    /* the rays of a pixel are the same every round and sample (rgen:37-43): one min_thit per pixel */
    const float tri = c->ntri ? closest_triangle(c->tris, c->ntri, &r) : 10000.0f;
    const int tri_hit = tri < 10000.0f; /* traversal_data.hit_geometry (:1094-1096) */
    gather_candidates(c, &r, tri * r.norm, cl);
    or_raystate st;
    st.trans = 1.0f; st.depth = 0.0f; st.gauss_num = 0; st.gauss_num_raw = 0;
    for (int j = 0; j < 8; ++j) { st.k[j][0] = 10000.0f; st.k[j][1] = -1.0f; } /* Scene.cpp:38-41 */
    uint32_t rounds = 0;
    int gnum = 0;
    for (uint32_t s = 0; s < u->samples; ++s) {
        for (uint32_t b = 0; b <= u->bounces; ++b) {
            ++rounds;
            gnum = 0;
            for (int j = 0; j < 8; ++j) st.k[j][0] = 10000.0f;
            int reported = tri_hit, gauss_rep = 0; /* instructions.cc:7036-7050: hit_geometry, world_min_thit */
            float closest = tri;
            for (uint32_t ci = 0; ci < cl->cnt; ++ci) {
                const splat2d* sp = c->proj + cl->ids[ci];
                float depth = sp->depth;
                if (depth <= st.depth) continue;
                float dx = (float)px - sp->ppx, dy = (float)py - sp->ppy;
                float g = 0.5f * (((sp->a * dx) * dx + ((2.0f * sp->b) * dx) * dy) + (sp->c * dy) * dy);
                if (g < 0.0f || g > thr_g) continue;
                if (g != g) continue; /* NaN: LinearExp -> NaN alpha -> alpha > 1/255 is false */
                float alpha = sp->opacity * or_linear_exp(c->lut, g);
                if (alpha > thr_a) {
                    float nd = depth, na = alpha;
                    int ins = 0;
                    for (int j = 0; j < 8; ++j) {
                        if (st.k[j][0] > nd) {
                            float td = st.k[j][0], ta = st.k[j][1];
                            st.k[j][0] = nd; st.k[j][1] = na;
                            nd = td; na = ta;
                            ins = 1;
                        }
                    }
                    if (ins) gnum += 1;
                    /* report_ray_intersection_impl (instructions.cc:7040-7046) */
                    if (0.001f <= depth && (reported ? depth < closest : depth <= 10000.0f)) {
                        reported = gauss_rep = 1;
                        closest = depth;
                    }
                }
            }
            if (gauss_rep) { /* rchit:15-33 with GaussNum clamped to 8 */
                int m = gnum < 8 ? gnum : 8;
                float ct = st.trans;
                for (int j = 0; j < m; ++j) ct *= (1.0f - st.k[j][1]);
                st.trans = ct;
                if (m > 0) st.depth = st.k[m - 1][0];
            } else if (tri_hit) {
                st.trans = 0.0f; /* the triangle's closest hit: RayTracing.rchit, Scatter() -> RayPayload(0, ...) */
            }
            st.gauss_num_raw = gnum;
            if (gnum == 0) break;
        }
    }
    st.gauss_num = gnum < 8 ? gnum : 8;
    size_t pix = (size_t)py * u->width + px;
    if (c->rgba) for (int k = 0; k < 4; ++k) c->rgba[4 * pix + k] = 0.0f; /* rgen:33,75 */
    if (c->rs) c->rs[pix] = st;
    if (c->stats) {
        c->stats[4 * pix + 0] = cl->cnt;
        c->stats[4 * pix + 1] = tri_hit ? rounds : 0; /* traversals with a triangle hit (vulkan-sim rt_num_hits) */
        c->stats[4 * pix + 2] = rounds;
        c->stats[4 * pix + 3] = 0;
    }
}

typedef struct { uint64_t key; uint32_t id; } keyed;
static int cmp_keyed(const void* a, const void* b) {
    uint64_t x = ((const keyed*)a)->key, y = ((const keyed*)b)->key;
    return x < y ? -1 : x > y;
}

static void render_cor_pixel(render_ctx* c, uint32_t px, uint32_t py, cand_list* cl, keyed** kbuf, uint32_t* kcap) {
    const or_ubo* u = c->ubo;
    const int use_lut = (c->mode & OR_FLAG_LUT) != 0;
    const uint32_t S = u->samples ? u->samples : 1;
    float acc[64][4];
    float* seqacc = NULL;
    int tree = (S <= 64) && ((S & (S - 1)) == 0);
    float sacc[4] = {0, 0, 0, 0};
    uint32_t seed = u->random_seed; /* RayTracing.rgen:27: pixelRandomSeed = Camera.RandomSeed */
    uint32_t ncand = 0, nblend = 0, nterm = 0;
    (void)seqacc;
    for (uint32_t s = 0; s < S; ++s) {
        float jx = random_float(&seed);
        float jy = random_float(&seed);
        float o[3], d[3];
        gen_ray(u, (float)px + jx, (float)py + jy, o, d);
        obj_ray r;
        make_obj_ray(o, d, &r);
        gather_candidates(c, &r, INFINITY, cl);
        if (cl->cnt > *kcap) {
            *kcap = cl->cnt * 2;
            *kbuf = (keyed*)realloc(*kbuf, sizeof(keyed) * *kcap);
        }
        uint32_t nk = 0;
        for (uint32_t i = 0; i < cl->cnt; ++i) {
            const splat2d* sp = c->proj + cl->ids[i];
            if (!sp->valid) continue;
            uint32_t bits;
            memcpy(&bits, &sp->depth, 4);
            (*kbuf)[nk].key = ((uint64_t)bits << 32) | cl->ids[i];
            (*kbuf)[nk].id = cl->ids[i];
            ++nk;
        }
        qsort(*kbuf, nk, sizeof(keyed), cmp_keyed);
        float bs[16];
        if (c->sh) sh_basis(d, bs);
        float T = 1.0f, C[3] = {0, 0, 0};
        float pxs = (float)px + jx, pys = (float)py + jy;
        for (uint32_t i = 0; i < nk; ++i) {
            uint32_t id = (*kbuf)[i].id;
            const splat2d* sp = c->proj + id;
            ++ncand;
            float dx = pxs - sp->ppx, dy = pys - sp->ppy;
            float g = 0.5f * fmaf(sp->c * dy, dy, fmaf(2.0f * sp->b * dx, dy, (sp->a * dx) * dx));
            if (!(g >= 0.0f && g <= 5.6f)) continue;
            float e = use_lut ? or_linear_exp(c->lut, g) : or_exp_neg(-g);
            float alpha = sp->opacity * e;
            if (alpha > 0.99f) alpha = 0.99f;
            if (!(alpha > 1.0f / 255.0f)) continue;
            float tn = T * (1.0f - alpha);
            if (tn < 1e-4f) { ++nterm; break; }
            float col[3] = {1.0f, 1.0f, 1.0f};
            if (c->sh) sh_color(c->sh + 48 * (size_t)id, bs, col);
            float w = alpha * T;
            for (int k = 0; k < 3; ++k) C[k] = fmaf(col[k], w, C[k]);
            T = tn;
            ++nblend;
        }
        float v[4] = {C[0], C[1], C[2], 1.0f - T};
        if (tree) {
            for (int k = 0; k < 4; ++k) acc[s][k] = v[k];
        } else {
            for (int k = 0; k < 4; ++k) sacc[k] += v[k];
        }
    }
    if (tree) {
        for (uint32_t stride = 1; stride < S; stride *= 2)
            for (uint32_t i = 0; i + stride < S; i += 2 * stride)
                for (int k = 0; k < 4; ++k) acc[i][k] = acc[i][k] + acc[i + stride][k];
        for (int k = 0; k < 4; ++k) sacc[k] = acc[0][k];
    }
    size_t pix = (size_t)py * u->width + px;
    if (c->rgba)
        for (int k = 0; k < 4; ++k) c->rgba[4 * pix + k] = sacc[k] / (float)S;
    if (c->stats) {
        c->stats[4 * pix + 0] = ncand;
        c->stats[4 * pix + 1] = nblend;
        c->stats[4 * pix + 2] = 1;
        c->stats[4 * pix + 3] = nterm;
    }
}

static void* render_worker(void* arg) {
    render_ctx* c = (render_ctx*)arg;
    cand_list cl = {0, 0, 0};
    keyed* kbuf = NULL;
    uint32_t kcap = 0;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        uint32_t row = c->next_row++;
        pthread_mutex_unlock(&c->mu);
        if (row >= c->row_end) break;
        for (uint32_t x = 0; x < c->ubo->width; ++x) {
            if ((c->mode & 0xff) == OR_MODE_REF) render_ref_pixel(c, x, row, &cl);
            else render_cor_pixel(c, x, row, &cl, &kbuf, &kcap);
        }
    }
    free(cl.ids);
    free(kbuf);
    return NULL;
}

int or_render(const or_gauss_param* params, const or_aabb* aabbs, const float* sh, uint32_t n, const or_bvh* bvh,
              const or_ubo* ubo, uint32_t mode, uint32_t threads, uint32_t row_begin, uint32_t row_end, float* rgba,
              or_raystate* raystate, uint32_t* stats) {
    return or_render_mesh(params, aabbs, sh, n, bvh, NULL, 0, ubo, mode, threads, row_begin, row_end, rgba, raystate,
                          stats);
}

int or_render_mesh(const or_gauss_param* params, const or_aabb* aabbs, const float* sh, uint32_t n, const or_bvh* bvh,
                   const float* tris, uint32_t ntri, const or_ubo* ubo, uint32_t mode, uint32_t threads,
                   uint32_t row_begin, uint32_t row_end, float* rgba, or_raystate* raystate, uint32_t* stats) {
    if (!ubo || ubo->width == 0 || ubo->height == 0 || row_end > ubo->height || row_begin > row_end) return -1;
    if ((mode & 0xff) > OR_MODE_COR) return -1;
    if (ntri && ((mode & 0xff) != OR_MODE_REF || !tris)) return -1;
    render_ctx* c = (render_ctx*)calloc(1, sizeof *c);
    c->params = params; c->aabbs = aabbs; c->sh = sh; c->n = n; c->bvh = bvh; c->ubo = ubo; c->mode = mode;
    c->tris = tris; c->ntri = ntri;
    c->rgba = rgba; c->rs = raystate; c->stats = stats;
    c->next_row = row_begin; c->row_end = row_end;
    or_exp_lut(c->lut);
    c->proj = (splat2d*)malloc(sizeof(splat2d) * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) {
        if ((mode & 0xff) == OR_MODE_REF) project_ref(ubo, params + i, c->proj + i);
        else project_cor(ubo, params + i, c->proj + i);
    }
    pthread_mutex_init(&c->mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (uint32_t t = 1; t < threads; ++t) pthread_create(&th[t], NULL, render_worker, c);
    render_worker(c);
    for (uint32_t t = 1; t < threads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&c->mu);
    free(c->proj);
    free(c);
    return 0;
}

/* Model::CreateSphere (Model.cpp:566-629): 33 x 17 vertices (cx + v sin(i0), cy + z, cz + v cos(i0)),
 * v = -r sin(j0), z = r cos(j0), j0 = pi j / 16, i0 = 2 pi i / 32 in float (std::sin of a float = sinf);
 * per quad the triangles (j0+i0, j1+i0, j1+i1) and (j0+i0, j1+i1, j0+i1) */
void or_sphere_mesh(const float center[3], float radius, float* vertices, uint32_t* indices) {
    const int slices = 32, stacks = 16;
    const float pi = 3.14159265358979f;
    size_t q = 0, t = 0;
    for (int j = 0; j <= stacks; ++j) {
        volatile float j0v = pi * j / stacks; /* keep sinf/cosf calls (no compile-time folding) */
        float j0 = j0v;
        float v = radius * -sinf(j0);
        float z = radius * cosf(j0);
        for (int i = 0; i <= slices; ++i) {
            volatile float i0v = 2 * pi * i / slices;
            float i0 = i0v;
            vertices[q++] = center[0] + v * sinf(i0);
            vertices[q++] = center[1] + z;
            vertices[q++] = center[2] + v * cosf(i0);
        }
    }
    for (int j = 0; j < stacks; ++j)
        for (int i = 0; i < slices; ++i) {
            uint32_t a = (uint32_t)(j * (slices + 1)), b = (uint32_t)((j + 1) * (slices + 1));
            uint32_t tri[6] = {a + i, b + i, b + i + 1, a + i, b + i + 1, a + i + 1};
            for (int k = 0; k < 6; ++k) indices[t++] = tri[k];
        }
}
