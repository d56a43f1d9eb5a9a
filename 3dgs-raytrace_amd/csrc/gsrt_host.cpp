// gsrt_host.cpp -- host-side pieces of the boundary: camera / UBO, ExpLUT, frame dumps, synthetic clouds.
//
// The camera code restates the glm calls RayTracer::GetUniformBufferObject makes
// (RayTracingInVulkan/src/RayTracer.cpp:38-65, ModelViewController.cpp:4-34, glm 2022.05.10 with
// GLM_FORCE_DEPTH_ZERO_TO_ONE + GLM_FORCE_RIGHT_HANDED, Utilities/Glm.hpp:3-4), in glm's summation order.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <random>
#include <string>
#include <vector>

#include "../../include/gsrt_test.h"

namespace gsrt {

namespace {

struct Mat4 { float m[16]; float& at(int c, int r) { return m[c * 4 + r]; } float at(int c, int r) const { return m[c * 4 + r]; } };

Mat4 identity() { Mat4 a{}; a.at(0, 0) = a.at(1, 1) = a.at(2, 2) = a.at(3, 3) = 1.0f; return a; }

// glm operator*(mat4, mat4): Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
Mat4 mul(const Mat4& a, const Mat4& b) {
    Mat4 r{};
    for (int c = 0; c < 4; ++c)
        for (int i = 0; i < 4; ++i)
            r.at(c, i) = ((a.at(0, i) * b.at(c, 0) + a.at(1, i) * b.at(c, 1)) + a.at(2, i) * b.at(c, 2)) + a.at(3, i) * b.at(c, 3);
    return r;
}

// glm operator*(mat4, vec4), non-SIMD path: (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
void mulv(const Mat4& m, const float v[4], float o[4]) {
    for (int i = 0; i < 4; ++i)
        o[i] = (m.at(0, i) * v[0] + m.at(1, i) * v[1]) + (m.at(2, i) * v[2] + m.at(3, i) * v[3]);
}

// glm::inverse (detail/func_matrix.inl, compute_inverse<4, 4>)
Mat4 inverse(const Mat4& m) {
    auto M = [&](int c, int r) { return m.at(c, r); };
    const float c00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3), c02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    const float c03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3), c04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    const float c06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3), c07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    const float c08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2), c10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    const float c11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2), c12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    const float c14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3), c15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    const float c16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2), c18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    const float c19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2), c20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    const float c22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1), c23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    const float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    const float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    const float v0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, v1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    const float v2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, v3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    const float sa[4] = {+1.f, -1.f, +1.f, -1.f}, sb[4] = {-1.f, +1.f, -1.f, +1.f};
    Mat4 inv{};
    for (int i = 0; i < 4; ++i) {
        inv.at(0, i) = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3[i] * f2[i]) * sa[i];
        inv.at(1, i) = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3[i] * f4[i]) * sb[i];
        inv.at(2, i) = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3[i] * f5[i]) * sa[i];
        inv.at(3, i) = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb[i];
    }
    float d0[4];
    for (int i = 0; i < 4; ++i) d0[i] = M(0, i) * inv.at(i, 0);
    const float det = (d0[0] + d0[1]) + (d0[2] + d0[3]);
    const float one_over = 1.0f / det;
    for (float& x : inv.m) x *= one_over;
    return inv;
}

float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
void cross3(const float x[3], const float y[3], float o[3]) {
    const float r0 = x[1] * y[2] - y[1] * x[2], r1 = x[2] * y[0] - y[2] * x[0], r2 = x[0] * y[1] - y[0] * x[1];
    o[0] = r0; o[1] = r1; o[2] = r2;
}
void normalize3(float v[3]) {
    const float is = 1.0f / std::sqrt(dot3(v, v));
    v[0] *= is; v[1] *= is; v[2] *= is;
}

}  // namespace

void exp_lut(float out[512]) {  // generateExpLUT(256, 0, 8): ExpLUT.hpp:10-24
    const float step = (8.0f - 0.0f) / 256;
    for (int i = 0; i < 256; ++i) {
        const float x = 0.0f + i * step;
        out[2 * i] = -std::exp(-x);
        out[2 * i + 1] = std::exp(-x);
    }
}

}  // namespace gsrt

using gsrt::Mat4;

extern "C" gsrt_status gsrt_lookat(const float eye[3], const float center[3], const float up[3], float out[16]) {
    if (!eye || !center || !up || !out) return GSRT_E_ARG;
    float f[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
    gsrt::normalize3(f);
    float s[3];
    gsrt::cross3(f, up, s);
    gsrt::normalize3(s);
    float u[3];
    gsrt::cross3(s, f, u);
    Mat4 r = gsrt::identity();
    r.at(0, 0) = s[0]; r.at(1, 0) = s[1]; r.at(2, 0) = s[2];
    r.at(0, 1) = u[0]; r.at(1, 1) = u[1]; r.at(2, 1) = u[2];
    r.at(0, 2) = -f[0]; r.at(1, 2) = -f[1]; r.at(2, 2) = -f[2];
    r.at(3, 0) = -gsrt::dot3(s, eye);
    r.at(3, 1) = -gsrt::dot3(u, eye);
    r.at(3, 2) = gsrt::dot3(f, eye);
    std::memcpy(out, r.m, sizeof r.m);
    return GSRT_OK;
}

extern "C" gsrt_status gsrt_camera_from_modelview(const float mv[16], float fovy_deg, uint32_t width, uint32_t height,
                                                  float focus_distance, uint32_t samples, uint32_t bounces,
                                                  gsrt_ubo* out) {
    if (!mv || !out || width == 0 || height == 0) return GSRT_E_ARG;
    Mat4 init;
    std::memcpy(init.m, mv, sizeof init.m);
    // ModelViewController::Reset: position = inverse(mv) * (0,0,0,1), orientation = mat4(mat3(mv))
    const Mat4 inv = gsrt::inverse(init);
    const float o4[4] = {0, 0, 0, 1};
    float pos[4];
    gsrt::mulv(inv, o4, pos);
    Mat4 orient{};
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) orient.at(c, r) = init.at(c, r);
    orient.at(3, 3) = 1.0f;
    // ModelView() at rest: orientation * translate(I, -position) * (identity model rotation)
    Mat4 tr = gsrt::identity();
    tr.at(3, 0) = -pos[0]; tr.at(3, 1) = -pos[1]; tr.at(3, 2) = -pos[2];
    const Mat4 view = gsrt::mul(orient, tr);
    // glm::perspective (RH_ZO) with glm::radians, then Projection[1][1] *= -1 (RayTracer.cpp:44-45)
    const float fovy = fovy_deg * 0.01745329251994329576923690768489f;
    const float aspect = (float)width / (float)height;
    const float tan_half = std::tan(fovy / 2.0f);
    Mat4 proj{};
    proj.at(0, 0) = 1.0f / (aspect * tan_half);
    proj.at(1, 1) = 1.0f / tan_half;
    proj.at(2, 2) = 10000.0f / (0.1f - 10000.0f);
    proj.at(2, 3) = -1.0f;
    proj.at(3, 2) = -(10000.0f * 0.1f) / (10000.0f - 0.1f);
    proj.at(1, 1) *= -1.0f;
    std::memset(out, 0, sizeof *out);
    std::memcpy(out->model_view, view.m, 64);
    std::memcpy(out->projection, proj.m, 64);
    const Mat4 vi = gsrt::inverse(view), pi = gsrt::inverse(proj);
    std::memcpy(out->model_view_inverse, vi.m, 64);
    std::memcpy(out->projection_inverse, pi.m, 64);
    out->focus_distance = focus_distance;
    out->total_samples = samples;
    out->samples = samples;
    out->bounces = bounces;
    out->random_seed = 1;  // RayTracer.cpp:59
    out->width = width;
    out->height = height;
    out->has_sky = 1;
    return GSRT_OK;
}

extern "C" gsrt_status gsrt_camera_from_file(const char* path, float fovy_deg, uint32_t width, uint32_t height,
                                             float focus_distance, uint32_t samples, uint32_t bounces, gsrt_ubo* out) {
    if (!path || !out) return GSRT_E_ARG;
    FILE* f = std::fopen(path, "r");
    if (!f) return GSRT_E_IO;
    float e[3], c[3];
    const int got = std::fscanf(f, "%f %f %f %f %f %f", &e[0], &e[1], &e[2], &c[0], &c[1], &c[2]);
    std::fclose(f);
    if (got != 6) return GSRT_E_IO;
    const float up[3] = {0.0f, 1.0f, 0.0f};
    float mv[16];
    gsrt_lookat(e, c, up, mv);  // SceneList.cpp:705-712
    return gsrt_camera_from_modelview(mv, fovy_deg, width, height, focus_distance, samples, bounces, out);
}

// vulkan_ray_tracing.cc:2216-2247: header "P3\n%d %d\n255\n", then each image_store fseeko()s to header + (x + y*W)*12
// and prints "%3.0f %3.0f %3.0f\n" of rgb*255. Emulated in launch (row-major) order into a buffer, so an over-wide value
// spills into the next slot exactly as the fseeko writes do. line(i, tmp) formats pixel i (its length, or < 0: fail).
template <class Line>
static gsrt_status write_p3(const char* path, uint32_t width, uint32_t height, Line line) {
    char hdr[64];
    const int hl = std::snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", width, height);
    const size_t body = (size_t)width * height * 12;
    std::vector<char> buf(hl + body + 64, 0);
    std::memcpy(buf.data(), hdr, hl);
    size_t end = hl + body;
    char tmp[128];
    for (size_t i = 0; i < (size_t)width * height; ++i) {
        const int l = line(i, tmp);
        if (l < 0) return GSRT_E_ARG;
        const size_t at = hl + i * 12;
        if (at + l > buf.size()) buf.resize(at + l);
        std::memcpy(buf.data() + at, tmp, l);
        if (at + l > end) end = at + l;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return GSRT_E_IO;
    const size_t w = std::fwrite(buf.data(), 1, end, f);
    std::fclose(f);
    return w == end ? GSRT_OK : GSRT_E_IO;
}

static int p3_line(char* tmp, float r, float g, float b) {
    return std::snprintf(tmp, 128, "%3.0f %3.0f %3.0f\n", r * 255, g * 255, b * 255);
}

extern "C" gsrt_status gsrt_dump_ppm(const char* path, const float* rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || width == 0 || height == 0) return GSRT_E_ARG;
    return write_p3(path, width, height,
                    [&](size_t i, char* tmp) { return p3_line(tmp, rgba[4 * i], rgba[4 * i + 1], rgba[4 * i + 2]); });
}

// the same bytes from a frame's dump codes (GSRT_FLAG_OUT_DUMP8): a code's channels are the integers "%3.0f" prints
// for them (so "%3u" prints the same), an escaped pixel's exact channels are printed as gsrt_dump_ppm prints them
extern "C" gsrt_status gsrt_dump8_ppm(const char* path, const uint32_t* codes, uint32_t width, uint32_t height,
                                      const gsrt_dump8_escape* esc, uint32_t n_esc) {
    if (!path || !codes || width == 0 || height == 0 || (n_esc && !esc)) return GSRT_E_ARG;
    std::vector<gsrt_dump8_escape> e(esc, esc + n_esc);
    std::sort(e.begin(), e.end(), [](const gsrt_dump8_escape& a, const gsrt_dump8_escape& b) { return a.pixel < b.pixel; });
    return write_p3(path, width, height, [&](size_t i, char* tmp) {
        const uint32_t c = codes[i];
        if (c & GSRT_DUMP8_ESCAPE) {
            auto it = std::lower_bound(e.begin(), e.end(), (uint32_t)i,
                                       [](const gsrt_dump8_escape& a, uint32_t px) { return a.pixel < px; });
            if (it == e.end() || it->pixel != i) return -1;  // an escaped pixel without its entry
            return p3_line(tmp, it->r, it->g, it->b);
        }
        return std::snprintf(tmp, 128, "%3u %3u %3u\n", c & 1023u, (c >> 10) & 1023u, (c >> 20) & 1023u);
    });
}

extern "C" gsrt_status gsrt_reference_ppm_name(char* out, size_t cap) {
    if (!out || cap == 0) return GSRT_E_ARG;
    std::time_t raw = std::time(nullptr);
    std::tm tmv;
    localtime_r(&raw, &tmv);
    char tb[30];
    std::strftime(tb, sizeof tb, "%d-%m-%Y-%H-%M-%S-", &tmv);
    const int l = std::snprintf(out, cap, "%sSCENE.ppm", tb);
    return (l > 0 && (size_t)l < cap) ? GSRT_OK : GSRT_E_ARG;
}

extern "C" gsrt_status gsrt_dump_image_binary(const char* path, const float* rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || width == 0 || height == 0) return GSRT_E_ARG;
    FILE* f = std::fopen(path, "wb");
    if (!f) return GSRT_E_IO;
    // vulkan_ray_tracing.cc:2165-2179: 3 floats then the u32 offset x + y*W, per image_store (launch order)
    std::vector<char> rec(16 * (size_t)width * height);
    for (uint32_t y = 0; y < height; ++y)
        for (uint32_t x = 0; x < width; ++x) {
            const size_t i = (size_t)y * width + x;
            const uint32_t off = y * width + x;
            std::memcpy(&rec[16 * i], rgba + 4 * i, 12);
            std::memcpy(&rec[16 * i + 12], &off, 4);
        }
    const size_t w = std::fwrite(rec.data(), 1, rec.size(), f);
    std::fclose(f);
    return w == rec.size() ? GSRT_OK : GSRT_E_IO;
}

extern "C" gsrt_status gsrt_synth_cloud(uint32_t kind, uint32_t n, uint32_t seed, int with_sh, float* center,
                                        float* rot, float* scale, float* opacity, float* sh) {
    if (n == 0 || !center || !rot || !scale || !opacity || (with_sh && !sh) || kind > GSRT_SYNTH_NEEDLE)
        return GSRT_E_ARG;
    std::mt19937 g(seed);
    auto U = [&](float a, float b) { return std::uniform_real_distribution<float>(a, b)(g); };
    const float sigma0 = 0.0107f * std::sqrt(1e6f / (float)n);
    for (uint32_t i = 0; i < n; ++i) {
        float* C = center + 3 * (size_t)i;
        float* Q = rot + 4 * (size_t)i;
        float* S = scale + 3 * (size_t)i;
        if (kind == GSRT_SYNTH_NEEDLE) {  // REF-active needles through the camera plane
            C[0] = U(-0.05f, 0.05f);
            C[1] = U(-0.05f, 0.05f);
            C[2] = U(0.05f, 1.0f);
            S[0] = U(0.0005f, 0.002f);
            S[1] = U(0.0005f, 0.002f);
            S[2] = U(0.4f, 1.0f);
            Q[0] = 1.0f; Q[1] = Q[2] = Q[3] = 0.0f;
        } else {
            C[0] = U(-4.0f, 4.0f);
            C[1] = U(-4.0f, 4.0f);
            C[2] = kind == GSRT_SYNTH_REF ? U(-4.0f, 4.0f) : U(-12.0f, -4.0f);
            for (int a = 0; a < 3; ++a) S[a] = sigma0 * std::exp(U(-0.5f, 0.5f));
            float q[4], qq = 0.0f;
            for (int a = 0; a < 4; ++a) { q[a] = U(-1.0f, 1.0f); qq += q[a] * q[a]; }
            const float inv = 1.0f / std::sqrt(qq);
            for (int a = 0; a < 4; ++a) Q[a] = q[a] * inv;
        }
        opacity[i] = U(0.05f, 0.95f);
        if (with_sh) {
            float* s = sh + 48 * (size_t)i;
            for (int k = 0; k < 16; ++k)
                for (int c = 0; c < 3; ++c) {
                    const float u = U(0.0f, 1.0f);
                    s[k * 3 + c] = k == 0 ? u - 0.5f : 0.2f * (u - 0.5f);
                }
        }
    }
    return GSRT_OK;
}
