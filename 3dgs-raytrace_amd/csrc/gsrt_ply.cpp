// gsrt_ply.cpp -- scene ingestion from 3D Gaussian Splatting .ply files and the
// dump_image.sh text dump (§8f item 3).
//
// The reference builds its Gaussians from hard-coded Model::CreateGauss calls (SceneList.cpp:123-125);
// trained 3DGS scenes come as PLY vertex lists with the properties
//   x y z  [nx ny nz]  f_dc_0..2  f_rest_0..(3*(K-1)-1)  opacity  scale_0..2  rot_0..3
// in the 3DGS activation-free convention: scale is log(sigma), opacity is logit(alpha), rot is an
// unnormalised quaternion (w, x, y, z), f_rest is channel-major (all R coefficients, then G, then B).
// gsrt_ply_read converts to the CreateGauss convention the rest of the ABI uses: scale = exp(scale),
// opacity = sigmoid(opacity), rot normalised (r, x, y, z), SH as [gauss][coef 0..15][rgb] with the
// degree cut or zero-padded to 3.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gsrt.h"
#include "gsrt_internal.hpp"

namespace {

enum class PlyFormat { Ascii, BinaryLE, BinaryBE };

struct PlyProp {
    std::string name;
    int type = 0;   // 0 f32, 1 f64, 2 u8, 3 i8, 4 u16, 5 i16, 6 u32, 7 i32
    int size = 4;
};

struct PlyHeader {
    PlyFormat fmt = PlyFormat::BinaryLE;
    uint64_t n = 0;
    std::vector<PlyProp> props;   // of the vertex element
    uint64_t vertex_stride = 0;
    long data_offset = 0;
    bool vertex_first = true;     // the vertex element precedes every other element
};

bool type_of(const std::string& t, int& type, int& size) {
    static const struct { const char* n[2]; int type, size; } tab[] = {
        {{"float", "float32"}, 0, 4}, {{"double", "float64"}, 1, 8}, {{"uchar", "uint8"}, 2, 1},
        {{"char", "int8"}, 3, 1},     {{"ushort", "uint16"}, 4, 2},  {{"short", "int16"}, 5, 2},
        {{"uint", "uint32"}, 6, 4},   {{"int", "int32"}, 7, 4}};
    for (const auto& e : tab)
        if (t == e.n[0] || t == e.n[1]) { type = e.type; size = e.size; return true; }
    return false;
}

bool read_header(FILE* f, PlyHeader& h, std::string& err) {
    char line[1024];
    if (!std::fgets(line, sizeof line, f) || std::strncmp(line, "ply", 3) != 0) { err = "not a PLY file"; return false; }
    bool in_vertex = false, seen_vertex = false, got_format = false;
    while (std::fgets(line, sizeof line, f)) {
        char a[256] = {0}, b[256] = {0}, c[256] = {0};
        const int k = std::sscanf(line, "%255s %255s %255s", a, b, c);
        if (k <= 0) continue;
        const std::string w = a;
        if (w == "end_header") {
            h.data_offset = std::ftell(f);
            if (!got_format) { err = "missing format line"; return false; }
            if (!seen_vertex) { err = "no vertex element"; return false; }
            return true;
        }
        if (w == "format") {
            const std::string fm = b;
            if (fm == "ascii") h.fmt = PlyFormat::Ascii;
            else if (fm == "binary_little_endian") h.fmt = PlyFormat::BinaryLE;
            else if (fm == "binary_big_endian") h.fmt = PlyFormat::BinaryBE;
            else { err = "unknown PLY format " + fm; return false; }
            got_format = true;
        } else if (w == "element") {
            in_vertex = std::string(b) == "vertex";
            if (in_vertex) {
                h.n = std::strtoull(c, nullptr, 10);
                seen_vertex = true;
            } else if (!seen_vertex) {
                h.vertex_first = false;
            }
        } else if (w == "property" && in_vertex) {
            if (std::string(b) == "list") { err = "list property in the vertex element"; return false; }
            PlyProp p;
            if (!type_of(b, p.type, p.size)) { err = std::string("unknown property type ") + b; return false; }
            p.name = c;
            h.vertex_stride += p.size;
            h.props.push_back(p);
        }
    }
    err = "truncated header";
    return false;
}

double decode(const unsigned char* p, int type, bool swap) {
    unsigned char b[8];
    const int sz = type == 1 ? 8 : (type == 2 || type == 3) ? 1 : (type == 4 || type == 5) ? 2 : 4;
    for (int i = 0; i < sz; ++i) b[i] = swap ? p[sz - 1 - i] : p[i];
    switch (type) {
        case 0: { float v; std::memcpy(&v, b, 4); return v; }
        case 1: { double v; std::memcpy(&v, b, 8); return v; }
        case 2: return b[0];
        case 3: return (int8_t)b[0];
        case 4: { uint16_t v; std::memcpy(&v, b, 2); return v; }
        case 5: { int16_t v; std::memcpy(&v, b, 2); return v; }
        case 6: { uint32_t v; std::memcpy(&v, b, 4); return v; }
        default: { int32_t v; std::memcpy(&v, b, 4); return v; }
    }
}

struct Columns {
    int xyz[3] = {-1, -1, -1}, scale[3] = {-1, -1, -1}, rot[4] = {-1, -1, -1, -1}, opacity = -1;
    int dc[3] = {-1, -1, -1};
    std::vector<int> rest;  // f_rest_i -> column
};

bool map_columns(const PlyHeader& h, Columns& c, std::string& err) {
    int max_rest = -1;
    for (size_t i = 0; i < h.props.size(); ++i) {
        const std::string& n = h.props[i].name;
        const int col = (int)i;
        if (n == "x") c.xyz[0] = col; else if (n == "y") c.xyz[1] = col; else if (n == "z") c.xyz[2] = col;
        else if (n == "opacity") c.opacity = col;
        else if (n.rfind("scale_", 0) == 0 && n.size() == 7 && n[6] >= '0' && n[6] <= '2') c.scale[n[6] - '0'] = col;
        else if (n.rfind("rot_", 0) == 0 && n.size() == 5 && n[4] >= '0' && n[4] <= '3') c.rot[n[4] - '0'] = col;
        else if (n.rfind("f_dc_", 0) == 0 && n.size() == 6 && n[5] >= '0' && n[5] <= '2') c.dc[n[5] - '0'] = col;
        else if (n.rfind("f_rest_", 0) == 0) {
            const int j = std::atoi(n.c_str() + 7);
            if (j < 0 || j > 1000) { err = "bad " + n; return false; }
            if ((int)c.rest.size() <= j) c.rest.resize(j + 1, -1);
            c.rest[j] = col;
            max_rest = std::max(max_rest, j);
        }
    }
    for (int k = 0; k < 3; ++k)
        if (c.xyz[k] < 0 || c.scale[k] < 0) { err = "missing x/y/z or scale_0..2"; return false; }
    for (int k = 0; k < 4; ++k)
        if (c.rot[k] < 0) { err = "missing rot_0..3"; return false; }
    if (c.opacity < 0) { err = "missing opacity"; return false; }
    for (int j = 0; j <= max_rest; ++j)
        if (c.rest[j] < 0) { err = "f_rest properties are not contiguous"; return false; }
    if (!c.rest.empty() && c.rest.size() % 3 != 0) { err = "f_rest count is not a multiple of 3"; return false; }
    return true;
}

gsrt_status ply_load(const char* path, PlyHeader& h, Columns& c, std::vector<double>& rows, std::string& err) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { err = std::string("cannot open ") + path; return GSRT_E_IO; }
    gsrt_status st = GSRT_OK;
    if (!read_header(f, h, err) || !map_columns(h, c, err)) st = GSRT_E_ARG;
    else if (!h.vertex_first) { err = "the vertex element must come first"; st = GSRT_E_ARG; }
    else if (h.n > 0xFFFFFFFFull) { err = "too many vertices"; st = GSRT_E_ARG; }
    if (st != GSRT_OK) { std::fclose(f); return st; }
    const size_t np = h.props.size();
    rows.assign(h.n * np, 0.0);
    if (h.fmt == PlyFormat::Ascii) {
        for (uint64_t i = 0; i < h.n * np; ++i)
            if (std::fscanf(f, "%lf", &rows[i]) != 1) { err = "truncated ASCII body"; st = GSRT_E_IO; break; }
    } else {
        const bool swap = h.fmt == PlyFormat::BinaryBE;
        std::vector<unsigned char> buf(h.vertex_stride * 4096);
        uint64_t done = 0;
        while (done < h.n && st == GSRT_OK) {
            const uint64_t chunk = std::min<uint64_t>(4096, h.n - done);
            if (std::fread(buf.data(), h.vertex_stride, chunk, f) != chunk) { err = "truncated binary body"; st = GSRT_E_IO; break; }
            for (uint64_t r = 0; r < chunk; ++r) {
                const unsigned char* p = buf.data() + r * h.vertex_stride;
                for (size_t k = 0; k < np; ++k) {
                    rows[(done + r) * np + k] = decode(p, h.props[k].type, swap);
                    p += h.props[k].size;
                }
            }
            done += chunk;
        }
    }
    std::fclose(f);
    return st;
}

}  // namespace

extern "C" {

gsrt_status gsrt_ply_info(const char* path, uint32_t* n, uint32_t* sh_degree) {
    if (!path || !n) return GSRT_E_ARG;
    FILE* f = std::fopen(path, "rb");
    if (!f) return GSRT_E_IO;
    PlyHeader h;
    Columns c;
    std::string err;
    const bool ok = read_header(f, h, err) && map_columns(h, c, err) && h.vertex_first && h.n <= 0xFFFFFFFFull;
    std::fclose(f);
    if (!ok) return GSRT_E_ARG;
    *n = (uint32_t)h.n;
    if (sh_degree) {
        const size_t per_channel = c.rest.size() / 3 + 1;  // coefficients per channel
        uint32_t d = 0;
        while ((d + 1) * (d + 1) < per_channel) ++d;
        *sh_degree = c.dc[0] < 0 ? 0u : d;
    }
    return GSRT_OK;
}

gsrt_status gsrt_ply_read(const char* path, float* center, float* rot_rxyz, float* scale, float* opacity, float* sh) {
    if (!path || !center || !rot_rxyz || !scale || !opacity) return GSRT_E_ARG;
    PlyHeader h;
    Columns c;
    std::vector<double> rows;
    std::string err;
    const gsrt_status st = ply_load(path, h, c, rows, err);
    if (st != GSRT_OK) return st;
    const size_t np = h.props.size();
    const size_t rest_per_ch = c.rest.size() / 3;
    for (uint64_t i = 0; i < h.n; ++i) {
        const double* r = rows.data() + i * np;
        for (int k = 0; k < 3; ++k) {
            center[3 * i + k] = (float)r[c.xyz[k]];
            scale[3 * i + k] = std::exp((float)r[c.scale[k]]);
        }
        float q[4], qq = 0.0f;
        for (int k = 0; k < 4; ++k) { q[k] = (float)r[c.rot[k]]; qq += q[k] * q[k]; }
        const float inv = qq > 0.0f ? 1.0f / std::sqrt(qq) : 0.0f;
        for (int k = 0; k < 4; ++k) rot_rxyz[4 * i + k] = qq > 0.0f ? q[k] * inv : (k == 0 ? 1.0f : 0.0f);
        opacity[i] = 1.0f / (1.0f + std::exp(-(float)r[c.opacity]));
        if (sh) {
            float* s = sh + 48 * i;  // [coef 0..15][rgb]
            for (int k = 0; k < 48; ++k) s[k] = 0.0f;
            for (int ch = 0; ch < 3; ++ch) {
                if (c.dc[ch] >= 0) s[ch] = (float)r[c.dc[ch]];
                for (size_t j = 0; j < rest_per_ch && j < 15; ++j) s[3 * (1 + j) + ch] = (float)r[c.rest[ch * rest_per_ch + j]];
            }
        }
    }
    return GSRT_OK;
}

gsrt_status gsrt_scene_from_ply(gsrt_ctx* ctx, const char* path, int with_sh, gsrt_scene** out) {
    if (!ctx || !path || !out) return GSRT_E_ARG;
    uint32_t n = 0, deg = 0;
    gsrt_status st = gsrt_ply_info(path, &n, &deg);
    if (st != GSRT_OK) return gsrt::fail(ctx, st, std::string("gsrt_scene_from_ply: cannot parse ") + path);
    if (n == 0) return gsrt::fail(ctx, GSRT_E_ARG, "gsrt_scene_from_ply: no vertices");
    std::vector<float> center(3ull * n), rot(4ull * n), scale(3ull * n), opacity(n), sh(with_sh ? 48ull * n : 0);
    st = gsrt_ply_read(path, center.data(), rot.data(), scale.data(), opacity.data(), with_sh ? sh.data() : nullptr);
    if (st != GSRT_OK) return gsrt::fail(ctx, st, std::string("gsrt_scene_from_ply: cannot read ") + path);
    return gsrt_scene_from_model(ctx, center.data(), rot.data(), scale.data(), opacity.data(),
                                 with_sh ? sh.data() : nullptr, n, out);
}

// dump_image.sh / RayTracing.rgen:98 debugPrintf text: "[x, y] rgba(r, g, b)" per pixel, rows in order
gsrt_status gsrt_dump_rgba_text(const char* path, const float* rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || width == 0 || height == 0) return GSRT_E_ARG;
    FILE* f = std::fopen(path, "w");
    if (!f) return GSRT_E_IO;
    bool ok = true;
    for (uint32_t y = 0; y < height && ok; ++y)
        for (uint32_t x = 0; x < width && ok; ++x) {
            const float* p = rgba + 4 * ((size_t)y * width + x);
            ok = std::fprintf(f, "[%u, %u] rgba(%f, %f, %f)\n", x, y, (double)p[0], (double)p[1], (double)p[2]) > 0;
        }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? GSRT_OK : GSRT_E_IO;
}

}  // extern "C"
