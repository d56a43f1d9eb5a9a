// gsrt_mesh.cpp -- triangle meshes co-traced with the Gaussians, host side.
//
// Reference: scene 33 adds Model::CreateSphere(vec3(200,200,0), 0.5, ..., isProcedural = false)
// (RayTracingInVulkan/src/SceneList.cpp:123) -- a triangle BLAS (Application.cpp:282-283, hit group 0,
// identity instance transform :361-362) that vulkan-sim tests with Moller-Trumbore
// (vulkan-sim/src/cuda-sim/vulkan_ray_tracing.cc:1184-1206) during the same traversal as the Gaussian AABBs.
//
// gsrt keeps a scene's triangles in HBM in leaf order of a binary BVH built here on the host (the reference
// builds its BLAS on the CPU with Embree too, lvp_acceleration_structure.c:1329-1351): per triangle three
// float4 {p0, id}, {p1 - p0}, {p2 - p0} -- the edge differences are the fp32 subtractions the reference's
// test performs (v0v1, v0v2), so precomputing them changes no rounding. k_mesh_thit (gsrt_mesh_trace.hip) walks it.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "gsrt_internal.hpp"

using gsrt::BvhNode;
using gsrt::fail;

namespace {

struct TriBox { float lo[3], hi[3], c[3]; };

constexpr uint32_t kMeshLeaf = 4;     // triangles per leaf at most
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// median split on the longest axis of the centroid box: depth <= ceil(log2(nt / kMeshLeaf)) + 1, far inside
// the kernel's per-lane stack (gsrt::kMeshStack)
struct Builder {
    const std::vector<TriBox>& tb;
    std::vector<uint32_t>& order;
    std::vector<BvhNode>& nodes;
    uint32_t depth = 0;

    void bounds(uint32_t b, uint32_t e, float lo[3], float hi[3]) const {
        for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
        for (uint32_t i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], tb[order[i]].lo[k]);
                hi[k] = std::max(hi[k], tb[order[i]].hi[k]);
            }
    }
    // child reference for [b, e): a leaf (kLeafBit | first, count in *key) or an internal node index
    uint32_t child(uint32_t b, uint32_t e, uint32_t* key, uint32_t d) {
        if (e - b <= kMeshLeaf) { *key = e - b; return gsrt::kLeafBit | b; }
        *key = 0;
        return node(b, e, d);
    }
    uint32_t node(uint32_t b, uint32_t e, uint32_t d) {
        depth = std::max(depth, d);
        const uint32_t id = (uint32_t)nodes.size();
        nodes.emplace_back();
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::min(clo[k], tb[order[i]].c[k]);
                chi[k] = std::max(chi[k], tb[order[i]].c[k]);
            }
        int ax = 0;
        for (int k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
        const uint32_t m = b + (e - b) / 2;
        std::nth_element(order.begin() + b, order.begin() + m, order.begin() + e, [&](uint32_t x, uint32_t y) {
            return tb[x].c[ax] < tb[y].c[ax] || (tb[x].c[ax] == tb[y].c[ax] && x < y);
        });
        BvhNode n;
        std::memset(&n, 0, sizeof n);
        bounds(b, m, n.l_lo, n.l_hi);
        bounds(m, e, n.r_lo, n.r_hi);
        n.l_ref = child(b, m, &n.l_key, d + 1);
        n.r_ref = child(m, e, &n.r_key, d + 1);
        nodes[id] = n;
        return id;
    }
};

}  // namespace

extern "C" {

// Model::CreateSphere (Model.cpp:566-629): vertex (i, j) of 33 x 17 at
// (cx + v sin(i0), cy + z, cz + v cos(i0)) with v = -r sin(j0), z = r cos(j0), j0 = pi j / 16, i0 = 2 pi i / 32,
// all in float with std::sin/std::cos of a float (sinf/cosf); two triangles per quad in the reference's order
gsrt_status gsrt_sphere_mesh(const float center[3], float radius, float* vertices, uint32_t* indices) {
    if (!center || !vertices || !indices) return GSRT_E_ARG;
    const int slices = 32, stacks = 16;
    const float pi = 3.14159265358979f;
    size_t q = 0;
    for (int j = 0; j <= stacks; ++j) {
        volatile float j0v = pi * j / stacks;  // volatile: sinf/cosf are called, never folded by the compiler
        const float j0 = j0v;
        const float v = radius * -std::sin(j0);
        const float z = radius * std::cos(j0);
        for (int i = 0; i <= slices; ++i) {
            volatile float i0v = 2 * pi * i / slices;
            const float i0 = i0v;
            vertices[q++] = center[0] + v * std::sin(i0);
            vertices[q++] = center[1] + z;
            vertices[q++] = center[2] + v * std::cos(i0);
        }
    }
    size_t t = 0;
    for (int j = 0; j < stacks; ++j)
        for (int i = 0; i < slices; ++i) {
            const uint32_t j0 = (uint32_t)(j * (slices + 1)), j1 = (uint32_t)((j + 1) * (slices + 1));
            const uint32_t i0 = (uint32_t)i, i1 = (uint32_t)(i + 1);
            const uint32_t tri[6] = {j0 + i0, j1 + i0, j1 + i1, j0 + i0, j1 + i1, j0 + i1};
            for (uint32_t x : tri) indices[t++] = x;
        }
    return GSRT_OK;
}

uint32_t gsrt_scene_mesh_triangles(const gsrt_scene* sc) { return sc ? sc->ntri : 0u; }

gsrt_status gsrt_scene_add_mesh(gsrt_scene* sc, const float* vertices, uint32_t nv, const uint32_t* indices,
                                uint32_t nt) {
    if (!sc || (nt && (!vertices || !indices))) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (nt == 0) return GSRT_OK;
    if ((uint64_t)sc->ntri + nt >= (uint64_t)gsrt::kLeafBit) return fail(ctx, GSRT_E_ARG, "too many triangles");
    for (uint64_t i = 0; i < 3ull * nt; ++i)
        if (indices[i] >= nv) return fail(ctx, GSRT_E_ARG, "mesh index out of range");
    for (uint64_t i = 0; i < 3ull * nv; ++i)
        if (!std::isfinite(vertices[i])) return fail(ctx, GSRT_E_ARG, "non-finite mesh vertex");
    // triangles of every mesh added so far, in the order added: p0 p1 p2 (9 floats)
    const size_t old = sc->h_tris.size();
    sc->h_tris.resize(old + 9ull * nt);
    for (uint32_t t = 0; t < nt; ++t)
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) sc->h_tris[old + 9ull * t + 3 * v + k] = vertices[3ull * indices[3ull * t + v] + k];
    const uint32_t n = (uint32_t)(sc->h_tris.size() / 9);

    std::vector<TriBox> tb(n);
    for (uint32_t t = 0; t < n; ++t) {
        const float* p = &sc->h_tris[9ull * t];
        for (int k = 0; k < 3; ++k) {
            tb[t].lo[k] = std::min(p[k], std::min(p[3 + k], p[6 + k]));
            tb[t].hi[k] = std::max(p[k], std::max(p[3 + k], p[6 + k]));
            tb[t].c[k] = 0.5f * (tb[t].lo[k] + tb[t].hi[k]);
        }
    }
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::vector<BvhNode> nodes;
    Builder B{tb, order, nodes};
    if (n <= kMeshLeaf) {  // one root whose left child is the only leaf; the right child is empty
        BvhNode r;
        std::memset(&r, 0, sizeof r);
        B.bounds(0, n, r.l_lo, r.l_hi);
        r.l_ref = gsrt::kLeafBit;
        r.l_key = n;
        r.r_ref = kEmpty;
        nodes.push_back(r);
    } else {
        B.node(0, n, 0);
    }
    if (B.depth + 2 > gsrt::kMeshStack) {
        sc->h_tris.resize(old);
        return fail(ctx, GSRT_E_ARG, "mesh BVH too deep");
    }
    std::vector<float4> dev(3ull * n);
    for (uint32_t i = 0; i < n; ++i) {
        const float* p = &sc->h_tris[9ull * order[i]];
        uint32_t id = order[i];
        float idf;
        std::memcpy(&idf, &id, 4);
        dev[3ull * i + 0] = make_float4(p[0], p[1], p[2], idf);
        dev[3ull * i + 1] = make_float4(p[3] - p[0], p[4] - p[1], p[5] - p[2], 0.0f);  // v0v1
        dev[3ull * i + 2] = make_float4(p[6] - p[0], p[7] - p[1], p[8] - p[2], 0.0f);  // v0v2
    }
    (void)hipSetDevice(ctx->device);
    gsrt_status s = gsrt::sync_all(ctx);  // earlier frames may still read the old mesh
    if (s != GSRT_OK) {
        sc->h_tris.resize(old);
        return s;
    }
    (void)hipFree(sc->d_tris);
    (void)hipFree(sc->d_mesh_nodes);
    sc->d_tris = nullptr;
    sc->d_mesh_nodes = nullptr;
    sc->ntri = 0;
    GSRT_HIP(ctx, hipMalloc(&sc->d_tris, sizeof(float4) * dev.size()));
    GSRT_HIP(ctx, hipMalloc(&sc->d_mesh_nodes, sizeof(BvhNode) * nodes.size()));
    GSRT_HIP(ctx, hipMemcpy(sc->d_tris, dev.data(), sizeof(float4) * dev.size(), hipMemcpyHostToDevice));
    GSRT_HIP(ctx, hipMemcpy(sc->d_mesh_nodes, nodes.data(), sizeof(BvhNode) * nodes.size(), hipMemcpyHostToDevice));
    sc->ntri = n;
    return GSRT_OK;
}

}  // extern "C"
