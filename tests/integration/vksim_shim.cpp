// vksim_shim.cpp -- the driver-side drop-in of INTEGRATION.md §2, compiled: the vulkan-sim entry points that
// lavapipe calls (mesa-vulkan-sim/src/gallium/frontends/lavapipe/gpgpusim_calls_from_mesa.h:39-59), implemented
// over include/gsrt.h instead of the PTX simulator. Built and exercised by tests/test_integration.py.
//
//   gpgpusim_setDescriptor(set, binding, address, size, type)   descriptor bindings of the Gauss pipeline
//       (RayTracingPipeline.cpp:32-77): 2 output image (rgba8, GaussTracing.rgen:14), 3 UBO, 12 GaussParam[]
//       (one per model, zeros for non-Gauss models, Scene.cpp:125-141), 13 NextK[ray][8] {depth, alpha},
//       14 RayInfo[ray] {Depth, GaussNum} (rgen:15-16)
//   gpgpusim_setGeometries(geometries, count)                  the BLAS geometries of one build; each Gaussian
//       BLAS holds one AABB (BottomLevelGeometry::AddGeometryGauss, Application.cpp:281)
//   gpgpusim_vkCmdTraceRaysKHR(..., W, H, D, ...)              the dispatch: scene upload + LBVH on the first
//       trace, then one REF frame; the bound NextK / RayInfo buffers receive the per-ray state the reference's
//       shaders leave there, the image the frame's pixels
//
// The Vulkan structures are declared here field for field from the Vulkan spec (VkAccelerationStructureGeometryKHR
// and its union members), with their sizes asserted, so the shim needs no Vulkan headers.
#include <cstdint>
#include <cstring>
#include <vector>

#include "gsrt.h"

namespace {

struct VkAabbsData { uint32_t sType; const void* pNext; const void* data; uint64_t stride; };
struct VkTrianglesData {
    uint32_t sType; const void* pNext; uint32_t vertexFormat; const void* vertexData; uint64_t vertexStride;
    uint32_t maxVertex; uint32_t indexType; const void* indexData; const void* transformData;
};
union VkGeometryData { VkTrianglesData triangles; VkAabbsData aabbs; };
struct VkGeometry { uint32_t sType; const void* pNext; uint32_t geometryType; VkGeometryData geometry; uint32_t flags; };
static_assert(sizeof(VkTrianglesData) == 64 && sizeof(VkAabbsData) == 32, "Vulkan geometry data layouts");
static_assert(offsetof(VkGeometry, geometry) == 24 && sizeof(VkGeometry) == 96, "VkAccelerationStructureGeometryKHR");
constexpr uint32_t kGeometryAabbs = 1;  // VK_GEOMETRY_TYPE_AABBS_KHR

struct Binding { void* address = nullptr; uint32_t size = 0; };
struct Shim {
    gsrt_ctx* ctx = nullptr;
    gsrt_scene* scene = nullptr;
    Binding bind[16];
    std::vector<gsrt_aabb> aabbs;  // every AABB geometry seen, in build order
    int status = GSRT_OK;
} g;

}  // namespace

extern "C" {

void gpgpusim_setDescriptor(uint32_t setID, uint32_t descID, void* address, uint32_t size, uint32_t type) {
    (void)type;
    if (setID == 0 && descID < 16) g.bind[descID] = Binding{address, size};
}

void gpgpusim_setGeometries(const void* pGeometries, uint32_t geometryCount) {
    const VkGeometry* geo = static_cast<const VkGeometry*>(pGeometries);
    for (uint32_t i = 0; i < geometryCount; ++i)
        if (geo[i].geometryType == kGeometryAabbs) {
            gsrt_aabb a;
            std::memcpy(&a, geo[i].geometry.aabbs.data, sizeof a);
            g.aabbs.push_back(a);
        }
}

void gpgpusim_vkCmdTraceRaysKHR(void* raygen_sbt, void* miss_sbt, void* hit_sbt, void* callable_sbt, bool is_indirect,
                                uint32_t launch_width, uint32_t launch_height, uint32_t launch_depth,
                                uint64_t launch_size_addr) {
    (void)raygen_sbt; (void)miss_sbt; (void)hit_sbt; (void)callable_sbt; (void)is_indirect; (void)launch_size_addr;
    g.status = GSRT_E_ARG;
    if (launch_depth != 1 || !g.bind[3].address || !g.bind[12].address) return;
    if (!g.ctx && (g.status = gsrt_create(&g.ctx, 0)) != GSRT_OK) return;
    if (!g.scene) {  // first trace: the Gaussian models (non-zero GaussParam entries) paired with the AABBs in order
        const gsrt_gauss_param* all = static_cast<const gsrt_gauss_param*>(g.bind[12].address);
        const uint32_t models = g.bind[12].size / sizeof(gsrt_gauss_param);
        std::vector<gsrt_gauss_param> params;
        for (uint32_t m = 0; m < models; ++m) {
            static const gsrt_gauss_param zero{};
            if (std::memcmp(&all[m], &zero, sizeof zero) != 0) params.push_back(all[m]);
        }
        if (params.size() != g.aabbs.size()) return;
        if ((g.status = gsrt_scene_from_params(g.ctx, params.data(), g.aabbs.data(), (uint32_t)params.size(), nullptr,
                                               &g.scene)) != GSRT_OK ||
            (g.status = gsrt_build_bvh(g.scene)) != GSRT_OK)
            return;
    }
    gsrt_ubo ubo;
    std::memcpy(&ubo, g.bind[3].address, sizeof ubo);
    if (ubo.width != launch_width || ubo.height != launch_height) return;
    const size_t n = (size_t)launch_width * launch_height;
    std::vector<float> rgba(4 * n);
    std::vector<gsrt_raystate> rs(n);
    if ((g.status = gsrt_render(g.scene, &ubo, GSRT_MODE_REF, 0, rgba.data(), rs.data())) != GSRT_OK) return;
    if (g.bind[2].address && g.bind[2].size >= 4 * n) {  // rgba8 (GaussTracing.rgen:14)
        uint8_t* img = static_cast<uint8_t*>(g.bind[2].address);
        for (size_t i = 0; i < 4 * n; ++i) {
            const float v = rgba[i] < 0.0f ? 0.0f : (rgba[i] > 1.0f ? 1.0f : rgba[i]);
            img[i] = (uint8_t)(v * 255.0f + 0.5f);
        }
    }
    if (g.bind[13].address && g.bind[13].size >= n * 64) {  // NextK[ray][8] {depth, alpha}
        float* nk = static_cast<float*>(g.bind[13].address);
        for (size_t r = 0; r < n; ++r) std::memcpy(nk + 16 * r, rs[r].k, 64);
    }
    if (g.bind[14].address && g.bind[14].size >= n * 8) {  // RayInfo {float Depth; int GaussNum}: the raw count
        char* ri = static_cast<char*>(g.bind[14].address);
        for (size_t r = 0; r < n; ++r) {
            std::memcpy(ri + 8 * r, &rs[r].depth, 4);
            std::memcpy(ri + 8 * r + 4, &rs[r].gauss_num_raw, 4);
        }
    }
    g.status = GSRT_OK;
}

// test hooks: the status of the last trace, and teardown
int vksim_shim_status(void) { return g.status; }
void vksim_shim_reset(void) {
    if (g.scene) gsrt_destroy_scene(g.scene);
    if (g.ctx) gsrt_destroy(g.ctx);
    g = Shim{};
}

}  // extern "C"
