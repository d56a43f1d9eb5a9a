// vksim_shim.cpp -- the driver-side drop-in of INTEGRATION.md §2, compiled: a replacement for vulkan-sim's
// simulator library (vulkan-sim/src/cuda-sim/gpgpusim_calls_from_mesa.cc) that exports every extern "C" entry
// point lavapipe declares and calls (mesa-vulkan-sim/src/gallium/frontends/lavapipe/gpgpusim_calls_from_mesa.h:
// 38-59) and implements the Gaussian render path over include/gsrt.h instead of the PTX simulator.
//
// Call sites in lavapipe, in the order the RayTracingInVulkan app reaches them for --scene 33 --shader-type 6:
//   gpgpusim_allocBuffer        lvp_BindBufferMemory2 / lvp_BindImageMemory2 (lvp_device.c:2620,2676): every
//                               buffer and image; the returned pointer is stored as pBuffer_gpgpusim /
//                               pmem_gpgpusim and is what descriptors later carry (lvp_descriptor_set.c:591,617)
//   gpgpusim_registerShader     vsim_compile_ray_tracing_pipeline (lvp_pipeline_rt.c:162): one call per stage,
//                               lavapipe asserts the returned id equals the stage index
//   gpgpusim_setPipelineInfo    lvp_CreateRayTracingPipelinesKHR (lvp_pipeline_rt.c:259)
//   gpgpusim_allocBLAS/TLAS     lvp_CreateAccelerationStructureKHR (lvp_acceleration_structure.c:261-264)
//   gpgpusim_setGeometries      lvp_cpu_build_acceleration_structures, once per build info (:1195)
//   gpgpusim_pass_child_addr    add_bvh_instances, one per TLAS instance (:1081)
//   gpgpusim_addTreelets        after a TLAS build (:1391)
//   gpgpusim_setDescriptorSet   handle_descriptor_sets for the ray-tracing bind point (lvp_execute.c:1551)
//   gpgpusim_vkCmdTraceRaysKHR  handle_trace_ray (lvp_execute.c:1220)
// plus gpgpusim_setDescriptor (the per-binding setter vulkan-sim also exports) and gpgpusim_testTraversal (a no-op
// in vulkan-sim too).
//
// What a trace does (vulkan-sim: VulkanRayTracing::vkCmdTraceRaysKHR, vulkan_ray_tracing.cc:1478-1652):
//   - bindings are resolved from the lvp_descriptor_set the way getDescriptorAddress does (:1957-1988): storage /
//     uniform buffers -> info.ssbo/ubo.pmem (the allocBuffer alias; buffer_offset is not added, as in vulkan-sim),
//     acceleration structure -> info.ubo.pmem + buffer_offset, storage image -> the descriptor itself;
//   - the scene is assembled from what the driver handed over: the TLAS instances (arrayOfPointers or packed
//     VkAccelerationStructureInstanceKHR, identity transforms, Application.cpp:339-367) name their BLAS by device
//     address (== the allocBLAS root, lvp_acceleration_structure.c:300) and their hit group by SBT record offset.
//     A procedural hit group makes the instance a Gaussian: GaussParam[instanceCustomIndex] from binding 12 and the
//     BLAS's AABB. A triangle hit group makes it a mesh, read from the buffers the triangle closest-hit shader
//     indexes (bindings 4 Vertices, 5 Indices, 7 Offsets[instanceCustomIndex], Scene.cpp:46-50,146-149);
//   - one REF frame (GaussTracing.rgen / .rint / .rchit) renders through gsrt_render;
//   - results land where the shaders leave them: NextK (binding 13) and RayInfo (binding 14) in the app's buffers,
//     and the P3 PPM that image_store writes (vulkan_ray_tracing.cc:2216-2247; the lavapipe build stores no pixels
//     into the image memory, and opens but never writes image.binary, :1506-1517).
//
// Two values never reach the simulator and are taken from the app's fixed conventions, as cited at their use:
// the AABB build range (primitiveOffset) and the instance count (the build range's primitiveCount).
//
// The lavapipe and Vulkan structures are mirrored below with their offsets asserted; the offsets are the ones
// oracle/ref/lvp_layout_probe.c measures on the reference's own headers (tests/golden/lvp_layout.json, checked by
// tests/test_integration.py through vksim_shim_layout_json()).
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gsrt.h"

namespace {

// ---- Vulkan API structures (vulkan_core.h; sizes from the reference's header, lvp_layout.json) ----------------
struct VkTrianglesData {
    uint32_t sType; const void* pNext; uint32_t vertexFormat; const void* vertexData; uint64_t vertexStride;
    uint32_t maxVertex; uint32_t indexType; const void* indexData; const void* transformData;
};
struct VkAabbsData { uint32_t sType; const void* pNext; const void* data; uint64_t stride; };
struct VkInstancesData { uint32_t sType; const void* pNext; uint32_t arrayOfPointers; const void* data; };
union VkGeometryData { VkTrianglesData triangles; VkAabbsData aabbs; VkInstancesData instances; };
struct VkGeometry { uint32_t sType; const void* pNext; uint32_t geometryType; VkGeometryData geometry; uint32_t flags; };
struct VkInstance {  // VkAccelerationStructureInstanceKHR
    float transform[12]; uint32_t custom_index_mask; uint32_t sbt_offset_flags; uint64_t as_reference;
};
struct VkStage { uint32_t sType; const void* pNext; uint32_t flags; uint32_t stage; uint64_t module;
                 const char* pName; const void* pSpecializationInfo; };
struct VkGroup { uint32_t sType; const void* pNext; uint32_t type; uint32_t generalShader; uint32_t closestHitShader;
                 uint32_t anyHitShader; uint32_t intersectionShader; const void* pShaderGroupCaptureReplayHandle; };
struct VkRtPipelineInfo {
    uint32_t sType; const void* pNext; uint32_t flags; uint32_t stageCount; const VkStage* pStages;
    uint32_t groupCount; const VkGroup* pGroups; uint32_t maxPipelineRayRecursionDepth; const void* pLibraryInfo;
    const void* pLibraryInterface; const void* pDynamicState; uint64_t layout; uint64_t basePipelineHandle;
    int32_t basePipelineIndex;
};
static_assert(sizeof(VkGeometry) == 96 && offsetof(VkGeometry, geometryType) == 16 &&
              offsetof(VkGeometry, geometry) == 24 && offsetof(VkGeometry, flags) == 88, "geometry");
static_assert(offsetof(VkTrianglesData, vertexFormat) == 16 && offsetof(VkTrianglesData, vertexData) == 24 &&
              offsetof(VkTrianglesData, vertexStride) == 32 && offsetof(VkTrianglesData, maxVertex) == 40 &&
              offsetof(VkTrianglesData, indexType) == 44 && offsetof(VkTrianglesData, indexData) == 48, "triangles");
static_assert(offsetof(VkAabbsData, data) == 16 && offsetof(VkAabbsData, stride) == 24, "aabbs");
static_assert(offsetof(VkInstancesData, arrayOfPointers) == 16 && offsetof(VkInstancesData, data) == 24, "instances");
static_assert(sizeof(VkInstance) == 64 && offsetof(VkInstance, as_reference) == 56, "instance");
static_assert(sizeof(VkStage) == 48 && offsetof(VkStage, stage) == 20, "shader stage");
static_assert(sizeof(VkGroup) == 48 && offsetof(VkGroup, type) == 16 && offsetof(VkGroup, intersectionShader) == 32,
              "shader group");
static_assert(sizeof(VkRtPipelineInfo) == 104 && offsetof(VkRtPipelineInfo, stageCount) == 20 &&
              offsetof(VkRtPipelineInfo, pStages) == 24 && offsetof(VkRtPipelineInfo, groupCount) == 32 &&
              offsetof(VkRtPipelineInfo, pGroups) == 40, "pipeline create info");

constexpr uint32_t kGeomTriangles = 0, kGeomAabbs = 1, kGeomInstances = 2;  // VkGeometryTypeKHR
constexpr uint32_t kDescStorageImage = 3, kDescUniformBuffer = 6, kDescStorageBuffer = 7;
constexpr uint32_t kDescAccelStruct = 1000150000;
constexpr uint32_t kGroupTriangles = 1, kGroupProcedural = 2;  // VkRayTracingShaderGroupTypeKHR
constexpr uint32_t kFormatRGB32F = 106, kFormatRGBA32F = 109, kFormatBGRA8 = 44, kIndexU32 = 1;
constexpr uint32_t kShaderUnused = ~0u;

// ---- lavapipe structures (lvp_private.h:257-265, 284-371 of the fork) ------------------------------------------
struct PipeBuffer {  // pipe_constant_buffer / pipe_shader_buffer prefix (p_state.h:670-688): the fork adds pmem
    void* buffer; void* pmem; uint32_t buffer_offset; uint32_t buffer_size;
};
struct LvpDescriptor {  // struct lvp_descriptor: type + union lvp_descriptor_info (40 B)
    uint32_t type;
    union {
        PipeBuffer buf;                                        // info.ubo / info.ssbo
        struct { void* resource; void* image; } image_view;    // pipe_image_view: resource, the fork's image
        uint8_t bytes[40];
    } info;
};
static_assert(sizeof(LvpDescriptor) == 48 && offsetof(LvpDescriptor, info) == 8, "lvp_descriptor");
constexpr size_t kDescPmem = offsetof(LvpDescriptor, info.buf.pmem);                 // 16
constexpr size_t kDescBufOffset = offsetof(LvpDescriptor, info.buf.buffer_offset);    // 24
constexpr size_t kDescBufSize = offsetof(LvpDescriptor, info.buf.buffer_size);        // 28
constexpr size_t kDescImage = offsetof(LvpDescriptor, info.image_view.image);         // 16
static_assert(kDescPmem == 16 && kDescBufOffset == 24 && kDescBufSize == 28 && kDescImage == 16, "descriptor info");
// struct lvp_descriptor_set: vk_object_base (64 B) base; layout*; list_head link; lvp_descriptor descriptors[]
constexpr size_t kSetLayout = 64, kSetDescriptors = 88;
// struct lvp_descriptor_set_layout: vk_descriptor_set_layout (80 B), u32 immutable_sampler_count, u16 binding_count,
// u16 size, u16 shader_stages, 15 x 32-B per-stage counts, u16 dynamic_offset_count, then binding[] (8-aligned)
constexpr size_t kLayoutBindingCount = 84, kLayoutBindings = 576;
// struct lvp_descriptor_set_binding_layout: u16 descriptor_index, VkDescriptorType type, u16 array_size, bool valid,
// i16 dynamic_index, 15 x 8 i16 per-stage indices, immutable_samplers*
constexpr size_t kBindingSize = 264, kBindingDescIndex = 0, kBindingType = 4;
// struct lvp_image { struct vk_image vk; ... }: vk_object_base, create_flags, image_type, format, extent, mip_levels,
// array_layers, samples, tiling
constexpr size_t kImageFormat = 72, kImageExtent = 76, kImageTiling = 100;

template <class T> T rd(const void* base, size_t off) { T v; std::memcpy(&v, static_cast<const char*>(base) + off, sizeof v); return v; }

// ---- what the driver has handed over --------------------------------------------------------------------------
struct Range { const char* base; uint64_t size; };
struct Geometry {                  // one VkAccelerationStructureGeometryKHR, copied at setGeometries
    uint32_t type = 0;
    gsrt_aabb aabb{};              // AABBs: the BLAS's box, read while the build runs
    const void* vertex_data = nullptr; uint64_t vertex_stride = 0; uint32_t max_vertex = 0, vertex_format = 0;
    const void* index_data = nullptr; uint32_t index_type = 0;
    const void* instances = nullptr; bool array_of_pointers = false;
};
struct Blas { void* root; uint64_t size; std::vector<Geometry> geoms; bool built = false; };
struct Binding { const void* addr = nullptr; uint64_t size = 0; uint32_t type = ~0u; const void* desc = nullptr; };

struct Shim {
    gsrt_ctx* ctx = nullptr;
    gsrt_scene* scene = nullptr;
    uint64_t scene_gen = ~0ull, gen = 0;     // scene rebuilt when an AS build happened since
    std::vector<Range> buffers;              // allocBuffer registrations (aliases are the host pointers)
    std::vector<std::pair<uint32_t, uint32_t>> shaders;  // registerShader: (id, gl_shader_stage)
    std::vector<VkGroup> groups;             // setPipelineInfo
    std::vector<uint32_t> stage_flags;
    std::vector<Blas> blas;                  // allocBLAS order
    size_t blas_builds = 0;                  // setGeometries calls for bottom-level builds so far
    void* tlas_root = nullptr; uint64_t tlas_size = 0;
    std::vector<Geometry> tlas_geoms;        // the last top-level build's geometries
    const void* tlas_built = nullptr;        // addTreelets
    std::vector<void*> child_addrs;          // pass_child_addr
    const void* set = nullptr;               // setDescriptorSet (first one; vulkan_ray_tracing.cc:1264-1274)
    Binding legacy[32];                      // setDescriptor(set 0, binding, ...)
    std::string ppm_name;                    // first image_store names the file (vulkan_ray_tracing.cc:2222-2239)
    bool image_binary_opened = false;
    int status = GSRT_OK;
    std::string error;
    // the scene as assembled from the driver's objects (host copies), uploaded to gsrt when it changes
    std::vector<gsrt_gauss_param> params;
    std::vector<gsrt_aabb> aabbs;
    std::vector<float> verts;
    std::vector<uint32_t> idx;
    uint64_t assembled_gen = ~0ull;
} g;

int fail(int status, const std::string& why) { g.status = status; g.error = why; return status; }

const Range* find_range(const void* p, uint64_t len = 0) {
    for (const Range& r : g.buffers)
        if (static_cast<const char*>(p) >= r.base && static_cast<const char*>(p) + len <= r.base + r.size) return &r;
    return nullptr;
}

// getDescriptorAddress (vulkan_ray_tracing.cc:1957-1988) plus the binding's byte size
bool resolve(uint32_t binding, Binding* out) {
    *out = Binding{};
    if (g.set) {
        const void* layout = rd<const void*>(g.set, kSetLayout);
        if (!layout || binding >= rd<uint16_t>(layout, kLayoutBindingCount)) return false;
        const char* bl = static_cast<const char*>(layout) + kLayoutBindings + binding * kBindingSize;
        const uint16_t di = rd<uint16_t>(bl, kBindingDescIndex);
        const char* desc = static_cast<const char*>(g.set) + kSetDescriptors + di * sizeof(LvpDescriptor);
        out->type = rd<uint32_t>(desc, 0);
        if (out->type != rd<uint32_t>(bl, kBindingType)) return false;
        out->desc = desc;
        switch (out->type) {
            case kDescStorageImage: out->addr = desc; return true;
            case kDescUniformBuffer:
            case kDescStorageBuffer:
                out->addr = rd<const void*>(desc, kDescPmem);
                out->size = rd<uint32_t>(desc, kDescBufSize);
                return out->addr != nullptr;
            case kDescAccelStruct:
                out->addr = rd<const char*>(desc, kDescPmem) + rd<uint32_t>(desc, kDescBufOffset);
                return true;
            default: return false;  // vulkan-sim aborts on other types; the Gauss pipeline has none it reads
        }
    }
    if (binding < 32 && g.legacy[binding].addr) { *out = g.legacy[binding]; return true; }
    return false;
}

// Assemble the scene from the TLAS instances (see the header comment) into host arrays.
int assemble() {
    Binding tlas, params;
    if (!resolve(0, &tlas) || tlas.type != kDescAccelStruct) return fail(GSRT_E_ARG, "binding 0 is not a TLAS");
    if (!g.tlas_root || tlas.addr != g.tlas_root) return fail(GSRT_E_ARG, "binding 0 is not the registered TLAS");
    if (!g.tlas_built) return fail(GSRT_E_STATE, "the TLAS was never built (no gpgpusim_addTreelets)");
    if (g.tlas_geoms.size() != 1 || g.tlas_geoms[0].type != kGeomInstances)
        return fail(GSRT_E_ARG, "the TLAS build must hold one instances geometry");
    if (!resolve(12, &params) || params.type != kDescStorageBuffer) return fail(GSRT_E_ARG, "binding 12 (GaussParam)");
    const uint32_t n_models = static_cast<uint32_t>(params.size / sizeof(gsrt_gauss_param));
    // The instance count is the TLAS build range's primitiveCount, which the simulator never receives: the app puts
    // exactly one instance per model (Application.cpp:339-367), i.e. one per BLAS, into a buffer of its own.
    const Geometry& ig = g.tlas_geoms[0];
    const size_t n_inst = g.blas.size();
    if (!ig.array_of_pointers && !find_range(ig.instances, n_inst * sizeof(VkInstance)))
        return fail(GSRT_E_ARG, "TLAS instances outside any allocated buffer");
    // hit groups: the SBT's hit region starts at the first non-general group (RayTracingPipeline.cpp:405-416)
    size_t hit_base = 0;
    while (hit_base < g.groups.size() && g.groups[hit_base].type != kGroupTriangles &&
           g.groups[hit_base].type != kGroupProcedural)
        ++hit_base;

    struct G { uint32_t model; gsrt_gauss_param p; gsrt_aabb a; };
    std::vector<G> gauss;
    std::vector<float> verts;
    std::vector<uint32_t> idx;
    uint32_t mesh_nv = 0;
    for (size_t i = 0; i < n_inst; ++i) {
        VkInstance inst;
        const void* src = ig.array_of_pointers ? static_cast<const void* const*>(ig.instances)[i]
                                               : static_cast<const VkInstance*>(ig.instances) + i;
        std::memcpy(&inst, src, sizeof inst);
        static const float kIdentity[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        if (std::memcmp(inst.transform, kIdentity, sizeof kIdentity) != 0)
            return fail(GSRT_E_ARG, "instance transforms must be identity (Application.cpp:361-362)");
        const uint32_t model = inst.custom_index_mask & 0xffffffu, sbt = inst.sbt_offset_flags & 0xffffffu;
        size_t b = 0;
        while (b < g.blas.size() && reinterpret_cast<uint64_t>(g.blas[b].root) != inst.as_reference) ++b;
        if (b == g.blas.size() || !g.blas[b].built || g.blas[b].geoms.size() != 1)
            return fail(GSRT_E_ARG, "instance " + std::to_string(i) + " names no built single-geometry BLAS");
        if (hit_base + sbt >= g.groups.size()) return fail(GSRT_E_ARG, "instance SBT offset past the hit groups");
        const VkGroup& grp = g.groups[hit_base + sbt];
        const Geometry& geo = g.blas[b].geoms[0];
        if (grp.type == kGroupProcedural) {  // a Gaussian (Gauss hit group, RayTracingPipeline.cpp:388-396)
            if (geo.type != kGeomAabbs || model >= n_models)
                return fail(GSRT_E_ARG, "Gaussian instance without an AABB BLAS or GaussParam entry");
            if (grp.intersectionShader == kShaderUnused || grp.intersectionShader >= g.stage_flags.size())
                return fail(GSRT_E_ARG, "procedural hit group without an intersection shader");
            G e{model, {}, geo.aabb};
            std::memcpy(&e.p, static_cast<const char*>(params.addr) + model * sizeof(gsrt_gauss_param), sizeof e.p);
            gauss.push_back(e);
        } else if (grp.type == kGroupTriangles) {  // a mesh: the buffers RayTracing.rchit indexes
            Binding vb, ib, ob;
            if (geo.type != kGeomTriangles || !resolve(4, &vb) || !resolve(5, &ib) || !resolve(7, &ob))
                return fail(GSRT_E_ARG, "triangle instance without vertex/index/offset bindings");
            if (geo.vertex_format != kFormatRGB32F || geo.index_type != kIndexU32 || geo.vertex_stride < 12 ||
                geo.vertex_data != vb.addr || geo.index_data != ib.addr)
                return fail(GSRT_E_ARG, "triangle geometry is not the app's vertex / index buffers");
            // Offsets[model] = {first index, first vertex} (Scene.cpp:49-50); the BLAS build range used the same
            // values (BottomLevelGeometry.cpp: firstVertex = vertexOffset / sizeof(Vertex), primitiveOffset =
            // indexOffset), and the next model's first index (or the end of Indices) bounds the index count.
            const uint32_t n_off = static_cast<uint32_t>(ob.size / 8), n_idx_all = static_cast<uint32_t>(ib.size / 4);
            if (model >= n_off) return fail(GSRT_E_ARG, "triangle instance past the Offsets buffer");
            const uint32_t* off = static_cast<const uint32_t*>(ob.addr);
            const uint32_t first = off[2 * model], first_v = off[2 * model + 1];
            const uint32_t end = model + 1 < n_off ? off[2 * (model + 1)] : n_idx_all;
            if (end < first || end > n_idx_all || (end - first) % 3) return fail(GSRT_E_ARG, "bad index range");
            const uint32_t nv = geo.max_vertex;
            if ((uint64_t)(first_v + nv) * geo.vertex_stride > vb.size) return fail(GSRT_E_ARG, "bad vertex range");
            const uint32_t* src_idx = static_cast<const uint32_t*>(ib.addr) + first;
            for (uint32_t k = 0; k < end - first; ++k) {
                if (src_idx[k] >= nv) return fail(GSRT_E_ARG, "index past maxVertex");
                idx.push_back(mesh_nv + src_idx[k]);
            }
            for (uint32_t v = 0; v < nv; ++v) {
                float pos[3];
                std::memcpy(pos, static_cast<const char*>(vb.addr) + (uint64_t)(first_v + v) * geo.vertex_stride, 12);
                verts.insert(verts.end(), pos, pos + 3);
            }
            mesh_nv += nv;
        } else {
            return fail(GSRT_E_ARG, "instance hit group is neither triangles nor procedural");
        }
    }
    // Gaussians in model order: the order of GaussParam / AABB entries in the app's arrays (Scene.cpp:125-141)
    std::vector<gsrt_gauss_param> p;
    std::vector<gsrt_aabb> a;
    for (uint32_t m = 0; m < n_models; ++m)
        for (const G& e : gauss)
            if (e.model == m) { p.push_back(e.p); a.push_back(e.a); }
    if (p.size() != gauss.size()) return fail(GSRT_E_ARG, "two instances share a model index");

    g.params = std::move(p);
    g.aabbs = std::move(a);
    g.verts = std::move(verts);
    g.idx = std::move(idx);
    g.assembled_gen = g.gen;
    return GSRT_OK;
}

int upload() {
    if (g.scene) { gsrt_destroy_scene(g.scene); g.scene = nullptr; }
    int s = gsrt_scene_from_params(g.ctx, g.params.data(), g.aabbs.data(), static_cast<uint32_t>(g.params.size()),
                                   nullptr, &g.scene);
    if (s == GSRT_OK && !g.idx.empty())
        s = gsrt_scene_add_mesh(g.scene, g.verts.data(), static_cast<uint32_t>(g.verts.size() / 3), g.idx.data(),
                                static_cast<uint32_t>(g.idx.size() / 3));
    if (s == GSRT_OK) s = gsrt_build_bvh(g.scene);
    if (s != GSRT_OK) return fail(s, std::string("scene: ") + gsrt_last_error(g.ctx));
    g.scene_gen = g.assembled_gen;
    return GSRT_OK;
}

int trace(uint32_t w, uint32_t h, uint32_t d) {
    if (d != 1) return fail(GSRT_E_ARG, "launch depth must be 1 (vulkan_ray_tracing.cc:1543)");
    if (!g.image_binary_opened) {  // vulkan_ray_tracing.cc:1506-1517: opened (truncated) once, never written here
        const char* name = std::getenv("VULKAN_IMAGE_FILE_NAME");
        if (FILE* f = std::fopen(name ? name : "image.binary", "wb")) std::fclose(f);
        g.image_binary_opened = true;
    }
    Binding ubo_b, lut_b;
    if (!resolve(3, &ubo_b) || ubo_b.type != kDescUniformBuffer || ubo_b.size < sizeof(gsrt_ubo))
        return fail(GSRT_E_ARG, "binding 3 (UniformBufferObject)");
    // the shaders' LinearExp table (binding 15, ExpLUT.hpp generateExpLUT(256, 0, 8)) must be the one gsrt evaluates
    if (resolve(15, &lut_b)) {
        float lut[512];
        if (gsrt_exp_lut(lut) != GSRT_OK || lut_b.size < sizeof lut || std::memcmp(lut, lut_b.addr, sizeof lut) != 0)
            return fail(GSRT_E_ARG, "binding 15 is not generateExpLUT(256, 0, 8)");
    }
    if (g.assembled_gen != g.gen)
        if (int s = assemble()) return s;
    if (!g.ctx && gsrt_create(&g.ctx, 0) != GSRT_OK) return fail(GSRT_E_DEVICE, "gsrt_create failed (no GPU)");
    if (!g.scene || g.scene_gen != g.assembled_gen)
        if (int s = upload()) return s;
    gsrt_ubo ubo;
    std::memcpy(&ubo, ubo_b.addr, sizeof ubo);
    if (ubo.width != w || ubo.height != h) return fail(GSRT_E_ARG, "UBO extent differs from the launch");
    const size_t n = static_cast<size_t>(w) * h;
    std::vector<float> rgba(4 * n);
    std::vector<gsrt_raystate> rs(n);
    if (int s = gsrt_render(g.scene, &ubo, GSRT_MODE_REF, 0, rgba.data(), rs.data()))
        return fail(s, std::string("render: ") + gsrt_last_error(g.ctx));

    Binding nk_b, ri_b, img_b;
    if (resolve(13, &nk_b) && nk_b.type == kDescStorageBuffer) {
        // NextK[ray][8] {depth, alpha}; ray = x + W*y (the shaders' x + 16*y is only valid at W = 16).
        // rgen resets only the depths each round (rgen:54-57): a slot no insert of this frame reached keeps the
        // alpha the buffer held before the trace (Scene.cpp:38-45's -1, or the previous frame's).
        float* nk = static_cast<float*>(const_cast<void*>(nk_b.addr));
        const size_t rays = std::min<size_t>(n, nk_b.size / 64);
        for (size_t r = 0; r < rays; ++r)
            for (int j = 0; j < 8; ++j) {
                nk[16 * r + 2 * j] = rs[r].k[j][0];
                if (rs[r].k[j][1] != -1.0f) nk[16 * r + 2 * j + 1] = rs[r].k[j][1];
            }
    }
    if (resolve(14, &ri_b) && ri_b.type == kDescStorageBuffer) {  // RayInfo {float Depth; int GaussNum} (raw count)
        char* ri = static_cast<char*>(const_cast<void*>(ri_b.addr));
        const size_t rays = std::min<size_t>(n, ri_b.size / 8);
        for (size_t r = 0; r < rays; ++r) {
            std::memcpy(ri + 8 * r, &rs[r].depth, 4);
            std::memcpy(ri + 8 * r + 4, &rs[r].gauss_num_raw, 4);
        }
    }
    if (resolve(2, &img_b) && img_b.type == kDescStorageImage) {  // image_store (vulkan_ray_tracing.cc:2203-2247)
        const void* image = rd<const void*>(img_b.desc, kDescImage);
        if (!image) return fail(GSRT_E_ARG, "binding 2 has no image");
        const uint32_t fmt = rd<uint32_t>(image, kImageFormat);
        const uint32_t iw = rd<uint32_t>(image, kImageExtent), ih = rd<uint32_t>(image, kImageExtent + 4);
        if (fmt != kFormatRGBA32F && fmt != kFormatBGRA8) return fail(GSRT_E_ARG, "unsupported image format");
        if (iw != w || ih != h) return fail(GSRT_E_ARG, "image extent differs from the launch");
        (void)rd<uint32_t>(image, kImageTiling);  // tiling only addresses the timing model's transactions
        if (g.ppm_name.empty()) {
            char name[64];
            if (gsrt_reference_ppm_name(name, sizeof name) != GSRT_OK) return fail(GSRT_E_IO, "ppm name");
            g.ppm_name = name;
        }
        if (int s = gsrt_dump_ppm(g.ppm_name.c_str(), rgba.data(), w, h)) return fail(s, "ppm write");
    }
    return GSRT_OK;
}

}  // namespace

extern "C" {

void gpgpusim_setPipelineInfo(const void* pCreateInfos) {
    const VkRtPipelineInfo* info = static_cast<const VkRtPipelineInfo*>(pCreateInfos);
    g.groups.assign(info->pGroups, info->pGroups + info->groupCount);
    g.stage_flags.clear();
    for (uint32_t i = 0; i < info->stageCount; ++i) g.stage_flags.push_back(info->pStages[i].stage);
}

void gpgpusim_setGeometries(const void* pGeometries, uint32_t geometryCount) {
    const VkGeometry* geo = static_cast<const VkGeometry*>(pGeometries);
    std::vector<Geometry> gs(geometryCount);
    bool top = false;
    for (uint32_t i = 0; i < geometryCount; ++i) {
        Geometry& o = gs[i];
        o.type = geo[i].geometryType;
        if (o.type == kGeomInstances) {
            top = true;
            o.instances = geo[i].geometry.instances.data;
            o.array_of_pointers = geo[i].geometry.instances.arrayOfPointers != 0;
        } else if (o.type == kGeomTriangles) {
            const VkTrianglesData& t = geo[i].geometry.triangles;
            o.vertex_data = t.vertexData; o.vertex_stride = t.vertexStride; o.max_vertex = t.maxVertex;
            o.vertex_format = t.vertexFormat; o.index_data = t.indexData; o.index_type = t.indexType;
        } else if (o.type == kGeomAabbs) {
            // data is the base of the app's GaussAABBs buffer; the build range's primitiveOffset (not passed on,
            // lvp_acceleration_structure.c:1195) is 24 B per preceding model (Application.cpp:264-312: one BLAS per
            // model in model order, aabbOffset += sizeof(VkAabbPositionsKHR) for every model)
            const size_t k = g.blas_builds;
            std::memcpy(&o.aabb, static_cast<const char*>(geo[i].geometry.aabbs.data) + k * geo[i].geometry.aabbs.stride,
                        sizeof o.aabb);
        }
    }
    if (top) {
        g.tlas_geoms = gs;
    } else {  // bottom-level builds run in creation order (Application.cpp:315-322), so build k is allocBLAS k
        if (g.blas_builds < g.blas.size()) {
            g.blas[g.blas_builds].geoms = gs;
            g.blas[g.blas_builds].built = true;
        }
        ++g.blas_builds;
    }
    ++g.gen;
}

void gpgpusim_addTreelets(const void* accelerationStructure) { g.tlas_built = accelerationStructure; ++g.gen; }

void gpgpusim_testTraversal(void* root) { (void)root; }  // empty in vulkan-sim as well

uint32_t gpgpusim_registerShader(char* shaderPath, uint32_t shader_type) {
    // vulkan-sim takes the id from the file name's last "_<n>" before the extension (vulkan_ray_tracing.cc:
    // 1346-1356); lavapipe names stage i's PTX with i and asserts the returned id == i (lvp_pipeline_rt.c:162-163)
    std::string name(shaderPath ? shaderPath : "");
    name = name.substr(name.find_last_of('/') + 1);
    const size_t start = name.find_first_not_of('.');
    std::string stem = start == std::string::npos ? std::string() : name.substr(start, name.find('.', start) - start);
    const uint32_t id = static_cast<uint32_t>(std::strtoul(stem.substr(stem.find_last_of('_') + 1).c_str(), nullptr, 10));
    g.shaders.emplace_back(id, shader_type);
    return id;
}

void gpgpusim_allocBLAS(void* rootAddr, uint64_t bufferSize, void* gpgpusimAddr) {
    (void)gpgpusimAddr;
    g.blas.push_back(Blas{rootAddr, bufferSize, {}, false});
}

void gpgpusim_allocTLAS(void* rootAddr, uint64_t bufferSize, void* gpgpusimAddr) {
    (void)gpgpusimAddr;
    g.tlas_root = rootAddr;
    g.tlas_size = bufferSize;
}

// vulkan-sim binds a simulator allocation to the driver's host buffer and returns the simulator address
// (vulkan_ray_tracing.cc:2987-2999); the renderer reads the driver's memory directly at trace time, so the alias
// is the host address itself
void* gpgpusim_allocBuffer(void* bufferAddr, uint64_t bufferSize) {
    g.buffers.push_back(Range{static_cast<const char*>(bufferAddr), bufferSize});
    return bufferAddr;
}

void gpgpusim_vkCmdTraceRaysKHR(void* raygen_sbt, void* miss_sbt, void* hit_sbt, void* callable_sbt, bool is_indirect,
                                uint32_t launch_width, uint32_t launch_height, uint32_t launch_depth,
                                uint64_t launch_size_addr) {
    (void)raygen_sbt; (void)miss_sbt; (void)hit_sbt; (void)callable_sbt; (void)is_indirect; (void)launch_size_addr;
    g.status = GSRT_OK;
    g.error.clear();
    trace(launch_width, launch_height, launch_depth);
}

void gpgpusim_setDescriptor(uint32_t setID, uint32_t descID, void* address, uint32_t size, uint32_t type) {
    if (setID == 0 && descID < 32) g.legacy[descID] = Binding{address, size, type, nullptr};
}

void gpgpusim_setDescriptorSet(const void* set) {
    if (!g.set) g.set = set;  // vulkan-sim keeps the first set and ignores later updates (vulkan_ray_tracing.cc:1266-1273)
}

void gpgpusim_pass_child_addr(void* address) { g.child_addrs.push_back(address); }

// ---- test hooks ---------------------------------------------------------------------------------------------
int vksim_shim_status(void) { return g.status; }
const char* vksim_shim_error(void) { return g.error.c_str(); }
// [gaussians, triangles, registered shaders, buffers, BLAS, child addresses, mesh vertices] of the assembled scene
void vksim_shim_counts(uint32_t out[7]) {
    out[0] = static_cast<uint32_t>(g.params.size()); out[1] = static_cast<uint32_t>(g.idx.size() / 3); out[2] = static_cast<uint32_t>(g.shaders.size());
    out[3] = static_cast<uint32_t>(g.buffers.size()); out[4] = static_cast<uint32_t>(g.blas.size());
    out[5] = static_cast<uint32_t>(g.child_addrs.size()); out[6] = static_cast<uint32_t>(g.verts.size() / 3);
}
// copies of the assembled scene (sizes from vksim_shim_counts; any pointer may be NULL)
void vksim_shim_assembly(gsrt_gauss_param* params, gsrt_aabb* aabbs, float* verts, uint32_t* idx) {
    if (params) std::memcpy(params, g.params.data(), g.params.size() * sizeof(gsrt_gauss_param));
    if (aabbs) std::memcpy(aabbs, g.aabbs.data(), g.aabbs.size() * sizeof(gsrt_aabb));
    if (verts) std::memcpy(verts, g.verts.data(), g.verts.size() * sizeof(float));
    if (idx) std::memcpy(idx, g.idx.data(), g.idx.size() * sizeof(uint32_t));
}
const char* vksim_shim_ppm_name(void) { return g.ppm_name.c_str(); }
// the mirror's offsets, keyed as oracle/ref/lvp_layout_probe.c prints them
const char* vksim_shim_layout_json(void) {
    static std::string s;
    char buf[2048];
    std::snprintf(buf, sizeof buf,
                  "{\"sizeof struct lvp_descriptor\": %zu, \"struct lvp_descriptor.info\": %zu, "
                  "\"struct lvp_descriptor.info.ssbo.pmem\": %zu, \"struct lvp_descriptor.info.ubo.pmem\": %zu, "
                  "\"struct lvp_descriptor.info.ubo.buffer_offset\": %zu, "
                  "\"struct lvp_descriptor.info.ssbo.buffer_size\": %zu, "
                  "\"struct lvp_descriptor.info.image_view.image\": %zu, "
                  "\"struct lvp_descriptor_set.layout\": %zu, \"struct lvp_descriptor_set.descriptors\": %zu, "
                  "\"struct lvp_descriptor_set_layout.binding_count\": %zu, "
                  "\"struct lvp_descriptor_set_layout.binding\": %zu, "
                  "\"sizeof struct lvp_descriptor_set_binding_layout\": %zu, "
                  "\"struct lvp_descriptor_set_binding_layout.descriptor_index\": %zu, "
                  "\"struct lvp_descriptor_set_binding_layout.type\": %zu, "
                  "\"struct lvp_image.vk.format\": %zu, \"struct lvp_image.vk.extent\": %zu, "
                  "\"struct lvp_image.vk.tiling\": %zu, "
                  "\"sizeof VkAccelerationStructureGeometryKHR\": %zu, "
                  "\"VkAccelerationStructureGeometryKHR.geometry\": %zu, "
                  "\"VkAccelerationStructureGeometryTrianglesDataKHR.vertexData\": %zu, "
                  "\"VkAccelerationStructureGeometryTrianglesDataKHR.maxVertex\": %zu, "
                  "\"VkAccelerationStructureGeometryTrianglesDataKHR.indexData\": %zu, "
                  "\"VkAccelerationStructureGeometryAabbsDataKHR.data\": %zu, "
                  "\"VkAccelerationStructureGeometryInstancesDataKHR.data\": %zu, "
                  "\"sizeof VkAccelerationStructureInstanceKHR\": %zu, "
                  "\"VkAccelerationStructureInstanceKHR.accelerationStructureReference\": %zu, "
                  "\"sizeof VkRayTracingPipelineCreateInfoKHR\": %zu, "
                  "\"VkRayTracingPipelineCreateInfoKHR.pGroups\": %zu, "
                  "\"sizeof VkRayTracingShaderGroupCreateInfoKHR\": %zu, "
                  "\"VkRayTracingShaderGroupCreateInfoKHR.intersectionShader\": %zu, "
                  "\"VK_DESCRIPTOR_TYPE_ACCELERATION_STRUCTURE_KHR\": %u, "
                  "\"VK_RAY_TRACING_SHADER_GROUP_TYPE_PROCEDURAL_HIT_GROUP_KHR\": %u, "
                  "\"VK_FORMAT_R32G32B32A32_SFLOAT\": %u}",
                  sizeof(LvpDescriptor), offsetof(LvpDescriptor, info), kDescPmem, kDescPmem, kDescBufOffset,
                  kDescBufSize, kDescImage, kSetLayout, kSetDescriptors, kLayoutBindingCount, kLayoutBindings,
                  kBindingSize, kBindingDescIndex, kBindingType, kImageFormat, kImageExtent, kImageTiling,
                  sizeof(VkGeometry), offsetof(VkGeometry, geometry), offsetof(VkTrianglesData, vertexData),
                  offsetof(VkTrianglesData, maxVertex), offsetof(VkTrianglesData, indexData),
                  offsetof(VkAabbsData, data), offsetof(VkInstancesData, data), sizeof(VkInstance),
                  offsetof(VkInstance, as_reference), sizeof(VkRtPipelineInfo), offsetof(VkRtPipelineInfo, pGroups),
                  sizeof(VkGroup), offsetof(VkGroup, intersectionShader), kDescAccelStruct, kGroupProcedural,
                  kFormatRGBA32F);
    s = buf;
    return s.c_str();
}
void vksim_shim_reset(void) {
    if (g.scene) gsrt_destroy_scene(g.scene);
    if (g.ctx) gsrt_destroy(g.ctx);
    g = Shim{};
}

}  // extern "C"
