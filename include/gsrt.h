/*
 * gsrt.h -- C ABI of the MI355X-native ray-traced 3D Gaussian Splatting renderer.
 *
 * This header is the drop-in surface a reference-side caller links against. The library's test and measurement hooks
 * (host mirrors of the sharded layout, emulated gathers, diagnostic counters, synthetic clouds, the test switches)
 * are declared separately in gsrt_test.h.
 *
 * Drop-in boundary for the reference's Gaussian render path. The
 * reference path is reached through three nested boundaries; each entry point below
 * names the reference interface it replaces (paths relative to the reference root):
 *
 *   scene upload   Assets::Scene ctor packing GaussParam/AABB/NextK/RayInfo/ExpLUT
 *                  (RayTracingInVulkan/src/Assets/Scene.cpp:16-182)
 *   AS build       vkCmdBuildAccelerationStructuresKHR -> lvp_cpu_build_acceleration_structures
 *                  (mesa-vulkan-sim/src/gallium/frontends/lavapipe/lvp_acceleration_structure.c:1182-1400)
 *   dispatch       vkCmdTraceRaysKHR(W,H,1) -> gpgpusim_vkCmdTraceRaysKHR
 *                  (vulkan-sim/src/cuda-sim/gpgpusim_calls_from_mesa.cc:60-74)
 *   frame dump     VulkanRayTracing::image_store P3 PPM (vulkan-sim/src/cuda-sim/vulkan_ray_tracing.cc:2203-2247)
 *
 * Conventions: every call returns a gsrt_status (no exceptions cross the ABI); input
 * arrays are copied (the caller keeps ownership); scene objects are owned by the library;
 * one gsrt_ctx per device; calls on one ctx are serialised by the caller.
 */
#ifndef GSRT_H
#define GSRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSRT_ABI_VERSION 2
/* largest scene: Gaussian ids are 31-bit (BVH child refs use bit 31 as the leaf flag) */
#define GSRT_MAX_GAUSSIANS 0x7fffffffu

typedef struct gsrt_ctx gsrt_ctx;
typedef struct gsrt_scene gsrt_scene;

typedef enum {
    GSRT_OK = 0,
    GSRT_E_ARG = -1,     /* bad argument (null pointer, size mismatch, unsupported mode) */
    GSRT_E_OOM = -2,     /* device or host allocation failed */
    GSRT_E_DEVICE = -3,  /* HIP runtime / kernel failure, or no device */
    GSRT_E_IO = -4,      /* file open/read/write failed */
    GSRT_E_STATE = -5,   /* call out of order (e.g. render before gsrt_build_bvh) */
    GSRT_E_COMM = -6     /* RCCL failure */
} gsrt_status;

/* == GaussParam (RayTracingInVulkan/assets/shaders/Gauss.glsl:1-6; Assets/Sphere.hpp:10-19), 48 B */
typedef struct { float center_opacity[4]; float cov3d[6]; float pad[2]; } gsrt_gauss_param;
/* == VkAabbPositionsKHR as packed by Scene.cpp:129-130, 24 B */
typedef struct { float min_x, min_y, min_z, max_x, max_y, max_z; } gsrt_aabb;
/* == UniformBufferObject (Assets/UniformBuffer.hpp:15-36; shaders/UniformBufferObject.glsl), 320 B,
 *    matrices column-major (glm layout) */
typedef struct {
    float model_view[16], projection[16], model_view_inverse[16], projection_inverse[16];
    float light_position[3], light_radius, aperture, focus_distance, heatmap_scale;
    uint32_t total_samples, samples, bounces, shadows, random_seed, width, height, has_sky, show_heatmap;
} gsrt_ubo;
/* Per-ray state after the frame: RayInfo {Depth, GaussNum} (RayPayload.glsl:11-16), Ray.Trans,
 * NextK[ray][8] {depth, alpha} (Gauss.glsl:8-12). gauss_num is clamped to 8; gauss_num_raw is the
 * unclamped insert count of the last round (the reference indexes NextK with it, rchit:23-31). 80 B */
typedef struct { float trans; float depth; int32_t gauss_num; int32_t gauss_num_raw; float k[8][2]; } gsrt_raystate;

/* render modes */
enum {
    GSRT_MODE_REF = 0,      /* bit-faithful restatement of GaussTracing.rgen/.rint/.rchit (K=8 rounds) */
    GSRT_MODE_COR = 1,      /* front-facing depth, conic = (V+0.3I)^-1, exp, alpha<=0.99, SH-3 colour,
                               depth-ordered blend, early stop at T<1e-4, jittered spp */
    GSRT_FLAG_LUT = 0x100,  /* COR: use the reference LinearExp LUT (ExpLUT.hpp) instead of exp */
    GSRT_FLAG_STATS = 0x200, /* also count candidates / blended hits (gsrt_last_stats) */
    GSRT_FLAG_OUT_DUMP8 = 0x400 /* sharded COR frames: exchange and keep the frame as the integers its PPM dump prints
                                   (gsrt_dump8_*), 4 bytes per pixel instead of RGBA32F's 16 */
};
/* synthetic cloud kinds */
enum { GSRT_SYNTH_COR = 0, GSRT_SYNTH_REF = 1, GSRT_SYNTH_NEEDLE = 2 };

const char* gsrt_status_string(gsrt_status s);
int gsrt_abi_version(void);

/* ---- context ------------------------------------------------------------------------------ */
/* device_ordinal >= 0: HIP device. Fails with GSRT_E_DEVICE when the device is absent. */
gsrt_status gsrt_create(gsrt_ctx** out, int device_ordinal);
void gsrt_destroy(gsrt_ctx* ctx);
const char* gsrt_last_error(const gsrt_ctx* ctx);
gsrt_status gsrt_synchronize(gsrt_ctx* ctx);
/* the HIP stream the render kernels of this ctx are enqueued on (hipStream_t), for callers timing with
 * events; gsrt_synchronize() also reports (and clears) a traversal failure of any frame since the last
 * check (GSRT_E_DEVICE) */
void* gsrt_stream(gsrt_ctx* ctx);
/* the HIP stream of the per-frame prep kernels and of scene updates / refits (hipStream_t). It can change
 * between frames: a COR frame may move the prep work to a stream of another priority class (ordered after
 * everything queued on the previous one), so query it right before each use */
void* gsrt_prep_stream(gsrt_ctx* ctx);
/* the HIP stream (hipStream_t) of gsrt_scene_update's and gsrt_refit_bvh's copies (created at the first call): a producer
 * on the GPU fills an update's device source on this stream before the call. The copies go into the array's second
 * buffer and overlap the frames already queued ("Scene updates") */
void* gsrt_update_stream(gsrt_ctx* ctx);
/* 1 when the last frame ran on slot streams: its prep and render kernels on its frame slot's stream, overlapping
 * the previous frame (chosen per frame from sampled render kernel times), else 0 */
int gsrt_slot_streams(const gsrt_ctx* ctx);

/* ---- scene (replaces Assets::Scene, Scene.cpp:16-182) -------------------------------------- */
/* params/aabbs as the reference packs them (one entry per Gaussian model); sh nullable, n*48 floats
 * laid out [gauss][coef 0..15][rgb]. Host pointers; copied to HBM. */
gsrt_status gsrt_scene_from_params(gsrt_ctx* ctx, const gsrt_gauss_param* params, const gsrt_aabb* aabbs,
                                   uint32_t n, const float* sh, gsrt_scene** out);
/* Model::CreateGauss + Gauss::init_cov3d/init_radius (Model.cpp:550-564, Sphere.hpp:108-165), computed
 * on the device. rot_rxyz is the reference's vec4(r, x, y, z). */
gsrt_status gsrt_scene_from_model(gsrt_ctx* ctx, const float* center, const float* rot_rxyz, const float* scale,
                                  const float* opacity, const float* sh, uint32_t n, gsrt_scene** out);
/* download the device-side GaussParam / AABB arrays (either may be NULL) */
gsrt_status gsrt_scene_download(gsrt_scene* scene, gsrt_gauss_param* params, gsrt_aabb* aabbs);
uint32_t gsrt_scene_size(const gsrt_scene* scene);
void gsrt_destroy_scene(gsrt_scene* scene);

/* 3DGS .ply ingestion (the reference only has hard-coded CreateGauss calls,
 * SceneList.cpp:123-125). Vertex properties x y z, scale_0..2 (log), rot_0..3 (w x y z, unnormalised),
 * opacity (logit), f_dc_0..2 and f_rest_* (channel-major); ascii or binary, any scalar type.
 * gsrt_ply_info: vertex count and SH degree (0 when only f_dc or none). gsrt_ply_read: arrays in the
 * gsrt_scene_from_model convention (scale = exp, opacity = sigmoid, rot normalised (r,x,y,z), sh
 * [gauss][coef 0..15][rgb], nullable, degree cut or zero-padded to 3). */
gsrt_status gsrt_ply_info(const char* path, uint32_t* n, uint32_t* sh_degree);
gsrt_status gsrt_ply_read(const char* path, float* center, float* rot_rxyz, float* scale, float* opacity, float* sh);
gsrt_status gsrt_scene_from_ply(gsrt_ctx* ctx, const char* path, int with_sh, gsrt_scene** out);

/* ---- triangle meshes co-traced with the Gaussians ---------------------- */
/* Scene 33 holds a triangle-mesh sphere beside its two Gaussians (SceneList.cpp:123, Model::CreateSphere,
 * isProcedural = false). A triangle hit takes part in the REF frame the way vulkan-sim orders it:
 *   - the closest triangle hit t_tri (Moller-Trumbore in the object space of the identity instance,
 *     vulkan_ray_tracing.cc:1184-1206, accepted when Tmin <= t/|d| <= Tmax, :925-931) becomes the
 *     traversal's min_thit;
 *   - Gaussian AABBs entered at or beyond it are culled (:806-807; gsrt restates the order-independent
 *     case: the mesh instance is traversed first);
 *   - a Gaussian report is accepted only when its depth < t_tri (instructions.cc:7050);
 *   - a round whose closest hit is the triangle runs RayTracing.rchit, whose Scatter() sets the payload's
 *     Trans to 0 (Scatter.glsl:14-70).
 * COR frames do not trace meshes (gsrt_render returns GSRT_E_ARG for a COR frame of a scene with a mesh). */
/* append an indexed triangle mesh (world coordinates, identity instance transform, Application.cpp:361-362);
 * vertices: nv*3 floats, indices: nt*3 u32 (< nv). Copied; the mesh BVH is rebuilt on the host and uploaded. */
gsrt_status gsrt_scene_add_mesh(gsrt_scene* scene, const float* vertices, uint32_t nv, const uint32_t* indices,
                                uint32_t nt);
uint32_t gsrt_scene_mesh_triangles(const gsrt_scene* scene);
/* Model::CreateSphere(center, radius) geometry (Model.cpp:566-629): 32 slices x 16 stacks,
 * GSRT_SPHERE_VERTICES positions (3 floats each) and GSRT_SPHERE_TRIANGLES triangles (3 u32 each) */
#define GSRT_SPHERE_VERTICES 561u
#define GSRT_SPHERE_TRIANGLES 1024u
gsrt_status gsrt_sphere_mesh(const float center[3], float radius, float* vertices, uint32_t* indices);

/* ---- camera (replaces RayTracer::GetUniformBufferObject, RayTracer.cpp:38-65) --------------- */
/* mv: initial camera modelview (CameraInitialSate::ModelView), run through ModelViewController. */
gsrt_status gsrt_camera_from_modelview(const float mv[16], float fovy_deg, uint32_t width, uint32_t height,
                                       float focus_distance, uint32_t samples, uint32_t bounces, gsrt_ubo* out);
/* .camera file: 6 floats eye, centre -> lookAt(eye, centre, (0,1,0)) (SceneList.cpp:705-712) */
gsrt_status gsrt_camera_from_file(const char* path, float fovy_deg, uint32_t width, uint32_t height,
                                  float focus_distance, uint32_t samples, uint32_t bounces, gsrt_ubo* out);
gsrt_status gsrt_lookat(const float eye[3], const float center[3], const float up[3], float out_mv[16]);

/* ---- acceleration structure (replaces the Embree TLAS build, lvp_acceleration_structure.c:1329-1351) */
/* LBVH on the device: Morton codes, LSD radix sort, Karras hierarchy, bottom-up AABB fit. */
gsrt_status gsrt_build_bvh(gsrt_scene* scene);
/* new AABBs (host or device pointer, n entries; NULL = the scene's current AABBs) with the topology
 * kept: a bottom-up refit without a host round trip (one-wave workgroups fit 256-leaf chunks in LDS, then spans
 * of 16K and 1M leaves and the top climb by arrival counts). The copy is enqueued on gsrt_update_stream() into the
 * array's second buffer, ordered after the frames that read that buffer; frames queued after the call read the new
 * AABBs. The fit itself runs lazily with the next frame that uses a frame slot (a REF or counting frame, or a BVH
 * download, also refits a slot whose leaf boxes a COR frame replaced by footprint boxes; a rank of a sharded frame
 * fits only the part of the tree its band can see). A device source must hold its data when the call is made
 * (filled synchronously, or on gsrt_update_stream()) and stay unchanged until gsrt_synchronize(). The
 * reference only builds (MODE_BUILD, TopLevelAccelerationStructure.cpp:34); refit serves dynamic
 * scenes. */
gsrt_status gsrt_refit_bvh(gsrt_scene* scene, const gsrt_aabb* aabbs);
/* replace the scene's GaussParam and/or AABB arrays (host or device pointers, n entries each, either may be NULL),
 * with the same stream, ordering and source rules as gsrt_refit_bvh (a producer on the GPU fills the source on
 * gsrt_update_stream()); follow with gsrt_refit_bvh(scene, NULL) when AABBs moved. The animation step of a dynamic scene
 * (config 5: per-frame centre jitter). */
gsrt_status gsrt_scene_update(gsrt_scene* scene, const gsrt_gauss_param* params, const gsrt_aabb* aabbs);
/* the zero-copy form of gsrt_scene_update for a producer that writes each frame's Gaussians into device arrays of its
 * own: frames queued from now on read params / aabbs (device pointers on the context's device, 16-byte aligned,
 * n entries; either may be NULL = unchanged) in place. The arrays must hold their data at the call (filled
 * synchronously or on gsrt_update_stream()) and stay unchanged and allocated until gsrt_scene_detach() or
 * gsrt_destroy_scene() returns; attaching again swaps in other arrays under the same rule. Follow with
 * gsrt_refit_bvh(scene, NULL) when AABBs moved. A gsrt_scene_update / gsrt_refit_bvh source for an attached array, or
 * gsrt_scene_stream_pages, copies into the scene's own buffers and ends that borrow (the caller's array is then read
 * until gsrt_synchronize()). */
gsrt_status gsrt_scene_attach(gsrt_scene* scene, const gsrt_gauss_param* params, const gsrt_aabb* aabbs);
/* end a borrow: copy the attached arrays into the scene's own buffers and wait for every queued frame, so nothing
 * reads the caller's arrays after it returns */
gsrt_status gsrt_scene_detach(gsrt_scene* scene);
/* Gaussian pages: a dynamic scene whose Gaussians change on the host streams
 * them into HBM page by page. Page p holds Gaussians [p * GSRT_PAGE_GAUSSIANS, min((p + 1) * GSRT_PAGE_GAUSSIANS, n)).
 * gsrt_scene_stream_pages copies the listed pages of the full-scene host arrays params / aabbs (either may be NULL)
 * into the scene, consecutive page ids as one transfer, on gsrt_prep_stream() with gsrt_scene_update's ordering
 * (after every queued frame that reads the arrays, before the next frame's prep); follow with
 * gsrt_refit_bvh(scene, NULL) when AABBs moved. The copies run on the DMA engines beside the render kernels and
 * return at once when the host arrays are page-locked (gsrt_host_register); the arrays must stay unchanged until
 * gsrt_synchronize(). pages: ascending or not, duplicates allowed, each < the page count. */
#define GSRT_PAGE_GAUSSIANS 4096u
gsrt_status gsrt_scene_stream_pages(gsrt_scene* scene, const gsrt_gauss_param* params, const gsrt_aabb* aabbs,
                                    const uint32_t* pages, uint32_t npages);
uint32_t gsrt_scene_pages(const gsrt_scene* scene);
/* page-lock (and unlock) caller memory for asynchronous streaming (hipHostRegister) */
gsrt_status gsrt_host_register(gsrt_ctx* ctx, void* ptr, size_t bytes);
gsrt_status gsrt_host_unregister(gsrt_ctx* ctx, void* ptr);
/* BVH introspection for tests: internal-node count, root box (6 floats), max depth */
gsrt_status gsrt_bvh_info(gsrt_scene* scene, uint32_t* n_internal, float root_box[6], uint32_t* max_depth);
/* raw node download for tests: nodes = (n-1)*16 u32/f32 words; leaf_gid = n u32 (sorted order) */
gsrt_status gsrt_bvh_download(gsrt_scene* scene, uint32_t* nodes, uint32_t* leaf_gid, uint32_t* morton_sorted);

/* ---- render (replaces vkCmdTraceRaysKHR(W,H,1) over GaussTracing.rgen, Application.cpp:223-225) */
/* mode: GSRT_MODE_* | flags. k: 0 = mode default (REF: 8, the reference's NextK width; COR: the
 * tile-shared nearest-hit buffer capacity). rgba_out: W*H*4 floats (RGBA32F, row-major), host or
 * device pointer, may be NULL (image stays in the ctx framebuffer). raystate_out: W*H entries, host
 * or device pointer, nullable. Blocks until the frame is done when any output is a host pointer.
 * The traversal error word is sticky across pipelined frames: a synchronous render (gsrt_render,
 * gsrt_render_sharded) that drains the ctx reports and clears a failure of
 * any earlier gsrt_render_async frame as well (GSRT_E_DEVICE), exactly as gsrt_synchronize does. */
gsrt_status gsrt_render(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out,
                        gsrt_raystate* raystate_out);
/* enqueue one frame on gsrt_stream(); outputs (device pointers only) may be NULL */
gsrt_status gsrt_render_async(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* d_rgba,
                              gsrt_raystate* d_raystate);
/* device pointer of the ctx framebuffer of the last render (W*H*4 floats). Frames on slot streams
 * (gsrt_slot_streams) alternate between two buffers, so query it after each render rather than keeping it. NULL after
 * a GSRT_FLAG_OUT_DUMP8 sharded frame (its image is read with gsrt_dump8_read), until the next RGBA32F frame */
const float* gsrt_framebuffer(gsrt_ctx* ctx);
/* counters of the last render with GSRT_FLAG_STATS: [0] rays, [1] sum candidates |C_r|, [2] sum blended
 * |H_r|, [3] terminated rays, [4] tile collection rounds, [5] narrow-traversal restarts, [6] tiles,
 * [7] max candidates in one tile. Per-ray uint4 {candidates, blended, rounds, terminated} into
 * per_ray (host, W*H*4) when non-NULL. */
gsrt_status gsrt_last_stats(gsrt_ctx* ctx, uint64_t out[8], uint32_t* per_ray);
/* vulkan-sim's ray-tracing statistics (gpu-sim.cc:1510-1518) for the last REF render with GSRT_FLAG_STATS:
 * out = {rt_n_total_rays (traversals: rounds summed over the rays), rt_num_hits (traversals with a triangle hit),
 * rt_max_tree_depth, rt_max_nodes_per_ray, rt_tot_nodes_per_ray, walks that overflowed (0), 0, 0}. Nodes are
 * counted on gsrt's binary LBVH (internal nodes visited + leaves reached per traversal), so they compare in kind,
 * not in value, with the simulator's 6-wide Embree BVH. Per ray: gsrt_last_stats per_ray .y = triangle-hit
 * traversals, .w = nodes of one traversal. gsrt_dump_vs_stats writes the simulator's "rt_... = v" lines. */
gsrt_status gsrt_vs_stats(gsrt_ctx* ctx, uint64_t out[8]);
gsrt_status gsrt_dump_vs_stats(gsrt_ctx* ctx, const char* path);
/* the ExpLUT of REF mode (generateExpLUT(256, 0, 8), ExpLUT.hpp:10-24 / Scene.cpp:47): 256 x {k, b}.
 * as the host computes it (no device needed); gsrt_create uploads it for the kernels */
gsrt_status gsrt_exp_lut(float out[512]);

/* HIP-event timing of the next `frames` renders on gsrt_stream() (0 disables): per frame the render
 * kernel alone (REF: k_render_ref; COR: k_render_cor, after the first-round list kernel k_collect_cor)
 * and the whole frame (projection + list + render [+ gather/unpack]). gsrt_timing_read waits for
 * the stream and returns the recorded frames (at most `cap`). */
gsrt_status gsrt_timing(gsrt_ctx* ctx, uint32_t frames);
gsrt_status gsrt_timing_read(gsrt_ctx* ctx, float* kernel_ms, float* frame_ms, uint32_t cap, uint32_t* nframes);
/* per recorded frame, the exchange of a gsrt_render_sharded_async frame on gsrt_comm_stream(): from the moment the
 * rank's share is rendered to the end of the gather (+ rank 0's unpack), in ms; 0 for frames without an exchange.
 * Waits for the render and comm streams. */
gsrt_status gsrt_timing_read_exchange(gsrt_ctx* ctx, float* exchange_ms, uint32_t cap, uint32_t* nframes);
/* on != 0: the timed frames record only the render kernel's two events (frame_ms then reads 0), so that the timing
 * adds as little as possible to the frames it measures; 0 (default): all of them. Takes effect at gsrt_timing. */
gsrt_status gsrt_timing_kernel_only(gsrt_ctx* ctx, int on);
/* stride >= 1: of the frames after gsrt_timing, record the events of frames 0, stride, 2 stride, ... only (the
 * `frames` of gsrt_timing count recorded frames); 1 (default): every frame. Takes effect at gsrt_timing. */
gsrt_status gsrt_timing_stride(gsrt_ctx* ctx, uint32_t stride);

/* ---- multi-GPU tile sharding ------------------------------------------------ */
/* RCCL unique id (128 bytes) created on rank 0 and shipped to the other ranks by the caller */
gsrt_status gsrt_comm_unique_id(uint8_t out[128]);
gsrt_status gsrt_comm_init(gsrt_ctx* ctx, const uint8_t id[128], int nranks, int rank);
/* ranks of the ctx's communicator and this rank in it, from RCCL itself (ncclCommCount / ncclCommUserRank);
 * 1 / 0 without gsrt_comm_init. rank may be NULL. */
gsrt_status gsrt_comm_size(gsrt_ctx* ctx, int* nranks, int* rank);
/* the HIP stream (hipStream_t) on which a sharded frame's gather and rank 0's unpack into the framebuffer run,
 * or NULL when frames render straight into the framebuffer (one rank, or no gsrt_comm_init): work that reads a
 * gsrt_render_sharded_async frame's image goes on this stream (or after gsrt_synchronize) */
void* gsrt_comm_stream(gsrt_ctx* ctx);
/* render this rank's band of the frame (below), then ncclGather the tiles to rank 0, which unpacks them into its
 * framebuffer (and rgba_out, host or device, when non-NULL on rank 0). Every rank calls it for every frame.
 * With GSRT_FLAG_OUT_DUMP8 (COR) the tiles travel as dump codes instead (below): rank 0 reads the frame with
 * gsrt_dump8_read, and rgba_out must be NULL. */
gsrt_status gsrt_render_sharded(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, uint32_t k,
                                float* rgba_out);
gsrt_status gsrt_render_sharded_async(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, uint32_t k);
/* The partition of a sharded frame: one band of whole tile rows per rank, rank r owning rows
 * [bands[r], bands[r + 1]) of every column (bands[0] = 0, bands[nranks] = tiles_y, non-decreasing). A rank's tiles are
 * numbered in the spatial order (super-tiles of 16x16 tiles, row-major) of its band's own grid; that is the order of
 * its block in the gather. On a communicator of N > 1 ranks the bands follow the shading cost: every 8th COR frame
 * the render kernel records each tile row's cost, one ncclAllReduce gives every rank the whole profile, and 8 frames
 * later every rank cuts the same new bands from it (gsrt_tile_bands' rule), kept only when they lower the heaviest
 * band's cost by 2 %. Profile frames follow a fixed schedule (every 8th sharded COR frame, pinned bands or not), and
 * the profile carries a hash of each rank's partition and pinning; ranks that disagree get GSRT_E_COMM.
 * A communicator holds at most 64 ranks (gsrt_comm_init returns GSRT_E_ARG beyond). */
/* tile decomposition of a frame under the even partition (no cost profile): out = {tile_w, tile_h, tiles_x, tiles_y,
 * tiles of `rank` among `nranks`, in-wave samples per pixel, first tile row of `rank`'s band, packed stride (the
 * largest band's tile count: the per-rank block size in the gathered buffer)}. Host-only. */
gsrt_status gsrt_tile_plan(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, uint32_t out[8]);
/* the bands (nranks + 1 boundaries) the balancing rule cuts from a per-tile-row cost profile (tiles_y entries; NULL:
 * every row costs the same): each rank's summed row cost over its weight as even as whole rows allow, rank 0 (the
 * gather's root, which also receives and unpacks the frame) weighted 1 - 0.09 (nranks - 1) / spp (>= 1/4) in COR
 * mode (0.07 for GSRT_FLAG_OUT_DUMP8's 4-byte pixels); every band gets a row when tiles_y >= nranks. Host-only and deterministic. */
gsrt_status gsrt_tile_bands(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* row_cost, uint32_t* bands);
/* pin the partition of this ctx's sharded frames to `bands` (nranks + 1 entries; every rank of the job must pin the
 * same), or back to automatic balancing with NULL. Needs gsrt_comm_init. */
gsrt_status gsrt_set_bands(gsrt_ctx* ctx, int nranks, const uint32_t* bands);
/* the bands of the last sharded frame on this ctx (n = nranks + 1 entries, at most cap written; n = 0 before any) */
gsrt_status gsrt_last_bands(gsrt_ctx* ctx, uint32_t* bands, uint32_t cap, uint32_t* n);
/* the per-tile-row shading cost of the last whole (unsharded) COR frame: per tile, the candidates it staged plus a
 * constant, summed over the row (the profile the balancing uses). Waits for the frame. */
gsrt_status gsrt_row_costs(gsrt_ctx* ctx, uint32_t* row_cost, uint32_t cap, uint32_t* rows);

/* ---- the compact exchange format (GSRT_FLAG_OUT_DUMP8) -----------------------------------------
 * A sharded COR frame rendered with GSRT_FLAG_OUT_DUMP8 travels and stays as what its PPM dump prints: per pixel one
 * code word, 10 bits per channel holding rint(channel * 255) (bits 0-9 r, 10-19 g, 20-29 b), when every channel's
 * product is a finite, non-negative (not -0) number that rounds to at most 1022. Any other pixel has bit 30 set and
 * its exact r, g, b in an escape entry. gsrt_dump8_ppm of a frame's codes and escapes is byte-identical to
 * gsrt_dump_ppm of the same frame in RGBA32F. Each rank's block holds up to max(256, pixels / 64) escapes; a frame
 * with more fails at gsrt_dump8_read (GSRT_E_STATE) and is rendered again without the flag. */
typedef struct { uint32_t pixel; float r, g, b; } gsrt_dump8_escape;  /* pixel = x + y * width */
#define GSRT_DUMP8_ESCAPE (1u << 30)
/* rank 0, after a GSRT_FLAG_OUT_DUMP8 sharded frame: its width x height code words (codes may be NULL) and its escapes
 * in pixel order (at most cap written; n_esc = how many the frame has). Waits for the frame. */
gsrt_status gsrt_dump8_read(gsrt_ctx* ctx, uint32_t* codes, gsrt_dump8_escape* esc, uint32_t cap, uint32_t* n_esc);
/* host: the code words of an RGBA32F frame (n pixels), and the escapes it needs (at most cap written, n_esc all) */
gsrt_status gsrt_dump8_encode(const float* rgba, size_t n, uint32_t* codes, gsrt_dump8_escape* esc, uint32_t cap,
                              uint32_t* n_esc);
/* host: the P3 PPM of a frame in codes + escapes (the bytes gsrt_dump_ppm writes for the frame) */
gsrt_status gsrt_dump8_ppm(const char* path, const uint32_t* codes, uint32_t width, uint32_t height,
                           const gsrt_dump8_escape* esc, uint32_t n_esc);

/* ---- frame dump (replaces VulkanRayTracing::image_store, vulkan_ray_tracing.cc:2203-2247) ---- */
/* P3 PPM, "%3.0f %3.0f %3.0f\n" of rgb*255 per pixel, host rgba pointer */
gsrt_status gsrt_dump_ppm(const char* path, const float* rgba, uint32_t width, uint32_t height);
/* "<dd-mm-YYYY-HH-MM-SS->SCENE.ppm" name the reference derives from local time */
gsrt_status gsrt_reference_ppm_name(char* out, size_t cap);
/* dump_image.sh text: "[x, y] rgba(r, g, b)" per pixel, the RayTracing.rgen:98 debugPrintf line
 * (RTV/dump_image.sh keeps the lines containing "rgba"), rows top to bottom */
gsrt_status gsrt_dump_rgba_text(const char* path, const float* rgba, uint32_t width, uint32_t height);
/* Intel-path image.binary records {float r, g, b; uint32 offset = x + y*W} (vulkan_ray_tracing.cc:2165-2179) */
gsrt_status gsrt_dump_image_binary(const char* path, const float* rgba, uint32_t width, uint32_t height);



#ifdef __cplusplus
}
#endif
#endif /* GSRT_H */
