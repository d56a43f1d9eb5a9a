// gsrt_internal.hpp -- host-side objects behind the C ABI and the kernel launchers they call.
#pragma once

#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/gsrt_test.h"
#include "gsrt_device.hpp"

struct gsrt_comm_state;

namespace gsrt {
// A band-restricted fit (a rank of a sharded frame): 256-leaf chunks none of whose splats the rank can see (inband, the
// slot's in-band bitmap: 1 bit per gaussian id, may_own_box under the frame's camera and band, k_classify) are not
// fitted, their subtrees get empty boxes
struct FitBand {
    const uint32_t* inband;
};
// what a band-restricted fit and an in-band bitmap depend on besides the AABBs: the camera, the frame size, the band
struct FitBandKey {
    float mv[16], proj[16];
    uint32_t width, height;
    RankTiles own;
};
inline FitBandKey make_band_key(const gsrt_ubo& u, const RankTiles& own) {
    FitBandKey k;
    std::memset(&k, 0, sizeof k);
    std::memcpy(k.mv, u.model_view, sizeof k.mv);
    std::memcpy(k.proj, u.projection, sizeof k.proj);
    k.width = u.width;
    k.height = u.height;
    k.own = own;
    return k;
}
inline bool same_key(const FitBandKey& a, const FitBandKey& b) { return std::memcmp(&a, &b, sizeof a) == 0; }
}  // namespace gsrt

// Per-frame buffers of the COR prep stage (k_project -> k_frontier -> k_group_list on ctx->pstream), kSlots
// slots: frames take the slots in rotation (ctx->nslots of them, choose_slots), so frame f's prep overlaps the render
// kernels of the frames before it (ctx->stream). A slot is rewritten only after its `rendered` event (the render of
// the frame that last used it) fired: with two slots frame f's prep waits for the render of frame f - 2, with three
// for f - 3. Slot streams (the frame's prep and render on its slot's stream) use two slots, one per prep stream.
constexpr uint32_t kSlots = 3;
constexpr uint32_t kStreamSlots = 2;  // prep streams per priority class: {pstream, fstream} (slot streams: slot 0, 1)
// float4s per splat in a COR footprint record: box, ellipse terms e0, e1, one unused (the record is one 64-B line
// sector: a filter test reads one sector instead of a box sector plus an ellipse sector)
constexpr uint32_t kFpWords = 4;
// The events that order the render, prep and frontier streams. They sync device work only; the host waits on
// streams. A device-scope release is enough, because every stream runs on this GPU and the data stays in HBM.
// The default system-scope release writes back every L2, and each cross-stream hop pays that.
constexpr unsigned kSyncEventFlags = hipEventDisableTiming | hipEventReleaseToDevice;
// Timing events (gsrt_timing, the sampled render kernel time) only timestamp the stream: without the default
// system-scope fence, recording one does not write back and invalidate the L2s in the middle of the frame's work
// (with it: C3 +0.3-0.4 %, 8-rank share +0.5-1.3 % against these flags; profiles/r04/event_fence_ab.txt).
// Their times are read after the streams are synchronised.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;
// Slot streams: a pipelined COR frame's prep kernels and its render kernel all go on its slot's stream (slot 0:
// pstream, slot 1: fstream), so the render kernel follows its lists in stream order, and the frames of the two
// slots overlap. Each frame renders into its own buffer (a sharded frame's packed[p], else one of two alternating
// ctx->d_share buffers copied into the framebuffer), so consecutive render kernels need no ordering. Without
// slot streams, the render stream waits on an event for the lists, and that cross-stream wait costs 18-27 us per
// frame (kernel traces, profiles/r02c). That only matters for short frames; long ones lose from the overlap.
// So each frame decides from the measured render kernel time (every kTimedEvery-th frame, timing events): slot streams
// below kSlotEnterUs, back above kSlotLeaveUs. Measured: C2 and the 8-rank C3 and C4 shares 6-10 % faster; the 4- and
// 2-rank C3 shares, C3 and C4 1-3 % slower with them. The test switch GSRT_DEBUG_SLOT_STREAMS=0|1 forces them.
constexpr float kSlotEnterUs = 280.0f, kSlotLeaveUs = 360.0f;
// Whole frames (their slot-stream frames render into the alternating share buffers that the framebuffer view follows,
// no copy) gain from slot streams up to longer render times: C4 (0.85 ms render) -2.5 %, C3 (1.34 ms) even, while
// the 4-rank C3 share (0.37 ms) loses 2.8 % (profiles/archive/r03/slot_*.txt). Sampled on slot streams, a frame's render
// kernel time includes the overlapping frame's (C4: 1.30 ms), hence the wide band.
constexpr float kSlotEnterUsFrame = 1000.0f, kSlotLeaveUsFrame = 1500.0f;
// Prep stream priority (GSRT_DEBUG_PREP_PRIORITY unset): the highest while the sampled render kernel time is short (frame
// f+1's prep must finish within frame f's render: its workgroups are dispatched ahead of the render kernel's as
// CUs free up), the lowest once it is long (the prep has the whole render to hide in; at high priority its
// workgroups only delay the render kernel's). Measured at r03: C3 (1.34 ms render) 2.5 % faster at the highest;
// C5 (4-5 ms render, update + refit + 5M projection per frame) 4 % faster at the lowest.
constexpr float kPrioLowAboveUs = 2500.0f, kPrioHighBelowUs = 2000.0f;
constexpr uint32_t kTimedEvery = 8;
struct FrameSlot {
    uint32_t* d_lists = nullptr;               // per-tile sorted candidate ids of the first round
    void* d_list_hdr = nullptr;                // per tile {count | more, group position, last key}
    size_t list_tiles = 0;
    void* d_glist = nullptr;                   // per tile group: sorted candidate keys (kGCap u64)
    void* d_ghdr = nullptr;                    // per group {count | more, 0, last key}
    uint32_t group_cap = 0;
    uint32_t* d_frontier = nullptr;            // per super-group: traversal frontier {count, node ids}
    uint32_t frontier_cap = 0;
    hipEvent_t prepared = nullptr;             // prep kernels done (pstream)
    hipEvent_t rendered = nullptr;             // render kernel done (stream): the slot may be rewritten
    bool render_pending = false;               // `rendered` has been recorded
    hipStream_t rstream = nullptr;             // the stream the slot's last render kernel went on
    hipEvent_t t0 = nullptr, t1 = nullptr;     // timing events around a sampled render kernel (slot streams)
    bool timed = false;                        // t0 / t1 recorded and not read yet
};

struct gsrt_ctx {
    int device = -1;
    hipStream_t stream = nullptr;              // render kernels, scene updates, BVH build/refit, copies
    hipStream_t pstream = nullptr;             // COR prep stage (see FrameSlot)
    hipStream_t fstream = nullptr;             // COR BVH frontier, beside the projection (needs only the boxes)
    // the prep streams come in two priority classes (choose_prep_priority): pstream / fstream point at one set
    hipStream_t prep_hi[kStreamSlots] = {};          // {pstream, fstream} at the highest stream priority
    hipStream_t prep_lo[kStreamSlots] = {};          // the same at the lowest
    bool prep_high = true;                     // pstream / fstream are prep_hi
    hipEvent_t ev_hop[kStreamSlots] = {};            // switching classes: the new set waits for the old one
    hipEvent_t ev_side[kStreamSlots] = {};           // order_update: scene copies on pstream wait for slot stream j's frames
    hipEvent_t ev_fit = nullptr;               // pstream: the slot's boxes are fitted (frontier may start)
    hipEvent_t ev_front = nullptr;             // fstream: the frontier is done (group lists may start)
    hipEvent_t ev_main = nullptr;              // stream position the prep stage must not overtake
    hipEvent_t ev_lists = nullptr;             // side lists: the frame's prep head is done (its group lists may start)
    bool scene_moved = false;                  // a scene update, page stream or refit came since the last COR frame
    bool main_dirty = true;                    // stream has work since ev_main that the next prep must wait for
    bool main_dirty_f = true;                  // the same for the next frame on fstream (slot streams)
    bool serial_pending = false;               // a REF / counting render on `stream` (reads d_params / d_aabbs)
                                               // that scene updates on pstream have not been ordered after
    hipEvent_t ev_serial = nullptr;            // stream: position of that render (update / refit copies wait)
    // scene updates (gsrt_scene_update / gsrt_refit_bvh from a source) copy into the array's other buffer on the update
    // stream, created at the first one (gsrt_update_stream); ev_copied marks the last copy, which the streams in
    // copy_unseen (bits: prep_hi[0], prep_hi[1], prep_lo[0], prep_lo[1], stream) wait for before they next read an array
    hipStream_t ustream = nullptr;
    hipStream_t cstream = nullptr;             // the comm stream (gsrt_comm_init takes it), created with the context
    hipEvent_t ev_copied = nullptr;
    uint32_t copy_unseen = 0;
    bool serial_reads = false;                 // a REF / counting frame read the arrays on `stream` since the last update
    uint32_t frame_no = 0;                     // COR frames launched
    uint32_t nslots = 2;                       // frame slots in rotation (choose_slots)
    uint32_t next_slot = 0;                    // the slot of the next COR frame
    uint32_t prev_slot = 0;                    // the slot of the last one
    bool slot_mode = false;                    // slot streams chosen for the next frames (use_slot_streams)
    bool last_slot_streams = false;            // the last frame went on slot streams (gsrt_slot_streams)
    float render_us = -1.0f;                   // the last sampled render kernel time (us), -1 = none yet
    bool side_frames[kStreamSlots] = {};             // slot streams: frames on slot stream j > 0 since scene updates last waited
    bool side_updates[kStreamSlots] = {};            // slot streams: update copies on pstream the next frame on slot stream j awaits
    float* d_share[2] = {nullptr, nullptr};    // slot streams: alternating frame outputs (packed shares or frames)
    float* fb_view = nullptr;                  // the last frame's output when it is not d_fb (a slot-stream frame)
    bool fb_dump8 = false;                     // the last frame was a GSRT_FLAG_OUT_DUMP8 sharded frame: no RGBA32F image
                                               // (gsrt_framebuffer returns NULL until the next RGBA32F frame)
    size_t share_floats = 0;
    uint32_t share_parity = 0;
    hipEvent_t ev_share[2] = {nullptr, nullptr};  // stream: share p copied out (it may be rendered into again)
    bool share_pending[2] = {false, false};
    FrameSlot slot[kSlots];
    std::string last_error;
    int num_cus = 256;
    // framebuffer + per-frame scratch, grown on demand
    float* d_fb = nullptr;
    size_t fb_pixels = 0;
    uint32_t* d_ray_stats = nullptr;
    size_t ray_stats_pixels = 0;
    unsigned long long* d_counters = nullptr;  // kCounters words: [0..7] stats, [kErrWord] sticky error word
    uint32_t* d_tile_counter = nullptr;
    uint32_t last_w = 0, last_h = 0;
    bool last_stats = false;
    bool last_ref = false;                     // the last render was REF (gsrt_vs_stats)
    gsrt_comm_state* comm = nullptr;
    float* d_lut = nullptr;                    // ExpLUT (256 segments, 2 floats each)
    float* d_tri_t = nullptr;                  // REF frames of a scene with a mesh: closest triangle t per pixel
    size_t tri_t_pixels = 0;
    uint32_t* d_group_order = nullptr;         // COR k_group_list dispatch order (centre-out), per frame geometry
    uint32_t group_order_key[5] = {};          // {groups_x, groups, mode, rank, nranks} it was built for
    uint32_t group_own = 0;                    // groups at the head of d_group_order with a tile of the rank's band
    uint32_t* d_run_order = nullptr;           // k_render_cor: centre-out order of its runs of local tiles
    uint32_t run_order_key[5] = {0, 0, 0, 0, 0};  // {local tiles, row0, row1, tiles_x, tiles_y} it was built for
    uint32_t* d_tile_cost[kSlots] = {};        // per frame slot: per tile, the shading cost in the slot's last whole COR
    uint32_t tile_cost_cap = 0;                // frame (k_render_cor: staged candidates + a constant; gsrt_row_costs)
    uint32_t tile_cost_slot = 0, tile_cost_tx = 0, tile_cost_ty = 0;  // the last whole COR frame's slot and tile grid
    // HIP-event timing (gsrt_timing): kTimingEvents events per frame {frame start, kernel start, kernel end, frame
    // end, exchange start, exchange end}; the last two (a sharded frame's gather + unpack, on the comm stream) only
    // where timing_ex[frame] is set
    std::vector<hipEvent_t> events;
    std::vector<uint8_t> timing_ex;
    uint32_t timing_cap = 0, timing_n = 0;
    bool timing_kernel_only = false;           // gsrt_timing_kernel_only: no frame start / end events
    bool timing_kernel_only_next = false;      // (set by the call, taken over at gsrt_timing)
    uint32_t timing_stride = 1, timing_stride_next = 1;  // gsrt_timing_stride: events on every stride-th frame
    uint32_t timing_frame = 0;                 // frames seen since gsrt_timing (recorded or not)
};

struct gsrt_scene {
    gsrt_ctx* ctx = nullptr;
    uint32_t n = 0;
    gsrt_gauss_param* d_params = nullptr;  // the current buffer of each array (d_buf[0][cur[0]], d_buf[1][cur[1]])
    gsrt_aabb* d_aabbs = nullptr;
    // double-buffered arrays ([0] params, [1] AABBs; buffer 1 allocated at the first update): an update fills the
    // buffer that is not current, after the kernels that read it while it was current (ev_ret, recorded on the reader
    // streams when it was retired: [0] pstream, [1] fstream, [2] the render stream when a REF / counting frame read it)
    void* d_buf[2][2] = {};
    uint32_t cur[2] = {0, 0};
    const void* attached[2] = {};                    // a borrowed caller array (gsrt_scene_attach) is current, else null
    hipEvent_t ev_ret[2][2][3] = {};
    bool ret_rec[2][2][3] = {};
    float* d_sh = nullptr;
    uint32_t* d_flags = nullptr;                     // [0]: a keyed centre lay outside its AABB's depth bound (k_project,
                                                     // sticky until the next build): the traversals' depth cull is off
    gsrt::SplatRec* d_recs[kSlots] = {};             // per frame slot (FrameSlot); REF and stats use [0]
    uint32_t* d_keyed[kSlots] = {};                  // per frame slot: k_project's keyed bitmap (1 bit per splat;
                                                     // all ones after a build or an unbooked write of the slot)
    float4* d_footprint[kSlots] = {};                // COR per frame slot: per splat one 64-B record (kFpWords
                                                     // float4s): pixel box {x0, x1, y0, y1}, two ellipse terms
    // LBVH
    bool bvh_built = false;
    gsrt::BvhNode* d_nodes[kSlots] = {};  // n-1 internal nodes per frame slot: one topology (copied at build), the
                                          // boxes fitted per slot (slot_geom), the slot's per-frame leaf keys
    uint32_t* d_leaf_parent = nullptr;    // per sorted leaf: parent index | side << 31
    uint32_t* d_node_parent = nullptr;    // per internal node: parent index | side << 31 (all ones: root)
    uint32_t* d_gid_slot = nullptr;       // per gaussian id: its leaf's parent | side << 31 (key slot)
    uint32_t* d_leaf_gid = nullptr;       // sorted leaf -> gaussian id
    uint32_t* d_morton = nullptr;         // sorted morton codes
    uint2* d_node_range = nullptr;        // per internal node: its sorted leaf range [lo, hi] (the chunked fit)
    uint32_t* d_fit_flags[kSlots] = {};   // per slot: arrival counts of the chunk-crossing nodes (zero between fits)
    uint32_t* d_fit_queue[kSlots] = {};   // per slot: the fit's counts and node queues (gsrt_lbvh.hip FitQueues)
    uint32_t* d_sort = nullptr;           // build scratch: radix ping-pong, block histograms, digit totals, bounds
    float* d_root_box[kSlots] = {};       // per slot: 6 floats, written by the fit on the device
    uint32_t root_ref = 0;
    // Refits are lazy: gsrt_refit_bvh bumps geom_version (after queueing the AABB copy on the prep stream);
    // a slot's boxes are fitted when a frame (or a download) uses it and slot_geom[b] != geom_version. So the
    // refit of frame f+1 runs on the prep stream beside frame f's render kernel, which reads its own slot.
    uint64_t geom_version = 1;
    uint64_t slot_geom[kSlots] = {};
    // the slot's nodes hold footprint boxes in their leaf slots (a COR frame's k_project wrote them, leaf_fp):
    // a frame or download that needs the leaf AABBs (REF, the counting pass, gsrt_bvh_*) refits the slot first
    bool slot_leaf_fp[kSlots] = {};
    // the slot's boxes come from a band-restricted fit (FitBand) for slot_band_key: valid for the frames of that band
    // and camera only; any other frame refits the slot
    bool slot_banded[kSlots] = {};
    gsrt::FitBandKey slot_band_key[kSlots] = {};
    // rank shares project in sorted-leaf order (k_prep_cor): the slot's keyed bitmap is then indexed by sorted leaf,
    // not by gaussian id, and 64-leaf chunks none of whose splats are in the band are rejected whole
    bool slot_keyed_leaf[kSlots] = {};
    // per slot, a rank share's in-band bitmap (k_classify: 1 bit per gaussian id, may_own_box of its AABB under the
    // frame's camera and band), valid for the AABBs of version slot_inband_ver and the key slot_inband_key: the band
    // fit and the projection read it instead of the AABBs of splats the band cannot see
    uint32_t* d_inband[kSlots] = {};
    uint64_t slot_inband_ver[kSlots] = {};
    gsrt::FitBandKey slot_inband_key[kSlots] = {};
    uint64_t aabb_version = 1;             // bumped whenever d_aabbs changes (update, page stream, refit from a source)
    uint32_t last_slot = 0;               // the slot of the last frame rendered (bvh_download shows its keys)
    // triangle meshes (gsrt_mesh.cpp): every mesh added, p0 p1 p2 per triangle on the host; in HBM in the mesh
    // BVH's leaf order, 3 float4 per triangle {p0, id bits}, {p1 - p0}, {p2 - p0}, and the BVH (node 0 = root)
    std::vector<float> h_tris;
    uint32_t ntri = 0;
    float4* d_tris = nullptr;
    gsrt::BvhNode* d_mesh_nodes = nullptr;
};

namespace gsrt {

inline gsrt_status fail(gsrt_ctx* ctx, gsrt_status s, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return s;
}

#define GSRT_HIP(ctx, expr)                                                                     \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return ::gsrt::fail((ctx), GSRT_E_DEVICE,                                           \
                                std::string(#expr) + ": " + hipGetErrorString(_e));             \
    } while (0)

// ---- kernels (gsrt_scene.hip) ----
void launch_cov3d(hipStream_t s, uint32_t n, const float* center, const float* rot, const float* scale,
                  const float* opacity, gsrt_gauss_param* params, gsrt_aabb* aabbs);
void launch_project(hipStream_t s, uint32_t n, uint32_t mode, const gsrt_ubo& ubo, const gsrt_gauss_param* params,
                    const gsrt_aabb* aabbs, SplatRec* recs, BvhNode* nodes, const uint32_t* gid_slot,
                    float4* footprint, unsigned long long* counters,  // also zeroes the counters but kErrWord
                    const RankTiles* own,   // sharded frames: keep only the splats this rank's tiles can see
                    uint32_t* keyed,        // COR: the slot's keyed bitmap (k_project), or nullptr
                    bool leaf_fp,           // COR: also write each leaf's footprint box into its node slot
                    uint32_t* depth_unsafe);  // COR: the scene's depth-cull guard word (depth_lo), or nullptr

// ---- LBVH (gsrt_lbvh.hip) ----
gsrt_status lbvh_alloc(gsrt_scene* sc);                          // every BVH buffer (at scene creation)
gsrt_status lbvh_build(gsrt_scene* sc);                          // on ctx->stream, every slot fitted
// slot's boxes from d_aabbs (async); band: restricted to what the band can see (FitBand), nullptr: every box
gsrt_status lbvh_fit(gsrt_scene* sc, uint32_t slot, hipStream_t st, const FitBand* band = nullptr);
// fit slot b on `st` if its boxes are older than the scene's geometry version, or restricted to another band than
// band_key (band nullptr: the frame needs every box; else the frame's in-band bitmap for band_key)
gsrt_status lbvh_fit_if_stale(gsrt_scene* sc, uint32_t slot, hipStream_t st, bool need_aabbs = false,
                              const FitBand* band = nullptr, const FitBandKey* band_key = nullptr);

// ---- meshes (gsrt_mesh_trace.hip): the closest triangle hit t per pixel of a REF frame (kTMax: none) into tri_t
void launch_mesh_thit(hipStream_t s, const gsrt_ubo& ubo, const gsrt_scene* sc, float* tri_t);

// ---- render (gsrt_render.hip) ----
struct RenderPlan {
    uint32_t mode = GSRT_MODE_COR;  // GSRT_MODE_* | flags
    uint32_t cap = 512;             // tile nearest-hit buffer capacity
    uint32_t tw = 8, th = 8;        // tile in pixels
    uint32_t s_lanes = 1;           // in-wave samples per pixel (tw*th*s_lanes == 64)
    uint32_t passes = 1;            // sequential sample passes (samples not in-wave)
    uint32_t tiles_x = 0, tiles_y = 0;
    uint32_t rank = 0, nranks = 1;  // tile ownership: rank owns the tile rows [bands.row[rank], bands.row[rank + 1])
    Bands bands{};
    bool packed = false;            // write packed tiles (sharded render) instead of the framebuffer
    uint32_t fg = 4;                // COR tile groups: fg x fg tiles share one candidate list
    uint32_t row0() const { return bands.row[rank]; }
    uint32_t row1() const { return bands.row[rank + 1]; }
};
// bands: the partition's nranks + 1 row boundaries, or nullptr for uniform_bands (no cost profile)
RenderPlan make_plan(const gsrt_ubo& ubo, uint32_t mode, uint32_t k, uint32_t rank, uint32_t nranks,
                     const uint32_t* bands = nullptr);
// rank 0's weight in the partition: it also receives the other ranks' tiles and unpacks the frame, a cost that grows
// with the exchanged bytes per pixel (mode: GSRT_FLAG_OUT_DUMP8) against a share's shading work (gsrt_comm.cpp)
float root_weight(uint32_t nranks, uint32_t spp, uint32_t mode);
// the boundaries (nranks + 1) that split tile rows 0..tiles_y so that every rank's summed row cost over its weight
// (rank 0: root_w, the others 1) is as even as whole rows allow; row_cost nullptr = every row costs the same. Every
// band gets at least one row when tiles_y >= nranks. Deterministic: every rank computes the same bands from the
// same costs.
void balance_bands(uint32_t tiles_y, uint32_t nranks, const uint32_t* row_cost, float root_w, uint32_t* out);
// the heaviest band's cost over its weight (the balance objective)
double band_peak(uint32_t nranks, const uint32_t* bands, const uint32_t* row_cost, float root_w);
// how a frame's render kernel is ordered against its output buffer's other users (launch_render)
struct RenderSync {
    bool slot = false;          // slot streams for this frame (use_slot_streams), with a private d_rgba
    bool private_out = false;   // d_rgba is not the previous frame's output: no ordering after its render kernel
    hipEvent_t wait = nullptr;  // the render kernel waits for this event (its output buffer is free again)
    hipStream_t stream = nullptr;  // out: the stream the render kernel went on
    bool sharded = false;       // a rank's share of a sharded frame: tile_cost below takes its tiles' costs
    uint32_t* tile_cost = nullptr;  // (sharded) per local tile, its shading cost, or nullptr (not a profile frame)
    // GSRT_FLAG_OUT_DUMP8 (a sharded COR frame): d_rgba is the packed block's code words (Dump8, gsrt_device.hpp),
    // esc its escape list (uint4 count header + esc_cap entries), accum the running sums of spp > 64 passes
    bool dump8 = false;
    uint4* esc = nullptr;
    uint32_t esc_cap = 0;
    float4* accum = nullptr;
};
gsrt_status launch_render(gsrt_scene* sc, const gsrt_ubo& ubo, const RenderPlan& plan, float* d_rgba,
                          gsrt_raystate* d_rs, RenderSync* sync = nullptr);
// row_cost[row0 .. row1) = the band's per-row sums of tile_cost (local tile order of the band)
void launch_row_sum(hipStream_t s, const uint32_t* tile_cost, uint32_t* row_cost, uint32_t tiles_x, uint32_t row0,
                    uint32_t row1);
// Dump8 blocks (gathered: nranks blocks of block_words u32, codes first) -> the code framebuffer (W x H u32)
void launch_unpack_dump8(hipStream_t s, const uint32_t* gathered, uint32_t* codes, const RenderPlan& plan, uint32_t width,
                         uint32_t height, uint32_t tiles_per_rank, size_t block_words);
void launch_unpack(hipStream_t s, const float* gathered, float* fb, const RenderPlan& plan, uint32_t width,
                   uint32_t height, uint32_t tiles_per_rank);
// whether the next pipelined frame (with a private output) goes on slot streams; reads the
// sampled render kernel times that have completed
bool use_slot_streams(gsrt_ctx* ctx, bool share);  // share: a rank's packed share (kSlotEnterUs), else a whole frame
inline uint32_t local_tiles(const RenderPlan& plan) { return plan.tiles_x * (plan.row1() - plan.row0()); }
// GSRT_DEBUG_RANK_OF=N[:r] on a loopback communicator: the sharded render runs rank r of N (gsrt_comm.cpp)
bool debug_rank_of(uint32_t mode, uint32_t& nranks, uint32_t& rank);
uint32_t max_local_tiles(const RenderPlan& plan);  // over all ranks: the packed stride of the gather

// device-to-device copy on s by a copy kernel of one-wave workgroups, each looping over its share (gsrt_scene.hip;
// unaligned pointers or sizes fall back to hipMemcpyAsync)
void launch_copy_d2d(hipStream_t s, void* dst, const void* src, size_t bytes);
// the last frame's framebuffer: d_fb, or the alternating buffer a slot-stream frame rendered into
inline float* framebuffer_of(gsrt_ctx* ctx) { return ctx->fb_view ? ctx->fb_view : ctx->d_fb; }
// the prep stream must not overtake what is on ctx->stream now (scene upload/update, BVH build/refit)
inline void mark_main_dirty(gsrt_ctx* ctx) { if (ctx) ctx->main_dirty = ctx->main_dirty_f = true; }
// slot b's stream on slot streams: pstream, fstream
inline hipStream_t slot_stream(const gsrt_ctx* ctx, uint32_t b) { return b == 0 ? ctx->pstream : ctx->fstream; }
// wait for both streams (before buffers they may use are freed or reallocated)
gsrt_status sync_all(gsrt_ctx* ctx);
// before stream s next reads (or writes) the scene arrays: wait for the update copies it has not seen yet
gsrt_status wait_updates(gsrt_ctx* ctx, hipStream_t s);
// the sticky error word (kErrWord): GSRT_E_DEVICE and cleared when a kernel set it since the last check; waits
// for the streams first
gsrt_status check_error_word(gsrt_ctx* ctx);

// ---- timing (gsrt_api.cpp): which = 0 frame start, 1 kernel start, 2 kernel end, 3 frame end (counts the frame),
// 4 exchange start, 5 exchange end (before the frame's mark 3)
constexpr uint32_t kTimingEvents = 6;
void timing_mark(gsrt_ctx* ctx, int which, hipStream_t s = nullptr);  // s: the render stream by default

// ---- host helpers (gsrt_host.cpp) ----
void exp_lut(float out[512]);

}  // namespace gsrt
