// gsrt_render.hip -- the hot path: per-ray Gaussian intersection + alpha compositing.
//
// Reference path: GaussTracing.rgen round loop -> VulkanRayTracing::traceRay (DFS over
// the Embree BVH, exact slab test, every procedural AABB hit becomes a candidate) ->
// RayTracing.ProceduralGauss.rint per candidate (EWA, LinearExp, K=8 insert) -> .rchit (transmittance).
//
// MI355X design: one wavefront = one 64-ray packet of primary rays (a TW x TH pixel tile x S samples,
// TW*TH*S = 64), one tile per single-wave workgroup. Per tile:
//   1. packet traversal of the LBVH: the wave pops up to 64 nodes at a time from an LDS stack, each lane
//      tests its node's two child boxes against the tile frustum, hit children / leaves are compacted
//      with ballots (no per-lane stacks, no divergence);
//   2. leaf candidates become 64-bit keys in an LDS buffer; a wave bitonic sort orders them (COR: by
//      (depth, id) -- the front-to-back order the reference's K-nearest rounds produce; REF: by id);
//      when more than CAP candidates exist the buffer keeps the CAP nearest and the tile re-traverses
//      for the next CAP beyond the last key (the rgen round loop, done once per 64 rays);
//   3. the sorted candidates are shaded in groups staged through LDS: while group g is shaded (every lane
//      reads the same record: a broadcast), group g+1's records and SH coefficients are already in flight
//      as coalesced vector loads; every lane runs the exact VS slab test for its own ray and the EWA /
//      blend arithmetic.
// The BVH and the frustum are conservative filters; the per-lane slab test decides membership exactly
// as the reference does, so the result does not depend on the BVH, the tile shape or CAP.
//
// Kernel arguments (camera + argument block, ~100 dwords) are never kept live: every use site re-reads
// them with scalar loads through a laundered constant-address-space view of the kernarg segment (kargs()),
// which keeps the SGPR budget for the shading loop instead of spilling it into VGPR lanes.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <type_traits>

#include "gsrt_internal.hpp"
#include "gsrt_project.hpp"

namespace gsrt {

constexpr uint32_t kStack = 512;   // LDS node stack of the 64-wide traversal (entries)
constexpr uint32_t kCap = 256;     // tile nearest-candidate buffer (keys are double-buffered: 2*kCap)
constexpr uint32_t kGroup = 4;     // candidates per LDS stage
constexpr uint32_t kRCap = 128;    // k_render_cor's own traversal rounds (rare: past a group list's end)
constexpr uint32_t kRBuf = 2 * kRCap;
constexpr uint32_t kRStack = 256;
constexpr uint32_t kFG = 4;        // default tile group (kFG x kFG tiles) sharing one sorted candidate list
constexpr uint32_t kGCap = 896;    // candidates per group-list segment
#ifndef GSRT_GROUP_SEGMENTS
#define GSRT_GROUP_SEGMENTS 2
#endif
constexpr uint32_t kGSegs = GSRT_GROUP_SEGMENTS;  // segments of an overflowing group list (k_group_more)
constexpr uint32_t kGStride = kGSegs * kGCap;     // glist entries per group
constexpr uint32_t kMoreLanes = 16;               // k_group_more runs where a tile holds >= 16 samples per pixel
constexpr uint32_t kGBuf = 1024;   // group key buffer (a power of two >= kGCap + 128)
constexpr uint32_t kGStack = 432;  // LDS node stack of the group traversal: 432 entries keep the
                                           // kernel at 10 KB of LDS, 16 waves/CU (1080p: 8160 groups, 2 rounds)
constexpr uint32_t kNoGroup = 0xFFFFFFFFu;
// k_group_list sorts its final list in registers (wave_sort<true>); A/B builds set GSRT_GROUP_REGSORT=0 (LDS network)
#ifndef GSRT_GROUP_REGSORT
#define GSRT_GROUP_REGSORT 1
#endif
constexpr bool kGroupRegSort = GSRT_GROUP_REGSORT != 0;
constexpr uint32_t kSG = 4;        // super-group: kSG x kSG groups sharing one traversal frontier
constexpr uint32_t kFront = 128;   // frontier entries per super-group


struct RenderArgs {
    const SplatRec* recs;
    const float* sh;                 // device layout [gauss][rgb][coef 16]
    const BvhNode* nodes;
    const float* lut;
    float* out;                      // framebuffer RGBA32F or packed tiles
    gsrt_raystate* rs;               // REF per-ray state (nullable)
    uint32_t* ray_stats;             // per-pixel uint4 (nullable)
    unsigned long long* counters;    // [0..7] stats, [8] error flags, [9..31] diagnostics (GSRT_DIAG)
    uint32_t n, root_ref;
    const float* root_box;           // device: 6 floats written by the fit (no host round trip per refit)
    uint32_t width, height, tiles_x, tiles_y, ntiles_local, rank, nranks;
    uint32_t row0, row1;             // this rank's band of tile rows (Bands): its local tiles (band_tile)
    uint32_t* tile_cost;             // COR: per local tile, its shading cost (the partition's profile), or nullptr
    // GSRT_FLAG_OUT_DUMP8 (packed COR frames): out holds one Dump8 code word per pixel, escapes go to esc (count at
    // esc[0].x, entries from esc[1]), passes > 1 sum into accum
    uint32_t dump8, esc_cap;
    uint4* esc;
    float4* accum;
    uint32_t tw, th, s_lanes, passes, packed, samples, bounces;
    uint32_t stack_limit;            // <= kStack; lowered only by the GSRT_DEBUG_STACK_LIMIT test knob
    uint32_t* lists;                 // COR: per local tile, the first round's sorted candidate ids (kCap)
    uint4* list_hdr;                 // per local tile: {count, total, last key lo, last key hi}
    uint32_t prelisted;              // 1: k_collect_cor filled lists/list_hdr for this frame
    uint32_t cull2d;                 // COR: drop listed candidates whose 2D footprint misses the tile (not with STATS)
    uint32_t leaf_fp;                // COR: leaf slots of the nodes hold footprint boxes (k_project): traversals test
                                     // those instead of the leaf AABB, and need no footprint cull afterwards
    uint32_t use_groups;             // COR: k_group_list builds the tile lists (else k_collect_cor per tile)
    uint32_t* frontier;              // per super-group: {count, kFront node ids} (k_frontier), or nullptr
    uint32_t sgroups_x, sgroups;
    uint64_t* glist;                 // per group: its sorted candidate keys (kGStride), for continuation rounds
    uint4* ghdr;                     // per group: {count | more << 31, 0, last key lo, hi}
    const float4* footprint;         // COR: per splat a kFpWords record: pixel box {x0, x1, y0, y1}, ellipse terms
                                     // e0, e1 (k_project)
    uint32_t groups_x, groups;       // tile groups of fg x fg tiles over the whole frame
    uint32_t fg;                     // tiles per group side (RenderPlan::fg: 4, or 2 with 4+ ranks)
    const uint32_t* group_order;     // k_group_list: workgroup -> group (centre first), or nullptr (row-major)
    RankTiles own;                   // sharded frames: the rank's tiles (k_frontier skips super-groups it does not own)
    const uint32_t* run_order;       // k_render_cor: dispatch order of the runs of kRun local tiles (xcd_local_tile_perm)
    const float* tri_t;              // REF with a mesh: closest triangle hit t per pixel (k_mesh_thit), or nullptr
    const uint32_t* depth_unsafe;    // COR: the scene's word k_project sets when a keyed centre lies outside its AABB's
                                     // depth bound (depth_lo): the traversals' depth cull is off while it is non-zero
    uint32_t depth_cull;             // the traversals' depth cull is on (where group lists overflow, launch_render)
};

#ifdef GSRT_WAVE_TIMES
// diagnostic build (profiles/wave_times.py): per workgroup of the last launch {start, end} of the 100-MHz
// real-time counter, HW_ID and XCC_ID; [0] k_render_cor, [1] k_group_list
__device__ uint4 g_wave_times[2][1u << 18];
__device__ uint32_t g_stamps[4];  // real-time counter when the render stream reaches the render kernel / after it
__global__ void k_stamp(uint32_t i) { g_stamps[i] = (uint32_t)__builtin_amdgcn_s_memrealtime(); }
__device__ GSRT_INLINE void wave_time(uint32_t kind, uint32_t idx, uint32_t t0) {
    if (__lane_id() == 0 && idx < (1u << 18))
        g_wave_times[kind][idx] = make_uint4(t0, (uint32_t)__builtin_amdgcn_s_memrealtime(),
                                                    __builtin_amdgcn_s_getreg((31 << 11) | 4),
                                                    __builtin_amdgcn_s_getreg((31 << 11) | 20));
}
#define GSRT_WT_START const uint32_t wt_start = (uint32_t)__builtin_amdgcn_s_memrealtime()
#define GSRT_WT_END(kind, idx) wave_time(kind, idx, wt_start)
#else
#define GSRT_WT_START
#define GSRT_WT_END(kind, idx)
#endif

struct KArgs {                       // the single by-value kernel argument
    gsrt_ubo ubo;
    RenderArgs a;
};

// Fresh view of the kernel arguments: the asm makes the pointer opaque, so loads through it cannot be
// hoisted to kernel entry and stay short-lived scalar loads at each use site.
__device__ GSRT_INLINE const KArgs& kargs() {
    const __attribute__((address_space(4))) KArgs* p =
        (const __attribute__((address_space(4))) KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const KArgs*)p;
}

// ---- tile order: spatial_tile / spatial_index / owner_of live in gsrt_device.hpp (the projection uses them too)
constexpr uint32_t kXcds = 8;

// Workgroup b of a launch over nl local tiles -> local tile index. Under round-robin dispatch the
// workgroups of XCD x are b = x, x+8, ...; they are given whole runs of kRun consecutive tiles of the
// spatial order (one super-tile), runs dealt round-robin over the XCDs: an XCD's in-flight tiles share
// their Gaussians in its L2, and neighbouring runs (similar cost) run on all XCDs at once. A bijection on
// every complete round of 8 runs; the final partial round maps to itself.
__host__ __device__ GSRT_INLINE uint32_t xcd_local_tile(uint32_t b, uint32_t nl) {
    const uint32_t round_len = kXcds * kRun;
    if (b >= (nl / round_len) * round_len) return b;
    const uint32_t x = b % kXcds, i = b / kXcds;
    return ((i / kRun) * kXcds + x) * kRun + i % kRun;
}
// As xcd_local_tile, with units of kDeal consecutive tiles (a quarter super-tile) of the complete rounds taken in
// the order perm lists (centre-out: the costly units first, so the launch ends on short tiles); perm == nullptr:
// spatial order. A rank of a sharded frame has few runs (63 at 8 ranks, C3): dealt whole, the XCDs' shares
// differed by 25 % in cost; quarter runs balance them better and stay spatially coherent.
constexpr uint32_t kDeal = kRun / 4;
__device__ GSRT_INLINE uint32_t xcd_local_tile_perm(uint32_t b, uint32_t nl, const uint32_t* perm) {
    const uint32_t round_len = kXcds * kDeal;
    if (!perm || b >= (nl / round_len) * round_len) return xcd_local_tile(b, nl);
    const uint32_t x = b % kXcds, i = b / kXcds;
    return perm[(i / kDeal) * kXcds + x] * kDeal + i % kDeal;
}


// ---- frustum -------------------------------------------------------------------------------------

struct Frustum { float n[4][3]; float o[3]; };

__device__ GSRT_INLINE void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// Cone from the pinhole through the pixel rectangle [x0,x1] x [y0,y1] (already widened by a margin).
__device__ GSRT_INLINE Frustum make_frustum(const gsrt_ubo& u, float x0, float y0, float x1, float y1) {
    Frustum f;
    float d[4][3];
    gen_ray(u, x0, y0, f.o, d[0]);
    gen_ray(u, x1, y0, f.o, d[1]);
    gen_ray(u, x1, y1, f.o, d[2]);
    gen_ray(u, x0, y1, f.o, d[3]);
    const float c[3] = {d[0][0] + d[1][0] + d[2][0] + d[3][0], d[0][1] + d[1][1] + d[2][1] + d[3][1],
                        d[0][2] + d[1][2] + d[2][2] + d[3][2]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        cross3(d[i], d[(i + 1) & 3], f.n[i]);
        const float s = f.n[i][0] * c[0] + f.n[i][1] * c[1] + f.n[i][2] * c[2];
        if (s < 0.0f) { f.n[i][0] = -f.n[i][0]; f.n[i][1] = -f.n[i][1]; f.n[i][2] = -f.n[i][2]; }
    }
    return f;
}

// true when the box lies strictly outside one side plane (positive-vertex test)
__device__ GSRT_INLINE bool box_outside(const Frustum& f, const float lo[3], const float hi[3]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float v = (f.n[p][k] >= 0.0f ? hi[k] : lo[k]) - f.o[k];
            s = fmaf(f.n[p][k], v, s);
        }
        if (s < 0.0f) return true;
    }
    return false;
}

// ---- wave helpers -------------------------------------------------------------------------------

__device__ GSRT_INLINE uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ GSRT_INLINE uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// the lane id recomputed at this point (laundered): values derived from it in a rarely taken block are not
// hoisted out of the loops around it into long (spilled) live ranges
__device__ GSRT_INLINE uint32_t lane_here() {
    uint32_t l = lane_id();
    asm volatile("" : "+v"(l));
    return l;
}
__device__ GSRT_INLINE uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ GSRT_INLINE unsigned long long wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Wave-wide bitonic sort of keys[0..count) ascending in LDS (padded to a power of two with ~0).
// Bitonic sort of n = 64 R keys held in registers, element r * 64 + lane in v[r]: stages whose partner is in
// another lane exchange through __shfl_xor (no LDS round trip, no barrier), the others within a lane.
template <uint32_t R>
__device__ GSRT_INLINE void wave_sort_regs(uint64_t (&v)[R], uint32_t lane) {
    constexpr uint32_t n = 64 * R;
#pragma unroll
    for (uint32_t k = 2; k <= n; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {  // partner: register r ^ (j / 64) of the same lane
#pragma unroll
                for (uint32_t r = 0; r < R; ++r) {
                    const uint32_t q = r ^ (j / 64);
                    if (q <= r) continue;
                    const bool asc = k == n || ((r * 64) & k) == 0;  // (e & k) == 0 for e = r * 64 + lane
                    const uint64_t a = v[r], c = v[q];
                    const bool sw = (a > c) == asc;
                    v[r] = sw ? c : a;
                    v[q] = sw ? a : c;
                }
            } else {  // partner: lane ^ j, same register
                // the lane id laundered per stage: the stage's lane masks are formed here, not hoisted to the top of
                // the kernel as dozens of live SGPR pairs (spilled once the sort is inlined into its caller)
                uint32_t ln = lane;
                asm volatile("" : "+v"(ln));
                const bool lower = (ln & j) == 0;
#pragma unroll
                for (uint32_t r = 0; r < R; ++r) {
                    const uint32_t e = r * 64 + ln;
                    const bool asc = (e & k) == 0;
                    const uint64_t a = v[r];
                    const uint32_t plo = (uint32_t)__shfl_xor((int)(uint32_t)a, (int)j);
                    const uint32_t phi = (uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), (int)j);
                    const uint64_t p = ((uint64_t)phi << 32) | plo;
                    const bool keep_min = lower == asc;
                    const bool a_small = a < p;
                    v[r] = (a_small == keep_min) ? a : p;
                }
            }
        }
    }
}

template <uint32_t R>
__device__ GSRT_INLINE void wave_sort_r(uint64_t* keys, uint32_t count, uint32_t lane) {
    uint64_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = r * 64 + lane;
        v[r] = e < count ? keys[e] : ~0ull;
    }
    wave_sort_regs<R>(v, lane);
    __syncthreads();  // every lane has read its elements
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) keys[r * 64 + lane] = v[r];
    __syncthreads();
}

// Sort keys[0..count) ascending; keys[count..n) (n = count rounded up to a power of two) become ~0.
// REGS (k_group_list, where the sort is on the latency chain of every group): counts up to 1024 sort in
// registers (wave_sort_r, up to 32 VGPRs of keys; the kernel takes 104 VGPRs instead of 75, which costs no
// occupancy: its 10 KB of LDS hold it to 4 waves/SIMD, and beside the render kernel a group-list wave takes the
// slot of one retiring 80-VGPR render wave either way; C3 -0.8 %, C2 -0.6 % against sorting 513-1024 keys in
// LDS); otherwise (the render kernels' rare traversals, whose occupancy depends on their VGPR count) the LDS
// bitonic network below.
template <bool REGS = false>
__device__ GSRT_INLINE void wave_sort(uint64_t* keys, uint32_t count) {
    const uint32_t lane = lane_id();
    if constexpr (REGS) {
        count = __builtin_amdgcn_readfirstlane(count);
        if (count <= 64) { wave_sort_r<1>(keys, count, lane); return; }
        if (count <= 128) { wave_sort_r<2>(keys, count, lane); return; }
        if (count <= 256) { wave_sort_r<4>(keys, count, lane); return; }
        if (count <= 512) { wave_sort_r<8>(keys, count, lane); return; }
        if (count <= 1024) { wave_sort_r<16>(keys, count, lane); return; }
    }
    uint32_t n = 2;
    while (n < count) n <<= 1;
    for (uint32_t i = count + lane; i < n; i += 64) keys[i] = ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = lane; t < (n >> 1); t += 64) {
                const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const uint32_t l = i + j;
                const bool up = (i & k) == 0;
                const uint64_t a = keys[i], b = keys[l];
                if ((a > b) == up) { keys[i] = b; keys[l] = a; }
            }
            __syncthreads();
        }
    }
}

// keys[0..P) sorted ascending, keys[P..count) not (count <= BUF, BUF a power of two, BUF - P = 64 R): afterwards keys[0..BUF)
// is sorted ascending (keys[count..BUF) hold ~0 first). The tail is sorted in registers (R keys per lane) and written back
// descending, so that keys[0..BUF) is one bitonic sequence, which a single bitonic merge (log2 BUF half-cleaner stages
// over LDS) sorts: the overflow of a traversal's key buffer re-sorts its 128 new keys instead of all BUF.
template <uint32_t BUF, uint32_t P>
__device__ GSRT_INLINE void merge_tail(uint64_t* keys, uint32_t count) {
    static_assert((BUF & (BUF - 1)) == 0 && BUF > P && (BUF - P) % 64 == 0, "merge_tail: BUF - P a multiple of 64");
    constexpr uint32_t R = (BUF - P) / 64;
    const uint32_t lane = lane_id();
    uint64_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t e = P + r * 64 + lane;
        v[r] = e < count ? keys[e] : ~0ull;
    }
    wave_sort_regs<R>(v, lane);
    __syncthreads();  // every lane has read its tail keys
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) keys[BUF - 1 - (r * 64 + lane)] = v[r];
    __syncthreads();
#pragma unroll 1
    for (uint32_t j = BUF >> 1; j > 0; j >>= 1) {
#pragma unroll 2
        for (uint32_t t = lane; t < (BUF >> 1); t += 64) {
            const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
            const uint64_t a = keys[i], b = keys[i + j];
            if (a > b) { keys[i] = b; keys[i + j] = a; }
        }
        __syncthreads();
    }
}

// ---- packet traversal ---------------------------------------------------------------------------

struct KeyRef {  // REF: candidates ordered by Gaussian id (the oracle's order)
    static constexpr bool kUsesDepth = false;
    __device__ GSRT_INLINE bool operator()(uint32_t, uint32_t gid, uint64_t& key) const { key = gid; return true; }
};
struct KeyCor {  // COR: (depth, id); invalid splats (behind the camera, singular: depth = +inf) never enter
    static constexpr bool kUsesDepth = true;
    __device__ GSRT_INLINE bool operator()(uint32_t depth_bits, uint32_t gid, uint64_t& key) const {
        key = ((uint64_t)depth_bits << 32) | gid;
        return depth_bits < 0x7f800000u;
    }
};
// COR inside k_render_cor: the same key, its depth read from the frame's own records. The leaf keys in the
// BVH nodes belong to the prep stage, which may already be writing the next frame's (FrameSlot).
struct KeyCorRec {
    static constexpr bool kUsesDepth = true;
    __device__ GSRT_INLINE bool operator()(uint32_t, uint32_t gid, uint64_t& key) const {
        return KeyCor{}(__float_as_uint(kargs().a.recs[gid].depth), gid, key);
    }
};

// pixel rectangle the tile's rays pass through (with margin)
struct TileRect { float x0, y0, x1, y1; };

__device__ GSRT_INLINE TileRect tile_rect(uint32_t tx, uint32_t ty, uint32_t tw, uint32_t th) {
    const uint32_t x0 = tx * tw, y0 = ty * th;
    return TileRect{(float)x0 - 0.5f, (float)y0 - 0.5f, (float)(x0 + tw) + 0.5f, (float)(y0 + th) + 0.5f};
}
// Footprint test of splat gid against a sample rectangle: its pixel box meets rect and the g-ellipse
// {g <= gcut} meets rect (k_project stores the ellipse widened by 2 % + 2e-3 in g). The rect is a TileRect (with
// its 0.5-px frustum margin); the samples lie in [x0 + 0.5, x1 - 0.5) and the footprints carry their own
// rounding margins, so the test uses the rect without the frustum margin.
constexpr float kFpInset = 0.5f;
// Exact ellipse-rectangle test. With d = p - centre and the ellipse q(d) = (A dx^2 + 2B dx dy + C dy^2) / T <= 1,
// q restricted to an edge dx = X is Cs (dy + kc X)^2 + Dc X^2 (Cs = C/T, kc = B/C, Dc = det/(C T)): a sum of two
// non-negative terms, no cancellation, minimised at dy = -kc X clamped to the edge; likewise for dy = Y edges.
// A convex q meets the rectangle iff its centre lies inside or its minimum over one of the four edges is <= 1.
// e0 = (cx, cy, kc, ka), e1 = (Cs, As, Dc, Da); the rectangle (x0, x1, y0, y1) is widened by kEllMargin.
constexpr float kEllMargin = 0.01f;
__device__ GSRT_INLINE float ell_edge(float X, float k, float s, float d, float lo, float hi) {
    const float m = -k * X;
    const float r = __builtin_amdgcn_fmed3f(m, lo, hi) - m;
    return fmaf(s * r, r, (d * X) * X);
}
__device__ GSRT_INLINE bool ell_meets(const float4 e0, const float4 e1, float x0, float x1, float y0, float y1) {
    const float ax = x0 - e0.x - kEllMargin, bx = x1 - e0.x + kEllMargin;
    const float ay = y0 - e0.y - kEllMargin, by = y1 - e0.y + kEllMargin;
    if (ax <= 0.0f && bx >= 0.0f && ay <= 0.0f && by >= 0.0f) return true;
    const float q = fminf(fminf(ell_edge(ax, e0.z, e1.x, e1.z, ay, by), ell_edge(bx, e0.z, e1.x, e1.z, ay, by)),
                          fminf(ell_edge(ay, e0.w, e1.y, e1.w, ax, bx), ell_edge(by, e0.w, e1.y, e1.w, ax, bx)));
    return q <= 1.0f;
}
template <bool SLABS = true>
__device__ GSRT_INLINE bool fp_meets(const float4* fps, uint32_t gid, const TileRect& r) {
    const float4* rec = fps + kFpWords * (size_t)gid;
    const float4 box = rec[0];
    const float x0 = r.x0 + kFpInset, x1 = r.x1 - kFpInset, y0 = r.y0 + kFpInset, y1 = r.y1 - kFpInset;
    if (!(box.x <= x1 && box.y >= x0 && box.z <= y1 && box.w >= y0)) return false;
    if (!SLABS) return true;
    const float4 e0 = rec[1], e1 = rec[2];
    return ell_meets(e0, e1, x0, x1, y0, y1);
}

// A super-group's BVH frontier (k_frontier: count, then at most kFront = 128 node refs) held in registers:
// lane l has entries l and 64 + l. The group-list kernel loads it all at once, one memory latency
// instead of two dependent ones (count, then entries). n = kNoGroup: start at the root.
struct FrontRegs { uint32_t n = kNoGroup; uint32_t a = 0u, b = 0u; };
static_assert(kFront <= 128, "FrontRegs holds two entries per lane");

// total: leaves passing the frustum test with key > lo; more: some such leaf (that the cull kept) is not in
// keys[0..count), so another round after keys[count-1] is needed
// n: keys held in the buffer (collect<REGSORT>: unsorted; its caller sorts them and keeps count = min(n, CAP))
struct Collected { uint32_t total; uint32_t count; bool restart; bool more; uint32_t n; bool sorted; };

// COR: compact keys[begin..count) in place (from begin) to the candidates that can contribute to some ray
// of the tile: those whose conservative footprint box (k_project: where g <= min(5.6, ln(255 op)), i.e.
// alpha > 1/255 is possible) meets the tile's sample rectangle. The others have alpha 0 for every ray of the
// tile, so dropping them changes nothing (results stay bit-identical); the shading loop just skips them.
// B chunks of 64 keys per round: their footprint boxes are loaded together (B independent loads per lane in
// flight, one memory latency per round instead of one per chunk); the group lists use B = 4, the render kernel's
// rare own traversal B = 1 (VGPR budget). In place: a round's keys are all read before its first write, and the
// writes land below the next round's keys.
template <uint32_t B = 1>
__device__ GSRT_INLINE uint32_t cull_footprints(uint64_t* keys, uint32_t begin, uint32_t count, const TileRect& rect) {
    const float4* fps = kargs().a.footprint;
    const uint32_t lane = lane_id();
    const float x0 = rect.x0 + kFpInset, x1 = rect.x1 - kFpInset, y0 = rect.y0 + kFpInset, y1 = rect.y1 - kFpInset;
    uint32_t out = begin;
    for (uint32_t base = begin; base < count; base += 64 * B) {
        uint64_t key[B];
        float4 box[B];
#pragma unroll
        for (uint32_t j = 0; j < B; ++j) {
            const uint32_t i = base + 64 * j + lane;
            key[j] = i < count ? keys[i] : 0ull;
        }
#pragma unroll
        for (uint32_t j = 0; j < B; ++j) {
            const uint32_t i = base + 64 * j + lane;
            box[j] = i < count ? fps[kFpWords * (size_t)(uint32_t)key[j]] : make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);
        }
#pragma unroll
        for (uint32_t j = 0; j < B; ++j) {
            // the box only (fp_meets<false>): a coarse cull on the traversal rect
            const bool keep = box[j].x <= x1 && box[j].y >= x0 && box[j].z <= y1 && box[j].w >= y0;
            const uint64_t b = __ballot(keep);
            if (keep) keys[out + popc_below(b)] = key[j];
            out += (uint32_t)__popcll(b);
        }
    }
    __syncthreads();
    return out;
}

// Gather the keys of every leaf whose box meets the frustum of rect and whose key > lo (when has_lo), keep
// the CAP smallest sorted in keys[0..count) (keys holds 2*CAP). width = nodes popped per step (64; 1 = plain
// DFS whose stack is bounded by the tree depth, used after the LDS stack of stack_limit entries ran out).
// cull: drop leaves whose 2D footprint misses rect (cull_footprints) before the buffer is truncated, so the
// CAP slots hold only splats that can contribute.
// depth_cull (COR keys, not the counting pass): once the buffer has overflowed (keys beyond the CAP nearest exist, so the
// list is `more` already), an internal child whose box's depth bound (depth_lo) lies beyond the current threshold's depth
// holds only keys the final CAP nearest cannot contain, and is not descended into: a volume's far side is not walked.
// MERGE (k_group_list): an overflowed buffer merges its new keys into its sorted CAP (merge_tail) instead of sorting
// all of it again; the render kernel's rare traversals keep the plain sort (the merge's registers spill there)
template <uint32_t CAP, uint32_t BUF, class KeyFn, bool REGSORT = false, bool MERGE = false>
__device__ GSRT_INLINE Collected collect(const TileRect& rect, uint64_t lo, bool has_lo, uint64_t* keys, uint32_t* stack,
                             uint32_t stack_limit, uint32_t width, KeyFn keyfn, bool cull,
                             const FrontRegs& front = FrontRegs{}, bool depth_cull = false) {
    const KArgs& K = kargs();
    const uint32_t lane = lane_id();
    Collected res{0u, 0u, false, false};
    const uint32_t n = K.a.n;
    if (n == 0) return res;
    const BvhNode* nodes = K.a.nodes;
    const SplatRec* recs = K.a.recs;
    const uint32_t root_ref = K.a.root_ref;
    const Frustum F = make_frustum(K.ubo, rect.x0, rect.y0, rect.x1, rect.y1);
    // COR frames with leaf_fp: a leaf passes when its footprint box meets the rectangle (the cull_footprints test,
    // done here on the box the node already holds), so no footprint cull follows
    const bool leaf_fp = K.a.leaf_fp != 0;
    if (leaf_fp) cull = false;
    const float fx0 = rect.x0 + kFpInset, fx1 = rect.x1 - kFpInset, fy0 = rect.y0 + kFpInset, fy1 = rect.y1 - kFpInset;
    uint32_t count = 0, total = 0, sp = 0, culled = 0;  // keys[0..culled) already passed the cull
    uint32_t sorted_n = 0;  // keys[0..sorted_n) sorted: 0, or CAP once the buffer has overflowed
    uint64_t thresh = ~0ull;
    if (!KeyFn::kUsesDepth || !K.a.depth_cull || (K.a.depth_unsafe && *K.a.depth_unsafe)) depth_cull = false;
    const ZRow zr = zrow_of(K.ubo.model_view);
    float tdepth = INFINITY;  // the depth of thresh (finite once the buffer has overflowed)
    bool more = false;
    const uint32_t nfront = front.n;
    if (nfront != kNoGroup && 2 * nfront + 2 <= stack_limit) {
        // start below the root: a frontier of a region containing rect (every node rect's rays can reach)
        if (lane < nfront) stack[lane] = front.a;
        if (64 + lane < nfront) stack[64 + lane] = front.b;
        sp = nfront;
    } else {
        const float rlo[3] = {K.a.root_box[0], K.a.root_box[1], K.a.root_box[2]};
        const float rhi[3] = {K.a.root_box[3], K.a.root_box[4], K.a.root_box[5]};
        if (!box_outside(F, rlo, rhi)) {
            if (root_ref & kLeafBit) {  // single-Gaussian scene: the root is a leaf, its key is in the record
                uint64_t key;
                const uint32_t gid = root_ref & ~kLeafBit;
                if (keyfn(__float_as_uint(recs[gid].depth), gid, key) && (!has_lo || key > lo)) {
                    total = 1;
                    if (lane == 0) keys[0] = key;
                    count = 1;
                }
            } else {
                if (lane == 0) stack[0] = root_ref;
                sp = 1;
            }
        }
    }
    __syncthreads();
#ifdef GSRT_DIAG  // diagnostic build only: traversal vs final cull+sort cycles, steps, popped nodes
    const unsigned long long dg0 = __builtin_amdgcn_s_memtime();
    unsigned long long dg_steps = 0, dg_nodes = 0;
#endif
    while (sp > 0) {
        uint32_t k = sp < width ? sp : width;
        if (sp + k > stack_limit) {  // each popped node pushes at most 2: keep sp - k + 2k <= limit
            k = sp < stack_limit ? stack_limit - sp : 0u;
            if (k == 0) { res.restart = true; break; }
        }
        if (count + 2 * k > BUF) {
            if (cull) {
                count = cull_footprints<REGSORT ? 4u : 1u>(keys, culled, count, rect);
                culled = count;
            }
            if (count + 2 * k > BUF) {  // keep the CAP nearest, tighten the threshold (the LDS sort)
                // after the first overflow keys[0..CAP) is sorted: merge the new keys in (merge_tail) instead of sorting
                // the whole buffer again (a deep frustum overflows every BUF - CAP keys). A footprint cull compacts the
                // sorted part too, so with one the buffer is sorted whole
                if (MERGE && sorted_n == CAP && !cull) merge_tail<BUF, CAP>(keys, count);
                else wave_sort<false>(keys, count);
                sorted_n = CAP;
                more = more || count > CAP;
                count = CAP;
                if (culled > count) culled = count;
                thresh = keys[CAP - 1];
                tdepth = __uint_as_float((uint32_t)(thresh >> 32));
            }
        }
#ifdef GSRT_DIAG
        ++dg_steps;
        dg_nodes += k;
#endif
        const bool act = lane < k;
        const uint32_t node = act ? stack[sp - k + lane] : 0u;
        __syncthreads();
        sp -= k;
        uint32_t np = 0, na = 0, nt = 0, nr = 0;
        uint32_t p0 = 0, p1 = 0;
        uint64_t a0 = 0, a1 = 0;
        if (act) {
            const BvhNode nd = nodes[node];
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const float* clo = side ? nd.r_lo : nd.l_lo;
                const float* chi = side ? nd.r_hi : nd.l_hi;
                const uint32_t ref = side ? nd.r_ref : nd.l_ref;
                if (leaf_fp && (ref & kLeafBit)) {  // the leaf's footprint box {x0, x1, y0, y1} (put_node_key_fp)
                    if (!(clo[0] <= fx1 && clo[1] >= fx0 && clo[2] <= fy1 && chi[0] >= fy0)) continue;
                } else if (box_outside(F, clo, chi)) {
                    continue;
                }
                if (ref & kLeafBit) {
                    uint64_t key;
                    if (keyfn(side ? nd.r_key : nd.l_key, ref & ~kLeafBit, key) && (!has_lo || key > lo)) {
                        ++nt;
                        if (key < thresh) { if (na == 0) a0 = key; else a1 = key; ++na; }
                        else nr = 1;
                    }
                } else if (!(depth_cull && depth_lo(zr, clo, chi) > tdepth)) {
                    if (np == 0) p0 = ref; else p1 = ref;
                    ++np;
                }
            }
        }
        uint64_t b1 = __ballot(np >= 1), b2 = __ballot(np >= 2);
        uint32_t off = popc_below(b1) + popc_below(b2);
        if (np >= 1) stack[sp + off] = p0;
        if (np >= 2) stack[sp + off + 1] = p1;
        sp += (uint32_t)__popcll(b1) + (uint32_t)__popcll(b2);
        b1 = __ballot(na >= 1); b2 = __ballot(na >= 2);
        off = popc_below(b1) + popc_below(b2);
        if (na >= 1) keys[count + off] = a0;
        if (na >= 2) keys[count + off + 1] = a1;
        count += (uint32_t)__popcll(b1) + (uint32_t)__popcll(b2);
        total += (uint32_t)__popcll(__ballot(nt >= 1)) + (uint32_t)__popcll(__ballot(nt >= 2));
        more = more || __ballot(nr != 0) != 0;  // a leaf beyond the threshold: it belongs to a later round
        __syncthreads();
    }
    if (res.restart) return res;
#ifdef GSRT_DIAG
    const unsigned long long dg1 = __builtin_amdgcn_s_memtime();
#endif
    if (cull) count = cull_footprints<REGSORT ? 4u : 1u>(keys, culled, count, rect);
    // REGSORT: the caller sorts keys[0..n) in registers (one inlined copy of the large register network per kernel);
    // the count and the continuation flag below are those of the sorted, truncated list either way. An overflowed
    // buffer (its first CAP keys sorted, no cull) merges its tail in here instead
    res.sorted = MERGE && sorted_n == CAP && !cull;
    if constexpr (MERGE) {
        if (res.sorted) merge_tail<BUF, CAP>(keys, count);
    }
    if (!res.sorted && !REGSORT) wave_sort<false>(keys, count);
#ifdef GSRT_DIAG
    if (lane == 0) {
        atomicAdd(K.a.counters + 12, dg1 - dg0);
        atomicAdd(K.a.counters + 13, __builtin_amdgcn_s_memtime() - dg1);
        atomicAdd(K.a.counters + 14, dg_steps);
        atomicAdd(K.a.counters + 15, dg_nodes);
    }
#endif
    res.total = total;
    res.more = more || count > CAP;
    res.count = count < CAP ? count : CAP;
    res.n = count;
    return res;
}

template <uint32_t CAP = kCap, uint32_t BUF = 2 * CAP, class KeyFn, bool REGSORT = false, bool MERGE = false>
__device__ GSRT_INLINE Collected collect_robust(const TileRect& rect, uint64_t lo, bool has_lo, uint64_t* keys,
                                           uint32_t* stack, KeyFn keyfn, uint32_t& restarts, bool cull = false,
                                           uint32_t stack_limit = 0, const FrontRegs& front = FrontRegs{},
                                           bool depth_cull = false) {
    if (!stack_limit) stack_limit = kargs().a.stack_limit;
    static_assert((BUF & (BUF - 1)) == 0 && BUF >= CAP + 128, "keys buffer: a power of two (wave_sort pads to one) with room for a step");
    // a 64-wide packet walk, and after a stack overflow the one-node-wide DFS
    Collected c;
    if constexpr (MERGE) {  // (one inlined copy of collect for both widths: the group-list kernel stays compact)
        for (uint32_t width = 64u;; width = 1u) {
            c = collect<CAP, BUF, KeyFn, REGSORT, MERGE>(rect, lo, has_lo, keys, stack, stack_limit, width, keyfn, cull,
                                                         front, depth_cull);
            if (!c.restart || width == 1u) break;
            ++restarts;
            __syncthreads();
        }
    } else {
        c = collect<CAP, BUF, KeyFn, REGSORT, MERGE>(rect, lo, has_lo, keys, stack, stack_limit, 64u, keyfn, cull, front,
                                                     depth_cull);
        if (c.restart) {
            ++restarts;
            __syncthreads();
            c = collect<CAP, BUF, KeyFn, REGSORT, MERGE>(rect, lo, has_lo, keys, stack, stack_limit, 1u, keyfn, cull, front,
                                                         depth_cull);
        }
    }
    if (c.restart && lane_id() == 0) atomicOr(kargs().a.counters + kErrWord, 1ull);
    if (REGSORT && !c.restart && !c.sorted) wave_sort<true>(keys, c.n);  // the one register-sort site of the kernel
    return c;
}

__device__ GSRT_INLINE void add_counters(unsigned long long rays, unsigned long long cand, unsigned long long blended,
                                    unsigned long long term, unsigned long long rounds, unsigned long long restarts,
                                    unsigned long long maxc) {
    if (lane_id() != 0) return;
    unsigned long long* c = kargs().a.counters;
    atomicAdd(c + 0, rays);
    atomicAdd(c + 1, cand);
    atomicAdd(c + 2, blended);
    atomicAdd(c + 3, term);
    atomicAdd(c + 4, rounds);
    atomicAdd(c + 5, restarts);
    atomicAdd(c + 6, 1ull);
    atomicMax(c + 7, maxc);
}

// ----------------------------------------------------------------------------------------- COR

// LDS stage of one group of sorted candidates: the 64-B records and the SH-3 coefficients. Filled by LDS-DMA
// (global_load_lds, 16 B per lane, no VGPR destination): the stage is 16-B pieces in lane order, records first.
struct Stage {
    SplatRec rec[kGroup];         // kGroup * 64 B
    float sh[kGroup][3][16];      // kGroup * 192 B, device layout [gauss][rgb][coef]
};
static_assert(sizeof(Stage) == kGroup * 256 && sizeof(Stage) % 1024 == 0, "whole wave-instructions of 16-B pieces");

// DMA instructions per stage (one 16-B piece per lane each), and the wait for the stage issued `younger`
// stages before the most recent one: vmcnt counts VMEM operations in issue order, so vmcnt(younger * ops)
// leaves the younger stages' DMAs in flight (any other younger VMEM operation only makes the wait stricter)
template <bool SH>
constexpr uint32_t kStagePieces = SH ? 16 * kGroup : 4 * kGroup;
template <bool SH>
constexpr uint32_t kStagePieceOps = (kStagePieces<SH> + 63) / 64;
template <uint32_t N>
__device__ GSRT_INLINE void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <bool SH>
__device__ GSRT_INLINE void wait_stage(uint32_t younger) {
    constexpr uint32_t P = kStagePieceOps<SH>;
    if (younger >= 2) wait_vmcnt<2 * P>();
    else if (younger == 1) wait_vmcnt<P>();
    else wait_vmcnt<0>();
}

// A read of LDS that no LDS-DMA in flight writes (the round's id list, complete before shading starts), hidden from
// the compiler's LDS-DMA tracking: a plain read of it after a stage's DMA makes the compiler wait for vmcnt(0), i.e.
// for every stage in flight, which would leave the stage pipeline one stage deep. The value is waited for here.
__device__ GSRT_INLINE uint32_t lds_read_settled(const uint32_t* p) {
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// issue the LDS-DMA of group g0 of ids[0..count) into dst: piece p < 4*kGroup is quarter p&3 of record p>>2,
// the next 12*kGroup pieces are the SH rows (12 pieces each); piece p lands at byte 16 p of the stage. Every
// lane computes its piece's address the same way (base, row stride and offset selected, no divergent paths).
// Waited for by wait_stage before the stage is read.
template <bool SH>
__device__ GSRT_INLINE void stage_issue(const uint32_t* ids, uint32_t count, uint32_t g0, uint32_t lane, Stage* dst,
                                   const SplatRec* recs, const float* sh) {
    constexpr uint32_t kRecPieces = 4 * kGroup, kPieces = kStagePieces<SH>;
#pragma unroll
    for (uint32_t i = 0; i < (kPieces + 63) / 64; ++i) {
        const uint32_t p = i * 64 + lane;
        const bool is_rec = p < kRecPieces;
        const uint32_t q = p - kRecPieces;
        uint32_t c = g0 + (is_rec ? p >> 2 : q / 12);
        c = c < count ? c : g0;  // past the list's end: a copy of candidate g0 (never read; keeps lane 0 active)
        if (p < kPieces) {       // lane 0 always loads: each stage is exactly kStagePieceOps DMA instructions
            const uint32_t id = lds_read_settled(ids + c);
            const char* base = is_rec ? reinterpret_cast<const char*>(recs) : reinterpret_cast<const char*>(sh);
            const uint32_t stride = is_rec ? 64u : 192u, off = is_rec ? (p & 3) * 16u : (q % 12) * 16u;
            __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)id * stride + off),
                                             (void*)(reinterpret_cast<char*>(dst) + i * 1024), 16, 0, 0);
        }
    }
}

// and its first 128 ids into ids[0..128) (waited for by the next vmcnt(0), i.e. __syncthreads)
__device__ GSRT_INLINE void list_issue(uint32_t lt, uint32_t lane, uint32_t* ids, uint32_t* hdr) {
    const KArgs& K = kargs();
    const uint32_t* src = K.a.lists + (size_t)lt * kCap;
    __builtin_amdgcn_global_load_lds((const void*)(src + lane), (void*)ids, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 64 + lane), (void*)(ids + 64), 4, 0, 0);
    if (lane < 4)
        __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const uint32_t*>(K.a.list_hdr + lt) + lane),
                                         (void*)hdr, 4, 0, 0);
}

struct CorRay {
    ObjRay R;
    float pxs, pys;
    float bs[16];
    float T, C[3];
    bool active;
    uint32_t cand, blended, term;
#ifdef GSRT_DIAG
    // wave-candidates (per wave, lane 0 adds): staged while some lane active; some lane passed g; some lane's
    // alpha > 0; some lane blended (SH evaluated); lane-candidates passing g; lane blends
    uint32_t dg_staged, dg_gpass, dg_contrib, dg_blend, dg_lanes_g, dg_lanes_blend;
#endif
};

// Front-to-back blend of candidate c (alpha 0: no contribution) into every lane's ray; the SH-3 colour only
// when some lane blends. A ray whose transmittance would drop below 1e-4 stops (the hit is not blended):
// returns true on the lane whose ray stopped here.
// channel colour 0.5 + sum basis * coef (the 0.5 and s_0 Y_0 folded into coefficient 0, gsrt_api.cpp upload_common),
// clamped at 0: the same fma chain whatever the coefficients' home
__device__ GSRT_INLINE float sh_channel(const float (&bs)[16], const float (&s)[16]) {
    float a = s[0];
#pragma unroll
    for (int q = 1; q < 16; ++q) a = fmaf(bs[q], s[q], a);
    return a > 0.0f ? a : 0.0f;
}
struct ShFromStage {  // the stage's LDS copy of candidate c's row
    const Stage* stg;
    uint32_t c;
    __device__ GSRT_INLINE void operator()(const float (&bs)[16], float (&col)[3]) const {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const float4* s4 = reinterpret_cast<const float4*>(stg->sh[c][ch]);
            const float4 q0 = s4[0], q1 = s4[1], q2 = s4[2], q3 = s4[3];
            const float s[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                 q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            col[ch] = sh_channel(bs, s);
        }
    }
};
template <bool SH, bool STATS, class ShSrc>
__device__ GSRT_INLINE bool blend_hit(const ShSrc& shsrc, float alpha, bool contrib, CorRay& ray) {
    const float tn = ray.T * (1.0f - alpha);
    const bool low = tn < 1e-4f;  // one compare serves both masks
    const bool term = contrib && low;
    const bool blend = contrib && !low;
    if (__ballot(blend)) {
        float col[3] = {1.0f, 1.0f, 1.0f};
        if (SH) shsrc(ray.bs, col);
        if (blend) {
            const float w = alpha * ray.T;
            ray.C[0] = fmaf(col[0], w, ray.C[0]);
            ray.C[1] = fmaf(col[1], w, ray.C[1]);
            ray.C[2] = fmaf(col[2], w, ray.C[2]);
            ray.T = tn;
            if (STATS) ++ray.blended;
        }
    }
    if (term) {
        ray.active = false;
        ray.pxs = __builtin_nanf("");  // every later g is NaN: the g-first test fails without an active flag
        if (STATS) ++ray.term;
    }
    return term;
}

// Shade candidates 0..m of one stage (sorted front to back) for every lane's ray.
template <bool SH, bool LUT, bool STATS>
__device__ GSRT_INLINE void shade_stage(const Stage* stg, uint32_t m, const float* lut_s, CorRay& ray) {
    if (!STATS) {
        // Phase 1, g of all kGroup candidates at once (independent chains, one LDS wait): g first because lanes
        // that miss mostly fail it, and a candidate no lane passes is skipped with one wave-uniform branch.
        // g <= gcut = max(0, min(kGMax, ln(255 op) + 0.01)) drops only alphas <= 1/255: the result is
        // unchanged. g in [0, gcut] is one unsigned compare of the bit patterns: gcut >= +0 (k_project); g is
        // never -0 (its first term (A/2 dx) dx is +0 or positive and an exact cancellation rounds to +0); a
        // negative g has the sign bit set; a terminated or invalid ray has pxs = NaN, so g is NaN and fails.
        float gv[kGroup];
        bool okg[kGroup];
#pragma unroll
        for (uint32_t c = 0; c < kGroup; ++c) {
            const float4 q2 = reinterpret_cast<const float4*>(&stg->rec[c])[2];  // ppx, ppy, A/2, B
            float4 q3 = reinterpret_cast<const float4*>(&stg->rec[c])[3];        // C/2, gcut, valid, pad
            asm volatile("" : "+v"(q3.w));  // one ds_read_b128 per record (4 LDS-array cycles), not ds_read2_b64 pairs (8)
            const float c2 = q3.x, cut = LUT ? kGMax : q3.y;
            const float dx = ray.pxs - q2.x, dy = ray.pys - q2.y;
            gv[c] = fmaf(c2 * dy, dy, fmaf(q2.w * dx, dy, (q2.z * dx) * dx));
            okg[c] = c < m && __float_as_uint(gv[c]) <= __float_as_uint(cut);  // stale records past m: never
        }
#ifdef GSRT_DIAG
        ray.dg_staged += __ballot(ray.active) ? m : 0u;
#endif
        // Phase 2, front to back over the candidates some lane passed: slab test, exp, alpha, blend
#pragma unroll
        for (uint32_t c = 0; c < kGroup; ++c) {
            if (!__ballot(okg[c])) continue;
            float4 q0 = reinterpret_cast<const float4*>(&stg->rec[c])[0];  // lo or near, depth
            const float4 q1 = reinterpret_cast<const float4*>(&stg->rec[c])[1];  // hi or far, +-opacity
            // q0.w (depth) is unused, but reading all 16 B keeps one ds_read_b128 (4 LDS-array cycles) instead of a
            // ds_read_b96 (8)
            asm volatile("" : "+v"(q0.w));
            // the slab test and exp run for the whole wave; a lane keeps alpha only if it passed both tests. The
            // record's layout (k_project) is wave-uniform: (near, far) when the opacity word is positive
            const float lo[3] = {q0.x, q0.y, q0.z}, hi[3] = {q1.x, q1.y, q1.z};
            const bool ordered = (int)__builtin_amdgcn_readfirstlane(__float_as_uint(q1.w)) >= 0;
            const bool ok = okg[c] & (ordered ? slab_hit_ordered(ray.R, lo, hi) : slab_hit_rel(ray.R, lo, hi));
            // the LUT index must stay in range on every lane (g in [0, kGMax]); exp_neg_nocheck takes any g (a
            // failed lane's value, even NaN, is discarded below)
            const float gs = LUT ? (ok ? gv[c] : 0.0f) : gv[c];
            const float e = LUT ? linear_exp(lut_s, gs) : exp_neg_nocheck(-gs);
            // min(a, 0.99) as v_min: a is never NaN where it is kept (ok: g in [0, gcut], e in (0, 1])
            const float a = __builtin_fminf(fabsf(q1.w) * e, 0.99f);
            const bool contrib = ok && a > kAlphaMin;
            const float alpha = contrib ? a : 0.0f;
#ifdef GSRT_DIAG
            ray.dg_gpass += 1u;
            ray.dg_lanes_g += (uint32_t)__popcll(__ballot(okg[c]));
            ray.dg_contrib += __ballot(alpha > 0.0f) ? 1u : 0u;
            ray.dg_blend += __ballot(alpha > 0.0f && ray.T * (1.0f - alpha) >= 1e-4f) ? 1u : 0u;
            ray.dg_lanes_blend += (uint32_t)__popcll(__ballot(alpha > 0.0f && ray.T * (1.0f - alpha) >= 1e-4f));
#endif
            if (blend_hit<SH, STATS>(ShFromStage{stg, c}, alpha, contrib, ray)) {
#pragma unroll
                for (uint32_t c1 = c + 1; c1 < kGroup; ++c1) okg[c1] = false;  // this lane's ray stopped
            }
        }
        return;
    }
    for (uint32_t c = 0; c < m; ++c) {
        // counting pass: every AABB candidate of every active ray is counted (no g-first skip)
        const float4* r4 = reinterpret_cast<const float4*>(&stg->rec[c]);
        float4 q0 = r4[0], q1 = r4[1], q2 = r4[2], q3 = r4[3];
        asm volatile("" : "+v"(q1.w), "+v"(q2.x), "+v"(q2.y), "+v"(q2.z), "+v"(q2.w), "+v"(q3.x), "+v"(q3.z));
        float alpha = 0.0f;
        if (ray.active) {
            const float lo[3] = {q0.x, q0.y, q0.z}, hi[3] = {q1.x, q1.y, q1.z};  // relative to the origin
            if (slab_hit_rel(ray.R, lo, hi)) {
                ++ray.cand;
                const float dx = ray.pxs - q2.x, dy = ray.pys - q2.y;  // ppx, ppy
                // A/2 = q2.z, B = q2.w, C/2 = q3.x: = 0.5 fma(C dy, dy, fma(2B dx, dy, (A dx) dx)) exactly
                const float g = fmaf(q3.x * dy, dy, fmaf(q2.w * dx, dy, (q2.z * dx) * dx));
                if (g >= 0.0f && g <= kGMax) {
                    const float e = LUT ? linear_exp(lut_s, g) : exp_neg(-g);
                    float a = fabsf(q1.w) * e;  // opacity (negated on a general-layout record, k_project)
                    if (a > 0.99f) a = 0.99f;
                    if (a > kAlphaMin) alpha = a;
                }
            }
        }
        blend_hit<SH, STATS>(ShFromStage{stg, c}, alpha, alpha > 0.0f, ray);
    }
}


// Shade ids[0..count) (sorted front to back) for every lane's ray; returns false once no lane is active.
// Three stage buffers: while stage k is shaded, the DMAs of stages k+1 and k+2 are in flight; wait_stage waits
// for stage k's own DMA only. No DMA stays in flight past a return (the LDS is reused by the next round or by
// the next workgroup).
template <bool SH, bool LUT, bool STATS>
__device__ GSRT_INLINE bool shade_sorted(const uint32_t* ids, uint32_t count, Stage* stA, Stage* stB, Stage* stC,
                             const float* lut_s, CorRay& ray, const SplatRec* recs, const float* sh) {
    const uint32_t lane = lane_id();
    count = __builtin_amdgcn_readfirstlane(count);  // wave-uniform: stage bounds as scalar compares
    if (count == 0) return __ballot(ray.active) != 0;
    auto issue = [&](uint32_t g, Stage* dst) { stage_issue<SH>(ids, count, g, lane, dst, recs, sh); };
    auto shade = [&](Stage* stg, uint32_t g) {
        const uint32_t m = count - g < kGroup ? count - g : kGroup;
        shade_stage<SH, LUT, STATS>(stg, m, lut_s, ray);
    };
    // stages issued after stage g's DMA when it is read: those of g + kGroup and g + 2 kGroup that exist
    auto wait = [count](uint32_t g) {
        wait_stage<SH>((g + kGroup < count ? 1u : 0u) + (g + 2 * kGroup < count ? 1u : 0u));
    };
    issue(0, stA);
    if (kGroup < count) issue(kGroup, stB);
    bool live = true;
    for (uint32_t g0 = 0; g0 < count; g0 += 3 * kGroup) {
        if (g0 + 2 * kGroup < count) issue(g0 + 2 * kGroup, stC);
        wait(g0);
        shade(stA, g0);
        if (!__ballot(ray.active)) { live = false; break; }
        const uint32_t g1 = g0 + kGroup;
        if (g1 >= count) break;
        if (g1 + 2 * kGroup < count) issue(g1 + 2 * kGroup, stA);
        wait(g1);
        shade(stB, g1);
        if (!__ballot(ray.active)) { live = false; break; }
        const uint32_t g2 = g1 + kGroup;
        if (g2 >= count) break;
        if (g2 + 2 * kGroup < count) issue(g2 + 2 * kGroup, stB);
        wait(g2);
        shade(stC, g2);
        if (!__ballot(ray.active)) { live = false; break; }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMAs issued past the last shaded stage
    __syncthreads();
    return live;
}

// Traversal frontier of each super-group (kSG x kSG tile groups): the top of the BVH walked once per
// super-group instead of once per group. Breadth first from the root against the super-group's frustum; a
// node with a leaf child stops (it goes to the frontier as is), the others are replaced by their children that
// meet the frustum, level by level while the frontier fits kFront. Every node a group's rays can reach lies
// below a frontier node (the group's frustum lies inside the super-group's), so groups start from it.
__device__ GSRT_INLINE void frontier_one(const uint32_t g) {
    __shared__ uint32_t cur[2 * kFront], nxt[2 * kFront], fin[2 * kFront];
    const uint32_t lane = lane_id();
    const KArgs& K = kargs();
    if (g >= K.a.sgroups) return;
    uint32_t* out = K.a.frontier + (size_t)g * (kFront + 1);
    const uint32_t gx = g % K.a.sgroups_x, gy = g / K.a.sgroups_x;
    if (K.a.own.active) {  // a super-group spans kSG * fg tile rows: no group of this rank reads a frontier outside
        const uint32_t span = kSG * K.a.fg;
        if ((gy + 1) * span <= K.a.row0 || gy * span >= K.a.row1) return;
    }
    const uint32_t span_x = kSG * K.a.fg * K.a.tw, span_y = kSG * K.a.fg * K.a.th;
    const Frustum F = make_frustum(K.ubo, (float)(gx * span_x) - 0.5f, (float)(gy * span_y) - 0.5f,
                                   (float)((gx + 1) * span_x) + 0.5f, (float)((gy + 1) * span_y) + 0.5f);
    const BvhNode* nodes = K.a.nodes;
    uint32_t ncur = 0, nfin = 0;
    {
        const float rlo[3] = {K.a.root_box[0], K.a.root_box[1], K.a.root_box[2]};
        const float rhi[3] = {K.a.root_box[3], K.a.root_box[4], K.a.root_box[5]};
        if (!box_outside(F, rlo, rhi)) {
            if (lane == 0) cur[0] = K.a.root_ref;
            ncur = 1;
        }
    }
    __syncthreads();
    while (ncur > 0) {
        uint32_t nn = 0, nf = 0;
        for (uint32_t base = 0; base < ncur; base += 64) {
            const uint32_t i = base + lane;
            uint32_t nc = 0, c0 = 0, c1 = 0;
            bool stays = false;
            if (i < ncur) {
                const uint32_t node = cur[i];
                const BvhNode nd = nodes[node];
                if ((nd.l_ref | nd.r_ref) & kLeafBit) {
                    stays = true;
                    c0 = node;
                } else {
                    if (!box_outside(F, nd.l_lo, nd.l_hi)) { c0 = nd.l_ref; ++nc; }
                    if (!box_outside(F, nd.r_lo, nd.r_hi)) { if (nc) c1 = nd.r_ref; else c0 = nd.r_ref; ++nc; }
                }
            }
            const uint64_t bs = __ballot(stays);
            if (stays) fin[nfin + nf + popc_below(bs)] = c0;
            nf += (uint32_t)__popcll(bs);
            const uint64_t b1 = __ballot(nc >= 1), b2 = __ballot(nc >= 2);
            const uint32_t off = popc_below(b1) + popc_below(b2);
            if (nc >= 1) nxt[nn + off] = c0;
            if (nc >= 2) nxt[nn + off + 1] = c1;
            nn += (uint32_t)__popcll(b1) + (uint32_t)__popcll(b2);
        }
        __syncthreads();
        if (nfin + nf + nn > kFront) break;  // the next level does not fit: keep this one
        nfin += nf;
        for (uint32_t i = lane; i < nn; i += 64) cur[i] = nxt[i];
        ncur = nn;
        __syncthreads();
    }
    for (uint32_t i = lane; i < nfin; i += 64) out[1 + i] = fin[i];
    for (uint32_t i = lane; i < ncur; i += 64) out[1 + nfin + i] = cur[i];
    if (lane == 0) out[0] = nfin + ncur;
}

__global__ __launch_bounds__(64) void k_frontier(const KArgs karg) {
    __builtin_amdgcn_s_setprio(kPrepSetprio);
    (void)karg;
    frontier_one(blockIdx.x);
}

// The COR projection's arguments (k_project's, less the camera: the fused kernel takes it from KArgs)
struct ProjArgs {
    uint32_t n;
    const gsrt_gauss_param* params;
    const gsrt_aabb* aabbs;
    SplatRec* recs;
    BvhNode* nodes;
    const uint32_t* gid_slot;
    float4* footprint;
    unsigned long long* counters;
    RankTiles own;
    uint32_t* keyed;
    uint32_t leaf_fp;
    // rank shares: projection block c takes sorted leaves 64 c .. 64 c + 63 (leaf_gid; keyed is then indexed by sorted
    // leaf), whose splats lie close together, so most blocks hold none the band can see
    const uint32_t* leaf_gid;  // nullptr: block c takes gaussian ids 64 c .. 64 c + 63
    const uint32_t* inband;    // rank shares: the slot's in-band bitmap (k_classify), or nullptr
    uint32_t* depth_unsafe;    // the scene's depth-cull guard word (RenderArgs::depth_unsafe)
};
static_assert(sizeof(KArgs) + sizeof(ProjArgs) <= 4096, "kernel argument segment");

// A pipelined COR frame's prep head in one launch: workgroups [0, sgroups) build the super-group frontiers
// (k_frontier), the others project 64 splats each (k_project<COR>). The two are independent, so they share the
// machine as two streams would, but without the cross-stream event between the frontier and the group lists
// (11-14 us per frame in the kernel traces). The frontier's workgroups come first: they are the longer
// latency chains. One-wave workgroups and <= 80 VGPRs, as k_project (they fill slots that retiring render waves free).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void k_prep_cor(const KArgs karg,
                                                                                          const ProjArgs pa) {
    __builtin_amdgcn_s_setprio(kPrepSetprio);
    (void)karg;
    const uint32_t nfb = kargs().a.sgroups;
    if (blockIdx.x < nfb) {
        frontier_one(blockIdx.x);
        return;
    }
    const uint32_t c = blockIdx.x - nfb;
    const uint32_t p = c * 64 + threadIdx.x;  // the bitmap index: gaussian id, or sorted leaf (leaf_gid)
    // the frame's stats words (see k_project)
    if (p < kCounters && p != kErrWord) pa.counters[p] = 0;
    const uint32_t i = pa.leaf_gid ? (p < pa.n ? pa.leaf_gid[p] : pa.n) : p;
    bool k = true;
    if (i < pa.n) {
        const bool prev = pa.keyed ? ((pa.keyed[p >> 5] >> (p & 31u)) & 1u) != 0 : true;
        if (pa.inband && !((pa.inband[i >> 5] >> (i & 31u)) & 1u)) {
            // no tile of the rank's band can see the splat (k_classify ran project_one's own first test, may_own_box):
            // its keys become +inf as project_one's reject path writes them, without its loads, and only when they may
            // still be finite in this slot
            if (prev) {
                if (pa.nodes) put_node_key(pa.nodes, pa.gid_slot, i, 0x7f800000u);
                pa.recs[i].depth = __uint_as_float(0x7f800000u);
            }
            k = false;
        } else {
            k = project_one<GSRT_MODE_COR>(i, pa.n, kargs().ubo, pa.params, pa.aabbs, pa.recs, pa.nodes, pa.gid_slot,
                                           pa.footprint, pa.own, prev, pa.leaf_fp != 0, pa.depth_unsafe);
        }
    }
    if (pa.keyed) {
        const uint64_t m = __ballot(k);
        if ((threadIdx.x & 31u) == 0 && p < pa.n) pa.keyed[p >> 5] = (uint32_t)(m >> (threadIdx.x & 32u));
    }
}

// A rank share's in-band bitmap (1 bit per gaussian id): whether a tile of the band may see the splat, may_own_box of
// its AABB under the frame's camera (project_one's first test, conservative and monotone in the box). The band fit
// (k_fit_chunks<true>) skips the 256-leaf chunks without a set bit, and k_prep_cor rejects the clear splats without
// loading them. One coalesced pass over the AABBs in id order; one-wave workgroups of 4 x 64 splats.
__global__ __launch_bounds__(64) void k_classify(uint32_t n, const gsrt_ubo ubo, const RankTiles own,
                                                 const gsrt_aabb* __restrict__ aabbs, uint32_t* __restrict__ inband) {
    __builtin_amdgcn_s_setprio(kPrepSetprio);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t i = (blockIdx.x * 4 + q) * 64 + threadIdx.x;
        const bool in = i < n && may_own_box(ubo, aabbs[i], own);
        const uint64_t m = __ballot(in);
        if ((threadIdx.x & 31u) == 0 && i < n) inband[i >> 5] = (uint32_t)(m >> (threadIdx.x & 32u));
    }
}

// First traversal round of the COR tiles, one wave per group of FG x FG tiles: one traversal + footprint
// cull + sort for the group (its frustum and footprint rectangle contain those of its tiles), then every
// tile's list is the group's sorted list filtered by the tile's footprint test (order kept), at most kCap
// entries, written to HBM (lists / list_hdr) for k_render_cor. Replaces a traversal and a sort per tile.
// The group list keeps the kGCap nearest; a tile that reaches its end continues after the group's last key.
template <uint32_t FG>
__global__ __launch_bounds__(64) void k_group_list(const KArgs karg) {
    GSRT_WT_START;
    __shared__ uint64_t keys[kGBuf];
    __shared__ uint32_t stack[kGStack];
    __shared__ float4 trect[FG * FG];      // per tile of the group: the samples' rectangle (x0, x1, y0, y1)
    __shared__ uint32_t tslot[FG * FG];    // local (packed) tile index, or kNoGroup when not this rank's
    __builtin_amdgcn_s_setprio(kPrepSetprio);
    (void)karg;
    const uint32_t lane = lane_id();
    const KArgs& K = kargs();
    if (blockIdx.x >= K.a.groups) return;
    const uint32_t g = K.a.group_order ? K.a.group_order[blockIdx.x] : blockIdx.x;
    const uint32_t gx = g % K.a.groups_x, gy = g / K.a.groups_x;
    constexpr uint32_t kT = FG * FG;
    bool mine = false;
    if (lane < kT) {
        const uint32_t tx = gx * FG + lane % FG, ty = gy * FG + lane / FG;
        uint32_t slot = kNoGroup;
        if (tx < K.a.tiles_x && ty >= K.a.row0 && ty < K.a.row1) {  // a tile of this rank's band: its local slot
            slot = band_index(tx, ty, K.a.row0, K.a.row1, K.a.tiles_x);
            mine = true;
        }
        tslot[lane] = slot;
        const float x0 = (float)(tx * K.a.tw), y0 = (float)(ty * K.a.th);
        trect[lane] = make_float4(x0, x0 + (float)K.a.tw, y0, y0 + (float)K.a.th);
    }
    if (!__ballot(mine)) return;
    FrontRegs front;
    if (K.a.frontier) {  // count and entries in one latency; entries past the count are never read from registers
        const uint32_t* fr = K.a.frontier + (size_t)((gy / kSG) * K.a.sgroups_x + gx / kSG) * (kFront + 1);
        front.n = fr[0];
        front.a = fr[1 + lane];
        front.b = 64 + lane < kFront ? fr[65 + lane] : 0u;
    }
    __syncthreads();
#ifdef GSRT_DIAG
    const unsigned long long dg0 = __builtin_amdgcn_s_memtime();
#endif
    const TileRect rect{(float)(gx * FG * K.a.tw) - 0.5f, (float)(gy * FG * K.a.th) - 0.5f,
                        (float)((gx + 1) * FG * K.a.tw) + 0.5f, (float)((gy + 1) * FG * K.a.th) + 0.5f};
    uint32_t restarts = 0;
    // the test knob GSRT_DEBUG_STACK_LIMIT lowers this stack too
    const uint32_t limit = K.a.stack_limit < kStack ? K.a.stack_limit : kGStack;
    const Collected cl = collect_robust<kGCap, kGBuf, KeyCor, kGroupRegSort, true>(rect, 0, false, keys, stack, KeyCor{}, restarts, true,
                                                                    limit, front, true);
    if (cl.restart) {  // the group traversal failed (stack): every tile of the group traverses for itself
        for (uint32_t t = 0; t < kT; ++t) {
            const uint32_t lt = tslot[t];
            if (lt == kNoGroup) continue;
            const float4 r4 = trect[t];
            const TileRect tr{r4.x - kFpInset, r4.z - kFpInset, r4.y + kFpInset, r4.w + kFpInset};  // = tile_rect
            __syncthreads();
            const Collected c1 = collect_robust(tr, 0, false, keys, stack, KeyCor{}, restarts, true, K.a.stack_limit);
            const uint64_t last = c1.count ? keys[c1.count - 1] : 0ull;
            for (uint32_t i = lane; i < c1.count; i += 64) K.a.lists[(size_t)lt * kCap + i] = (uint32_t)keys[i];
            if (lane == 0)
                K.a.list_hdr[lt] = make_uint4(c1.count | (c1.more ? 0x80000000u : 0u), c1.total, (uint32_t)last,
                                              (uint32_t)(last >> 32));
        }
        return;
    }
    // the group list stays in HBM for the tiles' continuation rounds (k_render_cor)
#ifdef GSRT_DIAG
    const unsigned long long dgw = __builtin_amdgcn_s_memtime();
#endif
    {
        uint64_t* gdst = K.a.glist + (size_t)g * kGStride;
        for (uint32_t i = lane; i < cl.count; i += 64) gdst[i] = keys[i];
        if (lane == 0) {
            const uint64_t gl = cl.count ? keys[cl.count - 1] : 0ull;
            K.a.ghdr[g] = make_uint4(cl.count | (cl.more ? 0x80000000u : 0u), 0u, (uint32_t)gl, (uint32_t)(gl >> 32));
        }
    }
    // filter the sorted group list into the tile lists
#ifdef GSRT_DIAG
    const unsigned long long dg1 = __builtin_amdgcn_s_memtime();
#endif
    const float4* fps = K.a.footprint;
    uint32_t cnt = 0;       // lane t < kT: tile t's list length
    bool trunc = false;     // lane t: tile t cut at kCap
    uint32_t last_i = kNoGroup;  // lane t: group-list index of tile t's last kept entry
    uint32_t pos = cl.count;  // lane t: where tile t resumes in the group list (after its last kept entry when cut)
    const uint32_t my_slot = lane < kT ? tslot[lane] : kNoGroup;  // lane t: tile t's packed slot
    uint32_t mine_mask = 0;  // bit t: tile t is this rank's
#pragma unroll
    for (uint32_t t = 0; t < kT; ++t) mine_mask |= (tslot[t] != kNoGroup) ? (1u << t) : 0u;
    mine_mask = __builtin_amdgcn_readfirstlane(mine_mask);
    // software-pipelined: the next chunk's key and footprint (box + ellipse terms) are loaded before this chunk is
    // filtered, so a chunk's loads wait behind the previous chunk's work instead of stalling the wave
    auto fetch = [&](uint32_t i, uint64_t& k, float4& f, float4& a, float4& b) {
        if (i < cl.count) {
            k = keys[i];
            const uint32_t gid = (uint32_t)k;
            const float4* rec = fps + kFpWords * (size_t)gid;
            f = rec[0];
            a = rec[1];
            b = rec[2];
        }
    };
    uint64_t nkey = 0;
    float4 nfp = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ne0 = nfp, ne1 = nfp;
    fetch(lane, nkey, nfp, ne0, ne1);
#ifdef GSRT_DIAG
    unsigned long long dg_test = 0, dg_out = 0;
#endif
    for (uint32_t base = 0; base < cl.count; base += 64) {
#ifdef GSRT_DIAG
        const unsigned long long dgc0 = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t i = base + lane;
        uint32_t m = 0;  // bit t: this candidate's footprint meets tile t
        const uint64_t key = nkey;
        const float4 fp = nfp, e0 = ne0, e1 = ne1;
        if (base + 64 < cl.count) fetch(i + 64, nkey, nfp, ne0, ne1);
        if (i < cl.count) {
            // the tiles whose rectangle the footprint box can meet, then the exact box and ellipse tests on those
            // tiles only. Tile i spans [i, i + 1] in units v = (x - X0) / tw; the box [v0, v1] meets it iff
            // v0 <= i + 1 and v1 >= i, i.e. ceil(v0 - 1) <= i <= floor(v1). floor(v0 - e) and floor(v1 + e),
            // e = 1e-3, bound that range from outside (v's rounding is below 1e-5 for |v| <= 64)
            const float X0 = (float)(gx * FG * K.a.tw), Y0 = (float)(gy * FG * K.a.th);
            const float itw = 1.0f / (float)K.a.tw, ith = 1.0f / (float)K.a.th;
            // (clamped in float first: empty boxes are +-inf, and huge ones must not overflow the conversion)
            auto tidx = [](float v) { return (int)floorf(__builtin_fminf(__builtin_fmaxf(v, -4.0f), 64.0f)); };
            const int tx0 = max(0, tidx((fp.x - X0) * itw - 1e-3f)), tx1 = min((int)FG - 1, tidx((fp.y - X0) * itw + 1e-3f));
            const int ty0 = max(0, tidx((fp.z - Y0) * ith - 1e-3f)), ty1 = min((int)FG - 1, tidx((fp.w - Y0) * ith + 1e-3f));
            uint32_t cand = 0;
            if (tx0 <= tx1 && ty0 <= ty1) {
                const uint32_t row = ((2u << (tx1 - tx0)) - 1u) << tx0;  // bits tx0..tx1
                for (int ty = ty0; ty <= ty1; ++ty) cand |= row << (ty * FG);
            }
            while (cand) {
                const uint32_t t = (uint32_t)__builtin_ctz(cand);
                cand &= cand - 1u;
                const float x0 = X0 + (float)((t % FG) * K.a.tw), y0 = Y0 + (float)((t / FG) * K.a.th);
                const float x1 = x0 + (float)K.a.tw, y1 = y0 + (float)K.a.th;  // = trect[t] (exact integers)
                const bool in = fp.x <= x1 && fp.y >= x0 && fp.z <= y1 && fp.w >= y0 && ell_meets(e0, e1, x0, x1, y0, y1);
                m |= in ? (1u << t) : 0u;
            }
        }
#ifdef GSRT_DIAG
        const unsigned long long dgc1 = __builtin_amdgcn_s_memtime();
        dg_test += dgc1 - dgc0;
#endif
#pragma unroll
        for (uint32_t t = 0; t < kT; ++t) {
            if (!((mine_mask >> t) & 1u)) continue;
            const uint64_t b = __ballot((m >> t) & 1u);
            if (!b) continue;
            const uint32_t lt = __builtin_amdgcn_readlane(my_slot, t);
            const uint32_t c = __builtin_amdgcn_readlane(cnt, t);
            const uint32_t room = kCap - c;
            const uint32_t rank = popc_below(b);
            const bool keep = ((m >> t) & 1u) && rank < room;
            if (keep) K.a.lists[(size_t)lt * kCap + c + rank] = (uint32_t)key;
            const uint32_t n = (uint32_t)__popcll(b);
            const uint32_t took = n < room ? n : room;
            if (took) {
                // lane holding the last kept candidate: the highest set bit of b, or of the kept ones when cut
                const uint64_t kb = n <= room ? b : __ballot(keep);
                const uint32_t hi = 63u - (uint32_t)__builtin_clzll(kb);
                if (lane == t) {
                    last_i = base + hi;
                    if (n > room) pos = base + hi + 1u;
                }
            }
            if (lane == t) {
                if (n > room && !trunc && !took) pos = base;  // cut before this chunk (list already full)
                cnt = c + took;
                trunc = trunc || n > room;
            }
        }
#ifdef GSRT_DIAG
        dg_out += __builtin_amdgcn_s_memtime() - dgc1;
#endif
    }
    const bool gmore = cl.more;
    const uint64_t glast = cl.count ? keys[cl.count - 1] : 0ull;
    const uint64_t last = last_i != kNoGroup ? keys[last_i] : 0ull;  // lane t: tile t's last kept key
    if (lane < kT && my_slot != kNoGroup) {
        // continuation: after the tile's last key when it was cut at kCap, else after the group's last key
        const uint64_t lo = trunc ? last : (gmore ? glast : last);
        K.a.list_hdr[my_slot] = make_uint4(cnt | ((trunc || gmore) ? 0x80000000u : 0u), pos, (uint32_t)lo,
                                               (uint32_t)(lo >> 32));
    }
#ifdef GSRT_DIAG  // [6] group kernel cycles, [7] of which the tile filter, [5] groups whose list overflowed
    if (lane == 0) {
        const unsigned long long dg2 = __builtin_amdgcn_s_memtime();
        atomicAdd(K.a.counters + 6, dg2 - dg0);
        atomicAdd(K.a.counters + 7, dg2 - dg1);
        atomicAdd(K.a.counters + 22, dg_test);  // per-lane tile tests (with the chunk's footprint loads)
        atomicAdd(K.a.counters + 23, dg_out);   // per-tile list output
        atomicAdd(K.a.counters + 24, dg1 - dgw);  // group list to HBM
        if (gmore) atomicAdd(K.a.counters + 5, 1ull);
        atomicMax(K.a.counters + 4, (unsigned long long)cl.count);
        atomicAdd(K.a.counters + 3, (unsigned long long)cl.count);
    }
#endif
    GSRT_WT_END(1, blockIdx.x);
}

// The next segment of an overflowing group list (launched after k_group_list where tiles hold many samples per
// pixel: a 4x4-tile group then spans few pixels and its list often overflows, C5): the next kGCap keys after the first
// segment's last one, once for the group, appended to its list. Its tiles' continuation rounds then read them from
// the group list (k_render_cor) instead of each traversing the BVH after the first segment's end; the candidates
// and their order are the same either way. A separate kernel, so that k_group_list keeps its registers.
template <uint32_t FG>
__global__ __launch_bounds__(64) void k_group_more(const KArgs karg) {
    __shared__ uint64_t keys[kGBuf];
    __shared__ uint32_t stack[kGStack];
    __builtin_amdgcn_s_setprio(kPrepSetprio);
    (void)karg;
    const uint32_t lane = lane_id();
    const KArgs& K = kargs();
    if (blockIdx.x >= K.a.groups) return;
    const uint32_t g = K.a.group_order ? K.a.group_order[blockIdx.x] : blockIdx.x;
    const uint32_t gx = g % K.a.groups_x, gy = g / K.a.groups_x;
    constexpr uint32_t kT = FG * FG;
    bool mine = false;  // (a group without a tile of this rank's band has no list this frame)
    if (lane < kT) {
        const uint32_t tx = gx * FG + lane % FG, ty = gy * FG + lane / FG;
        mine = tx < K.a.tiles_x && ty >= K.a.row0 && ty < K.a.row1;
    }
    if (!__ballot(mine)) return;
    const uint4 gh = K.a.ghdr[g];
    const uint32_t count = gh.x & 0x7fffffffu;
    // (complete; or the group fell back to per-tile traversals; or its list is at its last segment)
    if (!(gh.x >> 31) || count == 0 || count % kGCap != 0 || count >= kGStride) return;
    FrontRegs front;
    if (K.a.frontier) {
        const uint32_t* fr = K.a.frontier + (size_t)((gy / kSG) * K.a.sgroups_x + gx / kSG) * (kFront + 1);
        front.n = fr[0];
        front.a = fr[1 + lane];
        front.b = 64 + lane < kFront ? fr[65 + lane] : 0u;
    }
    const TileRect rect{(float)(gx * FG * K.a.tw) - 0.5f, (float)(gy * FG * K.a.th) - 0.5f,
                        (float)((gx + 1) * FG * K.a.tw) + 0.5f, (float)((gy + 1) * FG * K.a.th) + 0.5f};
    const uint64_t lo = ((uint64_t)gh.w << 32) | gh.z;
    uint32_t restarts = 0;
    const uint32_t limit = K.a.stack_limit < kStack ? K.a.stack_limit : kGStack;
    const Collected cl = collect_robust<kGCap, kGBuf, KeyCor, kGroupRegSort, true>(rect, lo, true, keys, stack,
                                                                                    KeyCor{}, restarts, true, limit,
                                                                                    front, true);
    if (cl.restart) return;  // (the tiles traverse after the first segment, as without this kernel)
    uint64_t* gdst = K.a.glist + (size_t)g * kGStride + count;
    for (uint32_t i = lane; i < cl.count; i += 64) gdst[i] = keys[i];
    if (lane == 0) {
        const uint64_t gl = cl.count ? keys[cl.count - 1] : lo;
        K.a.ghdr[g] = make_uint4((count + cl.count) | (cl.more ? 0x80000000u : 0u), 0u, (uint32_t)gl, (uint32_t)(gl >> 32));
    }
}

// First traversal round of every COR tile as its own kernel: traversal + sort need few registers, so this
// kernel runs at high occupancy and hides the dependent node loads that the shading kernel (occupancy set by
// its SH-3 blend) cannot. The sorted ids go to HBM (1 KiB per tile); k_render_cor picks them up.
__global__ __launch_bounds__(64) void k_collect_cor(const KArgs karg) {
    __shared__ uint64_t keys[2 * kCap];
    __shared__ uint32_t stack[kStack];
    (void)karg;
    const uint32_t lane = lane_id();
    uint32_t lt;
    TileRect rect;
    {
        const KArgs& K = kargs();
        const uint32_t t = blockIdx.x;
        if (t >= K.a.ntiles_local) return;
        lt = xcd_local_tile(t, K.a.ntiles_local);
        uint32_t tx, ty;
        band_tile(lt, K.a.row0, K.a.row1, K.a.tiles_x, tx, ty);
        rect = tile_rect(tx, ty, K.a.tw, K.a.th);
    }
    const KArgs& K = kargs();
    uint32_t* dst = K.a.lists + (size_t)lt * kCap;
    // without group lists (counting pass, a single Gaussian, GSRT_DEBUG_NO_GROUPS): traverse for this tile
    uint32_t restarts = 0;
    const Collected cl = collect_robust(rect, 0, false, keys, stack, KeyCor{}, restarts, K.a.cull2d != 0);
    const uint64_t last = cl.count ? keys[cl.count - 1] : 0ull;  // continuation key of the next round
    for (uint32_t i = lane; i < cl.count; i += 64) dst[i] = (uint32_t)keys[i];
    if (lane == 0)
        K.a.list_hdr[lt] = make_uint4(cl.count | (cl.more ? 0x80000000u : 0u), cl.total, (uint32_t)last, (uint32_t)(last >> 32));
}

template <bool SH, bool LUT, bool STATS>
// waves/SIMD targets (VGPR budget 512 / waves): the three 1-KB stage buffers + ids make 6 KB of LDS per wave, so
// at most 26 waves per CU; 6 per SIMD (80 VGPRs) for both variants. The no-SH kernel asked for 8 before the
// third stage buffer, and the compiler, unable to reach it, left it at 101 VGPRs = 4 waves (C4 -6 %, C5 -12 %).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SH ? (LUT ? 4 : 6) : (LUT ? 5 : 6))))
void k_render_cor(const KArgs karg) {
    // traversal buffers (keys, stack) and shading buffers (ids, two stages) are never live at once
    union CorLds {
        struct { uint64_t keys[kRBuf]; uint32_t stack[kRStack]; } t;
        struct { uint32_t ids[kCap]; uint32_t hdr[4]; } l;  // hdr: the first round's list header (LDS-DMA)
    };
    __shared__ CorLds L;
    __shared__ Stage stA, stB, stC;
    __shared__ float lut_s[LUT ? 512 : 1];
    uint64_t* const keys = L.t.keys;
    uint32_t* const stack = L.t.stack;
    uint32_t* const ids = L.l.ids;
    uint32_t* const lhdr = L.l.hdr;
    const SplatRec* const recs = kargs().a.recs;  // stage DMA sources, read once (kargs() is not hoisted)
    const float* const shp = kargs().a.sh;
    (void)karg;  // read through kargs()
    const uint32_t lane = lane_id();
#ifdef GSRT_DIAG
    const unsigned long long diag_entry = __builtin_amdgcn_s_memtime();
    unsigned long long diag_setup = 0, diag_last = 0;
#endif
    if (LUT) {
        const float* lut = kargs().a.lut;
        for (uint32_t i = lane; i < 512; i += 64) lut_s[i] = lut[i];
        __syncthreads();
    }
    GSRT_WT_START;
    // the tile's cost in the partition's profile (RenderArgs::tile_cost): its wave's wall time in ticks of the 100-MHz
    // real-time counter, from here to the store. Counted work (staged and shaded candidates) left the centre bands of
    // an 8-rank C3 frame 28 % slower than the outer ones at equal counts: time also follows the continuation rounds'
    // traversals, the blending depth and the L2 hit rate of the region
    const uint32_t t_tile0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    // ---- tile and ray setup
    uint32_t lt, x0, y0, tw, th, S, passes;
    {
        const KArgs& K = kargs();
        const uint32_t t = blockIdx.x;
        if (t >= K.a.ntiles_local) return;
        lt = xcd_local_tile_perm(t, K.a.ntiles_local, K.a.run_order);  // packed slot of this tile
        uint32_t tx, ty;
        band_tile(lt, K.a.row0, K.a.row1, K.a.tiles_x, tx, ty);
        tw = K.a.tw; th = K.a.th; S = K.a.s_lanes; passes = K.a.passes;
        x0 = tx * tw; y0 = ty * th;
    }
    // the first round's list (k_group_list / k_collect_cor wrote it): its header and first 128 ids go straight
    // into LDS (LDS-DMA: no VGPRs held across the setup), issued here so that their latency hides behind the
    // ray setup (the tile's list slot holds kCap entries, so the loads stay inside it whatever the count)
    lt = __builtin_amdgcn_readfirstlane(lt);
    bool prefetched = false;
    if (kargs().a.prelisted) {
        list_issue(lt, lane, ids, lhdr);
        prefetched = true;
    }
    // tw, th and S are powers of two (make_plan): shifts instead of divisions. The lane's pixel, its validity
    // and the tile's rectangle are recomputed where they are used (ray setup, rare continuation rounds, the
    // store) from uniform values and a laundered lane id, so that none of them lives (spilled) across the loop.
    x0 = __builtin_amdgcn_readfirstlane(x0);
    y0 = __builtin_amdgcn_readfirstlane(y0);
    const uint32_t lgS = (uint32_t)__builtin_ctz(S), lgtw = (uint32_t)__builtin_ctz(tw), lgth = (uint32_t)__builtin_ctz(th);
    auto pixel = [&](uint32_t& pit, uint32_t& si, uint32_t& qx, uint32_t& qy, bool& ok) {
        uint32_t l = lane_id();
        asm volatile("" : "+v"(l));  // a fresh lane id: no live range across the shading loop
        pit = l >> lgS;
        si = l & (S - 1u);
        qx = x0 + (pit & (tw - 1u));
        qy = y0 + (pit >> lgtw);
        ok = qx < kargs().a.width && qy < kargs().a.height;
    };
    auto tile_rect_here = [&]() {
        uint32_t tx = x0 >> lgtw, ty = y0 >> lgth;
        asm volatile("" : "+s"(tx), "+s"(ty));  // recomputed at the (rare) use, not hoisted and spilled
        return tile_rect(tx, ty, tw, th);
    };
    uint32_t pix_in_tile, s_in, px, py;
    bool valid;
    pixel(pix_in_tile, s_in, px, py, valid);
    // the pixel's sum over its samples: with one pass (spp <= 64) the pass's own values; with several passes
    // (spp > 64: one pixel per lane) the framebuffer entry holds the running sum between passes, so that no
    // accumulator lives (spilled) across the shading loop. The sums are formed in the same order either way.
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t st_cand = 0, st_blend = 0, st_term = 0, st_rounds = 0, restarts = 0, maxc = 0;
#ifdef GSRT_DIAG  // diagnostic build only: per-wave cycle split between traversal+sort and shading
    unsigned long long diag_collect = 0, diag_shade = 0;
#endif
    for (uint32_t pass = 0; pass < passes; ++pass) {
        CorRay ray;
        pixel(pix_in_tile, s_in, px, py, valid);  // recomputed per pass (see pixel)
        {
            const KArgs& K = kargs();
            // sample sidx takes draws 2*sidx, 2*sidx+1 of the pixel LCG seeded with Camera.RandomSeed
            // (RayTracing.rgen:27,39: the same sequence for every pixel)
            const uint32_t sidx = pass * S + s_in;
            uint32_t seed = K.ubo.random_seed;
            for (uint32_t q = 0; q < sidx; ++q) { random_float(&seed); random_float(&seed); }
            const float jx = random_float(&seed);
            const float jy = random_float(&seed);
            ray.pxs = (float)px + jx;
            ray.pys = (float)py + jy;
            float o[3], d[3];
            gen_ray(K.ubo, ray.pxs, ray.pys, o, d);
            ray.R = make_obj_ray(d);
            if (SH) sh_basis(d, ray.bs);
        }
        ray.T = 1.0f;
        ray.C[0] = ray.C[1] = ray.C[2] = 0.0f;
        ray.active = valid;
        if (!valid) ray.pxs = __builtin_nanf("");  // see blend_hit
        ray.cand = ray.blended = ray.term = 0;
#ifdef GSRT_DIAG
        ray.dg_staged = ray.dg_gpass = ray.dg_contrib = ray.dg_blend = ray.dg_lanes_g = ray.dg_lanes_blend = 0;
#endif
        uint64_t lo = 0;
        bool has_lo = false;
        uint32_t gpos = 0;  // with group lists: where this tile resumes in its group's sorted list
        for (;;) {
#ifdef GSRT_DIAG
            const unsigned long long d0 = __builtin_amdgcn_s_memtime();
            if (!has_lo) diag_setup += d0 - (pass == 0 ? diag_entry : diag_last);
#endif
            Collected cl;
            bool listed = false;
            {
                const KArgs& K = kargs();
                if (K.a.prelisted && !has_lo) {  // first round: the list k_group_list / k_collect_cor wrote
                    if (!prefetched) list_issue(lt, lane_here(), ids, lhdr);  // later passes: ids[] was reused
                    prefetched = false;
                    __syncthreads();  // vmcnt(0): header and ids[0..128) landed
                    const uint4 h = make_uint4(lhdr[0], lhdr[1], lhdr[2], lhdr[3]);
                    const uint32_t* src = K.a.lists + (size_t)lt * kCap;
                    cl.count = h.x & 0x7fffffffu;
                    cl.more = (h.x >> 31) != 0;
                    for (uint32_t i = 128u + lane_here(); i < cl.count; i += 64) ids[i] = src[i];
                    cl.total = cl.count;
                    cl.restart = false;
                    lo = ((uint64_t)h.w << 32) | h.z;
                    gpos = h.y;
                    listed = true;
                    __syncthreads();
                } else if (K.a.use_groups) {
                    // continuation inside the group list: the next entries after gpos that meet this tile's
                    // footprint test, in order; lo = the last entry considered
                    const uint32_t g = (y0 / th / K.a.fg) * K.a.groups_x + (x0 / tw / K.a.fg);
                    const uint4 gh = K.a.ghdr[g];
                    const uint32_t gcount = gh.x & 0x7fffffffu;
                    if (gpos < gcount) {
                        const uint64_t* gl = K.a.glist + (size_t)g * kGStride;
                        const float4* fps = K.a.footprint;
                        const TileRect rect_c = tile_rect_here();
                        uint32_t out = 0;
                        while (gpos < gcount && out < kCap) {
                            const uint32_t i = gpos + lane_here();
                            bool keep = false;
                            uint64_t key = 0;
                            if (i < gcount) {
                                key = gl[i];
                                keep = fp_meets(fps, (uint32_t)key, rect_c);
                            }
                            const uint64_t b = __ballot(keep);
                            const uint32_t rank = popc_below(b), n = (uint32_t)__popcll(b), room = kCap - out;
                            if (keep && rank < room) ids[out + rank] = (uint32_t)key;
                            if (n > room) {  // cut: resume after the last entry taken
                                const uint64_t kb = __ballot(keep && rank < room);
                                gpos += (uint32_t)(63 - __builtin_clzll(kb)) + 1u;
                                out = kCap;
                            } else {
                                gpos = gpos + 64u < gcount ? gpos + 64u : gcount;
                                out += n;
                            }
                        }
                        cl.count = out;
                        cl.total = out;
                        cl.restart = false;
                        cl.more = gpos < gcount || (gh.x >> 31) != 0;
                        lo = gl[gpos - 1];  // every group entry up to here was considered for this tile
                        listed = true;
                        __syncthreads();
                    }
                }
            }
            if (!listed) {  // traverse for the keys after lo (no group list, or past the end of an overflowing one)
                const uint32_t lim = kargs().a.stack_limit < kRStack ? kargs().a.stack_limit : kRStack;
                cl = collect_robust<kRCap, kRBuf>(tile_rect_here(), lo, has_lo, keys, stack, KeyCorRec{}, restarts,
                                                  !STATS && kargs().a.cull2d, lim, FrontRegs{}, !STATS);
                lo = cl.count ? keys[cl.count - 1] : lo;
                // narrow the sorted keys to ids in place (ids[i] overlays keys[i/2]: already read, in order)
                const uint32_t ln = lane_here();
                for (uint32_t base = 0; base < cl.count; base += 64) {
                    const uint32_t i = base + ln;
                    const uint32_t v = i < cl.count ? (uint32_t)keys[i] : 0u;
                    asm volatile("" ::: "memory");
                    if (i < cl.count) ids[i] = v;
                    asm volatile("" ::: "memory");
                }
                __syncthreads();
            }
#ifdef GSRT_DIAG
            const unsigned long long d1 = __builtin_amdgcn_s_memtime();
            diag_collect += d1 - d0;
#endif
            ++st_rounds;
            if (cl.total > maxc) maxc = cl.total;
            const bool live = shade_sorted<SH, LUT, STATS>(ids, cl.count, &stA, &stB, &stC, lut_s, ray, recs, shp);
#ifdef GSRT_DIAG
            diag_last = __builtin_amdgcn_s_memtime();
            diag_shade += diag_last - d1;
#endif
            if (!cl.more || !live) break;
            has_lo = true;  // lo = the last (largest) key of this round
            __syncthreads();
        }
        acc[0] = ray.C[0]; acc[1] = ray.C[1]; acc[2] = ray.C[2]; acc[3] = 1.0f - ray.T;  // = 0 + x exactly (x >= +0)
        if (passes > 1) {  // then S == 1 (make_plan): the lane's pixel accumulates its passes in order
            pixel(pix_in_tile, s_in, px, py, valid);
            if (valid) {
                const KArgs& K = kargs();
                float4* o = (K.a.dump8 ? K.a.accum : reinterpret_cast<float4*>(K.a.out)) +
                            (K.a.packed ? (size_t)lt * (tw * th) + pix_in_tile : (size_t)py * K.a.width + px);
                if (pass > 0) {
                    const float4 prev = *o;
                    acc[0] = prev.x + acc[0]; acc[1] = prev.y + acc[1]; acc[2] = prev.z + acc[2]; acc[3] = prev.w + acc[3];
                }
                if (pass + 1 < passes) *o = make_float4(acc[0], acc[1], acc[2], acc[3]);
            }
        }
        st_cand += ray.cand; st_blend += ray.blended; st_term += ray.term;
#ifdef GSRT_DIAG
        if (!STATS && lane == 0) {
            unsigned long long* dc = kargs().a.counters + 16;
            atomicAdd(dc + 0, (unsigned long long)ray.dg_staged);
            atomicAdd(dc + 1, (unsigned long long)ray.dg_gpass);
            atomicAdd(dc + 2, (unsigned long long)ray.dg_contrib);
            atomicAdd(dc + 3, (unsigned long long)ray.dg_blend);
            atomicAdd(dc + 4, (unsigned long long)ray.dg_lanes_g);
            atomicAdd(dc + 5, (unsigned long long)ray.dg_lanes_blend);

        }
#endif
    }
    // pairwise reduction over the S in-wave samples of a pixel (the oracle sums in the same tree); partners 1 and
    // 2 lanes away by DPP quad permutes (no LDS round trip), farther ones by shuffles
    if (S > 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[q] = acc[q] + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[q]), 0xB1, 0xF, 0xF, false));
    }
    if (S > 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[q] = acc[q] + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[q]), 0x4E, 0xF, 0xF, false));
    }
    for (uint32_t off = 4; off < S; off <<= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = acc[q] + __shfl_xor(acc[q], (int)off);
    }
    for (uint32_t off = 1; STATS && off < S; off <<= 1) {
        st_cand += __shfl_xor(st_cand, (int)off);
        st_blend += __shfl_xor(st_blend, (int)off);
        st_term += __shfl_xor(st_term, (int)off);
    }
    const KArgs& K = kargs();
    const uint32_t ns = S * passes;
    const float nsamp = (float)ns;
    pixel(pix_in_tile, s_in, px, py, valid);
    if (valid && s_in == 0) {
        float4 v;
        if ((ns & (ns - 1)) == 0) {  // x / 2^k == x * 2^-k exactly
            const float r = 1.0f / nsamp;
            v = make_float4(acc[0] * r, acc[1] * r, acc[2] * r, acc[3] * r);
        } else {
            v = make_float4(acc[0] / nsamp, acc[1] / nsamp, acc[2] / nsamp, acc[3] / nsamp);
        }
        const size_t idx = K.a.packed ? (size_t)lt * (tw * th) + pix_in_tile : (size_t)py * K.a.width + px;
        if (K.a.dump8) {  // the integers the frame dump prints (Dump8), exact values of the rest in the escape list
            const uint32_t code = dump8_code(v);
            reinterpret_cast<uint32_t*>(K.a.out)[idx] = code;
            if (code & kDump8Escape) {
                const uint32_t e = atomicAdd(&K.a.esc[0].x, 1u);
                if (e < K.a.esc_cap)
                    K.a.esc[1 + e] = make_uint4((uint32_t)idx, __float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z));
            }
        } else {
            reinterpret_cast<float4*>(K.a.out)[idx] = v;
        }
        if (STATS && K.a.ray_stats)
            reinterpret_cast<uint4*>(K.a.ray_stats)[(size_t)py * K.a.width + px] = make_uint4(st_cand, st_blend, st_rounds, st_term);
    }
#ifdef GSRT_DIAG
    if (lane == 0) {
        atomicAdd(K.a.counters + 9, diag_collect);
        atomicAdd(K.a.counters + 10, diag_shade);
        const unsigned long long dend = __builtin_amdgcn_s_memtime();
        atomicAdd(K.a.counters + 11, dend - diag_entry);
        atomicAdd(K.a.counters + 1, diag_setup);      // entry (or a pass's end) to the first round: tile + ray setup
        atomicAdd(K.a.counters + 2, dend - diag_last);  // last round's end to the end: reduction + store
    }
#endif
    // the partition's cost profile: one store per tile (device-scope atomics on a few row words serialise at the
    // memory side and slowed the frame by several percent)
    if (K.a.tile_cost && lane == 0) K.a.tile_cost[lt] = (uint32_t)__builtin_amdgcn_s_memrealtime() - t_tile0;
    if (STATS) {
        const uint32_t lead = (valid && s_in == 0) ? 1u : 0u;
        add_counters(wave_sum(valid ? 1u : 0u) * passes, wave_sum(lead ? st_cand : 0u), wave_sum(lead ? st_blend : 0u),
                     wave_sum(lead ? st_term : 0u), st_rounds, restarts, maxc);
    }
    GSRT_WT_END(0, lt);
}

// ----------------------------------------------------------------------------------------- REF

template <bool STATS>
__global__ __launch_bounds__(64) void k_render_ref(const KArgs karg) {
    __shared__ uint64_t keys[2 * kCap];
    __shared__ uint32_t stack[kStack];
    __shared__ float lut_s[512];
    (void)karg;
    const uint32_t lane = lane_id();
    {
        const float* lut = kargs().a.lut;
        for (uint32_t i = lane; i < 512; i += 64) lut_s[i] = lut[i];
    }
    __syncthreads();
    uint32_t lt, x0, y0, samples, bounces;
    {
        const KArgs& K = kargs();
        const uint32_t t = blockIdx.x;
        if (t >= K.a.ntiles_local) return;
        lt = xcd_local_tile(t, K.a.ntiles_local);
        uint32_t tx, ty;
        band_tile(lt, K.a.row0, K.a.row1, K.a.tiles_x, tx, ty);
        x0 = tx * 8; y0 = ty * 8;
        samples = K.a.samples; bounces = K.a.bounces;
    }
    const uint32_t px = x0 + (lane & 7u), py = y0 + (lane >> 3);
    bool valid;
    float o[3];
    ObjRay R;
    float tri = kTMax;  // min_thit after the triangles (vulkan_ray_tracing.cc:534, 929-931): kTMax = no triangle hit
    {
        const KArgs& K = kargs();
        valid = px < K.a.width && py < K.a.height;
        float d[3];
        gen_ray(K.ubo, (float)px, (float)py, o, d);  // rgen:39-43 at the integer launch id
        R = make_obj_ray(d);
        if (K.a.tri_t && valid) tri = K.a.tri_t[(size_t)py * K.a.width + px];
    }
    const bool tri_hit = tri < kTMax;  // traversal_data.hit_geometry after traceRay (:1094-1096)
    // BLAS boxes entered at or beyond min_thit are culled (:806-807: thit >= min_thit * worldToObject_tMultiplier);
    // with no triangle hit min_thit = Tmax, so only an entry at exactly tmax is dropped
    const float tcut = tri * R.norm;
    const TileRect rect{(float)x0 - 0.5f, (float)y0 - 0.5f, (float)(x0 + 7) + 0.5f, (float)(y0 + 7) + 0.5f};
    uint32_t restarts = 0, st_cand = 0, st_rounds = 0;
    const Collected first = collect_robust(rect, 0, false, keys, stack, KeyRef{}, restarts);
    const bool cached = first.total <= kCap;
    // per-ray state: RayInfo + payload Trans + NextK (Scene.cpp:38-45)
    float Depth = 0.0f, Trans = 1.0f;
    float kd[8], ka[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { kd[j] = kKEmpty; ka[j] = -1.0f; }
    int gnum = 0;
    for (uint32_t s = 0; s < samples; ++s) {
        bool alive = valid;
        for (uint32_t b = 0; b <= bounces; ++b) {
            if (!__ballot(alive)) break;
            // report_ray_intersection_impl (instructions.cc:7036-7050): after a triangle hit, a Gaussian report is
            // accepted only below world_min_thit = the triangle's t
            bool reported = tri_hit, gauss_rep = false;
            float closest = tri;
            if (alive) {
                ++st_rounds;
                gnum = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) kd[j] = kKEmpty;
            }
            uint64_t lo = 0;
            bool has_lo = false;
            for (;;) {  // chunks of kCap candidates in id order (one chunk unless the tile overflowed)
                Collected cl = first;
                if (!cached) cl = collect_robust(rect, lo, has_lo, keys, stack, KeyRef{}, restarts);
                const SplatRec* recs = kargs().a.recs;
                for (uint32_t c = 0; c < cl.count; ++c) {
                    const uint32_t gid = uni((uint32_t)keys[c]);
                    const SplatRec* __restrict__ r = recs + gid;
                    if (!alive) continue;
                    const float rlo[3] = {r->lo[0], r->lo[1], r->lo[2]};
                    const float rhi[3] = {r->hi[0], r->hi[1], r->hi[2]};
                    if (!slab_hit_rel_cut(R, rlo, rhi, tcut)) continue;
                    if (st_rounds == 1) ++st_cand;
                    const float depth = r->depth;
                    if (depth <= Depth) continue;  // rint:69-71
                    const float dx = (float)px - r->ppx, dy = (float)py - r->ppy;
                    const float g = 0.5f * (((r->a * dx) * dx + ((2.0f * r->b) * dx) * dy) + (r->c * dy) * dy);
                    if (g < 0.0f || g > kGMax) continue;  // rint:102
                    if (g != g) continue;                 // NaN never passes alpha > 1/255
                    const float alpha = r->opacity * linear_exp(lut_s, g);
                    if (alpha > kAlphaMin) {
                        float nd = depth, na = alpha;  // InsertNewSplat, rint:35-43
                        bool ins = false;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (kd[j] > nd) {
                                const float td = kd[j], ta = ka[j];
                                kd[j] = nd; ka[j] = na;
                                nd = td; na = ta;
                                ins = true;
                            }
                        }
                        if (ins) gnum += 1;
                        // report_ray_intersection_impl (instructions.cc:7040-7046)
                        if (0.001f <= depth && (reported ? depth < closest : depth <= kTMax)) {
                            reported = gauss_rep = true;
                            closest = depth;
                        }
                    }
                }
                if (cached || cl.total <= kCap) break;
                lo = keys[kCap - 1];
                has_lo = true;
                __syncthreads();
            }
            if (alive) {
                if (gauss_rep) {  // rchit:15-33, GaussNum clamped to 8
                    const int m = gnum < 8 ? gnum : 8;
                    float ct = Trans;
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < m) ct *= (1.0f - ka[j]);
                    Trans = ct;
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j == m - 1) Depth = kd[j];
                } else if (tri_hit) {
                    Trans = 0.0f;  // the triangle's closest hit: RayTracing.rchit, Scatter() returns RayPayload(0, ...)
                }
                if (gnum == 0) alive = false;  // rgen:64-68
            }
        }
    }
    const KArgs& K = kargs();
    if (valid) {
        const size_t pix = (size_t)py * K.a.width + px;
        reinterpret_cast<float4*>(K.a.out)[K.a.packed ? (size_t)lt * 64 + lane : pix] =
            make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // rgen:33,75: pixelColor is never written
        if (K.a.rs) {
            gsrt_raystate st;
            st.trans = Trans;
            st.depth = Depth;
            st.gauss_num = gnum < 8 ? gnum : 8;
            st.gauss_num_raw = gnum;
#pragma unroll
            for (int j = 0; j < 8; ++j) { st.k[j][0] = kd[j]; st.k[j][1] = ka[j]; }
            K.a.rs[pix] = st;
        }
        if (STATS && K.a.ray_stats) reinterpret_cast<uint4*>(K.a.ray_stats)[pix] = make_uint4(st_cand, 0u, st_rounds, 0u);
    }
    if (STATS) add_counters(wave_sum(valid ? 1u : 0u) * samples, wave_sum(valid ? st_cand : 0u), 0ull, 0ull,
                            uni(st_rounds), restarts, first.total);
}

// VS-style traversal statistics of a REF frame (GSRT_FLAG_STATS; gsrt_vs_stats, vulkan-sim gpu-sim.cc:1510-1518):
// after k_render_ref, one lane per pixel walks the LBVH depth first as VulkanRayTracing::traceRay walks its BVH
// (vulkan_ray_tracing.cc:560-1010: every visited internal node and every reached leaf counts, a child is entered
// when the object ray's slab test passes it and, past a triangle hit, its entry lies below min_thit). The node
// count is the LBVH's, not Embree's: comparable in kind, not in value. Per ray: ray_stats.w = nodes of one
// traversal, ray_stats.y = traversals that hit a triangle (rt_num_hits; every round re-traverses, rgen:58-62);
// counters [24] nodes summed over every round's traversal, [25] the most nodes of one traversal, [26] traversals
// with a triangle hit, [27] the deepest level reached (rt_max_tree_depth), [28] lanes whose walk overflowed,
// [29] traversals (rounds summed over the rays: rt_n_total_rays).
constexpr uint32_t kStatStack = 64;
__global__ __launch_bounds__(64) void k_ref_node_stats(const KArgs karg) {
    __shared__ uint32_t stack[kStatStack][64];
    __shared__ uint8_t level[kStatStack][64];
    (void)karg;
    const KArgs& K = kargs();
    const uint32_t lane = threadIdx.x, tiles_x = (K.a.width + 7) / 8;
    const uint32_t px = (blockIdx.x % tiles_x) * 8 + (lane & 7u), py = (blockIdx.x / tiles_x) * 8 + (lane >> 3);
    const bool valid = px < K.a.width && py < K.a.height;
    uint32_t nodes = 0, depth = 0, hits = 0, rounds = 0, over = 0;
    if (valid) {
        float o[3], d[3];
        gen_ray(K.ubo, (float)px, (float)py, o, d);
        const ObjRay R = make_obj_ray(d);
        const size_t pix = (size_t)py * K.a.width + px;
        const float tri = K.a.tri_t ? K.a.tri_t[pix] : kTMax;
        const float tcut = tri * R.norm;
        uint4 rs = reinterpret_cast<uint4*>(K.a.ray_stats)[pix];
        rounds = rs.z;
        auto enter = [&](const float lo[3], const float hi[3]) {
            float l0 = (lo[0] - o[0]) * R.idir[0], h0 = (hi[0] - o[0]) * R.idir[0];
            float l1 = (lo[1] - o[1]) * R.idir[1], h1 = (hi[1] - o[1]) * R.idir[1];
            float l2 = (lo[2] - o[2]) * R.idir[2], h2 = (hi[2] - o[2]) * R.idir[2];
            float t = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(l0, h0), R.tmin),
                                      __builtin_fmaxf(__builtin_fminf(l1, h1), __builtin_fminf(l2, h2)));
            float u = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(l0, h0), R.tmax),
                                      __builtin_fminf(__builtin_fmaxf(l1, h1), __builtin_fmaxf(l2, h2)));
            return t <= u && t < tcut;
        };
        if (K.a.n == 1) {
            nodes = 1;  // the root is the only leaf
            depth = 1;
        } else if (K.a.n > 1) {
            uint32_t sp = 0;
            stack[sp][lane] = K.a.root_ref;
            level[sp++][lane] = 1;
            while (sp) {
                --sp;
                const uint32_t ref = stack[sp][lane], lv = level[sp][lane];
                ++nodes;  // an internal node visited
                depth = depth > lv ? depth : lv;
                const BvhNode& nd = K.a.nodes[ref];
                const uint32_t refs[2] = {nd.l_ref, nd.r_ref};
                const float* los[2] = {nd.l_lo, nd.r_lo};
                const float* his[2] = {nd.l_hi, nd.r_hi};
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (!enter(los[c], his[c])) continue;
                    if (refs[c] & kLeafBit) {
                        ++nodes;  // a leaf reached (a candidate)
                        depth = depth > lv + 1 ? depth : lv + 1;
                    } else if (sp < kStatStack) {
                        stack[sp][lane] = refs[c];
                        level[sp++][lane] = (uint8_t)(lv + 1 < 255 ? lv + 1 : 255);
                    } else {
                        over = 1;
                    }
                }
            }
        }
        hits = tri < kTMax ? rounds : 0u;
        rs.y = hits;
        rs.w = nodes;
        reinterpret_cast<uint4*>(K.a.ray_stats)[pix] = rs;
    }
    const unsigned long long tot = wave_sum(valid ? nodes * rounds : 0u), th = wave_sum(valid ? hits : 0u);
    const unsigned long long nr = wave_sum(valid ? rounds : 0u);
    uint32_t mx = nodes, md = depth;
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
        md = max(md, (uint32_t)__shfl_xor((int)md, off));
    }
    const bool ov = __ballot(over != 0) != 0;
    if (lane == 0) {
        unsigned long long* c = K.a.counters;
        atomicAdd(c + 24, tot);
        atomicMax(c + 25, (unsigned long long)mx);
        atomicAdd(c + 26, th);
        atomicMax(c + 27, (unsigned long long)md);
        if (ov) atomicAdd(c + 28, 1ull);
        atomicAdd(c + 29, nr);
    }
}

// ----------------------------------------------------------------------------------------- host side

uint32_t max_local_tiles(const RenderPlan& p) {  // the packed stride of the gather: the largest share
    uint32_t m = 0;
    for (uint32_t r = 0; r < p.nranks; ++r) {
        const uint32_t n = p.tiles_x * (p.bands.row[r + 1] - p.bands.row[r]);
        m = n > m ? n : m;
    }
    return m;
}

// Rank 0 also lands the other N-1 blocks and unpacks the whole frame, a cost that grows with the framebuffer bytes
// (N - 1 blocks in, every pixel out) against a share's shading work (~ rays / N). Measured with the loopback stand-in
// (profiles/r04/): the 8-rank root's extra time is 0.2 of a share at C3 (4 spp) and 0.7 at C4 (1 spp), i.e. about
// 0.09 (N - 1) / spp of the root's frame; so rank 0 takes w0 = 1 - 0.09 (N - 1) / spp of a share (>= 1/4). A pure
// function of N and spp: every rank computes the same weight (no per-rank input reaches the partition).
float root_weight(uint32_t nranks, uint32_t spp, uint32_t mode) {
    if (nranks <= 1) return 1.0f;
    // the receive + unpack cost, in shares per (N - 1) / spp: measured for each exchange format (RGBA32F 16 B per
    // pixel, dump codes 4 B: not a quarter of it, since the root's receive and unpack are not bound by bytes alone;
    // the 8-rank C3 and C4 roots put it at 0.067-0.073)
    const float per_px = (mode & GSRT_FLAG_OUT_DUMP8) ? 0.07f : 0.09f;
    const float w0 = 1.0f - per_px * (float)(nranks - 1) / (float)(spp ? spp : 1);
    return w0 < 0.25f ? 0.25f : (w0 > 1.0f ? 1.0f : w0);
}

static void row_prefix(uint32_t tiles_y, const uint32_t* row_cost, std::vector<uint64_t>& P) {
    P.assign(tiles_y + 1, 0);
    for (uint32_t i = 0; i < tiles_y; ++i) P[i + 1] = P[i] + (row_cost ? (uint64_t)row_cost[i] : 1u);
}

void balance_bands(uint32_t tiles_y, uint32_t nranks, const uint32_t* row_cost, float root_w, uint32_t* out) {
    const uint32_t N = nranks ? nranks : 1;
    std::vector<uint64_t> P;
    row_prefix(tiles_y, row_cost, P);
    const double wtot = (double)root_w + (double)(N - 1);
    const uint32_t minrow = tiles_y >= N ? 1u : 0u;  // every band non-empty when there are enough rows
    out[0] = 0;
    out[N] = tiles_y;
    double wsum = 0.0;
    for (uint32_t r = 1; r < N; ++r) {
        wsum += r == 1 ? (double)root_w : 1.0;
        // the cumulative target of bands 0..r-1, met by the nearest row boundary the remaining bands leave room for
        const double target = (double)P[tiles_y] * wsum / wtot;
        const uint32_t lo = out[r - 1] + minrow, hi = tiles_y - (N - r) * minrow;
        uint32_t i = (uint32_t)(std::lower_bound(P.begin() + lo, P.begin() + hi + 1, (uint64_t)std::ceil(target)) - P.begin());
        if (i > hi) i = hi;
        if (i > lo && (double)P[i] - target > target - (double)P[i - 1]) --i;
        out[r] = i;
    }
}

double band_peak(uint32_t nranks, const uint32_t* bands, const uint32_t* row_cost, float root_w) {
    std::vector<uint64_t> P;
    row_prefix(bands[nranks], row_cost, P);
    double peak = 0.0;
    for (uint32_t r = 0; r < nranks; ++r) {
        const double c = (double)(P[bands[r + 1]] - P[bands[r]]) / (r == 0 ? (double)root_w : 1.0);
        peak = c > peak ? c : peak;
    }
    return peak;
}

RenderPlan make_plan(const gsrt_ubo& ubo, uint32_t mode, uint32_t k, uint32_t rank, uint32_t nranks,
                     const uint32_t* bands) {
    RenderPlan p;
    p.mode = mode;
    p.cap = kCap;
    (void)k;
    p.nranks = nranks ? (nranks < kMaxRanks ? nranks : kMaxRanks) : 1;
    p.rank = rank < p.nranks ? rank : 0;
    const uint32_t S = ubo.samples ? ubo.samples : 1;
    if ((mode & 0xffu) == GSRT_MODE_REF) {
        p.tw = p.th = 8; p.s_lanes = 1; p.passes = 1;
    } else if (S <= 64 && (S & (S - 1)) == 0) {
        uint32_t px = 64 / S, lg = 0;
        while ((1u << lg) < px) ++lg;
        p.tw = 1u << ((lg + 1) / 2);
        p.th = 1u << (lg / 2);
        p.s_lanes = S; p.passes = 1;
    } else {
        p.tw = p.th = 8; p.s_lanes = 1; p.passes = S;
    }
    p.tiles_x = (ubo.width + p.tw - 1) / p.tw;
    p.tiles_y = (ubo.height + p.th - 1) / p.th;
    // the partition: the given bands (a cost-balanced partition, gsrt_comm.cpp), else rows split evenly by weight
    p.bands.n = p.nranks;
    if (bands) {
        for (uint32_t r = 0; r <= p.nranks; ++r) p.bands.row[r] = bands[r];
    } else {
        const float w0 = (mode & 0xffu) == GSRT_MODE_COR ? root_weight(p.nranks, S, mode) : 1.0f;
        balance_bands(p.tiles_y, p.nranks, nullptr, w0, p.bands.row);
    }
    // tile groups: 4x4 tiles, or 2x2 when a rank would get fewer than 1500 groups of 4x4. A rank's group lists
    // are latency chains (traversal, sort, filter) beside the previous frame's render; with few groups there are
    // too few of them to fill the GPU, and smaller groups shorten each chain. Measured: C3 (8160), C4 (8160) and
    // C5 (32400) are 6-10 % faster with 4x4; the 8-rank C3 and C4 shares (1020 groups of 4x4) 15-20 % faster
    // with 2x2; C2 and the 4-rank C3 share (2040) 5-9 % faster with 4x4 since slot streams overlap their frames
    // (before them C2 was 9 % faster with 2x2; profiles/r02c/ab_group_tiles_slot.txt). The test switch
    // GSRT_DEBUG_GROUP_TILES=2|4 overrides.
    {
        const uint32_t g4 = ((p.tiles_x + kFG - 1) / kFG) * ((p.tiles_y + kFG - 1) / kFG);
        p.fg = g4 < 1500u * p.nranks ? 2u : kFG;
    }
    if (const char* e = std::getenv("GSRT_DEBUG_GROUP_TILES")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v == 2 || v == (long)kFG) p.fg = (uint32_t)v;
    }
    return p;
}

// GSRT_DEBUG_NO_FRONTIER=1: groups traverse from the root (A/B measurements, tests)
static bool debug_no_frontier() {
    const char* e = std::getenv("GSRT_DEBUG_NO_FRONTIER");
    return e && e[0] == '1';
}

// GSRT_DEBUG_PROJECT_ALL=1: a rank of a sharded frame keeps every splat in its projection (A/B, tests)
static bool debug_project_all() {
    const char* e = std::getenv("GSRT_DEBUG_PROJECT_ALL");
    return e && e[0] == '1';
}

// GSRT_DEBUG_NO_GROUPS=1: no group lists, every tile traverses the BVH itself (A/B measurements, tests)
static bool debug_no_groups() {
    const char* e = std::getenv("GSRT_DEBUG_NO_GROUPS");
    return e && e[0] == '1';
}

// test / A-B knob: COR traversals test the leaf AABBs and cull footprints from the footprint array, as before leaf_fp
static bool debug_no_leaf_fp() {
    const char* e = std::getenv("GSRT_DEBUG_NO_LEAF_FP");
    return e && e[0] == '1';
}

template <bool SH, bool LUT, bool STATS>
static void launch_cor_t(hipStream_t st, const KArgs& k) {
    hipLaunchKernelGGL((k_render_cor<SH, LUT, STATS>), dim3(k.a.ntiles_local), dim3(64), 0, st, k);
}

// A rank of a sharded frame projects in sorted-leaf chunks (k_prep_cor) from this many ranks on: most 64-leaf chunks
// then lie wholly outside its band and are rejected by one box test, while its own splats are gathered by leaf.
// At 2 ranks a band is half the frame and the chunked walk costs more than it saves (profiles/r05/leaf_ab.txt)
constexpr uint32_t kLeafOrderRanks = 4;

// Grow one slot buffer (only on the first frame of a geometry: both streams are drained first, since the old
// buffer may still be read by either of them).
template <class T>
static gsrt_status grow_slot(gsrt_ctx* ctx, T** p, size_t bytes) {
    (void)hipFree(*p);
    *p = nullptr;
    GSRT_HIP(ctx, hipMalloc(p, bytes));
    return GSRT_OK;
}

// The prep streams' priority class from the sampled render kernel time (kPrioLowAboveUs). A switch makes the new
// pair wait for everything queued on the old one, so stream order carries over; events recorded on the old
// streams stay valid.
static void choose_prep_priority(gsrt_ctx* ctx) {
    // test switch GSRT_DEBUG_PREP_PRIORITY: 0 / 1 forced low / high (at creation), 2 switch at every frame
    const char* e = std::getenv("GSRT_DEBUG_PREP_PRIORITY");
    if (e && (e[0] == '0' || e[0] == '1')) return;
    const bool flip = e && e[0] == '2';
    if (!flip && ctx->render_us < 0.0f) return;  // no render kernel time sampled yet
    bool high = ctx->prep_high;
    if (flip) high = !high;
    else if (high && ctx->render_us > kPrioLowAboveUs) high = false;
    else if (!high && ctx->render_us < kPrioHighBelowUs) high = true;
    if (high == ctx->prep_high) return;
    hipStream_t* to = high ? ctx->prep_hi : ctx->prep_lo;
    hipStream_t* from = high ? ctx->prep_lo : ctx->prep_hi;
    for (uint32_t j = 0; j < kStreamSlots; ++j) {
        if (hipEventRecord(ctx->ev_hop[j], from[j]) != hipSuccess || hipStreamWaitEvent(to[j], ctx->ev_hop[j], 0) != hipSuccess) {
            // the old set cannot be waited for by event: drain it instead
            (void)hipGetLastError();
            for (uint32_t i = 0; i < kStreamSlots; ++i) (void)hipStreamSynchronize(from[i]);
        }
    }
    ctx->pstream = to[0];
    ctx->fstream = to[1];
    ctx->prep_high = high;
}

// frame slots in rotation: three, so that a frame's prep (a moving scene's refit, projection and group lists) may start
// while the two frames before it still render; two on slot streams (one slot per prep stream).
// Test switch GSRT_DEBUG_SLOTS=2: always two.
static uint32_t choose_slots(bool slot_streams) {
    const char* e = std::getenv("GSRT_DEBUG_SLOTS");
    return slot_streams || (e && e[0] == '2') ? 2u : kSlots;
}

bool use_slot_streams(gsrt_ctx* ctx, bool share) {
    for (uint32_t j = 0; j < kSlots; ++j) {
        FrameSlot& S = ctx->slot[j];
        if (!S.timed || hipEventQuery(S.t1) != hipSuccess) continue;  // not sampled, or still running
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, S.t0, S.t1) == hipSuccess) ctx->render_us = ms * 1e3f;
        S.timed = false;
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    choose_prep_priority(ctx);
    if (const char* e = std::getenv("GSRT_DEBUG_SLOT_STREAMS"))  // test knob: 0 never, 1 always
        if (e[0] == '0' || e[0] == '1') return e[0] == '1';
    if (ctx->render_us >= 0.0f) {
        const float enter = share ? kSlotEnterUs : kSlotEnterUsFrame, leave = share ? kSlotLeaveUs : kSlotLeaveUsFrame;
        if (!ctx->slot_mode && ctx->render_us < enter) ctx->slot_mode = true;
        else if (ctx->slot_mode && ctx->render_us > leave) ctx->slot_mode = false;
    }
    return ctx->slot_mode;
}

// The deal of a rank share's R render units (R a multiple of kXcds) over the XCDs: by cost, longest first (ties in the
// centre-out order), each unit to the XCD with the least cost so far among those holding fewer than R / kXcds; perm
// position k kXcds + x holds XCD x's k-th unit (xcd_local_tile_perm), so each XCD starts its longest units first
void deal_units(const double* cost, const uint32_t* centre, uint32_t R, uint32_t* perm) {
    std::vector<uint32_t> by(centre, centre + R);
    std::stable_sort(by.begin(), by.end(), [&](uint32_t a, uint32_t c) { return cost[a] > cost[c]; });
    double load[kXcds] = {};
    uint32_t count[kXcds] = {};
    for (uint32_t q : by) {
        uint32_t x = kXcds;
        for (uint32_t j = 0; j < kXcds; ++j)
            if (count[j] < R / kXcds && (x == kXcds || load[j] < load[x])) x = j;
        perm[count[x] * kXcds + x] = q;
        load[x] += cost[q];
        ++count[x];
    }
}

gsrt_status launch_render(gsrt_scene* sc, const gsrt_ubo& ubo, const RenderPlan& plan, float* d_out,
                          gsrt_raystate* d_rs, RenderSync* sync) {
    gsrt_ctx* ctx = sc->ctx;
    hipStream_t st = ctx->stream;
    if (sync) sync->stream = st;
    const bool stats = (plan.mode & GSRT_FLAG_STATS) != 0;
    const bool cor = (plan.mode & 0xffu) == GSRT_MODE_COR;
    // COR frames rotate over the kSlots frame slots, their prep kernels on the prep stream; REF and the
    // counting pass run everything on the render stream in slot 0, ordered after all earlier prep work
    const bool pipelined = cor && !stats;
    // slot streams (use_slot_streams, gsrt_internal.hpp): the frame's prep and render kernels on its slot's stream
    const bool slot_streams = pipelined && sync && sync->slot && sync->private_out;
    const uint32_t prev = ctx->prev_slot;  // the slot of the frame before this one
    if (pipelined) ctx->nslots = choose_slots(slot_streams);
    if (pipelined && ctx->next_slot >= ctx->nslots) ctx->next_slot = 0;  // (the rotation shrank: never the last slot)
    const uint32_t b = pipelined ? ctx->next_slot : 0u;
    FrameSlot& S = ctx->slot[b];
    hipStream_t ps = pipelined ? (slot_streams ? slot_stream(ctx, b) : ctx->pstream) : st;
    if (slot_streams && b > 0) {
        // scene updates go on pstream: a frame on another slot stream follows those queued so far, and the next
        // update's copies wait for this frame (order_update)
        if (ctx->side_updates[b]) {
            GSRT_HIP(ctx, hipEventRecord(ctx->ev_fit, ctx->pstream));
            GSRT_HIP(ctx, hipStreamWaitEvent(ps, ctx->ev_fit, 0));
            ctx->side_updates[b] = false;
        }
        ctx->side_frames[b] = true;
    }
    KArgs k;
    std::memset(&k, 0, sizeof k);
    k.ubo = ubo;
    RenderArgs& A = k.a;
    A.sh = sc->d_sh;
    A.nodes = sc->d_nodes[b];
    A.lut = ctx->d_lut;
    A.out = d_out;
    A.rs = d_rs;
    A.ray_stats = stats ? ctx->d_ray_stats : nullptr;
    A.counters = ctx->d_counters;
    A.n = sc->n;
    A.root_ref = sc->root_ref;
    A.root_box = sc->d_root_box[b];
    A.width = ubo.width; A.height = ubo.height;
    A.tiles_x = plan.tiles_x;
    A.tiles_y = plan.tiles_y;
    A.ntiles_local = local_tiles(plan);
    A.rank = plan.rank; A.nranks = plan.nranks; A.row0 = plan.row0(); A.row1 = plan.row1();
    if (sync && sync->dump8) {
        A.dump8 = 1u;
        A.esc = sync->esc;
        A.esc_cap = sync->esc_cap;
        A.accum = sync->accum;
    }
    A.tw = plan.tw; A.th = plan.th; A.s_lanes = plan.s_lanes; A.passes = plan.passes;
    A.packed = plan.packed ? 1u : 0u;
    A.samples = ubo.samples; A.bounces = ubo.bounces;
    A.stack_limit = kStack;
    if (const char* e = std::getenv("GSRT_DEBUG_STACK_LIMIT")) {  // test knob: exercise the DFS restart
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 8 && v < (long)kStack) A.stack_limit = (uint32_t)v;
    }
    if (A.ntiles_local == 0) {  // a band without rows (fewer tile rows than ranks): nothing to render
        timing_mark(ctx, 1);
        timing_mark(ctx, 2);
        return GSRT_OK;
    }
    if (cor) {
        A.use_groups = sc->n > 1 && !stats && !debug_no_groups();
        if (A.use_groups) {
            A.fg = plan.fg;
            A.groups_x = (A.tiles_x + A.fg - 1) / A.fg;
            A.groups = A.groups_x * ((A.tiles_y + A.fg - 1) / A.fg);
            if (!debug_no_frontier()) {
                A.sgroups_x = (A.groups_x + kSG - 1) / kSG;
                A.sgroups = A.sgroups_x * ((A.groups / A.groups_x + kSG - 1) / kSG);
            }
        }
        // (re)allocation of the slots' buffers: only on the first frame of a scene / frame geometry, so simply
        // drain both streams first. Every slot is sized at once: a lazily grown second slot would drain the
        // pipeline again on the next frame.
        auto slot_short = [&](uint32_t j) {
            const FrameSlot& Sj = ctx->slot[j];
            return Sj.list_tiles < A.ntiles_local || (A.use_groups && Sj.group_cap < A.groups) ||
                   (A.sgroups && Sj.frontier_cap < A.sgroups) || (sc->n && (!sc->d_recs[j] || !sc->d_footprint[j]));
        };
        const uint32_t nslots = pipelined ? ctx->nslots : 1u;
        bool any_short = false;
        for (uint32_t j = 0; j < nslots; ++j) any_short = any_short || slot_short(j);
        if (any_short) {
            gsrt_status s = sync_all(ctx);
            if (s != GSRT_OK) return s;
            for (uint32_t j = 0; j < nslots; ++j) {
                FrameSlot& Sj = ctx->slot[j];
                if (Sj.list_tiles < A.ntiles_local) {
                    Sj.list_tiles = 0;
                    if ((s = grow_slot(ctx, &Sj.d_lists, sizeof(uint32_t) * kCap * A.ntiles_local)) != GSRT_OK ||
                        (s = grow_slot(ctx, &Sj.d_list_hdr, sizeof(uint4) * A.ntiles_local)) != GSRT_OK)
                        return s;
                    Sj.list_tiles = A.ntiles_local;
                }
                if (A.use_groups && Sj.group_cap < A.groups) {
                    Sj.group_cap = 0;
                    if ((s = grow_slot(ctx, &Sj.d_glist, sizeof(uint64_t) * kGStride * A.groups)) != GSRT_OK ||
                        (s = grow_slot(ctx, &Sj.d_ghdr, sizeof(uint4) * A.groups)) != GSRT_OK)
                        return s;
                    Sj.group_cap = A.groups;
                }
                if (A.sgroups && Sj.frontier_cap < A.sgroups) {
                    Sj.frontier_cap = 0;
                    if ((s = grow_slot(ctx, &Sj.d_frontier, sizeof(uint32_t) * (kFront + 1) * A.sgroups)) != GSRT_OK) return s;
                    Sj.frontier_cap = A.sgroups;
                }
                if (sc->n && !sc->d_recs[j]) {
                    GSRT_HIP(ctx, hipMalloc(&sc->d_recs[j], sizeof(SplatRec) * sc->n));
                    GSRT_HIP(ctx, hipMalloc(&sc->d_keyed[j], sizeof(uint32_t) * ((sc->n + 31) / 32 + 1)));
                    GSRT_HIP(ctx, hipMemset(sc->d_keyed[j], 0xFF, sizeof(uint32_t) * ((sc->n + 31) / 32 + 1)));
                }
                if (sc->n && !sc->d_footprint[j]) GSRT_HIP(ctx, hipMalloc(&sc->d_footprint[j], kFpWords * sizeof(float4) * sc->n));
            }
        }
        A.lists = S.d_lists;
        A.list_hdr = reinterpret_cast<uint4*>(S.d_list_hdr);
        if (A.use_groups) {
            // centre-out dispatch order (the groups with the longest lists first, the light border groups last: the
            // kernel's tail is short groups instead of the heaviest ones started late), whole super-groups (kSG x kSG
            // groups, one frontier) dealt round-robin over the 8 XCDs (workgroup i runs on XCD i % 8), so an XCD's
            // consecutive groups share the top of the BVH in its L2. Measured at r03 (profiles/archive/r03/
            // pmc_gorder.txt): k_group_list's C3 FETCH_SIZE 246 -> 139 MB per launch against single groups centre-out.
            if (ctx->group_order_key[0] != A.groups_x || ctx->group_order_key[1] != A.groups ||
                ctx->group_order_key[2] != A.row0 || ctx->group_order_key[3] != A.row1 ||
                ctx->group_order_key[4] != A.nranks) {
                gsrt_status s = sync_all(ctx);
                if (s != GSRT_OK) return s;
                const uint32_t gy_n = A.groups / A.groups_x;
                // a rank of a sharded frame orders (and deals) only the groups with a tile row of its band (group_own
                // of them); the others go last and are not launched
                std::vector<uint8_t> own_g(A.groups);
                for (uint32_t g = 0; g < A.groups; ++g) {
                    const uint32_t gy = g / A.groups_x;
                    own_g[g] = (A.nranks <= 1 || (gy * A.fg < A.row1 && (gy + 1) * A.fg > A.row0)) ? 1 : 0;
                }
                std::vector<uint32_t> ord;
                ord.reserve(A.groups);
                auto centre_d2 = [](float x, float y, float w, float h) {
                    const float dx = x - 0.5f * w, dy = y - 0.5f * h;
                    return dx * dx + dy * dy;
                };
                constexpr uint32_t kXcds = 8;
                const uint32_t sx_n = (A.groups_x + kSG - 1) / kSG, sy_n = (gy_n + kSG - 1) / kSG;
                std::vector<uint32_t> sgs(sx_n * sy_n);
                std::vector<float> d2(sgs.size());
                for (uint32_t k = 0; k < sgs.size(); ++k) {
                    sgs[k] = k;
                    const float cx = std::min((float)((k % sx_n) * kSG) + 0.5f * kSG, (float)A.groups_x);
                    const float cy = std::min((float)((k / sx_n) * kSG) + 0.5f * kSG, (float)gy_n);
                    d2[k] = centre_d2(cx, cy, (float)A.groups_x, (float)gy_n);
                }
                std::stable_sort(sgs.begin(), sgs.end(), [&](uint32_t a, uint32_t c) { return d2[a] < d2[c]; });
                // super-groups with a group of this rank's, dealt round-robin over the XCDs
                std::vector<std::vector<uint32_t>> xl(kXcds);
                uint32_t dealt = 0, total = 0;
                for (uint32_t j = 0; j < sgs.size(); ++j) {
                    const uint32_t sx = sgs[j] % sx_n, sy = sgs[j] / sx_n;
                    std::vector<uint32_t>& l = xl[dealt % kXcds];
                    const size_t before = l.size();
                    for (uint32_t gy = sy * kSG; gy < std::min((sy + 1) * kSG, gy_n); ++gy)
                        for (uint32_t gx = sx * kSG; gx < std::min((sx + 1) * kSG, A.groups_x); ++gx)
                            if (own_g[gy * A.groups_x + gx]) l.push_back(gy * A.groups_x + gx);
                    if (l.size() > before) {
                        total += (uint32_t)(l.size() - before);
                        ++dealt;
                    }
                }
                // workgroup i takes the next group of XCD i % 8's list (or of the longest list left)
                std::vector<size_t> pos(kXcds, 0);
                for (uint32_t i = 0; i < total; ++i) {
                    uint32_t x = i % kXcds;
                    if (pos[x] == xl[x].size()) {
                        size_t best = 0;
                        for (uint32_t y = 0; y < kXcds; ++y)
                            if (xl[y].size() - pos[y] > best) { best = xl[y].size() - pos[y]; x = y; }
                    }
                    ord.push_back(xl[x][pos[x]++]);
                }
                ctx->group_own = total;
                for (uint32_t g = 0; g < A.groups; ++g)
                    if (!own_g[g]) ord.push_back(g);
                (void)hipFree(ctx->d_group_order);
                ctx->d_group_order = nullptr;
                ctx->group_order_key[0] = ctx->group_order_key[1] = 0;
                GSRT_HIP(ctx, hipMalloc(&ctx->d_group_order, sizeof(uint32_t) * A.groups));
                GSRT_HIP(ctx, hipMemcpy(ctx->d_group_order, ord.data(), sizeof(uint32_t) * A.groups, hipMemcpyHostToDevice));
                ctx->group_order_key[0] = A.groups_x;
                ctx->group_order_key[1] = A.groups;
                ctx->group_order_key[2] = A.row0;
                ctx->group_order_key[3] = A.row1;
                ctx->group_order_key[4] = A.nranks;
            }
            A.group_order = ctx->d_group_order;
            A.glist = reinterpret_cast<uint64_t*>(S.d_glist);
            A.ghdr = reinterpret_cast<uint4*>(S.d_ghdr);
            if (A.sgroups) A.frontier = S.d_frontier;
        }
    } else if (sc->n && !sc->d_recs[0]) {
        GSRT_HIP(ctx, hipMalloc(&sc->d_recs[0], sizeof(SplatRec) * sc->n));
    }
    A.recs = sc->d_recs[b];
    A.footprint = cor ? sc->d_footprint[b] : nullptr;
    A.depth_unsafe = sc->d_flags;
    // the depth cull pays where group lists overflow: groups of many samples per pixel (C5) or 32 pixels wide (C2, C4);
    // on the smaller groups of C3 and the 8-rank shares its tests cost more than they cull (profiles/r06/depth_cull_ab.txt)
    A.depth_cull = A.s_lanes >= kMoreLanes || plan.fg * plan.tw >= 32 ? 1u : 0u;
    // k_render_cor dispatch order of a rank of a sharded frame: the units of kDeal local tiles of the complete XCD
    // rounds centre-out (centred on the band's middle row: the central runs cost the most; started first, the launch
    // ends on the light border runs): 8-rank C3 share 0.308 -> 0.292 ms (r03, round-robin deal). When the context has
    // rendered a whole COR frame of this tile grid, its measured tile costs order the units instead: longest first,
    // each to the least-loaded XCD (8-rank C3 shares 0.3-6 % faster, C4 even: profiles/r06/deal_ab.txt; test switch
    // GSRT_DEBUG_DEAL=0 keeps centre-out). One device keeps the spatial order (C3 -2 %, C2 -2 %, C4 +1.5 % with it).
    if (cor && plan.nranks > 1) {
        const uint32_t nl = A.ntiles_local, R = (nl / (kXcds * kDeal)) * kXcds;
        const uint32_t key[5] = {nl, plan.row0(), plan.row1(), plan.tiles_x, plan.tiles_y};
        if (R > 1 && std::memcmp(key, ctx->run_order_key, sizeof key) != 0) {
            gsrt_status s = sync_all(ctx);
            if (s != GSRT_OK) return s;
            std::vector<uint32_t> perm(R);
            std::vector<float> d2(R);
            const float cy = 0.5f * (float)(plan.row0() + plan.row1());
            for (uint32_t q = 0; q < R; ++q) {
                uint32_t tx, ty;
                band_tile(q * kDeal + kDeal / 2, plan.row0(), plan.row1(), plan.tiles_x, tx, ty);
                const float dx = ((float)tx + 0.5f) - 0.5f * (float)plan.tiles_x, dy = ((float)ty + 0.5f) - cy;
                d2[q] = dx * dx + dy * dy;
                perm[q] = q;
            }
            std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t c) { return d2[a] < d2[c]; });
            const char* de = std::getenv("GSRT_DEBUG_DEAL");
            if (!(de && de[0] == '0') && ctx->tile_cost_tx == plan.tiles_x && ctx->tile_cost_ty == plan.tiles_y) {
                // a whole frame's measured tile costs (its last one on this context): the units longest first, each to
                // the XCD with the least cost so far among those not yet full (every XCD takes R / 8 units)
                std::vector<uint32_t> t((size_t)plan.tiles_x * plan.tiles_y);
                GSRT_HIP(ctx, hipMemcpy(t.data(), ctx->d_tile_cost[ctx->tile_cost_slot], sizeof(uint32_t) * t.size(),
                                        hipMemcpyDeviceToHost));
                std::vector<double> uc(R, 0.0);
                for (uint32_t q = 0; q < R; ++q)
                    for (uint32_t i = 0; i < kDeal; ++i) {
                        uint32_t tx, ty;
                        band_tile(q * kDeal + i, plan.row0(), plan.row1(), plan.tiles_x, tx, ty);
                        uc[q] += t[band_index(tx, ty, 0, plan.tiles_y, plan.tiles_x)];
                    }
                const std::vector<uint32_t> centre(perm);
                deal_units(uc.data(), centre.data(), R, perm.data());
            }
            (void)hipFree(ctx->d_run_order);
            ctx->d_run_order = nullptr;
            std::memset(ctx->run_order_key, 0, sizeof ctx->run_order_key);
            GSRT_HIP(ctx, hipMalloc(&ctx->d_run_order, sizeof(uint32_t) * R));
            GSRT_HIP(ctx, hipMemcpy(ctx->d_run_order, perm.data(), sizeof(uint32_t) * R, hipMemcpyHostToDevice));
            std::memcpy(ctx->run_order_key, key, sizeof key);
        }
        if (R > 1) A.run_order = ctx->d_run_order;
    }

    // ordering of the prep stage: after every scene change queued on the render stream (update, refit,
    // build), and after the render that last read this slot (frame f-2); not after the render of frame f-1
    if (pipelined) {
        // one flag per prep stream
        bool& dirty = ps == ctx->pstream ? ctx->main_dirty : ctx->main_dirty_f;
        if (dirty) {
            GSRT_HIP(ctx, hipEventRecord(ctx->ev_main, st));
            GSRT_HIP(ctx, hipStreamWaitEvent(ps, ctx->ev_main, 0));
            dirty = false;
        }
        // (on slot streams the slot's last render kernel is on ps already, unless it ran without them)
        if (S.render_pending && (!slot_streams || S.rstream != ps)) GSRT_HIP(ctx, hipStreamWaitEvent(ps, S.rendered, 0));
        if (gsrt_status su = wait_updates(ctx, ps); su != GSRT_OK) return su;  // the arrays' update copies
        ++ctx->frame_no;
        ctx->prev_slot = b;
        ctx->next_slot = (b + 1) % ctx->nslots;
    } else {
        // everything on the render stream, after all prep work issued so far (both prep streams: with slot
        // streams, frames run on fstream too); the next prep waits for it, and so do scene updates and refits
        // (their copies run on the prep stream: serial_pending)
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_main, ctx->pstream));
        GSRT_HIP(ctx, hipStreamWaitEvent(st, ctx->ev_main, 0));
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_front, ctx->fstream));
        GSRT_HIP(ctx, hipStreamWaitEvent(st, ctx->ev_front, 0));
        mark_main_dirty(ctx);
        ctx->serial_pending = true;
        ctx->serial_reads = true;  // an update retiring the arrays' buffers records this stream's position
        if (gsrt_status su = wait_updates(ctx, st); su != GSRT_OK) return su;
    }
    const bool leaf_fp = cor && !stats && sc->n >= 2 && !debug_no_leaf_fp();
    A.leaf_fp = leaf_fp ? 1u : 0u;
    // a rank of a sharded COR frame: its projection keeps only what its band can see, its frontier kernel skips the
    // super-groups outside the band
    RankTiles own{};
    if (cor && !stats && plan.nranks > 1 && !debug_project_all())
        own = RankTiles{1u, (float)(plan.row0() * plan.th), (float)(plan.row1() * plan.th), (float)ubo.width};
    A.own = own;
    // the BVH frontier needs only the camera and the fitted boxes: pipelined, it runs on its own stream beside
    // the projection (two short latency chains in parallel instead of in a row)
    hipStream_t fr = ps;
    uint32_t* keyed = pipelined ? sc->d_keyed[b] : nullptr;
    // the fused prep head (k_prep_cor: frontier + projection in one launch) for pipelined COR frames; otherwise the
    // frontier runs on its own stream beside the projection (two short latency chains in parallel), except on slot
    // streams
    const bool fused = pipelined && cor && A.frontier && sc->n >= 2;
    const bool front_stream = !slot_streams;
    // a rank share projects in sorted-leaf chunks (k_prep_cor, kLeafOrderRanks): the slot's keyed bitmap follows the
    // order (switching it starts the bitmap over: all ones, every key rewritten once)
    const bool leaf_order = fused && own.active && plan.nranks >= kLeafOrderRanks;
    // the frame's tile cost profile (RenderArgs::tile_cost): a sharded frame's goes where the caller says (gsrt_comm.cpp:
    // its profile frames), a whole COR frame's into the slot's own buffer (gsrt_row_costs)
    if (sync && sync->sharded) {
        A.tile_cost = sync->tile_cost;
    } else if (cor) {
        const uint32_t nt = plan.tiles_x * plan.tiles_y;
        if (ctx->tile_cost_cap < nt) {
            gsrt_status s = sync_all(ctx);
            if (s != GSRT_OK) return s;
            ctx->tile_cost_cap = 0;
            for (uint32_t j = 0; j < kSlots; ++j)
                if ((s = grow_slot(ctx, &ctx->d_tile_cost[j], sizeof(uint32_t) * nt)) != GSRT_OK) return s;
            ctx->tile_cost_cap = nt;
        }
        A.tile_cost = ctx->d_tile_cost[b];
        ctx->tile_cost_slot = b;
        ctx->tile_cost_tx = plan.tiles_x;
        ctx->tile_cost_ty = plan.tiles_y;
    }
    if (keyed && sc->slot_keyed_leaf[b] != leaf_order) {
        GSRT_HIP(ctx, hipMemsetAsync(keyed, 0xFF, sizeof(uint32_t) * ((sc->n + 31) / 32 + 1), ps));
        sc->slot_keyed_leaf[b] = leaf_order;
    }
    // a pipelined rank share: the slot's in-band bitmap for this camera and band (k_classify, once per AABB version and
    // key), which its fit and projection read instead of the AABBs of the splats the band cannot see
    const bool band_frame = pipelined && own.active && sc->n >= 2;
    const FitBandKey bkey = band_frame ? make_band_key(ubo, own) : FitBandKey{};
    if (band_frame) {
        if (!sc->d_inband[b]) GSRT_HIP(ctx, hipMalloc(&sc->d_inband[b], sizeof(uint32_t) * ((sc->n + 31) / 32 + 1)));
        if (sc->slot_inband_ver[b] != sc->aabb_version || !same_key(bkey, sc->slot_inband_key[b])) {
            hipLaunchKernelGGL(k_classify, dim3((sc->n + 255) / 256), dim3(64), 0, ps, sc->n, ubo, own, sc->d_aabbs,
                               sc->d_inband[b]);
            sc->slot_inband_ver[b] = sc->aabb_version;
            sc->slot_inband_key[b] = bkey;
        }
    }
    // the slot's boxes, fitted to the current geometry if a refit came since (on the stream of the prep kernels). A
    // rank share fits only what its band can see (FitBand: the 256-leaf chunks without a splat in its bitmap get empty
    // boxes; its projection gives their splats +inf keys anyway). COR frames put each leaf's footprint box into its node
    // (leaf_fp); REF and counting frames need the AABBs there, which the slot's fit restores
    {
        const FitBand fb{band_frame ? sc->d_inband[b] : nullptr};
        if (gsrt_status fs = lbvh_fit_if_stale(sc, b, ps, !leaf_fp, band_frame ? &fb : nullptr, band_frame ? &bkey : nullptr);
            fs != GSRT_OK)
            return fs;
    }
    sc->last_slot = b;
    if (fused) {
        k.a.cull2d = 1u;  // as set below for the non-stats render (neither part reads it)
        const ProjArgs pa{sc->n, sc->d_params, sc->d_aabbs, sc->d_recs[b], sc->d_nodes[b], sc->d_gid_slot,
                          sc->d_footprint[b], ctx->d_counters, own, keyed, A.leaf_fp,
                          leaf_order ? sc->d_leaf_gid : nullptr, band_frame ? sc->d_inband[b] : nullptr,
                          sc->d_flags};
        hipLaunchKernelGGL(k_prep_cor, dim3(A.sgroups + (sc->n + 63) / 64), dim3(64), 0, ps, k, pa);
    } else if (front_stream && pipelined && cor && A.frontier) {
        fr = ctx->fstream;
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_fit, ps));
        GSRT_HIP(ctx, hipStreamWaitEvent(fr, ctx->ev_fit, 0));
        k.a.cull2d = 1u;  // as set below for the non-stats render (the frontier does not read it)
        hipLaunchKernelGGL(k_frontier, dim3(A.sgroups), dim3(64), 0, fr, k);
    }
    // pipelined COR frames keep the slot's keyed bitmap; any other projection of the slot (REF, counting pass)
    // writes every record unbooked, so the bitmap goes back to all ones behind it (the next prep waits for it)
    if (!fused)
        launch_project(ps, sc->n, plan.mode, ubo, sc->d_params, sc->d_aabbs, sc->d_recs[b], sc->d_nodes[b],
                       sc->d_gid_slot, cor ? sc->d_footprint[b] : nullptr, ctx->d_counters, &own, keyed, leaf_fp,
                       sc->d_flags);
    sc->slot_leaf_fp[b] = leaf_fp;  // (either projection above)
    if (!pipelined && sc->n && sc->d_keyed[b])
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_keyed[b], 0xFF, sizeof(uint32_t) * ((sc->n + 31) / 32 + 1), ps));
    if (!cor) {
        if (sc->ntri) {
            const size_t px = (size_t)ubo.width * ubo.height;
            if (ctx->tri_t_pixels < px) {
                gsrt_status s = sync_all(ctx);
                if (s != GSRT_OK) return s;
                ctx->tri_t_pixels = 0;
                if ((s = grow_slot(ctx, &ctx->d_tri_t, sizeof(float) * px)) != GSRT_OK) return s;
                ctx->tri_t_pixels = px;
            }
            launch_mesh_thit(st, ubo, sc, ctx->d_tri_t);
            k.a.tri_t = ctx->d_tri_t;
        }
        if (sync && sync->wait) GSRT_HIP(ctx, hipStreamWaitEvent(st, sync->wait, 0));
        if (sync) sync->stream = st;
        timing_mark(ctx, 1);
        if (stats) hipLaunchKernelGGL((k_render_ref<true>), dim3(A.ntiles_local), dim3(64), 0, st, k);
        else hipLaunchKernelGGL((k_render_ref<false>), dim3(A.ntiles_local), dim3(64), 0, st, k);
        if (stats && A.ray_stats && !plan.packed)  // VS-style traversal statistics (gsrt_vs_stats)
            hipLaunchKernelGGL(k_ref_node_stats, dim3(((ubo.width + 7) / 8) * ((ubo.height + 7) / 8)), dim3(64), 0, st, k);
        timing_mark(ctx, 2);
        GSRT_HIP(ctx, hipGetLastError());
        return GSRT_OK;
    }
    const bool sh = sc->d_sh != nullptr;
    const bool lut = (plan.mode & GSRT_FLAG_LUT) != 0;
    void (*render)(hipStream_t, const KArgs&) =
        sh ? (lut ? (stats ? launch_cor_t<true, true, true> : launch_cor_t<true, true, false>)
                  : (stats ? launch_cor_t<true, false, true> : launch_cor_t<true, false, false>))
           : (lut ? (stats ? launch_cor_t<false, true, true> : launch_cor_t<false, true, false>)
                  : (stats ? launch_cor_t<false, false, true> : launch_cor_t<false, false, false>));
    k.a.cull2d = stats ? 0u : 1u;  // the counting pass keeps every AABB candidate (|C_r| of SURVEY.md 8d)
    if (A.frontier && fr != ps) {  // pipelined: the frontier ran beside the projection; join it here
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_front, fr));
        GSRT_HIP(ctx, hipStreamWaitEvent(ps, ctx->ev_front, 0));
    } else if (A.frontier && !fused) {
        hipLaunchKernelGGL(k_frontier, dim3(A.sgroups), dim3(64), 0, ps, k);
    }
    // the first-round lists, on the prep stream beside the previous frame's render kernel. Side lists: a rank share of
    // a moving scene (an update or refit came before this frame, and likely comes before the next) runs them on the
    // other prep stream, which idles on the two-stream scheme, so that the next frame's update copies, refit and
    // projection on the prep stream (which read and write none of this slot's lists) need not wait for them: the rank's
    // serial chain is then max(lists, copies) + fit + projection instead of their sum. The lists read only this
    // slot's nodes, records and footprints, and the render kernel waits for them through `prepared` (recorded there)
    const bool side_lists = pipelined && !slot_streams && sync && sync->sharded && ctx->scene_moved && A.use_groups &&
                            ps == ctx->pstream;
    hipStream_t ls = ps;
    if (side_lists) {
        ls = ctx->fstream;
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_lists, ps));
        GSRT_HIP(ctx, hipStreamWaitEvent(ls, ctx->ev_lists, 0));
    }
    if (pipelined) ctx->scene_moved = false;
    if (A.use_groups) {
        // only the groups with a tile of this rank's band (the head of group_order); the others would return at once
        const uint32_t ng = std::max(1u, std::min(ctx->group_own, A.groups));
        if (A.fg == 2) hipLaunchKernelGGL(k_group_list<2>, dim3(ng), dim3(64), 0, ls, k);
        else hipLaunchKernelGGL(k_group_list<kFG>, dim3(ng), dim3(64), 0, ls, k);
        for (uint32_t seg = 1; seg < kGSegs && A.s_lanes >= kMoreLanes; ++seg) {
            if (A.fg == 2) hipLaunchKernelGGL(k_group_more<2>, dim3(ng), dim3(64), 0, ls, k);
            else hipLaunchKernelGGL(k_group_more<kFG>, dim3(ng), dim3(64), 0, ls, k);
        }
    }
    else hipLaunchKernelGGL(k_collect_cor, dim3(A.ntiles_local), dim3(64), 0, ps, k);
    GSRT_HIP(ctx, hipGetLastError());
    // the render kernel: on the render stream after the lists (cross-stream), or (slot streams) on the slot's
    // stream right behind them, after the previous frame's render kernel (cross-stream)
    hipStream_t rs = st;
    if (slot_streams) {
        rs = ps;
        const FrameSlot& O = ctx->slot[prev];
        if (O.render_pending && !(sync && sync->private_out)) GSRT_HIP(ctx, hipStreamWaitEvent(rs, O.rendered, 0));
    } else if (pipelined) {
        GSRT_HIP(ctx, hipEventRecord(S.prepared, ls));
        GSRT_HIP(ctx, hipStreamWaitEvent(st, S.prepared, 0));
    }
    if (sync && sync->wait) GSRT_HIP(ctx, hipStreamWaitEvent(rs, sync->wait, 0));
    if (sync) sync->stream = rs;
    k.a.prelisted = 1;
    // sampled render kernel time for the slot-stream and prep-priority decisions (use_slot_streams)
    const bool sample = pipelined && sync && !S.timed && ctx->frame_no % kTimedEvery == 1 &&
                        S.t0 && S.t1;
    if (sample) GSRT_HIP(ctx, hipEventRecord(S.t0, rs));
    timing_mark(ctx, 1, rs);  // the timed kernel is the shading/continuation kernel k_render_cor
#ifdef GSRT_WAVE_TIMES
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, rs, 0u);
#endif
    render(rs, k);
#ifdef GSRT_WAVE_TIMES
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, rs, 1u);
#endif
    GSRT_HIP(ctx, hipGetLastError());
    timing_mark(ctx, 2, rs);
    if (sample) {
        GSRT_HIP(ctx, hipEventRecord(S.t1, rs));
        S.timed = true;
    }
    if (pipelined) {
        GSRT_HIP(ctx, hipEventRecord(S.rendered, rs));
        S.render_pending = true;
        S.rstream = rs;
    }
    ctx->last_slot_streams = slot_streams;
    // whatever follows on the render stream (copies, gathers, downloads) comes after this frame
    if (slot_streams) GSRT_HIP(ctx, hipStreamWaitEvent(st, S.rendered, 0));
    return GSRT_OK;
}

// a band's row costs from its tiles' (k_render_cor's tile_cost, local order): one wave per row
__global__ __launch_bounds__(64) void k_row_sum(const uint32_t* __restrict__ tile_cost, uint32_t* __restrict__ row_cost,
                                               uint32_t tiles_x, uint32_t row0, uint32_t row1) {
    const uint32_t ty = row0 + blockIdx.x;
    uint32_t v = 0;
    for (uint32_t tx = threadIdx.x; tx < tiles_x; tx += 64) v += tile_cost[band_index(tx, ty, row0, row1, tiles_x)];
    v = (uint32_t)wave_sum(v);
    if (threadIdx.x == 0) row_cost[ty] = v;
}

void launch_row_sum(hipStream_t s, const uint32_t* tile_cost, uint32_t* row_cost, uint32_t tiles_x, uint32_t row0,
                    uint32_t row1) {
    if (row1 > row0) hipLaunchKernelGGL(k_row_sum, dim3(row1 - row0), dim3(64), 0, s, tile_cost, row_cost, tiles_x, row0, row1);
}

__global__ __launch_bounds__(256) void k_unpack(const float4* __restrict__ g, float4* __restrict__ fb, uint32_t W,
                                                uint32_t H, uint32_t tw, uint32_t th, uint32_t tiles_x, const Bands bands,
                                                uint32_t tiles_per_rank) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W, tx = x / tw, ty = y / th;
    const uint32_t r = band_of(bands, ty);
    const uint32_t lt = band_index(tx, ty, bands.row[r], bands.row[r + 1], tiles_x);
    const uint32_t pin = (y % th) * tw + (x % tw);
    fb[i] = g[((size_t)r * tiles_per_rank + lt) * (tw * th) + pin];
}

__global__ __launch_bounds__(256) void k_unpack_dump8(const uint32_t* __restrict__ g, uint32_t* __restrict__ codes,
                                                      uint32_t W, uint32_t H, uint32_t tw, uint32_t th, uint32_t tiles_x,
                                                      const Bands bands, size_t block_words) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W, tx = x / tw, ty = y / th;
    const uint32_t r = band_of(bands, ty);
    const uint32_t lt = band_index(tx, ty, bands.row[r], bands.row[r + 1], tiles_x);
    codes[i] = g[(size_t)r * block_words + (size_t)lt * (tw * th) + (y % th) * tw + (x % tw)];
}

void launch_unpack_dump8(hipStream_t s, const uint32_t* gathered, uint32_t* codes, const RenderPlan& p, uint32_t W,
                         uint32_t H, uint32_t tiles_per_rank, size_t block_words) {
    (void)tiles_per_rank;
    hipLaunchKernelGGL(k_unpack_dump8, dim3((W * H + 255) / 256), dim3(256), 0, s, gathered, codes, W, H, p.tw, p.th,
                       p.tiles_x, p.bands, block_words);
}

void launch_unpack(hipStream_t s, const float* gathered, float* fb, const RenderPlan& p, uint32_t W, uint32_t H,
                   uint32_t tiles_per_rank) {
    hipLaunchKernelGGL(k_unpack, dim3((W * H + 255) / 256), dim3(256), 0, s, reinterpret_cast<const float4*>(gathered),
                       reinterpret_cast<float4*>(fb), W, H, p.tw, p.th, p.tiles_x, p.bands, tiles_per_rank);
}

}  // namespace gsrt

#ifdef GSRT_WAVE_TIMES
extern "C" int gsrt_diag_stamps(uint32_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gsrt::g_stamps), 16, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int gsrt_diag_wave_times(uint32_t kind, void* out, uint32_t n) {
    if (kind > 1 || n > (1u << 18)) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gsrt::g_wave_times), sizeof(uint4) * n, sizeof(uint4) * (1u << 18) * kind,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" gsrt_status gsrt_deal_units(const double* cost, const uint32_t* centre, uint32_t units, uint32_t* perm) {
    if (!cost || !centre || !perm || units % gsrt::kXcds) return GSRT_E_ARG;
    std::vector<uint8_t> seen(units, 0);  // centre must be a permutation of the units
    for (uint32_t i = 0; i < units; ++i) {
        if (centre[i] >= units || seen[centre[i]]) return GSRT_E_ARG;
        seen[centre[i]] = 1;
    }
    gsrt::deal_units(cost, centre, units, perm);
    return GSRT_OK;
}
