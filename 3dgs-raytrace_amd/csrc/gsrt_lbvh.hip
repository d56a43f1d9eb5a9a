// gsrt_lbvh.hip -- on-device LBVH over the Gaussian AABBs (replaces the Embree rtcBuildBVH TLAS build,
// mesa-vulkan-sim/src/gallium/frontends/lavapipe/lvp_acceleration_structure.c:1329-1351, and the per-
// Gaussian BLAS of RayTracingInVulkan/src/Vulkan/RayTracing/Application.cpp:253-398).
//
//   1. centroid bounds         two-stage block reduction
//   2. 30-bit Morton codes     of AABB centroids quantised to 1024^3
//   3. LSD radix sort          8-bit digits, 4 passes: per-block histogram -> one-block exclusive scan ->
//                              stable scatter ranked by a wave-level multisplit (8 ballots per key)
//   4. Karras hierarchy        one thread per internal node (Karras 2012, duplicate codes tie-broken by index)
//   5. bottom-up AABB fit      level-synchronous: nodes ordered by depth once per build, then one launch
//                              per level from the deepest up (kernel boundaries order the levels; no
//                              cross-XCD fences). The same launches refit new AABBs (config 5). Trees deeper
//                              than kMaxLevels fall back to k_fit (one thread per leaf, second arriver climbs).
//
// Node boxes are exact unions of fp32 AABBs (min/max are exact), so any box that contains a leaf the
// exact slab test hits is itself hit: the BVH changes only the work, never the candidate set.
#include "gsrt_internal.hpp"

namespace gsrt {

namespace {

constexpr int kSortBlock = 256;
constexpr uint32_t kMaxLevels = 256;  // deeper trees (degenerate inputs) fall back to the atomic climb k_fit
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortBlock * kSortItems;

__global__ __launch_bounds__(256) void k_bounds_partial(uint32_t n, const gsrt_aabb* __restrict__ a,
                                                        float* __restrict__ partial) {
    __shared__ float red[6][256];
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        gsrt_aabb b = a[i];
        float c[3] = {0.5f * (b.min_x + b.max_x), 0.5f * (b.min_y + b.max_y), 0.5f * (b.min_z + b.max_z)};
#pragma unroll
        for (int k = 0; k < 3; ++k) { mn[k] = fminf(mn[k], c[k]); mx[k] = fmaxf(mx[k], c[k]); }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { red[k][threadIdx.x] = mn[k]; red[3 + k][threadIdx.x] = mx[k]; }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + s]);
                red[3 + k][threadIdx.x] = fmaxf(red[3 + k][threadIdx.x], red[3 + k][threadIdx.x + s]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) partial[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_bounds_final(uint32_t nparts, float* __restrict__ partial,
                                                      float* __restrict__ out) {
    __shared__ float red[6][256];
    float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = threadIdx.x; i < nparts; i += 256)
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] = k < 3 ? fminf(v[k], partial[i * 6 + k]) : fmaxf(v[k], partial[i * 6 + k]);
#pragma unroll
    for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s)
#pragma unroll
            for (int k = 0; k < 6; ++k)
                red[k][threadIdx.x] = k < 3 ? fminf(red[k][threadIdx.x], red[k][threadIdx.x + s])
                                            : fmaxf(red[k][threadIdx.x], red[k][threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x < 6) out[threadIdx.x] = red[threadIdx.x][0];
}

__device__ inline uint32_t expand_bits10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ __launch_bounds__(256) void k_morton(uint32_t n, const gsrt_aabb* __restrict__ a,
                                                const float* __restrict__ bounds, uint32_t* __restrict__ codes,
                                                uint32_t* __restrict__ ids) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    gsrt_aabb b = a[i];
    float c[3] = {0.5f * (b.min_x + b.max_x), 0.5f * (b.min_y + b.max_y), 0.5f * (b.min_z + b.max_z)};
    uint32_t q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float ext = bounds[3 + k] - bounds[k];
        float u = ext > 0.0f ? (c[k] - bounds[k]) / ext : 0.0f;
        u = fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
        q[k] = (uint32_t)u;
    }
    codes[i] = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
    ids[i] = i;
}

__global__ __launch_bounds__(kSortBlock) void k_radix_hist(uint32_t n, const uint32_t* __restrict__ keys,
                                                           uint32_t shift, uint32_t nblocks,
                                                           uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
#pragma unroll 4
    for (int it = 0; it < kSortItems; ++it) {
        uint32_t idx = base + it * kSortBlock + threadIdx.x;
        if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of hist[0..len) in place by one 1024-thread block
__global__ __launch_bounds__(1024) void k_scan_inplace(uint32_t len, uint32_t* __restrict__ v) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (len + 1023) / 1024;
    const uint32_t b = threadIdx.x * per, e = min(len, b + per);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += v[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t x = threadIdx.x >= (uint32_t)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = b; i < e; ++i) { uint32_t x = v[i]; v[i] = run; run += x; }
}

__device__ inline uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(kSortBlock) void k_radix_scatter(uint32_t n, const uint32_t* __restrict__ kin,
                                                              const uint32_t* __restrict__ vin,
                                                              uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                              uint32_t shift, uint32_t nblocks,
                                                              const uint32_t* __restrict__ hist) {
    __shared__ uint32_t gofs[256];
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcount[4][256];
    __shared__ uint32_t wbase[4][256];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    gofs[t] = hist[t * nblocks + blockIdx.x];
    run[t] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) wcount[k][t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
    for (int it = 0; it < kSortItems; ++it) {
        const uint32_t idx = base + it * kSortBlock + t;
        const bool valid = idx < n;
        uint32_t key = valid ? kin[idx] : 0u;
        uint32_t val = valid ? vin[idx] : 0u;
        uint32_t d = (key >> shift) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            bool bit = (d >> b) & 1u;
            uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t rank = popc_below(peers);
        if (valid && rank == 0) wcount[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            uint32_t r0 = run[t];
            uint32_t c0 = wcount[0][t], c1 = wcount[1][t], c2 = wcount[2][t], c3 = wcount[3][t];
            wbase[0][t] = r0;
            wbase[1][t] = r0 + c0;
            wbase[2][t] = r0 + c0 + c1;
            wbase[3][t] = r0 + c0 + c1 + c2;
            run[t] = r0 + c0 + c1 + c2 + c3;
            wcount[0][t] = wcount[1][t] = wcount[2][t] = wcount[3][t] = 0;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = gofs[d] + wbase[w][d] + rank;
            kout[pos] = key;
            vout[pos] = val;
        }
        (void)lane;
    }
}

__device__ inline int lbvh_delta(const uint32_t* __restrict__ codes, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    uint32_t a = codes[i], b = codes[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

__global__ __launch_bounds__(256) void k_karras(int n, const uint32_t* __restrict__ codes,
                                                const uint32_t* __restrict__ gid, BvhNode* __restrict__ nodes,
                                                uint32_t* __restrict__ leaf_parent, uint32_t* __restrict__ node_parent) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (lbvh_delta(codes, n, i, i + 1) - lbvh_delta(codes, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = lbvh_delta(codes, n, i, i - d);
    int lmax = 2;
    while (lbvh_delta(codes, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (lbvh_delta(codes, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = lbvh_delta(codes, n, i, j);
    int s = 0, step = l;
    do {
        step = (step + 1) >> 1;
        const int ns = s + step;
        if (ns < l && lbvh_delta(codes, n, i, i + ns * d) > dnode) s = ns;
    } while (step > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lo = min(i, j), hi = max(i, j);
    uint32_t lref, rref;
    if (lo == gamma) { lref = kLeafBit | gid[gamma]; leaf_parent[gamma] = (uint32_t)i; }
    else { lref = (uint32_t)gamma; node_parent[gamma] = (uint32_t)i; }
    if (hi == gamma + 1) { rref = kLeafBit | gid[gamma + 1]; leaf_parent[gamma + 1] = (uint32_t)i | kLeafBit; }
    else { rref = (uint32_t)(gamma + 1); node_parent[gamma + 1] = (uint32_t)i | kLeafBit; }
    nodes[i].l_ref = lref;
    nodes[i].r_ref = rref;
    nodes[i].l_key = 0u;
    nodes[i].r_key = 0u;
    if (i == 0) node_parent[0] = 0xFFFFFFFFu;  // root
}

__device__ inline void store_box(float* dst, const float b[6]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) __hip_atomic_store(dst + k, b[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < 3; ++k) __hip_atomic_store(dst + 4 + k, b[3 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void load_box(const float* src, float b[6]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) b[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < 3; ++k) b[3 + k] = __hip_atomic_load(src + 4 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bottom-up fit. Child box slots: left = {l_lo, l_hi} at float offset 0 (lo) / 4 (hi), right = {r_lo, r_hi}
// at 8 / 12. The second thread to reach a parent unions both slots and climbs on.
__global__ __launch_bounds__(256) void k_fit(uint32_t n, const gsrt_aabb* __restrict__ aabbs,
                                             const uint32_t* __restrict__ leaf_gid,
                                             const uint32_t* __restrict__ leaf_parent,
                                             const uint32_t* __restrict__ node_parent, BvhNode* nodes,
                                             uint32_t* flags, float* root_box) {
    uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const gsrt_aabb a = aabbs[leaf_gid[k]];
    float box[6] = {a.min_x, a.min_y, a.min_z, a.max_x, a.max_y, a.max_z};
    uint32_t lp = leaf_parent[k];
    uint32_t p = lp & ~kLeafBit, side = lp >> 31;
    for (;;) {
        float* slot = reinterpret_cast<float*>(nodes + p) + (side ? 8 : 0);
        store_box(slot, box);
        __threadfence();
        const uint32_t old = atomicAdd(flags + p, 1u);
        if (old == 0u) return;
        __threadfence();
        float lb[6], rb[6];
        load_box(reinterpret_cast<const float*>(nodes + p), lb);
        load_box(reinterpret_cast<const float*>(nodes + p) + 8, rb);
#pragma unroll
        for (int q = 0; q < 3; ++q) { box[q] = fminf(lb[q], rb[q]); box[3 + q] = fmaxf(lb[3 + q], rb[3 + q]); }
        const uint32_t np = node_parent[p];  // parent | side << 31; all ones at the root
        if (np == 0xFFFFFFFFu) {
#pragma unroll
            for (int q = 0; q < 6; ++q) root_box[q] = box[q];
            return;
        }
        side = np >> 31;
        p = np & ~kLeafBit;
    }
}

// gid -> (parent node, side) of its leaf slot: where the projection kernel writes the leaf's sort key
__global__ __launch_bounds__(256) void k_gid_slot(uint32_t n, const uint32_t* __restrict__ leaf_gid,
                                                  const uint32_t* __restrict__ leaf_parent, uint32_t* __restrict__ slot) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k < n) slot[leaf_gid[k]] = leaf_parent[k];
}

// Depth of every internal node (root = 0): walk the parent links up to the root. O(n * depth) loads of a
// 4-B array that stays in L2; run once per build to order the level-synchronous fit. The histogram is
// aggregated per block in LDS (a global atomic per node would serialise on a few hot lines).
__global__ __launch_bounds__(256) void k_node_depth(uint32_t ni, const uint32_t* __restrict__ node_parent,
                                                    uint32_t* __restrict__ depth, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kMaxLevels];
    for (uint32_t j = threadIdx.x; j < kMaxLevels; j += 256) h[j] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < ni) {
        uint32_t d = 0, p = i;
        while (node_parent[p] != 0xFFFFFFFFu && d < kMaxLevels - 1) {
            p = node_parent[p] & ~kLeafBit;
            ++d;
        }
        depth[i] = d;
        atomicAdd(h + d, 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < kMaxLevels; j += 256)
        if (h[j]) atomicAdd(hist + j, h[j]);
}

// nodes in level order: level_nodes[off[d] .. off[d+1]) are the nodes of depth d (any order inside a level).
// Per block: LDS ranks, one global cursor reservation per non-empty level.
__global__ __launch_bounds__(256) void k_level_scatter(uint32_t ni, const uint32_t* __restrict__ depth,
                                                       uint32_t* __restrict__ cursor, uint32_t* __restrict__ level_nodes) {
    __shared__ uint32_t h[kMaxLevels], base[kMaxLevels];
    for (uint32_t j = threadIdx.x; j < kMaxLevels; j += 256) h[j] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t d = 0, r = 0;
    if (i < ni) {
        d = depth[i];
        r = atomicAdd(h + d, 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < kMaxLevels; j += 256)
        if (h[j]) base[j] = atomicAdd(cursor + j, h[j]);
    __syncthreads();
    if (i < ni) level_nodes[base[d] + r] = i;
}

// Level-synchronous fit of the nodes of one depth: each child slot gets the child's box (a leaf's AABB, or
// the union of an internal child's two slots, fitted by the previous, deeper launch). Kernel boundaries
// order the levels, so no cross-XCD fences are needed.
__global__ __launch_bounds__(256) void k_fit_level(const uint32_t* __restrict__ level_nodes, uint32_t count,
                                                   const gsrt_aabb* __restrict__ aabbs, BvhNode* __restrict__ nodes,
                                                   float* __restrict__ root_box) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint32_t i = level_nodes[t];
    float* slots = reinterpret_cast<float*>(nodes + i);
    const uint32_t refs[2] = {nodes[i].l_ref, nodes[i].r_ref};
    float u[6];
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        float b[6];
        const uint32_t ref = refs[side];
        if (ref & kLeafBit) {
            const gsrt_aabb a = aabbs[ref & ~kLeafBit];
            b[0] = a.min_x; b[1] = a.min_y; b[2] = a.min_z; b[3] = a.max_x; b[4] = a.max_y; b[5] = a.max_z;
        } else {
            const float* c = reinterpret_cast<const float*>(nodes + ref);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                b[q] = fminf(c[q], c[8 + q]);
                b[3 + q] = fmaxf(c[4 + q], c[12 + q]);
            }
        }
        float* dst = slots + (side ? 8 : 0);
        dst[0] = b[0]; dst[1] = b[1]; dst[2] = b[2];
        dst[4] = b[3]; dst[5] = b[4]; dst[6] = b[5];
#pragma unroll
        for (int q = 0; q < 6; ++q) u[q] = side ? (q < 3 ? fminf(u[q], b[q]) : fmaxf(u[q], b[q])) : b[q];
    }
    if (i == 0) {
#pragma unroll
        for (int q = 0; q < 6; ++q) root_box[q] = u[q];
    }
}

}  // namespace

static gsrt_status alloc_bvh(gsrt_scene* sc) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n;
    const uint32_t ni = n > 1 ? n - 1 : 1;
    for (uint32_t b = 0; b < kSlots; ++b)
        if (!sc->d_nodes[b]) GSRT_HIP(ctx, hipMalloc(&sc->d_nodes[b], sizeof(BvhNode) * ni));
    if (!sc->d_leaf_parent) GSRT_HIP(ctx, hipMalloc(&sc->d_leaf_parent, sizeof(uint32_t) * n));
    if (!sc->d_node_parent) GSRT_HIP(ctx, hipMalloc(&sc->d_node_parent, sizeof(uint32_t) * ni));
    if (!sc->d_gid_slot) GSRT_HIP(ctx, hipMalloc(&sc->d_gid_slot, sizeof(uint32_t) * n));
    if (!sc->d_leaf_gid) GSRT_HIP(ctx, hipMalloc(&sc->d_leaf_gid, sizeof(uint32_t) * n));
    if (!sc->d_morton) GSRT_HIP(ctx, hipMalloc(&sc->d_morton, sizeof(uint32_t) * n));
    if (!sc->d_flags) GSRT_HIP(ctx, hipMalloc(&sc->d_flags, sizeof(uint32_t) * ni));
    for (uint32_t b = 0; b < kSlots; ++b)
        if (!sc->d_root_box[b]) GSRT_HIP(ctx, hipMalloc(&sc->d_root_box[b], sizeof(float) * 8));
    return GSRT_OK;
}

gsrt_status lbvh_fit(gsrt_scene* sc, uint32_t slot, hipStream_t st) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n;
    BvhNode* nodes = sc->d_nodes[slot];
    float* root_box = sc->d_root_box[slot];
    if (n == 0) return GSRT_OK;
    if (n == 1) {  // the root is the leaf: its AABB is the root box (same float order)
        GSRT_HIP(ctx, hipMemcpyAsync(root_box, sc->d_aabbs, sizeof(float) * 6, hipMemcpyDeviceToDevice, st));
        return GSRT_OK;
    }
    if (!sc->level_off.empty()) {
        for (size_t d = sc->level_off.size() - 1; d-- > 0;) {  // deepest level first
            const uint32_t cnt = sc->level_off[d + 1] - sc->level_off[d];
            if (!cnt) continue;
            hipLaunchKernelGGL(k_fit_level, dim3((cnt + 255) / 256), dim3(256), 0, st, sc->d_level_nodes + sc->level_off[d],
                               cnt, sc->d_aabbs, nodes, root_box);
        }
    } else {  // d_flags is shared: fits never run concurrently (the streams are ordered around them, §3 DESIGN)
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_flags, 0, sizeof(uint32_t) * (n - 1), st));
        hipLaunchKernelGGL(k_fit, dim3((n + 255) / 256), dim3(256), 0, st, n, sc->d_aabbs, sc->d_leaf_gid,
                           sc->d_leaf_parent, sc->d_node_parent, nodes, sc->d_flags, root_box);
    }
    GSRT_HIP(ctx, hipGetLastError());
    return GSRT_OK;  // asynchronous: the render kernels read the root box from d_root_box[slot]
}

gsrt_status lbvh_fit_if_stale(gsrt_scene* sc, uint32_t slot, hipStream_t st) {
    if (sc->slot_geom[slot] == sc->geom_version) return GSRT_OK;
    gsrt_status s = lbvh_fit(sc, slot, st);
    if (s == GSRT_OK) sc->slot_geom[slot] = sc->geom_version;
    return s;
}

// after a build: slot 0 fitted on st, its topology and boxes copied to the other slots
static gsrt_status fit_all_slots(gsrt_scene* sc, hipStream_t st) {
    gsrt_ctx* ctx = sc->ctx;
    gsrt_status s = lbvh_fit(sc, 0, st);
    if (s != GSRT_OK) return s;
    const size_t ni = sc->n > 1 ? sc->n - 1 : 1;
    for (uint32_t b = 1; b < kSlots; ++b) {
        GSRT_HIP(ctx, hipMemcpyAsync(sc->d_nodes[b], sc->d_nodes[0], sizeof(BvhNode) * ni, hipMemcpyDeviceToDevice, st));
        GSRT_HIP(ctx, hipMemcpyAsync(sc->d_root_box[b], sc->d_root_box[0], sizeof(float) * 8, hipMemcpyDeviceToDevice, st));
    }
    for (uint32_t b = 0; b < kSlots; ++b) sc->slot_geom[b] = sc->geom_version;
    // the slots' node keys are the copied (or stale) ones: k_project's keyed bitmaps start over (all ones)
    for (uint32_t b = 0; b < kSlots; ++b)
        if (sc->d_keyed[b]) GSRT_HIP(ctx, hipMemsetAsync(sc->d_keyed[b], 0xFF, sizeof(uint32_t) * ((sc->n + 31) / 32 + 1), st));
    return GSRT_OK;
}

gsrt_status lbvh_build(gsrt_scene* sc) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n;
    hipStream_t st = ctx->stream;
    sc->bvh_built = false;
    if (n == 0) { sc->bvh_built = true; return GSRT_OK; }
    gsrt_status s = alloc_bvh(sc);
    if (s != GSRT_OK) return s;
    if (n == 1) {
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_leaf_gid, 0, 4, st));
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_morton, 0, 4, st));
        sc->root_ref = kLeafBit | 0u;
        s = fit_all_slots(sc, st);
        if (s == GSRT_OK) sc->bvh_built = true;
        return s;
    }
    // scratch: partial bounds, keys/values ping-pong, histogram
    const uint32_t nblocks = (n + kSortTile - 1) / kSortTile;
    const uint32_t nparts = std::min<uint32_t>(1024u, (n + 255) / 256);
    float* d_part = nullptr;
    float* d_bounds = nullptr;
    uint32_t *k0 = nullptr, *v0 = nullptr, *k1 = nullptr, *v1 = nullptr, *hist = nullptr;
    auto cleanup = [&]() {
        for (void* p : {(void*)d_part, (void*)d_bounds, (void*)k0, (void*)v0, (void*)k1, (void*)v1, (void*)hist}) (void)hipFree(p);
    };
    if (hipMalloc(&d_part, sizeof(float) * 6 * nparts) != hipSuccess || hipMalloc(&d_bounds, sizeof(float) * 8) != hipSuccess ||
        hipMalloc(&k0, 4ull * n) != hipSuccess || hipMalloc(&v0, 4ull * n) != hipSuccess ||
        hipMalloc(&k1, 4ull * n) != hipSuccess || hipMalloc(&v1, 4ull * n) != hipSuccess ||
        hipMalloc(&hist, 4ull * 256 * nblocks) != hipSuccess) {
        cleanup();
        return fail(ctx, GSRT_E_OOM, "lbvh_build: scratch allocation failed");
    }
    hipLaunchKernelGGL(k_bounds_partial, dim3(nparts), dim3(256), 0, st, n, sc->d_aabbs, d_part);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(256), 0, st, nparts, d_part, d_bounds);
    hipLaunchKernelGGL(k_morton, dim3((n + 255) / 256), dim3(256), 0, st, n, sc->d_aabbs, d_bounds, k0, v0);
    for (uint32_t shift = 0; shift < 32; shift += 8) {
        hipLaunchKernelGGL(k_radix_hist, dim3(nblocks), dim3(kSortBlock), 0, st, n, k0, shift, nblocks, hist);
        hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(1024), 0, st, 256 * nblocks, hist);
        hipLaunchKernelGGL(k_radix_scatter, dim3(nblocks), dim3(kSortBlock), 0, st, n, k0, v0, k1, v1, shift, nblocks,
                           hist);
        std::swap(k0, k1);
        std::swap(v0, v1);
    }
    hipError_t e = hipMemcpyAsync(sc->d_morton, k0, 4ull * n, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(sc->d_leaf_gid, v0, 4ull * n, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_karras, dim3((n - 1 + 255) / 256), dim3(256), 0, st, (int)n, sc->d_morton,
                           sc->d_leaf_gid, sc->d_nodes[0], sc->d_leaf_parent, sc->d_node_parent);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_gid_slot, dim3((n + 255) / 256), dim3(256), 0, st, n, sc->d_leaf_gid, sc->d_leaf_parent,
                           sc->d_gid_slot);
        e = hipGetLastError();
    }
    // level order for the fit: depth per node, histogram, scatter (hist reuses the radix histogram buffer)
    uint32_t* d_depth = k1;  // free after the sort
    uint32_t* d_hist = hist;
    std::vector<uint32_t> h_hist(kMaxLevels);
    if (e == hipSuccess) e = hipMemsetAsync(d_hist, 0, sizeof(uint32_t) * kMaxLevels, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_node_depth, dim3((n - 1 + 255) / 256), dim3(256), 0, st, n - 1, sc->d_node_parent, d_depth, d_hist);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h_hist.data(), d_hist, sizeof(uint32_t) * kMaxLevels, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    sc->level_off.clear();
    if (e == hipSuccess && h_hist[kMaxLevels - 1] == 0) {
        uint32_t levels = kMaxLevels;
        while (levels > 0 && h_hist[levels - 1] == 0) --levels;
        sc->level_off.assign(levels + 1, 0u);
        for (uint32_t d = 0; d < levels; ++d) sc->level_off[d + 1] = sc->level_off[d] + h_hist[d];
        if (!sc->d_level_nodes) e = hipMalloc(&sc->d_level_nodes, sizeof(uint32_t) * (n - 1));
        if (e == hipSuccess) e = hipMemcpyAsync(d_hist, sc->level_off.data(), sizeof(uint32_t) * levels, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_level_scatter, dim3((n - 1 + 255) / 256), dim3(256), 0, st, n - 1, d_depth, d_hist,
                               sc->d_level_nodes);
            e = hipGetLastError();
        }
        if (e != hipSuccess) sc->level_off.clear();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return fail(ctx, GSRT_E_DEVICE, std::string("lbvh_build: ") + hipGetErrorString(e));
    sc->root_ref = 0u;
    s = fit_all_slots(sc, st);
    if (s == GSRT_OK) sc->bvh_built = true;
    return s;
}

}  // namespace gsrt
