// gsrt_lbvh.hip -- on-device LBVH over the Gaussian AABBs (replaces the Embree rtcBuildBVH TLAS build,
// mesa-vulkan-sim/src/gallium/frontends/lavapipe/lvp_acceleration_structure.c:1329-1351, and the per-
// Gaussian BLAS of RayTracingInVulkan/src/Vulkan/RayTracing/Application.cpp:253-398).
//
//   1. centroid bounds         two-stage block reduction
//   2. 30-bit Morton codes     of AABB centroids quantised to 1024^3
//   3. LSD radix sort          8-bit digits, 4 passes: per-block histogram (+ the pass's digit totals) -> per-digit
//                              scan over the blocks (256 workgroups, each adds its digit's global base) -> stable
//                              scatter ranked by a wave-level multisplit (8 ballots per key)
//   4. Karras hierarchy        one thread per internal node (Karras 2012, duplicate codes tie-broken by index);
//                              it also records each node's leaf range
//   5. bottom-up AABB fit      one-wave workgroups over chunks of 256 sorted leaves, then spans of 16384 and of
//                              1048576 leaves, then the top; a node crossing a launch's workgroup range is queued
//                              for a later launch, so no device-wide fence is ever issued (see the kernels). The
//                              same launches refit new AABBs (config 5).
// Every scratch buffer is allocated with the scene (lbvh_alloc): a build is kernels and copies on one stream.
//
// Node boxes are exact unions of fp32 AABBs (min/max are exact), so any box that contains a leaf the
// exact slab test hits is itself hit: the BVH changes only the work, never the candidate set.
#include "gsrt_internal.hpp"
#include "gsrt_project.hpp"

namespace gsrt {

namespace {

constexpr int kSortBlock = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortBlock * kSortItems;
// bottom-up fit: one-wave workgroups (they run on the prep stream beside the render kernel, whose retiring waves
// free one wave's registers at a time) over sorted-leaf ranges of growing size
constexpr uint32_t kFitLeaves0 = 256;                 // k_fit_chunks: leaves per workgroup (4 per lane)
constexpr uint32_t kFitSpan1 = kFitLeaves0 * 64;      // k_fit_span level 1: 16384 leaves
constexpr uint32_t kFitSpan2 = kFitSpan1 * 64;        // level 2: 1048576 leaves
constexpr uint32_t kFitLevels = 2;

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

// per block and digit: the count (hist[d * nblocks + block]); the pass's digit totals accumulate in digit_total
__global__ __launch_bounds__(kSortBlock) void k_radix_hist(uint32_t n, const uint32_t* __restrict__ keys,
                                                           uint32_t shift, uint32_t nblocks,
                                                           uint32_t* __restrict__ hist, uint32_t* __restrict__ digit_total) {
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
    if (h[threadIdx.x]) atomicAdd(digit_total + threadIdx.x, h[threadIdx.x]);
}

// hist[d * nblocks + b] = number of keys with digit d in block b. One workgroup per digit d: the row becomes its
// exclusive scan over the blocks plus the digit's global base (the keys of smaller digits, from the totals that
// k_radix_hist accumulated), i.e. where block b's first key of digit d goes.
__global__ __launch_bounds__(256) void k_scan_digits(uint32_t nblocks, const uint32_t* __restrict__ digit_total,
                                                     uint32_t* __restrict__ hist) {
    __shared__ uint32_t part[256];
    const uint32_t d = blockIdx.x, t = threadIdx.x;
    part[t] = t < d ? digit_total[t] : 0u;  // the digit's base: a block reduction of the smaller digits' totals
    __syncthreads();
    for (uint32_t s2 = 128; s2 > 0; s2 >>= 1) {
        if (t < s2) part[t] += part[t + s2];
        __syncthreads();
    }
    const uint32_t base = part[0];
    __syncthreads();
    uint32_t* row = hist + (size_t)d * nblocks;
    const uint32_t per = (nblocks + 255) / 256, b0 = t * per, b1 = min(nblocks, b0 + per);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; ++b) sum += row[b];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {  // inclusive scan of the per-thread sums
        const uint32_t x = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = base + part[t] - sum;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t x = row[b];
        row[b] = run;
        run += x;
    }
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
                                                uint32_t* __restrict__ leaf_parent, uint32_t* __restrict__ node_parent,
                                                uint2* __restrict__ node_range) {
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
    node_range[i] = make_uint2((uint32_t)lo, (uint32_t)hi);
    if (i == 0) node_parent[0] = 0xFFFFFFFFu;  // root
}

// child box -> its slot in the parent node (left: floats 0-2 / 4-6, right: 8-10 / 12-14)
__device__ inline void put_slot(BvhNode* nodes, uint32_t p, uint32_t side, const float b[6]) {
    float* dst = reinterpret_cast<float*>(nodes + p) + (side ? 8 : 0);
    dst[0] = b[0]; dst[1] = b[1]; dst[2] = b[2];
    dst[4] = b[3]; dst[5] = b[4]; dst[6] = b[5];
}

// Bottom-up fit, on one stream; a node is fitted by the second of its two children's arrivals.
// 1. k_fit_chunks: one wave per chunk of kFitLeaves0 sorted leaves. A node whose leaf range lies in the chunk also
//    has its index there (a Karras node is an end of its range); its arrival counts are in LDS, preloaded with the
//    chunk's node ranges and parents.
// 2. k_fit_span<1>, k_fit_span<2>: one wave per span of kFitSpan1 / kFitSpan2 leaves, fed the nodes that crossed a
//    smaller range but lie in the span; their arrival counts are in HBM.
// 3. k_fit_top: one wave, fed the nodes that cross every span; it ends at the root.
// A child's box always goes into its parent's slot in HBM, and the second arrival reads the sibling's slot from
// there. Inside a workgroup the two arrivals are ordered by a workgroup-scope acquire/release count (one CU). A node
// that crosses its workgroup's range is counted device-wide and its second arrival queues it for the first later
// launch whose spans contain it: the launch boundary orders every store before the next launch, so no device-wide
// fence is ever issued. Counts go back to 0 once their node is fitted, and k_fit_top empties the queues.
//
// The workgroup-scope counts need every arrival of a workgroup on one CU: the fit kernels' workgroups are single
// waves (__launch_bounds__(64), launched with 64 threads in lbvh_fit), so this holds in any code-object mode,
// tgsplit included.
//
// queue layout (per slot): counts [nb1 level-1 spans][nb2 level-2 spans][top], then the level-1 queues (span b:
// entries [b kFitSpan1, b kFitSpan1 + min(kFitSpan1, n - b kFitSpan1)) -- a span holds fewer internal nodes than
// leaves, so n entries in all), the level-2 queues likewise (n entries), then the top queue (n entries)
struct FitQueues {
    uint32_t* count[kFitLevels + 1];  // per level 1, 2: per span; [kFitLevels]: the top's single count
    uint32_t* queue[kFitLevels + 1];
};
__host__ __device__ inline size_t fit_queue_words(uint32_t n) {
    const size_t nb1 = (n + kFitSpan1 - 1) / kFitSpan1, nb2 = (n + kFitSpan2 - 1) / kFitSpan2;
    return nb1 + nb2 + 1 + 3ull * n;
}
__device__ inline FitQueues fit_queues(uint32_t* q, uint32_t n) {
    const uint32_t nb1 = (n + kFitSpan1 - 1) / kFitSpan1, nb2 = (n + kFitSpan2 - 1) / kFitSpan2;
    FitQueues f;
    f.count[0] = q;
    f.count[1] = q + nb1;
    f.count[2] = q + nb1 + nb2;
    f.queue[0] = q + nb1 + nb2 + 1;
    f.queue[1] = f.queue[0] + n;  // span b's entries start at b kFitSpan1: every span before the last one is full
    f.queue[2] = f.queue[1] + n;
    return f;
}
// an arrival at node p (leaf range r) from outside the caller's range: the second one queues p for the first span
// level >= min_level (1-based; kFitLevels + 1 = the top) whose span contains r
__device__ inline void cross_arrival(uint32_t p, uint2 r, uint32_t* flags, const FitQueues& fq, uint32_t min_level) {
    if (atomicAdd(flags + p, 1u) != 1u) return;
    flags[p] = 0u;
    if (min_level <= 1 && r.x / kFitSpan1 == r.y / kFitSpan1) {
        const uint32_t b = r.x / kFitSpan1;
        fq.queue[0][(size_t)b * kFitSpan1 + atomicAdd(fq.count[0] + b, 1u)] = p;
    } else if (min_level <= 2 && r.x / kFitSpan2 == r.y / kFitSpan2) {
        const uint32_t b = r.x / kFitSpan2;
        fq.queue[1][(size_t)b * kFitSpan2 + atomicAdd(fq.count[1] + b, 1u)] = p;
    } else {
        fq.queue[2][atomicAdd(fq.count[2], 1u)] = p;
    }
}
__device__ inline void root_store(float* root_box, const float b[6]) {
#pragma unroll
    for (int t = 0; t < 6; ++t) root_box[t] = b[t];
}
__device__ inline void slot_union(const BvhNode* nodes, uint32_t p, float b[6]) {
    const float* c = reinterpret_cast<const float*>(nodes + p);
    b[0] = fminf(c[0], c[8]); b[1] = fminf(c[1], c[9]); b[2] = fminf(c[2], c[10]);
    b[3] = fmaxf(c[4], c[12]); b[4] = fmaxf(c[5], c[13]); b[5] = fmaxf(c[6], c[14]);
}

// BAND (lbvh_fit with a FitBand, a rank of a sharded frame): a chunk none of whose splats the rank can see (the
// in-band bitmap k_classify wrote: may_own_box per splat, exactly the rank projection's own reject test, so every one of
// them gets a +inf key) is not fitted and its AABBs are not even read. Its subtrees' slots in the nodes crossing the
// chunk get the empty box kEmptyLo / kEmptyHi, which every traversal rejects and every union ignores, and the crossings
// are counted as a climb would count them.
template <bool BAND>
__global__ __launch_bounds__(64) void k_fit_chunks(uint32_t n, const gsrt_aabb* __restrict__ aabbs,
                                                   const uint32_t* __restrict__ leaf_gid,
                                                   const uint32_t* __restrict__ leaf_parent,
                                                   const uint32_t* __restrict__ node_parent,
                                                   const uint2* __restrict__ node_range, BvhNode* nodes,
                                                   uint32_t* __restrict__ flags, uint32_t* queues,
                                                   float* __restrict__ root_box, const FitBand band) {
    __shared__ uint32_t lflag[kFitLeaves0];
    __shared__ uint2 lrange[kFitLeaves0];
    __shared__ uint32_t lparent[kFitLeaves0];
    const FitQueues fq = fit_queues(queues, n);
    const uint32_t c0 = blockIdx.x * kFitLeaves0, c1 = min(n, c0 + kFitLeaves0);
    const uint32_t ni_here = min(n - 1, c1) > c0 ? min(n - 1, c1) - c0 : 0u;  // internal nodes indexed in [c0, c1)
    for (uint32_t j = threadIdx.x; j < kFitLeaves0; j += 64) {
        lflag[j] = 0u;
        if (j < ni_here) {
            lrange[j] = node_range[c0 + j];
            lparent[j] = node_parent[c0 + j];
        }
    }
    __syncthreads();
    constexpr uint32_t kPer = kFitLeaves0 / 64;
    float box[kPer][6];
    uint32_t lp[kPer];
    uint32_t gid[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {  // every leaf's loads first (one latency for all)
        const uint32_t k = c0 + q * 64 + threadIdx.x;
        lp[q] = 0xFFFFFFFFu;
        gid[q] = 0u;
        if (k < c1) {
            gid[q] = leaf_gid[k];
            lp[q] = leaf_parent[k];
        }
    }
    if constexpr (BAND) {
        bool any = false;
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q)
            any = any || (lp[q] != 0xFFFFFFFFu && ((band.inband[gid[q] >> 5] >> (gid[q] & 31u)) & 1u));
        if (!__ballot(any)) {
            const float empty[6] = {kEmptyLo, kEmptyLo, kEmptyLo, kEmptyHi, kEmptyHi, kEmptyHi};
            // a leaf of the chunk whose parent crosses it
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) {
                if (lp[q] == 0xFFFFFFFFu) continue;
                const uint32_t p = lp[q] & ~kLeafBit, j = p - c0;
                const bool here = p >= c0 && j < ni_here;
                const uint2 r = here ? lrange[j] : make_uint2(0u, 0u);
                if (!here || r.x < c0 || r.y >= c1) {
                    put_slot(nodes, p, lp[q] >> 31, empty);
                    cross_arrival(p, here ? r : node_range[p], flags, fq, 1u);
                }
            }
            // an internal node inside the chunk whose parent crosses it (or that is the root)
            for (uint32_t j = threadIdx.x; j < ni_here; j += 64) {
                const uint2 r = lrange[j];
                if (r.x < c0 || r.y >= c1) continue;
                const uint32_t np = lparent[j];
                if (np == 0xFFFFFFFFu) {
                    root_store(root_box, empty);
                    continue;
                }
                const uint32_t p = np & ~kLeafBit, jp = p - c0;
                const bool here = p >= c0 && jp < ni_here;
                const uint2 rp = here ? lrange[jp] : make_uint2(0u, 0u);
                if (!here || rp.x < c0 || rp.y >= c1) {
                    put_slot(nodes, p, np >> 31, empty);
                    cross_arrival(p, here ? rp : node_range[p], flags, fq, 1u);
                }
            }
            return;
        }
    }
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (lp[q] == 0xFFFFFFFFu) continue;
        const gsrt_aabb a = aabbs[gid[q]];
        box[q][0] = a.min_x; box[q][1] = a.min_y; box[q][2] = a.min_z;
        box[q][3] = a.max_x; box[q][4] = a.max_y; box[q][5] = a.max_z;
    }
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
        if (lp[q] == 0xFFFFFFFFu) continue;
        float b[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) b[t] = box[q][t];
        uint32_t p = lp[q] & ~kLeafBit, side = lp[q] >> 31;
        for (;;) {
            put_slot(nodes, p, side, b);
            const uint32_t j = p - c0;
            const bool here = p >= c0 && j < ni_here;
            const uint2 r = here ? lrange[j] : make_uint2(0u, 0u);
            if (!here || r.x < c0 || r.y >= c1) {  // crosses the chunk: the other child comes from another one
                cross_arrival(p, here ? r : node_range[p], flags, fq, 1u);
                break;
            }
            // release: the slot stores before the count; acquire: the sibling's slot after it
            if (__hip_atomic_fetch_add(lflag + j, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) break;
            slot_union(nodes, p, b);
            const uint32_t np = lparent[j];  // parent | side << 31; all ones at the root
            if (np == 0xFFFFFFFFu) {
                root_store(root_box, b);
                break;
            }
            side = np >> 31;
            p = np & ~kLeafBit;
        }
    }
}

// Climb from fitted node p inside one workgroup whose leaf range is [r0, r1): unite p's two slots, write the box
// into the parent's slot, count the arrival (workgroup scope); the second arrival climbs on. A parent that crosses
// [r0, r1) goes to cross_arrival with the levels above this one.
__device__ inline void climb_from(uint32_t p, uint32_t r0, uint32_t r1, uint32_t next_level,
                                  const uint32_t* __restrict__ node_parent, const uint2* __restrict__ node_range,
                                  BvhNode* nodes, uint32_t* flags, const FitQueues& fq, float* root_box) {
    for (;;) {
        float b[6];
        slot_union(nodes, p, b);
        const uint32_t np = node_parent[p];
        if (np == 0xFFFFFFFFu) {
            root_store(root_box, b);
            return;
        }
        const uint32_t q = np & ~kLeafBit;
        put_slot(nodes, q, np >> 31, b);
        const uint2 r = node_range[q];
        if (r.x < r0 || r.y >= r1) {
            cross_arrival(q, r, flags, fq, next_level);
            return;
        }
        if (__hip_atomic_fetch_add(flags + q, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) != 1u) return;
        flags[q] = 0u;
        p = q;
    }
}

template <uint32_t LEVEL>
__global__ __launch_bounds__(64) void k_fit_span(uint32_t n, const uint32_t* __restrict__ node_parent,
                                                 const uint2* __restrict__ node_range, BvhNode* nodes,
                                                 uint32_t* __restrict__ flags, uint32_t* queues,
                                                 float* __restrict__ root_box) {
    constexpr uint32_t kSpan = LEVEL == 1 ? kFitSpan1 : kFitSpan2;
    const FitQueues fq = fit_queues(queues, n);
    const uint32_t b = blockIdx.x, count = fq.count[LEVEL - 1][b];
    const uint32_t r0 = b * kSpan, r1 = min(n, r0 + kSpan);
    const uint32_t* q = fq.queue[LEVEL - 1] + (size_t)b * kSpan;
    for (uint32_t t = threadIdx.x; t < count; t += 64)
        climb_from(q[t], r0, r1, LEVEL + 1, node_parent, node_range, nodes, flags, fq, root_box);
}

__global__ __launch_bounds__(64) void k_fit_top(uint32_t n, const uint32_t* __restrict__ node_parent,
                                                const uint2* __restrict__ node_range, BvhNode* nodes,
                                                uint32_t* __restrict__ flags, uint32_t* queues,
                                                float* __restrict__ root_box) {
    const FitQueues fq = fit_queues(queues, n);
    const uint32_t count = *fq.count[kFitLevels];
    for (uint32_t t = threadIdx.x; t < count; t += 64)
        climb_from(fq.queue[kFitLevels][t], 0u, n, kFitLevels + 1, node_parent, node_range, nodes, flags, fq, root_box);
    __syncthreads();
    // empty every queue for the next fit (the span kernels that read them have finished)
    const uint32_t words = (uint32_t)(fq.queue[0] - fq.count[0]);
    for (uint32_t t = threadIdx.x; t < words; t += 64) fq.count[0][t] = 0u;
}

// gid -> (parent node, side) of its leaf slot: where the projection kernel writes the leaf's sort key
__global__ __launch_bounds__(256) void k_gid_slot(uint32_t n, const uint32_t* __restrict__ leaf_gid,
                                                  const uint32_t* __restrict__ leaf_parent, uint32_t* __restrict__ slot) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k < n) slot[leaf_gid[k]] = leaf_parent[k];
}

}  // namespace

// every buffer of the build and of the fits, allocated with the scene (a build or refit then allocates nothing)
gsrt_status lbvh_alloc(gsrt_scene* sc) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n ? sc->n : 1u;
    const uint32_t ni = n > 1 ? n - 1 : 1;
    const uint32_t nblocks = (n + kSortTile - 1) / kSortTile;
    const uint32_t nparts = std::min<uint32_t>(1024u, (n + 255) / 256);
    for (uint32_t b = 0; b < kSlots; ++b) {
        if (!sc->d_nodes[b]) GSRT_HIP(ctx, hipMalloc(&sc->d_nodes[b], sizeof(BvhNode) * ni));
        if (!sc->d_root_box[b]) GSRT_HIP(ctx, hipMalloc(&sc->d_root_box[b], sizeof(float) * 8));
        if (!sc->d_fit_flags[b]) {  // zero once: every fit leaves them at zero
            GSRT_HIP(ctx, hipMalloc(&sc->d_fit_flags[b], sizeof(uint32_t) * ni));
            GSRT_HIP(ctx, hipMemsetAsync(sc->d_fit_flags[b], 0, sizeof(uint32_t) * ni, ctx->stream));
        }
        if (!sc->d_fit_queue[b]) {  // counts (zero between fits) and queues
            GSRT_HIP(ctx, hipMalloc(&sc->d_fit_queue[b], sizeof(uint32_t) * fit_queue_words(n)));
            GSRT_HIP(ctx, hipMemsetAsync(sc->d_fit_queue[b], 0, sizeof(uint32_t) * fit_queue_words(n), ctx->stream));
        }
    }
    if (!sc->d_leaf_parent) GSRT_HIP(ctx, hipMalloc(&sc->d_leaf_parent, sizeof(uint32_t) * n));
    if (!sc->d_node_parent) GSRT_HIP(ctx, hipMalloc(&sc->d_node_parent, sizeof(uint32_t) * ni));
    if (!sc->d_node_range) GSRT_HIP(ctx, hipMalloc(&sc->d_node_range, sizeof(uint2) * ni));
    if (!sc->d_gid_slot) GSRT_HIP(ctx, hipMalloc(&sc->d_gid_slot, sizeof(uint32_t) * n));
    if (!sc->d_leaf_gid) GSRT_HIP(ctx, hipMalloc(&sc->d_leaf_gid, sizeof(uint32_t) * n));
    if (!sc->d_morton) GSRT_HIP(ctx, hipMalloc(&sc->d_morton, sizeof(uint32_t) * n));
    // sort scratch: ping-pong keys / values (the final pass lands in d_morton / d_leaf_gid), block histograms,
    // digit totals, partial and final centroid bounds
    if (!sc->d_sort) {
        const size_t words = 2ull * n + 256ull * nblocks + 4 * 256 + 6ull * nparts + 8;
        GSRT_HIP(ctx, hipMalloc(&sc->d_sort, sizeof(uint32_t) * words));
    }
    return GSRT_OK;
}

gsrt_status lbvh_fit(gsrt_scene* sc, uint32_t slot, hipStream_t st, const FitBand* band) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n;
    BvhNode* nodes = sc->d_nodes[slot];
    float* root_box = sc->d_root_box[slot];
    if (n == 0) return GSRT_OK;
    if (n == 1) {  // the root is the leaf: its AABB is the root box (same float order)
        GSRT_HIP(ctx, hipMemcpyAsync(root_box, sc->d_aabbs, sizeof(float) * 6, hipMemcpyDeviceToDevice, st));
        return GSRT_OK;
    }
    // the slot's own counts and queues: the two slots' fits may run on two streams at once (slot streams)
    uint32_t* q = sc->d_fit_queue[slot];
    uint32_t* flags = sc->d_fit_flags[slot];
    const dim3 g0((n + kFitLeaves0 - 1) / kFitLeaves0);
    if (band)
        hipLaunchKernelGGL(k_fit_chunks<true>, g0, dim3(64), 0, st, n, sc->d_aabbs, sc->d_leaf_gid, sc->d_leaf_parent,
                           sc->d_node_parent, sc->d_node_range, nodes, flags, q, root_box, *band);
    else
        hipLaunchKernelGGL(k_fit_chunks<false>, g0, dim3(64), 0, st, n, sc->d_aabbs, sc->d_leaf_gid, sc->d_leaf_parent,
                           sc->d_node_parent, sc->d_node_range, nodes, flags, q, root_box, FitBand{});
    if (n > kFitLeaves0) {
        hipLaunchKernelGGL(k_fit_span<1>, dim3((n + kFitSpan1 - 1) / kFitSpan1), dim3(64), 0, st, n, sc->d_node_parent,
                           sc->d_node_range, nodes, flags, q, root_box);
        hipLaunchKernelGGL(k_fit_span<2>, dim3((n + kFitSpan2 - 1) / kFitSpan2), dim3(64), 0, st, n, sc->d_node_parent,
                           sc->d_node_range, nodes, flags, q, root_box);
        hipLaunchKernelGGL(k_fit_top, dim3(1), dim3(64), 0, st, n, sc->d_node_parent, sc->d_node_range, nodes, flags, q,
                           root_box);
    }
    GSRT_HIP(ctx, hipGetLastError());
    return GSRT_OK;  // asynchronous: the render kernels read the root box from d_root_box[slot]
}

gsrt_status lbvh_fit_if_stale(gsrt_scene* sc, uint32_t slot, hipStream_t st, bool need_aabbs, const FitBand* band,
                              const FitBandKey* band_key) {
    if (need_aabbs || !band_key) band = nullptr;
    FitBandKey key{};
    if (band) key = *band_key;
    const bool geom_ok = sc->slot_geom[slot] == sc->geom_version && !(need_aabbs && sc->slot_leaf_fp[slot]);
    // a full fit serves every frame; a restricted one only its own band and camera
    if (geom_ok && (!sc->slot_banded[slot] ||
                    (band && std::memcmp(&key, &sc->slot_band_key[slot], sizeof key) == 0)))
        return GSRT_OK;
    gsrt_status s = lbvh_fit(sc, slot, st, band);
    if (s == GSRT_OK) {
        sc->slot_geom[slot] = sc->geom_version;
        sc->slot_leaf_fp[slot] = false;  // the fit wrote every leaf's AABB back (a restricted one: every one it can see)
        sc->slot_banded[slot] = band != nullptr;
        if (band) sc->slot_band_key[slot] = key;
    }
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
    for (uint32_t b = 0; b < kSlots; ++b) {
        sc->slot_geom[b] = sc->geom_version;
        sc->slot_leaf_fp[b] = false;
        sc->slot_banded[b] = false;
        sc->slot_inband_ver[b] = 0;  // (conservatively: a build may follow AABBs written by the caller's own means)
    }
    // the slots' node keys are the copied (or stale) ones: k_project's keyed bitmaps start over (all ones)
    for (uint32_t b = 0; b < kSlots; ++b)
        if (sc->d_keyed[b]) GSRT_HIP(ctx, hipMemsetAsync(sc->d_keyed[b], 0xFF, sizeof(uint32_t) * ((sc->n + 31) / 32 + 1), st));
    return GSRT_OK;
}

// The whole build on ctx->stream: no allocation, no host round trip until the final wait (gsrt_build_bvh reports
// errors synchronously).
gsrt_status lbvh_build(gsrt_scene* sc) {
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t n = sc->n;
    hipStream_t st = ctx->stream;
    sc->bvh_built = false;
    if (n == 0) { sc->bvh_built = true; return GSRT_OK; }
    gsrt_status s = lbvh_alloc(sc);  // a no-op unless the scene was created without it
    if (s != GSRT_OK) return s;
    if (sc->d_flags) GSRT_HIP(ctx, hipMemsetAsync(sc->d_flags, 0, sizeof(uint32_t) * 4, st));  // the depth-cull guard
    if (n == 1) {
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_leaf_gid, 0, 4, st));
        GSRT_HIP(ctx, hipMemsetAsync(sc->d_morton, 0, 4, st));
        sc->root_ref = kLeafBit | 0u;
        s = fit_all_slots(sc, st);
        if (s == GSRT_OK) s = hipStreamSynchronize(st) == hipSuccess ? GSRT_OK : fail(ctx, GSRT_E_DEVICE, "lbvh_build");
        if (s == GSRT_OK) sc->bvh_built = true;
        return s;
    }
    const uint32_t nblocks = (n + kSortTile - 1) / kSortTile;
    const uint32_t nparts = std::min<uint32_t>(1024u, (n + 255) / 256);
    // scratch layout (lbvh_alloc): k1 | v1 | hist | digit totals | partial bounds | bounds; the sort starts in
    // d_morton / d_leaf_gid and, after an even number of passes, ends there
    uint32_t* k0 = sc->d_morton;
    uint32_t* v0 = sc->d_leaf_gid;
    uint32_t* k1 = sc->d_sort;
    uint32_t* v1 = k1 + n;
    uint32_t* hist = v1 + n;
    uint32_t* digit_total = hist + 256ull * nblocks;
    float* d_part = reinterpret_cast<float*>(digit_total + 4 * 256);
    float* d_bounds = d_part + 6ull * nparts;
    GSRT_HIP(ctx, hipMemsetAsync(digit_total, 0, sizeof(uint32_t) * 4 * 256, st));
    hipLaunchKernelGGL(k_bounds_partial, dim3(nparts), dim3(256), 0, st, n, sc->d_aabbs, d_part);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(256), 0, st, nparts, d_part, d_bounds);
    hipLaunchKernelGGL(k_morton, dim3((n + 255) / 256), dim3(256), 0, st, n, sc->d_aabbs, d_bounds, k0, v0);
    for (uint32_t pass = 0; pass < 4; ++pass) {
        const uint32_t shift = 8 * pass;
        hipLaunchKernelGGL(k_radix_hist, dim3(nblocks), dim3(kSortBlock), 0, st, n, k0, shift, nblocks, hist,
                           digit_total + 256 * pass);
        hipLaunchKernelGGL(k_scan_digits, dim3(256), dim3(256), 0, st, nblocks, digit_total + 256 * pass, hist);
        hipLaunchKernelGGL(k_radix_scatter, dim3(nblocks), dim3(kSortBlock), 0, st, n, k0, v0, k1, v1, shift, nblocks,
                           hist);
        std::swap(k0, k1);
        std::swap(v0, v1);
    }
    // four passes: the sorted codes and ids are back in d_morton / d_leaf_gid
    hipLaunchKernelGGL(k_karras, dim3((n - 1 + 255) / 256), dim3(256), 0, st, (int)n, sc->d_morton, sc->d_leaf_gid,
                       sc->d_nodes[0], sc->d_leaf_parent, sc->d_node_parent, sc->d_node_range);
    hipLaunchKernelGGL(k_gid_slot, dim3((n + 255) / 256), dim3(256), 0, st, n, sc->d_leaf_gid, sc->d_leaf_parent,
                       sc->d_gid_slot);
    GSRT_HIP(ctx, hipGetLastError());
    sc->root_ref = 0u;
    s = fit_all_slots(sc, st);
    if (s != GSRT_OK) return s;
    if (hipError_t e = hipStreamSynchronize(st); e != hipSuccess)
        return fail(ctx, GSRT_E_DEVICE, std::string("lbvh_build: ") + hipGetErrorString(e));
    sc->bvh_built = true;
    return GSRT_OK;
}

}  // namespace gsrt
