/*
 * gsrt_test.h -- test and measurement hooks of libgsrt, beside the drop-in ABI of gsrt.h.
 *
 * Nothing here is part of the reference boundary: a reference-side caller links gsrt.h alone. These
 * entry points serve the test suite, the bench and multi-process transports other than RCCL: diagnostic counters,
 * host mirrors of the sharded layout and of the partition rule, emulated gathers on one device, and the synthetic
 * clouds of SURVEY.md §8d. They are exported by the same library.
 */
#ifndef GSRT_TEST_H
#define GSRT_TEST_H

#include "gsrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the copy of the ExpLUT in HBM that the kernels read (uploaded by gsrt_create; gsrt_exp_lut is the host's) */
gsrt_status gsrt_debug_exp_lut(gsrt_ctx* ctx, float out[512]);
/* diagnostic: the raw 16-word counter block of the last render */
gsrt_status gsrt_debug_counters(gsrt_ctx* ctx, uint64_t out[16]);
/* words 16..31 of the same block (diagnostic builds: shading-loop wave-candidate counts) */
gsrt_status gsrt_debug_counters_hi(gsrt_ctx* ctx, uint64_t out[16]);

/* test hooks for the partition: with gsrt_debug_share_costs(ctx, 1) every sharded COR frame stores its tiles' costs
 * (the profile frames' measurement, without the all-reduce); gsrt_debug_row_profile sums the last such frame's per
 * tile row of the frame (tiles_y entries, zero outside this rank's band). A rank share's own cost profile, which the
 * automatic balancing of an N-rank job all-reduces. */
gsrt_status gsrt_debug_share_costs(gsrt_ctx* ctx, int on);
gsrt_status gsrt_debug_row_profile(gsrt_ctx* ctx, uint32_t* rows, uint32_t cap, uint32_t* n);
/* the render-unit deal of a rank share (launch_render, host logic): units (a multiple of 8) with costs cost[units], ties
 * broken in the order centre[] lists them (a permutation); perm[k * 8 + x] = XCD x's k-th unit. Longest first, each unit
 * to the XCD with the least cost so far among those holding fewer than units / 8 */
gsrt_status gsrt_deal_units(const double* cost, const uint32_t* centre, uint32_t units, uint32_t* perm);
/* the context's streams (hipStream_t) in creation order: render, prep H 0, prep L 0, prep H 1, prep L 1, update, comm
 * (NULL before gsrt_comm_init); *n = 7. For the hardware-queue map (profiles/probes/gsrt_queue_map.py) */
gsrt_status gsrt_debug_streams(gsrt_ctx* ctx, void* out[8], uint32_t* n);
/* test hook: the first `floats` floats of rank 0's gather buffer after the last sharded frame (rank-major packed
 * blocks, as ncclGather leaves them; on a GSRT_DEBUG_COMM_LOOPBACK communicator block 0 is this process's share) */
gsrt_status gsrt_debug_gathered(gsrt_ctx* ctx, float* out, size_t floats);

/* Host mirror of the sharded layout (the same tile mappings the kernels use, no device): pack `rank`'s tiles
 * of a W x H RGBA32F frame into the packed layout its sharded render writes (packed stride x tile_w*tile_h x 4
 * floats, unused slots zero), and unpack all ranks' gathered blocks (nranks x stride x tile_w*tile_h x 4, rank-
 * major, as ncclGather leaves them) into a W x H frame as k_unpack does. bands: the partition, NULL = the even one.
 * For multi-process transports other than RCCL, and for tests. */
gsrt_status gsrt_tile_pack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const uint32_t* bands,
                                const float* rgba, float* packed);
gsrt_status gsrt_tile_unpack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands,
                                  const float* gathered, float* rgba_out);
/* test hook: every rank's packed tiles rendered on this device into the gather layout, then unpacked by the
 * same kernel rank 0 uses after ncclGather (the transport is the only part skipped). bands: NULL = even. */
gsrt_status gsrt_render_sharded_emulated(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                         const uint32_t* bands, float* rgba_out);

/* Host mirror of a rank's GSRT_FLAG_OUT_DUMP8 block (no device), for multi-process transports other than RCCL and
 * for tests. gsrt_dump8_layout: out = {words per rank block, code words (stride x tile_w*tile_h, padded to 4),
 * escape capacity}; the list header (count in the first word) is at word out[1], its entries {local pixel index,
 * r, g, b bits} follow it. gsrt_tile_pack_dump8_host writes `rank`'s block of a W x H RGBA32F frame as its sharded
 * render does (unused slots zero, escapes in local pixel order where the kernel's are in arrival order); more
 * escapes than the capacity return GSRT_E_STATE with the header holding the full count, as on the device.
 * gsrt_tile_unpack_dump8_host turns nranks gathered blocks (rank-major) into W x H codes and the escapes in pixel
 * order (at most cap written, n_esc = all), GSRT_E_STATE when a block's list overflowed. COR modes only. */
gsrt_status gsrt_dump8_layout(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, uint64_t out[3]);
gsrt_status gsrt_tile_pack_dump8_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const uint32_t* bands,
                                      const float* rgba, uint32_t* block);
gsrt_status gsrt_tile_unpack_dump8_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands,
                                        const uint32_t* gathered, uint32_t* codes, gsrt_dump8_escape* esc,
                                        uint32_t cap, uint32_t* n_esc);
/* test hook: gsrt_render_sharded_emulated with GSRT_FLAG_OUT_DUMP8 blocks (mode must carry the flag) */
gsrt_status gsrt_render_sharded_emulated_dump8(gsrt_scene* scene, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                               const uint32_t* bands, uint32_t* codes, gsrt_dump8_escape* esc,
                                               uint32_t cap, uint32_t* n_esc);

/* ---- synthetic inputs (std::mt19937(seed) + uniform_real_distribution<float>) ---- */
gsrt_status gsrt_synth_cloud(uint32_t kind, uint32_t n, uint32_t seed, int with_sh, float* center,
                             float* rot_rxyz, float* scale, float* opacity, float* sh);

/* The partition rule of a profile frame as every rank applies it (host-only, deterministic), for multi-process
 * transports and tests. gsrt_partition_hash: the hash a rank's profile carries for `bands` (FNV-1a over the tile grid,
 * the bands, the packed stride and whether the bands are pinned). gsrt_decide_bands: from the all-reduced profile
 * (tiles_y row costs, max over the ranks, then max(h) and max(~h) of the ranks' hashes) and this rank's hash, the
 * bands of the next frames (nranks + 1 into out): GSRT_E_COMM when the ranks' hashes differ; pinned bands are kept;
 * otherwise gsrt_tile_bands' cut of the profile when it lowers the heaviest band's cost by 2 %, else `bands`. */
gsrt_status gsrt_partition_hash(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, int pinned,
                                uint32_t* hash);
gsrt_status gsrt_decide_bands(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, int pinned,
                              const uint32_t* profile, uint32_t my_hash, uint32_t* out);

/* ---- test switches ------------------------------------------------------------------------------
 * Environment variables the library reads for its tests and measurements. Each forces a path the library otherwise
 * chooses itself; results are unchanged (the tests hold them bit-equal to the default path). Production leaves them
 * unset.
 *   GSRT_DEBUG_RANK_OF=N[:r]      on a loopback communicator, sharded COR frames run rank r's (default 0) share of an
 *                                 N-rank frame through the real exchange path (rank-share measurements)
 *   GSRT_DEBUG_COMM_LOOPBACK=1    gsrt_comm_init with one rank still builds an RCCL communicator and takes the
 *                                 exchange path (packed render, ncclGather, k_unpack on the comm stream)
 *   GSRT_DEBUG_SLOT_STREAMS=0|1   slot streams never / always (default: chosen per frame from render times)
 *   GSRT_DEBUG_LAZY_STREAMS=1     the update and comm streams created when first used, at the default priority
 *   GSRT_DEBUG_DEAL=0             a share's render units dealt centre-out (default: by the last whole frame's tile costs)
 *   GSRT_DEBUG_SLOTS=2            two frame slots in rotation (default three; two on slot streams)
 *   GSRT_DEBUG_PREP_PRIORITY=0|1|2  prep streams at the lowest / highest priority, or switching every frame
 *   GSRT_DEBUG_GROUP_TILES=2|4    COR tile groups of 2x2 or 4x4 tiles (default: by the rank's group count)
 *   GSRT_DEBUG_NO_GROUPS=1        no group lists: every tile traverses the BVH itself
 *   GSRT_DEBUG_NO_FRONTIER=1      group traversals start at the root (no super-group frontiers)
 *   GSRT_DEBUG_NO_LEAF_FP=1       COR traversals test leaf AABBs and cull footprints afterwards (no footprint boxes in
 *                                 the BVH leaves)
 *   GSRT_DEBUG_PROJECT_ALL=1      a rank of a sharded frame projects every splat (no band culling)
 *   GSRT_DEBUG_STACK_LIMIT=n      the traversals' LDS node stack cut to n entries (exercises the DFS restart) */

#ifdef __cplusplus
}
#endif
#endif /* GSRT_TEST_H */
