// gsrt_comm.cpp -- multi-GPU tile sharding.
//
// One process per GPU. The scene and its LBVH are replicated (each rank builds its own). The frame's tile rows are
// cut into one contiguous band per rank (Bands, gsrt_device.hpp), each rank renders its band's tiles into a packed
// buffer, and one ncclGather over xGMI brings the packed tiles to rank 0, which unpacks them into its framebuffer.
// The gather is the only exchange of the image; rendering needs no communication. It runs on the comm stream from one
// of two packed buffers into one of two gather buffers, followed there by rank 0's unpack, so frame k's exchange
// overlaps frame k+1's rendering.
//
// Balancing: a band is contiguous, so a rank's projection and group lists see only its part of the view, but the
// shading cost per row varies over the frame. Every kProfileEvery-th sharded frame the render kernel adds each tile's
// shading cost into a per-row profile; one ncclAllReduce (max: every row has one contributor) gives every rank the
// whole frame's profile, and kProfileEvery frames later every rank cuts new bands from it with the same deterministic
// rule (balance_bands, rank 0 weighted for its gather and unpack), adopting them only when they lower the heaviest
// band by kAdoptGain. The profile carries a hash of the partition each rank rendered: ranks that disagree fail with
// GSRT_E_COMM instead of gathering mismatched layouts.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gsrt_internal.hpp"

namespace {
constexpr uint32_t kProfileEvery = 8;    // sharded frames between cost profiles (and between partition changes)
constexpr double kAdoptGain = 0.02;      // new bands must lower the heaviest band's cost by this fraction
constexpr size_t kNoHeader = ~size_t(0);

// A GSRT_FLAG_OUT_DUMP8 block (32-bit words): stride x tile pixels code words (padded to 16 bytes), then the escape
// list: a uint4 header (count in .x) and cap uint4 entries {local pixel index, r, g, b bits}
struct Dump8Layout {
    size_t codes = 0, block = 0;
    uint32_t cap = 0;
};
Dump8Layout dump8_layout(uint32_t per_rank, uint32_t tile_px) {
    Dump8Layout L;
    const size_t px = (size_t)per_rank * tile_px;
    L.codes = (px + 3) & ~size_t(3);
    L.cap = (uint32_t)std::max<size_t>(256, px / 64);
    L.block = L.codes + 4 + 4ull * L.cap;
    return L;
}
}

struct gsrt_comm_state {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    hipStream_t cstream = nullptr;       // the gather, the profile all-reduce and rank 0's unpack: the comm stream
    hipEvent_t rendered[2] = {nullptr, nullptr};  // packed[p] written (compute stream)
    hipEvent_t gathered[2] = {nullptr, nullptr};  // packed[p] sent, gbuf[p] received (comm stream): packed[p] is free
    hipEvent_t unpacked[2] = {nullptr, nullptr};  // gbuf[p] unpacked (cstream): free for the next gather into it
    bool unpack_pending[2] = {false, false};
    float* packed[2] = {nullptr, nullptr};
    size_t packed_floats = 0;
    float* gbuf[2] = {nullptr, nullptr};  // rank 0: every rank's packed blocks, rank-major (ncclGather's layout)
    size_t gbuf_floats = 0;
    uint32_t last_p = 0;                 // the parity of the last sharded frame (gsrt_debug_gathered)
    // d_fb is written on two streams: rank 0's unpack (comm stream) and whole frames rendered on the render stream
    // (gsrt_render_async). Each side waits for the other's last write (and for what the caller queued after it on
    // that stream, e.g. a copy of the image) before it writes d_fb again.
    bool fb_on_comm = false;             // the comm stream wrote d_fb since the render stream last waited for it
    bool fb_on_render = false;           // the render stream wrote d_fb since the comm stream last waited for it
    hipEvent_t ev_fb = nullptr;          // the hop between the two
    float* inbound = nullptr;            // rank-share emulation of rank 0 (GSRT_DEBUG_RANK_OF=N): the other blocks' source
    size_t inbound_floats = 0;
    uint32_t parity = 0;
    // the partition (see the file comment)
    std::vector<uint32_t> bands;         // the current bands (nranks + 1 row boundaries), empty: even rows
    uint32_t bands_key[4] = {0, 0, 0, 0};  // {tiles_y, nranks, tile height, root weight bits} the bands are for
    bool pinned = false;                 // gsrt_set_bands: a fixed partition, no balancing
    std::vector<uint32_t> last_bands;    // the bands of the last sharded frame (gsrt_last_bands)
    uint32_t frames = 0;                 // sharded frames so far: the profile schedule, the same on every rank
    uint32_t* d_tcost = nullptr;         // the profile frame's tile costs (local order), k_render_cor
    uint32_t tcost_cap = 0;
    uint32_t* d_prof = nullptr;          // the profile frame's row costs + 2 hash words (zeroed after each all-reduce)
    uint32_t* d_prof_red = nullptr;      // the all-reduced profile
    uint32_t* h_prof[2] = {nullptr, nullptr};  // page-locked copies of it (two profiles in flight at most)
    uint32_t* h_hash[2] = {nullptr, nullptr};  // page-locked source of the hash words
    hipEvent_t ev_prof[2] = {nullptr, nullptr};
    bool prof_pending[2] = {false, false};
    uint32_t prof_key[2][4] = {};        // the bands_key each profile was taken under
    uint32_t prof_hash[2] = {0, 0};      // this rank's partition hash of each profile
    uint32_t prof_rows = 0;              // d_prof capacity in rows
    bool comm_error = false;             // the ranks' partitions differed (sticky: GSRT_E_COMM)
    // test hook gsrt_debug_share_costs: every sharded COR frame stores its tiles' costs (d_tcost) for
    // gsrt_debug_row_profile, which sums them per row of the frame (tiles_x, rows, band [row0, row1))
    bool share_costs = false;
    uint32_t sc_tiles_x = 0, sc_rows = 0, sc_row0 = 0, sc_row1 = 0;
    // GSRT_FLAG_OUT_DUMP8 frames
    size_t esc_at[2] = {kNoHeader, kNoHeader};  // the word offset in packed[p] of a zeroed escape header
    float4* d_accum[2] = {nullptr, nullptr};    // spp > 64: the running sums of packed[p]'s frame
    size_t accum_px = 0;
    uint32_t* d_codes = nullptr;         // rank 0: the last dump8 frame's code framebuffer (W x H)
    size_t codes_px = 0;
    bool d8_last = false, d8_root = false;  // the last sharded frame was a dump8 frame (on rank 0)
    gsrt::RenderPlan d8_plan;            // its partition and tiles
    Dump8Layout d8_layout;
    uint32_t d8_w = 0, d8_h = 0;
};

using gsrt::fail;

namespace gsrt {
// GSRT_DEBUG_RANK_OF=N or N:r (measurement knob, read on a loopback communicator): one GPU runs rank r's (default 0)
// share of an N-rank sharded COR frame through the real exchange path (the packed render, ncclGather on the comm
// stream), so the share's period is what a rank of an N-GPU job pays. For r = 0 the root's receive side is stood in
// for as well: the N-1 other ranks' blocks are copied into the gather buffer on the comm stream (the HBM writes and
// CU time of RCCL's receive; the xGMI link time is modelled, not emulated) and k_unpack scatters all
// N blocks into the framebuffer. The image of such a frame is not a picture.
bool debug_rank_of(uint32_t mode, uint32_t& nranks, uint32_t& rank) {
    const char* e = std::getenv("GSRT_DEBUG_RANK_OF");
    if (!e || (mode & 0xffu) != GSRT_MODE_COR || (mode & GSRT_FLAG_STATS)) return false;
    char* rest = nullptr;
    const long nr = std::strtol(e, &rest, 10);
    const long r = (rest && *rest == ':') ? std::strtol(rest + 1, nullptr, 10) : 0;
    if (nr < 2 || nr > 64 || r < 0 || r >= nr) return false;
    nranks = (uint32_t)nr;
    rank = (uint32_t)r;
    return true;
}
}  // namespace gsrt

extern "C" {

void gsrt_comm_destroy_internal(gsrt_ctx* ctx) {
    if (!ctx || !ctx->comm) return;
    gsrt_comm_state* c = ctx->comm;
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (int p = 0; p < 2; ++p) {
        if (c->rendered[p]) (void)hipEventDestroy(c->rendered[p]);
        if (c->gathered[p]) (void)hipEventDestroy(c->gathered[p]);
        if (c->unpacked[p]) (void)hipEventDestroy(c->unpacked[p]);
        if (c->ev_prof[p]) (void)hipEventDestroy(c->ev_prof[p]);
        (void)hipFree(c->packed[p]);
        (void)hipFree(c->gbuf[p]);
        (void)hipFree(c->d_accum[p]);
        (void)hipHostFree(c->h_prof[p]);
        (void)hipHostFree(c->h_hash[p]);
    }
    (void)hipFree(c->inbound);
    (void)hipFree(c->d_codes);
    (void)hipFree(c->d_prof);
    (void)hipFree(c->d_tcost);
    (void)hipFree(c->d_prof_red);
    if (c->ev_fb) (void)hipEventDestroy(c->ev_fb);
    if (c->cstream && c->cstream != ctx->cstream) (void)hipStreamDestroy(c->cstream);  // (a lazily created one)
    delete c;
    ctx->comm = nullptr;
}

// the comm stream of ctx (nullptr without a communicator)
hipStream_t gsrt_comm_stream_internal(gsrt_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->cstream : nullptr; }

// wait for the gather and unpack streams (gsrt_synchronize, reallocations)
gsrt_status gsrt_comm_sync_internal(gsrt_ctx* ctx) {
    if (!ctx || !ctx->comm) return GSRT_OK;
    if (ctx->comm->cstream) GSRT_HIP(ctx, hipStreamSynchronize(ctx->comm->cstream));
    return GSRT_OK;
}

// a whole frame is about to write d_fb on the render stream: wait for the comm stream's unpacks (and whatever was
// queued after them there), then remember that the next unpack must wait for this write
gsrt_status gsrt_comm_fb_render_write(gsrt_ctx* ctx) {
    gsrt_comm_state* c = ctx ? ctx->comm : nullptr;
    if (!c || !c->cstream) return GSRT_OK;
    if (c->fb_on_comm) {
        GSRT_HIP(ctx, hipEventRecord(c->ev_fb, c->cstream));
        GSRT_HIP(ctx, hipStreamWaitEvent(ctx->stream, c->ev_fb, 0));
        c->fb_on_comm = false;
    }
    c->fb_on_render = true;
    return GSRT_OK;
}

void* gsrt_comm_stream(gsrt_ctx* ctx) { return gsrt_comm_stream_internal(ctx); }

gsrt_status gsrt_comm_size(gsrt_ctx* ctx, int* nranks, int* rank) {
    if (!ctx || !nranks) return GSRT_E_ARG;
    int n = 1, r = 0;
    if (ctx->comm) {
        n = ctx->comm->nranks;
        r = ctx->comm->rank;
        if (ctx->comm->comm) {  // the communicator's own view (a loopback communicator has one rank)
            if (ncclCommCount(ctx->comm->comm, &n) != ncclSuccess || ncclCommUserRank(ctx->comm->comm, &r) != ncclSuccess)
                return fail(ctx, GSRT_E_COMM, "ncclCommCount / ncclCommUserRank failed");
        }
    }
    *nranks = n;
    if (rank) *rank = r;
    return GSRT_OK;
}

gsrt_status gsrt_timing_read_exchange(gsrt_ctx* ctx, float* exchange_ms, uint32_t cap, uint32_t* nframes) {
    if (!ctx || !exchange_ms) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (gsrt_status s = gsrt_comm_sync_internal(ctx); s != GSRT_OK) return s;
    const uint32_t n = ctx->timing_n < cap ? ctx->timing_n : cap;
    for (uint32_t i = 0; i < n; ++i) {
        float x = 0.f;
        const size_t e = (size_t)gsrt::kTimingEvents * i;
        if (ctx->timing_ex[i]) GSRT_HIP(ctx, hipEventElapsedTime(&x, ctx->events[e + 4], ctx->events[e + 5]));
        exchange_ms[i] = x;
    }
    if (nframes) *nframes = n;
    return GSRT_OK;
}

gsrt_status gsrt_debug_gathered(gsrt_ctx* ctx, float* out, size_t floats) {
    if (!ctx || !out) return GSRT_E_ARG;
    gsrt_comm_state* c = ctx->comm;
    if (!c || !c->gbuf[c->last_p] || floats > c->gbuf_floats) return fail(ctx, GSRT_E_STATE, "no gather buffer of that size");
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (gsrt_status s = gsrt_comm_sync_internal(ctx); s != GSRT_OK) return s;
    GSRT_HIP(ctx, hipMemcpy(out, c->gbuf[c->last_p], sizeof(float) * floats, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

gsrt_status gsrt_comm_unique_id(uint8_t out[128]) {
    if (!out) return GSRT_E_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GSRT_E_COMM;
    std::memcpy(out, &id, sizeof id);
    return GSRT_OK;
}

gsrt_status gsrt_comm_init(gsrt_ctx* ctx, const uint8_t id[128], int nranks, int rank) {
    // the partition holds at most kMaxRanks bands (Bands): more ranks would silently share rank 0's band
    if (!ctx || !id || nranks < 1 || nranks > (int)gsrt::kMaxRanks || rank < 0 || rank >= nranks) return GSRT_E_ARG;
    (void)hipSetDevice(ctx->device);
    gsrt_comm_destroy_internal(ctx);
    auto* st = new gsrt_comm_state();
    st->nranks = nranks;
    st->rank = rank;
    // GSRT_DEBUG_COMM_LOOPBACK=1 (test knob): a one-rank job still takes the exchange path -- a one-rank RCCL
    // communicator, the packed buffers, ncclGather and k_unpack on the comm stream -- so that the event and
    // buffer choreography of a sharded frame runs on one GPU (RCCL refuses two ranks on one device)
    const char* lb = std::getenv("GSRT_DEBUG_COMM_LOOPBACK");
    if (nranks > 1 || (lb && lb[0] == '1')) {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        ncclResult_t r = ncclCommInitRank(&st->comm, nranks, uid, rank);
        if (r != ncclSuccess) {
            delete st;
            return fail(ctx, GSRT_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        // one comm stream at the default priority for the gather, the profile all-reduce and the unpack. Measured
        // and dropped (profiles/r04): the highest priority (the exchange workgroups went ahead of the next frame's
        // render workgroups: 8-rank shares +12-47 %), and the unpack on a stream of its own (a seventh stream shares
        // a hardware queue with the render / prep streams: +30-48 %). The process's stream configuration (how many
        // streams of each priority exist, in which order) moves a share's period by up to 2x: the streams are created
        // with the context, in one fixed order (gsrt_create; profiles/r06/queue_map.txt)
        st->cstream = ctx->cstream;
        bool ok = (st->cstream || hipStreamCreateWithFlags(&st->cstream, hipStreamNonBlocking) == hipSuccess) &&
                  hipEventCreateWithFlags(&st->ev_fb, kSyncEventFlags) == hipSuccess;
        for (int p = 0; p < 2 && ok; ++p)
            ok = hipEventCreateWithFlags(&st->rendered[p], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&st->gathered[p], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&st->unpacked[p], kSyncEventFlags) == hipSuccess &&
                 hipEventCreateWithFlags(&st->ev_prof[p], hipEventDisableTiming) == hipSuccess &&
                 hipHostMalloc(&st->h_hash[p], 2 * sizeof(uint32_t)) == hipSuccess;
        if (!ok) {
            ctx->comm = st;
            gsrt_comm_destroy_internal(ctx);
            return fail(ctx, GSRT_E_DEVICE, "comm stream/events creation failed");
        }
    }
    ctx->comm = st;
    return GSRT_OK;
}

}  // extern "C"

namespace {
// FNV-1a over a sharded frame's partition and packed layout, and whether the bands are pinned: every rank must render
// the same one, and pin or balance alike (a pinned rank would not follow the others' next cut)
uint32_t plan_hash(uint32_t tiles_x, uint32_t tiles_y, uint32_t tw, uint32_t th, uint32_t nranks, const uint32_t* bands,
                   uint32_t per_rank, bool pinned) {
    uint32_t h = 2166136261u;
    auto mix = [&h](uint32_t v) {
        for (int i = 0; i < 4; ++i) {
            h ^= (v >> (8 * i)) & 0xffu;
            h *= 16777619u;
        }
    };
    mix(tiles_x); mix(tiles_y); mix(tw); mix(th); mix(nranks); mix(per_rank); mix(pinned ? 1u : 0u);
    for (uint32_t r = 0; r <= nranks; ++r) mix(bands[r]);
    return h;
}
uint32_t plan_hash(const gsrt::RenderPlan& p, uint32_t per_rank, bool pinned) {
    return plan_hash(p.tiles_x, p.tiles_y, p.tw, p.th, p.nranks, p.bands.row, per_rank, pinned);
}

// The band decision of a profile frame, a pure function every rank applies to the same inputs: the all-reduced
// profile (tiles_y row costs, then max(h) and max(~h) over the ranks' partition hashes), this rank's hash, its current
// bands and whether they are pinned. GSRT_E_COMM when the ranks' hashes differ (max(~h) != ~max(h)); else out = the
// bands balance_bands cuts from the profile when they lower the heaviest band's cost by kAdoptGain (never for pinned
// bands), otherwise the current ones.
gsrt_status decide_bands(uint32_t tiles_y, uint32_t nranks, const uint32_t* cur, bool pinned, const uint32_t* prof,
                         uint32_t my_hash, float root_w, uint32_t* out) {
    std::copy(cur, cur + nranks + 1, out);
    if (prof[tiles_y] != my_hash || prof[tiles_y + 1] != ~my_hash) return GSRT_E_COMM;
    if (pinned) return GSRT_OK;
    std::vector<uint32_t> nb(nranks + 1);
    gsrt::balance_bands(tiles_y, nranks, prof, root_w, nb.data());
    if (gsrt::band_peak(nranks, nb.data(), prof, root_w) < (1.0 - kAdoptGain) * gsrt::band_peak(nranks, cur, prof, root_w))
        std::copy(nb.begin(), nb.end(), out);
    return GSRT_OK;
}

// The partition of the next sharded frame (see the file comment): pinned bands, or the current bands of this frame
// geometry, updated from the profile taken kProfileEvery frames earlier. Profile frames follow a fixed schedule (every
// kProfileEvery-th sharded COR frame, pinned or not), so every rank joins the same all-reduces; each checks the
// partition hashes they carried. Deterministic on every rank.
gsrt_status choose_bands(gsrt_ctx* ctx, const gsrt_ubo& ubo, uint32_t mode, uint32_t PN, bool profiled,
                         const uint32_t key[4], float root_w, uint32_t tiles_y) {
    gsrt_comm_state* cs = ctx->comm;
    if (cs->pinned) {
        if (cs->bands.size() != PN + 1 || cs->bands[PN] != tiles_y)
            return gsrt::fail(ctx, GSRT_E_ARG, "the pinned bands (gsrt_set_bands) do not fit this frame");
    } else if (std::memcmp(key, cs->bands_key, sizeof cs->bands_key) != 0) {  // a new frame geometry: even bands
        const gsrt::RenderPlan p0 = gsrt::make_plan(ubo, mode, 0, 0, PN);
        cs->bands.assign(p0.bands.row, p0.bands.row + PN + 1);
        std::memcpy(cs->bands_key, key, sizeof cs->bands_key);
    }
    const uint32_t f = cs->frames;
    if (!profiled || f % kProfileEvery != 0 || f < kProfileEvery) return GSRT_OK;
    const uint32_t q = (f / kProfileEvery + 1) % 2;  // the profile of frame f - kProfileEvery
    if (!cs->prof_pending[q]) return GSRT_OK;
    GSRT_HIP(ctx, hipEventSynchronize(cs->ev_prof[q]));
    cs->prof_pending[q] = false;
    if (std::memcmp(cs->prof_key[q], key, sizeof cs->bands_key) != 0) return GSRT_OK;  // another geometry's
    std::vector<uint32_t> nb(PN + 1);
    if (decide_bands(tiles_y, PN, cs->bands.data(), cs->pinned, cs->h_prof[q], cs->prof_hash[q], root_w, nb.data()) !=
        GSRT_OK) {
        cs->comm_error = true;
        return gsrt::fail(ctx, GSRT_E_COMM, "the ranks rendered different partitions (profile hash mismatch)");
    }
    cs->bands = nb;
    return GSRT_OK;
}
}  // namespace

extern "C" {

gsrt_status gsrt_render_sharded_async(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k) {
    if (!sc || !ubo) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (!ctx->comm) return fail(ctx, GSRT_E_STATE, "gsrt_comm_init not called");
    if (!sc->bvh_built) return fail(ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
    if (ubo->width == 0 || ubo->height == 0 || (mode & 0xffu) > GSRT_MODE_COR) return GSRT_E_ARG;
    if (sc->ntri && (mode & 0xffu) != GSRT_MODE_REF)
        return fail(ctx, GSRT_E_ARG, "triangle meshes are co-traced in REF mode only");
    (void)hipSetDevice(ctx->device);
    gsrt_comm_state* cs = ctx->comm;
    if (cs->comm_error) return fail(ctx, GSRT_E_COMM, "the ranks rendered different partitions (profile hash mismatch)");
    const int N = cs->nranks, R = cs->rank;
    uint32_t en = 0, er = 0;  // rank-share emulation on a loopback communicator (debug_rank_of)
    const bool emu = N == 1 && cs->comm && gsrt::debug_rank_of(mode, en, er);
    const uint32_t PN = emu ? en : (uint32_t)N, PR = emu ? er : (uint32_t)R;  // the plan's ranks
    const bool root = emu ? er == 0 : R == 0;  // unpacks the gathered blocks
    const bool cor = (mode & 0xffu) == GSRT_MODE_COR;
    const bool d8 = (mode & GSRT_FLAG_OUT_DUMP8) != 0;
    if (d8 && (!cor || (mode & GSRT_FLAG_STATS) || !cs->comm))
        return fail(ctx, GSRT_E_ARG, "GSRT_FLAG_OUT_DUMP8: COR frames without GSRT_FLAG_STATS on a communicator only");
    // the partition: balanced from the ranks' cost profiles on a real N-rank communicator (COR frames)
    const gsrt::RenderPlan even = gsrt::make_plan(*ubo, mode, k, PR, PN);
    const float root_w = cor ? gsrt::root_weight(PN, ubo->samples, mode) : 1.0f;
    uint32_t wbits;
    std::memcpy(&wbits, &root_w, sizeof wbits);
    const uint32_t key[4] = {even.tiles_y, PN, even.th, wbits};
    // profile frames: a fixed schedule of the sharded COR frames, whether this rank pinned its bands or not, so every
    // rank of the job joins the same all-reduces (a rank share on a loopback communicator takes them too, from its own
    // rows' costs only: it exercises the profile path on one GPU; the bench pins its bands, which are then kept)
    const bool profiled = cor && !(mode & GSRT_FLAG_STATS) && cs->comm && (N > 1 || emu);
    if (gsrt_status sb = choose_bands(ctx, *ubo, mode, PN, profiled, key, root_w, even.tiles_y); sb != GSRT_OK) return sb;
    gsrt::RenderPlan plan = gsrt::make_plan(*ubo, mode, k, PR, PN, cs->bands.data());
    cs->last_bands = cs->bands;
    const uint32_t frame = cs->frames++;
    const size_t px = (size_t)ubo->width * ubo->height;
    if (ctx->fb_pixels < px * 4) {
        if (cs->cstream) GSRT_HIP(ctx, hipStreamSynchronize(cs->cstream));  // unpack in flight
        (void)hipFree(ctx->d_fb);
        ctx->d_fb = nullptr;
        ctx->fb_pixels = 0;
        GSRT_HIP(ctx, hipMalloc(&ctx->d_fb, sizeof(float) * 4 * px));
        ctx->fb_pixels = px * 4;
    }
    ctx->last_w = ubo->width;
    ctx->last_h = ubo->height;
    ctx->last_stats = false;
    ctx->fb_view = nullptr;  // sharded frames land in d_fb (rank 0's unpack)
    ctx->fb_dump8 = d8;      // a dump8 frame leaves no RGBA32F image (gsrt_dump8_read reads it)
    gsrt::timing_mark(ctx, 0);
    if (N == 1 && !cs->comm) {  // one rank without a communicator: straight into the framebuffer
        gsrt_status s1 = gsrt::launch_render(sc, *ubo, plan, ctx->d_fb, nullptr);
        gsrt::timing_mark(ctx, 3);
        return s1;
    }
    const uint32_t per_rank = gsrt::max_local_tiles(plan);  // packed stride of every rank in the gather
    const size_t tile_floats = 4ull * plan.tw * plan.th;
    // the block each rank sends (in 32-bit words): RGBA32F tiles, or dump codes + escape list
    const Dump8Layout L = dump8_layout(per_rank, plan.tw * plan.th);
    const size_t send_floats = d8 ? L.block : per_rank * tile_floats;
    if (cs->packed_floats < send_floats) {
        GSRT_HIP(ctx, hipDeviceSynchronize());  // the old buffers may still be in flight
        for (int p = 0; p < 2; ++p) {
            (void)hipFree(cs->packed[p]);
            cs->packed[p] = nullptr;
        }
        cs->packed_floats = 0;
        for (int p = 0; p < 2; ++p) {
            GSRT_HIP(ctx, hipMalloc(&cs->packed[p], sizeof(float) * send_floats));
            cs->esc_at[p] = kNoHeader;
        }
        cs->packed_floats = send_floats;
    }
    if (R == 0 && cs->gbuf_floats < send_floats * PN) {
        if (gsrt_status s0 = gsrt_comm_sync_internal(ctx); s0 != GSRT_OK) return s0;
        for (int q = 0; q < 2; ++q) {
            (void)hipFree(cs->gbuf[q]);
            cs->gbuf[q] = nullptr;
            cs->unpack_pending[q] = false;
        }
        cs->gbuf_floats = 0;
        for (int q = 0; q < 2; ++q) GSRT_HIP(ctx, hipMalloc(&cs->gbuf[q], sizeof(float) * send_floats * PN));
        cs->gbuf_floats = send_floats * PN;
    }
    if (emu && root && cs->inbound_floats < send_floats * (PN - 1)) {
        if (gsrt_status s0 = gsrt_comm_sync_internal(ctx); s0 != GSRT_OK) return s0;
        (void)hipFree(cs->inbound);
        cs->inbound = nullptr;
        cs->inbound_floats = 0;
        GSRT_HIP(ctx, hipMalloc(&cs->inbound, sizeof(float) * send_floats * (PN - 1)));
        GSRT_HIP(ctx, hipMemset(cs->inbound, 0, sizeof(float) * send_floats * (PN - 1)));
        cs->inbound_floats = send_floats * (PN - 1);
    }
    // a profile frame: the render kernel stores each tile's cost (d_tcost), summed per row into d_prof (zeroed after
    // its previous all-reduce) on the comm stream
    const uint32_t rows = plan.tiles_y;
    const bool profile = profiled && frame % kProfileEvery == 0;
    const bool costs = profile || (cs->share_costs && cor && !(mode & GSRT_FLAG_STATS));
    if (costs && cs->tcost_cap < per_rank) {
        if (gsrt_status s0 = gsrt_comm_sync_internal(ctx); s0 != GSRT_OK) return s0;
        GSRT_HIP(ctx, hipDeviceSynchronize());  // a render may still write the old buffer
        (void)hipFree(cs->d_tcost);
        cs->d_tcost = nullptr;
        cs->tcost_cap = 0;
        GSRT_HIP(ctx, hipMalloc(&cs->d_tcost, sizeof(uint32_t) * (per_rank ? per_rank : 1)));
        cs->tcost_cap = per_rank;
    }
    const uint32_t qp = (frame / kProfileEvery) % 2;
    if (profile && cs->prof_rows < rows + 2) {
        if (gsrt_status s0 = gsrt_comm_sync_internal(ctx); s0 != GSRT_OK) return s0;
        GSRT_HIP(ctx, hipDeviceSynchronize());  // a render may still add into the old profile
        (void)hipFree(cs->d_prof);
        (void)hipFree(cs->d_prof_red);
        cs->d_prof = cs->d_prof_red = nullptr;
        cs->prof_rows = 0;
        for (int q = 0; q < 2; ++q) {
            (void)hipHostFree(cs->h_prof[q]);
            cs->h_prof[q] = nullptr;
            cs->prof_pending[q] = false;
        }
        GSRT_HIP(ctx, hipMalloc(&cs->d_prof, sizeof(uint32_t) * (rows + 2)));
        GSRT_HIP(ctx, hipMalloc(&cs->d_prof_red, sizeof(uint32_t) * (rows + 2)));
        for (int q = 0; q < 2; ++q) GSRT_HIP(ctx, hipHostMalloc(&cs->h_prof[q], sizeof(uint32_t) * (rows + 2)));
        GSRT_HIP(ctx, hipMemset(cs->d_prof, 0, sizeof(uint32_t) * (rows + 2)));
        cs->prof_rows = rows + 2;
    }
    const uint32_t p = cs->parity;
    cs->parity ^= 1u;
    cs->last_p = p;
    const size_t tile_px = (size_t)per_rank * plan.tw * plan.th;
    if (d8 && plan.passes > 1 && cs->accum_px < tile_px) {
        GSRT_HIP(ctx, hipDeviceSynchronize());  // a render may still use the old sums
        for (int q = 0; q < 2; ++q) {
            (void)hipFree(cs->d_accum[q]);
            cs->d_accum[q] = nullptr;
        }
        cs->accum_px = 0;
        for (int q = 0; q < 2; ++q) GSRT_HIP(ctx, hipMalloc(&cs->d_accum[q], sizeof(float4) * tile_px));
        cs->accum_px = tile_px;
    }
    if (d8 && cs->esc_at[p] != L.codes) {
        // the render counts its escapes in the header, zeroed after the gather that last read packed[p] (below);
        // here it is at a new place: zero it there, after that gather
        GSRT_HIP(ctx, hipMemsetAsync(cs->packed[p] + L.codes, 0, 16, cs->cstream));
        GSRT_HIP(ctx, hipEventRecord(cs->gathered[p], cs->cstream));
    }
    cs->esc_at[p] = d8 ? L.codes : kNoHeader;  // an RGBA32F frame writes over the header
    // render into packed[p] once the gather two frames back has sent it; packed[p] is this frame's own buffer, so
    // its render kernel need not follow the previous frame's (slot streams)
    plan.packed = true;
    gsrt::RenderSync rsy;
    rsy.slot = gsrt::use_slot_streams(ctx, PN > 1);
    rsy.private_out = true;
    rsy.wait = cs->gathered[p];
    rsy.sharded = true;
    rsy.tile_cost = costs ? cs->d_tcost : nullptr;
    if (costs) {
        cs->sc_tiles_x = plan.tiles_x;
        cs->sc_rows = plan.tiles_y;
        cs->sc_row0 = plan.row0();
        cs->sc_row1 = plan.row1();
    }
    if (d8) {
        rsy.dump8 = true;
        rsy.esc = reinterpret_cast<uint4*>(cs->packed[p] + L.codes);
        rsy.esc_cap = L.cap;
        rsy.accum = plan.passes > 1 ? cs->d_accum[p] : nullptr;
    }
    gsrt_status s = gsrt::launch_render(sc, *ubo, plan, cs->packed[p], nullptr, &rsy);
    if (s != GSRT_OK) return s;
    GSRT_HIP(ctx, hipEventRecord(cs->rendered[p], rsy.stream));
    // the gather on the comm stream, into gbuf[p] once the unpack two frames back has read it
    GSRT_HIP(ctx, hipStreamWaitEvent(cs->cstream, cs->rendered[p], 0));
    if (root && cs->unpack_pending[p]) GSRT_HIP(ctx, hipStreamWaitEvent(cs->cstream, cs->unpacked[p], 0));
    gsrt::timing_mark(ctx, 4, cs->cstream);  // the exchange starts once this rank's share is rendered
    float* const gb = R == 0 ? cs->gbuf[p] : nullptr;
    ncclResult_t r = ncclGather(cs->packed[p], gb, send_floats, ncclFloat32, 0, cs->comm, cs->cstream);
    if (r != ncclSuccess) return fail(ctx, GSRT_E_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
    if (d8) GSRT_HIP(ctx, hipMemsetAsync(cs->packed[p] + L.codes, 0, 16, cs->cstream));  // the next render's count
    if (emu && root)  // the other ranks' blocks landing in the gather buffer (stand-in for the receive)
        gsrt::launch_copy_d2d(cs->cstream, gb + send_floats, cs->inbound, sizeof(float) * send_floats * (PN - 1));
    GSRT_HIP(ctx, hipGetLastError());
    GSRT_HIP(ctx, hipEventRecord(cs->gathered[p], cs->cstream));
    if (root && d8) {  // the unpack of the codes into rank 0's code framebuffer (gsrt_dump8_read)
        if (cs->codes_px < px) {
            if (gsrt_status s0 = gsrt_comm_sync_internal(ctx); s0 != GSRT_OK) return s0;
            (void)hipFree(cs->d_codes);
            cs->d_codes = nullptr;
            cs->codes_px = 0;
            GSRT_HIP(ctx, hipMalloc(&cs->d_codes, sizeof(uint32_t) * px));
            cs->codes_px = px;
        }
        gsrt::launch_unpack_dump8(cs->cstream, reinterpret_cast<const uint32_t*>(gb), cs->d_codes, plan, ubo->width,
                                  ubo->height, per_rank, L.block);
        GSRT_HIP(ctx, hipGetLastError());
        GSRT_HIP(ctx, hipEventRecord(cs->unpacked[p], cs->cstream));
        cs->unpack_pending[p] = true;
    } else if (root) {  // the unpack, after the gather on the comm stream
        if (cs->fb_on_render) {  // a whole frame rendered into d_fb on the render stream since the last unpack
            GSRT_HIP(ctx, hipEventRecord(cs->ev_fb, ctx->stream));
            GSRT_HIP(ctx, hipStreamWaitEvent(cs->cstream, cs->ev_fb, 0));
            cs->fb_on_render = false;
        }
        gsrt::launch_unpack(cs->cstream, gb, ctx->d_fb, plan, ubo->width, ubo->height, per_rank);
        GSRT_HIP(ctx, hipGetLastError());
        GSRT_HIP(ctx, hipEventRecord(cs->unpacked[p], cs->cstream));
        cs->unpack_pending[p] = true;
        cs->fb_on_comm = true;
    }
    gsrt::timing_mark(ctx, 5, cs->cstream);
    cs->d8_last = d8;
    cs->d8_root = root;
    if (d8) {
        cs->d8_plan = plan;
        cs->d8_layout = L;
        cs->d8_w = ubo->width;
        cs->d8_h = ubo->height;
    }
    if (profile) {
        // every rank's row costs to every rank (max: a row has one contributor), with this rank's partition hash
        if (cs->prof_pending[qp]) GSRT_HIP(ctx, hipEventSynchronize(cs->ev_prof[qp]));  // h_hash[qp] is free again
        gsrt::launch_row_sum(cs->cstream, cs->d_tcost, cs->d_prof, plan.tiles_x, plan.row0(), plan.row1());
        const uint32_t hsh = plan_hash(plan, per_rank, cs->pinned);
        cs->h_hash[qp][0] = hsh;
        cs->h_hash[qp][1] = ~hsh;
        GSRT_HIP(ctx, hipMemcpyAsync(cs->d_prof + rows, cs->h_hash[qp], 2 * sizeof(uint32_t), hipMemcpyHostToDevice,
                                     cs->cstream));
        r = ncclAllReduce(cs->d_prof, cs->d_prof_red, rows + 2, ncclUint32, ncclMax, cs->comm, cs->cstream);
        if (r != ncclSuccess) return fail(ctx, GSRT_E_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        GSRT_HIP(ctx, hipMemsetAsync(cs->d_prof, 0, sizeof(uint32_t) * (rows + 2), cs->cstream));
        GSRT_HIP(ctx, hipMemcpyAsync(cs->h_prof[qp], cs->d_prof_red, sizeof(uint32_t) * (rows + 2), hipMemcpyDeviceToHost,
                                     cs->cstream));
        GSRT_HIP(ctx, hipEventRecord(cs->ev_prof[qp], cs->cstream));
        cs->prof_pending[qp] = true;
        cs->prof_hash[qp] = hsh;
        std::memcpy(cs->prof_key[qp], key, sizeof key);
    }
    gsrt::timing_mark(ctx, 3);  // on the compute stream: the exchange overlaps the next frame
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out) {
    if (sc && rgba_out && (mode & GSRT_FLAG_OUT_DUMP8))
        return fail(sc->ctx, GSRT_E_ARG, "a dump8 frame is read with gsrt_dump8_read");
    gsrt_status s = gsrt_render_sharded_async(sc, ubo, mode, k);
    if (s != GSRT_OK) return s;
    gsrt_ctx* ctx = sc->ctx;
    if ((s = gsrt_comm_sync_internal(ctx)) != GSRT_OK) return s;
    if (rgba_out && ctx->comm->rank == 0) {
        hipPointerAttribute_t attr;
        bool dev = hipPointerGetAttributes(&attr, rgba_out) == hipSuccess && attr.type == hipMemoryTypeDevice;
        (void)hipGetLastError();
        GSRT_HIP(ctx, hipMemcpyAsync(rgba_out, ctx->d_fb, sizeof(float) * 4 * ubo->width * ubo->height,
                                     dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
    }
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return gsrt::check_error_word(ctx);
}

// bands: nranks + 1 boundaries, or nullptr for the even partition (make_plan); checked to cut tile rows 0..tiles_y
static bool bands_fit(const gsrt::RenderPlan& p, const uint32_t* bands) {
    if (!bands) return true;
    if (bands[0] != 0 || bands[p.nranks] != p.tiles_y) return false;
    for (uint32_t r = 0; r < p.nranks; ++r)
        if (bands[r + 1] < bands[r]) return false;
    return true;
}

gsrt_status gsrt_tile_plan(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, uint32_t out[8]) {
    if (!ubo || !out || nranks < 1 || nranks > (int)gsrt::kMaxRanks || rank < 0 || rank >= nranks || ubo->width == 0 ||
        ubo->height == 0)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)rank, (uint32_t)nranks);
    out[0] = p.tw;
    out[1] = p.th;
    out[2] = p.tiles_x;
    out[3] = p.tiles_y;
    out[4] = gsrt::local_tiles(p);
    out[5] = p.s_lanes;
    out[6] = p.row0();
    out[7] = gsrt::max_local_tiles(p);
    return GSRT_OK;
}

gsrt_status gsrt_tile_bands(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* row_cost, uint32_t* bands) {
    if (!ubo || !bands || nranks < 1 || nranks > (int)gsrt::kMaxRanks || ubo->width == 0 || ubo->height == 0)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks);
    const float w0 = (mode & 0xffu) == GSRT_MODE_COR ? gsrt::root_weight((uint32_t)nranks, ubo->samples, mode) : 1.0f;
    gsrt::balance_bands(p.tiles_y, (uint32_t)nranks, row_cost, w0, bands);
    return GSRT_OK;
}

gsrt_status gsrt_set_bands(gsrt_ctx* ctx, int nranks, const uint32_t* bands) {
    if (!ctx || !ctx->comm) return ctx ? fail(ctx, GSRT_E_STATE, "gsrt_comm_init not called") : GSRT_E_ARG;
    gsrt_comm_state* cs = ctx->comm;
    if (!bands) {
        cs->pinned = false;
        std::memset(cs->bands_key, 0, sizeof cs->bands_key);  // back to even bands, then balancing
        return GSRT_OK;
    }
    if (nranks < 1 || nranks > (int)gsrt::kMaxRanks || bands[0] != 0) return GSRT_E_ARG;
    for (int r = 0; r < nranks; ++r)
        if (bands[r + 1] < bands[r]) return GSRT_E_ARG;
    cs->bands.assign(bands, bands + nranks + 1);
    cs->pinned = true;
    return GSRT_OK;
}

gsrt_status gsrt_last_bands(gsrt_ctx* ctx, uint32_t* bands, uint32_t cap, uint32_t* n) {
    if (!ctx || !bands) return GSRT_E_ARG;
    const std::vector<uint32_t> empty;
    const std::vector<uint32_t>& b = ctx->comm ? ctx->comm->last_bands : empty;
    const uint32_t m = (uint32_t)b.size() < cap ? (uint32_t)b.size() : cap;
    for (uint32_t i = 0; i < m; ++i) bands[i] = b[i];
    if (n) *n = (uint32_t)b.size();
    return GSRT_OK;
}

gsrt_status gsrt_row_costs(gsrt_ctx* ctx, uint32_t* row_cost, uint32_t cap, uint32_t* rows) {
    if (!ctx || !row_cost) return GSRT_E_ARG;
    const uint32_t tx = ctx->tile_cost_tx, ty = ctx->tile_cost_ty;
    if (!ty) return fail(ctx, GSRT_E_STATE, "no whole COR frame rendered yet");
    if (gsrt_status s = gsrt::sync_all(ctx); s != GSRT_OK) return s;
    std::vector<uint32_t> t((size_t)tx * ty);
    GSRT_HIP(ctx, hipMemcpy(t.data(), ctx->d_tile_cost[ctx->tile_cost_slot], sizeof(uint32_t) * t.size(),
                            hipMemcpyDeviceToHost));
    std::vector<uint32_t> r(ty, 0u);
    for (uint32_t lt = 0; lt < t.size(); ++lt) {  // a whole frame: one band of every row, spatial tile order
        uint32_t x, y;
        gsrt::band_tile(lt, 0, ty, tx, x, y);
        r[y] += t[lt];
    }
    for (uint32_t i = 0; i < ty && i < cap; ++i) row_cost[i] = r[i];
    if (rows) *rows = ty;
    return GSRT_OK;
}

// Host mirror of the sharded layout, from the same inline mappings the kernels use (gsrt_device.hpp): local tile
// lt of a rank is band_tile(lt) (the packed render writes it to slot lt, pixel (y % th) tw + x % tw), and k_unpack
// finds pixel (x, y) in the band of its tile row at band_index.
gsrt_status gsrt_tile_pack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const uint32_t* bands,
                                const float* rgba, float* packed) {
    if (!ubo || !rgba || !packed || nranks < 1 || nranks > (int)gsrt::kMaxRanks || rank < 0 || rank >= nranks)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)rank, (uint32_t)nranks, bands);
    if (!bands_fit(p, bands)) return GSRT_E_ARG;
    const uint32_t W = ubo->width, H = ubo->height, nl = gsrt::local_tiles(p), stride = gsrt::max_local_tiles(p);
    std::memset(packed, 0, sizeof(float) * 4ull * p.tw * p.th * stride);
    for (uint32_t lt = 0; lt < nl; ++lt) {
        uint32_t tx, ty;
        gsrt::band_tile(lt, p.row0(), p.row1(), p.tiles_x, tx, ty);
        for (uint32_t q = 0; q < p.tw * p.th; ++q) {
            const uint32_t x = tx * p.tw + q % p.tw, y = ty * p.th + q / p.tw;
            if (x < W && y < H)
                std::memcpy(packed + 4 * ((size_t)lt * p.tw * p.th + q), rgba + 4 * ((size_t)y * W + x), 16);
        }
    }
    return GSRT_OK;
}

gsrt_status gsrt_tile_unpack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands,
                                  const float* gathered, float* rgba_out) {
    if (!ubo || !gathered || !rgba_out || nranks < 1 || nranks > (int)gsrt::kMaxRanks) return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks, bands);
    if (!bands_fit(p, bands)) return GSRT_E_ARG;
    const uint32_t W = ubo->width, H = ubo->height, stride = gsrt::max_local_tiles(p);
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            const uint32_t tx = x / p.tw, ty = y / p.th, r = gsrt::band_of(p.bands, ty);
            const uint32_t lt = gsrt::band_index(tx, ty, p.bands.row[r], p.bands.row[r + 1], p.tiles_x);
            const size_t src = ((size_t)r * stride + lt) * p.tw * p.th + (y % p.th) * p.tw + (x % p.tw);
            std::memcpy(rgba_out + 4 * ((size_t)y * W + x), gathered + 4 * src, 16);
        }
    return GSRT_OK;
}

}  // extern "C"

// block r's escape list (host memory: the uint4 header, then the entries) as frame pixels, appended to out; false and
// why when the list overflowed its capacity or names a pixel outside the frame
static bool map_escapes(const uint32_t* list, uint32_t r, const gsrt::RenderPlan& p, const Dump8Layout& L, uint32_t W,
                        uint32_t H, std::vector<gsrt_dump8_escape>& out, std::string& why) {
    const uint32_t n = list[0], tp = p.tw * p.th;
    if (n > L.cap) {
        why = "dump8: rank " + std::to_string(r) + " has " + std::to_string(n) + " escaped pixels, its list holds " +
              std::to_string(L.cap);
        return false;
    }
    const uint32_t* e = list + 4;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t idx = e[4 * i], lt = idx / tp, q = idx % tp;
        uint32_t tx, ty;
        gsrt::band_tile(lt, p.bands.row[r], p.bands.row[r + 1], p.tiles_x, tx, ty);
        const uint32_t x = tx * p.tw + q % p.tw, y = ty * p.th + q / p.tw;
        if (lt >= gsrt::max_local_tiles(p) || x >= W || y >= H) {
            why = "dump8: an escape outside the frame";
            return false;
        }
        gsrt_dump8_escape g;
        g.pixel = x + y * W;
        std::memcpy(&g.r, &e[4 * i + 1], 4);
        std::memcpy(&g.g, &e[4 * i + 2], 4);
        std::memcpy(&g.b, &e[4 * i + 3], 4);
        out.push_back(g);
    }
    return true;
}

static void sort_escapes(std::vector<gsrt_dump8_escape>& v) {
    std::sort(v.begin(), v.end(), [](const gsrt_dump8_escape& a, const gsrt_dump8_escape& b) { return a.pixel < b.pixel; });
}

// the escapes of dump8 blocks in device memory (gathered: nranks blocks, rank-major) as frame pixels, in pixel order;
// GSRT_E_STATE when a rank's list overflowed
static gsrt_status gather_escapes(gsrt_ctx* ctx, const float* gathered, const gsrt::RenderPlan& p, const Dump8Layout& L,
                                  uint32_t W, uint32_t H, std::vector<gsrt_dump8_escape>& out) {
    out.clear();
    std::vector<uint32_t> list;
    for (uint32_t r = 0; r < p.nranks; ++r) {
        const float* blk = gathered + (size_t)r * L.block + L.codes;
        list.assign(4, 0u);
        GSRT_HIP(ctx, hipMemcpy(list.data(), blk, 16, hipMemcpyDeviceToHost));
        const uint32_t n = std::min(list[0], L.cap);  // an overflowed count is reported by map_escapes
        list.resize(4 + 4ull * n);
        if (n) GSRT_HIP(ctx, hipMemcpy(list.data() + 4, blk + 4, sizeof(uint32_t) * 4 * n, hipMemcpyDeviceToHost));
        std::string why;
        if (!map_escapes(list.data(), r, p, L, W, H, out, why)) return fail(ctx, GSRT_E_STATE, why);
    }
    sort_escapes(out);
    return GSRT_OK;
}

static void copy_escapes(const std::vector<gsrt_dump8_escape>& v, gsrt_dump8_escape* esc, uint32_t cap, uint32_t* n_esc) {
    if (esc)
        for (size_t i = 0; i < v.size() && i < cap; ++i) esc[i] = v[i];
    if (n_esc) *n_esc = (uint32_t)v.size();
}

// every rank's share rendered on this device into the gather layout (RGBA32F tiles or dump8 blocks), then unpacked by
// the kernel rank 0 uses after the gather
static gsrt_status render_emulated(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands,
                                   float* rgba_out, uint32_t* codes, gsrt_dump8_escape* esc, uint32_t cap,
                                   uint32_t* n_esc) {
    gsrt_ctx* ctx = sc->ctx;
    if (!sc->bvh_built) return fail(ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
    if (sc->ntri && (mode & 0xffu) != GSRT_MODE_REF)
        return fail(ctx, GSRT_E_ARG, "triangle meshes are co-traced in REF mode only");
    const bool d8 = (mode & GSRT_FLAG_OUT_DUMP8) != 0;
    if (d8 && ((mode & 0xffu) != GSRT_MODE_COR || (mode & GSRT_FLAG_STATS)))
        return fail(ctx, GSRT_E_ARG, "GSRT_FLAG_OUT_DUMP8: COR frames without GSRT_FLAG_STATS only");
    (void)hipSetDevice(ctx->device);
    const gsrt::RenderPlan p0 = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks, bands);
    if (!bands_fit(p0, bands)) return GSRT_E_ARG;
    const uint32_t per_rank = gsrt::max_local_tiles(p0);
    const size_t tile_floats = 4ull * p0.tw * p0.th;
    const Dump8Layout L = dump8_layout(per_rank, p0.tw * p0.th);
    const size_t block = d8 ? L.block : tile_floats * per_rank;  // words per rank
    const size_t px = (size_t)ubo->width * ubo->height;
    const size_t fb_bytes = d8 ? sizeof(uint32_t) * px : sizeof(float) * 4 * px;
    const size_t accum_px = d8 && p0.passes > 1 ? (size_t)per_rank * p0.tw * p0.th : 0;
    float* gather = nullptr;
    void* fb = nullptr;
    float4* accum = nullptr;
    GSRT_HIP(ctx, hipMalloc(&gather, sizeof(float) * (block ? block : 1) * nranks));
    gsrt_status s = GSRT_OK;
    if (hipMalloc(&fb, fb_bytes) != hipSuccess || (accum_px && hipMalloc(&accum, sizeof(float4) * accum_px) != hipSuccess) ||
        hipMemset(gather, 0, sizeof(float) * (block ? block : 1) * nranks) != hipSuccess)
        s = fail(ctx, GSRT_E_OOM, "emulated gather: allocation failed");
    for (int r = 0; r < nranks && s == GSRT_OK; ++r) {
        gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)r, (uint32_t)nranks, bands);
        p.packed = true;
        gsrt::RenderSync rsy;  // a rank's share: no cost profile
        rsy.sharded = true;
        float* blk = gather + (size_t)r * block;
        if (d8) {
            rsy.dump8 = true;
            rsy.esc = reinterpret_cast<uint4*>(blk + L.codes);
            rsy.esc_cap = L.cap;
            rsy.accum = accum;  // the shares render one after the other on the stream
        }
        s = gsrt::launch_render(sc, *ubo, p, blk, nullptr, &rsy);
    }
    if (s == GSRT_OK) {
        if (d8)
            gsrt::launch_unpack_dump8(ctx->stream, reinterpret_cast<const uint32_t*>(gather), static_cast<uint32_t*>(fb), p0,
                                      ubo->width, ubo->height, per_rank, L.block);
        else
            gsrt::launch_unpack(ctx->stream, gather, static_cast<float*>(fb), p0, ubo->width, ubo->height, per_rank);
        void* dst = d8 ? static_cast<void*>(codes) : static_cast<void*>(rgba_out);
        if ((dst && hipMemcpyAsync(dst, fb, fb_bytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "emulated gather: copy failed");
    }
    (void)hipStreamSynchronize(ctx->stream);
    if (s == GSRT_OK) s = gsrt::check_error_word(ctx);
    if (s == GSRT_OK && d8) {
        std::vector<gsrt_dump8_escape> v;
        s = gather_escapes(ctx, gather, p0, L, ubo->width, ubo->height, v);
        if (s == GSRT_OK) copy_escapes(v, esc, cap, n_esc);
    }
    (void)hipFree(gather);
    (void)hipFree(fb);
    (void)hipFree(accum);
    return s;
}

extern "C" {

gsrt_status gsrt_render_sharded_emulated(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                         const uint32_t* bands, float* rgba_out) {
    if (!sc || !ubo || !rgba_out || nranks < 1 || nranks > (int)gsrt::kMaxRanks || (mode & GSRT_FLAG_OUT_DUMP8))
        return GSRT_E_ARG;
    return render_emulated(sc, ubo, mode, nranks, bands, rgba_out, nullptr, nullptr, 0, nullptr);
}

gsrt_status gsrt_render_sharded_emulated_dump8(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                               const uint32_t* bands, uint32_t* codes, gsrt_dump8_escape* esc,
                                               uint32_t cap, uint32_t* n_esc) {
    if (!sc || !ubo || nranks < 1 || nranks > (int)gsrt::kMaxRanks || !(mode & GSRT_FLAG_OUT_DUMP8)) return GSRT_E_ARG;
    return render_emulated(sc, ubo, mode, nranks, bands, nullptr, codes, esc, cap, n_esc);
}

gsrt_status gsrt_dump8_read(gsrt_ctx* ctx, uint32_t* codes, gsrt_dump8_escape* esc, uint32_t cap, uint32_t* n_esc) {
    if (!ctx) return GSRT_E_ARG;
    gsrt_comm_state* cs = ctx->comm;
    if (!cs || !cs->d8_last || !cs->d8_root || !cs->gbuf[cs->last_p])
        return fail(ctx, GSRT_E_STATE, "no GSRT_FLAG_OUT_DUMP8 sharded frame on rank 0");
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (gsrt_status s = gsrt::sync_all(ctx); s != GSRT_OK) return s;
    if (gsrt_status s = gsrt_comm_sync_internal(ctx); s != GSRT_OK) return s;
    if (codes)
        GSRT_HIP(ctx, hipMemcpy(codes, cs->d_codes, sizeof(uint32_t) * cs->d8_w * cs->d8_h, hipMemcpyDeviceToHost));
    std::vector<gsrt_dump8_escape> v;
    // the escape lists of the blocks in the gather buffer (on a loopback communicator with GSRT_DEBUG_RANK_OF the
    // stand-in blocks are zero: no escapes)
    if (gsrt_status s = gather_escapes(ctx, cs->gbuf[cs->last_p], cs->d8_plan, cs->d8_layout, cs->d8_w, cs->d8_h, v);
        s != GSRT_OK)
        return s;
    copy_escapes(v, esc, cap, n_esc);
    return gsrt::check_error_word(ctx);
}

gsrt_status gsrt_debug_share_costs(gsrt_ctx* ctx, int on) {
    if (!ctx || !ctx->comm) return ctx ? fail(ctx, GSRT_E_STATE, "gsrt_comm_init not called") : GSRT_E_ARG;
    ctx->comm->share_costs = on != 0;
    return GSRT_OK;
}

gsrt_status gsrt_debug_row_profile(gsrt_ctx* ctx, uint32_t* rows, uint32_t cap, uint32_t* n) {
    if (!ctx || !rows) return GSRT_E_ARG;
    gsrt_comm_state* cs = ctx->comm;
    if (!cs || !cs->d_tcost || !cs->sc_rows) return fail(ctx, GSRT_E_STATE, "no sharded frame with tile costs yet");
    if (gsrt_status s = gsrt::sync_all(ctx); s != GSRT_OK) return s;
    if (gsrt_status s = gsrt_comm_sync_internal(ctx); s != GSRT_OK) return s;
    uint32_t* d = nullptr;
    GSRT_HIP(ctx, hipMalloc(&d, sizeof(uint32_t) * cs->sc_rows));
    gsrt_status st = GSRT_OK;
    std::vector<uint32_t> h(cs->sc_rows, 0u);
    if (hipMemsetAsync(d, 0, sizeof(uint32_t) * cs->sc_rows, ctx->stream) != hipSuccess) st = GSRT_E_DEVICE;
    if (st == GSRT_OK) {
        gsrt::launch_row_sum(ctx->stream, cs->d_tcost, d, cs->sc_tiles_x, cs->sc_row0, cs->sc_row1);
        if (hipMemcpyAsync(h.data(), d, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            st = GSRT_E_DEVICE;
    }
    (void)hipFree(d);
    if (st != GSRT_OK) return fail(ctx, st, "row profile: device error");
    for (uint32_t i = 0; i < cs->sc_rows && i < cap; ++i) rows[i] = h[i];
    if (n) *n = cs->sc_rows;
    return GSRT_OK;
}

gsrt_status gsrt_dump8_encode(const float* rgba, size_t n, uint32_t* codes, gsrt_dump8_escape* esc, uint32_t cap,
                              uint32_t* n_esc) {
    if ((n && (!rgba || !codes))) return GSRT_E_ARG;
    uint32_t ne = 0;
    for (size_t i = 0; i < n; ++i) {
        const float4 v = make_float4(rgba[4 * i], rgba[4 * i + 1], rgba[4 * i + 2], rgba[4 * i + 3]);
        codes[i] = gsrt::dump8_code(v);
        if (codes[i] & gsrt::kDump8Escape) {
            if (esc && ne < cap) esc[ne] = gsrt_dump8_escape{(uint32_t)i, v.x, v.y, v.z};
            ++ne;
        }
    }
    if (n_esc) *n_esc = ne;
    return GSRT_OK;
}

// Host mirror of the dump8 blocks: the store path of k_render_cor (code word at slot lt * tile px + q, escapes
// appended to the block's list) and k_unpack_dump8 + gather_escapes on rank 0
static bool dump8_plan(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const uint32_t* bands,
                       gsrt::RenderPlan& p, Dump8Layout& L) {
    if (!ubo || nranks < 1 || nranks > (int)gsrt::kMaxRanks || rank < 0 || rank >= nranks || !ubo->width ||
        !ubo->height || (mode & 0xffu) != GSRT_MODE_COR)
        return false;
    p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)rank, (uint32_t)nranks, bands);
    if (!bands_fit(p, bands)) return false;
    L = dump8_layout(gsrt::max_local_tiles(p), p.tw * p.th);
    return true;
}

gsrt_status gsrt_dump8_layout(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, uint64_t out[3]) {
    gsrt::RenderPlan p;
    Dump8Layout L;
    if (!out || !dump8_plan(ubo, mode, nranks, 0, bands, p, L)) return GSRT_E_ARG;
    out[0] = L.block;
    out[1] = L.codes;
    out[2] = L.cap;
    return GSRT_OK;
}

gsrt_status gsrt_tile_pack_dump8_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const uint32_t* bands,
                                      const float* rgba, uint32_t* block) {
    gsrt::RenderPlan p;
    Dump8Layout L;
    if (!rgba || !block || !dump8_plan(ubo, mode, nranks, rank, bands, p, L)) return GSRT_E_ARG;
    const uint32_t W = ubo->width, H = ubo->height, tp = p.tw * p.th, nl = gsrt::local_tiles(p);
    std::memset(block, 0, sizeof(uint32_t) * L.block);
    uint32_t* list = block + L.codes;
    uint32_t n = 0;
    for (uint32_t lt = 0; lt < nl; ++lt) {
        uint32_t tx, ty;
        gsrt::band_tile(lt, p.row0(), p.row1(), p.tiles_x, tx, ty);
        for (uint32_t q = 0; q < tp; ++q) {
            const uint32_t x = tx * p.tw + q % p.tw, y = ty * p.th + q / p.tw;
            if (x >= W || y >= H) continue;
            const float* c = rgba + 4 * ((size_t)y * W + x);
            const uint32_t code = gsrt::dump8_code(make_float4(c[0], c[1], c[2], c[3]));
            block[(size_t)lt * tp + q] = code;
            if (!(code & gsrt::kDump8Escape)) continue;
            if (n < L.cap) {
                uint32_t* e = list + 4 + 4ull * n;
                e[0] = lt * tp + q;
                std::memcpy(e + 1, c, 12);
            }
            ++n;
        }
    }
    list[0] = n;
    return n > L.cap ? GSRT_E_STATE : GSRT_OK;
}

gsrt_status gsrt_tile_unpack_dump8_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands,
                                        const uint32_t* gathered, uint32_t* codes, gsrt_dump8_escape* esc,
                                        uint32_t cap, uint32_t* n_esc) {
    gsrt::RenderPlan p;
    Dump8Layout L;
    if (!gathered || !dump8_plan(ubo, mode, nranks, 0, bands, p, L)) return GSRT_E_ARG;
    const uint32_t W = ubo->width, H = ubo->height, tp = p.tw * p.th;
    if (codes)
        for (uint32_t y = 0; y < H; ++y)
            for (uint32_t x = 0; x < W; ++x) {
                const uint32_t tx = x / p.tw, ty = y / p.th, r = gsrt::band_of(p.bands, ty);
                const uint32_t lt = gsrt::band_index(tx, ty, p.bands.row[r], p.bands.row[r + 1], p.tiles_x);
                codes[(size_t)y * W + x] = gathered[(size_t)r * L.block + (size_t)lt * tp + (y % p.th) * p.tw + x % p.tw];
            }
    std::vector<gsrt_dump8_escape> v;
    std::string why;
    for (uint32_t r = 0; r < p.nranks; ++r)
        if (!map_escapes(gathered + (size_t)r * L.block + L.codes, r, p, L, W, H, v, why)) return GSRT_E_STATE;
    sort_escapes(v);
    copy_escapes(v, esc, cap, n_esc);
    return GSRT_OK;
}

gsrt_status gsrt_partition_hash(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, int pinned,
                                uint32_t* hash) {
    if (!ubo || !bands || !hash || nranks < 1 || nranks > (int)gsrt::kMaxRanks || !ubo->width || !ubo->height)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks, bands);
    if (!bands_fit(p, bands)) return GSRT_E_ARG;
    *hash = plan_hash(p, gsrt::max_local_tiles(p), pinned != 0);
    return GSRT_OK;
}

gsrt_status gsrt_decide_bands(const gsrt_ubo* ubo, uint32_t mode, int nranks, const uint32_t* bands, int pinned,
                              const uint32_t* profile, uint32_t my_hash, uint32_t* out) {
    if (!ubo || !bands || !profile || !out || nranks < 1 || nranks > (int)gsrt::kMaxRanks || !ubo->width || !ubo->height)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks, bands);
    if (!bands_fit(p, bands)) return GSRT_E_ARG;
    const float root_w = (mode & 0xffu) == GSRT_MODE_COR ? gsrt::root_weight((uint32_t)nranks, ubo->samples, mode) : 1.0f;
    return decide_bands(p.tiles_y, (uint32_t)nranks, bands, pinned != 0, profile, my_hash, root_w, out);
}

}  // extern "C"
