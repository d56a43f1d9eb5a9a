// gsrt_comm.cpp -- multi-GPU tile sharding.
//
// One process per GPU. The scene and its LBVH are replicated (each rank builds its own); the frame's
// tiles, in spatial order, are dealt round-robin over ranks in runs (whole 16x16-tile super-tiles on large
// frames, single tiles on small ones: RenderPlan::run), each rank renders its tiles into a packed buffer,
// and one ncclGather over xGMI brings the packed tiles to rank 0, which unpacks them into its framebuffer.
// The gather is the only exchange step; rendering needs no communication. The gather runs on its own stream
// (gstream) from one of two packed buffers into one of two gather buffers, and rank 0's unpack on another (cstream,
// the comm stream that finishes the image), so frame k's exchange overlaps frame k+1's rendering, and frame k's
// unpack overlaps frame k+1's gather.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>

#include "gsrt_internal.hpp"

struct gsrt_comm_state {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    hipStream_t cstream = nullptr;       // rank 0's unpack into d_fb: the comm stream (gsrt_comm_stream)
    hipStream_t gstream = nullptr;       // the gather (send; rank 0 also receives)
    hipEvent_t rendered[2] = {nullptr, nullptr};  // packed[p] written (compute stream)
    hipEvent_t gathered[2] = {nullptr, nullptr};  // packed[p] sent, gbuf[p] received (gstream): packed[p] is free
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
    if (c->gstream) (void)hipStreamSynchronize(c->gstream);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->gstream == c->cstream) c->gstream = nullptr;  // one stream for both
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (int p = 0; p < 2; ++p) {
        if (c->rendered[p]) (void)hipEventDestroy(c->rendered[p]);
        if (c->gathered[p]) (void)hipEventDestroy(c->gathered[p]);
        if (c->unpacked[p]) (void)hipEventDestroy(c->unpacked[p]);
        (void)hipFree(c->packed[p]);
        (void)hipFree(c->gbuf[p]);
    }
    (void)hipFree(c->inbound);
    if (c->ev_fb) (void)hipEventDestroy(c->ev_fb);
    if (c->gstream) (void)hipStreamDestroy(c->gstream);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    delete c;
    ctx->comm = nullptr;
}

// the comm stream of ctx (nullptr without a communicator)
hipStream_t gsrt_comm_stream_internal(gsrt_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->cstream : nullptr; }

// wait for the gather and unpack streams (gsrt_synchronize, reallocations)
gsrt_status gsrt_comm_sync_internal(gsrt_ctx* ctx) {
    if (!ctx || !ctx->comm) return GSRT_OK;
    if (ctx->comm->gstream) GSRT_HIP(ctx, hipStreamSynchronize(ctx->comm->gstream));
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
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return GSRT_E_ARG;
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
        // the comm stream at the default priority (GSRT_COMM_PRIORITY=1: the highest). At the highest, the exchange
        // workgroups went ahead of the next frame's render workgroups and the 8-rank shares got slower: root C3
        // 0.303 -> 0.374 ms, C4 0.304 -> 0.447 ms, the other ranks +12-16 % (profiles/r04/comm_priority.txt)
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        const char* cp = std::getenv("GSRT_COMM_PRIORITY");
        const int prio = (cp && cp[0] == '1') ? greatest : 0;
        // GSRT_COMM_SPLIT=1: the gather on a stream of its own (rank 0's unpack of frame f then overlaps the gather
        // of frame f+1); else one stream for both
        const char* sp = std::getenv("GSRT_COMM_SPLIT");
        const bool split = sp && sp[0] == '1';
        bool ok = hipStreamCreateWithPriority(&st->cstream, hipStreamNonBlocking, prio) == hipSuccess &&
                  (!split || hipStreamCreateWithPriority(&st->gstream, hipStreamNonBlocking, prio) == hipSuccess) &&
                  hipEventCreateWithFlags(&st->ev_fb, kSyncEventFlags) == hipSuccess;
        if (ok && !split) st->gstream = st->cstream;
        for (int p = 0; p < 2 && ok; ++p)
            ok = hipEventCreateWithFlags(&st->rendered[p], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&st->gathered[p], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&st->unpacked[p], kSyncEventFlags) == hipSuccess;
        if (!ok) {
            ctx->comm = st;
            gsrt_comm_destroy_internal(ctx);
            return fail(ctx, GSRT_E_DEVICE, "comm stream/events creation failed");
        }
    }
    ctx->comm = st;
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded_async(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k) {
    if (!sc || !ubo) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (!ctx->comm) return fail(ctx, GSRT_E_STATE, "gsrt_comm_init not called");
    if (!sc->bvh_built) return fail(ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
    if (ubo->width == 0 || ubo->height == 0 || (mode & 0xffu) > GSRT_MODE_COR) return GSRT_E_ARG;
    if (sc->ntri && (mode & 0xffu) != GSRT_MODE_REF)
        return fail(ctx, GSRT_E_ARG, "triangle meshes are co-traced in REF mode only");
    (void)hipSetDevice(ctx->device);
    const int N = ctx->comm->nranks, R = ctx->comm->rank;
    uint32_t en = 0, er = 0;  // rank-share emulation on a loopback communicator (debug_rank_of)
    const bool emu = N == 1 && ctx->comm->comm && gsrt::debug_rank_of(mode, en, er);
    const uint32_t PN = emu ? en : (uint32_t)N, PR = emu ? er : (uint32_t)R;  // the plan's ranks
    const bool root = emu ? er == 0 : R == 0;  // unpacks the gathered blocks
    gsrt::RenderPlan plan = gsrt::make_plan(*ubo, mode, k, PR, PN);
    const size_t px = (size_t)ubo->width * ubo->height;
    if (ctx->fb_pixels < px * 4) {
        if (ctx->comm->cstream) GSRT_HIP(ctx, hipStreamSynchronize(ctx->comm->cstream));  // unpack in flight
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
    gsrt::timing_mark(ctx, 0);
    if (N == 1 && !ctx->comm->comm) {  // one rank without a communicator: straight into the framebuffer
        gsrt_status s1 = gsrt::launch_render(sc, *ubo, plan, ctx->d_fb, nullptr);
        gsrt::timing_mark(ctx, 3);
        return s1;
    }
    gsrt_comm_state* cs = ctx->comm;
    const uint32_t per_rank = gsrt::max_local_tiles(plan);  // packed stride of every rank in the gather
    const size_t tile_floats = 4ull * plan.tw * plan.th;
    const size_t send_floats = per_rank * tile_floats;
    if (cs->packed_floats < send_floats) {
        GSRT_HIP(ctx, hipDeviceSynchronize());  // the old buffers may still be in flight
        for (int p = 0; p < 2; ++p) {
            (void)hipFree(cs->packed[p]);
            cs->packed[p] = nullptr;
        }
        cs->packed_floats = 0;
        for (int p = 0; p < 2; ++p) GSRT_HIP(ctx, hipMalloc(&cs->packed[p], sizeof(float) * send_floats));
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
    const uint32_t p = cs->parity;
    cs->parity ^= 1u;
    cs->last_p = p;
    // render into packed[p] once the gather two frames back has sent it; packed[p] is this frame's own buffer, so
    // its render kernel need not follow the previous frame's (slot streams)
    plan.packed = true;
    gsrt::RenderSync rsy;
    rsy.slot = gsrt::use_slot_streams(ctx, PN > 1);
    rsy.private_out = true;
    rsy.wait = cs->gathered[p];
    gsrt_status s = gsrt::launch_render(sc, *ubo, plan, cs->packed[p], nullptr, &rsy);
    if (s != GSRT_OK) return s;
    GSRT_HIP(ctx, hipEventRecord(cs->rendered[p], rsy.stream));
    // the gather on gstream, into gbuf[p] once the unpack two frames back has read it
    GSRT_HIP(ctx, hipStreamWaitEvent(cs->gstream, cs->rendered[p], 0));
    gsrt::timing_mark(ctx, 4, cs->gstream);  // the exchange starts once this rank's share is rendered
    if (root && cs->unpack_pending[p]) GSRT_HIP(ctx, hipStreamWaitEvent(cs->gstream, cs->unpacked[p], 0));
    float* const gb = R == 0 ? cs->gbuf[p] : nullptr;
    ncclResult_t r = ncclGather(cs->packed[p], gb, send_floats, ncclFloat32, 0, cs->comm, cs->gstream);
    if (r != ncclSuccess) return fail(ctx, GSRT_E_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
    if (emu && root)  // the other ranks' blocks landing in the gather buffer (stand-in for the receive)
        gsrt::launch_copy_d2d(cs->gstream, gb + send_floats, cs->inbound, sizeof(float) * send_floats * (PN - 1));
    GSRT_HIP(ctx, hipGetLastError());
    GSRT_HIP(ctx, hipEventRecord(cs->gathered[p], cs->gstream));
    if (root) {  // the unpack on cstream: overlaps the next frame's gather
        GSRT_HIP(ctx, hipStreamWaitEvent(cs->cstream, cs->gathered[p], 0));
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
        gsrt::timing_mark(ctx, 5, cs->cstream);
    } else {
        gsrt::timing_mark(ctx, 5, cs->gstream);
    }
    gsrt::timing_mark(ctx, 3);  // on the compute stream: the exchange overlaps the next frame
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out) {
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

gsrt_status gsrt_tile_plan(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, uint32_t out[8]) {
    if (!ubo || !out || nranks < 1 || rank < 0 || rank >= nranks || ubo->width == 0 || ubo->height == 0)
        return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)rank, (uint32_t)nranks);
    out[0] = p.tw;
    out[1] = p.th;
    out[2] = p.tiles_x;
    out[3] = p.tiles_y;
    out[4] = gsrt::local_tiles(p);
    out[5] = p.s_lanes;
    out[6] = p.run;
    out[7] = gsrt::max_local_tiles(p);
    return GSRT_OK;
}

gsrt_status gsrt_tile_deal(const gsrt_ubo* ubo, uint32_t mode, int nranks, uint32_t out[2]) {
    if (!ubo || !out || nranks < 1 || ubo->width == 0 || ubo->height == 0) return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks);
    out[0] = p.cq;
    out[1] = p.cs;
    return GSRT_OK;
}

// Host mirror of the sharded layout, from the same inline mappings the kernels use (gsrt_device.hpp): local tile
// lt of a rank is spatial tile global_pos(lt) (the packed render writes it to slot lt, pixel (y % th) tw + x % tw),
// and k_unpack finds pixel (x, y) at owner_of(spatial_index(x / tw, y / th)).
gsrt_status gsrt_tile_pack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, int rank, const float* rgba,
                                float* packed) {
    if (!ubo || !rgba || !packed || nranks < 1 || rank < 0 || rank >= nranks) return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)rank, (uint32_t)nranks);
    const uint32_t W = ubo->width, H = ubo->height, nl = gsrt::local_tiles(p), stride = gsrt::max_local_tiles(p);
    std::memset(packed, 0, sizeof(float) * 4ull * p.tw * p.th * stride);
    for (uint32_t lt = 0; lt < nl; ++lt) {
        uint32_t tx, ty;
        gsrt::spatial_tile(gsrt::global_pos(lt, (uint32_t)rank, gsrt::deal_of(p)), p.tiles_x, p.tiles_y, tx, ty);
        for (uint32_t q = 0; q < p.tw * p.th; ++q) {
            const uint32_t x = tx * p.tw + q % p.tw, y = ty * p.th + q / p.tw;
            if (x < W && y < H)
                std::memcpy(packed + 4 * ((size_t)lt * p.tw * p.th + q), rgba + 4 * ((size_t)y * W + x), 16);
        }
    }
    return GSRT_OK;
}

gsrt_status gsrt_tile_unpack_host(const gsrt_ubo* ubo, uint32_t mode, int nranks, const float* gathered,
                                  float* rgba_out) {
    if (!ubo || !gathered || !rgba_out || nranks < 1) return GSRT_E_ARG;
    const gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks);
    const uint32_t W = ubo->width, H = ubo->height, stride = gsrt::max_local_tiles(p);
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            uint32_t r, lt;
            gsrt::owner_of(gsrt::spatial_index(x / p.tw, y / p.th, p.tiles_x, p.tiles_y), gsrt::deal_of(p), r, lt);
            const size_t src = ((size_t)r * stride + lt) * p.tw * p.th + (y % p.th) * p.tw + (x % p.tw);
            std::memcpy(rgba_out + 4 * ((size_t)y * W + x), gathered + 4 * src, 16);
        }
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded_emulated(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                         float* rgba_out) {
    if (!sc || !ubo || !rgba_out || nranks < 1) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (!sc->bvh_built) return fail(ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
    if (sc->ntri && (mode & 0xffu) != GSRT_MODE_REF)
        return fail(ctx, GSRT_E_ARG, "triangle meshes are co-traced in REF mode only");
    (void)hipSetDevice(ctx->device);
    const gsrt::RenderPlan p0 = gsrt::make_plan(*ubo, mode, 0, 0, (uint32_t)nranks);
    const uint32_t per_rank = gsrt::max_local_tiles(p0);
    const size_t tile_floats = 4ull * p0.tw * p0.th;
    const size_t px = (size_t)ubo->width * ubo->height;
    float *gather = nullptr, *fb = nullptr;
    GSRT_HIP(ctx, hipMalloc(&gather, sizeof(float) * tile_floats * per_rank * nranks));
    if (hipMalloc(&fb, sizeof(float) * 4 * px) != hipSuccess) {
        (void)hipFree(gather);
        return fail(ctx, GSRT_E_OOM, "emulated gather: allocation failed");
    }
    gsrt_status s = GSRT_OK;
    for (int r = 0; r < nranks && s == GSRT_OK; ++r) {
        gsrt::RenderPlan p = gsrt::make_plan(*ubo, mode, 0, (uint32_t)r, (uint32_t)nranks);
        p.packed = true;
        s = gsrt::launch_render(sc, *ubo, p, gather + (size_t)r * per_rank * tile_floats, nullptr);
    }
    if (s == GSRT_OK) {
        gsrt::launch_unpack(ctx->stream, gather, fb, p0, ubo->width, ubo->height, per_rank);
        if (hipMemcpyAsync(rgba_out, fb, sizeof(float) * 4 * px, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "emulated gather: copy failed");
    }
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(gather);
    (void)hipFree(fb);
    if (s == GSRT_OK) s = gsrt::check_error_word(ctx);
    return s;
}

}  // extern "C"
