// gsrt_comm.cpp -- multi-GPU tile sharding.
//
// One process per GPU. The scene and its LBVH are replicated (each rank builds its own); the frame's
// tiles, in spatial order, are dealt round-robin over ranks in runs (whole 16x16-tile super-tiles on large
// frames, single tiles on small ones: RenderPlan::run), each rank renders its tiles into a packed buffer,
// and one ncclGather over xGMI brings the packed tiles to rank 0, which unpacks them into its framebuffer.
// The gather is the only exchange step; rendering needs no communication. The gather and the unpack run on
// their own stream from one of two packed buffers, so frame k's exchange overlaps frame k+1's rendering.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>

#include "gsrt_internal.hpp"

struct gsrt_comm_state {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    hipStream_t cstream = nullptr;       // gather + unpack
    hipEvent_t rendered[2] = {nullptr, nullptr};  // packed[p] written (compute stream)
    hipEvent_t gathered[2] = {nullptr, nullptr};  // packed[p] sent (comm stream): free for reuse
    float* packed[2] = {nullptr, nullptr};
    size_t packed_floats = 0;
    uint32_t parity = 0;
};

using gsrt::fail;

extern "C" {

void gsrt_comm_destroy_internal(gsrt_ctx* ctx) {
    if (!ctx || !ctx->comm) return;
    gsrt_comm_state* c = ctx->comm;
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (int p = 0; p < 2; ++p) {
        if (c->rendered[p]) (void)hipEventDestroy(c->rendered[p]);
        if (c->gathered[p]) (void)hipEventDestroy(c->gathered[p]);
        (void)hipFree(c->packed[p]);
    }
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    delete c;
    ctx->comm = nullptr;
}

// the comm stream of ctx (nullptr without a communicator): gsrt_synchronize waits for it too
hipStream_t gsrt_comm_stream_internal(gsrt_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->cstream : nullptr; }

void* gsrt_comm_stream(gsrt_ctx* ctx) { return gsrt_comm_stream_internal(ctx); }

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
        bool ok = hipStreamCreateWithFlags(&st->cstream, hipStreamNonBlocking) == hipSuccess;
        for (int p = 0; p < 2 && ok; ++p)
            ok = hipEventCreateWithFlags(&st->rendered[p], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&st->gathered[p], hipEventDisableTiming) == hipSuccess;
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
    gsrt::RenderPlan plan = gsrt::make_plan(*ubo, mode, k, (uint32_t)R, (uint32_t)N);
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
    if (R == 0 && ctx->gather_floats < send_floats * N) {
        GSRT_HIP(ctx, hipStreamSynchronize(cs->cstream));
        (void)hipFree(ctx->d_gather);
        ctx->d_gather = nullptr;
        GSRT_HIP(ctx, hipMalloc(&ctx->d_gather, sizeof(float) * send_floats * N));
        ctx->gather_floats = send_floats * N;
    }
    const uint32_t p = cs->parity;
    cs->parity ^= 1u;
    // render into packed[p] once the gather two frames back has sent it; packed[p] is this frame's own buffer, so
    // its render kernel need not follow the previous frame's (slot streams)
    plan.packed = true;
    gsrt::RenderSync rsy;
    rsy.slot = gsrt::use_slot_streams(ctx, N > 1);
    rsy.private_out = true;
    rsy.wait = cs->gathered[p];
    gsrt_status s = gsrt::launch_render(sc, *ubo, plan, cs->packed[p], nullptr, &rsy);
    if (s != GSRT_OK) return s;
    GSRT_HIP(ctx, hipEventRecord(cs->rendered[p], rsy.stream));
    // exchange on the comm stream: gather to rank 0, unpack into its framebuffer
    GSRT_HIP(ctx, hipStreamWaitEvent(cs->cstream, cs->rendered[p], 0));
    ncclResult_t r = ncclGather(cs->packed[p], R == 0 ? ctx->d_gather : nullptr, send_floats, ncclFloat32, 0,
                                cs->comm, cs->cstream);
    if (r != ncclSuccess) return fail(ctx, GSRT_E_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
    if (R == 0) gsrt::launch_unpack(cs->cstream, ctx->d_gather, ctx->d_fb, plan, ubo->width, ubo->height, per_rank);
    GSRT_HIP(ctx, hipGetLastError());
    GSRT_HIP(ctx, hipEventRecord(cs->gathered[p], cs->cstream));
    gsrt::timing_mark(ctx, 3);  // on the compute stream: the exchange overlaps the next frame
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out) {
    gsrt_status s = gsrt_render_sharded_async(sc, ubo, mode, k);
    if (s != GSRT_OK) return s;
    gsrt_ctx* ctx = sc->ctx;
    if (ctx->comm->cstream) GSRT_HIP(ctx, hipStreamSynchronize(ctx->comm->cstream));
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
        gsrt::spatial_tile(gsrt::global_pos(lt, (uint32_t)rank, (uint32_t)nranks, p.run), p.tiles_x, p.tiles_y, tx, ty);
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
            gsrt::owner_of(gsrt::spatial_index(x / p.tw, y / p.th, p.tiles_x, p.tiles_y), (uint32_t)nranks, p.run, r, lt);
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
