// gsrt_comm.cpp -- multi-GPU tile sharding.
//
// One process per GPU. The scene and its LBVH are replicated (each rank builds its own); the frame's
// tiles, in spatial order, are dealt round-robin over ranks in runs (whole 16x16-tile super-tiles on large
// frames, single tiles on small ones: RenderPlan::run), each rank renders its tiles into a packed buffer,
// and one ncclGather over xGMI brings the packed tiles to rank 0, which unpacks them into its framebuffer.
// The gather is the only exchange step; rendering needs no communication.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "gsrt_internal.hpp"

struct gsrt_comm_state {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
};

using gsrt::fail;

extern "C" {

void gsrt_comm_destroy_internal(gsrt_ctx* ctx) {
    if (!ctx || !ctx->comm) return;
    if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
    delete ctx->comm;
    ctx->comm = nullptr;
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
    if (nranks > 1) {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        ncclResult_t r = ncclCommInitRank(&st->comm, nranks, uid, rank);
        if (r != ncclSuccess) {
            delete st;
            return fail(ctx, GSRT_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
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
    (void)hipSetDevice(ctx->device);
    const int N = ctx->comm->nranks, R = ctx->comm->rank;
    gsrt::RenderPlan plan = gsrt::make_plan(*ubo, mode, k, (uint32_t)R, (uint32_t)N);
    const size_t px = (size_t)ubo->width * ubo->height;
    if (ctx->fb_pixels < px * 4) {
        (void)hipFree(ctx->d_fb);
        ctx->d_fb = nullptr;
        ctx->fb_pixels = 0;
        GSRT_HIP(ctx, hipMalloc(&ctx->d_fb, sizeof(float) * 4 * px));
        ctx->fb_pixels = px * 4;
    }
    ctx->last_w = ubo->width;
    ctx->last_h = ubo->height;
    ctx->last_stats = false;
    gsrt::timing_mark(ctx, 0);
    if (N == 1) {
        gsrt_status s1 = gsrt::launch_render(sc, *ubo, plan, ctx->d_fb, nullptr);
        gsrt::timing_mark(ctx, 3);
        return s1;
    }
    const uint32_t per_rank = gsrt::max_local_tiles(plan);  // packed stride of every rank in the gather
    const size_t tile_floats = 4ull * plan.tw * plan.th;
    const size_t send_floats = per_rank * tile_floats;
    if (ctx->packed_floats < send_floats) {
        (void)hipFree(ctx->d_packed);
        ctx->d_packed = nullptr;
        GSRT_HIP(ctx, hipMalloc(&ctx->d_packed, sizeof(float) * send_floats));
        ctx->packed_floats = send_floats;
    }
    if (R == 0 && ctx->gather_floats < send_floats * N) {
        (void)hipFree(ctx->d_gather);
        ctx->d_gather = nullptr;
        GSRT_HIP(ctx, hipMalloc(&ctx->d_gather, sizeof(float) * send_floats * N));
        ctx->gather_floats = send_floats * N;
    }
    plan.packed = true;
    gsrt_status s = gsrt::launch_render(sc, *ubo, plan, ctx->d_packed, nullptr);
    if (s != GSRT_OK) return s;
    ncclResult_t r = ncclGather(ctx->d_packed, R == 0 ? ctx->d_gather : nullptr, send_floats, ncclFloat32, 0,
                                ctx->comm->comm, ctx->stream);
    if (r != ncclSuccess) return fail(ctx, GSRT_E_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
    if (R == 0) gsrt::launch_unpack(ctx->stream, ctx->d_gather, ctx->d_fb, plan, ubo->width, ubo->height, per_rank);
    GSRT_HIP(ctx, hipGetLastError());
    gsrt::timing_mark(ctx, 3);
    return GSRT_OK;
}

gsrt_status gsrt_render_sharded(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out) {
    gsrt_status s = gsrt_render_sharded_async(sc, ubo, mode, k);
    if (s != GSRT_OK) return s;
    gsrt_ctx* ctx = sc->ctx;
    if (rgba_out && ctx->comm->rank == 0) {
        hipPointerAttribute_t attr;
        bool dev = hipPointerGetAttributes(&attr, rgba_out) == hipSuccess && attr.type == hipMemoryTypeDevice;
        (void)hipGetLastError();
        GSRT_HIP(ctx, hipMemcpyAsync(rgba_out, ctx->d_fb, sizeof(float) * 4 * ubo->width * ubo->height,
                                     dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
    }
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GSRT_OK;
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

gsrt_status gsrt_render_sharded_emulated(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, int nranks,
                                         float* rgba_out) {
    if (!sc || !ubo || !rgba_out || nranks < 1) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (!sc->bvh_built) return fail(ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
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
    return s;
}

}  // extern "C"
