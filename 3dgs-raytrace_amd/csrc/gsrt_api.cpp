// gsrt_api.cpp -- the C ABI (include/gsrt.h): context, scene upload, LBVH, render, stats.
#include <algorithm>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "gsrt_internal.hpp"

using gsrt::fail;

namespace {

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

template <class T>
gsrt_status grow(gsrt_ctx* ctx, T** p, size_t* have, size_t need) {
    if (*have >= need && *p) return GSRT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipMalloc(p, sizeof(T) * need) != hipSuccess) return fail(ctx, GSRT_E_OOM, "device allocation failed");
    *have = need;
    return GSRT_OK;
}

gsrt_status upload_common(gsrt_ctx* ctx, uint32_t n, const float* sh, gsrt_scene* sc) {
    sc->d_buf[0][0] = sc->d_params;
    sc->d_buf[1][0] = sc->d_aabbs;
    if (gsrt_status s = gsrt::lbvh_alloc(sc); s != GSRT_OK) return s;  // the BVH's buffers: a build allocates nothing
    GSRT_HIP(ctx, hipMalloc(&sc->d_flags, sizeof(uint32_t) * 4));
    GSRT_HIP(ctx, hipMemset(sc->d_flags, 0, sizeof(uint32_t) * 4));
    GSRT_HIP(ctx, hipMalloc(&sc->d_recs[0], sizeof(gsrt::SplatRec) * (n ? n : 1)));  // [1]: on the first COR frame
    GSRT_HIP(ctx, hipMalloc(&sc->d_keyed[0], sizeof(uint32_t) * ((n + 31) / 32 + 1)));
    GSRT_HIP(ctx, hipMemset(sc->d_keyed[0], 0xFF, sizeof(uint32_t) * ((n + 31) / 32 + 1)));
    if (sh) {
        // API layout [gauss][coef 16][rgb] -> device layout [gauss][rgb][coef 16]: one colour channel is 64
        // contiguous bytes, read as four 16-B LDS broadcasts by the blend loop. Word 0 of a channel holds the
        // ray-independent part of the colour, (s_0 Y_0) + 0.5 (Y_0 = 0.28209479 the constant DC basis), which
        // the shading loop's fma chain over k = 1..15 starts from (the COR colour's order, oracle sh_color)
        std::vector<float> t(48ull * n);
        for (size_t i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) {
                t[48 * i + 16 * c] = sh[48 * i + c] * gsrt::kShY0 + 0.5f;
                for (int k = 1; k < 16; ++k) t[48 * i + 16 * c + k] = sh[48 * i + 3 * k + c];
            }
        GSRT_HIP(ctx, hipMalloc(&sc->d_sh, sizeof(float) * 48ull * n));
        GSRT_HIP(ctx, hipMemcpy(sc->d_sh, t.data(), sizeof(float) * 48ull * n, hipMemcpyHostToDevice));
    }
    return GSRT_OK;
}

}  // namespace

namespace gsrt {
gsrt_status sync_all(gsrt_ctx* ctx) {
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->ustream) GSRT_HIP(ctx, hipStreamSynchronize(ctx->ustream));
    for (uint32_t j = 0; j < kStreamSlots; ++j)
        for (hipStream_t p : {ctx->prep_hi[j], ctx->prep_lo[j]})
            if (p) GSRT_HIP(ctx, hipStreamSynchronize(p));
    return GSRT_OK;
}

gsrt_status wait_updates(gsrt_ctx* ctx, hipStream_t s) {
    if (!ctx->copy_unseen) return GSRT_OK;
    const hipStream_t streams[5] = {ctx->prep_hi[0], ctx->prep_hi[1], ctx->prep_lo[0], ctx->prep_lo[1], ctx->stream};
    for (uint32_t i = 0; i < 5; ++i)
        if (streams[i] == s && ((ctx->copy_unseen >> i) & 1u)) {
            GSRT_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_copied, 0));
            ctx->copy_unseen &= ~(1u << i);
        }
    return GSRT_OK;
}

gsrt_status check_error_word(gsrt_ctx* ctx) {
    gsrt_status s = sync_all(ctx);
    if (s != GSRT_OK) return s;
    unsigned long long err = 0;
    GSRT_HIP(ctx, hipMemcpy(&err, ctx->d_counters + kErrWord, sizeof err, hipMemcpyDeviceToHost));
    if (!err) return GSRT_OK;
    // cleared on the render stream and waited for here, inside the sync window: the ctx's streams are non-blocking,
    // so a null-stream memset would not be ordered against the next frame's kernels (which atomicOr this word)
    GSRT_HIP(ctx, hipMemsetAsync(ctx->d_counters + kErrWord, 0, sizeof err, ctx->stream));
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return fail(ctx, GSRT_E_DEVICE, "render: traversal stack overflow (a frame since the last check is incomplete)");
}

void timing_mark(gsrt_ctx* ctx, int which, hipStream_t s) {
    if (ctx->timing_n >= ctx->timing_cap) return;
    const bool rec = ctx->timing_frame % ctx->timing_stride == 0;  // this frame is a sampled one
    if (rec) {
        if (!(ctx->timing_kernel_only && (which == 0 || which == 3)))
            (void)hipEventRecord(ctx->events[kTimingEvents * ctx->timing_n + which], s ? s : ctx->stream);
        if (which == 0) ctx->timing_ex[ctx->timing_n] = 0;
        if (which == 4) ctx->timing_ex[ctx->timing_n] = 1;
    }
    if (which == 3) {
        if (rec) ++ctx->timing_n;
        ++ctx->timing_frame;
    }
}
}  // namespace gsrt

extern "C" {

int gsrt_abi_version(void) { return GSRT_ABI_VERSION; }

const char* gsrt_status_string(gsrt_status s) {
    switch (s) {
        case GSRT_OK: return "ok";
        case GSRT_E_ARG: return "invalid argument";
        case GSRT_E_OOM: return "out of memory";
        case GSRT_E_DEVICE: return "device error";
        case GSRT_E_IO: return "i/o error";
        case GSRT_E_STATE: return "invalid state";
        case GSRT_E_COMM: return "communication error";
    }
    return "unknown";
}

gsrt_status gsrt_create(gsrt_ctx** out, int device) {
    if (!out) return GSRT_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
        (void)hipGetLastError();
        return GSRT_E_DEVICE;
    }
    gsrt_ctx* ctx = new (std::nothrow) gsrt_ctx();
    if (!ctx) return GSRT_E_OOM;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return GSRT_E_DEVICE;
    }
    // the prep streams in two priority classes (kPrioLowAboveUs): pstream / fstream start at the highest
    // (test switch GSRT_DEBUG_PREP_PRIORITY=0: always the lowest, 1: always the highest, 2: switch every frame)
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    const char* pe = std::getenv("GSRT_DEBUG_PREP_PRIORITY");
    ctx->prep_high = !(pe && pe[0] == '0');
    bool ev_ok = true;
    for (uint32_t j = 0; j < kStreamSlots; ++j)
        ev_ok = ev_ok && hipStreamCreateWithPriority(&ctx->prep_hi[j], hipStreamNonBlocking, prio_greatest) == hipSuccess &&
                hipStreamCreateWithPriority(&ctx->prep_lo[j], hipStreamNonBlocking, prio_least) == hipSuccess &&
                hipEventCreateWithFlags(&ctx->ev_hop[j], kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&ctx->ev_side[j], kSyncEventFlags) == hipSuccess;
    // The update and comm streams are created here too, so that the context's streams always come in one order:
    // render (default priority), prep H / L / H / L, update (H), comm (default); RCCL's own stream follows at
    // gsrt_comm_init. A hardware queue of the process holds streams of one priority only, so the render and comm streams
    // are the context's only default-priority ones and share no queue with a prep or update stream
    // (profiles/r06/queue_map.txt). Test switch GSRT_DEBUG_LAZY_STREAMS=1: both created when first used, at the
    // default priority (the round-5 order)
    const char* lz = std::getenv("GSRT_DEBUG_LAZY_STREAMS");
    if (ev_ok && !(lz && lz[0] == '1'))
        ev_ok = hipStreamCreateWithPriority(&ctx->ustream, hipStreamNonBlocking, prio_greatest) == hipSuccess &&
                hipEventCreateWithFlags(&ctx->ev_copied, kSyncEventFlags) == hipSuccess &&
                hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking) == hipSuccess;
    if (ev_ok) {
        hipStream_t* set = ctx->prep_high ? ctx->prep_hi : ctx->prep_lo;
        ctx->pstream = set[0];
        ctx->fstream = set[1];
    }
    ev_ok = ev_ok &&
                 hipEventCreateWithFlags(&ctx->ev_fit, kSyncEventFlags) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->ev_front, kSyncEventFlags) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->ev_lists, kSyncEventFlags) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->ev_main, kSyncEventFlags) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->ev_serial, kSyncEventFlags) == hipSuccess;
    for (FrameSlot& S : ctx->slot)
        ev_ok = ev_ok && hipEventCreateWithFlags(&S.prepared, kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&S.rendered, kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&S.t0, kTimingEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&S.t1, kTimingEventFlags) == hipSuccess;
    if (!ev_ok) {
        gsrt_destroy(ctx);
        return GSRT_E_DEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->num_cus = prop.multiProcessorCount;
    if (hipMalloc(&ctx->d_counters, sizeof(unsigned long long) * gsrt::kCounters) != hipSuccess ||
        hipMalloc(&ctx->d_tile_counter, sizeof(uint32_t) * 4) != hipSuccess ||
        hipMalloc(&ctx->d_lut, sizeof(float) * 512) != hipSuccess) {
        gsrt_destroy(ctx);
        return GSRT_E_OOM;
    }
    float lut[512];
    gsrt::exp_lut(lut);
    if (hipMemcpy(ctx->d_lut, lut, sizeof lut, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(ctx->d_counters, 0, sizeof(unsigned long long) * gsrt::kCounters) != hipSuccess) {
        gsrt_destroy(ctx);
        return GSRT_E_DEVICE;
    }
    *out = ctx;
    return GSRT_OK;
}

void gsrt_comm_destroy_internal(gsrt_ctx* ctx);
hipStream_t gsrt_comm_stream_internal(gsrt_ctx* ctx);
gsrt_status gsrt_comm_sync_internal(gsrt_ctx* ctx);
gsrt_status gsrt_comm_fb_render_write(gsrt_ctx* ctx);

void gsrt_destroy(gsrt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    gsrt_comm_destroy_internal(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (uint32_t j = 0; j < kStreamSlots; ++j)
        for (hipStream_t p : {ctx->prep_hi[j], ctx->prep_lo[j]})
            if (p) (void)hipStreamSynchronize(p);
    if (ctx->ustream) {
        (void)hipStreamSynchronize(ctx->ustream);
        (void)hipStreamDestroy(ctx->ustream);
    }
    if (ctx->ev_copied) (void)hipEventDestroy(ctx->ev_copied);
    if (ctx->cstream) (void)hipStreamDestroy(ctx->cstream);  // (the communicator, which used it, is gone)
    (void)hipFree(ctx->d_fb);
    for (int p = 0; p < 2; ++p) {
        (void)hipFree(ctx->d_share[p]);
        if (ctx->ev_share[p]) (void)hipEventDestroy(ctx->ev_share[p]);
    }
    (void)hipFree(ctx->d_ray_stats);
    (void)hipFree(ctx->d_counters);
    (void)hipFree(ctx->d_tile_counter);
    (void)hipFree(ctx->d_lut);
    (void)hipFree(ctx->d_tri_t);
    for (FrameSlot& S : ctx->slot) {
        (void)hipFree(S.d_lists);
        (void)hipFree(S.d_list_hdr);
        (void)hipFree(S.d_glist);
        (void)hipFree(S.d_ghdr);
        (void)hipFree(S.d_frontier);
        if (S.prepared) (void)hipEventDestroy(S.prepared);
        if (S.rendered) (void)hipEventDestroy(S.rendered);
        if (S.t0) (void)hipEventDestroy(S.t0);
        if (S.t1) (void)hipEventDestroy(S.t1);
    }
    (void)hipFree(ctx->d_group_order);
    (void)hipFree(ctx->d_run_order);
    for (uint32_t j = 0; j < kSlots; ++j) (void)hipFree(ctx->d_tile_cost[j]);
    for (hipEvent_t e : ctx->events) (void)hipEventDestroy(e);
    if (ctx->ev_main) (void)hipEventDestroy(ctx->ev_main);
    if (ctx->ev_serial) (void)hipEventDestroy(ctx->ev_serial);
    if (ctx->ev_fit) (void)hipEventDestroy(ctx->ev_fit);
    if (ctx->ev_front) (void)hipEventDestroy(ctx->ev_front);
    if (ctx->ev_lists) (void)hipEventDestroy(ctx->ev_lists);
    for (uint32_t j = 0; j < kStreamSlots; ++j) {
        if (ctx->ev_hop[j]) (void)hipEventDestroy(ctx->ev_hop[j]);
        if (ctx->ev_side[j]) (void)hipEventDestroy(ctx->ev_side[j]);
        if (ctx->prep_hi[j]) (void)hipStreamDestroy(ctx->prep_hi[j]);
        if (ctx->prep_lo[j]) (void)hipStreamDestroy(ctx->prep_lo[j]);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* gsrt_last_error(const gsrt_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

gsrt_status gsrt_synchronize(gsrt_ctx* ctx) {
    if (!ctx) return GSRT_E_ARG;
    gsrt_status s = gsrt::sync_all(ctx);
    if (s != GSRT_OK) return s;
    if (gsrt_status cs = gsrt_comm_sync_internal(ctx); cs != GSRT_OK) return cs;
    return gsrt::check_error_word(ctx);
}

void* gsrt_stream(gsrt_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }
void* gsrt_prep_stream(gsrt_ctx* ctx) { return ctx ? (void*)ctx->pstream : nullptr; }

gsrt_status gsrt_debug_streams(gsrt_ctx* ctx, void* out[8], uint32_t* n) {
    if (!ctx || !out || !n) return GSRT_E_ARG;
    const hipStream_t s[7] = {ctx->stream, ctx->prep_hi[0], ctx->prep_lo[0], ctx->prep_hi[1], ctx->prep_lo[1],
                              ctx->ustream, gsrt_comm_stream_internal(ctx)};
    for (uint32_t i = 0; i < 7; ++i) out[i] = (void*)s[i];
    out[7] = nullptr;
    *n = 7;
    return GSRT_OK;
}

void* gsrt_update_stream(gsrt_ctx* ctx) {
    if (!ctx) return nullptr;
    (void)hipSetDevice(ctx->device);
    if (!ctx->ustream) {  // (created with the context, unless GSRT_DEBUG_LAZY_STREAMS)
        if (hipStreamCreateWithFlags(&ctx->ustream, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (hipEventCreateWithFlags(&ctx->ev_copied, kSyncEventFlags) != hipSuccess) return nullptr;
    }
    return (void*)ctx->ustream;
}

gsrt_status gsrt_scene_from_params(gsrt_ctx* ctx, const gsrt_gauss_param* params, const gsrt_aabb* aabbs, uint32_t n,
                                   const float* sh, gsrt_scene** out) {
    if (!ctx || !out || (n && (!params || !aabbs)) || n > GSRT_MAX_GAUSSIANS) return GSRT_E_ARG;
    *out = nullptr;
    (void)hipSetDevice(ctx->device);
    gsrt_scene* sc = new (std::nothrow) gsrt_scene();
    if (!sc) return GSRT_E_OOM;
    sc->ctx = ctx;
    sc->n = n;
    gsrt_status s = GSRT_OK;
    if (hipMalloc(&sc->d_params, sizeof(gsrt_gauss_param) * (n ? n : 1)) != hipSuccess ||
        hipMalloc(&sc->d_aabbs, sizeof(gsrt_aabb) * (n ? n : 1)) != hipSuccess) {
        gsrt_destroy_scene(sc);
        return fail(ctx, GSRT_E_OOM, "scene allocation failed");
    }
    if (n) {
        if (hipMemcpyAsync(sc->d_params, params, sizeof(gsrt_gauss_param) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(sc->d_aabbs, aabbs, sizeof(gsrt_aabb) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "scene upload failed");
    }
    if (s == GSRT_OK) s = upload_common(ctx, n, sh, sc);
    if (s == GSRT_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(ctx, GSRT_E_DEVICE, "scene upload sync");
    if (s != GSRT_OK) { gsrt_destroy_scene(sc); return s; }
    *out = sc;
    return GSRT_OK;
}

gsrt_status gsrt_scene_from_model(gsrt_ctx* ctx, const float* center, const float* rot, const float* scale,
                                  const float* opacity, const float* sh, uint32_t n, gsrt_scene** out) {
    if (!ctx || !out || (n && (!center || !rot || !scale || !opacity)) || n > GSRT_MAX_GAUSSIANS) return GSRT_E_ARG;
    *out = nullptr;
    (void)hipSetDevice(ctx->device);
    gsrt_scene* sc = new (std::nothrow) gsrt_scene();
    if (!sc) return GSRT_E_OOM;
    sc->ctx = ctx;
    sc->n = n;
    float* tmp = nullptr;  // center | rot | scale | opacity staged in one block (11 floats per Gaussian)
    gsrt_status s = GSRT_OK;
    const size_t nn = n ? n : 1;
    if (hipMalloc(&sc->d_params, sizeof(gsrt_gauss_param) * nn) != hipSuccess ||
        hipMalloc(&sc->d_aabbs, sizeof(gsrt_aabb) * nn) != hipSuccess ||
        hipMalloc(&tmp, sizeof(float) * 11 * nn) != hipSuccess) {
        (void)hipFree(tmp);
        gsrt_destroy_scene(sc);
        return fail(ctx, GSRT_E_OOM, "scene allocation failed");
    }
    if (n) {
        hipStream_t st = ctx->stream;
        if (hipMemcpyAsync(tmp, center, 12ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(tmp + 3ull * n, rot, 16ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(tmp + 7ull * n, scale, 12ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(tmp + 10ull * n, opacity, 4ull * n, hipMemcpyHostToDevice, st) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "scene upload failed");
        if (s == GSRT_OK) {
            gsrt::launch_cov3d(st, n, tmp, tmp + 3ull * n, tmp + 7ull * n, tmp + 10ull * n, sc->d_params, sc->d_aabbs);
            if (hipGetLastError() != hipSuccess) s = fail(ctx, GSRT_E_DEVICE, "cov3d launch failed");
        }
    }
    if (s == GSRT_OK) s = upload_common(ctx, n, sh, sc);
    if (s == GSRT_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) s = fail(ctx, GSRT_E_DEVICE, "scene build sync");
    (void)hipFree(tmp);
    if (s != GSRT_OK) { gsrt_destroy_scene(sc); return s; }
    *out = sc;
    return GSRT_OK;
}

gsrt_status gsrt_scene_download(gsrt_scene* sc, gsrt_gauss_param* params, gsrt_aabb* aabbs) {
    if (!sc) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    if (gsrt_status s = gsrt::sync_all(ctx); s != GSRT_OK) return s;  // updates are queued on the prep stream
    if (params && sc->n)
        GSRT_HIP(ctx, hipMemcpyAsync(params, sc->d_params, sizeof(gsrt_gauss_param) * sc->n, hipMemcpyDeviceToHost, ctx->stream));
    if (aabbs && sc->n)
        GSRT_HIP(ctx, hipMemcpyAsync(aabbs, sc->d_aabbs, sizeof(gsrt_aabb) * sc->n, hipMemcpyDeviceToHost, ctx->stream));
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GSRT_OK;
}

uint32_t gsrt_scene_size(const gsrt_scene* sc) { return sc ? sc->n : 0u; }

void gsrt_destroy_scene(gsrt_scene* sc) {
    if (!sc) return;
    if (sc->ctx) {
        (void)hipSetDevice(sc->ctx->device);
        (void)gsrt::sync_all(sc->ctx);
    }
    // borrowed arrays (gsrt_scene_attach) are the caller's
    if (sc->attached[0]) sc->d_params = nullptr;
    if (sc->attached[1]) sc->d_aabbs = nullptr;
    // (a scene that failed before upload_common holds its arrays in d_params / d_aabbs only)
    if (sc->d_params && sc->d_params != sc->d_buf[0][0] && sc->d_params != sc->d_buf[0][1]) (void)hipFree(sc->d_params);
    if (sc->d_aabbs && sc->d_aabbs != sc->d_buf[1][0] && sc->d_aabbs != sc->d_buf[1][1]) (void)hipFree(sc->d_aabbs);
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(sc->d_buf[a][b]);
            for (int k = 0; k < 3; ++k)
                if (sc->ev_ret[a][b][k]) (void)hipEventDestroy(sc->ev_ret[a][b][k]);
        }
    (void)hipFree(sc->d_sh);
    (void)hipFree(sc->d_flags);
    for (uint32_t b = 0; b < kSlots; ++b) {
        (void)hipFree(sc->d_recs[b]);
        (void)hipFree(sc->d_keyed[b]);
        (void)hipFree(sc->d_inband[b]);
        (void)hipFree(sc->d_footprint[b]);
    }
    for (uint32_t b = 0; b < kSlots; ++b) {
        (void)hipFree(sc->d_nodes[b]);
        (void)hipFree(sc->d_root_box[b]);
    }
    (void)hipFree(sc->d_leaf_parent);
    (void)hipFree(sc->d_node_parent);
    (void)hipFree(sc->d_gid_slot);
    (void)hipFree(sc->d_node_range);
    for (uint32_t b = 0; b < kSlots; ++b) {
        (void)hipFree(sc->d_fit_flags[b]);
        (void)hipFree(sc->d_fit_queue[b]);
    }
    (void)hipFree(sc->d_sort);
    (void)hipFree(sc->d_leaf_gid);
    (void)hipFree(sc->d_morton);
    (void)hipFree(sc->d_tris);
    (void)hipFree(sc->d_mesh_nodes);
    delete sc;
}

gsrt_status gsrt_build_bvh(gsrt_scene* sc) {
    if (!sc) return GSRT_E_ARG;
    (void)hipSetDevice(sc->ctx->device);
    gsrt::mark_main_dirty(sc->ctx);
    gsrt_status s = gsrt::sync_all(sc->ctx);  // a rebuild may reallocate nodes an in-flight frame still reads
    return s != GSRT_OK ? s : gsrt::lbvh_build(sc);
}

// The copies of gsrt_refit_bvh / gsrt_scene_update go on the prep stream: after the prep kernels of the frames
// already queued (their projection read the old arrays), before the next frame's prep; the pipelined render
// kernels never read d_params / d_aabbs. A REF or counting render still queued on the render stream does (its
// projection and fit run there): the copies then wait for it too. The fit itself is lazy (geom_version).
// A scene array (a = 0 params, 1 AABBs) replaced from a host or device source: the copy goes into the array's other
// buffer on the update stream, which waits only for the kernels that read that buffer while it was current (recorded
// when it was retired). The buffer then becomes current: frames enqueued from now on read it, and each stream waits for
// the copy before it next reads an array (wait_updates). So frame f+1's update copy overlaps frame f's fit, projection,
// lists and render instead of queueing behind them on the prep stream (the 8-rank C5 share's chain: copies 0.41 ms of
// ~0.97 ms per frame, profiles/r06). Device sources go through gsrt::launch_copy_d2d (one-wave workgroups that loop),
// not the runtime's blit kernel, which beside a running render kernel took 2.9 ms for C5's 360 MB update.
static gsrt_status update_array(gsrt_scene* sc, int a, const void* src, size_t bytes) {
    gsrt_ctx* ctx = sc->ctx;
    if (!gsrt_update_stream(ctx)) return fail(ctx, GSRT_E_DEVICE, "update stream creation failed");
    const uint32_t c = sc->cur[a], x = c ^ 1u;
    if (!sc->d_buf[a][x]) {
        GSRT_HIP(ctx, hipMalloc(&sc->d_buf[a][x], bytes));
        for (int k = 0; k < 3; ++k) GSRT_HIP(ctx, hipEventCreateWithFlags(&sc->ev_ret[a][x][k], kSyncEventFlags));
        for (int k = 0; k < 3; ++k) GSRT_HIP(ctx, hipEventCreateWithFlags(&sc->ev_ret[a][c][k], kSyncEventFlags));
    }
    for (int k = 0; k < 3; ++k)
        if (sc->ret_rec[a][x][k]) GSRT_HIP(ctx, hipStreamWaitEvent(ctx->ustream, sc->ev_ret[a][x][k], 0));
    if (is_device_ptr(src)) {
        gsrt::launch_copy_d2d(ctx->ustream, sc->d_buf[a][x], src, bytes);
        GSRT_HIP(ctx, hipGetLastError());
    } else {
        GSRT_HIP(ctx, hipMemcpyAsync(sc->d_buf[a][x], src, bytes, hipMemcpyHostToDevice, ctx->ustream));
    }
    GSRT_HIP(ctx, hipEventRecord(ctx->ev_copied, ctx->ustream));
    ctx->copy_unseen = 0x1Fu;
    // retire the current buffer: where its readers stand on the prep streams (pipelined frames' fits and projections;
    // in slot-stream mode the second one's too) and, after a REF / counting frame, on the render stream
    const hipStream_t rs[3] = {ctx->pstream, ctx->fstream, ctx->stream};
    for (int k = 0; k < 3; ++k) {
        sc->ret_rec[a][c][k] = k < 2 || ctx->serial_reads;
        if (sc->ret_rec[a][c][k]) GSRT_HIP(ctx, hipEventRecord(sc->ev_ret[a][c][k], rs[k]));
    }
    sc->cur[a] = x;
    sc->attached[a] = nullptr;
    if (a == 0) sc->d_params = static_cast<gsrt_gauss_param*>(sc->d_buf[a][x]);
    else sc->d_aabbs = static_cast<gsrt_aabb*>(sc->d_buf[a][x]);
    ctx->scene_moved = true;
    return GSRT_OK;
}

// With slot streams, frames of slot 1 run on their own stream (fstream): the copies also wait for those
// queued there, and the next frame on each of those streams waits for the copies (launch_render).
static gsrt_status order_update(gsrt_ctx* ctx) {
    ctx->scene_moved = true;
    for (uint32_t j = 1; j < kStreamSlots; ++j) {
        if (ctx->side_frames[j]) {
            GSRT_HIP(ctx, hipEventRecord(ctx->ev_side[j], gsrt::slot_stream(ctx, j)));
            GSRT_HIP(ctx, hipStreamWaitEvent(ctx->pstream, ctx->ev_side[j], 0));
            ctx->side_frames[j] = false;
        }
        ctx->side_updates[j] = true;
    }
    if (!ctx->serial_pending) return GSRT_OK;
    GSRT_HIP(ctx, hipEventRecord(ctx->ev_serial, ctx->stream));
    GSRT_HIP(ctx, hipStreamWaitEvent(ctx->pstream, ctx->ev_serial, 0));
    ctx->serial_pending = false;
    return GSRT_OK;
}

gsrt_status gsrt_refit_bvh(gsrt_scene* sc, const gsrt_aabb* aabbs) {
    if (!sc) return GSRT_E_ARG;
    if (!sc->bvh_built) return fail(sc->ctx, GSRT_E_STATE, "refit before build");
    gsrt_ctx* ctx = sc->ctx;
    (void)hipSetDevice(ctx->device);
    if (aabbs && sc->n) {
        if (gsrt_status s = update_array(sc, 1, aabbs, sizeof(gsrt_aabb) * sc->n); s != GSRT_OK) return s;
        ++sc->aabb_version;
    }
    ctx->scene_moved = true;
    ctx->serial_reads = false;
    ++sc->geom_version;
    return GSRT_OK;
}

gsrt_status gsrt_scene_update(gsrt_scene* sc, const gsrt_gauss_param* params, const gsrt_aabb* aabbs) {
    if (!sc) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    (void)hipSetDevice(ctx->device);
    if (!sc->n) return GSRT_OK;
    if (params)
        if (gsrt_status s = update_array(sc, 0, params, sizeof(gsrt_gauss_param) * sc->n); s != GSRT_OK) return s;
    if (aabbs) {
        if (gsrt_status s = update_array(sc, 1, aabbs, sizeof(gsrt_aabb) * sc->n); s != GSRT_OK) return s;
        ++sc->aabb_version;  // the in-band bitmaps follow the AABBs
    }
    ctx->serial_reads = false;
    return GSRT_OK;
}

// Borrowed arrays: the scene's pointer is the caller's array, so frames read it in place (no copy, no second
// buffer). The update stream's current point is recorded for the frame streams to wait on, as after a copy: a producer
// on the GPU fills the array there. The scene's own current buffer keeps its retire events; the next copy into the
// other buffer (an update, or the copy of the borrowed array itself at detach / stream_pages) retires it then.
gsrt_status gsrt_scene_attach(gsrt_scene* sc, const gsrt_gauss_param* params, const gsrt_aabb* aabbs) {
    if (!sc) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    (void)hipSetDevice(ctx->device);
    const void* src[2] = {params, aabbs};
    for (int a = 0; a < 2; ++a)
        if (src[a] && (!is_device_ptr(src[a]) || reinterpret_cast<uintptr_t>(src[a]) % 16u))
            return fail(ctx, GSRT_E_ARG, "attach: an array is not a 16-byte aligned device pointer");
    if (!sc->n || (!params && !aabbs)) return GSRT_OK;
    if (!gsrt_update_stream(ctx)) return fail(ctx, GSRT_E_DEVICE, "update stream creation failed");
    GSRT_HIP(ctx, hipEventRecord(ctx->ev_copied, ctx->ustream));
    ctx->copy_unseen = 0x1Fu;
    if (params) {
        sc->attached[0] = params;
        sc->d_params = const_cast<gsrt_gauss_param*>(params);
    }
    if (aabbs) {
        sc->attached[1] = aabbs;
        sc->d_aabbs = const_cast<gsrt_aabb*>(aabbs);
        ++sc->aabb_version;
    }
    ctx->scene_moved = true;
    return GSRT_OK;
}

// copy borrowed arrays into the scene's own buffers (update_array: the copy ends the borrow)
static gsrt_status take_attached(gsrt_scene* sc) {
    const size_t bytes[2] = {sizeof(gsrt_gauss_param) * sc->n, sizeof(gsrt_aabb) * sc->n};
    for (int a = 0; a < 2; ++a)
        if (sc->attached[a])
            if (gsrt_status s = update_array(sc, a, sc->attached[a], bytes[a]); s != GSRT_OK) return s;
    return GSRT_OK;
}

gsrt_status gsrt_scene_detach(gsrt_scene* sc) {
    if (!sc) return GSRT_E_ARG;
    (void)hipSetDevice(sc->ctx->device);
    if (gsrt_status s = take_attached(sc); s != GSRT_OK) return s;
    return gsrt::sync_all(sc->ctx);  // the copies and every frame that read the caller's arrays are done
}

uint32_t gsrt_scene_pages(const gsrt_scene* sc) {
    return sc ? (sc->n + GSRT_PAGE_GAUSSIANS - 1) / GSRT_PAGE_GAUSSIANS : 0u;
}

gsrt_status gsrt_scene_stream_pages(gsrt_scene* sc, const gsrt_gauss_param* params, const gsrt_aabb* aabbs,
                                    const uint32_t* pages, uint32_t npages) {
    if (!sc || (npages && !pages)) return GSRT_E_ARG;
    gsrt_ctx* ctx = sc->ctx;
    const uint32_t np = gsrt_scene_pages(sc);
    for (uint32_t i = 0; i < npages; ++i)
        if (pages[i] >= np) return fail(ctx, GSRT_E_ARG, "page id out of range");
    if (!npages || (!params && !aabbs)) return GSRT_OK;
    (void)hipSetDevice(ctx->device);
    if (gsrt_status s = take_attached(sc); s != GSRT_OK) return s;  // pages land in the scene's own arrays
    if (gsrt_status s = order_update(ctx); s != GSRT_OK) return s;
    if (gsrt_status s = gsrt::wait_updates(ctx, ctx->pstream); s != GSRT_OK) return s;  // an update's copy into them
    // runs of consecutive page ids (in the order given) become one transfer per array
    std::vector<uint32_t> ids(pages, pages + npages);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const hipMemcpyKind kp = params && is_device_ptr(params) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const hipMemcpyKind ka = aabbs && is_device_ptr(aabbs) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    for (size_t i = 0; i < ids.size();) {
        size_t j = i + 1;
        while (j < ids.size() && ids[j] == ids[j - 1] + 1) ++j;
        const size_t g0 = (size_t)ids[i] * GSRT_PAGE_GAUSSIANS;
        const size_t g1 = std::min<size_t>((size_t)(ids[j - 1] + 1) * GSRT_PAGE_GAUSSIANS, sc->n);
        if (params && kp == hipMemcpyDeviceToDevice)
            gsrt::launch_copy_d2d(ctx->pstream, sc->d_params + g0, params + g0, sizeof(gsrt_gauss_param) * (g1 - g0));
        else if (params)
            GSRT_HIP(ctx, hipMemcpyAsync(sc->d_params + g0, params + g0, sizeof(gsrt_gauss_param) * (g1 - g0), kp, ctx->pstream));
        if (aabbs && ka == hipMemcpyDeviceToDevice)
            gsrt::launch_copy_d2d(ctx->pstream, sc->d_aabbs + g0, aabbs + g0, sizeof(gsrt_aabb) * (g1 - g0));
        else if (aabbs)
            GSRT_HIP(ctx, hipMemcpyAsync(sc->d_aabbs + g0, aabbs + g0, sizeof(gsrt_aabb) * (g1 - g0), ka, ctx->pstream));
        GSRT_HIP(ctx, hipGetLastError());
        i = j;
    }
    if (aabbs)
        ++sc->aabb_version;  // the in-band bitmaps follow the AABBs
    return GSRT_OK;
}

gsrt_status gsrt_host_register(gsrt_ctx* ctx, void* ptr, size_t bytes) {
    if (!ctx || !ptr || !bytes) return GSRT_E_ARG;
    (void)hipSetDevice(ctx->device);
    GSRT_HIP(ctx, hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return GSRT_OK;
}

gsrt_status gsrt_host_unregister(gsrt_ctx* ctx, void* ptr) {
    if (!ctx || !ptr) return GSRT_E_ARG;
    (void)hipSetDevice(ctx->device);
    GSRT_HIP(ctx, hipHostUnregister(ptr));
    return GSRT_OK;
}

// the BVH as the last rendered slot holds it, fitted to the current geometry (bvh_info / bvh_download)
static gsrt_status settled_bvh_slot(gsrt_scene* sc, uint32_t* slot) {
    gsrt_ctx* ctx = sc->ctx;
    gsrt_status s = gsrt::sync_all(ctx);
    if (s != GSRT_OK) return s;
    *slot = sc->last_slot;
    s = gsrt::lbvh_fit_if_stale(sc, *slot, ctx->stream, true);  // with the leaf AABBs (not a frame's footprints)
    if (s != GSRT_OK) return s;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return GSRT_OK;
}

gsrt_status gsrt_bvh_info(gsrt_scene* sc, uint32_t* n_internal, float root_box[6], uint32_t* max_depth) {
    if (!sc) return GSRT_E_ARG;
    if (!sc->bvh_built) return fail(sc->ctx, GSRT_E_STATE, "bvh not built");
    if (n_internal) *n_internal = sc->n > 1 ? sc->n - 1 : 0;
    uint32_t slot = 0;
    gsrt_status st = settled_bvh_slot(sc, &slot);
    if (st != GSRT_OK) return st;
    if (root_box) {
        if (sc->n) GSRT_HIP(sc->ctx, hipMemcpy(root_box, sc->d_root_box[slot], sizeof(float) * 6, hipMemcpyDeviceToHost));
        else std::memset(root_box, 0, sizeof(float) * 6);
    }
    if (max_depth) {
        uint32_t depth = 0;
        if (sc->n > 1) {
            std::vector<gsrt::BvhNode> nodes(sc->n - 1);
            gsrt_ctx* ctx = sc->ctx;
            GSRT_HIP(ctx, hipMemcpy(nodes.data(), sc->d_nodes[slot], sizeof(gsrt::BvhNode) * nodes.size(), hipMemcpyDeviceToHost));
            std::vector<uint32_t> d(nodes.size(), 0);
            std::vector<uint32_t> stack{0};
            d[0] = 1;
            while (!stack.empty()) {
                uint32_t i = stack.back();
                stack.pop_back();
                for (uint32_t ref : {nodes[i].l_ref, nodes[i].r_ref}) {
                    if (ref & gsrt::kLeafBit) depth = std::max(depth, d[i] + 1);
                    else if (ref < nodes.size()) { d[ref] = d[i] + 1; stack.push_back(ref); }
                }
            }
        } else if (sc->n == 1) {
            depth = 1;
        }
        *max_depth = depth;
    }
    return GSRT_OK;
}

gsrt_status gsrt_bvh_download(gsrt_scene* sc, uint32_t* nodes, uint32_t* leaf_gid, uint32_t* morton) {
    if (!sc) return GSRT_E_ARG;
    if (!sc->bvh_built) return fail(sc->ctx, GSRT_E_STATE, "bvh not built");
    gsrt_ctx* ctx = sc->ctx;
    uint32_t slot = 0;
    gsrt_status st = settled_bvh_slot(sc, &slot);
    if (st != GSRT_OK) return st;
    if (nodes && sc->n > 1) GSRT_HIP(ctx, hipMemcpy(nodes, sc->d_nodes[slot], sizeof(gsrt::BvhNode) * (sc->n - 1), hipMemcpyDeviceToHost));
    if (leaf_gid && sc->n) GSRT_HIP(ctx, hipMemcpy(leaf_gid, sc->d_leaf_gid, 4ull * sc->n, hipMemcpyDeviceToHost));
    if (morton && sc->n) GSRT_HIP(ctx, hipMemcpy(morton, sc->d_morton, 4ull * sc->n, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

static gsrt_status check_render_args(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode) {
    if (!sc || !ubo) return GSRT_E_ARG;
    if (ubo->width == 0 || ubo->height == 0 || ubo->width > 32768 || ubo->height > 32768)
        return fail(sc->ctx, GSRT_E_ARG, "bad frame size");
    if ((mode & 0xffu) > GSRT_MODE_COR || (mode & ~(0xffu | GSRT_FLAG_LUT | GSRT_FLAG_STATS)))
        return fail(sc->ctx, GSRT_E_ARG, "bad mode");
    if ((mode & 0xffu) == GSRT_MODE_COR && ubo->samples == 0) return fail(sc->ctx, GSRT_E_ARG, "samples == 0");
    if (!sc->bvh_built) return fail(sc->ctx, GSRT_E_STATE, "render before gsrt_build_bvh");
    if (sc->ntri && (mode & 0xffu) != GSRT_MODE_REF)
        return fail(sc->ctx, GSRT_E_ARG, "triangle meshes are co-traced in REF mode only");
    return GSRT_OK;
}

static gsrt_status prepare_frame(gsrt_ctx* ctx, const gsrt_ubo* ubo, uint32_t mode) {
    const size_t px = (size_t)ubo->width * ubo->height;
    gsrt_status s = grow(ctx, &ctx->d_fb, &ctx->fb_pixels, px * 4);
    if (s != GSRT_OK) return s;
    ctx->fb_pixels = ctx->fb_pixels;  // counted in floats
    if (mode & GSRT_FLAG_STATS) {
        s = grow(ctx, &ctx->d_ray_stats, &ctx->ray_stats_pixels, px * 4);
        if (s != GSRT_OK) return s;
    }
    ctx->last_w = ubo->width;
    ctx->last_h = ubo->height;
    ctx->last_stats = (mode & GSRT_FLAG_STATS) != 0;
    ctx->last_ref = (mode & 0xffu) == GSRT_MODE_REF;
    return GSRT_OK;
}

gsrt_status gsrt_render_async(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* d_rgba,
                              gsrt_raystate* d_rs) {
    gsrt_status s = check_render_args(sc, ubo, mode);
    if (s != GSRT_OK) return s;
    gsrt_ctx* ctx = sc->ctx;
    (void)hipSetDevice(ctx->device);
    s = prepare_frame(ctx, ubo, mode);
    if (s != GSRT_OK) return s;
    ctx->fb_dump8 = false;
    const gsrt::RenderPlan plan = gsrt::make_plan(*ubo, mode, k, 0, 1);
    gsrt::timing_mark(ctx, 0);
    // pipelined COR frames render into their own buffer while slot streams are chosen (their frames overlap); the
    // ray states are one buffer, so frames that write them stay in order
    const bool slot = (mode & 0xffu) == GSRT_MODE_COR && !(mode & GSRT_FLAG_STATS) && !d_rs &&
                      gsrt::use_slot_streams(ctx, false);
    if (slot) {
        // the frame goes into one of two alternating buffers (the previous frame's render kernel may still write the
        // other), which becomes the framebuffer view (gsrt_framebuffer)
        const size_t share = (size_t)4 * ubo->width * ubo->height;
        if (ctx->share_floats < share) {
            if ((s = gsrt::sync_all(ctx)) != GSRT_OK) return s;
            ctx->fb_view = nullptr;  // it may point into a buffer freed below; no early return may leave it dangling
            for (int p = 0; p < 2; ++p) {
                (void)hipFree(ctx->d_share[p]);
                ctx->d_share[p] = nullptr;
                ctx->share_pending[p] = false;
            }
            ctx->share_floats = 0;
            for (int p = 0; p < 2; ++p) GSRT_HIP(ctx, hipMalloc(&ctx->d_share[p], sizeof(float) * share));
            ctx->share_floats = share;
        }
        for (int p = 0; p < 2; ++p)
            if (!ctx->ev_share[p]) GSRT_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_share[p], kSyncEventFlags));
        const uint32_t p = ctx->share_parity;
        ctx->share_parity ^= 1u;
        gsrt::RenderSync rsy;
        rsy.slot = slot;
        rsy.private_out = true;
        rsy.wait = ctx->share_pending[p] ? ctx->ev_share[p] : nullptr;
        s = gsrt::launch_render(sc, *ubo, plan, ctx->d_share[p], d_rs, &rsy);
        if (s != GSRT_OK) return s;
        ctx->fb_view = ctx->d_share[p];  // the framebuffer of this render (gsrt_framebuffer)
        if (d_rgba && d_rgba != gsrt::framebuffer_of(ctx))
            GSRT_HIP(ctx, hipMemcpyAsync(d_rgba, gsrt::framebuffer_of(ctx), sizeof(float) * 4 * ubo->width * ubo->height,
                                         hipMemcpyDeviceToDevice, ctx->stream));
        GSRT_HIP(ctx, hipEventRecord(ctx->ev_share[p], ctx->stream));  // copies out of d_share[p] issued
        ctx->share_pending[p] = true;
    } else {
        if ((s = gsrt_comm_fb_render_write(ctx)) != GSRT_OK) return s;  // d_fb is also rank 0's unpack target
        gsrt::RenderSync rsy;  // a shared output: frames in order (and render times sampled for use_slot_streams)
        s = gsrt::launch_render(sc, *ubo, plan, ctx->d_fb, d_rs, d_rs ? nullptr : &rsy);
        if (s != GSRT_OK) return s;
        ctx->fb_view = nullptr;
        if (d_rgba && d_rgba != ctx->d_fb)
            GSRT_HIP(ctx, hipMemcpyAsync(d_rgba, ctx->d_fb, sizeof(float) * 4 * ubo->width * ubo->height,
                                         hipMemcpyDeviceToDevice, ctx->stream));
    }
    gsrt::timing_mark(ctx, 3);
    return GSRT_OK;
}

gsrt_status gsrt_render(gsrt_scene* sc, const gsrt_ubo* ubo, uint32_t mode, uint32_t k, float* rgba_out,
                        gsrt_raystate* rs_out) {
    gsrt_status s = check_render_args(sc, ubo, mode);
    if (s != GSRT_OK) return s;
    gsrt_ctx* ctx = sc->ctx;
    (void)hipSetDevice(ctx->device);
    const size_t px = (size_t)ubo->width * ubo->height;
    const bool rgba_dev = is_device_ptr(rgba_out), rs_dev = is_device_ptr(rs_out);
    gsrt_raystate* d_rs = nullptr;
    if (rs_out && !rs_dev) GSRT_HIP(ctx, hipMalloc(&d_rs, sizeof(gsrt_raystate) * px));
    s = gsrt_render_async(sc, ubo, mode, k, rgba_dev ? rgba_out : nullptr, rs_out ? (rs_dev ? rs_out : d_rs) : nullptr);
    if (s == GSRT_OK && rgba_out && !rgba_dev) {
        if (hipMemcpyAsync(rgba_out, gsrt::framebuffer_of(ctx), sizeof(float) * 4 * px, hipMemcpyDeviceToHost,
                           ctx->stream) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "framebuffer download failed");
    }
    if (s == GSRT_OK && d_rs) {
        if (hipMemcpyAsync(rs_out, d_rs, sizeof(gsrt_raystate) * px, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
            s = fail(ctx, GSRT_E_DEVICE, "raystate download failed");
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess && s == GSRT_OK)
        s = fail(ctx, GSRT_E_DEVICE, std::string("render: ") + hipGetErrorString(hipGetLastError()));
    (void)hipFree(d_rs);
    if (s == GSRT_OK) s = gsrt::check_error_word(ctx);
    return s;
}

gsrt_status gsrt_timing(gsrt_ctx* ctx, uint32_t frames) {
    if (!ctx) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    while (ctx->events.size() < (size_t)gsrt::kTimingEvents * frames) {
        hipEvent_t e;
        GSRT_HIP(ctx, hipEventCreateWithFlags(&e, kTimingEventFlags));
        ctx->events.push_back(e);
    }
    if (ctx->timing_ex.size() < frames) ctx->timing_ex.resize(frames, 0);
    ctx->timing_cap = frames;
    ctx->timing_n = 0;
    ctx->timing_kernel_only = ctx->timing_kernel_only_next;
    ctx->timing_stride = ctx->timing_stride_next;
    ctx->timing_frame = 0;
    return GSRT_OK;
}

gsrt_status gsrt_timing_read(gsrt_ctx* ctx, float* kernel_ms, float* frame_ms, uint32_t cap, uint32_t* nframes) {
    if (!ctx) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t n = ctx->timing_n < cap ? ctx->timing_n : cap;
    for (uint32_t i = 0; i < n; ++i) {
        float k = 0.f, f = 0.f;
        const size_t e = (size_t)gsrt::kTimingEvents * i;
        GSRT_HIP(ctx, hipEventElapsedTime(&k, ctx->events[e + 1], ctx->events[e + 2]));
        if (!ctx->timing_kernel_only) GSRT_HIP(ctx, hipEventElapsedTime(&f, ctx->events[e + 0], ctx->events[e + 3]));
        if (kernel_ms) kernel_ms[i] = k;
        if (frame_ms) frame_ms[i] = f;
    }
    if (nframes) *nframes = n;
    return GSRT_OK;
}

gsrt_status gsrt_timing_kernel_only(gsrt_ctx* ctx, int on) {
    if (!ctx) return GSRT_E_ARG;
    ctx->timing_kernel_only_next = on != 0;
    return GSRT_OK;
}

gsrt_status gsrt_timing_stride(gsrt_ctx* ctx, uint32_t stride) {
    if (!ctx || stride == 0) return GSRT_E_ARG;
    ctx->timing_stride_next = stride;
    return GSRT_OK;
}

// diagnostic: raw counter block of the last render (16 words; [9..11] are cycle sums in GSRT_DIAG builds)
gsrt_status gsrt_debug_counters(gsrt_ctx* ctx, uint64_t out[16]) {
    if (!ctx || !out) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GSRT_HIP(ctx, hipMemcpy(out, ctx->d_counters, sizeof(unsigned long long) * 16, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

// diagnostic: words 16..31 of the counter block (GSRT_DIAG builds: shading-loop wave-candidate counts)
gsrt_status gsrt_debug_counters_hi(gsrt_ctx* ctx, uint64_t out[16]) {
    if (!ctx || !out) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GSRT_HIP(ctx, hipMemcpy(out, ctx->d_counters + 16, sizeof(unsigned long long) * 16, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

gsrt_status gsrt_exp_lut(float out[512]) {
    if (!out) return GSRT_E_ARG;
    gsrt::exp_lut(out);
    return GSRT_OK;
}

gsrt_status gsrt_debug_exp_lut(gsrt_ctx* ctx, float out[512]) {
    if (!ctx || !out) return GSRT_E_ARG;
    GSRT_HIP(ctx, hipMemcpy(out, ctx->d_lut, sizeof(float) * 512, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

const float* gsrt_framebuffer(gsrt_ctx* ctx) { return ctx && !ctx->fb_dump8 ? gsrt::framebuffer_of(ctx) : nullptr; }
int gsrt_slot_streams(const gsrt_ctx* ctx) { return ctx && ctx->last_slot_streams ? 1 : 0; }

gsrt_status gsrt_vs_stats(gsrt_ctx* ctx, uint64_t out[8]) {
    if (!ctx || !out) return GSRT_E_ARG;
    if (!ctx->last_stats || !ctx->last_ref) return fail(ctx, GSRT_E_STATE, "last render was not a REF render with GSRT_FLAG_STATS");
    unsigned long long c[32];
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GSRT_HIP(ctx, hipMemcpy(c, ctx->d_counters, sizeof c, hipMemcpyDeviceToHost));
    const uint64_t v[8] = {c[29], c[26], c[27], c[25], c[24], c[28], 0, 0};
    std::memcpy(out, v, sizeof v);
    return GSRT_OK;
}

gsrt_status gsrt_dump_vs_stats(gsrt_ctx* ctx, const char* path) {
    uint64_t v[8];
    if (!path) return GSRT_E_ARG;
    if (gsrt_status s = gsrt_vs_stats(ctx, v); s != GSRT_OK) return s;
    FILE* f = std::fopen(path, "w");
    if (!f) return fail(ctx, GSRT_E_IO, std::string("cannot open ") + path);
    // the simulator's lines (gpu-sim.cc:1510-1518; any-hit rays: none, the Gaussian pipeline traces opaque)
    std::fprintf(f, "rt_num_hits = %llu\n", (unsigned long long)v[1]);
    std::fprintf(f, "rt_num_any_hits = 0\n");
    std::fprintf(f, "rt_n_anyhit_rays = 0\n");
    std::fprintf(f, "rt_n_closesthit_rays = %llu\n", (unsigned long long)v[0]);
    std::fprintf(f, "rt_n_total_rays = %llu\n", (unsigned long long)v[0]);
    std::fprintf(f, "rt_max_tree_depth = %llu\n", (unsigned long long)v[2]);
    std::fprintf(f, "rt_max_nodes_per_ray = %llu\n", (unsigned long long)v[3]);
    std::fprintf(f, "rt_tot_nodes_per_ray = %llu\n", (unsigned long long)v[4]);
    std::fprintf(f, "rt_avg_nodes_per_ray = %f\n", v[0] ? (float)v[4] / (float)v[0] : 0.0f);
    const bool ok = std::fclose(f) == 0;
    return ok ? GSRT_OK : fail(ctx, GSRT_E_IO, "write failed");
}

gsrt_status gsrt_last_stats(gsrt_ctx* ctx, uint64_t out[8], uint32_t* per_ray) {
    if (!ctx || !out) return GSRT_E_ARG;
    if (!ctx->last_stats) return fail(ctx, GSRT_E_STATE, "last render had no GSRT_FLAG_STATS");
    unsigned long long c[16];
    GSRT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    GSRT_HIP(ctx, hipMemcpy(c, ctx->d_counters, sizeof c, hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; ++i) out[i] = c[i];
    if (per_ray)
        GSRT_HIP(ctx, hipMemcpy(per_ray, ctx->d_ray_stats, 16ull * ctx->last_w * ctx->last_h, hipMemcpyDeviceToHost));
    return GSRT_OK;
}

}  // extern "C"
