// gsrt_render -- command-line front end of the renderer, taking the reference application's flags
// (RayTracingInVulkan/src/Options.cpp:13-44: --scene --shader-type --width --height --samples --bounces
// --benchmark) so scripts that drove the reference render path (RTV/dump_image.sh, lumibench.sh) can
// drive this one. Written against the C ABI only (include/gsrt.h).
//
//   gsrt_render --scene 33 --shader-type 6 --width 16 --height 16 --samples 1 --bounces 16
//       scene 33 (SceneList.cpp:108-128, the two Gaussians of GaussSplat), REF mode, writes the
//       reference-named "<dd-mm-YYYY-HH-MM-SS->SCENE.ppm" (vulkan_ray_tracing.cc:2216-2247)
//   gsrt_render --scene 100 --gaussians 1000000 --sh --width 1920 --height 1080 --samples 4 --mode cor
//       synthetic front-facing cloud, COR mode
//
// Extra flags: --mode ref|cor, --lut, --gaussians N, --seed S, --sh, --camera FILE (.camera: eye, centre),
// --fov DEG, --out PATH (PPM), --binary PATH (image.binary records), --text PATH (dump_image.sh lines),
// --ply PATH (3DGS scene: COR mode, camera from --camera or looking down -z from the origin), --no-dump,
// --device D, --frames F (with --benchmark: frames timed), --stats.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gsrt_test.h"  // gsrt_synth_cloud: the synthetic clouds of --benchmark

namespace {

struct Options {
    int scene = 33;
    int shader_type = 6;
    uint32_t width = 16, height = 16, samples = 1, bounces = 16;
    bool benchmark = false;
    std::string mode;  // empty: REF for scene 33 / 101, COR for scene 100
    bool lut = false, sh = false, stats = false, no_dump = false;
    uint32_t gaussians = 10000, seed = 42, frames = 10;
    int device = 0;
    float fov = 0.0f;  // 0: scene default
    std::string camera, out, binary, text, ply;
};

[[noreturn]] void usage(const char* msg) {
    if (msg) std::fprintf(stderr, "gsrt_render: %s\n", msg);
    std::fprintf(stderr,
                 "usage: gsrt_render [--scene 33|100|101] [--shader-type N] [--width W] [--height H] [--samples S]\n"
                 "                   [--bounces B] [--benchmark] [--mode ref|cor] [--lut] [--gaussians N] [--seed S]\n"
                 "                   [--sh] [--camera FILE] [--fov DEG] [--out PPM] [--binary FILE] [--no-dump]\n"
                 "                   [--text FILE] [--ply FILE] [--device D] [--frames F] [--stats]\n");
    std::exit(2);
}

uint32_t to_u32(const char* s, const char* flag) {
    char* end = nullptr;
    const unsigned long v = std::strtoul(s, &end, 10);
    if (!end || *end || v > 0xFFFFFFFFul) usage((std::string("bad value for ") + flag).c_str());
    return (uint32_t)v;
}

Options parse(int argc, char** argv) {
    Options o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) usage((a + " needs a value").c_str());
            return argv[++i];
        };
        if (a == "--scene") o.scene = (int)to_u32(val(), "--scene");
        else if (a == "--shader-type") o.shader_type = (int)to_u32(val(), "--shader-type");
        else if (a == "--width") o.width = to_u32(val(), "--width");
        else if (a == "--height") o.height = to_u32(val(), "--height");
        else if (a == "--samples") o.samples = to_u32(val(), "--samples");
        else if (a == "--bounces") o.bounces = to_u32(val(), "--bounces");
        else if (a == "--benchmark") o.benchmark = true;
        else if (a == "--mode") o.mode = val();
        else if (a == "--lut") o.lut = true;
        else if (a == "--sh") o.sh = true;
        else if (a == "--stats") o.stats = true;
        else if (a == "--no-dump") o.no_dump = true;
        else if (a == "--gaussians") o.gaussians = to_u32(val(), "--gaussians");
        else if (a == "--seed") o.seed = to_u32(val(), "--seed");
        else if (a == "--frames") o.frames = to_u32(val(), "--frames");
        else if (a == "--device") o.device = (int)to_u32(val(), "--device");
        else if (a == "--fov") o.fov = std::strtof(val(), nullptr);
        else if (a == "--camera") o.camera = val();
        else if (a == "--out") o.out = val();
        else if (a == "--binary") o.binary = val();
        else if (a == "--text") o.text = val();
        else if (a == "--ply") o.ply = val();
        else if (a == "--help" || a == "-h") usage(nullptr);
        else usage(("unknown option " + a).c_str());
    }
    if (o.scene != 33 && o.scene != 100 && o.scene != 101) usage("scene must be 33 (GaussSplat), 100 (COR cloud) or 101 (REF cloud)");
    if (o.mode.empty()) o.mode = (o.scene == 100 || !o.ply.empty()) ? "cor" : "ref";
    if (o.mode != "ref" && o.mode != "cor") usage("--mode must be ref or cor");
    if (!o.width || !o.height) usage("empty frame");
    return o;
}

int check(gsrt_status s, gsrt_ctx* ctx, const char* what) {
    if (s == GSRT_OK) return 0;
    std::fprintf(stderr, "gsrt_render: %s: %s%s%s\n", what, gsrt_status_string(s), ctx ? ": " : "",
                 ctx ? gsrt_last_error(ctx) : "");
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    const Options o = parse(argc, argv);
    gsrt_ctx* ctx = nullptr;
    if (check(gsrt_create(&ctx, o.device), nullptr, "gsrt_create")) return 1;
    int rc = 0;
    gsrt_scene* scene = nullptr;
    gsrt_ubo ubo;
    float mv[16];
    float fov = o.fov;
    float focus = 1.0f;
    if (!o.ply.empty()) {
        rc = check(gsrt_scene_from_ply(ctx, o.ply.c_str(), 1, &scene), ctx, "scene from ply");
        const float eye[3] = {0, 0, 0}, at[3] = {0, 0, -1}, up[3] = {0, 1, 0};
        if (!rc) rc = check(gsrt_lookat(eye, at, up, mv), ctx, "lookat");
        if (fov == 0.0f) fov = 60.0f;
    } else if (o.scene == 33) {
        // SceneList::GaussSplat: G1 mu (0,0,5) scale 1, G2 mu (0,0,3) scale 2, opacity 0.9, identity rotation;
        // camera translate(0,0,-2), 90 degrees, focus distance 2 (SceneList.cpp:108-128)
        const float center[6] = {0, 0, 5, 0, 0, 3}, rot[8] = {1, 0, 0, 0, 1, 0, 0, 0};
        const float scale[6] = {1, 1, 1, 2, 2, 2}, opacity[2] = {0.9f, 0.9f};
        rc = check(gsrt_scene_from_model(ctx, center, rot, scale, opacity, nullptr, 2, &scene), ctx, "scene");
        // ... and model 0, the triangle sphere CreateSphere((200,200,0), 0.5) (SceneList.cpp:123), co-traced in REF
        if (!rc && o.mode == "ref") {
            const float sc[3] = {200.0f, 200.0f, 0.0f};
            std::vector<float> v(3ull * GSRT_SPHERE_VERTICES);
            std::vector<uint32_t> ix(3ull * GSRT_SPHERE_TRIANGLES);
            rc = check(gsrt_sphere_mesh(sc, 0.5f, v.data(), ix.data()), ctx, "sphere mesh");
            if (!rc) rc = check(gsrt_scene_add_mesh(scene, v.data(), GSRT_SPHERE_VERTICES, ix.data(), GSRT_SPHERE_TRIANGLES),
                                ctx, "add mesh");
        }
        std::memset(mv, 0, sizeof mv);
        mv[0] = mv[5] = mv[10] = mv[15] = 1.0f;
        mv[14] = -2.0f;
        if (fov == 0.0f) fov = 90.0f;
        focus = 2.0f;
    } else {
        const uint32_t n = o.gaussians;
        std::vector<float> c(3ull * n), r(4ull * n), s(3ull * n), op(n), sh(o.sh ? 48ull * n : 0);
        const uint32_t kind = o.scene == 100 ? GSRT_SYNTH_COR : GSRT_SYNTH_REF;
        rc = check(gsrt_synth_cloud(kind, n, o.seed, o.sh ? 1 : 0, c.data(), r.data(), s.data(), op.data(),
                                    o.sh ? sh.data() : nullptr), ctx, "synth_cloud");
        if (!rc)
            rc = check(gsrt_scene_from_model(ctx, c.data(), r.data(), s.data(), op.data(), o.sh ? sh.data() : nullptr,
                                             n, &scene), ctx, "scene");
        const float eye[3] = {0, 0, 0}, at[3] = {0, 0, -1}, up[3] = {0, 1, 0};
        if (!rc) rc = check(gsrt_lookat(eye, at, up, mv), ctx, "lookat");
        if (fov == 0.0f) fov = 60.0f;
    }
    if (!rc) {
        if (!o.camera.empty())
            rc = check(gsrt_camera_from_file(o.camera.c_str(), fov, o.width, o.height, focus, o.samples, o.bounces, &ubo),
                       ctx, "camera file");
        else
            rc = check(gsrt_camera_from_modelview(mv, fov, o.width, o.height, focus, o.samples, o.bounces, &ubo), ctx,
                       "camera");
    }
    if (!rc) rc = check(gsrt_build_bvh(scene), ctx, "build_bvh");
    uint32_t mode = o.mode == "ref" ? GSRT_MODE_REF : GSRT_MODE_COR;
    if (o.lut) mode |= GSRT_FLAG_LUT;
    if (o.stats) mode |= GSRT_FLAG_STATS;
    std::vector<float> rgba((size_t)o.width * o.height * 4);
    if (!rc) rc = check(gsrt_render(scene, &ubo, mode, 0, rgba.data(), nullptr), ctx, "render");
    if (!rc && o.stats) {
        uint64_t st[8];
        rc = check(gsrt_last_stats(ctx, st, nullptr), ctx, "stats");
        if (!rc)
            std::printf("rays %llu candidates %llu blended %llu terminated %llu rounds %llu tiles %llu\n",
                        (unsigned long long)st[0], (unsigned long long)st[1], (unsigned long long)st[2],
                        (unsigned long long)st[3], (unsigned long long)st[4], (unsigned long long)st[6]);
    }
    if (!rc && o.benchmark) {
        const uint32_t frames = o.frames ? o.frames : 1;
        const uint32_t m = mode & ~(uint32_t)GSRT_FLAG_STATS;
        rc = check(gsrt_synchronize(ctx), ctx, "sync");
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t f = 0; f < frames && !rc; ++f) rc = check(gsrt_render_async(scene, &ubo, m, 0, nullptr, nullptr), ctx, "render");
        if (!rc) rc = check(gsrt_synchronize(ctx), ctx, "sync");
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double rays = (double)o.width * o.height * o.samples * frames;
        if (!rc) std::printf("%u frames %.3f ms/frame %.1f Mrays/s\n", frames, dt / frames * 1e3, rays / dt / 1e6);
    }
    if (!rc && !o.no_dump) {
        std::string path = o.out;
        if (path.empty()) {
            char name[128];
            rc = check(gsrt_reference_ppm_name(name, sizeof name), ctx, "ppm name");
            path = name;
        }
        if (!rc) rc = check(gsrt_dump_ppm(path.c_str(), rgba.data(), o.width, o.height), ctx, "dump_ppm");
        if (!rc) std::printf("wrote %s\n", path.c_str());
        if (!rc && !o.binary.empty())
            rc = check(gsrt_dump_image_binary(o.binary.c_str(), rgba.data(), o.width, o.height), ctx, "dump_image_binary");
        if (!rc && !o.text.empty())
            rc = check(gsrt_dump_rgba_text(o.text.c_str(), rgba.data(), o.width, o.height), ctx, "dump_rgba_text");
    }
    if (scene) gsrt_destroy_scene(scene);
    gsrt_destroy(ctx);
    return rc;
}
