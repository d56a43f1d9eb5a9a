"""Diagnostic: per-wave cycle split (traversal+sort vs shading) of the C3 render kernel.
Run with GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_diag.so (built by `make -C 3dgs-raytrace_amd diag`)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n, W, H, spp, with_sh = {"c3": (1_000_000, 1920, 1080, 4, True), "c2": (100_000, 1920, 1080, 1, False),
                          "c4": (1_000_000, 3840, 2160, 1, False), "c5": (5_000_000, 1920, 1080, 16, False)}[cfg]
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
share = bool(os.environ.get("GSRT_DEBUG_RANK_OF"))
if share:  # a rank share runs through the sharded path on a loopback communicator
    ctx.comm_init_loopback()
for _ in range(3):
    (sc.render_sharded_async if share else sc.render_async)(ubo, gsrt.MODE_COR)
ctx.synchronize()
if share:
    sc.render_sharded(ubo, gsrt.MODE_COR, want_image=False)
else:
    sc.render(ubo, gsrt.MODE_COR)  # one frame alone: the counters are this frame's (pipelined frames share them)
cnt = ctx.debug_counters()
col, sha, tot = int(cnt[9]), int(cnt[10]), int(cnt[11])
print(f"{cfg}: wave-cycles collect(traversal+sort) {col / tot:.3f}  shade {sha / tot:.3f}  other {(tot - col - sha) / tot:.3f}"
      f"  (sum of per-wave s_memtime, {tot / 1e9:.2f} G)")
print(f"{cfg}: collect() wave-cycles traversal {int(cnt[12]) / 1e9:.3f} G, final cull+sort {int(cnt[13]) / 1e9:.3f} G; "
      f"steps {int(cnt[14])}, popped nodes {int(cnt[15])} (per tile: {int(cnt[14]) / (W * H * spp / 64):.1f} steps, {int(cnt[15]) / (W * H * spp / 64):.0f} nodes)")
print(f"{cfg}: k_group_list wave-cycles {int(cnt[6]) / 1e9:.3f} G, of which tile filter {int(cnt[7]) / 1e9:.3f} G; "
      f"groups with an overflowing list: {int(cnt[5])}; group list length max {int(cnt[4])}, sum {int(cnt[3])}")
ng = max(int(cnt[3]) and 1, 1)
print(f"{cfg}: k_group_list tile filter split: per-lane tile tests (incl. the chunk's footprint loads) "
      f"{int(cnt[22]) / 1e9:.3f} G, per-tile list output {int(cnt[23]) / 1e9:.3f} G; group list to HBM {int(cnt[24]) / 1e9:.3f} G")
print(f"{cfg}: wave-cycles from entry: tile+ray setup {int(cnt[1]) / tot:.3f}, reduction+store tail {int(cnt[2]) / tot:.3f}")
waves = W * H * spp / 64
st, gp, co, bl, lg, lb = (int(x) for x in cnt[16:22])
print(f"{cfg}: per wave: staged candidates {st / waves:.1f}, some lane passes g {gp / waves:.1f}, some lane alpha > 0 "
      f"{co / waves:.1f}, some lane blends (SH) {bl / waves:.1f}; lanes per g-survivor {lg / max(gp, 1):.1f}, "
      f"lanes per blending candidate {lb / max(bl, 1):.1f}")
