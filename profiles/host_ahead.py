"""Diagnostic: does the host run ahead of the GPU? Host time to enqueue K C3 frames (render_async) against the
time until they completed. Run on the GPU box from the repo root. With GSRT_DEBUG_RANK_OF=N[:r] the frames are rank
r's share through the loopback exchange path (dump8 format, bands pinned as bench.py pins them)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1000000, 42, True)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
mode, frame = gsrt.MODE_COR, sc.render_async
if os.environ.get("GSRT_DEBUG_RANK_OF"):
    nr = int(os.environ["GSRT_DEBUG_RANK_OF"].split(":")[0])
    mode |= gsrt.FLAG_OUT_DUMP8
    ctx.comm_init_loopback()
    for _ in range(3):
        sc.render(ubo, gsrt.MODE_COR)
    ctx.set_bands(nr, gsrt.tile_bands(ubo, nr, ctx.row_costs(), mode))
    frame = sc.render_sharded_async
for _ in range(10):
    frame(ubo, mode)
ctx.synchronize()
for timed in (False, True):
    if timed:
        ctx.timing(K)
    t0 = time.perf_counter()
    per = []
    for _ in range(K):
        a = time.perf_counter()
        frame(ubo, mode)
        per.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    ctx.synchronize()
    t2 = time.perf_counter()
    if timed:
        ctx.timing(0)
    per.sort()
    print(f"timing events {timed}: enqueue {K} frames {1e3 * (t1 - t0):.2f} ms (per call median {1e6 * per[K // 2]:.0f} us, "
          f"max {1e6 * per[-1]:.0f} us), done after {1e3 * (t2 - t0):.2f} ms = {1e3 * (t2 - t0) / K:.3f} ms/frame")
sc.close()
ctx.close()
