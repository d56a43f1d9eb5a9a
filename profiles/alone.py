"""Frames one at a time (synchronised after each), so every kernel of a frame runs without the neighbouring frames'
kernels beside it: under `rocprofv3 --kernel-trace --stats` this gives each kernel's standalone duration.

  python profiles/alone.py [config] [frames]      (GSRT_DEBUG_RANK_OF=N[:r]: rank r's share of an N-rank frame)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 30
n, W, H, spp, with_sh = {"c3": (1_000_000, 1920, 1080, 4, True), "c2": (100_000, 1920, 1080, 1, False),
                          "c4": (1_000_000, 3840, 2160, 1, False), "c5": (5_000_000, 1920, 1080, 16, False)}[cfg]
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
share = bool(os.environ.get("GSRT_DEBUG_RANK_OF"))
mode = gsrt.MODE_COR
if share:  # a rank share runs through the sharded path on a loopback communicator, bands as bench.py
    mode |= gsrt.FLAG_OUT_DUMP8  # bench.py's default exchange format
    nr = int(os.environ["GSRT_DEBUG_RANK_OF"].split(":")[0])
    ctx.comm_init_loopback()
    for _ in range(3):
        sc.render(ubo, gsrt.MODE_COR)
    ctx.set_bands(nr, gsrt.tile_bands(ubo, nr, ctx.row_costs(), mode))
step = None
if cfg == "c5":  # bench.py's dynamic scene: two device-resident jitter sets alternate, attach + refit per frame
    import numpy as np
    import torch
    p0, a0 = sc.download()
    rng = np.random.default_rng(1234)
    sets = []
    for _ in range(2):
        d = rng.normal(0.0, 1e-3, (n, 3)).astype(np.float32)
        p1, a1 = p0.copy(), a0.copy()
        p1[:, :3] += d
        a1[:, :3] += d
        a1[:, 3:] += d
        sets.append((torch.from_numpy(p1).cuda(), torch.from_numpy(a1).cuda()))
    torch.cuda.synchronize()

    def step(i):  # bench.py's default (--update attach); GSRT_ALONE_COPY=1: --update copy
        (sc.update if os.environ.get("GSRT_ALONE_COPY") else sc.attach)(sets[i & 1][0].data_ptr(),
                                                                          sets[i & 1][1].data_ptr())
        sc.refit_bvh()
for i in range(frames):
    if step:
        step(i)
    (sc.render_sharded_async if share else sc.render_async)(ubo, mode)
    ctx.synchronize()
print(f"{cfg}: {frames} frames, one at a time")
