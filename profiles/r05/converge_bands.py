"""Emulated N-rank balancing on one GPU: the partition an N-GPU job's automatic balancing converges to, and every
rank's share period under it.

An N-rank job balances from its ranks' own share-context costs (each rank's profile frames, all-reduced). Here every
rank's share runs in turn on a loopback communicator (GSRT_DEBUG_RANK_OF=N:r, pipelined frames, dump8 exchange) under
pinned bands; each share's last frame's tile costs (gsrt_debug_share_costs / gsrt_debug_row_profile) fill its rows of
the profile, and the next iteration's bands are cut from the combined profile by the library's rule (gsrt_tile_bands).
Iteration 0 starts from the bands of a whole frame's profile (what bench.py pins).

  python profiles/r05/converge_bands.py [config] [N] [iterations]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "3dgs-raytrace_amd"), ROOT]
import bench  # noqa: E402
import gsrt  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n, W, H, spp, with_sh = bench.CONFIGS[cfg]
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
mode = gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8
ctx.comm_init_loopback()
for _ in range(3):
    sc.render(ubo, gsrt.MODE_COR)
bands = gsrt.tile_bands(ubo, N, ctx.row_costs(), mode)
ctx.debug_share_costs(True)
for it in range(iters + 1):
    ctx.set_bands(N, bands)
    prof = None
    times = []
    for rk in range(N):
        os.environ["GSRT_DEBUG_RANK_OF"] = f"{N}:{rk}"
        for _ in range(30):
            sc.render_sharded_async(ubo, mode)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            sc.render_sharded_async(ubo, mode)
        ctx.synchronize()
        times.append((time.perf_counter() - t0) / 200 * 1e3)
        rows = ctx.debug_row_profile().astype(np.int64)
        prof = rows if prof is None else prof + rows
    print(f"iteration {it}: bands {bands.tolist()}")
    print("   ms per frame by rank: " + " ".join(f"{t:.4f}" for t in times) + f"   slowest {max(times):.4f} (rank "
          f"{int(np.argmax(times))})", flush=True)
    bands = gsrt.tile_bands(ubo, N, np.minimum(prof, 2**32 - 1).astype(np.uint32), mode)
