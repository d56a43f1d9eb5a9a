"""Frame time of C3 variants (diagnostic): with/without SH-3, spp 1/4. Run on the GPU box from the repo root."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import numpy as np  # noqa: E402
import gsrt  # noqa: E402

ctx = gsrt.Context(0)
for with_sh, spp in ((True, 4), (False, 4), (True, 1), (False, 1)):
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1000000, 42, with_sh)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, spp, 16)
    for _ in range(3):
        sc.render_async(ubo, gsrt.MODE_COR)
    ctx.synchronize()
    ctx.timing(20)
    t0 = time.perf_counter()
    for _ in range(20):
        sc.render_async(ubo, gsrt.MODE_COR)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / 20
    k, f = ctx.timing_read()
    ctx.timing(0)
    print(f"sh={with_sh} spp={spp}: frame {dt * 1e3:.3f} ms, k_render_cor {np.mean(k):.3f} ms, "
          f"{1920 * 1080 * spp / dt / 1e6:.0f} Mrays/s")
    sc.close()
