"""Per-frame k_render_cor / frame times over consecutive C3 frames (diagnostic: how many warmup frames the
clocks need before the timed region). Run on the GPU box from the repo root."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import numpy as np  # noqa: E402
import gsrt  # noqa: E402

FRAMES = int(sys.argv[1]) if len(sys.argv) > 1 else 120
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1000000, 42, True)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
ctx.timing(FRAMES)
for _ in range(FRAMES):
    sc.render_async(ubo, gsrt.MODE_COR)
ctx.synchronize()
k, f = ctx.timing_read()
ctx.timing(0)
for i in range(0, FRAMES, 10):
    print(f"frames {i:3d}-{i + 9:3d}: kernel {np.mean(k[i:i + 10]):.4f} ms, frame {np.mean(f[i:i + 10]):.4f} ms")
sc.close()
ctx.close()
