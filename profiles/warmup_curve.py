"""Per-frame k_render_cor / frame times over consecutive C3 frames of a fresh process (diagnostic: what the
first frames of a process cost and why). Run on the GPU box from the repo root.

  python profiles/warmup_curve.py [frames] [idle_ms] [heat_ms]

Prints every one of the first 30 frames, then means over blocks of 10. idle_ms > 0 sleeps that long between
the scene build and the first frame (clock decay: a settled clock ramps down again while the host idles).
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402  (before gsrt: torch's HIP runtime first, as in bench.py)
import gsrt  # noqa: E402

FRAMES = int(sys.argv[1]) if len(sys.argv) > 1 else 120
IDLE = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
HEAT = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0  # ms of back-to-back fp32 matmuls (torch) just before
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1000000, 42, True)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
ctx.synchronize()
if IDLE > 0:
    time.sleep(IDLE / 1e3)
if HEAT > 0:
    a = torch.randn(4096, 4096, device="cuda:0")
    torch.cuda.synchronize()
    th = time.perf_counter()
    while time.perf_counter() - th < HEAT / 1e3:
        for _ in range(4):
            a = torch.tanh(a @ a)
        torch.cuda.synchronize()
ctx.timing(FRAMES)
t0 = time.perf_counter()
for _ in range(FRAMES):
    sc.render_async(ubo, gsrt.MODE_COR)
ctx.synchronize()
wall = time.perf_counter() - t0
k, f = ctx.timing_read()
ctx.timing(0)
for i in range(min(30, FRAMES)):
    print(f"frame {i:3d}: kernel {k[i]:.4f} ms, frame {f[i]:.4f} ms")
for i in range(0, FRAMES, 10):
    print(f"frames {i:3d}-{i + 9:3d}: kernel {np.mean(k[i:i + 10]):.4f} ms, frame {np.mean(f[i:i + 10]):.4f} ms")
print(f"wall {wall * 1e3 / FRAMES:.4f} ms/frame over {FRAMES}")
sc.close()
ctx.close()
