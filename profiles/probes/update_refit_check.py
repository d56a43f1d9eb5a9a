"""Diagnostic: tests/test_bvh_gpu.py::test_scene_update_and_refit_matches_rebuild as a script, printing where the GPU
frame and the CPU oracle differ (run on the GPU box from the repo root)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gsrt  # noqa: E402
import oracle as O  # noqa: E402  (oracle/oracle.py)

ctx = gsrt.Context(0)
n = 30000
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 5, True)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
p, a = sc.download()
rng = np.random.default_rng(11)
mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
ubo = gsrt.camera_from_modelview(mv, 60.0, 96, 64, 1.0, 4, 16)
for frame in range(3):
    d = rng.normal(0.0, 1e-3, (n, 3)).astype(np.float32)
    p2, a2 = p.copy(), a.copy()
    p2[:, :3] += d
    a2[:, :3] += d
    a2[:, 3:] += d
    sc.update(p2, a2)
    sc.refit_bvh()
    img, _ = sc.render(ubo, gsrt.MODE_COR)
    fresh = gsrt.Scene.from_params(ctx, p2, a2, sh)
    fresh.build_bvh()
    want, _ = fresh.render(ubo, gsrt.MODE_COR)
    ref = O.render(p2, a2, O.make_ubo(mv, 60.0, 96, 64, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a2))["rgba"]
    for name, x in (("refit", img), ("fresh", want)):
        dd = np.abs(x.astype(np.float64) - ref).max(-1)
        bad = np.argwhere(dd > 0)
        print(f"frame {frame} {name}: max |diff| {dd.max():.3g}, {len(bad)} pixels differ, first {bad[:5].tolist()}")
    p, a = p2, a2
print("slot streams:", ctx.slot_streams())
