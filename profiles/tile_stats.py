"""Counters of one C3 frame (COR, SH-3, 4 spp): rays, candidates, blends, terminations, tile rounds, restarts,
tiles, max candidates per tile. Run on the GPU box from the repo root: python profiles/tile_stats.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1000000, 42, True)
sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
sc.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
print(ctx.last_stats())
print(ctx.debug_counters())
