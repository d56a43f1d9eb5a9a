"""LBVH build and refit wall times at 1M / 5M Gaussians (run on the GPU box from the repo root). Both include
the host wait for the device (a build is synchronous; a refit is timed through bvh_info, which runs the lazy fit)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgs-raytrace_amd"))
import gsrt  # noqa: E402

ctx = gsrt.Context(0)
for n in (1_000_000, 5_000_000):
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, False)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    t0 = time.perf_counter()
    for _ in range(5):
        sc.build_bvh()
    tb = (time.perf_counter() - t0) / 5
    _, a = sc.download()
    sc.bvh_info(depth=False)
    t0 = time.perf_counter()
    for _ in range(10):  # refits are lazy: bvh_info runs the pending fit and waits for it
        sc.refit_bvh()
        sc.bvh_info(depth=False)
    tr = (time.perf_counter() - t0) / 10
    info = sc.bvh_info()
    print(f"n={n}: build {tb * 1e3:.2f} ms, refit {tr * 1e3:.3f} ms, max depth {info['max_depth']}")
    sc.close()
