"""How evenly the round-robin deal of super-tile runs spreads a frame's shading work over N ranks (diagnostic):

  python profiles/deal_balance.py [config] [N...]

renders the bench frame once with the counting pass (GSRT_FLAG_STATS: candidates and blended hits per pixel), prices
each tile with the roofline's operation counts (bench.py FLOP_*), sums the tiles of each run of the spatial order
(gsrt_device.hpp spatial_index, kRun tiles) and prints, per deal, the heaviest rank's work over the mean:
  rr     the product's deal (run j to rank j % N, global_pos / owner_of)
  snake  runs dealt 0..N-1, N-1..0, ... (still arithmetic)
  lpt    greedy longest-processing-time over the measured run costs (a cost-aware deal's bound)
Compare rr's per-rank work with every rank's measured share time (profiles/rank_shares_all.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3dgs-raytrace_amd"))
import bench  # noqa: E402  (CONFIGS, FLOP_* of the roofline)
import gsrt  # noqa: E402

SUPER, RUN = 16, 256


def spatial_index(tx, ty, tiles_x, tiles_y):
    R, C = ty // SUPER, tx // SUPER
    hR = np.minimum(SUPER, tiles_y - R * SUPER)
    wC = np.minimum(SUPER, tiles_x - C * SUPER)
    return R * SUPER * tiles_x + C * hR * SUPER + (ty - R * SUPER) * wC + (tx - C * SUPER)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    ranks = [int(a) for a in sys.argv[2:]] or [8, 4]
    n, W, H, spp, with_sh = bench.CONFIGS[cfg]
    ctx = gsrt.Context(0)
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
    scene = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    scene.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
    scene.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
    st = ctx.last_stats((H, W))["per_ray"].astype(np.float64)
    hit = bench.FLOP_HIT_SH if with_sh else bench.FLOP_HIT
    cost_px = bench.FLOP_RAY * spp + bench.FLOP_CAND * st[..., 0] + hit * st[..., 1]
    pl = gsrt.tile_plan(ubo, gsrt.MODE_COR, 1, 0)
    tw, th, tx_n, ty_n = pl["tile_w"], pl["tile_h"], pl["tiles_x"], pl["tiles_y"]
    pad = np.zeros((ty_n * th, tx_n * tw))
    pad[:H, :W] = cost_px
    tile_cost = pad.reshape(ty_n, th, tx_n, tw).sum(axis=(1, 3))
    ty, tx = np.mgrid[0:ty_n, 0:tx_n]
    k = spatial_index(tx, ty, tx_n, ty_n)
    runs = np.zeros((tx_n * ty_n + RUN - 1) // RUN)
    np.add.at(runs, (k // RUN).ravel(), tile_cost.ravel())
    print(f"{cfg}: {len(runs)} runs of {RUN} tiles, run cost max/mean {runs.max() / runs.mean():.2f}")
    for N in ranks:
        j = np.arange(len(runs))
        deals = {"rr": j % N, "snake": np.where((j // N) % 2 == 0, j % N, N - 1 - j % N)}
        lpt = np.zeros(len(runs), int)
        load = np.zeros(N)
        for q in np.argsort(-runs):
            lpt[q] = int(np.argmin(load))
            load[lpt[q]] += runs[q]
        deals["lpt"] = lpt
        for name, d in deals.items():
            per = np.bincount(d, weights=runs, minlength=N)
            print(f"  N={N} {name:5s} heaviest/mean {per.max() / per.mean():.4f}  per rank (/mean): "
                  + " ".join(f"{v:.3f}" for v in per / per.mean()))
    scene.close()
    ctx.close()


if __name__ == "__main__":
    main()
