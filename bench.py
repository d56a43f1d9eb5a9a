"""bench.py -- Mrays/s of the ray-traced 3DGS hot path on MI355X (BASELINE.json metric).

Workload (N=1, the config the metric is quoted on): 1M Gaussians with SH degree 3, 1920x1080, 4 spp,
COR mode (BASELINE.json configs[2]); synthetic cloud from std::mt19937(42).
A step = one frame: per-frame projection + packet traversal / blend kernel (+ RCCL tile gather for N>1),
scene and LBVH resident in HBM. rays = W*H*spp per frame (RayTracer.cpp:180-182).

Multi-GPU: `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`: one process per GPU,
the scene + LBVH replicated, the frame's tiles interleaved over ranks, ncclGather of the packed tiles to
rank 0. The frame is fixed as N grows: "scaling": "strong".

Extra JSON objects: roofline (render kernel, HIP events on the ctx stream, algorithmic bytes per
SURVEY.md §8d), cpu_baseline (the C oracle on this host's cores over a band of rows of the same frame).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "3dgs-raytrace_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (n_gauss, width, height, spp, sh)
    "c3": (1_000_000, 1920, 1080, 4, True),   # BASELINE configs[2]: the metric's config on one GPU
    "c2": (100_000, 1920, 1080, 1, False),    # configs[1]
    "c4": (1_000_000, 3840, 2160, 1, False),  # configs[3]
    "c5": (5_000_000, 1920, 1080, 16, False), # configs[4]: per-frame centre jitter + refit (DYNAMIC)
    "c1": (10_000, 256, 256, 1, False),       # configs[0]
}
DYNAMIC = {"c5"}  # a step also moves every centre (jitter 1e-3, two resident jitter sets alternate) and refits
HBM_PEAK_GBS = 8000.0
# BASELINE.json "metric", verbatim; value = primary rays W*H*spp per frame / frame wall time, in Mrays/s
METRIC = "Mrays/s @1080p, 1M Gaussians; achieved HBM GB/s vs peak; 1\u21928 GPU scaling"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the counting pass (roofline bytes)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def cpu_baseline(params, aabbs, sh, ubo_np, width, height, target_s, gpu_rgba=None):
    """Time the C oracle (COR mode, CPU BVH, all assigned host cores) on a band of rows of the frame."""
    import oracle as O

    threads = max(1, min(16, os.cpu_count() or 1))
    bvh = O.Bvh(aabbs)
    mid = height // 2

    def band(rows):
        r0 = max(0, min(height - rows, mid - rows // 2))
        t0 = time.perf_counter()
        out = O.render(params, aabbs, ubo_np, O.MODE_COR, sh=sh, bvh=bvh, threads=threads, rows=(r0, r0 + rows))
        return r0, out, time.perf_counter() - t0

    # a central band sized from a probe, grown once if it ran short of the target (rows differ in cost)
    rows = min(8, height)
    r0, out, dt = band(rows)
    for _ in range(2):
        if dt >= 0.6 * target_s or rows == height:
            break
        rows = int(max(rows + 1, min(height, rows * target_s / max(dt, 1e-6))))
        r0, out, dt = band(rows)
    mid = r0
    spp = int(ubo_np["samples"][0])
    rays = width * rows * spp
    res = {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"rows {mid}..{mid + rows - 1} of the same {width}x{height}x{spp}spp frame "
                     f"({rays} rays, {dt:.1f} s, C oracle COR mode + CPU BVH)"}
    if gpu_rgba is not None:
        gband = gpu_rgba[mid:mid + rows]
        res["gpu_vs_cpu_linf"] = float(np.abs(gband - out["rgba"][mid:mid + rows]).max())
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    import gsrt

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    n, W, H, spp, with_sh = CONFIGS[args.config]

    ctx = gsrt.Context(local)
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
    scene = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    tb = time.perf_counter()
    scene.build_bvh()
    bvh_ms = (time.perf_counter() - tb) * 1e3
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, W, H, 1.0, spp, 16)
    mode = gsrt.MODE_COR

    update = None
    if args.config in DYNAMIC:
        # two jittered copies of the scene (centre + AABB moved by N(0, 1e-3) per axis, seeded) resident in HBM;
        # each step pushes one of them with gsrt_scene_update (device to device), refits, renders
        p0, a0 = scene.download()
        rng = np.random.default_rng(1234 + rank)
        sets = []
        for _ in range(2):
            d = rng.normal(0.0, 1e-3, (n, 3)).astype(np.float32)
            p1, a1 = p0.copy(), a0.copy()
            p1[:, :3] += d
            a1[:, :3] += d
            a1[:, 3:] += d
            sets.append((torch.from_numpy(p1).to(f"cuda:{local}"), torch.from_numpy(a1).to(f"cuda:{local}")))
        torch.cuda.synchronize()
        step_no = [0]

        def update():
            tp, ta = sets[step_no[0] & 1]
            step_no[0] += 1
            scene.update(tp.data_ptr(), ta.data_ptr())
            scene.refit_bvh()

    if world > 1:
        uid = [gsrt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], world, rank)

        def frame():
            if update:
                update()
            scene.render_sharded_async(ubo, mode)
    else:
        def frame():
            if update:
                update()
            scene.render_async(ubo, mode)

    # counting pass for the algorithmic bytes: 16 + 48|C_r| + 192|H_r| per ray
    stats = None
    if not args.no_stats:
        scene.render_async(ubo, mode | gsrt.FLAG_STATS)
        ctx.synchronize()
        stats = ctx.last_stats()
    for _ in range(args.warmup):
        frame()
    ctx.synchronize()
    ctx.timing(args.steps)

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame()
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    kern_ms, frame_ms = ctx.timing_read()
    ctx.timing(0)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])

    rays_per_frame = W * H * spp
    value = rays_per_frame * args.steps / dt / 1e6
    out = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.config}: {n} Gaussians{' SH-3' if with_sh else ''}, {W}x{H}, {spp} spp, COR"
                               + (", per-frame centre jitter + refit" if args.config in DYNAMIC else ""),
                   "gaussians": n, "width": W, "height": H, "spp": spp, "sh_degree": 3 if with_sh else None,
                   "parallelism": f"tiles/{world}" if world > 1 else "1 GPU", "bvh_build_ms": round(bvh_ms, 2)},
    }
    if rank == 0 and stats is not None and len(kern_ms):
        k_ms = float(np.mean(kern_ms))
        alg_bytes = 16 * stats["rays"] + 48 * stats["candidates"] + 192 * (stats["blended"] if with_sh else 0)
        # per launch: the rays this rank's kernel processed (1/world of the frame for N>1 is approximated by
        # the full-frame counts divided evenly: tiles are interleaved round-robin)
        alg_launch = alg_bytes / world
        achieved = alg_launch / (k_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic) as f:
                tj = json.load(f)
            if tj.get("config") == args.config:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                           "kernel": "k_render_cor", "kernel_ms": round(k_ms, 4),
                           "frame_ms_events": round(float(np.mean(frame_ms)), 4),
                           "frame_achieved": round(alg_launch / (float(np.mean(frame_ms)) * 1e-3) / 1e9, 1),
                           "alg_bytes_per_launch": int(alg_launch),
                           "mean_candidates_per_ray": round(stats["candidates"] / max(stats["rays"], 1), 2),
                           "mean_blended_per_ray": round(stats["blended"] / max(stats["rays"], 1), 2)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rgba, _ = scene.render(ubo, mode)
        p, a = scene.download()
        out["cpu_baseline"] = cpu_baseline(p, a, sh, ubo, W, H, args.cpu_seconds, gpu_rgba=rgba)
    if rank == 0:
        print(json.dumps(out), flush=True)
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
