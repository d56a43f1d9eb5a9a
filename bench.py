"""bench.py -- Mrays/s of the ray-traced 3DGS hot path on MI355X (BASELINE.json metric).

Workload (N=1, the config the metric is quoted on): 1M Gaussians with SH degree 3, 1920x1080, 4 spp,
COR mode (BASELINE.json configs[2]); synthetic cloud from std::mt19937(42).
A step = one frame: per-frame projection + group lists + shading kernel (+ RCCL tile gather for N>1),
scene and LBVH resident in HBM. rays = W*H*spp per frame (RayTracer.cpp:180-182).

Multi-GPU: one process per GPU, the scene + LBVH replicated, the frame's tiles dealt over ranks, ncclGather of
the packed tiles to rank 0. The frame is fixed as N grows: "scaling": "strong".
- Under `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` (the driver's launch) every process
  is one rank; WORLD_SIZE must equal --gpus, else bench.py exits with status 2 before touching a GPU.
- `python bench.py --gpus N` (N > 1, no WORLD_SIZE) starts that same torch.distributed.run as a child process before
  any GPU call (no exec), relays its output and exits with its status, so an N-GPU request is always N ranks.
- The N > 1 line carries n_gpus as RCCL's communicator reports it (ncclCommCount), per-rank frame and render-kernel
  times (min / max over ranks), and the exchange time per frame (gather + rank 0's unpack, HIP events on the comm
  stream).

Warm-up: W frames as asked (in chunks of 8, each ended by a synchronisation), continued until the warm-up has
rendered for --warmup-min-s seconds (0.3 s by default); with N ranks every rank runs the same chunks (an all-reduce
decides when all are done). The MI355X lowers its clock when the render load starts and ramps it back over ~15 frames
(1.96 -> 2.36 GHz, profiles/archive/r02_clock_ramp.txt); a timed region that starts inside the ramp measures the
DVFS governor, not the kernels. The JSON line reports W and the frames the warm-up actually ran.

Extra JSON objects:
- roofline: the shading kernel k_render_cor is VALU-issue bound. `achieved` = the
  algorithmic FP32 operations of the frame (per ray, per AABB candidate |C_r| and per blended hit |H_r|,
  from the counting pass; the per-op tables OPS_* below, an FMA counted as 2 FLOP like the peak) / the kernel's
  mean duration from HIP events on its stream; peak = 157.3 TFLOP/s FP32 vector. `traffic` (HBM bytes per launch) and
  `valu_issue_frac` (VALU issue time / kernel time) come from the rocprofv3 PMC summary in profiles/pmc_traffic.json, and only when it was
  collected from these very kernel sources (source hash); else null and `traffic_stale` true.
- cpu_baseline: the C oracle (COR, CPU BVH) on this host's cores over a band of rows of the same frame,
  plus the C1 config (10k, 256x256) in REF mode (the reference's per-round re-traversal) and COR mode.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
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
JITTER_SEED = 1234  # the same on every rank: every rank renders the same geometry
HBM_PEAK_GBS = 8000.0
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (1024 SIMDs x 32 lanes/clk x FMA x 2.4 GHz)
EVENT_STRIDE = 4  # timed frames per recorded frame of HIP events (bench: kernel_ms)
SIMDS = 1024
CUS = 256
# Algorithmic FP32 operations of the COR per-ray algorithm, in the unit of the FP32 peak above: an FMA
# is 2 FLOP, every other arithmetic, min / max, compare or conversion op 1. Per unit:
OPS_CAND = {  # every AABB candidate of a ray (|C_r|): the exact slab test, then g and its range test
    "slab: 6 mul": 6, "slab: 12 min / max": 12, "slab: t <= u": 1,
    "g: dx, dy (2 sub), 4 mul": 6, "g: 2 fma": 4, "g in [0, gcut] (2 compares)": 2}
OPS_HIT = {  # every blended hit (|H_r|), without the colour
    "exp: mul, rint, ldexp": 3, "exp: 6 fma": 12, "alpha = min(op e, 0.99): mul, min": 2, "alpha > 1/255": 1,
    "T (1 - alpha): sub, mul": 2, "T' < 1e-4": 1, "w = alpha T": 1, "C += col w: 3 fma": 6}
OPS_SH = {"SH-3 colour: 3 x 15 fma": 90, "clamp at 0: 3 max": 3}  # per blended hit with SH-3
OPS_RAY = {  # per ray (sample), straight-line: generation, object-space ray, SH basis, the sample average
    "uv: 2 div, 2 mul, 2 sub": 6, "P^-1 (uv, 1, 1): 16 mul + 12 add": 28, "focus: 3 mul": 3, "normalise: 3 mul, 2 add, sqrt, 3 div": 9,
    "MV^-1 dir: 16 mul + 12 add": 28, "|d|, 3 div, 3 rcp, clamps": 18, "tmin, tmax": 2, "pixel + jitter: 2 add": 2,
    "average: 4 add, 4 mul": 8}
OPS_RAY_SH = {"SH-3 basis: 6 products, 30 mul / sub": 36}
FLOP_CAND = sum(OPS_CAND.values())                        # 31
FLOP_HIT = sum(OPS_HIT.values())                          # 28
FLOP_HIT_SH = FLOP_HIT + sum(OPS_SH.values())             # 121
FLOP_RAY = sum(OPS_RAY.values())                          # 104
FLOP_RAY_SH = FLOP_RAY + sum(OPS_RAY_SH.values())         # 140
# BASELINE.json "metric", verbatim; value = primary rays W*H*spp per frame / frame wall time, in Mrays/s
METRIC = "Mrays/s @1080p, 1M Gaussians; achieved HBM GB/s vs peak; 1→8 GPU scaling"
SRC_DIRS = ("3dgs-raytrace_amd/csrc",)
SRC_FILES = ("include/gsrt.h", "include/gsrt_test.h", "3dgs-raytrace_amd/Makefile")


def src_hash() -> str:
    """Hash of the kernel sources and build flags: ties a committed PMC summary to the code it measured."""
    h = hashlib.sha256()
    files = list(SRC_FILES)
    for d in SRC_DIRS:
        files += [os.path.join(d, f) for f in sorted(os.listdir(os.path.join(ROOT, d)))]
    for f in sorted(files):
        h.update(f.encode())
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warmup-min-s", type=float, default=0.3,
                    help="keep warming up until this many seconds of frames ran (DVFS clock ramp)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the counting pass (roofline operations)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--no-events", action="store_true",
                    help="no per-frame HIP events in the timed region (no kernel_ms / roofline): their cost A/B")
    ap.add_argument("--print-launch", action="store_true",
                    help="with --gpus N > 1 and no WORLD_SIZE: print the child torch.distributed.run command and exit")
    ap.add_argument("--out", default="dump8", choices=["dump8", "rgba32f"],
                    help="sharded frames' exchange format: dump8 = the integers the frame's PPM dump prints, 4 B/pixel "
                         "(GSRT_FLAG_OUT_DUMP8, exact: escapes for the rest), rgba32f = the float framebuffer, 16 B/pixel")
    ap.add_argument("--stream-pages", action="store_true",
                    help="c5: the two jitter sets live in page-locked host memory and every frame streams all of "
                         "the scene's Gaussian pages into HBM (gsrt_scene_stream_pages) instead of a device copy")
    ap.add_argument("--update", default="attach", choices=["attach", "copy"],
                    help="c5 with device-resident jitter sets: attach = the frame reads the set in place "
                         "(gsrt_scene_attach, the producer's arrays are the scene's), copy = gsrt_scene_update copies "
                         "it into the scene's own buffers first (360 MB device to device per frame)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpus():
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max: quota / period), or None when unlimited."""
    rel = ""
    try:
        with open("/proc/self/cgroup") as f:
            for line in f:
                if line.startswith("0::"):  # the cgroup v2 entry
                    rel = line.strip()[3:]
    except OSError:
        pass
    for path in (os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max"), "/sys/fs/cgroup/cpu.max"):
        try:
            with open(path) as f:
                quota, period = f.read().split()[:2]
            if quota != "max":
                return max(1, int(int(quota) // int(period)))
        except (OSError, ValueError):
            continue
    return None


def host_cores() -> dict:
    """The host's logical CPUs (os.cpu_count), those this process may run on (its affinity mask), the CPUs its cgroup
    quota allows, and the CPU share the job was given (OMP_NUM_THREADS; None when unset)."""
    n = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = n
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    except ValueError:
        share = None
    return {"nproc": n, "affinity": max(1, aff), "cgroup_cpus": cgroup_cpus(), "cpu_share": share}


def cpu_threads(cap: int | None = None) -> int:
    """Oracle threads: every core this job may use -- the affinity mask, limited by the cgroup's CPU quota (on the GPU
    pool the mask shows the whole 256-CPU host while the quota gives a one-GPU job 16: 256 threads under it ran at
    0.75 Mrays/s against 1.34 on 16) -- or at most `cap` (the tests' oracle checks)."""
    h = host_cores()
    n = min(h["affinity"], h["cgroup_cpus"] or h["affinity"])
    return max(1, min(cap, n)) if cap else n


def cpu_baseline(params, aabbs, sh, ubo_np, width, height, target_s, gpu_rgba=None):
    """Time the C oracle (COR mode, CPU BVH, all assigned host cores) on a band of rows of the frame."""
    import oracle as O

    threads = cpu_threads()
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
           "cpu_model": cpu_model(), **host_cores(), "threads": threads,
           "sample": f"rows {mid}..{mid + rows - 1} of the same {width}x{height}x{spp}spp frame "
                     f"({rays} rays, {dt:.1f} s, C oracle COR mode + CPU BVH)",
           "kind_note": "the reference's Embree/vulkan-sim CPU path cannot be built or run (SURVEY.md 8c): "
                        "the baseline is this project's C restatement of it (oracle/gsrt_oracle.c)"}
    if gpu_rgba is not None:
        gband = gpu_rgba[mid:mid + rows]
        res["gpu_vs_cpu_linf"] = float(np.abs(gband - out["rgba"][mid:mid + rows]).max())
    res["c1"] = cpu_c1(threads)
    return res


def cpu_c1(threads):
    """BASELINE configs[0] on the CPU oracle: 10k Gaussians, 256x256, 1 spp, in REF mode (the needle cloud: every
    AABB contains the camera, central rays blend through up to 17 rounds, each re-traversing as the reference
    does) and in COR mode (the front-facing cloud)."""
    import oracle as O

    out = {}
    for name, kind, mode in (("ref", O.SYNTH_NEEDLE, O.MODE_REF), ("cor", O.SYNTH_COR, O.MODE_COR)):
        c, r, s, o, _ = O.synth_cloud(kind, 10_000, 42, False)
        p, a = O.gauss_from_model(c, r, s, o)
        ubo = O.make_ubo(O.lookat((0, 0, 0), (0, 0, -1)), 60.0, 256, 256, 1.0, 1, 16)
        bvh = O.Bvh(a)
        t0 = time.perf_counter()
        O.render(p, a, ubo, mode, bvh=bvh, threads=threads)
        dt = time.perf_counter() - t0
        out[name] = {"value": 256 * 256 / dt / 1e6, "unit": "Mrays/s", "ms_per_frame": round(dt * 1e3, 2)}
    return out


def pmc_profile(path, config, kernel="k_render_cor"):
    """The committed rocprofv3 PMC summary for this config, if it was measured on these kernel sources."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, True
    if "config" not in tj:  # one entry per config
        tj = tj.get(config) or {}
    if tj.get("config") != config or kernel not in tj.get("kernel", ""):
        return None, True
    return tj, tj.get("src_hash") != src_hash()


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_command(argv, n: int, port: int):
    """The child that turns `bench.py --gpus n` into n ranks: torch.distributed.run on this node, one process per
    GPU, rendezvous on 127.0.0.1 (the container hostname may not resolve), the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 without WORLD_SIZE: run the N ranks as a child process (started before any GPU call in this
    process; no exec) and relay its output and status. Rank 0 prints the JSON line."""
    cmd = launch_command(argv, args.gpus, free_port())
    if args.print_launch:
        print(json.dumps(cmd), flush=True)
        return 0
    import torch  # device_count() does not initialise the GPU on this image

    have = torch.cuda.device_count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL peer buffers across processes
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def check_world(args) -> int:
    """0 when this process may run as a rank of --gpus ranks, else the exit status (2) after a message."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: an N-GPU measurement needs exactly N ranks "
              f"(run `python bench.py --gpus N`, or torch.distributed.run --nproc-per-node N bench.py --gpus N)",
              file=sys.stderr, flush=True)
        return 2
    return 0


WARM_CHUNK = 8  # warm-up frames between synchronisations (and, with N ranks, between agreements)


def warm_up(frame, sync, warmup, min_s, agree=None, clock=time.perf_counter):
    """Render warm-up frames in chunks of WARM_CHUNK until at least `warmup` frames ran and the warm-up has rendered
    for `min_s` seconds (the DVFS clock ramp), at most 100 * max(warmup, 10) frames. With several ranks `agree(done)`
    returns whether every rank is done (an all-reduce): all ranks then run the same number of frames, so every
    frame's gather has its partners and no rank waits in a synchronisation on a frame the others never issue.
    Returns the frames run."""
    t0 = clock()
    warm, cap = 0, 100 * max(warmup, 10)
    while True:
        for _ in range(WARM_CHUNK):
            frame()
        warm += WARM_CHUNK
        sync()
        done = warm >= cap or (warm >= warmup and clock() - t0 >= min_s)
        if agree is not None:
            done = agree(done)
        if done:
            return warm


def serialized_kernel_ms(ctx, frame, frames=12):
    """The render kernel's mean duration with every frame alone on the GPU: slot streams off and a synchronisation after
    each frame, so no other frame's kernels share the machine with it (on slot streams consecutive frames overlap and
    a render kernel's own events span shared machine time). Every rank runs it (its frames are collective)."""
    old = os.environ.get("GSRT_DEBUG_SLOT_STREAMS")
    os.environ["GSRT_DEBUG_SLOT_STREAMS"] = "0"
    try:
        for _ in range(4):  # the switch back to the two-stream scheme
            frame()
        ctx.synchronize()
        ctx.timing(frames, kernel_only=True)
        for _ in range(frames):
            frame()
            ctx.synchronize()
        k, _ = ctx.timing_read()
        ctx.timing(0)
    finally:
        if old is None:
            del os.environ["GSRT_DEBUG_SLOT_STREAMS"]
        else:
            os.environ["GSRT_DEBUG_SLOT_STREAMS"] = old
    return float(np.mean(k)) if len(k) else None


def sharded_frame_check(scene, ubo, mode, rank):
    """After the timed region of an N-rank run: one more sharded frame (every rank renders its share, the RCCL gather
    brings the packed tiles to rank 0, k_unpack places them), compared on rank 0 bit for bit with rank 0 rendering
    the whole frame alone (dump8 frames: the codes and escapes against the single frame's, and the PPM bytes). Every
    rank must call it (the gather is collective); returns the result on rank 0, else None."""
    import gsrt

    img = scene.render_sharded(ubo, mode, want_image=rank == 0)
    if rank != 0:
        return None
    try:
        return _compare_sharded(scene, ubo, mode, img)
    except gsrt.GsrtError as e:  # e.g. a dump8 frame whose escapes overflowed a rank's list: reported, not fatal
        return {"bit_exact": False, "error": str(e)}


def _compare_sharded(scene, ubo, mode, img):
    import gsrt
    import tempfile

    ref, _ = scene.render(ubo, mode & ~gsrt.FLAG_OUT_DUMP8)
    if not mode & gsrt.FLAG_OUT_DUMP8:
        return {"bit_exact": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32))),
                "linf": float(np.abs(img - ref).max()),
                "what": "the last sharded frame (RCCL gather + k_unpack) against rank 0 rendering the whole frame alone"}
    H, W = ref.shape[:2]
    codes, esc = scene.ctx.dump8_read(W, H)
    wc, we = gsrt.dump8_encode(ref)
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "a.ppm"), os.path.join(d, "b.ppm")
        gsrt.dump_ppm(a, ref)
        gsrt.dump8_ppm(b, codes, esc)
        same_ppm = open(a, "rb").read() == open(b, "rb").read()
    return {"bit_exact": bool(codes.tobytes() == wc.tobytes() and esc.tobytes() == we.tobytes()),
            "ppm_identical": bool(same_ppm), "escapes": int(esc.size),
            "what": "the last sharded frame's dump codes + escapes (RCCL gather + k_unpack_dump8) against those of rank "
                    "0 rendering the whole frame alone in RGBA32F, and the PPM dump of each"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, sys.argv[1:])
    if args.gpus < 1 or check_world(args):
        return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries exactly one line, the JSON: whatever the libraries print there (RCCL's version banner) goes to
    # stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    import gsrt

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    n, W, H, spp, with_sh = CONFIGS[args.config]
    # GSRT_DEBUG_RANK_OF=N or N:r: one GPU renders rank r's (default 0) share of an N-rank frame (libgsrt knob)
    rank_spec = (os.environ.get("GSRT_DEBUG_RANK_OF", "0") or "0").split(":")
    rank_of = int(rank_spec[0])
    rank_sel = int(rank_spec[1]) if len(rank_spec) > 1 else 0

    # (measurement switch: K idle default-priority streams created before the context, as another library's would be;
    # profiles/r06/queue_ab.txt)
    pad_streams = [torch.cuda.Stream(device=local) for _ in range(int(os.environ.get("GSRT_BENCH_PAD_STREAMS", "0")))]
    ctx = gsrt.Context(local)
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
    scene = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    # the LBVH build (synchronous): the first one also pays the runtime's lazy load of the build kernels, the second
    # is the steady-state cost of a rebuild
    tb = time.perf_counter()
    scene.build_bvh()
    bvh_cold_ms = (time.perf_counter() - tb) * 1e3
    tb = time.perf_counter()
    scene.build_bvh()
    bvh_ms = (time.perf_counter() - tb) * 1e3
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, W, H, 1.0, spp, 16)
    mode = gsrt.MODE_COR
    # sharded frames exchange (and keep on rank 0) the frame in this format
    smode = mode | (gsrt.FLAG_OUT_DUMP8 if args.out == "dump8" else 0)

    update = None
    if args.config in DYNAMIC:
        # two jittered copies of the scene (centre + AABB moved by N(0, 1e-3) per axis, seeded) resident in HBM;
        # each step hands one of them to the scene (gsrt_scene_attach, or with --update copy gsrt_scene_update device to
        # device), refits, renders
        p0, a0 = scene.download()
        rng = np.random.default_rng(JITTER_SEED)
        sets = []
        for _ in range(2):
            d = rng.normal(0.0, 1e-3, (n, 3)).astype(np.float32)
            p1, a1 = p0.copy(), a0.copy()
            p1[:, :3] += d
            a1[:, :3] += d
            a1[:, 3:] += d
            if args.stream_pages:
                ctx.host_register(p1)
                ctx.host_register(a1)
                sets.append((p1, a1))
            else:
                sets.append((torch.from_numpy(p1).to(f"cuda:{local}"), torch.from_numpy(a1).to(f"cuda:{local}")))
        torch.cuda.synchronize()
        step_no = [0]
        all_pages = np.arange(scene.pages, dtype=np.uint32)

        def update():
            tp, ta = sets[step_no[0] & 1]
            step_no[0] += 1
            if args.stream_pages:  # host -> HBM over the DMA engines, beside the previous frame's render
                scene.stream_pages(all_pages, tp, ta)
            elif args.update == "attach":
                scene.attach(tp.data_ptr(), ta.data_ptr())
            else:
                scene.update(tp.data_ptr(), ta.data_ptr())
            scene.refit_bvh()

    comm_ranks = 1
    if world > 1:
        uid = [gsrt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], world, rank)
        comm_ranks, comm_rank = ctx.comm_size()
        if comm_ranks != world or comm_rank != rank:
            raise RuntimeError(f"RCCL communicator has {comm_ranks} ranks (this one {comm_rank}); "
                               f"expected {world} (rank {rank})")
        for _ in range(3):  # a few whole frames: warm caches and clocks; the last one's tile costs order the share's
            scene.render(ubo, mode)  # render units (longest first, XCD-balanced: gsrt_render.hip launch_render)
    elif rank_of > 1:
        # a rank share on one GPU goes through the real exchange path: a loopback communicator, the packed render,
        # ncclGather on the comm stream, and for rank 0 the other blocks' arrival + k_unpack (libgsrt debug_rank_of).
        # Its partition is the one an N-rank job's balancing cuts from this frame's row cost profile (gsrt_tile_bands
        # on the whole frame's profile), pinned: one process cannot all-reduce the other ranks' profiles
        ctx.comm_init_loopback()
        for _ in range(3):  # (the last of a few whole frames: warm caches and clocks; its tile costs, as above)
            scene.render(ubo, mode)
        ctx.set_bands(rank_of, gsrt.tile_bands(ubo, rank_of, ctx.row_costs(), smode))

    if world > 1 or rank_of > 1:
        def frame():
            if update:
                update()
            scene.render_sharded_async(ubo, smode)
    else:
        def frame():
            if update:
                update()
            scene.render_async(ubo, mode)

    # counting pass for the algorithmic operations: |C_r|, |H_r| per ray
    stats = None
    if not args.no_stats:
        scene.render_async(ubo, mode | gsrt.FLAG_STATS)
        ctx.synchronize()
        stats = ctx.last_stats((H, W))
    tw = time.perf_counter()
    agree = None
    if world > 1:
        def agree(done):  # every rank stops after the same chunk: the frames' gathers pair up across ranks
            t = torch.tensor([1 if done else 0], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return bool(t[0])
    warm = warm_up(frame, ctx.synchronize, args.warmup, args.warmup_min_s, agree)
    warm_s = time.perf_counter() - tw
    if not args.no_events:
        # the render kernel's two events on every EVENT_STRIDE-th timed frame (no frame start / end events: the events
        # are what the line needs and no more; on every frame they cost the C3 frame ~1.2 %, profiles/r05/events_ab.txt)
        ctx.timing(-(-args.steps // EVENT_STRIDE), kernel_only=True, stride=EVENT_STRIDE)

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
    slot_streams = ctx.slot_streams()
    kern_ms, frame_ms = ctx.timing_read() if not args.no_events else ([], [])
    exch_ms = ctx.timing_read_exchange() if ((world > 1 or rank_of > 1) and not args.no_events) else []
    ctx.timing(0)
    # the roofline needs the render kernel's own duration: when frames overlapped (slot streams), or its events span
    # more than a frame, time it again with frames serialised (after the timed region; not part of `value`)
    ser_ms = None
    if len(kern_ms) and (slot_streams or float(np.mean(kern_ms)) > dt / args.steps * 1e3):
        ser_ms = serialized_kernel_ms(ctx, frame)
    per_rank = None
    if world > 1:
        # every rank's wall time of the K frames, mean render kernel and exchange; the job's time is the slowest
        mine = torch.tensor([dt, float(np.mean(kern_ms)) if len(kern_ms) else -1.0,
                             float(np.mean(exch_ms)) if len(exch_ms) else -1.0], dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        allr = torch.stack(allr).numpy()
        dt = float(allr[:, 0].max())

        def mm(col, scale):
            v = allr[:, col]
            v = v[v >= 0]
            return None if not len(v) else {"min": round(float(v.min()) * scale, 4), "max": round(float(v.max()) * scale, 4),
                                            "argmax_rank": int(np.argmax(allr[:, col]))}
        bands_used = ctx.last_bands()
        frame_check = sharded_frame_check(scene, ubo, smode, rank)
        per_rank = {"frame_ms": mm(0, 1e3 / args.steps), "render_kernel_ms": mm(1, 1.0),
                    "exchange_ms": mm(2, 1.0),
                    "exchange_ms_rank0": round(float(allr[0, 2]), 4) if allr[0, 2] >= 0 else None,
                    "bands": [int(v) for v in bands_used],
                    "note": "frame_ms = a rank's wall time / steps; render_kernel_ms = mean k_render_cor time (HIP "
                            "events); exchange_ms = mean time from the share rendered to the end of ncclGather "
                            "(+ k_unpack on rank 0) on the comm stream: it overlaps the next frame; bands = the tile-row "
                            "partition of the timed frames (cost-balanced from all-reduced row profiles)"}

    rays_per_frame = W * H * spp
    value = rays_per_frame * args.steps / dt / 1e6
    out = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "Mrays/s", "n_gpus": comm_ranks, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.config}: {n} Gaussians{' SH-3' if with_sh else ''}, {W}x{H}, {spp} spp, COR"
                               + (", per-frame centre jitter + refit" if args.config in DYNAMIC else "")
                   + (", Gaussian pages streamed from host memory" if args.config in DYNAMIC and args.stream_pages else "")
                   + (", jitter sets copied into the scene per frame" if args.config in DYNAMIC and not args.stream_pages
                      and args.update == "copy" else ""),
                   "gaussians": n, "width": W, "height": H, "spp": spp, "sh_degree": 3 if with_sh else None,
                   "parallelism": f"tiles/{world}" if world > 1 else "1 GPU",
                   "exchange_format": (("dump8: 4 B/pixel, the integers the PPM dump prints (exact; escapes for the "
                                        "rest)" if args.out == "dump8" else "rgba32f: 16 B/pixel")
                                       if world > 1 or rank_of > 1 else None),
                   "bvh_build_ms": round(bvh_ms, 2), "bvh_build_first_ms": round(bvh_cold_ms, 2)},
        "warmup_frames_run": warm, "warmup_s": round(warm_s, 3),
    }
    if per_rank is not None:
        out["per_rank"] = per_rank
        out["launch"] = "torch.distributed.run, one process per GPU, RCCL communicator of n_gpus ranks"
        if frame_check is not None:
            out["sharded_frame_check"] = frame_check
    if rank_of > 1:  # not a measurement of N GPUs: one GPU renders rank r's share (libgsrt GSRT_DEBUG_RANK_OF)
        out["rank_share"] = (f"rank {rank_sel} of {rank_of} rendered alone on one GPU (GSRT_DEBUG_RANK_OF) through the "
                             f"sharded path on a loopback communicator (packed render, ncclGather"
                             + (f", the other {rank_of - 1} blocks copied in, k_unpack" if rank_sel == 0 else "")
                             + f"): value = the whole frame's rays / the share's frame time, a projection of {rank_of} "
                             f"GPUs without the xGMI link time")
        if len(exch_ms):
            out["rank_share_exchange_ms"] = round(float(np.mean(exch_ms)), 4)
        out["rank_share_bands"] = [int(v) for v in ctx.last_bands()]
    if rank == 0 and stats is not None and len(kern_ms):
        k_ms_timed = float(np.mean(kern_ms))
        k_ms = ser_ms if ser_ms else k_ms_timed
        # per launch: this rank's kernel shades the pixel rows of its band (the whole frame on one GPU; with the
        # GSRT_DEBUG_RANK_OF=N:r measurement knob rank r's band): the counting pass's per-pixel counts over those rows
        pl = gsrt.tile_plan(ubo, mode, 1, 0)
        nr, rr = (world, rank) if world > 1 else ((rank_of, rank_sel) if rank_of > 1 else (1, 0))
        bands = ctx.last_bands() if nr > 1 else np.array([0, pl["tiles_y"]])
        y0, y1 = int(bands[rr]) * pl["tile_h"], min(H, int(bands[rr + 1]) * pl["tile_h"])
        per = stats["per_ray"][y0:y1].astype(np.int64)
        rays, cand, hits = spp * (y1 - y0) * W, int(per[..., 0].sum()), int(per[..., 1].sum())
        flops_launch = ((FLOP_RAY_SH if with_sh else FLOP_RAY) * rays + FLOP_CAND * cand
                        + (FLOP_HIT_SH if with_sh else FLOP_HIT) * hits)
        achieved = flops_launch / (k_ms * 1e-3) / 1e12
        stream_bytes = 16 * rays + 48 * cand + (192 * hits if with_sh else 0)
        prof, stale = pmc_profile(args.traffic, args.config)
        traffic = prof.get("hbm_bytes_per_launch") if prof and not stale else None
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "flop_unit": "FMA = 2 FLOP, as the FP32 peak counts it; per candidate %d, per blended hit %d, per ray %d"
                             % (FLOP_CAND, FLOP_HIT_SH if with_sh else FLOP_HIT, FLOP_RAY_SH if with_sh else FLOP_RAY),
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
                "kernel": "k_render_cor", "kernel_ms": round(k_ms, 4),
                "kernel_ms_timed_frames": round(k_ms_timed, 4),
                "kernel_ms_events": "HIP events around the render kernel of every %dth timed frame (%d of %d), on its "
                                    "own stream" % (EVENT_STRIDE, len(kern_ms), args.steps),
                "alg_flop_per_launch": int(flops_launch),
                "mean_candidates_per_ray": round(cand / max(rays, 1), 2),
                "mean_blended_per_ray": round(hits / max(rays, 1), 2),
                "per_ray_streaming_bytes": int(stream_bytes),
                "traffic_stale": bool(prof is None or stale), "src_hash": src_hash()}
        if ser_ms:
            roof["kernel_ms_from"] = ("frames serialised after the timed region (slot streams off, a synchronisation "
                                      "per frame): in the timed frames consecutive frames overlap (slot streams, "
                                      "DESIGN.md §3), so kernel_ms_timed_frames spans shared machine time")
        elif k_ms > dt / args.steps * 1e3:
            roof["frac"] = None  # not a kernel duration of its own
        if traffic:
            roof["hbm_gbs"] = round(traffic / (k_ms * 1e-3) / 1e9, 1)
            roof["hbm_frac"] = round(roof["hbm_gbs"] / HBM_PEAK_GBS, 4)
        if prof and not stale and prof.get("valu_issue_ms"):
            # VALU issue time of one launch (PMC: instructions x 2 cycles / 1024 SIMDs / clock) over this run's
            # kernel time: the fraction of the SIMDs' issue slots the kernel's VALU work occupies
            roof["valu_issue_frac"] = round(prof["valu_issue_ms"] / k_ms, 4)
            if prof.get("lds_array_ms"):
                # LDS-array busy time of one launch (PMC SQ_LDS_IDX_ACTIVE / 256 CUs / clock) over this run's kernel
                # time: the LDS array, shared by a CU's 4 SIMDs, is the render kernel's tightest pipe
                roof["lds_array_frac"] = round(prof["lds_array_ms"] / k_ms, 4)
            roof["pmc_profile"] = os.path.relpath(args.traffic, ROOT) + " (" + str(prof.get("tag")) + ")"
        out["roofline"] = roof
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rgba, _ = scene.render(ubo, mode)
        p, a = scene.download()
        out["cpu_baseline"] = cpu_baseline(p, a, sh, ubo, W, H, args.cpu_seconds, gpu_rgba=rgba)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
