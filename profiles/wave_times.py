"""Per-workgroup timeline of one C3 frame (diagnostic build, GSRT_WAVE_TIMES):

  make -C 3dgs-raytrace_amd gsrt/libgsrt_xwt.so XFLAGS=-DGSRT_WAVE_TIMES
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/libgsrt_xwt.so python profiles/wave_times.py [config] > out.txt

Renders 40 frames, then reads the last frame's {start, end, HW_ID, XCC_ID} per workgroup of k_render_cor and
k_group_list (100-MHz real-time counter) and prints: kernel span, wave-duration percentiles, concurrency over
time (waves in flight per SIMD, in 5 % bins of the span), the tail (time from the 95th/99th percentile end to the
last end), and the spread of per-XCD and per-CU finish times."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs-raytrace_amd"), ROOT]
import bench  # noqa: E402
import gsrt  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n, W, H, spp, with_sh = bench.CONFIGS[cfg]
ctx = gsrt.Context(0)
c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 42, with_sh)
scene = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
scene.build_bvh()
ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
share = bool(os.environ.get("GSRT_DEBUG_RANK_OF"))
spec = os.environ.get("GSRT_DEBUG_RANK_OF", "1").split(":")
nr, rk = int(spec[0]), int(spec[1]) if len(spec) > 1 else 0  # rank rk's share of an nr-rank sharded frame
if share:  # a rank share runs through the sharded path on a loopback communicator, bands as bench.py
    ctx.comm_init_loopback()
    for _ in range(3):
        scene.render(ubo, gsrt.MODE_COR)
    ctx.set_bands(nr, gsrt.tile_bands(ubo, nr, ctx.row_costs()))
for _ in range(40):
    (scene.render_sharded_async if share else scene.render_async)(ubo, gsrt.MODE_COR)
ctx.synchronize()
L = gsrt.lib
L.gsrt_diag_stamps.argtypes = [ctypes.c_void_p]
L.gsrt_diag_wave_times.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
plan = gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks=nr, rank=rk)
if share:
    b = ctx.last_bands()
    plan["local_tiles"] = plan["tiles_x"] * int(b[rk + 1] - b[rk])
stamps = np.zeros(4, np.uint32)
L.gsrt_diag_stamps(stamps.ctypes.data)
for kind, name, count in ((0, "k_render_cor", plan["local_tiles"]), (1, "k_group_list", None)):
    buf = np.zeros((1 << 18, 4), np.uint32)
    assert L.gsrt_diag_wave_times(kind, buf.ctypes.data, 1 << 18) == 0
    m = buf[:, 1] != 0
    if count is not None:
        m[count:] = False
    t = buf[m]
    t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    base = t0.min()
    t0 -= base; t1 -= base
    span = t1.max()
    dur = t1 - t0
    hw, xcc = t[:, 2], t[:, 3]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    print(f"== {name} (rank {rk} of {nr}): {len(t)} workgroups, span {span / 100:.1f} us (10 ns ticks)")
    if kind == 0:
        print(f"   render stream reaches the kernel -> first wave starts {(int(base) - int(stamps[0])) / 100:.1f} us; "
              f"last wave ends -> stream passes the kernel {(int(stamps[1]) - int(base + span)) / 100:.1f} us")
    print("   wave us p10/p50/p90/p99/max: " + " ".join(f"{np.percentile(dur, q) / 100:.1f}" for q in (10, 50, 90, 99, 100)))
    ends = np.sort(t1)
    print(f"   tail: last end - p95 end {(span - ends[int(0.95 * len(ends))]) / 100:.1f} us, - p99 end "
          f"{(span - ends[int(0.99 * len(ends))]) / 100:.1f} us; first-start spread {np.sort(t0)[len(t0) // 100] / 100:.1f} us")
    bins = 20
    edges = np.linspace(0, span, bins + 1)
    mid = 0.5 * (edges[:-1] + edges[1:])
    conc = [(np.sum((t0 <= x) & (t1 > x))) / 1024.0 for x in mid]
    print("   waves/SIMD in flight by 5 % of span: " + " ".join(f"{v:.1f}" for v in conc))
    xe = [t1[xcc == x].max() / 100 for x in np.unique(xcc)]
    print("   per-XCD last end us: " + " ".join(f"{v:.1f}" for v in xe))
    key = xcc.astype(np.int64) * 1024 + se * 64 + cu * 4 + simd
    cu_end = {}
    for k_, e in zip(key // 4, t1):
        cu_end[k_] = max(cu_end.get(k_, 0), e)
    ce = np.array(list(cu_end.values())) / 100
    print(f"   per-CU last end us: min {ce.min():.1f} p50 {np.median(ce):.1f} max {ce.max():.1f} ({len(ce)} CUs)")
    # the load of each SIMD: its waves' summed durations (co-resident waves share it, so a sum over-counts, but the
    # spread across SIMDs shows the balance) and its wave count
    sload, scount = {}, {}
    for k_, d_ in zip(key, dur):
        sload[k_] = sload.get(k_, 0) + d_
        scount[k_] = scount.get(k_, 0) + 1
    sl = np.array(list(sload.values())) / 100
    sc_ = np.array(list(scount.values()))
    print(f"   per-SIMD summed wave us: min {sl.min():.1f} p50 {np.median(sl):.1f} p99 {np.percentile(sl, 99):.1f} "
          f"max {sl.max():.1f}; waves per SIMD min {sc_.min()} p50 {np.median(sc_):.0f} max {sc_.max()} ({len(sl)} SIMDs)")
    xl = [dur[xcc == x].sum() / 100 for x in np.unique(xcc)]
    print("   per-XCD summed wave us: " + " ".join(f"{v:.0f}" for v in xl))
