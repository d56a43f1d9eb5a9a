"""N>1 tile sharding on CPU (gloo, world_size 2 and 3): every rank renders only its band of tile rows (the
partition gsrt_tile_bands cuts from a row cost profile), packs its tiles with the library's host mirror of the packed
render layout (gsrt_tile_pack_host), the packed buffers are gathered to rank 0, and rank 0's unpack
(gsrt_tile_unpack_host, the index map of the HIP k_unpack kernel, from the same inline mappings the kernels compile)
must rebuild the single-process frame bit for bit. The library's balancing rule and layout are also checked against
this file's independent restatement. The GPU variant of this check (same packing and unpack kernels, RCCL transport
skipped) is tests/test_render_gpu.py::test_sharded_*."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


SUPER = 16  # super-tile edge in tiles (gsrt_device.hpp kSuper)


def _spatial_tile(k, tiles_x, tiles_y):
    """Tile of position k in the spatial order of a tiles_x x tiles_y grid (super-tiles row-major, row-major inside)."""
    R = k // (SUPER * tiles_x)
    hR = min(SUPER, tiles_y - R * SUPER)
    k1 = k - R * SUPER * tiles_x
    C = k1 // (hR * SUPER)
    wC = min(SUPER, tiles_x - C * SUPER)
    k2 = k1 - C * hR * SUPER
    return C * SUPER + k2 % wC, R * SUPER + k2 // wC


def _root_weight(nranks, spp, cor=True, dump8=False):
    """rank 0's weight (restates gsrt_render.hip root_weight in float32): 1 - c (N - 1) / spp, in [1/4, 1], with
    c = 0.09 for RGBA32F tiles and 0.07 for the dump8 exchange format"""
    if nranks <= 1 or not cor:
        return 1.0
    f = np.float32
    w = f(1.0) - f(0.07 if dump8 else 0.09) * f(nranks - 1) / f(spp)
    return float(min(max(w, f(0.25)), f(1.0)))


def _balance(tiles_y, nranks, cost, w0):
    """The balancing rule as a spec: cumulative cost targets by weight (rank 0: w0, the others 1), each boundary at the
    row boundary nearest its target (ties to the upper rows' side), leaving every band at least one row when
    tiles_y >= nranks."""
    c = np.ones(tiles_y, np.int64) if cost is None else np.asarray(cost, np.int64)
    P = np.concatenate([[0], np.cumsum(c)])
    wtot = w0 + (nranks - 1)
    minrow = 1 if tiles_y >= nranks else 0
    out = [0] * (nranks + 1)
    out[nranks] = tiles_y
    wsum = 0.0
    for r in range(1, nranks):
        wsum += w0 if r == 1 else 1.0
        target = float(P[-1]) * wsum / wtot
        lo, hi = out[r - 1] + minrow, tiles_y - (nranks - r) * minrow
        ge = [i for i in range(lo, hi + 1) if P[i] >= np.ceil(target)]
        i = ge[0] if ge else hi
        if i > lo and P[i] - target > target - P[i - 1]:
            i -= 1
        out[r] = i
    return out


def _local_positions(tiles_x, bands, rank):
    """(tx, ty) of rank's local tiles in local order: the spatial order of its band's own grid"""
    r0, r1 = int(bands[rank]), int(bands[rank + 1])
    out = []
    for k in range(tiles_x * (r1 - r0)):
        cx, cy = _spatial_tile(k, tiles_x, r1 - r0)
        out.append((cx, r0 + cy))
    return out


def _stride(tiles_x, bands):
    return tiles_x * int(np.diff(np.asarray(bands, np.int64)).max())


def _pack(rgba, plan, bands, rank):
    tw, th = plan["tile_w"], plan["tile_h"]
    H, W = rgba.shape[:2]
    out = np.zeros((_stride(plan["tiles_x"], bands), th * tw, 4), np.float32)
    for i, (cx, cy) in enumerate(_local_positions(plan["tiles_x"], bands, rank)):
        x0, y0 = cx * tw, cy * th
        for p in range(tw * th):
            x, y = x0 + p % tw, y0 + p // tw
            if x < W and y < H:
                out[i, p] = rgba[y, x]
    return out


def _unpack(gathered, plan, bands, W, H, nranks):
    tw, th = plan["tile_w"], plan["tile_h"]
    owner = {}
    for r in range(nranks):
        for lt, t in enumerate(_local_positions(plan["tiles_x"], bands, r)):
            owner[t] = (r, lt)
    assert len(owner) == plan["tiles_x"] * plan["tiles_y"]  # the bands partition the tiles
    fb = np.zeros((H, W, 4), np.float32)
    for y in range(H):
        for x in range(W):
            r, lt = owner[(x // tw, y // th)]
            fb[y, x] = gathered[r, lt, (y % th) * tw + (x % tw)]
    assert gathered.shape[0] == nranks and gathered.shape[1] == _stride(plan["tiles_x"], bands)
    return fb


def _synthetic_cost(tiles_y, seed):
    """a row cost profile with a heavy middle, as a front-facing cloud produces"""
    rng = np.random.default_rng(seed)
    y = (np.arange(tiles_y) + 0.5) / tiles_y
    return (24 * 400 + 40000 * np.exp(-((y - 0.5) / 0.2) ** 2) + rng.integers(0, 3000, tiles_y)).astype(np.uint32)


@pytest.mark.parametrize("w,h,spp,nranks", [(1920, 1080, 4, 8), (1920, 1080, 4, 2), (3840, 2160, 1, 8),
                                            (1920, 1080, 16, 3), (640, 360, 1, 8), (48, 32, 1, 3), (64, 16, 1, 8)])
@pytest.mark.parametrize("profile", [False, True])
def test_bands_partition_and_balance(w, h, spp, nranks, profile):
    """Host-only: the library's bands equal the restated rule, partition the tile rows (non-empty when there are
    enough rows), the plan's local counts and packed stride follow them, and the heaviest band is within one row of the
    best whole-row split's."""
    import gsrt
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, w, h, 1.0, spp, 16)
    pl = gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks, 0)
    ty = pl["tiles_y"]
    cost = _synthetic_cost(ty, w + nranks) if profile else None
    w0 = _root_weight(nranks, spp)
    b = gsrt.tile_bands(ubo, nranks, cost)
    assert b.tolist() == _balance(ty, nranks, cost, w0)
    b8 = gsrt.tile_bands(ubo, nranks, cost, gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8)  # the dump8 exchange's root weight
    assert b8.tolist() == _balance(ty, nranks, cost, _root_weight(nranks, spp, dump8=True))
    assert b[0] == 0 and b[-1] == ty and np.all(np.diff(b.astype(np.int64)) >= (1 if ty >= nranks else 0))
    c = np.ones(ty, np.int64) if cost is None else cost.astype(np.int64)
    load = [c[b[r]:b[r + 1]].sum() / (w0 if r == 0 else 1.0) for r in range(nranks)]
    # every boundary sits within one row of its target: the heaviest band exceeds the ideal by < 2 rows' cost
    ideal = c.sum() / (w0 + nranks - 1)
    assert max(load) <= ideal + 2 * c.max() / min(w0, 1.0)
    if cost is None:  # the even partition is what gsrt_tile_plan reports
        plans = [gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks, r) for r in range(nranks)]
        assert [p["row0"] for p in plans] == b[:-1].tolist()
        assert [p["local_tiles"] for p in plans] == [pl["tiles_x"] * int(b[r + 1] - b[r]) for r in range(nranks)]
        assert plans[0]["stride"] == _stride(pl["tiles_x"], b)
        if w0 < 1.0 and ty >= 4 * nranks:  # the gather's root takes the lighter band
            assert plans[0]["local_tiles"] < min(p["local_tiles"] for p in plans[1:])


def test_bands_rule_edges():
    """a single rank owns every row; more ranks than rows leave some bands empty but still cut 0..tiles_y"""
    import gsrt
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 32, 16, 1.0, 1, 16)
    assert gsrt.tile_bands(ubo, 1).tolist() == [0, gsrt.tile_plan(ubo)["tiles_y"]]
    ty = gsrt.tile_plan(ubo)["tiles_y"]  # 2 rows of 8x8 tiles
    b = gsrt.tile_bands(ubo, 5)
    assert b.tolist() == _balance(ty, 5, None, _root_weight(5, 1)) and b[0] == 0 and b[-1] == ty
    assert np.all(np.diff(b.astype(np.int64)) >= 0)


def _worker(rank, nranks, port, mode, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "3dgs-raytrace_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import gsrt
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        g = np.load(os.path.join(GOLD, "cor_10k.npz" if mode == "cor" else "ref_needles_300.npz"), allow_pickle=False)
        p, a = O.gauss_from_model(g["center"], g["rot"], g["scale"], g["opacity"])
        ubo = g["ubo"].view(O.UBO_DTYPE)
        W, H = int(ubo["width"][0]), int(ubo["height"][0])
        m = gsrt.MODE_COR if mode == "cor" else gsrt.MODE_REF
        plan = gsrt.tile_plan(ubo, m, nranks, rank)
        # a cost-balanced partition (the bands a profile of this frame would give), the same on every rank
        bands = gsrt.tile_bands(ubo, nranks, _synthetic_cost(plan["tiles_y"], 7), m)
        # each rank renders the frame with the oracle and keeps only its own tiles
        full = O.render(p, a, ubo, O.MODE_COR if mode == "cor" else O.MODE_REF, bvh=O.Bvh(a), threads=2,
                        want_raystate=(mode == "ref"))
        img = full["rgba"] if mode == "cor" else np.stack([full["raystate"]["trans"]] * 4, -1).astype(np.float32)
        # the library's own host mirror of the packed layout (gsrt_tile_pack_host: the mappings the kernels use)
        # against this file's independent restatement of it
        packed = gsrt.tile_pack(ubo, img, nranks, rank, m, bands=bands)
        assert packed.tobytes() == _pack(img, plan, bands, rank).tobytes()
        import torch
        t = torch.from_numpy(packed)
        bufs = [torch.zeros_like(t) for _ in range(nranks)] if rank == 0 else None
        dist.gather(t, gather_list=bufs, dst=0)
        if rank == 0:
            gathered = np.stack([b.numpy() for b in bufs])
            fb = gsrt.tile_unpack(ubo, gathered, nranks, m, bands=bands)  # k_unpack's index map, on the host
            assert fb.tobytes() == _unpack(gathered, plan, bands, W, H, nranks).tobytes()
            want = g["rgba"] if mode == "cor" else np.stack([g["raystate"].view(O.RAYSTATE_DTYPE)["trans"]] * 4, -1)
            q.put(bool(fb.tobytes() == np.ascontiguousarray(want, np.float32).tobytes()))
    finally:
        dist.destroy_process_group()


def _worker_dump8(rank, nranks, port, q):
    """GSRT_FLAG_OUT_DUMP8 over a non-RCCL transport: each rank packs its dump8 block of the golden frame (with escapes
    added) by the host mirror, gloo gathers the blocks, rank 0 unpacks them; the codes, escapes and PPM are the frame's"""
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "3dgs-raytrace_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import gsrt
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        g = np.load(os.path.join(GOLD, "cor_10k.npz"), allow_pickle=False)
        ubo = g["ubo"].view(O.UBO_DTYPE)
        img = np.array(g["rgba"], np.float32)
        flat = img.reshape(-1, 4)
        at = np.random.default_rng(5).choice(flat.shape[0], 40, replace=False)
        flat[at, np.arange(40) % 3] = np.array([np.nan, -1.0, 7.5, -0.0], np.float32)[np.arange(40) % 4]
        plan = gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks, rank)
        bands = gsrt.tile_bands(ubo, nranks, _synthetic_cost(plan["tiles_y"], 3), gsrt.MODE_COR)
        import torch
        t = torch.from_numpy(gsrt.tile_pack_dump8(ubo, img, nranks, rank, bands=bands).view(np.int32))
        bufs = [torch.zeros_like(t) for _ in range(nranks)] if rank == 0 else None
        dist.gather(t, gather_list=bufs, dst=0)
        if rank == 0:
            gathered = np.stack([b.numpy().view(np.uint32) for b in bufs])
            codes, esc = gsrt.tile_unpack_dump8(ubo, gathered, nranks, bands=bands)
            c0, e0 = gsrt.dump8_encode(img)
            with tempfile.TemporaryDirectory() as d:
                a, b = os.path.join(d, "f.ppm"), os.path.join(d, "c.ppm")
                gsrt.dump_ppm(a, img)
                gsrt.dump8_ppm(b, codes, esc)
                same_ppm = open(a, "rb").read() == open(b, "rb").read()
            q.put(bool(np.array_equal(codes, c0) and esc.tobytes() == e0.tobytes() and esc.size == 40 and same_ppm))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nranks", [2, 3])
def test_dump8_exchange_gloo(nranks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_dump8, args=(r, nranks, port, q)) for r in range(nranks)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("nranks,mode", [(2, "cor"), (3, "cor"), (2, "ref")])
def test_tile_sharding_gloo(nranks, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, nranks, port, mode, q)) for r in range(nranks)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    assert q.get(timeout=5) is True


def _skewed_cost(tiles_y):
    """a row profile heavier towards the bottom of the frame: the even bands are far from balanced"""
    return (_synthetic_cost(tiles_y, 11) * (1.0 + 3.0 * np.arange(tiles_y) / tiles_y)).astype(np.uint32)


def _worker_decide(rank, nranks, port, case, q):
    """The partition rule of a profile frame over a real multi-process all-reduce (gloo standing in for RCCL's
    ncclAllReduce max): every rank contributes its own band's row costs (different on every rank) and its partition
    hash; each applies gsrt_decide_bands to the reduced profile. case "agree": all ranks adopt the same bands, those the
    balancing rule cuts from the whole profile; "pinned": one rank pinned its bands, the others did not; "bands": one
    rank renders other bands. The last two fail with E_COMM on every rank, before any gather could pair mismatched
    layouts."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "3dgs-raytrace_amd"))
    import gsrt
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
        ty = gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks, 0)["tiles_y"]
        bands = gsrt.tile_bands(ubo, nranks)  # the even partition every rank starts from
        if case == "bands" and rank == nranks - 1:
            bands = bands.copy()
            bands[1] += 1
        pinned = case == "pinned" and rank == 1
        full = _skewed_cost(ty)
        mine = np.zeros(ty, np.int64)
        mine[bands[rank]:bands[rank + 1]] = full[bands[rank]:bands[rank + 1]]  # only this rank's rows were measured
        h = gsrt.partition_hash(ubo, nranks, bands, pinned)
        t = torch.from_numpy(np.concatenate([mine, [h, (~h) & 0xffffffff]]).astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        prof = t.numpy().astype(np.uint32)
        try:
            out = gsrt.decide_bands(ubo, nranks, bands, prof, h, pinned).astype(np.int64)
            status = 0
        except gsrt.GsrtError as e:
            out, status = np.full(nranks + 1, -1, np.int64), e.status
        res = torch.from_numpy(np.concatenate([[status], out]))
        allr = [torch.zeros_like(res) for _ in range(nranks)]
        dist.all_gather(allr, res)
        if rank == 0:
            rows = np.stack([a.numpy() for a in allr])
            if case == "agree":
                want = gsrt.tile_bands(ubo, nranks, full)  # the whole profile's cut (it lowers the peak well over 2 %)
                ok = bool(np.all(rows[:, 0] == 0) and np.all(rows[:, 1:] == want.astype(np.int64)) and
                          want.tolist() != gsrt.tile_bands(ubo, nranks).tolist())
            else:
                ok = bool(np.all(rows[:, 0] == gsrt.E_COMM))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nranks,case", [(2, "agree"), (3, "agree"), (3, "pinned"), (2, "bands")])
def test_band_decision_gloo(nranks, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_decide, args=(r, nranks, port, case, q)) for r in range(nranks)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    assert q.get(timeout=5) is True


def test_band_decision_pinned_keeps_bands():
    """pinned bands are kept whatever the profile; unpinned ones only move when the new cut lowers the peak by 2 %"""
    import gsrt
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, 4, 16)
    ty = gsrt.tile_plan(ubo)["tiles_y"]
    even = gsrt.tile_bands(ubo, 4)
    prof = np.concatenate([_skewed_cost(ty), [0, 0]]).astype(np.uint32)
    for pinned in (False, True):
        h = gsrt.partition_hash(ubo, 4, even, pinned)
        assert h != gsrt.partition_hash(ubo, 4, even, not pinned)
        prof[ty], prof[ty + 1] = h, (~h) & 0xffffffff
        out = gsrt.decide_bands(ubo, 4, even, prof, h, pinned)
        want = even if pinned else gsrt.tile_bands(ubo, 4, prof[:ty])
        assert out.tolist() == want.tolist()
        assert pinned or out.tolist() != even.tolist()
    flat = np.concatenate([np.ones(ty, np.uint32), [0, 0]]).astype(np.uint32)  # a flat profile: even is within 2 %
    h = gsrt.partition_hash(ubo, 4, even)
    flat[ty], flat[ty + 1] = h, (~h) & 0xffffffff
    assert gsrt.decide_bands(ubo, 4, even, flat, h).tolist() == even.tolist()
