"""GPU LBVH checks: Morton codes and the radix sort against numpy, structural validity of the Karras
hierarchy, exact bottom-up boxes, and refit."""
import numpy as np
import pytest

import gsrt
import oracle as O

pytestmark = pytest.mark.gpu


def _expand(v):
    v = v.astype(np.uint64)
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v.astype(np.uint32)


def _morton_np(aabbs):
    a = aabbs.astype(np.float32)
    c = np.float32(0.5) * (a[:, :3] + a[:, 3:])
    lo, hi = c.min(0), c.max(0)
    ext = hi - lo
    u = np.where(ext > 0, (c - lo) / np.where(ext > 0, ext, 1), np.float32(0)).astype(np.float32)
    q = np.clip(u * np.float32(1024.0), 0, 1023).astype(np.uint32)
    return (_expand(q[:, 0]) << 2) | (_expand(q[:, 1]) << 1) | _expand(q[:, 2])


def _check_tree(sc, aabbs):
    n = aabbs.shape[0]
    nodes, gid, morton = sc.bvh_download()
    info = sc.bvh_info()
    assert info["n_internal"] == max(n - 1, 0)
    codes = _morton_np(aabbs) if n > 1 else np.zeros(1, np.uint32)
    if n > 1:
        order = np.argsort(codes, kind="stable")
        np.testing.assert_array_equal(gid, order.astype(np.uint32))   # stable LSD radix sort
        np.testing.assert_array_equal(morton, codes[order])
    fl = nodes.view(np.float32)
    leaf_seen = np.zeros(n, np.int32)
    # per node: [l_lo 3, l_ref, l_hi 3, r_ref, r_lo 3, l_key, r_hi 3, r_key]
    boxes = {}

    def box_of(ref):
        if ref & 0x80000000:
            return aabbs[ref & 0x7FFFFFFF]
        return boxes[ref]

    if n > 1:
        # post-order: compute each internal node's exact union and compare with the stored child boxes
        stack, post = [0], []
        while stack:
            i = stack.pop()
            post.append(i)
            for ref in (nodes[i, 3], nodes[i, 7]):
                if ref & 0x80000000:
                    leaf_seen[ref & 0x7FFFFFFF] += 1
                else:
                    stack.append(ref)
        assert len(post) == n - 1 and len(set(post)) == n - 1  # every internal node reached exactly once
        for i in reversed(post):
            lb, rb = box_of(nodes[i, 3]), box_of(nodes[i, 7])
            np.testing.assert_array_equal(fl[i, [0, 1, 2, 4, 5, 6]], lb)
            np.testing.assert_array_equal(fl[i, [8, 9, 10, 12, 13, 14]], rb)
            boxes[i] = np.concatenate([np.minimum(lb[:3], rb[:3]), np.maximum(lb[3:], rb[3:])])
        np.testing.assert_array_equal(info["root_box"], boxes[0])
        assert (leaf_seen == 1).all()
    else:
        np.testing.assert_array_equal(info["root_box"], aabbs[0])
    want_root = np.concatenate([aabbs[:, :3].min(0), aabbs[:, 3:].max(0)])
    np.testing.assert_array_equal(info["root_box"], want_root)
    return info


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 65537])
def test_lbvh_structure(ctx, n):
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 123)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    _, a = sc.download()
    info = _check_tree(sc, a)
    assert info["max_depth"] <= 64


def test_lbvh_duplicate_centroids(ctx):
    n = 5000
    c = np.zeros((n, 3), np.float32)
    c[: n // 2] = (1.0, 2.0, 3.0)        # half the Gaussians share one centroid (equal Morton codes)
    c[n // 2:] = np.random.default_rng(1).random((n - n // 2, 3), dtype=np.float32)
    rot = np.tile(np.float32([1, 0, 0, 0]), (n, 1))
    sc = gsrt.Scene.from_model(ctx, c, rot, np.full((n, 3), 0.01, np.float32), np.full(n, 0.5, np.float32))
    sc.build_bvh()
    _, a = sc.download()
    _check_tree(sc, a)


def test_refit(ctx):
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 7)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    p, a = sc.download()
    a2 = a.copy()
    rng = np.random.default_rng(3)
    shift = rng.normal(0, 1e-2, (a.shape[0], 3)).astype(np.float32)
    a2[:, :3] += shift
    a2[:, 3:] += shift
    sc.refit_bvh(a2)
    nodes, gid, _ = sc.bvh_download()
    _check_tree_boxes_only(sc, a2)
    # the refit tree renders exactly what a fresh build over the same AABBs renders
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 48, 1.0, 1, 16)
    img_refit, _ = sc.render(ubo, gsrt.MODE_COR)
    fresh = gsrt.Scene.from_params(ctx, p, a2)
    fresh.build_bvh()
    img_fresh, _ = fresh.render(ubo, gsrt.MODE_COR)
    assert img_refit.tobytes() == img_fresh.tobytes()


def _check_tree_boxes_only(sc, aabbs):
    nodes, _, _ = sc.bvh_download()
    fl = nodes.view(np.float32)
    n = aabbs.shape[0]
    boxes = {}
    stack, post = [0], []
    while stack:
        i = stack.pop()
        post.append(i)
        for ref in (nodes[i, 3], nodes[i, 7]):
            if not ref & 0x80000000:
                stack.append(ref)
    for i in reversed(post):
        bb = []
        for ref, cols in ((nodes[i, 3], [0, 1, 2, 4, 5, 6]), (nodes[i, 7], [8, 9, 10, 12, 13, 14])):
            want = aabbs[ref & 0x7FFFFFFF] if ref & 0x80000000 else boxes[ref]
            np.testing.assert_array_equal(fl[i, cols], want)
            bb.append(want)
        boxes[i] = np.concatenate([np.minimum(bb[0][:3], bb[1][:3]), np.maximum(bb[0][3:], bb[1][3:])])
    assert len(post) == n - 1


def test_leaf_keys_in_nodes(ctx):
    """COR projection scatters each leaf's depth key (-view z, +inf when invalid) into its parent node."""
    n = 3000
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 11)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    mv = gsrt.lookat((0.0, 0.0, 0.5), (0.0, 0.0, -1.0))   # camera inside the cloud: some depths <= 0
    ubo = gsrt.camera_from_modelview(mv, 60.0, 32, 24, 1.0, 1, 16)
    sc.render(ubo, gsrt.MODE_COR)
    nodes, _, _ = sc.bvh_download()
    m = np.asarray(ubo["model_view"], np.float32).reshape(4, 4)    # column-major: m[col, row]
    p, _ = sc.download()
    x, y, z = (p[:, k].astype(np.float32) for k in range(3))
    vz = ((m[0, 2] * x + m[1, 2] * y) + m[2, 2] * z) + m[3, 2]       # mul4v order, no contraction
    depth = (-vz).astype(np.float32)
    seen = 0
    for i in range(n - 1):
        for ref, col in ((nodes[i, 3], 11), (nodes[i, 7], 15)):
            if ref & 0x80000000:
                g = ref & 0x7FFFFFFF
                key = np.uint32(nodes[i, col]).view(np.float32)
                if depth[g] > 0:
                    assert key == depth[g] or np.isinf(key)   # inf only when the 2D covariance is singular
                else:
                    assert np.isinf(key) and key > 0
                seen += 1
    assert seen == n


def test_scene_update_and_refit_matches_rebuild(ctx):
    """Dynamic scene (config 5): jitter the centres, push the new GaussParam/AABB arrays with
    gsrt_scene_update, refit asynchronously and render: identical to a scene built from scratch over the moved
    Gaussians, and to the oracle. Device-pointer updates go through the same entry point (bench.py)."""
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
        p2 = p.copy()
        a2 = a.copy()
        p2[:, :3] += d
        a2[:, :3] += d
        a2[:, 3:] += d
        sc.update(p2, a2)
        sc.refit_bvh()
        img, _ = sc.render(ubo, gsrt.MODE_COR)
        fresh = gsrt.Scene.from_params(ctx, p2, a2, sh)
        fresh.build_bvh()
        want, _ = fresh.render(ubo, gsrt.MODE_COR)
        assert img.tobytes() == want.tobytes()
        np.testing.assert_array_equal(sc.bvh_info()["root_box"], np.concatenate([a2[:, :3].min(0), a2[:, 3:].max(0)]))
        p, a = p2, a2
    ref = O.render(p, a, O.make_ubo(mv, 60.0, 96, 64, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a))["rgba"]
    assert img.tobytes() == ref.tobytes()


def test_device_updates(ctx):
    """Updates from device memory (device-to-device copies on the prep stream): an odd Gaussian count (24 n bytes
    of AABBs is not a multiple of 16), whole-array update, a device-array refit, pages streamed from device arrays,
    and a source 4 B off 16-B alignment. Every frame equals a scene built from the same arrays."""
    import torch

    n = 30001
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 9, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    p, a = sc.download()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 96, 64, 1.0, 4, 16)

    def same_as_fresh(p2, a2):
        img, _ = sc.render(ubo, gsrt.MODE_COR)
        fresh = gsrt.Scene.from_params(ctx, p2, a2, sh)
        fresh.build_bvh()
        want, _ = fresh.render(ubo, gsrt.MODE_COR)
        fresh.close()
        assert img.tobytes() == want.tobytes()

    p1, a1 = _jittered(p, a, 21)
    tp, ta = torch.from_numpy(p1).cuda(), torch.from_numpy(a1).cuda()
    sc.update(tp.data_ptr(), ta.data_ptr())
    sc.refit_bvh()
    torch.cuda.synchronize()
    same_as_fresh(p1, a1)
    np.testing.assert_array_equal(sc.download()[1], a1)  # the tail of the AABB array too

    p2, a2 = _jittered(p1, a1, 22)
    tp2, ta2 = torch.from_numpy(p2).cuda(), torch.from_numpy(a2).cuda()
    sc.update(tp2.data_ptr(), None)
    sc.refit_bvh(ta2.data_ptr())
    same_as_fresh(p2, a2)

    p3, a3 = _jittered(p2, a2, 23)
    tp3, ta3 = torch.from_numpy(p3).cuda(), torch.from_numpy(a3).cuda()
    pages = [0, 2, sc.pages - 1]
    sc.stream_pages(pages, tp3.data_ptr(), ta3.data_ptr())
    sc.refit_bvh()
    pw, aw = p2.copy(), a2.copy()
    for q in pages:
        g0, g1 = q * gsrt.PAGE_GAUSSIANS, min((q + 1) * gsrt.PAGE_GAUSSIANS, n)
        pw[g0:g1], aw[g0:g1] = p3[g0:g1], a3[g0:g1]
    same_as_fresh(pw, aw)

    # a misaligned device source (4 B past a 16-B boundary)
    p4, a4 = _jittered(pw, aw, 24)
    buf = torch.zeros(a4.size + 1, dtype=torch.float32, device="cuda")
    buf[1:] = torch.from_numpy(a4.reshape(-1)).cuda()
    sc.refit_bvh(buf.data_ptr() + 4)
    same_as_fresh(pw, a4)


# ---- Gaussian pages: host-resident Gaussians streamed into HBM page by page


def _jittered(p, a, seed, scale=1e-3):
    rng = np.random.default_rng(seed)
    d = rng.normal(0.0, scale, (p.shape[0], 3)).astype(np.float32)
    p1, a1 = p.copy(), a.copy()
    p1[:, :3] += d
    a1[:, :3] += d
    a1[:, 3:] += d
    return p1, a1


@pytest.mark.gpu
def test_stream_pages_matches_fresh_scene(ctx):
    """stream a subset of pages (registered host memory, async), refit, render: equal to a scene built from the
    resulting arrays, and the downloaded arrays hold exactly the streamed pages"""
    n = 3 * gsrt.PAGE_GAUSSIANS + 1000  # a partial last page
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 5, False)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    assert sc.pages == 4
    p0, a0 = sc.download()
    p1, a1 = _jittered(p0, a0, 9, 2e-2)
    ctx.host_register(p1)
    ctx.host_register(a1)
    try:
        pages = [3, 1]
        sc.stream_pages(pages, p1, a1)
        sc.refit_bvh()
        mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
        ubo = gsrt.camera_from_modelview(mv, 60.0, 96, 64, 1.0, 4, 16)
        img, _ = sc.render(ubo, gsrt.MODE_COR)
        want_p, want_a = p0.copy(), a0.copy()
        P = gsrt.PAGE_GAUSSIANS
        for pg in pages:
            want_p[pg * P:(pg + 1) * P] = p1[pg * P:(pg + 1) * P]
            want_a[pg * P:(pg + 1) * P] = a1[pg * P:(pg + 1) * P]
        got_p, got_a = sc.download()
        assert got_p.tobytes() == want_p.tobytes() and got_a.tobytes() == want_a.tobytes()
        fresh = gsrt.Scene.from_params(ctx, want_p, want_a)
        fresh.build_bvh()
        img2, _ = fresh.render(ubo, gsrt.MODE_COR)
        assert img.tobytes() == img2.tobytes()
        want = O.render(want_p, want_a, O.make_ubo(mv, 60.0, 96, 64, 1.0, 4, 16), O.MODE_COR, bvh=O.Bvh(want_a))["rgba"]
        assert img.tobytes() == want.tobytes()
        with pytest.raises(gsrt.GsrtError):
            sc.stream_pages([4], p1, a1)
    finally:
        ctx.synchronize()
        ctx.host_unregister(p1)
        ctx.host_unregister(a1)


@pytest.mark.gpu
def test_stream_pages_pipelined_frames(ctx):
    """a dynamic scene fed from the host: every frame streams every page of one of two jitter sets (page-locked),
    refits and renders asynchronously; the last frame equals a synchronous render of its geometry"""
    n = 5 * gsrt.PAGE_GAUSSIANS
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 6, False)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    p0, a0 = sc.download()
    sets = [_jittered(p0, a0, 20 + k) for k in range(2)]
    for p, a in sets:
        ctx.host_register(p)
        ctx.host_register(a)
    try:
        import torch

        ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 80, 48, 1.0, 16, 16)
        pages = np.arange(sc.pages)
        out = torch.zeros((48, 80, 4), dtype=torch.float32, device="cuda:0")
        for f in range(7):
            p, a = sets[f & 1]
            sc.stream_pages(pages[::-1], p, a)  # any order: runs of consecutive pages are merged
            sc.refit_bvh()
            sc.render_async(ubo, gsrt.MODE_COR, d_rgba=out.data_ptr() if f == 6 else 0)
        ctx.synchronize()
        last = out.cpu().numpy()
        p, a = sets[0]  # frame 6 used set 0
        fresh = gsrt.Scene.from_params(ctx, p, a)
        fresh.build_bvh()
        want, _ = fresh.render(ubo, gsrt.MODE_COR)
        assert last.tobytes() == want.tobytes()
    finally:
        ctx.synchronize()
        for p, a in sets:
            ctx.host_unregister(p)
            ctx.host_unregister(a)


def test_double_buffered_updates_pipelined(ctx):
    """Scene updates copy into the array's second buffer on the update stream (gsrt_update_stream) while the frames
    queued before them still read the first: a pipelined sequence of updates (three device-resident jitter sets in
    turn), refits, COR frames, REF frames and a page stream between them, with no synchronisation; every frame's
    output equals that of a scene built from scratch over the geometry current when the frame was queued."""
    import torch

    n = 40000
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 17, False)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, None)
    sc.build_bvh()
    p, a = sc.download()
    rng = np.random.default_rng(23)
    sets = []
    for _ in range(3):
        d = rng.normal(0.0, 3e-3, (n, 3)).astype(np.float32)
        p1, a1 = p.copy(), a.copy()
        p1[:, :3] += d
        a1[:, :3] += d
        a1[:, 3:] += d
        sets.append((p1, a1))
    dev = [(torch.from_numpy(p1).cuda(), torch.from_numpy(a1).cuda()) for p1, a1 in sets]
    torch.cuda.synchronize()
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.05 * i, 0, 0.1 * i), (0, 0, -1)), 60.0, 128, 96, 1.0, 4, 16)
            for i in range(9)]
    # the page stream of frame 5 replaces pages 1 and 3 of set 2's arrays (current then) with set 0's
    mixed_p, mixed_a = sets[2][0].copy(), sets[2][1].copy()
    pg = gsrt.PAGE_GAUSSIANS
    for q in (1, 3):
        mixed_p[q * pg:(q + 1) * pg] = sets[0][0][q * pg:(q + 1) * pg]
        mixed_a[q * pg:(q + 1) * pg] = sets[0][1][q * pg:(q + 1) * pg]
    geo = []
    outs = [torch.zeros((96, 128, 4), dtype=torch.float32, device="cuda:0") for _ in range(9)]
    ref_rs = torch.zeros(96 * 128 * 20, dtype=torch.int32, device="cuda:0")
    for i in range(9):
        k = i % 3
        if i != 6:  # frame 6 renders set 2 + the pages again, with no update
            sc.update(dev[k][0].data_ptr(), dev[k][1].data_ptr())
        if i == 5:
            sc.stream_pages(np.array([3, 1], np.uint32), sets[0][0], sets[0][1])
        sc.refit_bvh()
        geo.append((mixed_p, mixed_a) if i in (5, 6) else sets[k])
        sc.render_async(ubos[i], gsrt.MODE_COR, d_rgba=outs[i].data_ptr())
        if i == 4:  # a REF frame between the pipelined ones (it reads the arrays on the render stream)
            sc.render_async(ubos[i], gsrt.MODE_REF, d_raystate=ref_rs.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    for i in range(9):
        fresh = gsrt.Scene.from_params(ctx, geo[i][0], geo[i][1])
        fresh.build_bvh()
        want, rs = fresh.render(ubos[i], gsrt.MODE_COR)
        assert outs[i].cpu().numpy().tobytes() == want.tobytes(), f"frame {i}"
        if i == 4:
            _, want_rs = fresh.render(ubos[i], gsrt.MODE_REF, raystate=True)
            assert ref_rs.cpu().numpy().tobytes() == want_rs.tobytes()
        fresh.close()
    pd, ad = sc.download()
    assert pd.tobytes() == sets[2][0].tobytes() and ad.tobytes() == sets[2][1].tobytes()


def test_attach_borrowed_arrays(ctx):
    """gsrt_scene_attach: frames read the caller's device arrays in place. A pipelined sequence of attaches (three
    device-resident jitter sets in turn), a copying update between them, a page stream while attached (it first copies
    the borrowed arrays into the scene, then replaces pages), refits, COR and REF frames: every frame's output equals a
    scene built from scratch over the geometry current when it was queued. After gsrt_scene_detach the scene holds its
    own copy (the caller's arrays change, frames do not); destroying a scene with attached arrays leaves them to the
    caller; host and misaligned pointers are refused."""
    import torch

    n = 40000
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 29, False)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, None)
    sc.build_bvh()
    p, a = sc.download()
    rng = np.random.default_rng(31)
    sets = []
    for _ in range(3):
        d = rng.normal(0.0, 3e-3, (n, 3)).astype(np.float32)
        p1, a1 = p.copy(), a.copy()
        p1[:, :3] += d
        a1[:, :3] += d
        a1[:, 3:] += d
        sets.append((p1, a1))
    dev = [(torch.from_numpy(p1).cuda(), torch.from_numpy(a1).cuda()) for p1, a1 in sets]
    torch.cuda.synchronize()
    with pytest.raises(gsrt.GsrtError):
        sc.attach(None, sets[0][1].ctypes.data)          # host memory
    with pytest.raises(gsrt.GsrtError):
        sc.attach(dev[0][0].data_ptr() + 4, None)        # not 16-byte aligned
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.05 * i, 0, 0.1 * i), (0, 0, -1)), 60.0, 128, 96, 1.0, 4, 16)
            for i in range(8)]
    mixed_p, mixed_a = sets[1][0].copy(), sets[1][1].copy()   # frame 6: set 1 attached, then pages 0 and 2 of set 0
    pg = gsrt.PAGE_GAUSSIANS
    for q in (0, 2):
        mixed_p[q * pg:(q + 1) * pg] = sets[0][0][q * pg:(q + 1) * pg]
        mixed_a[q * pg:(q + 1) * pg] = sets[0][1][q * pg:(q + 1) * pg]
    geo = []
    outs = [torch.zeros((96, 128, 4), dtype=torch.float32, device="cuda:0") for _ in range(8)]
    ref_rs = torch.zeros(96 * 128 * 20, dtype=torch.int32, device="cuda:0")
    for i in range(8):
        k = i % 3
        if i == 3:
            sc.update(dev[k][0].data_ptr(), dev[k][1].data_ptr())   # a copy between borrows
        else:
            sc.attach(dev[k][0].data_ptr(), dev[k][1].data_ptr())
        if i == 7:
            sc.stream_pages(np.array([2, 0], np.uint32), sets[0][0], sets[0][1])
        sc.refit_bvh()
        geo.append((mixed_p, mixed_a) if i == 7 else sets[k])
        sc.render_async(ubos[i], gsrt.MODE_COR, d_rgba=outs[i].data_ptr())
        if i == 4:
            sc.render_async(ubos[i], gsrt.MODE_REF, d_raystate=ref_rs.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    assert dev[1][0].cpu().numpy().tobytes() == sets[1][0].tobytes()   # the page stream wrote the scene's own copy
    for i in range(8):
        fresh = gsrt.Scene.from_params(ctx, geo[i][0], geo[i][1])
        fresh.build_bvh()
        want, _ = fresh.render(ubos[i], gsrt.MODE_COR)
        assert outs[i].cpu().numpy().tobytes() == want.tobytes(), f"frame {i}"
        if i == 4:
            _, want_rs = fresh.render(ubos[i], gsrt.MODE_REF, raystate=True)
            assert ref_rs.cpu().numpy().tobytes() == want_rs.tobytes()
        fresh.close()
    # detach: the scene keeps set 2 after the caller's arrays change
    sc.attach(dev[2][0].data_ptr(), dev[2][1].data_ptr())
    sc.refit_bvh()
    before, _ = sc.render(ubos[0], gsrt.MODE_COR)
    sc.detach()
    dev[2][0].add_(1.0)
    dev[2][1].add_(1.0)
    torch.cuda.synchronize()
    after, _ = sc.render(ubos[0], gsrt.MODE_COR)
    assert after.tobytes() == before.tobytes()
    pd, ad = sc.download()
    assert pd.tobytes() == sets[2][0].tobytes() and ad.tobytes() == sets[2][1].tobytes()
    # destroy while attached: the caller's arrays stay allocated and unchanged
    sc.attach(dev[0][0].data_ptr(), dev[0][1].data_ptr())
    sc.refit_bvh()
    sc.render(ubos[1], gsrt.MODE_COR)
    sc.close()
    torch.cuda.synchronize()
    assert dev[0][0].cpu().numpy().tobytes() == sets[0][0].tobytes()
    assert dev[0][1].cpu().numpy().tobytes() == sets[0][1].tobytes()
