"""GPU parity: the HIP render path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances: REF and COR are bit-exact by construction (both sides compiled with -ffp-contract=off,
IEEE-exact ops only, same op order; COR's exp is a shared IEEE-exact restatement), so the tests ask
for equality of the raw bytes. Where that is not met the north-star bound is L_inf <= 1e-3 on RGB.
"""
import os

import numpy as np
import pytest

import gsrt
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _scene(ctx, kind, n, seed=42, sh=False):
    c, r, s, o, shc = gsrt.synth_cloud(kind, n, seed, sh)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, shc)
    sc.build_bvh()
    p, a = sc.download()
    return sc, p, a, shc


def test_kat1_scene33(ctx):
    p_ref, a_ref = O.scene33()
    sc = gsrt.Scene.from_model(ctx, [[0, 0, 5], [0, 0, 3]], [[1, 0, 0, 0]] * 2, [[1, 1, 1], [2, 2, 2]], [0.9, 0.9])
    p, a = sc.download()
    assert p.tobytes() == p_ref.tobytes() and a.tobytes() == a_ref.tobytes()  # a1 on device == oracle
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.translate(0, 0, -2), 90.0, 16, 16, 2.0, 1, 16)
    rgba, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    assert not rgba.any()
    assert float(rs["trans"][8, 8]) == np.float32(0.100000024)
    assert float(rs["depth"][8, 8]) == 1.0
    mask = np.ones((16, 16), bool)
    mask[8, 8] = False
    assert (rs["trans"][mask] == 1.0).all() and (rs["depth"][mask] == 0.0).all()
    want = O.render(p_ref, a_ref, O.make_ubo(O.translate(0, 0, -2), 90.0, 16, 16, 2.0, 1, 16), O.MODE_REF,
                    want_raystate=True)["raystate"]
    assert rs.tobytes() == want.tobytes()


@pytest.mark.parametrize("n,w,h,samples,bounces", [(300, 64, 48, 1, 16), (1500, 96, 64, 2, 3), (40, 16, 16, 1, 0)])
def test_ref_needles_raystate(ctx, n, w, h, samples, bounces):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_NEEDLE, n)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, w, h, 1.0, samples, bounces)
    _, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    want = O.render(p, a, O.make_ubo(mv, 60.0, w, h, 1.0, samples, bounces), O.MODE_REF, want_raystate=True,
                    bvh=O.Bvh(a))["raystate"]
    assert (want["trans"] < 1.0).any(), "fixture must exercise the K-buffer"
    np.testing.assert_array_equal(rs["gauss_num"], want["gauss_num"])
    np.testing.assert_array_equal(rs["trans"], want["trans"])
    np.testing.assert_array_equal(rs["depth"], want["depth"])
    assert rs.tobytes() == want.tobytes()


def test_ref_camera_inside_cloud(ctx):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_REF, 10000)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 64, 1.0, 1, 16)
    _, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 64, 1.0, 1, 16), O.MODE_REF, want_raystate=True,
                    bvh=O.Bvh(a))["raystate"]
    assert rs.tobytes() == want.tobytes()


@pytest.mark.parametrize("samples", [1, 4, 3, 2, 8, 16, 32, 64])
def test_cor_cloud_rgba(ctx, samples):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_COR, 10000)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 96, 72, 1.0, samples, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 96, 72, 1.0, samples, 16), O.MODE_COR, bvh=O.Bvh(a))["rgba"]
    assert rgba[..., 3].max() > 0.5, "fixture must produce coverage"
    assert float(np.abs(rgba - want).max()) <= 1e-3
    assert rgba.tobytes() == want.tobytes()


def test_cor_sh3_rgba(ctx):
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 3000, seed=5, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 64, 1.0, 4, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 64, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a))["rgba"]
    assert float(np.abs(rgba - want).max()) <= 1e-3
    assert rgba.tobytes() == want.tobytes()


def test_cor_lut_flag(ctx):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_COR, 5000, seed=3)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 48, 1.0, 1, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_LUT)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 48, 1.0, 1, 16), O.MODE_COR | O.FLAG_LUT, bvh=O.Bvh(a))["rgba"]
    assert rgba.tobytes() == want.tobytes()


def test_stats_match_oracle(ctx):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_COR, 8000, seed=11)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 64, 1.0, 1, 16)
    sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
    st = ctx.last_stats((64, 64))
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 64, 1.0, 1, 16), O.MODE_COR, bvh=O.Bvh(a), want_stats=True)["stats"]
    np.testing.assert_array_equal(st["per_ray"][..., 0], want[..., 0])  # |C_r|
    np.testing.assert_array_equal(st["per_ray"][..., 1], want[..., 1])  # |H_r|
    np.testing.assert_array_equal(st["per_ray"][..., 3], want[..., 3])
    assert st["rays"] == 64 * 64
    assert st["candidates"] == int(want[..., 0].sum()) and st["blended"] == int(want[..., 1].sum())


# ------------------------------------------------------------------------- golden fixtures (pinned bytes)

GOLD = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["kat1_scene33.npz", "ref_needles_300.npz", "cor_10k.npz", "cor_sh3_1k.npz"])
def test_golden_fixture_bytes(ctx, name):
    g = np.load(GOLD + "/" + name, allow_pickle=False)
    ubo = g["ubo"].view(gsrt.UBO_DTYPE)
    if "params" in g.files:
        sc = gsrt.Scene.from_params(ctx, g["params"], g["aabbs"])
    else:
        sc = gsrt.Scene.from_model(ctx, g["center"], g["rot"], g["scale"], g["opacity"],
                                   g["sh"] if "sh" in g.files else None)
    sc.build_bvh()
    if "raystate" in g.files:
        rgba, rs = sc.render(ubo, gsrt.MODE_REF | gsrt.FLAG_STATS, raystate=True)
        assert rs.view(np.uint8).tobytes() == g["raystate"].tobytes()
        assert not rgba.any()
        st = ctx.last_stats(rgba.shape[:2])
        np.testing.assert_array_equal(st["per_ray"][..., [0, 2]], g["stats"][..., [0, 2]])
    else:
        rgba, _ = sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
        assert rgba.tobytes() == g["rgba"].tobytes()
        st = ctx.last_stats(rgba.shape[:2])
        np.testing.assert_array_equal(st["per_ray"][..., [0, 1, 3]], g["stats"][..., [0, 1, 3]])


# ------------------------------------------------------------------------- tile sharding (single device)

@pytest.mark.parametrize("nranks,samples", [(2, 1), (3, 4), (8, 4), (5, 3)])
def test_sharded_emulated_equals_single(ctx, nranks, samples):
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 5000, seed=21, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 75, 41, 1.0, samples, 16)
    single, _ = sc.render(ubo, gsrt.MODE_COR)
    sharded = sc.render_sharded_emulated(ubo, nranks, gsrt.MODE_COR)
    assert sharded.tobytes() == single.tobytes()


@pytest.mark.parametrize("samples", [80, 130])
def test_cor_multipass_samples(ctx, samples):
    """spp > 64 runs in passes over 8x8-pixel tiles, one pixel per lane; the framebuffer entry holds the running
    sum of the passes (no accumulator across the shading loop). Bit-exact against the oracle, also sharded."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 3000, seed=17, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 20, 12, 1.0, samples, 16)
    plan = gsrt.tile_plan(ubo, gsrt.MODE_COR)
    assert plan["spp_lanes"] == 1 and plan["tile_w"] == 8 and plan["tile_h"] == 8  # samples run as passes
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 20, 12, 1.0, samples, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a))["rgba"]
    assert rgba.tobytes() == want.tobytes()
    assert rgba[..., 3].max() > 0
    sharded = sc.render_sharded_emulated(ubo, 3, gsrt.MODE_COR)
    assert sharded.tobytes() == rgba.tobytes()


@pytest.mark.parametrize("nranks,w,h,samples", [(8, 1920, 1080, 4), (16, 1920, 1080, 4), (3, 1920, 1080, 16),
                                                (2, 3840, 2160, 1)])
def test_sharded_emulated_bands(ctx, nranks, w, h, samples):
    """Every rank's band (even, and cost-balanced from the frame's own row profile), its own tile groups only,
    gathered and unpacked, equals the single-device frame."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 20000, seed=9, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, w, h, 1.0, samples, 16)
    single, _ = sc.render(ubo, gsrt.MODE_COR)
    cost = ctx.row_costs()
    assert cost.size == gsrt.tile_plan(ubo)["tiles_y"] and cost.min() > 0
    balanced = gsrt.tile_bands(ubo, nranks, cost)
    even = gsrt.tile_bands(ubo, nranks)
    if nranks >= 8:
        assert not np.array_equal(balanced, even)  # the cloud is heavier in the middle rows
    for bands in (None, balanced):
        sharded = sc.render_sharded_emulated(ubo, nranks, gsrt.MODE_COR, bands=bands)
        assert sharded.tobytes() == single.tobytes()


@pytest.mark.parametrize("project_all", ["0", "1"])
def test_sharded_rank_culling(ctx, monkeypatch, project_all):
    """A rank of a sharded frame with whole super-tile runs keeps only the splats whose footprint meets one of its
    super-tiles (the rest get depth +inf; a cheap view-space box test skips the projection of most of them), and
    its frontier kernel skips super-groups it does not own. GSRT_DEBUG_PROJECT_ALL=1 keeps everything; both give
    the single-device frame, byte for byte."""
    monkeypatch.setenv("GSRT_DEBUG_PROJECT_ALL", project_all)
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 30000, seed=13, sh=True)
    mv = gsrt.lookat((0.2, -0.1, 0.5), (0, 0, -1))
    for w, h, spp, n in [(1920, 1080, 4, 8), (1920, 1080, 1, 3), (2560, 1440, 4, 5)]:
        ubo = gsrt.camera_from_modelview(mv, 60.0, w, h, 1.0, spp, 16)
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        bands = gsrt.tile_bands(ubo, n, ctx.row_costs())
        assert sc.render_sharded_emulated(ubo, n, gsrt.MODE_COR, bands=bands).tobytes() == single.tobytes()


def test_sharded_moving_camera_keyed_bitmaps(ctx):
    """k_project writes the +inf keys of a splat outside a rank's tiles only when the frame slot may hold finite
    ones (its keyed bitmap). Emulated 8- and 5-rank frames of a moving camera (every rank's share in turn, the
    frame slots alternating, so each slot sees other ranks' ownership from frame to frame), with a REF frame and a
    counting pass (unbooked writes of slot 0) and a rebuild in between: each equals the single-device frame."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 40000, seed=19, sh=True)
    ref_ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, -8), (0, 0, -9)), 60.0, 32, 16, 1.0, 1, 16)
    for i in range(7):
        mv = gsrt.lookat((0.3 * i - 0.9, 0.1 * i, 0.2 * i), (0.05 * i, 0.0, -1.0))
        ubo = gsrt.camera_from_modelview(mv, 60.0, 1920, 1080, 1.0, 1 if i % 2 else 4, 16)
        n = 8 if i < 4 else 5
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        bands = gsrt.tile_bands(ubo, n, ctx.row_costs())  # the partition moves with the camera
        assert sc.render_sharded_emulated(ubo, n, gsrt.MODE_COR, bands=bands).tobytes() == single.tobytes(), f"frame {i}"
        if i == 2:
            sc.render(ref_ubo, gsrt.MODE_REF, raystate=True)
            sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
        if i == 4:
            sc.build_bvh()


@pytest.mark.parametrize("w,h,spp,n,r", [(1920, 1080, 4, 8, 0), (1920, 1080, 4, 8, 5), (640, 360, 1, 3, 0),
                                         (640, 360, 1, 3, 2)])
def test_packed_share_matches_host_pack(monkeypatch, w, h, spp, n, r):
    """Rank r's share of an n-rank frame through the sharded path on a loopback communicator (GSRT_DEBUG_RANK_OF=n:r):
    the packed block it gathers equals the library's host mirror of the packed layout (gsrt_tile_pack_host) applied
    to the single-device frame, so the layout the CPU gloo test (tests/test_distributed.py) exchanges is the one the
    GPU produces. As the root (r = 0) the emulation also lands the other ranks' (zero) blocks and unpacks all n: the
    framebuffer is the single frame on rank 0's tiles and zero elsewhere (tile_unpack of the same blocks)."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 23, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, sh)
        sc.build_bvh()
        ubo = gsrt.camera_from_modelview(gsrt.lookat((0.1, 0.0, 0.3), (0, 0, -1)), 60.0, w, h, 1.0, spp, 16)
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        pl = gsrt.tile_plan(ubo, gsrt.MODE_COR, n, r)
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", f"{n}:{r}" if r else str(n))
        cx.comm_init_loopback()
        for bands in (None, gsrt.tile_bands(ubo, n, cx.row_costs())):  # even, then pinned cost-balanced bands
            if bands is not None:
                cx.set_bands(n, bands)
            want = gsrt.tile_pack(ubo, single, n, r, bands=bands).reshape(-1)
            fb = sc.render_sharded(ubo, gsrt.MODE_COR)
            used = cx.last_bands()
            assert np.array_equal(used, gsrt.tile_bands(ubo, n) if bands is None else bands)
            m = pl["tiles_x"] * int(used[r + 1] - used[r]) * pl["tile_w"] * pl["tile_h"] * 4
            assert cx.debug_gathered(m).tobytes() == want[:m].tobytes()
            if r == 0:
                blocks = np.zeros((n, want.size), np.float32)
                blocks[0] = want
                assert fb.tobytes() == gsrt.tile_unpack(ubo, blocks.reshape(-1), n, bands=bands).tobytes()


@pytest.mark.parametrize("n", [8, 3])
def test_band_restricted_refit_shares(monkeypatch, n):
    """After a refit a rank share fits only what its band can see (FitBand: the 256-leaf chunks no tile of the band can
    see get empty boxes, the crossings are counted as a climb would). Per frame: a new jitter of every centre (update +
    refit from host arrays), a moving camera, the single-device frame (its slot refitted in full again), then every
    rank's share through the exchange path (loopback, GSRT_DEBUG_RANK_OF=n:r, pinned cost bands): each gathered block
    equals the host pack of that frame's single-device image."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 60000, 47, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, sh)
        sc.build_bvh()
        p0, a0 = sc.download()
        rng = np.random.default_rng(5)
        cx.comm_init_loopback()
        for i in range(4):
            d = rng.normal(0.0, 2e-3, (p0.shape[0], 3)).astype(np.float32)
            p1, a1 = p0.copy(), a0.copy()
            p1[:, :3] += d
            a1[:, :3] += d
            a1[:, 3:] += d
            sc.update(p1, a1)
            sc.refit_bvh()
            u = gsrt.camera_from_modelview(gsrt.lookat((0.03 * i, 0.02 * i, 0.1 * i), (0.01 * i, 0, -1)), 60.0, 640, 360,
                                           1.0, 4, 16)
            monkeypatch.delenv("GSRT_DEBUG_RANK_OF", raising=False)
            single, _ = sc.render(u, gsrt.MODE_COR)
            bands = gsrt.tile_bands(u, n, cx.row_costs())
            cx.set_bands(n, bands)
            pl = gsrt.tile_plan(u, gsrt.MODE_COR, n, 0)
            for r in range(n):
                monkeypatch.setenv("GSRT_DEBUG_RANK_OF", f"{n}:{r}")
                sc.render_sharded(u, gsrt.MODE_COR, want_image=False)
                m = pl["tiles_x"] * int(bands[r + 1] - bands[r]) * pl["tile_w"] * pl["tile_h"] * 4
                want = gsrt.tile_pack(u, single, n, r, bands=bands).reshape(-1)
                assert cx.debug_gathered(m).tobytes() == want[:m].tobytes(), f"frame {i} rank {r}"


def test_depth_cull_guard(ctx):
    """The traversals' depth cull bounds a subtree's keys by its box (depth_lo), which holds while every centre lies in
    its AABB. A caller's AABBs that miss their centres (shifted away from the camera) set the scene's guard word in the
    projection and turn the cull off: the frame still equals the oracle's, and equals the same scene's frame with
    AABBs that contain the centres. (The cull runs where tile groups overflow: 16 or more samples per pixel here.)"""
    c, rr, s_, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, 100000, 53, False)
    base = gsrt.Scene.from_model(ctx, c, rr, s_, o, None)
    p, a = base.download()
    base.close()
    a2 = a.copy()
    a2[:, 2] -= 0.4  # z: away from a camera looking down -z, the boxes stay in front of it
    a2[:, 5] -= 0.4
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 48, 1.0, 16, 16)  # thousands of candidates per group: lists overflow
    for aa in (a, a2):
        sc = gsrt.Scene.from_params(ctx, p, aa)
        sc.build_bvh()
        img, _ = sc.render(ubo, gsrt.MODE_COR)
        want = O.render(p, aa, O.make_ubo(mv, 60.0, 64, 48, 1.0, 16, 16), O.MODE_COR, bvh=O.Bvh(aa), threads=16)["rgba"]
        assert img[..., 3].mean() > 0.5
        assert img.tobytes() == want.tobytes()
        sc.close()


def test_sharded_auto_balancing_moving_camera(monkeypatch):
    """The automatic partition on a loopback communicator (GSRT_DEBUG_RANK_OF=8:3, rank 3's share): every 8th frame the
    render kernel records its rows' costs, the profile all-reduce (one rank here) returns them with the partition hash,
    and 8 frames later the bands are recut from them (here from rank 3's rows alone, so they keep moving). Over a moving
    camera every frame's bands are a partition of the tile rows and its gathered block equals the host pack of the
    single-device frame under the bands that frame used."""
    n, r = 8, 3
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 29, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, sh)
        sc.build_bvh()
        ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.02 * i, -0.01 * i, 0.05 * i), (0.01 * i, 0, -1)), 60.0, 320,
                                           192, 1.0, 4, 16) for i in range(34)]
        singles = [sc.render(u, gsrt.MODE_COR)[0] for u in ubos]
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", f"{n}:{r}")
        cx.comm_init_loopback()
        seen = set()
        for i, u in enumerate(ubos):
            sc.render_sharded(u, gsrt.MODE_COR, want_image=False)
            used = cx.last_bands()
            pl = gsrt.tile_plan(u, gsrt.MODE_COR, n, r)
            assert used.size == n + 1 and used[0] == 0 and used[-1] == pl["tiles_y"] and np.all(np.diff(used) >= 1)
            seen.add(tuple(int(v) for v in used))
            m = pl["tiles_x"] * int(used[r + 1] - used[r]) * pl["tile_w"] * pl["tile_h"] * 4
            want = gsrt.tile_pack(u, singles[i], n, r, bands=used).reshape(-1)
            assert cx.debug_gathered(m).tobytes() == want[:m].tobytes(), f"frame {i}"
        assert len(seen) >= 2  # even, then recut from the first profile (frame 8)


def _dump8_want(single):
    codes, esc = gsrt.dump8_encode(single)
    return codes, esc


def _ppm_bytes(tmp_path, codes=None, esc=None, rgba=None):
    path = tmp_path / "x.ppm"
    if rgba is not None:
        gsrt.dump_ppm(str(path), rgba)
    else:
        gsrt.dump8_ppm(str(path), codes, esc)
    return path.read_bytes()


@pytest.mark.parametrize("nranks,w,h,samples", [(8, 75, 41, 4), (3, 20, 12, 80), (5, 640, 360, 1), (8, 1920, 1080, 4)])
def test_dump8_sharded_emulated(ctx, tmp_path, nranks, w, h, samples):
    """GSRT_FLAG_OUT_DUMP8: every rank's band rendered straight to dump code words + its escape list, gathered and unpacked by the rank-0 kernel: the codes and escapes are those of the
    single-device RGBA32F frame, and its PPM is byte-identical. spp > 64 sums its passes in the scratch buffer. The SH
    coefficients are scaled by 20 so that some pixels pass 1022/255 (escapes; colours are clamped at 0 below)."""
    c, r, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 5000, 21, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s_, o, 20.0 * sh)
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, w, h, 1.0, samples, 16)
    single, _ = sc.render(ubo, gsrt.MODE_COR)
    codes, esc = sc.render_sharded_emulated_dump8(ubo, nranks, bands=gsrt.tile_bands(ubo, nranks, ctx.row_costs()))
    wc, we = _dump8_want(single)
    assert codes.tobytes() == wc.tobytes() and esc.tobytes() == we.tobytes()
    assert _ppm_bytes(tmp_path, codes, esc) == _ppm_bytes(tmp_path, rgba=single)
    if w * h > 10000:
        assert 0 < esc.size < w * h // 64  # the fixture exercises the escape list


def test_dump8_sharded_exchange_path(tmp_path):
    """The real exchange path (loopback communicator: render into the packed block, ncclGather, unpack on the comm
    stream) with dump8 frames interleaved with RGBA32F frames in the same two packed buffers (the escape count is
    re-zeroed where the layout moves), a multi-pass frame, and an escape list that overflows: gsrt_dump8_read
    returns the single frame's codes and escapes, and the overflow fails with GSRT_E_STATE without poisoning the
    next frame."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 31, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, 20.0 * sh)  # ~100 escapes per 640x360 frame
        sc.build_bvh()
        neg = gsrt.Scene.from_model(cx, c, rr, s_, o, 80.0 * sh)  # half the pixels escape: the list overflows
        neg.build_bvh()
        frames = [(640, 360, 4, "d8"), (640, 360, 4, "d8"), (320, 200, 1, "rgba"), (640, 360, 4, "d8"),
                  (24, 16, 80, "d8"), (640, 360, 4, "rgba"), (640, 360, 1, "d8"), (640, 360, 4, "neg"),
                  (640, 360, 4, "d8")]
        ubos = {}
        for w, h, spp, _ in frames:
            ubos[(w, h, spp)] = gsrt.camera_from_modelview(gsrt.lookat((0.1, 0, 0.2), (0, 0, -1)), 60.0, w, h, 1.0, spp, 16)
        singles = {k: sc.render(u, gsrt.MODE_COR)[0] for k, u in ubos.items()}
        cx.comm_init_loopback()
        for i, (w, h, spp, kind) in enumerate(frames):
            u = ubos[(w, h, spp)]
            if kind == "rgba":
                assert sc.render_sharded(u, gsrt.MODE_COR).tobytes() == singles[(w, h, spp)].tobytes(), f"frame {i}"
                continue
            scene = neg if kind == "neg" else sc
            assert scene.render_sharded(u, gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8) is None
            if kind == "neg":
                with pytest.raises(gsrt.GsrtError) as e:
                    cx.dump8_read(w, h)
                assert e.value.status == gsrt.E_STATE
                continue
            codes, esc = cx.dump8_read(w, h)
            wc, we = _dump8_want(singles[(w, h, spp)])
            assert codes.tobytes() == wc.tobytes() and esc.tobytes() == we.tobytes(), f"frame {i}"
        assert _ppm_bytes(tmp_path, codes, esc) == _ppm_bytes(tmp_path, rgba=singles[(640, 360, 4)])
        with pytest.raises(gsrt.GsrtError):  # the image of a dump8 frame is read with dump8_read
            lib_out = np.zeros((360, 640, 4), np.float32)
            gsrt._check(gsrt.lib.gsrt_render_sharded(sc.handle, gsrt._p(u), gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8, 0,
                                                     gsrt._p(lib_out)), cx)


@pytest.mark.parametrize("n", [8, 3])
def test_dump8_root_share(monkeypatch, n):
    """Rank 0's share of an n-rank dump8 frame through the exchange path (GSRT_DEBUG_RANK_OF=n): its block lands in the
    gather buffer beside the other ranks' stand-in blocks (zeros: no escapes), and k_unpack_dump8 places them by the
    bands: on rank 0's rows the codes and escapes are the single-device frame's, elsewhere code 0. A rank other than
    0 has no frame to read."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 37, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, 20.0 * sh)
        sc.build_bvh()
        ubo = gsrt.camera_from_modelview(gsrt.lookat((0.1, 0.0, 0.3), (0, 0, -1)), 60.0, 640, 360, 1.0, 4, 16)
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        wc, we = gsrt.dump8_encode(single)
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", str(n))
        cx.comm_init_loopback()
        bands = gsrt.tile_bands(ubo, n, cx.row_costs(), gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8)
        cx.set_bands(n, bands)
        for _ in range(3):  # both packed / gather buffers
            sc.render_sharded(ubo, gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8)
        codes, esc = cx.dump8_read(640, 360)
        th = gsrt.tile_plan(ubo)["tile_h"]
        y1 = min(360, int(bands[1]) * th)
        assert np.array_equal(codes[:y1], wc[:y1]) and not codes[y1:].any()
        assert esc.tobytes() == we[we["pixel"] < y1 * 640].tobytes()
        # the block the kernel wrote is the host mirror's (gsrt_tile_pack_dump8_host) word for word on the rank's
        # tiles; its escape list holds the same entries in arrival order
        L = gsrt.dump8_layout(ubo, n, bands)
        dev = cx.debug_gathered(L["block"] * n).view(np.uint32).reshape(n, L["block"])
        host = gsrt.tile_pack_dump8(ubo, single, n, 0, bands=bands)
        used = int(bands[1]) * gsrt.tile_plan(ubo)["tiles_x"] * gsrt.tile_plan(ubo)["tile_w"] * th
        assert np.array_equal(dev[0, :used], host[:used]) and not dev[1:].any()
        ne = int(host[L["codes"]])
        assert ne == esc.size and int(dev[0, L["codes"]]) == ne
        de = dev[0, L["codes"] + 4:L["codes"] + 4 + 4 * ne].reshape(ne, 4)
        he = host[L["codes"] + 4:L["codes"] + 4 + 4 * ne].reshape(ne, 4)
        assert np.array_equal(de[np.argsort(de[:, 0])], he)
        hc, hesc = gsrt.tile_unpack_dump8(ubo, dev, n, bands=bands)  # the host unpack of the device blocks
        assert np.array_equal(hc, codes) and hesc.tobytes() == esc.tobytes()
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", f"{n}:1")
        sc.render_sharded(ubo, gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8)
        with pytest.raises(gsrt.GsrtError) as e:
            cx.dump8_read(640, 360)
        assert e.value.status == gsrt.E_STATE


def test_share_cost_profile_hook(monkeypatch):
    """gsrt_debug_share_costs / gsrt_debug_row_profile: a rank share's own row costs (its profile frames' measurement)
    are positive on the rows of its band and zero elsewhere."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 41, True)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, sh)
        sc.build_bvh()
        ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 640, 360, 1.0, 4, 16)
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", "4:2")
        cx.comm_init_loopback()
        cx.debug_share_costs(True)
        for _ in range(3):
            sc.render_sharded_async(ubo, gsrt.MODE_COR)
        rows = cx.debug_row_profile()
        b = cx.last_bands()
        assert rows.size == gsrt.tile_plan(ubo)["tiles_y"]
        assert np.all(rows[b[2]:b[3]] > 0) and not rows[:b[2]].any() and not rows[b[3]:].any()


def test_comm_rank_cap_and_dump8_framebuffer():
    """A communicator of more ranks than a partition holds (64) is refused (GSRT_E_ARG) instead of sharing rank 0's
    band; after a dump8 sharded frame gsrt_framebuffer is NULL (no RGBA32F image) until the next RGBA32F frame."""
    c, rr, s_, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 3000, 43, False)
    with gsrt.Context(0) as cx:
        uid = gsrt.comm_unique_id()
        for n in (65, 1000):
            with pytest.raises(gsrt.GsrtError) as e:
                cx.comm_init(uid, n, 0)
            assert e.value.status == gsrt.E_ARG
        sc = gsrt.Scene.from_model(cx, c, rr, s_, o, None)
        sc.build_bvh()
        ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 64, 48, 1.0, 4, 16)
        cx.comm_init_loopback()
        sc.render_sharded(ubo, gsrt.MODE_COR)
        assert gsrt.lib.gsrt_framebuffer(cx.handle)
        assert sc.render_sharded(ubo, gsrt.MODE_COR | gsrt.FLAG_OUT_DUMP8) is None
        assert not gsrt.lib.gsrt_framebuffer(cx.handle)
        single, _ = sc.render(ubo, gsrt.MODE_COR)
        assert gsrt.lib.gsrt_framebuffer(cx.handle)
        assert sc.render_sharded(ubo, gsrt.MODE_COR).tobytes() == single.tobytes()


def test_sharded_single_rank_comm(ctx):
    sc, p, a, _ = _scene(ctx, gsrt.SYNTH_COR, 3000, seed=2)
    ctx.comm_init(gsrt.comm_unique_id(), 1, 0)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 40, 24, 1.0, 1, 16)
    single, _ = sc.render(ubo, gsrt.MODE_COR)
    assert sc.render_sharded(ubo, gsrt.MODE_COR).tobytes() == single.tobytes()


def test_large_frame_matches_oracle(ctx):
    """A whole 512x512 frame at 4 spp (16384 tiles, 64 super-tiles, 1024 tile groups, full XCD rounds): every
    pixel equals the oracle's (SH-3, COR), and a second frame is the same."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 20000, seed=5, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 512, 512, 1.0, 4, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    want = O.render(p, a, O.make_ubo(mv, 60.0, 512, 512, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a),
                    threads=16)["rgba"]
    assert rgba[..., 3].mean() > 0.05
    assert rgba.tobytes() == want.tobytes()
    again, _ = sc.render(ubo, gsrt.MODE_COR)
    assert again.tobytes() == rgba.tobytes()


# ------------------------------------------------------------------------- edge cases

def test_empty_scene(ctx):
    sc = gsrt.Scene.from_params(ctx, np.zeros((0, 12), np.float32), np.zeros((0, 6), np.float32))
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 20, 10, 1.0, 1, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    assert not rgba.any()
    _, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    assert (rs["trans"] == 1.0).all() and (rs["gauss_num"] == 0).all()


def test_single_gaussian_and_ragged_frame(ctx):
    sc = gsrt.Scene.from_model(ctx, [[0.1, -0.2, -5.0]], [[1, 0, 0, 0]], [[0.3, 0.2, 0.1]], [0.8])
    sc.build_bvh()
    p, a = sc.download()
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    for w, h, s in [(37, 29, 1), (13, 7, 4), (5, 3, 2)]:
        ubo = gsrt.camera_from_modelview(mv, 60.0, w, h, 1.0, s, 16)
        rgba, _ = sc.render(ubo, gsrt.MODE_COR)
        want = O.render(p, a, O.make_ubo(mv, 60.0, w, h, 1.0, s, 16), O.MODE_COR)["rgba"]
        assert rgba.tobytes() == want.tobytes()
        assert rgba[..., 3].max() > 0


@pytest.mark.parametrize("opacity_scale", [0.05, 0.3])
def test_cor_tile_overflow_rounds(ctx, opacity_scale):
    """Far more candidates per tile than the tile buffer holds (CAP): the tile re-traverses for the next
    nearest CAP keys beyond the last one, and the result is unchanged. Checked with the counting pass
    (every AABB candidate kept) and with the production path (footprint cull before truncation)."""
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 4)
    s = s * 12.0                                   # big splats: thousands of candidates per tile
    o = o * opacity_scale                          # faint, so few rays terminate early
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    p, a = sc.download()
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 24, 16, 1.0, 1, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
    st = ctx.last_stats()
    assert st["max_tile_candidates"] > 256 and st["tile_rounds"] > st["tiles"]
    want = O.render(p, a, O.make_ubo(mv, 60.0, 24, 16, 1.0, 1, 16), O.MODE_COR, bvh=O.Bvh(a))["rgba"]
    assert rgba.tobytes() == want.tobytes()
    culled, _ = sc.render(ubo, gsrt.MODE_COR)
    assert culled.tobytes() == want.tobytes()


@pytest.mark.parametrize("stack_limit", [None, "48"])
def test_traversal_stack_restart(ctx, monkeypatch, stack_limit):
    """A tile whose frustum holds ~all of a large cloud drives the LDS node stack of the 64-wide
    traversal to its limit: the pop width throttles, and when no room is left the tile restarts with a
    one-node-per-step DFS (stack <= tree depth). GSRT_DEBUG_STACK_LIMIT lowers the limit so the restart
    is taken for certain; the image is unchanged either way."""
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_COR, 100000, 8)
    o = o * 0.02
    sc = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc.build_bvh()
    assert sc.bvh_info()["max_depth"] < 46
    p, a = sc.download()
    mv = gsrt.lookat((0, 0, 60.0), (0, 0, -8.0))   # far away: the whole cloud inside a few tiles
    ubo = gsrt.camera_from_modelview(mv, 20.0, 16, 16, 1.0, 1, 16)
    if stack_limit:
        monkeypatch.setenv("GSRT_DEBUG_STACK_LIMIT", stack_limit)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
    st = ctx.last_stats()
    want = O.render(p, a, O.make_ubo(mv, 20.0, 16, 16, 1.0, 1, 16), O.MODE_COR, bvh=O.Bvh(a))["rgba"]
    assert rgba.tobytes() == want.tobytes()
    if stack_limit:
        assert st["restarts"] > 0


# ------------------------------------------------------------------------- bench scale (size-independent properties)

@pytest.fixture(scope="module")
def c3(ctx):
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 1_000_000, 42, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 1920, 1080, 1.0, 4, 16)
    return sc, ubo, sh, mv


def test_c3_deterministic_and_bounded(ctx, c3):
    sc, ubo, _, _ = c3
    a, _ = sc.render(ubo, gsrt.MODE_COR)
    b, _ = sc.render(ubo, gsrt.MODE_COR)
    assert a.tobytes() == b.tobytes()
    assert np.isfinite(a).all() and (a >= 0).all() and (a[..., 3] <= 1).all()
    assert a[..., 3].mean() > 0.5


def test_c3_full_frame_matches_oracle(ctx, c3):
    """configs[2], the headline workload (1M SH-3, 1920x1080, 4 spp): every pixel equals the oracle's (~6 s of CPU
    on 16 threads)."""
    from bench import cpu_threads

    sc, ubo, sh, mv = c3
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    p, a = sc.download()
    want = O.render(p, a, O.make_ubo(mv, 60.0, 1920, 1080, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a),
                    threads=cpu_threads(16))["rgba"]
    assert rgba[..., 3].mean() > 0.5
    assert rgba.tobytes() == want.tobytes()


def test_cli_scene33_matches_reference_dump(tmp_path):
    """bin/gsrt_render with the reference's flags renders scene 33 (KAT-1) and dumps the reference PPM:
    an all-black 16x16 image, "  0   0   0" per pixel."""
    import subprocess
    cli = os.path.join(ROOT, "3dgs-raytrace_amd", "bin", "gsrt_render")
    out = tmp_path / "scene33.ppm"
    p = subprocess.run([cli, "--scene", "33", "--shader-type", "6", "--width", "16", "--height", "16",
                        "--samples", "1", "--bounces", "16", "--out", str(out), "--binary", str(tmp_path / "image.binary")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert out.read_bytes() == b"P3\n16 16\n255\n" + b"  0   0   0\n" * 256
    rec = np.fromfile(tmp_path / "image.binary", dtype=np.dtype([("rgb", "<f4", 3), ("off", "<u4")]))
    assert len(rec) == 256 and not rec["rgb"].any()


def test_cli_cor_cloud_matches_library(ctx, tmp_path):
    """The CLI's synthetic COR scene renders the same pixels as the library called directly."""
    import subprocess
    cli = os.path.join(ROOT, "3dgs-raytrace_amd", "bin", "gsrt_render")
    out = tmp_path / "cor.ppm"
    p = subprocess.run([cli, "--scene", "100", "--gaussians", "3000", "--sh", "--width", "48", "--height", "32",
                        "--samples", "2", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 3000, 42, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 48, 32, 1.0, 2, 16)
    rgba, _ = sc.render(ubo, gsrt.MODE_COR)
    ref = tmp_path / "lib.ppm"
    gsrt.dump_ppm(str(ref), rgba)
    assert out.read_bytes() == ref.read_bytes()


@pytest.mark.parametrize("eye,spp", [((0.0, 0.0, 0.0), 4), ((0.3, -0.2, -6.0), 1), ((0.0, 0.0, 40.0), 2)])
def test_group_lists_match_tile_traversal(ctx, monkeypatch, eye, spp):
    """Tiles take their candidates from their tile group's sorted list (k_group_list), filtered by their own
    footprint test; traversing per tile (GSRT_DEBUG_NO_GROUPS=1) gives the same image, and both equal the
    oracle. Cameras outside, inside and far from the cloud (group lists that overflow kGCap)."""
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 60000, 21, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    mv = gsrt.lookat(eye, (0.0, 0.0, -8.0))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 200, 120, 1.0, spp, 16)
    img, _ = sc.render(ubo, gsrt.MODE_COR)
    monkeypatch.setenv("GSRT_DEBUG_NO_FRONTIER", "1")        # groups traverse from the root
    nofront, _ = sc.render(ubo, gsrt.MODE_COR)
    assert img.tobytes() == nofront.tobytes()
    monkeypatch.setenv("GSRT_DEBUG_NO_GROUPS", "1")
    root, _ = sc.render(ubo, gsrt.MODE_COR)
    assert img.tobytes() == root.tobytes()
    p, a = sc.download()
    want = O.render(p, a, O.make_ubo(mv, 60.0, 200, 120, 1.0, spp, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a),
                    rows=(40, 72))["rgba"]
    assert img[40:72].tobytes() == want[40:72].tobytes()


# ------------------------------------------------------------------------- pipelined frames (two frame slots)

@pytest.mark.parametrize("n", [4, 8])
def test_pipelined_rank_shares_match_sync(monkeypatch, n, slot_knob):
    """Back-to-back frames of a small rank share (rank 0 of n, GSRT_DEBUG_RANK_OF=n) through the sharded path on a
    loopback communicator, on the slot streams (GSRT_SLOT_STREAMS): prep and render kernels of frame f on its slot's
    stream, frames f and f+1 overlapping, each rendering into one of two alternating packed buffers, then the gather,
    the other blocks' arrival and k_unpack on the comm stream. Every frame's framebuffer (copied out on the comm
    stream while later frames are queued) must equal its synchronous render on rank 0's tiles (zero elsewhere), also
    across a scene update + refit between frames and a counting pass in between."""
    import ctypes

    import torch

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 13, True)
    W, H = 256, 128
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.04 * i, -0.02 * i, 0.1 * i), (0.02 * i, 0, -1)), 60.0, W, H,
                                       1.0, 4, 16) for i in range(8)]
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, r, s, o, sh)
        sc.build_bvh()
        p, a = sc.download()
        d = np.random.default_rng(6).normal(0.0, 2e-2, (len(p), 3)).astype(np.float32)
        p1, a1 = p.copy(), a.copy()
        p1[:, :3] += d
        a1[:, :3] += d
        a1[:, 3:] += d

        def rank0_view(u, img):  # the single frame on rank 0's tiles, zero on the others'
            blk = gsrt.tile_pack(u, img, n, 0).reshape(-1)
            blocks = np.zeros((n, blk.size), np.float32)
            blocks[0] = blk
            return gsrt.tile_unpack(u, blocks.reshape(-1), n).tobytes()

        want = [rank0_view(u, sc.render(u, gsrt.MODE_COR)[0]) for u in ubos[:4]]
        sc2 = gsrt.Scene.from_params(cx, p1, a1, sh)
        sc2.build_bvh()
        want += [rank0_view(u, sc2.render(u, gsrt.MODE_COR)[0]) for u in ubos[4:]]
        sc2.close()
        monkeypatch.setenv("GSRT_DEBUG_RANK_OF", str(n))
        cx.comm_init_loopback()
        out = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in ubos]
        for i, u in enumerate(ubos):
            if i == 4:
                sc.update(p1, a1)
                sc.refit_bvh()
            sc.render_sharded_async(u, gsrt.MODE_COR)
            assert hip.hipMemcpyAsync(out[i].data_ptr(), cx.framebuffer_ptr, W * H * 16, 3, cx.comm_stream) == 0
            if i == 5:  # a counting pass (serialized on the render stream) between two pipelined frames
                sc.render_async(u, gsrt.MODE_COR | gsrt.FLAG_STATS)
        cx.synchronize()
        torch.cuda.synchronize()
        for i, (o_, w_) in enumerate(zip(out, want)):
            assert o_.cpu().numpy().tobytes() == w_, f"frame {i} differs from its synchronous render"


@pytest.fixture(params=["adaptive", "0", "1", "two_slots"])
def slot_knob(request, monkeypatch):
    """the slot-stream choice (GSRT_SLOT_STREAMS): measured per frame, or forced off / on (GSRT_DEBUG_SLOT_STREAMS);
    two_slots: two frame slots in rotation instead of three (GSRT_DEBUG_SLOTS=2)"""
    if request.param == "two_slots":
        monkeypatch.setenv("GSRT_DEBUG_SLOTS", "2")
    elif request.param != "adaptive":
        monkeypatch.setenv("GSRT_DEBUG_SLOT_STREAMS", request.param)
    return request.param


def test_pipelined_frames_match_sync(ctx, slot_knob):
    """Back-to-back render_async frames: frame f+1's prep kernels (projection, frontier, group lists) run on
    the prep stream while frame f's render kernel runs, in rotating frame slots. Every frame must equal
    its synchronous render, also across a scene update + refit between frames (the prep stage waits for it)
    and with REF / counting-pass renders interleaved (those run serialized in slot 0)."""
    _pipelined_frames(ctx)


@pytest.mark.parametrize("slots", ["0", "1"])
def test_prep_priority_switches(ctx, monkeypatch, slots):
    """The prep streams' priority class switches at every frame (GSRT_DEBUG_PREP_PRIORITY=2; in production it follows the
    sampled render kernel time): each switch orders the new stream pair after the old one, so the pipelined frames,
    the update + refit between them and the interleaved REF / counting renders still equal their synchronous
    renders."""
    monkeypatch.setenv("GSRT_DEBUG_PREP_PRIORITY", "2")
    monkeypatch.setenv("GSRT_DEBUG_SLOT_STREAMS", slots)
    _pipelined_frames(ctx)


def _pipelined_frames(ctx):
    import torch

    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 11, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    p, a = sc.download()
    d = np.random.default_rng(5).normal(0.0, 2e-2, (len(p), 3)).astype(np.float32)
    p1, a1 = p.copy(), a.copy()
    p1[:, :3] += d
    a1[:, :3] += d
    a1[:, 3:] += d
    W, H = 96, 64
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.05 * i, -0.03 * i, 0.1 * i), (0.02 * i, 0, -1)), 60.0, W, H,
                                       1.0, 4, 16) for i in range(8)]
    want = [sc.render(u, gsrt.MODE_COR)[0] for u in ubos[:4]]
    sc2 = gsrt.Scene.from_params(ctx, p1, a1, sh)
    sc2.build_bvh()
    want += [sc2.render(u, gsrt.MODE_COR)[0] for u in ubos[4:]]
    sc2.close()
    ref_ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, -8), (0, 0, -9)), 60.0, 32, 16, 1.0, 1, 16)
    want_ref = sc.render(ref_ubo, gsrt.MODE_REF, raystate=True)[1]

    out = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in ubos]
    for i in range(4):
        sc.render_async(ubos[i], gsrt.MODE_COR, d_rgba=out[i].data_ptr())
        if i == 1:  # a serialized REF frame between two pipelined ones
            _, rs = sc.render(ref_ubo, gsrt.MODE_REF, raystate=True)
            assert rs.tobytes() == want_ref.tobytes()
    sc.update(p1, a1)
    sc.refit_bvh()
    for i in range(4, 8):
        sc.render_async(ubos[i], gsrt.MODE_COR, d_rgba=out[i].data_ptr())
        if i == 5:  # and a counting pass
            sc.render_async(ubos[i], gsrt.MODE_COR | gsrt.FLAG_STATS)
    ctx.synchronize()
    torch.cuda.synchronize()
    for i, (o_, w_) in enumerate(zip(out, want)):
        assert o_.cpu().numpy().tobytes() == w_.tobytes(), f"frame {i} differs from its synchronous render"


def test_pipelined_moving_camera(ctx, slot_knob):
    """Twelve back-to-back frames of a moving camera over a 200k cloud (prep of frame f+1 beside the render of
    frame f, two frame slots, the frontier on its own stream), each equal to its synchronous render; a refit
    between frames (same boxes) puts the slot's fit into the prep chain."""
    import torch

    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 200000, 17, True)
    sc = gsrt.Scene.from_model(ctx, c, r, s, o, sh)
    sc.build_bvh()
    W, H = 640, 360
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.04 * i, -0.02 * i, 0.05 * i), (0.03 * i, 0.01 * i, -1)), 60.0,
                                       W, H, 1.0, 4, 16) for i in range(12)]
    want = [sc.render(u, gsrt.MODE_COR)[0] for u in ubos]
    out = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in ubos]
    for i, u in enumerate(ubos):
        if i == 8:
            sc.refit_bvh()
        sc.render_async(u, gsrt.MODE_COR, d_rgba=out[i].data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    for i, (o_, w_) in enumerate(zip(out, want)):
        assert o_.cpu().numpy().tobytes() == w_.tobytes(), f"frame {i} differs from its synchronous render"


@pytest.mark.parametrize("spp", [1, 4])
def test_group_size_2x2_equals_4x4(ctx, monkeypatch, spp):
    """Tile groups of 2x2 tiles (chosen below 1500 groups of 4x4 per rank) and of 4x4 tiles give the same frame: the group only
    decides which candidates the per-tile lists are filtered from, never a per-ray result."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 20000, seed=33, sh=True)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 160, 96, 1.0, spp, 16)
    monkeypatch.setenv("GSRT_DEBUG_GROUP_TILES", "4")
    four, _ = sc.render(ubo, gsrt.MODE_COR)
    monkeypatch.setenv("GSRT_DEBUG_GROUP_TILES", "2")
    two, _ = sc.render(ubo, gsrt.MODE_COR)
    assert two.tobytes() == four.tobytes()
    want = O.render(p, a, O.make_ubo(mv, 60.0, 160, 96, 1.0, spp, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a),
                    rows=(40, 48))["rgba"]
    assert two[40:48].tobytes() == want[40:48].tobytes()


@pytest.mark.parametrize("loopback", ["0", "1"])
@pytest.mark.parametrize("slots", ["0", "1"])
def test_sharded_async_choreography(monkeypatch, loopback, slots):
    """gsrt_render_sharded_async frames back to back on a one-rank communicator. With GSRT_DEBUG_COMM_LOOPBACK=1
    every frame takes the exchange path of gsrt_comm.cpp: render into packed[p] once gathered[p] says the gather two
    frames back has sent it, rendered[p] -> ncclGather -> k_unpack on the comm stream. Without it the frame renders
    straight into the framebuffer. Each frame's image, copied out on the stream that finishes it (gsrt_comm_stream)
    while later frames are already queued, equals its synchronous render, across a scene update + refit. The RCCL
    transport between GPUs itself is left to the driver's multi-GPU run."""
    import ctypes

    import torch

    monkeypatch.setenv("GSRT_DEBUG_COMM_LOOPBACK", loopback)
    monkeypatch.setenv("GSRT_DEBUG_SLOT_STREAMS", slots)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 13, True)
    W, H = 256, 128
    ubos = [gsrt.camera_from_modelview(gsrt.lookat((0.04 * i, -0.02 * i, 0.1 * i), (0.02 * i, 0, -1)), 60.0, W, H,
                                       1.0, 4, 16) for i in range(8)]
    with gsrt.Context(0) as cx:  # its own ctx: the communicator lives and dies with it
        cx.comm_init(gsrt.comm_unique_id(), 1, 0)
        assert (cx.comm_stream != 0) == (loopback == "1")
        sc = gsrt.Scene.from_model(cx, c, r, s, o, sh)
        sc.build_bvh()
        p, a = sc.download()
        d = np.random.default_rng(6).normal(0.0, 2e-2, (len(p), 3)).astype(np.float32)
        p1, a1 = p.copy(), a.copy()
        p1[:, :3] += d
        a1[:, :3] += d
        a1[:, 3:] += d
        want = [sc.render(u, gsrt.MODE_COR)[0] for u in ubos[:4]]
        sc2 = gsrt.Scene.from_params(cx, p1, a1, sh)
        sc2.build_bvh()
        want += [sc2.render(u, gsrt.MODE_COR)[0] for u in ubos[4:]]
        sc2.close()
        out = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in ubos]
        for i, u in enumerate(ubos):
            if i == 4:
                sc.update(p1, a1)
                sc.refit_bvh()
            sc.render_sharded_async(u, gsrt.MODE_COR)
            done = cx.comm_stream or cx.stream  # the stream that finishes the frame's image
            assert hip.hipMemcpyAsync(out[i].data_ptr(), cx.framebuffer_ptr, W * H * 16, 3, done) == 0
        cx.synchronize()
        torch.cuda.synchronize()
        for i, (o_, w_) in enumerate(zip(out, want)):
            assert o_.cpu().numpy().tobytes() == w_.tobytes(), f"frame {i} differs from its synchronous render"
        sc.close()


def test_bench_sharded_frame_check(monkeypatch):
    """bench.py's N-rank line carries sharded_frame_check: the last sharded frame against rank 0 rendering the whole
    frame alone. Run here on a one-rank loopback communicator (the exchange path without the transport), after
    pipelined sharded frames, as the bench does after its timed region."""
    import bench

    monkeypatch.setenv("GSRT_DEBUG_COMM_LOOPBACK", "1")
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 21, True)
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 320, 192, 1.0, 4, 16)
    with gsrt.Context(0) as cx:
        cx.comm_init(gsrt.comm_unique_id(), 1, 0)
        sc = gsrt.Scene.from_model(cx, c, r, s, o, sh)
        sc.build_bvh()
        for out in (0, gsrt.FLAG_OUT_DUMP8):  # the RGBA32F and the dump8 exchange format
            for _ in range(5):
                sc.render_sharded_async(ubo, gsrt.MODE_COR | out)
            res = bench.sharded_frame_check(sc, ubo, gsrt.MODE_COR | out, 0)
            assert res["bit_exact"], res
            assert res["ppm_identical"] if out else res["linf"] == 0.0, res
        sc.close()


def test_timing_kernel_only():
    """gsrt_timing records the render kernel and the whole frame per timed frame; with gsrt_timing_kernel_only only
    the kernel's two events (frame times read 0). The events carry no system-scope fence (kTimingEventFlags)."""
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, 20000, 5, True)
    ubo = gsrt.camera_from_modelview(gsrt.lookat((0, 0, 0), (0, 0, -1)), 60.0, 256, 128, 1.0, 4, 16)
    with gsrt.Context(0) as cx:
        sc = gsrt.Scene.from_model(cx, c, r, s, o, sh)
        sc.build_bvh()
        for kernel_only in (False, True):
            cx.timing(6, kernel_only=kernel_only)
            for _ in range(8):  # two frames past the cap: not recorded
                sc.render_async(ubo, gsrt.MODE_COR)
            cx.synchronize()
            k, f = cx.timing_read()
            cx.timing(0)
            assert len(k) == 6 and (k > 0).all(), k
            if kernel_only:
                assert (f == 0).all(), f
            else:
                assert (f >= k * 0.99).all(), (k, f)
        # gsrt_timing_stride: events on frames 0, 4, 8 of the 10 rendered (bench.py's sampled kernel_ms), the recorded
        # kernel times those of whole frames alone
        cx.timing(5, kernel_only=True, stride=4)
        for _ in range(10):
            sc.render_async(ubo, gsrt.MODE_COR)
        cx.synchronize()
        k, _ = cx.timing_read()
        cx.timing(0)
        assert len(k) == 3 and (k > 0).all(), k
        cx.timing(4, kernel_only=True)  # the stride goes back to 1 with the next call
        for _ in range(4):
            sc.render_async(ubo, gsrt.MODE_COR)
        cx.synchronize()
        k, _ = cx.timing_read()
        cx.timing(0)
        assert len(k) == 4 and (k > 0).all(), k
        sc.close()


def test_leaf_footprint_boxes(ctx, monkeypatch):
    """COR frames put each leaf's footprint box into its node slot (leaf_fp: the traversals test it instead of the
    leaf AABB and skip the footprint cull). The image equals the AABB-tested traversal's (GSRT_DEBUG_NO_LEAF_FP=1)
    and the oracle's; a REF frame and a counting pass that follow on the same slot get the AABBs back (the slot is
    refitted first) and equal the oracle; a BVH download shows AABB unions again."""
    sc, p, a, sh = _scene(ctx, gsrt.SYNTH_COR, 30000, seed=5, sh=True)
    mv = gsrt.lookat((0.1, -0.05, 0.2), (0.0, 0.0, -6.0))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 160, 96, 1.0, 4, 16)
    img, _ = sc.render(ubo, gsrt.MODE_COR)
    monkeypatch.setenv("GSRT_DEBUG_NO_LEAF_FP", "1")
    aabb_img, _ = sc.render(ubo, gsrt.MODE_COR)
    monkeypatch.delenv("GSRT_DEBUG_NO_LEAF_FP")
    assert img.tobytes() == aabb_img.tobytes()
    want = O.render(p, a, O.make_ubo(mv, 60.0, 160, 96, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a),
                    rows=(30, 50))["rgba"]
    assert img[30:50].tobytes() == want[30:50].tobytes()
    # REF after COR frames (camera inside the cloud so that REF's +z depths exist)
    sc.render(ubo, gsrt.MODE_COR)
    mv_in = gsrt.lookat((0.0, 0.0, -8.0), (0.0, 0.0, -9.0))
    ubo_in = gsrt.camera_from_modelview(mv_in, 60.0, 40, 24, 1.0, 1, 4)
    _, rs = sc.render(ubo_in, gsrt.MODE_REF, raystate=True)
    ref = O.render(p, a, O.make_ubo(mv_in, 60.0, 40, 24, 1.0, 1, 4), O.MODE_REF, bvh=O.Bvh(a), want_raystate=True)
    assert rs.tobytes() == ref["raystate"].tobytes()
    # a counting pass after a COR frame: |C_r| per ray is the AABB candidate count
    sc.render(ubo, gsrt.MODE_COR)
    sc.render(ubo, gsrt.MODE_COR | gsrt.FLAG_STATS)
    st = ctx.last_stats(per_ray_shape=(96, 160))
    cnt = O.render(p, a, O.make_ubo(mv, 60.0, 160, 96, 1.0, 4, 16), O.MODE_COR, sh=sh, bvh=O.Bvh(a), rows=(40, 44),
                   want_stats=True)["stats"]
    np.testing.assert_array_equal(st["per_ray"][40:44, :, 0], cnt[40:44, :, 0])
    # the downloaded BVH: every internal box is the union of its children's (leaf AABBs restored)
    sc.render(ubo, gsrt.MODE_COR)
    nodes, leaf_gid, _ = sc.bvh_download()
    f = nodes.view(np.float32)
    for i in range(0, len(nodes), 997):
        for ref, lo, hi in ((nodes[i, 3], f[i, 0:3], f[i, 4:7]), (nodes[i, 7], f[i, 8:11], f[i, 12:15])):
            if ref & 0x80000000:
                g = ref & 0x7FFFFFFF
                np.testing.assert_array_equal(lo, a[g, :3])
                np.testing.assert_array_equal(hi, a[g, 3:])
