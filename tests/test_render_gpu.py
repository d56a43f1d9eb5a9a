"""GPU parity: the HIP render path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances: REF and COR are bit-exact by construction (both sides compiled with -ffp-contract=off,
IEEE-exact ops only, same op order; COR's exp is a shared IEEE-exact restatement), so the tests ask
for equality of the raw bytes. Where that is not met the north-star bound is L_inf <= 1e-3 on RGB.
"""
import numpy as np
import pytest

import gsrt
import oracle as O

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


@pytest.mark.parametrize("samples", [1, 4, 3])
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
