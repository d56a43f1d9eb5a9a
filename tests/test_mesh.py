"""Triangle meshes co-traced with the Gaussians in REF mode.

Reference behaviour restated (include/gsrt.h "triangle meshes", oracle/gsrt_oracle.c closest_triangle):
scene 33's sphere is a triangle BLAS (SceneList.cpp:123, Model::CreateSphere); a triangle hit sets the
traversal's min_thit (vulkan_ray_tracing.cc:925-931), culls Gaussian boxes entered beyond it (:806-807), bounds
the Gaussian report rule (instructions.cc:7050), and a round whose closest hit is the triangle runs
RayTracing.rchit, whose Scatter() zeroes the payload's Trans (Scatter.glsl).

KAT-3 (hand-derived, like KAT-1): camera at the origin looking down -z (fovy 90, 16x16, B=16), one Gaussian
mu=(0,0,1), scale 1, opacity 0.9 -- its AABB [-3,3]^2 x [-2,4] holds the camera, view z = +1, V = diag(64, 64)
so only pixel (8,8) passes g <= 5.6 (g = 0 there, alpha = 0.9) -- and a sphere of radius 0.5 on the -z axis
(centre offset (0.03, 0.02) so the central ray meets no mesh vertex or edge):
  far sphere (centre z = -3, t_tri ~ 2.5 > depth 1): round 0 inserts (1, 0.9) and the report (1 < 2.5) is
      accepted -> Trans = 1 - 0.9f = 0.100000024, Depth = 1; round 1: the Gaussian is depth-culled (1 <= 1), the
      triangle is the closest hit -> Trans = 0; GaussNum = 0 ends the rounds. K[0] = {10000, 0.9} (alpha stale).
  near sphere (centre z = -1.2, t_tri ~ 0.7 < depth 1): the insert happens every round but the report is refused
      (1 < 0.7 fails), the triangle stays the closest hit -> Trans = 0, Depth = 0, GaussNum = 1, K[0] = {1, 0.9}.
Pixels that see only the sphere end with Trans = 0; pixels that see neither keep Trans = 1.
"""
import numpy as np
import pytest

import oracle as O

F32_TRANS = np.float32(1.0) - np.float32(0.9)  # 0.100000024


def _kat3(cz):
    p, a = O.gauss_from_model([[0, 0, 1]], [[1, 0, 0, 0]], [[1, 1, 1]], [0.9])
    v, i = O.sphere_mesh((0.03, 0.02, cz), 0.5)
    return p, a, v, i


def _kat3_ubo():
    return O.make_ubo(O.translate(0, 0, 0), 90.0, 16, 16, 1.0, 1, 16)


def _check_kat3(rs, cz):
    c = rs[8, 8]
    if cz == -3.0:
        assert float(c["trans"]) == 0.0 and float(c["depth"]) == 1.0 and int(c["gauss_num"]) == 0
        assert c["k"][0].tolist() == [10000.0, np.float32(0.9)]
    else:
        assert float(c["trans"]) == 0.0 and float(c["depth"]) == 0.0
        assert int(c["gauss_num"]) == 1 and int(c["gauss_num_raw"]) == 1
        assert c["k"][0].tolist() == [1.0, np.float32(0.9)]
    assert float(rs["trans"][0, 0]) == 1.0 and float(rs["trans"][15, 15]) == 1.0  # corners miss everything
    assert float(rs["trans"][8, 7]) == 0.0  # a neighbour sees only the sphere (g > 5.6 for the Gaussian)
    assert set(np.unique(rs["trans"]).tolist()) == {0.0, 1.0}


def test_kat3_trans_value_is_one_minus_alpha():
    assert F32_TRANS == np.float32(0.100000024)


@pytest.mark.parametrize("cz", [-3.0, -1.2])
def test_kat3_oracle(cz):
    p, a, v, i = _kat3(cz)
    rs = O.render(p, a, _kat3_ubo(), O.MODE_REF, want_raystate=True, tris=O.mesh_triangles(v, i))["raystate"]
    _check_kat3(rs, cz)
    # without the mesh the same pixel keeps the Gaussian's transmittance (KAT-1's answer)
    rs0 = O.render(p, a, _kat3_ubo(), O.MODE_REF, want_raystate=True)["raystate"]
    assert float(rs0["trans"][8, 8]) == F32_TRANS and float(rs0["depth"][8, 8]) == 1.0


def test_sphere_mesh_geometry():
    v, i = O.sphere_mesh((200.0, 200.0, 0.0), 0.5)
    assert v.shape == (561, 3) and i.shape == (1024, 3) and int(i.max()) == 560
    r = np.linalg.norm(v.astype(np.float64) - [200.0, 200.0, 0.0], axis=1)
    assert np.abs(r - 0.5).max() < 3e-5  # fp32 ulp at 200 is 1.5e-5
    # poles on the y axis (Model.cpp:581-595: y = cy + r cos(j0))
    assert np.allclose(v[0], [200.0, 200.5, 0.0], atol=3e-5)
    assert np.allclose(v[-1], [200.0, 199.5, 0.0], atol=3e-5)
    # the reference's winding: first quad (0, 33, 34), (0, 34, 1)
    assert i[0].tolist() == [0, 33, 34] and i[1].tolist() == [0, 34, 1]


def test_sphere_mesh_product_equals_oracle():
    import gsrt

    for c, r in (((200.0, 200.0, 0.0), 0.5), ((0.03, 0.02, -3.0), 0.5), ((-1.5, 2.25, 7.0), 3.0)):
        v, i = gsrt.sphere_mesh(c, r)
        vo, io = O.sphere_mesh(c, r)
        assert v.tobytes() == vo.tobytes() and i.tobytes() == io.tobytes()


def test_oracle_rejects_cor_with_mesh():
    p, a, v, i = _kat3(-3.0)
    with pytest.raises(ValueError):
        O.render(p, a, _kat3_ubo(), O.MODE_COR, tris=O.mesh_triangles(v, i))


# ---------------------------------------------------------------------------------------------- GPU


def _scene_with_mesh(ctx, center, rot, scale, opacity, meshes):
    import gsrt

    sc = gsrt.Scene.from_model(ctx, center, rot, scale, opacity)
    for v, i in meshes:
        sc.add_mesh(v, i)
    sc.build_bvh()
    p, a = sc.download()
    tris = np.concatenate([O.mesh_triangles(v, i) for v, i in meshes]) if meshes else None
    return sc, p, a, tris


@pytest.mark.gpu
@pytest.mark.parametrize("cz", [-3.0, -1.2])
def test_kat3_gpu(ctx, cz):
    import gsrt

    p, a, v, i = _kat3(cz)
    sc, p2, a2, tris = _scene_with_mesh(ctx, [[0, 0, 1]], [[1, 0, 0, 0]], [[1, 1, 1]], [0.9], [(v, i)])
    assert sc.mesh_triangles == 1024
    ubo = gsrt.camera_from_modelview(gsrt.translate(0, 0, 0), 90.0, 16, 16, 1.0, 1, 16)
    rgba, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    assert not rgba.any()
    _check_kat3(rs, cz)
    want = O.render(p2, a2, _kat3_ubo(), O.MODE_REF, want_raystate=True, tris=tris)["raystate"]
    assert rs.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("eye,center", [
    ((200.0, 200.0, 3.0), (200.0, 200.0, 0.0)),   # looking at the sphere from +z
    ((4.0, 4.0, 2.0), (200.0, 200.0, 0.0)),       # from inside G2's box towards the sphere
    ((199.0, 199.2, 1.0), (200.0, 200.0, 0.0)),   # close up, the sphere fills most of the frame
])
def test_scene33_sphere_cameras(ctx, eye, center):
    """SceneList::GaussSplat with its triangle sphere, cameras that see the sphere: raystate == oracle."""
    import gsrt

    v, i = gsrt.sphere_mesh((200.0, 200.0, 0.0), 0.5)
    sc, p, a, tris = _scene_with_mesh(ctx, [[0, 0, 5], [0, 0, 3]], [[1, 0, 0, 0]] * 2, [[1, 1, 1], [2, 2, 2]],
                                      [0.9, 0.9], [(v, i)])
    mv = gsrt.lookat(eye, center)
    ubo = gsrt.camera_from_modelview(mv, 90.0, 64, 48, 2.0, 1, 16)
    _, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    want = O.render(p, a, O.make_ubo(mv, 90.0, 64, 48, 2.0, 1, 16), O.MODE_REF, want_raystate=True,
                    tris=tris)["raystate"]
    assert (want["trans"] == 0.0).any(), "the camera must see the sphere"
    assert rs.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_needles_with_meshes(ctx, seed):
    """REF needle cloud (every AABB holds the camera) with several spheres and a random triangle soup inside it:
    triangle cull, report rule and Trans = 0 on many rays at once, multi-sample, bit-exact vs the oracle."""
    import gsrt

    rng = np.random.default_rng(seed)
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_NEEDLE, 400, 40 + seed, False)
    meshes = [gsrt.sphere_mesh(tuple(rng.uniform(-2, 2, 3) + (0, 0, -3)), float(rng.uniform(0.2, 1.0)))
              for _ in range(3)]
    nv = 60
    soup_v = rng.uniform(-3, 3, (nv, 3)).astype(np.float32)
    soup_v[:, 2] -= 4.0
    soup_i = rng.integers(0, nv, (30, 3)).astype(np.uint32)
    meshes.append((soup_v, soup_i))
    sc, p, a, tris = _scene_with_mesh(ctx, c, r, s, o, meshes)
    assert sc.mesh_triangles == 3 * 1024 + 30
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    for spp, bounces in ((1, 16), (2, 3)):
        ubo = gsrt.camera_from_modelview(mv, 60.0, 96, 64, 1.0, spp, bounces)
        _, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
        want = O.render(p, a, O.make_ubo(mv, 60.0, 96, 64, 1.0, spp, bounces), O.MODE_REF, want_raystate=True,
                        bvh=O.Bvh(a), tris=tris)["raystate"]
        t = want["trans"]
        # rays zeroed by a triangle after Gaussian reports, rays that blended and missed the mesh, rays that miss all
        assert ((t == 0.0) & (want["depth"] > 0)).any() and ((t > 0) & (t < 1)).any() and (t == 1).any()
        np.testing.assert_array_equal(rs["trans"], want["trans"])
        assert rs.tobytes() == want.tobytes()
    # the mesh changes the frame: without it the same rays keep transmittance
    sc0 = gsrt.Scene.from_model(ctx, c, r, s, o)
    sc0.build_bvh()
    ubo = gsrt.camera_from_modelview(mv, 60.0, 96, 64, 1.0, 1, 16)
    _, rs0 = sc0.render(ubo, gsrt.MODE_REF, raystate=True)
    assert (rs0["trans"] > 0).sum() > (rs["trans"] > 0).sum()


@pytest.mark.gpu
def test_mesh_sharded_emulated_and_cor_refused(ctx):
    import gsrt

    v, i = gsrt.sphere_mesh((0.03, 0.02, -3.0), 0.5)
    sc, p, a, tris = _scene_with_mesh(ctx, [[0, 0, 1]], [[1, 0, 0, 0]], [[1, 1, 1]], [0.9], [(v, i)])
    ubo = gsrt.camera_from_modelview(gsrt.translate(0, 0, 0), 90.0, 40, 24, 1.0, 1, 16)
    img, rs = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    for nr in (2, 3):
        assert sc.render_sharded_emulated(ubo, nr, gsrt.MODE_REF).tobytes() == img.tobytes()
    with pytest.raises(gsrt.GsrtError) as e:
        sc.render(ubo, gsrt.MODE_COR)
    assert e.value.status == gsrt.E_ARG
    # the frame after a refused call still renders
    _, rs2 = sc.render(ubo, gsrt.MODE_REF, raystate=True)
    assert rs2.tobytes() == rs.tobytes()


@pytest.mark.gpu
def test_vs_stats_ref(ctx, tmp_path):
    """vulkan-sim's rt_* statistics of a REF frame (gsrt_vs_stats): per ray the candidates, rounds and
    triangle-hit traversals equal the oracle's (BVH-independent); the node counts are the LBVH's own, checked
    for consistency (a traversal visits at least the root and every candidate leaf)"""
    import gsrt

    rng = np.random.default_rng(3)
    c, r, s, o, _ = gsrt.synth_cloud(gsrt.SYNTH_NEEDLE, 600, 44, False)
    meshes = [gsrt.sphere_mesh(tuple(rng.uniform(-2, 2, 3) + (0, 0, -3)), 0.8) for _ in range(2)]
    sc, p, a, tris = _scene_with_mesh(ctx, c, r, s, o, meshes)
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 48, 1.0, 2, 4)
    sc.render(ubo, gsrt.MODE_REF | gsrt.FLAG_STATS)
    per = ctx.last_stats(per_ray_shape=(48, 64))["per_ray"]
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 48, 1.0, 2, 4), O.MODE_REF, want_stats=True, tris=tris)["stats"]
    np.testing.assert_array_equal(per[..., 0], want[..., 0])  # candidates
    np.testing.assert_array_equal(per[..., 2], want[..., 2])  # rounds (traversals)
    np.testing.assert_array_equal(per[..., 1], want[..., 1])  # traversals with a triangle hit
    assert (want[..., 1] > 0).any() and (want[..., 1] == 0).any()
    assert (per[..., 3].astype(np.int64) >= per[..., 0].astype(np.int64) + 1).all()
    vs = ctx.vs_stats()
    rounds = per[..., 2].astype(np.int64)
    assert vs["rt_n_total_rays"] == int(rounds.sum())
    assert vs["rt_num_hits"] == int(per[..., 1].astype(np.int64).sum())
    assert vs["rt_tot_nodes_per_ray"] == int((per[..., 3].astype(np.int64) * rounds).sum())
    assert vs["rt_max_nodes_per_ray"] == int(per[..., 3].max())
    assert 2 <= vs["rt_max_tree_depth"] <= sc.bvh_info()["max_depth"] and vs["overflowed_walks"] == 0
    path = tmp_path / "vs_stats.txt"
    ctx.dump_vs_stats(str(path))
    lines = dict(l.split(" = ") for l in path.read_text().strip().split("\n"))
    assert int(lines["rt_n_total_rays"]) == vs["rt_n_total_rays"] and int(lines["rt_num_hits"]) == vs["rt_num_hits"]
    assert abs(float(lines["rt_avg_nodes_per_ray"]) - vs["rt_tot_nodes_per_ray"] / vs["rt_n_total_rays"]) < 1e-3
