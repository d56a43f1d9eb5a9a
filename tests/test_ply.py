"""3DGS .ply ingestion (gsrt_ply_info / gsrt_ply_read / gsrt_scene_from_ply) and the dump_image.sh text
dump. CPU-only except the last test. The files are written here with numpy in the 3DGS layout."""
import os

import numpy as np
import pytest

import gsrt

REST = 45  # SH degree 3: 15 coefficients per channel beyond DC


def _props(n_rest=REST, normals=True):
    names = ["x", "y", "z"] + (["nx", "ny", "nz"] if normals else []) + ["f_dc_0", "f_dc_1", "f_dc_2"]
    names += [f"f_rest_{i}" for i in range(n_rest)] + ["opacity", "scale_0", "scale_1", "scale_2"]
    return names + ["rot_0", "rot_1", "rot_2", "rot_3"]


def _random_rows(n, names, seed=0):
    rng = np.random.default_rng(seed)
    rows = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    for k in ("scale_0", "scale_1", "scale_2"):
        rows[k] = rng.uniform(-6, -3, n).astype(np.float32)
    return rows


def _write_binary(path, rows, names, endian="<", ftype="f4"):
    dt = np.dtype([(k, endian + ftype) for k in names])
    n = len(rows[names[0]])
    arr = np.zeros(n, dt)
    for k in names:
        arr[k] = rows[k]
    fmt = "binary_little_endian" if endian == "<" else "binary_big_endian"
    pt = "float" if ftype == "f4" else "double"
    head = f"ply\nformat {fmt} 1.0\nelement vertex {n}\n" + "".join(f"property {pt} {k}\n" for k in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(head.encode())
        f.write(arr.tobytes())


def _expected(rows, n_rest):
    c = np.stack([rows["x"], rows["y"], rows["z"]], 1)
    s = np.exp(np.stack([rows[f"scale_{k}"] for k in range(3)], 1).astype(np.float32))
    q = np.stack([rows[f"rot_{k}"] for k in range(4)], 1).astype(np.float32)
    q = q / np.sqrt((q * q).sum(1, keepdims=True))
    o = 1.0 / (1.0 + np.exp(-rows["opacity"].astype(np.float32)))
    sh = np.zeros((len(o), 16, 3), np.float32)
    per = n_rest // 3
    for ch in range(3):
        sh[:, 0, ch] = rows[f"f_dc_{ch}"]
        for j in range(min(per, 15)):
            sh[:, 1 + j, ch] = rows[f"f_rest_{ch * per + j}"]
    return c, q, s, o, sh.reshape(-1, 48)


@pytest.mark.parametrize("endian,ftype", [("<", "f4"), (">", "f4"), ("<", "f8")])
def test_binary_ply_conversion(tmp_path, endian, ftype):
    names = _props()
    rows = _random_rows(257, names, seed=3)
    path = tmp_path / "scene.ply"
    _write_binary(path, rows, names, endian, ftype)
    info = gsrt.ply_info(path)
    assert info == {"n": 257, "sh_degree": 3}
    got = gsrt.ply_read(path)
    want = _expected(rows, REST)
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=2e-6, atol=1e-7)
    np.testing.assert_array_equal(got[0], want[0])      # positions exact
    np.testing.assert_array_equal(got[4], want[4])      # SH reordered, exact


def test_ascii_ply_degree0(tmp_path):
    names = _props(n_rest=0, normals=False)
    rows = _random_rows(9, names, seed=5)
    path = tmp_path / "a.ply"
    with open(path, "w") as f:
        f.write("ply\nformat ascii 1.0\ncomment written by test_ply\nelement vertex 9\n")
        f.write("".join(f"property float {k}\n" for k in names) + "end_header\n")
        for i in range(9):
            f.write(" ".join(repr(float(rows[k][i])) for k in names) + "\n")
    assert gsrt.ply_info(path) == {"n": 9, "sh_degree": 0}
    c, r, s, o, sh = gsrt.ply_read(path)
    wc, wr, ws, wo, wsh = _expected(rows, 0)
    np.testing.assert_allclose(s, ws, rtol=2e-6)
    np.testing.assert_allclose(o, wo, rtol=2e-6)
    np.testing.assert_array_equal(sh, wsh)
    assert not sh[:, 3:].any()


def test_ply_errors(tmp_path):
    with pytest.raises(gsrt.GsrtError) as e:
        gsrt.ply_info(tmp_path / "missing.ply")
    assert e.value.status == gsrt.E_IO
    bad = tmp_path / "bad.ply"
    bad.write_bytes(b"not a ply\n")
    with pytest.raises(gsrt.GsrtError) as e:
        gsrt.ply_info(bad)
    assert e.value.status == gsrt.E_ARG
    names = [k for k in _props() if k != "rot_3"]           # a required property missing
    p = tmp_path / "norot.ply"
    _write_binary(p, _random_rows(4, names), names)
    with pytest.raises(gsrt.GsrtError):
        gsrt.ply_info(p)
    names = _props()
    p = tmp_path / "trunc.ply"
    _write_binary(p, _random_rows(50, names), names)
    data = p.read_bytes()
    p.write_bytes(data[:-100])                               # truncated body
    with pytest.raises(gsrt.GsrtError) as e:
        gsrt.ply_read(p)
    assert e.value.status == gsrt.E_IO


def test_dump_rgba_text(tmp_path):
    rgba = np.zeros((2, 3, 4), np.float32)
    rgba[1, 2] = (0.25, 0.5, 1.0, 1.0)
    rgba[0, 1] = (1e-7, 0.0, 0.75, 0.0)
    path = tmp_path / "image.txt"
    gsrt.dump_rgba_text(path, rgba)
    lines = path.read_text().splitlines()
    assert len(lines) == 6
    assert lines[0] == "[0, 0] rgba(0.000000, 0.000000, 0.000000)"
    assert lines[1] == "[1, 0] rgba(0.000000, 0.000000, 0.750000)"
    assert lines[5] == "[2, 1] rgba(0.250000, 0.500000, 1.000000)"


@pytest.mark.gpu
def test_scene_from_ply_renders_like_from_model(ctx, tmp_path):
    import oracle as O
    n = 4000
    c, r, s, o, sh = gsrt.synth_cloud(gsrt.SYNTH_COR, n, 17, True)
    names = _props()
    rows = {"x": c[:, 0], "y": c[:, 1], "z": c[:, 2], "nx": 0 * o, "ny": 0 * o, "nz": 0 * o,
            "opacity": np.log(o / (1 - o)).astype(np.float32)}
    for k in range(3):
        rows[f"scale_{k}"] = np.log(s[:, k]).astype(np.float32)
        rows[f"f_dc_{k}"] = sh.reshape(n, 16, 3)[:, 0, k]
        for j in range(15):
            rows[f"f_rest_{k * 15 + j}"] = sh.reshape(n, 16, 3)[:, 1 + j, k]
    for k in range(4):
        rows[f"rot_{k}"] = r[:, k]
    path = tmp_path / "cloud.ply"
    _write_binary(path, rows, names)
    sc = gsrt.Scene.from_ply(ctx, path)
    sc.build_bvh()
    pc, pr, ps, po, psh = gsrt.ply_read(path)
    ref = gsrt.Scene.from_model(ctx, pc, pr, ps, po, psh)
    ref.build_bvh()
    mv = gsrt.lookat((0, 0, 0), (0, 0, -1))
    ubo = gsrt.camera_from_modelview(mv, 60.0, 64, 48, 1.0, 4, 16)
    img, _ = sc.render(ubo, gsrt.MODE_COR)
    img2, _ = ref.render(ubo, gsrt.MODE_COR)
    assert img.tobytes() == img2.tobytes() and img[..., 3].max() > 0.1
    p, a = sc.download()
    want = O.render(p, a, O.make_ubo(mv, 60.0, 64, 48, 1.0, 4, 16), O.MODE_COR, sh=psh, bvh=O.Bvh(a))["rgba"]
    assert img.tobytes() == want.tobytes()
