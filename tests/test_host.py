"""Host-side checks that need no GPU: the C-ABI library loads and exports every declared symbol, the
host logic behind the boundary (camera / UBO, synthetic clouds, frame dumps, tile plan) agrees with
the oracle or the reference's formats, and the product refuses to run without a device."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

import gsrt
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _declared_functions(header=None):
    names = [header] if header else ["gsrt.h", "gsrt_test.h"]
    found = set()
    for h in names:
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        found |= set(re.findall(r"\b(gsrt_[a-z0-9_]+)\s*\(", text))
    return sorted(found)


def test_drop_in_header_holds_no_test_hooks():
    """gsrt.h is the surface a reference-side caller links: the debug counters, host mirrors of the
    sharded layout, emulated gathers, synthetic clouds and the partition-rule hooks live in gsrt_test.h only"""
    abi, hooks = set(_declared_functions("gsrt.h")), set(_declared_functions("gsrt_test.h"))
    assert not abi & hooks
    for f in abi:
        assert not re.search(r"debug|_host$|emulated|synth|partition_hash|decide_bands", f), f
    assert {"gsrt_debug_counters", "gsrt_tile_pack_host", "gsrt_render_sharded_emulated", "gsrt_synth_cloud",
            "gsrt_decide_bands"} <= hooks
    assert "GSRT_DEBUG_" not in open(os.path.join(ROOT, "include", "gsrt.h")).read()


def test_library_exports_every_declared_symbol():
    declared = _declared_functions()
    assert len(declared) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", gsrt.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\s[TW]\s+(gsrt_\w+)$", out, flags=re.M))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(declared) == sorted(gsrt.EXPORTS)
    assert gsrt.lib.gsrt_abi_version() == 2


def test_status_strings():
    for code in (0, -1, -2, -3, -4, -5, -6):
        assert gsrt.lib.gsrt_status_string(code)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU may be present")
def test_no_device_fails_loudly():
    with pytest.raises(gsrt.GsrtError) as e:
        gsrt.Context(0)
    assert e.value.status == gsrt.E_DEVICE


@pytest.mark.parametrize("mv,fov,w,h,f,s,b", [
    ("kat1", 90.0, 16, 16, 2.0, 1, 16),
    ("lookat", 60.0, 1920, 1080, 1.0, 4, 16),
    ("oblique", 45.0, 640, 360, 3.5, 16, 3),
])
def test_camera_matches_oracle(mv, fov, w, h, f, s, b):
    m = {"kat1": O.translate(0, 0, -2), "lookat": O.lookat((0, 0, 0), (0, 0, -1)),
         "oblique": O.lookat((1.5, -2.0, 7.0), (0.2, 0.4, -3.0))}[mv]
    a = O.make_ubo(m, fov, w, h, f, s, b)
    c = gsrt.camera_from_modelview(m, fov, w, h, f, s, b)
    assert a.tobytes() == c.tobytes()


def test_camera_file(tmp_path):
    with open(os.path.join(GOLD, "cameras.json")) as fh:
        cams = json.load(fh)
    for name, d in cams.items():
        p = tmp_path / os.path.basename(name)
        p.write_text(d["text"])
        ubo = gsrt.camera_from_file(str(p), 60.0, 1280, 720, 1.0, 8, 16)
        assert ubo.tobytes().hex() == d["ubo_hex"], name
    with pytest.raises(gsrt.GsrtError):
        gsrt.camera_from_file(str(tmp_path / "missing.camera"), 60.0, 16, 16)


@pytest.mark.parametrize("kind", [gsrt.SYNTH_COR, gsrt.SYNTH_REF, gsrt.SYNTH_NEEDLE])
def test_synth_matches_oracle(kind):
    x = O.synth_cloud(kind, 2000, 42, True)
    y = gsrt.synth_cloud(kind, 2000, 42, True)
    for p, q in zip(x, y):
        assert p.tobytes() == q.tobytes()


def test_ppm_matches_reference_format(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.random((5, 7, 4), dtype=np.float32)
    img[0, 0, :3] = (0.0, 0.5, 1.0)
    path = tmp_path / "f.ppm"
    gsrt.dump_ppm(str(path), img)
    data = path.read_bytes().decode()
    # the reference prints the fp32 products v*255 (vulkan_ray_tracing.cc:2240-2241)
    want = "P3\n7 5\n255\n" + "".join("%3.0f %3.0f %3.0f\n" % tuple(float(np.float32(v) * np.float32(255)) for v in px[:3])
                                       for px in img.reshape(-1, 4))
    assert data == want
    assert data.splitlines()[3] == "  0 128 255"


def test_ppm_overflow_spills_like_fseek(tmp_path):
    img = np.zeros((1, 3, 4), np.float32)
    img[0, 0, 0] = -1.0   # "-255" is 4 characters: spills into pixel 1's slot, which then overwrites it
    path = tmp_path / "o.ppm"
    gsrt.dump_ppm(str(path), img)
    body = path.read_bytes().decode().split("255\n", 1)[1]
    # pixel 0 writes 13 bytes at slot 0; pixel 1's write at byte 12 replaces the spilled newline
    assert body == "-255   0   0" + "  0   0   0\n" + "  0   0   0\n"


def _dump8_frame():
    """a frame with every class of value the dump prints: in range, exact halves (round to even), 999.5 / 1000+
    (a 4-character field that spills), 1022 / 1023 (the code limit), negatives, -0, NaN and infinities"""
    rng = np.random.default_rng(11)
    img = rng.uniform(0.0, 1.0, (37, 53, 4)).astype(np.float32)
    k = np.arange(0, 1023, dtype=np.float32)
    halves = (k + np.float32(0.5)) / np.float32(255)
    halves = halves[halves * np.float32(255) == k + np.float32(0.5)]  # v * 255 is exactly n + 1/2
    assert halves.size > 100
    flat = img.reshape(-1)
    flat[: 3 * halves.size: 3] = halves
    special = np.array([1022.49 / 255, 1022.5 / 255, 1022.51 / 255, 1023.0 / 255, 999.5 / 255, 1000.2 / 255, 4.0, 1e30,
                        -1e-9, -0.0, 0.0, np.nan, np.inf, -np.inf, -0.4, 0.4 / 255], np.float32)
    at = rng.choice(np.arange(3 * halves.size, flat.size), special.size * 4, replace=False)
    flat[at] = np.tile(special, 4)
    return img


def test_dump8_codes_print_the_float_dump(tmp_path):
    """GSRT_FLAG_OUT_DUMP8's exchange format: the PPM written from a frame's code words and escape list is byte for byte
    the PPM of the RGBA32F frame, over every class of value (escapes: anything outside 0..1022 after rounding, -0,
    non-finite); a code holds rint(v * 255) per channel."""
    img = _dump8_frame()
    codes, esc = gsrt.dump8_encode(img)
    a, b = tmp_path / "f.ppm", tmp_path / "c.ppm"
    gsrt.dump_ppm(str(a), img)
    gsrt.dump8_ppm(str(b), codes, esc)
    assert a.read_bytes() == b.read_bytes()
    rgb = img.reshape(-1, 4)[:, :3]
    x = rgb * np.float32(255)
    with np.errstate(invalid="ignore"):
        ok = np.all((x >= 0) & ~np.signbit(x) & (np.rint(x) <= 1022), axis=1)
    c = codes.reshape(-1)
    assert np.array_equal((c & gsrt.DUMP8_ESCAPE) == 0, ok) and 16 < esc.size < c.size
    for ch in range(3):
        assert np.array_equal((c[ok] >> (10 * ch)) & 1023, np.rint(x[ok, ch]).astype(np.uint32))
    assert np.array_equal(esc["pixel"], np.flatnonzero(~ok))
    got = np.stack([esc["r"], esc["g"], esc["b"]], 1)
    assert got.tobytes() == rgb[~ok].tobytes()
    # an escaped pixel whose entry is missing cannot be printed
    with pytest.raises(gsrt.GsrtError):
        gsrt.dump8_ppm(str(b), codes, esc[1:])


@pytest.mark.parametrize("spp,nranks", [(4, 1), (4, 3), (1, 5), (16, 2), (80, 2)])
def test_dump8_host_blocks(tmp_path, spp, nranks):
    """The host mirror of the GSRT_FLAG_OUT_DUMP8 exchange (gsrt_tile_pack_dump8_host / _unpack_dump8_host) on a
    ragged frame with every class of value: each rank's block holds the code words of its packed tiles (the RGBA32F
    packed layout, encoded), its list header the escape count and its entries {local pixel, r, g, b}; the blocks of
    all ranks unpack to the whole frame's codes and escapes, whose PPM is the float frame's."""
    img = _dump8_frame()
    H, W = img.shape[:2]
    ubo = gsrt.camera_from_modelview(O.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, spp, 16)
    ty = gsrt.tile_plan(ubo, gsrt.MODE_COR, nranks, 0)["tiles_y"]
    cost = np.random.default_rng(spp + nranks).integers(1, 100, ty).astype(np.uint32)
    bands = gsrt.tile_bands(ubo, nranks, cost, gsrt.MODE_COR)
    L = gsrt.dump8_layout(ubo, nranks, bands)
    blocks = np.stack([gsrt.tile_pack_dump8(ubo, img, nranks, r, bands=bands) for r in range(nranks)])
    assert blocks.shape == (nranks, L["block"]) and L["codes"] % 4 == 0
    for r in range(nranks):
        packed = gsrt.tile_pack(ubo, img, nranks, r, bands=bands)
        px = packed.shape[0] * packed.shape[1]
        pc, pe = gsrt.dump8_encode(packed.reshape(1, px, 4))
        blk = blocks[r]
        assert np.array_equal(blk[:px], pc.ravel()) and not blk[px:L["codes"]].any()
        n = int(blk[L["codes"]])
        assert n == pe.size and not blk[L["codes"] + 1:L["codes"] + 4].any()
        ent = blk[L["codes"] + 4:L["codes"] + 4 + 4 * n].reshape(n, 4)
        assert np.array_equal(ent[:, 0], pe["pixel"])
        assert ent[:, 1:].tobytes() == np.stack([pe["r"], pe["g"], pe["b"]], 1).tobytes()
        assert not blk[L["codes"] + 4 + 4 * n:].any()
    codes, esc = gsrt.tile_unpack_dump8(ubo, blocks, nranks, bands=bands)
    c0, e0 = gsrt.dump8_encode(img)
    assert np.array_equal(codes, c0) and esc.tobytes() == e0.tobytes()
    a, b = tmp_path / "f.ppm", tmp_path / "c.ppm"
    gsrt.dump_ppm(str(a), img)
    gsrt.dump8_ppm(str(b), codes, esc)
    assert a.read_bytes() == b.read_bytes()


def test_dump8_host_blocks_overflow():
    """more escapes than a block's list holds: the pack reports it (GSRT_E_STATE), and so does the unpack of a block
    whose header counts past the capacity or whose entry names a pixel outside the frame"""
    W, H = 96, 80
    ubo = gsrt.camera_from_modelview(O.lookat((0, 0, 0), (0, 0, -1)), 60.0, W, H, 1.0, 4, 16)
    L = gsrt.dump8_layout(ubo, 2)
    assert L["cap"] == 256
    img = np.full((H, W, 4), 0.5, np.float32)
    img.reshape(-1, 4)[::7, 0] = np.nan  # 1098 escapes, 549 per rank
    with pytest.raises(gsrt.GsrtError):
        gsrt.tile_pack_dump8(ubo, img, 2, 0)
    img = np.full((H, W, 4), 0.5, np.float32)
    img[0, :10, 1] = -1.0
    blocks = np.stack([gsrt.tile_pack_dump8(ubo, img, 2, r) for r in range(2)])
    codes, esc = gsrt.tile_unpack_dump8(ubo, blocks, 2)
    assert esc.size == 10 and np.array_equal(esc["pixel"], np.arange(10))
    bad = blocks.copy()
    bad[1, L["codes"]] = L["cap"] + 1
    with pytest.raises(gsrt.GsrtError):
        gsrt.tile_unpack_dump8(ubo, bad, 2)
    bad = blocks.copy()
    bad[0, L["codes"] + 4] = L["codes"] + 7  # a local pixel past the rank's tiles
    with pytest.raises(gsrt.GsrtError):
        gsrt.tile_unpack_dump8(ubo, bad, 2)
    with pytest.raises(gsrt.GsrtError):  # dump8 frames are COR frames
        gsrt.dump8_layout(ubo, 2, mode=gsrt.MODE_REF)


def test_image_binary_records(tmp_path):
    img = np.arange(2 * 3 * 4, dtype=np.float32).reshape(2, 3, 4)
    path = tmp_path / "image.binary"
    gsrt.dump_image_binary(str(path), img)
    rec = np.fromfile(path, dtype=np.dtype([("rgb", "<f4", 3), ("off", "<u4")]))
    assert len(rec) == 6
    np.testing.assert_array_equal(rec["rgb"], img.reshape(-1, 4)[:, :3])
    np.testing.assert_array_equal(rec["off"], np.arange(6))


def test_reference_ppm_name():
    assert re.fullmatch(r"\d\d-\d\d-\d{4}-\d\d-\d\d-\d\d-SCENE\.ppm", gsrt.reference_ppm_name())


@pytest.mark.parametrize("spp,tw,th", [(1, 8, 8), (2, 8, 4), (4, 4, 4), (8, 4, 2), (16, 2, 2), (64, 1, 1), (3, 8, 8)])
def test_tile_plan(spp, tw, th):
    ubo = gsrt.camera_from_modelview(O.lookat((0, 0, 0), (0, 0, -1)), 60.0, 1920, 1080, 1.0, spp, 16)
    p = gsrt.tile_plan(ubo, gsrt.MODE_COR, 1, 0)
    assert (p["tile_w"], p["tile_h"]) == (tw, th)
    assert p["tiles_x"] == -(-1920 // tw) and p["tiles_y"] == -(-1080 // th)
    assert p["spp_lanes"] * tw * th == 64 or (spp == 3 and p["spp_lanes"] == 1)
    total = p["tiles_x"] * p["tiles_y"]
    for n in (2, 3, 8):
        plans = [gsrt.tile_plan(ubo, gsrt.MODE_COR, n, r) for r in range(n)]
        counts = [q["local_tiles"] for q in plans]
        # even bands of whole tile rows (no cost profile): the ranks but the root within one row of each other, the
        # gather's root lighter by its weight (1 - 0.09 (n - 1) / spp, >= 1/4)
        assert sum(counts) == total and max(counts[1:]) - min(counts[1:]) <= p["tiles_x"]
        w0 = max(0.25, 1 - 0.09 * (n - 1) / spp)
        assert abs(counts[0] - np.mean(counts[1:]) * w0) <= 2 * p["tiles_x"], (counts, w0)
        assert [q["row0"] for q in plans] == sorted(q["row0"] for q in plans) and plans[0]["row0"] == 0
        assert plans[0]["stride"] == max(counts)
    ref = gsrt.tile_plan(ubo, gsrt.MODE_REF, 1, 0)
    assert (ref["tile_w"], ref["tile_h"], ref["spp_lanes"]) == (8, 8, 1)


def test_bad_arguments_rejected():
    with pytest.raises(gsrt.GsrtError):
        gsrt.camera_from_modelview(np.eye(4, dtype=np.float32).reshape(16), 60.0, 0, 10)
    with pytest.raises(gsrt.GsrtError):
        gsrt.tile_plan(gsrt.camera_from_modelview(np.eye(4, dtype=np.float32).reshape(16), 60.0, 8, 8), 0, 2, 5)


CLI = os.path.join(ROOT, "3dgs-raytrace_amd", "bin", "gsrt_render")


def test_cli_rejects_bad_flags():
    for argv in (["--bogus"], ["--scene", "7"], ["--mode", "fast"], ["--width", "0"], ["--width"]):
        p = subprocess.run([CLI] + argv, capture_output=True, text=True)
        assert p.returncode == 2, argv
        assert "usage: gsrt_render" in p.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU may be present")
def test_cli_without_device_fails_loudly():
    p = subprocess.run([CLI, "--scene", "33"], capture_output=True, text=True)
    assert p.returncode == 1 and "device error" in p.stderr


def _deal_py(cost, centre, xcds=8):
    """a restatement of the share's render-unit deal: longest first (stable over the centre-out order), each unit to
    the least-loaded XCD (lowest index on ties) among those not yet holding units / xcds"""
    R = len(cost)
    by = sorted(centre, key=lambda q: -cost[q])  # sorted() is stable
    load, count, perm = [0.0] * xcds, [0] * xcds, [0] * R
    for q in by:
        x = min((j for j in range(xcds) if count[j] < R // xcds), key=lambda j: (load[j], j))
        perm[count[x] * xcds + x] = q
        load[x] += cost[q]
        count[x] += 1
    return perm


@pytest.mark.parametrize("units,seed", [(8, 1), (64, 2), (224, 3), (1024, 4)])
def test_deal_units(units, seed):
    """gsrt_deal_units (the deal launch_render uses when a whole frame's tile costs are known) against the restatement:
    a permutation, R/8 units per XCD, each XCD's units longest first, XCD loads within one unit's cost of each other"""
    rng = np.random.default_rng(seed)
    cost = rng.gamma(2.0, 1000.0, units)
    cost[rng.integers(0, units, units // 4)] = 500.0  # ties
    centre = rng.permutation(units).astype(np.uint32)
    perm = gsrt.deal_units(cost, centre)
    assert perm.tolist() == _deal_py(cost.tolist(), centre.tolist())
    assert sorted(perm.tolist()) == list(range(units))
    per = perm.reshape(-1, 8)  # row k: the k-th unit of each XCD
    c = cost[per]
    assert np.all(np.diff(c, axis=0) <= 0)
    loads = c.sum(axis=0)
    assert loads.max() - loads.min() <= cost.max() + 1e-9
    with pytest.raises(gsrt.GsrtError):
        gsrt.deal_units(cost[:units - 1] if units > 8 else cost[:7])
