"""gsrt -- Python host mirror of the C ABI in include/gsrt.h (ctypes over gsrt/libgsrt.so).

Mirrors the reference's scene / camera / dispatch / frame-dump interface for the Gaussian render path
(SURVEY.md §8b): `Scene.from_params` ~ Assets::Scene packing (Scene.cpp:16-182), `Scene.from_model` ~
Model::CreateGauss (Model.cpp:550-564), `Scene.build_bvh` ~ the TLAS build, `Scene.render` ~
vkCmdTraceRaysKHR(W,H,1) over GaussTracing.rgen, `dump_ppm` ~ VulkanRayTracing::image_store.

Errors raise GsrtError carrying the C status. The native library is required: importing this module
without a built libgsrt.so raises ImportError (there is no CPU fallback in the product path).
"""
from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSRT_LIB_PATH") or os.path.join(_HERE, "libgsrt.so")  # override: A/B builds

OK, E_ARG, E_OOM, E_DEVICE, E_IO, E_STATE, E_COMM = 0, -1, -2, -3, -4, -5, -6
PAGE_GAUSSIANS = 4096  # GSRT_PAGE_GAUSSIANS
MODE_REF, MODE_COR = 0, 1
FLAG_LUT, FLAG_STATS, FLAG_OUT_DUMP8 = 0x100, 0x200, 0x400
DUMP8_ESCAPE = 1 << 30  # GSRT_DUMP8_ESCAPE
SYNTH_COR, SYNTH_REF, SYNTH_NEEDLE = 0, 1, 2

UBO_DTYPE = np.dtype([
    ("model_view", "<f4", 16), ("projection", "<f4", 16),
    ("model_view_inverse", "<f4", 16), ("projection_inverse", "<f4", 16),
    ("light_position", "<f4", 3), ("light_radius", "<f4"), ("aperture", "<f4"),
    ("focus_distance", "<f4"), ("heatmap_scale", "<f4"),
    ("total_samples", "<u4"), ("samples", "<u4"), ("bounces", "<u4"), ("shadows", "<u4"),
    ("random_seed", "<u4"), ("width", "<u4"), ("height", "<u4"), ("has_sky", "<u4"),
    ("show_heatmap", "<u4"),
])
RAYSTATE_DTYPE = np.dtype([("trans", "<f4"), ("depth", "<f4"), ("gauss_num", "<i4"),
                           ("gauss_num_raw", "<i4"), ("k", "<f4", (8, 2))])
ESCAPE_DTYPE = np.dtype([("pixel", "<u4"), ("r", "<f4"), ("g", "<f4"), ("b", "<f4")])  # gsrt_dump8_escape
assert UBO_DTYPE.itemsize == 320 and RAYSTATE_DTYPE.itemsize == 80 and ESCAPE_DTYPE.itemsize == 16

# every symbol include/gsrt.h (the drop-in ABI) and include/gsrt_test.h (test and measurement hooks) declare (tests check
# the library exports all of them)
EXPORTS = [
    "gsrt_status_string", "gsrt_abi_version", "gsrt_create", "gsrt_destroy", "gsrt_last_error",
    "gsrt_synchronize", "gsrt_stream", "gsrt_prep_stream", "gsrt_update_stream", "gsrt_slot_streams", "gsrt_scene_from_params", "gsrt_scene_from_model",
    "gsrt_scene_download", "gsrt_scene_size", "gsrt_destroy_scene", "gsrt_camera_from_modelview",
    "gsrt_camera_from_file", "gsrt_lookat", "gsrt_build_bvh", "gsrt_refit_bvh", "gsrt_scene_update", "gsrt_scene_attach",
    "gsrt_scene_detach", "gsrt_bvh_info",
    "gsrt_bvh_download", "gsrt_render", "gsrt_render_async", "gsrt_framebuffer", "gsrt_last_stats",
    "gsrt_comm_unique_id", "gsrt_comm_init", "gsrt_comm_stream", "gsrt_render_sharded", "gsrt_render_sharded_async",
    "gsrt_dump_ppm", "gsrt_reference_ppm_name", "gsrt_dump_image_binary", "gsrt_synth_cloud",
    "gsrt_timing", "gsrt_timing_read", "gsrt_tile_plan", "gsrt_render_sharded_emulated",
    "gsrt_debug_counters", "gsrt_debug_counters_hi", "gsrt_exp_lut", "gsrt_debug_exp_lut", "gsrt_ply_info",
    "gsrt_ply_read", "gsrt_scene_from_ply", "gsrt_dump_rgba_text", "gsrt_scene_add_mesh", "gsrt_scene_mesh_triangles",
    "gsrt_sphere_mesh", "gsrt_scene_stream_pages", "gsrt_scene_pages", "gsrt_host_register", "gsrt_host_unregister",
    "gsrt_vs_stats", "gsrt_dump_vs_stats", "gsrt_tile_pack_host", "gsrt_tile_unpack_host",
    "gsrt_timing_read_exchange", "gsrt_comm_size", "gsrt_debug_gathered", "gsrt_tile_bands", "gsrt_timing_kernel_only",
    "gsrt_set_bands", "gsrt_last_bands", "gsrt_row_costs", "gsrt_dump8_read", "gsrt_dump8_encode", "gsrt_dump8_ppm",
    "gsrt_render_sharded_emulated_dump8", "gsrt_debug_share_costs", "gsrt_debug_row_profile", "gsrt_debug_streams", "gsrt_deal_units", "gsrt_dump8_layout",
    "gsrt_tile_pack_dump8_host", "gsrt_tile_unpack_dump8_host", "gsrt_timing_stride", "gsrt_partition_hash",
    "gsrt_decide_bands",
]


class GsrtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"gsrt status {status}: {msg}")
        self.status = status


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"gsrt native library not built: {LIB_PATH} (run __graft_entry__.build() or make)")
    L = ctypes.CDLL(LIB_PATH)
    P, u32, i32, f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_float
    PP = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "gsrt_status_string": ([i32], ctypes.c_char_p),
        "gsrt_abi_version": ([], i32),
        "gsrt_create": ([PP, i32], i32),
        "gsrt_destroy": ([P], None),
        "gsrt_last_error": ([P], ctypes.c_char_p),
        "gsrt_synchronize": ([P], i32),
        "gsrt_stream": ([P], P),
        "gsrt_prep_stream": ([P], P),
        "gsrt_update_stream": ([P], P),
        "gsrt_slot_streams": ([P], i32),
        "gsrt_scene_from_params": ([P, P, P, u32, P, PP], i32),
        "gsrt_scene_from_model": ([P, P, P, P, P, P, u32, PP], i32),
        "gsrt_scene_download": ([P, P, P], i32),
        "gsrt_scene_size": ([P], u32),
        "gsrt_destroy_scene": ([P], None),
        "gsrt_camera_from_modelview": ([P, f32, u32, u32, f32, u32, u32, P], i32),
        "gsrt_camera_from_file": ([ctypes.c_char_p, f32, u32, u32, f32, u32, u32, P], i32),
        "gsrt_lookat": ([P, P, P, P], i32),
        "gsrt_build_bvh": ([P], i32),
        "gsrt_refit_bvh": ([P, P], i32),
        "gsrt_scene_update": ([P, P, P], i32),
        "gsrt_scene_attach": ([P, P, P], i32),
        "gsrt_scene_detach": ([P], i32),
        "gsrt_ply_info": ([ctypes.c_char_p, P, P], i32),
        "gsrt_ply_read": ([ctypes.c_char_p, P, P, P, P, P], i32),
        "gsrt_scene_from_ply": ([P, ctypes.c_char_p, i32, PP], i32),
        "gsrt_dump_rgba_text": ([ctypes.c_char_p, P, u32, u32], i32),
        "gsrt_bvh_info": ([P, P, P, P], i32),
        "gsrt_bvh_download": ([P, P, P, P], i32),
        "gsrt_render": ([P, P, u32, u32, P, P], i32),
        "gsrt_render_async": ([P, P, u32, u32, P, P], i32),
        "gsrt_framebuffer": ([P], P),
        "gsrt_last_stats": ([P, P, P], i32),
        "gsrt_comm_unique_id": ([P], i32),
        "gsrt_comm_init": ([P, P, i32, i32], i32),
        "gsrt_comm_stream": ([P], P),
        "gsrt_render_sharded": ([P, P, u32, u32, P], i32),
        "gsrt_render_sharded_async": ([P, P, u32, u32], i32),
        "gsrt_dump_ppm": ([ctypes.c_char_p, P, u32, u32], i32),
        "gsrt_reference_ppm_name": ([ctypes.c_char_p, ctypes.c_size_t], i32),
        "gsrt_dump_image_binary": ([ctypes.c_char_p, P, u32, u32], i32),
        "gsrt_synth_cloud": ([u32, u32, u32, i32, P, P, P, P, P], i32),
        "gsrt_timing": ([P, u32], i32),
        "gsrt_timing_read": ([P, P, P, u32, P], i32),
        "gsrt_timing_read_exchange": ([P, P, u32, P], i32),
        "gsrt_timing_kernel_only": ([P, i32], i32),
        "gsrt_comm_size": ([P, P, P], i32),
        "gsrt_debug_gathered": ([P, P, ctypes.c_size_t], i32),
        "gsrt_tile_bands": ([P, u32, i32, P, P], i32),
        "gsrt_set_bands": ([P, i32, P], i32),
        "gsrt_last_bands": ([P, P, u32, P], i32),
        "gsrt_row_costs": ([P, P, u32, P], i32),
        "gsrt_tile_plan": ([P, u32, i32, i32, P], i32),
        "gsrt_debug_counters": ([P, P], i32),
        "gsrt_debug_counters_hi": ([P, P], i32),
        "gsrt_exp_lut": ([P], i32),
        "gsrt_debug_exp_lut": ([P, P], i32),
        "gsrt_render_sharded_emulated": ([P, P, u32, i32, P, P], i32),
        "gsrt_scene_add_mesh": ([P, P, u32, P, u32], i32),
        "gsrt_scene_mesh_triangles": ([P], u32),
        "gsrt_sphere_mesh": ([P, f32, P, P], i32),
        "gsrt_scene_stream_pages": ([P, P, P, P, u32], i32),
        "gsrt_scene_pages": ([P], u32),
        "gsrt_host_register": ([P, P, ctypes.c_size_t], i32),
        "gsrt_host_unregister": ([P, P], i32),
        "gsrt_vs_stats": ([P, P], i32),
        "gsrt_tile_pack_host": ([P, u32, i32, i32, P, P, P], i32),
        "gsrt_tile_unpack_host": ([P, u32, i32, P, P, P], i32),
        "gsrt_dump_vs_stats": ([P, ctypes.c_char_p], i32),
        "gsrt_dump8_read": ([P, P, P, u32, P], i32),
        "gsrt_dump8_encode": ([P, ctypes.c_size_t, P, P, u32, P], i32),
        "gsrt_dump8_ppm": ([ctypes.c_char_p, P, u32, u32, P, u32], i32),
        "gsrt_render_sharded_emulated_dump8": ([P, P, u32, i32, P, P, P, u32, P], i32),
        "gsrt_dump8_layout": ([P, u32, i32, P, P], i32),
        "gsrt_timing_stride": ([P, u32], i32),
        "gsrt_tile_pack_dump8_host": ([P, u32, i32, i32, P, P, P], i32),
        "gsrt_tile_unpack_dump8_host": ([P, u32, i32, P, P, P, P, u32, P], i32),
        "gsrt_debug_share_costs": ([P, i32], i32),
        "gsrt_partition_hash": ([P, u32, i32, P, i32, P], i32),
        "gsrt_decide_bands": ([P, u32, i32, P, i32, P, u32, P], i32),
        "gsrt_debug_row_profile": ([P, P, u32, P], i32),
        "gsrt_debug_streams": ([P, P, P], i32),
        "gsrt_deal_units": ([P, P, u32, P], i32),
    }
    for name, (args, res) in sig.items():
        # an experiment build named by GSRT_LIB_PATH (an older revision under A/B) may predate a symbol; the
        # product library must export every one
        if os.environ.get("GSRT_LIB_PATH") and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


lib = _load()


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _check(status: int, ctx=None):
    if status != OK:
        msg = lib.gsrt_status_string(status).decode()
        if ctx is not None and ctx.handle:
            detail = lib.gsrt_last_error(ctx.handle).decode()
            if detail:
                msg = f"{msg}: {detail}"
        raise GsrtError(status, msg)


def _f32(a, shape):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a.reshape(shape)


# ---------------------------------------------------------------- camera (RayTracer.cpp:38-65)

def lookat(eye, center, up=(0.0, 1.0, 0.0)) -> np.ndarray:
    out = np.zeros(16, np.float32)
    e, c, u = _f32(eye, 3), _f32(center, 3), _f32(up, 3)  # keep the buffers alive across the call
    _check(lib.gsrt_lookat(_p(e), _p(c), _p(u), _p(out)))
    return out


def translate(x, y, z) -> np.ndarray:
    """glm::translate(mat4(1), vec3(x, y, z)), column-major."""
    m = np.eye(4, dtype=np.float32)
    m[3, :3] = (x, y, z)
    return m.reshape(16)


def camera_from_modelview(mv, fovy_deg, width, height, focus_distance=1.0, samples=1, bounces=16) -> np.ndarray:
    ubo = np.zeros(1, UBO_DTYPE)
    m = _f32(mv, 16)
    _check(lib.gsrt_camera_from_modelview(_p(m), fovy_deg, width, height, focus_distance,
                                          samples, bounces, _p(ubo)))
    return ubo


def camera_from_file(path, fovy_deg, width, height, focus_distance=1.0, samples=1, bounces=16) -> np.ndarray:
    ubo = np.zeros(1, UBO_DTYPE)
    _check(lib.gsrt_camera_from_file(os.fsencode(path), fovy_deg, width, height, focus_distance, samples,
                                     bounces, _p(ubo)))
    return ubo


# ---------------------------------------------------------------- frame dump / synthetic inputs

def dump_ppm(path, rgba):
    rgba = np.ascontiguousarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    _check(lib.gsrt_dump_ppm(os.fsencode(path), _p(rgba), w, h))


def dump8_encode(rgba):
    """(codes[H, W] uint32, escapes ESCAPE_DTYPE) of an RGBA32F frame: what GSRT_FLAG_OUT_DUMP8 exchanges"""
    rgba = np.ascontiguousarray(rgba, np.float32)
    H, W = rgba.shape[:2]
    codes = np.zeros((H, W), np.uint32)
    n = np.zeros(1, np.uint32)
    _check(lib.gsrt_dump8_encode(_p(rgba), W * H, _p(codes), None, 0, _p(n)))
    esc = np.zeros(int(n[0]), ESCAPE_DTYPE)
    _check(lib.gsrt_dump8_encode(_p(rgba), W * H, _p(codes), _p(esc), esc.size, _p(n)))
    return codes, esc


def dump8_ppm(path, codes, esc):
    """the P3 PPM of a frame in dump codes + escapes (the bytes dump_ppm writes for the same frame)"""
    codes = np.ascontiguousarray(codes, np.uint32)
    esc = np.ascontiguousarray(esc, ESCAPE_DTYPE)
    H, W = codes.shape
    _check(lib.gsrt_dump8_ppm(os.fsencode(path), _p(codes), W, H, _p(esc) if esc.size else None, esc.size))


def dump_image_binary(path, rgba):
    rgba = np.ascontiguousarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    _check(lib.gsrt_dump_image_binary(os.fsencode(path), _p(rgba), w, h))


def dump_rgba_text(path, rgba):
    """dump_image.sh text lines "[x, y] rgba(r, g, b)" (RayTracing.rgen:98)"""
    rgba = np.ascontiguousarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    _check(lib.gsrt_dump_rgba_text(os.fsencode(path), _p(rgba), w, h))


def ply_info(path) -> dict:
    n = np.zeros(1, np.uint32)
    d = np.zeros(1, np.uint32)
    _check(lib.gsrt_ply_info(os.fsencode(path), _p(n), _p(d)))
    return {"n": int(n[0]), "sh_degree": int(d[0])}


def ply_read(path, with_sh=True):
    """3DGS .ply -> (center, rot_rxyz, scale, opacity, sh|None) in the gsrt_scene_from_model convention"""
    n = ply_info(path)["n"]
    c = np.zeros((n, 3), np.float32)
    r = np.zeros((n, 4), np.float32)
    s = np.zeros((n, 3), np.float32)
    o = np.zeros(n, np.float32)
    sh = np.zeros((n, 48), np.float32) if with_sh else None
    _check(lib.gsrt_ply_read(os.fsencode(path), _p(c), _p(r), _p(s), _p(o), _p(sh)))
    return c, r, s, o, sh


def reference_ppm_name() -> str:
    buf = ctypes.create_string_buffer(64)
    _check(lib.gsrt_reference_ppm_name(buf, 64))
    return buf.value.decode()


def exp_lut() -> np.ndarray:
    """The REF ExpLUT as the host library computes it (256 x {k, b})."""
    out = np.zeros(512, np.float32)
    _check(lib.gsrt_exp_lut(_p(out)))
    return out


def synth_cloud(kind, n, seed=42, with_sh=False):
    c = np.zeros((n, 3), np.float32)
    r = np.zeros((n, 4), np.float32)
    s = np.zeros((n, 3), np.float32)
    o = np.zeros(n, np.float32)
    sh = np.zeros((n, 16, 3), np.float32) if with_sh else None
    _check(lib.gsrt_synth_cloud(kind, n, seed, int(with_sh), _p(c), _p(r), _p(s), _p(o), _p(sh)))
    return c, r, s, o, sh


def sphere_mesh(center, radius):
    """Model::CreateSphere geometry (Model.cpp:566-629): vertices (561, 3) f32, indices (1024, 3) u32"""
    c = np.asarray(center, np.float32)
    v = np.zeros((561, 3), np.float32)
    i = np.zeros((1024, 3), np.uint32)
    _check(lib.gsrt_sphere_mesh(_p(c), float(radius), _p(v), _p(i)))
    return v, i


def tile_plan(ubo, mode=MODE_COR, nranks=1, rank=0) -> dict:
    """the frame's tiles under the even partition (gsrt_tile_plan)"""
    out = np.zeros(8, np.uint32)
    _check(lib.gsrt_tile_plan(_p(ubo), mode, nranks, rank, _p(out)))
    return dict(zip(["tile_w", "tile_h", "tiles_x", "tiles_y", "local_tiles", "spp_lanes", "row0", "stride"],
                    (int(v) for v in out)))


def _bands_arg(bands):
    return None if bands is None else np.ascontiguousarray(bands, np.uint32)


def tile_bands(ubo, nranks, row_cost=None, mode=MODE_COR) -> np.ndarray:
    """the partition's nranks + 1 tile-row boundaries the balancing rule cuts from a row cost profile (None: even)"""
    out = np.zeros(nranks + 1, np.uint32)
    rc = None if row_cost is None else np.ascontiguousarray(row_cost, np.uint32)
    _check(lib.gsrt_tile_bands(_p(ubo), mode, nranks, _p(rc), _p(out)))
    return out


def partition_hash(ubo, nranks, bands, pinned=False, mode=MODE_COR) -> int:
    """the partition hash a rank's cost profile carries for `bands` (gsrt_partition_hash)"""
    out = np.zeros(1, np.uint32)
    b = np.ascontiguousarray(bands, np.uint32)
    _check(lib.gsrt_partition_hash(_p(ubo), mode, nranks, _p(b), 1 if pinned else 0, _p(out)))
    return int(out[0])


def decide_bands(ubo, nranks, bands, profile, my_hash, pinned=False, mode=MODE_COR) -> np.ndarray:
    """the bands every rank adopts from an all-reduced profile (tiles_y row costs, then max(h), max(~h) of the ranks'
    partition hashes): gsrt_decide_bands, GsrtError(E_COMM) when the ranks' hashes differ"""
    out = np.zeros(nranks + 1, np.uint32)
    b = np.ascontiguousarray(bands, np.uint32)
    pr = np.ascontiguousarray(profile, np.uint32)
    _check(lib.gsrt_decide_bands(_p(ubo), mode, nranks, _p(b), 1 if pinned else 0, _p(pr), my_hash & 0xffffffff, _p(out)))
    return out


def deal_units(cost, centre=None) -> np.ndarray:
    """a rank share's render-unit deal over the 8 XCDs (gsrt_deal_units): perm[k * 8 + x] = XCD x's k-th unit"""
    c = np.ascontiguousarray(cost, np.float64)
    ctr = np.arange(c.size, dtype=np.uint32) if centre is None else np.ascontiguousarray(centre, np.uint32)
    out = np.zeros(c.size, np.uint32)
    _check(lib.gsrt_deal_units(_p(c), _p(ctr), c.size, _p(out)))
    return out


def tile_stride(ubo, nranks, bands=None, mode=MODE_COR) -> int:
    """the packed stride (the largest band's tile count) of a partition"""
    pl = tile_plan(ubo, mode, nranks, 0)
    if bands is None:
        return pl["stride"]
    return int(np.diff(np.asarray(bands, np.int64)).max()) * pl["tiles_x"]


def tile_pack(ubo, rgba, nranks, rank, mode=MODE_COR, bands=None) -> np.ndarray:
    """rank's tiles of an (H, W, 4) f32 frame in the packed layout of its sharded render (gsrt_tile_pack_host)"""
    pl = tile_plan(ubo, mode, nranks, rank)
    out = np.zeros((tile_stride(ubo, nranks, bands, mode), pl["tile_w"] * pl["tile_h"], 4), np.float32)
    src = np.ascontiguousarray(rgba, np.float32)
    b = _bands_arg(bands)
    _check(lib.gsrt_tile_pack_host(_p(ubo), mode, nranks, rank, _p(b), _p(src), _p(out)))
    return out


def tile_unpack(ubo, gathered, nranks, mode=MODE_COR, bands=None) -> np.ndarray:
    """the frame from all ranks' packed blocks (nranks, stride, tile_w * tile_h, 4), as k_unpack builds it"""
    W, H = int(ubo["width"][0]), int(ubo["height"][0])
    out = np.zeros((H, W, 4), np.float32)
    g = np.ascontiguousarray(gathered, np.float32)
    b = _bands_arg(bands)
    _check(lib.gsrt_tile_unpack_host(_p(ubo), mode, nranks, _p(b), _p(g), _p(out)))
    return out


def dump8_layout(ubo, nranks, bands=None, mode=MODE_COR) -> dict:
    """a rank's GSRT_FLAG_OUT_DUMP8 block: {"block": words, "codes": code words (the list header's offset),
    "cap": escape capacity} (gsrt_dump8_layout)"""
    out = np.zeros(3, np.uint64)
    b = _bands_arg(bands)
    _check(lib.gsrt_dump8_layout(_p(ubo), mode, nranks, _p(b), _p(out)))
    return dict(block=int(out[0]), codes=int(out[1]), cap=int(out[2]))


def tile_pack_dump8(ubo, rgba, nranks, rank, mode=MODE_COR, bands=None) -> np.ndarray:
    """rank's dump8 block (uint32 words) of an (H, W, 4) f32 frame, as its sharded render writes it
    (gsrt_tile_pack_dump8_host; raises when the frame's escapes overflow the block's list)"""
    L = dump8_layout(ubo, nranks, bands, mode)
    out = np.zeros(L["block"], np.uint32)
    src = np.ascontiguousarray(rgba, np.float32)
    b = _bands_arg(bands)
    _check(lib.gsrt_tile_pack_dump8_host(_p(ubo), mode, nranks, rank, _p(b), _p(src), _p(out)))
    return out


def tile_unpack_dump8(ubo, gathered, nranks, mode=MODE_COR, bands=None):
    """(codes[H, W] uint32, escapes in pixel order) from all ranks' dump8 blocks (nranks, block words), as rank 0
    unpacks them after the gather (gsrt_tile_unpack_dump8_host)"""
    W, H = int(ubo["width"][0]), int(ubo["height"][0])
    L = dump8_layout(ubo, nranks, bands, mode)
    codes = np.zeros((H, W), np.uint32)
    esc = np.zeros(L["cap"] * nranks, ESCAPE_DTYPE)
    n = np.zeros(1, np.uint32)
    g = np.ascontiguousarray(gathered, np.uint32)
    assert g.size == L["block"] * nranks
    b = _bands_arg(bands)
    _check(lib.gsrt_tile_unpack_dump8_host(_p(ubo), mode, nranks, _p(b), _p(g), _p(codes), _p(esc), esc.size, _p(n)))
    return codes, esc[: int(n[0])].copy()


def comm_unique_id() -> bytes:
    buf = np.zeros(128, np.uint8)
    _check(lib.gsrt_comm_unique_id(_p(buf)))
    return buf.tobytes()


# ---------------------------------------------------------------- context / scene

class Context:
    """One gsrt_ctx per device (gsrt_create)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        st = lib.gsrt_create(ctypes.byref(h), device)
        if st != OK:
            raise GsrtError(st, f"gsrt_create(device={device}) failed: {lib.gsrt_status_string(st).decode()}")
        self.handle = h
        self._scenes = weakref.WeakSet()

    def close(self):
        if getattr(self, "handle", None):
            for sc in list(self._scenes):
                sc.close()
            lib.gsrt_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def synchronize(self):
        _check(lib.gsrt_synchronize(self.handle), self)

    @property
    def stream(self) -> int:
        return lib.gsrt_stream(self.handle) or 0

    @property
    def prep_stream(self) -> int:
        return lib.gsrt_prep_stream(self.handle) or 0

    @property
    def update_stream(self) -> int:
        """the stream of scene updates' copies (gsrt_update_stream): a GPU producer of an update's source fills it there"""
        return lib.gsrt_update_stream(self.handle) or 0

    def slot_streams(self) -> bool:
        """whether the last frame ran on slot streams (its prep and render kernels on its frame slot's stream)"""
        return bool(lib.gsrt_slot_streams(self.handle))

    @property
    def framebuffer_ptr(self) -> int:
        return lib.gsrt_framebuffer(self.handle) or 0

    def last_stats(self, per_ray_shape=None):
        out = np.zeros(8, np.uint64)
        per = np.zeros(per_ray_shape + (4,), np.uint32) if per_ray_shape else None
        _check(lib.gsrt_last_stats(self.handle, _p(out), _p(per)), self)
        keys = ["rays", "candidates", "blended", "terminated", "tile_rounds", "restarts", "tiles", "max_tile_candidates"]
        d = {k: int(v) for k, v in zip(keys, out)}
        if per is not None:
            d["per_ray"] = per
        return d

    def vs_stats(self) -> dict:
        """vulkan-sim's rt_* statistics of the last REF render with FLAG_STATS (gsrt_vs_stats)"""
        out = np.zeros(8, np.uint64)
        _check(lib.gsrt_vs_stats(self.handle, _p(out)), self)
        keys = ["rt_n_total_rays", "rt_num_hits", "rt_max_tree_depth", "rt_max_nodes_per_ray", "rt_tot_nodes_per_ray",
                "overflowed_walks"]
        return {k: int(v) for k, v in zip(keys, out)}

    def dump_vs_stats(self, path):
        _check(lib.gsrt_dump_vs_stats(self.handle, os.fsencode(path)), self)

    def debug_counters(self):
        """The 32-word counter block of the last render (diagnostic; [16..] filled by GSRT_DIAG builds)."""
        out = np.zeros(32, np.uint64)
        _check(lib.gsrt_debug_counters(self.handle, _p(out[:16])), self)
        _check(lib.gsrt_debug_counters_hi(self.handle, _p(out[16:])), self)
        return out

    def device_exp_lut(self) -> np.ndarray:
        """The ExpLUT copy in HBM the REF kernels read (uploaded by gsrt_create)."""
        out = np.zeros(512, np.float32)
        _check(lib.gsrt_debug_exp_lut(self.handle, _p(out)), self)
        return out

    def timing(self, frames: int, kernel_only: bool = False, stride: int = 1):
        """Record HIP events around the next `frames` renders: the render kernel and (kernel_only False) the whole
        frame; with kernel_only the frame times read 0 and the timed frames carry two events each. stride > 1: only
        every stride-th frame is recorded (`frames` recorded frames, the others carry no events)."""
        _check(lib.gsrt_timing_kernel_only(self.handle, 1 if kernel_only else 0), self)
        _check(lib.gsrt_timing_stride(self.handle, stride), self)
        _check(lib.gsrt_timing(self.handle, frames), self)

    def timing_read(self, cap: int = 4096):
        k = np.zeros(cap, np.float32)
        f = np.zeros(cap, np.float32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_timing_read(self.handle, _p(k), _p(f), cap, _p(n)), self)
        return k[: int(n[0])].copy(), f[: int(n[0])].copy()

    def timing_read_exchange(self, cap: int = 4096):
        """per timed frame: the sharded exchange (gather + rank 0's unpack) on the comm stream, ms (0: no exchange)"""
        x = np.zeros(cap, np.float32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_timing_read_exchange(self.handle, _p(x), cap, _p(n)), self)
        return x[: int(n[0])].copy()

    def comm_size(self):
        """(ranks, rank) of the communicator as RCCL reports them; (1, 0) without comm_init"""
        n = np.zeros(1, np.int32)
        r = np.zeros(1, np.int32)
        _check(lib.gsrt_comm_size(self.handle, _p(n), _p(r)), self)
        return int(n[0]), int(r[0])

    def host_register(self, arr: np.ndarray):
        """page-lock a numpy array for asynchronous host-to-HBM streaming (gsrt_scene_stream_pages)"""
        _check(lib.gsrt_host_register(self.handle, ctypes.c_void_p(arr.ctypes.data), arr.nbytes), self)

    def host_unregister(self, arr: np.ndarray):
        _check(lib.gsrt_host_unregister(self.handle, ctypes.c_void_p(arr.ctypes.data)), self)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = np.frombuffer(uid, np.uint8).copy()
        _check(lib.gsrt_comm_init(self.handle, _p(buf), nranks, rank), self)

    def debug_gathered(self, floats: int) -> np.ndarray:
        """rank 0's gather buffer after the last sharded frame (its first `floats` floats)"""
        out = np.zeros(floats, np.float32)
        _check(lib.gsrt_debug_gathered(self.handle, _p(out), floats), self)
        return out

    def comm_init_loopback(self):
        """A one-rank RCCL communicator that still takes the exchange path (packed buffers, ncclGather, k_unpack on
        the comm stream; GSRT_DEBUG_COMM_LOOPBACK). With GSRT_DEBUG_RANK_OF=N[:r] its sharded frames run rank r's
        share of an N-rank frame (the rank-share measurement)."""
        old = os.environ.get("GSRT_DEBUG_COMM_LOOPBACK")
        os.environ["GSRT_DEBUG_COMM_LOOPBACK"] = "1"
        try:
            self.comm_init(comm_unique_id(), 1, 0)
        finally:
            if old is None:
                del os.environ["GSRT_DEBUG_COMM_LOOPBACK"]
            else:
                os.environ["GSRT_DEBUG_COMM_LOOPBACK"] = old

    def set_bands(self, nranks: int, bands=None):
        """pin this ctx's sharded frames to a partition (nranks + 1 tile-row boundaries), or back to balancing (None)"""
        b = _bands_arg(bands)
        _check(lib.gsrt_set_bands(self.handle, nranks, _p(b)), self)

    def last_bands(self) -> np.ndarray:
        """the bands of the last sharded frame (empty before any)"""
        out = np.zeros(65, np.uint32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_last_bands(self.handle, _p(out), 65, _p(n)), self)
        return out[: int(n[0])].copy()

    def row_costs(self) -> np.ndarray:
        """the last whole COR frame's per-tile-row shading cost (the balancing profile)"""
        out = np.zeros(1 << 16, np.uint32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_row_costs(self.handle, _p(out), out.size, _p(n)), self)
        return out[: int(n[0])].copy()

    def dump8_read(self, width: int, height: int):
        """rank 0, after a FLAG_OUT_DUMP8 sharded frame: (codes[H, W], escapes in pixel order)"""
        codes = np.zeros((height, width), np.uint32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_dump8_read(self.handle, _p(codes), None, 0, _p(n)), self)
        esc = np.zeros(int(n[0]), ESCAPE_DTYPE)
        if esc.size:
            _check(lib.gsrt_dump8_read(self.handle, None, _p(esc), esc.size, _p(n)), self)
        return codes, esc

    def debug_share_costs(self, on: bool = True):
        """every sharded COR frame stores its tiles' costs (test hook; see debug_row_profile)"""
        _check(lib.gsrt_debug_share_costs(self.handle, 1 if on else 0), self)

    def debug_row_profile(self) -> np.ndarray:
        """the last cost-recording sharded frame's per-row costs over the frame's tile rows (this rank's band only)"""
        out = np.zeros(1 << 16, np.uint32)
        n = np.zeros(1, np.uint32)
        _check(lib.gsrt_debug_row_profile(self.handle, _p(out), out.size, _p(n)), self)
        return out[: int(n[0])].copy()

    @property
    def debug_streams(self) -> dict:
        """the context's streams by name, in creation order (gsrt_debug_streams; 0 = not created)"""
        out = (ctypes.c_void_p * 8)()
        n = ctypes.c_uint32()
        _check(lib.gsrt_debug_streams(self.handle, out, ctypes.byref(n)), self)
        names = ["render", "prep_hi0", "prep_lo0", "prep_hi1", "prep_lo1", "update", "comm"]
        return {k: int(out[i] or 0) for i, k in enumerate(names[: n.value])}

    @property
    def comm_stream(self) -> int:
        """the stream of sharded frames' gather + unpack (0: frames render straight into the framebuffer)"""
        return lib.gsrt_comm_stream(self.handle) or 0


class Scene:
    """gsrt_scene: Gaussians resident in HBM (params, AABBs, optional SH-3) + LBVH."""

    def __init__(self, ctx: Context, handle):
        self.ctx = ctx
        self.handle = handle
        ctx._scenes.add(self)

    @classmethod
    def from_ply(cls, ctx: Context, path, with_sh=True) -> "Scene":
        h = ctypes.c_void_p()
        _check(lib.gsrt_scene_from_ply(ctx.handle, os.fsencode(path), 1 if with_sh else 0, ctypes.byref(h)), ctx)
        return cls(ctx, h)

    @classmethod
    def from_params(cls, ctx: Context, params, aabbs, sh=None) -> "Scene":
        params = _f32(params, (-1, 12))
        n = params.shape[0]
        aabbs = _f32(aabbs, (n, 6))
        if sh is not None:
            sh = _f32(sh, (n, 48))
        h = ctypes.c_void_p()
        _check(lib.gsrt_scene_from_params(ctx.handle, _p(params), _p(aabbs), n, _p(sh), ctypes.byref(h)), ctx)
        return cls(ctx, h)

    @classmethod
    def from_model(cls, ctx: Context, center, rot, scale, opacity, sh=None) -> "Scene":
        center = _f32(center, (-1, 3))
        n = center.shape[0]
        rot, scale, opacity = _f32(rot, (n, 4)), _f32(scale, (n, 3)), _f32(opacity, (n,))
        if sh is not None:
            sh = _f32(sh, (n, 48))
        h = ctypes.c_void_p()
        _check(lib.gsrt_scene_from_model(ctx.handle, _p(center), _p(rot), _p(scale), _p(opacity), _p(sh), n,
                                         ctypes.byref(h)), ctx)
        return cls(ctx, h)

    @property
    def n(self) -> int:
        return lib.gsrt_scene_size(self.handle)

    @property
    def pages(self) -> int:
        return lib.gsrt_scene_pages(self.handle)

    def stream_pages(self, pages, params=None, aabbs=None):
        """copy the listed pages (GSRT_PAGE_GAUSSIANS Gaussians each) of the full-scene arrays params (n, 12) /
        aabbs (n, 6) into the scene: numpy arrays (page-lock them with Context.host_register for async copies)
        or device addresses (int)"""
        def arg(x, cols):
            if x is None:
                return None, None
            if isinstance(x, int):
                return ctypes.c_void_p(x), None
            a = _f32(x, (self.n, cols))
            return _p(a), a
        pp, kp = arg(params, 12)
        pa, ka = arg(aabbs, 6)
        ids = np.ascontiguousarray(pages, np.uint32).reshape(-1)
        _check(lib.gsrt_scene_stream_pages(self.handle, pp, pa, _p(ids), ids.size), self.ctx)
        del kp, ka

    def add_mesh(self, vertices, indices):
        """co-trace an indexed triangle mesh (REF frames): vertices (nv, 3), indices (nt, 3)"""
        v = _f32(vertices, (-1, 3))
        i = np.ascontiguousarray(indices, np.uint32).reshape(-1, 3)
        _check(lib.gsrt_scene_add_mesh(self.handle, _p(v), v.shape[0], _p(i), i.shape[0]), self.ctx)

    @property
    def mesh_triangles(self) -> int:
        return lib.gsrt_scene_mesh_triangles(self.handle)

    def download(self):
        params = np.zeros((self.n, 12), np.float32)
        aabbs = np.zeros((self.n, 6), np.float32)
        _check(lib.gsrt_scene_download(self.handle, _p(params), _p(aabbs)), self.ctx)
        return params, aabbs

    def build_bvh(self):
        _check(lib.gsrt_build_bvh(self.handle), self.ctx)

    def refit_bvh(self, aabbs=None):
        """aabbs: numpy (n, 6), a device address (int, e.g. a torch tensor's data_ptr()), or None"""
        if isinstance(aabbs, int):
            _check(lib.gsrt_refit_bvh(self.handle, ctypes.c_void_p(aabbs)), self.ctx)
            return
        a = None if aabbs is None else _f32(aabbs, (self.n, 6))
        _check(lib.gsrt_refit_bvh(self.handle, _p(a)), self.ctx)

    def update(self, params=None, aabbs=None):
        """Replace GaussParam (n, 12) and/or AABB (n, 6) arrays: numpy arrays or device addresses (int)."""
        def arg(x, cols):
            if x is None:
                return None, None
            if isinstance(x, int):
                return ctypes.c_void_p(x), None
            a = _f32(x, (self.n, cols))
            return _p(a), a  # keep the array alive across the call
        pp, keep_p = arg(params, 12)
        pa, keep_a = arg(aabbs, 6)
        _check(lib.gsrt_scene_update(self.handle, pp, pa), self.ctx)
        del keep_p, keep_a

    def attach(self, params=None, aabbs=None):
        """Borrow device arrays (device addresses, int; None = unchanged): frames read them in place until detach()
        (gsrt_scene_attach). The caller keeps them allocated and unchanged until then."""
        _check(lib.gsrt_scene_attach(self.handle, None if params is None else ctypes.c_void_p(params),
                                     None if aabbs is None else ctypes.c_void_p(aabbs)), self.ctx)

    def detach(self):
        """copy borrowed arrays into the scene and wait for the frames that read them (gsrt_scene_detach)"""
        _check(lib.gsrt_scene_detach(self.handle), self.ctx)

    def bvh_info(self, depth=True):
        """n_internal, root_box (the BVH fitted to the current AABBs: a pending refit runs first) and, unless
        depth=False, max_depth (a host walk over the downloaded nodes)"""
        ni = np.zeros(1, np.uint32)
        box = np.zeros(6, np.float32)
        d = np.zeros(1, np.uint32)
        _check(lib.gsrt_bvh_info(self.handle, _p(ni), _p(box), _p(d) if depth else None), self.ctx)
        return {"n_internal": int(ni[0]), "root_box": box, "max_depth": int(d[0]) if depth else None}

    def bvh_download(self):
        n = self.n
        nodes = np.zeros((max(n - 1, 0), 16), np.uint32)
        gid = np.zeros(n, np.uint32)
        morton = np.zeros(n, np.uint32)
        _check(lib.gsrt_bvh_download(self.handle, _p(nodes) if n > 1 else None, _p(gid), _p(morton)), self.ctx)
        return nodes, gid, morton

    def render(self, ubo, mode=MODE_COR, k=0, raystate=False):
        """One frame to host memory: returns (rgba[H,W,4], raystate[H,W] or None)."""
        W, H = int(ubo["width"][0]), int(ubo["height"][0])
        rgba = np.zeros((H, W, 4), np.float32)
        rs = np.zeros((H, W), RAYSTATE_DTYPE) if raystate else None
        _check(lib.gsrt_render(self.handle, _p(ubo), mode, k, _p(rgba), _p(rs)), self.ctx)
        return rgba, rs

    def render_async(self, ubo, mode=MODE_COR, k=0, d_rgba: int = 0, d_raystate: int = 0):
        """Enqueue one frame on ctx.stream; outputs are device pointers (0 = keep in the framebuffer)."""
        _check(lib.gsrt_render_async(self.handle, _p(ubo), mode, k, d_rgba or None, d_raystate or None), self.ctx)

    def render_sharded(self, ubo, mode=MODE_COR, k=0, want_image=True):
        W, H = int(ubo["width"][0]), int(ubo["height"][0])
        rgba = np.zeros((H, W, 4), np.float32) if want_image and not (mode & FLAG_OUT_DUMP8) else None
        _check(lib.gsrt_render_sharded(self.handle, _p(ubo), mode, k, _p(rgba)), self.ctx)
        return rgba

    def render_sharded_emulated(self, ubo, nranks, mode=MODE_COR, bands=None):
        """All ranks' packed tiles on this device + the rank-0 unpack (everything but the RCCL transport)."""
        W, H = int(ubo["width"][0]), int(ubo["height"][0])
        rgba = np.zeros((H, W, 4), np.float32)
        b = _bands_arg(bands)
        _check(lib.gsrt_render_sharded_emulated(self.handle, _p(ubo), mode, nranks, _p(b), _p(rgba)), self.ctx)
        return rgba

    def render_sharded_emulated_dump8(self, ubo, nranks, mode=MODE_COR, bands=None):
        """render_sharded_emulated with FLAG_OUT_DUMP8 blocks: (codes[H, W], escapes in pixel order)"""
        W, H = int(ubo["width"][0]), int(ubo["height"][0])
        codes = np.zeros((H, W), np.uint32)
        b = _bands_arg(bands)
        n = np.zeros(1, np.uint32)
        # every rank's list at its capacity (gsrt_dump8_layout: the capacity follows the largest band)
        cap = int(dump8_layout(ubo, nranks, bands, mode)["cap"]) * nranks
        esc = np.zeros(cap, ESCAPE_DTYPE)
        _check(lib.gsrt_render_sharded_emulated_dump8(self.handle, _p(ubo), mode | FLAG_OUT_DUMP8, nranks, _p(b),
                                                      _p(codes), _p(esc), esc.size, _p(n)), self.ctx)
        if int(n[0]) > esc.size:
            raise GsrtError(E_STATE, f"dump8: {int(n[0])} escapes, room for {esc.size}")
        return codes, esc[: int(n[0])].copy()

    def render_sharded_async(self, ubo, mode=MODE_COR, k=0):
        _check(lib.gsrt_render_sharded_async(self.handle, _p(ubo), mode, k), self.ctx)

    def close(self):
        if getattr(self, "handle", None):
            lib.gsrt_destroy_scene(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
