"""ctypes wrapper over the CPU oracle (oracle/_build/libgsrt_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker. The product never imports it.
See gsrt_oracle.c for the reference file:line each function restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgsrt_oracle.so")

MODE_REF = 0
MODE_COR = 1
FLAG_LUT = 0x100
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
assert UBO_DTYPE.itemsize == 320 and RAYSTATE_DTYPE.itemsize == 80

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        u32, f32 = ctypes.c_uint32, ctypes.c_float
        L.or_make_ubo.argtypes = [P, f32, u32, u32, f32, u32, u32, P]
        L.or_lookat_rh.argtypes = [P, P, P, P]
        L.or_gauss_from_model.argtypes = [u32, P, P, P, P, P, P]
        L.or_exp_lut.argtypes = [P]
        L.or_exp_neg.argtypes = [f32]
        L.or_exp_neg.restype = f32
        L.or_linear_exp.argtypes = [P, f32]
        L.or_linear_exp.restype = f32
        L.or_synth_cloud.argtypes = [u32, u32, u32, ctypes.c_int, P, P, P, P, P]
        L.or_bvh_build.argtypes = [P, u32]
        L.or_bvh_build.restype = P
        L.or_bvh_free.argtypes = [P]
        L.or_render.argtypes = [P, P, P, u32, P, P, u32, u32, u32, u32, P, P, P]
        L.or_render.restype = ctypes.c_int
        L.or_render_mesh.argtypes = [P, P, P, u32, P, P, u32, P, u32, u32, u32, u32, P, P, P]
        L.or_render_mesh.restype = ctypes.c_int
        L.or_sphere_mesh.argtypes = [P, f32, P, P]
        L.or_sizeof_ubo.restype = u32
        L.or_sizeof_raystate.restype = u32
        assert L.or_sizeof_ubo() == 320 and L.or_sizeof_raystate() == 80
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def lookat(eye, center, up=(0.0, 1.0, 0.0)) -> np.ndarray:
    out = np.zeros(16, np.float32)
    e, c, u = (np.asarray(v, np.float32) for v in (eye, center, up))
    lib().or_lookat_rh(_p(e), _p(c), _p(u), _p(out))
    return out


def translate(x, y, z) -> np.ndarray:
    m = np.eye(4, dtype=np.float32)
    m[3, :3] = (x, y, z)  # column 3 (column-major storage as [col][row])
    return m.reshape(16)


def make_ubo(init_mv, fovy_deg, width, height, focus_distance=1.0, samples=1, bounces=16) -> np.ndarray:
    ubo = np.zeros(1, UBO_DTYPE)
    mv = np.ascontiguousarray(init_mv, np.float32).reshape(16)
    lib().or_make_ubo(_p(mv), fovy_deg, width, height, focus_distance, samples, bounces, _p(ubo))
    return ubo


def gauss_from_model(center, rot, scale, opacity):
    center = np.ascontiguousarray(center, np.float32).reshape(-1, 3)
    n = center.shape[0]
    rot = np.ascontiguousarray(rot, np.float32).reshape(n, 4)
    scale = np.ascontiguousarray(scale, np.float32).reshape(n, 3)
    opacity = np.ascontiguousarray(opacity, np.float32).reshape(n)
    params = np.zeros((n, 12), np.float32)
    aabbs = np.zeros((n, 6), np.float32)
    lib().or_gauss_from_model(n, _p(center), _p(rot), _p(scale), _p(opacity), _p(params), _p(aabbs))
    return params, aabbs


def exp_lut() -> np.ndarray:
    out = np.zeros(512, np.float32)
    lib().or_exp_lut(_p(out))
    return out


def exp_neg(x: float) -> float:
    return lib().or_exp_neg(x)


def synth_cloud(kind, n, seed=42, with_sh=False):
    c = np.zeros((n, 3), np.float32)
    r = np.zeros((n, 4), np.float32)
    s = np.zeros((n, 3), np.float32)
    o = np.zeros(n, np.float32)
    sh = np.zeros((n, 16, 3), np.float32) if with_sh else None
    lib().or_synth_cloud(kind, n, seed, int(with_sh), _p(c), _p(r), _p(s), _p(o), _p(sh))
    return c, r, s, o, sh


class Bvh:
    def __init__(self, aabbs):
        self._aabbs = np.ascontiguousarray(aabbs, np.float32)
        self.handle = lib().or_bvh_build(_p(self._aabbs), self._aabbs.shape[0])

    def __del__(self):
        if getattr(self, "handle", None):
            lib().or_bvh_free(self.handle)
            self.handle = None


def sphere_mesh(center, radius):
    """Model::CreateSphere geometry (Model.cpp:566-629): vertices (561, 3) f32, indices (1024, 3) u32"""
    c = np.asarray(center, np.float32)
    v = np.zeros((561, 3), np.float32)
    i = np.zeros((1024, 3), np.uint32)
    lib().or_sphere_mesh(_p(c), float(radius), _p(v), _p(i))
    return v, i


def mesh_triangles(vertices, indices) -> np.ndarray:
    """(nt, 9) f32: p0 p1 p2 per triangle"""
    v = np.asarray(vertices, np.float32).reshape(-1, 3)
    return np.ascontiguousarray(v[np.asarray(indices, np.int64).reshape(-1, 3)].reshape(-1, 9))


def render(params, aabbs, ubo, mode, sh=None, bvh: Bvh | None = None, threads=None,
           rows=None, want_raystate=False, want_stats=False, tris=None):
    """Render (a band of rows of) one frame. Returns dict with rgba/raystate/stats (full-frame arrays).
    tris: (nt, 9) triangles co-traced in REF mode (mesh_triangles), or None."""
    params = np.ascontiguousarray(params, np.float32)
    aabbs = np.ascontiguousarray(aabbs, np.float32)
    n = params.shape[0]
    W, H = int(ubo["width"][0]), int(ubo["height"][0])
    r0, r1 = rows if rows is not None else (0, H)
    rgba = np.zeros((H, W, 4), np.float32)
    rs = np.zeros((H, W), RAYSTATE_DTYPE) if want_raystate else None
    st = np.zeros((H, W, 4), np.uint32) if want_stats else None
    if sh is not None:
        sh = np.ascontiguousarray(sh, np.float32)
    threads = threads or os.cpu_count() or 1
    tr = None if tris is None else np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    rc = lib().or_render_mesh(_p(params), _p(aabbs), _p(sh), n, bvh.handle if bvh else None, _p(tr),
                              0 if tr is None else tr.shape[0], _p(ubo), mode, threads, r0, r1, _p(rgba), _p(rs),
                              _p(st))
    if rc != 0:
        raise ValueError(f"or_render failed: {rc}")
    return {"rgba": rgba, "raystate": rs, "stats": st}


def scene33_mesh():
    """the triangle sphere of SceneList::GaussSplat (SceneList.cpp:123): CreateSphere((200,200,0), 0.5)"""
    return sphere_mesh((200.0, 200.0, 0.0), 0.5)


def scene33():
    """SceneList::GaussSplat (SceneList.cpp:108-128): the two Gaussian models (the far triangle
    sphere at (200,200,0) is a mesh, scene33_mesh(); no ray of the scene's own 16x16 camera reaches it)."""
    center = [[0, 0, 5], [0, 0, 3]]
    rot = [[1, 0, 0, 0], [1, 0, 0, 0]]
    scale = [[1, 1, 1], [2, 2, 2]]
    opacity = [0.9, 0.9]
    return gauss_from_model(center, rot, scale, opacity)
