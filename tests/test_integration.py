"""INTEGRATION.md §2 as compiled code: tests/integration/vksim_shim.cpp implements the vulkan-sim entry points
lavapipe calls (gpgpusim_setDescriptor, gpgpusim_setGeometries, gpgpusim_vkCmdTraceRaysKHR;
mesa-vulkan-sim/.../gpgpusim_calls_from_mesa.h:39-59) over include/gsrt.h. The CPU test builds it with g++
against the C ABI; the GPU test drives scene 33 through it the way lavapipe would (descriptor bindings from
RayTracingPipeline.cpp:32-77, one AABB geometry per Gaussian BLAS) and checks the NextK / RayInfo buffers and
the rgba8 image against the CPU oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import gsrt
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "integration", "vksim_shim.cpp")
OUT = os.path.join(ROOT, "tests", "integration", "libvksim_shim.so")


def _build():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-fPIC", "-shared", "-o", OUT, SRC,
                        "-I", os.path.join(ROOT, "include"), "-L", os.path.dirname(gsrt.LIB_PATH), "-lgsrt",
                        "-Wl,-rpath," + os.path.dirname(gsrt.LIB_PATH)], check=True)
    return OUT


class _Geometry(ctypes.Structure):  # VkAccelerationStructureGeometryKHR with the aabbs member of its union
    _fields_ = [("sType", ctypes.c_uint32), ("pNext", ctypes.c_void_p), ("geometryType", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32),  # the union is 8-byte aligned (it holds pointers): it starts at 24
                ("a_sType", ctypes.c_uint32), ("a_pNext", ctypes.c_void_p), ("a_data", ctypes.c_void_p),
                ("a_stride", ctypes.c_uint64), ("_rest", ctypes.c_uint8 * 32), ("flags", ctypes.c_uint32)]


def test_geometry_struct_layout():
    assert ctypes.sizeof(_Geometry) == 96 and _Geometry.a_data.offset == 40 and _Geometry.flags.offset == 88


def test_shim_compiles_and_exports():
    lib = _build()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    for sym in ("gpgpusim_setDescriptor", "gpgpusim_setGeometries", "gpgpusim_vkCmdTraceRaysKHR"):
        assert f" T {sym}\n" in out, sym


@pytest.mark.gpu
def test_scene33_through_the_simulator_entry_points():
    assert ctypes.sizeof(_Geometry) == 96
    L = ctypes.CDLL(_build())
    P, u32 = ctypes.c_void_p, ctypes.c_uint32
    L.gpgpusim_setDescriptor.argtypes = [u32, u32, P, u32, u32]
    L.gpgpusim_setGeometries.argtypes = [P, u32]
    L.gpgpusim_vkCmdTraceRaysKHR.argtypes = [P, P, P, P, ctypes.c_bool, u32, u32, u32, ctypes.c_uint64]
    L.vksim_shim_status.restype = ctypes.c_int
    W = H = 16
    # Scene.cpp packing for SceneList::GaussSplat: model 0 (the triangle sphere) gets a zero GaussParam
    p, a = O.scene33()
    params = np.zeros((3, 12), np.float32)
    params[1:] = p
    ubo = O.make_ubo(O.translate(0, 0, -2), 90.0, W, H, 2.0, 1, 16)
    image = np.full((H, W, 4), 7, np.uint8)
    nextk = np.zeros((W * H, 8, 2), np.float32)
    rayinfo = np.zeros(W * H, np.dtype([("depth", "<f4"), ("gauss_num", "<i4")]))
    try:
        for binding, arr in ((2, image), (3, ubo), (12, params), (13, nextk), (14, rayinfo)):
            L.gpgpusim_setDescriptor(0, binding, arr.ctypes.data, arr.nbytes, 0)
        boxes = [np.ascontiguousarray(a[i]) for i in range(2)]  # one BLAS build per Gaussian model
        for b in boxes:
            g = _Geometry(geometryType=1, a_data=b.ctypes.data, a_stride=24)
            L.gpgpusim_setGeometries(ctypes.byref(g), 1)
        L.gpgpusim_vkCmdTraceRaysKHR(None, None, None, None, False, W, H, 1, 0)
        assert L.vksim_shim_status() == 0
        want = O.render(p, a, ubo, O.MODE_REF, want_raystate=True)["raystate"].reshape(-1)
        assert nextk.tobytes() == want["k"].tobytes()
        np.testing.assert_array_equal(rayinfo["depth"], want["depth"])
        np.testing.assert_array_equal(rayinfo["gauss_num"], want["gauss_num_raw"])
        assert not image.any()  # pixelColor is never written (GaussTracing.rgen:33,75)
        assert float(rayinfo["depth"][8 * W + 8]) == 1.0  # KAT-1
    finally:
        L.vksim_shim_reset()
