"""INTEGRATION.md §2 as compiled code: tests/integration/vksim_shim.cpp replaces vulkan-sim's simulator library. It
exports every extern "C" entry point lavapipe calls (mesa-vulkan-sim/.../lavapipe/gpgpusim_calls_from_mesa.h:38-59)
and implements the Gaussian path over include/gsrt.h.

`Lavapipe` below plays the driver: it lays out lavapipe's own objects in memory with the byte layout the reference's
headers give (tests/golden/lvp_layout.json, measured by oracle/ref/lvp_layout_probe.c) and calls the shim in the
order the RayTracingInVulkan app drives lavapipe for --scene 33 --shader-type 6:
  allocBuffer (every buffer / image, lvp_device.c:2620,2676) -> registerShader x11 + setPipelineInfo
  (lvp_pipeline_rt.c:162,259; RayTracingPipeline.cpp:255-428) -> allocBLAS per model, setGeometries per BLAS build
  (one geometry each: triangles for the sphere, one AABB for a Gaussian; Application.cpp:253-323) -> allocTLAS,
  setGeometries(instances), pass_child_addr per instance, addTreelets (Application.cpp:325-398,
  lvp_acceleration_structure.c:1081,1391) -> setDescriptorSet(lvp_descriptor_set*) (lvp_execute.c:1551) ->
  vkCmdTraceRaysKHR(W, H, 1) (lvp_execute.c:1220).
The CPU tests check the layout mirror against the reference's headers and the scene the shim assembles from those
objects (GaussParam / AABB per Gaussian instance, the sphere mesh from the Vertices / Indices / Offsets bindings); the
GPU tests check bindings 13 (NextK) and 14 (RayInfo) byte for byte against the CPU oracle and the PPM image_store
writes."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

import gsrt
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "integration", "vksim_shim.cpp")
OUT = os.path.join(ROOT, "tests", "integration", "libvksim_shim.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")
LAYOUT = json.load(open(os.path.join(GOLDEN, "lvp_layout.json")))
ENTRY_POINTS = ("gpgpusim_setPipelineInfo", "gpgpusim_setGeometries", "gpgpusim_addTreelets", "gpgpusim_testTraversal",
                "gpgpusim_registerShader", "gpgpusim_allocBLAS", "gpgpusim_allocTLAS", "gpgpusim_allocBuffer",
                "gpgpusim_vkCmdTraceRaysKHR", "gpgpusim_setDescriptor", "gpgpusim_setDescriptorSet",
                "gpgpusim_pass_child_addr")


def _build():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-fPIC", "-shared", "-o", OUT, SRC,
                        "-I", os.path.join(ROOT, "include"), "-L", os.path.dirname(gsrt.LIB_PATH), "-lgsrt",
                        "-Wl,-rpath," + os.path.dirname(gsrt.LIB_PATH)], check=True)
    return OUT


def _lib():
    L = ctypes.CDLL(_build())
    P, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.gpgpusim_setPipelineInfo.argtypes = [P]
    L.gpgpusim_setGeometries.argtypes = [P, u32]
    L.gpgpusim_addTreelets.argtypes = [P]
    L.gpgpusim_registerShader.argtypes = [ctypes.c_char_p, u32]
    L.gpgpusim_registerShader.restype = u32
    L.gpgpusim_allocBLAS.argtypes = [P, u64, P]
    L.gpgpusim_allocTLAS.argtypes = [P, u64, P]
    L.gpgpusim_allocBuffer.argtypes = [P, u64]
    L.gpgpusim_allocBuffer.restype = P
    L.gpgpusim_vkCmdTraceRaysKHR.argtypes = [P, P, P, P, ctypes.c_bool, u32, u32, u32, u64]
    L.gpgpusim_setDescriptor.argtypes = [u32, u32, P, u32, u32]
    L.gpgpusim_setDescriptorSet.argtypes = [P]
    L.gpgpusim_pass_child_addr.argtypes = [P]
    L.vksim_shim_status.restype = ctypes.c_int
    L.vksim_shim_error.restype = ctypes.c_char_p
    L.vksim_shim_ppm_name.restype = ctypes.c_char_p
    L.vksim_shim_layout_json.restype = ctypes.c_char_p
    L.vksim_shim_counts.argtypes = [P]
    L.vksim_shim_assembly.argtypes = [P, P, P, P]
    return L


K = LAYOUT  # short alias for offsets / sizes / enum values
VERTEX = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("uv", "<f4", 2), ("material", "<i4")])  # Vertex.hpp


class Lavapipe:
    """The driver side for SceneList::GaussSplat (scene 33): models = [triangle sphere, G1, G2] (SceneList.cpp:120-125),
    their buffers packed as Assets::Scene packs them (Scene.cpp:16-170), every object lavapipe hands to the simulator
    laid out in memory as the reference's structs are. `mesh` adds the sphere (model 0)."""

    def __init__(self, L, ubo, width, height, mesh=True, nextk_init=None, lut=None):
        self.L, self.keep = L, []
        self.W, self.H = width, height
        p, a = O.scene33()
        sphere_v, sphere_i = O.scene33_mesh() if mesh else (np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32))
        self.kinds = (["mesh"] if mesh else []) + ["gauss", "gauss"]
        n_models = self.n_models = len(self.kinds)
        g0 = n_models - 2  # the Gaussians' first model index
        # Scene.cpp: vertices / indices concatenated, Offsets = {first index, first vertex} per model, one GaussParam
        # and one Gauss AABB per model (zeros for the sphere)
        verts = np.zeros(len(sphere_v), VERTEX)
        verts["pos"] = sphere_v
        verts["normal"] = 7.0
        verts["uv"] = 0.5
        self.vertices, self.indices = verts, np.ascontiguousarray(sphere_i.reshape(-1).astype(np.uint32))
        self.offsets = np.zeros((n_models, 2), np.uint32)
        self.offsets[g0:, 0] = len(self.indices)
        self.offsets[g0:, 1] = len(verts)
        self.gauss_params = np.zeros((n_models, 12), np.float32)
        self.gauss_params[g0:] = p
        self.gauss_aabbs = np.zeros((n_models, 6), np.float32)
        self.gauss_aabbs[g0:] = a
        self.ubo = np.frombuffer(ubo.tobytes(), np.uint8).copy()
        nk = np.zeros((width * height, 8, 2), np.float32)
        nk[..., 0], nk[..., 1] = 10000.0, -1.0  # Scene.cpp:38-45 default entries
        if nextk_init is not None:
            nk[...] = nextk_init
        self.nextk = nk
        self.rayinfo = np.zeros(width * height, np.dtype([("depth", "<f4"), ("gauss_num", "<i4")]))
        self.lut = np.fromfile(os.path.join(GOLDEN, "ref_explut_256_0_8.bin"), np.uint8) if lut is None else lut
        self.unused = np.zeros(64, np.uint8)
        self.out_image_mem = np.zeros(width * height * 16, np.uint8)
        self.accum_image_mem = np.zeros(width * height * 16, np.uint8)
        self.blas_mem = np.zeros(4096, np.uint8)   # one buffer for all BLASes (Application.cpp:295-300)
        self.tlas_mem = np.zeros(1024, np.uint8)
        self.instances = np.zeros((n_models, 64), np.uint8)
        self.mesh = mesh

    def _hold(self, obj):
        self.keep.append(obj)
        return obj

    @staticmethod
    def addr(arr):
        return arr.ctypes.data

    def bind_memory(self):
        """lvp_BindBufferMemory2 / lvp_BindImageMemory2: every buffer and image is aliased by the simulator."""
        for arr in (self.vertices, self.indices, self.offsets, self.gauss_aabbs, self.gauss_params, self.nextk,
                    self.rayinfo, self.lut, self.ubo, self.blas_mem, self.tlas_mem, self.instances, self.unused,
                    self.out_image_mem, self.accum_image_mem):
            alias = self.L.gpgpusim_allocBuffer(self.addr(arr), arr.nbytes)
            assert alias == self.addr(arr)

    def create_pipeline(self, tmpdir):
        """RayTracingPipeline.cpp shader type 6: 11 stages, 7 groups; lavapipe registers stage i's PTX as id i."""
        stage_bits = [0x100, 0x800, 0x400, 0x400, 0x400, 0x400, 0x400, 0x1000, 0x1000, 0x1000, 0x1000]
        mesa = {0x100: 8, 0x800: 11, 0x400: 10, 0x1000: 12}  # VkShaderStageFlagBits -> gl_shader_stage
        names = {8: "RAYGEN", 11: "MISS", 10: "CLOSEST_HIT", 12: "INTERSECTION"}
        for i, bit in enumerate(stage_bits):
            path = os.path.join(str(tmpdir), f"MESA_SHADER_{names[mesa[bit]]}_{i}.ptx").encode()
            assert self.L.gpgpusim_registerShader(path, mesa[bit]) == i  # lvp_pipeline_rt.c:163
        stages = np.zeros(len(stage_bits), np.dtype([("sType", "<u4"), ("pad0", "<u4"), ("pNext", "<u8"),
                                                     ("flags", "<u4"), ("stage", "<u4"), ("module", "<u8"),
                                                     ("pName", "<u8"), ("pSpec", "<u8")]))
        assert stages.itemsize == K["sizeof VkPipelineShaderStageCreateInfo"]
        stages["stage"] = stage_bits
        U = 0xFFFFFFFF
        gdt = np.dtype([("sType", "<u4"), ("pad0", "<u4"), ("pNext", "<u8"), ("type", "<u4"), ("general", "<u4"),
                        ("chit", "<u4"), ("ahit", "<u4"), ("isect", "<u4"), ("pad1", "<u4"), ("replay", "<u8")])
        assert gdt.itemsize == K["sizeof VkRayTracingShaderGroupCreateInfoKHR"]
        assert gdt.fields["isect"][1] == K["VkRayTracingShaderGroupCreateInfoKHR.intersectionShader"]
        GEN, TRI, PROC = (K["VK_RAY_TRACING_SHADER_GROUP_TYPE_GENERAL_KHR"],
                          K["VK_RAY_TRACING_SHADER_GROUP_TYPE_TRIANGLES_HIT_GROUP_KHR"],
                          K["VK_RAY_TRACING_SHADER_GROUP_TYPE_PROCEDURAL_HIT_GROUP_KHR"])
        groups = np.array([(0, 0, 0, GEN, 0, U, U, U, 0, 0), (0, 0, 0, GEN, 1, U, U, U, 0, 0),
                           (0, 0, 0, TRI, U, 2, U, U, 0, 0), (0, 0, 0, PROC, U, 3, U, 7, 0, 0),
                           (0, 0, 0, PROC, U, 4, U, 8, 0, 0), (0, 0, 0, PROC, U, 5, U, 9, 0, 0),
                           (0, 0, 0, PROC, U, 6, U, 10, 0, 0)], gdt)
        info = np.zeros(K["sizeof VkRayTracingPipelineCreateInfoKHR"], np.uint8)
        info[K["VkRayTracingPipelineCreateInfoKHR.stageCount"]:][:4] = np.frombuffer(np.uint32(11).tobytes(), np.uint8)
        info[K["VkRayTracingPipelineCreateInfoKHR.pStages"]:][:8] = np.frombuffer(
            np.uint64(self.addr(stages)).tobytes(), np.uint8)
        info[K["VkRayTracingPipelineCreateInfoKHR.groupCount"]:][:4] = np.frombuffer(np.uint32(7).tobytes(), np.uint8)
        info[K["VkRayTracingPipelineCreateInfoKHR.pGroups"]:][:8] = np.frombuffer(
            np.uint64(self.addr(groups)).tobytes(), np.uint8)
        self.L.gpgpusim_setPipelineInfo(self.addr(info))  # the app's structs only live during the call

    def _geometry(self, gtype, data_off_fields):
        g = np.zeros(K["sizeof VkAccelerationStructureGeometryKHR"], np.uint8)
        g[K["VkAccelerationStructureGeometryKHR.geometryType"]:][:4] = np.frombuffer(np.uint32(gtype).tobytes(), np.uint8)
        base = K["VkAccelerationStructureGeometryKHR.geometry"]
        for off, val, dt in data_off_fields:
            g[base + off:][:np.dtype(dt).itemsize] = np.frombuffer(np.array(val, dt).tobytes(), np.uint8)
        return self._hold(g)

    def build_acceleration_structures(self):
        n_models = self.n_models
        blas_roots = [self.addr(self.blas_mem) + 256 * m for m in range(n_models)]
        for m in range(n_models):  # lvp_CreateAccelerationStructureKHR per BLAS (Application.cpp:315-322)
            self.L.gpgpusim_allocBLAS(blas_roots[m], self.blas_mem.nbytes, blas_roots[m])
        for m in range(n_models):  # the builds, in the same order; the AABB data address is the buffer's base
            if self.kinds[m] == "mesh":
                g = self._geometry(K["VK_GEOMETRY_TYPE_TRIANGLES_KHR"], [
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.vertexFormat"],
                     K["VK_FORMAT_R32G32B32_SFLOAT"], "<u4"),
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.vertexData"], self.addr(self.vertices), "<u8"),
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.vertexStride"], VERTEX.itemsize, "<u8"),
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.maxVertex"], len(self.vertices), "<u4"),
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.indexType"], K["VK_INDEX_TYPE_UINT32"], "<u4"),
                    (K["VkAccelerationStructureGeometryTrianglesDataKHR.indexData"], self.addr(self.indices), "<u8")])
            else:
                g = self._geometry(K["VK_GEOMETRY_TYPE_AABBS_KHR"], [
                    (K["VkAccelerationStructureGeometryAabbsDataKHR.data"], self.addr(self.gauss_aabbs), "<u8"),
                    (K["VkAccelerationStructureGeometryAabbsDataKHR.stride"], 24, "<u8")])
            self.L.gpgpusim_setGeometries(self.addr(g), 1)
        # TLAS: one instance per model, identity transform, custom index = model, SBT offset = hit group
        # (0 triangles, 4 Gauss; Application.cpp:339-367), reference = the BLAS device address
        for m in range(n_models):
            inst = np.zeros(64, np.uint8)
            tr = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], np.float32)
            inst[:48] = np.frombuffer(tr.tobytes(), np.uint8)
            hit = 0 if self.kinds[m] == "mesh" else 4
            inst[48:52] = np.frombuffer(np.uint32(m | (0xFF << 24)).tobytes(), np.uint8)
            inst[52:56] = np.frombuffer(np.uint32(hit).tobytes(), np.uint8)
            inst[K["VkAccelerationStructureInstanceKHR.accelerationStructureReference"]:][:8] = np.frombuffer(
                np.uint64(blas_roots[m]).tobytes(), np.uint8)
            self.instances[m] = inst
        tlas_root = self.addr(self.tlas_mem) + 128
        self.L.gpgpusim_allocTLAS(tlas_root, self.tlas_mem.nbytes, tlas_root)
        g = self._geometry(K["VK_GEOMETRY_TYPE_INSTANCES_KHR"], [
            (K["VkAccelerationStructureGeometryInstancesDataKHR.data"], self.addr(self.instances), "<u8")])
        self.L.gpgpusim_setGeometries(self.addr(g), 1)
        for m in range(n_models):
            self.L.gpgpusim_pass_child_addr(blas_roots[m] - self.addr(self.tlas_mem))
        self.L.gpgpusim_addTreelets(tlas_root)
        self.tlas_root = tlas_root

    def descriptor_set(self):
        """lvp_descriptor_set_layout + lvp_descriptor_set for RayTracingPipeline.cpp:32-77's 16 bindings."""
        n = 16
        layout = self._hold(np.zeros(K["struct lvp_descriptor_set_layout.binding"] +
                                     n * K["sizeof struct lvp_descriptor_set_binding_layout"], np.uint8))
        layout[K["struct lvp_descriptor_set_layout.binding_count"]:][:2] = np.frombuffer(np.uint16(n).tobytes(), np.uint8)
        dsz = K["sizeof struct lvp_descriptor"]
        dset = self._hold(np.zeros(K["struct lvp_descriptor_set.descriptors"] + n * dsz, np.uint8))
        dset[K["struct lvp_descriptor_set.layout"]:][:8] = np.frombuffer(np.uint64(self.addr(layout)).tobytes(), np.uint8)
        SI, UB, SB, AS = (K["VK_DESCRIPTOR_TYPE_STORAGE_IMAGE"], K["VK_DESCRIPTOR_TYPE_UNIFORM_BUFFER"],
                          K["VK_DESCRIPTOR_TYPE_STORAGE_BUFFER"], K["VK_DESCRIPTOR_TYPE_ACCELERATION_STRUCTURE_KHR"])
        out_img = self._image(self.out_image_mem)
        acc_img = self._image(self.accum_image_mem)
        bufs = {4: self.vertices, 5: self.indices, 6: self.unused, 7: self.offsets, 9: self.unused, 10: self.unused,
                11: self.unused, 12: self.gauss_params, 13: self.nextk, 14: self.rayinfo, 15: self.lut}
        for b in range(n):
            # the descriptor array is in a different order than the bindings, as descriptor_index allows
            di = (b * 5) % n
            bl = K["struct lvp_descriptor_set_layout.binding"] + b * K["sizeof struct lvp_descriptor_set_binding_layout"]
            typ = {0: AS, 1: SI, 2: SI, 3: UB, 8: 1}.get(b, SB)  # 8: combined image sampler (no textures)
            layout[bl + K["struct lvp_descriptor_set_binding_layout.descriptor_index"]:][:2] = np.frombuffer(
                np.uint16(di).tobytes(), np.uint8)
            layout[bl + K["struct lvp_descriptor_set_binding_layout.type"]:][:4] = np.frombuffer(
                np.uint32(typ).tobytes(), np.uint8)
            d = K["struct lvp_descriptor_set.descriptors"] + di * dsz
            dset[d + K["struct lvp_descriptor.type"]:][:4] = np.frombuffer(np.uint32(typ).tobytes(), np.uint8)

            def put(off, val, dt):
                dset[d + off:][:np.dtype(dt).itemsize] = np.frombuffer(np.array(val, dt).tobytes(), np.uint8)
            if typ == AS:  # info.ubo.pmem = accel->address.bo, buffer_offset = address.offset (lvp_descriptor_set.c:642)
                put(K["struct lvp_descriptor.info.ubo.pmem"], self.addr(self.tlas_mem), "<u8")
                put(K["struct lvp_descriptor.info.ubo.buffer_offset"], self.tlas_root - self.addr(self.tlas_mem), "<u4")
            elif typ == SI:
                put(K["struct lvp_descriptor.info.image_view.image"], self.addr(out_img if b == 2 else acc_img), "<u8")
            elif typ == UB:
                put(K["struct lvp_descriptor.info.ubo.pmem"], self.addr(self.ubo), "<u8")
                put(K["struct lvp_descriptor.info.ubo.buffer_size"], self.ubo.nbytes, "<u4")
            elif typ == SB:
                arr = bufs[b]
                put(K["struct lvp_descriptor.info.ssbo.pmem"], self.addr(arr), "<u8")
                put(K["struct lvp_descriptor.info.ssbo.buffer_size"], arr.nbytes, "<u4")
        return dset

    def _image(self, mem):
        img = self._hold(np.zeros(256, np.uint8))  # struct lvp_image: vk.format / vk.extent / vk.tiling
        img[K["struct lvp_image.vk.format"]:][:4] = np.frombuffer(
            np.uint32(K["VK_FORMAT_R32G32B32A32_SFLOAT"]).tobytes(), np.uint8)
        img[K["struct lvp_image.vk.extent"]:][:12] = np.frombuffer(np.array([self.W, self.H, 1], np.uint32).tobytes(),
                                                                   np.uint8)
        return img

    def setup(self, tmpdir):
        self.bind_memory()
        self.create_pipeline(tmpdir)
        self.build_acceleration_structures()
        dset = self.descriptor_set()
        self.L.gpgpusim_setDescriptorSet(self.addr(dset))

    def trace(self):
        sbt = self._hold(np.zeros(4, np.uint64))
        self.L.gpgpusim_vkCmdTraceRaysKHR(self.addr(sbt), self.addr(sbt), self.addr(sbt), self.addr(sbt), False,
                                          self.W, self.H, 1, 0)
        return self.L.vksim_shim_status(), self.L.vksim_shim_error().decode()

    def counts(self):
        c = np.zeros(7, np.uint32)
        self.L.vksim_shim_counts(c.ctypes.data)
        return c

    def assembly(self):
        c = self.counts()
        p = np.zeros((c[0], 12), np.float32)
        a = np.zeros((c[0], 6), np.float32)
        v = np.zeros((c[6], 3), np.float32)
        i = np.zeros((c[1], 3), np.uint32)
        self.L.vksim_shim_assembly(p.ctypes.data, a.ctypes.data, v.ctypes.data, i.ctypes.data)
        return p, a, v, i


def _kat1_ubo(W=16, H=16):
    return O.make_ubo(O.translate(0, 0, -2), 90.0, W, H, 2.0, 1, 16)


@pytest.fixture
def shim():
    L = _lib()
    L.vksim_shim_reset()
    yield L
    L.vksim_shim_reset()


# ---------------------------------------------------------------------------------------------------------- CPU
def test_shim_compiles_and_exports_every_entry_point():
    lib = _build()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    for sym in ENTRY_POINTS:
        assert f" T {sym}\n" in out, sym


def test_layout_mirror_matches_reference_headers(shim):
    mirror = json.loads(shim.vksim_shim_layout_json().decode())
    for key, val in mirror.items():
        assert LAYOUT[key] == val, (key, LAYOUT[key], val)
    assert len(mirror) >= 30


def test_register_shader_ids(shim, tmp_path):
    """vulkan-sim's id is the file name's last _<n> (vulkan_ray_tracing.cc:1346-1356)."""
    for i, name in enumerate(["MESA_SHADER_RAYGEN_0.ptx", "/x/y/MESA_SHADER_MISS_1.ptx", "a/MESA_SHADER_CLOSEST_HIT_2.ptx"]):
        assert shim.gpgpusim_registerShader(name.encode(), 8) == i
    assert shim.gpgpusim_registerShader(b"/p/MESA_SHADER_INTERSECTION_10.ptx", 12) == 10


@pytest.mark.parametrize("mesh", [True, False])
def test_scene33_assembled_from_driver_objects(shim, tmp_path, monkeypatch, mesh):
    """Without a GPU the trace stops at gsrt_create; the scene it assembled from the driver's objects before that is
    scene 33: the two Gaussians (GaussParam + AABB per Gauss instance, model order) and the sphere mesh."""
    monkeypatch.chdir(tmp_path)
    lp = Lavapipe(shim, _kat1_ubo(), 16, 16, mesh=mesh)
    lp.setup(tmp_path)
    status, err = lp.trace()
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert status == gsrt.E_DEVICE, err
    c = lp.counts()
    assert c[2] == 11 and c[4] == lp.n_models and c[5] == lp.n_models and c[3] == 15
    p, a, v, i = lp.assembly()
    pw, aw = O.scene33()
    np.testing.assert_array_equal(p, pw)
    np.testing.assert_array_equal(a, aw)
    if mesh:
        sv, si = O.scene33_mesh()
        np.testing.assert_array_equal(v, sv)
        np.testing.assert_array_equal(i, si)
    else:
        assert c[1] == 0 and c[6] == 0
    assert os.path.exists("image.binary") and os.path.getsize("image.binary") == 0  # opened, never written


def test_bad_lut_is_refused(shim, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    lut = np.fromfile(os.path.join(GOLDEN, "ref_explut_256_0_8.bin"), np.uint8)
    lut[100] ^= 1
    lp = Lavapipe(shim, _kat1_ubo(), 16, 16, lut=lut)
    lp.setup(tmp_path)
    status, err = lp.trace()
    assert status == gsrt.E_ARG and "binding 15" in err


def test_second_descriptor_set_is_ignored(shim, tmp_path, monkeypatch):
    """vulkan-sim keeps the first set it is given (vulkan_ray_tracing.cc:1264-1273)."""
    monkeypatch.chdir(tmp_path)
    lp = Lavapipe(shim, _kat1_ubo(), 16, 16)
    lp.setup(tmp_path)
    junk = np.zeros(2048, np.uint8)
    shim.gpgpusim_setDescriptorSet(junk.ctypes.data)
    lp.trace()
    assert lp.counts()[0] == 2


# ---------------------------------------------------------------------------------------------------------- GPU
def _ppm_lines(path):
    with open(path) as f:
        return f.read()


@pytest.mark.gpu
def test_scene33_kat1_through_lavapipe_call_sequence(shim, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    W = H = 16
    ubo = _kat1_ubo(W, H)
    lp = Lavapipe(shim, ubo, W, H)
    lp.setup(tmp_path)
    status, err = lp.trace()
    assert status == 0, err
    p, a = O.scene33()
    want = O.render(p, a, ubo, O.MODE_REF, want_raystate=True, tris=O.mesh_triangles(*O.scene33_mesh()))["raystate"]
    want = want.reshape(-1)
    assert lp.nextk.tobytes() == want["k"].tobytes()
    np.testing.assert_array_equal(lp.rayinfo["depth"], want["depth"])
    np.testing.assert_array_equal(lp.rayinfo["gauss_num"], want["gauss_num_raw"])
    assert float(lp.rayinfo["depth"][8 * W + 8]) == 1.0  # KAT-1
    assert not lp.out_image_mem.any()  # the lavapipe build's image_store writes no pixels (:2306)
    name = shim.vksim_shim_ppm_name().decode()
    assert name.endswith("-SCENE.ppm")
    assert _ppm_lines(name) == "P3\n16 16\n255\n" + "  0   0   0\n" * 256


@pytest.mark.gpu
@pytest.mark.parametrize("eye,center", [((200.0, 200.0, 3.0), (200.0, 200.0, 0.0)),
                                        ((4.0, 4.0, 2.0), (200.0, 200.0, 0.0))])
def test_scene33_sphere_camera_and_stale_alphas(shim, tmp_path, monkeypatch, eye, center):
    """A camera that sees the triangle sphere (mesh rebuilt from bindings 4/5/7), then a second trace with another
    camera: NextK slots no insert reached keep the alpha the buffer held (rgen:54-57 resets only depths)."""
    monkeypatch.chdir(tmp_path)
    W, H = 64, 48
    mv = O.lookat(eye, center)
    ubo = O.make_ubo(mv, 90.0, W, H, 2.0, 1, 16)
    init = np.zeros((W * H, 8, 2), np.float32)
    init[..., 0] = 3.0
    init[..., 1] = 0.25
    lp = Lavapipe(shim, ubo, W, H, nextk_init=init)
    lp.setup(tmp_path)
    status, err = lp.trace()
    assert status == 0, err
    assert lp.counts()[1] == 1024
    p, a = O.scene33()
    tris = O.mesh_triangles(*O.scene33_mesh())
    want = O.render(p, a, ubo, O.MODE_REF, want_raystate=True, tris=tris)["raystate"].reshape(-1)
    assert (want["trans"] == 0.0).any(), "the camera must see the sphere"
    k = want["k"].copy()
    k[..., 1] = np.where(k[..., 1] == -1.0, 0.25, k[..., 1])
    assert lp.nextk.tobytes() == k.tobytes()
    np.testing.assert_array_equal(lp.rayinfo["depth"], want["depth"])
    np.testing.assert_array_equal(lp.rayinfo["gauss_num"], want["gauss_num_raw"])
    # second frame: the app updates its UBO in place (Application::UpdateUniformBuffer) and traces again
    before = lp.nextk.copy()
    ubo2 = O.make_ubo(O.translate(0, 0, -2), 90.0, W, H, 2.0, 1, 16)
    lp.ubo[:] = np.frombuffer(ubo2.tobytes(), np.uint8)
    status, err = lp.trace()
    assert status == 0, err
    want2 = O.render(p, a, ubo2, O.MODE_REF, want_raystate=True, tris=tris)["raystate"].reshape(-1)
    k2 = want2["k"].copy()
    k2[..., 1] = np.where(k2[..., 1] == -1.0, before[..., 1], k2[..., 1])
    assert lp.nextk.tobytes() == k2.tobytes()
    np.testing.assert_array_equal(lp.rayinfo["gauss_num"], want2["gauss_num_raw"])
