"""Build checks (CPU, hipcc cross-compiles gfx950): tools/check_isa.py, which the Makefile runs on every HIP object of
libgsrt.so, fails on a call instruction in device code -- a device function the compiler outlined, such as one that
reads the kernarg segment pointer outside a kernel (the kargs() pattern of gsrt_render.hip, which faulted once when a
tile body was outlined: profiles/r04/persist_ab.txt) -- and passes the product objects."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3dgs-raytrace_amd")
CHECK = os.path.join(PKG, "tools", "check_isa.py")
HIPCC = "/opt/rocm/bin/hipcc"

PROBE = r'''
#include <hip/hip_runtime.h>
struct Args { int x; float* out; };
__device__ INLINE float arg_x() {
    const __attribute__((address_space(4))) Args* p =
        (const __attribute__((address_space(4))) Args*)__builtin_amdgcn_kernarg_segment_ptr();
    return (float)p->x;
}
__device__ INLINE void body(float* o) { o[threadIdx.x] = arg_x(); }
__global__ void k_probe(Args a) { body(a.out); }
'''


def _probe(tmp_path, inline: str) -> str:
    src = tmp_path / "probe.hip"
    src.write_text(PROBE.replace("INLINE", inline))
    obj = tmp_path / "probe.o"
    subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "-c", "-o", str(obj), str(src)], check=True,
                   capture_output=True)
    return str(obj)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_check_isa_rejects_an_outlined_kernarg_reader(tmp_path):
    bad = subprocess.run([sys.executable, CHECK, _probe(tmp_path, "__attribute__((noinline))")], capture_output=True,
                         text=True)
    assert bad.returncode == 1
    assert "call in" in bad.stderr and "k_probe" in bad.stderr and "outlined functions" in bad.stderr
    good = subprocess.run([sys.executable, CHECK, _probe(tmp_path, "__attribute__((always_inline)) inline")],
                          capture_output=True, text=True)
    assert good.returncode == 0, good.stderr


def test_product_objects_pass_check_isa():
    objs = [os.path.join(PKG, "build", f) for f in ("gsrt_render.o", "gsrt_scene.o", "gsrt_lbvh.o", "gsrt_mesh_trace.o")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library not built")
    r = subprocess.run([sys.executable, CHECK] + objs, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
