"""Generates tests/golden/ref_explut_256_0_8.bin: the exp LUT the REFERENCE computes, by running its own
header-only generator (RayTracingInVulkan/src/Utilities/ExpLUT.hpp:10-24, generateExpLUT(256, 0, 8) as
Scene.cpp:47 calls it) compiled unchanged from /root/reference by `make -C oracle ref` (oracle/ref/explut_dump.cpp
includes it). 256 x {float k, float b}, little-endian. Run in the container that holds /root/reference:

  python tests/golden/make_ref_explut.py
"""
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "ref_explut_256_0_8.bin")

subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
subprocess.run([os.path.join(ROOT, "oracle", "_ref", "explut_dump"), OUT], check=True)
with open(OUT, "rb") as f:
    data = f.read()
assert len(data) == 2048
print(OUT, hashlib.sha256(data).hexdigest())
