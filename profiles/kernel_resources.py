"""VGPR / SGPR / scratch / LDS / occupancy of every kernel in one HIP source, from the gfx950 assembly
metadata (no GPU needed):

  python profiles/kernel_resources.py [source.hip] [filter]

Compiles with the product flags (3dgs-raytrace_amd/Makefile DEVFLAGS) and prints one line per kernel."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "3dgs-raytrace_amd", "csrc", "gsrt_render.hip")
FILT = sys.argv[2] if len(sys.argv) > 2 else ""
S = "/tmp/gsrt_resources.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                "--offload-arch=gfx950", "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics",
                "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "--offload-device-only", "-S", "-o", S,
                SRC], check=True, stderr=subprocess.DEVNULL)
text = open(S).read()
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", text, re.S):
    name, body = m.group(1), m.group(2)
    if not name.startswith("_Z") or FILT not in name:
        continue
    def get(key):
        k = re.search(r"\." + key + r":\s+(\d+)", body)
        return int(k.group(1)) if k else -1
    print(f"{name[:70]:70s} vgpr {get('vgpr_count'):4d} sgpr {get('sgpr_count'):3d} "
          f"scratch {get('private_segment_fixed_size'):5d} lds {get('group_segment_fixed_size'):6d} "
          f"spill v {get('vgpr_spill_count')} s {get('sgpr_spill_count')}")
