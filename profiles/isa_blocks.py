"""Per-basic-block instruction counts of one kernel in the hipcc assembly (no GPU needed):

  python profiles/isa_blocks.py [kernel-symbol-substring] [min-valu]

compiles 3dgs-raytrace_amd/csrc/gsrt_render.hip to gfx950 assembly with the product flags and prints, for every
block with at least min-valu VALU instructions, its VALU / SALU / LDS / FMA counts (the shading loop's
per-candidate blocks are the ones with ~50 FMAs: the SH-3 colour)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = sys.argv[1] if len(sys.argv) > 1 else "k_render_corILb1ELb0ELb0E"
MIN_VALU = int(sys.argv[2]) if len(sys.argv) > 2 else 20
S = "/tmp/gsrt_render_isa.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                "--offload-arch=gfx950", "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics",
                "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "--offload-device-only", "-S", "-o", S,
                os.path.join(ROOT, "3dgs-raytrace_amd", "csrc", "gsrt_render.hip")] + sys.argv[3:], check=True,
               stderr=subprocess.DEVNULL)
text = open(S).read().split("\n")
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\w*" + KERNEL + r"\w*:", l))
end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
blocks, cur = [], ["entry", []]
blocks.append(cur)
for l in text[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l.strip()) or re.match(r"^(; %bb\.\d+)", l.strip())
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    s = l.strip()
    if s and not s.startswith(";") and not s.startswith("."):
        cur[1].append(s)
tot = {"v": 0, "s": 0, "ds": 0}
for name, ins in blocks:
    v = sum(1 for s in ins if s.startswith("v_"))
    sa = sum(1 for s in ins if s.startswith("s_"))
    ds = sum(1 for s in ins if s.startswith("ds_"))
    fm = sum(1 for s in ins if re.match(r"v_fma|v_fmac|v_fmamk|v_fmaak", s))
    tot["v"] += v; tot["s"] += sa; tot["ds"] += ds
    if v >= MIN_VALU:
        print(f"{name:14s} valu {v:4d} salu {sa:3d} lds {ds:3d} fma {fm:3d}")
print("kernel total (static):", tot)
