"""Build check (Makefile): the gfx950 code objects hold no call instructions.

  python3 tools/check_isa.py [--arch gfx950] build/gsrt_render.o [more .o files]

Every device function must be inlined into its kernel (GSRT_INLINE, gsrt_device.hpp): the kernels re-read their
arguments through the kernarg segment pointer (kargs(), gsrt_render.hip), which is only defined inside a kernel -- an
outlined function reading it faulted once (an experiment build, profiles/r04/persist_ab.txt). So a call
(s_swappc_b64 / s_setpc_b64) anywhere in the device code fails the build, naming the function it sits in and the
outlined functions present."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
ARCH = "gfx950"  # the Makefile passes its $(ARCH) with --arch
CALLS = re.compile(r"\b(s_swappc_b64|s_setpc_b64|s_call_b64)\b")


def disassemble(obj: str, tmp: str) -> str:
    fat = os.path.join(tmp, "fat.bin")
    dev = os.path.join(tmp, "dev.co")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, obj], check=True, stderr=subprocess.DEVNULL)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--" + ARCH, "--output=" + dev], check=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", dev], check=True, capture_output=True,
                          text=True).stdout


def check(obj: str) -> list:
    with tempfile.TemporaryDirectory() as tmp:
        text = disassemble(obj, tmp)
    bad, func, funcs = [], "?", []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            func = m.group(1)
            funcs.append(func)
            continue
        if CALLS.search(line):
            bad.append(f"{obj}: call in {func}: {line.strip()}")
    if bad:
        # kernels are the symbols the runtime launches; anything else with code is an outlined function
        outlined = [f for f in funcs if not re.match(r"^_ZN4gsrt\d+k_", f) and not f.startswith("k_")]
        bad.append(f"{obj}: outlined functions: {', '.join(outlined) or 'none'}")
    return bad


def main(objs) -> int:
    errs = [e for o in objs for e in check(o)]
    for e in errs:
        print("check_isa:", e, file=sys.stderr)
    return 1 if errs else 0


if __name__ == "__main__":
    args = sys.argv[1:]
    if len(args) >= 2 and args[0] == "--arch":
        ARCH = args[1]
        args = args[2:]
    sys.exit(main(args))
