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


def long_branch(prev, ins) -> bool:
    """the compiler's long jump inside a function (a branch beyond the 16-bit offset of s_cbranch):
    s_getpc_b64 s[a:b]; s_add_u32 sa, sa, off; s_addc_u32 sb, sb, 0; s_setpc_b64 s[a:b] -- not a call or a return"""
    m = re.match(r"s_setpc_b64 (s\[\d+:\d+\])", ins)
    if not m or len(prev) < 3:
        return False
    reg = m.group(1)
    return (prev[0].startswith("s_getpc_b64 " + reg) and prev[1].startswith("s_add_u32 ") and
            prev[2].startswith("s_addc_u32 "))


def check(obj: str) -> list:
    with tempfile.TemporaryDirectory() as tmp:
        text = disassemble(obj, tmp)
    bad, func, funcs = [], "?", []
    recent = []  # the instructions before this one in the function
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            func = m.group(1)
            funcs.append(func)
            recent = []
            continue
        ins = line.strip()
        if CALLS.search(line) and not long_branch(recent, ins):
            bad.append(f"{obj}: call in {func}: {ins}")
        if ins:
            recent = (recent + [ins])[-3:]
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
