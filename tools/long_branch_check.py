"""Build-time guard against the gfx950 long-branch miscompile behind round 1's
"out-of-line glv_mul never terminates" (DESIGN.md §9).

Root cause (ROCm 7.2 / LLVM AMDGPU backend): when a NON-kernel device function
is larger than the s_cbranch range (+-2^15 dwords), branch relaxation rewrites
far branches as  s_getpc_b64 s[30:31]; s_add/addc; s_setpc_b64 s[30:31]  --
using s[30:31], the register pair that holds the function's RETURN ADDRESS in
the AMDGPU calling convention, without saving it.  The function's final
`s_setpc_b64 s[30:31]` then jumps to the last far-branch target instead of the
caller (in the round-1 build: to its own return block, an endless loop).  Kernel
entry points have no return address, so the same code inlined into a kernel is
correct.  Our point arithmetic inlines 136-MAD products (~1 KB of code each), so
an out-of-line scalar multiplication crosses the range; the inline-asm product
blocks also make the backend's size estimate (amdgpu-long-branch-factor) too
small to reserve a dedicated register pair up front.

Reproducer: tools/experiments/glv_noinline_repro.hip (a __noinline__ wrapper of
glv_mul): compile it and this check reports the function.

This script compiles every .hip source device-only, disassembles the gfx950
code objects and FAILS if any non-kernel function writes s[30:31] with
s_getpc_b64 (the far-branch expansion); kernels are exempt.
    python tools/long_branch_check.py [sources...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def functions(dis):
    """(name, body lines) of every function in an llvm-objdump listing"""
    cur, body = None, []
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(line)
    if cur:
        yield cur, body


def check(src, tmp):
    obj = os.path.join(tmp, os.path.basename(src) + ".o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                           "--no-gpu-bundle-output", "-x", "hip", "-c", src, "-o", obj],
                          cwd=os.path.dirname(src))
    dis = subprocess.check_output([OBJDUMP, "-d", obj], text=True)
    bad = []
    for name, body in functions(dis):
        if "s_getpc_b64 s[30:31]" in "\n".join(body):
            # kernels (entry points) are compiled with the .kd descriptor; their
            # bodies end in s_endpgm, callable functions in s_setpc_b64 s[30:31]
            returns = any("s_setpc_b64 s[30:31]" in l and "s_getpc" not in l for l in body)
            endpgm = any("s_endpgm" in l for l in body)
            if returns and not endpgm:
                bad.append(name)
    return bad


def main():
    srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "fabric-token-sdk_amd", "csrc", "*.hip")))
    bad = {}
    with tempfile.TemporaryDirectory() as tmp:
        for s in srcs:
            b = check(os.path.abspath(s), tmp)
            if b:
                bad[s] = b
            print("%-60s %s" % (os.path.relpath(s, ROOT), "FAIL " + ", ".join(b) if b else "ok"), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
