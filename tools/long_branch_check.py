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
glv_mul); the Makefile compiles it device-only to build/glv_noinline_repro.co
and tests/test_isa_cpu.py checks that it is flagged.

Inputs:
* a built host object or shared library (.o / .so): every gfx950 code object in
  its .hip_fatbin section (clang offload bundles) is disassembled;
* a device-only code object (ELF for amdgcn, .co);
* a .hip source: compiled device-only first.
The check FAILS if any non-kernel function writes s[30:31] with s_getpc_b64
(the far-branch expansion); kernels are exempt.
    python tools/long_branch_check.py [paths...]   (default: the product library)
__graft_entry__.build() runs it on lib/libfts_gpu.so after every build.
"""
import glob
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
LLVM = "/opt/rocm/lib/llvm/bin"
OBJDUMP = os.path.join(LLVM, "llvm-objdump")
OBJCOPY = os.path.join(LLVM, "llvm-objcopy")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PRODUCT = os.path.join(ROOT, "fabric-token-sdk_amd", "lib", "libfts_gpu.so")


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


def bad_functions(dis):
    """names of callable (non-kernel) functions with a relaxed branch through s[30:31]"""
    bad = []
    for name, body in functions(dis):
        text = "\n".join(body)
        if "s_getpc_b64 s[30:31]" not in text:
            continue
        # kernels end in s_endpgm; callable functions return through s_setpc_b64 s[30:31]
        returns = any("s_setpc_b64 s[30:31]" in l and "s_getpc" not in l for l in body)
        endpgm = any("s_endpgm" in l for l in body)
        if returns and not endpgm:
            bad.append(name)
    return bad


def bundles(blob):
    """gfx950 code objects inside a .hip_fatbin section (one clang offload bundle
    per translation unit, concatenated)"""
    out = []
    for m in re.finditer(re.escape(BUNDLE_MAGIC), blob):
        base = m.start()
        off = base + len(BUNDLE_MAGIC)
        (n,) = struct.unpack_from("<Q", blob, off)
        off += 8
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", blob, off)
            off += 24
            triple = blob[off:off + tl].decode()
            off += tl
            if "gfx950" in triple and es:
                out.append(blob[base + eo:base + eo + es])
    return out


def code_objects(path, tmp):
    """paths of the gfx950 code objects a built file holds"""
    with open(path, "rb") as f:
        head = f.read(20)
    if head[:4] != b"\x7fELF":
        raise ValueError("%s: not an ELF file" % path)
    (machine,) = struct.unpack_from("<H", head, 18)
    if machine == 224:  # EM_AMDGPU: already a device code object
        return [path]
    sec = os.path.join(tmp, os.path.basename(path) + ".fatbin")
    subprocess.check_call([OBJCOPY, "--dump-section=.hip_fatbin=" + sec, path, os.path.join(tmp, "scratch")])
    with open(sec, "rb") as f:
        blobs = bundles(f.read())
    outs = []
    for i, b in enumerate(blobs):
        p = os.path.join(tmp, "%s.%d.co" % (os.path.basename(path), i))
        with open(p, "wb") as f:
            f.write(b)
        outs.append(p)
    if not outs:
        raise ValueError("%s: no gfx950 code object found" % path)
    return outs


def compile_source(src, tmp):
    obj = os.path.join(tmp, os.path.basename(src) + ".co")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                           "--no-gpu-bundle-output", "-x", "hip", "-c", src, "-o", obj],
                          cwd=os.path.dirname(src))
    return obj


def check(path, tmp=None):
    """{code object: [bad function names]} for one input path (only offenders listed);
    raises if the input holds no gfx950 code."""
    own = tmp is None
    if own:
        td = tempfile.TemporaryDirectory()
        tmp = td.name
    try:
        path = os.path.abspath(path)
        cos = [compile_source(path, tmp)] if path.endswith(".hip") else code_objects(path, tmp)
        bad = {}
        for co in cos:
            dis = subprocess.check_output([OBJDUMP, "-d", co], text=True)
            if "s_endpgm" not in dis and "s_setpc_b64" not in dis:
                raise ValueError("%s: disassembly holds no gfx950 code" % co)
            b = bad_functions(dis)
            if b:
                bad[os.path.basename(co)] = b
        return bad
    finally:
        if own:
            td.cleanup()


def main():
    paths = sys.argv[1:] or [PRODUCT]
    failed = False
    for p in paths:
        bad = check(p)
        failed |= bool(bad)
        msg = "ok" if not bad else "FAIL " + "; ".join("%s: %s" % (k, ", ".join(v)) for k, v in bad.items())
        print("%-60s %s" % (os.path.relpath(os.path.abspath(p), ROOT), msg), flush=True)
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main()
