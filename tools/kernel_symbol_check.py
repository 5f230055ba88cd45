"""Build-time guard: every kernel the host side of a built library can launch
has device code in the library's gfx950 code objects.

Why: hipcc compiles a .hip file in two passes (device, then host).  A source
edited while its compile runs can give an object whose host stubs name kernels
its device code object does not hold (round 4: the identity kernels were split
while the old source was being compiled); the library then loads, and the
first launch aborts the process with "Cannot find Symbol with name: ...".
`make` does not rebuild such an object (it is newer than the source).

Host side: every `__device_stub__<kernel>` symbol of the library (llvm-readelf),
mapped back to the kernel's mangled name.  Device side: every `<kernel>.kd`
descriptor in the code objects of its .hip_fatbin section (the extraction of
tools/long_branch_check.py).  The check fails if a stub has no descriptor.
    python tools/kernel_symbol_check.py [lib ...]   (default: the product library)
__graft_entry__.build() runs it after every build."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from long_branch_check import LLVM, PRODUCT, ROOT, code_objects  # noqa: E402

READELF = os.path.join(LLVM, "llvm-readelf")
STUB = re.compile(r"(\d+)__device_stub__")


def kernel_of_stub(sym):
    """_ZN3idv27__device_stub__k_fooI...E... -> _ZN3idv5k_fooI...E... (the stub's
    source name is the kernel's, prefixed with __device_stub__)"""
    m = STUB.search(sym)
    if not m:
        return None
    n = int(m.group(1)) - len("__device_stub__")
    start = m.end()
    name = sym[start:start + n]
    return sym[:m.start()] + str(n) + name + sym[start + n:]


def symbols(path):
    """names in the ELF symbol tables of a file"""
    out = subprocess.check_output([READELF, "-sW", path], text=True)
    for line in out.splitlines():
        parts = line.split()
        if len(parts) >= 8 and parts[0].endswith(":"):
            yield parts[7]


def host_kernels(lib):
    ks = set()
    for name in symbols(lib):
        if "__device_stub__" in name:
            k = kernel_of_stub(name)
            if k:
                ks.add(k)
    return ks


def device_kernels(lib, tmp):
    ks = set()
    for co in code_objects(lib, tmp):
        for name in symbols(co):
            if name.endswith(".kd"):
                ks.add(name[:-3])
    return ks


def check(lib):
    """kernel names with a host stub but no device code (empty = ok)"""
    with tempfile.TemporaryDirectory() as tmp:
        host = host_kernels(lib)
        dev = device_kernels(lib, tmp)
    if not host:
        raise ValueError("%s: no kernel launch stubs found" % lib)
    return sorted(host - dev)


def main():
    failed = False
    for p in sys.argv[1:] or [PRODUCT]:
        missing = check(p)
        failed |= bool(missing)
        msg = "ok" if not missing else "FAIL no device code for: " + ", ".join(missing)
        print("%-60s %s" % (os.path.relpath(os.path.abspath(p), ROOT), msg), flush=True)
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main()
