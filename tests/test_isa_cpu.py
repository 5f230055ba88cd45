"""ISA guards on the built gfx950 code objects (CPU only: disassembly, no GPU).

* long-branch guard: no callable device function may contain a
  relaxed far branch through s[30:31] (its return address) -- the miscompile that
  made an out-of-line glv_mul loop forever. The product library must pass; the
  reproducer tools/experiments/glv_noinline_repro.hip (built device-only by the
  Makefile) must be flagged, so the guard is known to fire.
* the product code issues no MFMA instruction (DESIGN.md §5 "No MFMA": this is
  carry-propagating modular arithmetic on the INT32 VALU).
* every kernel the library's host side can launch has device code
  (tools/kernel_symbol_check.py: an object whose host and device passes saw
  different sources aborts at the first launch with "Cannot find Symbol").
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_symbol_check as ksc  # noqa: E402
import long_branch_check as lbc  # noqa: E402

LIB = os.path.join(ROOT, "fabric-token-sdk_amd", "lib", "libfts_gpu.so")
REPRO = os.path.join(ROOT, "fabric-token-sdk_amd", "build", "glv_noinline_repro.co")


def _need(p):
    if not os.path.exists(p):
        pytest.skip("%s not built (run __graft_entry__.build())" % os.path.relpath(p, ROOT))


def test_product_library_has_no_relaxed_branch_through_return_address():
    _need(LIB)
    assert lbc.check(LIB) == {}


def test_guard_flags_the_noinline_reproducer():
    _need(REPRO)
    bad = lbc.check(REPRO)
    names = [n for v in bad.values() for n in v]
    assert any("nl_glv_mul" in n for n in names), bad


def test_bad_function_detection_on_synthetic_listing():
    callee = ("0000000000001000 <_Z3foov>:\n"
              "  s_getpc_b64 s[30:31]\n  s_add_u32 s30, s30, 0x100\n  s_setpc_b64 s[30:31]\n"
              "  s_setpc_b64 s[30:31]\n")
    kernel = ("0000000000002000 <k_ok>:\n  s_getpc_b64 s[30:31]\n  s_setpc_b64 s[30:31]\n  s_endpgm\n")
    assert lbc.bad_functions(callee + kernel) == ["_Z3foov"]


def test_product_code_has_no_mfma(tmp_path):
    _need(LIB)
    cos = lbc.code_objects(LIB, str(tmp_path))
    assert len(cos) >= 7  # one bundle per .hip translation unit
    for co in cos:
        dis = subprocess.check_output([lbc.OBJDUMP, "-d", co], text=True)
        assert "v_mfma" not in dis, co


def test_every_host_kernel_stub_has_device_code():
    _need(LIB)
    assert ksc.check(LIB) == []


def test_kernel_symbol_guard_flags_a_host_device_mismatch(tmp_path):
    """a translation unit whose device pass defines k_a but whose host pass
    launches k_b: the library links, and the guard must name k_b"""
    src = tmp_path / "mismatch.hip"
    src.write_text("#include <hip/hip_runtime.h>\n"
                   "#ifdef __HIP_DEVICE_COMPILE__\n"
                   "__global__ void k_a(int* p) { *p = 1; }\n"
                   "#else\n"
                   "__global__ void k_b(int* p) { *p = 1; }\n"
                   "extern \"C\" void launch(int* p) { hipLaunchKernelGGL(k_b, 1, 1, 0, 0, p); }\n"
                   "#endif\n")
    lib = tmp_path / "libmismatch.so"
    subprocess.check_call([lbc.HIPCC, "--offload-arch=gfx950", "-O1", "-shared", "-fPIC", "-x", "hip", str(src),
                           "-o", str(lib)])
    missing = ksc.check(str(lib))
    assert len(missing) == 1 and "k_b" in missing[0], missing
