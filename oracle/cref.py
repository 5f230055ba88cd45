"""ctypes binding of the C oracle (oracle/c/ref_verify.c) — test
infrastructure and bench.py's cpu_baseline leg only.  Build: make -C oracle/c
(outputs oracle/_build/libref_verify.so and libcpu_batch.so)."""
import ctypes as C
import os
import subprocess

from . import bn254 as bn

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libref_verify.so")
LIB_BATCH = os.path.join(HERE, "_build", "libcpu_batch.so")
_lib = None
_blib = None


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "c")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.oracle_rp_verify.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t]
        _lib.oracle_rp_verify.restype = C.c_int
        _lib.oracle_rp_verify_many.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_char_p),
                                               C.POINTER(C.c_size_t), C.c_int, C.POINTER(C.c_int32)]
        _lib.oracle_rp_verify_many.restype = C.c_int
        _lib.oracle_msm.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int, C.c_char_p]
        _lib.oracle_msm.restype = C.c_int
    return _lib


def gens_blob(pp):
    """[G=ped1, H=ped2, P, Q, L..., R...] as in bulletproof.go's rangeVerifier"""
    pts = [pp.ped[1], pp.ped[2], pp.P, pp.Q] + list(pp.left) + list(pp.right)
    return b"".join(bn.g1_bytes(p) for p in pts)


def rp_verify(pp, com64, der):
    return lib().oracle_rp_verify(gens_blob(pp), pp.bit_length, com64, der, len(der))


def rp_verify_many(pp, coms, ders, threads=1):
    n = len(ders)
    arr = (C.c_char_p * n)(*ders)
    lens = (C.c_size_t * n)(*[len(d) for d in ders])
    out = (C.c_int32 * n)()
    rc = lib().oracle_rp_verify_many(gens_blob(pp), pp.bit_length, n, b"".join(coms), arr, lens, threads, out)
    assert rc == 0
    return list(out)


def msm(points64, scalars32, threads=1):
    """sum (k_i mod r) P_i term by term (G1.Mul + Add) -> 64-byte BE result"""
    n = len(points64) // 64
    out = C.create_string_buffer(64)
    rc = lib().oracle_msm(points64, scalars32, n, threads, out)
    assert rc == 0
    return out.raw


def open_check_many(pp, openings, threads=1):
    """Auditor.InspectOutput in reference order for (com64, type, value32, bf32)
    openings -> fts_status numbering (0 ok, 12 mismatch, 1 malformed data)"""
    lb = lib()
    if not hasattr(lb, "_open_sig"):
        lb.oracle_open_check_many.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.POINTER(C.c_char_p),
                                              C.POINTER(C.c_size_t), C.c_char_p, C.c_char_p, C.c_int,
                                              C.POINTER(C.c_int32)]
        lb.oracle_open_check_many.restype = C.c_int
        lb._open_sig = True
    n = len(openings)
    ped = b"".join(bn.g1_bytes(p) for p in pp.ped)
    types = (C.c_char_p * n)(*[o[1] for o in openings])
    tl = (C.c_size_t * n)(*[len(o[1]) for o in openings])
    out = (C.c_int32 * n)()
    rc = lb.oracle_open_check_many(ped, n, b"".join(o[0] for o in openings), types, tl,
                                   b"".join(o[2] for o in openings), b"".join(o[3] for o in openings), threads, out)
    assert rc == 0
    return list(out)


def action_verify_many(pp, actions, threads=1):
    """transfer / issue Verify in reference order (oracle_action_verify_many):
    actions = [(kind, inputs[list of 64 B], outputs[list of 64 B], proof)] with kind
    "transfer" or "issue" (issue: tokens as outputs, no inputs) ->
    [(fts_status, fail index)]"""
    lb = lib()
    if not hasattr(lb, "_act_sig"):
        P = C.POINTER
        lb.oracle_action_verify_many.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, P(C.c_int32),
                                                 P(C.c_int32), P(C.c_int32), P(C.c_char_p), P(C.c_char_p),
                                                 P(C.c_char_p), P(C.c_size_t), C.c_int, P(C.c_int32),
                                                 P(C.c_int32)]
        lb.oracle_action_verify_many.restype = C.c_int
        lb._act_sig = True
    n = len(actions)
    kind = (C.c_int32 * n)(*[0 if a[0] == "transfer" else 1 for a in actions])
    nin = (C.c_int32 * n)(*[len(a[1]) for a in actions])
    nout = (C.c_int32 * n)(*[len(a[2]) for a in actions])
    ins = (C.c_char_p * n)(*[b"".join(a[1]) or b"\0" for a in actions])
    outs = (C.c_char_p * n)(*[b"".join(a[2]) or b"\0" for a in actions])
    ders = (C.c_char_p * n)(*[a[3] for a in actions])
    lens = (C.c_size_t * n)(*[len(a[3]) for a in actions])
    st, ix = (C.c_int32 * n)(), (C.c_int32 * n)()
    ped = b"".join(bn.g1_bytes(p) for p in pp.ped)
    rc = lb.oracle_action_verify_many(ped, gens_blob(pp), pp.bit_length, n, kind, nin, nout, ins, outs, ders, lens,
                                      threads, st, ix)
    assert rc == 0
    return list(zip(list(st), list(ix)))


def _batch_lib():
    global _blib
    if _blib is None:
        if not os.path.exists(LIB_BATCH):
            build()
        _blib = C.CDLL(LIB_BATCH)
        _blib.cpu_batch_create.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int]
        _blib.cpu_batch_create.restype = C.c_void_p
        _blib.cpu_batch_verify.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_char_p),
                                           C.POINTER(C.c_size_t), C.c_int, C.POINTER(C.c_int32)]
        _blib.cpu_batch_verify.restype = C.c_int
        _blib.cpu_batch_verify_ex.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_char_p),
                                              C.POINTER(C.c_size_t), C.c_int, C.POINTER(C.c_int32), C.c_char_p,
                                              C.c_char_p]
        _blib.cpu_batch_verify_ex.restype = C.c_int
        _blib.cpu_batch_free.argtypes = [C.c_void_p]
        _blib.cpu_msm_pippenger.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int, C.c_char_p]
        _blib.cpu_msm_pippenger.restype = C.c_int
    return _blib


class CpuBatch:
    """The optimized CPU batch verifier (oracle/c/cpu_batch.c): the device's
    batch algorithm on host threads, bench.py's "optimized CPU batch" column.
    verify() -> (verdicts in fts_status numbering, proofs that took the
    per-proof fallback)."""

    def __init__(self, pp, window_bits=11, threads=1):
        self.h = _batch_lib().cpu_batch_create(gens_blob(pp), pp.bit_length, window_bits, threads)
        if not self.h:
            raise ValueError("cpu_batch_create failed")

    def verify(self, coms, ders, threads=1):
        n = len(ders)
        arr = (C.c_char_p * max(n, 1))(*ders)
        lens = (C.c_size_t * max(n, 1))(*[len(d) for d in ders])
        out = (C.c_int32 * max(n, 1))()
        nfb = _batch_lib().cpu_batch_verify(self.h, n, b"".join(coms), arr, lens, threads, out)
        assert nfb >= 0
        return list(out)[:n], nfb

    def verify_ex(self, coms, ders, threads=1):
        """verify() plus every proof's exact com (64 B) and x0 (32 B BE); zeros
        where the proof stopped before them (parse errors, IPA structure)"""
        n = len(ders)
        arr = (C.c_char_p * max(n, 1))(*ders)
        lens = (C.c_size_t * max(n, 1))(*[len(d) for d in ders])
        out = (C.c_int32 * max(n, 1))()
        com_out, x0_out = C.create_string_buffer(64 * max(n, 1)), C.create_string_buffer(32 * max(n, 1))
        nfb = _batch_lib().cpu_batch_verify_ex(self.h, n, b"".join(coms), arr, lens, threads, out, com_out, x0_out)
        assert nfb >= 0
        return (list(out)[:n], nfb, [com_out.raw[64 * i:64 * i + 64] for i in range(n)],
                [x0_out.raw[32 * i:32 * i + 32] for i in range(n)])

    def close(self):
        if self.h:
            _batch_lib().cpu_batch_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def msm_pippenger(points64, scalars32, threads=1):
    """sum (k_i mod r) P_i with oracle/c/cpu_batch.c's GLV Pippenger -> 64-byte BE result"""
    n = len(points64) // 64
    out = C.create_string_buffer(64)
    rc = _batch_lib().cpu_msm_pippenger(points64, scalars32, n, threads, out)
    if rc != 0:
        raise ValueError("bad point")
    return out.raw
