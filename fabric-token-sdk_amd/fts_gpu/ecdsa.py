"""ECDSA P-256 owner signatures on the device (libfts_gpu.so
``fts_ecdsa_verify_batch``; include/fts_gpu.h).

Mirrors validator/ecdsa/ecdsa.go:69-113:

* ``Verifier(pk).Verify(message, sigma)`` raises ``SignatureError`` with the
  reference's message ("signature is not in lowS", "signature not valid", or
  the asn1 failure) — one item per device pass;
* ``verify_batch(items, device)`` is the batched form a validator uses for
  all owner signatures of many requests (TransferSignatureValidate,
  validator/validator_transfer.go:29-62, checks one per input).

Public keys are ``(x, y)`` ints, 64-byte X||Y, or the DER SubjectPublicKeyInfo
/ PEM "PUBLIC KEY" that ``Verifier.Serialize`` wraps (ecdsa.go:115-150).
There is no CPU fallback: every verdict comes from the HIP kernels.
"""
import base64
import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import FTS_OK, FTS_E_SIG_MALFORMED, FTS_E_SIG_NOT_LOW_S, FTS_E_SIG_INVALID  # noqa: F401


class SignatureError(Exception):
    def __init__(self, msg, status):
        super().__init__(msg)
        self.status = status


def message(status):
    """Reference error string for a verdict (None for FTS_OK)."""
    if status == FTS_OK:
        return None
    if status == FTS_E_SIG_MALFORMED:
        return "asn1: structure error"
    return L.status_str(status)


def pk64_from_pkix(der):
    """x509.MarshalPKIXPublicKey bytes (or their PEM "PUBLIC KEY" block) -> X||Y."""
    if der.startswith(b"-----BEGIN"):
        lines = [ln for ln in der.decode().splitlines() if ln and not ln.startswith("-----")]
        der = base64.b64decode("".join(lines))
    out = (C.c_uint8 * 64)()
    L.check("fts_p256_pubkey_from_pkix", L.lib.fts_p256_pubkey_from_pkix(der, len(der), out))
    return bytes(out)


def _pk64(pk):
    if isinstance(pk, tuple):
        return pk[0].to_bytes(32, "big") + pk[1].to_bytes(32, "big")
    pk = bytes(pk)
    return pk if len(pk) == 64 else pk64_from_pkix(pk)


def parse_sig(sig):
    """Host-side asn1.Unmarshal + IsLowS + range checks -> (status, r, s)."""
    r, s, st = (C.c_uint8 * 32)(), (C.c_uint8 * 32)(), C.c_int32(0)
    L.check("fts_ecdsa_sig_parse", L.lib.fts_ecdsa_sig_parse(sig, len(sig), r, s, C.byref(st)))
    return st.value, int.from_bytes(bytes(r), "big"), int.from_bytes(bytes(s), "big")


def verify_batch(msgs, sigs, pks, device=0):
    """Verify n (message, DER signature, public key) triples in one device pass
    -> int32 status array."""
    n = len(msgs)
    if len(sigs) != n or len(pks) != n:
        raise ValueError("msgs, sigs and pks must have the same length")
    st = np.zeros(n, dtype=np.int32)
    if n == 0:
        return st
    keep = [(bytes(m), bytes(s), _pk64(p)) for m, s, p in zip(msgs, sigs, pks)]
    items = (L.EcdsaItem * n)()
    for i, (m, s, p) in enumerate(keep):
        items[i].msg = C.cast(C.c_char_p(m), C.c_void_p)
        items[i].msg_len = len(m)
        items[i].sig = C.cast(C.c_char_p(s), C.c_void_p)
        items[i].sig_len = len(s)
        items[i].pk64 = C.cast(C.c_char_p(p), C.c_void_p)
    L.check("fts_ecdsa_verify_batch",
            L.lib.fts_ecdsa_verify_batch(int(device), n, items, st.ctypes.data_as(C.POINTER(C.c_int32))))
    return st


def verify_packed(msg_buf, msg_off, msg_len, sig_buf, sig_off, sig_len, pk_buf, device=0):
    """Zero-copy batch form over contiguous buffers (bench / large batches).
    Every (offset, length) must lie inside its buffer and pk_buf must hold 64 bytes
    per item: the C library is handed raw pointers, so this is checked here
    (ValueError) before any pointer is formed."""
    n = len(msg_off)
    mo, ml = np.asarray(msg_off, dtype=np.uint64), np.asarray(msg_len, dtype=np.uint64)
    so, sl = np.asarray(sig_off, dtype=np.uint64), np.asarray(sig_len, dtype=np.uint64)
    if not (mo.shape == ml.shape == so.shape == sl.shape == (n,)):
        raise ValueError("offset and length arrays must be 1-D and of equal length")
    if len(pk_buf) < 64 * n:
        raise ValueError("pk_buf holds %d bytes, %d items need %d" % (len(pk_buf), n, 64 * n))
    for name, off, ln, buf in (("msg", mo, ml, msg_buf), ("sig", so, sl, sig_buf)):
        # end = off + len without uint64 wrap-around: off <= size and len <= size - off
        size = np.uint64(len(buf))
        if n and ((off > size).any() or (ln > size - np.minimum(off, size)).any()):
            raise ValueError("%s offset + length outside its buffer (%d bytes)" % (name, len(buf)))
    st = np.zeros(n, dtype=np.int32)
    items = np.zeros(n, dtype=[("msg", "u8"), ("msg_len", "u8"), ("sig", "u8"), ("sig_len", "u8"), ("pk64", "u8")])
    mb, sb, pb = (np.frombuffer(b, dtype=np.uint8) for b in (msg_buf, sig_buf, pk_buf))
    items["msg"] = mb.ctypes.data + mo
    items["msg_len"] = ml
    items["sig"] = sb.ctypes.data + so
    items["sig_len"] = sl
    items["pk64"] = pb.ctypes.data + 64 * np.arange(n, dtype=np.uint64)
    L.check("fts_ecdsa_verify_batch",
            L.lib.fts_ecdsa_verify_batch(int(device), n, items.ctypes.data_as(C.POINTER(L.EcdsaItem)),
                                         st.ctypes.data_as(C.POINTER(C.c_int32))))
    return st


def last_timings(device=0):
    """{kernel: ms} of the last verify call on `device` (HIP events)."""
    ms = (C.c_float * 2)()
    L.check("fts_ecdsa_last_timings", L.lib.fts_ecdsa_last_timings(int(device), ms))
    return {"k_ecdsa_digest": ms[0], "k_ecdsa_verify": ms[1]}


class Verifier:
    """ecdsa.Verifier{PK} (validator/ecdsa/ecdsa.go:69-113)."""

    def __init__(self, pk, device=0):
        self.pk64 = _pk64(pk)
        self.device = device

    def Verify(self, message_, sigma):
        st = int(verify_batch([message_], [sigma], [self.pk64], self.device)[0])
        if st != FTS_OK:
            raise SignatureError(message(st), st)
