"""Idemix pseudonym (nym) signatures on the device (libfts_gpu.so
``fts_nym_verify_batch``; include/fts_gpu.h).

Mirrors services/identity/idemix/crypto/id.go:145-161:

* ``NymSignatureVerifier(ipk, nym_pk).Verify(message, sigma)`` raises
  ``SignatureError`` with the reference's message;
* ``IssuerKey(ipk_bytes).verify_batch(nyms, sigs, msgs)`` is the batched form
  a validator uses for the owner signatures of idemix-owned inputs
  (TransferSignatureValidate, validator/validator_transfer.go:29-62).

The issuer key is the idemix IssuerPublicKey proto a zkatdlog PublicParams
carries, on BN254 (the tokengen key of zkatdlog_pp.json) or FP256BN_AMCL (the
validator's test keys).  There is no CPU fallback: every verdict comes from
the HIP kernel k_nym_verify.
"""
import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import FTS_OK, FTS_E_NYM_MALFORMED, FTS_E_NYM_BADKEY, FTS_E_NYM_INVALID  # noqa: F401
from ._lib import (FTS_E_ID_MALFORMED, FTS_E_ID_BADNYM, FTS_E_ID_NO_EIDNYM, FTS_E_ID_NO_RHNYM,  # noqa: F401
                   FTS_E_ID_REVOCATION, FTS_E_ID_APRIME, FTS_E_ID_PAIRING, FTS_E_ID_ZK)
from ._lib import FTS_CURVE_BN254, FTS_CURVE_FP256BN_AMCL  # noqa: F401


class SignatureError(Exception):
    def __init__(self, msg, status):
        super().__init__(msg)
        self.status = status


def message(status):
    """Reference error string for a verdict (None for FTS_OK)."""
    return None if status == FTS_OK else L.status_str(status)


def identity_nym(serialized_identity):
    """SerializedIdemixIdentity.nym_public_key (crypto/deserializer.go:41-56)."""
    raw = bytes(serialized_identity)
    p, n = C.c_void_p(), C.c_size_t()
    L.check("fts_idemix_identity_nym", L.lib.fts_idemix_identity_nym(raw, len(raw), C.byref(p), C.byref(n)))
    off = p.value - C.cast(C.c_char_p(raw), C.c_void_p).value
    return raw[off:off + n.value]


class IssuerKey:
    """Device-resident idemix issuer public key (HSk / HRand fixed-base tables)."""

    def __init__(self, ipk, device=0, curve=FTS_CURVE_BN254):
        """curve: mathlib CurveID (PublicParams.IdemixIssuerPublicKeys[i].Curve)."""
        self.ipk = bytes(ipk)
        self.device = device
        self.curve = curve
        self.nym_len = 64 if curve == FTS_CURVE_BN254 else 65
        h = C.c_void_p()
        L.check("fts_idemix_ipk_create",
                L.lib.fts_idemix_ipk_create(int(device), self.ipk, len(self.ipk), int(curve), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            L.lib.fts_idemix_ipk_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def verify_batch(self, nyms, sigs, msgs):
        """n (nym public key, NymSignature, message) triples in one device pass
        -> int32 status array."""
        n = len(nyms)
        if len(sigs) != n or len(msgs) != n:
            raise ValueError("nyms, sigs and msgs must have the same length")
        st = np.zeros(n, dtype=np.int32)
        if n == 0:
            return st
        keep = [(bytes(a), bytes(b), bytes(c)) for a, b, c in zip(nyms, sigs, msgs)]
        items = (L.NymItem * n)()
        for i, (a, b, c) in enumerate(keep):
            items[i].nym = C.cast(C.c_char_p(a), C.c_void_p)
            items[i].nym_len = len(a)
            items[i].sig = C.cast(C.c_char_p(b), C.c_void_p)
            items[i].sig_len = len(b)
            items[i].msg = C.cast(C.c_char_p(c), C.c_void_p)
            items[i].msg_len = len(c)
        L.check("fts_nym_verify_batch",
                L.lib.fts_nym_verify_batch(self.h, n, items, st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def verify_packed(self, nym_buf, sig_buf, sig_off, sig_len, msg_buf, msg_off, msg_len):
        """Zero-copy batch over contiguous buffers (nym keys of self.nym_len bytes back to back);
        bounds are checked here before any raw pointer is formed."""
        n = len(sig_off)
        so, sl = np.asarray(sig_off, dtype=np.uint64), np.asarray(sig_len, dtype=np.uint64)
        mo, ml = np.asarray(msg_off, dtype=np.uint64), np.asarray(msg_len, dtype=np.uint64)
        if not (so.shape == sl.shape == mo.shape == ml.shape == (n,)):
            raise ValueError("offset and length arrays must be 1-D and of equal length")
        nl = self.nym_len
        if len(nym_buf) < nl * n:
            raise ValueError("nym_buf holds %d bytes, %d items need %d" % (len(nym_buf), n, nl * n))
        for name, off, ln, buf in (("sig", so, sl, sig_buf), ("msg", mo, ml, msg_buf)):
            size = np.uint64(len(buf))
            if n and ((off > size).any() or (ln > size - np.minimum(off, size)).any()):
                raise ValueError("%s offset + length outside its buffer (%d bytes)" % (name, len(buf)))
        st = np.zeros(n, dtype=np.int32)
        items = np.zeros(n, dtype=[("nym", "u8"), ("nym_len", "u8"), ("sig", "u8"), ("sig_len", "u8"),
                                   ("msg", "u8"), ("msg_len", "u8")])
        nb, sb, mb = (np.frombuffer(b, dtype=np.uint8) for b in (nym_buf, sig_buf, msg_buf))
        items["nym"] = nb.ctypes.data + nl * np.arange(n, dtype=np.uint64)
        items["nym_len"] = nl
        items["sig"] = sb.ctypes.data + so
        items["sig_len"] = sl
        items["msg"] = mb.ctypes.data + mo
        items["msg_len"] = ml
        L.check("fts_nym_verify_batch",
                L.lib.fts_nym_verify_batch(self.h, n, items.ctypes.data_as(C.POINTER(L.NymItem)),
                                           st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def last_kernel_ms(self):
        ms = C.c_float()
        L.check("fts_nym_last_timings", L.lib.fts_nym_last_timings(self.h, C.byref(ms)))
        return ms.value


class NymSignatureVerifier:
    """crypto.NymSignatureVerifier{IPK, NymPK} (id.go:145-161)."""

    def __init__(self, issuer_key, nym_pk):
        self.ipk = issuer_key
        self.nym = bytes(nym_pk)

    def Verify(self, message_, sigma):
        st = int(self.ipk.verify_batch([self.nym], [sigma], [message_])[0])
        if st != FTS_OK:
            raise SignatureError(message(st), st)


class IdentityVerifier:
    """Idemix identity validity on the device (fts_idemix_identity_verify_batch):
    the check ``Deserializer.Deserialize(raw, true)`` makes for every idemix owner
    (services/identity/idemix/deserializer.go:82-93 -> crypto/id.go:74-108, IBM/idemix
    Signature.Ver with ExpectEidNymRhNym).  One handle per issuer public key."""

    def __init__(self, ipk, device=0, curve=FTS_CURVE_BN254):
        self.ipk = bytes(ipk)
        self.device = device
        self.curve = curve
        h = C.c_void_p()
        L.check("fts_idemix_idv_create",
                L.lib.fts_idemix_idv_create(int(device), self.ipk, len(self.ipk), int(curve), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            L.lib.fts_idemix_idv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, identities):
        """the C-ABI's pointer / length arrays for a batch of serialized identities,
        built once: verify_prepared then calls the library with no per-call Python
        marshaling (a Go caller hands its slices' pointers over the same way)"""
        keep = [bytes(x) for x in identities]
        n = len(keep)
        ptrs = (C.c_void_p * max(1, n))(*[C.cast(C.c_char_p(b), C.c_void_p).value for b in keep])
        lens = (C.c_size_t * max(1, n))(*[len(b) for b in keep])
        return keep, ptrs, lens

    def verify_prepared(self, prep):
        """prepare()d identities -> int32 status array (FTS_OK or FTS_E_ID_*)"""
        keep, ptrs, lens = prep
        n = len(keep)
        st = np.zeros(n, dtype=np.int32)
        if n == 0:
            return st
        L.check("fts_idemix_identity_verify_batch",
                L.lib.fts_idemix_identity_verify_batch(self.h, n, ptrs, lens, st.ctypes.data_as(C.POINTER(C.c_int32))))
        return st

    def verify_batch(self, identities):
        """serialized identities -> int32 status array (FTS_OK or FTS_E_ID_*)"""
        return self.verify_prepared(self.prepare(identities))

    def Deserialize(self, identity):
        """raises IdentityError with the reference's message, as Deserialize(raw, true) errors"""
        st = int(self.verify_batch([identity])[0])
        if st != FTS_OK:
            raise IdentityError(message(st), st)

    def last_kernel_ms(self):
        """(decode + t-values + transcript, pairings) HIP-event ms of the last batch"""
        ms = (C.c_float * 2)()
        L.check("fts_idemix_identity_last_timings", L.lib.fts_idemix_identity_last_timings(self.h, ms))
        return float(ms[0]), float(ms[1])

    def last_pairing_stats(self):
        """(groups checked with one randomised pairing product, identities paired one by
        one) of the last batch; (0, n) with FTS_IDV_BATCH=0"""
        out = (C.c_uint32 * 2)()
        L.check("fts_idemix_identity_last_stats", L.lib.fts_idemix_identity_last_stats(self.h, out))
        return int(out[0]), int(out[1])

    def pairing_debug(self, which, p64, final_exp=True):
        """e(W or g2, P) (BN254 only): 6 Fp2 coefficients (w^0..w^5) as Montgomery ints"""
        out = (C.c_uint32 * 192)()
        L.check("fts_idemix_pairing_debug",
                L.lib.fts_idemix_pairing_debug(self.h, int(which), bytes(p64), int(bool(final_exp)), out))
        w = list(out)
        val = lambda o: sum(w[o + i] << (32 * i) for i in range(8))  # noqa: E731
        return [(val(16 * k), val(16 * k + 8)) for k in range(6)]


class IdentityError(Exception):
    def __init__(self, msg, status):
        super().__init__(msg)
        self.status = status
