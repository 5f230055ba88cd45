"""Idemix pseudonym (nym) signatures over BN254 and FP256BN, restated in pure Python
(oracle; TEST INFRASTRUCTURE ONLY -- never imported by the product path).

Reference call sites (fabric-token-sdk):
* validator/validator_transfer.go:29-62   TransferSignatureValidate: one owner
  signature per input token, through Deserializer.GetOwnerVerifier
* services/identity/idemix/deserializer.go:82-105   the owner verifier of an
  idemix identity is crypto.NymSignatureVerifier{IPK, NymPK}
* services/identity/idemix/crypto/id.go:145-161   NymSignatureVerifier.Verify
  -> CSP.Verify(NymPK, sigma, message, IdemixNymSignerOpts{IssuerPK})
* services/identity/idemix/crypto/deserializer.go:41-72   NymPK = KeyImport of
  SerializedIdemixIdentity.nym_public_key (crypto/protos/idemix_config.proto)

The verifier itself lives in github.com/IBM/idemix v0.0.2-0.20240816143710-
3dce4618d760 (go.mod:6; NOT vendored), bccsp/schemes/dlog/crypto
nymsignature.go, NymSignature.Ver.  Restated (Fiat-Shamir proof of knowledge
of (sk, r) with Nym = HSk^sk * HRand^r):

    t      = HSk * s_sk + HRand * s_rnym - Nym * c
    c'     = HashToZr("sign" || t || Nym || ipk.Hash || msg)
    accept iff c == HashToZr(c' || Nonce)        (Zr.Equals on integers)

with G1 elements as G1.Bytes() and Zr as 32-byte big-endian.

What is pinned by the reference's own fixtures (tests/test_idemix_oracle.py):
* HashToZr on BN254 = SHA-256 mod r and Zr.Bytes = 32-byte big-endian: every
  IssuerPublicKey fixture's `hash` field equals HashToZr(proto bytes without
  it); the charlie.ExtraId2 key's digest exceeds r, so the reduction is pinned.
* the G1 (64-byte raw) and G2 (gnark raw, imaginary part first) encodings in
  idemix transcripts, and exact-size proof buffers: the issuer key's proof of
  knowledge (ProofC, ProofS over t1 || t2 || g2 || BarG1 || W || BarG2)
  verifies on the BN254 fixtures (the tokengen issuer secret key also gives
  BarG2 = ISk * BarG1 and g2 = W / ISk = the standard BN254 G2 generator).
* the protobuf layout of IssuerPublicKey / IdemixSignerConfig.
UNPINNED (no nym-signature vector in the reference): the "sign" label and the
two-hash structure of the nym proof, restated from the published idemix code.
"""
import hashlib

from .bn254 import P, R, g1_add, g1_bytes, g1_from_bytes, g1_mul, g1_neg, PointError

SIGN_LABEL = b"sign"
MSG_MALFORMED = "error unmarshalling signature"
MSG_BADKEY = "failed importing nym public key"
MSG_INVALID = "pseudonym signature invalid: zero-knowledge proof is invalid"


# ------------------------------------------------------------ protobuf (wire)
def _varint(b, i):
    """protowire.ConsumeVarint: at most 10 bytes, the 10th carrying only bit 63"""
    s = sh = 0
    while True:
        if i >= len(b):
            raise ValueError("truncated varint")
        c = b[i]
        i += 1
        if sh == 63 and c > 1:
            raise ValueError("varint overflow")
        s |= (c & 0x7F) << sh
        sh += 7
        if c < 0x80:
            return s, i
        if sh > 63:
            raise ValueError("varint overflow")


def _field_value(b, i, f, wt, depth=0):
    """(value, next index) of one field; groups (wire type 3 up to the matching 4)
    are consumed as protowire.ConsumeFieldValue does and return None"""
    if wt == 0:
        return _varint(b, i)
    if wt == 1:
        if i + 8 > len(b):
            raise ValueError("truncated fixed64")
        return b[i:i + 8], i + 8
    if wt == 5:
        if i + 4 > len(b):
            raise ValueError("truncated fixed32")
        return b[i:i + 4], i + 4
    if wt == 2:
        n, i = _varint(b, i)
        if i + n > len(b):
            raise ValueError("truncated bytes")
        return b[i:i + n], i + n
    if wt == 3:
        if depth >= 64:
            raise ValueError("group nesting")
        while True:
            key, i = _varint(b, i)
            gf, gw = key >> 3, key & 7
            if gf == 0 or gf > 0x1FFFFFFF:
                raise ValueError("bad field number")
            if gw == 4:
                if gf != f:
                    raise ValueError("mismatched end group")
                return None, i
            _, i = _field_value(b, i, gf, gw, depth + 1)
    raise ValueError("wire type %d" % wt)


def pb_fields(b):
    """[(field, wire_type, value)] of a protobuf message (wire types 0, 1, 2, 5;
    skipped groups appear with wire type 3 and value None)."""
    out, i = [], 0
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if f == 0 or f > 0x1FFFFFFF:
            raise ValueError("bad field number")
        v, i = _field_value(b, i, f, wt)
        out.append((f, wt, v))
    return out


def _pb_bytes(fields, f):
    v = b""
    for ff, wt, val in fields:
        if ff == f:
            if wt != 2:
                raise ValueError("field %d: wire type %d" % (f, wt))
            v = val  # proto3: the last occurrence wins
    return v


def _key(f, wt=2):
    k, out = (f << 3) | wt, b""
    while True:
        c = k & 0x7F
        k >>= 7
        out += bytes([c | (0x80 if k else 0)])
        if not k:
            return out


def pb_bytes_field(f, v):
    n, ln = len(v), b""
    while True:
        c = n & 0x7F
        n >>= 7
        ln += bytes([c | (0x80 if n else 0)])
        if not n:
            break
    return _key(f) + ln + v


# ----------------------------------------------------------------- BN254 G2
# Fp2 = Fp[u]/(u^2 + 1), elements (a0, a1); twist y^2 = x^3 + 3/(9 + u)
def _f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def _f2sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def _f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _f2inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)


G2_B = _f2mul((3, 0), _f2inv((9, 1)))
# the standard BN254 G2 generator (= W / ISk of the tokengen fixture, tested)
G2_GEN = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
           11559732032986387107991004021392285783925812861821192530917403151452391805634),
          (8495653923123431417604973247489272438418190587263600148770280649306958101930,
           4082367875863433681332203403145435568316851327593401208105741076214120093531))


def g2_on_curve(pt):
    x, y = pt
    return _f2sub(_f2mul(y, y), _f2add(_f2mul(_f2mul(x, x), x), G2_B)) == (0, 0)


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if _f2add(a[1], b[1]) == (0, 0):
            return None
        lam = _f2mul(_f2mul((3, 0), _f2mul(a[0], a[0])), _f2inv(_f2mul((2, 0), a[1])))
    else:
        lam = _f2mul(_f2sub(b[1], a[1]), _f2inv(_f2sub(b[0], a[0])))
    x = _f2sub(_f2sub(_f2mul(lam, lam), a[0]), b[0])
    return (x, _f2sub(_f2mul(lam, _f2sub(a[0], x)), a[1]))


def g2_mul(pt, k):
    acc = None
    for bit in bin(k % R)[2:]:
        acc = g2_add(acc, acc)
        if bit == "1":
            acc = g2_add(acc, pt)
    return acc


def g2_bytes(pt):
    """gnark-crypto bn254 G2Affine raw bytes: X.A1 | X.A0 | Y.A1 | Y.A0."""
    if pt is None:
        return bytes(128)
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(32, "big") for v in (x1, x0, y1, y0))


def g2_from_bytes(b):
    if len(b) != 128:
        raise PointError("invalid G2 length")
    x1, x0, y1, y0 = (int.from_bytes(b[32 * i:32 * i + 32], "big") for i in range(4))
    if max(x0, x1, y0, y1) >= P:
        raise PointError("non-canonical G2 coordinate")
    pt = ((x0, x1), (y0, y1))
    if pt == ((0, 0), (0, 0)):
        return None
    if not g2_on_curve(pt):
        raise PointError("G2 point not on curve")
    return pt


# ----------------------------------------------------------------- Zr, hash
def hash_to_zr(m):
    """mathlib BN254 Curve.HashToZr: SHA-256 as a big-endian integer mod r."""
    return int.from_bytes(hashlib.sha256(m).digest(), "big") % R


def zr_bytes(z):
    """Zr.Bytes(): 32-byte big-endian (mathlib BigToBytes; wider values keep their
    minimal big-endian form)."""
    n = max(32, (z.bit_length() + 7) // 8)
    return z.to_bytes(n, "big")


# --------------------------------------------------------------------- curves
class _Bn254:
    """mathlib BN254 (gurvy / gnark-crypto): G1.Bytes() = 64-byte raw X || Y,
    NewZrFromBytes = big-endian integer of any length (not reduced)."""
    name, p, r, g1_len = "BN254", P, R, 64

    add, neg, mul = staticmethod(g1_add), staticmethod(g1_neg), staticmethod(g1_mul)
    g1_bytes, g1_from_bytes = staticmethod(g1_bytes), staticmethod(g1_from_bytes)

    def hash_to_zr(self, m):
        return int.from_bytes(hashlib.sha256(m).digest(), "big") % R

    @staticmethod
    def zr_from_field(b):
        return int.from_bytes(b, "big")

    def ecp(self, x, y):
        return g1_from_bytes(x + y)


class _Fp256bn:
    """mathlib FP256BN_AMCL (y^2 = x^3 + 3): G1.Bytes() = ECP.ToBytes(uncompressed),
    0x04 || X || Y (65 bytes); Zr from bytes = AMCL FromBytes, which reads exactly
    the first 32 bytes (a shorter field makes the Go code panic)."""
    name = "FP256BN_AMCL"
    p = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49F0CDC65FB12980A82D3292DDBAED33013
    r = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49E0CDC65FB1299921AF62D536CD10B500D
    g1_len = 65

    def on_curve(self, pt):
        x, y = pt
        return (y * y - x * x * x - 3) % self.p == 0

    def add(self, a, b):
        p = self.p
        if a is None:
            return b
        if b is None:
            return a
        if a[0] == b[0]:
            if (a[1] + b[1]) % p == 0:
                return None
            lam = 3 * a[0] * a[0] * pow(2 * a[1], p - 2, p) % p
        else:
            lam = (b[1] - a[1]) * pow(b[0] - a[0], p - 2, p) % p
        x = (lam * lam - a[0] - b[0]) % p
        return (x, (lam * (a[0] - x) - a[1]) % p)

    def neg(self, a):
        return None if a is None else (a[0], (-a[1]) % self.p)

    def mul(self, pt, k):
        acc = None
        for bit in bin(k % self.r)[2:]:
            acc = self.add(acc, acc)
            if bit == "1":
                acc = self.add(acc, pt)
        return acc

    def g1_bytes(self, pt):
        if pt is None:  # AMCL ECP.ToBytes of infinity: projective (0, 1, 0), Affine() keeps it
            return b"\x04" + bytes(32) + (1).to_bytes(32, "big")
        return b"\x04" + pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")

    def g1_from_bytes(self, b):
        # 65-byte uncompressed only; an off-curve or non-canonical key is rejected
        # (AMCL would yield the point at infinity: the verdict is a rejection either way)
        if len(b) != 65 or b[0] != 4:
            raise PointError("invalid point encoding")
        x, y = int.from_bytes(b[1:33], "big"), int.from_bytes(b[33:], "big")
        if x >= self.p or y >= self.p or not self.on_curve((x, y)):
            raise PointError("point not on curve")
        return (x, y)

    def hash_to_zr(self, m):
        return int.from_bytes(hashlib.sha256(m).digest(), "big") % self.r

    @staticmethod
    def zr_from_field(b):
        if len(b) < 32:
            raise ValueError("short Zr")  # AMCL FromBytes indexes 32 bytes: the reference panics
        return int.from_bytes(b[:32], "big")

    def ecp(self, x, y):
        pt = (int.from_bytes(x, "big"), int.from_bytes(y, "big"))
        if not self.on_curve(pt):
            raise PointError("ECP not on curve")
        return pt


BN254C, FP256BNC = _Bn254(), _Fp256bn()
CURVES = {1: BN254C, 0: FP256BNC}  # mathlib CurveID: FP256BN_AMCL = 0, BN254 = 1


# ---------------------------------------------------------------- issuer key
def _ecp(raw, curve=BN254C):
    """idemix ECP{x, y} proto -> G1 point (translator: 32-byte big-endian x, y)."""
    f = pb_fields(raw)
    x, y = _pb_bytes(f, 1), _pb_bytes(f, 2)
    if len(x) != 32 or len(y) != 32:
        raise PointError("ECP coordinate length")
    return curve.ecp(x, y)


def _ecp2(raw):
    f = pb_fields(raw)
    parts = [_pb_bytes(f, i) for i in (1, 2, 3, 4)]
    if any(len(p) != 32 for p in parts):
        raise PointError("ECP2 coordinate length")
    return g2_from_bytes(b"".join(parts))


def parse_ipk(raw, curve=BN254C):
    """idemix IssuerPublicKey proto (fields: 1 attribute_names, 2 h_sk, 3 h_rand,
    4 h_attrs, 5 w, 6 bar_g1, 7 bar_g2, 8 proof_c, 9 proof_s, 10 hash).  W (G2)
    is decoded for BN254 only (the FP256BN G2 encoding is not needed for nyms)."""
    f = pb_fields(raw)
    return {
        "curve": curve,
        "attribute_names": [v.decode() for ff, _, v in f if ff == 1],
        "h_sk": _ecp(_pb_bytes(f, 2), curve),
        "h_rand": _ecp(_pb_bytes(f, 3), curve),
        "h_attrs": [_ecp(v, curve) for ff, _, v in f if ff == 4],
        "w": _ecp2(_pb_bytes(f, 5)) if curve is BN254C else _pb_bytes(f, 5),
        "bar_g1": _ecp(_pb_bytes(f, 6), curve),
        "bar_g2": _ecp(_pb_bytes(f, 7), curve),
        "proof_c": _pb_bytes(f, 8),
        "proof_s": _pb_bytes(f, 9),
        "hash": _pb_bytes(f, 10),
    }


def ipk_hash_input(raw):
    """The IssuerPublicKey proto re-serialised without its `hash` field (Go
    marshals fields in number order, so this is the pre-hash encoding)."""
    out, i = b"", 0
    while i < len(raw):
        j = i
        key, i = _varint(raw, i)
        wt = key & 7
        if wt == 0:
            _, i = _varint(raw, i)
        elif wt == 2:
            n, i = _varint(raw, i)
            i += n
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        if key >> 3 != 10:
            out += raw[j:i]
    return out


def ipk_proof_valid(ipk):
    """Issuer key proof of knowledge of ISk (W = g2^ISk, BarG2 = BarG1^ISk)."""
    c = int.from_bytes(ipk["proof_c"], "big")
    s = int.from_bytes(ipk["proof_s"], "big")
    t1 = g2_add(g2_mul(G2_GEN, s), g2_mul(ipk["w"], (-c) % R))
    t2 = g1_add(g1_mul(ipk["bar_g1"], s), g1_mul(ipk["bar_g2"], (-c) % R))
    data = (g2_bytes(t1) + g1_bytes(t2) + g2_bytes(G2_GEN) + g1_bytes(ipk["bar_g1"]) + g2_bytes(ipk["w"]) +
            g1_bytes(ipk["bar_g2"]))
    return hash_to_zr(data) == c


# -------------------------------------------------------------- nym signatures
def encode_nym_sig(c, s_sk, s_rnym, nonce):
    """NymSignature proto: 1 proof_c, 2 proof_s_sk, 3 proof_s_r_nym, 4 nonce."""
    return b"".join(pb_bytes_field(f, zr_bytes(v)) for f, v in ((1, c), (2, s_sk), (3, s_rnym), (4, nonce)))


def decode_nym_sig(raw, curve=BN254C):
    f = pb_fields(raw)
    return tuple(curve.zr_from_field(_pb_bytes(f, i)) for i in (1, 2, 3, 4))


def make_nym(ipk, sk, r_nym):
    """MakeNym: Nym = HSk^sk * HRand^r_nym."""
    C = ipk["curve"]
    return C.add(C.mul(ipk["h_sk"], sk), C.mul(ipk["h_rand"], r_nym))


def nym_bytes(ipk, nym):
    return ipk["curve"].g1_bytes(nym)


def _challenge(C, t, nym, ipk_hash, msg, nonce):
    data = SIGN_LABEL + C.g1_bytes(t) + C.g1_bytes(nym) + ipk_hash[:32].ljust(32, b"\0") + msg
    c1 = C.hash_to_zr(data)
    return C.hash_to_zr(zr_bytes(c1) + zr_bytes(nonce))


def nym_sign(ipk, sk, nym, r_nym, msg, rng):
    """NewNymSignature with randomness from `rng` (random.Random; fixtures only)."""
    C = ipk["curve"]
    nonce, r_sk, r_r = (rng.randrange(C.r) for _ in range(3))
    t = C.add(C.mul(ipk["h_sk"], r_sk), C.mul(ipk["h_rand"], r_r))
    c = _challenge(C, t, nym, ipk["hash"], msg, nonce)
    return encode_nym_sig(c, (r_sk + c * sk) % C.r, (r_r + c * r_nym) % C.r, nonce)


class NymError(ValueError):
    pass


def nym_verify(ipk, nym_bytes, sig, msg):
    """NymSignatureVerifier.Verify(message, sigma) (id.go:151): None or NymError."""
    # error classes (the library's status strings; the Go error chains append
    # proto / point details that are not part of the verdict)
    if len(sig) == 0:  # bccsp: an empty signature is rejected before Unmarshal
        raise NymError(MSG_MALFORMED)
    C = ipk["curve"]
    try:
        c, s_sk, s_r, nonce = decode_nym_sig(sig, C)
    except ValueError:
        raise NymError(MSG_MALFORMED)
    if nonce >> 256:  # mathlib BigToBytes panics on a Zr wider than 32 bytes
        raise NymError(MSG_MALFORMED)
    try:
        nym = C.g1_from_bytes(nym_bytes)
    except PointError:
        raise NymError(MSG_BADKEY)
    t = C.add(C.add(C.mul(ipk["h_sk"], s_sk), C.mul(ipk["h_rand"], s_r)), C.neg(C.mul(nym, c)))
    if c != _challenge(C, t, nym, ipk["hash"], msg, nonce):
        raise NymError(MSG_INVALID)


def identity_nym(raw):
    """SerializedIdemixIdentity.nym_public_key (idemix_config.proto field 1)."""
    return _pb_bytes(pb_fields(raw), 1)


def serialize_identity(nym_bytes, ou=b"", role=b"", proof=b""):
    return b"".join(pb_bytes_field(f, v) for f, v in ((1, nym_bytes), (2, ou), (3, role), (4, proof)) if v)
