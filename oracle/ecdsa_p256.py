"""ECDSA P-256 verification restated in pure Python (oracle; TEST INFRASTRUCTURE
ONLY — imported by tests/ and bench.py's cpu_baseline leg, never by the
product path).

Follows the reference's owner-signature verifier line by line:

* ``Verifier.Verify``  validator/ecdsa/ecdsa.go:82-113 (same logic:
  services/identity/x509/crypto/ecdsa.go:46-77)
    1. ``asn1.Unmarshal(sigma, &Signature{R, S})``   -> ``parse_sig`` (Go
       encoding/asn1 rules: DER-minimal lengths, minimally encoded two's
       complement INTEGERs, trailing bytes after the SEQUENCE and extra
       elements inside it ignored)
    2. ``digest = sha256(message)``
    3. ``IsLowS``  ecdsa.go:152-161: ``s <= n/2`` else "signature is not in lowS"
    4. ``ecdsa.Verify`` (Go crypto/ecdsa, FIPS 186-4 §6.4.2; not vendored):
       0 < r, s < n; e = digest as an integer; w = s^-1; u1 = e*w; u2 = r*w;
       X = u1*G + u2*Q; reject X = O; accept iff X.x mod n == r.  An
       off-curve public key makes Verify return false.

Parity is pinned by ``tests/golden/ecdsa_golden.json``: signatures produced
by OpenSSL (an independent implementation) over P-256/SHA-256, see
``tests/golden/make_ecdsa_golden.sh``.
"""
import hashlib

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
G = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
     0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)
HALF_N = N >> 1

OK, SIG_MALFORMED, SIG_NOT_LOW_S, SIG_INVALID = 0, 13, 14, 15


def on_curve(pt):
    x, y = pt
    return 0 <= x < P and 0 <= y < P and (y * y - (x * x * x - 3 * x + B)) % P == 0


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = (3 * a[0] * a[0] - 3) * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return (x, (lam * (a[0] - x) - a[1]) % P)


def mul(k, pt):
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = _add(acc, acc)
        if bit == "1":
            acc = _add(acc, pt)
    return acc


def _tl(b, off, tag):
    """Go asn1 parseTagAndLength for a single-byte tag -> (body_off, body_len)."""
    if off >= len(b) or b[off] != tag:
        raise ValueError("tag")
    off += 1
    if off >= len(b):
        raise ValueError("truncated")
    l0 = b[off]
    off += 1
    if l0 & 0x80 == 0:
        L = l0
    else:
        nb = l0 & 0x7F
        if nb == 0:
            raise ValueError("indefinite length")
        L = 0
        for _ in range(nb):
            if off >= len(b):
                raise ValueError("truncated")
            if L >= 1 << 23:
                raise ValueError("length too large")
            L = (L << 8) | b[off]
            off += 1
            if L == 0:
                raise ValueError("superfluous leading zeros in length")
        if L < 0x80:
            raise ValueError("non-minimal length")
    if L > len(b) - off:
        raise ValueError("data truncated")
    return off, L


def _int(body):
    if len(body) == 0:
        raise ValueError("empty integer")
    if len(body) > 1 and ((body[0] == 0 and body[1] & 0x80 == 0) or (body[0] == 0xFF and body[1] & 0x80)):
        raise ValueError("integer not minimally-encoded")
    return int.from_bytes(body, "big", signed=True)


def parse_sig(sig):
    """asn1.Unmarshal(sigma, &Signature{}) -> (r, s); raises ValueError."""
    o, L = _tl(sig, 0, 0x30)
    inner = sig[o:o + L]
    ro, rl = _tl(inner, 0, 0x02)
    so, sl = _tl(inner, ro + rl, 0x02)
    return _int(inner[ro:ro + rl]), _int(inner[so:so + sl])


def verify(msg, sig, pk):
    """Verifier.Verify(message, sigma) with pk = (x, y) -> status code."""
    try:
        r, s = parse_sig(sig)
    except ValueError:
        return SIG_MALFORMED
    e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    if s > HALF_N:
        return SIG_NOT_LOW_S
    if not (0 < r < N and 0 < s < N) or not on_curve(pk):
        return SIG_INVALID
    w = pow(s, -1, N)
    X = _add(mul(e * w % N, G), mul(r * w % N, pk))
    if X is None or X[0] % N != r:
        return SIG_INVALID
    return OK


def der_sig(r, s):
    """utils.MarshalECDSASignature(r, s) for r, s > 0 (minimal DER)."""
    def enc(v):
        b = v.to_bytes((v.bit_length() + 8) // 8, "big")
        return b"\x02" + bytes([len(b)]) + b
    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


def sign(d, msg, k):
    """Deterministic-nonce signer for synthetic data (low-S normalised as
    Signer.Sign does, ecdsa.go:49-63)."""
    e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    R = mul(k, G)
    r = R[0] % N
    s = pow(k, -1, N) * (e + r * d) % N
    if s > HALF_N:
        s = N - s
    return der_sig(r, s)
