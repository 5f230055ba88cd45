"""BN254 arithmetic restated in pure Python (oracle; test infrastructure only).

Restates the semantics of the mathlib/gnark-crypto calls used on the
verification path (SURVEY §8c "What must the CPU restatement follow"):

* ``G1.Mul(s)``       -> (s mod r)·P, canonical affine result
* ``G1.Add/Sub``      -> affine group law, canonical affine result
* ``G1.Bytes()``      -> 64 bytes X||Y big-endian; the identity is 64 zero bytes
* ``NewG1FromBytes``  -> 64 bytes, coordinates < p, top two flag bits 0, on curve
* ``Curve.HashToZr``  -> SHA-256(m) as a big-endian integer mod r   [PINNED by the
                         idemix IssuerPublicKey hash fields, tests/test_idemix_oracle.py]
* ``Zr.Bytes()``      -> 32-byte big-endian of (z mod r)            [PINNED, same test]
* ``Curve.HashToG1``  -> RFC 9380 hash_to_curve, expand_message_xmd(SHA-256),
                         empty DST, SVDW map with Z = 1              [PINNED by KAT-1]

Points are ``None`` (identity) or ``(x, y)`` tuples of ints.
"""
import hashlib

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
B = 3
GEN = (1, 2)


# --------------------------------------------------------------------- Fp
def finv(a, m=P):
    return pow(a % m, m - 2, m) if a % m else 0


def fsqrt(a):
    """sqrt in Fp (p = 3 mod 4); returns None for non-residues."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def sgn0(a):
    return (a % P) & 1


# --------------------------------------------------------------------- G1
def on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B) % P == 0


def _to_jac(pt):
    return (0, 1, 0) if pt is None else (pt[0], pt[1], 1)


def _from_jac(j):
    x, y, z = j
    if z % P == 0:
        return None
    zi = finv(z)
    zi2 = zi * zi % P
    return (x * zi2 % P, y * zi2 * zi % P)


def _jdbl(j):
    x, y, z = j
    if z == 0 or y == 0:
        return (0, 1, 0)
    a = x * x % P
    b = y * y % P
    c = b * b % P
    d = 2 * ((x + b) * (x + b) - a - c) % P
    e = 3 * a % P
    f = e * e % P
    x3 = (f - 2 * d) % P
    y3 = (e * (d - x3) - 8 * c) % P
    z3 = 2 * y * z % P
    return (x3, y3, z3)


def _jadd(j1, j2):
    x1, y1, z1 = j1
    x2, y2, z2 = j2
    if z1 == 0:
        return j2
    if z2 == 0:
        return j1
    z1z1 = z1 * z1 % P
    z2z2 = z2 * z2 % P
    u1 = x1 * z2z2 % P
    u2 = x2 * z1z1 % P
    s1 = y1 * z2 * z2z2 % P
    s2 = y2 * z1 * z1z1 % P
    if u1 == u2:
        if s1 == s2:
            return _jdbl(j1)
        return (0, 1, 0)
    h = (u2 - u1) % P
    i = 4 * h * h % P
    jj = h * i % P
    rr = 2 * (s2 - s1) % P
    v = u1 * i % P
    x3 = (rr * rr - jj - 2 * v) % P
    y3 = (rr * (v - x3) - 2 * s1 * jj) % P
    z3 = ((z1 + z2) * (z1 + z2) - z1z1 - z2z2) * h % P
    return (x3, y3, z3)


def g1_add(a, b):
    return _from_jac(_jadd(_to_jac(a), _to_jac(b)))


def g1_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def g1_sub(a, b):
    return g1_add(a, g1_neg(b))


def g1_mul(pt, k):
    """(k mod r)·pt, canonical affine (mathlib G1.Mul)."""
    k %= R
    if pt is None or k == 0:
        return None
    acc = (0, 1, 0)
    base = _to_jac(pt)
    for bit in bin(k)[2:]:
        acc = _jdbl(acc)
        if bit == "1":
            acc = _jadd(acc, base)
    return _from_jac(acc)


def g1_msm(points, scalars):
    acc = (0, 1, 0)
    for pt, k in zip(points, scalars):
        m = g1_mul(pt, k)
        acc = _jadd(acc, _to_jac(m))
    return _from_jac(acc)


def g1_bytes(pt):
    if pt is None:
        return bytes(64)
    return pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


class PointError(ValueError):
    pass


def g1_from_bytes(b):
    """NewG1FromBytes: 64-byte uncompressed; zeros = identity."""
    if len(b) != 64:
        raise PointError("invalid point length")
    if b[0] & 0xC0:
        raise PointError("invalid point encoding flags")
    x = int.from_bytes(b[:32], "big")
    y = int.from_bytes(b[32:], "big")
    if x >= P or y >= P:
        raise PointError("non-canonical coordinate")
    if x == 0 and y == 0:
        return None
    if not on_curve((x, y)):
        raise PointError("point not on curve")
    return (x, y)


# --------------------------------------------------------------------- Zr
def zr_bytes(z):
    return (z % R).to_bytes(32, "big")


def zr_from_bytes(b):
    """NewZrFromBytes: big-endian integer, NOT reduced (mathlib BaseZr)."""
    return int.from_bytes(b, "big")


def hash_to_zr(m):
    return int.from_bytes(hashlib.sha256(m).digest(), "big") % R


# --------------------------------------------------------------- hash to G1
def _expand_message_xmd(msg, dst, n):
    ell = (n + 31) // 32
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(64) + msg + n.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:n]


# SVDW constants for y^2 = x^3 + 3 with Z = 1 (RFC 9380 §6.6.1)
_Z = 1
_C1 = (_Z ** 3 + B) % P                      # g(Z)
_C2 = (-_Z * finv(2)) % P                    # -Z/2
_C3 = fsqrt((-_C1 * (3 * _Z * _Z)) % P)      # sqrt(-g(Z)(3Z^2 + 4A)), sgn0 = 0
if _C3 is not None and sgn0(_C3) == 1:
    _C3 = P - _C3
_C4 = (-4 * _C1 * finv(3 * _Z * _Z)) % P     # -4 g(Z) / (3Z^2 + 4A)


def _g(x):
    return (x * x * x + B) % P


def map_to_curve_svdw(u):
    tv1 = u * u % P * _C1 % P
    tv2 = (1 + tv1) % P
    tv1 = (1 - tv1) % P
    tv3 = finv(tv1 * tv2 % P)
    tv4 = u * tv1 % P * tv3 % P * _C3 % P
    x1 = (_C2 - tv4) % P
    e1 = is_square(_g(x1))
    x2 = (_C2 + tv4) % P
    e2 = is_square(_g(x2)) and not e1
    x3 = tv2 * tv2 % P * tv3 % P
    x3 = x3 * x3 % P * _C4 % P
    x3 = (x3 + _Z) % P
    x = x1 if e1 else (x2 if e2 else x3)
    y = fsqrt(_g(x))
    if sgn0(u) != sgn0(y):
        y = (-y) % P
    return (x, y)


def hash_to_g1(msg, dst=b""):
    """mathlib Curve.HashToG1 for BN254 (KAT-1 pinned)."""
    ub = _expand_message_xmd(msg, dst, 96)
    u0 = int.from_bytes(ub[:48], "big") % P
    u1 = int.from_bytes(ub[48:], "big") % P
    return g1_add(map_to_curve_svdw(u0), map_to_curve_svdw(u1))
