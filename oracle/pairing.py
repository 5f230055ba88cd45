"""Optimal-ate pairing on the two BN curves of the idemix identity proof
(BN254 = gnark-crypto bn254, FP256BN = AMCL FP256BN), restated in pure Python.
ORACLE / TEST INFRASTRUCTURE ONLY: never imported by the product path.

Where it is used (fabric-token-sdk, reference paths):
* services/identity/idemix/crypto/id.go:74-108 Identity.verifyProof ->
  CSP.Verify(IssuerPublicKey, AssociationProof, IdemixSignerOpts) -> IBM/idemix
  Signature.Ver (github.com/IBM/idemix v0.0.2-0.20240816143710-3dce4618d760,
  go.mod:6, NOT vendored): the pairing check
      e(W, A') == e(g2, ABar)
  of a randomised BBS+ credential, and IBM/idemix Credential.Ver (checked by
  services/identity/idemix/km.go:117-135 when a SignerConfig is loaded):
      e(W + g2 * E, A) == e(g2, B).
  mathlib (github.com/IBM/mathlib) delegates BN254 to gnark-crypto and
  FP256BN_AMCL to the AMCL (fabric-amcl) FP256BN package; neither is vendored.

Only equalities of FExp(pairings) are ever tested, so any non-degenerate
bilinear pairing gives the reference's verdicts; this module computes the
optimal ate pairing, the same function the device kernels compute, so their
GT values can be compared directly.

Representation: Fp12 = Fp[w] / (w^12 - 2 xi0 w^6 + xi0^2 + xi1^2) (w^6 = xi =
xi0 + xi1 i, i^2 = -1); G2 points of the sextic twist are untwisted into E(Fp12)
(D-type: (x w^2, y w^3); M-type: (x / w^2, y / w^3)) and the Miller loop runs
with affine chord/tangent lines there.  Slow (~0.3 s per pairing) but direct.

PINNED (tests/test_idemix_identity_oracle.py) by the reference's own credential
fixtures: the charlie.ExtraId2 SignerConfig (BN254) and the zkatdlog validator's
SignerConfig (FP256BN) each hold a credential (A, B, E, S, attributes) and the
user secret Sk under an IssuerPublicKey the reference ships; B is recomputed from
them and the pairing equation above holds, for both curves -- this pins the
curves' twists, their G2 encodings (gnark raw / AMCL xa||xb||ya||yb), and the G2
generators (idemix writes GenG2 as the dummy epoch key of a no-revocation CRI,
also in those SignerConfigs).
"""

# ------------------------------------------------------------------ curves


class BNCurve:
    def __init__(self, name, u, xi, twist, g2_gen, b=3):
        self.name, self.u, self.xi, self.twist, self.b = name, u, xi, twist, b
        self.p = 36 * u ** 4 + 36 * u ** 3 + 24 * u ** 2 + 6 * u + 1
        self.r = 36 * u ** 4 + 36 * u ** 3 + 18 * u ** 2 + 6 * u + 1
        p = self.p
        x0, x1 = xi
        # w^12 = 2 x0 w^6 - (x0^2 + x1^2)
        self.mod_c6, self.mod_c0 = (2 * x0) % p, (-(x0 * x0 + x1 * x1)) % p
        self.inv_x1 = pow(x1, p - 2, p)
        self.g2_gen = g2_gen
        self.g1_gen = (1, 2)
        self.ate = 6 * u + 2
        # twist b' = b / xi (D-type) or b * xi (M-type)
        if twist == "D":
            self.b2 = f2mul((b, 0), f2inv(xi, p), p)
        else:
            self.b2 = f2mul((b, 0), xi, p)

    # -------------------------------------------------------------- Fp12
    def f12(self, coeffs):
        c = [v % self.p for v in coeffs] + [0] * (12 - len(coeffs))
        return tuple(c)

    def one(self):
        return self.f12([1])

    def mul(self, a, b):
        p = self.p
        t = [0] * 23
        for i, ai in enumerate(a):
            if ai:
                for j, bj in enumerate(b):
                    if bj:
                        t[i + j] += ai * bj
        for k in range(22, 11, -1):  # w^k = w^(k-12) (c6 w^6 + c0)
            v = t[k] % p
            if v:
                t[k - 6] += v * self.mod_c6
                t[k - 12] += v * self.mod_c0
        return tuple(x % p for x in t[:12])

    def add(self, a, b):
        return tuple((x + y) % self.p for x, y in zip(a, b))

    def sub(self, a, b):
        return tuple((x - y) % self.p for x, y in zip(a, b))

    def scal(self, a, k):
        return tuple(x * k % self.p for x in a)

    def pow(self, a, e):
        r, base = self.one(), a
        while e:
            if e & 1:
                r = self.mul(r, base)
            base = self.mul(base, base)
            e >>= 1
        return r

    def inv(self, a):
        """extended Euclid over Fp[w] against the modulus polynomial"""
        p = self.p
        mod = [self.mod_c0 * -1 % p] + [0] * 5 + [(-self.mod_c6) % p] + [0] * 5 + [1]  # w^12 - c6 w^6 - c0
        lm, hm = [1] + [0] * 12, [0] * 13
        low, high = list(a) + [0], mod[:]

        def deg(v):
            d = len(v) - 1
            while d and v[d] % p == 0:
                d -= 1
            return d
        while deg(low):
            r = _poly_div(high, low, p)
            r += [0] * (13 - len(r))
            nm, new = hm[:], high[:]
            for i in range(13):
                for j in range(13 - i):
                    nm[i + j] -= lm[i] * r[j]
                    new[i + j] -= low[i] * r[j]
            nm = [x % p for x in nm]
            new = [x % p for x in new]
            lm, low, hm, high = nm, new, lm, low
        c = pow(low[0], p - 2, p)
        return tuple(x * c % p for x in lm[:12])

    def conj(self, a):
        """a^(p^6): w -> -w (odd powers negated)"""
        return tuple(v if i % 2 == 0 else (-v) % self.p for i, v in enumerate(a))

    def from_f2(self, z):
        """a + b i -> Fp12, i = (w^6 - xi0) / xi1"""
        a, b = z
        t = b * self.inv_x1 % self.p
        c = [0] * 12
        c[0] = (a - t * self.xi[0]) % self.p
        c[6] = t
        return tuple(c)

    # ---------------------------------------------------- E(Fp12) points
    def untwist(self, Q):
        x, y = self.from_f2(Q[0]), self.from_f2(Q[1])
        w2, w3 = self.f12([0, 0, 1]), self.f12([0, 0, 0, 1])
        if self.twist == "D":
            return self.mul(x, w2), self.mul(y, w3)
        return self.mul(x, self.inv(w2)), self.mul(y, self.inv(w3))

    def embed_g1(self, P):
        return self.f12([P[0]]), self.f12([P[1]])

    def pt_add(self, A, B):
        if A is None:
            return B
        if B is None:
            return A
        if A[0] == B[0]:
            if self.add(A[1], B[1]) == self.f12([]):
                return None
            lam = self.mul(self.scal(self.mul(A[0], A[0]), 3), self.inv(self.scal(A[1], 2)))
        else:
            lam = self.mul(self.sub(B[1], A[1]), self.inv(self.sub(B[0], A[0])))
        x = self.sub(self.sub(self.mul(lam, lam), A[0]), B[0])
        return x, self.sub(self.mul(lam, self.sub(A[0], x)), A[1])

    def pt_neg(self, A):
        return None if A is None else (A[0], self.scal(A[1], self.p - 1))

    def frob(self, A):
        return self.pow(A[0], self.p), self.pow(A[1], self.p)

    def line(self, A, B, P):
        """the line through A and B (tangent if equal) evaluated at P"""
        xp, yp = P
        if A[0] == B[0] and A[1] != B[1]:
            return self.sub(xp, A[0])  # vertical
        if A[0] == B[0]:
            lam = self.mul(self.scal(self.mul(A[0], A[0]), 3), self.inv(self.scal(A[1], 2)))
        else:
            lam = self.mul(self.sub(B[1], A[1]), self.inv(self.sub(B[0], A[0])))
        return self.sub(self.sub(yp, A[1]), self.mul(lam, self.sub(xp, A[0])))

    # -------------------------------------------------------- pairing
    def miller(self, Q, P):
        """optimal ate Miller value f (before the final exponentiation); Q on the
        twist (Fp2 pair), P in G1; both not the identity"""
        Qe, Pe = self.untwist(Q), self.embed_g1(P)
        s = self.ate
        T, f = Qe, self.one()
        for bit in bin(abs(s))[3:]:
            f = self.mul(self.mul(f, f), self.line(T, T, Pe))
            T = self.pt_add(T, T)
            if bit == "1":
                f = self.mul(f, self.line(T, Qe, Pe))
                T = self.pt_add(T, Qe)
        if s < 0:  # f_{-n} = 1 / f_n up to a vertical line (killed by the final exponentiation)
            f = self.inv(f)
            T = self.pt_neg(T)
        Q1 = self.frob(Qe)
        Q2n = self.pt_neg(self.frob(Q1))
        f = self.mul(f, self.line(T, Q1, Pe))
        T = self.pt_add(T, Q1)
        return self.mul(f, self.line(T, Q2n, Pe))

    def final_exp(self, f):
        f = self.mul(self.conj(f), self.inv(f))                 # ^(p^6 - 1)
        f = self.mul(self.pow(f, self.p * self.p), f)           # ^(p^2 + 1)
        return self.pow(f, (self.p ** 4 - self.p ** 2 + 1) // self.r)

    def pairing(self, Q, P):
        """e(Q, P) in GT, or 1 if either argument is the identity (None)"""
        if Q is None or P is None:
            return self.one()
        return self.final_exp(self.miller(Q, P))

    def pairing_product_is_one(self, pairs):
        """prod e(Q_i, P_i) == 1 with ONE final exponentiation"""
        f = self.one()
        for Q, P in pairs:
            if Q is not None and P is not None:
                f = self.mul(f, self.miller(Q, P))
        return self.final_exp(f) == self.one()

    # --------------------------------------------------------- twist G2
    def g2_on_curve(self, Q):
        x, y = Q
        p = self.p
        return f2sub(f2mul(y, y, p), f2add(f2mul(f2mul(x, x, p), x, p), self.b2, p), p) == (0, 0)

    def g2_add(self, A, B):
        p = self.p
        if A is None:
            return B
        if B is None:
            return A
        if A[0] == B[0]:
            if f2add(A[1], B[1], p) == (0, 0):
                return None
            lam = f2mul(f2mul((3, 0), f2mul(A[0], A[0], p), p), f2inv(f2mul((2, 0), A[1], p), p), p)
        else:
            lam = f2mul(f2sub(B[1], A[1], p), f2inv(f2sub(B[0], A[0], p), p), p)
        x = f2sub(f2sub(f2mul(lam, lam, p), A[0], p), B[0], p)
        return x, f2sub(f2mul(lam, f2sub(A[0], x, p), p), A[1], p)

    def g2_mul(self, Q, k):
        acc = None
        for bit in bin(k % self.r)[2:] if k % self.r else "":
            acc = self.g2_add(acc, acc)
            if bit == "1":
                acc = self.g2_add(acc, Q)
        return acc

    def g2_neg(self, Q):
        return None if Q is None else (Q[0], ((-Q[1][0]) % self.p, (-Q[1][1]) % self.p))


def _poly_div(a, b, p):
    """quotient of a / b over Fp (lists, low degree first)"""
    a = [x % p for x in a]

    def deg(v):
        d = len(v) - 1
        while d and v[d] % p == 0:
            d -= 1
        return d
    da, db = deg(a), deg(b)
    q = [0] * (max(da - db, 0) + 1)
    inv_lead = pow(b[db], p - 2, p)
    for i in range(da - db, -1, -1):
        c = a[db + i] * inv_lead % p
        q[i] = c
        if c:
            for j in range(db + 1):
                a[i + j] = (a[i + j] - c * b[j]) % p
    return q


def f2add(a, b, p):
    return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)


def f2sub(a, b, p):
    return ((a[0] - b[0]) % p, (a[1] - b[1]) % p)


def f2mul(a, b, p):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def f2inv(a, p):
    n = pow((a[0] * a[0] + a[1] * a[1]) % p, p - 2, p)
    return (a[0] * n % p, (-a[1]) * n % p)


# gnark-crypto bn254: u = 4965661367192848881, xi = 9 + i, D-type twist
BN254 = BNCurve(
    "BN254", 4965661367192848881, (9, 1), "D",
    ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
      11559732032986387107991004021392285783925812861821192530917403151452391805634),
     (8495653923123431417604973247489272438418190587263600148770280649306958101930,
      4082367875863433681332203403145435568316851327593401208105741076214120093531)))

# AMCL FP256BN: u = -0x6882F5C030B0A801, xi = 1 + i, M-type twist; the G2
# generator is the dummy epoch key of the validator fixture's CRI (pinned by the
# credential equation, tests/test_idemix_identity_oracle.py)
FP256BN = BNCurve(
    "FP256BN", -0x6882F5C030B0A801, (1, 1), "M",
    ((0xFE0C3350B4C96C2028560F577C28913ACE1C539A12BF843CD22616B689C09EFB,
      0x4EA66057738AC054DB5AE1C637D813B924DD78E287D03589D269ED34A37E6A2B),
     (0x702046E7C542A3B376770D75124E3E51EFCB24758D615848E909B481BEDC27FF,
      0x0554E3BCD388C29042EEA649297EB29F8B4CBE80821A98B3E01281114AAD049B)))
