"""Step-for-step Python model of the DEVICE pairing (csrc/device/pairing.hpp):
tower arithmetic, precomputed affine line coefficients, sparse line products,
multi-Miller loop, Frobenius maps and the u-chain final exponentiation.
ORACLE / TEST INFRASTRUCTURE ONLY (never imported by the product path).

It is checked against oracle/pairing.py (the direct E(Fp12) restatement, itself
pinned by the reference's credential fixtures) in tests/test_pairing_cpu.py, and
the device kernels are checked against it value for value (Miller output and
GT) through fts_idemix_pairing_debug.

Tower: Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v).
Lines through twist points T, R (slope lam, mu = lam x_T - y_T) at P = (xP, yP):
  D-type: l         = yP + (-lam xP) w + mu v w        (c0 = (yP,0,0), c1 = (-lam xP, mu, 0))
  M-type: l * w^3   = mu + (-lam xP) v + yP v w         (c0 = (mu, -lam xP, 0), c1 = (0, yP, 0))
(factors in Fp2 and w^3 vanish in the final exponentiation).
Final exponentiation: f^(p^6-1) = conj(f)/f, then ^(p^2+1), then the hard part
f^((p^4-p^2+1)/r) = y0 y1^2 y2^6 y3^12 y4^18 y5^30 y6^36 (Scott et al.'s BN
decomposition lambda_3 p^3 + lambda_2 p^2 + lambda_1 p + lambda_0, valid for
either sign of u), with the addition chain of the device code.
"""
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


class Tower:
    def __init__(self, C):
        import pairing_constants as pc
        self.C, self.p = C, C.p
        self.k = pc.constants(C)

    # ---------------------------------------------------------------- Fp2
    def a2(self, a, b):
        return ((a[0] + b[0]) % self.p, (a[1] + b[1]) % self.p)

    def s2(self, a, b):
        return ((a[0] - b[0]) % self.p, (a[1] - b[1]) % self.p)

    def m2(self, a, b):
        p = self.p
        return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)

    def n2(self, a):
        return ((-a[0]) % self.p, (-a[1]) % self.p)

    def sc2(self, a, s):
        return (a[0] * s % self.p, a[1] * s % self.p)

    def cj2(self, a):
        return (a[0], (-a[1]) % self.p)

    def xi(self, a):
        x0, x1 = self.C.xi
        p = self.p
        return ((a[0] * x0 - a[1] * x1) % p, (a[0] * x1 + a[1] * x0) % p)

    def inv2(self, a):
        p = self.p
        n = pow((a[0] * a[0] + a[1] * a[1]) % p, p - 2, p)
        return (a[0] * n % p, (-a[1]) * n % p)

    Z2 = (0, 0)
    O2 = (1, 0)

    # ---------------------------------------------------------------- Fp6
    def a6(self, a, b):
        return tuple(self.a2(x, y) for x, y in zip(a, b))

    def s6(self, a, b):
        return tuple(self.s2(x, y) for x, y in zip(a, b))

    def n6(self, a):
        return tuple(self.n2(x) for x in a)

    def m6(self, a, b):
        t0, t1, t2 = self.m2(a[0], b[0]), self.m2(a[1], b[1]), self.m2(a[2], b[2])
        c0 = self.a2(t0, self.xi(self.s2(self.s2(self.m2(self.a2(a[1], a[2]), self.a2(b[1], b[2])), t1), t2)))
        c1 = self.a2(self.s2(self.s2(self.m2(self.a2(a[0], a[1]), self.a2(b[0], b[1])), t0), t1), self.xi(t2))
        c2 = self.a2(self.s2(self.s2(self.m2(self.a2(a[0], a[2]), self.a2(b[0], b[2])), t0), t2), t1)
        return (c0, c1, c2)

    def mv6(self, a):
        return (self.xi(a[2]), a[0], a[1])

    def sc6(self, a, s):
        return tuple(self.sc2(x, s) for x in a)

    def m6_01(self, a, A, B):
        """a * (A + B v)"""
        c0 = self.a2(self.m2(a[0], A), self.xi(self.m2(a[2], B)))
        c1 = self.a2(self.m2(a[0], B), self.m2(a[1], A))
        c2 = self.a2(self.m2(a[1], B), self.m2(a[2], A))
        return (c0, c1, c2)

    def inv6(self, a):
        a0, a1, a2 = a
        c0 = self.s2(self.m2(a0, a0), self.xi(self.m2(a1, a2)))
        c1 = self.s2(self.xi(self.m2(a2, a2)), self.m2(a0, a1))
        c2 = self.s2(self.m2(a1, a1), self.m2(a0, a2))
        t = self.a2(self.m2(a0, c0), self.xi(self.a2(self.m2(a2, c1), self.m2(a1, c2))))
        ti = self.inv2(t)
        return (self.m2(c0, ti), self.m2(c1, ti), self.m2(c2, ti))

    # --------------------------------------------------------------- Fp12
    def one(self):
        return ((self.O2, self.Z2, self.Z2), (self.Z2, self.Z2, self.Z2))

    def m12(self, a, b):
        t0, t1 = self.m6(a[0], b[0]), self.m6(a[1], b[1])
        c0 = self.a6(t0, self.mv6(t1))
        c1 = self.s6(self.s6(self.m6(self.a6(a[0], a[1]), self.a6(b[0], b[1])), t0), t1)
        return (c0, c1)

    def sq12(self, a):
        t = self.m6(a[0], a[1])
        c0 = self.s6(self.s6(self.m6(self.a6(a[0], a[1]), self.a6(a[0], self.mv6(a[1]))), t), self.mv6(t))
        return (c0, self.a6(t, t))

    def cyc_sq12(self, a):
        """Granger-Scott squaring in the cyclotomic subgroup: Fp12 = Fp4[w]/(w^3 - s),
        s = w^3, s^2 = xi; A = z0 + z3 s, B = z1 + z4 s, C = z2 + z5 s;
        f^2 = (3A^2 - 2 conj A) + (3 s C^2 + 2 conj B) w + (3B^2 - 2 conj C) w^2"""
        z = self._zs(a)

        def sq4(x0, x1):  # (x0 + x1 s)^2 = (x0^2 + xi x1^2) + 2 x0 x1 s
            t0, t1 = self.m2(x0, x0), self.m2(x1, x1)
            t2 = self.s2(self.s2(self.m2(self.a2(x0, x1), self.a2(x0, x1)), t0), t1)
            return self.a2(t0, self.xi(t1)), t2
        a0, a1 = sq4(z[0], z[3])
        b0, b1 = sq4(z[1], z[4])
        c0, c1 = sq4(z[2], z[5])
        three = lambda x: self.a2(self.a2(x, x), x)  # noqa: E731
        two = lambda x: self.a2(x, x)  # noqa: E731
        # A' = 3A^2 - 2 conj(A): (3a0 - 2z0, 3a1 + 2z3)
        n0, n3 = self.s2(three(a0), two(z[0])), self.a2(three(a1), two(z[3]))
        # B' = 3 s C^2 + 2 conj(B): s (c0 + c1 s) = xi c1 + c0 s
        n1, n4 = self.a2(three(self.xi(c1)), two(z[1])), self.s2(three(c0), two(z[4]))
        # C' = 3B^2 - 2 conj(C)
        n2, n5 = self.s2(three(b0), two(z[2])), self.a2(three(b1), two(z[5]))
        return self._from_zs([n0, n1, n2, n3, n4, n5])

    def cj12(self, a):
        return (a[0], self.n6(a[1]))

    def inv12(self, a):
        t = self.s6(self.m6(a[0], a[0]), self.mv6(self.m6(a[1], a[1])))
        ti = self.inv6(t)
        return (self.m6(a[0], ti), self.n6(self.m6(a[1], ti)))

    def _zs(self, a):
        return [a[0][0], a[1][0], a[0][1], a[1][1], a[0][2], a[1][2]]

    def _from_zs(self, z):
        return ((z[0], z[2], z[4]), (z[1], z[3], z[5]))

    def frob(self, a, n):
        """a^(p^n), n in 1, 2, 3"""
        g = {1: self.k["G1"], 2: self.k["G2"], 3: self.k["G3"]}[n]
        z = self._zs(a)
        out = []
        for i, zi in enumerate(z):
            if n != 2:
                zi = self.cj2(zi)
            out.append(zi if i == 0 else self.m2(zi, g[i]))
        return self._from_zs(out)

    # --------------------------------------------------------- lines
    def lines(self, Q):
        """precomputed (lam, mu) of every Miller step for the twist point Q (affine)"""
        out = []
        T = Q
        bits = bin(abs(self.k["ate"]))[3:]

        def step(T, R):
            if T == R:
                lam = self.m2(self.sc2(self.m2(T[0], T[0]), 3), self.inv2(self.sc2(T[1], 2)))
            else:
                lam = self.m2(self.s2(R[1], T[1]), self.inv2(self.s2(R[0], T[0])))
            mu = self.s2(self.m2(lam, T[0]), T[1])
            x = self.s2(self.s2(self.m2(lam, lam), T[0]), R[0])
            y = self.s2(self.m2(lam, self.s2(T[0], x)), T[1])
            return (lam, mu), (x, y)
        for b in bits:
            ln, T = step(T, T)
            out.append(ln)
            if b == "1":
                ln, T = step(T, Q)
                out.append(ln)
        if self.k["ate"] < 0:
            T = (T[0], self.n2(T[1]))
        tw = self.k["TW"]
        Q1 = (self.m2(self.cj2(Q[0]), tw[0]), self.m2(self.cj2(Q[1]), tw[1]))
        Q2 = (self.m2(Q[0], tw[2]), self.m2(Q[1], tw[3]))
        Q2n = (Q2[0], self.n2(Q2[1]))
        ln, T = step(T, Q1)
        out.append(ln)
        ln, _ = step(T, Q2n)
        out.append(ln)
        return out

    def line_mul(self, f, ln, P):
        lam, mu = ln
        xP, yP = P
        A = self.n2(self.sc2(lam, xP))
        f0, f1 = f
        if not self.C.twist == "M":
            c0 = self.a6(self.sc6(f0, yP), self.mv6(self.m6_01(f1, A, mu)))
            c1 = self.a6(self.m6_01(f0, A, mu), self.sc6(f1, yP))
        else:
            c0 = self.a6(self.m6_01(f0, mu, A), self.sc6(self.mv6(self.mv6(f1)), yP))
            c1 = self.a6(self.sc6(self.mv6(f0), yP), self.m6_01(f1, mu, A))
        return (c0, c1)

    def miller(self, pairs):
        """multi-Miller loop: pairs = [(lines of Q, P affine in G1)] -> f"""
        bits = bin(abs(self.k["ate"]))[3:]
        f = self.one()
        idx = 0
        first = True
        for b in bits:
            if not first:
                f = self.sq12(f)
            first = False
            for L, P in pairs:
                f = self.line_mul(f, L[idx], P)
            idx += 1
            if b == "1":
                for L, P in pairs:
                    f = self.line_mul(f, L[idx], P)
                idx += 1
        if self.k["ate"] < 0:
            f = self.cj12(f)
        for _ in range(2):
            for L, P in pairs:
                f = self.line_mul(f, L[idx], P)
            idx += 1
        return f

    # ------------------------------------------------------- final exp
    def expt(self, f):
        """f^u (cyclotomic subgroup: inverse = conjugate)"""
        r = f
        for b in bin(abs(self.k["u"]))[3:]:
            r = self.cyc_sq12(r)
            if b == "1":
                r = self.m12(r, f)
        return self.cj12(r) if self.k["u"] < 0 else r

    def final_exp(self, f):
        f = self.m12(self.cj12(f), self.inv12(f))
        f = self.m12(self.frob(f, 2), f)
        fu = self.expt(f)
        fu2 = self.expt(fu)
        fu3 = self.expt(fu2)
        y0 = self.m12(self.m12(self.frob(f, 1), self.frob(f, 2)), self.frob(f, 3))
        y1 = self.cj12(f)
        y2 = self.frob(fu2, 2)
        y3 = self.cj12(self.frob(fu, 1))
        y4 = self.cj12(self.m12(fu, self.frob(fu2, 1)))
        y5 = self.cj12(fu2)
        y6 = self.cj12(self.m12(fu3, self.frob(fu3, 1)))
        t0 = self.m12(self.m12(self.cyc_sq12(y6), y4), y5)
        t1 = self.m12(self.m12(y3, y5), t0)
        t0 = self.m12(t0, y2)
        t1 = self.m12(self.cyc_sq12(t1), t0)
        t1 = self.cyc_sq12(t1)
        t0 = self.m12(t1, y1)
        t1 = self.m12(t1, y0)
        t0 = self.cyc_sq12(t0)
        return self.m12(t0, t1)

    # ------------------------------------------------------- helpers
    def to_poly(self, a):
        """tower element -> oracle/pairing.py's Fp[w] representation"""
        C = self.C
        out = C.f12([])
        w = C.f12([0, 1])
        wk = C.one()
        for z in self._zs(a):
            out = C.add(out, C.mul(C.from_f2(z), wk))
            wk = C.mul(wk, w)
        return out
