// NIST P-256 (secp256r1) arithmetic on gfx950 for batched ECDSA verification
// of owner signatures: 8 x 32-bit limbs, Montgomery form (R = 2^256), one
// signature per lane.
//
// Reference: validator/ecdsa/ecdsa.go:82-113 (Verifier.Verify) and
// services/identity/x509/crypto/ecdsa.go:46-77 both end in Go's
// crypto/ecdsa.Verify(pk, sha256(msg), r, s) on elliptic.P256().  Go's
// implementation (crypto/internal/nistec) is not vendored; the semantics
// restated here are the published ones (FIPS 186-4 section 6.4.2):
//   w = s^-1 mod n, u1 = e*w, u2 = r*w, X = u1*G + u2*Q, accept iff
//   X != O and X.x mod n == r.
//
// Unlike the BN254 fields (field.hpp), both P-256 moduli use the full 256
// bits, so this is the textbook CIOS with a 9th/10th carry word and an add
// with carry-out.  Curve a = -3: doubling is dbl-2001-b (3M + 5S).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"  // fts::mac96 / mac96s (96-bit column accumulators)

#ifndef FTS_DEV
#define FTS_DEV __device__ __forceinline__
#endif

namespace p256 {

struct PM {  // field prime p = 2^256 - 2^224 + 2^192 + 2^96 - 1
  static constexpr uint32_t M[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                    0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};
  static constexpr uint32_t INV = 0x00000001u;  // -p^-1 mod 2^32
  static constexpr uint32_t ONE[8] = {0x00000001u, 0x00000000u, 0x00000000u, 0xffffffffu,
                                      0xffffffffu, 0xffffffffu, 0xfffffffeu, 0x00000000u};
  static constexpr uint32_t R2[8] = {0x00000003u, 0x00000000u, 0xffffffffu, 0xfffffffbu,
                                     0xfffffffeu, 0xffffffffu, 0xfffffffdu, 0x00000004u};
  static constexpr uint32_t EXP_INV[8] = {0xfffffffdu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                          0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};  // p - 2
};

struct NM {  // group order n
  static constexpr uint32_t M[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                    0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
  static constexpr uint32_t INV = 0xee00bc4fu;
  static constexpr uint32_t ONE[8] = {0x039cdaafu, 0x0c46353du, 0x58e8617bu, 0x43190552u,
                                      0x00000000u, 0x00000000u, 0xffffffffu, 0x00000000u};
  static constexpr uint32_t R2[8] = {0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu,
                                     0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u};
  static constexpr uint32_t EXP_INV[8] = {0xfc63254fu, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                          0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};  // n - 2
};

// curve constants in Montgomery form (mod p)
__device__ constexpr uint32_t CB[8] = {0x29c4bddfu, 0xd89cdf62u, 0x78843090u, 0xacf005cdu,
                                       0xf7212ed6u, 0xe5a220abu, 0x04874834u, 0xdc30061du};
__device__ constexpr uint32_t CGX[8] = {0x18a9143cu, 0x79e730d4u, 0x5fedb601u, 0x75ba95fcu,
                                        0x77622510u, 0x79fb732bu, 0xa53755c6u, 0x18905f76u};
__device__ constexpr uint32_t CGY[8] = {0xce95560au, 0xddf25357u, 0xba19e45cu, 0x8b4ab8e4u,
                                        0xdd21f325u, 0xd2e88688u, 0x25885d85u, 0x8571ff18u};
// p - n (plain): r + n < p  <=>  r < p - n
__device__ constexpr uint32_t P_MINUS_N[8] = {0x039cdaaeu, 0x0c46353du, 0x58e8617bu, 0x43190553u, 0, 0, 0, 0};

template <class P>
struct F {
  uint32_t v[8];
};
using Fp = F<PM>;
using Fn = F<NM>;

template <class P>
FTS_DEV F<P> load(const uint32_t* s) {
  F<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = s[i];
  return r;
}
template <class P>
FTS_DEV bool is_zero(const F<P>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i];
  return o == 0;
}
template <class P>
FTS_DEV bool eq(const F<P>& a, const F<P>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}
// a < b as plain 256-bit integers
FTS_DEV bool lt256(const uint32_t* a, const uint32_t* b) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c;
    (void)__builtin_subc(a[i], b[i], bw, &c);
    bw = c;
  }
  return bw != 0;
}

// r = x - M if (carry || x >= M)
template <class P>
FTS_DEV void cond_sub(F<P>& x, uint32_t carry) {
  uint32_t t[8], bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c;
    t[i] = __builtin_subc(x.v[i], P::M[i], bw, &c);
    bw = c;
  }
  const bool take = carry || !bw;
#pragma unroll
  for (int i = 0; i < 8; i++) x.v[i] = take ? t[i] : x.v[i];
}

template <class P>
FTS_DEV F<P> add(const F<P>& a, const F<P>& b) {
  F<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t co;
    r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &co);
    c = co;
  }
  cond_sub(r, c);
  return r;
}
template <class P>
FTS_DEV F<P> sub(const F<P>& a, const F<P>& b) {
  F<P> r;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c;
    r.v[i] = __builtin_subc(a.v[i], b.v[i], bw, &c);
    bw = c;
  }
  const uint32_t mask = 0u - bw;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t co;
    r.v[i] = __builtin_addc(r.v[i], P::M[i] & mask, c, &co);
    c = co;
  }
  return r;
}

// Montgomery product a*b*2^-256 mod M for a, b < M: finely-integrated
// product scanning (as fts::f_mul_fips) with each column in a 96-bit
// accumulator (v_mad_u64_u32 + carry add per product).  Full-width moduli:
// the result is < 2M < 2^257, so the bit above column 15 is kept and folded
// into the final conditional subtraction.  Zero limbs of M (p has three) are
// skipped at compile time.
template <class P>
FTS_DEV F<P> mul(const F<P>& a, const F<P>& b) {
  uint32_t m[8];
  F<P> r;
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) fts::mac96(acc, ovf, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < (k < 8 ? k : 8); i++)
      if (P::M[k - i] != 0) fts::mac96s(acc, ovf, m[i], P::M[k - i]);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      fts::mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      r.v[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  r.v[7] = (uint32_t)acc;
  cond_sub(r, (uint32_t)(acc >> 32));
  return r;
}
template <class P>
FTS_DEV F<P> sqr(const F<P>& a) {
  return mul(a, a);
}
template <class P>
FTS_DEV F<P> to_mont(const F<P>& a) {
  return mul(a, load<P>(P::R2));
}
template <class P>
FTS_DEV F<P> from_mont(const F<P>& a) {
  F<P> one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.v[i] = i == 0;
  return mul(a, one);
}
// a^(M-2) (Fermat inverse; 0 -> 0), Montgomery in and out: fixed 4-bit
// window over a^1..a^15 (14 products) -> 252 squarings + one product per
// non-zero nibble, instead of one product per set bit.
template <class P>
FTS_DEV F<P> inv(const F<P>& a) {
  F<P> t[16];
  t[0] = load<P>(P::ONE);
  t[1] = a;
  for (int k = 2; k < 16; k++) t[k] = mul(t[k - 1], a);
  F<P> r = t[P::EXP_INV[7] >> 28];
  for (int nb = 62; nb >= 0; nb--) {
    r = sqr(sqr(sqr(sqr(r))));
    const uint32_t d = (P::EXP_INV[nb >> 3] >> (4 * (nb & 7))) & 15u;
    if (d) r = mul(r, t[d]);
  }
  return r;
}

// ------------------------------------------------------------ points (a = -3)
struct PJ {  // Jacobian; z == 0 <=> point at infinity
  Fp x, y, z;
};

FTS_DEV PJ pj_inf() {
  PJ r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.x.v[i] = PM::ONE[i], r.y.v[i] = PM::ONE[i], r.z.v[i] = 0;
  return r;
}

// dbl-2001-b
__device__ __forceinline__ PJ pj_dbl(PJ p) {
  if (is_zero(p.z)) return p;
  const Fp delta = sqr(p.z), gamma = sqr(p.y), beta = mul(p.x, gamma);
  const Fp t = mul(sub(p.x, delta), add(p.x, delta));
  const Fp alpha = add(add(t, t), t);
  const Fp b4 = add(add(beta, beta), add(beta, beta));
  PJ r;
  r.x = sub(sqr(alpha), add(b4, b4));
  r.z = sub(sub(sqr(add(p.y, p.z)), gamma), delta);
  Fp g2 = sqr(gamma);
  g2 = add(g2, g2);
  g2 = add(g2, g2);
  g2 = add(g2, g2);
  r.y = sub(mul(alpha, sub(b4, r.x)), g2);
  return r;
}

// add-2007-bl style full addition, complete over all Jacobian inputs
__device__ __forceinline__ PJ pj_add(PJ p, PJ q) {
  if (is_zero(p.z)) return q;
  if (is_zero(q.z)) return p;
  const Fp z1z1 = sqr(p.z), z2z2 = sqr(q.z);
  const Fp u1 = mul(p.x, z2z2), u2 = mul(q.x, z1z1);
  const Fp s1 = mul(mul(p.y, q.z), z2z2), s2 = mul(mul(q.y, p.z), z1z1);
  const Fp h = sub(u2, u1), rr = sub(s2, s1);
  if (is_zero(h)) return is_zero(rr) ? pj_dbl(p) : pj_inf();
  const Fp hh = sqr(h), hhh = mul(h, hh), v = mul(u1, hh);
  PJ r;
  r.x = sub(sub(sqr(rr), hhh), add(v, v));
  r.y = sub(mul(rr, sub(v, r.x)), mul(s1, hhh));
  r.z = mul(mul(p.z, q.z), h);
  return r;
}

// mixed addition with an affine (Montgomery) point q != O
__device__ __forceinline__ PJ pj_madd(PJ p, Fp qx, Fp qy) {
  if (is_zero(p.z)) {
    PJ r;
    r.x = qx, r.y = qy, r.z = load<PM>(PM::ONE);
    return r;
  }
  const Fp z1z1 = sqr(p.z);
  const Fp u2 = mul(qx, z1z1), s2 = mul(mul(qy, p.z), z1z1);
  const Fp h = sub(u2, p.x), rr = sub(s2, p.y);
  if (is_zero(h)) return is_zero(rr) ? pj_dbl(p) : pj_inf();
  const Fp hh = sqr(h), hhh = mul(h, hh), v = mul(p.x, hh);
  PJ r;
  r.x = sub(sub(sqr(rr), hhh), add(v, v));
  r.y = sub(mul(rr, sub(v, r.x)), mul(p.y, hhh));
  r.z = mul(p.z, h);
  return r;
}

// y^2 == x^3 - 3x + b, coordinates in Montgomery form
FTS_DEV bool on_curve(const Fp& x, const Fp& y) {
  const Fp x3 = mul(sqr(x), x);
  const Fp x3a = sub(x3, add(add(x, x), x));
  return eq(sqr(y), add(x3a, load<PM>(CB)));
}

}  // namespace p256
