// FP256BN (the BN curve of Apache Milagro / AMCL, mathlib CurveID
// FP256BN_AMCL) on gfx950: y^2 = x^3 + 3 over a full-width 256-bit prime, for
// idemix nym signatures under FP256BN issuer keys (idemix_kernels.hip).
//
// The field arithmetic is p256.hpp's generic full-width Montgomery code
// (textbook CIOS with the extra carry word, F<P> over any 256-bit modulus);
// only the moduli and the a = 0 point formulas differ: dbl-2009-l (2M + 5S),
// add-2007-bl, madd-2007-bl, as in g1.hpp for BN254.  Constants derived from
// p and r with Python (no library code copied).
#pragma once
#include "p256.hpp"

namespace fbn {

struct PM {  // p = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49F0CDC65FB12980A82D3292DDBAED33013
  static constexpr uint32_t M[8] = {0xaed33013u, 0xd3292ddbu, 0x12980a82u, 0x0cdc65fbu,
                                    0xee71a49fu, 0x46e5f25eu, 0xfffcf0cdu, 0xffffffffu};
  static constexpr uint32_t INV = 0x0537e5e5u;  // -p^-1 mod 2^32
  static constexpr uint32_t ONE[8] = {0x512ccfedu, 0x2cd6d224u, 0xed67f57du, 0xf3239a04u,
                                      0x118e5b60u, 0xb91a0da1u, 0x00030f32u, 0x00000000u};
  static constexpr uint32_t R2[8] = {0x1092b98fu, 0xfac8c610u, 0xd7f91154u, 0xdb90d49cu,
                                     0x32bf3141u, 0x4f325fc7u, 0x0e56a005u, 0x4de578eau};
  static constexpr uint32_t EXP_INV[8] = {0xaed33011u, 0xd3292ddbu, 0x12980a82u, 0x0cdc65fbu,
                                          0xee71a49fu, 0x46e5f25eu, 0xfffcf0cdu, 0xffffffffu};  // p - 2
};
struct RM {  // group order r = 0xFFFFFFFFFFFCF0CD46E5F25EEE71A49E0CDC65FB1299921AF62D536CD10B500D
  static constexpr uint32_t M[8] = {0xd10b500du, 0xf62d536cu, 0x1299921au, 0x0cdc65fbu,
                                    0xee71a49eu, 0x46e5f25eu, 0xfffcf0cdu, 0xffffffffu};
};
// 3 in Montgomery form (curve b)
__device__ constexpr uint32_t CB3[8] = {0xf3866fc7u, 0x8684766cu, 0xc837e077u, 0xd96ace0eu,
                                        0x34ab1222u, 0x2b4e28e3u, 0x00092d98u, 0x00000000u};

// GLV (j = 0): phi(x, y) = (beta x, y) = lambda (x, y) with
// lambda = 0x27311c281242030ce379baf3be321c37067081e9398533016 (mod r) and
// beta = 0x13988e140921018659bcdd79df1932d1edb1c0a24a3a1b807 (mod p); lattice
// basis from the extended Euclid of (r, lambda), g_i = floor(2^384 b_i / r),
// derived with Python the same way as glv.hpp's BN254 constants.  |k1|, |k2| < 2^128.
struct GlvK {
  static constexpr uint32_t BETA[8] = {0x84008c2cu, 0xac441038u, 0xf524db81u, 0x26e76706u,
                                       0xb51eaff8u, 0x49cc4e27u, 0x3c3f9cffu, 0x26664872u};  // Montgomery
  static constexpr uint32_t G1[7] = {0xf899d382u, 0x88097763u, 0xce889a08u, 0x859835ddu,
                                     0x6163cf7bu, 0xd105eb80u, 0x00000000u};
  static constexpr uint32_t G2[9] = {0xa170acebu, 0x8cb9048bu, 0xee129700u, 0xca13df5cu, 0xda9e04d4u,
                                     0xf40a1113u, 0x00018798u, 0x00000000u, 0x00000001u};
  static constexpr uint32_t A1[2] = {0x61615001u, 0xd105eb80u};                          // a1 (= b2)
  static constexpr uint32_t A2[4] = {0x7c669004u, 0x0bf5eeeeu, 0xfffe7867u, 0xffffffffu};  // a2
  static constexpr uint32_t NB1[4] = {0x1b054003u, 0x3af0036eu, 0xfffe7866u, 0xffffffffu}; // -b1
};

using Fp = p256::F<PM>;
using p256::add;
using p256::sub;
using p256::mul;
using p256::sqr;
using p256::is_zero;
using p256::eq;
using p256::load;

struct PJ {  // Jacobian; z == 0 <=> point at infinity
  Fp x, y, z;
};

FTS_DEV PJ pj_inf() {
  PJ r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.x.v[i] = PM::ONE[i], r.y.v[i] = PM::ONE[i], r.z.v[i] = 0;
  return r;
}

// dbl-2009-l (a = 0)
FTS_DEV PJ pj_dbl(const PJ& p) {
  if (is_zero(p.z)) return p;
  const Fp a = sqr(p.x), b = sqr(p.y), c = sqr(b);
  Fp d = sub(sqr(add(p.x, b)), add(a, c));
  d = add(d, d);
  const Fp e = add(add(a, a), a);
  const Fp f = sqr(e);
  PJ r;
  r.x = sub(f, add(d, d));
  Fp c8 = add(c, c);
  c8 = add(c8, c8);
  c8 = add(c8, c8);
  r.y = sub(mul(e, sub(d, r.x)), c8);
  const Fp yz = mul(p.y, p.z);
  r.z = add(yz, yz);
  return r;
}

// add-2007-bl style full addition, complete over all Jacobian inputs
FTS_DEV PJ pj_add(const PJ& p, const PJ& q) {
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
FTS_DEV PJ pj_madd(const PJ& p, const Fp& qx, const Fp& qy) {
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

// y^2 == x^3 + 3, coordinates in Montgomery form
FTS_DEV bool on_curve(const Fp& x, const Fp& y) { return eq(sqr(y), add(mul(sqr(x), x), load<PM>(CB3))); }

}  // namespace fbn
