// BN254 G1 (y^2 = x^3 + 3) on gfx950: Jacobian coordinates, one point per lane.
//
// Formulas (EFD, a = 0): dbl-2009-l (2M+5S), madd-2007-bl (7M+4S),
// add-2007-bl (11M+5S).  Exceptional cases (identity operands, P == Q,
// P == -Q) are handled with data-dependent branches that are never taken on
// honest inputs but keep adversarial inputs exact.
//
// Replaces the G1Affine/G1Jac arithmetic of gnark-crypto ecc/bn254 that
// mathlib G1.Add/Sub/Mul call on every step of rp/bulletproof.go:314-324,
// :477-492 and rp/ipa.go:215-259.
#pragma once
#include "field.hpp"

namespace fts {

struct G1A {  // affine; identity encoded as (0, 0) (not on the curve)
  Fp x, y;
};
struct G1J {  // Jacobian; identity <=> z == 0
  Fp x, y, z;
};
struct Scalar {  // canonical scalar, 8 LE limbs (passed by value: 8 VGPRs)
  uint32_t v[8];
};

struct G1J;
__device__ __noinline__ G1J nl_dbl(G1J p);

// f_mul_g: grouped-MAC FIPS (field.hpp); measured on MI355X (lib/int_peak):
// 1,590 cycles single-wave latency vs 1,840 for f_mul_fips, equal throughput;
// the dedicated squarings (100 MADs) are slower on gfx950 (extra 64-bit shifts)
// Products are inlined: an out-of-line product (one ~2 KB copy per kernel)
// was measured 4-8 % slower end to end (no cross-product scheduling, call
// overhead), and did not cure the co-residency slowdowns (those come from
// VALU arbitration by age).
FTS_DEV Fp fp_mul(const Fp& a, const Fp& b) { return f_mul_g(a, b); }
FTS_DEV Fp fp_sqr(const Fp& a) { return f_mul_g(a, a); }
FTS_DEV Fr fr_mul(const Fr& a, const Fr& b) { return f_mul_g(a, b); }
FTS_DEV Fr fr_sqr(const Fr& a) { return f_mul_g(a, a); }

FTS_DEV G1J g1j_identity() {
  G1J r;
  r.x = f_one<FpP>();
  r.y = f_one<FpP>();
  r.z = f_zero<FpP>();
  return r;
}
FTS_DEV bool g1j_is_identity(const G1J& p) { return f_is_zero(p.z); }
FTS_DEV bool g1a_is_identity(const G1A& p) { return f_is_zero(p.x) && f_is_zero(p.y); }

FTS_DEV G1J g1j_from_affine(const G1A& a) {
  if (g1a_is_identity(a)) return g1j_identity();
  G1J r;
  r.x = a.x;
  r.y = a.y;
  r.z = f_one<FpP>();
  return r;
}

FTS_DEV G1A g1a_neg(const G1A& a) {
  G1A r = a;
  if (!g1a_is_identity(a)) r.y = f_neg(a.y);
  return r;
}
FTS_DEV G1J g1j_neg(const G1J& a) {
  G1J r = a;
  r.y = f_neg(a.y);
  return r;
}

FTS_DEV G1J g1j_dbl(const G1J& p) {
  if (f_is_zero(p.z) || f_is_zero(p.y)) return g1j_identity();
  Fp A = fp_sqr(p.x);
  Fp B = fp_sqr(p.y);
  Fp C = fp_sqr(B);
  Fp t = f_add(p.x, B);
  Fp D = f_sub(f_sub(fp_sqr(t), A), C);
  D = f_dbl(D);
  Fp E = f_add(f_dbl(A), A);
  Fp F = fp_sqr(E);
  G1J r;
  r.x = f_sub(F, f_dbl(D));
  Fp C8 = f_dbl(f_dbl(f_dbl(C)));
  r.y = f_sub(fp_mul(E, f_sub(D, r.x)), C8);
  r.z = f_dbl(fp_mul(p.y, p.z));
  return r;
}

// p + q, q affine (madd-2007-bl)
FTS_DEV G1J g1j_add_affine(const G1J& p, const G1A& q) {
  if (g1a_is_identity(q)) return p;
  if (f_is_zero(p.z)) return g1j_from_affine(q);
  Fp z1z1 = fp_sqr(p.z);
  Fp u2 = fp_mul(q.x, z1z1);
  Fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  Fp h = f_sub(u2, p.x);
  Fp rr = f_sub(s2, p.y);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) return nl_dbl(p);
    return g1j_identity();
  }
  Fp hh = fp_sqr(h);
  Fp i = f_dbl(f_dbl(hh));
  Fp j = fp_mul(h, i);
  rr = f_dbl(rr);
  Fp v = fp_mul(p.x, i);
  G1J r;
  r.x = f_sub(f_sub(fp_sqr(rr), j), f_dbl(v));
  r.y = f_sub(fp_mul(rr, f_sub(v, r.x)), f_dbl(fp_mul(p.y, j)));
  r.z = f_sub(f_sub(fp_sqr(f_add(p.z, h)), z1z1), hh);
  return r;
}

// p + q (add-2007-bl)
FTS_DEV G1J g1j_add(const G1J& p, const G1J& q) {
  if (f_is_zero(p.z)) return q;
  if (f_is_zero(q.z)) return p;
  Fp z1z1 = fp_sqr(p.z);
  Fp z2z2 = fp_sqr(q.z);
  Fp u1 = fp_mul(p.x, z2z2);
  Fp u2 = fp_mul(q.x, z1z1);
  Fp s1 = fp_mul(fp_mul(p.y, q.z), z2z2);
  Fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  Fp h = f_sub(u2, u1);
  Fp rr = f_sub(s2, s1);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) return nl_dbl(p);
    return g1j_identity();
  }
  Fp i = fp_sqr(f_dbl(h));
  Fp j = fp_mul(h, i);
  rr = f_dbl(rr);
  Fp v = fp_mul(u1, i);
  G1J r;
  r.x = f_sub(f_sub(fp_sqr(rr), j), f_dbl(v));
  r.y = f_sub(fp_mul(rr, f_sub(v, r.x)), f_dbl(fp_mul(s1, j)));
  r.z = fp_mul(f_sub(f_sub(fp_sqr(f_add(p.z, q.z)), z1z1), z2z2), h);
  return r;
}

__device__ __noinline__ Fp nl_fp_inv(Fp a) { return f_inv_gcd(a); }
__device__ __noinline__ Fr nl_fr_inv(Fr a) { return f_inv_gcd(a); }

// equality of two Jacobian points (as group elements)
FTS_DEV bool g1j_eq(const G1J& p, const G1J& q) {
  bool pi = f_is_zero(p.z), qi = f_is_zero(q.z);
  if (pi || qi) return pi && qi;
  Fp z1z1 = fp_sqr(p.z), z2z2 = fp_sqr(q.z);
  if (!f_eq(fp_mul(p.x, z2z2), fp_mul(q.x, z1z1))) return false;
  return f_eq(fp_mul(fp_mul(p.y, q.z), z2z2), fp_mul(fp_mul(q.y, p.z), z1z1));
}

// single normalisation (one Fermat inversion)
FTS_DEV G1A g1j_to_affine(const G1J& p) {
  G1A r;
  if (f_is_zero(p.z)) {
    r.x = f_zero<FpP>();
    r.y = f_zero<FpP>();
    return r;
  }
  Fp zi = nl_fp_inv(p.z);
  Fp zi2 = fp_sqr(zi);
  r.x = fp_mul(p.x, zi2);
  r.y = fp_mul(fp_mul(p.y, zi2), zi);
  return r;
}

// ------------------------------------------------------- out-of-line wrappers
// Point operations are ~3-5k instructions each once the 136-MAD field product
// is inlined; hot loops call these out-of-line copies so every kernel's loop
// body stays inside the instruction cache.  Second operands come from memory
// (tables / lane scratch) so the call passes <= 32 argument VGPRs.
__device__ __noinline__ G1J nl_dbl(G1J p) { return g1j_dbl(p); }

// ---------------------------------------------------------- memory helpers
FTS_DEV void load_fp(const uint32_t* src, Fp& a) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4 u0 = s[0], u1 = s[1];
  a.v[0] = u0.x; a.v[1] = u0.y; a.v[2] = u0.z; a.v[3] = u0.w;
  a.v[4] = u1.x; a.v[5] = u1.y; a.v[6] = u1.z; a.v[7] = u1.w;
}
FTS_DEV void store_fp(uint32_t* dst, const Fp& a) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
template <class P>
FTS_DEV void load_f(const uint32_t* src, Field<P>& a) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4 u0 = s[0], u1 = s[1];
  a.v[0] = u0.x; a.v[1] = u0.y; a.v[2] = u0.z; a.v[3] = u0.w;
  a.v[4] = u1.x; a.v[5] = u1.y; a.v[6] = u1.z; a.v[7] = u1.w;
}
template <class P>
FTS_DEV void store_f(uint32_t* dst, const Field<P>& a) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
// G1A in memory: 16 words (x then y)
FTS_DEV G1A load_g1a(const uint32_t* src) {
  G1A a;
  load_fp(src, a.x);
  load_fp(src + 8, a.y);
  return a;
}
FTS_DEV void store_g1a(uint32_t* dst, const G1A& a) {
  store_fp(dst, a.x);
  store_fp(dst + 8, a.y);
}
// G1J in memory: 24 words
FTS_DEV G1J load_g1j(const uint32_t* src) {
  G1J a;
  load_fp(src, a.x);
  load_fp(src + 8, a.y);
  load_fp(src + 16, a.z);
  return a;
}
FTS_DEV void store_g1j(uint32_t* dst, const G1J& a) {
  store_fp(dst, a.x);
  store_fp(dst + 8, a.y);
  store_fp(dst + 16, a.z);
}

// p + (+-q), q affine at q_ptr (16 words)
__device__ __noinline__ G1J nl_madd_mem(G1J p, const uint32_t* q_ptr, uint32_t neg) {
  G1A q = load_g1a(q_ptr);
  if (neg) q = g1a_neg(q);
  return g1j_add_affine(p, q);
}
// p + (+-q), q Jacobian at q_ptr (24 words)
__device__ __noinline__ G1J nl_add_mem(G1J p, const uint32_t* q_ptr, uint32_t neg) {
  G1J q = load_g1j(q_ptr);
  if (neg) q.y = f_neg(q.y);
  return g1j_add(p, q);
}
__device__ __noinline__ G1A nl_to_affine(G1J p) { return g1j_to_affine(p); }

// --------------------------------------------------- scalar multiplication
// Variable-base: signed 4-bit windows, per-lane table of 1..8 * P kept in
// `scratch` (8 x 24 words, lane-private global memory; L1/L2 resident).
__device__ __noinline__ G1J var_base_mul(G1A p, Scalar k, uint32_t* __restrict__ scratch) {
  if (g1a_is_identity(p)) return g1j_identity();
  G1J t = g1j_from_affine(p);
  store_g1j(scratch, t);
  store_g1a(scratch + 8 * 24, p);  // affine copy for the table build
  G1J cur = nl_dbl(t);
  store_g1j(scratch + 24, cur);
  for (int i = 2; i < 8; i++) {
    cur = nl_madd_mem(cur, scratch + 8 * 24, 0);
    store_g1j(scratch + i * 24, cur);
  }
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = k.v[i];
  // carries of the signed recoding (LSB first), one bit per window
  uint64_t cm = 0;
  {
    uint32_t q[8];
#pragma unroll
    for (int i = 0; i < 8; i++) q[i] = s[i];
    int carry = 0;
    for (int w = 0; w < 64; w++) {
      cm |= (uint64_t)carry << w;
      int d = (int)(q[0] & 0xfu) + carry;
#pragma unroll
      for (int i = 0; i < 7; i++) q[i] = (q[i] >> 4) | (q[i + 1] << 28);
      q[7] >>= 4;
      carry = d > 8;
    }
  }
  G1J acc = g1j_identity();
  for (int w = 63; w >= 0; w--) {
    for (int q = 0; q < 4; q++) acc = nl_dbl(acc);
    int raw = (int)(s[7] >> 28);
#pragma unroll
    for (int i = 7; i > 0; i--) s[i] = (s[i] << 4) | (s[i - 1] >> 28);
    s[0] <<= 4;
    int cin = (int)((cm >> w) & 1u);
    int cout = w < 63 ? (int)((cm >> (w + 1)) & 1u) : 0;
    int d = raw + cin - 16 * cout;
    if (d != 0) {
      int ad = d < 0 ? -d : d;
      acc = nl_add_mem(acc, scratch + (ad - 1) * 24, d < 0);
    }
  }
  return acc;
}

}  // namespace fts
