// Optimal-ate pairing check on gfx950 for the idemix identity proof
// (services/identity/idemix/crypto/id.go:74-108 -> IBM/idemix Signature.Ver:
// e(W, A') == e(g2, ABar)), on both curves idemix keys use here: BN254
// (gnark-crypto, D-type twist, xi = 9 + i) and FP256BN (AMCL, M-type twist,
// xi = 1 + i).  One identity per lane.
//
// Tower: Fp2 = Fp[i]/(i^2 + 1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v).
// The G2 arguments (the issuer's W and the generator g2) are fixed per issuer
// key, so their Miller-loop line coefficients (lam, mu) are precomputed once
// (k_idm_lines, affine, one Fp2 inversion per step) and every identity's loop
// only evaluates them at its G1 points:
//   D-type:  l       = yP + (-lam xP) w + mu v w
//   M-type:  l * w^3 = mu + (-lam xP) v + yP v w
// (Fp2 factors and w^3 vanish in the final exponentiation).  The two pairings
// share one multi-Miller loop (one squaring per step), then one final
// exponentiation: easy part conj(f)/f, ^(p^2 + 1); hard part by Scott et al.'s
// BN decomposition with three exponentiations by u.  Step for step the same as
// oracle/pairing_tower.py, whose result equals the direct E(Fp12) pairing of
// oracle/pairing.py (pinned by the reference's credential fixtures).
//
// The field is abstracted by an adapter (BnField: fts::Fp with the grouped-MAC
// product; FbnField: the full-width Montgomery code of p256.hpp on FP256BN's p).
#pragma once
#include "g1.hpp"
#include "fp256bn.hpp"
#include "pairing_consts.hpp"

namespace pair {

struct BnField {
  using F = fts::Fp;
  using K = pairc::Bn254;
  static FTS_DEV F add(const F& a, const F& b) { return fts::f_add(a, b); }
  static FTS_DEV F sub(const F& a, const F& b) { return fts::f_sub(a, b); }
  static FTS_DEV F neg(const F& a) { return fts::f_neg(a); }
  // (the two-accumulator product f_mul_fips2 made k_idv_pairing slower, 21.9 ->
  // 26.7 ms per 65,536 identities: its extra column adds cost more than the
  // shorter MAD chain saves, even at one wave per SIMD)
  static FTS_DEV F mul(const F& a, const F& b) { return fts::fp_mul(a, b); }
  static FTS_DEV F zero() { return fts::f_zero<fts::FpP>(); }
  static FTS_DEV F one() { return fts::f_one<fts::FpP>(); }
  static FTS_DEV bool is_zero(const F& a) { return fts::f_is_zero(a); }
  static FTS_DEV bool eq(const F& a, const F& b) { return fts::f_eq(a, b); }
  static FTS_DEV F inv(const F& a) { return fts::nl_fp_inv(a); }
  static FTS_DEV F ld(const uint32_t* w) {
    F r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = w[i];
    return r;
  }
};

struct FbnField {
  using F = fbn::Fp;
  using K = pairc::Fp256bn;
  static FTS_DEV F add(const F& a, const F& b) { return p256::add(a, b); }
  static FTS_DEV F sub(const F& a, const F& b) { return p256::sub(a, b); }
  static FTS_DEV F zero() {
    F r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  static FTS_DEV F neg(const F& a) { return p256::sub(zero(), a); }
  static FTS_DEV F mul(const F& a, const F& b) { return p256::mul(a, b); }
  static FTS_DEV F one() { return p256::load<fbn::PM>(fbn::PM::ONE); }
  static FTS_DEV bool is_zero(const F& a) { return p256::is_zero(a); }
  static FTS_DEV bool eq(const F& a, const F& b) { return p256::eq(a, b); }
  static FTS_DEV F inv(const F& a) { return p256::inv(a); }
  static FTS_DEV F ld(const uint32_t* w) { return p256::load<fbn::PM>(w); }
};

// ------------------------------------------------------------------- Fp2
template <class B>
struct F2 {
  typename B::F a, b;  // a + b i
};
template <class B>
FTS_DEV F2<B> f2_zero() {
  return {B::zero(), B::zero()};
}
template <class B>
FTS_DEV F2<B> f2_one() {
  return {B::one(), B::zero()};
}
template <class B>
FTS_DEV F2<B> f2_ld(const uint32_t (&w)[2][8]) {
  return {B::ld(w[0]), B::ld(w[1])};
}
template <class B>
FTS_DEV F2<B> add(const F2<B>& x, const F2<B>& y) {
  return {B::add(x.a, y.a), B::add(x.b, y.b)};
}
template <class B>
FTS_DEV F2<B> sub(const F2<B>& x, const F2<B>& y) {
  return {B::sub(x.a, y.a), B::sub(x.b, y.b)};
}
template <class B>
FTS_DEV F2<B> neg(const F2<B>& x) {
  return {B::neg(x.a), B::neg(x.b)};
}
template <class B>
FTS_DEV F2<B> dbl(const F2<B>& x) {
  return add(x, x);
}
template <class B>
FTS_DEV F2<B> conj(const F2<B>& x) {
  return {x.a, B::neg(x.b)};
}
// Karatsuba: 3 products
template <class B>
FTS_DEV F2<B> mul(const F2<B>& x, const F2<B>& y) {
  const auto t0 = B::mul(x.a, y.a), t1 = B::mul(x.b, y.b);
  const auto t2 = B::mul(B::add(x.a, x.b), B::add(y.a, y.b));
  return {B::sub(t0, t1), B::sub(B::sub(t2, t0), t1)};
}
// (a + b i)^2 = (a + b)(a - b) + 2ab i: 2 products
template <class B>
FTS_DEV F2<B> sqr(const F2<B>& x) {
  const auto t = B::mul(x.a, x.b);
  return {B::mul(B::add(x.a, x.b), B::sub(x.a, x.b)), B::add(t, t)};
}
template <class B>
FTS_DEV F2<B> mul_fp(const F2<B>& x, const typename B::F& s) {
  return {B::mul(x.a, s), B::mul(x.b, s)};
}
// small constant multiple (xi's real part: 9 or 1)
template <class B, int C>
FTS_DEV typename B::F mul_small(const typename B::F& a) {
  if constexpr (C == 1) {
    return a;
  } else {
    static_assert(C == 9, "xi0");
    auto t = B::add(a, a);
    t = B::add(t, t);
    t = B::add(t, t);
    return B::add(t, a);
  }
}
// x * xi, xi = XI0 + i
template <class B>
FTS_DEV F2<B> mul_xi(const F2<B>& x) {
  constexpr int X0 = (int)B::K::XI0;
  static_assert(B::K::XI1 == 1, "xi = XI0 + i");
  return {B::sub(mul_small<B, X0>(x.a), x.b), B::add(x.a, mul_small<B, X0>(x.b))};
}
template <class B>
FTS_DEV F2<B> inv(const F2<B>& x) {
  const auto n = B::inv(B::add(B::mul(x.a, x.a), B::mul(x.b, x.b)));
  return {B::mul(x.a, n), B::neg(B::mul(x.b, n))};
}
template <class B>
FTS_DEV bool is_zero(const F2<B>& x) {
  return B::is_zero(x.a) && B::is_zero(x.b);
}
template <class B>
FTS_DEV bool eq(const F2<B>& x, const F2<B>& y) {
  return B::eq(x.a, y.a) && B::eq(x.b, y.b);
}

// ------------------------------------------------------------------- Fp6
template <class B>
struct F6 {
  F2<B> c0, c1, c2;
};
template <class B>
FTS_DEV F6<B> add(const F6<B>& x, const F6<B>& y) {
  return {add(x.c0, y.c0), add(x.c1, y.c1), add(x.c2, y.c2)};
}
template <class B>
FTS_DEV F6<B> sub(const F6<B>& x, const F6<B>& y) {
  return {sub(x.c0, y.c0), sub(x.c1, y.c1), sub(x.c2, y.c2)};
}
template <class B>
FTS_DEV F6<B> neg(const F6<B>& x) {
  return {neg(x.c0), neg(x.c1), neg(x.c2)};
}
// x * v
template <class B>
FTS_DEV F6<B> mul_v(const F6<B>& x) {
  return {mul_xi(x.c2), x.c0, x.c1};
}
template <class B>
FTS_DEV F6<B> mul_fp(const F6<B>& x, const typename B::F& s) {
  return {mul_fp(x.c0, s), mul_fp(x.c1, s), mul_fp(x.c2, s)};
}
// Karatsuba: 6 Fp2 products.  Fp6 / Fp12 operations are out of line (PAIR_FN): a
// fully inlined pairing is ~10^6 instructions (compile time and instruction cache);
// each callee stays far below the s_cbranch range (tools/long_branch_check.py).
// The hot loops (Miller squaring + line products, the cyclotomic squarings of
// expt) use the *_i inline bodies instead, so their Fp12 accumulator stays in
// VGPRs: every out-of-line call passes its Fp6/Fp12 operands through the
// private stack (round 3: 9.8 KB of stack per lane, ~1.7 MB of scratch traffic
// per identity).
#define PAIR_FN __device__ __noinline__
template <class B>
FTS_DEV F6<B> mul6_i(const F6<B>& x, const F6<B>& y) {
  const F2<B> t0 = mul(x.c0, y.c0), t1 = mul(x.c1, y.c1), t2 = mul(x.c2, y.c2);
  F6<B> r;
  r.c0 = add(t0, mul_xi(sub(sub(mul(add(x.c1, x.c2), add(y.c1, y.c2)), t1), t2)));
  r.c1 = add(sub(sub(mul(add(x.c0, x.c1), add(y.c0, y.c1)), t0), t1), mul_xi(t2));
  r.c2 = add(sub(sub(mul(add(x.c0, x.c2), add(y.c0, y.c2)), t0), t2), t1);
  return r;
}
template <class B>
PAIR_FN F6<B> mul(const F6<B>& x, const F6<B>& y) {
  return mul6_i(x, y);
}
// x * (A + B v): 5 Fp2 products
template <class B>
FTS_DEV F6<B> mul01_i(const F6<B>& x, const F2<B>& A, const F2<B>& Bv) {
  const F2<B> t0 = mul(x.c0, A), t1 = mul(x.c1, Bv);
  F6<B> r;
  r.c0 = add(t0, mul_xi(mul(x.c2, Bv)));
  r.c1 = sub(sub(mul(add(x.c0, x.c1), add(A, Bv)), t0), t1);
  r.c2 = add(t1, mul(x.c2, A));
  return r;
}
template <class B>
PAIR_FN F6<B> mul_01(const F6<B>& x, const F2<B>& A, const F2<B>& Bv) {
  return mul01_i(x, A, Bv);
}
template <class B>
PAIR_FN F6<B> inv(const F6<B>& x) {
  const F2<B> c0 = sub(sqr(x.c0), mul_xi(mul(x.c1, x.c2)));
  const F2<B> c1 = sub(mul_xi(sqr(x.c2)), mul(x.c0, x.c1));
  const F2<B> c2 = sub(sqr(x.c1), mul(x.c0, x.c2));
  const F2<B> t = inv(add(mul(x.c0, c0), mul_xi(add(mul(x.c2, c1), mul(x.c1, c2)))));
  return {mul(c0, t), mul(c1, t), mul(c2, t)};
}

// ------------------------------------------------------------------ Fp12
template <class B>
struct F12 {
  F6<B> c0, c1;
};
template <class B>
FTS_DEV F12<B> f12_one() {
  F12<B> r;
  r.c0.c0 = f2_one<B>();
  r.c0.c1 = r.c0.c2 = r.c1.c0 = r.c1.c1 = r.c1.c2 = f2_zero<B>();
  return r;
}
template <class B>
FTS_DEV bool is_one(const F12<B>& x) {
  return eq(x.c0.c0, f2_one<B>()) && is_zero(x.c0.c1) && is_zero(x.c0.c2) && is_zero(x.c1.c0) &&
         is_zero(x.c1.c1) && is_zero(x.c1.c2);
}
// (Fp6 products inline: one call per Fp12 product, not four; every kernel that
// reaches these functions has __launch_bounds__(64), so a callee may use the
// full register file instead of the 128 VGPRs of a 1,024-thread block)
template <class B>
FTS_DEV F12<B> mul12_i(const F12<B>& x, const F12<B>& y) {
  const F6<B> t0 = mul6_i(x.c0, y.c0), t1 = mul6_i(x.c1, y.c1);
  F12<B> r;
  r.c1 = sub(sub(mul6_i(add(x.c0, x.c1), add(y.c0, y.c1)), t0), t1);
  r.c0 = add(t0, mul_v(t1));
  return r;
}
template <class B>
PAIR_FN F12<B> mul(const F12<B>& x, const F12<B>& y) {
  return mul12_i(x, y);
}
// complex squaring: 2 Fp6 products
template <class B>
FTS_DEV F12<B> sqr12_i(const F12<B>& x) {
  const F6<B> t = mul6_i(x.c0, x.c1);
  F12<B> r;
  r.c0 = sub(sub(mul6_i(add(x.c0, x.c1), add(x.c0, mul_v(x.c1))), t), mul_v(t));
  r.c1 = add(t, t);
  return r;
}
template <class B>
PAIR_FN F12<B> sqr(const F12<B>& x) {
  return sqr12_i(x);
}
// Granger-Scott squaring in the cyclotomic subgroup (after the easy part of the
// final exponentiation): Fp12 = Fp4[w]/(w^3 - s), s = w^3, s^2 = xi;
// A = z0 + z3 s, B = z1 + z4 s, C = z2 + z5 s (z_k: coefficient of w^k);
// f^2 = (3A^2 - 2 conj A) + (3 s C^2 + 2 conj B) w + (3B^2 - 2 conj C) w^2:
// 9 Fp2 squarings (18 products) instead of 36 products
template <class B>
FTS_DEV void sq4(const F2<B>& x0, const F2<B>& x1, F2<B>& r0, F2<B>& r1) {
  const F2<B> t0 = sqr(x0), t1 = sqr(x1);
  r1 = sub(sub(sqr(add(x0, x1)), t0), t1);
  r0 = add(t0, mul_xi(t1));
}
template <class B>
FTS_DEV F2<B> three(const F2<B>& x) {
  return add(add(x, x), x);
}
template <class B>
FTS_DEV F12<B> cyc_sqr_i(const F12<B>& x) {
  // z0 = c0.c0, z1 = c1.c0, z2 = c0.c1, z3 = c1.c1, z4 = c0.c2, z5 = c1.c2
  F2<B> a0, a1, b0, b1, c0, c1;
  sq4(x.c0.c0, x.c1.c1, a0, a1);
  sq4(x.c1.c0, x.c0.c2, b0, b1);
  sq4(x.c0.c1, x.c1.c2, c0, c1);
  F12<B> r;
  r.c0.c0 = sub(three(a0), dbl(x.c0.c0));          // z0'
  r.c1.c1 = add(three(a1), dbl(x.c1.c1));          // z3'
  r.c1.c0 = add(three(mul_xi(c1)), dbl(x.c1.c0));  // z1'
  r.c0.c2 = sub(three(c0), dbl(x.c0.c2));          // z4'
  r.c0.c1 = sub(three(b0), dbl(x.c0.c1));          // z2'
  r.c1.c2 = add(three(b1), dbl(x.c1.c2));          // z5'
  return r;
}
template <class B>
PAIR_FN F12<B> cyc_sqr(const F12<B>& x) {
  return cyc_sqr_i(x);
}

template <class B>
FTS_DEV F12<B> conj(const F12<B>& x) {
  return {x.c0, neg(x.c1)};
}
template <class B>
PAIR_FN F12<B> inv(const F12<B>& x) {
  const F6<B> t = inv(sub(mul(x.c0, x.c0), mul_v(mul(x.c1, x.c1))));
  return {mul(x.c0, t), neg(mul(x.c1, t))};
}
// x^(p^n), n = 1, 2, 3: coefficient of w^k times G_n[k] (conjugated for odd n);
// w^k <-> (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2) for k = 0..5
template <class B, int N>
PAIR_FN F12<B> frob(const F12<B>& x) {
  using K = typename B::K;
  auto g = [](int k) -> F2<B> {
    if constexpr (N == 1) return f2_ld<B>(K::G1[k - 1]);
    else if constexpr (N == 2) return f2_ld<B>(K::G2[k - 1]);
    else return f2_ld<B>(K::G3[k - 1]);
  };
  auto c = [](const F2<B>& z) -> F2<B> {
    if constexpr (N == 2) return z;
    else return conj(z);
  };
  F12<B> r;
  r.c0.c0 = c(x.c0.c0);
  r.c1.c0 = mul(c(x.c1.c0), g(1));
  r.c0.c1 = mul(c(x.c0.c1), g(2));
  r.c1.c1 = mul(c(x.c1.c1), g(3));
  r.c0.c2 = mul(c(x.c0.c2), g(4));
  r.c1.c2 = mul(c(x.c1.c2), g(5));
  return r;
}

// --------------------------------------------------------------- lines
// precomputed line of one Miller step: lam, mu in Fp2 (16 words each, Montgomery)
constexpr int LINE_WORDS = 32;
template <class K>
FTS_DEV constexpr int ate_bits() {
  return K::ATE_BITS;
}
template <class K>
FTS_DEV bool ate_bit(int i) {  // bit i of |6u + 2|
  return (K::ATE[i >> 5] >> (i & 31)) & 1u;
}
// number of lines of the loop: one per doubling, one per set bit below the top, two Frobenius steps
template <class K>
__host__ __device__ constexpr int n_lines() {
  int n = 0;
  for (int i = K::ATE_BITS - 2; i >= 0; i--) n += 1 + (int)((K::ATE[i >> 5] >> (i & 31)) & 1u);
  return n + 2;
}

template <class B>
FTS_DEV void store_f2(uint32_t* w, const F2<B>& x) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = x.a.v[i], w[8 + i] = x.b.v[i];
}
template <class B>
FTS_DEV F2<B> load_f2(const uint32_t* w) {
  F2<B> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.a.v[i] = w[i], r.b.v[i] = w[8 + i];
  return r;
}

// one affine step T <- T + R (R == T: tangent): writes (lam, mu = lam x_T - y_T)
template <class B>
PAIR_FN void line_step(F2<B>& tx, F2<B>& ty, const F2<B>& rx, const F2<B>& ry, bool dbl_step, uint32_t* out) {
  F2<B> lam;
  if (dbl_step) {
    const F2<B> x2 = sqr(tx);
    lam = mul(add(add(x2, x2), x2), inv(dbl(ty)));
  } else {
    lam = mul(sub(ry, ty), inv(sub(rx, tx)));
  }
  const F2<B> mu = sub(mul(lam, tx), ty);
  store_f2(out, lam);
  store_f2(out + 16, mu);
  const F2<B> x3 = sub(sub(sqr(lam), tx), rx);
  ty = sub(mul(lam, sub(tx, x3)), ty);
  tx = x3;
}

// all n_lines<K>() lines of Q = (qx, qy) (affine twist point, not the identity)
template <class B>
FTS_DEV void precompute_lines(const F2<B>& qx, const F2<B>& qy, uint32_t* out) {
  using K = typename B::K;
  F2<B> tx = qx, ty = qy;
  int idx = 0;
  for (int i = K::ATE_BITS - 2; i >= 0; i--) {
    line_step<B>(tx, ty, tx, ty, true, out + (idx++) * LINE_WORDS);
    if (ate_bit<K>(i)) line_step<B>(tx, ty, qx, qy, false, out + (idx++) * LINE_WORDS);
  }
  if (K::ATE_NEG) ty = neg(ty);
  const F2<B> q1x = mul(conj(qx), f2_ld<B>(K::TW[0])), q1y = mul(conj(qy), f2_ld<B>(K::TW[1]));
  const F2<B> q2x = mul(qx, f2_ld<B>(K::TW[2])), q2y = neg(mul(qy, f2_ld<B>(K::TW[3])));
  line_step<B>(tx, ty, q1x, q1y, false, out + (idx++) * LINE_WORDS);
  line_step<B>(tx, ty, q2x, q2y, false, out + (idx++) * LINE_WORDS);
}

// f <- f * l(P) for the line (lam, mu) at P = (xP, yP) (affine G1, Montgomery)
template <class B>
FTS_DEV void line_mul_i(F12<B>& f, const uint32_t* ln, const typename B::F& xP, const typename B::F& yP) {
  const F2<B> lam = load_f2<B>(ln), mu = load_f2<B>(ln + 16);
  const F2<B> A = neg(mul_fp(lam, xP));
  F12<B> r;
  if constexpr (!B::K::M_TWIST) {
    // l = yP + A w + mu v w:  c0 = (yP, 0, 0), c1 = (A, mu, 0)
    r.c0 = add(mul_fp(f.c0, yP), mul_v(mul01_i(f.c1, A, mu)));
    r.c1 = add(mul01_i(f.c0, A, mu), mul_fp(f.c1, yP));
  } else {
    // l w^3 = mu + A v + yP v w:  c0 = (mu, A, 0), c1 = (0, yP, 0)
    r.c0 = add(mul01_i(f.c0, mu, A), mul_fp(mul_v(mul_v(f.c1)), yP));
    r.c1 = add(mul_fp(mul_v(f.c0), yP), mul01_i(f.c1, mu, A));
  }
  f = r;
}

// f <- f * l1(P1) * l2(P2) for two lines of the same Miller step: the lines'
// product first (sparse x sparse: 9 Fp2 + 8 Fp products; one Fp6 half has a
// zero coefficient), then one Fp12 product with that sparse half (17 Fp2
// products): ~73 base-field products instead of 2 x 44 for two line_mul_i
//   D-type l_j: c0 = (yP_j, 0, 0), c1 = (A_j, mu_j, 0)
//     L.c0 = (y1 y2 + xi mu1 mu2, A1 A2, A1 mu2 + mu1 A2), L.c1 = (y1 A2 + y2 A1, y1 mu2 + y2 mu1, 0)
//   M-type l_j: c0 = (mu_j, A_j, 0), c1 = (0, yP_j, 0)
//     L.c0 = (mu1 mu2 + xi y1 y2, mu1 A2 + A1 mu2, A1 A2), L.c1 = (0, y2 mu1 + y1 mu2, y2 A1 + y1 A2)
template <class B>
FTS_DEV void line2_mul_i(F12<B>& f, const uint32_t* ln1, const typename B::F& xP1, const typename B::F& yP1,
                         const uint32_t* ln2, const typename B::F& xP2, const typename B::F& yP2) {
  const F2<B> lam1 = load_f2<B>(ln1), mu1 = load_f2<B>(ln1 + 16);
  const F2<B> lam2 = load_f2<B>(ln2), mu2 = load_f2<B>(ln2 + 16);
  const F2<B> A1 = neg(mul_fp(lam1, xP1)), A2 = neg(mul_fp(lam2, xP2));
  const F2<B> aa = mul(A1, A2), mm = mul(mu1, mu2);
  const F2<B> am = sub(sub(mul(add(A1, mu1), add(A2, mu2)), aa), mm);  // A1 mu2 + mu1 A2
  F2<B> yy;
  yy.a = B::mul(yP1, yP2);
  yy.b = B::zero();
  F6<B> L0, L1;
  if constexpr (!B::K::M_TWIST) {
    L0 = {add(yy, mul_xi(mm)), aa, am};
    L1 = {add(mul_fp(A2, yP1), mul_fp(A1, yP2)), add(mul_fp(mu2, yP1), mul_fp(mu1, yP2)), f2_zero<B>()};
  } else {
    L0 = {add(mm, mul_xi(yy)), am, aa};
    L1 = {f2_zero<B>(), add(mul_fp(mu1, yP2), mul_fp(mu2, yP1)), add(mul_fp(A1, yP2), mul_fp(A2, yP1))};
  }
  const F6<B> t0 = mul6_i(f.c0, L0);
  F6<B> t1;
  if constexpr (!B::K::M_TWIST)
    t1 = mul01_i(f.c1, L1.c0, L1.c1);
  else  // (b1 v + b2 v^2) = v (b1 + b2 v)
    t1 = mul_v(mul01_i(f.c1, L1.c1, L1.c2));
  const F6<B> t2 = mul6_i(add(f.c0, f.c1), add(L0, L1));
  f.c1 = sub(sub(t2, t0), t1);
  f.c0 = add(t0, mul_v(t1));
}

// prod_j e(Q_j, P_j) Miller value for NP pairs: lines[j] = Q_j's precomputed table.
// One rolled loop over the steps (i = ATE_BITS-2 .. 0, then the two Frobenius
// lines as step -1) and, inside it, one rolled loop over the step's line
// products: a single inlined copy of the squaring and of the line product, f in
// VGPRs throughout.
template <class B, int NP>
FTS_DEV F12<B> miller(const uint32_t* const (&lines)[NP], const typename B::F (&xP)[NP],
                      const typename B::F (&yP)[NP]) {
  using K = typename B::K;
  using F = typename B::F;
  F12<B> f = f12_one<B>();
  int idx = 0;
#pragma unroll 1
  for (int i = K::ATE_BITS - 2; i >= -1; i--) {
    if (i >= 0 && i != K::ATE_BITS - 2) f = sqr12_i(f);
    if (i < 0 && K::ATE_NEG) f = conj(f);
    const int nl = i < 0 ? 2 : 1 + (int)ate_bit<K>(i);
    if constexpr (NP == 2) {
#pragma unroll 1
      for (int q = 0; q < nl; q++)
        line2_mul_i<B>(f, lines[0] + (idx + q) * LINE_WORDS, xP[0], yP[0], lines[1] + (idx + q) * LINE_WORDS, xP[1],
                       yP[1]);
    } else {
#pragma unroll 1
      for (int q = 0; q < nl * NP; q++) {
        const int j = q % NP;
        const uint32_t* L = lines[0];
        F x = xP[0], y = yP[0];
#pragma unroll
        for (int jj = 1; jj < NP; jj++)
          if (j == jj) L = lines[jj], x = xP[jj], y = yP[jj];
        line_mul_i<B>(f, L + (idx + q / NP) * LINE_WORDS, x, y);
      }
    }
    idx += nl;
  }
  return f;
}

// |u| in non-adjacent form: digit i is +1 (pos bit i), -1 (neg bit i) or 0;
// BN254's u has 28 set bits and 24 NAF digits, FP256BN's 22 and 18
struct Naf {
  uint64_t pos, neg;
  int top;
};
__host__ __device__ constexpr Naf naf_of(uint64_t k) {
  Naf r{0, 0, -1};
  for (int i = 0; k != 0; i++, k >>= 1) {
    if (k & 1) {
      if ((k & 3) == 1) {
        r.pos |= 1ull << i;
        k -= 1;
      } else {
        r.neg |= 1ull << i;
        k += 1;
      }
    }
    r.top = i;
  }
  return r;
}

// f^u in the cyclotomic subgroup (inverse = conjugate): signed digits of |u|
// (f^-1 = conj f), squarings and multiplications inline (round 4: with the
// ~24 multiplications out of line, their stack arguments were ~2/3 of the
// pairing kernel's 8 GB of memory traffic per 65,536 identities)
template <class B>
FTS_DEV F12<B> expt_i(const F12<B>& f) {
  using K = typename B::K;
  constexpr Naf N = naf_of(K::U);
  static_assert(N.top >= 1 && ((N.pos >> N.top) & 1ull), "leading NAF digit +1");
  const F12<B> fc = conj(f);
  F12<B> r = f;
#pragma unroll 1
  for (int i = N.top - 1; i >= 0; i--) {
    r = cyc_sqr_i(r);
    if (((N.pos | N.neg) >> i) & 1ull)  // inline: an out-of-line call passes three Fp12 values through the stack
      r = mul12_i(r, ((N.pos >> i) & 1ull) ? f : fc);
  }
  return K::U_NEG ? conj(r) : r;
}

// final exponentiation, inlined into the kernels (no out-of-line form: the
// round-4 build of an out-of-line wrapper around this body returned wrong GT
// values from k_idv_pairing_debug while the same code inlined into
// k_idv_pairing was right -- kept in kernels, like glv_mul); its three
// exponentiations by u (one rolled loop, one copy of the squaring) run with the
// kernel's register budget: a callee is held to 128 VGPRs and spilled its
// Fp12 accumulator on every squaring
template <class B>
FTS_DEV F12<B> final_exp_i(const F12<B>& f0) {
  F12<B> f = mul(conj(f0), inv(f0));
  f = mul(frob<B, 2>(f), f);
  F12<B> fu[3];
  F12<B> cur = f;
#pragma unroll 1
  for (int e = 0; e < 3; e++) {
    cur = expt_i(cur);
    fu[e] = cur;
  }
  const F12<B> y0 = mul(mul(frob<B, 1>(f), frob<B, 2>(f)), frob<B, 3>(f));
  const F12<B> y1 = conj(f);
  const F12<B> y2 = frob<B, 2>(fu[1]);
  const F12<B> y3 = conj(frob<B, 1>(fu[0]));
  const F12<B> y4 = conj(mul(fu[0], frob<B, 1>(fu[1])));
  const F12<B> y5 = conj(fu[1]);
  const F12<B> y6 = conj(mul(fu[2], frob<B, 1>(fu[2])));
  F12<B> t0 = mul(mul(cyc_sqr(y6), y4), y5);
  F12<B> t1 = mul(mul(y3, y5), t0);
  t0 = mul(t0, y2);
  t1 = cyc_sqr(mul(cyc_sqr(t1), t0));
  t0 = mul(t1, y1);
  t1 = mul(t1, y0);
  t0 = cyc_sqr(t0);
  return mul(t0, t1);
}

}  // namespace pair
