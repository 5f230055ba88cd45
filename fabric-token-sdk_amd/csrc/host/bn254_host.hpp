// Host-side BN254 arithmetic (4 x 64-bit Montgomery, x86-64 __int128).
//
// Used by the context builder (parsing / validating the public parameters)
// and by the host prover that produces synthetic inputs
// (rp/bulletproof.go:209-249,336-466; rp/ipa.go:158-186,267-322).
// The verification hot path runs on the GPU (device/*.hpp); nothing here is
// on the timed path.
#pragma once
#include <stdint.h>
#include <string.h>
#include <array>
#include <vector>

namespace fts {
namespace host {

typedef unsigned __int128 u128;

struct ModP {
  static constexpr uint64_t M[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL,
                                    0x30644e72e131a029ULL};
  static constexpr uint64_t INV = 0x87d20782e4866389ULL;
  static constexpr uint64_t ONE[4] = {0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL,
                                      0x0e0a77c19a07df2fULL};
  static constexpr uint64_t R2[4] = {0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL,
                                     0x06d89f71cab8351fULL};
};
struct ModR {
  static constexpr uint64_t M[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL,
                                    0x30644e72e131a029ULL};
  static constexpr uint64_t INV = 0xc2e1f593efffffffULL;
  static constexpr uint64_t ONE[4] = {0xac96341c4ffffffbULL, 0x36fc76959f60cd29ULL, 0x666ea36f7879462eULL,
                                      0x0e0a77c19a07df2fULL};
  static constexpr uint64_t R2[4] = {0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL, 0x8c49833d53bb8085ULL,
                                     0x0216d0b17f4e44a5ULL};
};

// A field element in Montgomery form, 4 little-endian 64-bit limbs.
template <class P>
struct F {
  uint64_t v[4];
  static F zero() { return F{{0, 0, 0, 0}}; }
  static F one() { return F{{P::ONE[0], P::ONE[1], P::ONE[2], P::ONE[3]}}; }
  bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
  bool operator==(const F& o) const { return memcmp(v, o.v, 32) == 0; }
  bool operator!=(const F& o) const { return !(*this == o); }
};

template <class P>
inline bool geq_mod(const uint64_t a[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != P::M[i]) return a[i] > P::M[i];
  }
  return true;
}

template <class P>
inline void sub_mod_raw(uint64_t a[4]) {
  u128 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - P::M[i] - b;
    a[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}

template <class P>
inline F<P> add(const F<P>& a, const F<P>& b) {
  F<P> r;
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.v[i] + b.v[i];
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  if (geq_mod<P>(r.v)) sub_mod_raw<P>(r.v);
  return r;
}

template <class P>
inline F<P> sub(const F<P>& a, const F<P>& b) {
  F<P> r;
  u128 bw = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - bw;
    r.v[i] = (uint64_t)d;
    bw = (d >> 64) & 1;
  }
  if (bw) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)r.v[i] + P::M[i];
      r.v[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}

template <class P>
inline F<P> neg(const F<P>& a) {
  return sub(F<P>::zero(), a);
}

// no-carry CIOS (top limb of both moduli < 2^63 - 1)
template <class P>
inline F<P> mul(const F<P>& a, const F<P>& b) {
  uint64_t t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 A = (u128)a.v[0] * b.v[i] + t[0];
    t[0] = (uint64_t)A;
    uint64_t m = t[0] * P::INV;
    u128 C = (u128)m * P::M[0] + t[0];
    for (int j = 1; j < 4; j++) {
      A = (u128)a.v[j] * b.v[i] + t[j] + (uint64_t)(A >> 64);
      t[j] = (uint64_t)A;
      C = (u128)m * P::M[j] + t[j] + (uint64_t)(C >> 64);
      t[j - 1] = (uint64_t)C;
    }
    t[3] = (uint64_t)(C >> 64) + (uint64_t)(A >> 64);
  }
  F<P> r;
  memcpy(r.v, t, 32);
  if (geq_mod<P>(r.v)) sub_mod_raw<P>(r.v);
  return r;
}

template <class P>
inline F<P> sqr(const F<P>& a) {
  return mul(a, a);
}

template <class P>
inline F<P> to_mont(const uint64_t canon[4]) {
  F<P> a;
  memcpy(a.v, canon, 32);
  F<P> r2{{P::R2[0], P::R2[1], P::R2[2], P::R2[3]}};
  return mul(a, r2);
}
template <class P>
inline void from_mont(const F<P>& a, uint64_t out[4]) {
  F<P> one{{1, 0, 0, 0}};
  F<P> r = mul(a, one);
  memcpy(out, r.v, 32);
}
template <class P>
inline F<P> from_u64(uint64_t x) {
  uint64_t c[4] = {x, 0, 0, 0};
  return to_mont<P>(c);
}

// a^e, e as 4 LE limbs
template <class P>
inline F<P> pow(const F<P>& a, const uint64_t e[4]) {
  F<P> r = F<P>::one();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = sqr(r);
      if ((e[i] >> b) & 1) r = mul(r, a);
    }
  return r;
}
template <class P>
inline F<P> inv(const F<P>& a) {
  uint64_t e[4];
  memcpy(e, P::M, 32);
  e[0] -= 2;
  return pow(a, e);
}

// big-endian 32 bytes <-> LE limbs
inline void be32_to_u64(const uint8_t* b, uint64_t out[4]) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[(3 - i) * 8 + k];
    out[i] = w;
  }
}
inline void u64_to_be32(const uint64_t in[4], uint8_t* b) {
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) b[(3 - i) * 8 + k] = (uint8_t)(in[i] >> (56 - 8 * k));
}

using Fp = F<ModP>;
using Fr = F<ModR>;

// Fr helpers in canonical form
inline Fr fr_from_be(const uint8_t* b32) {
  // reduce an arbitrary 256-bit big-endian value mod r
  uint64_t c[4];
  be32_to_u64(b32, c);
  while (geq_mod<ModR>(c)) sub_mod_raw<ModR>(c);
  return to_mont<ModR>(c);
}
inline void fr_to_be(const Fr& a, uint8_t* b32) {
  uint64_t c[4];
  from_mont(a, c);
  u64_to_be32(c, b32);
}
// SHA-256 digest as big-endian integer mod r (mathlib CurveBase.HashToZr)
inline Fr fr_from_digest(const uint8_t* d32) { return fr_from_be(d32); }

// ------------------------------------------------------------------ G1
struct G1A {  // affine, Montgomery coordinates; inf flag
  Fp x, y;
  bool inf;
};
struct G1J {  // Jacobian, Z = 0 <=> identity
  Fp x, y, z;
};

inline G1J jac_identity() { return G1J{Fp::one(), Fp::one(), Fp::zero()}; }
inline G1J to_jac(const G1A& a) { return a.inf ? jac_identity() : G1J{a.x, a.y, Fp::one()}; }

inline G1J jdbl(const G1J& p) {
  if (p.z.is_zero() || p.y.is_zero()) return jac_identity();
  Fp A = sqr(p.x), Bq = sqr(p.y), C = sqr(Bq);
  Fp t = add(p.x, Bq);
  Fp D = sub(sub(sqr(t), A), C);
  D = add(D, D);
  Fp E = add(add(A, A), A);
  Fp Fq = sqr(E);
  G1J r;
  r.x = sub(Fq, add(D, D));
  Fp C8 = add(C, C);
  C8 = add(C8, C8);
  C8 = add(C8, C8);
  r.y = sub(mul(E, sub(D, r.x)), C8);
  Fp yz = mul(p.y, p.z);
  r.z = add(yz, yz);
  return r;
}

inline G1J jadd(const G1J& p, const G1J& q) {
  if (p.z.is_zero()) return q;
  if (q.z.is_zero()) return p;
  Fp z1z1 = sqr(p.z), z2z2 = sqr(q.z);
  Fp u1 = mul(p.x, z2z2), u2 = mul(q.x, z1z1);
  Fp s1 = mul(mul(p.y, q.z), z2z2), s2 = mul(mul(q.y, p.z), z1z1);
  if (u1 == u2) {
    if (s1 == s2) return jdbl(p);
    return jac_identity();
  }
  Fp h = sub(u2, u1);
  Fp i = sqr(add(h, h));
  Fp j = mul(h, i);
  Fp rr = sub(s2, s1);
  rr = add(rr, rr);
  Fp v = mul(u1, i);
  G1J r;
  r.x = sub(sub(sqr(rr), j), add(v, v));
  Fp s1j = mul(s1, j);
  r.y = sub(mul(rr, sub(v, r.x)), add(s1j, s1j));
  r.z = mul(sub(sub(sqr(add(p.z, q.z)), z1z1), z2z2), h);
  return r;
}

// mixed add p + q (q affine)
inline G1J jadd_aff(const G1J& p, const G1A& q) {
  if (q.inf) return p;
  if (p.z.is_zero()) return to_jac(q);
  Fp z1z1 = sqr(p.z);
  Fp u2 = mul(q.x, z1z1);
  Fp s2 = mul(mul(q.y, p.z), z1z1);
  if (u2 == p.x) {
    if (s2 == p.y) return jdbl(p);
    return jac_identity();
  }
  Fp h = sub(u2, p.x);
  Fp hh = sqr(h);
  Fp i = add(hh, hh);
  i = add(i, i);
  Fp j = mul(h, i);
  Fp rr = sub(s2, p.y);
  rr = add(rr, rr);
  Fp v = mul(p.x, i);
  G1J r;
  r.x = sub(sub(sqr(rr), j), add(v, v));
  Fp yj = mul(p.y, j);
  r.y = sub(mul(rr, sub(v, r.x)), add(yj, yj));
  r.z = sub(sub(sqr(add(p.z, h)), z1z1), hh);
  return r;
}

inline G1A to_aff(const G1J& p) {
  if (p.z.is_zero()) return G1A{Fp::zero(), Fp::zero(), true};
  Fp zi = inv(p.z), zi2 = sqr(zi);
  return G1A{mul(p.x, zi2), mul(mul(p.y, zi2), zi), false};
}

inline G1A aff_neg(const G1A& a) {
  G1A r = a;
  if (!a.inf) r.y = neg(a.y);
  return r;
}

// batch normalisation (Montgomery trick)
inline void to_aff_batch(const G1J* in, G1A* out, size_t n) {
  std::vector<Fp> pre(n);
  Fp acc = Fp::one();
  for (size_t i = 0; i < n; i++) {
    pre[i] = acc;
    if (!in[i].z.is_zero()) acc = mul(acc, in[i].z);
  }
  Fp ia = inv(acc);
  for (size_t i = n; i-- > 0;) {
    if (in[i].z.is_zero()) {
      out[i] = G1A{Fp::zero(), Fp::zero(), true};
      continue;
    }
    Fp zi = mul(ia, pre[i]);
    ia = mul(ia, in[i].z);
    Fp zi2 = sqr(zi);
    out[i] = G1A{mul(in[i].x, zi2), mul(mul(in[i].y, zi2), zi), false};
  }
}

// variable-base scalar multiplication, 4-bit fixed window; k canonical LE limbs
inline G1J mul_var(const G1A& p, const uint64_t k[4]) {
  G1J tbl[16];
  tbl[0] = jac_identity();
  tbl[1] = to_jac(p);
  for (int i = 2; i < 16; i++) tbl[i] = jadd_aff(tbl[i - 1], p);
  G1J acc = jac_identity();
  for (int i = 63; i >= 0; i--) {
    for (int d = 0; d < 4; d++) acc = jdbl(acc);
    int nib = (int)((k[i / 16] >> ((i % 16) * 4)) & 15);
    if (nib) acc = jadd(acc, tbl[nib]);
  }
  return acc;
}
inline G1J mul_var(const G1A& p, const Fr& s) {
  uint64_t k[4];
  from_mont(s, k);
  return mul_var(p, k);
}

// Fixed-base table: for window w (8-bit, unsigned digits 1..255), entry
// d*2^(8w)*B in affine form.  32 windows x 255 entries.
struct FixedBase {
  std::vector<G1A> t;  // [32][256], entry 0 unused
  void build(const G1A& base) {
    t.assign(32 * 256, G1A{Fp::zero(), Fp::zero(), true});
    std::vector<G1J> j(32 * 256);
    G1J bw = to_jac(base);
    for (int w = 0; w < 32; w++) {
      j[w * 256] = jac_identity();
      G1J acc = jac_identity();
      for (int d = 1; d < 256; d++) {
        acc = jadd(acc, bw);
        j[w * 256 + d] = acc;
      }
      for (int s = 0; s < 8; s++) bw = jdbl(bw);
    }
    to_aff_batch(j.data(), t.data(), j.size());
  }
  G1J mul(const Fr& s) const {
    uint64_t k[4];
    from_mont(s, k);
    G1J acc = jac_identity();
    for (int w = 0; w < 32; w++) {
      int d = (int)((k[w / 8] >> ((w % 8) * 8)) & 255);
      if (d) acc = jadd_aff(acc, t[w * 256 + d]);
    }
    return acc;
  }
};

// affine point <-> 64-byte big-endian X||Y (identity = 64 zero bytes)
inline void g1_to_bytes(const G1A& a, uint8_t out[64]) {
  if (a.inf) {
    memset(out, 0, 64);
    return;
  }
  uint64_t c[4];
  from_mont(a.x, c);
  u64_to_be32(c, out);
  from_mont(a.y, c);
  u64_to_be32(c, out + 32);
}

// NewG1FromBytes semantics (see oracle/bn254.py g1_from_bytes); false on error
inline bool g1_from_bytes(const uint8_t* b, size_t len, G1A& out) {
  if (len != 64) return false;
  if (b[0] & 0xC0) return false;
  uint64_t x[4], y[4];
  be32_to_u64(b, x);
  be32_to_u64(b + 32, y);
  if (geq_mod<ModP>(x) || geq_mod<ModP>(y)) return false;
  if ((x[0] | x[1] | x[2] | x[3] | y[0] | y[1] | y[2] | y[3]) == 0) {
    out = G1A{Fp::zero(), Fp::zero(), true};
    return true;
  }
  Fp X = to_mont<ModP>(x), Y = to_mont<ModP>(y);
  Fp rhs = add(mul(sqr(X), X), from_u64<ModP>(3));
  if (sqr(Y) != rhs) return false;
  out = G1A{X, Y, false};
  return true;
}

}  // namespace host
}  // namespace fts
