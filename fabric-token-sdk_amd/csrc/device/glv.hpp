// GLV endomorphism of BN254 G1 (y^2 = x^3 + 3, j-invariant 0):
//   phi(x, y) = (beta x, y) = lambda * (x, y),   beta^3 = 1 in Fp, lambda^3 = 1 in Fr.
// A scalar k < r splits as k = k1 + k2 * lambda (mod r) with |k1|, |k2| < 2^126
// (lattice basis v1 = (a1, b1), v2 = (a2, b2) of {(x, y): x + y lambda = 0 mod r},
// Babai rounding with precomputed g_i = floor(2^384 * b_i / r); the rounding
// error only changes which short vector is found, never k1 + k2 lambda).
// This halves the doubling chain of every variable-base product: the
// per-proof x*D, the sigma proofs' challenge products and the RLC MSM's
// Horner (254 -> 127 doublings).  gnark-crypto uses the same endomorphism
// (ecc/bn254 G1 ScalarMultiplication); the values here are derived from the
// curve (tools/glv_constants.py), not copied.
#pragma once
#include "fixed_base.hpp"  // madd_inl (includes g1.hpp)

namespace fts {

struct Glv {
  // beta in Montgomery form (Fp), paired with lambda = 0xb3c4d79d...c90dd
  static constexpr uint32_t BETA[8] = {0xd782e155u, 0x71930c11u, 0xffbe3323u, 0xa6bb947cu,
                                       0xd4741444u, 0xaa303344u, 0x26594943u, 0x2c3b3f0du};
  static constexpr uint32_t G1[7] = {0x2fafba64u, 0x8fa7d32du, 0x773a6ef2u, 0x6eb9c714u,
                                     0xc7e0b3d7u, 0xd91d232eu, 0x00000002u};
  static constexpr uint32_t G2[9] = {0x9b9bdffau, 0x86937516u, 0x5eaa26d9u, 0xa5e38cfbu, 0x391eb18du,
                                     0x7a7bd9d4u, 0xa773d2cfu, 0x4ccef014u, 0x00000002u};
  static constexpr uint32_t A1[2] = {0x94d213e3u, 0x89d32568u};                          // a1 (= b2)
  static constexpr uint32_t A2[4] = {0x1221250bu, 0x0be4e154u, 0xeeb859fdu, 0x6f4d8248u};  // a2
  static constexpr uint32_t NB1[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u}; // -b1
};

// c = round(k * g / 2^384) for a G-limb constant g; returns the low 5 limbs
template <int G>
FTS_DEV void glv_round(const uint32_t k[8], const uint32_t (&g)[G], uint32_t c[5]) {
  // full product limbs 11 .. 8+G-1 are needed (limb 11 for the rounding bit)
  uint32_t t[8 + G];
#pragma unroll
  for (int i = 0; i < 8 + G; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < G; j++) {
      uint64_t v = (uint64_t)k[i] * g[j] + t[i + j] + carry;
      t[i + j] = (uint32_t)v;
      carry = v >> 32;
    }
    t[i + G] = (uint32_t)carry;
  }
  // + 2^383 (rounding), then >> 384 (limb 12)
  uint32_t cy = (t[11] >> 31);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint32_t v = (12 + i) < 8 + G ? t[12 + i] : 0u;
    c[i] = addc(v, 0u, cy, cy);
  }
}

// r -= a * b (mod 2^256), a: NA limbs, b: NB limbs
template <int NA, int NB>
FTS_DEV void sub_mul_256(uint32_t r[8], const uint32_t* a, const uint32_t* b) {
  uint32_t p[8];
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
      if (i + j < 8) {
        uint64_t v = (uint64_t)a[i] * b[j] + p[i + j] + carry;
        p[i + j] = (uint32_t)v;
        carry = v >> 32;
      }
    }
    if (i + NB < 8) p[i + NB] = (uint32_t)carry;
  }
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = subb(r[i], p[i], bw, bw);
}

// two's-complement 256-bit -> (|v| low 4 limbs, sign)
FTS_DEV uint32_t glv_abs(const uint32_t v[8], uint32_t out[4]) {
  const uint32_t neg = v[7] >> 31;
  uint32_t c = neg;
#pragma unroll
  for (int i = 0; i < 4; i++) out[i] = addc(neg ? ~v[i] : v[i], 0u, c, c);
  return neg;
}

// k (canonical, 8 limbs) -> k1, k2 (|.| in 4 limbs) with signs: k = k1 + k2 lambda mod r.
// K: the curve's constants (Glv for BN254; fbn::GlvK for FP256BN, same basis shape:
// a1 = b2 > 0 of 64 bits, a2 > 0 and -b1 > 0 of 128 bits)
template <class K = Glv>
FTS_DEV void glv_decompose(const uint32_t k[8], uint32_t k1[4], uint32_t& s1, uint32_t k2[4], uint32_t& s2) {
  uint32_t c1[5], c2[5];
  glv_round<7>(k, K::G1, c1);
  glv_round<9>(k, K::G2, c2);
  uint32_t r1[8], r2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r1[i] = k[i];
    r2[i] = 0;
  }
  // k1 = k - c1 a1 - c2 a2
  sub_mul_256<3, 2>(r1, c1, K::A1);
  sub_mul_256<5, 4>(r1, c2, K::A2);
  // k2 = c1 (-b1) - c2 b2 = -( c2 b2 - c1 (-b1) )   (b2 = a1)
  sub_mul_256<5, 2>(r2, c2, K::A1);  // r2 = -c2 b2
  {
    uint32_t p[8];
#pragma unroll
    for (int i = 0; i < 8; i++) p[i] = 0;
    sub_mul_256<3, 4>(p, c1, K::NB1);  // p = -c1 (-b1)
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r2[i] = subb(r2[i], p[i], bw, bw);  // r2 = -c2 b2 + c1 (-b1)
  }
  s1 = glv_abs(r1, k1);
  s2 = glv_abs(r2, k2);
}

FTS_DEV Fp glv_beta() {
  Fp b;
#pragma unroll
  for (int i = 0; i < 8; i++) b.v[i] = Glv::BETA[i];
  return b;
}

// p += q (both Jacobian): add-2007-bl, inlined (exceptional cases inline too,
// so the caller's loop never makes an out-of-line call)
FTS_DEV void add_inl(G1J& p, const G1J& q) {
  if (f_is_zero(q.z)) return;
  if (f_is_zero(p.z)) {
    p = q;
    return;
  }
  Fp z1z1 = fp_sqr(p.z);
  Fp z2z2 = fp_sqr(q.z);
  Fp u1 = fp_mul(p.x, z2z2);
  Fp u2 = fp_mul(q.x, z1z1);
  Fp s1 = fp_mul(fp_mul(p.y, q.z), z2z2);
  Fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  Fp h = f_sub(u2, u1);
  Fp rr = f_sub(s2, s1);
  if (f_is_zero(h)) {
    p = f_is_zero(rr) ? g1j_dbl(p) : g1j_identity();
    return;
  }
  Fp i = fp_sqr(f_dbl(h));
  Fp j = fp_mul(h, i);
  rr = f_dbl(rr);
  Fp v = fp_mul(u1, i);
  Fp x3 = f_sub(f_sub(fp_sqr(rr), j), f_dbl(v));
  Fp y3 = f_sub(fp_mul(rr, f_sub(v, x3)), f_dbl(fp_mul(s1, j)));
  p.z = fp_mul(f_sub(f_sub(fp_sqr(f_add(p.z, q.z)), z1z1), z2z2), h);
  p.x = x3;
  p.y = y3;
}

// Per-lane table of 1..8 * P in global memory, [entry][word][stride] with
// stride = lanes of the launch and idx = the lane's global id (coalesced when
// neighbouring lanes use the same entry; 768 B per lane, L2/MALL-resident).
// Kept out of LDS: a 48 KB LDS table per 64-lane block capped the kernel at
// 3 waves per CU.
FTS_DEV void vtab_store(uint32_t* __restrict__ tab, size_t stride, size_t idx, int e, const G1J& p) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    tab[((size_t)(e * 24) + i) * stride + idx] = p.x.v[i];
    tab[((size_t)(e * 24) + 8 + i) * stride + idx] = p.y.v[i];
    tab[((size_t)(e * 24) + 16 + i) * stride + idx] = p.z.v[i];
  }
}
FTS_DEV G1J vtab_load(const uint32_t* __restrict__ tab, size_t stride, size_t idx, int e) {
  G1J p;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p.x.v[i] = tab[((size_t)(e * 24) + i) * stride + idx];
    p.y.v[i] = tab[((size_t)(e * 24) + 8 + i) * stride + idx];
    p.z.v[i] = tab[((size_t)(e * 24) + 16 + i) * stride + idx];
  }
  return p;
}

// k * P for a 128-bit magnitude k (4 LE limbs, < 2^127): signed 4-bit
// windows (32 windows), 1 + 6 table additions, 124 doublings, <= 32 additions.
// The table entry of a window is loaded before that window's 4 doublings, so
// its latency hides behind them.
FTS_DEV G1J vb128j(const G1J& t, const uint32_t kk[4], uint32_t* __restrict__ tab, size_t stride, size_t idx) {
  if (f_is_zero(t.z)) return g1j_identity();
  {
    vtab_store(tab, stride, idx, 0, t);
    G1J cur = g1j_dbl(t);
    vtab_store(tab, stride, idx, 1, cur);
    for (int e = 2; e < 8; e++) {
      add_inl(cur, t);
      vtab_store(tab, stride, idx, e, cur);
    }
  }
  uint32_t s[4];
#pragma unroll
  for (int i = 0; i < 4; i++) s[i] = kk[i];
  // carries of the signed recoding (LSB first), one bit per window
  uint32_t cm = 0;
  {
    int carry = 0;
#pragma unroll
    for (int w = 0; w < 32; w++) {
      cm |= (uint32_t)carry << w;
      int d = (int)((s[w >> 3] >> (4 * (w & 7))) & 0xfu) + carry;
      carry = d > 8;
    }
  }
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    // window w raw nibble (s shifted left by 4 each step: MSB nibble of s[3])
    int raw = (int)(s[3] >> 28);
    s[3] = (s[3] << 4) | (s[2] >> 28);
    s[2] = (s[2] << 4) | (s[1] >> 28);
    s[1] = (s[1] << 4) | (s[0] >> 28);
    s[0] <<= 4;
    int cin = (int)((cm >> w) & 1u);
    int cout = w < 31 ? (int)((cm >> (w + 1)) & 1u) : 0;
    int d = raw + cin - 16 * cout;
    G1J q;
    if (d != 0) q = vtab_load(tab, stride, idx, (d < 0 ? -d : d) - 1);
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (d != 0) {
      if (d < 0) q.y = f_neg(q.y);
      add_inl(acc, q);
    }
  }
  return acc;
}

// Joint GLV/Straus half: a * P + b * Q for 127-bit magnitudes a, b (4 LE
// limbs each, signs already folded into P, Q): ONE chain of 124 doublings
// with <= 2 x 32 additions (two separate products double 2 x 124 times).
// Tables 1..8 * P (entries 0..7) and 1..8 * Q (8..15) in global memory as
// vtab_*; both window entries are loaded before the window's doublings.
FTS_DEV uint32_t recode_carries(const uint32_t s[4]) {
  uint32_t cm = 0;
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 32; w++) {
    cm |= (uint32_t)carry << w;
    int d = (int)((s[w >> 3] >> (4 * (w & 7))) & 0xfu) + carry;
    carry = d > 8;
  }
  return cm;
}
// s[q] for a runtime (wave-uniform) q by selects: indexing the array with a
// runtime value made the compiler promote it to LDS (k_rp_com_var: 16 KB per
// 64-lane block, holding every CU's LDS beside the x0 build; round 5)
FTS_DEV uint32_t word4(const uint32_t s[4], int q) {
  const uint32_t lo = (q & 1) ? s[1] : s[0], hi = (q & 1) ? s[3] : s[2];
  return (q & 2) ? hi : lo;
}
FTS_DEV int window_digit(const uint32_t s[4], uint32_t cm, int w) {
  const int raw = (int)((word4(s, w >> 3) >> (4 * (w & 7))) & 0xfu);
  const int cin = (int)((cm >> w) & 1u);
  const int cout = w < 31 ? (int)((cm >> (w + 1)) & 1u) : 0;
  return raw + cin - 16 * cout;
}
FTS_DEV void vtab_build(const G1J& t, uint32_t* __restrict__ tab, size_t stride, size_t idx, int e0) {
  vtab_store(tab, stride, idx, e0, t);
  if (f_is_zero(t.z)) {  // identity: every multiple is the identity
    for (int e = 1; e < 8; e++) vtab_store(tab, stride, idx, e0 + e, t);
    return;
  }
  G1J cur = g1j_dbl(t);
  vtab_store(tab, stride, idx, e0 + 1, cur);
  for (int e = 2; e < 8; e++) {
    add_inl(cur, t);
    vtab_store(tab, stride, idx, e0 + e, cur);
  }
}
FTS_DEV G1J straus2_128(const G1J& P, const uint32_t a[4], const G1J& Q, const uint32_t b[4], uint32_t* __restrict__ tab,
                        size_t stride, size_t idx) {
  vtab_build(P, tab, stride, idx, 0);
  vtab_build(Q, tab, stride, idx, 8);
  const uint32_t ca = recode_carries(a), cb = recode_carries(b);
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    const int da = window_digit(a, ca, w), db = window_digit(b, cb, w);
    G1J qa, qb;
    if (da != 0) qa = vtab_load(tab, stride, idx, (da < 0 ? -da : da) - 1);
    if (db != 0) qb = vtab_load(tab, stride, idx, 8 + (db < 0 ? -db : db) - 1);
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (da != 0) {
      if (da < 0) qa.y = f_neg(qa.y);
      add_inl(acc, qa);
    }
    if (db != 0) {
      if (db < 0) qb.y = f_neg(qb.y);
      add_inl(acc, qb);
    }
  }
  return acc;
}

// --------------------------------------------------------- affine lane tables
// Joint Straus a*P + b*Q over AFFINE tables (the work path's com chain,
// DESIGN.md §3.1): entries 0..7 = 1..8 * P, 8..15 = 1..8 * Q, affine
// Montgomery, one 64-byte row (x || y, four 16-byte loads) per lane and entry,
// entry-major: row (e, lane) at ((e * L) + lane) * 16 words, L = lanes of the
// launch.  The build phase writes and re-reads the same entry in every lane at
// once (fully coalesced 4 KB per wave); a window lookup reads one row per lane.
// The multiples are built Jacobian (X, Y into the row, Z and the running
// product of the z's beside), then normalised with ONE inversion per lane
// (Montgomery's trick over the 16 z's), so every window addition is mixed
// (madd-2007-bl, 7M + 4S) instead of full (11M + 5S).
// Region layout: XY [16][L][16] | Z [16][L][8] | PRE [16][L][8]  (2 KB per lane)
constexpr int ATAB_WORDS = 512;  // words per lane of the region
struct ATab {
  uint32_t* base;
  size_t L, lane;
  FTS_DEV uint32_t* xy(int e) const { return base + ((size_t)e * L + lane) * 16; }
  FTS_DEV uint32_t* z(int e) const { return base + (size_t)16 * L * 16 + ((size_t)e * L + lane) * 8; }
  FTS_DEV uint32_t* pre(int e) const { return base + (size_t)16 * L * 24 + ((size_t)e * L + lane) * 8; }
};

// entries e0 .. e0+7 <- Jacobian 1..8 * P; `pre` carries the running product of
// the z's over all entries built so far (written to PRE).  AFF: P.z == 1 (the
// multiples are mixed additions of P).  An identity P is stored as (0, 0, 1),
// which normalises to the affine identity encoding (0, 0); the chain skips it.
template <bool AFF>
FTS_DEV void atab_build8(const ATab& T, int e0, const G1J& P, Fp& pre, bool ident) {
  G1J cur = P;
  G1A pa;
  if (AFF) pa.x = P.x, pa.y = P.y;
  if (ident) {
    cur.x = f_zero<FpP>();
    cur.y = f_zero<FpP>();
    cur.z = f_one<FpP>();
  }
  for (int e = 0; e < 8; e++) {
    if (!ident && e == 1) cur = g1j_dbl(P);
    if (!ident && e > 1) {
      if (AFF) madd_inl(cur, pa);
      else add_inl(cur, P);
    }
    store_fp(T.xy(e0 + e), cur.x);
    store_fp(T.xy(e0 + e) + 8, cur.y);
    store_fp(T.z(e0 + e), cur.z);
    pre = (e0 == 0 && e == 0) ? cur.z : fp_mul(pre, cur.z);
    store_fp(T.pre(e0 + e), pre);
  }
}

// the first NE entries -> affine: z_e^-1 = (z_0 .. z_e)^-1 * (z_0 .. z_{e-1}), one inversion
template <int NE = 16>
FTS_DEV void atab_normalize(const ATab& T) {
  Fp inv;
  load_fp(T.pre(NE - 1), inv);
  inv = nl_fp_inv(inv);
  for (int e = NE - 1; e >= 0; e--) {
    Fp zi = inv;
    if (e > 0) {
      Fp pp, z;
      load_fp(T.pre(e - 1), pp);
      load_fp(T.z(e), z);
      zi = fp_mul(inv, pp);
      inv = fp_mul(inv, z);
    }
    Fp x, y;
    load_fp(T.xy(e), x);
    load_fp(T.xy(e) + 8, y);
    const Fp zi2 = fp_sqr(zi);
    store_fp(T.xy(e), fp_mul(x, zi2));
    store_fp(T.xy(e) + 8, fp_mul(fp_mul(y, zi2), zi));
  }
}

// a * P (127-bit magnitude, sign folded into P) over a normalised 8-entry
// table (entries 0..7 = 1..8 P): 124 doublings, <= 32 mixed additions
FTS_DEV G1J straus1_atab(const ATab& T, const uint32_t a[4], bool ida) {
  const uint32_t ca = recode_carries(a);
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    const int da = ida ? 0 : window_digit(a, ca, w);
    G1A qa;
    if (da != 0) qa = load_g1a(T.xy((da < 0 ? -da : da) - 1));
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (da != 0) {
      if (da < 0) qa.y = f_neg(qa.y);
      madd_inl(acc, qa);
    }
  }
  return acc;
}

// a * P + b * Q (127-bit magnitudes, signs folded into P, Q) over a normalised
// table: 124 doublings, <= 64 mixed additions; ida / idb: P / Q is the identity
FTS_DEV G1J straus2_atab(const ATab& T, const uint32_t a[4], const uint32_t b[4], bool ida, bool idb) {
  const uint32_t ca = recode_carries(a), cb = recode_carries(b);
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    const int da = ida ? 0 : window_digit(a, ca, w), db = idb ? 0 : window_digit(b, cb, w);
    G1A qa, qb;
    if (da != 0) qa = load_g1a(T.xy((da < 0 ? -da : da) - 1));
    if (db != 0) qb = load_g1a(T.xy(8 + (db < 0 ? -db : db) - 1));
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (da != 0) {
      if (da < 0) qa.y = f_neg(qa.y);
      madd_inl(acc, qa);
    }
    if (db != 0) {
      if (db < 0) qb.y = f_neg(qb.y);
      madd_inl(acc, qb);
    }
  }
  return acc;
}

// ------------------------------------------- per-proof shared tables (com chain)
// k_rp_com_var's two lanes of a proof share ONE affine table: lane 0 builds and
// normalises 1..8 D (entries 0..7), lane 1 1..8 S (entries 8..15), unsigned and
// without phi; each entry also carries beta*x, so the lane of the phi half reads
// phi(e P) = (beta x, y) and applies its GLV sign to y at lookup.  Half the table
// work and one inversion per lane of the per-lane tables (ATab).
// Region layout: XY [16][B][16] | BX [16][B][8] | Z [16][B][8] | PRE [16][B][8]
// (2,560 B per proof), row (e, proof) entry-major.
constexpr int CTAB_WORDS = 16 * 40;  // words per proof
struct CTab {
  uint32_t* base;
  size_t L, p;  // proofs in the launch, this proof
  FTS_DEV uint32_t* xy(int e) const { return base + ((size_t)e * L + p) * 16; }
  FTS_DEV uint32_t* bx(int e) const { return base + (size_t)16 * L * 16 + ((size_t)e * L + p) * 8; }
  FTS_DEV uint32_t* z(int e) const { return base + (size_t)16 * L * 24 + ((size_t)e * L + p) * 8; }
  FTS_DEV uint32_t* pre(int e) const { return base + (size_t)16 * L * 32 + ((size_t)e * L + p) * 8; }
};
// One point's 8-entry table in one lane (the sigma proofs' variable-base products,
// k_sig_var): the CTab row layout for entries 0..7 only.
// Region layout: XY [8][L][16] | BX [8][L][8] | Z [8][L][8] | PRE [8][L][8] (1,280 B per lane)
constexpr int CTAB8_WORDS = 8 * 40;  // words per lane
struct CTab8 {
  uint32_t* base;
  size_t L, p;  // lanes in the launch, this lane
  FTS_DEV uint32_t* xy(int e) const { return base + ((size_t)e * L + p) * 16; }
  FTS_DEV uint32_t* bx(int e) const { return base + (size_t)8 * L * 16 + ((size_t)e * L + p) * 8; }
  FTS_DEV uint32_t* z(int e) const { return base + (size_t)8 * L * 24 + ((size_t)e * L + p) * 8; }
  FTS_DEV uint32_t* pre(int e) const { return base + (size_t)8 * L * 32 + ((size_t)e * L + p) * 8; }
};
// entries e0 .. e0+7 <- 1..8 * P (Jacobian, then normalised with one inversion):
// AFF: P.z == 1 (mixed additions).  An identity P gives (0, 0) entries (skipped by
// the chain, which knows the identity flags).  TabT: CTab or CTab8.
template <bool AFF, class TabT>
FTS_DEV void ctab_build8(const TabT& T, int e0, const G1J& P, bool ident) {
  G1J cur = P;
  G1A pa;
  if (AFF) pa.x = P.x, pa.y = P.y;
  if (ident) {
    cur.x = f_zero<FpP>();
    cur.y = f_zero<FpP>();
    cur.z = f_one<FpP>();
  }
  Fp pre;
  for (int e = 0; e < 8; e++) {
    if (!ident && e == 1) cur = g1j_dbl(P);
    if (!ident && e > 1) {
      if (AFF) madd_inl(cur, pa);
      else add_inl(cur, P);
    }
    store_fp(T.xy(e0 + e), cur.x);
    store_fp(T.xy(e0 + e) + 8, cur.y);
    store_fp(T.z(e0 + e), cur.z);
    pre = e == 0 ? cur.z : fp_mul(pre, cur.z);
    store_fp(T.pre(e0 + e), pre);
  }
  Fp inv = nl_fp_inv(pre);
  const Fp beta = glv_beta();
  for (int e = 7; e >= 0; e--) {
    Fp zi = inv;
    if (e > 0) {
      Fp pp, z;
      load_fp(T.pre(e0 + e - 1), pp);
      load_fp(T.z(e0 + e), z);
      zi = fp_mul(inv, pp);
      inv = fp_mul(inv, z);
    }
    Fp x, y;
    load_fp(T.xy(e0 + e), x);
    load_fp(T.xy(e0 + e) + 8, y);
    const Fp zi2 = fp_sqr(zi);
    x = fp_mul(x, zi2);
    store_fp(T.xy(e0 + e), x);
    store_fp(T.xy(e0 + e) + 8, fp_mul(fp_mul(y, zi2), zi));
    store_fp(T.bx(e0 + e), fp_mul(x, beta));
  }
}
// a phi^h(sa D) + b phi^h(sb S) over the shared table (sa, sb: the GLV signs of the
// two half scalars, folded into y at lookup): 124 doublings, <= 64 mixed additions
FTS_DEV G1J straus2_ctab(const CTab& T, int h, const uint32_t a[4], bool sa, const uint32_t b[4], bool sb, bool ida,
                         bool idb) {
  const uint32_t ca = recode_carries(a), cb = recode_carries(b);
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    const int da = ida ? 0 : window_digit(a, ca, w), db = idb ? 0 : window_digit(b, cb, w);
    G1A qa, qb;
    if (da != 0) {
      const int e = (da < 0 ? -da : da) - 1;
      load_fp(h ? T.bx(e) : T.xy(e), qa.x);
      load_fp(T.xy(e) + 8, qa.y);
    }
    if (db != 0) {
      const int e = 8 + (db < 0 ? -db : db) - 1;
      load_fp(h ? T.bx(e) : T.xy(e), qb.x);
      load_fp(T.xy(e) + 8, qb.y);
    }
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (da != 0) {
      if ((da < 0) != sa) qa.y = f_neg(qa.y);
      madd_inl(acc, qa);
    }
    if (db != 0) {
      if ((db < 0) != sb) qb.y = f_neg(qb.y);
      madd_inl(acc, qb);
    }
  }
  return acc;
}

// k * P for a canonical scalar k < r and an affine P in one lane, over the lane's
// own affine table: GLV split k = k1 + k2 lambda, entries 1..8 P carry beta*x so
// phi(eP) = (beta x, y); the GLV signs fold into y at lookup.  124 doublings and
// <= 64 MIXED additions (glv_mul below: full additions over Jacobian tables), for
// one inversion and 8 beta products in the table.  One call site per kernel (as
// glv_mul).
FTS_DEV G1J glv_mul_ctab8(const CTab8& T, const G1A& p, const Scalar& k) {
  if (g1a_is_identity(p)) return g1j_identity();
  uint32_t k1[4], k2[4], s1, s2;
  glv_decompose(k.v, k1, s1, k2, s2);
  ctab_build8<true>(T, 0, g1j_from_affine(p), false);
  const uint32_t c1 = recode_carries(k1), c2 = recode_carries(k2);
  G1J acc = g1j_identity();
  for (int w = 31; w >= 0; w--) {
    const int da = window_digit(k1, c1, w), db = window_digit(k2, c2, w);
    G1A qa, qb;
    if (da != 0) {
      const int e = (da < 0 ? -da : da) - 1;
      load_fp(T.xy(e), qa.x);
      load_fp(T.xy(e) + 8, qa.y);
    }
    if (db != 0) {
      const int e = (db < 0 ? -db : db) - 1;
      load_fp(T.bx(e), qb.x);
      load_fp(T.xy(e) + 8, qb.y);
    }
    if (w != 31)
      for (int r = 0; r < 4; r++) acc = g1j_dbl(acc);
    if (da != 0) {
      if ((da < 0) != (s1 != 0)) qa.y = f_neg(qa.y);
      madd_inl(acc, qa);
    }
    if (db != 0) {
      if ((db < 0) != (s2 != 0)) qb.y = f_neg(qb.y);
      madd_inl(acc, qb);
    }
  }
  return acc;
}

// k * P for a canonical scalar k < r in one lane: GLV split k = k1 + k2 lambda,
// then the joint chain k1 P + k2 phi(P) (124 doublings instead of 252);
// tab/stride/idx: the lane's 16-entry table (straus2_128).  Keep it inlined
// at ONE call site per kernel: an out-of-line (__noinline__) build of this
// function never terminates on gfx950 -- branch relaxation in a callable
// function clobbers its return address s[30:31] (reproducer
// tools/experiments/glv_noinline_repro.hip, guard tools/long_branch_check.py,
// run by build() and tests/test_isa_cpu.py).
FTS_DEV G1J glv_mul(const G1A& p, const Scalar& k, uint32_t* __restrict__ tab, size_t stride, size_t idx) {
  if (g1a_is_identity(p)) return g1j_identity();
  uint32_t k1[4], k2[4], s1, s2;
  glv_decompose(k.v, k1, s1, k2, s2);
  G1J P = g1j_from_affine(p), Q = P;
  Q.x = fp_mul(Q.x, glv_beta());  // phi(P)
  if (s1) P.y = f_neg(P.y);
  if (s2) Q.y = f_neg(Q.y);
  return straus2_128(P, k1, Q, k2, tab, stride, idx);
}

}  // namespace fts
