// Fixed-base scalar multiplication over device-resident window tables.
//
// Every public generator the verifier multiplies (H_i, G_i, ped0..2, P, Q,
// K = sum H_i - sum G_i) gets a table
//     T[w][d-1] = d * 2^(FB_W * w) * B,   d = 1 .. 2^(FB_W-1),  w < FB_NW
// of affine Montgomery points (16 words).  A canonical scalar k < r < 2^254
// is recoded into FB_NW signed FB_W-bit digits, so k*B costs FB_NW mixed
// additions and no doublings.  With FB_W = 16 that is 16 additions per
// product (32 with byte windows) for 32 MiB of table per base: the
// 134 bases of a 64-bit context take 4.3 GiB of HBM, which the 288 GB part
// affords; every lookup is one 64-byte gather.
//
// The multiplication loop is fully inlined (no out-of-line calls: the call
// ABI would spill the accumulator to scratch on every addition) and
// prefetches the next table entry while the current addition runs.
#pragma once
#include "g1.hpp"

namespace fts {

constexpr int FB_W = 16;                                   // window bits
constexpr int FB_NW = (255 + FB_W - 1) / FB_W;             // windows (covers 255 bits)
constexpr int FB_E = 1 << (FB_W - 1);                      // entries per window
constexpr size_t FB_WORDS_PER_BASE = (size_t)FB_NW * FB_E * 16;
// two-level construction of a window: d - 1 = hi * FB_S + lo
constexpr int FB_S = 1 << ((FB_W) / 2);                    // small multiples per window
constexpr int FB_L = FB_E / FB_S;                          // large multiples per window

// The same layout for any window width W.  The per-proof bases of the
// range-proof pipeline (H_i, K, P: the n + 2 fixed-base products of every
// proof) use FBW_W = 20-bit windows: 13 mixed additions per product instead
// of 16, for 436 MiB per base (28.8 GiB at n = 64 -- the 288 GB part holds it).
template <int W>
struct FbCfg {
  static constexpr int NW = (255 + W - 1) / W;
  static constexpr int E = 1 << (W - 1);
  static constexpr size_t WORDS_PER_BASE = (size_t)NW * E * 16;
  static constexpr int S = 1 << (W / 2);
  static constexpr int L = E / S;
};
constexpr int FBW_W = 20;
using FbWide = FbCfg<FBW_W>;

// next signed digit of k (LSB first): consumes FB_W bits of s (shifted in
// place: constant register indices, no scratch), carry in/out via `carry`
FTS_DEV int fb_next_digit(uint32_t s[8], int& carry) {
  int d = (int)(s[0] & (uint32_t)(2 * FB_E - 1)) + carry;
#pragma unroll
  for (int i = 0; i < 7; i++) s[i] = (s[i] >> FB_W) | (s[i + 1] << (32 - FB_W));
  s[7] >>= FB_W;
  carry = d > FB_E;
  return carry ? d - 2 * FB_E : d;
}

// p += q (q affine, not the identity): madd-2007-bl, inlined
FTS_DEV void madd_inl(G1J& p, const G1A& q) {
  if (f_is_zero(p.z)) {
    p.x = q.x;
    p.y = q.y;
    p.z = f_one<FpP>();
    return;
  }
  Fp z1z1 = fp_sqr(p.z);
  Fp u2 = fp_mul(q.x, z1z1);
  Fp s2 = fp_mul(fp_mul(q.y, p.z), z1z1);
  Fp h = f_sub(u2, p.x);
  Fp rr = f_sub(s2, p.y);
  if (f_is_zero(h)) {  // P == +-Q: exceptional, out of line
    p = f_is_zero(rr) ? g1j_dbl(p) : g1j_identity();
    return;
  }
  Fp hh = fp_sqr(h);
  Fp i = f_dbl(f_dbl(hh));
  Fp j = fp_mul(h, i);
  rr = f_dbl(rr);
  Fp v = fp_mul(p.x, i);
  Fp x3 = f_sub(f_sub(fp_sqr(rr), j), f_dbl(v));
  Fp y3 = f_sub(fp_mul(rr, f_sub(v, x3)), f_dbl(fp_mul(p.y, j)));
  p.z = f_sub(f_sub(fp_sqr(f_add(p.z, h)), z1z1), hh);
  p.x = x3;
  p.y = y3;
}

FTS_DEV G1A fb_entry(const uint32_t* __restrict__ table, int w, int d) {
  const int ad = d < 0 ? -d : d;
  G1A q = load_g1a(table + ((size_t)w * FB_E + (ad - 1)) * 16);
  if (d < 0) q.y = f_neg(q.y);
  return q;
}

// k * B for a canonical scalar k (8 LE limbs)
FTS_DEV G1J fb_mul(const uint32_t* __restrict__ table, const Scalar& k) {
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = k.v[i];
  G1J acc = g1j_identity();
  int carry = 0, w = 0, d = 0;
  // first nonzero digit
  for (; w < FB_NW; w++) {
    d = fb_next_digit(s, carry);
    if (d != 0) break;
  }
  if (w == FB_NW) return acc;
  G1A cur = fb_entry(table, w, d);
  for (;;) {
    int wn = w + 1, dn = 0;
    for (; wn < FB_NW; wn++) {
      dn = fb_next_digit(s, carry);
      if (dn != 0) break;
    }
    G1A nxt;
    if (wn < FB_NW) nxt = fb_entry(table, wn, dn);  // in flight during the addition
    madd_inl(acc, cur);
    if (wn >= FB_NW) break;
    cur = nxt;
    w = wn;
  }
  return acc;
}

// ka * A + kb * B over two 16-bit-window tables in ONE accumulator: a
// fixed-base product is a sum of table entries (no doublings), so the joint sum
// takes the two products' additions with no final full addition; the next
// window's entries are loaded during the current window's additions
FTS_DEV G1J fb_mul2(const uint32_t* __restrict__ ta, const Scalar& ka, const uint32_t* __restrict__ tb,
                    const Scalar& kb) {
  uint32_t sa[8], sb[8];
#pragma unroll
  for (int i = 0; i < 8; i++) sa[i] = ka.v[i], sb[i] = kb.v[i];
  G1J acc = g1j_identity();
  int ca = 0, cb = 0;
  int da = fb_next_digit(sa, ca), db = fb_next_digit(sb, cb);
  G1A qa, qb;
  if (da != 0) qa = fb_entry(ta, 0, da);
  if (db != 0) qb = fb_entry(tb, 0, db);
  for (int w = 0; w < FB_NW; w++) {
    int dan = 0, dbn = 0;
    G1A na, nb;
    if (w + 1 < FB_NW) {
      dan = fb_next_digit(sa, ca);
      dbn = fb_next_digit(sb, cb);
      if (dan != 0) na = fb_entry(ta, w + 1, dan);
      if (dbn != 0) nb = fb_entry(tb, w + 1, dbn);
    }
    if (da != 0) madd_inl(acc, qa);
    if (db != 0) madd_inl(acc, qb);
    da = dan, db = dbn, qa = na, qb = nb;
  }
  return acc;
}

// k * B over a width-W table (FbCfg<W> layout)
template <int W>
FTS_DEV int fb_next_digit_w(uint32_t s[8], int& carry) {
  constexpr int E = FbCfg<W>::E;
  int d = (int)(s[0] & (uint32_t)(2 * E - 1)) + carry;
#pragma unroll
  for (int i = 0; i < 7; i++) s[i] = (s[i] >> W) | (s[i + 1] << (32 - W));
  s[7] >>= W;
  carry = d > E;
  return carry ? d - 2 * E : d;
}
template <int W>
FTS_DEV G1A fb_entry_w(const uint32_t* __restrict__ table, int w, int d) {
  const int ad = d < 0 ? -d : d;
  G1A q = load_g1a(table + ((size_t)w * FbCfg<W>::E + (ad - 1)) * 16);
  if (d < 0) q.y = f_neg(q.y);
  return q;
}
template <int W>
FTS_DEV G1J fb_mul_w(const uint32_t* __restrict__ table, const Scalar& k) {
  constexpr int NW = FbCfg<W>::NW;
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = k.v[i];
  G1J acc = g1j_identity();
  int carry = 0, w = 0, d = 0;
  for (; w < NW; w++) {
    d = fb_next_digit_w<W>(s, carry);
    if (d != 0) break;
  }
  if (w == NW) return acc;
  G1A cur = fb_entry_w<W>(table, w, d);
  for (;;) {
    int wn = w + 1, dn = 0;
    for (; wn < NW; wn++) {
      dn = fb_next_digit_w<W>(s, carry);
      if (dn != 0) break;
    }
    G1A nxt;
    if (wn < NW) nxt = fb_entry_w<W>(table, wn, dn);  // in flight during the addition
    madd_inl(acc, cur);
    if (wn >= NW) break;
    cur = nxt;
    w = wn;
  }
  return acc;
}

// acc += k * B over a 16-bit window table (fb_mul of fixed_base.hpp, but into
// an existing accumulator)
FTS_DEV void fb_mul_acc(G1J& acc, const uint32_t* __restrict__ table, const Scalar& k) {
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = k.v[i];
  int carry = 0, w = 0, d = 0;
  for (; w < FB_NW; w++) {
    d = fb_next_digit(s, carry);
    if (d != 0) break;
  }
  if (w == FB_NW) return;
  G1A cur = fb_entry(table, w, d);
  for (;;) {
    int wn = w + 1, dn = 0;
    for (; wn < FB_NW; wn++) {
      dn = fb_next_digit(s, carry);
      if (dn != 0) break;
    }
    G1A nxt;
    if (wn < FB_NW) nxt = fb_entry(table, wn, dn);  // in flight during the addition
    madd_inl(acc, cur);
    if (wn >= FB_NW) break;
    cur = nxt;
    w = wn;
  }
}

// acc += k * B over a width-W table (FbCfg<W> layout; fb_mul_w into a running accumulator)
template <int W>
FTS_DEV void fb_mul_acc_w(G1J& acc, const uint32_t* __restrict__ table, const Scalar& k) {
  constexpr int NW = FbCfg<W>::NW;
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = k.v[i];
  int carry = 0, w = 0, d = 0;
  for (; w < NW; w++) {
    d = fb_next_digit_w<W>(s, carry);
    if (d != 0) break;
  }
  if (w == NW) return;
  G1A cur = fb_entry_w<W>(table, w, d);
  for (;;) {
    int wn = w + 1, dn = 0;
    for (; wn < NW; wn++) {
      dn = fb_next_digit_w<W>(s, carry);
      if (dn != 0) break;
    }
    G1A nxt;
    if (wn < NW) nxt = fb_entry_w<W>(table, wn, dn);  // in flight during the addition
    madd_inl(acc, cur);
    if (wn >= NW) break;
    cur = nxt;
    w = wn;
  }
}

// out-of-line copy for cold call sites (keeps their kernels small)
__device__ __noinline__ G1J nl_fb_mul(const uint32_t* __restrict__ table, Scalar k) { return fb_mul(table, k); }

}  // namespace fts
