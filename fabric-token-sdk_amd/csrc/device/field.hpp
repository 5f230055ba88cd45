// BN254 base field Fp and scalar field Fr on gfx950: 8 x 32-bit limbs,
// Montgomery form (R = 2^256), one element per lane.
//
// The reference delegates all of this to github.com/IBM/mathlib -> gnark-crypto
// ecc/bn254 (go.mod:8, go.mod:75; not vendored).  Every G1.Mul/Add and
// Curve.ModMul on the verification path (rp/bulletproof.go:252-509,
// rp/ipa.go:190-356, transfer/typeandsum.go:230-277) bottoms out here.
//
// Multiplication is the "no-carry" CIOS variant: both moduli have a top limb
// < 2^31 - 1, so the extra carry word of textbook CIOS is never needed and one
// product costs 2*8*8 + 8 = 136 v_mad_u64_u32.  There is no MFMA here: this is
// carry-propagating modular integer arithmetic, not a dense contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FTS_DEV __device__ __forceinline__

namespace fts {

struct FpP {
  static constexpr uint32_t M[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xe4866389u;  // -M^-1 mod 2^32
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr uint32_t R3[8] = {0xda1530dfu, 0xb1cd6dafu, 0xa7283db6u, 0x62f210e6u,
                                     0x0ada0afbu, 0xef7f0b0cu, 0x2d592544u, 0x20fd6e90u};
  // 2^34 R^3 mod M: final factor of f_inv_gcd (17 outer steps x (32 - 30) bits)
  static constexpr uint32_t GCDC[8] = {0x13bd45e1u, 0x31d6a0d9u, 0x382c59a2u, 0x45fbf2bcu,
                                       0x1ab31dfbu, 0x5b5fa369u, 0xb36fd339u, 0x24811383u};
};

struct FrP {
  static constexpr uint32_t M[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xefffffffu;
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                                     0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};
  static constexpr uint32_t GCDC[8] = {0xdd8b6d21u, 0x352ff640u, 0x331ce10au, 0x011e8bd1u,
                                       0x55d392c2u, 0x438150aeu, 0x73335b20u, 0x21fe9388u};
};

template <class P>
struct Field {
  uint32_t v[8];
};

using Fp = Field<FpP>;
using Fr = Field<FrP>;

// ---------------------------------------------------------------- helpers
FTS_DEV uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
  uint32_t c;
  uint32_t s = __builtin_addc(a, b, cin, &c);
  cout = c;
  return s;
}
FTS_DEV uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
  uint32_t c;
  uint32_t s = __builtin_subc(a, b, bin, &c);
  bout = c;
  return s;
}

template <class P>
FTS_DEV Field<P> f_zero() {
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
  return r;
}
template <class P>
FTS_DEV Field<P> f_one() {
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = P::ONE[i];
  return r;
}
template <class P>
FTS_DEV bool f_is_zero(const Field<P>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i];
  return o == 0;
}
template <class P>
FTS_DEV bool f_eq(const Field<P>& a, const Field<P>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// r = a - M if a >= M else a   (a < 2M)
template <class P>
FTS_DEV void f_reduce_once(Field<P>& a) {
  uint32_t t[8], bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = subb(a.v[i], P::M[i], bw, bw);
  // bw == 1  <=> a < M  -> keep a
  const bool keep = bw != 0;
#pragma unroll
  for (int i = 0; i < 8; i++) a.v[i] = keep ? a.v[i] : t[i];
}

template <class P>
FTS_DEV Field<P> f_add(const Field<P>& a, const Field<P>& b) {
  Field<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc(a.v[i], b.v[i], c, c);
  // moduli < 2^254 so a + b < 2^255: no carry out of limb 7
  f_reduce_once(r);
  return r;
}

template <class P>
FTS_DEV Field<P> f_sub(const Field<P>& a, const Field<P>& b) {
  Field<P> r;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb(a.v[i], b.v[i], bw, bw);
  // if borrow: add M back
  const uint32_t mask = 0u - bw;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc(r.v[i], P::M[i] & mask, c, c);
  return r;
}

template <class P>
FTS_DEV Field<P> f_neg(const Field<P>& a) {
  return f_sub(f_zero<P>(), a);
}

template <class P>
FTS_DEV Field<P> f_dbl(const Field<P>& a) {
  return f_add(a, a);
}

// Montgomery product a*b*R^-1 mod M (no-carry CIOS, fully reduced output).
template <class P>
FTS_DEV Field<P> f_mul(const Field<P>& a, const Field<P>& b) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.v[i];
    uint64_t A = (uint64_t)a.v[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * P::INV;
    uint64_t C = (uint64_t)m * P::M[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      A = (uint64_t)a.v[j] * bi + t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * P::M[j] + t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[7] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// acc(96-bit: pair + ovf) += x*y.  v_mad_u64_u32's carry-out feeds the
// overflow word, so a column of products needs no extra register moves.
FTS_DEV void mac96(uint64_t& acc, uint32_t& ovf, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ovf)
      : "v"(x), "v"(y)
      : "vcc");
}
FTS_DEV void mac96s(uint64_t& acc, uint32_t& ovf, uint32_t x, uint32_t y_uniform) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ovf)
      : "v"(x), "s"(y_uniform)
      : "vcc");
}

// Runs of 2 / 4 MACs on one 96-bit accumulator inside one asm block.  The
// hazard recognizer pads every inline-asm boundary with an s_nop; grouping
// removes most of those pads from the dependent chain (the mad -> addc VCC
// dependency is interlocked, as in mac96).
#define FTS_MAC_LINE(X, Y) "v_mad_u64_u32 %0, vcc, %" #X ", %" #Y ", %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
FTS_DEV void mac96_2v(uint64_t& acc, uint32_t& ovf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
  asm(FTS_MAC_LINE(2, 3) FTS_MAC_LINE(4, 5) : "+v"(acc), "+v"(ovf) : "v"(x0), "v"(y0), "v"(x1), "v"(y1) : "vcc");
}
FTS_DEV void mac96_4v(uint64_t& acc, uint32_t& ovf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t x2,
                      uint32_t y2, uint32_t x3, uint32_t y3) {
  asm(FTS_MAC_LINE(2, 3) FTS_MAC_LINE(4, 5) FTS_MAC_LINE(6, 7) FTS_MAC_LINE(8, 9)
      : "+v"(acc), "+v"(ovf)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2), "v"(x3), "v"(y3)
      : "vcc");
}
FTS_DEV void mac96_2s(uint64_t& acc, uint32_t& ovf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
  asm(FTS_MAC_LINE(2, 3) FTS_MAC_LINE(4, 5) : "+v"(acc), "+v"(ovf) : "v"(x0), "s"(y0), "v"(x1), "s"(y1) : "vcc");
}
FTS_DEV void mac96_4s(uint64_t& acc, uint32_t& ovf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t x2,
                      uint32_t y2, uint32_t x3, uint32_t y3) {
  asm(FTS_MAC_LINE(2, 3) FTS_MAC_LINE(4, 5) FTS_MAC_LINE(6, 7) FTS_MAC_LINE(8, 9)
      : "+v"(acc), "+v"(ovf)
      : "v"(x0), "s"(y0), "v"(x1), "s"(y1), "v"(x2), "s"(y2), "v"(x3), "s"(y3)
      : "vcc");
}
// sum_{q < cnt} x[q] * y[q] into (acc, ovf); cnt is a compile-time constant after unrolling
template <bool UNIFORM_Y>
FTS_DEV void mac_run(uint64_t& acc, uint32_t& ovf, const uint32_t* x, const uint32_t* y, int cnt) {
  int q = 0;
#pragma unroll
  for (; q + 4 <= cnt; q += 4) {
    if (UNIFORM_Y) mac96_4s(acc, ovf, x[q], y[q], x[q + 1], y[q + 1], x[q + 2], y[q + 2], x[q + 3], y[q + 3]);
    else mac96_4v(acc, ovf, x[q], y[q], x[q + 1], y[q + 1], x[q + 2], y[q + 2], x[q + 3], y[q + 3]);
  }
  if (q + 2 <= cnt) {
    if (UNIFORM_Y) mac96_2s(acc, ovf, x[q], y[q], x[q + 1], y[q + 1]);
    else mac96_2v(acc, ovf, x[q], y[q], x[q + 1], y[q + 1]);
    q += 2;
  }
  if (q < cnt) {
    if (UNIFORM_Y) mac96s(acc, ovf, x[q], y[q]);
    else mac96(acc, ovf, x[q], y[q]);
  }
}

// Montgomery product, finely-integrated product scanning (FIPS): column k of
// a*b and of m*M are summed in a 96-bit accumulator, m[k] is produced as soon
// as column k < 8 is complete.  Same 136 multiplies as CIOS, but the
// accumulator stays in one register triple.
template <class P>
FTS_DEV Field<P> f_mul_fips(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) mac96(acc, ovf, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < (k < 8 ? k : 8); i++) mac96s(acc, ovf, m[i], P::M[k - i]);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// FIPS with two independent 96-bit accumulators per column (a*b products in
// one, m*M products in the other): halves the dependent mad chain, which is
// what bounds the latency-critical per-proof kernels.
FTS_DEV void add96(uint64_t& acc, uint32_t& ovf, uint64_t acc2, uint32_t ovf2) {
  uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32), c;
  lo = addc(lo, (uint32_t)acc2, 0, c);
  hi = addc(hi, (uint32_t)(acc2 >> 32), c, c);
  ovf = ovf + ovf2 + c;
  acc = ((uint64_t)hi << 32) | lo;
}

template <class P>
FTS_DEV Field<P> f_mul_fips2(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0, acc2;
  uint32_t ovf = 0, ovf2;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    acc2 = 0;
    ovf2 = 0;
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) mac96(acc, ovf, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < (k < 8 ? k : 8); i++) mac96s(acc2, ovf2, m[i], P::M[k - i]);
    add96(acc, ovf, acc2, ovf2);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// The carry of v_mad_u64_u32 in an SGPR pair instead of VCC, and the mad and
// its carry-add as separate asm statements: the compiler can interleave
// independent accumulator chains (with VCC every mad/addc pair of every chain
// serialises on the one flag register).
FTS_DEV void mad_sc(uint64_t& acc, uint64_t& c, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(x), "v"(y));
}
FTS_DEV void mad_scs(uint64_t& acc, uint64_t& c, uint32_t x, uint32_t y_uniform) {
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(x), "s"(y_uniform));
}
FTS_DEV void addc_sc(uint32_t& ovf, uint64_t c) {
  uint64_t d;
  asm("v_addc_co_u32 %0, %1, 0, %0, %2" : "+v"(ovf), "=s"(d) : "s"(c));
}

// Experimental variants kept for lib/int_peak only (measured on MI355X,
// profiles/r01_int_peak.log): a single wave already fills its SIMD's
// quarter-rate MAD issue, so extra ILP does not shorten a product
// (fips 1,840 cycles; sc 2,180; x2 2,050).
// two independent 96-bit accumulations in one asm block: both mads issue
// before either carry-add, carries in two distinct SGPR pairs
FTS_DEV void mac96x2(uint64_t& a0, uint32_t& o0, uint32_t x0, uint32_t y0, uint64_t& a1, uint32_t& o1, uint32_t x1,
                     uint32_t y1_uniform) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
      "v_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
      "v_addc_co_u32 %1, %4, 0, %1, %4\n\t"
      "v_addc_co_u32 %3, %5, 0, %3, %5"
      : "+v"(a0), "+v"(o0), "+v"(a1), "+v"(o1), "=&s"(c0), "=&s"(c1)
      : "v"(x0), "v"(y0), "v"(x1), "s"(y1_uniform));
}

// FIPS with the a*b and m*M products of each column in two accumulators,
// issued pairwise (mac96x2): half the dependent-chain length of f_mul_fips.
template <class P>
FTS_DEV Field<P> f_mul_x2(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t acc2 = 0;
    uint32_t ovf2 = 0;
    const int lo = k > 7 ? k - 7 : 0, hi = k < 7 ? k : 7;  // a_i b_{k-i}, i in [lo, hi]
    const int mhi = k < 8 ? k : 8;                          // m_j M_{k-j}, j in [lo, mhi)
    const int na = hi - lo + 1, nm = mhi - lo;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const bool ha = q < na, hm = q < nm;
      if (ha && hm) {
        mac96x2(acc, ovf, a.v[lo + q], b.v[k - lo - q], acc2, ovf2, m[lo + q], P::M[k - lo - q]);
      } else if (ha) {
        mac96(acc, ovf, a.v[lo + q], b.v[k - lo - q]);
      } else if (hm) {
        mac96s(acc2, ovf2, m[lo + q], P::M[k - lo - q]);
      }
    }
    add96(acc, ovf, acc2, ovf2);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// FIPS with two independent 96-bit accumulators per column (a*b and m*M),
// SGPR carries: the two chains overlap in the pipeline.
template <class P>
FTS_DEV Field<P> f_mul_sc2(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t acc2 = 0;
    uint32_t ovf2 = 0;
    const int lo = k > 7 ? k - 7 : 0, hi = k < 7 ? k : 7;
    const int mhi = k < 8 ? k : 8;
    // interleave the two chains product by product
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int i = lo + q, j = lo + q;
      if (i <= hi) {
        uint64_t c;
        mad_sc(acc, c, a.v[i], b.v[k - i]);
        addc_sc(ovf, c);
      }
      if (j < mhi) {
        uint64_t c;
        mad_scs(acc2, c, m[j], P::M[k - j]);
        addc_sc(ovf2, c);
      }
    }
    add96(acc, ovf, acc2, ovf2);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      uint64_t c;
      mad_scs(acc, c, m[k], P::M[0]);
      addc_sc(ovf, c);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// FIPS, single accumulator, SGPR carries (same dependency chain as
// f_mul_fips, but the mad/addc pairs are no longer fused in one asm block)
template <class P>
FTS_DEV Field<P> f_mul_sc(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) {
      uint64_t c;
      mad_sc(acc, c, a.v[i], b.v[k - i]);
      addc_sc(ovf, c);
    }
#pragma unroll
    for (int i = (k > 7 ? k - 7 : 0); i < (k < 8 ? k : 8); i++) {
      uint64_t c;
      mad_scs(acc, c, m[i], P::M[k - i]);
      addc_sc(ovf, c);
    }
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      uint64_t c;
      mad_scs(acc, c, m[k], P::M[0]);
      addc_sc(ovf, c);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// FIPS product with the column MACs grouped (mac_run): same 136 MADs as
// f_mul_fips, ~1/3 of the inline-asm boundary pads.
template <class P>
FTS_DEV Field<P> f_mul_g(const Field<P>& a, const Field<P>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    const int lo = k > 7 ? k - 7 : 0, hi = k < 7 ? k : 7;
    uint32_t xs[8], ys[8];
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      xs[i - lo] = a.v[i];
      ys[i - lo] = b.v[k - i];
    }
    mac_run<false>(acc, ovf, xs, ys, hi - lo + 1);
    const int mhi = k < 8 ? k : 8;
    uint32_t ms[8], cs[8];
#pragma unroll
    for (int i = lo; i < mhi; i++) {
      ms[i - lo] = m[i];
      cs[i - lo] = P::M[k - i];
    }
    mac_run<true>(acc, ovf, ms, cs, mhi - lo);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// Montgomery square with grouped MACs: 36 products + 64 reduction MADs.
template <class P>
FTS_DEV Field<P> f_sqr_g(const Field<P>& a) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t x = 0;
    uint32_t xo = 0;
    const int lo = k > 7 ? k - 7 : 0;
    uint32_t xs[4], ys[4];
    int nc = 0;
#pragma unroll
    for (int i = lo; 2 * i < k; i++) {
      xs[nc] = a.v[i];
      ys[nc] = a.v[k - i];
      nc++;
    }
    mac_run<false>(x, xo, xs, ys, nc);
    xo = (xo << 1) | (uint32_t)(x >> 63);
    x <<= 1;
    if ((k & 1) == 0) mac96(x, xo, a.v[k / 2], a.v[k / 2]);
    add96(acc, ovf, x, xo);
    const int mhi = k < 8 ? k : 8;
    uint32_t ms[8], cs[8];
#pragma unroll
    for (int i = lo; i < mhi; i++) {
      ms[i - lo] = m[i];
      cs[i - lo] = P::M[k - i];
    }
    mac_run<true>(acc, ovf, ms, cs, mhi - lo);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

template <class P>
FTS_DEV Field<P> f_sqr(const Field<P>& a) {
  return f_mul(a, a);
}

// Montgomery square, FIPS: column k of a^2 = 2 * sum_{i<j, i+j=k} a_i a_j
// (+ a_{k/2}^2 for even k).  The cross products go to their own 96-bit
// accumulator, doubled by a 1-bit shift before the square term and the
// running column value are added: 36 products + 64 for the reduction
// = 100 MADs instead of 136.
template <class P>
FTS_DEV Field<P> f_sqr_fips(const Field<P>& a) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t x = 0;
    uint32_t xo = 0;
    const int lo = k > 7 ? k - 7 : 0;
#pragma unroll
    for (int i = lo; 2 * i < k; i++) mac96(x, xo, a.v[i], a.v[k - i]);
    // x <<= 1 (96-bit)
    xo = (xo << 1) | (uint32_t)(x >> 63);
    x <<= 1;
    if ((k & 1) == 0) mac96(x, xo, a.v[k / 2], a.v[k / 2]);
    add96(acc, ovf, x, xo);
#pragma unroll
    for (int i = lo; i < (k < 8 ? k : 8); i++) mac96s(acc, ovf, m[i], P::M[k - i]);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac96s(acc, ovf, m[k], P::M[0]);
    } else {
      t[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
    ovf = 0;
  }
  t[7] = (uint32_t)acc;
  Field<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  f_reduce_once(r);
  return r;
}

// Montgomery form <-> canonical integer (both as 8 little-endian limbs)
template <class P>
FTS_DEV Field<P> f_to_mont(const Field<P>& a) {
  Field<P> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = P::R2[i];
  return f_mul(a, r2);
}
template <class P>
FTS_DEV Field<P> f_from_mont(const Field<P>& a) {
  Field<P> one = f_zero<P>();
  one.v[0] = 1;
  return f_mul(a, one);
}

// a^e for a 256-bit exponent given as 8 LE limbs (square-and-multiply, MSB first)
template <class P>
FTS_DEV Field<P> f_pow(const Field<P>& a, const uint32_t e[8]) {
  Field<P> r = f_one<P>();
  bool started = false;
  for (int i = 7; i >= 0; i--) {
    for (int b = 31; b >= 0; b--) {
      if (started) r = f_sqr(r);
      if ((e[i] >> b) & 1u) {
        r = started ? f_mul(r, a) : a;
        started = true;
      }
    }
  }
  return r;
}

// inverse via Fermat (a^(M-2)); inv(0) = 0
template <class P>
FTS_DEV Field<P> f_inv(const Field<P>& a) {
  uint32_t e[8];
  uint32_t bw = 0;
  e[0] = subb(P::M[0], 2u, 0, bw);
#pragma unroll
  for (int i = 1; i < 8; i++) e[i] = subb(P::M[i], 0u, bw, bw);
  return f_pow(a, e);
}

// Inverse by the binary extended Euclidean algorithm (variable time: every
// value inverted on the verification path is public).  Invariants
// x1 * A == u, x2 * A == v (mod M) for the Montgomery representative A = aR;
// each step halves u or v, so at most ~2*254 steps.  The result A^-1 is
// mapped back to Montgomery form with one product by R^3:
// mont(A^-1, R^3) = a^-1 R.  inv(0) = 0 (as Fermat gives).
// Latency: ~500 steps of 8-limb add/shift (full-rate VALU) instead of the
// ~380 dependent 136-MAD products of a^(M-2).
template <class P>
FTS_DEV void limbs_half_mod(uint32_t x[8]) {  // x <- x/2 mod M  (x < M)
  const uint32_t mask = 0u - (x[0] & 1u);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = addc(x[i], P::M[i] & mask, c, c);
  // x + M < 2^255: no carry out
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
  x[7] >>= 1;
}
template <class P>
FTS_DEV void limbs_sub_mod(uint32_t x[8], const uint32_t y[8]) {  // x <- x - y mod M
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = subb(x[i], y[i], bw, bw);
  const uint32_t mask = 0u - bw;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = addc(x[i], P::M[i] & mask, c, c);
}
FTS_DEV bool limbs_is_one(const uint32_t u[8]) {
  uint32_t o = u[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 8; i++) o |= u[i];
  return o == 0;
}
template <class P>
FTS_DEV Field<P> f_inv_bin(const Field<P>& a) {
  if (f_is_zero(a)) return a;
  uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a.v[i];
    v[i] = P::M[i];
    x1[i] = 0;
    x2[i] = 0;
  }
  x1[0] = 1;
  while (!limbs_is_one(u) && !limbs_is_one(v)) {
    if ((u[0] & 1u) == 0) {
#pragma unroll
      for (int i = 0; i < 7; i++) u[i] = (u[i] >> 1) | (u[i + 1] << 31);
      u[7] >>= 1;
      limbs_half_mod<P>(x1);
    } else if ((v[0] & 1u) == 0) {
#pragma unroll
      for (int i = 0; i < 7; i++) v[i] = (v[i] >> 1) | (v[i + 1] << 31);
      v[7] >>= 1;
      limbs_half_mod<P>(x2);
    } else {
      uint32_t t[8], bw = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) t[i] = subb(u[i], v[i], bw, bw);
      if (!bw) {  // u >= v: u <- (u - v)/2, x1 <- (x1 - x2)/2
#pragma unroll
        for (int i = 0; i < 7; i++) u[i] = (t[i] >> 1) | (t[i + 1] << 31);
        u[7] = t[7] >> 1;
        limbs_sub_mod<P>(x1, x2);
        limbs_half_mod<P>(x1);
      } else {  // v <- (v - u)/2, x2 <- (x2 - x1)/2
        uint32_t b2 = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) t[i] = subb(v[i], u[i], b2, b2);
#pragma unroll
        for (int i = 0; i < 7; i++) v[i] = (t[i] >> 1) | (t[i + 1] << 31);
        v[7] = t[7] >> 1;
        limbs_sub_mod<P>(x2, x1);
        limbs_half_mod<P>(x2);
      }
    }
  }
  Field<P> r, r3;
  const bool one_u = limbs_is_one(u);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i] = one_u ? x1[i] : x2[i];
    r3.v[i] = P::R3[i];
  }
  return f_mul(r, r3);
}


// Constant-time inverse by the optimised binary GCD (T. Pornin, "Optimized
// Binary GCD for Modular Inversion", 2020, Alg. 2), branch-free so the 64
// lanes of a wave never diverge (f_inv_bin's three-way branch serialises
// them).  Each of 17 outer steps runs 30 divsteps on 64-bit approximations
// of a, b (low 31 bits exact + top 33 bits), collecting the transition
// matrix (f0 g0; f1 g1), |f|,|g| <= 2^30; then applies it exactly to the
// 256-bit a, b and, divided by 2^32 (one Montgomery word step), to the
// Bezout coefficients u, v.  Invariant: b == v * y * 4^i (mod M) after i
// steps, ending at a = 0, b = 1, so y^-1 = v * 2^34.  With y = A = aR the
// Montgomery product by GCDC = 2^34 R^3 yields a^-1 R.  inv(0) = 0.
// 2 * 254 - 1 = 507 <= 17 * 30 divsteps suffice (Pornin, Thm. 1).
FTS_DEV uint32_t gcd_sel(bool c, uint32_t x, uint32_t y) { return c ? x : y; }

// r (9 limbs, two's complement) = a * f + b * g   (a, b < 2^256 unsigned; f, g signed, |.| <= 2^30)
FTS_DEV void gcd_lincomb(const uint32_t a[8], int32_t f, const uint32_t b[8], int32_t g, uint32_t r[9]) {
  const uint32_t fa = (uint32_t)(f < 0 ? -f : f), ga = (uint32_t)(g < 0 ? -g : g);
  uint32_t pa[9], pb[9];
  uint64_t ca = 0, cb = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    ca = (uint64_t)a[i] * fa + (ca >> 32);
    cb = (uint64_t)b[i] * ga + (cb >> 32);
    pa[i] = (uint32_t)ca;
    pb[i] = (uint32_t)cb;
  }
  pa[8] = (uint32_t)(ca >> 32);
  pb[8] = (uint32_t)(cb >> 32);
  // conditional negation: x -> (x ^ m) - m with m = all-ones if negative
  const uint32_t ma = f < 0 ? 0xffffffffu : 0u, mb = g < 0 ? 0xffffffffu : 0u;
  uint32_t c1 = ma & 1u, c2 = mb & 1u, c3 = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t x = addc(pa[i] ^ ma, 0u, c1, c1);
    const uint32_t y = addc(pb[i] ^ mb, 0u, c2, c2);
    r[i] = addc(x, y, c3, c3);
  }
}

template <class P>
FTS_DEV Field<P> f_inv_gcd(const Field<P>& y) {
  if (f_is_zero(y)) return y;
  uint32_t a[8], b[8], u[8], v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = y.v[i];
    b[i] = P::M[i];
    u[i] = 0;
    v[i] = 0;
  }
  u[0] = 1;
  for (int it = 0; it < 17; it++) {
    // n = max(len a, len b, 64); approximations: low 31 bits | top 33 bits << 31
    uint32_t top = 0;
    int ti = 1;
#pragma unroll
    for (int i = 1; i < 8; i++) {
      const uint32_t o = a[i] | b[i];
      ti = o ? i : ti;
      top = o ? o : top;
    }
    const int n = max(32 * ti + 32 - __clz(top | 1u), 64);
    const int sh = n - 33, wi = sh >> 5, bo = sh & 31;
    uint32_t al = 0, ah = 0, bl = 0, bh = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      al = gcd_sel(i == wi, a[i], al);
      ah = gcd_sel(i == wi + 1, a[i], ah);
      bl = gcd_sel(i == wi, b[i], bl);
      bh = gcd_sel(i == wi + 1, b[i], bh);
    }
    const uint64_t atop = ((((uint64_t)ah << 32) | al) >> bo) & 0x1ffffffffull;
    const uint64_t btop = ((((uint64_t)bh << 32) | bl) >> bo) & 0x1ffffffffull;
    uint64_t xa = (atop << 31) | (a[0] & 0x7fffffffu);
    uint64_t xb = (btop << 31) | (b[0] & 0x7fffffffu);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
    for (int j = 0; j < 30; j++) {
      const bool odd = (xa & 1u) != 0;
      const bool sw = odd && xa < xb;
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      xb = tb;
      f1 = tf1;
      g1 = tg1;
      xa = odd ? ta - tb : ta;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      xa >>= 1;
      f1 *= 2;
      g1 *= 2;
    }
    // (a, b) <- ((a f0 + b g0), (a f1 + b g1)) / 2^30, made non-negative
    uint32_t na[9], nb[9];
    gcd_lincomb(a, f0, b, g0, na);
    gcd_lincomb(a, f1, b, g1, nb);
    const bool nega = (int32_t)na[8] < 0, negb = (int32_t)nb[8] < 0;
    {
      const uint32_t m1 = nega ? 0xffffffffu : 0u, m2 = negb ? 0xffffffffu : 0u;
      uint32_t c1 = m1 & 1u, c2 = m2 & 1u;
#pragma unroll
      for (int i = 0; i < 9; i++) {
        na[i] = addc(na[i] ^ m1, 0u, c1, c1);
        nb[i] = addc(nb[i] ^ m2, 0u, c2, c2);
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        a[i] = (na[i] >> 30) | (na[i + 1] << 2);
        b[i] = (nb[i] >> 30) | (nb[i + 1] << 2);
      }
    }
    if (nega) {
      f0 = -f0;
      g0 = -g0;
    }
    if (negb) {
      f1 = -f1;
      g1 = -g1;
    }
    // (u, v) <- ((u f0 + v g0), (u f1 + v g1)) / 2^32 mod M
    uint32_t wu[9], wv[9];
    gcd_lincomb(u, f0, v, g0, wu);
    gcd_lincomb(u, f1, v, g1, wv);
    uint32_t* ws[2] = {wu, wv};
    uint32_t* outs[2] = {u, v};
#pragma unroll
    for (int q = 0; q < 2; q++) {
      uint32_t* w = ws[q];
      // w + m * M, m = w0 * (-M^-1) mod 2^32: low word cancels; (w + m M) / 2^32 in (-M/2, 3M/2)
      const uint32_t mq = w[0] * P::INV;
      uint64_t c = 0;
      uint32_t t[10];
      const uint32_t sgn = (int32_t)w[8] < 0 ? 0xffffffffu : 0u;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        c = (uint64_t)mq * P::M[i] + w[i] + (c >> 32);
        t[i] = (uint32_t)c;
      }
      uint32_t cc = 0;
      t[8] = addc(w[8], (uint32_t)(c >> 32), 0u, cc);
      t[9] = sgn + cc;  // sign extension + carry
      // r = t >> 32 (9 limbs: t[1..9]); add M if negative, subtract M if >= M
      const bool neg = (int32_t)t[9] < 0;
      uint32_t r[8], bw = 0, ce = 0;
      const uint32_t madd = neg ? 0xffffffffu : 0u;
#pragma unroll
      for (int i = 0; i < 8; i++) r[i] = addc(t[i + 1], P::M[i] & madd, ce, ce);
      uint32_t s2[8];
#pragma unroll
      for (int i = 0; i < 8; i++) s2[i] = subb(r[i], P::M[i], bw, bw);
      // r >= M iff no borrow (when r was non-negative; after +M a negative r is < M)
      const bool ge = !bw && !neg;
      // top word of the 9-limb value when positive can carry into limb 8 (t[9]) -> treat as >= M
      const bool big = !neg && t[9] != 0;
#pragma unroll
      for (int i = 0; i < 8; i++) outs[q][i] = (ge || big) ? s2[i] : r[i];
    }
  }
  Field<P> r, c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i] = v[i];
    c.v[i] = P::GCDC[i];
  }
  return f_mul(r, c);
}

// canonical (non-Montgomery) limbs < M ?
template <class P>
FTS_DEV bool limbs_lt_mod(const uint32_t a[8]) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)subb(a[i], P::M[i], bw, bw);
  return bw != 0;
}

// big-endian 32 bytes -> LE limbs (no reduction)
FTS_DEV void be32_to_limbs(const uint8_t* b, uint32_t out[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = b + 28 - 4 * i;
    out[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}
FTS_DEV void limbs_to_be32(const uint32_t in[8], uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(in[i] >> 24);
    q[1] = (uint8_t)(in[i] >> 16);
    q[2] = (uint8_t)(in[i] >> 8);
    q[3] = (uint8_t)in[i];
  }
}

}  // namespace fts
