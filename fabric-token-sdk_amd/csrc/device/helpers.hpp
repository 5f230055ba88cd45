// Small device helpers shared by the range-proof and sigma-proof kernels.
#pragma once
#include "g1.hpp"
#include "transcript.hpp"
#include "wave_prio.hpp"

namespace fts {

// Wave priority of the batch-verify pass's kernels (s_setprio).  A SIMD arbitrates
// VALU issue by wave priority, then age (MI355X_MICROARCH.md, "Two waves per SIMD"):
// the short dependent kernels of the batch check's MSM and of the x0 tail start while
// the long issue-bound chain waves (k_rp_com_var, the x0 prefix hash) are resident, so
// at equal priority they are the younger waves and get only the chain's leftover issue
// slots (r05 trace: k_msm_scan1 0.005 ms alone, 0.64 ms beside com_var; the MSM's sort
// 0.5 ms alone, 5.9 ms in the pass).  One static level per kernel group, set once at
// kernel entry from this table (a uniform scalar load; FTS_WAVE_PRIO overrides it per
// context, fts_api.cpp).
static __constant__ int g_wave_prio[PS_N] = FTS_WAVE_PRIO_DEFAULT;
template <int S>
FTS_DEV void wave_prio() {
  const int p = g_wave_prio[S];  // uniform: s_load + s_cbranch around one s_setprio
  if (p == 1)
    __builtin_amdgcn_s_setprio(1);
  else if (p == 2)
    __builtin_amdgcn_s_setprio(2);
  else if (p >= 3)
    __builtin_amdgcn_s_setprio(3);
}
// per translation unit (each holds its own copy of the table)
static inline hipError_t upload_wave_prio(const int* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wave_prio), p, sizeof(int) * PS_N, 0, hipMemcpyHostToDevice);
}

// ------------------------------------------------------------ small helpers
FTS_DEV Fr fr_from_canon(const uint32_t* c) {
  Fr a;
  load_f(c, a);
  return f_to_mont(a);
}
FTS_DEV Scalar fr_canon(const Fr& m) {
  Fr c = f_from_mont(m);
  Scalar s;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = c.v[i];
  return s;
}
// acc + q where q is in registers: spill q to lane scratch, add out-of-line
FTS_DEV G1J add_via(uint32_t* scr, const G1J& acc, const G1J& q) {
  store_g1j(scr, q);
  return nl_add_mem(acc, scr, 0);
}
FTS_DEV Fr fr_pow_small(const Fr& a, uint32_t e) {
  Fr r = f_one<FrP>();
  Fr b = a;
  while (e) {
    if (e & 1u) r = fr_mul(r, b);
    e >>= 1;
    if (e) b = fr_sqr(b);
  }
  return r;
}

// write hex(point) [+ "||"] of a raw BE point at byte offset off (even) of msg
FTS_DEV void put_hex_record(uint8_t* msg, uint32_t off, const uint32_t pw[16], bool sep) {
  uint16_t* d = reinterpret_cast<uint16_t*>(msg + off);
  write_hex_point_words(d, pw);
  if (sep) d[64] = 0x7c7c;
}

// SHA-256 over hex(p_0) || "||" || ... of m raw points, using `slot` as
// message scratch; returns canonical Fr (LE limbs)
FTS_DEV Fr hash_raw_points(uint8_t* slot, const uint8_t* const* pts, int m) {
  for (int i = 0; i < m; i++) {
    uint32_t pw[16];
    load_be_words(pts[i], pw);
    put_hex_record(slot, 130u * i, pw, i + 1 < m);
  }
  uint32_t len = 130u * m - 2u;
  write_sha_padding_u16(slot, len);
  uint32_t st[8];
  sha256_blocks(slot, sha_blocks(len), st);
  return digest_to_fr(st);
}


// decode + validate one raw BE point (NewG1FromBytes, asn1.go:148):
// flag bits 00, canonical coordinates, on the curve; zeros = identity.
FTS_DEV bool decode_point(const uint8_t* raw, G1A& a) {
  uint32_t pw[16];
  load_be_words(raw, pw);
  Fp x, y;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = pw[7 - i];
    y.v[i] = pw[15 - i];
  }
  bool ok = (pw[0] >> 30) == 0 && limbs_lt_mod<FpP>(x.v) && limbs_lt_mod<FpP>(y.v);
  if (ok && f_is_zero(x) && f_is_zero(y)) {
    a.x = x;
    a.y = y;
    return true;
  }
  a.x = f_to_mont(x);
  a.y = f_to_mont(y);
  Fp three = f_zero<FpP>();
  three.v[0] = 3;
  three = f_to_mont(three);
  Fp rhs = f_add(fp_mul(fp_sqr(a.x), a.x), three);
  ok = ok && f_eq(fp_sqr(a.y), rhs);
  if (!ok) {
    a.x = f_zero<FpP>();
    a.y = f_zero<FpP>();
  }
  return ok;
}

// affine Montgomery point -> 64 canonical BE bytes at dst (16-byte aligned)
FTS_DEV void store_point_be(uint8_t* dst, const G1A& a) {
  uint32_t pw[16];
  g1_mont_to_be_words(a.x, a.y, pw);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int q = 0; q < 4; q++)
    d[q] = make_uint4(__builtin_bswap32(pw[4 * q]), __builtin_bswap32(pw[4 * q + 1]), __builtin_bswap32(pw[4 * q + 2]),
                      __builtin_bswap32(pw[4 * q + 3]));
}

// batch normalisation of m Jacobian points (jac: [m][24]) into affine (aff: [m][16]);
// aff doubles as prefix-product storage
FTS_DEV void batch_to_affine(const uint32_t* jac, uint32_t* aff, int m) {
  Fp acc = f_one<FpP>();
  for (int i = 0; i < m; i++) {
    store_fp(aff + i * 16, acc);
    Fp z;
    load_fp(jac + i * 24 + 16, z);
    if (!f_is_zero(z)) acc = fp_mul(acc, z);
  }
  Fp inv = nl_fp_inv(acc);
  for (int i = m - 1; i >= 0; i--) {
    G1J p = load_g1j(jac + i * 24);
    G1A a;
    if (f_is_zero(p.z)) {
      a.x = f_zero<FpP>();
      a.y = f_zero<FpP>();
    } else {
      Fp pr;
      load_fp(aff + i * 16, pr);
      Fp zi = fp_mul(inv, pr);
      inv = fp_mul(inv, p.z);
      Fp zi2 = fp_sqr(zi);
      a.x = fp_mul(p.x, zi2);
      a.y = fp_mul(fp_mul(p.y, zi2), zi);
    }
    store_g1a(aff + i * 16, a);
  }
}

}  // namespace fts
