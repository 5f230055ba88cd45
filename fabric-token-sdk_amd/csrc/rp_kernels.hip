// Range-proof (Bulletproof + IPA) batch verification kernels for gfx950.
//
// One launch sequence verifies a whole batch of B proofs of bit length n
// (k = log2 n rounds).  Work is laid out per (proof, item) so a batch of a
// few thousand proofs fills the 256 CUs:
//
//   k_rp_decode        (proof, point)   NewG1FromBytes checks + Montgomery form
//   k_rp_hash_small    (proof, msg)     x, y, x_j transcripts (SHA-256 over hex)  bulletproof.go:266-281, ipa.go:230
//   k_rp_chal_fr       proof            z, polEval, batch inversion of y, x_j       bulletproof.go:282-311, ipa.go:236-244
//   k_rp_hprime        (proof, i)       H'_i = y^-i * H_i  fixed-base    bulletproof.go:483-489
//   k_rp_hp_normalize  proof            batch affine normalisation (Montgomery trick)
//   k_rp_com_terms     (proof, term)    com = x*D + C + z*K + sum (z^2 2^i y^-i) H_i - delta*P
//   k_rp_com_sum       proof (wave)     LDS tree + normalisation          bulletproof.go:477-492
//   k_rp_x0_build      (proof, record)  DER(hex(H'..., G..., Q, com) "||" Zb(ip))   ipa.go:200-212
//   k_rp_x0_hash       proof            x0 = HashToZr(...)                ipa.go:213
//   k_rp_terms_fixed   (proof, term)    fixed-base terms of E1 / E2
//   k_rp_terms_var     (proof, term)    variable-base terms of E1 / E2
//   k_rp_check         proof            E1 == O ("invalid range proof"), E2 == O ("invalid IPA")
//
// E1: (ip - polEval) G + tau H - x T1 - x^2 T2 - z^2 V            (bulletproof.go:314-324)
// E2: sum a s_i G_i + sum b s_i^-1 y^-i H_i + (ab - ip) x0 Q - com
//     - sum x_j^2 L_j - sum x_j^-2 R_j                              (ipa.go:214-259 unrolled:
//     G_fin = sum s_i G_i, H'_fin = sum s_i^-1 H'_i, s_i = prod_j x_j^{+-1} by bit k-1-j of i)
#include "device/g1.hpp"
#include "device/rp_kernels.hpp"
#include "device/transcript.hpp"
#include "device/helpers.hpp"
#include "device/msm.hpp"
#include "common/chacha20.hpp"
#include "../../include/fts_gpu.h"

namespace fts {

// ---------------------------------------------------------- context tables
// thread per (base, window w): entries d * 2^(8w) * B for d = 1..128, affine.
// scratch: [nb*32][128][32] words (Jacobian point + prefix product)
__global__ void __launch_bounds__(64) k_build_tables(const uint32_t* __restrict__ bases, int nb,
                                                     uint32_t* __restrict__ tables, uint32_t* __restrict__ scratch) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nb * FB_WINDOWS) return;
  int b = gid / FB_WINDOWS, w = gid % FB_WINDOWS;
  G1A B = load_g1a(bases + b * 16);
  G1J bw = g1j_from_affine(B);
  for (int i = 0; i < 8 * w; i++) bw = nl_dbl(bw);
  uint32_t* J = scratch + (size_t)gid * FB_ENTRIES * 32;
  G1J acc = bw;
  Fp pre = f_one<FpP>();
  for (int d = 1; d <= FB_ENTRIES; d++) {
    if (d > 1) acc = nl_add_mem(acc, J, 0);  // J[0] holds bw
    store_g1j(J + (d - 1) * 32, acc);
    store_fp(J + (d - 1) * 32 + 24, pre);
    if (!f_is_zero(acc.z)) pre = fp_mul(pre, acc.z);
  }
  Fp inv = nl_fp_inv(pre);
  uint32_t* T = tables + (size_t)b * FB_WORDS_PER_BASE + (size_t)w * FB_ENTRIES * 16;
  for (int d = FB_ENTRIES; d >= 1; d--) {
    G1J p = load_g1j(J + (d - 1) * 32);
    G1A a;
    if (f_is_zero(p.z)) {
      a.x = f_zero<FpP>();
      a.y = f_zero<FpP>();
    } else {
      Fp pr;
      load_fp(J + (d - 1) * 32 + 24, pr);
      Fp zi = fp_mul(inv, pr);
      inv = fp_mul(inv, p.z);
      Fp zi2 = fp_sqr(zi);
      a.x = fp_mul(p.x, zi2);
      a.y = fp_mul(fp_mul(p.y, zi2), zi);
    }
    store_g1a(T + (d - 1) * 16, a);
  }
}

// ------------------------------------------------------------------ decode
// NewG1FromBytes (asn1.go:148 -> gnark SetBytes): 64 bytes, flag bits 00,
// canonical coordinates, on the curve; 64 zero bytes = identity.
__global__ void __launch_bounds__(256) k_rp_decode(int B, int npts, const uint8_t* __restrict__ raw,
                                                   uint32_t* __restrict__ pts, int32_t* __restrict__ status) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * npts) return;
  G1A a;
  if (!decode_point(raw + (size_t)gid * 64, a)) status[gid / npts] = FTS_E_MALFORMED;
  store_g1a(pts + (size_t)gid * 16, a);
}

// -------------------------------------------------------------- challenges
// thread per (proof, message): message 0 = Arr(T1, T2) -> x; 1 = Arr(C, D, V)
// -> y; 2 + j = Arr(L_j, R_j) -> x_j  (bulletproof.go:266-281, ipa.go:230-235).
// Digests (canonical Fr) land in the challenge block, converted later.
__global__ void __launch_bounds__(64) k_rp_hash_small(int B, int n, int k, const uint8_t* __restrict__ raw,
                                                      const int32_t* __restrict__ status, uint32_t* __restrict__ ch,
                                                      uint8_t* __restrict__ small_msgs) {
  const int nm = 2 + k;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nm) return;
  const int b = gid / nm, m = gid % nm;
  if (status[b] != 0) return;
  const uint8_t* P = raw + (size_t)b * rp_npts(k) * 64;
  uint8_t* slot = small_msgs + (size_t)gid * SMALL_SLOT;
  uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  Fr h;
  int dst;
  if (m == 0) {
    const uint8_t* px[2] = {P + RP_PT_T1 * 64, P + RP_PT_T2 * 64};
    h = hash_raw_points(slot, px, 2);
    dst = CH_X;
  } else if (m == 1) {
    const uint8_t* py[3] = {P + RP_PT_C * 64, P + RP_PT_D * 64, P + RP_PT_V * 64};
    h = hash_raw_points(slot, py, 3);
    dst = CH_Y;
  } else {
    const int j = m - 2;
    const uint8_t* pl[2] = {P + (RP_PT_L + j) * 64, P + (RP_PT_L + k + j) * 64};
    h = hash_raw_points(slot, pl, 2);
    dst = CH_XJ + j;
  }
  store_f(C + dst * 8, h);  // canonical for now
}

// thread per proof: z = Hz(Zb(y)), Montgomery forms, polEval, and one batch
// inversion (Montgomery trick) for y and the k round challenges
__global__ void __launch_bounds__(64) k_rp_chal_fr(int B, int n, int k, const int32_t* __restrict__ status,
                                                   uint32_t* __restrict__ ch, uint32_t* __restrict__ tmp) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  uint32_t* T = tmp + (size_t)b * (k + 1) * 8;  // prefix products
  Fr yc, xc;
  load_f(C + CH_Y * 8, yc);
  load_f(C + CH_X * 8, xc);
  uint32_t w[16], st[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = yc.v[7 - i];
  w[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; i++) w[i] = 0;
  w[15] = 256;
  sha256_init(st);
  sha256_compress(st, w);
  Fr z = f_to_mont(digest_to_fr(st));
  Fr y = f_to_mont(yc), x = f_to_mont(xc);
  Fr x2 = fr_sqr(x), z2 = fr_sqr(z), z3 = fr_mul(z2, z);
  Fr yp = f_one<FrP>(), ipy = f_zero<FrP>(), p2 = f_one<FrP>(), ip2 = f_zero<FrP>();
  for (int i = 0; i < n; i++) {
    if (i) {
      yp = fr_mul(yp, y);
      p2 = f_dbl(p2);
    }
    ipy = f_add(ipy, yp);
    ip2 = f_add(ip2, p2);
  }
  Fr pol = f_sub(fr_mul(f_sub(z, z2), ipy), fr_mul(z3, ip2));  // bulletproof.go:307-311
  store_f(C + CH_X * 8, x);
  store_f(C + CH_X2 * 8, x2);
  store_f(C + CH_Y * 8, y);
  store_f(C + CH_Z * 8, z);
  store_f(C + CH_Z2 * 8, z2);
  store_f(C + CH_POL * 8, pol);
  // batch inversion of v_0 = y, v_{1+j} = x_j (zeros invert to zero, as Fermat does)
  Fr acc = f_one<FrP>();
  for (int q = 0; q <= k; q++) {
    Fr v;
    if (q == 0) v = y;
    else {
      load_f(C + (CH_XJ + q - 1) * 8, v);
      v = f_to_mont(v);
      store_f(C + (CH_XJ + q - 1) * 8, v);
    }
    store_f(T + q * 8, acc);
    if (!f_is_zero(v)) acc = fr_mul(acc, v);
  }
  Fr inv = nl_fr_inv(acc);
  for (int q = k; q >= 0; q--) {
    Fr v, pre;
    if (q == 0) v = y;
    else load_f(C + (CH_XJ + q - 1) * 8, v);
    load_f(T + q * 8, pre);
    Fr vi = f_zero<FrP>();
    if (!f_is_zero(v)) {
      vi = fr_mul(inv, pre);
      inv = fr_mul(inv, v);
    }
    store_f(C + (q == 0 ? CH_YINV : CH_XJ + k + q - 1) * 8, vi);
  }
}

// --------------------------------------------------------------------- H'
__global__ void __launch_bounds__(64) k_rp_hprime(int B, int n, int k, const int32_t* __restrict__ status,
                                                  const uint32_t* __restrict__ ch, const uint32_t* __restrict__ tables,
                                                  uint32_t* __restrict__ hpj) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * n) return;
  int b = gid / n, i = gid % n;
  if (status[b] != 0) return;
  Fr yinv;
  load_f(ch + ((size_t)b * rp_nch(k) + CH_YINV) * 8, yinv);
  G1J r = fixed_base_mul(tables + (size_t)(n + i) * FB_WORDS_PER_BASE, fr_canon(fr_pow_small(yinv, (uint32_t)i)));
  store_g1j(hpj + (size_t)gid * 24, r);
}

// batch affine normalisation of the n H'_i of one proof
__global__ void __launch_bounds__(64) k_rp_hp_normalize(int B, int n, const int32_t* __restrict__ status,
                                                        const uint32_t* __restrict__ hpj, uint32_t* __restrict__ hpa,
                                                        uint8_t* __restrict__ hp_be) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  const uint32_t* J = hpj + (size_t)b * n * 24;
  uint32_t* A = hpa + (size_t)b * n * 16;
  Fp acc = f_one<FpP>();
  for (int i = 0; i < n; i++) {
    store_fp(A + i * 16, acc);  // prefix product
    Fp z;
    load_fp(J + i * 24 + 16, z);
    if (!f_is_zero(z)) acc = fp_mul(acc, z);
  }
  Fp inv = nl_fp_inv(acc);
  for (int i = n - 1; i >= 0; i--) {
    G1J p = load_g1j(J + i * 24);
    G1A a;
    if (f_is_zero(p.z)) {
      a.x = f_zero<FpP>();
      a.y = f_zero<FpP>();
    } else {
      Fp pr;
      load_fp(A + i * 16, pr);
      Fp zi = fp_mul(inv, pr);
      inv = fp_mul(inv, p.z);
      Fp zi2 = fp_sqr(zi);
      a.x = fp_mul(p.x, zi2);
      a.y = fp_mul(fp_mul(p.y, zi2), zi);
    }
    store_g1a(A + i * 16, a);
    uint32_t pw[16];
    g1_mont_to_be_words(a.x, a.y, pw);
    uint4* d = reinterpret_cast<uint4*>(hp_be + ((size_t)b * n + i) * 64);
#pragma unroll
    for (int q = 0; q < 4; q++)
      d[q] = make_uint4(__builtin_bswap32(pw[4 * q]), __builtin_bswap32(pw[4 * q + 1]),
                        __builtin_bswap32(pw[4 * q + 2]), __builtin_bswap32(pw[4 * q + 3]));
  }
}

// -------------------------------------------------------------------- com
// com = x*D + C - z sum G_i + sum (z y^i + z^2 2^i) H'_i - delta*P   (bulletproof.go:477-492)
//     = x*D + C + z*K + sum_i (z^2 2^i y^-i) H_i - delta*P,   K = sum H_i - sum G_i
// (same group element; only the affine result is observable).  Terms per
// proof: slots 0..n-1 fixed-base on H_i, n: z*K, n+1: -delta*P, n+2: x*D.
inline __host__ __device__ int com_nterms(int n) { return n + 3; }

__global__ void __launch_bounds__(64) k_rp_com_terms(int B, int n, int k, const int32_t* __restrict__ status,
                                                     const uint32_t* __restrict__ pts, const uint32_t* __restrict__ sc,
                                                     const uint32_t* __restrict__ ch, const uint32_t* __restrict__ tables,
                                                     uint32_t* __restrict__ terms, uint32_t* __restrict__ scratch) {
  const int nt = com_nterms(n);
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nt) return;
  // variable-base slots first in the grid so their long chains start early
  int b, t;
  if (gid < B) {
    b = gid;
    t = n + 2;
  } else {
    b = (gid - B) / (nt - 1);
    t = (gid - B) % (nt - 1);
  }
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  uint32_t* out = terms + ((size_t)b * nt + t) * 24;
  G1J r;
  if (t < n) {
    Fr z2, yinv;
    load_f(C + CH_Z2 * 8, z2);
    load_f(C + CH_YINV * 8, yinv);
    // z^2 2^i y^-i
    Fr s = fr_mul(z2, fr_pow_small(yinv, (uint32_t)t));
    for (int q = 0; q < t; q++) s = f_dbl(s);
    r = fixed_base_mul(tables + (size_t)(n + t) * FB_WORDS_PER_BASE, fr_canon(s));
  } else if (t == n) {
    Fr z;
    load_f(C + CH_Z * 8, z);
    r = fixed_base_mul(tables + (size_t)tb_K(n) * FB_WORDS_PER_BASE, fr_canon(z));
  } else if (t == n + 1) {
    Fr d;
    load_f(sc + ((size_t)b * RP_NSC + RP_SC_DELTA) * 8, d);  // canonical
    Fr nd = f_neg(d);
    Scalar s;
#pragma unroll
    for (int q = 0; q < 8; q++) s.v[q] = nd.v[q];
    r = fixed_base_mul(tables + (size_t)tb_P(n) * FB_WORDS_PER_BASE, s);
  } else {
    Fr x;
    load_f(C + CH_X * 8, x);
    r = var_base_mul(load_g1a(pts + ((size_t)b * rp_npts(k) + RP_PT_D) * 16), fr_canon(x),
                     scratch + (size_t)b * 10 * 24);
  }
  store_g1j(out, r);
}

// one wave per proof: LDS tree over the n + 3 terms, + C, normalise
__global__ void __launch_bounds__(64) k_rp_com_sum(int B, int n, int k, const int32_t* __restrict__ status,
                                                   uint32_t* __restrict__ pts, const uint32_t* __restrict__ terms,
                                                   uint32_t* __restrict__ com, uint8_t* __restrict__ com_be) {
  __shared__ uint32_t sh[64 * 24];
  const int b = blockIdx.x, t = threadIdx.x;
  if (status[b] != 0) return;  // uniform per block
  const int nt = com_nterms(n);
  const uint32_t* T = terms + (size_t)b * nt * 24;
  uint32_t* Pt = pts + (size_t)b * rp_npts(k) * 16;
  G1J acc = g1j_identity();
  for (int q = t; q < nt; q += 64) acc = nl_add_mem(acc, T + q * 24, 0);
  if (t == 0) acc = nl_madd_mem(acc, Pt + RP_PT_C * 16, 0);  // + C
  store_g1j(sh + t * 24, acc);
  __syncthreads();
  for (int half = 32; half >= 1; half >>= 1) {
    if (t < half) acc = nl_add_mem(acc, sh + (t + half) * 24, 0);
    __syncthreads();
    if (t < half) store_g1j(sh + t * 24, acc);
    __syncthreads();
  }
  if (t == 0) {
    G1A ca = nl_to_affine(acc);
    store_g1a(com + (size_t)b * 16, ca);
    // C is consumed: the slot now holds -com for the RLC MSM (scalar rho')
    store_g1a(Pt + RP_PT_C * 16, g1a_neg(ca));
    store_point_be(com_be + (size_t)b * 64, ca);
  }
}

// --------------------------------------------------------- x0 transcript
// thread per (proof, record r in [0, 2n+2]); record 2n+2 writes DER framing
__global__ void __launch_bounds__(256) k_rp_x0_build(int B, int n, const int32_t* __restrict__ status,
                                                     const uint8_t* __restrict__ hp_be, const uint8_t* __restrict__ com_be,
                                                     const uint8_t* __restrict__ x0_const, const uint32_t* __restrict__ sc,
                                                     uint8_t* __restrict__ msgs) {
  const int nrec = 2 * n + 3;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nrec) return;
  int b = gid / nrec, r = gid % nrec;
  if (status[b] != 0) return;
  uint8_t* m = msgs + (size_t)b * x0_slot_bytes(n);
  const uint32_t A = x0_array_len(n);
  if (r < n) {
    uint32_t pw[16];
    load_be_words(hp_be + ((size_t)b * n + r) * 64, pw);
    put_hex_record(m, 8 + 130u * r, pw, true);
  } else if (r < 2 * n + 1) {
    const uint16_t* src = reinterpret_cast<const uint16_t*>(x0_const + 130u * (r - n));
    uint16_t* dst = reinterpret_cast<uint16_t*>(m + 8 + 130u * r);
    for (int q = 0; q < 65; q++) dst[q] = src[q];
  } else if (r == 2 * n + 1) {
    uint32_t pw[16];
    load_be_words(com_be + (size_t)b * 64, pw);
    put_hex_record(m, 8 + 130u * r, pw, false);
  } else {
    uint16_t* m16 = reinterpret_cast<uint16_t*>(m);
    const uint32_t L = A + 42u;  // SEQUENCE content
    m16[0] = 0x8230;
    m16[1] = (uint16_t)((L >> 8) | ((L & 0xffu) << 8));
    m16[2] = 0x8204;
    m16[3] = (uint16_t)((A >> 8) | ((A & 0xffu) << 8));
    uint16_t* t = reinterpret_cast<uint16_t*>(m + 8 + A);
    t[0] = 0x0204;
    t[1] = 0x7c7c;
    t[2] = 0x2004;
    const uint32_t* ip = sc + ((size_t)b * RP_NSC + RP_SC_IP) * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t wd = ip[7 - i];  // BE word i
      t[3 + 2 * i] = (uint16_t)((wd >> 24) | (((wd >> 16) & 0xffu) << 8));
      t[4 + 2 * i] = (uint16_t)(((wd >> 8) & 0xffu) | ((wd & 0xffu) << 8));
    }
    write_sha_padding_u16(m, x0_msg_len(n));
  }
}

__global__ void __launch_bounds__(64) k_rp_x0_hash(int B, int n, int k, const int32_t* __restrict__ status,
                                                   const uint8_t* __restrict__ msgs, uint32_t* __restrict__ ch) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  uint32_t st[8];
  sha256_blocks(msgs + (size_t)b * x0_slot_bytes(n), sha_blocks(x0_msg_len(n)), st);
  store_f(ch + ((size_t)b * rp_nch(k) + CH_X0) * 8, f_to_mont(digest_to_fr(st)));
}

// ------------------------------------------------------------------ terms
// term slots per proof: [0,1] E1 fixed (G, H); [2,3,4] E1 var (T1, T2, V);
// [5 .. 5+2n] E2 fixed (G_i, H_i, Q); [6+2n .. 6+2n+2k-1] E2 var (L_j, R_j)
inline __host__ __device__ int rp_nterms(int n, int k) { return 6 + 2 * n + 2 * k; }

FTS_DEV Fr s_vec(const uint32_t* C, int k, int i) {
  // s_i = prod_j x_j^{+1 if bit (k-1-j) of i else -1}
  Fr s = f_one<FrP>();
  for (int j = 0; j < k; j++) {
    Fr f;
    int bit = (i >> (k - 1 - j)) & 1;
    load_f(C + (CH_XJ + (bit ? 0 : k) + j) * 8, f);
    s = fr_mul(s, f);
  }
  return s;
}

__global__ void __launch_bounds__(64) k_rp_terms_fixed(int B, int n, int k, const int32_t* __restrict__ status,
                                                       const int32_t* __restrict__ ipa_flag,
                                                       const uint32_t* __restrict__ sc, const uint32_t* __restrict__ ch,
                                                       const uint32_t* __restrict__ tables, uint32_t* __restrict__ terms) {
  const int nf = 3 + 2 * n;  // 2 (E1) + 2n + 1 (E2)
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nf) return;
  int b = gid / nf, t = gid % nf;
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const uint32_t* S = sc + (size_t)b * RP_NSC * 8;
  int slot, base;
  Fr s;
  if (t < 2) {
    slot = t;
    if (t == 0) {  // (ip - polEval) * G
      Fr pol;
      load_f(C + CH_POL * 8, pol);
      s = f_sub(fr_from_canon(S + RP_SC_IP * 8), pol);
      base = tb_G(n);
    } else {  // tau * H
      s = fr_from_canon(S + RP_SC_TAU * 8);
      base = tb_H(n);
    }
  } else {
    slot = 5 + (t - 2);
    if (ipa_flag[b] != 0) {
      store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, g1j_identity());
      return;
    }
    int e = t - 2;
    if (e < n) {  // a * s_i * G_i
      s = fr_mul(fr_from_canon(S + RP_SC_A * 8), s_vec(C, k, e));
      base = e;
    } else if (e < 2 * n) {  // b * s_i^-1 * y^-i * H_i   (s_i^-1 = s_{n-1-i})
      int i = e - n;
      Fr yinv;
      load_f(C + CH_YINV * 8, yinv);
      s = fr_mul(fr_mul(fr_from_canon(S + RP_SC_B * 8), s_vec(C, k, n - 1 - i)), fr_pow_small(yinv, (uint32_t)i));
      base = n + i;
    } else {  // (a*b - ip) * x0 * Q
      Fr x0;
      load_f(C + CH_X0 * 8, x0);
      Fr ab = fr_mul(fr_from_canon(S + RP_SC_A * 8), fr_from_canon(S + RP_SC_B * 8));
      s = fr_mul(f_sub(ab, fr_from_canon(S + RP_SC_IP * 8)), x0);
      base = tb_Q(n);
    }
  }
  G1J r = fixed_base_mul(tables + (size_t)base * FB_WORDS_PER_BASE, fr_canon(s));
  store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, r);
}

__global__ void __launch_bounds__(64) k_rp_terms_var(int B, int n, int k, const int32_t* __restrict__ status,
                                                     const int32_t* __restrict__ ipa_flag,
                                                     const uint32_t* __restrict__ pts, const uint32_t* __restrict__ ch,
                                                     uint32_t* __restrict__ terms, uint32_t* __restrict__ scratch) {
  const int nv = 3 + 2 * k;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nv) return;
  int b = gid / nv, t = gid % nv;
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const uint32_t* Pt = pts + (size_t)b * rp_npts(k) * 16;
  int slot, pt;
  Fr s;
  if (t < 3) {
    slot = 2 + t;
    int chi = t == 0 ? CH_X : (t == 1 ? CH_X2 : CH_Z2);
    load_f(C + chi * 8, s);
    pt = t == 0 ? RP_PT_T1 : (t == 1 ? RP_PT_T2 : RP_PT_V);
  } else {
    slot = 6 + 2 * n + (t - 3);
    if (ipa_flag[b] != 0) {
      store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, g1j_identity());
      return;
    }
    int j = t - 3;
    if (j < k) {  // x_j^2 * L_j
      load_f(C + (CH_XJ + j) * 8, s);
      s = fr_sqr(s);
      pt = RP_PT_L + j;
    } else {  // x_j^-2 * R_j
      j -= k;
      load_f(C + (CH_XJ + k + j) * 8, s);
      s = fr_sqr(s);
      pt = RP_PT_L + k + j;
    }
  }
  // all variable terms enter with a minus sign
  G1J r = var_base_mul(load_g1a(Pt + pt * 16), fr_canon(f_neg(s)), scratch + (size_t)gid * 10 * 24);
  store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, r);
}

// ------------------------------------------------------------------ check
__global__ void __launch_bounds__(64) k_rp_check(int B, int n, int k, int32_t* __restrict__ status,
                                                 const int32_t* __restrict__ ipa_flag,
                                                 const uint32_t* __restrict__ terms, const uint32_t* __restrict__ com) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  const uint32_t* T = terms + (size_t)b * rp_nterms(n, k) * 24;
  G1J e1 = load_g1j(T);
  for (int t = 1; t < 5; t++) e1 = nl_add_mem(e1, T + t * 24, 0);
  if (!g1j_is_identity(e1)) {
    status[b] = FTS_E_RP_INVALID;
    return;
  }
  if (ipa_flag[b] != 0) {
    status[b] = ipa_flag[b];
    return;
  }
  G1J e2 = g1j_from_affine(g1a_neg(load_g1a(com + (size_t)b * 16)));
  for (int t = 5; t < rp_nterms(n, k); t++) e2 = nl_add_mem(e2, T + t * 24, 0);
  status[b] = g1j_is_identity(e2) ? FTS_OK : FTS_E_IPA_INVALID;
}

// ------------------------------------------------------------ RLC batch check
// Sum_p rho_p E1_p + rho'_p E2_p == O  (SURVEY Appendix B).  Fixed bases get
// batch-summed scalars (column reduction), variable points go to one MSM.
// coef per proof (Montgomery Fr): [rho(ip - polEval), rho tau, rho'(ab - ip)x0, rho' a, rho' b]
constexpr int RLC_NCOEF = 5;

// full-width weight: 256 random bits reduced mod r (Montgomery form).  Full
// width keeps every MSM window's digits uniform (a 128-bit weight would put
// all proofs' top-digit entries into a few buckets of one window).
FTS_DEV Fr fr_from_u256(const uint32_t w[8]) {
  uint32_t be[8];
#pragma unroll
  for (int i = 0; i < 8; i++) be[i] = w[7 - i];
  return f_to_mont(digest_to_fr(be));
}

__global__ void __launch_bounds__(64) k_rlc_prep(int B, int n, int k, const int32_t* __restrict__ status,
                                                 const int32_t* __restrict__ ipa_flag, const uint32_t* __restrict__ sc,
                                                 const uint32_t* __restrict__ ch, const uint32_t* __restrict__ key,
                                                 uint32_t* __restrict__ msc, uint32_t* __restrict__ coef) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int npts = rp_npts(k);
  uint32_t* M = msc + (size_t)b * npts * 8;
  uint32_t* K = coef + (size_t)b * RLC_NCOEF * 8;
  const bool e1 = status[b] == 0;
  const bool e2 = e1 && ipa_flag[b] == 0;
  Fr zero = f_zero<FrP>();
  for (int q = 0; q < npts; q++) store_f(M + q * 8, zero);
  for (int q = 0; q < RLC_NCOEF; q++) store_f(K + q * 8, zero);
  if (!e1) return;
  uint32_t kk[8], blk[16];
#pragma unroll
  for (int q = 0; q < 8; q++) kk[q] = key[q];
  chacha20_block(kk, (uint32_t)b, blk);
  Fr rho = fr_from_u256(blk), rho2 = fr_from_u256(blk + 8);
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const uint32_t* S = sc + (size_t)b * RP_NSC * 8;
  Fr x, x2, z2, pol;
  load_f(C + CH_X * 8, x);
  load_f(C + CH_X2 * 8, x2);
  load_f(C + CH_Z2 * 8, z2);
  load_f(C + CH_POL * 8, pol);
  Fr ip = fr_from_canon(S + RP_SC_IP * 8);
  auto put = [&](int slot, const Fr& v) { store_f(M + slot * 8, f_from_mont(f_neg(v))); };  // canonical, negated
  put(RP_PT_T1, fr_mul(rho, x));
  put(RP_PT_T2, fr_mul(rho, x2));
  put(RP_PT_V, fr_mul(rho, z2));
  store_f(K + 0 * 8, fr_mul(rho, f_sub(ip, pol)));
  store_f(K + 1 * 8, fr_mul(rho, fr_from_canon(S + RP_SC_TAU * 8)));
  if (!e2) return;
  Fr a = fr_from_canon(S + RP_SC_A * 8), bb = fr_from_canon(S + RP_SC_B * 8), x0;
  load_f(C + CH_X0 * 8, x0);
  store_f(M + RP_PT_C * 8, f_from_mont(rho2));  // slot C holds -com: scalar +rho' 
  for (int j = 0; j < k; j++) {
    Fr xj, xji;
    load_f(C + (CH_XJ + j) * 8, xj);
    load_f(C + (CH_XJ + k + j) * 8, xji);
    put(RP_PT_L + j, fr_mul(rho2, fr_sqr(xj)));
    put(RP_PT_L + k + j, fr_mul(rho2, fr_sqr(xji)));
  }
  store_f(K + 2 * 8, fr_mul(rho2, fr_mul(f_sub(fr_mul(a, bb), ip), x0)));
  store_f(K + 3 * 8, fr_mul(rho2, a));
  store_f(K + 4 * 8, fr_mul(rho2, bb));
}

// one block per column: col 0 G (ped1), 1 H (ped2), 2 Q, 3+i G_i, 3+n+i H_i
__global__ void __launch_bounds__(256) k_rlc_columns(int B, int n, int k, const uint32_t* __restrict__ ch,
                                                     const uint32_t* __restrict__ coef, uint32_t* __restrict__ colsum) {
  __shared__ uint32_t sh[256 * 8];
  const int col = blockIdx.x, t = threadIdx.x;
  Fr acc = f_zero<FrP>();
  for (int b = t; b < B; b += 256) {
    const uint32_t* K = coef + (size_t)b * RLC_NCOEF * 8;
    const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
    Fr v;
    if (col < 3) {
      load_f(K + col * 8, v);
    } else if (col < 3 + n) {
      Fr ra;
      load_f(K + 3 * 8, ra);
      v = f_is_zero(ra) ? ra : fr_mul(ra, s_vec(C, k, col - 3));
    } else {
      int i = col - 3 - n;
      Fr rb;
      load_f(K + 4 * 8, rb);
      if (!f_is_zero(rb)) {
        Fr yinv;
        load_f(C + CH_YINV * 8, yinv);
        v = fr_mul(fr_mul(rb, s_vec(C, k, n - 1 - i)), fr_pow_small(yinv, (uint32_t)i));
      } else {
        v = rb;
      }
    }
    acc = f_add(acc, v);
  }
  store_f(sh + t * 8, acc);
  __syncthreads();
  for (int half = 128; half >= 1; half >>= 1) {
    if (t < half) {
      Fr o;
      load_f(sh + (t + half) * 8, o);
      acc = f_add(acc, o);
      store_f(sh + t * 8, acc);
    }
    __syncthreads();
  }
  if (t == 0) store_f(colsum + col * 8, f_from_mont(acc));
}

__global__ void __launch_bounds__(64) k_rlc_fixed(int n, const uint32_t* __restrict__ colsum,
                                                  const uint32_t* __restrict__ tables, uint32_t* __restrict__ out) {
  int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= 3 + 2 * n) return;
  int base = col == 0 ? tb_G(n) : col == 1 ? tb_H(n) : col == 2 ? tb_Q(n) : col - 3;
  Scalar s;
#pragma unroll
  for (int q = 0; q < 8; q++) s.v[q] = colsum[col * 8 + q];
  store_g1j(out + (size_t)col * 24, fixed_base_mul(tables + (size_t)base * FB_WORDS_PER_BASE, s));
}

// batch verdict: flag = 1 if the combination is the identity; on success the
// deferred IPA structural verdicts become final (their E1 held)
__global__ void __launch_bounds__(64) k_rlc_finalize(int B, const uint32_t* __restrict__ msm_out,
                                                     int32_t* __restrict__ status, const int32_t* __restrict__ ipa_flag,
                                                     int32_t* __restrict__ flag) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  Fp z;
  load_fp(msm_out + 16, z);
  const bool pass = f_is_zero(z);
  if (b == 0) *flag = pass ? 1 : 0;
  if (b < B && pass && status[b] == 0 && ipa_flag[b] != 0) status[b] = ipa_flag[b];
}

// ------------------------------------------------------------ host launch
#define FTS_LAUNCH(kern, nthreads, bs, stream, ...)                                   \
  do {                                                                                \
    size_t nt_ = (size_t)(nthreads);                                                  \
    if (nt_) hipLaunchKernelGGL(kern, dim3((unsigned)((nt_ + (bs)-1) / (bs))), dim3(bs), 0, stream, __VA_ARGS__); \
  } while (0)



size_t rp_scratch_words(int B, int n, int k) { return (size_t)B * (3 + 2 * k) * 10 * 24; }
size_t rp_terms_words(int B, int n, int k) { return (size_t)B * rp_nterms(n, k) * 24; }

void launch_build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s) {
  FTS_LAUNCH(k_build_tables, nb * FB_WINDOWS, 64, s, bases, nb, tables, scratch);
}

void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, Timeline* tl);

// exact per-proof phase: everything that is hashed (challenges, H'_i, com, x0)
void launch_rp_exact(const RpBatchDev& d, const uint32_t* tables, const uint8_t* x0_const, hipStream_t s,
                     Timeline* tl) {
  const int B = d.B, n = d.n, k = d.k;
  FTS_LAUNCH(k_rp_decode, B * rp_npts(k), 256, s, B, rp_npts(k), d.raw, d.pts, d.status);
  if (tl) tl->mark("k_rp_decode", s);
  FTS_LAUNCH(k_rp_hash_small, B * (2 + k), 64, s, B, n, k, d.raw, d.status, d.ch, d.small_msgs);
  if (tl) tl->mark("k_rp_hash_small", s);
  FTS_LAUNCH(k_rp_chal_fr, B, 64, s, B, n, k, d.status, d.ch, d.scratch);
  if (tl) tl->mark("k_rp_chal_fr", s);
  FTS_LAUNCH(k_rp_hprime, B * n, 64, s, B, n, k, d.status, d.ch, tables, d.hpj);
  if (tl) tl->mark("k_rp_hprime", s);
  FTS_LAUNCH(k_rp_hp_normalize, B, 64, s, B, n, d.status, d.hpj, d.hpa, d.hp_be);
  if (tl) tl->mark("k_rp_hp_normalize", s);
  FTS_LAUNCH(k_rp_com_terms, B * com_nterms(n), 64, s, B, n, k, d.status, d.pts, d.sc, d.ch, tables, d.terms,
             d.scratch);
  if (tl) tl->mark("k_rp_com_terms", s);
  if (B) hipLaunchKernelGGL(k_rp_com_sum, dim3(B), dim3(64), 0, s, B, n, k, d.status, d.pts, d.terms, d.com, d.com_be);
  if (tl) tl->mark("k_rp_com_sum", s);
  FTS_LAUNCH(k_rp_x0_build, B * (2 * n + 3), 256, s, B, n, d.status, d.hp_be, d.com_be, x0_const, d.sc, d.x0_msgs);
  if (tl) tl->mark("k_rp_x0_build", s);
  FTS_LAUNCH(k_rp_x0_hash, B, 64, s, B, n, k, d.status, d.x0_msgs, d.ch);
  if (tl) tl->mark("k_rp_x0_hash", s);
}

// random-linear-combination check of all final equations (one MSM)
void launch_rp_rlc(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, hipStream_t s, Timeline* tl) {
  const int B = d.B, n = d.n, k = d.k;
  FTS_LAUNCH(k_rlc_prep, B, 64, s, B, n, k, d.status, d.ipa_flag, d.sc, d.ch, r.key, r.msc, r.coef);
  hipLaunchKernelGGL(k_rlc_columns, dim3(3 + 2 * n), dim3(256), 0, s, B, n, k, d.ch, r.coef, r.colsum);
  FTS_LAUNCH(k_rlc_fixed, 3 + 2 * n, 64, s, n, r.colsum, tables, r.fixed);
  if (tl) tl->mark("k_rlc_scalars", s);
  launch_msm(r.plan, d.pts, r.msc, r.fixed, 3 + 2 * n, r.msm_scratch, s, tl);
  FTS_LAUNCH(k_rlc_finalize, B > 0 ? B : 1, 64, s, B, r.plan.out, d.status, d.ipa_flag, r.flag);
  if (tl) tl->mark("k_rlc_finalize", s);
}

// per-proof final equations (fallback when the batch combination fails)
void launch_rp_fallback(const RpBatchDev& d, const uint32_t* tables, hipStream_t s, Timeline* tl) {
  const int B = d.B, n = d.n, k = d.k;
  FTS_LAUNCH(k_rp_terms_fixed, B * (3 + 2 * n), 64, s, B, n, k, d.status, d.ipa_flag, d.sc, d.ch, tables, d.terms);
  if (tl) tl->mark("k_rp_terms_fixed", s);
  FTS_LAUNCH(k_rp_terms_var, B * (3 + 2 * k), 64, s, B, n, k, d.status, d.ipa_flag, d.pts, d.ch, d.terms, d.scratch);
  if (tl) tl->mark("k_rp_terms_var", s);
  FTS_LAUNCH(k_rp_check, B, 64, s, B, n, k, d.status, d.ipa_flag, d.terms, d.com);
  if (tl) tl->mark("k_rp_check", s);
}

}  // namespace fts
