// Range-proof (Bulletproof + IPA) batch verification kernels for gfx950.
//
// One launch sequence verifies a whole batch of B proofs of bit length n
// (k = log2 n rounds).  Work is laid out per (proof, item) so a batch of a
// few thousand proofs fills the 256 CUs.  Streams of a lane: S main, S2 the
// x0 prefix (work path) / x*D (latency path), S3 the batch check's weights and
// MSM, S4 its x0-free fixed-base columns (fork/join through events).
// Work path (passes above FTS_COM_FIXED_MAX proofs):
//
//   S   k_rp_decode        (proof, point)   NewG1FromBytes checks + Montgomery form
//   S   k_rp_hash_small    (proof, msg)     x, y, x_j transcripts (SHA-256 over hex)  bulletproof.go:266-281, ipa.go:230
//   S   k_rp_chal_fr       proof            z, polEval, batch inversion of y, x_j       bulletproof.go:282-311, ipa.go:236-244
//   S   k_rp_powers        (chunk, proof)   y^-i, s_i, z^2 2^i y^-i                     ipa.go:343-356 (unrolled)
//   S   k_rp_fixed_exact   (proof, item)    H'_i = y^-i H_i, z K, -delta P (fixed base) bulletproof.go:483-489
//   S   k_rp_normalize     point (block)    batch affine normalisation of H'_i (one inversion per block)
//   S   k_rp_hsum_chunks   (proof, chunk)   S_c = sum_j 2^j H'_{16c+j} (Horner)
//   S   k_rp_hsum_join     proof            S = sum_c 2^(16c) S_c
//   S   k_rp_com_var       2 lanes/proof    x*D + z^2*S (joint GLV/Straus, affine lane tables),
//                                           com = C + z K - delta P + x D + z^2 S       bulletproof.go:477-492
//   S2  k_rp_x0_build/hash proof            x0 prefix: H' records + shared template     ipa.go:200-213
//   S   k_rp_x0_build/hash proof            x0 suffix after com: x0 = HashToZr(...)     ipa.go:213
//   S3  k_rlc_prep + MSM                    weights, variable points of the batch equation (no x0)
//   S4  k_rlc_columns/fixed                 x0-free fixed-base columns of the batch equation
//   S   k_rlc_columns/fixed (Q), finalize   column Q (needs x0), verdict
//   k_rp_terms_fixed / k_rp_terms_var / k_rp_check: per-proof fallback
//
#include <atomic>
#include "device/g1.hpp"
#include "device/fixed_base.hpp"
#include "device/glv.hpp"
#include "device/rp_kernels.hpp"
#include "device/transcript.hpp"
#include "device/helpers.hpp"
#include "device/msm.hpp"
#include "device/coop.hpp"
#include "common/chacha20.hpp"
#include "../../include/fts_gpu.h"

namespace fts {
// block size of the latency-bound per-proof kernels (few waves, long chains):
// 256-thread blocks put a block's 4 waves on the 4 SIMDs of one CU, and the
// dispatcher spreads blocks over CUs, so concurrent small kernels of the
// pass's streams rarely share a SIMD (64-thread blocks of two such kernels
// slowed each other by ~26 %, tools/experiments/colocate.cpp)
int g_lat_bs = 256;
// block size of the work path's per-proof latency kernels (k_rp_chal_fr, k_rlc_prep,
// k_rp_x0_hash; FTS_WORK_BS): they start beside another pass's fixed-base launch
// (64-thread blocks filling the register file), where a 256-thread block waits for
// four wave slots of one CU at once (k_rp_chal_fr 0.12 ms alone, 1.1 ms there;
// k_rlc_prep 0.18 -> 1.8 ms in a 20-batch burst, round 5)
std::atomic<int> g_work_bs{64};  // written by context creation while other lanes launch
// block size of the work path's S / com chain kernels
constexpr int g_chain_bs = 64;


constexpr int NORM_BS = 256;
// points per lane of k_rp_normalize (one inversion per lane, round 5): 16 for
// normalisations of >= NORM_BIG points, 4 below (more lanes for small batches)
constexpr int NORM_E = 16;  // nominal, for the cost model
constexpr size_t NORM_BIG = (size_t)1 << 16;
template <int E>
__global__ void __launch_bounds__(NORM_BS) k_rp_normalize(int total, int per, int stride, int first,
                                                          const int32_t* __restrict__ status,
                                                          const uint32_t* __restrict__ jac, uint32_t* __restrict__ aff,
                                                          uint8_t* __restrict__ be, uint8_t* __restrict__ x0msgs);
static void launch_normalize(size_t total, int per, int stride, int first, const int32_t* status, const uint32_t* jac,
                             uint32_t* aff, uint8_t* be, hipStream_t s, uint8_t* x0msgs = nullptr);
// Jacobian -> affine (Montgomery, 16 words) and BE bytes of ONE point by its own
// inversion (identity -> (0, 0)): com at the end of its chain (round 5: instead of
// a k_rp_normalize launch of one point per proof on the critical path)
FTS_DEV void store_affine_one(const G1J& p, uint32_t* aff, uint8_t* be) {
  G1A r;
  if (f_is_zero(p.z)) {
    r.x = f_zero<FpP>();
    r.y = f_zero<FpP>();
  } else {
    const Fp zi = nl_fp_inv(p.z), zi2 = fp_sqr(zi);
    r.x = fp_mul(p.x, zi2);
    r.y = fp_mul(fp_mul(p.y, zi2), zi);
  }
  store_g1a(aff, r);
  store_point_be(be, r);
}

// ---------------------------------------------------------- context tables
// Built once per context (device/fixed_base.hpp layout), for nb bases:
//   kt_window_bases  lane per (base, window)   B_w = 2^(W w) B            (Jacobian)
//   kt_small_large   lane per (base, window)   small[lo] = (lo+1) B_w, large[hi] = hi S B_w
//   kt_entries       lane per entry            T[w][d-1] = large[hi] + small[lo], d-1 = hi S + lo
// for window width W (FbCfg<W>: 16-bit for every base, 20-bit for H_i, K, P)
//   k_rp_normalize   block per 256 entries     affine (one inversion per block)
template <int W>
__global__ void __launch_bounds__(64) kt_window_bases(const uint32_t* __restrict__ bases, int nb,
                                                      uint32_t* __restrict__ bw) {
  using C = FbCfg<W>;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nb * C::NW) return;
  int b = gid / C::NW, w = gid % C::NW;
  G1J p = g1j_from_affine(load_g1a(bases + b * 16));
  for (int i = 0; i < W * w; i++) p = nl_dbl(p);
  store_g1j(bw + (size_t)gid * 24, p);
}

template <int W>
__global__ void __launch_bounds__(64) kt_small_large(int nb, const uint32_t* __restrict__ bw,
                                                     uint32_t* __restrict__ small, uint32_t* __restrict__ large) {
  using C = FbCfg<W>;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nb * C::NW) return;
  const uint32_t* Bw = bw + (size_t)gid * 24;
  uint32_t* S = small + (size_t)gid * C::S * 24;
  uint32_t* L = large + (size_t)gid * C::L * 24;
  G1J acc = load_g1j(Bw);
  store_g1j(S, acc);
  for (int lo = 1; lo < C::S; lo++) {
    acc = nl_add_mem(acc, Bw, 0);
    store_g1j(S + lo * 24, acc);
  }
  // acc = S * B_w
  store_g1j(L, g1j_identity());
  G1J big = g1j_identity();
  for (int hi = 1; hi < C::L; hi++) {
    big = nl_add_mem(big, S + (C::S - 1) * 24, 0);
    store_g1j(L + hi * 24, big);
  }
}

template <int W>
__global__ void __launch_bounds__(64) kt_entries(int nb, const uint32_t* __restrict__ small,
                                                 const uint32_t* __restrict__ large, uint32_t* __restrict__ jac) {
  using C = FbCfg<W>;
  size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)nb * C::NW * C::E) return;
  const size_t bw = gid / C::E;
  const int e = (int)(gid % C::E);  // d - 1
  const int hi = e / C::S, lo = e % C::S;
  G1J p = load_g1j(small + (bw * C::S + lo) * 24);
  if (hi) p = nl_add_mem(p, large + (bw * C::L + hi) * 24, 0);
  store_g1j(jac + gid * 24, p);
}

// ------------------------------------------------------------------ gather
// thread per (proof, 16-byte chunk) of the merged pass: raw points
// (npts x 64 B), canonical scalars (RP_NSC x 32 B), host verdicts, IPA flags
__global__ void __launch_bounds__(256) k_rp_gather(RpGather g, int npts, uint8_t* __restrict__ raw,
                                                   uint32_t* __restrict__ sc, int32_t* __restrict__ status,
                                                   int32_t* __restrict__ ipa) {
  wave_prio<PS_HEAD>();
  const int per = npts * 4 + RP_NSC * 2 + 1;  // uint4 chunks of raw, sc, + 1 lane for the two flags
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int B = g.off[g.G];
  if (gid >= (size_t)B * per) return;
  const int p = (int)(gid / per), c = (int)(gid % per);
  int q = 0;
  while (q + 1 < g.G && g.off[q + 1] <= p) q++;
  const int i = p - g.off[q];
  if (c < npts * 4) {
    reinterpret_cast<uint4*>(raw)[(size_t)p * npts * 4 + c] = reinterpret_cast<const uint4*>(g.raw[q])[(size_t)i * npts * 4 + c];
  } else if (c < npts * 4 + RP_NSC * 2) {
    const int cc = c - npts * 4;
    reinterpret_cast<uint4*>(sc)[(size_t)p * RP_NSC * 2 + cc] = reinterpret_cast<const uint4*>(g.sc[q])[(size_t)i * RP_NSC * 2 + cc];
  } else {
    status[p] = g.status0[q][i];
    ipa[p] = g.ipa[q][i];
  }
}

// ------------------------------------------------------------------ decode
// NewG1FromBytes (asn1.go:148 -> gnark SetBytes): 64 bytes, flag bits 00,
// canonical coordinates, on the curve; 64 zero bytes = identity.
__global__ void __launch_bounds__(256) k_rp_decode(int B, int npts, const uint8_t* __restrict__ raw,
                                                   uint32_t* __restrict__ pts, int32_t* __restrict__ status) {
  wave_prio<PS_HEAD>();
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
  wave_prio<PS_HEAD>();
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
    store_f(reinterpret_cast<uint32_t*>(slot), h);  // canonical x for k_rp_xd (runs beside k_rp_chal_fr)
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
__global__ void __launch_bounds__(256) k_rp_chal_fr(int B, int n, int k, const int32_t* __restrict__ status,
                                                   uint32_t* __restrict__ ch, uint32_t* __restrict__ tmp) {
  wave_prio<PS_HEAD>();
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
  // sum_{i<n} y^i by doubling (n = 2^k): S_2m = S_m (1 + y^m), y^2m = (y^m)^2
  // (same field element as the reference's loop, bulletproof.go:287-305)
  Fr ipy = f_one<FrP>(), ym = y;
  for (int m = 1; m < n; m <<= 1) {
    ipy = fr_mul(ipy, f_add(f_one<FrP>(), ym));
    ym = fr_sqr(ym);
  }
  // sum_{i<n} 2^i = 2^n - 1 (< r for n <= 64)
  Fr ip2 = f_zero<FrP>();
  ip2.v[0] = n >= 32 ? 0xffffffffu : (1u << n) - 1u;
  ip2.v[1] = n >= 64 ? 0xffffffffu : (n > 32 ? (1u << (n - 32)) - 1u : 0u);
  ip2 = f_to_mont(ip2);
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

// lane per (chunk c of PW_CH indices, proof b), chunk-major: for i in the chunk
//   ypow[i][b] = y^-i                                 (bulletproof.go:483-485)
//   svec[i][b] = s_i = prod_j x_j^(+1 if bit k-1-j of i else -1)
// (the generator folding of ipa.go:343-356 unrolled: G_fin = sum s_i G_i,
// H'_fin = sum s_i^-1 H'_i = sum s_{n-1-i} H'_i).  The chunk's high index
// bits give a common prefix product; the low bits expand as a binary tree.
constexpr int PW_LC = 3, PW_CH = 1 << PW_LC;
// (latency path, zvec != nullptr: also zvec[i][b] = z^2 2^i y^-i, the scalars of
// the com terms Z_i of k_rp_fixed_all)
__global__ void __launch_bounds__(64) k_rp_powers(int B, int n, int k, const int32_t* __restrict__ status,
                                                  const uint32_t* __restrict__ ch, uint32_t* __restrict__ ypow,
                                                  uint32_t* __restrict__ svec, uint32_t* __restrict__ zvec) {
  wave_prio<PS_HEAD>();
  const int lc = min(PW_LC, k), cs = 1 << lc, nch = n >> lc;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nch) return;
  const int c = gid / B, b = gid % B;
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const int i0 = c * cs;
  Fr yinv;
  load_f(C + CH_YINV * 8, yinv);
  Fr yp = fr_pow_small(yinv, (uint32_t)i0);
  Fr zv;  // z^2 2^i
  if (zvec) {
    load_f(C + CH_Z2 * 8, zv);
    for (int i = 0; i < i0; i++) zv = f_add(zv, zv);
  }
  for (int q = 0; q < cs; q++) {
    if (q) yp = fr_mul(yp, yinv);
    store_f(ypow + ((size_t)(i0 + q) * B + b) * 8, yp);
    if (zvec) {
      store_f(zvec + ((size_t)(i0 + q) * B + b) * 8, fr_mul(zv, yp));
      zv = f_add(zv, zv);
    }
  }
  // prefix over the high bits: j = 0 .. k-1-lc  (bit k-1-j of i0)
  Fr pre = f_one<FrP>();
  for (int j = 0; j < k - lc; j++) {
    Fr f;
    load_f(C + (CH_XJ + (((i0 >> (k - 1 - j)) & 1) ? 0 : k) + j) * 8, f);
    pre = j ? fr_mul(pre, f) : f;
  }
  if (lc == PW_LC) {
    Fr v[PW_CH];
    v[0] = pre;
#pragma unroll
    for (int l = 0; l < PW_LC; l++) {  // low bits, MSB first: index 2t + bit
      const int j = k - PW_LC + l;
      Fr xj, xji;
      load_f(C + (CH_XJ + j) * 8, xj);
      load_f(C + (CH_XJ + k + j) * 8, xji);
#pragma unroll
      for (int t = (1 << l) - 1; t >= 0; t--) {
        const Fr base = v[t];
        v[2 * t + 1] = fr_mul(base, xj);
        v[2 * t] = fr_mul(base, xji);
      }
    }
#pragma unroll
    for (int q = 0; q < PW_CH; q++) store_f(svec + ((size_t)(i0 + q) * B + b) * 8, v[q]);
  } else {  // n < 8: one chunk, direct products
    for (int q = 0; q < cs; q++) {
      Fr sv = f_one<FrP>();
      for (int j = 0; j < k; j++) {
        Fr f;
        load_f(C + (CH_XJ + (((q >> (k - 1 - j)) & 1) ? 0 : k) + j) * 8, f);
        sv = fr_mul(sv, f);
      }
      store_f(svec + ((size_t)q * B + b) * 8, sv);
    }
  }
}

// ------------------------------------------------------------ H' and com
// com = x*D + C - z sum G_i + sum (z y^i + z^2 2^i) H'_i - delta*P   (bulletproof.go:477-492)
//     = x*D + C + z*K - delta*P + z^2 * S,   K = sum H_i - sum G_i,  S = sum_i 2^i H'_i
// (z y^i H'_i = z H_i folds into z K; the same group element, and only its
// affine form is observable).  S is a Horner sum over the exact H'_i, so
// the n fixed-base products of the com terms become one variable-base product.
// Terms per proof (com_terms): 0 z*K, 1 -delta*P, 2,3 the GLV halves of x*D,
// 4,5 the GLV halves of z^2*S.
constexpr int COM_NTERMS = 4;  // z K, -delta P, the two joint GLV halves
// Horner chunks of S = sum_i 2^i H'_i: 16 H' per chunk (4 chunks at n = 64),
// joined once per proof by k_rp_hsum_join (slot 0 of the proof's chunks)
constexpr int HS_CHUNK = 16;
constexpr int HS_SCRATCH = 4 * 24;  // scratch words per proof for the chunks (n <= 64)
inline __host__ __device__ int com_nterms(int n) { return COM_NTERMS; }

// lane per (proof, item): items 0..n-1: H'_i = y^-i H_i (-> hpj[b][i]);
// n: z K; n+1: -delta P (-> terms[b][0..1])
// wtables: the 20-bit tables of [H_0 .. H_{n-1}, K, P] (FbWide layout)
template <int W>
__global__ void __launch_bounds__(64, 4) k_rp_fixed_exact(int B, int n, int k, const int32_t* __restrict__ status,
                                                          const uint32_t* __restrict__ sc, const uint32_t* __restrict__ ch,
                                                          const uint32_t* __restrict__ ypow,
                                                          const uint32_t* __restrict__ wtables, uint32_t* __restrict__ hpj,
                                                          uint32_t* __restrict__ terms) {
  wave_prio<PS_FIXED>();
  const int ni = n + 2;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)B * ni) return;
  // proof index fastest: a wave's 64 lanes gather from the same base's table (and
  // read ypow[t][b] coalesced): 6.9 -> 6.2 ms per 81,920-proof launch and 4.77 ->
  // 1.79 GB fetched against one proof's items side by side (round 2)
  const int b = (int)(gid % B), t = (int)(gid / B);
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  uint32_t* out;
  const uint32_t* tab;
  Scalar sk;
  if (t < n) {
    Fr yp;
    load_f(ypow + ((size_t)t * B + b) * 8, yp);
    tab = wtables + (size_t)t * FbCfg<W>::WORDS_PER_BASE;
    sk = fr_canon(yp);
    out = hpj + ((size_t)b * (n + 1) + t) * 24;
  } else if (t == n) {
    Fr z;
    load_f(C + CH_Z * 8, z);
    tab = wtables + (size_t)n * FbCfg<W>::WORDS_PER_BASE;
    sk = fr_canon(z);
    out = terms + ((size_t)b * COM_NTERMS + 0) * 24;
  } else {
    Fr d;
    load_f(sc + ((size_t)b * RP_NSC + RP_SC_DELTA) * 8, d);  // canonical
    Fr nd = f_neg(d);
#pragma unroll
    for (int q = 0; q < 8; q++) sk.v[q] = nd.v[q];
    tab = wtables + (size_t)(n + 1) * FbCfg<W>::WORDS_PER_BASE;
    out = terms + ((size_t)b * COM_NTERMS + 1) * 24;
  }
  G1J r = fb_mul_w<W>(tab, sk);
  store_g1j(out, r);
}

// lane per (proof, chunk c): S_c = sum_{j < 16} 2^j H'_{16c+j} (Horner over the
// Jacobian H' of k_rp_fixed_exact: full additions, so the chain does not wait for
// the H' normalisation, which runs beside it on the x0 stream)
__global__ void __launch_bounds__(256) k_rp_hsum_chunks(int B, int n, const int32_t* __restrict__ status,
                                                       const uint32_t* __restrict__ hpj, uint32_t* __restrict__ chunks) {
  wave_prio<PS_HSUM>();
  const int nc = (n + HS_CHUNK - 1) / HS_CHUNK;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nc) return;
  const int b = gid / nc, c = gid % nc;
  if (status[b] != 0) return;
  const int lo = c * HS_CHUNK, hi = min(n, lo + HS_CHUNK);
  const uint32_t* H = hpj + (size_t)b * (n + 1) * 24;  // Jacobian H'
  G1J acc = load_g1j(H + (hi - 1) * 24);
  for (int i = hi - 2; i >= lo; i--) {
    acc = g1j_dbl(acc);
    add_inl(acc, load_g1j(H + i * 24));
  }
  store_g1j(chunks + (size_t)gid * 24, acc);
}

// lane per proof: S = sum_c 2^(16c) S_c (Horner over k_rp_hsum_chunks' chunk sums,
// 3 x (16 doublings + 1 addition) at n = 64) -> slot 0 of the proof's chunks.
// Once per proof: the two lanes of k_rp_com_var used to join S each, 17 % of
// their chain
__global__ void __launch_bounds__(256) k_rp_hsum_join(int B, int n, const int32_t* __restrict__ status,
                                                     uint32_t* __restrict__ chunks) {
  wave_prio<PS_HSUM>();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  const int nc = (n + HS_CHUNK - 1) / HS_CHUNK;
  uint32_t* Sc = chunks + (size_t)b * nc * 24;
  G1J S = load_g1j(Sc + (nc - 1) * 24);
  for (int c = nc - 2; c >= 0; c--) {
    for (int q = 0; q < HS_CHUNK; q++) S = g1j_dbl(S);
    add_inl(S, load_g1j(Sc + c * 24));
  }
  store_g1j(Sc, S);
}

// x*D + z^2*S (bulletproof.go:478, 486-489 via S), two lanes per proof: with
// x = x1 + x2 lambda and z^2 = w1 + w2 lambda (GLV), lane h computes
// x_h phi^h(D) + w_h phi^h(S) in one joint Straus chain over an affine lane
// table (glv.hpp straus2_atab); S from k_rp_hsum_join -> terms[b][2 + h]
#ifndef FTS_COMVAR_OCC
#define FTS_COMVAR_OCC 3  // waves per SIMD the register budget allows (A/B builds: -DFTS_COMVAR_OCC=4)
#endif
__global__ void __launch_bounds__(256, FTS_COMVAR_OCC) k_rp_com_var(int B, int n, int k, const int32_t* __restrict__ status,
                                                   const uint32_t* __restrict__ pts, const uint32_t* __restrict__ ch,
                                                   const uint32_t* __restrict__ chunks, uint32_t* __restrict__ atab,
                                                   const uint32_t* __restrict__ terms, uint32_t* __restrict__ hpj,
                                                   uint32_t* __restrict__ hpa, uint8_t* __restrict__ hp_be) {
  wave_prio<PS_COMVAR>();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = gid >> 1, h = gid & 1;
  if (b >= B || status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  Fr x, z2;
  load_f(C + CH_X * 8, x);
  load_f(C + CH_Z2 * 8, z2);
  // this lane's GLV halves by selects, not by indexing [h]: a runtime index made
  // the compiler keep the arrays in LDS (16 KB per 64-lane block), and com_var's
  // blocks then held every CU's LDS and starved the x0 build beside them (round 5)
  uint32_t xa[4], xb[4], xs0, xs1, wa[4], wb[4], ws0, ws1, xh[4], wh[4];
  glv_decompose(fr_canon(x).v, xa, xs0, xb, xs1);
  glv_decompose(fr_canon(z2).v, wa, ws0, wb, ws1);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    xh[q] = h ? xb[q] : xa[q];
    wh[q] = h ? wb[q] : wa[q];
  }
  const bool xsh = (h ? xs1 : xs0) != 0, wsh = (h ? ws1 : ws0) != 0;
  const int nc = (n + HS_CHUNK - 1) / HS_CHUNK;
  G1J S = load_g1j(chunks + (size_t)b * nc * 24);  // k_rp_hsum_join
  const G1A Da = load_g1a(pts + ((size_t)b * rp_npts(k) + RP_PT_D) * 16);
  const bool idD = g1a_is_identity(Da), idS = f_is_zero(S.z);
  // the proof's shared table: lane 0 builds 1..8 D, lane 1 1..8 S (one instruction
  // stream on the lane's own point: no divergence).  Both lanes of a proof are
  // adjacent lanes (gid 2b, 2b + 1) of ONE wave64 wave, which runs them in
  // lockstep: the fence makes each lane's row stores visible, the wave barrier
  // keeps the compiler from moving the other lane's reads above it
  static_assert(256 % 64 == 0, "k_rp_com_var: a proof's lane pair must sit in one wave");
  const CTab T{atab, (size_t)B, (size_t)b};
  const G1J Dj = g1j_from_affine(Da);
  ctab_build8<false>(T, 8 * h, h ? S : Dj, h ? idS : idD);
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  G1J r = straus2_ctab(T, h, xh, xsh, wh, wsh, idD, idS);
  // com = C + z K - delta P + x D + z^2 S (bulletproof.go:477-492), summed by the
  // proof's two lanes (adjacent lanes of one wave; both exit or both run): lane h
  // adds its fixed-base term (z K or -delta P, k_rp_fixed_exact), lane 0 also C,
  // then lane 0 adds lane 1's partial (cross-lane shuffle) and writes com
  add_inl(r, load_g1j(terms + ((size_t)b * COM_NTERMS + h) * 24));
  G1J c = g1j_identity();
  if (h == 0) c = g1j_from_affine(load_g1a(pts + ((size_t)b * rp_npts(k) + RP_PT_C) * 16));
  add_inl(r, c);
  G1J o;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    o.x.v[q] = __shfl_xor(r.x.v[q], 1);
    o.y.v[q] = __shfl_xor(r.y.v[q], 1);
    o.z.v[q] = __shfl_xor(r.z.v[q], 1);
  }
  if (h == 0) {
    add_inl(r, o);
    const size_t q = (size_t)b * (n + 1) + n;
    store_g1j(hpj + q * 24, r);
    store_affine_one(r, hpa + q * 16, hp_be + q * 64);  // com for the x0 suffix (no normalize_com launch)
  }
}

// ----------------------------------------- com, latency path (small passes)
// The same group element as the work path below/above, computed without a
// per-proof doubling chain on the critical path (bulletproof.go:477-492):
//   com = C + x*D + z*K - delta*P + sum_i (z^2 2^i y^-i) H_i
// (z^2 2^i H'_i = z^2 2^i y^-i H_i): the n z^2-terms become fixed-base products
// on the 20-bit tables of H_i, computed by the same lanes as the H'_i
// (k_rp_fixed_all: two products per lane, same table), summed by an LDS tree
// (k_rp_com_tree); x*D runs beside them on the side stream (k_rp_xd, one GLV
// half per lane, started right after the x transcript).  ~3.8 k more products
// per rp64 than the work path, but every product runs at the fixed-base
// kernels' occupancy: used for passes of up to FTS_COM_FIXED_MAX proofs, where
// the work path's per-proof chains leave most SIMDs idle.
// terms layout [B][n + 4][24]: Z_0..Z_{n-1}, z K, -delta P, x*D halves
inline __host__ __device__ int com_fx_slots(int n) { return n + 4; }

// lane per (item, proof), proof index fastest (a wave's 64 lanes gather from
// the same table), one fixed-base product per lane: items i < n: H'_i = y^-i H_i
// -> hpj[b][i]; items n + i: Z_i = (z^2 2^i y^-i) H_i -> terms[b][i]; item 2n:
// z K -> terms[b][n]; item 2n + 1: -delta P -> terms[b][n + 1]
template <int W>
__global__ void __launch_bounds__(64, 4) k_rp_fixed_all(int B, int n, int k, const int32_t* __restrict__ status,
                                                        const uint32_t* __restrict__ sc, const uint32_t* __restrict__ ch,
                                                        const uint32_t* __restrict__ ypow,
                                                        const uint32_t* __restrict__ zvec,
                                                        const uint32_t* __restrict__ wtables, uint32_t* __restrict__ hpj,
                                                        uint32_t* __restrict__ terms) {
  wave_prio<PS_FIXED>();
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)(2 * n + 2) * B) return;
  const int t = (int)(gid / B), b = (int)(gid % B);
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const int base = t < n ? t : t - n;  // H_i (i < n), K (n), P (n + 1)
  Scalar sk;
  if (t < 2 * n) {
    Fr v;
    load_f((t < n ? ypow : zvec) + ((size_t)base * B + b) * 8, v);
    sk = fr_canon(v);
  } else if (t == 2 * n) {
    Fr z;
    load_f(C + CH_Z * 8, z);
    sk = fr_canon(z);
  } else {
    Fr d;
    load_f(sc + ((size_t)b * RP_NSC + RP_SC_DELTA) * 8, d);  // canonical
    const Fr nd = f_neg(d);
#pragma unroll
    for (int q = 0; q < 8; q++) sk.v[q] = nd.v[q];
  }
  const G1J r = fb_mul_w<W>(wtables + (size_t)base * FbCfg<W>::WORDS_PER_BASE, sk);
  uint32_t* out = t < n ? hpj + ((size_t)b * (n + 1) + t) * 24 : terms + ((size_t)b * com_fx_slots(n) + base) * 24;
  store_g1j(out, r);
}

// x*D (bulletproof.go:478), one GLV half per lane: x = x1 + x2 lambda, lane h
// computes x_h phi^h(D) -> terms[b][n + 2 + h]; lane tables 1..8 * P in vtab.
// x is read from the digest k_rp_hash_small left at the head of its slot
// (canonical), so this runs concurrently with k_rp_chal_fr.
__global__ void __launch_bounds__(256) k_rp_xd(int B, int n, int k, const int32_t* __restrict__ status,
                                              const uint32_t* __restrict__ pts, const uint8_t* __restrict__ small_msgs,
                                              uint32_t* __restrict__ vtab, uint32_t* __restrict__ terms, int tstride,
                                              int toff) {
  wave_prio<PS_COMVAR>();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= 2 * B) return;
  const int h = gid / B, b = gid % B;
  if (status[b] != 0) return;
  Fr x;
  load_f(reinterpret_cast<const uint32_t*>(small_msgs + (size_t)b * (2 + k) * SMALL_SLOT), x);
  uint32_t xk[2][4], xs[2];
  glv_decompose(x.v, xk[0], xs[0], xk[1], xs[1]);
  G1J D = g1j_from_affine(load_g1a(pts + ((size_t)b * rp_npts(k) + RP_PT_D) * 16));
  if (h) D.x = fp_mul(D.x, glv_beta());
  if (xs[h]) D.y = f_neg(D.y);
  const G1J r = vb128j(D, xk[h], vtab, (size_t)2 * B, (size_t)gid);
  store_g1j(terms + ((size_t)b * tstride + toff + h) * 24, r);
}

// com = C + sum of the n + 4 terms: CT_LANES lanes per proof (CT_PROOFS proofs
// per block), lane l sums slots l, l + CT_LANES, ... (5 full additions at
// n = 64), then a log2(CT_LANES)-level LDS tree -> hpj[b][n]
constexpr int CT_LANES = 16, CT_PROOFS = 16;
__global__ void __launch_bounds__(CT_LANES * CT_PROOFS) k_rp_com_tree(int B, int n, int k,
                                                                      const int32_t* __restrict__ status,
                                                                      const uint32_t* __restrict__ pts,
                                                                      const uint32_t* __restrict__ terms,
                                                                      uint32_t* __restrict__ hpj,
                                                                      uint32_t* __restrict__ hpa,
                                                                      uint8_t* __restrict__ hp_be) {
  wave_prio<PS_COMVAR>();
  __shared__ uint32_t sh[CT_LANES * CT_PROOFS * 24];
  const int l = threadIdx.x % CT_LANES, pl = threadIdx.x / CT_LANES;
  const int b = blockIdx.x * CT_PROOFS + pl;
  const bool live = b < B && status[b] == 0;
  const int ns = com_fx_slots(n);
  G1J acc = g1j_identity();
  if (live) {
    const uint32_t* T = terms + (size_t)b * ns * 24;
    if (l == 0) acc = g1j_from_affine(load_g1a(pts + ((size_t)b * rp_npts(k) + RP_PT_C) * 16));
    for (int q = l; q < ns; q += CT_LANES) add_inl(acc, load_g1j(T + q * 24));
  }
  uint32_t* S = sh + (size_t)pl * CT_LANES * 24;
  store_g1j(S + l * 24, acc);
  __syncthreads();
  for (int half = CT_LANES / 2; half >= 1; half >>= 1) {
    if (live && l < half) add_inl(acc, load_g1j(S + (l + half) * 24));
    __syncthreads();
    if (live && l < half) store_g1j(S + l * 24, acc);
    __syncthreads();
  }
  if (live && l == 0) {
    const size_t q = (size_t)b * (n + 1) + n;
    store_g1j(hpj + q * 24, acc);
    store_affine_one(acc, hpa + q * 16, hp_be + q * 64);
  }
}

// Batch affine normalisation (Montgomery's trick), E points per lane and ONE
// inversion per lane (point g of group g / per lives at index
// (g / per) * stride + g % per + first; points of proofs with status[g / per]
// != 0 are skipped, identities map to (0, 0)).  Lane l of wave w owns the points
// (w E + j) 64 + l, j < E (every load / store coalesced across the wave):
//   1. forward: the exclusive prefix product of the lane's z's, stored in the
//      point's own affine slot (scratch until step 2 overwrites it);
//   2. one inversion of the lane's product (f_inv_gcd, branch-free);
//   3. back-sweep: z_j^-1 = inv * prefix_j, inv *= z_j; then x z^-2, y z^-3.
// 7 products per point + one inversion per E points, no LDS and no barrier
// (round 5; the round-1..4 kernel scanned the lanes' totals across a 256-lane
// block in LDS and inverted once per block: ~13 products per point, 8 barrier
// levels and one lane inverting while the block waited -- 0.05-0.11 of the MAD
// peak beside the com chain).  Writes affine Montgomery (aff, 16 words) and,
// when be != nullptr, the canonical 64-byte BE encoding.
// x0 record r of a proof's message (ipa.go:200-213): hex(H'_r) + "||" at byte
// 8 + 130 r of its slot (bytes < 64 cb0 sit at their own offset), from the point's
// 16 BE words; 33 stores (4-byte ones where the record's parity allows)
FTS_DEV void x0_put_record(uint8_t* msg, uint32_t r, const uint32_t pw[16]) {
  uint8_t* d = msg + 8u + 130u * r;
  auto hx = [&](int i) -> uint32_t { return hex2((pw[i >> 2] >> (24 - 8 * (i & 3))) & 0xffu); };  // byte i
  if ((r & 1u) == 0) {  // 4-byte aligned
    uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
#pragma unroll
    for (int i = 0; i < 32; i++) d4[i] = hx(2 * i) | (hx(2 * i + 1) << 16);
    reinterpret_cast<uint16_t*>(d)[64] = 0x7c7cu;
  } else {  // 2 mod 4: one 2-byte store, 31 aligned words, then hex(byte 63) "||"
    reinterpret_cast<uint16_t*>(d)[0] = (uint16_t)hx(0);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(d + 2);
#pragma unroll
    for (int i = 0; i < 31; i++) d4[i] = hx(2 * i + 1) | (hx(2 * i + 2) << 16);
    d4[31] = hx(63) | (0x7c7cu << 16);
  }
}

template <int E>
__global__ void __launch_bounds__(NORM_BS) k_rp_normalize(int total, int per, int stride, int first,
                                                          const int32_t* __restrict__ status,
                                                          const uint32_t* __restrict__ jac, uint32_t* __restrict__ aff,
                                                          uint8_t* __restrict__ be, uint8_t* __restrict__ x0msgs) {
  wave_prio<PS_NORM>();
  const size_t gid = (size_t)blockIdx.x * NORM_BS + threadIdx.x;
  const size_t g0 = (gid >> 6) * (size_t)E * 64 + (gid & 63);
  auto slot = [&](int j) {
    const size_t g = g0 + (size_t)j * 64;
    return (g / per) * stride + g % per + first;
  };
  // liveness is read ONCE per point: status may change while this kernel runs
  // (k_sig_exclude on the batch-check stream marks excluded proofs NOT_RUN), and
  // the forward pass and the back-sweep must skip exactly the same points
  uint32_t livem = 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const size_t g = g0 + (size_t)j * 64;
    if (g < (size_t)total && !(status && status[g / per] != 0)) livem |= 1u << j;
  }
  if (!livem) return;
  Fp run = f_one<FpP>();
#pragma unroll
  for (int j = 0; j < E; j++) {
    if (!((livem >> j) & 1u)) continue;
    const size_t q = slot(j);
    store_fp(aff + q * 16, run);  // exclusive prefix (scratch)
    Fp z;
    load_fp(jac + q * 24 + 16, z);
    if (!f_is_zero(z)) run = fp_mul(run, z);
  }
  Fp inv = nl_fp_inv(run);
#pragma unroll
  for (int j = E - 1; j >= 0; j--) {
    if (!((livem >> j) & 1u)) continue;
    const size_t q = slot(j);
    const G1J p = load_g1j(jac + q * 24);
    Fp pre;
    load_fp(aff + q * 16, pre);
    G1A r;
    if (f_is_zero(p.z)) {
      r.x = f_zero<FpP>();
      r.y = f_zero<FpP>();
    } else {
      const Fp zi = fp_mul(inv, pre);
      inv = fp_mul(inv, p.z);
      const Fp zi2 = fp_sqr(zi);
      r.x = fp_mul(p.x, zi2);
      r.y = fp_mul(fp_mul(p.y, zi2), zi);
    }
    store_g1a(aff + q * 16, r);
    if (be || x0msgs) {
      uint32_t pw[16];
      g1_mont_to_be_words(r.x, r.y, pw);
      if (be) {
        uint4* d = reinterpret_cast<uint4*>(be + q * 64);
#pragma unroll
        for (int w = 0; w < 4; w++)
          d[w] = make_uint4(__builtin_bswap32(pw[4 * w]), __builtin_bswap32(pw[4 * w + 1]),
                            __builtin_bswap32(pw[4 * w + 2]), __builtin_bswap32(pw[4 * w + 3]));
      }
      // the x0 prefix's hex record of this point (H'_r of proof g / per)
      if (x0msgs) {
        const size_t g = g0 + (size_t)j * 64;
        x0_put_record(x0msgs + (g / per) * x0_var_bytes(per), (uint32_t)(g % per), pw);
      }
    }
  }
}

// --------------------------------------------------------- x0 transcript
// The x0 message DER(SEQUENCE{OCTET(Arr(H'_0..H'_{n-1}, G_0..G_{n-1}, Q, com)),
// OCTET("||"), OCTET(Zb(ip))}) + SHA-256 padding (ipa.go:200-213) as 16-bit
// units (2 hex chars, "||", DER bytes, padding; first byte in the low half).
struct X0Src {
  const uint8_t* hp;     // this proof's n+1 canonical BE points (H'..., com)
  const uint16_t* cst;   // hex(G_0) "||" ... hex(Q) "||"
  const uint32_t* ip;    // Zb(ip): canonical LE limbs
  uint32_t A, len, end;  // array length, message length, padded length (bytes)
  int n;
};
FTS_DEV uint32_t x0_unit(const X0Src& m, uint32_t u) {
  const uint32_t pos = 2u * u;
  if (pos < 8) {  // 30 82 L L 04 82 A A
    const uint32_t L = m.A + 42u;
    return pos == 0 ? 0x8230u : pos == 2 ? ((L >> 8) | ((L & 0xffu) << 8)) : pos == 4 ? 0x8204u
                                                                           : ((m.A >> 8) | ((m.A & 0xffu) << 8));
  }
  uint32_t off = pos - 8u;
  if (off < m.A) {
    const uint32_t r = off / 130u, o = off - 130u * r;
    if (r >= (uint32_t)m.n && r <= 2u * m.n) return m.cst[(130u * (r - m.n) + o) >> 1];
    if (o == 128u) return 0x7c7cu;
    return hex2(m.hp[(r < (uint32_t)m.n ? r : (uint32_t)m.n) * 64u + (o >> 1)]);
  }
  off -= m.A;
  if (off < 38u) {  // 04 02 "||" 04 20 Zb(ip)
    if (off < 6u) return off == 0 ? 0x0204u : off == 2 ? 0x7c7cu : 0x2004u;
    const uint32_t k = off - 6u;  // even byte index into Zb(ip)
    const uint32_t wd = m.ip[7 - (k >> 2)];
    return (k & 2u) ? (((wd >> 8) & 0xffu) | ((wd & 0xffu) << 8)) : ((wd >> 24) | (((wd >> 16) & 0xffu) << 8));
  }
  if (pos == m.len) return 0x0080u;
  if (pos >= m.end - 8u) {  // 64-bit big-endian bit length
    const uint64_t bits = (uint64_t)m.len * 8u;
    const uint32_t k = pos - (m.end - 8u);  // 0, 2, 4, 6
    const uint32_t b0 = (uint32_t)(bits >> (56 - 8 * k)) & 0xffu, b1 = (uint32_t)(bits >> (48 - 8 * k)) & 0xffu;
    return b0 | (b1 << 8);
  }
  return 0u;
}

// One wave per proof, X0_PPB proofs per block: the proof's variable message
// blocks (everything but the shared template blocks) are assembled in the
// wave's LDS region -- hex records of H'_i and com (one 16-byte quarter of a
// point per work item), the DER header, the constant bytes that share a block
// with variable ones, Zb(ip) and the SHA-256 padding -- then written to the
// compact slot with coalesced uint4 stores.  (One 256-thread block per proof,
// rounds 1-3, launched 4x the waves for the same work: at 81,920 proofs the
// launch's span beside the com chain was 5.8-6.8 ms.)
// LDS offset of message byte `pos` (outside the template blocks):
FTS_DEV uint32_t x0_lds_off(uint32_t pos, uint32_t cb0, uint32_t cb1) {
  return pos < 64u * cb0 ? pos : pos - 64u * (cb1 - cb0);
}
// part: 2 = every variable block; 0 = the blocks before the shared template
// (header, H'_0..H'_{n-1}: available right after their normalisation); 1 = the
// blocks after it (com, DER tail, Zb(ip), padding).  Parts 0 and 1 write
// disjoint byte ranges of the proof's slot.
constexpr int X0_PPB = 4;
__global__ void __launch_bounds__(64 * X0_PPB) k_rp_x0_build(int B, int n, const int32_t* __restrict__ status,
                                                            const uint8_t* __restrict__ hp_be,
                                                            const uint8_t* __restrict__ x0_const,
                                                            const uint32_t* __restrict__ sc, uint8_t* __restrict__ msgs,
                                                            int part) {
  wave_prio<PS_X0TAIL>();
  extern __shared__ uint4 x0_lds[];
  const uint32_t A = x0_array_len(n), len = x0_msg_len(n), end = x0_slot_bytes(n);
  const uint32_t cb0 = x0_cb0(n), cb1 = x0_cb1(n), var = x0_var_bytes(n);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * X0_PPB + wv;
  const bool live = b < B && status[b] == 0;  // uniform per wave
  // part 1 assembles only bytes >= 64 cb0 (its LDS region starts there)
  const uint32_t lbase = part == 1 ? 64u * cb0 : 0u;
  uint4* L4 = x0_lds + (size_t)wv * ((var - lbase) / 16u);
  uint8_t* Lb = reinterpret_cast<uint8_t*>(L4) - lbase;
  const uint32_t c_off = x0_const_off(n), c_end = x0_const_end(n);
  const uint8_t* hp = hp_be + (size_t)b * (n + 1) * 64;
  // hex records: H'_0..H'_{n-1} (records 0..n-1) and com (record 2n+1, no "||")
  const int r_lo = part == 1 ? n : 0, r_hi = part == 0 ? n : n + 1;  // records of this part
  for (int it = lane + 4 * r_lo; live && it < r_hi * 4; it += 64) {
    const int r = it >> 2, q = it & 3;
    const uint4 v = *reinterpret_cast<const uint4*>(hp + r * 64 + q * 16);
    const uint32_t rec = r < n ? (uint32_t)r : 2u * n + 1u;
    uint16_t* d = reinterpret_cast<uint16_t*>(Lb + x0_lds_off(8u + 130u * rec + 32u * q, cb0, cb1));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; j++) d[j] = hex2((w[j >> 2] >> (8 * (j & 3))) & 0xffu);
    if (q == 3 && r < n) d[16] = 0x7c7cu;
  }
  // header, constant bytes in variable blocks, trailer (DER tail, Zb(ip), padding, length)
  const uint32_t* ip = sc + ((size_t)(live ? b : 0) * RP_NSC + RP_SC_IP) * 8;
  const uint32_t t0 = 8u + A;
  auto put = [&](uint32_t pos) {
    uint32_t v;
    if (pos < 8u) {  // 30 82 L L 04 82 A A
      const uint32_t L = A + 42u;
      const uint8_t h[8] = {0x30, 0x82, (uint8_t)(L >> 8), (uint8_t)L, 0x04, 0x82, (uint8_t)(A >> 8), (uint8_t)A};
      v = h[pos];
    } else if (pos >= c_off && pos < c_end) {
      v = x0_const[pos - c_off];
    } else if (pos < t0 + 6u) {  // 04 02 "||" 04 20
      const uint8_t h[6] = {0x04, 0x02, 0x7c, 0x7c, 0x04, 0x20};
      v = h[pos - t0];
    } else if (pos < len) {  // Zb(ip): big-endian bytes of the canonical LE limbs
      const uint32_t k = pos - t0 - 6u;
      v = (ip[7 - (k >> 2)] >> (24 - 8 * (k & 3u))) & 0xffu;
    } else if (pos == len) {
      v = 0x80u;
    } else if (pos >= end - 8u) {
      v = (uint32_t)(((uint64_t)len * 8u) >> (8 * (end - 1u - pos))) & 0xffu;
    } else {
      v = 0u;
    }
    Lb[x0_lds_off(pos, cb0, cb1)] = (uint8_t)v;
  };
  const uint32_t nh = 8u, nc0 = 64u * cb0 - c_off, nc1 = c_end - 64u * cb1, nt = end - t0;
  // part 0: header + constants before the template; part 1: constants after it + trailer
  const uint32_t i_lo = part == 1 ? nh + nc0 : 0u, i_hi = part == 0 ? nh + nc0 : nh + nc0 + nc1 + nt;
  for (uint32_t it = lane + i_lo; live && it < i_hi; it += 64) {
    uint32_t pos;
    if (it < nh) pos = it;
    else if (it < nh + nc0) pos = c_off + (it - nh);
    else if (it < nh + nc0 + nc1) pos = 64u * cb1 + (it - nh - nc0);
    else pos = t0 + (it - nh - nc0 - nc1);
    put(pos);
  }
  __syncthreads();
  if (!live) return;
  uint4* dst = reinterpret_cast<uint4*>(msgs + (size_t)b * var);
  const uint32_t c_lo = part == 1 ? 4u * cb0 : 0u, c_hi = part == 0 ? 4u * cb0 : var / 16u;
  for (uint32_t c = lane + c_lo; c < c_hi; c += 64) dst[c] = L4[c - lbase / 16u];
}
// LDS bytes per proof of a part: part 1 assembles only the blocks after the template
inline uint32_t x0_part_lds_base(int n, int part) { return part == 1 ? 64u * x0_cb0(n) : 0u; }
inline size_t x0_build_lds(int n, int part = 2) {
  return (size_t)X0_PPB * (x0_var_bytes(n) - x0_part_lds_base(n, part));
}
inline unsigned x0_build_grid(int B) { return (unsigned)((B + X0_PPB - 1) / X0_PPB); }

// The bytes of part 0 of the x0 message that are not H' records (the DER header
// and the constant bytes sharing block cb0 - 1 with the last record), lane per
// proof; the records themselves are written by k_rp_normalize (x0msgs) as it
// normalises H' (round 5: a separate LDS-assembled build of part 0 waited for CU
// slots beside the com chain, and the x0 prefix it feeds became the pass's
// critical path, 0.4 -> 5.2 ms)
__global__ void __launch_bounds__(256) k_rp_x0_hdr(int B, int n, const int32_t* __restrict__ status,
                                                   const uint8_t* __restrict__ x0_const, uint8_t* __restrict__ msgs) {
  wave_prio<PS_NORM>();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  uint8_t* msg = msgs + (size_t)b * x0_var_bytes(n);
  const uint32_t A = x0_array_len(n), L = A + 42u;
  const uint8_t h[8] = {0x30, 0x82, (uint8_t)(L >> 8), (uint8_t)L, 0x04, 0x82, (uint8_t)(A >> 8), (uint8_t)A};
#pragma unroll
  for (int i = 0; i < 8; i++) msg[i] = h[i];
  const uint32_t c_off = x0_const_off(n), c_end = 64u * x0_cb0(n);
  for (uint32_t pos = c_off; pos < c_end; pos++) msg[pos] = x0_const[pos - c_off];
}

// SHA-256 over message blocks [b0, b1) of each proof's x0 message: b0 == 0
// starts from the initial state, else from mid[b]; b1 == every block finishes
// (x0 = HashToZr -> ch), else the state is left in mid[b].  The whole hash
// (0, all) or its prefix (0, cb1: H' records + the shared template, started
// while com is still being computed) and suffix (cb1, all).
__global__ void __launch_bounds__(256) k_rp_x0_hash(int B, int n, int k, const int32_t* __restrict__ status,
                                                   const uint8_t* __restrict__ msgs, const uint8_t* __restrict__ tmpl,
                                                   uint32_t b0, uint32_t b1, uint32_t* __restrict__ mid,
                                                   uint32_t* __restrict__ ch) {
  // the suffix is the pass's short tail; the prefix runs beside the com chain
  if (b0 != 0)
    wave_prio<PS_X0TAIL>();
  else
    wave_prio<PS_X0PRE>();
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || status[b] != 0) return;
  const uint32_t cb0 = x0_cb0(n), cb1 = x0_cb1(n), nb = sha_blocks(x0_msg_len(n));
  const uint32_t hi = b1 < nb ? b1 : nb;
  const uint4* own = reinterpret_cast<const uint4*>(msgs + (size_t)b * x0_var_bytes(n));
  uint32_t st[8];
  if (b0 == 0) {
    sha256_init(st);
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = mid[(size_t)b * 8 + i];
  }
  // one block ahead: the next block's 64 bytes are loaded before this block's
  // 64 rounds, so the load's latency (L2 / HBM, ~1 us under load) is hidden
  // behind them instead of exposed once per block
  const uint4* shared = reinterpret_cast<const uint4*>(tmpl);
  auto block_ptr = [&](uint32_t blk) {
    return blk < cb0 ? own + 4u * blk : blk < cb1 ? shared + 4u * (blk - cb0) : own + 4u * (blk - (cb1 - cb0));
  };
  uint4 nx[4];
  if (b0 < hi) {
    const uint4* m = block_ptr(b0);
#pragma unroll
    for (int i = 0; i < 4; i++) nx[i] = m[i];
  }
  for (uint32_t blk = b0; blk < hi; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      w[4 * i + 0] = __builtin_bswap32(nx[i].x);
      w[4 * i + 1] = __builtin_bswap32(nx[i].y);
      w[4 * i + 2] = __builtin_bswap32(nx[i].z);
      w[4 * i + 3] = __builtin_bswap32(nx[i].w);
    }
    if (blk + 1 < hi) {
      const uint4* m = block_ptr(blk + 1);
#pragma unroll
      for (int i = 0; i < 4; i++) nx[i] = m[i];
    }
    sha256_compress(st, w);
  }
  if (hi < nb) {
#pragma unroll
    for (int i = 0; i < 8; i++) mid[(size_t)b * 8 + i] = st[i];
    return;
  }
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

// sel != nullptr: lanes cover the B proofs sel[0 .. B) (the group test's failing
// proofs) instead of proofs 0 .. B
__global__ void __launch_bounds__(64) k_rp_terms_fixed(int B, int n, int k, const int32_t* __restrict__ sel,
                                                       const int32_t* __restrict__ status,
                                                       const int32_t* __restrict__ ipa_flag,
                                                       const uint32_t* __restrict__ sc, const uint32_t* __restrict__ ch,
                                                       const uint32_t* __restrict__ tables, uint32_t* __restrict__ terms) {
  const int nf = 3 + 2 * n;  // 2 (E1) + 2n + 1 (E2)
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nf) return;
  int b = gid / nf, t = gid % nf;
  if (sel) b = sel[b];
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
  G1J r = nl_fb_mul(tables + (size_t)base * FB_WORDS_PER_BASE, fr_canon(s));
  store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, r);
}

// the same terms with COOP_G lanes per product (device/coop.hpp): 12 products
// per wave, each doubling 3 product levels instead of 7 and each addition 5
// instead of 16, tables of 1..8 P and 1..8 phi(P) in LDS.  For a few
// thousand products on an otherwise idle GPU (the group test's last stage
// after a small failing group set) the chain latency, not the work, bounds the
// stage; the results are the same Jacobian triples as glv_mul's.
constexpr int TV_GPW = 64 / COOP_G;  // products per wave
constexpr size_t TV_COOP_MAX = 16384; // products up to which the cooperative form runs (~1,400 waves)
__global__ void __launch_bounds__(64) k_rp_terms_var_coop(int B, int n, int k, const int32_t* __restrict__ sel,
                                                          const int32_t* __restrict__ status,
                                                          const int32_t* __restrict__ ipa_flag,
                                                          const uint32_t* __restrict__ pts,
                                                          const uint32_t* __restrict__ ch,
                                                          uint32_t* __restrict__ terms) {
  __shared__ uint32_t T[TV_GPW][16][24];
  const int nv = 3 + 2 * k;
  const int lt = threadIdx.x, gi = lt / COOP_G, role = lt % COOP_G, base = gi * COOP_G;
  if (gi >= TV_GPW) return;  // lanes 60..63: no group
  const int item = blockIdx.x * TV_GPW + gi;
  if (item >= B * nv) return;  // whole groups leave together
  int b = item / nv;
  const int t = item % nv;
  if (sel) b = sel[b];
  if (status[b] != 0) return;
  const uint32_t* C = ch + (size_t)b * rp_nch(k) * 8;
  const uint32_t* Pt = pts + (size_t)b * rp_npts(k) * 16;
  int slot, pt;
  Fr s;
  if (t < 3) {
    slot = 2 + t;
    const int chi = t == 0 ? CH_X : (t == 1 ? CH_X2 : CH_Z2);
    load_f(C + chi * 8, s);
    pt = t == 0 ? RP_PT_T1 : (t == 1 ? RP_PT_T2 : RP_PT_V);
  } else {
    slot = 6 + 2 * n + (t - 3);
    if (ipa_flag[b] != 0) {
      if (role == 0) store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, g1j_identity());
      return;
    }
    int j = t - 3;
    if (j < k) {
      load_f(C + (CH_XJ + j) * 8, s);
      pt = RP_PT_L + j;
    } else {
      j -= k;
      load_f(C + (CH_XJ + k + j) * 8, s);
      pt = RP_PT_L + k + j;
    }
    s = fr_sqr(s);
  }
  const G1A pa = load_g1a(Pt + pt * 16);
  G1J acc = g1j_identity();
  if (!g1a_is_identity(pa)) {
    const Scalar sk = fr_canon(f_neg(s));
    uint32_t k1[4], k2[4], s1, s2;
    glv_decompose(sk.v, k1, s1, k2, s2);
    G1J P = g1j_from_affine(pa), Q = P;
    Q.x = fp_mul(Q.x, glv_beta());
    if (s1) P.y = f_neg(P.y);
    if (s2) Q.y = f_neg(Q.y);
    uint32_t(*tb)[24] = T[gi];
    // 1..8 P, 1..8 Q (every lane of the group writes the same words)
    for (int h = 0; h < 2; h++) {
      const G1J t0 = h ? Q : P;
      G1J cur = t0;
      store_g1j(tb[8 * h], cur);
      cur = coop_dbl(t0, role, base);
      store_g1j(tb[8 * h + 1], cur);
      for (int e = 2; e < 8; e++) {
        coop_add(cur, t0, role, base);
        store_g1j(tb[8 * h + e], cur);
      }
    }
    const uint32_t ca = recode_carries(k1), cb = recode_carries(k2);
    for (int w = 31; w >= 0; w--) {
      const int da = window_digit(k1, ca, w), db = window_digit(k2, cb, w);
      if (w != 31)
        for (int r = 0; r < 4; r++) acc = coop_dbl(acc, role, base);
      if (da != 0) {
        G1J q = load_g1j(tb[(da < 0 ? -da : da) - 1]);
        if (da < 0) q.y = f_neg(q.y);
        coop_add(acc, q, role, base);
      }
      if (db != 0) {
        G1J q = load_g1j(tb[8 + (db < 0 ? -db : db) - 1]);
        if (db < 0) q.y = f_neg(q.y);
        coop_add(acc, q, role, base);
      }
    }
  }
  if (role == 0) store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, acc);
}

__global__ void __launch_bounds__(64) k_rp_terms_var(int B, int n, int k, const int32_t* __restrict__ sel,
                                                     const int32_t* __restrict__ status,
                                                     const int32_t* __restrict__ ipa_flag,
                                                     const uint32_t* __restrict__ pts, const uint32_t* __restrict__ ch,
                                                     uint32_t* __restrict__ terms, uint32_t* __restrict__ scratch) {
  const int nv = 3 + 2 * k;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * nv) return;
  int b = gid / nv, t = gid % nv;
  if (sel) b = sel[b];
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
  // all variable terms enter with a minus sign; GLV + joint Straus (124 doublings)
  G1J r = glv_mul(load_g1a(Pt + pt * 16), fr_canon(f_neg(s)), scratch, (size_t)B * nv, (size_t)gid);
  store_g1j(terms + ((size_t)b * rp_nterms(n, k) + slot) * 24, r);
}

// ------------------------------------------------------------------ check
// CK_LANES lanes per proof: E1 (5 terms) on lane 0; E2 (-com + the 1 + 2n + 2k
// other terms, 81 at n = 64) as CK_LANES partial sums + a 4-level LDS tree
// instead of one chain of ~80 additions.  Group addition is associative, so the
// verdict (identity or not) is the same.
constexpr int CK_LANES = 16, CK_PROOFS = 16;
__global__ void __launch_bounds__(CK_LANES * CK_PROOFS) k_rp_check(int B, int n, int k, const int32_t* __restrict__ sel,
                                                                   int32_t* __restrict__ status,
                                                                   const int32_t* __restrict__ ipa_flag,
                                                                   const uint32_t* __restrict__ terms,
                                                                   const uint32_t* __restrict__ hpa) {
  __shared__ uint32_t sh[CK_LANES * CK_PROOFS * 24];
  __shared__ int e1_ok[CK_PROOFS];
  const int l = threadIdx.x % CK_LANES, pl = threadIdx.x / CK_LANES;
  const int bi = blockIdx.x * CK_PROOFS + pl;
  int b = bi < B ? (sel ? sel[bi] : bi) : -1;
  const bool live = b >= 0 && status[b] == 0;
  const uint32_t* T = live ? terms + (size_t)b * rp_nterms(n, k) * 24 : terms;
  if (live && l == 0) {
    G1J e1 = load_g1j(T);
    for (int t = 1; t < 5; t++) e1 = nl_add_mem(e1, T + t * 24, 0);
    e1_ok[pl] = g1j_is_identity(e1);
  }
  G1J acc = g1j_identity();
  if (live) {
    if (l == 0) acc = g1j_from_affine(g1a_neg(load_g1a(hpa + ((size_t)b * (n + 1) + n) * 16)));
    for (int t = 5 + l; t < rp_nterms(n, k); t += CK_LANES) add_inl(acc, load_g1j(T + t * 24));
  }
  uint32_t* S = sh + (size_t)pl * CK_LANES * 24;
  store_g1j(S + l * 24, acc);
  __syncthreads();
  for (int half = CK_LANES / 2; half >= 1; half >>= 1) {
    if (live && l < half) add_inl(acc, load_g1j(S + (l + half) * 24));
    __syncthreads();
    if (live && l < half) store_g1j(S + l * 24, acc);
    __syncthreads();
  }
  if (!live || l != 0) return;
  if (!e1_ok[pl]) {
    status[b] = FTS_E_RP_INVALID;
  } else if (ipa_flag[b] != 0) {
    status[b] = ipa_flag[b];
  } else {
    status[b] = g1j_is_identity(acc) ? FTS_OK : FTS_E_IPA_INVALID;
  }
}

// ------------------------------------------------------------ RLC batch check
// Sum_p rho_p E1_p + rho'_p E2_p == O  (SURVEY Appendix B).  Fixed bases get
// batch-summed scalars (column reduction), variable points go to one MSM.
// com never enters as a point: E2's -rho' com is expanded through its
// definition (bulletproof.go:477-492)
//   -rho' com = -rho' C - rho' x D - rho' z K + rho' delta P - rho' sum_i z^2 2^i y^-i H_i
// so the variable points are T1, T2, V, C, D, L_j, R_j (all decoded from the
// proof) and the K, P, H_i terms join the fixed-base columns.  The check then
// depends only on the challenges (not on H'_i, com or x0, except column Q =
// rho'(ab - ip) x0 Q): the MSM runs beside the exact per-proof phase.

// full-width weight: 256 random bits reduced mod r (Montgomery form).  Full
// width keeps every MSM window's digits uniform (a 128-bit weight would put
// all proofs' top-digit entries into a few buckets of one window).
FTS_DEV Fr fr_from_u256(const uint32_t w[8]) {
  uint32_t be[8];
#pragma unroll
  for (int i = 0; i < 8; i++) be[i] = w[7 - i];
  return f_to_mont(digest_to_fr(be));
}

__global__ void __launch_bounds__(256) k_rlc_prep(int B, int n, int k, const int32_t* __restrict__ status,
                                                 const int32_t* __restrict__ excl,
                                                 const int32_t* __restrict__ ipa_flag, const uint32_t* __restrict__ sc,
                                                 const uint32_t* __restrict__ ch, const uint32_t* __restrict__ key,
                                                 uint32_t* __restrict__ msc, uint32_t* __restrict__ coef, int idxw = 0) {
  wave_prio<PS_SORT>();
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int npts = rp_npts(k);
  uint32_t* M = msc + (size_t)b * npts * 8;
  uint32_t* K = coef + (size_t)b * RLC_NCOEF * 8;
  const bool e1 = status[b] == 0 && !(excl && excl[b]);
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
  if (idxw) {  // the single-fault locator's sum: both weights of proof b times b + 1
    const uint32_t w[8] = {(uint32_t)b + 1u, 0, 0, 0, 0, 0, 0, 0};
    const Fr wb = fr_from_canon(w);
    rho = fr_mul(rho, wb);
    rho2 = fr_mul(rho2, wb);
  }
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
  Fr a = fr_from_canon(S + RP_SC_A * 8), bb = fr_from_canon(S + RP_SC_B * 8), z;
  load_f(C + CH_Z * 8, z);
  put(RP_PT_C, rho2);
  put(RP_PT_D, fr_mul(rho2, x));
  for (int j = 0; j < k; j++) {
    Fr xj, xji;
    load_f(C + (CH_XJ + j) * 8, xj);
    load_f(C + (CH_XJ + k + j) * 8, xji);
    put(RP_PT_L + j, fr_mul(rho2, fr_sqr(xj)));
    put(RP_PT_L + k + j, fr_mul(rho2, fr_sqr(xji)));
  }
  store_f(K + 2 * 8, fr_mul(rho2, f_sub(fr_mul(a, bb), ip)));
  store_f(K + 3 * 8, fr_mul(rho2, a));
  store_f(K + 4 * 8, fr_mul(rho2, bb));
  store_f(K + 5 * 8, rho2);
  store_f(K + 6 * 8, f_neg(fr_mul(rho2, z)));
  store_f(K + 7 * 8, fr_mul(rho2, fr_from_canon(S + RP_SC_DELTA * 8)));
}

// proof b's scalar in RLC column col (layout: rlc_ncols), Montgomery form.
// s_i, y^-i and z^2 2^i y^-i come precomputed, i-major, from k_rp_powers.
FTS_DEV Fr rlc_col_value(int col, int b, int B, int n, int k, const uint32_t* __restrict__ ch,
                         const uint32_t* __restrict__ coef, const uint32_t* __restrict__ ypow,
                         const uint32_t* __restrict__ svec, const uint32_t* __restrict__ zvec) {
  const uint32_t* K = coef + (size_t)b * RLC_NCOEF * 8;
  Fr v;
  if (col < 2) {
    load_f(K + col * 8, v);
  } else if (col < 2 + n) {  // rho' a s_i
    Fr ra;
    load_f(K + 3 * 8, ra);
    if (!f_is_zero(ra)) {
      Fr sv;
      load_f(svec + ((size_t)(col - 2) * B + b) * 8, sv);
      v = fr_mul(ra, sv);
    } else {
      v = ra;
    }
  } else if (col < 2 + 2 * n) {  // rho' b s_i^-1 y^-i - rho' z^2 2^i y^-i
    const int i = col - 2 - n;
    Fr r2;
    load_f(K + 5 * 8, r2);
    if (!f_is_zero(r2)) {
      Fr rb, sv, yp, zv;
      load_f(K + 4 * 8, rb);
      load_f(svec + ((size_t)(n - 1 - i) * B + b) * 8, sv);
      load_f(ypow + ((size_t)i * B + b) * 8, yp);
      load_f(zvec + ((size_t)i * B + b) * 8, zv);
      v = f_sub(fr_mul(fr_mul(rb, sv), yp), fr_mul(r2, zv));
    } else {
      v = r2;
    }
  } else if (col < 2 * n + 4) {  // -rho' z (K), rho' delta (P)
    load_f(K + (col - 2 * n + 4) * 8, v);
  } else {  // rho'(ab - ip) x0 (Q)
    load_f(K + 2 * 8, v);
    if (!f_is_zero(v)) {
      Fr x0;
      load_f(ch + ((size_t)b * rp_nch(k) + CH_X0) * 8, x0);
      v = fr_mul(v, x0);
    }
  }
  return v;
}

// one block per (column, group), columns col0 + blockIdx.x.  The batch check
// has one group of all B proofs; the group test has G groups of gs proof slots
// (sel[g gs + j], -1 = empty) -> colsum[g][col]
__global__ void __launch_bounds__(256) k_rlc_columns(int B, int n, int k, int gs, int col0,
                                                     const int32_t* __restrict__ sel, const uint32_t* __restrict__ ch,
                                                     const uint32_t* __restrict__ coef, const uint32_t* __restrict__ ypow,
                                                     const uint32_t* __restrict__ svec,
                                                     const uint32_t* __restrict__ zvec, uint32_t* __restrict__ colsum) {
  wave_prio<PS_COLS>();
  __shared__ uint32_t sh[256 * 8];
  const int col = col0 + blockIdx.x, grp = blockIdx.y, t = threadIdx.x, nt = blockDim.x;  // nt: 64 or 256
  Fr acc = f_zero<FrP>();
  for (int j = t; j < gs; j += nt) {
    const int b = sel ? sel[(size_t)grp * gs + j] : grp * gs + j;
    if (b < 0 || b >= B) continue;
    acc = f_add(acc, rlc_col_value(col, b, B, n, k, ch, coef, ypow, svec, zvec));
  }
  store_f(sh + t * 8, acc);
  __syncthreads();
  for (int half = nt / 2; half >= 1; half >>= 1) {
    if (t < half) {
      Fr o;
      load_f(sh + (t + half) * 8, o);
      acc = f_add(acc, o);
      store_f(sh + t * 8, acc);
    }
    __syncthreads();
  }
  if (t == 0) store_f(colsum + ((size_t)grp * rlc_ncols(n) + col) * 8, f_from_mont(acc));
}

// column Q over the whole pass, second stage: sum the RQ_PARTS partial sums that
// k_rlc_columns wrote per slice of proofs (rows 1..RQ_PARTS of colsum) into row 0.
// (One block over all B proofs took 0.76 ms at 81,920 on the x0-dependent tail.)
constexpr int RQ_PARTS = 64;
// (block x sums column col + x: the locator splits every column this way)
__global__ void __launch_bounds__(64) k_rlc_qsum(int ncols, int col0, uint32_t* __restrict__ colsum) {
  wave_prio<PS_FIN>();
  __shared__ uint32_t sh[RQ_PARTS * 8];
  const int t = threadIdx.x, col = col0 + blockIdx.x;
  Fr v;  // plain residues: the sum is the same in either representation
  load_f(colsum + ((size_t)(1 + t) * ncols + col) * 8, v);
  store_f(sh + t * 8, v);
  __syncthreads();
  for (int half = RQ_PARTS / 2; half >= 1; half >>= 1) {
    if (t < half) {
      Fr o;
      load_f(sh + (t + half) * 8, o);
      v = f_add(v, o);
      store_f(sh + t * 8, v);
    }
    __syncthreads();
  }
  if (t == 0) store_f(colsum + (size_t)col * 8, v);
}

FTS_DEV int rlc_col_base(int n, int col) {
  return col == 0 ? tb_G(n) : col == 1 ? tb_H(n) : col < 2 * n + 2 ? col - 2 : col == 2 * n + 2 ? tb_K(n)
         : col == 2 * n + 3 ? tb_P(n) : tb_Q(n);
}

// fixed-base product of each column sum, FB_NW lanes per (group, column):
// lane w looks up its window's entry, then an LDS tree of log2(FB_NW) full
// additions (latency: 4 additions instead of a chain of 16)
constexpr int RF_ITEMS = 16;
static_assert(FB_NW == 16, "one lane per 16-bit window");
__global__ void __launch_bounds__(RF_ITEMS * FB_NW) k_rlc_fixed(int n, int G, int col0, int ncl,
                                                               const uint32_t* __restrict__ colsum,
                                                               const uint32_t* __restrict__ tables,
                                                               uint32_t* __restrict__ out) {
  wave_prio<PS_COLS>();
  __shared__ uint32_t sh[RF_ITEMS * FB_NW * 24];
  const int w = threadIdx.x % FB_NW, it = blockIdx.x * RF_ITEMS + threadIdx.x / FB_NW;
  const bool live = it < G * ncl;
  const int NC = rlc_ncols(n), grp = live ? it / ncl : 0, col = col0 + (live ? it % ncl : 0);
  G1J acc = g1j_identity();
  if (live) {
    uint32_t s[8];
#pragma unroll
    for (int q = 0; q < 8; q++) s[q] = colsum[((size_t)grp * NC + col) * 8 + q];
    int carry = 0, d = 0;
    for (int q = 0; q <= w; q++) d = fb_next_digit(s, carry);
    if (d != 0)
      acc = g1j_from_affine(fb_entry(tables + (size_t)rlc_col_base(n, col) * FB_WORDS_PER_BASE, w, d));
  }
  uint32_t* S = sh + (size_t)(threadIdx.x - w) * 24;
  store_g1j(S + w * 24, acc);
  __syncthreads();
  for (int half = FB_NW / 2; half >= 1; half >>= 1) {
    if (live && w < half) add_inl(acc, load_g1j(S + (w + half) * 24));
    __syncthreads();
    if (live && w < half) store_g1j(S + w * 24, acc);
    __syncthreads();
  }
  if (live && w == 0) store_g1j(out + ((size_t)grp * NC + col) * 24, acc);
}

// Group test over many small groups (gs <= GT_SMALL_MAX proof slots): lane per
// (chunk of GT_CC columns, group), chunk-major so a wave's lanes read the same
// columns' tables: the group's column scalars (sum over its proof slots, as
// k_rlc_columns) and their fixed-base products, 16 mixed additions each from
// the 16-bit tables, accumulated in the lane -> gfix[grp][chunk] (Jacobian).
// (The per-column LDS-tree form above is for a few large groups: with 10^4
// groups of 8 it ran at ~20 % of the MAD peak.)
__global__ void __launch_bounds__(256) k_rlc_group_cols_small(int B, int n, int k, int G, int gs,
                                                              const int32_t* __restrict__ sel,
                                                              const uint32_t* __restrict__ ch,
                                                              const uint32_t* __restrict__ coef,
                                                              const uint32_t* __restrict__ ypow,
                                                              const uint32_t* __restrict__ svec,
                                                              const uint32_t* __restrict__ zvec,
                                                              const uint32_t* __restrict__ tables,
                                                              uint32_t* __restrict__ gfix) {
  const int NC = rlc_ncols(n), nch = gt_nchunks(n);
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)G * nch) return;
  const int chk = (int)(gid / G), grp = (int)(gid % G);
  G1J acc = g1j_identity();
  const int c1 = min(NC, (chk + 1) * GT_CC);
  for (int col = chk * GT_CC; col < c1; col++) {
    Fr v = f_zero<FrP>();
    for (int j = 0; j < gs; j++) {
      const int b = sel[(size_t)grp * gs + j];
      if (b < 0 || b >= B) continue;
      v = f_add(v, rlc_col_value(col, b, B, n, k, ch, coef, ypow, svec, zvec));
    }
    if (f_is_zero(v)) continue;
    const Fr cv = f_from_mont(v);
    Scalar sk;
#pragma unroll
    for (int q = 0; q < 8; q++) sk.v[q] = cv.v[q];
    fb_mul_acc(acc, tables + (size_t)rlc_col_base(n, col) * FB_WORDS_PER_BASE, sk);
  }
  store_g1j(gfix + ((size_t)grp * nch + chk) * 24, acc);
}

// batch verdict: flag = 1 if the combination is the identity; on success the
// deferred IPA structural verdicts become final (their E1 held)
// (msm_out + addend: the Q column's product, computed after x0)
__global__ void __launch_bounds__(64) k_rlc_finalize(int B, const uint32_t* __restrict__ msm_out,
                                                     const uint32_t* __restrict__ addend,
                                                     const int32_t* __restrict__ excl,
                                                     int32_t* __restrict__ status, const int32_t* __restrict__ ipa_flag,
                                                     int32_t* __restrict__ flag) {
  wave_prio<PS_FIN>();
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && excl && excl[b] && status[b] == 0) status[b] = FTS_E_NOT_RUN;
  G1J e = load_g1j(msm_out);
  add_inl(e, load_g1j(addend));
  const bool pass = g1j_is_identity(e);
  if (b == 0) *flag = pass ? 1 : 0;
  if (b < B && pass && status[b] == 0 && ipa_flag[b] != 0) status[b] = ipa_flag[b];
}

// Single-fault locator (round 5).  When the batch combination S = sum_b rho_b E_b
// (E_b: proof b's final equations, rho_b its weights) is not the identity, the
// same combination with weights (b + 1) rho_b gives S' = sum_b (b + 1) rho_b E_b.
// If exactly one proof i is bad, S' = (i + 1) S; conversely S' = (j + 1) S means
// sum_b (b - j) rho_b E_b = 0, which for two or more bad proofs (or one bad proof
// other than j) holds only with probability ~1/r over the fresh random weights --
// the same soundness as the batch check itself.  Lane j tests S' == (j + 1) S.
__global__ void __launch_bounds__(64) k_rlc_total(const uint32_t* __restrict__ msm_out,
                                                  const uint32_t* __restrict__ addend, uint32_t* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  G1J e = load_g1j(msm_out);
  add_inl(e, load_g1j(addend));
  store_g1j(out, e);
}
__global__ void __launch_bounds__(64) k_rlc_locate(int B, const uint32_t* __restrict__ total,
                                                   const uint32_t* __restrict__ msm_out,
                                                   const uint32_t* __restrict__ addend, int32_t* __restrict__ loc) {
  wave_prio<PS_FIN>();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  G1J t = load_g1j(msm_out);
  add_inl(t, load_g1j(addend));
  const G1J S = load_g1j(total);
  const uint32_t m = (uint32_t)j + 1u;
  G1J P = g1j_identity();
  for (int bit = 31 - __builtin_clz(m); bit >= 0; bit--) {
    P = g1j_dbl(P);
    if ((m >> bit) & 1u) P = g1j_add(P, S);
  }
  if (g1j_eq(P, t)) loc[0] = j;
}
// after the locator: every proof but `skip` whose deferred IPA structural verdict is
// pending takes it (the combination of the others closed, as in k_rlc_finalize)
__global__ void __launch_bounds__(256) k_rlc_accept_except(int B, int skip, int32_t* __restrict__ status,
                                                           const int32_t* __restrict__ ipa_flag) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && b != skip && status[b] == 0 && ipa_flag[b] != 0) status[b] = ipa_flag[b];
}

// group test verdicts: lane per proof slot j of the selection (group j / gs);
// a group whose partial combination is the identity accepts its proofs (their
// deferred IPA structural verdicts become final, as in k_rlc_finalize), the
// proofs of the other groups are appended to `next` (the next round's list)
// the per-caller-batch combination (RlcDev::G > 1): slot j of group j / gs; group g
// closes when its MSM sum (x0-free columns included as extras) + column Q's product
// is the identity -> its proofs take their exact-phase verdicts, gflag[g] = 1; a
// failing group's proofs stay undecided (the group test runs over those batches only)
__global__ void __launch_bounds__(256) k_rlc_finalize_groups(int slots, int gs, int NC, const int32_t* __restrict__ sel,
                                                             const uint32_t* __restrict__ msm_out,
                                                             const uint32_t* __restrict__ qfix,
                                                             const int32_t* __restrict__ excl,
                                                             int32_t* __restrict__ status,
                                                             const int32_t* __restrict__ ipa_flag,
                                                             int32_t* __restrict__ gflag, int32_t* __restrict__ flag) {
  wave_prio<PS_FIN>();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= slots) return;
  const int b = sel[j], g = j / gs;
  if (b < 0) return;
  if (excl && excl[b] && status[b] == 0) status[b] = FTS_E_NOT_RUN;
  G1J e = load_g1j(msm_out + (size_t)g * 24);
  add_inl(e, load_g1j(qfix + ((size_t)g * NC + NC - 1) * 24));
  const bool pass = g1j_is_identity(e);
  if (j % gs == 0) {  // a group's first slot is a real proof (padding trails)
    gflag[g] = pass ? 1 : 0;
    if (!pass) *flag = 0;
  }
  if (pass && status[b] == 0 && ipa_flag[b] != 0) status[b] = ipa_flag[b];
}

__global__ void __launch_bounds__(256) k_rlc_group_final(int slots, int gs, const int32_t* __restrict__ sel,
                                                         const uint32_t* __restrict__ msm_out,
                                                         int32_t* __restrict__ status,
                                                         const int32_t* __restrict__ ipa_flag,
                                                         int32_t* __restrict__ next, uint32_t* __restrict__ next_count) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= slots) return;
  const int b = sel ? sel[j] : j;
  if (b < 0 || status[b] != 0) return;
  Fp z;
  load_fp(msm_out + (size_t)(j / gs) * 24 + 16, z);
  if (f_is_zero(z)) {
    if (ipa_flag[b] != 0) status[b] = ipa_flag[b];
  } else {
    next[atomicAdd(next_count, 1u)] = b;
  }
}

// ------------------------------------------------------------ host launch
#define FTS_LAUNCH(kern, nthreads, bs, stream, ...)                                   \
  do {                                                                                \
    size_t nt_ = (size_t)(nthreads);                                                  \
    if (nt_) hipLaunchKernelGGL(kern, dim3((unsigned)((nt_ + (bs)-1) / (bs))), dim3(bs), 0, stream, __VA_ARGS__); \
  } while (0)
static void launch_normalize(size_t total, int per, int stride, int first, const int32_t* status, const uint32_t* jac,
                             uint32_t* aff, uint8_t* be, hipStream_t s, uint8_t* x0msgs) {
  // lanes: one per E points, rounded to whole waves (E * 64 points per wave)
  if (total >= NORM_BIG)
    FTS_LAUNCH(k_rp_normalize<16>, (total + 16 * 64 - 1) / (16 * 64) * 64, NORM_BS, s, (int)total, per, stride, first,
               status, jac, aff, be, x0msgs);
  else
    FTS_LAUNCH(k_rp_normalize<4>, (total + 4 * 64 - 1) / (4 * 64) * 64, NORM_BS, s, (int)total, per, stride, first,
               status, jac, aff, be, x0msgs);
}




size_t rp_scratch_words(int B, int n, int k) {
  // per-proof fallback: 16-entry GLV lane tables of the 3 + 2k variable terms
  return std::max((size_t)B * (3 + 2 * k) * 16 * 24, (size_t)B * (HS_SCRATCH + 2 * ATAB_WORDS));
}
size_t rp_terms_words(int B, int n, int k) { return (size_t)B * rp_nterms(n, k) * 24; }

size_t fb_words_per_base() { return FB_WORDS_PER_BASE; }
// the per-proof bases' wide tables: 20-bit windows (13 per scalar, 436 MiB per base)
// or 22-bit (12, 1.5 GiB per base) where the device has the memory (fts_api.cpp)
size_t fbw_words_per_base(int wbits) { return wbits == 22 ? FbCfg<22>::WORDS_PER_BASE : FbWide::WORDS_PER_BASE; }
template <int W>
static size_t build_scratch_bytes(int nb) {
  using C = FbCfg<W>;
  const size_t nbw = (size_t)nb * C::NW;
  return nbw * 24 * 4 + nbw * (C::S + C::L) * 24 * 4 + nbw * C::E * 24 * 4;
}
size_t table_build_scratch_bytes(int nb) { return build_scratch_bytes<FB_W>(nb); }
size_t wide_build_scratch_bytes(int nb, int wbits) {
  return wbits == 22 ? build_scratch_bytes<22>(nb) : build_scratch_bytes<FBW_W>(nb);
}
// tables: nb * WORDS_PER_BASE words; scratch: build_scratch_bytes<W>(nb)
template <int W>
static void build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s) {
  using C = FbCfg<W>;
  const size_t nbw = (size_t)nb * C::NW;
  uint32_t* bw = scratch;
  uint32_t* small = bw + nbw * 24;
  uint32_t* large = small + nbw * C::S * 24;
  uint32_t* jac = large + nbw * C::L * 24;
  FTS_LAUNCH(kt_window_bases<W>, nbw, 64, s, bases, nb, bw);
  FTS_LAUNCH(kt_small_large<W>, nbw, 64, s, nb, bw, small, large);
  FTS_LAUNCH(kt_entries<W>, nbw * C::E, 64, s, nb, small, large, jac);
  const size_t tot = nbw * C::E;
  launch_normalize(tot, 1, 1, 0, (const int32_t*)nullptr, jac, tables, (uint8_t*)nullptr, s);
}
void launch_build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s) {
  build_tables<FB_W>(bases, nb, tables, scratch, s);
}
void launch_build_wide_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s,
                              int wbits) {
  if (wbits == 22) build_tables<22>(bases, nb, tables, scratch, s);
  else build_tables<FBW_W>(bases, nb, tables, scratch, s);
}

// ev_stage (optional): recorded on s after the counting sort (stage 1) or the bucket
// accumulation (stage 2)
void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, hipStream_t s_extra, Timeline* tl, hipEvent_t ev_stage = nullptr,
                int stage = 0);
void launch_msm_small(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra,
                      int nextra, hipStream_t s, Timeline* tl);
void launch_msm_sort(const MsmPlan& p, const uint32_t* scalars, hipStream_t s, Timeline* tl);
void launch_msm_reduce(const MsmPlan& p, const uint32_t* points, const uint32_t* extra, int nextra, uint32_t* scratch,
                       hipStream_t s, hipStream_t s_extra, Timeline* tl);

// Whole range-proof pipeline up to the batch verdict (flag): exact per-proof
// phase (everything that is hashed: challenges, H'_i, com, x0) and the
// random-linear-combination check of all final equations (one MSM).
// s = main stream (exact phase, then the x0-dependent tail), s2 = x*D beside
// the fixed-base products (latency path), s3 = the batch check's variable part
// (weights, x0-free columns, MSM), which needs only the challenges.
void launch_rp_batch(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, const uint32_t* wtables,
                     const uint8_t* x0_const, const uint8_t* x0_tmpl, hipStream_t s, hipStream_t s2, hipStream_t s3,
                     hipStream_t s4, Timeline* tl, int wbits) {
  // fixed-base products over the wide tables: 12 (20-bit) or 11 (22-bit) additions each
  const double cost_fbw = wbits == 22 ? 11.0 * COST_MADD : COST_FBW_FRESH;
  const int B = d.B, n = d.n, k = d.k, NC = rlc_ncols(n);
  if (!B) return;
  if (d.excl) (void)hipMemsetAsync(d.excl, 0, (size_t)B * 4, s);
  // 64-thread blocks for the elementwise head kernels: beside the previous pass's
  // fixed-base launch (64-thread blocks, the whole register file) a 256-thread block
  // waits for four wave slots of one CU to free at once (k_rp_decode 0.07 ms alone,
  // 1.15 ms there in a 20-batch burst, round 5)
  FTS_LAUNCH(k_rp_decode, B * rp_npts(k), 64, s, B, rp_npts(k), d.raw, d.pts, d.status);
  tl->mark("k_rp_decode", s, 0);
  FTS_LAUNCH(k_rp_hash_small, B * (2 + k), 64, s, B, n, k, d.raw, d.status, d.ch, d.small_msgs);
  tl->mark("k_rp_hash_small", s, 0);
  const int nhp = B * n;
  if (d.com_fixed) {
    // latency path: x*D on the side stream beside chal_fr and the fixed-base products
    tl->fork(s, s2);
    FTS_LAUNCH(k_rp_xd, 2 * B, g_lat_bs, s2, B, n, k, d.status, d.pts, d.small_msgs, d.scratch + (size_t)B * (k + 1) * 8,
               d.terms, com_fx_slots(n), n + 2);
    tl->mark("k_rp_xd", s2, (double)B * 2 * COST_VB128);
  }
  const int lbs = d.com_fixed ? g_lat_bs : g_work_bs.load(std::memory_order_relaxed);
  FTS_LAUNCH(k_rp_chal_fr, B, lbs, s, B, n, k, d.status, d.ch, d.scratch);
  tl->mark("k_rp_chal_fr", s, (double)B * (3 * k + 4 * (k + 1) + 12));
  // batch check on s3 (after the caller's hook, e.g. the exclusion of range
  // proofs whose action failed its sigma proof): the weights need only the
  // challenges, so on the latency path (d.rlc_fork = 0) they start right after
  // k_rp_chal_fr, before the exact phase's wide launches take the CUs; the
  // work path forks after its widest launch (d.rlc_fork = 1) so the check's
  // latency-bound chain does not share SIMDs with it.  The x0-free columns and
  // their fixed-base products run on s4 (they need k_rp_powers' vectors): the
  // MSM's bucket phase does not wait for them, only its window reduction.
  auto rlc_prep = [&]() {
    tl->fork(s, s3);
    if (d.pre_rlc) d.pre_rlc(d.pre_rlc_arg, s3);
    FTS_LAUNCH(k_rlc_prep, B, lbs, s3, B, n, k, d.status, d.excl, d.ipa_flag, d.sc, d.ch, r.key, r.msc, r.coef);
    tl->mark("k_rlc_prep", s3, (double)B * (3 * k + 33));
    (void)hipEventRecord(d.ev_coef, s3);
  };
  const bool grouped = r.G > 1;
  // presorted: the MSM's sort already ran on s3 (d.rlc_fork == 3); only its
  // accumulation and reduction are left
  auto rlc_rest = [&](bool presorted = false) {
    auto msm = [&](const uint32_t* extra, int nextra) {
      if (presorted) launch_msm_reduce(r.plan, d.pts, extra, nextra, r.msm_scratch, s3, s4, tl);
      else launch_msm(r.plan, d.pts, r.msc, extra, nextra, r.msm_scratch, s3, s4, tl);
    };
    tl->fork(s, s4);   // k_rp_powers' vectors
    tl->fork(s3, s4);  // the weights
    if (grouped) {
      // per caller batch: the x0-free column sums and products of every group (slot Q
      // left as the identity: zero words), the MSM's extras with stride NC
      (void)hipMemsetAsync(r.gfix, 0, (size_t)r.G * NC * 96, s4);
      hipLaunchKernelGGL(k_rlc_columns, dim3(NC - 1, r.G), dim3(256), 0, s4, B, n, k, r.gs, 0, r.sel, d.ch, r.coef,
                         d.ypow, d.svec, d.zvec, r.gcol);
      tl->mark("k_rlc_columns", s4, (double)B * 4 * n);
      FTS_LAUNCH(k_rlc_fixed, (size_t)r.G * (NC - 1) * FB_NW, RF_ITEMS * FB_NW, s4, n, r.G, 0, NC - 1, r.gcol, tables,
                 r.gfix);
      tl->mark("k_rlc_fixed", s4, (double)r.G * (NC - 1) * (FB_NW * 3 + (FB_NW - 1) * COST_ADD));
      msm(r.gfix, NC);
      return;
    }
    hipLaunchKernelGGL(k_rlc_columns, dim3(NC - 1, 1), dim3(256), 0, s4, B, n, k, B, 0, (const int32_t*)nullptr, d.ch,
                       r.coef, d.ypow, d.svec, d.zvec, r.colsum);
    tl->mark("k_rlc_columns", s4, (double)B * 4 * n);
    FTS_LAUNCH(k_rlc_fixed, (size_t)(NC - 1) * FB_NW, RF_ITEMS * FB_NW, s4, n, 1, 0, NC - 1, r.colsum, tables, r.fixed);
    tl->mark("k_rlc_fixed", s4, (double)(NC - 1) * (FB_NW * 3 + (FB_NW - 1) * COST_ADD));
    msm(r.fixed, NC - 1);
  };
  if (!d.rlc_fork) rlc_prep();
  FTS_LAUNCH(k_rp_powers, B * (n >> std::min(PW_LC, k)), 64, s, B, n, k, d.status, d.ch, d.ypow, d.svec, d.zvec);
  tl->mark("k_rp_powers", s, (double)B * (3.0 * n + 2.0 * k));
  // d.rlc_fork == 3 (work path): the weights and the MSM's counting sort (memory /
  // LDS work, no long chains) beside the fixed-base launch; its accumulation waits
  // for that launch (after it, below), so the MSM chain starts sorted
  // The weights run on s itself, ahead of the fixed-base launch (0.2 ms alone; on
  // s3 beside that launch the 320 blocks starved for 6 ms), then the sort on s3.
  // d.rlc_fork == 4: the whole sort on s itself (~0.6 ms alone, ahead of the
  // fixed-base launch): beside the chain kernels the sort's small latency-bound
  // launches starved (k_rs_hist 0.04 -> 2.2 ms in a 20-batch burst, round 5), and
  // beside the fixed-base launch too (3: k_msm_split 6 ms)
  const bool early_sort = (d.rlc_fork == 3 || d.rlc_fork == 4) && !d.com_fixed && d.ev_fx && !d.pre_rlc;
  if (early_sort) {
    FTS_LAUNCH(k_rlc_prep, B, lbs, s, B, n, k, d.status, d.excl, d.ipa_flag, d.sc, d.ch, r.key, r.msc, r.coef);
    tl->mark("k_rlc_prep", s, (double)B * (3 * k + 33));
    (void)hipEventRecord(d.ev_coef, s);
    if (d.rlc_fork == 4) {
      launch_msm_sort(r.plan, r.msc, s, tl);
    } else {
      tl->fork(s, s3);
      launch_msm_sort(r.plan, r.msc, s3, tl);
    }
  }
  auto rlc_side = [&]() {
    if (d.rlc_fork) rlc_prep();
    rlc_rest();
  };
  if (!d.rlc_fork) rlc_side();
  // exact per-proof phase on s
  // FTS_FX_SERIAL: one pass's fixed-base launch at a time across the lanes (the
  // previous pass's launch has ended), so the next pass's launch overlaps this
  // pass's latency-bound chain instead of its own twin
  if (d.fx_wait) (void)hipStreamWaitEvent(s, d.fx_wait, 0);
  if (d.com_fixed) {
    if (wbits == 22)
      FTS_LAUNCH(k_rp_fixed_all<22>, (size_t)B * (2 * n + 2), 64, s, B, n, k, d.status, d.sc, d.ch, d.ypow, d.zvec,
                 wtables, d.hpj, d.terms);
    else
      FTS_LAUNCH(k_rp_fixed_all<FBW_W>, (size_t)B * (2 * n + 2), 64, s, B, n, k, d.status, d.sc, d.ch, d.ypow, d.zvec,
                 wtables, d.hpj, d.terms);
    tl->mark("k_rp_fixed_all", s, (double)B * (2.0 * n + 2.0) * cost_fbw);
    if (d.ev_fx) (void)hipEventRecord(d.ev_fx, s);
    if (d.rlc_fork) rlc_side();
    // with the x0 prefix split (FTS_X0_SPLIT bit 1), the normalisation also writes the
    // H' records of the x0 messages, and the prefix is hashed on s2 beside com_tree
    if (d.x0_mid) FTS_LAUNCH(k_rp_x0_hdr, B, 256, s, B, n, d.status, x0_const, d.x0_msgs);
    launch_normalize(nhp, n, n + 1, 0, d.status, d.hpj, d.hpa, d.hp_be, s, d.x0_mid ? d.x0_msgs : nullptr);
    tl->mark("k_rp_normalize", s, (double)nhp * (7.0 + COST_INV / NORM_E));
    tl->fork(s2, s);  // x*D (k_rp_xd) before com_tree
    if (d.x0_mid) {   // after the fork above, so com_tree does not wait for the prefix
      tl->fork(s, s2);
      FTS_LAUNCH(k_rp_x0_hash, B, lbs, s2, B, n, k, d.status, d.x0_msgs, x0_tmpl, 0u, x0_cb1(n), d.x0_mid, d.ch);
      tl->mark("k_rp_x0_prefix", s2, 0);
    }
    hipLaunchKernelGGL(k_rp_com_tree, dim3((B + CT_PROOFS - 1) / CT_PROOFS), dim3(CT_LANES * CT_PROOFS), 0, s, B, n,
                       k, d.status, d.pts, d.terms, d.hpj, d.hpa, d.hp_be);
    tl->mark("k_rp_com_sum", s, (double)B * ((com_fx_slots(n) + 1) * COST_ADD + COST_NORM1));
  } else {
    if (wbits == 22)
      FTS_LAUNCH(k_rp_fixed_exact<22>, (size_t)B * (n + 2), 64, s, B, n, k, d.status, d.sc, d.ch, d.ypow, wtables,
                 d.hpj, d.terms);
    else
      FTS_LAUNCH(k_rp_fixed_exact<FBW_W>, (size_t)B * (n + 2), 64, s, B, n, k, d.status, d.sc, d.ch, d.ypow, wtables,
                 d.hpj, d.terms);
    tl->mark("k_rp_fixed_exact", s, (double)B * (n + 2) * cost_fbw);
    if (d.ev_fx) (void)hipEventRecord(d.ev_fx, s);
    if (early_sort) {
      (void)hipStreamWaitEvent(s3, d.ev_fx, 0);
      rlc_rest(true);
    } else if (d.rlc_fork) {
      rlc_side();
    }
    // H'_i -> affine + BE bytes (x0 transcript) on the side stream: the S / com
    // chain on s works on the Jacobian H' (k_rp_hsum_chunks) and does not wait
    // for it; com is normalised after com_var
    tl->fork(s, s2);
    // with the x0 prefix split, the normalisation also writes the H' hex records of
    // the x0 messages (k_rp_x0_hdr the header and constant bytes around them)
    if (d.x0_mid) FTS_LAUNCH(k_rp_x0_hdr, B, 256, s2, B, n, d.status, x0_const, d.x0_msgs);
    launch_normalize(nhp, n, n + 1, 0, d.status, d.hpj, d.hpa, d.hp_be, s2, d.x0_mid ? d.x0_msgs : nullptr);
    tl->mark("k_rp_normalize", s2, (double)nhp * (7.0 + COST_INV / NORM_E));
    if (d.x0_mid) {
      // x0 prefix on the side stream: the H' records and the shared template
      // (cb1 of the message's blocks) do not depend on com, so they are hashed
      // beside the S / com chain; only the suffix waits for com
      FTS_LAUNCH(k_rp_x0_hash, B, lbs, s2, B, n, k, d.status, d.x0_msgs, x0_tmpl, 0u, x0_cb1(n), d.x0_mid, d.ch);
      tl->mark("k_rp_x0_prefix", s2, 0);
    }
    const int nch = (n + HS_CHUNK - 1) / HS_CHUNK;
    FTS_LAUNCH(k_rp_hsum_chunks, B * nch, g_chain_bs, s, B, n, d.status, d.hpj, d.scratch);
    tl->mark("k_rp_hsum_chunks", s, (double)B * (n - nch) * (COST_DBL + COST_ADD));
    FTS_LAUNCH(k_rp_hsum_join, B, g_chain_bs, s, B, n, d.status, d.scratch);
    tl->mark("k_rp_hsum_join", s, (double)B * (nch - 1) * (HS_CHUNK * COST_DBL + COST_ADD));
    // scratch: [0, B*HS_SCRATCH) Horner chunks of S, then the 2B lanes' affine tables
    FTS_LAUNCH(k_rp_com_var, 2 * B, g_chain_bs, s, B, n, k, d.status, d.pts, d.ch, d.scratch,
               d.scratch + (size_t)B * HS_SCRATCH, d.terms, d.hpj, d.hpa, d.hp_be);
    tl->mark("k_rp_com_var", s, (double)B * (2 * (COST_STRAUS2_CTAB + 2.5 * COST_ADD) + COST_NORM1));
  }
  const bool split = d.x0_mid != nullptr;
  // work path without the prefix split: the whole message needs the H' bytes of s2
  if (!d.com_fixed && !split) tl->fork(s2, s);
  hipLaunchKernelGGL(k_rp_x0_build, dim3(x0_build_grid(B)), dim3(64 * X0_PPB), x0_build_lds(n, split ? 1 : 2), s, B,
                     n, d.status, d.hp_be, x0_const, d.sc, d.x0_msgs, split ? 1 : 2);
  tl->mark(split ? "k_rp_x0_build_tail" : "k_rp_x0_build", s, 0);
  if (split) tl->fork(s2, s);  // the prefix's midstate
  FTS_LAUNCH(k_rp_x0_hash, B, lbs, s, B, n, k, d.status, d.x0_msgs, x0_tmpl, split ? x0_cb1(n) : 0u, 0xffffffffu,
             d.x0_mid, d.ch);
  tl->mark("k_rp_x0_hash", s, 0);
  // x0 tail: column Q (needs the weights of k_rlc_prep) and its product, then
  // the verdict once the MSM is in
  (void)hipStreamWaitEvent(s, d.ev_coef, 0);
  if (grouped) {
    hipLaunchKernelGGL(k_rlc_columns, dim3(1, r.G), dim3(256), 0, s, B, n, k, r.gs, NC - 1, r.sel, d.ch, r.coef,
                       d.ypow, d.svec, d.zvec, r.gcol);
    FTS_LAUNCH(k_rlc_fixed, (size_t)r.G * FB_NW, RF_ITEMS * FB_NW, s, n, r.G, NC - 1, 1, r.gcol, tables, r.gqfix);
    tl->mark("k_rlc_q", s, (double)B + r.G * (FB_NW * 3 + (FB_NW - 1) * COST_ADD));
    (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(r.flag), 1, 1, s);
    tl->fork(s3, s);
    FTS_LAUNCH(k_rlc_finalize_groups, (size_t)r.G * r.gs, 256, s, r.G * r.gs, r.gs, NC, r.sel, r.plan.out, r.gqfix,
               d.excl, d.status, d.ipa_flag, r.gflag, r.flag);
    tl->mark("k_rlc_finalize", s, 0);
    return;
  }
  {
    const int gsq = (B + RQ_PARTS - 1) / RQ_PARTS;  // proofs per partial sum
    hipLaunchKernelGGL(k_rlc_columns, dim3(1, RQ_PARTS), dim3(256), 0, s, B, n, k, gsq, NC - 1,
                       (const int32_t*)nullptr, d.ch, r.coef, d.ypow, d.svec, d.zvec, r.colsum + (size_t)NC * 8);
    hipLaunchKernelGGL(k_rlc_qsum, dim3(1), dim3(RQ_PARTS), 0, s, NC, NC - 1, r.colsum);
  }
  FTS_LAUNCH(k_rlc_fixed, FB_NW, RF_ITEMS * FB_NW, s, n, 1, NC - 1, 1, r.colsum, tables, r.fixed);
  tl->mark("k_rlc_q", s, (double)B + FB_NW * 3 + (FB_NW - 1) * COST_ADD);
  tl->fork(s3, s);
  FTS_LAUNCH(k_rlc_finalize, B, 64, s, B, r.plan.out, r.fixed + (size_t)(NC - 1) * 24, d.excl, d.status, d.ipa_flag,
             r.flag);
  tl->mark("k_rlc_finalize", s, 0);
}

// the single-fault locator's device work on s, after a failed batch check of the
// (ungrouped) pass d: saves S, recomputes the combination with index weights into
// the same workspace (weights, columns, MSM, column Q) and writes to loc[0] the j
// with S' = (j + 1) S (loc[0] must be -1 before)
void launch_rlc_locate(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, uint32_t* save, int32_t* loc,
                       hipStream_t s, Timeline* tl) {
  const int B = d.B, n = d.n, k = d.k, NC = rlc_ncols(n);
  hipLaunchKernelGGL(k_rlc_total, dim3(1), dim3(64), 0, s, r.plan.out, r.fixed + (size_t)(NC - 1) * 24, save);
  FTS_LAUNCH(k_rlc_prep, B, 64, s, B, n, k, d.status, d.excl, d.ipa_flag, d.sc, d.ch, r.key, r.msc, r.coef, 1);
  tl->mark("k_rlc_prep", s, (double)B * (3 * k + 34));
  // alone on the GPU here: every column split over RQ_PARTS slices of proofs (NC x 64
  // blocks instead of NC), the partial rows then summed per column
  const int gsq = (B + RQ_PARTS - 1) / RQ_PARTS;
  hipLaunchKernelGGL(k_rlc_columns, dim3(NC - 1, RQ_PARTS), dim3(256), 0, s, B, n, k, gsq, 0,
                     (const int32_t*)nullptr, d.ch, r.coef, d.ypow, d.svec, d.zvec, r.colsum + (size_t)NC * 8);
  hipLaunchKernelGGL(k_rlc_qsum, dim3(NC - 1), dim3(RQ_PARTS), 0, s, NC, 0, r.colsum);
  tl->mark("k_rlc_columns", s, (double)B * 4 * n);
  FTS_LAUNCH(k_rlc_fixed, (size_t)(NC - 1) * FB_NW, RF_ITEMS * FB_NW, s, n, 1, 0, NC - 1, r.colsum, tables, r.fixed);
  tl->mark("k_rlc_fixed", s, (double)(NC - 1) * (FB_NW * 3 + (FB_NW - 1) * COST_ADD));
  launch_msm(r.plan, d.pts, r.msc, r.fixed, NC - 1, r.msm_scratch, s, s, tl);
  hipLaunchKernelGGL(k_rlc_columns, dim3(1, RQ_PARTS), dim3(256), 0, s, B, n, k, gsq, NC - 1,
                     (const int32_t*)nullptr, d.ch, r.coef, d.ypow, d.svec, d.zvec, r.colsum + (size_t)NC * 8);
  hipLaunchKernelGGL(k_rlc_qsum, dim3(1), dim3(RQ_PARTS), 0, s, NC, NC - 1, r.colsum);
  FTS_LAUNCH(k_rlc_fixed, FB_NW, RF_ITEMS * FB_NW, s, n, 1, NC - 1, 1, r.colsum, tables, r.fixed);
  tl->mark("k_rlc_q", s, (double)B + FB_NW * 3 + (FB_NW - 1) * COST_ADD);
  FTS_LAUNCH(k_rlc_locate, B, 64, s, B, save, r.plan.out, r.fixed + (size_t)(NC - 1) * 24, loc);
  tl->mark("k_rlc_locate", s, (double)B * 28 * COST_ADD);
}
void launch_rlc_accept_except(int B, int skip, int32_t* status, const int32_t* ipa_flag, hipStream_t s) {
  FTS_LAUNCH(k_rlc_accept_except, B, 256, s, B, skip, status, ipa_flag);
}

void launch_normalize_all(int total, const uint32_t* jac, uint32_t* aff, hipStream_t s) {
  launch_normalize(total, 1, 1, 0, (const int32_t*)nullptr, jac, aff, (uint8_t*)nullptr, s);
}

// per-proof final equations (fallback when the batch combination fails)
void launch_rp_gather(const RpGather& g, int k, uint8_t* raw, uint32_t* sc, int32_t* status, int32_t* ipa, hipStream_t s) {
  const int per = rp_npts(k) * 4 + RP_NSC * 2 + 1;
  FTS_LAUNCH(k_rp_gather, (size_t)g.off[g.G] * per, 64, s, g, rp_npts(k), raw, sc, status, ipa);
}

// per-proof final equations of the nsel proofs sel[0 .. nsel) (all B if sel == nullptr)
void launch_rp_fallback(const RpBatchDev& d, const uint32_t* tables, const int32_t* sel, int nsel, hipStream_t s,
                        Timeline* tl) {
  const int B = sel ? nsel : d.B, n = d.n, k = d.k;
  FTS_LAUNCH(k_rp_terms_fixed, B * (3 + 2 * n), 64, s, B, n, k, sel, d.status, d.ipa_flag, d.sc, d.ch, tables, d.terms);
  tl->mark("k_rp_terms_fixed", s, (double)B * (3 + 2 * n) * COST_FB_FRESH);
  const size_t nvar = (size_t)B * (3 + 2 * k);
  if (nvar <= TV_COOP_MAX)  // latency-bound: lane-cooperative chains
    FTS_LAUNCH(k_rp_terms_var_coop, (nvar + TV_GPW - 1) / TV_GPW * 64, 64, s, B, n, k, sel, d.status, d.ipa_flag, d.pts,
               d.ch, d.terms);
  else
    FTS_LAUNCH(k_rp_terms_var, nvar, 64, s, B, n, k, sel, d.status, d.ipa_flag, d.pts, d.ch, d.terms, d.scratch);
  tl->mark("k_rp_terms_var", s, (double)B * (3 + 2 * k) * (4.0 * 7.0 + 12.0 * COST_ADD + 124 * COST_DBL + 60 * COST_ADD));
  if (B > 0)
    hipLaunchKernelGGL(k_rp_check, dim3((B + CK_PROOFS - 1) / CK_PROOFS), dim3(CK_LANES * CK_PROOFS), 0, s, B, n, k,
                       sel, d.status, d.ipa_flag, d.terms, d.hpa);
  tl->mark("k_rp_check", s, (double)B * rp_nterms(n, k) * COST_ADD);
}

// Group test of the batch check (after it failed): G groups of gs proof slots
// sel[g gs + j] (-1 = empty); every group's partial random linear combination
// (the batch check's weights) from per-group column sums + one grouped MSM
// (plan p: G groups of gs * npts points, indirection sel).  Groups that close
// accept their proofs; the proofs of the others are appended to next[] /
// next_count for the next round (smaller groups, or per-proof checks).
void launch_rlc_group_test(const RpBatchDev& d, const RlcDev& r, const uint32_t* tables, const MsmPlan& p,
                           const int32_t* sel, int G, int gs, uint32_t* gcol, uint32_t* gfix, int32_t* next,
                           uint32_t* next_count, hipStream_t s, Timeline* tl) {
  const int n = d.n, k = d.k;
  const int NC = rlc_ncols(n);
  if (gs <= GT_SMALL_MAX) {
    const int nch = gt_nchunks(n);
    FTS_LAUNCH(k_rlc_group_cols_small, (size_t)G * nch, 256, s, d.B, n, k, G, gs, sel, d.ch, r.coef, d.ypow, d.svec,
               d.zvec, tables, gfix);
    tl->mark("k_rlc_group_cols", s, (double)G * (gs * 3.0 * n + NC * FB_NW * COST_MADD));
    launch_msm_small(p, d.pts, r.msc, gfix, nch, s, tl);
    FTS_LAUNCH(k_rlc_group_final, (size_t)G * gs, 256, s, G * gs, gs, sel, p.out, d.status, d.ipa_flag, next,
               next_count);
    tl->mark("k_rlc_group_final", s, 0);
    return;
  }
  hipLaunchKernelGGL(k_rlc_columns, dim3(NC, G), dim3(gs <= 64 ? 64 : 256), 0, s, d.B, n, k, gs, 0, sel, d.ch,
                     r.coef, d.ypow, d.svec, d.zvec, gcol);
  tl->mark("k_rlc_group_columns", s, (double)G * gs * 4 * n);
  FTS_LAUNCH(k_rlc_fixed, (size_t)NC * G * FB_NW, RF_ITEMS * FB_NW, s, n, G, 0, NC, gcol, tables, gfix);
  tl->mark("k_rlc_group_fixed", s, (double)G * NC * (FB_NW * 3 + (FB_NW - 1) * COST_ADD));
  launch_msm(p, d.pts, r.msc, gfix, NC, r.msm_scratch, s, s, tl);
  FTS_LAUNCH(k_rlc_group_final, (size_t)G * gs, 256, s, G * gs, gs, sel, p.out, d.status, d.ipa_flag, next,
             next_count);
  tl->mark("k_rlc_group_final", s, 0);
}

}  // namespace fts

namespace fts {
// Config C3 staging (fts_msm_stage_multiples): N distinct points P_i = k_i * B
// from a fixed-base table (16-bit windows), k_i = 32-byte BE integers mod r,
// as Jacobian into jac (normalised by the caller), and the MSM scalars s_i
// (BE, reduced mod r as G1.Mul does) as canonical limbs
__global__ void __launch_bounds__(256) k_msm_gen_points(int N, const uint8_t* __restrict__ raw_k,
                                                       const uint8_t* __restrict__ raw_s,
                                                       const uint32_t* __restrict__ table, uint32_t* __restrict__ jac,
                                                       uint32_t* __restrict__ sc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  auto be_fr = [](const uint8_t* p) {
    uint32_t w[8];
    const uint4* s4 = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint4 u = s4[q];
      w[4 * q + 0] = __builtin_bswap32(u.x);
      w[4 * q + 1] = __builtin_bswap32(u.y);
      w[4 * q + 2] = __builtin_bswap32(u.z);
      w[4 * q + 3] = __builtin_bswap32(u.w);
    }
    return digest_to_fr(w);  // canonical limbs mod r
  };
  const Fr k = be_fr(raw_k + (size_t)i * 32), sv = be_fr(raw_s + (size_t)i * 32);
  Scalar ks;
#pragma unroll
  for (int q = 0; q < 8; q++) ks.v[q] = k.v[q], sc[(size_t)i * 8 + q] = sv.v[q];
  store_g1j(jac + (size_t)i * 24, fb_mul(table, ks));
}
void launch_msm_gen_points(int N, const uint8_t* raw_k, const uint8_t* raw_s, const uint32_t* table, uint32_t* jac,
                           uint32_t* pts, uint32_t* sc, hipStream_t s) {
  FTS_LAUNCH(k_msm_gen_points, N, 256, s, N, raw_k, raw_s, table, jac, sc);
  launch_normalize(N, 1, 1, 0, (const int32_t*)nullptr, jac, pts, (uint8_t*)nullptr, s);
}
}  // namespace fts

namespace fts {
// x0 = Hz(DER(Arr(H'..., G..., Q, com), "||", Zb(ip))) for B proofs whose
// H'/com BE points are in hp_be and ip in sc (RP_SC_IP): the prover's entry
// to the same transcript kernels (prove_kernels.hip)
void launch_x0(int B, int n, int k, const int32_t* status, const uint8_t* hp_be, const uint8_t* x0_const,
               const uint8_t* x0_tmpl, const uint32_t* sc, uint8_t* msgs, uint32_t* ch, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(k_rp_x0_build, dim3(x0_build_grid(B)), dim3(64 * X0_PPB), x0_build_lds(n), s, B, n, status, hp_be, x0_const, sc, msgs, 2);
  FTS_LAUNCH(k_rp_x0_hash, B, g_lat_bs, s, B, n, k, status, msgs, x0_tmpl, 0u, 0xffffffffu, (uint32_t*)nullptr, ch);
}
hipError_t rp_set_wave_prio(const int* p) { return upload_wave_prio(p); }
}  // namespace fts
