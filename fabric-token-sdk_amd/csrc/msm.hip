// Pippenger bucket MSM on BN254 G1 (see device/msm.hpp for the plan layout).
//
// Used by the random-linear-combination batch check of the range proofs
// (SURVEY Appendix B): one MSM over the per-proof variable points
// (T1, T2, V, com, L_j, R_j) replaces the per-proof final equations of
// bulletproof.go:314-324 and ipa.go:254-259.  Also exposed as fts_msm_g1
// (BASELINE config C3 microbenchmark).
#include <algorithm>

#include "device/g1.hpp"
#include "device/glv.hpp"
#include "device/fixed_base.hpp"
#include "device/helpers.hpp"
#include "device/msm.hpp"
#include "device/rp_kernels.hpp"
#include "device/coop.hpp"

namespace fts {
extern int g_lat_bs;  // rp_kernels.hip


// bits [off, off+width) of a 128-bit LE magnitude (width <= 20)
FTS_DEV uint32_t scalar_bits4(const uint32_t s[4], int off, int width) {
  int q = off >> 5, r = off & 31;
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i == q) lo = s[i];
    if (i == q + 1) hi = s[i];
  }
  uint64_t v = (lo | (hi << 32)) >> r;
  return (uint32_t)(v & ((1ull << width) - 1));
}

// the point-indexing part of a plan, passed to the kernels by value
struct MsmIdx {
  int N, nw, ptsg, NBg, sel_pts, ch;
  const int32_t* sel;
};
inline MsmIdx msm_idx(const MsmPlan& p) { return MsmIdx{p.N, p.nw, p.ptsg, p.NBg, p.sel_pts, p.ch, p.sel}; }
// input index of plan point i (-1: absent padding point of a grouped plan)
FTS_DEV long msm_src(const MsmIdx& p, int i) {
  if (!p.sel) return i;
  const int q = p.sel[i / p.sel_pts];
  return q < 0 ? -1L : (long)q * p.sel_pts + i % p.sel_pts;
}

// lane per real point i: GLV split, then the signed digits of both halves
// (virtual points i and N + i) for every window; group g = i / ptsg owns the
// buckets [g NBg, (g + 1) NBg)
__global__ void __launch_bounds__(256) k_msm_digits(MsmIdx p, const MsmWindow* __restrict__ win,
                                                    const uint32_t* __restrict__ scalars, int32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ ranks, uint32_t* __restrict__ counts) {
  wave_prio<PS_SORT>();
  const int N = p.N, nw = p.nw;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const long src = msm_src(p, i);
  const int gb = (i / p.ptsg) * p.NBg;
  uint32_t s[8];
#pragma unroll
  for (int q = 0; q < 8; q++) s[q] = src < 0 ? 0u : scalars[(size_t)src * 8 + q];
  uint32_t k[2][4], sg[2];
  glv_decompose(s, k[0], sg[0], k[1], sg[1]);
  const int NV = 2 * N;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    int carry = 0;
    for (int w = 0; w < nw; w++) {
      const MsmWindow W = win[w];
      int d = (int)scalar_bits4(k[h], W.off, W.width) + carry;
      const int half = 1 << (W.width - 1);
      carry = d > half;
      d = carry ? d - (1 << W.width) : d;
      int key = -1;
      if (d != 0) {
        int b = gb + W.bbase + (d < 0 ? -d : d) - 1;
        key = ((d < 0) != (sg[h] != 0)) ? (b | (int)0x80000000) : b;
        ranks[(size_t)w * NV + h * N + i] = atomicAdd(&counts[b], 1u);  // rank within the bucket
      }
      keys[(size_t)w * NV + h * N + i] = key;
    }
  }
}

// Global exclusive scans over all NB buckets (windows are consecutive bucket
// ranges): offsets[b] = position of bucket b's first entry in the flat sorted
// array, chunk_off[b] = its first chunk slot.  Pass 1: block-local scans of
// MSM_SCAN_ITEMS buckets (4 per lane) + block totals; pass 2: one block scans
// the totals; pass 3: adds the block offsets, copies the cursor and fills the
// chunk map; k_msm_chunks ignores slots past the chunk total (blk[2 NBLK + 1]).
__global__ void __launch_bounds__(256) k_msm_scan1(int NB, int ch, const uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ offsets, uint32_t* __restrict__ chunk_off,
                                                   uint32_t* __restrict__ blk) {
  wave_prio<PS_SORT>();
  __shared__ uint32_t pe[256], pc[256];
  const int t = threadIdx.x;
  const int base = blockIdx.x * MSM_SCAN_ITEMS + t * 4;
  uint32_t cnt[4], le = 0, lc = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    cnt[j] = base + j < NB ? counts[base + j] : 0u;
    le += cnt[j];
    lc += (cnt[j] + ch - 1) / ch;
  }
  pe[t] = le;
  pc[t] = lc;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const uint32_t ve = t >= off ? pe[t - off] : 0, vc = t >= off ? pc[t - off] : 0;
    __syncthreads();
    pe[t] += ve;
    pc[t] += vc;
    __syncthreads();
  }
  uint32_t re = pe[t] - le, rc = pc[t] - lc;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (base + j < NB) {
      offsets[base + j] = re;
      chunk_off[base + j] = rc;
    }
    re += cnt[j];
    rc += (cnt[j] + ch - 1) / ch;
  }
  if (t == 255) {
    blk[2 * blockIdx.x] = pe[255];
    blk[2 * blockIdx.x + 1] = pc[255];
  }
}

__global__ void __launch_bounds__(256) k_msm_scan2(int nblk, uint32_t* __restrict__ blk) {
  wave_prio<PS_SORT>();
  __shared__ uint32_t pe[256], pc[256];
  const int t = threadIdx.x;
  const int per = (nblk + 255) / 256;
  uint32_t le = 0, lc = 0;
  for (int j = 0; j < per; j++) {
    const int q = t * per + j;
    if (q < nblk) {
      le += blk[2 * q];
      lc += blk[2 * q + 1];
    }
  }
  pe[t] = le;
  pc[t] = lc;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const uint32_t ve = t >= off ? pe[t - off] : 0, vc = t >= off ? pc[t - off] : 0;
    __syncthreads();
    pe[t] += ve;
    pc[t] += vc;
    __syncthreads();
  }
  uint32_t re = pe[t] - le, rc = pc[t] - lc;
  for (int j = 0; j < per; j++) {
    const int q = t * per + j;
    if (q < nblk) {
      const uint32_t e = blk[2 * q], c = blk[2 * q + 1];
      blk[2 * q] = re;
      blk[2 * q + 1] = rc;
      re += e;
      rc += c;
    }
  }
  if (t == 255) {  // totals: entries, chunk slots in use
    blk[2 * nblk] = pe[255];
    blk[2 * nblk + 1] = pc[255];
  }
}

__global__ void __launch_bounds__(256) k_msm_scan3(int NB, int ch, const uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ offsets, uint32_t* __restrict__ cursor,
                                                   uint32_t* __restrict__ chunk_off, int32_t* __restrict__ chunk_bkt,
                                                   const uint32_t* __restrict__ blk) {
  wave_prio<PS_SORT>();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= NB) return;
  const int q = b / MSM_SCAN_ITEMS;
  const uint32_t o = offsets[b] + blk[2 * q], oc = chunk_off[b] + blk[2 * q + 1];
  offsets[b] = o;
  chunk_off[b] = oc;
  const uint32_t nch = (counts[b] + ch - 1) / ch;
  for (uint32_t c = 0; c < nch; c++) chunk_bkt[oc + c] = b;
}

// counting-sort scatter without atomics: position = bucket offset + the
// rank the histogram atomic returned in k_msm_digits
__global__ void __launch_bounds__(256) k_msm_scatter(int NV, int nw, const int32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ ranks,
                                                     const uint32_t* __restrict__ offsets, uint32_t* __restrict__ sorted) {
  wave_prio<PS_SORT>();
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NV) return;
  for (int w = 0; w < nw; w++) {
    int key = keys[(size_t)w * NV + i];
    if (key == -1) continue;
    uint32_t b = (uint32_t)key & 0x7fffffffu;
    sorted[offsets[b] + ranks[(size_t)w * NV + i]] = (uint32_t)i | ((uint32_t)key & 0x80000000u);
  }
}

// ------------------------------------------------ two-level counting sort
// (round 5; one-group plans whose windows all have >= 2^RS_PSH buckets: the
// batch check's MSM and standalone MSMs).  k_msm_digits costs 2 x nw returning
// device-scope atomics per point (VALUBusy 4.5 %, 0.89 GB written per
// 81,920-proof pass) and k_msm_scatter one random 4-byte HBM write per entry
// (0.70 GB); the round-4 block-local sort held a window's whole histogram in
// 128 KB of LDS per 1,024-thread block and took whole CUs beside the chain
// kernels.  Here every LDS table is <= 32 KB per 256-thread block and no
// device-scope atomic is used:
//   k_rs_hist     block per slice of RS_SP points: GLV split, every window's
//                 signed digit, LDS histogram over PARTITIONS (bucket >> RS_PSH,
//                 NP <= RS_MAX_NP counters) -> hist[slice][p] (one coalesced row)
//   k_rs_pscan    lane per partition: exclusive prefix over the slices, in place
//   k_rs_pbase    one block: exclusive scan of the partition totals -> pbase
//   k_rs_scatter  block per slice: LDS cursors = pbase + the slice's prefix; each
//                 entry takes the next slot of its partition (a slice writes
//                 ~RS_SP * 2 nw / NP consecutive entries per partition: whole
//                 lines, combined in L2), entry = virtual index | low bucket
//                 bits << 24 | sign << 31
//   k_rs_part     block per partition: LDS counting sort of its ~5.4 k entries
//                 by the low bucket bits -> counts[b] and the final sorted array
// (k_msm_scan1/2/3 then derive the bucket offsets -- the same positions, the
// order is bucket-major in both -- and the chunk map).  Digits: with C = sum_w
// (2^(width_w-1) - 1) 2^off_w, window w's signed digit of a GLV half k is
// ((k + C) >> off_w mod 2^width_w) - (2^(width_w-1) - 1): the carries of k + C
// are exactly k_msm_digits' recoding carries (tests/test_msm_recode_cpu.py), so
// the digits are independent bit fields.  Same buckets and signs as
// k_msm_digits; the order inside a bucket differs, which changes no group
// element (only the affine result is observable).
constexpr int RS_PSH = 6;                 // buckets per partition: 64
constexpr int RS_SP = 4096;               // points per slice (block); 2 x for >= 2^21 points
constexpr int RS_MAX_NPG = 8192;          // partitions per group: LDS counters <= 32 KB
constexpr int RS_MIN_N = 4096;            // smaller plans keep k_msm_digits
constexpr int RS_PART_STAGE = 7680;       // k_rs_part: entries sorted in LDS (30 KB + 1 KB counters)
constexpr uint32_t RS_IDX_MASK = 0x00ffffffu;  // virtual index bits of an entry (NV < 2^24)
// Grouped plans (G > 1, e.g. the batch check per caller batch): slices never
// straddle two groups (SPG slices per group), a slice's LDS table holds its own
// group's NPg = NBg / 64 partitions, hist is [slice][NPg], and the global
// partition g NPg + lp covers the group's buckets g NBg + 64 lp .. + 63.

// lane per plan point: the GLV halves of its scalar with the recoding constant
// folded in, hk[h N + i] = (k_h + C) | sign_h << 127 (absent padding points of a
// grouped plan: k = 0, so every window's digit is 0).  One point per lane, so the
// split is spread over the chip instead of the hist / scatter blocks' slices
__global__ void __launch_bounds__(256) k_msm_split(MsmIdx p, uint4 rc, const uint32_t* __restrict__ scalars,
                                                   uint4* __restrict__ hk) {
  wave_prio<PS_SORT>();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.N) return;
  const long src = msm_src(p, i);
  uint32_t k[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, sg[2] = {0, 0};
  if (src >= 0) {
    uint32_t s[8];
    const uint4* s4 = reinterpret_cast<const uint4*>(scalars + (size_t)src * 8);
    const uint4 a = s4[0], b = s4[1];
    s[0] = a.x, s[1] = a.y, s[2] = a.z, s[3] = a.w, s[4] = b.x, s[5] = b.y, s[6] = b.z, s[7] = b.w;
    glv_decompose(s, k[0], sg[0], k[1], sg[1]);
  }
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t q0, q1, q2, q3, c;
    q0 = addc(k[h][0], rc.x, 0, c);
    q1 = addc(k[h][1], rc.y, c, c);
    q2 = addc(k[h][2], rc.z, c, c);
    q3 = addc(k[h][3], rc.w, c, c);  // k + C < 2^127
    hk[(size_t)h * p.N + i] = make_uint4(q0, q1, q2, (q3 & 0x7fffffffu) | (sg[h] ? 0x80000000u : 0u));
  }
}

// the nonzero window digits of plan point i's two GLV halves (from k_msm_split);
// f(local bucket, sign, virtual index) per digit
template <class F>
FTS_DEV void rs_point_digits(const MsmIdx& p, const MsmWindow* __restrict__ win, const uint4* __restrict__ hk, int i,
                             F&& f) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint4 u = hk[(size_t)h * p.N + i];
    const uint32_t q[4] = {u.x, u.y, u.z, u.w & 0x7fffffffu};
    const bool sg = (u.w >> 31) != 0;
    for (int w = 0; w < p.nw; w++) {
      const MsmWindow W = win[w];
      const int d = (int)scalar_bits4(q, W.off, W.width) - ((1 << (W.width - 1)) - 1);
      if (d != 0) f(W.bbase + (d < 0 ? -d : d) - 1, (d < 0) != sg, (uint32_t)(h * p.N + i));
    }
  }
}
// window w's digits of plan point i (both GLV halves): as rs_point_digits, one window
template <class F>
FTS_DEV void rs_point_digits_w(const MsmIdx& p, const MsmWindow& W, const uint4* __restrict__ hk, int i, F&& f) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint4 u = hk[(size_t)h * p.N + i];
    const uint32_t q[4] = {u.x, u.y, u.z, u.w & 0x7fffffffu};
    const bool sg = (u.w >> 31) != 0;
    const int d = (int)scalar_bits4(q, W.off, W.width) - ((1 << (W.width - 1)) - 1);
    if (d != 0) f(W.bbase + (d < 0 ? -d : d) - 1, (d < 0) != sg, (uint32_t)(h * p.N + i));
  }
}
// points [i0, i1) of block blockIdx.x's slice (group g).  Blocks are dealt to the 8
// XCDs round-robin; slices are dealt in contiguous ranges per XCD instead (a
// bijection on [0, gridDim.x)), so the neighbouring runs of one partition, which
// share cache lines at their ends, are written through the same L2 and leave it as
// whole lines (round-robin: every such line left two L2s partially written)
FTS_DEV int rs_xcd_slice(int b, int S) {
  const int xcd = b & 7, local = b >> 3, q = S >> 3, r = S & 7;
  return xcd < r ? xcd * (q + 1) + local : r * (q + 1) + (xcd - r) * q + local;
}
FTS_DEV void rs_slice(const MsmIdx& p, int spg, int& g, int& i0, int& i1, int& slice) {
  slice = rs_xcd_slice((int)blockIdx.x, (int)gridDim.x);
  g = slice / spg;
  const int ls = slice % spg;
  const int sp = (p.ptsg + spg - 1) / spg;  // the host's slice size, up to rounding
  i0 = g * p.ptsg + ls * sp;
  i1 = min(min(i0 + sp, (g + 1) * p.ptsg), p.N);
}

__global__ void __launch_bounds__(256) k_rs_hist(MsmIdx p, int spg, int npg, const MsmWindow* __restrict__ win,
                                                 const uint4* __restrict__ hk, uint32_t* __restrict__ hist) {
  wave_prio<PS_SORT>();
  extern __shared__ uint32_t rs_lds[];
  for (int q = threadIdx.x; q < npg; q += blockDim.x) rs_lds[q] = 0;
  __syncthreads();
  int g, i0, i1, slice;
  rs_slice(p, spg, g, i0, i1, slice);
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x)
    rs_point_digits(p, win, hk, i, [&](int bl, bool, uint32_t) { atomicAdd(&rs_lds[bl >> RS_PSH], 1u); });
  __syncthreads();
  uint32_t* out = hist + (size_t)slice * npg;
  for (int q = threadIdx.x; q < npg; q += blockDim.x) out[q] = rs_lds[q];
}

// lane per global partition g npg + lp: exclusive prefix over the group's slices, in place
__global__ void __launch_bounds__(256) k_rs_pscan(int G, int spg, int npg, uint32_t* __restrict__ hist,
                                                  uint32_t* __restrict__ ptot) {
  wave_prio<PS_SORT>();
  const int P = blockIdx.x * blockDim.x + threadIdx.x;
  if (P >= G * npg) return;
  const int g = P / npg, lp = P % npg;
  uint32_t* h = hist + (size_t)g * spg * npg + lp;
  uint32_t acc = 0;
  int s = 0;
  for (; s + 8 <= spg; s += 8) {  // 8 loads in flight per lane
    uint32_t c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = h[(size_t)(s + q) * npg];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      h[(size_t)(s + q) * npg] = acc;
      acc += c[q];
    }
  }
  for (; s < spg; s++) {
    const uint32_t c = h[(size_t)s * npg];
    h[(size_t)s * npg] = acc;
    acc += c;
  }
  ptot[P] = acc;
}

constexpr int RS_PB_BS = 1024;
__global__ void __launch_bounds__(RS_PB_BS) k_rs_pbase(int NP, const uint32_t* __restrict__ ptot,
                                                      uint32_t* __restrict__ pbase) {
  wave_prio<PS_SORT>();
  __shared__ uint32_t sh[RS_PB_BS];
  const int t = threadIdx.x, per = (NP + RS_PB_BS - 1) / RS_PB_BS;
  uint32_t loc = 0;
  for (int j = 0; j < per; j++) {
    const int q = t * per + j;
    if (q < NP) loc += ptot[q];
  }
  sh[t] = loc;
  __syncthreads();
  for (int off = 1; off < RS_PB_BS; off <<= 1) {
    const uint32_t v = t >= off ? sh[t - off] : 0u;
    __syncthreads();
    sh[t] += v;
    __syncthreads();
  }
  uint32_t run = sh[t] - loc;
  for (int j = 0; j < per; j++) {
    const int q = t * per + j;
    if (q < NP) {
      pbase[q] = run;
      run += ptot[q];
    }
  }
}

__global__ void __launch_bounds__(256) k_rs_scatter(MsmIdx p, int spg, int npg, const MsmWindow* __restrict__ win,
                                                    const uint4* __restrict__ hk, const uint32_t* __restrict__ hist,
                                                    const uint32_t* __restrict__ pbase, uint32_t* __restrict__ tmp) {
  wave_prio<PS_SORT>();
  extern __shared__ uint32_t rs_lds[];
  int g, i0, i1, slice;
  rs_slice(p, spg, g, i0, i1, slice);
  const uint32_t* pre = hist + (size_t)slice * npg;
  const uint32_t* pb = pbase + (size_t)g * npg;
  for (int q = threadIdx.x; q < npg; q += blockDim.x) rs_lds[q] = pb[q] + pre[q];
  __syncthreads();
  // window-major: while the block writes window w, its open partition runs are that
  // window's NPg / nw partitions (~16 entries = one line each per slice), so L2
  // combines them into whole-line writes; point-major, the runs of all nw windows
  // were open at once (2,048 x 64 B per block) and left L2 as partial lines
  // (0.55 GB written per 81,920-proof pass for 0.09 GB of entries, r05 PMC).
  // The slice's hk rows are re-read per window from L2.
  for (int w = 0; w < p.nw; w++) {
    const MsmWindow W = win[w];
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x)
      rs_point_digits_w(p, W, hk, i, [&](int bl, bool neg, uint32_t v) {
        const uint32_t pos = atomicAdd(&rs_lds[bl >> RS_PSH], 1u);
        tmp[pos] = v | ((uint32_t)(bl & ((1 << RS_PSH) - 1)) << 24) | (neg ? 0x80000000u : 0u);
      });
  }
}

// block per global partition P (buckets 64 P .. 64 P + 63: group P / npg's local
// partition P % npg, as NBg = 64 npg)
__global__ void __launch_bounds__(256) k_rs_part(const uint32_t* __restrict__ pbase, const uint32_t* __restrict__ ptot,
                                                 const uint32_t* __restrict__ tmp, uint32_t* __restrict__ counts,
                                                 uint32_t* __restrict__ sorted) {
  wave_prio<PS_SORT>();
  constexpr int PB = 1 << RS_PSH;
  __shared__ uint32_t cnt[PB], cur[PB];
  __shared__ uint32_t stage[RS_PART_STAGE];
  const int P = blockIdx.x, t = threadIdx.x;
  const uint32_t lo = pbase[P], n = ptot[P];
  if (t < PB) cnt[t] = 0;
  __syncthreads();
  for (uint32_t e = t; e < n; e += blockDim.x) atomicAdd(&cnt[(tmp[lo + e] >> 24) & (PB - 1)], 1u);
  __syncthreads();
  if (t < PB) {
    const uint32_t c = cnt[t];
    counts[(size_t)P * PB + t] = c;
    cur[t] = c;
  }
  __syncthreads();
  for (int off = 1; off < PB; off <<= 1) {  // inclusive scan of the PB counts
    const uint32_t v = (t < PB && t >= off) ? cur[t - off] : 0u;
    __syncthreads();
    if (t < PB) cur[t] += v;
    __syncthreads();
  }
  if (t < PB) cur[t] -= cnt[t];  // exclusive
  __syncthreads();
  if (n <= (uint32_t)RS_PART_STAGE) {  // the usual partition: sorted in LDS, one coalesced write
    for (uint32_t e = t; e < n; e += blockDim.x) {
      const uint32_t x = tmp[lo + e];
      const uint32_t pos = atomicAdd(&cur[(x >> 24) & (PB - 1)], 1u);
      stage[pos] = (x & RS_IDX_MASK) | (x & 0x80000000u);
    }
    __syncthreads();
    for (uint32_t e = t; e < n; e += blockDim.x) sorted[lo + e] = stage[e];
    return;
  }
  for (uint32_t e = t; e < n; e += blockDim.x) {  // oversized (adversarial scalars): in place
    const uint32_t x = tmp[lo + e];
    const uint32_t pos = atomicAdd(&cur[(x >> 24) & (PB - 1)], 1u);
    sorted[lo + pos] = (x & RS_IDX_MASK) | (x & 0x80000000u);
  }
}

// one lane per chunk slot: <= p.ch mixed additions of sorted virtual points
// (index >= N: phi(P_{index-N}) = (beta x, y))
__global__ void __launch_bounds__(64, 4) k_msm_chunks(MsmIdx p, const uint32_t* __restrict__ nc_total,
                                                   const MsmWindow* __restrict__ win,
                                                   const uint32_t* __restrict__ points,
                                                   const uint32_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ chunk_off,
                                                   const int32_t* __restrict__ chunk_bkt,
                                                   const uint32_t* __restrict__ sorted, uint32_t* __restrict__ partials) {
  wave_prio<PS_CHUNKS>();
  const int N = p.N;
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int)*nc_total) return;
  const int b = chunk_bkt[g];
  const uint32_t j = (uint32_t)g - chunk_off[b], cnt = counts[b];
  const uint32_t lo = j * (uint32_t)p.ch, hi = min(cnt, lo + (uint32_t)p.ch);
  const uint32_t* S = sorted + offsets[b];
  const Fp beta = glv_beta();
  G1J acc = g1j_identity();
  // the next entry's point is gathered while the current addition runs
  // (absent points never get a bucket entry, so msm_src is >= 0 here; a
  // two-deep prefetch measured slower: 2.29 -> 2.36 ms at 2^20 points)
  uint32_t e = S[lo];
  G1A q = load_g1a(points + (size_t)msm_src(p, (int)((e & 0x7fffffffu) >= (uint32_t)N ? (e & 0x7fffffffu) - N
                                                                                      : (e & 0x7fffffffu))) * 16);
  for (uint32_t t = lo; t < hi; t++) {
    uint32_t en = 0;
    G1A qn;
    if (t + 1 < hi) {
      en = S[t + 1];
      const uint32_t vn = en & 0x7fffffffu;
      qn = load_g1a(points + (size_t)msm_src(p, (int)(vn >= (uint32_t)N ? vn - N : vn)) * 16);
    }
    if (!g1a_is_identity(q)) {
      if ((e & 0x7fffffffu) >= (uint32_t)N) q.x = fp_mul(q.x, beta);
      if (e >> 31) q.y = f_neg(q.y);
      madd_inl(acc, q);
    }
    e = en;
    q = qn;
  }
  store_g1j(partials + (size_t)g * 24, acc);
}

// one lane per bucket: sum of its chunk partials (usually 1..4)
__global__ void __launch_bounds__(256) k_msm_bucket_sum(int NB, int ch, const uint32_t* __restrict__ counts,
                                                       const uint32_t* __restrict__ chunk_off,
                                                       const uint32_t* __restrict__ partials,
                                                       uint32_t* __restrict__ buckets) {
  wave_prio<PS_MSMTAIL>();
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= NB) return;
  const uint32_t nch = (counts[b] + ch - 1) / ch, c0 = chunk_off[b];
  G1J acc = g1j_identity();
  if (nch) acc = load_g1j(partials + (size_t)c0 * 24);
  for (uint32_t q = 1; q < nch; q++) add_inl(acc, load_g1j(partials + (size_t)(c0 + q) * 24));
  store_g1j(buckets + (size_t)b * 24, acc);
}

// running-sum reduction of MSM_SEG consecutive buckets of one (group, window):
// sum_j (j+1) B_j for the window-local bucket indices j of the segment
__global__ void __launch_bounds__(256) k_msm_segments(int nw, int NS, int NSg, int NBg, const MsmWindow* __restrict__ win,
                                                     const uint32_t* __restrict__ buckets,
                                                     uint32_t* __restrict__ segs, uint32_t* __restrict__ scratch) {
  wave_prio<PS_MSMTAIL>();
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= NS) return;
  const int grp = g / NSg, gl = g % NSg;
  int w = 0;
  while (w + 1 < nw && win[w + 1].sbase <= gl) w++;
  const MsmWindow W = win[w];
  const int nb = 1 << (W.width - 1);
  const int s = gl - W.sbase;
  const int lo = s * MSM_SEG, cnt = (nb - lo) < MSM_SEG ? (nb - lo) : MSM_SEG;
  const uint32_t* Bk = buckets + ((size_t)grp * NBg + W.bbase + lo) * 24;
  G1J sum = g1j_identity(), acc = g1j_identity();
  for (int j = cnt - 1; j >= 0; j--) {
    add_inl(sum, load_g1j(Bk + j * 24));
    add_inl(acc, sum);
  }
  uint32_t m = (uint32_t)lo;  // bucket lo+j carries multiplier lo + j + 1
  if (m) {
    G1J t = g1j_identity();
    for (int bit = 31 - __builtin_clz(m); bit >= 0; bit--) {
      t = g1j_dbl(t);
      if ((m >> bit) & 1u) add_inl(t, sum);
    }
    add_inl(acc, t);
  }
  store_g1j(segs + (size_t)g * 24, acc);
}

// LDS tree (block of 256 lanes) over <= MSM_WIN_ITEMS consecutive segments:
// block (w, j, group) with w < nw sums part j of the group's window-w segments;
// w = nw sums part j of the group's nextra extra Jacobian points (the fixed-base part)
__global__ void __launch_bounds__(256) k_msm_windows(int nw, int WB, int NSg, const MsmWindow* __restrict__ win,
                                                     const uint32_t* __restrict__ segs, const uint32_t* __restrict__ extra,
                                                     int nextra, uint32_t* __restrict__ parts) {
  wave_prio<PS_MSMTAIL>();
  __shared__ uint32_t sh[256 * 24];
  const int t = threadIdx.x, w = blockIdx.x, j = blockIdx.y, grp = blockIdx.z;
  const uint32_t* S;
  int cnt;
  if (w < nw) {
    const MsmWindow W = win[w];
    cnt = ((1 << (W.width - 1)) + MSM_SEG - 1) / MSM_SEG;
    S = segs + ((size_t)grp * NSg + W.sbase) * 24;
  } else {
    cnt = extra ? nextra : 0;
    S = extra + (size_t)grp * nextra * 24;
  }
  const int lo = j * MSM_WIN_ITEMS, hi = min(cnt, lo + MSM_WIN_ITEMS);
  G1J acc = g1j_identity();
  for (int s = lo + t; s < hi; s += 256) add_inl(acc, load_g1j(S + (size_t)s * 24));
  store_g1j(sh + t * 24, acc);
  __syncthreads();
  for (int half = 128; half >= 1; half >>= 1) {
    if (t < half) add_inl(acc, load_g1j(sh + (t + half) * 24));
    __syncthreads();
    if (t < half) store_g1j(sh + t * 24, acc);
    __syncthreads();
  }
  if (t == 0) store_g1j(parts + (((size_t)grp * (nw + 1) + w) * WB + j) * 24, acc);
}

// coop group per window w <= nw: W_w = sum of window w's parts, shifted to its
// bit offset (2^off_w W_w: the windows' doubling chains run in parallel, the
// longest is the top window's ~off_top doublings instead of one 127-doubling
// Horner chain), group nw: the extra points; then an LDS tree over the groups.
// Lane-cooperative (device/coop.hpp): 12 groups of COOP_G lanes per wave, and
// as many waves as the windows need (a grouped plan's narrower windows: 14-16
// of them; with one wave, two windows shared a group and its chain doubled).
constexpr int FINAL_GPW = 64 / COOP_G;  // coop groups per wave
constexpr int FINAL_MAXW = 4;           // waves per block (48 groups >= MSM windows + 1)
__global__ void __launch_bounds__(64 * FINAL_MAXW) k_msm_final(int nw, int WB, const MsmWindow* __restrict__ win,
                                                               const uint32_t* __restrict__ parts_all,
                                                               uint32_t* __restrict__ out_all) {
  wave_prio<PS_MSMTAIL>();
  __shared__ uint32_t sh[FINAL_MAXW * FINAL_GPW * 24];
  const int t = threadIdx.x, grp = blockIdx.x;  // one block per MSM group
  const int wave = t / 64, lt = t % 64;
  const int NG = (blockDim.x / 64) * FINAL_GPW;  // coop groups in the block
  const int gi = lt / COOP_G, role = lt % COOP_G, base = gi * COOP_G;  // base: lane within the wave
  const int g = wave * FINAL_GPW + gi;
  const bool live = gi < FINAL_GPW;
  const uint32_t* parts = parts_all + (size_t)grp * (nw + 1) * WB * 24;
  uint32_t* out = out_all + (size_t)grp * 24;
  G1J acc = g1j_identity();
  if (live) {
    for (int w = g; w <= nw; w += NG) {
      G1J W = load_g1j(parts + (size_t)w * WB * 24);
      for (int j = 1; j < WB; j++) coop_add(W, load_g1j(parts + ((size_t)w * WB + j) * 24), role, base);
      if (w < nw)
        for (int q = 0; q < win[w].off; q++) W = coop_dbl(W, role, base);
      coop_add(acc, W, role, base);
    }
    if (role == 0) store_g1j(sh + g * 24, acc);
  }
  __syncthreads();
  // tree over the NG groups' sums (NG = 12 * waves; pad to a power of two)
  int P2 = 1;
  while (P2 < NG) P2 <<= 1;
  for (int half = P2 / 2; half >= 1; half >>= 1) {
    const bool act = live && g < half && g + half < NG;
    if (act) coop_add(acc, load_g1j(sh + (g + half) * 24), role, base);
    __syncthreads();
    if (act && role == 0) store_g1j(sh + g * 24, acc);
    __syncthreads();
  }
  if (t == 0) store_g1j(out, acc);
}

// ------------------------------------------------ many small groups
// Finish of a grouped plan whose groups are small (the group test's later
// rounds: 10^4 groups of a few proofs, windows of <= 2^5 buckets): the
// segment / LDS-tree / one-block-per-group kernels above leave most lanes idle
// there.  Lane per (window, group), window-major so a wave's lanes run the
// same doubling count: W = sum_d d B_d by running sums over the window's
// buckets, then 2^off W -> wparts[group][window].
__global__ void __launch_bounds__(256) k_msm_small_windows(int nw, int G, int NBg, const MsmWindow* __restrict__ win,
                                                          const uint32_t* __restrict__ buckets,
                                                          uint32_t* __restrict__ wparts) {
  wave_prio<PS_MSMTAIL>();
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)nw * G) return;
  const int w = (int)(gid / G), grp = (int)(gid % G);
  const MsmWindow W = win[w];
  const int nb = 1 << (W.width - 1);
  const uint32_t* Bk = buckets + ((size_t)grp * NBg + W.bbase) * 24;
  G1J sum = g1j_identity(), acc = g1j_identity();
  for (int j = nb - 1; j >= 0; j--) {
    add_inl(sum, load_g1j(Bk + (size_t)j * 24));
    add_inl(acc, sum);
  }
  for (int q = 0; q < W.off; q++) acc = g1j_dbl(acc);
  store_g1j(wparts + ((size_t)grp * nw + w) * 24, acc);
}

// one wave per group: its nw window parts + nextra extra points, LDS tree -> out[group]
__global__ void __launch_bounds__(64) k_msm_small_final(int nw, const uint32_t* __restrict__ wparts,
                                                        const uint32_t* __restrict__ extra, int nextra,
                                                        uint32_t* __restrict__ out) {
  wave_prio<PS_MSMTAIL>();
  __shared__ uint32_t sh[64 * 24];
  const int t = threadIdx.x, grp = blockIdx.x;
  G1J acc = g1j_identity();
  for (int q = t; q < nw + nextra; q += 64)
    add_inl(acc, load_g1j(q < nw ? wparts + ((size_t)grp * nw + q) * 24 : extra + ((size_t)grp * nextra + q - nw) * 24));
  store_g1j(sh + t * 24, acc);
  __syncthreads();
  for (int half = 32; half >= 1; half >>= 1) {
    if (t < half) add_inl(acc, load_g1j(sh + (t + half) * 24));
    __syncthreads();
    if (t < half) store_g1j(sh + t * 24, acc);
    __syncthreads();
  }
  if (t == 0) store_g1j(out + (size_t)grp * 24, acc);
}

// ------------------------------------------------ standalone MSM (fts_msm_*)
// Inputs of fts_msm_stage: N raw points (64-byte X||Y BE, NewG1FromBytes
// checks; 64 zero bytes = identity) and N 32-byte BE scalars (any 256-bit
// integer, reduced mod r as G1.Mul does).  bad counts rejected points.
__global__ void __launch_bounds__(256) k_msm_load(int N, const uint8_t* __restrict__ raw_pts,
                                                  const uint8_t* __restrict__ raw_sc, uint32_t* __restrict__ pts,
                                                  uint32_t* __restrict__ sc, uint32_t* __restrict__ bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  G1A a;
  if (!decode_point(raw_pts + (size_t)i * 64, a)) {
    atomicAdd(bad, 1u);
    a.x = f_zero<FpP>();
    a.y = f_zero<FpP>();
  }
  store_g1a(pts + (size_t)i * 16, a);
  uint32_t w[8];
  const uint4* s4 = reinterpret_cast<const uint4*>(raw_sc + (size_t)i * 32);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint4 u = s4[q];
    w[4 * q + 0] = __builtin_bswap32(u.x);
    w[4 * q + 1] = __builtin_bswap32(u.y);
    w[4 * q + 2] = __builtin_bswap32(u.z);
    w[4 * q + 3] = __builtin_bswap32(u.w);
  }
  const Fr k = digest_to_fr(w);  // BE integer mod r (canonical limbs)
#pragma unroll
  for (int q = 0; q < 8; q++) sc[(size_t)i * 8 + q] = k.v[q];
}

// staged affine Montgomery points [lo, lo + n) -> 64-byte BE (fts_msm_points)
__global__ void __launch_bounds__(256) k_msm_pts_to_bytes(int n, const uint32_t* __restrict__ pts,
                                                         uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_point_be(out + (size_t)i * 64, load_g1a(pts + (size_t)i * 16));
}

// Jacobian result -> 64-byte BE affine (identity -> 64 zero bytes)
__global__ void k_msm_to_bytes(const uint32_t* __restrict__ jac, uint8_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  store_point_be(out, g1j_to_affine(load_g1j(jac)));
}

#define FTS_LAUNCH(kern, nthreads, bs, stream, ...)                                   \
  do {                                                                                \
    size_t nt_ = (size_t)(nthreads);                                                  \
    if (nt_) hipLaunchKernelGGL(kern, dim3((unsigned)((nt_ + (bs)-1) / (bs))), dim3(bs), 0, stream, __VA_ARGS__); \
  } while (0)

// scratch: NS * 24 words.  p.d_win must already hold p.win (uploaded by the caller).
// `extra` (nextra Jacobian points) is produced on stream s_extra: joined
// before the window reduction that sums it.
// digits and counting sort: every entry (window, virtual point) placed in its bucket
// (p.sorted / p.counts / p.offsets) and the chunk map -- needs only the scalars
void launch_msm_sort(const MsmPlan& p, const uint32_t* scalars, hipStream_t s, Timeline* tl) {
  // two-level counting sort (every window >= 2^RS_PSH buckets): tmp entries in
  // p.keys, slice histograms + partition totals / bases in p.cursor
  bool rs = p.local_sort && p.N >= RS_MIN_N && p.NV <= (int)RS_IDX_MASK && (p.NBg & ((1 << RS_PSH) - 1)) == 0;
  for (int w = 0; w < p.nw; w++) rs = rs && p.win[w].width > RS_PSH && (p.win[w].bbase & ((1 << RS_PSH) - 1)) == 0;
  const int npg = p.NBg >> RS_PSH, NP = p.G * npg;
  // slices of 8,192 points from 2^21 points per group on (C3 at 2^22: the scatter's
  // runs per partition twice as long, 2.23 -> 1.67 GB written, 0.90 -> 0.76 ms for
  // hist + scatter, round 5); the batch check keeps 4,096 (more blocks beside the chain)
  const int sp = p.ptsg >= (1 << 21) ? 2 * RS_SP : RS_SP;
  const int spg = (p.ptsg + sp - 1) / sp, S = p.G * spg;
  rs = rs && npg <= RS_MAX_NPG && p.ptsg > 0 && (size_t)S * npg + 2 * (size_t)NP <= (size_t)p.nw * p.NV &&
       p.nw >= 4;  // the split halves (NV x 16 B) fit in the sorted array (nw x NV x 4 B)
  if (rs) {
    uint32_t rc[4] = {0, 0, 0, 0};  // C = sum_w (2^(width_w-1) - 1) 2^off_w (< 2^126)
    for (int w = 0; w < p.nw; w++) {
      uint64_t add = (uint64_t)((1u << (p.win[w].width - 1)) - 1u);
      const int q = p.win[w].off >> 5, r = p.win[w].off & 31;
      uint64_t c = add << r;
      for (int j = q; j < 4 && c; j++) {
        const uint64_t t = (uint64_t)rc[j] + (c & 0xffffffffu);
        rc[j] = (uint32_t)t;
        c = (c >> 32) + (t >> 32);
      }
    }
    const uint4 rcv = make_uint4(rc[0], rc[1], rc[2], rc[3]);
    uint32_t* hist = p.cursor;                       // [S][npg]
    uint32_t* ptot = hist + (size_t)S * npg;         // [NP]
    uint32_t* pbase = ptot + NP;                     // [NP]
    uint32_t* tmp = reinterpret_cast<uint32_t*>(p.keys);
    // the split halves (NV x 16 B) in the sorted array's space: k_rs_part overwrites
    // it only after the scatter has read them
    uint4* hk = reinterpret_cast<uint4*>(p.sorted);
    const size_t lds = (size_t)npg * 4;
    const MsmIdx ix = msm_idx(p);
    FTS_LAUNCH(k_msm_split, p.N, 256, s, ix, rcv, scalars, hk);
    tl->mark("k_msm_split", s, 0);
    hipLaunchKernelGGL(k_rs_hist, dim3(S), dim3(256), lds, s, ix, spg, npg, p.d_win, hk, hist);
    tl->mark("k_rs_hist", s, 0);
    FTS_LAUNCH(k_rs_pscan, NP, 256, s, p.G, spg, npg, hist, ptot);
    hipLaunchKernelGGL(k_rs_pbase, dim3(1), dim3(RS_PB_BS), 0, s, NP, ptot, pbase);
    tl->mark("k_rs_pscan", s, 0);
    hipLaunchKernelGGL(k_rs_scatter, dim3(S), dim3(256), lds, s, ix, spg, npg, p.d_win, hk, hist, pbase, tmp);
    tl->mark("k_rs_scatter", s, 0);
    hipLaunchKernelGGL(k_rs_part, dim3(NP), dim3(256), 0, s, pbase, ptot, tmp, p.counts, p.sorted);
    tl->mark("k_rs_part", s, 0);
    FTS_LAUNCH(k_msm_scan1, (size_t)p.NBLK * 256, 256, s, p.NB, p.ch, p.counts, p.offsets, p.chunk_off, p.scratch);
    hipLaunchKernelGGL(k_msm_scan2, dim3(1), dim3(256), 0, s, p.NBLK, p.scratch);
    FTS_LAUNCH(k_msm_scan3, p.NB, 256, s, p.NB, p.ch, p.counts, p.offsets, nullptr, p.chunk_off, p.chunk_bkt,
               p.scratch);
    tl->mark("k_msm_scan", s, 0);
  } else {
    (void)hipMemsetAsync(p.counts, 0, (size_t)p.NB * 4, s);
    FTS_LAUNCH(k_msm_digits, p.N, 256, s, msm_idx(p), p.d_win, scalars, p.keys, p.cursor, p.counts);
    tl->mark("k_msm_digits", s, 0);
    FTS_LAUNCH(k_msm_scan1, (size_t)p.NBLK * 256, 256, s, p.NB, p.ch, p.counts, p.offsets, p.chunk_off, p.scratch);
    hipLaunchKernelGGL(k_msm_scan2, dim3(1), dim3(256), 0, s, p.NBLK, p.scratch);
    FTS_LAUNCH(k_msm_scan3, p.NB, 256, s, p.NB, p.ch, p.counts, p.offsets, p.cursor, p.chunk_off, p.chunk_bkt,
               p.scratch);
    tl->mark("k_msm_scan", s, 0);
    FTS_LAUNCH(k_msm_scatter, p.NV, 256, s, p.NV, p.nw, p.keys, p.cursor, p.offsets, p.sorted);
    tl->mark("k_msm_scatter", s, 0);
  }
}

// chunked bucket accumulation and bucket sums over a sorted plan (every plan)
static void launch_msm_accumulate(const MsmPlan& p, const uint32_t* points, hipStream_t s, Timeline* tl,
                                  hipEvent_t ev_stage = nullptr, int stage = 0) {
  FTS_LAUNCH(k_msm_chunks, p.NC, 64, s, msm_idx(p), p.scratch + 2 * (size_t)p.NBLK + 1, p.d_win, points, p.offsets,
             p.counts, p.chunk_off,
             p.chunk_bkt, p.sorted, p.partials);
  // expected nonzero digits: N * nw * (1 - 2^-c) ~ N * nw mixed additions
  tl->mark("k_msm_chunks", s, (double)p.NV * p.nw * (COST_MADD + 0.5));
  if (ev_stage && stage == 2) (void)hipEventRecord(ev_stage, s);
  FTS_LAUNCH(k_msm_bucket_sum, p.NB, g_lat_bs, s, p.NB, p.ch, p.counts, p.chunk_off, p.partials, p.buckets);
  tl->mark("k_msm_bucket_sum", s, 0);
}

static void launch_msm_buckets(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, hipStream_t s,
                               Timeline* tl, hipEvent_t ev_stage = nullptr, int stage = 0) {
  launch_msm_sort(p, scalars, s, tl);
  if (ev_stage && stage == 1) (void)hipEventRecord(ev_stage, s);
  launch_msm_accumulate(p, points, s, tl, ev_stage, stage);
}

// window reduction of the bucket sums: segments, windows (+ the extra points), final
static void launch_msm_tail(const MsmPlan& p, const uint32_t* extra, int nextra, uint32_t* scratch, hipStream_t s,
                            hipStream_t s_extra, Timeline* tl);

// accumulation and reduction of a plan sorted by launch_msm_sort (the batch check
// sorts beside the fixed-base launch and accumulates after it)
void launch_msm_reduce(const MsmPlan& p, const uint32_t* points, const uint32_t* extra, int nextra, uint32_t* scratch,
                       hipStream_t s, hipStream_t s_extra, Timeline* tl) {
  launch_msm_accumulate(p, points, s, tl);
  launch_msm_tail(p, extra, nextra, scratch, s, s_extra, tl);
}

void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, hipStream_t s_extra, Timeline* tl, hipEvent_t ev_stage, int stage) {
  launch_msm_sort(p, scalars, s, tl);
  if (ev_stage && stage == 1) (void)hipEventRecord(ev_stage, s);
  launch_msm_accumulate(p, points, s, tl, ev_stage, stage);
  launch_msm_tail(p, extra, nextra, scratch, s, s_extra, tl);
}

static void launch_msm_tail(const MsmPlan& p, const uint32_t* extra, int nextra, uint32_t* scratch, hipStream_t s,
                            hipStream_t s_extra, Timeline* tl) {
  FTS_LAUNCH(k_msm_segments, p.NS, g_lat_bs, s, p.nw, p.NS, p.NSg, p.NBg, p.d_win, p.buckets, p.segs, scratch);
  tl->mark("k_msm_segments", s, (double)p.NB * 2 * COST_ADD);
  if (s_extra != s) tl->fork(s_extra, s);
  uint32_t* parts = p.scratch + 2 * (size_t)p.NBLK + 2;
  hipLaunchKernelGGL(k_msm_windows, dim3(p.nw + 1, p.WB, p.G), dim3(256), 0, s, p.nw, p.WB, p.NSg, p.d_win, p.segs,
                     extra, nextra, parts);
  tl->mark("k_msm_windows", s, (double)(p.NS + (double)p.G * nextra) * COST_ADD);
  {
    const int waves = std::min(FINAL_MAXW, (p.nw + 1 + FINAL_GPW - 1) / FINAL_GPW);
    hipLaunchKernelGGL(k_msm_final, dim3(p.G), dim3(64 * waves), 0, s, p.nw, p.WB, p.d_win, parts, p.out);
  }
  {
    double dbl = 0;
    for (int w = 0; w < p.nw; w++) dbl += p.win[w].off;
    tl->mark("k_msm_final", s, p.G * (dbl * COST_DBL + (p.nw + 1) * (p.WB + 1) * COST_ADD));
  }
}

// grouped plan with small groups: buckets as usual, then k_msm_small_windows /
// k_msm_small_final (needs G * nw * 24 words of p.scratch past the scan sums)
void launch_msm_small(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra,
                      int nextra, hipStream_t s, Timeline* tl) {
  launch_msm_buckets(p, points, scalars, s, tl);
  uint32_t* wparts = p.scratch + 2 * (size_t)p.NBLK + 2;
  FTS_LAUNCH(k_msm_small_windows, (size_t)p.nw * p.G, 256, s, p.nw, p.G, p.NBg, p.d_win, p.buckets, wparts);
  {
    double dbl = 0;
    for (int w = 0; w < p.nw; w++) dbl += p.win[w].off;
    tl->mark("k_msm_small_windows", s, (double)p.G * (dbl * COST_DBL + 2.0 * p.NBg * COST_ADD));
  }
  hipLaunchKernelGGL(k_msm_small_final, dim3(p.G), dim3(64), 0, s, p.nw, wparts, extra, nextra, p.out);
  tl->mark("k_msm_small_final", s, (double)p.G * (p.nw + nextra) * COST_ADD);
}

void launch_msm_load(int N, const uint8_t* raw_pts, const uint8_t* raw_sc, uint32_t* pts, uint32_t* sc, uint32_t* bad,
                     hipStream_t s) {
  FTS_LAUNCH(k_msm_load, N, 256, s, N, raw_pts, raw_sc, pts, sc, bad);
}
void launch_msm_pts_to_bytes(int n, const uint32_t* pts, uint8_t* out, hipStream_t s) {
  FTS_LAUNCH(k_msm_pts_to_bytes, n, 256, s, n, pts, out);
}
void launch_msm_to_bytes(const uint32_t* jac, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_msm_to_bytes, dim3(1), dim3(64), 0, s, jac, out);
}

hipError_t msm_set_wave_prio(const int* p) { return upload_wave_prio(p); }
}  // namespace fts
