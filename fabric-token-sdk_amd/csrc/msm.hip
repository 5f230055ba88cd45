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
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NV) return;
  for (int w = 0; w < nw; w++) {
    int key = keys[(size_t)w * NV + i];
    if (key == -1) continue;
    uint32_t b = (uint32_t)key & 0x7fffffffu;
    sorted[offsets[b] + ranks[(size_t)w * NV + i]] = (uint32_t)i | ((uint32_t)key & 0x80000000u);
  }
}

// ------------------------------------------------ large one-group plans
// Counting sort without global atomics (N >= MSM_LS_MIN_N, one group, no
// indirection): k_msm_digits' 16 returning device-scope atomics per point were
// its cost at 2^22 points (3 ms).  Here the sort runs per (slice of virtual
// points, window) block with the window's histogram in LDS:
//   k_msm_split     lane per point: GLV halves + the recoding constant
//   k_msm_lhist     block (slice, window): LDS histogram -> hs[w][slice][b]
//   k_msm_lscan     lane per (window, bucket): prefix over the slices, counts
//   (k_msm_scan1/2/3 as before: bucket offsets and the chunk map)
//   k_msm_lscatter  block (slice, window): LDS cursors = bucket offset + slice
//                   prefix; each entry takes the next slot of its bucket
// Signed digits as bit fields: with C = sum_w (2^(width_w-1) - 1) 2^off_w,
// window w's digit of k is ((k + C) >> off_w mod 2^width_w) - (2^(width_w-1) - 1)
// (the carries of k + C are exactly the recoding carries of k_msm_digits:
// d > half <=> bits + carry + half - 1 >= 2^width), so every block extracts
// its window's digit without the lower windows.  Same buckets and signs as
// k_msm_digits; the order inside a bucket differs (bucket sums are the same
// group elements, and only the affine result is observable).
constexpr int MSM_LS_SLICES = 64;
constexpr int MSM_LS_MIN_N = 1 << 18;  // points
constexpr int MSM_LS_BS = 1024;

__global__ void __launch_bounds__(256) k_msm_split(int N, uint4 rc, const uint32_t* __restrict__ scalars,
                                                   uint4* __restrict__ hk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  uint32_t s[8];
#pragma unroll
  for (int q = 0; q < 8; q++) s[q] = scalars[(size_t)i * 8 + q];
  uint32_t k[2][4], sg[2];
  glv_decompose(s, k[0], sg[0], k[1], sg[1]);
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint64_t t = (uint64_t)k[h][0] + rc.x;
    const uint32_t w0 = (uint32_t)t;
    t = (t >> 32) + k[h][1] + rc.y;
    const uint32_t w1 = (uint32_t)t;
    t = (t >> 32) + k[h][2] + rc.z;
    const uint32_t w2 = (uint32_t)t;
    t = (t >> 32) + k[h][3] + rc.w;
    const uint32_t w3 = ((uint32_t)t & 0x7fffffffu) | (sg[h] ? 0x80000000u : 0u);  // k + C < 2^127
    hk[(size_t)h * N + i] = make_uint4(w0, w1, w2, w3);
  }
}

FTS_DEV int ls_digit(const uint4 q, const MsmWindow& W) {
  const uint32_t k[4] = {q.x, q.y, q.z, q.w & 0x7fffffffu};
  return (int)scalar_bits4(k, W.off, W.width) - ((1 << (W.width - 1)) - 1);
}

__global__ void __launch_bounds__(MSM_LS_BS) k_msm_lhist(int NV, int per, int S, int stride,
                                                        const MsmWindow* __restrict__ win,
                                                        const uint4* __restrict__ hk, uint32_t* __restrict__ hs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lh[];
  const int sl = blockIdx.x, w = blockIdx.y;
  const MsmWindow W = win[w];
  const int nb = 1 << (W.width - 1);
  for (int b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = 0;
  __syncthreads();
  const int v1 = min(NV, (sl + 1) * per);
  for (int v = sl * per + threadIdx.x; v < v1; v += blockDim.x) {
    const int d = ls_digit(hk[v], W);
    if (d != 0) atomicAdd(&lh[(d < 0 ? -d : d) - 1], 1u);
  }
  __syncthreads();
  uint32_t* out = hs + ((size_t)w * S + sl) * stride;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) out[b] = lh[b];
}

__global__ void __launch_bounds__(256) k_msm_lscan(int S, int stride, const MsmWindow* __restrict__ win,
                                                  uint32_t* __restrict__ hs, uint32_t* __restrict__ counts) {
  const int w = blockIdx.y, b = blockIdx.x * blockDim.x + threadIdx.x;
  const MsmWindow W = win[w];
  if (b >= (1 << (W.width - 1))) return;
  uint32_t acc = 0;
  for (int sl = 0; sl < S; sl++) {
    uint32_t* q = hs + ((size_t)w * S + sl) * stride + b;
    const uint32_t c = *q;
    *q = acc;
    acc += c;
  }
  counts[W.bbase + b] = acc;
}

__global__ void __launch_bounds__(MSM_LS_BS) k_msm_lscatter(int NV, int per, int S, int stride,
                                                           const MsmWindow* __restrict__ win,
                                                           const uint4* __restrict__ hk,
                                                           const uint32_t* __restrict__ hs,
                                                           const uint32_t* __restrict__ offsets,
                                                           uint32_t* __restrict__ sorted) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
  const int sl = blockIdx.x, w = blockIdx.y;
  const MsmWindow W = win[w];
  const int nb = 1 << (W.width - 1);
  const uint32_t* pre = hs + ((size_t)w * S + sl) * stride;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) cur[b] = offsets[W.bbase + b] + pre[b];
  __syncthreads();
  const int v1 = min(NV, (sl + 1) * per);
  for (int v = sl * per + threadIdx.x; v < v1; v += blockDim.x) {
    const uint4 q = hk[v];
    const int d = ls_digit(q, W);
    if (d != 0) {
      const uint32_t pos = atomicAdd(&cur[(d < 0 ? -d : d) - 1], 1u);
      sorted[pos] = (uint32_t)v | (((d < 0) != ((q.w >> 31) != 0)) ? 0x80000000u : 0u);
    }
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
// digits, counting sort, chunked bucket accumulation and bucket sums (every plan)
static void launch_msm_buckets(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, hipStream_t s,
                               Timeline* tl, hipEvent_t ev_stage = nullptr, int stage = 0) {
  // block-local counting sort for large one-group plans (keys: the split
  // halves, NV x 16 B; cursor: the slice histograms, nw x S x stride words)
  int nbmax = 1;
  for (int w = 0; w < p.nw; w++) nbmax = std::max(nbmax, 1 << (p.win[w].width - 1));
  const int S = std::min(MSM_LS_SLICES, p.NV / nbmax);
  const bool ls = p.local_sort && p.G == 1 && !p.sel && p.N >= MSM_LS_MIN_N && nbmax <= (1 << 15) && S >= 8 &&
                  p.nw >= 4;
  if (ls) {
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
    const int per = (p.NV + S - 1) / S;
    uint4* hk = reinterpret_cast<uint4*>(p.keys);
    FTS_LAUNCH(k_msm_split, p.N, 256, s, p.N, make_uint4(rc[0], rc[1], rc[2], rc[3]), scalars, hk);
    tl->mark("k_msm_split", s, 0);
    const size_t lds = (size_t)nbmax * 4;
    hipLaunchKernelGGL(k_msm_lhist, dim3(S, p.nw), dim3(MSM_LS_BS), lds, s, p.NV, per, S, nbmax, p.d_win, hk,
                       p.cursor);
    hipLaunchKernelGGL(k_msm_lscan, dim3((nbmax + 255) / 256, p.nw), dim3(256), 0, s, S, nbmax, p.d_win, p.cursor,
                       p.counts);
    tl->mark("k_msm_lhist", s, 0);
    FTS_LAUNCH(k_msm_scan1, (size_t)p.NBLK * 256, 256, s, p.NB, p.ch, p.counts, p.offsets, p.chunk_off, p.scratch);
    hipLaunchKernelGGL(k_msm_scan2, dim3(1), dim3(256), 0, s, p.NBLK, p.scratch);
    FTS_LAUNCH(k_msm_scan3, p.NB, 256, s, p.NB, p.ch, p.counts, p.offsets, nullptr, p.chunk_off, p.chunk_bkt,
               p.scratch);
    tl->mark("k_msm_scan", s, 0);
    hipLaunchKernelGGL(k_msm_lscatter, dim3(S, p.nw), dim3(MSM_LS_BS), lds, s, p.NV, per, S, nbmax, p.d_win, hk,
                       p.cursor, p.offsets, p.sorted);
    tl->mark("k_msm_lscatter", s, 0);
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
  if (ev_stage && stage == 1) (void)hipEventRecord(ev_stage, s);
  FTS_LAUNCH(k_msm_chunks, p.NC, 64, s, msm_idx(p), p.scratch + 2 * (size_t)p.NBLK + 1, p.d_win, points, p.offsets,
             p.counts, p.chunk_off,
             p.chunk_bkt, p.sorted, p.partials);
  // expected nonzero digits: N * nw * (1 - 2^-c) ~ N * nw mixed additions
  tl->mark("k_msm_chunks", s, (double)p.NV * p.nw * (COST_MADD + 0.5));
  if (ev_stage && stage == 2) (void)hipEventRecord(ev_stage, s);
  FTS_LAUNCH(k_msm_bucket_sum, p.NB, g_lat_bs, s, p.NB, p.ch, p.counts, p.chunk_off, p.partials, p.buckets);
  tl->mark("k_msm_bucket_sum", s, 0);
}

void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, hipStream_t s_extra, Timeline* tl, hipEvent_t ev_stage, int stage) {
  launch_msm_buckets(p, points, scalars, s, tl, ev_stage, stage);
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
void launch_msm_to_bytes(const uint32_t* jac, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_msm_to_bytes, dim3(1), dim3(64), 0, s, jac, out);
}

}  // namespace fts
