// Pippenger bucket MSM on BN254 G1 (see device/msm.hpp for the plan layout).
//
// Used by the random-linear-combination batch check of the range proofs
// (SURVEY Appendix B): one MSM over the per-proof variable points
// (T1, T2, V, com, L_j, R_j) replaces the per-proof final equations of
// bulletproof.go:314-324 and ipa.go:254-259.  Also exposed as fts_msm_g1
// (BASELINE config C3 microbenchmark).
#include "device/g1.hpp"
#include "device/helpers.hpp"
#include "device/msm.hpp"
#include "device/rp_kernels.hpp"

namespace fts {

// bits [off, off+width) of a 256-bit LE scalar (width <= 20)
FTS_DEV uint32_t scalar_bits(const uint32_t s[8], int off, int width) {
  int q = off >> 5, r = off & 31;
  uint64_t lo = s[q < 8 ? q : 7];
  uint64_t hi = (q + 1 < 8) ? s[q + 1] : 0;
  if (q >= 8) return 0;
  uint64_t v = (lo | (hi << 32)) >> r;
  return (uint32_t)(v & ((1ull << width) - 1));
}

__global__ void __launch_bounds__(256) k_msm_digits(int N, int nw, const MsmWindow* __restrict__ win,
                                                    const uint32_t* __restrict__ scalars, int32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ counts) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  uint32_t s[8];
#pragma unroll
  for (int q = 0; q < 8; q++) s[q] = scalars[(size_t)i * 8 + q];
  int carry = 0;
  for (int w = 0; w < nw; w++) {
    const MsmWindow W = win[w];
    int d = (int)scalar_bits(s, W.off, W.width) + carry;
    const int half = 1 << (W.width - 1);
    carry = d > half;
    d = carry ? d - (1 << W.width) : d;
    int key = -1;
    if (d != 0) {
      int b = W.bbase + (d < 0 ? -d : d) - 1;
      key = d < 0 ? (b | (int)0x80000000) : b;
      atomicAdd(&counts[b], 1u);
    }
    keys[(size_t)w * N + i] = key;
  }
}

// exclusive scan of the window's bucket counts -> offsets, cursor (block per window)
__global__ void __launch_bounds__(256) k_msm_scan(const MsmWindow* __restrict__ win, const uint32_t* __restrict__ counts,
                                                  uint32_t* __restrict__ offsets, uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[256];
  const int t = threadIdx.x;
  const MsmWindow W = win[blockIdx.x];
  const int nb = 1 << (W.width - 1);
  const uint32_t* C = counts + W.bbase;
  const int per = (nb + 255) / 256;
  uint32_t loc = 0;
  for (int j = 0; j < per; j++) {
    int b = t * per + j;
    if (b < nb) loc += C[b];
  }
  part[t] = loc;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - loc;
  for (int j = 0; j < per; j++) {
    int b = t * per + j;
    if (b < nb) {
      offsets[W.bbase + b] = run;
      cursor[W.bbase + b] = run;
      run += C[b];
    }
  }
}

__global__ void __launch_bounds__(256) k_msm_scatter(int N, int nw, const int32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ sorted) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  for (int w = 0; w < nw; w++) {
    int key = keys[(size_t)w * N + i];
    if (key == -1) continue;
    uint32_t b = (uint32_t)key & 0x7fffffffu;
    uint32_t pos = atomicAdd(&cursor[b], 1u);
    sorted[(size_t)w * N + pos] = (uint32_t)i | ((uint32_t)key & 0x80000000u);
  }
}

// window of a global bucket index (nw is small; linear scan over the table)
FTS_DEV int window_of_bucket(const MsmWindow* win, int nw, int b) {
  int w = 0;
  while (w + 1 < nw && win[w + 1].bbase <= b) w++;
  return w;
}

__global__ void __launch_bounds__(64) k_msm_buckets(int N, int nw, int NB, const MsmWindow* __restrict__ win,
                                                    const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ offsets,
                                                    const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ sorted, uint32_t* __restrict__ buckets) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= NB) return;
  const int w = window_of_bucket(win, nw, b);
  const uint32_t off = offsets[b], cnt = counts[b];
  const uint32_t* S = sorted + (size_t)w * N;
  G1J acc = g1j_identity();
  for (uint32_t t = 0; t < cnt; t++) {
    uint32_t e = S[off + t];
    acc = nl_madd_mem(acc, points + (size_t)(e & 0x7fffffffu) * 16, e >> 31);
  }
  store_g1j(buckets + (size_t)b * 24, acc);
}

// running-sum reduction of MSM_SEG consecutive buckets of one window:
// sum_j (j+1) B_j for the window-local bucket indices j of the segment
__global__ void __launch_bounds__(64) k_msm_segments(int nw, int NS, const MsmWindow* __restrict__ win,
                                                     const uint32_t* __restrict__ buckets,
                                                     uint32_t* __restrict__ segs, uint32_t* __restrict__ scratch) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= NS) return;
  int w = 0;
  while (w + 1 < nw && win[w + 1].sbase <= g) w++;
  const MsmWindow W = win[w];
  const int nb = 1 << (W.width - 1);
  const int s = g - W.sbase;
  const int lo = s * MSM_SEG, cnt = (nb - lo) < MSM_SEG ? (nb - lo) : MSM_SEG;
  const uint32_t* Bk = buckets + ((size_t)W.bbase + lo) * 24;
  uint32_t* scr = scratch + (size_t)g * 24;
  G1J sum = g1j_identity(), acc = g1j_identity();
  for (int j = cnt - 1; j >= 0; j--) {
    sum = nl_add_mem(sum, Bk + j * 24, 0);
    store_g1j(scr, sum);
    acc = nl_add_mem(acc, scr, 0);
  }
  uint32_t m = (uint32_t)lo;  // bucket lo+j carries multiplier lo + j + 1
  if (m) {
    store_g1j(scr, sum);
    G1J t = g1j_identity();
    for (int bit = 31 - __builtin_clz(m); bit >= 0; bit--) {
      t = nl_dbl(t);
      if ((m >> bit) & 1u) t = nl_add_mem(t, scr, 0);
    }
    store_g1j(scr, t);
    acc = nl_add_mem(acc, scr, 0);
  }
  store_g1j(segs + (size_t)g * 24, acc);
}

// tree over the segments of one window (block per window, 64 threads)
__global__ void __launch_bounds__(64) k_msm_windows(const MsmWindow* __restrict__ win, const uint32_t* __restrict__ segs,
                                                    uint32_t* __restrict__ wins) {
  __shared__ uint32_t sh[64 * 24];
  const int t = threadIdx.x;
  const MsmWindow W = win[blockIdx.x];
  const int nseg = ((1 << (W.width - 1)) + MSM_SEG - 1) / MSM_SEG;
  const uint32_t* S = segs + (size_t)W.sbase * 24;
  G1J acc = g1j_identity();
  for (int s = t; s < nseg; s += 64) acc = nl_add_mem(acc, S + s * 24, 0);
  store_g1j(sh + t * 24, acc);
  __syncthreads();
  for (int half = 32; half >= 1; half >>= 1) {
    if (t < half) acc = nl_add_mem(acc, sh + (t + half) * 24, 0);
    __syncthreads();
    if (t < half) store_g1j(sh + t * 24, acc);
    __syncthreads();
  }
  if (t == 0) store_g1j(wins + (size_t)blockIdx.x * 24, acc);
}

// result = sum_w 2^off_w W_w (+ extra Jacobian points, e.g. the fixed-base part)
__global__ void k_msm_final(int nw, const MsmWindow* __restrict__ win, const uint32_t* __restrict__ wins,
                            const uint32_t* __restrict__ extra, int nextra, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G1J acc = load_g1j(wins + (size_t)(nw - 1) * 24);
  for (int w = nw - 2; w >= 0; w--) {
    const int shift = win[w + 1].off - win[w].off;
    for (int q = 0; q < shift; q++) acc = nl_dbl(acc);
    acc = nl_add_mem(acc, wins + (size_t)w * 24, 0);
  }
  for (int e = 0; e < nextra; e++) acc = nl_add_mem(acc, extra + (size_t)e * 24, 0);
  store_g1j(out, acc);
}

#define FTS_LAUNCH(kern, nthreads, bs, stream, ...)                                   \
  do {                                                                                \
    size_t nt_ = (size_t)(nthreads);                                                  \
    if (nt_) hipLaunchKernelGGL(kern, dim3((unsigned)((nt_ + (bs)-1) / (bs))), dim3(bs), 0, stream, __VA_ARGS__); \
  } while (0)

// scratch: NS * 24 words.  p.d_win must already hold p.win (uploaded by the caller).
void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s, Timeline* tl) {
  (void)hipMemsetAsync(p.counts, 0, (size_t)p.NB * 4, s);
  FTS_LAUNCH(k_msm_digits, p.N, 256, s, p.N, p.nw, p.d_win, scalars, p.keys, p.counts);
  if (tl) tl->mark("k_msm_digits", s);
  hipLaunchKernelGGL(k_msm_scan, dim3(p.nw), dim3(256), 0, s, p.d_win, p.counts, p.offsets, p.cursor);
  if (tl) tl->mark("k_msm_scan", s);
  FTS_LAUNCH(k_msm_scatter, p.N, 256, s, p.N, p.nw, p.keys, p.cursor, p.sorted);
  if (tl) tl->mark("k_msm_scatter", s);
  FTS_LAUNCH(k_msm_buckets, p.NB, 64, s, p.N, p.nw, p.NB, p.d_win, points, p.offsets, p.counts, p.sorted, p.buckets);
  if (tl) tl->mark("k_msm_buckets", s);
  FTS_LAUNCH(k_msm_segments, p.NS, 64, s, p.nw, p.NS, p.d_win, p.buckets, p.segs, scratch);
  if (tl) tl->mark("k_msm_segments", s);
  hipLaunchKernelGGL(k_msm_windows, dim3(p.nw), dim3(64), 0, s, p.d_win, p.segs, p.wins);
  if (tl) tl->mark("k_msm_windows", s);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, s, p.nw, p.d_win, p.wins, extra, nextra, p.out);
  if (tl) tl->mark("k_msm_final", s);
}

}  // namespace fts
