// Pippenger bucket MSM on BN254 G1 (see device/msm.hpp for the plan layout).
//
// Used by the random-linear-combination batch check of the range proofs
// (SURVEY Appendix B): one MSM over the per-proof variable points
// (T1, T2, V, com, L_j, R_j) replaces the per-proof final equations of
// bulletproof.go:314-324 and ipa.go:254-259.  Also exposed as
// fts_msm_g1 (BASELINE config C3 microbenchmark).
#include "device/g1.hpp"
#include "device/helpers.hpp"
#include "device/msm.hpp"

namespace fts {

__global__ void __launch_bounds__(256) k_msm_digits(int N, int c, int nw, const uint32_t* __restrict__ scalars,
                                                    int32_t* __restrict__ keys, uint32_t* __restrict__ counts) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int nb = 1 << (c - 1);
  uint32_t s[8];
#pragma unroll
  for (int q = 0; q < 8; q++) s[q] = scalars[(size_t)i * 8 + q];
  int carry = 0;
  const uint32_t mask = (1u << c) - 1u;
  for (int w = 0; w < nw; w++) {
    int d = (int)(s[0] & mask) + carry;
    // shift the 256-bit scalar right by c (c <= 16)
#pragma unroll
    for (int q = 0; q < 7; q++) s[q] = (s[q] >> c) | (s[q + 1] << (32 - c));
    s[7] >>= c;
    carry = d > (nb);
    d = carry ? d - (1 << c) : d;
    int key = -1;
    if (d != 0) {
      int b = (d < 0 ? -d : d) - 1;
      key = d < 0 ? (b | (int)0x80000000) : b;
      atomicAdd(&counts[(size_t)w * nb + b], 1u);
    }
    keys[(size_t)w * N + i] = key;
  }
}

// exclusive scan of counts[w][0..nb) -> offsets, cursor (one block per window)
__global__ void __launch_bounds__(256) k_msm_scan(int nb, const uint32_t* __restrict__ counts,
                                                  uint32_t* __restrict__ offsets, uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[256];
  const int w = blockIdx.x, t = threadIdx.x;
  const uint32_t* C = counts + (size_t)w * nb;
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
  uint32_t run = part[t] - loc;  // exclusive prefix of this thread's chunk
  for (int j = 0; j < per; j++) {
    int b = t * per + j;
    if (b < nb) {
      offsets[(size_t)w * nb + b] = run;
      cursor[(size_t)w * nb + b] = run;
      run += C[b];
    }
  }
}

__global__ void __launch_bounds__(256) k_msm_scatter(int N, int nb, int nw, const int32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ sorted) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  for (int w = 0; w < nw; w++) {
    int key = keys[(size_t)w * N + i];
    if (key == -1) continue;
    uint32_t b = (uint32_t)key & 0x7fffffffu;
    uint32_t pos = atomicAdd(&cursor[(size_t)w * nb + b], 1u);
    sorted[(size_t)w * N + pos] = (uint32_t)i | ((uint32_t)key & 0x80000000u);
  }
}

__global__ void __launch_bounds__(64) k_msm_buckets(int N, int nb, int nw, const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ offsets,
                                                    const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ sorted, uint32_t* __restrict__ buckets) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nw * nb) return;
  const int w = gid / nb;
  const uint32_t off = offsets[gid], cnt = counts[gid];
  const uint32_t* S = sorted + (size_t)w * N;
  G1J acc = g1j_identity();
  for (uint32_t t = 0; t < cnt; t++) {
    uint32_t e = S[off + t];
    acc = nl_madd_mem(acc, points + (size_t)(e & 0x7fffffffu) * 16, e >> 31);
  }
  store_g1j(buckets + (size_t)gid * 24, acc);
}

// running-sum reduction of `seg` consecutive buckets: sum_{j in seg} (j+1) B_j
__global__ void __launch_bounds__(64) k_msm_segments(int nb, int nw, int seg, const uint32_t* __restrict__ buckets,
                                                     uint32_t* __restrict__ segs, uint32_t* __restrict__ scratch) {
  const int nseg = nb / seg;
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nw * nseg) return;
  const int w = gid / nseg, s = gid % nseg;
  const uint32_t* Bk = buckets + ((size_t)w * nb + (size_t)s * seg) * 24;
  uint32_t* scr = scratch + (size_t)gid * 24;
  G1J sum = g1j_identity(), acc = g1j_identity();
  for (int j = seg - 1; j >= 0; j--) {
    sum = nl_add_mem(sum, Bk + j * 24, 0);
    store_g1j(scr, sum);
    acc = nl_add_mem(acc, scr, 0);
  }
  // + (s * seg) * sum   (bucket j of this segment carries multiplier s*seg + j + 1)
  uint32_t m = (uint32_t)(s * seg);
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
  store_g1j(segs + (size_t)gid * 24, acc);
}

// tree over the segments of one window (block per window, 64 threads)
__global__ void __launch_bounds__(64) k_msm_windows(int nseg, const uint32_t* __restrict__ segs,
                                                    uint32_t* __restrict__ wins, uint32_t* __restrict__ scratch) {
  __shared__ uint32_t sh[64 * 24];
  const int w = blockIdx.x, t = threadIdx.x;
  const uint32_t* S = segs + (size_t)w * nseg * 24;
  G1J acc = g1j_identity();
  for (int s = t; s < nseg; s += 64) acc = nl_add_mem(acc, S + s * 24, 0);
  store_g1j(sh + t * 24, acc);
  __syncthreads();
  for (int half = 32; half >= 1; half >>= 1) {
    if (t < half) {
      acc = nl_add_mem(acc, sh + (t + half) * 24, 0);
    }
    __syncthreads();
    if (t < half) store_g1j(sh + t * 24, acc);
    __syncthreads();
  }
  if (t == 0) store_g1j(wins + (size_t)w * 24, acc);
}

// result = sum_w 2^(c w) W_w (+ extra Jacobian points, e.g. the fixed-base part)
__global__ void k_msm_final(int nw, int c, const uint32_t* __restrict__ wins, const uint32_t* __restrict__ extra,
                            int nextra, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G1J acc = load_g1j(wins + (size_t)(nw - 1) * 24);
  for (int w = nw - 2; w >= 0; w--) {
    for (int q = 0; q < c; q++) acc = nl_dbl(acc);
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

// scratch: nw * nseg * 24 words
void launch_msm(const MsmPlan& p, const uint32_t* points, const uint32_t* scalars, const uint32_t* extra, int nextra,
                uint32_t* scratch, hipStream_t s) {
  hipMemsetAsync(p.counts, 0, (size_t)p.nw * p.nb * 4, s);
  FTS_LAUNCH(k_msm_digits, p.N, 256, s, p.N, p.c, p.nw, scalars, p.keys, p.counts);
  hipLaunchKernelGGL(k_msm_scan, dim3(p.nw), dim3(256), 0, s, p.nb, p.counts, p.offsets, p.cursor);
  FTS_LAUNCH(k_msm_scatter, p.N, 256, s, p.N, p.nb, p.nw, p.keys, p.cursor, p.sorted);
  FTS_LAUNCH(k_msm_buckets, p.nw * p.nb, 64, s, p.N, p.nb, p.nw, points, p.offsets, p.counts, p.sorted, p.buckets);
  FTS_LAUNCH(k_msm_segments, p.nw * p.nseg, 64, s, p.nb, p.nw, p.seg, p.buckets, p.segs, scratch);
  hipLaunchKernelGGL(k_msm_windows, dim3(p.nw), dim3(64), 0, s, p.nseg, p.segs, p.wins, scratch);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, s, p.nw, p.c, p.wins, extra, nextra, p.out);
}

}  // namespace fts
