// Pippenger bucket MSM on BN254 G1: layout shared by msm.hip and the host.
//
// sum_i k_i * P_i over N affine points (Montgomery, 16 words each, identity =
// (0,0)) and canonical scalars (8 LE words each, < r < 2^254).
// Signed windows: window w covers bits [off_w, off_w + width_w); digit d in
// [-2^(width-1), 2^(width-1)] and bucket |d|-1 collects +-P_i.  Widths are c
// except the top window, which is widened (merged) when the leftover bits
// would leave it with a handful of huge buckets: every window then has
// ~N / 2^(c-1) points per bucket for uniform scalars.
// Kernels (msm.hip):
//   k_msm_digits   (point)            recode + bucket histogram (atomics)
//   k_msm_scan     (window)           exclusive prefix sum of bucket counts
//   k_msm_scatter  (point)            counting-sort scatter of (index|sign)
//   k_msm_buckets  (bucket)           bucket sums, mixed additions from HBM
//   k_msm_segments (segment)          running-sum reduction of SEG buckets
//   k_msm_windows  (window)           LDS tree over the window's segments
//   k_msm_final    (1 thread)         Horner over windows (+ extra points)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

constexpr int MSM_MAX_WINDOWS = 64;
constexpr int MSM_SEG = 16;  // buckets per running-sum segment

struct MsmWindow {
  int32_t width;   // bits
  int32_t off;     // first bit
  int32_t bbase;   // first bucket (global index)
  int32_t sbase;   // first segment (global index)
};

struct MsmPlan {
  int N;
  int nw;
  int NB;          // total buckets
  int NS;          // total segments
  MsmWindow win[MSM_MAX_WINDOWS];  // host copy
  MsmWindow* d_win;                // device copy
  int32_t* keys;     // [nw][N] bucket (global) index | sign<<31, or -1
  uint32_t* counts;  // [NB]
  uint32_t* offsets; // [NB] (within the window's sorted range)
  uint32_t* cursor;  // [NB]
  uint32_t* sorted;  // [nw][N] index | sign << 31
  uint32_t* buckets; // [NB][24] Jacobian
  uint32_t* segs;    // [NS][24]
  uint32_t* wins;    // [nw][24]
  uint32_t* out;     // [24] result (Jacobian)
};

// window layout for N points: base width c ~ log2(N) - 3; leftover top bits
// are merged into the previous window when <= 3, widths whose leftover
// would be unbalanced are skipped
inline void msm_layout(int N, MsmPlan& p) {
  int c = 4;
  while ((1 << (c + 3)) < N && c < 17) c++;
  for (;; c++) {
    int nw = (255 + c - 1) / c;
    int t = 255 - c * (nw - 1);
    if (t <= 3 || t >= c - 1 || c >= 17) break;
  }
  int nw = (255 + c - 1) / c;
  int t = 255 - c * (nw - 1);
  int widths[MSM_MAX_WINDOWS];
  for (int w = 0; w < nw; w++) widths[w] = c;
  if (t <= 3 && nw > 1) {
    nw -= 1;
    widths[nw - 1] = c + t;
  } else {
    widths[nw - 1] = t;
  }
  p.nw = nw;
  int off = 0, bb = 0, sb = 0;
  for (int w = 0; w < nw; w++) {
    int nb = 1 << (widths[w] - 1);
    int ns = (nb + MSM_SEG - 1) / MSM_SEG;
    p.win[w] = MsmWindow{widths[w], off, bb, sb};
    off += widths[w];
    bb += nb;
    sb += ns;
  }
  p.NB = bb;
  p.NS = sb;
  p.N = N;
}

}  // namespace fts
