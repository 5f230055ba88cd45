// Pippenger bucket MSM on BN254 G1: layout shared by msm.hip and the host.
//
// sum_i k_i * P_i over N affine points (Montgomery, 16 words each, identity =
// (0,0)) and canonical scalars (8 LE words each, < r).  Signed c-bit windows:
// digit d in [-2^(c-1), 2^(c-1)], bucket |d|-1 of window w collects +-P_i.
// Kernels (msm.hip):
//   k_msm_digits   (point)            recode + bucket histogram (atomics)
//   k_msm_scan     (window)           exclusive prefix sum of bucket counts
//   k_msm_scatter  (point)            counting-sort scatter of (index|sign)
//   k_msm_buckets  (window, bucket)   bucket sums, mixed additions from HBM
//   k_msm_segments (window, segment)  running-sum reduction of SEG buckets
//   k_msm_windows  (window)           LDS tree over the segments
//   k_msm_final    (1 thread)         Horner over windows (+ extra points)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

struct MsmPlan {
  int N;           // points
  int c;           // window bits
  int nw;          // windows = ceil(255 / c)
  int nb;          // buckets per window = 2^(c-1)
  int seg;         // buckets per segment
  int nseg;        // segments per window = nb / seg
  int32_t* keys;     // [nw][N] bucket index or -1
  uint32_t* counts;  // [nw][nb]
  uint32_t* offsets; // [nw][nb]
  uint32_t* cursor;  // [nw][nb]
  uint32_t* sorted;  // [nw][N] index | sign << 31
  uint32_t* buckets; // [nw][nb][24] Jacobian
  uint32_t* segs;    // [nw][nseg][24]
  uint32_t* wins;    // [nw][24]
  uint32_t* out;     // [24] result (Jacobian)
};

inline int msm_window_bits(int N) {
  int c = 4;
  while ((1 << (c + 3)) < N && c < 16) c++;
  return c;
}
inline int msm_windows(int c) { return (255 + c - 1) / c; }

}  // namespace fts
