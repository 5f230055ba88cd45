// Pippenger bucket MSM on BN254 G1: layout shared by msm.hip and the host.
//
// sum_i k_i * P_i over N affine points (Montgomery, 16 words each, identity =
// (0,0)) and canonical scalars (8 LE words each, < r < 2^254).
// GLV (device/glv.hpp): every scalar is split as k = k1 + k2 lambda with
// |k1|, |k2| < 2^126, so the MSM runs over NV = 2N virtual points
// (P_i with k1, phi(P_i) with k2; signs folded into the digit signs) with
// 127-bit scalars: half the windows and half the final doubling chain.
// Signed windows: window w covers bits [off_w, off_w + width_w); digit d in
// [-2^(width-1), 2^(width-1)] and bucket |d|-1 collects +-P.  The 127
// covered bits are split into nw windows of width c or c-1 (balanced), so
// every window has ~NV / 2^(c-1) points per bucket.
// Bucket accumulation is chunked (<= MSM_CH points per lane) so a bucket that
// attracts many points (adversarial or low-entropy scalars) is summed by
// several lanes instead of one long dependent chain.
// Kernels (msm.hip), all on one stream:
//   k_msm_digits      (point)          recode + bucket histogram (atomics)
//   k_msm_scan1/2/3   (bucket)         global exclusive scans over all buckets:
//                                      entry offsets into one flat sorted array
//                                      and the chunk map (3-pass block scan)
//   k_msm_scatter     (point)          counting-sort scatter of (index|sign)
//   k_msm_chunks      (chunk)          <= MSM_CH mixed additions from HBM
//   k_msm_bucket_sum  (bucket)         sum of the bucket's chunk partials
//   k_msm_segments    (segment)        running-sum reduction of MSM_SEG buckets
//   k_msm_windows     (window+1, part) LDS tree over <= MSM_WIN_ITEMS segments
//                                      (window nw: the extra fixed points)
//   k_msm_final       (1 wave)         per-window sum of the parts, then
//                                      Horner over the windows + extras
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

constexpr int MSM_MAX_WINDOWS = 64;
constexpr int MSM_SEG = 8;   // buckets per running-sum segment
constexpr int MSM_CH = 8;    // smallest bucket-accumulation chunk (points per lane); plans pick 8..64 (MsmPlan::ch)
constexpr int MSM_SCAN_ITEMS = 1024;  // buckets per block of the scan passes
constexpr int MSM_WIN_ITEMS = 1024;   // segments per block of k_msm_windows

struct MsmWindow {
  int32_t width;   // bits
  int32_t off;     // first bit
  int32_t bbase;   // first bucket (global index)
  int32_t sbase;   // first segment (global index)
  int32_t cbase;   // first chunk slot (global index); NV/MSM_CH + nb slots reserved
  int32_t pad[3];
};

constexpr int MSM_BITS = 127;  // magnitude < 2^126 + sign-recoding carry

// Grouped MSMs (G > 1): G independent sums over consecutive ranges of ptsg points
// each (point i belongs to group i / ptsg), sharing one digit / sort / bucket
// pass: bucket (g, window, digit) = g * NBg + window base + |digit| - 1, and the
// reduction kernels run per (group, window).  Used by the batch check's group
// test (one MSM gives every group's partial random linear combination).
// Optional indirection (sel != nullptr): point i is input point
// sel[i / sel_pts] * sel_pts + i % sel_pts, or absent (zero) if that entry is -1.
struct MsmPlan {
  int N;           // points (including absent padding points of a grouped plan)
  int NV;          // virtual points (2N)
  int nw;
  int NB;          // total buckets (G * NBg)
  int NS;          // total segments (G * NSg)
  int NC;          // total chunk slots
  int NBLK;        // scan blocks (ceil(NB / MSM_SCAN_ITEMS))
  int WB;          // k_msm_windows blocks per window
  int G;           // groups (1: one MSM)
  int ptsg;        // points per group
  int NBg, NSg;    // buckets / segments per group
  int ch;          // points per bucket-accumulation chunk (MSM_CH)
  // the two-level counting sort (msm.hip k_rs_*, <= 32 KB LDS per 256-thread
  // block, no device-scope atomics) instead of k_msm_digits' global atomics and
  // k_msm_scatter's random writes, where the plan allows it (one group, windows
  // of >= 128 buckets); false forces k_msm_digits (FTS_MSM_SORT=0, A/B)
  bool local_sort;
  const int32_t* sel;  // device: proof indirection (grouped fallback), or nullptr
  int sel_pts;         // points per proof of the indirection
  MsmWindow win[MSM_MAX_WINDOWS];  // host copy
  MsmWindow* d_win;                // device copy
  int32_t* keys;      // [nw][NV] bucket (global) index | sign<<31, or -1
  uint32_t* counts;   // [NB]
  uint32_t* offsets;  // [NB] (within the window's sorted range)
  uint32_t* cursor;   // [nw][NV] rank of each (window, virtual point) entry within its bucket
  uint32_t* chunk_off;// [NB] first chunk slot of the bucket (global)
  int32_t* chunk_bkt; // [NC] bucket of a chunk slot, -1 if unused
  uint32_t* sorted;   // [nw][NV] virtual index | sign << 31
  uint32_t* partials; // [NC][24] Jacobian
  uint32_t* buckets;  // [NB][24] Jacobian
  uint32_t* segs;     // [NS][24]
  uint32_t* wins;     // [nw + 1][24] (slot nw: sum of the extra points)
  uint32_t* out;      // [G][24] results (Jacobian)
  uint32_t* scratch;  // >= msm_scratch_words(p): scan block sums + window parts
};

inline size_t msm_scratch_words(const MsmPlan& p) {
  return (size_t)2 * p.NBLK + 2 + (size_t)p.G * (p.nw + 1) * p.WB * 24;
}

// Field-product count of the bucket phase for window width c (host cost model)
inline double msm_cost(int N, int c) {
  int nw = (MSM_BITS + c - 1) / c;
  return (double)nw * ((double)N * 11.0 + (double)(1 << c) * 16.0);
}

// G groups of ptsg points (N = G * ptsg, or fewer in the last group); the window
// width minimises the per-group bucket cost up to maxc (the context's FTS_MSM_MAXC:
// narrower windows trade bucket-phase work for a shorter reduction)
inline void msm_layout_groups(int N, int G, int ptsg, MsmPlan& p, int maxc = 16) {
  const int NV = 2 * N, NVg = 2 * ptsg;
  int best = 4;
  for (int c = 5; c <= maxc; c++)
    if (msm_cost(NVg, c) < msm_cost(NVg, best)) best = c;
  const int c = best;
  const int nw = (MSM_BITS + c - 1) / c;
  // balanced widths: (MSM_BITS mod nw) windows of ceil, the rest floor
  const int lo = MSM_BITS / nw, extra = MSM_BITS - lo * nw;
  p.nw = nw;
  int off = 0, bb = 0, sb = 0;
  for (int w = 0; w < nw; w++) {
    const int width = lo + (w < extra ? 1 : 0);
    const int nb = 1 << (width - 1);
    const int ns = (nb + MSM_SEG - 1) / MSM_SEG;
    p.win[w] = MsmWindow{width, off, bb, sb, 0, {0, 0, 0}};
    off += width;
    bb += nb;
    sb += ns;
  }
  p.G = G;
  p.ptsg = ptsg;
  p.NBg = bb;
  p.NSg = sb;
  p.NB = G * bb;
  p.NS = G * sb;
  // chunk size: MSM_CH.  Larger chunks from the average bucket load (~3 partials
  // per bucket) cut k_msm_bucket_sum 8x at 2^22 points but made k_msm_chunks
  // slower (fewer lanes in flight to hide the point gathers: 81,920-proof pass
  // 3.0 -> 6.1 ms, 512-step headline 4.77 -> 4.30 M/s); kept per plan for A/B
  p.ch = MSM_CH;
  // chunk slots: sum over buckets of ceil(count / ch) <= entries / ch + buckets
  p.NC = nw * (NV / p.ch + 1) + p.NB;
  p.NBLK = (p.NB + MSM_SCAN_ITEMS - 1) / MSM_SCAN_ITEMS;
  int maxs = 0;
  for (int w = 0; w < nw; w++) {
    const int ns = ((1 << (p.win[w].width - 1)) + MSM_SEG - 1) / MSM_SEG;
    maxs = ns > maxs ? ns : maxs;
  }
  p.WB = (maxs + MSM_WIN_ITEMS - 1) / MSM_WIN_ITEMS;
  if (p.WB < 1) p.WB = 1;
  p.N = N;
  p.NV = NV;
  p.sel = nullptr;
  p.sel_pts = 1;
  p.local_sort = true;
}
inline void msm_layout(int N, MsmPlan& p, int maxc = 16) { msm_layout_groups(N, 1, N > 0 ? N : 1, p, maxc); }
// points per bucket-accumulation chunk (and the chunk-slot count that follows)
inline void msm_set_chunk(MsmPlan& p, int ch) {
  p.ch = ch;
  p.NC = p.nw * (p.NV / ch + 1) + p.NB;
}

}  // namespace fts
