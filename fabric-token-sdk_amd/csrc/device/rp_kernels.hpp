// Device-side layout shared by the range-proof kernels and the host driver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

// per-proof point slots (raw BE on input, affine Montgomery after decode)
//   0 T1, 1 T2, 2 C, 3 D, 4 V, 5..5+k-1 L_j, 5+k..5+2k-1 R_j
constexpr int RP_PT_T1 = 0, RP_PT_T2 = 1, RP_PT_C = 2, RP_PT_D = 3, RP_PT_V = 4, RP_PT_L = 5;
inline __host__ __device__ int rp_npts(int k) { return 5 + 2 * k; }

// per-proof scalars (canonical Fr LE limbs, host-reduced mod r)
constexpr int RP_SC_TAU = 0, RP_SC_DELTA = 1, RP_SC_IP = 2, RP_SC_A = 3, RP_SC_B = 4, RP_NSC = 5;

// per-proof challenge block (Fr, Montgomery form, 8 words each)
//   0 x, 1 x^2, 2 y, 3 y^-1, 4 z, 5 z^2, 6 polEval, 7 x0, 8.. x_j, 8+k.. x_j^-1
constexpr int CH_X = 0, CH_X2 = 1, CH_Y = 2, CH_YINV = 3, CH_Z = 4, CH_Z2 = 5, CH_POL = 6, CH_X0 = 7, CH_XJ = 8;
inline __host__ __device__ int rp_nch(int k) { return 8 + 2 * k; }

// fixed-base table slots in the context (per base: FB_WORDS_PER_BASE words)
//   0..n-1 G_i (left), n..2n-1 H_i (right), 2n G=ped1, 2n+1 H=ped2, 2n+2 P,
//   2n+3 Q, 2n+4 K = sum H_i - sum G_i, 2n+5 ped0
inline __host__ __device__ int tb_G(int n) { return 2 * n; }
inline __host__ __device__ int tb_H(int n) { return 2 * n + 1; }
inline __host__ __device__ int tb_P(int n) { return 2 * n + 2; }
inline __host__ __device__ int tb_Q(int n) { return 2 * n + 3; }
inline __host__ __device__ int tb_K(int n) { return 2 * n + 4; }
inline __host__ __device__ int tb_ped0(int n) { return 2 * n + 5; }
inline __host__ __device__ int tb_count(int n) { return 2 * n + 6; }

// x0 transcript (rp/ipa.go:200-213): DER SEQUENCE{ OCTET(array), OCTET("||"), OCTET(Zb(ip)) }
// array = 2n+2 records (H'_0..H'_{n-1}, G_0..G_{n-1}, Q, com) of 130 bytes, last w/o "||"
inline __host__ __device__ uint32_t x0_array_len(int n) { return 130u * (2u * n + 2u) - 2u; }
inline __host__ __device__ uint32_t x0_msg_len(int n) { return x0_array_len(n) + 46u; }
inline __host__ __device__ uint32_t x0_slot_bytes(int n) { return ((x0_msg_len(n) + 9u + 63u) / 64u) * 64u; }
// SHA-256 blocks [x0_cb0, x0_cb1) of the x0 message lie entirely inside the
// constant records hex(G_0) "||" ... hex(Q) "||" (bytes [8 + 130n, 8 + 130(2n+1)))
// and are read by every proof from one shared template (x0_tmpl, L2-resident);
// a proof's own slot holds only the other blocks (x0_var_bytes).
inline __host__ __device__ uint32_t x0_const_off(int n) { return 8u + 130u * n; }
inline __host__ __device__ uint32_t x0_const_end(int n) { return 8u + 130u * (2u * n + 1u); }
inline __host__ __device__ uint32_t x0_cb0(int n) { return (x0_const_off(n) + 63u) / 64u; }
inline __host__ __device__ uint32_t x0_cb1(int n) { return x0_const_end(n) / 64u; }
inline __host__ __device__ uint32_t x0_var_bytes(int n) { return x0_slot_bytes(n) - 64u * (x0_cb1(n) - x0_cb0(n)); }

// small transcripts slot (x: 258 B, y: 388 B, x_j: 258 B, z: 32 B) -> 512 B scratch each
constexpr uint32_t SMALL_SLOT = 512;

// Algorithmic cost model, in Fp/Fr Montgomery products; one
// product = 136 u32 MADs (8x32-bit FIPS/CIOS).  Every kernel launch is marked
// with the products its algorithm needs, so bench.py can report
// achieved MAD/s = products * 136 / measured kernel time.
constexpr double MADS_PER_MUL = 136.0;
constexpr double COST_MADD = 11.0;    // madd-2007-bl 7M + 4S
constexpr double COST_ADD = 16.0;     // add-2007-bl 11M + 5S
constexpr double COST_DBL = 7.0;      // dbl-2009-l 2M + 5S
// one inversion is NOT priced in products (f_inv_gcd: ~17 x 2x2-matrix-times-256-bit
// steps, a few hundred MADs): 0 keeps achieved MAD/s a lower bound
constexpr double COST_INV = 0.0;
constexpr double COST_NORM1 = COST_INV + 4.0;  // one point to affine: zi^2, x zi^2, y zi^2 zi (+ the inversion)
// fixed-base products (fixed_base.hpp): one mixed addition per signed window; a
// product computed into a fresh accumulator starts from the identity, so its first
// window is a copy (fb_mul / fb_mul_w: 15 resp. 12 real additions), a product added
// into a running accumulator (fb_mul_acc, fbw_mul_acc) pays every window
constexpr double COST_FB = 16.0 * COST_MADD;         // accumulate, 16 signed 16-bit windows
constexpr double COST_FB_FRESH = 15.0 * COST_MADD;   // fresh, 16-bit windows
constexpr double COST_FBW = 13.0 * COST_MADD;        // accumulate, 13 signed 20-bit windows (FbWide)
constexpr double COST_FBW_FRESH = 12.0 * COST_MADD;  // fresh, 20-bit windows
constexpr double COST_VB4 = 7.0 + 6.0 * COST_MADD + 256.0 * COST_DBL + 60.0 * COST_ADD;  // 4-bit var-base
constexpr double COST_VB128 = 7.0 + 6.0 * COST_ADD + 124.0 * COST_DBL + 30.0 * COST_ADD;  // GLV half (glv.hpp)
constexpr double COST_STRAUS2 = 2.0 * (7.0 + 6.0 * COST_ADD) + 124.0 * COST_DBL + 60.0 * COST_ADD;  // glv.hpp straus2_128
// glv.hpp straus2_atab over an affine lane table: build 1..8 P (P affine: 1 dbl + 6
// madd) and 1..8 S (Jacobian: 1 dbl + 6 add), Montgomery-trick normalisation of the
// 16 entries (15 + 30 + 64 products; the one inversion is not priced), 124
// doublings and ~60 mixed additions
constexpr double COST_STRAUS2_ATAB = (COST_DBL + 6.0 * COST_MADD) + (COST_DBL + 6.0 * COST_ADD) + 109.0 +
                                     124.0 * COST_DBL + 60.0 * COST_MADD;
// straus2_ctab (k_rp_com_var, per lane): the lane's half of the shared table -- 1..8
// of one point (1 dbl + 6 full additions), its normalisation with beta*x (61
// products; the one inversion is not priced) -- then 124 doublings and ~60 mixed
// additions
constexpr double COST_STRAUS2_CTAB = (COST_DBL + 6.0 * COST_ADD) + 61.0 + 124.0 * COST_DBL + 60.0 * COST_MADD;
constexpr double COST_NORM = 7.0;
     // batched affine normalisation, per point

// Per-kernel device timeline: an event is recorded on the launching stream
// after each kernel; the time of mark i is elapsed(previous event on the same
// stream, mark i).  fork()/join() record the cross-stream dependencies (their
// events start the next kernel's interval on the waiting stream).
// Marks made after fallback() (the batch check's group test and per-proof
// checks) are reported under "fb:" names, apart from the main pass's kernels.
const char* fallback_name(const char* nm);
struct Timeline {
  static constexpr int CAP = 96;
  bool in_fallback = false;
  static constexpr int MAXS = 4;
  hipEvent_t ev[CAP + 1];
  const char* name[CAP];
  double work[CAP];
  int start[CAP];
  int n = 0;
  hipStream_t sl[MAXS];
  int last[MAXS];
  int ns = 0;
  bool created = false;
  void create() {
    if (created) return;
    for (int i = 0; i <= CAP; i++) (void)hipEventCreate(&ev[i]);
    created = true;
  }
  void destroy() {
    if (!created) return;
    for (int i = 0; i <= CAP; i++) (void)hipEventDestroy(ev[i]);
    created = false;
  }
  int& last_of(hipStream_t s) {
    for (int i = 0; i < ns; i++)
      if (sl[i] == s) return last[i];
    sl[ns] = s;
    last[ns] = 0;
    return last[ns++];
  }
  void fallback() { in_fallback = true; }
  void begin(hipStream_t s) {
    n = 0;
    ns = 0;
    in_fallback = false;
    (void)hipEventRecord(ev[0], s);
    last_of(s) = 0;
  }
  void mark(const char* nm, hipStream_t s, double w) {
    if (n >= CAP) return;
    int& l = last_of(s);
    name[n] = nm && in_fallback ? fallback_name(nm) : nm;
    work[n] = w;
    start[n] = l;
    (void)hipEventRecord(ev[n + 1], s);
    l = ++n;
  }
  // `to` waits for everything issued so far on `from`
  void fork(hipStream_t from, hipStream_t to) {
    if (from == to) return;
    if (n >= CAP) {
      hipEvent_t e;
      (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
      (void)hipEventRecord(e, from);
      (void)hipStreamWaitEvent(to, e, 0);
      (void)hipEventDestroy(e);
      return;
    }
    mark(nullptr, from, 0);
    (void)hipStreamWaitEvent(to, ev[n], 0);
    mark(nullptr, to, 0);  // completes once `to` has also drained its own work
  }
};

// device buffers of one range-proof batch (filled by fts_api.cpp)
// staged batches gathered into one device pass (fts_rp_batch_verify coalescing)
constexpr int RP_GATHER_MAX = 32;
struct RpGather {
  const uint8_t* raw[RP_GATHER_MAX];
  const uint32_t* sc[RP_GATHER_MAX];
  const int32_t* status0[RP_GATHER_MAX];
  const int32_t* ipa[RP_GATHER_MAX];
  int off[RP_GATHER_MAX + 1];  // first proof of each batch in the merged pass; off[G] = B
  int G;
};

struct RpBatchDev {
  int B, n, k;
  uint8_t* raw;        // [B][5+2k][64] raw BE points (slot V from the caller)
  uint32_t* sc;        // [B][5][8] canonical Fr
  int32_t* status;     // [B] verdicts (host-parse verdicts on entry)
  int32_t* ipa_flag;   // [B] deferred IPA structural verdicts
  uint32_t* pts;       // [B][5+2k][16] affine Montgomery
  uint32_t* ch;        // [B][8+2k][8] challenges (Montgomery Fr)
  uint8_t* small_msgs; // [B][2+k][SMALL_SLOT]
  uint32_t* hpj;       // [B][n+1][24] Jacobian H'_0..H'_{n-1}, com
  uint32_t* hpa;       // [B][n+1][16] affine Montgomery
  uint8_t* hp_be;      // [B][n+1][64] canonical big-endian encodings
  uint8_t* x0_msgs;    // [B][x0_var_bytes(n)]: the message blocks outside the shared template
  uint32_t* terms;     // [B][6+2n+2k][24]
  uint32_t* scratch;   // var-base lane tables
  uint32_t* ypow;      // [n][B][8] y^-i (Montgomery Fr), i-major (coalesced over proofs)
  uint32_t* svec;      // [n][B][8] s_i = prod_j x_j^(+-1) (ipa.go:343-356 unrolled), i-major
  uint32_t* zvec;      // [n][B][8] z^2 2^i y^-i, i-major (fixed-base com terms; H_i columns of the batch check)
  void (*pre_rlc)(void* arg, hipStream_t s);  // optional hook launched on the check's stream before k_rlc_prep
  void* pre_rlc_arg;
  int com_fixed;       // 1: com by fixed-base groups + x*D on the side stream (latency path,
                       //    small passes); 0: Horner sum + joint GLV/Straus chains (work path)
  int rlc_fork = 1;    // batch check's stream forks after the fixed-base products (1) or after the challenges (0);
                       //    fts_api.cpp picks 0 on the latency path, 1 on the work path (FTS_RLC_FORK=2)
  hipEvent_t ev_coef = nullptr;  // recorded on the check's stream after k_rlc_prep (column Q on s waits for it)
  hipEvent_t ev_fx = nullptr;    // recorded on s after the fixed-base launch (rlc_fork 3: the MSM accumulation waits;
                                 // FTS_FX_SERIAL: the next pass's fixed-base launch waits)
  hipEvent_t fx_wait = nullptr;  // FTS_FX_SERIAL: s waits for it right before the fixed-base launch
  uint32_t* x0_mid = nullptr;    // [B][8] SHA-256 midstate of the x0 prefix (work path; nullptr: one-piece hash)
  int32_t* excl = nullptr;       // [B] optional: 1 = left out of the batch check (set by the pre_rlc hook), NOT_RUN
};

}  // namespace fts

#include "msm.hpp"
namespace fts {
// device buffers of the random-linear-combination check
// Per-proof coefficients (Montgomery Fr): 0 rho(ip - polEval), 1 rho tau,
// 2 rho'(ab - ip) (times x0 in the Q column), 3 rho' a, 4 rho' b, 5 rho',
// 6 -rho' z, 7 rho' delta.
constexpr int RLC_NCOEF = 8;
// fixed-base columns of the batch equation: 0 G, 1 H, 2+i G_i, 2+n+i H_i,
// 2n+2 K, 2n+3 P, 2n+4 Q (last: the only column that needs x0)
inline __host__ __device__ int rlc_ncols(int n) { return 2 * n + 5; }
// group test over many small groups (k_rlc_group_cols_small + launch_msm_small):
// groups of at most GT_SMALL_MAX proof slots; GT_CC columns per lane, whose
// fixed-base products are summed in the lane (gfix: [G][gt_nchunks][24])
constexpr int GT_SMALL_MAX = 64;
constexpr int GT_CC = 8;
inline __host__ __device__ int gt_nchunks(int n) { return (rlc_ncols(n) + GT_CC - 1) / GT_CC; }
struct RlcDev {
  uint32_t* key;     // [8] ChaCha20 key (fresh per call)
  uint32_t* msc;     // [B][5+2k][8] MSM scalars (canonical)
  uint32_t* coef;    // [B][RLC_NCOEF][8]
  uint32_t* colsum;  // [1 + 64][rlc_ncols(n)][8]: the sums, then column Q's partial sums (k_rlc_qsum)
  uint32_t* fixed;   // [rlc_ncols(n)][24]
  int32_t* flag;     // [1]
  uint32_t* msm_scratch;
  MsmPlan plan;
  // the combination per caller batch (round 5): G groups of gs proof slots sel[g gs + j]
  // (-1 = padding); plan is then a G-group MSM over sel, the column sums / products are
  // per group and the verdict is per group (gflag[g] = 1: group g closed).  G == 1: one
  // combination over the whole pass (colsum / fixed above)
  int G = 1, gs = 0;
  const int32_t* sel = nullptr;
  uint32_t* gcol = nullptr;   // [G][rlc_ncols][8]
  uint32_t* gfix = nullptr;   // [G][rlc_ncols][24]: x0-free column products (the MSM's extras), slot Q zero
  uint32_t* gqfix = nullptr;  // [G][rlc_ncols][24]: column Q's product in slot rlc_ncols - 1
  int32_t* gflag = nullptr;   // [G]
};
}  // namespace fts
