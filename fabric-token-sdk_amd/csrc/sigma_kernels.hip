// Sigma-proof kernels: TypeAndSum (transfers) and SameType (issues).
//
//   k_sig_decode   (point)         NewG1FromBytes checks on CT / inputs / outputs / tokens
//   k_sig_prep     (action)        in'_i = In_i - CT, out'_j = Out_j - CT, sum = sum in' - sum out'
//                                  (transfer/typeandsum.go:241-258); V_j = out'_j feeds the
//                                  range-proof batch (transfer.go:171-185, issue/verifier.go:44-49)
//   k_sig_fixed    (action, term)  fixed-base products (ped0/1/2 tables; joint pairs in one accumulator)
//   k_sig_var      (action, term)  variable-base products c * P (GLV, one chain per lane)
//   k_sig_finish   (action)        inCom_i, sumCom, typeCom (typeandsum.go:249-265) or
//                                  com (sametype.go:169-171), exact affine, hex transcript,
//                                  SHA-256, Zr.Equals against the proof's challenge
#include "device/g1.hpp"
#include "device/fixed_base.hpp"
#include "device/glv.hpp"
#include "device/helpers.hpp"
#include "device/rp_kernels.hpp"
#include "device/sigma.hpp"
#include "device/transcript.hpp"
#include "../../include/fts_gpu.h"

namespace fts {

__global__ void __launch_bounds__(256) k_sig_decode(int npts, const uint8_t* __restrict__ raw,
                                                    const int32_t* __restrict__ owner, uint32_t* __restrict__ pts,
                                                    int32_t* __restrict__ status) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= npts) return;
  G1A a;
  if (!decode_point(raw + (size_t)gid * 64, a)) status[owner[gid]] = FTS_E_MALFORMED;
  store_g1a(pts + (size_t)gid * 16, a);
}

// aff / jac layout per action (from aff_off): TAS [in' (n_in), out' (n_out), sum, inCom (n_in), typeCom, sumCom]
//                                             ST  [V (n_out), com]
// Every per-action point is computed Jacobian into jac, then ALL slots of the
// batch are normalised at once (k_rp_normalize: one field inversion per 1,024
// points instead of one per action).
// lane per action: the primes In_i - CT, Out_j - CT and (TAS) their sum (typeandsum.go:240-252)
__global__ void __launch_bounds__(64) k_sig_prep(int A, const SigAction* __restrict__ act,
                                                 const uint32_t* __restrict__ pts, const int32_t* __restrict__ status,
                                                 const int32_t* __restrict__ aff_off, uint32_t* __restrict__ jscr) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || status[a] != 0) return;
  const SigAction ac = act[a];
  const uint32_t* P = pts + (size_t)ac.pt_off * 16;
  uint32_t* J = jscr + (size_t)aff_off[a] * 24;
  const int nin = ac.kind == SIG_TAS ? ac.n_in : 0;
  const int m = nin + ac.n_out;
  G1J sum = g1j_identity();
  for (int i = 0; i < m; i++) {
    G1J d = g1j_from_affine(load_g1a(P + (1 + i) * 16));
    d = nl_madd_mem(d, P, 1);  // - CT
    store_g1j(J + i * 24, d);
    if (ac.kind == SIG_TAS) sum = nl_add_mem(sum, J + i * 24, i >= nin);
  }
  if (ac.kind == SIG_TAS) store_g1j(J + m * 24, sum);
}

// lane per action: the range proofs' V_j = Out_j - CT (affine) into the rp batch's raw V slots
__global__ void __launch_bounds__(64) k_sig_vslots(int A, const SigAction* __restrict__ act,
                                                   const int32_t* __restrict__ status, const uint32_t* __restrict__ aff,
                                                   const int32_t* __restrict__ aff_off, uint8_t* __restrict__ rp_raw,
                                                   int rp_k) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || status[a] != 0) return;
  const SigAction ac = act[a];
  if (ac.rp_base < 0) return;
  const uint32_t* F = aff + (size_t)aff_off[a] * 16;
  const int nin = ac.kind == SIG_TAS ? ac.n_in : 0;
  const int npts_rp = rp_npts(rp_k);
  const int nv = ac.n_out < ac.rp_count ? ac.n_out : ac.rp_count;
  for (int j = 0; j < nv; j++)
    store_point_be(rp_raw + ((size_t)(ac.rp_base + j) * npts_rp + RP_PT_V) * 64, load_g1a(F + (nin + j) * 16));
}

// lane per action whose sigma proof failed: its range proofs leave the batch
// check (their verdicts are never observable: the TypeAndSum / SameType error
// wins, transfer.go:192-196, issue/verifier.go:40-43).  Only the exclusion mask
// is written here (the exact phase reads the range proofs' status concurrently);
// k_rlc_prep drops the proofs from the check and k_rlc_finalize marks them NOT_RUN.
__global__ void __launch_bounds__(256) k_sig_exclude(int A, const SigAction* __restrict__ act,
                                                     const int32_t* __restrict__ status, int32_t* __restrict__ rp_excl) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || status[a] == 0) return;
  const SigAction ac = act[a];
  if (ac.rp_base < 0) return;
  for (int j = 0; j < ac.rp_count; j++) rp_excl[ac.rp_base + j] = 1;
}

// The sigma proofs' products, one lane per (action, term) work item.  The work
// list holds every fixed-base term first (items [0, nfix)), then every
// variable-base term, and each kind has its own kernel: the fixed-base one is
// table lookups + mixed additions only (fb_mul / fb_mul2 inlined), the variable-
// base one one inlined GLV chain.  One kernel with both paths kept an out-of-line
// fixed-base product (the call ABI spilled the accumulator: 416 B of scratch per
// lane) and ran at 45 % VALU busy, 0.33 of the MAD peak (round 6 PMC).
FTS_DEV Scalar sig_canon(const uint32_t* p) {
  Scalar s;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = p[i];
  return s;
}

__global__ void __launch_bounds__(64) k_sig_fixed(int nfix, const int2* __restrict__ work,
                                                  const SigAction* __restrict__ act, const uint32_t* __restrict__ sc,
                                                  const int32_t* __restrict__ status,
                                                  const uint32_t* __restrict__ tables, int n,
                                                  uint32_t* __restrict__ terms) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nfix) return;
  const int a = work[gid].x, t = work[gid].y;
  if (status[a] != 0) return;
  const SigAction ac = act[a];
  const uint32_t* S = sc + (size_t)ac.sc_off * 8;
  const uint32_t* t_ped0 = tables + (size_t)tb_ped0(n) * FB_WORDS_PER_BASE;
  const uint32_t* t_ped1 = tables + (size_t)tb_G(n) * FB_WORDS_PER_BASE;
  const uint32_t* t_ped2 = tables + (size_t)tb_H(n) * FB_WORDS_PER_BASE;
  G1J r;
  if (ac.kind == SIG_TAS) {
    const int N = ac.n_in;
    if (t < 2 * N)  // iv_i ped1 + ibf_i ped2   (t even)
      r = fb_mul2(t_ped1, sig_canon(S + (TAS_SC_IV + (t >> 1)) * 8), t_ped2, sig_canon(S + (TAS_SC_IV + N + (t >> 1)) * 8));
    else if (t == 2 * N)  // EqualityOfSum ped2
      r = fb_mul(t_ped2, sig_canon(S + TAS_SC_EQ * 8));
    else  // Type ped0 + TBF ped2   (t == 2N + 2)
      r = fb_mul2(t_ped0, sig_canon(S + TAS_SC_TYPE * 8), t_ped2, sig_canon(S + TAS_SC_TBF * 8));
  } else {  // Type ped0 + BF ped2   (t == 0)
    r = fb_mul2(t_ped0, sig_canon(S + ST_SC_TYPE * 8), t_ped2, sig_canon(S + ST_SC_BF * 8));
  }
  store_g1j(terms + (size_t)(ac.term_off + t) * 24, r);
}

__global__ void __launch_bounds__(64) k_sig_var(int nfix, int nwork, const int2* __restrict__ work,
                                                const SigAction* __restrict__ act, const uint32_t* __restrict__ pts,
                                                const uint32_t* __restrict__ sc, const int32_t* __restrict__ status,
                                                const uint32_t* __restrict__ aff, const int32_t* __restrict__ aff_off,
                                                uint32_t* __restrict__ terms, uint32_t* __restrict__ scratch) {
  const int gid = nfix + blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nwork) return;
  const int a = work[gid].x, t = work[gid].y;
  if (status[a] != 0) return;
  const SigAction ac = act[a];
  const uint32_t* S = sc + (size_t)ac.sc_off * 8;
  const uint32_t* F = aff + (size_t)aff_off[a] * 16;
  // c in'_i (t = 2i + 1), c sum (t = 2N + 1), c CT (t = 2N + 3); ST: c CT (t = 1)
  G1A vp;
  Scalar vk;
  if (ac.kind == SIG_TAS) {
    const int N = ac.n_in;
    vk = sig_canon(S + TAS_SC_CHAL * 8);
    if (t < 2 * N) vp = load_g1a(F + (t >> 1) * 16);
    else if (t == 2 * N + 1) vp = load_g1a(F + (N + ac.n_out) * 16);
    else vp = load_g1a(pts + (size_t)ac.pt_off * 16);
  } else {
    vk = sig_canon(S + ST_SC_CHAL * 8);
    vp = load_g1a(pts + (size_t)ac.pt_off * 16);
  }
  // the lane's affine table (glv.hpp CTab8, 320 words per lane, rows coalesced
  // across lanes): mixed additions in the chain
  const CTab8 T{scratch, (size_t)nwork, (size_t)gid};
  store_g1j(terms + (size_t)(ac.term_off + t) * 24, glv_mul_ctab8(T, vp, vk));
}

FTS_DEV void put_hex_aff(uint8_t* msg, int idx, const uint32_t* aff_pt, bool sep) {
  G1A p = load_g1a(aff_pt);
  uint32_t pw[16];
  g1_mont_to_be_words(p.x, p.y, pw);
  put_hex_record(msg, 130u * idx, pw, sep);
}

// lane per action: the transcript commitments (Jacobian) from the terms
__global__ void __launch_bounds__(64) k_sig_coms(int A, const SigAction* __restrict__ act,
                                                 const int32_t* __restrict__ status, const uint32_t* __restrict__ terms,
                                                 const int32_t* __restrict__ aff_off, uint32_t* __restrict__ jscr) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || status[a] != 0) return;
  const SigAction ac = act[a];
  const uint32_t* T = terms + (size_t)ac.term_off * 24;
  uint32_t* J = jscr + (size_t)aff_off[a] * 24;
  if (ac.kind == SIG_TAS) {
    const int N = ac.n_in, M = ac.n_out;
    const int c0 = N + M + 1;  // first commitment slot
    for (int i = 0; i < N; i++) store_g1j(J + (c0 + i) * 24, nl_add_mem(load_g1j(T + (2 * i) * 24), T + (2 * i + 1) * 24, 1));
    store_g1j(J + (c0 + N) * 24, nl_add_mem(load_g1j(T + (2 * N + 2) * 24), T + (2 * N + 3) * 24, 1));  // typeCom
    store_g1j(J + (c0 + N + 1) * 24, nl_add_mem(load_g1j(T + (2 * N) * 24), T + (2 * N + 1) * 24, 1));  // sumCom
  } else {
    store_g1j(J + ac.n_out * 24, nl_add_mem(load_g1j(T), T + 24, 1));
  }
}

// lane per action: transcript (hex of the affine points) + SHA-256 + challenge compare
__global__ void __launch_bounds__(64) k_sig_finish(int A, const SigAction* __restrict__ act,
                                                   const uint32_t* __restrict__ pts, const uint32_t* __restrict__ sc,
                                                   int32_t* __restrict__ status, const uint32_t* __restrict__ aff,
                                                   const int32_t* __restrict__ aff_off, uint8_t* __restrict__ msgs) {
  int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A || status[a] != 0) return;
  const SigAction ac = act[a];
  const uint32_t* F = aff + (size_t)aff_off[a] * 16;
  const uint32_t* CT = pts + (size_t)ac.pt_off * 16;
  uint8_t* msg = msgs + ac.msg_off;
  const uint32_t* S = sc + (size_t)ac.sc_off * 8;
  int np;
  const uint32_t* chal;
  if (ac.kind == SIG_TAS) {
    const int N = ac.n_in, M = ac.n_out;
    const int c0 = N + M + 1;  // first commitment slot
    // Arr(inComs, typeCom, sumCom, in'..., out'..., CT, sum)     typeandsum.go:267
    int idx = 0;
    np = 2 * N + M + 4;
    for (int i = 0; i < N + 2; i++, idx++) put_hex_aff(msg, idx, F + (c0 + i) * 16, true);
    for (int i = 0; i < N + M; i++, idx++) put_hex_aff(msg, idx, F + i * 16, true);
    put_hex_aff(msg, idx++, CT, true);
    put_hex_aff(msg, idx++, F + (N + M) * 16, false);
    chal = S + TAS_SC_CHAL * 8;
  } else {
    const int M = ac.n_out;
    put_hex_aff(msg, 0, CT, true);  // Arr(CT, com)   sametype.go:174
    put_hex_aff(msg, 1, F + M * 16, false);
    np = 2;
    chal = S + ST_SC_CHAL * 8;
  }
  uint32_t len = 130u * np - 2u;
  write_sha_padding_u16(msg, len);
  uint32_t st[8];
  sha256_blocks(msg, sha_blocks(len), st);
  Fr h = digest_to_fr(st);
  bool eq = ac.chal_canonical != 0;
#pragma unroll
  for (int i = 0; i < 8; i++) eq = eq && (h.v[i] == chal[i]);
  status[a] = eq ? FTS_OK : (ac.kind == SIG_TAS ? FTS_E_TAS_INVALID : FTS_E_ST_INVALID);
}

#define FTS_LAUNCH(kern, nthreads, bs, stream, ...)                                   \
  do {                                                                                \
    size_t nt_ = (size_t)(nthreads);                                                  \
    if (nt_) hipLaunchKernelGGL(kern, dim3((unsigned)((nt_ + (bs)-1) / (bs))), dim3(bs), 0, stream, __VA_ARGS__); \
  } while (0)

// batch affine normalisation (rp_kernels.hip): all naff slots of the sigma batch
void launch_normalize_all(int total, const uint32_t* jac, uint32_t* aff, hipStream_t s);

// phase 1 (before the range-proof batch): decode + primes (writes the rp V slots)
void launch_sig_prep(const SigBatchDev& d, hipStream_t s) {
  FTS_LAUNCH(k_sig_decode, d.npts, 256, s, d.npts, d.raw, d.pt_owner, d.pts, d.status);
  FTS_LAUNCH(k_sig_prep, d.A, 64, s, d.A, d.act, d.pts, d.status, d.aff_off, d.jac);
  launch_normalize_all(d.naff, d.jac, d.aff, s);
  if (d.rp_raw) FTS_LAUNCH(k_sig_vslots, d.A, 64, s, d.A, d.act, d.status, d.aff, d.aff_off, d.rp_raw, d.rp_k);
}
// phase 2: sigma equations (independent of the range proofs)
void launch_sig_finish(const SigBatchDev& d, const uint32_t* tables, int n, hipStream_t s) {
  FTS_LAUNCH(k_sig_fixed, d.nfix, 64, s, d.nfix, d.work, d.act, d.sc, d.status, tables, n, d.terms);
  FTS_LAUNCH(k_sig_var, d.nwork - d.nfix, 64, s, d.nfix, d.nwork, d.work, d.act, d.pts, d.sc, d.status, d.aff,
             d.aff_off, d.terms, d.scratch);
  FTS_LAUNCH(k_sig_coms, d.A, 64, s, d.A, d.act, d.status, d.terms, d.aff_off, d.jac);
  launch_normalize_all(d.naff, d.jac, d.aff, s);
  FTS_LAUNCH(k_sig_finish, d.A, 64, s, d.A, d.act, d.pts, d.sc, d.status, d.aff, d.aff_off, d.msgs);
}
// the range proofs of actions whose sigma proof failed leave the batch check
void launch_sig_exclude(const SigBatchDev& d, int32_t* rp_excl, hipStream_t s) {
  FTS_LAUNCH(k_sig_exclude, d.A, 256, s, d.A, d.act, d.status, rp_excl);
}

}  // namespace fts
