// Layout shared by the sigma-proof kernels (TypeAndSum, SameType) and the
// host driver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

enum SigKind : int32_t { SIG_TAS = 0, SIG_ST = 1 };

// per action descriptor (one transfer or one issue)
struct SigAction {
  int32_t kind;      // SIG_TAS / SIG_ST
  int32_t n_in;      // TAS: #inputs ; ST: 0
  int32_t n_out;     // TAS: #outputs ; ST: #tokens
  int32_t pt_off;    // first point: [CT, In..., Out...] (ST: [CT, Tok...])
  int32_t sc_off;    // first scalar (8 words each)
  int32_t term_off;  // first term slot
  int32_t msg_off;   // transcript slot byte offset
  int32_t rp_base;   // first range proof of this action in the rp batch (-1: none)
  int32_t chal_canonical;  // Challenge < r and fits 32 bytes (Zr.Equals against HashToZr)
  int32_t rp_count;        // range proofs supplied for this action (V slots written: min(n_out, rp_count))
  int32_t pad[2];
};

// scalars: TAS [Type, TBF, EqSum, Chal, iv_0.., ibf_0..] ; ST [Type, BF, Chal]
constexpr int TAS_SC_TYPE = 0, TAS_SC_TBF = 1, TAS_SC_EQ = 2, TAS_SC_CHAL = 3, TAS_SC_IV = 4;
constexpr int ST_SC_TYPE = 0, ST_SC_BF = 1, ST_SC_CHAL = 2;

// k_sig_var scratch per work item: its 8-entry affine table (glv.hpp CTab8,
// 320 words) within a 16-entry Jacobian table's room + one point
constexpr int SIG_VTAB_WORDS = 16 * 24;
inline __host__ __device__ size_t sig_scratch_words(size_t nwork) { return nwork * (SIG_VTAB_WORDS + 24); }

inline __host__ __device__ int sig_nterms(int kind, int n_in) { return kind == SIG_TAS ? 2 * n_in + 4 : 2; }
// term t is a variable-base (GLV) product (k_sig_var); the others are fixed-base (k_sig_fixed)
inline __host__ __device__ bool sig_term_var(int kind, int n_in, int t) {
  return kind == SIG_TAS ? (t < 2 * n_in ? (t & 1) != 0 : (t == 2 * n_in + 1 || t == 2 * n_in + 3)) : t != 0;
}
inline __host__ __device__ int sig_nfixed(int kind, int n_in) { return kind == SIG_TAS ? n_in + 2 : 1; }
inline __host__ __device__ int sig_nscalars(int kind, int n_in) { return kind == SIG_TAS ? 4 + 2 * n_in : 3; }
// transcript points: TAS inComs(n_in), typeCom, sumCom, in'(n_in), out'(n_out), CT, sum ; ST CT, com
inline __host__ __device__ int sig_ntranscript(int kind, int n_in, int n_out) {
  return kind == SIG_TAS ? 2 * n_in + n_out + 4 : 2;
}
inline __host__ __device__ uint32_t sig_msg_slot(int kind, int n_in, int n_out) {
  uint32_t len = 130u * sig_ntranscript(kind, n_in, n_out) - 2u;
  return ((len + 9u + 63u) / 64u) * 64u;
}
// per-action affine scratch: primes (n_in + n_out + 1 sum) + transcript commitments (n_in + 2)
inline __host__ __device__ int sig_naff(int kind, int n_in, int n_out) {
  return kind == SIG_TAS ? (n_in + n_out + 1) + (n_in + 2) : (n_out + 1);
}

struct SigBatchDev {
  int A;              // #actions
  int npts;           // total points
  int naff;           // total per-action affine / Jacobian slots (aff_off of the end)
  int nwork;          // total (action, term) work items
  int nfix;           // the first nfix work items are the fixed-base terms (k_sig_fixed), the rest variable-base (k_sig_var)
  const SigAction* act;
  uint8_t* raw;       // [npts][64] raw BE
  int32_t* pt_owner;  // [npts] action index
  uint32_t* pts;      // [npts][16] affine Montgomery
  uint32_t* sc;       // scalars (canonical Fr, 8 words)
  int32_t* status;    // [A]
  int2* work;         // [nwork] (action, term)
  uint32_t* terms;    // [sum nterms][24]
  uint32_t* aff;      // per-action affine scratch [sum naff][16], offset = act.pt_off-based (see kernels)
  int32_t* aff_off;   // [A] first affine scratch slot
  uint8_t* msgs;      // transcript slots
  uint32_t* jac;      // per-action Jacobian scratch [sum naff][24] (same offsets as aff)
  uint32_t* scratch;  // sig_scratch_words(nwork): GLV lane tables + add_via temporaries
  uint8_t* rp_raw;    // rp batch raw points (V slots are written here), may be null
  int rp_k;           // rounds of the rp batch
};

}  // namespace fts
