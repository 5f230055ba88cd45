// Wave-priority slots of the batch-verify pass's kernels (host and device; the
// table and s_setprio helper live in helpers.hpp).
#pragma once

namespace fts {
enum PrioSlot {
  PS_FIXED,    // k_rp_fixed_exact / k_rp_fixed_all: the pass's bulk work
  PS_HSUM,     // k_rp_hsum_chunks / _join: head of the com chain
  PS_COMVAR,   // k_rp_com_var (work path); k_rp_com_tree, k_rp_xd (latency path)
  PS_NORM,     // k_rp_x0_hdr, k_rp_normalize: H' records (x0 stream)
  PS_X0PRE,    // k_rp_x0_hash prefix (beside com)
  PS_X0TAIL,   // k_rp_x0_build, k_rp_x0_hash suffix, Q columns: the pass's tail
  PS_SORT,     // k_rlc_prep and the MSM's digit / two-level sort and scans
  PS_CHUNKS,   // k_msm_chunks: bucket accumulation
  PS_MSMTAIL,  // k_msm_bucket_sum .. k_msm_final
  PS_COLS,     // k_rlc_columns / k_rlc_fixed: fixed-base column sums (s4)
  PS_FIN,      // k_rlc_qsum, k_rlc_finalize*
  PS_HEAD,     // k_rp_gather / decode / hash_small / chal_fr / powers: the next pass's
               // head, short kernels beside the previous pass's fixed-base launch
  PS_N
};
#define FTS_WAVE_PRIO_DEFAULT {0, 2, 2, 1, 1, 3, 3, 1, 3, 1, 3, 3}

}  // namespace fts
