// Token opening checks: the auditor's and the wallet's
// re-commitment of a token from its opening,
//
//   tokenComm = HashToZr(type) * ped0 + value * ped1 + bf * ped2
//   accept iff tokenComm == token.Data
//
// (crypto/audit/auditor.go:226-238 InspectOutput, crypto/token/token.go:69-83
// Token.ToClear, both through commit() token.go:208-217 / auditor.go:412-418).
//
// One lane per token: three fixed-base products over the context's 16-bit
// window tables of ped0/ped1/ped2 (tb_ped0 / tb_G / tb_H), accumulated into
// ONE Jacobian accumulator (no intermediate point additions), then compared
// with the affine commitment in projective form (X == x Z^2, Y == y Z^3): no
// inversion, no normalisation.  48 mixed additions per token at most.
//
// Record layout (host-staged, SoA): raw[n][64] = token.Data as X||Y
// big-endian (NewG1FromBytes input), sc[n][24] = canonical Fr limbs of
// (HashToZr(type), value mod r, bf mod r) -- G1.Mul(s) multiplies by s mod r.
#include "device/g1.hpp"
#include "device/fixed_base.hpp"
#include "device/helpers.hpp"
#include "device/rp_kernels.hpp"
#include "../../include/fts_gpu.h"

namespace fts {

__global__ void __launch_bounds__(64) k_open_check(int n, const uint8_t* __restrict__ raw,
                                                   const uint32_t* __restrict__ sc, const uint32_t* __restrict__ t_ped0,
                                                   const uint32_t* __restrict__ t_ped1,
                                                   const uint32_t* __restrict__ t_ped2, int32_t* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != FTS_OK) return;
  G1A com;
  if (!decode_point(raw + (size_t)i * 64, com)) {  // NewG1FromBytes of token.Data
    status[i] = FTS_E_MALFORMED;
    return;
  }
  const uint32_t* S = sc + (size_t)i * 24;
  Scalar k0, k1, k2;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    k0.v[j] = S[j];
    k1.v[j] = S[8 + j];
    k2.v[j] = S[16 + j];
  }
  G1J acc = g1j_identity();  // c.NewG1() then com.Add(g_i.Mul(v_i)) for i = 0..2
  fb_mul_acc(acc, t_ped0, k0);
  fb_mul_acc(acc, t_ped1, k1);
  fb_mul_acc(acc, t_ped2, k2);
  bool eq;
  if (g1a_is_identity(com)) {
    eq = g1j_is_identity(acc);
  } else if (g1j_is_identity(acc)) {
    eq = false;
  } else {
    const Fp z2 = fp_sqr(acc.z);
    eq = f_eq(acc.x, fp_mul(com.x, z2)) && f_eq(acc.y, fp_mul(com.y, fp_mul(z2, acc.z)));
  }
  status[i] = eq ? FTS_OK : FTS_E_OPEN_MISMATCH;
}

void launch_open_check(int n, const uint8_t* raw, const uint32_t* sc, const uint32_t* tables, int nb,
                       int32_t* status, hipStream_t s) {
  if (n <= 0) return;
  const uint32_t* t0 = tables + (size_t)tb_ped0(nb) * FB_WORDS_PER_BASE;
  const uint32_t* t1 = tables + (size_t)tb_G(nb) * FB_WORDS_PER_BASE;
  const uint32_t* t2 = tables + (size_t)tb_H(nb) * FB_WORDS_PER_BASE;
  hipLaunchKernelGGL(k_open_check, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, raw, sc, t0, t1, t2, status);
}

}  // namespace fts
