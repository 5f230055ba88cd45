// Reproducer of the gfx950 long-branch miscompile (tools/long_branch_check.py):
// an out-of-line (__noinline__) glv_mul. Its body exceeds the s_cbranch range, and
// branch relaxation clobbers the return-address pair s[30:31] -> the function
// never returns.  Compile only (do NOT run it):
//   python tools/long_branch_check.py tools/experiments/glv_noinline_repro.hip
#include <hip/hip_runtime.h>
#include "../../fabric-token-sdk_amd/csrc/device/g1.hpp"
#include "../../fabric-token-sdk_amd/csrc/device/glv.hpp"
namespace fts {
__device__ __noinline__ G1J nl_glv_mul(G1A p, Scalar k, uint32_t* __restrict__ tab, size_t stride, size_t idx) {
  return glv_mul(p, k, tab, stride, idx);
}
}
__global__ void __launch_bounds__(64) k_nl(int n, const uint32_t* sc, uint32_t* tab, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fts::G1A p;
  fts::Fp one = fts::f_one<fts::FpP>();
  p.x = one; p.y = fts::f_add(one, one);
  fts::Scalar k;
  for (int q = 0; q < 8; q++) k.v[q] = sc[(size_t)i * 8 + q];
  fts::G1J r = fts::nl_glv_mul(p, k, tab, (size_t)n, (size_t)i);
  for (int q = 0; q < 8; q++) { out[i * 24 + q] = r.x.v[q]; out[i*24+8+q] = r.y.v[q]; out[i*24+16+q] = r.z.v[q]; }
}
