// glv_mul (single-lane GLV + joint Straus) against var_base_mul on random
// points and scalars; prints mismatches and timings as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../device/g1.hpp"
#include "../device/glv.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void __launch_bounds__(64) k_check(int n, const uint32_t* sc, uint32_t* tab, uint32_t* scr, uint32_t* out, int mode) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fts::G1A g;
  // generator (1, 2) in Montgomery form
  fts::Fp one = fts::f_one<fts::FpP>();
  g.x = one;
  g.y = fts::f_add(one, one);
  // base point: G * (i + 3) via var_base_mul with a small scalar
  fts::Scalar s0;
  for (int q = 0; q < 8; q++) s0.v[q] = 0;
  s0.v[0] = (uint32_t)(i + 3);
  fts::G1A p = fts::g1j_to_affine(fts::var_base_mul(g, s0, scr + (size_t)i * 10 * 24));
  fts::Scalar k;
  for (int q = 0; q < 8; q++) k.v[q] = sc[(size_t)i * 8 + q];
  fts::G1J r = mode == 0 ? fts::glv_mul(p, k, tab, (size_t)n, (size_t)i) : fts::var_base_mul(p, k, scr + (size_t)i * 10 * 24);
  fts::G1A a = fts::g1j_to_affine(r);
  for (int q = 0; q < 8; q++) {
    out[(size_t)i * 16 + q] = a.x.v[q];
    out[(size_t)i * 16 + 8 + q] = a.y.v[q];
  }
}

int main() {
  const int n = 4096;
  std::vector<uint32_t> h((size_t)n * 8);
  uint64_t s = 88172645463325252ull;
  for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)s; }
  for (int i = 0; i < n; i++) h[(size_t)i * 8 + 7] &= 0x2fffffffu;  // < r
  uint32_t *dsc, *dtab, *dscr, *d0, *d1;
  CK(hipMalloc(&dsc, h.size() * 4));
  CK(hipMalloc(&dtab, (size_t)n * 16 * 24 * 4));
  CK(hipMalloc(&dscr, (size_t)n * 10 * 24 * 4));
  CK(hipMalloc(&d0, (size_t)n * 64));
  CK(hipMalloc(&d1, (size_t)n * 64));
  CK(hipMemcpy(dsc, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms[2];
  for (int m = 0; m < 2; m++) {
    hipEventRecord(a);
    k_check<<<n / 64, 64>>>(n, dsc, dtab, dscr, m == 0 ? d0 : d1, m);
    hipEventRecord(b);
    CK(hipEventSynchronize(b));
    hipEventElapsedTime(&ms[m], a, b);
    fprintf(stderr, "mode %d done\n", m);
  }
  std::vector<uint32_t> r0((size_t)n * 16), r1((size_t)n * 16);
  CK(hipMemcpy(r0.data(), d0, r0.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), d1, r1.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < n; i++)
    for (int q = 0; q < 16; q++)
      if (r0[(size_t)i * 16 + q] != r1[(size_t)i * 16 + q]) { bad++; break; }
  printf("{\"n\": %d, \"mismatch\": %d, \"glv_ms\": %.3f, \"varbase_ms\": %.3f}\n", n, bad, ms[0], ms[1]);
  return 0;
}
