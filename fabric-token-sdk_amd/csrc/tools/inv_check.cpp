// Field-inversion check + timing on gfx950: f_inv_gcd (constant-time
// optimised binary GCD) against f_inv_bin (variable-time binary extended
// Euclid) and Fermat, on random and edge-case inputs, for Fp and Fr.
// Prints one JSON line per field.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../device/field.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <class P, int V>
__global__ void __launch_bounds__(64) k_inv(const uint32_t* in, uint32_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fts::Field<P> a;
#pragma unroll
  for (int q = 0; q < 8; q++) a.v[q] = in[(size_t)i * 8 + q];
  fts::Field<P> r = V == 0 ? fts::f_inv_gcd(a) : (V == 1 ? fts::f_inv_bin(a) : fts::f_inv(a));
  // check a * r == 1 (Montgomery one) unless a == 0
  fts::Field<P> o = fts::f_mul(a, r);
  bool ok = fts::f_is_zero(a) ? fts::f_is_zero(r) : true;
  if (!fts::f_is_zero(a))
    for (int q = 0; q < 8; q++) ok = ok && o.v[q] == P::ONE[q];
#pragma unroll
  for (int q = 0; q < 8; q++) out[(size_t)i * 9 + q] = r.v[q];
  out[(size_t)i * 9 + 8] = ok ? 1u : 0u;
}

static uint32_t hsub(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
  uint64_t d = (uint64_t)a - b - bin;
  bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}
static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

template <class P>
void run(const char* name) {
  const int n = 1 << 20;
  std::vector<uint32_t> h((size_t)n * 8);
  for (int i = 0; i < n; i++) {
    for (int q = 0; q < 8; q++) h[(size_t)i * 8 + q] = next32();
    h[(size_t)i * 8 + 7] &= 0x1fffffffu;  // < M (top limb of M is 0x30644e72)
  }
  // edge cases: 0, 1, 2, M-1, M-2, 2^k, small values, one-limb values
  auto put = [&](int i, const uint32_t v[8]) { for (int q = 0; q < 8; q++) h[(size_t)i * 8 + q] = v[q]; };
  int e = 0;
  uint32_t z[8] = {0};
  put(e++, z);
  for (uint32_t s = 1; s < 40; s++) { uint32_t v[8] = {s}; put(e++, v); }
  { uint32_t v[8]; uint32_t bw = 0; for (int q = 0; q < 8; q++) v[q] = hsub(P::M[q], q == 0 ? 1u : 0u, bw, bw); put(e++, v); }
  { uint32_t v[8]; uint32_t bw = 0; for (int q = 0; q < 8; q++) v[q] = hsub(P::M[q], q == 0 ? 2u : 0u, bw, bw); put(e++, v); }
  for (int k = 0; k < 254; k++) { uint32_t v[8] = {0}; v[k / 32] = 1u << (k % 32); put(e++, v); }
  for (int k = 0; k < 254; k++) { uint32_t v[8]; for (int q = 0; q < 8; q++) v[q] = 0xffffffffu; for (int b = k; b < 256; b++) v[b / 32] &= ~(1u << (b % 32)); put(e++, v); }
  uint32_t *din, *d0, *d1;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMalloc(&d0, (size_t)n * 36));
  CK(hipMalloc(&d1, (size_t)n * 36));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms[3] = {0, 0, 0};
  // timing: n lanes (throughput) and 16384 lanes (latency-ish, 1 wave per 4 SIMDs)
  for (int v = 0; v < 2; v++) {
    uint32_t* d = v == 0 ? d0 : d1;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      if (v == 0) k_inv<P, 0><<<n / 64, 64>>>(din, d, n);
      else k_inv<P, 1><<<n / 64, 64>>>(din, d, n);
      hipEventRecord(b);
      CK(hipEventSynchronize(b));
      hipEventElapsedTime(&ms[v], a, b);
    }
  }
  float lat[2];
  for (int v = 0; v < 2; v++) {
    uint32_t* d = v == 0 ? d0 : d1;
    hipEventRecord(a);
    if (v == 0) k_inv<P, 0><<<256, 64>>>(din, d, 16384);
    else k_inv<P, 1><<<256, 64>>>(din, d, 16384);
    hipEventRecord(b);
    CK(hipEventSynchronize(b));
    hipEventElapsedTime(&lat[v], a, b);
  }
  std::vector<uint32_t> r0((size_t)n * 9), r1((size_t)n * 9);
  CK(hipMemcpy(r0.data(), d0, r0.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), d1, r1.size() * 4, hipMemcpyDeviceToHost));
  long bad_gcd = 0, bad_bin = 0, mism = 0;
  for (int i = 0; i < n; i++) {
    bad_gcd += r0[(size_t)i * 9 + 8] != 1;
    bad_bin += r1[(size_t)i * 9 + 8] != 1;
    for (int q = 0; q < 8; q++)
      if (r0[(size_t)i * 9 + q] != r1[(size_t)i * 9 + q]) { mism++; break; }
  }
  printf("{\"field\": \"%s\", \"n\": %d, \"edge_cases\": %d, \"bad_gcd\": %ld, \"bad_bin\": %ld, \"mismatch\": %ld, "
         "\"gcd_ms_1M\": %.3f, \"bin_ms_1M\": %.3f, \"gcd_ms_16k_lanes\": %.3f, \"bin_ms_16k_lanes\": %.3f}\n",
         name, n, e, bad_gcd, bad_bin, mism, ms[0], ms[1], lat[0], lat[1]);
  hipFree(din);
  hipFree(d0);
  hipFree(d1);
}

int main() {
  run<fts::FpP>("Fp");
  run<fts::FrP>("Fr");
  return 0;
}
