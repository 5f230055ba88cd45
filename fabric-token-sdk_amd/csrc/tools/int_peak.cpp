// Integer-ALU roofline microbenchmark for gfx950 ("measure the
// v_mad_u64_u32 rate with a microbenchmark").  Prints one JSON line:
//   mad_u64_u32 per second (chip), full-rate u32 ops per second, and the
//   8x32-limb Montgomery Fp multiplication rate of device/field.hpp.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../device/field.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

constexpr int MAD_ITERS = 4096;
constexpr int MAD_CHAINS = 8;

__global__ void __launch_bounds__(256) k_mad(const uint32_t* in, uint64_t* out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = in[tid & 1023] | 1u, b = in[(tid + 7) & 1023] | 3u;
  uint64_t acc[MAD_CHAINS];
#pragma unroll
  for (int c = 0; c < MAD_CHAINS; c++) acc[c] = tid + c;
  for (int i = 0; i < MAD_ITERS; i++) {
#pragma unroll
    for (int c = 0; c < MAD_CHAINS; c++) {
      // v_mad_u64_u32: acc = a*b + acc  (mix the high word back so it is not folded)
      acc[c] = (uint64_t)(a ^ (uint32_t)(acc[c] >> 32)) * b + (uint32_t)acc[c];
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < MAD_CHAINS; c++) s ^= acc[c];
  out[tid] = s;
}

constexpr int ADD_ITERS = 8192;
__global__ void __launch_bounds__(256) k_add(const uint32_t* in, uint32_t* out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[8];
#pragma unroll
  for (int c = 0; c < 8; c++) x[c] = in[(tid + c) & 1023];
  for (int i = 0; i < ADD_ITERS; i++) {
#pragma unroll
    for (int c = 0; c < 8; c++) x[c] = (x[c] + x[(c + 1) & 7]) ^ 0x9e3779b9u;
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) s ^= x[c];
  out[tid] = s;
}

constexpr int MUL_ITERS = 256;
__global__ void __launch_bounds__(256) k_fpmul(const uint32_t* in, uint32_t* out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fts::Fp a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i] = in[(tid * 8 + i) & 1023];
    b.v[i] = in[(tid * 8 + i + 5) & 1023];
  }
  a.v[7] &= 0x0fffffffu;
  b.v[7] &= 0x0fffffffu;
  for (int i = 0; i < MUL_ITERS; i++) {
    a = fts::f_mul(a, b);
    b = fts::f_mul(b, a);
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ b.v[i];
  out[tid] = s;
}

__global__ void __launch_bounds__(256) k_fpmul_fips(const uint32_t* in, uint32_t* out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fts::Fp a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i] = in[(tid * 8 + i) & 1023];
    b.v[i] = in[(tid * 8 + i + 5) & 1023];
  }
  a.v[7] &= 0x0fffffffu;
  b.v[7] &= 0x0fffffffu;
  for (int i = 0; i < MUL_ITERS; i++) {
    a = fts::f_mul_fips(a, b);
    b = fts::f_mul_fips(b, a);
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ b.v[i];
  out[tid] = s;
}

template <int V>
__device__ __forceinline__ fts::Fp mulv(const fts::Fp& a, const fts::Fp& b) {
  if constexpr (V == 0) return fts::f_mul(a, b);
  else if constexpr (V == 1) return fts::f_mul_fips(a, b);
  else if constexpr (V == 2) return fts::f_mul_g(a, b);
  else if constexpr (V == 3) return fts::f_sqr_fips(a);
  else if constexpr (V == 4) return fts::f_sqr_g(a);
  else return fts::f_mul_x2(a, b);
}
// dependent chain: latency per product when few waves are resident
template <int V>
__global__ void __launch_bounds__(256) k_lat(const uint32_t* in, uint32_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  fts::Fp a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i] = in[(tid * 8 + i) & 1023];
    b.v[i] = in[(tid * 8 + i + 5) & 1023];
  }
  a.v[7] &= 0x0fffffffu;
  b.v[7] &= 0x0fffffffu;
  for (int i = 0; i < iters; i++) a = (V == 3 || V == 4) ? mulv<V>(a, a) : (V == 5 ? fts::f_mul(a, a) : mulv<V>(a, b));
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a.v[i];
  out[tid] = s;
}
template <int V>
double time_lat(const uint32_t* d_in, uint32_t* d_out, int blocks, int threads, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_lat<V><<<blocks, threads>>>(d_in, d_out, 16);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  k_lat<V><<<blocks, threads>>>(d_in, d_out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e-3 / iters;  // seconds per dependent product
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, threads = 256;
  const size_t n = (size_t)blocks * threads;
  uint32_t* d_in;
  uint64_t* d_out;
  CK(hipMalloc(&d_in, 1024 * 4));
  CK(hipMalloc(&d_out, n * 8));
  uint32_t h[1024];
  for (int i = 0; i < 1024; i++) h[i] = 0x12345678u * (i + 1) ^ (i << 13);
  CK(hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;

  k_mad<<<blocks, threads>>>(d_in, d_out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) k_mad<<<blocks, threads>>>(d_in, d_out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double mad_rate = 5.0 * n * MAD_ITERS * MAD_CHAINS / (ms * 1e-3);

  k_add<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) k_add<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double add_rate = 5.0 * n * ADD_ITERS * 8 * 2 / (ms * 1e-3);  // add + xor

  k_fpmul<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) k_fpmul<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double fpmul_rate = 5.0 * n * MUL_ITERS * 2 / (ms * 1e-3);

  uint32_t* h1 = (uint32_t*)malloc(n * 4);
  uint32_t* h2 = (uint32_t*)malloc(n * 4);
  CK(hipMemcpy(h1, d_out, n * 4, hipMemcpyDeviceToHost));
  k_fpmul_fips<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h2, d_out, n * 4, hipMemcpyDeviceToHost));
  int mism = 0;
  for (size_t i = 0; i < n; i++) mism += h1[i] != h2[i];
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) k_fpmul_fips<<<blocks, threads>>>(d_in, (uint32_t*)d_out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double fips_rate = 5.0 * n * MUL_ITERS * 2 / (ms * 1e-3);
  printf("{\"fips_fp_mul_per_s\": %.4e, \"fips_mismatch\": %d}\n", fips_rate, mism);
  // latency regime: 1 wave per SIMD (256 blocks x 256 threads) and 1 wave per 16 SIMDs
  for (int cfg = 0; cfg < 2; cfg++) {
    int blocks = cfg == 0 ? cus : cus / 4, threads = cfg == 0 ? 256 : 64;
    double l0 = time_lat<0>(d_in, (uint32_t*)d_out, blocks, threads, 2000);
    double l1 = time_lat<1>(d_in, (uint32_t*)d_out, blocks, threads, 2000);
    double l2 = time_lat<2>(d_in, (uint32_t*)d_out, blocks, threads, 2000);
    double l3 = time_lat<3>(d_in, (uint32_t*)d_out, blocks, threads, 2000);
    double l4 = time_lat<4>(d_in, (uint32_t*)d_out, blocks, threads, 2000);
    printf("{\"latency_cfg\": \"%dx%d\", \"cios_cycles\": %.0f, \"fips_cycles\": %.0f, \"g_cycles\": %.0f, "
           "\"sqr_cycles\": %.0f, \"sqr_g_cycles\": %.0f}\n",
           blocks, threads, l0 * 2.4e9, l1 * 2.4e9, l2 * 2.4e9, l3 * 2.4e9, l4 * 2.4e9);
  }
  // throughput of fips2 (full occupancy, same shape as k_fpmul)
  {
    hipEvent_t a0, a1;
    hipEventCreate(&a0);
    hipEventCreate(&a1);
    hipEventRecord(a0);
    k_lat<2><<<cus * 8, 256>>>(d_in, (uint32_t*)d_out, 512);
    hipEventRecord(a1);
    hipEventSynchronize(a1);
    float m2;
    hipEventElapsedTime(&m2, a0, a1);
    hipEventRecord(a0);
    k_lat<1><<<cus * 8, 256>>>(d_in, (uint32_t*)d_out, 512);
    hipEventRecord(a1);
    hipEventSynchronize(a1);
    float m1;
    hipEventElapsedTime(&m1, a0, a1);
    float m3, m4;
    hipEventRecord(a0);
    k_lat<3><<<cus * 8, 256>>>(d_in, (uint32_t*)d_out, 512);
    hipEventRecord(a1);
    hipEventSynchronize(a1);
    hipEventElapsedTime(&m3, a0, a1);
    hipEventRecord(a0);
    k_lat<4><<<cus * 8, 256>>>(d_in, (uint32_t*)d_out, 512);
    hipEventRecord(a1);
    hipEventSynchronize(a1);
    hipEventElapsedTime(&m4, a0, a1);
    const double nm = (double)cus * 8 * 256 * 512;
    printf("{\"throughput_fips_per_s\": %.4e, \"throughput_g_per_s\": %.4e, \"throughput_sqr_per_s\": %.4e, "
           "\"throughput_sqr_g_per_s\": %.4e}\n", nm / (m1 * 1e-3), nm / (m2 * 1e-3), nm / (m3 * 1e-3), nm / (m4 * 1e-3));
    // correctness of the new variants against CIOS
    std::vector<uint32_t> r0(cus * 256), r3(cus * 256), r4(cus * 256), r5(cus * 256);
    k_lat<5><<<cus, 256>>>(d_in, (uint32_t*)d_out, 64);
    hipMemcpy(r5.data(), d_out, r5.size() * 4, hipMemcpyDeviceToHost);
    k_lat<0><<<cus, 256>>>(d_in, (uint32_t*)d_out, 64);
    hipMemcpy(r0.data(), d_out, r0.size() * 4, hipMemcpyDeviceToHost);
    k_lat<3><<<cus, 256>>>(d_in, (uint32_t*)d_out, 64);
    hipMemcpy(r3.data(), d_out, r3.size() * 4, hipMemcpyDeviceToHost);
    k_lat<4><<<cus, 256>>>(d_in, (uint32_t*)d_out, 64);
    hipMemcpy(r4.data(), d_out, r4.size() * 4, hipMemcpyDeviceToHost);
    int bad3 = 0, bad4 = 0;
    for (size_t i = 0; i < r0.size(); i++) {
      bad3 += r5[i] != r3[i];
      bad4 += r5[i] != r4[i];
    }
    printf("{\"sqr_mismatch\": %d, \"sqr_g_mismatch\": %d}\n", bad3, bad4);
  }
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"mad_u64_u32_per_s\": %.4e, "
         "\"u32_ops_per_s\": %.4e, \"fp_mul_per_s\": %.4e, \"fp_mul_mad_equiv_per_s\": %.4e}\n",
         prop.gcnArchName, cus, prop.clockRate, mad_rate, add_rate, fpmul_rate, fpmul_rate * 136.0);
  return 0;
}
