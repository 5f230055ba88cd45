// FETCH_SIZE calibration on gfx950 for the access patterns of this library.
//
// rocprofv3's FETCH_SIZE is derived from the L2's fabric read requests; the
// MI355X guide notes it reports half the bytes of wide coalesced streaming
// reads.  The hot kernels here read 64-byte table entries at random rows
// (fixed-base gathers), which is a different pattern, so the correction is
// measured instead of assumed: each kernel below reads a KNOWN number of bytes
// that no cache can hold (tables far larger than the 256 MiB Infinity Cache,
// every row touched at most once per launch), and bench.py's `traffic`
// multiplies FETCH_SIZE by known / FETCH_SIZE of the matching kernel.
//
//   k_calib_stream    16 B per lane, fully coalesced, 1 GiB once
//   k_calib_gather64  one 64-byte row per lane (4 x 16-B loads, the layout of
//                     load_g1a), rows drawn by a hash over an 8 GiB table
//   k_calib_gather64w the same rows, 64 lanes of a wave reading 64 rows of
//                     ONE 32 MiB window (the fixed-base kernels' pattern: a
//                     wave's lanes share a table window)
//
// Run:  rocprofv3 --pmc FETCH_SIZE -T -f csv -d <dir> -o run -- lib/fetch_calib
// Prints the known byte counts as JSON; tools/pmc_r02.py divides.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ull;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dull;
  x ^= x >> 33;
  return x;
}

__global__ void __launch_bounds__(256) k_calib_stream(const uint4* __restrict__ src, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads; (practically) never stores
}

// lane g reads row perm(g) of `rows` rows (bijective on [0, rows) for rows = 2^k)
__global__ void __launch_bounds__(64) k_calib_gather64(const uint4* __restrict__ tab, uint32_t log_rows, size_t lanes,
                                                       uint32_t* __restrict__ sink) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= lanes) return;
  const uint64_t mask = (1ull << log_rows) - 1;
  // odd multiplier + xor-shift on log_rows bits: a permutation of the row space
  uint64_t r = (g * 0x9e3779b97f4a7c15ull) & mask;
  r ^= r >> (log_rows / 2);
  const uint4* p = tab + r * 4;
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  const uint32_t acc = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// wave w reads 64 distinct rows of window w (2^19 rows = 32 MiB per window)
__global__ void __launch_bounds__(64) k_calib_gather64w(const uint4* __restrict__ tab, uint32_t log_rows, size_t lanes,
                                                        uint32_t* __restrict__ sink) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= lanes) return;
  const uint32_t lw = 19;
  const uint64_t nwin = 1ull << (log_rows - lw);
  const uint64_t wave = g / 64, lane = g % 64;
  const uint64_t win = mix64(wave) & (nwin - 1);
  // 64 distinct rows inside the window: stride a large odd number mod 2^19
  const uint64_t row = (win << lw) | (((mix64(wave ^ 0x55) + lane * 0x2f0b1ull) & ((1ull << lw) - 1)));
  const uint4* p = tab + row * 4;
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  const uint32_t acc = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// WRITE_SIZE calibration (round 5): stores of a KNOWN byte count
//   k_calib_store16   16 B per lane, fully coalesced, 1 GiB
//   k_calib_store4    4 B per lane, fully coalesced, 1 GiB
//   k_calib_store4p   4 B per lane, a random permutation inside each block's
//                     8 KiB region (k_rs_part's in-partition scatter), 256 MiB
__global__ void __launch_bounds__(256) k_calib_store16(uint4* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ void __launch_bounds__(256) k_calib_store4(uint32_t* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (uint32_t)i;
}
__global__ void __launch_bounds__(256) k_calib_store4p(uint32_t* __restrict__ dst) {
  uint32_t* r = dst + (size_t)blockIdx.x * 2048;
  for (uint32_t e = threadIdx.x; e < 2048; e += 256) r[(e * 1103u + 977u * blockIdx.x) & 2047u] = e;  // odd stride: a permutation
}

int main() {
  const uint32_t log_rows = 27;  // 2^27 rows x 64 B = 8 GiB
  const size_t rows = (size_t)1 << log_rows, tab_bytes = rows * 64;
  const size_t stream_bytes = (size_t)1 << 30;
  const size_t lanes = (size_t)1 << 22;  // 4 Mi rows = 256 MiB gathered per launch
  uint4* tab = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(tab, 0x3c, tab_bytes));
  CK(hipDeviceSynchronize());
  // every kernel twice; the profile keeps each dispatch
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_calib_stream, dim3(4096), dim3(256), 0, 0, tab, stream_bytes / 16, sink);
    hipLaunchKernelGGL(k_calib_gather64, dim3((unsigned)(lanes / 64)), dim3(64), 0, 0, tab, log_rows, lanes, sink);
    hipLaunchKernelGGL(k_calib_gather64w, dim3((unsigned)(lanes / 64)), dim3(64), 0, 0, tab, log_rows, lanes, sink);
    hipLaunchKernelGGL(k_calib_store16, dim3(4096), dim3(256), 0, 0, tab, stream_bytes / 16);
    hipLaunchKernelGGL(k_calib_store4, dim3(4096), dim3(256), 0, 0, (uint32_t*)tab, stream_bytes / 4);
    hipLaunchKernelGGL(k_calib_store4p, dim3((unsigned)((256u << 20) / 8192)), dim3(256), 0, 0, (uint32_t*)tab);
    CK(hipDeviceSynchronize());
  }
  CK(hipGetLastError());
  printf("{\"k_calib_stream\": %zu, \"k_calib_gather64\": %zu, \"k_calib_gather64w\": %zu, \"k_calib_store16\": %zu, "
         "\"k_calib_store4\": %zu, \"k_calib_store4p\": %zu}\n",
         stream_bytes, lanes * 64, lanes * 64, stream_bytes, stream_bytes, (size_t)256 << 20);
  hipFree(tab);
  hipFree(sink);
  return 0;
}
