// Do two small latency-bound kernels on different streams share SIMDs?
// Kernel: `waves` wavefronts each running a dependent chain of v_mad_u64_u32.
// Prints the time of one launch alone and of two launches on two streams,
// for 64-thread blocks (1 wave) and 256-thread blocks (4 waves).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// 8 independent chains per lane: one wave alone keeps its SIMD's issue slot busy
// (issue-bound, like the field arithmetic and SHA-256 kernels), so two waves on
// one SIMD would each run at half speed
__global__ void k_chain(uint64_t* out, int iters) {
  uint64_t a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) a[j] = threadIdx.x + blockIdx.x * 7 + j + 1;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = (uint64_t)(uint32_t)a[j] * (uint32_t)(a[j] >> 17) + (a[j] >> 32);
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= a[j];
  if (r == 0x1234567ull) out[0] = r;
}

int main() {
  uint64_t* out;
  hipMalloc(&out, 8);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 40000;
  for (int bs : {64, 256}) {
    for (int waves : {64, 128, 512}) {
      const int blocks = waves * 64 / bs;
      float alone = 0, both = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipDeviceSynchronize();
        hipEventRecord(e0, s1);
        hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(bs), 0, s1, out, iters);
        hipEventRecord(e1, s1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&alone, e0, e1);
        hipDeviceSynchronize();
        hipEventRecord(e0, 0);
        hipStreamWaitEvent(s1, e0, 0);
        hipStreamWaitEvent(s2, e0, 0);
        hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(bs), 0, s1, out, iters);
        hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(bs), 0, s2, out, iters);
        hipDeviceSynchronize();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&both, e0, e1);
      }
      printf("block %3d  waves %4d  alone %.3f ms  two streams %.3f ms  ratio %.2f\n", bs, waves, alone, both,
             both / alone);
    }
  }
  return 0;
}
