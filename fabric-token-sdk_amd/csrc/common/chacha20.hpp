// ChaCha20 block function (RFC 8439 §2.3), host + device.
//
// Source of the random-linear-combination weights rho_p of the batch check:
// the host draws a fresh 256-bit key per verification call from getrandom(),
// and proof p takes block (key, counter = p) on the device, so the weights
// are unpredictable to whoever produced the proofs (batch soundness error
// ~2^-253 per call with full-width weights).
#pragma once
#include <stdint.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define FTS_HD2 __host__ __device__ __forceinline__
#else
#define FTS_HD2 inline
#endif

namespace fts {

FTS_HD2 uint32_t cc_rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define FTS_QR(a, b, c, d) \
  a += b;                  \
  d ^= a;                  \
  d = cc_rotl(d, 16);      \
  c += d;                  \
  b ^= c;                  \
  b = cc_rotl(b, 12);      \
  a += b;                  \
  d ^= a;                  \
  d = cc_rotl(d, 8);       \
  c += d;                  \
  b ^= c;                  \
  b = cc_rotl(b, 7);

// out = ChaCha20(key, counter, nonce = 0) keystream block (16 words)
FTS_HD2 void chacha20_block(const uint32_t key[8], uint32_t counter, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4],      key[5],      key[6],      key[7],      counter, 0u,     0u,     0u};
  uint32_t x[16];
  for (int i = 0; i < 16; i++) x[i] = s[i];
  for (int r = 0; r < 10; r++) {
    FTS_QR(x[0], x[4], x[8], x[12]);
    FTS_QR(x[1], x[5], x[9], x[13]);
    FTS_QR(x[2], x[6], x[10], x[14]);
    FTS_QR(x[3], x[7], x[11], x[15]);
    FTS_QR(x[0], x[5], x[10], x[15]);
    FTS_QR(x[1], x[6], x[11], x[12]);
    FTS_QR(x[2], x[7], x[8], x[13]);
    FTS_QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
#undef FTS_QR

}  // namespace fts
