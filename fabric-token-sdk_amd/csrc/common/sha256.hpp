// SHA-256 (FIPS 180-4), shared by the host (prover, PP) and the device
// (Fiat-Shamir transcripts).  The reference hashes every transcript with
// mathlib Curve.HashToZr = SHA-256 (crypto/sha256) read big-endian mod r.
//
// Device use: one lane owns one transcript; the 16-word block is built in
// registers by the caller and fed to sha256_compress (fully unrolled, static
// register indexing, no scratch).
#pragma once
#include <stdint.h>
#include <string.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define FTS_HD __host__ __device__ __forceinline__
#else
#define FTS_HD inline
#endif

namespace fts {

struct Sha256Const {
  static constexpr uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
};

FTS_HD uint32_t sha_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// a ^ b ^ c: one v_bitop3_b32 (truth table 0x96) on gfx950 instead of two v_xor_b32
// (the compiler fuses Ch / Maj into bitop3 itself, not the 3-way xors of the
// Sigma / sigma functions); Ch / Maj get their truth tables explicitly
// (0xCA = e ? f : g, 0xE8 = majority); the host side (prover, PP) keeps plain C++
FTS_HD uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
FTS_HD uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
#else
  return (e & f) ^ (~e & g);
#endif
}
FTS_HD uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}

FTS_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// w: 16 big-endian message words (consumed)
FTS_HD void sha256_compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = sha_xor3(sha_rotr(w15, 7), sha_rotr(w15, 18), w15 >> 3);
      uint32_t s1 = sha_xor3(sha_rotr(w2, 17), sha_rotr(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = sha_xor3(sha_rotr(e, 6), sha_rotr(e, 11), sha_rotr(e, 25));
    uint32_t ch = sha_ch(e, f, g);
    uint32_t t1 = h + S1 + ch + Sha256Const::K[i] + wi;
    uint32_t S0 = sha_xor3(sha_rotr(a, 2), sha_rotr(a, 13), sha_rotr(a, 22));
    uint32_t mj = sha_maj(a, b, c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Byte-streaming context (host side and small device transcripts).
struct Sha256 {
  uint32_t st[8];
  uint8_t buf[64];
  uint32_t fill;
  uint64_t total;

  FTS_HD void init() {
    sha256_init(st);
    fill = 0;
    total = 0;
  }
  FTS_HD void block_from_buf() {
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[4 * i] << 24) | ((uint32_t)buf[4 * i + 1] << 16) | ((uint32_t)buf[4 * i + 2] << 8) |
             (uint32_t)buf[4 * i + 3];
    sha256_compress(st, w);
  }
  FTS_HD void byte(uint8_t c) {
    buf[fill++] = c;
    total++;
    if (fill == 64) {
      block_from_buf();
      fill = 0;
    }
  }
  FTS_HD void update(const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; i++) byte(p[i]);
  }
  FTS_HD void final(uint8_t out[32]) {
    uint64_t bits = total * 8;
    byte(0x80);
    while (fill != 56) byte(0);
    for (int i = 7; i >= 0; i--) byte((uint8_t)(bits >> (8 * i)));
    for (int i = 0; i < 8; i++) {
      out[4 * i] = (uint8_t)(st[i] >> 24);
      out[4 * i + 1] = (uint8_t)(st[i] >> 16);
      out[4 * i + 2] = (uint8_t)(st[i] >> 8);
      out[4 * i + 3] = (uint8_t)st[i];
    }
  }
};

FTS_HD void sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
  Sha256 s;
  s.init();
  s.update(p, n);
  s.final(out);
}

}  // namespace fts
