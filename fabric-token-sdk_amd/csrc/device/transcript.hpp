// Fiat-Shamir transcripts on the device.
//
// The reference hashes text: (*G1Array).Bytes (crypto/common/array.go:25-36)
// is the lowercase hex of every 64-byte point joined with "||", and the first
// IPA challenge wraps that string in DER (rp/ipa.go:200-213).  Every record
// is 130 bytes (128 hex + "||"), so all transcripts are sequences of 16-bit
// units; builders write them to a per-message HBM slot (with SHA-256 padding
// appended) and a separate kernel compresses the slots, one lane per message.
#pragma once
#include "../common/sha256.hpp"
#include "field.hpp"

namespace fts {

// two lowercase hex chars of byte b, in memory order (first char in low byte)
FTS_DEV uint16_t hex2(uint32_t b) {
  uint32_t hi = (b >> 4) & 15u, lo = b & 15u;
  uint32_t ch = hi + (hi < 10u ? 48u : 87u);
  uint32_t cl = lo + (lo < 10u ? 48u : 87u);
  return (uint16_t)(ch | (cl << 8));
}

// write hex(p) (128 bytes) at dst (2-byte aligned); p = 64 canonical BE bytes
// given as 16 big-endian-packed words (word i = bytes 4i..4i+3).
FTS_DEV void write_hex_point_words(uint16_t* dst, const uint32_t pw[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t w = pw[i];
    dst[4 * i + 0] = hex2(w >> 24);
    dst[4 * i + 1] = hex2(w >> 16);
    dst[4 * i + 2] = hex2(w >> 8);
    dst[4 * i + 3] = hex2(w);
  }
}

// load 64 raw bytes (4-byte aligned) as 16 words in big-endian order
FTS_DEV void load_be_words(const uint8_t* src, uint32_t pw[16]) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint4 u = s[i];
    pw[4 * i + 0] = __builtin_bswap32(u.x);
    pw[4 * i + 1] = __builtin_bswap32(u.y);
    pw[4 * i + 2] = __builtin_bswap32(u.z);
    pw[4 * i + 3] = __builtin_bswap32(u.w);
  }
}

// affine Montgomery point -> 16 BE words of its canonical encoding
// (identity (0,0) -> zeros, matching gnark RawBytes of the identity)
FTS_DEV void g1_mont_to_be_words(const Fp& x, const Fp& y, uint32_t pw[16]) {
  Fp cx = f_from_mont(x), cy = f_from_mont(y);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pw[i] = cx.v[7 - i];
    pw[8 + i] = cy.v[7 - i];
  }
}

// number of 64-byte SHA-256 blocks for a message of len bytes
FTS_HD uint32_t sha_blocks(uint32_t len) { return (len + 9 + 63) / 64; }

// write SHA-256 padding for a message of len bytes at msg (zero-filled tail)
FTS_DEV void write_sha_padding_u16(uint8_t* msg, uint32_t len) {
  // len is even: pad with 16-bit stores
  uint32_t nb = sha_blocks(len);
  uint32_t end = nb * 64;
  uint16_t* m16 = reinterpret_cast<uint16_t*>(msg);
  m16[len >> 1] = 0x0080;  // 0x80 then 0x00
  for (uint32_t o = len + 2; o < end - 8; o += 2) m16[o >> 1] = 0;
  uint64_t bits = (uint64_t)len * 8;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t b0 = (uint32_t)(bits >> (56 - 16 * i)) & 0xffu;
    uint32_t b1 = (uint32_t)(bits >> (48 - 16 * i)) & 0xffu;
    m16[((end - 8) >> 1) + i] = (uint16_t)(b0 | (b1 << 8));
  }
}

// hash nblocks of a padded message; digest as 8 BE words
FTS_DEV void sha256_blocks(const uint8_t* msg, uint32_t nblocks, uint32_t st[8]) {
  sha256_init(st);
  const uint4* m = reinterpret_cast<const uint4*>(msg);
  for (uint32_t b = 0; b < nblocks; b++) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      uint4 u = m[b * 4 + i];
      w[4 * i + 0] = __builtin_bswap32(u.x);
      w[4 * i + 1] = __builtin_bswap32(u.y);
      w[4 * i + 2] = __builtin_bswap32(u.z);
      w[4 * i + 3] = __builtin_bswap32(u.w);
    }
    sha256_compress(st, w);
  }
}

// HashToZr: digest (big-endian) mod r -> canonical Fr limbs (LE)
FTS_DEV Fr digest_to_fr(const uint32_t st[8]) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = st[7 - i];
  // digest < 2^256 < 6r: at most 5 subtractions
#pragma unroll
  for (int t = 0; t < 5; t++) {
    uint32_t s[8], bw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = subb(r.v[i], FrP::M[i], bw, bw);
    const bool keep = bw != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = keep ? r.v[i] : s[i];
  }
  return r;
}

}  // namespace fts
