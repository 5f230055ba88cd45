// Batched idemix pseudonym-signature verification over BN254 and FP256BN (SURVEY.md
// §8(f) row 4, the idemix half): the owner signatures of transfers whose
// input tokens are owned by idemix identities.
//
// Reference call chain:
//   validator/validator_transfer.go:29-62  TransferSignatureValidate, per input
//   services/identity/idemix/deserializer.go:82-105  owner verifier =
//       crypto.NymSignatureVerifier{IPK, NymPK}
//   services/identity/idemix/crypto/id.go:145-161  NymSignatureVerifier.Verify
//       -> bccsp Verify(NymPK, sigma, msg, IdemixNymSignerOpts{IssuerPK})
//   github.com/IBM/idemix (go.mod:6, not vendored) NymSignature.Ver:
//       t  = HSk^s_sk * HRand^s_rnym * Nym^-c
//       c' = HashToZr("sign" || t || Nym || ipk.Hash || msg)
//       ok = (c == HashToZr(c' || Nonce))
// (restated and pinned as far as the reference's fixtures allow in
// oracle/idemix.py).  The issuer key is the BN254 one that zkatdlog public
// parameters carry (IdemixIssuerPublicKeys, curve BN254 in zkatdlog_pp.json).
//
// Kernels (one signature per lane):
//   (build once per issuer key)  16-bit fixed-base tables of HSk and HRand
//       (rp_kernels.hip launch_build_tables, 32 MiB each)
//   k_nym_verify  nym decode + on-curve check, t = s_sk HSk + s_rnym HRand
//       (2 x 16 mixed additions) + (r - c) Nym (GLV, glv.hpp), affine t,
//       SHA-256 over the 164-byte prefix and the message (streamed from HBM
//       as aligned words), HashToZr, the second 64-byte hash, c == c''.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fts_gpu.h"
#include "common/sha256.hpp"
#include "device/fixed_base.hpp"
#include "device/glv.hpp"
#include "device/helpers.hpp"
#include "device/transcript.hpp"
#include "device/fp256bn.hpp"
#include "host/bn254_host.hpp"
#include "host/pb.hpp"

namespace fts {
void launch_build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s);
size_t table_build_scratch_bytes(int nb);
size_t fb_words_per_base();
}  // namespace fts

using namespace fts;

namespace fts {
void host_parallel_for(size_t n, const std::function<void(size_t)>& f);  // fts_api.cpp (persistent host pool)
}

namespace {

// per-item record (words): c[8] s_sk[8] s_rnym[8] (plain LE limbs, c < r,
// s mod r), nonce[8] (big-endian words, as hashed)
constexpr int NREC = 32;
constexpr uint32_t PREFIX_WORDS = 41;  // "sign"(1) + t(16) + Nym(16) + ipk.Hash(8)

// message word j of the hashed stream (big-endian), with the SHA-256 0x80
// terminator and zero fill; m: the message's words (4-byte aligned, padded
// to a whole word in the staging buffer)
FTS_DEV uint32_t msg_word(const uint32_t* __restrict__ m, uint32_t len, uint32_t j) {
  const uint32_t b = 4 * j;
  if (b > len) return 0u;
  if (b == len) return 0x80000000u;
  const uint32_t raw = __builtin_bswap32(m[j]);
  if (b + 4 <= len) return raw;
  const uint32_t keep = len - b;  // 1..3 bytes
  const uint32_t mask = 0xffffffffu << (32 - 8 * keep);
  return (raw & mask) | (0x80000000u >> (8 * keep));
}

// word g >= PREFIX_WORDS of the padded stream of nb blocks (length in the last two)
FTS_DEV uint32_t stream_word(const uint32_t* __restrict__ m, uint32_t len, uint32_t nb, uint32_t g) {
  const uint64_t bits = (uint64_t)(164u + len) * 8u;
  if (g == 16 * nb - 2) return (uint32_t)(bits >> 32);
  if (g == 16 * nb - 1) return (uint32_t)bits;
  return msg_word(m, len, g - PREFIX_WORDS);
}

// canonical plain limbs (LE) -> Scalar
FTS_DEV Scalar load_scalar(const uint32_t* p) {
  Scalar s;
#pragma unroll
  for (int k = 0; k < 8; k++) s.v[k] = p[k];
  return s;
}

__global__ __launch_bounds__(256) void k_nym_verify(int n, const uint32_t* __restrict__ rec,
                                                    const uint8_t* __restrict__ nym_raw,
                                                    const uint32_t* __restrict__ msgw,
                                                    const uint64_t* __restrict__ moff,  // word offsets
                                                    const uint32_t* __restrict__ mlen,
                                                    const uint32_t* __restrict__ tables,
                                                    const uint32_t* __restrict__ ipk_hash,  // 8 BE words
                                                    uint32_t* __restrict__ vtab, int32_t* __restrict__ status,
                                                    int base, int tile) {
  // one launch per tile of `tile` items starting at `base`; the GLV lane table is
  // [entry][word][tile] (bounded device memory whatever n is)
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = base + li;
  if (li >= tile || i >= n || status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * NREC;
  // Nym: NewG1FromBytes (64-byte raw, canonical coordinates, on the curve)
  G1A nym;
  if (!decode_point(nym_raw + (size_t)i * 64, nym)) {
    status[i] = FTS_E_NYM_BADKEY;
    return;
  }
  // t = s_sk HSk + s_rnym HRand + (r - c) Nym
  G1J acc = g1j_identity();
  fb_mul_acc(acc, tables, load_scalar(R + 8));
  fb_mul_acc(acc, tables + FB_WORDS_PER_BASE, load_scalar(R + 16));
  Scalar nc;  // r - c (c < r; c == 0 -> 0)
  {
    uint32_t bw = 0, nz = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) nz |= R[k];
#pragma unroll
    for (int k = 0; k < 8; k++) nc.v[k] = nz ? subb(FrP::M[k], R[k], bw, bw) : 0u;
  }
  const G1J cn = glv_mul(nym, nc, vtab, (size_t)tile, (size_t)li);
  add_inl(acc, cn);
  const G1A t = g1j_to_affine(acc);  // identity -> (0, 0) -> 64 zero bytes (gnark RawBytes)
  uint32_t tw[16], nw[16], hw[8];
  g1_mont_to_be_words(t.x, t.y, tw);
  load_be_words(nym_raw + (size_t)i * 64, nw);
#pragma unroll
  for (int k = 0; k < 8; k++) hw[k] = ipk_hash[k];
  const uint32_t* m = msgw + moff[i];
  const uint32_t len = mlen[i];
  const uint32_t nb = sha_blocks(164u + len);  // >= 3
  uint32_t st[8], w[16];
  sha256_init(st);
  // block 0: "sign" t[0..14]
  w[0] = 0x7369676eu;
#pragma unroll
  for (int k = 1; k < 16; k++) w[k] = tw[k - 1];
  sha256_compress(st, w);
  // block 1: t[15] Nym[0..14]
  w[0] = tw[15];
#pragma unroll
  for (int k = 1; k < 16; k++) w[k] = nw[k - 1];
  sha256_compress(st, w);
  // block 2: Nym[15] ipk.Hash[0..7] then the message
  w[0] = nw[15];
#pragma unroll
  for (int k = 1; k < 9; k++) w[k] = hw[k - 1];
#pragma unroll
  for (int k = 9; k < 16; k++) w[k] = stream_word(m, len, nb, 32 + k);
  sha256_compress(st, w);
  for (uint32_t blk = 3; blk < nb; blk++) {
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = stream_word(m, len, nb, 16 * blk + k);
    sha256_compress(st, w);
  }
  // c' = HashToZr(...) ; c'' = HashToZr(c' || Nonce)
  const Fr c1 = digest_to_fr(st);
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = c1.v[7 - k];
#pragma unroll
  for (int k = 0; k < 8; k++) w[8 + k] = R[24 + k];
  sha256_init(st);
  sha256_compress(st, w);
  w[0] = 0x80000000u;
#pragma unroll
  for (int k = 1; k < 15; k++) w[k] = 0u;
  w[15] = 512u;
  sha256_compress(st, w);
  const Fr c2 = digest_to_fr(st);
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) diff |= c2.v[k] ^ R[k];
  status[i] = diff ? FTS_E_NYM_INVALID : FTS_OK;
}

// ------------------------------------------------------------ FP256BN keys
// 16-bit unsigned fixed-base windows: entry (w, d) = d * 2^(16 w) * B, affine
// Montgomery (16 words), d = 0 unused; 64 MiB per base (as the ECDSA table)
constexpr int FBN_W = 16, FBN_NW = 16, FBN_ND = 1 << FBN_W;

// lane per (base, window, digit); bases: affine Montgomery (16 words each)
__global__ __launch_bounds__(256) void k_fbn_table(int nb, const uint32_t* __restrict__ bases,
                                                   uint32_t* __restrict__ table) {
  const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (size_t)nb * FBN_NW * FBN_ND) return;
  const int b = (int)(id / (FBN_NW * FBN_ND)), w = (int)((id / FBN_ND) % FBN_NW), d = (int)(id % FBN_ND);
  uint32_t* out = table + id * 16;
  if (d == 0) {
    for (int i = 0; i < 16; i++) out[i] = 0;
    return;
  }
  const fbn::Fp bx = fbn::load<fbn::PM>(bases + b * 16), by = fbn::load<fbn::PM>(bases + b * 16 + 8);
  fbn::PJ p = fbn::pj_inf();
  for (int k = FBN_W - 1; k >= 0; k--) {
    p = fbn::pj_dbl(p);
    if ((d >> k) & 1) p = fbn::pj_madd(p, bx, by);
  }
  for (int k = 0; k < FBN_W * w; k++) p = fbn::pj_dbl(p);
  const fbn::Fp zi = p256::inv(p.z), zi2 = fbn::sqr(zi);
  const fbn::Fp x = fbn::mul(p.x, zi2), y = fbn::mul(p.y, fbn::mul(zi2, zi));
  for (int i = 0; i < 8; i++) out[i] = x.v[i], out[8 + i] = y.v[i];
}

// big-endian word j of the materialised stream region (length ltot bytes), with
// the SHA-256 terminator / zero fill and the bit length in the last two words
FTS_DEV uint32_t region_word(const uint32_t* __restrict__ m, uint32_t ltot, uint32_t nb, uint32_t g) {
  const uint64_t bits = (uint64_t)ltot * 8u;
  if (g == 16 * nb - 2) return (uint32_t)(bits >> 32);
  if (g == 16 * nb - 1) return (uint32_t)bits;
  return msg_word(m, ltot, g);
}

// digest (state words) as a big-endian integer mod r_fbn, plain LE limbs
// (2^256 < 2 r: at most one subtraction)
FTS_DEV void digest_mod_rfbn(const uint32_t st[8], uint32_t out[8]) {
  uint32_t t[8], bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = st[7 - i];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = subb(out[i], fbn::RM::M[i], bw, bw);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = bw ? out[i] : t[i];
}

// FP256BN GLV chain helpers: the lane's 16-entry Jacobian table in global
// memory, [entry][word][stride] (as glv.hpp's vtab for BN254), and the signed
// 4-bit recoding of a 128-bit magnitude over 33 windows (window 32 = the carry)
__device__ inline void fbn_vtab_store(uint32_t* __restrict__ tab, size_t stride, size_t idx, int e, const fbn::PJ& p) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    tab[((size_t)(e * 24) + k) * stride + idx] = p.x.v[k];
    tab[((size_t)(e * 24) + 8 + k) * stride + idx] = p.y.v[k];
    tab[((size_t)(e * 24) + 16 + k) * stride + idx] = p.z.v[k];
  }
}
__device__ inline fbn::PJ fbn_vtab_load(const uint32_t* __restrict__ tab, size_t stride, size_t idx, int e) {
  fbn::PJ p;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    p.x.v[k] = tab[((size_t)(e * 24) + k) * stride + idx];
    p.y.v[k] = tab[((size_t)(e * 24) + 8 + k) * stride + idx];
    p.z.v[k] = tab[((size_t)(e * 24) + 16 + k) * stride + idx];
  }
  return p;
}
__device__ inline uint64_t fbn_recode(const uint32_t s[4]) {  // bit w = carry into window w
  uint64_t cm = 0;
  uint32_t c = 0;
#pragma unroll
  for (int w = 0; w < 33; w++) {
    cm |= (uint64_t)c << w;
    const uint32_t raw = w < 32 ? (s[w >> 3] >> (4 * (w & 7))) & 15u : 0u;
    c = raw + c > 8u;
  }
  return cm;
}
__device__ inline int fbn_digit(const uint32_t s[4], uint64_t cm, int w) {  // in [-8, 8]
  const int raw = w < 32 ? (int)((s[w >> 3] >> (4 * (w & 7))) & 15u) : 0;
  const int cin = (int)((cm >> w) & 1u);
  const int cout = w < 32 ? (int)((cm >> (w + 1)) & 1u) : 0;
  return raw + cin - 16 * cout;
}

// One FP256BN nym signature per lane.  The host materialises each item's hashed
// stream "sign" || 0x04 || t (64 zero bytes) || Nym (65) || ipk.Hash || msg in
// the region (word aligned); the kernel supplies t's words in registers.
// nymxy: X || Y (64 bytes, big-endian; the 0x04 prefix checked on the host).
__global__ __launch_bounds__(256) void k_nym_verify_fbn(int n, const uint32_t* __restrict__ rec,
                                                        const uint8_t* __restrict__ nymxy,
                                                        const uint32_t* __restrict__ region,
                                                        const uint64_t* __restrict__ roff,  // word offsets
                                                        const uint32_t* __restrict__ rlen,  // stream bytes
                                                        const uint32_t* __restrict__ tables,
                                                        uint32_t* __restrict__ vtab,
                                                        int32_t* __restrict__ status, int base, int tile) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;  // tiled as k_nym_verify
  const int i = base + li;
  if (li >= tile || i >= n || status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * NREC;
  uint32_t pw[16];
  load_be_words(nymxy + (size_t)i * 64, pw);
  uint32_t nx[8], ny[8];
#pragma unroll
  for (int k = 0; k < 8; k++) nx[k] = pw[7 - k], ny[k] = pw[15 - k];
  if (!p256::lt256(nx, fbn::PM::M) || !p256::lt256(ny, fbn::PM::M)) {
    status[i] = FTS_E_NYM_BADKEY;
    return;
  }
  const fbn::Fp Qx = p256::to_mont(fbn::load<fbn::PM>(nx)), Qy = p256::to_mont(fbn::load<fbn::PM>(ny));
  if (!fbn::on_curve(Qx, Qy)) {
    status[i] = FTS_E_NYM_BADKEY;
    return;
  }
  // s_sk HSk + s_rnym HRand: 2 x 16 mixed additions from the tables
  fbn::PJ acc = fbn::pj_inf();
#pragma unroll 1
  for (int q = 0; q < 2; q++) {
    const uint32_t* sc = R + 8 + 8 * q;
    const uint32_t* tb = tables + (size_t)q * FBN_NW * FBN_ND * 16;
    for (int w = 0; w < FBN_NW; w++) {
      const uint32_t d = (sc[w >> 1] >> (16 * (w & 1))) & 0xffffu;
      if (d) {
        const uint32_t* t = tb + ((size_t)w * FBN_ND + d) * 16;
        acc = fbn::pj_madd(acc, fbn::load<fbn::PM>(t), fbn::load<fbn::PM>(t + 8));
      }
    }
  }
  // (r - c) Nym by GLV: e = k1 + k2 lambda, one joint chain of k1 (+-Nym) +
  // k2 (+-phi(Nym)) over 33 signed 4-bit windows (|k_i| < 2^128), 128 doublings
  // instead of 252; tables 1..8 of both points in the lane's global slot
  uint32_t e[8];
  {
    uint32_t bw = 0, nz = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) nz |= R[k];
#pragma unroll
    for (int k = 0; k < 8; k++) e[k] = nz ? subb(fbn::RM::M[k], R[k], bw, bw) : 0u;
  }
  uint32_t k1[4], k2[4], s1, s2;
  fts::glv_decompose<fbn::GlvK>(e, k1, s1, k2, s2);
  const fbn::Fp nQy = fbn::sub(fbn::Fp{}, Qy);
  const fbn::Fp Px = Qx, Py = s1 ? nQy : Qy;
  const fbn::Fp Ex = fbn::mul(Qx, fbn::load<fbn::PM>(fbn::GlvK::BETA)), Ey = s2 ? nQy : Qy;
  const size_t stride = (size_t)tile;
  {
    fbn::PJ cp, ce;
    cp.x = Px, cp.y = Py, cp.z = fbn::load<fbn::PM>(fbn::PM::ONE);
    ce.x = Ex, ce.y = Ey, ce.z = cp.z;
    fbn_vtab_store(vtab, stride, (size_t)li, 0, cp);
    fbn_vtab_store(vtab, stride, (size_t)li, 8, ce);
    for (int k = 1; k < 8; k++) {
      cp = fbn::pj_madd(cp, Px, Py);
      ce = fbn::pj_madd(ce, Ex, Ey);
      fbn_vtab_store(vtab, stride, (size_t)li, k, cp);
      fbn_vtab_store(vtab, stride, (size_t)li, 8 + k, ce);
    }
  }
  const uint64_t ca = fbn_recode(k1), cb = fbn_recode(k2);
  fbn::PJ vb = fbn::pj_inf();
  for (int w = 32; w >= 0; w--) {
    const int da = fbn_digit(k1, ca, w), db = fbn_digit(k2, cb, w);
    fbn::PJ qa, qb;
    if (da) qa = fbn_vtab_load(vtab, stride, (size_t)li, (da < 0 ? -da : da) - 1);
    if (db) qb = fbn_vtab_load(vtab, stride, (size_t)li, 8 + (db < 0 ? -db : db) - 1);
    if (w != 32) vb = fbn::pj_dbl(fbn::pj_dbl(fbn::pj_dbl(fbn::pj_dbl(vb))));
    if (da) {
      if (da < 0) qa.y = fbn::sub(fbn::Fp{}, qa.y);
      vb = fbn::pj_add(vb, qa);
    }
    if (db) {
      if (db < 0) qb.y = fbn::sub(fbn::Fp{}, qb.y);
      vb = fbn::pj_add(vb, qb);
    }
  }
  const fbn::PJ X = fbn::pj_add(acc, vb);
  uint32_t tw[16];
  if (fbn::is_zero(X.z)) {
#pragma unroll
    for (int k = 0; k < 16; k++) tw[k] = 0u;  // t = O (zero nonces): AMCL ToBytes of infinity = 0x04 || 0 || 1
    tw[15] = 1u;
  } else {
    const fbn::Fp zi = p256::inv(X.z), zi2 = fbn::sqr(zi);
    const fbn::Fp ax = p256::from_mont(fbn::mul(X.x, zi2)), ay = p256::from_mont(fbn::mul(X.y, fbn::mul(zi2, zi)));
#pragma unroll
    for (int k = 0; k < 8; k++) tw[k] = ax.v[7 - k], tw[8 + k] = ay.v[7 - k];
  }
  const uint32_t* m = region + roff[i];
  const uint32_t ltot = rlen[i];
  const uint32_t nb = sha_blocks(ltot);  // >= 3
  uint32_t st[8], w[16];
  sha256_init(st);
  // block 0: "sign" 0x04 t[0..58]
  w[0] = 0x7369676eu;
  w[1] = 0x04000000u | (tw[0] >> 8);
#pragma unroll
  for (int k = 2; k < 16; k++) w[k] = (tw[k - 2] << 24) | (tw[k - 1] >> 8);
  sha256_compress(st, w);
  // block 1: t[59..63] then the host's bytes (Nym, ipk.Hash, message)
  w[0] = (tw[14] << 24) | (tw[15] >> 8);
  w[1] = (tw[15] << 24) | (region_word(m, ltot, nb, 17) & 0x00ffffffu);
#pragma unroll
  for (int k = 2; k < 16; k++) w[k] = region_word(m, ltot, nb, 16 + k);
  sha256_compress(st, w);
  for (uint32_t blk = 2; blk < nb; blk++) {
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = region_word(m, ltot, nb, 16 * blk + k);
    sha256_compress(st, w);
  }
  uint32_t c1[8], c2[8];
  digest_mod_rfbn(st, c1);
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = c1[7 - k];
#pragma unroll
  for (int k = 0; k < 8; k++) w[8 + k] = R[24 + k];
  sha256_init(st);
  sha256_compress(st, w);
  w[0] = 0x80000000u;
#pragma unroll
  for (int k = 1; k < 15; k++) w[k] = 0u;
  w[15] = 512u;
  sha256_compress(st, w);
  digest_mod_rfbn(st, c2);
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) diff |= c2[k] ^ R[k];
  status[i] = diff ? FTS_E_NYM_INVALID : FTS_OK;
}

// ------------------------------------------------------------------- host
const uint32_t kR[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                        0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

// big-endian bytes -> integer (LE limbs) if it fits 256 bits
bool be_to_limbs(const uint8_t* b, size_t len, uint32_t out[8]) {
  size_t st = 0;
  while (st < len && b[st] == 0) st++;
  memset(out, 0, 32);
  if (len - st > 32) return false;
  for (size_t k = st; k < len; k++) {
    const size_t bit = (len - 1 - k) * 8;
    out[bit / 32] |= (uint32_t)b[k] << (bit % 32);
  }
  return true;
}
bool ge_r(const uint32_t a[8]) {
  for (int k = 7; k >= 0; k--)
    if (a[k] != kR[k]) return a[k] > kR[k];
  return true;
}
void sub_r(uint32_t a[8]) {
  uint64_t bw = 0;
  for (int k = 0; k < 8; k++) {
    const uint64_t d = (uint64_t)a[k] - kR[k] - bw;
    a[k] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
}
// x * 256 + byte (x < r < 2^254): 9-limb then reduce
void mulacc_byte_mod_r(uint32_t x[8], uint8_t byte) {
  uint32_t t[9];
  uint64_t c = byte;
  for (int k = 0; k < 8; k++) {
    const uint64_t v = ((uint64_t)x[k] << 8) + c;
    t[k] = (uint32_t)v;
    c = v >> 32;
  }
  t[8] = (uint32_t)c;
  // t < 256 r + 256: subtract r until below (t[8] drops to 0 then compare)
  for (int guard = 0; guard < 300; guard++) {
    if (t[8] == 0) {
      memcpy(x, t, 32);
      if (!ge_r(x)) return;
    }
    uint64_t bw = 0;
    for (int k = 0; k < 9; k++) {
      const uint64_t d = (uint64_t)t[k] - (k < 8 ? kR[k] : 0u) - bw;
      t[k] = (uint32_t)d;
      bw = (d >> 63) & 1;
    }
  }
  memcpy(x, t, 32);
}
// G1.Mul semantics for an unreduced big-endian scalar: value mod r
void scalar_mod_r(const uint8_t* b, size_t len, uint32_t out[8]) {
  if (be_to_limbs(b, len, out)) {
    while (ge_r(out)) sub_r(out);
    return;
  }
  memset(out, 0, 32);
  for (size_t k = 0; k < len; k++) mulacc_byte_mod_r(out, b[k]);
}

// NymSignature (idemix.proto): 1 proof_c, 2 proof_s_sk, 3 proof_s_r_nym, 4 nonce
// -> record + host verdict (FTS_OK: goes to the device)
int32_t parse_nym_sig(const uint8_t* sig, size_t len, uint32_t* rec) {
  memset(rec, 0, NREC * 4);
  if (!sig || len == 0) return FTS_E_NYM_MALFORMED;  // "invalid signature, it must not be empty"
  Pb pb{sig, len};
  const uint8_t* fv[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t fl[5] = {0, 0, 0, 0, 0};
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(f, wt, v, vl, iv)) return FTS_E_NYM_MALFORMED;
    if (f >= 1 && f <= 4) {
      if (wt != 2) return FTS_E_NYM_MALFORMED;
      fv[f] = v, fl[f] = vl;  // proto3: the last occurrence wins
    }
  }
  uint32_t c[8], nonce[8];
  // Nonce.Bytes() of a value wider than 32 bytes panics in mathlib BigToBytes
  if (!be_to_limbs(fv[4], fl[4], nonce)) return FTS_E_NYM_MALFORMED;
  scalar_mod_r(fv[2], fl[2], rec + 8);
  scalar_mod_r(fv[3], fl[3], rec + 16);
  for (int k = 0; k < 8; k++) rec[24 + k] = nonce[7 - k];  // big-endian words
  // Zr.Equals compares integers: an unreduced challenge can never match
  if (!be_to_limbs(fv[1], fl[1], c) || ge_r(c)) return FTS_E_NYM_INVALID;
  memcpy(rec, c, 32);
  return FTS_OK;
}

const uint32_t kRfbn[8] = {0xd10b500du, 0xf62d536cu, 0x1299921au, 0x0cdc65fbu,
                           0xee71a49eu, 0x46e5f25eu, 0xfffcf0cdu, 0xffffffffu};
bool ge_m(const uint32_t a[8], const uint32_t m[8]) {
  for (int k = 7; k >= 0; k--)
    if (a[k] != m[k]) return a[k] > m[k];
  return true;
}
void sub_m(uint32_t a[8], const uint32_t m[8]) {
  uint64_t bw = 0;
  for (int k = 0; k < 8; k++) {
    const uint64_t d = (uint64_t)a[k] - m[k] - bw;
    a[k] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
}
// FP256BN_AMCL Zr from bytes: AMCL FromBytes reads exactly the first 32 bytes
// (a shorter field makes the Go code index out of range -> FTS_E_NYM_MALFORMED)
int32_t parse_nym_sig_fbn(const uint8_t* sig, size_t len, uint32_t* rec) {
  memset(rec, 0, NREC * 4);
  if (!sig || len == 0) return FTS_E_NYM_MALFORMED;
  Pb pb{sig, len};
  const uint8_t* fv[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t fl[5] = {0, 0, 0, 0, 0};
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(f, wt, v, vl, iv)) return FTS_E_NYM_MALFORMED;
    if (f >= 1 && f <= 4) {
      if (wt != 2) return FTS_E_NYM_MALFORMED;
      fv[f] = v, fl[f] = vl;
    }
  }
  for (int f = 1; f <= 4; f++)
    if (fl[f] < 32) return FTS_E_NYM_MALFORMED;
  uint32_t v[4][8];
  for (int f = 1; f <= 4; f++) be_to_limbs(fv[f], 32, v[f - 1]);
  for (int q = 1; q <= 2; q++)  // s mod r (2^256 < 2 r: one subtraction)
    if (ge_m(v[q], kRfbn)) sub_m(v[q], kRfbn);
  memcpy(rec + 8, v[1], 32);
  memcpy(rec + 16, v[2], 32);
  for (int k = 0; k < 8; k++) rec[24 + k] = v[3][7 - k];
  if (ge_m(v[0], kRfbn)) return FTS_E_NYM_INVALID;  // Zr.Equals: an unreduced c never matches
  memcpy(rec, v[0], 32);
  return FTS_OK;
}

// FP256BN issuer bases: plain big-endian ECP coordinates -> Montgomery, on-curve flags
__global__ void k_fbn_bases(int nb, const uint32_t* __restrict__ plain, uint32_t* __restrict__ mont,
                            int32_t* __restrict__ ok) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  uint32_t x[8], y[8];
  for (int k = 0; k < 8; k++) x[k] = plain[b * 16 + k], y[k] = plain[b * 16 + 8 + k];
  bool good = p256::lt256(x, fbn::PM::M) && p256::lt256(y, fbn::PM::M);
  const fbn::Fp mx = p256::to_mont(fbn::load<fbn::PM>(x)), my = p256::to_mont(fbn::load<fbn::PM>(y));
  good = good && fbn::on_curve(mx, my);
  for (int k = 0; k < 8; k++) mont[b * 16 + k] = mx.v[k], mont[b * 16 + 8 + k] = my.v[k];
  ok[b] = good ? 1 : 0;
}

}  // namespace

namespace fts {
// FP256BN fixed-base tables (FBN layout: FBN_NW windows x 2^16 unsigned digits,
// affine Montgomery) of nb bases given as plain LE-limb affine coordinates
// (16 words each, on the device); ok[b] <- base b canonical and on the curve.
// mont: nb * 16 words of scratch.  Used by the nym and identity-proof handles.
void fbn_build_tables(const uint32_t* plain, int nb, uint32_t* mont, int32_t* ok, uint32_t* tables, hipStream_t s) {
  k_fbn_bases<<<1, 64, 0, s>>>(nb, plain, mont, ok);
  const size_t ent = (size_t)nb * FBN_NW * FBN_ND;
  k_fbn_table<<<(unsigned)((ent + 255) / 256), 256, 0, s>>>(nb, mont, tables);
}
size_t fbn_words_per_base() { return (size_t)FBN_NW * FBN_ND * 16; }
}  // namespace fts

namespace {

#define ICHK(x)                                    \
  do {                                             \
    if ((x) != hipSuccess) return FTS_API_EDEVICE; \
  } while (0)

constexpr int NSLOT = 3;
// items per nym-kernel launch (the GLV lane tables are sized for one tile)
constexpr size_t NYM_TILE = 262144;
struct Slot {
  hipStream_t stream = nullptr;
  uint8_t* d_buf = nullptr;  // rec | nym | moff | mlen | status | vtab | messages
  size_t d_cap = 0;
  uint8_t* h_buf = nullptr;  // pinned staging of everything above but vtab
  size_t h_cap = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  float ms = 0.f;
};

}  // namespace

struct fts_idemix_ipk {
  int device = -1;
  int curve = 1;                 // mathlib CurveID: 1 BN254, 0 FP256BN_AMCL
  uint32_t* d_tables = nullptr;  // HSk, HRand (FB_W-bit windows)
  uint32_t* d_hash = nullptr;    // ipk.Hash as 8 big-endian words
  uint8_t hash[32];
  std::mutex mu;
  std::condition_variable cv;
  Slot slot[NSLOT];
  bool busy[NSLOT] = {false, false, false};
  float last_ms = 0.f;
  size_t tile = NYM_TILE;  // items per launch (FTS_NYM_TILE overrides, for tests)
};

namespace {
void ipk_free(fts_idemix_ipk* k) {
  if (!k) return;
  if (k->device >= 0) (void)hipSetDevice(k->device);
  for (auto& S : k->slot) {
    if (S.stream) (void)hipStreamSynchronize(S.stream), (void)hipStreamDestroy(S.stream);
    for (auto& e : S.ev)
      if (e) (void)hipEventDestroy(e);
    if (S.d_buf) (void)hipFree(S.d_buf);
    if (S.h_buf) (void)hipHostFree(S.h_buf);
  }
  if (k->d_tables) (void)hipFree(k->d_tables);
  if (k->d_hash) (void)hipFree(k->d_hash);
  delete k;
}

// ECP{x, y} -> affine Montgomery point (host), on-curve checked
bool ecp_point(const uint8_t* v, size_t vl, host::G1A& out) {
  Pb pb{v, vl};
  const uint8_t *x = nullptr, *y = nullptr;
  size_t xl = 0, yl = 0;
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* fv;
    size_t fl;
    uint64_t iv;
    if (!pb.next(f, wt, fv, fl, iv)) return false;
    if (f == 1 && wt == 2) x = fv, xl = fl;
    if (f == 2 && wt == 2) y = fv, yl = fl;
  }
  if (xl != 32 || yl != 32) return false;
  uint8_t raw[64];
  memcpy(raw, x, 32);
  memcpy(raw + 32, y, 32);
  return host::g1_from_bytes(raw, 64, out) && !out.inf;
}
}  // namespace

extern "C" {

int fts_idemix_ipk_create(int device, const uint8_t* ipk, size_t ipk_len, int curve_id, fts_idemix_ipk** out) {
  if (!out || !ipk || !ipk_len || (curve_id != FTS_CURVE_BN254 && curve_id != FTS_CURVE_FP256BN_AMCL))
    return FTS_API_EINVAL;
  *out = nullptr;
  // IssuerPublicKey: 2 h_sk, 3 h_rand (ECP), 10 hash
  Pb pb{ipk, ipk_len};
  const uint8_t *hsk = nullptr, *hr = nullptr, *hash = nullptr;
  size_t hskl = 0, hrl = 0, hashl = 0;
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(f, wt, v, vl, iv)) return FTS_API_EPP;
    if (wt != 2) continue;
    if (f == 2) hsk = v, hskl = vl;
    if (f == 3) hr = v, hrl = vl;
    if (f == 10) hash = v, hashl = vl;
  }
  if (!hsk || !hr) return FTS_API_EPP;
  host::G1A base[2]{};
  uint32_t plain[32];  // FP256BN: plain coordinates, little-endian limbs
  if (curve_id == FTS_CURVE_BN254) {
    if (!ecp_point(hsk, hskl, base[0]) || !ecp_point(hr, hrl, base[1])) return FTS_API_EPP;
  } else {
    const uint8_t* e[2] = {hsk, hr};
    const size_t el[2] = {hskl, hrl};
    for (int b = 0; b < 2; b++) {
      Pb q{e[b], el[b]};
      const uint8_t *x = nullptr, *y = nullptr;
      size_t xl = 0, yl = 0;
      while (q.o < q.n) {
        uint32_t f, wt;
        const uint8_t* fv;
        size_t fl;
        uint64_t iv;
        if (!q.next(f, wt, fv, fl, iv)) return FTS_API_EPP;
        if (f == 1 && wt == 2) x = fv, xl = fl;
        if (f == 2 && wt == 2) y = fv, yl = fl;
      }
      if (xl != 32 || yl != 32) return FTS_API_EPP;
      be_to_limbs(x, 32, plain + b * 16);
      be_to_limbs(y, 32, plain + b * 16 + 8);
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return FTS_API_EDEVICE;
  fts_idemix_ipk* k = new fts_idemix_ipk();
  k->device = device;
  k->curve = curve_id;
  if (const char* e = getenv("FTS_NYM_TILE")) k->tile = (size_t)std::max(64L, std::min((long)NYM_TILE, atol(e)));
  // copy(proofData[index:], ipk.Hash) into a FieldBytes window
  memset(k->hash, 0, 32);
  if (hash) memcpy(k->hash, hash, std::min<size_t>(hashl, 32));
  auto fail = [&](int rc) {
    ipk_free(k);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(FTS_API_EDEVICE);
  uint32_t hb[32];
  for (int b = 0; b < 2; b++) {
    memcpy(&hb[b * 16], base[b].x.v, 32);
    memcpy(&hb[b * 16 + 8], base[b].y.v, 32);
  }
  uint32_t hw[8];
  for (int q = 0; q < 8; q++)
    hw[q] = ((uint32_t)k->hash[4 * q] << 24) | ((uint32_t)k->hash[4 * q + 1] << 16) |
            ((uint32_t)k->hash[4 * q + 2] << 8) | k->hash[4 * q + 3];
  uint32_t* d_bases = nullptr;
  uint32_t* d_scr = nullptr;
  hipStream_t s0 = nullptr;
  const bool bn = curve_id == FTS_CURVE_BN254;
  const size_t tab_b = bn ? 2 * fb_words_per_base() * 4 : (size_t)2 * FBN_NW * FBN_ND * 16 * 4;
  const size_t scr_b = bn ? table_build_scratch_bytes(2) : 2 * 16 * 4 + 64;
  bool ok = hipStreamCreateWithFlags(&s0, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&k->d_tables, tab_b) == hipSuccess && hipMalloc(&k->d_hash, 32) == hipSuccess &&
            hipMalloc(&d_bases, sizeof(hb)) == hipSuccess && hipMalloc(&d_scr, scr_b) == hipSuccess &&
            hipMemcpyAsync(d_bases, bn ? hb : plain, sizeof(hb), hipMemcpyHostToDevice, s0) == hipSuccess &&
            hipMemcpyAsync(k->d_hash, hw, 32, hipMemcpyHostToDevice, s0) == hipSuccess;
  bool on_curve = true;
  if (ok && bn) {
    launch_build_tables(d_bases, 2, k->d_tables, d_scr, s0);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s0) == hipSuccess;
  } else if (ok) {
    // plain -> Montgomery + on-curve flags (into the scratch), then the window tables
    uint32_t* mont = d_scr;
    int32_t* flags = reinterpret_cast<int32_t*>(d_scr + 32);
    int32_t hf[2] = {0, 0};
    k_fbn_bases<<<1, 64, 0, s0>>>(2, d_bases, mont, flags);
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, s0) == hipSuccess &&
         hipStreamSynchronize(s0) == hipSuccess;
    on_curve = hf[0] == 1 && hf[1] == 1;
    if (ok && on_curve) {
      const size_t ent = (size_t)2 * FBN_NW * FBN_ND;
      k_fbn_table<<<(unsigned)((ent + 255) / 256), 256, 0, s0>>>(2, mont, k->d_tables);
      ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s0) == hipSuccess;
    }
  }
  if (s0) (void)hipStreamSynchronize(s0);  // an error path may leave copies queued on s0
  if (d_bases) (void)hipFree(d_bases);
  if (d_scr) (void)hipFree(d_scr);
  if (ok && !on_curve) {
    if (s0) (void)hipStreamDestroy(s0);
    return fail(FTS_API_EPP);
  }
  if (s0) (void)hipStreamDestroy(s0);
  for (auto& S : k->slot) {
    ok = ok && hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) == hipSuccess;
    for (auto& e : S.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  }
  if (!ok) return fail(FTS_API_EDEVICE);
  *out = k;
  return FTS_API_OK;
}

void fts_idemix_ipk_destroy(fts_idemix_ipk* k) { ipk_free(k); }

int fts_idemix_identity_nym(const uint8_t* id, size_t len, const uint8_t** nym, size_t* nym_len) {
  if (!id || !nym || !nym_len) return FTS_API_EINVAL;
  Pb pb{id, len};
  *nym = nullptr, *nym_len = 0;
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(f, wt, v, vl, iv)) return FTS_API_EINVAL;
    if (f == 1) {
      if (wt != 2) return FTS_API_EINVAL;
      *nym = v, *nym_len = vl;
    }
  }
  return *nym_len ? FTS_API_OK : FTS_API_EINVAL;  // crypto/deserializer.go:45-47: empty nym rejected
}

int fts_nym_verify_batch(fts_idemix_ipk* K, size_t n, const fts_nym_item* items, int32_t* status) {
  if (!K || n > (size_t)(1u << 24) || (n && (!items || !status))) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  // message words per item: BN254 the message alone; FP256BN the whole hashed
  // stream (166-byte prefix + message), each padded to whole words + 1
  const bool bn = K->curve == FTS_CURVE_BN254;
  const size_t pre = bn ? 0 : 166;
  size_t mtot_w = 0;
  for (size_t i = 0; i < n; i++) {
    if (items[i].msg_len > 0xffffff00u || (items[i].msg_len && !items[i].msg)) return FTS_API_EINVAL;
    mtot_w += (pre + items[i].msg_len + 3) / 4 + 1;
  }
  int k = -1;
  {
    std::unique_lock<std::mutex> l(K->mu);
    K->cv.wait(l, [&] {
      for (int j = 0; j < NSLOT; j++)
        if (!K->busy[j]) return true;
      return false;
    });
    for (int j = 0; j < NSLOT && k < 0; j++)
      if (!K->busy[j]) k = j;
    K->busy[k] = true;
  }
  struct Guard {
    fts_idemix_ipk* K;
    int k;
    ~Guard() {
      if (K->slot[k].stream) (void)hipStreamSynchronize(K->slot[k].stream);
      std::lock_guard<std::mutex> l(K->mu);
      K->last_ms = K->slot[k].ms;
      K->busy[k] = false;
      K->cv.notify_one();
    }
  } guard{K, k};
  Slot& D = K->slot[k];
  ICHK(hipSetDevice(K->device));
  // layout: rec | nym | moff | mlen | status | messages (| vtab on the device only)
  const size_t rec_b = n * NREC * 4, nym_b = n * 64, off_b = n * 8, len_b = n * 4, st_b = n * 4;
  const size_t o_nym = rec_b, o_off = o_nym + nym_b, o_len = o_off + off_b, o_st = o_len + len_b,
               o_msg = (o_st + st_b + 255) & ~size_t(255), h_need = o_msg + mtot_w * 4;
  // GLV lane tables (16 Jacobian entries, 1,536 B per lane) for one tile of NYM_TILE
  // items: bounded at 384 MiB per slot whatever n is; a call above NYM_TILE items
  // runs one launch per tile on the slot's stream (a 2^24-item call
  // asked for ~38 GB here)
  const size_t tile = std::min<size_t>(n, K->tile);
  const size_t vt_b = tile * 16 * 24 * 4, o_vt = (h_need + 255) & ~size_t(255), d_need = o_vt + vt_b;
  if (D.h_cap < h_need) {
    if (D.h_buf) (void)hipHostFree(D.h_buf);
    D.h_buf = nullptr, D.h_cap = 0;
    if (hipHostMalloc(&D.h_buf, h_need + h_need / 2, hipHostMallocDefault) != hipSuccess) return FTS_API_ENOMEM;
    D.h_cap = h_need + h_need / 2;
  }
  if (D.d_cap < d_need) {
    if (D.d_buf) (void)hipFree(D.d_buf);
    D.d_buf = nullptr, D.d_cap = 0;
    if (hipMalloc(&D.d_buf, d_need + d_need / 2) != hipSuccess) return FTS_API_ENOMEM;
    D.d_cap = d_need + d_need / 2;
  }
  uint8_t* h = D.h_buf;
  uint64_t* hoff = reinterpret_cast<uint64_t*>(h + o_off);
  {
    uint64_t o = 0;
    for (size_t i = 0; i < n; i++) hoff[i] = o, o += (pre + items[i].msg_len + 3) / 4 + 1;
  }
  auto pack = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const fts_nym_item& it = items[i];
      uint32_t* rec = reinterpret_cast<uint32_t*>(h) + i * NREC;
      int32_t st = bn ? parse_nym_sig(it.sig, it.sig_len, rec) : parse_nym_sig_fbn(it.sig, it.sig_len, rec);
      uint8_t* nr = h + o_nym + i * 64;
      // NymPublicKey import (crypto/deserializer.go:49-56) precedes Verify: a key of
      // the wrong length / form fails first; its point checks run on the device.
      // BN254: G1.Bytes() raw X||Y (64 B); FP256BN: ECP.ToBytes 0x04||X||Y (65 B).
      const bool key_ok = it.nym && (bn ? it.nym_len == 64 : it.nym_len == 65 && it.nym[0] == 0x04);
      if (key_ok) memcpy(nr, it.nym + (bn ? 0 : 1), 64);
      else memset(nr, 0, 64), st = FTS_E_NYM_BADKEY;
      reinterpret_cast<int32_t*>(h + o_st)[i] = st;
      reinterpret_cast<uint32_t*>(h + o_len)[i] = (uint32_t)(pre + it.msg_len);
      uint8_t* mw = h + o_msg + hoff[i] * 4;
      const size_t wl = ((pre + it.msg_len + 3) / 4 + 1) * 4;
      if (!bn) {  // "sign" || 0x04 || t (device) || Nym || ipk.Hash
        memcpy(mw, "sign", 4);
        mw[4] = 0x04;
        memset(mw + 5, 0, 64);
        if (key_ok) memcpy(mw + 69, it.nym, 65);
        else memset(mw + 69, 0, 65);
        memcpy(mw + 134, K->hash, 32);
      }
      if (it.msg_len) memcpy(mw + pre, it.msg, it.msg_len);
      memset(mw + pre + it.msg_len, 0, wl - pre - it.msg_len);
    }
  };
  const size_t CH = 2048, nch = (n + CH - 1) / CH;
  fts::host_parallel_for(nch, [&](size_t c) { pack(c * CH, std::min(n, (c + 1) * CH)); });
  uint8_t* d = D.d_buf;
  ICHK(hipMemcpyAsync(d, h, h_need, hipMemcpyHostToDevice, D.stream));
  ICHK(hipEventRecord(D.ev[0], D.stream));
  for (size_t base = 0; base < n; base += tile) {
    const unsigned grid = (unsigned)((tile + 255) / 256);
    if (bn)
      k_nym_verify<<<grid, 256, 0, D.stream>>>(
          (int)n, reinterpret_cast<const uint32_t*>(d), d + o_nym, reinterpret_cast<const uint32_t*>(d + o_msg),
          reinterpret_cast<const uint64_t*>(d + o_off), reinterpret_cast<const uint32_t*>(d + o_len), K->d_tables,
          K->d_hash, reinterpret_cast<uint32_t*>(d + o_vt), reinterpret_cast<int32_t*>(d + o_st), (int)base,
          (int)tile);
    else
      k_nym_verify_fbn<<<grid, 256, 0, D.stream>>>(
          (int)n, reinterpret_cast<const uint32_t*>(d), d + o_nym, reinterpret_cast<const uint32_t*>(d + o_msg),
          reinterpret_cast<const uint64_t*>(d + o_off), reinterpret_cast<const uint32_t*>(d + o_len), K->d_tables,
          reinterpret_cast<uint32_t*>(d + o_vt), reinterpret_cast<int32_t*>(d + o_st), (int)base, (int)tile);
  }
  ICHK(hipGetLastError());
  ICHK(hipEventRecord(D.ev[1], D.stream));
  ICHK(hipMemcpyAsync(h + o_st, d + o_st, st_b, hipMemcpyDeviceToHost, D.stream));
  ICHK(hipStreamSynchronize(D.stream));
  memcpy(status, h + o_st, st_b);
  ICHK(hipEventElapsedTime(&D.ms, D.ev[0], D.ev[1]));
  return FTS_API_OK;
}

int fts_nym_last_timings(fts_idemix_ipk* K, float* ms) {
  if (!K || !ms) return FTS_API_EINVAL;
  std::lock_guard<std::mutex> l(K->mu);
  *ms = K->last_ms;
  return FTS_API_OK;
}

}  // extern "C"
