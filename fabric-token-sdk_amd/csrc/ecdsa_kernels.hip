// Batched ECDSA P-256 owner-signature verification (SURVEY.md §8(f) row 4,
// the x509 half): one device pass verifies a batch of (message, DER
// signature, public key) triples.
//
// Reference: validator/ecdsa/ecdsa.go:82-113 and
// services/identity/x509/crypto/ecdsa.go:46-77:
//   asn1.Unmarshal(sigma, &Signature{R, S})        -> error   (host: parse_sig)
//   digest = sha256(message)                        -> k_ecdsa_digest
//   IsLowS(pk, S) else "signature is not in lowS"   -> host: parse_sig
//   ecdsa.Verify(pk, digest, R, S) else "signature not valid" -> k_ecdsa_verify
// Owner signatures are checked by TransferSignatureValidate
// (validator/validator_transfer.go:29-62) once per input token.
//
// Kernels (one signature per lane):
//   k_ecdsa_table   once per device: 16 x 65536 affine multiples d*2^(16w)*G
//                   (16-bit fixed-base windows, 64 MiB in HBM)
//   k_ecdsa_digest  SHA-256 of each message (full-rate INT32 work)
//   k_ecdsa_verify  pk on-curve check, w = s^-1 mod n (Fermat), u1*G as 16
//                   mixed additions from the table, u2*Q with a 4-bit window
//                   (252 doublings + <= 64 additions), X.x == r checked
//                   projectively (r*Z^2 == X, and (r+n)*Z^2 when r+n < p)
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
#include "device/p256.hpp"

using namespace p256;

namespace fts {
void host_parallel_for(size_t n, const std::function<void(size_t)>& f);  // fts_api.cpp (persistent host pool)
}

namespace {

constexpr int REC_WORDS = 32;  // r[8] s[8] qx[8] qy[8], little-endian u32 limbs

// FB_W-bit fixed-base windows for u1*G: entry (w, d) = d * 2^(FB_W w) * G,
// affine Montgomery (16 words); d = 0 unused
constexpr int FB_W = 16, FB_NW = 256 / FB_W, FB_ND = 1 << FB_W;

__global__ __launch_bounds__(256) void k_ecdsa_table(uint32_t* __restrict__ table) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= FB_NW * FB_ND) return;
  const int w = id / FB_ND, d = id % FB_ND;
  uint32_t* out = table + (size_t)id * 16;
  if (d == 0) {
    for (int i = 0; i < 16; i++) out[i] = 0;
    return;
  }
  const Fp gx = load<PM>(CGX), gy = load<PM>(CGY);
  PJ p = pj_inf();
  for (int b = FB_W - 1; b >= 0; b--) {
    p = pj_dbl(p);
    if ((d >> b) & 1) p = pj_madd(p, gx, gy);
  }
  for (int k = 0; k < FB_W * w; k++) p = pj_dbl(p);
  const Fp zi = inv(p.z), zi2 = sqr(zi);
  const Fp x = mul(p.x, zi2), y = mul(p.y, mul(zi2, zi));
  for (int i = 0; i < 8; i++) out[i] = x.v[i], out[8 + i] = y.v[i];
}

__global__ __launch_bounds__(256) void k_ecdsa_digest(int n, const uint8_t* __restrict__ msg,
                                                      const uint64_t* __restrict__ moff,
                                                      const uint32_t* __restrict__ mlen,
                                                      const int32_t* __restrict__ status,
                                                      uint32_t* __restrict__ e) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != FTS_OK) return;
  const uint8_t* m = msg + moff[i];
  const uint32_t len = mlen[i];
  fts::Sha256 h;
  h.init();
  uint32_t off = 0;
  for (; off + 64 <= len; off += 64) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
      w[k] = ((uint32_t)m[off + 4 * k] << 24) | ((uint32_t)m[off + 4 * k + 1] << 16) |
             ((uint32_t)m[off + 4 * k + 2] << 8) | (uint32_t)m[off + 4 * k + 3];
    fts::sha256_compress(h.st, w);
  }
  h.total = off;
  h.update(m + off, len - off);
  uint8_t dg[32];
  h.final(dg);
  // digest as a big-endian 256-bit integer -> little-endian limbs
  for (int k = 0; k < 8; k++)
    e[(size_t)i * 8 + k] = ((uint32_t)dg[28 - 4 * k] << 24) | ((uint32_t)dg[29 - 4 * k] << 16) |
                           ((uint32_t)dg[30 - 4 * k] << 8) | (uint32_t)dg[31 - 4 * k];
}

__global__ __launch_bounds__(256) void k_ecdsa_verify(int n, const uint32_t* __restrict__ rec,
                                                      const uint32_t* __restrict__ e,
                                                      const uint32_t* __restrict__ table,
                                                      int32_t* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * REC_WORDS;
  uint32_t r[8], s[8], qx[8], qy[8], ev[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = R[k], s[k] = R[8 + k], qx[k] = R[16 + k], qy[k] = R[24 + k], ev[k] = e[(size_t)i * 8 + k];
  // public key: canonical coordinates on the curve (Go: nistec SetBytes)
  if (!lt256(qx, PM::M) || !lt256(qy, PM::M)) {
    status[i] = FTS_E_SIG_INVALID;
    return;
  }
  const Fp Qx = to_mont(load<PM>(qx)), Qy = to_mont(load<PM>(qy));
  if (!on_curve(Qx, Qy)) {
    status[i] = FTS_E_SIG_INVALID;
    return;
  }
  // e mod n (e < 2^256 < 2n), w = s^-1, u1 = e*w, u2 = r*w  (plain, canonical)
  Fn em = load<NM>(ev);
  cond_sub(em, 0);
  const Fn wm = inv(to_mont(load<NM>(s)));
  const Fn u1 = mul(wm, em), u2 = mul(wm, load<NM>(r));
  // u1*G: FB_NW mixed additions from the fixed-base table
  PJ accg = pj_inf();
  for (int w = 0; w < FB_NW; w++) {
    const uint32_t d = (u1.v[(w * FB_W) >> 5] >> ((w * FB_W) & 31)) & (uint32_t)(FB_ND - 1);
    if (d) {
      const uint32_t* t = table + ((size_t)w * FB_ND + d) * 16;
      accg = pj_madd(accg, load<PM>(t), load<PM>(t + 8));
    }
  }
  // u2*Q: signed 4-bit window, digits in [-7, 8] over a table of 1..8 Q.
  // Carry into window w is bit w of cm (carry out of window 63 -> top digit).
  uint64_t cm = 0;
  {
    uint32_t c = 0;
    for (int w = 0; w < 64; w++) {
      cm |= (uint64_t)c << w;
      c = ((u2.v[w >> 3] >> (4 * (w & 7))) & 15u) + c > 8u;
    }
  }
  // carry out of window 63 = the top digit (0 or 1)
  const uint32_t c64 = (u2.v[7] >> 28) + ((uint32_t)(cm >> 63) & 1u) > 8u;
  PJ tab[9];
  tab[0] = pj_inf();
  tab[1].x = Qx, tab[1].y = Qy, tab[1].z = load<PM>(PM::ONE);
  for (int k = 2; k < 9; k++) tab[k] = pj_madd(tab[k - 1], Qx, Qy);
  PJ acc = c64 ? tab[1] : pj_inf();
  for (int nib = 63; nib >= 0; nib--) {
    acc = pj_dbl(pj_dbl(pj_dbl(pj_dbl(acc))));
    const int raw = (int)((u2.v[nib >> 3] >> (4 * (nib & 7))) & 15u);
    const int cin = (int)((cm >> nib) & 1u);
    const int cout = nib < 63 ? (int)((cm >> (nib + 1)) & 1u) : (int)c64;
    const int d = raw + cin - 16 * cout;
    if (d) {
      PJ q = tab[d < 0 ? -d : d];
      if (d < 0) q.y = sub(Fp{}, q.y);
      acc = pj_add(acc, q);
    }
  }
  const PJ X = pj_add(accg, acc);
  if (is_zero(X.z)) {
    status[i] = FTS_E_SIG_INVALID;
    return;
  }
  // X.x mod n == r  <=>  r*Z^2 == X  or  (r+n < p and (r+n)*Z^2 == X)
  const Fp z2 = sqr(X.z);
  bool ok = eq(mul(to_mont(load<PM>(r)), z2), X.x);
  if (!ok && lt256(r, P_MINUS_N)) {
    uint32_t rn[8], c = 0;
    for (int k = 0; k < 8; k++) {
      uint32_t co;
      rn[k] = __builtin_addc(r[k], NM::M[k], c, &co);
      c = co;
    }
    ok = eq(mul(to_mont(load<PM>(rn)), z2), X.x);
  }
  status[i] = ok ? FTS_OK : FTS_E_SIG_INVALID;
}

// ------------------------------------------------------------------- host

// n and floor(n/2) as big-endian bytes
const uint8_t kN[32] = {0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                        0xbc, 0xe6, 0xfa, 0xad, 0xa7, 0x17, 0x9e, 0x84, 0xf3, 0xb9, 0xca, 0xc2, 0xfc, 0x63, 0x25, 0x51};
const uint8_t kHalfN[32] = {0x7f, 0xff, 0xff, 0xff, 0x80, 0x00, 0x00, 0x00, 0x7f, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                            0xde, 0x73, 0x7d, 0x56, 0xd3, 0x8b, 0xcf, 0x42, 0x79, 0xdc, 0xe5, 0x61, 0x7e, 0x31, 0x92, 0xa8};

// Go encoding/asn1 tag+length (asn1.go parseTagAndLength): single-byte tag,
// DER-minimal lengths, no indefinite form.
bool der_tl(const uint8_t* b, size_t len, size_t& off, uint8_t tag, size_t& body) {
  if (off >= len || b[off] != tag) return false;
  off++;
  if (off >= len) return false;
  uint8_t l0 = b[off++];
  size_t L = 0;
  if (!(l0 & 0x80)) {
    L = l0;
  } else {
    const int nb = l0 & 0x7f;
    if (nb == 0) return false;  // indefinite length (not DER)
    for (int k = 0; k < nb; k++) {
      if (off >= len) return false;
      if (L >= (1u << 23)) return false;  // length too large
      L = (L << 8) | b[off++];
      if (L == 0) return false;  // superfluous leading zeros
    }
    if (L < 0x80) return false;  // non-minimal length
  }
  if (L > len - off) return false;  // data truncated
  body = L;
  return true;
}

// Go parseBigInt (asn1.go checkInteger): non-empty, minimally encoded,
// two's complement.  Returns false on a parse error; sets neg / mag (up to
// 32 big-endian bytes, big = magnitude wider than 32 bytes).
bool der_int(const uint8_t* p, size_t L, bool& neg, bool& zero, bool& big, uint8_t mag[32]) {
  if (L == 0) return false;
  if (L > 1 && ((p[0] == 0 && !(p[1] & 0x80)) || (p[0] == 0xff && (p[1] & 0x80)))) return false;
  neg = (p[0] & 0x80) != 0;
  memset(mag, 0, 32);
  zero = true;
  for (size_t k = 0; k < L; k++) zero &= p[k] == 0;
  if (neg) return true;  // rejected by ecdsa.Verify (r, s must be > 0); magnitude unused
  size_t st = 0;
  while (st < L && p[st] == 0) st++;
  big = L - st > 32;
  if (!big) memcpy(mag + 32 - (L - st), p + st, L - st);
  return true;
}

int cmp32(const uint8_t* a, const uint8_t* b) { return memcmp(a, b, 32); }

// One staging slot per concurrent call: its own stream, device buffers and
// pinned host staging, so one call's host parse/pack overlaps another's kernels.
constexpr int NSLOT = 3;
struct Slot {
  hipStream_t stream = nullptr;
  uint32_t* d_table = nullptr;  // the device's shared table
  uint8_t* d_msg = nullptr;
  size_t msg_cap = 0;
  uint8_t* d_rec = nullptr;  // rec | e | moff | mlen | status
  size_t rec_cap = 0;
  uint8_t* h_stage = nullptr;  // pinned host staging
  size_t h_cap = 0;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  float ms[2] = {0.f, 0.f};
};
struct DevState {
  std::mutex mu;
  std::condition_variable cv;
  bool init = false;
  int init_err = 0;  // a failed initialisation is cached (no re-allocation on every retry)
  uint32_t* d_table = nullptr;
  Slot slot[NSLOT];
  bool busy[NSLOT] = {false, false, false};
  float ms[2] = {0.f, 0.f};  // k_ecdsa_digest, k_ecdsa_verify of the last finished call
};
DevState g_dev[16];

struct SlotGuard {
  DevState& G;
  int k;
  ~SlotGuard() {
    // an error path may leave a copy or kernel queued on the slot's stream that
    // still reads its pinned staging / device buffers: drain it before the next
    // caller may reuse (or re-allocate) them
    if (G.slot[k].stream) (void)hipStreamSynchronize(G.slot[k].stream);
    std::lock_guard<std::mutex> l(G.mu);
    G.ms[0] = G.slot[k].ms[0];
    G.ms[1] = G.slot[k].ms[1];
    G.busy[k] = false;
    G.cv.notify_one();
  }
};

#define ECHK(x)                                 \
  do {                                          \
    if ((x) != hipSuccess) return FTS_API_EDEVICE; \
  } while (0)

}  // namespace

extern "C" {

int fts_ecdsa_sig_parse(const uint8_t* sig, size_t sig_len, uint8_t* r32, uint8_t* s32, int32_t* status) {
  if (!status || !r32 || !s32) return FTS_API_EINVAL;
  memset(r32, 0, 32);
  memset(s32, 0, 32);
  size_t off = 0, body = 0, rl = 0, sl = 0;
  // asn1.Unmarshal(sigma, &Signature{}): trailing bytes after the SEQUENCE
  // are returned as `rest` and ignored (ecdsa.go:84); extra elements inside
  // the SEQUENCE after S are allowed by encoding/asn1.
  if (!sig || !der_tl(sig, sig_len, off, 0x30, body)) {
    *status = FTS_E_SIG_MALFORMED;
    return FTS_API_OK;
  }
  const uint8_t* in = sig + off;
  size_t io = 0;
  if (!der_tl(in, body, io, 0x02, rl)) {
    *status = FTS_E_SIG_MALFORMED;
    return FTS_API_OK;
  }
  const uint8_t* rp = in + io;
  io += rl;
  if (!der_tl(in, body, io, 0x02, sl)) {
    *status = FTS_E_SIG_MALFORMED;
    return FTS_API_OK;
  }
  const uint8_t* sp = in + io;
  bool rneg, rzero, rbig = false, sneg, szero, sbig = false;
  if (!der_int(rp, rl, rneg, rzero, rbig, r32) || !der_int(sp, sl, sneg, szero, sbig, s32)) {
    *status = FTS_E_SIG_MALFORMED;
    return FTS_API_OK;
  }
  // IsLowS: s <= n/2 (a negative s passes and is rejected by Verify below)
  if (!sneg && (sbig || cmp32(s32, kHalfN) > 0)) {
    *status = FTS_E_SIG_NOT_LOW_S;
    return FTS_API_OK;
  }
  // ecdsa.Verify: 0 < r < n, 0 < s < n
  if (rneg || rzero || rbig || cmp32(r32, kN) >= 0 || sneg || szero) {
    *status = FTS_E_SIG_INVALID;
    return FTS_API_OK;
  }
  *status = FTS_OK;
  return FTS_API_OK;
}

int fts_p256_pubkey_from_pkix(const uint8_t* der, size_t len, uint8_t* pk64) {
  // SubjectPublicKeyInfo{ {id-ecPublicKey, prime256v1}, BIT STRING 04||X||Y }:
  // the P-256 uncompressed encoding has this one fixed 26-byte prefix.
  static const uint8_t pre[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                  0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
  if (!der || !pk64) return FTS_API_EINVAL;
  if (len != 91 || memcmp(der, pre, 26) != 0 || der[26] != 0x04) return FTS_API_EINVAL;
  memcpy(pk64, der + 27, 64);
  return FTS_API_OK;
}

int fts_ecdsa_verify_batch(int device, size_t n, const fts_ecdsa_item* items, int32_t* status) {
  if (device < 0 || device >= 16 || n > (size_t)(1u << 24) || (n && (!items || !status))) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return FTS_API_EDEVICE;
  DevState& G = g_dev[device];
  int k = -1;
  {
    std::unique_lock<std::mutex> l(G.mu);
    ECHK(hipSetDevice(device));
    if (G.init_err) return G.init_err;
    if (!G.init) {
      // all or nothing: on any failure release what was created and cache the error
      hipStream_t s0 = nullptr;
      bool ok = hipStreamCreateWithFlags(&s0, hipStreamNonBlocking) == hipSuccess &&
                hipMalloc(&G.d_table, (size_t)FB_NW * FB_ND * 16 * 4) == hipSuccess;
      if (ok) {
        k_ecdsa_table<<<FB_NW * FB_ND / 256, 256, 0, s0>>>(G.d_table);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s0) == hipSuccess;
      }
      if (s0) (void)hipStreamDestroy(s0);
      for (auto& S : G.slot) {
        ok = ok && hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) == hipSuccess;
        for (auto& e : S.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
        S.d_table = G.d_table;
      }
      if (!ok) {
        for (auto& S : G.slot) {
          for (auto& e : S.ev)
            if (e) (void)hipEventDestroy(e), e = nullptr;
          if (S.stream) (void)hipStreamDestroy(S.stream), S.stream = nullptr;
          S.d_table = nullptr;
        }
        if (G.d_table) (void)hipFree(G.d_table), G.d_table = nullptr;
        G.init_err = FTS_API_EDEVICE;
        return G.init_err;
      }
      G.init = true;
    }
    G.cv.wait(l, [&] {
      for (int j = 0; j < NSLOT; j++)
        if (!G.busy[j]) return true;
      return false;
    });
    for (int j = 0; j < NSLOT && k < 0; j++)
      if (!G.busy[j]) k = j;
    G.busy[k] = true;
  }
  SlotGuard guard{G, k};
  Slot& D = G.slot[k];
  ECHK(hipSetDevice(device));
  // host: parse + low-S + range checks, pack records and messages into one
  // pinned staging buffer (records | e | moff | mlen | status | messages),
  // chunks in parallel, one H2D copy
  const size_t rec_b = n * REC_WORDS * 4, e_b = n * 32, off_b = n * 8, len_b = n * 4, st_b = n * 4;
  const size_t tot = rec_b + e_b + off_b + len_b + st_b;
  size_t mtot = 0;
  for (size_t i = 0; i < n; i++) {
    if (items[i].msg_len > 0xffffffffu || (items[i].msg_len && !items[i].msg)) return FTS_API_EINVAL;
    mtot += items[i].msg_len;
  }
  const size_t need = tot + mtot;
  if (D.h_cap < need) {
    if (D.h_stage) hipHostFree(D.h_stage);
    D.h_stage = nullptr, D.h_cap = 0;
    const size_t cap = need + need / 2;
    if (hipHostMalloc(&D.h_stage, cap, hipHostMallocDefault) != hipSuccess) return D.h_stage = nullptr, FTS_API_ENOMEM;
    D.h_cap = cap;
  }
  uint8_t* h = D.h_stage;
  uint32_t* hrec = reinterpret_cast<uint32_t*>(h);
  uint64_t* hoff = reinterpret_cast<uint64_t*>(h + rec_b + e_b);
  uint32_t* hlen = reinterpret_cast<uint32_t*>(h + rec_b + e_b + off_b);
  int32_t* hst = reinterpret_cast<int32_t*>(h + rec_b + e_b + off_b + len_b);
  uint8_t* hm = h + tot;
  {
    uint64_t o = 0;
    for (size_t i = 0; i < n; i++) hoff[i] = o, o += items[i].msg_len;
  }
  auto pack = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const fts_ecdsa_item& it = items[i];
      uint8_t r32[32], s32[32];
      int32_t st = FTS_E_SIG_MALFORMED;
      fts_ecdsa_sig_parse(it.sig, it.sig_len, r32, s32, &st);
      if (st == FTS_OK && !it.pk64) st = FTS_E_SIG_INVALID;
      hst[i] = st;
      uint32_t* R = hrec + i * REC_WORDS;
      for (int k = 0; k < 8; k++) {
        auto be = [&](const uint8_t* b) {
          return ((uint32_t)b[28 - 4 * k] << 24) | ((uint32_t)b[29 - 4 * k] << 16) | ((uint32_t)b[30 - 4 * k] << 8) |
                 (uint32_t)b[31 - 4 * k];
        };
        R[k] = be(r32);
        R[8 + k] = be(s32);
        R[16 + k] = st == FTS_OK ? be(it.pk64) : 0;
        R[24 + k] = st == FTS_OK ? be(it.pk64 + 32) : 0;
      }
      hlen[i] = (uint32_t)it.msg_len;
      if (it.msg_len) memcpy(hm + hoff[i], it.msg, it.msg_len);
    }
  };
  const size_t CH = 2048, nch = (n + CH - 1) / CH;
  fts::host_parallel_for(nch, [&](size_t c) { pack(c * CH, std::min(n, (c + 1) * CH)); });
  if (D.rec_cap < tot) {
    if (D.d_rec) hipFree(D.d_rec);
    D.d_rec = nullptr, D.rec_cap = 0;
    const size_t cap = tot + tot / 2;
    if (hipMalloc(&D.d_rec, cap) != hipSuccess) return D.d_rec = nullptr, FTS_API_ENOMEM;
    D.rec_cap = cap;
  }
  if (D.msg_cap < std::max<size_t>(mtot, 1)) {
    if (D.d_msg) hipFree(D.d_msg);
    D.d_msg = nullptr, D.msg_cap = 0;
    const size_t cap = mtot + mtot / 2 + 1;
    if (hipMalloc(&D.d_msg, cap) != hipSuccess) return D.d_msg = nullptr, FTS_API_ENOMEM;
    D.msg_cap = cap;
  }
  uint32_t* drec = reinterpret_cast<uint32_t*>(D.d_rec);
  uint32_t* de = reinterpret_cast<uint32_t*>(D.d_rec + rec_b);
  uint64_t* doff = reinterpret_cast<uint64_t*>(D.d_rec + rec_b + e_b);
  uint32_t* dlen = reinterpret_cast<uint32_t*>(D.d_rec + rec_b + e_b + off_b);
  int32_t* dst = reinterpret_cast<int32_t*>(D.d_rec + rec_b + e_b + off_b + len_b);
  ECHK(hipMemcpyAsync(D.d_rec, h, tot, hipMemcpyHostToDevice, D.stream));
  if (mtot) ECHK(hipMemcpyAsync(D.d_msg, hm, mtot, hipMemcpyHostToDevice, D.stream));
  const int nb = (int)((n + 255) / 256);
  ECHK(hipEventRecord(D.ev[0], D.stream));
  k_ecdsa_digest<<<nb, 256, 0, D.stream>>>((int)n, D.d_msg, doff, dlen, dst, de);
  ECHK(hipGetLastError());
  ECHK(hipEventRecord(D.ev[1], D.stream));
  k_ecdsa_verify<<<nb, 256, 0, D.stream>>>((int)n, drec, de, D.d_table, dst);
  ECHK(hipGetLastError());
  ECHK(hipEventRecord(D.ev[2], D.stream));
  ECHK(hipMemcpyAsync(hst, dst, st_b, hipMemcpyDeviceToHost, D.stream));
  ECHK(hipStreamSynchronize(D.stream));
  memcpy(status, hst, st_b);
  ECHK(hipEventElapsedTime(&D.ms[0], D.ev[0], D.ev[1]));
  ECHK(hipEventElapsedTime(&D.ms[1], D.ev[1], D.ev[2]));
  return FTS_API_OK;
}

int fts_ecdsa_last_timings(int device, float* ms2) {
  if (device < 0 || device >= 16 || !ms2) return FTS_API_EINVAL;
  std::lock_guard<std::mutex> l(g_dev[device].mu);
  ms2[0] = g_dev[device].ms[0];
  ms2[1] = g_dev[device].ms[1];
  return FTS_API_OK;
}

}  // extern "C"
