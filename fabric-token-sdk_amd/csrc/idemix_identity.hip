// Idemix identity validity on the device (idemix half):
// the association proof every idemix owner identity carries, checked for EVERY
// transfer input by the reference with no cache:
//   validator/validator_transfer.go:46 GetOwnerVerifier(tok.Owner)
//   -> core/common/deserializer.go:63-64 DeserializeVerifier
//   -> services/identity/idemix/deserializer.go:83 Deserialize(raw, true)
//   -> services/identity/idemix/crypto/deserializer.go:36-86 (proto, nym import)
//   -> crypto/id.go:74-108 verifyProof -> IBM/idemix Signature.Ver
//      (ExpectEidNymRhNym, four hidden attributes, rhIndex 3, eidIndex 2, no message).
// Restated in oracle/idemix_identity.py (pairing pinned by the reference's
// credential fixtures; the proof's transcript layout is unpinned).
//
// One identity per lane, two kernels per curve:
//   k_idv_tvals    decode the 7 points (nym key, A', ABar, B', Nym, EidNym, RhNym)
//                  and the epoch key, the error precedence, then the five
//                  t-values (6 variable-base GLV products over affine lane
//                  tables + 11 fixed-base products from the issuer's tables),
//                  one batch normalisation, the Fiat-Shamir transcript in lane
//                  scratch ([byte][lane]: coalesced byte stores), SHA-256 and
//                  c == HashToZr(c' || Nonce)
//   k_idv_pairing  e(W, A') * e(g2, -ABar) == 1 (device/pairing.hpp: precomputed
//                  lines of W and g2, multi-Miller loop, final exponentiation)
// Curves: BN254 (gnark; G1 64-byte raw encodings, 16-bit signed fixed-base
// tables) and FP256BN (AMCL; 0x04 || X || Y, 16-bit unsigned tables), behind a
// traits struct each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/fts_gpu.h"
#include "common/chacha20.hpp"
#include "common/sha256.hpp"
#include "device/fixed_base.hpp"
#include "device/glv.hpp"
#include "device/helpers.hpp"
#include "device/transcript.hpp"
#include "device/fp256bn.hpp"
#include "device/pairing.hpp"
#include "host/bn254_host.hpp"
#include "host/pb.hpp"

namespace fts {
void launch_build_tables(const uint32_t* bases, int nb, uint32_t* tables, uint32_t* scratch, hipStream_t s);
size_t table_build_scratch_bytes(int nb);
size_t fb_words_per_base();
void fbn_build_tables(const uint32_t* plain, int nb, uint32_t* mont, int32_t* ok, uint32_t* tables, hipStream_t s);
size_t fbn_words_per_base();
void host_parallel_for(size_t n, const std::function<void(size_t)>& f);
}  // namespace fts

namespace idv {

using namespace fts;

// ------------------------------------------------------------- constants
// bases of the issuer tables: HSk, HRand, HAttrs[0..3], g1
constexpr int NB = 7, B_HSK = 0, B_HRAND = 1, B_HA = 2, B_G1 = 6;
constexpr int NPT = 7;   // raw points per item: nymPK, A', ABar, B', Nym, EidNym, RhNym
constexpr int P_NYMPK = 0, P_AP = 1, P_ABAR = 2, P_BP = 3, P_NYM = 4, P_EID = 5, P_RH = 6;
constexpr int NVAR = 6;  // variable-base products: A' sE, D (-c), B' sR3, Nym (-c), EidNym (-c), RhNym (-c)
constexpr int NFIX = 11;  // distinct fixed-base products (three serve two t-values each)
constexpr int NSC = NVAR + NFIX;
// record words: flags, c (raw LE limbs, compared), nonce (BE words, hashed), scalars
constexpr int R_FLAGS = 0, R_C = 1, R_NONCE = 9, R_SC = 17;
constexpr int REC_WORDS = R_SC + NSC * 8;  // 153
constexpr int REC_STRIDE = 156;            // 16-byte aligned records
static_assert(REC_STRIDE >= REC_WORDS && REC_STRIDE % 4 == 0, "record stride");
// flags (host parse), in the reference's order of checks
constexpr uint32_t F_EARLY_MALFORMED = 1u, F_NO_EID = 2u, F_NO_RH = 4u, F_LATE_MALFORMED = 8u, F_REVOCATION = 16u,
                   F_C_BIG = 32u;
// targets: t1..t5 = 0..4
__device__ constexpr int VAR_PT[NVAR] = {P_AP, -1, P_BP, P_NYM, P_EID, P_RH};  // -1: D = ABar - B'
__device__ constexpr int VAR_T[NVAR] = {0, 0, 1, 2, 3, 4};
// Fixed-base products and the t-value(s) each is added to: sSk HSk, sA2 HAttrs[2] and
// sA3 HAttrs[3] appear in t2 and again in t3 / t4 / t5 with the same scalar (the
// reference's t3 = HSk^sSk HRand^sRNym ..., t4 = HAttrs[eid]^sEid ..., t5 =
// HAttrs[rh]^sRh ...; IBM/idemix signature.go Ver), so each is computed once and
// added twice (FIX_T2; round 6: 14 -> 11 table gathers of 16 rows per identity)
__device__ constexpr int FIX_B[NFIX] = {B_HRAND, B_HRAND, B_HSK, B_HA + 0, B_HA + 1, B_HA + 2, B_HA + 3,
                                         B_G1,    B_HRAND, B_HRAND, B_HRAND};
__device__ constexpr int FIX_T[NFIX] = {0, 1, 1, 1, 1, 1, 1, 1, 2, 3, 4};
__device__ constexpr int FIX_T2[NFIX] = {-1, -1, 2, -1, -1, 3, 4, -1, -1, -1, -1};
// transcript: label || t1 t2 t3 A' ABar B' Nym EidNym t4 RhNym t5 || ipk.Hash || Disclosure (4 zero bytes)
constexpr char LABEL[] = "signWithEidNymRhNym";
constexpr int LABEL_LEN = 19;
constexpr int MSG_MAX = 832;  // 13 SHA-256 blocks (FP256BN: 19 + 11 * 65 + 36 = 770 bytes)

// ----------------------------------------------------------- curve traits
// BN254 (gnark-crypto through mathlib): G1.Bytes() = 64-byte raw X || Y, 64 zero
// bytes = identity; fixed-base tables of fixed_base.hpp (signed 16-bit windows)
struct BnCurve {
  using B = pair::BnField;
  using F = Fp;
  using PJ = G1J;
  static constexpr int G1_BYTES = 64;
  static FTS_DEV PJ inf() { return g1j_identity(); }
  static FTS_DEV bool is_inf(const PJ& p) { return f_is_zero(p.z); }
  static FTS_DEV PJ dbl(const PJ& p) { return g1j_dbl(p); }
  static FTS_DEV void add_to(PJ& acc, const PJ& q) { add_inl(acc, q); }
  static FTS_DEV void madd_to(PJ& acc, const F& x, const F& y) {
    G1A q;
    q.x = x, q.y = y;
    madd_inl(acc, q);
  }
  static FTS_DEV PJ from_affine(const F& x, const F& y) {
    PJ r;
    r.x = x, r.y = y, r.z = f_one<FpP>();
    return r;
  }
  // raw BE X || Y -> affine Montgomery; NewG1FromBytes rules (canonical, on the curve; zeros = identity)
  static FTS_DEV bool decode(const uint8_t* raw, F& x, F& y, bool& ident) {
    G1A a;
    const bool ok = decode_point(raw, a);
    ident = ok && g1a_is_identity(a);
    x = a.x, y = a.y;
    return ok;
  }
  // affine Montgomery (identity: zeros) -> G1.Bytes()
  template <class Sink>
  static FTS_DEV void encode(Sink& s, const F& x, const F& y) {
    uint32_t pw[16];
    g1_mont_to_be_words(x, y, pw);
    for (int k = 0; k < 16; k++) s.put_word(pw[k]);
  }
  static FTS_DEV void fixed_mul_acc(PJ& acc, const uint32_t* tables, int base, const uint32_t* k) {
    Scalar s;
#pragma unroll
    for (int q = 0; q < 8; q++) s.v[q] = k[q];
    fb_mul_acc(acc, tables + (size_t)base * FB_WORDS_PER_BASE, s);
  }
  static FTS_DEV void decompose(const uint32_t k[8], uint32_t k1[4], uint32_t& s1, uint32_t k2[4], uint32_t& s2) {
    glv_decompose<Glv>(k, k1, s1, k2, s2);
  }
  static FTS_DEV F beta() { return glv_beta(); }
  // HashToZr of a digest -> canonical LE limbs
  static FTS_DEV void digest_mod_r(const uint32_t st[8], uint32_t out[8]) {
    const Fr r = digest_to_fr(st);
#pragma unroll
    for (int q = 0; q < 8; q++) out[q] = r.v[q];
  }
};

// FP256BN (AMCL through mathlib): G1.Bytes() = 0x04 || X || Y; decoded points
// must be canonical and on the curve (no identity encoding); fixed-base tables
// of idemix_kernels.hip (unsigned 16-bit windows, 2^16 entries)
constexpr int FBN_NW = 16, FBN_ND = 1 << 16;
struct FbnCurve {
  using B = pair::FbnField;
  using F = fbn::Fp;
  using PJ = fbn::PJ;
  static constexpr int G1_BYTES = 65;
  static FTS_DEV PJ inf() { return fbn::pj_inf(); }
  static FTS_DEV bool is_inf(const PJ& p) { return fbn::is_zero(p.z); }
  static FTS_DEV PJ dbl(const PJ& p) { return fbn::pj_dbl(p); }
  static FTS_DEV void add_to(PJ& acc, const PJ& q) { acc = fbn::pj_add(acc, q); }
  static FTS_DEV void madd_to(PJ& acc, const F& x, const F& y) { acc = fbn::pj_madd(acc, x, y); }
  static FTS_DEV PJ from_affine(const F& x, const F& y) {
    PJ r;
    r.x = x, r.y = y, r.z = fbn::load<fbn::PM>(fbn::PM::ONE);
    return r;
  }
  static FTS_DEV bool decode(const uint8_t* raw, F& x, F& y, bool& ident) {
    uint32_t pw[16];
    load_be_words(raw, pw);
    uint32_t nx[8], ny[8];
#pragma unroll
    for (int k = 0; k < 8; k++) nx[k] = pw[7 - k], ny[k] = pw[15 - k];
    ident = false;
    if (!p256::lt256(nx, fbn::PM::M) || !p256::lt256(ny, fbn::PM::M)) return false;
    x = p256::to_mont(fbn::load<fbn::PM>(nx));
    y = p256::to_mont(fbn::load<fbn::PM>(ny));
    return fbn::on_curve(x, y);
  }
  template <class Sink>
  // AMCL ECP.ToBytes(b, false): the point at infinity (held here as (0, 0)) is
  // AMCL's projective (0, 1, 0), which Affine() leaves as is -> 0x04 || 0 || 1
  static FTS_DEV void encode(Sink& s, const F& x, const F& y) {
    s.put_byte(0x04);
    const F ax = p256::from_mont(x);
    F ay = p256::from_mont(y);
    if (fbn::is_zero(ax) && fbn::is_zero(ay)) ay.v[0] = 1u;
    for (int k = 7; k >= 0; k--) s.put_word(ax.v[k]);
    for (int k = 7; k >= 0; k--) s.put_word(ay.v[k]);
  }
  static FTS_DEV void fixed_mul_acc(PJ& acc, const uint32_t* tables, int base, const uint32_t* k) {
    const uint32_t* tb = tables + (size_t)base * FBN_NW * FBN_ND * 16;
    for (int w = 0; w < FBN_NW; w++) {
      const uint32_t d = (k[w >> 1] >> (16 * (w & 1))) & 0xffffu;
      if (d) {
        const uint32_t* t = tb + ((size_t)w * FBN_ND + d) * 16;
        acc = fbn::pj_madd(acc, fbn::load<fbn::PM>(t), fbn::load<fbn::PM>(t + 8));
      }
    }
  }
  static FTS_DEV void decompose(const uint32_t k[8], uint32_t k1[4], uint32_t& s1, uint32_t k2[4], uint32_t& s2) {
    glv_decompose<fbn::GlvK>(k, k1, s1, k2, s2);
  }
  static FTS_DEV F beta() { return fbn::load<fbn::PM>(fbn::GlvK::BETA); }
  static FTS_DEV void digest_mod_r(const uint32_t st[8], uint32_t out[8]) {
    uint32_t t[8], bw = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = st[7 - i];
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = subb(out[i], fbn::RM::M[i], bw, bw);
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = bw ? out[i] : t[i];
  }
};

// ------------------------------------------------------------ lane scratch
// [unit][lane] layouts: neighbouring lanes touch neighbouring addresses
struct LaneWords {
  uint32_t* base;
  size_t L, lane;
  FTS_DEV uint32_t& at(size_t w) const { return base[w * L + lane]; }
};
// transcript bytes, [byte][lane]
struct ByteSink {
  uint8_t* base;
  size_t L, lane;
  uint32_t off = 0;
  FTS_DEV void put_byte(uint32_t b) { base[(size_t)(off++) * L + lane] = (uint8_t)b; }
  FTS_DEV void put_word(uint32_t w) {  // big-endian
    put_byte(w >> 24), put_byte(w >> 16), put_byte(w >> 8), put_byte(w);
  }
  FTS_DEV uint32_t word(uint32_t j) const {
    const uint8_t* p = base + (size_t)(4 * j) * L + lane;
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[L] << 16) | ((uint32_t)p[2 * L] << 8) | p[3 * L];
  }
};

// affine lane table of 1..8 * P: XY rows [8][L][16] | Z, PRE [16][8][L] words (GTab)
constexpr int AT_WORDS = 8 * 16 + 8 * 8 + 8 * 8;
template <class CV>
FTS_DEV void put_f(const LaneWords& T, size_t w0, const typename CV::F& a) {
#pragma unroll
  for (int q = 0; q < 8; q++) T.at(w0 + q) = a.v[q];
}
template <class CV>
FTS_DEV typename CV::F get_f(const LaneWords& T, size_t w0) {
  typename CV::F a;
#pragma unroll
  for (int q = 0; q < 8; q++) a.v[q] = T.at(w0 + q);
  return a;
}

// Lane table of 1..8 * P for the GLV chains (round 6 layout): the affine entries as
// 64-byte rows, entry-major ([8][L][16] words: a window lookup reads ONE row per lane,
// four 16-byte loads, where the [word][lane] layout touched up to sixteen 128-byte
// lines per word and wave), then the build's z's and running products [16][8][L].
struct GTab {
  uint32_t* base;
  size_t L, lane;
  FTS_DEV uint32_t* row(int e) const { return base + ((size_t)e * L + lane) * 16; }
  FTS_DEV LaneWords zw() const { return LaneWords{base + (size_t)8 * 16 * L, L, lane}; }
};
template <class CV>
FTS_DEV void row_put(uint32_t* p, const typename CV::F& x, const typename CV::F& y) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
  q[2] = make_uint4(y.v[0], y.v[1], y.v[2], y.v[3]);
  q[3] = make_uint4(y.v[4], y.v[5], y.v[6], y.v[7]);
}
template <class CV>
FTS_DEV void row_get(const uint32_t* p, typename CV::F& x, typename CV::F& y) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  x.v[0] = a.x, x.v[1] = a.y, x.v[2] = a.z, x.v[3] = a.w, x.v[4] = b.x, x.v[5] = b.y, x.v[6] = b.z, x.v[7] = b.w;
  y.v[0] = c.x, y.v[1] = c.y, y.v[2] = c.z, y.v[3] = c.w, y.v[4] = d.x, y.v[5] = d.y, y.v[6] = d.z, y.v[7] = d.w;
}

// 1..8 * P (P Jacobian, not the identity) into the lane table T, normalised to
// affine with one inversion (Montgomery's trick over the eight z's)
template <class CV>
FTS_DEV void glv_table(const typename CV::PJ& P, const GTab& T) {
  using B = typename CV::B;
  using F = typename CV::F;
  using PJ = typename CV::PJ;
  const LaneWords Z = T.zw();
  PJ cur = P;
  F pre = P.z;
  for (int e = 0; e < 8; e++) {
    if (e == 1) cur = CV::dbl(P);
    if (e > 1) CV::add_to(cur, P);
    row_put<CV>(T.row(e), cur.x, cur.y);
    put_f<CV>(Z, e * 8, cur.z);
    if (e) pre = B::mul(pre, cur.z);
    put_f<CV>(Z, 64 + e * 8, pre);
  }
  F inv = B::inv(pre);
  for (int e = 7; e >= 0; e--) {
    F zi = inv;
    if (e > 0) {
      zi = B::mul(inv, get_f<CV>(Z, 64 + (e - 1) * 8));
      inv = B::mul(inv, get_f<CV>(Z, e * 8));
    }
    const F zi2 = B::mul(zi, zi);
    F x, y;
    row_get<CV>(T.row(e), x, y);
    row_put<CV>(T.row(e), B::mul(x, zi2), B::mul(B::mul(y, zi2), zi));
  }
}

// (-1)^s1 k1 * P + (-1)^s2 k2 * phi(P) over the table of glv_table: NW signed 4-bit
// windows from the top (magnitudes below 2^(4 NW - 1)), 4 (NW - 1) doublings,
// <= 2 NW mixed additions
template <class CV, int NW>
FTS_DEV typename CV::PJ glv_chain(const GTab& T, const uint32_t k1[4], uint32_t s1, const uint32_t k2[4],
                                  uint32_t s2) {
  using B = typename CV::B;
  using F = typename CV::F;
  using PJ = typename CV::PJ;
  const uint32_t c1 = recode_carries(k1), c2 = recode_carries(k2);
  const F beta = CV::beta();
  PJ acc = CV::inf();
  for (int w = NW - 1; w >= 0; w--) {
    const int d1 = window_digit(k1, c1, w), d2 = window_digit(k2, c2, w);
    F x1, y1, x2, y2;
    if (d1) row_get<CV>(T.row((d1 < 0 ? -d1 : d1) - 1), x1, y1);
    if (d2) row_get<CV>(T.row((d2 < 0 ? -d2 : d2) - 1), x2, y2);
    if (w != NW - 1)
      for (int r = 0; r < 4; r++) acc = CV::dbl(acc);
    if (d1) {
      if ((d1 < 0) != (s1 != 0)) y1 = B::neg(y1);
      CV::madd_to(acc, x1, y1);
    }
    if (d2) {
      if ((d2 < 0) != (s2 != 0)) y2 = B::neg(y2);
      CV::madd_to(acc, B::mul(x2, beta), y2);
    }
  }
  return acc;
}

// k * P (k canonical mod r, P Jacobian) by GLV: k = k1 + k2 lambda; one table of
// 1..8 * P, normalised with one inversion; phi(mP) = (beta x, y) read from the
// same entries; 32 signed 4-bit windows, 124 doublings, <= 64 mixed additions
template <class CV>
FTS_DEV typename CV::PJ glv_mul(const typename CV::PJ& P, const uint32_t k[8], const GTab& T) {
  uint32_t nz = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) nz |= k[q];
  if (CV::is_inf(P) || !nz) return CV::inf();
  glv_table<CV>(P, T);
  uint32_t k1[4], k2[4], s1, s2;
  CV::decompose(k, k1, s1, k2, s2);
  return glv_chain<CV, 32>(T, k1, s1, k2, s2);
}

// G2 point (affine Montgomery Fp2) on the twist y^2 = x^3 + b'
template <class B>
FTS_DEV bool g2_on_twist(const pair::F2<B>& x, const pair::F2<B>& y) {
  const pair::F2<B> rhs = pair::add(pair::mul(pair::sqr(x), x), pair::f2_ld<B>(B::K::TWB[0]));
  return pair::eq(pair::sqr(y), rhs);
}
// 128 raw bytes (four 32-byte big-endian coordinates in the curve's ECP2 order) ->
// affine Montgomery; false if a coordinate is >= p or the point is off the twist.
// BN254 (gnark raw): X.A1 X.A0 Y.A1 Y.A0; FP256BN (AMCL): xa xb ya yb
template <class CV>
FTS_DEV bool decode_g2(const uint8_t* raw, pair::F2<typename CV::B>& x, pair::F2<typename CV::B>& y);
template <>
FTS_DEV bool decode_g2<BnCurve>(const uint8_t* raw, pair::F2<pair::BnField>& x, pair::F2<pair::BnField>& y) {
  uint32_t pw[16], qw[16];
  load_be_words(raw, pw);
  load_be_words(raw + 64, qw);
  Fp c[4];
#pragma unroll
  for (int k = 0; k < 8; k++) c[0].v[k] = pw[7 - k], c[1].v[k] = pw[15 - k], c[2].v[k] = qw[7 - k], c[3].v[k] = qw[15 - k];
  bool ok = true, zero = true;
  for (int q = 0; q < 4; q++) ok = ok && limbs_lt_mod<FpP>(c[q].v), zero = zero && f_is_zero(c[q]);
  if (!ok) return false;
  if (zero) return true;  // the identity's raw encoding
  x.b = f_to_mont(c[0]), x.a = f_to_mont(c[1]), y.b = f_to_mont(c[2]), y.a = f_to_mont(c[3]);
  return g2_on_twist<pair::BnField>(x, y);
}
template <>
FTS_DEV bool decode_g2<FbnCurve>(const uint8_t* raw, pair::F2<pair::FbnField>& x, pair::F2<pair::FbnField>& y) {
  uint32_t pw[16], qw[16];
  load_be_words(raw, pw);
  load_be_words(raw + 64, qw);
  uint32_t c[4][8];
#pragma unroll
  for (int k = 0; k < 8; k++) c[0][k] = pw[7 - k], c[1][k] = pw[15 - k], c[2][k] = qw[7 - k], c[3][k] = qw[15 - k];
  uint32_t any = 0;
  for (int q = 0; q < 4; q++) {
    if (!p256::lt256(c[q], fbn::PM::M)) return false;
    for (int k = 0; k < 8; k++) any |= c[q][k];
  }
  if (!any) return true;  // all zero: the identity (as the oracle's decoding)
  x.a = p256::to_mont(fbn::load<fbn::PM>(c[0])), x.b = p256::to_mont(fbn::load<fbn::PM>(c[1]));
  y.a = p256::to_mont(fbn::load<fbn::PM>(c[2])), y.b = p256::to_mont(fbn::load<fbn::PM>(c[3]));
  return g2_on_twist<pair::FbnField>(x, y);
}

// ---------------------------------------------------- BN254 G2 subgroup check
// gnark-crypto's G2Affine.SetBytes (under mathlib's NewG2FromBytes) rejects twist
// points outside the order-r subgroup; the twist's cofactor is not 1, so decode_g2's
// on-twist check alone fails open.  [r - 1] Q == -Q  <=>  [r] Q == O, by
// double-and-add over Jacobian Fp2 coordinates with complete handling of the
// exceptional additions (points of small order hit them).
template <class B>
struct G2J {
  pair::F2<B> x, y, z;
};
template <class B>
FTS_DEV void g2j_dbl(G2J<B>& p) {  // dbl-2009-l (a = 0); the identity (z = 0) stays the identity
  using namespace pair;
  const F2<B> A = sqr(p.x), Bq = sqr(p.y), C = sqr(Bq);
  const F2<B> D = dbl(sub(sub(sqr(add(p.x, Bq)), A), C));
  const F2<B> E = add(dbl(A), A);
  const F2<B> X3 = sub(sqr(E), dbl(D));
  const F2<B> Y3 = sub(mul(E, sub(D, X3)), dbl(dbl(dbl(C))));
  p.z = dbl(mul(p.y, p.z));
  p.x = X3;
  p.y = Y3;
}
template <class B>
FTS_DEV void g2j_madd(G2J<B>& p, const pair::F2<B>& qx, const pair::F2<B>& qy) {  // madd-2007-bl, complete
  using namespace pair;
  if (is_zero(p.z)) {
    p.x = qx, p.y = qy, p.z = f2_one<B>();
    return;
  }
  const F2<B> Z1Z1 = sqr(p.z);
  const F2<B> U2 = mul(qx, Z1Z1), S2 = mul(mul(qy, p.z), Z1Z1);
  const F2<B> H = sub(U2, p.x), r = sub(S2, p.y);
  if (is_zero(H)) {
    if (is_zero(r)) g2j_dbl(p);  // p == q
    else p.z = f2_zero<B>();     // p == -q
    return;
  }
  const F2<B> HH = sqr(H), I = dbl(dbl(HH)), J = mul(H, I), rr = dbl(r), V = mul(p.x, I);
  const F2<B> X3 = sub(sub(sqr(rr), J), dbl(V));
  const F2<B> Y3 = sub(mul(rr, sub(V, X3)), dbl(mul(p.y, J)));
  p.z = sub(sub(sqr(add(p.z, H)), Z1Z1), HH);
  p.x = X3;
  p.y = Y3;
}
// (qx, qy) affine Montgomery on the twist, not the identity
FTS_DEV bool g2_in_subgroup_bn(const pair::F2<pair::BnField>& qx, const pair::F2<pair::BnField>& qy) {
  using namespace pair;
  using B = BnField;
  // r - 1 of BN254 (254 bits, little-endian words)
  constexpr uint32_t RM1[8] = {0xf0000000u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  G2J<B> acc{f2_zero<B>(), f2_one<B>(), f2_zero<B>()};
#pragma unroll 1
  for (int bit = 253; bit >= 0; bit--) {
    g2j_dbl(acc);
    if ((RM1[bit >> 5] >> (bit & 31)) & 1u) g2j_madd(acc, qx, qy);
  }
  if (is_zero(acc.z)) return false;
  const F2<B> z2 = sqr(acc.z), z3 = mul(z2, acc.z);
  return eq(acc.x, mul(qx, z2)) && eq(acc.y, neg(mul(qy, z3)));
}

#ifndef IDV_FBN_TU  // BN254 only: compiled in the main translation unit
// U distinct epoch keys (128 raw bytes each, BN254): ok[u] <- the key decodes (on the
// twist, canonical) and lies in the subgroup (the identity does)
// lane j checks distinct key idx[j] (the keys the context has not checked before)
__global__ void __launch_bounds__(64) k_idv_g2_check(int M, const int32_t* __restrict__ idx,
                                                     const uint8_t* __restrict__ keys, int32_t* __restrict__ ok) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= M) return;
  const int u = idx[j];
  pair::F2<pair::BnField> x, y;
  const uint8_t* kr = keys + (size_t)u * 128;
  bool good = decode_g2<BnCurve>(kr, x, y);
  bool zero = true;
  for (int q = 0; q < 128; q++) zero = zero && kr[q] == 0;
  if (good && !zero) good = g2_in_subgroup_bn(x, y);
  ok[u] = good ? 1 : 0;
}
#endif

// ----------------------------------------------------------------- kernels
// lines of W (lane 0) and g2 (lane 1); wraw: W as 128 raw bytes; ok[0] <- W valid
template <class CV>
__global__ void __launch_bounds__(64) k_idv_lines(const uint8_t* __restrict__ wraw, uint32_t* __restrict__ lines,
                                                  int32_t* __restrict__ ok) {
  using B = typename CV::B;
  using K = typename B::K;
  const int t = threadIdx.x;
  if (t > 1) return;
  pair::F2<B> qx, qy;
  if (t == 0) {
    if (!decode_g2<CV>(wraw, qx, qy) || (pair::is_zero(qx) && pair::is_zero(qy))) {
      ok[0] = 0;
      return;
    }
    if constexpr (std::is_same<CV, BnCurve>::value) {  // gnark SetBytes: subgroup check
      if (!g2_in_subgroup_bn(qx, qy)) {
        ok[0] = 0;
        return;
      }
    }
    ok[0] = 1;
  } else {
    qx = pair::f2_ld<B>(K::GEN2[0]);
    qy = pair::f2_ld<B>(K::GEN2[1]);
  }
  pair::precompute_lines<B>(qx, qy, lines + (size_t)t * pair::n_lines<K>() * pair::LINE_WORDS);
}

// Lane scratch ([word][lane], n lanes each): S = t1..t5 accumulators (5 x 24),
// DP = decoded points (NPT x 16), IDM = identity mask of the decoded points (1),
// VR = the NVAR variable-base then NFIX fixed-base products (NSC x 24), TV = the
// variable-base products' GLV lane tables
// (NVAR x AT_WORDS; TV[0] doubles as the normalisation's prefix products)
FTS_DEV size_t sc_s(size_t) { return 0; }
FTS_DEV size_t sc_dp(size_t n) { return (size_t)5 * 24 * n; }
FTS_DEV size_t sc_idm(size_t n) { return sc_dp(n) + (size_t)NPT * 16 * n; }
FTS_DEV size_t sc_vr(size_t n) { return sc_idm(n) + ((n + 3) & ~size_t(3)); }  // keeps sc_tv 16-byte aligned (GTab rows)
FTS_DEV size_t sc_tv(size_t n) { return sc_vr(n) + (size_t)NSC * 24 * n; }
inline size_t idv_scratch_words(size_t n) { return (5 * 24 + NPT * 16 + 1 + NSC * 24 + NVAR * AT_WORDS) * n + 3; }

// Three kernels per batch (round 4; one lane per identity for everything left
// 1,024 waves at one per SIMD, 30 % of the MAD peak):
//   k_idv_decode  identity per lane: status (pre-set by the host for identity-
//                 level errors), point decoding in the reference's order of
//                 checks, pin[i] <- (A', -ABar) for the pairing kernel
//   k_idv_var     lane per (product, identity): the six GLV products and the
//                 eleven fixed-base products of the t-values, 17x the lanes
//   k_idv_tvals   identity per lane: sum the products into t1..t5,
//                 normalisation, transcript, challenge;
//                 zk[i] <- 1 if c == c''
template <class CV>
__global__ void __launch_bounds__(256) k_idv_decode(int n, const uint32_t* __restrict__ rec,
                                                    const uint8_t* __restrict__ pts, const uint8_t* __restrict__ epk,
                                                    uint32_t* __restrict__ scratch, uint32_t* __restrict__ pin,
                                                    int32_t* __restrict__ zk, int32_t* __restrict__ status,
                                                    const int32_t* __restrict__ eidx, const int32_t* __restrict__ g2ok) {
  using B = typename CV::B;
  using F = typename CV::F;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  zk[i] = 0;
  if (status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * REC_STRIDE;
  const uint8_t* P = pts + (size_t)i * NPT * 64;
  const uint32_t flags = R[R_FLAGS];
  const LaneWords DP{scratch + sc_dp(n), (size_t)n, (size_t)i};
  uint32_t okm = 0, idm = 0;
#pragma unroll 1
  for (int q = 0; q < NPT; q++) {
    F px, py;
    bool id;
    if (CV::decode(P + q * 64, px, py, id)) okm |= 1u << q;
    if (id) idm |= 1u << q;
    put_f<CV>(DP, q * 16, px);
    put_f<CV>(DP, q * 16 + 8, py);
  }
  scratch[sc_idm(n) + i] = idm;
  // NymPublicKey import (crypto/deserializer.go:49-56) precedes the proof
  if (!(okm & (1u << P_NYMPK))) {
    status[i] = FTS_E_ID_BADNYM;
    return;
  }
  if (flags & F_EARLY_MALFORMED) {
    status[i] = FTS_E_ID_MALFORMED;
    return;
  }
  if (flags & F_NO_EID) {
    status[i] = FTS_E_ID_NO_EIDNYM;
    return;
  }
  if (flags & F_NO_RH) {
    status[i] = FTS_E_ID_NO_RHNYM;
    return;
  }
  bool all = okm == (1u << NPT) - 1;
  {
    pair::F2<B> ex, ey;
    all = all && decode_g2<CV>(epk + (size_t)i * 128, ex, ey);
    // BN254: the key's subgroup check, once per distinct key (k_idv_g2_check)
    if (g2ok) all = all && g2ok[eidx[i]] != 0;
  }
  if (!all || (flags & F_LATE_MALFORMED)) {
    status[i] = FTS_E_ID_MALFORMED;
    return;
  }
  if (flags & F_REVOCATION) {
    status[i] = FTS_E_ID_REVOCATION;
    return;
  }
  if (idm & (1u << P_AP)) {
    status[i] = FTS_E_ID_APRIME;
    return;
  }
  // pairing inputs: A' and -ABar
  uint32_t* pq = pin + (size_t)i * 32;
  const F ax = get_f<CV>(DP, P_AP * 16), ay = get_f<CV>(DP, P_AP * 16 + 8);
  const F bx = get_f<CV>(DP, P_ABAR * 16), by = get_f<CV>(DP, P_ABAR * 16 + 8);
  const F nby = (idm & (1u << P_ABAR)) ? by : B::neg(by);
#pragma unroll
  for (int q = 0; q < 8; q++) pq[q] = ax.v[q], pq[8 + q] = ay.v[q], pq[16 + q] = bx.v[q], pq[24 + q] = nby.v[q];
}

// lane g = v * n + i: identities fastest, so a wave runs one product kind
template <class CV>
__global__ void __launch_bounds__(256) k_idv_var(int n, const uint32_t* __restrict__ rec,
                                                 const uint32_t* __restrict__ tables,
                                                 uint32_t* __restrict__ scratch, const int32_t* __restrict__ status) {
  using B = typename CV::B;
  using PJ = typename CV::PJ;
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)NSC * n) return;
  const int v = (int)(g / n), i = (int)(g % n);
  if (status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * REC_STRIDE;
  const LaneWords VR{scratch + sc_vr(n) + (size_t)v * 24 * n, (size_t)n, (size_t)i};
  if (v >= NVAR) {  // fixed-base product (issuer tables)
    PJ acc = CV::inf();
    CV::fixed_mul_acc(acc, tables, FIX_B[v - NVAR], R + R_SC + v * 8);
    put_f<CV>(VR, 0, acc.x);
    put_f<CV>(VR, 8, acc.y);
    put_f<CV>(VR, 16, acc.z);
    return;
  }
  const LaneWords DP{scratch + sc_dp(n), (size_t)n, (size_t)i};
  const uint32_t idm = scratch[sc_idm(n) + i];
  const int pq_ = VAR_PT[v] < 0 ? P_ABAR : VAR_PT[v];
  PJ base = (idm >> pq_) & 1u ? CV::inf() : CV::from_affine(get_f<CV>(DP, pq_ * 16), get_f<CV>(DP, pq_ * 16 + 8));
  if (VAR_PT[v] < 0 && !((idm >> P_BP) & 1u))  // D = ABar - B'
    CV::madd_to(base, get_f<CV>(DP, P_BP * 16), B::neg(get_f<CV>(DP, P_BP * 16 + 8)));
  const GTab T{scratch + sc_tv(n) + (size_t)v * AT_WORDS * n, (size_t)n, (size_t)i};
  const PJ r = glv_mul<CV>(base, R + R_SC + v * 8, T);
  put_f<CV>(VR, 0, r.x);
  put_f<CV>(VR, 8, r.y);
  put_f<CV>(VR, 16, r.z);
}

template <class CV>
__global__ void __launch_bounds__(256) k_idv_tvals(int n, const uint32_t* __restrict__ rec,
                                                   const uint32_t* __restrict__ tables,
                                                   const uint32_t* __restrict__ ipk_hash,  // 8 BE words
                                                   uint32_t* __restrict__ scratch, uint8_t* __restrict__ msg,
                                                   int32_t* __restrict__ zk, const int32_t* __restrict__ status) {
  using B = typename CV::B;
  using F = typename CV::F;
  using PJ = typename CV::PJ;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != FTS_OK) return;
  const uint32_t* R = rec + (size_t)i * REC_STRIDE;
  const uint32_t flags = R[R_FLAGS];
  const LaneWords DP{scratch + sc_dp(n), (size_t)n, (size_t)i};
  const uint32_t idm = scratch[sc_idm(n) + i];
  // t-values: accumulators t1..t5 in lane scratch ([word][lane]), Jacobian
  const LaneWords S{scratch + sc_s(n), (size_t)n, (size_t)i};
  const LaneWords T{scratch + sc_tv(n), (size_t)n, (size_t)i};
  for (int t = 0; t < 5; t++) {
    const PJ z = CV::inf();
    put_f<CV>(S, t * 24, z.x);
    put_f<CV>(S, t * 24 + 8, z.y);
    put_f<CV>(S, t * 24 + 16, z.z);
  }
#pragma unroll 1
  for (int v = 0; v < NSC; v++) {
    const LaneWords VR{scratch + sc_vr(n) + (size_t)v * 24 * n, (size_t)n, (size_t)i};
    PJ r;
    r.x = get_f<CV>(VR, 0), r.y = get_f<CV>(VR, 8), r.z = get_f<CV>(VR, 16);
    const int t1 = v < NVAR ? VAR_T[v] : FIX_T[v - NVAR], t2 = v < NVAR ? -1 : FIX_T2[v - NVAR];
    for (int t : {t1, t2}) {
      if (t < 0) continue;
      PJ acc;
      acc.x = get_f<CV>(S, t * 24), acc.y = get_f<CV>(S, t * 24 + 8), acc.z = get_f<CV>(S, t * 24 + 16);
      CV::add_to(acc, r);
      put_f<CV>(S, t * 24, acc.x);
      put_f<CV>(S, t * 24 + 8, acc.y);
      put_f<CV>(S, t * 24 + 16, acc.z);
    }
  }
  // the five t-values -> affine with one inversion (Montgomery's trick; identity -> (0, 0))
  {
    F pre = B::one();
    for (int t = 0; t < 5; t++) {
      put_f<CV>(T, t * 8, pre);
      const F z = get_f<CV>(S, t * 24 + 16);
      if (!B::is_zero(z)) pre = B::mul(pre, z);
    }
    F inv = B::inv(pre);
    for (int t = 4; t >= 0; t--) {
      const F z = get_f<CV>(S, t * 24 + 16);
      F ax = B::zero(), ay = B::zero();
      if (!B::is_zero(z)) {
        const F zi = B::mul(inv, get_f<CV>(T, t * 8));
        inv = B::mul(inv, z);
        const F zi2 = B::mul(zi, zi);
        ax = B::mul(get_f<CV>(S, t * 24), zi2);
        ay = B::mul(B::mul(get_f<CV>(S, t * 24 + 8), zi2), zi);
      }
      put_f<CV>(S, t * 24, ax);
      put_f<CV>(S, t * 24 + 8, ay);
    }
  }
  // transcript
  ByteSink M{msg, (size_t)n, (size_t)i};
  for (int k = 0; k < LABEL_LEN; k++) M.put_byte((uint8_t)LABEL[k]);
  // t1 t2 t3 A' ABar B' Nym EidNym t4 RhNym t5: tags >= 0 are t-values, < 0 points (-1 - index)
  constexpr int ORDER[11] = {0, 1, 2, -1 - P_AP, -1 - P_ABAR, -1 - P_BP, -1 - P_NYM, -1 - P_EID, 3, -1 - P_RH, 4};
  for (int q = 0; q < 11; q++) {
    const int tag = ORDER[q];
    if (tag >= 0) {
      CV::encode(M, get_f<CV>(S, tag * 24), get_f<CV>(S, tag * 24 + 8));
    } else {
      const int pi = -1 - tag;
      F zx = get_f<CV>(DP, pi * 16), zy = get_f<CV>(DP, pi * 16 + 8);
      if ((idm >> pi) & 1u) zx = B::zero(), zy = B::zero();
      CV::encode(M, zx, zy);
    }
  }
  for (int k = 0; k < 8; k++) M.put_word(ipk_hash[k]);
  M.put_word(0u);  // Disclosure: four hidden attributes
  const uint32_t len = M.off;
  // SHA-256 padding
  const uint32_t nb = sha_blocks(len);
  M.put_byte(0x80);
  while (M.off < nb * 64 - 8) M.put_byte(0);
  M.put_word(0u);
  M.put_word(len * 8u);
  uint32_t st[8], w[16];
  sha256_init(st);
  for (uint32_t b = 0; b < nb; b++) {
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = M.word(16 * b + k);
    sha256_compress(st, w);
  }
  uint32_t c1[8], c2[8];
  CV::digest_mod_r(st, c1);
  // c'' = HashToZr(Zr.Bytes(c') || Zr.Bytes(Nonce))
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = c1[7 - k];
#pragma unroll
  for (int k = 0; k < 8; k++) w[8 + k] = R[R_NONCE + k];
  sha256_init(st);
  sha256_compress(st, w);
  w[0] = 0x80000000u;
#pragma unroll
  for (int k = 1; k < 15; k++) w[k] = 0u;
  w[15] = 512u;
  sha256_compress(st, w);
  CV::digest_mod_r(st, c2);
  uint32_t diff = (flags & F_C_BIG) ? 1u : 0u;
#pragma unroll
  for (int k = 0; k < 8; k++) diff |= c2[k] ^ R[R_C + k];
  zk[i] = diff ? 0 : 1;
}

// e(W, A') * e(g2, -ABar) == 1, then the verdict (pairing before the ZK proof, as Ver checks)
// waves per SIMD the pairing kernel is compiled for (A/B: -DFTS_IDV_OCC=2 caps it
// at 256 registers, with spills in the inlined Fp12 bodies)
#ifndef FTS_IDV_OCC
#define FTS_IDV_OCC 1
#endif
template <class CV>
__global__ void __launch_bounds__(64, FTS_IDV_OCC) k_idv_pairing(int n, const uint32_t* __restrict__ pin,
                                                    const uint32_t* __restrict__ lines, const int32_t* __restrict__ zk,
                                                    int32_t* __restrict__ status, const int32_t* __restrict__ list,
                                                    const int32_t* __restrict__ count) {
  using B = typename CV::B;
  using K = typename B::K;
  using F = typename B::F;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (list) {  // the identities of the groups whose batch check failed (k_idv_bp_sel)
    if (i >= *count) return;
    i = list[i];
  }
  if (i >= n || status[i] != FTS_OK) return;
  const uint32_t* pq = pin + (size_t)i * 32;
  const uint32_t* const L[2] = {lines, lines + (size_t)pair::n_lines<K>() * pair::LINE_WORDS};
  const F xP[2] = {B::ld(pq), B::ld(pq + 16)};
  const F yP[2] = {B::ld(pq + 8), B::ld(pq + 24)};
  pair::F12<B> f;
  if (B::is_zero(xP[1]) && B::is_zero(yP[1])) {  // ABar = O: e(g2, O) = 1
    const uint32_t* const L1[1] = {L[0]};
    const F x1[1] = {xP[0]}, y1[1] = {yP[0]};
    f = pair::miller<B, 1>(L1, x1, y1);
  } else {
    f = pair::miller<B, 2>(L, xP, yP);
  }
  const bool one = pair::is_one(pair::final_exp_i(f));
  status[i] = !one ? FTS_E_ID_PAIRING : (zk[i] ? FTS_OK : FTS_E_ID_ZK);
}

// ---- batch pairing check (round 6)
// The equations e(W, A'_i) e(g2, -ABar_i) = 1 of a group of BP_G identities are
// checked as ONE: e(W, sum rho_i A'_i) e(g2, sum rho_i (-ABar_i)) = 1, with secret
// weights rho_i = a_i + b_i lambda (a_i, b_i: 64-bit ChaCha20 words under a key drawn
// with getrandom for every call; the GLV lattice {(x, y): x + y lambda = 0 mod r} has
// no nonzero vector shorter than ~2^126, so the 2^128 pairs are 2^128 distinct rho
// mod r).  Pairing values live in the order-r subgroup of GT (r prime), so a group
// holding an identity whose equation fails passes with probability <= 2^-128 (the
// small-exponents batch test of Bellare, Garay and Rabin).  A group that fails has
// its identities paired one by one (k_idv_pairing over the k_idv_bp_sel list), so
// every verdict is the per-identity one.  Work per identity: two 64-bit GLV chains
// (17 windows) instead of a 2-pairing Miller loop and a final exponentiation.
constexpr int BP_G = 256;  // identities per group = threads of a k_idv_bp_terms block
struct Key8 {
  uint32_t k[8];
};
// scratch (the t-value kernels' scratch, free by then):
//   lane tables [2][AT_WORDS][n] | group sums [ng][2][24] | gok [ng] | count | list [n]
inline size_t bp_part_off(size_t n) { return (size_t)2 * AT_WORDS * n; }
inline size_t bp_gok_off(size_t n, size_t ng) { return bp_part_off(n) + ng * 48; }
inline size_t bp_cnt_off(size_t n, size_t ng) { return bp_gok_off(n, ng) + ng; }
inline size_t bp_list_off(size_t n, size_t ng) { return bp_cnt_off(n, ng) + 64; }
inline size_t bp_scratch_words(size_t n) {
  const size_t ng = (n + BP_G - 1) / BP_G;
  return bp_list_off(n, ng) + n;
}

// block = group g, blockIdx.y = which point (0: A', 1: -ABar): rho_i * P_i summed
// over the group's identities still OK (the others contribute O), LDS tree
template <class CV>
__global__ void __launch_bounds__(BP_G) k_idv_bp_terms(int n, const uint32_t* __restrict__ pin,
                                                       const int32_t* __restrict__ status, Key8 key,
                                                       uint32_t* __restrict__ scratch, uint32_t* __restrict__ part) {
  using B = typename CV::B;
  using F = typename CV::F;
  using PJ = typename CV::PJ;
  __shared__ uint32_t sh[24 * BP_G];
  const int t = threadIdx.x, which = blockIdx.y;
  const int i = blockIdx.x * BP_G + t;
  PJ r = CV::inf();
  if (i < n && status[i] == FTS_OK) {
    const uint32_t* pq = pin + (size_t)i * 32 + which * 16;
    const F x = B::ld(pq), y = B::ld(pq + 8);
    if (!(B::is_zero(x) && B::is_zero(y))) {  // -ABar = O: e(g2, O) = 1, no term
      uint32_t blk[16];
      fts::chacha20_block(key.k, (uint32_t)i, blk);
      const uint32_t a[4] = {blk[0], blk[1], 0u, 0u}, b[4] = {blk[2], blk[3], 0u, 0u};
      const GTab T{scratch + (size_t)which * AT_WORDS * n, (size_t)n, (size_t)i};
      glv_table<CV>(CV::from_affine(x, y), T);
      r = glv_chain<CV, 17>(T, a, 0u, b, 0u);
    }
  }
  const LaneWords S{sh, (size_t)BP_G, (size_t)t};
  put_f<CV>(S, 0, r.x);
  put_f<CV>(S, 8, r.y);
  put_f<CV>(S, 16, r.z);
  for (int h = BP_G / 2; h > 0; h >>= 1) {
    __syncthreads();
    if (t < h) {
      const LaneWords O{sh, (size_t)BP_G, (size_t)(t + h)};
      PJ a, b;
      a.x = get_f<CV>(S, 0), a.y = get_f<CV>(S, 8), a.z = get_f<CV>(S, 16);
      b.x = get_f<CV>(O, 0), b.y = get_f<CV>(O, 8), b.z = get_f<CV>(O, 16);
      CV::add_to(a, b);
      put_f<CV>(S, 0, a.x);
      put_f<CV>(S, 8, a.y);
      put_f<CV>(S, 16, a.z);
    }
  }
  __syncthreads();  // lane 0's last sum, read by lanes 0..23
  if (t < 24) part[((size_t)blockIdx.x * 2 + which) * 24 + t] = sh[(size_t)t * BP_G];
}

// lane pair per group (lanes 2g, 2g + 1 of one wave): lane h takes sum h to affine
// and runs its single-pair Miller loop (h = 0: W with the A' sum, h = 1: g2 with the
// -ABar sum; a sum at O contributes 1), lane 1 hands its Fp12 value to lane 0 by
// shuffles, and lane 0 multiplies, exponentiates and writes gok[g] <- 1 if the
// product is 1 in GT.  The two Miller loops run side by side instead of one 2-pair
// loop on one lane (the group check is a call's latency, not its device work).
// Lane 0 also clears the list counter.
template <class B>
FTS_DEV void shfl_f(typename B::F& a, int src) {
#pragma unroll
  for (int q = 0; q < 8; q++) a.v[q] = (uint32_t)__shfl((int)a.v[q], src, 64);
}
template <class B>
FTS_DEV void shfl_f12(pair::F12<B>& f, int src) {
  shfl_f<B>(f.c0.c0.a, src), shfl_f<B>(f.c0.c0.b, src), shfl_f<B>(f.c0.c1.a, src), shfl_f<B>(f.c0.c1.b, src);
  shfl_f<B>(f.c0.c2.a, src), shfl_f<B>(f.c0.c2.b, src), shfl_f<B>(f.c1.c0.a, src), shfl_f<B>(f.c1.c0.b, src);
  shfl_f<B>(f.c1.c1.a, src), shfl_f<B>(f.c1.c1.b, src), shfl_f<B>(f.c1.c2.a, src), shfl_f<B>(f.c1.c2.b, src);
}
template <class CV>
__global__ void __launch_bounds__(64, FTS_IDV_OCC) k_idv_bp_pair(int ng, const uint32_t* __restrict__ part,
                                                    const uint32_t* __restrict__ lines, int32_t* __restrict__ gok,
                                                    int32_t* __restrict__ count) {
  using B = typename CV::B;
  using K = typename B::K;
  using F = typename B::F;
  static_assert(64 % 2 == 0, "a group's lane pair must sit in one wave");
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = gid >> 1, h = gid & 1;
  if (gid == 0) *count = 0;
  // no early return before the shuffle: both lanes of every pair reach it
  const bool live = g < ng;
  const uint32_t* S = part + (size_t)(live ? g : 0) * 48 + h * 24;
  const F z = B::ld(S + 16);
  const bool o = !live || B::is_zero(z);
  pair::F12<B> f = pair::f12_one<B>();
  if (!o) {
    const F zi = B::inv(z), zi2 = B::mul(zi, zi);
    const F x1[1] = {B::mul(B::ld(S), zi2)}, y1[1] = {B::mul(B::mul(B::ld(S + 8), zi2), zi)};
    const uint32_t* const L1[1] = {lines + (size_t)h * pair::n_lines<K>() * pair::LINE_WORDS};
    f = pair::miller<B, 1>(L1, x1, y1);
  }
  pair::F12<B> f1 = f;
  shfl_f12<B>(f1, (threadIdx.x & ~1) | 1);
  if (h == 0 && live) gok[g] = pair::is_one(pair::final_exp_i(pair::mul12_i(f, f1))) ? 1 : 0;
}

// identity per lane: verdict of the identities of passing groups; the others are
// appended to the list k_idv_pairing pairs one by one
template <class CV>  // (per-curve instance: one per translation unit)
__global__ void __launch_bounds__(256) k_idv_bp_sel(int n, const int32_t* __restrict__ gok,
                                                    const int32_t* __restrict__ zk, int32_t* __restrict__ status,
                                                    int32_t* __restrict__ list, int32_t* __restrict__ count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != FTS_OK) return;
  if (gok[i / BP_G]) {
    status[i] = zk[i] ? FTS_OK : FTS_E_ID_ZK;
    return;
  }
  list[atomicAdd(count, 1)] = i;
}

// debug: e(Q, P) for Q = W (which 0) or g2 (1), P affine Montgomery -> GT (12 Fp2
// coefficients w^0..w^5 as (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2), plain LE limbs)
template <class CV>
__global__ void __launch_bounds__(64) k_idv_pairing_debug(const uint32_t* __restrict__ lines, int which, const uint32_t* __restrict__ p16,
                                    uint32_t* __restrict__ out, int final_exp) {
  using B = typename CV::B;
  using K = typename B::K;
  using F = typename B::F;
  if (threadIdx.x) return;
  const uint32_t* const L[1] = {lines + (size_t)which * pair::n_lines<K>() * pair::LINE_WORDS};
  const F xP[1] = {B::ld(p16)}, yP[1] = {B::ld(p16 + 8)};
  pair::F12<B> f = pair::miller<B, 1>(L, xP, yP);
  if (final_exp) f = pair::final_exp_i(f);
  const pair::F2<B> z[6] = {f.c0.c0, f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2, f.c1.c2};
  for (int k = 0; k < 6; k++) {
    pair::store_f2(out + k * 16, z[k]);
  }
}

// ------------------------------------------------- per-curve launch sequences
// Instantiated once per curve and translation unit: BN254 here, FP256BN in
// idemix_identity_fbn.hip (each curve's pairing kernels are minutes of device
// compilation; two units build in parallel).
struct Chain {
  hipStream_t s;
  int n;
  const uint32_t* rec;
  const uint8_t *pts, *epk;
  uint32_t *scr, *pin;
  int32_t *zk, *st;
  const int32_t *eidx, *g2ok;  // BN254 epoch keys (FP256BN: null)
  const uint32_t *tables, *hash, *lines;
  uint8_t* msg;
  int32_t *gok, *cnt, *list;
  Key8 key;
};
// decode, the t-value products, the t-values and the transcript
template <class CV>
void launch_tvals(const Chain& c) {
  const unsigned g256 = (unsigned)((c.n + 255) / 256), gvar = (unsigned)(((size_t)NSC * c.n + 255) / 256);
  k_idv_decode<CV><<<g256, 256, 0, c.s>>>(c.n, c.rec, c.pts, c.epk, c.scr, c.pin, c.zk, c.st, c.eidx, c.g2ok);
  k_idv_var<CV><<<gvar, 256, 0, c.s>>>(c.n, c.rec, c.tables, c.scr, c.st);
  k_idv_tvals<CV><<<g256, 256, 0, c.s>>>(c.n, c.rec, c.tables, c.hash, c.scr, c.msg, c.zk, c.st);
}
// the batch pairing check up to the list of identities to pair one by one
template <class CV>
void launch_batch(const Chain& c) {
  const size_t n = (size_t)c.n, ng = (n + BP_G - 1) / BP_G;
  k_idv_bp_terms<CV><<<dim3((unsigned)ng, 2), BP_G, 0, c.s>>>(c.n, c.pin, c.st, c.key, c.scr, c.scr + bp_part_off(n));
  k_idv_bp_pair<CV><<<(unsigned)((2 * ng + 63) / 64), 64, 0, c.s>>>((int)ng, c.scr + bp_part_off(n), c.lines, c.gok,
                                                                  c.cnt);
  k_idv_bp_sel<CV><<<(unsigned)((n + 255) / 256), 256, 0, c.s>>>(c.n, c.gok, c.zk, c.st, c.list, c.cnt);
}
// one-by-one pairings: `lanes` identities of the list (list) or all n
template <class CV>
void launch_pairing(const Chain& c, unsigned lanes, bool list) {
  k_idv_pairing<CV><<<(lanes + 63) / 64, 64, 0, c.s>>>(c.n, c.pin, c.lines, c.zk, c.st, list ? c.list : nullptr,
                                                        list ? c.cnt : nullptr);
}
template <class CV>
void launch_lines(const uint8_t* w, uint32_t* lines, int32_t* ok, hipStream_t s) {
  k_idv_lines<CV><<<1, 64, 0, s>>>(w, lines, ok);
}

#ifdef IDV_FBN_TU
}  // namespace idv (the FP256BN unit holds kernels only)
#else  // the host side
extern template void launch_tvals<FbnCurve>(const Chain&);
extern template void launch_batch<FbnCurve>(const Chain&);
extern template void launch_pairing<FbnCurve>(const Chain&, unsigned, bool);
extern template void launch_lines<FbnCurve>(const uint8_t*, uint32_t*, int32_t*, hipStream_t);

// ------------------------------------------------------------------- host
const uint32_t kRbn[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                          0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
const uint32_t kRfbn[8] = {0xd10b500du, 0xf62d536cu, 0x1299921au, 0x0cdc65fbu,
                           0xee71a49eu, 0x46e5f25eu, 0xfffcf0cdu, 0xffffffffu};

bool ge(const uint32_t a[8], const uint32_t m[8]) {
  for (int k = 7; k >= 0; k--)
    if (a[k] != m[k]) return a[k] > m[k];
  return true;
}
void subm(uint32_t a[8], const uint32_t m[8]) {
  uint64_t bw = 0;
  for (int k = 0; k < 8; k++) {
    const uint64_t d = (uint64_t)a[k] - m[k] - bw;
    a[k] = (uint32_t)d;
    bw = (d >> 63) & 1;
  }
}
// big-endian bytes -> LE limbs if the value fits 256 bits
bool be_limbs(const uint8_t* b, size_t len, uint32_t out[8]) {
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
// (x * 256 + byte) mod m for x < m < 2^256
void mulacc_byte(uint32_t x[8], uint8_t byte, const uint32_t m[8]) {
  uint32_t t[9];
  uint64_t c = byte;
  for (int k = 0; k < 8; k++) {
    const uint64_t v = ((uint64_t)x[k] << 8) + c;
    t[k] = (uint32_t)v;
    c = v >> 32;
  }
  t[8] = (uint32_t)c;
  for (int guard = 0; guard < 600; guard++) {
    if (t[8] == 0 && !ge(t, m)) break;
    uint64_t bw = 0;
    for (int k = 0; k < 9; k++) {
      const uint64_t d = (uint64_t)t[k] - (k < 8 ? m[k] : 0u) - bw;
      t[k] = (uint32_t)d;
      bw = (d >> 63) & 1;
    }
  }
  memcpy(x, t, 32);
}
void mod_m(const uint8_t* b, size_t len, const uint32_t m[8], uint32_t out[8]) {
  if (be_limbs(b, len, out)) {
    while (ge(out, m)) subm(out, m);
    return;
  }
  memset(out, 0, 32);
  for (size_t k = 0; k < len; k++) mulacc_byte(out, b[k], m);
}

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
  bool set = false;
};
// ECP{1 x, 2 y} -> 64 raw bytes; false if a coordinate is not 32 bytes or the message is malformed
bool ecp_raw(const Span& s, uint8_t out[64]) {
  if (!s.set) return false;
  Pb pb{s.p, s.n};
  Span f[3];
  while (pb.o < pb.n) {
    uint32_t fn, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(fn, wt, v, vl, iv)) return false;
    if (fn == 1 || fn == 2) {
      if (wt != 2) return false;
      f[fn].p = v, f[fn].n = vl, f[fn].set = true;
    }
  }
  if (f[1].n != 32 || f[2].n != 32) return false;
  memcpy(out, f[1].p, 32);
  memcpy(out + 32, f[2].p, 32);
  return true;
}
bool ecp2_raw(const Span& s, uint8_t out[128]) {
  if (!s.set) return false;
  Pb pb{s.p, s.n};
  Span f[5];
  while (pb.o < pb.n) {
    uint32_t fn, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(fn, wt, v, vl, iv)) return false;
    if (fn >= 1 && fn <= 4) {
      if (wt != 2) return false;
      f[fn].p = v, f[fn].n = vl, f[fn].set = true;
    }
  }
  for (int q = 1; q <= 4; q++) {
    if (f[q].n != 32) return false;
    memcpy(out + 32 * (q - 1), f[q].p, 32);
  }
  return true;
}

// SerializedIdemixIdentity + its Signature proto -> record, raw points, epoch key;
// returns the identity-level status (FTS_OK: to the device)
int32_t parse_identity(const uint8_t* id, size_t len, bool bn, const uint32_t* rmod, uint32_t* rec, uint8_t* pts,
                       uint8_t* epk) {
  memset(rec, 0, REC_STRIDE * 4);
  memset(pts, 0, NPT * 64);
  memset(epk, 0, 128);
  if (!id || !len) return FTS_E_ID_MALFORMED;  // "empty identity"
  Span nym, proof;
  {
    Pb pb{id, len};
    while (pb.o < pb.n) {
      uint32_t f, wt;
      const uint8_t* v;
      size_t vl;
      uint64_t iv;
      if (!pb.next(f, wt, v, vl, iv)) return FTS_E_ID_MALFORMED;
      if (f >= 1 && f <= 4 && wt != 2) return FTS_E_ID_MALFORMED;
      if (f == 1) nym.p = v, nym.n = vl, nym.set = true;
      if (f == 4) proof.p = v, proof.n = vl, proof.set = true;
    }
  }
  if (nym.n == 0) return FTS_E_ID_MALFORMED;  // "pseudonym's public key is empty"
  // KeyImport: G1.Bytes() form; its point checks run on the device
  if (bn ? nym.n != 64 : (nym.n != 65 || nym.p[0] != 0x04)) return FTS_E_ID_BADNYM;
  memcpy(pts + P_NYMPK * 64, nym.p + (bn ? 0 : 1), 64);
  uint32_t& flags = rec[R_FLAGS];
  // Signature proto (IBM/idemix idemix.proto, restated): 1 a_prime 2 a_bar 3 b_prime (ECP),
  // 4 c 5 s_sk 6 s_e 7 s_r2 8 s_r3 9 s_s_prime, 10 s_attrs (repeated), 11 nonce, 12 nym (ECP),
  // 13 s_r_nym, 14 revocation_epoch_pk (ECP2), 15 revocation_pk_sig, 16 epoch, 17 non_revocation_proof,
  // 18 eid_nym {1 nym, 2 s_eid}, 19 rh_nym {1 nym, 2 s_rh}
  Span f[20];
  std::vector<Span> attrs;
  attrs.reserve(4);
  if (proof.n == 0) {
    flags |= F_EARLY_MALFORMED;  // an empty signature is rejected before Unmarshal
  } else {
    Pb pb{proof.p, proof.n};
    while (pb.o < pb.n) {
      uint32_t fn, wt;
      const uint8_t* v;
      size_t vl;
      uint64_t iv;
      if (!pb.next(fn, wt, v, vl, iv)) {
        flags |= F_EARLY_MALFORMED;
        break;
      }
      if (fn >= 1 && fn <= 19 && fn != 16 && wt != 2) {
        flags |= F_EARLY_MALFORMED;
        break;
      }
      if (fn == 16 && wt != 0) {
        flags |= F_EARLY_MALFORMED;
        break;
      }
      if (fn == 10) attrs.push_back(Span{v, vl, true});
      else if (fn >= 1 && fn <= 19) f[fn] = Span{v, vl, true};
    }
  }
  // Zr fields: BN254 big-endian integers of any length; FP256BN AMCL FromBytes reads
  // exactly 32 bytes (a shorter field panics in the reference)
  auto zr = [&](const Span& s, uint32_t out[8], bool& wide) -> bool {
    wide = false;
    if (bn) {
      uint32_t raw[8];
      if (!be_limbs(s.p, s.n, raw)) wide = true;
      mod_m(s.p, s.n, rmod, out);
      return true;
    }
    if (s.n < 32) return false;
    be_limbs(s.p, 32, out);
    if (ge(out, rmod)) subm(out, rmod);
    return true;
  };
  uint32_t sc[24][8];
  memset(sc, 0, sizeof sc);
  Span eid_nym, rh_nym, s_eid, s_rh;
  uint32_t rev_alg = 0;
  if (!(flags & F_EARLY_MALFORMED)) {
    // sub-messages: 17 NonRevocationProof{1 revocation_alg}, 18 / 19 {1 nym, 2 s}
    auto sub = [&](const Span& s, Span& a, Span& b) -> bool {
      if (!s.set) return true;
      Pb pb{s.p, s.n};
      while (pb.o < pb.n) {
        uint32_t fn, wt;
        const uint8_t* v;
        size_t vl;
        uint64_t iv;
        if (!pb.next(fn, wt, v, vl, iv)) return false;
        if ((fn == 1 || fn == 2) && wt != 2) return false;
        if (fn == 1) a = Span{v, vl, true};
        if (fn == 2) b = Span{v, vl, true};
      }
      return true;
    };
    bool good = sub(f[18], eid_nym, s_eid) && sub(f[19], rh_nym, s_rh);
    if (f[17].set) {
      Pb pb{f[17].p, f[17].n};
      while (good && pb.o < pb.n) {
        uint32_t fn, wt;
        const uint8_t* v;
        size_t vl;
        uint64_t iv;
        if (!pb.next(fn, wt, v, vl, iv)) good = false;
        else if (fn == 1 && wt != 0) good = false;
        else if (fn == 1) rev_alg = (uint32_t)iv;
        else if (fn == 2 && wt != 2) good = false;
      }
    }
    // the scalars: c(4) sSk(5) sE(6) sR2(7) sR3(8) sS'(9) nonce(11) sRNym(13) sAttrs sEid sRh
    const int fld[8] = {4, 5, 6, 7, 8, 9, 11, 13};
    bool wide[8] = {false};
    for (int q = 0; q < 8 && good; q++) good = zr(f[fld[q]], sc[q], wide[q]);
    for (size_t a = 0; a < attrs.size() && a < 4 && good; a++) {
      bool w;
      good = zr(attrs[a], sc[8 + a], w);
    }
    for (size_t a = 4; a < attrs.size() && good; a++) {
      uint32_t tmp[8];
      bool w;
      good = zr(attrs[a], tmp, w);
    }
    if (good && f[18].set) {
      bool w;
      good = zr(s_eid, sc[12], w);
    }
    if (good && f[19].set) {
      bool w;
      good = zr(s_rh, sc[13], w);
    }
    if (!good) {
      flags |= F_EARLY_MALFORMED;
    } else {
      // nonce: Zr.Bytes() of a value wider than 32 bytes panics (mathlib BigToBytes)
      uint32_t nonce[8];
      if (bn) {
        if (!be_limbs(f[11].p, f[11].n, nonce)) flags |= F_EARLY_MALFORMED;
      } else {
        be_limbs(f[11].p, 32, nonce);
      }
      for (int k = 0; k < 8; k++) rec[R_NONCE + k] = nonce[7 - k];
      // c: compared as an integer with the recomputed (reduced) challenge
      uint32_t craw[8];
      if (bn) {
        if (!be_limbs(f[4].p, f[4].n, craw) || ge(craw, rmod)) flags |= F_C_BIG;
      } else {
        be_limbs(f[4].p, 32, craw);
        if (ge(craw, rmod)) flags |= F_C_BIG;
      }
      memcpy(rec + R_C, craw, 32);
    }
  }
  if (!(flags & F_EARLY_MALFORMED)) {
    if (!f[18].set) flags |= F_NO_EID;
    else if (!f[19].set) flags |= F_NO_RH;
  }
  if (!(flags & (F_EARLY_MALFORMED | F_NO_EID | F_NO_RH))) {
    bool good = ecp_raw(f[1], pts + P_AP * 64) && ecp_raw(f[2], pts + P_ABAR * 64) &&
                ecp_raw(f[3], pts + P_BP * 64) && ecp_raw(f[12], pts + P_NYM * 64) &&
                ecp_raw(eid_nym, pts + P_EID * 64) && ecp_raw(rh_nym, pts + P_RH * 64) && attrs.size() == 4 &&
                ecp2_raw(f[14], epk);
    if (!good) flags |= F_LATE_MALFORMED;
    if (rev_alg != 0) flags |= F_REVOCATION;
    // scalars: var [sE, -c, sR3, -c, -c, -c]; fixed as FIX_B / FIX_T
    uint32_t cm[8], nc[8];
    memcpy(cm, sc[0], 32);
    memset(nc, 0, 32);
    {
      uint32_t z = 0;
      for (int k = 0; k < 8; k++) z |= cm[k];
      if (z) {
        uint64_t bw = 0;
        for (int k = 0; k < 8; k++) {
          const uint64_t d = (uint64_t)rmod[k] - cm[k] - bw;
          nc[k] = (uint32_t)d;
          bw = (d >> 63) & 1;
        }
      }
    }
    const uint32_t* var[NVAR] = {sc[2], nc, sc[4], nc, nc, nc};
    // fixed: sR2, sS', sSk (t2, t3), sA0, sA1, sA2 (t2, t4), sA3 (t2, t5), c, sRNym, sEid, sRh
    const uint32_t* fix[NFIX] = {sc[3], sc[5], sc[1], sc[8], sc[9], sc[10], sc[11], cm, sc[7], sc[12], sc[13]};
    for (int v = 0; v < NVAR; v++) memcpy(rec + R_SC + v * 8, var[v], 32);
    for (int q = 0; q < NFIX; q++) memcpy(rec + R_SC + (NVAR + q) * 8, fix[q], 32);
  }
  return FTS_OK;
}

#define ICHK(x)                                    \
  do {                                             \
    if ((x) != hipSuccess) return FTS_API_EDEVICE; \
  } while (0)

constexpr int NSLOT = 8;  // calls in flight per handle (each slot: its own stream and buffers, grown on first use;
                          // 12 concurrent calls hit HSA_STATUS_ERROR_OUT_OF_RESOURCES dispatching the
                          // scratch-using pairing kernels, gpurun_out/ns)
struct Slot {
  hipStream_t stream = nullptr;
  uint8_t* d_buf = nullptr;
  size_t d_cap = 0;
  uint8_t* h_buf = nullptr;
  size_t h_cap = 0;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  float ms[2] = {0.f, 0.f};
  uint32_t stats[2] = {0u, 0u};
};

}  // namespace idv

struct fts_idemix_idv {
  int device = -1;
  int curve = 1;
  uint32_t* d_tables = nullptr;  // HSk, HRand, HAttrs[0..3], g1
  uint32_t* d_lines = nullptr;   // lines of W, then of g2
  uint32_t* d_hash = nullptr;    // ipk.Hash as 8 big-endian words
  std::mutex mu;
  std::condition_variable cv;
  idv::Slot slot[idv::NSLOT];
  bool busy[idv::NSLOT] = {};
  float last_ms[2] = {0.f, 0.f};
  // batch pairing check (k_idv_bp_*; FTS_IDV_BATCH=0 pairs every identity, the A/B
  // and pre-round-6 path); last call's groups and identities paired one by one
  bool batch = true;
  uint32_t last_stats[2] = {0u, 0u};
  // BN254 epoch keys already subgroup-checked by this context (128 raw bytes ->
  // verdict): an honest stream carries one key per epoch, and k_idv_g2_check is
  // one 254-step G2 chain on one lane (7.7 ms, on the call's critical path)
  std::unordered_map<std::string, int32_t> g2_seen;
};

namespace idv {
void idv_free(fts_idemix_idv* k) {
  if (!k) return;
  if (k->device >= 0) (void)hipSetDevice(k->device);
  for (auto& S : k->slot) {
    if (S.stream) (void)hipStreamSynchronize(S.stream), (void)hipStreamDestroy(S.stream);
    for (auto& e : S.ev)
      if (e) (void)hipEventDestroy(e);
    if (S.d_buf) (void)hipFree(S.d_buf);
    if (S.h_buf) (void)hipHostFree(S.h_buf);
  }
  for (uint32_t* p : {k->d_tables, k->d_lines, k->d_hash})
    if (p) (void)hipFree(p);
  delete k;
}
int nlines(bool bn) { return bn ? pair::n_lines<pairc::Bn254>() : pair::n_lines<pairc::Fp256bn>(); }
}  // namespace idv

extern "C" {

int fts_idemix_idv_create(int device, const uint8_t* ipk, size_t ipk_len, int curve_id, fts_idemix_idv** out) {
  using namespace idv;
  if (!out || !ipk || !ipk_len || (curve_id != FTS_CURVE_BN254 && curve_id != FTS_CURVE_FP256BN_AMCL))
    return FTS_API_EINVAL;
  *out = nullptr;
  const bool bn = curve_id == FTS_CURVE_BN254;
  // IssuerPublicKey: 2 h_sk, 3 h_rand, 4 h_attrs (repeated ECP), 5 w (ECP2), 10 hash
  Pb pb{ipk, ipk_len};
  Span hsk, hr, w, hash;
  std::vector<Span> ha;
  while (pb.o < pb.n) {
    uint32_t f, wt;
    const uint8_t* v;
    size_t vl;
    uint64_t iv;
    if (!pb.next(f, wt, v, vl, iv)) return FTS_API_EPP;
    if (wt != 2) continue;
    if (f == 2) hsk = Span{v, vl, true};
    if (f == 3) hr = Span{v, vl, true};
    if (f == 4) ha.push_back(Span{v, vl, true});
    if (f == 5) w = Span{v, vl, true};
    if (f == 10) hash = Span{v, vl, true};
  }
  if (ha.size() != 4) return FTS_API_EPP;  // OU, Role, EnrollmentID, RevocationHandle
  uint8_t raw[NB][64], wraw[128];
  if (!ecp_raw(hsk, raw[B_HSK]) || !ecp_raw(hr, raw[B_HRAND]) || !ecp2_raw(w, wraw)) return FTS_API_EPP;
  for (int a = 0; a < 4; a++)
    if (!ecp_raw(ha[a], raw[B_HA + a])) return FTS_API_EPP;
  memset(raw[B_G1], 0, 64);  // g1 = (1, 2) on both curves
  raw[B_G1][31] = 1, raw[B_G1][63] = 2;
  uint32_t bases[NB * 16];  // BN254: Montgomery (host decode); FP256BN: plain LE limbs
  for (int b = 0; b < NB; b++) {
    if (bn) {
      host::G1A a;
      if (!host::g1_from_bytes(raw[b], 64, a) || a.inf) return FTS_API_EPP;
      memcpy(&bases[b * 16], a.x.v, 32);
      memcpy(&bases[b * 16 + 8], a.y.v, 32);
    } else {
      be_limbs(raw[b], 32, &bases[b * 16]);
      be_limbs(raw[b] + 32, 32, &bases[b * 16 + 8]);
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return FTS_API_EDEVICE;
  fts_idemix_idv* k = new fts_idemix_idv();
  k->device = device;
  k->curve = curve_id;
  if (const char* e = getenv("FTS_IDV_BATCH")) k->batch = atoi(e) != 0;
  auto fail = [&](int rc) {
    idv_free(k);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(FTS_API_EDEVICE);
  uint32_t hw[8] = {0};
  {
    uint8_t h[32] = {0};
    if (hash.set) memcpy(h, hash.p, std::min<size_t>(hash.n, 32));
    for (int q = 0; q < 8; q++)
      hw[q] = ((uint32_t)h[4 * q] << 24) | ((uint32_t)h[4 * q + 1] << 16) | ((uint32_t)h[4 * q + 2] << 8) | h[4 * q + 3];
  }
  const size_t wpb = bn ? fb_words_per_base() : fbn_words_per_base();
  const size_t nl = (size_t)nlines(bn) * pair::LINE_WORDS;
  hipStream_t s0 = nullptr;
  uint32_t *d_bases = nullptr, *d_scr = nullptr;
  uint8_t* d_w = nullptr;
  int32_t* d_ok = nullptr;
  const size_t scr_b = bn ? table_build_scratch_bytes(NB) : (size_t)NB * 16 * 4;
  bool ok = hipStreamCreateWithFlags(&s0, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&k->d_tables, (size_t)NB * wpb * 4) == hipSuccess &&
            hipMalloc(&k->d_lines, 2 * nl * 4) == hipSuccess && hipMalloc(&k->d_hash, 32) == hipSuccess &&
            hipMalloc(&d_bases, sizeof bases) == hipSuccess && hipMalloc(&d_scr, scr_b) == hipSuccess &&
            hipMalloc(&d_w, 128) == hipSuccess && hipMalloc(&d_ok, 64) == hipSuccess &&
            hipMemcpyAsync(d_bases, bases, sizeof bases, hipMemcpyHostToDevice, s0) == hipSuccess &&
            hipMemcpyAsync(d_w, wraw, 128, hipMemcpyHostToDevice, s0) == hipSuccess &&
            hipMemcpyAsync(k->d_hash, hw, 32, hipMemcpyHostToDevice, s0) == hipSuccess &&
            hipMemsetAsync(d_ok, 0, 64, s0) == hipSuccess;
  int32_t hok[NB + 1] = {0};
  if (ok) {
    if (bn) {
      launch_build_tables(d_bases, NB, k->d_tables, d_scr, s0);
      launch_lines<BnCurve>(d_w, k->d_lines, d_ok + NB, s0);
    } else {
      fbn_build_tables(d_bases, NB, d_scr, d_ok, k->d_tables, s0);
      launch_lines<FbnCurve>(d_w, k->d_lines, d_ok + NB, s0);
    }
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(hok, d_ok, sizeof hok, hipMemcpyDeviceToHost, s0) == hipSuccess &&
         hipStreamSynchronize(s0) == hipSuccess;
  }
  if (s0) (void)hipStreamSynchronize(s0);
  for (void* p : {(void*)d_bases, (void*)d_scr, (void*)d_w, (void*)d_ok})
    if (p) (void)hipFree(p);
  if (s0) (void)hipStreamDestroy(s0);
  if (!ok) return fail(FTS_API_EDEVICE);
  bool valid = hok[NB] == 1;  // W on the twist
  if (!bn)
    for (int b = 0; b < NB; b++) valid = valid && hok[b] == 1;
  if (!valid) return fail(FTS_API_EPP);
  for (auto& S : k->slot) {
    ok = ok && hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) == hipSuccess;
    for (auto& e : S.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  }
  if (!ok) return fail(FTS_API_EDEVICE);
  *out = k;
  return FTS_API_OK;
}

void fts_idemix_idv_destroy(fts_idemix_idv* k) { idv::idv_free(k); }

int fts_idemix_identity_verify_batch(fts_idemix_idv* K, size_t n, const uint8_t* const* ids, const size_t* id_len,
                                     int32_t* status) {
  using namespace idv;
  if (!K || n > (size_t)(1u << 22) || (n && (!ids || !id_len || !status))) return FTS_API_EINVAL;
  if (n == 0) return FTS_API_OK;
  const bool bn = K->curve == FTS_CURVE_BN254;
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
    fts_idemix_idv* K;
    int k;
    ~Guard() {
      if (K->slot[k].stream) (void)hipStreamSynchronize(K->slot[k].stream);
      std::lock_guard<std::mutex> l(K->mu);
      K->last_ms[0] = K->slot[k].ms[0], K->last_ms[1] = K->slot[k].ms[1];
      K->last_stats[0] = K->slot[k].stats[0], K->last_stats[1] = K->slot[k].stats[1];
      K->busy[k] = false;
      K->cv.notify_one();
    }
  } guard{K, k};
  Slot& D = K->slot[k];
  ICHK(hipSetDevice(K->device));
  // staged (host + device): rec | pts | epk | status | eidx | distinct epoch keys (BN254);
  // device only: zk | pin | scratch | msg | g2ok
  const size_t rec_b = n * REC_STRIDE * 4, pts_b = n * NPT * 64, epk_b = n * 128, st_b = n * 4;
  const size_t o_pts = rec_b, o_epk = o_pts + pts_b, o_st = o_epk + epk_b, o_eidx = o_st + st_b,
               o_uk = o_eidx + n * 4;
  // host only: the distinct keys' verdicts (cached or read back) and the indices to check
  const size_t o_gk = (o_uk + epk_b + 255) & ~size_t(255), o_miss = o_gk + n * 4;
  const size_t o_cnt = o_miss + n * 4;  // the batch check's list length, read back
  const size_t h_need = (o_cnt + 4 + 255) & ~size_t(255);
  const size_t o_zk = h_need, o_pin = (o_zk + n * 4 + 255) & ~size_t(255), o_scr = o_pin + n * 32 * 4;
  const size_t scr_w = std::max(idv_scratch_words(n), bp_scratch_words(n));
  const size_t o_msg = (o_scr + scr_w * 4 + 255) & ~size_t(255);
  const size_t o_g2ok = (o_msg + (size_t)MSG_MAX * n + 255) & ~size_t(255);
  const size_t d_need = o_g2ok + 2 * n * 4;  // U verdicts, then the M key indices to check
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
  const uint32_t* rmod = bn ? kRbn : kRfbn;
  const size_t CH = 1024, nch = (n + CH - 1) / CH;
  host_parallel_for(nch, [&](size_t c) {
    for (size_t i = c * CH; i < std::min(n, (c + 1) * CH); i++)
      reinterpret_cast<int32_t*>(h + o_st)[i] =
          parse_identity(ids[i], id_len[i], bn, rmod, reinterpret_cast<uint32_t*>(h) + i * REC_STRIDE,
                         h + o_pts + i * NPT * 64, h + o_epk + i * 128);
  });
  // BN254 epoch keys: one subgroup check per DISTINCT key (honest batches carry one)
  size_t U = 0;
  int32_t* eidx = reinterpret_cast<int32_t*>(h + o_eidx);
  if (bn) {
    const uint8_t* E = h + o_epk;
    uint8_t* UK = h + o_uk;
    std::atomic<bool> same{true};
    host_parallel_for(nch, [&](size_t c) {
      for (size_t i = c * CH; i < std::min(n, (c + 1) * CH) && same.load(std::memory_order_relaxed); i++)
        if (memcmp(E + i * 128, E, 128) != 0) same = false;
    });
    if (same) {
      memcpy(UK, E, 128);
      std::fill(eidx, eidx + n, 0);
      U = 1;
    } else {  // sort by (hash, bytes), then one entry per run of equal keys
      std::vector<std::pair<uint64_t, uint32_t>> hk(n);
      for (size_t i = 0; i < n; i++) {
        uint64_t x = 0x9e3779b97f4a7c15ull;
        for (int q = 0; q < 16; q++) {
          uint64_t w;
          memcpy(&w, E + i * 128 + 8 * q, 8);
          x = (x ^ w) * 0xff51afd7ed558ccdull;
          x ^= x >> 29;
        }
        hk[i] = {x, (uint32_t)i};
      }
      std::sort(hk.begin(), hk.end(), [&](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) {
        if (a.first != b.first) return a.first < b.first;
        return memcmp(E + (size_t)a.second * 128, E + (size_t)b.second * 128, 128) < 0;
      });
      for (size_t j = 0; j < n; j++) {
        const uint32_t i = hk[j].second;
        if (j == 0 || hk[j].first != hk[j - 1].first ||
            memcmp(E + (size_t)i * 128, E + (size_t)hk[j - 1].second * 128, 128) != 0)
          memcpy(UK + 128 * U++, E + (size_t)i * 128, 128);
        eidx[i] = (int32_t)(U - 1);
      }
    }
  }
  // cached key verdicts; the misses are checked on the device and cached after the call
  int32_t* gk = reinterpret_cast<int32_t*>(h + o_gk);
  int32_t* miss = reinterpret_cast<int32_t*>(h + o_miss);
  size_t M = 0;
  if (bn) {
    std::lock_guard<std::mutex> l(K->mu);
    for (size_t j = 0; j < U; j++) {
      const auto it = K->g2_seen.find(std::string(reinterpret_cast<const char*>(h + o_uk + 128 * j), 128));
      if (it != K->g2_seen.end()) {
        gk[j] = it->second;
      } else {
        gk[j] = 0;
        miss[M++] = (int32_t)j;
      }
    }
  }
  uint8_t* d = D.d_buf;
  ICHK(hipMemcpyAsync(d, h, o_uk + U * 128, hipMemcpyHostToDevice, D.stream));
  ICHK(hipEventRecord(D.ev[0], D.stream));
  // batch pairing check: group sums, one pairing product per group, the identities
  // of failing groups listed for k_idv_pairing
  uint32_t* scr = reinterpret_cast<uint32_t*>(d + o_scr);
  const size_t ng = (n + BP_G - 1) / BP_G;
  Chain c;
  c.s = D.stream, c.n = (int)n, c.rec = reinterpret_cast<const uint32_t*>(d), c.pts = d + o_pts, c.epk = d + o_epk;
  c.scr = scr, c.pin = reinterpret_cast<uint32_t*>(d + o_pin);
  c.zk = reinterpret_cast<int32_t*>(d + o_zk), c.st = reinterpret_cast<int32_t*>(d + o_st);
  int32_t* g2ok = reinterpret_cast<int32_t*>(d + o_g2ok);
  c.eidx = bn ? reinterpret_cast<const int32_t*>(d + o_eidx) : nullptr, c.g2ok = bn ? g2ok : nullptr;
  c.tables = K->d_tables, c.hash = K->d_hash, c.lines = K->d_lines, c.msg = d + o_msg;
  c.gok = reinterpret_cast<int32_t*>(scr + bp_gok_off(n, ng));
  c.cnt = reinterpret_cast<int32_t*>(scr + bp_cnt_off(n, ng));
  c.list = reinterpret_cast<int32_t*>(scr + bp_list_off(n, ng));
  if (K->batch && getrandom(c.key.k, sizeof c.key.k, 0) != (ssize_t)sizeof c.key.k) return FTS_API_EDEVICE;
  if (bn) {
    ICHK(hipMemcpyAsync(g2ok, gk, U * 4, hipMemcpyHostToDevice, D.stream));
    if (M) {
      ICHK(hipMemcpyAsync(g2ok + U, miss, M * 4, hipMemcpyHostToDevice, D.stream));
      k_idv_g2_check<<<(unsigned)((M + 63) / 64), 64, 0, D.stream>>>((int)M, g2ok + U, d + o_uk, g2ok);
    }
  }
  bn ? launch_tvals<BnCurve>(c) : launch_tvals<FbnCurve>(c);
  ICHK(hipEventRecord(D.ev[1], D.stream));
  unsigned nlist = 0;  // identities of failing groups (read back after k_idv_bp_sel)
  if (K->batch) {
    bn ? launch_batch<BnCurve>(c) : launch_batch<FbnCurve>(c);
    ICHK(hipMemcpyAsync(h + o_cnt, c.cnt, 4, hipMemcpyDeviceToHost, D.stream));
    ICHK(hipStreamSynchronize(D.stream));
    nlist = *reinterpret_cast<const uint32_t*>(h + o_cnt);
    // exact grid: idle pairing waves (256 VGPRs and scratch each) would still queue
    // behind the other slots' kernels
    if (nlist) bn ? launch_pairing<BnCurve>(c, nlist, true) : launch_pairing<FbnCurve>(c, nlist, true);
  } else {
    bn ? launch_pairing<BnCurve>(c, (unsigned)n, false) : launch_pairing<FbnCurve>(c, (unsigned)n, false);
  }
  ICHK(hipGetLastError());
  ICHK(hipEventRecord(D.ev[2], D.stream));
  ICHK(hipMemcpyAsync(h + o_st, d + o_st, st_b, hipMemcpyDeviceToHost, D.stream));
  if (M) ICHK(hipMemcpyAsync(gk, g2ok, U * 4, hipMemcpyDeviceToHost, D.stream));
  ICHK(hipStreamSynchronize(D.stream));
  memcpy(status, h + o_st, st_b);
  D.stats[0] = K->batch ? (uint32_t)ng : 0u;
  D.stats[1] = K->batch ? nlist : (uint32_t)n;
  if (M) {
    std::lock_guard<std::mutex> l(K->mu);
    if (K->g2_seen.size() + M > 4096) K->g2_seen.clear();  // bounded: a new epoch's keys refill it
    for (size_t q = 0; q < M; q++) {
      const size_t j = (size_t)miss[q];
      K->g2_seen.emplace(std::string(reinterpret_cast<const char*>(h + o_uk + 128 * j), 128), gk[j]);
    }
  }
  ICHK(hipEventElapsedTime(&D.ms[0], D.ev[0], D.ev[1]));
  ICHK(hipEventElapsedTime(&D.ms[1], D.ev[1], D.ev[2]));
  return FTS_API_OK;
}

int fts_idemix_identity_last_timings(fts_idemix_idv* K, float* ms) {
  if (!K || !ms) return FTS_API_EINVAL;
  std::lock_guard<std::mutex> l(K->mu);
  ms[0] = K->last_ms[0], ms[1] = K->last_ms[1];
  return FTS_API_OK;
}

int fts_idemix_identity_last_stats(fts_idemix_idv* K, uint32_t* out) {
  if (!K || !out) return FTS_API_EINVAL;
  std::lock_guard<std::mutex> l(K->mu);
  out[0] = K->last_stats[0], out[1] = K->last_stats[1];
  return FTS_API_OK;
}

int fts_idemix_pairing_debug(fts_idemix_idv* K, int which, const uint8_t* p64, int final_exp, uint32_t* out192) {
  using namespace idv;
  if (!K || !p64 || !out192 || (which != 0 && which != 1)) return FTS_API_EINVAL;
  const bool bn = K->curve == FTS_CURVE_BN254;
  // P: 64 raw BE bytes -> affine Montgomery (host for BN254; device converts FP256BN)
  uint32_t pm[16];
  if (bn) {
    host::G1A a;
    if (!host::g1_from_bytes(p64, 64, a) || a.inf) return FTS_API_EINVAL;
    memcpy(pm, a.x.v, 32);
    memcpy(pm + 8, a.y.v, 32);
  } else {
    return FTS_API_EINVAL;  // FP256BN points go through fts_idemix_pairing_debug_mont
  }
  std::lock_guard<std::mutex> l(K->mu);
  ICHK(hipSetDevice(K->device));
  // private stream and buffers, released on every exit path
  struct Res {
    uint32_t *p = nullptr, *o = nullptr;
    hipStream_t s = nullptr;
    ~Res() {
      if (s) (void)hipStreamSynchronize(s);
      if (p) (void)hipFree(p);
      if (o) (void)hipFree(o);
      if (s) (void)hipStreamDestroy(s);
    }
  } r;
  ICHK(hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking));
  ICHK(hipMalloc(&r.p, 64));
  ICHK(hipMalloc(&r.o, 192 * 4));
  ICHK(hipMemcpyAsync(r.p, pm, 64, hipMemcpyHostToDevice, r.s));
  k_idv_pairing_debug<BnCurve><<<1, 64, 0, r.s>>>(K->d_lines, which, r.p, r.o, final_exp);
  ICHK(hipGetLastError());
  ICHK(hipMemcpyAsync(out192, r.o, 192 * 4, hipMemcpyDeviceToHost, r.s));
  ICHK(hipStreamSynchronize(r.s));
  return FTS_API_OK;
}

}  // extern "C"
#endif  // IDV_FBN_TU
