// Proof wire decoding into device records, and encoding for the host prover.
//
//   RangeProof       = Marshal(Data, IPA)                         rp/bulletproof.go:93-101
//   RangeProofData   = MarshalMath(T1, T2, Tau, C, D, Delta, IP)  rp/bulletproof.go:37-83
//   IPA              = MarshalMath(Left, Right, ElemArray(L), ElemArray(R))   rp/ipa.go:33-67
//   RangeCorrectness = Marshal(array{Marshal(rp_0..rp_m-1)})      rp/rangecorrectness.go:19-40
//   TypeAndSumProof  = MarshalMath(CT, EA(ibf), EA(iv), Type, TBF, EqSum, Chal)   transfer/typeandsum.go:37-93
//   transfer.Proof   = Marshal(TypeAndSum, RangeCorrectness)      transfer/transfer.go:29-40
//   SameType         = MarshalMath(Type, BF, Chal, CT)            issue/sametype.go:32-64
//   issue.Proof      = Marshal(SameType, RangeCorrectness)        issue/prover.go:27-37
//
// Host parsing does DER structure, element lengths, curve ids and scalar
// reduction; point validity (flags, canonical coordinates, on-curve) is
// checked on the device by k_rp_decode for every slotted point.
#pragma once
#include <stdint.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../../include/fts_gpu.h"
#include "bn254_host.hpp"
#include "der.hpp"

namespace fts {
namespace host {

// a decoded mathlib element (unmarshaller.Next* semantics, asn1.go:128-230)
struct Elem {
  bool present = false;  // false => Go nil (values exhausted)
  der::Span raw;
};

struct Unmarshaller {
  std::vector<der::Span> own;
  std::vector<der::Span>& v;  // own, or a caller's reused buffer (no allocation per proof)
  size_t i = 0;
  bool ok = false;
  Unmarshaller(der::Span raw) : v(own) { ok = der::unmarshal_values(raw, v); }
  Unmarshaller(der::Span raw, std::vector<der::Span>& buf) : v(buf) { ok = der::unmarshal_values(raw, v); }
  // returns false on a deserialization error
  bool next(Elem& e) {
    e.present = false;
    if (i >= v.size()) return true;
    int64_t curve;
    der::Span raw;
    if (!der::unmarshal_element(v[i], curve, raw)) return false;
    if (curve != 1) return false;  // mathlib.Curves[curve]: other curve / panic
    i++;
    e.present = true;
    e.raw = raw;
    return true;
  }
};

// big-endian bytes (any length) -> value mod r as canonical 8 x u32 LE limbs;
// canonical_out = (value < r), i.e. what Zr.Equals against a reduced value needs
inline void scalar_from_bytes(der::Span s, uint32_t out[8], bool* canonical_out) {
  size_t off = 0;
  while (off < s.n && s.p[off] == 0) off++;
  size_t len = s.n - off;
  uint64_t c[4] = {0, 0, 0, 0};
  bool canonical;
  if (len <= 32) {
    uint8_t b[32] = {0};
    memcpy(b + 32 - len, s.p + off, len);
    be32_to_u64(b, c);
    canonical = !geq_mod<ModR>(c);
    while (geq_mod<ModR>(c)) sub_mod_raw<ModR>(c);
  } else {
    canonical = false;
    Fr acc = Fr::zero(), b256 = from_u64<ModR>(256);
    for (size_t i = off; i < s.n; i++) acc = add(mul(acc, b256), from_u64<ModR>(s.p[i]));
    from_mont(acc, c);
  }
  for (int i = 0; i < 4; i++) {
    out[2 * i] = (uint32_t)c[i];
    out[2 * i + 1] = (uint32_t)(c[i] >> 32);
  }
  if (canonical_out) *canonical_out = canonical;
}

// generator (1, 2) encoding: filler for unused point slots
inline void filler_point(uint8_t out[64]) {
  memset(out, 0, 64);
  out[31] = 1;
  out[63] = 2;
}

// Parse one RangeProof.  pts: (5 + 2k) x 64 raw slots (slot RP_PT_V untouched),
// sc: 5 x 8 words.  status <- 0 / FTS_E_MALFORMED / FTS_E_RP_NIL;
// ipa_flag <- 0 / FTS_E_IPA_NIL / FTS_E_IPA_LEN (deferred: reported only if E1 holds).
// Every slot is written once: the proof's point, or the filler where the proof has
// none (nil element, unslotted IPA arrays, or a rejected proof) -- the records go
// straight to pinned staging memory, where a filler pass before the copy would double
// the bytes written per proof.
inline void parse_range_proof(der::Span rp, int k, uint8_t* pts, uint32_t* sc, int32_t& status, int32_t& ipa_flag) {
  status = 0;
  ipa_flag = 0;
  const int npts = 5 + 2 * k;
  memset(sc, 0, 5 * 32);
  bool data_pts = false, ipa_pts = false;  // slots 0-3 / 5.. written
  auto reject = [&]() {
    for (int j = 0; j < npts; j++)
      if (j != 4) filler_point(pts + j * 64);
    status = FTS_E_MALFORMED;
  };
  // per-thread reused buffers: the host pool parses thousands of proofs per call
  thread_local std::vector<der::Span> vals, ubuf, Ls, Rs;
  if (!der::unmarshal_values(rp, vals) || vals.size() != 2) return reject();
  bool nil = false;
  // ---- RangeProofData (bulletproof.go:49-83)
  if (vals[0].n == 0) {
    nil = true;
  } else {
    Unmarshaller u(vals[0], ubuf);
    if (!u.ok) return reject();
    // order T1, T2, Tau, C, D, Delta, IP ; kinds: 0 = G1 slot, 1 = Zr slot
    const int kind[7] = {0, 0, 1, 0, 0, 1, 1};
    const int slot[7] = {0, 1, 0, 2, 3, 1, 2};  // pt slot or scalar slot (Tau=0, Delta=1, IP=2)
    data_pts = true;
    for (int f = 0; f < 7; f++) {
      Elem e;
      if (!u.next(e)) return reject();
      if (!e.present) {
        nil = true;
        if (kind[f] == 0) filler_point(pts + slot[f] * 64);
        continue;
      }
      if (kind[f] == 0) {
        if (e.raw.n != 64) return reject();
        memcpy(pts + slot[f] * 64, e.raw.p, 64);
      } else {
        scalar_from_bytes(e.raw, sc + slot[f] * 8, nullptr);
      }
    }
  }
  if (!data_pts)
    for (int j = 0; j < 4; j++) filler_point(pts + j * 64);
  // ---- IPA (ipa.go:45-67)
  if (vals[1].n == 0) {
    ipa_flag = FTS_E_IPA_NIL;
  } else {
    Unmarshaller u(vals[1], ubuf);
    if (!u.ok) return reject();
    Elem eL, eR, aL, aR;
    if (!u.next(eL) || !u.next(eR) || !u.next(aL) || !u.next(aR)) return reject();
    if (eL.present) scalar_from_bytes(eL.raw, sc + 3 * 8, nullptr);
    if (eR.present) scalar_from_bytes(eR.raw, sc + 4 * 8, nullptr);
    Ls.clear();
    Rs.clear();
    if (aL.present && !der::unmarshal_values(aL.raw, Ls, true)) return reject();
    if (aR.present && !der::unmarshal_values(aR.raw, Rs, true)) return reject();
    for (auto& s : Ls)
      if (s.n != 64) return reject();
    for (auto& s : Rs)
      if (s.n != 64) return reject();
    if (!eL.present || !eR.present) {
      ipa_flag = FTS_E_IPA_NIL;
    } else if (Ls.size() != Rs.size() || (int)Ls.size() != k) {
      ipa_flag = FTS_E_IPA_LEN;
    }
    if (ipa_flag == 0) {
      ipa_pts = true;
      for (int j = 0; j < k; j++) {
        memcpy(pts + (5 + j) * 64, Ls[j].p, 64);
        memcpy(pts + (5 + k + j) * 64, Rs[j].p, 64);
      }
    } else {
      // unslotted points still have to decode (deserialization precedes verification)
      G1A tmp;
      for (auto& s : Ls)
        if (!g1_from_bytes(s.p, 64, tmp)) return reject();
      for (auto& s : Rs)
        if (!g1_from_bytes(s.p, 64, tmp)) return reject();
    }
  }
  if (!ipa_pts)
    for (int j = 5; j < npts; j++) filler_point(pts + j * 64);
  if (nil) status = FTS_E_RP_NIL;
}

// Parse a RangeCorrectness (rangecorrectness.go:27-40): list of RangeProof DERs.
inline bool parse_range_correctness(der::Span raw, std::vector<der::Span>& proofs) {
  thread_local std::vector<der::Span> outer;  // reused (the host pool parses thousands per call)
  if (!der::unmarshal_values(raw, outer) || outer.size() != 1) return false;
  proofs.clear();
  if (outer[0].n == 0) return true;
  return der::unmarshal_values(outer[0], proofs);
}

// ----------------------------------------------------------------- encode
inline std::string g1_raw(const G1A& p) {
  uint8_t b[64];
  g1_to_bytes(p, b);
  return std::string((const char*)b, 64);
}
inline std::string fr_raw(const Fr& z) {
  uint8_t b[32];
  fr_to_be(z, b);
  return std::string((const char*)b, 32);
}
inline std::string el_g1(const G1A& p) { return der::element(1, g1_raw(p)); }
inline std::string el_fr(const Fr& z) { return der::element(1, fr_raw(z)); }
inline std::string el_g1_array(const std::vector<G1A>& v) {
  std::vector<std::string> items;
  for (auto& p : v) items.push_back(g1_raw(p));
  return der::element(1, der::values(items));
}
inline std::string el_fr_array(const std::vector<Fr>& v) {
  std::vector<std::string> items;
  for (auto& z : v) items.push_back(fr_raw(z));
  return der::element(1, der::values(items));
}

}  // namespace host
}  // namespace fts
