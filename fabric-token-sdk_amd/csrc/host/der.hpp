// DER reader/writer for the proof wire format.
//
// Mirrors the Go encoding/asn1 behaviour the reference relies on
// (token/core/common/encoding/asn1/asn1.go):
//   Values  = SEQUENCE { SEQUENCE OF OCTET STRING }   (:27-29)
//   Element = SEQUENCE { INTEGER curveID, OCTET STRING raw }   (:31-34)
// * asn1.Unmarshal ignores bytes after the outer TLV, and extra elements at
//   the end of a SEQUENCE decoded into a struct (Go "allow extra bytes").
// * unmarshaller.Next / NextG1Array reject trailing bytes (:168-174, :214-220).
// * lengths must be definite and minimal; INTEGERs minimally encoded.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace fts {
namespace der {

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

// one TLV at b[i..]; returns false on malformed input
inline bool read_tlv(const uint8_t* b, size_t len, size_t& i, uint8_t& tag, Span& content) {
  if (i + 2 > len) return false;
  tag = b[i];
  if ((tag & 0x1f) == 0x1f) return false;
  size_t l = b[i + 1];
  i += 2;
  if (l & 0x80) {
    size_t nb = l & 0x7f;
    if (nb == 0 || nb > 4 || i + nb > len) return false;
    if (b[i] == 0) return false;
    l = 0;
    for (size_t k = 0; k < nb; k++) l = (l << 8) | b[i + k];
    i += nb;
    if (l < 0x80) return false;
  }
  if (l > len - i) return false;
  content.p = b + i;
  content.n = l;
  i += l;
  return true;
}

// SEQUENCE OF OCTET STRING content -> items
inline bool parse_octets(Span c, std::vector<Span>& out) {
  size_t i = 0;
  out.clear();
  while (i < c.n) {
    uint8_t t;
    Span s;
    if (!read_tlv(c.p, c.n, i, t, s) || t != 0x04) return false;
    out.push_back(s);
  }
  return true;
}

// asn1.Unmarshal(raw, &Values{}) ; strict => no trailing bytes after outer TLV
inline bool unmarshal_values(Span raw, std::vector<Span>& out, bool strict = false) {
  size_t i = 0;
  uint8_t t;
  Span c;
  if (!read_tlv(raw.p, raw.n, i, t, c) || t != 0x30) return false;
  if (strict && i != raw.n) return false;
  if (c.n == 0) return false;  // sequence truncated (field Values missing)
  size_t j = 0;
  Span inner;
  if (!read_tlv(c.p, c.n, j, t, inner) || t != 0x30) return false;
  return parse_octets(inner, out);
}

// asn1.Unmarshal(raw, &Element{}) with unmarshaller.Next's trailing check
inline bool unmarshal_element(Span raw, int64_t& curve, Span& elem) {
  size_t i = 0;
  uint8_t t;
  Span c;
  if (!read_tlv(raw.p, raw.n, i, t, c) || t != 0x30 || i != raw.n) return false;
  size_t j = 0;
  Span ci;
  if (!read_tlv(c.p, c.n, j, t, ci) || t != 0x02 || ci.n == 0 || ci.n > 8) return false;
  if (ci.n > 1 && ((ci.p[0] == 0 && ci.p[1] < 0x80) || (ci.p[0] == 0xff && ci.p[1] >= 0x80))) return false;
  int64_t v = (ci.p[0] & 0x80) ? -1 : 0;
  for (size_t k = 0; k < ci.n; k++) v = (int64_t)(((uint64_t)v << 8) | ci.p[k]);
  curve = v;
  if (!read_tlv(c.p, c.n, j, t, elem) || t != 0x04) return false;
  return true;
}

// ------------------------------------------------------------------ writer
inline void put_len(std::string& o, size_t n) {
  if (n < 0x80) {
    o.push_back((char)n);
    return;
  }
  uint8_t b[8];
  int k = 0;
  while (n) {
    b[k++] = (uint8_t)(n & 0xff);
    n >>= 8;
  }
  o.push_back((char)(0x80 | k));
  while (k) o.push_back((char)b[--k]);
}
inline std::string tlv(uint8_t tag, const std::string& c) {
  std::string o;
  o.push_back((char)tag);
  put_len(o, c.size());
  o += c;
  return o;
}
inline std::string octet(const uint8_t* p, size_t n) { return tlv(0x04, std::string((const char*)p, n)); }
inline std::string octet(const std::string& s) { return tlv(0x04, s); }
inline std::string values(const std::vector<std::string>& items) {
  std::string inner;
  for (auto& s : items) inner += octet(s);
  return tlv(0x30, tlv(0x30, inner));
}
inline std::string seq_of_octets(const std::vector<std::string>& items) {
  std::string inner;
  for (auto& s : items) inner += octet(s);
  return tlv(0x30, inner);
}
inline std::string element(int curve, const std::string& raw) {
  std::string in;
  in.push_back(0x02);
  in.push_back(0x01);
  in.push_back((char)curve);
  in += octet(raw);
  return tlv(0x30, in);
}

}  // namespace der
}  // namespace fts
