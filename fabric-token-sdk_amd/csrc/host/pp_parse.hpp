// Public-parameter parsing: PublicParams.Deserialize (crypto/setup.go:319-372).
//   container JSON {"identifier": "zkatdlog", "raw": base64}  (core/common/encoding/pp/pp.go:16-30)
//   raw = protobuf nogh.PublicParameters                      (nogh/protos/noghpp.proto:25-44)
//   G1  = protobuf nogh.G1{raw = mathlib JSON {"curve":1,"element":base64(64 B)}}
//                                                             (nogh/protos-go/utils/proto.go:22-50)
// and the checks of PublicParams.Validate / RangeProofParams.Validate
// (setup.go:444-489, :47-78) that matter for the verifier.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>
#include "bn254_host.hpp"

namespace fts {
namespace host {

struct PublicParams {
  std::string identifier, version;
  uint64_t curve_id = 0;
  std::vector<G1A> ped;            // PedersenGenerators (3)
  std::vector<G1A> left, right;    // RangeProofParams generators
  G1A P{}, Q{};
  bool hasP = false, hasQ = false;
  uint64_t bit_length = 0, rounds = 0, max_token = 0, precision = 0;
};

// minimal JSON: value of a top-level string field ("key": "value"); false if absent
inline bool json_string_field(const std::string& js, const std::string& key, std::string& out) {
  std::string pat = "\"" + key + "\"";
  size_t p = js.find(pat);
  if (p == std::string::npos) return false;
  p = js.find(':', p + pat.size());
  if (p == std::string::npos) return false;
  p = js.find('"', p);
  if (p == std::string::npos) return false;
  size_t e = p + 1;
  out.clear();
  while (e < js.size() && js[e] != '"') {
    if (js[e] == '\\' && e + 1 < js.size()) {
      char c = js[e + 1];
      if (c == '/' || c == '\\' || c == '"') out.push_back(c);
      else return false;
      e += 2;
      continue;
    }
    out.push_back(js[e++]);
  }
  return e < js.size();
}
inline bool json_int_field(const std::string& js, const std::string& key, long long& out) {
  std::string pat = "\"" + key + "\"";
  size_t p = js.find(pat);
  if (p == std::string::npos) return false;
  p = js.find(':', p + pat.size());
  if (p == std::string::npos) return false;
  p++;
  while (p < js.size() && (js[p] == ' ' || js[p] == '\t' || js[p] == '\n')) p++;
  size_t e = p;
  while (e < js.size() && (isdigit((unsigned char)js[e]) || js[e] == '-')) e++;
  if (e == p) return false;
  out = atoll(js.substr(p, e - p).c_str());
  return true;
}

inline bool b64_decode(const std::string& in, std::string& out) {
  struct Tbl {
    int8_t v[256];
    Tbl() {
      for (int i = 0; i < 256; i++) v[i] = -1;
      const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
      for (int i = 0; i < 64; i++) v[(uint8_t)a[i]] = (int8_t)i;
    }
  };
  static const Tbl T;  // thread-safe one-time init (request ingest decodes on many threads)
  const int8_t* tbl = T.v;
  out.clear();
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    if (c == '=') break;
    if (c == '\n' || c == '\r') continue;
    int v = tbl[(uint8_t)c];
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((char)((acc >> bits) & 0xff));
    }
  }
  return true;
}

struct PbField {
  uint32_t no, wt;
  uint64_t v;
  const uint8_t* p;
  size_t n;
};
inline bool pb_varint(const uint8_t* b, size_t len, size_t& i, uint64_t& v) {
  v = 0;
  for (int s = 0; s < 64; s += 7) {
    if (i >= len) return false;
    uint8_t c = b[i++];
    v |= (uint64_t)(c & 0x7f) << s;
    if (!(c & 0x80)) return true;
  }
  return false;
}
inline bool pb_fields(const uint8_t* b, size_t len, std::vector<PbField>& out) {
  out.clear();
  size_t i = 0;
  while (i < len) {
    uint64_t key;
    if (!pb_varint(b, len, i, key)) return false;
    PbField f{(uint32_t)(key >> 3), (uint32_t)(key & 7), 0, nullptr, 0};
    if (f.wt == 0) {
      if (!pb_varint(b, len, i, f.v)) return false;
    } else if (f.wt == 2) {
      uint64_t l;
      if (!pb_varint(b, len, i, l) || l > len - i) return false;
      f.p = b + i;
      f.n = (size_t)l;
      i += (size_t)l;
    } else if (f.wt == 1) {
      if (i + 8 > len) return false;
      i += 8;
    } else if (f.wt == 5) {
      if (i + 4 > len) return false;
      i += 4;
    } else {
      return false;
    }
    out.push_back(f);
  }
  return true;
}

// nogh.G1 message -> point (mathlib G1.UnmarshalJSON); empty -> nil (ok=false)
inline bool g1_from_proto(const uint8_t* b, size_t n, G1A& out, std::string& err) {
  std::vector<PbField> f;
  if (!pb_fields(b, n, f)) {
    err = "bad G1 proto";
    return false;
  }
  for (auto& x : f)
    if (x.no == 1 && x.wt == 2) {
      std::string js((const char*)x.p, x.n), el, raw;
      long long curve = -1;
      if (!json_int_field(js, "curve", curve) || curve != 1) {
        err = "unsupported curve in G1";
        return false;
      }
      if (!json_string_field(js, "element", el) || !b64_decode(el, raw)) {
        err = "bad G1 json";
        return false;
      }
      if (!g1_from_bytes((const uint8_t*)raw.data(), raw.size(), out)) {
        err = "invalid G1 element";
        return false;
      }
      return true;
    }
  err = "nil G1";
  return false;
}

inline bool parse_public_params(const uint8_t* data, size_t len, PublicParams& pp, std::string& err) {
  std::string js((const char*)data, len), ident, rawb64, raw;
  if (!json_string_field(js, "identifier", ident) || !json_string_field(js, "raw", rawb64)) {
    err = "failed to deserialize public parameters";
    return false;
  }
  if (ident != "zkatdlog") {
    err = "invalid identifier, expecting [zkatdlog], got [" + ident + "]";
    return false;
  }
  if (!b64_decode(rawb64, raw)) {
    err = "bad base64";
    return false;
  }
  std::vector<PbField> f;
  if (!pb_fields((const uint8_t*)raw.data(), raw.size(), f)) {
    err = "failed unmarshalling public parameters";
    return false;
  }
  bool have_curve = false;
  for (auto& x : f) {
    if (x.no == 1 && x.wt == 2) pp.identifier.assign((const char*)x.p, x.n);
    else if (x.no == 2 && x.wt == 2) pp.version.assign((const char*)x.p, x.n);
    else if (x.no == 3 && x.wt == 2) {
      std::vector<PbField> c;
      if (!pb_fields(x.p, x.n, c)) return err = "bad curve id", false;
      pp.curve_id = 0;
      for (auto& y : c)
        if (y.no == 1 && y.wt == 0) pp.curve_id = y.v;
      have_curve = true;
    } else if (x.no == 4 && x.wt == 2) {
      G1A g;
      if (!g1_from_proto(x.p, x.n, g, err)) return false;
      pp.ped.push_back(g);
    } else if (x.no == 5 && x.wt == 2) {
      std::vector<PbField> r;
      if (!pb_fields(x.p, x.n, r)) return err = "bad range proof params", false;
      for (auto& y : r) {
        G1A g;
        if (y.no >= 1 && y.no <= 4 && y.wt == 2) {
          if (!g1_from_proto(y.p, y.n, g, err)) return false;
          if (y.no == 1) pp.left.push_back(g);
          if (y.no == 2) pp.right.push_back(g);
          if (y.no == 3) pp.P = g, pp.hasP = true;
          if (y.no == 4) pp.Q = g, pp.hasQ = true;
        } else if (y.no == 5 && y.wt == 0) {
          pp.bit_length = y.v;
        } else if (y.no == 6 && y.wt == 0) {
          pp.rounds = y.v;
        }
      }
    } else if (x.no == 9 && x.wt == 0) {
      pp.max_token = x.v;
    } else if (x.no == 10 && x.wt == 0) {
      pp.precision = x.v;
    }
  }
  if (!have_curve) return err = "invalid curve id, expecting curve id, got nil", false;
  if (pp.curve_id != 1) return err = "unsupported curve (only BN254 = 1)", false;
  // Validate (setup.go:444-489) - the parts that constrain the verifier
  if (pp.ped.size() != 3) return err = "invalid pedersen generators", false;
  for (auto& g : pp.ped)
    if (g.inf) return err = "invalid pedersen generators: element is infinity", false;
  if (!pp.hasP || !pp.hasQ || pp.P.inf || pp.Q.inf) return err = "invalid range proof parameters: P/Q", false;
  if (pp.rounds == 0 || pp.rounds > 64 || pp.bit_length != (1ULL << pp.rounds))
    return err = "invalid range proof parameters: bit length / rounds", false;
  if (pp.left.size() != pp.bit_length || pp.right.size() != pp.bit_length)
    return err = "invalid range proof parameters: generator count", false;
  for (size_t i = 0; i < pp.left.size(); i++)
    if (pp.left[i].inf || pp.right[i].inf) return err = "invalid range proof parameters: infinity", false;
  return true;
}

}  // namespace host
}  // namespace fts
