// Raw TokenRequest ingest: the deserialisation and
// structural checks VerifyTokenRequestFromRaw performs before the ZK proofs.
//
//   TokenRequest  driver/protos/request.proto:95-100 (version=1, actions=2,
//                 signatures=3, auditor_signatures=4; Action{type=1, raw=2},
//                 Signature{raw=1}); decoded by TokenRequest.FromBytes /
//                 FromProtos (driver/request.go:46-95)
//   actions       nogh/protos/noghactions.proto (TransferAction, IssueAction,
//                 Token{owner=1, data=2 G1}, TokenID{id=1, index=2}, ...);
//                 decoded by transfer Action.Deserialize
//                 (crypto/transfer/action.go:76-111,326-362) and issue
//                 Action.Deserialize (crypto/issue/action.go:38-45,231-270)
//   order         ActionDeserializer.DeserializeActions: every issue, then every
//                 transfer (validator/validator.go:27-47); VerifyTokenRequest
//                 verifies issues first, then transfers (core/common/validator.go:112-130)
//   structure     issue Action.Validate (crypto/issue/action.go:161-185) +
//                 GetCommitments (:273-282); transfer Action.Validate
//                 (crypto/transfer/action.go:244-283) + Token.Validate
//                 (crypto/token/token.go:85-93)
//
// Wire semantics follow protobuf-go: a field whose wire type does not match
// its declaration is kept as an unknown field (skipped), a singular scalar or
// bytes field appearing twice keeps the last value, a singular message field
// appearing twice is merged (parsed as the concatenation of its occurrences),
// proto3 `string` fields must be valid UTF-8, field number 0 / > 2^29-1 and
// group wire types are errors.  Host-only (no HIP): linked into libfts_gpu and
// callable without a device (fts_request_inspect).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>
#include "../../../include/fts_gpu.h"
#include "pp_parse.hpp"

namespace fts {
namespace host {
namespace req {

struct Field {
  uint32_t no, wt;
  uint64_t v;
  const uint8_t* p;
  size_t n;
};

// one protobuf message -> its fields in wire order (protobuf-go's decoder errors)
inline bool fields(const uint8_t* b, size_t len, std::vector<Field>& out) {
  out.clear();
  size_t i = 0;
  while (i < len) {
    uint64_t key;
    if (!pb_varint(b, len, i, key)) return false;
    const uint64_t no = key >> 3;
    if (no == 0 || no > 0x1FFFFFFFull) return false;
    Field f{(uint32_t)no, (uint32_t)(key & 7), 0, nullptr, 0};
    if (f.wt == 0) {
      if (!pb_varint(b, len, i, f.v)) return false;
    } else if (f.wt == 2) {
      uint64_t l;
      if (!pb_varint(b, len, i, l) || l > len - i) return false;
      f.p = b + i;
      f.n = (size_t)l;
      i += (size_t)l;
    } else if (f.wt == 1) {
      if (len - i < 8) return false;
      i += 8;
    } else if (f.wt == 5) {
      if (len - i < 4) return false;
      i += 4;
    } else {
      return false;  // groups (3/4) and reserved wire types
    }
    out.push_back(f);
  }
  return true;
}

// Go's utf8.Valid (no overlongs, no surrogates, <= U+10FFFF)
inline bool utf8_valid(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    int len;
    uint32_t cp, min;
    if ((c & 0xE0) == 0xC0) len = 2, cp = c & 0x1F, min = 0x80;
    else if ((c & 0xF0) == 0xE0) len = 3, cp = c & 0x0F, min = 0x800;
    else if ((c & 0xF8) == 0xF0) len = 4, cp = c & 0x07, min = 0x10000;
    else return false;
    if (n - i < (size_t)len) return false;
    for (int k = 1; k < len; k++) {
      if ((s[i + k] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (s[i + k] & 0x3F);
    }
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    i += len;
  }
  return true;
}

// A singular sub-message: every occurrence of field `no` with wire type 2,
// merged (protobuf-go MergeFrom == parsing the concatenation).
struct Sub {
  Sub() = default;
  Sub(const Sub&) = delete;  // p may point into merged
  bool present = false;
  std::string merged;
  const uint8_t* p = nullptr;
  size_t n = 0;
  int count = 0;
  void add(const Field& f) {
    present = true;
    if (count++ == 0) {
      p = f.p, n = f.n;
    } else {
      if (count == 2) merged.assign((const char*)p, n);
      merged.append((const char*)f.p, f.n);
      p = (const uint8_t*)merged.data(), n = merged.size();
    }
  }
};

// last occurrence of a singular bytes/string field (wire type 2)
struct Bytes {
  bool present = false;
  const uint8_t* p = nullptr;
  size_t n = 0;
  void set(const Field& f) { present = true, p = f.p, n = f.n; }
};

// message with `bytes raw = 1` (G1, Zr, Identity, Signature, Proof{proof=1})
inline bool raw_field(const uint8_t* b, size_t n, Bytes& raw) {
  std::vector<Field> f;
  if (!fields(b, n, f)) return false;
  for (auto& x : f)
    if (x.no == 1 && x.wt == 2) raw.set(x);
  return true;
}

// mathlib G1.UnmarshalJSON on a nogh.G1's raw (FromG1Proto, protos-go/utils/proto.go:39-49):
// nil message or empty raw -> nil point (has = false)
inline bool g1_field(const Sub& g, bool& has, uint8_t out[64]) {
  has = false;
  if (!g.present) return true;
  Bytes raw;
  if (!raw_field(g.p, g.n, raw)) return false;
  if (!raw.n) return true;
  std::string js((const char*)raw.p, raw.n), el, bin;
  long long curve = -1;
  if (!json_int_field(js, "curve", curve) || curve != 1) return false;
  if (!json_string_field(js, "element", el) || !b64_decode(el, bin)) return false;
  G1A a;
  if (!g1_from_bytes((const uint8_t*)bin.data(), bin.size(), a)) return false;
  memcpy(out, bin.data(), 64);
  has = true;
  return true;
}

// FromZrProto (proto.go:62-72): non-nil message -> Zr.UnmarshalJSON(raw), even when raw is empty.
// mathlib's Zr JSON is {"curve":id,"element":base64}; the element is read as a big-endian
// integer, so only the JSON shape is checked here (parity unpinned beyond that shape).
inline bool zr_field(const Sub& z) {
  if (!z.present) return true;
  Bytes raw;
  if (!raw_field(z.p, z.n, raw)) return false;
  std::string js((const char*)raw.p, raw.n), el, bin;
  long long curve = -1;
  return json_int_field(js, "curve", curve) && json_string_field(js, "element", el) && b64_decode(el, bin);
}

// nogh.TokenID / fabtoken.Token / map<string,bytes> entries: the UTF-8 checks of proto3 strings
inline bool token_id_ok(const Sub& id, bool& txid_nonempty) {
  txid_nonempty = false;
  if (!id.present) return true;
  std::vector<Field> f;
  if (!fields(id.p, id.n, f)) return false;
  Bytes s;
  for (auto& x : f)
    if (x.no == 1 && x.wt == 2) {
      if (!utf8_valid(x.p, x.n)) return false;
      s.set(x);
    }
  txid_nonempty = s.n > 0;
  return true;
}
inline bool map_entry_ok(const Field& e) {  // map<string, bytes>: key = 1
  std::vector<Field> f;
  if (!fields(e.p, e.n, f)) return false;
  for (auto& x : f)
    if (x.no == 1 && x.wt == 2 && !utf8_valid(x.p, x.n)) return false;
  return true;
}
inline bool fabtoken_ok(const Sub& t) {  // fabtoken.Token{owner=1 bytes, type=2 string, quantity=3 string}
  if (!t.present) return true;
  std::vector<Field> f;
  if (!fields(t.p, t.n, f)) return false;
  for (auto& x : f)
    if ((x.no == 2 || x.no == 3) && x.wt == 2 && !utf8_valid(x.p, x.n)) return false;
  return true;
}

// nogh.Token{owner=1, data=2}
struct Tok {
  bool present = false, has_data = false;
  size_t owner_len = 0;
  uint8_t data[64];
};
inline bool token_msg(const Sub& s, Tok& t) {
  t = Tok{};
  if (!s.present) return true;
  t.present = true;
  std::vector<Field> f;
  if (!fields(s.p, s.n, f)) return false;
  Bytes owner;
  Sub data;
  for (auto& x : f) {
    if (x.wt != 2) continue;
    if (x.no == 1) owner.set(x);
    else if (x.no == 2) data.add(x);
  }
  t.owner_len = owner.n;
  return g1_field(data, t.has_data, t.data);
}

static const uint8_t kZero64[64] = {0};

// one action of a request, in reference verification order
struct Action {
  int kind = 0;                 // SIG_TAS (transfer) / SIG_ST (issue) numbering of the caller
  int index = -1;               // position in TokenRequest.actions
  bool transfer = false;
  std::string in, out;          // input / output commitments, 64-byte raw points
  size_t n_in = 0, n_out = 0;
  std::string proof;            // Proof.proof bytes (owned: a merged Proof message is a temporary)
  int32_t pre = -1;             // verdict decided before the ZK proof (FTS_E_ACTION_INVALID / FTS_E_MALFORMED)
};

struct Request {
  int32_t status = FTS_OK;      // request-level verdict (FTS_E_MALFORMED) when fail_action < 0 or deserialisation
  int32_t fail_action = -1;
  bool deser_failed = false;
  std::vector<Action> acts;     // issues (request order), then transfers (request order)
};

// transfer Action.Deserialize + Validate (transfer/action.go:326-362, 244-283)
inline bool transfer_action(const uint8_t* b, size_t n, Action& a) {
  std::vector<Field> f;
  if (!fields(b, n, f)) return false;
  Sub proof;
  bool invalid = false;
  for (auto& x : f) {
    if (x.wt != 2) continue;
    if (x.no == 1) {  // TransferActionInput
      std::vector<Field> g;
      if (!fields(x.p, x.n, g)) return false;
      Sub id, input, wit;
      for (auto& y : g) {
        if (y.wt != 2) continue;
        if (y.no == 1) id.add(y);
        else if (y.no == 2) input.add(y);
        else if (y.no == 3) wit.add(y);
      }
      bool txid;
      if (!token_id_ok(id, txid)) return false;
      Tok t;
      if (!token_msg(input, t)) return false;
      if (wit.present) {  // FromZrProto on the blinding factor; fabtoken strings
        std::vector<Field> w;
        if (!fields(wit.p, wit.n, w)) return false;
        Sub out, bf;
        for (auto& y : w) {
          if (y.wt != 2) continue;
          if (y.no == 1) out.add(y);
          else if (y.no == 2) bf.add(y);
        }
        if (!fabtoken_ok(out) || !zr_field(bf)) return false;
      }
      // Validate: ID set, tx id non-empty, token set, owner non-empty, data set (:248-263)
      if (!id.present || !txid || !t.present || !t.owner_len || !t.has_data) invalid = true;
      a.in.append((const char*)(t.has_data ? t.data : kZero64), 64);
      a.n_in++;
    } else if (x.no == 2) {  // TransferActionOutput{token=1}
      std::vector<Field> g;
      if (!fields(x.p, x.n, g)) return false;
      Sub tok;
      for (auto& y : g)
        if (y.no == 1 && y.wt == 2) tok.add(y);
      Tok t;
      if (!token_msg(tok, t)) return false;
      if (!t.present || !t.has_data) invalid = true;  // nil output / Token.Validate(false) (:274-280)
      a.out.append((const char*)(t.has_data ? t.data : kZero64), 64);
      a.n_out++;
    } else if (x.no == 3) {
      proof.add(x);
    } else if (x.no == 4) {
      if (!map_entry_ok(x)) return false;
    }
  }
  if (proof.present) {
    Bytes pb;
    std::vector<Field> g;
    if (!fields(proof.p, proof.n, g)) return false;
    for (auto& y : g)
      if (y.no == 1 && y.wt == 2) pb.set(y);
    a.proof.assign((const char*)pb.p, pb.n);
  }
  if (a.n_in == 0 || a.n_out == 0) invalid = true;  // (:245-247, :271-273)
  if (invalid) a.pre = FTS_E_ACTION_INVALID;
  return true;
}

// issue Action.Deserialize + Validate + GetCommitments (issue/action.go:231-270, 161-185, 273-282)
inline bool issue_action(const uint8_t* b, size_t n, Action& a) {
  std::vector<Field> f;
  if (!fields(b, n, f)) return false;
  Sub issuer, proof;
  bool invalid = false, nil_data = false;
  for (auto& x : f) {
    if (x.wt != 2) continue;
    if (x.no == 1) {
      issuer.add(x);
    } else if (x.no == 2) {  // IssueActionInput{id=1 TokenID, token=2 bytes}
      std::vector<Field> g;
      if (!fields(x.p, x.n, g)) return false;
      Sub id;
      Bytes tok;
      for (auto& y : g) {
        if (y.wt != 2) continue;
        if (y.no == 1) id.add(y);
        else if (y.no == 2) tok.set(y);
      }
      bool txid;
      if (!token_id_ok(id, txid)) return false;
      if (!tok.n || !txid) invalid = true;  // (:169-174)
    } else if (x.no == 3) {  // IssueActionOutput{token=1}
      std::vector<Field> g;
      if (!fields(x.p, x.n, g)) return false;
      Sub tok;
      for (auto& y : g)
        if (y.no == 1 && y.wt == 2) tok.add(y);
      Tok t;
      if (!token_msg(tok, t)) return false;
      if (!t.present) invalid = true;  // nil output (:179-183)
      else if (!t.has_data) nil_data = true;
      a.out.append((const char*)(t.has_data ? t.data : kZero64), 64);
      a.n_out++;
    } else if (x.no == 4) {
      proof.add(x);
    } else if (x.no == 5) {
      if (!map_entry_ok(x)) return false;
    }
  }
  Bytes iraw;
  if (issuer.present && !raw_field(issuer.p, issuer.n, iraw)) return false;
  if (proof.present) {
    Bytes pb;
    if (!raw_field(proof.p, proof.n, pb)) return false;
    a.proof.assign((const char*)pb.p, pb.n);
  }
  if (!iraw.n || a.n_out == 0) invalid = true;  // issuer not set (:162-164), no outputs (:176-178)
  if (invalid) a.pre = FTS_E_ACTION_INVALID;
  // a nil commitment reaches the verifier, which dereferences it (issue/verifier.go): a panic
  else if (nil_data) a.pre = FTS_E_MALFORMED;
  return true;
}

// TokenRequest.FromBytes + DeserializeActions + the per-action structural checks.
// The returned Request either carries a final verdict (status != FTS_OK, e.g.
// MALFORMED with the failing action's index), or the action list whose ZK
// proofs decide the verdict (first failing action in acts order).
inline void parse_request(const uint8_t* b, size_t n, int kind_transfer, int kind_issue, Request& r) {
  r = Request{};
  auto fail = [&](int32_t st, int32_t idx) {
    r.status = st;
    r.fail_action = idx;
    r.deser_failed = true;
    r.acts.clear();
  };
  if (n == 0) return fail(FTS_E_MALFORMED, -1);  // "empty token request" (validator.go:79-81)
  std::vector<Field> f;
  if (!fields(b, n, f)) return fail(FTS_E_MALFORMED, -1);
  struct Raw {
    int index;
    bool transfer;
    const uint8_t* p;
    size_t n;
  };
  std::vector<Raw> issues, transfers;
  // proto.Unmarshal of the request (Action / Signature messages included) fails first ...
  int idx = 0, unknown = -1;
  bool nil_sig = false;
  for (auto& x : f) {
    if (x.wt != 2) continue;
    if (x.no == 2) {  // Action{type=1 enum, raw=2 bytes}
      std::vector<Field> g;
      if (!fields(x.p, x.n, g)) return fail(FTS_E_MALFORMED, -1);
      int32_t type = 0;
      Bytes raw;
      for (auto& y : g) {
        if (y.no == 1 && y.wt == 0) type = (int32_t)(uint32_t)y.v;
        else if (y.no == 2 && y.wt == 2) raw.set(y);
      }
      if (type == 0) issues.push_back(Raw{idx, false, raw.p, raw.n});
      else if (type == 1) transfers.push_back(Raw{idx, true, raw.p, raw.n});
      else if (unknown < 0) unknown = idx;
      idx++;
    } else if (x.no == 3 || x.no == 4) {  // Signature{raw=1}
      Bytes raw;
      if (!raw_field(x.p, x.n, raw)) return fail(FTS_E_MALFORMED, -1);
      nil_sig |= !raw.n;
    }
  }
  // ... then FromProtos: unknown action type (request.go:73-80), nil / empty signature (:82-93)
  if (unknown >= 0) return fail(FTS_E_MALFORMED, unknown);
  if (nil_sig) return fail(FTS_E_MALFORMED, -1);
  r.acts.reserve(issues.size() + transfers.size());
  for (int pass = 0; pass < 2; pass++)
    for (const Raw& w : pass == 0 ? issues : transfers) {
      Action a;
      a.index = w.index;
      a.transfer = w.transfer;
      a.kind = w.transfer ? kind_transfer : kind_issue;
      bool ok = w.transfer ? transfer_action(w.p, w.n, a) : issue_action(w.p, w.n, a);
      if (!ok) return fail(FTS_E_MALFORMED, w.index);  // "failed to unmarshal actions"
      r.acts.push_back(std::move(a));
    }
}

}  // namespace req
}  // namespace host
}  // namespace fts
