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
#include <string.h>
#include <deque>
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

// Walk one protobuf message field by field (protobuf-go's decoder errors):
// fn(const Field&) -> bool; false from fn or a wire error ends the walk with false.
template <class Fn>
inline bool each(const uint8_t* b, size_t len, Fn&& fn) {
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
    if (!fn(f)) return false;
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

// A singular sub-message: every occurrence (wire type 2) merged -- protobuf-go
// MergeFrom == parsing the concatenation; the bytes are copied only when the
// field occurs more than once.
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
  return each(b, n, [&](const Field& x) {
    if (x.no == 1 && x.wt == 2) raw.set(x);
    return true;
  });
}

// mathlib's own encoding of a G1 (json.Marshal of {Curve, Element []byte}):
// {"curve":1,"element":"<88 base64 chars>"} -- decoded without allocations;
// any other spelling goes through the general JSON path below.
inline bool g1_json_fast(const uint8_t* s, size_t n, uint8_t out[64], bool& ok) {
  static const char pre[] = "{\"curve\":1,\"element\":\"";
  const size_t lp = sizeof(pre) - 1;
  if (n != lp + 88 + 2 || memcmp(s, pre, lp) || s[n - 2] != '"' || s[n - 1] != '}') return false;
  static const struct T {
    int8_t v[256];
    T() {
      for (int i = 0; i < 256; i++) v[i] = -1;
      const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
      for (int i = 0; i < 64; i++) v[(uint8_t)a[i]] = (int8_t)i;
    }
  } t;
  const uint8_t* e = s + lp;
  if (e[86] != '=' || e[87] != '=') return false;
  uint32_t acc = 0;
  int bits = 0, o = 0;
  for (int i = 0; i < 86; i++) {
    int v = t.v[e[i]];
    if (v < 0) return false;  // general path decides
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out[o++] = (uint8_t)(acc >> bits);
    }
  }
  G1A a;
  ok = o == 64 && g1_from_bytes(out, 64, a);
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
  bool ok;
  if (g1_json_fast(raw.p, raw.n, out, ok)) return has = ok;
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
  Bytes s;
  if (!each(id.p, id.n, [&](const Field& x) {
        if (x.no == 1 && x.wt == 2) {
          if (!utf8_valid(x.p, x.n)) return false;
          s.set(x);
        }
        return true;
      }))
    return false;
  txid_nonempty = s.n > 0;
  return true;
}
inline bool map_entry_ok(const Field& e) {  // map<string, bytes>: key = 1
  return each(e.p, e.n, [](const Field& x) { return !(x.no == 1 && x.wt == 2 && !utf8_valid(x.p, x.n)); });
}
inline bool fabtoken_ok(const Sub& t) {  // fabtoken.Token{owner=1 bytes, type=2 string, quantity=3 string}
  if (!t.present) return true;
  return each(t.p, t.n, [](const Field& x) {
    return !((x.no == 2 || x.no == 3) && x.wt == 2 && !utf8_valid(x.p, x.n));
  });
}

// nogh.Token{owner=1, data=2}
struct Tok {
  bool present = false, has_data = false;
  size_t owner_len = 0;
  uint8_t data[64];
};
inline bool token_msg(const Sub& s, Tok& t) {
  t.present = t.has_data = false;
  t.owner_len = 0;
  if (!s.present) return true;
  t.present = true;
  Bytes owner;
  Sub data;
  if (!each(s.p, s.n, [&](const Field& x) {
        if (x.wt == 2) {
          if (x.no == 1) owner.set(x);
          else if (x.no == 2) data.add(x);
        }
        return true;
      }))
    return false;
  t.owner_len = owner.n;
  return g1_field(data, t.has_data, t.data);
}

static const uint8_t kZero64[64] = {0};

// one action of a request, in reference verification order
struct Action {
  int kind = 0;                 // SIG_TAS (transfer) / SIG_ST (issue) numbering of the caller
  int index = -1;               // position in TokenRequest.actions
  bool transfer = false;
  uint32_t in_off = 0, out_off = 0;  // byte offsets of the commitments in Request::pts
  uint32_t n_in = 0, n_out = 0;
  const uint8_t* proof = nullptr;    // Proof.proof: into the caller's request bytes, or Request::owned
  size_t proof_len = 0;
  int32_t pre = -1;             // verdict decided before the ZK proof (FTS_E_ACTION_INVALID / FTS_E_MALFORMED)
};

struct Request {
  int32_t status = FTS_OK;      // request-level verdict (FTS_E_MALFORMED) when deserialisation fails
  int32_t fail_action = -1;
  bool deser_failed = false;
  std::vector<Action> acts;     // issues (request order), then transfers (request order)
  std::string pts;              // 64-byte raw commitments of every action (inputs, then outputs)
  std::deque<std::string> owned;  // proof bytes of merged Proof messages (stable addresses)
  void reset() {
    status = FTS_OK, fail_action = -1, deser_failed = false;
    acts.clear(), pts.clear(), owned.clear();
  }
  const uint8_t* in(const Action& a) const { return (const uint8_t*)pts.data() + a.in_off; }
  const uint8_t* out(const Action& a) const { return (const uint8_t*)pts.data() + a.out_off; }
};

// Proof{proof = 1}: the last proof bytes of the (merged) message
inline bool proof_msg(const Sub& proof, Request& r, Action& a) {
  if (!proof.present) return true;
  Bytes pb;
  if (!raw_field(proof.p, proof.n, pb)) return false;
  if (proof.count > 1 && pb.n) {  // points into the Sub's temporary merge buffer
    r.owned.emplace_back((const char*)pb.p, pb.n);
    pb.p = (const uint8_t*)r.owned.back().data();
  }
  a.proof = pb.p, a.proof_len = pb.n;
  return true;
}

// transfer Action.Deserialize + Validate (transfer/action.go:326-362, 244-283).
// Inputs are written to r.pts first, outputs after (two walks of the message).
inline bool transfer_action(const uint8_t* b, size_t n, Request& r, Action& a) {
  Sub proof;
  bool invalid = false;
  a.in_off = (uint32_t)r.pts.size();
  Tok t;
  if (!each(b, n, [&](const Field& x) {
        if (x.wt != 2) return true;
        if (x.no == 1) {  // TransferActionInput
          Sub id, input, wit;
          if (!each(x.p, x.n, [&](const Field& y) {
                if (y.wt == 2) {
                  if (y.no == 1) id.add(y);
                  else if (y.no == 2) input.add(y);
                  else if (y.no == 3) wit.add(y);
                }
                return true;
              }))
            return false;
          bool txid;
          if (!token_id_ok(id, txid) || !token_msg(input, t)) return false;
          if (wit.present) {  // FromZrProto on the blinding factor; fabtoken strings
            Sub out, bf;
            if (!each(wit.p, wit.n, [&](const Field& y) {
                  if (y.wt == 2) {
                    if (y.no == 1) out.add(y);
                    else if (y.no == 2) bf.add(y);
                  }
                  return true;
                }))
              return false;
            if (!fabtoken_ok(out) || !zr_field(bf)) return false;
          }
          // Validate: ID set, tx id non-empty, token set, owner non-empty, data set (:248-263)
          if (!id.present || !txid || !t.present || !t.owner_len || !t.has_data) invalid = true;
          r.pts.append((const char*)(t.has_data ? t.data : kZero64), 64);
          a.n_in++;
        } else if (x.no == 3) {
          proof.add(x);
        } else if (x.no == 4) {
          return map_entry_ok(x);
        }
        return true;
      }))
    return false;
  a.out_off = (uint32_t)r.pts.size();
  if (!each(b, n, [&](const Field& x) {
        if (x.wt != 2 || x.no != 2) return true;  // TransferActionOutput{token=1}
        Sub tok;
        if (!each(x.p, x.n, [&](const Field& y) {
              if (y.no == 1 && y.wt == 2) tok.add(y);
              return true;
            }))
          return false;
        if (!token_msg(tok, t)) return false;
        if (!t.present || !t.has_data) invalid = true;  // nil output / Token.Validate(false) (:274-280)
        r.pts.append((const char*)(t.has_data ? t.data : kZero64), 64);
        a.n_out++;
        return true;
      }))
    return false;
  if (!proof_msg(proof, r, a)) return false;
  if (a.n_in == 0 || a.n_out == 0) invalid = true;  // (:245-247, :271-273)
  if (invalid) a.pre = FTS_E_ACTION_INVALID;
  return true;
}

// issue Action.Deserialize + Validate + GetCommitments (issue/action.go:231-270, 161-185, 273-282)
inline bool issue_action(const uint8_t* b, size_t n, Request& r, Action& a) {
  Sub issuer, proof;
  bool invalid = false, nil_data = false;
  a.in_off = a.out_off = (uint32_t)r.pts.size();
  Tok t;
  if (!each(b, n, [&](const Field& x) {
        if (x.wt != 2) return true;
        if (x.no == 1) {
          issuer.add(x);
        } else if (x.no == 2) {  // IssueActionInput{id=1 TokenID, token=2 bytes}
          Sub id;
          Bytes tok;
          if (!each(x.p, x.n, [&](const Field& y) {
                if (y.wt == 2) {
                  if (y.no == 1) id.add(y);
                  else if (y.no == 2) tok.set(y);
                }
                return true;
              }))
            return false;
          bool txid;
          if (!token_id_ok(id, txid)) return false;
          if (!tok.n || !txid) invalid = true;  // (:169-174)
        } else if (x.no == 3) {  // IssueActionOutput{token=1}
          Sub tok;
          if (!each(x.p, x.n, [&](const Field& y) {
                if (y.no == 1 && y.wt == 2) tok.add(y);
                return true;
              }))
            return false;
          if (!token_msg(tok, t)) return false;
          if (!t.present) invalid = true;  // nil output (:179-183)
          else if (!t.has_data) nil_data = true;
          r.pts.append((const char*)(t.has_data ? t.data : kZero64), 64);
          a.n_out++;
        } else if (x.no == 4) {
          proof.add(x);
        } else if (x.no == 5) {
          return map_entry_ok(x);
        }
        return true;
      }))
    return false;
  Bytes iraw;
  if (issuer.present && !raw_field(issuer.p, issuer.n, iraw)) return false;
  if (!proof_msg(proof, r, a)) return false;
  if (!iraw.n || a.n_out == 0) invalid = true;  // issuer not set (:162-164), no outputs (:176-178)
  if (invalid) a.pre = FTS_E_ACTION_INVALID;
  // a nil commitment reaches the verifier, which dereferences it (issue/verifier.go): a panic
  else if (nil_data) a.pre = FTS_E_MALFORMED;
  return true;
}

// TokenRequest.FromBytes + DeserializeActions + the per-action structural checks.
// The returned Request either carries a final verdict (deser_failed: MALFORMED,
// with the failing action's index when one is to blame), or the action list
// whose structural verdicts and ZK proofs decide (first failing action in acts order).
inline void parse_request(const uint8_t* b, size_t n, int kind_transfer, int kind_issue, Request& r) {
  r.reset();
  auto fail = [&](int32_t st, int32_t idx) {
    r.status = st;
    r.fail_action = idx;
    r.deser_failed = true;
    r.acts.clear();
  };
  if (n == 0) return fail(FTS_E_MALFORMED, -1);  // "empty token request" (validator.go:79-81)
  struct Raw {
    int index;
    bool transfer;
    const uint8_t* p;
    size_t n;
  };
  Raw stack_raw[8];
  std::vector<Raw> heap_raw;
  int n_act = 0, n_iss = 0;
  // proto.Unmarshal of the request (Action / Signature messages included) fails first ...
  int unknown = -1;
  bool nil_sig = false;
  bool wire_ok = each(b, n, [&](const Field& x) {
    if (x.wt != 2) return true;
    if (x.no == 2) {  // Action{type=1 enum, raw=2 bytes}
      int32_t type = 0;
      Bytes raw;
      if (!each(x.p, x.n, [&](const Field& y) {
            if (y.no == 1 && y.wt == 0) type = (int32_t)(uint32_t)y.v;
            else if (y.no == 2 && y.wt == 2) raw.set(y);
            return true;
          }))
        return false;
      if (type == 0 || type == 1) {
        Raw w{n_act, type == 1, raw.p, raw.n};
        n_iss += type == 0;
        if (heap_raw.empty() && n_act < 8) {
          stack_raw[n_act] = w;
        } else {
          if (heap_raw.empty()) heap_raw.assign(stack_raw, stack_raw + n_act);
          heap_raw.push_back(w);
        }
      } else if (unknown < 0) {
        unknown = n_act;
      }
      n_act++;
    } else if (x.no == 3 || x.no == 4) {  // Signature{raw=1}
      Bytes raw;
      if (!raw_field(x.p, x.n, raw)) return false;
      nil_sig |= !raw.n;
    }
    return true;
  });
  if (!wire_ok) return fail(FTS_E_MALFORMED, -1);
  // ... then FromProtos: unknown action type (request.go:73-80), nil / empty signature (:82-93)
  if (unknown >= 0) return fail(FTS_E_MALFORMED, unknown);
  if (nil_sig) return fail(FTS_E_MALFORMED, -1);
  const Raw* raws = heap_raw.empty() ? stack_raw : heap_raw.data();
  const int n_known = heap_raw.empty() ? n_act : (int)heap_raw.size();
  r.acts.reserve(n_known);
  for (int pass = 0; pass < 2; pass++)  // every issue, then every transfer
    for (int k = 0; k < n_known; k++) {
      const Raw& w = raws[k];
      if (w.transfer != (pass == 1)) continue;
      r.acts.emplace_back();
      Action& a = r.acts.back();
      a.index = w.index;
      a.transfer = w.transfer;
      a.kind = w.transfer ? kind_transfer : kind_issue;
      bool ok = w.transfer ? transfer_action(w.p, w.n, r, a) : issue_action(w.p, w.n, r, a);
      if (!ok) return fail(FTS_E_MALFORMED, w.index);  // "failed to unmarshal actions"
    }
  (void)n_iss;
}


// ---------------------------------------------------------------------------
// token.Metadata.Deserialize (crypto/token/token.go:136-158) on driver.Metadata bytes:
//   comm.UnmarshalTypedToken (services/tokens/typed.go:28-35, core/comm/token.go:45-54):
//     asn1.Unmarshal into TypedToken{Type int32, Token []byte} = DER SEQUENCE{INTEGER,
//     OCTET STRING}; bytes after the outer TLV and extra elements inside the SEQUENCE are
//     ignored (Go encoding/asn1); Type must be comm.Type = 2 ("invalid token type")
//   proto TokenMetadata{type=1 string, value=2 Zr, blinding_factor=3 Zr, issuer=4 Identity}
//   FromZrProto (protos-go/utils/proto.go:62-72): nil message -> nil Zr; otherwise mathlib
//     Zr.UnmarshalJSON {"curve":id,"element":b64}: NewZrFromBytes = big-endian integer
//     (not reduced; G1.Mul uses it mod r).  Only curve 1 (BN254) is accepted here.
// Outputs the type bytes and value / bf reduced mod r as 32 BE bytes; has_* = false for
// a nil Zr (the caller's commit() then fails: FTS_E_MALFORMED).
struct TokenMeta {
  const uint8_t* type = nullptr;
  size_t type_len = 0;
  bool has_value = false, has_bf = false;
  uint8_t value[32], bf[32];
};
// big-endian integer of any length mod r -> 32 BE bytes
inline void be_mod_r(const uint8_t* p, size_t n, uint8_t out[32]) {
  Fr acc = Fr::zero();
  const Fr k256 = from_u64<ModR>(256);
  for (size_t i = 0; i < n; i++) acc = add(mul(acc, k256), from_u64<ModR>(p[i]));
  fr_to_be(acc, out);
}
inline bool zr_json_value(const Sub& z, bool& has, uint8_t out[32]) {
  has = false;
  if (!z.present) return true;
  Bytes raw;
  if (!raw_field(z.p, z.n, raw)) return false;
  std::string js((const char*)raw.p, raw.n), el, bin;
  long long curve = -1;
  if (!json_int_field(js, "curve", curve) || curve != 1) return false;
  if (!json_string_field(js, "element", el) || !b64_decode(el, bin)) return false;
  be_mod_r((const uint8_t*)bin.data(), bin.size(), out);
  has = true;
  return true;
}
inline bool token_metadata(const uint8_t* b, size_t n, TokenMeta& m) {
  using der::Span;
  size_t i = 0;
  uint8_t t;
  Span c;
  if (!der::read_tlv(b, n, i, t, c) || t != 0x30) return false;
  size_t j = 0;
  Span iv, tok;
  if (!der::read_tlv(c.p, c.n, j, t, iv) || t != 0x02 || iv.n == 0 || iv.n > 4) return false;  // int32
  if (iv.n > 1 && ((iv.p[0] == 0 && iv.p[1] < 0x80) || (iv.p[0] == 0xff && iv.p[1] >= 0x80))) return false;
  int64_t type = (iv.p[0] & 0x80) ? -1 : 0;
  for (size_t k = 0; k < iv.n; k++) type = (int64_t)(((uint64_t)type << 8) | iv.p[k]);
  if (!der::read_tlv(c.p, c.n, j, t, tok) || t != 0x04) return false;
  if (type != 2) return false;  // comm.Type
  Bytes ty;
  Sub value, bf, issuer;
  if (!each(tok.p, tok.n, [&](const Field& x) {
        if (x.wt != 2) return true;
        if (x.no == 1) {
          if (!utf8_valid(x.p, x.n)) return false;
          ty.set(x);
        } else if (x.no == 2) {
          value.add(x);
        } else if (x.no == 3) {
          bf.add(x);
        } else if (x.no == 4) {
          issuer.add(x);
        }
        return true;
      }))
    return false;
  Bytes iraw;
  if (issuer.present && !raw_field(issuer.p, issuer.n, iraw)) return false;
  m.type = ty.p;
  m.type_len = ty.n;
  return zr_json_value(value, m.has_value, m.value) && zr_json_value(bf, m.has_bf, m.bf);
}

}  // namespace req
}  // namespace host
}  // namespace fts
