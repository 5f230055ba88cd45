// Minimal protobuf wire reader shared by the idemix host code (nym signatures,
// identity proofs): Go proto.Unmarshal failure modes -- truncation, varint
// overflow, field 0, bad / group wire types; a known field with the wrong wire
// type is rejected by the callers.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace fts {

struct Pb {
  const uint8_t* p;
  size_t n, o = 0;
  bool varint(uint64_t& v) {
    v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (o >= n) return false;
      const uint8_t c = p[o++];
      v |= (uint64_t)(c & 0x7f) << sh;
      if (!(c & 0x80)) return true;
    }
    return false;
  }
  // next field: f, wire type, value span (bytes) / varint
  bool next(uint32_t& f, uint32_t& wt, const uint8_t*& v, size_t& vl, uint64_t& iv) {
    uint64_t key;
    if (!varint(key)) return false;
    f = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (f == 0 || (key >> 3) > 0x1fffffff) return false;
    v = nullptr, vl = 0, iv = 0;
    switch (wt) {
      case 0: return varint(iv);
      case 1: if (n - o < 8) return false; v = p + o, vl = 8, o += 8; return true;
      case 5: if (n - o < 4) return false; v = p + o, vl = 4, o += 4; return true;
      case 2: {
        uint64_t l;
        if (!varint(l) || l > n - o) return false;
        v = p + o, vl = (size_t)l, o += (size_t)l;
        return true;
      }
      default: return false;
    }
  }
};


}  // namespace fts
