// Minimal protobuf wire reader shared by the idemix host code (nym signatures,
// identity proofs): Go proto.Unmarshal failure modes -- truncation, varint
// overflow (protowire.ConsumeVarint), field 0 / numbers above 2^29 - 1, wire
// types 6 and 7, an end-group marker without its start.  Unknown groups
// (wire type 3 ... matching 4) are skipped as protowire.ConsumeFieldValue
// does; a known field with the wrong wire type is rejected by the callers.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace fts {

struct Pb {
  const uint8_t* p;
  size_t n, o = 0;
  // protowire.ConsumeVarint: at most 10 bytes, and the 10th may only carry bit 63
  bool varint(uint64_t& v) {
    v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (o >= n) return false;
      const uint8_t c = p[o++];
      if (sh == 63 && c > 1) return false;  // overflow
      v |= (uint64_t)(c & 0x7f) << sh;
      if (!(c & 0x80)) return true;
    }
    return false;
  }
  // the value of a field with wire type wt (key already read); groups nest up to
  // `depth` levels (protowire's recursion limit is far above any real message)
  bool skip_value(uint32_t f, uint32_t wt, int depth = 0) {
    uint64_t x;
    switch (wt) {
      case 0: return varint(x);
      case 1: if (n - o < 8) return false; o += 8; return true;
      case 5: if (n - o < 4) return false; o += 4; return true;
      case 2: if (!varint(x) || x > n - o) return false; o += (size_t)x; return true;
      case 3: {  // start group: fields until the end group of the same number
        if (depth >= 64) return false;
        for (;;) {
          uint64_t key;
          if (!varint(key)) return false;
          const uint32_t gf = (uint32_t)(key >> 3), gw = (uint32_t)(key & 7);
          if (gf == 0 || (key >> 3) > 0x1fffffff) return false;
          if (gw == 4) return gf == f;
          if (!skip_value(gf, gw, depth + 1)) return false;
        }
      }
      default: return false;  // 4 (end group without a start), 6, 7
    }
  }
  // next field: f, wire type, value span (bytes) / varint; groups are skipped
  // (v = nullptr, vl = 0) and reported with wt = 3
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
      case 3: return skip_value(f, 3);
      default: return false;
    }
  }
};


}  // namespace fts
