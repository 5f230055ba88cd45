/*
 * CPU ORACLE (test infrastructure + bench.py cpu_baseline only; never shipped,
 * never linked by the product).
 *
 * A plain-C restatement of the reference range-proof verifier in the
 * reference's exact operation order:
 *   (*rangeVerifier).Verify      rp/bulletproof.go:252-333
 *   (*rangeVerifier).verifyIPA   rp/bulletproof.go:469-509
 *   (*ipaVerifier).Verify        rp/ipa.go:190-262
 *   reduceGenerators             rp/ipa.go:343-356
 *   (*G1Array).Bytes             crypto/common/array.go:25-36
 * with mathlib/gnark semantics: every G1.Mul / Add / Sub returns a canonical
 * affine point (one field inversion per operation), Curve.HashToZr =
 * SHA-256 mod r, Zr.Bytes = 32-byte big-endian.  Per 64-bit proof this is
 * 7n + 2k + 9 = 469 variable-base scalar multiplications, as in the
 * reference.  Field arithmetic: 4 x 64-bit Montgomery (unsigned __int128).
 *
 * Entry points (ctypes, oracle/cref.py):
 *   int oracle_rp_verify(const uint8_t* gens, int n, const uint8_t* com64,
 *                        const uint8_t* der, size_t len)
 *   int oracle_rp_verify_many(const uint8_t* gens, int n, int count,
 *                             const uint8_t* coms, const uint8_t* const* ders,
 *                             const size_t* lens, int threads, int32_t* out)
 * gens = 64-byte points [G=ped1, H=ped2, P, Q, L_0..L_{n-1}, R_0..R_{n-1}].
 * Return: 0 ok, 1 malformed, 2 nil elements, 3 "invalid range proof",
 *         4 IPA nil, 5 IPA length, 6 "invalid IPA"  (same codes as fts_status).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;

static const uint64_t PM[4] = {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
static const uint64_t PINV = 0x87d20782e4866389ULL;
static const uint64_t PR2[4] = {0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL, 0x06d89f71cab8351fULL};
static const uint64_t RM[4] = {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL};
static const uint64_t RINV = 0xc2e1f593efffffffULL;
static const uint64_t RR2[4] = {0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL, 0x8c49833d53bb8085ULL, 0x0216d0b17f4e44a5ULL};

/* ------------------------------------------------------------ field */
static int geq(const uint64_t* a, const uint64_t* m) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != m[i]) return a[i] > m[i];
  return 1;
}
static void subm(uint64_t* a, const uint64_t* m) {
  u128 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - m[i] - b;
    a[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}
static inline __attribute__((always_inline)) fe fadd(fe a, fe b, const uint64_t* m) {
  fe r;
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.v[i] + b.v[i];
    r.v[i] = (uint64_t)c;
    c >>= 64;
  }
  if (geq(r.v, m)) subm(r.v, m);
  return r;
}
static inline __attribute__((always_inline)) fe fsub(fe a, fe b, const uint64_t* m) {
  fe r;
  u128 bw = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - bw;
    r.v[i] = (uint64_t)d;
    bw = (d >> 64) & 1;
  }
  if (bw) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)r.v[i] + m[i];
      r.v[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}
static inline __attribute__((always_inline)) fe fmul(fe a, fe b, const uint64_t* m, uint64_t inv) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.v[j] * b.v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t q = t[0] * inv;
    c = (u128)q * m[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)q * m[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  fe r;
  memcpy(r.v, t, 32);
  if (t[4] || geq(r.v, m)) subm(r.v, m);
  return r;
}
#define PMUL(a, b) fmul(a, b, PM, PINV)
#define PADD(a, b) fadd(a, b, PM)
#define PSUB(a, b) fsub(a, b, PM)
#define RMUL(a, b) fmul(a, b, RM, RINV)
#define RADD(a, b) fadd(a, b, RM)
#define RSUB(a, b) fsub(a, b, RM)

static int fzero(fe a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3]); }
static int feq(fe a, fe b) { return !memcmp(a.v, b.v, 32); }
static fe ftomont(fe a, const uint64_t* m, uint64_t inv, const uint64_t* r2) {
  fe R;
  memcpy(R.v, r2, 32);
  return fmul(a, R, m, inv);
}
static fe ffrommont(fe a, const uint64_t* m, uint64_t inv) {
  fe one = {{1, 0, 0, 0}};
  return fmul(a, one, m, inv);
}
static fe fpow(fe a, const uint64_t* e, const uint64_t* m, uint64_t inv, const uint64_t* r2) {
  fe one = {{1, 0, 0, 0}};
  fe r = ftomont(one, m, inv, r2);
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = fmul(r, r, m, inv);
      if ((e[i] >> b) & 1) r = fmul(r, a, m, inv);
    }
  return r;
}
static fe finv(fe a, const uint64_t* m, uint64_t inv, const uint64_t* r2) {
  uint64_t e[4];
  memcpy(e, m, 32);
  e[0] -= 2;
  return fpow(a, e, m, inv, r2);
}
static fe be_to_fe(const uint8_t* b) {
  fe r;
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[(3 - i) * 8 + k];
    r.v[i] = w;
  }
  return r;
}
static void fe_to_be(fe a, uint8_t* b) {
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) b[(3 - i) * 8 + k] = (uint8_t)(a.v[i] >> (56 - 8 * k));
}

/* Zr helpers: values kept canonical (non-Montgomery) as mathlib big.Ints */
static fe zr_mul(fe a, fe b) {
  fe am = ftomont(a, RM, RINV, RR2);
  return RMUL(am, b); /* (a R)(b) R^-1 = ab */
}
static fe zr_inv(fe a) {
  fe am = ftomont(a, RM, RINV, RR2);
  return ffrommont(finv(am, RM, RINV, RR2), RM, RINV);
}
static fe zr_red(fe a) {
  while (geq(a.v, RM)) subm(a.v, RM);
  return a;
}
static fe zr_u64(uint64_t x) {
  fe r = {{x, 0, 0, 0}};
  return r;
}

/* ------------------------------------------------------------ G1 (affine API, Jacobian inside) */
typedef struct { fe x, y; int inf; } g1;
typedef struct { fe x, y, z; } g1j;

static fe P_ONE, P_THREE;
static void init_consts(void) {
  fe one = {{1, 0, 0, 0}}, three = {{3, 0, 0, 0}};
  P_ONE = ftomont(one, PM, PINV, PR2);
  P_THREE = ftomont(three, PM, PINV, PR2);
}
static g1j jid(void) {
  g1j r;
  r.x = P_ONE;
  r.y = P_ONE;
  memset(&r.z, 0, sizeof r.z);
  return r;
}
static g1j tojac(g1 a) {
  if (a.inf) return jid();
  g1j r = {a.x, a.y, P_ONE};
  return r;
}
static g1j jdbl(g1j p) {
  if (fzero(p.z) || fzero(p.y)) return jid();
  fe A = PMUL(p.x, p.x), B = PMUL(p.y, p.y), C = PMUL(B, B);
  fe t = PADD(p.x, B);
  fe D = PSUB(PSUB(PMUL(t, t), A), C);
  D = PADD(D, D);
  fe E = PADD(PADD(A, A), A);
  fe F = PMUL(E, E);
  g1j r;
  r.x = PSUB(F, PADD(D, D));
  fe C8 = PADD(C, C);
  C8 = PADD(C8, C8);
  C8 = PADD(C8, C8);
  r.y = PSUB(PMUL(E, PSUB(D, r.x)), C8);
  fe yz = PMUL(p.y, p.z);
  r.z = PADD(yz, yz);
  return r;
}
static g1j jadd(g1j p, g1j q) {
  if (fzero(p.z)) return q;
  if (fzero(q.z)) return p;
  fe z1z1 = PMUL(p.z, p.z), z2z2 = PMUL(q.z, q.z);
  fe u1 = PMUL(p.x, z2z2), u2 = PMUL(q.x, z1z1);
  fe s1 = PMUL(PMUL(p.y, q.z), z2z2), s2 = PMUL(PMUL(q.y, p.z), z1z1);
  if (feq(u1, u2)) return feq(s1, s2) ? jdbl(p) : jid();
  fe h = PSUB(u2, u1), h2 = PADD(h, h);
  fe i = PMUL(h2, h2), j = PMUL(h, i);
  fe rr = PSUB(s2, s1);
  rr = PADD(rr, rr);
  fe v = PMUL(u1, i);
  g1j r;
  r.x = PSUB(PSUB(PMUL(rr, rr), j), PADD(v, v));
  fe s1j = PMUL(s1, j);
  r.y = PSUB(PMUL(rr, PSUB(v, r.x)), PADD(s1j, s1j));
  fe zz = PADD(p.z, q.z);
  r.z = PMUL(PSUB(PSUB(PMUL(zz, zz), z1z1), z2z2), h);
  return r;
}
static g1 toaff(g1j p) {
  g1 r;
  if (fzero(p.z)) {
    memset(&r, 0, sizeof r);
    r.inf = 1;
    return r;
  }
  fe zi = finv(p.z, PM, PINV, PR2), zi2 = PMUL(zi, zi);
  r.x = PMUL(p.x, zi2);
  r.y = PMUL(PMUL(p.y, zi2), zi);
  r.inf = 0;
  return r;
}
/* mathlib G1.Mul: (s mod r) * P, affine result (4-bit fixed window inside) */
static g1 g1_mul(g1 p, fe s) {
  s = zr_red(s);
  g1j tbl[16];
  tbl[0] = jid();
  tbl[1] = tojac(p);
  for (int i = 2; i < 16; i++) tbl[i] = jadd(tbl[i - 1], tbl[1]);
  g1j acc = jid();
  for (int w = 63; w >= 0; w--) {
    for (int d = 0; d < 4; d++) acc = jdbl(acc);
    int nib = (int)((s.v[w / 16] >> ((w % 16) * 4)) & 15);
    if (nib) acc = jadd(acc, tbl[nib]);
  }
  return toaff(acc);
}
static g1 g1_add(g1 a, g1 b) { return toaff(jadd(tojac(a), tojac(b))); }
static g1 g1_neg(g1 a) {
  if (!a.inf) {
    fe z = {{0, 0, 0, 0}};
    a.y = PSUB(z, a.y);
  }
  return a;
}
static g1 g1_sub(g1 a, g1 b) { return g1_add(a, g1_neg(b)); }
static int g1_eq(g1 a, g1 b) {
  if (a.inf || b.inf) return a.inf && b.inf;
  return feq(a.x, b.x) && feq(a.y, b.y);
}
static void g1_bytes(g1 a, uint8_t* out) {
  if (a.inf) {
    memset(out, 0, 64);
    return;
  }
  fe_to_be(ffrommont(a.x, PM, PINV), out);
  fe_to_be(ffrommont(a.y, PM, PINV), out + 32);
}
static int g1_from_bytes(const uint8_t* b, size_t len, g1* out) {
  if (len != 64 || (b[0] & 0xC0)) return 0;
  fe x = be_to_fe(b), y = be_to_fe(b + 32);
  if (geq(x.v, PM) || geq(y.v, PM)) return 0;
  if (fzero(x) && fzero(y)) {
    memset(out, 0, sizeof *out);
    out->inf = 1;
    return 1;
  }
  out->x = ftomont(x, PM, PINV, PR2);
  out->y = ftomont(y, PM, PINV, PR2);
  out->inf = 0;
  fe rhs = PADD(PMUL(PMUL(out->x, out->x), out->x), P_THREE);
  return feq(PMUL(out->y, out->y), rhs);
}

/* ------------------------------------------------------------ SHA-256 */
typedef struct { uint32_t h[8]; uint8_t buf[64]; uint32_t fill; uint64_t tot; } sha_t;
static const uint32_t SK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_blk(sha_t* s) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)s->buf[4 * i] << 24) | ((uint32_t)s->buf[4 * i + 1] << 16) | ((uint32_t)s->buf[4 * i + 2] << 8) |
           s->buf[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = s->h[0], b = s->h[1], c = s->h[2], d = s->h[3], e = s->h[4], f = s->h[5], g = s->h[6], h = s->h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s->h[0] += a; s->h[1] += b; s->h[2] += c; s->h[3] += d; s->h[4] += e; s->h[5] += f; s->h[6] += g; s->h[7] += h;
}
static void sha_init(sha_t* s) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, iv, 32);
  s->fill = 0;
  s->tot = 0;
}
static void sha_upd(sha_t* s, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++) {
    s->buf[s->fill++] = p[i];
    s->tot++;
    if (s->fill == 64) {
      sha_blk(s);
      s->fill = 0;
    }
  }
}
static void sha_fin(sha_t* s, uint8_t* out) {
  uint64_t bits = s->tot * 8;
  uint8_t one = 0x80, zero = 0;
  sha_upd(s, &one, 1);
  while (s->fill != 56) sha_upd(s, &zero, 1);
  uint8_t L[8];
  for (int i = 0; i < 8; i++) L[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_upd(s, L, 8);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = s->h[i] >> 24;
    out[4 * i + 1] = s->h[i] >> 16;
    out[4 * i + 2] = s->h[i] >> 8;
    out[4 * i + 3] = s->h[i];
  }
}
/* Curve.HashToZr over a G1Array transcript (array.go:25-36), streamed */
static void sha_points(sha_t* s, const g1* pts, int m) {
  static const char* hx = "0123456789abcdef";
  for (int i = 0; i < m; i++) {
    uint8_t b[64], h[128];
    g1_bytes(pts[i], b);
    for (int q = 0; q < 64; q++) {
      h[2 * q] = hx[b[q] >> 4];
      h[2 * q + 1] = hx[b[q] & 15];
    }
    if (i) sha_upd(s, (const uint8_t*)"||", 2);
    sha_upd(s, h, 128);
  }
}
static fe digest_zr(const uint8_t* d) { return zr_red(be_to_fe(d)); }
static fe hash_points(const g1* pts, int m) {
  sha_t s;
  uint8_t d[32];
  sha_init(&s);
  sha_points(&s, pts, m);
  sha_fin(&s, d);
  return digest_zr(d);
}

/* ------------------------------------------------------------ DER */
typedef struct { const uint8_t* p; size_t n; } span;
static int tlv(const uint8_t* b, size_t len, size_t* i, uint8_t* tag, span* c) {
  if (*i + 2 > len) return 0;
  *tag = b[*i];
  size_t l = b[*i + 1];
  *i += 2;
  if (l & 0x80) {
    size_t nb = l & 0x7f;
    if (nb == 0 || nb > 4 || *i + nb > len || b[*i] == 0) return 0;
    l = 0;
    for (size_t k = 0; k < nb; k++) l = (l << 8) | b[*i + k];
    *i += nb;
    if (l < 0x80) return 0;
  }
  if (l > len - *i) return 0;
  c->p = b + *i;
  c->n = l;
  *i += l;
  return 1;
}
/* Values{[][]byte} -> up to cap items */
static int values(span raw, span* out, int cap, int strict) {
  size_t i = 0, j = 0;
  uint8_t t;
  span c, inner;
  if (!tlv(raw.p, raw.n, &i, &t, &c) || t != 0x30) return -1;
  if (strict && i != raw.n) return -1;
  if (!tlv(c.p, c.n, &j, &t, &inner) || t != 0x30) return -1;
  int m = 0;
  size_t k = 0;
  while (k < inner.n) {
    span s;
    if (!tlv(inner.p, inner.n, &k, &t, &s) || t != 0x04) return -1;
    if (m < cap) out[m] = s;
    m++;
  }
  return m;
}
static int element(span raw, span* e) {
  size_t i = 0, j = 0;
  uint8_t t;
  span c, ci;
  if (!tlv(raw.p, raw.n, &i, &t, &c) || t != 0x30 || i != raw.n) return 0;
  if (!tlv(c.p, c.n, &j, &t, &ci) || t != 0x02 || ci.n != 1 || ci.p[0] != 1) return 0;
  if (!tlv(c.p, c.n, &j, &t, e) || t != 0x04) return 0;
  return 1;
}
static fe zr_from(span e) {
  uint8_t b[32] = {0};
  size_t off = 0;
  while (off < e.n && e.p[off] == 0) off++;
  size_t l = e.n - off;
  if (l > 32) l = 32, off = e.n - 32; /* oversized scalars: not produced by honest provers */
  memcpy(b + 32 - l, e.p + off, l);
  return be_to_fe(b);
}

/* ------------------------------------------------------------ verifier */
typedef struct {
  int n, k;
  g1 G, H, P, Q;
  g1 *L, *R;
} params;

static void reduce_gens(g1* lg, g1* rg, int m, fe x, fe xinv) { /* ipa.go:343-356, in place */
  for (int i = 0; i < m; i++) {
    g1 a = g1_mul(lg[i], xinv);
    a = g1_add(a, g1_mul(lg[i + m], x));
    g1 b = g1_mul(rg[i], x);
    b = g1_add(b, g1_mul(rg[i + m], xinv));
    lg[i] = a;
    rg[i] = b;
  }
}

/* a parsed range proof (rp/bulletproof.go RangeProof, ipa.go IPA) */
typedef struct {
  g1 T1, T2, C, D;
  fe tau, delta, ipv, a, b;
  int ipa_err, nl, nr;
  g1 Ls[70], Rs[70];
} rp_parsed;

/* DER -> rp_parsed.  Returns 1 malformed, 2 nil elements, else 0; IPA nil
 * errors are kept in ipa_err (ipv.Verify reports them after the E1 check). */
static int parse_rp(span rp, rp_parsed* o) {
  span dv[2], d[8], ip[4];
  if (values(rp, dv, 2, 0) != 2) return 1;
  if (dv[0].n == 0) return 2;
  int nd = values(dv[0], d, 8, 0);
  if (nd < 0) return 1;
  if (nd < 7) return 2;
  span e;
  if (!element(d[0], &e) || !g1_from_bytes(e.p, e.n, &o->T1)) return 1;
  if (!element(d[1], &e) || !g1_from_bytes(e.p, e.n, &o->T2)) return 1;
  if (!element(d[2], &e)) return 1;
  o->tau = zr_from(e);
  if (!element(d[3], &e) || !g1_from_bytes(e.p, e.n, &o->C)) return 1;
  if (!element(d[4], &e) || !g1_from_bytes(e.p, e.n, &o->D)) return 1;
  if (!element(d[5], &e)) return 1;
  o->delta = zr_from(e);
  if (!element(d[6], &e)) return 1;
  o->ipv = zr_from(e);
  /* IPA: structural errors are reported by ipv.Verify, i.e. only after the E1 check */
  int ni = 0;
  o->ipa_err = 0;
  o->nl = o->nr = 0;
  o->a = zr_u64(0);
  o->b = zr_u64(0);
  if (dv[1].n == 0) {
    o->ipa_err = 4;
  } else {
    ni = values(dv[1], ip, 4, 0);
    if (ni < 0) return 1;
    if (ni >= 1) {
      if (!element(ip[0], &e)) return 1;
      o->a = zr_from(e);
    }
    if (ni >= 2) {
      if (!element(ip[1], &e)) return 1;
      o->b = zr_from(e);
    }
    span la[70], ra[70], el, er;
    if (ni >= 3) {
      if (!element(ip[2], &el) || (o->nl = values(el, la, 70, 1)) < 0) return 1;
      for (int j = 0; j < o->nl && j < 70; j++)
        if (!g1_from_bytes(la[j].p, la[j].n, &o->Ls[j])) return 1;
    }
    if (ni >= 4) {
      if (!element(ip[3], &er) || (o->nr = values(er, ra, 70, 1)) < 0) return 1;
      for (int j = 0; j < o->nr && j < 70; j++)
        if (!g1_from_bytes(ra[j].p, ra[j].n, &o->Rs[j])) return 1;
    }
    if (ni < 2) o->ipa_err = 4;
  }
  return 0;
}

static int verify_one(const params* pp, g1 V, span rp) {
  int n = pp->n, k = pp->k;
  rp_parsed P;
  int pe = parse_rp(rp, &P);
  if (pe) return pe;
  g1 T1 = P.T1, T2 = P.T2, C = P.C, D = P.D, *Ls = P.Ls, *Rs = P.Rs;
  fe tau = P.tau, delta = P.delta, ipv = P.ipv, a = P.a, b = P.b;
  int ipa_err = P.ipa_err, nl = P.nl, nr = P.nr;

  /* bulletproof.go:266-311 */
  g1 arr[3] = {T1, T2};
  fe x = hash_points(arr, 2);
  fe x2 = zr_mul(x, x);
  arr[0] = C; arr[1] = D; arr[2] = V;
  fe y = hash_points(arr, 3);
  uint8_t yb[32], dg[32];
  fe_to_be(y, yb);
  sha_t s;
  sha_init(&s);
  sha_upd(&s, yb, 32);
  sha_fin(&s, dg);
  fe z = digest_zr(dg);
  fe z2 = zr_mul(z, z), z3 = zr_mul(z2, z);
  fe *ypow = malloc(sizeof(fe) * n), ipy = zr_u64(0), ip2 = zr_u64(0), p2 = zr_u64(1);
  for (int i = 0; i < n; i++) {
    if (i == 0) {
      ypow[0] = zr_u64(1);
      p2 = zr_u64(1);
    } else {
      ypow[i] = zr_mul(y, ypow[i - 1]);
      p2 = zr_mul(zr_u64(2), p2);
    }
    ipy = RADD(ipy, ypow[i]);
    ip2 = RADD(ip2, p2);
  }
  fe pol = zr_mul(RSUB(z, z2), ipy);
  pol = RSUB(pol, zr_mul(z3, ip2));
  /* :314-324 */
  g1 com = g1_mul(pp->G, ipv);
  com = g1_add(com, g1_mul(pp->H, tau));
  com = g1_sub(com, g1_mul(T1, x));
  com = g1_sub(com, g1_mul(T2, x2));
  g1 comp = g1_mul(V, z2);
  comp = g1_add(comp, g1_mul(pp->G, pol));
  if (!g1_eq(com, comp)) {
    free(ypow);
    return 3;
  }
  /* ipa.go:192-198 (after the E1 check, as in the reference) */
  if (ipa_err) {
    free(ypow);
    return ipa_err;
  }
  if (nl != nr || nl != k) {
    free(ypow);
    return 5;
  }
  /* verifyIPA :477-492 */
  g1 *rgp = malloc(sizeof(g1) * n), *lg = malloc(sizeof(g1) * n);
  g1 cm = g1_mul(D, x);
  cm = g1_add(cm, C);
  for (int i = 0; i < n; i++) {
    cm = g1_sub(cm, g1_mul(pp->L[i], z));
    fe yinv = zr_inv(ypow[i]);
    fe zi = zr_mul(z, ypow[i]);
    fe tp = zr_u64(1);
    for (int q = 0; q < i; q++) tp = RADD(tp, tp); /* 2^i (PowMod) */
    zi = RADD(zi, zr_mul(z2, tp));
    rgp[i] = g1_mul(pp->R[i], yinv);
    cm = g1_add(cm, g1_mul(rgp[i], zi));
    lg[i] = pp->L[i];
  }
  cm = g1_sub(cm, g1_mul(pp->P, delta));
  /* ipa.go:200-218: x0 over DER(SEQUENCE OF OCTET STRING [Arr(H', G, Q, com), "||", Zb(ip)]) */
  size_t alen = 130 * (size_t)(2 * n + 2) - 2, seqc = (4 + alen) + 4 + 34;
  uint8_t hdr[8] = {0x30, 0x82, (uint8_t)(seqc >> 8), (uint8_t)seqc, 0x04, 0x82, (uint8_t)(alen >> 8), (uint8_t)alen};
  sha_init(&s);
  sha_upd(&s, hdr, 8);
  g1* all = malloc(sizeof(g1) * (2 * n + 2));
  for (int i = 0; i < n; i++) all[i] = rgp[i], all[n + i] = pp->L[i];
  all[2 * n] = pp->Q;
  all[2 * n + 1] = cm;
  sha_points(&s, all, 2 * n + 2);
  free(all);
  uint8_t tail[6] = {0x04, 0x02, '|', '|', 0x04, 0x20}, ipb[32];
  sha_upd(&s, tail, 6);
  fe_to_be(zr_red(ipv), ipb);
  sha_upd(&s, ipb, 32);
  sha_fin(&s, dg);
  fe x0 = digest_zr(dg);
  g1 Cc = g1_mul(pp->Q, zr_mul(x0, zr_red(ipv)));
  Cc = g1_add(Cc, cm);
  g1 X = g1_mul(pp->Q, x0);
  int m = n;
  for (int j = 0; j < k; j++) { /* :224-252 */
    g1 lr[2] = {Ls[j], Rs[j]};
    fe xj = hash_points(lr, 2);
    fe xinv = zr_inv(xj);
    fe xs = zr_mul(xj, xj), xsi = zr_inv(xs);
    g1 cp = g1_mul(Ls[j], xs);
    cp = g1_add(cp, Cc);
    cp = g1_add(cp, g1_mul(Rs[j], xsi));
    Cc = cp;
    m /= 2;
    reduce_gens(lg, rgp, m, xj, xinv);
  }
  g1 cp = g1_mul(lg[0], a);
  cp = g1_add(cp, g1_mul(rgp[0], b));
  cp = g1_add(cp, g1_mul(X, zr_mul(zr_red(a), zr_red(b))));
  int ok = g1_eq(cp, Cc);
  free(ypow);
  free(rgp);
  free(lg);
  return ok ? 0 : 6;
}

static int load_params(const uint8_t* gens, int n, params* pp) {
  init_consts();
  pp->n = n;
  pp->k = 0;
  while ((1 << pp->k) < n) pp->k++;
  pp->L = malloc(sizeof(g1) * n);
  pp->R = malloc(sizeof(g1) * n);
  int ok = g1_from_bytes(gens, 64, &pp->G) & g1_from_bytes(gens + 64, 64, &pp->H) &
           g1_from_bytes(gens + 128, 64, &pp->P) & g1_from_bytes(gens + 192, 64, &pp->Q);
  for (int i = 0; i < n; i++) {
    ok &= g1_from_bytes(gens + 256 + 64 * i, 64, &pp->L[i]);
    ok &= g1_from_bytes(gens + 256 + 64 * (n + i), 64, &pp->R[i]);
  }
  return ok;
}

int oracle_rp_verify(const uint8_t* gens, int n, const uint8_t* com64, const uint8_t* der, size_t len) {
  params pp;
  if (!load_params(gens, n, &pp)) return -1;
  g1 V;
  int r;
  if (!g1_from_bytes(com64, 64, &V)) r = 1;
  else {
    span s = {der, len};
    r = verify_one(&pp, V, s);
  }
  free(pp.L);
  free(pp.R);
  return r;
}

typedef struct {
  const params* pp;
  const uint8_t* coms;
  const uint8_t* const* ders;
  const size_t* lens;
  int32_t* out;
  int count, next;
  pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->count) return NULL;
    g1 V;
    if (!g1_from_bytes(j->coms + 64 * (size_t)i, 64, &V)) {
      j->out[i] = 1;
      continue;
    }
    span s = {j->ders[i], j->lens[i]};
    j->out[i] = verify_one(j->pp, V, s);
  }
}

int oracle_rp_verify_many(const uint8_t* gens, int n, int count, const uint8_t* coms, const uint8_t* const* ders,
                          const size_t* lens, int threads, int32_t* out) {
  params pp;
  if (!load_params(gens, n, &pp)) return -1;
  job_t j = {&pp, coms, ders, lens, out, count, 0};
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &j);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(pp.L);
  free(pp.R);
  return 0;
}

/* ------------------------------------------------ MSM baseline (config C3)
 * int oracle_msm(const uint8_t* pts, const uint8_t* scs, size_t n, int threads, uint8_t* out64)
 * sum_i (k_i mod r) P_i term by term with the reference's G1.Mul + Add (no
 * Pippenger): the CPU baseline of the MSM microbenchmark, and an oracle for
 * it.  pts: n x 64-byte BE points, scs: n x 32-byte BE scalars.
 * Return 0, or -1 if a point fails NewG1FromBytes. */
typedef struct {
  const uint8_t *pts, *scs;
  size_t n, next;
  g1j acc;
  int bad;
  pthread_mutex_t mu;
} msm_job;
static void* msm_worker(void* arg) {
  msm_job* j = (msm_job*)arg;
  g1j acc = jid();
  int bad = 0;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t lo = j->next;
    j->next += 64;
    pthread_mutex_unlock(&j->mu);
    if (lo >= j->n) break;
    size_t hi = lo + 64 < j->n ? lo + 64 : j->n;
    for (size_t i = lo; i < hi; i++) {
      g1 p;
      if (!g1_from_bytes(j->pts + 64 * i, 64, &p)) {
        bad = 1;
        continue;
      }
      acc = jadd(acc, tojac(g1_mul(p, be_to_fe(j->scs + 32 * i))));
    }
  }
  pthread_mutex_lock(&j->mu);
  j->acc = jadd(j->acc, acc);
  j->bad |= bad;
  pthread_mutex_unlock(&j->mu);
  return NULL;
}
int oracle_msm(const uint8_t* pts, const uint8_t* scs, size_t n, int threads, uint8_t* out64) {
  init_consts();
  msm_job j;
  j.pts = pts;
  j.scs = scs;
  j.n = n;
  j.next = 0;
  j.acc = jid();
  j.bad = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, msm_worker, &j);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  g1_bytes(toaff(j.acc), out64);
  return j.bad ? -1 : 0;
}

/* ---------------------------------------------------------------- openings
 * int oracle_open_check_many(const uint8_t* ped, int count, const uint8_t* coms,
 *     const uint8_t* const* types, const size_t* type_lens, const uint8_t* values,
 *     const uint8_t* bfs, int threads, int32_t* out)
 * Auditor.InspectOutput's check in reference order (crypto/audit/auditor.go:226-238,
 * commit() :412-418): com = NewG1(); com.Add(ped_i.Mul(v_i)) for (HashToZr(type),
 * value, bf); Equals(token.Data).  ped: 3 x 64-byte BE generators; coms: count x 64;
 * values / bfs: count x 32-byte BE (used mod r).  out[i]: 0 ok, 12 mismatch,
 * 1 token.Data rejected by NewG1FromBytes (fts_status numbering). */
typedef struct {
  g1 ped[3];
  const uint8_t *coms, *values, *bfs;
  const uint8_t* const* types;
  const size_t* tlens;
  int32_t* out;
  int count, next;
  pthread_mutex_t mu;
} open_job;
static void* open_worker(void* arg) {
  open_job* j = (open_job*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int lo = j->next;
    j->next += 16;
    pthread_mutex_unlock(&j->mu);
    if (lo >= j->count) break;
    int hi = lo + 16 < j->count ? lo + 16 : j->count;
    for (int i = lo; i < hi; i++) {
      g1 data;
      if (!g1_from_bytes(j->coms + 64 * (size_t)i, 64, &data)) {
        j->out[i] = 1;
        continue;
      }
      sha_t s;
      uint8_t d[32];
      sha_init(&s);
      sha_upd(&s, j->types[i], j->tlens[i]);
      sha_fin(&s, d);
      g1 c;
      memset(&c, 0, sizeof c);
      c.inf = 1;
      c = g1_add(c, g1_mul(j->ped[0], digest_zr(d)));
      c = g1_add(c, g1_mul(j->ped[1], be_to_fe(j->values + 32 * (size_t)i)));
      c = g1_add(c, g1_mul(j->ped[2], be_to_fe(j->bfs + 32 * (size_t)i)));
      j->out[i] = g1_eq(c, data) ? 0 : 12;
    }
  }
  return NULL;
}
int oracle_open_check_many(const uint8_t* ped, int count, const uint8_t* coms, const uint8_t* const* types,
                           const size_t* type_lens, const uint8_t* values, const uint8_t* bfs, int threads,
                           int32_t* out) {
  init_consts();
  open_job j;
  for (int k = 0; k < 3; k++)
    if (!g1_from_bytes(ped + 64 * k, 64, &j.ped[k])) return -1;
  j.coms = coms;
  j.values = values;
  j.bfs = bfs;
  j.types = types;
  j.tlens = type_lens;
  j.out = out;
  j.count = count;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, open_worker, &j);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  return 0;
}

/* ---------------------------------------------------------------- actions
 * int oracle_action_verify_many(const uint8_t* ped, const uint8_t* gens, int n, int count,
 *     const int32_t* kind, const int32_t* n_in, const int32_t* n_out, const uint8_t* const* in64,
 *     const uint8_t* const* out64, const uint8_t* const* ders, const size_t* lens, int threads,
 *     int32_t* status, int32_t* index)
 * kind 0: transfer.NewVerifier(in, out, pp).Verify (transfer/transfer.go:153-197):
 *   TypeAndSumVerifier.Verify (typeandsum.go:230-277) then, unless 1-in/1-out,
 *   RangeCorrectnessVerifier.Verify on V_j = Out_j - CT (rangecorrectness.go:137-162);
 *   the TypeAndSum error wins.
 * kind 1: issue.NewVerifier(tokens, pp).Verify (issue/verifier.go:32-57): SameType
 *   (sametype.go:167-183), then RangeCorrectness on Tok_j - CT (tokens in out64).
 * Both in the reference's operation order: every G1 operation affine, one G1.Mul per
 * scalar multiplication, sequential range proofs (the reference's extra goroutine in
 * transfer.go:171 overlaps TypeAndSum with the range proofs; the verdicts do not
 * depend on it).  status: fts_status numbering (0 ok, 1 malformed, 3/6.. range-proof
 * class at index[i], 7 #proofs != #outputs, 8 TypeAndSum, 9 SameType). */
static int g1_el(span d, g1* out) {
  span e;
  return element(d, &e) && g1_from_bytes(e.p, e.n, out);
}
static int zr_el(span d, fe* out) {
  span e;
  if (!element(d, &e)) return 0;
  *out = zr_from(e);
  return 1;
}
static int zr_arr_el(span d, fe* out, int cap) {
  span e, it[16];
  if (!element(d, &e)) return -1;
  int m = values(e, it, 16, 1);
  if (m < 0 || m > cap) return -1;
  for (int i = 0; i < m; i++) out[i] = zr_from(it[i]);
  return m;
}
static int rc_verify(const params* pp, const g1* coms, int m, span rc, int32_t* idx) {
  span outer[2], rps[32];
  if (values(rc, outer, 2, 0) != 1) return 1;
  int np = values(outer[0], rps, 32, 0);
  if (np < 0) return 1;
  if (np != m) return 7;
  for (int j = 0; j < m; j++) {
    int r = verify_one(pp, coms[j], rps[j]);
    if (r) {
      *idx = j;
      return r;
    }
  }
  return 0;
}
static int tas_verify(const g1* ped, const g1* in, int nin, const g1* out, int nout, span raw, g1* ct) {
  span d[8];
  if (values(raw, d, 8, 0) != 7) return 1;
  fe ibf[16], iv[16], type, tbf, eqs, chal;
  if (!g1_el(d[0], ct)) return 1;
  if (zr_arr_el(d[1], ibf, 16) < nin || zr_arr_el(d[2], iv, 16) < nin) return 1;
  if (!zr_el(d[3], &type) || !zr_el(d[4], &tbf) || !zr_el(d[5], &eqs) || !zr_el(d[6], &chal)) return 1;
  g1 arr[40], ins[16], outs[16], incom[16];
  g1 sum;
  memset(&sum, 0, sizeof sum);
  sum.inf = 1;
  for (int i = 0; i < nin; i++) { /* typeandsum.go:240-252 */
    ins[i] = g1_sub(in[i], *ct);
    sum = g1_add(sum, ins[i]);
    g1 c = g1_mul(ped[1], iv[i]);
    c = g1_add(c, g1_mul(ped[2], ibf[i]));
    incom[i] = g1_sub(c, g1_mul(ins[i], chal));
  }
  for (int j = 0; j < nout; j++) {
    outs[j] = g1_sub(out[j], *ct);
    sum = g1_sub(sum, outs[j]);
  }
  g1 sumcom = g1_sub(g1_mul(ped[2], eqs), g1_mul(sum, chal)); /* :254-256 */
  g1 typecom = g1_add(g1_mul(ped[0], type), g1_mul(ped[2], tbf));
  typecom = g1_sub(typecom, g1_mul(*ct, chal));
  int m = 0;
  for (int i = 0; i < nin; i++) arr[m++] = incom[i];
  arr[m++] = typecom;
  arr[m++] = sumcom;
  for (int i = 0; i < nin; i++) arr[m++] = ins[i];
  for (int j = 0; j < nout; j++) arr[m++] = outs[j];
  arr[m++] = *ct;
  arr[m++] = sum;
  fe h = hash_points(arr, m); /* :267-274: raw Zr.Equals */
  return feq(h, chal) ? 0 : 8;
}
static int st_verify(const g1* ped, span raw, g1* ct) {
  span d[5];
  fe type, bf, chal;
  if (values(raw, d, 5, 0) != 4) return 1;
  if (!zr_el(d[0], &type) || !zr_el(d[1], &bf) || !zr_el(d[2], &chal) || !g1_el(d[3], ct)) return 1;
  g1 com = g1_add(g1_mul(ped[0], type), g1_mul(ped[2], bf));
  com = g1_sub(com, g1_mul(*ct, chal));
  g1 arr[2] = {*ct, com};
  return feq(hash_points(arr, 2), chal) ? 0 : 9;
}
static int action_one(const params* pp, const g1* ped, int kind, int nin, int nout, const uint8_t* in64,
                      const uint8_t* out64, span der, int32_t* idx) {
  g1 in[16], out[32], ct, coms[32];
  span v[3];
  *idx = -1;
  if (nin > 16 || nout > 32 || values(der, v, 3, 0) != 2 || v[0].n == 0) return 1;
  for (int i = 0; i < nin; i++)
    if (!g1_from_bytes(in64 + 64 * i, 64, &in[i])) return 1;
  for (int j = 0; j < nout; j++)
    if (!g1_from_bytes(out64 + 64 * j, 64, &out[j])) return 1;
  int sig = kind == 0 ? tas_verify(ped, in, nin, out, nout, v[0], &ct) : st_verify(ped, v[0], &ct);
  if (sig == 1) return 1;
  if (kind == 1 && sig) return sig; /* issue/verifier.go:40-43: SameType first */
  int rc = 0;
  if (kind == 1 || nin != 1 || nout != 1) {
    for (int j = 0; j < nout; j++) coms[j] = g1_sub(out[j], ct);
    if (v[1].n == 0) rc = 7;
    else rc = rc_verify(pp, coms, nout, v[1], idx);
  }
  if (sig) { /* transfer.go:192-196: the TypeAndSum error wins */
    *idx = -1;
    return sig;
  }
  if (rc == 1) *idx = -1;
  return rc;
}
typedef struct {
  const params* pp;
  g1 ped[3];
  const int32_t *kind, *nin, *nout;
  const uint8_t* const* in64;
  const uint8_t* const* out64;
  const uint8_t* const* ders;
  const size_t* lens;
  int32_t *status, *index;
  int count, next;
  pthread_mutex_t mu;
} act_job;
static void* act_worker(void* arg) {
  act_job* j = (act_job*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->count) return NULL;
    span s = {j->ders[i], j->lens[i]};
    j->status[i] = action_one(j->pp, j->ped, j->kind[i], j->nin[i], j->nout[i], j->in64[i], j->out64[i], s,
                              &j->index[i]);
  }
}
int oracle_action_verify_many(const uint8_t* ped, const uint8_t* gens, int n, int count, const int32_t* kind,
                              const int32_t* n_in, const int32_t* n_out, const uint8_t* const* in64,
                              const uint8_t* const* out64, const uint8_t* const* ders, const size_t* lens,
                              int threads, int32_t* status, int32_t* index) {
  params pp;
  if (!load_params(gens, n, &pp)) return -1;
  act_job j;
  for (int q = 0; q < 3; q++)
    if (!g1_from_bytes(ped + 64 * q, 64, &j.ped[q])) return -1;
  j.pp = &pp;
  j.kind = kind;
  j.nin = n_in;
  j.nout = n_out;
  j.in64 = in64;
  j.out64 = out64;
  j.ders = ders;
  j.lens = lens;
  j.status = status;
  j.index = index;
  j.count = count;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, act_worker, &j);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  free(pp.L);
  free(pp.R);
  return 0;
}
