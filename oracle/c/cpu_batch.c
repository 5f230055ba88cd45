/*
 * CPU BASELINE (test infrastructure + bench.py cpu_baseline only; never shipped,
 * never linked by the product).
 *
 * The "optimized CPU batch" column of SURVEY §8(d): the device's batch
 * algorithm on host threads, so the GPU number has an honest
 * CPU comparison beside the reference-order restatement in ref_verify.c.
 * Per proof (rp/bulletproof.go:252-333, 469-509; rp/ipa.go:190-262):
 *   - challenges x, y, z, polEval and the IPA challenges x_j, exact;
 *   - H'_i = y^-i H_i, z K and -delta P as fixed-base products over
 *     signed-window affine tables (K = sum H_i - sum G_i folds the z terms of
 *     com, as on the device);
 *   - S = sum_i 2^i H'_i by Horner, com = C + z K - delta P + x D + z^2 S with
 *     one GLV/Straus chain over D, phi(D), S, phi(S);
 *   - the x0 transcript over the exact H'_i and com (ipa.go:200-218).
 * Per batch: E1 and E2 (the IPA's final equation with G_fin = sum s_i G_i,
 * H'_fin = sum s_i^-1 H'_i unrolled) of every proof folded into ONE random
 * linear combination: fixed-base columns G, H, Q, G_i, H_i summed over the
 * batch, plus one Pippenger MSM (GLV split, signed digits) over T1, T2, V,
 * com, L_j, R_j.  A failing combination is bisected (each half's own
 * combination) down to groups of 4, whose proofs are re-verified in reference
 * order (verify_one): those are the reference's verdicts.  Proofs with IPA
 * structure errors go to verify_one directly (their verdict depends on E1
 * first).
 *
 * Entry points (ctypes, oracle/cref.py):
 *   void* cpu_batch_create(const uint8_t* gens, int n, int window_bits, int threads)
 *   int   cpu_batch_verify(void* ctx, int count, const uint8_t* coms, const uint8_t* const* ders,
 *                          const size_t* lens, int threads, int32_t* out)
 *         -> number of proofs that took the per-proof fallback, or -1
 *   int   cpu_batch_verify_ex(..., uint8_t* com_out, uint8_t* x0_out)
 *         the same, plus every proof's exact com (64 B) and x0 (32 B, BE) for
 *         parity checks at full batch size (zeros where the proof stopped earlier)
 *   void  cpu_batch_free(void* ctx)
 *   int   cpu_msm_pippenger(const uint8_t* pts, const uint8_t* scs, size_t n, int threads, uint8_t* out64)
 *         sum_i (k_i mod r) P_i with the batch's GLV Pippenger (msm_glv): the C3
 *         CPU baseline (BASELINE.md "the build's C++ Pippenger"); pts as oracle_msm
 *         (64-byte BE, NewG1FromBytes checks), scs 32-byte BE.  0, or -1 on a bad point
 * gens as in ref_verify.c: [G=ped1, H=ped2, P, Q, G_0..G_{n-1}, H_0..H_{n-1}].
 */
#include "ref_verify.c"

#include <stdatomic.h>
#include <sys/random.h>

typedef struct { fe x, y; } aff; /* affine, never the point at infinity */

/* ------------------------------------------------------------ point helpers */
/* p + q, q affine (madd-2007-bl) */
static g1j jmadd(g1j p, const aff* q) {
  if (fzero(p.z)) {
    g1j r = {q->x, q->y, P_ONE};
    return r;
  }
  fe z1z1 = PMUL(p.z, p.z);
  fe u2 = PMUL(q->x, z1z1);
  fe s2 = PMUL(PMUL(q->y, p.z), z1z1);
  fe h = PSUB(u2, p.x);
  fe rr = PSUB(s2, p.y);
  if (fzero(h)) return fzero(rr) ? jdbl(p) : jid();
  fe hh = PMUL(h, h);
  fe i = PADD(hh, hh);
  i = PADD(i, i);
  fe j = PMUL(h, i);
  rr = PADD(rr, rr);
  fe v = PMUL(p.x, i);
  g1j r;
  r.x = PSUB(PSUB(PMUL(rr, rr), j), PADD(v, v));
  fe yj = PMUL(p.y, j);
  r.y = PSUB(PMUL(rr, PSUB(v, r.x)), PADD(yj, yj));
  fe zh = PADD(p.z, h);
  r.z = PSUB(PSUB(PMUL(zh, zh), z1z1), hh);
  return r;
}
static aff aneg(aff a) {
  fe z = {{0, 0, 0, 0}};
  a.y = PSUB(z, a.y);
  return a;
}
/* Montgomery's trick: m Jacobian points -> affine (inf[i] set for z = 0) */
static void batch_norm(const g1j* in, aff* out, int* inf, int m, fe* pre) {
  fe acc = P_ONE;
  for (int i = 0; i < m; i++) {
    pre[i] = acc;
    if (!fzero(in[i].z)) acc = PMUL(acc, in[i].z);
  }
  fe inv = finv(acc, PM, PINV, PR2);
  for (int i = m - 1; i >= 0; i--) {
    if (fzero(in[i].z)) {
      if (inf) inf[i] = 1;
      continue;
    }
    if (inf) inf[i] = 0;
    fe zi = PMUL(inv, pre[i]);
    inv = PMUL(inv, in[i].z);
    fe zi2 = PMUL(zi, zi);
    out[i].x = PMUL(in[i].x, zi2);
    out[i].y = PMUL(PMUL(in[i].y, zi2), zi);
  }
}
static int is_inf_j(g1j p) { return fzero(p.z); }

/* ------------------------------------------------------------ scalars */
/* bits [pos, pos + w) of a 4 x 64-bit integer (w <= 32) */
static uint32_t bits_at(const uint64_t* k, int nlimb, int pos, int w) {
  int li = pos >> 6, sh = pos & 63;
  if (li >= nlimb) return 0;
  unsigned __int128 v = k[li] >> sh;
  if (sh && li + 1 < nlimb) v |= (unsigned __int128)k[li + 1] << (64 - sh);
  return (uint32_t)(v & ((1ull << w) - 1));
}
/* signed digits of width w: k = sum d_i 2^(w i), |d_i| <= 2^(w-1) */
static void signed_digits(const uint64_t* k, int nlimb, int w, int nwin, int32_t* d) {
  uint32_t carry = 0;
  for (int i = 0; i < nwin; i++) {
    uint32_t v = bits_at(k, nlimb, i * w, w) + carry;
    carry = 0;
    if (v > (1u << (w - 1))) {
      d[i] = (int32_t)v - (1 << w);
      carry = 1;
    } else {
      d[i] = (int32_t)v;
    }
  }
}

/* GLV of BN254 G1 (phi(x, y) = (beta x, y) = lambda (x, y)): k = k1 + k2 lambda
 * mod r, |k1|, |k2| < 2^128, by Babai rounding with g_i = floor(2^384 b_i / r)
 * (the constants of the device's glv.hpp, derived from the curve). */
static const uint32_t GLV_G1[7] = {0x2fafba64u, 0x8fa7d32du, 0x773a6ef2u, 0x6eb9c714u, 0xc7e0b3d7u, 0xd91d232eu, 2u};
static const uint32_t GLV_G2[9] = {0x9b9bdffau, 0x86937516u, 0x5eaa26d9u, 0xa5e38cfbu, 0x391eb18du,
                                   0x7a7bd9d4u, 0xa773d2cfu, 0x4ccef014u, 2u};
static const uint32_t GLV_A1[2] = {0x94d213e3u, 0x89d32568u};
static const uint32_t GLV_A2[4] = {0x1221250bu, 0x0be4e154u, 0xeeb859fdu, 0x6f4d8248u};
static const uint32_t GLV_NB1[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u};
static const uint32_t GLV_BETA[8] = {0xd782e155u, 0x71930c11u, 0xffbe3323u, 0xa6bb947cu,
                                     0xd4741444u, 0xaa303344u, 0x26594943u, 0x2c3b3f0du}; /* Montgomery */

static void glv_round_c(const uint32_t k[8], const uint32_t* g, int G, uint32_t c[5]) {
  uint32_t t[17] = {0};
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < G; j++) {
      uint64_t v = (uint64_t)k[i] * g[j] + t[i + j] + carry;
      t[i + j] = (uint32_t)v;
      carry = v >> 32;
    }
    t[i + G] = (uint32_t)carry;
  }
  uint64_t cy = t[11] >> 31;
  for (int i = 0; i < 5; i++) {
    uint64_t v = (uint64_t)(12 + i < 8 + G ? t[12 + i] : 0u) + cy;
    c[i] = (uint32_t)v;
    cy = v >> 32;
  }
}
static void sub_mul_c(uint32_t r[8], const uint32_t* a, int NA, const uint32_t* b, int NB) {
  uint32_t p[8] = {0};
  for (int i = 0; i < NA; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < NB; j++)
      if (i + j < 8) {
        uint64_t v = (uint64_t)a[i] * b[j] + p[i + j] + carry;
        p[i + j] = (uint32_t)v;
        carry = v >> 32;
      }
    if (i + NB < 8) p[i + NB] = (uint32_t)carry;
  }
  uint64_t bw = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)r[i] - p[i] - bw;
    r[i] = (uint32_t)v;
    bw = (v >> 32) & 1;
  }
}
static int glv_abs_c(const uint32_t v[8], uint64_t out[2]) {
  int neg = v[7] >> 31;
  uint32_t o[4];
  uint64_t c = neg;
  for (int i = 0; i < 4; i++) {
    uint64_t x = (uint64_t)(neg ? ~v[i] : v[i]) + c;
    o[i] = (uint32_t)x;
    c = x >> 32;
  }
  out[0] = o[0] | ((uint64_t)o[1] << 32);
  out[1] = o[2] | ((uint64_t)o[3] << 32);
  return neg;
}
/* k canonical (< r) -> |k1|, |k2| (2 limbs each) and their signs */
static void glv_split(fe k, uint64_t k1[2], int* s1, uint64_t k2[2], int* s2) {
  uint32_t kw[8], c1[5], c2[5], r1[8], r2[8] = {0}, p[8] = {0};
  for (int i = 0; i < 4; i++) kw[2 * i] = (uint32_t)k.v[i], kw[2 * i + 1] = (uint32_t)(k.v[i] >> 32);
  glv_round_c(kw, GLV_G1, 7, c1);
  glv_round_c(kw, GLV_G2, 9, c2);
  memcpy(r1, kw, 32);
  sub_mul_c(r1, c1, 3, GLV_A1, 2);
  sub_mul_c(r1, c2, 5, GLV_A2, 4);
  sub_mul_c(r2, c2, 5, GLV_A1, 2);
  sub_mul_c(p, c1, 3, GLV_NB1, 4);
  uint64_t bw = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)r2[i] - p[i] - bw;
    r2[i] = (uint32_t)v;
    bw = (v >> 32) & 1;
  }
  *s1 = glv_abs_c(r1, k1);
  *s2 = glv_abs_c(r2, k2);
}
static fe glv_beta(void) {
  fe b;
  for (int i = 0; i < 4; i++) b.v[i] = GLV_BETA[2 * i] | ((uint64_t)GLV_BETA[2 * i + 1] << 32);
  return b;
}

/* ------------------------------------------------------------ SHA-256 over a buffer */
static void sha_compress(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha256_buf(const uint8_t* m, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha_compress(h, m + i);
  uint8_t blk[128] = {0};
  size_t r = len - i;
  memcpy(blk, m + i, r);
  blk[r] = 0x80;
  size_t nb = r + 9 <= 64 ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int q = 0; q < 8; q++) blk[nb - 1 - q] = (uint8_t)(bits >> (8 * q));
  sha_compress(h, blk);
  if (nb == 128) sha_compress(h, blk + 64);
  for (int q = 0; q < 8; q++) {
    out[4 * q] = h[q] >> 24;
    out[4 * q + 1] = h[q] >> 16;
    out[4 * q + 2] = h[q] >> 8;
    out[4 * q + 3] = h[q];
  }
}
static void hex_point_aff(const aff* a, int inf, uint8_t* out128) {
  static const char* hx = "0123456789abcdef";
  uint8_t b[64];
  if (inf) memset(b, 0, 64);
  else {
    fe_to_be(ffrommont(a->x, PM, PINV), b);
    fe_to_be(ffrommont(a->y, PM, PINV), b + 32);
  }
  for (int q = 0; q < 64; q++) {
    out128[2 * q] = hx[b[q] >> 4];
    out128[2 * q + 1] = hx[b[q] & 15];
  }
}
static void hex_g1(g1 p, uint8_t* out128) {
  aff a = {p.x, p.y};
  hex_point_aff(&a, p.inf, out128);
}
/* Curve.HashToZr over a G1Array of m points (array.go:25-36) */
static fe hash_g1s(const g1* pts, int m) {
  uint8_t buf[130 * 4], d[32];
  size_t o = 0;
  for (int i = 0; i < m; i++) {
    if (i) buf[o++] = '|', buf[o++] = '|';
    hex_g1(pts[i], buf + o);
    o += 128;
  }
  sha256_buf(buf, o, d);
  return digest_zr(d);
}

/* ------------------------------------------------------------ fixed-base tables */
typedef struct {
  int W, nwin, half; /* window bits, windows, entries per window (2^(W-1)) */
  aff* t;            /* [base][win][half]: (e + 1) 2^(W win) B */
} fbtab;

static void fb_build_one(const fbtab* T, int bi, g1 B) {
  aff* out = T->t + (size_t)bi * T->nwin * T->half;
  g1j* jac = malloc(sizeof(g1j) * T->half);
  fe* pre = malloc(sizeof(fe) * T->half);
  aff base = {B.x, B.y};
  for (int w = 0; w < T->nwin; w++) {
    g1j acc = jid();
    for (int e = 0; e < T->half; e++) {
      acc = jmadd(acc, &base);
      jac[e] = acc;
    }
    batch_norm(jac, out + (size_t)w * T->half, NULL, T->half, pre);
    /* next window base: 2^W B_w = 2 * (2^(W-1) B_w) */
    g1j nb = jdbl(jac[T->half - 1]);
    g1 na = toaff(nb);
    base.x = na.x;
    base.y = na.y;
  }
  free(jac);
  free(pre);
}
static g1j fb_mul(const fbtab* T, int bi, fe k /* canonical < r */) {
  int32_t d[40];
  signed_digits(k.v, 4, T->W, T->nwin, d);
  const aff* tb = T->t + (size_t)bi * T->nwin * T->half;
  g1j acc = jid();
  for (int w = 0; w < T->nwin; w++) {
    if (!d[w]) continue;
    const aff* e = tb + (size_t)w * T->half + (abs(d[w]) - 1);
    if (d[w] < 0) {
      aff ne = aneg(*e);
      acc = jmadd(acc, &ne);
    } else {
      acc = jmadd(acc, e);
    }
  }
  return acc;
}

/* ------------------------------------------------------------ context */
enum { B_G = 0, B_H = 1, B_P = 2, B_Q = 3, B_K = 4 }; /* table bases; then G_i at 5.., H_i at 5+n.. */
typedef struct {
  params pp;
  int n, k, nb;
  fbtab T;
  uint8_t* x0_tmpl; /* x0 message with the G_i and Q records filled in */
  size_t x0_len;
} cpu_ctx;

typedef struct {
  cpu_ctx* c;
  g1* bases;
  atomic_int next;
} build_job;
static void* build_worker(void* arg) {
  build_job* j = arg;
  for (;;) {
    int i = atomic_fetch_add(&j->next, 1);
    if (i >= j->c->nb) return NULL;
    fb_build_one(&j->c->T, i, j->bases[i]);
  }
}
static void run_threads(int threads, void* (*fn)(void*), void* arg) {
  if (threads < 1) threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, fn, arg);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
}

void cpu_batch_free(void* p) {
  cpu_ctx* c = p;
  if (!c) return;
  free(c->T.t);
  free(c->x0_tmpl);
  free(c->pp.L);
  free(c->pp.R);
  free(c);
}

void* cpu_batch_create(const uint8_t* gens, int n, int window_bits, int threads) {
  if (n < 2 || n > 64 || (n & (n - 1)) || window_bits < 4 || window_bits > 16) return NULL;
  cpu_ctx* c = calloc(1, sizeof *c);
  if (!load_params(gens, n, &c->pp)) {
    cpu_batch_free(c);
    return NULL;
  }
  c->n = n;
  c->k = c->pp.k;
  c->nb = 5 + 2 * n;
  c->T.W = window_bits;
  c->T.nwin = 254 / window_bits + 1;
  c->T.half = 1 << (window_bits - 1);
  c->T.t = malloc(sizeof(aff) * (size_t)c->nb * c->T.nwin * c->T.half);
  g1* bases = malloc(sizeof(g1) * c->nb);
  bases[B_G] = c->pp.G;
  bases[B_H] = c->pp.H;
  bases[B_P] = c->pp.P;
  bases[B_Q] = c->pp.Q;
  /* K = sum H_i - sum G_i (bulletproof.go:477-492: the z terms of com) */
  g1j K = jid();
  for (int i = 0; i < n; i++) {
    K = jadd(K, tojac(c->pp.R[i]));
    K = jadd(K, tojac(g1_neg(c->pp.L[i])));
  }
  bases[B_K] = toaff(K);
  for (int i = 0; i < n; i++) bases[5 + i] = c->pp.L[i], bases[5 + n + i] = c->pp.R[i];
  for (int i = 0; i < c->nb; i++)
    if (bases[i].inf) { /* a generator at infinity: no table (not a valid PP) */
      free(bases);
      cpu_batch_free(c);
      return NULL;
    }
  build_job bj = {c, bases};
  atomic_init(&bj.next, 0);
  run_threads(threads, build_worker, &bj);
  free(bases);
  /* x0 message template (ipa.go:200-218) */
  size_t alen = 130 * (size_t)(2 * n + 2) - 2, seqc = (4 + alen) + 4 + 34;
  c->x0_len = 8 + alen + 6 + 32;
  c->x0_tmpl = calloc(1, c->x0_len);
  uint8_t* m = c->x0_tmpl;
  uint8_t hdr[8] = {0x30, 0x82, (uint8_t)(seqc >> 8), (uint8_t)seqc, 0x04, 0x82, (uint8_t)(alen >> 8), (uint8_t)alen};
  memcpy(m, hdr, 8);
  for (int r = 0; r < 2 * n + 2; r++) {
    uint8_t* rec = m + 8 + 130 * (size_t)r;
    if (r) rec[-2] = '|', rec[-1] = '|';
    if (r >= n && r < 2 * n) hex_g1(c->pp.L[r - n], rec);
    if (r == 2 * n) hex_g1(c->pp.Q, rec);
  }
  uint8_t tail[6] = {0x04, 0x02, '|', '|', 0x04, 0x20};
  memcpy(m + 8 + alen, tail, 6);
  return c;
}

/* ------------------------------------------------------------ per-proof phase */
#define MAXK 6
typedef struct {
  cpu_ctx* c;
  int count;
  const uint8_t* coms;
  const uint8_t* const* ders;
  const size_t* lens;
  int32_t* out;
  int npv;          /* variable points per proof: 4 + 2k */
  aff* vpts;        /* [count][npv] */
  uint8_t* vinf;    /* [count][npv] */
  fe* vsc;          /* [count][npv] canonical scalars */
  uint8_t* live;    /* [count]: in the combination */
  fe* col;          /* [count][5 + 2n]: the proof's column scalars (table base order) */
  uint64_t rng_key[4];
  uint8_t* com_out; /* optional [count][64]: com (BE x || y) of every proof that reached it */
  uint8_t* x0_out;  /* optional [count][32]: x0 (BE) */
  atomic_int next, tid;
} batch_job;

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
/* batch weight w_(i, which): keyed hash of the proof index, reduced mod r */
static fe weight(const batch_job* j, int i, int which) {
  fe r;
  for (int q = 0; q < 4; q++)
    r.v[q] = mix64(j->rng_key[q] ^ mix64(((uint64_t)i << 8) ^ ((uint64_t)which << 4) ^ (uint64_t)q));
  return zr_red(r);
}
static fe zneg(fe a) { return RSUB(zr_u64(0), a); }
static fe zmont(fe a) { return ftomont(a, RM, RINV, RR2); }

/* one proof: exact transcript values, com, and its share of the combination.
 * Returns 0 (joined the combination) or a final status. */
static int proof_phase(batch_job* j, int i, fe* cs, uint8_t* x0buf, g1j* jtmp, aff* atmp, fe* ftmp) {
  cpu_ctx* c = j->c;
  const int n = c->n, k = c->k;
  g1 V;
  if (!g1_from_bytes(j->coms + 64 * (size_t)i, 64, &V)) return 1;
  span sp = {j->ders[i], j->lens[i]};
  rp_parsed P;
  int pe = parse_rp(sp, &P);
  if (pe) return pe;
  if (P.ipa_err || P.nl != k || P.nr != k) return -1; /* verify_one decides (E1 first) */
  /* challenges (bulletproof.go:266-311) */
  g1 arr[3] = {P.T1, P.T2};
  fe x = hash_g1s(arr, 2), x2 = zr_mul(x, x);
  arr[0] = P.C, arr[1] = P.D, arr[2] = V;
  fe y = hash_g1s(arr, 3);
  uint8_t yb[32], dg[32];
  fe_to_be(y, yb);
  sha256_buf(yb, 32, dg);
  fe z = digest_zr(dg), z2 = zr_mul(z, z), z3 = zr_mul(z2, z);
  /* sum_{i<n} y^i by doubling; sum 2^i = 2^n - 1 */
  fe ym = zmont(y), ipy = zr_u64(1), yp = y;
  for (int m = 1; m < n; m *= 2) { /* ipy = sum_{i<m} y^i, yp = y^m */
    ipy = RADD(ipy, RMUL(zmont(ipy), yp));
    yp = RMUL(zmont(yp), yp);
  }
  fe ip2 = RSUB(n == 64 ? zr_u64(0) : zr_u64(1ull << n), zr_u64(1));
  if (n == 64) { /* 2^64 - 1 */
    ip2 = zr_u64(~0ull);
  }
  fe pol = RSUB(zr_mul(RSUB(z, z2), ipy), zr_mul(z3, ip2));
  /* IPA challenges x_j (ipa.go:224-230) */
  fe xj[MAXK], xjinv[MAXK], inv_in[MAXK + 1], inv_out[MAXK + 1];
  for (int q = 0; q < k; q++) {
    g1 lr[2] = {P.Ls[q], P.Rs[q]};
    xj[q] = hash_g1s(lr, 2);
  }
  /* one inversion for y and every x_j (Montgomery's trick, Montgomery form) */
  inv_in[0] = ym;
  for (int q = 0; q < k; q++) inv_in[q + 1] = zmont(xj[q]);
  {
    fe acc = zmont(zr_u64(1)), pre[MAXK + 1];
    for (int q = 0; q <= k; q++) {
      pre[q] = acc;
      acc = RMUL(acc, inv_in[q]);
    }
    fe iv = finv(acc, RM, RINV, RR2);
    for (int q = k; q >= 0; q--) {
      inv_out[q] = RMUL(iv, pre[q]);
      iv = RMUL(iv, inv_in[q]);
    }
  }
  fe yinv = ffrommont(inv_out[0], RM, RINV);
  for (int q = 0; q < k; q++) xjinv[q] = ffrommont(inv_out[q + 1], RM, RINV);
  if (fzero(y)) return -1; /* no inverse: leave it to the reference order */
  for (int q = 0; q < k; q++)
    if (fzero(xj[q])) return -1;
  /* H'_i = y^-i H_i, z K, -delta P (fixed base) */
  fe delta = zr_red(P.delta), ipv = zr_red(P.ipv), a = zr_red(P.a), b = zr_red(P.b), tau = zr_red(P.tau);
  fe* ypinv = ftmp; /* y^-i, canonical */
  ypinv[0] = zr_u64(1);
  fe yim = zmont(yinv);
  for (int q = 1; q < n; q++) ypinv[q] = RMUL(yim, ypinv[q - 1]);
  for (int q = 0; q < n; q++) jtmp[q] = fb_mul(&c->T, 5 + n + q, ypinv[q]);
  g1j zK = fb_mul(&c->T, B_K, z), dP = fb_mul(&c->T, B_P, zneg(delta));
  /* affine H' (one inversion), then S = sum 2^i H'_i by Horner */
  int* hinf = (int*)(ftmp + 2 * n);
  batch_norm(jtmp, atmp, hinf, n, ftmp + n);
  g1j S = jid();
  for (int q = n - 1; q >= 0; q--) {
    S = jdbl(S);
    if (!hinf[q]) S = jmadd(S, &atmp[q]);
  }
  /* x D + z^2 S: GLV/Straus over D, phi D, S, phi S, signed 4-bit windows */
  g1j acc = jid();
  {
    uint64_t kx[2][2], kw[2][2];
    int sx[2], sw[2];
    glv_split(x, kx[0], &sx[0], kx[1], &sx[1]);
    glv_split(z2, kw[0], &sw[0], kw[1], &sw[1]);
    int haveD = !P.D.inf, haveS = !is_inf_j(S);
    g1j tj[16];
    aff tab[16];
    fe pre[16];
    g1j Dj = tojac(P.D);
    for (int e = 0; e < 8; e++) {
      tj[e] = e == 0 ? Dj : (haveD ? jadd(tj[e - 1], Dj) : jid());
      tj[8 + e] = e == 0 ? S : (haveS ? jadd(tj[7 + e], S) : jid());
    }
    if (!haveD)
      for (int e = 0; e < 8; e++) tj[e] = tojac(c->pp.G); /* unused placeholders */
    if (!haveS)
      for (int e = 0; e < 8; e++) tj[8 + e] = tojac(c->pp.G);
    batch_norm(tj, tab, NULL, 16, pre);
    fe beta = glv_beta();
    aff tphi[16];
    for (int e = 0; e < 16; e++) tphi[e].x = PMUL(tab[e].x, beta), tphi[e].y = tab[e].y;
    int32_t dg4[4][40];
    const uint64_t* ks[4] = {kx[0], kx[1], kw[0], kw[1]};
    int sg[4] = {sx[0], sx[1], sw[0], sw[1]};
    const aff* tb[4] = {tab, tphi, tab + 8, tphi + 8};
    int use[4] = {haveD, haveD, haveS, haveS};
    const int NW = 33;
    for (int q = 0; q < 4; q++) signed_digits(ks[q], 2, 4, NW, dg4[q]);
    for (int w = NW - 1; w >= 0; w--) {
      for (int r = 0; r < 4; r++) acc = jdbl(acc);
      for (int q = 0; q < 4; q++) {
        int dd = dg4[q][w];
        if (!use[q] || !dd) continue;
        aff e = tb[q][abs(dd) - 1];
        if ((dd < 0) ^ sg[q]) e = aneg(e);
        acc = jmadd(acc, &e);
      }
    }
  }
  acc = jadd(acc, zK);
  acc = jadd(acc, dP);
  acc = jadd(acc, tojac(P.C));
  g1 com = toaff(acc);
  /* x0 (ipa.go:200-218) */
  memcpy(x0buf, c->x0_tmpl, c->x0_len);
  for (int q = 0; q < n; q++) hex_point_aff(&atmp[q], hinf[q], x0buf + 8 + 130 * (size_t)q);
  hex_g1(com, x0buf + 8 + 130 * (size_t)(2 * n + 1));
  fe_to_be(ipv, x0buf + c->x0_len - 32);
  sha256_buf(x0buf, c->x0_len, dg);
  fe x0 = digest_zr(dg);
  if (j->com_out) g1_bytes(com, j->com_out + 64 * (size_t)i);
  if (j->x0_out) fe_to_be(x0, j->x0_out + 32 * (size_t)i);
  /* the proof's share of sum_p rho_p E1_p + rho'_p E2_p = O */
  fe rho = weight(j, i, 0), rho2 = weight(j, i, 1), rhom = zmont(rho), rho2m = zmont(rho2);
  aff* vp = j->vpts + (size_t)i * j->npv;
  uint8_t* vi = j->vinf + (size_t)i * j->npv;
  fe* vs = j->vsc + (size_t)i * j->npv;
  g1 pts[4] = {P.T1, P.T2, V, com};
  fe scs[4] = {zneg(RMUL(rhom, x)), zneg(RMUL(rhom, x2)), zneg(RMUL(rhom, z2)), zneg(rho2)};
  for (int q = 0; q < 4; q++) {
    vp[q].x = pts[q].x, vp[q].y = pts[q].y, vi[q] = (uint8_t)pts[q].inf, vs[q] = scs[q];
  }
  for (int q = 0; q < k; q++) {
    fe x2j = zr_mul(xj[q], xj[q]), x2ji = zr_mul(xjinv[q], xjinv[q]);
    vp[4 + q].x = P.Ls[q].x, vp[4 + q].y = P.Ls[q].y, vi[4 + q] = (uint8_t)P.Ls[q].inf;
    vs[4 + q] = zneg(RMUL(rho2m, x2j));
    vp[4 + k + q].x = P.Rs[q].x, vp[4 + k + q].y = P.Rs[q].y, vi[4 + k + q] = (uint8_t)P.Rs[q].inf;
    vs[4 + k + q] = zneg(RMUL(rho2m, x2ji));
  }
  /* fixed columns: G rho (ip - pol), H rho tau, Q rho' (ab - ip) x0,
   * G_i rho' a s_i, H_i rho' b s_i^-1 y^-i  (s_i = prod_j x_j^(+-1), ipa.go:343-356) */
  cs[B_G] = RADD(cs[B_G], RMUL(rhom, RSUB(ipv, pol)));
  cs[B_H] = RADD(cs[B_H], RMUL(rhom, tau));
  cs[B_Q] = RADD(cs[B_Q], RMUL(rho2m, zr_mul(RSUB(zr_mul(a, b), ipv), x0)));
  fe* s = ftmp + n;     /* s_i (Montgomery) */
  fe* si = ftmp + 2 * n; /* s_i^-1 (Montgomery) -- hinf no longer needed */
  fe one = zmont(zr_u64(1)), sx0 = one, sxi0 = one;
  fe xsq[MAXK], xisq[MAXK];
  for (int q = 0; q < k; q++) {
    sx0 = RMUL(sx0, inv_out[q + 1]);  /* prod x_j^-1 */
    sxi0 = RMUL(sxi0, inv_in[q + 1]); /* prod x_j */
    xsq[q] = RMUL(inv_in[q + 1], inv_in[q + 1]);
    xisq[q] = RMUL(inv_out[q + 1], inv_out[q + 1]);
  }
  s[0] = sx0, si[0] = sxi0;
  for (int q = 1; q < n; q++) {
    int bpos = __builtin_ctz(q), jj = k - 1 - bpos;
    s[q] = RMUL(s[q - (1 << bpos)], xsq[jj]);
    si[q] = RMUL(si[q - (1 << bpos)], xisq[jj]);
  }
  fe ra = RMUL(rho2m, a), rb = RMUL(rho2m, b); /* canonical */
  fe ram = zmont(ra), rbm = zmont(rb);
  for (int q = 0; q < n; q++) {
    fe sq = ffrommont(s[q], RM, RINV), siq = ffrommont(si[q], RM, RINV);
    cs[5 + q] = RADD(cs[5 + q], RMUL(ram, sq));
    cs[5 + n + q] = RADD(cs[5 + n + q], RMUL(rbm, RMUL(zmont(siq), ypinv[q])));
  }
  return 0;
}

static void* proof_worker(void* arg) {
  batch_job* j = arg;
  cpu_ctx* c = j->c;
  uint8_t* x0buf = malloc(c->x0_len);
  g1j* jtmp = malloc(sizeof(g1j) * c->n);
  aff* atmp = malloc(sizeof(aff) * c->n);
  fe* ftmp = malloc(sizeof(fe) * 3 * c->n + 64);
  for (;;) {
    int i = atomic_fetch_add(&j->next, 1);
    if (i >= j->count) break;
    fe* cs = j->col + (size_t)i * c->nb;
    for (int q = 0; q < c->nb; q++) cs[q] = zr_u64(0);
    int r = proof_phase(j, i, cs, x0buf, jtmp, atmp, ftmp);
    j->live[i] = r == 0;
    if (r < 0) {
      g1 V;
      span sp = {j->ders[i], j->lens[i]};
      r = g1_from_bytes(j->coms + 64 * (size_t)i, 64, &V) ? verify_one(&c->pp, V, sp) : 1;
    }
    j->out[i] = r;
  }
  free(x0buf);
  free(jtmp);
  free(atmp);
  free(ftmp);
  return NULL;
}

/* ------------------------------------------------------------ Pippenger over GLV halves */
typedef struct {
  int npts, c, nwin, parts;
  const aff* pts; /* 2 per variable point: P, phi(P) (sign folded into y) */
  const int16_t* dig; /* [npts][nwin] */
  g1j* res;           /* [nwin][parts] */
  atomic_int next;
} pip_job;
static void* pip_worker(void* arg) {
  pip_job* m = arg;
  const int half = 1 << (m->c - 1);
  g1j* bk = malloc(sizeof(g1j) * half);
  for (;;) {
    int task = atomic_fetch_add(&m->next, 1);
    if (task >= m->nwin * m->parts) break;
    int w = task / m->parts, p = task % m->parts;
    for (int b = 0; b < half; b++) bk[b] = jid();
    size_t lo = (size_t)m->npts * p / m->parts, hi = (size_t)m->npts * (p + 1) / m->parts;
    for (size_t i = lo; i < hi; i++) {
      int d = m->dig[i * m->nwin + w];
      if (!d) continue;
      if (d > 0) bk[d - 1] = jmadd(bk[d - 1], &m->pts[i]);
      else {
        aff ne = aneg(m->pts[i]);
        bk[-d - 1] = jmadd(bk[-d - 1], &ne);
      }
    }
    g1j run = jid(), tot = jid();
    for (int b = half - 1; b >= 0; b--) {
      run = jadd(run, bk[b]);
      tot = jadd(tot, run);
    }
    m->res[task] = tot;
  }
  free(bk);
  return NULL;
}

static g1j msm_glv(const aff* pts, const uint8_t* inf, const fe* sc, size_t N, int threads) {
  size_t M = 0;
  for (size_t i = 0; i < N; i++) M += !inf[i] && !fzero(sc[i]);
  if (!M) return jid();
  /* c <= 15: a signed digit reaches +2^(c-1), which must fit the int16_t digit table
   * (c = 16 wrapped +32768 to -32768: wrong sums from ~2^18 points on, round 5) */
  int c = 4;
  while (c < 15 && ((size_t)1 << (c + 3)) < 2 * M) c++;
  const int nwin = 128 / c + 1;
  aff* gp = malloc(sizeof(aff) * 2 * M);
  int16_t* dig = malloc(sizeof(int16_t) * 2 * M * nwin);
  fe beta = glv_beta();
  size_t o = 0;
  for (size_t i = 0; i < N; i++) {
    if (inf[i] || fzero(sc[i])) continue;
    uint64_t k1[2], k2[2];
    int s1, s2;
    glv_split(sc[i], k1, &s1, k2, &s2);
    gp[o] = s1 ? aneg(pts[i]) : pts[i];
    aff ph = {PMUL(pts[i].x, beta), pts[i].y};
    gp[o + 1] = s2 ? aneg(ph) : ph;
    int32_t d[40];
    signed_digits(k1, 2, c, nwin, d);
    for (int w = 0; w < nwin; w++) dig[o * nwin + w] = (int16_t)d[w];
    signed_digits(k2, 2, c, nwin, d);
    for (int w = 0; w < nwin; w++) dig[(o + 1) * nwin + w] = (int16_t)d[w];
    o += 2;
  }
  pip_job mj = {(int)o, c, nwin, 1, gp, dig, NULL};
  if (threads < 1) threads = 1;
  mj.parts = (threads + nwin - 1) / nwin;
  if ((size_t)mj.parts * 64 > o) mj.parts = 1;
  mj.res = malloc(sizeof(g1j) * nwin * mj.parts);
  atomic_init(&mj.next, 0);
  run_threads(threads < nwin * mj.parts ? threads : nwin * mj.parts, pip_worker, &mj);
  g1j acc = jid();
  for (int w = nwin - 1; w >= 0; w--) {
    for (int q = 0; q < c; q++) acc = jdbl(acc);
    for (int p = 0; p < mj.parts; p++) acc = jadd(acc, mj.res[w * mj.parts + p]);
  }
  free(gp);
  free(dig);
  free(mj.res);
  return acc;
}

/* per-proof reference-order verdicts for the live proofs of [lo, hi) */
typedef struct {
  cpu_ctx* c;
  batch_job* b;
  int lo, hi;
  atomic_int next;
} fb_job;
static void* fb_worker(void* arg) {
  fb_job* f = arg;
  batch_job* j = f->b;
  for (;;) {
    int i = f->lo + atomic_fetch_add(&f->next, 1);
    if (i >= f->hi) return NULL;
    if (!j->live[i]) continue;
    g1 V;
    span sp = {j->ders[i], j->lens[i]};
    j->out[i] = g1_from_bytes(j->coms + 64 * (size_t)i, 64, &V) ? verify_one(&f->c->pp, V, sp) : 1;
  }
}

/* does the combination of the live proofs in [lo, hi) close? */
static int group_closes(batch_job* j, int lo, int hi, int threads) {
  cpu_ctx* c = j->c;
  size_t o = (size_t)lo * j->npv;
  g1j acc = msm_glv(j->vpts + o, j->vinf + o, j->vsc + o, (size_t)(hi - lo) * j->npv, threads);
  for (int b = 0; b < c->nb; b++) {
    fe s = zr_u64(0);
    for (int i = lo; i < hi; i++)
      if (j->live[i]) s = RADD(s, j->col[(size_t)i * c->nb + b]);
    if (!fzero(s)) acc = jadd(acc, fb_mul(&c->T, b, s));
  }
  return is_inf_j(acc);
}
/* [lo, hi) failed: bisect down to groups of 4, whose live proofs get the
 * reference-order verdicts ("fall back to per-proof checks
 * (bisection)") */
static int bisect(batch_job* j, int lo, int hi, int threads) {
  if (hi - lo <= 4) {
    fb_job f = {j->c, j, lo, hi};
    atomic_init(&f.next, 0);
    run_threads(threads < hi - lo ? threads : hi - lo, fb_worker, &f);
    int m = 0;
    for (int i = lo; i < hi; i++) m += j->live[i];
    return m;
  }
  int mid = lo + (hi - lo) / 2, m = 0;
  if (!group_closes(j, lo, mid, threads)) m += bisect(j, lo, mid, threads);
  if (!group_closes(j, mid, hi, threads)) m += bisect(j, mid, hi, threads);
  return m;
}

int cpu_batch_verify_ex(void* ctx, int count, const uint8_t* coms, const uint8_t* const* ders, const size_t* lens,
                        int threads, int32_t* out, uint8_t* com_out, uint8_t* x0_out) {
  cpu_ctx* c = ctx;
  if (!c || count < 0) return -1;
  if (count == 0) return 0;
  if (threads < 1) threads = 1;
  batch_job j;
  memset(&j, 0, sizeof j);
  j.c = c;
  j.count = count;
  j.coms = coms;
  j.ders = ders;
  j.lens = lens;
  j.out = out;
  j.com_out = com_out;
  j.x0_out = x0_out;
  if (com_out) memset(com_out, 0, 64 * (size_t)count);
  if (x0_out) memset(x0_out, 0, 32 * (size_t)count);
  j.npv = 4 + 2 * c->k;
  j.vpts = malloc(sizeof(aff) * (size_t)count * j.npv);
  j.vinf = calloc((size_t)count * j.npv, 1);
  j.vsc = calloc((size_t)count * j.npv, sizeof(fe));
  j.live = calloc(count, 1);
  j.col = malloc(sizeof(fe) * (size_t)count * c->nb);
  if (getrandom(j.rng_key, sizeof j.rng_key, 0) != (ssize_t)sizeof j.rng_key) return -1;
  atomic_init(&j.next, 0);
  atomic_init(&j.tid, 0);
  run_threads(threads, proof_worker, &j);
  for (int i = 0; i < count; i++)
    if (!j.live[i])
      for (int q = 0; q < j.npv; q++) j.vinf[(size_t)i * j.npv + q] = 1;
  /* batch check: MSM over the variable points of the live proofs + fixed columns */
  int nfb = group_closes(&j, 0, count, threads) ? 0 : bisect(&j, 0, count, threads);
  free(j.vpts);
  free(j.vinf);
  free(j.vsc);
  free(j.live);
  free(j.col);
  return nfb;
}

int cpu_batch_verify(void* ctx, int count, const uint8_t* coms, const uint8_t* const* ders, const size_t* lens,
                     int threads, int32_t* out) {
  return cpu_batch_verify_ex(ctx, count, coms, ders, lens, threads, out, NULL, NULL);
}

/* ------------------------------------------------ standalone MSM (config C3 baseline) */
int cpu_msm_pippenger(const uint8_t* pts, const uint8_t* scs, size_t n, int threads, uint8_t* out64) {
  init_consts();
  aff* a = malloc(sizeof(aff) * (n ? n : 1));
  uint8_t* inf = malloc(n ? n : 1);
  fe* sc = malloc(sizeof(fe) * (n ? n : 1));
  int bad = 0;
  for (size_t i = 0; i < n; i++) {
    g1 p;
    if (!g1_from_bytes(pts + 64 * i, 64, &p)) {
      bad = 1;
      p.inf = 1;
    }
    inf[i] = (uint8_t)p.inf;
    a[i].x = p.x;
    a[i].y = p.y;
    sc[i] = zr_red(be_to_fe(scs + 32 * i)); /* G1.Mul uses the scalar mod r */
  }
  g1j acc = msm_glv(a, inf, sc, n, threads);
  g1_bytes(toaff(acc), out64);
  free(a);
  free(inf);
  free(sc);
  return bad ? -1 : 0;
}
