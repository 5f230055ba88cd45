// Host prover: produces reference-format proofs for synthetic inputs.
//
// Semantics follow the reference provers (rp/bulletproof.go:209-249,336-466;
// rp/ipa.go:158-186,267-322; transfer/typeandsum.go:189-356;
// transfer/transfer.go:69-150; issue/sametype.go:103-148; issue/prover.go:46-112).
// Every group operation is evaluated over the ORIGINAL generators with
// fixed-base tables (the IPA's folded generators are tracked as per-generator
// coefficients), so one 64-bit range proof costs ~1.1k fixed-base products.
// Output is byte-compatible with the reference wire format; the proofs are
// checked by the independent oracle in tests/.
#pragma once
#include <stdint.h>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include "../common/sha256.hpp"
#include "bn254_host.hpp"
#include "der.hpp"
#include "pp_parse.hpp"
#include "proofs.hpp"

namespace fts {
namespace host {

// Prover randomness, uniform Fr by rejection, in one of two modes:
//  - seeded (tests and benchmarks ONLY): xoshiro256** from a 64-bit seed.  Two
//    proofs whose seeds collide reuse their nonces, which reveals the committed
//    values and blinding factors -- never use it for real tokens.
//  - secure: ChaCha20 (RFC 8439 block function) under a 256-bit key drawn from
//    getrandom() once per call, one keystream per proof / action (nonce = its
//    index), the role crypto/rand plays for the reference provers
//    (rp/bulletproof.go:336-466 via Curve.NewRandomZr).
// The C-ABI selects the mode by the seed argument: FTS_SEED_OS_RANDOM = secure.
struct Rng {
  bool secure = false;
  uint64_t s[4];
  uint32_t key[8], blk[16];
  uint64_t stream = 0;
  uint32_t ctr = 0;
  int pos = 16;
  explicit Rng(uint64_t seed) {
    uint64_t z = seed;
    for (int i = 0; i < 4; i++) {
      z += 0x9e3779b97f4a7c15ULL;
      uint64_t x = z;
      x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
      x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
      s[i] = x ^ (x >> 31);
    }
  }
  Rng(const uint32_t k[8], uint64_t stream_id) : secure(true), stream(stream_id) {
    for (int i = 0; i < 8; i++) key[i] = k[i];
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
  void refill() {  // ChaCha20 block (key, counter = ctr, nonce = stream)
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                       key[4], key[5], key[6], key[7], ctr++, (uint32_t)stream, (uint32_t)(stream >> 32), 0u};
    uint32_t x[16];
    for (int i = 0; i < 16; i++) x[i] = st[i];
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; r++) {
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; i++) blk[i] = x[i] + st[i];
    pos = 0;
  }
  uint64_t next() {
    if (secure) {
      if (pos > 14) refill();
      const uint64_t v = (uint64_t)blk[pos] | ((uint64_t)blk[pos + 1] << 32);
      pos += 2;
      return v;
    }
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  Fr fr() {
    for (;;) {
      uint64_t c[4] = {next(), next(), next(), next() & 0x3fffffffffffffffULL};
      if (!geq_mod<ModR>(c)) return to_mont<ModR>(c);
    }
  }
};

// the randomness of one prover call: item i draws from at(i) (seeded: seed + i)
struct RngSource {
  bool secure = false;
  uint64_t seed = 0;
  uint32_t key[8] = {0};
  bool ok = true;
  explicit RngSource(uint64_t sd);
  Rng at(uint64_t i) const { return secure ? Rng(key, i) : Rng(seed + i); }
};

inline std::string hex_of(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}
// (*G1Array).Bytes, common/array.go:25-36
inline std::string g1_array_bytes(const std::vector<G1A>& pts) {
  std::string out;
  for (size_t i = 0; i < pts.size(); i++) {
    uint8_t b[64];
    g1_to_bytes(pts[i], b);
    if (i) out += "||";
    out += hex_of(b, 64);
  }
  return out;
}
inline Fr hash_to_zr(const std::string& m) {
  uint8_t d[32];
  sha256((const uint8_t*)m.data(), m.size(), d);
  return fr_from_digest(d);
}
inline Fr fr_u64(uint64_t v) { return from_u64<ModR>(v); }
inline Fr fr_pow(const Fr& a, uint64_t e) {
  Fr r = Fr::one(), b = a;
  while (e) {
    if (e & 1) r = mul(r, b);
    e >>= 1;
    b = sqr(b);
  }
  return r;
}

struct ProverTables {
  // 0..n-1 G_i, n..2n-1 H_i, 2n ped0, 2n+1 ped1, 2n+2 ped2, 2n+3 P, 2n+4 Q
  std::vector<FixedBase> fb;
  int n = 0;
  const FixedBase& G(int i) const { return fb[i]; }
  const FixedBase& H(int i) const { return fb[n + i]; }
  const FixedBase& ped(int i) const { return fb[2 * n + i]; }
  const FixedBase& P() const { return fb[2 * n + 3]; }
  const FixedBase& Q() const { return fb[2 * n + 4]; }
};

void build_prover_tables(const PublicParams& pp, int n, ProverTables& t);  // multi-threaded (api.cpp)

// sum_i s_i * base_i over fixed-base tables
struct Msm {
  G1J acc = jac_identity();
  void add_fb(const FixedBase& fb, const Fr& s) {
    if (!s.is_zero()) acc = jadd(acc, fb.mul(s));
  }
  void add_pt(const G1A& p) { acc = jadd_aff(acc, p); }
  G1A aff() const { return to_aff(acc); }
};

struct RangeProofOut {
  G1A T1, T2, C, D;
  Fr tau, delta, ip, a, b;
  std::vector<G1A> L, R;
  std::string serialize() const {
    std::vector<std::string> data = {el_g1(T1), el_g1(T2), el_fr(tau), el_g1(C), el_g1(D), el_fr(delta), el_fr(ip)};
    std::string d = der::values(data);
    std::vector<std::string> ipa = {el_fr(a), el_fr(b), el_g1_array(L), el_g1_array(R)};
    std::string i = der::values(ipa);
    return der::values({d, i});
  }
};

// rangeProver.Prove (bulletproof.go:209-249) with preprocess (:336-466) and the
// IPA prover (ipa.go:158-186, reduce :267-322).  ped1/ped2 = CommitmentGenerators.
inline RangeProofOut prove_range(const ProverTables& T, const PublicParams& pp, int n, int k, const G1A& V,
                                 uint64_t value, const Fr& bf, Rng& rng) {
  RangeProofOut out;
  std::vector<Fr> left(n), right(n), rl(n), rr(n);
  Fr one = Fr::one();
  Fr rho = rng.fr(), eta = rng.fr();
  for (int i = 0; i < n; i++) {
    uint64_t bit = (value >> i) & 1ULL;
    left[i] = bit ? one : Fr::zero();
    right[i] = sub(left[i], one);
    rl[i] = rng.fr();
    rr[i] = rng.fr();
  }
  // C = <left, G> + <right, H> + rho P ; D = <rl, G> + <rr, H> + eta P
  Msm C, D;
  for (int i = 0; i < n; i++) {
    if (left[i] == one) C.add_pt(pp.left[i]);
    else C.add_pt(aff_neg(pp.right[i]));
    D.add_fb(T.G(i), rl[i]);
    D.add_fb(T.H(i), rr[i]);
  }
  C.add_fb(T.P(), rho);
  D.add_fb(T.P(), eta);
  out.C = C.aff();
  out.D = D.aff();
  Fr y = hash_to_zr(g1_array_bytes({out.C, out.D, V}));
  Fr z = hash_to_zr(fr_raw(y));
  Fr z2 = sqr(z);
  std::vector<Fr> lp(n), rp(n), rrp(n), zp(n);
  Fr yi = one, p2 = one;
  for (int i = 0; i < n; i++) {
    if (i) {
      yi = mul(yi, y);
      p2 = add(p2, p2);
    }
    lp[i] = sub(left[i], z);
    rp[i] = mul(add(right[i], z), yi);
    rrp[i] = mul(rr[i], yi);
    zp[i] = mul(z2, p2);
  }
  Fr t1 = Fr::zero(), t2 = Fr::zero();
  for (int i = 0; i < n; i++) {
    t1 = add(t1, mul(lp[i], rrp[i]));
    t1 = add(t1, mul(rp[i], rl[i]));
    t1 = add(t1, mul(zp[i], rl[i]));
    t2 = add(t2, mul(rl[i], rrp[i]));
  }
  Fr tau1 = rng.fr();
  Msm T1;
  T1.add_fb(T.ped(1), t1);
  T1.add_fb(T.ped(2), tau1);
  out.T1 = T1.aff();
  Fr tau2 = rng.fr();
  Msm T2;
  T2.add_fb(T.ped(1), t2);
  T2.add_fb(T.ped(2), tau2);
  out.T2 = T2.aff();
  Fr x = hash_to_zr(g1_array_bytes({out.T1, out.T2}));
  std::vector<Fr> a(n), b(n);
  for (int i = 0; i < n; i++) {
    a[i] = add(lp[i], mul(x, rl[i]));
    b[i] = add(add(rp[i], mul(x, rrp[i])), zp[i]);
  }
  out.tau = add(add(mul(x, tau1), mul(tau2, sqr(x))), mul(z2, bf));
  out.delta = add(rho, mul(eta, x));
  // H'_i = y^-i H_i ; com = <a, G> + <b, H'>
  Fr yinv = inv(y);
  std::vector<Fr> yinvp(n);
  yinvp[0] = one;
  for (int i = 1; i < n; i++) yinvp[i] = mul(yinvp[i - 1], yinv);
  std::vector<G1J> hpj(n);
  for (int i = 0; i < n; i++) hpj[i] = T.H(i).mul(yinvp[i]);
  std::vector<G1A> hp(n);
  to_aff_batch(hpj.data(), hp.data(), n);
  Msm com;
  Fr ip = Fr::zero();
  for (int i = 0; i < n; i++) {
    com.add_fb(T.G(i), a[i]);
    com.add_fb(T.H(i), mul(b[i], yinvp[i]));
    ip = add(ip, mul(a[i], b[i]));
  }
  G1A coma = com.aff();
  out.ip = ip;
  // IPA prove: x0 from DER(SEQUENCE OF OCTET STRING [Arr(H', G, Q, com), "||", Zb(ip)])
  std::vector<G1A> arr(hp);
  for (int i = 0; i < n; i++) arr.push_back(pp.left[i]);
  arr.push_back(pp.Q);
  arr.push_back(coma);
  std::string raw = der::seq_of_octets({g1_array_bytes(arr), std::string("||"), fr_raw(ip)});
  Fr x0 = hash_to_zr(raw);
  // folded-generator coefficients over the original G_t / H'_t
  std::vector<Fr> gc(n, one), hc(n, one);
  int m = n;
  for (int j = 0; j < k; j++) {
    m /= 2;
    // current vectors a, b have length 2m; folded index of t is t mod 2m
    Fr cl = Fr::zero(), cr = Fr::zero();
    for (int i = 0; i < m; i++) {
      cl = add(cl, mul(a[i], b[m + i]));
      cr = add(cr, mul(a[m + i], b[i]));
    }
    Msm Lm, Rm;
    for (int t = 0; t < n; t++) {
      int f = t % (2 * m);
      if (f >= m) {
        // G^(j)_{m+i} with i = f-m carries a_i in L ; H'^(j)_{f} carries b_{f-m}... in R
        Lm.add_fb(T.G(t), mul(a[f - m], gc[t]));
        Rm.add_fb(T.H(t), mul(mul(b[f - m], hc[t]), yinvp[t]));
      } else {
        Lm.add_fb(T.H(t), mul(mul(b[m + f], hc[t]), yinvp[t]));
        Rm.add_fb(T.G(t), mul(a[m + f], gc[t]));
      }
    }
    Lm.add_fb(T.Q(), mul(cl, x0));
    Rm.add_fb(T.Q(), mul(cr, x0));
    G1J lr[2] = {Lm.acc, Rm.acc};
    G1A lra[2];
    to_aff_batch(lr, lra, 2);
    out.L.push_back(lra[0]);
    out.R.push_back(lra[1]);
    Fr xj = hash_to_zr(g1_array_bytes({lra[0], lra[1]}));
    Fr xji = inv(xj);
    // reduceGenerators: G'_i = x^-1 G_i + x G_{i+m};  H'_i = x H_i + x^-1 H_{i+m}
    for (int t = 0; t < n; t++) {
      bool hi = (t % (2 * m)) >= m;
      gc[t] = mul(gc[t], hi ? xj : xji);
      hc[t] = mul(hc[t], hi ? xji : xj);
    }
    // reduceVectors: a_i = a_i x + a_{i+m} x^-1 ; b_i = b_i x^-1 + b_{i+m} x
    for (int i = 0; i < m; i++) {
      a[i] = add(mul(a[i], xj), mul(a[i + m], xji));
      b[i] = add(mul(b[i], xji), mul(b[i + m], xj));
    }
    a.resize(m);
    b.resize(m);
  }
  out.a = a[0];
  out.b = b[0];
  return out;
}

inline Fr type_to_zr(const uint8_t* type, size_t len) { return hash_to_zr(std::string((const char*)type, len)); }

// commit (crypto/token/token.go:208-217): H(type) ped0 + v ped1 + bf ped2
inline G1A token_commit(const ProverTables& T, const Fr& type_zr, uint64_t value, const Fr& bf) {
  Msm m;
  m.add_fb(T.ped(0), type_zr);
  m.add_fb(T.ped(1), fr_u64(value));
  m.add_fb(T.ped(2), bf);
  return m.aff();
}

inline std::string rc_serialize(const std::vector<std::string>& proofs) {
  return der::values({der::values(proofs)});
}

// transfer.NewProver(...).Prove()  transfer/transfer.go:69-150, typeandsum.go:189-356
inline std::string prove_transfer(const ProverTables& T, const PublicParams& pp, int n, int k, const Fr& type_zr,
                                  const std::vector<uint64_t>& inv, const std::vector<Fr>& inbf,
                                  const std::vector<uint64_t>& outv, const std::vector<Fr>& outbf, Rng& rng) {
  size_t nin = inv.size(), nout = outv.size();
  std::vector<G1A> ins(nin), outs(nout);
  for (size_t i = 0; i < nin; i++) ins[i] = token_commit(T, type_zr, inv[i], inbf[i]);
  for (size_t i = 0; i < nout; i++) outs[i] = token_commit(T, type_zr, outv[i], outbf[i]);
  Fr tbf = rng.fr();
  Msm ctm;
  ctm.add_fb(T.ped(0), type_zr);
  ctm.add_fb(T.ped(2), tbf);
  G1A ct = ctm.aff();
  std::string rc;
  bool has_rc = nin != 1 || nout != 1;
  if (has_rc) {
    std::vector<std::string> rps;
    for (size_t i = 0; i < nout; i++) {
      G1A V = to_aff(jadd_aff(to_jac(outs[i]), aff_neg(ct)));
      RangeProofOut rp = prove_range(T, pp, n, k, V, outv[i], sub(outbf[i], tbf), rng);
      rps.push_back(rp.serialize());
    }
    rc = rc_serialize(rps);
  }
  // TypeAndSum: commitments to randomness
  Fr r_t = rng.fr(), r_tbf = rng.fr();
  Msm cct;
  cct.add_fb(T.ped(0), r_t);
  cct.add_fb(T.ped(2), r_tbf);
  std::vector<Fr> r_iv(nin), r_ibf(nin);
  std::vector<G1J> cin(nin);
  for (size_t i = 0; i < nin; i++) {
    r_iv[i] = rng.fr();
    r_ibf[i] = rng.fr();
    Msm c;
    c.add_fb(T.ped(1), r_iv[i]);
    c.add_fb(T.ped(2), r_ibf[i]);
    cin[i] = c.acc;
  }
  Fr r_sum = rng.fr();
  Msm csum;
  csum.add_fb(T.ped(2), r_sum);
  // inputs/outputs minus CT, and their signed sum
  std::vector<G1A> arr;
  std::vector<G1A> cina(nin);
  to_aff_batch(cin.data(), cina.data(), nin);
  arr.insert(arr.end(), cina.begin(), cina.end());
  arr.push_back(cct.aff());
  arr.push_back(csum.aff());
  G1J sum = jac_identity();
  G1A nct = aff_neg(ct);
  for (size_t i = 0; i < nin; i++) {
    G1A d = to_aff(jadd_aff(to_jac(ins[i]), nct));
    arr.push_back(d);
    sum = jadd_aff(sum, d);
  }
  for (size_t i = 0; i < nout; i++) {
    G1A d = to_aff(jadd_aff(to_jac(outs[i]), nct));
    arr.push_back(d);
    sum = jadd_aff(sum, aff_neg(d));
  }
  arr.push_back(ct);
  arr.push_back(to_aff(sum));
  Fr chal = hash_to_zr(g1_array_bytes(arr));
  Fr ptype = add(mul(chal, type_zr), r_t);
  Fr ptbf = add(mul(chal, tbf), r_tbf);
  std::vector<Fr> piv(nin), pibf(nin);
  Fr sumbf = Fr::zero();
  for (size_t i = 0; i < nin; i++) {
    piv[i] = add(mul(chal, fr_u64(inv[i])), r_iv[i]);
    Fr t = sub(inbf[i], tbf);
    pibf[i] = add(mul(chal, t), r_ibf[i]);
    sumbf = add(sumbf, t);
  }
  for (size_t i = 0; i < nout; i++) sumbf = sub(sumbf, sub(outbf[i], tbf));
  Fr peq = add(mul(chal, sumbf), r_sum);
  std::string tas = der::values({el_g1(ct), el_fr_array(pibf), el_fr_array(piv), el_fr(ptype), el_fr(ptbf),
                                 el_fr(peq), el_fr(chal)});
  return der::values({tas, has_rc ? rc : std::string()});
}

// issue.NewProver(...).Prove()  issue/prover.go:46-112, sametype.go:103-148
inline std::string prove_issue(const ProverTables& T, const PublicParams& pp, int n, int k, const Fr& type_zr,
                               const std::vector<uint64_t>& vals, const std::vector<Fr>& bfs, Rng& rng) {
  size_t nt = vals.size();
  Fr tbf = rng.fr();
  Msm ctm;
  ctm.add_fb(T.ped(0), type_zr);
  ctm.add_fb(T.ped(2), tbf);
  G1A ct = ctm.aff();
  Fr r_t = rng.fr(), r_bf = rng.fr();
  Msm cm;
  cm.add_fb(T.ped(0), r_t);
  cm.add_fb(T.ped(2), r_bf);
  Fr chal = hash_to_zr(g1_array_bytes({ct, cm.aff()}));
  Fr ptype = add(mul(chal, type_zr), r_t);
  Fr pbf = add(mul(chal, tbf), r_bf);
  std::string st = der::values({el_fr(ptype), el_fr(pbf), el_fr(chal), el_g1(ct)});
  std::vector<std::string> rps;
  for (size_t i = 0; i < nt; i++) {
    G1A tok = token_commit(T, type_zr, vals[i], bfs[i]);
    G1A V = to_aff(jadd_aff(to_jac(tok), aff_neg(ct)));
    RangeProofOut rp = prove_range(T, pp, n, k, V, vals[i], sub(bfs[i], tbf), rng);
    rps.push_back(rp.serialize());
  }
  return der::values({st, rc_serialize(rps)});
}

}  // namespace host
}  // namespace fts
