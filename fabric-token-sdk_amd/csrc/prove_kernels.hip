// Batched range-proof PROVER on the device:
// rangeProver.Prove (rp/bulletproof.go:209-249) with preprocess (:336-466)
// and the IPA prover (rp/ipa.go:158-186, reduce :267-322), for B proofs at
// once.  Output is byte-identical to the library's host prover
// (host/prover.hpp prove_range) for the same randomness, which the host draws
// from the seeded generator in the reference's draw order and uploads.
//
// Every group element the prover publishes or hashes is a sum of fixed-base
// products over the context's 16-bit window tables: the folded IPA
// generators are never materialised; round j's L_j / R_j are sums over the
// ORIGINAL G_t / H_t with accumulated coefficients (gc_t, hc_t y^-t), exactly
// as the host prover does.  One stage = (Fr kernel, thread per proof) writes
// the stage's scalars -> k_pv_fbsum (thread per (proof, group of <= 8 terms),
// one Jacobian accumulator, mixed additions only) -> k_pv_segsum (thread per
// (proof, output point)) -> normalisation + Fiat-Shamir hash (thread per proof).
//
//   stage 1   V = v ped1 + bf ped2 ; C = rho P + sum(bit ? G_i : -H_i) ; D = <rl,G> + <rr,H> + eta P
//             y = Hz(C, D, V), z = Hz(Zb(y))                                  bulletproof.go:214-232,336-392
//   stage 2   T1 = t1 ped1 + tau1 ped2 ; T2 = t2 ped1 + tau2 ped2 ; x = Hz(T1, T2)   :393-432
//   stage 3   a, b, tau, delta, ip ; H'_i = y^-i H_i ; com = <a,G> + <b,H'>          :433-466, :236-249
//             x0 = Hz(DER(Arr(H', G, Q, com), "||", Zb(ip)))  (the verifier's x0 kernels)  ipa.go:158-176
//   round j   L_j, R_j (n + 1 terms each) ; x_j = Hz(L_j, R_j) ; fold a, b, gc, hc       ipa.go:267-322
#include "device/g1.hpp"
#include "device/fixed_base.hpp"
#include "device/helpers.hpp"
#include "device/rp_kernels.hpp"
#include "device/transcript.hpp"
#include "device/prove.hpp"

namespace fts {

// ------------------------------------------------------------------ helpers
FTS_DEV Fr pv_ld(const uint32_t* p) {  // Montgomery Fr
  Fr a;
  load_f(p, a);
  return a;
}
FTS_DEV void pv_put_canon(uint32_t* dst, const Fr& m) {  // Montgomery -> canonical limbs
  Fr c = f_from_mont(m);
  store_f(dst, c);
}
FTS_DEV Fr pv_canon_in(const uint32_t* p) { return fr_from_canon(p); }  // canonical -> Montgomery

// Hz(Zb(y)): SHA-256 of the 32-byte big-endian encoding, mod r
FTS_DEV Fr pv_hash_zr32(uint8_t* slot, const Fr& ym) {
  Fr c = f_from_mont(ym);
  for (int i = 0; i < 8; i++) {
    const uint32_t w = c.v[7 - i];
    slot[4 * i + 0] = (uint8_t)(w >> 24);
    slot[4 * i + 1] = (uint8_t)(w >> 16);
    slot[4 * i + 2] = (uint8_t)(w >> 8);
    slot[4 * i + 3] = (uint8_t)w;
  }
  write_sha_padding_u16(slot, 32);
  uint32_t st[8];
  sha256_blocks(slot, 1, st);
  return digest_to_fr(st);
}

// normalise jac[b][0..m) (one inversion) and write BE bytes to dst[i]
FTS_DEV void pv_norm(const PvDev& d, int b, int m, uint8_t* const* dst) {
  const uint32_t* J = d.jac + (size_t)b * (d.n + 1) * 24;
  uint32_t* A = d.aff + (size_t)b * (d.n + 1) * 16;
  batch_to_affine(J, A, m);
  for (int i = 0; i < m; i++) store_point_be(dst[i], load_g1a(A + i * 16));
}
FTS_DEV uint8_t* pv_out(const PvDev& d, int b, int slot) {
  return d.out_pts + ((size_t)b * pv_npts(d.k) + slot) * 64;
}
FTS_DEV uint32_t* pv_term(const PvDev& d, int b, int t) { return d.terms + ((size_t)b * pv_tmax(d.n) + t) * 8; }

// ------------------------------------------------------------- generic sums
// thread per (proof, group): sum of the group's terms sc_t * B_{base[t]}.
// Proof index fastest: the lanes of a wave walk the same bases (one table
// at a time, TLB- and L2-friendly gathers) and run the same number of terms.
__global__ void __launch_bounds__(64) k_pv_fbsum(PvDev d, PvStage s) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= d.B * s.G) return;
  const int g = gid / d.B, b = gid % d.B;
  const int4 gr = s.grp[g];
  G1J acc = g1j_identity();
  for (int t = gr.x; t < gr.y; t++) {
    const uint32_t* S = pv_term(d, b, t);
    Scalar k;
#pragma unroll
    for (int i = 0; i < 8; i++) k.v[i] = S[i];
    fb_mul_acc(acc, d.tables + (size_t)s.base[t] * FB_WORDS_PER_BASE, k);
  }
  store_g1j(d.partial + ((size_t)b * pv_gmax(d.n) + g) * 24, acc);
}
// thread per (proof, segment): jac[b][seg] = sum of the segment's group partials
// (proof index fastest: a wave's lanes sum equally many partials)
__global__ void __launch_bounds__(64) k_pv_segsum(PvDev d, PvStage s) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= d.B * s.S) return;
  const int q = gid / d.B, b = gid % d.B;
  const int2 sg = s.seg[q];
  const uint32_t* P = d.partial + (size_t)b * pv_gmax(d.n) * 24;
  G1J acc = load_g1j(P + sg.x * 24);
  for (int g = sg.x + 1; g < sg.y; g++) acc = nl_add_mem(acc, P + g * 24, 0);
  store_g1j(d.jac + ((size_t)b * (d.n + 1) + q) * 24, acc);
}

// ------------------------------------------------------------------ stage 1
// terms: [0] v (ped1), [1] bf (ped2) | [2] rho (P) | [3 + 2i] rl_i (G_i), [4 + 2i] rr_i (H_i), [3 + 2n] eta (P)
__global__ void __launch_bounds__(64) k_pv_stage1(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  const uint32_t* R = d.rnd + (size_t)b * pv_nrnd(n) * 8;
  uint32_t* t0 = pv_term(d, b, 0);
  const uint64_t v = d.values[b];
  t0[0] = (uint32_t)v;
  t0[1] = (uint32_t)(v >> 32);
  for (int i = 2; i < 8; i++) t0[i] = 0;
  const uint32_t* bf = d.bf + (size_t)b * 8;
  uint32_t* t1 = pv_term(d, b, 1);
  for (int i = 0; i < 8; i++) t1[i] = bf[i];
  auto cp = [&](int t, int r) {
    uint32_t* T = pv_term(d, b, t);
    const uint32_t* S = R + r * 8;
    for (int i = 0; i < 8; i++) T[i] = S[i];
  };
  cp(2, PV_R_RHO);
  for (int i = 0; i < n; i++) {
    cp(3 + 2 * i, PV_R_RL(i));
    cp(4 + 2 * i, PV_R_RR(i));
  }
  cp(3 + 2 * n, PV_R_ETA);
}
// C += sum_i (bit_i ? G_i : -H_i) (affine generators = entry (w 0, d 1) of their tables);
// normalise V, C, D; y = Hz(C, D, V), z = Hz(Zb(y))
__global__ void __launch_bounds__(64) k_pv_vcd(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  uint32_t* J = d.jac + (size_t)b * (n + 1) * 24;
  G1J c = load_g1j(J + 24);
  const uint64_t v = d.values[b];
  for (int i = 0; i < n; i++) {
    const bool bit = (v >> i) & 1ull;
    G1A q = fb_entry(d.tables + (size_t)(bit ? i : n + i) * FB_WORDS_PER_BASE, 0, bit ? 1 : -1);
    madd_inl(c, q);
  }
  store_g1j(J + 24, c);
  uint8_t* dst[3] = {pv_out(d, b, PV_V), pv_out(d, b, PV_C), pv_out(d, b, PV_D)};
  pv_norm(d, b, 3, dst);
  uint8_t* slot = d.hslot + (size_t)b * PV_HSLOT;
  const uint8_t* arr[3] = {dst[1], dst[2], dst[0]};  // Arr(C, D, V)   bulletproof.go:374
  Fr y = f_to_mont(hash_raw_points(slot, arr, 3));
  Fr z = f_to_mont(pv_hash_zr32(slot, y));
  uint32_t* ch = d.ch + (size_t)b * rp_nch(d.k) * 8;
  store_f(ch + CH_Y * 8, y);
  store_f(ch + CH_Z * 8, z);
}

// ------------------------------------------------------------------ stage 2
// the per-coordinate vectors of preprocess (bulletproof.go:393-432), in Montgomery form
struct PvCoord {
  Fr lp, rp, rrp, zp, rl;
};
FTS_DEV PvCoord pv_coord(const uint32_t* R, uint64_t v, int i, const Fr& yi, const Fr& z, const Fr& zp) {
  PvCoord c;
  const Fr one = f_one<FrP>();
  const Fr left = ((v >> i) & 1ull) ? one : f_zero<FrP>();
  const Fr right = f_sub(left, one);
  c.rl = pv_canon_in(R + PV_R_RL(i) * 8);
  const Fr rr = pv_canon_in(R + PV_R_RR(i) * 8);
  c.lp = f_sub(left, z);
  c.rp = fr_mul(f_add(right, z), yi);
  c.rrp = fr_mul(rr, yi);
  c.zp = zp;
  return c;
}
// terms: [0] t1 (ped1), [1] tau1 (ped2) | [2] t2 (ped1), [3] tau2 (ped2)
__global__ void __launch_bounds__(64) k_pv_stage2(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  const uint32_t* R = d.rnd + (size_t)b * pv_nrnd(n) * 8;
  const uint32_t* ch = d.ch + (size_t)b * rp_nch(d.k) * 8;
  const Fr y = pv_ld(ch + CH_Y * 8), z = pv_ld(ch + CH_Z * 8);
  const Fr z2 = fr_sqr(z);
  const uint64_t v = d.values[b];
  Fr yi = f_one<FrP>(), zp = z2, t1 = f_zero<FrP>(), t2 = f_zero<FrP>();
  for (int i = 0; i < n; i++) {
    if (i) {
      yi = fr_mul(yi, y);
      zp = f_add(zp, zp);
    }
    const PvCoord c = pv_coord(R, v, i, yi, z, zp);
    t1 = f_add(t1, fr_mul(c.lp, c.rrp));
    t1 = f_add(t1, fr_mul(c.rp, c.rl));
    t1 = f_add(t1, fr_mul(c.zp, c.rl));
    t2 = f_add(t2, fr_mul(c.rl, c.rrp));
  }
  pv_put_canon(pv_term(d, b, 0), t1);
  const uint32_t* tau1 = R + pv_r_tau1(n) * 8;
  const uint32_t* tau2 = R + pv_r_tau2(n) * 8;
  uint32_t* T1 = pv_term(d, b, 1);
  uint32_t* T3 = pv_term(d, b, 3);
  for (int i = 0; i < 8; i++) T1[i] = tau1[i], T3[i] = tau2[i];
  pv_put_canon(pv_term(d, b, 2), t2);
}
// normalise T1, T2; x = Hz(T1, T2)
__global__ void __launch_bounds__(64) k_pv_t12(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  uint8_t* dst[2] = {pv_out(d, b, PV_T1), pv_out(d, b, PV_T2)};
  pv_norm(d, b, 2, dst);
  const uint8_t* arr[2] = {dst[0], dst[1]};
  Fr x = f_to_mont(hash_raw_points(d.hslot + (size_t)b * PV_HSLOT, arr, 2));
  store_f(d.ch + ((size_t)b * rp_nch(d.k) + CH_X) * 8, x);
}

// ------------------------------------------------------------------ stage 3
// a, b, tau, delta, y^-i, ip; terms: [i] y^-i (H_i) for i < n | [n + 2i] a_i (G_i), [n + 2i + 1] b_i y^-i (H_i)
__global__ void __launch_bounds__(64) k_pv_stage3(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  const uint32_t* R = d.rnd + (size_t)b * pv_nrnd(n) * 8;
  uint32_t* ch = d.ch + (size_t)b * rp_nch(d.k) * 8;
  const Fr y = pv_ld(ch + CH_Y * 8), z = pv_ld(ch + CH_Z * 8), x = pv_ld(ch + CH_X * 8);
  const Fr z2 = fr_sqr(z);
  const uint64_t v = d.values[b];
  uint32_t* S = d.st + (size_t)b * pv_nst(n) * 8;
  const Fr yinv = nl_fr_inv(y);
  Fr yi = f_one<FrP>(), zp = z2, yim = f_one<FrP>(), ip = f_zero<FrP>();
  const Fr one = f_one<FrP>();
  for (int i = 0; i < n; i++) {
    if (i) {
      yi = fr_mul(yi, y);
      zp = f_add(zp, zp);
      yim = fr_mul(yim, yinv);
    }
    const PvCoord c = pv_coord(R, v, i, yi, z, zp);
    const Fr a = f_add(c.lp, fr_mul(x, c.rl));
    const Fr bb = f_add(f_add(c.rp, fr_mul(x, c.rrp)), c.zp);
    store_f(S + (PV_ST_A + i) * 8, a);
    store_f(S + (PV_ST_B + i) * 8, bb);
    store_f(S + (PV_ST_YI + i) * 8, yim);
    store_f(S + (PV_ST_GC + i) * 8, one);
    store_f(S + (PV_ST_HC + i) * 8, one);
    ip = f_add(ip, fr_mul(a, bb));
    pv_put_canon(pv_term(d, b, i), yim);
    pv_put_canon(pv_term(d, b, n + 2 * i), a);
    pv_put_canon(pv_term(d, b, n + 2 * i + 1), fr_mul(bb, yim));
  }
  const Fr tau1 = pv_canon_in(R + pv_r_tau1(n) * 8), tau2 = pv_canon_in(R + pv_r_tau2(n) * 8);
  const Fr rho = pv_canon_in(R + PV_R_RHO * 8), eta = pv_canon_in(R + PV_R_ETA * 8);
  const Fr bf = pv_canon_in(d.bf + (size_t)b * 8);
  const Fr tau = f_add(f_add(fr_mul(x, tau1), fr_mul(tau2, fr_sqr(x))), fr_mul(z2, bf));
  const Fr delta = f_add(rho, fr_mul(eta, x));
  uint32_t* O = d.out_fr + (size_t)b * PV_NFR * 8;
  pv_put_canon(O + PV_F_TAU * 8, tau);
  pv_put_canon(O + PV_F_DELTA * 8, delta);
  pv_put_canon(O + PV_F_IP * 8, ip);
  pv_put_canon(d.sc_ip + ((size_t)b * RP_NSC + RP_SC_IP) * 8, ip);  // Zb(ip) of the x0 transcript
}
// normalise H'_0..H'_{n-1}, com into the x0 layout (hp_be[b][0..n])
__global__ void __launch_bounds__(64) k_pv_hp(PvDev d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  const uint32_t* J = d.jac + (size_t)b * (n + 1) * 24;
  uint32_t* A = d.aff + (size_t)b * (n + 1) * 16;
  batch_to_affine(J, A, n + 1);
  uint8_t* H = d.hp_be + (size_t)b * (n + 1) * 64;
  for (int i = 0; i <= n; i++) store_point_be(H + i * 64, load_g1a(A + i * 16));
}

// ------------------------------------------------------------------ rounds
// fold with x_{j-1} (ipa.go:280-300: reduceGenerators / reduceVectors at m = n >> j),
// then write round j's terms (j < k):  L: [t] G_t or H_t, [n] Q ; R: [n + 1 + t], [2n + 1] Q
FTS_DEV void pv_fold(const PvDev& d, int b, int j) {
  const int n = d.n, m = n >> j;
  uint32_t* S = d.st + (size_t)b * pv_nst(n) * 8;
  const Fr xj = pv_ld(d.ch + ((size_t)b * rp_nch(d.k) + CH_XJ + j - 1) * 8);
  const Fr xji = nl_fr_inv(xj);
  for (int t = 0; t < n; t++) {
    const bool hi = (t % (2 * m)) >= m;
    store_f(S + (PV_ST_GC + t) * 8, fr_mul(pv_ld(S + (PV_ST_GC + t) * 8), hi ? xj : xji));
    store_f(S + (PV_ST_HC + t) * 8, fr_mul(pv_ld(S + (PV_ST_HC + t) * 8), hi ? xji : xj));
  }
  for (int i = 0; i < m; i++) {
    const Fr a = f_add(fr_mul(pv_ld(S + (PV_ST_A + i) * 8), xj), fr_mul(pv_ld(S + (PV_ST_A + i + m) * 8), xji));
    const Fr bb = f_add(fr_mul(pv_ld(S + (PV_ST_B + i) * 8), xji), fr_mul(pv_ld(S + (PV_ST_B + i + m) * 8), xj));
    store_f(S + (PV_ST_A + i) * 8, a);
    store_f(S + (PV_ST_B + i) * 8, bb);
  }
}
__global__ void __launch_bounds__(64) k_pv_round(PvDev d, int j) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  const int n = d.n;
  if (j > 0) pv_fold(d, b, j);
  uint32_t* S = d.st + (size_t)b * pv_nst(n) * 8;
  if (j == d.k) {  // final a, b (ipa.go:181-185)
    uint32_t* O = d.out_fr + (size_t)b * PV_NFR * 8;
    pv_put_canon(O + PV_F_A * 8, pv_ld(S + PV_ST_A * 8));
    pv_put_canon(O + PV_F_B * 8, pv_ld(S + PV_ST_B * 8));
    return;
  }
  const int m = n >> (j + 1);
  Fr cl = f_zero<FrP>(), cr = f_zero<FrP>();
  for (int i = 0; i < m; i++) {
    cl = f_add(cl, fr_mul(pv_ld(S + (PV_ST_A + i) * 8), pv_ld(S + (PV_ST_B + m + i) * 8)));
    cr = f_add(cr, fr_mul(pv_ld(S + (PV_ST_A + m + i) * 8), pv_ld(S + (PV_ST_B + i) * 8)));
  }
  for (int t = 0; t < n; t++) {
    const int f = t % (2 * m);
    const Fr gcoef = pv_ld(S + (PV_ST_GC + t) * 8);
    const Fr hcoef = fr_mul(pv_ld(S + (PV_ST_HC + t) * 8), pv_ld(S + (PV_ST_YI + t) * 8));
    Fr lv, rv;
    if (f >= m) {  // L: a_{f-m} on G_t ; R: b_{f-m} on H'_t
      lv = fr_mul(pv_ld(S + (PV_ST_A + f - m) * 8), gcoef);
      rv = fr_mul(pv_ld(S + (PV_ST_B + f - m) * 8), hcoef);
    } else {       // L: b_{m+f} on H'_t ; R: a_{m+f} on G_t
      lv = fr_mul(pv_ld(S + (PV_ST_B + m + f) * 8), hcoef);
      rv = fr_mul(pv_ld(S + (PV_ST_A + m + f) * 8), gcoef);
    }
    pv_put_canon(pv_term(d, b, t), lv);
    pv_put_canon(pv_term(d, b, n + 1 + t), rv);
  }
  const Fr x0 = pv_ld(d.ch + ((size_t)b * rp_nch(d.k) + CH_X0) * 8);
  pv_put_canon(pv_term(d, b, n), fr_mul(cl, x0));
  pv_put_canon(pv_term(d, b, 2 * n + 1), fr_mul(cr, x0));
}
// normalise L_j, R_j; x_j = Hz(L_j, R_j)
__global__ void __launch_bounds__(64) k_pv_lr(PvDev d, int j) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= d.B) return;
  uint8_t* dst[2] = {pv_out(d, b, PV_L(j)), pv_out(d, b, PV_R(j))};
  pv_norm(d, b, 2, dst);
  const uint8_t* arr[2] = {dst[0], dst[1]};
  Fr xj = f_to_mont(hash_raw_points(d.hslot + (size_t)b * PV_HSLOT, arr, 2));
  store_f(d.ch + ((size_t)b * rp_nch(d.k) + CH_XJ + j) * 8, xj);
}

// ------------------------------------------------------------------ launch
void launch_x0(int B, int n, int k, const int32_t* status, const uint8_t* hp_be, const uint8_t* x0_const,
               const uint8_t* x0_tmpl, const uint32_t* sc, uint8_t* msgs, uint32_t* ch, hipStream_t s);

static void pv_sum(const PvDev& d, const PvStage& s, hipStream_t st) {
  hipLaunchKernelGGL(k_pv_fbsum, dim3((unsigned)((d.B * s.G + 63) / 64)), dim3(64), 0, st, d, s);
  hipLaunchKernelGGL(k_pv_segsum, dim3((unsigned)((d.B * s.S + 63) / 64)), dim3(64), 0, st, d, s);
}

void launch_rp_prove(const PvDev& d, const PvStage* stages, const uint8_t* x0_const, const uint8_t* x0_tmpl,
                     hipStream_t s, Timeline* tl) {
  const dim3 gp((unsigned)((d.B + 63) / 64)), bs(64);
  const double B = d.B;
  // stage 1: V, C, D ; y, z
  hipLaunchKernelGGL(k_pv_stage1, gp, bs, 0, s, d);
  pv_sum(d, stages[0], s);
  hipLaunchKernelGGL(k_pv_vcd, gp, bs, 0, s, d);
  tl->mark("k_pv_stage1", s, B * (stages[0].T * COST_FB + d.n * COST_MADD));
  // stage 2: T1, T2 ; x
  hipLaunchKernelGGL(k_pv_stage2, gp, bs, 0, s, d);
  pv_sum(d, stages[1], s);
  hipLaunchKernelGGL(k_pv_t12, gp, bs, 0, s, d);
  tl->mark("k_pv_stage2", s, B * (stages[1].T * COST_FB + 8.0 * d.n));
  // stage 3: a, b, H', com ; x0 (per-kernel marks: the stage is latency-heavy)
  hipLaunchKernelGGL(k_pv_stage3, gp, bs, 0, s, d);
  tl->mark("k_pv_stage3_fr", s, B * 14.0 * d.n);
  hipLaunchKernelGGL(k_pv_fbsum, dim3((unsigned)((d.B * stages[2].G + 63) / 64)), dim3(64), 0, s, d, stages[2]);
  tl->mark("k_pv_stage3_fbsum", s, B * stages[2].T * COST_FB);
  hipLaunchKernelGGL(k_pv_segsum, dim3((unsigned)((d.B * stages[2].S + 63) / 64)), dim3(64), 0, s, d, stages[2]);
  tl->mark("k_pv_stage3_segsum", s, B * (stages[2].G - stages[2].S) * 16.0);
  hipLaunchKernelGGL(k_pv_hp, gp, bs, 0, s, d);
  tl->mark("k_pv_hp", s, B * (d.n + 1) * 9.0);
  launch_x0(d.B, d.n, d.k, d.status, d.hp_be, x0_const, x0_tmpl, d.sc_ip, d.x0_msgs, d.ch, s);
  tl->mark("k_pv_x0", s, 0);
  // IPA rounds (round 0 per kernel, the rest as one span)
  const PvStage& r0 = stages[3];
  for (int j = 0; j < d.k; j++) {
    hipLaunchKernelGGL(k_pv_round, gp, bs, 0, s, d, j);
    if (j == 0) tl->mark("k_pv_round_fr", s, B * 8.0 * d.n);
    hipLaunchKernelGGL(k_pv_fbsum, dim3((unsigned)((d.B * stages[3 + j].G + 63) / 64)), dim3(64), 0, s, d,
                       stages[3 + j]);
    if (j == 0) tl->mark("k_pv_round_fbsum", s, B * r0.T * COST_FB);
    hipLaunchKernelGGL(k_pv_segsum, dim3((unsigned)((d.B * stages[3 + j].S + 63) / 64)), dim3(64), 0, s, d,
                       stages[3 + j]);
    if (j == 0) tl->mark("k_pv_round_segsum", s, B * (r0.G - r0.S) * 16.0);
    hipLaunchKernelGGL(k_pv_lr, gp, bs, 0, s, d, j);
    if (j == 0) tl->mark("k_pv_round_lr", s, B * 20.0);
  }
  hipLaunchKernelGGL(k_pv_round, gp, bs, 0, s, d, d.k);
  tl->mark("k_pv_rounds_rest", s, B * (d.k - 1) * (r0.T * COST_FB + 8.0 * d.n));
}

}  // namespace fts

namespace fts {
// ------------------------------------------------------------ sigma provers
// TypeAndSum prover (transfer/typeandsum.go:189-227,280-356 as transfer.go:69-150
// calls it) and SameType prover (issue/sametype.go:103-149), thread per action.
// Every transcript point is a sum of two fixed-base products over ped0/ped1/ped2:
// in'_i = In_i - CT = v_i ped1 + (bf_i - tbf) ped2 (the type terms cancel), and
// sum = (sum v_in - sum v_out) ped1 + sumbf ped2 -- group-equal to the reference's
// subtractions, so the affine encodings (and the challenge) are identical.
FTS_DEV Scalar sp_canon(const Fr& m) { return fr_canon(m); }
FTS_DEV Scalar sp_raw(const uint32_t* p) {
  Scalar s;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = p[i];
  return s;
}
__global__ void __launch_bounds__(64) k_sp_prove(SpDev d) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= d.A) return;
  const SpAction ac = d.act[a];
  const uint32_t* S = d.sc + (size_t)ac.sc_off * 8;
  const uint32_t* t0 = d.tables + (size_t)tb_ped0(d.n) * FB_WORDS_PER_BASE;
  const uint32_t* t1 = d.tables + (size_t)tb_G(d.n) * FB_WORDS_PER_BASE;
  const uint32_t* t2 = d.tables + (size_t)tb_H(d.n) * FB_WORDS_PER_BASE;
  uint32_t* J = d.jac + (size_t)ac.pt_off * 24;
  auto pt2 = [&](int slot, const uint32_t* ta, const Scalar& ka, const uint32_t* tb, const Scalar& kb) {
    G1J acc = g1j_identity();
    if (ta) fb_mul_acc(acc, ta, ka);
    fb_mul_acc(acc, tb, kb);
    store_g1j(J + slot * 24, acc);
  };
  auto mont = [&](int i) { return fr_from_canon(S + i * 8); };
  const Fr type = mont(0), tbf = mont(1), r_t = mont(2);
  int m;
  if (ac.kind == 0) {
    const int N = ac.n_in, M = ac.n_out;
    const int IV = 5, IBF = 5 + N, RIV = 5 + 2 * N, RIBF = 5 + 3 * N, OV = 5 + 4 * N, OBF = 5 + 4 * N + M;
    for (int i = 0; i < N; i++) pt2(i, t1, sp_raw(S + (RIV + i) * 8), t2, sp_raw(S + (RIBF + i) * 8));  // cin_i
    pt2(N, t0, sp_raw(S + 2 * 8), t2, sp_raw(S + 3 * 8));                                           // cct
    pt2(N + 1, nullptr, Scalar{}, t2, sp_raw(S + 4 * 8));                                           // csum
    Fr sumv = f_zero<FrP>(), sumbf = f_zero<FrP>();
    for (int i = 0; i < N; i++) {
      const Fr d_bf = f_sub(mont(IBF + i), tbf);
      sumv = f_add(sumv, mont(IV + i));
      sumbf = f_add(sumbf, d_bf);
      pt2(N + 2 + i, t1, sp_raw(S + (IV + i) * 8), t2, sp_canon(d_bf));                             // in'_i
    }
    for (int j = 0; j < M; j++) {
      const Fr d_bf = f_sub(mont(OBF + j), tbf);
      sumv = f_sub(sumv, mont(OV + j));
      sumbf = f_sub(sumbf, d_bf);
      pt2(2 * N + 2 + j, t1, sp_raw(S + (OV + j) * 8), t2, sp_canon(d_bf));                         // out'_j
    }
    pt2(2 * N + M + 2, t0, sp_raw(S), t2, sp_raw(S + 8));                                           // CT
    pt2(2 * N + M + 3, t1, sp_canon(sumv), t2, sp_canon(sumbf));                                    // sum
    m = 2 * N + M + 4;
    // challenge over Arr(cin..., cct, csum, in'..., out'..., CT, sum)   typeandsum.go:210-221
    uint32_t* A = d.aff + (size_t)ac.pt_off * 16;
    batch_to_affine(J, A, m);
    uint8_t* msg = d.msgs + ac.msg_off;
    for (int i = 0; i < m; i++) {
      const G1A p = load_g1a(A + i * 16);
      store_point_be(d.be + ((size_t)ac.pt_off + i) * 64, p);
      uint32_t pw[16];
      g1_mont_to_be_words(p.x, p.y, pw);
      put_hex_record(msg, 130u * i, pw, i + 1 < m);
    }
    const uint32_t len = 130u * m - 2u;
    write_sha_padding_u16(msg, len);
    uint32_t st[8];
    sha256_blocks(msg, sha_blocks(len), st);
    const Fr chal = f_to_mont(digest_to_fr(st));
    uint32_t* O = d.out + (size_t)ac.out_off * 8;
    for (int i = 0; i < N; i++) {
      pv_put_canon(O + i * 8, f_add(fr_mul(chal, f_sub(mont(IBF + i), tbf)), mont(RIBF + i)));  // pibf_i
      pv_put_canon(O + (N + i) * 8, f_add(fr_mul(chal, mont(IV + i)), mont(RIV + i)));          // piv_i
    }
    pv_put_canon(O + (2 * N) * 8, f_add(fr_mul(chal, type), r_t));
    pv_put_canon(O + (2 * N + 1) * 8, f_add(fr_mul(chal, tbf), mont(3)));
    pv_put_canon(O + (2 * N + 2) * 8, f_add(fr_mul(chal, sumbf), mont(4)));
    pv_put_canon(O + (2 * N + 3) * 8, chal);
  } else {
    pt2(0, t0, sp_raw(S), t2, sp_raw(S + 8));          // CT
    pt2(1, t0, sp_raw(S + 2 * 8), t2, sp_raw(S + 3 * 8));  // r_t ped0 + r_bf ped2
    m = 2;
    uint32_t* A = d.aff + (size_t)ac.pt_off * 16;
    batch_to_affine(J, A, m);
    uint8_t* msg = d.msgs + ac.msg_off;
    for (int i = 0; i < m; i++) {
      const G1A p = load_g1a(A + i * 16);
      store_point_be(d.be + ((size_t)ac.pt_off + i) * 64, p);
      uint32_t pw[16];
      g1_mont_to_be_words(p.x, p.y, pw);
      put_hex_record(msg, 130u * i, pw, i + 1 < m);  // Arr(CT, com)   sametype.go:127
    }
    const uint32_t len = 130u * m - 2u;
    write_sha_padding_u16(msg, len);
    uint32_t st[8];
    sha256_blocks(msg, sha_blocks(len), st);
    const Fr chal = f_to_mont(digest_to_fr(st));
    uint32_t* O = d.out + (size_t)ac.out_off * 8;
    pv_put_canon(O, f_add(fr_mul(chal, type), r_t));
    pv_put_canon(O + 8, f_add(fr_mul(chal, tbf), mont(3)));
    pv_put_canon(O + 16, chal);
  }
}

void launch_sigma_prove(const SpDev& d, hipStream_t s) {
  if (d.A <= 0) return;
  hipLaunchKernelGGL(k_sp_prove, dim3((unsigned)((d.A + 63) / 64)), dim3(64), 0, s, d);
}
}  // namespace fts
