// Lane-cooperative Jacobian point arithmetic for latency-bound chains.
//
// A wave issues one instruction stream for all 64 lanes, so a kernel whose
// critical path is ONE dependent chain of point operations (the MSM's final
// window shifts: ~114 doublings on one lane) pays the full wave issue cost for
// every field product of the chain.  Here a group of COOP_G = 5 lanes holds the
// same point and each lane computes a different field product of the same
// formula level; the products are exchanged with ds_bpermute (__shfl).  The
// wave still issues one product per level, but a doubling takes 3 levels
// instead of 7 dependent products and an addition 5 instead of 16.
//
// The formulas and their operation order are those of g1j_dbl / add_inl
// (dbl-2009-l, add-2007-bl), so the results are the same Jacobian triples,
// bit for bit.  Every lane of a group must call with the same inputs and the
// same control flow (the branches below depend only on the shared values).
#pragma once
#include "g1.hpp"

namespace fts {

constexpr int COOP_G = 5;  // lanes per cooperative group

FTS_DEV Fp coop_shfl(const Fp& a, int src) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)__shfl((int)a.v[i], src, 64);
  return r;
}

// 2P; role = lane's index in its group (0..COOP_G-1), base = the group's first lane
FTS_DEV G1J coop_dbl(const G1J& p, int role, int base) {
  if (f_is_zero(p.z) || f_is_zero(p.y)) return g1j_identity();
  // level 1: A = X^2 (0), B = Y^2 (1), T = Y Z (2)
  const Fp a1 = role == 0 ? p.x : p.y;
  const Fp b1 = role == 0 ? p.x : role == 1 ? p.y : p.z;
  const Fp m1 = fp_mul(a1, b1);
  const Fp A = coop_shfl(m1, base), B = coop_shfl(m1, base + 1), T = coop_shfl(m1, base + 2);
  // level 2: C = B^2 (0), (X + B)^2 (1), F = E^2 with E = 3A (2)
  const Fp E = f_add(f_dbl(A), A);
  const Fp u = role == 0 ? B : role == 1 ? f_add(p.x, B) : E;
  const Fp m2 = fp_mul(u, u);
  const Fp C = coop_shfl(m2, base), S = coop_shfl(m2, base + 1), F = coop_shfl(m2, base + 2);
  Fp D = f_sub(f_sub(S, A), C);
  D = f_dbl(D);
  G1J r;
  r.x = f_sub(F, f_dbl(D));
  const Fp C8 = f_dbl(f_dbl(f_dbl(C)));
  // level 3 (every lane, one product)
  r.y = f_sub(fp_mul(E, f_sub(D, r.x)), C8);
  r.z = f_dbl(T);
  return r;
}

// p += q (both Jacobian)
FTS_DEV void coop_add(G1J& p, const G1J& q, int role, int base) {
  if (f_is_zero(q.z)) return;
  if (f_is_zero(p.z)) {
    p = q;
    return;
  }
  // level 1: z1z1 = Z1^2 (0), z2z2 = Z2^2 (1), Y1 Z2 (2), Y2 Z1 (3), (Z1 + Z2)^2 (4)
  const Fp zs = f_add(p.z, q.z);
  const Fp a1 = role == 0 ? p.z : role == 1 ? q.z : role == 2 ? p.y : role == 3 ? q.y : zs;
  const Fp b1 = role == 0 ? p.z : role == 1 ? q.z : role == 2 ? q.z : role == 3 ? p.z : zs;
  const Fp m1 = fp_mul(a1, b1);
  const Fp z1z1 = coop_shfl(m1, base), z2z2 = coop_shfl(m1, base + 1), y1z2 = coop_shfl(m1, base + 2),
           y2z1 = coop_shfl(m1, base + 3), zz = coop_shfl(m1, base + 4);
  // level 2: u1 = X1 z2z2 (0), u2 = X2 z1z1 (1), s1 = Y1 Z2 z2z2 (2), s2 = Y2 Z1 z1z1 (3)
  const Fp a2 = role == 0 ? p.x : role == 1 ? q.x : role == 2 ? y1z2 : y2z1;
  const Fp b2 = (role == 0 || role == 2) ? z2z2 : z1z1;
  const Fp m2 = fp_mul(a2, b2);
  const Fp u1 = coop_shfl(m2, base), u2 = coop_shfl(m2, base + 1), s1 = coop_shfl(m2, base + 2),
           s2 = coop_shfl(m2, base + 3);
  const Fp h = f_sub(u2, u1);
  Fp rr = f_sub(s2, s1);
  if (f_is_zero(h)) {
    p = f_is_zero(rr) ? coop_dbl(p, role, base) : g1j_identity();
    return;
  }
  rr = f_dbl(rr);
  // level 3: i = (2h)^2 (0), rr^2 (1), (zz - z1z1 - z2z2) h (2)
  const Fp h2 = f_dbl(h);
  const Fp zd = f_sub(f_sub(zz, z1z1), z2z2);
  const Fp a3 = role == 0 ? h2 : role == 1 ? rr : zd;
  const Fp b3 = role == 0 ? h2 : role == 1 ? rr : h;
  const Fp m3 = fp_mul(a3, b3);
  const Fp i = coop_shfl(m3, base), r2 = coop_shfl(m3, base + 1), z3 = coop_shfl(m3, base + 2);
  // level 4: j = h i (0), v = u1 i (1)
  const Fp m4 = fp_mul(role == 0 ? h : u1, i);
  const Fp j = coop_shfl(m4, base), v = coop_shfl(m4, base + 1);
  const Fp x3 = f_sub(f_sub(r2, j), f_dbl(v));
  // level 5: rr (v - x3) (0), s1 j (1)
  const Fp m5 = fp_mul(role == 0 ? rr : s1, role == 0 ? f_sub(v, x3) : j);
  const Fp ya = coop_shfl(m5, base), yb = coop_shfl(m5, base + 1);
  p.x = x3;
  p.y = f_sub(ya, f_dbl(yb));
  p.z = z3;
}

}  // namespace fts
