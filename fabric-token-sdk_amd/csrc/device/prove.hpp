// Layout shared by the batched range-proof prover kernels (prove_kernels.hip)
// and the host driver (fts_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fts {

// host-drawn randomness per proof, canonical Fr, in the reference's draw order
// (bulletproof.go:336-350 then :405-415): rho, eta, (rl_i, rr_i) for i < n, tau1, tau2
inline __host__ __device__ int pv_nrnd(int n) { return 2 * n + 4; }
constexpr int PV_R_RHO = 0, PV_R_ETA = 1;
inline __host__ __device__ int PV_R_RL(int i) { return 2 + 2 * i; }
inline __host__ __device__ int PV_R_RR(int i) { return 3 + 2 * i; }
inline __host__ __device__ int pv_r_tau1(int n) { return 2 * n + 2; }
inline __host__ __device__ int pv_r_tau2(int n) { return 2 * n + 3; }

// per-proof Fr state (Montgomery): a[n], b[n], gc[n], hc[n], y^-i[n]
inline __host__ __device__ int pv_nst(int n) { return 5 * n; }
#define PV_ST_A 0
#define PV_ST_B (n)
#define PV_ST_GC (2 * n)
#define PV_ST_HC (3 * n)
#define PV_ST_YI (4 * n)

// published points per proof (64-byte BE): V, C, D, T1, T2, L_0, R_0, ..., L_{k-1}, R_{k-1}
constexpr int PV_V = 0, PV_C = 1, PV_D = 2, PV_T1 = 3, PV_T2 = 4;
inline __host__ __device__ int PV_L(int j) { return 5 + 2 * j; }
inline __host__ __device__ int PV_R(int j) { return 6 + 2 * j; }
inline __host__ __device__ int pv_npts(int k) { return 5 + 2 * k; }
// published scalars per proof (canonical limbs): tau, delta, ip, a, b
constexpr int PV_F_TAU = 0, PV_F_DELTA = 1, PV_F_IP = 2, PV_F_A = 3, PV_F_B = 4, PV_NFR = 5;

// stage scalars / group partial sums (upper bounds over the stages)
inline __host__ __device__ int pv_tmax(int n) { return 3 * n + 4; }
inline __host__ __device__ int pv_gmax(int n) { return n + 2 * ((n + 7) / 8) + 8; }
constexpr int PV_TPG = 8;       // terms per k_pv_fbsum work item (one accumulator)
constexpr int PV_HSLOT = 512;   // per-proof SHA-256 message scratch (<= 3 hex points)

// one fixed-base stage: T terms (per-term table slot, proof-independent),
// G groups {t0, t1, segment} of <= PV_TPG terms, S output points {g0, g1}
struct PvStage {
  int T, G, S;
  const int32_t* base;
  const int4* grp;
  const int2* seg;
};

struct PvDev {
  int B, n, k;
  const uint32_t* tables;   // context 16-bit window tables (rp_kernels.hpp slots)
  const uint64_t* values;   // [B]
  const uint32_t* rnd;      // [B][pv_nrnd(n)][8] canonical
  const uint32_t* bf;       // [B][8] canonical
  uint32_t* st;             // [B][pv_nst(n)][8]
  uint32_t* terms;          // [B][pv_tmax(n)][8] canonical
  uint32_t* partial;        // [B][pv_gmax(n)][24]
  uint32_t* jac;            // [B][n + 1][24]
  uint32_t* aff;            // [B][n + 1][16]
  uint8_t* hp_be;           // [B][n + 1][64]  H'_0..H'_{n-1}, com (x0 transcript layout)
  uint8_t* out_pts;         // [B][pv_npts(k)][64]
  uint32_t* out_fr;         // [B][PV_NFR][8]
  uint32_t* ch;             // [B][rp_nch(k)][8] Montgomery (CH_* slots)
  uint32_t* sc_ip;          // [B][RP_NSC][8] (RP_SC_IP: Zb(ip) of the x0 transcript)
  int32_t* status;          // [B] zeros (x0 kernels skip non-zero)
  uint8_t* x0_msgs;         // [B][x0_var_bytes(n)]
  uint8_t* hslot;           // [B][PV_HSLOT]
};

}  // namespace fts

namespace fts {
// ---- sigma-proof provers (TypeAndSum for transfers, SameType for issues) ----
// one action to prove; scalar inputs (canonical limbs, 8 words each):
//   TAS [type, tbf, r_t, r_tbf, r_sum, in_v (n_in), in_bf (n_in), r_iv (n_in), r_ibf (n_in),
//        out_v (n_out), out_bf (n_out)]
//   ST  [type, tbf, r_t, r_bf]
// transcript points (sp_npts): TAS [cin_i (n_in), cct, csum, in'_i, out'_j, CT, sum]; ST [CT, cm]
// outputs (canonical): TAS [pibf_i (n_in), piv_i (n_in), ptype, ptbf, peq, chal]; ST [ptype, pbf, chal]
struct SpAction {
  int32_t kind;  // 0 = TypeAndSum (transfer), 1 = SameType (issue)
  int32_t n_in, n_out;
  int32_t sc_off;   // first input scalar
  int32_t pt_off;   // first point slot
  int32_t msg_off;  // transcript slot (bytes)
  int32_t out_off;  // first output scalar
  int32_t ct_idx;   // CT's index among the action's points
};
inline __host__ __device__ int sp_nsc(int kind, int n_in, int n_out) { return kind == 0 ? 5 + 4 * n_in + 2 * n_out : 4; }
inline __host__ __device__ int sp_npts(int kind, int n_in, int n_out) { return kind == 0 ? 2 * n_in + n_out + 4 : 2; }
inline __host__ __device__ int sp_nout(int kind, int n_in) { return kind == 0 ? 2 * n_in + 4 : 3; }
inline __host__ __device__ uint32_t sp_msg_slot(int m) { return ((130u * m - 2u + 9u + 63u) / 64u) * 64u; }

struct SpDev {
  int A;
  const uint32_t* tables;  // context 16-bit tables
  int n;                   // context bit length (table slots)
  const SpAction* act;
  const uint32_t* sc;      // input scalars
  uint32_t* jac;           // [points][24]
  uint32_t* aff;           // [points][16]
  uint8_t* be;             // [points][64]
  uint8_t* msgs;           // transcript slots
  uint32_t* out;           // output scalars
};
}  // namespace fts
