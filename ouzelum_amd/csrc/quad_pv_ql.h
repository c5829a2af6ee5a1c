// Quad-lane ("QL") PV-filter step of the latency-regime estimator kernels (gfx950).
//
// At 4096 envs an estimator wave is one dependent instruction chain on an otherwise idle CU, and the float64
// PV covariance step is ~35 % of its instructions.  Here the four lanes of an env split that step: lane c
// (c = lane & 3; lane 3 mirrors lane 0 and never writes) owns column c of every 3x3 block of the 9x9
// covariance, so each lane evaluates a third of the block products.  The covariance lives in LDS as the upper
// triangle of the symmetric 9x9 (f64) for the whole launch; after a wave-local fence any lane reads any element
// through its upper position (qcol).  The 3x3 matrices whose full
// rows every column needs (Z00 / Z01 / Z11 of the predict, the gains K of a correction) go through an LDS
// exchange slot.  Every stored element is computed by the element formulas of quad_math.h (pvf_g0, pvf_g1,
// pvf_z, dot3, dot3s, inv_sym3) on the same operands as the one-lane pv_step, so the two forms agree bit for
// bit (the large-N kernels keep the one-lane form); like it, the step's results are rounded to f32 once, at
// its end (RND marks the last phase of the step: every correction rewrites all 45 stored elements, the
// predict all but the bias block, which it leaves unchanged).
//
// LDS traffic (measured, profiles/r03/): only the upper triangle of the 9x9 is written and every read addresses
// an element by its upper position (row <= column), which halves the writes of a mirrored image; the per-env
// stride of 131 doubles (262 dwords = 6 mod 64 banks) spreads the 16 envs x 3 columns of a wave over the banks
// (the 108-double stride put envs 0 / 4 / 8 / 12 on one bank: ~45 cycles per ds_write_b64).
#pragma once
#include "quad_math.h"

#ifndef OUZ_QL_STAMP
#define OUZ_QL_STAMP(k) do {} while (0)   // instrumented builds (-DOUZ_STAMPS): sub-phase stamps
#endif

namespace ouz {

constexpr int kPvLdsP = 81;                  // doubles of the 9x9 covariance (upper triangle used)
constexpr int kPvLdsX = 27;                  // doubles of the exchange slot (three 3x3 matrices)
constexpr int kPvLdsEnv = 131;               // per env, padded: 131 doubles = 262 dwords = 6 (mod 64 banks)
static_assert(kPvLdsEnv >= kPvLdsP + kPvLdsX, "LDS image of one env");

struct PvQl {
  double* P;      // this env's 9x9 (row-major) in LDS; the upper triangle holds the covariance
  double* X;      // this env's exchange slot
  int c;          // this lane's block column (0..2)
  bool own;       // lanes 0..2 write; lane 3 computes lane 0's column and stays silent
};
// element k of column c of block (rb, bb), P[3 rb + k][3 bb + c], read at its upper position.  rb, bb and k
// are compile-time after unrolling, so only a diagonal block's element below the diagonal (k > c) costs a
// per-lane choice.
__device__ __forceinline__ double qcol(const PvQl& L, int rb, int bb, int k) {
  if (rb < bb) return L.P[(3 * rb + k) * 9 + 3 * bb + L.c];
  if (rb > bb) return L.P[(3 * bb + L.c) * 9 + 3 * rb + k];
  return k <= L.c ? L.P[(3 * rb + k) * 9 + 3 * bb + L.c] : L.P[(3 * bb + L.c) * 9 + 3 * rb + k];
}

// Wave-local LDS ordering: the wave's LDS accesses execute in program order; these keep the compiler from
// moving them across an exchange (the same fence pair as the obs staging's wave_lds_sync).
__device__ __forceinline__ void ql_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool RND>
__device__ __forceinline__ double rnd32(double v) { return RND ? (double)(float)v : v; }

// write element (r, k), r <= k, of the symmetric covariance (its upper position)
__device__ __forceinline__ void ql_put(const PvQl& L, int r, int k, double v) { L.P[r * 9 + k] = v; }

// one of three lane-indexed values: v[c] for this lane's c
__device__ __forceinline__ double ql_sel(int c, double v0, double v1, double v2) {
  return c == 0 ? v0 : (c == 1 ? v1 : v2);
}

template <bool RND>
__device__ __forceinline__ void pv_predict_ql(const PvQl& L, double x[9], const double acc[3], EkfQ q, double dt) {
  const M3T<double> M = pv_rot<double>(q);
  const double h = dt * dt * 0.5;
  pv_state_predict(x, acc, M, dt, h);
  const double q_a = (double)kPvAccVar, qhh = q_a * h * h, qhd = q_a * h * dt, qdd = q_a * dt * dt;
  const int c = L.c;
  // column c of the G blocks from column c of the P blocks (X_{r,b}[k][c] = P[3r + k][3b + c])
  double g0[3][3], g1[2][3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    double X0[3], X1[3], X2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      X0[k] = qcol(L, 0, b, k);
      X1[k] = qcol(L, 1, b, k);
      X2[k] = qcol(L, 2, b, k);
    }
    pvf_g0(M, X0, X1, X2, dt, h, g0[b]);
    if (b > 0) pvf_g1(M, X1, X2, dt, g1[b - 1]);
  }
  double z00[3], z01[3], z11[3];
  pvf_z(g0[1], g0[2], g1[0], g1[1], dt, h, z00, z01, z11);
  OUZ_QL_STAMP(14);
  // exchange the Z columns: X[m * 9 + col * 3 + row]
  if (L.own) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      L.X[c * 3 + i] = z00[i];
      L.X[9 + c * 3 + i] = z01[i];
      L.X[18 + c * 3 + i] = z11[i];
    }
  }
  ql_sync();
  double Z[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) Z[k] = L.X[k];
  OUZ_QL_STAMP(15);
  const double m0 = ql_sel(c, M.m[0], M.m[3], M.m[6]), m1 = ql_sel(c, M.m[1], M.m[4], M.m[7]),
               m2 = ql_sel(c, M.m[2], M.m[5], M.m[8]);   // row c of M
  double p00[3], p01[3], p11[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    p00[i] = rnd32<RND>(dot3s(Z[i], Z[3 + i], Z[6 + i], m0, m1, m2, i == c ? g0[0][i] + qhh : g0[0][i]));
    p01[i] = rnd32<RND>(dot3s(Z[9 + i], Z[12 + i], Z[15 + i], m0, m1, m2, i == c ? qhd : 0.0));
    p11[i] = rnd32<RND>(dot3s(Z[18 + i], Z[21 + i], Z[24 + i], m0, m1, m2, i == c ? qdd : 0.0));
  }
  OUZ_QL_STAMP(16);
  if (L.own) {   // the old P was read above (in-order LDS): overwrite its upper triangle
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i <= c) ql_put(L, i, c, p00[i]);
      ql_put(L, i, 3 + c, p01[i]);
      if (i <= c) ql_put(L, 3 + i, 3 + c, p11[i]);
      ql_put(L, i, 6 + c, rnd32<RND>(g0[2][i]));
      ql_put(L, 3 + i, 6 + c, rnd32<RND>(g1[1][i]));
    }
  }
  ql_sync();
  OUZ_QL_STAMP(17);
}

template <int MB, bool R0, bool RND>
__device__ __forceinline__ void pv_correct_ql(const PvQl& L, double x[9], const double z[3], double r) {
  constexpr int A = (MB == 0) ? 1 : 0;
  constexpr int B = 2;
  const int c = L.c;
  M3T<double> S;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) S.m[i * 3 + j] = S.m[j * 3 + i] = L.P[(3 * MB + i) * 9 + 3 * MB + j];
  S.m[0] += r; S.m[4] += r; S.m[8] += r;
  const M3T<double> Si = inv_sym3(S);
  // row c of K_A = P_{A,m} S^-1 and of K_B
  double ka[3], kb[3];
  {
    // row c of P_{A,m} and P_{B,m} = column c of P_{m,A} and P_{m,B}
    const double a0 = qcol(L, MB, A, 0), a1 = qcol(L, MB, A, 1), a2 = qcol(L, MB, A, 2);
    const double b0 = qcol(L, MB, B, 0), b1 = qcol(L, MB, B, 1), b2 = qcol(L, MB, B, 2);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ka[j] = dot3(a0, a1, a2, Si.m[j], Si.m[3 + j], Si.m[6 + j]);
      kb[j] = dot3(b0, b1, b2, Si.m[j], Si.m[3 + j], Si.m[6 + j]);
    }
  }
  if (L.own) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      L.X[c * 3 + j] = ka[j];
      L.X[9 + c * 3 + j] = kb[j];
    }
  }
  ql_sync();
  double KA[3][3], KB[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      KA[i][j] = L.X[i * 3 + j];
      KB[i][j] = L.X[9 + i * 3 + j];
    }
  {
#pragma clang fp contract(off)
    double y[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) y[k] = z[k] - x[MB * 3 + k];
    double xm[3], dA[3], dB[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      xm[i] = R0 ? z[i] : fma(-r, dot3(Si.m[i * 3], Si.m[i * 3 + 1], Si.m[i * 3 + 2], y[0], y[1], y[2]), z[i]);
      dA[i] = dot3(KA[i][0], KA[i][1], KA[i][2], y[0], y[1], y[2]);
      dB[i] = dot3(KB[i][0], KB[i][1], KB[i][2], y[0], y[1], y[2]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      x[MB * 3 + k] = xm[k];
      x[A * 3 + k] += dA[k];
      x[B * 3 + k] += dB[k];
    }
  }
  // column c of the other-other blocks
  double bb[3], ab[3], aa[3];
  {
    const double pb0 = qcol(L, MB, B, 0), pb1 = qcol(L, MB, B, 1), pb2 = qcol(L, MB, B, 2);
    const double pa0 = qcol(L, MB, A, 0), pa1 = qcol(L, MB, A, 1), pa2 = qcol(L, MB, A, 2);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      bb[i] = rnd32<RND>(dot3s(-KB[i][0], -KB[i][1], -KB[i][2], pb0, pb1, pb2, qcol(L, B, B, i)));
      ab[i] = rnd32<RND>(dot3s(-KA[i][0], -KA[i][1], -KA[i][2], pb0, pb1, pb2, qcol(L, A, B, i)));
      aa[i] = rnd32<RND>(dot3s(-KA[i][0], -KA[i][1], -KA[i][2], pa0, pa1, pa2, qcol(L, A, A, i)));
    }
  }
  // column c of the m-row blocks: MB < A: P_{m,A}[i][c] = r KA[c][i]; else P_{A,m}[i][c] = r KA[i][c];
  // P_{m,B}[i][c] = r KB[c][i]; P_mm[i][c] = r (delta - r S^-1[i][c])
  double ma[3], mb[3], mm[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if constexpr (R0) {
      ma[i] = mb[i] = mm[i] = 0.0;
    } else {
#pragma clang fp contract(off)
      ma[i] = rnd32<RND>(r * (MB < A ? ka[i] : ql_sel(c, KA[i][0], KA[i][1], KA[i][2])));
      mb[i] = rnd32<RND>(r * kb[i]);
      mm[i] = rnd32<RND>(r * fma(-r, ql_sel(c, Si.m[i * 3], Si.m[i * 3 + 1], Si.m[i * 3 + 2]), i == c ? 1.0 : 0.0));
    }
  }
  if (L.own) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i <= c) ql_put(L, 6 + i, 6 + c, bb[i]);
      ql_put(L, 3 * A + i, 6 + c, ab[i]);
      if (i <= c) ql_put(L, 3 * A + i, 3 * A + c, aa[i]);
      if (MB < A) ql_put(L, 3 * MB + i, 3 * A + c, ma[i]); else ql_put(L, 3 * A + i, 3 * MB + c, ma[i]);
      ql_put(L, 3 * MB + i, 6 + c, mb[i]);
      if (i <= c) ql_put(L, 3 * MB + i, 3 * MB + c, mm[i]);
    }
  }
  ql_sync();
}

// pv_step (quad_math.h) in the quad-lane form: x in every lane's registers, the covariance in LDS
__device__ __forceinline__ void pv_step_ql(const PvQl& L, float xf[9], V3 acc, EkfQ q, float dt, bool pos_fix, V3 zp,
                                           bool vel_fix, V3 zv) {
  double x[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = (double)xf[k];
  const double a[3] = {(double)acc.x, (double)acc.y, (double)acc.z};
  // the trigger flags are wave-uniform under the trigger-class layout: one specialised body per case
  const double zpd[3] = {(double)zp.x, (double)zp.y, (double)zp.z};
  const double zvd[3] = {(double)zv.x, (double)zv.y, (double)zv.z};
  if (!pos_fix && !vel_fix) {
    pv_predict_ql<true>(L, x, a, q, (double)dt);
  } else {
    pv_predict_ql<false>(L, x, a, q, (double)dt);
    if (pos_fix) {
      if (vel_fix) pv_correct_ql<0, false, false>(L, x, zpd, (double)kPvPosVar);
      else pv_correct_ql<0, false, true>(L, x, zpd, (double)kPvPosVar);
    }
    if (vel_fix) pv_correct_ql<1, true, true>(L, x, zvd, 0.0);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) xf[k] = (float)x[k];
}

// The covariance between HBM (packed upper f32, OUZ_F_PV_P) and LDS (upper triangle, f64).  Lane c moves the packed
// elements it owns: column c of the upper blocks and the upper part (i <= c) of column c of the diagonal
// blocks -- packed index s9(r, 3b + c) = g9(r) + 3b + c for r <= 3b + c, linear in c, so every access is the
// lane's one offset (c fields further) plus an immediate.
__host__ __device__ constexpr int g9(int r) { return r * 9 - (r * (r - 1)) / 2 - r; }   // s9(r, j) = g9(r) + j, j >= r
template <typename LD>
__device__ __forceinline__ void pv_lds_load(const PvQl& L, LD load_field) {
  if (!L.own) return;
  const int c = L.c;
#pragma unroll
  for (int b = 0; b < 3; ++b)
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      if (r >= 3 * b + 3) continue;                 // lower block: its mirror is loaded
      const int row_in = r - 3 * b;                  // diagonal block: upper part only (r <= 3b + c)
      if (row_in >= 0 && row_in > c) continue;
      const int f = g9(r) + 3 * b + c;               // = s9(r, 3b + c) since r <= 3b + c
      ql_put(L, r, 3 * b + c, (double)load_field(f));
    }
}
template <typename ST>
__device__ __forceinline__ void pv_lds_store(const PvQl& L, ST store_field) {
  if (!L.own) return;
  const int c = L.c;
#pragma unroll
  for (int b = 0; b < 3; ++b)
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      if (r >= 3 * b + 3) continue;
      const int row_in = r - 3 * b;
      if (row_in >= 0 && row_in > c) continue;
      store_field(g9(r) + 3 * b + c, (float)L.P[r * 9 + 3 * b + c]);
    }
}

}  // namespace ouz
