// Split-wave PV filter of the latency-regime estimator rollout (gfx950).
//
// At 4096 envs an estimator wave is one dependent instruction chain on an otherwise idle CU, and the float64 PV
// covariance step is ~35 % of it.  The covariance, though, feeds the state chain only through the gains of a
// fix: on the 12 of 21 steps without one (position fix every 7th step, velocity fix every 3rd, per env), nothing
// the step computes afterwards reads it.  So each 64-slot tile runs as a 128-thread workgroup of two waves on two
// SIMDs of one CU: the state wave (wave 0) runs the whole step except the covariance; the covariance wave (wave 1)
// holds the 9x9 covariance of the same 64 envs in its registers and runs predict / gains / corrections.  They
// meet in LDS:
//   * state -> covariance: the step's attitude estimate (the quaternion the PV rotation is formed from), one
//     ring slot per step of the launch, and the count of steps published;
//   * covariance -> state: the gains of a fix (S^-1 and the two other blocks' K rows, float64), one slot per
//     fix type, and the step whose gains it holds.
// The state wave waits only on a fix step, for the gains, and only after the part of its step that does not
// read the estimate (guidance, the rotation, the husky); the predict of every other step runs beside its chain.  Every element is computed by the quad_math.h formulas (pv_state_predict, pv_cov_predict_t, pv_gain_t,
// pv_x_correct_t, pv_cov_correct_t) on the same operands as the one-lane pv_step, so the state and covariance
// are bit for bit those of the one-lane kernels.
//
// Progress: each wave waits only for a count the other wave raises unconditionally in program order (the state
// wave publishes step k's attitude before it can wait for step k's gains; the covariance wave publishes those
// gains right after computing them from that attitude), both waves of the workgroup are resident together, and
// both run the same K steps with the same wave-uniform fix decisions.  A wait that still exceeds
// g_ouz_split_spin_limit polls (kSplitSpinLimit, ~70 ms, unless a test lowers it with ouz_set_split_spin_limit)
// gives up, counts itself in g_ouz_split_timeouts (ouz_split_timeouts) and lets the launch drain: a protocol error
// shows up as a count, never as a hung GPU.  The count is not silent: QuadVecTask reads it at its synchronisation
// points (check_health) and raises, and bench.py records it and fails on a non-zero count.
#pragma once
#include "quad_math.h"

namespace ouz {

constexpr int kSplitRing = 32;                  // attitude slots: one per step of a launch (kMaxRolloutChunk)
constexpr uint32_t kSplitSpinLimit = 1u << 20;  // polls of ~64 cycles before a wait gives up

__device__ uint32_t g_ouz_split_timeouts;
__device__ uint32_t g_ouz_split_spin_limit = kSplitSpinLimit;

struct SplitPvLds {
  float4 att[kSplitRing][64];   // [step][lane] the quaternion (w, x, y, z) the PV step of that step uses
  double gain[2][27][64];       // [fix][Si 9 | KA 9 | KB 9][lane]; fix 0 = position, 1 = velocity
  int att_count;                // steps whose attitude is published
  int gain_step[2];             // step + 1 whose gains the slot holds
};

struct SplitLane {
  SplitPvLds* L;
  int k;                        // the step of the launch (set by the caller before each step)
  uint32_t lane;
};

__device__ __forceinline__ void split_publish(int* f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Waits until *f >= v; returns the count it saw (v after a give-up), so that a caller may skip later waits the
// count already covers.
__device__ __forceinline__ int split_wait(int* f, int v) {
  for (uint32_t it = 0;; ++it) {
    const int seen = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (seen >= v) return seen;
    if (it >= g_ouz_split_spin_limit) {
      atomicAdd(&g_ouz_split_timeouts, 1u);
      return v;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The state wave's PV step, in three parts placed in its step (env_core): publish the attitude right after the
// EKF; predict the state (f64, kept in xd); after the work that does not read the estimate, wait for and apply
// the gains of this step's fixes and round to the f32 state.  The same operations on the same operands as
// pv_step's state part.
__device__ __forceinline__ void pv_split_publish(const SplitLane& sl, EkfQ q) {
  SplitPvLds& L = *sl.L;
  L.att[sl.k][sl.lane] = make_float4(q.w, q.x, q.y, q.z);
  split_publish(&L.att_count, sl.k + 1);
}

__device__ __forceinline__ void pv_split_predict(const float xf[9], V3 acc, EkfQ q, float dt, PvReal x[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = (PvReal)xf[k];
  const PvReal a[3] = {(PvReal)acc.x, (PvReal)acc.y, (PvReal)acc.z};
  const M3T<PvReal> M = pv_rot<PvReal>(q);
  const PvReal dtd = (PvReal)dt;
  pv_state_predict(x, a, M, dtd, dtd * dtd * PvReal(0.5));
}

__device__ __forceinline__ void pv_split_correct(const SplitLane& sl, PvReal x[9], float xf[9], bool pos_fix, V3 zp,
                                                 bool vel_fix, V3 zv) {
  SplitPvLds& L = *sl.L;
  M3T<PvReal> Si;
  PvReal KA[3][3], KB[3][3];
  const auto read_gains = [&](int f) {
#pragma unroll
    for (int j = 0; j < 9; ++j) Si.m[j] = L.gain[f][j][sl.lane];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      KA[j / 3][j % 3] = L.gain[f][9 + j][sl.lane];
      KB[j / 3][j % 3] = L.gain[f][18 + j][sl.lane];
    }
  };
  if (__any(pos_fix)) {
    split_wait(&L.gain_step[0], sl.k + 1);
    read_gains(0);
    const PvReal z[3] = {(PvReal)zp.x, (PvReal)zp.y, (PvReal)zp.z};
    if (pos_fix) pv_x_correct_t<0, PvReal>(x, z, (PvReal)kPvPosVar, Si, KA, KB);
  }
  if (__any(vel_fix)) {
    split_wait(&L.gain_step[1], sl.k + 1);
    read_gains(1);
    const PvReal z[3] = {(PvReal)zv.x, (PvReal)zv.y, (PvReal)zv.z};
    if (vel_fix) pv_x_correct_t<1, PvReal, true>(x, z, PvReal(0), Si, KA, KB);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) xf[k] = (float)x[k];
}

// The covariance wave's PV step k on its registers (pf: the f32-stored covariance, as the one-lane form keeps it
// between steps).  fixes: this lane's (valid) fix decisions, evaluated exactly as the state wave does.
__device__ __forceinline__ void pv_cov_split(SplitPvLds& L, int k, uint32_t lane, float pf[45], float dt,
                                             bool pos_fix, bool vel_fix) {
  split_wait(&L.att_count, k + 1);
  if (kStampSlots > 13 && k == 8) OUZ_STAMP(30, false);
  const float4 o = L.att[k][lane];
  PvReal P[45];
#pragma unroll
  for (int f = 0; f < 45; ++f) P[f] = (PvReal)pf[f];
  pv_cov_predict_t(P, pv_rot<PvReal>(EkfQ{o.x, o.y, o.z, o.w}), (PvReal)dt);
  M3T<PvReal> Si;
  PvReal KA[3][3], KB[3][3];
  const auto write_gains = [&](int f) {
#pragma unroll
    for (int j = 0; j < 9; ++j) L.gain[f][j][lane] = Si.m[j];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      L.gain[f][9 + j][lane] = KA[j / 3][j % 3];
      L.gain[f][18 + j][lane] = KB[j / 3][j % 3];
    }
  };
  if (__any(pos_fix)) {
    pv_gain_t<0, PvReal>(P, (PvReal)kPvPosVar, Si, KA, KB);
    write_gains(0);
    split_publish(&L.gain_step[0], k + 1);
    if (pos_fix) pv_cov_correct_t<0, PvReal>(P, (PvReal)kPvPosVar, Si, KA, KB);
  }
  if (__any(vel_fix)) {
    pv_gain_t<1, PvReal>(P, PvReal(0), Si, KA, KB);
    write_gains(1);
    split_publish(&L.gain_step[1], k + 1);
    if (vel_fix) pv_cov_correct_t<1, PvReal, true>(P, PvReal(0), Si, KA, KB);
  }
#pragma unroll
  for (int f = 0; f < 45; ++f) pf[f] = (float)P[f];
  if (kStampSlots > 13 && k == 8) OUZ_STAMP(31, false);
}

}  // namespace ouz
