// Fused per-env quadrotor step for MI355X (gfx950) + the C ABI of include/ouzelum.h.
//
// Design:
//  * one env per lane, wave64; per-env state is wave-tiled SoA f32 in HBM
//    (fstate[tile][field][64]) so every field load/store of a wave is one
//    coalesced 256-byte transaction and a wave's whole state is contiguous;
//  * the whole VecTask.step — lazy reset, controller / estimator, wrench,
//    2 integration sub-steps, reward/done/obs — is ONE kernel launch with no
//    host synchronisation (the reference does reset_buf.nonzero() + per-env
//    Python loops, ekf_lee_landed.py:312,378-444);
//  * the task is a template parameter so each config compiles to straight-line
//    code; the mixed curriculum assigns tasks per 64-env block, so every wave
//    is task-uniform and the runtime switch never diverges inside a wave.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ouzelum.h"
#include "quad_math.h"

#define OUZ_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

namespace ouz {


// Instrumented build only (-DOUZ_STAMPS, scripts/build_probe.sh): per-wave s_memtime stamps at the phase
// boundaries, read back with ouz_probe_stamps.  The results are those of the product build; the build reports
// itself through ouz_build_flags() and the Python shim refuses to load it unless OUZ_ALLOW_INSTRUMENTED=1.
#ifdef OUZ_STAMPS
constexpr int kStampSlots = 32, kStampWaves = 1024;   // 0-12 step phases, 13-29 rollout step starts, 30-31 mid-rollout step
__device__ uint64_t g_ouz_stamps[kStampWaves * kStampSlots];
#define OUZ_STAMP(k, wait)                                                                       \
  do {                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    if (wait) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");                               \
    const uint64_t _t = __builtin_amdgcn_s_memtime();                                            \
    const uint32_t _w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;   /* this wave's slot tile */  \
    if ((threadIdx.x & 63) == 0 && _w < (uint32_t)kStampWaves) g_ouz_stamps[_w * kStampSlots + (k)] = _t; \
    __builtin_amdgcn_sched_barrier(0);                                                           \
  } while (0)
#define OUZ_STAMP_RT(k)                                                                          \
  do {                                                                                           \
    const uint64_t _t = __builtin_amdgcn_s_memrealtime();                                        \
    const uint32_t _w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;   /* this wave's slot tile */  \
    if ((threadIdx.x & 63) == 0 && _w < (uint32_t)kStampWaves) g_ouz_stamps[_w * kStampSlots + (k)] = _t; \
  } while (0)
#else
#define OUZ_STAMP(k, wait) do {} while (0)
#define OUZ_STAMP_RT(k) do {} while (0)
constexpr int kStampSlots = 0;
#endif
#define OUZ_QL_STAMP(k) OUZ_STAMP(k, true)
}  // namespace ouz
#include "quad_pv_ql.h"
#include "quad_pv_split.h"
#include "quad_env.h"
namespace ouz {

// ---------------------------------------------------------------------------
// Per-step outputs.  obs is (N, 13) AoS for the learners (vec_task.py:254-258): each wave stages
// its 64 x 13 floats in LDS (lane stride 13 dwords: conflict-free) and writes its contiguous
// 3328-byte slice with 16-byte stores instead of 13 strided dword stores per lane.  Staging is
// wave-local, so waves of one block may run different task paths (mixed curriculum).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct OutPtrs {
  float* obs;
  float* rew;
  int64_t* reset;
  uint8_t* timeouts;
};

// One lane's outputs by env index e (the trigger-class layout: a wave's envs are 21 apart): the 52-byte obs
// row as three 16-byte stores + one dword, reward / flags at [e].  Plain (temporal) stores: the lanes of
// a wave write partial lines 21 envs apart, which the L2 merges with the other class waves' writes to the
// same lines; as non-temporal stores they reached memory as partial writes (QuadTracking 4096 fused step
// 5.23 -> 4.99 us, per-step kernel 8.7 -> 7.6 us with plain stores; profiles/r02/temporal_*).
__device__ __forceinline__ void emit_env(const OutPtrs& o, int e, bool valid, const float* ob, float rew, bool rs,
                                         bool to, bool keep_flags) {
  if (!valid) return;
  typedef float f4a4 __attribute__((ext_vector_type(4), aligned(4)));
  float* row = o.obs + (size_t)e * OUZ_NUM_OBS;
  *reinterpret_cast<f4a4*>(row) = f4a4{ob[0], ob[1], ob[2], ob[3]};
  *reinterpret_cast<f4a4*>(row + 4) = f4a4{ob[4], ob[5], ob[6], ob[7]};
  *reinterpret_cast<f4a4*>(row + 8) = f4a4{ob[8], ob[9], ob[10], ob[11]};
  row[12] = ob[12];
  o.rew[e] = rew;
  if (!(keep_flags && !rs)) {
    o.reset[e] = rs ? 1 : 0;
    o.timeouts[e] = to ? 1 : 0;
  }
}

__device__ __forceinline__ void emit(const OutPtrs& o, float* wave_lds, int i, int n, bool valid, const float* ob,
                                     float rew, bool rs, bool to, bool direct, bool keep_flags = false) {
  const uint32_t lane = (uint32_t)i & 63u;
  const uint32_t first = wave_tile(i) * 64u;   // wave-uniform: output bases live in SGPRs
  if (n <= kLatencyRegimeEnvs && !direct) {
    // Latency regime (a few waves per CU, the step is one dependent chain): each lane stores its own
    // 52-byte row as three 16-byte stores + one dword (rows are 4-byte aligned; gfx950 global stores
    // take dword alignment), skipping the LDS round trip and the wave barrier of the staged form.
    // The staged form's full-line writes only pay off when HBM bandwidth is the bound.
    if (valid) {
      typedef float f4a4 __attribute__((ext_vector_type(4), aligned(4)));
      float* row = o.obs + (size_t)i * OUZ_NUM_OBS;
      *reinterpret_cast<f4a4*>(row) = f4a4{ob[0], ob[1], ob[2], ob[3]};
      *reinterpret_cast<f4a4*>(row + 4) = f4a4{ob[4], ob[5], ob[6], ob[7]};
      *reinterpret_cast<f4a4*>(row + 8) = f4a4{ob[8], ob[9], ob[10], ob[11]};
      row[12] = ob[12];
      (o.rew + first)[lane] = rew;
      if (!(keep_flags && !rs)) {
        (o.reset + first)[lane] = rs ? 1 : 0;
        (o.timeouts + first)[lane] = to ? 1 : 0;
      }
    }
    return;
  }
  if (direct) {   // wave shared by two tasks (misaligned mixed shard): plain per-lane stores
    if (valid) {
#pragma unroll
      for (int k = 0; k < OUZ_NUM_OBS; ++k) o.obs[(size_t)i * OUZ_NUM_OBS + k] = ob[k];
      o.rew[i] = rew;
      o.reset[i] = rs ? 1 : 0;
      o.timeouts[i] = to ? 1 : 0;
    }
    return;
  }
  if (valid) {
#pragma unroll
    for (int k = 0; k < OUZ_NUM_OBS; ++k) wave_lds[lane * OUZ_NUM_OBS + k] = ob[k];
    OUZ_ST(&(o.rew + first)[lane], rew);
    // keep_flags: reset_buf and time_outs held 0 at the start of the step (read with the state); if
    // the env is still not done both buffers already hold this step's values: skip the 9-byte write
    // (a time-out left over from a manually cleared reset_buf is rewritten)
    if (!(keep_flags && !rs)) {
      OUZ_ST(&(o.reset + first)[lane], (int64_t)(rs ? 1 : 0));
      OUZ_ST(&(o.timeouts + first)[lane], (uint8_t)(to ? 1 : 0));
    }
  }
  wave_lds_sync();
  const uint32_t m = min(64u, (uint32_t)(n - (int)first));
  float* dst = o.obs + (size_t)first * OUZ_NUM_OBS;   // 16-B aligned: waves start at multiples of 64 envs
  const float4* src4 = reinterpret_cast<const float4*>(wave_lds);
  float4* dst4 = reinterpret_cast<float4*>(dst);
  if (m == 64) {   // full wave: 64 x 13 floats = 208 float4, 3.25 per lane
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v* d4 = reinterpret_cast<f4v*>(dst4);
    const f4v* s4 = reinterpret_cast<const f4v*>(src4);
#pragma unroll
    for (uint32_t r = 0; r < 3; ++r) OUZ_ST(&d4[lane + 64u * r], s4[lane + 64u * r]);
    if (lane < 16u) OUZ_ST(&d4[lane + 192u], s4[lane + 192u]);
  } else {
    const uint32_t nf = m * OUZ_NUM_OBS;
    for (uint32_t k = lane; k < nf / 4; k += 64) dst4[k] = src4[k];
    for (uint32_t k = (nf / 4) * 4 + lane; k < nf; k += 64) dst[k] = wave_lds[k];
  }
  wave_lds_sync();
}

// The output wave of a latency-regime rollout.  The step's observation, reward, episode
// statistics and output stores feed nothing the next step computes but the done flags, so a second wave of the
// tile forms them from the post-step state while the state wave runs the next step's chain.  The state wave
// publishes, per step, the post-step state (p, q, v, w, the target) with the progress counter and the done
// flags into a ring slot; the output wave reads it, runs obs_reward / the episode tracking / the stores, and
// releases the slot.  Waits: the state wave for a free slot (kOutRing steps ahead at most), the output wave for
// a published step; both run the same K steps (quad_pv_split.h's split_wait, the same give-up bound).  The
// slots are [field][lane] dwords, so the 16 values go out as 8 ds_write2st64_b32 straight from the registers
// they are in (a float4 row per lane needed a register quad per store, i.e. 16 moves per step), and the state
// wave re-reads the consumed count only when the count it last saw does not cover the slot it is about to reuse.
constexpr int kOutRing = 8;
constexpr int kOutFields = 16;   // p.xyz, q.xyzw, v.xyz, w.xyz, target.xyz
struct OutRingLds {
  float post[kOutRing][kOutFields][64];
  int32_t meta[kOutRing][64];     // progress << 4 | rst(step 0) << 3 | flags_clear(step 0) << 2 | time_out << 1 | reset
  int post_count;                 // steps published by the state wave
  int consumed;                   // steps read by the output wave
};

__device__ __forceinline__ void out_publish(OutRingLds& R, int k, int& seen, V3 p, Q4 q, V3 v, V3 w, V3 target,
                                            int32_t progress, bool rs, bool to, bool fc0, bool rst0) {
  if (k >= kOutRing && seen < k - kOutRing + 1) seen = split_wait(&R.consumed, k - kOutRing + 1);
  const int slot = k % kOutRing;
  const uint32_t lane = threadIdx.x & 63u;
  const float f[kOutFields] = {p.x, p.y, p.z, q.x, q.y, q.z, q.w, v.x, v.y, v.z, w.x, w.y, w.z,
                               target.x, target.y, target.z};
#pragma unroll
  for (int j = 0; j < kOutFields; ++j) R.post[slot][j][lane] = f[j];
  R.meta[slot][lane] = (progress << 4) | (rst0 ? 8 : 0) | (fc0 ? 4 : 0) | (to ? 2 : 0) | (rs ? 1 : 0);
  split_publish(&R.post_count, k + 1);
}

__device__ __forceinline__ void trace_count(const StepArgs& a, uint32_t step, bool did_reset, int slot, int e) {
  if (a.trace_cap <= 0) return;
  const uint64_t m = __ballot(did_reset);
  if ((threadIdx.x & 63u) == 0u && m) atomicAdd(&a.trace_resets[step % (uint32_t)a.trace_cap], (uint32_t)__popcll(m));
  if (e == 0) a.trace_resets[(step + 32u) % (uint32_t)a.trace_cap] = 0u;
}

// K steps of one env: load once, K x (step + emit), store once.  MULTI = false is the single
// VecTask.step kernel (K = 1, no loop, no rollout storage) and keeps the register budget of one step.
// Episode statistics of one lane, reduced over the grid by the fused rollout (RolloutStats).
struct LaneStats {
  double sum, cnt, len;
};

// i: state slot (its wave tile is wave-uniform); e: env index (== i except under the trigger-class layout,
// CLS), which keys the RNG and indexes the env-order buffers.
// QLN: the quad-lane estimator (quad_pv_ql.h, latency-regime estimator kernels): the four lanes of a quad step
// the same env (same slot i and env e) and split its PV covariance step; every other part of the step runs
// identically in all four, and lane 0 of the quad alone writes the env's outputs, statistics and state
// (the lanes 0-2 write the covariance elements they own).
// SPW: the state wave of the split-wave estimator rollout (quad_pv_split.h; MULTI only): the covariance is
// stepped by the workgroup's other wave (cov_wave), the two meet in `spl_lds`.
// OWV: the state wave of a rollout with an output wave (out_wave): the step's outputs, episode tracking and
// statistics are the output wave's; this wave publishes the post-step state into `orl` instead.
template <int CTRL, int TGT, bool MULTI, bool PRE = false, bool CLS = false, bool NTL = false, bool QLN = false,
          bool SPW = false, bool OWV = false>
__device__ __forceinline__ void run_env(const StepArgs& a, const StepCtx* ctx, int K, const OutPtrs* outs,
                                        size_t out_stride, float* wave_lds, int i, int e, bool valid, int task,
                                        bool direct = false, int stats_mode = 0, LaneStats* ls = nullptr,
                                        float* wrench = nullptr, SplitPvLds* spl_lds = nullptr,
                                        OutRingLds* orl = nullptr) {
  const TaskParams& tp = a.tp[tp_slot(task)];
  const uint32_t gid = a.env_offset + (uint32_t)e;
  // the env's outputs / statistics / state writes: every lane, or lane 0 of the quad
  const bool lead = QLN ? (threadIdx.x & 3u) == 0u : true;
  const bool vout = valid && lead;
  PvQl ql{};
  SplitLane spl{spl_lds, 0, threadIdx.x & 63u};
  static_assert(!SPW || (MULTI && !PRE && !QLN && CTRL == CTRL_LEE_EST), "the split form is the estimator rollout's");
  static_assert(!OWV || (MULTI && !PRE && !QLN), "the output wave is the rollout's");
  if constexpr (QLN) {
    static_assert(CTRL == CTRL_LEE_EST, "the quad-lane form is the estimator's");
    __shared__ double s_pv[16 * kPvLdsEnv];   // one 64-lane block = one wave = 16 envs
    const uint32_t sub = threadIdx.x & 3u;
    double* env_lds = s_pv + (threadIdx.x >> 2) * kPvLdsEnv;
    ql = PvQl{env_lds, env_lds + kPvLdsP, sub == 3u ? 0 : (int)sub, sub != 3u};
  }
  EnvRegs<CTRL, TGT> S;
  OUZ_STAMP_RT(8);
  OUZ_STAMP(0, false);
  S.T = tile_of(a, i);   // outside any divergent branch, so the base pointers stay scalar
  // fused statistics: the episode accumulators of earlier (unfused) steps, issued first so that they are in
  // flight with the state (issued after it, they were a second memory round trip of the prologue)
  float ep_sum_old = 0.0f;
  int32_t ep_cnt_old = 0, ep_len_old = 0;
  if (MULTI && !OWV && stats_mode && vout) {
    ep_sum_old = ld(S.T, OUZ_F_EP_SUM);
    ep_cnt_old = ldi(S.T, OUZ_I_EP_CNT);
    ep_len_old = ldi(S.T, OUZ_I_EP_LEN);
  }
  if (valid) env_load<CTRL, TGT, CLS, NTL, QLN || SPW>(a, e, tp, S, ctx[0].actions);
  if constexpr (QLN) {
    if (valid) pv_lds_load(ql, [&](int f) { return ld(S.T, OUZ_F_PV_P + f); });
    ql_sync();
  }
  OUZ_STAMP(1, true);
  if constexpr (PRE) {
    // pre_physics_step alone: lazy reset, controller / estimator / guidance, wrench; reset_idx clears
    // reset_buf (ekf_lee_landed.py:300-301); no integration, no outputs, the step counter stays
    float ob[OUZ_NUM_OBS];
    float rew = 0.0f;
    bool rs = false, to = false;
    const bool did_reset = vout && S.rst;
    if (valid) env_core<CTRL, TGT, true, QLN>(a, ctx[0], e, gid, task, S, ob, rew, rs, to, wrench, &ql);
    if (did_reset) a.reset[e] = 0;
  } else if constexpr (!MULTI) {
    float ob[OUZ_NUM_OBS];
    float rew = 0.0f;
    bool rs = false, to = false;
    const bool did_reset = vout && S.rst;
    const bool flags_clear = vout && S.flags_clear;
    if (valid) env_core<CTRL, TGT, false, QLN>(a, ctx[0], e, gid, task, S, ob, rew, rs, to, nullptr, &ql);
    trace_count(a, ctx[0].step, did_reset, i, e);
    OUZ_STAMP(5, false);
    if (CLS) emit_env(outs[1], e, vout, ob, rew, rs, to, flags_clear);
    else emit(outs[1], wave_lds, i, a.n, vout, ob, rew, rs, to, direct, flags_clear);
    OUZ_STAMP(6, false);
  } else {
    // Drain the state loads before the step loop.  vmcnt counts loads and stores in one in-order counter,
    // and the compiler's waits for the first use of each loaded register sat inside the loop body, where
    // from the second step on they waited for the previous step's output stores instead.  One wait here
    // (the loads were issued together: the first step pays that round trip anyway) leaves the loop with
    // waits only for its own loads.  Measured effect small: SQ_WAIT_ANY 477 -> 463 wave quad-cycles per
    // LeeLanded step at 4096 envs (profiles/r02/sq_*); the per-step time is VALU/SALU issue.
    __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    const bool fc0 = S.flags_clear, rst0 = S.rst;   // OWV: step 0's flag / reset state, for the output wave
    int out_seen = 0;                               // OWV: the output wave's consumed count last seen
    for (int k = 0; k < K; ++k) {
      if (kStampSlots > 13 && k <= 16) OUZ_STAMP(13 + k, false);
      float ob[OUZ_NUM_OBS];
      float rew = 0.0f;
      bool rs = false, to = false;
      const bool did_reset = vout && S.rst;
      // in the loop the buffers hold the previous step's flags: clear iff it was not done
      const bool flags_clear = vout && (k == 0 ? S.flags_clear : !did_reset);
      spl.k = k;
      V3 post_target = v3(0.0f, 0.0f, 0.0f);
      if (valid)
        env_core<CTRL, TGT, false, QLN, SPW, OWV>(a, ctx[k], e, gid, task, S, ob, rew, rs, to, nullptr, &ql, &spl,
                                                  &post_target);
      if (kStampSlots > 13 && k == 8) OUZ_STAMP(30, false);
      if (valid && k + 1 < K) load_actions<CTRL, TGT, CLS>(ctx[k + 1].actions, S, e);   // next step's row, before emit
      if constexpr (OWV) {   // (the reset counts of the trajectory log are the output wave's)
        out_publish(*orl, k, out_seen, S.p, S.q, S.v, S.w, post_target, S.progress, rs, to, fc0, rst0);
          if (kStampSlots > 13 && k == 8) OUZ_STAMP(31, false);
        continue;
      }
      trace_count(a, ctx[k].step, did_reset, i, e);
      OutPtrs o = outs[0];
      if (out_stride) {   // rollout storage: step k of (K, N, ...) buffers; the env buffers get the last step
        o.obs += (size_t)k * out_stride * OUZ_NUM_OBS;
        o.rew += (size_t)k * out_stride;
        o.reset += (size_t)k * out_stride;
        o.timeouts += (size_t)k * out_stride;
        if (CLS) {
          emit_env(o, e, vout, ob, rew, rs, to, false);
          if (k == K - 1) emit_env(outs[1], e, vout, ob, rew, rs, to, false);
        } else {
          emit(o, wave_lds, i, a.n, vout, ob, rew, rs, to, direct);
          if (k == K - 1) emit(outs[1], wave_lds, i, a.n, vout, ob, rew, rs, to, direct);
        }
      } else if (CLS) {
        emit_env(o, e, vout, ob, rew, rs, to, flags_clear);
      } else {
        emit(o, wave_lds, i, a.n, vout, ob, rew, rs, to, direct, flags_clear);
      }
      if (kStampSlots > 13 && k == 8) OUZ_STAMP(31, false);
    }
    if (kStampSlots > 13 && K <= 16) OUZ_STAMP(13 + K, false);
    if (!OWV && stats_mode && vout) {
      // RecordEpisodeStatisticsTorch over the rollout (PPO/utils.py:20-35) without a separate launch: this
      // lane's totals (accumulated before + finished in these K steps, same f32 adds as the atomics of
      // env_store) go to the grid reduction; drained accumulators are zeroed, kept ones written back.
      const float s_tot = ep_sum_old + S.ep_sum_add;
      const int32_t c_tot = ep_cnt_old + S.ep_cnt_add, l_tot = ep_len_old + S.ep_len_add;
      ls->sum += (double)s_tot;
      ls->cnt += (double)c_tot;
      ls->len += (double)l_tot;
      if (stats_mode == 2) {
        if (ep_cnt_old) {
          st(S.T, OUZ_F_EP_SUM, 0.0f);
          sti(S.T, OUZ_I_EP_CNT, 0);
          sti(S.T, OUZ_I_EP_LEN, 0);
        }
      } else if (S.ep_cnt_add) {
        st(S.T, OUZ_F_EP_SUM, s_tot);
        sti(S.T, OUZ_I_EP_CNT, c_tot);
        sti(S.T, OUZ_I_EP_LEN, l_tot);
      }
      S.ep_cnt_add = 0;   // env_store: no accumulator atomics
    }
  }
  if (vout) env_store<CTRL, TGT, QLN || SPW, !OWV>(a, i, tp, S);
  if constexpr (QLN) {
    if (valid) pv_lds_store(ql, [&](int f, float v) { st(S.T, OUZ_F_PV_P + f, v); });
  }
  OUZ_STAMP(7, true);
  OUZ_STAMP_RT(9);
}

// The output wave of a rollout (see OutRingLds): per step, the observation, reward, episode tracking and output
// stores of run_env's one-wave loop, from the state wave's published post-step state; at the end the episode
// fields and the fused statistics.  Same functions (obs_reward, emit / emit_env) on the same values: the
// outputs are bitwise those of the one-wave rollout.
template <bool CLS>
__device__ __forceinline__ void out_wave(const StepArgs& a, const StepCtx* ctx, int K, const OutPtrs* outs,
                                         size_t out_stride, float* wave_lds, int i, int e, bool valid, int task,
                                         int stats_mode, LaneStats* ls, OutRingLds& R) {
  const TaskParams& tp = a.tp[tp_slot(task)];
  const uint32_t gid = a.env_offset + (uint32_t)e, lane = threadIdx.x & 63u;
  const Tile T = tile_of(a, i);
  const bool vout = valid;
  float ep_sum_old = 0.0f, ep_ret = 0.0f, ep_sum_add = 0.0f;
  int32_t ep_cnt_old = 0, ep_len_old = 0, ep_cnt_add = 0, ep_len_add = 0;
  if (stats_mode && vout) {
    ep_sum_old = ld(T, OUZ_F_EP_SUM);
    ep_cnt_old = ldi(T, OUZ_I_EP_CNT);
    ep_len_old = ldi(T, OUZ_I_EP_LEN);
  }
  if (valid && a.track_episodes) ep_ret = ld(T, OUZ_F_EP_RET);
  bool prev_rs = false;
  for (int k = 0; k < K; ++k) {
    if (kStampSlots > 13 && k <= 16) OUZ_STAMP(13 + k, false);
    split_wait(&R.post_count, k + 1);
    if (kStampSlots > 13 && k == 8) OUZ_STAMP(30, false);
    const int slot = k % kOutRing;
    float f[kOutFields];
#pragma unroll
    for (int j = 0; j < kOutFields; ++j) f[j] = R.post[slot][j][lane];
    const int32_t meta = R.meta[slot][lane];
    split_publish(&R.consumed, k + 1);   // the values are in registers: the slot is free
    const V3 p = v3(f[0], f[1], f[2]), v = v3(f[7], f[8], f[9]), w = v3(f[10], f[11], f[12]),
             target = v3(f[13], f[14], f[15]);
    const Q4 q = Q4{f[3], f[4], f[5], f[6]};
    const int32_t progress = meta >> 4;
    const bool rs = (meta & 1) != 0, to = (meta & 2) != 0;
    // run_env's trajectory-log reset count: the step's resets are the envs its previous step ended (step 0:
    // the buffers' own flags)
    trace_count(a, ctx[k].step, vout && (k == 0 ? (meta & 8) != 0 : prev_rs), i, e);
    // run_env's flag state: at step 0 the buffers' own, later "not reset by the previous step"
    const bool flags_clear = vout && (k == 0 ? (meta & 4) != 0 : !prev_rs);
    float ob[OUZ_NUM_OBS];
    float rew = 0.0f;
    if (valid) {
      if (a.trace_cap > 0 && e == a.trace_env) {   // env_core's trajectory CSV row (ekf_lee_landed.py:667-674)
        float* t = a.trace + (size_t)(ctx[k].step % (uint32_t)a.trace_cap) * 9;
        t[0] = p.x; t[1] = p.y; t[2] = p.z;
        t[3] = target.x; t[4] = target.y; t[5] = target.z;
        t[6] = v.x; t[7] = v.y; t[8] = v.z;
      }
      float dist;
      obs_reward(a, ctx[k], tp, task, gid, p, q, v, w, target, ob, rew, dist);
      if (a.track_episodes) {   // RecordEpisodeStatisticsTorch.step (PPO/utils.py:20-35), as env_core
        ep_ret += rew;
        if (rs) { ep_sum_add += ep_ret; ep_cnt_add += 1; ep_len_add += progress; ep_ret = 0.0f; }
      }
    }
    prev_rs = rs;
    OutPtrs o = outs[0];
    if (out_stride) {   // rollout storage: step k of (K, N, ...) buffers; the env buffers get the last step
      o.obs += (size_t)k * out_stride * OUZ_NUM_OBS;
      o.rew += (size_t)k * out_stride;
      o.reset += (size_t)k * out_stride;
      o.timeouts += (size_t)k * out_stride;
      if (CLS) {
        emit_env(o, e, vout, ob, rew, rs, to, false);
        if (k == K - 1) emit_env(outs[1], e, vout, ob, rew, rs, to, false);
      } else {
        emit(o, wave_lds, i, a.n, vout, ob, rew, rs, to, false);
        if (k == K - 1) emit(outs[1], wave_lds, i, a.n, vout, ob, rew, rs, to, false);
      }
    } else if (CLS) {
      emit_env(o, e, vout, ob, rew, rs, to, flags_clear);
    } else {
      emit(o, wave_lds, i, a.n, vout, ob, rew, rs, to, false, flags_clear);
    }
    if (kStampSlots > 13 && k == 8) OUZ_STAMP(31, false);
  }
  if (kStampSlots > 13 && K <= 16) OUZ_STAMP(13 + K, false);
  if (stats_mode && vout) {   // run_env's fused statistics
    const float s_tot = ep_sum_old + ep_sum_add;
    const int32_t c_tot = ep_cnt_old + ep_cnt_add, l_tot = ep_len_old + ep_len_add;
    ls->sum += (double)s_tot;
    ls->cnt += (double)c_tot;
    ls->len += (double)l_tot;
    if (stats_mode == 2) {
      if (ep_cnt_old) {
        st(T, OUZ_F_EP_SUM, 0.0f);
        sti(T, OUZ_I_EP_CNT, 0);
        sti(T, OUZ_I_EP_LEN, 0);
      }
    } else if (ep_cnt_add) {
      st(T, OUZ_F_EP_SUM, s_tot);
      sti(T, OUZ_I_EP_CNT, c_tot);
      sti(T, OUZ_I_EP_LEN, l_tot);
    }
    ep_cnt_add = 0;
  }
  if (vout && a.track_episodes) {   // env_store's episode fields
    st(T, OUZ_F_EP_RET, ep_ret);
    if (ep_cnt_add) {
      atomicAdd(&T.f[(uint32_t)OUZ_F_EP_SUM * 64u + T.l], ep_sum_add);
      atomicAdd(&T.iv[(uint32_t)OUZ_I_EP_CNT * 64u + T.l], ep_cnt_add);
      atomicAdd(&T.iv[(uint32_t)OUZ_I_EP_LEN * 64u + T.l], ep_len_add);
    }
  }
}

constexpr int kMaxRolloutChunk = 32;
constexpr bool kSplitDefault = true;    // the split-wave estimator rollout is the default
constexpr bool kOutWaveDefault = true;  // the output wave in the latency-regime rollouts
constexpr int kOutWaveMaxSlots = 16384;
static_assert(kSplitRing >= kMaxRolloutChunk, "one attitude slot per step of a launch");

// The covariance wave of the split-wave estimator rollout (quad_pv_split.h): the PV covariance of the tile's 64
// envs through the K steps of the launch, loaded and stored once, stepped as the state wave publishes attitudes.
__device__ __forceinline__ void cov_wave(const StepArgs& a, const StepCtx* ctx, int K, int i, int e, bool valid,
                                         SplitPvLds& L) {
  if (!__any(valid)) return;   // the state wave steps no env of this tile either
  const Tile T = tile_of(a, i);
  const uint32_t lane = threadIdx.x & 63u, gid = a.env_offset + (uint32_t)e;
  float pf[45];
#pragma unroll
  for (int f = 0; f < 45; ++f) pf[f] = valid ? ld(T, OUZ_F_PV_P + f) : 0.0f;
  for (int k = 0; k < K; ++k) {
    // the fix decisions of env_core's PV step (g % 7 == 6 position, g % 3 == 0 velocity), for the lanes the
    // state wave steps
    const uint64_t g = (uint64_t)ctx[k].step * a.n_total + gid;
    if (kStampSlots > 13 && k <= 16) OUZ_STAMP(13 + k, false);
    pv_cov_split(L, k, lane, pf, a.c.dt, valid && g % 7u == 6u, valid && g % 3u == 0u);
  }
  if (kStampSlots > 13 && K <= 16) OUZ_STAMP(13 + K, false);
  if (valid) {
#pragma unroll
    for (int f = 0; f < 45; ++f) st(T, OUZ_F_PV_P + f, pf[f]);
  }
}

// Episode statistics fused into the last launch of a rollout (ouz_rollout_stats): each wave reduces its
// lanes' totals into partials[wave]; the last wave to finish (device-scope ticket) adds the partials in
// wave order, so the triple is deterministic.  mode 0: off, 1: report, 2: report and drain.
struct RolloutStats {
  double* out;
  double* partials;         // [tiles][3]
  uint32_t* ticket;         // returns to 0 after every launch
  int32_t mode;
};

struct RolloutArgs {
  int32_t K;
  OutPtrs outs[2];          // [0] per-step target (env buffers or rollout storage), [1] env buffers
  uint64_t out_stride;      // 0: write every step to outs[0]; else rollout storage with this env stride
  RolloutStats stats;
  StepCtx ctx[kMaxRolloutChunk];
};

// Launch block size, a function of n only (the host launches with the same rule): the kernel
// derives it from a.n instead of reading blockDim from the hidden kernel arguments, whose cache
// line would be one more scalar-memory miss at entry.
__host__ __device__ __forceinline__ int step_block_for(int n) { return n <= kLatencyRegimeEnvs ? 64 : 256; }

// Kernel-argument prefetch.  The step kernel reads its ~1 KB argument block through scalar loads
// that the compiler issues in several dependent batches (each waits for the previous: SGPR reuse,
// branches on loaded values), and in the latency regime every batch is a scalar-cache miss on a
// freshly written argument buffer.  One dword per 64-byte line, all issued together and waited for
// once, turns those serial misses into one; the later field loads hit the scalar cache.
// (All sixteen dwords are operands of one asm statement, so the compiler must have issued every
// load before it and waits once; folding them into one value let it wait after every eight.)
template <int NBYTES>
__device__ __forceinline__ void prefetch_kernargs() {
  const __attribute__((address_space(4))) uint32_t* kp =
      (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
  constexpr int kLines = (NBYTES + 63) / 64 < 16 ? (NBYTES + 63) / 64 : 16;
  uint32_t t[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = kp[(k < kLines ? k : kLines - 1) * 16];
  __asm__ volatile("" ::"s"(t[0]), "s"(t[1]), "s"(t[2]), "s"(t[3]), "s"(t[4]), "s"(t[5]), "s"(t[6]), "s"(t[7]),
                   "s"(t[8]), "s"(t[9]), "s"(t[10]), "s"(t[11]), "s"(t[12]), "s"(t[13]), "s"(t[14]), "s"(t[15]));
}

// The step kernel body: one env per lane, K steps (MULTI) or one.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Grid reduction of the lanes' episode statistics (see RolloutStats).  Called once by each of the nw live waves
// (w = its index in 0..nw-1, the partials' fixed summation order).  The last wave to add to the ticket sums the
// partials.  The hand-off is the write-through form of MI355X_MICROARCH.md "Valid forms" (first row): each wave's
// lane 0 stores its partials sc1 (write-through past the XCD's L2), drains them, then makes its agent-scope add;
// the last adder reads every partial with sc1 loads once its add has returned.  No __threadfence(): its L2
// writeback + invalidate (≈3.5 µs, the guide's price list) sat at the end of every fused rollout launch (16-step
// LeeLanded launch 26.8 -> 23.6 µs without the statistics: profiles/r04/stats_tail.jsonl).
__device__ __forceinline__ void reduce_stats(const RolloutStats& rs, uint32_t w, uint32_t nw, const LaneStats& ls) {
  const uint32_t lane = threadIdx.x & 63u;
  const double s = wave_sum(ls.sum), c = wave_sum(ls.cnt), l = wave_sum(ls.len);
  uint32_t last = 0;
  if (lane == 0u) {
    double* p = rs.partials + w * 3u;
    __hip_atomic_store(p + 0, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 2, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(rs.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nw - 1u ? 1u : 0u;
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  // ISA assumption this hand-off rests on (not the HIP/C++ memory model): gfx950 relaxed agent-scope atomic
  // stores are `global_store ... sc1` (write-through past this XCD's L2 to memory), the s_waitcnt vmcnt(0) above
  // retires them before the ticket add issues, and relaxed agent-scope atomic loads are `global_load ... sc1`
  // (they miss every non-coherent cache), so the last adder reads the memory the other waves' partials reached.
  // MI355X_MICROARCH.md "Valid forms", first row.  tests/test_gpu_timed_kernels.py checks the fused statistics
  // against ouz_episode_stats at 70 053 envs.  -DOUZ_STATS_ACQUIRE adds the agent-scope acquire the memory model
  // would ask for (an A/B build: DESIGN.md §5.1 prices it).
#ifdef OUZ_STATS_ACQUIRE
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
  double t[3] = {0.0, 0.0, 0.0};
  for (uint32_t j = lane; j < nw; j += 64u) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
      t[k] += __hip_atomic_load(&rs.partials[j * 3u + (uint32_t)k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = wave_sum(t[k]);
  if (lane == 0u) {
    rs.out[0] = t[0];
    rs.out[1] = t[1];
    rs.out[2] = t[2];
    *rs.ticket = 0u;   // ready for the next launch (visible to it after this kernel's end-of-kernel release)
  }
}

// XCD-packed class blocks (StepArgs.xcd_pack; the trigger-class layout above the latency regime): workgroup x runs
// on XCD x % 8 (the dispatcher deals workgroups round-robin over the XCDs), and the waves of XCD c take the tiles of
// class blocks c, c + 8, c + 16, ... in order, so the 21 waves of a block -- whose env-order outputs, 21 envs
// apart per lane, share partial lines -- run on one XCD at about the same time and their plain stores meet in
// that XCD's L2 instead of reaching memory as partial writes from eight L2s.  Returns this wave's tile, or -1
// past the last block (the grid is rounded up to whole blocks per XCD).
__device__ __forceinline__ int xcd_tile(int waves_per_wg, int n_blocks) {
  const uint32_t x = blockIdx.x, xcd = x & 7u;
  const uint32_t p = (x >> 3) * (uint32_t)waves_per_wg + (threadIdx.x >> 6);
  const uint32_t b = xcd + 8u * (p / (uint32_t)kTrigClasses);
  if (b >= (uint32_t)n_blocks) return -1;
  return (int)__builtin_amdgcn_readfirstlane(b * (uint32_t)kTrigClasses + p % (uint32_t)kTrigClasses);
}

// The quad-lane estimator (quad_pv_ql.h) runs the trigger-class layout of the estimator tasks and the
// QuadTracking chunks of the mixed curriculum's class layout: 64-lane blocks (the latency regime), four per
// 64-slot tile, each wave stepping 16 envs with 4 lanes each (quad_grid_blocks on the host).
__host__ __device__ constexpr bool quad_lane_kernel(int task, bool cls) {
  return cls && (task == OUZ_TASK_EKF_LEE_LANDED || task == OUZ_TASK_TRACKING || task == OUZ_TASK_MIXED);
}

// The mixed curriculum above the latency regime, one launch per task (StepArgs.mix_split; MIXT kernels): a task's
// launch steps only the 64-env tiles of its 1344-id chunks (chunk c runs task mixed_chunk_task(c), c % 3), with that
// task's own kernel and register budget, instead of every wave carrying the estimator's (228 VGPRs: two waves per
// SIMD for the LeeLanded / QuadFault chunks too).  Wave k of the launch of task TASK takes shard tile
// mixed_task_tile(a, TASK, k), or -1 past the shard; the shard starts on a 64-env tile (env_offset % 64 == 0, checked
// on the host), so every tile lies in one chunk.  Same per-env code as the one-launch kernel: bitwise its results.
__device__ __forceinline__ int mixed_task_tile(const StepArgs& a, int task, int k) {
  const uint32_t r = task == OUZ_TASK_LEE_LANDED ? 0u : (task == OUZ_TASK_TRACKING ? 1u : 2u);
  const uint32_t g0 = a.env_offset / 64u, cf = g0 / (uint32_t)kTrigClasses;   // shard's first tile, its chunk
  const uint32_t d = (r + 3u - cf % 3u) % 3u;                                   // first chunk of this task: cf + d
  const uint32_t uk = (uint32_t)k, per = (uint32_t)kTrigClasses;
  const int64_t t = (int64_t)((cf + d + 3u * (uk / per)) * per + uk % per) - (int64_t)g0;
  return (t >= 0 && t < (int64_t)((a.n + 63) / 64)) ? (int)t : -1;
}

template <int TASK, bool MULTI, bool PRE = false, bool CLS = false, bool NTL = false, bool QUAD = false,
          bool SPW = false, bool OWV = false, bool MIXT = false>
__device__ __forceinline__ void step_body(const StepArgs& a, const StepCtx* ctx, int K, const OutPtrs* outs,
                                          uint64_t out_stride, const RolloutStats* rst = nullptr,
                                          float* wrench = nullptr) {
  __shared__ float4 s_obs4[kMaxBlock * OUZ_NUM_OBS / 4];
  float* wave_lds = reinterpret_cast<float*>(s_obs4) + (threadIdx.x & ~63) * OUZ_NUM_OBS;
  const int sm = (MULTI && rst) ? rst->mode : 0;
  LaneStats ls{0.0, 0.0, 0.0};
  if constexpr (SPW || OWV) {
    // Multi-wave rollouts, one workgroup per 64-slot tile: wave 0 steps the tile's envs; with SPW (the
    // estimator's trigger-class layout, quad_pv_split.h) wave 1 steps their PV covariance; with OWV the last
    // wave forms the outputs (out_wave).
    static_assert(MULTI && !PRE && !QUAD, "the multi-wave forms are the rollout's");
    static_assert(!SPW || quad_lane_kernel(TASK, CLS), "the split form is the estimator's class layout");
    SplitPvLds* spl = nullptr;
    OutRingLds* orl = nullptr;
    if constexpr (SPW) {
      __shared__ SplitPvLds s_split;
      spl = &s_split;
    }
    if constexpr (OWV) {
      __shared__ OutRingLds s_out;
      orl = &s_out;
    }
    if (threadIdx.x == 0) {
      if (spl) {
        spl->att_count = 0;
        spl->gain_step[0] = 0;
        spl->gain_step[1] = 0;
      }
      if (orl) {
        orl->post_count = 0;
        orl->consumed = 0;
      }
    }
    __syncthreads();
    const int tile = (int)blockIdx.x, i = tile * 64 + (int)(threadIdx.x & 63u), role = (int)(threadIdx.x >> 6);
    int e = i;
    int chunk_task = TASK;
    if constexpr (CLS && TASK == OUZ_TASK_MIXED) {
      const int64_t e64 = mixed_slot_env(a.env_offset, i);
      e = (e64 >= 0 && e64 < a.n) ? (int)e64 : a.n;
      chunk_task = mixed_chunk_task(a.env_offset / kClassBlock + (uint32_t)(tile * 64) / kClassBlock);
    } else if constexpr (CLS) {
      e = slot_env(i);
    }
    const bool valid = e < a.n;
    const int run_task = TASK == OUZ_TASK_MIXED ? chunk_task : TASK;
    constexpr int kOutRole = SPW ? 2 : 1;
    if (role == 0) {
      if constexpr (TASK == OUZ_TASK_OUZELUM || TASK == OUZ_TASK_FAULT)
        run_env<CTRL_RL, TGT_GOAL, true, false, CLS, false, false, false, OWV>(
            a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, nullptr, nullptr, orl);
      else if constexpr (TASK == OUZ_TASK_LEE_LANDED)
        run_env<CTRL_LEE_TRUE, TGT_PLATFORM, true, false, CLS, false, false, false, OWV>(
            a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, nullptr, nullptr, orl);
      else if constexpr (TASK == OUZ_TASK_LANDING)
        run_env<CTRL_RL, TGT_TRAJ, true, false, CLS, false, false, false, OWV>(
            a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, nullptr, nullptr, orl);
      else if constexpr (TASK == OUZ_TASK_EKF_LEE_LANDED)
        run_env<CTRL_LEE_EST, TGT_PLATFORM, true, false, CLS, false, false, SPW, OWV>(
            a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, nullptr, spl, orl);
      else if constexpr (TASK == OUZ_TASK_TRACKING)
        run_env<CTRL_LEE_EST, TGT_TRAJ, true, false, CLS, false, false, SPW, OWV>(
            a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, nullptr, spl, orl);
      else if constexpr (TASK == OUZ_TASK_MIXED && CLS) {
        if (chunk_task == OUZ_TASK_TRACKING)
          run_env<CTRL_LEE_EST, TGT_TRAJ, true, false, true, false, false, SPW, OWV>(
              a, ctx, K, outs, out_stride, wave_lds, i, e, valid, OUZ_TASK_TRACKING, false, sm, &ls, nullptr, spl, orl);
        else if (chunk_task == OUZ_TASK_LEE_LANDED)
          run_env<CTRL_LEE_TRUE, TGT_PLATFORM, true, false, true, false, false, false, OWV>(
              a, ctx, K, outs, out_stride, wave_lds, i, e, valid, OUZ_TASK_LEE_LANDED, false, sm, &ls, nullptr, nullptr,
              orl);
        else
          run_env<CTRL_RL, TGT_GOAL, true, false, true, false, false, false, OWV>(
              a, ctx, K, outs, out_stride, wave_lds, i, e, valid, OUZ_TASK_FAULT, false, sm, &ls, nullptr, nullptr, orl);
      }
      if (!OWV && sm) reduce_stats(*rst, blockIdx.x, gridDim.x, ls);   // the state waves of the exact grid
    } else if (SPW && role == 1) {
      if (run_task == OUZ_TASK_TRACKING || run_task == OUZ_TASK_EKF_LEE_LANDED)
        cov_wave(a, ctx, K, i, e, valid, *spl);
    } else if (OWV && role == kOutRole) {
      out_wave<CLS>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, run_task, sm, &ls, *orl);
      if (sm) reduce_stats(*rst, blockIdx.x, gridDim.x, ls);   // the output waves of the exact grid
    }
    return;
  }
  if constexpr (QUAD && quad_lane_kernel(TASK, CLS)) {
    // 64-lane blocks, four per tile: quarter q of tile t holds slots t*64 + q*16 .. +15, four lanes per slot
    const int tile = (int)(blockIdx.x >> 2), quarter = (int)(blockIdx.x & 3u);
    const int iq = tile * 64 + quarter * 16 + (int)(threadIdx.x >> 2);   // this quad's slot
    bool quad = true;
    int i = iq;
    if constexpr (TASK == OUZ_TASK_MIXED) {
      // a tile lies in one 1344-id chunk (one task): the QuadTracking chunks run quad-lane, the other tasks
      // one lane per slot in the tile's first block (its other three exit at once)
      const uint32_t ch = a.env_offset / kClassBlock + (uint32_t)(tile * 64) / kClassBlock;
      quad = mixed_chunk_task(ch) == OUZ_TASK_TRACKING;
      if (!quad) i = tile * 64 + (int)threadIdx.x;
    }
    int e = a.n;
    if constexpr (TASK == OUZ_TASK_MIXED) {
      const int64_t e64 = mixed_slot_env(a.env_offset, i);
      e = (e64 >= 0 && e64 < a.n) ? (int)e64 : a.n;
    } else {
      e = slot_env(i);
    }
    const bool valid = e < a.n && (quad || quarter == 0);
    if (quad) {
      run_env<CTRL_LEE_EST, TASK == OUZ_TASK_EKF_LEE_LANDED ? TGT_PLATFORM : TGT_TRAJ, MULTI, PRE, true, false, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid,
                                      TASK == OUZ_TASK_MIXED ? OUZ_TASK_TRACKING : TASK, false, sm, &ls, wrench);
    } else if (quarter == 0) {
      if constexpr (TASK == OUZ_TASK_MIXED) {
        const uint32_t ch = a.env_offset / kClassBlock + (uint32_t)(tile * 64) / kClassBlock;
        if (mixed_chunk_task(ch) == OUZ_TASK_LEE_LANDED)
          run_env<CTRL_LEE_TRUE, TGT_PLATFORM, MULTI, PRE, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid,
                                                               OUZ_TASK_LEE_LANDED, false, sm, &ls, wrench);
        else
          run_env<CTRL_RL, TGT_GOAL, MULTI, PRE, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid,
                                                     OUZ_TASK_FAULT, false, sm, &ls, wrench);
      }
    }
    if (sm) reduce_stats(*rst, blockIdx.x, gridDim.x, ls);   // every wave of the exact grid takes part
    return;
  }
  int i = blockIdx.x * step_block_for(a.n) + threadIdx.x;   // state slot
  if constexpr (MIXT) {   // one task of the mixed curriculum: this wave's tile among that task's chunks
    static_assert(!CLS && TASK != OUZ_TASK_MIXED, "a task launch of the mixed curriculum's identity layout");
    const int t = (int)__builtin_amdgcn_readfirstlane(
        (uint32_t)mixed_task_tile(a, TASK, (int)(blockIdx.x * (step_block_for(a.n) / 64) + (threadIdx.x >> 6))));
    i = (t < 0 ? (a.n + 63) / 64 * 64 : t * 64) + (int)(threadIdx.x & 63u);
  }
  if constexpr (CLS) {
    if (a.xcd_pack) {   // class layout above the latency regime: this wave's tile on its XCD (xcd_tile)
      const int t = xcd_tile(step_block_for(a.n) / 64, a.n_slots / kClassBlock);
      i = (t < 0 ? a.n_slots : t * 64) + (int)(threadIdx.x & 63u);
    }
  }
  const int first = i - (int)(threadIdx.x & 63);
  if (first >= (CLS ? a.n_slots : a.n)) return;   // whole wave past the end
  int e = i;                                       // env index (a.n: an idle slot)
  if constexpr (CLS && TASK == OUZ_TASK_MIXED) {
    const int64_t e64 = mixed_slot_env(a.env_offset, i);
    e = (e64 >= 0 && e64 < a.n) ? (int)e64 : a.n;
  } else if constexpr (CLS) {
    e = slot_env(i);
  }
  const bool valid = e < a.n;
  if constexpr (TASK == OUZ_TASK_OUZELUM || TASK == OUZ_TASK_FAULT) {
    run_env<CTRL_RL, TGT_GOAL, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, wrench);
  } else if constexpr (TASK == OUZ_TASK_LEE_LANDED) {
    run_env<CTRL_LEE_TRUE, TGT_PLATFORM, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, wrench);
  } else if constexpr (TASK == OUZ_TASK_EKF_LEE_LANDED) {
    run_env<CTRL_LEE_EST, TGT_PLATFORM, MULTI, PRE, CLS, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, wrench);
  } else if constexpr (TASK == OUZ_TASK_LANDING) {
    run_env<CTRL_RL, TGT_TRAJ, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, wrench);
  } else if constexpr (TASK == OUZ_TASK_TRACKING) {
    run_env<CTRL_LEE_EST, TGT_TRAJ, MULTI, PRE, CLS, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, TASK, false, sm, &ls, wrench);
  } else if constexpr (CLS) {
    // mixed curriculum, class layout: a wave's slots lie in one 1344-id chunk, so its task is wave-uniform
    const uint32_t c = a.env_offset / kClassBlock + __builtin_amdgcn_readfirstlane((uint32_t)first) / kClassBlock;
    const int t = mixed_chunk_task(c);
    if (t == OUZ_TASK_LEE_LANDED)
      run_env<CTRL_LEE_TRUE, TGT_PLATFORM, MULTI, PRE, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid,
                                                           OUZ_TASK_LEE_LANDED, false, sm, &ls, wrench);
    else if (t == OUZ_TASK_TRACKING)
      run_env<CTRL_LEE_EST, TGT_TRAJ, MULTI, PRE, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid,
                                                      OUZ_TASK_TRACKING, false, sm, &ls, wrench);
    else
      run_env<CTRL_RL, TGT_GOAL, MULTI, PRE, true>(a, ctx, K, outs, out_stride, wave_lds, i, e, valid, OUZ_TASK_FAULT,
                                                 false, sm, &ls, wrench);
  } else {
    // Per-lane task; each task's lanes run in turn.  When the shard offset is a multiple of 64 the
    // curriculum's 64-env blocks coincide with waves and exactly one branch runs per wave.  Both
    // alignments execute the same code, so a sharded run stays bit-identical to the unsharded one.
    const int t = mixed_task(a.env_offset + (uint32_t)i);
    const bool direct = (a.env_offset & 63) != 0;   // a wave straddles two blocks: no LDS obs staging
    const bool vl = valid && t == OUZ_TASK_LEE_LANDED, vt = valid && t == OUZ_TASK_TRACKING;
    const bool vr = valid && !vl && !vt;
    if (__any(vl))
      run_env<CTRL_LEE_TRUE, TGT_PLATFORM, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, i, vl,
                                                  OUZ_TASK_LEE_LANDED, direct, sm, &ls, wrench);
    if (__any(vt))
      run_env<CTRL_LEE_EST, TGT_TRAJ, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, i, vt,
                                             OUZ_TASK_TRACKING, direct, sm, &ls, wrench);
    if (__any(vr))
      run_env<CTRL_RL, TGT_GOAL, MULTI, PRE, false, NTL>(a, ctx, K, outs, out_stride, wave_lds, i, i, vr, OUZ_TASK_FAULT,
                                        direct, sm, &ls, wrench);
  }
  if constexpr (!MIXT) {   // (a task launch of the split mixed curriculum never reduces statistics: rollout_impl)
    if (sm) reduce_stats(*rst, (uint32_t)first >> 6, (uint32_t)((CLS ? a.n_slots : a.n) + 63) >> 6, ls);
  }
}

// VecTask.step: one step, outputs into the env buffers.  Its arguments are StepArgs + one StepCtx
// (~390 B): the host copies the argument block on every launch (≈0.6 us more host time per launch
// for a 1.1 KB block, scripts/exp/launch_cost.hip), and at 4096 envs that host time is the bound.
template <int TASK, bool CLS = false, bool NTL = false, bool QUAD = false, bool MIXT = false>
__global__ void __launch_bounds__(kMaxBlock) quad_step_kernel(StepArgs a, StepCtx c) {
  prefetch_kernargs<(int)(sizeof(StepArgs) + sizeof(StepCtx) + 8)>();
  const OutPtrs env_out[2] = {OutPtrs{a.obs, a.rew, a.reset, a.timeouts}, OutPtrs{a.obs, a.rew, a.reset, a.timeouts}};
  step_body<TASK, false, false, CLS, NTL, QUAD, false, false, MIXT>(a, &c, 1, env_out, 0);
}

// ouz_pre_physics: pre_physics_step alone, the body wrench to `wrench` [n][6].
template <int TASK, bool CLS = false, bool QUAD = false>
__global__ void __launch_bounds__(kMaxBlock) quad_pre_kernel(StepArgs a, StepCtx c, float* wrench) {
  const OutPtrs env_out[2] = {OutPtrs{a.obs, a.rew, a.reset, a.timeouts}, OutPtrs{a.obs, a.rew, a.reset, a.timeouts}};
  step_body<TASK, false, true, CLS, false, QUAD>(a, &c, 1, env_out, 0, nullptr, wrench);
}

// ouz_rollout: K <= kMaxRolloutChunk steps in one launch, env state kept in registers.  SPW: the split-wave
// estimator form (quad_pv_split.h), 128-thread blocks.  WPE: waves per SIMD the register budget is cut for (1: no
// constraint).  The estimator tasks above the latency regime use WPE = 2 (rollout_wpe): unconstrained, their
// K-step state holds 256 VGPRs + ~80 AGPRs, one wave per SIMD, and the wave's dependent chain leaves the VALU
// idle a third of the time; at two waves per SIMD the compiler spills ~90 VGPRs to scratch (L1/L2-resident) and
// the rollout runs 10-12 % faster per step at 4 M envs (QuadTracking 410 -> 359 us, QuadMixed 380 -> 344:
// profiles/r04/wide_rollout_ab.txt).
template <int TASK, bool CLS = false, bool QUAD = false, bool SPW = false, bool OWV = false, int WPE = 1,
          bool MIXT = false>
__global__ void __launch_bounds__(kMaxBlock) __attribute__((amdgpu_waves_per_eu(WPE)))
quad_rollout_kernel(StepArgs a, RolloutArgs r) {
  prefetch_kernargs<(int)(sizeof(StepArgs) + sizeof(RolloutArgs) + 8)>();
  step_body<TASK, true, false, CLS, false, QUAD, SPW, OWV, MIXT>(a, r.ctx, r.K, r.outs, r.out_stride, &r.stats);
}
#ifndef OUZ_EST_ROLLOUT_WPE
#define OUZ_EST_ROLLOUT_WPE 2   // (A/B builds: -DOUZ_EST_ROLLOUT_WPE=3)
#endif
__host__ __device__ constexpr int rollout_wpe(int task, int n) {
  return class_layout_task(task) && n > kLatencyRegimeEnvs ? OUZ_EST_ROLLOUT_WPE : 1;
}

// Large-N VecTask.step with the next tile's state in flight during this tile's compute.  Each wave of a
// smaller grid walks tiles t, t + stride, ...; before computing tile t it issues the state loads of tile
// t + stride, so a wave keeps a load batch in flight while it computes instead of alternating load ->
// compute -> store (the QuadFault step kernel at 4 M envs spends 47 % of its wave-cycles parked on memory
// with 16 waves per CU: DESIGN.md §5).  Same per-env code as the VecTask.step path of run_env, so the
// results are bitwise those of quad_step_kernel.  Tasks without the estimator only (the EKF's state is
// 80 registers more: a second copy would cost the occupancy this buys).
constexpr size_t kCtxArgOffset = (sizeof(StepArgs) + alignof(StepCtx) - 1) / alignof(StepCtx) * alignof(StepCtx);

template <int CTRL, int TGT, bool NTL>
__device__ __forceinline__ void pipe_envs(const StepArgs& a, const StepCtx& c, const OutPtrs& o, float* wave_lds,
                                          int t, int tiles, int task) {
  const TaskParams& tp = a.tp[tp_slot(task)];
  const int lane = (int)(threadIdx.x & 63u);
  int i = t * 64 + lane;
  bool valid = i < a.n;
  EnvRegs<CTRL, TGT> S;
  S.T = tile_of(a, i);
  if (valid) env_load<CTRL, TGT, false, NTL>(a, i, tp, S, c.actions);
  for (;;) {
    // The argument blocks are re-read through laundered pointers every tile: otherwise the compiler
    // hoists the wave-uniform float arithmetic on them (VALU results, held in VGPRs) out of the loop,
    // ~80 registers that halved the occupancy.  The re-reads hit the scalar cache.
    // (The kernel's arguments are (StepArgs, StepCtx) in that order at the start of the kernarg segment.)
    const __attribute__((address_space(4))) char* kp =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    __asm__ volatile("" : "+s"(kp));
    const StepArgs& A = *(const StepArgs*)(const __attribute__((address_space(4))) StepArgs*)kp;
    const StepCtx& C = *(const StepCtx*)(const __attribute__((address_space(4))) StepCtx*)(kp + kCtxArgOffset);
    const TaskParams& TP = A.tp[tp_slot(task)];
    const int tn = t + A.pipe_stride;   // wave-uniform: the loop exit and the next tile's bases stay scalar
    const bool more = tn < tiles;
    const int in = tn * 64 + lane;
    const bool vn = more && in < A.n;
    EnvRegs<CTRL, TGT> N;
    N.T = tile_of(A, in);
    if (vn) env_load<CTRL, TGT, false, NTL>(A, in, TP, N, C.actions);
    float ob[OUZ_NUM_OBS];
    float rew = 0.0f;
    bool rs = false, to = false;
    const bool did_reset = valid && S.rst;
    const bool flags_clear = valid && S.flags_clear;
    if (valid) env_core<CTRL, TGT>(A, C, i, A.env_offset + (uint32_t)i, task, S, ob, rew, rs, to);
    trace_count(A, C.step, did_reset, i, i);
    emit(o, wave_lds, i, A.n, valid, ob, rew, rs, to, false, flags_clear);
    if (valid) env_store<CTRL, TGT>(A, i, TP, S);
    if (!more) break;
    S = N;
    t = tn;
    i = in;
    valid = vn;
  }
}

// Three waves per SIMD: unconstrained the loop takes 170 VGPRs (two waves); at four the allocator spills.
#define OUZ_PIPE_ATTR __attribute__((amdgpu_waves_per_eu(3, 3)))
__host__ __device__ constexpr bool pipe_task(int task) {
  return task == OUZ_TASK_OUZELUM || task == OUZ_TASK_FAULT || task == OUZ_TASK_LANDING;
}

// Non-temporal state loads in the step kernels above 2 M envs (LeeLanded: 4 M).  Below, part of the state
// is still MALL-resident from the previous step and plain loads keep it there; above, the loads only evict
// what the write stream needs.  Measured crossovers (profiles/r02/nt_loads_ab.txt, per-step kernel us
// plain -> non-temporal): QuadTracking 2 M 281 -> 301, 4 M 663 -> 581 / 671 -> 626; QuadMixed 1 M 97 -> 99,
// 2 M 196 -> 188, 4 M 376 -> 355; QuadFault 4 M 227 -> 223 / 239 -> 224; LeeLanded 4 M 124 -> 128 /
// 126 -> 140, 8 M 267 -> 244, 16 M 605 -> 566.
__host__ __device__ constexpr bool nt_loads_default(int task, int n) {
  return n > (task == OUZ_TASK_LEE_LANDED ? 4194304 : 2097152);
}

// Streamed ouz_rollout by default (see ouz_env::stream_rollout): the tasks without the estimator above
// 131 072 envs.  The estimator tasks keep the fused kernel at every size: their state (~600 B per env-step
// of step-kernel traffic) is what the register-resident rollout saves, and it stays faster
// (QuadTracking 4 M: 404 fused against 663 us per step streamed; LeeLanded 4 M: 262 against 147;
// profiles/r02/stream_rollout_ab.jsonl).
__host__ __device__ constexpr bool stream_rollout_default(int task, int n) {
  return n > 2 * kLatencyRegimeEnvs && task != OUZ_TASK_EKF_LEE_LANDED && task != OUZ_TASK_TRACKING &&
         task != OUZ_TASK_MIXED;
}

template <int TASK, bool NTL = false>
__global__ void __launch_bounds__(kMaxBlock) OUZ_PIPE_ATTR quad_step_pipe_kernel(StepArgs a, StepCtx c) {
  prefetch_kernargs<(int)(sizeof(StepArgs) + sizeof(StepCtx) + 8)>();
  __shared__ float4 s_obs4[kMaxBlock * OUZ_NUM_OBS / 4];
  float* wave_lds = reinterpret_cast<float*>(s_obs4) + (threadIdx.x & ~63) * OUZ_NUM_OBS;
  const OutPtrs o{a.obs, a.rew, a.reset, a.timeouts};
  const int t = (int)__builtin_amdgcn_readfirstlane(blockIdx.x * (kMaxBlock / 64) + (threadIdx.x >> 6));
  const int tiles = (a.n + 63) >> 6;
  if (t >= tiles) return;
  if constexpr (TASK == OUZ_TASK_LANDING) pipe_envs<CTRL_RL, TGT_TRAJ, NTL>(a, c, o, wave_lds, t, tiles, TASK);
  else if constexpr (pipe_task(TASK)) pipe_envs<CTRL_RL, TGT_GOAL, NTL>(a, c, o, wave_lds, t, tiles, TASK);
}

// Creation-time state (VecTask.allocate_buffers vec_task.py:254-277 + task __init__).
__global__ void init_state_kernel(StepArgs a, int task_cfg) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;   // state slot
  if (s >= a.n_slots) return;
  for (int k = 0; k < OUZ_F_COUNT; ++k) st(a, k, s, 0.0f);
  for (int k = 0; k < OUZ_I_COUNT; ++k) sti(a, k, s, 0);
  // env index (padding / idle slots stay zero)
  const int64_t e = a.cls == 2 ? mixed_slot_env(a.env_offset, s) : (a.cls ? slot_env(s) : s);
  if (e < 0 || e >= a.n) return;
  const uint32_t gid = a.env_offset + (uint32_t)e;
  const int task = task_cfg == OUZ_TASK_MIXED ? mixed_task(gid) : task_cfg;
  const TaskParams& tp = a.tp[tp_slot(task)];
  const int i = s;
  st(a, OUZ_F_P + 2, i, 1.0f);           // default_pose.p.z = 1 (ekf_lee_landed.py:228-229)
  st(a, OUZ_F_Q + 3, i, 1.0f);
  st(a, OUZ_F_TARGET + 2, i, tp.target_mode == TGT_GOAL ? 1.0f : 0.377f);   // ouzelum.py:73, ekf_lee_landed.py:87
  st(a, OUZ_F_EKF_P + s4(0, 0), i, 1.0f); st(a, OUZ_F_EKF_P + s4(1, 1), i, 1.0f);   // ahrs_ekf.py:997
  st(a, OUZ_F_EKF_P + s4(2, 2), i, 1.0f); st(a, OUZ_F_EKF_P + s4(3, 3), i, 1.0f);
  for (int k = 0; k < 9; ++k) st(a, OUZ_F_PV_P + s9(k, k), i, kPvP0);        // PVFilter.py:12
  st(a, OUZ_F_DR, i, 1.0f); st(a, OUZ_F_DR + 1, i, 1.0f); st(a, OUZ_F_DR + 2, i, 1.0f);
  sti(a, OUZ_I_RAND_STEP, i, -1);        // never randomized: the first reset is due (vec_task.py:555-557)
  st(a, OUZ_F_FAULT_ETA, i, 1.0f);
  if (tp.target_mode == TGT_TRAJ) {      // landing.py:209-213
    U4 r = draw(a.seed, gid, INIT_STEP, RNG_TRAJ);
    sti(a, OUZ_I_TRAJ_TYPE, i, (int)(r.x % 3u));
    st(a, OUZ_F_TRAJ_SD, i, (r.z & 1u) ? uniform_f32(r.y, 0.8f, 1.2f) : -uniform_f32(r.y, 0.8f, 1.2f));
  }
  for (int k = 0; k < OUZ_NUM_OBS; ++k) a.obs[(size_t)e * OUZ_NUM_OBS + k] = 0.0f;
  a.rew[e] = 0.0f;
  a.reset[e] = 1;                        // reset_buf starts at ones (vec_task.py:269-270)
  a.timeouts[e] = 0;
}

// ouz_env_split_timeouts: the device's split-wave give-up count, read (and zeroed) in one atomic.
__global__ void split_timeouts_read_kernel(uint32_t* out, int reset) {
  *out = reset ? atomicExch(&g_ouz_split_timeouts, 0u) : atomicAdd(&g_ouz_split_timeouts, 0u);
}

__global__ void mark_reset_kernel(int64_t* reset, const int32_t* ids, int32_t n, int32_t n_envs) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) {
    int32_t e = ids[k];
    if (e >= 0 && e < n_envs) reset[e] = 1;
  }
}
__global__ void mark_all_kernel(int64_t* reset, int32_t n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) reset[k] = 1;
}

// Episode statistics in one launch (RecordEpisodeStatisticsTorch, PPO/utils.py:20-35): [sum of
// finished-episode returns, count] over all envs, optionally drained.  Each block reduces a fixed
// grid-stride slice into partials[block]; the last block to finish (ticket counter) adds the
// partials in block order, so the result is deterministic run to run.
constexpr int kStatsBlock = 256;
constexpr int kStatsMaxBlocks = 256;


__global__ void __launch_bounds__(kStatsBlock) episode_stats_kernel(StepArgs a, double* partials, uint32_t* ticket,
                                                                    double* out, int drain) {
  __shared__ double s_part[3][kStatsBlock / 64];
  __shared__ bool s_last;
  double acc[3] = {0.0, 0.0, 0.0};   // sum of returns, count, sum of lengths
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n_slots; i += gridDim.x * blockDim.x) {
    acc[0] += (double)ld(a, OUZ_F_EP_SUM, i);
    acc[1] += (double)ldi(a, OUZ_I_EP_CNT, i);
    acc[2] += (double)ldi(a, OUZ_I_EP_LEN, i);
    if (drain) {
      st(a, OUZ_F_EP_SUM, i, 0.0f);
      sti(a, OUZ_I_EP_CNT, i, 0);
      sti(a, OUZ_I_EP_LEN, i, 0);
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) s_part[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; ++k) {
      double p = 0.0;
      for (int j = 0; j < kStatsBlock / 64; ++j) p += s_part[k][j];
      partials[blockIdx.x * 3 + k] = p;
    }
    __threadfence();
    s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    __threadfence();
    double t[3] = {0.0, 0.0, 0.0};
    for (unsigned b = 0; b < gridDim.x; ++b)
      for (int k = 0; k < 3; ++k) t[k] += partials[b * 3 + k];
    out[0] = t[0];
    out[1] = t[1];
    out[2] = t[2];
    *ticket = 0u;   // ready for the next launch on this stream
  }
}

// The same statistics for n <= kStatsOneBlockEnvs: ONE block of 1024 threads strides over every env
// (at 4096 envs four independent loads per field and thread, all in flight together) and reduces
// through its waves in fixed order.  No partials, no device-scope fence, no ticket: the multi-block
// form's fence + atomic + last-block pass made a 6 us kernel out of 48 KB of reads, 40 % of a
// 16-step rollout's step time at 4096 envs.  Deterministic (fixed order), but not bitwise equal
// to the multi-block form's order.
constexpr int kStatsOneBlock = 1024;
constexpr int kStatsOneBlockEnvs = 65536;

__global__ void __launch_bounds__(kStatsOneBlock) episode_stats_one_block_kernel(StepArgs a, double* out, int drain) {
  __shared__ double s_part[3][kStatsOneBlock / 64];
  double acc[3] = {0.0, 0.0, 0.0};   // sum of returns, count, sum of lengths
  constexpr int kUnroll = 4;
  for (int base = threadIdx.x; base < a.n_slots; base += kStatsOneBlock * kUnroll) {
    float s[kUnroll];
    int32_t c[kUnroll], l[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int i = base + u * kStatsOneBlock;
      const bool ok = i < a.n_slots;
      s[u] = ok ? ld(a, OUZ_F_EP_SUM, i) : 0.0f;
      c[u] = ok ? ldi(a, OUZ_I_EP_CNT, i) : 0;
      l[u] = ok ? ldi(a, OUZ_I_EP_LEN, i) : 0;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int i = base + u * kStatsOneBlock;
      acc[0] += (double)s[u];
      acc[1] += (double)c[u];
      acc[2] += (double)l[u];
      if (drain && i < a.n_slots) {
        st(a, OUZ_F_EP_SUM, i, 0.0f);
        sti(a, OUZ_I_EP_CNT, i, 0);
        sti(a, OUZ_I_EP_LEN, i, 0);
      }
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) s_part[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double t = 0.0;
    for (int j = 0; j < kStatsOneBlock / 64; ++j) t += s_part[threadIdx.x][j];
    out[threadIdx.x] = t;
  }
}

// ---------------------------------------------------------------------------
// component kernels (AoS in/out; parity entry points)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) lee_kernel(int mode, const float* s, const float* cmd, float* thrust, float* torque, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* x = s + (size_t)i * 13;
  const float* c = cmd + (size_t)i * 4;
  V3 p = v3(x[0], x[1], x[2]), v = v3(x[7], x[8], x[9]), w = v3(x[10], x[11], x[12]);
  Q4 q{x[3], x[4], x[5], x[6]};
  float T;
  V3 tau;
  LeeGains g = default_gains();
  if (mode == OUZ_LEE_POSITION) lee_position(p, q, v, w, v3(c[0], c[1], c[2]), c[3], g, T, tau);
  else if (mode == OUZ_LEE_VELOCITY) lee_velocity(q, v, w, v3(c[0], c[1], c[2]), c[3], g, T, tau);
  else lee_attitude(q, w, c[0], c[1], c[2], c[3], g, T, tau);
  thrust[i] = T;
  torque[i * 3 + 0] = tau.x; torque[i * 3 + 1] = tau.y; torque[i * 3 + 2] = tau.z;
}

__global__ void __launch_bounds__(64) ekf_kernel(const float* q, const float* P, const float* gyr, const float* ang, float dt, float* qo,
                           float* Po, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  EkfQ e{q[i * 4], q[i * 4 + 1], q[i * 4 + 2], q[i * 4 + 3]};
  float p[10];
  #pragma unroll
  for (int k = 0; k < 10; ++k) p[k] = P[i * 10 + k];
  ekf_update(e, p, v3(gyr[i * 3], gyr[i * 3 + 1], gyr[i * 3 + 2]), EkfQ{ang[i * 4], ang[i * 4 + 1], ang[i * 4 + 2], ang[i * 4 + 3]}, dt);
  qo[i * 4] = e.w; qo[i * 4 + 1] = e.x; qo[i * 4 + 2] = e.y; qo[i * 4 + 3] = e.z;
  #pragma unroll
  for (int k = 0; k < 10; ++k) Po[i * 10 + k] = p[k];
}

__global__ void __launch_bounds__(64) pv_predict_kernel(float* x, float* P, const float* acc, const float* q, float dt, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float xx[9], pp[45];
  #pragma unroll
  for (int k = 0; k < 9; ++k) xx[k] = x[i * 9 + k];
  #pragma unroll
  for (int k = 0; k < 45; ++k) pp[k] = P[i * 45 + k];
  pv_predict(xx, pp, v3(acc[i * 3], acc[i * 3 + 1], acc[i * 3 + 2]), EkfQ{q[i * 4], q[i * 4 + 1], q[i * 4 + 2], q[i * 4 + 3]}, dt);
  #pragma unroll
  for (int k = 0; k < 9; ++k) x[i * 9 + k] = xx[k];
  #pragma unroll
  for (int k = 0; k < 45; ++k) P[i * 45 + k] = pp[k];
}

__global__ void __launch_bounds__(64) pv_correct_kernel(float* x, float* P, const float* z, int block, float var, const uint8_t* mask, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  float xx[9], pp[45];
  #pragma unroll
  for (int k = 0; k < 9; ++k) xx[k] = x[i * 9 + k];
  #pragma unroll
  for (int k = 0; k < 45; ++k) pp[k] = P[i * 45 + k];
  V3 zz = v3(z[i * 3], z[i * 3 + 1], z[i * 3 + 2]);
  if (block == 0) pv_correct<0>(xx, pp, zz, var);
  else pv_correct<1>(xx, pp, zz, var);
  #pragma unroll
  for (int k = 0; k < 9; ++k) x[i * 9 + k] = xx[k];
  #pragma unroll
  for (int k = 0; k < 45; ++k) P[i * 45 + k] = pp[k];
}

__global__ void __launch_bounds__(64) pv_step_kernel(float* x, float* P, const float* acc, const float* q, float dt,
                                                     const float* zp, const uint8_t* pmask, const float* zv,
                                                     const uint8_t* vmask, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float xx[9], pp[45];
#pragma unroll
  for (int k = 0; k < 9; ++k) xx[k] = x[i * 9 + k];
#pragma unroll
  for (int k = 0; k < 45; ++k) pp[k] = P[i * 45 + k];
  pv_step(xx, pp, v3(acc[i * 3], acc[i * 3 + 1], acc[i * 3 + 2]), EkfQ{q[i * 4], q[i * 4 + 1], q[i * 4 + 2], q[i * 4 + 3]}, dt,
          pmask && pmask[i], zp ? v3(zp[i * 3], zp[i * 3 + 1], zp[i * 3 + 2]) : v3(0, 0, 0), vmask && vmask[i],
          zv ? v3(zv[i * 3], zv[i * 3 + 1], zv[i * 3 + 2]) : v3(0, 0, 0));
#pragma unroll
  for (int k = 0; k < 9; ++k) x[i * 9 + k] = xx[k];
#pragma unroll
  for (int k = 0; k < 45; ++k) P[i * 45 + k] = pp[k];
}

// The quad-lane form of pv_step_kernel (quad_pv_ql.h): 16 envs per 64-lane block, four lanes each.
__global__ void __launch_bounds__(64) pv_step_quad_kernel(float* x, float* P, const float* acc, const float* q, float dt,
                                                          const float* zp, const uint8_t* pmask, const float* zv,
                                                          const uint8_t* vmask, int n) {
  __shared__ double s_pv[16 * kPvLdsEnv];
  const int i = blockIdx.x * 16 + (int)(threadIdx.x >> 2);
  const uint32_t sub = threadIdx.x & 3u;
  if (i >= n) return;   // whole quads only: the four lanes of an env share its fate
  double* env_lds = s_pv + (threadIdx.x >> 2) * kPvLdsEnv;
  const PvQl L{env_lds, env_lds + kPvLdsP, sub == 3u ? 0 : (int)sub, sub != 3u};
  float xx[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) xx[k] = x[i * 9 + k];
  pv_lds_load(L, [&](int f) { return P[i * 45 + f]; });
  ql_sync();
  pv_step_ql(L, xx, v3(acc[i * 3], acc[i * 3 + 1], acc[i * 3 + 2]), EkfQ{q[i * 4], q[i * 4 + 1], q[i * 4 + 2], q[i * 4 + 3]},
             dt, pmask && pmask[i], zp ? v3(zp[i * 3], zp[i * 3 + 1], zp[i * 3 + 2]) : v3(0, 0, 0), vmask && vmask[i],
             zv ? v3(zv[i * 3], zv[i * 3 + 1], zv[i * 3 + 2]) : v3(0, 0, 0));
  if (sub == 0u) {
#pragma unroll
    for (int k = 0; k < 9; ++k) x[i * 9 + k] = xx[k];
  }
  pv_lds_store(L, [&](int f, float v) { P[i * 45 + f] = v; });
}

__global__ void __launch_bounds__(64) integrate_kernel(float* root, const float* fb, const float* tb, const float* mass, const float* inertia,
                                 float dt, int substeps, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* s = root + (size_t)i * 13;
  V3 p = v3(s[0], s[1], s[2]), v = v3(s[7], s[8], s[9]), w = v3(s[10], s[11], s[12]);
  Q4 q{s[3], s[4], s[5], s[6]};
  const V3 I = v3(inertia[i * 3], inertia[i * 3 + 1], inertia[i * 3 + 2]);
  integrate(p, q, v, w, v3(fb[i * 3], fb[i * 3 + 1], fb[i * 3 + 2]), v3(tb[i * 3], tb[i * 3 + 1], tb[i * 3 + 2]),
            1.0f / mass[i], I, v3(1.0f / I.x, 1.0f / I.y, 1.0f / I.z), dt, substeps, 4.0f * kPiF);
  s[0] = p.x; s[1] = p.y; s[2] = p.z; s[3] = q.x; s[4] = q.y; s[5] = q.z; s[6] = q.w;
  s[7] = v.x; s[8] = v.y; s[9] = v.z; s[10] = w.x; s[11] = w.y; s[12] = w.z;
}

__global__ void __launch_bounds__(64) reward_kernel(const float* root, const float* target, const int32_t* progress, int max_ep, float z_die,
                              float* rew, int64_t* reset, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* s = root + (size_t)i * 13;
  float dist;
  float r = reward(v3(s[0], s[1], s[2]), v3(target[i * 3], target[i * 3 + 1], target[i * 3 + 2]), Q4{s[3], s[4], s[5], s[6]},
                   v3(s[10], s[11], s[12]), dist);
  bool die = dist > 8.0f || s[2] < z_die;
  rew[i] = r;
  reset[i] = (progress[i] >= max_ep - 1 || die) ? 1 : 0;
}

__global__ void __launch_bounds__(64) philox_kernel(uint64_t seed, const uint32_t* env, uint32_t step, uint32_t stream, uint32_t sub, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  U4 r = draw(seed, env[i], step, stream, sub);
  out[i * 4] = r.x; out[i * 4 + 1] = r.y; out[i * 4 + 2] = r.z; out[i * 4 + 3] = r.w;
}

}  // namespace ouz

// ===========================================================================
// C ABI
// ===========================================================================
using namespace ouz;

static_assert(sizeof(ouz_config) == 88, "ctypes OuzConfig mirror (ouzelum_amd/_lib.py)");
static_assert(sizeof(ouz_buffers) == 48, "ctypes OuzBuffers mirror");
static_assert(sizeof(ouz_task_info) == 32, "ctypes OuzTaskInfo mirror");
static_assert(sizeof(ouz_dr_noise) == 40, "ctypes OuzDrNoise mirror");
static_assert(sizeof(ouz_dr_param) == 32 && sizeof(ouz_dr_physical) == 104, "ctypes OuzDrPhysical mirror");

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(OUZ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return OUZ_OK;
}
inline int grid_for(int n, int block) { return (n + block - 1) / block; }
inline int block_for(int n) { return step_block_for(n); }   // the step kernel assumes this rule

#define OUZ_LAUNCH_CHECK(what)                                         \
  do {                                                                 \
    hipError_t _e = hipGetLastError();                                 \
    if (_e != hipSuccess) return hip_check(_e, what);                  \
  } while (0)
}  // namespace

// shared with learner_kernels.hip (one ouz_last_error for the whole library)
int set_error(int code, const std::string& msg) { return fail(code, msg); }

struct ouz_env {
  ouz_config cfg;
  ouz_buffers buf;
  bool bound;
  int64_t step;
  float2* wp_tab;   // device waypoint tables
  double* stats_partials;    // [kStatsMaxBlocks][3] per-block partials of episode_stats_kernel
  ouz_dr_noise* drn_dev;     // DrNonEnv: [2] DR noise params + sim_params gravity (read only when enabled)
  DrNonEnv drn_host;
  uint32_t* stats_ticket;    // its last-block counter (returns to 0 after every launch)
  double* wave_partials;     // [tiles][3] per-wave partials of the fused rollout statistics
  uint32_t* wave_ticket;     // their last-wave counter (returns to 0 after every launch)
  uint32_t* health_word;     // ouz_env_split_timeouts' read-back word (in the wave partials' tail)
  StepArgs args;    // pre-filled launch arguments
  // ouz_rollout as one step launch per step, outputs straight into the storage rows (streamed rollout):
  // above the latency regime the fused kernel's 16 steps of state in registers cost occupancy (LeeLanded
  // 177 VGPRs, 2 waves per SIMD, against the step kernel's 5) and it runs ~2x slower per step than the
  // step kernel.  OUZ_ROLLOUT_STREAM=0/1 overrides.
  bool stream_rollout;
  // The mixed curriculum's rollout above the latency regime as one launch per task (mixed_rollout: fused
  // QuadTracking chunks, streamed LeeLanded / QuadFault chunks): OUZ_MIXED_SPLIT_ROLLOUT=1, opt-in -- measured 3 %
  // slower than the one-launch fused kernel at 4 M envs (profiles/r05/mixed_split_rollout_probe.jsonl).
  bool mix_split_rollout;
  // Whole-batch flicker coins of steps [mask_lo, mask_lo + kMaskCache): a pure function of (seed, task,
  // step), drawn on the host (6 Philox blocks per step for a flickering task, ~0.3 us).  Filled for the
  // next launch's steps right after a launch is submitted, while the GPU runs it, so a launch does not
  // wait for its own coins (the first launch of a short timed region paid ~5 us of host time for them).
  static constexpr int kMaskCache = 64;
  int64_t mask_lo;
  int32_t mask_n;
  uint32_t mask[kMaskCache];
};

extern "C" {

int ouz_split_timeouts(uint32_t* out, int32_t reset) {
  if (!out) return fail(OUZ_ERR_INVALID, "ouz_split_timeouts: null pointer");
  int r = hip_check(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ouz_split_timeouts), sizeof(uint32_t)),
                    "hipMemcpyFromSymbol(split timeouts)");
  if (r || !reset) return r;
  const uint32_t zero = 0;
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_ouz_split_timeouts), &zero, sizeof(uint32_t)),
                   "hipMemcpyToSymbol(split timeouts)");
}

int ouz_env_split_timeouts(ouz_env* env, uint32_t* out, int32_t reset) {
  if (!env || !out) return fail(OUZ_ERR_INVALID, "ouz_env_split_timeouts: null pointer");
  int prev = 0;
  int r = hip_check(hipGetDevice(&prev), "hipGetDevice");
  if (r) return r;
  if (prev != env->cfg.device && (r = hip_check(hipSetDevice(env->cfg.device), "hipSetDevice"))) return r;
  // the read and the reset in ONE device atomic: a give-up counted between them is neither lost nor read twice
  hipLaunchKernelGGL(split_timeouts_read_kernel, dim3(1), dim3(1), 0, nullptr, env->health_word, reset ? 1 : 0);
  r = hip_check(hipGetLastError(), "split_timeouts_read_kernel");
  if (!r) r = hip_check(hipMemcpy(out, env->health_word, sizeof(uint32_t), hipMemcpyDeviceToHost),
                        "hipMemcpy(split timeouts)");
  if (prev != env->cfg.device) (void)hipSetDevice(prev);
  return r;
}

int ouz_set_split_spin_limit(uint32_t polls) {
  const uint32_t v = polls ? polls : kSplitSpinLimit;
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_ouz_split_spin_limit), &v, sizeof(uint32_t)),
                   "hipMemcpyToSymbol(split spin limit)");
}

#ifdef OUZ_STAMPS
int ouz_probe_stamps(uint64_t* host, int32_t count) {
  const int n = count < kStampWaves * kStampSlots ? count : kStampWaves * kStampSlots;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ouz_stamps), (size_t)n * sizeof(uint64_t)) == hipSuccess ? n : -1;
}
#endif

int32_t ouz_abi_version(void) { return OUZ_ABI_VERSION; }

#ifndef OUZ_SOURCE_ID
#define OUZ_SOURCE_ID "unknown"
#endif
const char* ouz_source_id(void) { return OUZ_SOURCE_ID; }

uint32_t ouz_build_flags(void) {
  uint32_t f = 0;
#ifdef OUZ_STAMPS
  f |= OUZ_BUILD_STAMPS;
#endif
#ifdef OUZ_TEMPORAL_STORES
  f |= OUZ_BUILD_TEMPORAL_STORES;
#endif
  return f;
}

int64_t ouz_state_slots(int32_t task, int32_t num_envs) {
  if (task < 0 || task >= OUZ_NUM_TASKS || num_envs <= 0) return fail(OUZ_ERR_INVALID, "ouz_state_slots: bad task / size");
  return state_slots(task, num_envs);
}
int ouz_env_slots(int32_t task, int32_t num_envs, int64_t env_id_offset, int32_t* env_slot) {
  if (task < 0 || task >= OUZ_NUM_TASKS || num_envs <= 0 || !env_slot || env_id_offset < 0 ||
      env_id_offset + num_envs > 0xFFFFFFFFll)
    return fail(OUZ_ERR_INVALID, "ouz_env_slots: bad arguments");
  const bool cls = class_layout_rt(task, num_envs);
  for (int32_t e = 0; e < num_envs; ++e)
    env_slot[e] = !cls ? e : (task == OUZ_TASK_MIXED ? mixed_env_slot((uint32_t)env_id_offset, e) : env_slot_of(e));
  return OUZ_OK;
}
const char* ouz_last_error(void) { return g_err.c_str(); }

void ouz_default_config(ouz_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->task = OUZ_TASK_LEE_LANDED;
  c->num_envs = 4096;
  c->pomdp = -1;
  c->pomdp_prob = -1.0f;
  c->dt = 0.01f;
  c->substeps = 2;
  c->convergence_time = 300;
  c->plat_speed = 15.0f * 0.165f;   // max husky speed: 15 rad/s wheels (utils/controllers.py:22-24)
  c->dr_lo = 0.9f;
  c->dr_hi = 1.1f;
  c->fault_eta_hi = 0.5f;
  c->thrust_max = 2000.0f;
  c->thrust_rate = 2000.0f;
}

int ouz_task_info_get(int32_t task, ouz_task_info* out) {
  if (!out || task < 0 || task >= OUZ_NUM_TASKS) return fail(OUZ_ERR_INVALID, "ouz_task_info_get: bad task");
  if (task == OUZ_TASK_MIXED) {
    *out = ouz_task_info{2000, 0.3f, 0.2f, -1, -1.0f, 1, -1, 0.0f};
    return OUZ_OK;
  }
  TaskParams t = task_preset(task);
  *out = ouz_task_info{t.max_ep, t.z_die, t.land_radius, t.pomdp, t.pomdp_prob, t.ctrl == CTRL_RL ? 1 : 0,
                       t.target_mode, t.plat_off_x};
  return OUZ_OK;
}

int ouz_create(const ouz_config* cfg, ouz_env** out) {
  if (!cfg || !out) return fail(OUZ_ERR_INVALID, "ouz_create: null argument");
  if (const char* bad = config_error(cfg)) return fail(OUZ_ERR_INVALID, std::string("ouz_create: ") + bad);
  const int64_t total = cfg->num_envs_total > 0 ? cfg->num_envs_total : cfg->num_envs;
  int r = hip_check(hipSetDevice(cfg->device), "hipSetDevice");
  if (r) return r;
  ouz_env* e = new ouz_env();
  e->cfg = *cfg;
  e->cfg.num_envs_total = total;
  e->bound = false;
  e->step = 0;
  float2 host_tab[204];
  build_waypoints(host_tab);
  r = hip_check(hipMalloc(&e->wp_tab, sizeof(host_tab)), "hipMalloc(waypoints)");
  if (r) { delete e; return r; }
  r = hip_check(hipMemcpy(e->wp_tab, host_tab, sizeof(host_tab), hipMemcpyHostToDevice), "hipMemcpy(waypoints)");
  if (r) { (void)hipFree(e->wp_tab); delete e; return r; }
  r = hip_check(hipMalloc(&e->stats_partials, kStatsMaxBlocks * 3 * sizeof(double) + sizeof(uint32_t)),
                "hipMalloc(stats)");
  if (r) { (void)hipFree(e->wp_tab); delete e; return r; }
  e->stats_ticket = reinterpret_cast<uint32_t*>(e->stats_partials + kStatsMaxBlocks * 3);
  r = hip_check(hipMalloc(&e->drn_dev, sizeof(DrNonEnv)), "hipMalloc(dr noise)");
  if (r) { (void)hipFree(e->stats_partials); (void)hipFree(e->wp_tab); delete e; return r; }
  // one partial per wave of the rollout grid: four per tile under the quad-lane class layout
  const size_t n_waves = (size_t)OUZ_TILES(state_slots(cfg->task, cfg->num_envs)) * 4;
  r = hip_check(hipMalloc(&e->wave_partials, n_waves * 3 * sizeof(double) + 64), "hipMalloc(wave partials)");
  if (r) { (void)hipFree(e->drn_dev); (void)hipFree(e->stats_partials); (void)hipFree(e->wp_tab); delete e; return r; }
  e->wave_ticket = reinterpret_cast<uint32_t*>(e->wave_partials + n_waves * 3);
  e->health_word = e->wave_ticket + 2;
  r = hip_check(hipMemset(e->wave_ticket, 0, sizeof(uint32_t)), "hipMemset(wave ticket)");
  if (r) { (void)hipFree(e->wave_partials); (void)hipFree(e->drn_dev); (void)hipFree(e->stats_partials);
           (void)hipFree(e->wp_tab); delete e; return r; }
  std::memset(&e->drn_host, 0, sizeof(e->drn_host));
  r = hip_check(hipMemset(e->stats_ticket, 0, sizeof(uint32_t)), "hipMemset(stats)");
  if (r) { (void)hipFree(e->stats_partials); (void)hipFree(e->wp_tab); delete e; return r; }
  StepArgs& a = e->args;
  fill_step_args(cfg, a);   // quad_env.h: the constants the host build fills the same way
  a.wp_tab = e->wp_tab;
  if (pipe_task(cfg->task) && cfg->num_envs > kLatencyRegimeEnvs) {
    // tiles per wave of quad_step_pipe_kernel (OUZ_PIPE_TILES; default and <= 1: the one-tile-per-wave kernel)
    const char* pt = std::getenv("OUZ_PIPE_TILES");
    const int per_wave = pt ? std::atoi(pt) : kPipeTilesDefault;
    if (per_wave > 1) {
      const int tiles = (cfg->num_envs + 63) / 64, wpb = kMaxBlock / 64;
      const int waves = (tiles + per_wave - 1) / per_wave;
      a.pipe_stride = (waves + wpb - 1) / wpb * wpb;
    }
  }
  {
    const char* nl = std::getenv("OUZ_NT_LOADS");
    a.nt_loads = (nl ? std::atoi(nl) != 0 : nt_loads_default(cfg->task, cfg->num_envs)) ? 1 : 0;
    if (a.cls) a.nt_loads = 0;   // the trigger-class layout (<= 64 K envs) has no such instantiation
  }
  {
    // the mixed curriculum above the latency regime as one launch per task (mixed_task_tile); OUZ_MIXED_SPLIT=0
    // keeps the one-launch kernel (bitwise the same results)
    const char* ms = std::getenv("OUZ_MIXED_SPLIT");
    a.mix_split = (cfg->task == OUZ_TASK_MIXED && !a.cls && a.env_offset % 64u == 0u &&
                   (ms ? std::atoi(ms) != 0 : true)) ? 1 : 0;
    const char* mr = std::getenv("OUZ_MIXED_SPLIT_ROLLOUT");
    e->mix_split_rollout = a.mix_split && mr && std::atoi(mr) != 0;
  }
  {
    // the quad-lane estimator kernels (quad_pv_ql.h): bit-identical results, opt-in -- measured slower than the
    // one-lane kernels at 4096 envs (its LDS exchanges cost more than the f64 work they split)
    const char* ql = std::getenv("OUZ_QUAD_LANE");
    const bool lat = cfg->num_envs <= kLatencyRegimeEnvs;   // the multi-wave forms are latency-regime grids
    a.quad = (a.cls && lat && ql && std::atoi(ql) != 0) ? 1 : 0;
    // the split-wave estimator rollout (quad_pv_split.h): bit-identical results; OUZ_SPLIT_PV=0 / 1 overrides
    const char* sp = std::getenv("OUZ_SPLIT_PV");
    a.split = (a.cls && lat && !a.quad && (sp ? std::atoi(sp) != 0 : kSplitDefault)) ? 1 : 0;
    // the output wave while the rollout's waves stay within one per SIMD (256 tiles); OUZ_OUT_WAVE=0 / 1 overrides
    const char* ow = std::getenv("OUZ_OUT_WAVE");
    // (the mixed curriculum has the output-wave form in its class layout only)
    const bool ow_size = a.n_slots <= kOutWaveMaxSlots && !a.quad && (a.cls || cfg->task != OUZ_TASK_MIXED);
    a.outw = (ow_size && (ow ? std::atoi(ow) != 0 : kOutWaveDefault)) ? 1 : 0;
  }
  {
    const char* rs = std::getenv("OUZ_ROLLOUT_STREAM");
    e->stream_rollout = rs ? std::atoi(rs) != 0 : stream_rollout_default(cfg->task, cfg->num_envs);
  }
  *out = e;
  return OUZ_OK;
}

int ouz_destroy(ouz_env* env) {
  if (!env) return OUZ_OK;
  if (env->wp_tab) (void)hipFree(env->wp_tab);
  if (env->stats_partials) (void)hipFree(env->stats_partials);
  if (env->drn_dev) (void)hipFree(env->drn_dev);
  if (env->wave_partials) (void)hipFree(env->wave_partials);
  delete env;
  return OUZ_OK;
}

int ouz_bind(ouz_env* env, const ouz_buffers* b) {
  if (!env || !b) return fail(OUZ_ERR_INVALID, "ouz_bind: null argument");
  if (!b->fstate || !b->istate || !b->obs || !b->rew || !b->reset || !b->timeouts)
    return fail(OUZ_ERR_INVALID, "ouz_bind: every buffer pointer must be set");
  env->buf = *b;
  env->bound = true;
  StepArgs& a = env->args;
  a.f = b->fstate;
  a.iv = b->istate;
  a.obs = b->obs;
  a.rew = b->rew;
  a.reset = b->reset;
  a.timeouts = b->timeouts;
  a.rst_in = b->reset;
  a.to_in = b->timeouts;
  return OUZ_OK;
}

int ouz_init_state(ouz_env* env, void* stream) {
  if (!env || !env->bound) return fail(OUZ_ERR_UNBOUND, "ouz_init_state: env not bound");
  const int n = env->cfg.num_envs, blk = block_for(n);
  hipLaunchKernelGGL(init_state_kernel, dim3(grid_for(env->args.n_slots, blk)), dim3(blk), 0, (hipStream_t)stream,
                     env->args, env->cfg.task);
  OUZ_LAUNCH_CHECK("init_state_kernel");
  env->step = 0;
  return OUZ_OK;
}

// One task's step or rollout kernel; the estimator tasks have a trigger-class-layout instantiation.
extern "C++" template <int T>
static void launch_task(bool single, const StepArgs& a, const RolloutArgs& r, dim3 g, dim3 b, hipStream_t s) {
  if constexpr (pipe_task(T)) {
    if (single && a.pipe_stride) {
      const dim3 pg(a.pipe_stride / (kMaxBlock / 64)), pb(kMaxBlock);
      if (a.nt_loads) hipLaunchKernelGGL((quad_step_pipe_kernel<T, true>), pg, pb, 0, s, a, r.ctx[0]);
      else hipLaunchKernelGGL((quad_step_pipe_kernel<T, false>), pg, pb, 0, s, a, r.ctx[0]);
      return;
    }
  }
  if constexpr (class_layout_task(T)) {
    if (a.cls && a.quad) {   // the quad-lane grid: four 64-lane blocks per 64-slot tile (step_body)
      const dim3 g4(g.x * 4);
      if (single) hipLaunchKernelGGL((quad_step_kernel<T, true, false, true>), g4, b, 0, s, a, r.ctx[0]);
      else hipLaunchKernelGGL((quad_rollout_kernel<T, true, true>), g4, b, 0, s, a, r);
      return;
    }
    if (a.cls && !single && (a.split || a.outw)) {   // multi-wave rollouts: one workgroup per 64-slot tile
      if (a.split && a.outw) hipLaunchKernelGGL((quad_rollout_kernel<T, true, false, true, true>), g, dim3(192), 0, s, a, r);
      else if (a.split) hipLaunchKernelGGL((quad_rollout_kernel<T, true, false, true, false>), g, dim3(128), 0, s, a, r);
      else hipLaunchKernelGGL((quad_rollout_kernel<T, true, false, false, true>), g, dim3(128), 0, s, a, r);
      return;
    }
    if (a.cls) {
      if (single) hipLaunchKernelGGL((quad_step_kernel<T, true>), g, b, 0, s, a, r.ctx[0]);
      else if (rollout_wpe(T, a.n) > 1)
        hipLaunchKernelGGL((quad_rollout_kernel<T, true, false, false, false, OUZ_EST_ROLLOUT_WPE>), g, b, 0, s, a, r);
      else hipLaunchKernelGGL((quad_rollout_kernel<T, true>), g, b, 0, s, a, r);
      return;
    }
  }
  if (single && a.nt_loads) hipLaunchKernelGGL((quad_step_kernel<T, false, true>), g, b, 0, s, a, r.ctx[0]);
  else if (single) hipLaunchKernelGGL((quad_step_kernel<T, false, false>), g, b, 0, s, a, r.ctx[0]);
  else if (T != OUZ_TASK_MIXED && a.outw)
    hipLaunchKernelGGL((quad_rollout_kernel<T, false, false, false, T != OUZ_TASK_MIXED>), g, dim3(128), 0, s, a, r);
  else if (class_layout_task(T) && rollout_wpe(T, a.n) > 1)
    hipLaunchKernelGGL((quad_rollout_kernel<T, false, false, false, false, (class_layout_task(T) ? OUZ_EST_ROLLOUT_WPE : 1)>), g, b,
                       0, s, a, r);
  else hipLaunchKernelGGL((quad_rollout_kernel<T, false>), g, b, 0, s, a, r);
}

// Waves of the launch of task T over the mixed curriculum's shard (mixed_task_tile): 21 per chunk of that task
// that touches the shard (the first and last chunk may be partial: their waves past the shard exit at once).
static int mixed_task_waves(const StepArgs& a, int task) {
  const uint32_t r = task == OUZ_TASK_LEE_LANDED ? 0u : (task == OUZ_TASK_TRACKING ? 1u : 2u);
  const uint32_t g0 = a.env_offset / 64u, cf = g0 / (uint32_t)kTrigClasses;
  const uint32_t last = (g0 + (uint32_t)((a.n + 63) / 64) - 1u) / (uint32_t)kTrigClasses;   // last chunk touched
  const uint32_t d = (r + 3u - cf % 3u) % 3u;
  if (cf + d > last) return 0;
  return (int)((last - cf - d) / 3u + 1u) * kTrigClasses;
}

extern "C++" template <int T>
static void launch_mixed_task(bool single, const StepArgs& a, const RolloutArgs& r, dim3 b, hipStream_t s) {
  const int waves = mixed_task_waves(a, T), wpb = (int)b.x / 64;
  if (waves == 0) return;
  const dim3 g((waves + wpb - 1) / wpb);
  if (single && a.nt_loads) hipLaunchKernelGGL((quad_step_kernel<T, false, true, false, true>), g, b, 0, s, a, r.ctx[0]);
  else if (single) hipLaunchKernelGGL((quad_step_kernel<T, false, false, false, true>), g, b, 0, s, a, r.ctx[0]);
  else if (T == OUZ_TASK_TRACKING)
    hipLaunchKernelGGL((quad_rollout_kernel<T, false, false, false, false, OUZ_EST_ROLLOUT_WPE, true>), g, b, 0, s, a, r);
  else hipLaunchKernelGGL((quad_rollout_kernel<T, false, false, false, false, 1, true>), g, b, 0, s, a, r);
}

static uint32_t cached_flicker_mask(ouz_env* env, int64_t step) {
  const int64_t off = step - env->mask_lo;
  if (off >= 0 && off < env->mask_n) return env->mask[off];
  return flicker_mask(env->args, env->cfg.task, (uint32_t)step);
}

// Coins of steps [from, from + count) into the cache (the window slides forward; count <= kMaskCache).
static void prefill_flicker_masks(ouz_env* env, int64_t from, int count) {
  if (from < env->mask_lo || from > env->mask_lo + env->mask_n) {   // not contiguous with the cached run: restart
    env->mask_lo = from;
    env->mask_n = 0;
  }
  const int64_t end = from + count;
  if (end - env->mask_lo > ouz_env::kMaskCache) {   // slide: keep the tail still needed
    const int64_t keep_lo = from;
    const int drop = (int)(keep_lo - env->mask_lo);
    const int kept = env->mask_n - drop > 0 ? env->mask_n - drop : 0;
    for (int i = 0; i < kept; ++i) env->mask[i] = env->mask[i + drop];
    env->mask_lo = keep_lo;
    env->mask_n = kept;
  }
  for (int64_t st = env->mask_lo + env->mask_n; st < end; ++st)
    env->mask[env->mask_n++] = flicker_mask(env->args, env->cfg.task, (uint32_t)st);
}

// Launch K (<= kMaxRolloutChunk) consecutive steps as ONE kernel.  K = 1 is VecTask.step.
// ring: action batches [ring_len][N][4] (step k uses batch (ring_pos + k) % ring_len) or null.
// storage: per-step outputs for these K steps ([K][N][...]) or null (outputs go to the env buffers).
static int launch_steps(ouz_env* env, const float* ring, int32_t ring_len, int64_t ring_pos, int32_t K,
                        const OutPtrs* storage, hipStream_t s, double* stats_out = nullptr, int stats_mode = 0,
                        const StepArgs* args = nullptr) {
  const StepArgs& a = args ? *args : env->args;
  const int n = env->cfg.num_envs, blk = block_for(n);
  RolloutArgs r;
  std::memset(&r, 0, sizeof(r));
  r.K = K;
  if (stats_mode) r.stats = RolloutStats{stats_out, env->wave_partials, env->wave_ticket, stats_mode};
  const OutPtrs envout{env->buf.obs, env->buf.rew, env->buf.reset, env->buf.timeouts};
  r.outs[0] = storage ? *storage : envout;
  r.outs[1] = envout;
  r.out_stride = storage ? (uint64_t)n : 0;
  for (int k = 0; k < K; ++k) {
    const uint32_t step = (uint32_t)(env->step + k);
    r.ctx[k].step = step;
    r.ctx[k].flick_mask = cached_flicker_mask(env, env->step + k);
    r.ctx[k].actions = ring ? ring + (size_t)((ring_pos + k) % ring_len) * n * OUZ_NUM_ACT : nullptr;
  }
  dim3 g(grid_for(a.n_slots, blk)), b(blk);   // one lane per state slot
  if (a.xcd_pack) {   // whole class blocks per XCD (xcd_tile)
    const int per_xcd = (a.n_slots / kClassBlock + 7) / 8 * kTrigClasses;
    g = dim3(8 * ((per_xcd + blk / 64 - 1) / (blk / 64)));
  }
  const bool single = K == 1 && !storage && !stats_mode;
  if (env->cfg.task == OUZ_TASK_MIXED && a.mix_split && single) {
    // VecTask.step as one launch per task over its chunks' tiles (mixed_task_tile).  A fused rollout keeps the
    // one-launch kernel unless OUZ_MIXED_SPLIT_ROLLOUT=1 (rollout_impl -> mixed_rollout)
    launch_mixed_task<OUZ_TASK_LEE_LANDED>(single, a, r, b, s);
    launch_mixed_task<OUZ_TASK_TRACKING>(single, a, r, b, s);
    launch_mixed_task<OUZ_TASK_FAULT>(single, a, r, b, s);
    OUZ_LAUNCH_CHECK("quad_step_kernel (mixed, per task)");
    env->step += K;
    prefill_flicker_masks(env, env->step, kMaxRolloutChunk);
    return OUZ_OK;
  }
#define OUZ_LAUNCH_TASK(T) launch_task<T>(single, a, r, g, b, s)
  switch (env->cfg.task) {
    case OUZ_TASK_OUZELUM: OUZ_LAUNCH_TASK(OUZ_TASK_OUZELUM); break;
    case OUZ_TASK_LEE_LANDED: OUZ_LAUNCH_TASK(OUZ_TASK_LEE_LANDED); break;
    case OUZ_TASK_EKF_LEE_LANDED: OUZ_LAUNCH_TASK(OUZ_TASK_EKF_LEE_LANDED); break;
    case OUZ_TASK_TRACKING: OUZ_LAUNCH_TASK(OUZ_TASK_TRACKING); break;
    case OUZ_TASK_FAULT: OUZ_LAUNCH_TASK(OUZ_TASK_FAULT); break;
    case OUZ_TASK_LANDING: OUZ_LAUNCH_TASK(OUZ_TASK_LANDING); break;
    default: OUZ_LAUNCH_TASK(OUZ_TASK_MIXED); break;
  }
#undef OUZ_LAUNCH_TASK
  OUZ_LAUNCH_CHECK("quad_step_kernel");
  env->step += K;
  prefill_flicker_masks(env, env->step, kMaxRolloutChunk);   // the next launch's coins, while this one runs
  return OUZ_OK;
}

static bool needs_actions(int task) {
  return task == OUZ_TASK_OUZELUM || task == OUZ_TASK_FAULT || task == OUZ_TASK_MIXED || task == OUZ_TASK_LANDING;
}

static int check_ring(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, const char* fn) {
  if (!env || !env->bound) return fail(OUZ_ERR_UNBOUND, std::string(fn) + ": env not bound");
  if (n_steps < 0 || (ring && ring_len <= 0)) return fail(OUZ_ERR_INVALID, std::string(fn) + ": bad sizes");
  if (!ring && needs_actions(env->cfg.task)) return fail(OUZ_ERR_INVALID, std::string(fn) + ": this task needs actions");
  if (ring && (reinterpret_cast<uintptr_t>(ring) & 15u)) return fail(OUZ_ERR_INVALID, std::string(fn) + ": actions must be 16-byte aligned");
  return OUZ_OK;
}

int ouz_step(ouz_env* env, const float* actions, void* stream) {
  int rc = check_ring(env, actions, 1, 1, "ouz_step");
  if (rc) return rc;
  return launch_steps(env, actions, 1, 0, 1, nullptr, (hipStream_t)stream);
}

int ouz_step_n(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, void* stream) {
  int rc = check_ring(env, ring, ring_len, n_steps, "ouz_step_n");
  if (rc) return rc;
  for (int32_t k = 0; k < n_steps; ++k) {
    rc = launch_steps(env, ring, ring_len, k, 1, nullptr, (hipStream_t)stream);
    if (rc) return rc;
  }
  return OUZ_OK;
}

// The mixed curriculum's rollout above the latency regime, one launch per task (StepArgs.mix_split): its
// QuadTracking chunks as the fused estimator rollout (up to kMaxRolloutChunk steps per launch, state in registers);
// its LeeLanded and QuadFault chunks streamed (one step launch per step, outputs straight into the storage rows),
// the form those tasks take at this size on their own.  Every env runs the same per-env code as in the one-launch
// kernel (equal within float tolerance, as the fused and streamed forms are).  The episode statistics are one
// ouz_episode_stats launch after the steps, as for a streamed rollout.
static int mixed_rollout(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, float* obs_out,
                         float* rew_out, int64_t* reset_out, uint8_t* timeouts_out, double* stats_out, int stats_mode,
                         hipStream_t s) {
  const bool store = obs_out != nullptr;
  const size_t n = (size_t)env->cfg.num_envs;
  const dim3 b(block_for((int)n));
  const OutPtrs envout{env->buf.obs, env->buf.rew, env->buf.reset, env->buf.timeouts};
  for (int32_t k0 = 0; k0 < n_steps; k0 += kMaxRolloutChunk) {
    const int32_t K = (n_steps - k0) < kMaxRolloutChunk ? (n_steps - k0) : kMaxRolloutChunk;
    const int64_t base = env->step;
    RolloutArgs r;
    std::memset(&r, 0, sizeof(r));
    r.K = K;
    for (int k = 0; k < K; ++k) {
      r.ctx[k].step = (uint32_t)(base + k);
      r.ctx[k].flick_mask = cached_flicker_mask(env, base + k);
      r.ctx[k].actions = ring ? ring + (size_t)((k0 + k) % ring_len) * n * OUZ_NUM_ACT : nullptr;
    }
    r.outs[0] = store ? OutPtrs{obs_out + (size_t)k0 * n * OUZ_NUM_OBS, rew_out + (size_t)k0 * n,
                                reset_out + (size_t)k0 * n, timeouts_out + (size_t)k0 * n} : envout;
    r.outs[1] = envout;
    r.out_stride = store ? (uint64_t)n : 0;
    launch_mixed_task<OUZ_TASK_TRACKING>(false, env->args, r, b, s);
    for (int32_t k = 0; k < K; ++k) {   // the streamed tasks, step by step (rollout_impl's streamed path)
      const int32_t g = k0 + k;
      StepArgs a = env->args;
      if (store && g > 0) {
        a.rst_in = reset_out + (size_t)(g - 1) * n;
        a.to_in = timeouts_out + (size_t)(g - 1) * n;
      }
      if (store && g + 1 < n_steps) {
        a.obs = obs_out + (size_t)g * n * OUZ_NUM_OBS;
        a.rew = rew_out + (size_t)g * n;
        a.reset = reset_out + (size_t)g * n;
        a.timeouts = timeouts_out + (size_t)g * n;
      }
      RolloutArgs r1;
      std::memset(&r1, 0, sizeof(r1));
      r1.K = 1;
      r1.ctx[0] = r.ctx[k];
      launch_mixed_task<OUZ_TASK_LEE_LANDED>(true, a, r1, b, s);
      launch_mixed_task<OUZ_TASK_FAULT>(true, a, r1, b, s);
    }
    OUZ_LAUNCH_CHECK("quad kernels (mixed rollout, per task)");
    env->step = base + K;
    prefill_flicker_masks(env, env->step, kMaxRolloutChunk);
  }
  if (store && n_steps > 0) {   // the streamed tasks' last step wrote the env buffers (the fused one wrote both)
    const size_t last = (size_t)(n_steps - 1) * n;
    const ouz_buffers& bf = env->buf;
    int rc = hip_check(hipMemcpyAsync(obs_out + last * OUZ_NUM_OBS, bf.obs, n * OUZ_NUM_OBS * sizeof(float),
                                      hipMemcpyDeviceToDevice, s), "hipMemcpyAsync(rollout obs)");
    if (!rc) rc = hip_check(hipMemcpyAsync(rew_out + last, bf.rew, n * sizeof(float), hipMemcpyDeviceToDevice, s),
                            "hipMemcpyAsync(rollout rew)");
    if (!rc) rc = hip_check(hipMemcpyAsync(reset_out + last, bf.reset, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s),
                            "hipMemcpyAsync(rollout reset)");
    if (!rc) rc = hip_check(hipMemcpyAsync(timeouts_out + last, bf.timeouts, n, hipMemcpyDeviceToDevice, s),
                            "hipMemcpyAsync(rollout timeouts)");
    if (rc) return rc;
  }
  return stats_mode ? ouz_episode_stats(env, stats_out, stats_mode == 2 ? 1 : 0, s) : OUZ_OK;
}

static int rollout_impl(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, float* obs_out,
                        float* rew_out, int64_t* reset_out, uint8_t* timeouts_out, double* stats_out, int stats_mode,
                        void* stream, const char* fn) {
  int rc = check_ring(env, ring, ring_len, n_steps, fn);
  if (rc) return rc;
  const bool store = obs_out || rew_out || reset_out || timeouts_out;
  if (store && !(obs_out && rew_out && reset_out && timeouts_out))
    return fail(OUZ_ERR_INVALID, std::string(fn) + ": give all four storage pointers or none");
  const size_t n = (size_t)env->cfg.num_envs;
  if (env->cfg.task == OUZ_TASK_MIXED && env->args.mix_split && env->mix_split_rollout)
    return mixed_rollout(env, ring, ring_len, n_steps, obs_out, rew_out, reset_out, timeouts_out, stats_out,
                         stats_mode, (hipStream_t)stream);
  if (env->stream_rollout) {
    // Streamed: step k reads the flags of row k - 1 and writes row k; the last step writes the env buffers,
    // which are then copied into the last row.  Bitwise K VecTask.step calls (the fused kernel is the same
    // per-env code in another loop, equal within float tolerance: tests/test_gpu_env.py).
    const hipStream_t s = (hipStream_t)stream;
    for (int32_t k = 0; k < n_steps; ++k) {
      StepArgs a = env->args;
      if (store && k > 0) {
        a.rst_in = reset_out + (size_t)(k - 1) * n;
        a.to_in = timeouts_out + (size_t)(k - 1) * n;
      }
      if (store && k + 1 < n_steps) {
        a.obs = obs_out + (size_t)k * n * OUZ_NUM_OBS;
        a.rew = rew_out + (size_t)k * n;
        a.reset = reset_out + (size_t)k * n;
        a.timeouts = timeouts_out + (size_t)k * n;
      }
      rc = launch_steps(env, ring, ring_len, k, 1, nullptr, s, nullptr, 0, &a);
      if (rc) return rc;
    }
    if (store && n_steps > 0) {
      const size_t last = (size_t)(n_steps - 1) * n;
      const ouz_buffers& b = env->buf;
      rc = hip_check(hipMemcpyAsync(obs_out + last * OUZ_NUM_OBS, b.obs, n * OUZ_NUM_OBS * sizeof(float),
                                    hipMemcpyDeviceToDevice, s), "hipMemcpyAsync(rollout obs)");
      if (!rc) rc = hip_check(hipMemcpyAsync(rew_out + last, b.rew, n * sizeof(float), hipMemcpyDeviceToDevice, s),
                              "hipMemcpyAsync(rollout rew)");
      if (!rc) rc = hip_check(hipMemcpyAsync(reset_out + last, b.reset, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s),
                              "hipMemcpyAsync(rollout reset)");
      if (!rc) rc = hip_check(hipMemcpyAsync(timeouts_out + last, b.timeouts, n, hipMemcpyDeviceToDevice, s),
                              "hipMemcpyAsync(rollout timeouts)");
      if (rc) return rc;
    }
    return stats_mode ? ouz_episode_stats(env, stats_out, stats_mode == 2 ? 1 : 0, stream) : OUZ_OK;
  }
  for (int32_t k0 = 0; k0 < n_steps; k0 += kMaxRolloutChunk) {
    const int32_t K = (n_steps - k0) < kMaxRolloutChunk ? (n_steps - k0) : kMaxRolloutChunk;
    OutPtrs st{obs_out + (size_t)k0 * n * OUZ_NUM_OBS, rew_out + (size_t)k0 * n, reset_out + (size_t)k0 * n,
               timeouts_out + (size_t)k0 * n};
    const bool last = k0 + K >= n_steps;
    rc = launch_steps(env, ring, ring_len, k0, K, store ? &st : nullptr, (hipStream_t)stream, stats_out,
                      last ? stats_mode : 0);
    if (rc) return rc;
  }
  return OUZ_OK;
}

int ouz_rollout(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, float* obs_out, float* rew_out,
                int64_t* reset_out, uint8_t* timeouts_out, void* stream) {
  return rollout_impl(env, ring, ring_len, n_steps, obs_out, rew_out, reset_out, timeouts_out, nullptr, 0, stream,
                      "ouz_rollout");
}

int ouz_rollout_stats(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, float* obs_out,
                      float* rew_out, int64_t* reset_out, uint8_t* timeouts_out, double* stats_out, int32_t drain,
                      void* stream) {
  if (!stats_out) return fail(OUZ_ERR_INVALID, "ouz_rollout_stats: null stats_out");
  if (env && !env->cfg.track_episodes)
    return fail(OUZ_ERR_INVALID, "ouz_rollout_stats: env created without track_episodes");
  if (n_steps <= 0) return fail(OUZ_ERR_INVALID, "ouz_rollout_stats: n_steps must be > 0");
  return rollout_impl(env, ring, ring_len, n_steps, obs_out, rew_out, reset_out, timeouts_out, stats_out,
                      drain ? 2 : 1, stream, "ouz_rollout_stats");
}

int ouz_pre_physics(ouz_env* env, const float* actions, float* wrench, void* stream) {
  int rc = check_ring(env, actions, 1, 1, "ouz_pre_physics");
  if (rc) return rc;
  if (!wrench) return fail(OUZ_ERR_INVALID, "ouz_pre_physics: null wrench");
  const StepArgs& a = env->args;
  const int n = env->cfg.num_envs, blk = block_for(n);
  StepCtx c{(uint32_t)env->step, cached_flicker_mask(env, env->step), actions};
  dim3 g(grid_for(a.n_slots, blk)), b(blk);
  const dim3 g4(g.x * 4);   // the quad-lane grid of the class layout (step_body)
  hipStream_t s = (hipStream_t)stream;
  switch (env->cfg.task) {
    case OUZ_TASK_OUZELUM: hipLaunchKernelGGL(quad_pre_kernel<OUZ_TASK_OUZELUM>, g, b, 0, s, a, c, wrench); break;
    case OUZ_TASK_LEE_LANDED: hipLaunchKernelGGL(quad_pre_kernel<OUZ_TASK_LEE_LANDED>, g, b, 0, s, a, c, wrench); break;
    case OUZ_TASK_EKF_LEE_LANDED:
      if (a.cls && a.quad) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_EKF_LEE_LANDED, true, true>), g4, b, 0, s, a, c, wrench);
      else if (a.cls) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_EKF_LEE_LANDED, true>), g, b, 0, s, a, c, wrench);
      else hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_EKF_LEE_LANDED, false>), g, b, 0, s, a, c, wrench);
      break;
    case OUZ_TASK_TRACKING:
      if (a.cls && a.quad) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_TRACKING, true, true>), g4, b, 0, s, a, c, wrench);
      else if (a.cls) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_TRACKING, true>), g, b, 0, s, a, c, wrench);
      else hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_TRACKING, false>), g, b, 0, s, a, c, wrench);
      break;
    case OUZ_TASK_FAULT: hipLaunchKernelGGL(quad_pre_kernel<OUZ_TASK_FAULT>, g, b, 0, s, a, c, wrench); break;
    case OUZ_TASK_LANDING: hipLaunchKernelGGL(quad_pre_kernel<OUZ_TASK_LANDING>, g, b, 0, s, a, c, wrench); break;
    default:
      if (a.cls && a.quad) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_MIXED, true, true>), g4, b, 0, s, a, c, wrench);
      else if (a.cls) hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_MIXED, true>), g, b, 0, s, a, c, wrench);
      else hipLaunchKernelGGL((quad_pre_kernel<OUZ_TASK_MIXED, false>), g, b, 0, s, a, c, wrench);
      break;
  }
  OUZ_LAUNCH_CHECK("quad_pre_kernel");
  return OUZ_OK;
}

int ouz_reset_idx(ouz_env* env, const int32_t* ids, int32_t n, void* stream) {
  if (!env || !env->bound) return fail(OUZ_ERR_UNBOUND, "ouz_reset_idx: env not bound");
  if (n < 0 || (n > 0 && !ids)) return fail(OUZ_ERR_INVALID, "ouz_reset_idx: bad ids");
  if (n == 0) return OUZ_OK;
  hipLaunchKernelGGL(mark_reset_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, env->buf.reset, ids, n,
                     env->cfg.num_envs);
  OUZ_LAUNCH_CHECK("mark_reset_kernel");
  return OUZ_OK;
}

int ouz_reset_all(ouz_env* env, void* stream) {
  if (!env || !env->bound) return fail(OUZ_ERR_UNBOUND, "ouz_reset_all: env not bound");
  const int n = env->cfg.num_envs;
  hipLaunchKernelGGL(mark_all_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, env->buf.reset, n);
  OUZ_LAUNCH_CHECK("mark_all_kernel");
  return OUZ_OK;
}

int ouz_episode_stats(ouz_env* env, double* out, int32_t drain, void* stream) {
  if (!env || !env->bound) return fail(OUZ_ERR_UNBOUND, "ouz_episode_stats: env not bound");
  if (!out) return fail(OUZ_ERR_INVALID, "ouz_episode_stats: null out");
  if (!env->cfg.track_episodes) return fail(OUZ_ERR_INVALID, "ouz_episode_stats: env created without track_episodes");
  const int n = env->cfg.num_envs;
  if (n <= kStatsOneBlockEnvs) {
    hipLaunchKernelGGL(episode_stats_one_block_kernel, dim3(1), dim3(kStatsOneBlock), 0, (hipStream_t)stream,
                       env->args, out, drain ? 1 : 0);
    OUZ_LAUNCH_CHECK("episode_stats_one_block_kernel");
    return OUZ_OK;
  }
  int grid = grid_for(n, kStatsBlock);
  if (grid > kStatsMaxBlocks) grid = kStatsMaxBlocks;
  hipLaunchKernelGGL(episode_stats_kernel, dim3(grid), dim3(kStatsBlock), 0, (hipStream_t)stream, env->args,
                     env->stats_partials, env->stats_ticket, out, drain ? 1 : 0);
  OUZ_LAUNCH_CHECK("episode_stats_kernel");
  return OUZ_OK;
}

int ouz_step_n_stats(ouz_env* env, const float* ring, int32_t ring_len, int32_t n_steps, double* stats_out,
                     int32_t drain, void* stream) {
  if (!stats_out) return fail(OUZ_ERR_INVALID, "ouz_step_n_stats: null stats_out");
  if (env && !env->cfg.track_episodes)
    return fail(OUZ_ERR_INVALID, "ouz_step_n_stats: env created without track_episodes");
  const int rc = ouz_step_n(env, ring, ring_len, n_steps, stream);
  if (rc) return rc;
  return ouz_episode_stats(env, stats_out, drain, stream);
}

int ouz_set_trace(ouz_env* env, float* trace, uint32_t* resets, int32_t env_index, int32_t capacity) {
  if (!env) return fail(OUZ_ERR_INVALID, "ouz_set_trace: null env");
  if (capacity == 0) {
    env->args.trace = nullptr;
    env->args.trace_resets = nullptr;
    env->args.trace_cap = 0;
    env->args.trace_env = -1;
    return OUZ_OK;
  }
  if (capacity < 64) return fail(OUZ_ERR_INVALID, "ouz_set_trace: capacity must be >= 64 (or 0 to disable)");
  if (!trace || !resets) return fail(OUZ_ERR_INVALID, "ouz_set_trace: null buffer");
  if (env_index < 0 || env_index >= env->cfg.num_envs) return fail(OUZ_ERR_INVALID, "ouz_set_trace: bad env_index");
  env->args.trace = trace;
  env->args.trace_resets = resets;
  env->args.trace_env = env_index;
  env->args.trace_cap = capacity;
  return OUZ_OK;
}

// The non-environment DR block (noise + gravity) to the device and the step's enable bits.  Synchronous: the
// parameters are in place before the next launch.
static int sync_dr_nonenv(ouz_env* env) {
  int r = hip_check(hipMemcpy(env->drn_dev, &env->drn_host, sizeof(env->drn_host), hipMemcpyHostToDevice),
                    "hipMemcpy(dr noise)");
  if (r) return r;
  env->args.drn = env->drn_dev;
  env->args.drn_mask = (env->drn_host.noise[0].distribution ? 1 : 0) | (env->drn_host.noise[1].distribution ? 2 : 0) |
                       (env->drn_host.grav.p.distribution ? 4 : 0);
  return OUZ_OK;
}

int ouz_set_dr_noise(ouz_env* env, int32_t target, const ouz_dr_noise* dr) {
  if (!env || target < 0 || target > 1) return fail(OUZ_ERR_INVALID, "ouz_set_dr_noise: bad env or target");
  ouz_dr_noise p{};
  if (dr) p = *dr;
  if (p.distribution < 0 || p.distribution > 2 || p.operation < 0 || p.operation > 1 || p.schedule < 0 ||
      p.schedule > 2 || (p.schedule && p.schedule_steps <= 0) || p.frequency < 0)
    return fail(OUZ_ERR_INVALID, "ouz_set_dr_noise: bad distribution / operation / schedule / frequency");
  env->drn_host.noise[target] = p;
  return sync_dr_nonenv(env);
}

int ouz_set_dr_gravity(ouz_env* env, const ouz_dr_param* dr, int32_t frequency) {
  if (!env) return fail(OUZ_ERR_INVALID, "ouz_set_dr_gravity: null env");
  ouz_dr_param p{};
  if (dr) p = *dr;
  if (const char* bad = dr_gravity_error(&p, frequency)) return fail(OUZ_ERR_INVALID, std::string("ouz_set_dr_gravity: ") + bad);
  env->drn_host.grav.p = p;
  env->drn_host.grav.frequency = frequency;
  return sync_dr_nonenv(env);
}

int ouz_set_dr_physical(ouz_env* env, const ouz_dr_physical* dr) {
  if (!env) return fail(OUZ_ERR_INVALID, "ouz_set_dr_physical: null env");
  if (dr)
    if (const char* bad = dr_physical_error(dr)) return fail(OUZ_ERR_INVALID, std::string("ouz_set_dr_physical: ") + bad);
  set_phys_dr(env->args, env->cfg.task, dr);   // by value in the launch arguments: read on the reset path only
  return OUZ_OK;
}

int64_t ouz_get_step(const ouz_env* env) { return env ? env->step : -1; }
int ouz_set_step(ouz_env* env, int64_t step) {
  if (!env || step < 0 || step > 0xFFFFFFFFll) return fail(OUZ_ERR_INVALID, "ouz_set_step: bad step");
  env->step = step;
  return OUZ_OK;
}

#define OUZ_CHECK_N(fn)                                                    \
  if (n < 0) return fail(OUZ_ERR_INVALID, fn ": n must be >= 0");          \
  if (n == 0) return OUZ_OK;

int ouz_lee_control(int32_t mode, const float* state, const float* cmd, float* thrust, float* torque, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_lee_control");
  if (mode < 0 || mode > 2) return fail(OUZ_ERR_INVALID, "ouz_lee_control: Invalid controller name");
  if (!state || !cmd || !thrust || !torque) return fail(OUZ_ERR_INVALID, "ouz_lee_control: null pointer");
  hipLaunchKernelGGL(lee_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, mode, state, cmd, thrust, torque, n);
  OUZ_LAUNCH_CHECK("lee_kernel");
  return OUZ_OK;
}

int ouz_ekf_update(const float* q, const float* P, const float* gyr, const float* ang, float dt, float* qo, float* Po,
                   int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_ekf_update");
  if (!q || !P || !gyr || !ang || !qo || !Po) return fail(OUZ_ERR_INVALID, "ouz_ekf_update: null pointer");
  hipLaunchKernelGGL(ekf_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, q, P, gyr, ang, dt, qo, Po, n);
  OUZ_LAUNCH_CHECK("ekf_kernel");
  return OUZ_OK;
}

int ouz_pv_predict(float* x, float* P, const float* acc, const float* q, float dt, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_pv_predict");
  if (!x || !P || !acc || !q) return fail(OUZ_ERR_INVALID, "ouz_pv_predict: null pointer");
  hipLaunchKernelGGL(pv_predict_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, x, P, acc, q, dt, n);
  OUZ_LAUNCH_CHECK("pv_predict_kernel");
  return OUZ_OK;
}

int ouz_pv_correct(float* x, float* P, const float* z, int32_t block, float var, const uint8_t* mask, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_pv_correct");
  if (!x || !P || !z) return fail(OUZ_ERR_INVALID, "ouz_pv_correct: null pointer");
  if (block != 0 && block != 1) return fail(OUZ_ERR_INVALID, "ouz_pv_correct: block must be 0 (position) or 1 (velocity)");
  hipLaunchKernelGGL(pv_correct_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, x, P, z, block, var, mask, n);
  OUZ_LAUNCH_CHECK("pv_correct_kernel");
  return OUZ_OK;
}

int ouz_pv_step(float* x, float* P, const float* acc, const float* q, float dt, const float* pos_z,
                const uint8_t* pos_mask, const float* vel_z, const uint8_t* vel_mask, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_pv_step");
  if (!x || !P || !acc || !q) return fail(OUZ_ERR_INVALID, "ouz_pv_step: null pointer");
  if ((pos_mask && !pos_z) || (vel_mask && !vel_z)) return fail(OUZ_ERR_INVALID, "ouz_pv_step: mask without data");
  hipLaunchKernelGGL(pv_step_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, x, P, acc, q, dt, pos_z,
                     pos_mask, vel_z, vel_mask, n);
  OUZ_LAUNCH_CHECK("pv_step_kernel");
  return OUZ_OK;
}

int ouz_pv_step_quad(float* x, float* P, const float* acc, const float* q, float dt, const float* pos_z,
                     const uint8_t* pos_mask, const float* vel_z, const uint8_t* vel_mask, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_pv_step_quad");
  if (!x || !P || !acc || !q) return fail(OUZ_ERR_INVALID, "ouz_pv_step_quad: null pointer");
  if ((pos_mask && !pos_z) || (vel_mask && !vel_z)) return fail(OUZ_ERR_INVALID, "ouz_pv_step_quad: mask without data");
  hipLaunchKernelGGL(pv_step_quad_kernel, dim3(grid_for(n, 16)), dim3(64), 0, (hipStream_t)stream, x, P, acc, q, dt,
                     pos_z, pos_mask, vel_z, vel_mask, n);
  OUZ_LAUNCH_CHECK("pv_step_quad_kernel");
  return OUZ_OK;
}

int ouz_integrate(float* root, const float* fb, const float* tb, const float* mass, const float* inertia, float dt,
                  int32_t substeps, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_integrate");
  if (!root || !fb || !tb || !mass || !inertia || substeps <= 0) return fail(OUZ_ERR_INVALID, "ouz_integrate: bad argument");
  hipLaunchKernelGGL(integrate_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, root, fb, tb, mass, inertia, dt,
                     substeps, n);
  OUZ_LAUNCH_CHECK("integrate_kernel");
  return OUZ_OK;
}

int ouz_reward(const float* root, const float* target, const int32_t* progress, int32_t max_ep, float z_die, float* rew,
               int64_t* reset, int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_reward");
  if (!root || !target || !progress || !rew || !reset) return fail(OUZ_ERR_INVALID, "ouz_reward: null pointer");
  hipLaunchKernelGGL(reward_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, root, target, progress, max_ep,
                     z_die, rew, reset, n);
  OUZ_LAUNCH_CHECK("reward_kernel");
  return OUZ_OK;
}

int ouz_philox(uint64_t seed, const uint32_t* env_ids, uint32_t step, uint32_t stream_id, uint32_t sub, uint32_t* out4,
               int32_t n, void* stream) {
  OUZ_CHECK_N("ouz_philox");
  if (!env_ids || !out4) return fail(OUZ_ERR_INVALID, "ouz_philox: null pointer");
  hipLaunchKernelGGL(philox_kernel, dim3(grid_for(n, 64)), dim3(64), 0, (hipStream_t)stream, seed, env_ids, step, stream_id, sub,
                     out4, n);
  OUZ_LAUNCH_CHECK("philox_kernel");
  return OUZ_OK;
}

}  // extern "C"
