// The per-env VecTask.step of the quadrotor tasks: register state, lazy reset, controller / estimator, wrench,
// integration, observation / reward / done.  ONE source for two builds:
//  * the HIP kernels (quad_kernels.hip, gfx950): OUZ_DEV = __device__ __forceinline__, one env per lane of a
//    wave64, the wave-tiled SoA state addressed through wave-uniform tile bases;
//  * the host build (quad_host.cpp, -DOUZ_HOST, g++ -fopenmp): OUZ_DEV = inline, one env per loop iteration
//    over the same state layout (include/ouzelum.h OUZ_FIDX), the CPU product path behind make(sim_device="cpu").
// Only memory access (tile bases, non-temporal hints, the accumulators' atomics), the LDS parking of the f64 PV
// step's register peak and the split-wave / quad-lane estimator forms (device-only files) differ between them.
#pragma once
#ifdef OUZ_HOST
#include "host_compat.h"
#endif
#include <cstddef>
#include <cstdlib>
#include "../../include/ouzelum.h"
#include "quad_math.h"

#ifdef OUZ_HOST
#define OUZ_DEV inline __attribute__((always_inline))
// one host thread owns an env: the accumulators are plain read-add-writes
#define OUZ_ACC_ADD(p, v) (*(p) += (v))
#define OUZ_STAMP(k, wait) do {} while (0)
namespace ouz {
// the device-only estimator forms (quad_pv_ql.h, quad_pv_split.h) are never instantiated on the host: their
// names are declared so that env_core's discarded `if constexpr` branches still parse
struct PvQl;
struct SplitLane;
void pv_split_publish(const SplitLane&, EkfQ);
void pv_split_predict(const float*, V3, EkfQ, float, PvReal*);
void pv_split_correct(const SplitLane&, PvReal*, float*, bool, V3, bool, V3);
void pv_step_ql(const PvQl&, float*, V3, EkfQ, float, bool, V3, bool, V3);
}  // namespace ouz
#else
#define OUZ_DEV __device__ __forceinline__
// accumulators: one lane owns each address, so a no-return atomic add is the same f32 / i32 read-add-write
// without a load round trip before the wave can retire
#define OUZ_ACC_ADD(p, v) atomicAdd((p), (v))
#endif

namespace ouz {

enum Ctrl { CTRL_RL = 0, CTRL_LEE_TRUE = 1, CTRL_LEE_EST = 2 };
enum TargetMode { TGT_GOAL = 0, TGT_PLATFORM = 1, TGT_TRAJ = 2 };
constexpr int kMaxBlock = 256;   // step/rollout kernel launch bound (LDS staging is sized for it)
// At or below this many envs a launch has at most 4 waves per CU and the step is latency-bound;
// above it, bandwidth-bound (the launch grid switches from 64- to 256-lane blocks at the same size).
constexpr int kLatencyRegimeEnvs = 65536;
// quad_step_pipe_kernel (the RL tasks' large-N VecTask.step with the next tile's state in flight): opt-in
// through OUZ_PIPE_TILES=<tiles per wave> at env creation.  It beat the one-tile kernel only while the
// state loads were plain (4 M envs QuadFault 215-241 against 245-262 us); with the non-temporal loads of
// nt_loads_default the one-tile kernel is faster (QuadFault 4 M 190-200 against 210-223 us, 8 M 410-423
// against 416-458; Ouzelum equal within 2 %: profiles/r02/pipe_step_kernel_sizes_ab.jsonl).
constexpr int kPipeTilesDefault = 1;
// s_waitcnt immediate (gfx9 encoding): vmcnt(0), expcnt / lgkmcnt left at their maxima (no wait)
constexpr int kWaitVmcnt0 = (0x7 << 4) | (0xF << 8);

// Trigger-class slot layout of the estimator tasks.  The PV filter's shared trigger
// counters fire the position fix on g % 7 == 6 and the velocity fix on g % 3 == 0 (g = step * N_total +
// global id, ekf_lee_landed.py:425-440), so an env's trigger pattern is fixed by its id mod 21.  The state
// slots of these tasks are grouped in blocks of 21 waves (1344 slots): wave k of block b holds envs
// b*1344 + k + 21*l (l = lane), one trigger class per wave, so the PV corrections are wave-uniform
// branches instead of every wave paying for both.  Slots past num_envs are idle lanes; the env-order
// buffers (obs, rew, reset, time_outs, actions) are indexed by env.
constexpr int kTrigClasses = 21;
constexpr int kClassBlock = kTrigClasses * 64;
// Latency regime only: at large N the env-order buffers' per-lane accesses 21 envs apart would cost more
// HBM traffic (a 64-byte line per lane for the 8-byte reset flag, measured 0.74 -> 0.30 of HBM peak at
// 4 M envs) than the uniform triggers save; there the step is HBM-bound and keeps slot i = env i.
// The mixed curriculum (config E) assigns tasks to chunks of 1344 global ids (LeeLanded, QuadTracking,
// QuadFault, repeating): a chunk is one class block, so in the latency regime its QuadTracking chunks take
// the trigger-class layout too.  Its slot space is chunk-aligned in global ids: slot s of a shard holds
// global id c*1344 + r' with c = env_offset/1344 + s/1344, r = s % 1344 and r' = the class permutation of
// r in a QuadTracking chunk, r' = r otherwise; ids outside the shard are idle slots.  At most
// ceil(n/1344) + 1 chunks touch a shard of n envs.
constexpr int kMixedChunk = kClassBlock;
__host__ __device__ constexpr int mixed_chunk_task(uint32_t chunk) {
  return chunk % 3u == 0u ? OUZ_TASK_LEE_LANDED : (chunk % 3u == 1u ? OUZ_TASK_TRACKING : OUZ_TASK_FAULT);
}
__host__ __device__ constexpr bool class_layout_task(int task) {
  return task == OUZ_TASK_EKF_LEE_LANDED || task == OUZ_TASK_TRACKING || task == OUZ_TASK_MIXED;
}
__host__ __device__ constexpr bool class_layout(int task, int n) {
  return class_layout_task(task) && n <= kLatencyRegimeEnvs;
}
// The trigger-class layout above the latency regime as well (OUZ_CLS_LARGE=1 in the environment at env creation
// and for ouz_state_slots / ouz_env_slots, which must agree): there the class blocks' waves are packed onto one
// XCD each (StepArgs.xcd_pack), so the partial output lines of a block's waves meet in that XCD's L2.
inline bool cls_large_requested() {
  const char* v = std::getenv("OUZ_CLS_LARGE");
  return v && std::atoi(v) != 0;
}
inline bool class_layout_rt(int task, int n) {
  return class_layout(task, n) || (class_layout_task(task) && cls_large_requested());
}
inline int state_slots(int task, int n) {
  if (!class_layout_rt(task, n)) return n;
  const int blocks = (n + kClassBlock - 1) / kClassBlock;
  return (task == OUZ_TASK_MIXED ? blocks + 1 : blocks) * kClassBlock;
}
__host__ __device__ inline int slot_env(int s) {   // class layout: env held by state slot s
  const int b = s / kClassBlock, r = s - b * kClassBlock;
  return b * kClassBlock + (r >> 6) + kTrigClasses * (r & 63);
}
__host__ __device__ inline int env_slot_of(int e) {   // its inverse
  const int b = e / kClassBlock, r = e - b * kClassBlock;
  return b * kClassBlock + (r % kTrigClasses) * 64 + r / kTrigClasses;
}
// Mixed curriculum, latency regime: the env (shard-local index; < 0 or >= n: an idle slot) held by slot s.
__host__ __device__ inline int64_t mixed_slot_env(uint32_t env_offset, int s) {
  const uint32_t c = env_offset / kClassBlock + (uint32_t)(s / kClassBlock);
  const int r = s % kClassBlock;
  const int rel = mixed_chunk_task(c) == OUZ_TASK_TRACKING ? (r >> 6) + kTrigClasses * (r & 63) : r;
  return (int64_t)c * kClassBlock + rel - (int64_t)env_offset;
}
__host__ inline int mixed_env_slot(uint32_t env_offset, int e) {   // its inverse
  const uint32_t gid = env_offset + (uint32_t)e, c = gid / kClassBlock;
  const int r = (int)(gid % kClassBlock);
  const int rel = mixed_chunk_task(c) == OUZ_TASK_TRACKING ? (r % kTrigClasses) * 64 + r / kTrigClasses : r;
  return (int)(c - env_offset / kClassBlock) * kClassBlock + rel;
}

// Task presets — mirror oracle/quad_oracle.py::task_spec.
struct TaskParams {
  int32_t ctrl, target_mode, max_ep, pomdp;
  float z_die, land_radius, plat_off_x, pomdp_prob;
  float noise_lo, noise_hi;   // 1 -/+ sigma rounded to f32 (utils/POMDP.py:10)
  int32_t land_vs_ctrl, dr, fault, motor_yaw;
};

static TaskParams task_preset(int task) {
  TaskParams t{};
  switch (task) {
    case OUZ_TASK_OUZELUM:  // tasks/ouzelum.py, cfg/task/Ouzelum.yaml
      t = TaskParams{CTRL_RL, TGT_GOAL, 2000, OUZ_POMDP_NONE, 0.5f, 0.0f, 0.0f, 0.0f, 1, 1, 0, 0, 0, 0};
      break;
    case OUZ_TASK_LEE_LANDED:  // tasks/lee_landed.py:25,263-330
      t = TaskParams{CTRL_LEE_TRUE, TGT_PLATFORM, 2000, OUZ_POMDP_FLICKER, 0.3f, 0.2f, 0.08f, 0.01f, 1, 1, 1, 0, 0, 0};
      break;
    case OUZ_TASK_EKF_LEE_LANDED:  // tasks/ekf_lee_landed.py
      t = TaskParams{CTRL_LEE_EST, TGT_PLATFORM, 700, OUZ_POMDP_FLICKER, 0.3f, 0.25f, -0.08f, 0.0f, 1, 1, 0, 0, 0, 0};
      break;
    case OUZ_TASK_TRACKING:
      t = TaskParams{CTRL_LEE_EST, TGT_TRAJ, 700, OUZ_POMDP_FLICKER, 0.3f, 0.25f, -0.08f, 0.0f, 1, 1, 0, 1, 0, 0};
      break;
    case OUZ_TASK_FAULT:
      t = TaskParams{CTRL_RL, TGT_GOAL, 2000, OUZ_POMDP_NOISE, 0.5f, 0.0f, 0.0f, 0.1f, 1, 1, 0, 0, 1, 1};
      break;
    case OUZ_TASK_LANDING:  // tasks/landing.py, cfg/task/Landing.yaml: RL thrust + husky on its trajectories
      t = TaskParams{CTRL_RL, TGT_TRAJ, 2000, OUZ_POMDP_NONE, 0.3f, 0.0f, 0.08f, 0.0f, 1, 1, 0, 0, 0, 0};
      break;
    default:
      break;
  }
  return t;
}

struct EnvConsts {
  float dt, thrust_step, thrust_max, plat_speed, dr_lo, dr_hi, fault_eta_hi, wmax;
  int32_t substeps, conv_time;
  float mass, ixx, iyy, izz;
  float inv_mass, inv_ixx, inv_iyy, inv_izz;
};

// Physical domain randomisation as the step reads it (include/ouzelum.h ouz_dr_physical): the ABI parameters and
// what the host derives from them once.
struct PhysDr {
  ouz_dr_physical p;
  int32_t need_last;     // frequency > 1 or a setup_only parameter: the reset reads the env's OUZ_I_RAND_STEP
  int32_t gauss;         // a gaussian parameter: the reset draws a second Philox block for its Box-Muller pairs
  int32_t inertia_add;   // additive inertia: the zz scale follows from the xx scale (the same sample on each axis)
};

struct StepArgs {
  float* f;
  int32_t* iv;
  float* obs;
  float* rew;
  int64_t* reset;
  uint8_t* timeouts;
  // reset_buf / time_outs as the step reads them (the previous step's flags): the env buffers, or the
  // previous storage row of a streamed rollout (ouz_rollout above the latency regime)
  const int64_t* rst_in;
  const uint8_t* to_in;
  const float2* wp_tab;        // lemniscate[100] | circle[100] | square[4]
  int32_t n;
  int32_t n_slots;             // state slots: n, or the trigger-class layout's padded count
  int32_t cls;                 // 1: trigger-class slot layout (estimator tasks), 2: the mixed curriculum's
  uint32_t env_offset;
  uint64_t n_total;
  uint64_t seed;
  int32_t track_episodes;
  int32_t pipe_stride;         // quad_step_pipe_kernel: waves in its grid (0: that kernel is not used)
  int32_t nt_loads;            // step kernels: non-temporal state loads (large N: nt_loads_default)
  int32_t quad;                // trigger-class layout: the quad-lane estimator kernels (OUZ_QUAD_LANE=1; quad_pv_ql.h)
  int32_t split;               // trigger-class layout: the split-wave estimator rollout (OUZ_SPLIT_PV; quad_pv_split.h)
  int32_t outw;                // latency-regime rollouts with an output wave (OUZ_OUT_WAVE; out_wave)
  int32_t xcd_pack;            // class layout above the latency regime: a class block's waves on one XCD (xcd_tile)
  int32_t mix_split;           // mixed curriculum above the latency regime: one launch per task (mixed_task_tile)
  const ouz_dr_noise* drn;    // VecTask DR noise params in device memory: [0] observations, [1] actions
  int32_t drn_mask;            // bit 0: observation noise on, bit 1: action noise on
  float* trace;                // ouz_set_trace: [trace_cap][9] (p, target, v) of env trace_env
  uint32_t* trace_resets;      // [trace_cap] envs reset at the start of each step
  int32_t trace_env, trace_cap;
  EnvConsts c;
  TaskParams tp[3];            // by tp_slot(task): the configured task, or the three curriculum tasks
  PhysDr pdr;                  // physical DR of the tasks whose TaskParams.dr is set
};

// Task-parameter slot: a single-task env fills only its task's slot, the mixed curriculum the slots of
// LeeLanded (0), QuadTracking (1) and QuadFault (2).  Three slots instead of one per task keep the
// kernel arguments (copied by the host on every launch) at 168 instead of 336 bytes of parameters.
__host__ __device__ constexpr int tp_slot(int task) {
  return task == OUZ_TASK_TRACKING ? 1 : (task == OUZ_TASK_FAULT ? 2 : 0);
}

// x500 lumped body (assets/x500/x500.urdf).  Rotor arms, x500.urdf:3-29.
#ifdef OUZ_HOST
constexpr float kRotorX[4] = {0.174f, -0.174f, 0.174f, -0.174f};
constexpr float kRotorY[4] = {-0.174f, 0.174f, 0.174f, -0.174f};
constexpr float kRotorDir[4] = {1.0f, 1.0f, -1.0f, -1.0f};
#else
__device__ __constant__ float kRotorX[4] = {0.174f, -0.174f, 0.174f, -0.174f};
__device__ __constant__ float kRotorY[4] = {-0.174f, 0.174f, 0.174f, -0.174f};
__device__ __constant__ float kRotorDir[4] = {1.0f, 1.0f, -1.0f, -1.0f};   // ccw ccw cw cw (model.sdf:516-575)
#endif
constexpr float kMotorKm = 0.016f;
// husky differential drive (utils/controllers.py:15-43; gains landing.py:361)
constexpr float kWheelBase = 0.54f, kWheelRadius = 0.165f;
constexpr float kDriveGainLin = 3.0f, kDriveGainAng = 1000.0f, kDriveAngThresh = 0.005f;
constexpr float kPiF32 = 3.14159265358979f;
OUZ_DEV float map_to_pi(float a) {   // utils/controllers.py:5-13 (one wrap)
  a = a > kPiF32 ? a - 2.0f * kPiF32 : a;
  return a <= -kPiF32 ? a + 2.0f * kPiF32 : a;
}
constexpr int kTrajLen[3] = {100, 100, 4};
constexpr int kTrajBase[3] = {0, 100, 200};

OUZ_DEV int mixed_task(uint32_t gid) { return mixed_chunk_task(gid / kMixedChunk); }

// Per-step context: the step counter (keys every draw, drives the convergence window),
// the host-drawn whole-batch flicker coins and this step's action batch.
struct StepCtx {
  uint32_t step;
  uint32_t flick_mask;
  const float* actions;
};

// A copy of the RNG seed the compiler cannot treat as loop invariant, for draws in branches that are off
// unless configured (DR noise): hoisted out of the fused rollout's step loop, their Philox round-key
// schedules held SGPRs across the whole loop (spilled to VGPR lanes).  Not used for the reset / goal
// draws: the RL tasks reset in some lane of most waves on most steps, and recomputing the key schedule
// there cost QuadFault 12 % per step (6 080 -> 6 812 cycles).
OUZ_DEV uint64_t cold_seed(uint64_t seed) {
#ifdef OUZ_HOST
  return seed;
#else
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  __asm__ volatile("" : "+s"(lo), "+s"(hi));
  return ((uint64_t)hi << 32) | lo;
#endif
}

// ---------------------------------------------------------------------------
// POMDP corruption (utils/POMDP.py:23-43) with counter-RNG draws
// ---------------------------------------------------------------------------
template <int D>
OUZ_DEV void pomdp_apply(float* x, const TaskParams& tp, int task, const StepArgs& a,
                                            const StepCtx& sc, uint32_t gid, uint32_t site, bool per_env_coin) {
  const int mode = tp.pomdp;
  if (mode == OUZ_POMDP_NONE) return;
  if (mode == OUZ_POMDP_FLICKER || mode == OUZ_POMDP_FLICKER_NOISE) {
    bool fire;
    if (per_env_coin) {
      const float p = (mode == OUZ_POMDP_FLICKER) ? tp.pomdp_prob : 0.1f;
      fire = unit_f32(draw(a.seed, gid, sc.step, RNG_POMDP + site, 0).x) <= p;
    } else {
      fire = (sc.flick_mask >> (tp_slot(task) * 8 + site)) & 1u;
    }
    if (fire) {
#pragma unroll
      for (int e = 0; e < D; ++e) x[e] = 0.0f;
    }
  }
  if (mode == OUZ_POMDP_NOISE || mode == OUZ_POMDP_FLICKER_NOISE) {
#pragma unroll
    for (int g = 0; g < (D + 3) / 4; ++g) {
      U4 r = draw(a.seed, gid, sc.step, RNG_POMDP + site, 128 + g);
      uint32_t w4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (g * 4 + k < D) x[g * 4 + k] *= uniform_f32(w4[k], tp.noise_lo, tp.noise_hi);
    }
  }
}

// ---------------------------------------------------------------------------
// VecTask DR noise lambdas (tasks/base/vec_task.py:576-646), counter-RNG normals (Box-Muller)
// ---------------------------------------------------------------------------
OUZ_DEV float normal_from(uint32_t a, uint32_t b, bool second) {
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);    // (0, 1]
  const float u2 = unit_f32(b);
  const float r = sqrtf(-2.0f * logf(u1));
  float sn, cs;
  sincospif(2.0f * u2, &sn, &cs);   // sin / cos(2 pi u2) with the exact reduction of sinpi (no Payne-Hanek code)
  return second ? r * sn : r * cs;
}

// Schedule scaling of a DR range at `step` (vec_task.py:584-589, dr_utils.py:82-87)
OUZ_DEV float dr_schedule(int32_t sched, int32_t sched_steps, uint32_t step) {
  if (sched == 1) return fminf((float)step, (float)sched_steps) / (float)sched_steps;
  if (sched == 2) return step < (uint32_t)sched_steps ? 0.0f : 1.0f;
  return 1.0f;
}

// D values of env gid (D <= 16): noise drawn from `stream`.  The parameters are those of the epoch
// e = step - step % frequency (the apply_randomizations call that last re-derived them, vec_task.py:559,577-646):
// the schedule is evaluated at e and the correlated draw corr (subs 64..) is keyed by e, so it is redrawn at every
// epoch (a new params dict has no 'corr', :610-615); the fresh draws (subs 0..3) are keyed by the step.
template <int D>
OUZ_DEV void dr_noise_apply(float* x, const ouz_dr_noise& p, uint64_t seed, uint32_t gid,
                                               uint32_t step, uint32_t stream) {
  if (p.distribution == 0) return;
  const uint32_t ep = p.frequency > 1 ? step - step % (uint32_t)p.frequency : step;
  const float s = dr_schedule(p.schedule, p.schedule_steps, ep);
  float a = p.range[0], b = p.range[1], ac = p.range_correlated[0], bc = p.range_correlated[1];
  const bool add = p.operation == 0, gauss = p.distribution == 1;
  if (add) {
    a *= s; b *= s; ac *= s; bc *= s;
  } else if (gauss) {                                                    // :601-606
    b *= s; a = a * s + (1.0f - s); bc *= s; ac = ac * s + (1.0f - s);
  } else {                                                               // :629-633
    a = a * s + (1.0f - s); b = b * s + (1.0f - s); ac = ac * s + (1.0f - s); bc = bc * s + (1.0f - s);
  }
  // Keep the correlated draws inside this rarely enabled branch: loop-invariant code motion hoisted them with
  // their Box-Muller log / sincos out of the fused rollout's step loop and speculated them unconditionally,
  // ~1500 instructions (~5000 cycles) before the first step of every launch whether or not DR noise was on
  // (scripts/stamp_rollout.py prologue, LeeLanded 8520 -> 3316 cycles).
#ifndef OUZ_HOST
  __asm__ volatile("" : "+v"(gid));
#endif
  seed = cold_seed(seed);
#pragma unroll
  for (int g = 0; g < (D + 3) / 4; ++g) {
    const U4 f = draw(seed, gid, step, stream, (uint32_t)g);
    const U4 c = draw(seed, gid, ep, stream, 64u + (uint32_t)g);
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w}, cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = g * 4 + k;
      if (e >= D) break;
      const float corr = normal_from(cw[k & 2], cw[(k & 2) + 1], k & 1);
      float n;
      if (gauss) n = corr * bc + ac + normal_from(fw[k & 2], fw[(k & 2) + 1], k & 1) * b + a;
      else n = corr * (bc - ac) + ac + unit_f32(fw[k]) * (b - a) + a;
      x[e] = add ? x[e] + n : x[e] * n;
    }
  }
}

// ---------------------------------------------------------------------------
// Physical DR (include/ouzelum.h ouz_dr_physical): one sample of dr_utils.generate_random_samples (:71-133) with the
// counter RNG -- u (and u2, the gaussian's Box-Muller partner) two draws of the env -- and the env's scale of the
// nominal value after apply_random_samples (:186-188: nominal * sample, or nominal + sample).
// ---------------------------------------------------------------------------
OUZ_DEV float dr_sample(const ouz_dr_param& p, uint32_t u, uint32_t u2, uint32_t step) {
  const float s = dr_schedule(p.schedule, p.schedule_steps, step);
  float a = p.range[0], b = p.range[1];
  if (p.operation == 0) { a *= s; b *= s; }                                  // additive: toward 0
  else if (p.distribution == 1) { b *= s; a = a * s + (1.0f - s); }          // scaling gaussian: mu toward 1
  else { a = a * s + (1.0f - s); b = b * s + (1.0f - s); }                   // scaling (log)uniform: toward 1
  if (p.distribution == 1) return a + b * normal_from(u, u2, false);         // np.random.normal(mu, var)
  if (p.distribution == 3) return expf(uniform_f32(u, logf(a), logf(b)));    // exp(np.random.uniform(log lo, log hi))
  return uniform_f32(u, a, b);                                               // np.random.uniform(lo, hi)
}
OUZ_DEV float dr_scale(const ouz_dr_param& p, float sample, float nominal) {
  return p.operation == 0 ? (nominal + sample) / nominal : sample;
}
constexpr float kMotorConstant = 8.54858e-06f;   // assets/x500/model.sdf:523 (T = k_f w^2 per rotor)

// sim_params gravity DR (include/ouzelum.h ouz_set_dr_gravity; vec_task.py:556-566,648-660, dr_utils.py:162-172):
// kept in device memory right after the two VecTask noise entries (StepArgs.drn), on when drn_mask bit 2 is set.
struct GravDr {
  ouz_dr_param p;
  int32_t frequency;
  int32_t reserved;
};
struct DrNonEnv {            // the device block StepArgs.drn points at
  ouz_dr_noise noise[2];     // [0] observations, [1] actions
  GravDr grav;
};
static_assert(offsetof(DrNonEnv, grav) == 2 * sizeof(ouz_dr_noise), "StepArgs.drn + 2 is the gravity entry");
OUZ_DEV const GravDr& grav_dr_of(const ouz_dr_noise* drn) { return *reinterpret_cast<const GravDr*>(drn + 2); }

// The gravity of step `step`: the non-environment gate re-randomizes every `frequency` steps, so it is the sample of
// the epoch e = step - step % frequency (schedule at e), one whole-sim draw of generate_random_samples(params, 3, e)
// (words k of the BATCH_ENV draws of stream RNG_GRAV), applied per axis to the nominal (0, 0, -9.81) as
// apply_random_samples does (nominal * sample or nominal + sample).  Wave-uniform.  oracle: quad_oracle.gravity_dr.
OUZ_DEV V3 gravity_dr(const GravDr& g, uint64_t seed, uint32_t step) {
  const uint32_t f = (uint32_t)g.frequency;
  const uint32_t ep = f > 1u ? step - step % f : step;
  seed = cold_seed(seed);
  const U4 u = draw(seed, BATCH_ENV, ep, RNG_GRAV, 0u);
  const U4 u2 = g.p.distribution == 1 ? draw(seed, BATCH_ENV, ep, RNG_GRAV, 1u) : U4{0u, 0u, 0u, 0u};
  const float s0 = dr_sample(g.p, u.x, u2.x, ep), s1 = dr_sample(g.p, u.y, u2.y, ep), s2 = dr_sample(g.p, u.z, u2.z, ep);
  const float nz = -kGravity;
  return g.p.operation == 0 ? v3(0.0f + s0, 0.0f + s1, nz + s2) : v3(0.0f * s0, 0.0f * s1, nz * s2);
}

// Wave-tiled SoA (include/ouzelum.h OUZ_FIDX): a wave's fields are contiguous
// 256-byte rows, field f at offset f*256 from the wave's tile base.  The tile base is
// wave-uniform (readfirstlane -> SGPR pair), the per-lane part a 32-bit offset, so every
// access is one `global_load/store v, v_off, s[base] offset:f*256` with no 64-bit VALU
// address arithmetic and no VGPR pairs held for pointers.
#ifdef OUZ_HOST
// host build (quad_host.cpp): one env per loop iteration, plain loads and stores
OUZ_DEV uint32_t wave_tile(int i) { return (uint32_t)i >> 6; }
OUZ_DEV float* ftile(const StepArgs& a, int i) { return a.f + (size_t)wave_tile(i) * (OUZ_F_COUNT * 64); }
OUZ_DEV int32_t* itile(const StepArgs& a, int i) { return a.iv + (size_t)wave_tile(i) * (OUZ_I_COUNT * 64); }
OUZ_DEV uint32_t lane_off(int field, int i) { return (uint32_t)field * 64u + ((uint32_t)i & 63u); }
OUZ_DEV float ld(const StepArgs& a, int field, int i) { return ftile(a, i)[lane_off(field, i)]; }
OUZ_DEV void st(const StepArgs& a, int field, int i, float v) { ftile(a, i)[lane_off(field, i)] = v; }
OUZ_DEV int32_t ldi(const StepArgs& a, int field, int i) { return itile(a, i)[lane_off(field, i)]; }
OUZ_DEV void sti(const StepArgs& a, int field, int i, int32_t v) { itile(a, i)[lane_off(field, i)] = v; }
OUZ_DEV V3 ld3(const StepArgs& a, int f, int i) { return v3(ld(a, f, i), ld(a, f + 1, i), ld(a, f + 2, i)); }
OUZ_DEV void st3(const StepArgs& a, int f, int i, V3 v) { st(a, f, i, v.x); st(a, f + 1, i, v.y); st(a, f + 2, i, v.z); }
struct Tile {
  float* f;
  int32_t* iv;
  uint32_t l;       // lane = env index within the tile
  uint32_t first;   // env index of lane 0
};
OUZ_DEV Tile tile_of(const StepArgs& a, int i) {
  return Tile{ftile(a, i), itile(a, i), (uint32_t)i & 63u, wave_tile(i) * 64u};
}
OUZ_DEV float ld(const Tile& t, int field) { return t.f[(uint32_t)field * 64u + t.l]; }
OUZ_DEV float ld_nt(const Tile& t, int field) { return ld(t, field); }
OUZ_DEV void st(const Tile& t, int field, float v) { t.f[(uint32_t)field * 64u + t.l] = v; }
OUZ_DEV int32_t ldi(const Tile& t, int field) { return t.iv[(uint32_t)field * 64u + t.l]; }
OUZ_DEV int32_t ldi_nt(const Tile& t, int field) { return ldi(t, field); }
OUZ_DEV void sti(const Tile& t, int field, int32_t v) { t.iv[(uint32_t)field * 64u + t.l] = v; }
#else
OUZ_DEV uint32_t wave_tile(int i) {
  return __builtin_amdgcn_readfirstlane((uint32_t)i >> 6);
}
OUZ_DEV float* ftile(const StepArgs& a, int i) {
  return a.f + (size_t)wave_tile(i) * (OUZ_F_COUNT * 64);
}
OUZ_DEV int32_t* itile(const StepArgs& a, int i) {
  return a.iv + (size_t)wave_tile(i) * (OUZ_I_COUNT * 64);
}
OUZ_DEV uint32_t lane_off(int field, int i) { return (uint32_t)field * 64u + ((uint32_t)i & 63u); }
OUZ_DEV float ld(const StepArgs& a, int field, int i) { return ftile(a, i)[lane_off(field, i)]; }
OUZ_DEV void st(const StepArgs& a, int field, int i, float v) { ftile(a, i)[lane_off(field, i)] = v; }
OUZ_DEV int32_t ldi(const StepArgs& a, int field, int i) { return itile(a, i)[lane_off(field, i)]; }
OUZ_DEV void sti(const StepArgs& a, int field, int i, int32_t v) { itile(a, i)[lane_off(field, i)] = v; }
OUZ_DEV V3 ld3(const StepArgs& a, int f, int i) { return v3(ld(a, f, i), ld(a, f + 1, i), ld(a, f + 2, i)); }
OUZ_DEV void st3(const StepArgs& a, int f, int i, V3 v) { st(a, f, i, v.x); st(a, f + 1, i, v.y); st(a, f + 2, i, v.z); }
// One wave's tile, resolved once per env pass: uniform base pointers + this lane's index.
struct Tile {
  float* f;
  int32_t* iv;
  uint32_t l;       // lane = env index within the tile
  uint32_t first;   // env index of lane 0 (wave-uniform)
};
OUZ_DEV Tile tile_of(const StepArgs& a, int i) {
  return Tile{ftile(a, i), itile(a, i), (uint32_t)i & 63u, wave_tile(i) * 64u};
}
OUZ_DEV float ld(const Tile& t, int field) { return t.f[(uint32_t)field * 64u + t.l]; }
OUZ_DEV float ld_nt(const Tile& t, int field) {
  return __builtin_nontemporal_load(&t.f[(uint32_t)field * 64u + t.l]);
}
// State and staged-output stores are non-temporal (`global_store ... nt`): nothing in the step reads
// them back, and at large N they are a write stream of 118-700 B per env-step.  Measured against
// plain stores: 4 M envs LeeLanded HBM fraction 0.59 -> 0.76, QuadFault 0.47 -> 0.54,
// QuadMixed 0.53 -> 0.57, estimator tasks +-1 %, the 4096-env step unchanged (3.51 us).
// -DOUZ_TEMPORAL_STORES restores plain stores for comparison (an A/B build: ouz_build_flags reports it).
#ifdef OUZ_TEMPORAL_STORES
#define OUZ_ST(p, v) (*(p) = (v))
#else
#define OUZ_ST(p, v) __builtin_nontemporal_store((v), (p))
#endif
OUZ_DEV void st(const Tile& t, int field, float v) { OUZ_ST(&t.f[(uint32_t)field * 64u + t.l], v); }
OUZ_DEV int32_t ldi(const Tile& t, int field) { return t.iv[(uint32_t)field * 64u + t.l]; }
OUZ_DEV int32_t ldi_nt(const Tile& t, int field) {
  return __builtin_nontemporal_load(&t.iv[(uint32_t)field * 64u + t.l]);
}
OUZ_DEV void sti(const Tile& t, int field, int32_t v) { OUZ_ST(&t.iv[(uint32_t)field * 64u + t.l], v); }
#endif  // OUZ_HOST
OUZ_DEV V3 ld3(const Tile& t, int f) { return v3(ld(t, f), ld(t, f + 1), ld(t, f + 2)); }
OUZ_DEV void st3(const Tile& t, int f, V3 v) { st(t, f, v.x); st(t, f + 1, v.y); st(t, f + 2, v.z); }

OUZ_DEV float2 traj_point(const StepArgs& a, int type, int idx, float sd) {
  int len = type == 0 ? kTrajLen[0] : (type == 1 ? kTrajLen[1] : kTrajLen[2]);
  int base = type == 0 ? kTrajBase[0] : (type == 1 ? kTrajBase[1] : kTrajBase[2]);
  idx = idx < len - 1 ? idx : len - 1;
  float2 p = a.wp_tab[base + idx];
  return make_float2(p.x * sd, p.y * sd);
}

// ---------------------------------------------------------------------------
// Register-resident state of one env for one task path.  load() reads what the path
// needs every step; fields that change only on reset / landing / episode end are
// tracked with dirty bits and written back only when they changed.
// ---------------------------------------------------------------------------
enum Dirty : uint32_t { D_DR = 1, D_FAULT = 2, D_TRAJ = 4, D_LAND = 8 };

template <int CTRL, int TGT>
struct EnvRegs {
  Tile T;                         // this env's tile in fstate / istate
  V3 p, v, w;
  Q4 q;
  int32_t progress;
  bool rst;                       // reset_buf != 0: lazy reset at the start of the next step
  bool flags_clear;               // reset_buf == 0 and time_outs == 0 in the buffers (emit may skip them)
  V3 target;                      // TGT_GOAL: stored random goal
  float thrust[4];                // CTRL_RL
  float4 act;                     // CTRL_RL: this step's action row, loaded with the state
  int32_t frot, fonset;           // fault
  float eta;
  float dr_m, dr_i, dr_t;         // domain randomisation scales
  int32_t rand_step;              // step of the last physical randomization (stored with the scales)
  V3 prev_v, wp;                  // CTRL_LEE_EST
  EkfQ eq;
  float eP[10], px[9], pP[45];
  float2 plat;                    // platform xy (TGT_TRAJ state; (0, 0) for TGT_PLATFORM)
  float2 plat_v;                  // this step's platform velocity (deck contact)
  int32_t ttype, tidx;            // TGT_TRAJ: trajectory type and waypoint index, scale * direction and
  float tsd, heading;             //   the husky's heading (landing.py:208-213), loaded with the state
  float2 wp_cur, wp_next;         //   waypoints tidx and tidx + 1, fetched at the start of the step
  int32_t land_flag;              // -1: not loaded (only needed on reset / landing)
  int32_t landings_add, ep_cnt_add, ep_len_add;
  float ep_ret, ep_sum_add;
  uint32_t dirty;
};

// One env's action row (vec_task.py:313: actions (N, 4) f32 on rl_device): a 16-byte load per lane.
// CLS: the slot layout is not env order (the mixed curriculum's class layout): the row of env e.
template <int CTRL, int TGT, bool CLS = false>
OUZ_DEV void load_actions(const float* actions, EnvRegs<CTRL, TGT>& S, int e = 0) {
  if constexpr (CTRL == CTRL_RL) {
    if constexpr (CLS) S.act = reinterpret_cast<const float4*>(actions)[e];
    else S.act = reinterpret_cast<const float4*>(actions + (size_t)S.T.first * OUZ_NUM_ACT)[S.T.l];
  }
}

// QLN: the quad-lane estimator (quad_pv_ql.h): the PV covariance goes to LDS (pv_lds_load), not to registers.
template <int CTRL, int TGT, bool CLS = false, bool NTL = false, bool QLN = false>
OUZ_DEV void env_load(const StepArgs& a, int i, const TaskParams& tp, EnvRegs<CTRL, TGT>& S,
                                         const float* actions) {
  // reset_buf and time_outs are read unconditionally and combined without a branch, so the two flag
  // loads and the state loads below are in flight together (one memory round trip, not three:
  // a short-circuit `!rst && timeouts == 0` made the time-out load wait for the reset load).
  // i: env index (the class layout's env-order buffers are not lane-contiguous)
  const int64_t rv = CLS ? a.rst_in[i] : (a.rst_in + S.T.first)[S.T.l];
  const uint32_t tv = CLS ? a.to_in[i] : (a.to_in + S.T.first)[S.T.l];
  // NTL: non-temporal state loads (large N: see nt_loads_default)
  const auto L = [&](int f) -> float { return NTL ? ld_nt(S.T, f) : ld(S.T, f); };
  const auto LI = [&](int f) -> int32_t { return NTL ? ldi_nt(S.T, f) : ldi(S.T, f); };
  const auto L3 = [&](int f) -> V3 { return v3(L(f), L(f + 1), L(f + 2)); };
  S.p = L3(OUZ_F_P);
  S.q = Q4{L(OUZ_F_Q), L(OUZ_F_Q + 1), L(OUZ_F_Q + 2), L(OUZ_F_Q + 3)};
  S.v = L3(OUZ_F_V);
  S.w = L3(OUZ_F_W);
  S.progress = LI(OUZ_I_PROGRESS);
  S.dirty = 0;
  // The landing flag is only needed on reset.  In the latency regime (few waves per CU: the step is
  // one dependent chain, load -> compute -> store) it is fetched with the state so the reset branch,
  // taken by most waves once episodes desynchronise, does not wait on a second memory round trip.
  // At large N that 4-byte load would be bandwidth; there the reset branch fetches it on demand.
  S.land_flag = a.n <= kLatencyRegimeEnvs ? LI(OUZ_I_LAND_FLAG) : -1;
  S.landings_add = 0;
  S.ep_cnt_add = 0;
  S.ep_len_add = 0;
  S.ep_sum_add = 0.0f;
  S.ep_ret = a.track_episodes ? L(OUZ_F_EP_RET) : 0.0f;
  S.dr_m = S.dr_i = S.dr_t = 1.0f;
  if (tp.dr) { S.dr_m = L(OUZ_F_DR); S.dr_i = L(OUZ_F_DR + 1); S.dr_t = L(OUZ_F_DR + 2); }
  if constexpr (TGT == TGT_GOAL) S.target = L3(OUZ_F_TARGET);
  if constexpr (CTRL == CTRL_RL) {
#pragma unroll
    for (int k = 0; k < 4; ++k) S.thrust[k] = L(OUZ_F_THRUST + k);
    S.frot = -1; S.fonset = 0; S.eta = 1.0f;
    if (tp.fault) { S.frot = LI(OUZ_I_FAULT_ROTOR); S.fonset = LI(OUZ_I_FAULT_ONSET); S.eta = L(OUZ_F_FAULT_ETA); }
    // in flight with the state loads: issued inside the step it would be a second memory round trip
    // behind the reset branch (every wave's critical path, and half the bytes in flight at large N)
    load_actions<CTRL, TGT, CLS>(actions, S, i);
  }
  if constexpr (CTRL == CTRL_LEE_EST) {
    S.prev_v = L3(OUZ_F_PREV_V);
    S.wp = L3(OUZ_F_WAYPOINT);
    S.eq = EkfQ{L(OUZ_F_EKF_Q), L(OUZ_F_EKF_Q + 1), L(OUZ_F_EKF_Q + 2), L(OUZ_F_EKF_Q + 3)};
#pragma unroll
    for (int k = 0; k < 10; ++k) S.eP[k] = L(OUZ_F_EKF_P + k);
#pragma unroll
    for (int k = 0; k < 9; ++k) S.px[k] = L(OUZ_F_PV_X + k);
    if constexpr (!QLN) {
#pragma unroll
      for (int k = 0; k < 45; ++k) S.pP[k] = L(OUZ_F_PV_P + k);
    }
  }
  if constexpr (TGT == TGT_TRAJ) {
    S.plat = make_float2(L(OUZ_F_PLAT), L(OUZ_F_PLAT + 1));
    S.ttype = LI(OUZ_I_TRAJ_TYPE); S.tidx = LI(OUZ_I_TRAJ_IDX);
    S.tsd = L(OUZ_F_TRAJ_SD); S.heading = L(OUZ_F_PLAT_HEADING);

  } else {
    S.plat = make_float2(0.0f, 0.0f);
  }
  S.plat_v = make_float2(0.0f, 0.0f);
  // The flags are used last: a use right after their loads made the compiler wait for every load issued so
  // far and issue the conditional loads above (DR scales, landing flag) in a second memory round trip.
  S.rst = rv != 0;
  // flags read from another buffer than the outputs (streamed rollout): the outputs are always written
  S.flags_clear = (rv == 0) & (tv == 0u) & (a.rst_in == a.reset);
}

// EPW: this wave owns the episode-tracking fields (false for the state wave of a rollout with an output wave)
template <int CTRL, int TGT, bool QLN = false, bool EPW = true>
OUZ_DEV void env_store(const StepArgs& a, int i, const TaskParams& tp, const EnvRegs<CTRL, TGT>& S) {
  st3(S.T, OUZ_F_P, S.p);
  st(S.T, OUZ_F_Q, S.q.x); st(S.T, OUZ_F_Q + 1, S.q.y); st(S.T, OUZ_F_Q + 2, S.q.z); st(S.T, OUZ_F_Q + 3, S.q.w);
  st3(S.T, OUZ_F_V, S.v);
  st3(S.T, OUZ_F_W, S.w);
  sti(S.T, OUZ_I_PROGRESS, S.progress);
  if (EPW && a.track_episodes) {
    st(S.T, OUZ_F_EP_RET, S.ep_ret);
    // accumulators: one lane owns each address, so a no-return atomic add is the same f32 / i32
    // read-add-write without a load round trip before the wave can retire
    if (S.ep_cnt_add) {
      OUZ_ACC_ADD(&S.T.f[(uint32_t)OUZ_F_EP_SUM * 64u + S.T.l], S.ep_sum_add);
      OUZ_ACC_ADD(&S.T.iv[(uint32_t)OUZ_I_EP_CNT * 64u + S.T.l], S.ep_cnt_add);
      OUZ_ACC_ADD(&S.T.iv[(uint32_t)OUZ_I_EP_LEN * 64u + S.T.l], S.ep_len_add);
    }
  }
  if (S.landings_add) OUZ_ACC_ADD(&S.T.iv[(uint32_t)OUZ_I_LANDINGS * 64u + S.T.l], S.landings_add);
  if (S.dirty & D_LAND) sti(S.T, OUZ_I_LAND_FLAG, S.land_flag);
  if (S.dirty & D_DR) {
    st(S.T, OUZ_F_DR, S.dr_m); st(S.T, OUZ_F_DR + 1, S.dr_i); st(S.T, OUZ_F_DR + 2, S.dr_t);
    sti(S.T, OUZ_I_RAND_STEP, S.rand_step);
  }
  if constexpr (TGT == TGT_GOAL) st3(S.T, OUZ_F_TARGET, S.target);
  if constexpr (CTRL == CTRL_RL) {
#pragma unroll
    for (int k = 0; k < 4; ++k) st(S.T, OUZ_F_THRUST + k, S.thrust[k]);
    if (S.dirty & D_FAULT) { sti(S.T, OUZ_I_FAULT_ROTOR, S.frot); sti(S.T, OUZ_I_FAULT_ONSET, S.fonset); st(S.T, OUZ_F_FAULT_ETA, S.eta); }
  }
  if constexpr (CTRL == CTRL_LEE_EST) {
    st3(S.T, OUZ_F_PREV_V, S.prev_v);
    st3(S.T, OUZ_F_WAYPOINT, S.wp);
    st(S.T, OUZ_F_EKF_Q, S.eq.w); st(S.T, OUZ_F_EKF_Q + 1, S.eq.x); st(S.T, OUZ_F_EKF_Q + 2, S.eq.y); st(S.T, OUZ_F_EKF_Q + 3, S.eq.z);
#pragma unroll
    for (int k = 0; k < 10; ++k) st(S.T, OUZ_F_EKF_P + k, S.eP[k]);
#pragma unroll
    for (int k = 0; k < 9; ++k) st(S.T, OUZ_F_PV_X + k, S.px[k]);
    if constexpr (!QLN) {
#pragma unroll
      for (int k = 0; k < 45; ++k) st(S.T, OUZ_F_PV_P + k, S.pP[k]);
    }
  }
  if constexpr (TGT == TGT_TRAJ) {
    st(S.T, OUZ_F_PLAT, S.plat.x); st(S.T, OUZ_F_PLAT + 1, S.plat.y);
    sti(S.T, OUZ_I_TRAJ_IDX, S.tidx); st(S.T, OUZ_F_PLAT_HEADING, S.heading);
    if (S.dirty & D_TRAJ) { sti(S.T, OUZ_I_TRAJ_TYPE, S.ttype); st(S.T, OUZ_F_TRAJ_SD, S.tsd); }
  }
}

// Waypoints tidx and tidx + 1 of the env's trajectory (table reads), issued at the start of the step
// so that their latency hides behind the estimator; platform_step picks one of them.
template <int CTRL, int TGT>
OUZ_DEV void platform_prefetch(const StepArgs& a, EnvRegs<CTRL, TGT>& S) {
  if constexpr (TGT == TGT_TRAJ) {
    S.wp_cur = traj_point(a, S.ttype, S.tidx, S.tsd);
    S.wp_next = traj_point(a, S.ttype, S.tidx + 1, S.tsd);   // clamped to the last waypoint
  }
}

// The husky following its waypoints (landing.py:319-364) as a kinematic differential-drive unicycle
// (oracle OracleEnv._platform_step).  Runs right before the integrator: nothing earlier in the step
// reads the platform (the target comes from the previous step's position).  The trajectory state is
// loaded with the env state and the two candidate waypoints at the start of the step, so the only
// memory access left here is the first waypoint of a freshly drawn trajectory.
template <int CTRL, int TGT>
OUZ_DEV void platform_step(const StepArgs& a, const StepCtx& sc, uint32_t gid,
                                              EnvRegs<CTRL, TGT>& S) {
  const EnvConsts& c = a.c;
  float2 wpp = S.wp_cur;
  float dx = wpp.x - S.plat.x, dy = wpp.y - S.plat.y;
  if (sqrtf(dx * dx + dy * dy) < 0.2f) { S.tidx += 1; wpp = S.wp_next; }
  const int len = S.ttype == 0 ? kTrajLen[0] : (S.ttype == 1 ? kTrajLen[1] : kTrajLen[2]);
  if (S.tidx >= len) {   // reset_completed_trajectories (landing.py:215-235)
    U4 r = draw(a.seed, gid, sc.step, RNG_TRAJ);
    S.ttype = (int)(r.x % 3u);
    S.tsd = (r.z & 1u) ? uniform_f32(r.y, 0.8f, 1.2f) : -uniform_f32(r.y, 0.8f, 1.2f);
    S.tidx = 0;
    S.dirty |= D_TRAJ;
    wpp = traj_point(a, S.ttype, 0, S.tsd);
  }
  // differential_drive (utils/controllers.py:15-43, gains (3, 1000) landing.py:361) on a
  // kinematic unicycle; wheel speeds saturate at plat_speed / wheel radius (15 rad/s)
  dx = wpp.x - S.plat.x; dy = wpp.y - S.plat.y;
  float th = S.heading;
  float dth = map_to_pi(atan2f(dy, dx) - map_to_pi(th));
  if (fabsf(dth) < kDriveAngThresh) dth = 0.0f;
  float lin = sqrtf(dx * dx + dy * dy) * kDriveGainLin, ang = dth * kDriveGainAng;
  const float wl = (2.0f * lin + ang * kWheelBase) / (2.0f * kWheelRadius);
  const float wr = (2.0f * lin - ang * kWheelBase) / (2.0f * kWheelRadius);
  const float mx = fmaxf(fabsf(wl), fabsf(wr)), max_w = c.plat_speed / kWheelRadius;
  if (mx > max_w) { const float scl = max_w / mx; lin *= scl; ang *= scl; }
  th = map_to_pi(th + ang * c.dt);
  float sn, cs;
  sincosf(th, &sn, &cs);
  S.plat_v = make_float2(lin * cs, lin * sn);
  S.plat.x += S.plat_v.x * c.dt; S.plat.y += S.plat_v.y * c.dt;
  S.heading = th;
}

// compute_observations + compute_ingenuity_reward of the post-step state (ekf_lee_landed.py:653-723,
// vec_task.py:351-353): one body for the one-wave step and the output wave (out_wave).
OUZ_DEV void obs_reward(const StepArgs& a, const StepCtx& sc, const TaskParams& tp, int task,
                                           uint32_t gid, V3 p, Q4 q, V3 v, V3 w, V3 target, float* ob, float& rew,
                                           float& dist) {
  ob[0] = (target.x - p.x) / 3.0f; ob[1] = (target.y - p.y) / 3.0f; ob[2] = (target.z - p.z) / 3.0f;
  ob[3] = q.x; ob[4] = q.y; ob[5] = q.z; ob[6] = q.w;
  ob[7] = v.x * 0.5f; ob[8] = v.y * 0.5f; ob[9] = v.z * 0.5f;
  ob[10] = w.x / kPiF; ob[11] = w.y / kPiF; ob[12] = w.z / kPiF;
  pomdp_apply<13>(ob, tp, task, a, sc, gid, SITE_OBS, false);
  if (a.drn_mask & 1) dr_noise_apply<13>(ob, a.drn[0], a.seed, gid, sc.step, RNG_DRN_OBS);   // vec_task.py:351-352
#pragma unroll
  for (int k = 0; k < 13; ++k) ob[k] = fminf(fmaxf(ob[k], -5.0f), 5.0f);   // vec_task.py:353
  rew = reward(p, target, q, w, dist);
}

// ---------------------------------------------------------------------------
// One VecTask.step of one env on register state (mirrors oracle/quad_oracle.py::OracleEnv.step)
// ---------------------------------------------------------------------------
// PRE: pre_physics_step only (ouz_pre_physics) -- stop before the integrator and write the body wrench
// [6] (force, torque; body frame at the COM) that gym.simulate would integrate to `wrench`.
// QLN: the quad-lane estimator (four lanes per env, the PV covariance in LDS at `ql`).
// SPW: the state wave of the split-wave estimator (quad_pv_split.h): the covariance is the other wave's.
// OWV: a rollout with an output wave: the step stops at the done decision; the output wave forms the
// observation, reward and episode statistics from the post-step state (out_wave), so `ob` / `rew` are not
// written here and the step's target goes to *post_target.
template <int CTRL, int TGT, bool PRE = false, bool QLN = false, bool SPW = false, bool OWV = false>
OUZ_DEV void env_core(const StepArgs& a, const StepCtx& sc, int i, uint32_t gid, int task,
                                         EnvRegs<CTRL, TGT>& S, float* ob, float& rew, bool& rs, bool& timeout,
                                         float* wrench = nullptr, const PvQl* ql = nullptr,
                                         const SplitLane* spl = nullptr, V3* post_target = nullptr) {
  const TaskParams& tp = a.tp[tp_slot(task)];
  const EnvConsts& c = a.c;
  const bool rst = S.rst;
  // target_root_positions: random goals are state (ouzelum.py:180-190); a platform target is
  // platform xy + offset at z 0.377 (ekf_lee_landed.py:87,628-629), recomputed rather than stored.
  // Before the first post_physics_step it is still (0, 0, 0.377).
  V3 target;
  if constexpr (TGT == TGT_GOAL) target = S.target;
  else target = sc.step == 0 ? v3(0.0f, 0.0f, 0.377f) : v3(S.plat.x + tp.plat_off_x, S.plat.y, 0.377f);

  // ---- lazy reset (ekf_lee_landed.py:271-306,312-335; ouzelum.py:192-233) ----
  if (rst) {
    U4 r = draw(a.seed, gid, sc.step, RNG_RESET_POS);
    S.p = v3(uniform_f32(r.x, -1.5f, 1.5f), uniform_f32(r.y, -1.5f, 1.5f), __fadd_rn(1.0f, uniform_f32(r.z, -0.2f, 1.5f)));
    S.q = Q4{0.0f, 0.0f, 0.0f, 1.0f};
    S.v = v3(0.0f, 0.0f, 0.0f);
    S.w = v3(0.0f, 0.0f, 0.0f);
    S.progress = 0;
    if (S.land_flag < 0) S.land_flag = ldi(S.T, OUZ_I_LAND_FLAG);   // landing counter (ekf_lee_landed.py:323-331)
    if (S.land_flag) { S.landings_add += S.land_flag; S.land_flag = 0; S.dirty |= D_LAND; }
    if (tp.dr) {
      // VecTask.apply_randomizations at reset (vec_task.py:547-563): the envs in the reset buffer whose
      // randomize_buf = step - OUZ_I_RAND_STEP >= frequency, and every env on its first randomization.  With
      // frequency <= 1 and no setup_only parameter every reset is due (an env resets at most once per step), so
      // the last step is read only otherwise.
      const PhysDr& pd = a.pdr;
      const int32_t last = pd.need_last ? ldi(S.T, OUZ_I_RAND_STEP) : -1;
      const bool first = last < 0;
      if (first || (int64_t)sc.step - (int64_t)last >= (int64_t)pd.p.frequency) {
        const U4 d = draw(a.seed, gid, sc.step, RNG_DR);
        U4 e{0u, 0u, 0u, 0u};
        if (pd.gauss) e = draw(cold_seed(a.seed), gid, sc.step, RNG_DR, 1u);
        const ouz_dr_param& pm = pd.p.param[OUZ_DRP_MASS];
        const ouz_dr_param& pi = pd.p.param[OUZ_DRP_INERTIA];
        const ouz_dr_param& pt = pd.p.param[OUZ_DRP_MOTOR_CONSTANT];
        if (pm.distribution && (first || !pm.setup_only)) S.dr_m = dr_scale(pm, dr_sample(pm, d.x, e.x, sc.step), c.mass);
        if (pi.distribution && (first || !pi.setup_only)) S.dr_i = dr_scale(pi, dr_sample(pi, d.y, e.y, sc.step), c.ixx);
        if (pt.distribution && (first || !pt.setup_only))
          S.dr_t = dr_scale(pt, dr_sample(pt, d.z, e.z, sc.step), kMotorConstant);
        S.rand_step = (int32_t)sc.step;
        S.dirty |= D_DR;
      }
    }
    if constexpr (CTRL == CTRL_RL) {
      if (tp.fault) {
        U4 d = draw(a.seed, gid, sc.step, RNG_FAULT);
        S.frot = (int32_t)(d.x >> 30);
        S.eta = uniform_f32(d.y, 0.0f, c.fault_eta_hi);
        S.fonset = (int32_t)(d.z % (uint32_t)(tp.max_ep / 2 + 1));
        S.dirty |= D_FAULT;
      }
    }
  }

  OUZ_STAMP(2, false);
  platform_prefetch<CTRL, TGT>(a, S);
  V3 f_b = v3(0.0f, 0.0f, 0.0f), tau_b = v3(0.0f, 0.0f, 0.0f);
  M3 R0;   // quat_to_mat of the (post-reset) state quaternion: shared by the controller and the integrator

  if constexpr (CTRL == CTRL_RL) {
    // ---- RL per-rotor thrust model (ouzelum.py:218-251) ----
    if constexpr (TGT == TGT_GOAL) {
      if ((S.progress % 500) == 0 || rst) {   // set_targets (ouzelum.py:180-190)
        U4 r = draw(a.seed, gid, sc.step, RNG_TARGET);
        target = v3(__fsub_rn(__fmul_rn(unit_f32(r.x), 10.0f), 5.0f), __fsub_rn(__fmul_rn(unit_f32(r.y), 10.0f), 5.0f),
                    __fadd_rn(unit_f32(r.z), 1.0f));
      }
    }
    float av[4] = {S.act.x, S.act.y, S.act.z, S.act.w};
    if (a.drn_mask & 2) dr_noise_apply<4>(av, a.drn[1], a.seed, gid, sc.step, RNG_DRN_ACT);   // vec_task.py:323-325
    float eff[4];
    const bool on = tp.fault && S.progress >= S.fonset;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float ak = fminf(fmaxf(av[k], -1.0f), 1.0f);                 // vec_task.py:327
      float th = S.thrust[k] + c.thrust_step * ak;
      th = fminf(fmaxf(th, 0.0f), c.thrust_max);                   // tensor_clamp
      eff[k] = (on && S.frot == k) ? th * S.eta : th;
      if (rst) { th = 0.0f; eff[k] = 0.0f; }                        // thrusts/forces[reset] = 0
      S.thrust[k] = th;
    }
    if (tp.dr) {   // the rotors' motorConstant scale (ouz_dr_physical OUZ_DRP_MOTOR_CONSTANT)
#pragma unroll
      for (int k = 0; k < 4; ++k) eff[k] *= S.dr_t;
    }
    float tot = 0.0f, tx = 0.0f, ty = 0.0f, tz = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      tot += eff[k];
      tx += eff[k] * kRotorY[k];
      ty -= eff[k] * kRotorX[k];
      tz -= eff[k] * (kMotorKm * kRotorDir[k]);
    }
    f_b = v3(0.0f, 0.0f, tot);
    tau_b = v3(tx, ty, tp.motor_yaw ? tz : 0.0f);
  } else if constexpr (CTRL == CTRL_LEE_TRUE) {
    // ---- Lee on true state, hover at (0,0,1) (lee_landed.py:263-330) ----
    float T;
    V3 tau;
    const V3 cmd = v3(0.0f, 0.0f, 1.0f);
    R0 = quat_to_mat(S.q);
    lee_position_R(R0, S.p, S.v, S.w, cmd, 0.0f, default_gains(), T, tau);
    float fz = 2.0f * kGravity * T;
    V3 dd = cmd - S.p;
    if (sqrtf(dot(dd, dd)) < tp.land_radius) {
      S.land_flag = 1;
      S.dirty |= D_LAND;
      fz = 0.0f;
      tau = v3(0.0f, 0.0f, 0.0f);
    }
    if (rst) fz = 0.0f;                        // forces[reset] = 0, torques kept
    f_b = v3(0.0f, 0.0f, fz * S.dr_t);
    tau_b = tau;
  } else {
    // ---- AHRS-EKF + PV-KF + waypoint guidance + Lee (ekf_lee_landed.py:308-530) ----
    const bool conv = sc.step < (uint32_t)c.conv_time;
    V3 lin_acc = v3((S.v.x - S.prev_v.x) / c.dt, (S.v.y - S.prev_v.y) / c.dt, (S.v.z - S.prev_v.z) / c.dt);
    lin_acc.z += 9.8f;                                 // aliasing quirk (ekf_lee_landed.py:366-367)
    EkfQ qt{S.q.w, S.q.x, S.q.y, S.q.z};
    if (conv || rst) S.eq = qt;                        // :349-353
    if (rst) {                                         // :355-360
      S.px[0] = S.p.x; S.px[1] = S.p.y; S.px[2] = S.p.z; S.px[3] = S.v.x; S.px[4] = S.v.y; S.px[5] = S.v.z;
      S.px[6] = S.px[7] = S.px[8] = 0.0f;
    }
    float gyr[3] = {S.w.x, S.w.y, S.w.z};
    float ang[4] = {qt.w, qt.x, qt.y, qt.z};
    if (!conv) {
      pomdp_apply<3>(gyr, tp, task, a, sc, gid, SITE_GYR, false);
      pomdp_apply<4>(ang, tp, task, a, sc, gid, SITE_ANG, true);
    }
    {
      float inv = 1.0f / sqrtf(S.eq.w * S.eq.w + S.eq.x * S.eq.x + S.eq.y * S.eq.y + S.eq.z * S.eq.z);
      S.eq = EkfQ{S.eq.w * inv, S.eq.x * inv, S.eq.y * inv, S.eq.z * inv};
    }
    OUZ_STAMP(10, false);
    ekf_update(S.eq, S.eP, v3(gyr[0], gyr[1], gyr[2]), EkfQ{ang[0], ang[1], ang[2], ang[3]}, c.dt);
    OUZ_STAMP(11, false);
    // SPW: the covariance wave starts this step's predict as soon as the attitude is known
    if constexpr (SPW) pv_split_publish(*spl, conv ? qt : S.eq);
    EkfQ orient = S.eq;
    float pm[3] = {S.p.x, S.p.y, S.p.z}, vm[3] = {S.v.x, S.v.y, S.v.z}, am[3] = {lin_acc.x, lin_acc.y, lin_acc.z};
    if (conv) {
      orient = qt;
    } else {
      pomdp_apply<3>(am, tp, task, a, sc, gid, SITE_ACC, false);
      pomdp_apply<3>(pm, tp, task, a, sc, gid, SITE_POS, false);
      pomdp_apply<3>(vm, tp, task, a, sc, gid, SITE_VEL, false);
    }
    if constexpr (SPW) OUZ_STAMP(5, false);
    // predict, position fix, velocity fix with R = 0 (PVFilter.py:76-79); shared trigger counters (:425-440)
    const uint64_t g = (uint64_t)sc.step * a.n_total + gid;
    PvReal xd[9];   // SPW: the state estimate in f64 between its predict and the gains of this step's fixes
    if constexpr (SPW) {
      // The state wave: the state predict; the fixes wait for the covariance wave's gains after the guidance, the
      // rotation and the husky's step (none of which reads the estimate), right before the controller that does.
      // (Every form contracts only within an expression, -ffp-contract=on in build.py, so the split, quad-lane
      // and one-lane forms round alike without the LDS round trip of the one-lane form's parking.)
      pv_split_predict(S.px, v3(am[0], am[1], am[2]), orient, c.dt, xd);
      OUZ_STAMP(12, false);
    } else if constexpr (QLN) {
      // The covariance is in LDS and split over the env's lanes: no register peak to park around.
      pv_step_ql(*ql, S.px, v3(am[0], am[1], am[2]), orient, c.dt, g % 7u == 6u, v3(pm[0], pm[1], pm[2]),
                 g % 3u == 0u, v3(vm[0], vm[1], vm[2]));
      OUZ_STAMP(12, false);
    } else {
#ifdef OUZ_HOST
      pv_step(S.px, S.pP, v3(am[0], am[1], am[2]), orient, c.dt, g % 7u == 6u, v3(pm[0], pm[1], pm[2]),
              g % 3u == 0u, v3(vm[0], vm[1], vm[2]));
#else
      // The float64 PV step is the register peak of the estimator kernels.  Everything the env holds
      // that the step does not read (true state, target, waypoint, platform, DR scales) is parked in
      // LDS around it (lane-contiguous slots: conflict-free) so those registers are free at the peak
      // (QuadTracking 270 -> fits 256: two waves per SIMD without scratch spills).
      constexpr int kPark = 24;
      __shared__ float s_park[kPark * kMaxBlock];
      float* pk = s_park + threadIdx.x;
      float vals[kPark] = {S.p.x, S.p.y, S.p.z, S.v.x, S.v.y, S.v.z, S.w.x, S.w.y, S.w.z, S.q.x, S.q.y, S.q.z,
                           S.q.w, target.x, target.y, target.z, S.wp.x, S.wp.y, S.wp.z, S.plat.x, S.plat.y,
                           S.dr_m, S.dr_i, S.dr_t};
#pragma unroll
      for (int k = 0; k < kPark; ++k) pk[k * kMaxBlock] = vals[k];
      __asm__ volatile("" ::: "memory");   // no store-to-load forwarding: the registers die here
      pv_step(S.px, S.pP, v3(am[0], am[1], am[2]), orient, c.dt, g % 7u == 6u, v3(pm[0], pm[1], pm[2]),
              g % 3u == 0u, v3(vm[0], vm[1], vm[2]));
      __asm__ volatile("" ::: "memory");
      OUZ_STAMP(12, false);
#pragma unroll
      for (int k = 0; k < kPark; ++k) vals[k] = pk[k * kMaxBlock];
      S.p = v3(vals[0], vals[1], vals[2]); S.v = v3(vals[3], vals[4], vals[5]); S.w = v3(vals[6], vals[7], vals[8]);
      S.q = Q4{vals[9], vals[10], vals[11], vals[12]};
      target = v3(vals[13], vals[14], vals[15]);
      S.wp = v3(vals[16], vals[17], vals[18]);
      S.plat = make_float2(vals[19], vals[20]);
      S.dr_m = vals[21]; S.dr_i = vals[22]; S.dr_t = vals[23];
#endif
    }
    S.prev_v = S.v;                                    // :454
    // waypoint guidance (:464-492)
    V3 wp = conv ? target : S.wp;
    V3 tv = target - S.p;
    float td = sqrtf(dot(tv, tv));
    if (!conv) {
      V3 wv = wp - S.p;
      float wd = sqrtf(dot(wv, wv));
      if (wd < 0.5f || wd > 1.0f) {
        V3 vec = (target + v3(0.0f, 0.0f, 0.7f)) - S.p;
        float nv = sqrtf(dot(vec, vec));
        wp = v3(vec.x / nv * 0.75f + S.p.x, vec.y / nv * 0.75f + S.p.y, vec.z / nv * 0.75f + S.p.z);
      }
      if (td < 0.75f) wp = target + v3(0.0f, 0.0f, 0.09f);
    }
    S.wp = wp;
    float T;
    V3 tau;
    R0 = quat_to_mat(S.q);   // after the PV step's register peak
    if constexpr (SPW) {
      if constexpr (TGT == TGT_TRAJ) platform_step<CTRL, TGT>(a, sc, gid, S);   // (not in the physics block below)
      OUZ_STAMP(6, false);
      pv_split_correct(*spl, xd, S.px, g % 7u == 6u, v3(pm[0], pm[1], pm[2]), g % 3u == 0u, v3(vm[0], vm[1], vm[2]));
    }
    if (conv) lee_position_R(R0, S.p, S.v, S.w, wp, 0.0f, default_gains(), T, tau);
    else lee_position_R(R0, v3(S.px[0], S.px[1], S.px[2]), v3(S.px[3], S.px[4], S.px[5]), S.w, wp, 0.0f, default_gains(), T, tau);
    float fz = 2.0f * kGravity * T;
    if (td < tp.land_radius) {                       // :508-515
      if (!conv) { S.land_flag = 1; S.dirty |= D_LAND; }
      fz = 0.0f;
      tau = v3(0.0f, 0.0f, 0.0f);
    }
    if (rst) fz = 0.0f;                              // :521
    if (conv) { fz = 2.09f * kGravity; tau = v3(0.0f, 0.0f, 0.0f); }   // :526-530
    f_b = v3(0.0f, 0.0f, fz * S.dr_t);
    tau_b = tau;
  }

  if constexpr (PRE) {
    float* wr = wrench + (size_t)i * 6;
    wr[0] = f_b.x; wr[1] = f_b.y; wr[2] = f_b.z;
    wr[3] = tau_b.x; wr[4] = tau_b.y; wr[5] = tau_b.z;
    return;
  }
  OUZ_STAMP(3, false);
  // ---- physics: gym.simulate -> lumped rigid body, c.substeps sub-steps ----
  {
    // additive inertia DR adds the same sample to each diagonal entry: the zz scale follows from the xx scale
    const float dr_iz = a.pdr.inertia_add ? 1.0f + (S.dr_i - 1.0f) * (c.ixx * c.inv_izz) : S.dr_i;
    const V3 I = v3(c.ixx * S.dr_i, c.iyy * S.dr_i, c.izz * dr_iz);
    const float inv_m = tp.dr ? 1.0f / (c.mass * S.dr_m) : c.inv_mass;
    const V3 inv_I = tp.dr ? v3(1.0f / I.x, 1.0f / I.y, 1.0f / I.z) : v3(c.inv_ixx, c.inv_iyy, c.inv_izz);
    if constexpr (TGT == TGT_TRAJ && !SPW) platform_step<CTRL, TGT>(a, sc, gid, S);
    if constexpr (CTRL == CTRL_RL) R0 = quat_to_mat(S.q);
    const DeckContact deck{TGT != TGT_GOAL, S.plat.x, S.plat.y, S.plat_v.x, S.plat_v.y};
    const float h = c.dt / (float)c.substeps;
    // sim_params gravity (gym.set_sim_params after apply_randomizations, vec_task.py:648-660): nominal unless DR'd
    const V3 grav = (a.drn_mask & 4) ? gravity_dr(grav_dr_of(a.drn), a.seed, sc.step) : v3(0.0f, 0.0f, -kGravity);
    if (c.substeps == 2)   // the configured sub-step count (EKFLeeLanded.yaml:29), unrolled
      integrate_thrust_body<2>(S.p, S.q, S.v, S.w, R0, f_b.z, tau_b, inv_m, I, inv_I, h, c.wmax, deck, grav);
    else
      integrate_thrust_body<0>(S.p, S.q, S.v, S.w, R0, f_b.z, tau_b, inv_m, I, inv_I, h, c.wmax, deck, grav,
                               c.substeps);
  }

  OUZ_STAMP(4, false);
  // ---- post_physics_step (ekf_lee_landed.py:620-685) ----
  S.progress += 1;
  if constexpr (TGT == TGT_GOAL) {
    S.target = target;
  } else {
    target.x = S.plat.x + tp.plat_off_x;
    target.y = S.plat.y;
    target.z = 0.377f;
  }
  // (the output wave, out_wave, forms the observation / reward from these values read back from LDS: with
  // contraction only within expressions both forms round alike)
  const V3 p = S.p, v = S.v, w = S.w;
  const Q4 q = S.q;
  float dist;
  if constexpr (OWV) {
    dist = target_dist(p, target);
    *post_target = target;
  } else {
    obs_reward(a, sc, tp, task, gid, p, q, v, w, target, ob, rew, dist);
  }
  const bool timeout_len = S.progress >= tp.max_ep - 1;
  const bool die = dist > 8.0f || p.z < tp.z_die;
  rs = timeout_len || die;
  timeout = timeout_len && rs;                                             // vec_task.py:345
  if constexpr (!OWV) {
    if (a.track_episodes) {   // RecordEpisodeStatisticsTorch.step (PPO/utils.py:20-35), summed on device
      S.ep_ret += rew;
      if (rs) { S.ep_sum_add += S.ep_ret; S.ep_cnt_add += 1; S.ep_len_add += S.progress; S.ep_ret = 0.0f; }
    }
  }
  S.rst = rs;
  if (!OWV && a.trace_cap > 0 && i == a.trace_env) {   // trajectory CSV row (ekf_lee_landed.py:667-674)
    float* t = a.trace + (size_t)(sc.step % (uint32_t)a.trace_cap) * 9;
    t[0] = p.x; t[1] = p.y; t[2] = p.z;
    t[3] = target.x; t[4] = target.y; t[5] = target.z;
    t[6] = v.x; t[7] = v.y; t[8] = v.z;
  }
}

// ---------------------------------------------------------------------------
// Host side, shared by both builds: configuration checks, the env constants and task parameters of StepArgs,
// the waypoint tables and the whole-batch flicker coins.
// ---------------------------------------------------------------------------
// nullptr if the configuration is valid, else what is wrong with it
inline const char* config_error(const ouz_config* cfg) {
  if (cfg->task < 0 || cfg->task >= OUZ_NUM_TASKS) return "unknown task";
  if (cfg->num_envs <= 0) return "num_envs must be > 0";
  if (cfg->substeps <= 0 || !(cfg->dt > 0.0f)) return "bad dt/substeps";
  if (cfg->max_episode_length < 0) return "max_episode_length must be >= 0";
  const int64_t total = cfg->num_envs_total > 0 ? cfg->num_envs_total : cfg->num_envs;
  if (cfg->env_id_offset < 0 || cfg->env_id_offset + cfg->num_envs > total || total > 0xFFFFFFFFll)
    return "env ids out of range";
  return nullptr;
}

// The tasks an env object of task cfg_task steps (the mixed curriculum: its three).
inline bool task_used(int cfg_task, int t) {
  return cfg_task == OUZ_TASK_MIXED ? (t == OUZ_TASK_LEE_LANDED || t == OUZ_TASK_TRACKING || t == OUZ_TASK_FAULT)
                                    : t == cfg_task;
}

// nullptr if the physical DR parameters are valid, else what is wrong with them
inline const char* dr_physical_error(const ouz_dr_physical* p) {
  if (p->frequency < 0) return "frequency must be >= 0";
  for (int k = 0; k < OUZ_DRP_COUNT; ++k) {
    const ouz_dr_param& q = p->param[k];
    if (q.distribution < 0 || q.distribution > 3 || q.operation < 0 || q.operation > 1 || q.schedule < 0 ||
        q.schedule > 2)
      return "bad distribution / operation / schedule";
    if (q.distribution == 0) continue;
    if (q.schedule != 0 && q.schedule_steps <= 0) return "a schedule needs schedule_steps > 0";
    if (q.distribution == 3 && !(q.range[0] > 0.0f && q.range[1] > 0.0f)) return "a loguniform range must be positive";
  }
  return nullptr;
}

// nullptr if the sim_params gravity DR parameters are valid, else what is wrong with them
inline const char* dr_gravity_error(const ouz_dr_param* p, int32_t frequency) {
  if (frequency < 0) return "frequency must be >= 0";
  if (p->distribution < 0 || p->distribution > 3 || p->operation < 0 || p->operation > 1 || p->schedule < 0 ||
      p->schedule > 2)
    return "bad distribution / operation / schedule";
  if (p->distribution && p->schedule != 0 && p->schedule_steps <= 0) return "a schedule needs schedule_steps > 0";
  if (p->distribution == 3 && !(p->range[0] > 0.0f && p->range[1] > 0.0f)) return "a loguniform range must be positive";
  return nullptr;
}

// The step's view of physical DR parameters (PhysDr).
inline PhysDr derive_phys_dr(const ouz_dr_physical& p) {
  PhysDr d;
  memset(&d, 0, sizeof(d));
  d.p = p;
  bool setup = false;
  for (int k = 0; k < OUZ_DRP_COUNT; ++k) {
    if (!p.param[k].distribution) continue;
    setup |= p.param[k].setup_only != 0;
    d.gauss |= p.param[k].distribution == 1 ? 1 : 0;
  }
  d.need_last = (p.frequency > 1 || setup) ? 1 : 0;
  d.inertia_add = (p.param[OUZ_DRP_INERTIA].distribution && p.param[OUZ_DRP_INERTIA].operation == 0) ? 1 : 0;
  return d;
}

// ouz_set_dr_physical: the parameters for every task of the env object (p == nullptr or nothing enabled: off).
inline void set_phys_dr(StepArgs& a, int cfg_task, const ouz_dr_physical* p) {
  bool on = false;
  if (p)
    for (int k = 0; k < OUZ_DRP_COUNT; ++k) on |= p->param[k].distribution != 0;
  if (on) a.pdr = derive_phys_dr(*p);
  else memset(&a.pdr, 0, sizeof(a.pdr));
  for (int t = 0; t < OUZ_NUM_TASKS; ++t)
    if (task_used(cfg_task, t)) a.tp[tp_slot(t)].dr = on ? 1 : 0;
}

// The task default (QuadTracking; BASELINE.json config C): mass, inertia and motor-constant scaling ~ U(dr_lo, dr_hi)
// at every reset, as a dr_params entry {range: [dr_lo, dr_hi], operation: scaling, distribution: uniform}.
inline ouz_dr_physical default_phys_dr(const ouz_config* cfg) {
  ouz_dr_physical p;
  memset(&p, 0, sizeof(p));
  p.frequency = 1;
  for (int k = 0; k < OUZ_DRP_COUNT; ++k) {
    p.param[k].distribution = 2;
    p.param[k].operation = 1;
    p.param[k].range[0] = cfg->dr_lo;
    p.param[k].range[1] = cfg->dr_hi;
  }
  return p;
}

// StepArgs from a (valid) configuration: sizes, slot layout, ids, seed, body constants, task parameters.  The
// buffer pointers, the waypoint table and the device-only kernel-form knobs are the caller's.
inline void fill_step_args(const ouz_config* cfg, StepArgs& a) {
  const int64_t total = cfg->num_envs_total > 0 ? cfg->num_envs_total : cfg->num_envs;
  memset(&a, 0, sizeof(a));
  a.n = cfg->num_envs;
  a.n_slots = state_slots(cfg->task, cfg->num_envs);
  a.cls = class_layout_rt(cfg->task, cfg->num_envs) ? (cfg->task == OUZ_TASK_MIXED ? 2 : 1) : 0;
  a.xcd_pack = (a.cls && cfg->num_envs > kLatencyRegimeEnvs) ? 1 : 0;
  a.env_offset = (uint32_t)cfg->env_id_offset;
  a.n_total = (uint64_t)total;
  a.seed = cfg->seed;
  a.track_episodes = cfg->track_episodes;
  a.pipe_stride = 0;
  a.trace_env = -1;
  // x500 lumped mass properties (assets/x500/x500.urdf:31-35,98-177)
  const double base_m = 2.0, rm = 0.016076923076923075;
  const double mass = base_m + 4 * rm;
  const double zc = 4 * rm * 0.3 / mass;
  const double r_avg = 0.5 * (3.8464910483993325e-07 + 2.6115851691700804e-05);
  double ixx = 0.02166666666666667 + base_m * zc * zc, izz = 0.04000000000000001;
  const double rx[4] = {0.174, -0.174, 0.174, -0.174}, ry[4] = {-0.174, 0.174, 0.174, -0.174};
  for (int k = 0; k < 4; ++k) {
    ixx += r_avg + rm * (ry[k] * ry[k] + (0.3 - zc) * (0.3 - zc));
    izz += 2.649858234714004e-05 + rm * (rx[k] * rx[k] + ry[k] * ry[k]);
  }
  a.c = EnvConsts{cfg->dt, (float)((double)cfg->dt * (double)cfg->thrust_rate), cfg->thrust_max, cfg->plat_speed,
                  cfg->dr_lo, cfg->dr_hi, cfg->fault_eta_hi, (float)(4.0 * 3.14159265358979323846),
                  cfg->substeps, cfg->convergence_time, (float)mass, (float)ixx, (float)ixx, (float)izz,
                  1.0f / (float)mass, 1.0f / (float)ixx, 1.0f / (float)ixx, 1.0f / (float)izz};
  bool preset_dr = false;
  for (int t = 0; t < OUZ_NUM_TASKS; ++t) {
    if (!task_used(cfg->task, t)) continue;
    TaskParams tp = task_preset(t);
    preset_dr |= tp.dr != 0;
    if (cfg->pomdp >= 0) tp.pomdp = cfg->pomdp;
    if (cfg->pomdp_prob >= 0.0f) tp.pomdp_prob = cfg->pomdp_prob;
    if (cfg->max_episode_length > 0) tp.max_ep = cfg->max_episode_length;
    double prob = (double)tp.pomdp_prob;
    tp.noise_lo = (float)(1.0 - prob);
    tp.noise_hi = (float)(1.0 + prob);
    a.tp[tp_slot(t)] = tp;
  }
  if (preset_dr) a.pdr = derive_phys_dr(default_phys_dr(cfg));   // the DR tasks' flags stay their presets'
}

// Waypoint tables of landing.py:108-112 (lemniscate(a=4,100), circle(r=2,100), square(4,8)),
// computed the way utils/trajectories.py:5-60 does (f32 theta for the lemniscate).
inline void build_waypoints(float2* tab) {
  const double pi = 3.14159265358979323846;
  for (int i = 0; i < 100; ++i) {
    // torch.linspace(-pi/2, 3pi/2, 100) in f32
    double step = (1.5 * pi - (-0.5 * pi)) / 99.0;
    float th = (i < 50) ? (float)(-0.5 * pi + step * i) : (float)(1.5 * pi - step * (99 - i));
    float s = sinf(th), c = cosf(th);
    tab[i] = make_float2(4.0f * c / (s * s + 1.0f), 4.0f * c * s / (s * s + 1.0f));
  }
  for (int i = 0; i < 100; ++i) {
    double ang = (i * (360.0 / 100.0)) * pi / 180.0;
    tab[100 + i] = make_float2((float)(2.0 * std::cos(ang)), (float)(2.0 * std::sin(ang)));
  }
  const float sq[4][2] = {{0, 0}, {4, 0}, {4, 4}, {0, 4}};
  for (int i = 0; i < 4; ++i) tab[200 + i] = make_float2(-(sq[i][0] - 2.0f), -(sq[i][1] - 2.0f));
}

// Whole-batch flicker coins (utils/POMDP.py:25: one torch.rand(1) per call) — identical for
// every env, so they are drawn once per step here instead of once per lane.
inline uint32_t flicker_mask(const StepArgs& a, int cfg_task, uint32_t step) {
  uint32_t m = 0;
  for (int t = 0; t < OUZ_NUM_TASKS; ++t) {
    if (!task_used(cfg_task, t)) continue;
    const TaskParams& tp = a.tp[tp_slot(t)];
    if (tp.pomdp != OUZ_POMDP_FLICKER && tp.pomdp != OUZ_POMDP_FLICKER_NOISE) continue;
    const float p = tp.pomdp == OUZ_POMDP_FLICKER ? tp.pomdp_prob : 0.1f;
    for (uint32_t site = 0; site < 6; ++site) {
      U4 r = draw(a.seed, BATCH_ENV, step, RNG_POMDP + site, (uint32_t)t);
      if (unit_f32(r.x) <= p) m |= 1u << (tp_slot(t) * 8 + site);
    }
  }
  return m;
}

}  // namespace ouz
