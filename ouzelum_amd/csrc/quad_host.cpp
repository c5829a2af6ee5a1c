// Host build of the quadrotor step (libouzelum_cpu.so): make(sim_device="cpu").
//
// The same per-env step as the HIP kernels -- quad_env.h's env_load / env_core / env_store and quad_math.h's
// controllers, estimator and integrator, compiled by g++ with -DOUZ_HOST -- over the same wave-tiled SoA state
// (include/ouzelum.h OUZ_FIDX, the same state slots), one env per loop iteration, the envs of a step split over
// OpenMP threads.  f32 storage and arithmetic like the kernels (the PV step in f64 registers, as there); no FMA
// contraction (-ffp-contract=off), so results agree with the GPU within the parity tolerances, not bitwise.
//
// This is the reference's CPU-device VecTask (tasks/base/vec_task.py:169-223 accepts sim_device="cpu": the same
// task on torch CPU tensors) and BASELINE.md §4.2's vectorised f32 CPU step.  It does not use the test oracle.
#define OUZ_HOST 1
#include "../../include/ouzelum_host.h"

#include <omp.h>

#include <string>

#include "quad_env.h"

using namespace ouz;

namespace {
thread_local std::string g_host_err;
int host_fail(int code, const std::string& msg) {
  g_host_err = msg;
  return code;
}
}  // namespace

struct ouz_host_env {
  ouz_config cfg;
  bool bound;
  int64_t step;
  int32_t threads;          // OpenMP threads of a step (0: the runtime's default)
  float2 wp_tab[204];       // waypoint tables (lemniscate | circle | square)
  DrNonEnv drn;             // VecTask DR noise ([0] observations, [1] actions) and sim_params gravity
  StepArgs a;
};

namespace {

// One env's VecTask.step on the host (the HIP kernel's run_env, K = 1): load, step, outputs by env index,
// store.  i: state slot, e: env index.
template <int CTRL, int TGT>
inline void host_env_step(const StepArgs& a, const StepCtx& sc, int i, int e, int task) {
  const TaskParams& tp = a.tp[tp_slot(task)];
  const uint32_t gid = a.env_offset + (uint32_t)e;
  EnvRegs<CTRL, TGT> S;
  S.T = tile_of(a, i);
  env_load<CTRL, TGT, /*CLS: env-order buffers by env index*/ true>(a, e, tp, S, sc.actions);
  const bool did_reset = S.rst, flags_clear = S.flags_clear;
  float ob[OUZ_NUM_OBS];
  float rew = 0.0f;
  bool rs = false, to = false;
  env_core<CTRL, TGT>(a, sc, e, gid, task, S, ob, rew, rs, to);
  if (a.trace_cap > 0) {   // per-step reset counts of the trajectory log (the kernel's trace_count)
    if (did_reset) __atomic_fetch_add(&a.trace_resets[sc.step % (uint32_t)a.trace_cap], 1u, __ATOMIC_RELAXED);
  }
  float* row = a.obs + (size_t)e * OUZ_NUM_OBS;
  for (int k = 0; k < OUZ_NUM_OBS; ++k) row[k] = ob[k];
  a.rew[e] = rew;
  if (!(flags_clear && !rs)) {
    a.reset[e] = rs ? 1 : 0;
    a.timeouts[e] = to ? 1 : 0;
  }
  env_store<CTRL, TGT>(a, i, tp, S);
}

inline void host_slot_step(const StepArgs& a, const StepCtx& sc, int cfg_task, int i) {
  int64_t e = i;
  if (a.cls == 2) e = mixed_slot_env(a.env_offset, i);
  else if (a.cls) e = slot_env(i);
  if (e < 0 || e >= a.n) return;   // idle / padding slot
  const int task = cfg_task == OUZ_TASK_MIXED ? mixed_task(a.env_offset + (uint32_t)e) : cfg_task;
  switch (task) {
    case OUZ_TASK_OUZELUM:
    case OUZ_TASK_FAULT: host_env_step<CTRL_RL, TGT_GOAL>(a, sc, i, (int)e, task); break;
    case OUZ_TASK_LEE_LANDED: host_env_step<CTRL_LEE_TRUE, TGT_PLATFORM>(a, sc, i, (int)e, task); break;
    case OUZ_TASK_LANDING: host_env_step<CTRL_RL, TGT_TRAJ>(a, sc, i, (int)e, task); break;
    case OUZ_TASK_EKF_LEE_LANDED: host_env_step<CTRL_LEE_EST, TGT_PLATFORM>(a, sc, i, (int)e, task); break;
    default: host_env_step<CTRL_LEE_EST, TGT_TRAJ>(a, sc, i, (int)e, task); break;   // QuadTracking
  }
}

// Creation-time state of one slot (the kernel's init_state_kernel).
inline void host_init_slot(const StepArgs& a, int cfg_task, int s) {
  for (int k = 0; k < OUZ_F_COUNT; ++k) st(a, k, s, 0.0f);
  for (int k = 0; k < OUZ_I_COUNT; ++k) sti(a, k, s, 0);
  const int64_t e = a.cls == 2 ? mixed_slot_env(a.env_offset, s) : (a.cls ? slot_env(s) : s);
  if (e < 0 || e >= a.n) return;
  const uint32_t gid = a.env_offset + (uint32_t)e;
  const int task = cfg_task == OUZ_TASK_MIXED ? mixed_task(gid) : cfg_task;
  const TaskParams& tp = a.tp[tp_slot(task)];
  st(a, OUZ_F_P + 2, s, 1.0f);           // default_pose.p.z = 1 (ekf_lee_landed.py:228-229)
  st(a, OUZ_F_Q + 3, s, 1.0f);
  st(a, OUZ_F_TARGET + 2, s, tp.target_mode == TGT_GOAL ? 1.0f : 0.377f);   // ouzelum.py:73, ekf_lee_landed.py:87
  for (int k = 0; k < 4; ++k) st(a, OUZ_F_EKF_P + s4(k, k), s, 1.0f);       // ahrs_ekf.py:997
  for (int k = 0; k < 9; ++k) st(a, OUZ_F_PV_P + s9(k, k), s, kPvP0);        // PVFilter.py:12
  st(a, OUZ_F_DR, s, 1.0f); st(a, OUZ_F_DR + 1, s, 1.0f); st(a, OUZ_F_DR + 2, s, 1.0f);
  sti(a, OUZ_I_RAND_STEP, s, -1);        // never randomized: the first reset is due (vec_task.py:555-557)
  st(a, OUZ_F_FAULT_ETA, s, 1.0f);
  if (tp.target_mode == TGT_TRAJ) {      // landing.py:209-213
    U4 r = draw(a.seed, gid, INIT_STEP, RNG_TRAJ);
    sti(a, OUZ_I_TRAJ_TYPE, s, (int)(r.x % 3u));
    st(a, OUZ_F_TRAJ_SD, s, (r.z & 1u) ? uniform_f32(r.y, 0.8f, 1.2f) : -uniform_f32(r.y, 0.8f, 1.2f));
  }
  for (int k = 0; k < OUZ_NUM_OBS; ++k) a.obs[(size_t)e * OUZ_NUM_OBS + k] = 0.0f;
  a.rew[e] = 0.0f;
  a.reset[e] = 1;                        // reset_buf starts at ones (vec_task.py:269-270)
  a.timeouts[e] = 0;
}

int host_threads(const ouz_host_env* env) { return env->threads > 0 ? env->threads : omp_get_max_threads(); }

bool host_needs_actions(int task) {
  return task == OUZ_TASK_OUZELUM || task == OUZ_TASK_FAULT || task == OUZ_TASK_MIXED || task == OUZ_TASK_LANDING;
}

int host_steps(ouz_host_env* env, const float* ring, int32_t ring_len, int32_t n_steps, const char* fn) {
  if (!env || !env->bound) return host_fail(OUZ_ERR_UNBOUND, std::string(fn) + ": env not bound");
  if (n_steps < 0 || (ring && ring_len <= 0)) return host_fail(OUZ_ERR_INVALID, std::string(fn) + ": bad sizes");
  if (!ring && host_needs_actions(env->cfg.task))
    return host_fail(OUZ_ERR_INVALID, std::string(fn) + ": this task needs actions");
  const StepArgs& a = env->a;
  const int n_slots = a.n_slots, task = env->cfg.task, nt = host_threads(env);
  for (int32_t k = 0; k < n_steps; ++k) {
    const uint32_t step = (uint32_t)env->step;
    const StepCtx sc{step, flicker_mask(a, task, step),
                     ring ? ring + (size_t)(k % ring_len) * (size_t)a.n * OUZ_NUM_ACT : nullptr};
    if (a.trace_cap > 0) a.trace_resets[step % (uint32_t)a.trace_cap] = 0u;
    // one state tile (64 slots) per scheduling unit, handed out dynamically: tiles differ in cost (the PV
    // fixes of a trigger class, the curriculum's task per 1344-id chunk)
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt) if (n_slots > 256)
    for (int t = 0; t < (n_slots + 63) / 64; ++t) {
      const int hi = (t + 1) * 64 < n_slots ? (t + 1) * 64 : n_slots;
      for (int i = t * 64; i < hi; ++i) host_slot_step(a, sc, task, i);
    }
    env->step += 1;
  }
  return OUZ_OK;
}

}  // namespace

extern "C" {

int32_t ouz_host_abi_version(void) { return OUZ_ABI_VERSION; }
const char* ouz_host_last_error(void) { return g_host_err.c_str(); }

int ouz_host_create(const ouz_config* cfg, ouz_host_env** out) {
  if (!cfg || !out) return host_fail(OUZ_ERR_INVALID, "ouz_host_create: null argument");
  if (const char* bad = config_error(cfg)) return host_fail(OUZ_ERR_INVALID, std::string("ouz_host_create: ") + bad);
  ouz_host_env* e = new ouz_host_env();
  e->cfg = *cfg;
  e->cfg.num_envs_total = cfg->num_envs_total > 0 ? cfg->num_envs_total : cfg->num_envs;
  e->bound = false;
  e->step = 0;
  e->threads = 0;
  build_waypoints(e->wp_tab);
  memset(&e->drn, 0, sizeof(e->drn));
  fill_step_args(cfg, e->a);
  e->a.wp_tab = e->wp_tab;
  e->a.drn = e->drn.noise;
  *out = e;
  return OUZ_OK;
}

int ouz_host_destroy(ouz_host_env* env) {
  delete env;
  return OUZ_OK;
}

int ouz_host_bind(ouz_host_env* env, const ouz_buffers* b) {
  if (!env || !b) return host_fail(OUZ_ERR_INVALID, "ouz_host_bind: null argument");
  if (!b->fstate || !b->istate || !b->obs || !b->rew || !b->reset || !b->timeouts)
    return host_fail(OUZ_ERR_INVALID, "ouz_host_bind: every buffer pointer must be set");
  StepArgs& a = env->a;
  a.f = b->fstate;
  a.iv = b->istate;
  a.obs = b->obs;
  a.rew = b->rew;
  a.reset = b->reset;
  a.timeouts = b->timeouts;
  a.rst_in = b->reset;
  a.to_in = b->timeouts;
  env->bound = true;
  return OUZ_OK;
}

int ouz_host_set_threads(ouz_host_env* env, int32_t threads) {
  if (!env || threads < 0) return host_fail(OUZ_ERR_INVALID, "ouz_host_set_threads: bad arguments");
  env->threads = threads;
  return OUZ_OK;
}

int ouz_host_init_state(ouz_host_env* env) {
  if (!env || !env->bound) return host_fail(OUZ_ERR_UNBOUND, "ouz_host_init_state: env not bound");
  const StepArgs& a = env->a;
  for (int s = 0; s < a.n_slots; ++s) host_init_slot(a, env->cfg.task, s);
  env->step = 0;
  return OUZ_OK;
}

int ouz_host_step(ouz_host_env* env, const float* actions) {
  return host_steps(env, actions, 1, 1, "ouz_host_step");
}

int ouz_host_step_n(ouz_host_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps) {
  return host_steps(env, action_ring, ring_len, n_steps, "ouz_host_step_n");
}

int ouz_host_reset_idx(ouz_host_env* env, const int32_t* env_ids, int32_t n) {
  if (!env || !env->bound || (n > 0 && !env_ids) || n < 0)
    return host_fail(OUZ_ERR_INVALID, "ouz_host_reset_idx: bad arguments");
  for (int32_t k = 0; k < n; ++k)
    if (env_ids[k] >= 0 && env_ids[k] < env->a.n) env->a.reset[env_ids[k]] = 1;
  return OUZ_OK;
}

int ouz_host_reset_all(ouz_host_env* env) {
  if (!env || !env->bound) return host_fail(OUZ_ERR_UNBOUND, "ouz_host_reset_all: env not bound");
  for (int32_t e = 0; e < env->a.n; ++e) env->a.reset[e] = 1;
  return OUZ_OK;
}

int ouz_host_episode_stats(ouz_host_env* env, double* out, int32_t drain) {
  if (!env || !env->bound || !out) return host_fail(OUZ_ERR_INVALID, "ouz_host_episode_stats: bad arguments");
  const StepArgs& a = env->a;
  double t[3] = {0.0, 0.0, 0.0};   // slot order: deterministic
  for (int i = 0; i < a.n_slots; ++i) {
    t[0] += (double)ld(a, OUZ_F_EP_SUM, i);
    t[1] += (double)ldi(a, OUZ_I_EP_CNT, i);
    t[2] += (double)ldi(a, OUZ_I_EP_LEN, i);
    if (drain) {
      st(a, OUZ_F_EP_SUM, i, 0.0f);
      sti(a, OUZ_I_EP_CNT, i, 0);
      sti(a, OUZ_I_EP_LEN, i, 0);
    }
  }
  out[0] = t[0];
  out[1] = t[1];
  out[2] = t[2];
  return OUZ_OK;
}

int ouz_host_set_trace(ouz_host_env* env, float* trace, uint32_t* resets, int32_t env_index, int32_t capacity) {
  if (!env || capacity < 0 || (capacity > 0 && (!trace || !resets || env_index < 0 || env_index >= env->a.n)))
    return host_fail(OUZ_ERR_INVALID, "ouz_host_set_trace: bad arguments");
  env->a.trace = capacity ? trace : nullptr;
  env->a.trace_resets = capacity ? resets : nullptr;
  env->a.trace_env = capacity ? env_index : -1;
  env->a.trace_cap = capacity;
  return OUZ_OK;
}

int ouz_host_set_dr_noise(ouz_host_env* env, int32_t target, const ouz_dr_noise* dr) {
  if (!env || (target != 0 && target != 1)) return host_fail(OUZ_ERR_INVALID, "ouz_host_set_dr_noise: bad target");
  if (dr && (dr->distribution < 0 || dr->distribution > 2 || dr->operation < 0 || dr->operation > 1 ||
             dr->schedule < 0 || dr->schedule > 2 || (dr->schedule && dr->schedule_steps <= 0) || dr->frequency < 0))
    return host_fail(OUZ_ERR_INVALID, "ouz_host_set_dr_noise: bad distribution / operation / schedule / frequency");
  if (dr) env->drn.noise[target] = *dr;
  else memset(&env->drn.noise[target], 0, sizeof(ouz_dr_noise));
  const bool on = env->drn.noise[target].distribution != 0;
  env->a.drn_mask = on ? (env->a.drn_mask | (1 << target)) : (env->a.drn_mask & ~(1 << target));
  return OUZ_OK;
}

int ouz_host_set_dr_gravity(ouz_host_env* env, const ouz_dr_param* dr, int32_t frequency) {
  if (!env) return host_fail(OUZ_ERR_INVALID, "ouz_host_set_dr_gravity: null env");
  ouz_dr_param p{};
  if (dr) p = *dr;
  if (const char* bad = dr_gravity_error(&p, frequency))
    return host_fail(OUZ_ERR_INVALID, std::string("ouz_host_set_dr_gravity: ") + bad);
  env->drn.grav.p = p;
  env->drn.grav.frequency = frequency;
  env->a.drn_mask = p.distribution ? (env->a.drn_mask | 4) : (env->a.drn_mask & ~4);
  return OUZ_OK;
}

int ouz_host_set_dr_physical(ouz_host_env* env, const ouz_dr_physical* dr) {
  if (!env) return host_fail(OUZ_ERR_INVALID, "ouz_host_set_dr_physical: null env");
  if (dr)
    if (const char* bad = dr_physical_error(dr))
      return host_fail(OUZ_ERR_INVALID, std::string("ouz_host_set_dr_physical: ") + bad);
  set_phys_dr(env->a, env->cfg.task, dr);
  return OUZ_OK;
}

int64_t ouz_host_get_step(const ouz_host_env* env) { return env ? env->step : -1; }

int ouz_host_set_step(ouz_host_env* env, int64_t step) {
  if (!env || step < 0) return host_fail(OUZ_ERR_INVALID, "ouz_host_set_step: bad arguments");
  env->step = step;
  return OUZ_OK;
}

}  // extern "C"
