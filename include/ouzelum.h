/*
 * ouzelum.h — C ABI of the MI355X-native quadrotor step (libouzelum_hip.so).
 *
 * Drop-in boundary for the reference's VecTask hot path.  Plain
 * pointers and sizes only: no torch or C++ types cross this line, so ctypes
 * (ouzelum_amd/_lib.py), cgo, JNI or N-API can bind it.  Device buffers are
 * owned by the caller (PyTorch tensors in the Python shim); the library only
 * keeps their pointers.  Every call returns 0 on success or a negative
 * OUZ_ERR_* code; ouz_last_error() gives a thread-local message.
 * Launch functions never synchronise the stream and never allocate, so a
 * caller may capture them into a hipGraph.
 *
 * Reference interface each entry point replaces (paths under isaacgymenvs/):
 *   ouz_create / ouz_bind / ouz_init_state
 *        VecTask.__init__ + allocate_buffers   tasks/base/vec_task.py:169-223,254-277
 *        task __init__ (tensor views, EKF/PV objects, controller)
 *                                              tasks/ekf_lee_landed.py:48-171, tasks/ouzelum.py:42-110
 *   ouz_step        VecTask.step               tasks/base/vec_task.py:313-359
 *                   = pre_physics_step + gym.simulate x controlFrequencyInv + post_physics_step
 *                                              tasks/ekf_lee_landed.py:308-530,620-685
 *   ouz_step_n      K consecutive VecTask.step calls over a ring of action batches, one launch each
 *                   (the train_vec.py:14-18 env-only loop); ouz_step_n_stats adds the rollout's
 *                   episode statistics (RecordEpisodeStatisticsTorch, PPO/utils.py:20-35)
 *   ouz_rollout     the same K steps fused into launches of up to 32 steps each: env state stays in
 *                   registers, per-step obs/rew/reset/time_outs go to rollout storage [K][N][...]
 *                   (the learners' obs[step] = next_obs buffers, PPO/main.py:67-73,88-96) or to the
 *                   env buffers.  For the Lee tasks actions are ignored (ekf_lee_landed.py:308), so a
 *                   fused rollout is exactly K VecTask.step calls.  Above 131 072 envs for the tasks
 *                   without the estimator (not EKFLeeLanded / QuadTracking / QuadMixed), or with
 *                   OUZ_ROLLOUT_STREAM=1 at ouz_create (=0 keeps the fused launches at every size), the
 *                   rollout is streamed instead: one step launch per step writing straight into the
 *                   storage rows, the statistics from a separate launch; bitwise K ouz_step calls.  The
 *                   fused launches agree with those within float tolerance (other code generation), so
 *                   results go from bitwise-equal-to-ouz_step to within-tolerance at that boundary.
 *   ouz_pre_physics the task's pre_physics_step alone (ekf_lee_landed.py:308-530, lee_landed.py:263-330,
 *                   ouzelum.py:218-251): lazy reset, estimator / controller / guidance / thrust model, and the
 *                   body wrench handed to apply_rigid_body_force_tensors; no integration, no outputs, the
 *                   step counter does not advance (a component entry for parity tests, not half a step).
 *                   It writes the pre-physics env state back (lazy reset, thrusts, EKF / PV filters,
 *                   waypoint; reset_buf cleared): restore the state before stepping on with the same step
 *   ouz_reset_idx   VecTask.reset_idx / reset_done (lazy: marks reset_buf)
 *                                              tasks/base/vec_task.py:369-406, ekf_lee_landed.py:271-306
 *   ouz_lee_control Controller.__call__        controllers/controller.py:45-48 (+ position/velocity/attitude)
 *   ouz_ekf_update  EKF.update (ang branch)    ahrs_ekf.py:1280-1337
 *   ouz_pv_predict  PVFilter.prediction_step   PVFilter.py:25-64
 *   ouz_pv_correct  PVFilter.correction_step   PVFilter.py:67-110
 *   ouz_pv_step     the driver's per-env predict -> position fix -> velocity fix (ekf_lee_landed.py:417-444),
 *                   evaluated in f64 with f32 storage, as inside ouz_step
 *   ouz_integrate   gym.simulate (PhysX)       tasks/base/vec_task.py:332-335 (build-defined integrator)
 *   ouz_reward      compute_ingenuity_reward   tasks/ekf_lee_landed.py:692-723
 *   ouz_philox      the counter RNG every draw of the step uses (replaces torch_rand_float /
 *                   torch.rand: ekf_lee_landed.py:284-286, ouzelum.py:183-184, utils/POMDP.py:25,30)
 */
#ifndef OUZELUM_H_
#define OUZELUM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OUZ_ABI_VERSION 6   /* 2: trigger-class state layout of the estimator tasks (ouz_state_slots);
                               3: 1344-id curriculum chunks of OUZ_TASK_MIXED with the class layout, ouz_env_slots;
                               4: physical domain randomisation (ouz_dr_physical, OUZ_I_RAND_STEP), DR noise
                                  frequency (ouz_dr_noise.frequency);
                               5: learner kernels (ouz_ppo_policy_loss, ouz_ppo_value_loss, ouz_tanh_bwd_bias,
                                  ouz_policy_sample);
                               6: sim_params gravity domain randomisation (ouz_set_dr_gravity), the fused LSTM
                                  sequence kernels (ouz_lstm_seq_fwd / ouz_lstm_seq_bwd), clipped Adam
                                  (ouz_adam_clip_step), the small-K first layer (ouz_linear_tanh_small_k) */

/* error codes */
#define OUZ_OK 0
#define OUZ_ERR_INVALID (-1)
#define OUZ_ERR_HIP (-2)
#define OUZ_ERR_UNBOUND (-3)

/* tasks (BASELINE.json configs) */
#define OUZ_TASK_OUZELUM 0        /* RL per-rotor thrust, random goals (tasks/ouzelum.py)        config A */
#define OUZ_TASK_LEE_LANDED 1     /* Lee position control on true state (tasks/lee_landed.py)   config B */
#define OUZ_TASK_EKF_LEE_LANDED 2 /* AHRS-EKF + PV-KF + Lee (tasks/ekf_lee_landed.py)                    */
#define OUZ_TASK_TRACKING 3       /* EKF pipeline + trajectory platform + DR                    config C */
#define OUZ_TASK_FAULT 4          /* RL thrust + single-rotor fault + obs noise                 config D */
#define OUZ_TASK_MIXED 5          /* curriculum of tasks 1/3/4 per OUZ_MIXED_CHUNK global ids   config E */
#define OUZ_TASK_LANDING 6        /* RL thrust, land on the husky following its trajectories (tasks/landing.py);
                                     the reference learners' default env (RPO-LSTM/main.py:18)              */
#define OUZ_NUM_TASKS 7

/* POMDP modes (utils/POMDP.py:5-20); -1 = task default */
#define OUZ_POMDP_NONE 0
#define OUZ_POMDP_FLICKER 1
#define OUZ_POMDP_NOISE 2
#define OUZ_POMDP_FLICKER_NOISE 3

/* Lee controller modes (controllers/controller.py:13-17) */
#define OUZ_LEE_POSITION 0
#define OUZ_LEE_VELOCITY 1
#define OUZ_LEE_ATTITUDE 2

/* observation / action sizes (tasks/ekf_lee_landed.py:56,61) */
#define OUZ_NUM_OBS 13
#define OUZ_NUM_ACT 4

/* State layout: wave-tiled SoA.  Envs are grouped in tiles of OUZ_TILE (= one
 * wave64); a tile holds every field of its 64 envs as contiguous 64-wide rows:
 *   fstate[ceil(num_envs/64)][OUZ_F_COUNT][64],  istate[...][OUZ_I_COUNT][64].
 * Field f of env i lives at OUZ_FIDX(f, i, OUZ_F_COUNT).  A wave's whole state
 * is one contiguous block, so its field loads walk DRAM pages in order instead
 * of touching OUZ_F_COUNT rows num_envs*4 bytes apart.
 *
 * State slots.  The tiles hold ouz_state_slots(task, num_envs) slots.  For most
 * tasks that is num_envs and slot i is env i.  The estimator tasks
 * (OUZ_TASK_EKF_LEE_LANDED, OUZ_TASK_TRACKING) up to 65536 envs (the latency
 * regime; above it the step is HBM-bound and slot i is env i) use the
 * trigger-class layout: the
 * PV filter's shared trigger counters (ekf_lee_landed.py:425-440) fire on
 * g % 7 == 6 and g % 3 == 0 of g = step * num_envs_total + global id, so slots
 * are grouped in blocks of 21 tiles (1344 slots) and tile k of block b holds
 * envs b*1344 + k + 21*lane: one trigger class per wave.  The slot count is
 * rounded up to a multiple of 1344; padding slots stay zero.  Slot of env e:
 * b*1344 + (r % 21)*64 + r/21 with b = e/1344, r = e - b*1344.  Buffers must
 * hold OUZ_TILED_SIZE(ouz_state_slots(task, num_envs), count) elements.  The
 * env-order buffers (obs, rew, reset, time_outs, actions) are indexed by env.
 * OUZ_TASK_MIXED assigns LeeLanded / QuadTracking / QuadFault to consecutive
 * chunks of OUZ_MIXED_CHUNK (= 1344, one class block) global ids; up to 65536
 * envs its slot space is chunk-aligned in global ids (slot s holds global id
 * c*1344 + r' with c = env_id_offset/1344 + s/1344, r = s % 1344, r' the class
 * permutation above in a QuadTracking chunk and r elsewhere; ids outside the
 * shard are idle slots), ouz_state_slots = (ceil(num_envs/1344) + 1) * 1344.
 * ouz_env_slots gives every env's slot for any task, size and offset. */
#define OUZ_MIXED_CHUNK 1344
#define OUZ_TILE 64
#define OUZ_TILES(n) (((n) + OUZ_TILE - 1) / OUZ_TILE)
#define OUZ_TILED_SIZE(n, count) ((size_t)OUZ_TILES(n) * (count) * OUZ_TILE)
#define OUZ_FIDX(f, i, count) \
  (((size_t)((i) / OUZ_TILE) * (count) + (f)) * OUZ_TILE + (size_t)((i) % OUZ_TILE))

/* Float fields of fstate. */
enum {
  OUZ_F_P = 0,          /* position (3)                    root_states[:, 0:3]  */
  OUZ_F_Q = 3,          /* orientation xyzw (4)            root_states[:, 3:7]  */
  OUZ_F_V = 7,          /* linear velocity, world (3)      root_states[:, 7:10] */
  OUZ_F_W = 10,         /* angular velocity, world (3)     root_states[:, 10:13]*/
  OUZ_F_TARGET = 13,    /* target_root_positions (3)                            */
  OUZ_F_PREV_V = 16,    /* prev_root_linvels (3)                                */
  OUZ_F_THRUST = 19,    /* RL rotor thrusts (4)                                 */
  OUZ_F_EKF_Q = 23,     /* EKF estimate, wxyz (4)          Q_state              */
  OUZ_F_EKF_P = 27,     /* EKF covariance, packed sym 4x4 (10)                  */
  OUZ_F_PV_X = 37,      /* PV filter state [p, v, b_a] (9)                      */
  OUZ_F_PV_P = 46,      /* PV covariance, packed sym 9x9 upper (45)             */
  OUZ_F_WAYPOINT = 91,  /* target_waypoints (3)                                 */
  OUZ_F_PLAT = 94,      /* landing-platform xy (2)                              */
  OUZ_F_TRAJ_SD = 96,   /* trajectory scale * direction (1)                     */
  OUZ_F_DR = 97,        /* DR scales of the nominal mass, inertia xx/yy, motor constant (3)        */
  OUZ_F_FAULT_ETA = 100,/* faulty-rotor efficiency (1)                          */
  OUZ_F_EP_RET = 101,   /* running episode return (RecordEpisodeStatisticsTorch) */
  OUZ_F_EP_SUM = 102,   /* sum of returns of episodes finished since last drain  */
  OUZ_F_PLAT_HEADING = 103, /* husky heading, rad (differential-drive platform)    */
  OUZ_F_COUNT = 104
};
/* Int32 fields of istate. */
enum {
  OUZ_I_PROGRESS = 0,   /* progress_buf                                         */
  OUZ_I_TRAJ_TYPE = 1,  /* 0 lemniscate, 1 circle, 2 square                     */
  OUZ_I_TRAJ_IDX = 2,
  OUZ_I_FAULT_ROTOR = 3,
  OUZ_I_FAULT_ONSET = 4,
  OUZ_I_LAND_FLAG = 5,  /* self.flag                                            */
  OUZ_I_LANDINGS = 6,   /* per-env landing count (self.Landoa summed)           */
  OUZ_I_EP_CNT = 7,     /* episodes finished since last drain                   */
  OUZ_I_EP_LEN = 8,     /* summed lengths of those episodes (info["l"])          */
  OUZ_I_RAND_STEP = 9,  /* step of the env's last physical randomization (-1: never); the reference's
                           randomize_buf (vec_task.py:275,560-563) is step - this                  */
  OUZ_I_COUNT = 10
};

typedef struct ouz_config {
  int32_t task;             /* OUZ_TASK_*                                        */
  int32_t num_envs;         /* envs on this device                               */
  int64_t env_id_offset;    /* global id of env 0 (rank * num_envs when sharded) */
  int64_t num_envs_total;   /* envs over all ranks (0 -> num_envs)               */
  uint64_t seed;
  int32_t device;           /* HIP device ordinal                                */
  int32_t pomdp;            /* OUZ_POMDP_* or -1 for the task default            */
  float pomdp_prob;         /* < 0 -> task default                               */
  float dt;                 /* sim.dt (0.01)                                     */
  int32_t substeps;         /* sim.substeps (2)                                  */
  int32_t convergence_time; /* EKF tasks: steps of estimator warm-up (300)       */
  float plat_speed;         /* max husky speed, m/s (15 rad/s x 0.165 m wheels)   */
  float dr_lo, dr_hi;       /* DR scale range                                    */
  float fault_eta_hi;       /* faulty rotor efficiency ~ U(0, fault_eta_hi)      */
  float thrust_max;         /* RL thrust clamp (2000 N, ouzelum.py:91)           */
  float thrust_rate;        /* RL thrust action scale (2000, ouzelum.py:237)     */
  int32_t track_episodes;   /* 1: accumulate episodic return/count in-kernel
                               (PPO/utils.py:4-35 RecordEpisodeStatisticsTorch)  */
  int32_t max_episode_length; /* env.maxEpisodeLength (cfg/task/<Task>.yaml); 0 -> task default */
} ouz_config;

typedef struct ouz_buffers {
  float* fstate;            /* [tiles][OUZ_F_COUNT][64] f32 (see OUZ_FIDX)        */
  int32_t* istate;          /* [tiles][OUZ_I_COUNT][64] i32                       */
  float* obs;               /* [num_envs][13] f32, clamped to +-5 (vec_task.py:353) */
  float* rew;               /* [num_envs] f32                                    */
  int64_t* reset;           /* [num_envs] i64  reset_buf                         */
  uint8_t* timeouts;        /* [num_envs] bool time_outs                         */
} ouz_buffers;

/* VecTask domain-randomisation noise on observations / actions (tasks/base/vec_task.py:576-646 "observations" /
 * "actions" entries; applied in step() before the clamps, :323-325,352-353).  noise = corr * b_c + a_c + fresh * b + a
 * (gaussian, a = mu, b = the reference's "var", used there as a standard deviation) or
 * corr * (hi_c - lo_c) + lo_c + U[0,1) * (hi - lo) + lo (uniform); x + noise (additive) or x * noise (scaling).
 * The parameters are re-derived every `frequency` steps (do_nonenv_randomize, :559,577): at step t they are those of
 * the epoch e = t - t % frequency, the schedule (0 none, 1 linear over schedule_steps, 2 constant: off until
 * schedule_steps) is evaluated at e, and corr ~ N(0,1), drawn per env element, is redrawn at every epoch (each
 * re-derivation builds a new params dict without 'corr', :610-620).  frequency <= 1: every step. */
typedef struct ouz_dr_noise {
  int32_t distribution;     /* 0 off, 1 gaussian, 2 uniform                       */
  int32_t operation;        /* 0 additive, 1 scaling                              */
  float range[2];           /* (mu, sigma) or (lo, hi)                            */
  float range_correlated[2];
  int32_t schedule;         /* 0 none, 1 linear, 2 constant                       */
  int32_t schedule_steps;
  int32_t frequency;        /* dr_params["frequency"] (default 1)                 */
  int32_t reserved;
} ouz_dr_noise;

/* Physical domain randomisation: VecTask.apply_randomizations' actor_params of the drone actor ("Drone",
 * ekf_lee_landed.py:242; vec_task.py:680-756) on the build's lumped rigid body.  At the lazy reset
 * of an env (reset_idx -> apply_randomizations, e.g. ant.py:246-248) whose randomize_buf = step - OUZ_I_RAND_STEP
 * >= frequency (vec_task.py:547-563; an env never randomized always is), each enabled parameter draws one sample
 * as dr_utils.generate_random_samples does (:71-133: the schedule at the current step scales the range, additive
 * ranges toward 0, scaling ranges toward 1; uniform lo + U(hi - lo), loguniform exp(U(log lo, log hi)), gaussian
 * mu + var * N(0, 1)) from the counter RNG, and sets the value from the nominal one as apply_random_samples does
 * (:148-205: nominal * sample or nominal + sample, never cumulative).  setup_only: only at the env's first
 * randomization.  Stored per env as scales of the nominal value (OUZ_F_DR). */
typedef struct ouz_dr_param {
  int32_t distribution;     /* 0 off, 1 gaussian, 2 uniform, 3 loguniform         */
  int32_t operation;        /* 0 additive, 1 scaling                              */
  float range[2];           /* (mu, var) or (lo, hi)                              */
  int32_t schedule;         /* 0 none, 1 linear, 2 constant                       */
  int32_t schedule_steps;
  int32_t setup_only;
  int32_t reserved;
} ouz_dr_param;
/* parameters: rigid_body_properties.mass (2.064 kg), rigid_body_properties.inertia (diag(0.0293, 0.0293, 0.0440):
 * scaling multiplies the tensor, additive adds the sample to each diagonal entry), and the rotors' motorConstant
 * (assets/x500/model.sdf:523, 8.54858e-6: every rotor's thrust scales with it) */
#define OUZ_DRP_MASS 0
#define OUZ_DRP_INERTIA 1
#define OUZ_DRP_MOTOR_CONSTANT 2
#define OUZ_DRP_COUNT 3
typedef struct ouz_dr_physical {
  int32_t frequency;        /* dr_params["frequency"] (default 1)                 */
  int32_t reserved;
  ouz_dr_param param[OUZ_DRP_COUNT];
} ouz_dr_physical;

typedef struct ouz_task_info {
  int32_t max_episode_length;
  float z_die;
  float land_radius;
  int32_t pomdp;
  float pomdp_prob;
  int32_t uses_actions;     /* 1 for RL-thrust tasks; Lee tasks ignore actions (ekf_lee_landed.py:308) */
  int32_t target_mode;      /* 0 random goal (stored), 1 fixed platform, 2 trajectory platform       */
  float plat_offset_x;      /* target x = platform x + offset (lee_landed.py:629, ekf_lee_landed.py:629) */
} ouz_task_info;

typedef struct ouz_env ouz_env;

int32_t ouz_abi_version(void);
/* 16 hex digits identifying the sources and flags this library was built from (ouzelum_amd/build.py source_id):
 * two builds of the same sources differ in bytes (hipcc's per-build unit ids), so profiling evidence is tied to
 * a library by this id. */
const char* ouz_source_id(void);
/* Instrumentation compiled into this library (0 for the product build): timing-stamp builds and
 * store-policy A/B builds give the product's results but are not the product; the Python shim
 * refuses them unless OUZ_ALLOW_INSTRUMENTED=1 (tests/test_abi.py checks the shipped library is 0). */
#define OUZ_BUILD_STAMPS 1u
#define OUZ_BUILD_TEMPORAL_STORES 2u
uint32_t ouz_build_flags(void);
/* Waits of the split-wave estimator rollout (two waves per tile meeting in LDS) that gave up
 * after ~70 ms instead of hanging the GPU, since the last reset: 0 unless the protocol is broken (its
 * results are then wrong).  reset != 0 zeroes the counter after reading it.  Synchronous. */
int ouz_split_timeouts(uint32_t* out, int32_t reset);
/* The same count on the env's device (switching to it for the call), read and zeroed in ONE device atomic, so a
 * give-up that lands during the call is neither lost nor read twice.  The count is per device: it covers every
 * env on that device (QuadVecTask.check_health raises if any of them gave up since the last read). */
int ouz_env_split_timeouts(ouz_env* env, uint32_t* out, int32_t reset);
/* Test-only: polls before a split-wave / output-wave wait gives up (0 restores the default, ~70 ms).  A small
 * value forces give-ups, so a test can check that they are reported (QuadVecTask.check_health raises). */
int ouz_set_split_spin_limit(uint32_t polls);
/* State slots of a task at num_envs (see "State slots" above); negative on bad arguments. */
int64_t ouz_state_slots(int32_t task, int32_t num_envs);
/* State slot of each of num_envs envs of a shard starting at global id env_id_offset, into the host
 * array env_slot[num_envs] (host-side, no GPU; the inverse of the kernels' slot -> env map). */
int ouz_env_slots(int32_t task, int32_t num_envs, int64_t env_id_offset, int32_t* env_slot);
const char* ouz_last_error(void);
void ouz_default_config(ouz_config* cfg);
int ouz_task_info_get(int32_t task, ouz_task_info* out);

int ouz_create(const ouz_config* cfg, ouz_env** out);
int ouz_destroy(ouz_env* env);
int ouz_bind(ouz_env* env, const ouz_buffers* bufs);
int ouz_init_state(ouz_env* env, void* stream);
int ouz_step(ouz_env* env, const float* actions, void* stream);
int ouz_step_n(ouz_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps, void* stream);
int ouz_rollout(ouz_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps, float* obs_out,
                float* rew_out, int64_t* reset_out, uint8_t* timeouts_out, void* stream);
/* ouz_rollout followed by the rollout's episode statistics (as ouz_episode_stats would write them),
 * reduced inside the last rollout launch: one launch per rollout of <= 32 steps, no statistics kernel
 * (RPO-LSTM/main.py:96-110: T env steps, then RecordEpisodeStatisticsTorch's returns).  A streamed
 * rollout (see ouz_rollout) writes them with ouz_episode_stats after its last step. */
int ouz_rollout_stats(ouz_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps, float* obs_out,
                      float* rew_out, int64_t* reset_out, uint8_t* timeouts_out, double* stats_out, int32_t drain,
                      void* stream);
/* pre_physics_step of the next step on the env state (see the table above): wrench [num_envs][6] f32 gets
 * (force xyz, torque xyz) in the body frame at the COM -- the lumped form of the forces / torques the
 * reference passes to gym.apply_rigid_body_force_tensors (LOCAL_SPACE).  reset_buf is cleared for the
 * envs it reset (reset_idx, ekf_lee_landed.py:300-301); obs / rew / time_outs are not written. */
int ouz_pre_physics(ouz_env* env, const float* actions, float* wrench, void* stream);
int ouz_reset_idx(ouz_env* env, const int32_t* env_ids, int32_t n, void* stream);
int ouz_reset_all(ouz_env* env, void* stream);
/* Episode statistics of envs created with track_episodes: writes the f64 triple
 * out[0] = sum of returns, out[1] = count, out[2] = sum of lengths, of the
 * episodes finished since the last drain (device pointer, stream-ordered; one launch, deterministic order).
 * drain != 0 zeroes the accumulators.  Replaces RecordEpisodeStatisticsTorch's
 * per-step host bookkeeping (PPO/utils.py:20-35); the pair is what config E
 * all-reduces over RCCL (sum and count; the lengths give info["l"]). */
int ouz_episode_stats(ouz_env* env, double* out, int32_t drain, void* stream);
/* ouz_step_n followed by ouz_episode_stats in one call: the rollout shape of the learners
 * (T env steps, then RecordEpisodeStatisticsTorch's returns, PPO/utils.py:20-35 /
 * RPO-LSTM/main.py:96-110) for one host call per rollout instead of two. */
int ouz_step_n_stats(ouz_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps, double* stats_out,
                     int32_t drain, void* stream);

/* Per-step trace of one env + per-step reset counts, written by the step kernel
 * itself (no extra launch, no host sync).  Feeds the reference's trajectory CSV
 * (ekf_lee_landed.py:132-135,667-674: env 0's position, target, velocity every
 * step, one file per cumulative episode count) and metrics/<pomdp>_<prob>_ep_count.txt
 * (:319-331).  Slot s % capacity of trace[capacity][9] holds (p, target, v) of
 * env_index after step s; resets[s % capacity] = envs reset at the start of
 * step s.  capacity >= 64 (the fused rollout runs waves up to 32 steps apart);
 * capacity 0 disables.  The host must read slots before they are reused. */
int ouz_set_trace(ouz_env* env, float* trace, uint32_t* resets, int32_t env_index, int32_t capacity);
/* target 0 = observations, 1 = actions; dr == NULL or distribution 0 disables. */
int ouz_set_dr_noise(ouz_env* env, int32_t target, const ouz_dr_noise* dr);
/* Physical DR of every env of this env object (all tasks of a curriculum), replacing the task default (QuadTracking:
 * mass / inertia / motor constant scaling ~ U(dr_lo, dr_hi) at every reset; the other tasks: none).  dr == NULL or
 * every distribution 0: off.  Takes effect at the next launch. */
int ouz_set_dr_physical(ouz_env* env, const ouz_dr_physical* dr);
/* sim_params gravity DR (VecTask.apply_randomizations' "sim_params": {"gravity": ...}, vec_task.py:556-566,648-660 ->
 * dr_utils.apply_random_samples :162-172).  The non-environment gate re-samples every `frequency` steps (<= 1: every
 * step): at step t the sim's gravity is that of the epoch e = t - t % frequency, ONE draw for the whole sim (not per
 * env) of generate_random_samples(params, 3, e) (the schedule at e; setup_only is not read, as in the reference's
 * sim_params path) from the counter RNG, applied per axis to the nominal (0, 0, -9.81): nominal * sample (scaling)
 * or nominal + sample (additive).  It enters the integrator only (the Lee controller's mg and the RL thrust scale are
 * the tasks' own constants, as in the reference).  dr == NULL or distribution 0: nominal gravity. */
int ouz_set_dr_gravity(ouz_env* env, const ouz_dr_param* dr, int32_t frequency);
int64_t ouz_get_step(const ouz_env* env);
int ouz_set_step(ouz_env* env, int64_t step);

/* component entry points (same device functions as the fused step) */
int ouz_lee_control(int32_t mode, const float* state, const float* cmd, float* thrust, float* torque, int32_t n,
                    void* stream);
int ouz_ekf_update(const float* q_wxyz, const float* P10, const float* gyr, const float* ang_wxyz, float dt,
                   float* q_out, float* P10_out, int32_t n, void* stream);
int ouz_pv_predict(float* x9, float* P45, const float* acc, const float* q_wxyz, float dt, int32_t n,
                   void* stream);
int ouz_pv_correct(float* x9, float* P45, const float* z, int32_t block, float var, const uint8_t* mask,
                   int32_t n, void* stream);
int ouz_pv_step(float* x9, float* P45, const float* acc, const float* q_wxyz, float dt, const float* pos_z,
                const uint8_t* pos_mask, const float* vel_z, const uint8_t* vel_mask, int32_t n, void* stream);
/* ouz_pv_step in the quad-lane form of the latency-regime estimator kernels (four lanes per env, the
 * covariance in LDS; quad_pv_ql.h): the same results bit for bit (tests/test_gpu_components.py). */
int ouz_pv_step_quad(float* x9, float* P45, const float* acc, const float* q_wxyz, float dt, const float* pos_z,
                     const uint8_t* pos_mask, const float* vel_z, const uint8_t* vel_mask, int32_t n, void* stream);
int ouz_integrate(float* root13, const float* f_b, const float* tau_b, const float* mass, const float* inertia,
                  float dt, int32_t substeps, int32_t n, void* stream);
int ouz_reward(const float* root13, const float* target, const int32_t* progress, int32_t max_episode_length,
               float z_die, float* rew, int64_t* reset, int32_t n, void* stream);
int ouz_philox(uint64_t seed, const uint32_t* env_ids, uint32_t step, uint32_t stream_id, uint32_t sub,
               uint32_t* out4, int32_t n, void* stream);

/* ---- learner-side kernels (recurrent PPO/RPO on MI355X) ---- */

/* Generalized advantage estimation over a (T, N) rollout (RPO-LSTM/agent.py:40-55,
 * PPO/agent.py:40-55).  rewards/values/dones [T][N] f32 (dones[t] = done flag
 * observed before step t), next_value/next_done [N] f32, outputs [T][N] f32.
 * gamma_lam = f32(gamma * lambda) as the reference's Python scalar product.
 * torch float32 operation order: bit-identical to the reference formula. */
int ouz_gae(const float* rewards, const float* values, const float* dones, const float* next_value,
            const float* next_done, int32_t T, int32_t N, float gamma, float gamma_lam, float* advantages,
            float* returns, void* stream);

/* POMDPWrapper.observation (utils/POMDP.py:23-43) applied by the learner to a
 * (rows, dim) f32 batch (RPO-LSTM/main.py:103): flicker zeroes the whole batch
 * with one coin per call, random_noise multiplies by U(1-prob, 1+prob) per
 * element, flickering_and_random_noise = flicker p 0.1 then noise.  Draws are
 * keyed (seed, row_offset + row, call); in == out is allowed. */
int ouz_pomdp_obs(const float* in, float* out, int32_t rows, int32_t dim, int32_t mode, float prob, uint64_t seed,
                  int64_t row_offset, uint32_t call, void* stream);

/* Fused LSTM cell for the recurrent actor (RPO-LSTM/model.py:27-50; torch gate order
 * i, f, g, o).  gates [B][4H] = x W_ih^T + b + (keep * h) W_hh^T, pre-activation;
 * c_prev_m [B][H] the masked carry; keep_next [B] (1 - done of the next step, or
 * null = 1).  Writes the activated gates act [B][4H] (saved for BPTT), c_out, h_out
 * and the next step's masked carry h_next_m / c_next_m. */
int ouz_lstm_cell_fwd(const float* gates, const float* c_prev_m, const float* keep_next, float* act, float* c_out,
                      float* h_out, float* h_next_m, float* c_next_m, int32_t B, int32_t H, void* stream);
/* BPTT of one step: dh = dhid + keep_next * G (G = dgates_{t+1} W_hh, or null),
 * dc = keep_next * dc_next (or null) + dh o (1 - tanh(c)^2); writes dgates [B][4H]
 * (pre-activation) and dc_prev [B][H] (gradient of the masked carry). */
int ouz_lstm_cell_bwd(const float* act, const float* c, const float* c_prev_m, const float* dhid, const float* G,
                      const float* dc_next, const float* keep_next, float* dgates, float* dc_prev, int32_t B, int32_t H,
                      void* stream);

/* The whole LSTM recurrence of a (T, B) sequence in one launch each way, hidden size H = 128 (the reference actor's
 * LSTM(256, 128), RPO-LSTM/model.py:34-50): the per-step GEMM + ouz_lstm_cell_fwd / _bwd pairs fused, the carry kept
 * on chip, the recurrent product on the f32 MFMA.  Forward: x_proj [T][B][4H] (x W_ih^T + b_ih + b_hh), h0 / c0
 * [B][H], keep [T][B] (1 - done before step t), w_hh the packed W_hh (w_fwd of ouz_lstm_seq_pack); writes hid
 * [T][B][H] and, when not
 * null, act [T][B][4H], c_all [T][B][H], hm / cm [T + 1][B][H] (the masked carry entering each step; row T the final
 * carry unless h_out / c_out [B][H] take it, which may alias h0 / c0).  Backward: the saved act / c_all / cm, keep,
 * the packed W_hh^T (w_bwd of ouz_lstm_seq_pack), dhid [T][B][H], dhT / dcT [B][H] or null; writes dgates
 * [T][B][4H] and, when not null, dh0 = (dgates_0 W_hh) keep_0 and dc0 [B][H].  Same arithmetic per element as the
 * per-step kernels; the products sum in another order (f32, within rounding of the GEMM path).  Every buffer except
 * keep and h0 (x_proj, c0, the outputs, the saved tensors and gradients) must be 16-byte aligned (one 16-byte access
 * per lane); OUZ_ERR_INVALID otherwise. */
/* ouz_lstm_seq_pack: W_hh [4H][H] into the two fragment layouts the sequence kernels read (w_fwd, w_bwd: 4H * H
 * floats each, 16-byte aligned; one contiguous 1 KB per wave per load), after every change of W_hh.  The forward
 * takes w_fwd as its w_hh argument, the backward w_bwd as its w_hh_t argument. */
int ouz_lstm_seq_pack(const float* w_hh, int32_t H, float* w_fwd, float* w_bwd, void* stream);
int ouz_lstm_seq_fwd(const float* x_proj, const float* h0, const float* c0, const float* keep, const float* w_hh,
                     int32_t T, int32_t B, int32_t H, float* act, float* c_all, float* hid, float* hm, float* cm,
                     float* h_out, float* c_out, void* stream);
int ouz_lstm_seq_bwd(const float* act, const float* c_all, const float* cm, const float* keep, const float* w_hh_t,
                     const float* dhid, const float* dhT, const float* dcT, int32_t T, int32_t B, int32_t H,
                     float* dgates, float* dh0, float* dc0, void* stream);

/* The trunks' first layer in one pass: y [rows][cols] = tanh(x [rows][K] W^T + b), W [cols][K] (nn.Linear's
 * weight), 1 <= K <= 16 (the 13 observations: RPO-LSTM/model.py:11-20 and the critic), cols a power of two in
 * [4, 1024], y 16-byte aligned.  tanh to ~1e-7 absolute (hardware exp2 / reciprocal). */
int ouz_linear_tanh_small_k(const float* x, const float* w, const float* b, int32_t rows, int32_t K, int32_t cols,
                            float* y, void* stream);

/* Gradient-norm clipping + Adam over one network's parameter tensors in two launches (RPO-LSTM/agent.py:124-134:
 * nn.utils.clip_grad_norm_(params, max_norm) then torch.optim.Adam.step(); torch/optim/adam.py single-tensor order).
 * The table lists up to OUZ_ADAM_MAX_TENSORS f32 tensors (contiguous, numel elements each): gradient (read only),
 * parameter, exp_avg and exp_avg_sq (updated in place).  step: the Adam step count after this step (1, 2, ...);
 * max_norm <= 0: no clipping.  workspace: OUZ_ADAM_WS_FLOATS floats of device memory. */
#define OUZ_ADAM_MAX_TENSORS 16
#define OUZ_ADAM_WS_FLOATS 512
typedef struct ouz_adam_table {
  int32_t n_tensors;
  int32_t reserved;
  int64_t numel[OUZ_ADAM_MAX_TENSORS];
  const float* grad[OUZ_ADAM_MAX_TENSORS];
  float* param[OUZ_ADAM_MAX_TENSORS];
  float* exp_avg[OUZ_ADAM_MAX_TENSORS];
  float* exp_avg_sq[OUZ_ADAM_MAX_TENSORS];
} ouz_adam_table;
int ouz_adam_clip_step(const ouz_adam_table* t, double lr, double beta1, double beta2, double eps, int64_t step,
                       double max_norm, float* workspace, void* stream);

/* PPO losses of one minibatch, forward + gradient for a unit upstream gradient in one call (the losses end the
 * graph).  Reductions are deterministic (fixed grid of OUZ_LOSS_BLOCKS per-block f64 partials summed in order).
 * Workspace: OUZ_LOSS_WS_DOUBLES doubles, device memory, not kept between calls.
 *
 * Clipped policy loss (RPO-LSTM/agent.py:86-110; PPO/agent.py same lines): with lp = Normal(mean_z,
 * exp(logstd)).log_prob(actions).sum(1) (torch's Normal: var = scale^2, log_scale = log(scale)), ratio =
 * exp(lp - old_logp), A = advantages normalised by their mean and unbiased std + 1e-8 when norm_adv,
 *   loss = mean(max(-A ratio, -A clamp(ratio, 1 - clip, 1 + clip))), approx_kl = mean((ratio - 1) - log ratio),
 *   clipfrac = mean(|ratio - 1| > clip);
 * dmean [n][4] = d loss / d mean_z and dlogstd [4] = d loss / d logstd (torch's maximum / clamp tie rules).
 * mean_z (the RPO-perturbed mean), actions, dmean [n][OUZ_NUM_ACT] 16-byte aligned; logstd [OUZ_NUM_ACT];
 * old_logp, advantages [n]; loss / approx_kl / clipfrac single floats. */
#define OUZ_LOSS_BLOCKS 256
#define OUZ_LOSS_WS_DOUBLES (10 * OUZ_LOSS_BLOCKS)
int ouz_ppo_policy_loss(const float* mean_z, const float* logstd, const float* actions, const float* old_logp,
                        const float* advantages, int32_t n, float clip, int32_t norm_adv, double* workspace,
                        float* dmean, float* loss, float* approx_kl, float* clipfrac, float* dlogstd, void* stream);
/* Value loss 0.5 * mean((values - returns)^2) (agent.py:104-105, clip_vloss False) and dvalues = (values -
 * returns) / n. */
int ouz_ppo_value_loss(const float* values, const float* returns, int32_t n, double* workspace, float* dvalues,
                       float* loss, void* stream);

/* Backward of y = tanh(x W^T + b) (the MLP trunks, RPO-LSTM/model.py:17-24,72-84): dz = dy (1 - y^2) and
 * dbias = column sums of dz in one pass.  dy, y, dz [rows][cols] row-major, cols a power of two in [4, 1024];
 * workspace OUZ_COLSUM_BLOCKS * cols floats; all 16-byte aligned.  Deterministic. */
#define OUZ_COLSUM_BLOCKS 1024
int ouz_tanh_bwd_bias(const float* dy, const float* y, int32_t rows, int32_t cols, float* workspace, float* dz,
                      float* dbias, void* stream);

/* The rollout policy's mean head and sample in one launch (RPO-LSTM/model.py:52-70, PPO/model.py:31-40 with
 * action None): mean = hidden W^T + b, action = mean + exp(logstd) eps, logprob = -1/2 sum eps^2 - sum logstd -
 * A log sqrt(2 pi), entropy = sum logstd + A (1/2 + log sqrt(2 pi)); A = OUZ_NUM_ACT.  hidden [B][H] (H a multiple
 * of 4) and W [A][H] 16-byte aligned, b / logstd [A], eps / action [B][A], logprob / entropy [B]. */
int ouz_policy_sample(const float* hidden, const float* w, const float* b, const float* logstd, const float* eps,
                      int32_t B, int32_t H, float* action, float* logprob, float* entropy, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OUZELUM_H_ */
