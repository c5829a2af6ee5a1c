/*
 * ouzelum_host.h — C ABI of the host build of the quadrotor step (libouzelum_cpu.so).
 *
 * The reference's VecTask runs on a CPU device too: tasks/base/vec_task.py:169-223 takes sim_device="cpu" and
 * keeps every buffer a torch CPU tensor (BASELINE.json config A, "CPU torch plumbing").  This library is that
 * path for the build: the SAME per-env step as libouzelum_hip.so (ouzelum_amd/csrc/quad_env.h + quad_math.h
 * compiled for the host with OpenMP over envs), over the same wave-tiled SoA state (ouzelum.h OUZ_FIDX, the
 * same state slots), f32 like the kernels.  Buffers are host memory owned by the caller; calls are synchronous.
 * Return codes and ouz_config / ouz_buffers / ouz_dr_noise are those of ouzelum.h.
 *
 * Entry point                 replaces (reference)                           GPU counterpart (ouzelum.h)
 *   ouz_host_create/bind/init VecTask.__init__ + allocate_buffers            ouz_create / ouz_bind / ouz_init_state
 *                             tasks/base/vec_task.py:169-223,254-277
 *   ouz_host_step             VecTask.step  tasks/base/vec_task.py:313-359   ouz_step
 *   ouz_host_step_n           K VecTask.step calls over an action ring        ouz_step_n
 *   ouz_host_reset_idx/_all   VecTask.reset_idx / reset_done (lazy)          ouz_reset_idx / ouz_reset_all
 *                             tasks/base/vec_task.py:369-406
 *   ouz_host_episode_stats    RecordEpisodeStatisticsTorch  PPO/utils.py:20-35  ouz_episode_stats
 *   ouz_host_set_trace        trajectory CSV + metrics counts                ouz_set_trace
 *                             tasks/ekf_lee_landed.py:132-135,319-331,667-674
 *   ouz_host_set_dr_noise     VecTask DR noise  tasks/base/vec_task.py:576-646  ouz_set_dr_noise
 *   ouz_host_set_dr_physical  VecTask physical DR  vec_task.py:547-563,680-756   ouz_set_dr_physical
 *   ouz_host_set_dr_gravity   sim_params gravity DR  vec_task.py:556-566,648-660  ouz_set_dr_gravity
 *   ouz_host_get/set_step     the step counter (sim_step_count)              ouz_get_step / ouz_set_step
 */
#ifndef OUZELUM_HOST_H_
#define OUZELUM_HOST_H_

#include <stdint.h>

#include "ouzelum.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ouz_host_env ouz_host_env;

int32_t ouz_host_abi_version(void);
const char* ouz_host_last_error(void);
int ouz_host_create(const ouz_config* cfg, ouz_host_env** out);
int ouz_host_destroy(ouz_host_env* env);
/* host pointers, sized as for ouz_bind (state over ouz_state_slots(task, num_envs) slots) */
int ouz_host_bind(ouz_host_env* env, const ouz_buffers* bufs);
/* OpenMP threads a step uses (0: the runtime's default, OMP_NUM_THREADS) */
int ouz_host_set_threads(ouz_host_env* env, int32_t threads);
int ouz_host_init_state(ouz_host_env* env);
int ouz_host_step(ouz_host_env* env, const float* actions);
int ouz_host_step_n(ouz_host_env* env, const float* action_ring, int32_t ring_len, int32_t n_steps);
int ouz_host_reset_idx(ouz_host_env* env, const int32_t* env_ids, int32_t n);
int ouz_host_reset_all(ouz_host_env* env);
int ouz_host_episode_stats(ouz_host_env* env, double* out, int32_t drain);
int ouz_host_set_trace(ouz_host_env* env, float* trace, uint32_t* resets, int32_t env_index, int32_t capacity);
int ouz_host_set_dr_noise(ouz_host_env* env, int32_t target, const ouz_dr_noise* dr);
int ouz_host_set_dr_physical(ouz_host_env* env, const ouz_dr_physical* dr);
int ouz_host_set_dr_gravity(ouz_host_env* env, const ouz_dr_param* dr, int32_t frequency);
int64_t ouz_host_get_step(const ouz_host_env* env);
int ouz_host_set_step(ouz_host_env* env, int64_t step);

#ifdef __cplusplus
}
#endif
#endif /* OUZELUM_HOST_H_ */
