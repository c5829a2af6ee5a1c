// A C/C++ host driving the step through the C ABI alone: no Python, no torch.
// hipMalloc's the buffers of include/ouzelum.h, creates a LeeLanded env, runs steps,
// reads the episode statistics, and prints one line with the step time.
//
//   hipcc --offload-arch=gfx950 -O2 examples/c_host_step.cpp -Iinclude \
//         -Louzelum_amd -louzelum_hip -Wl,-rpath,$PWD/ouzelum_amd -o examples/c_host_step
//   ./examples/c_host_step [num_envs] [steps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ouzelum.h"

#define CHECK(x)                                                                 \
  do {                                                                           \
    int _r = (x);                                                                \
    if (_r != 0) {                                                               \
      std::fprintf(stderr, "%s failed (%d): %s\n", #x, _r, ouz_last_error());    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)
#define HIPCHECK(x)                                                              \
  do {                                                                           \
    hipError_t _e = (x);                                                         \
    if (_e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(_e));               \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 1000;
  if (ouz_abi_version() != OUZ_ABI_VERSION) {
    std::fprintf(stderr, "ABI mismatch\n");
    return 1;
  }
  ouz_config cfg;
  ouz_default_config(&cfg);
  cfg.task = OUZ_TASK_LEE_LANDED;
  cfg.num_envs = n;
  cfg.seed = 7;
  cfg.track_episodes = 1;
  ouz_env* env = nullptr;
  CHECK(ouz_create(&cfg, &env));

  ouz_buffers b{};
  const int64_t slots = ouz_state_slots(cfg.task, n);   // == n except for the estimator tasks' class layout
  if (slots < n) { std::fprintf(stderr, "ouz_state_slots: %s\n", ouz_last_error()); return 1; }
  HIPCHECK(hipMalloc(&b.fstate, OUZ_TILED_SIZE(slots, OUZ_F_COUNT) * sizeof(float)));
  HIPCHECK(hipMalloc(&b.istate, OUZ_TILED_SIZE(slots, OUZ_I_COUNT) * sizeof(int32_t)));
  HIPCHECK(hipMalloc(&b.obs, (size_t)n * OUZ_NUM_OBS * sizeof(float)));
  HIPCHECK(hipMalloc(&b.rew, (size_t)n * sizeof(float)));
  HIPCHECK(hipMalloc(&b.reset, (size_t)n * sizeof(int64_t)));
  HIPCHECK(hipMalloc(&b.timeouts, (size_t)n));
  double* stats = nullptr;
  HIPCHECK(hipMalloc(&stats, 3 * sizeof(double)));
  hipStream_t s;
  HIPCHECK(hipStreamCreate(&s));
  CHECK(ouz_bind(env, &b));
  CHECK(ouz_init_state(env, s));

  for (int k = 0; k < 50; ++k) CHECK(ouz_step(env, nullptr, s));   // Lee tasks ignore actions
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  HIPCHECK(hipEventRecord(e0, s));
  for (int k = 0; k < steps; ++k) CHECK(ouz_step(env, nullptr, s));
  HIPCHECK(hipEventRecord(e1, s));
  CHECK(ouz_episode_stats(env, stats, 1, s));
  HIPCHECK(hipStreamSynchronize(s));
  float ms = 0.0f;
  HIPCHECK(hipEventElapsedTime(&ms, e0, e1));

  double h_stats[3];
  float h_obs[OUZ_NUM_OBS];
  HIPCHECK(hipMemcpy(h_stats, stats, sizeof(h_stats), hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(h_obs, b.obs, sizeof(h_obs), hipMemcpyDeviceToHost));
  int finite = 1;
  for (float v : h_obs) finite &= (v == v) && v <= 5.0f && v >= -5.0f;
  std::printf("{\"num_envs\": %d, \"steps\": %d, \"us_per_step\": %.3f, \"env_steps_per_s\": %.4g, "
              "\"episodes\": %.0f, \"obs0_finite\": %d, \"step\": %lld}\n",
              n, steps, 1e3 * ms / steps, (double)n * steps / (ms * 1e-3), h_stats[1], finite,
              (long long)ouz_get_step(env));

  CHECK(ouz_destroy(env));
  (void)hipFree(b.fstate); (void)hipFree(b.istate); (void)hipFree(b.obs); (void)hipFree(b.rew);
  (void)hipFree(b.reset); (void)hipFree(b.timeouts); (void)hipFree(stats);
  (void)hipStreamDestroy(s);
  return finite ? 0 : 2;
}
