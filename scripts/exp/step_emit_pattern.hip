// Per-step (VecTask.step) form of scripts/exp/emit_pattern.hip: what the trigger-class
// layout's env-order accesses cost the ONE-step kernel at 4096 envs.
//
// One-wave workgroups over the slot tiles (84 for 4096 envs in 1344-env class blocks), each lane: read the env's
// reset_buf (i64) and time_outs (u8) at its env index (env_load), wait about one per-step estimator chain (s_sleep),
// then write the 52-byte obs row (three 16-byte stores + one dword), the reward, reset and time-out at the env
// index (emit_env).  Layout 0: slot s holds env s (lanes adjacent); layout 1: the class layout (lanes 21 envs
// apart, quad_env.h slot_env).  Launched back to back, 200 per timing, layouts interleaved; prints the mean per
// launch.  Under rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE the bytes that leave / enter the L2s per launch.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/step_emit_pattern scripts/exp/step_emit_pattern.hip
//   /tmp/step_emit_pattern [envs] [sleep_iters] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kClasses = 21, kBlock = kClasses * 64, kObs = 13;

__device__ __forceinline__ int slot_env(int s) {
  const int b = s / kBlock, r = s - b * kBlock;
  return b * kBlock + (r >> 6) + kClasses * (r & 63);
}

template <int LAYOUT>
__global__ __launch_bounds__(64) void step_emit(float* obs, float* rew, long long* reset, unsigned char* tos, int n,
                                                int sleep_iters) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  const int e = LAYOUT ? slot_env(s) : s;
  if (e >= n) return;
  const long long rv = reset[e];                 // env_load: the previous step's flags, by env index
  const unsigned tv = tos[e];
  for (int t = 0; t < sleep_iters; ++t) __builtin_amdgcn_s_sleep(127);   // ~ the step's chain
  float v = (float)(rv + tv) + (float)e;
  typedef float f4a4 __attribute__((ext_vector_type(4), aligned(4)));
  float* row = obs + (size_t)e * kObs;
  *reinterpret_cast<f4a4*>(row) = f4a4{v, v + 1, v + 2, v + 3};
  *reinterpret_cast<f4a4*>(row + 4) = f4a4{v + 4, v + 5, v + 6, v + 7};
  *reinterpret_cast<f4a4*>(row + 8) = f4a4{v + 8, v + 9, v + 10, v + 11};
  row[12] = v + 12;
  rew[e] = v;
  reset[e] = (rv + 1) & 1;
  tos[e] = (unsigned char)((tv + 1) & 1);
}

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t err_ = (x);                                                          \
    if (err_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_));               \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int sleep_iters = argc > 2 ? std::atoi(argv[2]) : 2;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 5;
  if (n <= 0 || n > (1 << 20)) return 2;
  const int slots = (n + kBlock - 1) / kBlock * kBlock;
  float *obs, *rew;
  long long* reset;
  unsigned char* tos;
  CK(hipMalloc(&obs, sizeof(float) * (size_t)n * kObs));
  CK(hipMalloc(&rew, sizeof(float) * (size_t)n));
  CK(hipMalloc(&reset, sizeof(long long) * (size_t)n));
  CK(hipMalloc(&tos, (size_t)n));
  CK(hipMemset(reset, 0, sizeof(long long) * (size_t)n));
  CK(hipMemset(tos, 0, (size_t)n));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int launches = 200;
  std::vector<float> us[2];
  for (int r = 0; r < rounds; ++r)
    for (int layout = 0; layout < 2; ++layout) {
      const int grid = layout ? slots / 64 : (n + 63) / 64;
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < launches; ++k) {
        if (layout) hipLaunchKernelGGL(step_emit<1>, dim3(grid), dim3(64), 0, 0, obs, rew, reset, tos, n, sleep_iters);
        else hipLaunchKernelGGL(step_emit<0>, dim3(grid), dim3(64), 0, 0, obs, rew, reset, tos, n, sleep_iters);
      }
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t = 0;
      CK(hipEventElapsedTime(&t, a, b));
      us[layout].push_back(t * 1e3f / launches);
    }
  for (int layout = 0; layout < 2; ++layout) {
    std::sort(us[layout].begin(), us[layout].end());
    std::printf("{\"layout\": \"%s\", \"envs\": %d, \"sleep_iters\": %d, \"launches_per_timing\": %d, \"rounds\": %d, "
                "\"median_us_per_launch\": %.3f, \"min_us_per_launch\": %.3f, \"algorithmic_bytes_per_env_step\": {\"read\": 9, \"write\": 65}}\n",
                layout ? "class (lanes 21 envs apart)" : "identity (lanes adjacent)", n, sleep_iters, launches, rounds,
                us[layout][us[layout].size() / 2], us[layout][0]);
  }
  CK(hipFree(obs));
  CK(hipFree(rew));
  CK(hipFree(reset));
  CK(hipFree(tos));
  return 0;
}
