// Write-pattern probe for the trigger-class layout's env-order output rows.
//
// Mimics the fused QuadTracking rollout's output stores at 4096 envs with nothing else in the kernel: one-wave
// workgroups over the slot tiles (84 for 4096 envs in 1344-env class blocks), 16 steps spaced by an s_sleep
// wait of about one estimator step, and per step and env the 52-byte obs row (three 16-byte stores + one
// dword), the reward (f32), reset (i64) and time-out (u8) at the env's index into (16, N, ...) storage.
// Layout 0: slot s holds env s (rows of neighbouring lanes adjacent).  Layout 1: the class layout, slot
// b*1344 + 64c + l holds env b*1344 + c + 21 l (quad_kernels.hip slot_env): neighbouring lanes 21 envs apart.
// Prints the median kernel time of each layout; run under rocprofv3 --pmc WRITE_SIZE for the bytes that
// leave the L2s (the same two launches, in order: layout 0 first).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/emit_pattern scripts/exp/emit_pattern.hip
//   /tmp/emit_pattern [envs] [sleep]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kClasses = 21, kBlock = kClasses * 64, kSteps = 16, kObs = 13;

__device__ __forceinline__ int slot_env(int s) {
  const int b = s / kBlock, r = s - b * kBlock;
  return b * kBlock + (r >> 6) + kClasses * (r & 63);
}

template <int LAYOUT>
__global__ __launch_bounds__(64) void emit_pattern(float* obs, float* rew, long long* reset, unsigned char* tos,
                                                   int n, int sleep_iters) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  const int e = LAYOUT ? slot_env(s) : s;
  float v = (float)e;
  for (int k = 0; k < kSteps; ++k) {
    for (int t = 0; t < sleep_iters; ++t) __builtin_amdgcn_s_sleep(127);   // ~one estimator step of work
    if (e < n) {
      typedef float f4a4 __attribute__((ext_vector_type(4), aligned(4)));
      float* row = obs + ((size_t)k * n + e) * kObs;
      *reinterpret_cast<f4a4*>(row) = f4a4{v, v + 1, v + 2, v + 3};
      *reinterpret_cast<f4a4*>(row + 4) = f4a4{v + 4, v + 5, v + 6, v + 7};
      *reinterpret_cast<f4a4*>(row + 8) = f4a4{v + 8, v + 9, v + 10, v + 11};
      row[12] = v + 12;
      rew[(size_t)k * n + e] = v;
      reset[(size_t)k * n + e] = k & 1;
      tos[(size_t)k * n + e] = (unsigned char)(k & 1);
    }
    v += 1.0f;
  }
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
  const int sleep_iters = argc > 2 ? std::atoi(argv[2]) : 1;
  if (n <= 0 || n > (1 << 20)) return 2;
  const int slots = (n + kBlock - 1) / kBlock * kBlock;   // the class layout's slot count (whole 1344-env blocks)
  float *obs, *rew;
  long long* reset;
  unsigned char* tos;
  CK(hipMalloc(&obs, sizeof(float) * kSteps * (size_t)n * kObs));
  CK(hipMalloc(&rew, sizeof(float) * kSteps * (size_t)n));
  CK(hipMalloc(&reset, sizeof(long long) * kSteps * (size_t)n));
  CK(hipMalloc(&tos, kSteps * (size_t)n));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 20;
  for (int layout = 0; layout < 2; ++layout) {
    const int grid = layout ? slots / 64 : (n + 63) / 64;
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a, 0));
      if (layout) hipLaunchKernelGGL(emit_pattern<1>, dim3(grid), dim3(64), 0, 0, obs, rew, reset, tos, n, sleep_iters);
      else hipLaunchKernelGGL(emit_pattern<0>, dim3(grid), dim3(64), 0, 0, obs, rew, reset, tos, n, sleep_iters);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t = 0;
      CK(hipEventElapsedTime(&t, a, b));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("{\"layout\": \"%s\", \"envs\": %d, \"workgroups\": %d, \"sleep_iters\": %d, \"median_us\": %.3f, "
                "\"min_us\": %.3f, \"algorithmic_write_bytes_per_env_step\": 65}\n",
                layout ? "class (lanes 21 envs apart)" : "identity (lanes adjacent)", n, grid, sleep_iters,
                ms[reps / 2] * 1e3, ms[0] * 1e3);
  }
  CK(hipFree(obs));
  CK(hipFree(rew));
  CK(hipFree(reset));
  CK(hipFree(tos));
  return 0;
}
