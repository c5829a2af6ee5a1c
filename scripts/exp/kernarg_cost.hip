// Host time of one hipLaunchKernelGGL by kernel-argument size, and the GPU round trip of a launch + sync
// (empty kernels taking one struct of B bytes; 1 workgroup of 64).  Tells how much of a rollout launch's ~4.7 us
// of host time and of the region's wall is the ~1.1 KB StepArgs + RolloutArgs block.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/kernarg_cost scripts/exp/kernarg_cost.hip && /tmp/kernarg_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int B>
struct Blob {
  unsigned char b[B];
};

template <int B>
__global__ __launch_bounds__(64) void touch(Blob<B> a, float* out) {
  // read the first and last byte so the block is live (the rollout kernel reads its whole block)
  if (threadIdx.x == 0 && a.b[0] == 7 && a.b[B - 1] == 9) out[0] = 1.0f;
}

using clk = std::chrono::steady_clock;

template <int B>
void run(float* out) {
  Blob<B> a{};
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(touch<B>, dim3(1), dim3(64), 0, 0, a, out);
  hipDeviceSynchronize();
  // (1) host time per launch, 2000 back to back (queue kept busy)
  const int n = 2000;
  auto t0 = clk::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(touch<B>, dim3(1), dim3(64), 0, 0, a, out);
  auto t1 = clk::now();
  hipDeviceSynchronize();
  auto t2 = clk::now();
  // (2) one launch on an idle GPU + hipDeviceSynchronize, median of 300
  std::vector<double> rt, lh;
  for (int i = 0; i < 300; ++i) {
    auto s0 = clk::now();
    hipLaunchKernelGGL(touch<B>, dim3(1), dim3(64), 0, 0, a, out);
    auto s1 = clk::now();
    hipDeviceSynchronize();
    auto s2 = clk::now();
    lh.push_back(std::chrono::duration<double, std::micro>(s1 - s0).count());
    rt.push_back(std::chrono::duration<double, std::micro>(s2 - s0).count());
  }
  std::sort(rt.begin(), rt.end());
  std::sort(lh.begin(), lh.end());
  std::printf("{\"kernarg_bytes\": %d, \"host_us_per_launch_b2b\": %.3f, \"gpu_us_per_launch_b2b\": %.3f, "
              "\"idle_launch_host_us\": %.3f, \"idle_launch_sync_roundtrip_us\": %.3f}\n",
              B, std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
              std::chrono::duration<double, std::micro>(t2 - t0).count() / n, lh[150], rt[150]);
}

int main() {
  float* out;
  hipMalloc(&out, 16);
  run<16>(out);
  run<128>(out);
  run<512>(out);
  run<1024>(out);
  run<1152>(out);
  run<2048>(out);
  run<16>(out);
  run<1152>(out);
  return 0;
}
