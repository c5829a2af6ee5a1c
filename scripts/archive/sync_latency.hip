// Host-visible completion latency of hipDeviceSynchronize by kernel duration: one launch of a kernel that spins
// for D microseconds (s_memrealtime, 100 MHz) on an idle GPU, then hipDeviceSynchronize; median of 200 of
// (sync return - launch return) - D.  If the runtime's wait turns from an active poll into a blocking
// (interrupt) wait past some time, the overhead jumps there.  argv[1] == "spin": hipSetDeviceFlags
// (hipDeviceScheduleSpin) first; "yield": hipDeviceScheduleYield; "block": hipDeviceScheduleBlockingSync.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sync_latency scripts/exp/sync_latency.hip && /tmp/sync_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ __launch_bounds__(64) void spin_us(uint64_t ticks, float* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0 && ticks == 12345) out[0] = 1.0f;
}

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "default";
  unsigned flags = 0;
  if (!std::strcmp(mode, "spin")) flags = hipDeviceScheduleSpin;
  if (!std::strcmp(mode, "yield")) flags = hipDeviceScheduleYield;
  if (!std::strcmp(mode, "block")) flags = hipDeviceScheduleBlockingSync;
  hipError_t fe = hipSuccess;
  if (flags) fe = hipSetDeviceFlags(flags);
  float* out;
  if (hipMalloc(&out, 16) != hipSuccess) return 1;
  const double dus[] = {0, 5, 10, 20, 30, 40, 60, 100};
  for (double d : dus) {
    const uint64_t ticks = (uint64_t)(d * 100.0);   // s_memrealtime: 100 MHz
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(spin_us, dim3(1), dim3(64), 0, 0, ticks, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<double> ov;
    for (int i = 0; i < 200; ++i) {
      hipLaunchKernelGGL(spin_us, dim3(1), dim3(64), 0, 0, ticks, out);
      auto s1 = clk::now();
      if (hipDeviceSynchronize() != hipSuccess) return 3;
      auto s2 = clk::now();
      ov.push_back(std::chrono::duration<double, std::micro>(s2 - s1).count() - d);
    }
    std::sort(ov.begin(), ov.end());
    std::printf("{\"mode\": \"%s\", \"set_flags_rc\": %d, \"kernel_us\": %.0f, \"sync_minus_kernel_us_median\": %.2f, "
                "\"p10\": %.2f, \"p90\": %.2f}\n", mode, (int)fe, d, ov[100], ov[20], ov[180]);
  }
  return 0;
}
