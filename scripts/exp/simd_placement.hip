// Where do the waves of one workgroup run?  For 128- and 256-thread workgroups (84 of them, the split-wave
// rollout's grid at 4096 envs) every wave records HW_REG_HW_ID (gfx9 layout: wave slot [3:0], SIMD [5:4],
// CU [11:8], shader array [12], shader engine [15:13]) and spins ~20 us so that the whole grid is resident at
// once; the host prints, per block size, how many workgroups have waves 0 and 1 on one SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/simd_placement scripts/exp/simd_placement.hip && /tmp/simd_placement
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void placement(uint32_t* out) {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // hwreg(HW_REG_HW_ID, 0, 32)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(10);   // 100 MHz: 20 us
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = hw;
}

int main() {
  const int grid = 84;
  uint32_t* d;
  if (hipMalloc(&d, grid * 4 * sizeof(uint32_t)) != hipSuccess) return 1;
  for (int block : {128, 256}) {
    const int wpb = block / 64;
    hipLaunchKernelGGL(placement, dim3(grid), dim3(block), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<uint32_t> h(grid * wpb);
    if (hipMemcpy(h.data(), d, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int same01 = 0, same02 = 0, same_cu = 0;
    for (int b = 0; b < grid; ++b) {
      const uint32_t w0 = h[b * wpb], w1 = h[b * wpb + 1];
      const auto simd = [](uint32_t x) { return (x >> 4) & 3u; };
      const auto cu = [](uint32_t x) { return (x >> 8) & 15u; };
      same01 += simd(w0) == simd(w1);
      same_cu += cu(w0) == cu(w1);
      if (wpb > 2) same02 += simd(w0) == simd(h[b * wpb + 2]);
    }
    std::printf("{\"block\": %d, \"workgroups\": %d, \"waves_0_1_same_simd\": %d, \"waves_0_2_same_simd\": %d, "
                "\"waves_0_1_same_cu\": %d, \"first\": [", block, grid, same01, same02, same_cu);
    for (int k = 0; k < wpb * 3; ++k)
      std::printf("%s{\"simd\": %u, \"cu\": %u, \"se\": %u}", k ? ", " : "", (h[k] >> 4) & 3u, (h[k] >> 8) & 15u,
                  (h[k] >> 13) & 7u);
    std::printf("]}\n");
  }
  return hipFree(d) == hipSuccess ? 0 : 1;
}
