// The fused rollout's statistics tail in isolation (quad_kernels.hip reduce_stats): 64 one-wave workgroups (the
// 4096-env latency regime), each wave sums 3 doubles over its lanes, hands them to the last wave through a
// ticket, the last wave sums the partials.  Forms: 0 = no hand-off (exit after the wave sums); 1 = flat (write-
// through sc1 partials, drain, one agent-scope ticket add per wave, last adder reads with sc1 loads: the
// product form); 2 = two levels (waves grouped by 8: the group's last adder sums its group and adds to a top
// ticket); 3 = the old form (plain stores + __threadfence + atomicAdd).  200 launches back to back per timing,
// forms interleaved over 5 rounds; prints the median per launch.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ticket_probe scripts/exp/ticket_probe.hip && /tmp/ticket_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } \
  } while (0)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void st_wt(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_wt(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t add_ticket(uint32_t* t) {
  return __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int FORM>
__global__ __launch_bounds__(64) void tail(double* partials, double* group_partials, uint32_t* tickets, double* out) {
  const uint32_t lane = threadIdx.x, w = blockIdx.x, nw = gridDim.x;
  const double s = wave_sum((double)(w * 64 + lane)), c = wave_sum(1.0), l = wave_sum((double)lane);
  if (FORM == 0) {
    if (lane == 0 && s < 0) out[0] = s;   // keep the sums live
    return;
  }
  if (FORM == 3) {
    uint32_t last = 0;
    if (lane == 0u) {
      partials[w * 3] = s; partials[w * 3 + 1] = c; partials[w * 3 + 2] = l;
      __threadfence();
      last = atomicAdd(&tickets[0], 1u) == nw - 1u;
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    __threadfence();
    double t[3] = {0, 0, 0};
    for (uint32_t j = lane; j < nw; j += 64) for (int k = 0; k < 3; ++k) t[k] += __builtin_nontemporal_load(&partials[j * 3 + k]);
    for (int k = 0; k < 3; ++k) t[k] = wave_sum(t[k]);
    if (lane == 0) { out[0] = t[0]; out[1] = t[1]; out[2] = t[2]; tickets[0] = 0; }
    return;
  }
  if (FORM == 1) {
    uint32_t last = 0;
    if (lane == 0u) {
      st_wt(&partials[w * 3], s); st_wt(&partials[w * 3 + 1], c); st_wt(&partials[w * 3 + 2], l);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = add_ticket(&tickets[0]) == nw - 1u;
    }
    last = __shfl(last, 0, 64);
    if (!last) return;
    double t[3] = {0, 0, 0};
    for (uint32_t j = lane; j < nw; j += 64) for (int k = 0; k < 3; ++k) t[k] += ld_wt(&partials[j * 3 + k]);
    for (int k = 0; k < 3; ++k) t[k] = wave_sum(t[k]);
    if (lane == 0) { out[0] = t[0]; out[1] = t[1]; out[2] = t[2]; tickets[0] = 0; }
    return;
  }
  // FORM 2: groups of 8 waves (w % 8 shares an XCD under the round-robin dispatch)
  const uint32_t g = w % 8u, ng = (nw + 7u) / 8u, gsize = (nw - g + 7u) / 8u;
  uint32_t last = 0;
  if (lane == 0u) {
    st_wt(&partials[w * 3], s); st_wt(&partials[w * 3 + 1], c); st_wt(&partials[w * 3 + 2], l);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = add_ticket(&tickets[1 + g * 16]) == gsize - 1u;
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  double t[3] = {0, 0, 0};
  for (uint32_t j = g + 8u * lane; j < nw; j += 8u * 64u) for (int k = 0; k < 3; ++k) t[k] += ld_wt(&partials[j * 3 + k]);
  for (int k = 0; k < 3; ++k) t[k] = wave_sum(t[k]);
  uint32_t top = 0;
  if (lane == 0u) {
    tickets[1 + g * 16] = 0;
    st_wt(&group_partials[g * 3], t[0]); st_wt(&group_partials[g * 3 + 1], t[1]); st_wt(&group_partials[g * 3 + 2], t[2]);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    top = add_ticket(&tickets[0]) == (ng < 8u ? nw < 8u ? nw : 8u : 8u) - 1u;
  }
  top = __shfl(top, 0, 64);
  if (!top) return;
  double u[3] = {0, 0, 0};
  if (lane < 8u && lane < nw) for (int k = 0; k < 3; ++k) u[k] = ld_wt(&group_partials[lane * 3 + k]);
  for (int k = 0; k < 3; ++k) u[k] = wave_sum(u[k]);
  if (lane == 0) { out[0] = u[0]; out[1] = u[1]; out[2] = u[2]; tickets[0] = 0; }
}

int main(int argc, char** argv) {
  const int nw = argc > 1 ? std::atoi(argv[1]) : 64;
  double *partials, *gp, *out;
  uint32_t* tickets;
  CK(hipMalloc(&partials, sizeof(double) * 3 * 4096));
  CK(hipMalloc(&gp, sizeof(double) * 3 * 8));
  CK(hipMalloc(&out, sizeof(double) * 3));
  CK(hipMalloc(&tickets, sizeof(uint32_t) * 256));
  CK(hipMemset(tickets, 0, sizeof(uint32_t) * 256));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int launches = 200;
  std::vector<float> us[4];
  double res[4][3];
  for (int r = 0; r < 5; ++r)
    for (int f = 0; f < 4; ++f) {
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < launches; ++k) {
        if (f == 0) hipLaunchKernelGGL(tail<0>, dim3(nw), dim3(64), 0, 0, partials, gp, tickets, out);
        if (f == 1) hipLaunchKernelGGL(tail<1>, dim3(nw), dim3(64), 0, 0, partials, gp, tickets, out);
        if (f == 2) hipLaunchKernelGGL(tail<2>, dim3(nw), dim3(64), 0, 0, partials, gp, tickets, out);
        if (f == 3) hipLaunchKernelGGL(tail<3>, dim3(nw), dim3(64), 0, 0, partials, gp, tickets, out);
      }
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t = 0;
      CK(hipEventElapsedTime(&t, a, b));
      us[f].push_back(t * 1e3f / launches);
      CK(hipMemcpy(res[f], out, sizeof(double) * 3, hipMemcpyDeviceToHost));
    }
  const char* names[4] = {"no hand-off", "flat sc1 (product)", "two-level sc1", "threadfence (round 3)"};
  for (int f = 0; f < 4; ++f) {
    std::sort(us[f].begin(), us[f].end());
    std::printf("{\"form\": \"%s\", \"waves\": %d, \"median_us_per_launch\": %.3f, \"min_us\": %.3f, \"sum\": %.1f, \"count\": %.1f}\n",
                names[f], nw, us[f][2], us[f][0], res[f][0], res[f][1]);
  }
  return 0;
}
