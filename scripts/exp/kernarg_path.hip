// Kernel-argument path probe: 400 B of arguments passed by value (copied by the host on every launch)
// vs a 16 B argument holding a pointer to the same 400 B kept in device memory (written once).
// Each kernel reads every dword of its arguments, then one dependent global load per lane, and
// stores (the shape of the step kernel's entry).  Not part of the product; scripts/exp/ probes only.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Args { unsigned v[100]; };
__global__ void spin_kernel(long long cycles) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}
__device__ __forceinline__ void body(const Args& a, unsigned step, const float* src, float* out) {
  unsigned s = step;
#pragma unroll
  for (int k = 0; k < 100; ++k) s += a.v[k];
  const int i = blockIdx.x * 64 + threadIdx.x;
  out[i] = src[i] + (float)(s & 7u);
}
__global__ void by_value(Args a, unsigned step, const float* src, float* out) { body(a, step, src, out); }
__global__ void by_pointer(const Args* __restrict__ p, unsigned step, const float* src, float* out) {
  body(*p, step, src, out);
}

__device__ Args g_args;
__global__ void from_global(unsigned step, const float* src, float* out) { body(g_args, step, src, out); }

template <class F> double host_us(hipStream_t s, int reps, F launch) {
  spin_kernel<<<1, 64, 0, s>>>(200000000LL);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; ++k) launch(k);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}
template <class F> double gpu_us(hipStream_t s, int reps, F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  spin_kernel<<<1, 64, 0, s>>>(20000000LL);
  (void)hipEventRecord(e0, s);
  for (int k = 0; k < reps; ++k) launch(k);
  (void)hipEventRecord(e1, s);
  (void)hipStreamSynchronize(s);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps;
}

int main() {
  hipStream_t s; (void)hipStreamCreate(&s);
  float *src, *out; Args* dargs;
  (void)hipMalloc(&src, 4096 * 4); (void)hipMalloc(&out, 4096 * 4); (void)hipMalloc(&dargs, sizeof(Args));
  (void)hipMemset(src, 0, 4096 * 4);
  Args a{};
  for (int k = 0; k < 100; ++k) a.v[k] = k;
  (void)hipMemcpy(dargs, &a, sizeof(Args), hipMemcpyHostToDevice);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_args), &a, sizeof(Args));
  auto glb = [&](int k) { hipLaunchKernelGGL(from_global, dim3(64), dim3(64), 0, s, (unsigned)k, src, out); };
  auto val = [&](int k) { hipLaunchKernelGGL(by_value, dim3(64), dim3(64), 0, s, a, (unsigned)k, src, out); };
  auto ptr = [&](int k) { hipLaunchKernelGGL(by_pointer, dim3(64), dim3(64), 0, s, dargs, (unsigned)k, src, out); };
  for (int w = 0; w < 3; ++w) { host_us(s, 200, val); host_us(s, 200, ptr); }
  for (int r = 0; r < 2; ++r)
    printf("host us/launch: from_global %.3f | gpu us/launch: from_global %.3f\n", host_us(s, 400, glb),
           gpu_us(s, 400, glb));
  for (int r = 0; r < 3; ++r)
    printf("host us/launch: by_value %.3f  by_pointer %.3f | gpu us/launch: by_value %.3f  by_pointer %.3f\n",
           host_us(s, 400, val), host_us(s, 400, ptr), gpu_us(s, 400, val), gpu_us(s, 400, ptr));
  return 0;
}
