// Host cost of hipLaunchKernelGGL vs kernel-argument size (empty kernels; GPU held by a spin kernel
// so every launch is queued behind it).  Not part of the product; scripts/exp/ probes only.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int N> struct Blob { unsigned char b[N]; };
template <int N> __global__ void empty_kernel(Blob<N> a, int* out) { if (threadIdx.x == 9999) out[0] = a.b[N - 1]; }
__global__ void spin_kernel(long long cycles) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}
__global__ void dep_kernel(int* out) { if (threadIdx.x == 0) out[blockIdx.x] += 1; }

template <int N> double host_us(hipStream_t s, int* out, int reps) {
  Blob<N> a{};
  spin_kernel<<<1, 64, 0, s>>>(200000000LL);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(empty_kernel<N>, dim3(64), dim3(64), 0, s, a, out);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}
template <int N> double gpu_us(hipStream_t s, int* out, int reps) {
  Blob<N> a{};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  spin_kernel<<<1, 64, 0, s>>>(20000000LL);
  (void)hipEventRecord(e0, s);
  for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(empty_kernel<N>, dim3(64), dim3(64), 0, s, a, out);
  (void)hipEventRecord(e1, s);
  (void)hipStreamSynchronize(s);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps;
}

// same launches through hipModuleLaunchKernel on a hipFunction_t resolved once (no per-launch
// host-function lookup), arguments as one buffer (extra) or as a parameter array
template <int N> double host_us_module(hipStream_t s, int* out, int reps, bool buffer) {
  struct { Blob<N> a; int* o; } args{};
  args.o = out;
  size_t size = sizeof(args);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  void* params[] = {&args.a, &args.o};
  hipFunction_t f;
  (void)hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&empty_kernel<N>));
  spin_kernel<<<1, 64, 0, s>>>(200000000LL);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; ++k)
    (void)hipModuleLaunchKernel(f, 64, 1, 1, 64, 1, 1, 0, s, buffer ? nullptr : params, buffer ? extra : nullptr);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
  hipStream_t s; (void)hipStreamCreate(&s);
  int* out; (void)hipMalloc(&out, 4096 * sizeof(int)); (void)hipMemset(out, 0, 4096 * sizeof(int));
  for (int w = 0; w < 3; ++w) host_us<16>(s, out, 200);
  printf("host us/launch: 16B %.3f  256B %.3f  640B %.3f  1152B %.3f  2048B %.3f\n", host_us<16>(s, out, 400),
         host_us<256>(s, out, 400), host_us<640>(s, out, 400), host_us<1152>(s, out, 400), host_us<2048>(s, out, 400));
  for (int w = 0; w < 3; ++w) host_us_module<16>(s, out, 200, true);
  printf("host us/module-launch (extra buffer): 16B %.3f  256B %.3f  640B %.3f  1152B %.3f\n",
         host_us_module<16>(s, out, 400, true), host_us_module<256>(s, out, 400, true),
         host_us_module<640>(s, out, 400, true), host_us_module<1152>(s, out, 400, true));
  printf("host us/module-launch (param array):  16B %.3f  256B %.3f  640B %.3f  1152B %.3f\n",
         host_us_module<16>(s, out, 400, false), host_us_module<256>(s, out, 400, false),
         host_us_module<640>(s, out, 400, false), host_us_module<1152>(s, out, 400, false));
  printf("host us/launch again: 16B %.3f  640B %.3f\n", host_us<16>(s, out, 400), host_us<640>(s, out, 400));
  printf("gpu  us/launch: 16B %.3f  256B %.3f  640B %.3f  1152B %.3f  2048B %.3f\n", gpu_us<16>(s, out, 400),
         gpu_us<256>(s, out, 400), gpu_us<640>(s, out, 400), gpu_us<1152>(s, out, 400), gpu_us<2048>(s, out, 400));
  // graph of 16 dependent launches: host cost per replay and GPU time per node
  hipGraph_t g; hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int k = 0; k < 16; ++k) hipLaunchKernelGGL(dep_kernel, dim3(64), dim3(64), 0, s, out);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 10; ++w) (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  spin_kernel<<<1, 64, 0, s>>>(200000000LL);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < 100; ++k) (void)hipGraphLaunch(ge, s);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  printf("graph(16 nodes) host us/replay %.3f\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  spin_kernel<<<1, 64, 0, s>>>(20000000LL);
  (void)hipEventRecord(e0, s);
  for (int k = 0; k < 100; ++k) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(e1, s);
  (void)hipStreamSynchronize(s);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("graph(16 nodes) gpu us/node %.3f\n", ms * 1e3 / 1600);
  spin_kernel<<<1, 64, 0, s>>>(20000000LL);
  (void)hipEventRecord(e0, s);
  for (int k = 0; k < 1600; ++k) hipLaunchKernelGGL(dep_kernel, dim3(64), dim3(64), 0, s, out);
  (void)hipEventRecord(e1, s);
  (void)hipStreamSynchronize(s);
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("eager dep_kernel gpu us/launch %.3f\n", ms * 1e3 / 1600);
  return 0;
}
