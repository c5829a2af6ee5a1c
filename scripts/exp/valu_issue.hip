// Issue rate of one wave64 on an otherwise idle SIMD (gfx950): a dependent chain of v_fma_f32, two and four
// interleaved independent chains, a dependent chain of v_pk_fma_f32 (two f32 FMAs per lane per instruction),
// and dependent v_sqrt_f32 / v_rcp_f32 / v_mul_f32.  Cycles per instruction from s_memtime around 1024
// instructions; one 64-thread workgroup, so the wave has its SIMD to itself.  Answers whether the latency-
// regime step (one wave per SIMD) is bound by issue (4 cycles per wave64 VALU op) or by dependent latency, and
// whether packed FP32 halves the issue cost of paired f32 math.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_issue scripts/exp/valu_issue.hip && /tmp/valu_issue
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void probe(float* out, unsigned long long* cyc, float a, float b) {
  float x = out[threadIdx.x], y = x + 1.0f, z = x + 2.0f, w = x + 3.0f;
  f2 p = {x, y}, pa = {a, a}, pb = {b, b};
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (MODE == 0) {
    asm volatile(".rept 1024\n v_fma_f32 %0, %0, %1, %2\n .endr" : "+v"(x) : "v"(a), "v"(b));
  } else if constexpr (MODE == 1) {
    asm volatile(".rept 512\n v_fma_f32 %0, %0, %2, %3\n v_fma_f32 %1, %1, %2, %3\n .endr" : "+v"(x), "+v"(y) : "v"(a), "v"(b));
  } else if constexpr (MODE == 2) {
    asm volatile(".rept 256\n v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n"
                 " v_fma_f32 %3, %3, %4, %5\n .endr" : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(b));
  } else if constexpr (MODE == 3) {
    asm volatile(".rept 1024\n v_pk_fma_f32 %0, %0, %1, %2\n .endr" : "+v"(p) : "v"(pa), "v"(pb));
  } else if constexpr (MODE == 4) {
    asm volatile(".rept 1024\n v_sqrt_f32 %0, %0\n .endr" : "+v"(x));
  } else if constexpr (MODE == 5) {
    asm volatile(".rept 1024\n v_rcp_f32 %0, %0\n .endr" : "+v"(x));
  } else if constexpr (MODE == 6) {
    asm volatile(".rept 1024\n v_mul_f32 %0, %0, %1\n .endr" : "+v"(x) : "v"(a));
  } else if constexpr (MODE == 7) {
    asm volatile(".rept 512\n v_pk_fma_f32 %0, %0, %2, %3\n v_pk_fma_f32 %1, %1, %2, %3\n .endr" : "+v"(p), "+v"(pb) : "v"(pa), "v"(pa));
  } else if constexpr (MODE == 8) {
    asm volatile(".rept 1024\n s_add_u32 s0, s0, 1\n .endr" ::: "s0", "scc");
  } else if constexpr (MODE == 9) {   // VOP2 accumulate form: x = a * b + x
    asm volatile(".rept 1024\n v_fmac_f32 %0, %1, %2\n .endr" : "+v"(x) : "v"(a), "v"(b));
  } else if constexpr (MODE == 10) {  // VOP3 fma, the chain through the addend
    asm volatile(".rept 1024\n v_fma_f32 %0, %1, %2, %0\n .endr" : "+v"(x) : "v"(a), "v"(b));
  } else if constexpr (MODE == 11) {  // VOP3 encoding of a multiply
    asm volatile(".rept 1024\n v_mul_f32_e64 %0, %0, %1\n .endr" : "+v"(x) : "v"(a));
  } else if constexpr (MODE == 12) {
    asm volatile(".rept 1024\n v_add_f32 %0, %0, %1\n .endr" : "+v"(x) : "v"(a));
  } else if constexpr (MODE == 13) {
    asm volatile(".rept 1024\n v_pk_mul_f32 %0, %0, %1\n .endr" : "+v"(p) : "v"(pa));
  } else if constexpr (MODE == 14) {
    asm volatile(".rept 1024\n v_pk_add_f32 %0, %0, %1\n .endr" : "+v"(p) : "v"(pa));
  } else if constexpr (MODE == 15) {  // pk fma, the chain through the addend
    asm volatile(".rept 1024\n v_pk_fma_f32 %0, %1, %2, %0\n .endr" : "+v"(p) : "v"(pa), "v"(pb));
  } else if constexpr (MODE == 16) {  // fma chain with the product operand from a freshly written register
    asm volatile(".rept 512\n v_mul_f32 %1, %1, %2\n v_fma_f32 %0, %1, %2, %0\n .endr" : "+v"(x), "+v"(y) : "v"(a));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[threadIdx.x] = x + y + z + w + p.x + p.y + pb.x;
  if (threadIdx.x == 0) { cyc[MODE] = t1 - t0; cyc[32 + MODE] = r1 - r0; }
}

int main() {
  float* d;
  unsigned long long* c;
  if (hipMalloc(&d, 256 * sizeof(float)) != hipSuccess || hipMalloc(&c, 64 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  if (hipMemset(d, 0, 256 * sizeof(float)) != hipSuccess) return 1;
  const char* names[] = {"v_fma_f32 dependent", "v_fma_f32 2 chains", "v_fma_f32 4 chains", "v_pk_fma_f32 dependent",
                         "v_sqrt_f32 dependent", "v_rcp_f32 dependent", "v_mul_f32 dependent",
                         "v_pk_fma_f32 2 chains", "s_add_u32 dependent", "v_fmac_f32 dependent (VOP2)",
                         "v_fma_f32 dependent through the addend", "v_mul_f32_e64 dependent", "v_add_f32 dependent",
                         "v_pk_mul_f32 dependent", "v_pk_add_f32 dependent", "v_pk_fma_f32 dependent through the addend",
                         "v_mul_f32 + v_fma_f32 pairs (per instruction)"};
  unsigned long long h[64];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<5>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<6>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<7>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<8>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<9>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<10>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<11>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<12>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<13>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<14>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<15>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    hipLaunchKernelGGL(probe<16>, dim3(1), dim3(64), 0, 0, d, c, 1.0001f, 0.5f);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  unsigned long long r[64];
  if (hipMemcpy(r, c, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int m = 0; m < 17; ++m)
    std::printf("{\"probe\": \"%s\", \"instructions\": 1024, \"cycles\": %llu, \"cycles_per_instruction\": %.2f, "
                "\"realtime_100MHz_ticks\": %llu, \"memtime_GHz\": %.3f}\n",
                names[m], h[m], h[m] / 1024.0, r[32 + m], r[32 + m] ? h[m] / (r[32 + m] * 10.0) : 0.0);
  return hipFree(d) == hipSuccess && hipFree(c) == hipSuccess ? 0 : 1;
}
