// Issue cost / latency of the VALU operations a lane-split estimator would use, one wave per CU
// (the 4096-env latency regime).  Shader cycles per instruction from s_memtime around unrolled loops.
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/valu_rates.hip -o scripts/exp/valu_rates && ./scripts/exp/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 256;

template <int MODE>
__global__ void __launch_bounds__(64) probe(float* out, double* outd, long long* cyc, float seed) {
  const int l = threadIdx.x;
  float f[8];
  double d[8];
  for (int k = 0; k < 8; ++k) { f[k] = seed + l * 0.001f + k; d[k] = (double)f[k]; }
  const float a = 1.0000001f, b = 1e-7f;
  const double ad = 1.0000000001, bd = 1e-10;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < kIters; ++it) {
    if constexpr (MODE == 0) {   // 8 independent f32 FMA chains
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = __builtin_fmaf(f[k], a, b);
    } else if constexpr (MODE == 1) {   // 8 independent f64 FMA chains
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = __builtin_fma(d[k], ad, bd);
    } else if constexpr (MODE == 2) {   // one dependent f32 chain
      f[0] = __builtin_fmaf(f[0], a, b);
    } else if constexpr (MODE == 3) {   // one dependent f64 chain
      d[0] = __builtin_fma(d[0], ad, bd);
    } else if constexpr (MODE == 4) {   // 8 independent DPP quad_perm moves (b32, bound_ctrl) feeding adds
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int v = __builtin_amdgcn_mov_dpp(__float_as_int(f[k]), 0x39 /*quad_perm [1,2,3,0]*/, 0xF, 0xF, true);
        f[k] = __int_as_float(v) + b;
      }
    } else if constexpr (MODE == 5) {   // 8 independent f64 DPP moves (two b32 DPP each) feeding f64 adds
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        long long x = __double_as_longlong(d[k]);
        int lo = __builtin_amdgcn_mov_dpp((int)x, 0x39, 0xF, 0xF, true);
        int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), 0x39, 0xF, 0xF, true);
        d[k] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) + bd;
      }
    } else if constexpr (MODE == 9) {   // 24 DPP moves of 8 values computed long before (no hazard), summed
      float g[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f[k]), 0x39, 0xF, 0xF, true))
                                     + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f[k]), 0x4E, 0xF, 0xF, true))
                                     + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f[k]), 0x93, 0xF, 0xF, true));
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = __builtin_fmaf(f[k], a, g[k] * 1e-9f);
    } else if constexpr (MODE == 10) {   // ds_swizzle quad_perm-like moves, 8 independent
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int v = __builtin_amdgcn_ds_swizzle(__float_as_int(f[k]), 0x8039);
        f[k] = __int_as_float(v) + b;
      }
    } else if constexpr (MODE == 6) {   // 8 independent f64 muls
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = d[k] * ad;
    } else if constexpr (MODE == 7) {   // f32<->f64 conversions, 8 independent
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = (double)((float)d[k] + b);
    } else if constexpr (MODE == 8) {   // 8 independent f32 adds with a plain v_mov (no DPP) for reference
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = f[k] + b;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  double sd = 0;
  for (int k = 0; k < 8; ++k) { s += f[k]; sd += d[k]; }
  out[blockIdx.x * 64 + l] = s;
  outd[blockIdx.x * 64 + l] = sd;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int M>
static double run(const char* name, int per_iter) {
  float* o;
  double* od;
  long long* c;
  const int blocks = 256;
  hipMalloc(&o, blocks * 64 * 4);
  hipMalloc(&od, blocks * 64 * 8);
  hipMalloc(&c, blocks * 8);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(probe<M>, dim3(blocks), dim3(64), 0, 0, o, od, c, 1.0f);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  long long mn = h[0];
  for (int i = 0; i < blocks; ++i) mn = h[i] < mn ? h[i] : mn;
  // s_memtime ticks at the shader clock on gfx9 (stamps are shader cycles)
  const double per = (double)mn / (kIters * (double)per_iter);
  printf("%-44s %7.2f cycles per instruction (min over 256 waves, %lld total)\n", name, per, mn);
  hipFree(o); hipFree(od); hipFree(c);
  return per;
}

int main() {
  run<0>("v_fma_f32, 8 independent chains", 8);
  run<1>("v_fma_f64, 8 independent chains", 8);
  run<6>("v_mul_f64, 8 independent", 8);
  run<2>("v_fma_f32, one dependent chain (latency)", 1);
  run<3>("v_fma_f64, one dependent chain (latency)", 1);
  run<8>("v_add_f32, 8 independent", 8);
  run<4>("DPP b32 move + f32 add, 8 independent (per pair)", 8);
  run<5>("f64 DPP (2 b32 DPP) + f64 add, 8 indep (per triple)", 8);
  run<7>("cvt f64->f32, add, cvt f32->f64, 8 indep (per triple)", 8);
  run<9>("3 DPP of old values + 2 add + 1 fma (per 6)", 8);
  run<10>("ds_swizzle + f32 add, 8 indep (per pair)", 8);
  return 0;
}
