// The few HIP names the shared step code (quad_math.h, quad_env.h, philox.h) uses, for its host build
// (quad_host.cpp, -DOUZ_HOST, g++): function-space qualifiers, the vector types, and the device math
// intrinsics in their plain host forms.  Nothing here is compiled into the HIP library.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <cstring>

#define __host__
#define __device__
#define __forceinline__ inline __attribute__((always_inline))

struct float2 { float x, y; };
struct float4 { float x, y, z, w; };
inline float2 make_float2(float x, float y) { return float2{x, y}; }
inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }

// round-to-nearest single operations (the host build never contracts: -ffp-contract=off)
inline float __fadd_rn(float a, float b) { return a + b; }
inline float __fsub_rn(float a, float b) { return a - b; }
inline float __fmul_rn(float a, float b) { return a * b; }
inline float __sinf(float x) { return sinf(x); }
inline float __cosf(float x) { return cosf(x); }
// sin / cos of pi x (the device's sincospif): the product formed in double, so the reduction stays exact
inline void sincospif(float x, float* s, float* c) {
  const double a = 3.14159265358979323846 * (double)x;
  *s = (float)sin(a);
  *c = (float)cos(a);
}
