// Philox4x32-10 counter-based RNG shared by every kernel (gfx950).
//
// Bit-identical to oracle/philox.py (pinned there by the Random123 known-answer
// vectors).  Every random draw of the step is a pure function of
// (seed, global_env_id, step, stream, sub), so results do not depend on launch
// order or on how many GPUs the envs are sharded over.  The reference instead
// draws from torch's global generators (ekf_lee_landed.py:284-286,
// ouzelum.py:183-184, utils/POMDP.py:25,30), which no other device can replay.
#pragma once
#include <stdint.h>

#ifndef OUZ_HD
#define OUZ_HD __host__ __device__ __forceinline__
#endif

namespace ouz {

enum RngStream : uint32_t {
  RNG_RESET_POS = 1,
  RNG_TARGET = 2,
  RNG_TRAJ = 3,
  RNG_DR = 4,
  RNG_FAULT = 5,
  RNG_DRN_OBS = 6,  // VecTask DR noise on observations (vec_task.py:576-646)
  RNG_DRN_ACT = 7,  // ... on actions
  RNG_GRAV = 8,     // sim_params.gravity DR (vec_task.py:648-660): one whole-batch draw per epoch, env BATCH_ENV
  RNG_POMDP = 16,  // + call site
};
constexpr uint32_t BATCH_ENV = 0xFFFFFFFFu;
constexpr uint32_t INIT_STEP = 0xFFFFFFFFu;
enum PomdpSite : uint32_t { SITE_OBS = 0, SITE_GYR = 1, SITE_ANG = 2, SITE_ACC = 3, SITE_POS = 4, SITE_VEL = 5,
                            SITE_LEARNER = 6 /* learner-side POMDPWrapper (RPO-LSTM/main.py:103) */ };

struct U4 { uint32_t x, y, z, w; };

OUZ_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

OUZ_HD U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c0, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c2, hi1, lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

OUZ_HD U4 draw(uint64_t seed, uint32_t env, uint32_t step, uint32_t stream, uint32_t sub = 0) {
  return philox4x32_10(env, step, (stream << 8) | sub, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// [0,1) with 24 random bits, exact in f32.
OUZ_HD float unit_f32(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// lo + (hi - lo) * u with each op rounded separately (no FMA contraction), so the
// CPU oracle's float32 numpy expression gives the same bits.
OUZ_HD float uniform_f32(uint32_t x, float lo, float hi) {
#pragma clang fp contract(off)   // two roundings, never an FMA (the oracle's numpy order)
#if defined(__HIP_DEVICE_COMPILE__)
  // (hi - lo) * unit_f32(x) with the 2^-24 scale moved onto the span: both scalings by a power of two are
  // exact (spans are normal floats), so the one rounding of the product is the same -- one multiply less
  // per draw (QuadFault draws 13 noise factors per env-step)
  const float span_s = (hi - lo) * (1.0f / 16777216.0f);
  return lo + span_s * (float)(x >> 8);
#else
  volatile float span = hi - lo;
  volatile float m = span * unit_f32(x);
  return lo + m;
#endif
}

}  // namespace ouz
