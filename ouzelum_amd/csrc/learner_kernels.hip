// Learner-side kernels for the recurrent PPO/RPO loop.
//
//  * ouz_gae: generalized advantage estimation over a (T, N) rollout, one env per
//    lane walking t = T-1 .. 0 in registers.  Replaces the reference's Python loop
//    of ~6 torch launches per time step (RPO-LSTM/agent.py:40-55) with one launch;
//    the f32 operation order is the torch one, so results are bit-identical to the
//    reference formula evaluated in float32 (oracle/learner_oracle.py::gae_f32).
//  * ouz_pomdp_obs: the learner's POMDPWrapper.observation (utils/POMDP.py:23-43)
//    on device with the counter RNG, keyed (seed, global row, call index), instead
//    of a CPU torch.rand coin + a CPU noise tensor copied H2D every step.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ouzelum.h"
#include "philox.h"

int set_error(int code, const std::string& msg);   // quad_kernels.hip

namespace {

using namespace ouz;

__global__ void __launch_bounds__(256) gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ done, const float* __restrict__ next_val,
                                                  const float* __restrict__ next_done, int T, int N, float gamma,
                                                  float gamma_lam, float* __restrict__ adv, float* __restrict__ ret) {
#pragma clang fp contract(off)   // torch's f32 op order, one rounding per operation
  // (plain operators: the __f*_rn helpers are header functions outside this pragma's scope)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float last = 0.0f;
  float nv = next_val[i];
  float nnt = 1.0f - next_done[i];
  for (int t = T - 1; t >= 0; --t) {
    const size_t k = (size_t)t * N + i;
    const float v = val[k];
    // delta = r + gamma * nv * nnt - v ; adv = delta + (gamma*lam) * nnt * last   (torch f32 op order)
    const float delta = (rew[k] + (gamma * nv) * nnt) - v;
    last = delta + (gamma_lam * nnt) * last;
    adv[k] = last;
    ret[k] = last + v;
    nv = v;
    nnt = 1.0f - done[k];
  }
}

__global__ void __launch_bounds__(256) pomdp_obs_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        int rows, int dim, int zero, int noise, float lo, float hi,
                                                        uint64_t seed, uint32_t row0, uint32_t call) {
#pragma clang fp contract(off)
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* x = in + (size_t)r * dim;
  float* y = out + (size_t)r * dim;
  for (int g = 0; g < (dim + 3) / 4; ++g) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (noise) {
      U4 u = draw(seed, row0 + (uint32_t)r, call, RNG_POMDP + SITE_LEARNER, 128u + (uint32_t)g);
      w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = g * 4 + k;
      if (e < dim) {
        float v = zero ? 0.0f : x[e];
        if (noise) v = v * uniform_f32(w[k], lo, hi);
        y[e] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Fused LSTM cell (RPO-LSTM/model.py:27-50, torch's gate order i, f, g, o).  The recurrent
// GEMM gates = x W_ih^T + b + h W_hh^T stays in hipBLASLt; everything element-wise around it —
// 4 activations, the cell update, tanh(c), the done-mask of the NEXT step's carry and the
// saved activations for BPTT — is one launch per step instead of ~10 torch kernels.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void __launch_bounds__(256) lstm_cell_fwd_kernel(const float* __restrict__ gates,
                                                            const float* __restrict__ c_prev_m,
                                                            const float* __restrict__ keep_next,
                                                            float* __restrict__ act, float* __restrict__ c_out,
                                                            float* __restrict__ h_out, float* __restrict__ h_next_m,
                                                            float* __restrict__ c_next_m, int B, int H) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx - b * H;
  const float* g = gates + (size_t)b * 4 * H;
  const float ig = sigm(g[j]), fg = sigm(g[H + j]), gg = tanhf(g[2 * H + j]), og = sigm(g[3 * H + j]);
  const float c = fg * c_prev_m[idx] + ig * gg;
  const float h = og * tanhf(c);
  float* a = act + (size_t)b * 4 * H;
  a[j] = ig; a[H + j] = fg; a[2 * H + j] = gg; a[3 * H + j] = og;
  c_out[idx] = c;
  h_out[idx] = h;
  const float k = keep_next ? keep_next[b] : 1.0f;
  h_next_m[idx] = k * h;
  c_next_m[idx] = k * c;
}

// BPTT for one step.  dh = dhid + keep_next * G (G = dgates_{t+1} W_hh, null at the last step),
// dc = dc_next * keep_next (dc_next = the next step's d c_prev, or the loss's dcT at the last step).
__global__ void __launch_bounds__(256) lstm_cell_bwd_kernel(const float* __restrict__ act, const float* __restrict__ c,
                                                            const float* __restrict__ c_prev_m,
                                                            const float* __restrict__ dhid, const float* __restrict__ G,
                                                            const float* __restrict__ dc_next,
                                                            const float* __restrict__ keep_next,
                                                            float* __restrict__ dgates, float* __restrict__ dc_prev,
                                                            int B, int H) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx - b * H;
  const float k = keep_next ? keep_next[b] : 1.0f;
  const float dh = dhid[idx] + (G ? k * G[idx] : 0.0f);
  const float* a = act + (size_t)b * 4 * H;
  const float ig = a[j], fg = a[H + j], gg = a[2 * H + j], og = a[3 * H + j];
  const float tc = tanhf(c[idx]);
  const float dc = (dc_next ? k * dc_next[idx] : 0.0f) + dh * og * (1.0f - tc * tc);
  float* d = dgates + (size_t)b * 4 * H;
  d[j] = dc * gg * ig * (1.0f - ig);
  d[H + j] = dc * c_prev_m[idx] * fg * (1.0f - fg);
  d[2 * H + j] = dc * ig * (1.0f - gg * gg);
  d[3 * H + j] = dh * tc * og * (1.0f - og);
  dc_prev[idx] = dc * fg;
}

inline int grid(int n, int b) { return (n + b - 1) / b; }

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(OUZ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return OUZ_OK;
}

}  // namespace

extern "C" {

int ouz_gae(const float* rewards, const float* values, const float* dones, const float* next_value,
            const float* next_done, int32_t T, int32_t N, float gamma, float gamma_lam, float* advantages,
            float* returns, void* stream) {
  if (T <= 0 || N <= 0) return set_error(OUZ_ERR_INVALID, "ouz_gae: T and N must be > 0");
  if (!rewards || !values || !dones || !next_value || !next_done || !advantages || !returns)
    return set_error(OUZ_ERR_INVALID, "ouz_gae: null buffer");
  hipLaunchKernelGGL(gae_kernel, dim3(grid(N, 256)), dim3(256), 0, (hipStream_t)stream, rewards, values, dones,
                     next_value, next_done, T, N, gamma, gamma_lam, advantages, returns);
  return launch_status("gae_kernel");
}

int ouz_pomdp_obs(const float* in, float* out, int32_t rows, int32_t dim, int32_t mode, float prob, uint64_t seed,
                  int64_t row_offset, uint32_t call, void* stream) {
  if (rows < 0 || dim <= 0 || dim > 64) return set_error(OUZ_ERR_INVALID, "ouz_pomdp_obs: bad shape");
  if (rows > 0 && (!in || !out)) return set_error(OUZ_ERR_INVALID, "ouz_pomdp_obs: null buffer");
  if (row_offset < 0 || row_offset + rows > 0xFFFFFFFFll) return set_error(OUZ_ERR_INVALID, "ouz_pomdp_obs: bad row offset");
  int zero = 0, noise = 0;
  switch (mode) {
    case OUZ_POMDP_NONE: break;
    case OUZ_POMDP_FLICKER:
    case OUZ_POMDP_FLICKER_NOISE: {
      // one coin per call for the whole batch (POMDP.py:25,35): host-side, same key as the oracle
      const float p = mode == OUZ_POMDP_FLICKER ? prob : 0.1f;
      zero = unit_f32(draw(seed, BATCH_ENV, call, RNG_POMDP + SITE_LEARNER, 0u).x) <= p;
      noise = mode == OUZ_POMDP_FLICKER_NOISE;
      break;
    }
    case OUZ_POMDP_NOISE: noise = 1; break;
    default: return set_error(OUZ_ERR_INVALID, "ouz_pomdp_obs: unknown mode");
  }
  if (rows == 0) return OUZ_OK;
  // noise range 1 -/+ sigma rounded to f32 like the in-env sites (POMDP.py:10)
  const float lo = (float)(1.0 - (double)prob), hi = (float)(1.0 + (double)prob);
  hipLaunchKernelGGL(pomdp_obs_kernel, dim3(grid(rows, 256)), dim3(256), 0, (hipStream_t)stream, in, out, rows, dim,
                     zero, noise, lo, hi, seed, (uint32_t)row_offset, call);
  return launch_status("pomdp_obs_kernel");
}

int ouz_lstm_cell_fwd(const float* gates, const float* c_prev_m, const float* keep_next, float* act, float* c_out,
                      float* h_out, float* h_next_m, float* c_next_m, int32_t B, int32_t H, void* stream) {
  if (B <= 0 || H <= 0) return set_error(OUZ_ERR_INVALID, "ouz_lstm_cell_fwd: B and H must be > 0");
  if (!gates || !c_prev_m || !act || !c_out || !h_out || !h_next_m || !c_next_m)
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_cell_fwd: null buffer");
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(grid(B * H, 256)), dim3(256), 0, (hipStream_t)stream, gates, c_prev_m,
                     keep_next, act, c_out, h_out, h_next_m, c_next_m, B, H);
  return launch_status("lstm_cell_fwd_kernel");
}

int ouz_lstm_cell_bwd(const float* act, const float* c, const float* c_prev_m, const float* dhid, const float* G,
                      const float* dc_next, const float* keep_next, float* dgates, float* dc_prev, int32_t B, int32_t H,
                      void* stream) {
  if (B <= 0 || H <= 0) return set_error(OUZ_ERR_INVALID, "ouz_lstm_cell_bwd: B and H must be > 0");
  if (!act || !c || !c_prev_m || !dhid || !dgates || !dc_prev)
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_cell_bwd: null buffer");
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(grid(B * H, 256)), dim3(256), 0, (hipStream_t)stream, act, c, c_prev_m,
                     dhid, G, dc_next, keep_next, dgates, dc_prev, B, H);
  return launch_status("lstm_cell_bwd_kernel");
}

}  // extern "C"
