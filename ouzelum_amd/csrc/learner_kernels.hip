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

#include <algorithm>
#include <cmath>
#include <cstdlib>
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

// ---------------------------------------------------------------------------
// PPO losses of one minibatch (RPO-LSTM/agent.py:86-110, PPO/agent.py): the clipped policy loss with the
// advantage normalisation, and the value loss, each as a forward that also writes the loss's gradient with
// respect to its inputs for a unit upstream gradient (the loss is the end of the graph; the autograd
// wrapper scales it).  torch's form is ~60 element-wise / reduction launches per minibatch (Normal.log_prob,
// exp, max / clamp and their backward, six means); here 3 + 2.  Reductions are deterministic: per-block
// f64 partials in a fixed grid (kLossBlocks), summed in block order by one finishing block.
// ---------------------------------------------------------------------------
constexpr int kLossThreads = 256;
constexpr int kLossBlocks = OUZ_LOSS_BLOCKS;

// sum over the block of v (f64), deterministic (fixed shuffle tree, then the 4 waves in order); all threads
// receive the total
__device__ double block_sum(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kLossThreads / 64; ++k) t += sh[k];
  return t;
}

__global__ void __launch_bounds__(kLossThreads) adv_moments_kernel(const float* __restrict__ adv, int n,
                                                                   double* __restrict__ part) {
  __shared__ double sh[kLossThreads / 64];
  double s = 0.0, ss = 0.0;
  for (int i = blockIdx.x * kLossThreads + threadIdx.x; i < n; i += kLossBlocks * kLossThreads) {
    const double a = adv[i];
    s += a;
    ss += a * a;
  }
  s = block_sum(s, sh);
  ss = block_sum(ss, sh);
  if (threadIdx.x == 0) { part[2 * blockIdx.x] = s; part[2 * blockIdx.x + 1] = ss; }
}

// Normal(mean_z, exp(logstd)).log_prob(action).sum(1) as torch/distributions/normal.py forms it (scale = exp,
// var = scale**2, log_scale = log(scale)), the ratio against the rollout's log-prob, the clipped surrogate and
// its gradient, with torch's tie rule for maximum (equal arguments share the gradient) and clamp's inclusive
// pass-through.  Per row: dmean (n, 4) for a unit upstream gradient; per block: loss, approx-kl and clip-count
// sums and the four logstd gradient sums.
__global__ void __launch_bounds__(kLossThreads) policy_loss_kernel(
    const float* __restrict__ mean_z, const float* __restrict__ logstd, const float* __restrict__ act,
    const float* __restrict__ old_logp, const float* __restrict__ adv, int n, float clip, int norm_adv,
    const double* __restrict__ adv_part, float* __restrict__ dmean, double* __restrict__ part) {
#pragma clang fp contract(off)
  __shared__ double sh[kLossThreads / 64];
  float mu = 0.0f, den = 1.0f;
  if (norm_adv) {   // (adv - adv.mean()) / (adv.std() + 1e-8), std unbiased; moments summed by block_sum's fixed tree
    static_assert(kLossBlocks == kLossThreads, "one thread per partial block");
    const double s = block_sum(adv_part[2 * threadIdx.x], sh);
    const double ss = block_sum(adv_part[2 * threadIdx.x + 1], sh);
    const double m = s / n;
    const double var = (ss - s * m) / (double)(n - 1);
    mu = (float)m;
    den = (float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f;
  }
  float sd[OUZ_NUM_ACT], var[OUZ_NUM_ACT], lsc[OUZ_NUM_ACT];
#pragma unroll
  for (int j = 0; j < OUZ_NUM_ACT; ++j) {
    sd[j] = expf(logstd[j]);
    var[j] = sd[j] * sd[j];
    lsc[j] = logf(sd[j]);
  }
  const float kLogSqrt2Pi = 0.918938533204672742f;
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  const float inv_n = 1.0f / (float)n;
  double s_loss = 0.0, s_kl = 0.0, s_cf = 0.0, s_ls[OUZ_NUM_ACT] = {0.0, 0.0, 0.0, 0.0};
  for (int i = blockIdx.x * kLossThreads + threadIdx.x; i < n; i += kLossBlocks * kLossThreads) {
    const float4 m4 = reinterpret_cast<const float4*>(mean_z)[i];
    const float4 a4 = reinterpret_cast<const float4*>(act)[i];
    const float d[OUZ_NUM_ACT] = {a4.x - m4.x, a4.y - m4.y, a4.z - m4.z, a4.w - m4.w};
    float lp = 0.0f;
#pragma unroll
    for (int j = 0; j < OUZ_NUM_ACT; ++j) lp += ((-(d[j] * d[j])) / (2.0f * var[j]) - lsc[j]) - kLogSqrt2Pi;
    const float logratio = lp - old_logp[i];
    const float ratio = expf(logratio);
    const float a = norm_adv ? (adv[i] - mu) / den : adv[i];
    const float na = -a;
    const float l1 = na * ratio;
    const float cr = fminf(fmaxf(ratio, lo), hi);
    const float l2 = na * cr;
    s_loss += (double)fmaxf(l1, l2);
    s_kl += (double)((ratio - 1.0f) - logratio);
    s_cf += fabsf(ratio - 1.0f) > clip ? 1.0 : 0.0;
    // d loss / d ratio for loss = mean(max(l1, l2)): maximum's backward gives each side the gradient where it is
    // the larger and half of it on a tie; clamp passes its gradient where lo <= ratio <= hi
    const float g = inv_n;
    const float g1 = l1 > l2 ? g : (l1 == l2 ? g * 0.5f : 0.0f);
    const float g2 = l2 > l1 ? g : (l1 == l2 ? g * 0.5f : 0.0f);
    const float dratio = g1 * na + ((ratio >= lo && ratio <= hi) ? g2 * na : 0.0f);
    const float dlp = dratio * ratio;   // exp's backward; logratio = lp - old
    float4 dm;
    dm.x = dlp * d[0] / var[0];
    dm.y = dlp * d[1] / var[1];
    dm.z = dlp * d[2] / var[2];
    dm.w = dlp * d[3] / var[3];
    reinterpret_cast<float4*>(dmean)[i] = dm;
#pragma unroll
    for (int j = 0; j < OUZ_NUM_ACT; ++j) s_ls[j] += (double)(dlp * (d[j] * d[j] / var[j] - 1.0f));
  }
  s_loss = block_sum(s_loss, sh);
  s_kl = block_sum(s_kl, sh);
  s_cf = block_sum(s_cf, sh);
#pragma unroll
  for (int j = 0; j < OUZ_NUM_ACT; ++j) s_ls[j] = block_sum(s_ls[j], sh);
  if (threadIdx.x == 0) {
    double* p = part + 8 * blockIdx.x;
    p[0] = s_loss; p[1] = s_kl; p[2] = s_cf;
#pragma unroll
    for (int j = 0; j < OUZ_NUM_ACT; ++j) p[3 + j] = s_ls[j];
  }
}

// 0.5 * mean((v - r)^2) (agent.py:104-105 with clip_vloss False) and dv = (v - r) / n for a unit upstream gradient
__global__ void __launch_bounds__(kLossThreads) value_loss_kernel(const float* __restrict__ v,
                                                                  const float* __restrict__ r, int n,
                                                                  float* __restrict__ dv, double* __restrict__ part) {
#pragma clang fp contract(off)
  __shared__ double sh[kLossThreads / 64];
  const float inv_n = 1.0f / (float)n;
  double s = 0.0;
  for (int i = blockIdx.x * kLossThreads + threadIdx.x; i < n; i += kLossBlocks * kLossThreads) {
    const float d = v[i] - r[i];
    s += (double)(d * d);
    dv[i] = d * inv_n;
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[8 * blockIdx.x] = s;
}

// One block, one thread per partial block: out_k = (sum over blocks of part[8 b + k]) * scale for k < 3 (the
// means); k >= 3: dlogstd[k - 3] = the sum itself (dlp already carries 1 / n).  Each sum is block_sum's fixed tree.
static_assert(kLossBlocks == kLossThreads, "loss_finish_kernel: one thread per partial block");
__global__ void __launch_bounds__(kLossThreads) loss_finish_kernel(const double* __restrict__ part, int nk,
                                                                   double scale, float* __restrict__ o0,
                                                                   float* __restrict__ o1, float* __restrict__ o2,
                                                                   float* __restrict__ o3) {
  __shared__ double sh[kLossThreads / 64];
  const double* p = part + 8 * threadIdx.x;
  for (int k = 0; k < nk; ++k) {
    const double t = block_sum(p[k], sh);
    if (threadIdx.x == 0) {
      if (k == 0) *o0 = (float)(t * scale);
      else if (k == 1) *o1 = (float)(t * scale);
      else if (k == 2) *o2 = (float)(t * scale);
      else o3[k - 3] = (float)t;
    }
  }
}

// ---------------------------------------------------------------------------
// Backward of y = tanh(x W^T + b) for the MLP trunks (RPO-LSTM/model.py:17-24,72-84): dz = dy (1 - y^2)
// (torch's tanh_backward) and the bias gradient db = sum over rows of dz in the same pass, instead of a
// tanh_backward launch and a column-sum launch that reads dz again.  Rows are split over a fixed grid
// (deterministic: per-block column partials, then a column-wise sum in block order).
// ---------------------------------------------------------------------------
constexpr int kColBlocks = OUZ_COLSUM_BLOCKS;

__global__ void __launch_bounds__(256) tanh_bwd_colsum_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ y, float* __restrict__ dz,
                                                              float* __restrict__ part, int rows, int cols) {
#pragma clang fp contract(off)
  __shared__ float4 sh[256];
  const int cg = cols >> 2;                 // float4 column groups; 256 % cg == 0 (host-checked)
  const int rp = 256 / cg;                  // rows per pass
  const int c4 = threadIdx.x % cg, r0 = threadIdx.x / cg;
  const int per = (rows + kColBlocks - 1) / kColBlocks;
  const int rb = blockIdx.x * per, re = min(rows, rb + per);
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll 4
  for (int r = rb + r0; r < re; r += rp) {
    const size_t k = (size_t)r * cg + c4;
    const float4 g = reinterpret_cast<const float4*>(dy)[k];
    const float4 t = reinterpret_cast<const float4*>(y)[k];
    float4 o;
    o.x = g.x * (1.0f - t.x * t.x);
    o.y = g.y * (1.0f - t.y * t.y);
    o.z = g.z * (1.0f - t.z * t.z);
    o.w = g.w * (1.0f - t.w * t.w);
    reinterpret_cast<float4*>(dz)[k] = o;
    acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  if (r0 == 0) {
    for (int q = 1; q < rp; ++q) {
      const float4 b = sh[q * cg + c4];
      acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    }
    reinterpret_cast<float4*>(part)[(size_t)blockIdx.x * cg + c4] = acc;
  }
}

// db[c] = sum over the kColBlocks partial rows, 16 columns per block: the block's 16 row groups (threadIdx / 16)
// each sum partial rows g, g + 16, ... in order (64 loads per thread, 8 in flight), then the 16 group sums are added
// in group order
__global__ void __launch_bounds__(256) colsum_finish_kernel(const float* __restrict__ part, int cols,
                                                            float* __restrict__ db) {
  __shared__ float sh[16][16];
  const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
  const int c = blockIdx.x * 16 + l;
  float t = 0.0f;
  if (c < cols) {
#pragma unroll 8
    for (int b = g; b < kColBlocks; b += 16) t += part[(size_t)b * cols + c];
  }
  sh[g][l] = t;
  __syncthreads();
  if (g == 0 && c < cols) {
    float s = sh[0][l];
#pragma unroll
    for (int q = 1; q < 16; ++q) s += sh[q][l];
    db[c] = s;
  }
}

// ---------------------------------------------------------------------------
// The rollout policy's head and sample in one launch (RPO-LSTM/model.py:52-70 get_action_and_value with
// action None; PPO/model.py:31-40): mean = h W^T + b (A = 4 actions), action = mean + exp(logstd) eps, and the
// Normal log-prob / entropy summed over the actions in the form of models._sample_head:
//   log-prob = -1/2 sum eps^2 - (sum logstd + A log sqrt(2 pi)),  entropy = sum logstd + A (1/2 + log sqrt(2 pi)).
// Four threads per row, one per action (the row's hidden vector read once per wave: the four lanes share each
// address); the log-prob's sum over actions is a shuffle across the four lanes.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) policy_sample_kernel(const float* __restrict__ hid, const float* __restrict__ w,
                                                            const float* __restrict__ b,
                                                            const float* __restrict__ logstd,
                                                            const float* __restrict__ eps, int B, int H,
                                                            float* __restrict__ action, float* __restrict__ logprob,
                                                            float* __restrict__ entropy) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int row = t >> 2, a = t & 3;
  const bool live = row < B;
  float dot = 0.0f;
  if (live) {
    const float4* hr = reinterpret_cast<const float4*>(hid + (size_t)row * H);
    const float4* wr = reinterpret_cast<const float4*>(w + (size_t)a * H);
    for (int k = 0; k < (H >> 2); ++k) {
      const float4 hv = hr[k], wv = wr[k];
      dot = fmaf(hv.x, wv.x, dot);
      dot = fmaf(hv.y, wv.y, dot);
      dot = fmaf(hv.z, wv.z, dot);
      dot = fmaf(hv.w, wv.w, dot);
    }
  }
  const float ls = logstd[a];
  const float e = live ? eps[(size_t)row * OUZ_NUM_ACT + a] : 0.0f;
  const float m = dot + b[a];
  // -1/2 sum eps^2 over the row's four lanes (lanes 4j .. 4j+3 of the wave)
  float q = e * e;
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  float lsum = ls;
  lsum += __shfl_xor(lsum, 1, 64);
  lsum += __shfl_xor(lsum, 2, 64);
  const float kLogSqrt2Pi = 0.918938533204672742f;
  const float c = lsum + (float)OUZ_NUM_ACT * kLogSqrt2Pi;
  if (!live) return;
  action[(size_t)row * OUZ_NUM_ACT + a] = m + expf(ls) * e;
  if (a == 0) {
    logprob[row] = -c + (-0.5f) * q;
    entropy[row] = c + 0.5f * (float)OUZ_NUM_ACT;
  }
}

// ---------------------------------------------------------------------------
// The whole done-masked LSTM recurrence of one sequence in ONE launch, forward and BPTT (RPO-LSTM/model.py:34-50;
// torch's gate order i, f, g, o), for hidden size 128 (the reference actor's LSTM(256, 128)).  A row's carry
// depends on that row only, so each workgroup owns 16 batch rows for all T steps and needs no grid
// synchronisation: the carry stays on chip (c in registers, the masked h in LDS as the next step's MFMA operand)
// instead of 2 launches + 4 B x H round trips per step.  The recurrent product runs on the f32 MFMA
// (v_mfma_f32_16x16x4_f32, exact f32 products, f32 accumulation).
//   wave w of the workgroup owns hidden units [32 w, 32 w + 32): two 16-unit blocks jb, and for each the four
//   gate tiles (gate rows q H + 32 w + 16 jb + [0, 16), q = i, f, g, o), so a lane's accumulators hold all four gates
//   of its (row, unit) elements and the cell update needs no data movement.  The product is computed transposed,
//   gates^T = W_hh h^T (the weight fragment is the MFMA's A operand, the carry tile its B operand), so that with the
//   MFMA's C / D map (lane l holds rows 4 (l >> 4) + r, r = 0..3, of column l & 15) a lane holds FOUR CONSECUTIVE
//   hidden units of ONE batch row: every global load and store of a step is one 16-byte access per lane (a
//   16-row x 64-byte block per instruction), 4x fewer memory instructions than the untransposed map, whose lanes
//   held one unit of four rows.  The K loop visits k in the order 16 p + 4 (l >> 4) + s (p: 16-wide slab, s = 0..3
//   the MFMA's step), so every lane's operands of four consecutive steps are one 16-byte load (LDS for the carry /
//   gradient tile, registers for the weights).
// ---------------------------------------------------------------------------
constexpr int kSeqH = 128;
constexpr int kSeqG = 4 * kSeqH;
constexpr int kSeqRows = 16;
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(f32x4 a, f32x4 b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
}
// The cell's transcendentals in the sequence kernels from the hardware's exp2 / reciprocal (v_exp_f32, v_rcp_f32,
// ~1 ulp each): 4 and 7 instructions against ~12 and ~30 for the libm forms the per-step cell kernels keep.  sigmoid
// to ~3 ulp; tanh to ~1e-7 absolute (1 - t loses the relative precision of tanh near 0, not its absolute one).
__device__ __forceinline__ float fsigm(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
__device__ __forceinline__ float ftanh(float x) {
  const float t = __builtin_amdgcn_exp2f(-2.88539008177792681f * fabsf(x));   // exp(-2|x|) in (0, 1]
  return copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), x);
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// Forward over T steps.  x_proj [T][B][4H] = x W_ih^T + b (pre-activation without the recurrent term), h0 / c0 [B][H],
// keep [T][B] (1 - done: zeroes the carry entering step t), w [4H][H] (W_hh).  Writes, as the per-step path does,
// act [T][B][4H] (activated gates), c_all / hid [T][B][H] and the masked carries hm / cm [T + 1][B][H] entering each
// step (row T: the final carry, or h_out / c_out when given).  act, c_all, hm, cm may be null (inference).  Every
// [.][B][.] buffer is 16-byte aligned (ouz_lstm_seq_fwd checks).
// FULL: all 16 rows of the workgroup are valid (every workgroup but a ragged last one), so no load or store is
// predicated.  SAVED: act / c_all / hm / cm are written (training; all four or none).  With a fixed number of stores
// per step, the waitcnt pass can wait for a prefetched input with vmcnt(stores issued since) instead of vmcnt(0),
// which drained the step's stores before the next step could start.
template <int NJB, bool FULL, bool SAVED>
__device__ __forceinline__ void lstm_seq_fwd_body(
    float (*sh)[kSeqRows][kSeqH + 4], const float* __restrict__ xp, const float* h0, const float* c0,
    const float* __restrict__ keep, const float* __restrict__ w, int T, int B, float* __restrict__ act,
    float* __restrict__ c_all, float* __restrict__ hid, float* __restrict__ hm, float* __restrict__ cm, float* h_out,
    float* c_out) {
  // (h_out / c_out may alias h0 / c0: each workgroup reads its rows of h0 / c0 first and writes the same rows last)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.x * kSeqRows;
  for (int e = threadIdx.x; e < kSeqRows * kSeqH; e += 512 / NJB) {
    const int row = e / kSeqH, j = e - row * kSeqH, b = r0 + row;
    const float v = b < B ? h0[(size_t)b * kSeqH + j] * keep[b] : 0.0f;
    sh[0][row][j] = v;
    if (SAVED && b < B) hm[(size_t)b * kSeqH + j] = v;
  }
  // this lane's batch row (a ragged last workgroup computes zero rows and stores nothing for them) and its units
  // j0[jb] + 0..3 of each block
  const int b = r0 + li;
  const bool bv = FULL || b < B;
  int j0[NJB];
#pragma unroll
  for (int jb = 0; jb < NJB; ++jb) j0[jb] = 16 * (NJB * wv + jb) + 4 * lg;
  f32x4 c[NJB];
  {
    const float k0 = bv ? keep[b] : 0.0f;
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      c[jb] = bv ? ld4(c0 + (size_t)b * kSeqH + j0[jb]) * k0 : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (SAVED && bv) st4(cm + (size_t)b * kSeqH + j0[jb], c[jb]);
    }
  }
  // the wave's weight fragments, packed by ouz_lstm_seq_pack in the order the lanes consume them (wf [wave][slab]
  // [jb][q][lane] f32x4): every fragment load is one contiguous 1 KB (eight full cache lines) per wave.
  // The wave's whole weight slice (128 gate rows x 128, 64 KB: 256 registers per lane) is loaded once and kept in
  // registers for all T steps (one wave per SIMD: the register file has room), so the steps read no weights at all.
  // (block gb = NJB wv + jb of the eight 16-unit blocks sits at wf[gb >> 1][.][gb & 1])
  const f32x4* wl = reinterpret_cast<const f32x4*>(w) + lane;
  f32x4 wreg[kSeqH / 16][NJB][4];
#pragma unroll
  for (int p = 0; p < kSeqH / 16; ++p)
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      const int gb = NJB * wv + jb;
#pragma unroll
      for (int q = 0; q < 4; ++q) wreg[p][jb][q] = wl[((((size_t)(gb >> 1) * 8 + p) * 2 + (gb & 1)) * 4 + q) * 64];
    }
  // A step's inputs (its input projection, the next step's keep) are loaded one step ahead, before the previous
  // step's output stores: gfx950's single vmcnt counter retires loads and stores in order, so loads issued after
  // a step's stores could not be waited for without waiting for those stores too.  The inputs alternate between two
  // register sets (the loop runs two steps per trip): with one set, the hand-over of the prefetched keep to the next
  // step was a register copy, and that copy's s_waitcnt vmcnt(0) drained every store of the step before the next
  // one could start.
  f32x4 xa[NJB][4], xb[NJB][4];
  float ka, kb;
  const auto load_inputs = [&](int t, f32x4 (&xd)[NJB][4], float& kd) {
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        xd[jb][q] = bv ? ld4(xp + ((size_t)t * B + b) * kSeqG + q * kSeqH + j0[jb]) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    kd = (t + 1 < T && bv) ? keep[(size_t)(t + 1) * B + b] : 1.0f;
  };
  const auto step = [&](int t, const f32x4 (&x)[NJB][4], float kn, f32x4 (&xn)[NJB][4], float& knn) {
    const int cur = t & 1;
    const bool last = t == T - 1;
    __syncthreads();   // sh[cur] holds this step's carry (and every wave is done with sh[cur ^ 1])
    f32x4 ig[NJB], fg[NJB], gg[NJB], og[NJB], cn[NJB], hn[NJB], hv[NJB];
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      // the product of unit block jb; block 0's cell update below is independent of block 1's MFMAs, so the
      // scheduler can issue its VALU work while those run
      f32x4 acc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int p = 0; p < kSeqH / 16; ++p) {
        const f32x4 h = ld4(&sh[cur][li][16 * p + 4 * lg]);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = mfma4(wreg[p][jb][q], h, acc[q]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // gates = x_proj + h W_hh^T (the GEMM path's beta = 1 accumulation: the projection added to the product)
        ig[jb][r] = fsigm(x[jb][0][r] + acc[0][r]);
        fg[jb][r] = fsigm(x[jb][1][r] + acc[1][r]);
        gg[jb][r] = ftanh(x[jb][2][r] + acc[2][r]);
        og[jb][r] = fsigm(x[jb][3][r] + acc[3][r]);
        cn[jb][r] = fg[jb][r] * c[jb][r] + ig[jb][r] * gg[jb][r];
        hn[jb][r] = og[jb][r] * ftanh(cn[jb][r]);
        hv[jb][r] = kn * hn[jb][r];   // the masked carry: the next step's operand (LDS) and hm / h_out
        c[jb][r] = kn * cn[jb][r];
      }
      st4(&sh[cur ^ 1][li][j0[jb]], hv[jb]);
    }
    if (!last) load_inputs(t + 1, xn, knn);   // ahead of this step's stores
    if (bv) {
      const size_t base = (size_t)t * B + b;
#pragma unroll
      for (int jb = 0; jb < NJB; ++jb) {
        if (SAVED) {
          float* a = act + base * kSeqG + j0[jb];
          st4(a, ig[jb]); st4(a + kSeqH, fg[jb]); st4(a + 2 * kSeqH, gg[jb]); st4(a + 3 * kSeqH, og[jb]);
        }
        if (SAVED) st4(c_all + base * kSeqH + j0[jb], cn[jb]);
        st4(hid + base * kSeqH + j0[jb], hn[jb]);
        if (last && h_out) {
          st4(h_out + (size_t)b * kSeqH + j0[jb], hv[jb]);
          st4(c_out + (size_t)b * kSeqH + j0[jb], c[jb]);
        } else {
          const size_t nx = ((size_t)(t + 1) * B + b) * kSeqH + j0[jb];
          if (SAVED) {
            st4(hm + nx, hv[jb]);
            st4(cm + nx, c[jb]);
          }
        }
      }
    }
  };
  // the weight loads complete here, once: otherwise the waitcnt pass, merging the loop's entry state (32 fragment
  // loads in flight) into its header, put an s_waitcnt vmcnt(0) before the first MFMA on each fragment in EVERY step,
  // draining the previous step's stores too
  __builtin_amdgcn_s_waitcnt(0);
  // step 0 is peeled so that the loop is entered, like its back edge, right after a step's prefetch and stores:
  // the waitcnt pass merges both into the loop header, and an entry straight after load_inputs(0) would make the
  // loop's first wait for the inputs a vmcnt(0) on every trip
  load_inputs(0, xa, ka);
  step(0, xa, ka, xb, kb);
  int t = 1;
  for (; t + 1 < T; t += 2) {
    step(t, xb, kb, xa, ka);
    step(t + 1, xa, ka, xb, kb);
  }
  if (t < T) step(t, xb, kb, xa, ka);
}

template <int NJB, bool SAVED>
__global__ void __launch_bounds__(512 / NJB) lstm_seq_fwd_kernel(
    const float* __restrict__ xp, const float* h0, const float* c0, const float* __restrict__ keep,
    const float* __restrict__ w, int T, int B, float* __restrict__ act, float* __restrict__ c_all,
    float* __restrict__ hid, float* __restrict__ hm, float* __restrict__ cm, float* h_out, float* c_out) {
  // the masked h entering the step (the MFMA's B operand), double-buffered by step parity so that a wave's cell
  // update can run beside the MFMAs of the next unit block (rows padded: conflict-free)
  __shared__ float sh[2][kSeqRows][kSeqH + 4];
  if ((int)(blockIdx.x + 1) * kSeqRows <= B)
    lstm_seq_fwd_body<NJB, true, SAVED>(sh, xp, h0, c0, keep, w, T, B, act, c_all, hid, hm, cm, h_out, c_out);
  else
    lstm_seq_fwd_body<NJB, false, SAVED>(sh, xp, h0, c0, keep, w, T, B, act, c_all, hid, hm, cm, h_out, c_out);
}

// BPTT over T steps (the mirror of lstm_seq_fwd_kernel and of the per-step lstm_cell_bwd_kernel + GEMM): per step
// dh = dhid + keep_{t+1} G with G = dgates_{t+1} W_hh (the MFMA product, K = 4H, from the dgates tile kept in LDS;
// at t = T - 1 G is dhT, or nothing), dc = keep_{t+1} dc_next + dh o (1 - tanh(c)^2).  Writes dgates [T][B][4H]
// (pre-activation), dh0 = (dgates_0 W_hh) keep_0 and dc0 = dc keep_0 [B][H].  Same transposed product and lane map
// as the forward (G^T = W_hh^T dgates^T: a lane holds four consecutive units of one row).
template <int NJB, bool FULL>
__device__ __forceinline__ void lstm_seq_bwd_body(
    float (*sg)[kSeqRows][kSeqG + 4], const float* __restrict__ act, const float* __restrict__ c_all,
    const float* __restrict__ cm, const float* __restrict__ keep, const float* __restrict__ wt,
    const float* __restrict__ dhid, const float* __restrict__ dhT, const float* __restrict__ dcT, int T, int B,
    float* __restrict__ dgates, float* __restrict__ dh0, float* __restrict__ dc0) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.x * kSeqRows;
  // packed W_hh fragments (ouz_lstm_seq_pack: wb [wave][slab][jb][lane] f32x4, one contiguous 1 KB per load): the
  // wave's slice (32 hidden units x 512 gate columns, 64 KB: 256 registers per lane) is loaded once for all T steps
  // (block gb = NJB wv + jb of the eight 16-unit blocks sits at wb[gb >> 1][.][gb & 1])
  const f32x4* wl = reinterpret_cast<const f32x4*>(wt) + lane;
  f32x4 wreg[kSeqG / 16][NJB];
#pragma unroll
  for (int p = 0; p < kSeqG / 16; ++p)
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      const int gb = NJB * wv + jb;
      wreg[p][jb] = wl[(((size_t)(gb >> 1) * 32 + p) * 2 + (gb & 1)) * 64];
    }
  // G of unit block jb (transposed: lane holds units j0[jb] + 0..3 of row li) = sg[buf] W_hh over the 4H gates
  const auto product = [&](int buf, int jb) {
    f32x4 acc = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int p = 0; p < kSeqG / 16; ++p) acc = mfma4(wreg[p][jb], ld4(&sg[buf][li][16 * p + 4 * lg]), acc);
    return acc;
  };
  const int b = r0 + li;
  const bool bv = FULL || b < B;
  int j0[NJB];
#pragma unroll
  for (int jb = 0; jb < NJB; ++jb) j0[jb] = 16 * (NJB * wv + jb) + 4 * lg;
  const f32x4 zero4 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  f32x4 dc[NJB];
  // the cell's saved values of a step are loaded one step ahead, before the later step's dgates stores (one
  // in-order vmcnt counter for loads and stores: see lstm_seq_fwd_kernel)
  // (two register sets, alternating by step: see lstm_seq_fwd_kernel)
  struct Saved {
    f32x4 ag[NJB][4], cv[NJB], cp[NJB], dy[NJB];
    float kn;
  };
  Saved sa, sb;
  const auto load_saved = [&](int t, Saved& sv) {
    sv.kn = (t + 1 < T && bv) ? keep[(size_t)(t + 1) * B + b] : 1.0f;
    const size_t base = (size_t)t * B + b;
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) sv.ag[jb][q] = bv ? ld4(act + base * kSeqG + q * kSeqH + j0[jb]) : zero4;
      sv.cv[jb] = bv ? ld4(c_all + base * kSeqH + j0[jb]) : zero4;
      sv.cp[jb] = bv ? ld4(cm + base * kSeqH + j0[jb]) : zero4;
      sv.dy[jb] = bv ? ld4(dhid + base * kSeqH + j0[jb]) : zero4;
    }
  };
  const auto step = [&](int t, const Saved& sv, Saved& nx) {
    const auto& ag = sv.ag;
    const auto& cv = sv.cv;
    const auto& cp = sv.cp;
    const auto& dy = sv.dy;
    const float kn = sv.kn;
    const bool lastt = t == T - 1;
    const int cur = t & 1;   // the buffer this step writes; it reads cur ^ 1 (written by step t + 1)
    const bool has_g = !lastt || dhT != nullptr;
    const bool has_dc = !lastt || dcT != nullptr;
    // sg[cur ^ 1] holds dgates_{t+1}, and every wave is done with sg[cur] (read by step t + 1)
    if (!lastt) __syncthreads();
    f32x4 di[NJB], df[NJB], dg[NJB], d_o[NJB];
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      f32x4 acc, dcn;
      if (lastt) {
        acc = (dhT && bv) ? ld4(dhT + (size_t)b * kSeqH + j0[jb]) : zero4;
        dcn = (dcT && bv) ? ld4(dcT + (size_t)b * kSeqH + j0[jb]) : zero4;
      } else {
        acc = product(cur ^ 1, jb);
        dcn = dc[jb];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dh = dy[jb][r] + (has_g ? kn * acc[r] : 0.0f);
        const float ig = ag[jb][0][r], fg = ag[jb][1][r], gg = ag[jb][2][r], og = ag[jb][3][r];
        const float tc = ftanh(cv[jb][r]);
        const float dcv = (has_dc ? kn * dcn[r] : 0.0f) + dh * og * (1.0f - tc * tc);
        di[jb][r] = dcv * gg * ig * (1.0f - ig);
        df[jb][r] = dcv * cp[jb][r] * fg * (1.0f - fg);
        dg[jb][r] = dcv * ig * (1.0f - gg * gg);
        d_o[jb][r] = dh * tc * og * (1.0f - og);
        dc[jb][r] = dcv * fg;
      }
      float* srow = &sg[cur][li][j0[jb]];
      st4(srow, di[jb]); st4(srow + kSeqH, df[jb]); st4(srow + 2 * kSeqH, dg[jb]); st4(srow + 3 * kSeqH, d_o[jb]);
    }
    if (t > 0) load_saved(t - 1, nx);   // ahead of this step's stores
    if (bv) {
#pragma unroll
      for (int jb = 0; jb < NJB; ++jb) {
        float* d = dgates + ((size_t)t * B + b) * kSeqG + j0[jb];
        st4(d, di[jb]); st4(d + kSeqH, df[jb]); st4(d + 2 * kSeqH, dg[jb]); st4(d + 3 * kSeqH, d_o[jb]);
      }
    }
  };
  __builtin_amdgcn_s_waitcnt(0);   // the weight loads complete once, before the loop (see lstm_seq_fwd_kernel)
  load_saved(T - 1, sa);
  step(T - 1, sa, sb);   // peeled, as in lstm_seq_fwd_kernel
  int t = T - 2;
  for (; t >= 1; t -= 2) {
    step(t, sb, sa);
    step(t - 1, sa, sb);
  }
  if (t == 0) step(0, sb, sa);
  // dh0 = (dgates_0 W_hh) keep_0, dc0 = dc keep_0
  __syncthreads();
#pragma unroll
  for (int jb = 0; jb < NJB; ++jb) {
    const f32x4 acc = product(0, jb);
    if (!bv) continue;
    const float k0 = keep[b];
    if (dh0) st4(dh0 + (size_t)b * kSeqH + j0[jb], acc * k0);
    if (dc0) st4(dc0 + (size_t)b * kSeqH + j0[jb], dc[jb] * k0);
  }
}

template <int NJB>
__global__ void __launch_bounds__(512 / NJB) lstm_seq_bwd_kernel(
    const float* __restrict__ act, const float* __restrict__ c_all, const float* __restrict__ cm,
    const float* __restrict__ keep, const float* __restrict__ wt, const float* __restrict__ dhid,
    const float* __restrict__ dhT, const float* __restrict__ dcT, int T, int B, float* __restrict__ dgates,
    float* __restrict__ dh0, float* __restrict__ dc0) {
  // dgates of the step after (B operand of G), double-buffered by step parity: one barrier per step
  __shared__ float sg[2][kSeqRows][kSeqG + 4];
  if ((int)(blockIdx.x + 1) * kSeqRows <= B)
    lstm_seq_bwd_body<NJB, true>(sg, act, c_all, cm, keep, wt, dhid, dhT, dcT, T, B, dgates, dh0, dc0);
  else
    lstm_seq_bwd_body<NJB, false>(sg, act, c_all, cm, keep, wt, dhid, dhT, dcT, T, B, dgates, dh0, dc0);
}

// The weight fragments of lstm_seq_fwd_kernel / lstm_seq_bwd_kernel in consumption order (one thread per f32x4):
//   wf[w][p][jb][q][l] = W_hh[q H + 32 w + 16 jb + (l & 15)][16 p + 4 (l >> 4) + 0..3]        (8 slabs of K = H)
//   wb[w][p][jb][l]    = W_hh[16 p + 4 (l >> 4) + 0..3][32 w + 16 jb + (l & 15)]              (32 slabs of K = 4H)
__global__ void __launch_bounds__(256) lstm_seq_pack_kernel(const float* __restrict__ w, f32x4* __restrict__ wf,
                                                            f32x4* __restrict__ wb) {
  const int e = blockIdx.x * 256 + threadIdx.x;   // kSeqH * kSeqG / 4 fragments per layout
  if (e >= kSeqH * kSeqG / 4) return;
  {
    const int l = e & 63, q = (e >> 6) & 3, jb = (e >> 8) & 1, p = (e >> 9) & 7, wv = e >> 12;
    const float* src = w + (size_t)(q * kSeqH + 32 * wv + 16 * jb + (l & 15)) * kSeqH + 16 * p + 4 * (l >> 4);
    wf[e] = f32x4{src[0], src[1], src[2], src[3]};
  }
  {
    const int l = e & 63, jb = (e >> 6) & 1, p = (e >> 7) & 31, wv = e >> 12;
    const int n = 32 * wv + 16 * jb + (l & 15), k = 16 * p + 4 * (l >> 4);
    wb[e] = f32x4{w[(size_t)k * kSeqH + n], w[(size_t)(k + 1) * kSeqH + n], w[(size_t)(k + 2) * kSeqH + n],
                  w[(size_t)(k + 3) * kSeqH + n]};
  }
}

inline int grid(int n, int b) { return (n + b - 1) / b; }

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(OUZ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return OUZ_OK;
}

// ---------------------------------------------------------------------------
// Gradient-norm clipping + Adam over one network's parameters in two launches (RPO-LSTM/agent.py:124-134:
// nn.utils.clip_grad_norm_(parameters, max_grad_norm) then optim.Adam.step()), in place of torch's per-tensor norms,
// their stack / norm / clamp / scale launches and the multi-tensor Adam kernel (~6 launches and ~70 us per step on a
// < 1 M-parameter network: the multi-tensor kernel's grid is sized by tensor chunks, not by the chip).
//   the parameters are cut into chunks of ch elements, one block per chunk (a uniform scan finds the block's tensor),
//   ch = max(1024, the total / 256 rounded up to 1024), so at most 256 + 16 blocks; each thread loads its (up to) four
//   elements of a pass before it uses them, one memory round trip per pass;
//   adam_sqnorm_kernel: one partial sum of g^2 per chunk (fixed order);
//   adam_step_kernel: every block reduces the same partials in the same order (so all agree on the norm without a
//   third launch), clip coefficient min(max_norm / (||g|| + 1e-6), 1) as torch computes it, then the Adam update in
//   torch's single-tensor order (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_, denom = sqrt(v) / sqrt(bc2) + eps,
//   param.addcdiv_(m, denom, -lr / bc1)).  The clipped gradient is not written back (nothing reads it after step).
// ---------------------------------------------------------------------------
constexpr int kAdamMinChunk = 1024;

__device__ __forceinline__ float block_sum256(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// The block's tensor and element range [lo, hi) (uniform across the block).
__device__ __forceinline__ int adam_chunk(const ouz_adam_table& t, int64_t ch, int64_t& lo, int64_t& hi) {
  int64_t cb = blockIdx.x;
  int i = 0;
  for (; i < t.n_tensors; ++i) {
    const int64_t n = (t.numel[i] + ch - 1) / ch;
    if (cb < n) break;
    cb -= n;
  }
  lo = cb * ch;
  hi = lo + ch < t.numel[i] ? lo + ch : t.numel[i];
  return i;
}

__global__ void __launch_bounds__(256) adam_sqnorm_kernel(ouz_adam_table t, int64_t ch, float* __restrict__ part) {
  __shared__ float red[256];
  int64_t lo, hi;
  const int i = adam_chunk(t, ch, lo, hi);
  const float* __restrict__ g = t.grad[i];
  float acc = 0.0f;
  for (int64_t e0 = lo + threadIdx.x; e0 < hi; e0 += 4 * 256) {
    float gv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) gv[u] = e0 + 256 * u < hi ? g[e0 + 256 * u] : 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += gv[u] * gv[u];
  }
  const float s = block_sum256(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) adam_step_kernel(ouz_adam_table t, int64_t ch, const float* __restrict__ part,
                                                        int nparts, float lr_bc1, float w1, float beta2, float w2,
                                                        float eps, float bc2_sqrt, float max_norm) {
  __shared__ float red[256];
  float coef = 1.0f;
  if (max_norm > 0.0f) {
    float v = 0.0f;
    for (int j = threadIdx.x; j < nparts; j += 256) v += part[j];
    const float total = sqrtf(block_sum256(v, red));
    coef = fminf(max_norm / (total + 1e-6f), 1.0f);
  }
  int64_t lo, hi;
  const int i = adam_chunk(t, ch, lo, hi);
  const float* __restrict__ g = t.grad[i];
  float* __restrict__ p = t.param[i];
  float* __restrict__ m = t.exp_avg[i];
  float* __restrict__ v = t.exp_avg_sq[i];
  for (int64_t e0 = lo + threadIdx.x; e0 < hi; e0 += 4 * 256) {
    float gv[4], mv[4], vv[4], pv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = e0 + 256 * u;
      if (e < hi) { gv[u] = g[e]; mv[u] = m[e]; vv[u] = v[e]; pv[u] = p[e]; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = e0 + 256 * u;
      if (e >= hi) continue;
      const float gc = gv[u] * coef;
      const float mn = mv[u] + w1 * (gc - mv[u]);   // lerp(m, g, 1 - beta1)
      const float vn = vv[u] * beta2 + w2 * gc * gc;
      m[e] = mn;
      v[e] = vn;
      p[e] = pv[u] + (-lr_bc1) * (mn / (sqrtf(vn) / bc2_sqrt + eps));
    }
  }
}

// ---------------------------------------------------------------------------
// The trunks' first layer, y = tanh(x W^T + b) with K <= 16 inputs (the 13 observations; RPO-LSTM/model.py:11-20,
// agent.py critic), in ONE pass: hipBLASLt's K = 13 GEMM writes the pre-activation and torch's tanh reads and rewrites
// it, where this layer is a write of y and nothing else.  W^T, b and a chunk of rows' inputs sit in LDS; each thread
// makes four consecutive outputs of a row (one 16-byte store).  tanh is the sequence kernels' ftanh.
// (A round-5 form with one thread per row and a column loop waited on its rows' loads one after another and lost to
// the GEMM + tanh pair at 65 536 rows; docs/HISTORY.md.)
// ---------------------------------------------------------------------------
constexpr int kSmallKMax = 16;
constexpr int kSmallKBlocks = 1024;
constexpr int kSmallKChunk = 64;   // at most this many rows' inputs staged in LDS at a time (fewer below 32 K rows)

__global__ void __launch_bounds__(256) linear_tanh_smallk_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                                 const float* __restrict__ b, int rows, int K, int cols,
                                                                 int chunk, float* __restrict__ y) {
  extern __shared__ float sw[];   // W^T [K][cols], b [cols], then the chunk's inputs [chunk][K]
  float* sx = sw + (K + 1) * cols;
  for (int e = threadIdx.x; e < K * cols; e += 256) {
    const int k = e / cols, c = e - k * cols;
    sw[e] = w[(size_t)c * K + k];
  }
  for (int c = threadIdx.x; c < cols; c += 256) sw[K * cols + c] = b[c];
  const int tpr = cols >> 2, rpb = 256 / tpr;   // threads per row, rows per pass (cols a power of two)
  const int c4 = (int)threadIdx.x % tpr, rs = (int)threadIdx.x / tpr;
  // the block's rows: contiguous chunks, dealt round robin over the blocks; each chunk's inputs are one coalesced
  // load into LDS, so no thread waits on its rows' input loads one after another
  for (int r0 = blockIdx.x * chunk; r0 < rows; r0 += gridDim.x * chunk) {
    const int nr = rows - r0 < chunk ? rows - r0 : chunk;
    __syncthreads();   // W^T / b written (first chunk), every thread done with the previous chunk's inputs
    for (int e = threadIdx.x; e < nr * K; e += 256) sx[e] = x[(size_t)r0 * K + e];
    __syncthreads();
    const f32x4 bias = ld4(&sw[K * cols + 4 * c4]);
    for (int r = rs; r < nr; r += rpb) {
      f32x4 acc = bias;
#pragma unroll 4
      for (int k = 0; k < K; ++k) acc += sx[r * K + k] * ld4(&sw[k * cols + 4 * c4]);
      f32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = ftanh(acc[i]);
      st4(y + (size_t)(r0 + r) * cols + 4 * c4, o);
    }
  }
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


static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Waves per workgroup of the sequence kernels: 8 (one 16-unit block per wave, two waves per SIMD: one wave's cell
// update and stores run beside the other's MFMAs) or 4 (two blocks per wave, one wave per SIMD; 10-15 % slower,
// profiles/r06/learn/lstm_seq_ab.txt); OUZ_LSTM_SEQ_WAVES=4 selects the latter.
static int seq_waves() {
  static const int w = [] {
    const char* e = std::getenv("OUZ_LSTM_SEQ_WAVES");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();
  return w;
}

int ouz_lstm_seq_pack(const float* w_hh, int32_t H, float* w_fwd, float* w_bwd, void* stream) {
  if (H != kSeqH) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_pack: H must be 128");
  if (!w_hh || !w_fwd || !w_bwd) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_pack: null buffer");
  if (!aligned16(w_fwd) || !aligned16(w_bwd))
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_pack: packed buffers must be 16-byte aligned");
  hipLaunchKernelGGL(lstm_seq_pack_kernel, dim3(grid(kSeqH * kSeqG / 4, 256)), dim3(256), 0, (hipStream_t)stream, w_hh,
                     reinterpret_cast<f32x4*>(w_fwd), reinterpret_cast<f32x4*>(w_bwd));
  return launch_status("lstm_seq_pack_kernel");
}

int ouz_lstm_seq_fwd(const float* x_proj, const float* h0, const float* c0, const float* keep, const float* w_hh,
                     int32_t T, int32_t B, int32_t H, float* act, float* c_all, float* hid, float* hm, float* cm,
                     float* h_out, float* c_out, void* stream) {
  if (H != kSeqH) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_fwd: H must be 128");
  if (T <= 0 || B <= 0) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_fwd: T and B must be > 0");
  if (!x_proj || !h0 || !c0 || !keep || !w_hh || !hid || (!h_out) != (!c_out))
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_fwd: null buffer (h_out and c_out: both or neither)");
  if ((!act) != (!c_all) || (!act) != (!hm) || (!act) != (!cm))
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_fwd: act, c_all, hm and cm: all four or none");
  for (const void* p : {(const void*)x_proj, (const void*)c0, (const void*)w_hh, (const void*)act, (const void*)c_all,
                        (const void*)hid, (const void*)hm, (const void*)cm, (const void*)h_out, (const void*)c_out})
    if (!aligned16(p)) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_fwd: every buffer must be 16-byte aligned");
  const dim3 g(grid(B, kSeqRows));
  const hipStream_t s = (hipStream_t)stream;
  const bool saved = act != nullptr;
#define OUZ_SEQ_FWD(NJB, SAVED)                                                                                    \
  hipLaunchKernelGGL((lstm_seq_fwd_kernel<NJB, SAVED>), g, dim3(512 / NJB), 0, s, x_proj, h0, c0, keep, w_hh, T, B, \
                     act, c_all, hid, hm, cm, h_out, c_out)
  if (seq_waves() == 8) {
    if (saved) OUZ_SEQ_FWD(1, true); else OUZ_SEQ_FWD(1, false);
  } else {
    if (saved) OUZ_SEQ_FWD(2, true); else OUZ_SEQ_FWD(2, false);
  }
#undef OUZ_SEQ_FWD
  return launch_status("lstm_seq_fwd_kernel");
}

int ouz_lstm_seq_bwd(const float* act, const float* c_all, const float* cm, const float* keep, const float* w_hh_t,
                     const float* dhid, const float* dhT, const float* dcT, int32_t T, int32_t B, int32_t H,
                     float* dgates, float* dh0, float* dc0, void* stream) {
  if (H != kSeqH) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_bwd: H must be 128");
  if (T <= 0 || B <= 0) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_bwd: T and B must be > 0");
  if (!act || !c_all || !cm || !keep || !w_hh_t || !dhid || !dgates)
    return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_bwd: null buffer");
  for (const void* p : {(const void*)act, (const void*)c_all, (const void*)cm, (const void*)w_hh_t, (const void*)dhid,
                        (const void*)dhT, (const void*)dcT, (const void*)dgates, (const void*)dh0, (const void*)dc0})
    if (!aligned16(p)) return set_error(OUZ_ERR_INVALID, "ouz_lstm_seq_bwd: every buffer must be 16-byte aligned");
  if (seq_waves() == 8)
    hipLaunchKernelGGL(lstm_seq_bwd_kernel<1>, dim3(grid(B, kSeqRows)), dim3(512), 0, (hipStream_t)stream, act, c_all,
                       cm, keep, w_hh_t, dhid, dhT, dcT, T, B, dgates, dh0, dc0);
  else
    hipLaunchKernelGGL(lstm_seq_bwd_kernel<2>, dim3(grid(B, kSeqRows)), dim3(256), 0, (hipStream_t)stream, act, c_all,
                       cm, keep, w_hh_t, dhid, dhT, dcT, T, B, dgates, dh0, dc0);
  return launch_status("lstm_seq_bwd_kernel");
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

int ouz_ppo_policy_loss(const float* mean_z, const float* logstd, const float* actions, const float* old_logp,
                        const float* advantages, int32_t n, float clip, int32_t norm_adv, double* workspace,
                        float* dmean, float* loss, float* approx_kl, float* clipfrac, float* dlogstd, void* stream) {
  if (n <= 0 || (norm_adv && n < 2)) return set_error(OUZ_ERR_INVALID, "ouz_ppo_policy_loss: n must be > 0 (> 1 with norm_adv)");
  if (!mean_z || !logstd || !actions || !old_logp || !advantages || !workspace || !dmean || !loss || !approx_kl ||
      !clipfrac || !dlogstd)
    return set_error(OUZ_ERR_INVALID, "ouz_ppo_policy_loss: null buffer");
  if (((reinterpret_cast<uintptr_t>(mean_z) | reinterpret_cast<uintptr_t>(actions) | reinterpret_cast<uintptr_t>(dmean)) & 15u))
    return set_error(OUZ_ERR_INVALID, "ouz_ppo_policy_loss: mean_z / actions / dmean must be 16-byte aligned");
  const hipStream_t s = (hipStream_t)stream;
  double* adv_part = workspace;
  double* part = workspace + 2 * kLossBlocks;
  if (norm_adv) hipLaunchKernelGGL(adv_moments_kernel, dim3(kLossBlocks), dim3(kLossThreads), 0, s, advantages, n, adv_part);
  hipLaunchKernelGGL(policy_loss_kernel, dim3(kLossBlocks), dim3(kLossThreads), 0, s, mean_z, logstd, actions, old_logp,
                     advantages, n, clip, norm_adv, adv_part, dmean, part);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(kLossThreads), 0, s, part, 3 + OUZ_NUM_ACT, 1.0 / (double)n, loss,
                     approx_kl, clipfrac, dlogstd);
  return launch_status("policy_loss_kernel");
}

int ouz_ppo_value_loss(const float* values, const float* returns, int32_t n, double* workspace, float* dvalues,
                       float* loss, void* stream) {
  if (n <= 0) return set_error(OUZ_ERR_INVALID, "ouz_ppo_value_loss: n must be > 0");
  if (!values || !returns || !workspace || !dvalues || !loss) return set_error(OUZ_ERR_INVALID, "ouz_ppo_value_loss: null buffer");
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(value_loss_kernel, dim3(kLossBlocks), dim3(kLossThreads), 0, s, values, returns, n, dvalues, workspace);
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(kLossThreads), 0, s, workspace, 1, 0.5 / (double)n, loss, nullptr, nullptr,
                     nullptr);
  return launch_status("value_loss_kernel");
}

int ouz_tanh_bwd_bias(const float* dy, const float* y, int32_t rows, int32_t cols, float* workspace, float* dz,
                      float* dbias, void* stream) {
  if (rows <= 0 || cols <= 0 || cols % 4 || cols > 1024 || 256 % (cols / 4))
    return set_error(OUZ_ERR_INVALID, "ouz_tanh_bwd_bias: rows > 0 and cols a power of two in [4, 1024]");
  if (!dy || !y || !workspace || !dz || !dbias) return set_error(OUZ_ERR_INVALID, "ouz_tanh_bwd_bias: null buffer");
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(dz) |
        reinterpret_cast<uintptr_t>(workspace)) & 15u))
    return set_error(OUZ_ERR_INVALID, "ouz_tanh_bwd_bias: buffers must be 16-byte aligned");
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(tanh_bwd_colsum_kernel, dim3(kColBlocks), dim3(256), 0, s, dy, y, dz, workspace, rows, cols);
  hipLaunchKernelGGL(colsum_finish_kernel, dim3(grid(cols, 16)), dim3(256), 0, s, workspace, cols, dbias);
  return launch_status("tanh_bwd_colsum_kernel");
}

int ouz_policy_sample(const float* hidden, const float* w, const float* b, const float* logstd, const float* eps,
                      int32_t B, int32_t H, float* action, float* logprob, float* entropy, void* stream) {
  if (B <= 0 || H <= 0 || H % 4 || H > 4096) return set_error(OUZ_ERR_INVALID, "ouz_policy_sample: B > 0, H a multiple of 4");
  if (!hidden || !w || !b || !logstd || !eps || !action || !logprob || !entropy)
    return set_error(OUZ_ERR_INVALID, "ouz_policy_sample: null buffer");
  if (((reinterpret_cast<uintptr_t>(hidden) | reinterpret_cast<uintptr_t>(w)) & 15u))
    return set_error(OUZ_ERR_INVALID, "ouz_policy_sample: hidden and w must be 16-byte aligned");
  hipLaunchKernelGGL(policy_sample_kernel, dim3(grid(B * OUZ_NUM_ACT, 256)), dim3(256), 0, (hipStream_t)stream, hidden,
                     w, b, logstd, eps, B, H, action, logprob, entropy);
  return launch_status("policy_sample_kernel");
}


int ouz_adam_clip_step(const ouz_adam_table* t, double lr, double beta1, double beta2, double eps, int64_t step,
                       double max_norm, float* workspace, void* stream) {
  if (!t || !workspace) return set_error(OUZ_ERR_INVALID, "ouz_adam_clip_step: null table or workspace");
  if (t->n_tensors < 1 || t->n_tensors > OUZ_ADAM_MAX_TENSORS)
    return set_error(OUZ_ERR_INVALID, "ouz_adam_clip_step: 1 to OUZ_ADAM_MAX_TENSORS tensors");
  if (step < 1) return set_error(OUZ_ERR_INVALID, "ouz_adam_clip_step: step counts from 1");
  for (int i = 0; i < t->n_tensors; ++i)
    if (t->numel[i] < 0 || (t->numel[i] && (!t->grad[i] || !t->param[i] || !t->exp_avg[i] || !t->exp_avg_sq[i])))
      return set_error(OUZ_ERR_INVALID, "ouz_adam_clip_step: null tensor in the table");
  // torch's host-side scalars (Adam's non-capturable path): computed in double (Python floats), used as f32
  const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
  int64_t total = 0;
  for (int i = 0; i < t->n_tensors; ++i) total += t->numel[i];
  if (total == 0) return OUZ_OK;
  const int64_t ch = std::max<int64_t>(kAdamMinChunk, (total / 256 + kAdamMinChunk) / kAdamMinChunk * kAdamMinChunk);
  int64_t chunks = 0;
  for (int i = 0; i < t->n_tensors; ++i) chunks += (t->numel[i] + ch - 1) / ch;
  // (chunks <= 256 + OUZ_ADAM_MAX_TENSORS <= OUZ_ADAM_WS_FLOATS; a zero-element tensor owns no chunk and no block)
  const hipStream_t s = (hipStream_t)stream;
  if (max_norm > 0.0)
    hipLaunchKernelGGL(adam_sqnorm_kernel, dim3((unsigned)chunks), dim3(256), 0, s, *t, ch, workspace);
  hipLaunchKernelGGL(adam_step_kernel, dim3((unsigned)chunks), dim3(256), 0, s, *t, ch, workspace, (int)chunks,
                     (float)(lr / bc1), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     (float)std::sqrt(bc2), (float)max_norm);
  return launch_status("adam_step_kernel");
}


int ouz_linear_tanh_small_k(const float* x, const float* w, const float* b, int32_t rows, int32_t K, int32_t cols,
                            float* y, void* stream) {
  if (rows < 0 || K < 1 || K > kSmallKMax || cols < 4 || cols > 1024 || (cols & (cols - 1)))
    return set_error(OUZ_ERR_INVALID, "ouz_linear_tanh_small_k: rows >= 0, 1 <= K <= 16, cols a power of two in [4, 1024]");
  if (rows == 0) return OUZ_OK;   // (torch's empty tensors have null data pointers)
  if (!x || !w || !b || !y) return set_error(OUZ_ERR_INVALID, "ouz_linear_tanh_small_k: null buffer");
  if (!aligned16(y)) return set_error(OUZ_ERR_INVALID, "ouz_linear_tanh_small_k: y must be 16-byte aligned");
  // chunks of 8-64 rows: at least ~512 blocks where the rows allow (the rollout's 8 192 rows: 16-row chunks)
  const int chunk = std::max(8, std::min(kSmallKChunk, (rows + 511) / 512));
  const int blocks = std::min((rows + chunk - 1) / chunk, kSmallKBlocks);
  hipLaunchKernelGGL(linear_tanh_smallk_kernel, dim3(blocks), dim3(256),
                     ((size_t)(K + 1) * cols + (size_t)chunk * K) * sizeof(float), (hipStream_t)stream, x, w, b, rows, K,
                     cols, chunk, y);
  return launch_status("linear_tanh_smallk_kernel");
}

}  // extern "C"
