// Which stage of the PV step (PVFilter.py:25-110, quad_math.h's stable forms) can run in f32?
// Host build of quad_math.h (-DOUZ_HOST): the step in f64 with one stage at a time (or several) evaluated in f32;
// scripts/exp/pv_precision.py replays tests/golden/pvfilter.npz's adversarial sequences (random fixes every step)
// and reports each mode's error against the reference's f64 run as a multiple of the reference's own f32 run's
// error (the test's bar: >= 100x).  No GPU.
//   g++ -O2 -std=c++17 -march=x86-64-v3 -ffp-contract=off -fPIC -shared -o /tmp/libpvm.so scripts/exp/pv_precision.cpp
#define OUZ_HOST 1
#include "../../ouzelum_amd/csrc/quad_math.h"
using namespace ouz;
// mode bits: 1 = predict in f32, 2 = gains (S^-1, K) in f32, 4 = state correct in f32, 8 = covariance correct in f32,
// 16 = state predict in f32
template <typename A, typename B> static void cvt(const A* a, B* b, int n) { for (int i = 0; i < n; ++i) b[i] = (B)a[i]; }
template <int MB, bool R0>
static void correct(int mode, double x[9], double P[45], const double z[3], double r) {
  M3T<double> Si; double KA[3][3], KB[3][3];
  if (mode & 2) {
    float Pf[45]; cvt(P, Pf, 45); M3T<float> Sf; float KAf[3][3], KBf[3][3];
    pv_gain_t<MB, float>(Pf, (float)r, Sf, KAf, KBf);
    cvt(Sf.m, Si.m, 9); cvt(&KAf[0][0], &KA[0][0], 9); cvt(&KBf[0][0], &KB[0][0], 9);
  } else pv_gain_t<MB, double>(P, r, Si, KA, KB);
  if (mode & 4) {
    float xf[9], zf[3] = {(float)z[0], (float)z[1], (float)z[2]}; cvt(x, xf, 9);
    M3T<float> Sf; float KAf[3][3], KBf[3][3]; cvt(Si.m, Sf.m, 9); cvt(&KA[0][0], &KAf[0][0], 9); cvt(&KB[0][0], &KBf[0][0], 9);
    pv_x_correct_t<MB, float, R0>(xf, zf, (float)r, Sf, KAf, KBf); cvt(xf, x, 9);
  } else pv_x_correct_t<MB, double, R0>(x, z, r, Si, KA, KB);
  if (mode & 8) {
    float Pf[45]; cvt(P, Pf, 45);
    M3T<float> Sf; float KAf[3][3], KBf[3][3]; cvt(Si.m, Sf.m, 9); cvt(&KA[0][0], &KAf[0][0], 9); cvt(&KB[0][0], &KBf[0][0], 9);
    pv_cov_correct_t<MB, float, R0>(Pf, (float)r, Sf, KAf, KBf); cvt(Pf, P, 45);
  } else pv_cov_correct_t<MB, double, R0>(P, r, Si, KA, KB);
}
static void step(int mode, float* xf, float* Pf, const float* acc, const float* q, float dt, int pf, const float* zp, int vf, const float* zv) {
  double x[9], P[45];
  cvt(xf, x, 9); cvt(Pf, P, 45);
  EkfQ qq{q[0], q[1], q[2], q[3]};
  if (mode & 16) { float xs[9], a[3] = {acc[0], acc[1], acc[2]}; cvt(x, xs, 9); pv_state_predict(xs, a, pv_rot<float>(qq), dt, dt * dt * 0.5f); cvt(xs, x, 9); }
  else { const double a[3] = {acc[0], acc[1], acc[2]}; pv_state_predict(x, a, pv_rot<double>(qq), (double)dt, (double)dt * dt * 0.5); }
  if (mode & 1) { float Ps[45]; cvt(P, Ps, 45); pv_cov_predict_t<float>(Ps, pv_rot<float>(qq), dt); cvt(Ps, P, 45); }
  else pv_cov_predict_t<double>(P, pv_rot<double>(qq), (double)dt);
  if (pf) { const double z[3] = {zp[0], zp[1], zp[2]}; correct<0, false>(mode, x, P, z, (double)kPvPosVar); }
  if (vf) { const double z[3] = {zv[0], zv[1], zv[2]}; correct<1, true>(mode, x, P, z, 0.0); }
  cvt(x, xf, 9); cvt(P, Pf, 45);
}
extern "C" void pv_batch(int mode, int n, float* x, float* P, const float* acc, const float* q, float dt, const unsigned char* tp,
                         const float* zp, const unsigned char* tv, const float* zv) {
  for (int i = 0; i < n; ++i) step(mode, x + 9 * i, P + 45 * i, acc + 3 * i, q + 4 * i, dt, tp[i], zp + 3 * i, tv[i], zv + 3 * i);
}
