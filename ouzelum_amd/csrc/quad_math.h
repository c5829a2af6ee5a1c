// Per-env quadrotor math for the fused step kernel (gfx950, one env per lane).
//
// Everything here is register-resident f32 scalar code: 3x3 / 4x4 / 9x9 work is
// far too small for MFMA (no dense contraction on this path), so it
// is written as straight-line VALU math that the compiler keeps in VGPRs.
//
// Each function names the reference routine it restates.  Where the reference
// evaluates an ill-conditioned Kalman update literally — (I - K H) P with
// R = 1e-7 against P = O(1..1000) — the algebraically identical, f32-stable
// form is used instead (derivations in DESIGN.md §4); the literal float64 form
// lives in the CPU oracle, pinned against the reference's own modules.
#pragma once
#ifdef OUZ_HOST
#include "host_compat.h"   // the host build of the step (quad_host.cpp)
#else
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include <type_traits>

#include "philox.h"

namespace ouz {

// ---------------------------------------------------------------------------
// small vector / matrix types
// ---------------------------------------------------------------------------
struct V3 { float x, y, z; };
struct Q4 { float x, y, z, w; };          // xyzw (Isaac root-state order)
template <typename T>
struct M3T { T m[9]; };                    // row-major
using M3 = M3T<float>;

OUZ_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
OUZ_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
OUZ_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
OUZ_HD V3 operator*(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
OUZ_HD V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
OUZ_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
OUZ_HD V3 cross(V3 a, V3 b) { return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
OUZ_HD float norm(V3 a) { return sqrtf(dot(a, a)); }

OUZ_HD V3 mv(const M3& A, V3 v) {
  return V3{A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
            A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z};
}
OUZ_HD V3 mtv(const M3& A, V3 v) {  // A^T v
  return V3{A.m[0] * v.x + A.m[3] * v.y + A.m[6] * v.z, A.m[1] * v.x + A.m[4] * v.y + A.m[7] * v.z,
            A.m[2] * v.x + A.m[5] * v.y + A.m[8] * v.z};
}
// A (3x3) times the 3-vector a[0..2], into out[0..2]
template <typename T>
OUZ_HD void mva(const M3T<T>& A, const T* a, T* out) {
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = A.m[i * 3 + 0] * a[0] + A.m[i * 3 + 1] * a[1] + A.m[i * 3 + 2] * a[2];
}
template <typename T>
OUZ_HD M3T<T> mm(const M3T<T>& A, const M3T<T>& B) {
  M3T<T> C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C.m[i * 3 + j] = A.m[i * 3 + 0] * B.m[0 * 3 + j] + A.m[i * 3 + 1] * B.m[1 * 3 + j] + A.m[i * 3 + 2] * B.m[2 * 3 + j];
  return C;
}
template <typename T>
OUZ_HD M3T<T> mmt(const M3T<T>& A, const M3T<T>& B) {  // A B^T
  M3T<T> C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C.m[i * 3 + j] = A.m[i * 3 + 0] * B.m[j * 3 + 0] + A.m[i * 3 + 1] * B.m[j * 3 + 1] + A.m[i * 3 + 2] * B.m[j * 3 + 2];
  return C;
}
template <typename T>
OUZ_HD M3T<T> tr(const M3T<T>& A) {
  M3T<T> C;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C.m[i * 3 + j] = A.m[j * 3 + i];
  return C;
}
// 1 / x.  On the device, f64: the hardware reciprocal estimate refined by two Newton steps (full
// double precision for the normal, positive determinants of SPD 3x3 blocks) instead of the
// correctly rounded division sequence (div_scale / div_fmas / div_fixup), ~2x fewer f64 issues.
template <typename T>
OUZ_HD T recip(T x) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same_v<T, double>) {
    double y = __builtin_amdgcn_rcp(x);
    y = y * (2.0 - x * y);
    return y * (2.0 - x * y);
  }
#endif
  return T(1) / x;
}

// 1 / sqrt(x) for x > 0.  On the device, f64: the hardware estimate refined by two Newton steps (full double
// precision) instead of the correctly rounded sqrt sequence followed by a division.
template <typename T>
OUZ_HD T rsqrt_r(T x) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same_v<T, double>) {
    double y = __builtin_amdgcn_rsq(x);
    double h = 0.5 * x;
    y = y * (1.5 - h * y * y);
    return y * (1.5 - h * y * y);
  }
#endif
  return T(1) / sqrt(x);
}

// ---------------------------------------------------------------------------
// rotations
// ---------------------------------------------------------------------------
// quaternion_to_matrix on the wxyz reorder of an xyzw quaternion
// (controllers/rotation_conversions.py:36-64; position_control.py:28-29).
OUZ_HD M3 quat_to_mat(Q4 q) {
  float r = q.w, i = q.x, j = q.y, k = q.z;
  float two_s = 2.0f / (r * r + i * i + j * j + k * k);
  return M3{{1.0f - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
             two_s * (i * j + k * r), 1.0f - two_s * (i * i + k * k), two_s * (j * k - i * r),
             two_s * (i * k - j * r), two_s * (j * k + i * r), 1.0f - two_s * (i * i + j * j)}};
}

// matrix_to_euler_angles(R, "ZYX")[:, [2,1,0]] (rotation_conversions.py:216-255):
// roll = atan2(R21, R22), pitch = asin(-R20), yaw = atan2(R10, R00).
// The controllers only consume sin/cos of these angles (position_control.py:51-52,75-79),
// so they are formed directly from R: cos(atan2(y, x)) = x / hypot(x, y), etc. — the
// same numbers without 2 atan2 + 1 asin + 6 sin/cos per env.  Only the position
// controller needs the yaw angle itself (its yaw-rate error, :89-92).
struct EulerSC { float sr, cr, sp, cp, sy, cy; };

OUZ_HD void unit2(float y, float x, float& s, float& c) {
  float h2 = x * x + y * y;
  if (h2 > 0.0f) { float ih = 1.0f / sqrtf(h2); s = y * ih; c = x * ih; }
  else { s = 0.0f; c = 1.0f; }     // atan2(0, 0) = 0
}

OUZ_HD EulerSC euler_sc(const M3& R) {
  EulerSC e;
  unit2(R.m[7], R.m[8], e.sr, e.cr);
  e.sp = -R.m[6];
  e.cp = sqrtf(fmaxf(0.0f, 1.0f - R.m[6] * R.m[6]));   // cos(asin(x)) >= 0
  unit2(R.m[3], R.m[0], e.sy, e.cy);
  return e;
}

OUZ_HD void mat_to_rpy(const M3& R, float& roll, float& pitch, float& yaw) {
  roll = atan2f(R.m[7], R.m[8]);
  pitch = asinf(-R.m[6]);
  yaw = atan2f(R.m[3], R.m[0]);
}

// euler_angles_to_matrix((yaw, pitch, roll), "ZYX") = Rz Ry Rx from sines/cosines.
OUZ_HD M3 rpy_to_mat_sc(float cz, float sz, float cy, float sy, float cx, float sx) {
  return M3{{cz * cy, cz * sy * sx - sz * cx, cz * sy * cx + sz * sx, sz * cy, sz * sy * sx + cz * cx,
             sz * sy * cx - cz * sx, -sy, cy * sx, cy * cx}};
}

// euler_angles_to_matrix((yaw, pitch, roll), "ZYX") = Rz Ry Rx (rotation_conversions.py:149-171).
OUZ_HD M3 rpy_to_mat(float yaw, float pitch, float roll) {
  return rpy_to_mat_sc(cosf(yaw), sinf(yaw), cosf(pitch), sinf(pitch), cosf(roll), sinf(roll));
}

// my_quat_rotate / quat_rotate, xyzw (utils/torch_jit_utils.py:198-208).
OUZ_HD V3 quat_rotate(Q4 q, V3 v) {
  V3 qv = v3(q.x, q.y, q.z);
  V3 a = (2.0f * q.w * q.w - 1.0f) * v;
  V3 b = (q.w * 2.0f) * cross(qv, v);
  V3 c = (dot(qv, v) * 2.0f) * qv;
  return a + b + c;
}

OUZ_HD Q4 quat_mul(Q4 a, Q4 b) {  // xyzw Hamilton product a (x) b
  return Q4{a.w * b.x + b.w * a.x + (a.y * b.z - a.z * b.y), a.w * b.y + b.w * a.y + (a.z * b.x - a.x * b.z),
            a.w * b.z + b.w * a.z + (a.x * b.y - a.y * b.x), a.w * b.w - (a.x * b.x + a.y * b.y + a.z * b.z)};
}

// ---------------------------------------------------------------------------
// Lee geometric controllers
// ---------------------------------------------------------------------------
struct LeeGains { V3 kP, kV, kR, kW; };

OUZ_HD LeeGains default_gains() {  // controllers/control_config.py:14-17
  return LeeGains{v3(0.8f, 0.8f, 1.0f), v3(0.5f, 0.5f, 0.4f), v3(3.0f, 3.0f, 1.0f), v3(0.5f, 0.5f, 1.2f)};
}

constexpr float kTwoPiF = 6.28318530717958647692f;
constexpr float kPiF = 3.14159265358979323846f;

// torch.remainder for floats: fmod, then shift into the divisor's sign.  fmod(a, b) == a
// exactly when |a| < b, which is the common case here (a = yaw command - yaw); only larger
// arguments pay for the libm fmodf.
OUZ_HD float remainder_f(float a, float b) {
  float m = (fabsf(a) < b) ? a : fmodf(a, b);
  if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
  return m;
}

// Shared attitude loop (position_control.py:66-108): returns torque.
OUZ_HD V3 lee_attitude_loop(const M3& R, const M3& Rd, V3 omega, const EulerSC& e, float yaw_rate,
                            const LeeGains& g) {
  // A = Rd^T R ; vee(A - A^T) = (A21 - A12, A02 - A20, A10 - A01)
  M3 A;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      A.m[i * 3 + j] = Rd.m[0 * 3 + i] * R.m[0 * 3 + j] + Rd.m[1 * 3 + i] * R.m[1 * 3 + j] + Rd.m[2 * 3 + i] * R.m[2 * 3 + j];
  V3 e_R = v3(0.5f * (A.m[7] - A.m[5]), 0.5f * (A.m[2] - A.m[6]), 0.5f * (A.m[3] - A.m[1]));
  // omega_d = E (0, 0, yaw_rate), E = rotmat_euler_to_body_rates (:73-86)
  V3 wd = v3(-e.sp * yaw_rate, e.sr * e.cp * yaw_rate, e.cr * e.cp * yaw_rate);
  V3 des = mtv(A, wd);   // R^T Rd wd = (Rd^T R)^T wd
  V3 act = mtv(R, omega);
  V3 e_w = act - des;
  // + cross(w, w) == 0 (position_control.py:108)
  return v3(-g.kR.x * e_R.x - g.kW.x * e_w.x, -g.kR.y * e_R.y - g.kW.y * e_w.y, -g.kR.z * e_R.z - g.kW.z * e_w.z);
}

// LeePositionController.__call__ (controllers/position_control.py:19-109).
// cmd = (x, y, z, yaw); thrust in units of m*g, torque "inertia normalised".
// R = quat_to_mat(q) of the state quaternion (the step kernel shares it with the integrator).
OUZ_HD void lee_position_R(const M3& R, V3 p, V3 v, V3 w, V3 cmd_p, float cmd_yaw, const LeeGains& g,
                           float& thrust, V3& torque) {
  EulerSC e = euler_sc(R);
  V3 a = mul(g.kP, cmd_p - p) - mul(g.kV, v);
  a.z += 1.0f;
  thrust = a.x * R.m[2] + a.y * R.m[5] + a.z * R.m[8];
  V3 b3 = (1.0f / norm(a)) * a;
  V3 b2 = cross(b3, v3(e.cy, e.sy, 0.0f));
  b2 = (1.0f / norm(b2)) * b2;
  V3 b1 = cross(b2, b3);
  M3 Rd{{b1.x, b2.x, b3.x, b1.y, b2.y, b3.y, b1.z, b2.z, b3.z}};
  float yr = remainder_f(cmd_yaw - atan2f(R.m[3], R.m[0]), kTwoPiF);
  if (yr > kPiF) yr -= kTwoPiF;
  torque = lee_attitude_loop(R, Rd, w, e, yr, g);
}

OUZ_HD void lee_position(V3 p, Q4 q, V3 v, V3 w, V3 cmd_p, float cmd_yaw, const LeeGains& g, float& thrust,
                         V3& torque) {
  lee_position_R(quat_to_mat(q), p, v, w, cmd_p, cmd_yaw, g, thrust, torque);
}

// LeeVelocityController.__call__ (controllers/velocity_control.py:17-112).
OUZ_HD void lee_velocity(Q4 q, V3 v, V3 w, V3 cmd_v, float yaw_rate, const LeeGains& g, float& thrust,
                         V3& torque) {
  M3 R = quat_to_mat(q);
  EulerSC e = euler_sc(R);
  // vehicle frame Rz(yaw): v_vehicle = Rz^T v
  V3 vv = v3(e.cy * v.x + e.sy * v.y, -e.sy * v.x + e.cy * v.y, v.z);
  V3 a = mul(g.kV, cmd_v - vv);
  a.z += 1.0f;
  thrust = a.x * R.m[2] + a.y * R.m[5] + a.z * R.m[8];
  // pitch_sp = atan2(a0, a2), roll_sp = atan2(-a1, hypot(a0, a2)) (:58-60) as sin/cos
  float spt, cpt, srl, crl;
  unit2(a.x, a.z, spt, cpt);
  unit2(-a.y, sqrtf(a.z * a.z + a.x * a.x), srl, crl);
  M3 Rd = rpy_to_mat_sc(e.cy, e.sy, cpt, spt, crl, srl);
  torque = lee_attitude_loop(R, Rd, w, e, yaw_rate, g);
}

// LeeAttitudeContoller.__call__ (controllers/attitude_control.py:17-78): cmd = (T, roll, pitch, yaw_rate).
OUZ_HD void lee_attitude(Q4 q, V3 w, float cmd_t, float cmd_roll, float cmd_pitch, float yaw_rate,
                         const LeeGains& g, float& thrust, V3& torque) {
  M3 R = quat_to_mat(q);
  EulerSC e = euler_sc(R);
  M3 Rd = rpy_to_mat_sc(e.cy, e.sy, cosf(cmd_pitch), sinf(cmd_pitch), cosf(cmd_roll), sinf(cmd_roll));
  torque = lee_attitude_loop(R, Rd, w, e, yaw_rate, g);
  thrust = cmd_t + 1.0f;
}

// ---------------------------------------------------------------------------
// AHRS-EKF, executed "ang" branch (ahrs_ekf.py:1301-1337), SURVEY a12.
// q = (w, x, y, z) scalar-first; P symmetric 4x4 packed (00,01,02,03,11,12,13,22,23,33).
// ---------------------------------------------------------------------------
struct EkfQ { float w, x, y, z; };

OUZ_HD int s4(int i, int j) {  // packed index, any order
  int a = i < j ? i : j, b = i < j ? j : i;
  return a * 4 - (a * (a - 1)) / 2 + (b - a);
}

// Full symmetric 4x4 inverse via Cholesky (S is SPD: P_t + 1e-7 I), in R.  The pivots L[j][j] are only ever used
// through their inverses (the off-diagonal sums and Linv run over k < j), so each is one reciprocal square root.
template <typename R>
OUZ_HD void inv_spd4(const R S[10], R Si[10]) {
  R L[4][4] = {};
  R Ld[4];   // 1 / L[j][j]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    R d = S[s4(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
    const R inv = rsqrt_r(d);
    Ld[j] = inv;
#pragma unroll
    for (int i = j + 1; i < 4; ++i) {
      R s = S[s4(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      L[i][j] = s * inv;
    }
  }
  // Linv (lower)
  R Li[4][4] = {};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Li[i][i] = Ld[i];
#pragma unroll
    for (int j = 0; j < i; ++j) {
      R s = R(0);
#pragma unroll
      for (int k = j; k < i; ++k) s += L[i][k] * Li[k][j];
      Li[i][j] = -s * Li[i][i];
    }
  }
  // S^-1 = Linv^T Linv
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = i; j < 4; ++j) {
      R s = R(0);
#pragma unroll
      for (int k = j; k < 4; ++k) s += Li[k][i] * Li[k][j];
      Si[s4(i, j)] = s;
    }
}

constexpr float kEkfGNoise = 0.09f;   // 0.3**2, ahrs_ekf.py:1004
constexpr float kEkfAngR = 1e-7f;      // ahrs_ekf.py:1332

// The EKF update is evaluated in EkfReal and stored in f32 (q, P), like the PV step: the reference's EKF is
// numpy float64 (ahrs_ekf.py:1280-1337).  float restores the round-4 f32 evaluation (an A/B build: -DOUZ_EKF_F32).
#ifdef OUZ_EKF_F32
typedef float EkfReal;
#else
typedef double EkfReal;
#endif

// In: q (normalised prior), P. Out: q, P updated in place.  Constants are the reference's Python floats (f64):
// 0.5 * Dt with Dt = 1 / frequency, g_noise = 0.3 ** 2, the 1e-7 measurement noise.
template <typename R>
OUZ_HD void ekf_update_t(EkfQ& q, float Pf[10], V3 gf, EkfQ ang, float Dt) {
  const R h = R(0.5) * R(Dt);
  const R gx = gf.x, gy = gf.y, gz = gf.z;
  const R r = sizeof(R) == 8 ? R(1e-7) : R(kEkfAngR);
  const R gnoise = sizeof(R) == 8 ? R(0.09) : R(kEkfGNoise);
  R P[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) P[k] = (R)Pf[k];
  // Omega(x) rows (ahrs_ekf.py:1072-1106)
  const R O[4][4] = {{R(0), -gx, -gy, -gz}, {gx, R(0), gz, -gy}, {gy, -gz, R(0), gx}, {gz, gy, -gx, R(0)}};
  const R qv[4] = {(R)q.w, (R)q.x, (R)q.y, (R)q.z};
  R qt[4];
  R F[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    R s = R(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      R fij = (i == j ? R(1) : R(0)) + h * O[i][j];   // f(): (I + 0.5 Dt Omega(g)) q
      s += fij * qv[j];
      F[i][j] = (i == j ? R(1) : R(0)) + O[i][j] * h;  // dfdq: I + Omega(0.5 Dt g)
    }
    qt[i] = s;
  }
  // W = 0.5 Dt [ -q_v^T ; q_w I + skew(q_v) ]   (4x3), Q_t = 0.5 Dt g_noise W W^T
  R W[4][3] = {{-qv[1], -qv[2], -qv[3]}, {qv[0], -qv[3], qv[2]}, {qv[3], qv[0], -qv[1]}, {-qv[2], qv[1], qv[0]}};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) W[i][j] *= h;
  // FP (4x4 full)
  R FP[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      R s = R(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) s += F[i][k] * P[s4(k, j)];
      FP[i][j] = s;
    }
  R Pt[10];
  const R qs = h * gnoise;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = i; j < 4; ++j) {
      R s = R(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) s += FP[i][k] * F[j][k];
      R ww = W[i][0] * W[j][0] + W[i][1] * W[j][1] + W[i][2] * W[j][2];
      Pt[s4(i, j)] = s + qs * ww;
    }
  // S = P_t + r I ; stable identities:
  //   (I - K) P_t = r I - r^2 S^-1 ,  q_t + K v = ang - r S^-1 v
  R S[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) S[k] = Pt[k];
  S[s4(0, 0)] += r; S[s4(1, 1)] += r; S[s4(2, 2)] += r; S[s4(3, 3)] += r;
  R Si[10];
  inv_spd4<R>(S, Si);
  const R av[4] = {(R)ang.w, (R)ang.x, (R)ang.y, (R)ang.z};
  const R vv[4] = {av[0] - qt[0], av[1] - qt[1], av[2] - qt[2], av[3] - qt[3]};
  R qn[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    R s = R(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) s += Si[s4(i, j)] * vv[j];
    qn[i] = av[i] - r * s;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = i; j < 4; ++j) Pf[s4(i, j)] = (float)((i == j ? r : R(0)) - (r * r) * Si[s4(i, j)]);
  const R inv = rsqrt_r(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
  q = EkfQ{(float)(qn[0] * inv), (float)(qn[1] * inv), (float)(qn[2] * inv), (float)(qn[3] * inv)};
}

OUZ_HD void ekf_update(EkfQ& q, float P[10], V3 g, EkfQ ang, float Dt) { ekf_update_t<EkfReal>(q, P, g, ang, Dt); }

// ---------------------------------------------------------------------------
// Position/velocity KF (PVFilter.py:25-110), SURVEY a13.
// x = [p, v, b_a]; P symmetric 9x9 packed upper triangle (45 floats).
// ---------------------------------------------------------------------------
OUZ_HD constexpr int s9(int i, int j) {
  return (i <= j) ? (i * 9 - (i * (i - 1)) / 2 + (j - i)) : (j * 9 - (j * (j - 1)) / 2 + (i - j));
}

constexpr float kPvAccVar = 1.0f;     // [0.01]*3 * 100 (ekf_lee_landed.py:137)
constexpr float kPvPosVar = 1e-7f;    // ekf_lee_landed.py:408
constexpr float kPvP0 = 1000.0f;      // PVFilter.py:12

// The PV step's element formulas.  Every entry the step computes is ONE chain of explicit
// fmas in a fixed order, written once below and evaluated by two data layouts:
//  * the one-lane form (pv_predict_t / pv_correct_t): the packed covariance in one lane's registers -- the
//    large-N step kernels and the component entries;
//  * the quad-lane form (quad_pv_ql.h): the four lanes of an env split every 3x3 block by column, the full
//    symmetric covariance in LDS -- the latency-regime estimator kernels.
// Both take the same operations on the same operands for every stored element, so they agree bit for bit
// (contraction is off here: a * b + c is never fused behind the formulas' back).
template <typename T>
OUZ_HD T dot3(T a0, T a1, T a2, T b0, T b1, T b2) {   // a . b, the a0 * b0 product seeding the chain
#pragma clang fp contract(off)
  return fma(a2, b2, fma(a1, b1, a0 * b0));
}
template <typename T>
OUZ_HD T dot3s(T a0, T a1, T a2, T b0, T b1, T b2, T seed) {   // seed + a . b
#pragma clang fp contract(off)
  return fma(a2, b2, fma(a1, b1, fma(a0, b0, seed)));
}

// Inverse of a symmetric 3x3 via the adjugate (SPD inputs only).  Reads only the upper triangle.
template <typename T>
OUZ_HD M3T<T> inv_sym3(const M3T<T>& S) {
#pragma clang fp contract(off)
  const T a = S.m[0], b = S.m[1], c = S.m[2], d = S.m[4], e = S.m[5], f = S.m[8];
  const T A = fma(d, f, -(e * e)), B = fma(c, e, -(b * f)), C = fma(b, e, -(c * d));
  const T D = fma(a, f, -(c * c)), E = fma(b, c, -(a * e)), F = fma(a, d, -(b * b));
  const T inv_det = recip<T>(fma(c, C, fma(b, B, a * A)));
  return M3T<T>{{A * inv_det, B * inv_det, C * inv_det, B * inv_det, D * inv_det, E * inv_det,
                 C * inv_det, E * inv_det, F * inv_det}};
}

// M = R(q/|q|)^T, formed in f32 from the f32 quaternion as the reference's torch f32 does (PVFilter.py:31-35)
template <typename T>
OUZ_HD M3T<T> pv_rot(EkfQ q) {
  const float inv = 1.0f / sqrtf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  const M3 Mf = tr(quat_to_mat(Q4{q.x * inv, q.y * inv, q.z * inv, q.w * inv}));
  M3T<T> M;
#pragma unroll
  for (int k = 0; k < 9; ++k) M.m[k] = (T)Mf.m[k];
  return M;
}

// prediction_step, state part: x = F x + G (a - b), F = [[I, M dt, M h],[0, M, M dt],[0, 0, I]], h = dt^2 / 2
template <typename T>
OUZ_HD void pv_state_predict(T x[9], const T acc[3], const M3T<T>& M, T dt, T h) {
#pragma clang fp contract(off)
  T a1[3], a2[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T u = acc[k] - x[6 + k];
    a1[k] = fma(h, u, fma(dt, x[3 + k], h * x[6 + k]));   // -> position
    a2[k] = fma(dt, u, fma(dt, x[6 + k], x[3 + k]));      // -> velocity
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) x[i] += dot3(M.m[i * 3], M.m[i * 3 + 1], M.m[i * 3 + 2], a1[0], a1[1], a1[2]);
#pragma unroll
  for (int i = 0; i < 3; ++i) x[3 + i] = dot3(M.m[i * 3], M.m[i * 3 + 1], M.m[i * 3 + 2], a2[0], a2[1], a2[2]);
}

// prediction_step, covariance part, P' = F P F^T + q_a G G^T, by columns.  With X_{r,b} the 3x3 blocks of P and
// G_{r,b} = (F P)_{r,b}:  G_{0,b} = X_{0,b} + M (dt X_{1,b} + h X_{2,b}),  G_{1,b} = M (X_{1,b} + dt X_{2,b}),
// G_{2,b} = X_{2,b};  then with Z00 = dt G_{0,1} + h G_{0,2}, Z01 = G_{0,1} + dt G_{0,2}, Z11 = G_{1,1} + dt G_{1,2}:
//   P'_00 = G_{0,0} + Z00 M^T + q h^2 I,   P'_01 = Z01 M^T + q h dt I,   P'_11 = Z11 M^T + q dt^2 I,
//   P'_02 = G_{0,2},   P'_12 = G_{1,2},   P'_22 = X_{2,2}
// (G Q G^T = q_a [[h^2 M M^T, h dt M M^T], [dt h M M^T, dt^2 M M^T]] with M M^T = I up to M's f32 rounding,
// the same as in the reference's own f32 product: the noise is diagonal).  Column c of G_{r,b} needs only
// column c of the blocks (r, b): the quad-lane form computes its column locally and exchanges the Z's.
template <typename T>
OUZ_HD void pvf_g0(const M3T<T>& M, const T X0[3], const T X1[3], const T X2[3], T dt, T h, T out[3]) {
#pragma clang fp contract(off)
  T s[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = fma(dt, X1[k], h * X2[k]);
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = dot3s(M.m[i * 3], M.m[i * 3 + 1], M.m[i * 3 + 2], s[0], s[1], s[2], X0[i]);
}
template <typename T>
OUZ_HD void pvf_g1(const M3T<T>& M, const T X1[3], const T X2[3], T dt, T out[3]) {
#pragma clang fp contract(off)
  T s[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = fma(dt, X2[k], X1[k]);
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = dot3(M.m[i * 3], M.m[i * 3 + 1], M.m[i * 3 + 2], s[0], s[1], s[2]);
}
// column c of Z00, Z01, Z11 from column c of G_{0,1}, G_{0,2}, G_{1,1}, G_{1,2}
template <typename T>
OUZ_HD void pvf_z(const T g01[3], const T g02[3], const T g11[3], const T g12[3], T dt, T h, T z00[3], T z01[3],
                  T z11[3]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    z00[i] = fma(dt, g01[i], h * g02[i]);
    z01[i] = fma(dt, g02[i], g01[i]);
    z11[i] = fma(dt, g12[i], g11[i]);
  }
}

// prediction_step, covariance part only (the split form's covariance wave: quad_kernels.hip SplitPv)
template <typename T>
OUZ_HD void pv_cov_predict_t(T P[45], const M3T<T>& M, T dt) {
  const T h = dt * dt * T(0.5);
  const T q_a = (T)kPvAccVar, qhh = q_a * h * h, qhd = q_a * h * dt, qdd = q_a * dt * dt;
  // every G column from the old P before anything is written: g[b][c][i] = G_{0,b}[i][c], g1[b-1][c][i] = G_{1,b}
  T g0[3][3][3], g1[2][3][3];
#pragma unroll
  for (int b = 0; b < 3; ++b)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      T X0[3], X1[3], X2[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        X0[k] = P[s9(k, 3 * b + c)];
        X1[k] = P[s9(3 + k, 3 * b + c)];
        X2[k] = P[s9(6 + k, 3 * b + c)];
      }
      pvf_g0(M, X0, X1, X2, dt, h, g0[b][c]);
      if (b > 0) pvf_g1(M, X1, X2, dt, g1[b - 1][c]);
    }
  T z00[3][3], z01[3][3], z11[3][3];   // [column][row]
#pragma unroll
  for (int c = 0; c < 3; ++c) pvf_z(g0[1][c], g0[2][c], g1[0][c], g1[1][c], dt, h, z00[c], z01[c], z11[c]);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const T m0 = M.m[c * 3], m1 = M.m[c * 3 + 1], m2 = M.m[c * 3 + 2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i <= c) P[s9(i, c)] = dot3s(z00[0][i], z00[1][i], z00[2][i], m0, m1, m2, i == c ? g0[0][c][i] + qhh : g0[0][c][i]);
      P[s9(i, 3 + c)] = dot3s(z01[0][i], z01[1][i], z01[2][i], m0, m1, m2, i == c ? qhd : T(0));
      if (i <= c) P[s9(3 + i, 3 + c)] = dot3s(z11[0][i], z11[1][i], z11[2][i], m0, m1, m2, i == c ? qdd : T(0));
      P[s9(i, 6 + c)] = g0[2][c][i];
      P[s9(3 + i, 6 + c)] = g1[1][c][i];
    }
  }
}

template <typename T>
OUZ_HD void pv_predict_t(T x[9], T P[45], const T acc[3], EkfQ q, T dt) {
  const M3T<T> M = pv_rot<T>(q);
  const T h = dt * dt * T(0.5);
  pv_state_predict(x, acc, M, dt, h);
  pv_cov_predict_t(P, M, dt);
}

// correction_step for one measured block m (0 = position, 1 = velocity) with R = r I.
// Stable form of x += K (z - x_m); P = (I - K H) P  (DESIGN.md §4), the other blocks A < B:
//   S = P_mm + r I;  K_o = P_om S^-1;  x_m = z - r S^-1 y;  x_o += K_o y   (y = z - x_m)
//   P_oo' = P_oo' - K_o P_mo';  P_mo = r K_o^T;  P_mm = r (I - r S^-1)
// R0 = true: the velocity fix as the reference runs it, R = 0 (PVFilter.py:76-79 tests gps_var): x_m = z and
// P_mm = P_mo = 0, written as zeros (IEEE f64 cannot fold 0 * x).
// Row i of K_o = row i of P_om times S^-1; element (i, c) of an updated block = seed - (row i of K) . (column c
// of P_mo); the quad-lane form computes row c of each K and column c of each block.
// The correction in three parts, each element by the same formula wherever it is evaluated: the gains from
// the covariance, the state update from the gains, the covariance update from the gains.
template <int MB, typename T>
OUZ_HD void pv_gain_t(const T P[45], T r, M3T<T>& Si, T KA[3][3], T KB[3][3]) {
#pragma clang fp contract(off)
  constexpr int A = (MB == 0) ? 1 : 0;   // the two other blocks, A < B
  constexpr int B = 2;
  M3T<T> S;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) S.m[i * 3 + j] = P[s9(3 * MB + i, 3 * MB + j)];
  S.m[0] += r; S.m[4] += r; S.m[8] += r;
  Si = inv_sym3(S);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      KA[i][j] = dot3(P[s9(3 * A + i, 3 * MB)], P[s9(3 * A + i, 3 * MB + 1)], P[s9(3 * A + i, 3 * MB + 2)],
                      Si.m[j], Si.m[3 + j], Si.m[6 + j]);
      KB[i][j] = dot3(P[s9(3 * B + i, 3 * MB)], P[s9(3 * B + i, 3 * MB + 1)], P[s9(3 * B + i, 3 * MB + 2)],
                      Si.m[j], Si.m[3 + j], Si.m[6 + j]);
    }
}

template <int MB, typename T, bool R0 = false>
OUZ_HD void pv_x_correct_t(T x[9], const T z[3], T r, const M3T<T>& Si, const T KA[3][3], const T KB[3][3]) {
#pragma clang fp contract(off)
  constexpr int A = (MB == 0) ? 1 : 0;
  constexpr int B = 2;
  T y[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) y[k] = z[k] - x[MB * 3 + k];
  T xm[3], dA[3], dB[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    xm[i] = R0 ? z[i] : fma(-r, dot3(Si.m[i * 3], Si.m[i * 3 + 1], Si.m[i * 3 + 2], y[0], y[1], y[2]), z[i]);
    dA[i] = dot3(KA[i][0], KA[i][1], KA[i][2], y[0], y[1], y[2]);
    dB[i] = dot3(KB[i][0], KB[i][1], KB[i][2], y[0], y[1], y[2]);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    x[MB * 3 + k] = xm[k];
    x[A * 3 + k] += dA[k];
    x[B * 3 + k] += dB[k];
  }
}

template <int MB, typename T, bool R0 = false>
OUZ_HD void pv_cov_correct_t(T P[45], T r, const M3T<T>& Si, const T KA[3][3], const T KB[3][3]) {
#pragma clang fp contract(off)
  constexpr int A = (MB == 0) ? 1 : 0;
  constexpr int B = 2;
  // the other-other blocks first: they read the m-row blocks, which are overwritten below
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const T pb0 = P[s9(3 * MB, 6 + c)], pb1 = P[s9(3 * MB + 1, 6 + c)], pb2 = P[s9(3 * MB + 2, 6 + c)];
    const T pa0 = P[s9(3 * MB, 3 * A + c)], pa1 = P[s9(3 * MB + 1, 3 * A + c)], pa2 = P[s9(3 * MB + 2, 3 * A + c)];
    T bb[3], ab[3], aa[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      bb[i] = dot3s(-KB[i][0], -KB[i][1], -KB[i][2], pb0, pb1, pb2, P[s9(6 + i, 6 + c)]);
      ab[i] = dot3s(-KA[i][0], -KA[i][1], -KA[i][2], pb0, pb1, pb2, P[s9(3 * A + i, 6 + c)]);
      aa[i] = dot3s(-KA[i][0], -KA[i][1], -KA[i][2], pa0, pa1, pa2, P[s9(3 * A + i, 3 * A + c)]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i <= c) P[s9(6 + i, 6 + c)] = bb[i];
      P[s9(3 * A + i, 6 + c)] = ab[i];
      if (i <= c) P[s9(3 * A + i, 3 * A + c)] = aa[i];
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if constexpr (R0) {
        if (MB < A) P[s9(3 * MB + i, 3 * A + c)] = T(0); else P[s9(3 * A + i, 3 * MB + c)] = T(0);
        P[s9(3 * MB + i, 6 + c)] = T(0);
        if (i <= c) P[s9(3 * MB + i, 3 * MB + c)] = T(0);
      } else {
        if (MB < A) P[s9(3 * MB + i, 3 * A + c)] = r * KA[c][i]; else P[s9(3 * A + i, 3 * MB + c)] = r * KA[i][c];
        P[s9(3 * MB + i, 6 + c)] = r * KB[c][i];
        if (i <= c) P[s9(3 * MB + i, 3 * MB + c)] = r * fma(-r, Si.m[i * 3 + c], i == c ? T(1) : T(0));
      }
    }
}

template <int MB, typename T, bool R0 = false>
OUZ_HD void pv_correct_t(T x[9], T P[45], const T z[3], T r) {
  M3T<T> Si;
  T KA[3][3], KB[3][3];
  pv_gain_t<MB, T>(P, r, Si, KA, KB);
  pv_x_correct_t<MB, T, R0>(x, z, r, Si, KA, KB);
  pv_cov_correct_t<MB, T, R0>(P, r, Si, KA, KB);
}

// One PV-filter step as the driver runs it (ekf_lee_landed.py:417-444): predict, then the
// position fix if triggered, then the velocity fix (R = 0) if triggered.  The state and
// covariance are STORED in f32 but the whole step is evaluated in PvReal: the covariance
// carries ~10 decades between the R = 1e-7 fixed position and the O(1e3) bias directions,
// and rounding it to f32 between predict and correct loses the bias information
// (the reference's own f32 evaluation drifts by ~2x the state).
typedef double PvReal;

OUZ_HD void pv_step(float xf[9], float Pf[45], V3 acc, EkfQ q, float dt, bool pos_fix, V3 zp, bool vel_fix, V3 zv) {
  PvReal x[9], P[45];
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = (PvReal)xf[k];
#pragma unroll
  for (int k = 0; k < 45; ++k) P[k] = (PvReal)Pf[k];
  const PvReal a[3] = {(PvReal)acc.x, (PvReal)acc.y, (PvReal)acc.z};
  pv_predict_t<PvReal>(x, P, a, q, (PvReal)dt);
  if (pos_fix) {
    const PvReal z[3] = {(PvReal)zp.x, (PvReal)zp.y, (PvReal)zp.z};
    pv_correct_t<0, PvReal>(x, P, z, (PvReal)kPvPosVar);
  }
  if (vel_fix) {
    const PvReal z[3] = {(PvReal)zv.x, (PvReal)zv.y, (PvReal)zv.z};
    pv_correct_t<1, PvReal, true>(x, P, z, PvReal(0));
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) xf[k] = (float)x[k];
#pragma unroll
  for (int k = 0; k < 45; ++k) Pf[k] = (float)P[k];
}

// Single-call forms (PVFilter.prediction_step / correction_step) on f32 storage.
OUZ_HD void pv_predict(float xf[9], float Pf[45], V3 acc, EkfQ q, float dt) {
  pv_step(xf, Pf, acc, q, dt, false, acc, false, acc);
}
template <int MB>
OUZ_HD void pv_correct(float xf[9], float Pf[45], V3 z, float r) {
  PvReal x[9], P[45];
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = (PvReal)xf[k];
#pragma unroll
  for (int k = 0; k < 45; ++k) P[k] = (PvReal)Pf[k];
  const PvReal zz[3] = {(PvReal)z.x, (PvReal)z.y, (PvReal)z.z};
  pv_correct_t<MB, PvReal>(x, P, zz, (PvReal)r);
#pragma unroll
  for (int k = 0; k < 9; ++k) xf[k] = (float)x[k];
#pragma unroll
  for (int k = 0; k < 45; ++k) Pf[k] = (float)P[k];
}

// ---------------------------------------------------------------------------
// Reward / observation
// ---------------------------------------------------------------------------
// compute_ingenuity_reward (tasks/ekf_lee_landed.py:692-723).
// distance to the target: the reward's position term and the die test (one formula for both)
OUZ_HD float target_dist(V3 p, V3 target) {
  V3 d = target - p;
  return sqrtf(dot(d, d));
}

OUZ_HD float reward(V3 p, V3 target, Q4 q, V3 w, float& dist) {
  dist = target_dist(p, target);
  float pos_r = 1.0f / (1.0f + dist * dist);
  float ups_z = 2.0f * q.w * q.w - 1.0f + q.z * q.z * 2.0f;      // quat_axis(q, 2).z
  float tilt = fabsf(1.0f - ups_z);
  float up_r = 5.0f / (1.0f + tilt * tilt);
  float spin = fabsf(w.z);
  float spin_r = 1.0f / (1.0f + spin * spin);
  return pos_r + pos_r * (up_r + spin_r);
}

// ---------------------------------------------------------------------------
// Lumped rigid-body integrator (build-defined; PhysX is closed — DESIGN.md §3)
// ---------------------------------------------------------------------------
constexpr float kGravity = 9.81f;

// f_b / tau_b: body-frame force and torque at the COM (LOCAL_SPACE, ekf_lee_landed.py:525);
// inv_I = 1/I (diagonal).  Semi-implicit Euler; exact exponential map for the attitude.
// Landing deck of the husky (build-defined contact; oracle deck_contact): the drone
// root rests at z 0.375 (the reference's recorded landings), footprint = the disk inscribed in the
// 0.5709 m wide chassis (husky.urdf:61-69).  Inelastic, sticking: on the deck the drone moves with
// the platform and stops rotating.
constexpr float kDeckZRest = 0.375f;
constexpr float kDeckRadius2 = (0.5709f * 0.5f) * (0.5709f * 0.5f);
struct DeckContact {
  bool on;
  float px, py, vx, vy;   // platform position / velocity (xy)
};

// kThrustOnly: f_b = (0, 0, f_b.z) (every task's rotor force is along body z); the world force is then
// R's third column times f_b.z, the same value mv(R, f_b) rounds to without its multiplies by zero.
template <bool kThrustOnly = false>
OUZ_HD void integrate(V3& p, Q4& q, V3& v, V3& w, V3 f_b, V3 tau_b, float inv_m, V3 I, V3 inv_I, float dt,
                      int substeps, float wmax, DeckContact deck = DeckContact{false, 0.f, 0.f, 0.f, 0.f}) {
  const float h = dt / (float)substeps;
  for (int s = 0; s < substeps; ++s) {
    M3 R = quat_to_mat(q);
    V3 fw = kThrustOnly ? v3(R.m[2] * f_b.z, R.m[5] * f_b.z, R.m[8] * f_b.z) : mv(R, f_b);
    v = v + h * v3(fw.x * inv_m, fw.y * inv_m, fw.z * inv_m - kGravity);
    V3 wb = mtv(R, w);
    V3 c = cross(wb, mul(I, wb));
    wb = wb + h * mul(inv_I, tau_b - c);
    w = mv(R, wb);
    float n2 = dot(w, w);
    if (n2 > wmax * wmax) w = (wmax / sqrtf(n2)) * w;
    p = p + h * v;
    if (deck.on) {
      const float dx = p.x - deck.px, dy = p.y - deck.py;
      if (dx * dx + dy * dy < kDeckRadius2 && p.z < kDeckZRest) {
        p.z = kDeckZRest;
        v = v3(deck.vx, deck.vy, fmaxf(v.z, 0.0f));
        w = v3(0.0f, 0.0f, 0.0f);
      }
    }
    // dq = [sin(th) w/|w|, cos(th)], th = |w| h / 2.  |w| <= wmax keeps th small at the
    // configured dt (4 pi * 0.005 / 2 = 0.031 rad): there the Taylor series to th^5 / th^6
    // is exact in f32 and replaces the libm sin/cos.
    float n = sqrtf(dot(w, w));
    float th = 0.5f * h * n, th2 = th * th;
    float sc, co;
    if (th < 0.1f) {
      sc = 0.5f * h * (1.0f - th2 * (1.0f / 6.0f) * (1.0f - th2 * (1.0f / 20.0f)));        // sin(th)/|w|
      co = 1.0f - 0.5f * th2 * (1.0f - th2 * (1.0f / 12.0f) * (1.0f - th2 * (1.0f / 30.0f)));
    } else {
      sc = sinf(th) / n;
      co = cosf(th);
    }
    Q4 dq{w.x * sc, w.y * sc, w.z * sc, co};
    q = quat_mul(dq, q);
    float qi = 1.0f / sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q = Q4{q.x * qi, q.y * qi, q.z * qi, q.w * qi};
  }
}

// The same integrator specialised for the fused step (every task's body force is a thrust along
// body z) with the angular velocity carried in the body frame across sub-steps.  The attitude
// increment of a sub-step rotates about w itself (dq = exp(w h / 2) ⊗ q), so R_{s+1}^T w = R_s^T w:
// the body rate after sub-step s is the next sub-step's input without the world -> body -> world
// round trip, and dq ⊗ q = q ⊗ exp(w_b h / 2).  Algebraically identical to integrate<true>
// (the oracle keeps the world-frame form); it needs R(q) once at entry (shared with the
// controller), R(q)'s third column between sub-steps and R(q) once at exit for the world-frame w.
// |w| = |w_b| (the clamp) and w = 0 <=> w_b = 0 (the deck) carry over unchanged.
// NSUB > 0: that many sub-steps, unrolled; NSUB = 0: nsub sub-steps in a loop.  g: the gravity vector.
template <int NSUB>
OUZ_HD void integrate_thrust_body(V3& p, Q4& q, V3& v, V3& w, const M3& R0, float fz, V3 tau_b, float inv_m, V3 I,
                                  V3 inv_I, float h, float wmax, DeckContact deck, V3 g, int nsub = NSUB) {
  V3 wb = mtv(R0, w);
  V3 z = v3(R0.m[2], R0.m[5], R0.m[8]);
  const float acc = fz * inv_m;
  for (int s = 0; s < (NSUB > 0 ? NSUB : nsub); ++s) {   // a constant NSUB unrolls by itself
    if (s > 0)   // third column of R(q) for the unit quaternion q (normalised at the end of every sub-step)
      z = v3(2.0f * (q.x * q.z + q.y * q.w), 2.0f * (q.y * q.z - q.x * q.w), 1.0f - 2.0f * (q.x * q.x + q.y * q.y));
    // g: the sim's gravity, (0, 0, -kGravity) unless sim_params DR'd (with g.x = g.y = 0 the x / y terms round as
    // the plain products: a * b + 0 is the product)
    v = v + h * v3(z.x * acc + g.x, z.y * acc + g.y, z.z * acc + g.z);
    const V3 c = cross(wb, mul(I, wb));
    wb = wb + h * mul(inv_I, tau_b - c);
    float n2 = dot(wb, wb);
    if (n2 > wmax * wmax) { wb = (wmax / sqrtf(n2)) * wb; n2 = wmax * wmax; }
    p = p + h * v;
    if (deck.on) {
      const float dx = p.x - deck.px, dy = p.y - deck.py;
      if (dx * dx + dy * dy < kDeckRadius2 && p.z < kDeckZRest) {
        p.z = kDeckZRest;
        v = v3(deck.vx, deck.vy, fmaxf(v.z, 0.0f));
        wb = v3(0.0f, 0.0f, 0.0f);
        n2 = 0.0f;
      }
    }
    const float n = sqrtf(n2);
    const float th = 0.5f * h * n, th2 = th * th;
    float sc, co;
    if (th < 0.04f) {
      // |w| <= 4 pi at the configured dt keeps th <= 0.0315: the series to th^2 (sin) / th^4 (cos) is
      // exact in f32 there (the next terms are < 1e-8 relative)
      sc = 0.5f * h * (1.0f - th2 * (1.0f / 6.0f));
      co = 1.0f - 0.5f * th2 * (1.0f - th2 * (1.0f / 12.0f));
    } else {   // only at other dt / sub-step settings (th <= h |w|max / 2): small arguments, no range reduction
      sc = __sinf(th) / n;
      co = __cosf(th);
    }
    q = quat_mul(q, Q4{wb.x * sc, wb.y * sc, wb.z * sc, co});
    // renormalise once, after the last sub-step: a product of unit quaternions stays unit to a few
    // ulp, which the next sub-step's third-column formula tolerates
    const bool last = NSUB > 0 ? s == NSUB - 1 : s == nsub - 1;
    if (last) {
      const float qi = 1.0f / sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
      q = Q4{q.x * qi, q.y * qi, q.z * qi, q.w * qi};
    }
  }
  w = mv(quat_to_mat(q), wb);
}

}  // namespace ouz
