"""CPU oracle for the per-env quadrotor step (TEST INFRASTRUCTURE ONLY).

Header (read this first)
------------------------
* This module is the *checker*, never the product.  Only ``tests/``,
  ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
  import it.  The product path (``ouzelum_amd``) runs the hand-written HIP
  kernels in ``ouzelum_amd/csrc`` and fails loudly when they are missing.
* It is a vectorised numpy restatement of the reference algorithm for the hot
  path named in ``BASELINE.json``.  Every function
  cites the reference ``file:line`` it restates (paths relative to the
  reference root ``isaacgymenvs/``).
* It computes in float64 by default (``dtype`` switchable) and states each
  formula *literally* as the reference writes it (e.g. the Kalman covariance
  update ``(I - K H) P``), so that it can be pinned against the reference's own
  modules: ``tests/golden/make_golden.py`` imports the reference controller,
  EKF, PV filter, trajectory and quaternion code in the build container and
  writes the fixtures in ``tests/golden/*.npz``; ``tests/test_oracle_golden.py``
  checks this file against them.
* Parity status: the Lee controllers (a4-a7), the AHRS-EKF update (a12), the
  PV filter (a13), the trajectory tables (a20) and the xyzw quaternion rotate
  (a7/a17) are PINNED by those fixtures.  The rigid-body integrator (a9) is
  build-defined because the reference integrates inside the closed-source
  PhysX binary (``tasks/base/vec_task.py:335``) — "parity unpinned" for the
  integrator, see DESIGN.md §3.  The task glue (reset, guidance, wrench modes,
  reward/done, POMDP) is restated from the task source text.
* Random numbers come from ``oracle.philox`` (bit-identical to the HIP side).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, replace

import numpy as np

from . import philox as rng

# ---------------------------------------------------------------------------
# Physical constants
# ---------------------------------------------------------------------------
GRAVITY = 9.81                        # cfg/task/EKFLeeLanded.yaml:31 (gravity [0,0,-9.81])
DT = 0.01                             # cfg/task/*.yaml sim.dt
SUBSTEPS = 2                          # cfg/task/*.yaml sim.substeps
MAX_ANGVEL = 4.0 * math.pi            # tasks/ekf_lee_landed.py:202 (asset max_angular_velocity)

# x500 lumped rigid body (assets/x500/x500.urdf:31-35 base; :98-102 x4 rotors;
# rotor joint origins :3-29).  Rotor spin inertia is averaged over spin angle.
# The 9.3 mm COM offset along body z is neglected.
_BASE_M = 2.0
_ROTOR_M = 0.016076923076923075
_ROTOR_IXX, _ROTOR_IYY, _ROTOR_IZZ = 3.8464910483993325e-07, 2.6115851691700804e-05, 2.649858234714004e-05
ROTOR_POS = np.array([[0.174, -0.174, 0.3],
                      [-0.174, 0.174, 0.3],
                      [0.174, 0.174, 0.3],
                      [-0.174, -0.174, 0.3]])
MASS = _BASE_M + 4 * _ROTOR_M


def _lumped_inertia():
    zc = 4 * _ROTOR_M * 0.3 / MASS
    ixx = 0.02166666666666667 + _BASE_M * zc * zc
    izz = 0.04000000000000001
    r_avg = 0.5 * (_ROTOR_IXX + _ROTOR_IYY)
    for (x, y, z) in ROTOR_POS:
        ixx += r_avg + _ROTOR_M * (y * y + (z - zc) ** 2)
        izz += _ROTOR_IZZ + _ROTOR_M * (x * x + y * y)
    return np.array([ixx, ixx, izz])


INERTIA = _lumped_inertia()
# Gazebo motor model constants (assets/x500/model.sdf:516-575) — used only by the
# build-defined rotor yaw-torque model of the fault task.
MOTOR_KM = 0.016
ROTOR_DIR = np.array([1.0, 1.0, -1.0, -1.0])   # ccw, ccw, cw, cw

# Lee gains (controllers/control_config.py:14-17)
KP = np.array([0.8, 0.8, 1.0])
KV = np.array([0.5, 0.5, 0.4])
KR = np.array([3.0, 3.0, 1.0])
KOMEGA = np.array([0.5, 0.5, 1.2])

TWO_PI_F32 = float(np.float32(3.14159265358979323846 * 2.0))
PI_F32 = float(np.float32(3.14159265358979323846))


# ---------------------------------------------------------------------------
# Rotation helpers (a7)
# ---------------------------------------------------------------------------
def quat_to_matrix_wxyz(q):
    """controllers/rotation_conversions.py:36-64 (real part first, divides by |q|^2)."""
    r, i, j, k = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    two_s = 2.0 / (q * q).sum(-1)
    o = np.stack((
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
    ), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def xyzw_to_wxyz(q):
    """``robot_state[:, [6, 3, 4, 5]]`` reorder (controllers/position_control.py:28-29)."""
    return q[..., [3, 0, 1, 2]]


def matrix_to_euler_rpy(R):
    """``matrix_to_euler_angles(R, "ZYX")[:, [2, 1, 0]]`` (rotation_conversions.py:216-255).

    Returns (roll, pitch, yaw) = (atan2(R21, R22), asin(-R20), atan2(R10, R00)).
    """
    roll = np.arctan2(R[..., 2, 1], R[..., 2, 2])
    pitch = np.arcsin(-R[..., 2, 0])
    yaw = np.arctan2(R[..., 1, 0], R[..., 0, 0])
    return roll, pitch, yaw


def euler_zyx_to_matrix(yaw, pitch, roll):
    """``euler_angles_to_matrix((yaw, pitch, roll), "ZYX")`` = Rz @ Ry @ Rx
    (rotation_conversions.py:149-171 with _axis_angle_rotation :121-147)."""
    cz, sz = np.cos(yaw), np.sin(yaw)
    cy, sy = np.cos(pitch), np.sin(pitch)
    cx, sx = np.cos(roll), np.sin(roll)
    R = np.empty(np.shape(yaw) + (3, 3), dtype=np.result_type(yaw, 1.0))
    R[..., 0, 0] = cz * cy
    R[..., 0, 1] = cz * sy * sx - sz * cx
    R[..., 0, 2] = cz * sy * cx + sz * sx
    R[..., 1, 0] = sz * cy
    R[..., 1, 1] = sz * sy * sx + cz * cx
    R[..., 1, 2] = sz * sy * cx - cz * sx
    R[..., 2, 0] = -sy
    R[..., 2, 1] = cy * sx
    R[..., 2, 2] = cy * cx
    return R


def quat_rotate_xyzw(q, v):
    """``my_quat_rotate`` / ``isaacgym.torch_utils.quat_rotate`` (utils/torch_jit_utils.py:198-208)."""
    qw = q[..., 3:4]
    qv = q[..., 0:3]
    a = v * (2.0 * qw * qw - 1.0)
    b = np.cross(qv, v) * qw * 2.0
    c = qv * (qv * v).sum(-1, keepdims=True) * 2.0
    return a + b + c


def quat_axis_z(q):
    """``quat_axis(q, 2)`` (utils/torch_jit_utils.py:66-71)."""
    e = np.zeros(q.shape[:-1] + (3,), dtype=q.dtype)
    e[..., 2] = 1
    return quat_rotate_xyzw(q, e)


def vee(M):
    """controllers/math_control.py:10-16."""
    return np.stack([-M[..., 1, 2], M[..., 0, 2], -M[..., 0, 1]], -1)


def _euler_rate_to_body(roll, pitch, yaw_rate):
    """rotmat_euler_to_body_rates @ (0, 0, yaw_rate) (position_control.py:73-94)."""
    sp, cp = np.sin(pitch), np.cos(pitch)
    sr, cr = np.sin(roll), np.cos(roll)
    return np.stack([-sp * yaw_rate, sr * cp * yaw_rate, cr * cp * yaw_rate], -1)


def _lee_attitude_loop(R, Rd, omega, omega_d_body, kR, kOmega):
    """Shared tail of the three Lee controllers (position_control.py:66-108)."""
    Rt = np.swapaxes(R, -1, -2)
    Rdt = np.swapaxes(Rd, -1, -2)
    rot_err = 0.5 * vee(Rdt @ R - Rt @ Rd)
    des = (Rt @ (Rd @ omega_d_body[..., None]))[..., 0]
    act = (Rt @ omega[..., None])[..., 0]
    angvel_err = act - des
    # + torch.cross(w, w) == 0 (position_control.py:108)
    return -kR * rot_err - kOmega * angvel_err


def lee_position(state, cmd, kP=KP, kV=KV, kR=KR, kOmega=KOMEGA):
    """LeePositionController.__call__ (controllers/position_control.py:19-109).

    state: (N,13) [p, q_xyzw, v, w]; cmd: (N,4) [x, y, z, yaw].
    Returns (thrust (N,) in units of m*g, torque (N,3)).
    """
    R = quat_to_matrix_wxyz(xyzw_to_wxyz(state[:, 3:7]))
    roll, pitch, yaw = matrix_to_euler_rpy(R)
    a = kP * (cmd[:, :3] - state[:, 0:3]) - kV * state[:, 7:10]
    a[:, 2] += 1
    thrust = (a * R[:, :, 2]).sum(1)
    b3 = a / np.linalg.norm(a, axis=1, keepdims=True)
    c = np.stack([np.cos(yaw), np.sin(yaw), np.zeros_like(yaw)], 1)
    b2 = np.cross(b3, c)
    b2 = b2 / np.linalg.norm(b2, axis=1, keepdims=True)
    # torch.cross(b2_c, b3_c) without dim (position_control.py:60): dim 1 unless N == 3
    # (SURVEY App. B item 4).  The intended per-env cross product is restated here.
    b1 = np.cross(b2, b3)
    Rd = np.stack([b1, b2, b3], -1)
    yaw_rate = np.remainder(cmd[:, 3] - yaw, TWO_PI_F32)
    yaw_rate = np.where(yaw_rate > PI_F32, yaw_rate - TWO_PI_F32, yaw_rate)
    wd = _euler_rate_to_body(roll, pitch, yaw_rate)
    return thrust, _lee_attitude_loop(R, Rd, state[:, 10:13], wd, kR, kOmega)


def lee_velocity(state, cmd, kV=KV, kR=KR, kOmega=KOMEGA):
    """LeeVelocityController.__call__ (controllers/velocity_control.py:17-112)."""
    R = quat_to_matrix_wxyz(xyzw_to_wxyz(state[:, 3:7]))
    roll, pitch, yaw = matrix_to_euler_rpy(R)
    Rv = euler_zyx_to_matrix(yaw, np.zeros_like(yaw), np.zeros_like(yaw))
    vv = (np.swapaxes(Rv, 1, 2) @ state[:, 7:10, None])[..., 0]
    a = kV * (cmd[:, :3] - vv)
    a[:, 2] += 1
    thrust = (a * R[:, :, 2]).sum(1)
    pitch_sp = np.arctan2(a[:, 0], a[:, 2])
    roll_sp = np.arctan2(-a[:, 1], np.sqrt(a[:, 2] ** 2 + a[:, 0] ** 2))
    Rd = euler_zyx_to_matrix(yaw, pitch_sp, roll_sp)
    wd = _euler_rate_to_body(roll, pitch, cmd[:, 3])
    return thrust, _lee_attitude_loop(R, Rd, state[:, 10:13], wd, kR, kOmega)


def lee_attitude(state, cmd, kR=KR, kOmega=KOMEGA):
    """LeeAttitudeContoller.__call__ (controllers/attitude_control.py:17-78).

    cmd = [thrust, roll, pitch, yaw_rate]; returns (cmd0 + 1, torque).
    """
    R = quat_to_matrix_wxyz(xyzw_to_wxyz(state[:, 3:7]))
    roll, pitch, yaw = matrix_to_euler_rpy(R)
    wd = _euler_rate_to_body(roll, pitch, cmd[:, 3])
    Rd = euler_zyx_to_matrix(yaw, cmd[:, 2], cmd[:, 1])
    return cmd[:, 0] + 1, _lee_attitude_loop(R, Rd, state[:, 10:13], wd, kR, kOmega)


LEE_POSITION, LEE_VELOCITY, LEE_ATTITUDE = 0, 1, 2


def controller(mode, state, cmd):
    """Controller.__call__ dispatch (controllers/controller.py:20-48); scale_input = 1."""
    if mode == LEE_POSITION:
        return lee_position(state, cmd)
    if mode == LEE_VELOCITY:
        return lee_velocity(state, cmd)
    if mode == LEE_ATTITUDE:
        return lee_attitude(state, cmd)
    raise ValueError(f"Invalid controller name: {mode}")


# ---------------------------------------------------------------------------
# AHRS-EKF, executed branch (a12): ahrs_ekf.py:1280-1337
# ---------------------------------------------------------------------------
EKF_G_NOISE = 0.3 ** 2          # ahrs_ekf.py:1004 default noises[0]
EKF_ANG_R = 1e-7                # ahrs_ekf.py:1332


def _omega4(x):
    """EKF.Omega (ahrs_ekf.py:1072-1106)."""
    z = np.zeros_like(x[..., 0])
    return np.stack([
        np.stack([z, -x[..., 0], -x[..., 1], -x[..., 2]], -1),
        np.stack([x[..., 0], z, x[..., 2], -x[..., 1]], -1),
        np.stack([x[..., 1], -x[..., 2], z, x[..., 0]], -1),
        np.stack([x[..., 2], x[..., 1], -x[..., 0], z], -1)], -2)


def _skew(x):
    """ahrs.common.mathfuncs.skew (third-party, un-vendored): standard cross-product matrix."""
    z = np.zeros_like(x[..., 0])
    return np.stack([
        np.stack([z, -x[..., 2], x[..., 1]], -1),
        np.stack([x[..., 2], z, -x[..., 0]], -1),
        np.stack([-x[..., 1], x[..., 0], z], -1)], -2)


def ekf_update(q, P, gyr, ang, Dt=DT, g_noise=EKF_G_NOISE):
    """EKF.update with the ``ang`` measurement (ahrs_ekf.py:1301-1337), batched.

    q: (N,4) wxyz prior (already normalised by the driver, ekf_lee_landed.py:387);
    P: (N,4,4); gyr: (N,3) rad/s; ang: (N,4) wxyz measurement.
    The accelerometer input only feeds a normalisation whose result the
    executed branch never reads (ahrs_ekf.py:1306-1309), so it is not an input.
    Returns (q_new, P_new).
    """
    I4 = np.eye(4, dtype=q.dtype)
    q_t = ((I4 + 0.5 * Dt * _omega4(gyr)) @ q[..., None])[..., 0]           # f()  :1108-1133
    F = I4 + _omega4(0.5 * Dt * gyr)                                          # dfdq :1135-1158
    qv = q[..., 1:]
    W = 0.5 * Dt * np.concatenate([-qv[..., None, :],
                                   q[..., 0, None, None] * np.eye(3, dtype=q.dtype) + _skew(qv)], -2)
    Q_t = 0.5 * Dt * g_noise * (W @ np.swapaxes(W, -1, -2))
    P_t = F @ P @ np.swapaxes(F, -1, -2) + Q_t
    v = ang - q_t
    S = P_t + I4 * EKF_ANG_R
    K = P_t @ np.linalg.inv(S)
    P_new = (I4 - K) @ P_t
    qn = q_t + (K @ v[..., None])[..., 0]
    qn = qn / np.linalg.norm(qn, axis=-1, keepdims=True)
    return qn, P_new


# ---------------------------------------------------------------------------
# Position/velocity Kalman filter (a13): PVFilter.py:25-110
# ---------------------------------------------------------------------------
PV_ACC_VAR = 1.0     # acc_var = [0.01]*3 * 100 (ekf_lee_landed.py:137)
PV_POS_VAR = 1e-7    # ekf_lee_landed.py:408
PV_P0 = 1000.0       # PVFilter.py:12


def _quat_to_matrix_pv(q):
    """PVFilter.quaternion_to_matrix (PVFilter.py:113-142): normalise, then rotation_conversions."""
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    return quat_to_matrix_wxyz(q)


def pv_predict(x, P, acc, q_wxyz, dt=DT, acc_var=PV_ACC_VAR):
    """PVFilter.prediction_step (PVFilter.py:25-64), batched.

    x: (N,9); P: (N,9,9); acc: (N,3); q_wxyz: (N,4) (the driver's flip_Qw reorder is
    done by the caller).  Returns (x, P).
    """
    M = np.swapaxes(_quat_to_matrix_pv(q_wxyz), -1, -2)        # R_body_to_nav = R(q).T
    n = x.shape[0]
    F = np.broadcast_to(np.eye(9, dtype=x.dtype), (n, 9, 9)).copy()
    F[:, 0:3, 3:6] = M * dt
    F[:, 0:3, 6:9] = M * (dt ** 2) * 0.5
    F[:, 3:6, 3:6] = M
    F[:, 3:6, 6:9] = M * dt
    G = np.zeros((n, 9, 3), dtype=x.dtype)
    G[:, 0:6, 0:3] = F[:, 0:6, 6:9]
    u = acc - x[:, 6:9]
    xn = (F @ x[..., None])[..., 0] + (G @ u[..., None])[..., 0]
    Pn = F @ P @ np.swapaxes(F, 1, 2) + acc_var * (G @ np.swapaxes(G, 1, 2))
    return xn, Pn


def pv_correct(x, P, z, block, var):
    """PVFilter.correction_step for one measurement block (PVFilter.py:67-110).

    block 0 = position (gps, R = diag(var)); block 1 = velocity.  The driver's
    velocity call passes no ``gps_var`` so R = 0 (PVFilter.py:76-79, SURVEY
    App. B item 2): pass var=0.0 for the reference behaviour.
    """
    s = slice(0, 3) if block == 0 else slice(3, 6)
    R = np.eye(3, dtype=x.dtype) * var
    K = P[:, :, s] @ np.linalg.inv(P[:, s, s] + R)
    xn = x + (K @ (z - x[:, s])[..., None])[..., 0]
    IKH = np.broadcast_to(np.eye(9, dtype=x.dtype), P.shape).copy()
    IKH[:, :, s] -= K
    return xn, IKH @ P


# ---------------------------------------------------------------------------
# Trajectories (a20): utils/trajectories.py:5-60, tasks/landing.py:108-112
# ---------------------------------------------------------------------------
def lemniscate(a=math.sqrt(2), num_points=200):
    """utils/trajectories.py:5-17 (torch.linspace in f32)."""
    theta = np.linspace(-math.pi / 2, 3 * math.pi / 2, num_points).astype(np.float32)
    s, c = np.sin(theta), np.cos(theta)
    x = a * c / (s ** 2 + 1)
    y = a * c * s / (s ** 2 + 1)
    return np.stack([x, y], 1).astype(np.float32)


def circle(r=math.sqrt(2), num_points=200):
    """utils/trajectories.py:19-29."""
    step = 360 / num_points
    pts = [(r * math.cos(math.radians(i * step)), r * math.sin(math.radians(i * step)))
           for i in range(num_points)]
    return np.array(pts, dtype=np.float32)


def square(side_length=5.0, num_points=8):
    """utils/trajectories.py:31-60 (with num_points=8 this yields 4 corners)."""
    if num_points < 4:
        raise ValueError("A square needs at least 4 waypoints.")
    wps = num_points // 4
    inc = side_length / (wps - 1)
    pts = [(i * inc, 0) for i in range(wps)]
    pts += [(side_length, i * inc) for i in range(1, wps)]
    pts += [(side_length - i * inc, side_length) for i in range(1, wps)]
    pts += [(0, side_length - i * inc) for i in range(1, wps - 1)]
    return (-(np.array(pts, dtype=np.float32) - (side_length / 2))).astype(np.float32)


def waypoint_tables():
    """The three tables landing.py:108-112 builds: lemniscate(a=4,100), circle(r=2,100), square(4,8)."""
    return [lemniscate(4, 100), circle(2, 100), square(4, 8)]


# ---------------------------------------------------------------------------
# Reward / observation (a16, a17)
# ---------------------------------------------------------------------------
def compute_reward(p, target, q, w, reset_buf, progress, max_episode_length, z_die):
    """compute_ingenuity_reward (tasks/ekf_lee_landed.py:692-723; ouzelum.py:302-332)."""
    d = np.sqrt(((target - p) ** 2).sum(-1))
    pos_r = 1.0 / (1.0 + d * d)
    ups = quat_axis_z(q)
    tilt = np.abs(1 - ups[..., 2])
    up_r = 5.0 / (1.0 + tilt * tilt)
    spin = np.abs(w[..., 2])
    spin_r = 1.0 / (1.0 + spin * spin)
    rew = pos_r + pos_r * (up_r + spin_r)
    die = np.where(d > 8.0, 1, 0)
    die = np.where(p[..., 2] < z_die, 1, die)
    reset = np.where(progress >= max_episode_length - 1, 1, die)
    return rew, reset.astype(np.int64)


def compute_obs(p, target, q, v, w):
    """compute_observations (tasks/ekf_lee_landed.py:653-657; ouzelum.py:280-285)."""
    return np.concatenate([(target - p) / 3, q, v / 2, w / math.pi], -1)


# ---------------------------------------------------------------------------
# Rigid-body integrator (a9) — BUILD-DEFINED (PhysX is closed; parity unpinned)
# ---------------------------------------------------------------------------
def quat_mul_xyzw(a, b):
    aw, av = a[..., 3:4], a[..., 0:3]
    bw, bv = b[..., 3:4], b[..., 0:3]
    w = aw * bw - (av * bv).sum(-1, keepdims=True)
    v = aw * bv + bw * av + np.cross(av, bv)
    return np.concatenate([v, w], -1)


# Landing deck of the husky (build-defined contact): the drone's root rests at
# z 0.375 on the deck (the reference's recorded landings, trajectories/flicker_0.01_ep_5.csv),
# footprint = the disk inscribed in the 0.5709 m wide chassis (husky.urdf:61-69).
DECK_Z_REST = 0.375
DECK_RADIUS = 0.5709 / 2
# husky differential drive (utils/controllers.py:15-43; gains from landing.py:361)
WHEEL_BASE, WHEEL_RADIUS, MAX_WHEEL_SPEED = 0.54, 0.165, 15.0
DRIVE_GAIN_LIN, DRIVE_GAIN_ANG, DRIVE_ANG_THRESH = 3.0, 1000.0, 0.005


def map_to_pi(a):
    """utils/controllers.py:5-13 (one wrap; inputs lie in (-3 pi, 3 pi))."""
    a = np.where(a > math.pi, a - 2 * math.pi, a)
    return np.where(a <= -math.pi, a + 2 * math.pi, a)


def drive_command(cur, tgt, heading, gains=(DRIVE_GAIN_LIN, DRIVE_GAIN_ANG), max_wheel=MAX_WHEEL_SPEED):
    """differential_drive (utils/controllers.py:15-43) -> saturated (linear, angular) velocity and the
    wheel speeds (right, left, right, left) it returns."""
    dx, dy = tgt[:, 0] - cur[:, 0], tgt[:, 1] - cur[:, 1]
    dth = map_to_pi(np.arctan2(dy, dx) - map_to_pi(heading))
    dth = np.where((dth < DRIVE_ANG_THRESH) & (dth > -DRIVE_ANG_THRESH), 0.0, dth)
    lin = np.sqrt(dx ** 2 + dy ** 2) * gains[0]
    ang = dth * gains[1]
    left = (2 * lin + ang * WHEEL_BASE) / (2 * WHEEL_RADIUS)
    right = (2 * lin - ang * WHEEL_BASE) / (2 * WHEEL_RADIUS)
    mx = np.maximum(np.abs(left), np.abs(right))
    sc = np.where(mx > max_wheel, max_wheel / np.maximum(mx, 1e-30), 1.0)
    wheels = np.stack([right * sc, left * sc, right * sc, left * sc], -1)
    return lin * sc, ang * sc, wheels


def deck_contact(p, v, w, on, plat, plat_v):
    """Inelastic sticking contact with the deck: a drone inside the footprint and below the rest
    height is put on the deck, moves with the platform, and stops rotating."""
    dxy = p[:, 0:2] - plat
    hit = on & ((dxy ** 2).sum(-1) < DECK_RADIUS ** 2) & (p[:, 2] < DECK_Z_REST)
    if hit.any():
        p, v, w = p.copy(), v.copy(), w.copy()
        p[hit, 2] = DECK_Z_REST
        v[hit, 0:2] = plat_v[hit]
        v[hit, 2] = np.maximum(v[hit, 2], 0.0)
        w[hit] = 0.0
    return p, v, w


def integrate(p, q, v, w, f_b, tau_b, mass, inertia, dt=DT, substeps=SUBSTEPS, wmax=MAX_ANGVEL, contact=None,
              gravity=None):
    """Semi-implicit Euler over ``substeps`` sub-steps on a lumped rigid body.

    f_b, tau_b: body-frame force (N) and torque (N m) at the COM (LOCAL_SPACE,
    ekf_lee_landed.py:525).  mass (N,), inertia (N,3) diagonal.  Velocities are
    world frame (Isaac root-state convention).  |w| is clamped to
    ``wmax`` (asset max_angular_velocity).  Orientation uses the exact
    exponential map of the world-frame angular velocity.  ``contact`` adds the landing
    deck after each sub-step's position update (``deck_contact``).  ``gravity``: the sim's gravity vector
    (default (0, 0, -9.81); sim_params gravity DR, ``gravity_dr``).
    """
    h = dt / substeps
    g = np.array([0.0, 0.0, -GRAVITY] if gravity is None else gravity, dtype=p.dtype)
    for _ in range(substeps):
        R = quat_to_matrix_wxyz(xyzw_to_wxyz(q))
        v = v + h * ((R @ f_b[..., None])[..., 0] / mass[:, None] + g)
        wb = (np.swapaxes(R, -1, -2) @ w[..., None])[..., 0]
        wdot = (tau_b - np.cross(wb, inertia * wb)) / inertia
        wb = wb + h * wdot
        w = (R @ wb[..., None])[..., 0]
        n = np.linalg.norm(w, axis=-1)
        scale = np.where(n > wmax, wmax / np.maximum(n, 1e-30), 1.0)
        w = w * scale[:, None]
        p = p + h * v
        if contact is not None:          # (on mask, platform xy, platform velocity xy)
            p, v, w = deck_contact(p, v, w, *contact)
        n = np.linalg.norm(w, axis=-1)
        th = 0.5 * h * n
        s = np.where(th < 1e-4, 0.5 * h * (1.0 - th * th / 6.0), np.sin(th) / np.maximum(n, 1e-30))
        dq = np.concatenate([w * s[:, None], np.cos(th)[:, None]], -1)
        q = quat_mul_xyzw(dq, q)
        q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    return p, q, v, w


# ---------------------------------------------------------------------------
# POMDP sensor/observation corruption (a15): utils/POMDP.py:4-43
# ---------------------------------------------------------------------------
POMDP_NONE, POMDP_FLICKER, POMDP_NOISE, POMDP_FLICKER_NOISE = 0, 1, 2, 3
POMDP_NAMES = {"none": POMDP_NONE, "flicker": POMDP_FLICKER, "random_noise": POMDP_NOISE,
               "flickering_and_random_noise": POMDP_FLICKER_NOISE}


def pomdp_apply(x, mode, prob, seed, env_ids, step, site, batch_tag=0, per_env_coin=False):
    """POMDPWrapper.observation (utils/POMDP.py:23-43) with counter-RNG draws.

    flicker: one coin ``u <= p`` per call zeroes the whole batch (POMDP.py:25);
    ``per_env_coin`` gives the per-env calls of ekf_lee_landed.py:383 their own coin.
    random_noise: x * U(1-sigma, 1+sigma) elementwise (POMDP.py:30-31).
    flickering_and_random_noise: flicker with p=0.1, then noise sigma=prob (POMDP.py:16-18,33-40).
    """
    if mode == POMDP_NONE:
        return x
    out = x.copy()
    flick_p = prob if mode == POMDP_FLICKER else 0.1
    if mode in (POMDP_FLICKER, POMDP_FLICKER_NOISE):
        if per_env_coin:
            u = rng.u32_to_unit_f32(rng.draw_u32(seed, env_ids, step, rng.RNG_POMDP + site, 0)[0])
            out = np.where((u <= np.float32(flick_p))[:, None], 0.0, out)
        else:
            u = rng.u32_to_unit_f32(rng.draw_u32(seed, rng.BATCH_ENV, step, rng.RNG_POMDP + site, batch_tag)[0])
            if u <= np.float32(flick_p):
                out = np.zeros_like(out)
    if mode in (POMDP_NOISE, POMDP_FLICKER_NOISE):
        d = x.shape[1]
        lo = np.float32(1 - prob)
        hi = np.float32(1 + prob)
        noise = np.empty(x.shape, dtype=np.float32)
        for grp in range((d + 3) // 4):
            words = rng.draw_u32(seed, env_ids, step, rng.RNG_POMDP + site, 128 + grp)
            for k in range(4):
                e = grp * 4 + k
                if e < d:
                    noise[:, e] = rng.uniform_f32(words[k], lo, hi)
        out = out * noise.astype(out.dtype)
    return out


# ---------------------------------------------------------------------------
# VecTask DR noise lambdas (a22): tasks/base/vec_task.py:576-646, applied in step() :323-325,351-353
# ---------------------------------------------------------------------------
DRN_DIST = {"gaussian": 1, "uniform": 2}
DRN_OP = {"additive": 0, "scaling": 1}
DRN_SCHED = {None: 0, "linear": 1, "constant": 2}


def _normal_from(a, b, second):
    u1 = ((a >> np.uint32(8)).astype(np.float64) + 1.0) / 16777216.0
    u2 = rng.u32_to_unit_f32(b).astype(np.float64)
    r = np.sqrt(-2.0 * np.log(u1))
    return r * (np.sin(2 * math.pi * u2) if second else np.cos(2 * math.pi * u2))


def dr_schedule(sched, sched_steps, step):
    """Schedule scaling of a DR range at ``step`` (vec_task.py:584-589, dr_utils.py:82-87), in float32 as the
    kernel evaluates it."""
    if sched == 1:
        return float(np.float32(min(float(step), float(sched_steps))) / np.float32(sched_steps))
    if sched == 2:
        return 0.0 if step < sched_steps else 1.0
    return 1.0


def dr_noise_apply(x, p, seed, env_ids, step, stream):
    """One noise_lambda call.  p: dict with distribution/operation/range/range_correlated/schedule/schedule_steps/
    frequency (the reference's dr_params entry, names mapped to ints).  The parameters are those of the epoch
    e = step - step % frequency (do_nonenv_randomize re-derives them every ``frequency`` steps, vec_task.py:559,
    577-646): schedule at e, corr redrawn at every epoch (a new params dict has no 'corr', :610-615)."""
    if not p or p.get("distribution", 0) == 0:
        return x
    freq = int(p.get("frequency", 1))
    ep = step - step % freq if freq > 1 else step
    s = dr_schedule(p["schedule"], p["schedule_steps"], ep)
    a, b = (float(np.float32(v)) for v in p["range"])
    ac, bc = (float(np.float32(v)) for v in p["range_correlated"])
    add, gauss = p["operation"] == 0, p["distribution"] == 1
    if add:
        a, b, ac, bc = a * s, b * s, ac * s, bc * s
    elif gauss:
        b, a, bc, ac = b * s, a * s + (1 - s), bc * s, ac * s + (1 - s)
    else:
        a, b, ac, bc = (v * s + (1 - s) for v in (a, b, ac, bc))
    out = np.array(x, dtype=np.float64, copy=True)
    d = out.shape[1]
    for g in range((d + 3) // 4):
        f = rng.draw_u32(seed, env_ids, step, stream, g)
        c = rng.draw_u32(seed, env_ids, ep, stream, 64 + g)
        for k in range(4):
            e = g * 4 + k
            if e >= d:
                break
            pair = k & 2
            corr = _normal_from(c[pair], c[pair + 1], k & 1)
            if gauss:
                n = corr * bc + ac + _normal_from(f[pair], f[pair + 1], k & 1) * b + a
            else:
                n = corr * (bc - ac) + ac + rng.u32_to_unit_f32(f[k]).astype(np.float64) * (b - a) + a
            out[:, e] = out[:, e] + n if add else out[:, e] * n
    return out


# ---------------------------------------------------------------------------
# Physical DR (a22): VecTask.apply_randomizations' actor_params (vec_task.py:547-563,680-756) of the drone's lumped
# body, samples as dr_utils.generate_random_samples (:71-133), values as apply_random_samples (:148-205)
# ---------------------------------------------------------------------------
DRP_DIST = {"gaussian": 1, "uniform": 2, "loguniform": 3}
MOTOR_CONSTANT = 8.54858e-06     # assets/x500/model.sdf:523


def dr_phys_default(lo=0.9, hi=1.1):
    """QuadTracking's default: mass, inertia and motor-constant scaling ~ U(lo, hi) at every reset."""
    prm = {"distribution": 2, "operation": 1, "range": (lo, hi), "schedule": 0, "schedule_steps": 0, "setup_only": 0}
    return {"frequency": 1, "params": [dict(prm) for _ in range(3)]}


def dr_sample(p, u, u2, step):
    """generate_random_samples with the counter RNG: u (and u2, the gaussian's Box-Muller partner) uint32 draws.
    The range and schedule in float32, as the kernel forms them."""
    s = np.float32(dr_schedule(p["schedule"], p["schedule_steps"], step))
    a, b = np.float32(p["range"][0]), np.float32(p["range"][1])
    one = np.float32(1.0)
    if p["operation"] == 0:
        a, b = a * s, b * s
    elif p["distribution"] == 1:
        b, a = b * s, a * s + (one - s)
    else:
        a, b = a * s + (one - s), b * s + (one - s)
    if p["distribution"] == 1:
        return float(a) + float(b) * _normal_from(u, u2, False)
    if p["distribution"] == 3:
        return np.exp(rng.uniform_f32(u, float(np.log(a).astype(np.float32)), float(np.log(b).astype(np.float32)))
                      .astype(np.float64))
    return rng.uniform_f32(u, float(a), float(b)).astype(np.float64)


def dr_scale(p, sample, nominal):
    """apply_random_samples' new value (:186-188) as a scale of the nominal one."""
    return (nominal + sample) / nominal if p["operation"] == 0 else sample


GRAVITY_NOMINAL = (0.0, 0.0, -GRAVITY)   # sim_params.gravity of every drone task (cfg/task/EKFLeeLanded.yaml:31)


def gravity_dr(p, seed, step):
    """sim_params gravity DR (vec_task.py:556-566,648-660 -> dr_utils.apply_random_samples :162-172).  The
    non-environment gate re-randomizes when ``last_step - last_rand_step >= frequency``: at step t the sample of the
    epoch e = t - t % frequency (frequency <= 1: every step), drawn ONCE for the whole sim (not per env) as
    generate_random_samples(params, 3, e) -- three samples, schedule evaluated at e -- from the counter RNG
    (words k of draw(seed, BATCH_ENV, e, RNG_GRAV, 0) and, the gaussian's Box-Muller partners, of sub-block 1).
    gravity[k] = nominal[k] * sample[k] (scaling) or nominal[k] + sample[k] (additive), per axis: a scaling sample
    leaves the zero x / y components at zero, exactly as the reference's.  ``p``: an ouz_dr_param-shaped dict plus
    ``frequency``.  Returns the (3,) gravity vector, evaluated as the kernel does (f32 sample and value)."""
    freq = int(p.get("frequency", 1))
    ep = step - step % freq if freq > 1 else step
    ids = np.array([rng.BATCH_ENV], np.int64)
    u = rng.draw_u32(seed, ids, ep, rng.RNG_GRAV, 0)
    u2 = rng.draw_u32(seed, ids, ep, rng.RNG_GRAV, 1)
    out = np.empty(3)
    for k in range(3):
        s = np.float32(np.asarray(dr_sample(p, u[k], u2[k], ep)).reshape(-1)[0])
        nom = np.float32(GRAVITY_NOMINAL[k])
        out[k] = float(nom + s if p["operation"] == 0 else nom * s)
    return out


# ---------------------------------------------------------------------------
# Task presets (BASELINE.json configs)
# ---------------------------------------------------------------------------
CTRL_RL, CTRL_LEE_TRUE, CTRL_LEE_EST = 0, 1, 2
TGT_GOAL, TGT_PLATFORM, TGT_TRAJ = 0, 1, 2

TASK_OUZELUM, TASK_LEE_LANDED, TASK_EKF_LEE_LANDED, TASK_TRACKING, TASK_FAULT, TASK_MIXED, TASK_LANDING = range(7)
TASK_NAMES = {"Ouzelum": TASK_OUZELUM, "LeeLanded": TASK_LEE_LANDED, "EKFLeeLanded": TASK_EKF_LEE_LANDED,
              "QuadTracking": TASK_TRACKING, "QuadFault": TASK_FAULT, "QuadMixed": TASK_MIXED,
              "Landing": TASK_LANDING}
MIXED_CHUNK = 1344                     # global ids per task chunk of the mixed curriculum (21 waves)
MIXED_TASKS = (TASK_LEE_LANDED, TASK_TRACKING, TASK_FAULT)


@dataclass
class TaskSpec:
    ctrl: int
    target_mode: int
    max_episode_length: int
    z_die: float
    land_radius: float          # wrench cut radius (0 = none)
    land_vs_ctrl_target: bool   # LeeLanded measures to (0,0,1), EKF to target_root_positions
    plat_offset_x: float        # target x = platform x + offset (lee_landed.py:629 / ekf_lee_landed.py:629)
    pomdp: int = POMDP_NONE
    pomdp_prob: float = 0.0
    dr: bool = False
    fault: bool = False
    motor_yaw: bool = False


def task_spec(task, pomdp=None, pomdp_prob=None, max_episode_length=0):
    if task == TASK_OUZELUM:      # tasks/ouzelum.py, cfg/task/Ouzelum.yaml
        s = TaskSpec(CTRL_RL, TGT_GOAL, 2000, 0.5, 0.0, False, 0.0)
    elif task == TASK_LEE_LANDED:  # tasks/lee_landed.py:25,263-330, cfg/task/LeeLanded.yaml
        s = TaskSpec(CTRL_LEE_TRUE, TGT_PLATFORM, 2000, 0.3, 0.2, True, 0.08, POMDP_FLICKER, 0.01)
    elif task == TASK_EKF_LEE_LANDED:  # tasks/ekf_lee_landed.py, cfg/task/EKFLeeLanded.yaml
        s = TaskSpec(CTRL_LEE_EST, TGT_PLATFORM, 700, 0.3, 0.25, False, -0.08, POMDP_FLICKER, 0.0)
    elif task == TASK_TRACKING:   # config C: EKF pipeline + kinematic trajectory platform + DR
        s = TaskSpec(CTRL_LEE_EST, TGT_TRAJ, 700, 0.3, 0.25, False, -0.08, POMDP_FLICKER, 0.0, dr=True)
    elif task == TASK_LANDING:    # tasks/landing.py, cfg/task/Landing.yaml: RL thrust, husky on its trajectories
        s = TaskSpec(CTRL_RL, TGT_TRAJ, 2000, 0.3, 0.0, False, 0.08)
    elif task == TASK_FAULT:      # config D: RL thrust + single-rotor fault + obs noise
        s = TaskSpec(CTRL_RL, TGT_GOAL, 2000, 0.5, 0.0, False, 0.0, POMDP_NOISE, 0.1,
                     fault=True, motor_yaw=True)
    else:
        raise ValueError(f"no single spec for task {task}")
    if pomdp is not None:
        s = replace(s, pomdp=pomdp)
    if pomdp_prob is not None:
        s = replace(s, pomdp_prob=pomdp_prob)
    if max_episode_length:       # env.maxEpisodeLength from the task YAML
        s = replace(s, max_episode_length=int(max_episode_length))
    return s


@dataclass
class EnvConfig:
    task: int = TASK_LEE_LANDED
    num_envs: int = 64
    seed: int = 0
    env_id_offset: int = 0
    num_envs_total: int = 0      # 0 -> num_envs
    pomdp: int | None = None     # None -> task default
    pomdp_prob: float | None = None
    dt: float = DT
    substeps: int = SUBSTEPS
    convergence_time: int = 300  # cfg/task/EKFLeeLanded.yaml:18 (in sim steps, ekf_lee_landed.py:339)
    plat_speed: float = MAX_WHEEL_SPEED * WHEEL_RADIUS   # max husky speed (m/s): 15 rad/s wheels
    dr_lo: float = 0.9
    dr_hi: float = 1.1
    fault_eta_hi: float = 0.5
    thrust_max: float = 2000.0   # ouzelum.py:91
    thrust_rate: float = 2000.0  # ouzelum.py:237
    max_episode_length: int = 0  # 0 -> task default
    dr_phys: dict | None = None  # physical DR ({frequency, params: [mass, inertia, motor constant]}); None: task default
    dr_obs: dict | None = None   # VecTask DR noise on observations / actions (dr_noise_apply's p)
    dr_act: dict | None = None
    dr_gravity: dict | None = None   # sim_params gravity DR (gravity_dr's p); None: (0, 0, -9.81)


def env_task_ids(cfg: EnvConfig):
    gid = cfg.env_id_offset + np.arange(cfg.num_envs)
    if cfg.task == TASK_MIXED:
        return np.array(MIXED_TASKS)[(gid // MIXED_CHUNK) % len(MIXED_TASKS)]
    return np.full(cfg.num_envs, cfg.task)


class OracleEnv:
    """Vectorised CPU restatement of VecTask.step for every task preset.

    Mirrors the device kernel ``quad_step`` in ``ouzelum_amd/csrc/quad_kernels.hip``
    (same lazy-reset order, same counter-RNG draws).  Float work is done in
    ``dtype`` (float64 default); RNG-derived values are formed in float32 exactly.
    """

    def __init__(self, cfg: EnvConfig, dtype=np.float64):
        self.cfg = cfg
        self.dt_ = dtype
        n = cfg.num_envs
        self.n = n
        self.n_total = cfg.num_envs_total or n
        self.gid = (cfg.env_id_offset + np.arange(n)).astype(np.int64)
        self.task_ids = env_task_ids(cfg)
        self.specs = {t: task_spec(t, cfg.pomdp, cfg.pomdp_prob, cfg.max_episode_length)
                      for t in np.unique(self.task_ids)}
        self.sim_step = 0
        f = lambda *s: np.zeros((n,) + s, dtype=dtype)
        self.p, self.v, self.w = f(3), f(3), f(3)
        self.p[:, 2] = 1.0
        self.q = f(4)
        self.q[:, 3] = 1.0
        self.target = f(3)
        self.progress = np.zeros(n, np.int64)
        self.reset_buf = np.ones(n, np.int64)           # vec_task.py:269-270
        self.timeouts = np.zeros(n, bool)
        self.rew = f()
        self.obs = f(13)
        self.thrust = f(4)
        self.prev_v = f(3)
        self.ekf_q = f(4)
        self.ekf_P = np.broadcast_to(np.eye(4, dtype=dtype), (n, 4, 4)).copy()   # ahrs_ekf.py:997
        self.pv_x = f(9)
        self.pv_P = np.broadcast_to(np.eye(9, dtype=dtype) * PV_P0, (n, 9, 9)).copy()
        self.waypoint = f(3)
        self.plat = f(2)
        self.plat_heading = f()
        self.plat_v = f(2)            # per-step platform velocity (0 for the static platform)
        self.traj_type = np.zeros(n, np.int64)
        self.traj_sd = f()
        self.traj_idx = np.zeros(n, np.int64)
        self.dr = np.ones((n, 3), dtype)         # mass, inertia (xx / yy), motor-constant scales
        self.rand_step = np.full(n, -1, np.int64)  # step of the last physical randomization (-1: never)
        if cfg.dr_phys is not None:              # set for every env of the env object (ouz_set_dr_physical)
            on = any(q["distribution"] for q in cfg.dr_phys["params"])
            self.dr_phys = cfg.dr_phys if on else None
            self.dr_on = np.full(n, on)
        else:                                    # the task default: QuadTracking's envs
            self.dr_phys = dr_phys_default(cfg.dr_lo, cfg.dr_hi)
            self.dr_on = np.array([self.specs[t].dr for t in self.task_ids], bool)
        self.fault_rotor = np.zeros(n, np.int64)
        self.fault_eta = np.ones(n, dtype)
        self.fault_onset = np.zeros(n, np.int64)
        self.land_flag = np.zeros(n, np.int64)
        self.landings = np.zeros(n, np.int64)
        self.tables = waypoint_tables()
        for t, s in self.specs.items():
            m = self.task_ids == t
            if s.target_mode in (TGT_PLATFORM, TGT_TRAJ):
                self.target[m, 2] = 0.377            # ekf_lee_landed.py:87, lee_landed.py:41
            else:
                self.target[m, 2] = 1.0              # ouzelum.py:73
            if s.target_mode == TGT_TRAJ:
                self._new_traj(m, rng.INIT_STEP)

    # -- draws ---------------------------------------------------------------
    def _new_traj(self, m, step):
        """reset_completed_trajectories (tasks/landing.py:215-235): type U{0,1,2}, scale U(0.8,1.2), dir ±1."""
        w = rng.draw_u32(self.cfg.seed, self.gid, step, rng.RNG_TRAJ)
        ttype = (w[0] % np.uint32(3)).astype(np.int64)
        scale = rng.uniform_f32(w[1], 0.8, 1.2)
        sdir = np.where((w[2] & np.uint32(1)) == 1, np.float32(1), np.float32(-1))
        self.traj_type[m] = ttype[m]
        self.traj_sd[m] = (scale * sdir).astype(np.float32)[m]
        self.traj_idx[m] = 0

    def _traj_point(self, idx):
        out = np.zeros((self.n, 2), dtype=self.dt_)
        for t, tab in enumerate(self.tables):
            m = self.traj_type == t
            out[m] = tab[np.minimum(idx[m], len(tab) - 1)]
        return out * self.traj_sd[:, None]

    def _traj_len(self):
        return np.array([len(tb) for tb in self.tables])[self.traj_type]

    # -- one step ------------------------------------------------------------
    def step(self, actions):
        cfg = self.cfg
        n = self.n
        t = self.sim_step
        dt = cfg.dt
        dtype = self.dt_
        a = np.asarray(actions, dtype=dtype)
        a = dr_noise_apply(a, cfg.dr_act, cfg.seed, self.gid, t, rng.RNG_DRN_ACT)   # vec_task.py:323-325
        a = np.clip(a, -1.0, 1.0)                                        # vec_task.py:327
        rst = self.reset_buf != 0
        ids = self.gid
        f_b = np.zeros((n, 3), dtype)
        tau_b = np.zeros((n, 3), dtype)

        # ---- lazy reset (ekf_lee_landed.py:312-335; ouzelum.py:221-233) ----
        wr = rng.draw_u32(cfg.seed, ids, t, rng.RNG_RESET_POS)
        off = np.stack([rng.uniform_f32(wr[0], -1.5, 1.5), rng.uniform_f32(wr[1], -1.5, 1.5),
                        rng.uniform_f32(wr[2], -0.2, 1.5)], 1)
        p0 = (np.array([0, 0, 1], np.float32) + off).astype(np.float32)
        self.p[rst] = p0[rst]
        self.q[rst] = [0, 0, 0, 1]
        self.v[rst] = 0
        self.w[rst] = 0
        self.progress[rst] = 0
        self.reset_buf[rst] = 0
        self.landings[rst] += self.land_flag[rst]
        self.land_flag[rst] = 0
        if self.dr_on.any():   # apply_randomizations at reset (vec_task.py:547-563)
            ph = self.dr_phys
            first = self.rand_step < 0
            due = rst & self.dr_on & (first | (t - self.rand_step >= ph["frequency"]))
            wd = rng.draw_u32(cfg.seed, ids, t, rng.RNG_DR)
            we = rng.draw_u32(cfg.seed, ids, t, rng.RNG_DR, 1)
            for k, nominal in enumerate((MASS, INERTIA[0], MOTOR_CONSTANT)):
                q = ph["params"][k]
                if not q["distribution"]:
                    continue
                sel = due & (first | (not q.get("setup_only", 0)))
                val = dr_scale(q, dr_sample(q, wd[k], we[k], t), nominal)
                self.dr[sel, k] = np.broadcast_to(val, (n,))[sel]
            self.rand_step[due] = t
        if any(s.fault for s in self.specs.values()):
            wf = rng.draw_u32(cfg.seed, ids, t, rng.RNG_FAULT)
            m = rst & np.array([self.specs[tt].fault for tt in self.task_ids])
            self.fault_rotor[m] = (wf[0] >> np.uint32(30)).astype(np.int64)[m]
            self.fault_eta[m] = rng.uniform_f32(wf[1], 0.0, cfg.fault_eta_hi)[m]
            mx = np.array([self.specs[tt].max_episode_length for tt in self.task_ids])
            self.fault_onset[m] = (wf[2] % (mx // 2 + 1).astype(np.uint32)).astype(np.int64)[m]

        for task, spec in self.specs.items():
            m = self.task_ids == task
            if spec.ctrl == CTRL_RL:
                self._pre_rl(m, spec, a, rst, t, f_b, tau_b)
                if spec.target_mode == TGT_TRAJ:        # set_husky_actions (landing.py:298,319-364)
                    self._platform_step(m, t)
            elif spec.ctrl == CTRL_LEE_TRUE:
                self._pre_lee_true(m, spec, rst, f_b, tau_b)
            else:
                self._pre_lee_est(m, spec, rst, t, f_b, tau_b)

        self.last_f_b, self.last_tau_b = f_b.copy(), tau_b.copy()   # the wrench gym.simulate integrates
        # ---- physics (vec_task.py:332-335 -> build-defined integrator) ----
        mass = MASS * self.dr[:, 0]
        inertia = INERTIA[None, :] * self.dr[:, 1:2]
        ph = self.dr_phys
        if ph is not None and ph["params"][1]["distribution"] and ph["params"][1]["operation"] == 0:
            # additive inertia: the same sample on each diagonal entry, so the zz scale follows from the xx scale
            inertia = inertia.copy()
            inertia[:, 2] = INERTIA[2] * (1.0 + (self.dr[:, 1] - 1.0) * INERTIA[0] / INERTIA[2])
        deck_on = np.array([self.specs[tt].target_mode != TGT_GOAL for tt in self.task_ids])
        grav = gravity_dr(cfg.dr_gravity, cfg.seed, t) if cfg.dr_gravity and cfg.dr_gravity["distribution"] else None
        self.p, self.q, self.v, self.w = integrate(self.p, self.q, self.v, self.w, f_b, tau_b,
                                                   mass.astype(dtype), inertia.astype(dtype), dt, cfg.substeps,
                                                   contact=(deck_on, self.plat, self.plat_v), gravity=grav)

        # ---- post_physics_step (ekf_lee_landed.py:620-685) ----
        self.progress += 1
        for task, spec in self.specs.items():
            m = self.task_ids == task
            if spec.target_mode in (TGT_PLATFORM, TGT_TRAJ):
                self.target[m, 0] = self.plat[m, 0] + spec.plat_offset_x
                self.target[m, 1] = self.plat[m, 1]
        obs = compute_obs(self.p, self.target, self.q, self.v, self.w)
        rew = np.zeros(n, dtype)
        reset = np.zeros(n, np.int64)
        maxlen = np.zeros(n, np.int64)
        for task, spec in self.specs.items():
            m = self.task_ids == task
            obs[m] = pomdp_apply(obs[m], spec.pomdp, spec.pomdp_prob, cfg.seed, ids[m], t, rng.SITE_OBS, task)
            r, rs = compute_reward(self.p[m], self.target[m], self.q[m], self.w[m], self.reset_buf[m],
                                   self.progress[m], spec.max_episode_length, spec.z_die)
            rew[m] = r
            reset[m] = rs
            maxlen[m] = spec.max_episode_length
        self.rew = rew
        self.reset_buf = reset
        self.timeouts = (self.progress >= maxlen - 1) & (self.reset_buf != 0)   # vec_task.py:345
        obs = dr_noise_apply(obs, cfg.dr_obs, cfg.seed, ids, t, rng.RNG_DRN_OBS)  # vec_task.py:351-352
        self.obs = np.clip(obs, -5.0, 5.0)                                       # vec_task.py:353
        self.sim_step += 1
        return self.obs, self.rew, self.reset_buf, self.timeouts

    # -- RL thrust tasks (ouzelum.py:218-251) ---------------------------------
    def _pre_rl(self, m, spec, a, rst, t, f_b, tau_b):
        cfg = self.cfg
        set_t = m & ((self.progress % 500 == 0) | rst) & (spec.target_mode == TGT_GOAL)
        wt = rng.draw_u32(cfg.seed, self.gid, t, rng.RNG_TARGET)
        tx = (rng.u32_to_unit_f32(wt[0]) * np.float32(10) - np.float32(5)).astype(np.float32)
        ty = (rng.u32_to_unit_f32(wt[1]) * np.float32(10) - np.float32(5)).astype(np.float32)
        tz = (rng.u32_to_unit_f32(wt[2]) + np.float32(1)).astype(np.float32)
        self.target[set_t] = np.stack([tx, ty, tz], 1)[set_t]
        th = self.thrust[m] + cfg.dt * cfg.thrust_rate * a[m]
        th = np.clip(th, 0.0, cfg.thrust_max)
        eff = th.copy()
        if spec.fault:
            on = self.progress[m] >= self.fault_onset[m]
            k = self.fault_rotor[m]
            rows = np.nonzero(on)[0]
            eff[rows, k[rows]] *= self.fault_eta[m][rows]
        eff[rst[m]] = 0.0
        th[rst[m]] = 0.0
        if self.dr_on[m].any():   # the rotors' motor-constant scale (physical DR)
            eff = np.where(self.dr_on[m][:, None], eff * self.dr[m, 2:3], eff)
        self.thrust[m] = th
        tot = eff.sum(1)
        fb = np.zeros((m.sum(), 3), self.dt_)
        fb[:, 2] = tot
        tb = np.zeros((m.sum(), 3), self.dt_)
        tb[:, 0] = (eff * ROTOR_POS[:, 1]).sum(1)
        tb[:, 1] = -(eff * ROTOR_POS[:, 0]).sum(1)
        if spec.motor_yaw:
            tb[:, 2] = -(eff * (MOTOR_KM * ROTOR_DIR)).sum(1)
        f_b[m] = fb
        tau_b[m] = tb

    # -- Lee on true state (lee_landed.py:263-330) ----------------------------
    def _pre_lee_true(self, m, spec, rst, f_b, tau_b):
        state = np.concatenate([self.p, self.q, self.v, self.w], 1)[m]
        cmd = np.zeros((m.sum(), 4), self.dt_)
        cmd[:, 2] = 1.0
        T, tau = lee_position(state, cmd)
        fz = 2 * GRAVITY * T
        dist = np.sqrt(((cmd[:, 0:3] - state[:, 0:3]) ** 2).sum(-1))
        cut = dist < spec.land_radius
        self.land_flag[np.nonzero(m)[0][cut]] = 1
        fz = np.where(cut, 0.0, fz)
        tau = np.where(cut[:, None], 0.0, tau)
        fz = np.where(rst[m], 0.0, fz)        # forces[reset]=0; torques are kept (lee_landed.py:324-325)
        fb = np.zeros((m.sum(), 3), self.dt_)
        fb[:, 2] = fz * self.dr[m, 2]
        f_b[m] = fb
        tau_b[m] = tau

    # -- EKF + PV + Lee (ekf_lee_landed.py:308-530) ---------------------------
    def _pre_lee_est(self, m, spec, rst, t, f_b, tau_b):
        cfg = self.cfg
        dt = cfg.dt
        seed = cfg.seed
        ids = self.gid[m]
        conv = t < cfg.convergence_time
        rs = rst[m]
        p, q, v, w = self.p[m], self.q[m], self.v[m], self.w[m]
        if spec.target_mode == TGT_TRAJ:
            self._platform_step(m, t)
        lin_acc = (v - self.prev_v[m]) / dt                     # :345-346
        lin_acc[:, 2] += 9.8                                    # :366-367 (aliases into linear_accels)
        q_true_wxyz = xyzw_to_wxyz(q)
        ekf_q = self.ekf_q[m]
        if conv:
            ekf_q = q_true_wxyz.copy()                          # :349-350
        ekf_q[rs] = q_true_wxyz[rs]                             # :352-353
        pv_x = self.pv_x[m]
        pv_x[rs] = np.concatenate([p, v, np.zeros_like(p)], 1)[rs]    # :355-360
        gyr, ang = w, q_true_wxyz
        if not conv:
            gyr = pomdp_apply(w, spec.pomdp, spec.pomdp_prob, seed, ids, t, rng.SITE_GYR, self._tag(m))
            ang = pomdp_apply(q_true_wxyz, spec.pomdp, spec.pomdp_prob, seed, ids, t, rng.SITE_ANG,
                              self._tag(m), per_env_coin=True)
        qn = ekf_q / np.linalg.norm(ekf_q, axis=1, keepdims=True)
        ekf_q, ekf_P = ekf_update(qn, self.ekf_P[m], gyr, ang, Dt=dt)
        if conv:
            orient, pos_m, vel_m = q_true_wxyz, p, v
        else:
            lin_acc = pomdp_apply(lin_acc, spec.pomdp, spec.pomdp_prob, seed, ids, t, rng.SITE_ACC, self._tag(m))
            orient = ekf_q
            pos_m = pomdp_apply(p, spec.pomdp, spec.pomdp_prob, seed, ids, t, rng.SITE_POS, self._tag(m))
            vel_m = pomdp_apply(v, spec.pomdp, spec.pomdp_prob, seed, ids, t, rng.SITE_VEL, self._tag(m))
        pv_x, pv_P = pv_predict(pv_x, self.pv_P[m], lin_acc, orient, dt=dt)
        g = np.int64(t) * self.n_total + ids                    # shared trigger counters (:425-440)
        trig_p = (g % 7) == 6
        trig_v = (g % 3) == 0
        if trig_p.any():
            xc, Pc = pv_correct(pv_x[trig_p], pv_P[trig_p], pos_m[trig_p], 0, PV_POS_VAR)
            pv_x[trig_p], pv_P[trig_p] = xc, Pc
        if trig_v.any():
            xc, Pc = pv_correct(pv_x[trig_v], pv_P[trig_v], vel_m[trig_v], 1, 0.0)
            pv_x[trig_v], pv_P[trig_v] = xc, Pc
        self.prev_v[m] = v                                      # :454
        target = self.target[m]
        wp = self.waypoint[m]
        if conv:
            wp = target.copy()                                  # :464-466
        td = np.sqrt(((target - p) ** 2).sum(-1))
        wd = np.sqrt(((wp - p) ** 2).sum(-1))
        if not conv:                                            # :476-490
            chk = (wd < 0.5) | (wd > 1.0)
            raised = target + np.array([0, 0, 0.7])
            vec = raised - p
            nv = vec / np.sqrt((vec ** 2).sum(-1, keepdims=True)) * 0.75 + p
            wp = np.where(chk[:, None], nv, wp)
            chk2 = td < 0.75
            wp = np.where(chk2[:, None], target + np.array([0, 0, 0.09]), wp)
        cmd = np.concatenate([wp, np.zeros((wp.shape[0], 1))], 1)
        if conv:
            st = np.concatenate([p, q, v, w], 1)
        else:
            st = np.concatenate([pv_x[:, 0:3], q, pv_x[:, 3:6], w], 1)  # :497-500
        T, tau = lee_position(st, cmd)
        fz = 2 * GRAVITY * T                                    # :458,504
        cut = td < spec.land_radius                             # :508-515
        if not conv:
            idx = np.nonzero(m)[0][cut]
            self.land_flag[idx] = 1
        fz = np.where(cut, 0.0, fz)
        tau = np.where(cut[:, None], 0.0, tau)
        fz = np.where(rs, 0.0, fz)                              # :521
        if conv:                                                # :526-530
            fz = np.full_like(fz, -2.09 * -GRAVITY)
            tau = np.zeros_like(tau)
        fb = np.zeros((m.sum(), 3), self.dt_)
        fb[:, 2] = fz * self.dr[m, 2]
        f_b[m] = fb
        tau_b[m] = tau
        self.ekf_q[m], self.ekf_P[m] = ekf_q, ekf_P
        self.pv_x[m], self.pv_P[m] = pv_x, pv_P
        self.waypoint[m] = wp

    def _tag(self, m):
        return int(self.task_ids[np.nonzero(m)[0][0]])

    def _platform_step(self, m, t):
        """The husky following its waypoints (landing.py:319-364) as a kinematic differential-drive
        unicycle: wheel speeds from differential_drive (utils/controllers.py:15-43, gains (3, 1000)),
        saturated at 15 rad/s, integrated over dt (PhysX's skid-steer dynamics are not modelled)."""
        cfg = self.cfg
        wp = self._traj_point(self.traj_idx)
        d = np.sqrt(((wp - self.plat) ** 2).sum(-1))
        margin = np.abs(d - 0.2)                 # distance of this step's decisions from their thresholds
        adv = m & (d < 0.2)
        self.traj_idx[adv] += 1
        done = m & (self.traj_idx >= self._traj_len())
        if done.any():
            self._new_traj(done, t)
        wp = self._traj_point(self.traj_idx)
        lin, ang, _ = drive_command(self.plat, wp, self.plat_heading, max_wheel=cfg.plat_speed / WHEEL_RADIUS)
        dth = map_to_pi(np.arctan2(wp[:, 1] - self.plat[:, 1], wp[:, 0] - self.plat[:, 0]) - map_to_pi(self.plat_heading))
        margin = np.minimum(margin, np.abs(np.abs(dth) - DRIVE_ANG_THRESH))
        self.plat_margin = np.where(m, margin, np.inf) if getattr(self, "plat_margin", None) is None \
            else np.where(m, margin, self.plat_margin)
        th = map_to_pi(self.plat_heading + ang * cfg.dt)
        pv = np.stack([lin * np.cos(th), lin * np.sin(th)], 1)
        self.plat_heading[m] = th[m]
        self.plat_v[m] = pv[m]
        self.plat[m] = (self.plat + pv * cfg.dt)[m]
