"""Philox4x32-10 counter-based RNG — numpy restatement (TEST INFRASTRUCTURE ONLY).

This file is part of the CPU oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product path draws
its random numbers from the bit-identical HIP implementation in
``ouzelum_amd/csrc/philox.h``.

Why a counter RNG at all: the reference draws every random number from torch's
global generators (``torch_rand_float`` via ``isaacgym.torch_utils``,
``ekf_lee_landed.py:284-286``; ``torch.rand`` in ``ouzelum.py:183-184``;
``POMDP.py:25,30``).  Those streams depend on launch order and device and
cannot be reproduced bit-for-bit on another GPU or on the CPU.  Every draw in
this build is instead a pure function of ``(seed, global_env_id, step,
stream, sub)`` so that CPU oracle and HIP kernel agree bit-exactly and results
do not depend on how many GPUs the envs are sharded over (SURVEY §7 hard part 6).

Algorithm: Salmon et al., "Parallel random numbers: as easy as 1, 2, 3"
(SC'11), Philox4x32 with 10 rounds; constants from that paper.  Pinned by the
Random123 known-answer vectors in ``tests/test_oracle_rng.py``.
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint32(0x9E3779B9)
PHILOX_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)

# Stream ids — must match ouzelum_amd/csrc/philox.h
RNG_RESET_POS = 1
RNG_TARGET = 2
RNG_TRAJ = 3
RNG_DR = 4
RNG_FAULT = 5
RNG_DRN_OBS = 6         # VecTask DR noise on observations
RNG_DRN_ACT = 7         # ... on actions
RNG_GRAV = 8            # sim_params.gravity DR (one whole-batch draw per epoch, env id BATCH_ENV)
RNG_POMDP = 16          # + call-site id
BATCH_ENV = 0xFFFFFFFF  # env id used for whole-batch draws (one coin per call)
INIT_STEP = 0xFFFFFFFF  # step id used for draws made at env creation

# POMDP call sites (reference call sites: ekf_lee_landed.py:374-375,383,403-406,659)
SITE_OBS = 0
SITE_GYR = 1
SITE_ANG = 2
SITE_ACC = 3
SITE_POS = 4
SITE_VEL = 5


def _mulhilo(a, b):
    p = a.astype(np.uint64) * b
    return (p >> np.uint64(32)).astype(np.uint32), (p & _MASK32).astype(np.uint32)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. All inputs broadcastable uint32 arrays.

    Returns four uint32 arrays (x0, x1, x2, x3).
    """
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    c0, c1, c2, c3, k0, k1 = np.broadcast_arrays(c0, c1, c2, c3, k0, k1)
    c0, c1, c2, c3 = (x.copy() for x in (c0, c1, c2, c3))
    k0 = k0.copy()
    k1 = k1.copy()
    with np.errstate(over="ignore"):
        for r in range(10):
            if r > 0:
                k0 = (k0 + PHILOX_W0).astype(np.uint32)
                k1 = (k1 + PHILOX_W1).astype(np.uint32)
            hi0, lo0 = _mulhilo(c0, PHILOX_M0)
            hi1, lo1 = _mulhilo(c2, PHILOX_M1)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def draw_u32(seed, env_id, step, stream, sub=0):
    """Four uint32 words for counter (env_id, step, stream<<8 | sub, 0), key = seed."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32(seed >> 32)
    env_id = np.asarray(env_id, dtype=np.uint64).astype(np.uint32)
    step = np.asarray(step, dtype=np.uint64).astype(np.uint32)
    c2 = np.uint32(((int(stream) << 8) | int(sub)) & 0xFFFFFFFF)
    return philox4x32_10(env_id, step, c2, np.uint32(0), k0, k1)


def u32_to_unit_f32(x):
    """[0,1) float32 with 24 random bits: (x >> 8) * 2^-24 (exact in f32)."""
    x = np.asarray(x, dtype=np.uint32)
    return ((x >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def uniform_f32(x, lo, hi):
    """lo + (hi - lo) * u, each op rounded in f32 (torch_rand_float semantics).

    The HIP side uses __fmul_rn/__fadd_rn so no FMA contraction happens and
    the two agree bit for bit.
    """
    u = u32_to_unit_f32(x)
    lo = np.float32(lo)
    hi = np.float32(hi)
    span = np.float32(hi - lo)
    return (np.float32(lo) + (span * u).astype(np.float32)).astype(np.float32)
