"""ctypes binding of ``libouzelum_hip.so`` (the C ABI declared in ``include/ouzelum.h``).

This is the whole shim between Python and the HIP kernels: plain pointers
and sizes cross it, nothing else.  There is no CPU fallback: if the shared
library is missing or fails to load, importing this module raises
``OuzelumError`` — the product path never silently runs anything else.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so ours binds to the same libamdhip64

LIB_NAME = "libouzelum_hip.so"
# OUZ_LIB: an alternative in-tree build (probe builds of scripts/; never the product default)
LIB_PATH = os.environ.get("OUZ_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# the host build of the same step (include/ouzelum_host.h): make(sim_device="cpu")
HOST_LIB_NAME = "libouzelum_cpu.so"
HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), HOST_LIB_NAME)


class OuzelumError(RuntimeError):
    pass


# --- constants mirrored from include/ouzelum.h (checked against the library in tests) ---
ABI_VERSION = 6
LAYOUT_VERSION = 4  # the ABI version whose state-slot rules (include/ouzelum.h "State slots") the layout follows
TASK_OUZELUM, TASK_LEE_LANDED, TASK_EKF_LEE_LANDED, TASK_TRACKING, TASK_FAULT, TASK_MIXED, TASK_LANDING = range(7)
NUM_TASKS = 7
POMDP_NONE, POMDP_FLICKER, POMDP_NOISE, POMDP_FLICKER_NOISE = range(4)
LEE_POSITION, LEE_VELOCITY, LEE_ATTITUDE = range(3)
NUM_OBS, NUM_ACT = 13, 4
TGT_GOAL, TGT_PLATFORM, TGT_TRAJ = range(3)
MIXED_CHUNK = 1344
MIXED_TASKS = (TASK_LEE_LANDED, TASK_TRACKING, TASK_FAULT)
F_P, F_Q, F_V, F_W, F_TARGET, F_PREV_V, F_THRUST = 0, 3, 7, 10, 13, 16, 19
F_EKF_Q, F_EKF_P, F_PV_X, F_PV_P, F_WAYPOINT, F_PLAT, F_TRAJ_SD, F_DR, F_FAULT_ETA = 23, 27, 37, 46, 91, 94, 96, 97, 100
F_EP_RET, F_EP_SUM, F_PLAT_HEADING = 101, 102, 103
F_COUNT = 104
I_PROGRESS, I_TRAJ_TYPE, I_TRAJ_IDX, I_FAULT_ROTOR, I_FAULT_ONSET, I_LAND_FLAG, I_LANDINGS, I_EP_CNT, I_EP_LEN, \
    I_RAND_STEP = range(10)
I_COUNT = 10
DRP_MASS, DRP_INERTIA, DRP_MOTOR_CONSTANT = range(3)
DRP_COUNT = 3
BUILD_STAMPS, BUILD_TEMPORAL_STORES = 1, 2  # ouz_build_flags bits
TILE = 64  # OUZ_TILE: state is [tiles][fields][64] (ouzelum.h OUZ_FIDX)


def tiles(n):
    return (n + TILE - 1) // TILE


class OuzConfig(ctypes.Structure):
    _fields_ = [
        ("task", ctypes.c_int32), ("num_envs", ctypes.c_int32), ("env_id_offset", ctypes.c_int64),
        ("num_envs_total", ctypes.c_int64), ("seed", ctypes.c_uint64), ("device", ctypes.c_int32),
        ("pomdp", ctypes.c_int32), ("pomdp_prob", ctypes.c_float), ("dt", ctypes.c_float),
        ("substeps", ctypes.c_int32), ("convergence_time", ctypes.c_int32), ("plat_speed", ctypes.c_float),
        ("dr_lo", ctypes.c_float), ("dr_hi", ctypes.c_float), ("fault_eta_hi", ctypes.c_float),
        ("thrust_max", ctypes.c_float), ("thrust_rate", ctypes.c_float), ("track_episodes", ctypes.c_int32),
        ("max_episode_length", ctypes.c_int32),
    ]


class OuzDrNoise(ctypes.Structure):
    _fields_ = [("distribution", ctypes.c_int32), ("operation", ctypes.c_int32), ("range", ctypes.c_float * 2),
                ("range_correlated", ctypes.c_float * 2), ("schedule", ctypes.c_int32),
                ("schedule_steps", ctypes.c_int32), ("frequency", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class OuzDrParam(ctypes.Structure):
    _fields_ = [("distribution", ctypes.c_int32), ("operation", ctypes.c_int32), ("range", ctypes.c_float * 2),
                ("schedule", ctypes.c_int32), ("schedule_steps", ctypes.c_int32), ("setup_only", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class OuzDrPhysical(ctypes.Structure):
    _fields_ = [("frequency", ctypes.c_int32), ("reserved", ctypes.c_int32), ("param", OuzDrParam * 3)]


class OuzBuffers(ctypes.Structure):
    _fields_ = [("fstate", ctypes.c_void_p), ("istate", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("rew", ctypes.c_void_p), ("reset", ctypes.c_void_p), ("timeouts", ctypes.c_void_p)]


class OuzTaskInfo(ctypes.Structure):
    _fields_ = [("max_episode_length", ctypes.c_int32), ("z_die", ctypes.c_float), ("land_radius", ctypes.c_float),
                ("pomdp", ctypes.c_int32), ("pomdp_prob", ctypes.c_float), ("uses_actions", ctypes.c_int32),
                ("target_mode", ctypes.c_int32), ("plat_offset_x", ctypes.c_float)]


ADAM_MAX_TENSORS = 16   # OUZ_ADAM_MAX_TENSORS
ADAM_WS_FLOATS = 512    # OUZ_ADAM_WS_FLOATS


class OuzAdamTable(ctypes.Structure):
    _fields_ = [("n_tensors", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("numel", ctypes.c_int64 * ADAM_MAX_TENSORS), ("grad", ctypes.c_void_p * ADAM_MAX_TENSORS),
                ("param", ctypes.c_void_p * ADAM_MAX_TENSORS), ("exp_avg", ctypes.c_void_p * ADAM_MAX_TENSORS),
                ("exp_avg_sq", ctypes.c_void_p * ADAM_MAX_TENSORS)]


_P = ctypes.c_void_p
_I = ctypes.c_int32
_F = ctypes.c_float
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I64 = ctypes.c_int64

# name -> (restype, argtypes).  This table IS the list of symbols include/ouzelum.h declares.
SIGNATURES = {
    "ouz_abi_version": (_I, []),
    "ouz_source_id": (ctypes.c_char_p, []),
    "ouz_build_flags": (_U32, []),
    "ouz_split_timeouts": (_I, [_P, _I]),
    "ouz_env_split_timeouts": (_I, [_P, ctypes.POINTER(ctypes.c_uint32), _I]),
    "ouz_set_split_spin_limit": (_I, [_U32]),
    "ouz_state_slots": (_I64, [_I, _I]),
    "ouz_env_slots": (_I, [_I, _I, _I64, _P]),
    "ouz_last_error": (ctypes.c_char_p, []),
    "ouz_default_config": (None, [ctypes.POINTER(OuzConfig)]),
    "ouz_task_info_get": (_I, [_I, ctypes.POINTER(OuzTaskInfo)]),
    "ouz_create": (_I, [ctypes.POINTER(OuzConfig), ctypes.POINTER(_P)]),
    "ouz_destroy": (_I, [_P]),
    "ouz_bind": (_I, [_P, ctypes.POINTER(OuzBuffers)]),
    "ouz_init_state": (_I, [_P, _P]),
    "ouz_step": (_I, [_P, _P, _P]),
    "ouz_step_n": (_I, [_P, _P, _I, _I, _P]),
    "ouz_rollout": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "ouz_rollout_stats": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _I, _P]),
    "ouz_pre_physics": (_I, [_P, _P, _P, _P]),
    "ouz_reset_idx": (_I, [_P, _P, _I, _P]),
    "ouz_reset_all": (_I, [_P, _P]),
    "ouz_episode_stats": (_I, [_P, _P, _I, _P]),
    "ouz_step_n_stats": (_I, [_P, _P, _I, _I, _P, _I, _P]),
    "ouz_set_trace": (_I, [_P, _P, _P, _I, _I]),
    "ouz_set_dr_noise": (_I, [_P, _I, ctypes.POINTER(OuzDrNoise)]),
    "ouz_set_dr_physical": (_I, [_P, ctypes.POINTER(OuzDrPhysical)]),
    "ouz_set_dr_gravity": (_I, [_P, ctypes.POINTER(OuzDrParam), _I]),
    "ouz_get_step": (_I64, [_P]),
    "ouz_set_step": (_I, [_P, _I64]),
    "ouz_lee_control": (_I, [_I, _P, _P, _P, _P, _I, _P]),
    "ouz_ekf_update": (_I, [_P, _P, _P, _P, _F, _P, _P, _I, _P]),
    "ouz_pv_predict": (_I, [_P, _P, _P, _P, _F, _I, _P]),
    "ouz_pv_correct": (_I, [_P, _P, _P, _I, _F, _P, _I, _P]),
    "ouz_pv_step": (_I, [_P, _P, _P, _P, _F, _P, _P, _P, _P, _I, _P]),
    "ouz_pv_step_quad": (_I, [_P, _P, _P, _P, _F, _P, _P, _P, _P, _I, _P]),
    "ouz_integrate": (_I, [_P, _P, _P, _P, _P, _F, _I, _I, _P]),
    "ouz_reward": (_I, [_P, _P, _P, _I, _F, _P, _P, _I, _P]),
    "ouz_philox": (_I, [_U64, _P, _U32, _U32, _U32, _P, _I, _P]),
    "ouz_gae": (_I, [_P, _P, _P, _P, _P, _I, _I, _F, _F, _P, _P, _P]),
    "ouz_pomdp_obs": (_I, [_P, _P, _I, _I, _I, _F, _U64, _I64, _U32, _P]),
    "ouz_lstm_cell_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "ouz_lstm_cell_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "ouz_lstm_seq_pack": (_I, [_P, _I, _P, _P, _P]),
    "ouz_lstm_seq_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ouz_lstm_seq_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "ouz_ppo_policy_loss": (_I, [_P, _P, _P, _P, _P, _I, _F, _I, _P, _P, _P, _P, _P, _P, _P]),
    "ouz_ppo_value_loss": (_I, [_P, _P, _I, _P, _P, _P, _P]),
    "ouz_tanh_bwd_bias": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "ouz_policy_sample": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P]),
    "ouz_linear_tanh_small_k": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "ouz_adam_clip_step": (_I, [ctypes.POINTER(OuzAdamTable), ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, _I64, ctypes.c_double, _P, _P]),
}
LOSS_WS_DOUBLES = 10 * 256      # OUZ_LOSS_WS_DOUBLES
COLSUM_BLOCKS = 1024            # OUZ_COLSUM_BLOCKS


# include/ouzelum_host.h, the same way: this table IS the list of symbols that header declares.
HOST_SIGNATURES = {
    "ouz_host_abi_version": (_I, []),
    "ouz_host_last_error": (ctypes.c_char_p, []),
    "ouz_host_create": (_I, [ctypes.POINTER(OuzConfig), ctypes.POINTER(_P)]),
    "ouz_host_destroy": (_I, [_P]),
    "ouz_host_bind": (_I, [_P, ctypes.POINTER(OuzBuffers)]),
    "ouz_host_set_threads": (_I, [_P, _I]),
    "ouz_host_init_state": (_I, [_P]),
    "ouz_host_step": (_I, [_P, _P]),
    "ouz_host_step_n": (_I, [_P, _P, _I, _I]),
    "ouz_host_reset_idx": (_I, [_P, _P, _I]),
    "ouz_host_reset_all": (_I, [_P]),
    "ouz_host_episode_stats": (_I, [_P, _P, _I]),
    "ouz_host_set_trace": (_I, [_P, _P, _P, _I, _I]),
    "ouz_host_set_dr_noise": (_I, [_P, _I, ctypes.POINTER(OuzDrNoise)]),
    "ouz_host_set_dr_physical": (_I, [_P, ctypes.POINTER(OuzDrPhysical)]),
    "ouz_host_set_dr_gravity": (_I, [_P, ctypes.POINTER(OuzDrParam), _I]),
    "ouz_host_get_step": (_I64, [_P]),
    "ouz_host_set_step": (_I, [_P, _I64]),
}

_hostlib = None


def _missing_host_features():
    """The x86-64-v3 features (ouzelum_amd/build.py HOST_FLAGS) this CPU's /proc/cpuinfo does not list; [] where the
    file cannot be read (not Linux) or on other architectures."""
    import platform
    if platform.machine() not in ("x86_64", "AMD64"):
        return []
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("flags"):
                    have = set(line.split(":", 1)[1].split())
                    return [f for f in ("avx2", "fma", "bmi2", "movbe") if f not in have]
    except OSError:
        pass
    return []


def host_lib():
    """``libouzelum_cpu.so`` (loaded on first use: only make(sim_device="cpu") needs it)."""
    global _hostlib
    if _hostlib is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise OuzelumError(f"{HOST_LIB_NAME} not found at {HOST_LIB_PATH}: build it first "
                               "(python -m ouzelum_amd.build)")
        missing = _missing_host_features()
        if missing:   # built with -march=x86-64-v3: it would die of SIGILL on this CPU
            raise OuzelumError(f"{HOST_LIB_NAME} needs x86-64-v3 (AVX2 / FMA); this CPU lacks {missing}")
        try:
            h = ctypes.CDLL(HOST_LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise OuzelumError(f"failed to load {HOST_LIB_PATH}: {e}") from e
        for name, (res, args) in HOST_SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.ouz_host_abi_version() != ABI_VERSION:
            raise OuzelumError(f"ABI mismatch: host library {h.ouz_host_abi_version()} != binding {ABI_VERSION}")
        _hostlib = h
    return _hostlib


def host_check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = host_lib().ouz_host_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise OuzelumError(f"{what} failed ({rc}): {msg}")


def _load():
    if not os.path.exists(LIB_PATH):
        raise OuzelumError(
            f"{LIB_NAME} not found at {LIB_PATH}: build it first (python -c 'import __graft_entry__ as g; g.build()'"
            " or python -m ouzelum_amd.build). There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the machine
        raise OuzelumError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ouz_abi_version() != ABI_VERSION:
        raise OuzelumError(f"ABI mismatch: library {lib.ouz_abi_version()} != binding {ABI_VERSION}")
    flags = lib.ouz_build_flags()
    if flags and os.environ.get("OUZ_ALLOW_INSTRUMENTED") != "1":
        raise OuzelumError(f"{LIB_PATH} is an instrumented build (ouz_build_flags = {flags:#x}: "
                           f"{'stamps ' if flags & BUILD_STAMPS else ''}"
                           f"{'temporal-stores' if flags & BUILD_TEMPORAL_STORES else ''}); "
                           "set OUZ_ALLOW_INSTRUMENTED=1 to load it on purpose")
    return lib


lib = _load()

_raw_lib = None


def raw_function(name: str):
    """``name`` without ctypes' per-call argument conversion: the same entry point through a second handle of the
    already-loaded library (``RTLD_NOLOAD``: no second copy) with only its return type set.  Every argument must
    then be a ctypes instance of the declared C type (``SIGNATURES``), e.g. ``c_void_p`` / ``c_int32``.  For
    pre-bound hot calls (``QuadVecTask.rollout_plan``): about half the host time of an ``argtypes`` call."""
    global _raw_lib
    if _raw_lib is None:
        _raw_lib = ctypes.CDLL(LIB_PATH, mode=getattr(os, "RTLD_NOLOAD", 4) | getattr(os, "RTLD_NOW", 2))
    fn = getattr(_raw_lib, name)
    fn.restype = SIGNATURES[name][0]
    return fn


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib.ouz_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        raise OuzelumError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """hipStream_t of torch's current stream on ``device``.  The raw accessor costs ~0.1 us
    against ~2 us for ``torch.cuda.current_stream().cuda_stream`` — a third of a step call."""
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) else device
        return _raw_stream(torch.cuda.current_device() if idx is None else idx)
    return torch.cuda.current_stream(device).cuda_stream


def require_hip_tensor(t, name: str):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise OuzelumError(f"{name} must be a torch tensor on a HIP device (got {getattr(t, 'device', type(t))}); "
                           "the HIP path has no CPU fallback")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
