"""CPU-side checks of the C ABI: the library loads, exports every symbol
include/ouzelum.h declares, the Python mirror of its constants matches the
header, and argument validation fails loudly (no GPU compute is called)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ouzelum.h")


@pytest.fixture(scope="module")
def L():
    from ouzelum_amd import _lib
    return _lib


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ouz_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(L):
    names = header_functions()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ouz_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(L.SIGNATURES), "ctypes SIGNATURES table must list exactly the header's functions"
    for n in names:
        assert hasattr(L.lib, n)


def test_header_constants_match_python_mirror(L):
    src = open(HEADER).read()
    defines = dict(re.findall(r"#define (OUZ_\w+) \(?(-?\d+)\)?", src))
    assert int(defines["OUZ_ABI_VERSION"]) == L.ABI_VERSION == L.lib.ouz_abi_version()
    assert int(defines["OUZ_TASK_MIXED"]) == L.TASK_MIXED and int(defines["OUZ_NUM_TASKS"]) == L.NUM_TASKS
    assert int(defines["OUZ_POMDP_FLICKER_NOISE"]) == L.POMDP_FLICKER_NOISE
    enums = dict(re.findall(r"(OUZ_[FI]_\w+) = (\d+)", src))
    for k, v in enums.items():
        assert getattr(L, k[4:]) == int(v), k


def test_struct_layout(L):
    # must equal the static_asserts in quad_kernels.hip
    assert ctypes.sizeof(L.OuzConfig) == 88
    assert ctypes.sizeof(L.OuzBuffers) == 48
    assert ctypes.sizeof(L.OuzTaskInfo) == 32 and ctypes.sizeof(L.OuzDrNoise) == 32


def test_argument_validation_without_gpu(L):
    cfg = L.OuzConfig()
    L.lib.ouz_default_config(cfg)
    assert cfg.dt == pytest.approx(0.01) and cfg.substeps == 2 and cfg.convergence_time == 300
    h = ctypes.c_void_p()
    bad = L.OuzConfig.from_buffer_copy(cfg)
    bad.task = 17
    assert L.lib.ouz_create(bad, h) == -1 and b"unknown task" in L.lib.ouz_last_error()
    bad = L.OuzConfig.from_buffer_copy(cfg)
    bad.num_envs = 0
    assert L.lib.ouz_create(bad, h) == -1
    bad = L.OuzConfig.from_buffer_copy(cfg)
    bad.env_id_offset, bad.num_envs_total = 4096, 4096
    assert L.lib.ouz_create(bad, h) == -1 and b"out of range" in L.lib.ouz_last_error()
    assert L.lib.ouz_step(None, None, None) == -3
    assert L.lib.ouz_lee_control(0, None, None, None, None, 0, None) == 0          # n == 0 is a no-op
    assert L.lib.ouz_lee_control(5, None, None, None, None, 4, None) == -1
    with pytest.raises(ValueError):
        L.check(-1, "x")


def test_task_info(L):
    import ouzelum_amd as o
    assert o.task_info(L.TASK_EKF_LEE_LANDED).max_episode_length == 700       # EKFLeeLanded.yaml:10
    assert o.task_info(L.TASK_OUZELUM).max_episode_length == 2000             # Ouzelum.yaml:10
    assert o.task_info(L.TASK_OUZELUM).z_die == pytest.approx(0.5)            # ouzelum.py:327
    assert o.task_info(L.TASK_LEE_LANDED).uses_actions == 0


def test_no_cpu_fallback():
    import ouzelum_amd as o
    from ouzelum_amd._lib import OuzelumError
    with pytest.raises(OuzelumError):
        o.make(seed=0, task="LeeLanded", num_envs=64, sim_device="cpu", rl_device="cpu")


def test_state_slots_and_class_layout_map(L):
    """ouz_state_slots (host-side, no GPU): the estimator tasks up to 64 K envs use the trigger-class layout
    (blocks of 21 waves, one PV trigger class g % 21 per wave), every other task and size slot i = env i.
    The Python slot map (vec_task._class_layout_slots) is the inverse of the kernel's slot -> env map."""
    import numpy as np
    import torch
    from ouzelum_amd.vec_task import _class_layout_slots
    est = (L.TASK_EKF_LEE_LANDED, L.TASK_TRACKING)
    for task in range(L.NUM_TASKS):
        for n in (1, 63, 64, 4096, 8192, 65536, 65537, 4194304):
            want = ((n + 1343) // 1344) * 1344 if task in est and n <= 65536 else n
            assert L.lib.ouz_state_slots(task, n) == want, (task, n)
    assert L.lib.ouz_state_slots(99, 64) < 0 and L.lib.ouz_state_slots(0, 0) < 0
    for n, off in ((4096, 0), (456 // 2, 456 // 2), (8192, 4096), (1000, 77)):
        slot = _class_layout_slots(n, torch.device("cpu")).numpy()
        slots = L.lib.ouz_state_slots(L.TASK_TRACKING, n)
        assert len(set(slot.tolist())) == n and slot.max() < slots
        env = np.full(slots, -1)
        env[slot] = np.arange(n)
        s = np.arange(slots)
        b, r = s // 1344, s % 1344
        np.testing.assert_array_equal(env[env >= 0], (b * 1344 + (r >> 6) + 21 * (r & 63))[env >= 0])
        for w in range(slots // 64):                    # every wave holds one trigger class
            e = env[w * 64:(w + 1) * 64]
            e = e[e >= 0]
            assert len({int(x) for x in (off + e) % 21}) <= 1
