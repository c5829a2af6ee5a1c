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


def test_library_built_from_these_sources(L):
    """ouz_source_id() of the in-tree library = the id of the sources and flags in this tree (build.source_id):
    the .so the tests and the bench load is the build of this checkout, and PMC evidence matched by that id
    (bench.py load_traffic) belongs to it."""
    from ouzelum_amd import build as b
    assert L.lib.ouz_source_id().decode() == b.source_id()


def test_host_library_exports_every_host_header_symbol(L):
    """libouzelum_cpu.so (make(sim_device="cpu")) exports exactly what include/ouzelum_host.h declares."""
    src = open(os.path.join(ROOT, "include", "ouzelum_host.h")).read()
    names = sorted(set(re.findall(r"\b(ouz_host_[a-z0-9_]+)\s*\(", src)))
    assert len(names) >= 14
    out = subprocess.run(["nm", "-D", "--defined-only", L.HOST_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (ouz_\w+)", out))
    assert set(names) == exported, (set(names) ^ exported)
    assert set(names) == set(L.HOST_SIGNATURES)
    H = L.host_lib()
    assert H.ouz_host_abi_version() == L.ABI_VERSION
    cfg = L.OuzConfig()
    L.lib.ouz_default_config(cfg)
    cfg.task = 17
    h = ctypes.c_void_p()
    assert H.ouz_host_create(cfg, h) == -1 and b"unknown task" in H.ouz_host_last_error()
    assert H.ouz_host_step(None, None) == -3


def test_header_constants_match_python_mirror(L):
    src = open(HEADER).read()
    defines = dict(re.findall(r"#define (OUZ_\w+) \(?(-?\d+)\)?", src))
    assert int(defines["OUZ_ABI_VERSION"]) == L.ABI_VERSION == L.lib.ouz_abi_version()
    assert int(defines["OUZ_TASK_MIXED"]) == L.TASK_MIXED and int(defines["OUZ_NUM_TASKS"]) == L.NUM_TASKS
    assert int(defines["OUZ_POMDP_FLICKER_NOISE"]) == L.POMDP_FLICKER_NOISE
    assert 10 * int(defines["OUZ_LOSS_BLOCKS"]) == L.LOSS_WS_DOUBLES
    assert int(defines["OUZ_COLSUM_BLOCKS"]) == L.COLSUM_BLOCKS
    enums = dict(re.findall(r"(OUZ_[FI]_\w+) = (\d+)", src))
    for k, v in enums.items():
        assert getattr(L, k[4:]) == int(v), k


def test_learner_loss_entry_points_validate_without_gpu(L):
    """The loss / trunk-backward entry points refuse bad sizes and null buffers before launching anything."""
    assert L.lib.ouz_ppo_policy_loss(*([None] * 5), 1, 0.2, 1, *([None] * 7)) == -1      # norm_adv needs n > 1
    assert b"n must be" in L.lib.ouz_last_error()
    assert L.lib.ouz_ppo_policy_loss(*([None] * 5), 8, 0.2, 0, *([None] * 7)) == -1
    assert b"null buffer" in L.lib.ouz_last_error()
    assert L.lib.ouz_ppo_value_loss(None, None, 0, None, None, None, None) == -1
    assert L.lib.ouz_tanh_bwd_bias(None, None, 16, 12, None, None, None, None) == -1      # 12 columns
    assert b"power of two" in L.lib.ouz_last_error()
    assert L.lib.ouz_tanh_bwd_bias(None, None, 16, 2048, None, None, None, None) == -1
    assert L.lib.ouz_tanh_bwd_bias(None, None, 16, 256, None, None, None, None) == -1
    assert b"null buffer" in L.lib.ouz_last_error()


def test_lstm_seq_and_adam_entry_points_validate_without_gpu(L):
    """The sequence-kernel and clipped-Adam entry points refuse bad sizes, misaligned or inconsistent buffers and bad
    tables before launching anything (fake device addresses: nothing is dereferenced on the host)."""
    A, M = 0x10000, 0x10004   # a 16-byte aligned and a misaligned fake address
    fwd = L.lib.ouz_lstm_seq_fwd
    assert fwd(A, A, A, A, A, 16, 8, 64, None, None, A, None, None, None, None, None) == -1
    assert b"H must be 128" in L.lib.ouz_last_error()
    assert fwd(M, A, A, A, A, 16, 8, 128, None, None, A, None, None, None, None, None) == -1
    assert b"16-byte aligned" in L.lib.ouz_last_error()
    assert fwd(A, A, A, A, A, 16, 8, 128, A, None, A, A, A, None, None, None) == -1
    assert b"all four or none" in L.lib.ouz_last_error()
    assert fwd(A, A, A, A, A, 16, 8, 128, None, None, A, None, None, A, None, None) == -1   # h_out without c_out
    bwd = L.lib.ouz_lstm_seq_bwd
    assert bwd(A, A, A, A, A, A, None, None, 16, 8, 128, M, None, None, None) == -1
    assert b"16-byte aligned" in L.lib.ouz_last_error()
    assert bwd(A, A, A, A, A, A, None, None, 0, 8, 128, A, None, None, None) == -1
    assert ctypes.sizeof(L.OuzAdamTable) == 8 + 5 * 8 * L.ADAM_MAX_TENSORS
    t = L.OuzAdamTable()
    ws = A
    for n in (0, L.ADAM_MAX_TENSORS + 1):
        t.n_tensors = n
        assert L.lib.ouz_adam_clip_step(t, 1e-3, 0.9, 0.999, 1e-5, 1, 1.0, ws, None) == -1
        assert b"tensors" in L.lib.ouz_last_error()
    t.n_tensors, t.numel[0] = 1, 4
    t.grad[0] = t.param[0] = t.exp_avg[0] = A
    assert L.lib.ouz_adam_clip_step(t, 1e-3, 0.9, 0.999, 1e-5, 1, 1.0, ws, None) == -1      # exp_avg_sq null
    assert b"null tensor" in L.lib.ouz_last_error()
    t.exp_avg_sq[0] = A
    assert L.lib.ouz_adam_clip_step(t, 1e-3, 0.9, 0.999, 1e-5, 0, 1.0, ws, None) == -1      # steps count from 1
    assert L.lib.ouz_adam_clip_step(t, 1e-3, 0.9, 0.999, 1e-5, 1, 1.0, None, None) == -1    # no workspace
    st = L.lib.ouz_linear_tanh_small_k
    assert st(A, A, A, 16, 17, 512, A, None) == -1 and b"K <= 16" in L.lib.ouz_last_error()
    assert st(A, A, A, 16, 13, 384, A, None) == -1 and b"power of two" in L.lib.ouz_last_error()
    assert st(A, A, A, 16, 13, 512, M, None) == -1 and b"16-byte aligned" in L.lib.ouz_last_error()
    assert st(A, None, A, 16, 13, 512, A, None) == -1 and b"null buffer" in L.lib.ouz_last_error()
    assert st(A, A, A, 0, 13, 512, A, None) == 0   # no rows: nothing to launch


def test_struct_layout(L):
    # must equal the static_asserts in quad_kernels.hip
    assert ctypes.sizeof(L.OuzConfig) == 88
    assert ctypes.sizeof(L.OuzBuffers) == 48
    assert ctypes.sizeof(L.OuzTaskInfo) == 32 and ctypes.sizeof(L.OuzDrNoise) == 40
    assert ctypes.sizeof(L.OuzDrParam) == 32 and ctypes.sizeof(L.OuzDrPhysical) == 104


def test_dr_physical_validation_without_gpu(L):
    """ouz_set_dr_physical / ouz_host_set_dr_physical refuse bad parameters before touching the env."""
    p = L.OuzDrPhysical()
    p.frequency = -1
    assert L.lib.ouz_set_dr_physical(None, p) == -1
    cfg = L.OuzConfig()
    L.lib.ouz_default_config(cfg)
    H = L.host_lib()
    h = ctypes.c_void_p()
    assert H.ouz_host_create(cfg, h) == 0
    try:
        assert H.ouz_host_set_dr_physical(h, p) == -1 and b"frequency" in H.ouz_host_last_error()
        p.frequency = 1
        p.param[0].distribution = 3
        p.param[0].range[0], p.param[0].range[1] = 0.0, 1.0
        assert H.ouz_host_set_dr_physical(h, p) == -1 and b"loguniform" in H.ouz_host_last_error()
        p.param[0].range[0] = 0.5
        p.param[0].schedule = 1
        assert H.ouz_host_set_dr_physical(h, p) == -1 and b"schedule_steps" in H.ouz_host_last_error()
        p.param[0].schedule_steps = 10
        assert H.ouz_host_set_dr_physical(h, p) == 0
        assert H.ouz_host_set_dr_physical(h, None) == 0
    finally:
        H.ouz_host_destroy(h)


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
    """A HIP env never falls back to the CPU: without a visible device, sim_device="cuda:0" raises.  The host
    build is reached only by asking for it (sim_device="cpu"), and reports itself as such."""
    import torch

    import ouzelum_amd as o
    from ouzelum_amd._lib import OuzelumError
    if not torch.cuda.is_available():
        with pytest.raises(OuzelumError):
            o.make(seed=0, task="LeeLanded", num_envs=64, sim_device="cuda:0", rl_device="cuda:0")
    env = o.make(seed=0, task="LeeLanded", num_envs=64, sim_device="cpu", rl_device="cpu")
    assert env._host and env.fstate.device.type == "cpu"
    with pytest.raises(ValueError):
        o.make(seed=0, task="LeeLanded", num_envs=64, sim_device="meta")


def test_state_slots_and_class_layout_map(L):
    """ouz_state_slots / ouz_env_slots (host-side, no GPU): the estimator tasks and the mixed curriculum up to
    64 K envs use the trigger-class layout (blocks of 21 waves, one PV trigger class g % 21 per wave; the
    mixed curriculum's slot space chunk-aligned in global ids, one 1344-id task chunk per 21 waves), every
    other task and size slot i = env i.  The env -> slot map is checked against the kernels' slot -> env
    formulas restated here."""
    import numpy as np
    from ouzelum_amd.vec_task import env_slots
    est = (L.TASK_EKF_LEE_LANDED, L.TASK_TRACKING)
    for task in range(L.NUM_TASKS):
        for n in (1, 63, 64, 4096, 8192, 65536, 65537, 4194304):
            if task in est and n <= 65536:
                want = ((n + 1343) // 1344) * 1344
            elif task == L.TASK_MIXED and n <= 65536:
                want = ((n + 1343) // 1344 + 1) * 1344
            else:
                want = n
            assert L.lib.ouz_state_slots(task, n) == want, (task, n)
    assert L.lib.ouz_state_slots(99, 64) < 0 and L.lib.ouz_state_slots(0, 0) < 0
    assert L.MIXED_CHUNK == 1344
    for task in (L.TASK_TRACKING, L.TASK_MIXED, L.TASK_FAULT):
        for n, off in ((4096, 0), (456 // 2, 456 // 2), (4096, 4096), (8192, 4096), (1000, 77), (4096, 28672),
                       (65536, 1344 * 5 + 3), (70000, 64)):
            slot = env_slots(task, n, off)
            slots = L.lib.ouz_state_slots(task, n)
            assert len(set(slot.tolist())) == n and slot.min() >= 0 and slot.max() < slots, (task, n, off)
            env = np.full(slots + 63, -1)
            env[slot] = np.arange(n)
            s = np.arange(slots)
            if slots == n:
                np.testing.assert_array_equal(slot, np.arange(n))
                continue
            r = s % 1344
            perm = (r >> 6) + 21 * (r & 63)
            if task == L.TASK_MIXED:      # chunk-aligned in global ids
                c = off // 1344 + s // 1344
                gid = c * 1344 + np.where(c % 3 == 1, perm, r)
                e_of_s = gid - off
            else:                         # blocks of the shard's own env index
                e_of_s = (s // 1344) * 1344 + perm
            ok = env[:slots] >= 0
            np.testing.assert_array_equal(env[:slots][ok], e_of_s[ok])
            assert not np.any((e_of_s >= 0) & (e_of_s < n) & ~ok)     # every in-range id has its slot
            for w in range(slots // 64):
                e = env[w * 64:(w + 1) * 64]
                e = e[e >= 0]
                if len(e) == 0:
                    continue
                gid = off + e
                tasks = {int(x) for x in (gid // 1344) % 3} if task == L.TASK_MIXED else {1}
                assert len(tasks) == 1                                  # one chunk task per wave
                if task == L.TASK_TRACKING or tasks == {1}:
                    cls = (gid if task == L.TASK_MIXED else e + off) % 21
                    assert len({int(x) for x in cls}) == 1              # one trigger class per wave
                else:
                    assert np.all(np.diff(e) == 1)                      # identity chunks: consecutive envs
    bad = np.empty(4, dtype=np.int32)
    assert L.lib.ouz_env_slots(L.TASK_MIXED, 4, -1, bad.ctypes.data) < 0



def test_shipped_library_is_not_instrumented(L):
    """The product library carries no instrumentation: ouz_build_flags() is 0, the
    wrong-result probe paths of earlier rounds are gone from the kernel source, and the shim refuses an
    instrumented build (a timing-stamp or store-policy A/B library) unless OUZ_ALLOW_INSTRUMENTED=1."""
    assert L.lib.ouz_build_flags() == 0
    src = open(os.path.join(ROOT, "ouzelum_amd", "csrc", "quad_kernels.hip")).read()
    for gone in ("OUZ_PROBE_SKIP", "OUZ_PROBE_UNIFORM_TRIGGER", "OUZ_PROBE_EMIT", "OUZ_PROBE_NOCORE",
                 "OUZ_PIPE_NOPREF"):
        assert gone not in src, gone
    shim = open(os.path.join(ROOT, "ouzelum_amd", "_lib.py")).read()
    assert "OUZ_ALLOW_INSTRUMENTED" in shim and "ouz_build_flags" in shim


def test_raw_function_is_the_same_entry_point_without_argtypes(L):
    """rollout_plan's unconverted call goes to the same code as the declared one (one mapped library), and
    taking it leaves the declared signature of ``L.lib`` untouched."""
    import ctypes
    raw = L.raw_function("ouz_rollout_stats")
    assert raw.argtypes is None and raw.restype is ctypes.c_int
    decl = L.lib.ouz_rollout_stats
    assert decl.argtypes is not None and len(decl.argtypes) == 11
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    assert addr(raw) == addr(decl)
    # a call with a null env is rejected by the library itself (no GPU involved)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    rc = raw(vp(None), vp(None), i32(1), i32(1), vp(None), vp(None), vp(None), vp(None), vp(None), i32(1), vp(None))
    assert rc != 0
