"""ouzelum_amd — MI355X-native vectorised quadrotor environment (x500 hover / tracking / faults).

The per-env step of the reference's drone tasks (sesem738/Ouzelum, an
IsaacGymEnvs fork) runs as one hand-written HIP kernel per step behind the C
ABI in ``include/ouzelum.h``; this package is the thin Python side of that
boundary: ``make()`` (isaacgymenvs.make signature) returning a VecTask-shaped
env whose tensors live on the GPU.

The HIP library is loaded on first use of the env API (so ``ouzelum_amd.build``
can rebuild it without loading a stale copy).
"""
import os as _os

__all__ = ["make", "QuadVecTask", "TASK_IDS", "POMDP_IDS", "task_info"]

# hipGraph replay: the ROCm runtime's graph packet-capture path (DEBUG_CLR_GRAPH_PACKET_CAPTURE, on by
# default) replays a captured graph with racy, run-to-run different results once it engages after the
# first few launches (a torch-only PPO-update graph drifts from its eager twin and from itself from the
# ~9th replay; with the knob off every replay is bitwise equal: DESIGN.md §9,
# scripts/exp/graph_update_repro.py).  The learners replay hipGraphs (learners/ppo.py GraphedPolicy), so
# importing this package sets the knob to 0 for the process (a process-wide side effect, stated here and in
# DESIGN.md §9) unless the caller chose a value.  The runtime reads it once, when it starts; whether that has
# already happened is decided from the process itself, not from torch's lazy-init flag
# (torch.cuda.is_available() / device_count() start the HIP runtime but leave torch.cuda.is_initialized()
# False): a started ROCm runtime holds /dev/kfd open.  GRAPH_REPLAY_SAFE is True only if the knob is 0 and
# was either in the process's initial environment or set before the runtime started; otherwise the
# graphed policy runs eagerly (with a warning).
def _hip_runtime_started() -> bool:
    try:
        fds = _os.listdir("/proc/self/fd")
    except OSError:  # pragma: no cover - not Linux: assume the worst
        return True
    for fd in fds:
        try:
            if _os.readlink(f"/proc/self/fd/{fd}").startswith("/dev/kfd"):
                return True
        except OSError:
            continue
    return False


def _initial_env(name: str):
    """Value of ``name`` in the environment the process was started with (None if absent)."""
    try:
        with open("/proc/self/environ", "rb") as f:
            for kv in f.read().split(b"\0"):
                k, _, v = kv.partition(b"=")
                if k == name.encode():
                    return v.decode(errors="replace")
    except OSError:  # pragma: no cover
        pass
    return None


_hip_started = _hip_runtime_started()
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
GRAPH_REPLAY_SAFE = _os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] == "0" and (
    _initial_env("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0" or not _hip_started)

def __getattr__(name):
    if name in __all__:
        from . import vec_task
        return getattr(vec_task, name)
    raise AttributeError(name)
