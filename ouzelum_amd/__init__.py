"""ouzelum_amd — MI355X-native vectorised quadrotor environment (x500 hover / tracking / faults).

The per-env step of the reference's drone tasks (sesem738/Ouzelum, an
IsaacGymEnvs fork) runs as one hand-written HIP kernel per step behind the C
ABI in ``include/ouzelum.h``; this package is the thin Python side of that
boundary: ``make()`` (isaacgymenvs.make signature) returning a VecTask-shaped
env whose tensors live on the GPU.

The HIP library is loaded on first use of the env API (so ``ouzelum_amd.build``
can rebuild it without loading a stale copy).
"""
__all__ = ["make", "QuadVecTask", "TASK_IDS", "POMDP_IDS", "task_info"]


def __getattr__(name):
    if name in __all__:
        from . import vec_task
        return getattr(vec_task, name)
    raise AttributeError(name)
