"""ouzelum_amd — MI355X-native vectorised quadrotor environment (x500 hover / tracking / faults).

The per-env step of the reference's drone tasks (sesem738/Ouzelum, an
IsaacGymEnvs fork) runs as one hand-written HIP kernel per step behind the C
ABI in ``include/ouzelum.h``; this package is the thin Python side of that
boundary: ``make()`` (isaacgymenvs.make signature) returning a VecTask-shaped
env whose tensors live on the GPU.
"""
from .vec_task import POMDP_IDS, TASK_IDS, QuadVecTask, make, task_info  # noqa: F401

__all__ = ["make", "QuadVecTask", "TASK_IDS", "POMDP_IDS", "task_info"]
