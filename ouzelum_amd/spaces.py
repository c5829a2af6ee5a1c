"""Minimal ``gym.spaces.Box`` stand-in (``gym`` is not installed here or on the GPU box).

Mirrors what the reference's VecTask builds (tasks/base/vec_task.py:102-105)
and what its learners read (``.shape``, ``.low``, ``.high``, ``.dtype``;
PPO/agent.py, RPO-LSTM/model.py).  If the real ``gym`` is importable its Box
is used instead, so ``isinstance(space, gym.spaces.Box)`` checks
(PPO/main.py:58) keep passing.
"""
import numpy as np

try:  # pragma: no cover - gym absent in this image
    from gym.spaces import Box  # type: ignore
except Exception:  # noqa: BLE001
    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            low = np.asarray(low, dtype=dtype)
            high = np.asarray(high, dtype=dtype)
            if shape is not None:
                low = np.broadcast_to(low, shape).copy()
                high = np.broadcast_to(high, shape).copy()
            self.low, self.high = low, high
            self.shape = tuple(low.shape)
            self.dtype = np.dtype(dtype)

        def sample(self, rng=None):
            rng = rng or np.random
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
