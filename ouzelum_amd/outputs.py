"""The reference's on-disk outputs, fed from device-side counters.

* Trajectory CSV (``ekf_lee_landed.py:132-135,667-674``; ``landed.py:346-353``): every
  step, env 0's position and target (EKF tasks also its linear velocity) are appended
  to ``trajectories/<pomdp>_<prob>_ep_<epi>.csv``, where ``epi`` is the cumulative number
  of env resets; a new file starts whenever ``epi`` changes, created with the header
  ``Position X, Position Y, Position Z``.  The reference does a D2H copy every step; here
  the step kernel writes the row and the per-step reset count into a device ring
  (``ouz_set_trace``) and ``flush()`` writes whole blocks of steps.
* Metrics (``ekf_lee_landed.py:315-331``): ``metrics/<pomdp>_<prob>_ep_count.txt`` holds
  ``epi`` and ``metrics/<pomdp>_<prob>.txt`` the total landings ("Landoa").
* Env-state checkpoint: ``save_env_state`` / ``load_env_state`` (tensors only, loaded with
  ``weights_only=True``) for deterministic resume — the counter RNG is keyed by the step.
"""
import csv
import os

import numpy as np
import torch

from .vec_task import POMDP_IDS

_POMDP_NAMES = {v: k for k, v in POMDP_IDS.items() if k}


def run_tag(env):
    """'<pomdp>_<prob>' of the env's task (the reference's POMDPWrapper.pomdp / .prob)."""
    from .vec_task import task_info
    info = task_info(env.task)
    mode = env.cfg.pomdp if env.cfg.pomdp >= 0 else info.pomdp
    prob = env.cfg.pomdp_prob if env.cfg.pomdp_prob >= 0 else info.pomdp_prob
    return f"{_POMDP_NAMES.get(mode, 'none')}_{float(np.float32(prob)):g}"


class TrajectoryLogger:
    def __init__(self, env, traj_dir="trajectories", metrics_dir="metrics", env_index=0, capacity=4096,
                 with_velocity=None, tag=None):
        self.env = env
        self.traj_dir, self.metrics_dir = traj_dir, metrics_dir
        self.tag = tag or run_tag(env)
        # EKFLeeLanded logs (pos, target, linvel) (ekf_lee_landed.py:671); Landed/LeeLanded (pos, target)
        self.with_velocity = (env.task_name in ("EKFLeeLanded", "QuadTracking")) if with_velocity is None \
            else with_velocity
        self.epi = 0
        self.next_step = env.sim_step_count
        self._opened = set()
        os.makedirs(traj_dir, exist_ok=True)
        os.makedirs(metrics_dir, exist_ok=True)
        env.enable_trace(env_index, capacity)

    def _path(self, epi):
        return os.path.join(self.traj_dir, f"{self.tag}_ep_{epi}.csv")

    def flush(self):
        """Write the rows of every step since the last flush; returns the number of rows."""
        steps, rows, resets = self.env.trace_since(self.next_step)
        if len(steps) == 0:
            return 0
        epis = self.epi + np.cumsum(resets)
        ncol = 9 if self.with_velocity else 6
        for epi in np.unique(epis):
            sel = rows[epis == epi, :ncol]
            path = self._path(int(epi))
            new = path not in self._opened and not os.path.exists(path)
            with open(path, "a", newline="") as fh:
                w = csv.writer(fh)
                if new:
                    w.writerow(["Position X", "Position Y", "Position Z"])   # ekf_lee_landed.py:135
                w.writerows(sel.tolist())
            self._opened.add(path)
        self.epi = int(epis[-1])
        self.next_step = int(steps[-1]) + 1
        self.write_metrics()
        return len(steps)

    def write_metrics(self):
        with open(os.path.join(self.metrics_dir, f"{self.tag}_ep_count.txt"), "w") as fh:
            fh.write(str(self.epi))
        with open(os.path.join(self.metrics_dir, f"{self.tag}.txt"), "w") as fh:
            fh.write(str(self.env.landings()))


def save_env_state(env, path):
    torch.save({k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in env.state_dict().items()}, path)


def load_env_state(env, path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    env.load_state_dict({k: (v.to(env.device) if isinstance(v, torch.Tensor) else v) for k, v in sd.items()})
