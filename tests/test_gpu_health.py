"""Failure reporting of the fused rollouts and bench.py's own N-rank launcher, on the GPU.

* A split-wave / output-wave LDS wait that gives up (quad_pv_split.h) lets the launch drain with wrong results;
  that must never be silent: ``QuadVecTask.check_health`` (called by ``rollout(check=True)``, ``state_dict``,
  ``landings``, ``trace_since``, ``episode_stats(check=True)``) raises.  The spin limit is lowered through the
  test-only ``ouz_set_split_spin_limit`` to force give-ups, then restored.
* ``bench.py --gpus 2`` without torchrun starts its two ranks itself (here rehearsed over gloo, two ranks on
  the box's one GPU) and prints one line for the whole job.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(task, n):
    from ouzelum_amd import QuadVecTask
    return QuadVecTask(task=task, num_envs=n, sim_device="cuda:0", seed=3, track_episodes=True)


def _storage(n, k=16):
    dev = torch.device("cuda", 0)
    return (torch.empty((k, n, 13), device=dev), torch.empty((k, n), device=dev),
            torch.empty((k, n), dtype=torch.int64, device=dev), torch.empty((k, n), dtype=torch.bool, device=dev))


@pytest.mark.parametrize("task", ["QuadTracking", "LeeLanded"])
def test_split_wave_give_up_raises(task):
    """QuadTracking at 4096 envs runs the split-wave + output-wave rollout, LeeLanded the output-wave one: with a
    one-poll spin limit their waits give up, and the env raises instead of handing on the rollout."""
    from ouzelum_amd import _lib as L
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    env = _env(task, 4096)
    st = _storage(4096)
    stats = torch.zeros(3, dtype=torch.float64, device="cuda:0")
    env.rollout(None, 16, fused=True, storage=st, stats_out=stats, check=True)   # healthy: no raise
    try:
        L.check(L.lib.ouz_set_split_spin_limit(1), "ouz_set_split_spin_limit")
        with pytest.raises(L.OuzelumError, match="gave up"):
            for _ in range(8):
                env.rollout(None, 16, fused=True, storage=st, stats_out=stats, check=True)
    finally:
        L.check(L.lib.ouz_set_split_spin_limit(0), "ouz_set_split_spin_limit")
    env.check_health()                       # the raising check reset the counter
    env.rollout(None, 16, fused=True, storage=st, stats_out=stats, check=True)
    sd = env.state_dict()                    # a checkpoint checks too (healthy here)
    assert sd["layout"]["abi"] == L.LAYOUT_VERSION


def test_bench_spawns_its_ranks():
    """``bench.py --gpus 2`` with no torchrun: two ranks (gloo rehearsal on one GPU), one line, n_gpus 2."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    env = dict(os.environ, OUZ_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "5", "--no-configs", "--no-sweep", "--no-cpu-baseline",
                        "--detail", os.path.join(ROOT, "gpurun_out", "bench_detail_spawn_test.json")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 8192 and d["config"]["ranks_joined"] == 2
    assert d["config"]["launcher"] == "bench.py" and d["config"]["backend"] == "gloo"
    assert d["split_timeouts"] == 0 and d["value"] > 0
