"""Probe: where the large-N estimator fused rollout (WPE = 2) and single VecTask.step launches part (the failing
segment of tests/test_gpu_timed_kernels.py).  Per segment: envs whose obs differ beyond the fused test's tolerance,
the step they first differ, and their distances from the guidance / landing / done thresholds on the single-step
side at that step.  Prints JSON lines."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ouzelum_amd as ouz  # noqa: E402
from ouzelum_amd import _lib as L  # noqa: E402


def main(task="QuadTracking", n=70016 + 37):
    kw = dict(seed=19, task=task, num_envs=n, sim_device="cuda:0", track_episodes=True, convergence_time=10,
              max_episode_length=30)
    a, b = ouz.make(**kw), ouz.make(**kw)
    g = torch.Generator(device="cuda").manual_seed(14)
    ring = (torch.rand((16, n, 4), device="cuda", generator=g) * 2 - 1).contiguous()
    for seg, (k_steps, drain) in enumerate(((16, True), (40, False), (1, True), (16, True))):
        b.load_state_dict(a.state_dict())
        st = (torch.empty((k_steps, n, 13), device="cuda"), torch.empty((k_steps, n), device="cuda"),
              torch.empty((k_steps, n), dtype=torch.int64, device="cuda"),
              torch.empty((k_steps, n), dtype=torch.bool, device="cuda"))
        got = torch.zeros(3, dtype=torch.float64, device="cuda")
        a.rollout(ring, k_steps, fused=True, storage=st, stats_out=got, drain=drain)
        obs, td, wd, rst = [], [], [], []
        for k in range(k_steps):
            p = b.root_states[:, :3]
            tgt = b.target_root_positions
            wp = b.frows(L.F_WAYPOINT, L.F_WAYPOINT + 3).t()
            td.append((tgt - p).norm(dim=1))
            wd.append((wp - p).norm(dim=1))
            b.step(ring[k % 16])
            obs.append(b.obs_buf.clone())
            rst.append(b.reset_buf.clone())
        obs = torch.stack(obs)
        td, wd = torch.stack(td), torch.stack(wd)
        err = (st[0] - obs).abs() - (2e-5 + 1e-5 * obs.abs())
        bad_step = (err > 0).any(dim=2)              # (K, n)
        bad = bad_step.any(dim=0)
        nb = int(bad.sum())
        rec = {"task": task, "seg": seg, "k": k_steps, "bad_envs": nb,
               "max_obs_err": float((st[0] - obs).abs().max()),
               "reset_mismatch": int((st[2] != torch.stack(rst)).any(dim=0).sum())}
        if nb:
            first = torch.where(bad_step.any(dim=1))[0]
            rec["first_bad_step_hist"] = torch.bincount(bad_step.float().argmax(dim=0)[bad], minlength=k_steps).tolist()
            envs = torch.where(bad)[0][:8].tolist()
            det = []
            for e in envs:
                k0 = int(bad_step[:, e].float().argmax())
                m_td = torch.minimum((td[:k0 + 1, e] - 0.25).abs(), (td[:k0 + 1, e] - 0.75).abs()).min()
                m_wd = torch.minimum((wd[:k0 + 1, e] - 0.5).abs(), (wd[:k0 + 1, e] - 1.0).abs()).min()
                det.append({"env": e, "first_bad": k0, "err": float((st[0][k0, e] - obs[k0, e]).abs().max()),
                            "comp": int((st[0][k0, e] - obs[k0, e]).abs().argmax()),
                            "min_td_margin": float(m_td), "min_wd_margin": float(m_wd),
                            "fused_obs": st[0][k0, e].tolist(), "step_obs": obs[k0, e].tolist()})
            rec["examples"] = det
            rec["first_bad_global"] = int(first[0])
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["QuadTracking"]))
