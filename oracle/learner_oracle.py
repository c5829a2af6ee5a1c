"""CPU restatement of the learner-side kernels (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module.  Pinned by tests/golden/learner.npz, which the
reference's own ``RPO-LSTM/agent.py::PPO.getGAE`` produced (tests/golden/make_golden.py).
"""
import numpy as np

from . import quad_oracle as Q

SITE_LEARNER = 6   # csrc/philox.h PomdpSite


def gae_f32(rewards, values, dones, next_value, next_done, gamma=0.99, lam=0.95):
    """RPO-LSTM/agent.py:40-55 in float32 with torch's operation order:
    delta = (r + (gamma * nv) * nnt) - v;  adv = delta + ((gamma*lam) * nnt) * last."""
    f = np.float32
    r, v, d = (np.asarray(x, f) for x in (rewards, values, dones))
    T, N = r.shape
    g, gl = f(gamma), f(gamma * lam)      # gamma*lam: one Python (double) product, then f32
    adv = np.zeros((T, N), f)
    last = np.zeros(N, f)
    for t in reversed(range(T)):
        if t == T - 1:
            nnt = f(1.0) - np.asarray(next_done, f)
            nv = np.asarray(next_value, f)
        else:
            nnt = f(1.0) - d[t + 1]
            nv = v[t + 1]
        delta = (r[t] + (g * nv) * nnt) - v[t]
        last = delta + (gl * nnt) * last
        adv[t] = last
    return adv + v, adv


def pomdp_obs(x, mode, prob, seed, row_offset, call):
    """utils/POMDP.py:23-43 as evaluated by ``ouz_pomdp_obs`` (prob passes through float32)."""
    x = np.asarray(x, np.float32)
    rows = np.arange(x.shape[0], dtype=np.uint64) + np.uint64(row_offset)
    out = Q.pomdp_apply(x.astype(np.float64), mode, float(np.float32(prob)), seed, rows.astype(np.uint32), call,
                        SITE_LEARNER, batch_tag=0)
    return np.asarray(out, np.float32)
