"""gym-free equivalents of the learners' env glue (``gym`` is not installed here).

* ``ExtractObsWrapper``         PPO/utils.py:37-39, RPO-LSTM/utils.py:36-38
* ``RecordEpisodeStatisticsTorch`` RPO-LSTM/utils.py:4-34 (same info["r"] / info["l"])
* ``POMDPWrapper``              utils/POMDP.py:5-43, evaluated by the HIP kernel
  ``ouz_pomdp_obs`` (one launch, device counter-RNG) instead of a CPU coin / CPU noise
  tensor copied to ``cuda:0`` on every call.
"""
import torch

from .. import _lib as L


class _Wrapper:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):          # forward everything else (num_envs, spaces, ...)
        return getattr(self.env, name)

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, action):
        return self.env.step(action)


class ExtractObsWrapper(_Wrapper):
    """obs dict -> the "obs" tensor."""

    def reset(self, **kw):
        return self.env.reset(**kw)["obs"]

    def step(self, action):
        obs, rew, done, info = self.env.step(action)
        return obs["obs"], rew, done, info


class RecordEpisodeStatisticsTorch(_Wrapper):
    """Running episodic return / length per env on the device; info["r"], info["l"] hold the
    values at the current step (before the done envs are zeroed)."""

    def __init__(self, env, device):
        super().__init__(env)
        self.num_envs = getattr(env, "num_envs", 1)
        self.device = device

    def reset(self, **kw):
        obs = self.env.reset(**kw)
        n, d = self.num_envs, self.device
        self.episode_returns = torch.zeros(n, dtype=torch.float32, device=d)
        self.episode_lengths = torch.zeros(n, dtype=torch.int32, device=d)
        self.returned_episode_returns = torch.zeros(n, dtype=torch.float32, device=d)
        self.returned_episode_lengths = torch.zeros(n, dtype=torch.int32, device=d)
        return obs

    def step(self, action):
        obs, rew, done, info = self.env.step(action)
        self.episode_returns += rew
        self.episode_lengths += 1
        self.returned_episode_returns.copy_(self.episode_returns)
        self.returned_episode_lengths.copy_(self.episode_lengths)
        self.episode_returns *= 1 - done
        self.episode_lengths *= 1 - done
        info["r"] = self.returned_episode_returns
        info["l"] = self.returned_episode_lengths
        return obs, rew, done, info


POMDP_MODES = {"none": L.POMDP_NONE, "flicker": L.POMDP_FLICKER, "random_noise": L.POMDP_NOISE,
               "flickering_and_random_noise": L.POMDP_FLICKER_NOISE}


class POMDPWrapper:
    """Learner-side observation corruption (utils/POMDP.py).  ``observation(obs)`` returns a new
    (N, d) tensor; draws are keyed (seed, row_offset + row, call index), so a sharded run
    reproduces the unsharded one."""

    def __init__(self, pomdp="flicker", pomdp_prob=0.1, seed=0, row_offset=0):
        if pomdp not in POMDP_MODES:
            raise ValueError(f"pomdp was not in {sorted(POMDP_MODES)}!")   # POMDP.py:20
        self.pomdp = pomdp
        self.mode = POMDP_MODES[pomdp]
        self.prob = float(pomdp_prob)
        self.seed = int(seed)
        self.row_offset = int(row_offset)
        self.calls = 0

    def observation(self, obs, out=None):
        L.require_hip_tensor(obs, "obs")
        if obs.dtype != torch.float32 or obs.dim() != 2:
            raise ValueError("obs must be a (N, d) float32 tensor")
        out = torch.empty_like(obs) if out is None else out
        L.check(L.lib.ouz_pomdp_obs(L.ptr(obs), L.ptr(out), obs.shape[0], obs.shape[1], self.mode, self.prob,
                                    self.seed, self.row_offset, self.calls & 0xFFFFFFFF, L.stream_ptr(obs.device)),
                "ouz_pomdp_obs")
        self.calls += 1
        return out
