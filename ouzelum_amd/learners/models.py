"""Policy / value networks of the reference learners, re-laid for MI355X.

Same architectures and parameter names as ``RPO-LSTM/model.py:11-84`` and
``PPO/model.py:11-55`` (so the reference's ``*_actor`` / ``*_critic`` state dicts
load unchanged), with the recurrent actor restructured for the GPU:

* ``LSTMActor.get_states`` (reference ``model.py:34-50``) calls ``nn.LSTM`` once
  per time step because the done mask resets the carry between steps.  Here the
  input projection ``x W_ihᵀ + b_ih + b_hh`` of all T steps is one GEMM over
  (T·B, 256) — hipBLASLt at a useful size — and on the GPU each step is one
  (B,128)x(128,512) recurrent GEMM plus ONE fused HIP cell kernel, with a matching
  fused BPTT (``fused.LSTMSequence``).  Gate order and arithmetic are torch's LSTM
  cell (i, f, g, o); on CPU tensors the same math runs as torch ops.
* Large-row linear layers take a split-K weight gradient (``fused.SplitKLinear``).
* RPO's policy-update noise ``z ~ U(-alpha, alpha)`` (``model.py:61-64``) is drawn
  on the actor's device instead of a CPU ``FloatTensor`` copied to ``cuda:0``.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn
from torch.distributions.normal import Normal

from .fused import (LSTMSequence, SplitKLinear, linear, lstm_sequence_carry_inplace, policy_sample, policy_sample_ok,
                    run_mlp)

L_NUM_ACT = 4   # the action width ouz_policy_sample computes (OUZ_NUM_ACT)


def layer_init(layer, std=math.sqrt(2), bias_const=0.0):
    """Orthogonal weights, constant bias (model.py:6-9)."""
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


def _flat(space):
    return int(np.prod(space.shape))


class MLPActor(nn.Module):
    """PPO actor: 13 -> 256 -> 256 -> 4 tanh MLP mean + state-independent log-std (PPO/model.py:11-40)."""

    def __init__(self, observation_space, action_space, rpo_alpha=0.0):
        super().__init__()
        self.rpo_alpha = rpo_alpha
        n_obs, n_act = _flat(observation_space), _flat(action_space)
        self.actor_mean = nn.Sequential(
            layer_init(nn.Linear(n_obs, 256)), nn.Tanh(),
            layer_init(nn.Linear(256, 256)), nn.Tanh(),
            layer_init(nn.Linear(256, n_act), std=0.01),
        )
        self.actor_logstd = nn.Parameter(torch.zeros(1, n_act))

    def forward(self, state, action=None, eps=None):
        head = self.actor_mean[-1]
        if action is None and _SAMPLE_FORM == "direct":
            hidden = run_mlp(self.actor_mean[:-1], state)
            if policy_sample_ok(hidden, head):
                e = torch.randn((hidden.shape[0], L_NUM_ACT), device=hidden.device) if eps is None else eps
                return policy_sample(hidden, head, self.actor_logstd, e)
            return _policy_head(torch.nn.functional.linear(hidden, head.weight, head.bias), self.actor_logstd,
                                action, self.rpo_alpha, eps)
        mean = run_mlp(self.actor_mean, state)
        return _policy_head(mean, self.actor_logstd, action, self.rpo_alpha, eps)

    def update_mean(self, state):
        """The mean the policy update scores its actions under (RPO's noise added), for ``fused.PolicyLoss``."""
        return _rpo_mean(run_mlp(self.actor_mean, state), self.rpo_alpha)


class LSTMActor(nn.Module):
    """RPO-LSTM actor (RPO-LSTM/model.py:11-70): 13 -> 512 -> 256 tanh trunk, LSTM(256, 128),
    linear mean head, state-independent log-std, RPO alpha 0.5."""

    def __init__(self, observation_space, action_space, rpo_alpha=0.5, hidden=128):
        super().__init__()
        self.rpo_alpha = rpo_alpha
        n_obs, n_act = _flat(observation_space), _flat(action_space)
        self.network = nn.Sequential(
            layer_init(nn.Linear(n_obs, 512)), nn.Tanh(),
            layer_init(nn.Linear(512, 256)), nn.Tanh(),
        )
        self.lstm = nn.LSTM(256, hidden)
        for name, param in self.lstm.named_parameters():
            if "bias" in name:
                nn.init.constant_(param, 0)
            elif "weight" in name:
                nn.init.orthogonal_(param, 1.0)
        self.actor_mean = layer_init(nn.Linear(hidden, n_act), std=0.01)
        self.actor_logstd = nn.Parameter(torch.zeros(1, n_act))
        # (h, c) buffers of shape (1, B, H) that inference calls write their final carry into (GraphedPolicy)
        self.carry_inplace = None

    def initial_state(self, num_envs, device):
        shape = (self.lstm.num_layers, num_envs, self.lstm.hidden_size)
        return torch.zeros(shape, device=device), torch.zeros(shape, device=device)

    def get_states(self, state, lstm_state, done):
        """(T·B, obs) trunk features -> (T·B, H) LSTM outputs; the carry of env b is zeroed
        before step t when done[t, b] (model.py:34-50).  Returns (hidden, (h, c))."""
        feats = run_mlp(self.network, state)
        h, c = lstm_state
        B = h.shape[1]
        H = self.lstm.hidden_size
        bias = self.lstm.bias_ih_l0 + self.lstm.bias_hh_l0
        if feats.is_cuda:
            # HIP path: split-K input projection + fused cell kernels (fused.py)
            x_proj = (SplitKLinear.apply(feats, self.lstm.weight_ih_l0, bias) if torch.is_grad_enabled()
                      else torch.addmm(bias, feats, self.lstm.weight_ih_l0.t()))
            keep = (1.0 - done).float().view(-1, B)
            if self.carry_inplace is not None and not torch.is_grad_enabled():
                # GraphedPolicy's static carry: the final (h, c) overwrite these buffers (no copies per step)
                ho, co = self.carry_inplace
                hid = lstm_sequence_carry_inplace(x_proj.view(-1, B, 4 * H), h[0], c[0], keep,
                                                  self.lstm.weight_hh_l0, ho[0], co[0])
                return hid.view(-1, H), (ho, co)
            hid, hT, cT = LSTMSequence.apply(x_proj.view(-1, B, 4 * H), h[0], c[0], keep, self.lstm.weight_hh_l0)
            return hid.view(-1, H), (hT.unsqueeze(0), cT.unsqueeze(0))
        x_proj = torch.addmm(bias, feats, self.lstm.weight_ih_l0.t())
        x_proj = x_proj.view(-1, B, 4 * H)
        keep = (1.0 - done).view(-1, B, 1)
        h, c = h[0], c[0]
        w_hh_t = self.lstm.weight_hh_l0.t()
        outs = []
        for t in range(x_proj.shape[0]):
            h = keep[t] * h
            c = keep[t] * c
            gates = torch.addmm(x_proj[t], h, w_hh_t)
            i, f, g, o = gates.chunk(4, dim=1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            h = torch.sigmoid(o) * torch.tanh(c)
            outs.append(h)
        return torch.cat(outs, 0), (h.unsqueeze(0), c.unsqueeze(0))

    def forward(self, state, lstm_state, done, action=None, eps=None):
        hidden, lstm_state = self.get_states(state, lstm_state, done)
        if action is None and _SAMPLE_FORM == "direct" and policy_sample_ok(hidden, self.actor_mean):
            e = torch.randn((hidden.shape[0], L_NUM_ACT), device=hidden.device) if eps is None else eps
            return (*policy_sample(hidden, self.actor_mean, self.actor_logstd, e), lstm_state)
        mean = linear(hidden, self.actor_mean)
        return (*_policy_head(mean, self.actor_logstd, action, self.rpo_alpha, eps), lstm_state)

    def update_mean(self, state, lstm_state, done):
        """The mean the policy update scores its actions under (RPO's noise added, model.py:61-64), for
        ``fused.PolicyLoss``."""
        hidden, _ = self.get_states(state, lstm_state, done)
        # 128 -> 4 over T·B rows: the split-K weight gradient (a plain GEMM puts its 4 x 128 output on one tile)
        return _rpo_mean(linear(hidden, self.actor_mean), self.rpo_alpha)


def _rpo_mean(mean, rpo_alpha):
    # the same draw, in the same order, as _policy_head's
    if rpo_alpha > 0.0:
        mean = mean + torch.empty_like(mean).uniform_(-rpo_alpha, rpo_alpha)
    return mean


def _policy_head(mean, logstd, action, rpo_alpha, eps=None):
    # validate_args=False: the default argument check is a device->host sync on every call (and
    # cannot be captured in a hipGraph); mean / std are finite by construction.  The sample is
    # mean + std * eps, eps ~ N(0, 1) (given by the caller, or drawn here): Normal.sample() calls
    # torch.normal(mean_tensor, std_tensor), whose std >= 0 check is a std.min().item() device->host
    # sync on every call, and which cannot be captured in a hipGraph
    if action is None:
        if _SAMPLE_FORM == "normal":
            std = torch.exp(logstd.expand_as(mean))
            probs = Normal(mean, std, validate_args=False)
            action = mean + std * (torch.randn_like(mean) if eps is None else eps)
            return action, probs.log_prob(action).sum(1), probs.entropy().sum(1)
        return _sample_head(mean, logstd, torch.randn_like(mean) if eps is None else eps)
    std = torch.exp(logstd.expand_as(mean))
    mean = _rpo_mean(mean, rpo_alpha)   # RPO: perturb the mean for the policy update (RPO-LSTM/model.py:61-64)
    probs = Normal(mean, std, validate_args=False)
    return action, probs.log_prob(action).sum(1), probs.entropy().sum(1)


_LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
_SAMPLE_FORM = os.environ.get("OUZ_SAMPLE_FORM", "direct")


def _sample_head(mean, logstd, eps):
    """The rollout's sample, its log-prob and entropy with the per-dimension terms on the (1, A) log-std
    instead of (B, A) tensors: action = mean + σ ε, log N(action; mean, σ) summed over A = -½ Σ ε² - Σ log σ - A
    log √(2π) (since (action - mean) / σ = ε), entropy = Σ log σ + A (½ + log √(2π)), the same for every row.
    Four (B, ·) launches instead of Normal's ~17 (each a few µs inside the rollout's graph); equal to the Normal
    form within f32 rounding (``test_graphed_policy_matches_eager`` checks the log-prob against it)."""
    A = mean.shape[1]
    action = torch.addcmul(mean, torch.exp(logstd), eps)
    const = logstd.sum() + A * _LOG_SQRT_2PI
    logprob = torch.add(-const, eps.square().sum(1), alpha=-0.5)
    entropy = (const + 0.5 * A).expand(mean.shape[0])
    return action, logprob, entropy


class Critic(nn.Module):
    """Value MLP 13 -> 256 -> 256 -> 1 (RPO-LSTM/model.py:72-84)."""

    def __init__(self, observation_space):
        super().__init__()
        self.critic = nn.Sequential(
            layer_init(nn.Linear(_flat(observation_space), 256)), nn.Tanh(),
            layer_init(nn.Linear(256, 256)), nn.Tanh(),
            layer_init(nn.Linear(256, 1), std=1.0),
        )

    def forward(self, state):
        return run_mlp(self.critic, state)
