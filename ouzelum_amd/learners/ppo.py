"""PPO / RPO-LSTM update on MI355X with the rollout size as a parameter.

Mirrors ``RPO-LSTM/agent.py:9-147`` (recurrent, env-wise minibatches, RPO noise) and
``PPO/agent.py`` (feed-forward, sample-wise minibatches): same hyper-parameters
(clip 0.2, gamma 0.99, lambda 0.95, 4 epochs, 2 minibatches, vf_coef 2, grad-norm 1,
Adam lr 2.6e-3 eps 1e-5, advantage normalisation) and the same checkpoint files.
Differences, all MI355X-side:

* N and T are parameters: the reference hard-codes ``values.reshape(16, 4096)``
  (``agent.py:61``), so any other env count crashes there.
* GAE is one HIP launch (``ouz_gae``) instead of a T-step Python loop; values are
  computed without building an autograd graph (the reference's graph there is
  never used: ``clip_vloss`` is False).
* Minibatch permutations come from device RNG (no H2D copy of a numpy permutation) and the clip fractions stay on the device until the end of
  the update (the reference syncs with ``.item()`` every minibatch).
* The minibatch losses run as HIP kernels on the GPU (``fused.PolicyLoss`` / ``ValueLoss``: forward and input
  gradients in a handful of launches instead of ~60) whenever they are exactly the loss asked for (ent_coef 0,
  no clipped value loss; ``OUZ_FUSED_LOSS=0`` keeps the torch form).
* Under torchrun (one process per GPU, env ids sharded) the learner is data
  parallel: rank 0's initial weights are broadcast and every optimizer step
  all-reduces one flattened gradient bucket over RCCL.  The reference learners are
  single-GPU.
"""
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import _lib as L
from .fused import ClipAdam, PolicyLoss, ValueLoss
from .gemm_tuning import enable_tuned_gemms
from .models import Critic, LSTMActor, MLPActor


def _graph_replay_safe():
    """hipGraph replay gives correct results only with the runtime's packet-capture path off (set by
    ``ouzelum_amd/__init__.py`` before the HIP runtime starts)."""
    import warnings
    from .. import GRAPH_REPLAY_SAFE
    if not GRAPH_REPLAY_SAFE and not getattr(_graph_replay_safe, "warned", False):
        warnings.warn("HIP runtime started with DEBUG_CLR_GRAPH_PACKET_CAPTURE on: the rollout policy runs eagerly "
                      "(import ouzelum_amd before initialising the GPU, or set the variable to 0)")
        _graph_replay_safe.warned = True
    return GRAPH_REPLAY_SAFE


def broadcast_params(module, src=0):
    """Same initial weights on every rank (one flattened broadcast)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    flat = torch.cat([p.data.reshape(-1) for p in module.parameters()])
    dist.broadcast(flat, src)
    off = 0
    for p in module.parameters():
        n = p.numel()
        p.data.copy_(flat[off:off + n].view_as(p))
        off += n


def allreduce_grads(module):
    """Data-parallel gradient mean over ranks: ONE all-reduce of the flattened gradients per
    optimizer step (the networks are < 1 M parameters, so a single bucket beats per-tensor calls
    on xGMI's per-link ring)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    params = [p for p in module.parameters() if p.grad is not None]
    flat = torch.cat([p.grad.reshape(-1) for p in params])
    dist.all_reduce(flat)
    flat /= dist.get_world_size()
    off = 0
    for p in params:
        n = p.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n


def gae(rewards, values, dones, next_value, next_done, gamma=0.99, lam=0.95):
    """(returns, advantages), each (T, N) f32, from the HIP kernel (RPO-LSTM/agent.py:40-55)."""
    T, N = rewards.shape
    ts = [t.contiguous().float() for t in (rewards, values, dones, next_value.reshape(N), next_done.reshape(N))]
    for t, name in zip(ts, ("rewards", "values", "dones", "next_value", "next_done")):
        L.require_hip_tensor(t, name)
    adv = torch.empty_like(ts[0])
    ret = torch.empty_like(ts[0])
    # the reference multiplies by the Python product gamma * lambda (a double), rounded once to f32
    L.check(L.lib.ouz_gae(*(L.ptr(t) for t in ts), T, N, gamma, float(gamma * lam), L.ptr(adv), L.ptr(ret),
                          L.stream_ptr(adv.device)), "ouz_gae")
    return ret, adv


class PPOLearner:
    def __init__(self, observation_space, action_space, num_envs, device, recurrent=True, rollout_steps=16,
                 lr=0.0026, num_minibatches=2, update_epochs=4, tuned_gemms=True):
        self.obs_dim = observation_space
        self.act_dim = action_space
        self.num_envs = num_envs
        self.rollout_steps = rollout_steps
        self.device = torch.device(device)
        self.recurrent = recurrent
        self.clip_coef = 0.2
        self.gamma = 0.99
        self.gae_lamda = 0.95
        self.norm_adv = True
        self.update_epochs = update_epochs
        self.ent_coef = 0.0
        self.vf_coef = 2
        self.clip_vloss = False
        self.target_kl = None
        self.max_grad_norm = 1
        self.num_minibatches = num_minibatches
        self.batch_size = num_envs * rollout_steps
        self.minibatch_size = self.batch_size // num_minibatches
        if recurrent and num_envs % num_minibatches:
            raise ValueError("num_envs must divide into the minibatches")   # agent.py:72
        if tuned_gemms:
            enable_tuned_gemms(self.device)   # per-shape GEMM solutions (gemm_tuning.py); OUZ_TUNABLEOP=0: off
        self.actor = (LSTMActor(observation_space, action_space) if recurrent
                      else MLPActor(observation_space, action_space)).to(self.device)
        self.critic = Critic(observation_space).to(self.device)
        broadcast_params(self.actor)
        broadcast_params(self.critic)
        # fused Adam on the GPU: one multi-tensor kernel per optimizer step instead of the foreach
        # form's handful per parameter group (the update is launch-bound)
        fused = self.device.type == "cuda" and os.environ.get("OUZ_ADAM_FUSED", "1") != "0"
        # gradient clipping + Adam as two HIP launches per optimizer step (fused.ClipAdam; the torch optimizer keeps
        # the state and the checkpoint format); OUZ_CLIP_ADAM=0 keeps clip_grad_norm_ + the torch step
        clip_adam = fused and os.environ.get("OUZ_CLIP_ADAM", "1") != "0"
        opt_kw = {"foreach": False} if clip_adam else {"fused": fused}
        self.actor_optimizer = torch.optim.Adam(self.actor.parameters(), lr=lr, eps=1e-5, **opt_kw)
        self.critic_optimizer = torch.optim.Adam(self.critic.parameters(), lr=lr, eps=1e-5, **opt_kw)
        self._clip_adam = ((ClipAdam(self.actor_optimizer), ClipAdam(self.critic_optimizer)) if clip_adam
                           else None)

    # ------------------------------------------------------------------ rollout
    @torch.no_grad()
    def get_action(self, state, lstm_state=None, done=None, eps=None):
        if self.recurrent:
            return self.actor(state, lstm_state, done, eps=eps)
        return (*self.actor(state, eps=eps), None)

    def initial_state(self):
        return self.actor.initial_state(self.num_envs, self.device) if self.recurrent else None

    def act(self, state, lstm_state=None, done=None, alias=False):
        """``get_action`` for one rollout step, replayed from a hipGraph on the GPU (``GraphedPolicy``)
        unless ``OUZ_GRAPH_POLICY=0``.  Returns fresh tensors; ``alias=True`` returns the graph's static
        output tensors instead, overwritten by the next call (the rollout loop copies them into its
        buffers at once and passes the LSTM carry straight back)."""
        if (self.device.type != "cuda" or os.environ.get("OUZ_GRAPH_POLICY", "1") == "0"
                or not _graph_replay_safe()):
            return self.get_action(state, lstm_state, done)
        if getattr(self, "_graphed", None) is None:
            self._graphed = GraphedPolicy(self)
        return self._graphed(state, lstm_state, done, alias=alias)

    @torch.no_grad()
    def get_gae(self, next_obs, next_done, rewards, dones, values):
        next_value = self.critic(next_obs).reshape(-1)
        return gae(rewards, values, dones, next_value, next_done, self.gamma, self.gae_lamda)

    # ------------------------------------------------------------------- update
    def _perm(self, n):
        """A uniform random permutation from device RNG (no host round trip)."""
        return torch.argsort(torch.rand(n, device=self.device))

    def train(self, obs, pomdps, actions, next_obs, next_done, initial_lstm_state, logprobs, rewards, dones):
        """One PPO update on a (T, N) rollout.  ``pomdps`` are the observations the actor trains on
        (RPO-LSTM trains on the POMDP-corrupted ones, agent.py:83); pass ``obs`` for plain PPO."""
        T, N = rewards.shape
        with torch.no_grad():
            values = self.critic(obs.reshape(T * N, -1)).reshape(T, N)
        returns, advantages = self.get_gae(next_obs, next_done, rewards, dones, values)
        b_obs = obs.reshape(T * N, -1)
        b_pomdps = pomdps.reshape(T * N, -1)
        b_actions = actions.reshape(T * N, -1)
        b_logprobs = logprobs.reshape(-1)
        b_dones = dones.reshape(-1)
        b_advantages = advantages.reshape(-1)
        b_returns = returns.reshape(-1)
        flatinds = torch.arange(T * N, device=self.device).reshape(T, N)
        # the minibatch's four per-row scalars as ONE gather of their stacked rows (each result row contiguous)
        # instead of four (OUZ_STACKED_GATHER=0: one per tensor); exact either way
        scalars = [b_logprobs, b_dones, b_advantages, b_returns]
        stacked = (torch.stack([x.float() for x in scalars]) if self.device.type == "cuda"
                   and os.environ.get("OUZ_STACKED_GATHER", "1") != "0" else None)
        clipfracs = torch.zeros((), device=self.device)
        n_mb = 0
        # the HIP loss kernels where they compute exactly the loss asked for: no entropy bonus (ent_coef 0, as both
        # reference learners) and no clipped value loss; OUZ_FUSED_LOSS=0 keeps the torch form
        fused_loss = (self.device.type == "cuda" and self.ent_coef == 0 and not self.clip_vloss
                      and os.environ.get("OUZ_FUSED_LOSS", "1") != "0")
        stats = {}
        for _ in range(self.update_epochs):
            if self.recurrent:
                envinds = self._perm(N)
                per = N // self.num_minibatches
                batches = [(flatinds[:, envinds[s:s + per]].reshape(-1), envinds[s:s + per])
                           for s in range(0, N, per)]
            else:
                b_inds = self._perm(T * N)
                batches = [(b_inds[s:s + self.minibatch_size], None) for s in range(0, T * N, self.minibatch_size)]
            for mb_inds, mbenvinds in batches:
                mb_state = ((initial_lstm_state[0][:, mbenvinds], initial_lstm_state[1][:, mbenvinds])
                            if self.recurrent else None)
                if stacked is not None:
                    mb_logp, mb_done, mb_advs, mb_ret = torch.index_select(stacked, 1, mb_inds).unbind(0)
                else:
                    mb_logp, mb_done, mb_advs, mb_ret = (x[mb_inds] for x in scalars)
                mb_pomdps, mb_obs = b_pomdps.index_select(0, mb_inds), b_obs.index_select(0, mb_inds)
                mb_actions = b_actions.index_select(0, mb_inds)
                if fused_loss:
                    # the HIP losses (fused.PolicyLoss / ValueLoss): same quantities, ~5 launches instead of ~60
                    mean_z = (self.actor.update_mean(mb_pomdps, mb_state, mb_done) if self.recurrent
                              else self.actor.update_mean(mb_pomdps))
                    pg_loss, approx_kl, clipfrac = PolicyLoss.apply(
                        mean_z, self.actor.actor_logstd, mb_actions, mb_logp,
                        mb_advs, self.clip_coef, self.norm_adv)
                    newvalue = self.critic(mb_obs).view(-1)
                    v_loss = ValueLoss.apply(newvalue, mb_ret)
                    clipfracs += clipfrac
                    n_mb += 1
                    actor_loss = pg_loss
                else:
                    if self.recurrent:
                        _, newlogprob, entropy, _ = self.actor(mb_pomdps, mb_state, mb_done,
                                                               mb_actions)
                    else:
                        _, newlogprob, entropy = self.actor(mb_pomdps, mb_actions)
                    newvalue = self.critic(mb_obs).view(-1)
                    logratio = newlogprob - mb_logp
                    ratio = logratio.exp()
                    with torch.no_grad():
                        approx_kl = ((ratio - 1) - logratio).mean()
                        clipfracs += ((ratio - 1.0).abs() > self.clip_coef).float().mean()
                        n_mb += 1
                    mb_adv = mb_advs
                    if self.norm_adv:
                        mb_adv = (mb_adv - mb_adv.mean()) / (mb_adv.std() + 1e-8)
                    pg_loss = torch.max(-mb_adv * ratio,
                                        -mb_adv * torch.clamp(ratio, 1 - self.clip_coef, 1 + self.clip_coef)).mean()
                    v_loss = 0.5 * ((newvalue - mb_ret) ** 2).mean()
                    actor_loss = pg_loss - self.ent_coef * entropy.mean()
                critic_loss = v_loss * self.vf_coef

                self.actor_optimizer.zero_grad()
                actor_loss.backward()
                allreduce_grads(self.actor)            # data parallel over ranks (no-op on one GPU)
                self._clip_step(0, self.actor, self.actor_optimizer)

                self.critic_optimizer.zero_grad()
                critic_loss.backward()
                allreduce_grads(self.critic)
                self._clip_step(1, self.critic, self.critic_optimizer)
                stats = {"pg_loss": pg_loss.detach(), "v_loss": v_loss.detach(), "approx_kl": approx_kl}
            if self.target_kl is not None and float(stats["approx_kl"]) > self.target_kl:
                break
        stats["clipfrac"] = clipfracs / max(n_mb, 1)
        return stats

    def _clip_step(self, which, net, optimizer):
        """clip_grad_norm_(net, max_grad_norm) + optimizer.step() (agent.py:124-134)."""
        if self._clip_adam is not None:
            self._clip_adam[which].step(self.max_grad_norm)
        else:
            nn.utils.clip_grad_norm_(net.parameters(), self.max_grad_norm)
            optimizer.step()

    # -------------------------------------------------------------- checkpoints
    def save(self, filename):
        """Same four files as agent.py:127-131."""
        torch.save(self.critic.state_dict(), filename + "_critic")
        torch.save(self.critic_optimizer.state_dict(), filename + "_critic_optimizer")
        torch.save(self.actor.state_dict(), filename + "_actor")
        torch.save(self.actor_optimizer.state_dict(), filename + "_actor_optimizer")

    def load(self, filename):
        """agent.py:133-139; tensors only (weights_only)."""
        m = self.device
        self.critic.load_state_dict(torch.load(filename + "_critic", map_location=m, weights_only=True))
        self.critic_optimizer.load_state_dict(torch.load(filename + "_critic_optimizer", map_location=m,
                                                         weights_only=True))
        self.actor.load_state_dict(torch.load(filename + "_actor", map_location=m, weights_only=True))
        self.actor_optimizer.load_state_dict(torch.load(filename + "_actor_optimizer", map_location=m,
                                                        weights_only=True))


class GraphedPolicy:
    """The rollout step's policy call (trunk MLP, input projection, LSTM GEMM + fused cell kernel,
    mean head, Normal sample, log-prob, entropy: ~25 launches) captured once in a hipGraph and
    replayed per step.  Eagerly each of those launches costs several µs of host time, ~440 µs per
    4096-env step in all, 100x the env step; a replay is one host call.

    Inputs are copied into static buffers before each replay; the parameters are read in place
    (Adam updates them in place, so every replay sees the current policy).  The sample's standard
    normal draws are made by ``normal_`` into a static buffer before each replay (models._policy_head:
    the sample is mean + std * eps).  The LSTM's final carry is written into the static carry input
    buffers themselves (``LSTMActor.carry_inplace``), so a carry handed back from the previous replay
    (``alias=True``) needs no copy; any other carry is copied in.
    """

    def __init__(self, learner, warmup=3):
        self.learner = learner
        self.warmup = warmup
        self.graph = None

    def _capture(self, state, lstm_state, done):
        ln = self.learner
        self.s_in = state.detach().clone()
        self.s_done = done.detach().clone()
        self.s_lstm = (lstm_state[0].detach().clone(), lstm_state[1].detach().clone()) if ln.recurrent else None
        self.s_eps = torch.zeros((state.shape[0], ln.actor.actor_logstd.shape[1]), device=ln.device)
        side = torch.cuda.Stream(device=ln.device)
        side.wait_stream(torch.cuda.current_stream(ln.device))
        # the LSTM's final carry is written back into the static input buffers (models.LSTMActor.carry_inplace),
        # so the replay's output carry IS its next input: no copy in or out when the caller hands it back
        if ln.recurrent and os.environ.get("OUZ_GRAPH_CARRY_INPLACE", "1") != "0":
            ln.actor.carry_inplace = self.s_lstm
        try:
            with torch.cuda.stream(side):   # warm-up: lazy workspaces / kernels resolved outside the capture
                for _ in range(self.warmup):
                    ln.get_action(self.s_in, self.s_lstm, self.s_done, eps=self.s_eps)
            torch.cuda.current_stream(ln.device).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            # relaxed: the caching allocator may map a fresh segment for the graph's private pool during
            # the capture
            with torch.cuda.graph(self.graph, capture_error_mode="relaxed"):
                self.out = ln.get_action(self.s_in, self.s_lstm, self.s_done, eps=self.s_eps)
        finally:
            if ln.recurrent:
                ln.actor.carry_inplace = None

    def _matches(self, state, lstm_state, done):
        """The call has the captured shapes, dtypes and device (a broadcastable but different batch would
        otherwise be silently broadcast by copy_ into the static buffers)."""
        def same(a, b):
            return a.shape == b.shape and a.dtype == b.dtype and a.device == b.device
        if not (same(state, self.s_in) and same(done, self.s_done)):
            return False
        if self.s_lstm is None:
            return lstm_state is None
        return lstm_state is not None and same(lstm_state[0], self.s_lstm[0]) and same(lstm_state[1], self.s_lstm[1])

    def __call__(self, state, lstm_state, done, alias=False):
        """One replay.  ``alias=False`` (the default) returns copies, as ``get_action`` would; ``alias=True``
        returns the graph's output buffers themselves, which the next replay overwrites (the rollout loop
        copies them into its storage right away, train.py)."""
        if self.graph is None or not self._matches(state, lstm_state, done):
            self._capture(state, lstm_state, done)
        self.s_in.copy_(state)
        self.s_done.copy_(done)
        self.s_eps.normal_()
        if self.s_lstm is not None:
            for dst, src in zip(self.s_lstm, lstm_state):
                if src is not dst:          # the previous replay's carry handed back (alias=True): already there
                    dst.copy_(src)
        self.graph.replay()
        if alias:
            return self.out
        return tuple(None if x is None else (tuple(y.clone() for y in x) if isinstance(x, tuple) else x.clone())
                     for x in self.out)
