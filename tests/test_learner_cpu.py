"""Learner pieces that run without a GPU: the GAE oracle against the reference's own getGAE
(tests/golden/learner.npz), and the re-laid LSTM actor / critic against the reference modules'
outputs with the reference's parameters loaded by their state_dict names."""
import os

import numpy as np
import pytest
import torch

from oracle import learner_oracle as LO
from ouzelum_amd.learners.models import Critic, LSTMActor, MLPActor
from ouzelum_amd.spaces import Box


@pytest.fixture(scope="module")
def lg(golden):
    return golden("learner.npz")


def _spaces():
    return Box(-np.inf * np.ones(13), np.inf * np.ones(13)), Box(-np.ones(4), np.ones(4))


def test_gae_oracle_bit_exact_vs_reference(lg):
    ret, adv = LO.gae_f32(lg["gae_rewards"], lg["gae_values"], lg["gae_dones"], lg["gae_next_value"],
                          lg["gae_next_done"])
    np.testing.assert_array_equal(adv, lg["gae_advantages"])
    np.testing.assert_array_equal(ret, lg["gae_returns"])


def _load(module, lg, prefix):
    sd = {k[len(prefix):]: torch.tensor(lg[k]) for k in lg.files if k.startswith(prefix)}
    module.load_state_dict(sd, strict=True)
    return module


def test_parameter_names_match_reference(lg):
    obs_s, act_s = _spaces()
    ref_actor = {k[len("actor."):] for k in lg.files if k.startswith("actor.")}
    ref_critic = {k[len("critic."):] for k in lg.files if k.startswith("critic.")}
    assert set(LSTMActor(obs_s, act_s).state_dict()) == ref_actor
    assert set(Critic(obs_s).state_dict()) == ref_critic


def test_lstm_actor_matches_reference(lg):
    obs_s, act_s = _spaces()
    actor = _load(LSTMActor(obs_s, act_s), lg, "actor.")
    critic = _load(Critic(obs_s), lg, "critic.")
    with torch.no_grad():
        hid, (h1, c1) = actor.get_states(torch.tensor(lg["lstm_x"]), (torch.tensor(lg["lstm_h0"]),
                                                                       torch.tensor(lg["lstm_c0"])),
                                         torch.tensor(lg["lstm_done"]))
        mean = actor.actor_mean(hid)
        v = critic(torch.tensor(lg["lstm_x"]))
    # one GEMM for the input projection vs nn.LSTM per step: f32 reassociation only
    np.testing.assert_allclose(hid.numpy(), lg["lstm_hidden"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(h1.numpy(), lg["lstm_h1"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(c1.numpy(), lg["lstm_c1"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(mean.numpy(), lg["actor_mean_out"], atol=1e-6, rtol=1e-5)
    np.testing.assert_allclose(v.numpy(), lg["critic_out"], atol=1e-5, rtol=1e-5)


def test_policy_heads():
    obs_s, act_s = _spaces()
    torch.manual_seed(0)
    x = torch.randn(24, 13)
    a, lp, ent = MLPActor(obs_s, act_s)(x)
    assert a.shape == (24, 4) and lp.shape == (24,) and ent.shape == (24,)
    actor = LSTMActor(obs_s, act_s)
    h = actor.initial_state(8, "cpu")
    a, lp, ent, (h1, c1) = actor(x, h, torch.zeros(24))
    assert a.shape == (24, 4) and h1.shape == (1, 8, 128)
    # RPO: with an action given the mean is perturbed by U(-0.5, 0.5): log-probs differ from the clean head
    _, lp2, _, _ = actor(x, h, torch.zeros(24), a)
    assert not torch.allclose(lp, lp2)


def test_learner_pomdp_oracle_modes():
    rs = np.random.RandomState(0)
    x = rs.normal(0, 1, (300, 13)).astype(np.float32)
    flick = [LO.pomdp_obs(x, 1, 0.3, 11, 0, c) for c in range(200)]
    frac = np.mean([float(np.all(f == 0)) for f in flick])
    assert 0.2 < frac < 0.4                                   # one coin per call, p = 0.3
    assert all(np.all(f == 0) or np.array_equal(f, x) for f in flick)
    y = LO.pomdp_obs(x, 2, 0.25, 11, 0, 0)
    r = y / x
    assert r.min() >= 0.75 - 1e-6 and r.max() <= 1.25 + 1e-6
    # sharded rows draw what the unsharded run draws for the same global rows
    np.testing.assert_array_equal(LO.pomdp_obs(x[100:], 2, 0.25, 11, 100, 0), y[100:])


def test_gemm_tuning_is_gpu_only_and_can_be_turned_off(monkeypatch):
    from ouzelum_amd.learners import gemm_tuning as G
    assert not G.enable_tuned_gemms("cpu")
    monkeypatch.setenv("OUZ_TUNABLEOP", "0")
    assert not G.enable_tuned_gemms("cuda:0")
    with open(G.SHIPPED) as fh:
        head = fh.read()
    assert "Validator,GCN_ARCH_NAME,gfx950" in head and "GemmTunableOp_float" in head


def test_play_builds_its_learner_without_tunableop():
    """the inference-only player does not turn on process-wide TunableOp."""
    import inspect
    from ouzelum_amd import play as P
    from ouzelum_amd.learners.ppo import PPOLearner
    assert inspect.signature(PPOLearner).parameters["tuned_gemms"].default is True
    assert "tuned_gemms=False" in inspect.getsource(P._actions_fn)


def test_direct_sample_head_equals_the_normal_form():
    """models._sample_head (the rollout's sample on the (1, A) log-std terms) against torch's Normal: same action,
    log-prob and entropy within f32 rounding."""
    import torch
    from torch.distributions.normal import Normal
    from ouzelum_amd.learners.models import _sample_head
    g = torch.Generator().manual_seed(3)
    mean = torch.randn(4096, 4, generator=g)
    logstd = torch.randn(1, 4, generator=g) * 0.5
    eps = torch.randn(4096, 4, generator=g)
    a, lp, ent = _sample_head(mean, logstd, eps)
    std = torch.exp(logstd.expand_as(mean))
    p = Normal(mean, std, validate_args=False)
    torch.testing.assert_close(a, mean + std * eps, rtol=0, atol=1e-6)
    torch.testing.assert_close(lp, p.log_prob(a).sum(1), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ent, p.entropy().sum(1), rtol=1e-6, atol=1e-6)


def test_tensorboard_event_file_round_trips(tmp_path):
    """learners/tbevents.py writes the reference's SummaryWriter scalars (PPO/main.py:101-109) as a TensorBoard event
    file: TFRecord framing with masked CRC-32C, tensorflow.Event protobufs.  Parsed back by its own reader, and the
    payloads checked independently against the Event / Summary schema with google.protobuf."""
    import struct
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    from ouzelum_amd.learners import tbevents as TB
    assert TB.crc32c(b"123456789") == 0xE3069283          # the CRC-32C check value
    w = TB.EventWriter(str(tmp_path / "RPO_LSTM_flicker_0.1"))
    pts = [("charts/episodic_return", 65536, 1.25), ("charts/episodic_length", 65536, 212.0),
           ("average/average_reward", 65536, 0.0625), ("average/average_reward", 131072, -3.5)]
    for tag, step, v in pts:
        w.add_scalar(tag, v, step)
    w.close()
    assert os.path.basename(w.path).startswith("events.out.tfevents.")
    got, version = TB.read_scalars(w.path)
    assert version == "brain.Event:2"
    assert [(t, s, v) for t, s, v, _ in got] == pts
    # the schema, declared here from tensorflow/core/util/event.proto and framework/summary.proto (field numbers)
    fd = descriptor_pb2.FileDescriptorProto(name="ev.proto", package="tf")
    val = fd.message_type.add(name="Value")
    val.field.add(name="tag", number=1, type=9, label=1)
    val.field.add(name="simple_value", number=2, type=2, label=1)
    summ = fd.message_type.add(name="Summary")
    summ.field.add(name="value", number=1, type=11, label=3, type_name=".tf.Value")
    ev = fd.message_type.add(name="Event")
    ev.field.add(name="wall_time", number=1, type=1, label=1)
    ev.field.add(name="step", number=2, type=3, label=1)
    ev.field.add(name="file_version", number=3, type=9, label=1)
    ev.field.add(name="summary", number=5, type=11, label=1, type_name=".tf.Summary")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    Event = message_factory.GetMessageClass(pool.FindMessageTypeByName("tf.Event"))
    recs = TB.read_records(w.path)
    first = Event.FromString(recs[0])
    assert first.file_version == "brain.Event:2"
    for rec, (tag, step, v) in zip(recs[1:], pts):
        e = Event.FromString(rec)
        assert e.step == step and e.summary.value[0].tag == tag and e.summary.value[0].simple_value == v
        assert e.SerializeToString() == rec                      # canonical protobuf encoding
    with open(w.path, "rb") as fh:
        data = bytearray(fh.read())
    data[-1] ^= 1
    bad = tmp_path / "bad"
    bad.write_bytes(bytes(data))
    with pytest.raises(ValueError, match="CRC"):
        TB.read_records(str(bad))
    assert struct.calcsize("<Q") == 8


def test_clip_adam_refuses_cpu_and_unsupported_optimizers():
    """fused.ClipAdam (the two-launch clip + Adam step) takes plain Adam over f32 CUDA tensors only; anything else is
    refused at construction, and PPOLearner on the CPU keeps torch's clip_grad_norm_ + Adam."""
    import torch
    from ouzelum_amd.learners.fused import ClipAdam
    lin = torch.nn.Linear(4, 4)
    with pytest.raises(ValueError):
        ClipAdam(torch.optim.Adam(lin.parameters()))
    from ouzelum_amd.learners import PPOLearner
    from ouzelum_amd.spaces import Box
    obs_s, act_s = Box(-np.inf * np.ones(13), np.inf * np.ones(13)), Box(-np.ones(4), np.ones(4))
    ag = PPOLearner(obs_s, act_s, 8, "cpu", recurrent=False, num_minibatches=1, update_epochs=1)
    assert ag._clip_adam is None


def test_store_copies_every_pair():
    """fused.store (the rollout loop's storage writes; one multi-tensor copy on a GPU) copies each source into its
    destination slice, here through the per-tensor fallback of CPU tensors."""
    import torch
    from ouzelum_amd.learners.fused import store
    obs, dones = torch.zeros(4, 8, 13), torch.zeros(4, 8)
    o, d = torch.randn(8, 13), torch.rand(8)
    store((obs[2], dones[2]), (o, d))
    assert torch.equal(obs[2], o) and torch.equal(dones[2], d)
    assert float(obs[[0, 1, 3]].abs().sum()) == 0.0 and float(dones[[0, 1, 3]].abs().sum()) == 0.0
