"""Recurrent PPO / RPO-LSTM learners driving the HIP env."""
from .models import Critic, LSTMActor, MLPActor
from .ppo import PPOLearner, gae
from .wrappers import ExtractObsWrapper, POMDPWrapper, RecordEpisodeStatisticsTorch

__all__ = ["Critic", "LSTMActor", "MLPActor", "PPOLearner", "gae", "ExtractObsWrapper", "POMDPWrapper",
           "RecordEpisodeStatisticsTorch"]
