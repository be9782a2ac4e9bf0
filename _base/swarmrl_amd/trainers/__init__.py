"""Training loops over the engine (reference: swarmrl/trainers/)."""

from swarmrl_amd.trainers.continuous_trainer import ContinuousTrainer
from swarmrl_amd.trainers.episode_parallel import (EpisodeParallelEpisodicTrainer,
                                                   EpisodeParallelTrainer)
from swarmrl_amd.trainers.episodic_trainer import EpisodicTrainer
from swarmrl_amd.trainers.trainer import Trainer

__all__ = ["Trainer", "ContinuousTrainer", "EpisodicTrainer", "EpisodeParallelTrainer",
           "EpisodeParallelEpisodicTrainer"]
