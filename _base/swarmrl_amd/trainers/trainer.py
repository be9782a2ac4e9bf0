"""
Trainer base (reference: swarmrl/trainers/trainer.py:13-150).

The trainers are the callers of the hot path, not part of it: an episode is
one ``engine.integrate(episode_length, force_fn)``, after which every learning
agent runs its update.  They are restated here because the reference's
``Trainer.update_rl`` only updates agents that are instances of *its*
``swarmrl.agents.actor_critic.ActorCriticAgent`` (trainer.py:93-97) and builds
*its* ``ForceFunction``: with this package's agents it would silently skip
every update.  Same constructor, methods and return values as the reference.
"""

from __future__ import annotations

from typing import Iterable, Tuple

import numpy as np
import torch

from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.force_functions.force_fn import ForceFunction


def mean_reward(rewards) -> float:
    """Mean of an agent's episode rewards: a list of per-chunk arrays (host
    path) or of device tensors (device path; one host sync per episode)."""
    if rewards is None or len(rewards) == 0:
        return 0.0
    if isinstance(rewards[0], torch.Tensor):
        return float(torch.stack([r.float() for r in rewards]).mean().item())
    return float(np.mean(rewards))


def _is_killed(flag) -> bool:
    if isinstance(flag, torch.Tensor):
        return bool(flag.any().item())
    return bool(flag)


class Trainer:
    """Holds the agents by particle type and the engine of the current run."""

    _engine = None

    def __init__(self, agents: Iterable):
        self.agents = {str(agent.particle_type): agent for agent in agents}

    @property
    def engine(self):
        """The engine the trainer is currently driving."""
        return self._engine

    @engine.setter
    def engine(self, value):
        self._engine = value

    def initialize_training(self) -> ForceFunction:
        """The force function of the first episode (trainer.py:61-74)."""
        return ForceFunction(agents=self.agents)

    def update_rl(self) -> Tuple[ForceFunction, np.ndarray, bool]:
        """Update every learning agent after an episode (trainer.py:76-101).

        Returns the force function of the next episode, the summed mean
        episode reward of the learning agents, and whether any task asked to
        stop."""
        total = 0.0
        stop = False
        for agent in self.agents.values():
            if not isinstance(agent, ActorCriticAgent):
                continue  # classical / scripted agents do not learn
            rewards, killed = self._update_agent(agent)
            total += mean_reward(rewards)
            stop = stop or _is_killed(killed)
        return ForceFunction(agents=self.agents), np.array(total), stop

    def _update_agent(self, agent):
        """One learning agent's update after an episode (the episode-parallel
        trainers gather the episode over the ranks first)."""
        return agent.update_agent()

    def export_models(self, directory: str = "Models"):
        """Save every agent's network into `directory` (trainer.py:103-118)."""
        for agent in self.agents.values():
            agent.save_agent(directory)

    def restore_models(self, directory: str = "Models"):
        """Load every agent's network from `directory` (trainer.py:120-135)."""
        for agent in self.agents.values():
            agent.restore_agent(directory)

    def initialize_models(self):
        """Re-initialise every agent's network (trainer.py:137-142)."""
        for agent in self.agents.values():
            agent.initialize_network()

    def perform_rl_training(self, **kwargs):
        """Run the training; implemented by the concrete trainers."""
        raise NotImplementedError("Implemented in child class")

    # ------------------------------------------------------------ helpers
    @staticmethod
    def _progress(title: str, n_episodes: int, visible: bool):
        """A rich progress bar with the episode and running-reward fields of
        the reference's trainers (a no-op display when not visible)."""
        from rich.progress import BarColumn, Progress, TimeRemainingColumn

        bar = Progress(
            "Episode: {task.fields[Episode]}",
            BarColumn(),
            "Episode reward: {task.fields[current_reward]} Running Reward:"
            " {task.fields[running_reward]}",
            TimeRemainingColumn(),
            disable=not visible,
        )
        task = bar.add_task(title, total=n_episodes, Episode=0, current_reward=0.0,
                            running_reward=0.0, visible=visible)
        return bar, task

    @staticmethod
    def _advance(bar, task, episode: int, history):
        bar.update(task, advance=1, Episode=episode,
                   current_reward=np.round(history[-1], 2),
                   running_reward=np.round(np.mean(history[-10:]), 2))
