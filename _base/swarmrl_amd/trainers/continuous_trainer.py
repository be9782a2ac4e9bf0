"""
One engine, many episodes (reference: swarmrl/trainers/continuous_trainer.py:
13-89): the swarm keeps evolving across episodes; after each episode of
``episode_length`` slices every learning agent updates.
"""

from __future__ import annotations

import numpy as np

from swarmrl_amd.trainers.trainer import Trainer


class ContinuousTrainer(Trainer):
    """Continuous training on a single, never-reset engine."""

    def perform_rl_training(self, system_runner, n_episodes: int, episode_length: int,
                            load_bar: bool = True) -> np.ndarray:
        """Train for `n_episodes` episodes; returns [0.0, reward of episode
        1, ...].  An episode whose task raised the kill switch ends the
        training: the engine is finalized and that reward is not recorded
        (continuous_trainer.py:72-76)."""
        self.engine = system_runner
        history = [0.0]
        force_fn = self.initialize_training()
        for agent in self.agents.values():
            agent.reset_agent(self.engine.colloids)
        bar, task = self._progress("RL Training", n_episodes, load_bar)
        with bar:
            for episode in range(1, n_episodes + 1):
                self.engine.integrate(episode_length, force_fn)
                force_fn, reward, stop = self.update_rl()
                if stop:
                    print("Simulation has been ended by the task, ending training.")
                    system_runner.finalize()
                    break
                history.append(float(reward))
                self._advance(bar, task, episode, history)
        return np.array(history)
