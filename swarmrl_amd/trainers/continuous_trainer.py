"""
Continuous trainer (reference: swarmrl/trainers/continuous_trainer.py:22-89).
"""

import numpy as np

from swarmrl_amd.trainers.trainer import Trainer


class ContinuousTrainer(Trainer):
    def perform_rl_training(self, system_runner, n_episodes: int, episode_length: int,
                            load_bar: bool = True):
        self.engine = system_runner
        rewards = [0.0]
        force_fn = self.initialize_training()
        for agent in self.agents.values():
            agent.reset_agent(self.engine.colloids)
        for _ in range(n_episodes):
            self.engine.integrate(episode_length, force_fn)
            force_fn, current_reward, killed = self.update_rl()
            if killed:
                print("Simulation has been ended by the task, ending training.")
                system_runner.finalize()
                break
            rewards.append(current_reward)
        return np.array(rewards)
