"""
Episodic trainer (reference: swarmrl/trainers/episodic_trainer.py:26-130).
"""

import numpy as np

from swarmrl_amd.trainers.trainer import Trainer


class EpisodicTrainer(Trainer):
    def perform_rl_training(self, get_engine: callable, system, n_episodes: int,
                            episode_length: int, reset_frequency: int = 1,
                            load_bar: bool = True, save_episodic_data: bool = True):
        killed = False
        rewards = [0.0]
        force_fn = self.initialize_training()
        cycle_index = 0
        for episode in range(n_episodes):
            if episode % reset_frequency == 0 or killed:
                self.engine = None
                if save_episodic_data:
                    try:
                        self.engine = get_engine(system, f"{cycle_index}")
                        cycle_index += 1
                    except TypeError:
                        raise ValueError(
                            "The system runner does not support episodic data saving. Your"
                            " get_engine function should take a system and a str(cycle_index)"
                            " as arguments."
                        )
                else:
                    self.engine = get_engine(system)
                for agent in self.agents.values():
                    agent.reset_agent(self.engine.colloids)
            self.engine.integrate(episode_length, force_fn)
            force_fn, current_reward, killed = self.update_rl()
            rewards.append(current_reward)
            self.engine.finalize()
        return np.array(rewards)
