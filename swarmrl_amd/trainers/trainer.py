"""
Trainer parent (reference: swarmrl/trainers/trainer.py:13-142).
"""

from typing import List, Tuple

import numpy as np
import torch

from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.force_functions.force_fn import ForceFunction


def _mean_reward(rewards) -> float:
    if len(rewards) == 0:
        return 0.0
    if isinstance(rewards[0], torch.Tensor):
        return float(torch.stack([r.float() for r in rewards]).mean().item())
    return float(np.mean(rewards))


class Trainer:
    _engine = None

    @property
    def engine(self):
        return self._engine

    @engine.setter
    def engine(self, value):
        self._engine = value

    def __init__(self, agents: List[ActorCriticAgent]):
        self.agents = {}
        for agent in agents:
            self.agents[str(agent.particle_type)] = agent

    def initialize_training(self) -> ForceFunction:
        return ForceFunction(agents=self.agents)

    def update_rl(self) -> Tuple[ForceFunction, np.ndarray, bool]:
        reward = 0.0
        switches = []
        for agent in self.agents.values():
            if isinstance(agent, ActorCriticAgent):
                ag_reward, ag_killed = agent.update_agent()
                reward += _mean_reward(ag_reward)
                switches.append(ag_killed)
        interaction_model = ForceFunction(agents=self.agents)
        return interaction_model, np.array(reward), any(switches)

    def export_models(self, directory: str = "Models"):
        for agent in self.agents.values():
            agent.save_agent(directory)

    def restore_models(self, directory: str = "Models"):
        for agent in self.agents.values():
            agent.restore_agent(directory)

    def initialize_models(self):
        for agent in self.agents.values():
            agent.initialize_network()

    def perform_rl_training(self, **kwargs):
        raise NotImplementedError("Implemented in child class")
