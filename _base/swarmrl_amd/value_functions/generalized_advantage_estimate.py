"""
Generalized advantage estimate (reference:
swarmrl/value_functions/generalized_advantage_estimate.py:14-72), in torch.
"""

import numpy as np
import torch


class GAE:
    def __init__(self, gamma: float = 0.99, lambda_: float = 0.95):
        self.gamma = gamma
        self.lambda_ = lambda_
        self.eps = np.finfo(np.float32).eps.item()

    def __call__(self, rewards: torch.Tensor, values: torch.Tensor):
        """rewards, values: (n_time_steps, n_particles) -> (advantages, returns)."""
        rewards = torch.as_tensor(rewards, dtype=torch.float32)
        values = torch.as_tensor(values, dtype=torch.float32, device=rewards.device)
        T = rewards.shape[0]
        gae = torch.zeros_like(rewards[0])
        advantages = torch.zeros_like(rewards)
        for t in reversed(range(T)):
            if t != T - 1:
                delta = rewards[t] + self.gamma * values[t + 1] - values[t]
            else:
                delta = rewards[t] - values[t]
            gae = delta + self.gamma * self.lambda_ * gae
            advantages[t] = gae
        returns = advantages + values
        advantages = (advantages - advantages.mean()) / (
            advantages.std(unbiased=False) + self.eps
        )
        return advantages, returns
