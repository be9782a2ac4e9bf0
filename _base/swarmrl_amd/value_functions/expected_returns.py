"""
Discounted expected returns (reference: swarmrl/value_functions/expected_returns.py).
"""

import numpy as np
import torch


class ExpectedReturns:
    def __init__(self, gamma: float = 0.99, standardize: bool = True):
        self.gamma = gamma
        self.standardize = standardize
        self.eps = np.finfo(np.float32).eps.item()

    def __call__(self, rewards: torch.Tensor) -> torch.Tensor:
        rewards = torch.as_tensor(rewards, dtype=torch.float32)
        T = rewards.shape[0]
        out = torch.zeros_like(rewards)
        acc = torch.zeros_like(rewards[0])
        for t in reversed(range(T)):
            acc = rewards[t] + self.gamma * acc
            out[t] = acc
        if self.standardize:
            mean = out.mean(dim=0)
            std = out.std(dim=0, unbiased=False)
            out = (out - mean) / (std + self.eps)
        return out
