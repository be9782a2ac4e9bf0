"""
Random Network Distillation configuration (reference:
swarmrl/intrinsic_reward/rnd_configs.py:17-101).  The reference trains with
ZnNL (SimpleTraining + MeanPowerLoss(order=2), OrderNDifference(order=2)
metric, optax.adam(1e-3)); ZnNL is not available here, the same recipe is
restated in PyTorch.
"""

from dataclasses import dataclass, field
from typing import Optional

import torch
from torch import nn


class RNDArchitecture(nn.Module):
    """Dense(32) -> ReLU -> Dense(32) -> ReLU -> Dense(32) (rnd_configs.py:17-38)."""

    def __init__(self, input_dim: int, width: int = 32):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(input_dim, width), nn.ReLU(), nn.Linear(width, width),
                                 nn.ReLU(), nn.Linear(width, width))

    def forward(self, x):
        return self.net(x)


def order_n_difference(a: torch.Tensor, b: torch.Tensor, order: int = 2) -> torch.Tensor:
    """ZnNL OrderNDifference: per point, (sum |a - b|^order)^(1/order)."""
    return torch.sum(torch.abs(a - b) ** order, dim=-1) ** (1.0 / order)


@dataclass
class RNDConfig:
    input_shape: tuple
    n_epochs: int = 100
    batch_size: int = 8
    clip_rewards: Optional[tuple] = (-5.0, 5.0)
    learning_rate: float = 1e-3
    distance_order: int = 2
    loss_order: int = 2
    training_kwargs: Optional[dict] = field(default_factory=dict)
    device: Optional[torch.device] = None
