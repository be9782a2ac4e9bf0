"""
Parent class for sampling strategies (reference:
swarmrl/sampling_strategies/sampling_strategy.py:13-24).
"""

import torch


class SamplingStrategy:
    """Turns logits into action indices."""

    def compute_entropy(self, probabilities: torch.Tensor) -> torch.Tensor:
        """-sum p log p with eps = 1e-8 added to p (sampling_strategy.py)."""
        eps = 1e-8
        probabilities = probabilities + eps
        return -torch.sum(probabilities * torch.log(probabilities))

    def __call__(self, logits: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError("Implemented in child classes.")
