"""
Random exploration (reference:
swarmrl/exploration_policies/random_exploration.py:14-73): with probability
p an agent's action is replaced by a uniform random index.  The reference's
clip arithmetic is kept verbatim, on device tensors.
"""

import torch


class ExplorationPolicy:
    def __call__(self, model_actions, action_space_length: int, seed=None):
        raise NotImplementedError


class RandomExploration(ExplorationPolicy):
    def __init__(self, probability: float = 0.1):
        self.probability = probability

    def __call__(self, model_actions: torch.Tensor, action_space_length: int,
                 generator: torch.Generator = None) -> torch.Tensor:
        if self.probability == 0.0:
            return model_actions
        dev = model_actions.device
        sample = torch.rand(model_actions.shape, device=dev, generator=generator)
        to_be_changed = torch.clamp(sample - self.probability, 0, 1)
        to_be_changed = torch.clamp(to_be_changed * 1e6, 0, 1)
        not_to_be_changed = torch.clamp(to_be_changed * -10 + 1, 0, 1)
        exploration_actions = torch.randint(
            0, action_space_length, model_actions.shape, device=dev, generator=generator
        )
        out = model_actions * to_be_changed + exploration_actions * not_to_be_changed
        return out.to(torch.int64)
