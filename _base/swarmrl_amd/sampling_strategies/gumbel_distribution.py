"""
Gumbel-max sampling (reference:
swarmrl/sampling_strategies/gumbel_distribution.py:14-42):
idx = argmax(logits - log(-log U)), U ~ Uniform[0, 1).
JAX's threefry stream is replaced by torch's device generator, so parity with
the reference is statistical (test_gumbel.py style), not per draw.
"""

import torch

from swarmrl_amd.sampling_strategies.sampling_strategy import SamplingStrategy


class GumbelDistribution(SamplingStrategy):
    """Gumbel-max trick for categorical sampling on device."""

    def __call__(self, logits: torch.Tensor, generator: torch.Generator = None) -> torch.Tensor:
        noise = torch.rand(logits.shape, device=logits.device, dtype=logits.dtype,
                           generator=generator)
        return torch.argmax(logits - torch.log(-torch.log(noise)), dim=-1)
