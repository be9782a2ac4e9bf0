from swarmrl_amd.sampling_strategies.categorical_distribution import CategoricalDistribution
from swarmrl_amd.sampling_strategies.gumbel_distribution import GumbelDistribution
from swarmrl_amd.sampling_strategies.sampling_strategy import SamplingStrategy

__all__ = ["SamplingStrategy", "GumbelDistribution", "CategoricalDistribution"]
