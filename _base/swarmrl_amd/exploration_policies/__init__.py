from swarmrl_amd.exploration_policies.random_exploration import (
    ExplorationPolicy,
    RandomExploration,
)

__all__ = ["ExplorationPolicy", "RandomExploration"]
