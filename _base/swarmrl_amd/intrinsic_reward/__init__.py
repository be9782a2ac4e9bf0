from swarmrl_amd.intrinsic_reward.intrinsic_reward import IntrinsicReward
from swarmrl_amd.intrinsic_reward.random_network_distillation import RNDReward
from swarmrl_amd.intrinsic_reward.rnd_configs import RNDArchitecture, RNDConfig

__all__ = ["IntrinsicReward", "RNDArchitecture", "RNDConfig", "RNDReward"]
