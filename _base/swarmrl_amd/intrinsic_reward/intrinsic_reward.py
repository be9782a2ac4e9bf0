"""
Intrinsic reward interface (reference:
swarmrl/intrinsic_reward/intrinsic_reward.py:11-42).
"""


class IntrinsicReward:
    """Reward computed from the agent's own trajectory (e.g. novelty)."""

    #: True when compute_reward / update accept device trajectories
    supports_device = False

    def update(self, episode_data):
        raise NotImplementedError("Implemented in child class.")

    def compute_reward(self, episode_data):
        raise NotImplementedError("Implemented in child class.")
