"""
Trajectory buffer of an agent (reference: swarmrl/utils/colloid_utils.py:15-26).
"""

from dataclasses import dataclass, field


@dataclass
class TrajectoryInformation:
    """Per-episode features, actions, log-probs and rewards of one agent."""

    particle_type: int
    features: list = field(default_factory=list)
    actions: list = field(default_factory=list)
    log_probs: list = field(default_factory=list)
    rewards: list = field(default_factory=list)
    killed: bool = False
