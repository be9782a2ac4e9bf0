"""
Action data class (reference: swarmrl/actions/actions.py:10-19).
"""

import dataclasses

import numpy as np


@dataclasses.dataclass
class Action:
    """
    The quantities applied to one colloid: a swim force along the director,
    a lab-frame torque and an optional new direction.
    """

    id = 0
    force: float = 0.0
    torque: np.ndarray = None
    new_direction: np.ndarray = None
