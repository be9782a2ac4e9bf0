"""
Director observable (reference: swarmrl/observables/director.py): the
director of every colloid of the observable's type.  With a SwarmView the
result is a device tensor [E, A, 3] (no host sync).
"""

from typing import List

import numpy as np

from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.observables.observable import Observable


class Director(Observable):
    supports_device = True

    def __init__(self, particle_type: int = 0):
        super().__init__(particle_type=particle_type)

    def compute_single_observable(self, index: int, colloids: list):
        return np.copy(colloids[index].director)

    def compute_observable(self, colloids) -> List:
        if is_view(colloids):
            idx = self.get_colloid_indices(colloids).long()
            return colloids.directors()[:, idx]
        return [self.compute_single_observable(i, colloids)
                for i in self.get_colloid_indices(colloids)]
