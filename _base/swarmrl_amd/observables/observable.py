"""
Parent class for observables (reference: swarmrl/observables/observable.py:10-96).
"""

from typing import List

from swarmrl_amd.engine.swarm_view import is_view


class Observable:
    """Observables are the inputs of the agents' networks."""

    #: True when compute_observable accepts a SwarmView (device tensors).
    supports_device = False

    def __init__(self, particle_type: int):
        self._shape = None
        self.particle_type: int = particle_type

    def initialize(self, colloids):
        """Initialise with the starting positions (default: nothing to do)."""
        pass

    def get_colloid_indices(self, colloids, p_type: int = None) -> List[int]:
        """Indices of the colloids of one type (observable.py:40-68)."""
        if p_type is None:
            p_type = self.particle_type
        if is_view(colloids):
            return colloids.indices_of_type(p_type)
        indices = []
        for i, colloid in enumerate(colloids):
            if colloid.type == p_type:
                indices.append(i)
        return indices

    def compute_observable(self, colloids):
        raise NotImplementedError("Implemented in child class.")

    @property
    def observable_shape(self):
        return self._shape
