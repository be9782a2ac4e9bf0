"""
Parent class for tasks (reference: swarmrl/tasks/task.py:15-118).
"""

from typing import List

from swarmrl_amd.engine.swarm_view import is_view


class Task:
    """A task turns the state of the colloids into rewards."""

    supports_device = False

    def __init__(self, particle_type: int = 0):
        self.particle_type = particle_type
        self._kill_switch = False

    @property
    def kill_switch(self):
        return self._kill_switch

    @kill_switch.setter
    def kill_switch(self, value: bool):
        self._kill_switch = value

    def initialize(self, colloids):
        pass

    def get_colloid_indices(self, colloids, p_type: int = None) -> List[int]:
        if p_type is None:
            p_type = self.particle_type
        if is_view(colloids):
            return colloids.indices_of_type(p_type)
        indices = []
        for i, colloid in enumerate(colloids):
            if colloid.type == p_type:
                indices.append(i)
        return indices

    def __call__(self, colloids):
        raise NotImplementedError("Implemented in child class.")
