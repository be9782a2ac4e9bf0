"""
Sum of several tasks (reference: swarmrl/tasks/multi_tasking.py).  Works on
Colloid lists and, when every task does, on SwarmViews (device rewards).
"""

from typing import List

import numpy as np

from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.tasks.task import Task


class MultiTasking(Task):
    def __init__(self, particle_type: int = 0, tasks: List[Task] = []):
        super().__init__(particle_type)
        self.tasks = tasks

    @property
    def supports_device(self):
        return all(getattr(t, "supports_device", False) for t in self.tasks)

    def initialize(self, colloids):
        for item in self.tasks:
            item.initialize(colloids)

    def __call__(self, colloids):
        if is_view(colloids):
            rewards = None
            for task in self.tasks:
                ts = task(colloids)
                rewards = ts if rewards is None else rewards + ts
            return rewards
        species_indices = self.get_colloid_indices(colloids)
        rewards = np.zeros(len(species_indices), dtype=np.float32)
        for task in self.tasks:
            rewards += np.asarray(task(colloids), dtype=np.float32)
        return rewards
