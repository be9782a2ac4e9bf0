"""
Several observables at once (reference: swarmrl/observables/multi_sensing.py).

List path: the reference's object array of shape (n_colloids, n_observables).
SwarmView path: every observable's device tensor flattened per agent and
concatenated along the last axis, [E, A, sum of feature sizes] (the form a
network consumes; the reference flattens the object array the same way when
it stacks features).
"""

from typing import List

import numpy as np
import torch

from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.observables.observable import Observable


class MultiSensing(Observable):
    def __init__(self, observables: List[Observable]):
        self.observables = observables
        self._shape = None

    @property
    def supports_device(self):
        return all(getattr(o, "supports_device", False) for o in self.observables)

    @property
    def particle_type(self):
        return self.observables[0].particle_type if self.observables else 0

    def initialize(self, colloids):
        for item in self.observables:
            item.initialize(colloids)

    def compute_observable(self, colloids):
        if is_view(colloids):
            parts = [o.compute_observable(colloids) for o in self.observables]
            E, A = parts[0].shape[0], parts[0].shape[1]
            return torch.cat([p.reshape(E, A, -1).to(torch.float32) for p in parts], dim=-1)
        unshaped = [item.compute_observable(colloids) for item in self.observables]
        n_colloids = len(unshaped[0])
        observable = [[] for _ in range(n_colloids)]
        for item in unshaped:
            for j, value in enumerate(item):
                observable[j].append(value)
        return np.array(observable, dtype=object)
