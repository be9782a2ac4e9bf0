"""
SpeciesSearch task (reference: swarmrl/tasks/searching/species_search.py:17-184):
reward = scale * clip(field - previous field, 0, inf) (or (-inf, 0] with
``avoid``), the field being ``sum(decay(|x_j - x_i| / L))`` over the sensed
colloids; history per colloid id.  Distances in HIP, see
``swarmrl_amd.engine.pair_field``.
"""

import numpy as np
import torch

from swarmrl_amd.engine.pair_field import list_pair_field, pair_field
from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.tasks.task import Task


class SpeciesSearch(Task):
    supports_device = True

    def __init__(self, decay_fn: callable, box_length: np.ndarray, sensing_type: int = 0,
                 avoid: bool = False, scale_factor: int = 100, particle_type: int = 0):
        super().__init__(particle_type=particle_type)
        self.decay_fn = decay_fn
        self.box_length = box_length
        self.sensing_type = sensing_type
        self.scale_factor = scale_factor
        self.avoid = avoid
        self.historical_field = {}
        self._dev_hist = None

    def _field(self, colloids):
        if is_view(colloids):
            view = colloids
            return pair_field(view.engine._native, view.n_envs,
                              view.indices_of_type(self.particle_type),
                              view.indices_of_type(self.sensing_type), self.box_length,
                              self.decay_fn)
        ids = self.get_colloid_indices(colloids)
        return list_pair_field(colloids, ids, self.sensing_type, self.box_length, self.decay_fn)

    def initialize(self, colloids):
        field = self._field(colloids)
        if is_view(colloids):
            self._dev_hist = (id(colloids.engine), field)
            self.historical_field = {"__device__": True}
            return
        for i, value in zip(self.get_colloid_indices(colloids), field):
            self.historical_field[str(colloids[i].id)] = float(value)

    def __call__(self, colloids):
        """Rewards: (A,) numpy for lists, [E, A] device tensor for views."""
        if self.historical_field == {}:
            msg = (
                f"{type(self).__name__} requires initialization. Please set the "
                "initialize attribute of the gym to true and try again."
            )
            raise ValueError(msg)
        field = self._field(colloids)
        if is_view(colloids):
            if self._dev_hist is None or self._dev_hist[0] != id(colloids.engine):
                raise ValueError(f"{type(self).__name__} was initialised for another engine")
            delta = field - self._dev_hist[1]
            self._dev_hist = (self._dev_hist[0], field)
            delta = torch.clamp(delta, max=0.0) if self.avoid else torch.clamp(delta, min=0.0)
            return self.scale_factor * delta
        ids = self.get_colloid_indices(colloids)
        keys = [str(colloids[i].id) for i in ids]
        hist = np.array([self.historical_field[k] for k in keys], dtype=np.float32)
        for k, v in zip(keys, field):
            self.historical_field[k] = float(v)
        delta = field - hist
        delta = np.clip(delta, None, 0) if self.avoid else np.clip(delta, 0, None)
        return (self.scale_factor * delta).astype(np.float32)
