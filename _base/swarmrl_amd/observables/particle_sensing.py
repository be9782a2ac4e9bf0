"""
ParticleSensing observable (reference:
swarmrl/observables/particle_sensing.py:17-178): per agent, the change of
``sum(decay(|x_j - x_i| / L))`` over the sensed colloids since the last call,
times ``scale_factor``; history per colloid id.  Distances in HIP
(``swarm_pair_distances``), see ``swarmrl_amd.engine.pair_field``.
"""

import numpy as np
import torch

from swarmrl_amd.engine.pair_field import list_pair_field, pair_field
from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.observables.observable import Observable


class ParticleSensing(Observable):
    supports_device = True

    def __init__(self, decay_fn: callable, box_length: np.ndarray, sensing_type: int = 0,
                 scale_factor: int = 100, particle_type: int = 0):
        super().__init__(particle_type=particle_type)
        self.decay_fn = decay_fn
        self.box_length = box_length
        self.sensing_type = sensing_type
        self.scale_factor = scale_factor
        self.historical_field = {}
        self._dev_hist = None  # (engine id, [E, A] field)

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
        """Store the field of every agent (particle_sensing.py:63-93)."""
        field = self._field(colloids)
        if is_view(colloids):
            self._dev_hist = (id(colloids.engine), field)
            self.historical_field = {"__device__": True}
            return
        for i, value in zip(self.get_colloid_indices(colloids), field):
            self.historical_field[str(colloids[i].id)] = float(value)

    def compute_observable(self, colloids):
        """scale * (field - previous field): (A, 1), or [E, A, 1] on the device."""
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
            return (self.scale_factor * delta).unsqueeze(-1)
        ids = self.get_colloid_indices(colloids)
        keys = [str(colloids[i].id) for i in ids]
        hist = np.array([self.historical_field[k] for k in keys], dtype=np.float32)
        for k, v in zip(keys, field):
            self.historical_field[k] = float(v)
        return (self.scale_factor * (field - hist)).reshape(-1, 1).astype(np.float32)
