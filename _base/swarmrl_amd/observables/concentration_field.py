"""
Concentration-field observable (reference:
swarmrl/observables/concentration_field.py:22-138).

Per agent: ``scale * (f(|src/L - x_t/L|) - f(|src/L - x_{t-1}/L|))`` with a
per-id history of the previous position.  The distances (fp64 difference,
fp32 norm as in the reference) and the history update run in the HIP kernel
``k_field``; ``decay_fn`` is applied to the distance tensors (it must be
written with arithmetic operators, as the reference's are, e.g. ``1 - d``).
"""

import logging

import numpy as np
import torch

from swarmrl_amd.engine import ops
from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.observables.observable import Observable

logger = logging.getLogger(__name__)


class ConcentrationField(Observable):
    """Change of a field value along each agent's path."""

    supports_device = True

    def __init__(
        self,
        source: np.ndarray,
        decay_fn: callable,
        box_length: np.ndarray,
        scale_factor: int = 100,
        particle_type: int = 0,
    ):
        super().__init__(particle_type=particle_type)
        self.source = source / box_length
        self._source_raw = np.asarray(source, dtype=float)
        self.decay_fn = decay_fn
        self._historic_positions = {}
        self.box_length = box_length
        self.scale_factor = scale_factor
        self._observable_shape = (3,)
        self._dev_hist = None  # (engine id, hist_q, hist_img)
        self._pending = None
        self._affine = None

    # ------------------------------------------------------------ init
    def initialize(self, colloids):
        """Store the starting positions (concentration_field.py:66-82)."""
        if is_view(colloids):
            self._init_device(colloids)
            return
        engine = ops.engine_of(colloids)
        self._pending = None
        self._dev_hist = None
        if engine is not None:
            # engine handles: remember the raw coordinates for the GPU path
            self._pending = (id(engine), *ops.snapshot_history(engine, self.particle_type))
        for item in colloids:
            index = np.copy(item.id)
            position = np.copy(item.pos) / self.box_length
            self._historic_positions[str(index)] = position

    def _init_device(self, view):
        agents = view.indices_of_type(self.particle_type)
        A = int(agents.numel()) * view.n_envs
        hq = torch.zeros((3, A), dtype=torch.int32, device=view.device)
        hi = torch.zeros((3, A), dtype=torch.int32, device=view.device)
        ops.field_distance(
            view.engine._native, view.n_envs, agents, self._source_raw, self.box_length,
            hq, hi, update=True, init_only=True,
        )
        self._dev_hist = (id(view.engine), hq, hi)
        # keep the host dict non-empty so the "requires initialization"
        # check of the reference behaves the same for both paths
        self._historic_positions = {"__device__": True}

    # ---------------------------------------------------------- compute
    def _delta(self, d_cur, d_prev):
        return self.scale_factor * (self.decay_fn(d_cur) - self.decay_fn(d_prev))

    def compute_single_observable(self, index: int, colloids) -> float:
        reference_colloid = colloids[index]
        position = np.copy(reference_colloid.pos) / self.box_length
        key = str(np.copy(reference_colloid.id))
        previous_position = self._historic_positions[key]
        self._historic_positions[key] = position
        d_cur, d_prev = ops.list_field_distance(position[None], previous_position[None], self.source)
        return self._delta(d_cur, d_prev)[0]

    def compute_observable(self, colloids):
        """(N_agents, 1) per env; SwarmView input gives a device tensor [E, A, 1]."""
        if self._historic_positions == {}:
            msg = (
                f"{type(self).__name__} requires initialization. Please set the "
                "initialize attribute of the gym to true and try again."
            )
            raise ValueError(msg)
        if is_view(colloids):
            view = colloids
            if self._dev_hist is None and getattr(self, "_pending", None) is not None:
                if self._pending[0] == id(view.engine):
                    self._dev_hist = (self._pending[0], *ops.history_tensors(
                        self._pending[1], self._pending[2], view.device))
                self._pending = None
            if self._dev_hist is None or self._dev_hist[0] != id(view.engine):
                raise ValueError(f"{type(self).__name__} was initialised for another engine")
            agents = view.indices_of_type(self.particle_type)
            _, hq, hi = self._dev_hist
            if self._affine is None:
                self._affine = ops.affine_coefficients(self.decay_fn) or False
            if self._affine:
                return ops.field_transform(
                    view.engine._native, view.n_envs, agents, self._source_raw, self.box_length,
                    hq, hi, self._affine[0], self._affine[1], float(self.scale_factor), False,
                ).unsqueeze(-1)
            d_cur, d_prev = ops.field_distance(
                view.engine._native, view.n_envs, agents, self._source_raw, self.box_length,
                hq, hi, update=True,
            )
            return self._delta(d_cur, d_prev).unsqueeze(-1)
        reference_ids = self.get_colloid_indices(colloids)
        if len(reference_ids) == 0:
            return np.zeros((0, 1), dtype=np.float32)
        cur = np.stack([np.copy(colloids[i].pos) / self.box_length for i in reference_ids])
        keys = [str(np.copy(colloids[i].id)) for i in reference_ids]
        prev = np.stack([self._historic_positions[k] for k in keys])
        for k, p in zip(keys, cur):
            self._historic_positions[k] = p
        d_cur, d_prev = ops.list_field_distance(cur, prev, self.source)
        obs = self._delta(d_cur, d_prev)
        return np.asarray(obs, dtype=np.float32).reshape(-1, 1)
