"""
Subdivided vision cones (reference:
swarmrl/observables/subdivided_vision_cones.py:17-258).

For every agent i of ``particle_type`` and every colloid j the reference adds
``min(1, 2 r_j / d)`` into cone k and type slot t when j is closer than
``vision_range`` (unwrapped positions, no minimum image, line 116) and the
signed angle between i's director and the direction to j lies strictly
inside cone k (lines 138-153, utils.py:297-332).  Self and coincident
colloids contribute nothing (the reference gets NaN angles there).  Here the
reduction runs in the HIP kernel ``k_vision`` through the C ABI
(swarm_vision_cone); sums are exact (int64 fixed point) and rounded once.
"""

from typing import List

import numpy as np

from swarmrl_amd.engine import ops
from swarmrl_amd.engine.swarm_view import is_view
from swarmrl_amd.observables.observable import Observable


class SubdividedVisionCones(Observable):
    """Camera-like observable of the other colloids in angular sectors."""

    supports_device = True

    def __init__(
        self,
        vision_range: float,
        vision_half_angle: float,
        n_cones: int,
        radii: List[float],
        detected_types=None,
        particle_type: int = 0,
    ):
        super().__init__(particle_type=particle_type)
        self.vision_range = vision_range
        self.vision_half_angle = vision_half_angle
        self.n_cones = n_cones
        self.radii = radii
        self.detected_types = detected_types
        self._radii_device = None
        self._vp = None

    def _detect_all_things_to_see(self, types):
        """Sorted unique types present (subdivided_vision_cones.py:62-81)."""
        all_types = []
        for t in types:
            if t not in all_types:
                all_types.append(t)
        self.detected_types = np.array(np.sort(all_types))

    def _params(self):
        if self._vp is None:
            self._vp = ops.vision_params(
                self.vision_range, self.vision_half_angle, self.n_cones, self.detected_types
            )
        return self._vp

    def compute_single_observable(self, index: int, colloids) -> np.ndarray:
        """Vision cones of one colloid, shape (n_cones, n_detected_types)."""
        return self._compute_list([index], colloids)[0]

    def _compute_list(self, indices, colloids):
        types = np.array([int(c.type) for c in colloids])
        if self.detected_types is None:
            self._detect_all_things_to_see(types)
        pos = np.stack([np.asarray(c.pos, dtype=float) for c in colloids])
        dirs = np.stack([np.asarray(c.director, dtype=float) for c in colloids])
        out = ops.list_vision_cone(
            pos, dirs, types, indices, np.asarray(self.radii, dtype=np.float32),
            self.vision_range, self.vision_half_angle, self.n_cones, self.detected_types,
        )
        return [out[k] for k in range(len(indices))]

    def compute_observable(self, colloids):
        """
        List input: list of (n_cones, n_types) arrays, one per agent (as the
        reference).  SwarmView input: device tensor [E, A, n_cones, n_types].
        """
        if is_view(colloids):
            view = colloids
            if self.detected_types is None:
                self._detect_all_things_to_see(view.engine._types_host.tolist())
            if self._radii_device is None:
                import torch

                self._radii_device = torch.as_tensor(
                    np.asarray(self.radii, dtype=np.float32), device=view.device
                )
            # agents (cached by the view), radii (cached here) and types (the
            # engine's) outlive the engine's use of them: persistent call
            agents = view.indices_of_type(self.particle_type)
            return ops.vision_cone(
                view.engine._native, view.n_envs, agents, self._radii_device, view.types,
                self._params(), persistent=True,
            )
        reference_ids = self.get_colloid_indices(colloids)
        if len(reference_ids) == 0:
            return []
        return self._compute_list(reference_ids, colloids)
