"""
Colloid data class (reference: swarmrl/components/colloid.py:11-49).

Frozen dataclass with equality by ``id``.  The reference registers it as a
JAX pytree; JAX is not part of this stack, so that registration is omitted.
"""

import dataclasses

import numpy as np


@dataclasses.dataclass(frozen=True)
class Colloid:
    """Snapshot of one particle as seen by observables, tasks and agents."""

    pos: np.ndarray
    director: np.ndarray
    id: int
    velocity: np.ndarray = None
    type: int = 0

    def __repr__(self):
        return (
            f"Colloid(pos={self.pos}, director={self.director}, id={self.id},"
            f" velocity={self.velocity}, type={self.type})"
        )

    def __eq__(self, other):
        return self.id == other.id

    __hash__ = None
