"""
Helpers of the reference's utils module that lie on the hot path
(reference: swarmrl/utils/utils.py).
"""

import numpy as np


def get_random_angles(rng: np.random.Generator):
    """utils.py:19-21."""
    return np.arccos(2.0 * rng.random() - 1), 2.0 * np.pi * rng.random()


def vector_from_angles(theta, phi):
    """utils.py:24-27."""
    return np.array(
        [np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi), np.cos(theta)]
    )


def angles_from_vector(director):
    """utils.py:30-34."""
    director = np.asarray(director, dtype=float)
    director = director / np.linalg.norm(director)
    theta = np.arccos(director[2])
    phi = np.arctan2(director[1], director[0])
    return theta, phi


def create_colloids(n_cols: int, type_: int = 0, center=np.array([500, 500, 0]),
                    dist: float = 200.0, face_middle: bool = False):
    """Colloids on a circle (utils.py:335-377)."""
    from swarmrl_amd.components.colloid import Colloid

    cols = []
    for i in range(n_cols):
        theta = np.random.random(1)[0] * 2 * np.pi
        position = center + dist * np.array([np.cos(theta), np.sin(theta), 0])
        if face_middle:
            direction = -position / np.linalg.norm(position)
        else:
            direction = np.random.random(3)
            direction[-1] = 0
            direction = direction / np.linalg.norm(direction)
        cols.append(Colloid(pos=position, director=direction, type=type_, id=i))
    return cols
