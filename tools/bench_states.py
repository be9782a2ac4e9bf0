"""Seeded bench-like placements for the tools (the headline's disc at area
fraction 0.1): one oracle state per env."""
import numpy as np

from oracle import oracle


def disc_states(rng, n, L, E):
    out = []
    for _ in range(E):
        r = L / 2 * np.sqrt(rng.random(n))
        th = 2 * np.pi * rng.random(n)
        pos = np.stack([L / 2 + r * np.cos(th), L / 2 + r * np.sin(th), np.zeros(n)], 1)
        a = 2 * np.pi * rng.random(n)
        out.append(oracle.state_from_positions(pos, np.stack([np.cos(a), np.sin(a), 0 * a], 1),
                                               [L, L, L]))
    return out
