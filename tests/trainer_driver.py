"""
Test-only training driver.

The reference's trainers (swarmrl/trainers/continuous_trainer.py:22-89,
episodic_trainer.py:26-130) are callers of the engine, not part of the
replaced hot path: with this package they plug in unchanged.  The tests
need a loop of the same shape to exercise the device path end to end
(episode of `integrate(episode_length, force_fn)`, then every agent's
`update_agent`), so this is that loop and nothing more.
"""

import numpy as np
import torch

from swarmrl_amd.force_functions import ForceFunction


def _mean(values) -> float:
    if len(values) == 0:
        return 0.0
    if isinstance(values[0], torch.Tensor):
        return float(torch.stack([v.float() for v in values]).mean().item())
    return float(np.mean(values))


def continuous_training(engine, agents, n_episodes: int, episode_length: int) -> np.ndarray:
    """One engine, n_episodes episodes; returns [0, mean reward of episode 1, ...]."""
    by_type = {str(a.particle_type): a for a in agents}
    force_fn = ForceFunction(agents=by_type)
    for a in agents:
        a.reset_agent(engine.colloids)
    history = [0.0]
    for _ in range(n_episodes):
        engine.integrate(episode_length, force_fn)
        total, killed = 0.0, False
        for a in agents:
            rewards, k = a.update_agent()
            total += _mean(rewards)
            killed |= bool(k)
        history.append(total)
        if killed:
            engine.finalize()
            break
        force_fn = ForceFunction(agents=by_type)
    return np.array(history)
