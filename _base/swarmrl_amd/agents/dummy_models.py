"""
Constant-action agents (reference: swarmrl/agents/dummy_models.py:9-38).
On a SwarmView they return DeviceActions without leaving the GPU.
"""

import numpy as np
import torch

from swarmrl_amd.actions.actions import Action
from swarmrl_amd.agents.classical_agent import ClassicalAgent
from swarmrl_amd.engine.swarm_view import DeviceActions, is_view


def _const_actions(view, action: Action) -> DeviceActions:
    """The same action for every colloid, as broadcastable (1, 1) tensors."""
    tz = 0.0 if action.torque is None else float(np.asarray(action.torque, dtype=float)[2])
    f = torch.full((1, 1), float(action.force), dtype=torch.float32, device=view.device)
    t = torch.full((1, 1), tz, dtype=torch.float32, device=view.device)
    nd = None if action.new_direction is None else np.asarray(action.new_direction, dtype=float)
    return DeviceActions(f, t, nd)


class _ConstAgent(ClassicalAgent):
    def supports_device(self) -> bool:
        return True


class ConstForce(_ConstAgent):
    def __init__(self, force: float):
        self.action = Action(force=force)

    def calc_action(self, colloids):
        if is_view(colloids):
            return _const_actions(colloids, self.action)
        return len(colloids) * [self.action]


class ConstTorque(_ConstAgent):
    def __init__(self, torque: np.ndarray):
        self.action = Action(torque=torque)

    def calc_action(self, colloids):
        if is_view(colloids):
            return _const_actions(colloids, self.action)
        return len(colloids) * [self.action]


class ConstForceAndTorque(_ConstAgent):
    def __init__(self, force: float, torque: np.ndarray):
        self.action = Action(force=force, torque=torque)

    def calc_action(self, colloids):
        if is_view(colloids):
            return _const_actions(colloids, self.action)
        return len(colloids) * [self.action]


class ToConstDirection(_ConstAgent):
    def __init__(self, direction: np.ndarray):
        self.action = Action(new_direction=direction)

    def calc_action(self, colloids):
        if is_view(colloids):
            return _const_actions(colloids, self.action)
        return len(colloids) * [self.action]


