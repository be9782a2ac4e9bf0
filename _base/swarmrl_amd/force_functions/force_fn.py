"""
Bridge between agents and the engine (reference:
swarmrl/force_functions/force_fn.py:13-106).

``calc_action`` fans out per particle type to the agents and merges their
actions in colloid order; colloids without an agent get ``Action()``; the
kill switch is the OR of the agents' switches.  With a SwarmView (device
path) the same merge is done on device tensors and a ``DeviceActions`` of
shape [E, N] is returned.
"""


import numpy as np
import torch

from swarmrl_amd.actions.actions import Action
from swarmrl_amd.engine.swarm_view import DeviceActions, is_view


class ForceFunction:
    """Class to bridge agents with an engine."""

    _kill_switch: bool = False

    def __init__(self, agents: dict):
        super().__init__()
        self.agents = agents
        self.particle_types = [type_ for type_ in self.agents]

    @property
    def kill_switch(self):
        return self._kill_switch

    @kill_switch.setter
    def kill_switch(self, value):
        self._kill_switch = value

    def absorbs_build(self) -> bool:
        """True when an agent's device calc_action carries a deferred cluster
        build along in its launches (ActorCriticAgent.absorbs_build)."""
        return any(getattr(a, "absorbs_build", lambda: False)() for a in self.agents.values())

    def supports_device(self) -> bool:
        """True when every agent can act on a SwarmView (the GPU fast path)."""
        if len(self.agents) == 0:
            return False
        for agent in self.agents.values():
            fn = getattr(agent, "supports_device", None)
            if not (fn and fn()):
                return False
        return True

    def calc_action(self, colloids):
        if is_view(colloids):
            return self._calc_action_device(colloids)
        actions = {int(np.copy(colloid.id)): Action() for colloid in colloids}
        switches = []
        for agent in self.agents:
            computed_actions = self.agents[agent].calc_action(colloids=colloids)
            switches.append(self.agents[agent].kill_switch)
            count = 0
            for colloid in colloids:
                if str(colloid.type) == agent:
                    actions[colloid.id] = computed_actions[count]
                    count += 1
        self.kill_switch = any(switches)
        return list(actions.values())

    def _calc_action_device(self, view) -> DeviceActions:
        E, N = view.n_envs, view.n_particles
        if len(self.agents) == 1:
            agent_type, agent = next(iter(self.agents.items()))
            if view.covers_all(int(agent_type)):
                # one agent acts on every colloid: its [E, N] actions are the
                # merged actions (no scatter needed)
                acts = agent.calc_action(colloids=view)
                self.kill_switch = bool(agent.kill_switch)
                return acts
        f = torch.zeros((E, N), dtype=torch.float32, device=view.device)
        tz = torch.zeros((E, N), dtype=torch.float32, device=view.device)
        new_dir = None
        new_mask = None
        switches = []
        for agent_type, agent in self.agents.items():
            idx = view.indices_of_type(int(agent_type)).long()
            acts = agent.calc_action(colloids=view)
            switches.append(agent.kill_switch)
            if idx.numel() == 0:
                continue
            f[:, idx] = acts.f_swim
            tz[:, idx] = acts.torque_z
            if acts.new_direction is not None:
                if new_dir is None:
                    new_dir = np.zeros((E, N, 3))
                    new_mask = np.zeros((E, N), dtype=bool)
                host_idx = idx.cpu().numpy()
                nd = np.broadcast_to(np.asarray(acts.new_direction, dtype=float),
                                     (E, len(host_idx), 3))
                m = acts.new_direction_mask
                m = np.ones((E, len(host_idx)), dtype=bool) if m is None else \
                    np.broadcast_to(m, (E, len(host_idx)))
                new_dir[:, host_idx] = nd
                new_mask[:, host_idx] = m
        self.kill_switch = any(switches)
        return DeviceActions(f, tz, new_dir, new_mask)

    def calc_reward(self, colloids, external_reward: float = 0.0) -> None:
        for agent in self.agents:
            self.agents[agent].calc_reward(colloids=colloids, external_reward=external_reward)


__all__ = ["ForceFunction"]
