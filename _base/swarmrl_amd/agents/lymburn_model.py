"""
Lymburn flocking/predator model (reference: swarmrl/agents/lymburn_model.py).

Alignment, repulsion, homing, friction and predator-escape forces of every
non-predator colloid; the neighbour sums (within the detection radii, no
cone) come from the fused HIP neighbour kernel (swarm_neighbor_reduce,
fp64).  Returns one Action(force=|F|, new_direction=F/|F|) per non-predator
colloid, in order, predators skipped (as the reference does).
"""

import numpy as np
import torch

from swarmrl_amd.actions.actions import Action
from swarmrl_amd.agents.bechinger_models import _list_inputs
from swarmrl_amd.agents.classical_agent import ClassicalAgent
from swarmrl_amd.engine import ops


class Lymburn(ClassicalAgent):
    def __init__(self, force_params: dict, detection_radius_position_colls=np.inf,
                 detection_radius_position_pred=np.inf, home_pos=np.array([500, 500, 0]),
                 agent_speed=10, predator_type: int = 1):
        self.force_params = force_params
        self.detection_radius_position_colls = detection_radius_position_colls
        self.detection_radius_position_pred = detection_radius_position_pred
        self.home_pos = home_pos
        self.predator_type = predator_type
        self.agent_speed = agent_speed

    def update_force_params(self, K_a=None, K_r=None, K_h=None, K_f=None, K_p=None):
        update_params = {"K_a": K_a, "K_r": K_r, "K_h": K_h, "K_f": K_f, "K_p": K_p}
        for key, value in update_params.items():
            if value is not None:
                self.force_params[key] = value

    def calc_action(self, colloids):
        pos, dirs, vel, types = _list_inputs(colloids)
        th = types.cpu().numpy()
        agents_h = np.nonzero(th != self.predator_type)[0].astype(np.int32)
        if len(agents_h) == 0:
            return []
        agents = torch.as_tensor(agents_h, device=pos.device)
        others = sorted(set(int(t) for t in th) - {int(self.predator_type)})
        sc = ops.neighbor_reduce(pos, dirs, vel, types, agents, others,
                                 self.detection_radius_position_colls, -1.0)[0].cpu().numpy()
        sp = ops.neighbor_reduce(pos, dirs, vel, types, agents, [self.predator_type],
                                 self.detection_radius_position_pred, -1.0)[0].cpu().numpy()
        P = pos[0].cpu().numpy()
        V = vel[0].cpu().numpy().astype(float)
        K = self.force_params
        actions = []
        for k, i in enumerate(agents_h):
            x, v = P[i], V[i]
            cnt = sc[k, ops.NB_COUNT]
            force_a, force_r = np.zeros(3), np.zeros(3)
            if cnt > 0:
                force_a = sc[k, ops.NB_SUM_V:ops.NB_SUM_V + 3] - cnt * v
                force_r = sc[k, ops.NB_SUM_D:ops.NB_SUM_D + 3] / np.sqrt(sc[k, ops.NB_SUM_D2])
            force_h = self.home_pos - x
            force_p = np.zeros(3)
            if sp[k, ops.NB_COUNT] > 0:
                force_p = -sp[k, ops.NB_SUM_D:ops.NB_SUM_D + 3] / np.sqrt(sp[k, ops.NB_SUM_D2])
            force_f = -v * (np.abs(v) - self.agent_speed) / self.agent_speed
            force = (K["K_a"] * force_a + K["K_r"] * force_r + K["K_h"] * force_h
                     + K["K_p"] * force_p + K["K_f"] * force_f)
            mag = np.linalg.norm(force)
            actions.append(Action(force=mag, new_direction=force / mag))
        return actions
