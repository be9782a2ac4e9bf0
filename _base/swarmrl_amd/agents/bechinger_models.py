"""
Classical neighbour-rule agents of Bechinger's group (reference:
swarmrl/agents/bechinger_models.py).

The reference loops in Python over every agent and every other colloid
(get_colloids_in_vision, bechinger_models.py:156-171); here the neighbour
search and the sums the agents take over it run as one HIP kernel
(swarm_neighbor_reduce, fp64 like numpy), and the per-agent decisions are
vectorised.  Called with a Colloid list (the reference contract) they return
a list of Action; with a SwarmView they return DeviceActions and stay on the
GPU.
"""

import typing

import numpy as np
import torch

from swarmrl_amd.actions.actions import Action
from swarmrl_amd.agents.classical_agent import ClassicalAgent
from swarmrl_amd.engine import ops
from swarmrl_amd.engine.swarm_view import DeviceActions, is_view


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def _list_inputs(colloids):
    """[1, N, 3] device tensors (pos fp64, director, velocity) and types [N]."""
    dev = _device()
    pos = torch.as_tensor(np.stack([np.asarray(c.pos, dtype=float) for c in colloids]),
                          device=dev)[None]
    dirs = torch.as_tensor(np.stack([np.asarray(c.director, dtype=float) for c in colloids]),
                           device=dev)[None]
    vel = torch.as_tensor(np.stack([np.zeros(3) if getattr(c, "velocity", None) is None
                                    else np.asarray(c.velocity, dtype=float)
                                    for c in colloids]),
                          device=dev)[None]
    types = torch.as_tensor(np.array([int(c.type) for c in colloids], dtype=np.int32), device=dev)
    return pos, dirs, vel, types


def _view_inputs(view):
    return (view.positions(), view.directors().to(torch.float64),
            view.velocities().to(torch.float64), view.types)


def _all_types(types: torch.Tensor):
    return sorted(set(int(t) for t in torch.unique(types).cpu().tolist()))


def _agents_of(types_host: np.ndarray, acts_on_types) -> np.ndarray:
    return np.nonzero(np.isin(types_host, np.asarray(acts_on_types)))[0].astype(np.int32)


class Lavergne2019(ClassicalAgent):
    """
    Perception-threshold swimmers (Lavergne et al., Science 2019;
    bechinger_models.py:9-50): a colloid of an acting type swims with
    act_force when sum 1 / (2 pi |d|) over the colloids in its vision cone
    reaches perception_threshold.
    """

    def __init__(self, vision_half_angle=np.pi / 2.0, act_force=1, perception_threshold=1,
                 acts_on_types: typing.List[int] = None):
        self.vision_half_angle = vision_half_angle
        self.act_force = act_force
        self.perception_threshold = perception_threshold
        if acts_on_types is None:
            acts_on_types = [0]
        self.acts_on_types = acts_on_types

    def supports_device(self) -> bool:
        return True

    def _perception(self, pos, dirs, types, agents):
        sums = ops.neighbor_reduce(pos, dirs, None, types, agents, _all_types(types), np.inf,
                                   self.vision_half_angle)
        return sums[..., ops.NB_PERCEPTION]

    def calc_action(self, colloids):
        if is_view(colloids):
            pos, dirs, _, types = _view_inputs(colloids)
            agents = colloids.indices_of_type(self.acts_on_types[0]) \
                if len(self.acts_on_types) == 1 else torch.as_tensor(
                    _agents_of(colloids.engine._types_host, self.acts_on_types),
                    device=colloids.device)
            perc = self._perception(pos, dirs, types, agents)
            E, N = colloids.n_envs, colloids.n_particles
            f = torch.zeros((E, N), dtype=torch.float32, device=colloids.device)
            on = (perc >= self.perception_threshold).to(torch.float32) * float(self.act_force)
            f[:, agents.long()] = on
            return DeviceActions(f, torch.zeros_like(f))
        pos, dirs, _, types = _list_inputs(colloids)
        agents_h = _agents_of(types.cpu().numpy(), self.acts_on_types)
        perc = self._perception(pos, dirs, types, torch.as_tensor(agents_h, device=pos.device))
        perc = perc[0].cpu().numpy()
        actions = [Action() for _ in colloids]
        for k, i in enumerate(agents_h):
            if perc[k] >= self.perception_threshold:
                actions[i] = Action(force=self.act_force)
        return actions


class Baeuerle2020(ClassicalAgent):
    """
    Cohesion/alignment rule (Baeuerle et al., Nat. Commun. 2020;
    bechinger_models.py:53-153): turn towards the centre of mass of the
    colloids in the position cone, offset by +-angular_deviation towards the
    mean orientation of the colloids in the orientation cone (plus self);
    torque_z = act_torque sin(angle difference), force = act_force.  No
    neighbour in either cone: Action().
    """

    def __init__(self, act_force=1.0, act_torque=1, detection_radius_position=1.0,
                 detection_radius_orientation=1.0, vision_half_angle=np.pi / 2.0,
                 angular_deviation=1, acts_on_types: typing.List[int] = None):
        self.act_force = act_force
        self.act_torque = act_torque
        self.detection_radius_position = detection_radius_position
        self.detection_radius_orientation = detection_radius_orientation
        self.vision_half_angle = vision_half_angle
        self.angular_deviation = angular_deviation
        if acts_on_types is None:
            acts_on_types = [0]
        self.acts_on_types = acts_on_types

    def supports_device(self) -> bool:
        return True

    def _decide(self, pos, dirs, types, agents):
        """(active [E, A] bool, torque_z [E, A]) on the device, fp64."""
        cand = _all_types(types)
        sp = ops.neighbor_reduce(pos, dirs, None, types, agents, cand,
                                 self.detection_radius_position, self.vision_half_angle)
        so = ops.neighbor_reduce(pos, dirs, None, types, agents, cand,
                                 self.detection_radius_orientation, self.vision_half_angle)
        cnt_p, cnt_o = sp[..., ops.NB_COUNT], so[..., ops.NB_COUNT]
        to_com = sp[..., ops.NB_SUM_D:ops.NB_SUM_D + 3] / cnt_p.clamp(min=1.0)[..., None]
        to_com_angle = torch.atan2(to_com[..., 1], to_com[..., 0])
        own = dirs[:, agents.long()].to(torch.float64)
        mean_o = so[..., ops.NB_SUM_DIR:ops.NB_SUM_DIR + 3] + own
        mean_o = mean_o / (cnt_o + 1.0)[..., None]
        mean_o = mean_o / torch.linalg.norm(mean_o, dim=-1, keepdim=True)
        cands = torch.stack([to_com_angle + self.angular_deviation,
                             to_com_angle - self.angular_deviation], dim=-1)
        vecs = torch.stack([torch.cos(cands), torch.sin(cands), torch.zeros_like(cands)], dim=-1)
        dev = torch.arccos((vecs * mean_o[..., None, :]).sum(-1))
        # argmin, first minimum on ties (np.argmin); NaN is never smaller
        pick = torch.where(dev[..., 1] < dev[..., 0], 1, 0)
        target = torch.gather(cands, -1, pick[..., None])[..., 0]
        current = torch.atan2(own[..., 1], own[..., 0])
        diff = target - current
        diff = torch.where(diff >= np.pi, diff - 2 * np.pi, diff)
        diff = torch.where(diff <= -np.pi, diff + 2 * np.pi, diff)
        active = (cnt_p > 0) & (cnt_o > 0)
        return active, torch.sin(diff) * self.act_torque

    def calc_action(self, colloids):
        if is_view(colloids):
            pos, dirs, _, types = _view_inputs(colloids)
            agents = torch.as_tensor(_agents_of(colloids.engine._types_host, self.acts_on_types),
                                     device=colloids.device)
            active, tz = self._decide(pos, dirs, types, agents)
            E, N = colloids.n_envs, colloids.n_particles
            f = torch.zeros((E, N), dtype=torch.float32, device=colloids.device)
            t = torch.zeros_like(f)
            f[:, agents.long()] = active.to(torch.float32) * float(self.act_force)
            t[:, agents.long()] = torch.where(active, tz, torch.zeros_like(tz)).to(torch.float32)
            return DeviceActions(f, t)
        pos, dirs, _, types = _list_inputs(colloids)
        agents_h = _agents_of(types.cpu().numpy(), self.acts_on_types)
        active, tz = self._decide(pos, dirs, types, torch.as_tensor(agents_h, device=pos.device))
        active, tz = active[0].cpu().numpy(), tz[0].cpu().numpy()
        actions = [Action() for _ in colloids]
        for k, i in enumerate(agents_h):
            if active[k]:
                actions[i] = Action(force=self.act_force, torque=np.array([0, 0, tz[k]]))
        return actions


def get_colloids_in_vision(coll, other_coll, vision_half_angle=np.pi, vision_range=np.inf) -> list:
    """bechinger_models.py:156-171: the colloids of other_coll within
    vision_range and inside the cone of coll's director (fp64 device
    tensors; the agents above use the fused neighbour kernel instead)."""
    if len(other_coll) == 0:
        return []
    dev = _device()
    my_pos = torch.as_tensor(np.asarray(coll.pos, dtype=float), device=dev)
    my_dir = torch.as_tensor(np.asarray(coll.director, dtype=float), device=dev)
    pos = torch.as_tensor(np.stack([np.asarray(c.pos, dtype=float) for c in other_coll]),
                          device=dev)
    d = pos - my_pos
    dn = torch.linalg.norm(d, dim=1)
    in_range = dn < vision_range
    in_cone = torch.arccos((d / dn[:, None]) @ my_dir) < vision_half_angle
    keep = (in_range & in_cone).cpu().numpy()
    return [c for c, k in zip(other_coll, keep) if k]


def angle_from_vector(vec) -> float:
    return np.arctan2(vec[1], vec[0])


def vector_from_angle(angle) -> np.ndarray:
    return np.array([np.cos(angle), np.sin(angle), 0])
