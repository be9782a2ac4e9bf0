"""
Episode-parallel rollout plumbing: device trajectory buffers and their
exchange between ranks.

The reference runs independent trainings as separate Dask worker processes
and never exchanges trajectories (swarmrl/training_routines/
ensemble_submit.py:76-138).  Here every rank (one process per GPU) runs its
own envs with no communication during the rollout; at the end of an episode
the per-rank trajectory buffers are concatenated on every rank with one
all_gather (RCCL over xGMI for backend "nccl", gloo on CPU) so each rank can
run the identical PPO update.

``EpisodeRecorder`` keeps [T, E, A, ...] ring buffers on the device and
advances its slot with a device-side counter, so the whole slice (observable,
policy, physics, reward, recording) can be captured once into a HIP graph and
replayed.
"""

from __future__ import annotations

from typing import Dict

import torch
import torch.distributed as dist


class EpisodeRecorder:
    """Device ring buffers for one agent type: features, actions, log-probs, rewards."""

    def __init__(self, episode_length: int, n_envs: int, n_agents: int, obs_shape,
                 device: torch.device):
        T, E, A = episode_length, n_envs, n_agents
        self.T = T
        self.features = torch.zeros((T, E, A, *obs_shape), dtype=torch.float32, device=device)
        self.actions = torch.zeros((T, E, A), dtype=torch.int64, device=device)
        self.log_probs = torch.zeros((T, E, A), dtype=torch.float32, device=device)
        self.rewards = torch.zeros((T, E, A), dtype=torch.float32, device=device)
        self._slot_a = torch.zeros(1, dtype=torch.int64, device=device)
        self._slot_r = torch.zeros(1, dtype=torch.int64, device=device)

    def record_action(self, features, actions, log_probs):
        self.features.index_copy_(0, self._slot_a, features.reshape(self.features.shape[1:]).unsqueeze(0))
        self.actions.index_copy_(0, self._slot_a, actions.reshape(self.actions.shape[1:]).unsqueeze(0))
        self.log_probs.index_copy_(0, self._slot_a,
                                   log_probs.reshape(self.log_probs.shape[1:]).unsqueeze(0))
        self._slot_a.add_(1).remainder_(self.T)

    def record_reward(self, rewards):
        self.rewards.index_copy_(0, self._slot_r, rewards.reshape(self.rewards.shape[1:]).unsqueeze(0))
        self._slot_r.add_(1).remainder_(self.T)

    def buffers(self) -> Dict[str, torch.Tensor]:
        return {
            "features": self.features,
            "actions": self.actions,
            "log_probs": self.log_probs,
            "rewards": self.rewards,
        }


def gather_episode(recorder: EpisodeRecorder, group=None) -> Dict[str, torch.Tensor]:
    """
    All-gather every trajectory buffer along the env axis: each [T, E, ...]
    buffer becomes [T, world * E, ...] on every rank (rank-major env order).
    One flat all_gather per buffer; without an initialised process group the
    local buffers are returned unchanged.
    """
    bufs = recorder.buffers()
    if not (dist.is_available() and dist.is_initialized()):
        return bufs
    world = dist.get_world_size(group)
    out = {}
    for name, t in bufs.items():
        t = t.contiguous()
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        out[name] = torch.cat(parts, dim=1)
    return out


def shard_envs(total_envs: int, rank: int, world: int):
    """Env ids owned by a rank: e with e mod world == rank."""
    return [e for e in range(total_envs) if e % world == rank]


def gather_trajectory(trajectory, group=None) -> Dict[str, torch.Tensor]:
    """
    Stack an agent's device trajectory (lists of [E, A, ...] tensors, one entry
    per slice) into [T, E, ...] tensors and all-gather them along the env axis
    -> [T, world * E, ...] on every rank.
    """
    bufs = {
        "features": torch.stack(list(trajectory.features)),
        "actions": torch.stack(list(trajectory.actions)),
        "log_probs": torch.stack(list(trajectory.log_probs)),
        "rewards": torch.stack(list(trajectory.rewards)),
    }
    if not (dist.is_available() and dist.is_initialized()):
        return bufs
    world = dist.get_world_size(group)
    out = {}
    for name, t in bufs.items():
        t = t.contiguous()
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        out[name] = torch.cat(parts, dim=1)
    return out
