"""
Episode-parallel rollout plumbing: the exchange of trajectory buffers
between ranks at the end of an episode, and the replicated update built on it.

The reference runs independent trainings as separate Dask worker processes
and never exchanges trajectories (swarmrl/training_routines/
ensemble_submit.py:76-138).  Here every rank (one process per GPU) runs its
own envs with no communication during the rollout; at the end of an episode
the per-rank trajectory buffers are concatenated on every rank, and every
rank runs the identical update on the gathered episode:
the replicas start from rank 0's parameters (``broadcast_agent``) and each
update is a deterministic function of the gathered data, so they stay
bit-identical with no gradient all-reduce or parameter broadcast per episode
(``replicated_update``; tests/test_distributed.py checks the parameters of
two gloo ranks after two updates).

The four buffers (features, actions, log-probs, rewards) plus the kill flag
are packed into ONE flat byte buffer and exchanged with ONE
all_gather_into_tensor (RCCL over xGMI for backend "nccl", gloo on CPU): a
ring all-gather is bound per xGMI link, so one large collective per episode
beats five small ones.
"""

from __future__ import annotations

import os
import time
from typing import Dict, Optional, Sequence

import torch
import torch.distributed as dist

from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

_NAMES = ("features", "actions", "log_probs", "rewards")


def shard_envs(total_envs: int, rank: int, world: int):
    """Env ids owned by a rank: one contiguous block, rank r of G owning
    envs [r E, (r + 1) E) with E = total / G (the first total mod G ranks one
    more).  Contiguous blocks, not SURVEY 8(e)'s e mod G: the all-gather
    below concatenates the ranks' [T, E, ...] buffers rank-major, so the
    gathered env axis is then the global env id (gather_trajectory pads
    uneven blocks).  bench.py creates each rank's engine with seed 42 + its
    first env id, so env g is placed with default_rng(42 + g) whatever the
    world size."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside a world of {world}")
    per, extra = divmod(total_envs, world)
    lo = rank * per + min(rank, extra)
    return list(range(lo, lo + per + (1 if rank < extra else 0)))


_FORCE_COLLECTIVE = [False]


def force_collectives(flag: bool = True) -> None:
    """Run every collective of this module even in a world of one process
    (a world-size-1 RCCL group then executes the real device-tensor
    all-gather, broadcast and all-reduce on one GPU: the path N GPUs take,
    minus the transfers; tests/test_gpu_rccl.py, bench.py
    --force-collective).  Also on with SWARMRL_AMD_FORCE_COLLECTIVE=1."""
    _FORCE_COLLECTIVE[0] = bool(flag)


def _is_distributed(group=None) -> bool:
    if not (dist.is_available() and dist.is_initialized()):
        return False
    if dist.get_world_size(group) > 1:
        return True
    return _FORCE_COLLECTIVE[0] or os.environ.get("SWARMRL_AMD_FORCE_COLLECTIVE", "0") == "1"


def _as_tensor(x, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device)
    return torch.as_tensor(x, device=device)


def _stacked(trajectory) -> Dict[str, torch.Tensor]:
    dev = None
    for x in trajectory.features:
        if isinstance(x, torch.Tensor):
            dev = x.device
            break
    dev = dev or torch.device("cpu")
    return {k: torch.stack([_as_tensor(x, dev) for x in getattr(trajectory, k)])
            for k in _NAMES}


def _killed_flag(killed, device) -> torch.Tensor:
    """The kill switch as one uint8 on `device` (no host sync for a tensor)."""
    if isinstance(killed, torch.Tensor):
        return killed.reshape(-1).any().to(device=device, dtype=torch.uint8).reshape(1)
    return torch.tensor([1 if killed else 0], dtype=torch.uint8, device=device)


def _env_counts(bufs, group, env_counts: Optional[Sequence[int]]) -> list:
    """Env count of every rank: given by the caller (shard_envs: the packed
    all-gather is then the episode's only collective), or exchanged with a
    small all-gather on every call -- every rank takes the same branch, so
    the collectives always match (a per-rank cache could let one rank skip
    the count exchange while another runs it)."""
    world = dist.get_world_size(group)
    if env_counts is not None:
        if len(env_counts) != world:
            raise ValueError(f"env_counts has {len(env_counts)} entries for a world of {world}")
        return [int(c) for c in env_counts]
    dev = bufs["actions"].device
    mine = torch.tensor([bufs["actions"].shape[1]], dtype=torch.int64, device=dev)
    allc = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, mine, group=group)
    return [int(c) for c in allc.cpu()]


def gather_trajectory(trajectory, group=None, stats: Optional[dict] = None,
                      env_counts: Optional[Sequence[int]] = None) -> Dict[str, torch.Tensor]:
    """
    Stack an agent's device trajectory (lists of [E, A, ...] tensors, one entry
    per slice) into [T, E, ...] tensors and all-gather them along the env axis
    -> [T, sum(E), ...] on every rank (rank-major env order), plus "killed":
    whether any rank's task raised the kill switch (a bool on the host when
    not distributed, else a uint8 device tensor).

    Ranks may hold different env counts (shard_envs of a total that the
    world does not divide): each rank's block is padded to the largest count
    for the collective and the padding dropped after it.

    stats (optional dict): receives "bytes" (this rank's packed buffer) and
    the collective's duration: "ms" on the host (CPU tensors) or "events"
    (a pair of timing events on the current stream; read them with
    gather_ms after synchronising).
    """
    bufs = _stacked(trajectory)
    if not _is_distributed(group):
        bufs["killed"] = trajectory.killed
        return bufs
    world = dist.get_world_size(group)
    counts = _env_counts(bufs, group, env_counts)
    if counts[dist.get_rank(group)] != bufs["actions"].shape[1]:
        raise ValueError("env_counts does not match this rank's trajectory")
    emax = max(counts)
    dev = bufs["actions"].device
    padded = {}
    for k in _NAMES:
        b = bufs[k]
        if b.shape[1] < emax:
            pad = torch.zeros((b.shape[0], emax - b.shape[1]) + tuple(b.shape[2:]), dtype=b.dtype,
                              device=dev)
            b = torch.cat([b, pad], 1)
        padded[k] = b
    parts = [padded[k].contiguous().reshape(-1).view(torch.uint8) for k in _NAMES]
    parts.append(_killed_flag(trajectory.killed, dev))
    sizes = [p.numel() for p in parts]
    packed = torch.cat(parts)
    out = torch.empty(world * packed.numel(), dtype=torch.uint8, device=dev)
    if stats is None:
        dist.all_gather_into_tensor(out, packed, group=group)
    elif packed.is_cuda:
        # events on the current stream (no host synchronisation): ev0 fires
        # when the episode's work is done, ev1 once the collective is
        stats["bytes"] = int(packed.numel())
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        dist.all_gather_into_tensor(out, packed, group=group, async_op=True).wait()
        ev1.record()
        stats["events"] = (ev0, ev1)
    else:
        stats["bytes"] = int(packed.numel())
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(out, packed, group=group)
        stats["ms"] = (time.perf_counter() - t0) * 1e3
    per_rank = out.view(world, packed.numel())
    result = {}
    off = 0
    for name, sz in zip(_NAMES, sizes):
        src = padded[name]
        # a fresh copy: .contiguous() keeps a one-rank slice as a view with
        # the packed row's stride, which cannot be reinterpreted as src.dtype
        # (found by the world-1 RCCL test, tests/test_gpu_rccl.py)
        chunk = per_rank[:, off:off + sz].clone(memory_format=torch.contiguous_format)
        chunk = chunk.view(src.dtype)
        chunk = chunk.view(world, *src.shape)  # [world, T, Emax, ...]
        if all(c == emax for c in counts):
            result[name] = chunk.transpose(0, 1).reshape(src.shape[0], world * emax,
                                                         *src.shape[2:])
        else:
            result[name] = torch.cat([chunk[r, :, :counts[r]] for r in range(world)], 1)
        off += sz
    result["killed"] = per_rank[:, off].amax()
    return result


def gather_episode(trajectory, group=None, stats: Optional[dict] = None,
                   env_counts: Optional[Sequence[int]] = None) -> TrajectoryInformation:
    """The episode of every rank as one TrajectoryInformation: per slice one
    [sum(E), A, ...] tensor (views into the gathered buffers), the kill
    switch raised when any rank raised it."""
    g = gather_trajectory(trajectory, group=group, stats=stats, env_counts=env_counts)
    return TrajectoryInformation(
        particle_type=trajectory.particle_type,
        features=list(g["features"].unbind(0)),
        actions=list(g["actions"].unbind(0)),
        log_probs=list(g["log_probs"].unbind(0)),
        rewards=list(g["rewards"].unbind(0)),
        killed=g["killed"],
    )


def gather_ms(stats: dict) -> float:
    """Duration of a gather recorded with stats (after synchronisation)."""
    if "events" in stats:
        ev0, ev1 = stats["events"]
        return float(ev0.elapsed_time(ev1))
    return float(stats.get("ms", 0.0))


# ------------------------------------------------------- replicated update
def _agent_tensors(agent):
    """Every tensor that determines an agent's future updates: the network's
    parameters and buffers, its optimizer's state, and those of an intrinsic
    reward (RND target / predictor and its optimizer), in a fixed order."""
    out = []

    def add_module(m):
        out.extend(t for t in m.state_dict().values() if isinstance(t, torch.Tensor))

    def add_optimizer(opt):
        if opt is None:
            return
        for group in opt.param_groups:
            for p in group["params"]:
                for k in sorted(opt.state.get(p, {})):
                    v = opt.state[p][k]
                    if isinstance(v, torch.Tensor):
                        out.append(v)

    net = getattr(agent, "network", None)
    if net is not None and getattr(net, "model", None) is not None:
        add_module(net.model)
        add_optimizer(getattr(net, "optimizer", None))
    ir = getattr(agent, "intrinsic_reward", None)
    if ir is not None:
        for name in ("target_network", "predictor_network"):
            if getattr(ir, name, None) is not None:
                add_module(getattr(ir, name))
        add_optimizer(getattr(ir, "optimizer", None))
    return out


@torch.no_grad()
def broadcast_agent(agent, src: int = 0, group=None) -> None:
    """Make every rank's replica of `agent` equal to rank `src`'s (group
    rank): parameters, buffers and optimizer state, broadcast in place.  Run
    once before the first episode (EpisodeParallelTrainer)."""
    if not _is_distributed(group):
        return
    root = src if group is None else dist.get_global_rank(group, src)
    dev = _collective_device(group)
    for t in _agent_tensors(agent):
        if t.device == dev or dev.type == "cpu":
            dist.broadcast(t, root, group=group)
        else:
            # RCCL only moves device tensors: a host-side state tensor (e.g. a
            # non-capturable optimizer's step counter) goes through a device
            # copy
            tmp = t.detach().to(dev)
            dist.broadcast(tmp, root, group=group)
            t.copy_(tmp.to(t.device))


def _collective_device(group=None) -> torch.device:
    """Where the group's collectives take their tensors: the current GPU for
    an RCCL ("nccl") group, the host otherwise."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def any_rank(flag: bool, group=None) -> bool:
    """True on every rank when `flag` is true on any rank (one small
    all-reduce; the flag itself when not distributed)."""
    if not _is_distributed(group):
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=_collective_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


@torch.no_grad()
def replica_checksum(agent, device=None) -> torch.Tensor:
    """A cheap fingerprint of _agent_tensors on `device`: per tensor the sum
    of its 32-bit words (int64, wrapping) and a position-weighted sum of
    them -- equal replicas give equal checksums, and a drifted bit changes
    them (replicas check each other with it, _ReplicatedUpdate)."""
    sums = []
    for t in _agent_tensors(agent):
        x = t.detach().reshape(-1).contiguous()
        if device is not None:
            x = x.to(device)
        b = x.view(torch.uint8)
        pad = (-b.numel()) % 4
        if pad:
            b = torch.cat([b, torch.zeros(pad, dtype=torch.uint8, device=b.device)])
        w = b.view(torch.int32).to(torch.int64)
        pos = torch.arange(1, w.numel() + 1, dtype=torch.int64, device=w.device)
        sums.append(torch.stack([w.sum(), (w * pos).sum()]))
    if not sums:
        return torch.zeros(0, dtype=torch.int64, device=device)
    return torch.cat(sums)


def replicas_match(agent, group=None) -> bool:
    """Whether every rank's replica of `agent` has the same checksum (one
    all-gather of a few int64 per tensor)."""
    if not _is_distributed(group):
        return True
    dev = _collective_device(group)
    mine = replica_checksum(agent, dev)
    world = dist.get_world_size(group)
    allc = torch.empty(world * mine.numel(), dtype=mine.dtype, device=dev)
    dist.all_gather_into_tensor(allc, mine, group=group)
    allc = allc.view(world, -1)
    return bool((allc == allc[0:1]).all().item())


@torch.no_grad()
def replica_digest(agent) -> torch.Tensor:
    """The bytes of every tensor of _agent_tensors as one uint8 vector on the
    host (tests: replicas are identical iff their digests are)."""
    parts = [t.detach().reshape(-1).contiguous().cpu().view(torch.uint8)
             for t in _agent_tensors(agent)]
    return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8)


def replicated_update(agent, episode: TrajectoryInformation, seed: int):
    """One learning agent's update on a gathered episode, run identically
    on every rank: the loss (ProximalPolicyLoss.compute_loss, deterministic:
    the fused HIP gradient sums in a fixed order, tests/test_gpu_ppo.py) and
    an intrinsic reward's predictor update, whose minibatch permutation
    (random_network_distillation.py:105-120) draws from torch's generators,
    here re-seeded with `seed` (the same on every rank) inside a forked RNG
    state so the rollout's own streams are untouched."""
    devices = []
    for t in episode.features[:1]:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            devices = [t.device.index]
    agent.loss.compute_loss(network=agent.network, episode_data=episode)
    if getattr(agent, "intrinsic_reward", None):
        with torch.random.fork_rng(devices=devices):
            torch.manual_seed(seed)
            agent.intrinsic_reward.update(episode)
