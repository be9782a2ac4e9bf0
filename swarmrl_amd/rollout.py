"""
Episode-parallel rollout plumbing: the exchange of trajectory buffers
between ranks at the end of an episode.

The reference runs independent trainings as separate Dask worker processes
and never exchanges trajectories (swarmrl/training_routines/
ensemble_submit.py:76-138).  Here every rank (one process per GPU) runs its
own envs with no communication during the rollout; at the end of an episode
the per-rank trajectory buffers are concatenated on every rank so each rank
can run the identical PPO update.

The four buffers (features, actions, log-probs, rewards) are packed into ONE
flat byte buffer and exchanged with ONE all_gather_into_tensor (RCCL over
xGMI for backend "nccl", gloo on CPU): a ring all-gather is bound per xGMI
link, so one large collective per episode beats four small ones.
"""

from __future__ import annotations

import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

_NAMES = ("features", "actions", "log_probs", "rewards")


def shard_envs(total_envs: int, rank: int, world: int):
    """Env ids owned by a rank: one contiguous block, rank r of G owning
    envs [r E, (r + 1) E) with E = total / G (the first total mod G ranks one
    more).  Contiguous blocks, not SURVEY 8(e)'s e mod G: the all-gather
    below concatenates the ranks' [T, E, ...] buffers rank-major, so the
    gathered env axis is then the global env id.  bench.py creates each
    rank's engine with seed 42 + its first env id, so env g is placed with
    default_rng(42 + g) whatever the world size."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside a world of {world}")
    per, extra = divmod(total_envs, world)
    lo = rank * per + min(rank, extra)
    return list(range(lo, lo + per + (1 if rank < extra else 0)))


def _stacked(trajectory) -> Dict[str, torch.Tensor]:
    return {
        "features": torch.stack(list(trajectory.features)),
        "actions": torch.stack(list(trajectory.actions)),
        "log_probs": torch.stack(list(trajectory.log_probs)),
        "rewards": torch.stack(list(trajectory.rewards)),
    }


def gather_trajectory(trajectory, group=None, stats: Optional[dict] = None
                      ) -> Dict[str, torch.Tensor]:
    """
    Stack an agent's device trajectory (lists of [E, A, ...] tensors, one entry
    per slice) into [T, E, ...] tensors and all-gather them along the env axis
    -> [T, world * E, ...] on every rank (rank-major env order).

    stats (optional dict): receives "bytes" (this rank's packed buffer) and
    the collective's duration: "ms" on the host (CPU tensors) or "events"
    (a pair of timing events on the current stream; read them with
    gather_ms after synchronising).
    """
    bufs = _stacked(trajectory)
    if not (dist.is_available() and dist.is_initialized()):
        return bufs
    world = dist.get_world_size(group)
    parts = [bufs[k].contiguous().reshape(-1).view(torch.uint8) for k in _NAMES]
    sizes = [p.numel() for p in parts]
    packed = torch.cat(parts)
    out = torch.empty(world * packed.numel(), dtype=torch.uint8, device=packed.device)
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
        src = bufs[name]
        chunk = per_rank[:, off:off + sz].contiguous().view(src.dtype)
        chunk = chunk.view(world, *src.shape)  # [world, T, E, ...]
        result[name] = chunk.transpose(0, 1).reshape(src.shape[0], world * src.shape[1],
                                                     *src.shape[2:])
        off += sz
    return result


def gather_ms(stats: dict) -> float:
    """Duration of a gather recorded with stats (after synchronisation)."""
    if "events" in stats:
        ev0, ev1 = stats["events"]
        return float(ev0.elapsed_time(ev1))
    return float(stats.get("ms", 0.0))
