"""Episode-parallel exchange on CPU: world_size 2 over gloo."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from swarmrl_amd.rollout import gather_trajectory, shard_envs
        from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

        T, E, A = 3, 2, 4
        traj = TrajectoryInformation(particle_type=0)
        for t in range(T):
            base = rank * 1000 + t * 10
            traj.features.append(torch.full((E, A, 3, 1), float(base)))
            traj.actions.append(torch.full((E, A), base, dtype=torch.int64))
            traj.log_probs.append(torch.full((E, A), -float(base)))
            traj.rewards.append(torch.full((E, A), float(base) + 0.5))
        out = gather_trajectory(traj)
        ok = out["features"].shape == (T, world * E, A, 3, 1)
        for r in range(world):
            for t in range(T):
                v = r * 1000 + t * 10
                ok &= bool(torch.all(out["actions"][t, r * E:(r + 1) * E] == v))
                ok &= bool(torch.all(out["rewards"][t, r * E:(r + 1) * E] == v + 0.5))
        envs = shard_envs(64, rank, world)
        ok &= envs == list(range(32 * rank, 32 * rank + 32))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_gather_trajectory_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_shard_envs_contiguous_blocks_cover_every_env():
    """Rank r owns a contiguous block; the blocks tile the env ids in rank
    order, which is the env order of the rank-major all-gather."""
    from swarmrl_amd.rollout import shard_envs

    for total in (1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            blocks = [shard_envs(total, r, world) for r in range(world)]
            assert sum(blocks, []) == list(range(total))
            assert max(map(len, blocks)) - min(map(len, blocks)) <= 1
    assert shard_envs(64, 3, 8) == list(range(24, 32))
    with pytest.raises(ValueError):
        shard_envs(8, 2, 2)


def test_gather_single_process_is_identity():
    from swarmrl_amd.rollout import gather_trajectory
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    traj = TrajectoryInformation(particle_type=0)
    for t in range(2):
        traj.features.append(torch.zeros(1, 3, 3, 1))
        traj.actions.append(torch.zeros(1, 3, dtype=torch.int64))
        traj.log_probs.append(torch.zeros(1, 3))
        traj.rewards.append(torch.zeros(1, 3))
    out = gather_trajectory(traj)
    assert out["actions"].shape == (2, 1, 3)
