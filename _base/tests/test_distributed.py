"""Episode-parallel exchange on CPU: world_size 2 over gloo."""

import os

import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    """A port nothing listens on (the OS picks it), for one test's rendezvous."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


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
    port = _free_port()
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


def _episode(rank, ep, T=4, E=2, A=6):
    """A synthetic device-path episode of one rank: per slice [E, A, 3, 1]
    features, [E, A] actions / log-probs / rewards (different on every rank)."""
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    g = torch.Generator().manual_seed(1000 * rank + ep)
    traj = TrajectoryInformation(particle_type=0)
    for _ in range(T):
        traj.features.append(torch.randn(E, A, 3, 1, generator=g))
        traj.actions.append(torch.randint(0, 4, (E, A), generator=g))
        traj.log_probs.append(-torch.rand(E, A, generator=g) * 1.4)
        traj.rewards.append(torch.randn(E, A, generator=g))
    return traj


def _make_agent(seed):
    from swarmrl_amd.agents import ActorCriticAgent
    from swarmrl_amd.intrinsic_reward import RNDConfig, RNDReward
    from swarmrl_amd.losses import ProximalPolicyLoss
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel

    class _Task:  # the update only resets the kill switch
        kill_switch = False

    torch.manual_seed(seed)
    net = TorchModel(ActorCriticMLP(3, 4, 32), input_shape=(3,), device="cpu")
    rnd = RNDReward(RNDConfig(input_shape=(3,), n_epochs=2, batch_size=16, device="cpu"))
    return ActorCriticAgent(0, net, _Task(), None, {}, loss=ProximalPolicyLoss(n_epochs=3),
                            intrinsic_reward=rnd)


def _replica_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _replica_body(rank, world, q)
    except Exception:  # report instead of leaving the parent waiting
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


def _replica_body(rank, world, q):
    from swarmrl_amd import rollout
    from swarmrl_amd.trainers import EpisodeParallelTrainer, Trainer
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    def digests(agent):
        d = rollout.replica_digest(agent)
        allv = torch.zeros(world * d.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(allv, d)
        return allv.view(world, -1)

    res = {}
    # the episode-parallel trainer: replicas seeded differently, synced
    # by initialize_training, then two updates on gathered episodes
    agent = _make_agent(seed=17 + rank)
    trainer = EpisodeParallelTrainer([agent], update_seed=5, verify_every=1)
    trainer.initialize_training()
    init = rollout.replica_digest(agent).clone()
    rewards = []
    for ep in range(2):
        agent.trajectory = _episode(rank, ep)
        _, r, stop = trainer.update_rl()
        rewards.append(float(r))
        res[f"stop{ep}"] = bool(stop)
    d = digests(agent)
    res["identical"] = bool(torch.equal(d[0], d[1]))
    res["changed"] = not torch.equal(d[rank], init)
    res["rewards"] = rewards
    # the same two updates in one process on the rank-major concatenation
    # of both ranks' episodes (what the gathered episode must equal)
    ref = _make_agent(seed=17)
    for ep in range(2):
        parts = [_episode(r, ep) for r in range(world)]
        full = TrajectoryInformation(particle_type=0)
        for k in ("features", "actions", "log_probs", "rewards"):
            setattr(full, k, [torch.cat([getattr(p, k)[t] for p in parts], 0)
                              for t in range(len(parts[0].actions))])
        seed = 5 + ep + 1
        rollout.replicated_update(ref, full, seed)
    res["equals_single_process"] = bool(torch.equal(rollout.replica_digest(ref), d[rank]))
    # control: the plain Trainer updates on rank-local data and diverges
    plain = _make_agent(seed=17)
    for ep in range(2):
        plain.trajectory = _episode(rank, ep)
        Trainer([plain]).update_rl()
    dp = digests(plain)
    res["plain_diverges"] = not torch.equal(dp[0], dp[1])
    res["plain_checksums_differ"] = not rollout.replicas_match(plain)
    # initialize_training again after updates (the optimizers now
    # hold state) broadcasts rank 0's replica, state included
    trainer.initialize_training()
    res["rebroadcast_match"] = rollout.replicas_match(agent)
    # a kill switch raised on one rank only (a non-learning agent's task):
    # update_rl stops every rank
    frozen = _make_agent(seed=3)
    frozen.train = False
    frozen.task.kill_switch = rank == 1
    kt = EpisodeParallelTrainer([frozen])
    frozen.trajectory = _episode(rank, 0)
    frozen.trajectory.killed = rank == 1
    _, _, kstop = kt.update_rl()
    res["kill_everywhere"] = bool(kstop)
    q.put((rank, res))


def test_episode_parallel_trainer_keeps_replicas_identical_gloo():
    """VERDICT r3 / SURVEY 8(e): after two episode-parallel updates both
    ranks hold bit-identical parameters and optimizer state (policy and RND
    predictor), equal to one process updating on the concatenated episodes;
    the rank-local update (no gather) would diverge."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r]["identical"], res[r]
        assert res[r]["changed"] and res[r]["equals_single_process"], res[r]
        assert res[r]["plain_diverges"] and res[r]["plain_checksums_differ"], res[r]
        assert not res[r]["stop0"] and not res[r]["stop1"]
        assert res[r]["rebroadcast_match"] and res[r]["kill_everywhere"], res[r]
    assert res[0]["rewards"] == res[1]["rewards"]


def _uneven_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from swarmrl_amd.rollout import gather_trajectory, shard_envs
        from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

        envs = shard_envs(5, rank, world)          # 3 + 2 envs
        traj = TrajectoryInformation(particle_type=0)
        for t in range(2):
            ids = torch.tensor(envs, dtype=torch.float32)[:, None].expand(len(envs), 4)
            traj.features.append(ids[..., None] + 0.5)
            traj.actions.append(ids.to(torch.int64) + 10 * t)
            traj.log_probs.append(-ids)
            traj.rewards.append(ids * 2)
        traj.killed = rank == 1
        ok = True
        for counts in (None, [len(shard_envs(5, r, world)) for r in range(world)]):
            out = gather_trajectory(traj, env_counts=counts)
            ok &= out["actions"].shape == (2, 5, 4)
            for g in range(5):
                ok &= bool(torch.all(out["actions"][1, g] == g + 10))
                ok &= bool(torch.all(out["rewards"][0, g] == 2 * g))
            ok &= int(out["killed"]) == 1
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_gather_uneven_env_blocks_gloo():
    """shard_envs gives the first total mod G ranks one more env;
    the gather pads them for the collective and returns every global env
    once, in env order (counts exchanged, or given by the caller), and the
    kill switch of any rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uneven_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
