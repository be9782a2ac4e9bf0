"""
The episode-parallel collectives (swarmrl_amd/rollout.py) on
RCCL with device tensors, on ONE GPU: a world-size-1 "nccl" group with the
collectives forced on (rollout.force_collectives), so the packed
all_gather_into_tensor of the trajectory, the broadcast of an agent's
replica (including a non-capturable optimizer whose step count lives on the
host) and the replica checksum all-gather execute through RCCL exactly as
they do at N GPUs, minus the xGMI transfers.  The reference fans episodes out
to one worker process per trainer (ensemble_submit.py:76-138); cross-GPU
replica identity and the 1 -> 8 curve stay with the driver's 8-GPU run.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    from swarmrl_amd import _capi
    from swarmrl_amd import rollout

    _capi.require_gpu()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    rollout.force_collectives(True)
    assert dist.get_backend() == "nccl" and rollout._is_distributed()
    yield
    rollout.force_collectives(False)
    dist.destroy_process_group()


class _Traj:
    def __init__(self, dev, T=5, E=3, A=7, d=3, killed=False, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.particle_type = 0
        self.features = [f.to(dev) for f in torch.randn(T, E, A, d, generator=g)]
        self.actions = [a.to(dev) for a in torch.randint(0, 4, (T, E, A), generator=g)]
        self.log_probs = [x.to(dev) for x in torch.randn(T, E, A, generator=g)]
        self.rewards = [x.to(dev) for x in torch.randn(T, E, A, generator=g)]
        self.killed = killed


def test_packed_trajectory_all_gather_on_rccl(rccl_group):
    from swarmrl_amd import rollout

    dev = torch.device("cuda", 0)
    for killed in (False, True):
        tr = _Traj(dev, killed=killed)
        st = {}
        out = rollout.gather_trajectory(tr, stats=st, env_counts=[3])
        torch.cuda.synchronize()
        for k in ("features", "actions", "log_probs", "rewards"):
            want = torch.stack(getattr(tr, k))
            assert out[k].device == dev and out[k].dtype == want.dtype
            assert torch.equal(out[k], want), k
        assert int(out["killed"]) == int(killed)
        # one packed buffer: the four tensors' bytes plus the kill flag
        assert st["bytes"] == sum(torch.stack(getattr(tr, k)).numel() *
                                  torch.stack(getattr(tr, k)).element_size()
                                  for k in ("features", "actions", "log_probs", "rewards")) + 1
        assert rollout.gather_ms(st) >= 0.0
    # env counts exchanged by the collective itself (no env_counts given)
    tr = _Traj(dev, seed=3)
    out = rollout.gather_trajectory(tr)
    assert torch.equal(out["actions"], torch.stack(tr.actions))
    ep = rollout.gather_episode(tr)
    assert len(ep.features) == 5 and torch.equal(ep.rewards[2], tr.rewards[2])


def _rnd_agent(dev, seed):
    """A C5-shaped agent (actor-critic MLP + RND intrinsic reward) whose RND
    optimizer is a NON-capturable Adam: its step counts stay on the host."""
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    ns = argparse.Namespace(colloids=512, envs_per_gpu=1, write_interval=1.0)
    torch.manual_seed(seed)
    eng, ff, agent = bench.build_c5_workload(ns, 42 + seed, dev)
    ir = agent.intrinsic_reward
    ir.optimizer = torch.optim.Adam(ir.predictor_network.parameters(), lr=1e-3,
                                    capturable=False)
    for p in ir.predictor_network.parameters():  # one step: state exists
        p.grad = torch.randn_like(p)
    ir.optimizer.step()
    return eng, ff, agent


def test_broadcast_agent_and_replica_checks_on_rccl(rccl_group):
    from swarmrl_amd import rollout

    dev = torch.device("cuda", 0)
    _, _, agent = _rnd_agent(dev, 1)
    steps = [s["step"] for s in agent.intrinsic_reward.optimizer.state.values()]
    assert steps and all(not t.is_cuda for t in steps)  # the host-side state
    before = rollout.replica_digest(agent)
    rollout.broadcast_agent(agent, 0)
    torch.cuda.synchronize()
    assert torch.equal(rollout.replica_digest(agent), before)
    # the host-side step counts went through a device copy and came back
    assert all(not s["step"].is_cuda for s in agent.intrinsic_reward.optimizer.state.values())
    assert rollout.replicas_match(agent)
    assert rollout.any_rank(True) and not rollout.any_rank(False)


def test_replicated_update_through_rccl_equals_local_update(rccl_group):
    """One gathered episode's replicated update (PPO + RND predictor) through
    the world-1 RCCL group ends on the same bytes as the local update on the
    un-gathered episode with the same seed."""
    import copy

    from swarmrl_amd import rollout

    dev = torch.device("cuda", 0)
    eng, ff, agent = _rnd_agent(dev, 2)
    agent.reset_trajectory()
    eng.integrate(4, ff)
    traj = agent.trajectory
    twin = copy.deepcopy(agent)
    ep = rollout.gather_episode(traj)
    rollout.replicated_update(agent, ep, seed=77)
    rollout.force_collectives(False)
    try:
        local = rollout.gather_episode(traj)  # no collective: the stacked local buffers
        rollout.replicated_update(twin, local, seed=77)
    finally:
        rollout.force_collectives(True)
    torch.cuda.synchronize()
    assert torch.equal(rollout.replica_digest(agent), rollout.replica_digest(twin))


def test_bench_c3train_through_a_world1_rccl_group():
    """bench.py's c3train line (rollout + PPO update per episode) with
    --force-collective: every episode is all-gathered through RCCL and
    updated by rollout.replicated_update, as at N GPUs."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--only", "c3train", "--force-collective",
           "--train-episodes", "2", "--warmup", "40", "--no-cpu-baseline", "--dims3", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and "world-size-1 RCCL" in line["config"]["parallelism"]
    assert line["gather"]["per_run"] >= 1 and line["gather"]["bytes_per_rank"] > 0
    assert np.isfinite(line["value"]) and line["value"] > 0
