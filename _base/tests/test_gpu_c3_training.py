"""
BASELINE config 3 end to end at full size: 4096 colloids, the
find-centre task of the reference's PPO test (test_rl_trainers.py:105-118:
ConcentrationField observable, GradientSensing reward, f(d) = 1 - d), trained
by ContinuousTrainer (continuous_trainer.py:22-89) with the PPO update
(proximal_policy_loss.py:140-170) between episodes, all on the device path.

The sampled actions are the only input the CPU oracle cannot reproduce (JAX
threefry / our Gumbel counters are parity-unpinned), so they are recorded and
replayed: from the same placement, the oracle's overlap removal, then per
slice 100 BD+WCA sub-steps with the recorded actions (reuse_forces,
espresso.py:1304-1306), the field observable and the clipped gradient
reward -- and the engine's features, rewards and final state must match it
bit for bit.  The PPO update must have changed the policy.
"""

import argparse
import os
import sys

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _field(p, st, agents, src, box, hist, fa, fb, scale, clip):
    """k_field's fused transform (mode 1 / 2) on the oracle's distances:
    scale * ((fa + fb dc) - (fa + fb dp)) in fp32, clipped at 0 for the task."""
    dc, dp = oracle.field_distance(p, st, agents, src, box, hist, update=True)
    f32 = np.float32
    fc = f32(fa) + f32(fb) * dc
    fp = f32(fa) + f32(fb) * dp
    v = (f32(scale) * (fc - fp)).astype(np.float32)
    return np.where(v < 0, f32(0), v).astype(np.float32) if clip else v


def test_c3_training_4096_matches_oracle(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    from swarmrl_amd.trainers import ContinuousTrainer

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, T, episodes = 4096, 5, 2
    ns = argparse.Namespace(colloids=N, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_c3_workload(ns, 42, dev)
    agent.loss.n_epochs = 4
    pos0 = np.stack(eng._pos[0])
    dir0 = np.stack(eng._dir[0])
    recorded = []
    update = agent.update_agent

    def recording_update():
        tr = agent.trajectory
        recorded.append({k: [torch.as_tensor(x).clone() for x in getattr(tr, k)]
                         for k in ("features", "actions", "rewards")})
        return update()

    agent.update_agent = recording_update
    w_before = [p.detach().clone() for p in agent.network.model.parameters()]
    rewards = ContinuousTrainer([agent]).perform_rl_training(eng, n_episodes=episodes,
                                                              episode_length=T, load_bar=False)
    assert rewards.shape == (episodes + 1,) and np.all(np.isfinite(rewards))
    assert any(not torch.equal(a, b) for a, b in zip(agent.network.model.parameters(), w_before))
    got = eng.get_raw_state()

    # ---- oracle replay
    L = float(eng._box[0])
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           eng.params.WCA_epsilon.m_as("sim_energy"), 42, [eng._species_keys[0]])
    st = oracle.state_from_positions(pos0, dir0, eng._box)
    agents = np.arange(N)
    # the trainer initialises the observable and the task on engine.colloids
    # before the first integrate: the placement, ahead of the overlap removal
    obs_hist = oracle.history_from_state(st, agents)   # ConcentrationField.initialize
    task_hist = oracle.history_from_state(st, agents)  # GradientSensing.initialize
    sp = np.zeros(N, np.uint8)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    ftab = np.array([0.0, 10.0, 0.0, 0.0], np.float32)  # bench's action table
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    prev = {"f": np.zeros(N, np.float32), "t": np.zeros(N, np.float32), "ang": st["ang"].copy()}
    step = 0
    for ep in recorded:
        assert len(ep["actions"]) == T and len(ep["rewards"]) == T
        for s in range(T):
            obs = _field(p, st, agents, src, box, obs_hist, 1.0, -1.0, 10000.0, False)
            assert np.array_equal(ep["features"][s].cpu().numpy().reshape(-1), obs), (step, "obs")
            idx = ep["actions"][s].cpu().numpy().reshape(-1)
            f, t = ftab[idx], ttab[idx]
            st, _, _ = oracle.bd_run(p, st, sp, f, t, 100, step0=100 * step, prev=prev)
            prev = {"f": f, "t": t, "ang": st["ang"].copy()}
            rew = _field(p, st, agents, src, box, task_hist, 1.0, -1.0, 10.0, True)
            assert np.array_equal(ep["rewards"][s].cpu().numpy().reshape(-1), rew), (step, "reward")
            step += 1
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], st[k]), k


def test_replicated_update_on_graph_episode_matches_local_update():
    """The episode-parallel update path on the GPU (rollout.gather_episode +
    replicated_update, as bench.py's c3train runs it at world > 1), here in
    one process: the gathered episode of a replayed episode graph equals the
    local trajectory, and the replicated update (fused PPO gradient, the PPO
    graph from the second update on) leaves bit for bit the parameters and
    Adam state of a twin agent updated with compute_loss on the local data."""
    sys.path.insert(0, ROOT)
    import copy

    import bench
    from swarmrl_amd import rollout

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(colloids=1024, envs_per_gpu=2, write_interval=1.0)
    eng, ff, agent = bench.build_c3_workload(ns, 42, dev)
    agent.loss.n_epochs = 3
    twin = copy.deepcopy(agent.network)
    eng.integrate(1, ff)
    _, graph, _ = bench.capture_episode(eng, ff, agent, 5)
    for ep in range(3):
        graph.replay()
        episode = rollout.gather_episode(agent.trajectory)
        for k in ("features", "actions", "log_probs", "rewards"):
            assert all(torch.equal(a, b) for a, b in zip(getattr(episode, k),
                                                          getattr(agent.trajectory, k))), k
        rollout.replicated_update(agent, episode, seed=ep)
        agent.loss.compute_loss(network=twin, episode_data=agent.trajectory)
        torch.cuda.synchronize()
    a = rollout.replica_digest(agent)
    tw = copy.copy(agent)
    tw.network = twin
    tw.intrinsic_reward = None
    assert torch.equal(a, rollout.replica_digest(tw))


def test_replicated_update_with_rnd_is_deterministic():
    """a C5-shaped agent (ConcentrationField observable,
    GradientSensing + RND intrinsic reward) and its deep copy each run
    rollout.replicated_update on the same gathered episode for three
    episodes -- the fused PPO gradient and Adam step, then the RND
    predictor's update with its forked, re-seeded torch RNG (torch.randperm
    on the device) and its capturable Adam -- and end bit-identical:
    replica_digest covers the policy, the value head, both optimizers and the
    RND target / predictor.  The replicas of an episode-parallel run on
    different GPUs rely on exactly this (no gradient all-reduce; cross-device
    identity itself is not measured here)."""
    sys.path.insert(0, ROOT)
    import copy

    import bench
    from swarmrl_amd import rollout

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(colloids=1024, envs_per_gpu=2, write_interval=1.0)
    eng, ff, agent = bench.build_c5_workload(ns, 42, dev, rnd=True)
    assert agent.intrinsic_reward is not None
    agent.loss.n_epochs = 3
    # the reference's RND recipe (100 epochs of batch 8) is 128 k predictor
    # steps per update at this size; a few large batches exercise the same
    # code paths (randperm, minibatches, capturable Adam)
    agent.intrinsic_reward.n_epochs = 2
    agent.intrinsic_reward.batch_size = 2048
    # the twin shares nothing a replicated update writes: its own network +
    # optimizer, loss (and so PPO graph) and RND networks + optimizer
    twin = copy.copy(agent)
    twin.network = copy.deepcopy(agent.network)
    twin.loss = copy.deepcopy(agent.loss)
    twin.intrinsic_reward = copy.deepcopy(agent.intrinsic_reward)
    eng.integrate(1, ff)
    _, graph, _ = bench.capture_episode(eng, ff, agent, 5)
    digests = []
    for ep in range(3):
        graph.replay()
        episode = rollout.gather_episode(agent.trajectory)
        rollout.replicated_update(agent, episode, seed=100 + ep)
        rollout.replicated_update(twin, episode, seed=100 + ep)
        torch.cuda.synchronize()
        a, b = rollout.replica_digest(agent), rollout.replica_digest(twin)
        assert torch.equal(a, b), ep
        assert torch.equal(rollout.replica_checksum(agent), rollout.replica_checksum(twin))
        digests.append(a)
    # the updates did something: the replica changed from episode to episode
    assert not torch.equal(digests[0], digests[-1])
    # and a drifted bit is seen by the checksum the trainers compare
    with torch.no_grad():
        p = next(twin.intrinsic_reward.predictor_network.parameters())
        p.view(-1)[0] = torch.nextafter(p.view(-1)[0], torch.tensor(1e9, device=p.device))
    assert not torch.equal(rollout.replica_checksum(agent), rollout.replica_checksum(twin))
