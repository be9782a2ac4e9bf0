"""
The slice schedule of latency-bound engines with the pair search in the
slice's first launch (l1_pairs, DESIGN.md section 6 "Pair search a window
ahead") and the rollout policy fused into the vision-cone launch
(swarm_engine_vision_policy), against the oracle on the headline's workload
(bench.build_workload: 4096 colloids, SubdividedVisionCones, actor-critic MLP,
GradientSensing).

Two speeds of the Translate action: the bench's (every particle moves well
under the candidate lists' 1.5 um per window, so the first launch filters the
lists built during the last run) and ten times it (translating agents move
~2 um per window: the lists are unusable, the pair blocks wait for the
launch's fresh sort and search its cells).  Either way the decomposition may
not change a bit of the result: features, rewards, the final state and the
trajectory ring must equal the oracle's replay of the recorded actions
(espresso.py:1251-1308, as tests/test_gpu_headline.py).
"""

import argparse
import ctypes
import os
import sys

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reward(p, st, agents, src, box, hist):
    dc, dp = oracle.field_distance(p, st, agents, src, box, hist, update=True)
    f32 = np.float32
    v = (f32(10.0) * ((f32(1.0) - dc) - (f32(1.0) - dp))).astype(np.float32)
    return np.where(v < 0, f32(0), v).astype(np.float32)


def _host(traj):
    return {k: [torch.as_tensor(x).detach().cpu().numpy().copy() for x in getattr(traj, k)]
            for k in ("features", "actions", "rewards", "log_probs")}


@pytest.mark.parametrize("force", [10.0, 100.0], ids=["lists", "fallback"])
def test_l1_pairs_and_fused_policy_match_oracle(force):
    sys.path.insert(0, ROOT)
    import bench
    from swarmrl_amd.actions import Action

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, T = 4096, 6
    ns = argparse.Namespace(colloids=N, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_workload(ns, 42, dev)
    agent.actions["Translate"] = Action(force=force)
    agent._tables = None
    pos0 = np.stack(eng._pos[0])
    dir0 = np.stack(eng._dir[0])
    eng.integrate(1, ff)
    _, episode_graph, warm = bench.capture_episode(eng, ff, agent, T)
    slices = [_host(warm)]
    episode_graph.replay()
    torch.cuda.synchronize()
    slices.append(_host(agent.trajectory))
    eng.drain_trajectory(block=True)
    got = eng.get_raw_state()
    del episode_graph
    stats = (ctypes.c_uint64 * 4)()
    eng._native.call("swarm_engine_build_stats", stats, 0)
    filtered, waited, reruns, windows = list(stats)

    L = float(eng._box[0])
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           eng.params.WCA_epsilon.m_as("sim_energy"), 42, [eng._species_keys[0]])
    agents = np.arange(N)
    radii = np.ones(N, np.float32)
    types = np.zeros(N, np.int32)
    ftab = np.array([0.0, force, 0.0, 0.0], np.float32)
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    sp = np.zeros(N, np.uint8)
    st = oracle.state_from_positions(pos0, dir0, eng._box)
    hist = oracle.history_from_state(st, agents)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    prev = {"f": np.zeros(N, np.float32), "t": np.zeros(N, np.float32), "ang": st["ang"].copy()}
    step = 0
    moved = []
    for block in slices:
        for s in range(len(block["actions"])):
            obs = oracle.vision_cone(p, st, agents, radii, types, 10.0, np.pi / 2, 3, [0],
                                     cells=True)
            assert np.array_equal(block["features"][s].reshape(obs.shape), obs), (step, "cone")
            # the fused policy's log-probabilities are those of the network
            # on these features (fp32 tolerance: another summation split)
            with torch.no_grad():
                x = torch.as_tensor(obs.reshape(N, 3), device=dev)
                w1, b1, w2, b2 = agent.network.model.rollout_layers()
                lg = torch.relu(x @ w1.T + b1) @ w2.T + b2
                ref = torch.log(torch.softmax(lg, -1) + 1e-8)
            idx = block["actions"][s].reshape(-1)
            want = ref.gather(1, torch.as_tensor(idx, device=dev).view(-1, 1)).view(-1).cpu().numpy()
            np.testing.assert_allclose(block["log_probs"][s].reshape(-1), want, rtol=0, atol=2e-5)
            f, t = ftab[idx], ttab[idx]
            q0 = st["q"].copy()
            st, _, _ = oracle.bd_run(p, st, sp, f, t, 100, step0=100 * step, prev=prev)
            d = (st["q"][:2].astype(np.int64) - q0[:2].astype(np.int64))
            d = (d + 2**31) % 2**32 - 2**31
            moved.append(float(np.max(np.hypot(d[0], d[1]) * L / 2.0**32)))
            prev = {"f": f, "t": t, "ang": st["ang"].copy()}
            rew = _reward(p, st, agents, src, box, hist)
            assert np.array_equal(block["rewards"][s].reshape(-1), rew), (step, "reward")
            step += 1
    assert step == 3 + T
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], st[k]), k
    # the two parametrisations do exercise the two pair searches: at the
    # bench's speed every list is usable but (perhaps) the first window's,
    # where the overlap removal's contacts push apart; ten times faster the
    # translating agents outrun the lists
    assert windows == step and filtered + waited == step, list(stats)
    if force == 10.0:
        assert waited <= 1 and filtered >= step - 1, (moved, list(stats))
    else:
        assert max(moved) > 1.5 and waited > 0, (moved, list(stats))


def test_field_observable_rides_the_build_and_matches_oracle():
    """The same schedule with a concentration-field observable (BASELINE C3's
    find-centre workload, bench.build_c3_workload): the deferred build rides
    in the reward launch (sort + pair search, no vision grid) and the policy
    launch (cluster build), no side stream.  Features (the field observable,
    its own history), rewards, the final state and the window statistics
    against the oracle's replay of the recorded actions."""
    sys.path.insert(0, ROOT)
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, T = 4096, 6
    ns = argparse.Namespace(colloids=N, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_c3_workload(ns, 42, dev)
    assert ff.absorbs_build()
    pos0 = np.stack(eng._pos[0])
    dir0 = np.stack(eng._dir[0])
    eng.integrate(1, ff)
    _, episode_graph, warm = bench.capture_episode(eng, ff, agent, T)
    slices = [_host(warm)]
    episode_graph.replay()
    torch.cuda.synchronize()
    slices.append(_host(agent.trajectory))
    eng.drain_trajectory(block=True)
    got = eng.get_raw_state()
    del episode_graph
    stats = (ctypes.c_uint64 * 4)()
    eng._native.call("swarm_engine_build_stats", stats, 0)
    filtered, waited, reruns, windows = list(stats)

    L = float(eng._box[0])
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           eng.params.WCA_epsilon.m_as("sim_energy"), 42, [eng._species_keys[0]])
    agents = np.arange(N)
    ftab = np.array([0.0, 10.0, 0.0, 0.0], np.float32)
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    sp = np.zeros(N, np.uint8)
    st = oracle.state_from_positions(pos0, dir0, eng._box)
    hist_task = oracle.history_from_state(st, agents)
    hist_obs = oracle.history_from_state(st, agents)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    prev = {"f": np.zeros(N, np.float32), "t": np.zeros(N, np.float32), "ang": st["ang"].copy()}
    f32 = np.float32
    step = 0
    for block in slices:
        for s in range(len(block["actions"])):
            dc, dp = oracle.field_distance(p, st, agents, src, box, hist_obs, update=True)
            obs = (f32(10000.0) * ((f32(1.0) - dc) - (f32(1.0) - dp))).astype(np.float32)
            assert np.array_equal(block["features"][s].reshape(-1), obs), (step, "field")
            idx = block["actions"][s].reshape(-1)
            f, t = ftab[idx], ttab[idx]
            st, _, _ = oracle.bd_run(p, st, sp, f, t, 100, step0=100 * step, prev=prev)
            prev = {"f": f, "t": t, "ang": st["ang"].copy()}
            rew = _reward(p, st, agents, src, box, hist_task)
            assert np.array_equal(block["rewards"][s].reshape(-1), rew), (step, "reward")
            step += 1
    assert step == 3 + T
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], st[k]), k
    # every window's pair search ran in the reward launch (lists or the
    # fresh sort), none re-ran
    assert windows == step and filtered + waited == step and reruns == 0, list(stats)


def test_fused_vision_policy_samples_follow_softmax_and_own_stream():
    """swarm_engine_vision_policy's Gumbel-max draws (gumbel_distribution.py:
    37-40): pooled over 4096 agents x 40 calls on fixed positions, each
    action's count is within 5 sigma of the sum of the agents' softmax
    probabilities; and the per-agent counters run on a key of their own, so
    the group-counter sampler (compute_action_fused) on the same network,
    seed and counter values does not replay the same draws."""
    sys.path.insert(0, ROOT)
    import bench
    from swarmrl_amd.engine import ops

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, calls = 4096, 40
    ns = argparse.Namespace(colloids=N, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_workload(ns, 43, dev)
    eng.integrate(1, ff)
    torch.cuda.synchronize()
    view = eng.swarm_view()
    obs_fn, net = agent.observable, agent.network
    _, ftab, ttab, _ = agent._action_tables(dev)
    st0 = getattr(net, "_agent_state", None)
    c0 = int(st0[0].item()) if st0 is not None else 0  # the first call's counter
    counts = torch.zeros(4, dtype=torch.float64, device=dev)
    expect = torch.zeros(4, dtype=torch.float64, device=dev)
    var = torch.zeros(4, dtype=torch.float64, device=dev)
    first = None
    for c in range(calls):
        out = obs_fn.compute_with_policy(view, net, ftab, ttab)
        assert out is not None
        feats, idx, logp, f, t = out
        if c == 0:
            first = (feats.reshape(N, -1).clone(), idx.clone())
        with torch.no_grad():
            w1, b1, w2, b2 = net.model.rollout_layers()
            lg = torch.relu(feats.reshape(N, -1) @ w1.T + b1) @ w2.T + b2
            p = torch.softmax(lg.double(), -1)
        counts += torch.bincount(idx, minlength=4).double()
        expect += p.sum(0)
        var += (p * (1 - p)).sum(0)
    counts, expect, sd = counts.cpu().numpy(), expect.cpu().numpy(), np.sqrt(var.cpu().numpy())
    assert np.all(np.abs(counts - expect) < 5 * sd + 1), (counts, expect, sd)
    # the group-counter path with the same seed and zeroed counters
    feats0, idx0 = first
    w1, b1, w2, b2 = net.model.rollout_layers()
    state = ops.counter_state(None, N, dev)
    state.fill_(c0)
    idx_g = ops.policy_mlp_sample(feats0, w1, b1, w2, b2, net._fused_seed, state, 0.0,
                                  ftab, ttab)[0]
    agree = float((idx_g == idx0).double().mean())
    with torch.no_grad():
        p0 = torch.softmax((torch.relu(feats0 @ w1.T + b1) @ w2.T + b2).double(), -1)
    chance = float((p0 * p0).sum(-1).mean())
    assert agree < chance + 0.05, (agree, chance)
