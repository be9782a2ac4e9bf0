"""
The exact headline workload against the oracle (it was only
compared with itself across build modes): one env x 4096 colloids, the
bench's vision-cone observable (SubdividedVisionCones(10, pi/2, 3),
subdivided_vision_cones.py:17-258), the actor-critic MLP with Gumbel
sampling (flax_network.py:153-195), the GradientSensing reward
(gradient_sensing.py:92-126) and the reference's 1 s trajectory writes,
driven exactly as bench.py drives it: three eager slices, then the episode
graph (bench.capture_episode) replayed twice -- 40 slices with the ride-along
build, the speculative vision grid, the one-kernel policy, the noise table
filled beside the run and the device trajectory ring, all inside the replayed
graph (espresso.py:1251-1308).

The sampled actions are the only input the CPU oracle cannot reproduce (JAX
threefry / our Gumbel counters are parity-unpinned), so they are recorded and
replayed: from the same placement, the oracle's overlap removal, then per
slice the vision cones of every agent (the reference's loop over a cell list:
same bits), 100 BD+WCA sub-steps with the recorded actions (reuse_forces,
espresso.py:1304-1306) and the clipped gradient reward.  Features, rewards,
the final q / img / ang and every trajectory entry the ring recorded must
match bit for bit.
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


def _reward(p, st, agents, src, box, hist):
    """k_field's clipped transform: 10 * ((1 - d_cur) - (1 - d_prev)), >= 0."""
    dc, dp = oracle.field_distance(p, st, agents, src, box, hist, update=True)
    f32 = np.float32
    v = (f32(10.0) * ((f32(1.0) - dc) - (f32(1.0) - dp))).astype(np.float32)
    return np.where(v < 0, f32(0), v).astype(np.float32)


def _host(traj):
    return {k: [torch.as_tensor(x).detach().cpu().numpy().copy() for x in getattr(traj, k)]
            for k in ("features", "actions", "rewards")}


# switches read at engine creation: the default, the pair search's
# block-local union-find (SWARMRL_AMD_LOCAL_UF) and the run without its
# rotation helper waves (SWARMRL_AMD_ROT_HELPER=0: each run wave turns its
# own directors); every mode integrates the same bits
@pytest.mark.parametrize("mode", [{}, {"SWARMRL_AMD_LOCAL_UF": "1"},
                                  {"SWARMRL_AMD_ROT_HELPER": "0"}],
                         ids=["default", "local_uf", "no_rot_helper"])
def test_headline_episode_graph_replays_match_oracle(tmp_path, monkeypatch, mode):
    for k, v in mode.items():
        monkeypatch.setenv(k, v)
    sys.path.insert(0, ROOT)
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, T, replays = 4096, 20, 2
    ns = argparse.Namespace(colloids=N, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_workload(ns, 42, dev)
    pos0 = np.stack(eng._pos[0])
    dir0 = np.stack(eng._dir[0])
    eng.integrate(1, ff)  # bench.measure: set-up, overlap removal, first slice (eager)
    _, episode_graph, warm = bench.capture_episode(eng, ff, agent, T)
    slices = [_host(warm)]
    assert len(slices[0]["actions"]) == 3
    for _ in range(replays):
        episode_graph.replay()
        torch.cuda.synchronize()
        slices.append(_host(agent.trajectory))
        assert len(slices[-1]["actions"]) == T and len(slices[-1]["rewards"]) == T
    eng.drain_trajectory(block=True)
    got = eng.get_raw_state()
    frames = [(float(np.asarray(t).reshape(-1)[0]), np.asarray(x).copy())
              for t, x in zip(eng.traj_holder["Times"], eng.traj_holder["Unwrapped_Positions"])]
    del episode_graph

    L = float(eng._box[0])
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           eng.params.WCA_epsilon.m_as("sim_energy"), 42, [eng._species_keys[0]])
    agents = np.arange(N)
    radii = np.ones(N, np.float32)
    types = np.zeros(N, np.int32)
    ftab = np.array([0.0, 10.0, 0.0, 0.0], np.float32)  # bench's action table
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    sp = np.zeros(N, np.uint8)
    st = oracle.state_from_positions(pos0, dir0, eng._box)
    hist = oracle.history_from_state(st, agents)  # GradientSensing.initialize (reset_agent)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    prev = {"f": np.zeros(N, np.float32), "t": np.zeros(N, np.float32), "ang": st["ang"].copy()}

    def unwrapped(state):  # the conversion of get_particle_data / the ring drain
        return np.stack([(state["img"][a].astype(np.float64) +
                          state["q"][a].astype(np.float64) / 2.0**32) * float(eng._box[a])
                         for a in range(2)], 1)

    snaps = {0: unwrapped(st)}  # unwrapped positions at every slice boundary (step)
    step = 0
    for block in slices:
        for s in range(len(block["actions"])):
            obs = oracle.vision_cone(p, st, agents, radii, types, 10.0, np.pi / 2, 3, [0],
                                     cells=True)
            assert np.array_equal(block["features"][s].reshape(obs.shape), obs), (step, "cone")
            idx = block["actions"][s].reshape(-1)
            f, t = ftab[idx], ttab[idx]
            st, _, _ = oracle.bd_run(p, st, sp, f, t, 100, step0=100 * step, prev=prev)
            prev = {"f": f, "t": t, "ang": st["ang"].copy()}
            rew = _reward(p, st, agents, src, box, hist)
            assert np.array_equal(block["rewards"][s].reshape(-1), rew), (step, "reward")
            step += 1
            snaps[100 * step] = unwrapped(st)
    assert step == 3 + replays * T
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], st[k]), k
    # every trajectory write (device ring, 1 s interval, recorded inside the
    # replayed graph at the device step counter) holds the oracle's state of
    # its time step
    matched = 0
    for t, x in frames:
        k = int(round((t - eng._time_offset) / eng._time_step))
        assert k in snaps, (t, k)
        assert np.array_equal(x[:, :2], snaps[k]), ("trajectory entry", k)
        matched += 1
    assert matched >= 3, frames
