"""
BASELINE config 2 end to end (the C2 workload was only compared
with itself): 1024 colloids per env, two envs batched in one engine, the
bench's vision-cone observable (SubdividedVisionCones(10, pi/2, 3),
subdivided_vision_cones.py:17-258), the actor-critic MLP with Gumbel
sampling (flax_network.py:153-195) and the GradientSensing reward
(gradient_sensing.py:92-126), driven by SwarmEngine.integrate exactly as the
bench runs it (ride-along build, speculative vision grid, fused policy).

The sampled actions are the only input the CPU oracle cannot reproduce
(JAX threefry / our Gumbel counters are parity-unpinned), so they are
recorded and replayed: from the same placement, the oracle's overlap
removal, then per slice the vision cones of every agent (the reference's
loop, over a cell list: same bits), 100 BD+WCA sub-steps with the recorded
actions (reuse_forces, espresso.py:1304-1306) and the clipped gradient
reward -- the engine's features, rewards and final state must match bit for
bit, in both envs.
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


def test_c2_rollout_two_envs_match_oracle():
    sys.path.insert(0, ROOT)
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, E, T = 1024, 2, 6
    ns = argparse.Namespace(colloids=N, envs_per_gpu=E, write_interval=1.0)
    eng, ff, agent = bench.build_workload(ns, 42, dev)
    pos0 = [np.stack(eng._pos[e]) for e in range(E)]
    dir0 = [np.stack(eng._dir[e]) for e in range(E)]
    eng.integrate(T, ff)
    tr = agent.trajectory
    feats = [torch.as_tensor(x).cpu().numpy() for x in tr.features]
    acts = [torch.as_tensor(x).cpu().numpy() for x in tr.actions]
    rews = [torch.as_tensor(x).cpu().numpy() for x in tr.rewards]
    assert len(feats) == T and len(acts) == T and len(rews) == T
    got = eng.get_raw_state()

    L = float(eng._box[0])
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           eng.params.WCA_epsilon.m_as("sim_energy"), 42, [eng._species_keys[0]])
    agents = np.arange(N)
    radii = np.ones(N, np.float32)
    types = np.zeros(N, np.int32)
    ftab = np.array([0.0, 10.0, 0.0, 0.0], np.float32)  # the bench's action table
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    sp = np.zeros(N, np.uint8)
    for e in range(E):
        st = oracle.state_from_positions(pos0[e], dir0[e], eng._box)
        hist = oracle.history_from_state(st, agents)  # GradientSensing.initialize (reset_agent)
        st, _ = oracle.sd_run(p, st, sp, 1000)
        prev = {"f": np.zeros(N, np.float32), "t": np.zeros(N, np.float32),
                "ang": st["ang"].copy()}
        for s in range(T):
            obs = oracle.vision_cone(p, st, agents, radii, types, 10.0, np.pi / 2, 3, [0],
                                     cells=True)
            assert np.array_equal(feats[s][e].reshape(obs.shape), obs), (e, s, "vision cone")
            idx = acts[s][e].reshape(-1)
            f, t = ftab[idx], ttab[idx]
            st, _, _ = oracle.bd_run(p, st, sp, f, t, 100, step0=100 * s, env=e, prev=prev)
            prev = {"f": f, "t": t, "ang": st["ang"].copy()}
            rew = _reward(p, st, agents, src, box, hist)
            assert np.array_equal(rews[s][e].reshape(-1), rew), (e, s, "reward")
        sl = slice(e * N, (e + 1) * N)  # raw state: [3, E*N] / [E*N], env-major
        assert np.array_equal(got["q"][:, sl], st["q"]), (e, "q")
        assert np.array_equal(got["img"][:, sl], st["img"]), (e, "img")
        assert np.array_equal(got["ang"][sl], st["ang"]), (e, "ang")
