"""
reuse_forces (espresso.py:1304-1306: integrator.run(k, reuse_forces=True)).
ESPResSo's Brownian propagator advances each step with the forces of the
force calculation that ended the previous step, and a run with reuse_forces
does not recompute them first: sub-step 0 of every run swims with the
previous run's swim force and torque, along the orientation that run ended
with.  Every integration path (cluster run, wide run, global path, big
clusters in the check, 3-D) against the oracle's restatement, bit for bit,
and the closed form at kT = 0 through the product API.
"""

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


def _eq(a, b):
    for k in ("q", "img", "ang"):
        assert np.array_equal(a[k], b[k]), k


def _disc(rng, n, L):
    r = L / 2 * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    pos = np.stack([L / 2 + r * np.cos(th), L / 2 + r * np.sin(th), np.zeros(n)], 1)
    a = 2 * np.pi * rng.random(n)
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    return pos, dirs


@pytest.mark.parametrize("wide,E", [("1", 1), ("0", 1), ("0", 9)])
def test_reuse_cluster_path_4096_bit_exact(wide, E, monkeypatch):
    """Bench-size envs (4096 colloids, area fraction 0.1): new actions every
    window, including a window shorter than a slice; the wide latency-bound
    run, the 256-thread run and the throughput engine (9 envs)."""
    monkeypatch.setenv("SWARMRL_AMD_WIDE_RUN", wide)
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(31)
    n = 4096
    L = 2 * np.sqrt(n / 0.1)
    box = [L, L, L]
    states = []
    for _ in range(E):
        pos, dirs = _disc(rng, n, L)
        states.append(oracle.state_from_positions(pos, dirs, box))
    h = Harness(box, 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int),
                n_envs=E, reuse=True)
    h.upload(states)
    h.sd(300)
    states = [oracle.sd_run(h.op, s, np.zeros(n), 300)[0] for s in states]
    track = [oracle.ReuseForces(s) for s in states]
    check = sorted({0, E - 1})
    step = 0
    for nsteps in (100, 37, 1, 100):  # 1: the saved actions of a one-sub-step window
        f = rng.choice([0.0, 10.0], E * n).astype(np.float32)
        t = rng.choice([-10.0, 0.0, 10.0], E * n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        got = h.download()
        vel = h.velocities()
        for e in check:
            sl = slice(e * n, (e + 1) * n)
            states[e], v, _ = track[e].run(h.op, states[e], np.zeros(n), f[sl], t[sl], nsteps,
                                           step0=step, env=e)
            _eq(got[e], states[e])
            assert np.array_equal(vel[:, sl], v)
        step += nsteps


def test_reuse_differs_from_fresh_forces():
    """The semantics is observable: with reuse the trajectory after an action
    change differs from the fresh-force one (and equals its restatement)."""
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(32)
    box = [100.0, 100.0, 100.0]
    n = 500
    st0 = random_state(rng, n, box)
    out = {}
    for reuse in (False, True):
        h = Harness(box, 1e-3, 0.0, 1.0239, 3, species_list()[:1], np.zeros(n, int),
                    reuse=reuse)
        h.upload([st0])
        h.set_actions(np.full(n, 10.0, np.float32), np.full(n, 5.0, np.float32))
        h.integrate(50)
        out[reuse] = h.download()[0]
    assert not np.array_equal(out[False]["q"], out[True]["q"])
    # nothing swam before the first run: sub-step 0 has zero swim force and torque
    ref, _, _ = oracle.bd_run(h.op, st0, np.zeros(n), np.full(n, 10.0), np.full(n, 5.0), 50,
                              prev={"f": np.zeros(n), "t": np.zeros(n), "ang": st0["ang"]})
    _eq(out[True], ref)


def test_reuse_global_path_and_directors():
    """A small box runs on the global path (one workgroup per env); between
    runs set_directors turns every colloid: sub-step 0 still swims along the
    orientation of the last force calculation (the reference rotates the
    particle, the stored force keeps the old director)."""
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(33)
    box = [12.0, 12.0, 12.0]
    n = 20
    sp = np.zeros(n, int)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 9, species_list()[:1], sp, reuse=True)
    st = random_state(rng, n, box)
    h.upload([st])
    h.sd(300)
    st = oracle.sd_run(h.op, st, sp, 300)[0]
    _eq(h.download()[0], st)
    track = oracle.ReuseForces(st)
    step = 0
    for k, nsteps in enumerate((40, 1, 25)):
        f = rng.normal(size=n).astype(np.float32) * 10
        t = rng.normal(size=n).astype(np.float32) * 10
        if k == 2:  # new_direction before this run
            a = 2 * np.pi * rng.random(n)
            d = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
            mask = np.ones(n, np.uint8)
            h.native.bind_stream()
            h.native.call("swarm_engine_set_directors",
                          np.ascontiguousarray(d).ctypes.data, mask.ctypes.data)
            st = dict(st, ang=h.download()[0]["ang"])
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, v, _ = track.run(h.op, st, sp, f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), v)


def test_reuse_big_clusters_and_rerun_bit_exact():
    """Clusters wider than a wave (run in k_check) and fast swimmers that fail
    the decomposition check (exact re-run from the snapshot) with reuse."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(34)
    box = [200.0, 200.0, 200.0]
    pts = []
    for cx, cy in ((40.0, 40.0), (120.0, 60.0)):
        for gx in range(10):
            for gy in range(10):
                pts.append((cx + 2.5 * gx, cy + 2.5 * gy))
    while len(pts) < 900:
        p = rng.random(2) * 200.0
        if min((p[0] - q[0]) ** 2 + (p[1] - q[1]) ** 2 for q in pts) > 16.0:
            pts.append((p[0], p[1]))
    n = len(pts)
    pos = np.zeros((n, 3))
    pos[:, :2] = pts
    a = 2 * np.pi * rng.random(n)
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    st = oracle.state_from_positions(pos, dirs, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], np.zeros(n, int), reuse=True)
    h.upload([st])
    track = oracle.ReuseForces(st)
    step = 0
    reran = False
    for nsteps, fmax in ((100, 5.0), (60, 5.0), (100, 400.0), (100, 5.0)):
        f = rng.choice([0.0, fmax], n).astype(np.float32)
        t = rng.choice([-5.0, 0.0, 5.0], n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, v, _ = track.run(h.op, st, np.zeros(n), f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), v)
        fb = np.zeros(1, np.int32)
        h.native.call("swarm_engine_window_stats", fb.ctypes.data, None)
        reran |= fb[0] == 2
    assert reran  # the 400-force window took the exact re-run


def test_reuse_3d_bit_exact():
    from gpu_harness import Harness, random_state3, species_list

    rng = np.random.default_rng(35)
    box = [30.0, 30.0, 30.0]
    n = 120
    sp = rng.integers(0, 2, n)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 4, species_list(), sp, n_dims=3, reuse=True)
    st = random_state3(rng, n, box)
    h.upload([st])
    track = oracle.ReuseForces(st, dims=3)
    step = 0
    for k, nsteps in enumerate((30, 20)):
        f = rng.normal(size=n).astype(np.float32) * 10
        tq = rng.normal(size=(3, n)).astype(np.float32) * 5
        if k == 1:  # 3-D new_direction: the director is set, the reused one is not
            d = rng.normal(size=(n, 3))
            h.native.bind_stream()
            h.native.call("swarm_engine_set_directors", np.ascontiguousarray(d).ctypes.data,
                          np.ones(n, np.uint8).ctypes.data)
            st = dict(st, dir=h.download()[0]["dir"])
        h.set_torque_xy(tq[:2])
        h.set_actions(f, tq[2])
        h.integrate(nsteps)
        st, v, w = track.run(h.op, st, sp, f, tq, nsteps, step0=step)
        step += nsteps
        got = h.download()[0]
        for key in ("q", "img", "dir"):
            assert np.array_equal(got[key], st[key]), key
        assert np.array_equal(h.velocities(), v)


def test_reuse_kt0_closed_form_through_engine(tmp_path):
    """kT = 0, no neighbours: after a slice whose action changed from v_old
    to v_new, x = x0 + dt v_old + (n - 1) dt v_new (one sub-step of lag);
    with reuse_forces=False, x = x0 + n dt v_new."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    res = {}
    for reuse in (True, False):
        ureg = UnitRegistry()
        p = MDParams(ureg=ureg, box_length=ureg.Quantity([1000.0] * 3, "micrometer"),
                     WCA_epsilon=ureg.Quantity(1e-20, "joule"),
                     temperature=ureg.Quantity(0, "kelvin"),
                     time_step=ureg.Quantity(0.01, "second"),
                     time_slice=ureg.Quantity(0.1, "second"),
                     write_interval=ureg.Quantity(0.1, "second"))
        eng = SwarmEngine(p, n_dims=2, seed=5, out_folder=tmp_path / str(reuse),
                          reuse_forces=reuse)
        eng.add_colloids(4, ureg.Quantity(1.0, "micrometer"),
                         ureg.Quantity(np.array([500.0, 500.0, 0.0]), "micrometer"),
                         ureg.Quantity(400, "micrometer"), type_colloid=0)
        eng.integrate(1, ForceFunction({"0": dummy_models.ConstForce(2.0)}))
        x1 = eng.get_particle_data()["Unwrapped_Positions"]
        d = eng.get_particle_data()["Directors"]
        eng.integrate(1, ForceFunction({"0": dummy_models.ConstForce(7.0)}))
        x2 = eng.get_particle_data()["Unwrapped_Positions"]
        gt, _ = eng.get_friction_coefficients(0)
        n_sub = eng.params.steps_per_slice
        dt = 0.01
        res[reuse] = (x2 - x1, d, gt, n_sub, dt)
        eng.finalize()
    dx, d, gt, n_sub, dt = res[True]
    want = d * (dt * 2.0 / gt + (n_sub - 1) * dt * 7.0 / gt)
    np.testing.assert_allclose(dx[:, :2], want[:, :2], rtol=1e-5, atol=5e-6)
    dx, d, gt, n_sub, dt = res[False]
    np.testing.assert_allclose(dx[:, :2], d[:, :2] * n_sub * dt * 7.0 / gt, rtol=1e-5, atol=5e-6)
