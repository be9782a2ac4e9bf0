"""
The 2-D neighbour-list window (k_build_sort -> k_build_nlist2 -> one
k_nl_step2 per sub-step -> k_check,
swarm_integrator.cuh) against the CPU
oracle, bit for bit.  It serves dense boxes, where the rc + skin graph
percolates and per-wave clusters do not exist (a 4096-colloid square lattice
of spacing 3: area fraction 0.35, every colloid linked to its neighbours);
the engine picks it from the density (SWARMRL_AMD_NLIST=0|1 overrides).
Covered: several envs and species, the three 2-D paths against each other,
reuse_forces with one-sub-step windows, fast movers that fail the check and
re-run, and walls.
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


def _eq(got, ref):
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], ref[k]), k


def _lattice2(rng, n, a=3.0, jitter=0.3):
    """n colloids on a jittered square lattice of spacing a; box k a."""
    k = int(np.ceil(np.sqrt(n) - 1e-9))
    g = np.stack(np.meshgrid(np.arange(k), np.arange(k), indexing="ij"), -1).reshape(-1, 2)[:n]
    pos = np.zeros((n, 3))
    pos[:, :2] = (g + 0.5) * a + rng.uniform(-jitter, jitter, (n, 2))
    th = 2 * np.pi * rng.random(n)
    dirs = np.stack([np.cos(th), np.sin(th), np.zeros(n)], 1)
    return pos, dirs, k * a


def _stats(h):
    fb = np.zeros(h.E, np.int32)
    w = np.zeros(h.E, np.int32)
    h.native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
    return fb, w


@pytest.mark.parametrize("E,n_species", [(1, 1), (3, 2)])
def test_nlist2d_4096_dense_bit_exact(E, n_species):
    """One k_nl_step2 launch per sub-step, bit-exact against the oracle."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(51)
    n = 4096
    lat = [_lattice2(rng, n) for _ in range(E)]
    L = lat[0][2]
    box = [L, L, L]
    sp = rng.integers(0, n_species, n)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 21, species_list()[:n_species], sp, n_envs=E)
    states = [oracle.state_from_positions(p, d, box) for p, d, _ in lat]
    h.upload(states)
    check = sorted({0, E - 1})
    step = 0
    for nsteps in (100, 100, 37):
        f = rng.choice([0.0, 10.0], E * n).astype(np.float32)
        t = rng.choice([-10.0, 0.0, 10.0], E * n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        fb, waves = _stats(h)
        assert (fb == 0).all() and (waves == 0).all()  # neighbour-list window, check passed
        got = h.download()
        vel = h.velocities()
        for e in check:
            s = slice(e * n, (e + 1) * n)
            states[e], v, _ = oracle.bd_run(h.op, states[e], sp, f[s], t[s], nsteps, step0=step,
                                            env=e)
            _eq(got[e], states[e])
            assert np.array_equal(vel[:, s], v)
        step += nsteps


def test_nlist2d_matches_cluster_and_global_paths(monkeypatch):
    """Dense box on the three 2-D paths: neighbour-list window, cluster
    window forced (one giant cluster: the global path re-runs it) and the
    global path: the same bits."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(52)
    n = 2500
    pos, d, L = _lattice2(rng, n)
    box = [L, L, L]
    st = oracle.state_from_positions(pos, d, box)
    f = rng.choice([0.0, 20.0], n).astype(np.float32)
    t = rng.normal(scale=5.0, size=n).astype(np.float32)
    out = {}
    for path in ("nl", "cl", "gl"):
        monkeypatch.setenv("SWARMRL_AMD_CLUSTER_PATH", "0" if path == "gl" else "1")
        monkeypatch.setenv("SWARMRL_AMD_NLIST", "1" if path == "nl" else "0")
        h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], np.zeros(n, int))
        h.upload([st])
        h.set_actions(f, t)
        h.integrate(150)
        out[path] = (h.download()[0], h.velocities(), _stats(h))
    for p in ("cl", "gl"):
        _eq(out["nl"][0], out[p][0])
        assert np.array_equal(out["nl"][1], out[p][1])
    assert out["nl"][2][0][0] == 0  # the neighbour-list window passed its check
    assert out["cl"][2][0][0] == 2  # the giant cluster re-ran on the global path


def test_nlist2d_reuse_one_substep_window(monkeypatch):
    monkeypatch.setenv("SWARMRL_AMD_NLIST", "1")
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(53)
    n = 1600
    pos, d, L = _lattice2(rng, n)
    box = [L, L, L]
    st = oracle.state_from_positions(pos, d, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 6, species_list()[:1], np.zeros(n, int), reuse=True)
    h.upload([st])
    track = oracle.ReuseForces(st)
    step = 0
    for nsteps in (100, 1, 1, 60):
        f = rng.normal(size=n).astype(np.float32) * 10
        t = rng.normal(size=n).astype(np.float32) * 10
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, v, _ = track.run(h.op, st, np.zeros(n), f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), v)
        assert _stats(h)[0][0] == 0


def test_nlist2d_fast_movers_rerun_bit_exact(monkeypatch):
    monkeypatch.setenv("SWARMRL_AMD_NLIST", "1")
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(54)
    n = 1600
    pos, d, L = _lattice2(rng, n, a=3.5)
    box = [L, L, L]
    st = oracle.state_from_positions(pos, d, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 7, species_list()[:1], np.zeros(n, int))
    h.upload([st])
    step = 0
    seen = set()
    for nsteps, fmax in ((100, 5.0), (100, 400.0), (100, 5.0)):
        f = rng.choice([0.0, fmax], n).astype(np.float32)
        t = rng.choice([-5.0, 0.0, 5.0], n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, v, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), v)
        seen.add(int(_stats(h)[0][0]))
    assert 2 in seen and 0 in seen


def test_nlist2d_walls_bit_exact(monkeypatch):
    monkeypatch.setenv("SWARMRL_AMD_NLIST", "1")
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(55)
    n = 1600
    pos, d, L = _lattice2(rng, n)
    box = [L, L, L]
    walls = [{"kind": 0, "normal": [1, 0, 0], "offset": 0.0},
             {"kind": 0, "normal": [-1, 0, 0], "offset": -L},
             {"kind": 0, "normal": [0, 1, 0], "offset": 0.0},
             {"kind": 0, "normal": [0, -1, 0], "offset": -L}]
    st = oracle.state_from_positions(pos, d, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 8, species_list()[:1], np.zeros(n, int))
    h.set_walls(walls)
    h.upload([st])
    f = np.full(n, 10.0, np.float32)
    t = rng.normal(scale=5.0, size=n).astype(np.float32)
    h.set_actions(f, t)
    h.integrate(200)
    ref, v, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, 200, walls=walls)
    _eq(h.download()[0], ref)
    assert np.array_equal(h.velocities(), v)
