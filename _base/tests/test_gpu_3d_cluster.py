"""
3-D at scale: the two windowed 3-D paths against the CPU oracle, bit for
bit (swarm_integrator3.cuh):
  cluster  k_build_sort3 -> k_build_pairs3 -> k_cluster_build ->
           k_cluster_run3 -> k_check3 (dilute boxes)
  nlist    k_build_sort3 -> k_build_nlist3 -> one k_nl_step3 per sub-step
           -> k_check3 (boxes whose rc + skin
           graph percolates)
SWARMRL_AMD_NLIST=0|1 picks the path (by default the engine picks it from
the density).

The reference engine's default dimension is 3 (EspressoMD(n_dims=3),
espresso.py:143-152; free rotation about all axes, espresso.py:415-426);
the BD update is or_bd_run3's sequence (oracle/swarm_oracle.c).  Covered:
bench-size envs (4096 colloids) that pass the decomposition check, several
envs, two species, reuse_forces with a one-sub-step window, walls, and
windows that fail the check or are flagged by the build (a cluster wider
than a wave) and re-run on the 3-D global path.
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


def _eq3(got, ref):
    for k in ("q", "img", "dir"):
        assert np.array_equal(got[k], ref[k]), k


def _lattice3(rng, n, a=4.6, jitter=0.3):
    """n colloids on a jittered cubic lattice of spacing a (no overlaps; few
    links within r_i + r_j + skin = 4, so small clusters); the box is k a."""
    k = int(np.ceil(n ** (1.0 / 3.0) - 1e-9))
    g = np.stack(np.meshgrid(np.arange(k), np.arange(k), np.arange(k), indexing="ij"), -1)
    pos = (g.reshape(-1, 3)[:n] + 0.5) * a + rng.uniform(-jitter, jitter, (n, 3))
    d = rng.normal(size=(n, 3))
    return pos, d, k * a


@pytest.fixture(params=["cluster", "nlist"])
def path3(request, monkeypatch):
    """cluster: the cluster window; nlist: one k_nl_step3 launch per
    sub-step over per-colloid Verlet lists."""
    monkeypatch.setenv("SWARMRL_AMD_NLIST", "0" if request.param == "cluster" else "1")
    return request.param


def _stats(h):
    fb = np.zeros(h.E, np.int32)
    w = np.zeros(h.E, np.int32)
    h.native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
    return fb, w


@pytest.mark.parametrize("E,n_species", [(1, 1), (3, 2)])
def test_cluster3_4096_bit_exact(E, n_species, path3):
    """4096 colloids at volume fraction ~0.04: every window passes the check (no re-run), three slices with new
    actions, positions / images / directors / velocities bit-exact."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(41)
    n = 4096
    lat = [_lattice3(rng, n) for _ in range(E)]
    L = lat[0][2]
    box = [L, L, L]
    sp = rng.integers(0, n_species, n)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 17, species_list()[:n_species], sp, n_envs=E,
                n_dims=3)
    states = [oracle.state3_from_positions(p, d, box) for p, d, _ in lat]
    h.upload(states)
    check = sorted({0, E - 1})
    step = 0
    for nsteps in (100, 100, 37):
        f = rng.choice([0.0, 10.0], E * n).astype(np.float32)
        tq = rng.normal(scale=5.0, size=(3, E * n)).astype(np.float32)
        h.set_actions(f, tq[2])
        h.set_torque_xy(tq[:2])
        h.integrate(nsteps)
        fb, waves = _stats(h)
        assert (fb == 0).all()  # check passed, no re-run
        assert (waves > 0).all() == (path3 == "cluster")
        got = h.download()
        vel = h.velocities()
        om = h.omegas3()
        for e in check:
            s = slice(e * n, (e + 1) * n)
            states[e], v, w = oracle.bd_run3(h.op, states[e], sp, f[s], tq[:, s], nsteps,
                                             step0=step, env=e)
            _eq3(got[e], states[e])
            assert np.array_equal(vel[:, s], v) and np.array_equal(om[:, s], w)
        step += nsteps


def test_cluster3_matches_global_path(monkeypatch):
    """The same engine run on the three 3-D paths (SWARMRL_AMD_CLUSTER_PATH=0
    forces the global one) gives the same bits."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(42)
    n = 2000
    pos, d, L = _lattice3(rng, n)
    box = [L, L, L]
    st = oracle.state3_from_positions(pos, d, box)
    f = rng.choice([0.0, 20.0], n).astype(np.float32)
    tq = rng.normal(scale=5.0, size=(3, n)).astype(np.float32)
    out = {}
    for path in ("1", "0", "nl"):
        monkeypatch.setenv("SWARMRL_AMD_CLUSTER_PATH", "0" if path == "0" else "1")
        monkeypatch.setenv("SWARMRL_AMD_NLIST", "1" if path == "nl" else "0")
        h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], np.zeros(n, int),
                    n_dims=3)
        h.upload([st])
        h.set_actions(f, tq[2])
        h.set_torque_xy(tq[:2])
        h.integrate(150)
        out[path] = (h.download()[0], h.velocities(), h.omegas3(), _stats(h))
    for p in ("1", "nl"):
        _eq3(out[p][0], out["0"][0])
        assert np.array_equal(out[p][1], out["0"][1]) and np.array_equal(out[p][2], out["0"][2])
        assert out[p][3][0][0] == 0  # windowed path, check passed
    assert out["1"][3][1][0] > 0 and out["0"][3][1][0] == 0  # waves: cluster vs global


def test_cluster3_reuse_one_substep_window(path3):
    """reuse_forces on the 3-D cluster path, including a window of one
    sub-step (its saved actions are this run's, not the reused ones)."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(43)
    n = 1500
    pos, d, L = _lattice3(rng, n)
    box = [L, L, L]
    st = oracle.state3_from_positions(pos, d, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 6, species_list()[:1], np.zeros(n, int), n_dims=3,
                reuse=True)
    h.upload([st])
    track = oracle.ReuseForces(st, dims=3)
    step = 0
    for nsteps in (100, 1, 1, 60):
        f = rng.normal(size=n).astype(np.float32) * 10
        tq = rng.normal(size=(3, n)).astype(np.float32) * 10
        h.set_actions(f, tq[2])
        h.set_torque_xy(tq[:2])
        h.integrate(nsteps)
        st, v, w = track.run(h.op, st, np.zeros(n), f, tq, nsteps, step0=step)
        step += nsteps
        _eq3(h.download()[0], st)
        assert np.array_equal(h.velocities(), v) and np.array_equal(h.omegas3(), w)
        fb, waves = _stats(h)
        assert fb[0] == 0 and (waves[0] > 0) == (path3 == "cluster")


def test_cluster3_rerun_and_big_cluster_bit_exact(path3):
    """A dense block of touching colloids (one cluster wider than a wave: the
    build flags the env) and fast swimmers (movers that fail the check) both
    re-run on the 3-D global path from the window-start snapshot."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(44)
    rest, _, L = _lattice3(rng, 1000, a=6.0, jitter=0.2)
    box = [L, L, L]
    g = np.stack(np.meshgrid(np.arange(5), np.arange(5), np.arange(5), indexing="ij"), -1)
    block = 10.0 + 2.3 * g.reshape(-1, 3)  # 125 colloids within rc + skin of their neighbours
    rest = rest[np.min(np.linalg.norm(rest[:, None] - block[None], axis=2), axis=1) > 5.0]
    pos = np.concatenate([block, rest])
    n = len(pos)
    st = oracle.state3_from_positions(pos, rng.normal(size=(n, 3)), box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 8, species_list()[:1], np.zeros(n, int), n_dims=3)
    h.upload([st])
    step = 0
    seen = set()
    for nsteps, fmax in ((100, 5.0), (100, 400.0)):
        f = rng.choice([0.0, fmax], n).astype(np.float32)
        tq = rng.normal(scale=5.0, size=(3, n)).astype(np.float32)
        h.set_actions(f, tq[2])
        h.set_torque_xy(tq[:2])
        h.integrate(nsteps)
        st, v, w = oracle.bd_run3(h.op, st, np.zeros(n), f, tq, nsteps, step0=step)
        step += nsteps
        _eq3(h.download()[0], st)
        assert np.array_equal(h.velocities(), v) and np.array_equal(h.omegas3(), w)
        seen.add(int(_stats(h)[0][0]))
    assert 2 in seen  # re-run on the global path


def test_cluster3_walls_bit_exact(path3):
    """Plane walls (espresso.py:667-711) on the 3-D cluster path."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(45)
    n = 1000
    pos, d, L = _lattice3(rng, n)
    box = [L, L, L]
    pos[:, 2] = 2.0 + (pos[:, 2] / L) * (L - 4.0)  # keep clear of the z walls at start
    st = oracle.state3_from_positions(pos, d, box)
    walls = [{"kind": 0, "normal": (0.0, 0.0, 1.0), "offset": 0.5},
             {"kind": 0, "normal": (0.0, 0.0, -1.0), "offset": -(L - 0.5)}]
    h = Harness(box, 1e-3, 1.0239, 1.0239, 9, species_list()[:1], np.zeros(n, int), n_dims=3)
    h.set_walls(walls)
    h.upload([st])
    f = np.full(n, 10.0, np.float32)
    tq = rng.normal(scale=5.0, size=(3, n)).astype(np.float32)
    h.set_actions(f, tq[2])
    h.set_torque_xy(tq[:2])
    h.integrate(200)
    ref, v, w = oracle.bd_run3(h.op, st, np.zeros(n), f, tq, 200, walls=walls)
    _eq3(h.download()[0], ref)
    assert np.array_equal(h.velocities(), v)
    fb, waves = _stats(h)
    assert (waves[0] > 0) == (path3 == "cluster")
