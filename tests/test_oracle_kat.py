"""
Pins the CPU oracle (and the numpy restatement of the reference semantics)
against the reference's own known-answer tests and published vectors.
"""

import math

import numpy as np
import pytest

from oracle import refsem


# ---------------------------------------------------------------- Philox
def test_philox_random123_kat(oracle_mod):
    # Random123 kat_vectors, philox4x32 10 rounds
    assert oracle_mod.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle_mod.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [
        0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle_mod.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                             [0xA4093822, 0x299F31D0]) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_normals_are_standard(oracle_mod):
    g = np.array([oracle_mod.normals3(42, 0, i, s, 0) for i in range(64) for s in range(160)])
    g = g.reshape(-1)
    assert abs(g.mean()) < 0.02
    assert abs(g.std() - 1.0) < 0.02
    # fourth moment of a normal is 3
    assert abs(np.mean(g**4) - 3.0) < 0.15


def test_step_normals_are_standard_and_independent(oracle_mod):
    # the grouped four-word stream: every position j of a group standard
    # normal, no correlation between the three components of a sub-step or
    # between consecutive sub-steps (the sine and cosine legs of one pair
    # land in different positions of the group)
    g = np.array([oracle_mod.step_normals(42, 0, i, t) for i in range(48) for t in range(240)])
    g = g.reshape(48, 240, 3)
    for j in range(4):
        x = g[:, j::4, :].reshape(-1)
        assert abs(x.mean()) < 0.03 and abs(x.std() - 1.0) < 0.03
    flat = g.reshape(-1, 3)
    c = np.corrcoef(flat.T)
    assert np.all(np.abs(c - np.eye(3)) < 0.03)
    seq = g.reshape(48, -1)  # the stream in draw order
    for lag in (1, 2, 3, 4):
        r = np.mean(seq[:, :-lag] * seq[:, lag:])
        assert abs(r) < 0.03, lag
    # a group's sub-steps use disjoint normals: 12 distinct values per group
    grp = g[0, 8:12, :].reshape(-1)
    assert len(set(grp.tolist())) == 12


def test_elementary_functions_accuracy(oracle_mod):
    rng = np.random.default_rng(0)
    for x in rng.random(2000) * 0.999 + 1e-6:
        assert abs(oracle_mod.logf(x) - math.log(x)) < 5e-7 * max(1.0, abs(math.log(x)))
    for x in (rng.random(2000) * 2 - 1).astype(np.float32):
        assert abs(oracle_mod.acosf(x) - math.acos(float(x))) < 5e-7
    for a in rng.integers(0, 2**32, 2000):
        s, c = oracle_mod.sincos_turn(int(a))
        th = int(a) * 2 * math.pi / 2**32
        assert abs(s - math.sin(th)) < 2e-7 and abs(c - math.cos(th)) < 2e-7
    assert oracle_mod.acosf(-1.0) == np.float32(np.pi)
    assert oracle_mod.acosf(1.0) == 0.0


# ------------------------------------------- signed angle (test_utils.py:79-119)
def _angle_cases():
    my1 = np.array([1, 0, 0])
    my2 = np.array([-1 / np.sqrt(2), -1 / np.sqrt(2), 0])
    o1 = np.array([1, 0, 0])
    o2 = np.array([0, 1, 0])
    o3 = np.array([1 / 2, np.sqrt(3) / 2, 0])
    return my1, my2, o1, o2, o3


@pytest.mark.parametrize("fn_name", ["refsem", "oracle"])
def test_signed_angle_kat(fn_name, oracle_mod):
    fn = refsem.signed_angle if fn_name == "refsem" else oracle_mod.signed_angle
    my1, my2, o1, o2, o3 = _angle_cases()
    assert fn(my1, o1) == 0
    assert fn(my1, o2) == pytest.approx(np.pi / 2, rel=1e-6)
    assert fn(my1, o3) == pytest.approx(np.pi / 3, rel=1e-6)
    assert fn(my2, o1) == pytest.approx(np.pi * 3 / 4, rel=1e-6)
    assert fn(my2, o2) == pytest.approx(-np.pi * 3 / 4, rel=1e-6)
    assert abs(fn(my2, o3) + np.pi * 11 / 12) < 10e-6
    assert abs(fn(my1, o3 * 4.5) - fn(my1, o3)) < 10e-6
    assert abs(fn(my2 * 1.5, o3) - fn(my2, o3)) < 10e-6
    assert np.float32(fn(my1, -1 * o1)) == np.float32(np.pi)


# ------------------------------- vision cone (test_subdivided_vision_cone.py:17-53)
KAT_POS = np.array([[0, 0, 0], [0, 5, 0], [0, 8, 0], [-7, 8, 0], [1, 1, 0]], dtype=float)
KAT_DIR = np.array([[0, 1.0, 0], [1.0, 0, 0], [1.0, 0, 0], [0, 1.0, 0], [0, 1.0, 0]])
KAT_TYPES = np.array([0, 0, 1, 1, 0])
KAT_RADII = np.array([1, 2, 3, 4, 1], dtype=float)
KAT_EXPECT = np.array([[1.0, 0.0], [0.8, 0.75], [0.0, 0.0]])


def test_vision_cone_kat_refsem():
    obs = refsem.vision_cones(KAT_POS, KAT_DIR, KAT_TYPES, KAT_RADII, 10, np.pi / 2, 3)
    np.testing.assert_allclose(obs[0], KAT_EXPECT, atol=1e-12)


def test_vision_cone_kat_oracle(oracle_mod):
    box = [64.0, 64.0, 64.0]
    p = oracle_mod.make_params(box, 1.0, 0.0, 0.0, 0, [(1.0, 1.0, 1.0, 1.0, 1.0)])
    st = oracle_mod.state_from_positions(KAT_POS, KAT_DIR, box)
    obs = oracle_mod.vision_cone(p, st, [0, 1, 4], KAT_RADII, KAT_TYPES, 10, np.pi / 2, 3, [0, 1])
    # the reference asserts exact equality in fp32
    assert obs[0, 0, 0] == np.float32(1.0)
    assert obs[0, 1, 0] == np.float32(0.8)
    assert obs[0, 2, 0] == 0.0
    assert obs[0, 0, 1] == 0.0
    assert obs[0, 1, 1] == np.float32(0.75)
    assert obs[0, 2, 1] == 0.0


def test_vision_cone_oracle_vs_refsem_random(oracle_mod):
    """C oracle (fixed-point, fp32) vs fp64 restatement on random swarms."""
    rng = np.random.default_rng(3)
    box = [128.0, 128.0, 128.0]
    n = 120
    pos = np.zeros((n, 3))
    pos[:, :2] = 40 + rng.random((n, 2)) * 48
    ang = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(ang), np.sin(ang), np.zeros(n)], axis=1)
    types = rng.integers(0, 2, n)
    radii = 0.5 + rng.random(n)
    p = oracle_mod.make_params(box, 1.0, 0.0, 0.0, 0, [(1.0, 1.0, 1.0, 1.0, 1.0)])
    st = oracle_mod.state_from_positions(pos, dirs, box)
    dirs_q = np.zeros_like(dirs)
    for i in range(n):
        s, c = oracle_mod.sincos_turn(int(st["ang"][i]))
        dirs_q[i] = [c, s, 0]
    pos_q = oracle_mod.unwrapped(st, box)
    agents = [i for i in range(n) if types[i] == 0]
    got = oracle_mod.vision_cone(p, st, agents, radii, types, 9.0, 1.2, 4, [0, 1])
    ref = refsem.vision_cones(pos_q, dirs_q, types, radii, 9.0, 1.2, 4, [0, 1], 0)
    ref = np.stack(ref)
    # identical except where a colloid sits within fp32 rounding of a cone rim
    bad = np.abs(got - ref) > 1e-5
    assert bad.sum() <= 2, (got[bad], ref[bad])


# -------------------------------- concentration / gradient (reference KATs)
def test_concentration_and_gradient_kat_refsem():
    # test_concentration_field.py: decay -x, scale 100, box 1 -> all deltas 0
    src = np.array([0.5, 0.5, 0.0])
    box = np.array([1.0, 1.0, 1.0])
    old = [np.array([0.0, 0.0, 0.0]), np.array([0.0, 1.0, 0.0]), np.array([1.0, 1.0, 0.0])]
    new = [np.array([1.0, 0.0, 0.0]), np.array([1.0, 1.0, 0.0]), np.array([0.0, 1.0, 0.0])]
    for o, n_ in zip(old, new):
        assert refsem.concentration_observable(n_, o, src, box, lambda x: -1 * x, 100) == 0.0
    # test_gradient_sensing.py: decay 1 - x, scale 1
    old = [np.array([0.0, 0.0, 0.0]), np.array([0.0, 0.6, 0.0]), np.array([1.0, 0.0, 0.0])]
    new = [np.array([0.2, 0.2, 0.0]), np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0.0])]
    r = [refsem.gradient_reward(n_, o, src, box, lambda x: 1 - x, 1) for o, n_ in zip(old, new)]
    expect0 = (1 - np.linalg.norm(new[0] - src)) - (1 - np.linalg.norm(old[0] - src))
    assert r[0] > 0 and r[0] == pytest.approx(expect0, rel=1e-6)
    assert r[1] == 0.0
    assert r[2] == 0.0


def test_field_distance_oracle_vs_refsem(oracle_mod):
    rng = np.random.default_rng(5)
    box = [1000.0, 1000.0, 1000.0]
    n = 200
    pos0 = np.zeros((n, 3))
    pos0[:, :2] = rng.random((n, 2)) * 1000
    pos1 = pos0.copy()
    pos1[:, :2] += rng.normal(size=(n, 2))
    dirs = np.tile([1.0, 0, 0], (n, 1))
    p = oracle_mod.make_params(box, 1.0, 0.0, 0.0, 0, [(1.0, 1.0, 1.0, 1.0, 1.0)])
    st0 = oracle_mod.state_from_positions(pos0, dirs, box)
    st1 = oracle_mod.state_from_positions(pos1, dirs, box)
    agents = np.arange(n)
    hist = oracle_mod.history_from_state(st0, agents)
    src = np.array([500.0, 500.0, 0.0])
    scale = np.array([1000.0, 1000.0, 1000.0])
    d_cur, d_prev = oracle_mod.field_distance(p, st1, agents, src, scale, hist)
    u1 = oracle_mod.unwrapped(st1, box)
    u0 = oracle_mod.unwrapped(st0, box)
    for i in range(n):
        assert d_cur[i] == pytest.approx(refsem.field_distance(u1[i], src, scale), rel=2e-7)
        assert d_prev[i] == pytest.approx(refsem.field_distance(u0[i], src, scale), rel=2e-7)
    # history now holds the current positions
    assert np.array_equal(hist["q"], st1["q"][:, agents])


# ---------------------------------------------------------- BD, deterministic
def test_bd_kt0_velocity_and_drift_kat(oracle_mod):
    """test_espresso.py:102-111 in 2-D: kT = 0, v = F d / gamma_t and
    x = x0 + t v (rtol 2e-6); eta = 8.9e-3 Pa s, r = 1 um, dt = 0.01 s."""
    gt, gr = refsem.friction(8.9e-3, 1.0)
    box = [1000.0, 1000.0, 1000.0]
    rng = np.random.default_rng(1)
    n = 5
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * 1000
    direc = np.array([1 / np.sqrt(2), 1 / np.sqrt(2), 0.0])
    dirs = np.tile(direc, (n, 1))
    p = oracle_mod.make_params(box, 0.01, 0.0, 1e-20 / refsem.SIM_ENERGY, 42,
                               [(1.0, gt, gr, 1.0, 1.0)])
    st = oracle_mod.state_from_positions(pos, dirs, box)
    force = 1.234
    st1, vel, _ = oracle_mod.bd_run(p, st, np.zeros(n), np.full(n, force), np.zeros(n), 100)
    v_expect = force * direc / gt
    np.testing.assert_array_almost_equal(vel.T, np.tile(v_expect, (n, 1)))
    x0 = oracle_mod.unwrapped(st, box)
    x1 = oracle_mod.unwrapped(st1, box)
    np.testing.assert_allclose(x0 + 1.0 * v_expect, x1, rtol=2e-6)


def test_bd_kt0_reuse_forces_closed_form(oracle_mod):
    """reuse_forces (espresso.py:1304-1306): sub-step 0 swims with the
    previous run's force along the previous orientation, with the previous
    torque: x = x0 + dt v_old d_old + (n - 1) dt v_new d, and the orientation
    turns by dt tau_old / gamma_r + (n - 1) dt tau_new / gamma_r."""
    gt, gr = refsem.friction(1e-3, 1.0)
    box = [1000.0, 1000.0, 1000.0]
    p = oracle_mod.make_params(box, 0.01, 0.0, 0.0, 1, [(1.0, gt, gr, 1.0, 1.0)])
    st = oracle_mod.state_from_positions([[500.0, 500.0, 0]], [[1.0, 0, 0]], box)
    old = {"f": [2.0], "t": [0.0], "ang": oracle_mod.angle_fixed(0.0, 1.0)[None]}  # swam along +y
    n = 10
    st1, vel, om = oracle_mod.bd_run(p, st, [0], [7.0], [0.0], n, prev=old)
    dx = oracle_mod.unwrapped(st1, box) - oracle_mod.unwrapped(st, box)
    np.testing.assert_allclose(dx[0, :2], [(n - 1) * 0.01 * 7.0 / gt, 0.01 * 2.0 / gt],
                               rtol=1e-5, atol=2e-6)
    assert vel[0, 0] == pytest.approx(7.0 / gt, rel=1e-6)  # last sub-step: current force
    # torque lag
    st2, _, _ = oracle_mod.bd_run(p, st, [0], [0.0], [3.0], n,
                                  prev={"f": [0.0], "t": [1.0], "ang": st["ang"]})
    dth = ((int(st2["ang"][0]) - int(st["ang"][0])) % 2**32) * 2 * np.pi / 2**32
    assert dth == pytest.approx(0.01 * (1.0 + (n - 1) * 3.0) / gr, rel=1e-5)
    # prev equal to the current actions: the same bits as no reuse
    a, _, _ = oracle_mod.bd_run(p, st, [0], [7.0], [3.0], n)
    b, _, _ = oracle_mod.bd_run(p, st, [0], [7.0], [3.0], n,
                                prev={"f": [7.0], "t": [3.0], "ang": st["ang"]})
    for k in ("q", "img", "ang"):
        assert np.array_equal(a[k], b[k])


def test_bd_kt0_torque_kat(oracle_mod):
    """test_espresso_2d.py:168-179 analogue: omega_z = tau / gamma_rot."""
    gt, gr = refsem.friction(8.9e-4, 1.0)
    box = [100.0, 100.0, 100.0]
    p = oracle_mod.make_params(box, 0.01, 0.0, 0.0, 1, [(1.0, gt, gr, 1.0, 1.0)])
    st = oracle_mod.state_from_positions([[50.0, 50.0, 0]], [[0, 1.0, 0]], box)
    st1, _, om = oracle_mod.bd_run(p, st, [0], [0.0], [1.0], 100)
    assert om[0] == pytest.approx(1 / gr, rel=1e-6)
    dth = ((int(st1["ang"][0]) - int(st["ang"][0])) % 2**32) * 2 * np.pi / 2**32
    assert dth == pytest.approx(1.0 / gr * 1.0, rel=1e-5)


def test_wca_cutoff_is_two_radii(oracle_mod):
    """test_espresso.py:113-118 / test_rod.py:69-74: cutoff = r_i + r_j."""
    box = [50.0, 50.0, 50.0]
    p = oracle_mod.make_params(box, 1e-3, 0.0, 1.0, 0, [(1.0, 1.0, 1.0, 1.0, 1.0)])
    for sep, moves in [(1.999, True), (2.001, False)]:
        st = oracle_mod.state_from_positions([[20.0, 20, 0], [20.0 + sep, 20, 0]],
                                             [[1, 0, 0], [1, 0, 0]], box)
        st1, _, _ = oracle_mod.bd_run(p, st, [0, 0], [0, 0], [0, 0], 1)
        assert (not np.array_equal(st1["q"], st["q"])) == moves


def test_wca_force_matches_restatement(oracle_mod):
    """One BD step of a pair at kT = 0 reproduces the fp64 WCA force."""
    box = [50.0, 50.0, 50.0]
    eps = 1.0239
    dt = 1e-4
    p = oracle_mod.make_params(box, dt, 0.0, eps, 0, [(1.0, 4.66, 6.2, 1.0, 1.0)])
    sep = 1.95
    st = oracle_mod.state_from_positions([[20.0, 20, 0], [20.0 + sep, 20, 0]],
                                         [[1, 0, 0], [1, 0, 0]], box)
    _, vel, _ = oracle_mod.bd_run(p, st, [0, 0], [0, 0], [0, 0], 1)
    f = refsem.wca_force(np.array([-sep, 0.0]), 1.0, 1.0, eps)
    assert vel[0, 0] * 4.66 == pytest.approx(f[0], rel=1e-5)
    assert vel[0, 1] * 4.66 == pytest.approx(-f[0], rel=1e-5)


def test_cell_list_equals_brute_force(oracle_mod):
    rng = np.random.default_rng(11)
    box = [60.0, 60.0, 60.0]
    n = 300
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * 60
    ang = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(ang), np.sin(ang), 0 * ang], 1)
    p = oracle_mod.make_params(box, 1e-3, 1.02, 1.02, 9,
                               [(1.0, 4.66, 6.2, 1e-6, 4e-7), (0.7, 3.3, 2.1, 1e-6, 4e-7)])
    sp = rng.integers(0, 2, n).astype(np.uint8)
    st = oracle_mod.state_from_positions(pos, dirs, box)
    a, _, _ = oracle_mod.bd_run(p, st, sp, np.full(n, 3.0), np.full(n, 0.5), 25, use_cells=True)
    b, _, _ = oracle_mod.bd_run(p, st, sp, np.full(n, 3.0), np.full(n, 0.5), 25, use_cells=False)
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_overlap_removal_separates(oracle_mod):
    box = [30.0, 30.0, 30.0]
    p = oracle_mod.make_params(box, 1e-3, 0.0, 1.02, 0, [(1.0, 4.66, 6.2, 1.0, 1.0)])
    rng = np.random.default_rng(2)
    n = 60
    pos = np.zeros((n, 3))
    pos[:, :2] = 10 + rng.random((n, 2)) * 10
    st = oracle_mod.state_from_positions(pos, np.tile([1.0, 0, 0], (n, 1)), box)
    st1, steps = oracle_mod.sd_run(p, st, np.zeros(n), 1000)
    pairs = oracle_mod.neighbor_pairs(p, st1, 2.0 * 0.999)
    assert len(pairs) == 0
    assert steps <= 1000


# ------------------------------------------------ schedule (test_integration.py)
@pytest.mark.parametrize(
    "slice_, write, calls, expect",
    [
        (5, 9, [2, 3], [(10, 2, 2, 2), (25, 5, 3, 3)]),
        (7, 3, [4, 2], [(28, 4, 10, 0), (42, 6, 14, 4)]),
        (2, 2, [4, 2], [(8, 4, 4, 4), (12, 6, 6, 6)]),
    ],
)
def test_schedule_kat(slice_, write, calls, expect):
    res = refsem.schedule(slice_, write, calls, write_chunk_size=10)
    for r, (step, sl, wr, tl) in zip(res, expect):
        assert (r["step_idx"], r["slice_idx"], r["write_idx"], r["traj_len"]) == (step, sl, wr, tl)


def test_schedule_reward_cadence():
    # PPO-test timings (slice 10 s, write 1 s, dt 0.1 s) give 5
    # actions and 50 calc_reward calls per 5-slice episode.
    r = refsem.schedule(100, 10, [5], write_chunk_size=10)[0]
    assert r["n_manage"] == 5 and r["n_reward"] == 50
    r = refsem.schedule(100, 1000, [5], write_chunk_size=10)[0]
    assert r["n_manage"] == 5 and r["n_reward"] == 5


def test_placement_restatement_draw_order():
    pos, dirs = refsem.placement(4, 10.0, np.array([50.0, 50.0, 0.0]), 42)
    rng = np.random.default_rng(42)
    u = rng.random(12)
    r = 10 * np.sqrt(u[0])
    th = 2 * np.pi * u[1]
    np.testing.assert_allclose(pos[0, :2], [50 + r * np.cos(th), 50 + r * np.sin(th)])
    np.testing.assert_allclose(dirs[0, :2], [np.cos(2 * np.pi * u[2]), np.sin(2 * np.pi * u[2])],
                               atol=1e-12)


def test_refsem_pair_field_reference_kats():
    """particle_sensing / species_search KATs (test_particle_sensing.py:46-121,
    test_species_search.py:46-118): fields -2 and -sqrt(2)-1 for the unit
    triangle with decay -x; approaching colloid 1 to (0, 0.5) gives +0.5."""
    from oracle import refsem

    pos = np.array([[0.0, 0.0, 0.0], [0.0, 1.0, 0.0], [1.0, 0.0, 0.0]])
    f = refsem.pair_field(pos, [0, 0, 0], [0, 1, 2], 0, np.ones(3), lambda x: -1 * x)
    assert f[0] == -2.0
    assert f[1] == pytest.approx(-np.sqrt(2) - 1.0)
    assert f[2] == pytest.approx(-np.sqrt(2) - 1.0)
    pos2 = pos.copy()
    pos2[1, 1] = 0.5
    f2 = refsem.pair_field(pos2, [0, 0, 0], [0, 1, 2], 0, np.ones(3), lambda x: -1 * x)
    assert f2[0] - f[0] == 0.5


def test_refsem_pair_field_nonzero_size_quirk():
    """jnp.nonzero(size=M-1): an agent that is not sensed keeps only the first
    M-1 sensed colloids; coincident colloids pad with column 0."""
    from oracle import refsem

    pos = np.array([[0.0, 0.0, 0.0], [0.0, 1.0, 0.0], [2.0, 0.0, 0.0], [0.0, 0.0, 0.0]])
    types = [0, 1, 1, 0]
    # agent 0 (type 0) senses type 1: d = [1, 2] -> only the first (M-1 = 1)
    f = refsem.pair_field(pos, types, [0], 1, np.ones(3), lambda x: x)
    assert f[0] == 1.0
    # sensing type 0 from agent 0: d = [0 (self), 0 (coincident)] -> pad with col 0
    f = refsem.pair_field(pos, types, [0], 0, np.ones(3), lambda x: x + 10)
    assert f[0] == 10.0


def test_cell_list_vision_cone_equals_all_pairs(oracle_mod):
    """The CPU comparator's cell-list vision cone (bench.py cpu_baseline)
    gives the bits of the reference's all-pairs loop, with mixed image
    counters (unwrapped differences, no minimum image), several types and
    one to eight OpenMP threads."""
    rng = np.random.default_rng(5)
    box = [60.0, 60.0, 60.0]
    n = 700
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * 60.0 + rng.integers(-2, 3, (n, 2)) * 60.0
    a = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    p = oracle_mod.make_params(box, 1e-3, 1.0, 1.0, 1, [(1.0, 4.66, 6.21, 1.0, 1.0)])
    st = oracle_mod.state_from_positions(pos, dirs, box)
    assert np.count_nonzero(st["img"][:2]) > n
    agents = np.arange(0, n, 3)
    radii = rng.random(n).astype(np.float32) + 0.5
    types = rng.integers(0, 3, n)
    ref = oracle_mod.vision_cone(p, st, agents, radii, types, 9.0, np.pi / 2, 5, [0, 2])
    assert np.count_nonzero(ref) > 50
    for threads in (1, 8):
        oracle_mod.set_threads(threads)
        got = oracle_mod.vision_cone(p, st, agents, radii, types, 9.0, np.pi / 2, 5, [0, 2],
                                     cells=True)
        assert np.array_equal(got, ref)
    oracle_mod.set_threads(1)


def test_oracle_threads_do_not_change_dynamics(oracle_mod):
    """OpenMP threads in the BD loop (bench.py's all-cores CPU leg) leave the
    trajectory bit-identical."""
    rng = np.random.default_rng(6)
    box = [80.0, 80.0, 80.0]
    n = 600
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * 80.0
    a = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    p = oracle_mod.make_params(box, 1e-3, 1.0239, 1.0239, 3, [(1.0, 4.66, 6.21, 1.0, 1.0)])
    st = oracle_mod.state_from_positions(pos, dirs, box)
    f = rng.random(n) * 10
    t = rng.normal(size=n)
    outs = []
    for threads in (1, 6):
        oracle_mod.set_threads(threads)
        outs.append(oracle_mod.bd_run(p, st, np.zeros(n), f, t, 40)[0])
    oracle_mod.set_threads(1)
    for k in ("q", "img", "ang"):
        assert np.array_equal(outs[0][k], outs[1][k])


def test_normal_from_word_is_the_inverse_cdf(oracle_mod):
    """The word -> normal transform (round 6, tools/make_normal_table.py):
    the sign is the word's top bit and the magnitude the inverse normal CDF
    of the low 31 bits' centre, -Phi^-1((t + 0.5) / 2^32), to 2e-5; flipping
    the top bit negates the normal exactly, the magnitude falls as t grows,
    and the tails reach 6.3 sigma at t = 0."""
    from scipy.special import ndtri

    rng = np.random.default_rng(11)
    r = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64),
                        np.array([0, 1, 2, 2**31 - 1, 2**31, 2**32 - 2, 2**32 - 1], np.uint64)])
    z = np.array([oracle_mod.normal_from_word(int(w)) for w in r])
    g = -ndtri(((r & 0x7FFFFFFF).astype(np.float64) + 0.5) / 2.0**32)
    assert np.max(np.abs(z - np.where(r >> 31 != 0, -g, g))) < 2e-5
    for w in (0, 5, 12345, 2**20, 2**31 - 1):  # w and w with the top bit set
        assert oracle_mod.normal_from_word(w) == -oracle_mod.normal_from_word(w | 2**31)
    low = np.sort(r & 0x7FFFFFFF)
    zs = np.array([oracle_mod.normal_from_word(int(w)) for w in low])
    assert np.all(zs >= 0) and np.all(np.diff(zs) <= 0)
    assert oracle_mod.normal_from_word(0) > 6.3 and oracle_mod.normal_from_word(2**31) < -6.3


def test_normal_table_header_is_generated():
    """include/swarm_normal_table.h is what tools/make_normal_table.py
    writes (the table the engine and the oracle share)."""
    import importlib.util

    from conftest import ROOT

    spec = importlib.util.spec_from_file_location("mnt", ROOT / "tools" / "make_normal_table.py")
    mnt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mnt)
    a, d = mnt.table()
    text = (ROOT / "include" / "swarm_normal_table.h").read_text()
    body = text.split("#define SWARM_NTAB_DATA", 1)[1].replace("\\", " ")
    vals = np.array([float.fromhex(v.strip()[:-1]) for v in body.split(",") if v.strip()],
                    np.float32)
    assert np.array_equal(vals[0::2], a) and np.array_equal(vals[1::2], d)


def test_normal_table_numpy_restatement_matches_oracle(oracle_mod):
    """tools/make_normal_table.py's numpy transform (the generator's own
    accuracy check) and the C oracle's or_normal_from_word give the same
    fp32 bits for the same words (edge words included)."""
    import importlib.util

    from conftest import ROOT

    spec = importlib.util.spec_from_file_location("mnt", ROOT / "tools" / "make_normal_table.py")
    mnt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mnt)
    a, d = mnt.table()
    rng = np.random.default_rng(5)
    r = np.concatenate([rng.integers(0, 2**32, 4000, dtype=np.uint64),
                        np.array([0, 1, 2**31 - 1, 2**31, 2**31 + 1, 2**32 - 1], np.uint64)])
    z_np = mnt.transform(r.astype(np.uint32), a, d)
    z_c = np.array([oracle_mod.normal_from_word(int(w)) for w in r], np.float32)
    assert np.array_equal(z_np.view(np.uint32), z_c.view(np.uint32))

