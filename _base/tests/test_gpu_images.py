"""
GPU parity at nonzero and mixed image counters.

The reference's vision cone takes differences of UNWRAPPED positions with no
minimum image and no range limit (swarmrl/observables/
subdivided_vision_cones.py:116-121), while the engine's cell grid lives in
the folded box.  The concentration field and gradient-sensing task scale
unwrapped positions and their history (concentration_field.py:84-108,
gradient_sensing.py:92-126).  These tests compare the HIP kernels with the
oracle bit for bit on states where the image counters matter:

* pairs that are close in the folded box but in different images (the
  reference does not see them),
* pairs that are close only once unwrapped (across the box edge, in
  neighbouring images: the reference sees them),
* a history that crossed the box edge between two field evaluations,
* the bench workload's engine after enough swimming for the engine itself
  to produce image changes.
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


def _mixed_image_positions(rng, n, L, R):
    """Unwrapped positions: a third spread over images -1..1, a third in
    tight groups straddling box edges (close only once unwrapped, mixed
    images), a third as folded-box twins of other colloids shifted by +-L
    (close in the folded box, far once unwrapped)."""
    k = n // 3
    pos = np.zeros((n, 3))
    pos[:k, :2] = rng.uniform(-L, 2 * L, (k, 2))
    centres = np.zeros((k, 2))
    edge = rng.integers(-1, 3, (k, 2)) * L  # a box edge x = m L or y = m L
    axis = rng.integers(0, 2, k)
    centres[:, 0] = np.where(axis == 0, edge[:, 0], rng.uniform(-L, 2 * L, k))
    centres[:, 1] = np.where(axis == 1, edge[:, 1], rng.uniform(-L, 2 * L, k))
    pos[k:2 * k, :2] = centres + rng.uniform(-0.4 * R, 0.4 * R, (k, 2))
    src = rng.integers(0, 2 * k, n - 2 * k)
    shift = rng.choice([-L, L], (n - 2 * k, 2)) * rng.integers(0, 2, (n - 2 * k, 2))
    shift[np.all(shift == 0, axis=1), 0] = L
    pos[2 * k:, :2] = pos[src, :2] + shift + rng.uniform(-0.3 * R, 0.3 * R, (n - 2 * k, 2))
    ang = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(ang), np.sin(ang), np.zeros(n)], 1)
    return pos, dirs


def test_vision_cone_mixed_images_bit_exact():
    from gpu_harness import Harness, species_list
    from swarmrl_amd.engine import ops

    rng = np.random.default_rng(21)
    L, R = 60.0, 10.0
    box = [L, L, L]
    n, E = 900, 2
    types = rng.integers(0, 2, n)
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int), n_envs=E)
    states = []
    for _ in range(E):
        pos, dirs = _mixed_image_positions(rng, n, L, R)
        states.append(oracle.state_from_positions(pos, dirs, box))
    assert all(np.count_nonzero(s["img"][:2]) > n // 2 for s in states)
    h.upload(states)
    agents = np.arange(n, dtype=np.int32)
    radii = (0.5 + rng.random(n)).astype(np.float32)
    dev = torch.device("cuda", 0)
    vp = ops.vision_params(R, np.pi / 2, 3, [0, 1])
    out = ops.vision_cone(h.native, E, torch.as_tensor(agents, device=dev),
                          torch.as_tensor(radii, device=dev),
                          torch.as_tensor(types.astype(np.int32), device=dev), vp).cpu().numpy()
    for e in range(E):
        ref = oracle.vision_cone(h.op, states[e], agents, radii, types, R, np.pi / 2, 3, [0, 1])
        assert np.array_equal(out[e], ref)
        assert np.count_nonzero(ref) > 200
    # the folded-box twins are really invisible: the same scene with every
    # image counter zeroed sees more
    flat = [dict(s, img=np.zeros_like(s["img"])) for s in states]
    ref_flat = oracle.vision_cone(h.op, flat[0], agents, radii, types, R, np.pi / 2, 3, [0, 1])
    ref_img = oracle.vision_cone(h.op, states[0], agents, radii, types, R, np.pi / 2, 3, [0, 1])
    assert np.count_nonzero(ref_flat) > np.count_nonzero(ref_img)


def test_field_history_across_the_box_edge_bit_exact():
    from gpu_harness import Harness, species_list
    from swarmrl_amd.engine import ops

    rng = np.random.default_rng(22)
    L = 50.0
    box = [L, L, L]
    n, E = 600, 2
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int), n_envs=E)
    pos0 = [_mixed_image_positions(rng, n, L, 10.0) for _ in range(E)]
    st0 = [oracle.state_from_positions(p, d, box) for p, d in pos0]
    h.upload(st0)
    agents = np.arange(0, n, 2, dtype=np.int32)
    A = len(agents)
    dev = torch.device("cuda", 0)
    ag_t = torch.as_tensor(agents, device=dev)
    hq = torch.zeros((3, E * A), dtype=torch.int32, device=dev)
    hi = torch.zeros((3, E * A), dtype=torch.int32, device=dev)
    src = np.array([0.5 * L, 0.5 * L, 0.0])
    scale = np.array([L, L, L])
    ops.field_distance(h.native, E, ag_t, src, scale, hq, hi, update=True, init_only=True)
    hists = [oracle.history_from_state(s, agents) for s in st0]
    # every colloid moves by up to two boxes: its image changes
    st1 = []
    for p, d in pos0:
        p = p.copy()
        p[:, :2] += rng.uniform(-2 * L, 2 * L, (n, 2))
        st1.append(oracle.state_from_positions(p, d, box))
    assert np.count_nonzero(st1[0]["img"][:, agents] != st0[0]["img"][:, agents]) > A
    h.upload(st1)
    d_cur, d_prev = ops.field_distance(h.native, E, ag_t, src, scale, hq, hi, update=True)
    for e in range(E):
        rc, rp = oracle.field_distance(h.op, st1[e], agents, src, scale, hists[e])
        assert np.array_equal(d_cur[e].cpu().numpy(), rc)
        assert np.array_equal(d_prev[e].cpu().numpy(), rp)
    # the fused transform (gradient sensing: clipped at 0) on the next move
    st2 = []
    for s in st1:
        p = oracle.unwrapped(s, box)
        p[:, :2] += rng.uniform(-L, L, (n, 2))
        st2.append(oracle.state_from_positions(p, np.tile([1.0, 0, 0], (n, 1)), box))
    h.upload(st2)
    got = ops.field_transform(h.native, E, ag_t, src, scale, hq, hi, 1.0, -1.0, 10.0,
                              True).cpu().numpy()
    for e in range(E):
        rc, rp = oracle.field_distance(h.op, st2[e], agents, src, scale, hists[e])
        one, ten = np.float32(1.0), np.float32(10.0)
        ref = ten * ((one - rc) - (one - rp))
        ref = np.where(ref < 0, np.float32(0), ref).astype(np.float32)
        assert np.array_equal(got[e], ref)


def test_engine_made_images_vision_and_field_bit_exact(tmp_path):
    """The bench workload's physics in a box small enough that the swimmers
    leave it: after the engine's own integration, images are nonzero and
    mixed, and the vision cone and field kernels still equal the oracle on
    the engine's raw state."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import MDParams, SwarmEngine, ops
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    n = 1024
    L = 2.0 * np.sqrt(n / 0.1)  # 202.4: the bench's area fraction in the placement disc
    params = MDParams(ureg=ureg, box_length=ureg.Quantity([L, L, L], "micrometer"),
                      time_slice=ureg.Quantity(0.1, "second"),
                      write_interval=ureg.Quantity(100.0, "second"))
    eng = SwarmEngine(params, n_dims=2, seed=42, out_folder=str(tmp_path))
    eng.add_colloids(n, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([L / 2, L / 2, 0.0]), "micrometer"),
                     ureg.Quantity(L / 2, "micrometer"))
    ff = ForceFunction({"0": dummy_models.ConstForce(100.0)})  # ~21 um/s
    eng.integrate(1, ff)
    view = eng.swarm_view()
    agents = np.arange(n, dtype=np.int32)
    dev = torch.device("cuda", 0)
    ag_t = torch.as_tensor(agents, device=dev)
    hq = torch.zeros((3, n), dtype=torch.int32, device=dev)
    hi = torch.zeros((3, n), dtype=torch.int32, device=dev)
    src = np.array([L / 2, L / 2, 0.0])
    scale = np.array([L, L, L])
    ops.field_distance(eng._native, 1, ag_t, src, scale, hq, hi, update=True, init_only=True)
    raw0 = eng.get_raw_state()
    eng.integrate(40, ff)  # 4 s: ~85 um, across the box edge for the outer colloids
    raw = eng.get_raw_state()
    assert np.count_nonzero(raw["img"][:2]) > 20
    assert len(np.unique(raw["img"][:2])) >= 3
    key = eng._species_keys[0]
    p = oracle.make_params(eng._box, eng._time_step, eng._kT(),
                           params.WCA_epsilon.m_as("sim_energy"), 42, [key])
    st = {"q": raw["q"], "img": raw["img"], "ang": raw["ang"]}
    radii = np.ones(n, np.float32)
    types = np.zeros(n, np.int32)
    vp = ops.vision_params(10.0, np.pi / 2, 3, [0])
    out = ops.vision_cone(eng._native, 1, ag_t, torch.as_tensor(radii, device=dev),
                          torch.as_tensor(types, device=dev), vp).cpu().numpy()
    ref = oracle.vision_cone(p, st, agents, radii, types, 10.0, np.pi / 2, 3, [0])
    assert np.array_equal(out[0], ref)
    d_cur, d_prev = ops.field_distance(eng._native, 1, ag_t, src, scale, hq, hi, update=True)
    hist = oracle.history_from_state({"q": raw0["q"], "img": raw0["img"], "ang": raw0["ang"]},
                                     agents)
    rc, rp = oracle.field_distance(p, st, agents, src, scale, hist)
    assert np.array_equal(d_cur[0].cpu().numpy(), rc)
    assert np.array_equal(d_prev[0].cpu().numpy(), rp)
    del view


@pytest.mark.parametrize("R", [20.0, 35.0, 130.0])
def test_vision_range_beyond_half_box_bit_exact(R):
    """The reference has no range limit and no minimum image
    (subdivided_vision_cones.py:116-121): a vision range of half the box or
    more scans every record of the env on its unwrapped separation (the
    all-records variant of k_vision), bit-exact against the oracle, with
    colloids several images away."""
    from gpu_harness import Harness, species_list
    from swarmrl_amd.engine import ops

    rng = np.random.default_rng(22)
    L = 40.0
    box = [L, L, L]
    n, E = 700, 2
    types = rng.integers(0, 2, n)
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int), n_envs=E)
    states = []
    for _ in range(E):
        pos = np.zeros((n, 3))
        pos[:, :2] = rng.random((n, 2)) * L + rng.integers(-3, 4, (n, 2)) * L
        a = 2 * np.pi * rng.random(n)
        dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
        states.append(oracle.state_from_positions(pos, dirs, box))
    h.upload(states)
    agents = np.arange(0, n, 2, dtype=np.int32)
    radii = (0.5 + rng.random(n)).astype(np.float32)
    dev = torch.device("cuda", 0)
    vp = ops.vision_params(R, np.pi / 3, 4, [0, 1])
    out = ops.vision_cone(h.native, E, torch.as_tensor(agents, device=dev),
                          torch.as_tensor(radii, device=dev),
                          torch.as_tensor(types.astype(np.int32), device=dev), vp).cpu().numpy()
    for e in range(E):
        ref = oracle.vision_cone(h.op, states[e], agents, radii, types, R, np.pi / 3, 4, [0, 1])
        assert np.array_equal(out[e], ref)
        assert np.count_nonzero(ref) > 100
