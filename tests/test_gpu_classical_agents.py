"""
Classical neighbour-rule agents: Lavergne2019 and
Baeuerle2020 (bechinger_models.py) and Lymburn (lymburn_model.py) on the
fused fp64 neighbour kernel, against the numpy restatement of the
reference's loops (oracle/refsem.py; fp64 both, summation order differs:
rtol 1e-9).  Parity is pinned by the restatement only (the reference has no
unit test of these agents): "parity unpinned" beyond it.
"""

import numpy as np
import pytest
import torch

from oracle import refsem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


def _colloids(rng, n, L, types, vel=True):
    from swarmrl_amd.components import Colloid

    pos = rng.random((n, 3)) * L
    pos[:, 2] = 0.0
    a = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    v = rng.normal(size=(n, 3)) * 3.0 if vel else np.zeros((n, 3))
    v[:, 2] = 0.0
    cols = [Colloid(pos[i], dirs[i], i, velocity=v[i], type=int(types[i])) for i in range(n)]
    return cols, pos, dirs, v


def test_lavergne_matches_reference_loops():
    from swarmrl_amd.agents.bechinger_models import Lavergne2019

    rng = np.random.default_rng(1)
    n = 300
    types = rng.integers(0, 2, n)
    cols, pos, dirs, _ = _colloids(rng, n, 40.0, types)
    ag = Lavergne2019(vision_half_angle=np.pi / 3, act_force=2.5, perception_threshold=0.6,
                      acts_on_types=[0])
    acts = ag.calc_action(cols)
    ref = refsem.lavergne_forces(pos, dirs, types, np.pi / 3, 2.5, 0.6, [0])
    got = np.array([a.force for a in acts])
    assert np.array_equal(got, ref)
    assert 0 < np.count_nonzero(got) < np.count_nonzero(types == 0)


def test_baeuerle_matches_reference_loops():
    from swarmrl_amd.agents.bechinger_models import Baeuerle2020

    rng = np.random.default_rng(2)
    n = 250
    types = rng.integers(0, 2, n)
    cols, pos, dirs, _ = _colloids(rng, n, 50.0, types)
    ag = Baeuerle2020(act_force=3.0, act_torque=2.0, detection_radius_position=8.0,
                      detection_radius_orientation=5.0, vision_half_angle=np.pi / 2,
                      angular_deviation=0.7, acts_on_types=[0, 1])
    acts = ag.calc_action(cols)
    f_ref, t_ref = refsem.baeuerle_actions(pos, dirs, types, 3.0, 2.0, 8.0, 5.0, np.pi / 2, 0.7,
                                           [0, 1])
    got_f = np.array([a.force for a in acts])
    got_t = np.array([0.0 if a.torque is None else a.torque[2] for a in acts])
    assert np.array_equal(got_f, f_ref)
    np.testing.assert_allclose(got_t, t_ref, rtol=1e-9, atol=1e-12)
    assert np.count_nonzero(got_t) > 20


def test_lymburn_matches_reference_loops():
    from swarmrl_amd.agents.lymburn_model import Lymburn

    rng = np.random.default_rng(3)
    n = 200
    types = np.zeros(n, int)
    types[:3] = 1  # predators
    cols, pos, _, vel = _colloids(rng, n, 60.0, types)
    K = {"K_a": 0.3, "K_r": -1.5, "K_h": 0.05, "K_f": 0.2, "K_p": 4.0}
    ag = Lymburn(dict(K), detection_radius_position_colls=9.0,
                 detection_radius_position_pred=15.0, home_pos=np.array([30.0, 30.0, 0.0]),
                 agent_speed=5.0, predator_type=1)
    acts = ag.calc_action(cols)
    ref = refsem.lymburn_actions(pos, vel, types, K, 9.0, 15.0, np.array([30.0, 30.0, 0.0]),
                                 5.0, 1)
    assert len(acts) == len(ref) == n - 3
    for a, (fm, d) in zip(acts, ref):
        np.testing.assert_allclose(a.force, fm, rtol=1e-9)
        np.testing.assert_allclose(a.new_direction, d, rtol=1e-9, atol=1e-12)


def test_get_colloids_in_vision_matches_reference():
    from swarmrl_amd.agents.bechinger_models import get_colloids_in_vision

    rng = np.random.default_rng(4)
    cols, pos, dirs, _ = _colloids(rng, 100, 20.0, np.zeros(100, int))
    got = get_colloids_in_vision(cols[0], cols[1:], vision_half_angle=1.0, vision_range=6.0)
    ref = refsem.colloids_in_vision(pos[0], dirs[0], pos[1:], 1.0, 6.0)
    assert [c.id for c in got] == [1 + k for k in ref]


def test_bechinger_device_path_equals_list_path(tmp_path):
    """On a SwarmView the agents return DeviceActions equal to the list
    path's actions on the same state."""
    from swarmrl_amd.agents.bechinger_models import Baeuerle2020, Lavergne2019
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    p = MDParams(ureg=ureg, box_length=ureg.Quantity([60.0, 60.0, 60.0], "micrometer"))
    eng = SwarmEngine(p, n_dims=2, seed=5, out_folder=tmp_path)
    eng.add_colloids(150, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([30.0, 30.0, 0.0]), "micrometer"),
                     ureg.Quantity(25.0, "micrometer"), type_colloid=0)
    eng.integrate(1)
    view = eng.swarm_view()
    cols = eng.colloids
    from swarmrl_amd.components import Colloid

    lst = [Colloid(c.pos, c.director, c.id, velocity=c.v, type=c.type) for c in cols]
    for ag in (Lavergne2019(perception_threshold=0.3, act_force=4.0),
               Baeuerle2020(detection_radius_position=10.0, detection_radius_orientation=10.0)):
        dv = ag.calc_action(view)
        la = ag.calc_action(lst)
        np.testing.assert_array_equal(dv.f_swim[0].cpu().numpy(),
                                      np.array([a.force for a in la], np.float32))
        t_list = np.array([0.0 if a.torque is None else a.torque[2] for a in la], np.float32)
        np.testing.assert_allclose(dv.torque_z[0].cpu().numpy(), t_list, rtol=1e-6, atol=1e-6)
