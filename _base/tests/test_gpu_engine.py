"""
GPU tests through the product's Python surface (the SwarmRL-compatible API):
reference known answers, device path == list path, a full PPO training run,
and size-independent statistics of the noisy dynamics at full size.
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


def _params(ureg, **kw):
    from swarmrl_amd.engine import MDParams

    return MDParams(ureg=ureg, **kw)


# ------------------------------------------------ reference unit-test KATs
def test_vision_cone_kat_product_list_path():
    from swarmrl_amd.components import Colloid
    from swarmrl_amd.observables import SubdividedVisionCones

    vc = SubdividedVisionCones(vision_range=10, vision_half_angle=np.pi / 2, n_cones=3,
                               radii=[1, 2, 3, 4, 1], particle_type=0)
    cols = [
        Colloid(np.array([0, 0, 0]), np.array([0, 1.0, 0]), 0, np.array([0, 0, 0]), 0),
        Colloid(np.array([0, 5, 0]), np.array([1.0, 0, 0]), 1, np.array([0, 0, 0]), 0),
        Colloid(np.array([0, 8, 0]), np.array([1.0, 0, 0]), 2, np.array([0, 0, 0]), 1),
        Colloid(np.array([-7, 8, 0]), np.array([0.0, 1.0, 0]), 3, np.array([0, 0, 0]), 1),
        Colloid(np.array([1, 1, 0]), np.array([0.0, 1.0, 0]), 4, np.array([0, 0, 0]), 0),
    ]
    obs = vc.compute_observable(cols)[0]
    assert obs[0, 0] == 1.0
    assert obs[1, 0] == 0.8
    assert obs[2, 0] == 0.0
    assert obs[0, 1] == 0.0
    assert obs[1, 1] == 0.75
    assert obs[2, 1] == 0.0


def test_concentration_field_kat_product():
    from swarmrl_amd.components import Colloid
    from swarmrl_amd.observables import ConcentrationField

    ob = ConcentrationField(source=np.array([0.5, 0.5, 0.0]), decay_fn=lambda x: -1 * x,
                            box_length=np.array([1.0, 1.0, 1.0]), particle_type=0)
    old = [Colloid(np.array([0.0, 0.0, 0.0]), np.array([0.0, 1.0, 0]), 0, 0),
           Colloid(np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 1, 0),
           Colloid(np.array([1.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 2, 0)]
    ob.initialize(old)
    assert list(ob._historic_positions.keys()) == ["0", "1", "2"]
    np.testing.assert_array_equal(ob._historic_positions["1"], [0.0, 1.0, 0.0])
    assert ob.scale_factor == 100.0
    new = [Colloid(np.array([1.0, 0.0, 0.0]), np.array([0.0, 1.0, 0]), 0, 0),
           Colloid(np.array([1.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 1, 0),
           Colloid(np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 2, 0)]
    obs = ob.compute_observable(new)
    expect = np.array([
        -100 * (np.linalg.norm(n.pos - ob.source) - np.linalg.norm(o.pos - ob.source))
        for n, o in zip(new, old)
    ]).reshape(-1, 1)
    np.testing.assert_array_equal(obs, expect)
    with pytest.raises(ValueError):
        ConcentrationField(np.zeros(3), lambda x: x, np.ones(3)).compute_observable(new)


def test_gradient_sensing_kat_product():
    from swarmrl_amd.components import Colloid
    from swarmrl_amd.tasks.searching import GradientSensing

    task = GradientSensing(source=np.array([0.5, 0.5, 0.0]), decay_function=lambda x: 1 - x,
                           box_length=np.array([1.0, 1.0, 1.0]), particle_type=0,
                           reward_scale_factor=1)
    old = [Colloid(np.array([0.0, 0.0, 0.0]), np.array([0.0, 1.0, 0]), 0, 0),
           Colloid(np.array([0.0, 0.6, 0.0]), np.array([0.0, 1.0, 0]), 1, 0),
           Colloid(np.array([1.0, 0.0, 0.0]), np.array([0.0, 1.0, 0]), 2, 0)]
    task.initialize(old)
    new = [Colloid(np.array([0.2, 0.2, 0.0]), np.array([0.0, 1.0, 0]), 0, 0),
           Colloid(np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 1, 0),
           Colloid(np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 2, 0)]
    r = task(new)
    d1 = np.linalg.norm(new[0].pos - task.source)
    d0 = np.linalg.norm(old[0].pos - task.source)
    assert r[0] > 0 and r[0] == pytest.approx((1 - d1) - (1 - d0), rel=1e-6)
    assert r[1] == 0.0
    assert r[2] == 0.0


# ------------------------------------------------------ engine semantics
def _engine(ureg, tmp_path, n, L, seed=42, n_envs=1, **kw):
    from swarmrl_amd.engine import SwarmEngine

    p = _params(ureg, box_length=ureg.Quantity([L, L, L], "micrometer"), **kw)
    eng = SwarmEngine(p, n_dims=2, seed=seed, out_folder=tmp_path, write_chunk_size=1,
                      n_envs=n_envs)
    eng.add_colloids(n, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([L / 2, L / 2, 0.0]), "micrometer"),
                     ureg.Quantity(L / 2 - 2, "micrometer"), type_colloid=1)
    return eng


def test_kt0_drift_and_velocity_kat(tmp_path):
    """test_espresso.py:89-111 in 2-D: rotate to a fixed director, then
    ConstForce(1.234): v = F d / gamma_t and x = x0 + t v (rtol 2e-6)."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    eng = _engine(ureg, tmp_path, 5, 1000.0,
                  fluid_dyn_viscosity=ureg.Quantity(8.9e-3, "pascal * second"),
                  WCA_epsilon=ureg.Quantity(1e-20, "joule"),
                  temperature=ureg.Quantity(0, "kelvin"),
                  time_step=ureg.Quantity(0.01, "second"),
                  time_slice=ureg.Quantity(0.1, "second"),
                  write_interval=ureg.Quantity(0.1, "second"))
    old = eng.get_particle_data()
    direc = np.array([1 / np.sqrt(2), 1 / np.sqrt(2), 0])
    eng.integrate(1, ForceFunction({"1": dummy_models.ToConstDirection(direc)}))
    eng.system.time = 0.0
    for d in eng.get_particle_data()["Directors"]:
        np.testing.assert_array_almost_equal(d, direc)
    force = 1.234
    eng.integrate(10, ForceFunction({"1": dummy_models.ConstForce(force)}))
    new = eng.get_particle_data()
    gt, _ = eng.get_friction_coefficients(1)
    for v in new["Velocities"]:
        np.testing.assert_array_almost_equal(v, force * direc / gt)
    # reuse_forces (espresso.py:1304-1306): the first sub-step of the 10
    # slices still swims with the rotation slice's zero force, so the drift
    # lasts t - dt.  (The reference's x0 + t v at rtol 2e-6 admits that lag,
    # dt v = 3e-4 um, only where |x| > 150 um; this port's seed places a
    # colloid at x = 77 um.)
    dt = eng.params.time_step.m_as("second")
    np.testing.assert_allclose(
        old["Unwrapped_Positions"] + (eng.system.time - dt) * force * direc / gt,
        new["Unwrapped_Positions"], rtol=2e-6)
    eng.finalize()


def test_isotropic_2d_rotation_and_set_direction(tmp_path):
    """test_espresso_2d.py:29-92."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    eng = _engine(ureg, tmp_path, 14, 1000.0,
                  fluid_dyn_viscosity=ureg.Quantity(8.9e-4, "pascal * second"),
                  WCA_epsilon=ureg.Quantity(1e-20, "joule"),
                  temperature=ureg.Quantity(300, "kelvin"),
                  time_step=ureg.Quantity(0.05, "second"),
                  time_slice=ureg.Quantity(0.1, "second"),
                  write_interval=ureg.Quantity(0.1, "second"))
    d0 = eng.get_particle_data()["Directors"]
    np.testing.assert_allclose(eng.get_particle_data()["Unwrapped_Positions"][:, 2], 0)
    eng.integrate(10, ForceFunction({"1": dummy_models.ConstForce(force=0)}))
    d1 = eng.get_particle_data()["Directors"]
    np.testing.assert_array_almost_equal(d1[:, 2], 0)
    assert not np.allclose(d0, d1, atol=1e-6)
    orientation = np.array([1 / np.sqrt(2), 1 / np.sqrt(2), 0])
    eng.manage_forces(ForceFunction({"1": dummy_models.ToConstDirection(orientation)}))
    for d in eng.get_particle_data()["Directors"]:
        np.testing.assert_array_almost_equal(d, orientation)


def test_device_path_equals_list_path(tmp_path, monkeypatch):
    """The batched SwarmView path and the reference list-of-Colloid path give
    bit-identical engine states (same actions, same kernels)."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    states = []
    for use_device in (True, False):
        ureg = UnitRegistry()
        eng = _engine(ureg, tmp_path / str(use_device), 300, 120.0)
        if not use_device:
            monkeypatch.setattr(SwarmEngine, "_device_capable", staticmethod(lambda fm: False))
        ff = ForceFunction({"1": dummy_models.ConstForceAndTorque(4.0, np.array([0, 0, 3.0]))})
        eng.integrate(3, ff)
        states.append(eng.get_raw_state())
        monkeypatch.undo()
    for k in ("q", "img", "ang"):
        assert np.array_equal(states[0][k], states[1][k])


@pytest.mark.parametrize("n_envs,n", [(1, 300), (12, 3000)])
def test_prebuild_overlap_equals_serial(tmp_path, n_envs, n):
    """The build forked on a side stream (latency-bound engines: launched
    first; throughput-bound ones, E x N > 32768: forked first, launched after
    the observables) gives the same bits as the serial single-stream slice."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    states = []
    for overlap in (True, False):
        ureg = UnitRegistry()
        eng = _engine(ureg, tmp_path / str(overlap), n, 2.0 * np.sqrt(n / 0.1), n_envs=n_envs)
        eng.overlap_build = overlap
        ff = ForceFunction({"1": dummy_models.ConstForceAndTorque(4.0, np.array([0, 0, 3.0]))})
        eng.integrate(3, ff)
        states.append(eng.get_raw_state())
    for k in ("q", "img", "ang"):
        assert np.array_equal(states[0][k], states[1][k])


def test_observables_device_vs_list(tmp_path):
    from swarmrl_amd.components import Colloid
    from swarmrl_amd.observables import SubdividedVisionCones
    from swarmrl_amd.units import UnitRegistry
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction

    ureg = UnitRegistry()
    n = 500
    eng = _engine(ureg, tmp_path, n, 150.0)
    eng.integrate(1, ForceFunction({"1": dummy_models.ConstForce(5.0)}))
    vc = SubdividedVisionCones(12.0, 1.1, 4, radii=[1.0] * n, particle_type=1)
    dev = vc.compute_observable(eng.swarm_view())[0].cpu().numpy()
    data = eng.get_particle_data()
    cols = [Colloid(data["Unwrapped_Positions"][i], data["Directors"][i], i, None, 1)
            for i in range(n)]
    lst = np.stack(vc.compute_observable(cols))
    # the list path re-quantises fp64 positions into a virtual box: equal up
    # to fp32 rounding, except a colloid exactly on a cone rim
    bad = np.abs(dev - lst) > 1e-5
    assert bad.sum() <= 2


def test_ppo_training_device_path(tmp_path):
    """ContinuousTrainer (swarmrl_amd.trainers, the reference's
    continuous_trainer.py:22-89) + ActorCriticAgent (vision cones, gradient
    sensing, PPO) entirely on the device path."""
    from swarmrl_amd.actions import Action
    from swarmrl_amd.agents import ActorCriticAgent
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel
    from swarmrl_amd.observables import SubdividedVisionCones
    from swarmrl_amd.tasks.searching import GradientSensing
    from swarmrl_amd.trainers import ContinuousTrainer
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    n, L = 200, 100.0
    eng = _engine(ureg, tmp_path, n, L, n_envs=2,
                  time_slice=ureg.Quantity(0.1, "second"),
                  write_interval=ureg.Quantity(1.0, "second"))
    net = TorchModel(ActorCriticMLP(3, 4, 32), input_shape=(3,), rng_key=3)
    before = [p.detach().clone() for p in net.model.parameters()]
    actions = {"a": Action(torque=np.array([0, 0, 10.0])), "b": Action(force=10.0),
               "c": Action(torque=np.array([0, 0, -10.0])), "d": Action()}
    agent = ActorCriticAgent(
        1, net, GradientSensing(np.array([L / 2, L / 2, 0]), lambda d: 1 - d,
                                np.array([L, L, L]), 10, particle_type=1),
        SubdividedVisionCones(10.0, np.pi / 2, 3, [1.0] * n, particle_type=1), actions)
    agent.loss.n_epochs = 3
    rewards = ContinuousTrainer([agent]).perform_rl_training(eng, n_episodes=3, episode_length=4,
                                                              load_bar=False)
    assert rewards.shape == (4,) and np.all(np.isfinite(rewards))
    after = list(net.model.parameters())
    assert any(not torch.equal(a, b) for a, b in zip(after, before))


# --------------------------------------------------- statistics, full size
def test_free_diffusion_statistics_4096(tmp_path):
    """MSD = 4 D_t t and <cos dtheta> = exp(-D_r t) at 4096 colloids x 2 envs."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    n = 4096
    L = 2 * np.sqrt(n / 0.1)
    # 1e-26 J ~ 2.5e-6 sim energy: no repulsion (1e-20 J would be ~2.5 kT)
    eng = _engine(ureg, tmp_path, n, L, n_envs=2,
                  WCA_epsilon=ureg.Quantity(1e-26, "joule"),
                  write_interval=ureg.Quantity(100.0, "second"))
    ff = ForceFunction({"1": dummy_models.ConstForce(0.0)})
    eng.integrate(1, ff)
    p0 = eng.get_particle_data()
    eng.integrate(10, ff)  # t = 1 s
    p1 = eng.get_particle_data()
    gt, gr = eng.get_friction_coefficients(1)
    kT = eng._kT()
    t = 1.0
    disp = p1["Unwrapped_Positions"] - p0["Unwrapped_Positions"]
    msd = np.mean(np.sum(disp[..., :2] ** 2, axis=-1))
    assert msd == pytest.approx(refsem.expected_msd_2d(kT, gt, t), rel=0.04)
    cosd = np.mean(np.sum(p0["Directors"] * p1["Directors"], axis=-1))
    assert cosd == pytest.approx(refsem.expected_orientation_corr(kT, gr, t), abs=0.02)
    # the two envs are independent replicas (own placement, own noise)
    assert not np.allclose(disp[0], disp[1])


def test_wca_slows_self_diffusion(tmp_path):
    """Property check at full size: with WCA on, collisions reduce the MSD
    below the free value (the reference's epsilon = k_B 300 K)."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    n = 4096
    L = 2 * np.sqrt(n / 0.3)  # area fraction 0.3
    eng = _engine(ureg, tmp_path, n, L, write_interval=ureg.Quantity(100.0, "second"))
    ff = ForceFunction({"1": dummy_models.ConstForce(0.0)})
    eng.integrate(1, ff)
    p0 = eng.get_particle_data()
    eng.integrate(10, ff)
    p1 = eng.get_particle_data()
    gt, _ = eng.get_friction_coefficients(1)
    msd = np.mean(np.sum((p1["Unwrapped_Positions"] - p0["Unwrapped_Positions"])[:, :2] ** 2, 1))
    assert msd < 0.95 * refsem.expected_msd_2d(eng._kT(), gt, 1.0)


# ------------------------------------- 3-D and walls (reference unit tests)
def test_espresso_3d_kat(tmp_path):
    """test_espresso.py:20-118 as written (n_dims = 3, the reference's
    default): two types added at random in a 500 um ball, ToConstDirection
    to (1,1,1)/sqrt(3), then 10 slices of ConstForce(1.234) at kT = 0:
    v = F d / gamma_t and x = x0 + t v (rtol 2e-6); WCA cutoff = 2 r; the
    trajectory file holds the last positions/velocities/time."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    params = _params(ureg, fluid_dyn_viscosity=ureg.Quantity(8.9e-3, "pascal * second"),
                     WCA_epsilon=ureg.Quantity(1e-20, "joule"),
                     temperature=ureg.Quantity(0, "kelvin"),
                     box_length=ureg.Quantity(3 * [1000], "micrometer"),
                     time_step=ureg.Quantity(0.01, "second"),
                     time_slice=ureg.Quantity(0.1, "second"),
                     write_interval=ureg.Quantity(0.1, "second"))
    runner = SwarmEngine(params, out_folder=tmp_path, write_chunk_size=1)
    assert runner.n_dims == 3 and runner.colloids == []
    coll_radius = ureg.Quantity(1, "micrometer")
    center = ureg.Quantity(np.array(3 * [500]), "micrometer")
    runner.add_colloids(2, coll_radius, center, ureg.Quantity(500, "micrometer"), type_colloid=1)
    runner.add_colloids(3, coll_radius, center, ureg.Quantity(500, "micrometer"), type_colloid=2)
    old = runner.get_particle_data()
    assert np.ptp(old["Unwrapped_Positions"][:, 2]) > 1.0  # a 3-D placement
    direc = np.array([1 / np.sqrt(3), 1 / np.sqrt(3), 1 / np.sqrt(3)])
    rot = dummy_models.ToConstDirection(direc)
    runner.integrate(1, ForceFunction({"1": rot, "2": rot}))
    runner.system.time = 0.0
    for d in runner.get_particle_data()["Directors"]:
        np.testing.assert_array_almost_equal(d, direc)
    force = 1.234
    cf = dummy_models.ConstForce(force)
    runner.integrate(10, ForceFunction({"1": cf, "2": cf}))
    runner._update_traj_holder()
    runner.write_idx += 1
    runner._write_traj_chunk_to_file()
    new = runner.get_particle_data()
    gt, _ = runner.get_friction_coefficients(1)
    for v in new["Velocities"]:
        np.testing.assert_array_almost_equal(v, force * direc / gt)
    np.testing.assert_allclose(old["Unwrapped_Positions"]
                               + runner.system.time * new["Velocities"],
                               new["Unwrapped_Positions"], rtol=2e-6)
    sigma = (2 * coll_radius.m_as("sim_length")) * 2 ** (-1 / 6)
    np.testing.assert_allclose(sigma * 2 ** (1 / 6), 2 * coll_radius.m_as("sim_length"))
    runner.finalize()


def test_confining_walls_3d_engine(tmp_path):
    """test_confining_walls.py: 3-D, five colloids in a 10 um box with box
    walls, ConstForce(10) for 300 slices: everyone stays inside (< 10)."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    params = _params(ureg, fluid_dyn_viscosity=ureg.Quantity(8.9e-4, "pascal * second"),
                     WCA_epsilon=0.1 * ureg.Quantity(300, "kelvin") * ureg.boltzmann_constant,
                     temperature=ureg.Quantity(300, "kelvin"),
                     box_length=ureg.Quantity(3 * [10], "micrometer"),
                     time_step=ureg.Quantity(0.0001, "second"),
                     time_slice=ureg.Quantity(0.1, "second"),
                     write_interval=ureg.Quantity(0.1, "second"))
    runner = SwarmEngine(params, n_dims=3, out_folder=tmp_path, write_chunk_size=1)
    coll_type = 1
    runner.add_colloids(5, radius_colloid=ureg.Quantity(1.0, "micrometer"),
                        random_placement_center=ureg.Quantity(np.array(3 * [5.0]), "micrometer"),
                        random_placement_radius=ureg.Quantity(4, "micrometer"),
                        type_colloid=coll_type)
    with pytest.raises(ValueError):
        runner.add_confining_walls(coll_type)
    runner.add_confining_walls(coll_type + 1)
    assert len(runner.system.constraints) == 2 * runner.n_dims
    runner.integrate(300, ForceFunction({"0": dummy_models.ConstForce(force=10)}))
    poss = runner.get_particle_data()["Unwrapped_Positions"]
    assert np.all(poss < 10)
    assert np.all(poss > 0)


def test_add_walls_2d_engine(tmp_path):
    """test_add_walls.py: 2-D, five colloids inside a square of four 2 um
    thick walls (40..60 um), ConstForce(10) on type 0 for 300 slices: the
    colloids stay within (40, 60)."""
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.engine import SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    params = _params(ureg, fluid_dyn_viscosity=ureg.Quantity(8.9e-4, "pascal * second"),
                     WCA_epsilon=0.1 * ureg.Quantity(300, "kelvin") * ureg.boltzmann_constant,
                     temperature=ureg.Quantity(300, "kelvin"),
                     box_length=ureg.Quantity(3 * [100], "micrometer"),
                     time_step=ureg.Quantity(0.005, "second"),
                     time_slice=ureg.Quantity(0.1, "second"),
                     write_interval=ureg.Quantity(0.1, "second"))
    runner = SwarmEngine(params, n_dims=2, out_folder=tmp_path, write_chunk_size=1)
    coll_type = 1
    runner.add_colloids(5, radius_colloid=ureg.Quantity(1.0, "micrometer"),
                        random_placement_center=ureg.Quantity(np.array([50, 50, 0]),
                                                              "micrometer"),
                        random_placement_radius=ureg.Quantity(4, "micrometer"),
                        type_colloid=coll_type)
    start = ureg.Quantity(np.array([[40, 40], [40, 40], [60, 60], [60, 60]]), "micrometer")
    end = ureg.Quantity(np.array([[40, 60], [60, 40], [40, 60], [60, 40]]), "micrometer")
    thickness = ureg.Quantity(2, "micrometer")
    with pytest.raises(ValueError):
        runner.add_walls(start, end, coll_type, thickness)
    runner.add_walls(start, end, coll_type + 1, thickness)
    assert len(runner.system.constraints) == 4
    runner.integrate(300, ForceFunction({"0": dummy_models.ConstForce(force=10)}))
    poss = np.array(runner.get_particle_data()["Unwrapped_Positions"])
    assert np.all(poss[:, :2] < 60)
    assert np.all(poss[:, :2] > 40)
    assert runner.wall_violations() == 0


@pytest.mark.parametrize("E,N", [(1, 1024), (8, 1024), (1, 4096)])
def test_bench_workload_build_modes_bit_identical(E, N):
    """The bench workload (vision cones, actor-critic sampling, GradientSensing
    reward) over 4 slices of one integrate call, the next window's cluster
    build (a) riding along in the vision-cone and policy launches
    (swarm_engine_defer_build, the default for latency-bound engines),
    (b) forked onto a side stream beside the observables and policy, (c) in
    the serial single-stream slice: the same positions, observables, actions
    and rewards, bit for bit.  Also (d) the ride-along episode captured in a
    HIP graph and replayed."""
    import argparse
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dev = torch.device("cuda", 0)
    out = []
    for mode in ("ride", "fork", "serial", "graph"):
        ns = argparse.Namespace(colloids=N, envs_per_gpu=E)
        eng, ff, agent = bench.build_workload(ns, 7, dev)
        eng.overlap_build = mode != "serial"
        eng.ride_along_build = mode in ("ride", "graph")
        if mode == "graph":
            eng.integrate(1, ff)  # set-up, overlap removal (eager), first slice
            st0 = eng.get_raw_state()
            agent.reset_trajectory()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                eng.integrate(3, ff)
            # capture does not run the work: restart from the first slice's state
            eng.set_raw_state(st0["q"], st0["img"], st0["ang"])
            g.replay()
            torch.cuda.synchronize()
        else:
            eng.integrate(1, ff)
            agent.reset_trajectory()
            eng.integrate(3, ff)
        assert eng._ride_along == (mode in ("ride", "graph"))
        st = eng.get_raw_state()
        tr = agent.trajectory
        out.append((mode, st, torch.stack([torch.as_tensor(a) for a in tr.actions]).cpu(),
                    torch.stack([torch.as_tensor(r) for r in tr.rewards]).cpu(),
                    torch.stack([torch.as_tensor(f) for f in tr.features]).cpu()))
    ref = out[0]
    for mode, st, a, r, f in out[1:]:
        for k in ("q", "img", "ang"):
            assert np.array_equal(ref[1][k], st[k]), (mode, k)
        assert torch.equal(ref[2], a) and torch.equal(ref[3], r) and torch.equal(ref[4], f), mode


def test_bench_workload_overlap_equals_serial():
    """The bench workload (vision cones, actor-critic sampling, GradientSensing
    reward) over 4 slices of one integrate call: the build on a side stream
    beside the observables and policy gives the same positions, actions and
    rewards as the serial single-stream slice."""
    import argparse
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dev = torch.device("cuda", 0)
    out = []
    for overlap in (True, False):
        ns = argparse.Namespace(colloids=1024, envs_per_gpu=1)
        eng, ff, agent = bench.build_workload(ns, 7, dev)
        eng.overlap_build = overlap
        eng.integrate(4, ff)
        st = eng.get_raw_state()
        tr = agent.trajectory
        out.append((st, torch.stack([torch.as_tensor(a) for a in tr.actions]).cpu(),
                    torch.stack([torch.as_tensor(r) for r in tr.rewards]).cpu()))
    (s0, a0, r0), (s1, a1, r1) = out
    for k in ("q", "img", "ang"):
        assert np.array_equal(s0[k], s1[k])
    assert torch.equal(a0, a1) and torch.equal(r0, r1)
