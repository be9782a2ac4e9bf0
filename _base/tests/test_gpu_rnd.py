"""
The RND intrinsic reward's metric in one launch (swarm_rnd_distance) against
the torch forward of the same two networks (random_network_distillation.py:
126-143, rnd_configs.py:17-38).  fp32 with fused multiply-adds in a fixed
order vs hipBLASLt GEMMs: agreement within rtol 2e-5 / atol 2e-6 per
observation (parity vs ZnNL is unpinned: ZnNL is absent here).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


@pytest.mark.parametrize("d_in,order,n", [(1, 2, 16384), (3, 2, 1000), (7, 3, 513), (16, 2, 77)])
def test_rnd_distance_matches_torch(d_in, order, n):
    from swarmrl_amd.engine import ops
    from swarmrl_amd.intrinsic_reward.rnd_configs import RNDArchitecture, order_n_difference

    dev = torch.device("cuda", 0)
    torch.manual_seed(d_in * 10 + order)
    target = RNDArchitecture(d_in).to(dev)
    predictor = RNDArchitecture(d_in).to(dev)
    x = torch.randn(n, d_in, device=dev) * 3
    got = ops.rnd_distance(x, target, predictor, order)
    with torch.no_grad():
        ref = order_n_difference(target(x), predictor(x), order)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-6)
    # float64 restatement: the fused kernel is at least as close to it
    with torch.no_grad():
        t64 = target.double()(x.double())
        p64 = predictor.double()(x.double())
    ref64 = order_n_difference(t64, p64, order).float()
    torch.testing.assert_close(got, ref64, rtol=2e-5, atol=2e-6)


def test_rnd_reward_device_path_uses_the_fused_metric(monkeypatch):
    """RNDReward.compute_reward on device features [E, A, 1] (the C5 path):
    fused and torch metric give the same per-env clipped rewards."""
    from swarmrl_amd.intrinsic_reward import RNDConfig, RNDReward
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    rnd = RNDReward(RNDConfig(input_shape=(1,), device=dev))
    traj = TrajectoryInformation(particle_type=0)
    traj.features.append(torch.randn(4, 4096, 1, device=dev))
    calls = []
    from swarmrl_amd.engine import ops

    orig = ops.rnd_env_reward
    monkeypatch.setattr(ops, "rnd_env_reward", lambda *a, **k: calls.append(1) or orig(*a, **k))
    fused = rnd.compute_reward(traj)
    assert calls, "the fused metric was not used"
    monkeypatch.setattr(RNDReward, "_fused_ok", lambda self, p: False)
    ref = rnd.compute_reward(traj)
    assert fused.shape == (4, 1)
    torch.testing.assert_close(fused, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("E,A,clip", [(1, 16384, (-5.0, 5.0)), (3, 1000, None), (2, 77, (0.0, 0.1))])
def test_rnd_env_reward_added_to_task_reward(E, A, clip):
    """The agent's task + intrinsic sum on the device path (RNDReward.
    add_to_reward -> swarm_rnd_env_reward: metric, per-env fp64 mean, clip
    and the sum in two launches) against the torch composition of the same
    steps: torch metric, per-env mean, clamp, broadcast add (rtol 2e-5);
    ragged env sizes (not a multiple of the 256-observation blocks)."""
    from swarmrl_amd.intrinsic_reward import RNDConfig, RNDReward
    from swarmrl_amd.intrinsic_reward.rnd_configs import order_n_difference
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    dev = torch.device("cuda", 0)
    torch.manual_seed(E * 100 + A)
    rnd = RNDReward(RNDConfig(input_shape=(1,), device=dev, clip_rewards=clip))
    traj = TrajectoryInformation(particle_type=0)
    traj.features.append(torch.randn(E, A, 1, device=dev) * 2)
    base = torch.rand(E, A, device=dev)
    got = rnd.add_to_reward(base, traj)
    assert got.shape == (E, A)
    x = traj.features[-1].reshape(-1, 1)
    with torch.no_grad():
        m = order_n_difference(rnd.target_network(x), rnd.predictor_network(x), 2)
    torch.testing.assert_close(rnd.metric_results, m, rtol=2e-5, atol=2e-6)
    r = m.double().reshape(E, A).mean(dim=1, keepdim=True).float()
    if clip is not None:
        r = torch.clamp(r, *clip)
    torch.testing.assert_close(got, base + r, rtol=2e-5, atol=2e-6)
    # run-to-run: the fixed-order reduction gives the same bits
    again = rnd.add_to_reward(base, traj)
    assert torch.equal(got, again)

