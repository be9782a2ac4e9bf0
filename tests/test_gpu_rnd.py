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

    orig = ops.rnd_distance
    monkeypatch.setattr(ops, "rnd_distance", lambda *a: calls.append(1) or orig(*a))
    fused = rnd.compute_reward(traj)
    assert calls, "the fused metric was not used"
    monkeypatch.setattr(RNDReward, "_fused_ok", lambda self, p: False)
    ref = rnd.compute_reward(traj)
    assert fused.shape == (4, 1)
    torch.testing.assert_close(fused, ref, rtol=2e-5, atol=2e-6)
