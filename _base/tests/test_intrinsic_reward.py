"""
RND intrinsic reward (reference: swarmrl/intrinsic_reward/
random_network_distillation.py:16-149).  ZnNL (the reference's training
library) is absent, so parity is unpinned: the tests check the contract —
shapes, the reshape of (T, N, obs) data, clipping to clip_rewards, a scalar
mean reward — and that training the predictor lowers the reward on the
visited states but not on novel ones.
"""

import numpy as np
import torch

from swarmrl_amd.intrinsic_reward import RNDConfig, RNDReward
from swarmrl_amd.utils.colloid_utils import TrajectoryInformation


def _traj(features):
    t = TrajectoryInformation(particle_type=0)
    t.features = list(features)
    return t


def test_rnd_shapes_clip_and_novelty():
    torch.manual_seed(0)
    rnd = RNDReward(RNDConfig(input_shape=(3,), n_epochs=60, batch_size=32,
                              device=torch.device("cpu")))
    rng = np.random.default_rng(0)
    seen = torch.as_tensor(rng.normal(size=(10, 64, 3)), dtype=torch.float32)
    novel = torch.as_tensor(rng.normal(size=(1, 64, 3)) + 6.0, dtype=torch.float32)
    assert RNDReward._reshape_data(seen).shape == (640, 3)
    r0 = float(rnd.compute_reward(_traj(seen)))
    rnd.update(_traj(seen))
    r1 = float(rnd.compute_reward(_traj(seen)))
    rn = float(rnd.compute_reward(_traj(novel)))
    assert r1 < 0.5 * r0
    assert rn > r1
    assert -5.0 <= r0 <= 5.0 and rnd.metric_results.shape == (64,)
    rnd.clip_rewards = (0.0, 1e-6)
    assert float(rnd.compute_reward(_traj(novel))) <= 1e-6


def test_rnd_fused_path_only_for_the_stock_architecture():
    """k_rnd_distance hard-codes Linear(d, 32) -> ReLU -> Linear(32, 32) ->
    ReLU -> Linear(32, 32) read as contiguous fp32 rows: any other network
    swapped into RNDReward must take the torch path."""
    from swarmrl_amd.intrinsic_reward.rnd_configs import RNDArchitecture

    ok = RNDReward.fused_architecture_ok
    assert ok(RNDArchitecture(3), 3)
    assert not ok(RNDArchitecture(3), 2)          # in_features != the observation size
    tanh = RNDArchitecture(3)
    tanh.net[1] = torch.nn.Tanh()
    assert not ok(tanh, 3)
    norm = RNDArchitecture(3)
    norm.net.append(torch.nn.LayerNorm(32))
    assert not ok(norm, 3)
    wide = RNDArchitecture(3, width=64)
    assert not ok(wide, 3)
    trans = RNDArchitecture(3)
    with torch.no_grad():
        trans.net[2].weight = torch.nn.Parameter(trans.net[2].weight.detach().t().contiguous().t())
    assert not trans.net[2].weight.is_contiguous()
    assert not ok(trans, 3)
    half = RNDArchitecture(3).to(torch.float64)
    assert not ok(half, 3)
    assert not ok(torch.nn.Sequential(*RNDArchitecture(3).net), 3)
