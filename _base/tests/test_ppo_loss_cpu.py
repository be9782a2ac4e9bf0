"""
PPO loss and GAE on the CPU (torch path) against the reference's own
known-answer tests: CI/unit_tests/value_functions/test_gae.py:8-28 and
CI/unit_tests/losses/test_proximal_policy_loss.py:33-133 (dummy network
with logits 2 and values 1, dummy value function, three ratio regimes).
Plus the critic gradient of the reference's loss -- returns R = A + V stay
differentiable (proximal_policy_loss.py:101-124, only the normalised
advantages are stop_gradient-ed) -- checked against a float64 finite
difference of the loss, and the closed form the device kernel k_ppo_gae
uses (swarm_ppo.cuh) against both.  Also ExpectedReturns against
CI/unit_tests/value_functions/test_expected_returns.py and the
PolicyGradientLoss (policy_gradient_loss.py:47-106) against its formula.
"""

import numpy as np
import torch
import torch.nn.functional as F

from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
from swarmrl_amd.sampling_strategies.gumbel_distribution import GumbelDistribution
from swarmrl_amd.value_functions.generalized_advantage_estimate import GAE


def test_gae_reference_kat():
    gae = GAE(gamma=1, lambda_=1)
    rewards = torch.tensor([1.0, 1, 1, 1, 1])
    values = torch.tensor([1.0, 2, 3, 4, 5])
    expected = np.array([4.0, 2, 0, -2, -4])
    expected_returns = expected + values.numpy()
    expected = (expected - expected.mean()) / (expected.std() + np.finfo(np.float32).eps)
    adv, ret = gae(rewards, values)
    np.testing.assert_allclose(adv.numpy(), expected, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ret.numpy(), expected_returns, rtol=1e-4, atol=1e-4)


class _DummyNetwork:
    def __call__(self, features, obs_ndim=1):
        T, P = features.shape[0], features.shape[1]
        return 2.0 * torch.ones(T, P, 4), torch.ones(T, P, 1)


def _dummy_value_function(rewards, values):
    return torch.sign(rewards) * torch.ones_like(rewards), 2.0 * torch.ones_like(rewards)


def test_ppo_loss_reference_kat():
    eps, c_h, T, P = 0.2, 0.01, 20, 10
    strategy = GumbelDistribution()
    loss = ProximalPolicyLoss(value_function=_dummy_value_function,
                              sampling_strategy=strategy, entropy_coefficient=c_h)
    features = torch.ones(T, P, 4)
    actions = torch.ones(T, P, dtype=torch.int64)
    # ratio 1, e^2 > 1 + eps, e^-2 < 1 - eps
    olds = [2.0 * torch.ones(T, P), torch.zeros(T, P), 3.0 * torch.ones(T, P)]
    rewards_list = [torch.ones(T, P), -torch.ones(T, P)]
    logits = 2.0 * np.ones((T, P, 4))
    probs = np.exp(logits) / np.exp(logits).sum(-1, keepdims=True)
    new_logp = np.log(probs + 1e-8)[..., 1]
    entropy = -np.sum((probs + 1e-8) * np.log(probs + 1e-8))
    for old in olds:
        for rewards in rewards_list:
            got = float(loss._calculate_loss(_DummyNetwork(), features, actions, rewards, old))
            r = np.exp(new_logp - old.numpy())
            adv = np.sign(rewards.numpy())
            clipped = -np.minimum(r * adv, np.clip(r, 1 - eps, 1 + eps) * adv)
            huber = 0.5 * (1.0 - 2.0) ** 2  # |V - R| = 1 <= delta
            want = clipped.sum() - c_h * entropy + 0.5 * huber * T * P
            np.testing.assert_almost_equal(got, want, decimal=3)


def _gae64(rewards, values, gamma, lam):
    T = rewards.shape[0]
    adv = np.zeros_like(values)
    gae = np.zeros_like(values[0])
    for t in reversed(range(T)):
        nxt = gamma * values[t + 1] if t != T - 1 else 0.0
        gae = rewards[t] + nxt - values[t] + gamma * lam * gae
        adv[t] = gae
    return adv, adv + values


def _critic_loss64(rewards, values, gamma, lam):
    _, ret = _gae64(rewards, values, gamma, lam)
    d = values - ret
    hub = np.where(np.abs(d) <= 1.0, 0.5 * d * d, np.abs(d) - 0.5)
    return 0.5 * hub.sum()


def _critic_grad_closed_form(rewards, values, gamma, lam):
    """dL/dV as k_ppo_gae computes it (swarm_ppo.cuh): direct term minus the
    returns' dependence on later values, one forward pass per column."""
    adv, _ = _gae64(rewards, values, gamma, lam)
    g = 0.5 * np.clip(-adv, -1.0, 1.0)
    out = np.empty_like(g)
    carry = np.zeros_like(g[0])
    for t in range(g.shape[0]):
        out[t] = g[t] - gamma * (1.0 - lam) * carry
        carry = gamma * lam * carry + g[t]
    return out


def test_critic_gradient_flows_through_returns():
    rng = np.random.default_rng(3)
    T, S, gamma, lam = 12, 7, 0.99, 0.95
    rewards = rng.normal(0.0, 1.0, (T, S))
    values = rng.normal(0.0, 2.0, (T, S))
    closed = _critic_grad_closed_form(rewards, values, gamma, lam)
    # float64 central differences of the loss itself
    h = 1e-6
    fd = np.empty_like(values)
    for t in range(T):
        for s in range(S):
            vp, vm = values.copy(), values.copy()
            vp[t, s] += h
            vm[t, s] -= h
            fd[t, s] = (_critic_loss64(rewards, vp, gamma, lam)
                        - _critic_loss64(rewards, vm, gamma, lam)) / (2 * h)
    np.testing.assert_allclose(closed, fd, rtol=1e-6, atol=1e-7)
    # the torch loss differentiates the same way (GAE with autograd)
    v = torch.tensor(values, dtype=torch.float32, requires_grad=True)
    r = torch.tensor(rewards, dtype=torch.float32)
    _, ret = GAE(gamma, lam)(r, v)
    (0.5 * F.huber_loss(v, ret, reduction="sum", delta=1.0)).backward()
    np.testing.assert_allclose(v.grad.numpy(), closed, rtol=1e-4, atol=1e-5)


def test_expected_returns_reference_kats():
    """CI/unit_tests/value_functions/test_expected_returns.py:16-53."""
    from swarmrl_amd.value_functions.expected_returns import ExpectedReturns

    got = ExpectedReturns(gamma=1.0, standardize=False)(
        torch.tensor([[1.0, 4], [2, 5], [3, 6]]))
    np.testing.assert_array_equal(got.numpy(), [[6, 15], [5, 11], [3, 6]])
    rewards = torch.tensor([[1.0, 4], [2, 5], [3, 6], [4, 7], [5, 8], [6, 9], [7, 10]])
    got = ExpectedReturns(gamma=0.79, standardize=True)(rewards).numpy()
    np.testing.assert_array_almost_equal(got.mean(0), [0.0, 0.0], decimal=6)
    np.testing.assert_array_almost_equal(got.std(0), [1.0, 1.0], decimal=6)


def test_policy_gradient_loss_matches_hand_computation():
    """PolicyGradientLoss._calculate_loss (policy_gradient_loss.py:47-106) on
    a small random network against the formula evaluated in float64 numpy:
    -sum(log(p_a + 1e-8) (R - V)) + sum(huber(V, R)), R the standardised
    discounted returns (gamma 0.99); the critic gradient flows through V only."""
    from swarmrl_amd.losses.policy_gradient_loss import PolicyGradientLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP

    torch.manual_seed(0)
    net = ActorCriticMLP(3, 4, 16)
    T, P = 5, 7
    g = torch.Generator().manual_seed(1)
    x = torch.randn(T, P, 3, generator=g)
    actions = torch.randint(0, 4, (T, P), generator=g)
    rewards = torch.randn(T, P, generator=g)

    class Wrap:
        def __call__(self, features, obs_ndim=1):
            return net(features)

    loss = PolicyGradientLoss()._calculate_loss(Wrap(), x, actions, rewards)
    with torch.no_grad():
        logits, v = net(x)
    logits, v = logits.double().numpy(), v.double().numpy()[..., 0]
    p = np.exp(logits - logits.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    pa = np.take_along_axis(p, actions.numpy()[..., None], -1)[..., 0]
    r = rewards.double().numpy()
    ret = np.zeros_like(r)
    acc = np.zeros(P)
    for t in reversed(range(T)):
        acc = r[t] + 0.99 * acc
        ret[t] = acc
    ret = (ret - ret.mean(0)) / (ret.std(0) + np.finfo(np.float32).eps)
    d = v - ret
    hub = np.where(np.abs(d) <= 1.0, 0.5 * d * d, np.abs(d) - 0.5)
    want = -(np.log(pa + 1e-8) * (ret - v)).sum() + hub.sum()
    np.testing.assert_allclose(float(loss.detach()), want, rtol=1e-5)
    # critic gradient through V only: d/dV = clip(V - R, -1, 1) (returns fixed)
    net.zero_grad()
    vv = torch.tensor(v, requires_grad=True)
    F.huber_loss(vv, torch.tensor(ret), reduction="sum", delta=1.0).backward()
    np.testing.assert_allclose(vv.grad.numpy(), np.clip(d, -1, 1), rtol=1e-12)
