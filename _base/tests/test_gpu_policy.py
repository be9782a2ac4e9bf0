"""
Fused action sampling (swarm_sample_actions) against the reference's
definitions: Gumbel-max sampling (gumbel_distribution.py:37-40), the chosen
log-probability log(softmax + 1e-8) (flax_network.py:185-192), random
exploration (random_exploration.py:54-71) and the action-table lookup
(actor_critic.py:159-184).  Draws differ from JAX's threefry stream, so the
sampling is checked statistically, the rest exactly.
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


def _tables(dev):
    return (torch.tensor([0.0, 10.0, 0.0, 0.0], device=dev),
            torch.tensor([10.0, 0.0, -10.0, 0.0], device=dev))


def test_sampling_frequencies_logp_and_tables():
    from swarmrl_amd.engine import ops

    dev = torch.device("cuda", 0)
    n = 400_000
    row = torch.tensor([0.1, 1.0, -0.5, 0.3], device=dev)
    logits = row.repeat(n, 1)
    state = ops.counter_state(None, n, dev)
    ftab, ttab = _tables(dev)
    idx, logp, f, t = ops.sample_actions(logits, 1234, state, 0.0, ftab, ttab)
    freq = torch.bincount(idx, minlength=4).double().cpu().numpy() / n
    p = torch.softmax(row.double(), 0).cpu().numpy()
    assert np.all(np.abs(freq - p) < 4 * np.sqrt(p * (1 - p) / n) + 1e-4), (freq, p)
    ref_logp = torch.log(torch.softmax(logits, -1) + 1e-8).gather(1, idx[:, None])[:, 0]
    assert torch.allclose(logp, ref_logp, rtol=0, atol=2e-6)
    assert torch.equal(f, ftab[idx]) and torch.equal(t, ttab[idx])
    assert state.numel() == (n + 63) // 64 and bool((state == 1).all())


def test_counter_advances_and_seed_determinism():
    from swarmrl_amd.engine import ops

    dev = torch.device("cuda", 0)
    logits = torch.zeros(10_000, 4, device=dev)
    ftab, ttab = _tables(dev)
    s1 = ops.counter_state(None, 10_000, dev)
    s2 = ops.counter_state(None, 10_000, dev)
    a = ops.sample_actions(logits, 7, s1, 0.0, ftab, ttab)[0]
    b = ops.sample_actions(logits, 7, s2, 0.0, ftab, ttab)[0]
    c = ops.sample_actions(logits, 7, s1, 0.0, ftab, ttab)[0]
    assert torch.equal(a, b)  # same seed, same counter
    assert not torch.equal(a, c)  # counter advanced
    d = ops.sample_actions(logits, 8, torch.zeros_like(s1), 0.0, ftab, ttab)[0]
    assert not torch.equal(a, d)


def test_exploration_probability_one_is_uniform():
    from swarmrl_amd.engine import ops

    dev = torch.device("cuda", 0)
    n = 200_000
    logits = torch.tensor([[50.0, 0.0, 0.0, 0.0]], device=dev).repeat(n, 1)
    state = ops.counter_state(None, n, dev)
    ftab, ttab = _tables(dev)
    idx0 = ops.sample_actions(logits, 3, state, 0.0, ftab, ttab)[0]
    assert bool((idx0 == 0).all())  # greedy without exploration
    idx1 = ops.sample_actions(logits, 3, state, 1.0, ftab, ttab)[0]
    freq = torch.bincount(idx1, minlength=4).double().cpu().numpy() / n
    assert np.all(np.abs(freq - 0.25) < 0.01), freq


def test_agent_uses_fused_path_under_graph_capture(tmp_path):
    """The actor-critic device path runs the fused kernel inside a captured
    HIP graph and draws new actions on every replay."""
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = TorchModel(ActorCriticMLP(3, 4, 32), input_shape=(3,), device=dev)
    obs = torch.randn(4096, 3, device=dev)
    ftab, ttab = _tables(dev)
    assert net.fused_sampling_ok(obs)
    out = {}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        net.compute_action_fused(obs, ftab, ttab)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out["r"] = net.compute_action_fused(obs, ftab, ttab)
    g.replay()
    first = out["r"][0].clone()
    g.replay()
    assert not torch.equal(first, out["r"][0])
    logits, _ = net.model(obs)
    ref = torch.log(torch.softmax(logits, -1) + 1e-8).gather(1, out["r"][0][:, None])[:, 0]
    assert torch.allclose(out["r"][1], ref, atol=1e-5)


@pytest.mark.parametrize("n,d_in,hidden,k", [(4096, 3, 128, 4), (1000, 9, 64, 6),
                                             (40_000, 3, 128, 4), (100_000, 16, 256, 16),
                                             (100_001, 3, 128, 4)])
def test_fused_mlp_policy_matches_torch_and_sampler(n, d_in, hidden, k):
    """swarm_policy_mlp_sample: logits within fp32 tolerance of the torch
    module (rtol 1e-5, atol 1e-5: summation order differs from the GEMM), and
    the sampled actions/log-probs bit-identical to swarm_sample_actions on the
    kernel's own logits with the same counters; counters advance by one.
    Covers the 4/2/1 lanes-per-agent variants and the padded widths."""
    from swarmrl_amd.engine import ops
    from swarmrl_amd.networks import ActorCriticMLP

    dev = torch.device("cuda", 0)
    torch.manual_seed(n + d_in)
    net = ActorCriticMLP(d_in, k, hidden).to(dev)
    obs = torch.randn(n, d_in, device=dev) * 3.0
    ftab = torch.arange(k, dtype=torch.float32, device=dev) * 2.0
    ttab = -torch.arange(k, dtype=torch.float32, device=dev)
    state = ops.counter_state(None, n, dev)
    state += 5
    ref_state = state.clone()
    w1, b1, w2, b2 = net.rollout_layers()
    with torch.no_grad():
        idx, logp, f, t, lg = ops.policy_mlp_sample(obs, w1, b1, w2, b2, 99, state, 0.0, ftab,
                                                    ttab, want_logits=True)
        ref_logits, _ = net(obs)
    torch.testing.assert_close(lg, ref_logits, rtol=1e-5, atol=1e-5)
    i2, lp2, f2, t2 = ops.sample_actions(lg, 99, ref_state, 0.0, ftab, ttab)
    assert torch.equal(idx, i2) and torch.equal(logp, lp2)
    assert torch.equal(f, ftab[idx]) and torch.equal(t, ttab[idx])
    assert torch.equal(state, ref_state) and bool((state == 6).all())


def test_fused_mlp_policy_exploration_and_agent_path():
    """Exploration through the fused kernel (p = 1: uniform), and the agent
    picks the one-kernel path for the stock MLP."""
    from swarmrl_amd.engine import ops
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    n = 200_000
    torch.manual_seed(1)
    net = ActorCriticMLP(3, 4, 32).to(dev)
    with torch.no_grad():
        net.actor.bias.copy_(torch.tensor([60.0, 0.0, 0.0, 0.0]))
        net.actor.weight.zero_()
    obs = torch.randn(n, 3, device=dev)
    ftab, ttab = _tables(dev)
    state = ops.counter_state(None, n, dev)
    idx0 = ops.policy_mlp_sample(obs, *net.rollout_layers(), 5, state, 0.0, ftab, ttab)[0]
    assert bool((idx0 == 0).all())
    idx1 = ops.policy_mlp_sample(obs, *net.rollout_layers(), 5, state, 1.0, ftab, ttab)[0]
    freq = torch.bincount(idx1, minlength=4).double().cpu().numpy() / n
    assert np.all(np.abs(freq - 0.25) < 0.01), freq
    tm = TorchModel(net, input_shape=(3,), device=dev)
    assert tm._mlp_layers(3, 4) is not None
