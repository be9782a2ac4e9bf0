"""
The fused PPO epoch gradient (swarm_ppo_epoch_grad, csrc/swarm_ppo.cuh)
against torch autograd of ProximalPolicyLoss._calculate_loss (the restatement
of swarmrl/losses/proximal_policy_loss.py:62-138 pinned by
tests/test_ppo_loss_cpu.py) on the same fp32 parameters and samples.

Tolerance: both sides are fp32 with different summation orders, and a
sample whose ReLU pre-activation or ratio sits within rounding of a kink
may take the other branch, so each parameter tensor's gradient is compared
in norm: |g_fused - g_torch| <= 2e-4 |g_torch| (+1e-6), and elementwise
within 2e-3 of the tensor's largest entry.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


def _episode(T, S, d, k, hidden, seed):
    from swarmrl_amd.networks.torch_network import ActorCriticMLP

    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    net = ActorCriticMLP(d, n_actions=k, hidden=hidden).to(dev)
    x = torch.randn(T, S, d, generator=g).to(dev)
    actions = torch.randint(0, k, (T, S), generator=g).to(dev)
    rewards = torch.randn(T, S, generator=g).to(dev)
    with torch.no_grad():
        logits, _ = net(x)
        logp = torch.log(torch.softmax(logits, -1) + 1e-8).gather(-1, actions[..., None])[..., 0]
    # old policy off by up to ~e^0.4: ratios on both sides of the clip range
    old = (logp + 0.4 * torch.randn(T, S, generator=g).to(dev)).contiguous()
    return net, x, actions, old, rewards


class _Wrap:
    def __init__(self, net):
        self.net = net

    def __call__(self, features, obs_ndim=1):
        lead = features.shape[: features.ndim - obs_ndim]
        return self.net(features.reshape(*lead, -1))


def _torch_grads(loss, net, x, actions, old, rewards):
    net.zero_grad(set_to_none=True)
    loss._calculate_loss(_Wrap(net), x, actions, rewards, old).backward()
    return [p.grad.detach().clone() for p in net.ppo_layers()]


def _fused_grads(loss, net, x, actions, old, rewards):
    from swarmrl_amd.engine import ops

    layers = net.ppo_layers()
    flat = ops.ppo_epoch_grad(x, actions, old, rewards, layers, loss.value_function.gamma,
                              loss.value_function.lambda_, loss.epsilon,
                              loss.entropy_coefficient)
    out, off = [], 0
    for t in layers:
        out.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    assert off == flat.numel()
    return out, flat


def _check(got, want):
    names = ["W1", "b1", "Wa", "ba", "Wc", "bc"]
    for name, a, b in zip(names, got, want):
        err = (a - b).norm().item()
        assert err <= 2e-4 * b.norm().item() + 1e-6, (name, err, b.norm().item())
        assert (a - b).abs().max().item() <= 2e-3 * b.abs().max().item() + 1e-6, name


@pytest.mark.parametrize("T,S,d,k,hidden", [
    (20, 1000, 1, 4, 128),     # concentration-field agents, stock network
    (20, 4096, 4, 4, 128),
    (7, 333, 10, 3, 100),      # ragged: hidden 100 in a 128-thread block, k < K
    (5, 517, 32, 6, 256),      # widest: 32 features, 256 units, 16-action variant
    (3, 64, 2, 4, 64),
    (40, 150, 2, 4, 128),      # T > 32: the GAE kernel's uncached loop
    (20, 53000, 4, 4, 128),    # >= 2^20 samples: the packed two-sample values kernel
])
def test_fused_epoch_grad_matches_autograd(T, S, d, k, hidden):
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss

    loss = ProximalPolicyLoss()
    net, x, actions, old, rewards = _episode(T, S, d, k, hidden, seed=T * 1000 + S)
    want = _torch_grads(loss, net, x, actions, old, rewards)
    got, _ = _fused_grads(loss, net, x, actions, old, rewards)
    _check(got, want)


def test_fused_epoch_grad_deterministic():
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss

    loss = ProximalPolicyLoss()
    net, x, actions, old, rewards = _episode(20, 20000, 1, 4, 128, seed=5)
    _, a = _fused_grads(loss, net, x, actions, old, rewards)
    _, b = _fused_grads(loss, net, x, actions, old, rewards)
    assert torch.equal(a, b)


def test_compute_loss_fused_equals_torch_path(monkeypatch):
    """Two epochs of compute_loss with SGD: the fused path and the torch
    path end on the same parameters."""
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    T, E, A, d = 20, 2, 500, 1
    g = torch.Generator().manual_seed(11)
    feats = torch.randn(T, E, A, d, generator=g)
    acts = torch.randint(0, 4, (T, E, A), generator=g)
    rews = torch.randn(T, E, A, generator=g)
    olp = -1.386 + 0.3 * torch.randn(T, E, A, generator=g)

    class Episode:
        features = [f.to(dev) for f in feats]
        actions = [a.to(dev) for a in acts]
        rewards = [r.to(dev) for r in rews]
        log_probs = [lp.to(dev) for lp in olp]

    steps = []
    for fused in ("1", "0"):
        monkeypatch.setenv("SWARMRL_AMD_FUSED_PPO", fused)
        torch.manual_seed(0)
        model = TorchModel(ActorCriticMLP(d, 4, 128), input_shape=(d,), device=dev,
                           optimizer=lambda ps: torch.optim.SGD(ps, lr=1e-4))
        before = [p.detach().clone() for p in model.model.ppo_layers()]
        loss = ProximalPolicyLoss(n_epochs=2)
        assert (loss._fused_layers(model, feats.reshape(T, E * A, d).to(dev),
                                   acts.reshape(T, E * A)) is not None) == (fused == "1")
        loss.compute_loss(model, Episode())
        steps.append([p.detach() - b for p, b in zip(model.model.ppo_layers(), before)])
    for a, b in zip(*steps):
        # SGD: the parameter change is lr x the summed gradients of the two epochs
        assert (a - b).norm().item() <= 1e-3 * b.norm().item() + 1e-7


def test_graph_epochs_equal_eager(monkeypatch):
    """Three episodes of compute_loss with the default (fused, capturable)
    Adam, the optimizer's own step (SWARMRL_AMD_FUSED_ADAM=0): the
    captured-graph epochs (episode 1 eager, 2 captured + replayed, 3
    replayed) end on bit-identical parameters to the eager loop."""
    monkeypatch.setenv("SWARMRL_AMD_FUSED_ADAM", "0")
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    T, E, A, d = 20, 1, 300, 4

    def episode(seed):
        g = torch.Generator().manual_seed(seed)

        class Episode:
            features = [f.to(dev) for f in torch.randn(T, E, A, d, generator=g)]
            actions = [a.to(dev) for a in torch.randint(0, 4, (T, E, A), generator=g)]
            rewards = [r.to(dev) for r in torch.randn(T, E, A, generator=g)]
            log_probs = [lp.to(dev) for lp in -1.386 + 0.3 * torch.randn(T, E, A, generator=g)]
        return Episode()

    finals = []
    for graph in ("1", "0"):
        monkeypatch.setenv("SWARMRL_AMD_PPO_GRAPH", graph)
        torch.manual_seed(0)
        model = TorchModel(ActorCriticMLP(d, 4, 128), input_shape=(d,), device=dev)
        loss = ProximalPolicyLoss(n_epochs=5)
        for ep in range(3):
            loss.compute_loss(model, episode(100 + ep))
        assert (getattr(loss, "_ppo_graph", None) is not None) == (graph == "1")
        assert model.epoch_count == 15
        finals.append([p.detach().clone() for p in model.model.ppo_layers()])
    for a, b in zip(*finals):
        assert torch.equal(a, b)


def test_fused_adam_step_matches_torch_adam(monkeypatch):
    """The Adam step fused into each epoch's last launch (swarm_ppo_epoch_step,
    the default for torch Adam on the six layers) against torch's fused Adam
    after the same gradients: parameters, moments and step counts of three
    episodes x 5 epochs (episode 1 eager with torch's step, 2-3 captured),
    fp32 rounding apart (another operation order); and run to run the fused
    path is bit-identical."""
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    T, E, A, d = 20, 1, 300, 1

    def episode(seed):
        g = torch.Generator().manual_seed(seed)

        class Episode:
            features = [f.to(dev) for f in torch.randn(T, E, A, d, generator=g)]
            actions = [a.to(dev) for a in torch.randint(0, 4, (T, E, A), generator=g)]
            rewards = [r.to(dev) for r in torch.randn(T, E, A, generator=g)]
            log_probs = [lp.to(dev) for lp in -1.386 + 0.3 * torch.randn(T, E, A, generator=g)]
        return Episode()

    runs = {}
    for tag, fused in (("fused", "1"), ("fused2", "1"), ("torch", "0")):
        monkeypatch.setenv("SWARMRL_AMD_FUSED_ADAM", fused)
        torch.manual_seed(0)
        model = TorchModel(ActorCriticMLP(d, 4, 128), input_shape=(d,), device=dev)
        loss = ProximalPolicyLoss(n_epochs=5)
        for ep in range(3):
            loss.compute_loss(model, episode(200 + ep))
        assert loss._ppo_graph["sig"][0] == (fused == "1")
        layers = model.model.ppo_layers()
        st = [model.optimizer.state[p] for p in layers]
        runs[tag] = ([p.detach().clone() for p in layers],
                     [s["exp_avg"].clone() for s in st], [s["exp_avg_sq"].clone() for s in st],
                     [float(s["step"]) for s in st])
    for a, b in zip(runs["fused"][0] + runs["fused"][1] + runs["fused"][2],
                    runs["fused2"][0] + runs["fused2"][1] + runs["fused2"][2]):
        assert torch.equal(a, b)
    assert runs["fused"][3] == runs["torch"][3] == [15.0] * 6
    for a, b in zip(runs["fused"][0], runs["torch"][0]):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-6)
    # the moments integrate 15 epochs of gradients: Adam's per-entry
    # normalisation turns 1-ulp parameter differences into order-one relative
    # differences in entries whose gradient is near zero, so a few moment
    # entries move by ~1e-5 (absolute); one step alone agrees to fp32
    # rounding (test_fused_adam_single_epoch_matches_torch_tightly)
    for a, b in zip(runs["fused"][1] + runs["fused"][2], runs["torch"][1] + runs["torch"][2]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


def _random_episode(dev, T, E, A, d, seed):
    g = torch.Generator().manual_seed(seed)

    class Episode:
        features = [f.to(dev) for f in torch.randn(T, E, A, d, generator=g)]
        actions = [a.to(dev) for a in torch.randint(0, 4, (T, E, A), generator=g)]
        rewards = [r.to(dev) for r in torch.randn(T, E, A, generator=g)]
        log_probs = [lp.to(dev) for lp in -1.386 + 0.3 * torch.randn(T, E, A, generator=g)]
    return Episode()


def _train(monkeypatch, fused, epsilon, episodes=3, n_epochs=5, d=1, A=300, seed0=200):
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    monkeypatch.setenv("SWARMRL_AMD_FUSED_ADAM", fused)
    torch.manual_seed(0)
    model = TorchModel(ActorCriticMLP(d, 4, 128), input_shape=(d,), device=dev)
    loss = ProximalPolicyLoss(n_epochs=n_epochs, epsilon=epsilon)
    for ep in range(episodes):
        loss.compute_loss(model, _random_episode(dev, 20, 1, A, d, seed0 + ep))
    layers = model.model.ppo_layers()
    st = [model.optimizer.state[p] for p in layers]
    return ([p.detach().clone() for p in layers],
            [s["exp_avg"].clone() for s in st] + [s["exp_avg_sq"].clone() for s in st])


def test_fused_adam_single_epoch_matches_torch_tightly(monkeypatch):
    """The fused Adam step's arithmetic, measured: from bit-identical
    states (episode 1 eager with torch's step on both sides), one captured
    epoch with the fused step and one with torch's fused Adam end on
    parameters AND moments equal to fp32 rounding (rtol 1e-5, absolute
    1e-5 of the tensor's largest entry: torch's lerp-form moment update
    rounds differently, and entries where history and gradient cancel keep
    only the absolute error), with the
    clipped surrogate active (epsilon 0.2) or not (1e6).  Over many epochs
    the moments drift further apart (test_fused_adam_step_matches_torch_adam):
    Adam divides each gradient entry by its own RMS, so the 1-ulp parameter
    differences of one step, fed back through the next gradients, become
    relative differences of order one in entries whose gradient is near
    zero -- with or without clip-boundary flips (measured: 7 of 128 entries
    of a W1 moment beyond 2e-5 after 15 epochs at epsilon 1e6)."""
    for eps in (0.2, 1e6):
        f1 = _train(monkeypatch, "1", epsilon=eps, episodes=2, n_epochs=1)
        r1 = _train(monkeypatch, "0", epsilon=eps, episodes=2, n_epochs=1)
        for a, b in zip(f1[0] + f1[1], r1[0] + r1[1]):
            # absolute slack scaled to the tensor: a moment entry where the
            # decayed history and the new gradient nearly cancel keeps only
            # the absolute rounding (measured: 1.4e-6 absolute, 4.8e-5 relative in
            # one entry of 512)
            torch.testing.assert_close(a, b, rtol=1e-5, atol=float(1e-5 * b.abs().max()) + 1e-9)


def test_two_losses_of_different_sizes_share_a_device(monkeypatch):
    """Two PPO losses whose episodes have different T*S on one device
    (ADVICE r5): each keeps its own fused-PPO workspace, so interleaving
    their captured epoch graphs ends on exactly the parameters each reaches
    alone."""
    from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
    from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

    dev = torch.device("cuda", 0)
    monkeypatch.setenv("SWARMRL_AMD_FUSED_ADAM", "1")

    def make(seed):
        torch.manual_seed(seed)
        return (TorchModel(ActorCriticMLP(2, 4, 64), input_shape=(2,), device=dev),
                ProximalPolicyLoss(n_epochs=3))

    sizes = {0: 300, 1: 700}
    alone = {}
    for k, A in sizes.items():
        model, loss = make(k)
        for ep in range(3):
            loss.compute_loss(model, _random_episode(dev, 20, 1, A, 2, 50 * k + ep))
        alone[k] = [p.detach().clone() for p in model.model.ppo_layers()]
    pairs = {k: make(k) for k in sizes}
    for ep in range(3):
        for k, A in sizes.items():
            model, loss = pairs[k]
            loss.compute_loss(model, _random_episode(dev, 20, 1, A, 2, 50 * k + ep))
    for k in sizes:
        assert pairs[k][1]._ppo_graph is not None
        for a, b in zip(alone[k], pairs[k][0].model.ppo_layers()):
            assert torch.equal(a, b.detach())
