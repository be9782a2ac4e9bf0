"""
Actor-critic network on PyTorch-ROCm (reference: swarmrl/networks/flax_network.py).

``TorchModel.compute_action`` mirrors FlaxModel.compute_action
(flax_network.py:153-195): logits, values = model(obs); Gumbel sampling;
log_probs = log(softmax(logits) + 1e-8); exploration; gather the chosen
log-prob.  Observables of shape (n_agents, ...) are flattened per agent.
With a device tensor input everything stays on the GPU (no host sync).
"""

import os

import numpy as np
import torch
from torch import nn

from swarmrl_amd.exploration_policies.random_exploration import RandomExploration
from swarmrl_amd.sampling_strategies.gumbel_distribution import GumbelDistribution


class ActorCriticMLP(nn.Module):
    """Dense(hidden) -> ReLU -> {Dense(n_actions) logits, Dense(1) value}
    (the network of CI/espresso_tests/integration_tests/test_rl_trainers.py:17-26)."""

    def __init__(self, input_dim: int, n_actions: int = 4, hidden: int = 128):
        super().__init__()
        self.hidden = nn.Linear(input_dim, hidden)
        self.actor = nn.Linear(hidden, n_actions)
        self.critic = nn.Linear(hidden, 1)

    def forward(self, x):
        h = torch.relu(self.hidden(x))
        return self.actor(h), self.critic(h)

    def logits(self, x):
        """Actor head only (the rollout never reads the value); the hidden
        layer's bias + ReLU run in the GEMM epilogue."""
        h = torch._addmm_activation(self.hidden.bias, x, self.hidden.weight.t())
        return self.actor(h)

    def rollout_layers(self):
        """(W1, b1, W2, b2) of the actor path, for the one-kernel rollout
        policy (swarm_policy_mlp_sample)."""
        return (self.hidden.weight, self.hidden.bias, self.actor.weight, self.actor.bias)

    def ppo_layers(self):
        """(W1, b1, Wa, ba, Wc, bc), the order of the fused PPO gradient
        (swarm_ppo_epoch_grad)."""
        return (self.hidden.weight, self.hidden.bias, self.actor.weight, self.actor.bias,
                self.critic.weight, self.critic.bias)


class TorchModel:
    """Network wrapper with the FlaxModel surface used by the agents."""

    def __init__(
        self,
        torch_model: nn.Module,
        input_shape: tuple = None,
        optimizer=None,
        exploration_policy=RandomExploration(probability=0.0),
        sampling_strategy=GumbelDistribution(),
        rng_key: int = None,
        deployment_mode: bool = False,
        device=None,
        learning_rate: float = 1e-3,
    ):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) \
                if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        if rng_key is not None:
            torch.manual_seed(int(rng_key))
        self.model = torch_model.to(self.device)
        self.input_shape = input_shape
        self.sampling_strategy = sampling_strategy
        self.exploration_policy = exploration_policy
        self.deployment_mode = deployment_mode
        if optimizer is None:
            # optax.adam of the reference; on the GPU one fused launch per step,
            # capturable so the fused PPO epochs can run as one graph
            fused = self.device.type == "cuda"
            optimizer = lambda params: torch.optim.Adam(  # noqa: E731
                params, lr=learning_rate, fused=fused, capturable=fused)
        self._optimizer_factory = optimizer
        self.optimizer = None if deployment_mode else optimizer(self.model.parameters())
        self.epoch_count = 0
        self.generator = None
        # fused device sampling (swarm_sample_actions): Philox seed drawn from
        # torch's generator, call counter in device memory
        self._fused_seed = int(torch.randint(0, 2**62, (1,)).item())
        self._fused_state = None
        self._agent_state = None  # per-agent call counters (swarm_engine_vision_policy)

    def reinitialize_network(self):
        for m in self.model.modules():
            if hasattr(m, "reset_parameters"):
                m.reset_parameters()
        self.optimizer = self._optimizer_factory(self.model.parameters())

    def __call__(self, features: torch.Tensor, obs_ndim: int = 1):
        """Forward over features (..., n_agents, *obs); the trailing obs_ndim
        dims are flattened per agent.  Returns (logits, values)."""
        lead = features.shape[: features.ndim - obs_ndim]
        return self.model(features.reshape(*lead, -1).to(torch.float32))

    @torch.no_grad()
    def compute_action(self, observables):
        """(indices, log_probs) for every agent; tensors in -> tensors out."""
        host = not isinstance(observables, torch.Tensor)
        if host:
            obs = torch.as_tensor(np.asarray(observables, dtype=np.float32), device=self.device)
        else:
            obs = observables.to(torch.float32)
        obs = obs.reshape(obs.shape[0], -1)
        logits, _ = self.model(obs)
        indices = self.sampling_strategy(logits, generator=self.generator)
        eps = 1e-8
        log_probs = torch.log(torch.softmax(logits, dim=-1) + eps)
        indices = self.exploration_policy(indices, logits.shape[-1], generator=self.generator)
        chosen = torch.gather(log_probs, 1, indices.reshape(-1, 1)).reshape(-1)
        if host:
            return indices.cpu().numpy(), chosen.cpu().numpy()
        return indices, chosen

    def fused_sampling_ok(self, observables) -> bool:
        """The one-kernel sampling path applies: stock Gumbel sampling and
        random exploration, device tensors, the HIP library present."""
        return (isinstance(observables, torch.Tensor) and observables.is_cuda
                and type(self.sampling_strategy) is GumbelDistribution
                and type(self.exploration_policy) is RandomExploration)

    # compute_action_fused takes the engine whose deferred build may ride
    # along in the policy launch (SwarmEngine._prebuild, ride-along mode)
    accepts_engine = True

    @torch.no_grad()
    def compute_action_fused(self, observables: torch.Tensor, f_table: torch.Tensor,
                             t_table: torch.Tensor, engine=None):
        """compute_action + action-table lookup in one sampling kernel:
        returns (indices, log_probs, f_swim, torque_z) device tensors.
        engine: the native engine of the slice (its deferred build's last
        stage rides along in the one-kernel policy launch)."""
        from swarmrl_amd.engine import ops

        obs = observables.to(torch.float32)
        obs = obs.reshape(obs.shape[0], -1)
        p = float(self.exploration_policy.probability)
        self._fused_state = ops.counter_state(self._fused_state, obs.shape[0], obs.device)
        layers = self._mlp_layers(obs.shape[1], int(f_table.numel()))
        if layers is not None:  # stock MLP: network + sampling in one kernel
            return ops.policy_mlp_sample(obs, *layers, self._fused_seed, self._fused_state, p,
                                         f_table, t_table, engine=engine)
        if hasattr(self.model, "logits"):
            logits = self.model.logits(obs)
        else:
            logits, _ = self.model(obs)
        return ops.sample_actions(logits.float(), self._fused_seed, self._fused_state, p,
                                  f_table, t_table)

    def fused_policy_args(self, n: int, d_in: int, k: int, device):
        """What an observable needs to run this network's rollout policy in
        its own launch (swarm_engine_vision_policy): (w1, b1, w2, b2, seed,
        per-agent counters for n agents, exploration probability), or None
        when the one-kernel policy does not apply (another network, sampling
        strategy or exploration policy, or sizes beyond the fused kernel's:
        d_in <= 4, k <= 4)."""
        if not (type(self.sampling_strategy) is GumbelDistribution
                and type(self.exploration_policy) is RandomExploration):
            return None
        if d_in > 4 or k > 4:
            return None
        layers = self._mlp_layers(d_in, k)
        if layers is None:
            return None
        st = self._agent_state
        if st is None or st.device != device or st.numel() < n:
            grown = torch.zeros(max(n, 1), dtype=torch.int64, device=device)
            if st is not None and st.device == device:
                grown[: st.numel()] = st
            self._agent_state = st = grown
        # a key of its own: the group counters of compute_action_fused also
        # start at zero, so one network serving both paths would otherwise
        # replay the same Gumbel noise on them
        return (*layers, self._fused_seed ^ 0x2545F4914F6CDD1D, st,
                float(self.exploration_policy.probability))

    def _mlp_layers(self, d_in: int, k: int):
        """The actor weights when the one-kernel policy applies (fp32 device
        parameters within swarm_policy_mlp_sample's limits), else None."""
        get = getattr(self.model, "rollout_layers", None)
        if get is None:
            return None
        w1, b1, w2, b2 = get()
        ok = all(t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
                 for t in (w1, b1, w2, b2))
        ok = ok and w1.shape[1] == d_in and w2.shape[0] == k and w2.shape[1] == w1.shape[0]
        ok = ok and d_in <= 16 and w1.shape[0] <= 256 and k <= 16
        return (w1, b1, w2, b2) if ok else None

    def ppo_layers(self, d_in: int):
        """The actor-critic weights when the fused PPO gradient applies (fp32
        contiguous device parameters within swarm_ppo_epoch_grad's limits and
        every trainable parameter among them), else None."""
        get = getattr(self.model, "ppo_layers", None)
        if get is None or self.optimizer is None:
            return None
        layers = get()
        w1, b1, wa, ba, wc, bc = layers
        ok = all(t.dtype == torch.float32 and t.is_cuda and t.is_contiguous() for t in layers)
        ok = ok and w1.shape[1] == d_in and wa.shape[1] == w1.shape[0]
        ok = ok and tuple(wc.shape) == (1, w1.shape[0]) and bc.numel() == 1
        ok = ok and d_in <= 32 and w1.shape[0] <= 256 and wa.shape[0] <= 16
        ids = {id(t) for t in layers}
        ok = ok and all(id(p) in ids for p in self.model.parameters() if p.requires_grad)
        return layers if ok else None

    def apply_gradients(self, layers, flat_grad: torch.Tensor):
        """One optimizer step with the gradient given as the concatenation of
        the layers' gradients (the layout of swarm_ppo_epoch_grad)."""
        self.optimizer.zero_grad(set_to_none=True)
        off = 0
        for t in layers:
            n = t.numel()
            t.grad = flat_grad[off:off + n].view_as(t)
            off += n
        self.optimizer.step()
        self.epoch_count += 1

    def update_model(self, loss: torch.Tensor):
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        self.optimizer.step()
        self.epoch_count += 1

    def export_model(self, filename: str = "model", directory: str = "Models"):
        os.makedirs(directory, exist_ok=True)
        torch.save(
            {
                "model": self.model.state_dict(),
                "optimizer": self.optimizer.state_dict() if self.optimizer else None,
                "epoch": self.epoch_count,
            },
            os.path.join(directory, filename + ".pt"),
        )

    def restore_model_state(self, filename, directory):
        state = torch.load(os.path.join(directory, filename + ".pt"), weights_only=True,
                           map_location=self.device)
        self.model.load_state_dict(state["model"])
        if self.optimizer is not None and state["optimizer"] is not None:
            self.optimizer.load_state_dict(state["optimizer"])
        self.epoch_count = int(state["epoch"])


