"""
PPO loss (reference: swarmrl/losses/proximal_policy_loss.py:23-170), in torch.

loss = sum(-min(r A, clip(r, 1-eps, 1+eps) A)) - c_H * entropy
       + 0.5 * sum(huber(V, returns)),   r = exp(log p_new(a) - log p_old(a)),
advantages/returns from GAE on the episode's rewards and predicted values;
n_epochs gradient steps per episode.  On the GPU, for the stock
actor-critic MLP, each epoch's gradient comes from the fused kernels of
swarm_ppo_epoch_grad (csrc/swarm_ppo.cuh) and torch's optimizer takes the
step; otherwise torch autograd differentiates _calculate_loss.
"""

import os

import torch
import torch.nn.functional as F

from swarmrl_amd.engine import ops
from swarmrl_amd.sampling_strategies.sampling_strategy import SamplingStrategy

from swarmrl_amd.sampling_strategies.gumbel_distribution import GumbelDistribution
from swarmrl_amd.value_functions.generalized_advantage_estimate import GAE


class Loss:
    def compute_loss(self, network, episode_data):
        raise NotImplementedError


def _stack(items, device):
    out = []
    for x in items:
        out.append(torch.as_tensor(x, device=device))
    return torch.stack(out)


class ProximalPolicyLoss(Loss):
    def __init__(self, value_function: GAE = None, sampling_strategy=None, n_epochs: int = 20,
                 epsilon: float = 0.2, entropy_coefficient: float = 0.01):
        self.value_function = value_function if value_function is not None else GAE()
        self.sampling_strategy = sampling_strategy or GumbelDistribution()
        self.n_epochs = n_epochs
        self.epsilon = epsilon
        self.entropy_coefficient = entropy_coefficient
        self.eps = 1e-8

    def _calculate_loss(self, network, feature_data, action_indices, rewards, old_log_probs):
        obs_ndim = feature_data.ndim - 2
        new_logits, predicted_values = network(feature_data, obs_ndim=obs_ndim)
        predicted_values = predicted_values.squeeze(-1)
        # as in the reference (:101-124), only the normalised advantages are
        # held constant: the returns R = A + V stay differentiable in V
        advantages, returns = self.value_function(rewards=rewards, values=predicted_values)
        advantages = advantages.detach()
        new_probabilities = torch.softmax(new_logits, dim=-1)
        entropy = self.sampling_strategy.compute_entropy(new_probabilities)
        chosen = torch.gather(new_probabilities, -1, action_indices.unsqueeze(-1)).squeeze(-1)
        chosen_log_probs = torch.log(chosen + self.eps)
        ratio = torch.exp(chosen_log_probs - old_log_probs)
        total_critic_loss = F.huber_loss(predicted_values, returns, reduction="sum", delta=1.0)
        clipped = -torch.minimum(
            ratio * advantages, torch.clamp(ratio, 1 - self.epsilon, 1 + self.epsilon) * advantages
        )
        actor_loss = clipped.sum()
        return actor_loss - self.entropy_coefficient * entropy + 0.5 * total_critic_loss

    def compute_loss(self, network, episode_data):
        dev = network.device
        old_log_probs = _stack(episode_data.log_probs, dev).float()
        features = _stack(episode_data.features, dev).float()
        actions = _stack(episode_data.actions, dev).long()
        rewards = _stack(episode_data.rewards, dev).float()
        # device path: [T, E, A, ...] -> merge env and agent axes
        if actions.ndim == 3:
            T, E, A = actions.shape
            actions = actions.reshape(T, E * A)
            old_log_probs = old_log_probs.reshape(T, E * A)
            features = features.reshape(T, E * A, *features.shape[3:])
            rewards = rewards.reshape(rewards.shape[0], E * A)
        layers = self._fused_layers(network, features, actions)
        if layers is not None:
            features = features.reshape(features.shape[0], features.shape[1], -1).contiguous()
            if self._graph_epochs(network, layers, features, actions, old_log_probs, rewards):
                return
        for _ in range(self.n_epochs):
            if layers is not None:
                grad = ops.ppo_epoch_grad(features, actions, old_log_probs, rewards, layers,
                                          self.value_function.gamma,
                                          self.value_function.lambda_, self.epsilon,
                                          self.entropy_coefficient,
                                          workspaces=self._workspaces())
                network.apply_gradients(layers, grad)
                continue
            loss = self._calculate_loss(network, features, actions, rewards, old_log_probs)
            network.update_model(loss)

    def _graph_epochs(self, network, layers, features, actions, old_log_probs, rewards):
        """
        The n_epochs fused steps (gradient kernels + the optimizer's step) as
        one captured HIP graph, replayed per episode with the episode's data
        copied into the graph's input buffers: the epochs are launch-bound at
        small sizes (E = 1: ~100 us of host work per epoch).  Needs an
        optimizer whose every param group is capturable (the default fused
        Adam is) and state already initialised (the first episode runs
        eagerly).  Recaptured when shapes, learning rates or the optimizer's
        state tensors change.  SWARMRL_AMD_PPO_GRAPH=0 disables it.
        Returns False when the eager loop should run instead.
        """
        opt = getattr(network, "optimizer", None)
        if os.environ.get("SWARMRL_AMD_PPO_GRAPH", "1") == "0" or opt is None:
            return False
        if not all(g.get("capturable", False) for g in opt.param_groups):
            return False
        states = [opt.state.get(p, {}) for p in layers]
        if not all(states) or any(p.grad is None for p in layers):
            return False  # optimizer state not initialised yet: first episode is eager
        # torch Adam on exactly these layers: its step fused into each epoch's
        # last launch (swarm_ppo_epoch_step; SWARMRL_AMD_FUSED_ADAM=0: the
        # optimizer's own step after the gradient)
        adam = (ops.adam_args(opt, layers)
                if os.environ.get("SWARMRL_AMD_FUSED_ADAM", "1") != "0" else None)
        # every hyper-parameter the fused step bakes into its captured
        # arguments (betas / eps were missing)
        sig = (adam is not None, id(network), id(opt), tuple(features.shape),
               tuple(actions.shape),
               tuple((float(g["lr"]), tuple(float(b) for b in g.get("betas", ())),
                      float(g.get("eps", 0.0)), float(g.get("weight_decay", 0.0)),
                      bool(g.get("amsgrad", False)), bool(g.get("maximize", False)))
                     for g in opt.param_groups),
               tuple(t.data_ptr() for st in states for t in st.values()
                     if isinstance(t, torch.Tensor)),
               tuple(p.data_ptr() for p in layers), self.n_epochs,
               self.value_function.gamma, self.value_function.lambda_, self.epsilon,
               self.entropy_coefficient)
        cache = getattr(self, "_ppo_graph", None)
        if cache is None or cache["sig"] != sig:
            cache = None
            self._ppo_graph = None
            x = features.clone()
            act = actions.to(torch.int64).clone()
            olp = old_log_probs.to(torch.float32).clone()
            rew = rewards.to(torch.float32).clone()
            grad = torch.zeros(sum(p.numel() for p in layers), dtype=torch.float32,
                               device=features.device)
            off = 0
            for p in layers:
                p.grad = grad[off:off + p.numel()].view_as(p)
                off += p.numel()
            args = (x, act, olp, rew, layers, self.value_function.gamma,
                    self.value_function.lambda_, self.epsilon, self.entropy_coefficient)
            ws = self._workspaces()
            # sizes the workspace outside the capture
            ops.ppo_epoch_grad(*args, out=grad, workspaces=ws)
            torch.cuda.synchronize(features.device)
            graph = torch.cuda.CUDAGraph()
            # (thread-local: a process group's watchdog thread may query
            # events while this thread captures)
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                for _ in range(self.n_epochs):
                    if adam is not None:
                        ops.ppo_epoch_grad(*args, out=grad, adam=adam, workspaces=ws)
                    else:
                        ops.ppo_epoch_grad(*args, out=grad, workspaces=ws)
                        opt.step()
            cache = self._ppo_graph = {"sig": sig, "graph": graph, "inputs": (x, act, olp, rew),
                                       "grad": grad}
        x, act, olp, rew = cache["inputs"]
        x.copy_(features)
        act.copy_(actions)
        olp.copy_(old_log_probs)
        rew.copy_(rewards)
        cache["graph"].replay()
        if hasattr(network, "epoch_count"):
            network.epoch_count += self.n_epochs
        return True

    def _workspaces(self):
        """This loss's fused-PPO workspaces (one per device and size), kept
        for its lifetime: its captured epoch graph reads them in place."""
        ws = getattr(self, "_ppo_ws", None)
        if ws is None:
            ws = self._ppo_ws = {}
        return ws

    def _fused_layers(self, network, features, actions):
        """The network's layers when the epoch gradient runs as the fused
        device kernels (swarm_ppo_epoch_grad): stock GAE and entropy, the
        actor-critic MLP on the GPU, [T, S, ...] samples; else None (the
        torch autograd path).  SWARMRL_AMD_FUSED_PPO=0 forces the torch path."""
        if os.environ.get("SWARMRL_AMD_FUSED_PPO", "1") == "0" or not features.is_cuda:
            return None
        if type(self.value_function) is not GAE or actions.ndim != 2:
            return None
        if type(self.sampling_strategy).compute_entropy is not SamplingStrategy.compute_entropy:
            return None
        get = getattr(network, "ppo_layers", None)
        if get is None:
            return None
        d_in = 1
        for n in features.shape[2:]:
            d_in *= int(n)
        return get(d_in)
