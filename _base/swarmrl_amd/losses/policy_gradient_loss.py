"""
Vanilla policy-gradient loss (reference: swarmrl/losses/policy_gradient_loss.py:27-141),
in torch on the network's device.

loss = -sum(log(p(a) + 1e-8) * stop_grad(R - V)) + sum(huber(V, R)),
R = ExpectedReturns(rewards) (discounted, standardised per agent); one
gradient step per episode.
"""

import torch
import torch.nn.functional as F

from swarmrl_amd.losses.proximal_policy_loss import Loss, _stack
from swarmrl_amd.value_functions.expected_returns import ExpectedReturns


class PolicyGradientLoss(Loss):
    def __init__(self, value_function: ExpectedReturns = None):
        self.value_function = value_function if value_function is not None else ExpectedReturns()
        self.n_particles = None
        self.n_time_steps = None

    def _calculate_loss(self, network, feature_data, action_indices, rewards):
        """The reference's _calculate_loss (:47-106): actor term on the
        detached advantage, Huber critic term summed over time and agents."""
        obs_ndim = feature_data.ndim - 2
        logits, predicted_values = network(feature_data, obs_ndim=obs_ndim)
        predicted_values = predicted_values.squeeze(-1)
        probabilities = torch.softmax(logits, dim=-1)
        chosen = torch.gather(probabilities, -1, action_indices.unsqueeze(-1)).squeeze(-1)
        log_probs = torch.log(chosen + 1e-8)
        with torch.no_grad():
            returns = self.value_function(rewards).to(predicted_values.device)
        advantage = (returns - predicted_values).detach()
        critic_loss = F.huber_loss(predicted_values, returns, reduction="sum", delta=1.0)
        actor_loss = -(log_probs * advantage).sum()
        return actor_loss + critic_loss

    def compute_loss(self, network, episode_data):
        dev = network.device
        features = _stack(episode_data.features, dev).float()
        actions = _stack(episode_data.actions, dev).long()
        rewards = _stack(episode_data.rewards, dev).float()
        if actions.ndim == 3:  # device path: [T, E, A, ...] -> merge env and agent axes
            T, E, A = actions.shape
            actions = actions.reshape(T, E * A)
            features = features.reshape(T, E * A, *features.shape[3:])
            rewards = rewards.reshape(rewards.shape[0], E * A)
        self.n_time_steps, self.n_particles = int(features.shape[0]), int(features.shape[1])
        loss = self._calculate_loss(network, features, actions, rewards)
        network.update_model(loss)
