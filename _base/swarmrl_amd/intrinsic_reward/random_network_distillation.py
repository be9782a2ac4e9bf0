"""
Random Network Distillation intrinsic reward (reference:
swarmrl/intrinsic_reward/random_network_distillation.py:16-149,
Burda et al. 2018): a fixed random target network and a predictor trained on
the visited observations; the reward of the latest state is the mean
distance between their representations, clipped.  PyTorch on the device
holding the trajectory (the C5 workload's "intrinsic reward").
"""

import numpy as np
import torch

from swarmrl_amd.intrinsic_reward.intrinsic_reward import IntrinsicReward
from swarmrl_amd.intrinsic_reward.rnd_configs import RNDArchitecture, RNDConfig, order_n_difference


class RNDReward(IntrinsicReward):
    supports_device = True

    def __init__(self, rnd_config: RNDConfig):
        self.__dict__.update(rnd_config.__dict__)
        self.iterations = 0
        self.metric_results = None
        in_dim = int(np.prod(rnd_config.input_shape))
        self.in_dim = in_dim
        dev = rnd_config.device or (torch.device("cuda", torch.cuda.current_device())
                                    if torch.cuda.is_available() else torch.device("cpu"))
        self.device = torch.device(dev)
        self.target_network = RNDArchitecture(in_dim).to(self.device)
        self.predictor_network = RNDArchitecture(in_dim).to(self.device)
        for p in self.target_network.parameters():
            p.requires_grad_(False)
        # capturable on the GPU: its step counters live on the device like the
        # parameters (no host sync per step; broadcast_agent sends them over
        # RCCL like every other tensor of the replica)
        self.optimizer = torch.optim.Adam(self.predictor_network.parameters(),
                                          lr=rnd_config.learning_rate,
                                          capturable=self.device.type == "cuda")
        self._ws = {}  # swarm_rnd_env_reward partial-sum workspaces (ops.rnd_env_reward)

    @staticmethod
    def _stack(x) -> torch.Tensor:
        if isinstance(x, (list, tuple)):
            x = torch.stack([torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor)
                             else v for v in x])
        return torch.as_tensor(x)

    @staticmethod
    def _reshape_data(x) -> torch.Tensor:
        """Flatten time and ensemble axes: (T, N, *obs) -> (T * N, prod(obs))
        (random_network_distillation.py:58-77)."""
        x = RNDReward._stack(x)
        return x.reshape(x.shape[0] * x.shape[1], -1).to(torch.float32)

    def _features(self, episode_data, last_only: bool):
        """Every leading axis (time, and on the device path env and agent)
        is a sample axis; the observation is the trailing prod(input_shape).
        The latest observations of a device trajectory are read in place (no
        stacking copy)."""
        feats = episode_data.features
        if last_only and isinstance(feats[-1], torch.Tensor):
            x = feats[-1]
        else:
            x = self._stack(feats[-1:] if last_only else feats)
        return x.reshape(-1, self.in_dim).to(torch.float32).to(self.device)

    def _per_env(self, last) -> bool:
        """Device-path observations [E, A, *obs]: one reward per env."""
        return isinstance(last, torch.Tensor) and last.dim() == len(self.input_shape) + 2

    @staticmethod
    def fused_architecture_ok(net: torch.nn.Module, in_dim: int) -> bool:
        """k_rnd_distance hard-codes the stock network: an RNDArchitecture
        whose Sequential is exactly Linear(in_dim, 32) -> ReLU -> Linear(32, 32)
        -> ReLU -> Linear(32, 32) with contiguous fp32 parameters (read in place
        as [out][in] rows).  Anything else -- another activation, an extra
        layer, a transposed or non-contiguous parameter -- takes the torch
        path."""
        if type(net) is not RNDArchitecture or not isinstance(net.net, torch.nn.Sequential):
            return False
        layers = list(net.net)
        kinds = [torch.nn.Linear, torch.nn.ReLU, torch.nn.Linear, torch.nn.ReLU, torch.nn.Linear]
        if len(layers) != len(kinds) or any(type(m) is not k for m, k in zip(layers, kinds)):
            return False
        for m, fan_in in zip(layers[0::2], (in_dim, 32, 32)):
            if m.in_features != fan_in or m.out_features != 32 or m.bias is None:
                return False
            if tuple(m.weight.shape) != (32, fan_in) or tuple(m.bias.shape) != (32,):
                return False
            for t in (m.weight, m.bias):
                if t.dtype != torch.float32 or not t.is_contiguous():
                    return False
        return True

    def _fused_ok(self, points: torch.Tensor) -> bool:
        """The one-launch HIP metric applies to the stock architecture on the
        GPU (fused_architecture_ok), for inputs of 1..16 features."""
        if not (points.is_cuda and points.dtype == torch.float32 and 1 <= self.in_dim <= 16):
            return False
        return all(self.fused_architecture_ok(net, self.in_dim) and
                   all(p.is_cuda for p in net.parameters())
                   for net in (self.target_network, self.predictor_network))

    @torch.no_grad()
    def compute_distance(self, points: torch.Tensor) -> torch.Tensor:
        if self._fused_ok(points):
            from swarmrl_amd.engine import ops

            self.metric_results = ops.rnd_distance(points, self.target_network,
                                                   self.predictor_network, self.distance_order)
        else:
            self.metric_results = order_n_difference(self.target_network(points),
                                                     self.predictor_network(points),
                                                     self.distance_order)
        return torch.mean(self.metric_results)

    def update(self, episode_data):
        """Train the predictor on the episode's observations (MeanPowerLoss)."""
        domain = self._features(episode_data, last_only=False)
        with torch.no_grad():
            codomain = self.target_network(domain)
        n = domain.shape[0]
        for _ in range(self.n_epochs):
            perm = torch.randperm(n, device=domain.device)
            for b in range(0, n, self.batch_size):
                idx = perm[b:b + self.batch_size]
                pred = self.predictor_network(domain[idx])
                loss = torch.mean(torch.abs(pred - codomain[idx]) ** self.loss_order)
                self.optimizer.zero_grad(set_to_none=True)
                loss.backward()
                self.optimizer.step()
        self.iterations += 1

    def compute_reward(self, episode_data):
        """Mean clipped RND distance of the latest observations
        (random_network_distillation.py:126-143): a scalar tensor, or on the
        device path (features [E, A, *obs]) one mean per env, [E, 1], which
        broadcasts over the env's agents."""
        last = episode_data.features[-1]
        points = self._features(episode_data, last_only=True)
        if self._per_env(last) and self._fused_ok(points):
            from swarmrl_amd.engine import ops

            self.metric_results, r, _ = ops.rnd_env_reward(
                points, int(last.shape[0]), self.target_network, self.predictor_network,
                self.distance_order, self.clip_rewards, workspaces=self._ws)
            return r
        r = self.compute_distance(points)
        if self._per_env(last):
            r = self.metric_results.reshape(last.shape[0], -1).mean(dim=1, keepdim=True)
        if self.clip_rewards is not None:
            r = torch.clamp(r, *self.clip_rewards)
        return r

    def add_to_reward(self, rewards, episode_data):
        """rewards + compute_reward(episode_data) (the agent's task +
        intrinsic sum); on the device path with the stock networks the metric,
        the per-env mean, the clip and the sum are two launches
        (swarm_rnd_env_reward) instead of five and a copy."""
        last = episode_data.features[-1]
        if (isinstance(rewards, torch.Tensor) and rewards.is_cuda and self._per_env(last)
                and rewards.numel() == last.shape[0] * last.shape[1]):
            points = self._features(episode_data, last_only=True)
            if self._fused_ok(points):
                from swarmrl_amd.engine import ops

                self.metric_results, _, out = ops.rnd_env_reward(
                    points, int(last.shape[0]), self.target_network, self.predictor_network,
                    self.distance_order, self.clip_rewards, base=rewards, workspaces=self._ws)
                return out.reshape(rewards.shape)
        return rewards + self.compute_reward(episode_data)
