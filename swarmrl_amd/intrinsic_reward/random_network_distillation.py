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
        self.optimizer = torch.optim.Adam(self.predictor_network.parameters(),
                                          lr=rnd_config.learning_rate)

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
        is a sample axis; the observation is the trailing prod(input_shape)."""
        feats = episode_data.features
        if last_only:
            feats = feats[-1:]
        x = self._stack(feats)
        return x.reshape(-1, self.in_dim).to(torch.float32).to(self.device)

    def _fused_ok(self, points: torch.Tensor) -> bool:
        """The one-launch HIP metric applies to the stock architecture
        (three Linear(32) layers, fp32 parameters) on the GPU."""
        if not (points.is_cuda and points.dtype == torch.float32 and 1 <= self.in_dim <= 16):
            return False
        for net in (self.target_network, self.predictor_network):
            lin = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
            if len(lin) != 3 or any(m.out_features != 32 or m.bias is None or
                                    m.weight.dtype != torch.float32 or not m.weight.is_cuda
                                    for m in lin):
                return False
        return True

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
        r = self.compute_distance(points)
        per_env = isinstance(last, torch.Tensor) and last.dim() == len(self.input_shape) + 2
        if per_env:
            r = self.metric_results.reshape(last.shape[0], -1).mean(dim=1, keepdim=True)
        if self.clip_rewards is not None:
            r = torch.clamp(r, *self.clip_rewards)
        return r
