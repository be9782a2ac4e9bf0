"""
Actor-critic agent (reference: swarmrl/agents/actor_critic.py:20-216).

calc_action: observable -> network -> action table -> trajectory append;
calc_reward: task (+ intrinsic) + external -> trajectory append (called by
the engine after every integration chunk).  With a SwarmView the whole slice
stays on the GPU: the observable is a HIP kernel, the policy a torch MLP,
the action table a device gather, and the trajectory holds device tensors.
"""

import numpy as np
import torch

from swarmrl_amd.agents.agent import Agent
from swarmrl_amd.engine.swarm_view import DeviceActions, is_view
from swarmrl_amd.losses.proximal_policy_loss import ProximalPolicyLoss
from swarmrl_amd.utils.colloid_utils import TrajectoryInformation


class ActorCriticAgent(Agent):
    """Class to handle the actor-critic RL protocol."""

    def __init__(
        self,
        particle_type: int,
        network,
        task,
        observable,
        actions: dict,
        loss=None,
        train: bool = True,
        intrinsic_reward=None,
    ):
        self.network = network
        self.particle_type = particle_type
        self.task = task
        self.observable = observable
        self.actions = actions
        self.train = train
        self.loss = loss if loss is not None else ProximalPolicyLoss()
        self.intrinsic_reward = intrinsic_reward
        self.trajectory = TrajectoryInformation(particle_type=self.particle_type)
        self._tables = None

    def __name__(self) -> str:
        return "ActorCriticAgent"

    def absorbs_build(self) -> bool:
        """True when this agent's device calc_action launches the engine-bound
        kernels a deferred cluster build rides along in (the vision cone, or
        with a concentration field the field reward, then the one-kernel
        policy): SwarmEngine then defers the build instead of forking it onto
        a second stream.  Engines that cannot carry it decline the deferral
        (swarm_engine_defer_build) and fork as before."""
        from swarmrl_amd.observables.concentration_field import ConcentrationField
        from swarmrl_amd.observables.subdivided_vision_cones import SubdividedVisionCones

        return (isinstance(self.observable, (SubdividedVisionCones, ConcentrationField))
                and getattr(self.network, "accepts_engine", False))

    def supports_device(self) -> bool:
        ok = getattr(self.observable, "supports_device", False) and getattr(
            self.task, "supports_device", False
        )
        if self.intrinsic_reward is not None:
            ok = ok and getattr(self.intrinsic_reward, "supports_device", False)
        return bool(ok) and hasattr(self.network, "compute_action")

    # ----------------------------------------------------------- training
    def update_agent(self, episode_data=None, update_fn=None) -> tuple:
        """Train on the episode and start a new trajectory (actor_critic.py:
        80-109).  episode_data: the episode to learn from, by default this
        agent's own trajectory -- the episode-parallel trainer passes the
        trajectory all-gathered over the ranks (rollout.gather_episode), and
        update_fn(agent, episode) replaces the loss + intrinsic-reward step
        (rollout.replicated_update).  Returns the rewards and the kill switch
        of that episode."""
        episode = self.trajectory if episode_data is None else episode_data
        rewards = episode.rewards
        killed = episode.killed
        if update_fn is not None:
            update_fn(self, episode)
        else:
            self.loss.compute_loss(network=self.network, episode_data=episode)
            if self.intrinsic_reward:
                self.intrinsic_reward.update(episode)
        self.reset_trajectory()
        return rewards, killed

    def reset_agent(self, colloids):
        self.observable.initialize(colloids)
        self.task.initialize(colloids)

    def reset_trajectory(self):
        self.task.kill_switch = False
        self.trajectory = TrajectoryInformation(particle_type=self.particle_type)

    def initialize_network(self):
        self.network.reinitialize_network()

    def save_agent(self, directory: str):
        self.network.export_model(
            filename=f"{self.__name__()}_{self.particle_type}", directory=directory
        )

    def restore_agent(self, directory: str):
        self.network.restore_model_state(
            filename=f"{self.__name__()}_{self.particle_type}", directory=directory
        )

    # ------------------------------------------------------------- acting
    def _action_tables(self, device):
        if self._tables is None or self._tables[0] != device:
            acts = list(self.actions.values())
            f = torch.tensor([float(a.force) for a in acts], dtype=torch.float32, device=device)
            tz = torch.tensor(
                [0.0 if a.torque is None else float(np.asarray(a.torque, dtype=float)[2])
                 for a in acts],
                dtype=torch.float32, device=device,
            )
            has_dir = any(a.new_direction is not None for a in acts)
            self._tables = (device, f, tz, has_dir)
        return self._tables

    def calc_action(self, colloids):
        joint = None
        if is_view(colloids):
            # the observable and the network's rollout policy in one launch
            # when both allow it (SubdividedVisionCones + the stock MLP)
            with_policy = getattr(self.observable, "compute_with_policy", None)
            if with_policy is not None:
                _, ftab, ttab, _ = self._action_tables(colloids.device)
                joint = with_policy(colloids, self.network, ftab, ttab)
        state_description = (joint[0] if joint is not None
                             else self.observable.compute_observable(colloids))
        if is_view(colloids):
            E = colloids.n_envs
            A = int(state_description.shape[1])
            flat = state_description.reshape(E * A, -1)
            _, ftab, ttab, has_dir = self._action_tables(colloids.device)
            fused = getattr(self.network, "fused_sampling_ok", None)
            if joint is not None:
                idx, logp, f_act, t_act = joint[1:]
                f_act, t_act = f_act.reshape(E, A), t_act.reshape(E, A)
            elif fused is not None and fused(flat):
                if getattr(self.network, "accepts_engine", False):
                    idx, logp, f_act, t_act = self.network.compute_action_fused(
                        flat, ftab, ttab, engine=colloids.engine._native)
                else:
                    idx, logp, f_act, t_act = self.network.compute_action_fused(flat, ftab, ttab)
                f_act, t_act = f_act.reshape(E, A), t_act.reshape(E, A)
            else:
                idx, logp = self.network.compute_action(observables=flat)
                f_act = t_act = None
            idx = idx.reshape(E, A)
            logp = logp.reshape(E, A)
            new_dir = None
            mask = None
            if has_dir:
                acts = list(self.actions.values())
                host_idx = idx.cpu().numpy()
                new_dir = np.zeros((E, A, 3))
                mask = np.zeros((E, A), dtype=bool)
                for k, a in enumerate(acts):
                    if a.new_direction is not None:
                        sel = host_idx == k
                        new_dir[sel] = a.new_direction
                        mask[sel] = True
            if f_act is None:
                f_act, t_act = ftab[idx], ttab[idx]
            chosen = DeviceActions(f_act, t_act, new_dir, mask)
            if self.train:
                self.trajectory.features.append(state_description)
                self.trajectory.actions.append(idx)
                self.trajectory.log_probs.append(logp)
                self.trajectory.killed = self.task.kill_switch
            return chosen
        action_indices, log_probs = self.network.compute_action(observables=state_description)
        chosen_actions = np.take(list(self.actions.values()), action_indices, axis=-1)
        if self.train:
            self.trajectory.features.append(state_description)
            self.trajectory.actions.append(action_indices)
            self.trajectory.log_probs.append(log_probs)
            self.trajectory.killed = self.task.kill_switch
        return chosen_actions

    def calc_reward(self, colloids, external_reward: float = 0.0):
        rewards = self.task(colloids)
        if self.intrinsic_reward:
            add = getattr(self.intrinsic_reward, "add_to_reward", None)
            if add is not None:  # task + intrinsic fused on the device (RNDReward)
                rewards = add(rewards, self.trajectory)
            else:
                rewards = rewards + self.intrinsic_reward.compute_reward(
                    episode_data=self.trajectory)
        if not (isinstance(external_reward, (int, float)) and external_reward == 0):
            rewards = rewards + external_reward
        if self.train:
            self.trajectory.rewards.append(rewards)
        self.kill_switch = self.task.kill_switch
        return rewards
