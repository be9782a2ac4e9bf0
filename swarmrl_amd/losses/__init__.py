from swarmrl_amd.losses.proximal_policy_loss import Loss, ProximalPolicyLoss

__all__ = ["Loss", "ProximalPolicyLoss"]
