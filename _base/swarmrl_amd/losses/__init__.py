from swarmrl_amd.losses.policy_gradient_loss import PolicyGradientLoss
from swarmrl_amd.losses.proximal_policy_loss import Loss, ProximalPolicyLoss

__all__ = ["Loss", "PolicyGradientLoss", "ProximalPolicyLoss"]
