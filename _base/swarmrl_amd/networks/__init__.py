from swarmrl_amd.networks.torch_network import ActorCriticMLP, TorchModel

__all__ = ["ActorCriticMLP", "TorchModel"]
