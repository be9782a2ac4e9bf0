from swarmrl_amd.components.colloid import Colloid

__all__ = ["Colloid"]
