from swarmrl_amd.actions.actions import Action

__all__ = ["Action"]
