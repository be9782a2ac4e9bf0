from swarmrl_amd.force_functions.force_fn import ForceFunction

__all__ = ["ForceFunction"]
