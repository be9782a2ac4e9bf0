from swarmrl_amd.tasks.searching.gradient_sensing import GradientSensing

__all__ = ["GradientSensing"]
