from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

__all__ = ["TrajectoryInformation"]
