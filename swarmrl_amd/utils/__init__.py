from swarmrl_amd.utils import utils
from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

__all__ = ["utils", "TrajectoryInformation"]
