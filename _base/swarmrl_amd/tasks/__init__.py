from swarmrl_amd.tasks import searching
from swarmrl_amd.tasks.multi_tasking import MultiTasking
from swarmrl_amd.tasks.task import Task

__all__ = ["Task", "MultiTasking", "searching"]
