from swarmrl_amd.engine.engine import Engine
from swarmrl_amd.engine.swarm_engine import EspressoMD, MDParams, SwarmEngine

__all__ = ["Engine", "SwarmEngine", "EspressoMD", "MDParams"]
