from swarmrl_amd.tasks.searching.gradient_sensing import GradientSensing
from swarmrl_amd.tasks.searching.species_search import SpeciesSearch

__all__ = ["GradientSensing", "SpeciesSearch"]
