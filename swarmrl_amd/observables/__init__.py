from swarmrl_amd.observables.concentration_field import ConcentrationField
from swarmrl_amd.observables.observable import Observable
from swarmrl_amd.observables.particle_sensing import ParticleSensing
from swarmrl_amd.observables.subdivided_vision_cones import SubdividedVisionCones

__all__ = ["Observable", "ConcentrationField", "ParticleSensing", "SubdividedVisionCones"]
