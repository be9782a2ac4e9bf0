from swarmrl_amd.observables.concentration_field import ConcentrationField
from swarmrl_amd.observables.director import Director
from swarmrl_amd.observables.multi_sensing import MultiSensing
from swarmrl_amd.observables.observable import Observable
from swarmrl_amd.observables.particle_sensing import ParticleSensing
from swarmrl_amd.observables.position import PositionObservable
from swarmrl_amd.observables.subdivided_vision_cones import SubdividedVisionCones

__all__ = ["Observable", "ConcentrationField", "Director", "MultiSensing", "ParticleSensing",
           "PositionObservable", "SubdividedVisionCones"]
