"""
Parent class for the engine (reference: swarmrl/engine/engine.py:8-45).
"""


class Engine:
    """
    Parent class for an engine: something that generates data for the
    environment.  ``integrate`` advances the system by ``n_slices`` RL time
    slices, calling the force model at every slice boundary.
    """

    def integrate(self, n_slices: int, force_model) -> None:
        raise NotImplementedError

    def get_particle_data(self) -> dict:
        """Type, id, position, velocity and director of the particles."""
        raise NotImplementedError

    def finalize(self):
        """Optional clean-up after the simulation (e.g. flush trajectories)."""
        pass
