"""
MI355X swarm engine: drop-in for ``swarmrl.engine.espresso.EspressoMD``.

Reference: swarmrl/engine/espresso.py.  The Python surface (MDParams,
constructor, add_colloids / add_colloid_on_point, integrate, manage_forces,
get_particle_data, finalize, the step/slice/write counters and the trajectory
holder) mirrors the reference line by line; the physics that ESPResSo did
(Brownian dynamics, WCA with a cell system, steepest descent) runs in the HIP
library through the C ABI of include/swarmrl_amd.h.  There is no CPU
fallback: without a HIP device the engine raises.

Scope of this build: 2-D, periodic box, isotropic spheres
(WCA), Brownian thermostat.  3-D, walls, rods, Gay-Berne, LB and the Langevin
integrator raise NotImplementedError.
"""

from __future__ import annotations

import ctypes
import os
import logging
import pathlib
import typing

import numpy as np
import torch

from swarmrl_amd import _capi
from swarmrl_amd.components.colloid import Colloid
from swarmrl_amd.engine.engine import Engine
from swarmrl_amd.engine.swarm_view import DeviceActions, SwarmView
from swarmrl_amd.units import Quantity, UnitRegistry, ensure_quantity_array

logger = logging.getLogger(__name__)


class MDParams:
    """
    All information needed to set up and run the simulation
    (reference: espresso.py:30-88).  Quantities may be given in any unit;
    they are converted to simulation units during setup.
    """

    def __init__(
        self,
        ureg: UnitRegistry,
        box_length: Quantity = None,
        fluid_dyn_viscosity: Quantity = None,
        WCA_epsilon: Quantity = None,
        temperature: Quantity = None,
        time_step: Quantity = None,
        time_slice: Quantity = None,
        write_interval: Quantity = None,
        periodic: bool = True,
        thermostat_type: str = "brownian",
    ):
        if box_length is None:
            box_length = ureg.Quantity(3 * [1000], "micrometer")
        if fluid_dyn_viscosity is None:
            fluid_dyn_viscosity = ureg.Quantity(1e-3, "pascal*second")
        if WCA_epsilon is None:
            WCA_epsilon = ureg.Quantity(300, "kelvin") * ureg.boltzmann_constant
        if temperature is None:
            temperature = ureg.Quantity(300, "kelvin")
        if time_step is None:
            time_step = ureg.Quantity(1e-3, "second")
        if time_slice is None:
            time_slice = ureg.Quantity(1e-1, "second")
        if write_interval is None:
            write_interval = ureg.Quantity(1, "second")

        self.ureg = ureg
        self.box_length = box_length
        self.fluid_dyn_viscosity = fluid_dyn_viscosity
        self.WCA_epsilon = WCA_epsilon
        self.temperature = temperature
        self.time_step = time_step
        self.time_slice = time_slice
        self.write_interval = write_interval
        self.periodic = periodic
        self.thermostat_type = thermostat_type


def _get_random_start_pos(
    init_radius: float, init_center: np.ndarray, dim: int, rng: np.random.Generator
):
    """Uniform point in a disc (2-D) or ball (3-D), espresso.py:91-105."""
    if dim == 2:
        r = init_radius * np.sqrt(rng.random())
        theta = 2 * np.pi * rng.random()
        pos = r * np.array([np.cos(theta), np.sin(theta), 0])
        assert init_center[2] == 0.0
    elif dim == 3:
        r = init_radius * np.cbrt(rng.random())
        pos = r * _vector_from_angles(*_get_random_angles(rng))
    else:
        raise ValueError("Random position finder only implemented for 2d and 3d")
    return pos + init_center


def _get_random_angles(rng: np.random.Generator):
    """utils.get_random_angles (utils.py:19-21): uniform on the sphere."""
    return np.arccos(2.0 * rng.random() - 1), 2.0 * np.pi * rng.random()


def _calc_friction_coefficients(dyn_visc: float, radius: float):
    """Stokes friction of a sphere (espresso.py:108-113)."""
    particle_gamma_translation = 6 * np.pi * dyn_visc * radius
    particle_gamma_rotation = 8 * np.pi * dyn_visc * radius**3
    return particle_gamma_translation, particle_gamma_rotation


def _vector_from_angles(theta, phi):
    """utils.vector_from_angles (utils.py:24-27)."""
    return np.array(
        [np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi), np.cos(theta)]
    )


def _angles_from_vector(director):
    """utils.angles_from_vector (utils.py:30-34)."""
    director = director / np.linalg.norm(director)
    theta = np.arccos(director[2])
    phi = np.arctan2(director[1], director[0])
    return theta, phi


class _SystemState:
    """The part of espressomd.System the engine surface exposes: the time."""

    def __init__(self):
        self.time = 0.0
        self.constraints = []  # wall shapes (espressomd.constraints analogue)


class _Particle:
    """
    Particle handle with the attributes SwarmRL reads from ESPResSo handles
    (pos, v, director, id, type).  Values come from the engine's host mirror
    of env 0, refreshed after every integration chunk.
    """

    __slots__ = ("_engine", "_index", "id", "type")

    def __init__(self, engine, index: int, p_type: int):
        self._engine = engine
        self._index = index
        self.id = index
        self.type = p_type

    @property
    def pos(self):
        return self._engine._host()["pos"][0, self._index].copy()

    @property
    def v(self):
        return self._engine._host()["vel"][0, self._index].copy()

    velocity = v

    @property
    def director(self):
        return self._engine._host()["dir"][0, self._index].copy()

    def __repr__(self):
        return f"Particle(id={self.id}, type={self.type})"


# Engine handles whose owner was collected while a HIP graph capture was in
# progress: freeing device memory then would invalidate the capture (the
# garbage collector may run a finalizer at any allocation), so they are
# destroyed at the next engine creation instead.
_DEFERRED_DESTROY = []


def _destroy_deferred():
    while _DEFERRED_DESTROY:
        lib, ptr = _DEFERRED_DESTROY.pop()
        lib.swarm_engine_destroy(ptr)


class _NativeEngine:
    """Owner of one C-ABI engine handle."""

    def __init__(self, params: _capi.SwarmParams, n_envs: int, species: np.ndarray):
        if not torch.cuda.is_current_stream_capturing():
            _destroy_deferred()
        self._lib = _capi.lib()
        self.ptr = ctypes.c_void_p()
        sp = np.ascontiguousarray(species, dtype=np.int32)
        _capi.check(
            self._lib.swarm_engine_create(
                ctypes.byref(params), n_envs, len(sp), sp.ctypes.data, ctypes.byref(self.ptr)
            )
        )

    def call(self, name, *args):
        _capi.check(getattr(self._lib, name)(self.ptr, *args))

    def bind_stream(self):
        stream = torch.cuda.current_stream().cuda_stream
        _capi.check(self._lib.swarm_engine_set_stream(self.ptr, ctypes.c_void_p(stream)))

    def __del__(self):
        try:
            if self.ptr:
                if torch.cuda.is_current_stream_capturing():
                    _DEFERRED_DESTROY.append((self._lib, self.ptr))
                else:
                    self._lib.swarm_engine_destroy(self.ptr)
                self.ptr = ctypes.c_void_p()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


class SwarmEngine(Engine):
    """
    Drop-in replacement of EspressoMD (espresso.py:132-1347) on MI355X.

    Methods may add particles until the first call to integrate().  Extra
    keyword ``n_envs``: number of independent replicas (episode-parallel
    envs) integrated by the same kernels; env e is placed with
    ``np.random.default_rng(seed + e)`` (env 0 reproduces the reference).
    """

    def __init__(
        self,
        md_params: MDParams,
        n_dims: int = 3,
        seed: int = 42,
        out_folder=".",
        write_chunk_size: int = 100,
        system=None,
        h5_group_tag: str = None,
        n_envs: int = 1,
        reuse_forces: bool = True,
    ):
        self.params: MDParams = md_params
        # integrator.run(k, reuse_forces=True) (espresso.py:1304-1306): the
        # first sub-step of every run uses the forces of the previous run's
        # last force calculation (swim force, torque, director), as ESPResSo's
        # Brownian propagator does; False: the current actions throughout
        self.reuse_forces = bool(reuse_forces)
        self.out_folder = pathlib.Path(out_folder).resolve()
        self.seed = seed
        self.rng = np.random.default_rng(self.seed)
        if n_dims not in [2, 3]:
            raise ValueError("Only 2d and 3d are allowed")
        self.n_dims = n_dims
        if int(n_envs) < 1:
            raise ValueError("n_envs must be >= 1")
        self.n_envs = int(n_envs)
        self._env_rngs = [self.rng] + [
            np.random.default_rng(seed + e) for e in range(1, self.n_envs)
        ]

        self._init_unit_system()
        self.write_chunk_size = write_chunk_size
        self.h5_group_tag = "colloids" if h5_group_tag is None else h5_group_tag

        # a passed system is "reset" (espresso.py:193-196): nothing carries over
        self.system = _SystemState()
        self._init_system()

        self.colloids = list()
        self.colloid_radius_register = {}
        self.integration_initialised = False

        # host registry of added particles (per env)
        self._pos: typing.List[list] = [list() for _ in range(self.n_envs)]
        self._dir: typing.List[list] = [list() for _ in range(self.n_envs)]
        self._types_list: typing.List[int] = []
        self._species_keys: typing.List[tuple] = []
        self._species_of: typing.List[int] = []
        self._ext_force = None
        self._walls = []  # swarm_wall_t dicts (add_confining_walls / add_walls)
        self._native: _NativeEngine = None
        self._host_cache = None
        self._view = None
        self._type_index_cache = {}
        # device path: prepare each window's build on a side stream while
        # the force model computes the slice's actions (see _prebuild); the
        # tests turn these off to compare the schedules
        self.overlap_build = True
        # fork the next slice's build right after the run (before the reward)
        self.early_fork = True
        # latency-bound engines: the next window's build rides along in the
        # vision-cone and policy launches instead of a forked side stream
        # (swarm_engine_defer_build; the engine declines when it cannot)
        self.ride_along_build = True
        self._ride_along = False
        self._side_stream = None
        self._prebuild_pending = None
        self.traj_holder = None
        self._ring = None  # device trajectory ring (_init_traj_ring)
        self._steps_run = 0  # BD sub-steps launched (= the device step counter)
        self._time_offset = 0.0
        self.write_idx = 0
        self.slice_idx = 0
        self.step_idx = 0

    # ------------------------------------------------------------ units
    def _init_unit_system(self):
        """Simulation units (espresso.py:211-234)."""
        self.ureg = self.params.ureg
        self.ureg.define("sim_length = 1e-6 meter")
        self.ureg.define("sim_time = 1 second")
        self.ureg.define("sim_energy = 293 kelvin * boltzmann_constant")
        self.ureg.define("sim_velocity = sim_length / sim_time")
        self.ureg.define("sim_angular_velocity = 1 / sim_time")
        self.ureg.define("sim_mass = sim_energy / sim_velocity**2")
        self.ureg.define("sim_rinertia = sim_length**2 * sim_mass")
        self.ureg.define("sim_dyn_viscosity = sim_mass / (sim_length * sim_time)")
        self.ureg.define("sim_kin_viscosity = sim_length**2 / sim_time")
        self.ureg.define("sim_force = sim_mass * sim_length / sim_time**2")
        self.ureg.define("sim_torque = sim_length * sim_force")

    def _init_system(self):
        """Box, time step and the slice/write schedule (espresso.py:236-288)."""
        time_step = self.params.time_step.m_as("sim_time")
        time_slice = self.params.time_slice.m_as("sim_time")
        write_interval = self.params.write_interval.m_as("sim_time")
        box_l = np.array(self.params.box_length.m_as("sim_length"))
        if np.isscalar(box_l) or box_l.ndim == 0:
            raise ValueError("box_length must be a 3d vector (or 2d if you have a 2d system)")
        if self.n_dims == 2 and len(box_l) == 2:
            box_l = np.array([box_l[0], box_l[1], box_l[0]])
        if len(box_l) != 3:
            raise ValueError(f"box_length must be a 3d vector. You gave {self.params.box_length}")

        self._box = np.asarray(box_l, dtype=float)
        self._time_step = float(time_step)

        steps_per_write_interval = int(round(write_interval / time_step))
        self.params.steps_per_write_interval = steps_per_write_interval
        if abs(steps_per_write_interval - write_interval / time_step) > 1e-10:
            raise ValueError(
                "inconsistent parameters: write_interval must be integer multiple of time_step"
            )
        steps_per_slice = int(round(time_slice / time_step))
        self.params.steps_per_slice = steps_per_slice
        if abs(steps_per_slice - time_slice / time_step) > 1e-10:
            raise ValueError(
                "inconsistent parameters: time_slice must be integer multiple of time_step"
            )

    def _check_already_initialised(self):
        if self.integration_initialised:
            raise RuntimeError(
                "You cannot change the system configuration after the first call to integrate()"
            )

    # ------------------------------------------------------ particle setup
    def _register_particle(self, positions, directions, p_type, species_key):
        """Append one particle to every env (positions/directions per env)."""
        index = len(self._types_list)
        for e in range(self.n_envs):
            self._pos[e].append(np.asarray(positions[e], dtype=float))
            self._dir[e].append(np.asarray(directions[e], dtype=float))
        self._types_list.append(int(p_type))
        if species_key not in self._species_keys:
            if len(self._species_keys) >= _capi.SWARM_MAX_SPECIES:
                raise ValueError("too many distinct particle species for this build")
            self._species_keys.append(species_key)
        self._species_of.append(self._species_keys.index(species_key))
        handle = _Particle(self, index, int(p_type))
        self.colloids.append(handle)
        return handle

    def _particle_properties(
        self, radius_colloid, type_colloid, gamma_translation, gamma_rotation, aspect_ratio,
        mass, rinertia,
    ):
        """Radius/friction/mass handling of add_colloid_on_point (espresso.py:345-413)."""
        if radius_colloid is None:
            radius_colloid = self.ureg.Quantity(1, "micrometer")
        radius_simunits = radius_colloid.m_as("sim_length")
        if type_colloid in self.colloid_radius_register.keys():
            if self.colloid_radius_register[type_colloid]["radius"] != radius_simunits:
                raise ValueError(
                    f"The chosen type {type_colloid} is already taken and used with a"
                    " different radius"
                    f" {self.colloid_radius_register[type_colloid]['radius']}. Choose a"
                    " new combination"
                )
        if aspect_ratio != 1.0:
            raise NotImplementedError(
                "aspect_ratio != 1 (Gay-Berne) is not implemented in this build"
            )
        gt_sphere, gr_sphere = _calc_friction_coefficients(
            self.params.fluid_dyn_viscosity.m_as("sim_dyn_viscosity"), radius_simunits
        )
        if gamma_translation is None:
            gamma_translation = gt_sphere
        else:
            gamma_translation = gamma_translation.m_as("sim_force/sim_velocity")
        if gamma_rotation is None:
            gamma_rotation = gr_sphere
        else:
            gamma_rotation = gamma_rotation.m_as("sim_torque/sim_angular_velocity")
        gamma_translation = np.atleast_1d(np.asarray(gamma_translation, dtype=float))
        gamma_rotation = np.atleast_1d(np.asarray(gamma_rotation, dtype=float))
        if np.ptp(gamma_translation) != 0.0 or np.ptp(gamma_rotation) != 0.0:
            raise NotImplementedError("anisotropic friction is not implemented in this build")

        if self.params.thermostat_type == "langevin":
            if mass is None:
                raise ValueError("If you use the Langevin thermostat, you must set a particle mass")
            if rinertia is None:
                raise ValueError(
                    "If you use the Langevin thermostat, you must set a particle rotational inertia"
                )
        else:
            water_dens = self.params.ureg.Quantity(1000, "kg/meter**3")
            if mass is None:
                mass = water_dens * 4.0 / 3.0 * np.pi * radius_colloid**3
            if rinertia is None:
                rinertia = 2.0 / 5.0 * mass * radius_colloid**2
                rinertia = ensure_quantity_array(3 * [rinertia], self.params.ureg)
        mass_s = float(np.atleast_1d(mass.m_as("sim_mass"))[0])
        rin = np.atleast_1d(rinertia.m_as("sim_rinertia"))
        # 2-D rotation is about lab z = body x after _rotate_colloid_to_2d
        rin_z = float(rin[0])
        key = (
            float(radius_simunits),
            float(gamma_translation[0]),
            float(gamma_rotation[0]),
            mass_s,
            rin_z,
        )
        return radius_simunits, key

    def add_colloid_on_point(
        self,
        radius_colloid: Quantity = None,
        init_position: Quantity = None,
        init_direction: np.ndarray = np.array([1, 0, 0]),
        type_colloid=0,
        gamma_translation: Quantity = None,
        gamma_rotation: Quantity = None,
        aspect_ratio: float = 1.0,
        mass: Quantity = None,
        rinertia: Quantity = None,
    ):
        """Add one colloid at a point (espresso.py:307-457); same point in every env."""
        self._check_already_initialised()
        if init_position is None:
            init_position = 0.5 * self.params.box_length
        radius_simunits, key = self._particle_properties(
            radius_colloid, type_colloid, gamma_translation, gamma_rotation, aspect_ratio,
            mass, rinertia,
        )
        init_pos = np.array(init_position.m_as("sim_length"), dtype=float)
        init_direction = np.asarray(init_direction, dtype=float)
        init_direction = init_direction / np.linalg.norm(init_direction)
        if self.n_dims == 3:  # espresso.py:415-426
            handle = self._register_particle(
                [init_pos] * self.n_envs, [init_direction] * self.n_envs, type_colloid, key
            )
            self.colloid_radius_register.update(
                {type_colloid: {"radius": radius_simunits, "aspect_ratio": aspect_ratio}}
            )
            return handle
        init_pos[2] = 0
        theta, phi = _angles_from_vector(init_direction)
        if abs(theta - np.pi / 2) > 10e-6:
            raise ValueError(
                "It seems like you want to have a 2D simulation"
                " with colloids that point some amount in Z-direction."
                " Change something in your colloid setup."
            )
        direction = np.array([np.cos(phi), np.sin(phi), 0.0])
        handle = self._register_particle(
            [init_pos] * self.n_envs, [direction] * self.n_envs, type_colloid, key
        )
        self.colloid_radius_register.update(
            {type_colloid: {"radius": radius_simunits, "aspect_ratio": aspect_ratio}}
        )
        return handle

    def add_colloids(
        self,
        n_colloids: int,
        radius_colloid: Quantity = None,
        random_placement_center: Quantity = None,
        random_placement_radius: Quantity = None,
        type_colloid: int = 0,
        gamma_translation: Quantity = None,
        gamma_rotation: Quantity = None,
        aspect_ratio: float = 1.0,
        mass: Quantity = None,
        rinertia: Quantity = None,
    ):
        """
        Random placement in a disc (espresso.py:459-544).  Per colloid the
        generator draws r, theta, then the director angle (espresso.py:95-96,
        532); env e uses its own generator.
        """
        self._check_already_initialised()
        if random_placement_center is None:
            random_placement_center = self.ureg.Quantity(
                0.5 * self.params.box_length.m_as("sim_length"), "sim_length"
            )
        if random_placement_radius is None:
            random_placement_radius = 0.5 * min(self.params.box_length)
        init_center = np.array(random_placement_center.m_as("sim_length"), dtype=float)
        init_rad = random_placement_radius.m_as("sim_length")
        radius_simunits, key = self._particle_properties(
            radius_colloid, type_colloid, gamma_translation, gamma_rotation, aspect_ratio,
            mass, rinertia,
        )
        for _ in range(n_colloids):
            positions, directions = [], []
            for e in range(self.n_envs):
                rng = self._env_rngs[e]
                start_pos = _get_random_start_pos(init_rad, init_center, self.n_dims, rng)
                if self.n_dims == 3:  # espresso.py:526-529
                    d = _vector_from_angles(*_get_random_angles(rng))
                    positions.append(np.array(start_pos, dtype=float))
                    directions.append(d / np.linalg.norm(d))
                    continue
                start_angle = 2 * np.pi * rng.random()
                init_direction = _vector_from_angles(np.pi / 2, start_angle)
                init_direction = init_direction / np.linalg.norm(init_direction)
                _, phi = _angles_from_vector(init_direction)
                pos = np.array(start_pos, dtype=float)
                pos[2] = 0
                positions.append(pos)
                directions.append(np.array([np.cos(phi), np.sin(phi), 0.0]))
            self._register_particle(positions, directions, type_colloid, key)
        self.colloid_radius_register.update(
            {type_colloid: {"radius": radius_simunits, "aspect_ratio": aspect_ratio}}
        )

    def add_const_force_to_colloids(self, force: Quantity, type: int):
        """Constant external force on every colloid of a type (espresso.py:834-851)."""
        f = np.asarray(force.m_as("sim_force"), dtype=float)
        if self._ext_force is None:
            self._ext_force = np.zeros((self.n_envs, len(self._types_list), 3))
        mask = np.asarray(self._types_list) == type
        self._ext_force[:, mask, :] = f
        if self._native is not None:
            self._native.bind_stream()
            ext = np.ascontiguousarray(self._ext_force.reshape(-1, 3))
            self._native.call("swarm_engine_set_external_force", ext.ctypes.data)

    def add_confining_walls(self, wall_type: int):
        """WCA walls on the box faces (espresso.py:667-704): x = 0, x = L_x,
        y = 0, y = L_y (and z in 3-D), interacting with every particle."""
        self._check_already_initialised()
        if wall_type in self.colloid_radius_register.keys():
            raise ValueError(
                f"wall type {wall_type} is already taken by other system component. "
                "Choose a new one"
            )
        L = self._box
        normals = [([1, 0, 0], 0.0), ([-1, 0, 0], -L[0]), ([0, 1, 0], 0.0), ([0, -1, 0], -L[1])]
        if self.n_dims == 3:
            normals += [([0, 0, 1], 0.0), ([0, 0, -1], -L[2])]
        for n, off in normals:
            self._add_wall({"kind": 0, "normal": n, "offset": off})
        self.colloid_radius_register.update({wall_type: {"radius": 0.0, "aspect_ratio": 1.0}})

    def add_walls(self, wall_start_point: Quantity, wall_end_point: Quantity, wall_type: int,
                  wall_thickness: Quantity):
        """Rectangular walls from start to end points of the given thickness,
        spanning the box in z (espresso.py:706-800, Rhomboid constraints)."""
        start = np.asarray(wall_start_point.m_as("sim_length"), dtype=float)
        end = np.asarray(wall_end_point.m_as("sim_length"), dtype=float)
        thickness = float(wall_thickness.m_as("sim_length"))
        if len(start) != len(end):
            raise ValueError(
                " Please double check your walls. There are more or less "
                f" starting points {len(start)} than "
                f" end points {len(end)}. They should be equal."
            )
        self._check_already_initialised()
        if wall_type in self.colloid_radius_register.keys():
            if self.colloid_radius_register[wall_type] != 0.0:
                raise ValueError(
                    f" The chosen type {wall_type} is already taken"
                    "and used with a different radius "
                    f"{self.colloid_radius_register[wall_type]['radius']}."
                    " Choose a new combination"
                )
        z_height = self._box[2]
        for k in range(len(start)):
            a = np.array([end[k, 0] - start[k, 0], end[k, 1] - start[k, 1], 0.0])
            c = np.array([0.0, 0.0, z_height])
            b = np.cross(a / np.linalg.norm(a), c / np.linalg.norm(c)) * thickness
            corner = [start[k, 0] - b[0] / 2, start[k, 1] - b[1] / 2, 0.0]
            self._add_wall({"kind": 1, "corner": corner, "a": a, "b": b})
        self.colloid_radius_register.update({wall_type: {"radius": 0.0, "aspect_ratio": 1.0}})

    def _add_wall(self, wall: dict):
        if len(self._walls) >= _capi.SWARM_MAX_WALLS:
            raise ValueError(f"at most {_capi.SWARM_MAX_WALLS} walls are supported")
        self._walls.append(wall)
        self.system.constraints.append(wall)

    def wall_violations(self) -> int:
        """Wall contacts with distance <= 0 so far (ESPResSo raises on those)."""
        if self._native is None:
            return 0
        v = np.zeros(1, np.uint64)
        self._native.call("swarm_engine_wall_violations", v.ctypes.data)
        return int(v[0])

    def get_friction_coefficients(self, type: int):
        """espresso.py:1038-1052."""
        property_dict = self.colloid_radius_register.get(type, None)
        if property_dict is None:
            raise ValueError(
                f"cannot get friction coefficient for type {type}. Did you actually add"
                " that particle type?"
            )
        return _calc_friction_coefficients(
            self.params.fluid_dyn_viscosity.m_as("sim_dyn_viscosity"),
            property_dict["radius"],
        )

    # ------------------------------------------------------- native setup
    @property
    def n_particles(self) -> int:
        return len(self._types_list)

    @property
    def device(self):
        if torch.cuda.is_available():
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _kT(self) -> float:
        return (self.params.temperature * self.ureg.boltzmann_constant).m_as("sim_energy")

    def _setup_interactions(self):
        """WCA between every pair of types (espresso.py:802-832) + engine creation."""
        _capi.require_gpu()
        if self.n_particles == 0:
            raise ValueError("no colloids were added to the engine")
        aspect_ratios = [d["aspect_ratio"] for d in self.colloid_radius_register.values()]
        if len(np.unique(aspect_ratios)) > 1:
            raise ValueError("All particles in the system must have the same aspect ratio.")
        if self.params.thermostat_type not in ["brownian", "langevin"]:
            raise ValueError("integrator_type must be one of ['brownian', 'langevin']")
        if self.params.thermostat_type == "langevin":
            raise NotImplementedError("the Langevin integrator is not implemented in this build")

        p = _capi.SwarmParams()
        p.n_dims = self.n_dims
        p.periodic = 1 if self.params.periodic else 0
        for a in range(3):
            p.box[a] = float(self._box[a])
        p.time_step = self._time_step
        p.kT = float(self._kT())
        p.wca_epsilon = float(self.params.WCA_epsilon.m_as("sim_energy"))
        p.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        p.n_species = len(self._species_keys)
        p.reuse_forces = 1 if self.reuse_forces else 0
        for s, (r, gt, gr, m, rin) in enumerate(self._species_keys):
            p.radius[s], p.gamma_t[s], p.gamma_r[s] = r, gt, gr
            p.mass[s], p.rinertia[s] = m, rin
        self._params_c = p
        self._native = _NativeEngine(p, self.n_envs, np.asarray(self._species_of))
        self._native.bind_stream()

        pos = np.ascontiguousarray(np.stack([np.stack(v) for v in self._pos]), dtype=float)
        dirs = np.ascontiguousarray(np.stack([np.stack(v) for v in self._dir]), dtype=float)
        self._native.call("swarm_engine_upload_state", pos.ctypes.data, dirs.ctypes.data)
        if self._ext_force is not None:
            ext = np.ascontiguousarray(self._ext_force.reshape(-1, 3))
            self._native.call("swarm_engine_set_external_force", ext.ctypes.data)
        if self._walls:
            arr = (_capi.SwarmWall * len(self._walls))()
            for k, w in enumerate(self._walls):
                arr[k].kind = w["kind"]
                for key in ("normal", "corner", "a", "b"):
                    if key in w:
                        for a in range(3):
                            getattr(arr[k], key)[a] = float(w[key][a])
                arr[k].offset = float(w.get("offset", 0.0))
            self._native.call("swarm_engine_set_walls", ctypes.cast(arr, ctypes.c_void_p),
                              len(self._walls))

        self._types_host = np.asarray(self._types_list, dtype=np.int32)
        self._types_device = torch.as_tensor(self._types_host, device=self.device)
        radii = np.array([self._species_keys[s][0] for s in self._species_of], dtype=np.float32)
        self._radii_device = torch.as_tensor(radii, device=self.device)
        self._host_cache = None

    def _remove_overlap(self):
        """Steepest descent, 1000 steps (espresso.py:1161-1168); time is restored."""
        time = self.system.time
        self._native.bind_stream()
        self._native.call("swarm_engine_remove_overlap", 1000, 0.1, 0.1)
        self.system.time = time
        self._host_cache = None

    # --------------------------------------------------------- trajectory
    def _init_h5_output(self):
        """Trajectory holder + writer (espresso.py:1054-1108)."""
        self.h5_filename = self.out_folder / "trajectory.hdf5"
        self.out_folder.mkdir(parents=True, exist_ok=True)
        self.traj_holder = {
            "Times": list(),
            "Ids": list(),
            "Types": list(),
            "Unwrapped_Positions": list(),
            "Velocities": list(),
            "Directors": list(),
        }
        from swarmrl_amd.engine import trajectory_writer

        self._writer = trajectory_writer.make_writer(
            self.h5_filename, self.h5_group_tag, self.n_particles, self.write_chunk_size
        )
        self.write_idx = 0
        self.h5_time_steps_written = 0
        self._init_traj_ring()

    def _init_traj_ring(self):
        """Device trajectory recording (swarm_engine_traj_ring): each write
        point copies env 0's state into a host-pinned ring from the engine
        stream, with no host synchronisation, so writes can sit inside a
        captured episode graph; the host drains the ring into traj_holder
        (eagerly after each write when not capturing, as the reference's
        _update_traj_holder; otherwise at flush_trajectory / finalize)."""
        self._ring = None
        if self._native is None or len(self.colloids) == 0 or \
                os.environ.get("SWARMRL_AMD_DEVICE_TRAJ", "1") == "0":
            return
        host = ctypes.c_void_p()
        eb = ctypes.c_int64()
        entry_bytes = 8 + 4 * self.n_particles * (3 * self.n_dims + (3 if self.n_dims == 3 else 1))
        cap = max(16, min(2 * int(self.write_chunk_size), (256 << 20) // max(entry_bytes, 1)))
        self._native.bind_stream()
        self._native.call("swarm_engine_traj_ring", int(cap), 0, ctypes.byref(host),
                          ctypes.byref(eb))
        if not host.value:  # a backend without the ring: host-path writes
            return
        self._ring = {"ptr": host.value, "cap": cap, "entry": eb.value, "drained": 0,
                      "count": np.ctypeslib.as_array((ctypes.c_uint64 * 1).from_address(host.value))}
        self._time_offset = self.system.time - self._steps_run * self._time_step

    def _update_traj_holder(self):
        """espresso.py:1110-1130 (env 0)."""
        if len(self.colloids) == 0:
            logger.warning("No colloids in the system. Not writing to hdf5")
            return
        if self._ring is not None:
            # Times = step * dt + offset: a replayed graph records at the
            # device step counter, which the host does not see
            self._time_offset = self.system.time - self._steps_run * self._time_step
            self._native.bind_stream()
            self._native.call("swarm_engine_traj_record")
            if not torch.cuda.is_current_stream_capturing():
                self.drain_trajectory(block=True)
            return
        h = self._host()
        self._append_traj(self.system.time, h["pos"][0].copy(), h["vel"][0].copy(),
                          h["dir"][0].copy())

    def _append_traj(self, time, pos, vel, dirs):
        self.traj_holder["Times"].append(np.array([time])[:, np.newaxis])
        self.traj_holder["Ids"].append(np.arange(self.n_particles)[:, np.newaxis])
        self.traj_holder["Types"].append(np.asarray(self._types_list)[:, np.newaxis])
        self.traj_holder["Unwrapped_Positions"].append(pos)
        self.traj_holder["Velocities"].append(vel)
        self.traj_holder["Directors"].append(dirs)

    def drain_trajectory(self, block: bool = True) -> int:
        """Move the ring entries recorded so far into traj_holder, writing a
        chunk whenever write_chunk_size entries are held (espresso.py:
        1278-1285).  block=False reads what the device has published without
        waiting (entries of work still queued stay for a later call).
        Returns the number of entries drained."""
        ring = self._ring
        if ring is None or self.traj_holder is None:
            return 0
        if block:
            torch.cuda.current_stream().synchronize()
        count = int(ring["count"][0])
        start = ring["drained"]
        cap = ring["cap"]
        # Entry k lives in slot k % cap and is overwritten by entry k + cap,
        # whose write starts as soon as the published count reaches k + cap
        # (before the count moves past it).  With the stream drained nothing
        # is in flight, so cap entries are readable; without waiting, entry k
        # is readable only while the count stays below k + cap.
        if count - start > (cap if block else cap - 1):
            raise RuntimeError(
                f"trajectory ring overflow: {count - start} entries since the last drain, "
                f"capacity {cap} (drain more often)")
        N = self.n_particles
        step = np.zeros(1, np.uint64)
        for k in range(start, count):
            addr = ring["ptr"] + 64 + (k % cap) * ring["entry"]
            pos = np.zeros((N, 3))
            dirs = np.zeros((N, 3))
            vel = np.zeros((N, 3))
            self._native.call("swarm_traj_entry_to_host", ctypes.c_void_p(addr), pos.ctypes.data,
                              dirs.ctypes.data, vel.ctypes.data, step.ctypes.data)
            if not block and int(ring["count"][0]) >= k + cap:  # overwritten while being read
                # entries start..k-1 are in traj_holder already: a caller that
                # catches this and drains again must not append them twice
                ring["drained"] = k
                raise RuntimeError("trajectory ring overflow while draining (drain more often)")
            self._append_traj(self._time_offset + int(step[0]) * self._time_step, pos, vel, dirs)
            ring["drained"] = k + 1
            if len(self.traj_holder["Times"]) >= self.write_chunk_size:
                self._write_traj_chunk_to_file()
                for val in self.traj_holder.values():
                    val.clear()
        ring["drained"] = count
        return count - start

    def flush_trajectory(self):
        """Drain the device ring and write everything held to the file."""
        self.drain_trajectory(block=True)
        self._write_traj_chunk_to_file()
        for val in self.traj_holder.values():
            val.clear()

    def _write_traj_chunk_to_file(self):
        """espresso.py:1132-1159."""
        n_new_timesteps = len(self.traj_holder["Times"])
        if n_new_timesteps == 0:
            return
        values = {k: np.stack(v, axis=0) for k, v in self.traj_holder.items()}
        self._writer.write(values, self.h5_time_steps_written)
        logger.debug(f"wrote {n_new_timesteps} time steps to the trajectory file")
        self.h5_time_steps_written += n_new_timesteps

    # ------------------------------------------------------- host mirror
    def _host(self) -> dict:
        """fp64 copies of pos/dir/vel [E, N, 3], refreshed after integration."""
        if self._host_cache is None:
            E, N = self.n_envs, self.n_particles
            pos = np.zeros((E, N, 3))
            dirs = np.zeros((E, N, 3))
            vel = np.zeros((E, N, 3))
            if self._native is None:
                pos[:] = np.stack([np.stack(v) for v in self._pos])
                dirs[:] = np.stack([np.stack(v) for v in self._dir])
            else:
                self._native.bind_stream()
                self._native.call(
                    "swarm_engine_download_state", pos.ctypes.data, dirs.ctypes.data,
                    vel.ctypes.data,
                )
            self._host_cache = {"pos": pos, "dir": dirs, "vel": vel}
        return self._host_cache

    def _device_views(self) -> _capi.SwarmDeviceViews:
        v = _capi.SwarmDeviceViews()
        _capi.check(self._native._lib.swarm_engine_device_views(self._native.ptr, ctypes.byref(v)))
        return v

    def swarm_view(self) -> SwarmView:
        """Batched device view (the fast path handed to device-capable models)."""
        if self._view is None:
            self._view = SwarmView(self)
        return self._view

    # ------------------------------------------------------------- forces
    @staticmethod
    def _device_capable(force_model) -> bool:
        fn = getattr(force_model, "supports_device", None)
        return bool(fn and fn())

    def apply_device_actions(self, actions: DeviceActions):
        """Write per-particle actions from device tensors [E, N]."""
        E, N = self.n_envs, self.n_particles
        f = actions.f_swim.to(torch.float32).expand(E, N).reshape(E * N).contiguous()
        t = actions.torque_z.to(torch.float32).expand(E, N).reshape(E * N).contiguous()
        # bind (zero copy): the engine reads these buffers until the next
        # set_actions; keep them alive until then
        self._actions_keepalive = (f, t)
        self._native.bind_stream()
        self._native.call("swarm_engine_set_actions", f.data_ptr(), t.data_ptr(), 2)
        if actions.new_direction is not None:
            nd = np.broadcast_to(np.asarray(actions.new_direction, dtype=float), (E, N, 3))
            mask = actions.new_direction_mask
            if mask is None:
                mask = np.ones((E, N), dtype=bool)
            self._set_new_directions(nd, np.broadcast_to(mask, (E, N)))

    def _set_new_directions(self, new_dir: np.ndarray, mask: np.ndarray):
        """espresso.py:1236-1249: 3-D sets the director; 2-D rotates about +-z
        if the angle exceeds 1e-6."""
        if self.n_dims == 3:
            nd = np.ascontiguousarray(new_dir.reshape(-1, 3), dtype=float)
            m = np.ascontiguousarray(mask.reshape(-1), dtype=np.uint8)
            if m.any():
                self._native.bind_stream()
                self._native.call("swarm_engine_set_directors", nd.ctypes.data, m.ctypes.data)
                self._host_cache = None
            return
        old = self._host()["dir"]
        nd = np.ascontiguousarray(new_dir.reshape(-1, 3), dtype=float)
        dots = np.einsum("ij,ij->i", nd, old.reshape(-1, 3))
        with np.errstate(invalid="ignore"):
            ang = np.arccos(dots)
        m = np.ascontiguousarray(mask.reshape(-1) & (ang > 1e-6), dtype=np.uint8)
        if m.any():
            self._native.bind_stream()
            self._native.call("swarm_engine_set_directors", nd.ctypes.data, m.ctypes.data)
            self._host_cache = None

    def manage_forces(self, force_model=None) -> bool:
        """Collect actions from the force function and apply them (espresso.py:1203-1249)."""
        if force_model is None:
            return
        if self._device_capable(force_model):
            actions = force_model.calc_action(self.swarm_view())
            if not isinstance(actions, DeviceActions):
                raise TypeError("device-capable force model must return DeviceActions")
            self.apply_device_actions(actions)
            return
        if self.n_envs != 1:
            raise ValueError("n_envs > 1 requires a device-capable force model")
        h = self._host()
        swarmrl_colloids = [
            Colloid(
                pos=h["pos"][0, i].copy(),
                velocity=h["vel"][0, i].copy(),
                director=h["dir"][0, i].copy(),
                id=i,
                type=self._types_list[i],
            )
            for i in range(self.n_particles)
        ]
        actions = force_model.calc_action(swarmrl_colloids)
        N = self.n_particles
        f = np.zeros(N, dtype=np.float32)
        tz = np.zeros(N, dtype=np.float32)
        txy = np.zeros((2, N), dtype=np.float32)
        new_dir = np.zeros((1, N, 3))
        mask = np.zeros((1, N), dtype=bool)
        for i, action in enumerate(actions):
            f[i] = action.force
            if action.torque is not None:
                tq = np.asarray(action.torque, dtype=float)
                tz[i] = tq[2]
                txy[:, i] = tq[:2]
            if action.new_direction is not None:
                new_dir[0, i] = action.new_direction
                mask[0, i] = True
        self._native.bind_stream()
        self._native.call("swarm_engine_set_actions", f.ctypes.data, tz.ctypes.data, 0)
        if self.n_dims == 3:
            self._native.call("swarm_engine_set_torque_xy", txy.ctypes.data, 0)
        if mask.any():
            self._set_new_directions(new_dir, mask)

    # ---------------------------------------------------------- integrate
    def _prebuild(self, n_steps: int):
        """
        Fork the next window's position-only preparation (cluster build,
        noise table) onto a side stream so it overlaps the observable and
        policy kernels of manage_forces; _run joins it.  Positions cannot
        change in between (espresso.py:1253-1306), see swarm_engine_prebuild.
        """
        if self._ride_along:
            # the force model's vision-cone and policy launches carry the
            # three build stages along (swarm_engine_defer_build): no side
            # stream, fork or join in the slice
            self._native.bind_stream()
            deferred = ctypes.c_int32()
            self._native.call("swarm_engine_defer_build", ctypes.byref(deferred))
            if deferred.value:
                self._prebuild_pending = ("ride",)
                return
        main = torch.cuda.current_stream()
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(device=main.device)
        side = self._side_stream
        if self.n_envs * self.n_particles > 32768:
            # Throughput-bound engines: the observables outlast the build, and
            # in a captured graph the branch captured first after a fork keeps
            # the launch queue (the other pays the cross-queue latencies,
            # DESIGN.md section 6): fork here, launch the build in _run.
            fork = torch.cuda.Event()
            fork.record(main)
            self._prebuild_pending = (side, fork, int(n_steps))
            return
        side.wait_stream(main)
        self._native.call("swarm_engine_prebuild", ctypes.c_void_p(side.cuda_stream), int(n_steps))
        self._prebuild_pending = (side, None, 0)

    def _run(self, n_steps: int):
        if self._prebuild_pending is not None and self._prebuild_pending[0] == "ride":
            # stages no launch carried along run in swarm_engine_integrate
            self._prebuild_pending = None
            self._native.bind_stream()
            self._native.call("swarm_engine_prebuild_noise", None, int(n_steps))
        if self._prebuild_pending is not None:
            # The noise table (latency-bound engines) runs on the main stream
            # after the policy kernels, ahead of the join: the build usually
            # finishes later, and a third stream would add a graph join.
            side, fork, hint = self._prebuild_pending
            if fork is not None:  # deferred build (throughput-bound engines)
                side.wait_event(fork)
                self._native.call("swarm_engine_prebuild", ctypes.c_void_p(side.cuda_stream), hint)
            self._native.bind_stream()
            self._native.call("swarm_engine_prebuild_noise", None, int(n_steps))
            torch.cuda.current_stream().wait_stream(side)
            self._prebuild_pending = None
        self._native.bind_stream()
        self._native.call("swarm_engine_integrate", int(n_steps))
        self.system.time += n_steps * self._time_step
        self._steps_run += n_steps
        self._host_cache = None

    def integrate(self, n_slices, force_model=None):
        """The slice/write schedule of espresso.py:1251-1308."""
        if not self.integration_initialised:
            self.slice_idx = 0
            self.step_idx = 0
            self._setup_interactions()
            self._remove_overlap()
            self._init_h5_output()
            self.integration_initialised = True

        device_path = force_model is not None and self._device_capable(force_model)
        # ride-along builds (ride_along_build = False: fork onto a side stream)
        self._ride_along = bool(device_path and self.ride_along_build and
                                getattr(force_model, "absorbs_build", lambda: False)())
        old_slice_idx = self.slice_idx

        while self.step_idx < self.params.steps_per_slice * (old_slice_idx + n_slices):
            if self.step_idx == self.params.steps_per_write_interval * self.write_idx:
                self._update_traj_holder()
                self.write_idx += 1
                if len(self.traj_holder["Times"]) >= self.write_chunk_size:  # host path
                    self._write_traj_chunk_to_file()
                    for val in self.traj_holder.values():
                        val.clear()

            if force_model is not None:
                if force_model.kill_switch:
                    break

            if self.step_idx == self.params.steps_per_slice * self.slice_idx:
                self.slice_idx += 1
                if device_path and self.overlap_build and self._prebuild_pending is None:
                    self._prebuild(min(
                        self.params.steps_per_write_interval * self.write_idx - self.step_idx,
                        self.params.steps_per_slice * self.slice_idx - self.step_idx))
                self.manage_forces(force_model)

            steps_to_next_write = (
                self.params.steps_per_write_interval * self.write_idx - self.step_idx
            )
            steps_to_next_slice = self.params.steps_per_slice * self.slice_idx - self.step_idx
            steps_to_next = min(steps_to_next_write, steps_to_next_slice)

            self._run(steps_to_next)
            nxt = self.step_idx + steps_to_next
            if (device_path and self.overlap_build and self.early_fork
                    and nxt == self.params.steps_per_slice * self.slice_idx
                    and nxt < self.params.steps_per_slice * (old_slice_idx + n_slices)):
                # the next slice's cluster build depends on the positions
                # only: fork it now, so it overlaps this chunk's reward as
                # well as the next slice's observables and policy
                self._prebuild(self.params.steps_per_slice)
            if force_model is not None:
                force_model.calc_reward(self.swarm_view() if device_path else self.colloids)
            self.step_idx += steps_to_next

    def finalize(self):
        """Write the last trajectory chunk (espresso.py:1310-1318)."""
        if self.traj_holder is None:
            return
        self.drain_trajectory(block=True)
        self._write_traj_chunk_to_file()
        for val in self.traj_holder.values():
            val.clear()

    def get_particle_data(self):
        """espresso.py:1320-1336 (env 0; [E, N, ...] arrays when n_envs > 1)."""
        h = self._host()
        ids = np.arange(self.n_particles)
        types = np.asarray(self._types_list)
        if self.n_envs == 1:
            return {
                "Id": ids,
                "Type": types,
                "Unwrapped_Positions": h["pos"][0].copy(),
                "Velocities": h["vel"][0].copy(),
                "Directors": h["dir"][0].copy(),
            }
        return {
            "Id": np.broadcast_to(ids, (self.n_envs, self.n_particles)).copy(),
            "Type": np.broadcast_to(types, (self.n_envs, self.n_particles)).copy(),
            "Unwrapped_Positions": h["pos"].copy(),
            "Velocities": h["vel"].copy(),
            "Directors": h["dir"].copy(),
        }

    def get_unit_system(self):
        return self.ureg

    # ---------------------------------------------------- raw state (tests)
    def get_raw_state(self) -> dict:
        """Exact engine state: q/img uint32/int32 [3, E*N], ang uint32 [E*N]."""
        M = self.n_envs * self.n_particles
        q = np.zeros((3, M), dtype=np.uint32)
        img = np.zeros((3, M), dtype=np.int32)
        ang = np.zeros(M, dtype=np.uint32)
        self._native.bind_stream()
        self._native.call(
            "swarm_engine_download_raw", q.ctypes.data, img.ctypes.data, ang.ctypes.data
        )
        return {"q": q, "img": img, "ang": ang}

    def set_raw_state(self, q: np.ndarray, img: np.ndarray, ang: np.ndarray):
        q = np.ascontiguousarray(q, dtype=np.uint32)
        img = np.ascontiguousarray(img, dtype=np.int32)
        ang = np.ascontiguousarray(ang, dtype=np.uint32)
        self._native.bind_stream()
        self._native.call("swarm_engine_upload_raw", q.ctypes.data, img.ctypes.data, ang.ctypes.data)
        self._host_cache = None

    def window_stats(self) -> dict:
        """Per-env diagnostics of the last integration window (see C ABI)."""
        fb = np.zeros(self.n_envs, np.int32)
        w = np.zeros(self.n_envs, np.int32)
        self._native.bind_stream()
        self._native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
        return {"fallback": fb, "waves": w}

    def step_count(self) -> int:
        self._native.bind_stream()
        return int(self._native._lib.swarm_engine_step_count(self._native.ptr))


EspressoMD = SwarmEngine
