"""
ctypes binding of the C ABI in include/swarmrl_amd.h.

The shared library ``libswarmrl_amd.so`` is built in-tree by
``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).  There is no CPU
fallback: if the library is missing or no HIP device is present, every engine
operation raises.  ``torch`` is imported before the library is loaded so both
use the single HIP runtime that torch brings into the process.
"""

from __future__ import annotations

import ctypes
import os
import pathlib

import torch  # noqa: F401  (load torch's HIP runtime first)

SWARM_MAX_SPECIES = 16
SWARM_MAX_CONES = 16
SWARM_MAX_DETECTED_TYPES = 8

SWARM_OK = 0
SWARM_EINVAL = 1
SWARM_ESTATE = 2
SWARM_EDEVICE = 3
SWARM_ECAPACITY = 4

# SWARMRL_AMD_LIB selects another build of the same library (e.g. the
# profiling variants tools/build_variants.sh makes); default: in-tree build.
_LIB_PATH = pathlib.Path(os.environ.get(
    "SWARMRL_AMD_LIB", pathlib.Path(__file__).resolve().parent / "libswarmrl_amd.so"))


class SwarmParams(ctypes.Structure):
    _fields_ = [
        ("n_dims", ctypes.c_int32),
        ("periodic", ctypes.c_int32),
        ("box", ctypes.c_double * 3),
        ("time_step", ctypes.c_double),
        ("kT", ctypes.c_double),
        ("wca_epsilon", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("n_species", ctypes.c_int32),
        ("reuse_forces", ctypes.c_int32),
        ("radius", ctypes.c_double * SWARM_MAX_SPECIES),
        ("gamma_t", ctypes.c_double * SWARM_MAX_SPECIES),
        ("gamma_r", ctypes.c_double * SWARM_MAX_SPECIES),
        ("mass", ctypes.c_double * SWARM_MAX_SPECIES),
        ("rinertia", ctypes.c_double * SWARM_MAX_SPECIES),
    ]


class SwarmDeviceViews(ctypes.Structure):
    _fields_ = [
        ("q", ctypes.c_void_p),
        ("img", ctypes.c_void_p),
        ("ang", ctypes.c_void_p),
        ("f_swim", ctypes.c_void_p),
        ("torque_z", ctypes.c_void_p),
        ("f_ext", ctypes.c_void_p),
        ("vel", ctypes.c_void_p),
        ("omega_z", ctypes.c_void_p),
        ("species", ctypes.c_void_p),
        ("n_envs", ctypes.c_int32),
        ("n_particles", ctypes.c_int32),
        ("n_dims", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("dir3", ctypes.c_void_p),
        ("torque_xy", ctypes.c_void_p),
        ("omega_xy", ctypes.c_void_p),
    ]


SWARM_MAX_WALLS = 16


class SwarmWall(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("normal", ctypes.c_double * 3),
        ("offset", ctypes.c_double),
        ("corner", ctypes.c_double * 3),
        ("a", ctypes.c_double * 3),
        ("b", ctypes.c_double * 3),
    ]


class SwarmVisionParams(ctypes.Structure):
    _fields_ = [
        ("vision_range", ctypes.c_float),
        ("vision_half_angle", ctypes.c_float),
        ("n_cones", ctypes.c_int32),
        ("n_types", ctypes.c_int32),
        ("detected_types", ctypes.c_int32 * SWARM_MAX_DETECTED_TYPES),
        ("rims", ctypes.c_float * (SWARM_MAX_CONES + 1)),
    ]


class SwarmAdam(ctypes.Structure):
    """swarm_adam_t: torch Adam's hyper-parameters and the device tensors
    of the six PPO layers (w1 | b1 | wa | ba | wc | bc)."""
    _fields_ = [
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("param", ctypes.c_void_p * 6),
        ("exp_avg", ctypes.c_void_p * 6),
        ("exp_avg_sq", ctypes.c_void_p * 6),
        ("step", ctypes.c_void_p * 6),
    ]


# name -> (restype, argtypes)
_P = ctypes.c_void_p
_SIGNATURES = {
    "swarm_last_error": (ctypes.c_char_p, []),
    "swarm_build_id": (ctypes.c_char_p, []),
    "swarm_engine_create": (
        ctypes.c_int,
        [ctypes.POINTER(SwarmParams), ctypes.c_int32, ctypes.c_int32, _P, ctypes.POINTER(_P)],
    ),
    "swarm_engine_destroy": (None, [_P]),
    "swarm_engine_set_stream": (ctypes.c_int, [_P, _P]),
    "swarm_engine_upload_state": (ctypes.c_int, [_P, _P, _P]),
    "swarm_engine_upload_raw": (ctypes.c_int, [_P, _P, _P, _P]),
    "swarm_engine_download_raw": (ctypes.c_int, [_P, _P, _P, _P]),
    "swarm_engine_download_state": (ctypes.c_int, [_P, _P, _P, _P]),
    "swarm_engine_set_actions": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32]),
    "swarm_engine_set_external_force": (ctypes.c_int, [_P, _P]),
    "swarm_engine_set_directors": (ctypes.c_int, [_P, _P, _P]),
    "swarm_engine_remove_overlap": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_double, ctypes.c_double],
    ),
    "swarm_engine_integrate": (ctypes.c_int, [_P, ctypes.c_int32]),
    "swarm_engine_prebuild": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_engine_prebuild_noise": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_engine_profile": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P]),
    "swarm_engine_profile_graph": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, ctypes.c_int32,
                                                  _P]),
    "swarm_engine_profile_stamps": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, ctypes.c_int32,
                                                   _P]),
    "swarm_engine_profile_roles": (ctypes.c_int, [_P, _P, ctypes.c_int32, _P]),
    "swarm_engine_time_run": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P]),
    "swarm_engine_debug_phases": (ctypes.c_int, [_P, _P]),
    "swarm_engine_debug_wave_stamps": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_pair_distances": (
        ctypes.c_int,
        [_P, _P, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_int32,
         ctypes.POINTER(ctypes.c_double), _P],
    ),
    "swarm_sample_actions": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, _P, ctypes.c_int32,
         ctypes.c_float, _P, _P, _P, _P, _P, _P, _P],
    ),
    "swarm_policy_mlp_sample": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P, ctypes.c_int32,
         ctypes.c_uint64, _P, ctypes.c_int32, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "swarm_engine_policy_mlp_sample": (
        ctypes.c_int,
        [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P, ctypes.c_int32,
         ctypes.c_uint64, _P, ctypes.c_int32, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "swarm_engine_defer_build": (ctypes.c_int, [_P, _P]),
    "swarm_ppo_workspace_bytes": (
        ctypes.c_int64,
        [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32],
    ),
    "swarm_ppo_epoch_grad": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _P, ctypes.c_int32,
         _P, _P, ctypes.c_int32, _P, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float,
         ctypes.c_float, _P, ctypes.c_int64, _P, _P],
    ),
    "swarm_ppo_epoch_step": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, ctypes.c_int32,
         ctypes.c_int32, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
         ctypes.POINTER(SwarmAdam), _P, ctypes.c_int64, _P, _P],
    ),
    "swarm_ppo_profile": (ctypes.c_int, [ctypes.c_int32, _P, _P]),
    "swarm_engine_step_count": (ctypes.c_int64, [_P]),
    "swarm_rnd_distance": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P],
    ),
    "swarm_rnd_env_reward": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P,
         ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P,
         ctypes.c_int64, _P],
    ),
    "swarm_rnd_env_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "swarm_engine_traj_ring": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "swarm_engine_traj_record": (ctypes.c_int, [_P]),
    "swarm_traj_entry_to_host": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "swarm_engine_window_stats": (ctypes.c_int, [_P, _P, _P]),
    "swarm_engine_device_views": (ctypes.c_int, [_P, ctypes.POINTER(SwarmDeviceViews)]),
    "swarm_vision_cone": (
        ctypes.c_int,
        [_P, ctypes.POINTER(SwarmVisionParams), _P, ctypes.c_int32, _P, _P, _P],
    ),
    "swarm_vision_cone_persistent": (
        ctypes.c_int,
        [_P, ctypes.POINTER(SwarmVisionParams), _P, ctypes.c_int32, _P, _P, _P],
    ),
    "swarm_engine_build_stats": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_engine_vision_policy": (
        ctypes.c_int,
        [_P, ctypes.POINTER(SwarmVisionParams), _P, ctypes.c_int32, _P, _P, _P, _P, _P,
         ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_uint64, _P, ctypes.c_int32,
         ctypes.c_float, _P, _P, _P, _P, _P, _P, _P],
    ),
    "swarm_field_distance": (
        ctypes.c_int,
        [_P, _P, ctypes.c_int32, _P, _P, _P, _P, _P, _P, ctypes.c_int32, ctypes.c_int32],
    ),
    "swarm_field_transform": (
        ctypes.c_int,
        [_P, _P, ctypes.c_int32, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float,
         ctypes.c_float, ctypes.c_int32, _P],
    ),
    "swarm_engine_set_torque_xy": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_engine_upload_directors": (ctypes.c_int, [_P, _P]),
    "swarm_engine_download_directors": (ctypes.c_int, [_P, _P]),
    "swarm_engine_set_walls": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "swarm_engine_wall_violations": (ctypes.c_int, [_P, _P]),
    "swarm_neighbor_reduce": (
        ctypes.c_int,
        [_P, _P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int32, ctypes.c_uint32,
         ctypes.c_double, ctypes.c_double, _P, _P],
    ),
    "swarm_engine_neighbor_pairs": (
        ctypes.c_int,
        [_P, ctypes.c_int32, ctypes.c_double, _P, ctypes.c_int32, _P],
    ),
}

_lib = None


def library_path() -> pathlib.Path:
    return _LIB_PATH


def source_hash(root: pathlib.Path = None) -> str:
    """12-hex-digit hash of the HIP sources (swarmrl_amd/csrc/*) and the
    C-ABI header the library is built from: compiled into the library
    (swarm_build_id) and carried by the profiles' rows (bench.py)."""
    import hashlib

    root = pathlib.Path(root) if root is not None else pathlib.Path(__file__).resolve().parents[1]
    h = hashlib.sha256()
    files = sorted([*(root / "swarmrl_amd" / "csrc").glob("*"), *(root / "include").glob("*.h")],
                   key=os.fspath)
    for path in files:
        h.update(path.name.encode())
        h.update(path.read_bytes())
    return h.hexdigest()[:12]


def build_id() -> str:
    """The source hash the loaded library was compiled from."""
    return lib().swarm_build_id().decode()


def lib() -> ctypes.CDLL:
    """Load the HIP engine library (raises if it was not built).  Warns when
    the library was built from other sources than the checkout's."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise RuntimeError(
            f"HIP engine library not found at {_LIB_PATH}; run "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)."
        )
    handle = ctypes.CDLL(os.fspath(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGNATURES.items():
        if name == "swarm_build_id" and not hasattr(handle, name):
            continue  # a library from before round 6 (A/B variants): no provenance
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    try:
        built, here = handle.swarm_build_id().decode(), source_hash()
    except (OSError, AttributeError):  # no sources beside the library / an old library
        built, here = None, None
    if built is not None and built != here:
        import warnings

        warnings.warn(f"{_LIB_PATH} was built from sources {built}, the checkout has {here}: "
                      "rebuild (__graft_entry__.build())", RuntimeWarning, stacklevel=2)
    return _lib


def exported_symbols():
    """Names of every entry point declared in include/swarmrl_amd.h."""
    return list(_SIGNATURES)


def check(rc: int) -> None:
    """Map a C-ABI status onto the exception the reference would raise."""
    if rc == SWARM_OK:
        return
    msg = lib().swarm_last_error().decode(errors="replace")
    if rc in (SWARM_EINVAL, SWARM_ECAPACITY):
        raise ValueError(msg)
    raise RuntimeError(msg)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "swarmrl_amd needs a HIP device (MI355X); no GPU is visible and "
            "there is no CPU fallback."
        )
