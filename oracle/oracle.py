"""
ctypes wrapper of the CPU oracle (oracle/swarm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker (or the timed CPU
comparator), never by the product package swarmrl_amd/.

The parameter struct is declared here independently of the product's binding
so that a layout slip in either shows up as a parity failure.
"""

from __future__ import annotations

import ctypes
import math
import pathlib
import subprocess

import numpy as np

_DIR = pathlib.Path(__file__).resolve().parent
_LIB_PATH = _DIR / "_build" / "liboracle.so"
MAX_SPECIES = 16
TWO32 = 4294967296.0


def build() -> pathlib.Path:
    # one make at a time (parallel test workers would otherwise rewrite the
    # library while another loads it)
    import fcntl

    with open(_DIR / ".build.lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", str(_DIR)], check=True)
    return _LIB_PATH


class Params(ctypes.Structure):
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
        ("radius", ctypes.c_double * MAX_SPECIES),
        ("gamma_t", ctypes.c_double * MAX_SPECIES),
        ("gamma_r", ctypes.c_double * MAX_SPECIES),
        ("mass", ctypes.c_double * MAX_SPECIES),
        ("rinertia", ctypes.c_double * MAX_SPECIES),
    ]


MAX_WALLS = 16


class Wall(ctypes.Structure):
    """swarm_wall_t (declared independently of the product binding)."""
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("normal", ctypes.c_double * 3),
        ("offset", ctypes.c_double),
        ("corner", ctypes.c_double * 3),
        ("a", ctypes.c_double * 3),
        ("b", ctypes.c_double * 3),
    ]


def make_walls(walls):
    """walls: list of dicts {'kind': 0, 'normal', 'offset'} or {'kind': 1,
    'corner', 'a', 'b'} -> (ctypes array, count)."""
    arr = (Wall * max(1, len(walls)))()
    for k, w in enumerate(walls):
        arr[k].kind = int(w["kind"])
        for key in ("normal", "corner", "a", "b"):
            if key in w:
                for a in range(3):
                    getattr(arr[k], key)[a] = float(w[key][a])
        arr[k].offset = float(w.get("offset", 0.0))
    return arr, len(walls)


_lib = None
_P = ctypes.c_void_p


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(_LIB_PATH))
        L.or_philox4x32_10.argtypes = [_P, _P, _P]
        L.or_logf.restype = ctypes.c_float
        L.or_logf.argtypes = [ctypes.c_float]
        L.or_acosf.restype = ctypes.c_float
        L.or_acosf.argtypes = [ctypes.c_float]
        L.or_sincos_turn.argtypes = [ctypes.c_uint32, _P, _P]
        L.or_signed_angle.restype = ctypes.c_float
        L.or_signed_angle.argtypes = [_P, _P]
        L.or_normal_from_word.restype = ctypes.c_float
        L.or_normal_from_word.argtypes = [ctypes.c_uint32]
        L.or_normals3.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint64, ctypes.c_uint32, _P]
        L.or_step_normals.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint64, _P]
        L.or_bd_run.restype = ctypes.c_int
        L.or_bd_run.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                _P, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, _P, _P,
                                ctypes.c_int]
        L.or_sd_run.restype = ctypes.c_int
        L.or_sd_run.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                _P, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                ctypes.c_int]
        L.or_vision_cone.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P, _P,
                                     ctypes.c_int, _P, _P, ctypes.c_float, ctypes.c_int, _P,
                                     ctypes.c_int, _P, _P]
        L.or_vision_cone_cells.restype = ctypes.c_int
        L.or_vision_cone_cells.argtypes = L.or_vision_cone.argtypes
        L.or_set_threads.argtypes = [ctypes.c_int]
        L.or_get_threads.restype = ctypes.c_int
        L.or_set_threads(1)  # the scalar restatement unless a caller asks for threads
        L.or_field_distance.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P,
                                        ctypes.c_int, _P, _P, _P, _P, _P, _P, ctypes.c_int]
        L.or_neighbor_pairs.restype = ctypes.c_int
        L.or_neighbor_pairs.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P,
                                        ctypes.c_double, _P, ctypes.c_int]
        L.or_cell_grid.argtypes = [ctypes.POINTER(Params), ctypes.c_int, ctypes.c_double, _P, _P]
        L.or_bd_run_walls.restype = ctypes.c_int
        L.or_bd_run_walls.argtypes = L.or_bd_run.argtypes + [_P, ctypes.c_int, _P, _P, _P, _P]
        L.or_sd_run_walls.restype = ctypes.c_int
        L.or_sd_run_walls.argtypes = L.or_sd_run.argtypes + [_P, ctypes.c_int]
        L.or_bd_run3.restype = ctypes.c_int
        L.or_bd_run3.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                 _P, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, _P, _P,
                                 _P, ctypes.c_int, _P, _P, _P, _P]
        L.or_sd_run3.restype = ctypes.c_int
        L.or_sd_run3.argtypes = [ctypes.POINTER(Params), ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                 _P, ctypes.c_int, ctypes.c_double, ctypes.c_double, _P,
                                 ctypes.c_int]
        L.or_rotate_director.argtypes = [_P, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data if a is not None else None


# ------------------------------------------------------------ parameters
def make_params(box, time_step, kT, wca_epsilon, seed, species, periodic=True, n_dims=2):
    """species: list of (radius, gamma_t, gamma_r, mass, rinertia)."""
    p = Params()
    p.n_dims = n_dims
    p.periodic = 1 if periodic else 0
    for a in range(3):
        p.box[a] = float(box[a])
    p.time_step = float(time_step)
    p.kT = float(kT)
    p.wca_epsilon = float(wca_epsilon)
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.n_species = len(species)
    for s, (r, gt, gr, m, rin) in enumerate(species):
        p.radius[s], p.gamma_t[s], p.gamma_r[s], p.mass[s], p.rinertia[s] = r, gt, gr, m, rin
    return p


def to_fixed(x, L):
    """fp64 position -> (uint32 box fraction, int32 image) (DESIGN.md spec)."""
    u = np.asarray(x, dtype=np.float64) / L
    fl = np.floor(u)
    qd = np.rint((u - fl) * TWO32)
    wrap = qd >= TWO32
    qd = np.where(wrap, qd - TWO32, qd)
    fl = np.where(wrap, fl + 1.0, fl)
    return qd.astype(np.uint64).astype(np.uint32), fl.astype(np.int32)


def angle_fixed(dx, dy):
    phi = np.arctan2(np.asarray(dy, dtype=float), np.asarray(dx, dtype=float))
    a = np.rint(phi / (2 * math.pi) * TWO32).astype(np.int64)
    return (a & 0xFFFFFFFF).astype(np.uint32)


def state_from_positions(pos, dirs, box):
    """pos/dirs (N, 3) fp64 -> {'q' [3,N] u32, 'img' [3,N] i32, 'ang' [N] u32}."""
    pos = np.asarray(pos, dtype=float)
    n = len(pos)
    q = np.zeros((3, n), np.uint32)
    img = np.zeros((3, n), np.int32)
    for a in range(2):
        q[a], img[a] = to_fixed(pos[:, a], box[a])
    ang = angle_fixed(np.asarray(dirs)[:, 0], np.asarray(dirs)[:, 1])
    return {"q": q, "img": img, "ang": ang}


def state3_from_positions(pos, dirs, box):
    """3-D: pos/dirs (N, 3) fp64 -> {'q' [3,N] u32, 'img' [3,N] i32,
    'dir' [3,N] f32 (normalised), 'ang' [N] u32 (unused, 0)}."""
    pos = np.asarray(pos, dtype=float)
    n = len(pos)
    q = np.zeros((3, n), np.uint32)
    img = np.zeros((3, n), np.int32)
    for a in range(3):
        q[a], img[a] = to_fixed(pos[:, a], box[a])
    d = np.asarray(dirs, dtype=float)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).T.astype(np.float32)
    return {"q": q, "img": img, "dir": np.ascontiguousarray(d), "ang": np.zeros(n, np.uint32)}


def unwrapped(state, box, dims=None):
    q, img = state["q"], state["img"]
    out = np.zeros((q.shape[1], 3))
    if dims is None:
        dims = 3 if "dir" in state else 2
    for a in range(dims):
        out[:, a] = (img[a].astype(np.float64) + q[a].astype(np.float64) / TWO32) * box[a]
    return out


def _copy_state(state):
    out = {
        "q": np.ascontiguousarray(state["q"], dtype=np.uint32).copy(),
        "img": np.ascontiguousarray(state["img"], dtype=np.int32).copy(),
        "ang": np.ascontiguousarray(state["ang"], dtype=np.uint32).copy(),
    }
    if "dir" in state:
        out["dir"] = np.ascontiguousarray(state["dir"], dtype=np.float32).copy()
    return out


# ------------------------------------------------------------- dynamics
def bd_run(params, state, species, f_swim, torque_z, n_steps, step0=0, env=0, f_ext=None,
           use_cells=True, walls=None, violations=None, prev=None):
    """n_steps BD sub-steps of one env; returns (new_state, vel [3,N], omega [N]).
    walls: list of wall dicts (make_walls); violations: 1-element uint64
    array that receives the added count of wall contacts.  prev: None, or
    reuse_forces (espresso.py:1304-1306) -- {"f": f_swim, "t": torque_z,
    "ang": orientation} of the previous run's last force calculation, used by
    sub-step 0 (see ReuseForces)."""
    st = _copy_state(state)
    n = st["ang"].shape[0]
    sp = np.ascontiguousarray(species, dtype=np.uint8)
    fs = np.ascontiguousarray(f_swim, dtype=np.float32)
    tz = np.ascontiguousarray(torque_z, dtype=np.float32)
    fe = None if f_ext is None else np.ascontiguousarray(f_ext, dtype=np.float32)
    vel = np.zeros((3, n), np.float32)
    om = np.zeros(n, np.float32)
    wa, nw = make_walls(walls or [])
    viol = np.zeros(1, np.uint64) if violations is None else violations
    f0 = t0 = a0 = None
    if prev is not None:
        f0 = np.ascontiguousarray(prev["f"], dtype=np.float32)
        t0 = np.ascontiguousarray(prev["t"], dtype=np.float32)
        a0 = np.ascontiguousarray(prev["ang"], dtype=np.uint32)
    rc = lib().or_bd_run_walls(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]),
                               _ptr(st["ang"]), _ptr(sp), _ptr(fs), _ptr(tz), _ptr(fe),
                               int(step0), int(n_steps), int(env), _ptr(vel), _ptr(om),
                               1 if use_cells else 0, ctypes.cast(wa, _P), nw, _ptr(viol),
                               _ptr(f0), _ptr(t0), _ptr(a0))
    if rc != 0:
        raise ValueError(f"or_bd_run failed ({rc})")
    return st, vel, om


def bd_run3(params, state, species, f_swim, torque, n_steps, step0=0, env=0, f_ext=None,
            walls=None, violations=None, prev=None):
    """3-D: n_steps BD sub-steps of one env (state with 'dir' [3,N]); torque
    [3,N] lab frame.  Returns (new_state, vel [3,N], omega [3,N]).  prev:
    reuse_forces, {"f", "t" [3,N], "dir" [3,N]} (see bd_run)."""
    st = _copy_state(state)
    n = st["q"].shape[1]
    sp = np.ascontiguousarray(species, dtype=np.uint8)
    fs = np.ascontiguousarray(f_swim, dtype=np.float32)
    tq = np.ascontiguousarray(torque, dtype=np.float32).reshape(3, n)
    fe = None if f_ext is None else np.ascontiguousarray(f_ext, dtype=np.float32)
    vel = np.zeros((3, n), np.float32)
    om = np.zeros((3, n), np.float32)
    wa, nw = make_walls(walls or [])
    viol = np.zeros(1, np.uint64) if violations is None else violations
    f0 = t0 = d0 = None
    if prev is not None:
        f0 = np.ascontiguousarray(prev["f"], dtype=np.float32)
        t0 = np.ascontiguousarray(prev["t"], dtype=np.float32).reshape(3, n)
        d0 = np.ascontiguousarray(prev["dir"], dtype=np.float32).reshape(3, n)
    rc = lib().or_bd_run3(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]),
                          _ptr(st["dir"]), _ptr(sp), _ptr(fs), _ptr(tq), _ptr(fe), int(step0),
                          int(n_steps), int(env), _ptr(vel), _ptr(om), ctypes.cast(wa, _P), nw,
                          _ptr(viol), _ptr(f0), _ptr(t0), _ptr(d0))
    if rc != 0:
        raise ValueError(f"or_bd_run3 failed ({rc})")
    return st, vel, om


def sd_run3(params, state, species, n_steps, gamma=0.1, max_disp=0.1, f_swim=None,
            torque=None, f_ext=None, walls=None):
    st = _copy_state(state)
    n = st["q"].shape[1]
    sp = np.ascontiguousarray(species, dtype=np.uint8)
    fs = np.zeros(n, np.float32) if f_swim is None else np.ascontiguousarray(f_swim, np.float32)
    tq = np.zeros((3, n), np.float32) if torque is None else \
        np.ascontiguousarray(torque, np.float32).reshape(3, n)
    fe = None if f_ext is None else np.ascontiguousarray(f_ext, dtype=np.float32)
    wa, nw = make_walls(walls or [])
    steps = lib().or_sd_run3(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]),
                             _ptr(st["dir"]), _ptr(sp), _ptr(fs), _ptr(tq), _ptr(fe),
                             int(n_steps), float(gamma), float(max_disp), ctypes.cast(wa, _P), nw)
    return st, steps


class ReuseForces:
    """Oracle-side bookkeeping of reuse_forces for a sequence of runs of one
    env (the engine's f_prev / tz_prev / ang_prev): starts from zero actions
    (nothing swims before the first manage_forces, espresso.py:1228-1235) and
    the initial orientation; run() integrates and remembers what the next
    run's sub-step 0 reuses."""

    def __init__(self, state, dims=2):
        n = state["q"].shape[1]
        self.dims = dims
        if dims == 3:
            self.prev = {"f": np.zeros(n, np.float32), "t": np.zeros((3, n), np.float32),
                         "dir": np.asarray(state["dir"], np.float32).copy()}
        else:
            self.prev = {"f": np.zeros(n, np.float32), "t": np.zeros(n, np.float32),
                         "ang": np.asarray(state["ang"], np.uint32).copy()}

    def run(self, params, state, species, f_swim, torque, n_steps, **kw):
        fn = bd_run3 if self.dims == 3 else bd_run
        st, vel, om = fn(params, state, species, f_swim, torque, n_steps, prev=self.prev, **kw)
        key = "dir" if self.dims == 3 else "ang"
        self.prev = {"f": np.asarray(f_swim, np.float32).copy(),
                     "t": np.asarray(torque, np.float32).copy(), key: st[key].copy()}
        return st, vel, om


def rotate_director(v, phi):
    out = np.ascontiguousarray(v, dtype=np.float32).copy()
    lib().or_rotate_director(_ptr(out), float(phi[0]), float(phi[1]), float(phi[2]))
    return out


def sd_run(params, state, species, n_steps, gamma=0.1, max_disp=0.1, f_swim=None,
           torque_z=None, f_ext=None, use_cells=True, walls=None):
    st = _copy_state(state)
    n = st["ang"].shape[0]
    sp = np.ascontiguousarray(species, dtype=np.uint8)
    fs = np.zeros(n, np.float32) if f_swim is None else np.ascontiguousarray(f_swim, np.float32)
    tz = np.zeros(n, np.float32) if torque_z is None else np.ascontiguousarray(torque_z, np.float32)
    fe = None if f_ext is None else np.ascontiguousarray(f_ext, dtype=np.float32)
    wa, nw = make_walls(walls or [])
    steps = lib().or_sd_run_walls(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]),
                                  _ptr(st["ang"]), _ptr(sp), _ptr(fs), _ptr(tz), _ptr(fe),
                                  int(n_steps), float(gamma), float(max_disp),
                                  1 if use_cells else 0, ctypes.cast(wa, _P), nw)
    return st, steps


# ---------------------------------------------------------- observables
def vision_rims(half_angle, n_cones):
    a = np.float32(half_angle)
    k = np.arange(n_cones + 1, dtype=np.float32)
    return (-a + ((k * a) * np.float32(2)) / np.float32(n_cones)).astype(np.float32)


def set_threads(n):
    """OpenMP threads of the oracle's per-particle / per-agent loops (the
    results do not depend on it)."""
    lib().or_set_threads(int(n))


def vision_cone(params, state, agents, radii, types, vision_range, half_angle, n_cones,
                detected_types, cells=False):
    """cells=False: the reference's all-pairs loop; True: over a cell list
    (same bits; needs 2 vision_range < box)."""
    n = state["ang"].shape[0]
    ag = np.ascontiguousarray(agents, dtype=np.int32)
    rad = np.ascontiguousarray(radii, dtype=np.float32)
    ty = np.ascontiguousarray(types, dtype=np.int32)
    det = np.ascontiguousarray(detected_types, dtype=np.int32)
    rims = vision_rims(half_angle, n_cones)
    out = np.zeros((len(ag), n_cones, len(det)), np.float32)
    st = _copy_state(state)
    fn = lib().or_vision_cone_cells if cells else lib().or_vision_cone
    rc = fn(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]), _ptr(st["ang"]), _ptr(ag),
            len(ag), _ptr(rad), _ptr(ty), float(vision_range), int(n_cones), _ptr(rims), len(det),
            _ptr(det), _ptr(out))
    if cells and rc:
        raise ValueError("or_vision_cone_cells needs a periodic box wider than 2 vision_range")
    return out


def field_distance(params, state, agents, source, box_scale, hist, update=True):
    """hist: {'q': [3,A] u32, 'img': [3,A] i32} (updated in place if update)."""
    n = state["ang"].shape[0]
    ag = np.ascontiguousarray(agents, dtype=np.int32)
    st = _copy_state(state)
    src = np.ascontiguousarray(source, dtype=np.float64)
    bs = np.ascontiguousarray(box_scale, dtype=np.float64)
    d_cur = np.zeros(len(ag), np.float32)
    d_prev = np.zeros(len(ag), np.float32)
    lib().or_field_distance(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]), _ptr(ag),
                            len(ag), _ptr(src), _ptr(bs), _ptr(hist["q"]), _ptr(hist["img"]),
                            _ptr(d_cur), _ptr(d_prev), 1 if update else 0)
    return d_cur, d_prev


def history_from_state(state, agents):
    ag = np.asarray(agents)
    return {
        "q": np.ascontiguousarray(state["q"][:, ag], dtype=np.uint32),
        "img": np.ascontiguousarray(state["img"][:, ag], dtype=np.int32),
    }


def neighbor_pairs(params, state, cutoff, max_pairs=1 << 20):
    n = state["ang"].shape[0]
    st = _copy_state(state)
    pairs = np.zeros((max_pairs, 2), np.int32)
    k = lib().or_neighbor_pairs(ctypes.byref(params), n, _ptr(st["q"]), _ptr(st["img"]),
                                float(cutoff), _ptr(pairs), max_pairs)
    if k > max_pairs:
        raise ValueError("too many pairs")
    return pairs[:k].copy()


# ------------------------------------------------------------ primitives
def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return list(o)


def step_normals(seed, env, pid, t):
    """Sub-step t's three translation/rotation normals (swarm_oracle.c
    or_step_normals: four-word Philox groups of four sub-steps)."""
    out = np.zeros(3, np.float32)
    lib().or_step_normals(int(seed), int(env), int(pid), int(t), _ptr(out))
    return out


def normal_from_word(r):
    """The standard normal of one 32-bit Philox word (or_normal_from_word)."""
    return lib().or_normal_from_word(int(r) & 0xFFFFFFFF)


def normals3(seed, env, pid, step, tag):
    """Three standard normals of one Philox block (swarm_oracle.c or_normals3)."""
    out = np.zeros(3, np.float32)
    lib().or_normals3(int(seed), int(env), int(pid), int(step), int(tag), _ptr(out))
    return out


def sincos_turn(a):
    s = ctypes.c_float()
    c = ctypes.c_float()
    lib().or_sincos_turn(int(a) & 0xFFFFFFFF, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def logf(x):
    return lib().or_logf(float(x))


def acosf(x):
    return lib().or_acosf(float(x))


def signed_angle(my, other):
    m = np.ascontiguousarray(my, dtype=np.float32)
    o = np.ascontiguousarray(other, dtype=np.float32)
    return lib().or_signed_angle(_ptr(m), _ptr(o))


def cell_grid(params, n, cutoff):
    lx = ctypes.c_int()
    ly = ctypes.c_int()
    lib().or_cell_grid(ctypes.byref(params), int(n), float(cutoff), ctypes.byref(lx),
                       ctypes.byref(ly))
    return lx.value, ly.value
