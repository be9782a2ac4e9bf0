"""Shared helpers for the GPU parity tests: drive the C ABI and the oracle
from the same raw numbers."""

import ctypes

import numpy as np
import torch

from oracle import oracle
from swarmrl_amd import _capi
from swarmrl_amd.engine.swarm_engine import _NativeEngine


def species_list(kT_scale=1.0):
    # (radius, gamma_t, gamma_r, mass, rinertia) in simulation units
    return [(1.0, 4.6595, 6.2126, 1.0358e-6, 4.143e-7), (0.7, 3.2617, 2.1309, 3.55e-7, 7.0e-8)]


def capi_params(box, dt, kT, eps, seed, species, n_dims=2, reuse=False, periodic=True):
    p = _capi.SwarmParams()
    p.n_dims = n_dims
    p.periodic = 1 if periodic else 0
    p.reuse_forces = 1 if reuse else 0
    for a in range(3):
        p.box[a] = float(box[a])
    p.time_step = dt
    p.kT = kT
    p.wca_epsilon = eps
    p.seed = seed
    p.n_species = len(species)
    for s, (r, gt, gr, m, rin) in enumerate(species):
        p.radius[s], p.gamma_t[s], p.gamma_r[s], p.mass[s], p.rinertia[s] = r, gt, gr, m, rin
    return p


class Harness:
    def __init__(self, box, dt, kT, eps, seed, species, sp_of, n_envs=1, n_dims=2,
                 reuse=False, periodic=True):
        self.box = box
        self.n = len(sp_of)
        self.E = n_envs
        self.dims = n_dims
        self.sp = np.asarray(sp_of, dtype=np.int32)
        self.cp = capi_params(box, dt, kT, eps, seed, species, n_dims, reuse, periodic)
        self.op = oracle.make_params(box, dt, kT, eps, seed, species, periodic=periodic,
                                     n_dims=n_dims)
        self.native = _NativeEngine(self.cp, n_envs, self.sp)

    def upload(self, states):
        """states: list (per env) of oracle state dicts."""
        q = np.concatenate([s["q"] for s in states], axis=1)
        img = np.concatenate([s["img"] for s in states], axis=1)
        ang = np.concatenate([s["ang"] for s in states])
        q = np.ascontiguousarray(q, np.uint32)
        img = np.ascontiguousarray(img, np.int32)
        ang = np.ascontiguousarray(ang, np.uint32)
        self.native.bind_stream()
        self.native.call("swarm_engine_upload_raw", q.ctypes.data, img.ctypes.data, ang.ctypes.data)
        if self.dims == 3:
            d = np.ascontiguousarray(np.concatenate([s["dir"] for s in states], axis=1),
                                     np.float32)
            self.native.call("swarm_engine_upload_directors", d.ctypes.data)

    def set_torque_xy(self, txy):
        t = np.ascontiguousarray(txy, np.float32).reshape(2, -1)
        self.native.bind_stream()
        self.native.call("swarm_engine_set_torque_xy", t.ctypes.data, 0)

    def set_walls(self, walls):
        arr = (_capi.SwarmWall * max(1, len(walls)))()
        for k, w in enumerate(walls):
            arr[k].kind = int(w["kind"])
            for key in ("normal", "corner", "a", "b"):
                if key in w:
                    for a in range(3):
                        getattr(arr[k], key)[a] = float(w[key][a])
            arr[k].offset = float(w.get("offset", 0.0))
        self.native.bind_stream()
        self.native.call("swarm_engine_set_walls", ctypes.cast(arr, ctypes.c_void_p), len(walls))

    def wall_violations(self):
        v = np.zeros(1, np.uint64)
        self.native.call("swarm_engine_wall_violations", v.ctypes.data)
        return int(v[0])

    def download(self):
        M = self.E * self.n
        q = np.zeros((3, M), np.uint32)
        img = np.zeros((3, M), np.int32)
        ang = np.zeros(M, np.uint32)
        self.native.bind_stream()
        self.native.call("swarm_engine_download_raw", q.ctypes.data, img.ctypes.data, ang.ctypes.data)
        out = [
            {"q": q[:, e * self.n:(e + 1) * self.n].copy(),
             "img": img[:, e * self.n:(e + 1) * self.n].copy(),
             "ang": ang[e * self.n:(e + 1) * self.n].copy()}
            for e in range(self.E)
        ]
        if self.dims == 3:
            d = np.zeros((3, M), np.float32)
            self.native.call("swarm_engine_download_directors", d.ctypes.data)
            for e in range(self.E):
                out[e]["dir"] = d[:, e * self.n:(e + 1) * self.n].copy()
        return out

    def set_actions(self, f, t):
        f = np.ascontiguousarray(f, np.float32).reshape(-1)
        t = np.ascontiguousarray(t, np.float32).reshape(-1)
        self.native.bind_stream()
        self.native.call("swarm_engine_set_actions", f.ctypes.data, t.ctypes.data, 0)

    def integrate(self, n):
        self.native.bind_stream()
        self.native.call("swarm_engine_integrate", int(n))

    def prebuild(self, n_hint, stream=None, noise_stream=None):
        """swarm_engine_prebuild on `stream` and swarm_engine_prebuild_noise on
        `noise_stream` (torch streams; default: both on the current stream)."""
        import torch

        st = stream if stream is not None else torch.cuda.current_stream()
        ns = noise_stream if noise_stream is not None else st
        self.native.call("swarm_engine_prebuild", ctypes.c_void_p(st.cuda_stream), int(n_hint))
        self.native.call("swarm_engine_prebuild_noise", ctypes.c_void_p(ns.cuda_stream),
                         int(n_hint))

    def sd(self, n, gamma=0.1, maxd=0.1):
        self.native.bind_stream()
        self.native.call("swarm_engine_remove_overlap", int(n), float(gamma), float(maxd))

    def velocities(self):
        v = _capi.SwarmDeviceViews()
        _capi.check(self.native._lib.swarm_engine_device_views(self.native.ptr, ctypes.byref(v)))
        M = self.E * self.n
        torch.cuda.synchronize()
        from swarmrl_amd.engine.swarm_view import wrap_device_pointer

        vel = wrap_device_pointer(v.vel, (3, M), torch.float32, torch.device("cuda", 0))
        return vel.cpu().numpy().copy()

    def omegas3(self):
        """3-D angular velocities [3, M] (x, y from omega_xy, z from omega_z)."""
        v = _capi.SwarmDeviceViews()
        _capi.check(self.native._lib.swarm_engine_device_views(self.native.ptr, ctypes.byref(v)))
        M = self.E * self.n
        torch.cuda.synchronize()
        from swarmrl_amd.engine.swarm_view import wrap_device_pointer

        dev = torch.device("cuda", 0)
        xy = wrap_device_pointer(v.omega_xy, (2, M), torch.float32, dev).cpu().numpy()
        z = wrap_device_pointer(v.omega_z, (M,), torch.float32, dev).cpu().numpy()
        return np.concatenate([xy, z[None]], 0)


def random_state3(rng, n, box, lo=0.0, hi=None):
    hi = box[0] if hi is None else hi
    pos = lo + rng.random((n, 3)) * (hi - lo)
    d = rng.normal(size=(n, 3))
    return oracle.state3_from_positions(pos, d, box)


def random_state(rng, n, box, lo=0.0, hi=None, min_sep=None):
    hi = box[0] if hi is None else hi
    pos = np.zeros((n, 3))
    pos[:, :2] = lo + rng.random((n, 2)) * (hi - lo)
    ang = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(ang), np.sin(ang), np.zeros(n)], 1)
    return oracle.state_from_positions(pos, dirs, box)
