"""
Device-resident views of the engine state for the batched (GPU) path.

The reference hands every callback a Python list of ``Colloid`` objects built
from ESPResSo particle handles (swarmrl/engine/espresso.py:1214-1226).  That
contract is kept (``SwarmEngine.colloids`` / the list path), but when every
agent of a force model can consume device tensors, the engine passes a
``SwarmView`` instead: zero-copy torch views of the HIP engine's SoA arrays,
shaped [n_envs, n_particles].  Observables and tasks of this package accept
either form.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, Optional

import numpy as np
import torch

from swarmrl_amd import _capi

_TWO32 = 4294967296.0


class _CudaArray:
    """Minimal __cuda_array_interface__ exporter for a raw device pointer."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.__cuda_array_interface__ = {
            "shape": tuple(int(s) for s in shape),
            "typestr": typestr,
            "data": (int(ptr), False),
            "version": 2,
            "strides": None,
        }


def wrap_device_pointer(ptr: int, shape, dtype: torch.dtype, device) -> torch.Tensor:
    """Zero-copy torch tensor over memory owned by the HIP engine."""
    typestr = {
        torch.uint32: "<u4",
        torch.int32: "<i4",
        torch.float32: "<f4",
        torch.uint8: "|u1",
    }[dtype]
    if dtype == torch.uint32:
        # torch has limited uint32 support: view the words as int32
        t = torch.as_tensor(_CudaArray(ptr, shape, "<i4"), device=device)
        return t
    return torch.as_tensor(_CudaArray(ptr, shape, typestr), device=device)


@dataclasses.dataclass
class DeviceActions:
    """Actions for every particle of every env, as device tensors [E, N]."""

    f_swim: torch.Tensor
    torque_z: torch.Tensor
    new_direction: Optional[np.ndarray] = None  # host (3,) or (E, N, 3)
    new_direction_mask: Optional[np.ndarray] = None


class SwarmView:
    """
    Batched device view of one engine's state.

    Attributes are torch tensors on the engine's device:
      q      int32 [3, E, N]  (uint32 box fractions reinterpreted as int32)
      img    int32 [3, E, N]
      ang    int32 [E, N]     (uint32 turn fractions reinterpreted as int32)
      types  int32 [N]
    """

    def __init__(self, engine):
        self.engine = engine
        self.n_envs = engine.n_envs
        self.n_particles = engine.n_particles
        self.device = engine.device
        views = engine._device_views()
        E, N = self.n_envs, self.n_particles
        dev = self.device
        self.q = wrap_device_pointer(views.q, (3, E, N), torch.uint32, dev)
        self.img = wrap_device_pointer(views.img, (3, E, N), torch.int32, dev)
        self.ang = wrap_device_pointer(views.ang, (E, N), torch.uint32, dev)
        self.n_dims = int(engine.n_dims)
        self.dir3 = (wrap_device_pointer(views.dir3, (3, E, N), torch.float32, dev)
                     if self.n_dims == 3 else None)
        self.types = engine._types_device
        self.radii = engine._radii_device
        self.ids = np.arange(N)
        self._type_index: Dict[int, torch.Tensor] = engine._type_index_cache

    # ------------------------------------------------------------------
    def indices_of_type(self, p_type: int) -> torch.Tensor:
        """Sorted particle indices of one type (int32, device)."""
        idx = self._type_index.get(int(p_type))
        if idx is None:
            host = np.nonzero(self.engine._types_host == int(p_type))[0].astype(np.int32)
            idx = torch.as_tensor(host, device=self.device)
            self._type_index[int(p_type)] = idx
        return idx

    def covers_all(self, p_type: int) -> bool:
        """True when every particle has this type (indices == arange(N))."""
        return bool(np.all(self.engine._types_host == int(p_type)))

    def positions(self) -> torch.Tensor:
        """Unwrapped positions, float64 [E, N, 3]."""
        box = self.engine._box
        qf = (self.q.to(torch.int64) & 0xFFFFFFFF).to(torch.float64)
        pos = (self.img.to(torch.float64) + qf / _TWO32)
        pos = pos * torch.as_tensor(box, dtype=torch.float64, device=self.device).view(3, 1, 1)
        out = pos.permute(1, 2, 0).contiguous()
        if self.n_dims == 2:
            out[..., 2] = 0.0
        return out

    def directors(self) -> torch.Tensor:
        """Directors, float32 [E, N, 3] (2-D: torch sin/cos of the stored
        angle; 3-D: the stored unit vectors)."""
        if self.n_dims == 3:
            return self.dir3.permute(1, 2, 0).contiguous()
        a = (self.ang.to(torch.int64) & 0xFFFFFFFF).to(torch.float64) * (2.0 * math.pi / _TWO32)
        d = torch.stack([torch.cos(a), torch.sin(a), torch.zeros_like(a)], dim=-1)
        return d.to(torch.float32)

    def velocities(self) -> torch.Tensor:
        """BD velocities of the last sub-step, float32 [E, N, 3]."""
        v = self.engine._device_views()
        vel = wrap_device_pointer(v.vel, (3, self.n_envs, self.n_particles), torch.float32,
                                  self.device)
        return vel.permute(1, 2, 0).contiguous()

    def __len__(self):
        return self.n_particles


def is_view(obj) -> bool:
    return isinstance(obj, SwarmView)


__all__ = ["SwarmView", "DeviceActions", "is_view", "wrap_device_pointer", "_capi"]
