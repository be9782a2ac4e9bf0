"""
Pairwise field sums for ParticleSensing and SpeciesSearch (reference:
swarmrl/observables/particle_sensing.py:95-121,
swarmrl/tasks/searching/species_search.py:97-130).

Per agent i, over the sensed colloids j (type == sensing_type, colloid order):
    d_j   = || (x_j - x_i) / L ||                      (fp32, unwrapped)
    field = sum(decay(d[nonzero(d, size=M - 1)]))
The reference's ``jnp.nonzero(..., size=M - 1)`` keeps the FIRST M - 1
non-zero distances and pads with index 0 when there are fewer; that is
reproduced exactly:
    field = S_nz - [n_nz == M] decay(d_{M-1}) + max(0, M - 1 - n_nz) decay(d_0).
The O(A M) distances come from the HIP kernel ``swarm_pair_distances`` in
column tiles; the user's decay callable runs on each device tile (write it
with arithmetic operators / torch functions, as the reference's are jnp).
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from swarmrl_amd import _capi

_TILE_BYTES = 64 << 20


def pair_field(native, n_envs: int, agents: torch.Tensor, sensed: torch.Tensor, box_scale,
               decay_fn) -> torch.Tensor:
    """Field values [E, A] (fp32, device) for the agents of every env."""
    dev = agents.device
    A = int(agents.numel())
    Ms = int(sensed.numel())
    E = int(n_envs)
    if A == 0 or Ms == 0:
        return torch.zeros((E, A), dtype=torch.float32, device=dev)
    agents = agents.to(torch.int32).contiguous()
    sensed = sensed.to(torch.int32).contiguous()
    box = (ctypes.c_double * 3)(*[float(b) for b in np.asarray(box_scale, dtype=float)[:3]])
    mc = max(1, min(Ms, _TILE_BYTES // (4 * A * E)))
    s_nz = torch.zeros((E, A), dtype=torch.float32, device=dev)
    n_nz = torch.zeros((E, A), dtype=torch.int64, device=dev)
    first = last = None
    native.bind_stream()
    for m0 in range(0, Ms, mc):
        n = min(mc, Ms - m0)
        d = torch.empty((E, n, A), dtype=torch.float32, device=dev)
        native.call("swarm_pair_distances", agents.data_ptr(), A, sensed.data_ptr(), m0, n, box,
                    d.data_ptr())
        nz = d != 0
        s_nz += torch.where(nz, decay_fn(d), torch.zeros((), device=dev)).sum(dim=1)
        n_nz += nz.sum(dim=1)
        if m0 == 0:
            first = d[:, 0, :]
        if m0 + n == Ms:
            last = d[:, n - 1, :]
    zero = torch.zeros((), device=dev)
    field = s_nz - torch.where(n_nz == Ms, decay_fn(last), zero)
    pad = torch.clamp(Ms - 1 - n_nz, min=0).to(torch.float32)
    field = field + torch.where(pad > 0, pad * decay_fn(first), zero)
    return field


def list_pair_field(colloids, agent_indices, sensing_type: int, box_scale, decay_fn) -> np.ndarray:
    """Field values (A,) for a Colloid list, through a scratch points engine."""
    from swarmrl_amd.engine import ops

    pos = np.stack([np.asarray(c.pos, dtype=np.float64) for c in colloids])
    dims = ops.points_dims(pos)  # 3-D norms when any colloid is off z = 0
    n = len(pos)
    eng = ops.points_engine(n, ops.virtual_box(float(np.max(np.abs(pos[:, :dims]))) + 1.0), dims)
    dirs = np.zeros((n, 3))
    dirs[:, 0] = 1.0
    eng.upload(pos, dirs)
    dev = torch.device("cuda", torch.cuda.current_device())
    sensed = [i for i, c in enumerate(colloids) if c.type == sensing_type]
    a_t = torch.as_tensor(np.asarray(agent_indices, dtype=np.int32), device=dev)
    s_t = torch.as_tensor(np.asarray(sensed, dtype=np.int32), device=dev)
    return pair_field(eng.native, 1, a_t, s_t, box_scale, decay_fn)[0].cpu().numpy()
