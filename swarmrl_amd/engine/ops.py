"""
Thin Python wrappers over the observable entry points of the C ABI.

Both call forms of the reference observables/tasks run through the HIP
kernels:
  * batched: a ``SwarmView`` of a live engine -> device tensors [E, A, ...];
  * list:    a Python list of ``Colloid`` objects (the reference contract,
             e.g. its unit tests) -> the points are uploaded into a small
             scratch engine with a power-of-two virtual box (exact for
             integer coordinates) and the same kernels run on it.
There is no CPU implementation of these computations in the product.
"""

from __future__ import annotations

import ctypes
import math
from typing import Dict, Tuple

import numpy as np
import torch

from swarmrl_amd import _capi

_TWO32 = 4294967296.0


def to_fixed_host(x: np.ndarray, L: float) -> Tuple[np.ndarray, np.ndarray]:
    """Same rounding as to_fixed() in swarm_engine.hip (fp64, ties to even)."""
    u = np.asarray(x, dtype=np.float64) / L
    fl = np.floor(u)
    qd = np.rint((u - fl) * _TWO32)
    wrap = qd >= _TWO32
    qd = np.where(wrap, qd - _TWO32, qd)
    fl = np.where(wrap, fl + 1.0, fl)
    return qd.astype(np.uint64).astype(np.uint32), fl.astype(np.int32)


def vision_params(vision_range, half_angle, n_cones, detected_types) -> _capi.SwarmVisionParams:
    """Pack SubdividedVisionCones parameters; rims in the reference's fp32 order
    (-a + ((k * a) * 2) / n, subdivided_vision_cones.py:145-148)."""
    det = [int(t) for t in detected_types]
    if len(det) > _capi.SWARM_MAX_DETECTED_TYPES:
        raise ValueError("too many detected types for this build")
    if n_cones > _capi.SWARM_MAX_CONES:
        raise ValueError("too many cones for this build")
    vp = _capi.SwarmVisionParams()
    vp.vision_range = float(vision_range)
    vp.vision_half_angle = float(half_angle)
    vp.n_cones = int(n_cones)
    vp.n_types = len(det)
    for i, t in enumerate(det):
        vp.detected_types[i] = t
    a = np.float32(half_angle)
    k = np.arange(n_cones + 1, dtype=np.float32)
    rims = -a + ((k * a) * np.float32(2)) / np.float32(n_cones)
    for i, r in enumerate(rims.astype(np.float32)):
        vp.rims[i] = float(r)
    return vp


def vision_cone(native, n_envs: int, agent_idx: torch.Tensor, radii: torch.Tensor,
                types: torch.Tensor, vp: _capi.SwarmVisionParams,
                persistent: bool = False) -> torch.Tensor:
    """[E, A, n_cones, n_types] fp32 device tensor (k_vision).  persistent:
    the caller keeps agent_idx, radii and types alive and unchanged for the
    engine's lifetime (swarm_vision_cone_persistent: the next slice's grid
    may then be built by the reward launch)."""
    A = int(agent_idx.numel())
    out = torch.empty((n_envs, A, vp.n_cones, vp.n_types), dtype=torch.float32,
                      device=agent_idx.device)
    if A == 0:
        return out
    native.bind_stream()
    native.call(
        "swarm_vision_cone_persistent" if persistent else "swarm_vision_cone", ctypes.byref(vp),
        agent_idx.data_ptr(), A, radii.data_ptr(), types.data_ptr(), out.data_ptr(),
    )
    return out


def vision_policy(native, n_envs: int, agent_idx: torch.Tensor, radii: torch.Tensor,
                  types: torch.Tensor, vp: _capi.SwarmVisionParams, w1, b1, w2, b2, seed: int,
                  agent_state: torch.Tensor, explore_p: float, f_table: torch.Tensor,
                  t_table: torch.Tensor):
    """The persistent vision cone and the actor's rollout policy on it in one
    launch (swarm_engine_vision_policy): returns (features [E, A, n_cones,
    n_types], idx int64 [E * A], log_prob [E * A], f_swim [E * A], torque_z
    [E * A]).  agent_state: int64 device counters, one per agent."""
    A = int(agent_idx.numel())
    dev = agent_idx.device
    n = n_envs * A
    feats = torch.empty((n_envs, A, vp.n_cones, vp.n_types), dtype=torch.float32, device=dev)
    idx = torch.empty(n, dtype=torch.int64, device=dev)
    logp = torch.empty(n, dtype=torch.float32, device=dev)
    f = torch.empty(n, dtype=torch.float32, device=dev)
    t = torch.empty(n, dtype=torch.float32, device=dev)
    if A == 0:
        return feats, idx, logp, f, t
    hidden, k = int(w1.shape[0]), int(w2.shape[0])
    native.bind_stream()
    native.call(
        "swarm_engine_vision_policy", ctypes.byref(vp), agent_idx.data_ptr(), A,
        radii.data_ptr(), types.data_ptr(), feats.data_ptr(), w1.data_ptr(), b1.data_ptr(),
        hidden, w2.data_ptr(), b2.data_ptr(), k, ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
        agent_state.data_ptr(), int(agent_state.numel()), ctypes.c_float(explore_p),
        f_table.data_ptr(), t_table.data_ptr(), idx.data_ptr(), logp.data_ptr(), f.data_ptr(),
        t.data_ptr(), None,
    )
    return feats, idx, logp, f, t


def field_distance(native, n_envs: int, agent_idx: torch.Tensor, source, box_scale,
                   hist_q: torch.Tensor, hist_img: torch.Tensor, update: bool,
                   init_only: bool = False):
    """(d_cur, d_prev) fp32 [E, A] device tensors (k_field); updates the history."""
    A = int(agent_idx.numel())
    dev = agent_idx.device
    d_cur = torch.empty((n_envs, A), dtype=torch.float32, device=dev)
    d_prev = torch.empty((n_envs, A), dtype=torch.float32, device=dev)
    if A == 0:
        return d_cur, d_prev
    src = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(source, dtype=float)[:3]])
    bs = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(box_scale, dtype=float)[:3]])
    native.bind_stream()
    native.call(
        "swarm_field_distance", agent_idx.data_ptr(), A, ctypes.cast(src, ctypes.c_void_p),
        ctypes.cast(bs, ctypes.c_void_p), hist_q.data_ptr(), hist_img.data_ptr(),
        d_cur.data_ptr(), d_prev.data_ptr(), 1 if update else 0, 1 if init_only else 0,
    )
    return d_cur, d_prev


# ------------------------------------------------------------ list path
class _PointsEngine:
    """A scratch single-env engine that holds an arbitrary point set (2-D, or
    3-D for points off the z = 0 plane)."""

    def __init__(self, n: int, box: float, dims: int = 2):
        from swarmrl_amd.engine.swarm_engine import _NativeEngine

        _capi.require_gpu()
        p = _capi.SwarmParams()
        p.n_dims = int(dims)
        p.periodic = 1
        for a in range(3):
            p.box[a] = box
        p.time_step = 1.0
        p.kT = 0.0
        p.wca_epsilon = 0.0
        p.n_species = 1
        p.radius[0] = 0.0
        p.gamma_t[0] = 1.0
        p.gamma_r[0] = 1.0
        self.native = _NativeEngine(p, 1, np.zeros(n, dtype=np.int32))
        self.n = n
        self.box = box

    def upload(self, pos: np.ndarray, director: np.ndarray):
        pos = np.ascontiguousarray(pos, dtype=np.float64).reshape(self.n, 3)
        director = np.ascontiguousarray(director, dtype=np.float64).reshape(self.n, 3)
        self.native.bind_stream()
        self.native.call("swarm_engine_upload_state", pos.ctypes.data, director.ctypes.data)


_points_cache: Dict[tuple, _PointsEngine] = {}


def virtual_box(extent: float) -> float:
    """Power-of-two box comfortably larger than every coordinate/range."""
    return float(2.0 ** max(4, math.ceil(math.log2(max(extent, 1.0) * 4.0 + 1.0))))


def points_engine(n: int, box: float, dims: int = 2) -> _PointsEngine:
    key = (n, box, int(dims), torch.cuda.current_device())
    eng = _points_cache.get(key)
    if eng is None:
        if len(_points_cache) > 32:
            _points_cache.clear()
        eng = _PointsEngine(n, box, dims)
        _points_cache[key] = eng
    return eng


def points_dims(*arrays) -> int:
    """3 when any point of the (k, 3) arrays lies off the z = 0 plane (the
    reference's observables take norms of 3-vectors, concentration_field.py:
    100-101), else 2."""
    return 3 if any(np.any(np.asarray(a, dtype=np.float64).reshape(-1, 3)[:, 2] != 0)
                    for a in arrays) else 2


def list_vision_cone(positions: np.ndarray, directors: np.ndarray, types: np.ndarray,
                     agent_indices, radii: np.ndarray, vision_range: float,
                     half_angle: float, n_cones: int, detected_types) -> np.ndarray:
    """Vision cones for a Colloid list: [A, n_cones, n_types] (numpy fp32)."""
    positions = np.asarray(positions, dtype=np.float64)
    n = len(positions)
    extent = float(np.max(np.abs(positions[:, :2]))) + float(vision_range)
    eng = points_engine(n, virtual_box(extent))
    eng.upload(positions, directors)
    dev = torch.device("cuda", torch.cuda.current_device())
    agent_t = torch.as_tensor(np.asarray(agent_indices, dtype=np.int32), device=dev)
    radii_t = torch.as_tensor(np.asarray(radii, dtype=np.float32), device=dev)
    types_t = torch.as_tensor(np.asarray(types, dtype=np.int32), device=dev)
    vp = vision_params(vision_range, half_angle, n_cones, detected_types)
    out = vision_cone(eng.native, 1, agent_t, radii_t, types_t, vp)
    return out[0].cpu().numpy()


def list_field_distance(cur_scaled: np.ndarray, prev_scaled: np.ndarray,
                        source_scaled: np.ndarray):
    """
    Distances for the list path: positions and source are already divided by
    the box (fp64, as the reference does); returns fp32 numpy (d_cur, d_prev).
    """
    cur_scaled = np.asarray(cur_scaled, dtype=np.float64).reshape(-1, 3)
    prev_scaled = np.asarray(prev_scaled, dtype=np.float64).reshape(-1, 3)
    A = len(cur_scaled)
    if A == 0:
        return np.zeros(0, np.float32), np.zeros(0, np.float32)
    src = np.asarray(source_scaled, dtype=np.float64).reshape(3)
    dims = points_dims(cur_scaled, prev_scaled)
    extent = max(
        float(np.max(np.abs(cur_scaled[:, :dims]))), float(np.max(np.abs(prev_scaled[:, :dims]))),
        1.0)
    L = virtual_box(extent)
    eng = points_engine(A, L, dims)
    dirs = np.zeros((A, 3))
    dirs[:, 0] = 1.0
    pos = cur_scaled.copy()
    if dims == 2:
        pos[:, 2] = 0.0
    eng.upload(pos, dirs)
    dev = torch.device("cuda", torch.cuda.current_device())
    hq = np.zeros((3, A), dtype=np.uint32)
    hi = np.zeros((3, A), dtype=np.int32)
    for a in range(dims):
        hq[a], hi[a] = to_fixed_host(prev_scaled[:, a], L)
    hq_t = torch.as_tensor(hq.view(np.int32), device=dev)
    hi_t = torch.as_tensor(hi, device=dev)
    agent_t = torch.arange(A, dtype=torch.int32, device=dev)
    # the kernel scales engine coordinates by box[a] / box_scale[a]; the
    # engine already holds scaled coordinates, so box_scale = 1.
    d_cur, d_prev = field_distance(eng.native, 1, agent_t, src, np.ones(3), hq_t, hi_t,
                                   update=False)
    return d_cur[0].cpu().numpy(), d_prev[0].cpu().numpy()


# ------------------------------------------------- history initialisation
def engine_of(colloids):
    """The SwarmEngine behind a list of engine particle handles, else None."""
    if isinstance(colloids, (list, tuple)) and len(colloids) > 0:
        eng = getattr(colloids[0], "_engine", None)
        if eng is not None and all(getattr(c, "_engine", None) is eng for c in colloids):
            return eng
    return None


def snapshot_history(engine, p_type: int):
    """
    Raw engine coordinates (q [3, E*A] uint32, img [3, E*A] int32) of the
    agents of one type, taken now: from the registry before the first
    integrate (exactly what upload_state will convert), else from the device.
    """
    types = np.asarray(engine._types_list, dtype=np.int64)
    idx = np.nonzero(types == int(p_type))[0]
    E, N = engine.n_envs, engine.n_particles
    A = len(idx)
    hq = np.zeros((3, E, A), dtype=np.uint32)
    hi = np.zeros((3, E, A), dtype=np.int32)
    if engine._native is None:
        pos = np.stack([np.stack(v) for v in engine._pos])  # [E, N, 3]
        for a in range(int(engine.n_dims)):
            q, im = to_fixed_host(pos[:, idx, a], float(engine._box[a]))
            hq[a], hi[a] = q, im
    else:
        raw = engine.get_raw_state()
        hq[:] = raw["q"].reshape(3, E, N)[:, :, idx]
        hi[:] = raw["img"].reshape(3, E, N)[:, :, idx]
    return hq.reshape(3, E * A), hi.reshape(3, E * A)


def history_tensors(hq: np.ndarray, hi: np.ndarray, device):
    return (
        torch.as_tensor(np.ascontiguousarray(hq).view(np.int32), device=device).clone(),
        torch.as_tensor(np.ascontiguousarray(hi), device=device).clone(),
    )


# ------------------------------------------------ fused affine field tasks
def affine_coefficients(decay_fn):
    """
    (a, b) if decay_fn(d) == a + b * d exactly in fp32 on probe values (the
    reference's decay functions, e.g. ``1 - d`` or ``-1 * d``), else None.
    Affine decays run fused inside the HIP field kernel.
    """
    try:
        probe = torch.tensor([0.0, 1.0, 2.0, 0.3712, 123.5, 7.25e-3], dtype=torch.float32)
        y = decay_fn(probe)
        if not isinstance(y, torch.Tensor) or y.shape != probe.shape or y.dtype != torch.float32:
            return None
        a = y[0]
        b = y[1] - y[0]
        if not torch.equal(a + b * probe, y):
            return None
        return float(a), float(b)
    except Exception:
        return None


def field_transform(native, n_envs: int, agent_idx: torch.Tensor, source, box_scale,
                    hist_q: torch.Tensor, hist_img: torch.Tensor, a: float, b: float,
                    scale: float, clip: bool) -> torch.Tensor:
    """scale * (f(d_cur) - f(d_prev)) [E, A] for affine f (k_field, fused)."""
    A = int(agent_idx.numel())
    out = torch.empty((n_envs, A), dtype=torch.float32, device=agent_idx.device)
    if A == 0:
        return out
    src = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(source, dtype=float)[:3]])
    bs = (ctypes.c_double * 3)(*[float(v) for v in np.asarray(box_scale, dtype=float)[:3]])
    native.bind_stream()
    native.call(
        "swarm_field_transform", agent_idx.data_ptr(), A, ctypes.cast(src, ctypes.c_void_p),
        ctypes.cast(bs, ctypes.c_void_p), hist_q.data_ptr(), hist_img.data_ptr(), float(a),
        float(b), float(scale), 1 if clip else 0, out.data_ptr(),
    )
    return out


def counter_state(state, n: int, device):
    """Device call counters of the sampling kernels: one int64 per group of
    64 agents (grown, never shrunk; new groups start at zero)."""
    need = max(1, (n + 63) // 64)
    if state is None or state.device != device:
        return torch.zeros(need, dtype=torch.int64, device=device)
    if state.numel() < need:
        grown = torch.zeros(need, dtype=torch.int64, device=device)
        grown[: state.numel()] = state
        return grown
    return state


def sample_actions(logits: torch.Tensor, seed: int, state: torch.Tensor, explore_p: float,
                   f_table: torch.Tensor, t_table: torch.Tensor):
    """
    Fused Gumbel-max sampling + exploration + log(softmax + 1e-8) of the
    chosen action + action-table lookup (swarm_sample_actions, one kernel on
    the current stream).  logits [n, k] fp32 (device); state: int64 device
    counters, at least ceil(n / 64) (counter_state).  Returns
    (idx int64 [n], log_prob [n], f_swim [n], torque_z [n]).
    """
    logits = logits.contiguous()
    n, k = logits.shape
    dev = logits.device
    idx = torch.empty(n, dtype=torch.int64, device=dev)
    logp = torch.empty(n, dtype=torch.float32, device=dev)
    f = torch.empty(n, dtype=torch.float32, device=dev)
    t = torch.empty(n, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().swarm_sample_actions(
        logits.data_ptr(), n, k, ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), state.data_ptr(),
        int(state.numel()), ctypes.c_float(explore_p), f_table.data_ptr(), t_table.data_ptr(),
        idx.data_ptr(), logp.data_ptr(), f.data_ptr(), t.data_ptr(), ctypes.c_void_p(stream)))
    return idx, logp, f, t


def policy_mlp_sample(obs: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
                      b2: torch.Tensor, seed: int, state: torch.Tensor, explore_p: float,
                      f_table: torch.Tensor, t_table: torch.Tensor, want_logits: bool = False,
                      engine=None):
    """
    The rollout policy in one kernel (swarm_policy_mlp_sample): actor logits
    W2 relu(W1 obs + b1) + b2 from the torch Linear weights in place, then the
    sampling of sample_actions (same counters and bits).  obs [n, d_in] fp32
    device.  Returns (idx, log_prob, f_swim, torque_z[, logits]).  engine: a
    native engine whose deferred build's last stage rides along in the same
    launch (swarm_engine_policy_mlp_sample); same results.
    """
    obs = obs.contiguous()
    n, d_in = obs.shape
    hidden, k = int(w1.shape[0]), int(w2.shape[0])
    dev = obs.device
    idx = torch.empty(n, dtype=torch.int64, device=dev)
    logp = torch.empty(n, dtype=torch.float32, device=dev)
    f = torch.empty(n, dtype=torch.float32, device=dev)
    t = torch.empty(n, dtype=torch.float32, device=dev)
    logits = torch.empty(n, k, dtype=torch.float32, device=dev) if want_logits else None
    stream = torch.cuda.current_stream(dev).cuda_stream
    args = (obs.data_ptr(), n, d_in, w1.data_ptr(), b1.data_ptr(), hidden, w2.data_ptr(),
            b2.data_ptr(), k, ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), state.data_ptr(),
            int(state.numel()), ctypes.c_float(explore_p), f_table.data_ptr(), t_table.data_ptr(),
            idx.data_ptr(), logp.data_ptr(), f.data_ptr(), t.data_ptr(),
            logits.data_ptr() if want_logits else None, ctypes.c_void_p(stream))
    if engine is not None:
        _capi.check(_capi.lib().swarm_engine_policy_mlp_sample(engine.ptr, *args))
    else:
        _capi.check(_capi.lib().swarm_policy_mlp_sample(*args))
    if want_logits:
        return idx, logp, f, t, logits
    return idx, logp, f, t


def adam_args(optimizer, layers):
    """swarm_adam_t for a torch Adam whose only parameters are the six PPO
    layers, or None when the fused step does not apply (another optimizer,
    weight decay, amsgrad / maximize, several groups, state not on the
    device yet).  Holds device pointers: valid while the tensors live."""
    if type(optimizer) is not torch.optim.Adam or len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    if (g.get("weight_decay", 0) != 0 or g.get("amsgrad") or g.get("maximize")
            or not g.get("capturable") or g.get("differentiable")
            or isinstance(g["lr"], torch.Tensor)):
        return None
    if len(g["params"]) != 6 or {id(p) for p in g["params"]} != {id(t) for t in layers}:
        return None
    a = _capi.SwarmAdam()
    a.lr, a.beta1, a.beta2, a.eps = float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), \
        float(g["eps"])
    for k, t in enumerate(layers):
        st = optimizer.state.get(t, {})
        need = ("exp_avg", "exp_avg_sq", "step")
        if not all(isinstance(st.get(n), torch.Tensor) and st[n].is_cuda for n in need):
            return None
        if (st["step"].dtype != torch.float32 or st["exp_avg"].dtype != torch.float32
                or not t.is_contiguous() or t.dtype != torch.float32):
            return None
        a.param[k] = t.data_ptr()
        a.exp_avg[k] = st["exp_avg"].data_ptr()
        a.exp_avg_sq[k] = st["exp_avg_sq"].data_ptr()
        a.step[k] = st["step"].data_ptr()
    return a


def ppo_epoch_grad(features: torch.Tensor, actions: torch.Tensor, old_logp: torch.Tensor,
                   rewards: torch.Tensor, layers, gamma: float, lambda_: float,
                   clip_eps: float, entropy_coef: float, out: torch.Tensor = None,
                   adam=None, workspaces: dict = None) -> torch.Tensor:
    """
    The gradient of one PPO epoch (swarm_ppo_epoch_grad): features [T, S, d]
    fp32, actions [T, S] int64, old_logp / rewards [T, S] fp32 (all device),
    layers = (w1, b1, wa, ba, wc, bc) of the actor-critic MLP in torch
    layouts.  Returns the flat gradient w1 | b1 | wa | ba | wc | bc (fp32),
    written into `out` when given.  Inputs already fp32/int64 and contiguous
    are used in place (no copies: the launches can be graph-captured).
    adam: a swarm_adam_t (adam_args) -- the optimizer's step then runs in the
    epoch's last launch (swarm_ppo_epoch_step) and updates the layers.
    workspaces: the caller's own cache of workspaces (one per device and
    size, never dropped while the caller lives, so a captured graph that
    holds a workspace's pointer never replays into freed memory); without
    one every call takes a fresh zeroed buffer (a module-wide
    single-entry cache freed a buffer another loss's graph still used).
    """
    T, S = int(actions.shape[0]), int(actions.shape[1])
    x = features.reshape(T * S, -1).to(torch.float32).contiguous()
    d_in = int(x.shape[1])
    w1, b1, wa, ba, wc, bc = layers
    hidden, k = int(w1.shape[0]), int(wa.shape[0])
    dev = x.device
    lib = _capi.lib()
    nbytes = int(lib.swarm_ppo_workspace_bytes(T, S, d_in, hidden, k))
    if nbytes < 0:
        raise ValueError("bad PPO sizes")
    key = (dev.index or 0, nbytes)
    ws = workspaces.get(key) if workspaces is not None else None
    if ws is None:  # zeroed once: the fused Adam's ticket is left at zero after use
        ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        if workspaces is not None:
            workspaces[key] = ws
    size = hidden * d_in + hidden + k * hidden + k + hidden + 1
    grad = out if out is not None else torch.empty(size, dtype=torch.float32, device=dev)
    if grad.numel() != size or grad.dtype != torch.float32 or not grad.is_contiguous():
        raise ValueError("out must be a contiguous fp32 tensor of the gradient's size")
    acts = actions.to(torch.int64).contiguous()
    olp = old_logp.to(torch.float32).contiguous()
    rew = rewards.to(torch.float32).contiguous()
    stream = torch.cuda.current_stream(dev).cuda_stream
    if adam is not None:  # the optimizer step fused into the epoch (swarm_ppo_epoch_step)
        _capi.check(lib.swarm_ppo_epoch_step(
            x.data_ptr(), T, S, d_in, acts.data_ptr(), olp.data_ptr(), rew.data_ptr(), hidden, k,
            ctypes.c_float(gamma), ctypes.c_float(lambda_), ctypes.c_float(clip_eps),
            ctypes.c_float(entropy_coef), ctypes.byref(adam), ws.data_ptr(), nbytes,
            grad.data_ptr(), ctypes.c_void_p(stream)))
        return grad
    _capi.check(lib.swarm_ppo_epoch_grad(
        x.data_ptr(), T, S, d_in, acts.data_ptr(), olp.data_ptr(), rew.data_ptr(),
        w1.data_ptr(), b1.data_ptr(), hidden, wa.data_ptr(), ba.data_ptr(), k, wc.data_ptr(),
        bc.data_ptr(), ctypes.c_float(gamma), ctypes.c_float(lambda_), ctypes.c_float(clip_eps),
        ctypes.c_float(entropy_coef), ws.data_ptr(), nbytes, grad.data_ptr(),
        ctypes.c_void_p(stream)))
    return grad


NB_COUNT, NB_PERCEPTION, NB_SUM_D, NB_SUM_D2, NB_SUM_DIR, NB_SUM_V = 0, 1, 2, 5, 6, 9


def neighbor_reduce(pos: torch.Tensor, directors: torch.Tensor, velocities, types: torch.Tensor,
                    agent_idx: torch.Tensor, cand_types, vision_range: float,
                    half_angle: float) -> torch.Tensor:
    """
    Neighbour sums of the classical agents (swarm_neighbor_reduce, one HIP
    kernel): pos [E, N, 3] fp64, directors / velocities [E, N, 3] (velocities
    may be None), types [N] int32, agent_idx [A] int32 (all device).  Returns
    fp64 [E, A, 12]: count, sum 1/(2 pi |d|), sum d (3), sum |d|^2, sum
    dir_j (3), sum v_j (3) over the candidates (types in cand_types, not the
    agent) within vision_range and, for half_angle >= 0, inside the cone.
    """
    E, N = int(pos.shape[0]), int(pos.shape[1])
    dev = pos.device
    pos = pos.to(torch.float64).contiguous()
    dirs = directors.to(torch.float64).contiguous()
    vel = None if velocities is None else velocities.to(torch.float64).contiguous()
    A = int(agent_idx.numel())
    out = torch.empty((E, A, 12), dtype=torch.float64, device=dev)
    mask = 0
    for t in cand_types:
        if not 0 <= int(t) < 32:
            raise ValueError("particle types must be in [0, 32) for the neighbour kernel")
        mask |= 1 << int(t)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _capi.check(_capi.lib().swarm_neighbor_reduce(
        pos.data_ptr(), dirs.data_ptr(), None if vel is None else vel.data_ptr(),
        types.to(torch.int32).contiguous().data_ptr(), E, N,
        agent_idx.to(torch.int32).contiguous().data_ptr(), A, ctypes.c_uint32(mask),
        float(vision_range), float(half_angle), out.data_ptr(), ctypes.c_void_p(stream)))
    return out


def rnd_distance(points: torch.Tensor, target: torch.nn.Module, predictor: torch.nn.Module,
                 order: int) -> torch.Tensor:
    """The RND metric of every observation in one launch (swarm_rnd_distance):
    points [n, d] fp32 device; target / predictor: the stock RNDArchitecture
    (three Linear layers of width 32), weights read in place.  Returns [n]."""
    points = points.contiguous()
    n, d = points.shape
    out = torch.empty(n, dtype=torch.float32, device=points.device)

    def ptrs(net):
        lin = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
        arr = (ctypes.c_void_p * 6)()
        for k, m in enumerate(lin):
            arr[2 * k] = m.weight.data_ptr()
            arr[2 * k + 1] = m.bias.data_ptr()
        return arr

    stream = torch.cuda.current_stream(points.device).cuda_stream
    tp, pp = ptrs(target), ptrs(predictor)
    _capi.check(_capi.lib().swarm_rnd_distance(
        points.data_ptr(), n, d, 32, ctypes.cast(tp, ctypes.c_void_p),
        ctypes.cast(pp, ctypes.c_void_p), int(order), out.data_ptr(), ctypes.c_void_p(stream)))
    return out


def rnd_env_reward(points: torch.Tensor, n_envs: int, target: torch.nn.Module,
                   predictor: torch.nn.Module, order: int, clip, base: torch.Tensor = None,
                   workspaces: dict = None):
    """The per-env RND reward added to the task reward (swarm_rnd_env_reward):
    points [n_envs * per_env, d] fp32 device (env-major); returns (metric [n],
    env_reward [n_envs, 1], rewards [n_envs, per_env] = base + env_reward, or
    env_reward broadcast when base is None).  clip: (lo, hi) or None.
    workspaces: the caller's own cache of partial-sum workspaces (one per
    device and size, kept alive for captured graphs that read them); without
    one every call takes a fresh stream-ordered buffer, so no two callers
    ever share one."""
    points = points.contiguous()
    n, d = points.shape
    per_env = n // n_envs
    dev = points.device
    metric = torch.empty(n, dtype=torch.float32, device=dev)
    env_r = torch.empty(n_envs, 1, dtype=torch.float32, device=dev)
    rewards = torch.empty(n_envs, per_env, dtype=torch.float32, device=dev)
    if base is not None:
        base = base.to(torch.float32).reshape(n_envs, per_env).contiguous()
    lib = _capi.lib()
    nbytes = int(lib.swarm_rnd_env_workspace_bytes(n_envs, per_env))
    key = (dev, nbytes)
    ws = workspaces.get(key) if workspaces is not None else None
    if ws is None:  # zeroed once: the kernel leaves its tickets at zero after use
        ws = torch.zeros(max(nbytes, 8), dtype=torch.uint8, device=dev)
        if workspaces is not None:
            workspaces[key] = ws

    def ptrs(net):
        lin = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
        arr = (ctypes.c_void_p * 6)()
        for k, m in enumerate(lin):
            arr[2 * k] = m.weight.data_ptr()
            arr[2 * k + 1] = m.bias.data_ptr()
        return arr

    stream = torch.cuda.current_stream(dev).cuda_stream
    tp, pp = ptrs(target), ptrs(predictor)
    lo, hi = (float(clip[0]), float(clip[1])) if clip is not None else (0.0, 0.0)
    _capi.check(lib.swarm_rnd_env_reward(
        points.data_ptr(), n_envs, per_env, d, 32, ctypes.cast(tp, ctypes.c_void_p),
        ctypes.cast(pp, ctypes.c_void_p), int(order), 1 if clip is not None else 0, lo, hi,
        base.data_ptr() if base is not None else None, metric.data_ptr(), env_r.data_ptr(),
        rewards.data_ptr(), ws.data_ptr(), ctypes.c_int64(ws.numel()), ctypes.c_void_p(stream)))
    return metric, env_r, rewards

