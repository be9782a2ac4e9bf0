"""
Plain numpy (fp64) restatement of the reference's semantics on the hot path.

TEST INFRASTRUCTURE ONLY.  The reference (/root/reference, pure Python over
jax/pint/h5py/espressomd) cannot be imported in this image
(ModuleNotFoundError: jax) and never travels to the GPU box,
so its behaviour is restated here from its source text, function by
function, with the file:line it follows.  These restatements are pinned by
the reference's own known-answer tests (tests/test_oracle_kat.py) and then
used to check the C oracle's number formats on random inputs.
"""

from __future__ import annotations

import math

import numpy as np


# --------------------------------------------------------- schedule (a1)
def schedule(steps_per_slice: int, steps_per_write: int, calls, write_chunk_size: int):
    """
    Restates EspressoMD.integrate's bookkeeping (espresso.py:1251-1308)
    including _update_traj_holder/_write_traj_chunk_to_file cadence.
    ``calls`` is a list of n_slices per integrate() call.  Returns one dict
    per call with step/slice/write indices, traj-holder length and the
    numbers of manage_forces / calc_reward / integrator.run invocations.
    """
    step_idx = slice_idx = write_idx = 0
    holder = 0
    out = []
    n_manage = n_reward = 0
    runs = []
    for n_slices in calls:
        old = slice_idx
        while step_idx < steps_per_slice * (old + n_slices):
            if step_idx == steps_per_write * write_idx:
                holder += 1
                write_idx += 1
                if holder >= write_chunk_size:
                    holder = 0
            if step_idx == steps_per_slice * slice_idx:
                slice_idx += 1
                n_manage += 1
            to_write = steps_per_write * write_idx - step_idx
            to_slice = steps_per_slice * slice_idx - step_idx
            k = min(to_write, to_slice)
            runs.append(k)
            n_reward += 1
            step_idx += k
        out.append(dict(step_idx=step_idx, slice_idx=slice_idx, write_idx=write_idx,
                        traj_len=holder, n_manage=n_manage, n_reward=n_reward,
                        runs=list(runs)))
    return out


# ------------------------------------------------------ placement (a3 init)
def placement(n, init_radius, center, seed, n_calls_before=0):
    """
    add_colloids 2-D placement (espresso.py:91-105, 521-533): per colloid
    r = R sqrt(U), theta = 2 pi U, then director angle 2 pi U; the director
    goes through vector_from_angles / angles_from_vector (utils.py:24-34).
    """
    rng = np.random.default_rng(seed)
    pos = np.zeros((n, 3))
    dirs = np.zeros((n, 3))
    for i in range(n):
        r = init_radius * np.sqrt(rng.random())
        th = 2 * np.pi * rng.random()
        pos[i] = r * np.array([np.cos(th), np.sin(th), 0]) + center
        pos[i, 2] = 0
        a = 2 * np.pi * rng.random()
        d = np.array([np.sin(np.pi / 2) * np.cos(a), np.sin(np.pi / 2) * np.sin(a),
                      np.cos(np.pi / 2)])
        d = d / np.linalg.norm(d)
        phi = np.arctan2(d[1], d[0])
        dirs[i] = [np.cos(phi), np.sin(phi), 0.0]
    return pos, dirs


def placement3(n, init_radius, center, seed):
    """
    add_colloids 3-D placement (espresso.py:91-105, 521-529): per colloid
    r = R cbrt(U), direction from get_random_angles (theta = arccos(2U - 1),
    phi = 2 pi U, utils.py:19-27) for the position, then again for the
    director.
    """
    rng = np.random.default_rng(seed)
    pos = np.zeros((n, 3))
    dirs = np.zeros((n, 3))

    def unit(theta, phi):
        return np.array([np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi),
                         np.cos(theta)])

    for i in range(n):
        r = init_radius * np.cbrt(rng.random())
        th = np.arccos(2.0 * rng.random() - 1)
        ph = 2.0 * np.pi * rng.random()
        pos[i] = r * unit(th, ph) + center
        th = np.arccos(2.0 * rng.random() - 1)
        ph = 2.0 * np.pi * rng.random()
        dirs[i] = unit(th, ph)
    return pos, dirs


def wall_distance_plane(x, normal, offset):
    """espressomd.shapes.Wall: dist = n . x - offset (folded position)."""
    return float(np.dot(normal, x) - offset)


# ----------------------------------------------------------- units (a3)
K_B = 1.380649e-23
SIM_ENERGY = 293 * K_B                       # espresso.py:223
SIM_MASS = SIM_ENERGY / (1e-6) ** 2          # sim_energy / sim_velocity^2
SIM_DYN_VISC = SIM_MASS / (1e-6 * 1.0)       # sim_mass / (sim_length sim_time)


def friction(eta_si, radius_um):
    """espresso.py:108-113 in simulation units."""
    eta = eta_si / SIM_DYN_VISC
    return 6 * np.pi * eta * radius_um, 8 * np.pi * eta * radius_um**3


# ------------------------------------------------------- signed angle (a10)
def signed_angle(my_director, other_director):
    """calc_signed_angle_between_directors (utils.py:297-332), fp64."""
    my = np.asarray(my_director, dtype=float)
    ot = np.asarray(other_director, dtype=float)
    my = my / np.linalg.norm(my)
    ot = ot / np.linalg.norm(ot)
    angle = np.arccos(np.clip(np.dot(ot, my), -1.0, 1.0))
    orth = np.dot(ot, np.array([-my[1], my[0], my[2]]))
    return angle * (1 if orth >= 0 else -1)


# -------------------------------------------------------- vision cone (a10)
def vision_cones(positions, directors, types, radii, vision_range, half_angle, n_cones,
                 detected_types=None, particle_type=0):
    """
    SubdividedVisionCones.compute_observable (subdivided_vision_cones.py:
    105-258) in fp64: for each agent (type == particle_type), sum over ALL
    colloids j (the `c is not index` filter never removes anything, line 232)
    of in_range * min(1, 2 r_j / d) * type_mask * in_cone; the self term is
    NaN-masked to 0 (d = 0 gives NaN angles).
    """
    positions = np.asarray(positions, dtype=float)
    directors = np.asarray(directors, dtype=float)
    types = np.asarray(types)
    if detected_types is None:
        seen = []
        for t in types:
            if t not in seen:
                seen.append(t)
        detected_types = np.sort(seen)
    detected_types = np.asarray(detected_types)
    rims = -half_angle + np.arange(n_cones + 1) * half_angle * 2 / n_cones
    agents = [i for i, t in enumerate(types) if t == particle_type]
    out = []
    for i in agents:
        acc = np.zeros((n_cones, len(detected_types)))
        for j in range(len(positions)):
            dist = positions[j] - positions[i]
            d = np.linalg.norm(dist)
            if not d < vision_range or d == 0.0:
                continue
            amp = min(1.0, 2 * radii[j] / d)
            col = np.nonzero(detected_types == types[j])[0]
            if len(col) == 0:
                continue
            ang = signed_angle(directors[i], dist / d)
            for k in range(n_cones):
                if rims[k] < ang < rims[k + 1]:
                    acc[k, col[0]] += amp
        out.append(acc)
    return out


# ------------------------------------------- concentration / gradient (a11/12)
def field_distance(pos, source, box_length):
    """|| fp32(source/L - pos/L) || as the reference computes it
    (concentration_field.py:100-101; gradient_sensing.py:110-111)."""
    diff = np.asarray(source, dtype=float) / box_length - np.asarray(pos, dtype=float) / box_length
    d32 = diff.astype(np.float32)
    return np.float32(np.sqrt(np.sum(d32.astype(np.float64) ** 2)))


def concentration_observable(cur, prev, source, box_length, decay_fn, scale):
    """scale * (f(d_cur) - f(d_prev)) (concentration_field.py:102-104)."""
    dc = field_distance(cur, source, box_length)
    dp = field_distance(prev, source, box_length)
    return scale * (decay_fn(dc) - decay_fn(dp))


def gradient_reward(cur, prev, source, box_length, decay_fn, scale):
    """clip(scale * (f(d_cur) - f(d_prev)), 0, inf) (gradient_sensing.py:108-121)."""
    return max(0.0, float(concentration_observable(cur, prev, source, box_length, decay_fn,
                                                   scale)))


# --------------------------------------------------- BD, deterministic (a3)
def pair_field(positions, types, agent_indices, sensing_type, box_length, decay_fn):
    """
    particle_sensing.py:95-121 / species_search.py:97-130 in numpy fp32:
    d = ||(x_j - x_i) / L|| over the sensed colloids (colloid order); the
    first M - 1 non-zero distances, padded with index 0 when fewer
    (jnp.nonzero(..., size=M - 1), fill 0); field = decay(d).sum().
    """
    pos = np.asarray(positions, dtype=np.float32)
    box = np.asarray(box_length, dtype=np.float32)
    test = pos[[j for j, t in enumerate(types) if t == sensing_type]]
    m = len(test)
    out = []
    for i in agent_indices:
        d = np.linalg.norm((test - pos[i]) / box, axis=-1).astype(np.float32)
        nz = np.nonzero(d)[0][: m - 1]
        idx = np.concatenate([nz, np.zeros(max(0, m - 1 - len(nz)), dtype=int)])
        out.append(np.float32(np.sum(decay_fn(d[idx]), dtype=np.float32)))
    return np.array(out, dtype=np.float32)


def bd_free_deterministic(pos0, theta0, f_swim, torque_z, gamma_t, gamma_r, dt, n_steps):
    """kT = 0, no pair forces: x += f d(theta)/gamma_t dt, theta += tau/gamma_r dt."""
    pos = np.array(pos0, dtype=float)
    th = np.array(theta0, dtype=float)
    for _ in range(n_steps):
        d = np.stack([np.cos(th), np.sin(th)], axis=-1)
        pos[:, :2] += (np.asarray(f_swim)[:, None] * d) / gamma_t * dt
        th = th + np.asarray(torque_z) / gamma_r * dt
    return pos, th


def wca_force(r_vec, r_i, r_j, eps):
    """ESPResSo WCA (espresso.py:814-819): sigma = (r_i + r_j) 2^(-1/6)."""
    sig = (r_i + r_j) * 2 ** (-1 / 6)
    r = np.linalg.norm(r_vec)
    if r >= (r_i + r_j):
        return np.zeros_like(r_vec)
    s6 = (sig / r) ** 6
    return 48 * eps / r**2 * (s6 * s6 - 0.5 * s6) * r_vec


def expected_msd_2d(kT, gamma_t, t):
    return 4 * kT / gamma_t * t


def expected_orientation_corr(kT, gamma_r, t):
    return math.exp(-kT / gamma_r * t)


# ------------------------------------------ classical agents (rank 4, 8f)
def colloids_in_vision(my_pos, my_dir, others_pos, vision_half_angle=np.pi,
                       vision_range=np.inf, cone=True):
    """bechinger_models.py:156-171 / lymburn_model.py:113-125: indices of
    others within range (and, with cone, acos(d/|d| . dir) < half angle)."""
    out = []
    for k, p in enumerate(others_pos):
        d = p - my_pos
        dn = np.linalg.norm(d)
        if not dn < vision_range:
            continue
        if cone and not np.arccos(np.dot(d / dn, my_dir)) < vision_half_angle:
            continue
        out.append(k)
    return out


def lavergne_forces(pos, dirs, types, half_angle, act_force, threshold, acts_on):
    """bechinger_models.py:29-50: per colloid the swim force (0 if off)."""
    f = np.zeros(len(pos))
    for i in range(len(pos)):
        if types[i] not in acts_on:
            continue
        others = [j for j in range(len(pos)) if j != i]
        vis = colloids_in_vision(pos[i], dirs[i], pos[others], half_angle)
        perception = sum(1 / (2 * np.pi * np.linalg.norm(pos[i] - pos[others[k]])) for k in vis)
        if perception >= threshold:
            f[i] = act_force
    return f


def baeuerle_actions(pos, dirs, types, act_force, act_torque, r_pos, r_orient, half_angle,
                     dev, acts_on):
    """bechinger_models.py:81-153: (force, torque_z) per colloid."""
    f = np.zeros(len(pos))
    tz = np.zeros(len(pos))
    for i in range(len(pos)):
        if types[i] not in acts_on:
            continue
        others = [j for j in range(len(pos)) if j != i]
        vp = colloids_in_vision(pos[i], dirs[i], pos[others], half_angle, r_pos)
        if len(vp) == 0:
            continue
        com = np.mean(np.stack([pos[others[k]] for k in vp]), axis=0)
        to_com = com - pos[i]
        to_com_angle = np.arctan2(to_com[1], to_com[0])
        vo = colloids_in_vision(pos[i], dirs[i], pos[others], half_angle, r_orient)
        if len(vo) == 0:
            continue
        mo = np.mean(np.stack([dirs[others[k]] for k in vo] + [dirs[i]]), axis=0)
        mo /= np.linalg.norm(mo)
        choices = [to_com_angle + dev, to_com_angle - dev]
        devs = [np.arccos(np.dot(np.array([np.cos(a), np.sin(a), 0]), mo)) for a in choices]
        target = choices[np.argmin(devs)]
        diff = target - np.arctan2(dirs[i][1], dirs[i][0])
        if diff >= np.pi:
            diff -= 2 * np.pi
        if diff <= -np.pi:
            diff += 2 * np.pi
        f[i] = act_force
        tz[i] = np.sin(diff) * act_torque
    return f, tz


def lymburn_actions(pos, vel, types, K, r_colls, r_pred, home, speed, pred_type):
    """lymburn_model.py:55-110: (force magnitude, direction) per non-predator."""
    out = []
    pred = [j for j in range(len(pos)) if types[j] == pred_type]
    for i in range(len(pos)):
        if types[i] == pred_type:
            continue
        others = [j for j in range(len(pos)) if j != i and types[j] != pred_type]
        vis = [others[k] for k in colloids_in_vision(pos[i], None, pos[others], vision_range=r_colls,
                                                     cone=False)]
        pv = [pred[k] for k in colloids_in_vision(pos[i], None, pos[pred], vision_range=r_pred,
                                                  cone=False)] if pred else []
        fa, fr = np.zeros(3), np.zeros(3)
        if vis:
            fa = np.sum(vel[vis] - vel[i], axis=0)
            fr = np.sum(pos[vis] - pos[i], axis=0) / np.linalg.norm(pos[vis] - pos[i])
        fh = home - pos[i]
        fp = np.zeros(3)
        if pv:
            fp = np.sum(pos[i] - pos[pv], axis=0) / np.linalg.norm(pos[i] - pos[pv])
        ff = -vel[i] * (np.abs(vel[i]) - speed) / speed
        F = K["K_a"] * fa + K["K_r"] * fr + K["K_h"] * fh + K["K_p"] * fp + K["K_f"] * ff
        out.append((np.linalg.norm(F), F / np.linalg.norm(F)))
    return out
