"""
Generate the golden vectors in tests/golden/ from the CPU oracle (seeded).

The reference itself cannot run here (jax, ESPResSo absent),
so these vectors pin the oracle restatement against drift between rounds:
tests/test_golden.py checks the oracle reproduces them bit for bit on the
CPU, and the HIP engine on the GPU.  Inputs and outputs only (no reference
source).  Run:  python tests/golden/make_golden.py
"""

import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle  # noqa: E402

OUT = pathlib.Path(__file__).resolve().parent
SPECIES = [(1.0, 4.6595, 6.2126, 1.0358e-6, 4.143e-7), (0.7, 3.2617, 2.1309, 3.55e-7, 7.0e-8)]


def bd2d():
    rng = np.random.default_rng(2024)
    n, L = 400, 60.0
    box = [L, L, L]
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * L
    a = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    sp = rng.integers(0, 2, n).astype(np.uint8)
    f = rng.choice([0.0, 10.0], n).astype(np.float32)
    t = rng.choice([-10.0, 0.0, 10.0], n).astype(np.float32)
    p = oracle.make_params(box, 1e-3, 1.0239, 1.0239, 77, SPECIES)
    st0 = oracle.state_from_positions(pos, dirs, box)
    st1, _ = oracle.sd_run(p, st0, sp, 200)
    st2, vel, om = oracle.bd_run(p, st1, sp, f, t, 100, step0=0)
    np.savez_compressed(OUT / "bd2d_wca.npz", box=np.array(box), seed=77, species=sp,
                        f_swim=f, torque_z=t, q0=st0["q"], img0=st0["img"], ang0=st0["ang"],
                        sd_steps=200, bd_steps=100, q=st2["q"], img=st2["img"], ang=st2["ang"],
                        vel=vel, omega=om)


def bd3d():
    rng = np.random.default_rng(2025)
    n, L = 300, 18.0
    box = [L, L, L]
    pos = rng.random((n, 3)) * L
    dirs = rng.normal(size=(n, 3))
    sp = np.zeros(n, np.uint8)
    f = rng.choice([0.0, 10.0], n).astype(np.float32)
    tq = rng.normal(scale=5.0, size=(3, n)).astype(np.float32)
    p = oracle.make_params(box, 1e-3, 1.0239, 1.0239, 78, SPECIES[:1], n_dims=3)
    st0 = oracle.state3_from_positions(pos, dirs, box)
    st1, _ = oracle.sd_run3(p, st0, sp, 100)
    st2, vel, om = oracle.bd_run3(p, st1, sp, f, tq, 100)
    np.savez_compressed(OUT / "bd3d_wca.npz", box=np.array(box), seed=78, species=sp,
                        f_swim=f, torque=tq, q0=st0["q"], img0=st0["img"], dir0=st0["dir"],
                        sd_steps=100, bd_steps=100, q=st2["q"], img=st2["img"], dir=st2["dir"],
                        vel=vel, omega=om)


def vision():
    rng = np.random.default_rng(2026)
    n, L = 500, 80.0
    box = [L, L, L]
    pos = np.zeros((n, 3))
    pos[:, :2] = rng.random((n, 2)) * L
    # mixed image counters (the reference compares UNWRAPPED positions with
    # no minimum image, subdivided_vision_cones.py:116-121): half of the
    # colloids move to a neighbouring image, so folded-box neighbours in
    # different images are invisible and colloids across a box edge in
    # adjacent images are seen
    moved = rng.random(n) < 0.5
    pos[moved, :2] += rng.integers(-1, 2, (int(moved.sum()), 2)) * L
    a = rng.random(n) * 2 * np.pi
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    types = rng.integers(0, 3, n).astype(np.int32)
    radii = (0.5 + rng.random(n)).astype(np.float32)
    agents = np.nonzero(types == 1)[0].astype(np.int32)
    p = oracle.make_params(box, 1e-3, 0.0, 1.0, 0, SPECIES[:1])
    st = oracle.state_from_positions(pos, dirs, box)
    out = oracle.vision_cone(p, st, agents, radii, types, 10.0, 1.3, 5, [0, 1, 2])
    np.savez_compressed(OUT / "vision_cone.npz", box=np.array(box), q=st["q"], img=st["img"],
                        ang=st["ang"], types=types, radii=radii, agents=agents,
                        vision_range=10.0, half_angle=1.3, n_cones=5,
                        detected=np.array([0, 1, 2]), out=out)


if __name__ == "__main__":
    oracle.build()
    bd2d()
    bd3d()
    vision()
    print("golden vectors written to", OUT)
