"""
Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py from
the seeded oracle): the CPU oracle must keep reproducing them bit for bit
(guards the restatement against drift between rounds), and the HIP engine
must reproduce them bit for bit on the GPU.
"""

import pathlib

import numpy as np
import pytest

from oracle import oracle

G = pathlib.Path(__file__).resolve().parent / "golden"
SPECIES = [(1.0, 4.6595, 6.2126, 1.0358e-6, 4.143e-7), (0.7, 3.2617, 2.1309, 3.55e-7, 7.0e-8)]


def _load(name):
    with np.load(G / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_oracle_reproduces_bd2d_golden():
    z = _load("bd2d_wca.npz")
    p = oracle.make_params(z["box"], 1e-3, 1.0239, 1.0239, int(z["seed"]), SPECIES)
    st = {"q": z["q0"], "img": z["img0"], "ang": z["ang0"]}
    st, _ = oracle.sd_run(p, st, z["species"], int(z["sd_steps"]))
    st, vel, om = oracle.bd_run(p, st, z["species"], z["f_swim"], z["torque_z"],
                                int(z["bd_steps"]))
    for k in ("q", "img", "ang"):
        assert np.array_equal(st[k], z[k]), k
    assert np.array_equal(vel, z["vel"]) and np.array_equal(om, z["omega"])


def test_oracle_reproduces_bd3d_golden():
    z = _load("bd3d_wca.npz")
    p = oracle.make_params(z["box"], 1e-3, 1.0239, 1.0239, int(z["seed"]), SPECIES[:1], n_dims=3)
    st = {"q": z["q0"], "img": z["img0"], "dir": z["dir0"], "ang": np.zeros(len(z["species"]),
                                                                               np.uint32)}
    st, _ = oracle.sd_run3(p, st, z["species"], int(z["sd_steps"]))
    st, vel, om = oracle.bd_run3(p, st, z["species"], z["f_swim"], z["torque"],
                                 int(z["bd_steps"]))
    for k in ("q", "img", "dir"):
        assert np.array_equal(st[k], z[k]), k
    assert np.array_equal(vel, z["vel"]) and np.array_equal(om, z["omega"])


def test_oracle_reproduces_vision_golden():
    z = _load("vision_cone.npz")
    p = oracle.make_params(z["box"], 1e-3, 0.0, 1.0, 0, SPECIES[:1])
    st = {"q": z["q"], "img": z["img"], "ang": z["ang"]}
    out = oracle.vision_cone(p, st, z["agents"], z["radii"], z["types"], float(z["vision_range"]),
                             float(z["half_angle"]), int(z["n_cones"]), list(z["detected"]))
    assert np.array_equal(out, z["out"])


@pytest.mark.gpu
def test_gpu_reproduces_golden_vectors():
    import torch

    from gpu_harness import Harness
    from swarmrl_amd import _capi
    from swarmrl_amd.engine import ops

    _capi.require_gpu()
    torch.cuda.set_device(0)
    z = _load("bd2d_wca.npz")
    h = Harness(list(z["box"]), 1e-3, 1.0239, 1.0239, int(z["seed"]), SPECIES,
                z["species"].astype(int))
    h.upload([{"q": z["q0"], "img": z["img0"], "ang": z["ang0"]}])
    h.sd(int(z["sd_steps"]))
    h.set_actions(z["f_swim"], z["torque_z"])
    h.integrate(int(z["bd_steps"]))
    got = h.download()[0]
    for k in ("q", "img", "ang"):
        assert np.array_equal(got[k], z[k]), k
    assert np.array_equal(h.velocities(), z["vel"])

    z = _load("bd3d_wca.npz")
    n = len(z["species"])
    h = Harness(list(z["box"]), 1e-3, 1.0239, 1.0239, int(z["seed"]), SPECIES[:1],
                z["species"].astype(int), n_dims=3)
    h.upload([{"q": z["q0"], "img": z["img0"], "dir": z["dir0"], "ang": np.zeros(n, np.uint32)}])
    h.sd(int(z["sd_steps"]))
    h.set_actions(z["f_swim"], z["torque"][2])
    h.set_torque_xy(z["torque"][:2])
    h.integrate(int(z["bd_steps"]))
    got = h.download()[0]
    for k in ("q", "img", "dir"):
        assert np.array_equal(got[k], z[k]), k
    assert np.array_equal(h.omegas3(), z["omega"])

    z = _load("vision_cone.npz")
    n = len(z["types"])
    h = Harness(list(z["box"]), 1e-3, 0.0, 1.0, 0, SPECIES[:1], np.zeros(n, int))
    h.upload([{"q": z["q"], "img": z["img"], "ang": z["ang"]}])
    dev = torch.device("cuda", 0)
    vp = ops.vision_params(float(z["vision_range"]), float(z["half_angle"]), int(z["n_cones"]),
                           list(z["detected"]))
    out = ops.vision_cone(h.native, 1, torch.as_tensor(z["agents"], device=dev),
                          torch.as_tensor(z["radii"], device=dev),
                          torch.as_tensor(z["types"], device=dev), vp)
    assert np.array_equal(out.cpu().numpy()[0], z["out"])
