"""
Device trajectory recording (espresso.py:1110-1159): the engine records each
write point into a host-pinned ring from the engine stream, so writes can sit
inside a captured episode graph (bench.py runs the reference's 1 s write
interval this way).  The ring's entries equal the host path's
(download-and-append, SWARMRL_AMD_DEVICE_TRAJ=0) bit for bit, eagerly and
under graph replay.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


def _engine(tmp_path, tag, n=600, write_slices=2, chunk=3):
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.units import UnitRegistry

    ureg = UnitRegistry()
    L = 2 * np.sqrt(n / 0.1)
    p = MDParams(ureg=ureg, box_length=ureg.Quantity([L, L, L], "micrometer"),
                 time_step=ureg.Quantity(1e-3, "second"),
                 time_slice=ureg.Quantity(0.1, "second"),
                 write_interval=ureg.Quantity(0.1 * write_slices, "second"))
    eng = SwarmEngine(p, n_dims=2, seed=13, out_folder=tmp_path / tag, write_chunk_size=chunk)
    eng.add_colloids(n, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([L / 2, L / 2, 0.0]), "micrometer"),
                     ureg.Quantity(L / 2, "micrometer"))
    return eng


def _ff():
    from swarmrl_amd.agents import dummy_models
    from swarmrl_amd.force_functions import ForceFunction

    return ForceFunction({"0": dummy_models.ConstForceAndTorque(4.0, np.array([0, 0, 2.0]))})


def _read(eng):
    from swarmrl_amd.engine.trajectory_writer import read_trajectory

    return read_trajectory(eng.h5_filename)


def _same(a, b):
    assert a["Times"].shape == b["Times"].shape, (a["Times"].shape, b["Times"].shape)
    np.testing.assert_allclose(a["Times"], b["Times"], rtol=1e-12, atol=1e-12)
    for k in ("Ids", "Types", "Unwrapped_Positions", "Velocities", "Directors"):
        assert np.array_equal(a[k], b[k]), k


def test_ring_equals_host_path_eager(tmp_path, monkeypatch):
    ring = _engine(tmp_path, "ring")
    ring.integrate(7, _ff())
    assert ring._ring is not None
    assert len(ring.traj_holder["Times"]) == 1  # 4 writes, one chunk of 3 on disk
    ring.finalize()
    monkeypatch.setenv("SWARMRL_AMD_DEVICE_TRAJ", "0")
    host = _engine(tmp_path, "host")
    host.integrate(7, _ff())
    assert host._ring is None
    host.finalize()
    a, b = _read(ring), _read(host)
    assert a["Times"].shape[0] == 4
    _same(a, b)


def test_ring_records_inside_captured_episode(tmp_path, monkeypatch):
    """Capture integrate(4) (two write points) as bench.py does, replay it
    three times, drain without blocking between replays: the entries equal
    an eager host-path run of the same slices."""
    eng = _engine(tmp_path, "graph", chunk=100)
    ff = _ff()
    eng.integrate(1, ff)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            eng.integrate(1, ff)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eng.integrate(4, ff)
    assert len(eng.traj_holder["Times"]) == 2  # steps 0 and 200, eager
    for _ in range(3):
        g.replay()
        eng.drain_trajectory(block=False)
    eng.finalize()
    got = _read(eng)
    assert got["Times"].shape[0] == 8
    monkeypatch.setenv("SWARMRL_AMD_DEVICE_TRAJ", "0")
    host = _engine(tmp_path, "host2", chunk=100)
    ffh = _ff()
    host.integrate(3, ffh)
    host.integrate(12, ffh)
    host.finalize()
    _same(got, _read(host))
    np.testing.assert_allclose(got["Times"][:, 0, 0], 0.2 * np.arange(8), atol=1e-9)


def test_ring_overflow_is_reported(tmp_path):
    eng = _engine(tmp_path, "ovf", write_slices=1, chunk=2)
    ff = _ff()
    eng.integrate(1, ff)
    cap = eng._ring["cap"]
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        eng.integrate(1, ff)
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(g):
        eng.integrate(1, ff)
    for _ in range(cap + 2):
        g.replay()
    with pytest.raises(RuntimeError, match="overflow"):
        eng.drain_trajectory(block=True)
