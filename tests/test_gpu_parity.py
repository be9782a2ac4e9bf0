"""
GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the
same seeded inputs.  Integer/index results must be bit-exact; with the shared
number formats the fp32 dynamics are bit-exact as well.
"""

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from swarmrl_amd import _capi

    _capi.require_gpu()
    torch.cuda.set_device(0)


def _eq(a, b):
    for k in ("q", "img", "ang"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("table", ["0", "1"])
def test_bd_parity_dilute_multi_chunk(table, monkeypatch):
    """Both noise paths: normals computed in the run kernel (table=0) and
    read from the chip-wide k_noise table (table=1)."""
    from gpu_harness import Harness, random_state, species_list

    monkeypatch.setenv("SWARMRL_AMD_NOISE_TABLE", table)

    rng = np.random.default_rng(1)
    box = [120.0, 120.0, 120.0]
    n = 700
    sp = rng.integers(0, 2, n)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 42, species_list(), sp)
    st = random_state(rng, n, box)
    h.upload([st])
    step = 0
    for chunk, nsteps in enumerate([37, 1, 100]):
        f = rng.normal(size=n).astype(np.float32) * 10
        t = rng.normal(size=n).astype(np.float32) * 10
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, vel, _ = oracle.bd_run(h.op, st, sp, f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), vel)


def test_bd_parity_dense_wca_multi_env():
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(2)
    box = [40.0, 40.0, 40.0]
    n = 300  # area fraction ~0.6: many WCA contacts
    E = 3
    sp = rng.integers(0, 2, n)
    h = Harness(box, 1e-4, 1.0239, 1.0239, 7, species_list(), sp, n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    sd_states = [oracle.sd_run(h.op, s, sp, 200)[0] for s in states]
    h.upload(states)
    h.sd(200)
    got = h.download()
    for e in range(E):
        _eq(got[e], sd_states[e])
    f = np.full(n * E, 5.0, np.float32)
    t = np.zeros(n * E, np.float32)
    h.set_actions(f, t)
    h.integrate(50)
    got = h.download()
    for e in range(E):
        ref, _, _ = oracle.bd_run(h.op, sd_states[e], sp, f[:n], t[:n], 50, step0=0, env=e)
        _eq(got[e], ref)
    # the dense case really exercised pair forces: without WCA the oracle
    # trajectory differs
    import copy

    p0 = copy.copy(h.op)
    p0.wca_epsilon = 0.0
    free, _, _ = oracle.bd_run(p0, sd_states[0], sp, f[:n], t[:n], 50, step0=0, env=0)
    assert not np.array_equal(free["q"], got[0]["q"])
    assert len(oracle.neighbor_pairs(h.op, got[0], 2.0)) > 10


@pytest.mark.parametrize("E", [8, 16])
def test_bd_parity_throughput_kernel_xcd_envs(E, monkeypatch):
    """The throughput run kernel (SWARMRL_AMD_WIDE_RUN=0) at E = 8 and 16 envs:
    its XCD-aware block placement (env e on XCD e mod 8, block-major over
    each XCD's envs, blocks past an env's wave count leaving before they
    stage anything) on dilute swimmers, against the oracle env by env."""
    from gpu_harness import Harness, random_state, species_list

    monkeypatch.setenv("SWARMRL_AMD_WIDE_RUN", "0")
    rng = np.random.default_rng(11)
    n = 512
    L = float(np.sqrt(n * np.pi / 0.1))  # area fraction 0.1
    box = [L, L, L]
    sp = np.zeros(n, int)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], sp, n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    sd_states = [oracle.sd_run(h.op, s, sp, 100)[0] for s in states]
    h.upload(states)
    h.sd(100)
    f = rng.choice([0.0, 10.0], n * E).astype(np.float32)
    t = rng.choice([-10.0, 0.0, 10.0], n * E).astype(np.float32)
    h.set_actions(f, t)
    h.integrate(100)
    got = h.download()
    for e in range(E):
        ref, _, _ = oracle.bd_run(h.op, sd_states[e], sp, f[e * n:(e + 1) * n],
                                  t[e * n:(e + 1) * n], 100, step0=0, env=e)
        _eq(got[e], ref)


def test_bd_parity_kt0_deterministic():
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(3)
    box = [80.0, 80.0, 80.0]
    n = 400
    sp = np.zeros(n, int)
    h = Harness(box, 1e-3, 0.0, 1.0239, 1, species_list(), sp)
    st = random_state(rng, n, box)
    h.upload([st])
    f = rng.random(n).astype(np.float32) * 10
    t = rng.normal(size=n).astype(np.float32)
    h.set_actions(f, t)
    h.integrate(200)
    ref, vel, _ = oracle.bd_run(h.op, st, sp, f, t, 200)
    _eq(h.download()[0], ref)
    assert np.array_equal(h.velocities(), vel)


def test_step_counter_advances_noise():
    """Two 50-step runs equal one 100-step run (noise keyed by global step)."""
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(4)
    box = [100.0, 100.0, 100.0]
    n = 256
    sp = np.zeros(n, int)
    st = random_state(rng, n, box)
    a = Harness(box, 1e-3, 1.0239, 1.0239, 3, species_list(), sp)
    a.upload([st])
    a.set_actions(np.ones(n), np.zeros(n))
    a.integrate(50)
    a.integrate(50)
    b = Harness(box, 1e-3, 1.0239, 1.0239, 3, species_list(), sp)
    b.upload([st])
    b.set_actions(np.ones(n), np.zeros(n))
    b.integrate(100)
    _eq(a.download()[0], b.download()[0])


def test_neighbor_pairs_bit_exact():
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(5)
    box = [50.0, 50.0, 50.0]
    n = 900
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int))
    st = random_state(rng, n, box)
    h.upload([st])
    for cutoff in [1.0, 2.0, 3.7]:
        pairs = np.zeros((200000, 2), np.int32)
        cnt = np.zeros(1, np.int32)
        h.native.bind_stream()
        h.native.call("swarm_engine_neighbor_pairs", 0, cutoff, pairs.ctypes.data, 200000,
                      cnt.ctypes.data)
        got = {tuple(p) for p in pairs[: cnt[0]]}
        ref = {tuple(p) for p in oracle.neighbor_pairs(h.op, st, cutoff)}
        assert got == ref and len(ref) > 0


def test_vision_cone_parity_random():
    from gpu_harness import Harness, random_state, species_list
    from swarmrl_amd.engine import ops

    rng = np.random.default_rng(6)
    box = [90.0, 90.0, 90.0]
    n = 800
    E = 2
    types = rng.integers(0, 3, n)
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int), n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    h.upload(states)
    agents = np.nonzero(types == 1)[0].astype(np.int32)
    radii = (0.5 + rng.random(n)).astype(np.float32)
    dev = torch.device("cuda", 0)
    vp = ops.vision_params(10.0, 1.3, 5, [0, 1, 2])
    out = ops.vision_cone(h.native, E, torch.as_tensor(agents, device=dev),
                          torch.as_tensor(radii, device=dev),
                          torch.as_tensor(types.astype(np.int32), device=dev), vp)
    out = out.cpu().numpy()
    for e in range(E):
        ref = oracle.vision_cone(h.op, states[e], agents, radii, types, 10.0, 1.3, 5, [0, 1, 2])
        assert np.array_equal(out[e], ref)
        assert np.count_nonzero(ref) > 100


def test_field_distance_parity():
    from gpu_harness import Harness, random_state, species_list
    from swarmrl_amd.engine import ops

    rng = np.random.default_rng(7)
    box = [400.0, 400.0, 400.0]
    n = 1000
    E = 2
    h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list(), np.zeros(n, int), n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    h.upload(states)
    agents = np.arange(0, n, 3, dtype=np.int32)
    A = len(agents)
    dev = torch.device("cuda", 0)
    ag_t = torch.as_tensor(agents, device=dev)
    hq = torch.zeros((3, E * A), dtype=torch.int32, device=dev)
    hi = torch.zeros((3, E * A), dtype=torch.int32, device=dev)
    src = np.array([200.0, 200.0, 0.0])
    scale = np.array([400.0, 400.0, 400.0])
    ops.field_distance(h.native, E, ag_t, src, scale, hq, hi, update=True, init_only=True)
    hists = [oracle.history_from_state(s, agents) for s in states]
    h.set_actions(np.full(E * n, 10.0), np.zeros(E * n))
    h.integrate(100)
    d_cur, d_prev = ops.field_distance(h.native, E, ag_t, src, scale, hq, hi, update=True)
    got = h.download()
    for e in range(E):
        rc, rp = oracle.field_distance(h.op, got[e], agents, src, scale, hists[e])
        assert np.array_equal(d_cur[e].cpu().numpy(), rc)
        assert np.array_equal(d_prev[e].cpu().numpy(), rp)
    hq_host = hq.cpu().numpy().view(np.uint32).reshape(3, E, A)
    for e in range(E):
        assert np.array_equal(hq_host[:, e], hists[e]["q"])


@pytest.mark.parametrize("table,wide,env_build", [
    ("0", "0", "0"),  # normals drawn in the run kernel
    ("1", "0", "0"),  # k_noise table, 256-thread run blocks
    ("1", "1", "0"),  # default latency-bound path: wide run, next table beside the run
    ("1", "1", "1"),  # ... with the one-launch LDS build (k_build_env)
])
def test_full_size_4096_slice_bit_exact(table, wide, env_build, monkeypatch):
    """BASELINE workload size: 4096 colloids, windows of 100, 37 and 100
    sub-steps (the second and third read noise tables filled beside the
    previous run), vs the oracle, for every run/noise/build variant."""
    monkeypatch.setenv("SWARMRL_AMD_NOISE_TABLE", table)
    monkeypatch.setenv("SWARMRL_AMD_WIDE_RUN", wide)
    monkeypatch.setenv("SWARMRL_AMD_ENV_BUILD", env_build)
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(8)
    n = 4096
    L = 2 * np.sqrt(n * 1.0 / 0.1)
    box = [L, L, L]
    pos, dirs = _disc(rng, n, L)
    st = oracle.state_from_positions(pos, dirs, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int))
    h.upload([st])
    h.sd(1000)
    st, _ = oracle.sd_run(h.op, st, np.zeros(n), 1000)
    _eq(h.download()[0], st)
    step = 0
    for nsteps in (100, 37, 100):
        f = rng.choice([0.0, 10.0], n).astype(np.float32)
        t = rng.choice([-10.0, 0.0, 10.0], n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, vel, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), vel)


def _disc(rng, n, L):
    r = L / 2 * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    pos = np.stack([L / 2 + r * np.cos(th), L / 2 + r * np.sin(th), np.zeros(n)], 1)
    a = 2 * np.pi * rng.random(n)
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    return pos, dirs


@pytest.mark.parametrize("env_build", ["0", "1"])
@pytest.mark.parametrize("force", [40.0, 400.0])
def test_fast_swimmers_cross_skin_bit_exact(force, env_build, monkeypatch):
    """Swimmers faster than skin / window exercise the decomposition check and
    the global-path re-run; results must stay bit-exact.  env_build = "1":
    the one-launch LDS build (k_build_env), whose cell-sorted snapshot the
    check's cell-based exact test reads from global memory."""
    from gpu_harness import Harness, random_state, species_list

    monkeypatch.setenv("SWARMRL_AMD_ENV_BUILD", env_build)

    rng = np.random.default_rng(9)
    box = [150.0, 150.0, 150.0]
    n = 1500
    E = 2
    sp = np.zeros(n, int)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 11, species_list()[:1], sp, n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    states = [oracle.sd_run(h.op, s, sp, 300)[0] for s in states]
    h.upload(states)
    f = np.full(E * n, force, np.float32)
    t = rng.normal(size=E * n).astype(np.float32) * 5
    h.set_actions(f, t)
    for _ in range(2):
        h.integrate(100)
    got = h.download()
    for e in range(E):
        ref = states[e]
        for k in range(2):
            ref, _, _ = oracle.bd_run(h.op, ref, sp, f[e * n:(e + 1) * n], t[e * n:(e + 1) * n],
                                      100, step0=100 * k, env=e)
        _eq(got[e], ref)


def test_long_run_is_windowed_bit_exact():
    """integrate(n) longer than one window (128 sub-steps) splits into windows."""
    from gpu_harness import Harness, random_state, species_list

    rng = np.random.default_rng(10)
    box = [100.0, 100.0, 100.0]
    n = 800
    sp = np.zeros(n, int)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 12, species_list()[:1], sp)
    st = oracle.sd_run(h.op, random_state(rng, n, box), sp, 300)[0]
    h.upload([st])
    f = np.full(n, 10.0, np.float32)
    t = np.zeros(n, np.float32)
    h.set_actions(f, t)
    h.integrate(300)
    ref, _, _ = oracle.bd_run(h.op, st, sp, f, t, 300)
    _eq(h.download()[0], ref)


@pytest.mark.parametrize("hint", [100, 37])
def test_prebuild_on_side_stream_bit_exact(hint):
    """swarm_engine_prebuild on a side stream, joined before integrate, gives
    the oracle trajectory; a hint shorter than the window makes integrate top
    up the noise table; an upload after a prebuild discards it."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(21)
    n = 2048
    L = 2 * np.sqrt(n / 0.1)
    box = [L, L, L]
    pos, dirs = _disc(rng, n, L)
    st = oracle.state_from_positions(pos, dirs, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], np.zeros(n, int))
    h.upload([st])
    h.sd(300)
    st, _ = oracle.sd_run(h.op, st, np.zeros(n), 300)
    f = rng.choice([0.0, 10.0], n).astype(np.float32)
    t = rng.choice([-10.0, 0.0, 10.0], n).astype(np.float32)
    side, side2 = torch.cuda.Stream(), torch.cuda.Stream()
    step = 0
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream())
        side2.wait_stream(torch.cuda.current_stream())
        h.prebuild(hint, side, side2)
        h.set_actions(f, t)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.current_stream().wait_stream(side2)
        h.integrate(100)
        st, _, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, 100, step0=step)
        step += 100
        _eq(h.download()[0], st)
    # prebuild from the current positions, then replace them: must not be used
    h.prebuild(hint)
    pos2, dirs2 = _disc(rng, n, L)
    st2 = oracle.state_from_positions(pos2, dirs2, box)
    h.upload([st2])
    h.sd(300)  # steepest descent sees the swim forces / torques set above
    st2, _ = oracle.sd_run(h.op, st2, np.zeros(n), 300, f_swim=f, torque_z=t)
    h.integrate(100)
    st2, _, _ = oracle.bd_run(h.op, st2, np.zeros(n), f, t, 100, step0=step)
    _eq(h.download()[0], st2)


def test_c5_16384_large_build_bit_exact():
    """C5 size (16 384 colloids): the large-N cluster build (cluster arrays in
    global memory) integrates a slice bit-exactly and without fallback."""
    import ctypes

    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(16)
    n = 16384
    L = 2 * np.sqrt(n / 0.1)
    box = [L, L, L]
    pos, dirs = _disc(rng, n, L)
    st = oracle.state_from_positions(pos, dirs, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 3, species_list()[:1], np.zeros(n, int))
    h.upload([st])
    h.sd(300)
    st, _ = oracle.sd_run(h.op, st, np.zeros(n), 300)
    f = rng.choice([0.0, 10.0], n).astype(np.float32)
    t = rng.choice([-10.0, 0.0, 10.0], n).astype(np.float32)
    h.set_actions(f, t)
    h.integrate(100)
    ref, _, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, 100)
    _eq(h.download()[0], ref)
    fb = np.zeros(1, np.int32)
    w = np.zeros(1, np.int32)
    h.native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
    assert fb[0] == 0 and w[0] > 0, (fb, w)


@pytest.mark.parametrize("E,n,box_len,env", [
    (1, 2000, 90.0, {}),                                   # 16 lanes per agent
    (20, 4096, 200.0, {"SWARMRL_AMD_VISION_G": "4"}),
    (20, 4096, 200.0, {}),                                 # 16 lanes per agent
    (64, 4096, 160.0, {"SWARMRL_AMD_VISION_G": "16"}),
    (64, 4096, 160.0, {}),                                 # 4 lanes per agent
])
def test_vision_cone_parity_lane_variants_and_dense(E, n, box_len, env, monkeypatch):
    """k_vision with 16 / 4 lanes per agent (by size, or by override), with
    dense neighbourhoods (more in-range hits per lane than its LDS hit list
    holds, so the list is drained mid-scan), bit-exact against the oracle on
    the first and last env."""
    from gpu_harness import Harness, random_state, species_list
    from swarmrl_amd.engine import ops

    for k, v in env.items():
        monkeypatch.setenv(k, v)

    rng = np.random.default_rng(60 + E)
    box = [box_len, box_len, box_len]
    types = rng.integers(0, 2, n)
    h = Harness(box, 1e-3, 0.0, 1.0, 0, species_list(), np.zeros(n, int), n_envs=E)
    states = [random_state(rng, n, box) for _ in range(E)]
    h.upload(states)
    agents = np.nonzero(types == 1)[0].astype(np.int32)
    radii = (0.5 + rng.random(n)).astype(np.float32)
    dev = torch.device("cuda", 0)
    vp = ops.vision_params(12.0, 1.0, 3, [0, 1])
    out = ops.vision_cone(h.native, E, torch.as_tensor(agents, device=dev),
                          torch.as_tensor(radii, device=dev),
                          torch.as_tensor(types.astype(np.int32), device=dev), vp)
    out = out.cpu().numpy()
    for e in sorted({0, E - 1}):
        ref = oracle.vision_cone(h.op, states[e], agents, radii, types, 12.0, 1.0, 3, [0, 1])
        assert np.array_equal(out[e], ref)
        assert np.count_nonzero(ref) > len(agents)


@pytest.mark.parametrize("wide", ["1", "0"])
def test_big_clusters_run_in_check_bit_exact(wide, monkeypatch):
    """Clusters wider than a wave (three 10 x 10 patches at 2.5 um spacing:
    100 colloids each, within r_c + skin of their neighbours) run in k_check's
    workgroup instead of sending the env to the global path, after either run
    kernel (wide = "1": k_cluster_run_wide, "0": the throughput
    k_cluster_run): bit-exact against the oracle over several windows,
    without a global-path re-run."""
    from gpu_harness import Harness, species_list

    monkeypatch.setenv("SWARMRL_AMD_WIDE_RUN", wide)

    rng = np.random.default_rng(21)
    box = [200.0, 200.0, 200.0]
    pts = []
    for cx, cy in ((40.0, 40.0), (120.0, 60.0), (80.0, 150.0)):
        for gx in range(10):
            for gy in range(10):
                pts.append((cx + 2.5 * gx, cy + 2.5 * gy))
    n_free = 700
    while len(pts) < 300 + n_free:
        p = rng.random(2) * 200.0
        if min((p[0] - q[0]) ** 2 + (p[1] - q[1]) ** 2 for q in pts) > 16.0:
            pts.append((p[0], p[1]))
    n = len(pts)
    pos = np.zeros((n, 3))
    pos[:, :2] = pts
    a = 2 * np.pi * rng.random(n)
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
    st = oracle.state_from_positions(pos, dirs, box)
    h = Harness(box, 1e-3, 1.0239, 1.0239, 5, species_list()[:1], np.zeros(n, int))
    h.upload([st])
    step = 0
    for nsteps in (100, 60):
        f = rng.choice([0.0, 5.0], n).astype(np.float32)
        t = rng.choice([-5.0, 0.0, 5.0], n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        st, vel, _ = oracle.bd_run(h.op, st, np.zeros(n), f, t, nsteps, step0=step)
        step += nsteps
        _eq(h.download()[0], st)
        assert np.array_equal(h.velocities(), vel)
        fb = np.zeros(1, np.int32)
        w = np.zeros(1, np.int32)
        h.native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
        assert fb[0] == 0 and w[0] > 0, (fb, w)


@pytest.mark.parametrize("E", [1, 2])
def test_large_build_clusters_of_every_width_bit_exact(E):
    """The multi-workgroup large-N build (k_mwb_*, 2-D envs above 4096
    colloids): 8192 colloids of two species on a jittered lattice (no pairs)
    with patches at 2.5 um spacing -- 10 x 10 (big clusters: run by k_check's
    workgroup), 6 x 6 (110 pairs: a two-pass wave), 4 x 4 and 2 x 1 --
    three windows bit-exact against the oracle on every env, no global-path
    re-run.  E = 2: one grid row per env."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(88)
    n, L, sp = 8192, 528.0, 5.5
    box = [L, L, L]
    patches = [(10, 30.0, 30.0), (10, 300.0, 100.0), (6, 150.0, 400.0), (6, 420.0, 420.0),
               (4, 60.0, 250.0), (4, 250.0, 250.0), (2, 480.0, 40.0)]
    pts = []
    for k, cx, cy in patches:
        for gx in range(k):
            for gy in range(k if k > 2 else 1):
                pts.append((cx + 2.5 * gx, cy + 2.5 * gy))
    taken = np.array(pts)
    g = int(L / sp)
    cells = [(i, j) for i in range(g) for j in range(g)]
    rng.shuffle(cells)
    for i, j in cells:
        if len(pts) >= n:
            break
        p = (sp * (i + 0.5) + rng.uniform(-0.4, 0.4), sp * (j + 0.5) + rng.uniform(-0.4, 0.4))
        if np.min(np.hypot(taken[:, 0] - p[0], taken[:, 1] - p[1])) > 8.0:
            pts.append(p)
    assert len(pts) == n
    pos = np.zeros((n, 3))
    pos[:, :2] = pts
    types = (rng.random(n) < 0.3).astype(int)
    types[:len(taken)] = 0  # the patches: radius 1 (2.5 um apart, within r_c + skin)
    states = []
    for e in range(E):
        a = 2 * np.pi * rng.random(n)
        dirs = np.stack([np.cos(a), np.sin(a), np.zeros(n)], 1)
        states.append(oracle.state_from_positions(pos, dirs, box))
    h = Harness(box, 1e-3, 1.0239, 1.0239, 7, species_list(), types, n_envs=E)
    h.upload(states)
    step = 0
    for nsteps in (100, 100, 40):
        f = rng.choice([0.0, 5.0], E * n).astype(np.float32)
        t = rng.choice([-5.0, 0.0, 5.0], E * n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        got = h.download()
        for e in range(E):
            sl = slice(e * n, (e + 1) * n)
            states[e], _, _ = oracle.bd_run(h.op, states[e], types, f[sl], t[sl], nsteps,
                                            step0=step, env=e)
            _eq(got[e], states[e])
        step += nsteps
        fb = np.zeros(E, np.int32)
        w = np.zeros(E, np.int32)
        h.native.call("swarm_engine_window_stats", fb.ctypes.data, w.ctypes.data)
        assert np.all(fb == 0) and np.all(w > 0), (fb, w)


def test_c4_size_8_envs_x_1024_bit_exact():
    """SURVEY config C4 per GPU (8 envs x 1024 colloids, area fraction 0.1):
    the latency-bound wide run with its next-window noise, three windows,
    bit-exact on every env."""
    from gpu_harness import Harness, species_list

    rng = np.random.default_rng(31)
    n, E = 1024, 8
    L = 2 * np.sqrt(n / 0.1)
    box = [L, L, L]
    states = []
    for _ in range(E):
        pos, dirs = _disc(rng, n, L)
        states.append(oracle.state_from_positions(pos, dirs, box))
    h = Harness(box, 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int), n_envs=E)
    h.upload(states)
    h.sd(500)
    states = [oracle.sd_run(h.op, s, np.zeros(n), 500)[0] for s in states]
    step = 0
    for nsteps in (100, 100, 50):
        f = rng.choice([0.0, 10.0], E * n).astype(np.float32)
        t = rng.choice([-10.0, 0.0, 10.0], E * n).astype(np.float32)
        h.set_actions(f, t)
        h.integrate(nsteps)
        got = h.download()
        for e in range(E):
            states[e], _, _ = oracle.bd_run(h.op, states[e], np.zeros(n), f[e * n:(e + 1) * n],
                                            t[e * n:(e + 1) * n], nsteps, step0=step, env=e)
            _eq(got[e], states[e])
        step += nsteps
