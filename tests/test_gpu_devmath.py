"""Device arithmetic (swarm_device.cuh) is bit-identical to the host's:
correctly rounded sqrt, the fixed-sequence log/acos/sincos polynomials and
the Philox/Box-Muller normals."""

import ctypes
import math

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(x, a):
    import torch  # noqa: F401  (HIP runtime first)

    lib_path = ROOT / "tests" / "csrc" / "libdevmath.so"
    if not lib_path.exists():
        import __graft_entry__ as g

        g.build()
    lib = ctypes.CDLL(str(lib_path))
    n = len(x)
    out = np.zeros(9 * n + 30 * min(n, 4096), np.float32)
    rc = lib.devmath_selftest(x.ctypes.data_as(ctypes.c_void_p), a.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_int(n), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


def test_device_math_bit_exact(oracle_mod):
    rng = np.random.default_rng(0)
    n = 1 << 18
    # sqrt over many binades, including tiny values
    x = np.concatenate([
        rng.random(n // 2).astype(np.float32),
        (10.0 ** rng.uniform(-35, 30, n // 2)).astype(np.float32),
    ])
    x = np.clip(x, np.float32(1e-37), None).astype(np.float32)
    a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    out = _run(x, a)
    o_sqrt, o_log, o_acos = out[:n], out[n:2 * n], out[2 * n:3 * n]
    o_sin, o_cos = out[3 * n:4 * n], out[4 * n:5 * n]
    g = out[5 * n:8 * n].reshape(n, 3)
    o_sqrtp = out[8 * n:9 * n]
    steps = out[9 * n:].reshape(-1, 30)
    assert np.array_equal(o_sqrt, np.sqrt(x))  # numpy sqrt is IEEE correctly rounded
    xp = (np.float32(1.1920929e-07) + x * np.float32(40.0)).astype(np.float32)
    bm = xp < np.float32(41.0)  # the radius range sqrt_pos serves (x < 1 part)
    assert np.array_equal(o_sqrtp[bm], np.sqrt(xp[bm]))
    sub = np.arange(0, n, 97)
    for i in sub[:3000]:
        if x[i] < 1.0:
            assert o_log[i] == np.float32(oracle_mod.logf(float(x[i]))), i
            assert o_acos[i] == np.float32(oracle_mod.acosf(float(x[i] * np.float32(2) - np.float32(1)))), i
        s, c = oracle_mod.sincos_turn(int(a[i]))
        assert o_sin[i] == np.float32(s) and o_cos[i] == np.float32(c), i
        assert np.array_equal(g[i], oracle_mod.normals3(42, 0, int(i), 7, 0)), i
    assert math.isfinite(float(o_log[0]))
    # grouped step normals (StepNoise): sub-steps carried across a group and
    # started at every alignment equal the oracle's from-scratch restatement
    for i in list(range(0, 64 * 8, 9)) + list(range(4000, 4096, 7)):
        t0 = 1000 + i // 64
        for s_ in range(9):
            ref = oracle_mod.step_normals(42, 5, i % 64, t0 + s_)
            assert np.array_equal(steps[i, 3 * s_:3 * s_ + 3], ref), (i, s_)
        assert np.array_equal(steps[i, 27:30], oracle_mod.step_normals(42, 5, i % 64, t0 + 8))


def _lib():
    import torch  # noqa: F401  (HIP runtime first)

    lib_path = ROOT / "tests" / "csrc" / "libdevmath.so"
    if not lib_path.exists():
        import __graft_entry__ as g

        g.build()
    return ctypes.CDLL(str(lib_path))


def test_rcp_rn_exhaustive():
    """rcp_rn (the run kernels' 1/r^2, swarm_device.cuh) equals the IEEE
    division 1.0f / x for EVERY float in [2^-96, 2^96] -- the range the
    engine admits for in-range squared pair distances (box >= 2^-16, radii
    < 2^40; swarm_engine_create rejects the rest)."""
    lib = _lib()
    bad = ctypes.c_ulonglong(0)
    first = ctypes.c_uint32(0)
    lo, hi = 31 << 23, 223 << 23  # 2^-96 .. 2^96
    rc = lib.devmath_rcp_check(ctypes.c_uint32(lo), ctypes.c_uint32(hi), ctypes.byref(bad),
                               ctypes.byref(first))
    assert rc == 0
    assert bad.value == 0, (bad.value, hex(first.value))


def test_i64_to_f32_paths():
    """The int32 fast path and the fp64 wide path of the force-sum
    conversion both round to nearest (numpy's int64 -> float32 cast)."""
    lib = _lib()
    rng = np.random.default_rng(3)
    n = 1 << 16
    small = rng.integers(-2**31, 2**31, n // 2, dtype=np.int64)
    wide = rng.integers(-2**62, 2**62, n // 2, dtype=np.int64) >> rng.integers(0, 40, n // 2)
    for v in (small, np.concatenate([small, wide])):
        v = np.ascontiguousarray(v)
        out = np.zeros(3 * len(v), np.float32)
        rc = lib.devmath_i64_to_f32(v.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(len(v)),
                                    out.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0
        ref = v.astype(np.float32)
        assert np.array_equal(out[0::3], ref)
        assert np.array_equal(out[1::3], np.roll(ref, -1))
        assert np.array_equal(out[2::3], ref)


def test_f2i32_sat_rounds_and_saturates():
    """f2i32_sat (the 2-D translation's fp32 -> int32, round 6) rounds to
    nearest even and saturates to the int32 range, NaN -> 0: the oracle's
    f2i32_sat (oracle/swarm_oracle.c) on halves, the range edges and
    beyond, infinities and NaN."""
    lib_path = ROOT / "tests" / "csrc" / "libdevmath.so"
    import torch  # noqa: F401  (HIP runtime first)

    lib = ctypes.CDLL(str(lib_path))
    rng = np.random.default_rng(5)
    v = np.concatenate([
        np.array([0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 0.0, -0.0, 2147483520.0, 2147483648.0,
                  -2147483648.0, -2147483904.0, 3.0e9, -3.0e9, 1e30, -1e30, np.inf, -np.inf,
                  np.nan], np.float32),
        (rng.standard_normal(1 << 16) * 10.0 ** rng.uniform(-3, 10, 1 << 16)).astype(np.float32),
    ])
    v = np.ascontiguousarray(v)
    out = np.zeros(len(v), np.int32)
    rc = lib.devmath_f2i32_sat(v.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(len(v)),
                               out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    r = np.rint(v.astype(np.float64))
    want = np.where(np.isnan(r), 0, np.clip(np.nan_to_num(r, posinf=2**31, neginf=-2**31),
                                            -2**31, 2**31 - 1)).astype(np.int64)
    assert np.array_equal(out.astype(np.int64), want)
