"""Ablation timings of the integration window (GPU): kT on/off, WCA on/off,
env counts; prints window time and fallback statistics."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from gpu_harness import Harness, species_list  # noqa: E402
from oracle import oracle  # noqa: E402


def disc_states(rng, n, L, E):
    out = []
    for _ in range(E):
        r = L / 2 * np.sqrt(rng.random(n))
        th = 2 * np.pi * rng.random(n)
        pos = np.stack([L / 2 + r * np.cos(th), L / 2 + r * np.sin(th), np.zeros(n)], 1)
        a = 2 * np.pi * rng.random(n)
        out.append(oracle.state_from_positions(pos, np.stack([np.cos(a), np.sin(a), 0 * a], 1),
                                               [L, L, L]))
    return out


def run(E, kT, eps, label, reps=20, force=10.0):
    torch.cuda.set_device(0)
    n = 4096
    L = 2 * np.sqrt(n / 0.1)
    rng = np.random.default_rng(1)
    h = Harness([L, L, L], 1e-3, kT, eps, 42, species_list()[:1], np.zeros(n, int), n_envs=E)
    h.upload(disc_states(rng, n, L, E))
    h.sd(1000)
    f = rng.choice([0.0, force], E * n).astype(np.float32)
    t = rng.choice([-10.0, 0.0, 10.0], E * n).astype(np.float32)
    h.set_actions(f, t)
    h.integrate(100)
    torch.cuda.synchronize()
    fb_total = 0
    t0 = time.perf_counter()
    for _ in range(reps):
        h.integrate(100)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    from swarmrl_amd import _capi
    import ctypes
    fb = np.zeros(E, np.int32)
    w = np.zeros(E, np.int32)
    _capi.check(h.native._lib.swarm_engine_window_stats(h.native.ptr, fb.ctypes.data, w.ctypes.data))
    print(f"{label:28s} E={E:4d} window {dt*1e3:8.3f} ms  fallback_last={int((fb>0).sum())} "
          f"waves/env mean {w.mean():.1f} max {w.max()}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # e.g. "64,1" -> E=64 with noise; "256,0" -> kT=0
        import os
        for spec in sys.argv[1:]:  # "E,noisy[,table]" with table 0/1 (default: auto)
            parts = spec.split(",")
            E, noisy = int(parts[0]), int(parts[1])
            if len(parts) > 2:
                os.environ["SWARMRL_AMD_NOISE_TABLE"] = parts[2]
            else:
                os.environ.pop("SWARMRL_AMD_NOISE_TABLE", None)
            run(E, 1.0239 if noisy else 0.0, 1.0239,
                f"kT{'>' if noisy else '='}0, WCA, table={parts[2] if len(parts) > 2 else 'auto'}")
        sys.exit(0)
    for E in [1, 64, 256]:
        run(E, 1.0239, 1.0239, "kT>0, WCA")
        run(E, 0.0, 1.0239, "kT=0, WCA")
        run(E, 1.0239, 0.0, "kT>0, no WCA")
