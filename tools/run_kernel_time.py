"""Average k_cluster_run duration (engine HIP events, swarm_engine_profile)
on the bench-like window: 4096 colloids per env, area fraction 0.1, kT > 0.
Usage: [SWARMRL_AMD_LIB=<variant .so>] python tools/run_kernel_time.py E [E ...]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
sys.path.insert(0, "tests")
from bench_states import disc_states  # noqa: E402
from gpu_harness import Harness, species_list  # noqa: E402


def main():
    torch.cuda.set_device(0)
    n = 4096
    L = 2 * np.sqrt(n / 0.1)
    for E in [int(a) for a in sys.argv[1:]] or [1, 64]:
        rng = np.random.default_rng(1)
        h = Harness([L, L, L], 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int),
                    n_envs=E)
        h.upload(disc_states(rng, n, L, E))
        h.sd(1000)
        h.set_actions(rng.choice([0.0, 10.0], E * n).astype(np.float32),
                      rng.choice([-10.0, 0.0, 10.0], E * n).astype(np.float32))
        h.integrate(100)
        torch.cuda.synchronize()
        ms, cnt = ctypes.c_double(), ctypes.c_int32()
        h.native.call("swarm_engine_profile", 1, ctypes.byref(ms), ctypes.byref(cnt))
        for _ in range(30):
            h.integrate(100)
        torch.cuda.synchronize()
        h.native.call("swarm_engine_profile", 0, ctypes.byref(ms), ctypes.byref(cnt))
        line = f"E={E:3d} k_cluster_run {1e3 * ms.value / max(cnt.value, 1):7.2f} us ({cnt.value})"
        out = np.zeros(32, np.uint64)
        try:
            h.native.call("swarm_engine_debug_phases", out.ctypes.data)
        except Exception:  # noqa: BLE001 - only the PHASE_TIMING variant fills it
            pass
        if out[19]:
            ns = int(out[19])
            line += (f"  cycles/sub-step: pairs {int(out[16]) // ns} read-back "
                     f"{int(out[17]) // ns} bd {int(out[18]) // ns} (npass {int(out[20])})")
        print(line, flush=True)


if __name__ == "__main__":
    main()
