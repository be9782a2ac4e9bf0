"""Cost of an exact re-run on the global path (k_check after a failed
cluster window): 4096 colloids, swimmers fast enough (f = 400) that every
window fails the decomposition check.  Prints the window time."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
sys.path.insert(0, "tests")
from bench_states import disc_states  # noqa: E402
from gpu_harness import Harness, species_list  # noqa: E402

torch.cuda.set_device(0)
n = 4096
L = 2 * np.sqrt(n / 0.1)
rng = np.random.default_rng(1)
h = Harness([L, L, L], 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int))
h.upload(disc_states(rng, n, L, 1))
t0 = time.perf_counter()
h.sd(1000)
torch.cuda.synchronize()
print(f"overlap removal, 1000 SD steps: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
for force in (10.0, 400.0):
    h.set_actions(np.full(n, force, np.float32), np.zeros(n, np.float32))
    h.integrate(100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        h.integrate(100)
    torch.cuda.synchronize()
    fb = np.zeros(1, np.int32)
    h.native.call("swarm_engine_window_stats", fb.ctypes.data, None)
    print(f"f={force:5.0f}: window {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms "
          f"(last window fallback code {fb[0]})", flush=True)
out = np.zeros(32, np.uint64)
h.native.call("swarm_engine_debug_phases", out.ctypes.data)
if out[26]:
    print(f"global path (PHASE_TIMING build): cycles/sub-step sort {int(out[24]) // int(out[26])} "
          f"forces+step {int(out[25]) // int(out[26])}", flush=True)
