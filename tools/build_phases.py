"""Phase timing of k_cluster_build (needs the PHASE_TIMING variant library):
SWARMRL_AMD_LIB=tools/_variants/libswarmrl_amd_PHASE_TIMING.so python tools/build_phases.py"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from bench_states import disc_states  # noqa: E402

sys.path.insert(0, "tests")
from gpu_harness import Harness, species_list  # noqa: E402

torch.cuda.set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = 2 * np.sqrt(n / 0.1)
rng = np.random.default_rng(1)
h = Harness([L, L, L], 1e-3, 1.0239, 1.0239, 42, species_list()[:1], np.zeros(n, int))
h.upload(disc_states(rng, n, L, 1))
h.sd(1000)
h.set_actions(rng.choice([0.0, 10.0], n).astype(np.float32),
              rng.choice([-10.0, 0.0, 10.0], n).astype(np.float32))
for rep in range(5):
    h.integrate(100)
    out = np.zeros(32, np.uint64)
    h.native.call("swarm_engine_debug_phases", out.ctypes.data)
    if out[19]:
        ns = int(out[19])
        print(f"run (wave 0, npass {int(out[20])}): cycles/sub-step pairs {int(out[16]) // ns} "
              f"read-back {int(out[17]) // ns} bd {int(out[18]) // ns}")
    t = out.astype(np.int64)
    # k_build_sort: 0 load, 1 count, 2 scan, 3 starts, 4 scatter, 5 end;
    # k_cluster_build: 6 start, 11 init + pair copy, 7 union-find, 8 roots /
    # sizes / classes, 9 packing, 10 per-wave pair lists (s_memtime is per
    # XCD: compare stamps of one kernel only)
    sort = [("load", 0, 1), ("count", 1, 2), ("scan", 2, 3), ("starts", 3, 4), ("scatter", 4, 5)]
    build = [("init+copy", 6, 11), ("union", 11, 7), ("roots/classes", 7, 8), ("packing", 8, 9),
             ("wave pairs", 9, 10)]
    for name, rows in (("sort", sort), ("cluster build", build)):
        print(f"{name} cycles: " + "  ".join(f"{n} {int(t[b] - t[a])}" for n, a, b in rows))
