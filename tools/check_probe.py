"""Per-env phase times of k_check on the bench workload (needs the CT
variant library: bash tools/build_variants.sh CT -DSWARM_CHECK_TIMING):
  SWARMRL_AMD_LIB=tools/_variants/lib_CT.so python tools/check_probe.py E SLICES
Prints, per slice, the slowest env's check: total, loads+big clusters, the
exact test, the tail (us, 100 MHz realtime clock), movers, big clusters, kc."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1
S = int(sys.argv[2]) if len(sys.argv) > 2 else 30
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
ns = argparse.Namespace(colloids=4096, envs_per_gpu=E, write_interval=1.0)
eng, ff, agent = bench.build_workload(ns, 42, dev)
buf = (ctypes.c_uint64 * (8 * E))()
rows = []
for s in range(S):
    eng.integrate(1, ff)
    torch.cuda.synchronize()
    eng._native.call("swarm_engine_debug_wave_stamps", buf, 8 * E)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(E, 8).astype(np.int64)
    tot = (a[:, 3] - a[:, 0]) / 100.0
    k = int(np.argmax(tot))
    r = a[k]
    rows.append(tot[k])
    print(f"slice {s:3d} env {k:2d} total {tot[k]:6.2f} us  loads+big {(r[1]-r[0])/100:6.2f}"
          f"  test {(r[2]-r[1])/100:6.2f}  tail {(r[3]-r[2])/100:6.2f}  movers {r[4]:4d}"
          f"  big {r[5]:3d}  kc {r[6]:3d}  rerun {r[7]}  | env-median total {np.median(tot):.2f}"
          f"  movers median {np.median(a[:, 4]):.0f} max {a[:, 4].max()}  envs with big {int((a[:, 5] > 0).sum())}",
          flush=True)
print("mean of slowest-env totals", np.mean(rows[3:]))
