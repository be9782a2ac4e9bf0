"""Per-window fallback statistics of the bench workload (GPU):
python tools/fallback_stats.py [envs] [slices] [seed]"""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = int(sys.argv[2]) if len(sys.argv) > 2 else 60
SEED = int(sys.argv[3]) if len(sys.argv) > 3 else 42
ns = argparse.Namespace(colloids=4096, envs_per_gpu=E)
torch.cuda.set_device(0)
eng, ff, agent = bench.build_workload(ns, SEED, torch.device("cuda", 0))
flagged = rerun = 0
waves = []
for s in range(S):
    eng.integrate(1, ff)
    st = eng.window_stats()
    fb, w = st["fallback"], st["waves"]
    flagged += int((fb == 1).sum())
    rerun += int((fb == 2).sum())
    waves.append(w[fb == 0].mean() if (fb == 0).any() else 0)
    if s % 10 == 9:
        print(f"slice {s+1}: flagged {flagged} rerun {rerun} of {E*(s+1)} env-windows, "
              f"mean waves/env {np.mean(waves[-10:]):.1f}", flush=True)
