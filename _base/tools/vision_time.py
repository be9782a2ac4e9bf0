"""Time the vision-cone observable (k_vision_grid + k_vision) on the bench
workload for E envs: python tools/vision_time.py E [E ...]"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

torch.cuda.set_device(0)
for E in [int(a) for a in sys.argv[1:]] or [1, 64]:
    ns = argparse.Namespace(colloids=4096, envs_per_gpu=E)
    eng, ff, agent = bench.build_workload(ns, 42, torch.device("cuda", 0))
    eng.integrate(2, ff)
    view = eng.swarm_view()
    obs = agent.observable
    for _ in range(3):
        obs.compute_observable(view)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        obs.compute_observable(view)
    b.record()
    b.synchronize()
    print(f"E={E:3d} vision observable {a.elapsed_time(b) / 20 * 1e3:8.1f} us", flush=True)
    del eng, ff, agent
