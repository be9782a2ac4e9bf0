"""End-to-end PPO training cost on the bench workload (4096 colloids, one
env): per episode, the rollout (20 slices through the engine, eager) and
the agent update (GAE + n_epochs PPO steps).  python tools/train_time.py [E]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.cuda.set_device(0)
ns = argparse.Namespace(colloids=4096, envs_per_gpu=E)
eng, ff, agent = bench.build_workload(ns, 42, torch.device("cuda", 0))
eng.integrate(1, ff)
agent.reset_trajectory()
for ep in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.integrate(20, ff)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    agent.update_agent()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"episode {ep}: rollout {1e3 * (t1 - t0):7.2f} ms  update "
          f"({agent.loss.n_epochs} epochs) {1e3 * (t2 - t1):7.2f} ms", flush=True)
