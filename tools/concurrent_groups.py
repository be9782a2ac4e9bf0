"""Throughput of E envs per GPU split into K engines of E/K envs whose
captured episode graphs replay concurrently on K streams (the run kernel of
one group overlapping the observables / policy of another).
python tools/concurrent_groups.py E K [K ...]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
E = int(sys.argv[1])
T = 20
for K in [int(a) for a in sys.argv[2:]]:
    groups = []
    for g in range(K):
        ns = argparse.Namespace(colloids=4096, envs_per_gpu=E // K, write_interval=1.0)
        eng, ff, agent = bench.build_workload(ns, 42 + g * (E // K), dev)
        eng.integrate(1, ff)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                eng.integrate(1, ff)
        torch.cuda.current_stream().wait_stream(side)
        agent.reset_trajectory()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            eng.integrate(T, ff)
        groups.append((eng, ff, agent, graph, torch.cuda.Stream()))
    torch.cuda.synchronize()

    def episodes(n):
        main = torch.cuda.current_stream()
        for _ in range(n):
            for eng, ff, agent, graph, st in groups:
                st.wait_stream(main)
                with torch.cuda.stream(st):
                    graph.replay()
            for eng, ff, agent, graph, st in groups:
                main.wait_stream(st)
            for g in groups:
                g[0].drain_trajectory(block=False)

    episodes(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_ep = 5
    episodes(n_ep)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = 4096 * E * T * n_ep
    print(f"E={E} K={K}: {steps / dt / 1e6:8.1f} M agent-steps/s, {dt / (T * n_ep) * 1e6:7.1f} us "
          f"per slice", flush=True)
    del groups
    torch.cuda.synchronize()
