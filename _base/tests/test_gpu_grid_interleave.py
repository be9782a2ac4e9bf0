"""
The speculative vision grid against other users of the cell-start scratch
(ADVICE r3): the reward launch builds the next slice's observable grid
(k_field_vgrid_sort) and the next vision cone reuses it.  A neighbour-pair
query between two slices (swarm_engine_neighbor_pairs: its own cell grid in
the same scratch, reallocated when it needs more cells) must invalidate that grid, so that
the cone rebuilds it.  Two engines from the same placement and seed, one with
queries at several cutoffs between its slices, must record the same features,
actions and rewards and end in the same state, bit for bit (the plain engine's
trajectory is the oracle's, tests/test_gpu_headline.py).
"""

import argparse
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _episode(n, slices, query):
    sys.path.insert(0, ROOT)
    import bench

    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(colloids=n, envs_per_gpu=1, write_interval=1.0)
    eng, ff, agent = bench.build_workload(ns, 42, dev)
    agent.reset_trajectory()
    counts = []
    for s in range(slices):
        eng.integrate(1, ff)
        if query:
            # a grid of its own between the reward and the cone: cutoff 2 has
            # more cells than the observable grid (a larger start buffer), the
            # larger cutoffs overwrite the cell starts in place
            cutoff = 2.0 + 3.0 * s
            pairs = np.zeros((400000, 2), np.int32)
            cnt = np.zeros(1, np.int32)
            eng._native.bind_stream()
            eng._native.call("swarm_engine_neighbor_pairs", 0, cutoff, pairs.ctypes.data,
                             400000, cnt.ctypes.data)
            counts.append(int(cnt[0]))
    torch.cuda.synchronize()
    traj = {k: [torch.as_tensor(x).detach().cpu().numpy().copy()
                for x in getattr(agent.trajectory, k)]
            for k in ("features", "actions", "rewards")}
    return traj, eng.get_raw_state(), counts


def test_neighbor_pairs_between_slices_keeps_observables():
    torch.cuda.set_device(0)
    n, slices = 1024, 6
    a, sa, _ = _episode(n, slices, query=False)
    b, sb, counts = _episode(n, slices, query=True)
    assert len(counts) == slices and all(c > 0 for c in counts)
    for k in ("features", "actions", "rewards"):
        assert len(a[k]) == len(b[k]) >= slices - 1, k
        for s, (x, y) in enumerate(zip(a[k], b[k])):
            assert np.array_equal(x, y), (k, s)
    for k in ("q", "img", "ang"):
        assert np.array_equal(sa[k], sb[k]), k
