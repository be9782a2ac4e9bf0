"""Per-wave timing of the cluster run on the bench workload (needs the
SWARM_PHASE_TIMING variant: bash tools/build_variants.sh, then
SWARMRL_AMD_LIB=tools/_variants/lib_PT.so python tools/wave_times.py [E] [slices]).
Prints, for the last window of a few slices, the spread of wave durations,
the slowest waves with their pair passes/pairs, and the launch span."""
import argparse
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("envs", nargs="?", type=int, default=1)
ap.add_argument("slices", nargs="?", type=int, default=30)
ap.add_argument("--c5", action="store_true", help="the C5 workload (16384 colloids, field + RND)")
ap.add_argument("--colloids", type=int, default=0, help="colloids per env (C4: 1024 with E = 8)")
a = ap.parse_args()
n = a.colloids or (16384 if a.c5 else 4096)
ns = bench.argparse.Namespace(colloids=n, envs_per_gpu=a.envs)
torch.cuda.set_device(0)
eng, ff, agent = (bench.build_c5_workload if a.c5 else bench.build_workload)(
    ns, 42, torch.device("cuda", 0))
eng.integrate(1, ff)
nat = eng._native
wmax_words = 4 * a.envs * ((4 * n + 4224) // 64)
for rep in range(4):
    eng.integrate(a.slices // 4, ff)
    torch.cuda.synchronize()
    out = np.zeros(wmax_words, np.uint64)
    nat.call("swarm_engine_debug_wave_stamps", out.ctypes.data, ctypes.c_int32(wmax_words))
    w = out.reshape(-1, 4)
    w = w[w[:, 1] > 0].astype(np.int64)
    w = w[w[:, 1] >= w[:, 1].max() - 20000]  # this window's waves (stale stamps are older)
    t0 = w[:, 0].min()
    dur = (w[:, 1] - w[:, 0]) / 100.0  # us (100 MHz realtime)
    start = (w[:, 0] - t0) / 100.0
    end = (w[:, 1] - t0) / 100.0
    npass = w[:, 2] & 0xFF
    xcc = (w[:, 2] >> 16) & 0xFF
    hw = w[:, 2] >> 32
    # the SIMD a wave ran on: XCD, shader engine, array, CU, SIMD (HW_ID fields)
    simd_key = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | \
        (((hw >> 8) & 15) << 3) | ((hw >> 4) & 3)
    order = np.argsort(-dur)
    print(f"rep {rep}: {len(w)} waves, span {end.max():.1f} us; duration p50 {np.median(dur):.1f} "
          f"p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}; start skew max {start.max():.1f}")
    for k in order[:6]:
        print(f"   wave: start {start[k]:6.1f} dur {dur[k]:6.1f} npass {npass[k]} pairs {w[k, 3]}")
    keys, inv, cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
    simd_end = np.zeros(len(keys))
    np.maximum.at(simd_end, inv, end)
    print(f"   {len(keys)} SIMDs in {len(np.unique(simd_key >> 2))} CUs; waves per SIMD: " +
          ", ".join(f"{c}: {n} SIMDs (last end mean {simd_end[cnt == c].mean():.1f} max "
                    f"{simd_end[cnt == c].max():.1f} us)"
                    for c, n in zip(*np.unique(cnt, return_counts=True))))
    for p in sorted(set(npass.tolist())):
        m = npass == p
        print(f"   npass {p}: {m.sum()} waves, mean {dur[m].mean():.1f} max {dur[m].max():.1f}")
