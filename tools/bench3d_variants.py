"""Timing of the 3-D neighbour-list window (bench.py measure_dims3) for the
library named by SWARMRL_AMD_LIB: prints one JSON line with the E=1 and
E=64 ms per slice (HIP-graph replays).  Used with the timing-ablation
builds under tools/_variants (SWARM_ABL_NL_* macros)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--colloids", type=int, default=4096)
    ap.add_argument("--envs", type=int, nargs="+", default=[1, 64])
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    out = {"lib": os.environ.get("SWARMRL_AMD_LIB", "default")}
    for E in a.envs:
        r = bench.measure_dims3(a, E, 30 if E == 1 else 10, global_reps=0)
        out[f"E{E}"] = round(r["ms_per_slice"], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
