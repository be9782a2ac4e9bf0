"""
Summarize a profiles/profile_round.sh run into committed files:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats (copied)
  profiles/<tag>_bench.json         the bench line of the traced run
  profiles/<tag>_pmc_summary.csv    per-kernel, per-grid averages of FETCH_SIZE,
                                    WRITE_SIZE, SQ_INSTS_VALU, SQ_WAVES
  profiles/<tag>_traffic.json       per-launch HBM bytes of k_cluster_run by
                                    env count (FETCH_SIZE x 2 + WRITE_SIZE,
                                    MI355X_MICROARCH.md gfx950 correction)
Usage: python tools/summarize_profiles.py <tag> [colloids]
"""
import collections
import csv
import re
import json
import os
import shutil
import sys

tag = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N_C5 = int(sys.argv[3]) if len(sys.argv) > 3 else 16384  # bench.py --c5-colloids


def envs_of_grid(g, wide):
    """Envs of a run launch of g threads: ceil(E * wmax / 4) blocks of 256
    (k_cluster_run), or of 1024 after 64 noise blocks when E * N <= 8192
    (k_cluster_run_wide); wmax = slots_per_env / 64 (dense: 2 N, one-pass:
    4 N slots)."""
    for E in range(1, 4097):
        for slots in (2 * N + 64 * 66, 4 * N + 64 * 66):
            blocks = (E * (slots // 64) + 3) // 4
            if wide:
                nnb = 64 if E * N <= 8192 else 0
                if (nnb + blocks) * 1024 == g:
                    return E
            elif blocks * 256 == g:
                return E
    return None

src = f"gpurun_out/prof_{tag}"
dst = "profiles"
shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"{dst}/{tag}_kernel_stats.csv")
for line in open(f"{src}/trace_bench.log"):
    if line.startswith("{"):
        with open(f"{dst}/{tag}_bench.json", "w") as f:
            f.write(line)

acc = collections.defaultdict(lambda: collections.defaultdict(list))
first = {}
for sub in ("fetch", "write", "valu"):
    path = f"{src}/{sub}/run_counter_collection.csv"
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        name = re.sub(r"^void ", "", name).split("(")[0][:80]
        key = (name, int(r["Grid_Size"]))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        first.setdefault(key, int(r["Dispatch_Id"]))
names = ["FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_WAVES"]
with open(f"{dst}/{tag}_pmc_summary.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "grid_size", "dispatches"] + [f"mean_{n}" for n in names])
    for (k, g), cs in sorted(acc.items()):
        n = max(len(v) for v in cs.values())
        w.writerow([k, g, n] + [f"{sum(cs[c]) / len(cs[c]):.1f}" if cs.get(c) else "" for c in names])

# bench.py measures E = 1 (4096 colloids), then the batched envs, then the
# config-5 env (16384 colloids): the latency-bound (wide) launches in order of
# their first dispatch are the E = 1 line and the C5 line.
wide_keys = sorted((key for key in acc if "k_cluster_run_wide" in key[0]), key=lambda kk: first[kk])
traffic = []
for (k, g), cs in acc.items():
    if "k_cluster_run" not in k or not cs.get("FETCH_SIZE") or not cs.get("WRITE_SIZE"):
        continue
    n_env = N
    if "wide" in k:
        E = 1
        if wide_keys.index((k, g)) > 0:
            n_env = N_C5
    else:
        E = envs_of_grid(g, False)
    fetch_kb = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
    write_kb = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
    traffic.append({
        "kernel": k, "envs": E, "colloids": n_env,
        "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
        # FETCH_SIZE/WRITE_SIZE are in KB; FETCH_SIZE reads half the bytes on gfx950
        "bytes_per_launch": (2 * fetch_kb + write_kb) * 1024.0,
        "valu_insts_per_launch": (sum(cs["SQ_INSTS_VALU"]) / len(cs["SQ_INSTS_VALU"])
                                  if cs.get("SQ_INSTS_VALU") else None),
        "source": f"{tag}_pmc_summary.csv",
    })
with open(f"{dst}/{tag}_traffic.json", "w") as f:
    json.dump(traffic, f, indent=1)
print(json.dumps(traffic, indent=1))
