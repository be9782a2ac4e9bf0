"""Per-variant run-kernel counters of a tools/ab_variants.sh run:
python tools/ab_summary.py TAG -> mean FETCH_SIZE x 2 + WRITE_SIZE per grid."""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1]
root = f"gpurun_out/ab_{tag}"
acc = collections.defaultdict(list)
for path in glob.glob(f"{root}/*_*_SIZE/run_counter_collection.csv"):
    v = os.path.basename(os.path.dirname(path)).rsplit("_", 2)[0]
    for r in csv.DictReader(open(path)):
        if "k_cluster_run" in r["Kernel_Name"]:
            acc[(v, r["Counter_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
for (v, c, g), vals in sorted(acc.items()):
    print(f"{v:8s} {c:11s} grid {g:8d} n={len(vals):3d} mean {sum(vals) / len(vals) / 1024:8.2f} MB")
