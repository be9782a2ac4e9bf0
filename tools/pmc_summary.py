"""Per-kernel, per-grid averages of the SQ counter passes of tools/pmc_run.sh.
Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel substring]"""
import collections
import csv
import glob
import re
import sys

src = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"{src}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        name = re.sub(r"^void ", "", name).split("(")[0][:60]
        if key not in name:
            continue
        acc[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), cs in sorted(acc.items()):
    print(f"== {k} grid={g}")
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
