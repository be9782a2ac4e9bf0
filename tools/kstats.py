"""Print the top kernels of a rocprofv3 --stats CSV (tools/kstats.py <dir>)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f}us {float(r['TotalDurationNs'])/tot*100:5.1f}% "
          f"{r['Name'][:100]}")
