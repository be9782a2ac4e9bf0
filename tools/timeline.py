"""Print one slice of a rocprofv3 kernel trace around the n-th launch of a
kernel (per-kernel start/end relative to the first row shown, queue id).
Usage: python tools/timeline.py <run_kernel_trace.csv> <kernel substring> [n] [before] [after]"""
import csv
import re
import sys

path, key = sys.argv[1], sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 20
before = int(sys.argv[4]) if len(sys.argv) > 4 else 12
after = int(sys.argv[5]) if len(sys.argv) > 5 else 14
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i0 = idx[min(nth, len(idx) - 1)]
lo = max(0, i0 - before)
t0 = int(rows[lo]["Start_Timestamp"])
for r in rows[lo:i0 + after]:
    n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:50]
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    print(f"{n:50s} q{r['Queue_Id']} grid={r['Grid_Size_X']:>7} {s:8.1f} {e:8.1f} {e - s:6.1f}")
