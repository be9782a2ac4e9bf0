"""Per-kernel totals from a rocprofv3 results database:
python tools/db_stats.py <run_results.db> [top]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = c.execute("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels "
                 "group by name order by sum(end-start) desc limit ?", (top,)).fetchall()
for name, cnt, tot, avg in rows:
    print(f"{tot:10.1f} us  n={cnt:5d} avg={avg:8.2f}  {name[:100]}")
