#!/usr/bin/env python3
"""Per-slice kernel timeline from a rocprofv3 kernel trace: the launches
between consecutive run-kernel ends, as start / end offsets (us) from the
previous run's end, averaged over the slices of the trace.
usage: slice_trace.py run_kernel_trace.csv [run_kernel_substring]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_cluster_run"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("swarm::", "")
            short = short.replace("(anonymous namespace)::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r["Queue_Id"]))
    rows.sort()
    runs = [r for r in rows if key in r[2]]
    acc = collections.defaultdict(list)
    n = 0
    for a, b in zip(runs, runs[1:]):
        t0 = a[1]
        seq = [r for r in rows if r[0] >= t0 and r[0] <= b[0]]
        if b[0] - t0 > 2e6:  # > 2 ms: not one slice
            continue
        n += 1
        cnt = collections.Counter()
        for s, e, name, q in seq:
            cnt[name] += 1
            acc[(name, cnt[name])].append(((s - t0) / 1e3, (e - t0) / 1e3, q))
    print(f"{n} slices (offsets in us from the previous run's end)")
    items = sorted(acc.items(), key=lambda kv: sum(x[0] for x in kv[1]) / len(kv[1]))
    for (name, k), v in items:
        if len(v) < n // 2:
            continue
        s = sum(x[0] for x in v) / len(v)
        e = sum(x[1] for x in v) / len(v)
        print(f"  {s:8.1f} {e:8.1f} {e - s:7.1f}  q{v[0][2]}  {name}" + (f" #{k}" if k > 1 else ""))


if __name__ == "__main__":
    main()
