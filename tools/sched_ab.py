#!/usr/bin/env python3
"""A/B of the engine's slice schedules on one bench line (development
tool): runs bench.py's line with the engine attributes of each named
schedule set on the workload's engine, prints value per schedule.
usage: python tools/sched_ab.py LINE SCHED [SCHED ...]
  SCHED: default | no_early_fork | serial"""
import json
import os
import subprocess
import sys

SCHEDS = {
    "default": {},
    "no_early_fork": {"early_fork": False},
    "serial": {"overlap_build": False},
}

CHILD = r"""
import sys, json
sys.argv = ["bench.py", "--only", LINE, "--no-cpu-baseline"]
sys.path.insert(0, ".")
import bench
attrs = json.loads(ATTRS)
for name in ("build_workload", "build_c5_workload", "build_c3_workload"):
    f = getattr(bench, name)
    def wrap(*a, _f=f, **k):
        out = _f(*a, **k)
        for key, v in attrs.items():
            setattr(out[0], key, v)
        return out
    setattr(bench, name, wrap)
bench.main()
"""


def main():
    line = sys.argv[1]
    for sched in sys.argv[2:]:
        code = CHILD.replace("LINE", repr(line)).replace("ATTRS", repr(json.dumps(SCHEDS[sched])))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=300, env=dict(os.environ))
        vals = None
        for ln in r.stdout.splitlines():
            if ln.startswith("{"):
                d = json.loads(ln)
                vals = {k: round(v["value"] / 1e6, 2) for k, v in d.items()
                        if isinstance(v, dict) and "value" in v}
                vals["head"] = round(d["value"] / 1e6, 2)
        print(sched, vals if vals is not None else r.stderr[-2000:], flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
