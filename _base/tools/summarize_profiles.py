"""
Summarize a profiles/profile_round.sh run (one config-pure bench.py --only
<line> run per line) into committed files:
  profiles/<tag>_<line>_kernel_stats.csv  rocprofv3 --stats of that line's run
  profiles/<tag>_<line>_bench.json        its bench line
  profiles/<tag>_pmc_summary.csv          per line and kernel: dispatches, mean
                                          duration (kernel trace), FETCH_SIZE,
                                          WRITE_SIZE, SQ_INSTS_VALU,
                                          SQ_INSTS_VALU_TRANS_F32, SQ_WAVES and
                                          (sq pass) SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
                                          SQ_WAIT_INST_ANY, SQ_WAIT_INST_LDS,
                                          SQ_INSTS_LDS, SQ_ACTIVE_INST_VALU
  profiles/<tag>_traffic.json             per line, the dominant kernels' rows:
                                          bytes per launch (FETCH_SIZE x 2 +
                                          WRITE_SIZE, KB -> B; MI355X_MICROARCH.md
                                          gfx950 correction), VALU counts, mean
                                          duration, the source hash bench.py
                                          checks (src_sha)
Usage: python tools/summarize_profiles.py <tag>
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (source_sha, LINES)

tag = sys.argv[1]
src = f"gpurun_out/prof_{tag}"
dst = "profiles"
DOMINANT = {"head": r"k_cluster_run", "batched": r"k_cluster_run", "c2": r"k_cluster_run",
            "c4": r"k_cluster_run", "c5": r"k_cluster_run", "c3train": r"k_cluster_run|k_ppo_grads"}
TIMED_TAIL = 20  # bench.py --bd-reps
COUNTERS = ["FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_WAVES",
            "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
            "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU"]


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"^void ", "", name).split("(")[0][:90]


sha = bench.source_sha()
summary, traffic = [], []
for line in bench.LINES:
    d = f"{src}/{line}"
    if not os.path.isdir(d):
        continue
    shutil.copy(f"{d}/trace/run_kernel_stats.csv", f"{dst}/{tag}_{line}_kernel_stats.csv")
    timed_n = {}  # kernel regex -> launches bench.py timed at the end of the run
    for ln in open(f"{d}/trace_bench.log"):
        if ln.startswith("{"):
            with open(f"{dst}/{tag}_{line}_bench.json", "w") as f:
                f.write(ln)
            rec = json.loads(ln)
            roof = rec.get("roofline") or {}
            if roof.get("kernel_timing_launches"):
                # the run kernel: event-timed inside an episode graph replayed
                # after the timed region (bench.time_run_kernel)
                timed_n[r"k_cluster_run"] = int(roof["kernel_timing_launches"])
            if (rec.get("roofline_update") or {}).get("kernel"):
                timed_n[r"k_ppo_grads"] = TIMED_TAIL  # swarm_ppo_profile's back-to-back reps
    dur = collections.defaultdict(list)
    rows = sorted(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")),
                  key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        dur[short(r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)  # ns -> us
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("fetch", "write", "valu", "sq"):
        path = f"{d}/{sub}/run_counter_collection.csv"
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(set(dur) | set(acc)):
        cs = acc.get(k, {})
        mean = {c: (sum(cs[c]) / len(cs[c]) if cs.get(c) else None) for c in COUNTERS}
        us = sum(dur[k]) / len(dur[k]) if dur.get(k) else None
        summary.append([line, k, len(dur.get(k, [])), f"{us:.2f}" if us else ""] +
                       [f"{mean[c]:.1f}" if mean[c] is not None else "" for c in COUNTERS])
        if re.search(DOMINANT.get(line, "$^"), k) and mean["FETCH_SIZE"] and mean["WRITE_SIZE"]:
            n = next((v for rx, v in timed_n.items() if re.search(rx, k)), TIMED_TAIL)
            ks = dur.get(k, [])
            traffic.append({
                "line": line, "kernel": k, "dispatches": len(ks),
                "mean_duration_us": us,
                # the launches bench.py's HIP events time: the kernel's last n
                # dispatches (the run kernel: the windows of the episode graph
                # replayed after the timed region; k_ppo_grads: --bd-reps
                # back-to-back launches)
                "timed_launches": n,
                "mean_duration_timed_us": sum(ks[-n:]) / n if len(ks) >= n else None,
                # every earlier launch (the workload itself: warmup and the
                # timed region, mostly graph replays)
                "mean_duration_graph_us": (sum(ks[:-n]) / len(ks[:-n]) if len(ks) > n else None),
                "fetch_size_kb": mean["FETCH_SIZE"], "write_size_kb": mean["WRITE_SIZE"],
                "bytes_per_launch": (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0,
                "valu_insts_per_launch": mean["SQ_INSTS_VALU"],
                "valu_trans_per_launch": mean["SQ_INSTS_VALU_TRANS_F32"],
                "waves_per_launch": mean["SQ_WAVES"],
                # the sq pass (when run): wave-cycles and the cycles waves
                # waited on any instruction / on LDS, per launch
                "sq_wave_cycles": mean["SQ_WAVE_CYCLES"],
                "sq_wait_inst_any": mean["SQ_WAIT_INST_ANY"],
                "sq_wait_inst_lds": mean["SQ_WAIT_INST_LDS"],
                "sq_insts_lds": mean["SQ_INSTS_LDS"],
                "sq_active_inst_valu": mean["SQ_ACTIVE_INST_VALU"],
                "src_sha": sha,
            })
with open(f"{dst}/{tag}_pmc_summary.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["line", "kernel", "dispatches", "mean_us"] + [f"mean_{c}" for c in COUNTERS])
    w.writerows(summary)
with open(f"{dst}/{tag}_traffic.json", "w") as f:
    json.dump(traffic, f, indent=1)
print(json.dumps(traffic, indent=1))
