#!/usr/bin/env python
"""
bench.py -- agent-steps/s of the 4096-colloid WCA + vision-cone rollout.

One step = one RL slice for every agent of every env on every rank:
vision-cone observable (HIP) -> actor-critic MLP + Gumbel sampling (torch) ->
action table -> 100 Brownian-dynamics sub-steps with WCA (HIP) -> gradient-
sensing reward (HIP + torch) -> device trajectory ring buffers.  The slice is
captured once into a HIP graph and replayed.  With N > 1 ranks (one process
per GPU, RCCL) every rank runs its own envs (seed 42 + env id) and the
trajectory buffers are all-gathered at the end of each episode.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement".
"""

import argparse
import json
import math
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec, 4096-colloid WCA+vision-cone rollout @1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue roofline (MI355X_MICROARCH.md:489, 'vector-instruction ISSUE
# cost'): one wave's stream issues v_fma/v_add-class instructions at 4 cycles
# and transcendentals (v_exp/log/rcp/rsq/sqrt/sin/cos) at 8 on its SIMD;
# 1024 SIMDs at 2.4 GHz.  (The 2-cycle rate of line 473 needs two waves
# issuing on a SIMD; it is the 157.3 TF f32 vector peak.)
SIMD_CLOCKS_PER_S = 1024 * 2.4e9
VALU_CYCLES, TRANS_CYCLES = 4, 8
VALU_PEAK_WAVE_INSTS = SIMD_CLOCKS_PER_S / VALU_CYCLES
F32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: F32 row (= vector peak)
BYTES_PER_PARTICLE_SUBSTEP = 40
PPO_MAC_PER_SAMPLE = 2944        # DESIGN.md section 6 "PPO update" (3-128-(4+1) MLP)
# the lines one bench.py run can measure (--only): see main()
LINES = ("head", "batched", "c2", "c4", "c5", "c3train", "dims3", "dense2d")


def source_sha() -> str:
    """Hash of the HIP sources and the C-ABI header the library is built from
    (swarmrl_amd._capi.source_hash, compiled into the library as
    swarm_build_id): profiles/<tag>_traffic.json rows carry it, so a kernel
    change is not reported with stale counter numbers."""
    import hashlib
    import pathlib

    root = pathlib.Path(ROOT)
    h = hashlib.sha256()
    files = sorted([*(root / "swarmrl_amd" / "csrc").glob("*"), *(root / "include").glob("*.h")],
                   key=os.fspath)
    for path in files:
        h.update(path.name.encode())
        h.update(path.read_bytes())
    return h.hexdigest()[:12]


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--colloids", type=int, default=4096)
    ap.add_argument("--envs-per-gpu", type=int, default=1,
                    help="headline: one env (4096 colloids) per GPU, as BASELINE's north star")
    ap.add_argument("--batched-envs", type=int, default=64,
                    help="also report envs-per-GPU batching in 'batched' (0: off)")
    ap.add_argument("--episode-length", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-slices", type=int, default=200)
    ap.add_argument("--cpu-all-core-slices", type=int, default=200,
                    help="slices of the all-cores (OpenMP) CPU baseline (0: skip it)")
    ap.add_argument("--cpu-all-pairs-slices", type=int, default=10,
                    help="slices of the all-pairs-vision CPU context row (0: skip it)")
    ap.add_argument("--bd-reps", type=int, default=20)
    ap.add_argument("--c5-colloids", type=int, default=16384,
                    help="BASELINE config 5 line ('c5': chemotaxis + RND, one env; 0: off)")
    ap.add_argument("--write-interval", type=float, default=1.0,
                    help="trajectory write interval in seconds (the reference default, "
                         "espresso.py:64-77); recorded on the device inside the captured "
                         "episode and drained without blocking between episodes")
    ap.add_argument("--dims3", type=int, default=1,
                    help="3-D at scale line ('dims3': BD+WCA slices of --colloids colloids in a "
                         "periodic 3-D box on the cluster path vs the 3-D global path; 0: off)")
    ap.add_argument("--only", default="all",
                    help="comma-separated lines to measure (" + ", ".join(LINES) + "; default all): "
                         "config-pure runs for profiles/profile_round.sh")
    ap.add_argument("--c2-colloids", type=int, default=1024,
                    help="BASELINE config 2 line ('c2': vision cone + random MLP, one env)")
    ap.add_argument("--c4-envs", type=int, default=8,
                    help="BASELINE config 4 per-rank shard ('c4': envs per GPU of 64 x 1024)")
    ap.add_argument("--c4-colloids", type=int, default=1024)
    ap.add_argument("--train-episodes", type=int, default=4,
                    help="timed episodes of the 'c3train' line (rollout + PPO update)")
    ap.add_argument("--force-collective", action="store_true",
                    help="at --gpus 1: a world-size-1 RCCL group, and the episode-parallel "
                         "collectives (broadcast, packed trajectory all-gather, replicated "
                         "update) run through it as at N GPUs (rollout.force_collectives)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU plumbing test: no GPU, gloo, synthetic trajectories")
    return ap.parse_args()


def build_workload(args, env_seed, device):
    import torch

    from swarmrl_amd.actions import Action
    from swarmrl_amd.agents import ActorCriticAgent
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel
    from swarmrl_amd.observables import SubdividedVisionCones
    from swarmrl_amd.tasks.searching import GradientSensing
    from swarmrl_amd.units import UnitRegistry

    N, E = args.colloids, args.envs_per_gpu
    L = 2.0 * math.sqrt(N * 1.0**2 / 0.1)  # area fraction 0.1 in the placement disc
    ureg = UnitRegistry()
    params = MDParams(
        ureg=ureg,
        box_length=ureg.Quantity([L, L, L], "micrometer"),
        time_step=ureg.Quantity(1e-3, "second"),
        time_slice=ureg.Quantity(0.1, "second"),
        write_interval=ureg.Quantity(getattr(args, "write_interval", 1.0), "second"),
    )
    eng = SwarmEngine(params, n_dims=2, seed=env_seed, n_envs=E,
                      out_folder=f"/tmp/swarm_bench_{os.getpid()}")
    eng.add_colloids(N, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([L / 2, L / 2, 0.0]), "micrometer"),
                     ureg.Quantity(L / 2, "micrometer"))
    observable = SubdividedVisionCones(10.0, np.pi / 2, 3, radii=[1.0] * N)
    task = GradientSensing(source=np.array([L / 2, L / 2, 0.0]), decay_function=lambda d: 1 - d,
                           box_length=np.array([L, L, L]), reward_scale_factor=10)
    torch.manual_seed(env_seed)
    net = TorchModel(ActorCriticMLP(3, 4, 128), input_shape=(3,), device=device)
    actions = {
        "RotateClockwise": Action(torque=np.array([0.0, 0.0, 10.0])),
        "Translate": Action(force=10.0),
        "RotateCounterClockwise": Action(torque=np.array([0.0, 0.0, -10.0])),
        "DoNothing": Action(),
    }
    agent = ActorCriticAgent(0, net, task, observable, actions, train=True)
    ff = ForceFunction({"0": agent})
    agent.reset_agent(eng.colloids)
    return eng, ff, agent


def build_c3_workload(args, env_seed, device):
    """BASELINE config 3: the find-centre task of the reference's PPO test
    (test_rl_trainers.py:105-118): ConcentrationField
    observable (scale 10000) + GradientSensing reward (scale 10), f(d) = 1 - d,
    source at the box centre, MLP 1-128-(4+1), PPO defaults."""
    return build_c5_workload(args, env_seed, device, rnd=False)


def build_c5_workload(args, env_seed, device, rnd=True):
    """BASELINE config 5: 16384 colloids, concentration-field chemotaxis +
    intrinsic reward: ConcentrationField observable (scale
    10000) + GradientSensing task (scale 10), f(d) = 1 - d, source at the box
    centre, and an RND intrinsic reward (3 x Dense(32) target/predictor) on
    the device; MLP 1-128-(4+1)."""
    import torch

    from swarmrl_amd.actions import Action
    from swarmrl_amd.agents import ActorCriticAgent
    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.force_functions import ForceFunction
    from swarmrl_amd.intrinsic_reward import RNDConfig, RNDReward
    from swarmrl_amd.networks import ActorCriticMLP, TorchModel
    from swarmrl_amd.observables import ConcentrationField
    from swarmrl_amd.tasks.searching import GradientSensing
    from swarmrl_amd.units import UnitRegistry

    N, E = args.colloids, args.envs_per_gpu
    L = 2.0 * math.sqrt(N * 1.0**2 / 0.1)
    ureg = UnitRegistry()
    params = MDParams(
        ureg=ureg,
        box_length=ureg.Quantity([L, L, L], "micrometer"),
        time_step=ureg.Quantity(1e-3, "second"),
        time_slice=ureg.Quantity(0.1, "second"),
        write_interval=ureg.Quantity(getattr(args, "write_interval", 1.0), "second"),
    )
    eng = SwarmEngine(params, n_dims=2, seed=env_seed, n_envs=E,
                      out_folder=f"/tmp/swarm_bench_c5_{os.getpid()}")
    eng.add_colloids(N, ureg.Quantity(1.0, "micrometer"),
                     ureg.Quantity(np.array([L / 2, L / 2, 0.0]), "micrometer"),
                     ureg.Quantity(L / 2, "micrometer"))
    box = np.array([L, L, L])
    src = np.array([L / 2, L / 2, 0.0])
    obs = ConcentrationField(src, lambda d: 1 - d, box, scale_factor=10000)
    task = GradientSensing(source=src, decay_function=lambda d: 1 - d, box_length=box,
                           reward_scale_factor=10)
    torch.manual_seed(env_seed)
    intrinsic = RNDReward(RNDConfig(input_shape=(1,), device=device)) if rnd else None
    net = TorchModel(ActorCriticMLP(1, 4, 128), input_shape=(1,), device=device)
    actions = {
        "RotateClockwise": Action(torque=np.array([0.0, 0.0, 10.0])),
        "Translate": Action(force=10.0),
        "RotateCounterClockwise": Action(torque=np.array([0.0, 0.0, -10.0])),
        "DoNothing": Action(),
    }
    agent = ActorCriticAgent(0, net, task, obs, actions, train=True, intrinsic_reward=intrinsic)
    ff = ForceFunction({"0": agent})
    agent.reset_agent(eng.colloids)
    return eng, ff, agent


def measure_dims3(args, E, reps, global_reps=0, dims=3, fraction=0.04):
    """3-D at scale: n_dims=3 is the reference engine's default
    (EspressoMD(n_dims=3), espresso.py:143-152).  E envs of --colloids
    colloids at volume fraction 0.04 (placed in the centred sphere, overlaps
    removed), random swim forces and lab-frame torques, timed over `reps`
    HIP-graph replays of a slice of 100 BD+WCA sub-steps (engine only: the reference's vision
    cones are 2-D).  At this density the rc + skin graph percolates, so the
    engine takes the neighbour-list window (one chip-wide launch per
    sub-step); also timed: the cluster window forced (its clusters exceed a
    wave, so every window re-runs) and the 3-D global path (one workgroup
    per env per window, the round-1 3-D path), global_reps slices each."""
    import torch

    from swarmrl_amd.engine import MDParams, SwarmEngine
    from swarmrl_amd.units import UnitRegistry

    N = args.colloids
    if dims == 3:
        L = (N * (4.0 / 3.0) * math.pi / fraction) ** (1.0 / 3.0)
    else:  # dense 2-D (dims=2): area fraction in the box, placed in the centred disc
        L = math.sqrt(N * math.pi / fraction)
    ureg = UnitRegistry()
    params = MDParams(ureg=ureg, box_length=ureg.Quantity([L, L, L], "micrometer"),
                      time_step=ureg.Quantity(1e-3, "second"),
                      time_slice=ureg.Quantity(0.1, "second"),
                      write_interval=ureg.Quantity(1e4, "second"))
    rng = np.random.default_rng(7)
    f = rng.choice([0.0, 10.0], E * N).astype(np.float32)
    tq = rng.normal(scale=5.0, size=(3, E * N)).astype(np.float32)

    def make(mode):
        os.environ["SWARMRL_AMD_CLUSTER_PATH"] = "0" if mode == "global" else "1"
        os.environ["SWARMRL_AMD_NLIST"] = "1" if mode == "nlist" else "0"
        try:
            eng = SwarmEngine(params, n_dims=dims, seed=11, n_envs=E,
                              out_folder=f"/tmp/swarm_bench_3d_{os.getpid()}")
            eng.add_colloids(N, ureg.Quantity(1.0, "micrometer"),
                             ureg.Quantity(np.array([L / 2, L / 2, L / 2 if dims == 3 else 0.0]),
                                           "micrometer"),
                             ureg.Quantity(L / 2, "micrometer"))
            eng.integrate(1)  # set-up, overlap removal, one slice
        finally:
            del os.environ["SWARMRL_AMD_CLUSTER_PATH"]
            del os.environ["SWARMRL_AMD_NLIST"]
        nat = eng._native
        nat.bind_stream()
        nat.call("swarm_engine_set_actions", f.ctypes.data, tq[2].copy().ctypes.data, 0)
        if dims == 3:
            nat.call("swarm_engine_set_torque_xy", np.ascontiguousarray(tq[:2]).ctypes.data, 0)
        return eng

    def time_slices(eng, n):
        # one slice captured in a HIP graph (as the rollout captures its
        # episodes), replayed n times
        for _ in range(3):
            eng._run(100)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            eng._run(100)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            eng._run(100)
        graph.replay()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(n):
            graph.replay()
        t1.record()
        t1.synchronize()
        return t0.elapsed_time(t1) / n

    eng = make("nlist")
    ms = time_slices(eng, reps)
    fb = np.zeros(E, np.int32)
    waves = np.zeros(E, np.int32)
    eng._native.call("swarm_engine_window_stats", fb.ctypes.data, waves.ctypes.data)
    out = {"envs": E, "colloids_per_env": N, "path": "neighbour-list window", "ms_per_slice": ms,
           "value": E * N / (ms * 1e-3), "unit": "colloid-slices/s (100 sub-steps each)",
           "last_window_reruns": int((fb == 2).sum()), "last_window_flagged": int((fb == 1).sum())}
    del eng
    if global_reps > 0:
        for mode in ("cluster", "global"):
            g = make(mode)
            out[f"{mode}_path_ms_per_slice"] = time_slices(g, global_reps)
            del g
        out["speedup_vs_global_path"] = out["global_path_ms_per_slice"] / ms
    return out


def time_run_kernel(eng, ff, agent, episode_length, replays=3):
    """Duration (ms) of the dominant kernel -- the 2-D run kernel of the
    latency- (k_cluster_run_wide) or throughput-bound (k_cluster_run) cluster
    window -- as it runs in the workload: after the timed region
    one more episode of the workload is captured with engine profiling on,
    so every run node stamps its own earliest workgroup start and latest wave
    end on the device wall clock (and the other launches of the slice their
    workgroup roles), and that graph is replayed `replays` times; every
    replay's stamps are read back (swarm_engine_profile_stamps / _roles).
    Returns (mean ms, kernel name, note,
    number of run launches timed): the rocprofv3 trace of the same command
    holds those launches as the kernel's last dispatches
    (tools/summarize_profiles.py reads the count from the bench line)."""
    import ctypes

    import torch

    nat = eng._native
    wide = eng.n_envs * eng.n_particles <= 32768  # latency-bound engines
    name = ("k_cluster_run_wide (100 fused BD+WCA sub-steps; the next window's noise table "
            "filled beside them)" if wide else "k_cluster_run (100 fused BD+WCA sub-steps)")
    torch.cuda.synchronize()
    ms = ctypes.c_double()
    cnt = ctypes.c_int32()
    saved = agent.trajectory
    agent.reset_trajectory()
    samples = []
    how = (f"an episode graph of the workload captured after the timed region with engine "
           f"profiling on, {replays} replays")
    nat.call("swarm_engine_profile", 1, ctypes.byref(ms), ctypes.byref(cnt))
    graph = None
    try:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            eng.integrate(episode_length, ff)
    except RuntimeError as err:  # no event nodes in this HIP: eager episodes instead
        graph = None
        how = (f"HIP events around each run launch of {replays} eager episodes after the "
               f"timed region (graph event nodes refused: {err})")
    finally:
        nat.call("swarm_engine_profile", 0, ctypes.byref(ms), ctypes.byref(cnt))
    buf = (ctypes.c_float * 4096)()
    cal = (ctypes.c_float * 4096)()
    dev = (ctypes.c_float * 4096)()
    cal_samples, dev_samples = [], []
    n_roles = ctypes.c_int32(0)
    rbuf = (ctypes.c_double * (2 * 16 * 512))()
    role_samples = {}
    try:
        if graph is not None:
            for _ in range(replays):
                nat.call("swarm_engine_profile_stamps", 1,
                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), None, 0,
                         ctypes.byref(cnt))
                graph.replay()
                nat.call("swarm_engine_profile_graph", 0, buf, cal, 4096, ctypes.byref(cnt))
                samples.extend(buf[k] for k in range(min(cnt.value, 4096)))
                cal_samples.extend(cal[k] for k in range(min(cnt.value, 4096)))
                nat.call("swarm_engine_profile_stamps", 0, None, dev, 4096, ctypes.byref(cnt))
                dev_samples.extend(dev[k] for k in range(min(cnt.value, 4096)))
                nat.call("swarm_engine_profile_roles", rbuf, len(rbuf), ctypes.byref(n_roles))
                for k in range(min(cnt.value, 512)):
                    for q in range(n_roles.value):
                        b, e = rbuf[2 * (k * n_roles.value + q)], rbuf[2 * (k * n_roles.value + q) + 1]
                        if b == b and e == e:  # not NaN
                            role_samples.setdefault(q, []).append((b, e))
        else:
            torch.cuda.synchronize()
            agent.reset_trajectory()
            nat.call("swarm_engine_profile", 1, ctypes.byref(ms), ctypes.byref(cnt))
            for _ in range(replays):
                eng.integrate(episode_length, ff)
            nat.call("swarm_engine_profile", 0, ctypes.byref(ms), ctypes.byref(cnt))
            samples = [ms.value / max(cnt.value, 1)] * cnt.value
        eng.drain_trajectory(block=True)
    finally:
        del graph
        torch.cuda.synchronize()
        nat.call("swarm_engine_profile_graph", 1, None, None, 0, ctypes.byref(cnt))
        agent.trajectory = saved
    # the run kernel's own launch stamps (earliest block start, latest wave
    # end, device wall clock) time each run node as it ran in the replayed
    # workload; HIP events only where there are no stamps (eager episodes)
    dev_ok = [x for x in dev_samples if x > 0.0]
    if not dev_ok and not samples:  # no 2-D cluster windows (global path)
        return None, name, "no run-kernel launches recorded", 0, {}
    if dev_ok:
        mean = sum(dev_ok) / len(dev_ok)
        n_timed = len(dev_ok)
        note = (f"{how}: {n_timed} run nodes timed by their own start / end stamps (device "
                f"wall clock): mean {mean:.5f} ms, min {min(dev_ok):.5f}, max {max(dev_ok):.5f}")
    else:
        samples.sort()
        mean = sum(samples) / len(samples)
        n_timed = len(samples)
        note = (f"{how}: HIP events around {n_timed} run launches: mean {mean:.5f} ms, median "
                f"{samples[len(samples) // 2]:.5f}, min {samples[0]:.5f}, max {samples[-1]:.5f}")
    if samples and cal_samples:
        over = sum(cal_samples) / len(cal_samples)
        note += (f"; event-record nodes around the run node: mean {sum(samples) / len(samples):.5f}"
                 f" ms, an empty pair of them alone {over:.5f} ms")
    # the workgroup roles of the launches between run nodes (role stamps):
    # mean start / end after the previous run node's end, and mean duration
    names = ("k_check", "build sort", "vision grid", "field (reward)", "pair search",
             "vision cone", "cluster build", "policy MLP", "pair search: lists tested",
             "pair search: output reserved", "vision cone: bins summed")
    timeline = {}
    for q, v in sorted(role_samples.items()):
        timeline[names[q] if q < len(names) else f"role{q}"] = {
            "start_us": round(sum(b for b, _ in v) / len(v), 2),
            "end_us": round(sum(e for _, e in v) / len(v), 2),
            "dur_us": round(sum(e - b for b, e in v) / len(v), 2), "n": len(v)}
    return mean, name, note, n_timed, timeline


def time_ppo_grads(agent, traj, line, reps):
    """Roofline of the PPO update's dominant kernel, k_ppo_grads (the caller
    side of the rollout): one eager epoch of the episode
    `traj` whose gradient kernel is launched `reps` times back to back between
    two HIP events (swarm_ppo_profile), useful work = PPO_MAC_PER_SAMPLE
    multiply-adds per sample per launch against the f32 vector peak."""
    import ctypes

    import torch

    from swarmrl_amd import _capi

    lib = _capi.lib()
    ms, cnt = ctypes.c_double(), ctypes.c_int32()
    loss = agent.loss
    epochs = loss.n_epochs
    prev = os.environ.get("SWARMRL_AMD_PPO_GRAPH")
    os.environ["SWARMRL_AMD_PPO_GRAPH"] = "0"  # one eager epoch, events around its launches
    try:
        torch.cuda.synchronize()
        lib.swarm_ppo_profile(max(1, reps), ctypes.byref(ms), ctypes.byref(cnt))
        loss.n_epochs = 1
        loss.compute_loss(network=agent.network, episode_data=traj)
        lib.swarm_ppo_profile(0, ctypes.byref(ms), ctypes.byref(cnt))
    finally:
        loss.n_epochs = epochs
        if prev is None:
            del os.environ["SWARMRL_AMD_PPO_GRAPH"]
        else:
            os.environ["SWARMRL_AMD_PPO_GRAPH"] = prev
    if cnt.value == 0:
        return None  # not the fused path (another network or sampling strategy)
    kernel_ms = ms.value / cnt.value
    samples = len(traj.actions) * int(traj.actions[0].numel())
    tflops = 2.0 * PPO_MAC_PER_SAMPLE * samples / (kernel_ms * 1e-3) / 1e12
    out = {"bound": "valu", "kernel": "k_ppo_grads (one PPO epoch's gradient)",
           "achieved": tflops, "peak": F32_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": tflops / F32_VECTOR_PEAK_TFLOPS, "kernel_ms": kernel_ms,
           "kernel_timing": f"HIP events around {max(1, reps)} back-to-back launches of one "
                            f"epoch's gradient kernel, after the timed region",
           "samples_per_launch": samples,
           "algorithmic_flops": f"2 x {PPO_MAC_PER_SAMPLE} per sample (DESIGN.md 6) x {samples}"}
    row = profile_row(line, r"k_ppo_grads")
    if row:
        out["profile"] = {"source": row["source"], "src_sha": row.get("src_sha"),
                          "stale": bool(row.get("stale")),
                          "rocprof_timed_mean_ms": (row.get("mean_duration_timed_us") or 0.0) * 1e-3
                          or None,
                          "traffic": row.get("bytes_per_launch")}
    return out


def _round_key(path):
    """profiles/r<round><letter>_<line>_traffic.json -> sortable (round, letter)."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), m.group(2)) if m else (-1, "")


def profile_row(line, kernel_re):
    """The counter row of `line`'s dominant kernel from the newest committed
    config-pure profile (profiles/r*_traffic.json, tools/summarize_profiles.py):
    per-launch HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md
    gfx950 correction), VALU and transcendental wave-instructions, and the
    rocprofv3 mean duration.  A row of other sources than the ones built here
    is returned flagged stale."""
    import glob

    sha = source_sha()
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")), key=_round_key,
                   reverse=True)
    fallback = None
    for path in paths:
        try:
            with open(path) as f:
                rows = json.load(f)
        except (OSError, ValueError):
            continue
        for r in rows:
            if r.get("line") != line or not re.search(kernel_re, r.get("kernel", "")):
                continue
            r = dict(r, source=f"profiles/{os.path.basename(path)}")
            if r.get("src_sha") == sha:
                return r
            if fallback is None:
                fallback = dict(r, stale=True)
    return fallback


def make_roofline(line, kernel_re, kernel, kernel_ms, units, bytes_per_unit, unit_desc):
    """HBM roofline of one line's dominant kernel: algorithmic bytes per
    launch (SURVEY 8(d)'s per-unit figure x the units of one launch) over the
    live HIP-event launch duration, the counter traffic of the same kernel
    from its config-pure profile, and the VALU issue roofline from the
    profile's instruction counts."""
    bytes_per_launch = bytes_per_unit * units
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms else None
    row = profile_row(line, kernel_re)
    out = {
        "bound": "hbm",
        "kernel": kernel,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved else None,
        "traffic": row["bytes_per_launch"] if row else None,
        "kernel_ms": kernel_ms,
        "bytes_per_launch": bytes_per_launch,
        "algorithmic_bytes": f"{bytes_per_unit} B per {unit_desc} (SURVEY 8d) x {units}",
    }
    if row:
        out["profile"] = {"source": row["source"], "src_sha": row.get("src_sha"),
                          "stale": bool(row.get("stale")),
                          "rocprof_timed_mean_ms": (row.get("mean_duration_timed_us") or 0.0) * 1e-3
                          or None,
                          "rocprof_graph_mean_ms": (row.get("mean_duration_graph_us") or 0.0) * 1e-3
                          or None,
                          "launches": row.get("dispatches")}
        valu, trans = row.get("valu_insts_per_launch"), row.get("valu_trans_per_launch")
        if valu and kernel_ms:
            # issue cycles the launch needs on its SIMDs over the cycles the
            # chip offers in the measured duration
            cycles = VALU_CYCLES * (valu - (trans or 0.0)) + TRANS_CYCLES * (trans or 0.0)
            out["valu"] = {
                "achieved": valu / (kernel_ms * 1e-3),
                "peak": VALU_PEAK_WAVE_INSTS,
                "unit": "VALU wave-instructions/s",
                "frac": cycles / (SIMD_CLOCKS_PER_S * kernel_ms * 1e-3),
                "issue_model": f"{VALU_CYCLES} cycles per VALU, {TRANS_CYCLES} per transcendental "
                               f"wave-instruction (MI355X_MICROARCH.md:489)"
                               + ("" if trans is not None else "; transcendentals not counted"),
                "insts_per_launch": valu,
                "trans_per_launch": trans,
            }
    return out


def _cpu_env(N, slices, seed, threads=1, cells=True):
    """One env of the CPU comparator: the C restatement of the
    path -- cell-list WCA + Brownian dynamics, the vision cone over a cell
    list (cells=False: the reference's all-pairs loop), the field reward --
    plus the torch-CPU policy, on `threads` threads (OpenMP over particles /
    agents in the C code, torch intra-op threads for the MLP).  Returns
    (agent-steps, seconds) of the timed loop (after setup)."""
    import torch

    from oracle import oracle

    torch.set_num_threads(threads)
    oracle.set_threads(threads)
    L = 2.0 * math.sqrt(N / 0.1)
    box = [L, L, L]
    rng = np.random.default_rng(seed)
    r = L / 2 * np.sqrt(rng.random(N))
    th = 2 * np.pi * rng.random(N)
    pos = np.stack([L / 2 + r * np.cos(th), L / 2 + r * np.sin(th), np.zeros(N)], 1)
    a = 2 * np.pi * rng.random(N)
    dirs = np.stack([np.cos(a), np.sin(a), np.zeros(N)], 1)
    gt = 6 * np.pi * (1e-3 / 4.0453e-3)
    gr = 8 * np.pi * (1e-3 / 4.0453e-3)
    kT = 300.0 / 293.0
    p = oracle.make_params(box, 1e-3, kT, kT, seed, [(1.0, gt, gr, 1.0358e-6, 4.143e-7)])
    st = oracle.state_from_positions(pos, dirs, box)
    sp = np.zeros(N, np.uint8)
    st, _ = oracle.sd_run(p, st, sp, 1000)
    agents = np.arange(N)
    hist = oracle.history_from_state(st, agents)
    net = torch.nn.Sequential(torch.nn.Linear(3, 128), torch.nn.ReLU(), torch.nn.Linear(128, 5))
    ftab = np.array([0.0, 10.0, 0.0, 0.0], np.float32)
    ttab = np.array([10.0, 0.0, -10.0, 0.0], np.float32)
    src = np.array([L / 2, L / 2, 0.0])
    ones, zeros = np.ones(N, np.float32), np.zeros(N, np.int32)
    t0 = time.perf_counter()
    for s in range(slices):
        obs = oracle.vision_cone(p, st, agents, ones, zeros, 10.0, np.pi / 2, 3, [0], cells=cells)
        with torch.no_grad():
            logits = net(torch.as_tensor(obs.reshape(N, 3)))[:, :4]
            u = torch.rand(logits.shape)
            idx = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1).numpy()
            torch.log(torch.softmax(logits, -1) + 1e-8)
        st, _, _ = oracle.bd_run(p, st, sp, ftab[idx], ttab[idx], 100, step0=100 * s)
        dc, dp = oracle.field_distance(p, st, agents, src, np.array(box), hist)
        np.clip(10 * ((1 - dc) - (1 - dp)), 0, None)
    dt = time.perf_counter() - t0
    oracle.set_threads(1)
    return N * slices, dt


def _cpu_host():
    """CPU model and the cores this process may run on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    return model, avail


def cpu_baseline(args):
    """The CPU comparator on one 4096-colloid env, one thread, for a bounded
    number of slices (the reference CI runs single-threaded,
    .github/workflows/espresso.yml:41)."""
    import torch

    torch_threads = torch.get_num_threads()
    try:
        steps, dt = _cpu_env(args.colloids, args.cpu_sample_slices, 42, threads=1, cells=True)
    finally:
        torch.set_num_threads(torch_threads)
    model, avail = _cpu_host()
    return {
        "value": steps / dt,
        "unit": "agent-steps/s",
        "cores": 1,
        "kind": "port",
        "cpu_model": model,
        "nproc": avail,
        "sample": f"{args.cpu_sample_slices} slices x {args.colloids} colloids (1 env, 100 "
                  f"sub-steps each; cell-list WCA and vision cone, C restatement + torch-CPU "
                  f"policy) on 1 host core, {dt:.1f} s",
    }


def cpu_baseline_all_pairs(args):
    """Context row: the same with the reference's all-pairs vision cone
    (subdivided_vision_cones.py:178-205 is O(N^2)), a short sample."""
    import torch

    torch_threads = torch.get_num_threads()
    try:
        steps, dt = _cpu_env(args.colloids, args.cpu_all_pairs_slices, 42, threads=1, cells=False)
    finally:
        torch.set_num_threads(torch_threads)
    return {
        "value": steps / dt,
        "unit": "agent-steps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{args.cpu_all_pairs_slices} slices x {args.colloids} colloids with the "
                  f"reference's all-pairs vision cone, 1 core, {dt:.1f} s (context, not the "
                  f"comparator)",
    }


def cpu_baseline_all_cores(args):
    """The CPU comparator with OpenMP over the particles / agents of one env
    on all the cores this process may use (up to the 16-core share of a
    one-GPU box), torch intra-op threads for the policy."""
    import torch

    model, avail = _cpu_host()
    cores = int(os.environ.get("OMP_NUM_THREADS") or avail)
    cores = max(1, min(cores, 16, avail))
    torch_threads = torch.get_num_threads()
    try:
        steps, dt = _cpu_env(args.colloids, args.cpu_all_core_slices, 42, threads=cores,
                             cells=True)
    finally:
        torch.set_num_threads(torch_threads)
    return {
        "value": steps / dt,
        "unit": "agent-steps/s",
        "cores": cores,
        "kind": "port",
        "cpu_model": model,
        "nproc": avail,
        "sample": f"{args.cpu_all_core_slices} slices x {args.colloids} colloids (1 env), "
                  f"OpenMP over particles and agents on {cores} threads, {dt:.1f} s",
    }


def capture_episode(eng, ff, agent, T):
    """Two eager warm-up slices on a side stream, then the graphs the bench
    replays: one per slice (for step counts that are not a multiple of T) and
    one per episode, whose T slices write T distinct trajectory tensors, so
    replaying it records a whole episode with no copies (agent.trajectory
    holds references to those tensors).  Returns (slice graph, episode graph,
    the trajectory of the eager slices so far)."""
    import torch

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            eng.integrate(1, ff)
    torch.cuda.current_stream().wait_stream(side)
    warm = agent.trajectory
    agent.reset_trajectory()
    slice_graph = torch.cuda.CUDAGraph()
    # thread-local capture: a process group's watchdog thread polls its
    # collectives' events during the capture (global mode fails those
    # queries: hipErrorStreamCaptureUnsupported, seen on a world-1 RCCL group)
    with torch.cuda.graph(slice_graph, capture_error_mode="thread_local"):
        eng.integrate(1, ff)
    agent.reset_trajectory()
    episode_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(episode_graph, pool=slice_graph.pool(),
                          capture_error_mode="thread_local"):
        # one episode as the trainers run it (episodic_trainer.py:35 ->
        # engine.integrate(episode_length, force_fn))
        eng.integrate(T, ff)
    return slice_graph, episode_graph, warm


def measure(args, E, rank, world, device, builder=None, colloids=None, line="head",
            train=False):
    """Build, capture and time one workload of E envs per GPU; returns the
    timing and roofline numbers (all ranks).  train: each episode is also
    followed by the agent's PPO update (ProximalPolicyLoss.compute_loss,
    proximal_policy_loss.py:140-170) inside the timed region."""
    import torch
    import torch.distributed as dist

    from swarmrl_amd.rollout import (broadcast_agent, gather_episode, gather_trajectory,
                                     replicated_update)

    args_e = argparse.Namespace(**vars(args))
    args_e.envs_per_gpu = E
    if colloids is not None:
        args_e.colloids = colloids
    args = args_e
    from swarmrl_amd.rollout import shard_envs

    # this rank's contiguous block of the world * E envs (rollout.shard_envs):
    # env g is placed with default_rng(42 + g) (swarm_engine.add_colloids)
    envs = shard_envs(world * E, rank, world)
    eng, ff, agent = (builder or build_workload)(args_e, 42 + envs[0], device)
    # the collectives run at world > 1, or through a world-1 group when forced
    coll = world > 1 or getattr(args, "force_collective", False)
    if train and coll:
        broadcast_agent(agent)  # rank 0's replica everywhere (EpisodeParallelTrainer)
    eng.integrate(1, ff)  # setup, overlap removal, first slice (eager)

    def one_slice():
        eng.integrate(1, ff)

    T = args.episode_length
    slice_graph = episode_graph = None
    if not args.no_graph:
        slice_graph, episode_graph, _ = capture_episode(eng, ff, agent, T)
    else:
        agent.reset_trajectory()

    gstats = []
    n_updates = [0]

    def episode_end(timed):
        """After an episode: the update (train) and the trajectory gather.
        At world > 1 every rank all-gathers the episode's trajectory (one
        packed collective) and, when training, runs the identical update on
        the gathered [T, world E, ...] episode (rollout.replicated_update,
        SURVEY 8(e)); at world 1 the update runs on the local episode."""
        traj = agent.trajectory  # in graph mode: the episode graph's output tensors
        st = {} if (timed and coll and len(gstats) < 4) else None
        if train:
            n_updates[0] += 1
            if coll:
                episode = gather_episode(traj, stats=st)
                replicated_update(agent, episode, seed=1000 + n_updates[0])
            else:
                agent.loss.compute_loss(network=agent.network, episode_data=traj)
        elif timed and coll:
            gather_trajectory(traj, stats=st)
        if st:
            gstats.append(st)
        # trajectory entries the device has published so far (the ring is
        # filled by the replayed graph; no host wait)
        eng.drain_trajectory(block=False)

    def run(n_steps, timed):
        k = 0
        while k < n_steps:
            if episode_graph is not None and n_steps - k >= T:
                episode_graph.replay()
                k += T
                episode_end(timed)
            elif slice_graph is not None:
                slice_graph.replay()
                k += 1
            else:
                one_slice()
                k += 1
                if len(agent.trajectory.actions) >= T:
                    episode_end(timed)
                    agent.reset_trajectory()

    if episode_graph is not None:
        # the first launch of a captured graph uploads it: one untimed
        # episode replay (and its update) before the W warmup steps, so the
        # timed region never holds a graph's first launch
        run(T, False)
    run(args.warmup, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    import ctypes

    wstats = (ctypes.c_uint64 * 4)()
    eng._native.call("swarm_engine_build_stats", None, 1)  # (not under capture: counts windows)
    t0 = time.perf_counter()
    run(args.steps, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    eng._native.call("swarm_engine_build_stats", wstats, 0)
    timing = _finish_timing(args, E, world, device, elapsed, gstats, None, None)
    timing["windows"] = {
        "checked": int(wstats[3]),
        "pairs_from_candidate_lists": int(wstats[0]),
        "pairs_after_waiting_for_the_sort": int(wstats[1]),
        "exact_reruns": int(wstats[2]),
        "note": "timed region, all envs of this rank: the slice's pair search filtered the "
                "lists built during the previous run (hit) or waited for the fresh sort (miss); "
                "re-runs: windows the exact check sent to the global path",
    }

    eng.drain_trajectory(block=True)
    traj_written = eng.h5_time_steps_written + len(eng.traj_holder["Times"])
    kernel_ms, kernel, timing_note, timed_launches, timeline = time_run_kernel(eng, ff, agent, T)
    N = args.colloids
    sub = eng.params.steps_per_slice
    out = dict(timing)
    out.update({
        "hip_graph": episode_graph is not None,
        "trajectory": {"write_interval_s": args.write_interval, "entries_recorded": traj_written,
                       "recorder": "device ring (swarm_engine_traj_record) inside the graph"
                       if eng._ring is not None else "host"},
        # the 2-D run kernels (not k_cluster_run3 of the dims3 line)
        "roofline": make_roofline(line, r"k_cluster_run(_wide)?<", kernel, kernel_ms,
                                  N * sub * E, BYTES_PER_PARTICLE_SUBSTEP,
                                  f"colloid-sub-step; {N} colloids x {sub} sub-steps x {E} env(s)"),
        "src_sha": source_sha(),
    })
    out["roofline"]["kernel_timing"] = timing_note
    out["roofline"]["kernel_timing_launches"] = timed_launches
    if timeline:
        # after each run node: its check, then the next window's build and
        # observable workgroups (device wall-clock role stamps, same replays)
        out["slice_timeline_us"] = timeline
    valu = out["roofline"].get("valu")
    if valu:
        valu["lane_insts_per_colloid_substep"] = valu["insts_per_launch"] * 64 / (N * sub * E)
    if train:
        traj = agent.trajectory  # the episode graph's tensors (eager: the last episode's)
        if len(traj.actions) > 0:
            out["roofline_update"] = time_ppo_grads(agent, traj, line, args.bd_reps)
    del eng, ff, agent, slice_graph, episode_graph
    torch.cuda.synchronize()
    return out


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run
    would) before anything touches the GPU, wait for all, return the worst
    exit code.  Rank 0 prints the JSON line.  The reference's fan-out this
    replaces is training_routines/ensemble_submit.py:76-85."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def stub_measure(args, E, rank, world, device):
    """--stub: the launch / rendezvous / gather / max-over-ranks plumbing
    without a GPU (CPU tests): a synthetic trajectory of the bench's shapes
    (E envs x colloids agents, episode_length slices) is all-gathered once
    per episode, the 'rollout' is a host sleep."""
    import torch
    import torch.distributed as dist

    from swarmrl_amd.rollout import gather_trajectory
    from swarmrl_amd.utils.colloid_utils import TrajectoryInformation

    T, A = args.episode_length, args.colloids
    traj = TrajectoryInformation(particle_type=0)
    for t in range(T):
        traj.features.append(torch.full((E, A, 3), float(rank), device=device))
        traj.actions.append(torch.full((E, A), rank, dtype=torch.int64, device=device))
        traj.log_probs.append(torch.zeros((E, A), device=device))
        traj.rewards.append(torch.zeros((E, A), device=device))
    gstats = []
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(0, args.steps, T):
        time.sleep(1e-4 * min(T, args.steps - k))
        st = {}
        out = gather_trajectory(traj, stats=st)
        if st:
            gstats.append(st)
        assert out["actions"].shape[1] == world * E
        assert all(int(out["actions"][0, r * E, 0]) == r for r in range(world))
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return _finish_timing(args, E, world, device, elapsed, gstats, None, None, stub=True)


def _finish_timing(args, E, world, device, elapsed, gstats, kernel_ms, kernel, stub=False):
    """Per-rank values, max-over-ranks time, gather statistics."""
    import torch
    import torch.distributed as dist

    from swarmrl_amd.rollout import gather_ms

    N = args.colloids
    mine = N * E * args.steps / elapsed
    per_rank = [mine]
    if world > 1:
        t = torch.tensor([elapsed, mine], dtype=torch.float64, device=device)
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        elapsed = max(float(v[0]) for v in allv)
        per_rank = [float(v[1]) for v in allv]
    out = {
        "E": E,
        "value": N * E * world * args.steps / elapsed,
        "ms_per_step": elapsed / args.steps * 1e3,
        "per_rank": per_rank,
    }
    if gstats:
        out["gather"] = {
            "collective": "all_gather_into_tensor (one packed buffer per episode)",
            "bytes_per_rank": gstats[-1].get("bytes"),
            "ms_mean": sum(gather_ms(g) for g in gstats) / len(gstats),
            "per_run": len(gstats),
        }
    return out


def _sub_line(res, workload, extra=None):
    """A sub-line of the JSON record from a measure() result."""
    out = {"workload": workload, "value": res["value"], "unit": "agent-steps/s",
           "envs_per_gpu": res["E"], "ms_per_step": res["ms_per_step"],
           "per_rank_value": res["per_rank"], "roofline": res["roofline"]}
    for k in ("gather", "roofline_update", "slice_timeline_us", "windows"):
        if res.get(k) is not None:
            out[k] = res[k]
    out.update(extra or {})
    return out


def run_lines(args, lines, rank, world, device):
    """Measure the selected lines; returns {line: record}."""
    res = {}
    if "head" in lines:
        res["head"] = measure(args, args.envs_per_gpu, rank, world, device, line="head")
    if "batched" in lines and args.batched_envs > 0:
        r = measure(args, args.batched_envs, rank, world, device, line="batched")
        res["batched"] = _sub_line(r, f"{args.batched_envs} envs x {args.colloids} colloids per "
                                      f"GPU batched per launch, the headline's slice")
    if "c2" in lines and args.c2_colloids > 0:
        r = measure(args, 1, rank, world, device, colloids=args.c2_colloids, line="c2")
        res["c2"] = _sub_line(r, f"BASELINE config 2: {args.c2_colloids} colloids, WCA + "
                                 f"vision-cone observable, random-init MLP policy, one env per GPU")
    if "c4" in lines and args.c4_envs > 0:
        r = measure(args, args.c4_envs, rank, world, device, colloids=args.c4_colloids, line="c4")
        res["c4"] = _sub_line(r, f"BASELINE config 4 per-rank shard: {args.c4_envs} envs x "
                                 f"{args.c4_colloids} colloids per GPU (64 x {args.c4_colloids} "
                                 f"over 8 GPUs), vision cone + MLP, trajectory all-gather per "
                                 f"episode when world > 1")
    if "c5" in lines and args.c5_colloids > 0:
        r = measure(args, 1, rank, world, device, builder=build_c5_workload,
                    colloids=args.c5_colloids, line="c5")
        res["c5"] = _sub_line(r, f"BASELINE config 5: {args.c5_colloids} colloids, "
                                 f"ConcentrationField observable + GradientSensing reward + RND "
                                 f"intrinsic reward, one env per GPU")
    if "c3train" in lines and args.train_episodes > 0:
        targs = argparse.Namespace(**vars(args))
        T = args.episode_length
        targs.steps = args.train_episodes * T
        targs.warmup = max(args.warmup, 2 * T)  # eager first update, then the PPO graph capture
        r = measure(targs, 1, rank, world, device, builder=build_c3_workload, colloids=4096,
                    line="c3train", train=True)
        res["c3train"] = _sub_line(r, "BASELINE config 3: 4096 colloids, find-centre task "
                                      "(ConcentrationField + GradientSensing), actor-critic PPO "
                                      "training: each 20-slice episode's rollout and its PPO "
                                      "update (20 epochs, fused gradient kernels + Adam) timed "
                                      "together", {"episodes": args.train_episodes})
    if world == 1:
        for key, dims, frac, desc in (
                ("dims3", 3, 0.04, "3-D at scale: {N} colloids per env, periodic box at volume "
                                   "fraction 0.04, BD+WCA slices of 100 sub-steps (engine only)"),
                ("dense2d", 2, 0.3, "dense 2-D: {N} colloids per env at area fraction 0.3 "
                                    "(placed in the centred disc), BD+WCA slices of 100 "
                                    "sub-steps (engine only); the rc + skin graph percolates")):
            if key in lines and args.dims3:
                res[key] = {
                    "workload": desc.format(N=args.colloids),
                    "E1": measure_dims3(args, 1, 50, global_reps=3, dims=dims, fraction=frac),
                    f"E{args.batched_envs}": measure_dims3(args, max(args.batched_envs, 1), 20,
                                                           global_reps=2, dims=dims,
                                                           fraction=frac),
                }
    return res


def main():
    args = parse_args()
    lines = LINES if args.only == "all" else tuple(x.strip() for x in args.only.split(","))
    bad = [x for x in lines if x not in LINES]
    if bad:
        print(f"bench.py: unknown line(s) {bad}; choose from {LINES}", file=sys.stderr)
        sys.exit(2)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if args.stub:
        if world > 1:
            dist.init_process_group("gloo", init_method="env://")
        device = torch.device("cpu")
        head = stub_measure(args, args.envs_per_gpu, rank, world, device)
        head["roofline"] = None
        head["hip_graph"] = False
        res = {"head": head}
    else:
        if world > 1:
            dist.init_process_group("nccl", init_method="env://")
        elif args.force_collective:
            # one rank, one GPU: a world-size-1 RCCL group on a free local port
            import socket

            from swarmrl_amd.rollout import force_collectives

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                    world_size=1, device_id=torch.device("cuda", local_rank))
            force_collectives(True)
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        res = run_lines(args, lines, rank, world, device)
    if world > 1 and dist.get_world_size() != args.gpus:
        print("bench.py: process group size differs from --gpus", file=sys.stderr)
        sys.exit(2)
    N = args.colloids
    head = res.get("head")
    if head is None:  # a config-pure run of other lines: the first one heads the record
        name = next((k for k in lines if "value" in res.get(k, {})), None)
        rec = res.pop(name) if name else {"value": None, "ms_per_step": None, "roofline": None}
        head = dict(rec, E=rec.get("envs_per_gpu"), per_rank=rec.get("per_rank_value"))
        workload = f"{name}: {rec.get('workload')}"
    else:
        res.pop("head")
        workload = "4096-colloid WCA+vision-cone rollout"
    line = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "agent-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (uint32 fixed-point positions)",
        "data": "synthetic: seeded disc placement (area fraction 0.1), random-init actor-critic",
        "config": {
            "workload": workload,
            "colloids_per_env": N,
            "envs_per_gpu": head.get("E"),
            "substeps_per_slice": 100,
            "episode_length": args.episode_length,
            "policy": "MLP 3-128-(4+1), Gumbel sampling",
            "task": "GradientSensing (find centre)",
            "parallelism": f"episode-parallel, {world} process(es), one env per GPU, "
                           f"one packed all-gather of the trajectory per episode",
            "hip_graph": head.get("hip_graph"),
            "trajectory": head.get("trajectory"),
        },
        "world": world,
        "per_rank_value": head.get("per_rank"),
        "roofline": head["roofline"],
        "src_sha": source_sha(),
    }
    if "gather" in head:
        line["gather"] = head["gather"]
    if head.get("slice_timeline_us"):
        line["slice_timeline_us"] = head["slice_timeline_us"]
    if head.get("windows"):
        line["windows"] = head["windows"]
    for k in LINES:
        if k in res:
            line[k] = res[k]
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.stub:
        line["cpu_baseline"] = cpu_baseline(args)
        if args.cpu_all_core_slices > 0:
            line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(args)
        if args.cpu_all_pairs_slices > 0:
            line["cpu_baseline_all_pairs_vision"] = cpu_baseline_all_pairs(args)
    if args.force_collective and world == 1:
        line["config"]["parallelism"] += " (forced through a world-size-1 RCCL group)"
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1 or (args.force_collective and dist.is_initialized()):
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
