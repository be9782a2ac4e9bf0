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
# MI355X_MICROARCH.md: a wave issues a VALU instruction over 2 cycles; 1024
# SIMDs at 2.4 GHz -> 1.2288e12 VALU wave-instructions/s (= the 157.3 TF f32
# vector peak / (64 lanes x 2 flop))
VALU_PEAK_WAVE_INSTS = 1024 * 2.4e9 / 2
BYTES_PER_PARTICLE_SUBSTEP = 40


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


def build_c5_workload(args, env_seed, device):
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
    rnd = RNDReward(RNDConfig(input_shape=(1,), device=device))
    net = TorchModel(ActorCriticMLP(1, 4, 128), input_shape=(1,), device=device)
    actions = {
        "RotateClockwise": Action(torque=np.array([0.0, 0.0, 10.0])),
        "Translate": Action(force=10.0),
        "RotateCounterClockwise": Action(torque=np.array([0.0, 0.0, -10.0])),
        "DoNothing": Action(),
    }
    agent = ActorCriticAgent(0, net, task, obs, actions, train=True, intrinsic_reward=rnd)
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
        with torch.cuda.graph(graph):
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


def time_run_kernel(eng, reps):
    """Average duration (ms) of k_cluster_run, the dominant kernel: HIP events
    recorded by the engine around each launch on the stream it runs on
    (swarm_engine_profile), over `reps` eager 100-sub-step windows."""
    import ctypes

    import torch

    nat = eng._native
    ms = ctypes.c_double()
    cnt = ctypes.c_int32()
    eng._run(eng.params.steps_per_slice)
    torch.cuda.synchronize()
    nat.call("swarm_engine_profile", 1, ctypes.byref(ms), ctypes.byref(cnt))
    for _ in range(reps):
        eng._run(eng.params.steps_per_slice)
    nat.call("swarm_engine_profile", 0, ctypes.byref(ms), ctypes.byref(cnt))
    if cnt.value == 0:  # global path only (no cluster windows): whole windows
        start = torch.cuda.Event(enable_timing=True)
        stop = torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(reps):
            eng._run(eng.params.steps_per_slice)
        stop.record()
        stop.synchronize()
        return start.elapsed_time(stop) / reps, "k_global (100 sub-steps)"
    wide = eng.n_envs * eng.n_particles <= 32768  # latency-bound engines
    name = ("k_cluster_run_wide (100 fused BD+WCA sub-steps; the next window's noise table "
            "filled beside them)" if wide else "k_cluster_run (100 fused BD+WCA sub-steps)")
    return ms.value / cnt.value, name


def pmc_traffic(kernel_re, E, N):
    """Per-launch HBM bytes and VALU wave-instructions of the dominant kernel
    from the newest committed rocprofv3 PMC summary (profiles/<tag>_traffic.json:
    separate FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes, FETCH_SIZE x2 per
    MI355X_MICROARCH.md), when it was collected on this workload."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")), reverse=True)
    for path in paths:  # the newest round's summary first (r2b > r2a > r1)
        try:
            with open(path) as f:
                rows = json.load(f)
        except (OSError, ValueError):
            continue
        for r in rows:
            if re.search(kernel_re, r.get("kernel", "")) and r.get("envs") == E and \
                    r.get("colloids") == N:
                return (float(r["bytes_per_launch"]), r.get("valu_insts_per_launch"),
                        f"profiles/{r['source']}")
    return None, None, None


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


def measure(args, E, rank, world, device, builder=None, colloids=None):
    """Build, capture and time one workload of E envs per GPU; returns the
    timing and roofline numbers (all ranks)."""
    import torch
    import torch.distributed as dist

    from swarmrl_amd.rollout import gather_trajectory

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
    eng.integrate(1, ff)  # setup, overlap removal, first slice (eager)

    def one_slice():
        eng.integrate(1, ff)

    T = args.episode_length
    slice_graph = episode_graph = None
    if not args.no_graph:
        # One graph per slice (for step counts that are not a multiple of T)
        # and one per episode: the episode graph's T slices write T distinct
        # trajectory tensors, so replaying it records a whole episode with no
        # copies (agent.trajectory holds references to those tensors).
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                one_slice()
        torch.cuda.current_stream().wait_stream(side)
        slice_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(slice_graph):
            one_slice()
        agent.reset_trajectory()
        episode_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(episode_graph, pool=slice_graph.pool()):
            # one episode as the trainers run it (episodic_trainer.py:35 ->
            # engine.integrate(episode_length, force_fn))
            eng.integrate(T, ff)
    else:
        agent.reset_trajectory()

    gstats = []

    def run(n_steps, timed):
        k = 0
        while k < n_steps:
            if episode_graph is not None and n_steps - k >= T:
                episode_graph.replay()
                k += T
                # trajectory entries the device has published so far (the
                # ring is filled by the replayed graph; no host wait)
                eng.drain_trajectory(block=False)
                if timed and world > 1:
                    st = {}
                    gather_trajectory(agent.trajectory, stats=st if len(gstats) < 4 else None)
                    if st:
                        gstats.append(st)
            elif slice_graph is not None:
                slice_graph.replay()
                k += 1
            else:
                one_slice()
                k += 1
                if timed and world > 1 and len(agent.trajectory.actions) >= T:
                    gather_trajectory(agent.trajectory)
                    agent.reset_trajectory()

    run(args.warmup, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timing = _finish_timing(args, E, world, device, elapsed, gstats, None, None)

    eng.drain_trajectory(block=True)
    traj_written = eng.h5_time_steps_written + len(eng.traj_holder["Times"])
    kernel_ms, kernel = time_run_kernel(eng, args.bd_reps)
    N = args.colloids
    sub = eng.params.steps_per_slice
    bytes_per_launch = BYTES_PER_PARTICLE_SUBSTEP * N * sub * E
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    # the 2-D run kernels (not k_cluster_run3 of the dims3 line)
    traffic, valu, traffic_src = pmc_traffic(r"k_cluster_run(_wide)?<", E, N)
    out = dict(timing)
    out.update({
        "hip_graph": episode_graph is not None,
        "trajectory": {"write_interval_s": args.write_interval, "entries_recorded": traj_written,
                       "recorder": "device ring (swarm_engine_traj_record) inside the graph"
                       if eng._ring is not None else "host"},
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel_ms": kernel_ms,
            "bytes_per_launch": bytes_per_launch,
            "algorithmic_bytes": f"{BYTES_PER_PARTICLE_SUBSTEP} B per colloid-sub-step "
                                 f"(SURVEY 8d) x {N} colloids x {sub} sub-steps x {E} env(s)",
        },
    })
    if traffic_src:
        out["roofline"]["traffic_source"] = traffic_src
    if valu:
        # the bound that binds (SURVEY 8d asks for HBM; the fused kernel keeps
        # its state in registers, so VALU issue is what it runs into)
        out["roofline"]["valu"] = {
            "achieved": valu / (kernel_ms * 1e-3),
            "peak": VALU_PEAK_WAVE_INSTS,
            "unit": "VALU wave-instructions/s",
            "frac": valu / (kernel_ms * 1e-3) / VALU_PEAK_WAVE_INSTS,
            "insts_per_launch": valu,
            "lane_insts_per_colloid_substep": valu * 64 / (N * sub * E),
            "source": traffic_src,
        }
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


def main():
    args = parse_args()
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
        batched = None
    else:
        if world > 1:
            dist.init_process_group("nccl", init_method="env://")
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        E = args.envs_per_gpu
        head = measure(args, E, rank, world, device)
        batched = None
        if args.batched_envs > 0 and args.batched_envs != E:
            batched = measure(args, args.batched_envs, rank, world, device)
        if args.c5_colloids > 0:
            c5 = measure(args, 1, rank, world, device, builder=build_c5_workload,
                         colloids=args.c5_colloids)
            head["c5"] = {
                "workload": f"BASELINE config 5: {args.c5_colloids} colloids, ConcentrationField "
                            f"observable + GradientSensing reward + RND intrinsic reward, "
                            f"one env per GPU",
                "value": c5["value"],
                "unit": "agent-steps/s",
                "ms_per_step": c5["ms_per_step"],
                "per_rank_value": c5["per_rank"],
                "roofline": c5["roofline"],
            }
        if args.dims3 and world == 1:
            head["dims3"] = {
                "workload": f"3-D at scale: {args.colloids} colloids per env, periodic box at "
                            f"volume fraction 0.04, BD+WCA slices of 100 sub-steps (engine only)",
                "E1": measure_dims3(args, 1, 50, global_reps=3),
                f"E{args.batched_envs}": measure_dims3(args, max(args.batched_envs, 1), 20,
                                                       global_reps=2),
            }
            head["dense2d"] = {
                "workload": f"dense 2-D: {args.colloids} colloids per env at area fraction 0.3 "
                            f"(placed in the centred disc), BD+WCA slices of 100 sub-steps "
                            f"(engine only); the rc + skin graph percolates",
                "E1": measure_dims3(args, 1, 50, global_reps=3, dims=2, fraction=0.3),
                f"E{args.batched_envs}": measure_dims3(args, max(args.batched_envs, 1), 20,
                                                       global_reps=2, dims=2, fraction=0.3),
            }
    if world > 1 and dist.get_world_size() != args.gpus:
        print("bench.py: process group size differs from --gpus", file=sys.stderr)
        sys.exit(2)
    N = args.colloids
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
            "workload": "4096-colloid WCA+vision-cone rollout",
            "colloids_per_env": N,
            "envs_per_gpu": head["E"],
            "substeps_per_slice": 100,
            "episode_length": args.episode_length,
            "policy": "MLP 3-128-(4+1), Gumbel sampling",
            "task": "GradientSensing (find centre)",
            "parallelism": f"episode-parallel, {world} process(es), one env per GPU, "
                           f"one packed all-gather of the trajectory per episode",
            "hip_graph": head["hip_graph"],
            "trajectory": head.get("trajectory"),
        },
        "world": world,
        "per_rank_value": head["per_rank"],
        "roofline": head["roofline"],
    }
    if "gather" in head:
        line["gather"] = head["gather"]
    for k in ("c5", "dims3", "dense2d"):
        if k in head:
            line[k] = head[k]
    if batched is not None:
        line["batched"] = {
            "envs_per_gpu": batched["E"],
            "value": batched["value"],
            "unit": "agent-steps/s",
            "ms_per_step": batched["ms_per_step"],
            "per_rank_value": batched["per_rank"],
            "roofline": batched["roofline"],
        }
        if "gather" in batched:
            line["batched"]["gather"] = batched["gather"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.stub:
        line["cpu_baseline"] = cpu_baseline(args)
        if args.cpu_all_core_slices > 0:
            line["cpu_baseline_all_cores"] = cpu_baseline_all_cores(args)
        if args.cpu_all_pairs_slices > 0:
            line["cpu_baseline_all_pairs_vision"] = cpu_baseline_all_pairs(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
