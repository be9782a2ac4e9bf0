"""End-to-end PPO training cost on the bench workload (4096 colloids per env):
per episode, the rollout (20 slices through the engine) and the agent update
(GAE + n_epochs PPO steps).

  python tools/train_time.py [E]           eager rollout, as the trainers run it
  python tools/train_time.py [E] --graph   rollout replayed from one captured
                                           episode graph (as bench.py times it)

The update takes the fused device path (captured epochs from the second
episode on) unless SWARMRL_AMD_FUSED_PPO=0."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1
graph = "--graph" in sys.argv
torch.cuda.set_device(0)
ns = argparse.Namespace(colloids=4096, envs_per_gpu=E)
eng, ff, agent = bench.build_workload(ns, 42, torch.device("cuda", 0))
eng.integrate(1, ff)
T = 20
episode_graph = None
if graph:
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            eng.integrate(1, ff)
    torch.cuda.current_stream().wait_stream(side)
    agent.reset_trajectory()
    episode_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(episode_graph):
        eng.integrate(T, ff)
    traj = agent.trajectory  # the graph's output tensors, rewritten by every replay
else:
    agent.reset_trajectory()
steps = 0
t_all = 0.0
for ep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph:
        episode_graph.replay()
    else:
        eng.integrate(T, ff)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if graph:
        agent.loss.compute_loss(agent.network, traj)
    else:
        agent.update_agent()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if ep >= 2:  # after the first eager update and the PPO graph capture
        steps += E * 4096 * T
        t_all += t2 - t0
    print(f"episode {ep}: rollout {1e3 * (t1 - t0):7.2f} ms  update "
          f"({agent.loss.n_epochs} epochs) {1e3 * (t2 - t1):7.2f} ms", flush=True)
print(f"E={E} {'graph' if graph else 'eager'} rollout: training throughput "
      f"{steps / t_all / 1e6:.2f} M agent-steps/s (rollout + update, episodes 2-5)")
