"""Time the one-launch RND reward kernel alone (swarm_rnd_env_reward, HIP
events over 50 back-to-back calls) at C5's size: 16384 observations, d = 1.
usage: [SWARMRL_AMD_LIB=<variant .so>] python tools/rnd_time.py"""
import sys

import torch

sys.path.insert(0, ".")
from swarmrl_amd.engine import ops  # noqa: E402


def net(d):
    return torch.nn.Sequential(torch.nn.Linear(d, 32), torch.nn.ReLU(), torch.nn.Linear(32, 32),
                               torch.nn.ReLU(), torch.nn.Linear(32, 32)).cuda()


def main():
    torch.manual_seed(0)
    for n, d in ((16384, 1), (4096, 1), (65536, 1)):
        x = torch.rand(n, d, device="cuda")
        base = torch.rand(1, n, device="cuda")
        t, p = net(d), net(d)
        ws = {}
        ops.rnd_env_reward(x, 1, t, p, 2, (-5.0, 5.0), base, workspaces=ws)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.rnd_env_reward(x, 1, t, p, 2, (-5.0, 5.0), base, workspaces=ws)
        e1.record()
        torch.cuda.synchronize()
        print(f"n={n:6d} k_rnd_env {1e3 * e0.elapsed_time(e1) / 50:7.2f} us per call "
              "(incl. host launch)", flush=True)


if __name__ == "__main__":
    main()
