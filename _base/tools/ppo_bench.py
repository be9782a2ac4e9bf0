"""
Time one PPO epoch's gradient (swarm_ppo_epoch_grad) on an episode of E envs
x 4096 agents x T slices of the stock 1-128-(4+1) network, synthetic data:
the whole epoch (pack, values, GAE, gradient, reduce) by HIP events around
`reps` back-to-back epochs, and k_ppo_grads alone through swarm_ppo_profile.

usage: python tools/ppo_bench.py [E ...]     (default 1 64)
"""

import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(envs):
    from swarmrl_amd import _capi
    from swarmrl_amd.engine import ops
    from swarmrl_amd.networks.torch_network import ActorCriticMLP

    _capi.require_gpu()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    lib = _capi.lib()
    T, d, k, hidden, reps = 20, 1, 4, 128, 10
    for E in envs:
        S = E * 4096
        g = torch.Generator().manual_seed(E)
        torch.manual_seed(E)
        net = ActorCriticMLP(d, n_actions=k, hidden=hidden).to(dev)
        x = torch.randn(T, S, d, generator=g).to(dev)
        actions = torch.randint(0, k, (T, S), generator=g).to(dev)
        rewards = torch.randn(T, S, generator=g).to(dev)
        old = (-1.4 + 0.4 * torch.randn(T, S, generator=g)).to(dev)
        layers = [p.detach() for p in net.ppo_layers()]
        out = ops.ppo_epoch_grad(x, actions, old, rewards, layers, 0.99, 0.95, 0.2, 0.01)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.ppo_epoch_grad(x, actions, old, rewards, layers, 0.99, 0.95, 0.2, 0.01, out=out)
        e1.record()
        torch.cuda.synchronize()
        epoch_ms = e0.elapsed_time(e1) / reps
        ms, cnt = ctypes.c_double(0.0), ctypes.c_int32(0)
        lib.swarm_ppo_profile(reps, ctypes.byref(ms), ctypes.byref(cnt))
        ops.ppo_epoch_grad(x, actions, old, rewards, layers, 0.99, 0.95, 0.2, 0.01, out=out)
        torch.cuda.synchronize()
        lib.swarm_ppo_profile(0, ctypes.byref(ms), ctypes.byref(cnt))
        grads_ms = ms.value / max(1, cnt.value)
        n = T * S
        tflops = 2.0 * 2944 * n / (grads_ms * 1e-3) / 1e12
        print(f"E={E:3d} samples {n:9d}: epoch {epoch_ms * 1e3:8.1f} us, k_ppo_grads "
              f"{grads_ms * 1e3:8.1f} us ({tflops:.1f} TFLOP/s of 157.3), "
              f"grad norm {out.norm().item():.6e}", flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [1, 64])
