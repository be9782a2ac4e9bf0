// swarm_policy.cuh -- fused action sampling for the device rollout path.
//
// One kernel replaces the chain of small PyTorch kernels that turns policy
// logits into actions (rand, log, neg, log, sub, argmax, softmax, add, log,
// gather, table lookups):
//   idx  = argmax_j(logits_j - log(-log u_j))        gumbel_distribution.py:37-40
//   idx  = RandomExploration(idx)  (p > 0 only)       random_exploration.py:54-71
//   logp = log(softmax(logits)_idx + 1e-8)            flax_network.py:185-192
//   f_swim, torque_z = action tables[idx]             actor_critic.py:159-184
// Uniforms come from Philox4x32-10 keyed by a per-model seed, counter =
// (agent, call counter lo/hi, word block); the call counter lives in device
// memory and is advanced by the last workgroup, so a captured HIP graph
// draws fresh numbers on every replay.  Parity with the reference is
// statistical (its draws come from JAX's threefry), see tests.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swarm_device.cuh"

namespace swarm {

constexpr int kMaxActions = 64;

__device__ __forceinline__ float uniform24(uint32_t r) {
  return ((float)(r >> 8) + 0.5f) * 5.9604644775390625e-08f;  // (0, 1), 2^-24 grid
}

__global__ __launch_bounds__(256) void k_sample_actions(
    const float* __restrict__ logits, int n, int k, uint32_t key0, uint32_t key1,
    unsigned long long* __restrict__ state, float explore_p, const float* __restrict__ ftab,
    const float* __restrict__ ttab, int64_t* __restrict__ out_idx, float* __restrict__ out_logp,
    float* __restrict__ out_f, float* __restrict__ out_t) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long ctr = state[0];
  if (a < n) {
    const float* l = logits + (size_t)a * k;
    float best = -__builtin_inff(), m = -__builtin_inff();
    int idx = 0;
    for (int j0 = 0; j0 < k; j0 += 4) {
      u32x4 c = {(uint32_t)a, (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)(j0 >> 2)};
      const u32x4 r = philox4x32_10(c, key0, key1);
      const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = j0 + q;
        if (j < k) {
          const float lj = l[j];
          const float g = lj - logf(-logf(uniform24(rw[q])));
          if (g > best) {  // first maximum, as argmax
            best = g;
            idx = j;
          }
          m = fmaxf(m, lj);
        }
      }
    }
    if (explore_p > 0.0f) {
      u32x4 c = {(uint32_t)a, (uint32_t)ctr, (uint32_t)(ctr >> 32), 0x80000000u};
      const u32x4 r = philox4x32_10(c, key0, key1);
      // the reference's clip arithmetic, in fp32
      float tbc = fminf(fmaxf(uniform24(r.x) - explore_p, 0.0f), 1.0f);
      tbc = fminf(fmaxf(tbc * 1e6f, 0.0f), 1.0f);
      const float keep = fminf(fmaxf(tbc * -10.0f + 1.0f, 0.0f), 1.0f);
      const int rnd = min((int)(uniform24(r.y) * (float)k), k - 1);
      idx = (int)((float)idx * tbc + (float)rnd * keep);
    }
    float s = 0.0f;
    for (int j = 0; j < k; ++j) s += expf(l[j] - m);
    const float p = expf(l[idx] - m) / s;
    out_idx[a] = idx;
    out_logp[a] = logf(p + 1e-8f);
    out_f[a] = ftab[idx];
    out_t[a] = ttab[idx];
  }
  // every thread has read the counter; the last workgroup to arrive advances it
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned long long t = atomicAdd(&state[1], 1ull);
    if (t == gridDim.x - 1) {
      state[0] = ctr + 1ull;
      state[1] = 0ull;
      __threadfence();
    }
  }
}

}  // namespace swarm
