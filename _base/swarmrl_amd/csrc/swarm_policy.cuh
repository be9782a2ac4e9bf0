// swarm_policy.cuh -- the policy step of the device rollout path.
//
// Two kernels:
//
//   k_sample_actions     logits (any producer) -> actions.  Replaces the
//                        chain of small PyTorch kernels (rand, log, neg, log,
//                        sub, argmax, softmax, add, log, gather, table
//                        lookups).
//   k_policy_mlp_sample  the whole rollout policy in one launch: the MLP
//                        actor (Linear -> ReLU -> Linear, weights read in
//                        place from the torch module) and the same sampling.
//                        The critic head is not evaluated: the rollout never
//                        reads it (flax_network.py:174-195 returns actions
//                        and log-probs only).
//
// Sampling (both kernels, one device function, so they agree bit for bit on
// the same logits and counters):
//   idx  = argmax_j(logits_j - log(-log u_j))        gumbel_distribution.py:37-40
//   idx  = RandomExploration(idx)  (p > 0 only)       random_exploration.py:54-71
//   logp = log(softmax(logits)_idx + 1e-8)            flax_network.py:185-192
//   f_swim, torque_z = action tables[idx]             actor_critic.py:159-184
// Uniforms come from Philox4x32-10 keyed by a per-model seed, counter =
// (agent, call counter lo/hi, word block).  Call counters live in device
// memory, one per group of 64 agents (state[a >> 6]); the block that owns a
// group advances it after every thread has read it, so a captured HIP graph
// draws fresh numbers on every replay without any cross-workgroup atomics.
// Parity with the reference is statistical (its draws come from JAX's
// threefry), see tests.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swarm_device.cuh"

namespace swarm {

constexpr int kMaxActions = 64;
constexpr int kMlpMaxIn = 16;      // fused MLP: observable features per agent
constexpr int kMlpMaxHidden = 256;  // LDS: hidden x 36 floats <= 36 KB
constexpr int kMlpMaxActions = 16;

__device__ __forceinline__ float uniform24(uint32_t r) {
  return ((float)(r >> 8) + 0.5f) * 5.9604644775390625e-08f;  // (0, 1), 2^-24 grid
}

struct Sampled {
  int idx;
  float logp;
};

// Gumbel-max + exploration + log(softmax + 1e-8) of agent a over k logits
// read through L(j) (j < k); ctr = the agent's call counter.
template <typename Logit>
__device__ __forceinline__ Sampled sample_logits(Logit L, int k, int a,
                                                 unsigned long long ctr, uint32_t key0,
                                                 uint32_t key1, float explore_p) {
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
        const float lj = L(j);
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
  float s = 0.0f, li = 0.0f;
  for (int j = 0; j < k; ++j) {
    const float lj = L(j);
    s += expf(lj - m);
    li = j == idx ? lj : li;
  }
  const float p = expf(li - m) / s;
  return {idx, logf(p + 1e-8f)};
}

// sample_logits over logits held in registers (lg[K], K the padded width):
// every loop is unrolled over compile-time indices guarded by q < k, so no
// logit is read through a run-time index (which spilled lg to scratch for
// K = 16).  Same draws and operation sequence as sample_logits.
template <int K>
__device__ __forceinline__ Sampled sample_logits_reg(const float (&lg)[K], int k, int a,
                                                     unsigned long long ctr, uint32_t key0,
                                                     uint32_t key1, float explore_p) {
  float best = -__builtin_inff(), m = -__builtin_inff();
  int idx = 0;
#pragma unroll
  for (int j0 = 0; j0 < K; j0 += 4) {
    if (j0 < k) {
      u32x4 c = {(uint32_t)a, (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)(j0 >> 2)};
      const u32x4 r = philox4x32_10(c, key0, key1);
      const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = j0 + q;
        if (j < k) {
          const float lj = lg[j];
          const float g = lj - logf(-logf(uniform24(rw[q])));
          if (g > best) {  // first maximum, as argmax
            best = g;
            idx = j;
          }
          m = fmaxf(m, lj);
        }
      }
    }
  }
  if (explore_p > 0.0f) {
    u32x4 c = {(uint32_t)a, (uint32_t)ctr, (uint32_t)(ctr >> 32), 0x80000000u};
    const u32x4 r = philox4x32_10(c, key0, key1);
    float tbc = fminf(fmaxf(uniform24(r.x) - explore_p, 0.0f), 1.0f);
    tbc = fminf(fmaxf(tbc * 1e6f, 0.0f), 1.0f);
    const float keep = fminf(fmaxf(tbc * -10.0f + 1.0f, 0.0f), 1.0f);
    const int rnd = min((int)(uniform24(r.y) * (float)k), k - 1);
    idx = (int)((float)idx * tbc + (float)rnd * keep);
  }
  float s = 0.0f, li = 0.0f;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (j < k) {
      s += expf(lg[j] - m);
      li = j == idx ? lg[j] : li;
    }
  }
  const float p = expf(li - m) / s;
  return {idx, logf(p + 1e-8f)};
}

// The block's threads have all read their group counters: advance them.
// Groups of 64 agents never straddle a block (agents per block % 64 == 0).
__device__ __forceinline__ void advance_group_counter(unsigned long long* state, int a, int n,
                                                      bool leader, unsigned long long ctr) {
  __syncthreads();
  if (leader && a < n && (a & 63) == 0) state[a >> 6] = ctr + 1ull;
}

__global__ __launch_bounds__(256) void k_sample_actions(
    const float* __restrict__ logits, int n, int k, uint32_t key0, uint32_t key1,
    unsigned long long* __restrict__ state, float explore_p, const float* __restrict__ ftab,
    const float* __restrict__ ttab, int64_t* __restrict__ out_idx, float* __restrict__ out_logp,
    float* __restrict__ out_f, float* __restrict__ out_t) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long ctr = a < n ? state[a >> 6] : 0ull;
  if (a < n) {
    const float* l = logits + (size_t)a * k;
    const Sampled s =
        sample_logits([&](int j) { return l[j]; }, k, a, ctr, key0, key1, explore_p);
    out_idx[a] = s.idx;
    out_logp[a] = s.logp;
    out_f[a] = ftab[s.idx];
    out_t[a] = ttab[s.idx];
  }
  advance_group_counter(state, a, n, true, ctr);
}

// LDS row of hidden unit j: [W1[j][0..D) | b1[j] 0 0 0 | W2[0..K)[j]],
// zero-padded to the template widths (padding adds exact zeros).
template <int D, int K>
struct MlpRow {
  static constexpr int kStride = D + 4 + K;  // floats, a multiple of 4
};

// One agent per G lanes; lane `sub` of an agent takes hidden units
// j = sub, sub + G, ...; the partial logits are summed with xor-shuffles.
// D, K: padded widths of the observable and of the action set.
// The policy's launch arguments (one struct, so fused launches can carry it).
struct MlpArgs {
  const float* obs;
  int n, d_in;
  const float* w1;
  const float* b1;
  int hidden;
  const float* w2;
  const float* b2;
  int k;
  uint32_t key0, key1;
  unsigned long long* state;
  float explore_p;
  const float* ftab;
  const float* ttab;
  int64_t* out_idx;
  float* out_logp;
  float* out_f;
  float* out_t;
  float* out_logits;
};

// Body for block vb of the policy (k_policy_mlp_sample, or a workgroup of a
// fused launch: k_policy_cbuild); sw: the block's dynamic LDS.
template <int G, int D, int K>
__device__ __forceinline__ void policy_body(const MlpArgs& m, int vb, float* sw) {
  const float* __restrict__ obs = m.obs;
  const int n = m.n, d_in = m.d_in, hidden = m.hidden, k = m.k;
  const float* __restrict__ w1 = m.w1;
  const float* __restrict__ b1 = m.b1;
  const float* __restrict__ w2 = m.w2;
  const float* __restrict__ b2 = m.b2;
  const uint32_t key0 = m.key0, key1 = m.key1;
  unsigned long long* __restrict__ state = m.state;
  const float explore_p = m.explore_p;
  const float* __restrict__ ftab = m.ftab;
  const float* __restrict__ ttab = m.ttab;
  int64_t* __restrict__ out_idx = m.out_idx;
  float* __restrict__ out_logp = m.out_logp;
  float* __restrict__ out_f = m.out_f;
  float* __restrict__ out_t = m.out_t;
  float* __restrict__ out_logits = m.out_logits;
  constexpr int R = MlpRow<D, K>::kStride;
  // the weights into LDS rows, four entries per thread loaded together
  for (int t0 = threadIdx.x; t0 < hidden * R; t0 += 4 * (int)blockDim.x) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u * (int)blockDim.x;
      const int j = t / R, c = t - j * R;
      v[u] = 0.0f;
      if (t < hidden * R) {
        if (c < D) {
          v[u] = c < d_in ? w1[(size_t)j * d_in + c] : 0.0f;
        } else if (c == D) {
          v[u] = b1[j];
        } else if (c >= D + 4) {
          const int q = c - D - 4;
          v[u] = q < k ? w2[(size_t)q * hidden + j] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u * (int)blockDim.x < hidden * R) sw[t0 + u * (int)blockDim.x] = v[u];
  }
  float* sb2 = sw + hidden * R;
  if (threadIdx.x < K) sb2[threadIdx.x] = (int)threadIdx.x < k ? b2[threadIdx.x] : 0.0f;
  const int gt = vb * blockDim.x + threadIdx.x;
  const int a = gt / G, sub = gt & (G - 1);
  const bool valid = a < n;
  const unsigned long long ctr = valid ? state[a >> 6] : 0ull;
  float x[D];
#pragma unroll
  for (int c = 0; c < D; ++c) x[c] = (valid && c < d_in) ? obs[(size_t)a * d_in + c] : 0.0f;
  __syncthreads();
  float acc[K];
#pragma unroll
  for (int q = 0; q < K; ++q) acc[q] = 0.0f;
  for (int j = sub; j < hidden; j += G) {
    const float4* r = reinterpret_cast<const float4*>(sw + j * R);
    float w[R];
#pragma unroll
    for (int v = 0; v < R / 4; ++v) {
      const float4 t4 = r[v];
      w[4 * v + 0] = t4.x;
      w[4 * v + 1] = t4.y;
      w[4 * v + 2] = t4.z;
      w[4 * v + 3] = t4.w;
    }
    float h = 0.0f;
#pragma unroll
    for (int c = 0; c < D; ++c) h = fmaf(w[c], x[c], h);
    h = fmaxf(h + w[D], 0.0f);  // bias + ReLU
#pragma unroll
    for (int q = 0; q < K; ++q) acc[q] = fmaf(h, w[D + 4 + q], acc[q]);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
#pragma unroll
    for (int q = 0; q < K; ++q) acc[q] += __shfl_xor(acc[q], o, 64);
  }
  float lg[K];
#pragma unroll
  for (int q = 0; q < K; ++q) lg[q] = acc[q] + sb2[q];
  if (valid && sub == 0) {
    const Sampled s = sample_logits_reg<K>(lg, k, a, ctr, key0, key1, explore_p);
    out_idx[a] = s.idx;
    out_logp[a] = s.logp;
    out_f[a] = ftab[s.idx];
    out_t[a] = ttab[s.idx];
    if (out_logits) {
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < k) out_logits[(size_t)a * k + q] = lg[q];
    }
  }
  advance_group_counter(state, a, n, sub == 0, ctr);
}

template <int G, int D, int K>
__global__ __launch_bounds__(256) void k_policy_mlp_sample(MlpArgs m) {
  extern __shared__ __align__(16) float sw[];
  policy_body<G, D, K>(m, blockIdx.x, sw);
}

}  // namespace swarm
