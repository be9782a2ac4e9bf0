// swarm_ppo.cuh -- the gradient of one PPO epoch of the actor-critic MLP.
//
// The caller side of the rollout: ProximalPolicyLoss.compute_loss
// (swarmrl/losses/proximal_policy_loss.py:140-170) takes n_epochs gradient
// steps per episode on _calculate_loss (:62-138).  With torch autograd an
// epoch over 64 envs x 4096 agents x 20 slices (5.2 M samples) costs ~24 ms,
// 50x the rollout of the episode.  Here the gradient of an epoch is four
// launches over the episode's samples, for the stock network Dense(hidden)
// -> ReLU -> {Dense(k) logits, Dense(1) value}:
//
//   k_ppo_values  V = critic(relu(W1 x + b1)) of every sample
//   k_ppo_gae     per agent column: the generalized advantages and returns
//                 (generalized_advantage_estimate.py:42-72), the sum and sum
//                 of squares of the advantages (fp64 block partials, summed
//                 in a fixed order by each grads workgroup, for their
//                 normalisation), and dL/dV of the critic term -- which, as
//                 in the reference, differentiates the returns too
//                 (R = A + V is built from the predicted values; only the
//                 normalised advantages are stop_gradient-ed, :124)
//   k_ppo_grads   per sample: forward, the gradient of the clipped surrogate
//                 and the entropy term (eps = 1e-8) w.r.t. the logits, back
//                 through both layers; each block sums its samples'
//                 parameter gradients in registers
//   k_ppo_reduce  block partials -> the gradient of every parameter (fp64
//                 sums in a fixed order: deterministic), torch layouts
//
// The loss is a sum over samples, so its gradient is the sum of the
// per-sample gradients; the caller's optimizer takes the step.  Before them,
// k_ppo_pack lays the parameters out as per-unit rows (the wave-uniform
// scalar-load operands of the sample-major loops).  All fp32 arithmetic with
// explicit fmaf; cross-sample sums in a fixed order (run-to-run identical).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swarm {

constexpr int kPpoMaxIn = 32;
constexpr int kPpoMaxK = 16;
constexpr int kPpoMaxHidden = 256;
constexpr int kPpoBlocks = 2048;  // grad blocks (one or two waves each)

// Gradient layout (floats): W1 [H][D] | b1 [H] | Wa [K][H] | ba [K] | Wc [H] | bc
__host__ __device__ inline int ppo_grad_size(int d, int h, int k) {
  return h * d + h + k * h + k + h + 1;
}

// Per-unit parameter rows, the wave-uniform operands of the sample-major
// loops (one scalar-load row per unit): [Wa[:, u], Wc[u], 0 ... | W1[u, :], b1[u], 0 ...]
template <int D, int K>
struct PpoTable {
  static constexpr int kHeads = (K + 1 + 7) / 8 * 8;
  static constexpr int kW1 = kHeads;
  static constexpr int kB1 = kHeads + D;
  static constexpr int kStride = kHeads + (D + 1 + 7) / 8 * 8;
};

// rows = hidden rounded up to the grads block (zero rows past hidden)
template <int D, int K>
__global__ __launch_bounds__(256) void k_ppo_pack(const float* __restrict__ w1,
                                                  const float* __restrict__ b1, int d,
                                                  int hidden, const float* __restrict__ wa,
                                                  int k, const float* __restrict__ wc, int rows,
                                                  float* __restrict__ table) {
  using Tb = PpoTable<D, K>;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * Tb::kStride) return;
  const int u = t / Tb::kStride, col = t - u * Tb::kStride;
  float v = 0.0f;
  if (u < hidden) {
    if (col < k)
      v = wa[(size_t)col * hidden + u];
    else if (col == K)
      v = wc[u];
    else if (col >= Tb::kW1 && col < Tb::kW1 + d)
      v = w1[(size_t)u * d + (col - Tb::kW1)];
    else if (col == Tb::kB1)
      v = b1[u];
  }
  table[t] = v;
}

typedef float ppo_f2 __attribute__((ext_vector_type(2)));

// V of every sample: one thread per two adjacent samples (packed fp32 FMAs,
// v_pk_fma_f32), their features in registers, the unit rows wave-uniform
// scalar loads.
template <int D, int K>
__global__ __launch_bounds__(256) void k_ppo_values(const float* __restrict__ x, int n, int d,
                                                    const float* __restrict__ table, int hidden,
                                                    const float* __restrict__ bc,
                                                    float* __restrict__ values) {
  using Tb = PpoTable<D, K>;
  const long s = 2 * ((long)blockIdx.x * blockDim.x + threadIdx.x);
  if (s >= n) return;
  const long s1 = min(s + 1, (long)n - 1);  // an odd n pairs the last sample with itself
  ppo_f2 xs[D];
  const float* xa = x + (size_t)s * d;
  const float* xb = x + (size_t)s1 * d;
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const float va = xa[min(c, d - 1)], vb = xb[min(c, d - 1)];
    xs[c] = c < d ? ppo_f2{va, vb} : ppo_f2{0.0f, 0.0f};
  }
  ppo_f2 v = bc[0];
#pragma unroll 4
  for (int j = 0; j < hidden; ++j) {
    const float* row = table + (size_t)j * Tb::kStride;
    ppo_f2 h = row[Tb::kB1];
#pragma unroll
    for (int c = 0; c < D; ++c) h = __builtin_elementwise_fma((ppo_f2)row[Tb::kW1 + c], xs[c], h);
    h = __builtin_elementwise_max(h, (ppo_f2)0.0f);
    v = __builtin_elementwise_fma((ppo_f2)row[K], h, v);
  }
  values[s] = v.x;
  if (s + 1 < n) values[s + 1] = v.y;
}

// V at small sample counts, where the per-thread chain over all units is
// the latency: a workgroup of 4 waves takes 64 samples (lane = sample) and
// wave w sums units [w H/4, (w + 1) H/4) (wave-uniform rows); the four
// partials are added in a fixed order.
template <int D, int K>
__global__ __launch_bounds__(256) void k_ppo_values_split(const float* __restrict__ x, int n,
                                                          int d,
                                                          const float* __restrict__ table,
                                                          int hidden,
                                                          const float* __restrict__ bc,
                                                          float* __restrict__ values) {
  using Tb = PpoTable<D, K>;
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long s = (long)blockIdx.x * 64 + lane;
  const float* xp = x + (size_t)min(s, (long)n - 1) * d;
  float xs[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    const float v = xp[min(c, d - 1)];
    xs[c] = c < d ? v : 0.0f;
  }
  const int per = (hidden + 3) / 4, j0 = w * per, j1 = min(hidden, j0 + per);
  float v = 0.0f;
#pragma unroll 4
  for (int j = j0; j < j1; ++j) {
    const float* row = table + (size_t)j * Tb::kStride;
    float h = row[Tb::kB1];
#pragma unroll
    for (int c = 0; c < D; ++c) h = fmaf(row[Tb::kW1 + c], xs[c], h);
    v = fmaf(row[K], fmaxf(h, 0.0f), v);
  }
  red[w][lane] = v;
  __syncthreads();
  if (w == 0 && s < n) values[s] = bc[0] + ((red[0][lane] + red[1][lane]) + red[2][lane]) +
                                   red[3][lane];
}

// One thread per agent column of the T x S sample grid (sample t * S + col).
// adv: raw advantages; dv: dL/dV = 0.5 huber'(V - R) minus the returns'
// dependence on later values, dR_t/dV_u = gamma (1 - lambda) (gamma
// lambda)^(u-1-t) for u > t; part[2 block + 0..1] = the block's sum A, sum A^2.
// TM > 0: the column's T <= TM rewards and values are loaded into registers
// up front (one memory latency instead of a dependent chain of T); the
// arithmetic is the same in either form.
template <int TM>
__global__ __launch_bounds__(256) void k_ppo_gae(const float* __restrict__ rewards,
                                                 const float* __restrict__ values, int T, int S,
                                                 float gamma, float lambda,
                                                 float* __restrict__ adv, float* __restrict__ dv,
                                                 double* __restrict__ part) {
  __shared__ double red[2][4];
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  const float gl = gamma * lambda, g1 = gamma * (1.0f - lambda);
  if (col < S && TM > 0) {
    float vr[TM > 0 ? TM : 1], rr[TM > 0 ? TM : 1];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      vr[t] = t < T ? values[(size_t)t * S + col] : 0.0f;
      rr[t] = t < T ? rewards[(size_t)t * S + col] : 0.0f;
    }
    float gae = 0.0f;
#pragma unroll
    for (int t = TM - 1; t >= 0; --t) {
      if (t < T) {
        const float v = vr[t];
        const float delta = t != T - 1 ? rr[t] + gamma * vr[t < TM - 1 ? t + 1 : t] - v : rr[t] - v;
        gae = delta + gl * gae;
        adv[(size_t)t * S + col] = gae;
        rr[t] = 0.5f * fminf(fmaxf(v - (gae + v), -1.0f), 1.0f);  // direct dL/dV
        s1 += (double)gae;
        s2 += (double)gae * (double)gae;
      }
    }
    float carry = 0.0f;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t < T) {
        const float g = rr[t];
        dv[(size_t)t * S + col] = g - g1 * carry;
        carry = gl * carry + g;
      }
    }
  } else if (col < S) {
    float gae = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * S + col;
      const float v = values[i];
      const float delta = t != T - 1 ? rewards[i] + gamma * values[i + S] - v : rewards[i] - v;
      gae = delta + gl * gae;
      adv[i] = gae;
      // critic term 0.5 huber(V, R), R = A + V: d/dV (direct) = 0.5 clip(V - R, -1, 1)
      dv[i] = 0.5f * fminf(fmaxf(v - (gae + v), -1.0f), 1.0f);
      s1 += (double)gae;
      s2 += (double)gae * (double)gae;
    }
    // through the returns: dL/dV_u -= gamma (1 - lambda) sum_{t<u} g_t (gamma lambda)^(u-1-t)
    float carry = 0.0f;
    for (int t = 0; t < T; ++t) {
      const size_t i = (size_t)t * S + col;
      const float g = dv[i];
      dv[i] = g - g1 * carry;
      carry = gl * carry + g;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = s1;
    red[1][wv] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// The sums of the GAE blocks' partials, in a fixed order (thread-strided
// sums, xor-shuffle tree, waves in order): every workgroup of the grads
// kernel computes the same two numbers.  Needs blockDim = 64 * nw, nw <= 4.
__device__ inline void ppo_advantage_sums(const double* __restrict__ part, int n_part,
                                          double* out) {
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < n_part; i += blockDim.x) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (lane == 0) {
    red[0][w] = a;
    red[1][w] = b;
  }
  __syncthreads();
  a = 0.0;
  b = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
    a += red[0][i];
    b += red[1][i];
  }
  out[0] = a;
  out[1] = b;
}

// Value of lane l of a wave (v_readlane: wave-uniform result).
__device__ __forceinline__ float lane_value(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <int K>
struct PpoHeads {
  static constexpr int kP = K + 1;                  // logits + value
  static constexpr int kRow = (K + 1 + 3) / 4 * 4;  // a sample's dL/d(heads) row in LDS
};

template <int NW, int K>
__host__ __device__ constexpr int ppo_grads_lds_floats() {
  // per-wave H half-block transpose [64][65] | head partials of waves 1..
  // [K+1][64] | dL/d(logits, value) [64][kRow]
  return NW * 64 * 65 + (NW - 1) * (K + 1) * 64 + 64 * PpoHeads<K>::kRow;
}

__device__ __forceinline__ ppo_f2 ppo_splat(float v) { return ppo_f2{v, v}; }

// Per-block parameter gradients; NW waves, each owning 128 hidden units --
// thread (w, lane) holds units u0 = 128 w + lane and u1 = u0 + 64 as the two
// halves of packed fp32 registers, so every broadcast operand feeds a
// v_pk_fma_f32 for two units.  Dynamic LDS ppo_grads_lds_floats<NW, K>()
// floats; partial: [gridDim.x][ppo_grad_size].  Tiles of 64 samples:
//   A  h of both units for the tile's 64 samples into registers, each
//      sample's features broadcast from its lane by v_readlane
//   B  lane = sample: the heads' partial sums over the wave's 128 units, H
//      transposed through LDS one 64-unit half at a time, the unit's head
//      weights one scalar-load row of the packed table; wave 0 adds the other
//      waves' partials (fixed order) and forms dL/dz, dL/dV of its lane's
//      sample
//   C  gradient accumulation over the 64 samples, dL/dz of each broadcast by
//      v_readlane
template <int NW, int D, int K>
__global__ __launch_bounds__(64 * NW) void k_ppo_grads(
    const float* __restrict__ x, int n, int d, const float* __restrict__ w1,
    const float* __restrict__ b1, int hidden, const float* __restrict__ wa,
    const float* __restrict__ ba, int k, const float* __restrict__ wc,
    const float* __restrict__ bc, const int64_t* __restrict__ actions,
    const float* __restrict__ old_logp, const float* __restrict__ adv,
    const float* __restrict__ dvalue, const double* __restrict__ gae_part, int n_part,
    const float* __restrict__ table, float clip_eps, float c_ent, float* __restrict__ partial) {
  constexpr int KP = K + 1, kTab = PpoTable<D, K>::kStride, kRow = PpoHeads<K>::kRow;
  extern __shared__ float ppo_lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  float* sh = ppo_lds + w * 64 * 65;   // this wave's H half-block, [sample][unit]
  float* red = ppo_lds + NW * 64 * 65; // [NW - 1][KP][64]
  float* sz = red + (NW - 1) * KP * 64;
  const int u0 = 128 * w + lane, u1 = u0 + 64;
  const bool in0 = u0 < hidden, in1 = u1 < hidden;
  ppo_f2 w1p[D], wop[KP];
#pragma unroll
  for (int c = 0; c < D; ++c)
    w1p[c] = ppo_f2{in0 && c < d ? w1[(size_t)u0 * d + c] : 0.0f,
                    in1 && c < d ? w1[(size_t)u1 * d + c] : 0.0f};
  const ppo_f2 b1p{in0 ? b1[u0] : 0.0f, in1 ? b1[u1] : 0.0f};
#pragma unroll
  for (int q = 0; q < KP; ++q) {
    const float* col = q < k ? wa + (size_t)q * hidden : wc;
    const bool live = q < k || q == K;
    wop[q] = ppo_f2{live && in0 ? col[u0] : 0.0f, live && in1 ? col[u1] : 0.0f};
  }
  float bo[KP];
#pragma unroll
  for (int q = 0; q < KP; ++q) bo[q] = q < k ? ba[q] : (q == K ? bc[0] : 0.0f);
  // normalised advantages (A - mean) / (std + eps): population std, fp32 eps
  double stats[2];
  ppo_advantage_sums(gae_part, n_part, stats);
  const double mean = stats[0] / (double)n;
  const double var = fmax(stats[1] / (double)n - mean * mean, 0.0);
  const float a_mean = (float)mean;
  const float a_den = (float)sqrt(var) + 1.1920928955078125e-07f;
  ppo_f2 gw1p[D], gwop[KP], gb1p = ppo_splat(0.0f);
  float gbias[KP];
#pragma unroll
  for (int c = 0; c < D; ++c) gw1p[c] = ppo_splat(0.0f);
#pragma unroll
  for (int q = 0; q < KP; ++q) {
    gwop[q] = ppo_splat(0.0f);
    gbias[q] = 0.0f;
  }
  const float* rows = table + (size_t)wu * 128 * kTab;
  const long tiles = ((long)n + 63) / 64;
  for (long tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const long si = tile * 64 + lane;
    const bool valid = si < n;
    float xr[D];
    {
      // clamped loads and a select, no branches (a feature c >= d meets a
      // zero weight; a sample past n has dL/dz = 0 below, so adds nothing)
      const float* xs = x + (size_t)min(si, (long)n - 1) * d;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        const float v = xs[min(c, d - 1)];
        xr[c] = c < d ? v : 0.0f;
      }
    }
    // A: hidden activations of both units for the 64 samples
    ppo_f2 hs[64];
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      ppo_f2 h = b1p;
#pragma unroll
      for (int c = 0; c < D; ++c)
        h = __builtin_elementwise_fma(w1p[c], ppo_splat(lane_value(xr[c], s)), h);
      hs[s] = __builtin_elementwise_max(h, ppo_splat(0.0f));
    }
    // B: heads, lane = sample, the wave's units one 64-unit half at a time
    float acc[KP];
#pragma unroll
    for (int q = 0; q < KP; ++q) acc[q] = 0.0f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half) __syncthreads();  // the first half's readers are done
#pragma unroll
      for (int s = 0; s < 64; ++s) sh[s * 65 + lane] = half ? hs[s].y : hs[s].x;
      __syncthreads();
      const float* row = rows + (size_t)half * 64 * kTab;
#pragma unroll 4
      for (int u = 0; u < 64; ++u) {
        const float h = sh[lane * 65 + u];
#pragma unroll
        for (int q = 0; q < KP; ++q) acc[q] = fmaf(row[u * kTab + q], h, acc[q]);
      }
    }
    if (NW > 1 && w > 0) {
#pragma unroll
      for (int q = 0; q < KP; ++q) red[((w - 1) * KP + q) * 64 + lane] = acc[q];
    }
    if (NW > 1) __syncthreads();
    float g[KP];
#pragma unroll
    for (int q = 0; q < KP; ++q) g[q] = 0.0f;
    if (w == 0) {
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
#pragma unroll
        for (int q = 0; q < KP; ++q) acc[q] += red[((ww - 1) * KP + q) * 64 + lane];
      }
      if (valid) {
        float p[K];
        float m = acc[0] + bo[0];
#pragma unroll
        for (int q = 1; q < K; ++q)
          if (q < k) m = fmaxf(m, acc[q] + bo[q]);
        float sum = 0.0f;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          p[q] = q < k ? expf(acc[q] + bo[q] - m) : 0.0f;
          sum += p[q];
        }
        const int a = (int)actions[si];
        float pa = 0.0f;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          p[q] = p[q] / sum;
          pa = q == a ? p[q] : pa;
        }
        // -min(r A, clip(r, 1 - eps, 1 + eps) A): a tie splits the gradient
        // evenly between the two arguments, clip passes it on its closed range
        const float A = (adv[si] - a_mean) / a_den;
        const float r = expf(logf(pa + 1e-8f) - old_logp[si]);
        const float lo = 1.0f - clip_eps, hi = 1.0f + clip_eps;
        const float rc = fminf(fmaxf(r, lo), hi);
        const float t1 = r * A, t2 = rc * A;
        const float w1st = t1 < t2 ? 1.0f : (t1 > t2 ? 0.0f : 0.5f);
        const float in = (r >= lo && r <= hi) ? 1.0f : 0.0f;
        const float d_r = -A * (w1st + (1.0f - w1st) * in);
        const float d_pa = d_r * r / (pa + 1e-8f);
        // entropy term: + c_ent sum_q (p_q + eps) log(p_q + eps)
        float dp[K], pdp = 0.0f;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          dp[q] = q < k ? c_ent * (logf(p[q] + 1e-8f) + 1.0f) + (q == a ? d_pa : 0.0f) : 0.0f;
          pdp = fmaf(p[q], dp[q], pdp);
        }
#pragma unroll
        for (int q = 0; q < K; ++q) g[q] = p[q] * (dp[q] - pdp);
        g[K] = dvalue[si];
      }
#pragma unroll
      for (int q = 0; q < KP; ++q) gbias[q] += g[q];
      if (NW > 1) {
#pragma unroll
        for (int q = 0; q < KP; ++q) sz[lane * kRow + q] = g[q];
      }
    }
    if (NW > 1) {
      __syncthreads();
#pragma unroll
      for (int q = 0; q < KP; ++q) g[q] = sz[lane * kRow + q];
    }
    // broadcast the features again in C rather than keep phase A's 64 x D
    // uniform copies alive (they would spill the SGPR file)
#pragma unroll
    for (int c = 0; c < D; ++c) asm volatile("" : "+v"(xr[c]));
    // C: both units' gradients over the 64 samples, dL/dz of each broadcast
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const ppo_f2 h = hs[s];
      ppo_f2 dh = ppo_splat(0.0f);
#pragma unroll
      for (int q = 0; q < KP; ++q) {
        const ppo_f2 gs = ppo_splat(lane_value(g[q], s));
        gwop[q] = __builtin_elementwise_fma(gs, h, gwop[q]);
        dh = __builtin_elementwise_fma(wop[q], gs, dh);
      }
      dh.x = h.x > 0.0f ? dh.x : 0.0f;
      dh.y = h.y > 0.0f ? dh.y : 0.0f;
      gb1p += dh;
#pragma unroll
      for (int c = 0; c < D; ++c)
        gw1p[c] = __builtin_elementwise_fma(dh, ppo_splat(lane_value(xr[c], s)), gw1p[c]);
    }
    if (NW > 1) __syncthreads();  // sz and red are rewritten next tile
  }
  // output-bias gradients: wave 0's per-lane sums, reduced across the wave
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < KP; ++q) {
      float v = gbias[q];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      gbias[q] = v;
    }
  }
  float* out = partial + (size_t)blockIdx.x * ppo_grad_size(d, hidden, k);
  const int o_b1 = hidden * d, o_wa = o_b1 + hidden, o_ba = o_wa + k * hidden;
  const int o_wc = o_ba + k, o_bc = o_wc + hidden;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int u = half ? u1 : u0;
    if (u < hidden) {
#pragma unroll
      for (int c = 0; c < D; ++c)
        if (c < d) out[u * d + c] = half ? gw1p[c].y : gw1p[c].x;
      out[o_b1 + u] = half ? gb1p.y : gb1p.x;
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (q < k) out[o_wa + q * hidden + u] = half ? gwop[q].y : gwop[q].x;
      out[o_wc + u] = half ? gwop[K].y : gwop[K].x;
    }
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (q < k) out[o_ba + q] = gbias[q];
    out[o_bc] = gbias[K];
  }
}

// Sum of the block partials, fp64 in a fixed order.  Workgroup 1024 = 64
// parameters x 16 block strides.
__global__ __launch_bounds__(1024) void k_ppo_reduce(const float* __restrict__ partial,
                                                     int n_blocks, int size,
                                                     float* __restrict__ grad) {
  __shared__ double red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + lane;
  double acc = 0.0;
  if (p < size) {
#pragma unroll 8
    for (int b = w; b < n_blocks; b += 16) acc += (double)partial[(size_t)b * size + p];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && p < size) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    grad[p] = (float)t;
  }
}

}  // namespace swarm
