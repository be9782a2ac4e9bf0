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
//                 of squares of the advantages (fp64, for their
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
// per-sample gradients; the caller's optimizer takes the step.
// Workgroup: HB threads (HB = hidden rounded up to 64/128/256), thread j owns
// hidden unit j (its W1 row, W2 column and their gradient accumulators live
// in registers); tiles of samples stream through LDS.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swarm {

constexpr int kPpoMaxIn = 32;
constexpr int kPpoMaxK = 16;
constexpr int kPpoMaxHidden = 256;
constexpr int kPpoBlocks = 512;  // grad blocks: 2 per CU (LDS-limited)

// Gradient layout (floats): W1 [H][D] | b1 [H] | Wa [K][H] | ba [K] | Wc [H] | bc
__host__ __device__ inline int ppo_grad_size(int d, int h, int k) {
  return h * d + h + k * h + k + h + 1;
}

// V of every sample (one thread per sample, hidden layer + critic in LDS).
__global__ __launch_bounds__(256) void k_ppo_values(const float* __restrict__ x, int n, int d,
                                                    const float* __restrict__ w1,
                                                    const float* __restrict__ b1, int hidden,
                                                    const float* __restrict__ wc,
                                                    const float* __restrict__ bc,
                                                    float* __restrict__ values) {
  extern __shared__ float sv[];  // w1 [hidden][d] | b1 [hidden] | wc [hidden]
  float* sw1 = sv;
  float* sb1 = sv + hidden * d;
  float* swc = sb1 + hidden;
  for (int t = threadIdx.x; t < hidden * d; t += blockDim.x) sw1[t] = w1[t];
  for (int t = threadIdx.x; t < hidden; t += blockDim.x) {
    sb1[t] = b1[t];
    swc[t] = wc[t];
  }
  __syncthreads();
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const float* xs = x + (size_t)s * d;
  float v = bc[0];
  for (int j = 0; j < hidden; ++j) {
    float h = sb1[j];
    for (int c = 0; c < d; ++c) h = fmaf(sw1[j * d + c], xs[c], h);
    v = fmaf(swc[j], fmaxf(h, 0.0f), v);
  }
  values[s] = v;
}

// One thread per agent column of the T x S sample grid (sample t * S + col).
// adv: raw advantages; dv: dL/dV = 0.5 huber'(V - R) minus the returns'
// dependence on later values, dR_t/dV_u = gamma (1 - lambda) (gamma
// lambda)^(u-1-t) for u > t; stats[0..1] += sum A, sum A^2.
__global__ __launch_bounds__(256) void k_ppo_gae(const float* __restrict__ rewards,
                                                 const float* __restrict__ values, int T, int S,
                                                 float gamma, float lambda,
                                                 float* __restrict__ adv, float* __restrict__ dv,
                                                 double* __restrict__ stats) {
  __shared__ double red[2][4];
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (col < S) {
    float gae = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t i = (size_t)t * S + col;
      const float v = values[i];
      const float delta = t != T - 1 ? rewards[i] + gamma * values[i + S] - v : rewards[i] - v;
      gae = delta + gamma * lambda * gae;
      adv[i] = gae;
      // critic term 0.5 huber(V, R), R = A + V: d/dV (direct) = 0.5 clip(V - R, -1, 1)
      dv[i] = 0.5f * fminf(fmaxf(v - (gae + v), -1.0f), 1.0f);
      s1 += (double)gae;
      s2 += (double)gae * (double)gae;
    }
    // through the returns: dL/dV_u -= gamma (1 - lambda) sum_{t<u} g_t (gamma lambda)^(u-1-t)
    const float gl = gamma * lambda, g1 = gamma * (1.0f - lambda);
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
    atomicAdd(&stats[0], a);
    atomicAdd(&stats[1], b);
  }
}

template <int HB>
struct PpoTile {
  static constexpr int kTile = HB == 256 ? 32 : 64;  // samples per tile (LDS < 64 KB)
  static constexpr int kPer = HB / kTile;             // threads per sample for the heads
};

// Per-block parameter gradients; blockDim = HB >= hidden.
// partial: [gridDim.x][ppo_grad_size(d, hidden, k)].
template <int HB, int D, int K>
__global__ __launch_bounds__(HB) void k_ppo_grads(
    const float* __restrict__ x, int n, int d, const float* __restrict__ w1,
    const float* __restrict__ b1, int hidden, const float* __restrict__ wa,
    const float* __restrict__ ba, int k, const float* __restrict__ wc,
    const float* __restrict__ bc, const int64_t* __restrict__ actions,
    const float* __restrict__ old_logp, const float* __restrict__ adv,
    const float* __restrict__ dvalue, const double* __restrict__ stats, float clip_eps,
    float c_ent, float* __restrict__ partial) {
  constexpr int kTile = PpoTile<HB>::kTile, kPer = PpoTile<HB>::kPer;
  __shared__ float sx[kTile][D];
  __shared__ float sh[kTile][HB + 1];
  __shared__ float sz[kTile][K + 1];  // dL/d(logits, value) per sample
  __shared__ float swo[K + 1][HB];    // [Wa; Wc] columns
  const int j = threadIdx.x;
  const bool unit = j < hidden;
  float w1j[D], woj[K + 1];
#pragma unroll
  for (int c = 0; c < D; ++c) w1j[c] = unit && c < d ? w1[(size_t)j * d + c] : 0.0f;
  const float b1j = unit ? b1[j] : 0.0f;
#pragma unroll
  for (int q = 0; q < K + 1; ++q) {
    woj[q] = !unit ? 0.0f : (q < k ? wa[(size_t)q * hidden + j] : (q == K ? wc[j] : 0.0f));
    swo[q][j] = woj[q];
  }
  float bo[K + 1];
#pragma unroll
  for (int q = 0; q < K + 1; ++q) bo[q] = q < k ? ba[q] : (q == K ? bc[0] : 0.0f);
  // normalised advantages (A - mean) / (std + eps): population std, fp32 eps
  const double mean = stats[0] / (double)n;
  const double var = fmax(stats[1] / (double)n - mean * mean, 0.0);
  const float a_mean = (float)mean;
  const float a_den = (float)sqrt(var) + 1.1920928955078125e-07f;
  float gw1[D], gwo[K + 1], gb1 = 0.0f, gbo = 0.0f;
#pragma unroll
  for (int c = 0; c < D; ++c) gw1[c] = 0.0f;
#pragma unroll
  for (int q = 0; q < K + 1; ++q) gwo[q] = 0.0f;
  const long tiles = ((long)n + kTile - 1) / kTile;
  for (long tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const long s0 = tile * kTile;
    __syncthreads();  // the previous tile's readers are done
    for (int t = j; t < kTile * D; t += HB) {
      const int s = t / D, c = t - s * D;
      sx[s][c] = s0 + s < n && c < d ? x[(size_t)(s0 + s) * d + c] : 0.0f;
    }
    __syncthreads();
    if (unit) {
      for (int s = 0; s < kTile; ++s) {
        float h = b1j;
#pragma unroll
        for (int c = 0; c < D; ++c) h = fmaf(w1j[c], sx[s][c], h);
        sh[s][j] = fmaxf(h, 0.0f);
      }
    }
    __syncthreads();
    {
      // heads: kPer threads per sample split the hidden units
      const int s = j / kPer, part = j - s * kPer;
      float acc[K + 1];
#pragma unroll
      for (int q = 0; q < K + 1; ++q) acc[q] = 0.0f;
      for (int u = part; u < hidden; u += kPer) {
        const float h = sh[s][u];
#pragma unroll
        for (int q = 0; q < K + 1; ++q) acc[q] = fmaf(swo[q][u], h, acc[q]);
      }
#pragma unroll
      for (int o = 1; o < kPer; o <<= 1) {
#pragma unroll
        for (int q = 0; q < K + 1; ++q) acc[q] += __shfl_xor(acc[q], o, 64);
      }
      const long si = s0 + s;
      if (part == 0) {
        float g[K + 1];
#pragma unroll
        for (int q = 0; q < K + 1; ++q) g[q] = 0.0f;
        if (si < n) {
          float z[K], p[K];
#pragma unroll
          for (int q = 0; q < K; ++q) z[q] = acc[q] + bo[q];
          float m = z[0];
#pragma unroll
          for (int q = 1; q < K; ++q)
            if (q < k) m = fmaxf(m, z[q]);
          float sum = 0.0f;
#pragma unroll
          for (int q = 0; q < K; ++q) {
            p[q] = q < k ? expf(z[q] - m) : 0.0f;
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
        for (int q = 0; q < K + 1; ++q) sz[s][q] = g[q];
      }
    }
    __syncthreads();
    // back through the layers: thread j sums its unit's gradients
    if (unit) {
      for (int s = 0; s < kTile; ++s) {
        const float h = sh[s][j];
        float dh = 0.0f;
#pragma unroll
        for (int q = 0; q < K + 1; ++q) {
          const float gq = sz[s][q];
          gwo[q] = fmaf(gq, h, gwo[q]);
          dh = fmaf(woj[q], gq, dh);
        }
        dh = h > 0.0f ? dh : 0.0f;
        gb1 += dh;
#pragma unroll
        for (int c = 0; c < D; ++c) gw1[c] = fmaf(dh, sx[s][c], gw1[c]);
      }
    }
    if (j <= K) {
      for (int s = 0; s < kTile; ++s) gbo += sz[s][j];
    }
  }
  float* out = partial + (size_t)blockIdx.x * ppo_grad_size(d, hidden, k);
  const int o_b1 = hidden * d, o_wa = o_b1 + hidden, o_ba = o_wa + k * hidden;
  const int o_wc = o_ba + k, o_bc = o_wc + hidden;
  if (unit) {
#pragma unroll
    for (int c = 0; c < D; ++c)
      if (c < d) out[j * d + c] = gw1[c];
    out[o_b1 + j] = gb1;
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (q < k) out[o_wa + q * hidden + j] = gwo[q];
    out[o_wc + j] = gwo[K];
  }
  if (j < k) out[o_ba + j] = gbo;
  if (j == K) out[o_bc] = gbo;
}

// Sum of the block partials, fp64 in a fixed order.  Workgroup 256 = 64
// parameters x 4 block strides.
__global__ __launch_bounds__(256) void k_ppo_reduce(const float* __restrict__ partial,
                                                    int n_blocks, int size,
                                                    float* __restrict__ grad) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + lane;
  double acc = 0.0;
  if (p < size) {
    for (int b = w; b < n_blocks; b += 4) acc += (double)partial[(size_t)b * size + p];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && p < size)
    grad[p] = (float)(((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
}

}  // namespace swarm
