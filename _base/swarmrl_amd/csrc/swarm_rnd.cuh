// swarm_rnd.cuh -- Random Network Distillation distance in one launch.
//
// The C5 workload's intrinsic reward (swarmrl/intrinsic_reward/
// random_network_distillation.py:126-143 with rnd_configs.py:17-38): per
// observation x, the fixed random target network and the trained predictor,
// both Dense(W) -> ReLU -> Dense(W) -> ReLU -> Dense(W), and the ZnNL
// OrderNDifference metric (sum_k |t_k - p_k|^order)^(1/order).  The torch
// forward of the two networks is six GEMMs and their epilogues (~20 small
// launches per slice, ~110 us at 16384 agents); here one thread per
// observation runs both networks from LDS-staged weights (torch Linear
// layouts, read in place) and reduces the metric.  fp32, checked against the
// torch networks within a stated tolerance (tests/test_gpu_rnd.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swarm {

constexpr int kRndWidth = 32;   // rnd_configs.py:17-38 (Dense(32) x 3)
constexpr int kRndMaxIn = 16;

// The six parameter tensors of one network: w1, b1, w2, b2, w3, b3.
struct RndPtrs {
  const float* w[6];
};

// One network's weights in LDS: w1 [W][D], b1, and the square layers
// transposed (w2t[k][j] = w2[j][k]) so that one input k feeds a row of W
// outputs read as float4 broadcasts.
template <int D>
struct RndNet {
  float w1[kRndWidth][D];
  float b1[kRndWidth];
  float4 w2t[kRndWidth][kRndWidth / 4];
  float b2[kRndWidth];
  float4 w3t[kRndWidth][kRndWidth / 4];
  float b3[kRndWidth];
};

template <int D>
__device__ __forceinline__ void rnd_stage(RndNet<D>* net, const float* const* w, int d_in) {
  constexpr int W = kRndWidth;
  for (int k = threadIdx.x; k < W * D; k += blockDim.x) {
    const int j = k / D, i = k - j * D;
    net->w1[j][i] = i < d_in ? w[0][j * d_in + i] : 0.0f;
  }
  float* w2t = reinterpret_cast<float*>(net->w2t);
  float* w3t = reinterpret_cast<float*>(net->w3t);
  for (int k = threadIdx.x; k < W * W; k += blockDim.x) {
    const int j = k / W, i = k - j * W;  // torch w[j][i] (out j, in i)
    w2t[i * W + j] = w[2][k];
    w3t[i * W + j] = w[4][k];
  }
  for (int k = threadIdx.x; k < W; k += blockDim.x) {
    net->b1[k] = w[1][k];
    net->b2[k] = w[3][k];
    net->b3[k] = w[5][k];
  }
}

// a[j] = b[j] + sum_k wt[k][j] h[k] with h from the thread's LDS column
// (hb[k][tid]); k in order, one float4 row broadcast at a time.
__device__ __forceinline__ void rnd_square(const float4 (*wt)[kRndWidth / 4], const float* b,
                                           const float (*hb)[256], float* a) {
  constexpr int W = kRndWidth;
#pragma unroll
  for (int j = 0; j < W; ++j) a[j] = b[j];
#pragma unroll 2
  for (int k = 0; k < W; ++k) {
    const float hk = hb[k][threadIdx.x];
#pragma unroll
    for (int q = 0; q < W / 4; ++q) {
      const float4 r = wt[k][q];
      a[4 * q + 0] = __builtin_fmaf(r.x, hk, a[4 * q + 0]);
      a[4 * q + 1] = __builtin_fmaf(r.y, hk, a[4 * q + 1]);
      a[4 * q + 2] = __builtin_fmaf(r.z, hk, a[4 * q + 2]);
      a[4 * q + 3] = __builtin_fmaf(r.w, hk, a[4 * q + 3]);
    }
  }
}

// Output layer of one network for one observation (x in registers).
template <int D>
__device__ __forceinline__ void rnd_forward(const RndNet<D>& net, const float* x,
                                            float (*hb)[256], float* out) {
  constexpr int W = kRndWidth;
  float a[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    float v = net.b1[j];
#pragma unroll
    for (int i = 0; i < D; ++i) v = __builtin_fmaf(net.w1[j][i], x[i], v);
    a[j] = v;
  }
#pragma unroll
  for (int j = 0; j < W; ++j) hb[j][threadIdx.x] = fmaxf(a[j], 0.0f);
  rnd_square(net.w2t, net.b2, hb, a);
#pragma unroll
  for (int j = 0; j < W; ++j) hb[j][threadIdx.x] = fmaxf(a[j], 0.0f);
  rnd_square(net.w3t, net.b3, hb, out);
}

// The metric of observation a (both networks from the block's LDS copies).
template <int D>
__device__ __forceinline__ float rnd_metric(const RndNet<D>& tnet, const RndNet<D>& pnet,
                                            const float* __restrict__ x, int a, int d_in,
                                            int order, float (*hb)[256]) {
  constexpr int W = kRndWidth;
  float xi[D];
#pragma unroll
  for (int i = 0; i < D; ++i) xi[i] = i < d_in ? x[(size_t)a * d_in + i] : 0.0f;
  float t[W], p[W];
  rnd_forward<D>(tnet, xi, hb, t);
  rnd_forward<D>(pnet, xi, hb, p);
  float acc = 0.0f;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const float dlt = fabsf(t[j] - p[j]);
    acc += order == 2 ? dlt * dlt : powf(dlt, (float)order);
  }
  return order == 2 ? sqrtf(acc) : powf(acc, 1.0f / (float)order);
}

template <int D>
__global__ __launch_bounds__(256) void k_rnd_distance(const float* __restrict__ x, int n,
                                                      int d_in, RndPtrs tp, RndPtrs pp,
                                                      int order, float* __restrict__ out) {
  __shared__ RndNet<D> tnet, pnet;
  __shared__ float hb[kRndWidth][256];  // the thread's hidden activations (column tid)
  rnd_stage<D>(&tnet, tp.w, d_in);
  rnd_stage<D>(&pnet, pp.w, d_in);
  __syncthreads();
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;  // no barrier below
  out[a] = rnd_metric<D>(tnet, pnet, x, a, d_in, order, hb);
}

// The per-env intrinsic reward (random_network_distillation.py:126-143 on
// the device path: the mean metric of the env's latest observations,
// clipped) added to the task reward, in two launches instead of the metric
// kernel + torch's mean, clamp and add (five launches and a copy on C5's
// critical path).  Pass 1 (grid E x kb, 256 threads): the metric of every
// observation of env e = blockIdx.y and the block's fp64 partial sum.
template <int D>
__global__ __launch_bounds__(256) void k_rnd_env_partial(const float* __restrict__ x, int per_env,
                                                         int d_in, RndPtrs tp, RndPtrs pp,
                                                         int order, float* __restrict__ metric,
                                                         double* __restrict__ partial) {
  __shared__ RndNet<D> tnet, pnet;
  __shared__ float hb[kRndWidth][256];
  __shared__ double wsum[4];
  rnd_stage<D>(&tnet, tp.w, d_in);
  rnd_stage<D>(&pnet, pp.w, d_in);
  __syncthreads();
  const int e = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  double v = 0.0;
  if (k < per_env) {
    const int a = e * per_env + k;
    const float m = rnd_metric<D>(tnet, pnet, x, a, d_in, order, hb);
    metric[a] = m;
    v = (double)m;
  }
  // fixed-order block sum: xor butterfly in the wave, then the four waves
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    partial[(size_t)e * gridDim.x + blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

// Pass 2 (one 1024-thread block per env): the env's partials summed in block
// order (deterministic), mean -> fp32 -> clip, then
// rewards[e][a] = base[e][a] + r_e (base null: rewards[e][a] = r_e).
__global__ __launch_bounds__(1024) void k_rnd_env_finish(const double* __restrict__ partial,
                                                         int kb, int per_env, int clip,
                                                         float lo, float hi,
                                                         const float* __restrict__ base,
                                                         float* __restrict__ env_reward,
                                                         float* __restrict__ rewards) {
  __shared__ float r_e;
  const int e = blockIdx.x;
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < kb; ++k) s += partial[(size_t)e * kb + k];
    float r = (float)(s / (double)per_env);
    if (clip) r = fminf(fmaxf(r, lo), hi);
    r_e = r;
    env_reward[e] = r;
  }
  __syncthreads();
  const float r = r_e;
  for (int a = threadIdx.x; a < per_env; a += blockDim.x) {
    const size_t g = (size_t)e * per_env + a;
    rewards[g] = base ? base[g] + r : r;
  }
}

}  // namespace swarm
