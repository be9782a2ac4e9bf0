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
// clipped) added to the task reward, in ONE launch instead of the metric
// kernel + torch's mean, clamp and add (five launches and a copy on C5's
// critical path).  Grid E x kb blocks of 256 threads, eight lanes per
// observation (32 a block): lane `sub` of a group computes outputs
// 4 sub .. 4 sub + 3 of every layer (each output's sum over its inputs in
// order, as rnd_forward), the group's hidden activations go through an LDS
// row (one wave's group: wave-scope ordering only), and the group adds its
// lanes' parts of the metric with xor-shuffles.  Each block writes its fp64
// partial sum (fixed order); the last block of an env (a ticket) adds the
// env's partials in a fixed tree, takes the mean, clips it and writes
// rewards[e][a] = base[e][a] + r_e (base null: r_e).  Deterministic: the
// same bits on every call and device.
constexpr int kRndLanes = 8;                      // lanes per observation
constexpr int kRndObsPerBlock = 256 / kRndLanes;  // 32
constexpr int kRndOut = kRndWidth / kRndLanes;    // outputs per lane and layer

// One network's weights in LDS, torch layouts (rows = outputs), the square
// layers' rows padded to kRndStride floats: lane `sub` of a group takes the
// outputs j = sub + 8 r, so the eight lanes of a group read rows 8 r .. 8 r
// + 7 together, which start 36 floats (= 36 banks mod 64) apart and cover
// disjoint bank quads -- no LDS bank conflict (unpadded rows 4 apart put all
// eight in one quad: an 8-way conflict on every float4 read).
constexpr int kRndStride = kRndWidth + 4;  // floats per padded row (16-B aligned)
template <int D>
struct RndRows {
  float w1[kRndWidth][D];
  float b1[kRndWidth];
  float4 w2[kRndWidth][kRndStride / 4];
  float b2[kRndWidth];
  float4 w3[kRndWidth][kRndStride / 4];
  float b3[kRndWidth];
};

// Both networks' weights into LDS (torch layouts, w1 zero-padded to D
// inputs).  Every load of the block's share of BOTH networks is issued
// before any LDS store: one memory latency (a load -> store -> load chain
// per loop trip took ~14 us per workgroup, SQ_WAIT_ANY 62 % of its wave
// cycles).  blockDim = 256.
template <int D>
__device__ __forceinline__ void rnd_stage_rows(RndRows<D>* tnet, RndRows<D>* pnet,
                                               const float* const* tw, const float* const* pw,
                                               int d_in) {
  constexpr int W = kRndWidth, T = 256;
  constexpr int N1 = (W * D + T - 1) / T, N2 = W * W / T;
  const int tid = threadIdx.x;
  RndRows<D>* nets[2] = {tnet, pnet};
  const float* const* ws[2] = {tw, pw};
  float v1[2][N1], v2[2][N2], v3[2][N2], bb[2][3];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const float* const* w = ws[n];
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int k = tid + u * T, j = k / D, i = k - j * D;
      v1[n][u] = k < W * D && i < d_in ? w[0][j * d_in + i] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      v2[n][u] = w[2][tid + u * T];
      v3[n][u] = w[4][tid + u * T];
    }
    if (tid < W) {
      bb[n][0] = w[1][tid];
      bb[n][1] = w[3][tid];
      bb[n][2] = w[5][tid];
    }
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    RndRows<D>* net = nets[n];
#pragma unroll
    for (int u = 0; u < N1; ++u) {
      const int k = tid + u * T;
      if (k < W * D) net->w1[k / D][k % D] = v1[n][u];
    }
    float* w2 = reinterpret_cast<float*>(net->w2);
    float* w3 = reinterpret_cast<float*>(net->w3);
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int t = tid + u * T, j = t / W, c = t - j * W;
      w2[j * kRndStride + c] = v2[n][u];
      w3[j * kRndStride + c] = v3[n][u];
    }
    if (tid < W) {
      net->b1[tid] = bb[n][0];
      net->b2[tid] = bb[n][1];
      net->b3[tid] = bb[n][2];
    }
  }
}

// A square layer: the lane's outputs j = sub + 8 r, a[r] = b[j] + sum_k
// w[j][k] h[k] over the group's activations h (LDS row, float4 reads).
__device__ __forceinline__ void rnd_square_lanes(const float4 (*w)[kRndStride / 4], const float* b,
                                                 const float4* h, int sub, float* a) {
#pragma unroll
  for (int r = 0; r < kRndOut; ++r) a[r] = b[sub + kRndLanes * r];
#pragma unroll
  for (int q = 0; q < kRndWidth / 4; ++q) {
    const float4 hv = h[q];
#pragma unroll
    for (int r = 0; r < kRndOut; ++r) {
      const float4 wv = w[sub + kRndLanes * r][q];
      a[r] = __builtin_fmaf(wv.x, hv.x, a[r]);
      a[r] = __builtin_fmaf(wv.y, hv.y, a[r]);
      a[r] = __builtin_fmaf(wv.z, hv.z, a[r]);
      a[r] = __builtin_fmaf(wv.w, hv.w, a[r]);
    }
  }
}

// The lane's four outputs of one network for the group's observation x;
// row: the group's LDS activation row (kRndStride floats, float4-aligned).
template <int D>
__device__ __forceinline__ void rnd_forward_lanes(const RndRows<D>& net, const float* x, int sub,
                                                  float* row, float* out) {
  float a[kRndOut];
#pragma unroll
  for (int r = 0; r < kRndOut; ++r) {
    const int j = sub + kRndLanes * r;
    float v = net.b1[j];
#pragma unroll
    for (int i = 0; i < D; ++i) v = __builtin_fmaf(net.w1[j][i], x[i], v);
    a[r] = fmaxf(v, 0.0f);
  }
  auto publish = [&](const float* v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the group's previous reads of the row are done
#pragma unroll
    for (int r = 0; r < kRndOut; ++r) row[sub + kRndLanes * r] = v[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const float4* h = reinterpret_cast<const float4*>(row);
  publish(a);
  rnd_square_lanes(net.w2, net.b2, h, sub, a);
#pragma unroll
  for (int r = 0; r < kRndOut; ++r) a[r] = fmaxf(a[r], 0.0f);
  publish(a);
  rnd_square_lanes(net.w3, net.b3, h, sub, out);
}

template <int D>
__global__ __launch_bounds__(256) void k_rnd_env(const float* __restrict__ x, int per_env,
                                                 int d_in, RndPtrs tp, RndPtrs pp, int order,
                                                 int clip, float lo, float hi,
                                                 const float* __restrict__ base,
                                                 float* __restrict__ metric,
                                                 float* __restrict__ env_reward,
                                                 float* __restrict__ rewards,
                                                 double* __restrict__ partial,
                                                 uint32_t* __restrict__ tickets) {
  static_assert(kRndOut == 4, "float4 activation rows");
  __shared__ RndRows<D> tnet, pnet;
  __shared__ __align__(16) float rows[kRndObsPerBlock][kRndStride];
  __shared__ double red[256];
  __shared__ int last;
  const int e = blockIdx.y, kb = gridDim.x, tid = threadIdx.x;
  const int sub = tid & (kRndLanes - 1), grp = tid / kRndLanes;
  rnd_stage_rows<D>(&tnet, &pnet, tp.w, pp.w, d_in);
  __syncthreads();
  // the block's groups of 32 observations (blockIdx.x, + gridDim.x, ...):
  // the networks are staged once per block, not once per 32 observations;
  // each group's metric sum in a fixed order per thread
  double own = 0.0;
  for (int k0 = blockIdx.x * kRndObsPerBlock; k0 < per_env; k0 += kb * kRndObsPerBlock) {
    const int k = k0 + grp;
    const bool valid = k < per_env;
    const size_t a = (size_t)e * per_env + (valid ? k : 0);
    float xi[D];
#pragma unroll
    for (int i = 0; i < D; ++i) xi[i] = i < d_in ? x[a * d_in + i] : 0.0f;
    float t[kRndOut], p[kRndOut];
    rnd_forward_lanes<D>(tnet, xi, sub, rows[grp], t);
    rnd_forward_lanes<D>(pnet, xi, sub, rows[grp], p);
    float acc = 0.0f;
#pragma unroll
    for (int r = 0; r < kRndOut; ++r) {
      const float dlt = fabsf(t[r] - p[r]);
      acc += order == 2 ? dlt * dlt : powf(dlt, (float)order);
    }
#pragma unroll
    for (int o = 1; o < kRndLanes; o <<= 1) acc += __shfl_xor(acc, o, 64);
    const float m = order == 2 ? sqrtf(acc) : powf(acc, 1.0f / (float)order);
    if (valid && sub == 0) {
      metric[a] = m;
      own += (double)m;
    }
  }
  // the block's sum: fixed tree over its threads
  red[tid] = own;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  double* pe = partial + (size_t)e * kb;
  if (tid == 0) {
    // the partial by a returning agent-scope atomic, waited for before the
    // ticket counts it (no __threadfence: an agent-scope release writes the
    // L2 back, ~0.1 us per block and a stall for every kernel beside it --
    // this launch took 51 us beside C5's build instead of ~20)
    __hip_atomic_exchange(reinterpret_cast<unsigned long long*>(pe + blockIdx.x),
                          (unsigned long long)__double_as_longlong(red[0]), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    last = atomicAdd(&tickets[e], 1u) == (uint32_t)(kb - 1);
  }
  __syncthreads();
  if (!last) return;
  // the env's last block: its partials in a fixed tree (kb <= 256 x 16 per
  // thread), read by agent-scope atomic loads
  double v = 0.0;
  for (int b = tid; b < kb; b += 256)
    v += __hip_atomic_load(&pe[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  red[tid] = v;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  float r = (float)(red[0] / (double)per_env);
  if (clip) r = fminf(fmaxf(r, lo), hi);
  if (tid == 0) {
    env_reward[e] = r;
    tickets[e] = 0u;  // the next call's count (graph replays)
  }
  for (int q = tid; q < per_env; q += 256) {
    const size_t g = (size_t)e * per_env + q;
    rewards[g] = base ? base[g] + r : r;
  }
}

}  // namespace swarm
