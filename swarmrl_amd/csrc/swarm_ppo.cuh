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
// per-sample gradients; the caller's optimizer takes the step.  Each unit's
// parameters are read as wave-uniform scalar loads by the sample-major loops
// (for the gradient kernel from a per-unit table laid out beside the GAE).
// All fp32 arithmetic with explicit fmaf; cross-sample sums in a fixed order
// (run-to-run identical).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swarm {

constexpr int kPpoMaxIn = 32;
constexpr int kPpoMaxK = 16;
constexpr int kPpoMaxHidden = 256;
constexpr int kPpoBlocks = 2048;  // grad blocks (four tile waves or two unit waves each)

// Gradient layout (floats): W1 [H][D] | b1 [H] | Wa [K][H] | ba [K] | Wc [H] | bc
__host__ __device__ inline int ppo_grad_size(int d, int h, int k) {
  return h * d + h + k * h + k + h + 1;
}

// Per-unit parameter rows, the wave-uniform operands of the gradient
// kernel's sample-major loop (one scalar-load row per unit):
// [Wa[:, u], Wc[u], 0 ... | W1[u, :], b1[u], 0 ...]
template <int D, int K>
struct PpoTable {
  static constexpr int kHeads = (K + 1 + 7) / 8 * 8;
  static constexpr int kW1 = kHeads;
  static constexpr int kB1 = kHeads + D;
  static constexpr int kStride = kHeads + (D + 1 + 7) / 8 * 8;
};

// Entry t of the table (rows = hidden rounded up to the grads block, zero
// rows past hidden); written by extra workgroups of the GAE launch.
template <int D, int K>
__device__ __forceinline__ void ppo_pack_entry(const float* __restrict__ w1,
                                               const float* __restrict__ b1, int d, int hidden,
                                               const float* __restrict__ wa, int k,
                                               const float* __restrict__ wc, int rows, int t,
                                               float* __restrict__ table) {
  using Tb = PpoTable<D, K>;
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

// V of every sample: one thread per four samples -- two pairs of adjacent
// samples in packed fp32 registers (v_pk_fma_f32), their features in
// registers, each unit's parameters wave-uniform scalar loads (amortised
// over the four).
template <int D>
__global__ __launch_bounds__(256) void k_ppo_values(const float* __restrict__ x, int n, int d,
                                                    const float* __restrict__ w1,
                                                    const float* __restrict__ b1, int hidden,
                                                    const float* __restrict__ wc,
                                                    const float* __restrict__ bc,
                                                    float* __restrict__ values) {
  const long s = 4 * ((long)blockIdx.x * blockDim.x + threadIdx.x);
  if (s >= n) return;
  ppo_f2 xs[2][D];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    // past n: the last sample again (computed, not stored)
    const float* xa = x + (size_t)min(s + 2 * p, (long)n - 1) * d;
    const float* xb = x + (size_t)min(s + 2 * p + 1, (long)n - 1) * d;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const float va = xa[min(c, d - 1)], vb = xb[min(c, d - 1)];
      xs[p][c] = c < d ? ppo_f2{va, vb} : ppo_f2{0.0f, 0.0f};
    }
  }
  ppo_f2 v[2] = {(ppo_f2)bc[0], (ppo_f2)bc[0]};
#pragma unroll 4
  for (int j = 0; j < hidden; ++j) {
    const float bj = b1[j], cj = wc[j];
    float wj[D];
#pragma unroll
    for (int c = 0; c < D; ++c) wj[c] = w1[(size_t)j * d + min(c, d - 1)];  // c >= d: x is 0
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      ppo_f2 h = bj;
#pragma unroll
      for (int c = 0; c < D; ++c) h = __builtin_elementwise_fma((ppo_f2)wj[c], xs[p][c], h);
      h = __builtin_elementwise_max(h, (ppo_f2)0.0f);
      v[p] = __builtin_elementwise_fma((ppo_f2)cj, h, v[p]);
    }
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (s + 2 * p < n) values[s + 2 * p] = v[p].x;
    if (s + 2 * p + 1 < n) values[s + 2 * p + 1] = v[p].y;
  }
}

// V at small sample counts, where the per-thread chain over all units is
// the latency: a workgroup of 4 waves takes 64 samples (lane = sample) and
// wave w sums units [w H/4, (w + 1) H/4) (wave-uniform rows); the four
// partials are added in a fixed order.
template <int D>
__global__ __launch_bounds__(256) void k_ppo_values_split(const float* __restrict__ x, int n,
                                                          int d, const float* __restrict__ w1,
                                                          const float* __restrict__ b1,
                                                          int hidden,
                                                          const float* __restrict__ wc,
                                                          const float* __restrict__ bc,
                                                          float* __restrict__ values) {
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
    float h = b1[j];
#pragma unroll
    for (int c = 0; c < D; ++c)  // clamped load: a feature c >= d is zero
      h = fmaf(w1[(size_t)j * d + min(c, d - 1)], xs[c], h);
    v = fmaf(wc[j], fmaxf(h, 0.0f), v);
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
// Workgroups past n_gae (blockIdx.x >= n_gae) lay out the gradient
// kernel's parameter table instead (PpoPack: no launch of their own).
struct PpoPack {
  const float *w1, *b1, *wa, *wc;
  int d, hidden, k, rows;
  float* table;
};

template <int TM, int D, int K>
__global__ __launch_bounds__(256) void k_ppo_gae(const float* __restrict__ rewards,
                                                 const float* __restrict__ values, int T, int S,
                                                 float gamma, float lambda,
                                                 float* __restrict__ adv, float* __restrict__ dv,
                                                 double* __restrict__ part, int n_gae,
                                                 PpoPack pk) {
  __shared__ double red[2][4];
  if ((int)blockIdx.x >= n_gae) {
    ppo_pack_entry<D, K>(pk.w1, pk.b1, pk.d, pk.hidden, pk.wa, pk.k, pk.wc, pk.rows,
                         ((int)blockIdx.x - n_gae) * blockDim.x + threadIdx.x, pk.table);
    return;
  }
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

// A sample's row in LDS: dL/d(logits) [K] | dL/dV | features [D], padded to
// whole float4s (read back by every lane at one address: a broadcast).
template <int D, int K>
struct PpoRow {
  static constexpr int kRow = (K + 1 + D + 3) / 4 * 4;
};

// Floats a lane hands over in the final combine of a block's tile waves.
template <int D, int K>
__host__ __device__ constexpr int ppo_combine_floats() {
  return 2 * (D + 1 + K + 1) + K + 1;
}

template <int NW, int NT, bool kCoop, int D, int K>
__host__ __device__ constexpr int ppo_grads_lds_floats() {
  // sample rows [128][kRow] per tile in flight (NT, or one shared by the
  // kCoop waves) | logit partials of the other waves of a tile
  // [max(NW, NT) - 1][K][128]; after the tiles, the combine buffer [kC][64]
  // aliases them
  constexpr int rows = (kCoop ? 1 : NT) * 128 * PpoRow<D, K>::kRow;
  constexpr int part = ((kCoop ? NT : NW) - 1) * K * 128;
  constexpr int comb = NT > 1 ? 64 * ppo_combine_floats<D, K>() : 0;
  return rows + part > comb ? rows + part : comb;
}

// The LDS hand-over between the phases of one tile: the whole block when
// units are split over NW > 1 waves, else the one wave that owns the tile
// (LDS operations of a wave complete in order; the fences keep the compiler
// from moving memory operations across).
template <int NW>
__device__ __forceinline__ void ppo_group_sync() {
  if constexpr (NW > 1) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

__device__ __forceinline__ ppo_f2 ppo_splat(float v) { return ppo_f2{v, v}; }

// Per-block parameter gradients.  NW waves each own 128 hidden units of a
// tile (hidden > 128), or (NW = 1) NT waves each take their own tiles and
// add their sums in a fixed order at the end; kCoop (few samples: a wave per
// tile would leave most SIMDs idle): the NT waves share each tile, phase F
// split over their units and phase B over their samples.  Dynamic LDS
// ppo_grads_lds_floats<NW, NT, kCoop, D, K>() floats; partial:
// [gridDim.x][ppo_grad_size].  Tiles of 128 samples, three phases, no
// cross-lane broadcasts (v_readlane) and no transposes:
//   F  lane = the sample pair (s, s + 64) as the two halves of packed fp32
//      registers: the logits over the wave's units, each unit's hidden
//      activation recomputed from its wave-uniform table row (scalar loads)
//      -- D + 1 + K v_pk_fma_f32 per unit and pair.  The value head is not
//      needed: dL/dV comes from k_ppo_gae.
//   P  wave 0, lane = sample: the other waves' logit partials added in a
//      fixed order, dL/dz of the clipped surrogate and the entropy term, the
//      output-bias sums; each sample's row [dL/dz, dL/dV, x] to LDS
//   B  lane = the unit pair (u, u + 64), the 128 samples in order: each row
//      read by every lane at one address (LDS broadcast, float4), h
//      recomputed, then dWo += g h, dh = Wo g (masked by h > 0), db1 += dh,
//      dW1 += dh x -- packed FMAs over the two units.
// Every sum runs in a fixed order (run-to-run identical).  The tensor shapes
// (1-128-(4+1) stock) make matrix cores a poor fit: the heads' 5 columns
// would fill 5 of every 16 rows of a v_mfma_f32_16x16x4_f32, whose f32 rate
// is the packed-VALU rate on gfx950 (MI355X_MICROARCH.md, "Peak FP32").
template <int NW, int NT, bool kCoop, int D, int K>
__global__ __launch_bounds__(64 * NW * NT) void k_ppo_grads(
    const float* __restrict__ x, int n, int d, const float* __restrict__ w1,
    const float* __restrict__ b1, int hidden, const float* __restrict__ wa,
    const float* __restrict__ ba, int k, const float* __restrict__ wc,
    const float* __restrict__ bc, const int64_t* __restrict__ actions,
    const float* __restrict__ old_logp, const float* __restrict__ adv,
    const float* __restrict__ dvalue, const double* __restrict__ gae_part, int n_part,
    const float* __restrict__ table, float clip_eps, float c_ent, float* __restrict__ partial) {
  using Tb = PpoTable<D, K>;
  constexpr int KP = K + 1, kTab = Tb::kStride, kRow = PpoRow<D, K>::kRow;
  extern __shared__ float ppo_lds[];
  static_assert(NW == 1 || NT == 1, "tile waves or unit waves, not both");
  static_assert(!kCoop || (NW == 1 && 128 % NT == 0), "kCoop splits one 128-unit wave's work");
  // the waves that share a tile (their logit partials meet in LDS)
  constexpr int NX = kCoop ? NT : NW;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int w = NW > 1 ? wid : 0;  // unit wave
  const int t = NW > 1 ? 0 : wid;  // tile wave
  const int wx = NX > 1 ? wid : 0;  // index among the waves of a tile
  const int wu = __builtin_amdgcn_readfirstlane(w);
  float* srow = ppo_lds + (kCoop ? 0 : t) * 128 * kRow;  // [128][kRow]
  float* red = ppo_lds + (kCoop ? 1 : NT) * 128 * kRow;  // [NX - 1][K][128]
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
  float bo[K];
#pragma unroll
  for (int q = 0; q < K; ++q) bo[q] = q < k ? ba[q] : 0.0f;
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
  // this wave's unit rows (zero rows past hidden up to 128 NW), whole quads;
  // kCoop: its share of them in phase F, and its share of the samples in B
  const float* urows = table + (size_t)wu * 128 * kTab;
  int nunits = (min(128, hidden - 128 * wu) + 3) & ~3;
  int s_lo = 0, s_hi = 128;
  if constexpr (kCoop) {
    const int tu = __builtin_amdgcn_readfirstlane(t);
    const int per_u = 128 / NT;
    urows += (size_t)tu * per_u * kTab;
    nunits = max(0, min(per_u, nunits - tu * per_u));
    s_lo = tu * (128 / NT);
    s_hi = s_lo + 128 / NT;
  }
  const long tiles = ((long)n + 127) / 128;
  const long t0 = kCoop ? (long)blockIdx.x : (long)blockIdx.x * NT + t;
  const long tstep = kCoop ? (long)gridDim.x : (long)gridDim.x * NT;
  for (long tile = t0; tile < tiles; tile += tstep) {
    const long sa = tile * 128 + lane, sb = sa + 64;
    ppo_f2 xs[D];
    {
      // clamped loads and a select, no branches (a feature c >= d meets a
      // zero weight; a sample past n has dL/dz = 0 below, so adds nothing)
      const float* xa = x + (size_t)min(sa, (long)n - 1) * d;
      const float* xb = x + (size_t)min(sb, (long)n - 1) * d;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        const float va = xa[min(c, d - 1)], vb = xb[min(c, d - 1)];
        xs[c] = c < d ? ppo_f2{va, vb} : ppo_splat(0.0f);
      }
    }
    // F: logits of the sample pair over this wave's units
    ppo_f2 z[K];
#pragma unroll
    for (int q = 0; q < K; ++q) z[q] = ppo_splat(0.0f);
#pragma unroll 8
    for (int u = 0; u < nunits; ++u) {
      const float* r = urows + (size_t)u * kTab;
      ppo_f2 h = ppo_splat(r[Tb::kB1]);
#pragma unroll
      for (int c = 0; c < D; ++c) h = __builtin_elementwise_fma(ppo_splat(r[Tb::kW1 + c]), xs[c], h);
      h = __builtin_elementwise_max(h, ppo_splat(0.0f));
#pragma unroll
      for (int q = 0; q < K; ++q) z[q] = __builtin_elementwise_fma(ppo_splat(r[q]), h, z[q]);
    }
    if (NX > 1 && wx > 0) {
#pragma unroll
      for (int q = 0; q < K; ++q) {
        red[((wx - 1) * K + q) * 128 + lane] = z[q].x;
        red[((wx - 1) * K + q) * 128 + 64 + lane] = z[q].y;
      }
    }
    if (NX > 1) __syncthreads();
    // P: dL/dz and dL/dV of each sample, its row to LDS
    if (wx == 0) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const long si = half ? sb : sa;
        const int slot = half * 64 + lane;
        float acc[K];
#pragma unroll
        for (int q = 0; q < K; ++q) {
          acc[q] = half ? z[q].y : z[q].x;
#pragma unroll
          for (int ww = 1; ww < NX; ++ww) acc[q] += red[((ww - 1) * K + q) * 128 + slot];
        }
        float g[KP];
#pragma unroll
        for (int q = 0; q < KP; ++q) g[q] = 0.0f;
        if (si < n) {
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
        float* row = srow + slot * kRow;
#pragma unroll
        for (int q = 0; q < KP; ++q) {
          gbias[q] += g[q];
          row[q] = g[q];
        }
#pragma unroll
        for (int c = 0; c < D; ++c) row[KP + c] = half ? xs[c].y : xs[c].x;
      }
    }
    ppo_group_sync<NX>();
    // B: both units' gradients over the tile's samples (kCoop: this wave's
    // share); the next sample's row is read while this one's is used
    float4 nxt[kRow / 4];
#pragma unroll
    for (int i = 0; i < kRow / 4; ++i)
      nxt[i] = reinterpret_cast<const float4*>(srow + s_lo * kRow)[i];
#pragma unroll 2
    for (int s = s_lo; s < s_hi; ++s) {
      float rv[kRow];
#pragma unroll
      for (int i = 0; i < kRow / 4; ++i) {
        const float4 v = nxt[i];
        rv[4 * i] = v.x;
        rv[4 * i + 1] = v.y;
        rv[4 * i + 2] = v.z;
        rv[4 * i + 3] = v.w;
      }
      const int sn = min(s + 1, s_hi - 1);
#pragma unroll
      for (int i = 0; i < kRow / 4; ++i)
        nxt[i] = reinterpret_cast<const float4*>(srow + sn * kRow)[i];
      ppo_f2 h = b1p;
#pragma unroll
      for (int c = 0; c < D; ++c) h = __builtin_elementwise_fma(w1p[c], ppo_splat(rv[KP + c]), h);
      h = __builtin_elementwise_max(h, ppo_splat(0.0f));
      ppo_f2 dh = ppo_splat(0.0f);
#pragma unroll
      for (int q = 0; q < KP; ++q) {
        const ppo_f2 gs = ppo_splat(rv[q]);
        gwop[q] = __builtin_elementwise_fma(gs, h, gwop[q]);
        dh = __builtin_elementwise_fma(wop[q], gs, dh);
      }
      dh.x = h.x > 0.0f ? dh.x : 0.0f;
      dh.y = h.y > 0.0f ? dh.y : 0.0f;
      gb1p += dh;
#pragma unroll
      for (int c = 0; c < D; ++c)
        gw1p[c] = __builtin_elementwise_fma(dh, ppo_splat(rv[KP + c]), gw1p[c]);
    }
    ppo_group_sync<NX>();  // the rows (and red) are rewritten next tile
  }
  if constexpr (NT > 1) {
    // tile waves 1.. hand their sums to wave 0 in order: ((s0 + s1) + s2) + ...
    float* cb = ppo_lds + lane;  // [ppo_combine_floats][64]
    auto xfer = [&](bool put) {
      int i = 0;
      auto two = [&](ppo_f2& v) {
        if (put) {
          cb[64 * i] = v.x;
          cb[64 * (i + 1)] = v.y;
        } else {
          v += ppo_f2{cb[64 * i], cb[64 * (i + 1)]};
        }
        i += 2;
      };
#pragma unroll
      for (int c = 0; c < D; ++c) two(gw1p[c]);
      two(gb1p);
#pragma unroll
      for (int q = 0; q < KP; ++q) two(gwop[q]);
#pragma unroll
      for (int q = 0; q < KP; ++q) {
        if (put)
          cb[64 * i] = gbias[q];
        else
          gbias[q] += cb[64 * i];
        ++i;
      }
    };
    for (int src = 1; src < NT; ++src) {
      __syncthreads();  // the tiles' rows, or the previous round's buffer, are done with
      if (t == src) xfer(true);
      __syncthreads();
      if (t == 0) xfer(false);
    }
  }
  // output-bias gradients: wave 0's per-lane sums, reduced across the wave
  if (wid == 0) {
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
    if (t == 0 && u < hidden) {
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

// The optimizer step fused into the reduce (swarm_ppo_epoch_step): torch
// Adam (torch.optim.Adam, weight_decay 0, no amsgrad / maximize) on the six
// tensors w1 | b1 | wa | ba | wc | bc, their moments and per-tensor step
// counts in place -- the sequence of torch's fused Adam: step + 1,
// m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p -= lr / (1 - b1^step) * m
// / (sqrt(v) / sqrt(1 - b2^step) + eps), in fp32.
struct AdamArgs {
  float lr, beta1, beta2, eps;
  float* param[6];
  float* m[6];
  float* v[6];
  float* step[6];
  int seg[7];  // parameter index ranges of the six tensors
};

__global__ __launch_bounds__(1024) void k_ppo_reduce_adam(const float* __restrict__ partial,
                                                          int n_blocks, int size,
                                                          float* __restrict__ grad, AdamArgs a,
                                                          uint32_t* __restrict__ ticket) {
  __shared__ double red[16][64];
  __shared__ int last;
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
    const float g = (float)t;
    grad[p] = g;
    int sg = 0;
    while (sg < 5 && p >= a.seg[sg + 1]) ++sg;
    const int off = p - a.seg[sg];
    // the step count before this step: every workgroup reads it before its
    // ticket, the last one writes step + 1
    const float step = *a.step[sg] + 1.0f;
    const float bc1 = 1.0f - powf(a.beta1, step);
    const float bc2 = 1.0f - powf(a.beta2, step);
    const float bc2s = sqrtf(bc2);
    float m = a.m[sg][off], v = a.v[sg][off];
    m = a.beta1 * m + (1.0f - a.beta1) * g;
    v = a.beta2 * v + (1.0f - a.beta2) * g * g;
    const float step_size = a.lr / bc1;
    const float denom = sqrtf(v) / bc2s + a.eps;
    a.param[sg][off] = a.param[sg][off] - step_size * m / denom;
    a.m[sg][off] = m;
    a.v[sg][off] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tk = atomicAdd(ticket, 1u);
    last = tk == gridDim.x - 1;
    if (last) *ticket = 0u;  // the next step's count (graph replays)
  }
  __syncthreads();
  if (last && threadIdx.x < 6) *a.step[threadIdx.x] = *a.step[threadIdx.x] + 1.0f;
}

}  // namespace swarm
