// PPO phase B on f32 MFMA versus the packed-VALU loop of k_ppo_grads
// (swarm_ppo.cuh): cycles per 128-sample tile of one
// wave owning 128 hidden units, the C3 policy's shapes (D = 1 feature,
// K + 1 = 5 output columns).  Measurement only; not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mfma_probe.hip -o tools/_variants/mfma_probe
//   ./tools/_variants/mfma_probe
// VALU: the whole phase B per sample (h, dWo += g h, dh = Wo g, mask,
//   db1 += dh, dW1 += dh x), two units per lane as packed fp32.
// MFMA: only the dWo product, v_mfma_f32_16x16x4_f32 with units as M (8
//   tiles of 16), the 5 columns padded to N = 16, samples as K (32 steps of
//   4), h recomputed per A fragment.  It is a lower bound on an MFMA phase B
//   (dh, the mask and the dW1 / db1 reductions would come on top).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kRow = 8;  // [g0..g4 | x | pad 2]
constexpr int kTiles = 64;

__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }

__global__ __launch_bounds__(256) void k_valu(const float* __restrict__ rows_g,
                                              const float* __restrict__ par,
                                              float* __restrict__ out,
                                              unsigned long long* __restrict__ cyc) {
  __shared__ __align__(16) float rows[4][128 * kRow];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = lane; k < 128 * kRow; k += 64) rows[wv][k] = rows_g[k];
  __syncthreads();
  const f2 w1p{par[lane], par[lane + 64]}, b1p{par[128 + lane], par[192 + lane]};
  f2 wop[5];
  for (int q = 0; q < 5; ++q) wop[q] = f2{par[256 + q * 128 + lane], par[256 + q * 128 + 64 + lane]};
  f2 gwop[5], gb1 = splat(0.0f), gw1 = splat(0.0f);
  for (int q = 0; q < 5; ++q) gwop[q] = splat(0.0f);
  const float* srow = rows[wv];
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_readcyclecounter();
  f4 na = *reinterpret_cast<const f4*>(srow), nb = *reinterpret_cast<const f4*>(srow + 4);
  for (int tile = 0; tile < kTiles; ++tile) {
#pragma unroll 2
    for (int s = 0; s < 128; ++s) {
      // the next sample's row is read while this one's is used (k_ppo_grads)
      const f4 a = na, b = nb;
      const int sn = (s + 1) & 127;
      na = *reinterpret_cast<const f4*>(srow + sn * kRow);
      nb = *reinterpret_cast<const f4*>(srow + sn * kRow + 4);
      const float g[5] = {a.x, a.y, a.z, a.w, b.x};
      const float x = b.y;
      f2 h = __builtin_elementwise_fma(w1p, splat(x), b1p);
      h = __builtin_elementwise_max(h, splat(0.0f));
      f2 dh = splat(0.0f);
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        gwop[q] = __builtin_elementwise_fma(splat(g[q]), h, gwop[q]);
        dh = __builtin_elementwise_fma(wop[q], splat(g[q]), dh);
      }
      dh.x = h.x > 0.0f ? dh.x : 0.0f;
      dh.y = h.y > 0.0f ? dh.y : 0.0f;
      gb1 += dh;
      gw1 = __builtin_elementwise_fma(dh, splat(x), gw1);
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float acc = gb1.x + gb1.y + gw1.x + gw1.y;
  for (int q = 0; q < 5; ++q) acc += gwop[q].x + gwop[q].y;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * 4 + wv] = t1 - t0;
}

// The VALU phase B with the rows of the next FOUR samples read while these
// four are used (one LDS wait per four samples instead of one per sample).
__global__ __launch_bounds__(256) void k_valu4(const float* __restrict__ rows_g,
                                               const float* __restrict__ par,
                                               float* __restrict__ out,
                                               unsigned long long* __restrict__ cyc) {
  __shared__ __align__(16) float rows[4][128 * kRow];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = lane; k < 128 * kRow; k += 64) rows[wv][k] = rows_g[k];
  __syncthreads();
  const f2 w1p{par[lane], par[lane + 64]}, b1p{par[128 + lane], par[192 + lane]};
  f2 wop[5];
  for (int q = 0; q < 5; ++q) wop[q] = f2{par[256 + q * 128 + lane], par[256 + q * 128 + 64 + lane]};
  f2 gwop[5], gb1 = splat(0.0f), gw1 = splat(0.0f);
  for (int q = 0; q < 5; ++q) gwop[q] = splat(0.0f);
  const float* srow = rows[wv];
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_readcyclecounter();
  f4 na[4], nb[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    na[u] = *reinterpret_cast<const f4*>(srow + u * kRow);
    nb[u] = *reinterpret_cast<const f4*>(srow + u * kRow + 4);
  }
  for (int tile = 0; tile < kTiles; ++tile) {
    for (int s0 = 0; s0 < 128; s0 += 4) {
      f4 a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = na[u];
        b[u] = nb[u];
        const int sn = (s0 + 4 + u) & 127;
        na[u] = *reinterpret_cast<const f4*>(srow + sn * kRow);
        nb[u] = *reinterpret_cast<const f4*>(srow + sn * kRow + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float g[5] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x};
        const float x = b[u].y;
        f2 h = __builtin_elementwise_fma(w1p, splat(x), b1p);
        h = __builtin_elementwise_max(h, splat(0.0f));
        f2 dh = splat(0.0f);
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          gwop[q] = __builtin_elementwise_fma(splat(g[q]), h, gwop[q]);
          dh = __builtin_elementwise_fma(wop[q], splat(g[q]), dh);
        }
        dh.x = h.x > 0.0f ? dh.x : 0.0f;
        dh.y = h.y > 0.0f ? dh.y : 0.0f;
        gb1 += dh;
        gw1 = __builtin_elementwise_fma(dh, splat(x), gw1);
      }
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float acc = gb1.x + gb1.y + gw1.x + gw1.y;
  for (int q = 0; q < 5; ++q) acc += gwop[q].x + gwop[q].y;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * 4 + wv] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_mfma(const float* __restrict__ rows_g,
                                              const float* __restrict__ par,
                                              float* __restrict__ out,
                                              unsigned long long* __restrict__ cyc) {
  __shared__ __align__(16) float rows[4][128 * kRow];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = lane; k < 128 * kRow; k += 64) rows[wv][k] = rows_g[k];
  __syncthreads();
  // A fragment of unit tile ut: row (unit) lane & 15, k (sample) lane >> 4
  float w1r[8], b1r[8];
  for (int ut = 0; ut < 8; ++ut) {
    w1r[ut] = par[ut * 16 + (lane & 15)];
    b1r[ut] = par[128 + ut * 16 + (lane & 15)];
  }
  f4 acc[8];
  for (int ut = 0; ut < 8; ++ut) acc[ut] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  const float* srow = rows[wv];
  const int col = lane & 15, kk = lane >> 4;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_readcyclecounter();
  float nx = srow[kk * kRow + 5], ng = col < 5 ? srow[kk * kRow + col] : 0.0f;
  for (int tile = 0; tile < kTiles; ++tile) {
#pragma unroll 2
    for (int kc = 0; kc < 32; ++kc) {
      const float x = nx, g = ng;  // B[k = sample][n = column]
      const int sn = (((kc + 1) & 31) * 4 + kk) * kRow;
      nx = srow[sn + 5];
      ng = col < 5 ? srow[sn + col] : 0.0f;
#pragma unroll
      for (int ut = 0; ut < 8; ++ut) {
        const float h = fmaxf(__builtin_fmaf(w1r[ut], x, b1r[ut]), 0.0f);
        acc[ut] = __builtin_amdgcn_mfma_f32_16x16x4f32(h, g, acc[ut], 0, 0, 0);
      }
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  float a = 0.0f;
  for (int ut = 0; ut < 8; ++ut) a += acc[ut].x + acc[ut].y + acc[ut].z + acc[ut].w;
  out[blockIdx.x * 256 + threadIdx.x] = a;
  if (lane == 0) cyc[blockIdx.x * 4 + wv] = t1 - t0;
}

int main() {
  const int blocks = 256;
  std::vector<float> rows(128 * kRow), par(256 + 5 * 128);
  for (int s = 0; s < 128; ++s)
    for (int c = 0; c < kRow; ++c) rows[s * kRow + c] = 0.01f * ((s * 7 + c * 3) % 17) - 0.05f;
  for (size_t i = 0; i < par.size(); ++i) par[i] = 0.02f * (float)((i * 13) % 23) - 0.2f;
  float *d_rows, *d_par, *d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_rows, rows.size() * 4);
  hipMalloc(&d_par, par.size() * 4);
  hipMalloc(&d_out, blocks * 256 * 4);
  hipMalloc(&d_cyc, blocks * 4 * 8);
  hipMemcpy(d_rows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_par, par.data(), par.size() * 4, hipMemcpyHostToDevice);
  std::vector<unsigned long long> cyc(blocks * 4);
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (v == 0)
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, d_rows, d_par, d_out, d_cyc);
      else if (v == 2)
        hipLaunchKernelGGL(k_valu4, dim3(blocks), dim3(256), 0, 0, d_rows, d_par, d_out, d_cyc);
      else
        hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, d_rows, d_par, d_out, d_cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.0f;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost);
      double mean = 0.0;
      for (auto c : cyc) mean += (double)c;
      mean /= (double)cyc.size();
      printf("%s rep %d: %.1f cycles per 128-sample tile per wave (128 units), launch %.3f ms\n",
             v == 0 ? "VALU phase B (all of it)       "
                    : (v == 2 ? "VALU phase B, rows 4 ahead     " : "MFMA dWo only                  "),
             rep,
             mean / kTiles, ms);
    }
  }
  hipFree(d_rows);
  hipFree(d_par);
  hipFree(d_out);
  hipFree(d_cyc);
  return 0;
}
