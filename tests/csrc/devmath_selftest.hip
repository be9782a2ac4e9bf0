// Test-only kernel: evaluates the engine's device arithmetic (swarm_device.cuh)
// on host-supplied inputs so tests can compare it bit for bit with the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../swarmrl_amd/csrc/swarm_device.cuh"

__global__ void k_math(const float* x, const uint32_t* a, int n, float* o_sqrt, float* o_log,
                       float* o_acos, float* o_sin, float* o_cos, float* o_g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o_sqrt[i] = swarm::sqrt_rn(x[i]);
  o_log[i] = swarm::logf_fixed(x[i]);
  o_acos[i] = swarm::acosf_fixed(x[i] * 2.0f - 1.0f);
  float s, c;
  swarm::sincos_turn(a[i], &s, &c);
  o_sin[i] = s;
  o_cos[i] = c;
  float g[3];
  swarm::normals3(42u, 0u, (uint32_t)i, 7ull, 0u, g);
  for (int k = 0; k < 3; ++k) o_g[3 * i + k] = g[k];
  // grouped step normals: particle i % 64, 9 consecutive sub-steps carried
  // by one StepNoise from t0 = 1000 + i / 64 (every alignment), the last
  // also from scratch
  if (i < 4096) {
    swarm::StepNoise sn;
    const uint64_t t0 = 1000ull + (uint64_t)(i / 64);
    float* o = o_g + 4 * (size_t)n + 30 * (size_t)i;
    for (int s = 0; s < 9; ++s) {
      sn.next(42u, 5u, (uint32_t)(i % 64), t0 + s, s == 0, g);
      for (int k = 0; k < 3; ++k) o[3 * s + k] = g[k];
    }
    swarm::step_normals(42u, 5u, (uint32_t)(i % 64), t0 + 8, g);
    for (int k = 0; k < 3; ++k) o[27 + k] = g[k];
  }
  // branchless sqrt on the Box-Muller radius range [1.19e-7, 33.3]
  const float xp = 1.1920929e-07f + x[i] * 40.0f;
  o_g[3 * (size_t)n + i] = swarm::sqrt_pos(xp > 0.0f ? xp : 1.0f);
}

extern "C" int devmath_selftest(const float* x, const uint32_t* a, int n, float* out) {
  float *dx, *dout;
  uint32_t* da;
  const size_t words = (size_t)n * 9 + 30 * (size_t)(n < 4096 ? n : 4096);
  if (hipMalloc(&dx, n * 4) || hipMalloc(&da, n * 4) || hipMalloc(&dout, words * 4)) return 1;
  (void)hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_math, dim3((n + 255) / 256), dim3(256), 0, 0, dx, da, n, dout, dout + n,
                     dout + 2 * (size_t)n, dout + 3 * (size_t)n, dout + 4 * (size_t)n,
                     dout + 5 * (size_t)n);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  (void)hipMemcpy(out, dout, words * 4, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(da);
  (void)hipFree(dout);
  return 0;
}

// rcp_rn (the run kernels' 1/r^2) against the compiler's IEEE division
// 1.0f / x for every float bit pattern in [lo, hi): mismatch count and the
// first mismatching pattern (0 if none).
__global__ void k_rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
  const uint32_t stride = gridDim.x * blockDim.x;
  unsigned long long nb = 0;
  for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
    const float x = __uint_as_float(b);
    if (__float_as_uint(swarm::rcp_rn(x)) != __float_as_uint(1.0f / x)) {
      ++nb;
      atomicCAS(first, 0u, b);
    }
  }
  if (nb) atomicAdd(bad, nb);
}

// i64 -> fp32 conversions (fast int32 path and the wide path) on given values
__global__ void k_i64(const int64_t* v, int n, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a, b;
  swarm::i64x2_to_f32(v[i], v[(i + 1) % n], &a, &b);
  out[3 * i] = a;
  out[3 * i + 1] = b;
  out[3 * i + 2] = swarm::i64_to_f32(v[i]);
}

extern "C" int devmath_rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad,
                                 uint32_t* first) {
  unsigned long long* d;
  if (hipMalloc(&d, 16)) return 1;
  (void)hipMemset(d, 0, 16);
  hipLaunchKernelGGL(k_rcp_check, dim3(4096), dim3(256), 0, 0, lo, hi, d,
                     reinterpret_cast<uint32_t*>(d + 1));
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  unsigned long long h[2];
  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  *bad = h[0];
  *first = (uint32_t)h[1];
  return 0;
}

extern "C" int devmath_i64_to_f32(const int64_t* v, int n, float* out) {
  int64_t* dv;
  float* dout;
  if (hipMalloc(&dv, n * 8) || hipMalloc(&dout, n * 12)) return 1;
  (void)hipMemcpy(dv, v, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_i64, dim3((n + 255) / 256), dim3(256), 0, 0, dv, n, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  (void)hipMemcpy(out, dout, n * 12, hipMemcpyDeviceToHost);
  (void)hipFree(dv);
  (void)hipFree(dout);
  return 0;
}

// f2i32_sat (the 2-D translation's conversion) on host-supplied values
__global__ void k_f2i32_sat(const float* v, int n, int32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = swarm::f2i32_sat(v[i]);
}

extern "C" int devmath_f2i32_sat(const float* v, int n, int32_t* out) {
  float* dv;
  int32_t* dout;
  if (hipMalloc(&dv, n * 4) || hipMalloc(&dout, n * 4)) return 1;
  (void)hipMemcpy(dv, v, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_f2i32_sat, dim3((n + 255) / 256), dim3(256), 0, 0, dv, n, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  (void)hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
  (void)hipFree(dv);
  (void)hipFree(dout);
  return 0;
}
