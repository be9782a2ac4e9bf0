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
