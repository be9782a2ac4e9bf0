// Dependent-chain latencies of one lone wave on gfx950 (round 6): the
// E = 1 run kernel is one wave per CU running a 100-sub-step recurrence, so
// what a sub-step costs is the latency of its dependency chain, not the
// issue rate.  Each test runs a chain of kIters dependent operations in one
// 64-thread block and reports shader cycles (s_memtime) per operation.
// Measurement only; not part of the library.
//   hipcc --offload-arch=gfx950 -O3 tools/chain_probe.hip -o tools/_variants/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

constexpr int kIters = 512;

#define PIN(x) __asm__ volatile("" : "+v"(x))

__device__ __forceinline__ unsigned long long now() {
  __builtin_amdgcn_s_waitcnt(0);
  return __builtin_amdgcn_s_memtime();
}

__global__ void k_probe(int test, float fa, float fb, unsigned long long* out, float* sink,
                        const int* chase) {
  __shared__ unsigned long long lds[128];
  const int lane = threadIdx.x;
  lds[lane] = 0;
  lds[lane + 64] = 0;
  __syncthreads();
  float x = fa + (float)lane * 1e-7f, y = fb, z = fa * 0.5f, w = fb * 0.25f;
  double dx = (double)x;
  int ix = lane;
  unsigned long long t0 = now(), t1 = 0;
  switch (test) {
    case 0:  // dependent v_fma_f32
      for (int k = 0; k < kIters; ++k) {
        x = __builtin_fmaf(x, fa, fb);
        PIN(x);
      }
      break;
    case 1:  // four independent fma chains interleaved (issue rate)
      for (int k = 0; k < kIters / 4; ++k) {
        x = __builtin_fmaf(x, fa, fb);
        y = __builtin_fmaf(y, fa, fb);
        z = __builtin_fmaf(z, fa, fb);
        w = __builtin_fmaf(w, fa, fb);
        PIN(x);
        PIN(y);
        PIN(z);
        PIN(w);
      }
      break;
    case 2:  // dependent v_rcp_f32
      for (int k = 0; k < kIters; ++k) {
        x = __builtin_amdgcn_rcpf(x);
        PIN(x);
      }
      break;
    case 3:  // dependent ds_bpermute (lane ^ 1)
      for (int k = 0; k < kIters; ++k) {
        ix = __builtin_amdgcn_ds_bpermute((lane ^ 1) << 2, ix);
        PIN(ix);
      }
      break;
    case 4:  // ds_add_u64 x4 then ds_read_b64 of the sum (the run's force round trip)
      for (int k = 0; k < kIters; ++k) {
        const unsigned long long v = (unsigned long long)(unsigned)ix;
        __hip_atomic_fetch_add(&lds[lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(&lds[lane + 64], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(&lds[lane ^ 1], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(&lds[(lane ^ 1) + 64], v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ix = (int)lds[lane];
        PIN(ix);
      }
      break;
    case 5:  // wave vote through SALU into a uniform branch, dependent
      for (int k = 0; k < kIters; ++k) {
        const bool all = __builtin_amdgcn_ballot_w64(x < 1e30f) == __builtin_amdgcn_read_exec();
        if (all)
          x = x + 1.0f;
        else
          x = x * 0.5f;
        PIN(x);
      }
      break;
    case 6:  // dependent v_fma_f64
      for (int k = 0; k < kIters; ++k) {
        dx = __builtin_fma(dx, (double)fa, (double)fb);
        __asm__ volatile("" : "+v"(dx));
      }
      break;
    case 7:  // f32 -> i32 -> f32 (v_cvt pair), dependent
      for (int k = 0; k < kIters; ++k) {
        x = (float)__float2int_rn(x);
        PIN(x);
      }
      break;
    case 8:  // dependent global loads (L2-resident pointer chase)
      for (int k = 0; k < kIters; ++k) {
        ix = chase[ix];
        PIN(ix);
      }
      break;
    case 9:  // dependent v_add_u32
      for (int k = 0; k < kIters; ++k) {
        ix = ix + 3;
        PIN(ix);
      }
      break;
    case 10:  // dependent v_mul_f32
      for (int k = 0; k < kIters; ++k) {
        x = x * fa;
        PIN(x);
      }
      break;
    case 11:  // ds_write_b64 then ds_read_b64 of another lane's word (LDS publish round trip)
      for (int k = 0; k < kIters; ++k) {
        lds[lane] = (unsigned long long)(unsigned)ix;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ix = (int)lds[lane ^ 1];
        PIN(ix);
      }
      break;
#define FOUR_CHAINS(CASE, ASM)                                   \
    case CASE: {                                                 \
      uint32_t a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3; \
      const uint32_t m = 0xD2511F53u;                            \
      for (int k = 0; k < kIters / 4; ++k) {                     \
        ASM(a0);                                                 \
        ASM(a1);                                                 \
        ASM(a2);                                                 \
        ASM(a3);                                                 \
      }                                                          \
      ix = (int)(a0 ^ a1 ^ a2 ^ a3);                             \
      break;                                                     \
    }
#define MAD64(a)                                                                         \
  {                                                                                      \
    uint64_t r_, c_;                                                                     \
    __asm__ volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r_), "=s"(c_) : "v"(a), "v"(m)); \
    a = (uint32_t)r_;                                                                    \
  }
#define MULHI(a) __asm__ volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(m))
#define MULLO(a) __asm__ volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(m))
#define XOR(a) __asm__ volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(m))
#define CVT(a) __asm__ volatile("v_cvt_f32_u32 %0, %0" : "+v"(a))
#define PK_CHAINS(CASE, INSN)                                              \
    case CASE: {                                                           \
      typedef float f2 __attribute__((ext_vector_type(2)));               \
      f2 a0 = {x, y}, a1 = {z, w}, a2 = {x, w}, a3 = {z, y};               \
      const f2 m = {fa, fb};                                               \
      for (int k = 0; k < kIters / 4; ++k) {                               \
        __asm__ volatile(INSN : "+v"(a0) : "v"(m));                        \
        __asm__ volatile(INSN : "+v"(a1) : "v"(m));                        \
        __asm__ volatile(INSN : "+v"(a2) : "v"(m));                        \
        __asm__ volatile(INSN : "+v"(a3) : "v"(m));                        \
      }                                                                    \
      x = a0.x + a1.y + a2.x + a3.y;                                       \
      break;                                                               \
    }
    // packed fp32 (two floats per lane per instruction)
    PK_CHAINS(18, "v_pk_fma_f32 %0, %0, %1, %1")
    PK_CHAINS(19, "v_pk_mul_f32 %0, %0, %1")
    // issue rates of Philox's and the table normals' integer operations
    FOUR_CHAINS(13, MAD64)
    FOUR_CHAINS(14, MULHI)
    FOUR_CHAINS(15, MULLO)
    FOUR_CHAINS(16, XOR)
    FOUR_CHAINS(17, CVT)
    case 12:  // DPP row swap (quad_perm [1,0,3,2]) dependent
      for (int k = 0; k < kIters; ++k) {
        ix = __builtin_amdgcn_mov_dpp(ix, 0xB1, 0xF, 0xF, false);
        PIN(ix);
      }
      break;
  }
  t1 = now();
  if (lane == 0) out[test] = t1 - t0;
  sink[lane] = x + y + z + w + (float)dx + (float)ix;
}

// Shorter correctly rounded reciprocals for the pair force's 1/r^2: every
// float in [2^-96, 2^96] against 1.0f / x.  variant 0: rcp + one residual
// correction (3 dependent ops); 1: rcp + Newton step + correction (5).
__global__ void k_rcp_variants(int variant, unsigned long long* bad, unsigned* first) {
  const uint32_t lo = 31u << 23, hi = 223u << 23;
  const uint32_t stride = gridDim.x * blockDim.x;
  unsigned long long nb = 0;
  for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi; b += stride) {
    const float x = __uint_as_float(b);
    float y = __builtin_amdgcn_rcpf(x);
    if (variant == 1) {
      const float e = __builtin_fmaf(-x, y, 1.0f);
      y = __builtin_fmaf(e, y, y);
    }
    const float r = __builtin_fmaf(-x, y, 1.0f);
    const float res = __builtin_fmaf(r, y, y);
    if (__float_as_uint(res) != __float_as_uint(1.0f / x)) {
      ++nb;
      atomicCAS(first, 0u, b);
    }
  }
  if (nb) atomicAdd(bad, nb);
}

// WRITE_SIZE calibration: the noise table's store
// patterns over a known byte count.  k_write_f4: one streaming 16-B store
// per lane at consecutive 16-B addresses (the round-6 fill); k_write_3x4:
// three streaming 4-B stores per lane at a 48-B lane stride (round 5's).
// Each writes `bytes` bytes exactly once; rocprofv3 --pmc WRITE_SIZE on
// `chain_probe --write-cal` gives the counter's reading of each.
__global__ void k_write_f4(float* __restrict__ out, size_t n4) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) {
    const f32x4 v = {(float)i, 1.0f, 2.0f, 3.0f};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out) + i);
  }
}
__global__ void k_write_3x4(float* __restrict__ out, size_t n12) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n12) {
    float* o = out + 12 * i;  // 48-B record group; stores at words 0, 1, 2 (x 4 sub-steps)
    for (int j = 0; j < 4; ++j) {
      __builtin_nontemporal_store((float)i, o + 3 * j);
      __builtin_nontemporal_store(1.0f, o + 3 * j + 1);
      __builtin_nontemporal_store(2.0f, o + 3 * j + 2);
    }
  }
}

static int write_cal() {
  const size_t bytes = (size_t)24 << 20;  // C5's table size
  float* d;
  if (hipMalloc(&d, bytes)) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_write_f4, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, d,
                       bytes / 16);
    hipLaunchKernelGGL(k_write_3x4, dim3((unsigned)(bytes / 48 / 256)), dim3(256), 0, 0, d,
                       bytes / 48);
  }
  hipDeviceSynchronize();
  printf("write calibration: %zu bytes per launch of k_write_f4 and k_write_3x4\n", bytes);
  hipFree(d);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "--write-cal") return write_cal();
  const char* names[] = {"v_fma_f32 dependent",   "v_fma_f32 4 chains",   "v_rcp_f32 dependent",
                         "ds_bpermute dependent", "4 ds_add_u64 + read",  "ballot vote + branch",
                         "v_fma_f64 dependent",   "cvt f32->i32->f32",    "global load chase (L2)",
                         "v_add_u32 dependent",   "v_mul_f32 dependent",  "ds_write + ds_read other lane",
                         "DPP quad swap dependent", "v_mad_u64_u32 4 chains",
                         "v_mul_hi_u32 4 chains",   "v_mul_lo_u32 4 chains", "v_xor_b32 4 chains",
                         "v_cvt_f32_u32 4 chains", "v_pk_fma_f32 4 chains",
                         "v_pk_mul_f32 4 chains"};
  const int ntest = 20;
  unsigned long long* d_out;
  float* d_sink;
  int* d_chase;
  hipMalloc(&d_out, 64 * sizeof(unsigned long long));
  hipMalloc(&d_sink, 64 * sizeof(float));
  int h_chase[4096];
  for (int k = 0; k < 4096; ++k) h_chase[k] = (k * 37 + 11) & 4095;
  hipMalloc(&d_chase, sizeof(h_chase));
  hipMemcpy(d_chase, h_chase, sizeof(h_chase), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
    for (int t = 0; t < ntest; ++t)
      hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, t, 1.0000001f, 1e-7f, d_out, d_sink,
                         d_chase);
    hipDeviceSynchronize();
    unsigned long long h[64];
    hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    if (rep == 2)
      for (int t = 0; t < ntest; ++t)
        printf("%-32s %7.1f cycles/op\n", names[t], (double)h[t] / kIters);
  }
  for (int v = 0; v < 2; ++v) {
    unsigned long long* d;
    hipMalloc(&d, 16);
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL(k_rcp_variants, dim3(8192), dim3(256), 0, 0, v, d,
                       reinterpret_cast<unsigned*>(d + 1));
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("rcp variant %d: %llu mismatches over [2^-96, 2^96] (first 0x%08x)\n", v, h[0],
           (unsigned)h[1]);
    hipFree(d);
  }
  return 0;
}
