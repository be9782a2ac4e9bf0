// swarm_device.cuh -- device arithmetic shared by the engine kernels.
//
// Every function here fixes its fp32 operation sequence (the file is compiled
// with -ffp-contract=off), so a kernel result is a deterministic function of
// its inputs and is reproduced bit for bit by the CPU oracle (oracle/), which
// restates the same number formats independently.  See DESIGN.md "Number
// formats".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/swarm_normal_table.h"

namespace swarm {

// ---------------------------------------------------------------- Philox
// Philox4x32-10 (Salmon et al., SC'11).  Key = (seed lo, seed hi ^ env),
// counter = (particle id, step lo, step hi, stream tag).
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c.z;
    u32x4 n;
    if (r == 0) {  // (the first round's x word is wave-uniform: scalar ALU)
      n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
      n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    } else {  // three-input XOR in one v_bitop3_b32 (gfx950; two v_xor_b32 otherwise)
      n.x = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96);
      n.z = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96);
    }
    n.y = (uint32_t)p1;
    n.w = (uint32_t)p0;
    c = n;
  }
  return c;
}

// ------------------------------------------------- elementary functions
// Correctly rounded fp32 square root.  hipcc (ROCm 7.2) lowers sqrtf and
// __fsqrt_rn to the bare v_sqrt_f32 (<= 1 ulp); the host's sqrtf is IEEE
// exact.  Refine the hardware value by testing its two neighbours with an
// exact-residual FMA (the sequence LLVM emits for correctly rounded sqrt).
__device__ __forceinline__ float sqrt_rn(float x) {
  if (!(x > 0.0f) || x == __builtin_inff()) return __builtin_sqrtf(x);
  const bool tiny = x < 1.2621774483536189e-29f;  // 2^-96: keep clear of denormals
  const float xs = tiny ? x * 4294967296.0f : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const uint32_t si = __float_as_uint(s);
  const float s_dn = __uint_as_float(si - 1u);
  const float s_up = __uint_as_float(si + 1u);
  const float r_dn = __builtin_fmaf(-s_dn, s, xs);
  const float r_up = __builtin_fmaf(-s_up, s, xs);
  s = (r_dn <= 0.0f) ? s_dn : s;
  s = (r_up > 0.0f) ? s_up : s;
  return tiny ? s * 1.52587890625e-05f : s;  // * 2^-16
}

// Correctly rounded sqrt for a positive normal finite x (the Box-Muller
// radius -2 ln u >= 1.19e-7): no special-case or denormal branch.
__device__ __forceinline__ float sqrt_pos(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  const uint32_t si = __float_as_uint(s);
  const float s_dn = __uint_as_float(si - 1u);
  const float s_up = __uint_as_float(si + 1u);
  const float r_dn = __builtin_fmaf(-s_dn, s, x);
  const float r_up = __builtin_fmaf(-s_up, s, x);
  s = (r_dn <= 0.0f) ? s_dn : s;
  s = (r_up > 0.0f) ? s_up : s;
  return s;
}

// Polynomials below are Horner chains of fused multiply-adds: one rounding
// per step, reproduced by C fmaf() in the oracle.
__device__ __forceinline__ float logf_fixed(float x) {
  const uint32_t b = __float_as_uint(x);
  int e = (int)((b >> 23) & 0xffu) - 126;
  float m = __uint_as_float((b & 0x007fffffu) | 0x3f000000u);
  if (m < 0.70710678118654752440f) {
    e -= 1;
    m = m + m;
    m = m - 1.0f;
  } else {
    m = m - 1.0f;
  }
  const float z = m * m;
  float y = 7.0376836292e-2f;
  y = __builtin_fmaf(y, m, -1.1514610310e-1f);
  y = __builtin_fmaf(y, m, 1.1676998740e-1f);
  y = __builtin_fmaf(y, m, -1.2420140846e-1f);
  y = __builtin_fmaf(y, m, 1.4249322787e-1f);
  y = __builtin_fmaf(y, m, -1.6668057665e-1f);
  y = __builtin_fmaf(y, m, 2.0000714765e-1f);
  y = __builtin_fmaf(y, m, -2.4999993993e-1f);
  y = __builtin_fmaf(y, m, 3.3333331174e-1f);
  y = y * m;
  y = y * z;
  const float fe = (float)e;
  y = __builtin_fmaf(-2.12194440e-4f, fe, y);
  y = __builtin_fmaf(-0.5f, z, y);
  float r = m + y;
  r = __builtin_fmaf(0.693359375f, fe, r);
  return r;
}

// sin/cos of a * 2 pi / 2^32
// (quadrant q = (a + 2^29) >> 30; the reduced angle is a's low 30 bits
// sign-extended -- one v_bfe_i32 -- and the quadrant's swap and sign bits
// are read off a + 2^29 and a + 3 2^29 directly: the same values as the
// quad arithmetic for every a, checked exhaustively; oracle/swarm_oracle.c
// or_sincos_turn keeps the quad form)
__device__ __forceinline__ void sincos_turn(uint32_t a, float* s_out, float* c_out) {
  const uint32_t b = a + 0x20000000u;
  const int32_t rem = ((int32_t)(a << 2)) >> 2;
  const float x = (float)rem * 1.46291807926715968e-09f;
  const float z = x * x;
  float sp = -1.9515295891e-4f;
  sp = __builtin_fmaf(sp, z, 8.3321608736e-3f);
  sp = __builtin_fmaf(sp, z, -1.6666654611e-1f);
  sp = sp * z;
  const float s = __builtin_fmaf(sp, x, x);
  float cp = 2.443315711809948e-5f;
  cp = __builtin_fmaf(cp, z, -1.388731625493765e-3f);
  cp = __builtin_fmaf(cp, z, 4.166664568298827e-2f);
  cp = cp * z;
  const float h = __builtin_fmaf(-0.5f, z, 1.0f);
  const float c = __builtin_fmaf(cp, z, h);
  // quadrant rotation: a swap and two sign flips on the float bits (exact)
  const bool swap = (b & 0x40000000u) != 0u;
  const float so0 = swap ? c : s;
  const float co0 = swap ? s : c;
  const float so = __uint_as_float(__float_as_uint(so0) ^ (b & 0x80000000u));
  const float co = __uint_as_float(__float_as_uint(co0) ^ ((a + 0x60000000u) & 0x80000000u));
  *s_out = so;
  *c_out = co;
}

__device__ __forceinline__ float asinf_small(float a) {
  const float z = a * a;
  float p = 4.2163199048e-2f;
  p = __builtin_fmaf(p, z, 2.4181311049e-2f);
  p = __builtin_fmaf(p, z, 4.5470025998e-2f);
  p = __builtin_fmaf(p, z, 7.4953002686e-2f);
  p = __builtin_fmaf(p, z, 1.6666752422e-1f);
  p = p * z;
  return __builtin_fmaf(p, a, a);
}

// acos by the three-range asin reduction, branch-free: the outer ranges'
// 0.5 (1 + x) for x < -0.5 is 0.5 (1 - |x|) bit for bit (a + (-b) = a - b),
// so one correctly rounded sqrt (t >= 2^-25 or 0: sqrt_pos holds) and one
// asin polynomial serve every lane (a divergent wave ran all three ranges).
__device__ __forceinline__ float acosf_fixed(float x) {
  const bool outer = x < -0.5f || x > 0.5f;
  const float t = 0.5f * (1.0f - fabsf(x));
  const float a = asinf_small(outer ? sqrt_pos(t) : x);
  const float two_a = 2.0f * a;
  if (!outer) return 1.57079632679489661923f - a;
  return x < 0.0f ? 3.14159265358979323846f - two_a : two_a;
}

// One standard normal from one 32-bit Philox word (round 6): a
// piecewise-linear inverse normal CDF over 2112 bins (64 per octave),
// tabulated by tools/make_normal_table.py into include/swarm_normal_table.h
// and shared with the oracle (oracle/swarm_oracle.c:or_normal_from_word):
// |z - Phi^-1(u)| <= 1.3e-5, tails to 6.4 sigma.  7 VALU instructions and
// one table load per normal, where Box-Muller took a fixed-polynomial log, a
// correctly rounded sqrt and a sin/cos polynomial per pair (~32 per normal;
// 41 % of the throughput run kernel's sub-step).
//   y = fp32(2 t + 1), t = r's low 31 bits  (in [1, 2^32]; one v_lshl_or_b32)
//   bin k from y's exponent and top 6 mantissa bits
//   m = y's mantissa as a float in [1, 2)   (one v_and_or_b32)
//   z = fma(D_k, m, A_k) = |Phi^-1((t + 0.5) / 2^32)|, linear within the bin
//   the sign is r's top bit                  (one v_bfi_b32)
__constant__ float kNtab[2 * SWARM_NTAB_BINS] = {SWARM_NTAB_DATA};

__device__ __forceinline__ const float2* ntab_global() {
  return reinterpret_cast<const float2*>(kNtab);
}

// tab: the table (kNtab, or a copy in the caller's LDS)
__device__ __forceinline__ float normal_from_word(uint32_t r, const float2* tab = ntab_global()) {
  const float y = __uint2float_rn((r << 1) | 1u);
  const uint32_t b = __float_as_uint(y);
  const uint32_t k = (b >> 17) - (127u << 6);
  const float m = __uint_as_float((b & 0x007FFFFFu) | 0x3F800000u);
  const float2 ad = tab[k];
  const float z = __builtin_fmaf(ad.y, m, ad.x);
  return __uint_as_float((__float_as_uint(z) & 0x7FFFFFFFu) | (r & 0x80000000u));
}

// Three standard normals from one Philox block (words x, y, z).
__device__ __forceinline__ void normals3(uint32_t k0, uint32_t k1, uint32_t id,
                                         uint64_t step, uint32_t tag, float g[3]) {
  u32x4 c;
  c.x = id;
  c.y = (uint32_t)step;
  c.z = (uint32_t)(step >> 32);
  c.w = tag;
  const u32x4 r = philox4x32_10(c, k0, k1);
  g[0] = normal_from_word(r.x);
  g[1] = normal_from_word(r.y);
  g[2] = normal_from_word(r.z);
}

// Translation/rotation normals of the Brownian step (tag 0 stream), all
// four Philox words used: sub-steps t = 4 g .. 4 g + 3 ("group" g) take the
// twelve normals n[0..11] of three Philox blocks with counter (id, g lo,
// g hi, kGroupTag + b), b = 0, 1, 2; block b gives n[4b..4b+3], one per
// word.  Sub-step t takes n[3j..3j+2], j = t & 3.  Per sub-step 0.75 Philox
// blocks.
constexpr uint32_t kGroupTag = 0x10u;

// the four normals of block b of group g
__device__ __forceinline__ void group_block(uint32_t k0, uint32_t k1, uint32_t id, uint64_t g,
                                            uint32_t b, float n[4],
                                            const float2* tab = ntab_global()) {
  u32x4 c;
  c.x = id;
  c.y = (uint32_t)g;
  c.z = (uint32_t)(g >> 32);
  c.w = kGroupTag + b;
  const u32x4 r = philox4x32_10(c, k0, k1);
  n[0] = normal_from_word(r.x, tab);
  n[1] = normal_from_word(r.y, tab);
  n[2] = normal_from_word(r.z, tab);
  n[3] = normal_from_word(r.w, tab);
}

// The normals of consecutive sub-steps: next(t) returns sub-step t's three,
// generating a block only when the group reaches it and carrying the rest
// (at most three floats).  fresh: t does not follow the previous call (the
// first sub-step of a window), so the blocks it shares are drawn again.
// tab: the normal table (global, or the throughput run kernel's LDS copy).
struct StepNoise {
  float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f;
  const float2* tab = ntab_global();
  __device__ __forceinline__ void next(uint32_t k0, uint32_t k1, uint32_t id, uint64_t t,
                                       bool fresh, float g[3]) {
    const uint32_t j = (uint32_t)t & 3u;
    const uint64_t grp = t >> 2;
    float n[4];
    if (j == 0u) {
      group_block(k0, k1, id, grp, 0u, n, tab);
      g[0] = n[0];
      g[1] = n[1];
      g[2] = n[2];
      c0 = n[3];
    } else if (j == 1u) {
      if (fresh) {
        group_block(k0, k1, id, grp, 0u, n, tab);
        c0 = n[3];
      }
      group_block(k0, k1, id, grp, 1u, n, tab);
      g[0] = c0;
      g[1] = n[0];
      g[2] = n[1];
      c0 = n[2];
      c1 = n[3];
    } else if (j == 2u) {
      if (fresh) {
        group_block(k0, k1, id, grp, 1u, n, tab);
        c0 = n[2];
        c1 = n[3];
      }
      group_block(k0, k1, id, grp, 2u, n, tab);
      g[0] = c0;
      g[1] = c1;
      g[2] = n[0];
      c0 = n[1];
      c1 = n[2];
      c2 = n[3];
    } else {
      if (fresh) {
        group_block(k0, k1, id, grp, 2u, n, tab);
        c0 = n[1];
        c1 = n[2];
        c2 = n[3];
      }
      g[0] = c0;
      g[1] = c1;
      g[2] = c2;
    }
  }
};

// Sub-step t's three normals from scratch (paths that are not a run of
// consecutive sub-steps of one particle in one thread).
__device__ __forceinline__ void step_normals(uint32_t k0, uint32_t k1, uint32_t id, uint64_t t,
                                             float g[3]) {
  StepNoise sn;
  sn.next(k0, k1, id, t, true, g);
}

// --------------------------------------------------- fixed-point helpers
__device__ __forceinline__ int32_t f2i32(float v) {
  v = fminf(fmaxf(v, -2147483520.0f), 2147483520.0f);
  return __float2int_rn(v);
}

// f2i32 for the 2-D translation (round 6): round to nearest even, then
// v_cvt_i32_f32's saturation to the int32 range (NaN -> 0) instead of a
// clamp before it -- one dependent operation fewer on the run kernels'
// chain (oracle/swarm_oracle.c:f2i32_sat; tests/test_gpu_devmath.py checks
// the edge values).  The conversion is written as the instruction itself:
// the compiler's fptosi leaves out-of-range values undefined.
__device__ __forceinline__ int32_t f2i32_sat(float v) {
  int32_t r;
  __asm__("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(__builtin_rintf(v)));
  return r;
}

__device__ __forceinline__ int64_t f2fix24(float v) {
  v = v * 16777216.0f;
  // |v| < 2^31 (force below 128): one int32 conversion, same value
  if (__builtin_expect(fabsf(v) < 2147483520.0f, 1)) return (int64_t)__float2int_rn(v);
  v = fminf(fmaxf(v, -4.611686018427387904e18f), 4.611686018427387904e18f);
  return __float2ll_rn(v);
}

// int64 -> fp32 round-to-nearest.  |a| < 2^53 (every realistic force sum):
// hi * 2^32 + lo is exact in fp64, so one fp64 -> fp32 rounding gives the
// correctly rounded value in four branch-free instructions; larger values
// (never in practice) take the generic conversion behind a wave-uniform
// branch.
__device__ __forceinline__ float i64_to_f32_wide(int64_t a) {
  const double d = fma((double)(int32_t)(a >> 32), 4294967296.0, (double)(uint32_t)a);
  float r = (float)d;
  const bool big = a >= (int64_t)9007199254740992LL || a <= -(int64_t)9007199254740992LL;
  if (__builtin_expect(__any(big), 0)) r = big ? (float)a : r;
  return r;
}

// every active lane's predicate (one v_cmp into an SGPR pair and a scalar
// compare with exec; __all goes through a VGPR select and a second compare)
__device__ __forceinline__ bool wave_all(bool p) {
  return __builtin_amdgcn_ballot_w64(p) == __builtin_amdgcn_read_exec();
}

// both predicates on every active lane: two compares straight into SGPR
// masks and one scalar AND
__device__ __forceinline__ bool wave_all2(bool p, bool q) {
  return (__builtin_amdgcn_ballot_w64(p) & __builtin_amdgcn_ballot_w64(q)) ==
         __builtin_amdgcn_read_exec();
}

__device__ __forceinline__ bool fits_i32(int64_t a) {
  return (int32_t)(a >> 32) == ((int32_t)a >> 31);
}

// int64 -> fp32 round-to-nearest; when every lane's value fits in int32
// (force sums below 128 in 2^-24 fixed point: the common case) one
// v_cvt_f32_i32 -- the same correctly rounded value -- instead of the fp64
// path.
__device__ __forceinline__ float i64_to_f32(int64_t a) {
  if (__builtin_expect(wave_all(fits_i32(a)), 1)) return (float)(int32_t)a;
  return i64_to_f32_wide(a);
}

// both components behind one wave-uniform test
__device__ __forceinline__ void i64x2_to_f32(int64_t ax, int64_t ay, float* fx, float* fy) {
  if (__builtin_expect(wave_all2(fits_i32(ax), fits_i32(ay)), 1)) {
    *fx = (float)(int32_t)ax;
    *fy = (float)(int32_t)ay;
  } else {
    *fx = i64_to_f32_wide(ax);
    *fy = i64_to_f32_wide(ay);
  }
}

// 1 / x correctly rounded, for x in [2^-96, 2^96] (every in-range squared
// pair distance: the fixed-point grid step is >= 2^-48): the hardware
// estimate v_rcp_f32 and ONE residual correction -- r = 1 - x y exactly
// (fma), then y + r y rounded once.  No v_div_scale / v_div_fixup range
// handling is needed on this range (no scaling: the exponents of 1 and x
// differ by < 96, neither is denormal).  Bit-identical to the IEEE division
// 1.0f / x for every float in the range on gfx950 (1.6e9 values, checked
// exhaustively on the GPU by tests/test_gpu_devmath.py::
// test_rcp_rn_exhaustive).  Round 6: three dependent operations where the
// compiler's division sequence (a Newton step, then two corrections) takes
// seven, on the run kernels' force chain, where a dependent VALU operation
// of a lone wave costs ~11 cycles (tools/chain_probe.hip).
__device__ __forceinline__ float rcp_rn(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float r = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(r, y, y);
}

// q + dq with the box crossing carried into the image counter: the high
// word of the 64-bit sum (q zero-extended, dq sign-extended) is -1, 0 or +1.
// The new q is one 32-bit add (the next sub-step's position exchange waits
// on it); the carry comes from comparing it with the old q, off that chain:
// dq >= 0 wrapped past 2^32 iff the sum is below q, dq < 0 wrapped below 0
// iff it is above q.
__device__ __forceinline__ void advance(uint32_t& q, int32_t& img, int32_t dq) {
  const uint32_t qn = q + (uint32_t)dq;
  img += dq >= 0 ? (qn < q ? 1 : 0) : (qn > q ? -1 : 0);
  q = qn;
}

// The same update as one 64-bit add of (img, q) and dq sign-extended:
// v_add_co_u32 + v_addc_co_u32 and the sign word, three VALU operations
// where advance takes seven.  For the throughput run kernel, bound by VALU
// issue (E = 64 run 176 -> 172 us); the latency-bound run keeps advance
// (E = 1 run 33.9 vs 34.9 us with this form, same box, round 6).
__device__ __forceinline__ void advance_adc(uint32_t& q, int32_t& img, int32_t dq) {
  const uint64_t v = (((uint64_t)(uint32_t)img << 32) | q) + (uint64_t)(int64_t)dq;
  q = (uint32_t)v;
  img = (int32_t)(uint32_t)(v >> 32);
}

}  // namespace swarm
