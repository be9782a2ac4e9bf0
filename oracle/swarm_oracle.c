/*
 * swarm_oracle.c -- CPU restatement of the SwarmRL rollout hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this code, and only as the checker
 * (or the timed CPU comparator).  The product (swarmrl_amd/) never links or
 * calls it.
 *
 * What it restates (reference = /root/reference, read as text):
 *   - overdamped Brownian dynamics with swim force and torque, as configured
 *     by swarmrl/engine/espresso.py:1179-1186 (thermostat), 376-389 and
 *     108-113 (per-particle friction 6 pi eta r / 8 pi eta r^3), 431-449
 *     (2-D: z fixed, rotation about lab z only), 1228-1235 (f_swim along the
 *     director, ext_torque);
 *   - the WCA pair force set up at espresso.py:814-819
 *     (sigma = (r_i + r_j) 2^(-1/6), cutoff = r_i + r_j, epsilon);
 *   - steepest-descent overlap removal, espresso.py:1161-1168
 *     (f_max = 0, gamma, max_displacement, n steps);
 *   - SubdividedVisionCones, swarmrl/observables/subdivided_vision_cones.py:
 *     105-203 with calc_signed_angle_between_directors,
 *     swarmrl/utils/utils.py:297-332;
 *   - the distance part of ConcentrationField
 *     (swarmrl/observables/concentration_field.py:84-108) and GradientSensing
 *     (swarmrl/tasks/searching/gradient_sensing.py:92-126).
 *
 * The BD/WCA arithmetic of ESPResSo itself is third-party code that is not
 * in /root/reference (pinned only as ESPResSo dc87ede3..., see
 * .github/workflows/espresso.yml:24).  Its documented algorithm is restated
 * here; its Philox noise stream is unknowable, so the noise below is this
 * project's own counter-based stream (Philox4x32-10 keyed by seed/env,
 * counter = particle id / step / tag) -- noisy trajectories are pinned
 * statistically, deterministic (kT = 0) ones by the reference's tests.
 *
 * Number formats (shared spec with the GPU path):
 *   position  = uint32 fraction of the box + int32 image counter,
 *   angle     = uint32 turn fraction,
 *   WCA force = sum of per-pair fp32 forces in int64 fixed point (2^-24),
 *   vision    = sum of per-colloid fp32 amplitudes in int64 fixed point
 *               (2^-32),
 * so every sum is exact and independent of neighbour order.  Build with
 * -ffp-contract=off: every fp32 operation below is rounded separately.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/swarmrl_amd.h"
#include "../include/swarm_normal_table.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* Threads of the per-particle / per-agent loops (OpenMP; 1 = the scalar
 * restatement).  Every parallel loop writes only its own particle's or
 * agent's outputs and sums in int64, so results do not depend on it. */
void or_set_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n > 0 ? n : 1);
#else
  (void)n;
#endif
}

int or_get_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11 "Parallel random   */
/* numbers: as easy as 1, 2, 3").                                      */
/* ------------------------------------------------------------------ */
void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                      uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* ------------------------------------------------------------------ */
/* Elementary functions with a fixed operation sequence (cephes        */
/* single-precision polynomials) so CPU and GPU round identically.      */
/* ------------------------------------------------------------------ */
static float f_from_bits(uint32_t b) {
  float f;
  memcpy(&f, &b, 4);
  return f;
}
static uint32_t bits_from_f(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}

/* natural log for normal x > 0 */
float or_logf(float x) {
  uint32_t b = bits_from_f(x);
  int e = (int)((b >> 23) & 0xffu) - 126;
  float m = f_from_bits((b & 0x007fffffu) | 0x3f000000u); /* [0.5, 1) */
  if (m < 0.70710678118654752440f) {
    e -= 1;
    m = m + m;
    m = m - 1.0f;
  } else {
    m = m - 1.0f;
  }
  float z = m * m;
  float y = 7.0376836292e-2f;
  y = fmaf(y, m, -1.1514610310e-1f);
  y = fmaf(y, m, 1.1676998740e-1f);
  y = fmaf(y, m, -1.2420140846e-1f);
  y = fmaf(y, m, 1.4249322787e-1f);
  y = fmaf(y, m, -1.6668057665e-1f);
  y = fmaf(y, m, 2.0000714765e-1f);
  y = fmaf(y, m, -2.4999993993e-1f);
  y = fmaf(y, m, 3.3333331174e-1f);
  y = y * m;
  y = y * z;
  float fe = (float)e;
  y = fmaf(-2.12194440e-4f, fe, y);
  y = fmaf(-0.5f, z, y);
  float r = m + y;
  r = fmaf(0.693359375f, fe, r);
  return r;
}

/* sin and cos of the angle a * 2 pi / 2^32 */
void or_sincos_turn(uint32_t a, float *s_out, float *c_out) {
  uint32_t b = a + 0x20000000u; /* shift by 1/8 turn */
  uint32_t quad = b >> 30;
  int32_t rem = (int32_t)(b & 0x3FFFFFFFu) - 0x20000000; /* [-2^29, 2^29) */
  float x = (float)rem * 1.46291807926715968e-09f;      /* 2 pi / 2^32 */
  float z = x * x;
  float sp = -1.9515295891e-4f;
  sp = fmaf(sp, z, 8.3321608736e-3f);
  sp = fmaf(sp, z, -1.6666654611e-1f);
  sp = sp * z;
  float s = fmaf(sp, x, x);
  float cp = 2.443315711809948e-5f;
  cp = fmaf(cp, z, -1.388731625493765e-3f);
  cp = fmaf(cp, z, 4.166664568298827e-2f);
  cp = cp * z;
  float h = fmaf(-0.5f, z, 1.0f);
  float c = fmaf(cp, z, h);
  float so, co;
  switch (quad) {
  case 0:
    so = s;
    co = c;
    break;
  case 1:
    so = c;
    co = -s;
    break;
  case 2:
    so = -s;
    co = -c;
    break;
  default:
    so = -c;
    co = s;
    break;
  }
  *s_out = so;
  *c_out = co;
}

static float asinf_small(float a) { /* |a| <= 0.5 */
  float z = a * a;
  float p = 4.2163199048e-2f;
  p = fmaf(p, z, 2.4181311049e-2f);
  p = fmaf(p, z, 4.5470025998e-2f);
  p = fmaf(p, z, 7.4953002686e-2f);
  p = fmaf(p, z, 1.6666752422e-1f);
  p = p * z;
  return fmaf(p, a, a);
}

float or_acosf(float x) {
  if (x < -0.5f) {
    float t = 1.0f + x;
    t = 0.5f * t;
    return 3.14159265358979323846f - 2.0f * asinf_small(sqrtf(t));
  }
  if (x > 0.5f) {
    float t = 1.0f - x;
    t = 0.5f * t;
    return 2.0f * asinf_small(sqrtf(t));
  }
  return 1.57079632679489661923f - asinf_small(x);
}

/* calc_signed_angle_between_directors, utils.py:297-332, in fp32 */
float or_signed_angle(const float my[3], const float other[3]) {
  float nm = sqrtf(my[0] * my[0] + my[1] * my[1] + my[2] * my[2]);
  float m0 = my[0] / nm, m1 = my[1] / nm, m2 = my[2] / nm;
  float no = sqrtf(other[0] * other[0] + other[1] * other[1] +
                   other[2] * other[2]);
  float o0 = other[0] / no, o1 = other[1] / no, o2 = other[2] / no;
  float dot = o0 * m0 + o1 * m1 + o2 * m2;
  dot = fminf(fmaxf(dot, -1.0f), 1.0f);
  float ang = or_acosf(dot);
  float orth = o0 * (-m1) + o1 * m0 + o2 * m2;
  return orth >= 0.0f ? ang : -ang;
}

/* One standard normal from one 32-bit Philox word: the engine's
 * piecewise-linear inverse normal CDF (swarm_device.cuh:normal_from_word,
 * table include/swarm_normal_table.h from tools/make_normal_table.py):
 * y = fp32(2 t + 1) for t = r's low 31 bits, bin k from y's exponent and
 * top 6 mantissa bits, m = y's mantissa in [1, 2), |z| = fma(D_k, m, A_k),
 * the sign r's top bit.  The reference's thermostat draws ESPResSo's own
 * Gaussian stream (espresso.py:1179-1186), unknowable here: noisy
 * trajectories are pinned statistically. */
static const float ntab[2 * SWARM_NTAB_BINS] = {SWARM_NTAB_DATA};

float or_normal_from_word(uint32_t r) {
  float y = (float)((r << 1) | 1u);
  uint32_t b = bits_from_f(y);
  uint32_t k = (b >> 17) - (127u << 6);
  float m = f_from_bits((b & 0x007FFFFFu) | 0x3F800000u);
  float z = fmaf(ntab[2 * k + 1], m, ntab[2 * k]);
  return f_from_bits((bits_from_f(z) & 0x7FFFFFFFu) | (r & 0x80000000u));
}

/* Three standard normals for (seed, env, particle id, step, tag): Philox
 * words 0, 1, 2. */
void or_normals3(uint64_t seed, uint32_t env, uint32_t id, uint64_t step,
                 uint32_t tag, float out[3]) {
  uint32_t ctr[4] = {id, (uint32_t)step, (uint32_t)(step >> 32), tag};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ env};
  uint32_t r[4];
  or_philox4x32_10(ctr, key, r);
  out[0] = or_normal_from_word(r[0]);
  out[1] = or_normal_from_word(r[1]);
  out[2] = or_normal_from_word(r[2]);
}

/* Translation/rotation normals of sub-step t (the tag-0 stream; the
 * engine's swarm_device.cuh StepNoise): sub-steps 4g..4g+3 take the twelve
 * normals of three Philox blocks with counter (id, g lo, g hi, 0x10 + b),
 * block b giving one normal per word; sub-step t takes normals 3j..3j+2 of
 * its group, j = t & 3. */
static void group_block(uint64_t seed, uint32_t env, uint32_t id, uint64_t g,
                        uint32_t b, float n[4]) {
  uint32_t ctr[4] = {id, (uint32_t)g, (uint32_t)(g >> 32), 0x10u + b};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ env};
  uint32_t r[4];
  or_philox4x32_10(ctr, key, r);
  for (int w = 0; w < 4; ++w)
    n[w] = or_normal_from_word(r[w]);
}

void or_step_normals(uint64_t seed, uint32_t env, uint32_t id, uint64_t t,
                     float out[3]) {
  float n[12];
  uint64_t g = t >> 2;
  int j = (int)(t & 3u);
  /* the blocks holding normals 3j .. 3j+2 */
  int b_lo = (3 * j) / 4, b_hi = (3 * j + 2) / 4;
  for (int b = b_lo; b <= b_hi; ++b) group_block(seed, env, id, g, (uint32_t)b, n + 4 * b);
  out[0] = n[3 * j];
  out[1] = n[3 * j + 1];
  out[2] = n[3 * j + 2];
}

/* ------------------------------------------------------------------ */
/* Derived fp32 constants (same derivation as swarm_engine.hip).       */
/* ------------------------------------------------------------------ */
typedef struct {
  float sx[3], inv_sx[3];
  float mob_dt[SWARM_MAX_SPECIES], sig_t[SWARM_MAX_SPECIES];
  float rot_dt[SWARM_MAX_SPECIES], sig_r[SWARM_MAX_SPECIES];
  float inv_gt[SWARM_MAX_SPECIES], inv_gr[SWARM_MAX_SPECIES];
  float sig_v[SWARM_MAX_SPECIES], sig_w[SWARM_MAX_SPECIES];
  float cut2[SWARM_MAX_SPECIES][SWARM_MAX_SPECIES];
  float sig6[SWARM_MAX_SPECIES][SWARM_MAX_SPECIES];
  float eps24;
  double rc_max;
  /* walls (espresso.py:667-800), see swarm_wall_t */
  int n_walls;
  int wkind[SWARM_MAX_WALLS];
  float wp[SWARM_MAX_WALLS][8]; /* plane: n0 n1 n2 off; slab: o0 o1 a0 a1 b0 b1 la lb */
  float wcut2[SWARM_MAX_SPECIES], wsig6[SWARM_MAX_SPECIES];
} derived_t;

#define TWO32 4294967296.0
#define TWO_PI 6.283185307179586476925
#define ANG_INV_SCALE 683565275.57643158f /* 2^32 / (2 pi) */

static void derive(const swarm_params_t *p, derived_t *d) {
  memset(d, 0, sizeof(*d));
  for (int a = 0; a < 3; ++a) {
    double L = p->box[a];
    d->sx[a] = (float)(L / TWO32);
    d->inv_sx[a] = (float)(TWO32 / L);
  }
  double kT = p->kT, dt = p->time_step;
  for (int s = 0; s < p->n_species; ++s) {
    double gt = p->gamma_t[s], gr = p->gamma_r[s];
    d->mob_dt[s] = (float)(dt / gt);
    d->rot_dt[s] = (float)(dt / gr);
    d->sig_t[s] = (float)sqrt(2.0 * kT * dt / gt);
    d->sig_r[s] = (float)sqrt(2.0 * kT * dt / gr);
    d->inv_gt[s] = (float)(1.0 / gt);
    d->inv_gr[s] = (float)(1.0 / gr);
    d->sig_v[s] = p->mass[s] > 0.0 ? (float)sqrt(kT / p->mass[s]) : 0.0f;
    d->sig_w[s] = p->rinertia[s] > 0.0 ? (float)sqrt(kT / p->rinertia[s]) : 0.0f;
  }
  d->rc_max = 0.0;
  for (int s = 0; s < p->n_species; ++s)
    for (int t = 0; t < p->n_species; ++t) {
      double rc = p->radius[s] + p->radius[t];
      double rc2 = rc * rc;
      d->cut2[s][t] = (float)rc2;
      d->sig6[s][t] = (float)(rc2 * rc2 * rc2 * 0.5);
      if (rc > d->rc_max)
        d->rc_max = rc;
    }
  d->eps24 = (float)(24.0 * p->wca_epsilon);
  for (int s = 0; s < p->n_species; ++s) {
    double rc2 = p->radius[s] * p->radius[s];
    d->wcut2[s] = (float)rc2;
    d->wsig6[s] = (float)(rc2 * rc2 * rc2 * 0.5);
  }
}

/* wall table in fp32 (same derivation as the engine's set_walls) */
static void derive_walls(derived_t *d, const swarm_wall_t *w, int n_walls) {
  d->n_walls = n_walls;
  for (int k = 0; k < n_walls; ++k) {
    d->wkind[k] = w[k].kind;
    float *o = d->wp[k];
    if (w[k].kind == 0) {
      for (int a = 0; a < 3; ++a)
        o[a] = (float)w[k].normal[a];
      o[3] = (float)w[k].offset;
    } else {
      double la = sqrt(w[k].a[0] * w[k].a[0] + w[k].a[1] * w[k].a[1]);
      double lb = sqrt(w[k].b[0] * w[k].b[0] + w[k].b[1] * w[k].b[1]);
      o[0] = (float)w[k].corner[0];
      o[1] = (float)w[k].corner[1];
      o[2] = (float)(w[k].a[0] / la);
      o[3] = (float)(w[k].a[1] / la);
      o[4] = (float)(w[k].b[0] / lb);
      o[5] = (float)(w[k].b[1] / lb);
      o[6] = (float)la;
      o[7] = (float)lb;
    }
  }
}

static int32_t f2i32(float v) {
  v = fminf(fmaxf(v, -2147483520.0f), 2147483520.0f);
  return (int32_t)lrintf(v);
}
static int64_t f2fix24(float v) {
  v = v * 16777216.0f;
  v = fminf(fmaxf(v, -4.611686018427387904e18f), 4.611686018427387904e18f);
  return (int64_t)llrintf(v);
}

/* displacement j - i along axis a, fp32 sim units */
static float pair_disp(const swarm_params_t *p, const derived_t *d,
                       const uint32_t *q, const int32_t *img, int n, int a,
                       int i, int j) {
  if (p->periodic) {
    int32_t dq = (int32_t)(q[a * n + j] - q[a * n + i]);
    return (float)dq * d->sx[a];
  }
  int64_t dq = ((int64_t)(img[a * n + j] - img[a * n + i]) * (int64_t)4294967296LL) +
               ((int64_t)q[a * n + j] - (int64_t)q[a * n + i]);
  return (float)dq * d->sx[a];
}

/* a 2^24-scaled force value to int64 fixed point (round to nearest even,
 * clamped to +-2^62) */
static int64_t fix_scaled(float v) {
  v = fminf(fmaxf(v, -4.611686018427387904e18f), 4.611686018427387904e18f);
  return (int64_t)llrintf(v);
}

/* WCA force on i from j accumulated in 2^-24 fixed point (2-D).  The
 * engine's round-6 operation sequence (swarm_integrator.cuh:pair_vals, chosen
 * for a short dependency chain on the GPU), the WCA law of
 * espresso.py:802-832 (pinned by refsem.wca_force in fp64):
 *   r2 = fma(rx, rx, ry ry); ir2 = 1 / r2
 *   s6 = (ir2 ir2)(sig6 ir2); t = fma(s6, 2, -1)
 *   v  = ((eps24 s6) t)(ir2 (-rx 2^24)) */
static void wca_pair(const derived_t *d, int si, int sj, float rx, float ry,
                     int64_t *ax, int64_t *ay) {
  float r2 = fmaf(rx, rx, ry * ry);
  if (r2 < d->cut2[si][sj] && r2 > 0.0f) {
    float ir2 = 1.0f / r2;
    float s6 = (ir2 * ir2) * (d->sig6[si][sj] * ir2);
    float t = fmaf(s6, 2.0f, -1.0f);
    float fr = (d->eps24 * s6) * t;
    *ax += fix_scaled(fr * (ir2 * (rx * -16777216.0f)));
    *ay += fix_scaled(fr * (ir2 * (ry * -16777216.0f)));
  }
}

/* round to nearest even, then saturate to the int32 range (NaN -> 0): the
 * GPU's v_rndne_f32 + v_cvt_i32_f32 (swarm_integrator.cuh:f2i32_sat) */
static int32_t f2i32_sat(float v) {
  float r = rintf(v);
  if (r != r)
    return 0;
  if (r >= 2147483648.0f)
    return INT32_MAX;
  if (r <= -2147483648.0f)
    return INT32_MIN;
  return (int32_t)r;
}

/* WCA force of every wall on a particle of species sp at the folded
 * position (x, y, z), added to acc[0..dims) in 2^-24 fixed point
 * (ShapeBasedConstraint + WCA, espresso.py:667-800, 814-819). */
static void wall_forces(const derived_t *d, int sp, float x, float y, float z, int dims,
                        int64_t *ax, int64_t *ay, int64_t *az, uint64_t *viol) {
  for (int k = 0; k < d->n_walls; ++k) {
    const float *w = d->wp[k];
    float vx, vy, vz, r2;
    if (d->wkind[k] == 0) {
      float dist = w[0] * x + w[1] * y;
      dist = dist + w[2] * z;
      dist = dist - w[3];
      if (!(dist > 0.0f)) {
        ++*viol;
        continue;
      }
      vx = w[0] * dist;
      vy = w[1] * dist;
      vz = w[2] * dist;
      r2 = dist * dist;
    } else {
      float px = x - w[0], py = y - w[1];
      float u = px * w[2] + py * w[3];
      float t = px * w[4] + py * w[5];
      float du = u - fminf(fmaxf(u, 0.0f), w[6]);
      float dt = t - fminf(fmaxf(t, 0.0f), w[7]);
      if (du == 0.0f && dt == 0.0f) {
        ++*viol;
        continue;
      }
      vx = du * w[2] + dt * w[4];
      vy = du * w[3] + dt * w[5];
      vz = 0.0f;
      r2 = vx * vx + vy * vy;
    }
    if (r2 < d->wcut2[sp]) {
      float ir2 = 1.0f / r2;
      float ir6 = ir2 * ir2;
      ir6 = ir6 * ir2;
      float s6 = d->wsig6[sp] * ir6;
      float t = 2.0f * s6;
      t = t - 1.0f;
      float fr = d->eps24 * s6;
      fr = fr * t;
      fr = fr * ir2;
      *ax += f2fix24(fr * vx);
      *ay += f2fix24(fr * vy);
      if (dims == 3)
        *az += f2fix24(fr * vz);
    }
  }
}

/* cell index of particle i (2-D), grid ncx x ncy (powers of two) */
static int cell_of(const swarm_params_t *p, const uint32_t *q, const int32_t *img,
                   int n, int i, int lx, int ly) {
  int c[2];
  int lg[2] = {lx, ly};
  for (int a = 0; a < 2; ++a) {
    int nc = 1 << lg[a];
    int v = lg[a] == 0 ? 0 : (int)(q[a * n + i] >> (32 - lg[a]));
    if (!p->periodic) {
      if (img[a * n + i] < 0)
        v = 0;
      else if (img[a * n + i] > 0)
        v = nc - 1;
    }
    c[a] = v;
  }
  return c[1] * (1 << lx) + c[0];
}

static int ilog2_floor(double v) {
  int l = 0;
  while ((double)(1 << (l + 1)) <= v && l < 20)
    ++l;
  return l;
}

/* cell grid: power-of-two cells per axis, cell side >= rc_max and at most
 * max(n, 64) cells in total (same rule as the GPU path). */
void or_cell_grid(const swarm_params_t *p, int n, double cutoff, int *lx,
                  int *ly) {
  int l[2];
  for (int a = 0; a < 2; ++a) {
    double m = cutoff > 0.0 ? p->box[a] / cutoff : 1024.0;
    l[a] = m >= 1.0 ? ilog2_floor(m) : 0;
    if (l[a] > 15)
      l[a] = 15;
  }
  int cap = n > 64 ? n : 64;
  while ((1 << (l[0] + l[1])) > cap) {
    if (l[0] >= l[1] && l[0] > 0)
      l[0]--;
    else if (l[1] > 0)
      l[1]--;
    else
      break;
  }
  *lx = l[0];
  *ly = l[1];
}

/* Neighbour candidate iteration helper: builds a cell list (counting sort). */
typedef struct {
  int lx, ly, ncell;
  int *start; /* ncell + 1 */
  int *list;  /* n */
  int *cell;  /* n */
} celllist_t;

static void cl_build(celllist_t *cl, const swarm_params_t *p, const uint32_t *q,
                     const int32_t *img, int n) {
  memset(cl->start, 0, sizeof(int) * (size_t)(cl->ncell + 1));
  for (int i = 0; i < n; ++i) {
    cl->cell[i] = cell_of(p, q, img, n, i, cl->lx, cl->ly);
    cl->start[cl->cell[i] + 1]++;
  }
  for (int c = 0; c < cl->ncell; ++c)
    cl->start[c + 1] += cl->start[c];
  int *fill = (int *)malloc(sizeof(int) * (size_t)cl->ncell);
  memcpy(fill, cl->start, sizeof(int) * (size_t)cl->ncell);
  for (int i = 0; i < n; ++i)
    cl->list[fill[cl->cell[i]]++] = i;
  free(fill);
}

/* total WCA forces (int64 fixed point) for all particles */
static void wca_forces(const swarm_params_t *p, const derived_t *d, int n,
                       const uint32_t *q, const int32_t *img,
                       const uint8_t *species, int64_t *acc, celllist_t *cl) {
  memset(acc, 0, sizeof(int64_t) * 2 * (size_t)n);
  if (!cl) { /* brute force */
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        if (j == i)
          continue;
        float rx = pair_disp(p, d, q, img, n, 0, i, j);
        float ry = pair_disp(p, d, q, img, n, 1, i, j);
        wca_pair(d, species[i], species[j], rx, ry, &acc[i], &acc[n + i]);
      }
    return;
  }
  cl_build(cl, p, q, img, n);
  int ncx = 1 << cl->lx, ncy = 1 << cl->ly;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    int c = cl->cell[i];
    int cx = c % ncx, cy = c / ncx;
    int lox = ncx >= 3 ? -1 : 0, hix = ncx >= 3 ? 1 : ncx - 1;
    int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
    for (int oy = loy; oy <= hiy; ++oy)
      for (int ox = lox; ox <= hix; ++ox) {
        int x = cx + ox, y = cy + oy;
        if (p->periodic) {
          x = (x + ncx) % ncx;
          y = (y + ncy) % ncy;
        } else if (x < 0 || x >= ncx || y < 0 || y >= ncy)
          continue;
        int cc = y * ncx + x;
        for (int k = cl->start[cc]; k < cl->start[cc + 1]; ++k) {
          int j = cl->list[k];
          if (j == i)
            continue;
          float rx = pair_disp(p, d, q, img, n, 0, i, j);
          float ry = pair_disp(p, d, q, img, n, 1, i, j);
          wca_pair(d, species[i], species[j], rx, ry, &acc[i], &acc[n + i]);
        }
      }
  }
}

static void advance(uint32_t *q, int32_t *img, int32_t dq) {
  uint32_t old = *q;
  uint32_t nq = old + (uint32_t)dq;
  if (dq > 0 && nq < old)
    *img += 1;
  else if (dq < 0 && nq > old)
    *img -= 1;
  *q = nq;
}

static int cl_alloc(celllist_t *cl, const swarm_params_t *p, const derived_t *d,
                    int n) {
  or_cell_grid(p, n, d->rc_max, &cl->lx, &cl->ly);
  cl->ncell = 1 << (cl->lx + cl->ly);
  cl->start = (int *)malloc(sizeof(int) * (size_t)(cl->ncell + 1));
  cl->list = (int *)malloc(sizeof(int) * (size_t)n);
  cl->cell = (int *)malloc(sizeof(int) * (size_t)n);
  return cl->start && cl->list && cl->cell;
}
static void cl_free(celllist_t *cl) {
  free(cl->start);
  free(cl->list);
  free(cl->cell);
}

/*
 * n_steps Brownian-dynamics sub-steps of ONE env (2-D).
 * q/img: [3][n], ang: [n]; f_swim, torque_z: [n]; f_ext: [3][n] or NULL.
 * vel/omega (NULL allowed) receive the BD velocity of the last sub-step.
 * step0: global step index of the first sub-step (noise counter).
 * use_cells: 0 = O(n^2) pair search, 1 = cell list (same result).
 * f_swim0 / torque0 / ang0 (NULL: the current ones): what sub-step 0 uses --
 * ESPResSo's run(k, reuse_forces=True) (espresso.py:1304-1306) propagates
 * with the forces of the previous run's last force calculation, i.e. that
 * run's swim force and torque along the orientation it ended with.
 */
int or_bd_run_walls(const swarm_params_t *p, int n, uint32_t *q, int32_t *img,
                    uint32_t *ang, const uint8_t *species, const float *f_swim,
                    const float *torque_z, const float *f_ext, uint64_t step0,
                    int n_steps, uint32_t env, float *vel, float *omega,
                    int use_cells, const swarm_wall_t *walls, int n_walls,
                    uint64_t *violations, const float *f_swim0, const float *torque0,
                    const uint32_t *ang0) {
  if (p->n_dims != 2)
    return SWARM_EINVAL;
  derived_t d;
  derive(p, &d);
  derive_walls(&d, walls, n_walls);
  uint64_t viol = 0;
  int64_t *acc = (int64_t *)malloc(sizeof(int64_t) * 2 * (size_t)(n > 0 ? n : 1));
  celllist_t cl;
  int have_cl = use_cells && cl_alloc(&cl, p, &d, n);
  const int noisy = p->kT > 0.0;
  for (int s = 0; s < n_steps; ++s) {
    uint64_t step = step0 + (uint64_t)s;
    wca_forces(p, &d, n, q, img, species, acc, have_cl ? &cl : NULL);
#pragma omp parallel for schedule(static) reduction(+ : viol)
    for (int i = 0; i < n; ++i) {
      int sp = species[i];
      float sn, cs;
      if (d.n_walls) {
        uint64_t vi = 0;
        wall_forces(&d, sp, (float)q[i] * d.sx[0], (float)q[n + i] * d.sx[1], 0.0f, 2,
                    &acc[i], &acc[n + i], NULL, &vi);
        viol += vi;
      }
      const int first = s == 0;
      const float fs = first && f_swim0 ? f_swim0[i] : f_swim[i];
      const float tz = first && torque0 ? torque0[i] : torque_z[i];
      or_sincos_turn(first && ang0 ? ang0[i] : ang[i], &sn, &cs);
      /* translation in fixed-point units, the engine's round-6 sequence
       * (swarm_integrator.cuh:bd_dq): f = fma(F, 2^-24, f_ext + f_swim d),
       * dq = f2i32_sat(fma(f, mob_dt / sx, (sig_t / sx) g)) */
      float g[3] = {0.0f, 0.0f, 0.0f};
      float dth = tz * d.rot_dt[sp];
      if (noisy) {
        or_step_normals(p->seed, env, (uint32_t)i, step, g);
        dth = dth + d.sig_r[sp] * g[2];
      }
      const float c1x = (f_ext ? f_ext[i] : 0.0f) + fs * cs;
      const float c1y = (f_ext ? f_ext[n + i] : 0.0f) + fs * sn;
      float fx = fmaf((float)acc[i], 5.9604644775390625e-08f, c1x);
      float fy = fmaf((float)acc[n + i], 5.9604644775390625e-08f, c1y);
      const float mobx = d.mob_dt[sp] * d.inv_sx[0], moby = d.mob_dt[sp] * d.inv_sx[1];
      const float sigx = noisy ? d.sig_t[sp] * d.inv_sx[0] : 0.0f;
      const float sigy = noisy ? d.sig_t[sp] * d.inv_sx[1] : 0.0f;
      advance(&q[i], &img[i], f2i32_sat(fmaf(fx, mobx, sigx * g[0])));
      advance(&q[n + i], &img[n + i], f2i32_sat(fmaf(fy, moby, sigy * g[1])));
      /* the rotation's increment saturates like the translation's
       * (swarm_integrator.cuh:bd_step, f2i32_sat) */
      ang[i] = ang[i] + (uint32_t)f2i32_sat(dth * ANG_INV_SCALE);
      if (s == n_steps - 1) {
        float vx = fx * d.inv_gt[sp], vy = fy * d.inv_gt[sp];
        float w = tz * d.inv_gr[sp];
        if (noisy) {
          float g[3];
          or_normals3(p->seed, env, (uint32_t)i, step, 1u, g);
          vx = vx + d.sig_v[sp] * g[0];
          vy = vy + d.sig_v[sp] * g[1];
          w = w + d.sig_w[sp] * g[2];
        }
        if (vel) {
          vel[i] = vx;
          vel[n + i] = vy;
          vel[2 * n + i] = 0.0f;
        }
        if (omega)
          omega[i] = w;
      }
    }
  }
  if (have_cl)
    cl_free(&cl);
  free(acc);
  if (violations)
    *violations += viol;
  return SWARM_OK;
}

int or_bd_run(const swarm_params_t *p, int n, uint32_t *q, int32_t *img,
              uint32_t *ang, const uint8_t *species, const float *f_swim,
              const float *torque_z, const float *f_ext, uint64_t step0,
              int n_steps, uint32_t env, float *vel, float *omega,
              int use_cells) {
  return or_bd_run_walls(p, n, q, img, ang, species, f_swim, torque_z, f_ext, step0,
                         n_steps, env, vel, omega, use_cells, NULL, 0, NULL, NULL, NULL, NULL);
}

/*
 * Steepest descent (espresso.py:1161-1168): per step F = WCA + ext + swim,
 * dp = clamp(gamma F, -max_disp, max_disp) per free coordinate; stops early
 * once every force is exactly zero (later steps would not move anything).
 * Returns the number of steps executed.
 */
int or_sd_run_walls(const swarm_params_t *p, int n, uint32_t *q, int32_t *img,
                    uint32_t *ang, const uint8_t *species, const float *f_swim,
                    const float *torque_z, const float *f_ext, int n_steps,
                    double gamma, double max_disp, int use_cells,
                    const swarm_wall_t *walls, int n_walls) {
  derived_t d;
  derive(p, &d);
  derive_walls(&d, walls, n_walls);
  uint64_t viol = 0;
  const float g = (float)gamma, md = (float)max_disp;
  int64_t *acc = (int64_t *)malloc(sizeof(int64_t) * 2 * (size_t)(n > 0 ? n : 1));
  celllist_t cl;
  int have_cl = use_cells && cl_alloc(&cl, p, &d, n);
  int s;
  for (s = 0; s < n_steps; ++s) {
    wca_forces(p, &d, n, q, img, species, acc, have_cl ? &cl : NULL);
    int any = 0;
    for (int i = 0; i < n; ++i) {
      float sn, cs;
      if (d.n_walls)
        wall_forces(&d, species[i], (float)q[i] * d.sx[0], (float)q[n + i] * d.sx[1], 0.0f,
                    2, &acc[i], &acc[n + i], NULL, &viol);
      or_sincos_turn(ang[i], &sn, &cs);
      float fx = (float)acc[i] * 5.9604644775390625e-08f;
      float fy = (float)acc[n + i] * 5.9604644775390625e-08f;
      if (f_ext) {
        fx = fx + f_ext[i];
        fy = fy + f_ext[n + i];
      }
      fx = fx + f_swim[i] * cs;
      fy = fy + f_swim[i] * sn;
      float tz = torque_z[i];
      if (fx != 0.0f || fy != 0.0f || tz != 0.0f)
        any = 1;
      float px = fminf(fmaxf(g * fx, -md), md);
      float py = fminf(fmaxf(g * fy, -md), md);
      float pa = fminf(fmaxf(g * tz, -md), md);
      advance(&q[i], &img[i], f2i32(px * d.inv_sx[0]));
      advance(&q[n + i], &img[n + i], f2i32(py * d.inv_sx[1]));
      ang[i] = ang[i] + (uint32_t)f2i32(pa * ANG_INV_SCALE);
    }
    if (!any)
      break;
  }
  if (have_cl)
    cl_free(&cl);
  free(acc);
  return s;
}

int or_sd_run(const swarm_params_t *p, int n, uint32_t *q, int32_t *img,
              uint32_t *ang, const uint8_t *species, const float *f_swim,
              const float *torque_z, const float *f_ext, int n_steps,
              double gamma, double max_disp, int use_cells) {
  return or_sd_run_walls(p, n, q, img, ang, species, f_swim, torque_z, f_ext, n_steps, gamma,
                         max_disp, use_cells, NULL, 0);
}

/* ------------------------------------------------------------------ */
/* 3-D (espresso.py:415-426: rotation about all three axes, no fixed    */
/* coordinate).  Pair search is O(n^2): sums are exact, so the GPU's     */
/* cell lists give the same bits.                                        */
/* ------------------------------------------------------------------ */
static void wca_pair3(const derived_t *d, int si, int sj, float rx, float ry, float rz,
                      int64_t *ax, int64_t *ay, int64_t *az) {
  float r2 = rx * rx + ry * ry;
  r2 = r2 + rz * rz;
  if (r2 < d->cut2[si][sj] && r2 > 0.0f) {
    float ir2 = 1.0f / r2;
    float ir6 = ir2 * ir2;
    ir6 = ir6 * ir2;
    float s6 = d->sig6[si][sj] * ir6;
    float t = 2.0f * s6;
    t = t - 1.0f;
    float fr = d->eps24 * s6;
    fr = fr * t;
    fr = fr * ir2;
    *ax += f2fix24(-fr * rx);
    *ay += f2fix24(-fr * ry);
    *az += f2fix24(-fr * rz);
  }
}

static void wca_forces3(const swarm_params_t *p, const derived_t *d, int n, const uint32_t *q,
                        const int32_t *img, const uint8_t *species, int64_t *acc) {
  memset(acc, 0, sizeof(int64_t) * 3 * (size_t)n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (j == i)
        continue;
      float rx = pair_disp(p, d, q, img, n, 0, i, j);
      float ry = pair_disp(p, d, q, img, n, 1, i, j);
      float rz = pair_disp(p, d, q, img, n, 2, i, j);
      wca_pair3(d, species[i], species[j], rx, ry, rz, &acc[i], &acc[n + i], &acc[2 * n + i]);
    }
}

/* Rotate the unit director v by the rotation vector (px, py, pz) (Rodrigues,
 * angle = |p|) and renormalise. */
void or_rotate_director(float v[3], float px, float py, float pz) {
  float th2 = px * px + py * py;
  th2 = th2 + pz * pz;
  if (!(th2 > 0.0f))
    return;
  float th = sqrtf(th2);
  float kx = px / th, ky = py / th, kz = pz / th;
  float sn, cs;
  or_sincos_turn((uint32_t)f2i32(th * ANG_INV_SCALE), &sn, &cs);
  float kd = kx * v[0] + ky * v[1];
  kd = kd + kz * v[2];
  float cx = ky * v[2] - kz * v[1];
  float cy = kz * v[0] - kx * v[2];
  float cz = kx * v[1] - ky * v[0];
  float kdo = kd * (1.0f - cs);
  float n0 = v[0] * cs + cx * sn;
  float n1 = v[1] * cs + cy * sn;
  float n2 = v[2] * cs + cz * sn;
  n0 = n0 + kx * kdo;
  n1 = n1 + ky * kdo;
  n2 = n2 + kz * kdo;
  float nn = n0 * n0 + n1 * n1;
  nn = nn + n2 * n2;
  float nm = sqrtf(nn);
  v[0] = n0 / nm;
  v[1] = n1 / nm;
  v[2] = n2 / nm;
}

/*
 * n_steps 3-D Brownian-dynamics sub-steps of ONE env.  q/img [3][n];
 * dir [3][n] fp32 unit directors; torque [3][n] lab frame; f_ext [3][n] or
 * NULL; vel/omega [3][n] (NULL allowed): BD velocity and angular velocity of
 * the last sub-step.  Noise tags: 0 translation, 2 rotation, 1 velocity,
 * 3 angular velocity.  f_swim0 / torque0 [3][n] / dir0 [3][n] (NULL: the
 * current ones): sub-step 0's swim force, torque and swim direction
 * (reuse_forces, see or_bd_run_walls).
 */
int or_bd_run3(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, float *dir,
               const uint8_t *species, const float *f_swim, const float *torque,
               const float *f_ext, uint64_t step0, int n_steps, uint32_t env, float *vel,
               float *omega, const swarm_wall_t *walls, int n_walls, uint64_t *violations,
               const float *f_swim0, const float *torque0, const float *dir0) {
  if (p->n_dims != 3)
    return SWARM_EINVAL;
  derived_t d;
  derive(p, &d);
  derive_walls(&d, walls, n_walls);
  uint64_t viol = 0;
  int64_t *acc = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(n > 0 ? n : 1));
  const int noisy = p->kT > 0.0;
  for (int s = 0; s < n_steps; ++s) {
    uint64_t step = step0 + (uint64_t)s;
    wca_forces3(p, &d, n, q, img, species, acc);
    for (int i = 0; i < n; ++i) {
      int sp = species[i];
      if (d.n_walls)
        wall_forces(&d, sp, (float)q[i] * d.sx[0], (float)q[n + i] * d.sx[1],
                    (float)q[2 * n + i] * d.sx[2], 3, &acc[i], &acc[n + i], &acc[2 * n + i],
                    &viol);
      float f[3], dq[3], ph[3], v[3] = {dir[i], dir[n + i], dir[2 * n + i]};
      const int first = s == 0;
      const float fs = first && f_swim0 ? f_swim0[i] : f_swim[i];
      const float *tq = first && torque0 ? torque0 : torque;
      for (int a = 0; a < 3; ++a) {
        const float va = first && dir0 ? dir0[a * n + i] : v[a];
        f[a] = (float)acc[a * n + i] * 5.9604644775390625e-08f;
        if (f_ext)
          f[a] = f[a] + f_ext[a * n + i];
        f[a] = f[a] + fs * va;
        dq[a] = f[a] * d.mob_dt[sp];
        ph[a] = tq[a * n + i] * d.rot_dt[sp];
      }
      if (noisy) {
        float g[3], h[3];
        or_step_normals(p->seed, env, (uint32_t)i, step, g);
        or_normals3(p->seed, env, (uint32_t)i, step, 2u, h);
        for (int a = 0; a < 3; ++a) {
          dq[a] = dq[a] + d.sig_t[sp] * g[a];
          ph[a] = ph[a] + d.sig_r[sp] * h[a];
        }
      }
      for (int a = 0; a < 3; ++a)
        advance(&q[a * n + i], &img[a * n + i], f2i32(dq[a] * d.inv_sx[a]));
      or_rotate_director(v, ph[0], ph[1], ph[2]);
      dir[i] = v[0];
      dir[n + i] = v[1];
      dir[2 * n + i] = v[2];
      if (s == n_steps - 1) {
        float vv[3], ww[3];
        for (int a = 0; a < 3; ++a) {
          vv[a] = f[a] * d.inv_gt[sp];
          ww[a] = tq[a * n + i] * d.inv_gr[sp];
        }
        if (noisy) {
          float g[3], h[3];
          or_normals3(p->seed, env, (uint32_t)i, step, 1u, g);
          or_normals3(p->seed, env, (uint32_t)i, step, 3u, h);
          for (int a = 0; a < 3; ++a) {
            vv[a] = vv[a] + d.sig_v[sp] * g[a];
            ww[a] = ww[a] + d.sig_w[sp] * h[a];
          }
        }
        for (int a = 0; a < 3; ++a) {
          if (vel)
            vel[a * n + i] = vv[a];
          if (omega)
            omega[a * n + i] = ww[a];
        }
      }
    }
  }
  free(acc);
  if (violations)
    *violations += viol;
  return SWARM_OK;
}

/* 3-D steepest descent: dp = clamp(gamma F) per coordinate, rotation by the
 * rotation vector clamp(gamma tau) (espresso.py:1161-1168). */
int or_sd_run3(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, float *dir,
               const uint8_t *species, const float *f_swim, const float *torque,
               const float *f_ext, int n_steps, double gamma, double max_disp,
               const swarm_wall_t *walls, int n_walls) {
  derived_t d;
  derive(p, &d);
  derive_walls(&d, walls, n_walls);
  uint64_t viol = 0;
  const float g = (float)gamma, md = (float)max_disp;
  int64_t *acc = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(n > 0 ? n : 1));
  int s;
  for (s = 0; s < n_steps; ++s) {
    wca_forces3(p, &d, n, q, img, species, acc);
    int any = 0;
    for (int i = 0; i < n; ++i) {
      int sp = species[i];
      if (d.n_walls)
        wall_forces(&d, sp, (float)q[i] * d.sx[0], (float)q[n + i] * d.sx[1],
                    (float)q[2 * n + i] * d.sx[2], 3, &acc[i], &acc[n + i], &acc[2 * n + i],
                    &viol);
      float v[3] = {dir[i], dir[n + i], dir[2 * n + i]}, pr[3];
      for (int a = 0; a < 3; ++a) {
        float f = (float)acc[a * n + i] * 5.9604644775390625e-08f;
        if (f_ext)
          f = f + f_ext[a * n + i];
        f = f + f_swim[i] * v[a];
        if (f != 0.0f || torque[a * n + i] != 0.0f)
          any = 1;
        float dp = fminf(fmaxf(g * f, -md), md);
        pr[a] = fminf(fmaxf(g * torque[a * n + i], -md), md);
        advance(&q[a * n + i], &img[a * n + i], f2i32(dp * d.inv_sx[a]));
      }
      or_rotate_director(v, pr[0], pr[1], pr[2]);
      dir[i] = v[0];
      dir[n + i] = v[1];
      dir[2 * n + i] = v[2];
    }
    if (!any)
      break;
  }
  free(acc);
  return s;
}

/*
 * Vision cones of ONE env, O(n_agents * n): out[a][k][t] (fp32).
 * radii[n]: radius of the seen colloid by list position; types[n]: type of
 * every colloid; det[n_types]: detected types; rims[n_cones + 1].
 */
/* What colloid j adds to agent i's cone bins (subdivided_vision_cones.py:
 * 116-153, 199-205); director (mx, my) of i. */
static void vision_pair(const derived_t *d, int n, const uint32_t *q, const int32_t *img,
                        int i, int j, float mx, float my, const float *radii,
                        const int *types, float vision_range, int n_cones, const float *rims,
                        int n_types, const int *det, int64_t *acc) {
  if (j == i)
    return;
  int ti = -1;
  for (int t = 0; t < n_types; ++t)
    if (det[t] == types[j])
      ti = t;
  if (ti < 0)
    return;
  /* unwrapped difference, no minimum image and no range limit
   * (subdivided_vision_cones.py:116-121) */
  float dd[2];
  for (int a = 0; a < 2; ++a) {
    int64_t dq = ((int64_t)(img[a * n + j] - img[a * n + i]) * (int64_t)4294967296LL) +
                 ((int64_t)q[a * n + j] - (int64_t)q[a * n + i]);
    dd[a] = (float)dq * d->sx[a];
  }
  float dist2 = dd[0] * dd[0] + dd[1] * dd[1];
  float dist = sqrtf(dist2);
  if (!(dist < vision_range) || dist == 0.0f)
    return;
  float amp = (2.0f * radii[j]) / dist;
  amp = fminf(1.0f, amp);
  float ux = dd[0] / dist, uy = dd[1] / dist;
  float dot = ux * mx + uy * my;
  dot = fminf(fmaxf(dot, -1.0f), 1.0f);
  float an = or_acosf(dot);
  float orth = ux * (-my) + uy * mx;
  if (orth < 0.0f)
    an = -an;
  for (int k = 0; k < n_cones; ++k)
    if (rims[k] < an && an < rims[k + 1])
      acc[k * n_types + ti] += (int64_t)llrintf(amp * 4294967296.0f);
}

static void vision_director(const uint32_t *ang, int i, float *mx, float *my) {
  float sn, cs;
  or_sincos_turn(ang[i], &sn, &cs);
  float nm = sqrtf(cs * cs + sn * sn);
  *mx = cs / nm;
  *my = sn / nm;
}

static void vision_store(const int64_t *acc, int ai, int nb, float *out) {
  for (int k = 0; k < nb; ++k)
    out[(size_t)ai * (size_t)nb + (size_t)k] = (float)acc[k] * 2.3283064365386963e-10f;
}

void or_vision_cone(const swarm_params_t *p, int n, const uint32_t *q,
                    const int32_t *img, const uint32_t *ang, const int *agents,
                    int n_agents, const float *radii, const int *types,
                    float vision_range, int n_cones, const float *rims,
                    int n_types, const int *det, float *out) {
  derived_t d;
  derive(p, &d);
#pragma omp parallel for schedule(dynamic, 16)
  for (int ai = 0; ai < n_agents; ++ai) {
    int64_t acc[SWARM_MAX_CONES * SWARM_MAX_DETECTED_TYPES];
    int i = agents[ai];
    memset(acc, 0, sizeof(acc));
    float mx, my;
    vision_director(ang, i, &mx, &my);
    for (int j = 0; j < n; ++j)
      vision_pair(&d, n, q, img, i, j, mx, my, radii, types, vision_range, n_cones, rims,
                  n_types, det, acc);
    vision_store(acc, ai, n_cones * n_types, out);
  }
}

/*
 * The same vision cones over a cell list (the CPU comparator of SURVEY
 * 8(d)): cells of side >= vision_range over the folded positions, the 3 x 3
 * cells around each agent (periodic).  A colloid within vision_range of the
 * agent by its unwrapped difference is within vision_range by the minimum
 * image too (vision_range < L / 2), so it lies in those cells; the bins are
 * int64 sums, so the result has the bits of or_vision_cone.  Returns
 * SWARM_EINVAL when 2 vision_range >= the box (use or_vision_cone).
 */
int or_vision_cone_cells(const swarm_params_t *p, int n, const uint32_t *q,
                         const int32_t *img, const uint32_t *ang, const int *agents,
                         int n_agents, const float *radii, const int *types,
                         float vision_range, int n_cones, const float *rims,
                         int n_types, const int *det, float *out) {
  if (!p->periodic || !(2.0 * vision_range < p->box[0]) || !(2.0 * vision_range < p->box[1]))
    return SWARM_EINVAL;
  derived_t d;
  derive(p, &d);
  celllist_t cl;
  or_cell_grid(p, n, vision_range, &cl.lx, &cl.ly);
  cl.ncell = 1 << (cl.lx + cl.ly);
  cl.start = (int *)malloc(sizeof(int) * (size_t)(cl.ncell + 1));
  cl.list = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  cl.cell = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  cl_build(&cl, p, q, img, n);
  const int ncx = 1 << cl.lx, ncy = 1 << cl.ly;
  const int lox = ncx >= 3 ? -1 : 0, hix = ncx >= 3 ? 1 : ncx - 1;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
#pragma omp parallel for schedule(dynamic, 16)
  for (int ai = 0; ai < n_agents; ++ai) {
    int64_t acc[SWARM_MAX_CONES * SWARM_MAX_DETECTED_TYPES];
    int i = agents[ai];
    memset(acc, 0, sizeof(acc));
    float mx, my;
    vision_director(ang, i, &mx, &my);
    const int c = cl.cell[i], cx = c % ncx, cy = c / ncx;
    for (int oy = loy; oy <= hiy; ++oy)
      for (int ox = lox; ox <= hix; ++ox) {
        const int cc = ((cy + oy + ncy) % ncy) * ncx + (cx + ox + ncx) % ncx;
        for (int k = cl.start[cc]; k < cl.start[cc + 1]; ++k)
          vision_pair(&d, n, q, img, i, cl.list[k], mx, my, radii, types, vision_range,
                      n_cones, rims, n_types, det, acc);
      }
    vision_store(acc, ai, n_cones * n_types, out);
  }
  cl_free(&cl);
  return SWARM_OK;
}

/* unwrapped position along axis a, fp64 */
static double unwrap(const swarm_params_t *p, const uint32_t *q,
                     const int32_t *img, int n, int a, int i) {
  return ((double)img[a * n + i] + (double)q[a * n + i] * (1.0 / TWO32)) *
         p->box[a];
}

/* Field distances of ONE env (see swarm_field_distance in the C ABI).
 * hist_q / hist_img: [3][n_agents]. */
void or_field_distance(const swarm_params_t *p, int n, const uint32_t *q,
                       const int32_t *img, const int *agents, int n_agents,
                       const double source[3], const double box_scale[3],
                       uint32_t *hist_q, int32_t *hist_img, float *d_cur,
                       float *d_prev, int update_history) {
  double src[3];
  for (int a = 0; a < 3; ++a)
    src[a] = source[a] / box_scale[a];
#pragma omp parallel for schedule(static)
  for (int ai = 0; ai < n_agents; ++ai) {
    int i = agents[ai];
    float cur[3], prev[3];
    for (int a = 0; a < 3; ++a) {
      double pc = a < p->n_dims ? unwrap(p, q, img, n, a, i) / box_scale[a] : 0.0 / box_scale[a];
      double hp = a < p->n_dims ? ((double)hist_img[a * n_agents + ai] +
                           (double)hist_q[a * n_agents + ai] * (1.0 / TWO32)) *
                              p->box[a] / box_scale[a]
                        : 0.0 / box_scale[a];
      cur[a] = (float)(src[a] - pc);
      prev[a] = (float)(src[a] - hp);
    }
    d_cur[ai] = sqrtf(cur[0] * cur[0] + cur[1] * cur[1] + cur[2] * cur[2]);
    d_prev[ai] = sqrtf(prev[0] * prev[0] + prev[1] * prev[1] + prev[2] * prev[2]);
    if (update_history)
      for (int a = 0; a < 3; ++a) {
        hist_q[a * n_agents + ai] = q[a * n + i];
        hist_img[a * n_agents + ai] = img[a * n + i];
      }
  }
}

/* All pairs i<j closer than cutoff (minimum image if periodic). */
int or_neighbor_pairs(const swarm_params_t *p, int n, const uint32_t *q,
                      const int32_t *img, double cutoff, int *pairs,
                      int max_pairs) {
  derived_t d;
  derive(p, &d);
  float c2 = (float)(cutoff * cutoff);
  int np = 0;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      float rx = pair_disp(p, &d, q, img, n, 0, i, j);
      float ry = pair_disp(p, &d, q, img, n, 1, i, j);
      if (rx * rx + ry * ry < c2) {
        if (np < max_pairs) {
          pairs[2 * np] = i;
          pairs[2 * np + 1] = j;
        }
        np++;
      }
    }
  return np;
}
