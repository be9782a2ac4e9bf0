/*
 * Sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY, SURVEY.md
 * section 5: AddressSanitizer / UndefinedBehaviorSanitizer on host code, the
 * only sanitizers this pool runs).  `make -C oracle sanitize` compiles it with
 * swarm_oracle.c under -fsanitize=address,undefined and
 * -fno-sanitize-recover=all, so any out-of-bounds access, leak, signed
 * overflow, misaligned load or bad shift in the oracle aborts the program.
 *
 * It drives every entry point tests/ uses, on seeded random swarms sized to
 * hit the edge cases: empty and single-particle systems, multi-species pair
 * tables, crowded boxes (many WCA contacts), periodic and non-periodic boxes,
 * walls of both kinds, 2-D and 3-D, vision cones with ranges near half the
 * box, and the cell-list / all-pairs paths against each other (same bits).
 * Exit status 0 and "sanitize: ok" on success.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/swarmrl_amd.h"

/* oracle entry points (swarm_oracle.c) */
int or_bd_run_walls(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, uint32_t *ang,
                    const uint8_t *species, const float *f_swim, const float *torque_z,
                    const float *f_ext, uint64_t step0, int n_steps, uint32_t env, float *vel,
                    float *omega, int use_cells, const swarm_wall_t *walls, int n_walls,
                    uint64_t *violations, const float *f_swim0, const float *torque0,
                    const uint32_t *ang0);
int or_sd_run_walls(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, uint32_t *ang,
                    const uint8_t *species, const float *f_swim, const float *torque_z,
                    const float *f_ext, int n_steps, double gamma, double max_disp,
                    int use_cells, const swarm_wall_t *walls, int n_walls);
int or_bd_run3(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, float *dir,
               const uint8_t *species, const float *f_swim, const float *torque,
               const float *f_ext, uint64_t step0, int n_steps, uint32_t env, float *vel,
               float *omega, const swarm_wall_t *walls, int n_walls, uint64_t *violations,
               const float *f_swim0, const float *torque0, const float *dir0);
int or_sd_run3(const swarm_params_t *p, int n, uint32_t *q, int32_t *img, float *dir,
               const uint8_t *species, const float *f_swim, const float *torque,
               const float *f_ext, int n_steps, double gamma, double max_disp,
               const swarm_wall_t *walls, int n_walls);
void or_vision_cone(const swarm_params_t *p, int n, const uint32_t *q, const int32_t *img,
                    const uint32_t *ang, const int *agents, int n_agents, const float *radii,
                    const int *types, float vision_range, int n_cones, const float *rims,
                    int n_types, const int *det, float *out);
int or_vision_cone_cells(const swarm_params_t *p, int n, const uint32_t *q, const int32_t *img,
                         const uint32_t *ang, const int *agents, int n_agents,
                         const float *radii, const int *types, float vision_range, int n_cones,
                         const float *rims, int n_types, const int *det, float *out);
void or_field_distance(const swarm_params_t *p, int n, const uint32_t *q, const int32_t *img,
                       const int *agents, int n_agents, const double source[3],
                       const double box_scale[3], uint32_t *hist_q, int32_t *hist_img,
                       float *d_cur, float *d_prev, int update_history);
int or_neighbor_pairs(const swarm_params_t *p, int n, const uint32_t *q, const int32_t *img,
                      double cutoff, int *pairs, int max_pairs);

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd32(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)(rng_state >> 16);
}
static float rndf(void) { return (float)(rnd32() >> 8) * (1.0f / 16777216.0f); }

static void fail(const char *what) {
  fprintf(stderr, "sanitize: FAILED: %s\n", what);
  exit(1);
}

static swarm_params_t params(int dims, int periodic, double L, int n_species) {
  swarm_params_t p;
  memset(&p, 0, sizeof(p));
  p.n_dims = dims;
  p.periodic = periodic;
  p.box[0] = p.box[1] = p.box[2] = L;
  p.time_step = 1e-3;
  p.kT = 1.0239;
  p.wca_epsilon = 1.0239;
  p.seed = 42;
  p.n_species = n_species;
  p.reuse_forces = 1;
  for (int s = 0; s < n_species; ++s) {
    p.radius[s] = 0.5 + 0.5 * s;
    p.gamma_t[s] = 4.66 * p.radius[s];
    p.gamma_r[s] = 6.21 * p.radius[s] * p.radius[s] * p.radius[s];
    p.mass[s] = 1.0358e-6;
    p.rinertia[s] = 4.143e-7;
  }
  return p;
}

/* one 2-D system: overlap removal, Brownian dynamics with and without cell
 * lists (same bits), walls, vision cones, field distances, neighbour pairs */
static void run2d(int n, double L, int periodic, int n_species, int n_walls) {
  swarm_params_t p = params(2, periodic, L, n_species);
  const size_t m = (size_t)(n > 0 ? n : 1);
  uint32_t *q = calloc(3 * m, 4), *q2 = calloc(3 * m, 4), *ang = calloc(m, 4), *ang2 = calloc(m, 4);
  int32_t *img = calloc(3 * m, 4), *img2 = calloc(3 * m, 4);
  uint8_t *sp = calloc(m, 1);
  float *fs = calloc(m, 4), *tz = calloc(m, 4), *fx = calloc(3 * m, 4);
  float *vel = calloc(3 * m, 4), *om = calloc(m, 4), *vel2 = calloc(3 * m, 4), *om2 = calloc(m, 4);
  for (int i = 0; i < n; ++i) {
    q[i] = rnd32();
    q[m + i] = rnd32();
    img[i] = (int32_t)(rnd32() % 5) - 2;
    img[m + i] = (int32_t)(rnd32() % 5) - 2;
    ang[i] = rnd32();
    sp[i] = (uint8_t)(rnd32() % (uint32_t)n_species);
    fs[i] = 10.0f * rndf();
    tz[i] = 10.0f * (rndf() - 0.5f);
    fx[i] = rndf() - 0.5f;
  }
  if (!periodic)
    for (int i = 0; i < n; ++i) img[i] = img[m + i] = 0;
  swarm_wall_t walls[2];
  memset(walls, 0, sizeof(walls));
  walls[0].kind = 0; /* plane y > 0.05 L */
  walls[0].normal[1] = 1.0;
  walls[0].offset = 0.05 * L;
  walls[1].kind = 1; /* a slab in the middle */
  walls[1].corner[0] = 0.4 * L;
  walls[1].corner[1] = 0.4 * L;
  walls[1].a[0] = 0.1 * L;
  walls[1].b[1] = 0.1 * L;
  or_sd_run_walls(&p, n, q, img, ang, sp, fs, tz, fx, 50, 0.1, 0.1, 1, walls, n_walls);
  memcpy(q2, q, 12 * m);
  memcpy(img2, img, 12 * m);
  memcpy(ang2, ang, 4 * m);
  uint64_t v1 = 0, v2 = 0;
  or_bd_run_walls(&p, n, q, img, ang, sp, fs, tz, fx, 0, 37, 1, vel, om, 1, walls, n_walls, &v1,
                  NULL, NULL, NULL);
  or_bd_run_walls(&p, n, q2, img2, ang2, sp, fs, tz, fx, 0, 37, 1, vel2, om2, 0, walls, n_walls,
                  &v2, NULL, NULL, NULL);
  if (memcmp(q, q2, 12 * m) || memcmp(img, img2, 12 * m) || memcmp(ang, ang2, 4 * m) || v1 != v2)
    fail("2-D cell-list and all-pairs runs differ");
  /* reuse_forces: sub-step 0 from the previous run's actions */
  or_bd_run_walls(&p, n, q, img, ang, sp, fs, tz, fx, 37, 5, 1, vel, om, 1, walls, n_walls, &v1,
                  tz, fs, ang2);
  int *agents = calloc(m, sizeof(int)), *types = calloc(m, sizeof(int));
  float *radii = calloc(m, 4);
  int na = 0;
  for (int i = 0; i < n; ++i) {
    types[i] = (int)(rnd32() % 3u);
    radii[i] = 0.5f + rndf();
    if (i % 2 == 0) agents[na++] = i;
  }
  const int det[2] = {0, 2};
  const float rims[4] = {-1.5f, -0.5f, 0.5f, 1.5f};
  const float R = (float)(0.45 * L);
  float *o1 = calloc(m * 6, 4), *o2 = calloc(m * 6, 4);
  or_vision_cone(&p, n, q, img, ang, agents, na, radii, types, R, 3, rims, 2, det, o1);
  if (periodic) {
    if (or_vision_cone_cells(&p, n, q, img, ang, agents, na, radii, types, R, 3, rims, 2, det,
                             o2) != 0)
      fail("vision cone cells refused a range below half the box");
    if (memcmp(o1, o2, (size_t)na * 6 * 4)) fail("vision cone cells != all pairs");
  }
  uint32_t *hq = calloc(3 * m, 4);
  int32_t *hi = calloc(3 * m, 4);
  float *dc = calloc(m, 4), *dp = calloc(m, 4);
  const double src[3] = {0.5 * L, 0.5 * L, 0.0}, scale[3] = {L, L, L};
  or_field_distance(&p, n, q, img, agents, na, src, scale, hq, hi, dc, dp, 1);
  or_field_distance(&p, n, q, img, agents, na, src, scale, hq, hi, dc, dp, 0);
  int *pairs = calloc(2 * m * 8, sizeof(int));
  or_neighbor_pairs(&p, n, q, img, 2.5, pairs, (int)(m * 8));
  free(q), free(q2), free(ang), free(ang2), free(img), free(img2), free(sp), free(fs), free(tz);
  free(fx), free(vel), free(om), free(vel2), free(om2), free(agents), free(types), free(radii);
  free(o1), free(o2), free(hq), free(hi), free(dc), free(dp), free(pairs);
}

static void run3d(int n, double L, int n_species, int n_walls) {
  swarm_params_t p = params(3, 1, L, n_species);
  const size_t m = (size_t)(n > 0 ? n : 1);
  uint32_t *q = calloc(3 * m, 4);
  int32_t *img = calloc(3 * m, 4);
  float *dir = calloc(3 * m, 4), *tq = calloc(3 * m, 4), *fx = calloc(3 * m, 4);
  float *fs = calloc(m, 4), *vel = calloc(3 * m, 4), *om = calloc(3 * m, 4);
  uint8_t *sp = calloc(m, 1);
  for (int i = 0; i < n; ++i) {
    for (int a = 0; a < 3; ++a) {
      q[a * m + i] = rnd32();
      img[a * m + i] = (int32_t)(rnd32() % 3u) - 1;
      tq[a * m + i] = 5.0f * (rndf() - 0.5f);
    }
    dir[i] = 1.0f;
    sp[i] = (uint8_t)(rnd32() % (uint32_t)n_species);
    fs[i] = 10.0f * rndf();
  }
  swarm_wall_t w;
  memset(&w, 0, sizeof(w));
  w.kind = 0;
  w.normal[2] = 1.0;
  w.offset = 0.02 * L;
  uint64_t v = 0;
  or_sd_run3(&p, n, q, img, dir, sp, fs, tq, fx, 30, 0.1, 0.1, &w, n_walls);
  or_bd_run3(&p, n, q, img, dir, sp, fs, tq, fx, 0, 23, 2, vel, om, &w, n_walls, &v, NULL, NULL,
             NULL);
  or_bd_run3(&p, n, q, img, dir, sp, fs, tq, fx, 23, 4, 2, vel, om, &w, n_walls, &v, fs, tq, dir);
  free(q), free(img), free(dir), free(tq), free(fx), free(fs), free(vel), free(om), free(sp);
}

int main(void) {
  /* edge cases first: empty, one particle, two overlapping species */
  run2d(0, 20.0, 1, 1, 0);
  run2d(1, 20.0, 1, 1, 2);
  run2d(2, 4.0, 1, 2, 0);
  /* crowded (many contacts), dilute, non-periodic, walls, several species */
  run2d(400, 40.0, 1, 3, 2);
  run2d(300, 120.0, 1, 1, 0);
  run2d(200, 60.0, 0, 2, 1);
  run3d(0, 20.0, 1, 0);
  run3d(1, 20.0, 1, 1);
  run3d(300, 30.0, 2, 1);
  printf("sanitize: ok\n");
  return 0;
}
