// swarm_integrator3.cuh -- 3-D Brownian dynamics + WCA (+ walls).
//
// The reference's default engine dimension is 3 (EspressoMD(n_dims=3),
// espresso.py:143-152; particles added with rotation about all three axes
// and no fixed coordinate, espresso.py:415-426).  3-D runs on the global
// path: one workgroup per env does every sub-step (per sub-step a counting
// sort into 3-D cells of side >= rc_max, the 27-cell pair search, then the
// update), so it needs no cluster decomposition.  The 2-D RL workloads of
// the benchmark use the cluster path (swarm_integrator.cuh).
//
// Orientation is an fp32 unit director.  Per sub-step the rotation vector
//   phi = tau dt / gamma_r + sqrt(2 kT dt / gamma_r) xi     (lab frame)
// turns the director by |phi| about phi/|phi| (Rodrigues), followed by a
// renormalisation; translation is x += F dt / gamma_t + sqrt(2 kT dt /
// gamma_t) xi with F = WCA + walls + f_ext + f_swim * director.  Same
// operation sequence as oracle/swarm_oracle.c:or_bd_run3, so the result is
// bit-identical to the oracle (pair sums are int64 fixed point).
#pragma once

#include "swarm_integrator.cuh"

namespace swarm {

__device__ __forceinline__ int cell_index3(uint32_t qx, uint32_t qy, uint32_t qz, int lx, int ly,
                                           int lz) {
  const int cx = lx == 0 ? 0 : (int)(qx >> (32 - lx));
  const int cy = ly == 0 ? 0 : (int)(qy >> (32 - ly));
  const int cz = lz == 0 ? 0 : (int)(qz >> (32 - lz));
  return (((cz << ly) | cy) << lx) | cx;
}

__device__ __forceinline__ void pair_force3(float cut2, float sig6, float eps24, float rx,
                                            float ry, float rz, int64_t& ax, int64_t& ay,
                                            int64_t& az) {
  float r2 = rx * rx + ry * ry;
  r2 = r2 + rz * rz;
  if (r2 < cut2 && r2 > 0.0f) {
    const float ir2 = 1.0f / r2;
    float ir6 = ir2 * ir2;
    ir6 = ir6 * ir2;
    const float s6 = sig6 * ir6;
    float t = 2.0f * s6;
    t = t - 1.0f;
    float fr = eps24 * s6;
    fr = fr * t;
    fr = fr * ir2;
    ax += f2fix24(-fr * rx);
    ay += f2fix24(-fr * ry);
    az += f2fix24(-fr * rz);
  }
}

// Rotate the unit director v by the rotation vector p and renormalise
// (oracle: or_rotate_director).
__device__ __forceinline__ void rotate_director(float v[3], float px, float py, float pz) {
  float th2 = px * px + py * py;
  th2 = th2 + pz * pz;
  if (!(th2 > 0.0f)) return;
  const float th = sqrt_rn(th2);
  const float kx = px / th, ky = py / th, kz = pz / th;
  float sn, cs;
  sincos_turn((uint32_t)f2i32(th * kAngInvScale), &sn, &cs);
  float kd = kx * v[0] + ky * v[1];
  kd = kd + kz * v[2];
  const float cx = ky * v[2] - kz * v[1];
  const float cy = kz * v[0] - kx * v[2];
  const float cz = kx * v[1] - ky * v[0];
  const float kdo = kd * (1.0f - cs);
  float n0 = v[0] * cs + cx * sn;
  float n1 = v[1] * cs + cy * sn;
  float n2 = v[2] * cs + cz * sn;
  n0 = n0 + kx * kdo;
  n1 = n1 + ky * kdo;
  n2 = n2 + kz * kdo;
  float nn = n0 * n0 + n1 * n1;
  nn = nn + n2 * n2;
  const float nm = sqrt_rn(nn);
  v[0] = n0 / nm;
  v[1] = n1 / nm;
  v[2] = n2 / nm;
}

// All sub-steps (or steepest-descent steps) of env e, 3-D, by one
// workgroup.  cnt: LDS counts of the 2^(lx+ly+lz) cells.
__device__ void block_global_run3(const Derived* __restrict__ d, const DevState& st,
                                  const Scratch& sc, int e, int n_steps, uint64_t step0, int lx,
                                  int ly, int lz, bool sd_mode, float g, float md, int32_t* cnt,
                                  int32_t* wave_sums, const PairTables* pt, int rp) {
  const PrevSlot prv = prev_slot(st, rp);  // reuse_forces: sub-step 0 reads slot rp
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly + lz);
  const int nc[3] = {1 << lx, 1 << ly, 1 << lz};
  int lo[3], hi[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    lo[a] = nc[a] >= 3 ? -1 : 0;
    hi[a] = nc[a] >= 3 ? 1 : nc[a] - 1;
  }
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx[3] = {d->sx[0], d->sx[1], d->sx[2]};
  const float eps24 = d->eps24;
  const bool noisy = d->noisy != 0;
  const bool per = d->periodic != 0;  // non-periodic: edge cells, unwrapped differences
  auto cell_of3 = [&](size_t gi) {
    return (((cell_coord(st.q[2 * M + gi], st.img[2 * M + gi], lz, per) << ly) |
             cell_coord(st.q[M + gi], st.img[M + gi], ly, per))
            << lx) |
           cell_coord(st.q[gi], st.img[gi], lx, per);
  };
  for (int s = 0; s < n_steps; ++s) {
    for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += T) atomicAdd(&cnt[cell_of3(base + i)], 1);
    __syncthreads();
    block_exclusive_scan(cnt, ncell, wave_sums);
    __syncthreads();
    for (int i = tid; i < N; i += T) {
      const uint32_t qx = st.q[base + i], qy = st.q[M + base + i], qz = st.q[2 * M + base + i];
      const int pos = atomicAdd(&cnt[cell_of3(base + i)], 1);
      sc.sqx[base + pos] = qx;
      sc.sqy[base + pos] = qy;
      sc.sqz[base + pos] = qz;
      sc.sidx[base + pos] = i;
    }
    __syncthreads();  // cell c now spans [c ? cnt[c-1] : 0, cnt[c])
    int any = 0;
    for (int i = tid; i < N; i += T) {
      const size_t gi = base + i;
      uint32_t q[3];
      int32_t im[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        q[a] = st.q[a * M + gi];
        im[a] = st.img[a * M + gi];
      }
      float v[3] = {st.dir3[gi], st.dir3[M + gi], st.dir3[2 * M + gi]};
      // reuse_forces: sub-step 0 takes the previous run's actions and director
      const bool first = st.reuse && s == 0 && !sd_mode;
      const int si = st.species[i];
      int64_t acc[3] = {0, 0, 0};
      const int c0 = cell_of3(gi);
      const int cc[3] = {c0 & (nc[0] - 1), (c0 >> lx) & (nc[1] - 1), c0 >> (lx + ly)};
      for (int oz = lo[2]; oz <= hi[2]; ++oz) {
        if (!per && (cc[2] + oz < 0 || cc[2] + oz >= nc[2])) continue;
        const int z = (cc[2] + oz + nc[2]) & (nc[2] - 1);
        for (int oy = lo[1]; oy <= hi[1]; ++oy) {
          if (!per && (cc[1] + oy < 0 || cc[1] + oy >= nc[1])) continue;
          const int y = (cc[1] + oy + nc[1]) & (nc[1] - 1);
          for (int ox = lo[0]; ox <= hi[0]; ++ox) {
            if (!per && (cc[0] + ox < 0 || cc[0] + ox >= nc[0])) continue;
            const int x = (cc[0] + ox + nc[0]) & (nc[0] - 1);
            const int cell = (((z << ly) | y) << lx) | x;
            const int jb = cell ? cnt[cell - 1] : 0, je = cnt[cell];
            for (int jj = jb; jj < je; ++jj) {
              const int j = sc.sidx[base + jj];
              if (j == i) continue;
              const size_t gj = base + j;
              float rx, ry, rz;
              if (per) {
                rx = (float)(int32_t)(sc.sqx[base + jj] - q[0]) * sx[0];
                ry = (float)(int32_t)(sc.sqy[base + jj] - q[1]) * sx[1];
                rz = (float)(int32_t)(sc.sqz[base + jj] - q[2]) * sx[2];
              } else {
                rx = pair_disp(sc.sqx[base + jj], st.img[gj], q[0], im[0], sx[0], false);
                ry = pair_disp(sc.sqy[base + jj], st.img[M + gj], q[1], im[1], sx[1], false);
                rz = pair_disp(sc.sqz[base + jj], st.img[2 * M + gj], q[2], im[2], sx[2], false);
              }
              const int pk = si * kMaxSpecies + st.species[j];
              pair_force3(pt->cut2[pk], pt->sig6[pk], eps24, rx, ry, rz, acc[0], acc[1],
                          acc[2]);
            }
          }
        }
      }
      if (d->n_walls)
        wall_forces<3>(d, si, (float)q[0] * sx[0], (float)q[1] * sx[1], (float)q[2] * sx[2],
                       acc[0], acc[1], acc[2], st.wall_viol);
      const float fs = first ? prv.f[gi] : st.f_swim[gi];
      const float tq[3] = {first ? prv.txy[gi] : st.torque_xy[gi],
                           first ? prv.txy[M + gi] : st.torque_xy[M + gi],
                           first ? prv.tz[gi] : st.torque_z[gi]};
      const float vs[3] = {first ? prv.dir3[gi] : v[0], first ? prv.dir3[M + gi] : v[1],
                           first ? prv.dir3[2 * M + gi] : v[2]};
      float f[3], dq[3], ph[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        f[a] = i64_to_f32(acc[a]) * 5.9604644775390625e-08f;
        f[a] = f[a] + st.f_ext[a * M + gi];
        f[a] = f[a] + fs * vs[a];
      }
      if (sd_mode) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          if (f[a] != 0.0f || tq[a] != 0.0f) any = 1;
          const float dp = fminf(fmaxf(g * f[a], -md), md);
          ph[a] = fminf(fmaxf(g * tq[a], -md), md);
          advance(q[a], im[a], f2i32(dp * d->inv_sx[a]));
        }
        rotate_director(v, ph[0], ph[1], ph[2]);
      } else {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          dq[a] = f[a] * d->mob_dt[si];
          ph[a] = tq[a] * d->rot_dt[si];
        }
        const uint64_t step = step0 + (uint64_t)s;
        if (noisy) {
          float gt[3], gr[3];
          step_normals(k0, k1, (uint32_t)i, step, gt);
          normals3(k0, k1, (uint32_t)i, step, 2u, gr);
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            dq[a] = dq[a] + d->sig_t[si] * gt[a];
            ph[a] = ph[a] + d->sig_r[si] * gr[a];
          }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) advance(q[a], im[a], f2i32(dq[a] * d->inv_sx[a]));
        rotate_director(v, ph[0], ph[1], ph[2]);
        if (s == n_steps - 1) {
          float vv[3], ww[3];
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            vv[a] = f[a] * d->inv_gt[si];
            ww[a] = tq[a] * d->inv_gr[si];
          }
          if (noisy) {
            float gv[3], gw[3];
            normals3(k0, k1, (uint32_t)i, step, 1u, gv);
            normals3(k0, k1, (uint32_t)i, step, 3u, gw);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
              vv[a] = vv[a] + d->sig_v[si] * gv[a];
              ww[a] = ww[a] + d->sig_w[si] * gw[a];
            }
          }
#pragma unroll
          for (int a = 0; a < 3; ++a) st.vel[a * M + gi] = vv[a];
          st.omega_xy[gi] = ww[0];
          st.omega_xy[M + gi] = ww[1];
          st.omega[gi] = ww[2];
        }
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        st.q[a * M + gi] = q[a];
        st.img[a * M + gi] = im[a];
        st.dir3[a * M + gi] = v[a];
      }
    }
    if (sd_mode) {
      if (!__syncthreads_or(any)) break;
    } else {
      __syncthreads();
    }
  }
}

// 3-D global-path launch: n_steps sub-steps (or SD steps) of every env.
__global__ __launch_bounds__(1024) void k_global3(const Derived* __restrict__ d, DevState st,
                                                  Scratch sc, int n_steps,
                                                  uint64_t* __restrict__ step_ctr,
                                                  uint32_t* __restrict__ arrive, int lx, int ly,
                                                  int lz, int sd_mode, float g, float md) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ PairTables pt;
  stage_pair_tables(d, &pt);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  const uint64_t step0 = sd_mode ? 0ull : *step_ctr;
  const int par = window_parity(step_ctr);  // reuse_forces slots (k_global)
  block_global_run3(d, st, sc, blockIdx.x, n_steps, step0, lx, ly, lz, sd_mode != 0, g, md, cnt,
                    wave_sums, &pt, par);
  save_forces_env(st, blockIdx.x, sd_mode ? par : par ^ 1);
  if (!sd_mode) advance_counter(step_ctr, arrive, step0, n_steps);
}

}  // namespace swarm
