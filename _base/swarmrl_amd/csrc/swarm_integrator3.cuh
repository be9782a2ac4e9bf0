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
      if (!per)  // the images too: the update below rewrites st.img in place
        for (int a = 0; a < 3; ++a) sc.simg[(size_t)a * M + base + pos] = st.img[a * M + base + i];
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
              float rx, ry, rz;
              if (per) {
                rx = (float)(int32_t)(sc.sqx[base + jj] - q[0]) * sx[0];
                ry = (float)(int32_t)(sc.sqy[base + jj] - q[1]) * sx[1];
                rz = (float)(int32_t)(sc.sqz[base + jj] - q[2]) * sx[2];
              } else {
                rx = pair_disp(sc.sqx[base + jj], sc.simg[base + jj], q[0], im[0], sx[0], false);
                ry = pair_disp(sc.sqy[base + jj], sc.simg[M + base + jj], q[1], im[1], sx[1],
                               false);
                rz = pair_disp(sc.sqz[base + jj], sc.simg[2 * M + base + jj], q[2], im[2], sx[2],
                               false);
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


// ------------------------------------------------- 3-D cluster window
// Build step 1 (3-D), one workgroup per env: counting sort into cells of
// side >= rc_max + skin.  Same output layout as k_build_sort with a third
// position row: bsq[0..2][M], bsid, bcstart[E][ncb + 1].
template <int CH>
__global__ __launch_bounds__(1024) void k_build_sort3(DevState st, Scratch sc, int lx, int ly,
                                                      int lz) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly + lz);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  // cell of particle i: folded positions in a periodic box; in a
  // non-periodic one a particle outside the box takes the edge cell on its
  // side (cell_coord, as the 2-D build sort and the global path)
  const bool per = sc.periodic != 0;
  auto cell_of = [&](int i, uint32_t qx, uint32_t qy, uint32_t qz) {
    if (per) return cell_index3(qx, qy, qz, lx, ly, lz);
    return (((cell_coord(qz, st.img[2 * M + base + i], lz, false) << ly) |
             cell_coord(qy, st.img[M + base + i], ly, false))
            << lx) |
           cell_coord(qx, st.img[base + i], lx, false);
  };
  uint32_t cq[CH][3];
  int32_t cid[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int i = tid + k * T;
    const bool ok = i < N;
#pragma unroll
    for (int a = 0; a < 3; ++a) cq[k][a] = ok ? st.q[a * M + base + i] : 0u;
    cid[k] = ok ? (i | ((int32_t)st.species[i] << 24)) : -1;
  }
  for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
  if (tid == 0) {
    sc.gnpairs[e] = 0;
    sc.gnx[e] = 0;
    sc.fallback[e] = 0;  // the neighbour-list build sets it on overflow
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CH; ++k)
    if (cid[k] >= 0) atomicAdd(&cnt[cell_of(tid + k * T, cq[k][0], cq[k][1], cq[k][2])], 1);
  for (int i = tid + CH * T; i < N; i += T)
    atomicAdd(&cnt[cell_of(i, st.q[base + i], st.q[M + base + i], st.q[2 * M + base + i])], 1);
  __syncthreads();
  block_exclusive_scan(cnt, ncell, wave_sums);
  __syncthreads();
  int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  for (int c = tid; c <= ncell; c += T) cs[c] = cnt[c];
  __syncthreads();  // cnt is read above and incremented below
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    if (cid[k] < 0) continue;
    const size_t pos = base + atomicAdd(&cnt[cell_of(tid + k * T, cq[k][0], cq[k][1], cq[k][2])], 1);
#pragma unroll
    for (int a = 0; a < 3; ++a) sc.bsq[a * M + pos] = cq[k][a];
    sc.bsid[pos] = cid[k];
  }
  for (int i = tid + CH * T; i < N; i += T) {
    const uint32_t qx = st.q[base + i], qy = st.q[M + base + i], qz = st.q[2 * M + base + i];
    const size_t pos = base + atomicAdd(&cnt[cell_of(i, qx, qy, qz)], 1);
    sc.bsq[pos] = qx;
    sc.bsq[M + pos] = qy;
    sc.bsq[2 * M + pos] = qz;
    sc.bsid[pos] = i | ((int32_t)st.species[i] << 24);
  }
  for (int k = tid; k < sc.S; k += T) sc.perm[(size_t)e * sc.S + k] = -1;
}

// Build step 2 (3-D), chip-wide (grid.y = env, one thread per sorted
// entry): every pair within r_i + r_j + skin once (i < j), into the same
// pair list k_cluster_build consumes.  The 27-cell stencil is nine rows
// (y, z offsets), each a contiguous x range of the sorted order plus a wrap
// range at the grid edge: 18 range bounds, loaded together.
__global__ __launch_bounds__(256) void k_build_pairs3(const Derived* __restrict__ d, DevState st,
                                                      Scratch sc, int lx, int ly, int lz) {
  constexpr int kKeep = 8;
  constexpr int kR = 18;
  __shared__ float nb2[kMaxSpecies * kMaxSpecies];
  for (int k = threadIdx.x; k < kMaxSpecies * kMaxSpecies; k += blockDim.x) nb2[k] = d->nb2[k];
  const int e = blockIdx.y, N = st.n;
  const int ps = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = ps < N;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly + lz);
  const int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  const int ncx = 1 << lx, ncy = 1 << ly, ncz = 1 << lz;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const int loz = ncz >= 3 ? -1 : 0, hiz = ncz >= 3 ? 1 : ncz - 1;
  const float sx0 = d->sx[0], sx1 = d->sx[1], sx2 = d->sx[2];
  // non-periodic box (d->periodic == 0): edge cells, no wrap of the stencil,
  // unwrapped pair distances (pair_disp) -- a pair near across the box edge
  // only in the folded sense must not be listed
  const bool per = d->periodic != 0;
  int pk = 0, i = 0;
  uint32_t qx = 0, qy = 0, qz = 0;
  int32_t ix = 0, iy = 0, iz = 0;
  if (valid) {
    pk = sc.bsid[base + ps];
    i = pk & 0xffffff;
    qx = sc.bsq[base + ps];
    qy = sc.bsq[M + base + ps];
    qz = sc.bsq[2 * M + base + ps];
    if (!per) {
      ix = st.img[base + i];
      iy = st.img[M + base + i];
      iz = st.img[2 * M + base + i];
    }
  }
  const int c0 = per ? cell_index3(qx, qy, qz, lx, ly, lz)
                     : (((cell_coord(qz, iz, lz, false) << ly) | cell_coord(qy, iy, ly, false))
                        << lx) |
                           cell_coord(qx, ix, lx, false);
  const int cx = c0 & (ncx - 1), cy = (c0 >> lx) & (ncy - 1), cz = c0 >> (lx + ly);
  const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
  const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
  const int xw = ncx >= 3 && per ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
  int rb[kR], re[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int row = r >> 1, part = r & 1;
    const int oy = loy + row % 3, oz = loz + row / 3;
    const bool use = valid && oy <= hiy && oz <= hiz && (part == 0 || xw >= 0) &&
                     (per || (cy + oy >= 0 && cy + oy < ncy && cz + oz >= 0 && cz + oz < ncz));
    const int rowc = ((((cz + oz + ncz) & (ncz - 1)) << ly) | ((cy + oy + ncy) & (ncy - 1))) << lx;
    const int c_lo = rowc | (part == 0 ? xa : xw), c_hi = rowc | (part == 0 ? xb : xw);
    rb[r] = use ? cs[c_lo] : 0;
    re[r] = use ? cs[c_hi + 1] : 0;
  }
  __syncthreads();  // nb2
  const float* nb2_row = nb2 + (pk >> 24) * kMaxSpecies;
  int found = 0;
  uint32_t keep[kKeep];
#pragma unroll
  for (int v = 0; v < kKeep; ++v) keep[v] = 0u;
  // separation of sorted entry jj (particle j) from this particle: minimum
  // image, or the unwrapped difference in a non-periodic box
  auto sep = [&](uint32_t xj, uint32_t yj, uint32_t zj, int j, float* rx, float* ry, float* rz) {
    if (per) {
      *rx = (float)(int32_t)(xj - qx) * sx0;
      *ry = (float)(int32_t)(yj - qy) * sx1;
      *rz = (float)(int32_t)(zj - qz) * sx2;
    } else {
      *rx = pair_disp(xj, st.img[base + j], qx, ix, sx0, false);
      *ry = pair_disp(yj, st.img[M + base + j], qy, iy, sx1, false);
      *rz = pair_disp(zj, st.img[2 * M + base + j], qz, iz, sx2, false);
    }
  };
  auto near = [&](int jj, int packed) {
    float rx, ry, rz;
    sep(sc.bsq[base + jj], sc.bsq[M + base + jj], sc.bsq[2 * M + base + jj], packed & 0xffffff,
        &rx, &ry, &rz);
    float r2 = rx * rx + ry * ry;
    r2 = r2 + rz * rz;
    return i < (packed & 0xffffff) && r2 < nb2_row[packed >> 24];
  };
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    for (int jj0 = rb[r]; jj0 < re[r]; jj0 += 4) {
      int pk4[4];
      uint32_t x4[4], y4[4], z4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int jj = jj0 + u;
        const bool ok = jj < re[r];
        pk4[u] = ok ? sc.bsid[base + jj] : -1;
        x4[u] = ok ? sc.bsq[base + jj] : 0u;
        y4[u] = ok ? sc.bsq[M + base + jj] : 0u;
        z4[u] = ok ? sc.bsq[2 * M + base + jj] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (pk4[u] < 0) continue;
        const int j = pk4[u] & 0xffffff;
        float rx, ry, rz;
        sep(x4[u], y4[u], z4[u], j, &rx, &ry, &rz);
        float r2 = rx * rx + ry * ry;
        r2 = r2 + rz * rz;
        if (i < j && r2 < nb2_row[pk4[u] >> 24]) {
#pragma unroll
          for (int v = 0; v < kKeep; ++v) keep[v] = found == v ? (uint32_t)j : keep[v];
          ++found;
        }
      }
    }
  }
  const int lane = threadIdx.x & 63;
  int v = found;
  v = wave_incl_scan(v);
  int wbase = 0;
  if (lane == 63) wbase = atomicAdd(&sc.gnpairs[e], v);
  wbase = __builtin_amdgcn_readlane(wbase, 63);
  const int my_off = wbase + v - found;
  uint32_t* out = sc.gplist + (size_t)e * sc.pair_cap;
  if (!__any(found > kKeep)) {
#pragma unroll
    for (int u = 0; u < kKeep; ++u) {
      const int k = my_off + u;
      if (u < found && k < sc.pair_cap) out[k] = (uint32_t)i | (keep[u] << 16);
    }
    return;
  }
  // a lane found more than kKeep pairs: rescan and write in order
  int w = 0;
  for (int r = 0; r < kR; ++r) {
    for (int jj = rb[r]; jj < re[r]; ++jj) {
      const int packed = sc.bsid[base + jj];
      if (near(jj, packed)) {
        const int k = my_off + w;
        if (k < sc.pair_cap) out[k] = (uint32_t)i | ((uint32_t)(packed & 0xffffff) << 16);
        ++w;
      }
    }
  }
}

// Branch-free pair_force3 for the run kernel's pair passes (pair_fix_sel
// with a third component): the force on the first particle in 2^-24 fixed
// point, zero out of range or for an empty slot (r2 = 0).
__device__ __forceinline__ void pair_fix_sel3(float cut2, float sig6, float eps24, float rx,
                                              float ry, float rz, int64_t& fx, int64_t& fy,
                                              int64_t& fz) {
  float r2 = rx * rx + ry * ry;
  r2 = r2 + rz * rz;
  const bool in = r2 < cut2 && r2 > 0.0f;
  const float ir2 = rcp_rn(in ? r2 : 1.0f);  // = 1.0f / r2 (in range: r2 >= 2^-96)
  float ir6 = ir2 * ir2;
  ir6 = ir6 * ir2;
  const float s6 = sig6 * ir6;
  float t = 2.0f * s6;
  t = t - 1.0f;
  float fr = eps24 * s6;
  fr = fr * t;
  fr = fr * ir2;
  const float vx = (in ? -fr * rx : 0.0f) * 16777216.0f;
  const float vy = (in ? -fr * ry : 0.0f) * 16777216.0f;
  const float vz = (in ? -fr * rz : 0.0f) * 16777216.0f;
  if (__builtin_expect(wave_all(fabsf(vx) < 2147483520.0f && fabsf(vy) < 2147483520.0f &&
                             fabsf(vz) < 2147483520.0f),
                       1)) {
    fx = (int64_t)__float2int_rn(vx);
    fy = (int64_t)__float2int_rn(vy);
    fz = (int64_t)__float2int_rn(vz);
  } else {
    constexpr float kLim = 4.611686018427387904e18f;
    fx = __float2ll_rn(fminf(fmaxf(vx, -kLim), kLim));
    fy = __float2ll_rn(fminf(fmaxf(vy, -kLim), kLim));
    fz = __float2ll_rn(fminf(fmaxf(vz, -kLim), kLim));
  }
}

// One wave of the 3-D cluster run: all n_steps sub-steps of the particles
// in its 64 slots (lane = particle), the wave's neighbour pairs one per lane
// and pass, positions exchanged through the wave's LDS row, force sums as
// int64 LDS atomics (order-free, so the bits of block_global_run3).  The
// update is block_global_run3's sequence: translation from F = WCA + walls +
// f_ext + f_swim * director, then the Rodrigues turn of the director; the
// turn does not depend on the forces, so it is computed while the force sums
// are in flight.  Normals are drawn here (translation: StepNoise, the
// step_normals numbers; rotation: normals3 tag 2).
template <bool kMulti, bool kWalls>
__device__ __forceinline__ void run_wave3(const Derived* __restrict__ d, const DevState& st,
                                          const Scratch& sc, int n_envs, int n_steps,
                                          uint64_t step0, int gw, int lane, uint4* lpos_w,
                                          unsigned long long* lacc_x, unsigned long long* lacc_y,
                                          unsigned long long* lacc_z, const PairTables& pt,
                                          int par) {
  const int e = gw / sc.wmax;
  const int w = gw - e * sc.wmax;
  if (e >= n_envs) return;
  if (sc.fallback[e] != 0 || w >= sc.env_waves[e]) return;
  const int N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int slot = w * 64 + lane;
  const int i = sc.perm[(size_t)e * sc.S + slot];
  const bool active = i >= 0;
  const size_t gi = base + (active ? i : 0);
  const int si = kMulti ? st.species[active ? i : 0] : 0;
  uint32_t q[3];
  int32_t im[3];
  float v[3], vs0[3], fex[3], tq[3];
  float fs;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    q[a] = st.q[a * M + gi];
    im[a] = st.img[a * M + gi];
    v[a] = st.dir3[a * M + gi];
    fex[a] = st.f_ext[a * M + gi];
  }
  {
    // sub-step 0's swim force, torque and swim direction: with
    // reuse_forces the previous run's (the current ones load after it)
    const PrevSlot prv = prev_slot(st, par);
    fs = st.reuse ? prv.f[gi] : st.f_swim[gi];
    tq[0] = st.reuse ? prv.txy[gi] : st.torque_xy[gi];
    tq[1] = st.reuse ? prv.txy[M + gi] : st.torque_xy[M + gi];
    tq[2] = st.reuse ? prv.tz[gi] : st.torque_z[gi];
#pragma unroll
    for (int a = 0; a < 3; ++a) vs0[a] = st.reuse ? prv.dir3[a * M + gi] : v[a];
  }
  if (active) {  // window-start snapshot (k_check3's exact test and re-run)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      sc.bq[a * M + gi] = q[a];
      sc.bimg[a * M + gi] = im[a];
      sc.bdir3[a * M + gi] = v[a];
    }
  }
  const int np = sc.wave_npairs[(size_t)e * sc.wmax + w];
  const int npass = (np + 63) >> 6;
  const uint32_t* pw = sc.pairs + ((size_t)e * sc.wmax + w) * kPairsPerWave;
  const uint32_t pr0 = lane < np ? pw[lane] : 0xffffffffu;
  lacc_x[lane] = 0ull;
  lacc_y[lane] = 0ull;
  lacc_z[lane] = 0ull;
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx[3] = {d->sx[0], d->sx[1], d->sx[2]};
  const float isx[3] = {d->inv_sx[0], d->inv_sx[1], d->inv_sx[2]};
  const float eps24 = d->eps24;
  const bool noisy = d->noisy != 0;
  const float mob_dt = d->mob_dt[si], sig_t = d->sig_t[si], rot_dt = d->rot_dt[si],
              sig_r = d->sig_r[si];
  const float cut2_0 = d->cut2[0], sig6_0 = d->sig6[0];
  const uint32_t q0[3] = {q[0], q[1], q[2]};
  float dmax2 = 0.0f;
  StepNoise noise;
  auto substep = [&](const int s, auto first_t, auto last_t, auto pass_t)
                     __attribute__((always_inline)) {
    constexpr bool kFirst = decltype(first_t)::value;
    constexpr bool kLast = decltype(last_t)::value;
    constexpr int kPass = decltype(pass_t)::value;  // 0, 1, or 4: up to npass
    const uint64_t step = step0 + (uint64_t)s;
    float gt[3] = {0.0f, 0.0f, 0.0f}, gr[3] = {0.0f, 0.0f, 0.0f};
    if (noisy) {
      noise.next(k0, k1, (uint32_t)i, step, kFirst, gt);
      normals3(k0, k1, (uint32_t)i, step, 2u, gr);
    }
    if (kPass > 0) {
      lpos_w[lane] = make_uint4(q[0], q[1], q[2], 0u);
      wave_lds_sync();
      for (int p = 0; p < (kPass == 1 ? 1 : npass); ++p) {
        const uint32_t e_ =
            p == 0 ? pr0 : (p * 64 + lane < np ? pw[p * 64 + lane] : 0xffffffffu);
        const int a = e_ == 0xffffffffu ? lane : (int)(e_ & 63u);
        const int b = e_ == 0xffffffffu ? lane : (int)((e_ >> 6) & 63u);
        const uint4 pa = lpos_w[a], pb = lpos_w[b];
        const float rx = (float)(int32_t)(pb.x - pa.x) * sx[0];
        const float ry = (float)(int32_t)(pb.y - pa.y) * sx[1];
        const float rz = (float)(int32_t)(pb.z - pa.z) * sx[2];
        int64_t fx, fy, fz;  // on a; b receives exactly the negation
        if (kMulti) {
          const int sp = (int)((e_ >> 12) & 255u);
          pair_fix_sel3(pt.cut2[sp], pt.sig6[sp], eps24, rx, ry, rz, fx, fy, fz);
        } else {
          pair_fix_sel3(cut2_0, sig6_0, eps24, rx, ry, rz, fx, fy, fz);
        }
        atomicAdd(&lacc_x[a], (unsigned long long)fx);
        atomicAdd(&lacc_y[a], (unsigned long long)fy);
        atomicAdd(&lacc_z[a], (unsigned long long)fz);
        atomicSub(&lacc_x[b], (unsigned long long)fx);
        atomicSub(&lacc_y[b], (unsigned long long)fy);
        atomicSub(&lacc_z[b], (unsigned long long)fz);
      }
    }
    // the director's turn (independent of the forces) while the sums land
    __builtin_amdgcn_sched_barrier(0);
    float ph[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ph[a] = tq[a] * rot_dt;
      if (noisy) ph[a] = ph[a] + sig_r * gr[a];
    }
    float vn[3] = {v[0], v[1], v[2]};
    rotate_director(vn, ph[0], ph[1], ph[2]);
    __builtin_amdgcn_sched_barrier(0);
    __asm__ volatile("" ::: "memory");
    int64_t acc[3] = {0, 0, 0};
    if (kPass > 0) {
      wave_lds_sync();
      acc[0] = (int64_t)lacc_x[lane];
      acc[1] = (int64_t)lacc_y[lane];
      acc[2] = (int64_t)lacc_z[lane];
      lacc_x[lane] = 0ull;
      lacc_y[lane] = 0ull;
      lacc_z[lane] = 0ull;
    }
    if (kWalls && active)
      wall_forces<3>(d, si, (float)q[0] * sx[0], (float)q[1] * sx[1], (float)q[2] * sx[2], acc[0],
                     acc[1], acc[2], st.wall_viol);
    float f[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      f[a] = i64_to_f32(acc[a]) * 5.9604644775390625e-08f;
      f[a] = f[a] + fex[a];
      f[a] = f[a] + fs * (kFirst ? vs0[a] : v[a]);
      float dq = f[a] * mob_dt;
      if (noisy) dq = dq + sig_t * gt[a];
      advance(q[a], im[a], f2i32(dq * isx[a]));
    }
    if (kLast && active) {  // velocities of the last sub-step
      const float inv_gt = d->inv_gt[si], inv_gr = d->inv_gr[si];
      float vv[3], ww[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        vv[a] = f[a] * inv_gt;
        ww[a] = tq[a] * inv_gr;
      }
      if (noisy) {
        float gv[3], gw[3];
        normals3(k0, k1, (uint32_t)i, step, 1u, gv);
        normals3(k0, k1, (uint32_t)i, step, 3u, gw);
        const float sig_v = d->sig_v[si], sig_w = d->sig_w[si];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          vv[a] = vv[a] + sig_v * gv[a];
          ww[a] = ww[a] + sig_w * gw[a];
        }
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) st.vel[a * M + gi] = vv[a];
      st.omega_xy[gi] = ww[0];
      st.omega_xy[M + gi] = ww[1];
      st.omega[gi] = ww[2];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) v[a] = vn[a];
    float dd[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) dd[a] = (float)(int32_t)(q[a] - q0[a]) * sx[a];
    float d2 = dd[0] * dd[0] + dd[1] * dd[1];
    d2 = d2 + dd[2] * dd[2];
    dmax2 = fmaxf(dmax2, d2);
  };
  auto run_steps = [&](auto pass_t) __attribute__((always_inline)) {
    if (n_steps == 1) {
      substep(0, std::true_type{}, std::true_type{}, pass_t);
      return;
    }
    substep(0, std::true_type{}, std::false_type{}, pass_t);
    if (st.reuse) {  // this run's actions from sub-step 1 on
      fs = st.f_swim[gi];
      tq[0] = st.torque_xy[gi];
      tq[1] = st.torque_xy[M + gi];
      tq[2] = st.torque_z[gi];
    }
    int s = 1;
    for (; s < n_steps - 1; ++s) substep(s, std::false_type{}, std::false_type{}, pass_t);
    substep(s, std::false_type{}, std::true_type{}, pass_t);
  };
  if (npass == 0)
    run_steps(std::integral_constant<int, 0>{});
  else if (npass == 1)
    run_steps(std::integral_constant<int, 1>{});
  else
    run_steps(std::integral_constant<int, 4>{});
  if (active) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      st.q[a * M + gi] = q[a];
      st.img[a * M + gi] = im[a];
      st.dir3[a * M + gi] = v[a];
    }
    const float disp = sqrt_rn(dmax2);
    sc.disp[gi] = disp;
    if (!(disp < 0.5f * d->skin)) {  // a mover (k_check3's exact test)
      const int k = atomicAdd(&sc.nmov[e], 1);
      if (k < kMaxMovers) sc.movers[(size_t)e * kMaxMovers + k] = i;
    }
    if (st.reuse) {  // the next window's sub-step 0 (the other slot)
      // (fs, tq hold this run's actions unless the window was one sub-step)
      const PrevSlot wsl = prev_slot(st, par ^ 1);
      const bool one = n_steps == 1;
      wsl.f[gi] = one ? st.f_swim[gi] : fs;
      wsl.tz[gi] = one ? st.torque_z[gi] : tq[2];
      wsl.txy[gi] = one ? st.torque_xy[gi] : tq[0];
      wsl.txy[M + gi] = one ? st.torque_xy[M + gi] : tq[1];
#pragma unroll
      for (int a = 0; a < 3; ++a) wsl.dir3[a * M + gi] = v[a];
    }
  }
}

// 3-D cluster run: 64 or 256 threads per block (one wave per CU for
// latency-bound windows, four otherwise), one wave per 64 slots.
template <bool kMulti, bool kWalls>
__global__ __launch_bounds__(256) void k_cluster_run3(const Derived* __restrict__ d, DevState st,
                                                      Scratch sc, int n_envs, int n_steps,
                                                      const uint64_t* __restrict__ ctl) {
  __shared__ PairTables pt;
  __shared__ uint4 lpos[4][64];
  __shared__ unsigned long long lacc[4][3][64];
  stage_pair_tables(d, &pt);
  const int par = window_parity(ctl);
  const uint64_t step0 = ctl[kCtlStep];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  run_wave3<kMulti, kWalls>(d, st, sc, n_envs, n_steps, step0, gw, lane, lpos[wv], lacc[wv][0],
                            lacc[wv][1], lacc[wv][2], pt, par);
}

// 3-D check, one workgroup per env: k_check's exact validity test of the
// window (every mover against every colloid at the window-start positions,
// d0 < rc + D_i + D_j only for listed neighbour pairs) in three dimensions;
// a failed window (or one the build flagged: overflow, or any cluster wider
// than a wave) is re-run from the snapshot on the 3-D global path.
// LDS: 16 + 16 + kMaxMovers words, then the global path's cell counts.
__global__ __launch_bounds__(1024) void k_check3(const Derived* __restrict__ d, DevState st,
                                                 Scratch sc, int n_steps,
                                                 uint64_t* __restrict__ step_ctr,
                                                 uint32_t* __restrict__ arrive, int lx, int ly,
                                                 int lz, int nlist) {
  extern __shared__ __align__(16) unsigned char smem[];
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);  // 16
  int32_t* misc = wave_sums + 16;                          // 16
  int32_t* movers = misc + 16;                             // kMaxMovers
  int32_t* cnt = movers + kMaxMovers;                      // global-path cell counts
  __shared__ PairTables pt;
  stage_pair_tables(d, &pt);
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const uint64_t step0 = step_ctr[kCtlStep];
  const int par = window_parity(step_ctr);
  if (tid < 16) misc[tid] = 0;
  __syncthreads();
  // flagged by the build: the env did not run (its state is the window start)
  const bool flagged_build = sc.fallback[e] == 1;
  if (!flagged_build) {
    const int nm = sc.nmov[e];
    for (int k = tid; k < min(nm, kMaxMovers); k += T) movers[k] = sc.movers[(size_t)e * kMaxMovers + k];
    __syncthreads();
    if (nm > kMaxMovers) {
      if (tid == 0) misc[1] = 1;
    } else if (nm > 0) {
      const bool multi = d->n_species > 1;  // else every pair's cutoff is cut2[0]
      const float rc0 = sqrtf(pt.cut2[0]);
      const float sx0 = d->sx[0], sx1 = d->sx[1], sx2 = d->sx[2];
      const bool per = d->periodic != 0;
      const long total = (long)nm * N;
      for (long t = tid; t < total; t += T) {
        const int m = movers[t / N];
        const int j = (int)(t % N);
        if (j == m) continue;
        // window-start separation: minimum image, or (non-periodic box) the
        // unwrapped difference -- the folded one would only be stricter
        const float rx = pair_disp(sc.bq[base + j], sc.bimg[base + j], sc.bq[base + m],
                                   sc.bimg[base + m], sx0, per);
        const float ry = pair_disp(sc.bq[M + base + j], sc.bimg[M + base + j], sc.bq[M + base + m],
                                   sc.bimg[M + base + m], sx1, per);
        const float rz = pair_disp(sc.bq[2 * M + base + j], sc.bimg[2 * M + base + j],
                                   sc.bq[2 * M + base + m], sc.bimg[2 * M + base + m], sx2, per);
        // the pair's own WCA cutoff r_m + r_j (not the largest one: a dense
        // mixture would fail the test for pairs that cannot interact)
        const float rc = multi ? sqrtf(pt.cut2[st.species[m] * kMaxSpecies + st.species[j]]) : rc0;
        const float lim = rc + sc.disp[base + m] + sc.disp[base + j] + 1e-3f;
        float r2 = rx * rx + ry * ry;
        r2 = r2 + rz * rz;
        if (r2 < lim * lim) {
          bool listed = false;
          if (nlist) {  // j among m's listed neighbours
            const int nn = sc.nn[base + m];
            for (int k = 0; k < nn; ++k)
              listed |= (sc.nl[(size_t)k * M + base + m] & 0xffffff) == j;
          } else if (sc.root[base + j] == sc.root[base + m]) {  // same wave: its pairs
            const int sm = sc.slot_of[base + m], sj = sc.slot_of[base + j];
            const int wv = sm >> 6;
            const uint32_t lm = (uint32_t)(sm & 63), lj = (uint32_t)(sj & 63);
            const uint32_t* pw = sc.pairs + ((size_t)e * sc.wmax + wv) * kPairsPerWave;
            const int np = sc.wave_npairs[(size_t)e * sc.wmax + wv];
            for (int k = 0; k < np; ++k) {
              const uint32_t a = pw[k] & 63u, b = (pw[k] >> 6) & 63u;
              listed |= (a == lm && b == lj) || (a == lj && b == lm);
            }
          }
          if (!listed) misc[1] = 1;
        }
      }
    }
    __syncthreads();
  }
  if (flagged_build || misc[1] != 0) {
    for (int i = tid; i < N && !flagged_build; i += T) {
      const size_t gi = base + i;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        st.q[a * M + gi] = sc.bq[a * M + gi];
        st.img[a * M + gi] = sc.bimg[a * M + gi];
        st.dir3[a * M + gi] = sc.bdir3[a * M + gi];
      }
    }
    if (tid == 0) sc.fallback[e] = 2;  // diagnostics: env re-run on the global path
    __syncthreads();
    block_global_run3(d, st, sc, e, n_steps, step0, lx, ly, lz, false, 0.0f, 0.0f, cnt, wave_sums,
                      &pt, par);
    save_forces_env(st, e, par ^ 1);  // the re-run replaced the run kernel's final state
  }
  __syncthreads();  // every read of nmov above is done
  if (tid == 0) sc.nmov[e] = 0;
  advance_counter(step_ctr, arrive, step0, n_steps);
}


// ------------------------------------------- 3-D neighbour-list window
// Dense boxes (the rc + skin graph percolates: most colloids in clusters
// wider than a wave) cannot be cut into per-wave clusters.  There the window
// keeps the same build grid, exact check and re-run, but the sub-steps run
// chip-wide: a Verlet list (every j within r_i + r_j + skin) per colloid,
// then one launch per sub-step with one thread per colloid, reading the
// positions of sub-step s from one buffer and writing the other (st.q and
// sc.qalt alternate; k_check3 copies back after an odd window).  Forces,
// noise and update are block_global_run3's, so the bits are the same.

// Build step 2 (neighbour-list path), grid (ceil(N / 256), E), one thread
// per sorted entry: its neighbours into nl[k][gi] (neighbour-major, so the
// sub-step's reads coalesce).
__global__ __launch_bounds__(256) void k_build_nlist3(const Derived* __restrict__ d, DevState st,
                                                      Scratch sc, int lx, int ly, int lz) {
  constexpr int kR = 18;
  __shared__ float nb2[kMaxSpecies * kMaxSpecies];
  for (int k = threadIdx.x; k < kMaxSpecies * kMaxSpecies; k += blockDim.x) nb2[k] = d->nb2[k];
  __syncthreads();
  const int e = blockIdx.y, N = st.n;
  const int ps = blockIdx.x * blockDim.x + threadIdx.x;
  if (ps >= N) return;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly + lz);
  const int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  const int ncx = 1 << lx, ncy = 1 << ly, ncz = 1 << lz;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const int loz = ncz >= 3 ? -1 : 0, hiz = ncz >= 3 ? 1 : ncz - 1;
  const float sx0 = d->sx[0], sx1 = d->sx[1], sx2 = d->sx[2];
  const int pk = sc.bsid[base + ps];
  const int i = pk & 0xffffff;
  const uint32_t qx = sc.bsq[base + ps], qy = sc.bsq[M + base + ps], qz = sc.bsq[2 * M + base + ps];
  const int c0 = cell_index3(qx, qy, qz, lx, ly, lz);
  const int cx = c0 & (ncx - 1), cy = (c0 >> lx) & (ncy - 1), cz = c0 >> (lx + ly);
  const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
  const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
  const int xw = ncx >= 3 ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
  int rb[kR], re[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int row = r >> 1, part = r & 1;
    const int oy = loy + row % 3, oz = loz + row / 3;
    const bool use = oy <= hiy && oz <= hiz && (part == 0 || xw >= 0);
    const int rowc = ((((cz + oz + ncz) & (ncz - 1)) << ly) | ((cy + oy + ncy) & (ncy - 1))) << lx;
    const int c_lo = rowc | (part == 0 ? xa : xw), c_hi = rowc | (part == 0 ? xb : xw);
    rb[r] = use ? cs[c_lo] : 0;
    re[r] = use ? cs[c_hi + 1] : 0;
  }
  const float* nb2_row = nb2 + (pk >> 24) * kMaxSpecies;
  int cnt = 0;
  int32_t* out = sc.nl + base + i;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    for (int jj0 = rb[r]; jj0 < re[r]; jj0 += 4) {
      int pk4[4];
      uint32_t x4[4], y4[4], z4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int jj = jj0 + u;
        const bool ok = jj < re[r];
        pk4[u] = ok ? sc.bsid[base + jj] : -1;
        x4[u] = ok ? sc.bsq[base + jj] : 0u;
        y4[u] = ok ? sc.bsq[M + base + jj] : 0u;
        z4[u] = ok ? sc.bsq[2 * M + base + jj] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (pk4[u] < 0 || (pk4[u] & 0xffffff) == i) continue;
        const float rx = (float)(int32_t)(x4[u] - qx) * sx0;
        const float ry = (float)(int32_t)(y4[u] - qy) * sx1;
        const float rz = (float)(int32_t)(z4[u] - qz) * sx2;
        float r2 = rx * rx + ry * ry;
        r2 = r2 + rz * rz;
        if (r2 < nb2_row[pk4[u] >> 24]) {
          if (cnt < kNlMax) out[(size_t)cnt * M] = pk4[u];
          ++cnt;
        }
      }
    }
  }
  sc.nn[base + i] = min(cnt, kNlMax);
  sc.qa[base + i] = make_uint4(qx, qy, qz, 0u);  // sub-step 0's read buffer
  if (cnt > kNlMax) sc.fallback[e] = 1;  // -> the env re-runs on the global path
}

// Sub-step s of the neighbour-list window, one thread per colloid of every
// env: block_global_run3's force sum (over the listed neighbours: pairs
// beyond them cannot be in range while k_check3's test holds) and update.
// Positions ping-pong between two AoS buffers (one 16-B load per
// neighbour): sub-step s reads qa[s & 1] (the build filled qa[0]) and writes
// the other; the last sub-step writes st.q.  Image counters and directors
// are the colloid's own and update in place.
// sc.disp holds the squared maximum displacement until the last sub-step.
template <bool kMulti, bool kWalls>
__global__ __launch_bounds__(256) void k_nl_step3(const Derived* __restrict__ d, DevState st,
                                                  Scratch sc, int n_steps, int s,
                                                  const uint64_t* __restrict__ ctl) {
  __shared__ PairTables pt;
  if (kMulti) stage_pair_tables(d, &pt);
  const size_t M = (size_t)st.m;
  // XCD-aware order: workgroup b runs on XCD b % 8, so consecutive logical
  // blocks (one env's colloids, whose positions the neighbour reads share)
  // go to the same XCD and its L2 (grid: a multiple of 8 blocks)
  const unsigned per_xcd = gridDim.x >> 3;
  const unsigned lb = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
  const size_t gi = (size_t)lb * blockDim.x + threadIdx.x;
  if (gi >= M) return;
  const int N = st.n;
  const int e = (int)(gi / N), i = (int)(gi - (size_t)e * N);
  if (sc.fallback[e] != 0) return;
  const size_t base = (size_t)e * N;
  const bool first = s == 0, last = s == n_steps - 1;
  const uint4* R = sc.qa + (s & 1) * M;
  uint4* W = sc.qa + ((s & 1) ^ 1) * M;
  const int par = window_parity(ctl);
  const uint64_t step = ctl[kCtlStep] + (uint64_t)s;
  const int si = kMulti ? st.species[i] : 0;
  const float sx[3] = {d->sx[0], d->sx[1], d->sx[2]};
  uint32_t q[3], q0[3];
  int32_t im[3];
  float v[3];
  // issue every own load first: one memory latency
  const int nn = sc.nn[gi];
  const uint4 qo = R[gi];
  q[0] = qo.x;
  q[1] = qo.y;
  q[2] = qo.z;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    im[a] = st.img[a * M + gi];
    v[a] = st.dir3[a * M + gi];
  }
  float dmax2 = 0.0f;
  if (first) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      q0[a] = q[a];
      sc.bq[a * M + gi] = q[a];
      sc.bimg[a * M + gi] = im[a];
      sc.bdir3[a * M + gi] = v[a];
    }
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) q0[a] = sc.bq[a * M + gi];
    dmax2 = sc.disp[gi];
  }
  const bool reuse0 = st.reuse && first;  // sub-step 0 reuses the previous run's actions
  const PrevSlot prv = prev_slot(st, par);
  const float fs = reuse0 ? prv.f[gi] : st.f_swim[gi];
  const float tq[3] = {reuse0 ? prv.txy[gi] : st.torque_xy[gi],
                       reuse0 ? prv.txy[M + gi] : st.torque_xy[M + gi],
                       reuse0 ? prv.tz[gi] : st.torque_z[gi]};
  float vs[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) vs[a] = reuse0 ? prv.dir3[a * M + gi] : v[a];
  const float eps24 = d->eps24;
  int64_t acc[3] = {0, 0, 0};
  const int32_t* nlp = sc.nl + gi;
  for (int k0 = 0; k0 < nn; k0 += 8) {
    // eight neighbours per round: their indices, then their positions, in
    // flight together (two memory latencies per round)
    int32_t pk[8];
    uint4 qj[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pk[u] = k0 + u < nn ? nlp[(size_t)(k0 + u) * M] : -1;
#pragma unroll
    for (int u = 0; u < 8; ++u) qj[u] = R[base + (pk[u] < 0 ? i : (pk[u] & 0xffffff))];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (pk[u] < 0) continue;
      const float rx = (float)(int32_t)(qj[u].x - q[0]) * sx[0];
      const float ry = (float)(int32_t)(qj[u].y - q[1]) * sx[1];
      const float rz = (float)(int32_t)(qj[u].z - q[2]) * sx[2];
      if (kMulti) {
        const int sp = si * kMaxSpecies + (pk[u] >> 24);
        pair_force3(pt.cut2[sp], pt.sig6[sp], eps24, rx, ry, rz, acc[0], acc[1], acc[2]);
      } else {
        pair_force3(d->cut2[0], d->sig6[0], eps24, rx, ry, rz, acc[0], acc[1], acc[2]);
      }
    }
  }
  if (kWalls)
    wall_forces<3>(d, si, (float)q[0] * sx[0], (float)q[1] * sx[1], (float)q[2] * sx[2], acc[0],
                   acc[1], acc[2], st.wall_viol);
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const bool noisy = d->noisy != 0;
  float f[3], ph[3];
  float gt[3] = {0.0f, 0.0f, 0.0f}, gr[3] = {0.0f, 0.0f, 0.0f};
  if (noisy) {
    step_normals(k0, k1, (uint32_t)i, step, gt);
    normals3(k0, k1, (uint32_t)i, step, 2u, gr);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    f[a] = i64_to_f32(acc[a]) * 5.9604644775390625e-08f;
    f[a] = f[a] + st.f_ext[a * M + gi];
    f[a] = f[a] + fs * vs[a];
    float dq = f[a] * d->mob_dt[si];
    ph[a] = tq[a] * d->rot_dt[si];
    if (noisy) {
      dq = dq + d->sig_t[si] * gt[a];
      ph[a] = ph[a] + d->sig_r[si] * gr[a];
    }
    advance(q[a], im[a], f2i32(dq * d->inv_sx[a]));
  }
  rotate_director(v, ph[0], ph[1], ph[2]);
  if (last) {  // nobody reads st.q during the window
#pragma unroll
    for (int a = 0; a < 3; ++a) st.q[a * M + gi] = q[a];
  } else {
    W[gi] = make_uint4(q[0], q[1], q[2], 0u);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    st.img[a * M + gi] = im[a];
    st.dir3[a * M + gi] = v[a];
  }
  float dd[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) dd[a] = (float)(int32_t)(q[a] - q0[a]) * sx[a];
  float d2 = dd[0] * dd[0] + dd[1] * dd[1];
  d2 = d2 + dd[2] * dd[2];
  dmax2 = fmaxf(dmax2, d2);
  if (!last) {
    sc.disp[gi] = dmax2;
    return;
  }
  {  // velocities of the last sub-step (block_global_run3's sequence)
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
  const float disp = sqrt_rn(dmax2);
  sc.disp[gi] = disp;
  if (!(disp < 0.5f * d->skin)) {  // a mover (k_check3's exact test)
    const int k = atomicAdd(&sc.nmov[e], 1);
    if (k < kMaxMovers) sc.movers[(size_t)e * kMaxMovers + k] = i;
  }
  if (st.reuse) save_forces(st, gi, par ^ 1);  // this run's actions, the final director
}


}  // namespace swarm
