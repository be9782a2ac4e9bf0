// swarm_engine.hip -- MI355X (gfx950) active-Brownian swarm engine.
//
// Implements the C ABI of include/swarmrl_amd.h.  The per-step hot path of
// the reference (ESPResSo Brownian dynamics + WCA via a cell system, driven by
// swarmrl/engine/espresso.py:1251-1308) runs here as hand-written HIP:
//
//   integrator      swarm_integrator.cuh: per window k_cluster_build ->
//                   k_cluster_run -> k_check (cluster-parallel Brownian
//                   dynamics + WCA, exact fallback to the global path);
//                   k_global also runs steepest descent (espresso.py:1161-1168).
//   k_grid_build    per-env cell list in global memory (for the observables).
//   k_vision        SubdividedVisionCones, one thread per (env, agent).
//   k_field         ConcentrationField / GradientSensing distances + history.
//   k_pairs         neighbour pairs (parity helper).
//
// Number formats: positions are uint32 box fractions + int32
// image counters, angles uint32 turn fractions, pair sums int64 fixed point,
// so results are independent of neighbour order and bit-identical to the
// CPU oracle.  Compile with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/swarmrl_amd.h"
#include "swarm_device.cuh"
#include "swarm_integrator.cuh"
#include "swarm_integrator3.cuh"
#include "swarm_policy.cuh"
#include "swarm_ppo.cuh"
#include "swarm_rnd.cuh"

namespace {

using swarm::Derived;
using swarm::DevState;
using swarm::Scratch;
using swarm::cell_index;
using swarm::block_exclusive_scan;

// Cell-sorted 32-byte record of one particle for the observables, read as
// two 16-byte loads: {qx, qy, ix, iy}, {radius bits, particle, type slot, 0}.
struct VisionSorted {
  uint4* rec;          // [E * N][2]
  int32_t* agent_row;  // [N] row of a particle in the agent list, -1 if none
};

constexpr int kMaxSpecies = SWARM_MAX_SPECIES;
constexpr double kTwo32 = 4294967296.0;
constexpr double kTwoPi = 6.283185307179586476925;
// Verlet skin of the cluster decomposition (um): pairs closer than
// r_i + r_j + skin at the window start share a cluster.  Performance only:
// results do not depend on it.  2 um keeps inter-cluster approaches below
// the cutoff over a 100-step slice a ~5-sigma event at the reference's
// defaults.
double skin_um() { return 2.0; }

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess)                                                    \
      return fail(SWARM_EDEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

void derive(const swarm_params_t& p, Derived& d) {
  std::memset(&d, 0, sizeof(d));
  for (int a = 0; a < 3; ++a) {
    d.sx[a] = (float)(p.box[a] / kTwo32);
    d.inv_sx[a] = (float)(kTwo32 / p.box[a]);
  }
  const double kT = p.kT, dt = p.time_step;
  for (int s = 0; s < p.n_species; ++s) {
    const double gt = p.gamma_t[s], gr = p.gamma_r[s];
    d.mob_dt[s] = (float)(dt / gt);
    d.rot_dt[s] = (float)(dt / gr);
    d.sig_t[s] = (float)std::sqrt(2.0 * kT * dt / gt);
    d.sig_r[s] = (float)std::sqrt(2.0 * kT * dt / gr);
    d.inv_gt[s] = (float)(1.0 / gt);
    d.inv_gr[s] = (float)(1.0 / gr);
    d.sig_v[s] = p.mass[s] > 0.0 ? (float)std::sqrt(kT / p.mass[s]) : 0.0f;
    d.sig_w[s] = p.rinertia[s] > 0.0 ? (float)std::sqrt(kT / p.rinertia[s]) : 0.0f;
  }
  d.rc_max = 0.0;
  for (int s = 0; s < p.n_species; ++s)
    for (int t = 0; t < p.n_species; ++t) {
      const double rc = p.radius[s] + p.radius[t];
      const double rc2 = rc * rc;
      d.cut2[s * kMaxSpecies + t] = (float)rc2;
      d.sig6[s * kMaxSpecies + t] = (float)(rc2 * rc2 * rc2 * 0.5);
      d.rc_max = std::max(d.rc_max, rc);
    }
  for (int s = 0; s < p.n_species; ++s)
    for (int t = 0; t < p.n_species; ++t) {
      const double r = p.radius[s] + p.radius[t] + skin_um();
      d.nb2[s * kMaxSpecies + t] = (float)(r * r);
    }
  d.skin = (float)skin_um();
  d.rc_max_f = (float)d.rc_max;
  d.eps24 = (float)(24.0 * p.wca_epsilon);
  d.n_species = p.n_species;
  d.key0 = (uint32_t)p.seed;
  d.key1 = (uint32_t)(p.seed >> 32);
  d.noisy = p.kT > 0.0 ? 1 : 0;
  d.periodic = p.periodic;
  for (int s = 0; s < p.n_species; ++s) {  // walls: WCA with a radius-0 wall type
    const double rc2 = p.radius[s] * p.radius[s];
    d.wcut2[s] = (float)rc2;
    d.wsig6[s] = (float)(rc2 * rc2 * rc2 * 0.5);
  }
}

int ilog2_floor(double v) {
  int l = 0;
  while ((double)(1 << (l + 1)) <= v && l < 20) ++l;
  return l;
}

// Power-of-two cell grid with side >= cutoff and at most max(n, 64) cells
// (identical rule in oracle/swarm_oracle.c:or_cell_grid).
void cell_grid(const swarm_params_t& p, int n, double cutoff, int* lx, int* ly) {
  int l[2];
  for (int a = 0; a < 2; ++a) {
    const double m = cutoff > 0.0 ? p.box[a] / cutoff : 1024.0;
    l[a] = m >= 1.0 ? ilog2_floor(m) : 0;
    if (l[a] > 15) l[a] = 15;
  }
  const int cap = n > 64 ? n : 64;
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

// 3-D: the same rule over three axes (3-D global path).
void cell_grid3(const swarm_params_t& p, int n, double cutoff, int* lx, int* ly, int* lz) {
  int l[3];
  for (int a = 0; a < 3; ++a) {
    const double m = cutoff > 0.0 ? p.box[a] / cutoff : 1024.0;
    l[a] = m >= 1.0 ? ilog2_floor(m) : 0;
    if (l[a] > 10) l[a] = 10;
  }
  const int cap = std::min(n > 64 ? n : 64, 8192);  // counts fit the default 64 KB of LDS
  while ((1 << (l[0] + l[1] + l[2])) > cap) {
    int k = 0;
    for (int a = 1; a < 3; ++a)
      if (l[a] > l[k]) k = a;
    if (l[k] == 0) break;
    l[k]--;
  }
  *lx = l[0];
  *ly = l[1];
  *lz = l[2];
}

// ------------------------------------------------- global per-env grid
// Counting sort of every env into cells (side >= cutoff), written to global
// memory: start[E][ncell+1], sorted particle index order[E][N].
__global__ __launch_bounds__(1024) void k_grid_build(DevState st, int lx, int ly,
                                                     int32_t* __restrict__ start,
                                                     int32_t* __restrict__ order) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x, N = st.n;
  const int ncell = 1 << (lx + ly);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
  __syncthreads();
  const size_t M = (size_t)st.m;
  for (int i = tid; i < N; i += T) {
    const size_t g = (size_t)e * N + i;
    atomicAdd(&cnt[cell_index(st.q[g], st.q[M + g], lx, ly)], 1);
  }
  __syncthreads();
  block_exclusive_scan(cnt, ncell, wave_sums);
  __syncthreads();
  int32_t* so = start + (size_t)e * (ncell + 1);
  for (int c = tid; c <= ncell; c += T) so[c] = cnt[c];
  __syncthreads();
  for (int i = tid; i < N; i += T) {
    const size_t g = (size_t)e * N + i;
    const int pos = atomicAdd(&cnt[cell_index(st.q[g], st.q[M + g], lx, ly)], 1);
    order[(size_t)e * N + pos] = i;
  }
}

// Vision records (cell-sorted, 2 x uint4 per colloid):
//   {q_x, q_y, img_x, img_y}, {radius bits, id | (type slot + 1) << 24, angle, 0}
// (type slot -1: a type the observable does not detect).  The angle rides
// along so an agent's director needs no dependent load.
__device__ __forceinline__ uint32_t vision_id_word(int i, int ti) {
  return (uint32_t)i | ((uint32_t)(ti + 1) << 24);
}
__device__ __forceinline__ int vision_rec_id(uint32_t w) { return (int)(w & 0xffffffu); }
__device__ __forceinline__ int vision_rec_type(uint32_t w) { return (int)(w >> 24) - 1; }

// Vision grid: counting sort of every env into cells of side >= vision range,
// writing cell-sorted records so a candidate cell is one contiguous run; the
// env-0 workgroup also inverts the agent list (agent_row).
// The vision-cone launch arguments (one struct, so fused launches carry it).
struct VisionArgs {
  swarm_vision_params_t vp;
  int lx, ly;
  const float* radii;
  const int32_t* types;
  const int32_t* agents;
  int n_agents;
  int32_t* start;
  VisionSorted vs;
  float* out;
  int n_envs;
  int staged;  // 1: the records are scattered into LDS, then written in order
  unsigned long long* rstamp;  // role stamps of the launch (profiling), or null
};

// LDS of the vision grid's workgroup: wave sums, cell counts and, staged,
// the env's 2 x uint4 records (host and device agree through va.staged).
inline size_t vision_grid_lds_bytes(int lx, int ly, int n, bool staged) {
  const size_t counts = (16 + ((size_t)1 << (lx + ly)) + 1) * 4;
  return staged ? ((counts + 15) & ~(size_t)15) + 32 * (size_t)n : counts;
}

// Body for the workgroup of env e (k_vision_grid, or k_vgrid_sort).
__device__ __forceinline__ void vision_grid_body(const DevState& st, const VisionArgs& va, int e,
                                                 unsigned char* smem) {
  const swarm_vision_params_t& vp = va.vp;
  const int lx = va.lx, ly = va.ly;
  const float* __restrict__ radii = va.radii;
  const int32_t* __restrict__ types = va.types;
  const int32_t* __restrict__ agents = va.agents;
  const int n_agents = va.n_agents;
  int32_t* __restrict__ start = va.start;
  const VisionSorted& vs = va.vs;
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const int ncell = 1 << (lx + ly);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
  if (e == 0)
    for (int i = tid; i < N; i += T) vs.agent_row[i] = -1;
  __syncthreads();
  if (e == 0) {  // agents' rows: their ids loaded together (one memory latency)
    constexpr int kA = 8;
    for (int a0 = tid; a0 < n_agents; a0 += kA * T) {
      int ag[kA];
#pragma unroll
      for (int u = 0; u < kA; ++u) ag[u] = a0 + u * T < n_agents ? agents[a0 + u * T] : -1;
#pragma unroll
      for (int u = 0; u < kA; ++u)
        if ((unsigned)ag[u] < (unsigned)N) vs.agent_row[ag[u]] = a0 + u * T;
    }
  }
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  int32_t* so = start + (size_t)e * (ncell + 1);
  constexpr int kPer = 8;  // colloids per thread kept in registers (N <= 8 T)
  if (N <= kPer * T) {
    // every colloid's record fields are loaded once, up front, so their
    // latency overlaps the count and the scan
    uint4 r0[kPer], r1[kPer];
    int cell[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = tid + k * T;
      if (i < N) {
        const size_t g = base + i;
        const uint32_t qx = st.q[g], qy = st.q[M + g];
        const int tj = types[i];
        int ti = -1;
        for (int tt = 0; tt < vp.n_types; ++tt)
          if (vp.detected_types[tt] == tj) ti = tt;
        r0[k] = make_uint4(qx, qy, (uint32_t)st.img[g], (uint32_t)st.img[M + g]);
        r1[k] = make_uint4(__float_as_uint(radii[i]), vision_id_word(i, ti), st.ang[g], 0u);
        cell[k] = cell_index(qx, qy, lx, ly);
        atomicAdd(&cnt[cell[k]], 1);
      }
    }
    __syncthreads();
    block_exclusive_scan(cnt, ncell, wave_sums);
    __syncthreads();
    for (int c = tid; c <= ncell; c += T) so[c] = cnt[c];
    __syncthreads();
    if (va.staged) {
      // scatter into LDS (16-byte aligned after the counts), then write the
      // records in order: coalesced stores instead of 2 N scattered ones
      uint4* lrec = reinterpret_cast<uint4*>(
          smem + (((16 + (size_t)ncell + 1) * 4 + 15) & ~(size_t)15));
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        if (tid + k * T < N) {
          const int pos = atomicAdd(&cnt[cell[k]], 1);
          lrec[2 * pos] = r0[k];
          lrec[2 * pos + 1] = r1[k];
        }
      }
      __syncthreads();
      uint4* grec = vs.rec + 2 * base;
      for (int p = tid; p < 2 * N; p += T) grec[p] = lrec[p];
      return;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (tid + k * T < N) {
        const size_t pos = base + atomicAdd(&cnt[cell[k]], 1);
        vs.rec[2 * pos] = r0[k];
        vs.rec[2 * pos + 1] = r1[k];
      }
    }
    return;
  }
  for (int i = tid; i < N; i += T)
    atomicAdd(&cnt[cell_index(st.q[base + i], st.q[M + base + i], lx, ly)], 1);
  __syncthreads();
  block_exclusive_scan(cnt, ncell, wave_sums);
  __syncthreads();
  for (int c = tid; c <= ncell; c += T) so[c] = cnt[c];
  __syncthreads();
  for (int i = tid; i < N; i += T) {
    const size_t g = base + i;
    const uint32_t qx = st.q[g], qy = st.q[M + g];
    const size_t pos = base + atomicAdd(&cnt[cell_index(qx, qy, lx, ly)], 1);
    const int tj = types[i];
    int ti = -1;
    for (int tt = 0; tt < vp.n_types; ++tt)
      if (vp.detected_types[tt] == tj) ti = tt;
    vs.rec[2 * pos] = make_uint4(qx, qy, (uint32_t)st.img[g], (uint32_t)st.img[M + g]);
    vs.rec[2 * pos + 1] = make_uint4(__float_as_uint(radii[i]), vision_id_word(i, ti), st.ang[g], 0u);
  }
}

__global__ __launch_bounds__(1024) void k_vision_grid(DevState st, VisionArgs va) {
  extern __shared__ __align__(16) unsigned char smem[];
  vision_grid_body(st, va, blockIdx.x, smem);
}

// ---------------------------------------------------------- vision cone
// One group of G lanes per cell-sorted particle (neighbouring groups share
// candidate cells, so their record loads coalesce); groups of particles
// that are not agents exit.  The candidates of the 3x3 cell stencil form one
// flat index range that the G lanes split.  Two phases, so that the lanes of
// a wave stay converged: a cheap range test over the candidates appends the
// hits to a per-lane list in LDS, and the cone arithmetic (sqrt, divisions,
// acos) then runs over the hits only, four at a time; a full list is drained
// early.  Each lane keeps NB bins (>= n_cones * n_types) of 2^-32
// fixed-point amplitude in registers, and the group adds them with
// xor-shuffles.  Integer sums make the result independent of G, of the
// visiting order and of the phase split.
constexpr int kVisionHits = 16;  // per-lane hit list (LDS, [kVisionHits][256])

struct VisionLane {
  uint32_t qxi, qyi;
  int32_t ixi, iyi;
  int i;
  float mx, my, sx0, sx1, R;
};

// The in-range test of one candidate record (shared by both phases).
// kAny: vision_range may reach half the box or more (the all-records scan):
// every unwrapped separation is converted from int64.
template <bool kAny = false>
__device__ __forceinline__ bool vision_offsets(const VisionLane& L, const uint4& c0, float* dx,
                                               float* dy) {
  const int64_t dqx = ((int64_t)((int32_t)c0.z - L.ixi) * (int64_t)4294967296LL) +
                      ((int64_t)c0.x - (int64_t)L.qxi);
  const int64_t dqy = ((int64_t)((int32_t)c0.w - L.iyi) * (int64_t)4294967296LL) +
                      ((int64_t)c0.y - (int64_t)L.qyi);
  if (kAny) {
    *dx = (float)dqx * L.sx0;
    *dy = (float)dqy * L.sx1;
  } else {
    // unwrapped separations beyond half a box are never within range
    // (vision_range < L/2): skip them and convert the rest from int32, whose
    // conversion is a single exact-rounding instruction.
    if (dqx < -2147483647LL || dqx > 2147483647LL || dqy < -2147483647LL ||
        dqy > 2147483647LL)
      return false;
    *dx = (float)(int32_t)dqx * L.sx0;
    *dy = (float)(int32_t)dqy * L.sx1;
  }
  const float dist2 = *dx * *dx + *dy * *dy;
  // conservative pre-test on dist^2 (the exact test is on the fp32 sqrt)
  return dist2 < L.R * L.R * 1.0001f && dist2 != 0.0f;
}

// Cheap pre-test for the candidate scan: the minimum-image separation (int32
// wrap of the fraction difference) in range.  A candidate that passes
// vision_offsets passes this one (its unwrapped separation fits int32 and so
// equals the wrapped one); vision_hit re-tests the listed ones exactly.
__device__ __forceinline__ bool vision_near(const VisionLane& L, const uint4& c0) {
  const float dx = (float)(int32_t)(c0.x - L.qxi) * L.sx0;
  const float dy = (float)(int32_t)(c0.y - L.qyi) * L.sx1;
  const float dist2 = dx * dx + dy * dy;
  return dist2 < L.R * L.R * 1.0001f && dist2 != 0.0f;
}

template <int NB, bool kAny = false>
__device__ __forceinline__ void vision_hit(const VisionLane& L, const swarm_vision_params_t& vp,
                                           const uint4& c0, const uint4& c1, int64_t* acc) {
  float dx, dy;
  if (!vision_offsets<kAny>(L, c0, &dx, &dy)) return;
  const int ti = vision_rec_type(c1.y);
  if (ti < 0 || vision_rec_id(c1.y) == L.i) return;
  // (dist^2 >= sx0^2 ~ 1e-14: positive and normal, no special cases)
  const float dist = swarm::sqrt_pos(dx * dx + dy * dy);
  if (!(dist < L.R)) return;
  float amp = (2.0f * __uint_as_float(c1.x)) / dist;
  amp = fminf(1.0f, amp);
  const float ux = dx / dist, uy = dy / dist;
  float dot = ux * L.mx + uy * L.my;
  dot = fminf(fmaxf(dot, -1.0f), 1.0f);
  float an = swarm::acosf_fixed(dot);
  const float orth = ux * (-L.my) + uy * L.mx;
  if (orth < 0.0f) an = -an;
  const int64_t fixed = __float2ll_rn(amp * 4294967296.0f);
  int bin = -1;
  for (int k = 0; k < vp.n_cones; ++k)
    if (vp.rims[k] < an && an < vp.rims[k + 1]) bin = k * vp.n_types + ti;
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] += (b == bin) ? fixed : 0;
}

// Cone arithmetic over a lane's listed hits, records fetched four at a time.
template <int NB, bool kAny = false, int BS = 256>
__device__ __forceinline__ void vision_drain(const VisionLane& L, const swarm_vision_params_t& vp,
                                             const uint4* __restrict__ rec, size_t base,
                                             const uint32_t (*hits)[BS], int nh, int64_t* acc) {
  for (int k0 = 0; __any(k0 < nh); k0 += 4) {  // over the active lanes' longest list
    uint4 c0[4], c1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u < nh) {
        const size_t jj = base + hits[k0 + u][threadIdx.x];
        c0[u] = rec[2 * jj];
        c1[u] = rec[2 * jj + 1];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (k0 + u < nh) vision_hit<NB, kAny>(L, vp, c0[u], c1[u], acc);
  }
}

// The same over the G lanes' lists of a group together: the group's hits,
// concatenated in lane order, are dealt round-robin to its lanes, so a lane
// evaluates ceil(total / G) of them instead of its own list's length (the
// wave runs as long as its longest: ~6 hits of Poisson(2) lists against ~4
// of the balanced ones at E = 64).  Integer bin sums: the same result.
// Whole groups are active together (they share one agent).
template <int NB, int G, bool kAny = false, int BS = 256>
__device__ __forceinline__ void vision_drain_group(const VisionLane& L,
                                                   const swarm_vision_params_t& vp,
                                                   const uint4* __restrict__ rec, size_t base,
                                                   const uint32_t (*hits)[BS], int nh,
                                                   int64_t* acc) {
  // the other lanes' list entries are read below: keep the compiler from
  // moving those LDS reads above this lane's writes (one wave's LDS
  // operations complete in order)
  __asm__ volatile("" ::: "memory");
  const int sub = threadIdx.x & (G - 1);
  const int lane0 = (threadIdx.x & 63) - sub;  // the group's first lane in the wave
  const int tid0 = threadIdx.x - sub;
  int cnt[G];
  int total = 0;
#pragma unroll
  for (int l = 0; l < G; ++l) {
    cnt[l] = __shfl(nh, lane0 + l, 64);
    total += cnt[l];
  }
  for (int h0 = sub; __any(h0 < total); h0 += 4 * G) {
    uint4 c0[4], c1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = h0 + u * G;
      if (h < total) {
        int owner = 0, k = h, pre = 0;
#pragma unroll
        for (int l = 0; l < G; ++l) {
          const bool in = h >= pre && h < pre + cnt[l];
          owner = in ? l : owner;
          k = in ? h - pre : k;
          pre += cnt[l];
        }
        const size_t jj = base + hits[k][tid0 + owner];
        c0[u] = rec[2 * jj];
        c1[u] = rec[2 * jj + 1];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (h0 + u * G < total) vision_hit<NB, kAny>(L, vp, c0[u], c1[u], acc);
  }
}

// What a vision group does with its agent's summed bins (every lane of the
// group holds them): FeatureTail writes the observable row; PolicyTail
// (swarm_vision_policy) also runs the actor MLP and the sampling on them.
// pre() runs as soon as the agent's row is known (its loads overlap the
// candidate scan), done() after the group's reduction.
struct FeatureTail {
  using Pre = int;
  __device__ Pre pre(const VisionArgs&, int, int) const { return 0; }
  template <int NB, int G>
  __device__ void done(const VisionArgs& va, int e, int row, int sub, const int64_t (&acc)[NB],
                       Pre) const {
    if (sub != 0) return;
    const int nb = va.vp.n_cones * va.vp.n_types;
    float* o = va.out + ((size_t)e * va.n_agents + row) * nb;
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (k < nb) o[k] = (float)acc[k] * 2.3283064365386963e-10f;
  }
};

// The observable row, then the rollout policy of the same agent (flat agent
// a = e * n_agents + row, as swarm_policy_mlp_sample sees the flattened
// observable): the actor MLP over the group's G lanes, weights read in place
// (mlp_group_logits_direct), and lane 0 samples with the agent's own call
// counter state[a] (one group handles an agent per launch, so it reads and
// advances it alone: no block barrier, no atomic).
template <int D, int K>
struct PolicyTail {
  swarm::MlpArgs m;
  const float* sw = nullptr;  // the weights staged in LDS (stage_mlp_rows), or read in place
  using Pre = unsigned long long;
  __device__ Pre pre(const VisionArgs& va, int e, int row) const {
    return m.state[(size_t)e * va.n_agents + row];
  }
  template <int NB, int G>
  __device__ void done(const VisionArgs& va, int e, int row, int sub, const int64_t (&acc)[NB],
                       Pre ctr) const {
    static_assert(NB <= D, "the fused policy takes the bins as its features");
    const int nb = va.vp.n_cones * va.vp.n_types;
    const int a = e * va.n_agents + row;
    float x[D];
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (k < nb) x[k] = (float)acc[k] * 2.3283064365386963e-10f;
    if (sub == 0) {
      float* o = va.out + (size_t)a * nb;
#pragma unroll
      for (int k = 0; k < D; ++k)
        if (k < nb) o[k] = x[k];
    }
    float lg[K];
    if (sw)
      swarm::mlp_group_logits<G, D, K>(m, sw, x, sub, lg);
    else
      swarm::mlp_group_logits_direct<G, D, K>(m, x, sub, lg);
    if (sub == 0) {
      swarm::policy_emit<K>(m, a, lg, ctr);
      m.state[a] = ctr + 1ull;
    }
  }
};

// kAll: vision_range >= half the box (the reference has no range limit,
// subdivided_vision_cones.py:116-121): every record of the env is a
// candidate, tested on its unwrapped (int64) separation.
// xcd_bpe > 0: blocks placed on XCDs by env (swarm::xcd_env_block, xcd_bpe
// blocks per env), so the records an env's agents read stay in one L2.
// Body for block vb (k_vision, or a workgroup of k_vision_pairs /
// k_vision_cbuild); hits: the block's [kVisionHits][BS] LDS hit lists
// (blockDim BS).
template <int NB, int G, bool kAll = false, int BS = 256, class Tail = FeatureTail>
__device__ __forceinline__ void vision_body(const DevState& st, const Derived* __restrict__ d,
                                            const VisionArgs& va, int vb, int xcd_bpe,
                                            uint32_t (*hits)[BS], const Tail& tail = Tail{}) {
  const swarm_vision_params_t& vp = va.vp;
  const int lx = va.lx, ly = va.ly;
  const int32_t* __restrict__ start = va.start;
  const VisionSorted& vs = va.vs;
  const int n_envs = va.n_envs;
  const int N = st.n;
  const int sub = threadIdx.x & (G - 1);
  int e, ps;
  if (xcd_bpe > 0) {
    int lb;
    if (!swarm::xcd_env_block(vb, xcd_bpe, n_envs, &e, &lb)) return;
    ps = (lb * (int)blockDim.x + (int)threadIdx.x) / G;
    if (ps >= N) return;  // whole groups only (G divides 64)
  } else {
    const int grp = (vb * (int)blockDim.x + (int)threadIdx.x) / G;
    if (grp >= n_envs * N) return;
    e = grp / N;
    ps = grp - e * N;
  }
  const size_t base = (size_t)e * N;
  const uint4 own0 = vs.rec[2 * (base + ps)];
  const uint4 own1 = vs.rec[2 * (base + ps) + 1];
  VisionLane L;
  L.i = vision_rec_id(own1.y);
  const int row = vs.agent_row[L.i];
  // (the candidate ranges below load beside agent_row: both wait on the own
  // record only; a non-agent group leaves after them)
  L.qxi = own0.x;
  L.qyi = own0.y;
  L.ixi = (int32_t)own0.z;
  L.iyi = (int32_t)own0.w;
  float sn, cs;
  swarm::sincos_turn(own1.z, &sn, &cs);
  const float nm = swarm::sqrt_pos(cs * cs + sn * sn);  // ~1
  L.mx = cs / nm;
  L.my = sn / nm;
  L.sx0 = d->sx[0];
  L.sx1 = d->sx[1];
  L.R = vp.vision_range;
  int64_t acc[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) acc[k] = 0;
  const int ncell = 1 << (lx + ly);
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const int cc0 = cell_index(L.qxi, L.qyi, lx, ly);
  const int cx = cc0 & (ncx - 1), cy = cc0 >> lx;
  const int32_t* so = start + (size_t)e * (ncell + 1);
  int nh = 0;
  // the 3x3 candidate cells as one flat index range [0, total): a stencil
  // row (cells x-1..x+1) is one contiguous sorted range, plus one wrap cell
  // at the grid edge -- six ranges, their 12 bounds loaded together; then
  // candidates four at a time per lane (their record loads in flight
  // together), a lane taking f = sub, sub + G, ...; record index j = f +
  // off[r] of the range r holding f
  const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
  const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
  const int xw = ncx >= 3 ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
  int off[6], pre[7];
  pre[0] = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int oy = loy + (r >> 1), part = r & 1;
    int jb = 0, je = 0;
    if (kAll) {  // one range: all records
      je = r == 0 ? N : 0;
    } else if (oy <= hiy && (part == 0 || xw >= 0)) {
      const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
      jb = so[row | (part == 0 ? xa : xw)];
      je = so[(row | (part == 0 ? xb : xw)) + 1];
    }
    off[r] = jb - pre[r];
    pre[r + 1] = pre[r] + (je - jb);
  }
  if (row < 0) return;
  const typename Tail::Pre tail_pre = tail.pre(va, e, row);
  const int total = pre[6];
  // kVF candidates per lane in flight per round
  constexpr int kVF = 4;
  // (group-uniform trip count: a drain below always finds whole groups)
  for (int f00 = 0; f00 < total; f00 += kVF * G) {
    const int f0 = f00 + sub;
    uint4 c0[kVF];
    int jj[kVF];
#pragma unroll
    for (int u = 0; u < kVF; ++u) {
      const int f = f0 + u * G;
      int o = off[0];
#pragma unroll
      for (int r = 1; r < 6; ++r) o = f >= pre[r] ? off[r] : o;
      const int j = f + o;
      jj[u] = j;
      if (f < total) c0[u] = vs.rec[2 * (base + j)];
    }
#pragma unroll
    for (int u = 0; u < kVF; ++u) {
      float ddx, ddy;
      if (f0 + u * G < total &&
          (kAll ? vision_offsets<true>(L, c0[u], &ddx, &ddy) : vision_near(L, c0[u])))
        hits[nh++][threadIdx.x] = jj[u];
    }
    if (__any(nh > kVisionHits - kVF)) {  // no room for kVF more: drain every lane's
      if (G <= 8)
        vision_drain_group<NB, G, kAll>(L, vp, vs.rec, base, hits, nh, acc);
      else
        vision_drain<NB, kAll>(L, vp, vs.rec, base, hits, nh, acc);
      nh = 0;
    }
  }
  if (G <= 8)
    vision_drain_group<NB, G, kAll>(L, vp, vs.rec, base, hits, nh, acc);
  else
    vision_drain<NB, kAll>(L, vp, vs.rec, base, hits, nh, acc);
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)acc[b], off, 64);
      const int32_t hi = __shfl_xor((int)(acc[b] >> 32), off, 64);
      acc[b] += (int64_t)(((uint64_t)(uint32_t)hi << 32) | lo);
    }
  }
  swarm::role_mark(va.rstamp, swarm::kMarkConeReduced);
  tail.template done<NB, G>(va, e, row, sub, acc, tail_pre);
}

template <int NB, int G, bool kAll = false>
__global__ __launch_bounds__(256) void k_vision(DevState st, const Derived* __restrict__ d,
                                                VisionArgs va, int xcd_bpe) {
  __shared__ uint32_t hits[kVisionHits][256];
  vision_body<NB, G, kAll>(st, d, va, blockIdx.x, xcd_bpe, hits);
}

// The vision cone and the rollout policy of its agents in one launch
// (swarm_engine_vision_policy): each agent's group computes its bins, writes
// the observable row and runs the MLP + sampling on them (PolicyTail).
template <int NB, int G, int D, int K>
__global__ __launch_bounds__(256) void k_vision_policy(DevState st, const Derived* __restrict__ d,
                                                       VisionArgs va, swarm::MlpArgs m,
                                                       int xcd_bpe) {
  __shared__ uint32_t hits[kVisionHits][256];
  const PolicyTail<D, K> tail{m};
  vision_body<NB, G, false, 256, PolicyTail<D, K>>(st, d, va, blockIdx.x, xcd_bpe, hits, tail);
}

// ------------------------------------------- build stages riding along
// Latency-bound engines (swarm_engine_defer_build): the next window's
// cluster decomposition does not fork onto a second stream; its three
// stages ride along in the slice's observable and policy launches instead,
// as extra workgroups of the same kernels (no graph fork/join edges, no
// launch of their own):
//   k_vgrid_sort     the vision grid's env workgroups + k_build_sort's
//   k_vision_pairs   the vision cone's blocks + k_build_pairs's
//   k_policy_cbuild  the policy's blocks (1024 threads) + k_cluster_build's
// Each stage needs the previous one complete, which the launch order on
// the engine stream guarantees.  The build's workgroups take the first block
// indices of each launch: the build chain (sort -> pairs -> cluster build)
// is the longer one, so its workgroups are dealt out first.
// Block index of a fused launch whose first `nfirst` roles are the build's
// (dealt out first).
__device__ __forceinline__ int fused_block(int nfirst) {
  (void)nfirst;
  return (int)blockIdx.x;
}

// The l1_pairs pair-search role of the slice's first launch: n_fb blocks
// per env of blockDim threads after the sort and grid workgroups
// (swarm::pair_filter_body; ctl: the device control block, whose window
// counter names this window's build sort).  smem: the launch's dynamic LDS,
// at least l1_role_lds_bytes() (the fallback cell search's tables).
constexpr size_t l1_role_lds_bytes() {
  return (kMaxSpecies * kMaxSpecies + 2 * 1024) * sizeof(int32_t);
}
__device__ __forceinline__ void l1_pairs_role(const Derived* __restrict__ d, const DevState& st,
                                              const Scratch& sc, int lxb, int lyb, int fb, int n_fb,
                                              const uint64_t* ctl, unsigned char* smem) {
  float* nb2 = reinterpret_cast<float*>(smem);
  int32_t* uf = reinterpret_cast<int32_t*>(smem) + kMaxSpecies * kMaxSpecies;
  swarm::role_begin(sc, swarm::kRolePairs);
  swarm::pair_filter_body(d, st, sc, lxb, lyb, fb % n_fb, fb / n_fb, ctl[swarm::kCtlWin] + 1ull,
                          nb2, uf);
  swarm::role_end(sc, swarm::kRolePairs);
}

template <int CH>
__global__ __launch_bounds__(1024) void k_vgrid_sort(DevState st, VisionArgs va, Scratch sc,
                                                     int lxb, int lyb, const Derived* __restrict__ d,
                                                     int n_fb, const uint64_t* __restrict__ ctl) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = fused_block(va.n_envs);
  const int E = va.n_envs;
  if (b >= 2 * E) {  // l1_pairs: the pair search beside the sort (n_fb > 0)
    l1_pairs_role(d, st, sc, lxb, lyb, b - 2 * E, n_fb, ctl, smem);
    return;
  }
  const int role = b < E ? swarm::kRoleSort : swarm::kRoleVgrid;
  swarm::role_begin(sc, role);
  if (b < E)
    swarm::build_sort_body<CH>(st, sc, lxb, lyb, b, smem, n_fb > 0 ? ctl[swarm::kCtlWin] + 1ull : 0ull);
  else
    vision_grid_body(st, va, b - E, smem);
  swarm::role_end(sc, role);
}

// The pair blocks come first: theirs is the longer chain (the cluster build
// waits on it), so they are dealt out before the cone blocks.
template <int NB, int G, bool kLocal>
__global__ __launch_bounds__(256) void k_vision_pairs(DevState st, const Derived* __restrict__ d,
                                                      VisionArgs va, int n_pblocks, Scratch sc,
                                                      int lxb, int lyb, int pair_bx) {
  __shared__ uint32_t hits[kVisionHits][256];
  __shared__ float nb2[swarm::kMaxSpecies * swarm::kMaxSpecies];
  __shared__ int32_t uf[2 * 256];
  const int b = fused_block(n_pblocks);
  const int role = b < n_pblocks ? swarm::kRolePairs : swarm::kRoleCone;
  swarm::role_begin(sc, role);
  if (b < n_pblocks) {
    swarm::build_pairs_body<kLocal>(d, st, sc, lxb, lyb, b % pair_bx, b / pair_bx, nb2, uf);
  } else {
    vision_body<NB, G, false>(st, d, va, b - n_pblocks, 0, hits);
  }
  swarm::role_end(sc, role);
}

// The same with the fused rollout policy on the cone side (PolicyTail): the
// pair blocks first, then the cone + MLP + sampling blocks.
template <int NB, int G, bool kLocal, int D, int K>
__global__ __launch_bounds__(256) void k_vision_policy_pairs(DevState st,
                                                             const Derived* __restrict__ d,
                                                             VisionArgs va, swarm::MlpArgs m,
                                                             int n_pblocks, Scratch sc, int lxb,
                                                             int lyb, int pair_bx) {
  __shared__ uint32_t hits[kVisionHits][256];
  __shared__ float nb2[swarm::kMaxSpecies * swarm::kMaxSpecies];
  __shared__ int32_t uf[2 * 256];
  const int b = fused_block(n_pblocks);
  const int role = b < n_pblocks ? swarm::kRolePairs : swarm::kRoleCone;
  swarm::role_begin(sc, role);
  if (b < n_pblocks) {
    swarm::build_pairs_body<kLocal>(d, st, sc, lxb, lyb, b % pair_bx, b / pair_bx, nb2, uf);
  } else {
    const PolicyTail<D, K> tail{m};
    vision_body<NB, G, false, 256, PolicyTail<D, K>>(st, d, va, b - n_pblocks, 0, hits, tail);
  }
  swarm::role_end(sc, role);
}

// l1_pairs slices: the pair list is ready when the cone runs, so the
// cluster build rides beside the cone + MLP + sampling (1024-thread blocks:
// the build's workgroup per env first, then the cone's, whose hit lists
// share the build's dynamic LDS).
template <int NB, int G, int D, int K>
__global__ __launch_bounds__(1024) void k_vision_policy_cbuild(DevState st,
                                                               const Derived* __restrict__ d,
                                                               VisionArgs va, swarm::MlpArgs m,
                                                               Scratch sc) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = fused_block(va.n_envs);
  const int role = b < va.n_envs ? swarm::kRoleCbuild : swarm::kRoleCone;
  swarm::role_begin(sc, role);
  if (b < va.n_envs) {
    swarm::cluster_build_env<false, true, false>(st, sc, b, smem, sc.gnpairs[b]);
  } else {
    auto* hits = reinterpret_cast<uint32_t(*)[1024]>(smem);
    // the actor's rows into LDS behind the hit lists before any group starts
    // (the groups' tails then read them at LDS latency, not L2's)
    float* sw = reinterpret_cast<float*>(smem + (size_t)kVisionHits * 1024 * sizeof(uint32_t));
    swarm::stage_mlp_rows<D, K>(m, sw);
    __syncthreads();
    const PolicyTail<D, K> tail{m, sw};
    vision_body<NB, G, false, 1024, PolicyTail<D, K>>(st, d, va, b - va.n_envs, 0, hits, tail);
  }
  swarm::role_end(sc, role);
}

template <int G, int D, int K>
__global__ __launch_bounds__(1024) void k_policy_cbuild(swarm::MlpArgs m, int n_envs,
                                                        DevState st, Scratch sc) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = fused_block(n_envs);
  const int role = b < n_envs ? swarm::kRoleCbuild : swarm::kRoleMlp;
  swarm::role_begin(sc, role);
  if (b < n_envs) {
    if (sc.local_uf)
      swarm::cluster_build_env<false, true, true>(st, sc, b, smem, sc.gnpairs[b]);
    else
      swarm::cluster_build_env<false, true, false>(st, sc, b, smem, sc.gnpairs[b]);
  } else {
    swarm::policy_body<G, D, K>(m, b - n_envs, reinterpret_cast<float*>(smem));
  }
  swarm::role_end(sc, role);
}

// ------------------------------------------- neighbour reductions (fp64)
// For the classical neighbour-rule agents (bechinger_models.py:156-171
// get_colloids_in_vision; lymburn_model.py:113-125): per agent i and every
// candidate j != i whose type bit is set in cand_mask, with d = x_j - x_i,
// |d| < range and (half_angle >= 0) acos(d/|d| . dir_i) < half_angle:
//   out[0] = count, out[1] = sum 1/(2 pi |d|), out[2..4] = sum d,
//   out[5] = sum |d|^2, out[6..8] = sum dir_j, out[9..11] = sum v_j.
// fp64 like the reference's numpy; candidates staged in LDS tiles.
constexpr int kNbOut = 12;

__global__ __launch_bounds__(256) void k_neighbor_reduce(
    const double* __restrict__ pos, const double* __restrict__ dir, const double* __restrict__ vel,
    const int32_t* __restrict__ types, int n, const int32_t* __restrict__ agents, int n_agents,
    uint32_t cand_mask, double range, double half_angle, double* __restrict__ out) {
  __shared__ double tp[256][3], td[256][3], tv[256][3];
  __shared__ int32_t tid_[256];
  const int e = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = a < n_agents;
  const size_t base = (size_t)e * n;
  int i = -1;
  double xi[3] = {0.0, 0.0, 0.0}, mi[3] = {0.0, 0.0, 0.0};
  if (valid) {
    i = agents[a];
    for (int k = 0; k < 3; ++k) {
      xi[k] = pos[(base + i) * 3 + k];
      mi[k] = dir[(base + i) * 3 + k];
    }
  }
  double acc[kNbOut];
#pragma unroll
  for (int k = 0; k < kNbOut; ++k) acc[k] = 0.0;
  for (int j0 = 0; j0 < n; j0 += 256) {
    const int j = j0 + (int)threadIdx.x;
    __syncthreads();
    if (j < n) {
      const bool ok = (cand_mask >> (types[j] & 31)) & 1u;
      tid_[threadIdx.x] = ok ? j : -1;
      for (int k = 0; k < 3; ++k) {
        tp[threadIdx.x][k] = pos[(base + j) * 3 + k];
        td[threadIdx.x][k] = dir[(base + j) * 3 + k];
        tv[threadIdx.x][k] = vel ? vel[(base + j) * 3 + k] : 0.0;
      }
    } else {
      tid_[threadIdx.x] = -1;
    }
    __syncthreads();
    if (!valid) continue;
    const int cn = min(256, n - j0);
    for (int c = 0; c < cn; ++c) {
      const int jj = tid_[c];
      if (jj < 0 || jj == i) continue;
      const double dx = tp[c][0] - xi[0], dy = tp[c][1] - xi[1], dz = tp[c][2] - xi[2];
      const double d2 = dx * dx + dy * dy + dz * dz;
      const double dn = sqrt(d2);
      if (!(dn < range)) continue;
      if (half_angle >= 0.0) {
        const double dot = (dx / dn) * mi[0] + (dy / dn) * mi[1] + (dz / dn) * mi[2];
        if (!(acos(dot) < half_angle)) continue;
      }
      acc[0] += 1.0;
      acc[1] += 1.0 / (2.0 * 3.14159265358979323846 * dn);
      acc[2] += dx;
      acc[3] += dy;
      acc[4] += dz;
      acc[5] += d2;
      acc[6] += td[c][0];
      acc[7] += td[c][1];
      acc[8] += td[c][2];
      acc[9] += tv[c][0];
      acc[10] += tv[c][1];
      acc[11] += tv[c][2];
    }
  }
  if (valid) {
    double* o = out + ((size_t)e * n_agents + a) * kNbOut;
#pragma unroll
    for (int k = 0; k < kNbOut; ++k) o[k] = acc[k];
  }
}

// ------------------------------------------------ pairwise field distances
// For ParticleSensing / SpeciesSearch (particle_sensing.py:95-121,
// species_search.py:97-130): d = || fp32(x_j) - fp32(x_i) || / L per agent
// i and sensed colloid j (unwrapped positions, no minimum image), written
// [E][mc][A] for sensed columns m0 .. m0 + mc - 1.  The sensed positions of
// the block's column tile are staged in LDS once and read by all agents.
__global__ __launch_bounds__(256) void k_pair_dist(DevState st, const double* __restrict__ box,
                                                   const int32_t* __restrict__ agents,
                                                   int n_agents,
                                                   const int32_t* __restrict__ sensed, int m0,
                                                   int mc, float b0, float b1, float b2,
                                                   float* __restrict__ out) {
  __shared__ float tile[256][3];
  const int e = blockIdx.z;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const int N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const double inv32 = 1.0 / 4294967296.0;
  float xi[3] = {0.0f, 0.0f, 0.0f};
  if (a < n_agents) {
    const size_t gi = base + agents[a];
    for (int k = 0; k < st.dims; ++k)
      xi[k] = (float)(((double)st.img[k * M + gi] + (double)st.q[k * M + gi] * inv32) * box[k]);
  }
  const int c0 = blockIdx.y * 256;
  const int cn = min(256, mc - c0);
  if (threadIdx.x < cn) {
    const size_t gj = base + sensed[m0 + c0 + threadIdx.x];
    tile[threadIdx.x][2] = 0.0f;
    for (int k = 0; k < st.dims; ++k)
      tile[threadIdx.x][k] =
          (float)(((double)st.img[k * M + gj] + (double)st.q[k * M + gj] * inv32) * box[k]);
  }
  __syncthreads();
  if (a >= n_agents) return;
  const size_t A = (size_t)n_agents;
  float* o = out + ((size_t)e * mc + c0) * A + a;
  for (int c = 0; c < cn; ++c) {
    const float dx = (tile[c][0] - xi[0]) / b0;
    const float dy = (tile[c][1] - xi[1]) / b1;
    const float dz = (tile[c][2] - xi[2]) / b2;
    o[(size_t)c * A] = swarm::sqrt_rn(dx * dx + dy * dy + dz * dz);
  }
}

// ------------------------------------------------------- field distance
struct FieldArgs {
  const double* box;
  const int32_t* agents;
  int n_agents;
  double s0, s1, s2;  // source
  double b0, b1, b2;  // box scale
  uint32_t* hq;
  int32_t* himg;
  float* d_cur;
  float* d_prev;
  int update, init_only, n_envs;
  int mode;  // 0: distances; 1: scale (f(d_cur) - f(d_prev)), f(d) = fa + fb d; 2: same, clipped at 0
  float fa, fb, fscale;
  float* out;
};

// Agent slot t (env-major) of k_field, or of a workgroup of k_field_vgrid_sort.
__device__ __forceinline__ void field_body(const DevState& st, const FieldArgs& f, int t) {
  const int A = f.n_agents * f.n_envs;
  if (t >= A) return;
  const int e = t / f.n_agents, ai = t - e * f.n_agents;
  const int N = st.n;
  const size_t M = (size_t)st.m;
  const size_t gi = (size_t)e * N + f.agents[ai];
  const double inv32 = 1.0 / 4294967296.0;
  if (!f.init_only) {
    const double src[3] = {f.s0 / f.b0, f.s1 / f.b1, f.s2 / f.b2};
    const double bs[3] = {f.b0, f.b1, f.b2};
    float cur[3], prev[3];
    for (int a = 0; a < 3; ++a) {
      double pc, hp;
      if (a < st.dims) {
        pc = ((double)st.img[a * M + gi] + (double)st.q[a * M + gi] * inv32) * f.box[a] / bs[a];
        hp = ((double)f.himg[(size_t)a * A + t] + (double)f.hq[(size_t)a * A + t] * inv32) *
             f.box[a] / bs[a];
      } else {
        pc = 0.0 / bs[a];
        hp = 0.0 / bs[a];
      }
      cur[a] = (float)(src[a] - pc);
      prev[a] = (float)(src[a] - hp);
    }
    const float dc = swarm::sqrt_rn(cur[0] * cur[0] + cur[1] * cur[1] + cur[2] * cur[2]);
    const float dp = swarm::sqrt_rn(prev[0] * prev[0] + prev[1] * prev[1] + prev[2] * prev[2]);
    if (f.mode == 0) {
      f.d_cur[t] = dc;
      f.d_prev[t] = dp;
    } else {
      // affine decay f(d) = fa + fb * d; value = scale * (f(d_cur) - f(d_prev))
      // (concentration_field.py:102-104); mode 2 clips at 0
      // (gradient_sensing.py:117-118; NaN propagates as in torch.clamp)
      const float fc = f.fa + f.fb * dc;
      const float fp = f.fa + f.fb * dp;
      float v = f.fscale * (fc - fp);
      if (f.mode == 2) v = v < 0.0f ? 0.0f : v;
      f.out[t] = v;
    }
  }
  if (f.update || f.init_only) {
    for (int a = 0; a < 3; ++a) {
      f.hq[(size_t)a * A + t] = a < st.dims ? st.q[a * M + gi] : 0u;
      f.himg[(size_t)a * A + t] = a < st.dims ? st.img[a * M + gi] : 0;
    }
  }
}

__global__ __launch_bounds__(256) void k_field(DevState st, FieldArgs f) {
  field_body(st, f, blockIdx.x * blockDim.x + threadIdx.x);
}

// The reward launch of a slice whose observable is a persistent vision
// cone (swarm_vision_cone_persistent) and whose next build is deferred:
// the field's agents, the NEXT observable's vision grid (from the positions
// the reward sees, which the observable will see too) and build stage 1,
// so the observable launch only runs the cone (beside stage 2).
// l1_pairs (n_fb > 0): the next window's pair search rides here too,
// n_fb blocks per env after the grid workgroups (l1_pairs_role).
// with_grid = 0 (a field observable, l1_pairs): no vision grid, the reward
// carries the sort and the pair search only (its grid workgroups return).
template <int CH>
__global__ __launch_bounds__(1024) void k_field_vgrid_sort(FieldArgs f, int n_fblocks, DevState st,
                                                           VisionArgs va, Scratch sc, int lxb,
                                                           int lyb, const Derived* __restrict__ d,
                                                           int n_fb, const uint64_t* __restrict__ ctl,
                                                           int with_grid) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = fused_block(2 * va.n_envs);
  const int E = va.n_envs, npb = n_fb * E;
  if (b >= 2 * E && b < 2 * E + npb) {
    l1_pairs_role(d, st, sc, lxb, lyb, b - 2 * E, n_fb, ctl, smem);
    return;
  }
  if (!with_grid && b >= E && b < 2 * E) return;
  const int role = b < E ? swarm::kRoleSort : b < 2 * E ? swarm::kRoleVgrid : swarm::kRoleField;
  swarm::role_begin(sc, role);
  if (b < E)
    swarm::build_sort_body<CH>(st, sc, lxb, lyb, b, smem, n_fb > 0 ? ctl[swarm::kCtlWin] + 1ull : 0ull);
  else if (b < 2 * E)
    vision_grid_body(st, va, b - E, smem);
  else
    field_body(st, f, (b - 2 * E - npb) * blockDim.x + threadIdx.x);
  swarm::role_end(sc, role);
}

// --------------------------------------------------------- pair listing
__global__ __launch_bounds__(256) void k_pairs(DevState st, const Derived* __restrict__ d,
                                               int env, float cut2, int lx, int ly,
                                               const int32_t* __restrict__ start,
                                               const int32_t* __restrict__ order,
                                               int32_t* __restrict__ pairs, int max_pairs,
                                               int32_t* __restrict__ count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int N = st.n;
  if (i >= N) return;
  const size_t M = (size_t)st.m;
  const size_t gi = (size_t)env * N + i;
  const uint32_t qxi = st.q[gi], qyi = st.q[M + gi];
  const int ncell = 1 << (lx + ly);
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int lox = ncx >= 3 ? -1 : 0, hix = ncx >= 3 ? 1 : ncx - 1;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const int cc0 = cell_index(qxi, qyi, lx, ly);
  const int cx = cc0 & (ncx - 1), cy = cc0 >> lx;
  const int32_t* so = start + (size_t)env * (ncell + 1);
  const int32_t* oo = order + (size_t)env * N;
  for (int oy = loy; oy <= hiy; ++oy) {
    const int y = (cy + oy + ncy) & (ncy - 1);
    for (int ox = lox; ox <= hix; ++ox) {
      const int x = (cx + ox + ncx) & (ncx - 1);
      const int cc = (y << lx) | x;
      for (int jj = so[cc]; jj < so[cc + 1]; ++jj) {
        const int j = oo[jj];
        if (j <= i) continue;
        const size_t gj = (size_t)env * N + j;
        // minimum image in a periodic box, else the unwrapped difference
        // (the grid search wraps either way: a pair within cutoff < L / 2 is
        // within it by the minimum image too)
        const bool per = d->periodic != 0;
        const float rx = swarm::pair_disp(st.q[gj], st.img[gj], qxi, st.img[gi], d->sx[0], per);
        const float ry = swarm::pair_disp(st.q[M + gj], st.img[M + gj], qyi, st.img[M + gi], d->sx[1], per);
        if (rx * rx + ry * ry < cut2) {
          const int slot = atomicAdd(count, 1);
          if (slot < max_pairs) {
            pairs[2 * slot] = i;
            pairs[2 * slot + 1] = j;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------- trajectory ring
// One trajectory entry of env `env` (espresso.py:1110-1130: the state at a
// write point) into slot count % cap of a host-pinned, device-mapped ring:
// the step counter, then q[D][N], img[D][N], ang[N] (2-D) or dir3[3][N]
// (3-D), vel[D][N].  The slot comes from a device counter, so captured
// graphs record into successive slots on every replay; k_traj_bump
// publishes the count after the entry is complete (stream order).
__global__ __launch_bounds__(256) void k_traj_write(DevState st, int env,
                                                    unsigned char* __restrict__ ring, int cap,
                                                    size_t entry_bytes,
                                                    const uint64_t* __restrict__ count,
                                                    const uint64_t* __restrict__ ctl) {
  const int N = st.n, D = st.dims;
  const size_t M = (size_t)st.m;
  const uint64_t slot = *count % (uint64_t)cap;
  unsigned char* ent = ring + 64 + slot * entry_bytes;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *reinterpret_cast<uint64_t*>(ent) = ctl[0];
  if (i >= N) return;
  const size_t gi = (size_t)env * N + i;
  uint32_t* w = reinterpret_cast<uint32_t*>(ent + 8);
  for (int a = 0; a < D; ++a) w[(size_t)a * N + i] = st.q[a * M + gi];
  w += (size_t)D * N;
  for (int a = 0; a < D; ++a) w[(size_t)a * N + i] = (uint32_t)st.img[a * M + gi];
  w += (size_t)D * N;
  if (D == 3) {
    float* f = reinterpret_cast<float*>(w);
    for (int a = 0; a < 3; ++a) f[(size_t)a * N + i] = st.dir3[a * M + gi];
    w += (size_t)3 * N;
  } else {
    w[i] = st.ang[gi];
    w += N;
  }
  float* v = reinterpret_cast<float*>(w);
  for (int a = 0; a < D; ++a) v[(size_t)a * N + i] = st.vel[a * M + gi];
}

__global__ void k_traj_bump(uint64_t* __restrict__ count, unsigned char* __restrict__ ring) {
  if (threadIdx.x == 0) {
    const uint64_t c = *count + 1;
    *count = c;
    __threadfence_system();
    *reinterpret_cast<volatile uint64_t*>(ring) = c;
  }
}

}  // namespace

// =================================================================== C ABI
struct swarm_engine {
  swarm_params_t params;
  Derived derived;
  int32_t n_envs = 0, n = 0;
  hipStream_t stream = nullptr;
  int device = 0;
  DevState st{};
  Scratch sc{};
  Derived* d_derived = nullptr;
  double* d_box = nullptr;
  uint64_t* d_step = nullptr;
  uint32_t* d_arrive = nullptr;
  // trajectory ring (swarm_engine_traj_ring): host-pinned, device-mapped
  unsigned char* traj_host = nullptr;
  unsigned char* traj_dev = nullptr;
  uint64_t* d_traj_count = nullptr;
  int traj_cap = 0, traj_env = 0;
  size_t traj_entry = 0;
  // observable grid scratch
  int32_t* d_start = nullptr;
  size_t start_cap = 0;
  int32_t* d_order = nullptr;
  int32_t* d_count = nullptr;
  int32_t* d_pairs = nullptr;
  size_t pairs_cap = 0;
  int lxg = 0, lyg = 0, lzg = 0;  // global-path grid: cell side >= rc_max (lzg: 3-D)
  int lxb = 0, lyb = 0, lzb = 0;  // cluster-build grid: cell side >= rc_max + skin
  bool cluster_path = false;
  // 3-D boxes whose rc + skin graph percolates: chip-wide sub-steps over a
  // per-window Verlet list instead of per-wave clusters (swarm_integrator3.cuh)
  bool nlist_path = false;
  bool big_build = false;  // k_cluster_build<true>: cluster arrays in global memory
  bool chip_sort = false;  // 2-D envs above 4096 colloids: the three-launch chip-wide sort
  VisionSorted vs{};
  // latency-bound windows read their normals from a table (k_noise)
  bool noise_table = false;
  float* d_noise = nullptr;
  // swarm_engine_prebuild: the next window's build (and noise table) were
  // launched ahead on another stream from the current positions
  bool prebuilt = false;
  // swarm_engine_defer_build: the next stage of the deferred three-launch
  // build (1 sort, 2 pairs, 3 cluster build; 0 none) that rides along in the
  // next observable / policy launch; flushed before a window runs
  int ride_stage = 0;
  // speculative vision grid (swarm_vision_cone_persistent): the last
  // persistent call's arguments; vgrid_ready: the reward launch built the
  // grid of the current positions for them (honoured while the deferred
  // build is at stage 2, i.e. nothing moved the colloids since).
  bool spec_ok = false;
  VisionArgs spec_va{};
  bool vgrid_ready = false;
  // swarm_engine_prebuild_noise: the next window's noise table for this many
  // sub-steps was launched ahead (on a stream of the caller's)
  int prebuilt_noise_steps = 0;
  // Latency-bound engines run k_cluster_run_wide: one block per CU, and
  // (noise_blocks > 0) the next window's noise table filled beside the run;
  // next_table_ready: the last window did that (the table's first step and
  // length are checked on the device, this flag only skips k_noise).
  bool wide_run = false;
  int run_wpb = 4;  // run waves per block (= per CU) of k_cluster_run_wide
  // a rotation helper wave beside each run wave of k_cluster_run_wide
  // (swarm::rot_helper; run_wpb <= 2)
  bool rot_helper = true;
  // k_build_env: the whole build in one LDS-resident workgroup per env
  bool env_build = false;
  int noise_blocks = 0;
  bool next_table_ready = false;
  // swarm_engine_profile: HIP events around every k_cluster_run launch;
  // launches captured into a graph get event-record nodes whose events are
  // kept (graph_events) for swarm_engine_profile_graph after each replay
  bool profile = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> graph_events;
  // per captured run node, an empty event pair recorded right after it: the
  // cost of an event-record node pair itself (swarm_engine_profile_graph)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> graph_cal;
  // and each captured run node's own start / end stamps (swarm::stamp_start,
  // stamp_end): d_tstamp[k][kStampSub][2] for the k-th captured run node
  unsigned long long* d_tstamp = nullptr;
  int stamp_next = 0;
  // [kMaxStamps][kRoles][2]: the workgroup roles of the launches that follow
  // the k-th captured run node (its k_check, then the next window's build and
  // observable launches), swarm::role_begin / role_end
  unsigned long long* d_rstamp = nullptr;
  float* own_f_swim = nullptr;
  float* own_torque_z = nullptr;
  void* allocs[96] = {};
  int n_allocs = 0;
};

namespace {

template <typename T>
int dev_alloc(swarm_engine* e, T** p, size_t count) {
  if (e->n_allocs >= (int)(sizeof(e->allocs) / sizeof(e->allocs[0])))
    return fail(SWARM_ECAPACITY, "engine allocation table full");
  void* v = nullptr;
  HIP_TRY(hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T)));
  HIP_TRY(hipMemsetAsync(v, 0, std::max<size_t>(count, 1) * sizeof(T), e->stream));
  e->allocs[e->n_allocs++] = v;
  *p = reinterpret_cast<T*>(v);
  return SWARM_OK;
}

constexpr size_t kMaxLds = 160 * 1024;

// k_global: wave sums, cell counts and (2-D, N <= 4096) the register-resident
// path's sorted copy
size_t global_lds_bytes(int lx, int ly, int n, int dims) {
  return (16 + (size_t)(1 << (lx + ly)) + 1 + swarm::global_lds_extra_words(n, dims, 1 << (lx + ly))) * 4;
}

// Pair-list capacity of the cluster build: up to 3 N pairs (mean degree 6),
// at least N, within the LDS left after the other arrays of k_cluster_build;
// 3 N in global memory for the large-N variant.
int build_pair_cap(int n, bool big) {
  if (big) return 3 * n;
  const size_t fixed = swarm::build_lds_words(n, 0) * 4;
  const size_t room = fixed < kMaxLds ? (kMaxLds - fixed) / 4 : 0;
  return (int)std::min<size_t>(room, 3 * (size_t)n);
}

// The LDS build needs room for at least N pairs; beyond that, the large-N
// variant keeps only the union-find forest in LDS.
bool build_is_big(int n) { return swarm::build_lds_words(n, n) * 4 > kMaxLds; }

size_t build_lds_bytes(int n, int pair_cap) { return swarm::build_lds_words(n, pair_cap) * 4; }

size_t check_lds_bytes(int lx, int ly, int n, int dims) {
  // the global-path re-run region (cell counts + LDS path) or the big
  // clusters' positions and force sums, after 16 + 16 + 1024 words
  const size_t rerun = (size_t)(1 << (lx + ly)) + 1 + swarm::global_lds_extra_words(n, dims, 1 << (lx + ly));
  const size_t big = 6 * (size_t)swarm::kBigMax + 2;  // uint2 positions, 2 x u64 sums
  return (16 + 16 + 1024 + std::max(rerun, big)) * 4;
}

// k_build_sort (and the fused launches carrying it): wave sums, cell counts
// and, staged, the sorted x | y | id rows.
size_t sort_lds_bytes(const swarm_engine* e);

// k_check3: wave sums, misc, movers, then the 3-D global path's cell counts
size_t check3_lds_bytes(const swarm_engine* e) {
  return (16 + 16 + (size_t)swarm::kMaxMovers + (size_t)(1 << (e->lxg + e->lyg + e->lzg)) + 1) * 4;
}

// ROCm admits dynamic LDS up to the device limit at launch; this attribute
// is only a hint, a refusal is not an error (a launch that really exceeds the
// limit fails at hipGetLastError after the launch).
void set_lds_attributes() {
  static bool done = false;
  if (done) return;
  const void* fns[] = {reinterpret_cast<const void*>(&swarm::k_global),
                       reinterpret_cast<const void*>(&swarm::k_cluster_build<false, false>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_build<false, true>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_build<true, false>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_build_packed),
                       reinterpret_cast<const void*>(&swarm::k_build_sort<4>),
                       reinterpret_cast<const void*>(&swarm::k_sort_scan),
                       reinterpret_cast<const void*>(&swarm::k_build_sort<16>),
                       reinterpret_cast<const void*>(&swarm::k_build_env),
                       reinterpret_cast<const void*>(&swarm::k_check),
                       reinterpret_cast<const void*>(&k_grid_build),
                       reinterpret_cast<const void*>(&k_vision_grid),
                       reinterpret_cast<const void*>(&swarm::k_cluster_run_wide<false, false>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_run_wide<true, false>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_run_wide<false, true>),
                       reinterpret_cast<const void*>(&swarm::k_cluster_run_wide<true, true>),
                       reinterpret_cast<const void*>(&k_vgrid_sort<4>),
                       reinterpret_cast<const void*>(&k_vgrid_sort<16>),
                       reinterpret_cast<const void*>(&k_field_vgrid_sort<4>),
                       reinterpret_cast<const void*>(&k_field_vgrid_sort<16>),
                       reinterpret_cast<const void*>(&k_policy_cbuild<4, 4, 4>)};
  for (const void* f : fns)
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
  (void)hipGetLastError();
  done = true;
}

int launch_global(swarm_engine* e, int n_steps, int sd_mode, float g, float md) {
  if (e->params.n_dims == 3) {
    hipLaunchKernelGGL(swarm::k_global3, dim3(e->n_envs), dim3(1024),
                       (16 + (size_t)(1 << (e->lxg + e->lyg + e->lzg)) + 1) * 4, e->stream,
                       e->d_derived, e->st, e->sc, n_steps, e->d_step, e->d_arrive, e->lxg,
                       e->lyg, e->lzg, sd_mode, g, md);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  hipLaunchKernelGGL(swarm::k_global, dim3(e->n_envs), dim3(1024),
                     global_lds_bytes(e->lxg, e->lyg, e->n, e->params.n_dims), e->stream, e->d_derived, e->st, e->sc,
                     n_steps, e->d_step, e->d_arrive, e->lxg, e->lyg, sd_mode, g, md);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

// Noise table (latency-bound windows) for n sub-steps from the current
// step counter.
int launch_noise(swarm_engine* e, hipStream_t stream, int n) {
  const long M = (long)e->n_envs * e->n;
  const long items = M * (long)swarm::noise_items(n);
  hipLaunchKernelGGL(swarm::k_noise, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, stream,
                     e->d_derived, e->st, e->d_step, e->d_noise, n);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

// Cluster build of the next window.
int launch_build(swarm_engine* e, hipStream_t stream) {
  if (e->env_build) {
    hipLaunchKernelGGL(swarm::k_build_env, dim3(e->n_envs), dim3(1024),
                       build_lds_bytes(e->n, e->sc.pair_cap), stream, e->d_derived, e->st, e->sc,
                       e->lxb, e->lyb);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  if (e->params.n_dims == 3) {
    if (e->n > 4096)
      hipLaunchKernelGGL(swarm::k_build_sort3<16>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                         stream, e->st, e->sc, e->lxb, e->lyb, e->lzb);
    else
      hipLaunchKernelGGL(swarm::k_build_sort3<4>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                         stream, e->st, e->sc, e->lxb, e->lyb, e->lzb);
    HIP_TRY(hipGetLastError());
    if (e->nlist_path) {  // Verlet lists, no clusters
      hipLaunchKernelGGL(swarm::k_build_nlist3, dim3((unsigned)((e->n + 255) / 256), e->n_envs),
                         dim3(256), 0, stream, e->d_derived, e->st, e->sc, e->lxb, e->lyb, e->lzb);
      HIP_TRY(hipGetLastError());
      return SWARM_OK;
    }
    hipLaunchKernelGGL(swarm::k_build_pairs3, dim3((unsigned)((e->n + 255) / 256), e->n_envs),
                       dim3(256), 0, stream, e->d_derived, e->st, e->sc, e->lxb, e->lyb, e->lzb);
  } else if (e->chip_sort) {
    const dim3 pgrid((unsigned)((e->n + 255) / 256), (unsigned)e->n_envs);
    hipLaunchKernelGGL(swarm::k_sort_count, pgrid, dim3(256), 0, stream, e->st, e->sc, e->lxb,
                       e->lyb);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_sort_scan, dim3(e->n_envs), dim3(1024),
                       (size_t)(16 + (1 << (e->lxb + e->lyb)) + 1) * 4, stream, e->sc, e->lxb,
                       e->lyb);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_sort_scatter, pgrid, dim3(256), 0, stream, e->st, e->sc, e->lxb,
                       e->lyb);
  } else if (e->n > 4096) {
    hipLaunchKernelGGL(swarm::k_build_sort<16>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                       stream, e->st, e->sc, e->lxb, e->lyb);
  } else {
    hipLaunchKernelGGL(swarm::k_build_sort<4>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                       stream, e->st, e->sc, e->lxb, e->lyb);
  }
  HIP_TRY(hipGetLastError());
  if (e->params.n_dims != 3 && e->nlist_path) {  // Verlet lists, no clusters
    hipLaunchKernelGGL(swarm::k_build_nlist2, dim3((unsigned)((e->n + 255) / 256), e->n_envs),
                       dim3(256), 0, stream, e->d_derived, e->st, e->sc, e->lxb, e->lyb);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  if (e->params.n_dims != 3)
  {
    const dim3 pg((unsigned)((e->n + 255) / 256), (unsigned)e->n_envs);
    if (e->sc.local_uf)
      hipLaunchKernelGGL(swarm::k_build_pairs<true>, pg, dim3(256), 0, stream, e->d_derived,
                         e->st, e->sc, e->lxb, e->lyb);
    else
      hipLaunchKernelGGL(swarm::k_build_pairs<false>, pg, dim3(256), 0, stream, e->d_derived,
                         e->st, e->sc, e->lxb, e->lyb);
  }
  HIP_TRY(hipGetLastError());
  // 2-D: the pair search left block-local union-find roots and a cross list
  // (build_pairs_body); 3-D (k_build_pairs3): the whole pair list is unioned
  const bool local = e->params.n_dims == 2 && e->sc.local_uf;
  if (e->sc.bmisc) {  // multi-workgroup build: union, sizes, classes, slots, wave pair lists
    const unsigned nbp = (unsigned)((e->n + 255) / 256);
    hipLaunchKernelGGL(swarm::k_mwb_union, dim3((nbp + 3) / 4, e->n_envs), dim3(256), 0, stream,
                       e->st, e->sc);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_mwb_size, dim3(nbp, e->n_envs), dim3(256), 0, stream, e->st, e->sc);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_mwb_class, dim3((unsigned)((e->n + 1023) / 1024), e->n_envs),
                       dim3(1024), 0, stream, e->st, e->sc);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_mwb_slots, dim3(nbp, e->n_envs), dim3(256), 0, stream, e->st,
                       e->sc);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_mwb_pairs, dim3((unsigned)((e->sc.wmax + 3) / 4), e->n_envs),
                       dim3(256), 0, stream, e->st, e->sc);
  } else if (e->big_build && !local && swarm::build_lds_words_packed(e->n) * 4 <= kMaxLds) {
    hipLaunchKernelGGL(swarm::k_cluster_build_packed, dim3(e->n_envs), dim3(1024),
                       swarm::build_lds_words_packed(e->n) * 4, stream, e->st, e->sc);
  } else if (e->big_build) {  // (2-D envs with the local pair search took k_mwb_*)
    hipLaunchKernelGGL((swarm::k_cluster_build<true, false>), dim3(e->n_envs), dim3(1024),
                       swarm::build_lds_words_big(e->n) * 4, stream, e->st, e->sc);
  } else if (local) {
    hipLaunchKernelGGL((swarm::k_cluster_build<false, true>), dim3(e->n_envs), dim3(1024),
                       build_lds_bytes(e->n, e->sc.pair_cap), stream, e->st, e->sc);
  } else {
    hipLaunchKernelGGL((swarm::k_cluster_build<false, false>), dim3(e->n_envs), dim3(1024),
                       build_lds_bytes(e->n, e->sc.pair_cap), stream, e->st, e->sc);
  }
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

// Launch the deferred build's pending stages on the engine stream (no
// consumer carried them along); the window then uses the build.
int flush_ride_along(swarm_engine* e) {
  const int stage = e->ride_stage;
  e->vgrid_ready = false;
  if (stage == 0) return SWARM_OK;
  e->ride_stage = 0;
  if (stage <= 1) {
    if (e->n > 4096)
      hipLaunchKernelGGL(swarm::k_build_sort<16>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                         e->stream, e->st, e->sc, e->lxb, e->lyb);
    else
      hipLaunchKernelGGL(swarm::k_build_sort<4>, dim3(e->n_envs), dim3(1024), sort_lds_bytes(e),
                         e->stream, e->st, e->sc, e->lxb, e->lyb);
    HIP_TRY(hipGetLastError());
  }
  if (stage <= 2) {
    if (e->sc.local_uf)
      hipLaunchKernelGGL(swarm::k_build_pairs<true>, dim3((unsigned)((e->n + 255) / 256), e->n_envs),
                         dim3(256), 0, e->stream, e->d_derived, e->st, e->sc, e->lxb, e->lyb);
    else
      hipLaunchKernelGGL(swarm::k_build_pairs<false>, dim3((unsigned)((e->n + 255) / 256), e->n_envs),
                         dim3(256), 0, e->stream, e->d_derived, e->st, e->sc, e->lxb, e->lyb);
    HIP_TRY(hipGetLastError());
  }
  if (e->sc.local_uf)
    hipLaunchKernelGGL((swarm::k_cluster_build<false, true>), dim3(e->n_envs), dim3(1024),
                       build_lds_bytes(e->n, e->sc.pair_cap), e->stream, e->st, e->sc);
  else
    hipLaunchKernelGGL((swarm::k_cluster_build<false, false>), dim3(e->n_envs), dim3(1024),
                       build_lds_bytes(e->n, e->sc.pair_cap), e->stream, e->st, e->sc);
  HIP_TRY(hipGetLastError());
  e->prebuilt = true;
  return SWARM_OK;
}

// The 2-D cluster window's run kernel (k_cluster_run_wide for latency-bound
// engines, else k_cluster_run) over the current decomposition.
constexpr int kMaxStamps = 512;  // captured run nodes with launch stamps

int launch_run(swarm_engine* e, int n_steps, unsigned long long* tstamp = nullptr) {
  const long waves = (long)e->n_envs * e->sc.wmax;
  const bool multi = e->params.n_species > 1;
  const bool walls = e->derived.n_walls != 0;
  if (e->wide_run) {
    // dynamic LDS beyond half a CU's keeps one block (run_wpb run waves) per CU
    const int R = e->run_wpb;
    // l1_pairs: the next window's candidate lists built beside the run
    const int ncb = e->sc.l1_pairs ? e->n_envs * ((e->n + 1023) / 1024) : 0;
    const dim3 grid((unsigned)(e->noise_blocks + ncb + (waves + R - 1) / R));
    // one block per CU; with rotation helpers (run_wpb <= 2, round 6) their
    // director tables in the dynamic LDS
    const int helpers = e->rot_helper && R <= 2 ? 1 : 0;
    const size_t lds = helpers ? std::max<size_t>(96 * 1024, R * swarm::helper_lds_bytes())
                               : 96 * 1024;
#define SWARM_WIDE(MULTI, WALLS)                                                             \
  hipLaunchKernelGGL((swarm::k_cluster_run_wide<MULTI, WALLS>), grid, dim3(1024), lds, e->stream, \
                     e->d_derived, e->st, e->sc, e->n_envs, n_steps, e->d_step, e->d_noise,      \
                     e->noise_blocks, R, ncb, e->lxb, e->lyb, tstamp, helpers)
    if (walls) {
      if (multi)
        SWARM_WIDE(true, true);
      else
        SWARM_WIDE(false, true);
    } else {
      if (multi)
        SWARM_WIDE(true, false);
      else
        SWARM_WIDE(false, false);
    }
#undef SWARM_WIDE
    e->next_table_ready = e->noise_blocks > 0;
  } else {
    // XCD-aware env placement (swarm::xcd_env_block) once the envs fill the
    // eight XCDs evenly (or nearly: 64 and more)
    const int E = e->n_envs;
    const int bpe = (e->sc.wmax + 3) / 4;
    const bool xcd = E >= 8 && (E % 8 == 0 || E >= 64);
    const dim3 run_grid((unsigned)(xcd ? 8 * ((E + 7) / 8) * bpe : (waves + 3) / 4)),
        run_block(256);
#define SWARM_RUN(MULTI, TABLE, WALLS)                                                     \
  hipLaunchKernelGGL((swarm::k_cluster_run<MULTI, TABLE, WALLS>), run_grid, run_block, 0,   \
                     e->stream, e->d_derived, e->st, e->sc, e->n_envs, n_steps, e->d_step,  \
                     e->d_noise, xcd ? bpe : 0, tstamp)
#define SWARM_RUN_W(MULTI, TABLE)      \
  do {                                 \
    if (walls)                         \
      SWARM_RUN(MULTI, TABLE, true);   \
    else                               \
      SWARM_RUN(MULTI, TABLE, false);  \
  } while (0)
    if (e->noise_table) {
      if (multi)
        SWARM_RUN_W(true, true);
      else
        SWARM_RUN_W(false, true);
    } else {
      if (multi)
        SWARM_RUN_W(true, false);
      else
        SWARM_RUN_W(false, false);
    }
#undef SWARM_RUN_W
#undef SWARM_RUN
    e->next_table_ready = false;
  }
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

// The 2-D cluster window's exact check (and re-run on failure).
// k_check takes each mover's candidates from the cells of the window's
// cell-sorted snapshot in global memory.
size_t sort_lds_bytes(const swarm_engine* e) {
  const size_t ncb = (size_t)1 << (e->lxb + e->lyb + e->lzb);
  return (16 + ((ncb + 4) & ~(size_t)3) + 3 * (size_t)e->sc.sort_stage_k) * 4;
}

// every 2-D build leaves its cell-sorted snapshot in global memory (k_build_env
// too), so the check searches the movers' candidate cells
int check_cell_lx(const swarm_engine* e) { return e->lxb; }
int check_cell_ly(const swarm_engine* e) { return e->lyb; }

int launch_check(swarm_engine* e, int n_steps) {
  hipLaunchKernelGGL(swarm::k_check, dim3(e->n_envs), dim3(1024),
                     check_lds_bytes(e->lxg, e->lyg, e->n, e->params.n_dims), e->stream,
                     e->d_derived, e->st, e->sc, n_steps, e->d_step, e->d_arrive, e->lxg, e->lyg,
                     0, check_cell_lx(e), check_cell_ly(e));
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

// One integration window: cluster build -> cluster run -> check/fallback.
// use_prebuilt: the build ran already; noise_ready: the noise table holds
// this many sub-steps from the current counter.
int launch_window(swarm_engine* e, int n_steps, bool use_prebuilt, int noise_ready) {
  if (!use_prebuilt) {
    const int rc = launch_build(e, e->stream);
    if (rc) return rc;
  }
  if (e->noise_table && !e->next_table_ready && n_steps > noise_ready) {
    const int rc = launch_noise(e, e->stream, n_steps);
    if (rc) return rc;
  }
  const long waves = (long)e->n_envs * e->sc.wmax;
  const bool multi = e->params.n_species > 1;
  const bool walls = e->derived.n_walls != 0;
  if (e->params.n_dims == 2 && e->nlist_path) {
    const long M = (long)e->n_envs * e->n;
    const int tpb = M <= 32768 ? 64 : 256;
    const dim3 grid((unsigned)(((M + tpb - 1) / tpb + 7) & ~7L));
    for (int s = 0; s < n_steps; ++s) {
#define SWARM_NL2(MULTI, WALLS)                                                               \
  hipLaunchKernelGGL((swarm::k_nl_step2<MULTI, WALLS>), grid, dim3(tpb), 0, e->stream,         \
                     e->d_derived, e->st, e->sc, n_steps, s, e->d_step)
      if (walls) {
        if (multi)
          SWARM_NL2(true, true);
        else
          SWARM_NL2(false, true);
      } else {
        if (multi)
          SWARM_NL2(true, false);
        else
          SWARM_NL2(false, false);
      }
#undef SWARM_NL2
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(swarm::k_check, dim3(e->n_envs), dim3(1024),
                       check_lds_bytes(e->lxg, e->lyg, e->n, e->params.n_dims), e->stream,
                       e->d_derived, e->st, e->sc, n_steps, e->d_step, e->d_arrive, e->lxg, e->lyg, 1,
                       check_cell_lx(e), check_cell_ly(e));
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  if (e->params.n_dims == 3 && e->nlist_path) {
    const long M = (long)e->n_envs * e->n;
    // latency-bound windows: one wave per workgroup (spread over more CUs);
    // a multiple of 8 workgroups (k_nl_step3's XCD-aware order)
    const int tpb = M <= 32768 ? 64 : 256;
    const dim3 grid((unsigned)(((M + tpb - 1) / tpb + 7) & ~7L));
    for (int s = 0; s < n_steps; ++s) {
#define SWARM_NL(MULTI, WALLS)                                                                \
  hipLaunchKernelGGL((swarm::k_nl_step3<MULTI, WALLS>), grid, dim3(tpb), 0, e->stream,         \
                     e->d_derived, e->st, e->sc, n_steps, s, e->d_step)
      if (walls) {
        if (multi)
          SWARM_NL(true, true);
        else
          SWARM_NL(false, true);
      } else {
        if (multi)
          SWARM_NL(true, false);
        else
          SWARM_NL(false, false);
      }
#undef SWARM_NL
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(swarm::k_check3, dim3(e->n_envs), dim3(1024), check3_lds_bytes(e), e->stream,
                       e->d_derived, e->st, e->sc, n_steps, e->d_step, e->d_arrive, e->lxg, e->lyg,
                       e->lzg, 1);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  if (e->params.n_dims == 3) {
    // one wave per block (so per CU) while the waves fit the chip, else four
    const int tpb = waves <= 256 ? 64 : 256;
    const dim3 grid((unsigned)((waves * 64 + tpb - 1) / tpb));
#define SWARM_RUN3(MULTI, WALLS)                                                              \
  hipLaunchKernelGGL((swarm::k_cluster_run3<MULTI, WALLS>), grid, dim3(tpb), 0, e->stream,     \
                     e->d_derived, e->st, e->sc, e->n_envs, n_steps, e->d_step)
    if (walls) {
      if (multi)
        SWARM_RUN3(true, true);
      else
        SWARM_RUN3(false, true);
    } else {
      if (multi)
        SWARM_RUN3(true, false);
      else
        SWARM_RUN3(false, false);
    }
#undef SWARM_RUN3
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(swarm::k_check3, dim3(e->n_envs), dim3(1024), check3_lds_bytes(e), e->stream,
                       e->d_derived, e->st, e->sc, n_steps, e->d_step, e->d_arrive, e->lxg, e->lyg,
                       e->lzg, 0);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool in_graph = false, events = false;
  if (e->profile) {
    // eager: HIP events around the run launch; under stream capture the run
    // node stamps itself (launch stamps below: event-record nodes put ~15 us
    // gaps into the replayed graph)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(e->stream, &cs));
    in_graph = cs == hipStreamCaptureStatusActive;
    events = !in_graph;
  }
  if (events) {
    HIP_TRY(hipEventCreate(&ev0));
    HIP_TRY(hipEventCreate(&ev1));
    HIP_TRY(hipEventRecord(ev0, e->stream));
  }
  unsigned long long* tstamp = nullptr;
  if (e->profile && in_graph && e->d_tstamp && e->stamp_next < kMaxStamps)
    tstamp = e->d_tstamp + (size_t)2 * swarm::kStampSub * e->stamp_next++;
  // the check and the launches up to the next run record their roles in
  // this run's slot (profiling under capture only)
  e->sc.rstamp = tstamp && e->d_rstamp
                     ? e->d_rstamp + (size_t)(e->stamp_next - 1) * 2 * swarm::kRoles *
                                         swarm::kStampSub
                     : nullptr;
  int rc = launch_run(e, n_steps, tstamp);
  if (rc) return rc;
  if (events) {
    HIP_TRY(hipEventRecord(ev1, e->stream));
    e->prof_events.emplace_back(ev0, ev1);
  }
  return launch_check(e, n_steps);
}

int run_bd(swarm_engine* e, int n_steps) {
  if (e->ride_stage > 0) {  // a deferred build no launch carried along
    const int rc = flush_ride_along(e);
    if (rc) return rc;
  }
  bool pre = e->prebuilt;
  int noise_ready = e->prebuilt_noise_steps;
  e->prebuilt = false;
  e->prebuilt_noise_steps = 0;
  while (n_steps > 0) {
    const int w = std::min(n_steps, swarm::kMaxWindow);
    const int rc = e->cluster_path ? launch_window(e, w, pre, noise_ready)
                                   : launch_global(e, w, 0, 0.0f, 0.0f);
    if (rc) return rc;
    pre = false;
    noise_ready = 0;
    n_steps -= w;
  }
  return SWARM_OK;
}

int ensure_grid_scratch(swarm_engine* e, int lx, int ly) {
  const size_t need = (size_t)e->n_envs * ((size_t)(1 << (lx + ly)) + 1);
  if (need > e->start_cap) {
    // the speculative vision grid's saved arguments point into the old buffer
    e->vgrid_ready = false;
    e->spec_ok = false;
    if (e->d_start) HIP_TRY(hipFree(e->d_start));
    HIP_TRY(hipMalloc(&e->d_start, need * sizeof(int32_t)));
    e->start_cap = need;
  }
  return SWARM_OK;
}

int build_grid(swarm_engine* e, int lx, int ly) {
  int rc = ensure_grid_scratch(e, lx, ly);
  if (rc) return rc;
  // this grid overwrites the cell starts a speculative vision grid left
  e->vgrid_ready = false;
  const int ncell = 1 << (lx + ly);
  const size_t lds = 16 * 4 + (size_t)(ncell + 1) * 4;
  if (lds > kMaxLds) return fail(SWARM_ECAPACITY, "observable cell grid too large");
  hipLaunchKernelGGL(k_grid_build, dim3(e->n_envs), dim3(1024), lds, e->stream, e->st, lx, ly,
                     e->d_start, e->d_order);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

void to_fixed(double x, double L, uint32_t* q, int32_t* img) {
  const double u = x / L;
  double fl = std::floor(u);
  double qd = std::nearbyint((u - fl) * kTwo32);
  if (qd >= kTwo32) {
    qd -= kTwo32;
    fl += 1.0;
  }
  *q = (uint32_t)qd;
  *img = (int32_t)fl;
}

// host copy of swarm::sincos_turn (same fp32 operation sequence)
void host_sincos_turn(uint32_t a, float* s_out, float* c_out) {
  const uint32_t b = a + 0x20000000u;
  const uint32_t quad = b >> 30;
  const int32_t rem = (int32_t)(b & 0x3FFFFFFFu) - 0x20000000;
  const float x = (float)rem * 1.46291807926715968e-09f;
  const float z = x * x;
  float sp = -1.9515295891e-4f;
  sp = sp * z;
  sp = sp + 8.3321608736e-3f;
  sp = sp * z;
  sp = sp + -1.6666654611e-1f;
  sp = sp * z;
  sp = sp * x;
  const float s = sp + x;
  float cp = 2.443315711809948e-5f;
  cp = cp * z;
  cp = cp + -1.388731625493765e-3f;
  cp = cp * z;
  cp = cp + 4.166664568298827e-2f;
  cp = cp * z;
  cp = cp * z;
  float c = cp - 0.5f * z;
  c = c + 1.0f;
  float so, co;
  switch (quad) {
    case 0: so = s; co = c; break;
    case 1: so = c; co = -s; break;
    case 2: so = -s; co = -c; break;
    default: so = -c; co = s; break;
  }
  *s_out = so;
  *c_out = co;
}

uint32_t angle_fixed(double dx, double dy) {
  const double phi = std::atan2(dy, dx);
  const int64_t a = (int64_t)std::nearbyint(phi / kTwoPi * kTwo32);
  return (uint32_t)(a & 0xFFFFFFFFLL);
}

}  // namespace

extern "C" {

const char* swarm_last_error(void) { return g_err.c_str(); }

#ifndef SWARM_BUILD_ID
#define SWARM_BUILD_ID "unknown"
#endif
const char* swarm_build_id(void) { return SWARM_BUILD_ID; }

int swarm_engine_create(const swarm_params_t* params, int32_t n_envs, int32_t n_particles,
                        const int32_t* species, swarm_engine_t** out) {
  if (!params || !out) return fail(SWARM_EINVAL, "null argument");
  *out = nullptr;
  if (params->n_dims != 2 && params->n_dims != 3)
    return fail(SWARM_EINVAL, "n_dims must be 2 or 3");
  if (n_envs < 1 || n_particles < 1) return fail(SWARM_EINVAL, "n_envs and n_particles must be >= 1");
  if (params->n_species < 1 || params->n_species > kMaxSpecies)
    return fail(SWARM_EINVAL, "n_species out of range");
  for (int a = 0; a < params->n_dims; ++a)
    if (!(params->box[a] > 0.0)) return fail(SWARM_EINVAL, "box lengths must be positive");
  // the run kernels' 1/r^2 (rcp_rn) is exact for r^2 in [2^-96, 2^96]: a
  // fixed-point grid step of at least 2^-48 and radii below 2^40
  for (int a = 0; a < params->n_dims; ++a)
    if (!(params->box[a] >= 0x1p-16)) return fail(SWARM_EINVAL, "box lengths must be >= 2^-16");
  if (!(params->time_step > 0.0)) return fail(SWARM_EINVAL, "time_step must be positive");
  for (int s = 0; s < params->n_species; ++s) {
    if (!(params->gamma_t[s] > 0.0) || !(params->gamma_r[s] > 0.0) || !(params->radius[s] >= 0.0))
      return fail(SWARM_EINVAL, "friction coefficients must be positive");
    if (!(params->radius[s] < 0x1p40)) return fail(SWARM_EINVAL, "radius must be < 2^40");
  }
  if (n_particles > (1 << 20))
    return fail(SWARM_ECAPACITY, "more than 2^20 particles per env are not supported");
  for (int i = 0; i < n_particles; ++i)
    if (species[i] < 0 || species[i] >= params->n_species)
      return fail(SWARM_EINVAL, "species index out of range");

  swarm_engine* e = new swarm_engine();
  e->params = *params;
  derive(*params, e->derived);
  e->n_envs = n_envs;
  e->n = n_particles;
  if (hipGetDevice(&e->device) != hipSuccess) {
    delete e;
    return fail(SWARM_EDEVICE, "no HIP device");
  }
  const bool three_d = params->n_dims == 3;
  if (three_d)
    cell_grid3(*params, n_particles, e->derived.rc_max, &e->lxg, &e->lyg, &e->lzg);
  else
    cell_grid(*params, n_particles, e->derived.rc_max, &e->lxg, &e->lyg);
  if (three_d)
    cell_grid3(*params, n_particles, e->derived.rc_max + skin_um(), &e->lxb, &e->lyb, &e->lzb);
  else
    cell_grid(*params, n_particles, e->derived.rc_max + skin_um(), &e->lxb, &e->lyb);
  const int lcb = e->lxb + e->lyb + e->lzb;  // build cells 2^lcb
  // static LDS of the kernels: pair tables (k_global, k_check, k_cluster_run)
  // and the link table of k_cluster_build
  constexpr size_t kStaticLds = sizeof(swarm::PairTables);
  if (check_lds_bytes(e->lxg, e->lyg, n_particles, params->n_dims) + kStaticLds > kMaxLds) {
    delete e;
    return fail(SWARM_ECAPACITY, "env cell grid does not fit the LDS of one workgroup");
  }
  // the cluster path needs the build workgroup's LDS and a non-degenerate
  // build grid; otherwise every window runs on the global path
  e->big_build = build_is_big(n_particles);
  e->sc.pair_cap = build_pair_cap(n_particles, e->big_build);
  // non-periodic boxes run windowed in 2-D and 3-D (edge cells and
  // unwrapped distances in the build and the exact check; a listed pair's
  // folded difference is its unwrapped one), the neighbour-list window is
  // periodic-only; SWARMRL_AMD_CLUSTER_PATH=0 forces the global path (A/B
  // and parity)
  e->sc.periodic = params->periodic ? 1 : 0;
  // block-local union-find in the 2-D pair search (SWARMRL_AMD_LOCAL_UF=0|1;
  // default: for envs above 4096 colloids, whose one-workgroup union phase
  // is long; at 4096 the pair search's block barriers cost more than the
  // union saves, measured)
  e->sc.local_uf = n_particles > 4096 ? 1 : 0;
  if (const char* olu = std::getenv("SWARMRL_AMD_LOCAL_UF")) e->sc.local_uf = olu[0] != '0';
  e->sc.rstamp = nullptr;
  e->sc.multi_species = params->n_species > 1 ? 1 : 0;
  // the 2-D build sort stages its scatter in LDS: the sorted rows of up to
  // K entries per pass beside the cell counts (K a multiple of 4, at least
  // N / 4)
  {
    const size_t counts = (16 + ((size_t)1 << (e->lxb + e->lyb)) + 1) * 4;
    const size_t room = counts + 4096 < kMaxLds ? kMaxLds - counts - 4096 : 0;
    const size_t k = std::min((size_t)n_particles, room / 12) & ~(size_t)3;
    e->sc.sort_stage_k = params->n_dims == 2 && n_particles <= 16 * 1024 &&
                                 4 * k >= (size_t)n_particles
                             ? (int32_t)k
                             : 0;
  }
  e->cluster_path = e->sc.pair_cap >= n_particles &&
                    n_particles < 65536 &&
                    swarm::build_lds_words_big(n_particles) * 4 <= kMaxLds &&
                    (size_t)(16 + (1 << lcb) + 1) * 4 <= kMaxLds &&
                    (1 << e->lxb) >= 3 && (1 << e->lyb) >= 3 && (!three_d || (1 << e->lzb) >= 3) &&
                    (!three_d || check3_lds_bytes(e) <= kMaxLds);
  {
    const char* oc = std::getenv("SWARMRL_AMD_CLUSTER_PATH");
    if (oc && oc[0] == '0') e->cluster_path = false;
  }
  if (e->cluster_path) {
    // mean number of colloids within 2 r_max + skin of one (deg): above ~2
    // in 3-D, ~3 in 2-D the links percolate into clusters wider than a wave
    // (3-D: re-run on the global path; 2-D: k_check's one-workgroup big
    // cluster run, then the global path), so the window runs on the
    // neighbour-list path instead.  SWARMRL_AMD_NLIST=0|1 overrides.
    double rmax = 0.0;
    for (int s = 0; s < params->n_species; ++s) rmax = std::max(rmax, params->radius[s]);
    const double link = 2.0 * rmax + skin_um();
    const double deg =
        three_d ? (double)n_particles / (params->box[0] * params->box[1] * params->box[2]) *
                      (2.0 / 3.0) * kTwoPi * link * link * link
                : (double)n_particles / (params->box[0] * params->box[1]) * 0.5 * kTwoPi * link *
                      link;
    e->nlist_path = deg > (three_d ? 2.0 : 3.0);
    const char* on = std::getenv("SWARMRL_AMD_NLIST");
    if (on && on[0] == '0') e->nlist_path = false;
    if (on && on[0] == '1') e->nlist_path = true;
    if (!params->periodic) e->nlist_path = false;  // the Verlet-list window is periodic-only
  }
  const size_t M = (size_t)n_envs * n_particles;
  int rc = SWARM_OK;
  rc = rc ? rc : dev_alloc(e, &e->st.q, 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.img, 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.ang, M);
  rc = rc ? rc : dev_alloc(e, &e->st.f_swim, M);
  rc = rc ? rc : dev_alloc(e, &e->st.torque_z, M);
  rc = rc ? rc : dev_alloc(e, &e->st.f_ext, 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.vel, 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.omega, M);
  e->own_f_swim = e->st.f_swim;
  e->own_torque_z = e->st.torque_z;
  rc = rc ? rc : dev_alloc(e, &e->st.species, (size_t)n_particles);
  rc = rc ? rc : dev_alloc(e, &e->d_derived, 1);
  rc = rc ? rc : dev_alloc(e, &e->d_box, 3);
  rc = rc ? rc : dev_alloc(e, &e->d_order, M);
  rc = rc ? rc : dev_alloc(e, &e->d_count, 1);
  rc = rc ? rc : dev_alloc(e, &e->d_step, swarm::kCtlWords);
  rc = rc ? rc : dev_alloc(e, &e->d_arrive, 1);
  // integrator scratch
  // One pair pass per wave and sub-step (k_cluster_build): the run kernel
  // lasts as long as its slowest waves, at any env count.  Latency-bound
  // launches (few envs x particles fill few SIMDs) also read their normals
  // from a table (k_noise; SWARMRL_AMD_NOISE_TABLE=0|1 overrides).
  const bool latency_bound = (long)n_envs * n_particles <= 32768;
  e->sc.one_pass = 1;
  // fewer, fuller waves only pay when the waves compete for the SIMDs; a
  // latency-bound launch has SIMDs to spare and a shorter build is worth more
  e->sc.fill_singletons = latency_bound ? 0 : 1;
  const int S = swarm::slots_per_env(n_particles, e->sc.one_pass != 0);
  e->sc.S = S;
  e->sc.wmax = S / 64;
  rc = rc ? rc : dev_alloc(e, &e->sc.sqx, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.sqy, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.sqz, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.simg, params->periodic ? 1 : 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.dir3, 3 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.torque_xy, 2 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.omega_xy, 2 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.wall_viol, 1);
  rc = rc ? rc : dev_alloc(e, &e->st.f_prev, 2 * M);  // two slots (window parity)
  rc = rc ? rc : dev_alloc(e, &e->st.tz_prev, 2 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.ang_prev, 2 * M);
  rc = rc ? rc : dev_alloc(e, &e->st.dir3_prev, three_d ? 6 * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->st.txy_prev, three_d ? 4 * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.nmov, (size_t)n_envs);
  rc = rc ? rc : dev_alloc(e, &e->sc.movers, (size_t)n_envs * swarm::kMaxMovers);
  rc = rc ? rc : dev_alloc(e, &e->sc.sidx, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.bq, (three_d ? 3 : 2) * M);
  rc = rc ? rc : dev_alloc(e, &e->sc.bimg, (three_d ? 3 : 2) * M);
  rc = rc ? rc : dev_alloc(e, &e->sc.bdir3, three_d ? 3 * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.bang, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.root, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.slot_of, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.perm, (size_t)n_envs * S);
  rc = rc ? rc : dev_alloc(e, &e->sc.pairs, (size_t)n_envs * (S / 64) * swarm::kPairsPerWave);
  rc = rc ? rc : dev_alloc(e, &e->sc.bsq, (three_d ? 3 : 2) * M);
  rc = rc ? rc : dev_alloc(e, &e->sc.nl, e->nlist_path ? (size_t)swarm::kNlMax * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.nn, e->nlist_path ? M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.qalt, e->nlist_path ? (three_d ? 3 : 2) * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.qa, e->nlist_path ? 2 * M : 1);
  rc = rc ? rc : dev_alloc(e, &e->sc.bsid, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.bcstart, (size_t)n_envs * ((1 << lcb) + 1));
  rc = rc ? rc : dev_alloc(e, &e->sc.gplist, (size_t)n_envs * std::max(e->sc.pair_cap, 1));
  rc = rc ? rc : dev_alloc(e, &e->sc.xpairs, (size_t)n_envs * std::max(e->sc.pair_cap, 1));
  rc = rc ? rc : dev_alloc(e, &e->sc.lroot, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.gnx, (size_t)n_envs);
  // chip-wide build sort of large 2-D envs (k_sort_count/scan/scatter):
  // per-cell counters (zero between builds) and each particle's cell / rank
  e->chip_sort = params->n_dims == 2 && n_particles > 4096;
  if (e->chip_sort) {
    rc = rc ? rc : dev_alloc(e, &e->sc.gcnt, (size_t)n_envs << (e->lxb + e->lyb));
    rc = rc ? rc : dev_alloc(e, &e->sc.gcell, M);
    rc = rc ? rc : dev_alloc(e, &e->sc.grank, M);
  }
  rc = rc ? rc : dev_alloc(e, &e->sc.gnpairs, (size_t)n_envs);
  // 2-D envs of the large-N build after the block-local pair search: the
  // build spread over the chip (k_mwb_*) instead of one workgroup, with a
  // fourth per-particle word (the offset of its pairs in the pair list)
  e->sc.bmisc = nullptr;
  const bool mwb = e->big_build && params->n_dims == 2 && e->sc.local_uf;
  if (e->big_build) rc = rc ? rc : dev_alloc(e, &e->sc.gclus, (mwb ? 4 : 3) * M);
  if (mwb) rc = rc ? rc : dev_alloc(e, &e->sc.bmisc, (size_t)n_envs * swarm::kBmWords);
  rc = rc ? rc : dev_alloc(e, &e->sc.wave_npairs, (size_t)n_envs * (S / 64));
  rc = rc ? rc : dev_alloc(e, &e->sc.phase, 32 + 4 * (size_t)n_envs * (S / 64));
  rc = rc ? rc : dev_alloc(e, &e->sc.disp, M);
  rc = rc ? rc : dev_alloc(e, &e->sc.env_waves, (size_t)n_envs);
  rc = rc ? rc : dev_alloc(e, &e->sc.fallback, (size_t)n_envs);
  rc = rc ? rc : dev_alloc(e, &e->sc.big_list, (size_t)n_envs * swarm::kBigMax);
  rc = rc ? rc : dev_alloc(e, &e->sc.big_pairs, (size_t)n_envs * swarm::kBigPairs);
  rc = rc ? rc : dev_alloc(e, &e->sc.big_n, (size_t)n_envs);
  rc = rc ? rc : dev_alloc(e, &e->sc.big_np, (size_t)n_envs);
  rc = rc ? rc : dev_alloc(e, &e->vs.rec, 2 * M);
  rc = rc ? rc : dev_alloc(e, &e->vs.agent_row, (size_t)n_particles);
  // noise table for latency-bound windows: few envs fill few SIMDs, so the
  // normals are better produced chip-wide ahead of the run.
  {
    const char* ov = std::getenv("SWARMRL_AMD_NOISE_TABLE");
    bool want = latency_bound;
    if (ov && ov[0] == '0') want = false;
    if (ov && ov[0] == '1') want = true;
    // 3-D and neighbour-list windows draw their normals in the kernels
    e->noise_table = want && e->derived.noisy && e->cluster_path && !three_d && !e->nlist_path;
    if (e->noise_table)
      rc = rc ? rc : dev_alloc(e, &e->d_noise, 2 * swarm::noise_table_words(M));
    // the one-launch build (one CU per env) for throughput-bound engines
    // when its sort region fits below the pair list; latency-bound ones keep
    // the three-launch build, whose pair search spreads over the chip
    // (one env: 42 us for the three launches, 52 us for k_build_env)
    {
      const int wm = S / 64;
      const size_t below = 16 + 16 + 3 * 68 + (size_t)((wm + 3) & ~3) + 4 * (size_t)n_particles;
      e->env_build = e->cluster_path && !e->big_build && !latency_bound && !three_d &&
                     !e->nlist_path && params->periodic &&
                     swarm::build_env_sort_words(n_particles, 1 << (e->lxb + e->lyb)) <= below;
      const char* ob = std::getenv("SWARMRL_AMD_ENV_BUILD");
      if (ob && ob[0] == '0') e->env_build = false;
      if (ob && ob[0] == '1')
        e->env_build = e->cluster_path && !e->big_build && !three_d && !e->nlist_path &&
                       params->periodic &&
                       swarm::build_env_sort_words(n_particles, 1 << (e->lxb + e->lyb)) <= below;
    }
    // one block per CU for latency-bound runs; beside a run of up to 16384
    // particles, 64 CUs produce the next window's table in its shadow (C5:
    // no k_noise launch between the policy and the run)
    e->wide_run = e->noise_table;
    // (32 noise workgroups above 4096 colloids, so that C4's 8 x 1024 gets one
    // run wave per CU, measured slower: C4 81.1 -> 72.9 M, same box)
    e->noise_blocks = e->wide_run && M <= 16384 ? 64 : 0;
    const char* orh = std::getenv("SWARMRL_AMD_ROT_HELPER");
    if (orh && orh[0] == '0') e->rot_helper = false;
    const char* ow = std::getenv("SWARMRL_AMD_WIDE_RUN");
    if (ow && ow[0] == '0') e->wide_run = false, e->noise_blocks = 0;
    // run waves per CU: a wave alone on its CU does not share the CU's
    // texture path with other waves' scattered noise-table gathers; four per
    // CU once the run's waves (~1 per 46 particles) would not fit one per CU
    {
      const long est = (long)M / 46 + 1;
      e->run_wpb = est + e->noise_blocks <= 224 ? 1 : (est / 2 + e->noise_blocks <= 256 ? 2 : 4);
    }
    // l1_pairs: the ride-along build's pair search moves into the slice's
    // first launch as a filter of candidate lists prepared during the last
    // run (periodic 2-D, the plain pair search, a build grid of at least 5
    // cells a side for the 5 x 5 candidate stencil)
    e->sc.l1_pairs = e->wide_run && e->cluster_path && !e->nlist_path && !e->env_build &&
                             !e->big_build && !three_d && params->periodic && !e->sc.local_uf &&
                             (1 << e->lxb) >= 5 && (1 << e->lyb) >= 5
                         ? 1
                         : 0;
    if (e->sc.l1_pairs) {
      // widening of the candidate radius: up to 1.5 um of motion per window
      // (the bench's swimmers move ~0.3 um; > 1.5 um is a > 6 sigma event),
      // at most half a cell side (the 5 x 5 stencil) and at least skin / 2
      // (k_check sees every particle that moved more: the movers)
      const double side = std::min(params->box[0] / (1 << e->lxb), params->box[1] / (1 << e->lyb));
      const double cd = std::max(0.5 * skin_um(), std::min(1.5, 0.5 * side));
      e->derived.cand_disp = (float)cd;
      for (int a = 0; a < params->n_species; ++a)
        for (int b = 0; b < params->n_species; ++b) {
          const double r = params->radius[a] + params->radius[b] + skin_um() + 2.0 * cd;
          e->derived.nbc2[a * kMaxSpecies + b] = (float)(r * r);
        }
      rc = rc ? rc : dev_alloc(e, &e->sc.cand, (size_t)swarm::kCandMax * M);
      rc = rc ? rc : dev_alloc(e, &e->sc.ncand, M);
    }
    rc = rc ? rc : dev_alloc(e, &e->sc.cand_ok, (size_t)n_envs);
    rc = rc ? rc : dev_alloc(e, &e->sc.cand_ovf, (size_t)n_envs);
    rc = rc ? rc : dev_alloc(e, &e->sc.sort_done, (size_t)n_envs);
    rc = rc ? rc : dev_alloc(e, &e->sc.stats, 4);

  }
  set_lds_attributes();
  if (rc) {
    swarm_engine_destroy(e);
    return rc;
  }
  e->st.n = n_particles;
  e->st.m = (int32_t)M;
  e->st.dims = params->n_dims;
  e->st.reuse = params->reuse_forces ? 1 : 0;
  std::vector<uint8_t> sp(n_particles);
  for (int i = 0; i < n_particles; ++i) sp[i] = (uint8_t)species[i];
  if (hipMemcpy(e->st.species, sp.data(), sp.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(e->d_derived, &e->derived, sizeof(Derived), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(e->d_box, params->box, 3 * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    swarm_engine_destroy(e);
    return fail(SWARM_EDEVICE, "initial upload failed");
  }
  *out = e;
  return SWARM_OK;
}

void swarm_engine_destroy(swarm_engine_t* e) {
  if (!e) return;
  (void)hipDeviceSynchronize();
  if (e->d_tstamp) (void)hipFree(e->d_tstamp);
  if (e->d_rstamp) (void)hipFree(e->d_rstamp);
  for (auto* v : {&e->prof_events, &e->graph_events, &e->graph_cal})
    for (auto& pr : *v) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (int k = 0; k < e->n_allocs; ++k) (void)hipFree(e->allocs[k]);
  if (e->d_start) (void)hipFree(e->d_start);
  if (e->d_pairs) (void)hipFree(e->d_pairs);
  if (e->traj_host) (void)hipHostFree(e->traj_host);
  if (e->d_traj_count) (void)hipFree(e->d_traj_count);
  delete e;
}

int swarm_engine_set_stream(swarm_engine_t* e, void* stream) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  e->stream = reinterpret_cast<hipStream_t>(stream);
  return SWARM_OK;
}

int swarm_engine_upload_raw(swarm_engine_t* e, const uint32_t* q, const int32_t* img,
                            const uint32_t* ang) {
  if (e) e->prebuilt = false, e->prebuilt_noise_steps = 0, e->ride_stage = 0;
  if (!e || !q || !img || !ang) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  HIP_TRY(hipMemcpyAsync(e->st.q, q, 3 * M * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->st.img, img, 3 * M * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipMemcpyAsync(e->st.ang, ang, M * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
  // a fresh state: the last force calculation saw these orientations (both
  // reuse_forces slots: the device window counter's parity is not known here)
  for (int k = 0; k < 2; ++k)
    HIP_TRY(hipMemcpyAsync(e->st.ang_prev + k * M, ang, M * sizeof(uint32_t),
                           hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_download_raw(swarm_engine_t* e, uint32_t* q, int32_t* img, uint32_t* ang) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  const size_t M = (size_t)e->st.m;
  if (q) HIP_TRY(hipMemcpyAsync(q, e->st.q, 3 * M * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  if (img) HIP_TRY(hipMemcpyAsync(img, e->st.img, 3 * M * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  if (ang) HIP_TRY(hipMemcpyAsync(ang, e->st.ang, M * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_upload_state(swarm_engine_t* e, const double* pos, const double* director) {
  if (!e || !pos || !director) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  std::vector<uint32_t> q(3 * M, 0u), ang(M);
  std::vector<int32_t> img(3 * M, 0);
  const int D = e->params.n_dims;
  std::vector<float> d3(D == 3 ? 3 * M : 0);
  for (size_t g = 0; g < M; ++g) {
    for (int a = 0; a < D; ++a) to_fixed(pos[3 * g + a], e->params.box[a], &q[a * M + g], &img[a * M + g]);
    ang[g] = angle_fixed(director[3 * g + 0], director[3 * g + 1]);
    if (D == 3) {
      const double* v = director + 3 * g;
      const double nm = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      for (int a = 0; a < 3; ++a) d3[a * M + g] = (float)(nm > 0.0 ? v[a] / nm : (a == 2));
    }
  }
  if (D == 3) {
    const int rc = swarm_engine_upload_directors(e, d3.data());
    if (rc) return rc;
  }
  return swarm_engine_upload_raw(e, q.data(), img.data(), ang.data());
}

int swarm_engine_download_state(swarm_engine_t* e, double* pos, double* director, double* velocity) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  const size_t M = (size_t)e->st.m;
  std::vector<uint32_t> q(3 * M), ang(M);
  std::vector<int32_t> img(3 * M);
  std::vector<float> vel(velocity ? 3 * M : 0);
  const int D = e->params.n_dims;
  std::vector<float> d3(D == 3 && director ? 3 * M : 0);
  if (!d3.empty())
    HIP_TRY(hipMemcpyAsync(d3.data(), e->st.dir3, 3 * M * sizeof(float), hipMemcpyDeviceToHost,
                           e->stream));
  HIP_TRY(hipMemcpyAsync(q.data(), e->st.q, 3 * M * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(img.data(), e->st.img, 3 * M * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(ang.data(), e->st.ang, M * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  if (velocity)
    HIP_TRY(hipMemcpyAsync(vel.data(), e->st.vel, 3 * M * sizeof(float), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (size_t g = 0; g < M; ++g) {
    if (pos) {
      for (int a = 0; a < 3; ++a)
        pos[3 * g + a] = a < D ? ((double)img[a * M + g] + (double)q[a * M + g] / kTwo32) *
                                     e->params.box[a]
                               : 0.0;
    }
    if (director && D == 3) {
      for (int a = 0; a < 3; ++a) director[3 * g + a] = d3[a * M + g];
    } else if (director) {
      float so, co;
      host_sincos_turn(ang[g], &so, &co);
      director[3 * g + 0] = co;
      director[3 * g + 1] = so;
      director[3 * g + 2] = 0.0;
    }
    if (velocity)
      for (int a = 0; a < 3; ++a) velocity[3 * g + a] = vel[a * M + g];
  }
  return SWARM_OK;
}

int swarm_engine_set_actions(swarm_engine_t* e, const float* f_swim, const float* torque_z,
                             int32_t on_device) {
  if (!e || !f_swim || !torque_z) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  if (on_device == 2) {
    // bind: later launches read the caller's buffers directly (zero copy);
    // the caller keeps them alive and unchanged until the next set_actions
    e->st.f_swim = const_cast<float*>(f_swim);
    e->st.torque_z = const_cast<float*>(torque_z);
    return SWARM_OK;
  }
  e->st.f_swim = e->own_f_swim;
  e->st.torque_z = e->own_torque_z;
  const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIP_TRY(hipMemcpyAsync(e->st.f_swim, f_swim, M * sizeof(float), kind, e->stream));
  HIP_TRY(hipMemcpyAsync(e->st.torque_z, torque_z, M * sizeof(float), kind, e->stream));
  if (!on_device) HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_set_external_force(swarm_engine_t* e, const double* f_ext) {
  if (!e || !f_ext) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  std::vector<float> f(3 * M);
  for (size_t g = 0; g < M; ++g)
    for (int a = 0; a < 3; ++a) f[a * M + g] = (float)f_ext[3 * g + a];
  HIP_TRY(hipMemcpyAsync(e->st.f_ext, f.data(), 3 * M * sizeof(float), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_set_directors(swarm_engine_t* e, const double* dir, const uint8_t* mask) {
  if (!e || !dir || !mask) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  if (e->params.n_dims == 3) {  // coll.director = new_direction (espresso.py:1238-1239)
    std::vector<float> d3(3 * M);
    HIP_TRY(hipMemcpyAsync(d3.data(), e->st.dir3, 3 * M * sizeof(float), hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (size_t g = 0; g < M; ++g) {
      if (!mask[g]) continue;
      const double* v = dir + 3 * g;
      const double nm = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      if (!(nm > 0.0)) return fail(SWARM_EINVAL, "new_direction must be non-zero");
      for (int a = 0; a < 3; ++a) d3[a * M + g] = (float)(v[a] / nm);
    }
    // the director only: with reuse_forces the next run's sub-step 0 still
    // swims along the director of the last force calculation (dir3_prev)
    HIP_TRY(hipMemcpyAsync(e->st.dir3, d3.data(), 3 * M * sizeof(float), hipMemcpyHostToDevice,
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return SWARM_OK;
  }
  std::vector<uint32_t> ang(M);
  HIP_TRY(hipMemcpyAsync(ang.data(), e->st.ang, M * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  for (size_t g = 0; g < M; ++g)
    if (mask[g]) ang[g] = angle_fixed(dir[3 * g + 0], dir[3 * g + 1]);
  HIP_TRY(hipMemcpyAsync(e->st.ang, ang.data(), M * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_remove_overlap(swarm_engine_t* e, int32_t n_steps, double gamma, double max_disp) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  e->prebuilt = false;
  e->ride_stage = 0;
  e->prebuilt_noise_steps = 0;
  if (n_steps <= 0) return SWARM_OK;
  return launch_global(e, n_steps, 1, (float)gamma, (float)max_disp);
}

int swarm_engine_integrate(swarm_engine_t* e, int32_t n_steps) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (n_steps < 0) return fail(SWARM_EINVAL, "n_steps must be >= 0");
  if (n_steps == 0) return SWARM_OK;
  return run_bd(e, n_steps);
}

namespace {
// Sum the event pairs (all recorded launches have run), destroy them.
int read_event_pairs(std::vector<std::pair<hipEvent_t, hipEvent_t>>& ev, double* total_ms,
                     int32_t* count) {
  double total = 0.0;
  int rc = SWARM_OK;
  for (auto& pr : ev) {
    float ms = 0.0f;
    if (rc == SWARM_OK) {
      hipError_t err = hipEventSynchronize(pr.second);
      if (err == hipSuccess) err = hipEventElapsedTime(&ms, pr.first, pr.second);
      if (err != hipSuccess) rc = fail(SWARM_EDEVICE, hipGetErrorString(err));
    }
    total += ms;
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (total_ms) *total_ms = total;
  if (count) *count = (int32_t)ev.size();
  ev.clear();
  return rc;
}
}  // namespace

int swarm_engine_profile(swarm_engine_t* e, int32_t enable, double* run_ms, int32_t* launches) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  const int rc = read_event_pairs(e->prof_events, run_ms, launches);
  e->profile = enable != 0;
  // the launch stamps of captured run nodes (allocated here: never under capture)
  if (e->profile && !e->d_tstamp)
    HIP_TRY(hipMalloc(&e->d_tstamp, 2 * (size_t)kMaxStamps * swarm::kStampSub *
                                        sizeof(unsigned long long)));
  if (e->profile && !e->d_rstamp)
    HIP_TRY(hipMalloc(&e->d_rstamp, 2 * (size_t)kMaxStamps * swarm::kRoles * swarm::kStampSub *
                                        sizeof(unsigned long long)));
  if (!e->profile) e->sc.rstamp = nullptr;
  return rc;
}

int swarm_engine_profile_graph(swarm_engine_t* e, int32_t release, float* ms_out, float* cal_out,
                               int32_t cap, int32_t* launches) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (cap < 0 || (cap > 0 && !ms_out)) return fail(SWARM_EINVAL, "ms_out needs cap entries");
  // the replay ran on a stream the engine does not know: wait for the device
  HIP_TRY(hipDeviceSynchronize());
  int rc = SWARM_OK;
  auto read = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, float* out) {
    int k = 0;
    for (auto& pr : v) {
      float ms = 0.0f;
      const hipError_t err = hipEventElapsedTime(&ms, pr.first, pr.second);
      if (err != hipSuccess && rc == SWARM_OK) rc = fail(SWARM_EDEVICE, hipGetErrorString(err));
      if (out && k < cap) out[k] = ms;
      ++k;
    }
    return k;
  };
  const int k = read(e->graph_events, ms_out);
  read(e->graph_cal, cal_out);
  if (launches) *launches = k;
  if (release) {
    for (auto* v : {&e->graph_events, &e->graph_cal}) {
      for (auto& pr : *v) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
      }
      v->clear();
    }
    e->stamp_next = 0;
  }
  return rc;
}

namespace {
// The (min start, max end) of each of `n` stamp records of kStampSub pairs.
void reduce_stamps(const std::vector<unsigned long long>& raw, int n,
                   std::vector<unsigned long long>* out) {
  out->assign(2 * (size_t)n, 0ull);
  for (int k = 0; k < n; ++k) {
    unsigned long long b = ~0ull, en = 0ull;
    for (int j = 0; j < swarm::kStampSub; ++j) {
      b = std::min(b, raw[2 * ((size_t)k * swarm::kStampSub + j)]);
      en = std::max(en, raw[2 * ((size_t)k * swarm::kStampSub + j) + 1]);
    }
    (*out)[2 * (size_t)k] = b;
    (*out)[2 * (size_t)k + 1] = en;
  }
}

// The run nodes' (start, end) stamps, reduced over their pairs.
int read_run_stamps(swarm_engine* e, std::vector<unsigned long long>* t) {
  const int n = e->stamp_next;
  HIP_TRY(hipDeviceSynchronize());
  std::vector<unsigned long long> raw(2 * (size_t)n * swarm::kStampSub);
  HIP_TRY(hipMemcpy(raw.data(), e->d_tstamp, raw.size() * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  reduce_stamps(raw, n, t);
  return SWARM_OK;
}

__global__ void k_stamp_reset(unsigned long long* t, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) {
    t[2 * k] = ~0ull;
    t[2 * k + 1] = 0ull;
  }
}
}  // namespace

int swarm_engine_profile_stamps(swarm_engine_t* e, int32_t reset, void* stream, float* ms_out,
                                int32_t cap, int32_t* launches) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  const int n = e->stamp_next;
  if (launches) *launches = n;
  if (!e->d_tstamp || n == 0) return SWARM_OK;
  if (reset) {
    const int nt = n * swarm::kStampSub;
    hipLaunchKernelGGL(k_stamp_reset, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), e->d_tstamp, nt);
    if (e->d_rstamp) {
      const int nr = n * swarm::kRoles * swarm::kStampSub;
      hipLaunchKernelGGL(k_stamp_reset, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0,
                         reinterpret_cast<hipStream_t>(stream), e->d_rstamp, nr);
    }
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  if (cap < 0 || (cap > 0 && !ms_out)) return fail(SWARM_EINVAL, "ms_out needs cap entries");
  std::vector<unsigned long long> t;
  int rc = read_run_stamps(e, &t);
  if (rc) return rc;
  int dev = 0, khz = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) return fail(SWARM_EDEVICE, "no wall clock rate");
  for (int k = 0; k < n && k < cap; ++k)
    ms_out[k] = t[2 * k + 1] > t[2 * k] ? (float)((double)(t[2 * k + 1] - t[2 * k]) / khz) : 0.0f;
  return SWARM_OK;
}

int swarm_engine_profile_roles(swarm_engine_t* e, double* us_out, int32_t cap,
                               int32_t* n_roles) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (n_roles) *n_roles = swarm::kRoles;
  const int n = e->stamp_next;
  if (cap < 0 || (cap > 0 && !us_out)) return fail(SWARM_EINVAL, "us_out needs cap entries");
  const size_t per = 2 * (size_t)swarm::kRoles;
  for (int32_t k = 0; k < cap; ++k) us_out[k] = std::nan("");
  if (!e->d_tstamp || !e->d_rstamp || n == 0) return SWARM_OK;
  std::vector<unsigned long long> t, r;
  int rc = read_run_stamps(e, &t);
  if (rc) return rc;
  std::vector<unsigned long long> raw(per * n * swarm::kStampSub);
  HIP_TRY(hipMemcpy(raw.data(), e->d_rstamp, raw.size() * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  reduce_stamps(raw, n * swarm::kRoles, &r);
  int dev = 0, khz = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) return fail(SWARM_EDEVICE, "no wall clock rate");
  const double us_per_tick = 1000.0 / khz;
  for (int k = 0; k < n; ++k) {
    const unsigned long long ref = t[2 * k + 1];  // end of the k-th run node
    if (ref == 0) continue;
    for (int q = 0; q < swarm::kRoles; ++q) {
      const unsigned long long b = r[per * k + 2 * q], en = r[per * k + 2 * q + 1];
      const size_t o = per * k + 2 * q;
      if (b == ~0ull || en == 0 || o + 1 >= (size_t)cap) continue;
      us_out[o] = ((double)b - (double)ref) * us_per_tick;
      us_out[o + 1] = ((double)en - (double)ref) * us_per_tick;
    }
  }
  return SWARM_OK;
}

int swarm_engine_time_run(swarm_engine_t* e, int32_t n_steps, int32_t reps, double* run_ms) {
  if (!e || !run_ms) return fail(SWARM_EINVAL, "null argument");
  if (n_steps < 1 || n_steps > swarm::kMaxWindow || reps < 1)
    return fail(SWARM_EINVAL, "1 <= n_steps <= 128 and reps >= 1");
  if (!e->cluster_path || e->nlist_path || e->params.n_dims != 2)
    return fail(SWARM_ESTATE, "swarm_engine_time_run times the 2-D cluster window only");
  if (e->prebuilt) {  // a pending side-stream build would race with this one
    HIP_TRY(hipDeviceSynchronize());
    e->prebuilt = false;
  }
  e->ride_stage = 0;  // a deferred build is superseded by the one below
  int rc = launch_build(e, e->stream);
  if (!rc && e->noise_table && !e->next_table_ready) rc = launch_noise(e, e->stream, n_steps);
  if (rc) return rc;
  hipEvent_t ev0, ev1;
  HIP_TRY(hipEventCreate(&ev0));
  HIP_TRY(hipEventCreate(&ev1));
  HIP_TRY(hipEventRecord(ev0, e->stream));
  for (int r = 0; r < reps && !rc; ++r) rc = launch_run(e, n_steps);
  HIP_TRY(hipEventRecord(ev1, e->stream));
  // the exact check restores a consistent state (the repeated windows ran on
  // one decomposition and their movers overflow the list: exact re-run)
  if (!rc) rc = launch_check(e, n_steps);
  float ms = 0.0f;
  hipError_t err = hipEventSynchronize(ev1);
  if (err == hipSuccess) err = hipEventElapsedTime(&ms, ev0, ev1);
  (void)hipEventDestroy(ev0);
  (void)hipEventDestroy(ev1);
  if (rc) return rc;
  if (err != hipSuccess) return fail(SWARM_EDEVICE, hipGetErrorString(err));
  *run_ms = (double)ms / reps;
  return SWARM_OK;
}

int swarm_engine_debug_phases(swarm_engine_t* e, uint64_t* out32) {
  if (!e || !out32) return fail(SWARM_EINVAL, "null argument");
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(out32, e->sc.phase, 32 * sizeof(uint64_t), hipMemcpyDeviceToHost));
#ifdef SWARM_PHASE_TIMING
  HIP_TRY(hipMemcpyFromSymbol(out32 + 24, HIP_SYMBOL(swarm::g_global_phase), 3 * sizeof(uint64_t)));
#endif
  return SWARM_OK;
}

int swarm_engine_debug_wave_stamps(swarm_engine_t* e, uint64_t* out, int32_t n_words) {
  if (!e || !out) return fail(SWARM_EINVAL, "null argument");
  const size_t cap = 4 * (size_t)e->n_envs * (e->sc.S / 64);
  if (n_words < 0 || (size_t)n_words > cap) return fail(SWARM_EINVAL, "n_words out of range");
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(out, e->sc.phase + 32, (size_t)n_words * sizeof(uint64_t),
                    hipMemcpyDeviceToHost));
  return SWARM_OK;
}

int swarm_engine_prebuild(swarm_engine_t* e, void* stream, int32_t n_steps_hint) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (n_steps_hint < 0) return fail(SWARM_EINVAL, "n_steps_hint must be >= 0");
  if (!e->cluster_path) return SWARM_OK;  // the global path has no build step
  const int rc = launch_build(e, stream ? reinterpret_cast<hipStream_t>(stream) : e->stream);
  if (rc) return rc;
  e->prebuilt = true;
  return SWARM_OK;
}

int swarm_engine_prebuild_noise(swarm_engine_t* e, void* stream, int32_t n_steps_hint) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (n_steps_hint < 0) return fail(SWARM_EINVAL, "n_steps_hint must be >= 0");
  if (!e->noise_table || n_steps_hint == 0) return SWARM_OK;
  if (e->next_table_ready) return SWARM_OK;  // filled beside the last run
  const int n = std::min<int>(n_steps_hint, swarm::kMaxWindow);
  const int rc = launch_noise(e, stream ? reinterpret_cast<hipStream_t>(stream) : e->stream, n);
  if (rc) return rc;
  e->prebuilt_noise_steps = n;
  return SWARM_OK;
}

int swarm_engine_build_stats(swarm_engine_t* e, uint64_t* out4, int32_t reset) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (!e->sc.stats) {  // (not a cluster-window engine)
    if (out4) std::memset(out4, 0, 4 * sizeof(uint64_t));
    return SWARM_OK;
  }
  if (out4) {
    HIP_TRY(hipMemcpyAsync(out4, e->sc.stats, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  if (reset) HIP_TRY(hipMemsetAsync(e->sc.stats, 0, 4 * sizeof(uint64_t), e->stream));
  return SWARM_OK;
}

int swarm_engine_window_stats(swarm_engine_t* e, int32_t* fallback, int32_t* waves) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  const size_t E = (size_t)e->n_envs;
  if (fallback)
    HIP_TRY(hipMemcpyAsync(fallback, e->sc.fallback, E * sizeof(int32_t), hipMemcpyDeviceToHost,
                           e->stream));
  if (waves)
    HIP_TRY(hipMemcpyAsync(waves, e->sc.env_waves, E * sizeof(int32_t), hipMemcpyDeviceToHost,
                           e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

// ---------------------------------------------------- trajectory ring
static size_t traj_entry_bytes(int n, int dims) {
  const size_t b = 8 + 4 * (size_t)n * (size_t)(3 * dims + (dims == 3 ? 3 : 1));
  return (b + 255) & ~(size_t)255;
}

int swarm_engine_traj_ring(swarm_engine_t* e, int32_t capacity, int32_t env, void** host_ring,
                           int64_t* entry_bytes) {
  if (!e || !host_ring || !entry_bytes) return fail(SWARM_EINVAL, "null argument");
  if (capacity < 1 || env < 0 || env >= e->n_envs)
    return fail(SWARM_EINVAL, "trajectory ring: capacity >= 1 and 0 <= env < n_envs");
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (e->traj_host) {
    HIP_TRY(hipHostFree(e->traj_host));
    e->traj_host = e->traj_dev = nullptr;
  }
  if (!e->d_traj_count) HIP_TRY(hipMalloc(&e->d_traj_count, sizeof(uint64_t)));
  HIP_TRY(hipMemset(e->d_traj_count, 0, sizeof(uint64_t)));
  const size_t eb = traj_entry_bytes(e->n, e->params.n_dims);
  const size_t bytes = 64 + eb * (size_t)capacity;
  void* h = nullptr;
  HIP_TRY(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h, 0, bytes);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return fail(SWARM_EDEVICE, "hipHostGetDevicePointer failed");
  }
  e->traj_host = reinterpret_cast<unsigned char*>(h);
  e->traj_dev = reinterpret_cast<unsigned char*>(d);
  e->traj_cap = capacity;
  e->traj_env = env;
  e->traj_entry = eb;
  *host_ring = h;
  *entry_bytes = (int64_t)eb;
  return SWARM_OK;
}

int swarm_engine_traj_record(swarm_engine_t* e) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (!e->traj_dev) return fail(SWARM_ESTATE, "no trajectory ring (swarm_engine_traj_ring)");
  hipLaunchKernelGGL(k_traj_write, dim3((unsigned)((e->n + 255) / 256)), dim3(256), 0, e->stream,
                     e->st, e->traj_env, e->traj_dev, e->traj_cap, e->traj_entry,
                     e->d_traj_count, e->d_step);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_traj_bump, dim3(1), dim3(64), 0, e->stream, e->d_traj_count, e->traj_dev);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

int swarm_traj_entry_to_host(const swarm_engine_t* e, const void* entry, double* pos,
                             double* director, double* velocity, uint64_t* step) {
  if (!e || !entry) return fail(SWARM_EINVAL, "null argument");
  const int N = e->n, D = e->params.n_dims;
  const unsigned char* b = reinterpret_cast<const unsigned char*>(entry);
  if (step) std::memcpy(step, b, 8);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(b + 8);
  const int32_t* img = reinterpret_cast<const int32_t*>(q + (size_t)D * N);
  const uint32_t* ang = reinterpret_cast<const uint32_t*>(img + (size_t)D * N);
  const float* d3 = reinterpret_cast<const float*>(ang);
  const float* vel = reinterpret_cast<const float*>(ang + (D == 3 ? (size_t)3 * N : (size_t)N));
  for (size_t g = 0; g < (size_t)N; ++g) {  // as swarm_engine_download_state
    if (pos)
      for (int a = 0; a < 3; ++a)
        pos[3 * g + a] = a < D ? ((double)img[a * N + g] + (double)q[a * N + g] / kTwo32) *
                                     e->params.box[a]
                               : 0.0;
    if (director && D == 3) {
      for (int a = 0; a < 3; ++a) director[3 * g + a] = d3[a * N + g];
    } else if (director) {
      float so, co;
      host_sincos_turn(ang[g], &so, &co);
      director[3 * g + 0] = co;
      director[3 * g + 1] = so;
      director[3 * g + 2] = 0.0;
    }
    if (velocity)
      for (int a = 0; a < 3; ++a) velocity[3 * g + a] = a < D ? vel[a * N + g] : 0.0;
  }
  return SWARM_OK;
}

int swarm_rnd_distance(const float* x, int32_t n, int32_t d_in, int32_t width,
                       const float* const* target, const float* const* predictor, int32_t order,
                       float* out, void* stream) {
  if (!x || !target || !predictor || !out) return fail(SWARM_EINVAL, "null argument");
  if (width != swarm::kRndWidth) return fail(SWARM_ECAPACITY, "RND width must be 32");
  if (d_in < 1 || d_in > swarm::kRndMaxIn) return fail(SWARM_ECAPACITY, "1 <= d_in <= 16");
  if (order < 1) return fail(SWARM_EINVAL, "distance order must be >= 1");
  swarm::RndPtrs tp, pp;
  for (int k = 0; k < 6; ++k) {
    if (!target[k] || !predictor[k]) return fail(SWARM_EINVAL, "null parameter");
    tp.w[k] = target[k];
    pp.w[k] = predictor[k];
  }
  if (n <= 0) return SWARM_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (d_in <= 4)
    hipLaunchKernelGGL(swarm::k_rnd_distance<4>, dim3(blocks), dim3(256), 0, s, x, n, d_in, tp,
                       pp, order, out);
  else
    hipLaunchKernelGGL(swarm::k_rnd_distance<16>, dim3(blocks), dim3(256), 0, s, x, n, d_in, tp,
                       pp, order, out);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

namespace {
// swarm_rnd_env_reward's workspace: the blocks' fp64 partials, then one
// ticket per env (zero between calls: the caller zeroes it once).
// Workgroups per env: one per 32-observation group (capping them at 64 or
// 128 so that each stages the networks once for several groups measured
// slower: C5 106.8 -> 100.9 M, same box).
int rnd_blocks(int per_env) {
  return (per_env + swarm::kRndObsPerBlock - 1) / swarm::kRndObsPerBlock;
}
size_t rnd_partials_bytes(int n_envs, int per_env) {
  return ((size_t)n_envs * rnd_blocks(per_env) * sizeof(double) + 255) & ~(size_t)255;
}
}  // namespace

int swarm_rnd_env_reward(const float* x, int32_t n_envs, int32_t per_env, int32_t d_in,
                         int32_t width, const float* const* target, const float* const* predictor,
                         int32_t order, int32_t clip, float clip_lo, float clip_hi,
                         const float* base, float* metric, float* env_reward, float* rewards,
                         void* workspace, int64_t workspace_bytes, void* stream) {
  if (!x || !target || !predictor || !metric || !env_reward || !rewards || !workspace)
    return fail(SWARM_EINVAL, "null argument");
  if (width != swarm::kRndWidth) return fail(SWARM_ECAPACITY, "RND width must be 32");
  if (d_in < 1 || d_in > swarm::kRndMaxIn) return fail(SWARM_ECAPACITY, "1 <= d_in <= 16");
  if (order < 1) return fail(SWARM_EINVAL, "distance order must be >= 1");
  if (n_envs < 0 || per_env < 0) return fail(SWARM_EINVAL, "n_envs, per_env >= 0");
  if (n_envs == 0 || per_env == 0) return SWARM_OK;
  const int kb = rnd_blocks(per_env);
  const size_t pb = rnd_partials_bytes(n_envs, per_env);
  if (workspace_bytes < (int64_t)(pb + (size_t)n_envs * sizeof(uint32_t)))
    return fail(SWARM_ECAPACITY, "workspace below swarm_rnd_env_workspace_bytes");
  swarm::RndPtrs tp, pp;
  for (int k = 0; k < 6; ++k) {
    if (!target[k] || !predictor[k]) return fail(SWARM_EINVAL, "null parameter");
    tp.w[k] = target[k];
    pp.w[k] = predictor[k];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* partial = static_cast<double*>(workspace);
  uint32_t* tickets = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + pb);
  const dim3 grid((unsigned)kb, (unsigned)n_envs);
  if (d_in <= 4)
    hipLaunchKernelGGL(swarm::k_rnd_env<4>, grid, dim3(256), 0, s, x, per_env, d_in, tp, pp,
                       order, clip ? 1 : 0, clip_lo, clip_hi, base, metric, env_reward, rewards,
                       partial, tickets);
  else
    hipLaunchKernelGGL(swarm::k_rnd_env<16>, grid, dim3(256), 0, s, x, per_env, d_in, tp, pp,
                       order, clip ? 1 : 0, clip_lo, clip_hi, base, metric, env_reward, rewards,
                       partial, tickets);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

int64_t swarm_rnd_env_workspace_bytes(int32_t n_envs, int32_t per_env) {
  if (n_envs < 0 || per_env < 0) return -1;
  return (int64_t)(rnd_partials_bytes(n_envs, per_env) + (size_t)n_envs * sizeof(uint32_t));
}

int64_t swarm_engine_step_count(const swarm_engine_t* e) {
  if (!e) return -1;
  uint64_t v = 0;
  if (hipMemcpyAsync(&v, e->d_step, sizeof(v), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess)
    return -1;
  return (int64_t)v;
}

int swarm_engine_device_views(swarm_engine_t* e, swarm_device_views_t* v) {
  if (!e || !v) return fail(SWARM_EINVAL, "null argument");
  v->q = e->st.q;
  v->img = e->st.img;
  v->ang = e->st.ang;
  v->f_swim = e->st.f_swim;
  v->torque_z = e->st.torque_z;
  v->f_ext = e->st.f_ext;
  v->vel = e->st.vel;
  v->omega_z = e->st.omega;
  v->species = e->st.species;
  v->n_envs = e->n_envs;
  v->n_particles = e->n;
  v->n_dims = e->params.n_dims;
  v->dir3 = e->st.dir3;
  v->torque_xy = e->st.torque_xy;
  v->omega_xy = e->st.omega_xy;
  return SWARM_OK;
}

namespace {
bool same_grid_args(const VisionArgs& a, const VisionArgs& b) {
  return std::memcmp(&a.vp, &b.vp, sizeof(a.vp)) == 0 && a.lx == b.lx && a.ly == b.ly &&
         a.radii == b.radii && a.types == b.types && a.agents == b.agents &&
         a.n_agents == b.n_agents && a.n_envs == b.n_envs;
}

// LDS of a launch carrying the l1_pairs pair search (its fallback tables)
// beside workgroups that need `other` bytes.
size_t l1_launch_lds(const swarm_engine* e, size_t other) {
  return e->sc.l1_pairs ? std::max(other, l1_role_lds_bytes()) : other;
}
int l1_blocks_per_env(const swarm_engine* e) { return e->sc.l1_pairs ? (e->n + 1023) / 1024 : 0; }

// pol (swarm_engine_vision_policy): the rollout policy of the cone's agents
// runs in the cone's launch (PolicyTail); the caller checked its limits
// (n_cones * n_types <= 4 = d_in, k <= 4, hidden <= 256).
int vision_cone_impl(swarm_engine_t* e, const swarm_vision_params_t* vp, const int32_t* agent_idx,
                     int32_t n_agents, const float* radii, const int32_t* types, float* out,
                     bool persistent, const swarm::MlpArgs* pol = nullptr) {
  if (!e || !vp || !agent_idx || !radii || !types || !out) return fail(SWARM_EINVAL, "null argument");
  if (e->params.n_dims != 2) return fail(SWARM_EINVAL, "the vision-cone kernel is 2-D only");
  if (vp->n_cones < 1 || vp->n_cones > SWARM_MAX_CONES || vp->n_types < 1 ||
      vp->n_types > SWARM_MAX_DETECTED_TYPES || vp->n_cones * vp->n_types > 2 * SWARM_MAX_CONES)
    return fail(SWARM_ECAPACITY, "n_cones * n_types exceeds this build's limit (32)");
  if (n_agents <= 0) return SWARM_OK;
  if (e->n >= (1 << 24)) return fail(SWARM_ECAPACITY, "vision records hold particle ids < 2^24");
  // a range of half the box or more: every record is a candidate (k_vision<.., kAll>)
  const bool all = !(2.0 * vp->vision_range < std::min(e->params.box[0], e->params.box[1]));
  int lx, ly;
  cell_grid(e->params, e->n, (double)vp->vision_range, &lx, &ly);
  int rc = ensure_grid_scratch(e, lx, ly);
  if (rc) return rc;
  // records staged in LDS when the env's fit (N <= 8 x 1024: the register path)
  const bool staged = e->n <= 8 * 1024 && vision_grid_lds_bytes(lx, ly, e->n, true) <= kMaxLds;
  const VisionArgs va{*vp,          lx,        ly,    radii, types, agent_idx, n_agents,
                      e->d_start,   e->vs,     out,   e->n_envs, staged ? 1 : 0, e->sc.rstamp};
  const long total = (long)e->n * e->n_envs;  // one group per sorted particle
  const int nb = vp->n_cones * vp->n_types;
  // lanes per agent: enough threads to give every SIMD a few waves, few
  // enough that the lanes of a wave stay busy (measured, tools/vision_time.py:
  // 64 x 4096 agents 107 -> 93 us with G = 4 instead of 1)
  constexpr int kVisionGWide = 4;
  int G = total >= (1L << 15) ? kVisionGWide : 16;
  if (const char* og = std::getenv("SWARMRL_AMD_VISION_G")) {
    const int v = std::atoi(og);
    if (v == kVisionGWide || v == 16) G = v;
  }
  const size_t glds = vision_grid_lds_bytes(lx, ly, e->n, staged);
  if (glds > kMaxLds) return fail(SWARM_ECAPACITY, "observable cell grid too large");
  // the grid of the current positions for these arguments, built by the
  // reward launch (launch_field) while nothing moved the colloids since
  const bool l1 = e->sc.l1_pairs != 0;
  const bool have_grid = !all && e->vgrid_ready && e->ride_stage == (l1 ? 3 : 2) &&
                         same_grid_args(e->spec_va, va);
  e->vgrid_ready = false;
  e->spec_ok = persistent && !all;
  if (e->spec_ok) e->spec_va = va;
  // a deferred build rides along in the grid and cone launches (stages 1, 2;
  // with l1_pairs the pair search rides in the grid's launch and the
  // cluster build, stage 3, in the fused policy's or the policy's launch)
  // when their fused variants apply; else its pending stages launch first
  const bool ride_ok = !all && nb <= 4 && G == 16;
  if (e->ride_stage > 0 && !(ride_ok && (e->ride_stage <= 2 || (l1 && e->ride_stage == 3)))) {
    rc = flush_ride_along(e);
    if (rc) return rc;
  }
  if (e->ride_stage == 1) {  // grid | sort (| pairs), then cone | pairs or cluster build
    const size_t slds = sort_lds_bytes(e);
    const int nfb = l1_blocks_per_env(e);
    const dim3 grid((unsigned)((2 + nfb) * e->n_envs));
    const size_t lds = l1_launch_lds(e, std::max(glds, slds));
    if (e->n > 4096)
      hipLaunchKernelGGL((k_vgrid_sort<16>), grid, dim3(1024), lds, e->stream, e->st, va, e->sc,
                         e->lxb, e->lyb, e->d_derived, nfb, e->d_step);
    else
      hipLaunchKernelGGL((k_vgrid_sort<4>), grid, dim3(1024), lds, e->stream, e->st, va, e->sc,
                         e->lxb, e->lyb, e->d_derived, nfb, e->d_step);
    HIP_TRY(hipGetLastError());
    e->ride_stage = l1 ? 3 : 2;
  } else if (!have_grid) {
    hipLaunchKernelGGL(k_vision_grid, dim3(e->n_envs), dim3(1024), glds, e->stream, e->st, va);
    HIP_TRY(hipGetLastError());
  }
  if (pol && ride_ok && e->ride_stage == 3) {  // cluster build | cone + policy (l1_pairs)
    // 32 lanes per agent: with the actor rows staged in LDS the cone's bins
    // are summed ~1.5 us sooner and the MLP tail no longer outweighs it
    // (same box: head 53.1 -> 53.3 M, C2 14.5 -> 14.8 M; with the rows read
    // from L2 the tail took ~2 us longer and 16 lanes won)
    constexpr int GC = 32;
    const int ncb = (int)((total * GC + 1023) / 1024);
    const size_t rows = ((size_t)pol->hidden * swarm::MlpRow<4, 4>::kStride + 4) * sizeof(float);
    const size_t lds = std::max(build_lds_bytes(e->n, e->sc.pair_cap),
                                (size_t)kVisionHits * 1024 * sizeof(uint32_t) + rows);
    hipLaunchKernelGGL((k_vision_policy_cbuild<4, GC, 4, 4>), dim3((unsigned)(e->n_envs + ncb)),
                       dim3(1024), lds, e->stream, e->st, e->d_derived, va, *pol, e->sc);
    HIP_TRY(hipGetLastError());
    e->ride_stage = 0;
    e->prebuilt = true;
    return SWARM_OK;
  }
  if (pol && e->ride_stage == 2) {  // pairs | cone + policy
    const int nvb = (int)((total * 16 + 255) / 256);
    const int pbx = (e->n + 255) / 256;
    const int npb = pbx * e->n_envs;
    const dim3 grid((unsigned)(nvb + npb));
    if (e->sc.local_uf)
      hipLaunchKernelGGL((k_vision_policy_pairs<4, 16, true, 4, 4>), grid, dim3(256), 0,
                         e->stream, e->st, e->d_derived, va, *pol, npb, e->sc, e->lxb, e->lyb, pbx);
    else
      hipLaunchKernelGGL((k_vision_policy_pairs<4, 16, false, 4, 4>), grid, dim3(256), 0,
                         e->stream, e->st, e->d_derived, va, *pol, npb, e->sc, e->lxb, e->lyb, pbx);
    HIP_TRY(hipGetLastError());
    e->ride_stage = 3;
    return SWARM_OK;
  }
  if (e->ride_stage == 2) {  // pairs | cone
    const int nvb = (int)((total * 16 + 255) / 256);
    const int pbx = (e->n + 255) / 256;
    const int npb = pbx * e->n_envs;
    const dim3 grid((unsigned)(nvb + npb));
    if (e->sc.local_uf)
      hipLaunchKernelGGL((k_vision_pairs<4, 16, true>), grid, dim3(256), 0, e->stream, e->st,
                         e->d_derived, va, npb, e->sc, e->lxb, e->lyb, pbx);
    else
      hipLaunchKernelGGL((k_vision_pairs<4, 16, false>), grid, dim3(256), 0, e->stream, e->st,
                         e->d_derived, va, npb, e->sc, e->lxb, e->lyb, pbx);
    HIP_TRY(hipGetLastError());
    e->ride_stage = 3;
    return SWARM_OK;
  }
  if (all) {
    if (pol) return fail(SWARM_ECAPACITY, "the fused policy needs vision_range < half the box");
    const dim3 agrid((unsigned)((total * 16 + 255) / 256)), ablock(256);
#define SWARM_VALL(NBV)                                                                          \
  hipLaunchKernelGGL((k_vision<NBV, 16, true>), agrid, ablock, 0, e->stream, e->st, e->d_derived, \
                     va, 0)
    if (nb <= 4) {
      SWARM_VALL(4);
    } else if (nb <= 8) {
      SWARM_VALL(8);
    } else if (nb <= 16) {
      SWARM_VALL(16);
    } else {
      SWARM_VALL(32);
    }
#undef SWARM_VALL
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
  // XCD-aware env placement once the envs fill the eight XCDs (as k_cluster_run)
  const int E = e->n_envs;
  const int bpe = (int)(((long)e->n * G + 255) / 256);
  const bool xcd = E >= 8 && (E % 8 == 0 || E >= 64);
  const dim3 grid((unsigned)(xcd ? 8L * ((E + 7) / 8) * bpe : (total * G + 255) / 256)),
      block(256);
  if (pol) {  // cone + policy, no build stage riding along
    if (G == kVisionGWide)
      hipLaunchKernelGGL((k_vision_policy<4, kVisionGWide, 4, 4>), grid, block, 0, e->stream,
                         e->st, e->d_derived, va, *pol, xcd ? bpe : 0);
    else
      hipLaunchKernelGGL((k_vision_policy<4, 16, 4, 4>), grid, block, 0, e->stream, e->st,
                         e->d_derived, va, *pol, xcd ? bpe : 0);
    HIP_TRY(hipGetLastError());
    return SWARM_OK;
  }
#define SWARM_VISION(NBV, GV)                                                                  \
  hipLaunchKernelGGL((k_vision<NBV, GV>), grid, block, 0, e->stream, e->st, e->d_derived, va, \
                     xcd ? bpe : 0)
#define SWARM_VISION_G(NBV)                      \
  if (G == kVisionGWide)                  \
    SWARM_VISION(NBV, kVisionGWide);      \
  else                                           \
    SWARM_VISION(NBV, 16)
  if (nb <= 4) {
    SWARM_VISION_G(4);
  } else if (nb <= 8) {
    SWARM_VISION_G(8);
  } else if (nb <= 16) {
    SWARM_VISION_G(16);
  } else {
    SWARM_VISION_G(32);
  }
#undef SWARM_VISION_G
#undef SWARM_VISION
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}
}  // namespace

int swarm_vision_cone(swarm_engine_t* e, const swarm_vision_params_t* vp, const int32_t* agent_idx,
                      int32_t n_agents, const float* radii, const int32_t* types, float* out) {
  return vision_cone_impl(e, vp, agent_idx, n_agents, radii, types, out, false);
}

int swarm_vision_cone_persistent(swarm_engine_t* e, const swarm_vision_params_t* vp,
                                 const int32_t* agent_idx, int32_t n_agents, const float* radii,
                                 const int32_t* types, float* out) {
  return vision_cone_impl(e, vp, agent_idx, n_agents, radii, types, out, true);
}

namespace {
int policy_launch(const float* obs, int32_t n, int32_t d_in, const float* w1, const float* b1,
                  int32_t hidden, const float* w2, const float* b2, int32_t k, uint64_t seed,
                  uint64_t* state, int32_t n_state, float explore_p, const float* f_table,
                  const float* t_table, int64_t* out_idx, float* out_logp, float* out_f,
                  float* out_t, float* out_logits, void* stream, swarm_engine* ride);
}  // namespace

int swarm_engine_vision_policy(swarm_engine_t* e, const swarm_vision_params_t* vp,
                               const int32_t* agent_idx, int32_t n_agents, const float* radii,
                               const int32_t* types, float* features, const float* w1,
                               const float* b1, int32_t hidden, const float* w2, const float* b2,
                               int32_t k, uint64_t seed, uint64_t* agent_state, int32_t n_state,
                               float explore_p, const float* f_table, const float* t_table,
                               int64_t* out_idx, float* out_logp, float* out_f, float* out_t,
                               float* out_logits) {
  if (!e || !vp || !w1 || !b1 || !w2 || !b2 || !agent_state || !f_table || !t_table || !out_idx ||
      !out_logp || !out_f || !out_t)
    return fail(SWARM_EINVAL, "null argument");
  const int nb = vp->n_cones * vp->n_types;
  if (nb < 1 || nb > 4) return fail(SWARM_ECAPACITY, "the fused policy takes <= 4 cone bins");
  if (hidden < 1 || hidden > swarm::kMlpMaxHidden)
    return fail(SWARM_ECAPACITY, "1 <= hidden <= 256");
  if (k < 1 || k > 4) return fail(SWARM_ECAPACITY, "the fused policy takes 1 <= k <= 4 actions");
  if (!(explore_p >= 0.0f && explore_p <= 1.0f))
    return fail(SWARM_EINVAL, "exploration probability must be in [0, 1]");
  if (n_agents <= 0) return SWARM_OK;
  const long n = (long)e->n_envs * n_agents;
  if (n_state < n) return fail(SWARM_EINVAL, "agent_state needs one counter per agent");
  const swarm::MlpArgs m{features, (int)n, nb, w1, b1, hidden, w2, b2, k, (uint32_t)seed,
                         (uint32_t)(seed >> 32), reinterpret_cast<unsigned long long*>(agent_state),
                         explore_p, f_table, t_table, out_idx, out_logp, out_f, out_t, out_logits};
  if (!e->wide_run) {
    // throughput-bound engines (many envs): the cone is VALU-bound and the
    // MLP's four lanes per agent would lengthen every group; the two kernels
    // of the calls this replaces, the policy drawing with the first
    // ceil(n / 64) counters as its group counters
    const int rc = vision_cone_impl(e, vp, agent_idx, n_agents, radii, types, features, true);
    if (rc) return rc;
    return policy_launch(features, (int32_t)n, nb, w1, b1, hidden, w2, b2, k, seed, agent_state,
                         n_state, explore_p, f_table, t_table, out_idx, out_logp, out_f, out_t,
                         out_logits, e->stream, e);
  }
  return vision_cone_impl(e, vp, agent_idx, n_agents, radii, types, features, true, &m);
}

namespace {
// k_field, or with a pending deferred build and a persistent vision cone the
// fused k_field_vgrid_sort (stage 1 and the next observable's grid ride
// along in the reward launch).
int launch_field(swarm_engine* e, const FieldArgs& f) {
  const int total = f.n_agents * e->n_envs;
  // the reward launch of a slice with a deferred build carries stage 1 (and
  // the l1_pairs pair search), and for a persistent vision cone the next
  // observable's grid; without a vision cone only with l1_pairs (the
  // cluster build then rides in the policy launch: k_policy_cbuild)
  const bool grid_too = e->spec_ok;
  if (e->ride_stage == 1 && (grid_too || e->sc.l1_pairs)) {
    VisionArgs none{};
    none.n_envs = e->n_envs;
    const VisionArgs& va = grid_too ? e->spec_va : none;
    const size_t glds = grid_too ? vision_grid_lds_bytes(va.lx, va.ly, e->n, va.staged != 0) : 0;
    const size_t slds = sort_lds_bytes(e);
    const int nfb = (total + 1023) / 1024;
    const int npf = l1_blocks_per_env(e);  // l1_pairs: the pair search rides here too
    const dim3 grid((unsigned)(nfb + (2 + npf) * e->n_envs));
    const size_t lds = l1_launch_lds(e, std::max(glds, slds));
    if (e->n > 4096)
      hipLaunchKernelGGL((k_field_vgrid_sort<16>), grid, dim3(1024), lds, e->stream, f, nfb,
                         e->st, va, e->sc, e->lxb, e->lyb, e->d_derived, npf, e->d_step,
                         grid_too ? 1 : 0);
    else
      hipLaunchKernelGGL((k_field_vgrid_sort<4>), grid, dim3(1024), lds, e->stream, f, nfb,
                         e->st, va, e->sc, e->lxb, e->lyb, e->d_derived, npf, e->d_step,
                         grid_too ? 1 : 0);
    HIP_TRY(hipGetLastError());
    e->ride_stage = e->sc.l1_pairs ? 3 : 2;
    e->vgrid_ready = grid_too;
    return SWARM_OK;
  }
  hipLaunchKernelGGL(k_field, dim3((total + 255) / 256), dim3(256), 0, e->stream, e->st, f);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}
}  // namespace

int swarm_field_distance(swarm_engine_t* e, const int32_t* agent_idx, int32_t n_agents,
                         const double source[3], const double box_scale[3], uint32_t* hist_q,
                         int32_t* hist_img, float* d_cur, float* d_prev, int32_t update_history,
                         int32_t init_only) {
  if (!e || !agent_idx || !hist_q || !hist_img) return fail(SWARM_EINVAL, "null argument");
  if (!init_only && (!d_cur || !d_prev || !source || !box_scale)) return fail(SWARM_EINVAL, "null argument");
  if (n_agents <= 0) return SWARM_OK;
  const double s[3] = {source ? source[0] : 0.0, source ? source[1] : 0.0, source ? source[2] : 0.0};
  const double b[3] = {box_scale ? box_scale[0] : 1.0, box_scale ? box_scale[1] : 1.0,
                       box_scale ? box_scale[2] : 1.0};
  const FieldArgs f{e->d_box, agent_idx, n_agents, s[0], s[1], s[2], b[0], b[1], b[2], hist_q,
                    hist_img, d_cur, d_prev, update_history, init_only, e->n_envs, 0, 0.0f, 0.0f,
                    0.0f, nullptr};
  return launch_field(e, f);
}

int swarm_field_transform(swarm_engine_t* e, const int32_t* agent_idx, int32_t n_agents,
                          const double source[3], const double box_scale[3], uint32_t* hist_q,
                          int32_t* hist_img, float decay_a, float decay_b, float scale,
                          int32_t clip_at_zero, float* out) {
  if (!e || !agent_idx || !hist_q || !hist_img || !source || !box_scale || !out)
    return fail(SWARM_EINVAL, "null argument");
  if (n_agents <= 0) return SWARM_OK;
  const FieldArgs f{e->d_box, agent_idx, n_agents, source[0], source[1], source[2],
                    box_scale[0], box_scale[1], box_scale[2], hist_q, hist_img, nullptr, nullptr,
                    1, 0, e->n_envs, clip_at_zero ? 2 : 1, decay_a, decay_b, scale, out};
  return launch_field(e, f);
}

int swarm_pair_distances(swarm_engine_t* e, const int32_t* agent_idx, int32_t n_agents,
                         const int32_t* sensed_idx, int32_t m0, int32_t mc,
                         const double box_scale[3], float* out) {
  if (!e || !agent_idx || !sensed_idx || !box_scale || !out)
    return fail(SWARM_EINVAL, "null argument");
  if (m0 < 0 || mc < 0) return fail(SWARM_EINVAL, "negative sensed range");
  if (n_agents <= 0 || mc == 0) return SWARM_OK;
  const dim3 grid((unsigned)((n_agents + 255) / 256), (unsigned)((mc + 255) / 256),
                  (unsigned)e->n_envs);
  hipLaunchKernelGGL(k_pair_dist, grid, dim3(256), 0, e->stream, e->st, e->d_box, agent_idx,
                     n_agents, sensed_idx, m0, mc, (float)box_scale[0], (float)box_scale[1],
                     (float)box_scale[2], out);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

int swarm_engine_neighbor_pairs(swarm_engine_t* e, int32_t env, double cutoff, int32_t* pairs,
                                int32_t max_pairs, int32_t* n_pairs) {
  if (!e || !pairs || !n_pairs) return fail(SWARM_EINVAL, "null argument");
  if (env < 0 || env >= e->n_envs) return fail(SWARM_EINVAL, "env out of range");
  if (e->params.n_dims != 2) return fail(SWARM_EINVAL, "neighbor_pairs is 2-D only");
  if (!(2.0 * cutoff < std::min(e->params.box[0], e->params.box[1])))
    return fail(SWARM_EINVAL, "cutoff must be below half the box length");
  int lx, ly;
  cell_grid(e->params, e->n, cutoff, &lx, &ly);
  int rc = build_grid(e, lx, ly);
  if (rc) return rc;
  if ((size_t)max_pairs > e->pairs_cap) {
    if (e->d_pairs) HIP_TRY(hipFree(e->d_pairs));
    HIP_TRY(hipMalloc(&e->d_pairs, 2 * (size_t)std::max(max_pairs, 1) * sizeof(int32_t)));
    e->pairs_cap = (size_t)max_pairs;
  }
  HIP_TRY(hipMemsetAsync(e->d_count, 0, sizeof(int32_t), e->stream));
  const float c2 = (float)(cutoff * cutoff);
  hipLaunchKernelGGL(k_pairs, dim3((e->n + 255) / 256), dim3(256), 0, e->stream, e->st,
                     e->d_derived, env, c2, lx, ly, e->d_start, e->d_order, e->d_pairs, max_pairs,
                     e->d_count);
  HIP_TRY(hipGetLastError());
  int32_t cnt = 0;
  HIP_TRY(hipMemcpyAsync(&cnt, e->d_count, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  *n_pairs = cnt;
  const int32_t got = std::min(cnt, max_pairs);
  if (got > 0)
    HIP_TRY(hipMemcpy(pairs, e->d_pairs, 2 * (size_t)got * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (cnt > max_pairs) return fail(SWARM_ECAPACITY, "more pairs than max_pairs");
  return SWARM_OK;
}

int swarm_engine_set_torque_xy(swarm_engine_t* e, const float* torque_xy, int32_t on_device) {
  if (!e || !torque_xy) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIP_TRY(hipMemcpyAsync(e->st.torque_xy, torque_xy, 2 * M * sizeof(float), kind, e->stream));
  if (!on_device) HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_upload_directors(swarm_engine_t* e, const float* dir3) {
  if (!e || !dir3) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  HIP_TRY(hipMemcpyAsync(e->st.dir3, dir3, 3 * M * sizeof(float), hipMemcpyHostToDevice,
                         e->stream));
  for (int k = 0; k < 2; ++k)
    HIP_TRY(hipMemcpyAsync(e->st.dir3_prev + k * 3 * M, dir3, 3 * M * sizeof(float),
                           hipMemcpyHostToDevice, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_download_directors(swarm_engine_t* e, float* dir3) {
  if (!e || !dir3) return fail(SWARM_EINVAL, "null argument");
  const size_t M = (size_t)e->st.m;
  HIP_TRY(hipMemcpyAsync(dir3, e->st.dir3, 3 * M * sizeof(float), hipMemcpyDeviceToHost,
                         e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_set_walls(swarm_engine_t* e, const swarm_wall_t* walls, int32_t n_walls) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  if (n_walls < 0 || n_walls > SWARM_MAX_WALLS) return fail(SWARM_ECAPACITY, "0 <= n_walls <= 16");
  if (n_walls > 0 && !walls) return fail(SWARM_EINVAL, "null walls");
  Derived& d = e->derived;
  d.n_walls = n_walls;
  for (int k = 0; k < n_walls; ++k) {
    const swarm_wall_t& w = walls[k];
    float* o = d.wp[k];
    d.wkind[k] = w.kind;
    if (w.kind == 0) {
      for (int a = 0; a < 3; ++a) o[a] = (float)w.normal[a];
      o[3] = (float)w.offset;
    } else if (w.kind == 1) {
      const double la = std::sqrt(w.a[0] * w.a[0] + w.a[1] * w.a[1]);
      const double lb = std::sqrt(w.b[0] * w.b[0] + w.b[1] * w.b[1]);
      if (!(la > 0.0) || !(lb > 0.0)) return fail(SWARM_EINVAL, "degenerate wall");
      o[0] = (float)w.corner[0];
      o[1] = (float)w.corner[1];
      o[2] = (float)(w.a[0] / la);
      o[3] = (float)(w.a[1] / la);
      o[4] = (float)(w.b[0] / lb);
      o[5] = (float)(w.b[1] / lb);
      o[6] = (float)la;
      o[7] = (float)lb;
    } else {
      return fail(SWARM_EINVAL, "wall kind must be 0 (plane) or 1 (slab)");
    }
  }
  HIP_TRY(hipMemcpyAsync(e->d_derived, &e->derived, sizeof(Derived), hipMemcpyHostToDevice,
                         e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return SWARM_OK;
}

int swarm_engine_wall_violations(swarm_engine_t* e, uint64_t* count) {
  if (!e || !count) return fail(SWARM_EINVAL, "null argument");
  unsigned long long v = 0;
  HIP_TRY(hipMemcpyAsync(&v, e->st.wall_viol, sizeof(v), hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  *count = v;
  return SWARM_OK;
}

}  // extern "C"

int swarm_sample_actions(const float* logits, int32_t n, int32_t k, uint64_t seed,
                         uint64_t* state, int32_t n_state, float explore_p,
                         const float* f_table, const float* t_table, int64_t* out_idx,
                         float* out_logp, float* out_f, float* out_t, void* stream) {
  if (!logits || !state || !f_table || !t_table || !out_idx || !out_logp || !out_f || !out_t)
    return fail(SWARM_EINVAL, "null argument");
  if (k < 1 || k > swarm::kMaxActions) return fail(SWARM_ECAPACITY, "1 <= k <= 64 actions");
  if (!(explore_p >= 0.0f && explore_p <= 1.0f))
    return fail(SWARM_EINVAL, "exploration probability must be in [0, 1]");
  if (n <= 0) return SWARM_OK;
  if (n_state < (n + 63) / 64) return fail(SWARM_EINVAL, "state needs ceil(n / 64) counters");
  hipLaunchKernelGGL(swarm::k_sample_actions, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), logits, n, k, (uint32_t)seed,
                     (uint32_t)(seed >> 32), reinterpret_cast<unsigned long long*>(state),
                     explore_p, f_table, t_table, out_idx, out_logp, out_f, out_t);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}

namespace {
// The rollout policy launch (swarm_policy_mlp_sample); ride: the engine whose
// deferred build's last stage (the cluster build) rides along as extra
// workgroups of the same launch (k_policy_cbuild), or null.
int policy_launch(const float* obs, int32_t n, int32_t d_in, const float* w1, const float* b1,
                  int32_t hidden, const float* w2, const float* b2, int32_t k, uint64_t seed,
                  uint64_t* state, int32_t n_state, float explore_p, const float* f_table,
                  const float* t_table, int64_t* out_idx, float* out_logp, float* out_f,
                  float* out_t, float* out_logits, void* stream, swarm_engine* ride) {
  if (!obs || !w1 || !b1 || !w2 || !b2 || !state || !f_table || !t_table || !out_idx ||
      !out_logp || !out_f || !out_t)
    return fail(SWARM_EINVAL, "null argument");
  if (d_in < 1 || d_in > swarm::kMlpMaxIn) return fail(SWARM_ECAPACITY, "1 <= d_in <= 16");
  if (hidden < 1 || hidden > swarm::kMlpMaxHidden)
    return fail(SWARM_ECAPACITY, "1 <= hidden <= 256");
  if (k < 1 || k > swarm::kMlpMaxActions) return fail(SWARM_ECAPACITY, "1 <= k <= 16 actions");
  if (!(explore_p >= 0.0f && explore_p <= 1.0f))
    return fail(SWARM_EINVAL, "exploration probability must be in [0, 1]");
  if (n <= 0) return SWARM_OK;
  if (n_state < (n + 63) / 64) return fail(SWARM_EINVAL, "state needs ceil(n / 64) counters");
  // lanes per agent: enough waves to cover the SIMDs when agents are few
  const int G = n <= 16384 ? 4 : (n <= 65536 ? 2 : 1);
  const bool small_in = d_in <= 4, small_k = k <= 4;
  const unsigned blocks = (unsigned)(((long)n * G + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  auto* st = reinterpret_cast<unsigned long long*>(state);
  const swarm::MlpArgs m{obs,   n,          d_in,    w1,      b1,       hidden, w2,
                         b2,    k,          k0,      k1,      st,       explore_p, f_table,
                         t_table, out_idx,  out_logp, out_f,  out_t,    out_logits};
  // the build stage may only ride along on the engine's stream: stages 1-2
  // and the run that consumes the build are ordered on it
  if (ride && s == ride->stream && ride->ride_stage == 3 && G == 4 && small_in && small_k) {
    // policy blocks of 1024 threads (256 agents: whole counter groups) and
    // one cluster-build workgroup per env
    const int pblocks = (int)(((long)n * G + 1023) / 1024);
    const size_t plds = (size_t)(hidden * swarm::MlpRow<4, 4>::kStride + 4) * sizeof(float);
    const size_t lds = std::max(plds, build_lds_bytes(ride->n, ride->sc.pair_cap));
    hipLaunchKernelGGL((k_policy_cbuild<4, 4, 4>), dim3((unsigned)(pblocks + ride->n_envs)),
                       dim3(1024), lds, s, m, ride->n_envs, ride->st, ride->sc);
    HIP_TRY(hipGetLastError());
    ride->ride_stage = 0;
    ride->prebuilt = true;
    return SWARM_OK;
  }
  if (ride && ride->ride_stage > 0) {
    const int rc = flush_ride_along(ride);
    if (rc) return rc;
  }
#define SWARM_MLP(GG, DD, KK)                                                                   \
  hipLaunchKernelGGL((swarm::k_policy_mlp_sample<GG, DD, KK>), dim3(blocks), dim3(256),        \
                     (size_t)(hidden * swarm::MlpRow<DD, KK>::kStride + KK) * sizeof(float), s, m)
#define SWARM_MLP_G(GG)                 \
  do {                                  \
    if (small_in && small_k)            \
      SWARM_MLP(GG, 4, 4);              \
    else if (small_in)                  \
      SWARM_MLP(GG, 4, 16);             \
    else if (small_k)                   \
      SWARM_MLP(GG, 16, 4);             \
    else                                \
      SWARM_MLP(GG, 16, 16);            \
  } while (0)
  if (G == 4)
    SWARM_MLP_G(4);
  else if (G == 2)
    SWARM_MLP_G(2);
  else
    SWARM_MLP_G(1);
#undef SWARM_MLP_G
#undef SWARM_MLP
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}
}  // namespace

int swarm_policy_mlp_sample(const float* obs, int32_t n, int32_t d_in, const float* w1,
                            const float* b1, int32_t hidden, const float* w2, const float* b2,
                            int32_t k, uint64_t seed, uint64_t* state, int32_t n_state,
                            float explore_p, const float* f_table, const float* t_table,
                            int64_t* out_idx, float* out_logp, float* out_f, float* out_t,
                            float* out_logits, void* stream) {
  return policy_launch(obs, n, d_in, w1, b1, hidden, w2, b2, k, seed, state, n_state, explore_p,
                       f_table, t_table, out_idx, out_logp, out_f, out_t, out_logits, stream,
                       nullptr);
}

int swarm_engine_policy_mlp_sample(swarm_engine_t* e, const float* obs, int32_t n, int32_t d_in,
                                   const float* w1, const float* b1, int32_t hidden,
                                   const float* w2, const float* b2, int32_t k, uint64_t seed,
                                   uint64_t* state, int32_t n_state, float explore_p,
                                   const float* f_table, const float* t_table, int64_t* out_idx,
                                   float* out_logp, float* out_f, float* out_t, float* out_logits,
                                   void* stream) {
  if (!e) return fail(SWARM_EINVAL, "null engine");
  return policy_launch(obs, n, d_in, w1, b1, hidden, w2, b2, k, seed, state, n_state, explore_p,
                       f_table, t_table, out_idx, out_logp, out_f, out_t, out_logits, stream, e);
}

int swarm_engine_defer_build(swarm_engine_t* e, int32_t* deferred) {
  if (!e || !deferred) return fail(SWARM_EINVAL, "null argument");
  *deferred = 0;
  // the three-launch 2-D cluster build of a latency-bound engine only (the
  // stages the fused observable / policy launches know how to carry)
  const bool ok = e->cluster_path && !e->nlist_path && !e->env_build && !e->big_build &&
                  e->params.n_dims == 2 && e->wide_run;
  if (!ok) return SWARM_OK;
  e->prebuilt = false;
  e->ride_stage = 1;
  e->vgrid_ready = false;
  *deferred = 1;
  return SWARM_OK;
}

namespace {
struct PpoWorkspace {
  size_t values, adv, dv, spart, table, partial, ticket, total;
};
PpoWorkspace ppo_workspace(long n, long S, int d, int hidden, int k) {
  PpoWorkspace w;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  w.values = 0;
  w.adv = up(w.values + (size_t)n * 4);
  w.dv = up(w.adv + (size_t)n * 4);
  w.spart = up(w.dv + (size_t)n * 4);
  w.table = up(w.spart + (size_t)((S + 255) / 256) * 2 * sizeof(double));
  // unit rows: at most 256 units x PpoTable<32, 16>::kStride floats
  w.partial = up(w.table + (size_t)swarm::kPpoMaxHidden * swarm::PpoTable<32, 16>::kStride * 4);
  w.ticket = up(w.partial + (size_t)swarm::kPpoBlocks * swarm::ppo_grad_size(d, hidden, k) * 4);
  w.total = up(w.ticket + 4);
  return w;
}
}  // namespace

int64_t swarm_ppo_workspace_bytes(int32_t T, int32_t S, int32_t d_in, int32_t hidden,
                                  int32_t k) {
  if (T < 1 || S < 1 || d_in < 1 || hidden < 1 || k < 1) return -1;
  return (int64_t)ppo_workspace((long)T * S, S, d_in, hidden, k).total;
}

// swarm_ppo_profile: HIP events around every k_ppo_grads launch of this
// thread (bench.py's roofline of the update); not under graph capture.
namespace {
struct PpoProfile {
  bool on = false;
  int reps = 1;  // back-to-back k_ppo_grads launches per epoch while timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};
thread_local PpoProfile g_ppo_prof;
}  // namespace

int swarm_ppo_profile(int32_t enable, double* grads_ms, int32_t* launches) {
  int32_t pairs = 0;
  const int rc = read_event_pairs(g_ppo_prof.ev, grads_ms, &pairs);
  if (launches) *launches = pairs * g_ppo_prof.reps;
  g_ppo_prof.reps = enable > 0 ? enable : 1;
  g_ppo_prof.on = enable > 0;
  return rc;
}

namespace {
// Workgroups of `fn` resident at once on a whole MI355X (256 CUs).  The grid
// size sets the fixed cross-block summation order of the gradient, so it is
// a function of the kernel and n only -- never of the device it runs on or
// its partition mode: replicas on any GPUs sum in the same order and stay
// bit-identical.
constexpr int kPpoOrderCUs = 256;
int ppo_resident_blocks(const void* fn, int threads, size_t lds) {
  const int cus = kPpoOrderCUs;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  return std::max(1, per_cu * cus);
}
}  // namespace

namespace {
int ppo_epoch(const float* x, int32_t T, int32_t S, int32_t d_in, const int64_t* actions,
              const float* old_logp, const float* rewards, const float* w1, const float* b1,
              int32_t hidden, const float* wa, const float* ba, int32_t k, const float* wc,
              const float* bc, float gamma, float lambda, float clip_eps, float entropy_coef,
              void* workspace, int64_t workspace_bytes, float* grad, void* stream,
              const swarm_adam_t* adam) {
  if (!x || !actions || !old_logp || !rewards || !w1 || !b1 || !wa || !ba || !wc || !bc ||
      !workspace || !grad)
    return fail(SWARM_EINVAL, "null argument");
  if (T < 1 || S < 1) return fail(SWARM_EINVAL, "T, S >= 1");
  if ((long)T * S > INT32_MAX) return fail(SWARM_ECAPACITY, "T x S < 2^31 samples");
  if (d_in < 1 || d_in > swarm::kPpoMaxIn) return fail(SWARM_ECAPACITY, "1 <= d_in <= 32");
  if (hidden < 1 || hidden > swarm::kPpoMaxHidden)
    return fail(SWARM_ECAPACITY, "1 <= hidden <= 256");
  if (k < 1 || k > swarm::kPpoMaxK) return fail(SWARM_ECAPACITY, "1 <= k <= 16 actions");
  const int n = T * S;
  const PpoWorkspace ws = ppo_workspace(n, S, d_in, hidden, k);
  if (workspace_bytes < (int64_t)ws.total)
    return fail(SWARM_EINVAL, "workspace smaller than swarm_ppo_workspace_bytes");
  char* base = static_cast<char*>(workspace);
  float* values = reinterpret_cast<float*>(base + ws.values);
  float* adv = reinterpret_cast<float*>(base + ws.adv);
  float* dv = reinterpret_cast<float*>(base + ws.dv);
  float* partial = reinterpret_cast<float*>(base + ws.partial);
  float* table = reinterpret_cast<float*>(base + ws.table);
  double* spart = reinterpret_cast<double*>(base + ws.spart);
  const int gae_blocks = (S + 255) / 256;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int NW = hidden <= 128 ? 1 : 2;  // waves of 128 units
  const long tiles = ((long)n + 63) / 64;  // k_ppo_values_split: 64 samples a block
  // k_ppo_grads: tiles of 128 samples; every block writes its partial row and
  // the reduce reads exactly the rows written
  // hidden <= 128: blocks of 4 tile waves (NT), else 2 unit waves (NW);
  // fewer tiles than 4 per grads block: the 4 waves share each tile (coop)
  const int NT = NW == 1 ? 4 : 1;
  const long tiles128 = ((long)n + 127) / 128;
  const bool coop = NW == 1 && tiles128 < 4L * swarm::kPpoBlocks;
  int blocks = (int)std::min<long>(coop ? tiles128 : (tiles128 + NT - 1) / NT,
                                   swarm::kPpoBlocks);
  const unsigned vblocks = (unsigned)(((n + 3) / 4 + 255) / 256);  // k_ppo_values: 4 a thread
  // V of every sample, GAE + dL/dV (+ the table), then the gradients
#define SWARM_PPO(NN, DD, KK)                                                                 \
  do {                                                                                        \
    using Tb = swarm::PpoTable<DD, KK>;                                                       \
    const swarm::PpoPack pk{w1, b1, wa, wc, d_in, hidden, k, 128 * NN, table};                \
    const int pack_blocks = (128 * NN * Tb::kStride + 255) / 256;                             \
    const dim3 ggrid((unsigned)(gae_blocks + pack_blocks));                                   \
    if (n < (1 << 20))                                                                        \
      hipLaunchKernelGGL((swarm::k_ppo_values_split<DD>), dim3((unsigned)tiles), dim3(256),   \
                         0, s, x, n, d_in, w1, b1, hidden, wc, bc, values);                   \
    else                                                                                      \
      hipLaunchKernelGGL((swarm::k_ppo_values<DD>), dim3(vblocks), dim3(256), 0, s, x, n,     \
                         d_in, w1, b1, hidden, wc, bc, values);                               \
    if (T <= 32)                                                                              \
      hipLaunchKernelGGL((swarm::k_ppo_gae<32, DD, KK>), ggrid, dim3(256), 0, s, rewards,     \
                         values, T, S, gamma, lambda, adv, dv, spart, gae_blocks, pk);        \
    else                                                                                      \
      hipLaunchKernelGGL((swarm::k_ppo_gae<0, DD, KK>), ggrid, dim3(256), 0, s, rewards,      \
                         values, T, S, gamma, lambda, adv, dv, spart, gae_blocks, pk);        \
    constexpr int TT = NN == 1 ? 4 : 1;                                                       \
    if (NN == 1 && coop) SWARM_PPO_GRADS(NN, TT, NN == 1, DD, KK);                            \
    else SWARM_PPO_GRADS(NN, TT, false, DD, KK);                                              \
  } while (0)
#define SWARM_PPO_GRADS(NN, TT, CO, DD, KK)                                                   \
  do {                                                                                        \
    const void* fn = reinterpret_cast<const void*>(&swarm::k_ppo_grads<NN, TT, CO, DD, KK>);  \
    const int lds = swarm::ppo_grads_lds_floats<NN, TT, CO, DD, KK>() * (int)sizeof(float);   \
    if (lds > 65536)                                                                          \
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);         \
    /* no more blocks than are resident at once: a second round of blocks */                  \
    /* would leave most SIMDs idle for its tail */                                            \
    if (!(CO)) blocks = std::min(blocks, ppo_resident_blocks(fn, 64 * NN * TT, lds));         \
    hipEvent_t ev0 = nullptr, ev1 = nullptr;                                                 \
    if (g_ppo_prof.on && hipEventCreate(&ev0) == hipSuccess &&                                \
        hipEventCreate(&ev1) == hipSuccess)                                                   \
      (void)hipEventRecord(ev0, s);                                                           \
    for (int rep = 0; rep < (ev1 ? g_ppo_prof.reps : 1); ++rep) /* same partial rows */      \
      hipLaunchKernelGGL((swarm::k_ppo_grads<NN, TT, CO, DD, KK>), dim3((unsigned)blocks),   \
                         dim3(64 * NN * TT),                                                  \
                         (size_t)lds, s, x, n, d_in, w1, b1, hidden, wa, ba, k, wc, bc,       \
                         actions, old_logp, adv, dv, spart, gae_blocks, table, clip_eps,      \
                         entropy_coef, partial);                                              \
    if (ev1) {                                                                                \
      (void)hipEventRecord(ev1, s);                                                           \
      g_ppo_prof.ev.emplace_back(ev0, ev1);                                                   \
    }                                                                                         \
  } while (0)
#define SWARM_PPO_H(NN)                          \
  do {                                           \
    if (d_in == 1 && k <= 4)                     \
      SWARM_PPO(NN, 1, 4);                       \
    else if (d_in <= 4 && k <= 4)                \
      SWARM_PPO(NN, 4, 4);                       \
    else if (d_in <= 4)                          \
      SWARM_PPO(NN, 4, 16);                      \
    else if (d_in <= 16 && k <= 4)               \
      SWARM_PPO(NN, 16, 4);                      \
    else if (d_in <= 16)                         \
      SWARM_PPO(NN, 16, 16);                     \
    else if (k <= 4)                             \
      SWARM_PPO(NN, 32, 4);                      \
    else                                         \
      SWARM_PPO(NN, 32, 16);                     \
  } while (0)
  if (NW == 1)
    SWARM_PPO_H(1);
  else
    SWARM_PPO_H(2);
#undef SWARM_PPO_H
#undef SWARM_PPO_GRADS
#undef SWARM_PPO
  const int size = swarm::ppo_grad_size(d_in, hidden, k);
  if (adam) {  // the optimizer step fused into the reduce
    swarm::AdamArgs a;
    a.lr = adam->lr;
    a.beta1 = adam->beta1;
    a.beta2 = adam->beta2;
    a.eps = adam->eps;
    const int sizes[6] = {hidden * d_in, hidden, k * hidden, k, hidden, 1};
    a.seg[0] = 0;
    for (int t = 0; t < 6; ++t) {
      if (!adam->param[t] || !adam->exp_avg[t] || !adam->exp_avg_sq[t] || !adam->step[t])
        return fail(SWARM_EINVAL, "null Adam tensor");
      a.param[t] = adam->param[t];
      a.m[t] = adam->exp_avg[t];
      a.v[t] = adam->exp_avg_sq[t];
      a.step[t] = adam->step[t];
      a.seg[t + 1] = a.seg[t] + sizes[t];
    }
    uint32_t* ticket = reinterpret_cast<uint32_t*>(base + ws.ticket);
    hipLaunchKernelGGL(swarm::k_ppo_reduce_adam, dim3((unsigned)((size + 63) / 64)), dim3(1024), 0,
                       s, partial, blocks, size, grad, a, ticket);
  } else {
    hipLaunchKernelGGL(swarm::k_ppo_reduce, dim3((unsigned)((size + 63) / 64)), dim3(1024), 0, s,
                       partial, blocks, size, grad);
  }
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}
}  // namespace

int swarm_ppo_epoch_grad(const float* x, int32_t T, int32_t S, int32_t d_in,
                         const int64_t* actions, const float* old_logp, const float* rewards,
                         const float* w1, const float* b1, int32_t hidden, const float* wa,
                         const float* ba, int32_t k, const float* wc, const float* bc,
                         float gamma, float lambda, float clip_eps, float entropy_coef,
                         void* workspace, int64_t workspace_bytes, float* grad, void* stream) {
  return ppo_epoch(x, T, S, d_in, actions, old_logp, rewards, w1, b1, hidden, wa, ba, k, wc, bc,
                   gamma, lambda, clip_eps, entropy_coef, workspace, workspace_bytes, grad, stream,
                   nullptr);
}

int swarm_ppo_epoch_step(const float* x, int32_t T, int32_t S, int32_t d_in,
                         const int64_t* actions, const float* old_logp, const float* rewards,
                         int32_t hidden, int32_t k, float gamma, float lambda, float clip_eps,
                         float entropy_coef, const swarm_adam_t* adam, void* workspace,
                         int64_t workspace_bytes, float* grad, void* stream) {
  if (!adam) return fail(SWARM_EINVAL, "null argument");
  if (!(adam->beta1 >= 0.0f && adam->beta1 < 1.0f && adam->beta2 >= 0.0f && adam->beta2 < 1.0f))
    return fail(SWARM_EINVAL, "Adam betas must be in [0, 1)");
  return ppo_epoch(x, T, S, d_in, actions, old_logp, rewards, adam->param[0], adam->param[1],
                   hidden, adam->param[2], adam->param[3], k, adam->param[4], adam->param[5],
                   gamma, lambda, clip_eps, entropy_coef, workspace, workspace_bytes, grad, stream,
                   adam);
}

int swarm_neighbor_reduce(const double* pos, const double* dir, const double* vel,
                          const int32_t* types, int32_t n_envs, int32_t n,
                          const int32_t* agent_idx, int32_t n_agents, uint32_t cand_type_mask,
                          double vision_range, double half_angle, double* out, void* stream) {
  if (!pos || !dir || !types || !agent_idx || !out) return fail(SWARM_EINVAL, "null argument");
  if (n_envs < 1 || n < 0 || n_agents < 0) return fail(SWARM_EINVAL, "bad sizes");
  if (n_agents == 0) return SWARM_OK;
  const dim3 grid((unsigned)((n_agents + 255) / 256), (unsigned)n_envs);
  hipLaunchKernelGGL(k_neighbor_reduce, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     pos, dir, vel, types, n, agent_idx, n_agents, cand_type_mask, vision_range,
                     half_angle, out);
  HIP_TRY(hipGetLastError());
  return SWARM_OK;
}
