// swarm_integrator.cuh -- Brownian dynamics + WCA integrator kernels.
//
// One integration window (<= kMaxWindow sub-steps, normally one RL slice of
// 100) is three launches:
//
//   k_cluster_build  one workgroup per env: cell list (side >= rc + skin),
//                    neighbour lists, union-find connected components
//                    ("clusters") of the rc+skin graph, and a packing of the
//                    clusters into 64-lane wave slots that never straddle a
//                    wave.  Depends on positions only, so it may run ahead
//                    (swarm_engine_prebuild) while the slice's actions are
//                    being computed.
//   k_cluster_run    one wave per 64 slots, one lane per particle: all
//                    sub-steps of the window with no block or grid barrier;
//                    neighbour positions move lane-to-lane (ds_bpermute).
//                    Snapshots the window-start state and tracks every
//                    particle's maximum displacement D.
//   k_check          one workgroup per env: exact validity test of the
//                    decomposition (no pair that is not a listed neighbour
//                    pair can have come within the WCA cutoff:
//                    d0 >= rc + D_i + D_j for every such pair with a mover,
//                    D >= skin / 2), and, if it failed (or the build flagged a
//                    cluster > 64 / a neighbour-list overflow), re-runs the
//                    env from the snapshot with the global per-sub-step
//                    algorithm.  Advances the device noise counter.
//
// Both paths call the same pair_force() / bd_step() functions and sum pair
// forces in int64 fixed point, so the result is independent of the
// decomposition and bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/swarmrl_amd.h"
#include "swarm_device.cuh"

// Sub-step schedule of the run kernels (round 6): off-chain work placed in
// the latency windows of the position exchange and the force-sum round trip.
#ifndef SWARM_RUN_SCHED
#define SWARM_RUN_SCHED 3
#endif
// helper mode: the displacement and carries in the exchange window (0,
// measured faster: head 62.4 / 61.8 vs 60.0 / 60.5 M with them in the force
// round trip's window, same box) or in the round trip's window (1)
#ifndef SWARM_HELPER_WIN2
#define SWARM_HELPER_WIN2 0
#endif

namespace swarm {

constexpr int kMaxSpecies = SWARM_MAX_SPECIES;
// k_cluster_run: 5 blocks (waves) per CU (SIMD), so <= 96 VGPRs (the 24 B/lane
// spill this costs measured cheaper than 4 waves per SIMD)
constexpr int kRunMinBlocks = 5;
constexpr int kMaxWindow = 128;   // sub-steps per cluster window
constexpr int kPairsPerWave = 256;  // neighbour pairs of one 64-lane wave (4 passes)
// Clusters wider than a wave ("big" clusters) run in k_check's workgroup, one
// member per thread: up to kBigMax members and kBigPairs pairs per env.
constexpr int kBigMax = 1024;
constexpr int kBigPairs = 4096;
constexpr int kBigMark = -0x40000000;  // cbase of a big cluster's root
// multi-workgroup build (k_mwb_*): sc.bmisc layout per env
constexpr int kBmWords = 256;  // sc.bmisc words per env
constexpr int kBmMisc = 0;     // [16]: 0 overflow, 1 waves, 2 pair overflow, 3 free lanes,
                               // 4 big members, 6 big pairs, 8 / 9 tickets
constexpr int kBmClass = 16;   // [68] cluster count per class
constexpr int kBmWave = 84;    // [68] first wave of a class
constexpr int kBmFree = 152;   // [68] first free tail lane of a class (singletons)
constexpr uint32_t kMwbBig = 0x80000000u;  // B of a big cluster's root: kMwbBig | first member
constexpr int kMaxMovers = 1024;       // listed movers per env (more: exact re-run)
// Candidate lists of the next window's pair search (latency-bound ride-along
// builds, see cand_build_body): per particle up to kCandMax partners j > i
// within r_i + r_j + skin + 2 cand_disp of the window-start positions.
constexpr int kCandMax = 24;

// Wave slots per env: every cluster packs into one wave, worst case 2 N
// slots plus per-size-class rounding.  One-pass packing (latency-bound
// launches, see k_cluster_build) reserves up to 2 s lanes for a cluster of
// s particles: worst case 4 N.
__host__ __device__ inline int slots_per_env(int n, bool one_pass = false) {
  return (one_pass ? 4 : 2) * n + 64 * 66;
}
constexpr float kAngInvScale = 683565275.57643158f;  // 2^32 / (2 pi)

// fp32 constants derived from swarm_params_t (same derivation as the oracle).
struct Derived {
  float sx[3], inv_sx[3];
  float mob_dt[kMaxSpecies], sig_t[kMaxSpecies];
  float rot_dt[kMaxSpecies], sig_r[kMaxSpecies];
  float inv_gt[kMaxSpecies], inv_gr[kMaxSpecies];
  float sig_v[kMaxSpecies], sig_w[kMaxSpecies];
  float cut2[kMaxSpecies * kMaxSpecies];
  float sig6[kMaxSpecies * kMaxSpecies];
  float nb2[kMaxSpecies * kMaxSpecies];  // (r_i + r_j + skin)^2: cluster links
  // (r_i + r_j + skin + 2 cand_disp)^2: candidate partners of the next
  // window's pair search (cand_build_body), valid while no particle moves
  // more than cand_disp in the window
  float nbc2[kMaxSpecies * kMaxSpecies];
  float cand_disp;
  float eps24;
  float skin;
  float rc_max_f;
  int32_t n_species;
  uint32_t key0, key1;
  int32_t noisy;
  int32_t periodic;
  double rc_max;
  // walls (swarm_engine_set_walls): plane n0 n1 n2 off | slab o0 o1 a0 a1 b0 b1 la lb
  int32_t n_walls;
  int32_t wkind[SWARM_MAX_WALLS];
  float wp[SWARM_MAX_WALLS][8];
  float wcut2[kMaxSpecies], wsig6[kMaxSpecies];  // wall WCA per species (radius 0 wall)
};

struct DevState {
  uint32_t* q;       // [3][M]
  int32_t* img;      // [3][M]
  uint32_t* ang;     // [M]
  float* f_swim;     // [M]
  float* torque_z;   // [M]
  float* f_ext;      // [3][M]
  float* vel;        // [3][M]
  float* omega;      // [M]
  uint8_t* species;  // [N]
  int32_t n;         // particles per env
  int32_t m;         // E * N
  int32_t dims;      // 2 or 3
  // 3-D only
  float* dir3;       // [3][M] unit directors
  float* torque_xy;  // [2][M] (z: torque_z)
  float* omega_xy;   // [2][M] (z: omega)
  unsigned long long* wall_viol;  // [1] wall contacts with dist <= 0
  // reuse_forces (swarm_params_t): what the last force calculation of the
  // previous run used -- sub-step 0 of a run takes its swim force, torque
  // and director from here (espresso.py:1304-1306).  Two slots, by the
  // device window counter's parity: window w reads slot w & 1 and writes
  // slot (w + 1) & 1 (the run kernel for its particles, the check only after
  // an exact re-run), so a re-run still finds the old values.
  int32_t reuse;
  float* f_prev;       // [2][M]
  float* tz_prev;      // [2][M]
  uint32_t* ang_prev;  // [2][M]    2-D orientation
  float* dir3_prev;    // [2][3][M] 3-D director
  float* txy_prev;     // [2][2][M] 3-D torque x, y
};

// The reuse_forces slot p of the engine (see DevState).
struct PrevSlot {
  float* f;
  float* tz;
  uint32_t* ang;
  float* dir3;
  float* txy;
};

__device__ __forceinline__ PrevSlot prev_slot(const DevState& st, int p) {
  const size_t M = (size_t)st.m;
  PrevSlot s;
  s.f = st.f_prev + p * M;
  s.tz = st.tz_prev + p * M;
  s.ang = st.ang_prev + p * M;
  s.dir3 = st.dir3_prev + (st.dims == 3 ? p * 3 * M : 0);
  s.txy = st.txy_prev + (st.dims == 3 ? p * 2 * M : 0);
  return s;
}

// End of a window: the actions and orientation particle gi's next run
// reuses at sub-step 0, into slot wp.  Called by the thread that wrote gi's
// final state.
__device__ __forceinline__ void save_forces(const DevState& st, size_t gi, int wp) {
  const size_t M = (size_t)st.m;
  const PrevSlot w = prev_slot(st, wp);
  w.f[gi] = st.f_swim[gi];
  w.tz[gi] = st.torque_z[gi];
  if (st.dims == 3) {
    w.dir3[gi] = st.dir3[gi];
    w.dir3[M + gi] = st.dir3[M + gi];
    w.dir3[2 * M + gi] = st.dir3[2 * M + gi];
    w.txy[gi] = st.torque_xy[gi];
    w.txy[M + gi] = st.torque_xy[M + gi];
  } else {
    w.ang[gi] = st.ang[gi];
  }
}

__device__ __forceinline__ void save_forces_env(const DevState& st, int e, int wp) {
  if (!st.reuse) return;
  __syncthreads();
  const size_t base = (size_t)e * st.n;
  for (int i = threadIdx.x; i < st.n; i += blockDim.x) save_forces(st, base + i, wp);
}

// Device control block (uint64 words): step counter, window counter, and
// the two noise tables' first step / length (by window parity, see k_noise).
constexpr int kCtlStep = 0, kCtlWin = 1, kCtlTStep = 2, kCtlTLen = 4, kCtlWords = 8;

__device__ __forceinline__ int window_parity(const uint64_t* ctl) {
  return (int)(ctl[kCtlWin] & 1ull);  // written by earlier launches only
}

struct Scratch {
  uint32_t* sqx;      // [M] positions sorted by cell
  uint32_t* sqy;      // [M]
  uint32_t* sqz;      // [M] (3-D global path)
  int32_t* simg;      // [3][M] image counters sorted with sqx/sqy/sqz (non-periodic global path)
  int32_t* sidx;      // [M] particle index of a sorted entry
  uint32_t* bq;       // [dims][M] window-start snapshot
  int32_t* bimg;      // [dims][M]
  uint32_t* bang;     // [M]
  int32_t* root;      // [M] cluster id (root particle)
  int32_t* slot_of;   // [M] wave slot of a particle
  int32_t* perm;      // [E][S] particle of a slot (-1: idle lane)
  uint32_t* pairs;    // [E][wmax][kPairsPerWave]: lane a | lane b << 6 | species pair << 12
  int32_t* wave_npairs;  // [E][wmax]
  float* disp;        // [M] max displacement over the window
  float* bdir3;       // [3][M] window-start directors (3-D cluster path)
  int32_t* env_waves; // [E]
  int32_t* fallback;  // [E]
  int32_t* big_list;  // [E][kBigMax] particles of the env's big clusters (member order)
  uint32_t* big_pairs;  // [E][kBigPairs] member a | member b << 10 | species pair << 20
  int32_t* big_n;     // [E] members
  int32_t* big_np;    // [E] pairs
  // colloids that moved >= skin / 2 in the window (appended by the run
  // kernel and the big-cluster run, consumed and reset by k_check)
  int32_t* nmov;      // [E]
  int32_t* movers;    // [E][kMaxMovers]
  // neighbour-list path (boxes whose rc + skin graph percolates)
  int32_t* nl;        // [kNlMax][M] neighbours j | species << 24 of particle gi
  int32_t* nn;        // [M] neighbour count
  uint32_t* qalt;     // [dims][M] second position buffer (sub-steps alternate)
  uint4* qa;          // [2][M] AoS position ping-pong of the per-launch window:
                      // (x, y, z, 0) in 3-D, uint2 (x, y) in 2-D
  // cluster build (k_build_sort -> k_build_pairs -> k_cluster_build)
  uint32_t* bsq;      // [dims][M] cell-sorted positions (x, y[, z])
  int32_t* bsid;      // [M] particle | species << 24 of a sorted entry
  int32_t* bcstart;   // [E][ncb + 1] first sorted entry of every cell, [ncb] = N
  uint32_t* gplist;   // [E][pair_cap] neighbour pairs i | j << 16, i < j
  int32_t* gnpairs;   // [E] pairs found (may exceed pair_cap: overflow)
  // 2-D pair search (build_pairs_body): every block unions the pairs whose
  // both ends lie in its range of sorted entries (a compact band of cells)
  // in LDS and writes each particle's block-local root; the pairs between
  // blocks go to a cross list, the only pairs the cluster build still unions
  int32_t* gcnt;      // [E][ncb] per-cell counters of the chip-wide sort (zero between builds)
  int32_t* gcell;     // [M] cell of a particle (chip-wide sort)
  int32_t* grank;     // [M] its rank within the cell
  int32_t* lroot;     // [M] block-local union-find root (a particle of the env) | pairs << 16
  uint32_t* xpairs;   // [E][pair_cap] cross-block pairs i | j << 16
  int32_t* gnx;       // [E] cross-block pairs found
  int32_t local_uf;   // 1: the 2-D pair search unions its blocks' pairs (lroot, xpairs)
  int32_t* gclus;     // [3][M] cluster sizes / bases / slots (large-N build only)
  int32_t* bmisc;     // [E][kBmWords] multi-workgroup build counters (null: one-workgroup build)
  int32_t pair_cap;   // pairs per env
  int32_t one_pass;   // 1: pack clusters so that a wave has <= 64 pairs
  int32_t fill_singletons;  // 1: singletons take the tail lanes of the other classes
  int32_t periodic;   // 0: non-periodic box (edge cells, unwrapped pair distances; 2-D build)
  int32_t multi_species;  // 0: one species (species pair bits 0, no species loads in the build)
  int32_t sort_stage_k;   // > 0: the build sort scatters into LDS, this many sorted entries per
                          // pass, and writes its output coalesced (0: scattered stores)
  int32_t S;          // slots per env
  int32_t wmax;       // S / 64
  // The next window's pair search as a filter of candidate lists (l1_pairs:
  // latency-bound periodic 2-D ride-along builds): the run kernel's extra
  // workgroups list every particle's candidates from the window's sort
  // (cand_build_body); k_check marks them usable for the next window
  // (cand_ok) when no particle moved more than cand_disp and nothing
  // overflowed or re-ran; the next slice's first launch then filters them at
  // the new positions beside the fresh sort (pair_filter_body), which
  // otherwise waits for that sort (sort_done) and searches its cells.
  int32_t l1_pairs;
  int32_t* cand;      // [kCandMax][M] partner j | species << 24 (j > i)
  int32_t* ncand;     // [M] candidates of a particle
  int32_t* cand_ok;   // [E] the lists hold every pair of the next window
  int32_t* cand_ovf;  // [E] a list overflowed (set by the builder, reset by k_check)
  uint64_t* sort_done;  // [E] window counter + 1 of the last finished build sort
  // [4] window statistics summed over the envs (swarm_engine_build_stats):
  // pair searches that filtered candidate lists, that waited for the fresh
  // sort, exact re-runs, windows checked
  unsigned long long* stats;
  uint64_t* phase;    // [32] build phase stamps (SWARM_PHASE_TIMING builds only)
  // profiling only (else null): [kRoles][kStampSub][2] earliest start /
  // latest end (device wall clock) of each workgroup role of the launches of
  // one window
  unsigned long long* rstamp;
};

// Launch stamps are spread over kStampSub (min, max) pairs by workgroup
// (blockIdx.x mod kStampSub) so that the atomics of a launch's waves do not
// queue on one address (which stretched the stamped launches); the reader
// takes the min / max over the pairs.
constexpr int kStampSub = 64;

// Workgroup roles of the window's launches (role_begin / role_end, rstamp)
enum RoleId {
  kRoleCheck = 0,
  kRoleSort,
  kRoleVgrid,
  kRoleField,
  kRolePairs,
  kRoleCone,
  kRoleCbuild,
  kRoleMlp,
  // progress marks inside roles (first / last wave to reach the point)
  kMarkFilterLoaded,    // pair filter: lists and positions in registers, tested
  kMarkFilterReserved,  // pair filter: the wave's output range reserved (atomic returned)
  kMarkConeReduced,     // vision cone: the group's bins summed (before the tail)
  kRoles
};

__device__ __forceinline__ void role_begin(const Scratch& sc, int r) {
  if (sc.rstamp && threadIdx.x == 0)
    atomicMin(&sc.rstamp[2 * (r * kStampSub + (blockIdx.x & (kStampSub - 1)))],
              (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void role_end(const Scratch& sc, int r) {
  if (sc.rstamp && (threadIdx.x & 63) == 0)
    atomicMax(&sc.rstamp[2 * (r * kStampSub + (blockIdx.x & (kStampSub - 1))) + 1],
              (unsigned long long)wall_clock64());
}
// A wave reached progress mark r (first and last arrival are recorded).
__device__ __forceinline__ void role_mark(unsigned long long* rstamp, int r) {
  if (rstamp && (threadIdx.x & 63) == 0) {
    const unsigned long long t = wall_clock64();
    const size_t o = 2 * (r * kStampSub + (blockIdx.x & (kStampSub - 1)));
    atomicMin(&rstamp[o], t);
    atomicMax(&rstamp[o + 1], t);
  }
}
__device__ __forceinline__ void role_mark(const Scratch& sc, int r) { role_mark(sc.rstamp, r); }

#ifdef SWARM_PHASE_TIMING
#define SWARM_STAMP(k)                                                    \
  do {                                                                    \
    if (blockIdx.x == 0 && threadIdx.x == 0) sc.phase[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define SWARM_STAMP(k) \
  do {                 \
  } while (0)
#endif

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ int cell_index(uint32_t qx, uint32_t qy, int lx, int ly) {
  const int cx = lx == 0 ? 0 : (int)(qx >> (32 - lx));
  const int cy = ly == 0 ? 0 : (int)(qy >> (32 - ly));
  return (cy << lx) | cx;
}

// Non-periodic boxes (MDParams.periodic = False, espresso.py:270; global
// path only): the cell of a particle outside the box is the edge cell on its
// side, and pair displacements are plain differences of the unwrapped
// positions (no minimum image) -- the oracle's cell_of / pair_disp.
__device__ __forceinline__ int cell_coord(uint32_t q, int32_t im, int l, bool periodic) {
  const int v = l == 0 ? 0 : (int)(q >> (32 - l));
  if (periodic) return v;
  return im < 0 ? 0 : (im > 0 ? (1 << l) - 1 : v);
}

__device__ __forceinline__ float pair_disp(uint32_t qj, int32_t ij, uint32_t qi, int32_t ii,
                                           float sx, bool periodic) {
  if (periodic) return (float)(int32_t)(qj - qi) * sx;
  const int64_t dq = (int64_t)(ij - ii) * 4294967296LL + ((int64_t)qj - (int64_t)qi);
  return (float)dq * sx;
}

// floor(n / d) for 0 <= n < 2^20 and 1 <= d < 2^20: a float reciprocal
// estimate (within one of the quotient) and one correction, instead of the
// compiler's ~40-instruction integer division (the cluster build's packing
// divides per cluster: 64 / s, r / per).
__device__ __forceinline__ int udiv_small(int n, int d) {
  int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
  const int r = n - q * d;
  q += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
  return q;
}

// Inclusive prefix sum over a wave's 64 lanes on the DPP network: row
// shifts 1, 2, 4, 8 scan each 16-lane row, the gfx9 row broadcasts 15 and 31
// carry rows into the next ones.  VALU only (no ds_bpermute round trip per
// step, as __shfl_up's).  Every lane of the wave must be active.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Exclusive scan of data[0..n) in LDS by the whole block; data[n] = total.
// Each wave scans a contiguous chunk 64 entries at a time (lane k reads
// entry base + k: no LDS bank conflicts, unlike one contiguous run per
// thread), carrying its running total; a second pass adds the exclusive
// prefix of the waves' totals.
// Up to 4 entries per thread the one-run-per-thread scan is shorter (its
// few strided reads conflict little): measured 2.6 vs 1.8 us at 4096 cells,
// 7.0 vs 11.5 us at 16384.
__device__ inline void block_exclusive_scan_runs(int32_t* data, int n, int32_t* wave_sums) {
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const int per = (n + T - 1) / T;
  const int lo = min(tid * per, n), hi = min(lo + per, n);
  // four entries per thread, 16-byte aligned: one ds_read_b128 / write_b128
  const bool quad = per == 4 && (n & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0;
  int4 x4 = make_int4(0, 0, 0, 0);
  int32_t local = 0;
  if (quad) {
    if (lo < n) x4 = reinterpret_cast<const int4*>(data)[tid];
    local = x4.x + x4.y + x4.z + x4.w;
  } else {
    for (int k = lo; k < hi; ++k) local += data[k];
  }
  const int lane = tid & 63, wave = tid >> 6;
  int32_t v = local;
  v = wave_incl_scan(v);
  if (lane == 63) wave_sums[wave] = v;
  __syncthreads();
  if (wave == 0) {
    const int nw = (T + 63) >> 6;
    int32_t w = lane < nw ? wave_sums[lane] : 0;
    w = wave_incl_scan(w);
    if (lane < nw) wave_sums[lane] = w;
  }
  __syncthreads();
  int32_t run = v - local + (wave > 0 ? wave_sums[wave - 1] : 0);
  if (quad) {
    if (lo < n) {
      int4 y;
      y.x = run;
      y.y = run + x4.x;
      y.z = y.y + x4.y;
      y.w = y.z + x4.z;
      reinterpret_cast<int4*>(data)[tid] = y;
    }
    if (tid == T - 1) data[n] = run + local;
    return;
  }
  for (int k = lo; k < hi; ++k) {
    const int32_t c = data[k];
    data[k] = run;
    run += c;
  }
  if (tid == T - 1) data[n] = run;
}

__device__ inline void block_exclusive_scan(int32_t* data, int n, int32_t* wave_sums) {
  const int T = blockDim.x;
  if (n <= 4 * T) {
    block_exclusive_scan_runs(data, n, wave_sums);
    return;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int nw = (T + 63) >> 6;
  const int chunk = (((n + nw - 1) / nw) + 63) & ~63;
  const int lo = min(wave * chunk, n), hi = min(lo + chunk, n);
  int32_t carry = 0;
  for (int b = lo; b < hi; b += 64) {
    const int k = b + lane;
    const int32_t x = k < hi ? data[k] : 0;
    int32_t v = x;
    v = wave_incl_scan(v);
    if (k < hi) data[k] = carry + v - x;
    carry += __builtin_amdgcn_readlane(v, 63);
  }
  if (lane == 0) wave_sums[wave] = carry;
  __syncthreads();
  if (wave == 0) {
    int32_t w = lane < nw ? wave_sums[lane] : 0;
    w = wave_incl_scan(w);
    if (lane < nw) wave_sums[lane] = w;  // inclusive prefix of the wave totals
  }
  __syncthreads();
  const int32_t add = wave > 0 ? wave_sums[wave - 1] : 0;
  if (add != 0)
    for (int k = lo + lane; k < hi; k += 64) data[k] += add;
  if (tid == T - 1) data[n] = wave_sums[nw - 1];
}

// WCA pair force of the 2-D paths (round 6 operation sequence, restated in
// oracle/swarm_oracle.c:wca_pair): the force on the first particle scaled
// by 2^24 (fp32), zero out of range.  The sequence is chosen for a short
// dependency chain in the run kernels (a dependent VALU operation of a lone
// wave costs ~11 cycles):
//   r2 = fma(rx, rx, ry ry); ir2 = 1 / r2 (rcp_rn)
//   s6 = (ir2 ir2) (sig6 ir2); t = fma(s6, 2, -1)
//   v  = ((eps24 s6) t) (ir2 (-rx 2^24))
// No select before the reciprocal: an out-of-range lane's value is
// discarded by the final select (in range r2 >= 2^-96, rcp_rn's range).
// cut2 = (r_i + r_j)^2, sig6 = sigma^6, eps24 = 24 epsilon (Derived tables).
__device__ __forceinline__ void pair_vals(float cut2, float sig6, float eps24, float rx, float ry,
                                          float& vx, float& vy) {
  const float r2 = __builtin_fmaf(rx, rx, ry * ry);
  const bool in = r2 < cut2 && r2 > 0.0f;
  const float ir2 = rcp_rn(r2);  // = 1.0f / r2 on every in-range lane
  const float s6 = (ir2 * ir2) * (sig6 * ir2);
  const float t = __builtin_fmaf(s6, 2.0f, -1.0f);
  const float fr = (eps24 * s6) * t;
  const float gx = ir2 * (rx * -16777216.0f), gy = ir2 * (ry * -16777216.0f);
  vx = in ? fr * gx : 0.0f;
  vy = in ? fr * gy : 0.0f;
}

// a 2^24-scaled force value to int64 fixed point: round to nearest even,
// clamped to +-2^62 (one int32 conversion below 2^31, the same value)
__device__ __forceinline__ int64_t fix_scaled(float v) {
  if (__builtin_expect(fabsf(v) < 2147483520.0f, 1)) return (int64_t)__float2int_rn(v);
  return __float2ll_rn(fminf(fmaxf(v, -4.611686018427387904e18f), 4.611686018427387904e18f));
}

// WCA force on i from j (r = x_j - x_i), accumulated in 2^-24 fixed point.
__device__ __forceinline__ void pair_force(float cut2, float sig6, float eps24, float rx,
                                           float ry, int64_t& ax, int64_t& ay) {
  float vx, vy;
  pair_vals(cut2, sig6, eps24, rx, ry, vx, vy);
  ax += fix_scaled(vx);
  ay += fix_scaled(vy);
}

// pair_force's fixed-point values for the run kernel's pair passes (every
// lane: zero out of range, and for an empty slot that names one particle
// twice); the int32 conversion is taken when every lane fits.
__device__ __forceinline__ void pair_fix_sel(float cut2, float sig6, float eps24, float rx,
                                             float ry, int64_t& fx, int64_t& fy) {
  float vx, vy;
  pair_vals(cut2, sig6, eps24, rx, ry, vx, vy);
  if (__builtin_expect(wave_all2(fabsf(vx) < 2147483520.0f, fabsf(vy) < 2147483520.0f), 1)) {
    fx = (int64_t)__float2int_rn(vx);
    fy = (int64_t)__float2int_rn(vy);
  } else {
    fx = __float2ll_rn(fminf(fmaxf(vx, -4.611686018427387904e18f), 4.611686018427387904e18f));
    fy = __float2ll_rn(fminf(fmaxf(vy, -4.611686018427387904e18f), 4.611686018427387904e18f));
  }
}

// WCA force of every wall on a particle of species si at the folded
// position (x, y, z) in 2^-24 fixed point (same operation sequence as
// oracle/swarm_oracle.c:wall_forces); contacts with dist <= 0 are counted.
template <int D>
__device__ __forceinline__ void wall_forces(const Derived* __restrict__ d, int si, float x, float y,
                                            float z, int64_t& ax, int64_t& ay, int64_t& az,
                                            unsigned long long* viol) {
  const int nw = d->n_walls;
  for (int k = 0; k < nw; ++k) {
    const float* w = d->wp[k];
    float vx, vy, vz, r2;
    if (d->wkind[k] == 0) {
      float dist = w[0] * x + w[1] * y;
      dist = dist + w[2] * z;
      dist = dist - w[3];
      if (!(dist > 0.0f)) {
        atomicAdd(viol, 1ull);
        continue;
      }
      vx = w[0] * dist;
      vy = w[1] * dist;
      vz = w[2] * dist;
      r2 = dist * dist;
    } else {
      const float px = x - w[0], py = y - w[1];
      const float u = px * w[2] + py * w[3];
      const float t = px * w[4] + py * w[5];
      const float du = u - fminf(fmaxf(u, 0.0f), w[6]);
      const float dt = t - fminf(fmaxf(t, 0.0f), w[7]);
      if (du == 0.0f && dt == 0.0f) {
        atomicAdd(viol, 1ull);
        continue;
      }
      vx = du * w[2] + dt * w[4];
      vy = du * w[3] + dt * w[5];
      vz = 0.0f;
      r2 = vx * vx + vy * vy;
    }
    if (r2 < d->wcut2[si]) {
      const float ir2 = 1.0f / r2;
      float ir6 = ir2 * ir2;
      ir6 = ir6 * ir2;
      const float s6 = d->wsig6[si] * ir6;
      float t = 2.0f * s6;
      t = t - 1.0f;
      float fr = d->eps24 * s6;
      fr = fr * t;
      fr = fr * ir2;
      ax += f2fix24(fr * vx);
      ay += f2fix24(fr * vy);
      if (D == 3) az += f2fix24(fr * vz);
    }
  }
}

struct PState {
  uint32_t qx, qy, an;
  int32_t ix, iy;
};

// Per-colloid constants, read once per launch (not per sub-step).
struct PConst {
  float mob_dt, sig_t, rot_dt, sig_r, inv_gt, inv_gr, sig_v, sig_w;
  float inv_sx0, inv_sx1;
  // the translation in fixed-point units per axis (2-D, round 6):
  // mob_dt / sx and sig_t / sx (0 without noise) as fp32 products
  float mobx, moby, sigx, sigy;
  float sigr;  // sig_r, 0 without noise (the rotation adds sigr g unconditionally)
  bool noisy;
};

__device__ __forceinline__ PConst load_pconst(const Derived* __restrict__ d, int si) {
  PConst c;
  c.mob_dt = d->mob_dt[si];
  c.sig_t = d->sig_t[si];
  c.rot_dt = d->rot_dt[si];
  c.sig_r = d->sig_r[si];
  c.inv_gt = d->inv_gt[si];
  c.inv_gr = d->inv_gr[si];
  c.sig_v = d->sig_v[si];
  c.sig_w = d->sig_w[si];
  c.inv_sx0 = d->inv_sx[0];
  c.inv_sx1 = d->inv_sx[1];
  c.noisy = d->noisy != 0;
  c.mobx = c.mob_dt * c.inv_sx0;
  c.moby = c.mob_dt * c.inv_sx1;
  c.sigx = c.noisy ? c.sig_t * c.inv_sx0 : 0.0f;
  c.sigy = c.noisy ? c.sig_t * c.inv_sx1 : 0.0f;
  c.sigr = c.noisy ? c.sig_r : 0.0f;
  return c;
}

// Pair tables staged in LDS by the whole block (call before any early exit).
struct PairTables {
  float cut2[kMaxSpecies * kMaxSpecies];
  float sig6[kMaxSpecies * kMaxSpecies];
};

__device__ __forceinline__ void stage_pair_tables(const Derived* __restrict__ d, PairTables* t) {
  for (int k = threadIdx.x; k < kMaxSpecies * kMaxSpecies; k += blockDim.x) {
    t->cut2[k] = d->cut2[k];
    t->sig6[k] = d->sig6[k];
  }
  __syncthreads();
}

// The translation of one BD sub-step in fixed-point units (2-D, round 6
// sequence; oracle/swarm_oracle.c:or_bd_run_walls): from the WCA sum F
// (fp32, 2^24 units),
//   f  = fma(F, 2^-24, f_ext + f_swim d)      (the force, d the director)
//   dq = f2i32_sat(fma(f, mob_dt / sx, (sig_t / sx) g))
// (F 2^-24 is exact; the per-axis constants are PConst's fp32 products).
__device__ __forceinline__ void bd_dq(const PConst& c, float Fx, float Fy, float fs, float fex,
                                      float fey, float sn, float cs, const float* g, float* fx,
                                      float* fy, int32_t* dqx, int32_t* dqy) {
  const float c1x = fex + fs * cs, c1y = fey + fs * sn;
  *fx = __builtin_fmaf(Fx, 5.9604644775390625e-08f, c1x);
  *fy = __builtin_fmaf(Fy, 5.9604644775390625e-08f, c1y);
  *dqx = f2i32_sat(__builtin_fmaf(*fx, c.mobx, c.sigx * g[0]));
  *dqy = f2i32_sat(__builtin_fmaf(*fy, c.moby, c.sigy * g[1]));
}

// One Brownian-dynamics sub-step of one particle from its summed WCA force.
// an_swim: the orientation the swim force points along (p.an, or with
// reuse_forces at sub-step 0 the previous run's last one).
// kTable: the step's three normals come precomputed in gt (k_noise).
template <bool kTable = false>
__device__ __forceinline__ void bd_step(const PConst& c, PState& p, int64_t ax, int64_t ay,
                                        float fs, float tz, float fex, float fey, uint32_t k0,
                                        uint32_t k1, uint32_t id, uint64_t step, bool last,
                                        float* vx, float* vy, float* w, uint32_t an_swim,
                                        const float* gt = nullptr, StepNoise* noise = nullptr,
                                        bool fresh = true) {
  float sn, cs;
  sincos_turn(an_swim, &sn, &cs);
  float g[3] = {0.0f, 0.0f, 0.0f};
  float dth = tz * c.rot_dt;
  if (c.noisy) {
    if (kTable) {
      g[0] = gt[0];
      g[1] = gt[1];
      g[2] = gt[2];
    } else if (noise) {  // consecutive sub-steps of one particle: carried normals
      noise->next(k0, k1, id, step, fresh, g);
    } else {
      step_normals(k0, k1, id, step, g);
    }
    dth = dth + c.sig_r * g[2];
  }
  float fx, fy;
  int32_t dqx, dqy;
  bd_dq(c, i64_to_f32(ax), i64_to_f32(ay), fs, fex, fey, sn, cs, g, &fx, &fy, &dqx, &dqy);
  advance(p.qx, p.ix, dqx);
  advance(p.qy, p.iy, dqy);
  p.an = p.an + (uint32_t)f2i32_sat(dth * kAngInvScale);
  if (last) {
    float v0 = fx * c.inv_gt, v1 = fy * c.inv_gt;
    float om = tz * c.inv_gr;
    if (c.noisy) {
      float g[3];
      normals3(k0, k1, id, step, 1u, g);
      v0 = v0 + c.sig_v * g[0];
      v1 = v1 + c.sig_v * g[1];
      om = om + c.sig_w * g[2];
    }
    *vx = v0;
    *vy = v1;
    *w = om;
  }
}

// bd_step without the rotation, for the cluster run (which turns the
// director apart from the force chain): the same translation (bd_dq) and
// velocities, from the force sums already converted to fp32 (2^24 units).
// Carry: with a Carry record the image counters are left to the caller
// (apply_carry, off the next sub-step's chain); q is updated here.
struct Carry {
  uint32_t qx0, qy0;
  int32_t dqx, dqy;
};
__device__ __forceinline__ void apply_carry(PState& p, const Carry& c) {
  p.ix += (int32_t)(((int64_t)(uint64_t)c.qx0 + (int64_t)c.dqx) >> 32);
  p.iy += (int32_t)(((int64_t)(uint64_t)c.qy0 + (int64_t)c.dqy) >> 32);
}
__device__ __forceinline__ void bd_translate_f(const PConst& c, PState& p, float fx, float fy,
                                               float fs, float tz, float fex, float fey,
                                               uint32_t k0, uint32_t k1, uint32_t id,
                                               uint64_t step, bool last, float* vx, float* vy,
                                               float* w, const float* g, float sn, float cs,
                                               Carry* carry = nullptr, bool adc = false) {
  const float F[2] = {fx, fy};
  int32_t dqx, dqy;
  // (without noise sigx = sigy = 0: g is finite, so sig g = +-0 changes no
  // displacement)
  bd_dq(c, F[0], F[1], fs, fex, fey, sn, cs, g, &fx, &fy, &dqx, &dqy);
  if (carry) {
    *carry = Carry{p.qx, p.qy, dqx, dqy};
    p.qx += (uint32_t)dqx;
    p.qy += (uint32_t)dqy;
  } else if (adc) {  // (a compile-time constant at every call)
    advance_adc(p.qx, p.ix, dqx);
    advance_adc(p.qy, p.iy, dqy);
  } else {
    advance(p.qx, p.ix, dqx);
    advance(p.qy, p.iy, dqy);
  }
  if (last) {
    float v0 = fx * c.inv_gt, v1 = fy * c.inv_gt;
    float om = tz * c.inv_gr;
    if (c.noisy) {
      float gv[3];
      normals3(k0, k1, id, step, 1u, gv);
      v0 = v0 + c.sig_v * gv[0];
      v1 = v1 + c.sig_v * gv[1];
      om = om + c.sig_w * gv[2];
    }
    *vx = v0;
    *vy = v1;
    *w = om;
  }
}

__device__ __forceinline__ void bd_translate(const PConst& c, PState& p, int64_t ax, int64_t ay,
                                             float fs, float tz, float fex, float fey,
                                             uint32_t k0, uint32_t k1, uint32_t id, uint64_t step,
                                             bool last, float* vx, float* vy, float* w,
                                             const float* g, float sn, float cs,
                                             bool adc = false) {
  float fx, fy;
  i64x2_to_f32(ax, ay, &fx, &fy);
  bd_translate_f(c, p, fx, fy, fs, tz, fex, fey, k0, k1, id, step, last, vx, vy, w, g, sn, cs,
                 nullptr, adc);
}

// One steepest-descent step of one particle (espresso.py:1163-1168).
__device__ __forceinline__ bool sd_step(const PConst& c, PState& p, int64_t ax, int64_t ay,
                                        float fs, float tz, float fex, float fey, float g,
                                        float md) {
  float sn, cs;
  sincos_turn(p.an, &sn, &cs);
  float fx = i64_to_f32(ax) * 5.9604644775390625e-08f;
  float fy = i64_to_f32(ay) * 5.9604644775390625e-08f;
  fx = fx + fex;
  fy = fy + fey;
  fx = fx + fs * cs;
  fy = fy + fs * sn;
  const bool any = fx != 0.0f || fy != 0.0f || tz != 0.0f;
  const float px = fminf(fmaxf(g * fx, -md), md);
  const float py = fminf(fmaxf(g * fy, -md), md);
  const float pa = fminf(fmaxf(g * tz, -md), md);
  advance(p.qx, p.ix, f2i32(px * c.inv_sx0));
  advance(p.qy, p.iy, f2i32(py * c.inv_sx1));
  p.an = p.an + (uint32_t)f2i32(pa * kAngInvScale);
  return any;
}

// ------------------------------------------------------- global path
// All sub-steps of env e by one workgroup: per sub-step a counting sort into
// cells of side >= rc_max (counts in LDS, sorted copy in global scratch), then
// every particle sums its pair forces over the 3x3 cells and is advanced.
// Spill-free: no per-thread particle arrays.
__device__ void block_global_run(const Derived* __restrict__ d, const DevState& st,
                                 const Scratch& sc, int e, int n_steps, uint64_t step0, int lx,
                                 int ly, bool sd_mode, float g, float md, int32_t* cnt,
                                 int32_t* wave_sums, const PairTables* pt, int rp) {
  const PrevSlot prv = prev_slot(st, rp);  // reuse_forces: sub-step 0 reads slot rp
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int lox = ncx >= 3 ? -1 : 0, hix = ncx >= 3 ? 1 : ncx - 1;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float eps24 = d->eps24;
  const bool per = d->periodic != 0;
  auto cell_of = [&](size_t gi) {
    return (cell_coord(st.q[M + gi], st.img[M + gi], ly, per) << lx) |
           cell_coord(st.q[gi], st.img[gi], lx, per);
  };
  for (int s = 0; s < n_steps; ++s) {
    for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += T) atomicAdd(&cnt[cell_of(base + i)], 1);
    __syncthreads();
    block_exclusive_scan(cnt, ncell, wave_sums);
    __syncthreads();
    for (int i = tid; i < N; i += T) {
      const uint32_t qx = st.q[base + i], qy = st.q[M + base + i];
      const int pos = atomicAdd(&cnt[cell_of(base + i)], 1);
      sc.sqx[base + pos] = qx;
      sc.sqy[base + pos] = qy;
      sc.sidx[base + pos] = i;
      if (!per) {  // the images too: the update below rewrites st.img in place
        sc.simg[base + pos] = st.img[base + i];
        sc.simg[M + base + pos] = st.img[M + base + i];
      }
    }
    __syncthreads();  // cell c now spans [c ? cnt[c-1] : 0, cnt[c])
    int any = 0;
    for (int i = tid; i < N; i += T) {
      const size_t gi = base + i;
      PState p;
      p.qx = st.q[gi];
      p.qy = st.q[M + gi];
      p.ix = st.img[gi];
      p.iy = st.img[M + gi];
      p.an = st.ang[gi];
      const int si = st.species[i];
      int64_t ax = 0, ay = 0;
      const int c0 = cell_of(gi);
      const int cx = c0 & (ncx - 1), cy = c0 >> lx;
      for (int oy = loy; oy <= hiy; ++oy) {
        if (!per && (cy + oy < 0 || cy + oy >= ncy)) continue;
        const int y = (cy + oy + ncy) & (ncy - 1);
        for (int ox = lox; ox <= hix; ++ox) {
          if (!per && (cx + ox < 0 || cx + ox >= ncx)) continue;
          const int x = (cx + ox + ncx) & (ncx - 1);
          const int cc = (y << lx) | x;
          const int jb = cc ? cnt[cc - 1] : 0, je = cnt[cc];
          for (int jj = jb; jj < je; ++jj) {
            const int j = sc.sidx[base + jj];
            if (j == i) continue;
            const float rx = per ? (float)(int32_t)(sc.sqx[base + jj] - p.qx) * sx0
                                 : pair_disp(sc.sqx[base + jj], sc.simg[base + jj], p.qx, p.ix,
                                             sx0, false);
            const float ry = per ? (float)(int32_t)(sc.sqy[base + jj] - p.qy) * sx1
                                 : pair_disp(sc.sqy[base + jj], sc.simg[M + base + jj], p.qy, p.iy,
                                             sx1, false);
            const int pk = si * kMaxSpecies + st.species[j];
            pair_force(pt->cut2[pk], pt->sig6[pk], eps24, rx, ry, ax, ay);
          }
        }
      }
      if (d->n_walls) {
        int64_t az = 0;
        wall_forces<2>(d, si, (float)p.qx * sx0, (float)p.qy * sx1, 0.0f, ax, ay, az,
                       st.wall_viol);
      }
      const bool first = st.reuse && s == 0 && !sd_mode;  // reuse_forces: previous run's
      const float fs = first ? prv.f[gi] : st.f_swim[gi];
      const float tz = first ? prv.tz[gi] : st.torque_z[gi];
      const float fex = st.f_ext[gi], fey = st.f_ext[M + gi];
      const PConst pc = load_pconst(d, si);
      if (sd_mode) {
        any |= sd_step(pc, p, ax, ay, fs, tz, fex, fey, g, md) ? 1 : 0;
      } else {
        float vx, vy, w;
        const bool last = s == n_steps - 1;
        bd_step(pc, p, ax, ay, fs, tz, fex, fey, k0, k1, (uint32_t)i, step0 + (uint64_t)s, last,
                &vx, &vy, &w, first ? prv.ang[gi] : p.an);
        if (last) {
          st.vel[gi] = vx;
          st.vel[M + gi] = vy;
          st.vel[2 * M + gi] = 0.0f;
          st.omega[gi] = w;
        }
      }
      st.q[gi] = p.qx;
      st.q[M + gi] = p.qy;
      st.img[gi] = p.ix;
      st.img[M + gi] = p.iy;
      st.ang[gi] = p.an;
    }
    if (sd_mode) {
      if (!__syncthreads_or(any)) break;
    } else {
      __syncthreads();
    }
  }
}

#ifdef SWARM_PHASE_TIMING
__device__ unsigned long long g_global_phase[4];  // cycles: sort, forces+step, steps
#endif

// LDS words the register-resident global path needs after the cell counts
// (sorted positions as uint2 + ids), 0 when it does not apply (3-D, or more
// than kGlobalCH particles per thread of a 1024-thread block).
constexpr int kGlobalCH = 4;
__host__ __device__ inline size_t global_lds_extra_words(int n, int dims, int ncell) {
  const size_t extra = 8 * (size_t)n + 2;
  // k_check's layout (the larger): 16 + 16 + 1024 + ncell + 1 words first,
  // and 4 KB of static LDS beside it
  const bool fits = (16 + 16 + 1024 + (size_t)ncell + 1 + extra) * 4 + 4096 <= 160 * 1024;
  return dims == 2 && n <= kGlobalCH * 1024 && fits ? extra : 0;
}

// The global path with the particle state and the per-sub-step cell sort in
// LDS (up to kGlobalCH particles per thread): same pair_force / bd_step /
// sd_step sequence and int64 force sums as block_global_run, so the same
// bits, but no global round trip inside a sub-step (it is the exact re-run
// of an env whose cluster window failed k_check, and the overlap removal).
// lsq: 8 N + 2 LDS words after cnt[ncell + 1].
__device__ __forceinline__ void block_global_run_lds(const Derived* __restrict__ d, const DevState& st, int e,
                                     int n_steps, uint64_t step0, int lx, int ly, bool sd_mode,
                                     float g, float md, int32_t* cnt, int32_t* wave_sums,
                                     int32_t* lsq, const PairTables* pt, int rp) {
  const PrevSlot prv = prev_slot(st, rp);  // reuse_forces: sub-step 0 reads slot rp
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float eps24 = d->eps24;
  uint2* sq = reinterpret_cast<uint2*>(lsq + ((reinterpret_cast<uintptr_t>(lsq) >> 2) & 1));
  int32_t* sid = reinterpret_cast<int32_t*>(sq + N);
  // particle state by particle index (the forces, velocities and species
  // are re-read from global memory, L1-resident, where used)
  uint32_t* lqx = reinterpret_cast<uint32_t*>(sid + N);
  uint32_t* lqy = lqx + N;
  int32_t* lix = reinterpret_cast<int32_t*>(lqy + N);
  int32_t* liy = lix + N;
  uint32_t* lan = reinterpret_cast<uint32_t*>(liy + N);
  for (int i = tid; i < N; i += T) {
    const size_t gi = base + i;
    lqx[i] = st.q[gi];
    lqy[i] = st.q[M + gi];
    lix[i] = st.img[gi];
    liy[i] = st.img[M + gi];
    lan[i] = st.ang[gi];
  }
  __syncthreads();
#ifdef SWARM_PHASE_TIMING
  uint64_t t_sort = 0, t_force = 0, tA = 0;
#endif
  for (int s = 0; s < n_steps; ++s) {
#ifdef SWARM_PHASE_TIMING
    if (tid == 0) tA = __builtin_amdgcn_s_memtime();
#endif
    for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += T) atomicAdd(&cnt[cell_index(lqx[i], lqy[i], lx, ly)], 1);
    __syncthreads();
    block_exclusive_scan(cnt, ncell, wave_sums);
    __syncthreads();
    for (int i = tid; i < N; i += T) {
      const uint32_t qx = lqx[i], qy = lqy[i];
      const int pos = atomicAdd(&cnt[cell_index(qx, qy, lx, ly)], 1);
      sq[pos] = make_uint2(qx, qy);
      sid[pos] = i | ((int)st.species[i] << 24);
    }
    __syncthreads();  // cell c now spans [c ? cnt[c-1] : 0, cnt[c])
#ifdef SWARM_PHASE_TIMING
    if (tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      t_sort += t - tA;
      tA = t;
    }
#endif
    int any = 0;
    // sorted order: the lanes of a wave take neighbouring particles, so their
    // candidate ranges (a stencil row = one contiguous sorted range, plus a
    // wrap range at the grid edge) are alike and the loops stay converged
    for (int ps = tid; ps < N; ps += T) {
      const int pki = sid[ps];
      const int i = pki & 0xffffff, sik = pki >> 24;
      const size_t gi = base + i;
      PState pp = {lqx[i], lqy[i], lan[i], lix[i], liy[i]};
      const bool first = st.reuse && s == 0 && !sd_mode;  // reuse_forces: previous run's
      const float fs = first ? prv.f[gi] : st.f_swim[gi];
      const float tz = first ? prv.tz[gi] : st.torque_z[gi];
      const float fex = st.f_ext[gi], fey = st.f_ext[M + gi];
      int64_t ax = 0, ay = 0;
      const int c0 = cell_index(pp.qx, pp.qy, lx, ly);
      const int cx = c0 & (ncx - 1), cy = c0 >> lx;
      const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
      const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
      const int xw = ncx >= 3 ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
      for (int oy = loy; oy <= hiy; ++oy) {
        const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
#pragma unroll
        for (int part = 0; part < 2; ++part) {
          if (part == 1 && xw < 0) continue;
          const int c_lo = row | (part == 0 ? xa : xw), c_hi = row | (part == 0 ? xb : xw);
          const int jb = c_lo ? cnt[c_lo - 1] : 0, je = cnt[c_hi];
          for (int jj = jb; jj < je; ++jj) {
            const int pj = sid[jj];
            if ((pj & 0xffffff) == i) continue;
            const uint2 qj = sq[jj];
            const float rx = (float)(int32_t)(qj.x - pp.qx) * sx0;
            const float ry = (float)(int32_t)(qj.y - pp.qy) * sx1;
            const int pk = sik * kMaxSpecies + (pj >> 24);
            pair_force(pt->cut2[pk], pt->sig6[pk], eps24, rx, ry, ax, ay);
          }
        }
      }
      if (d->n_walls) {
        int64_t az = 0;
        wall_forces<2>(d, sik, (float)pp.qx * sx0, (float)pp.qy * sx1, 0.0f, ax, ay, az,
                       st.wall_viol);
      }
      const PConst pc = load_pconst(d, sik);
      if (sd_mode) {
        any |= sd_step(pc, pp, ax, ay, fs, tz, fex, fey, g, md) ? 1 : 0;
      } else {
        float vx, vy, w;
        const bool last = s == n_steps - 1;
        bd_step(pc, pp, ax, ay, fs, tz, fex, fey, k0, k1, (uint32_t)i, step0 + (uint64_t)s,
                last, &vx, &vy, &w, first ? prv.ang[gi] : pp.an);
        if (last) {
          st.vel[gi] = vx;
          st.vel[M + gi] = vy;
          st.vel[2 * M + gi] = 0.0f;
          st.omega[gi] = w;
        }
      }
      lqx[i] = pp.qx;  // the sort of the next sub-step reads lqx/lqy after a barrier
      lqy[i] = pp.qy;
      lix[i] = pp.ix;
      liy[i] = pp.iy;
      lan[i] = pp.an;
    }
#ifdef SWARM_PHASE_TIMING
    __syncthreads();
    if (tid == 0) t_force += __builtin_amdgcn_s_memtime() - tA;
#endif
    if (sd_mode) {
      if (!__syncthreads_or(any)) break;
    } else {
      __syncthreads();
    }
  }
#ifdef SWARM_PHASE_TIMING
  if (tid == 0) {
    g_global_phase[0] = t_sort;
    g_global_phase[1] = t_force;
    g_global_phase[2] = (uint64_t)n_steps;
  }
#endif
  __syncthreads();
  for (int i = tid; i < N; i += T) {
    const size_t gi = base + i;
    st.q[gi] = lqx[i];
    st.q[M + gi] = lqy[i];
    st.img[gi] = lix[i];
    st.img[M + gi] = liy[i];
    st.ang[gi] = lan[i];
  }
}

// Advance the device noise counter once every workgroup of the launch has
// read it (the last arriving workgroup does it).
__device__ __forceinline__ void advance_counter(uint64_t* step_ctr, uint32_t* arrive,
                                                uint64_t step0, int n_steps) {
  if (threadIdx.x == 0) {
    const uint32_t ticket = atomicAdd(arrive, 1u);
    if (ticket == gridDim.x - 1) {
      step_ctr[kCtlStep] = step0 + (uint64_t)n_steps;
      step_ctr[kCtlWin] += 1ull;  // window counter (noise table parity)
      *arrive = 0u;
    }
  }
}

// Global-path launch: n_steps sub-steps (or SD steps) of every env.
__global__ __launch_bounds__(1024) void k_global(const Derived* __restrict__ d, DevState st,
                                                 Scratch sc, int n_steps,
                                                 uint64_t* __restrict__ step_ctr,
                                                 uint32_t* __restrict__ arrive, int lx, int ly,
                                                 int sd_mode, float g, float md) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ PairTables pt;
  stage_pair_tables(d, &pt);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  const uint64_t step0 = sd_mode ? 0ull : *step_ctr;
  // reuse_forces slots: a BD window reads w & 1 and writes the next window's
  // (w + 1) & 1; steepest descent does not advance the window counter, so it
  // writes the slot the next window reads
  const int par = window_parity(step_ctr);
  // the LDS variant assumes a periodic box (minimum image, folded cells)
  if (global_lds_extra_words(st.n, st.dims, 1 << (lx + ly)) && blockDim.x == 1024 && d->periodic)
    block_global_run_lds(d, st, blockIdx.x, n_steps, step0, lx, ly, sd_mode != 0, g, md, cnt,
                         wave_sums, cnt + (1 << (lx + ly)) + 1, &pt, par);
  else
    block_global_run(d, st, sc, blockIdx.x, n_steps, step0, lx, ly, sd_mode != 0, g, md, cnt,
                     wave_sums, &pt, par);
  save_forces_env(st, blockIdx.x, sd_mode ? par : par ^ 1);
  if (!sd_mode) advance_counter(step_ctr, arrive, step0, n_steps);
}

// ------------------------------------------------------ cluster build
// Concurrent union-find on LDS: find with path halving (a lane only ever
// points a node at one of its ancestors), union hooks the larger root under
// the smaller with CAS, so no cycle can form.
// The forest always lives in LDS: typed LDS pointers give ds_* operations
// (a generic volatile pointer compiles to flat accesses that wait on both
// the vector-memory and the LDS counters).
typedef __attribute__((address_space(3))) int32_t lds_i32;

__device__ __forceinline__ int uf_find(int32_t* parent_g, int x) {
  volatile lds_i32* parent = (volatile lds_i32*)(parent_g);
  while (true) {
    const int p = parent[x];
    if (p == x) return x;
    const int gp = parent[p];
    if (gp != p) parent[x] = gp;
    x = gp;
  }
}

// The roots of a and b, both walks in lockstep (path halving): each step's
// two LDS reads are in flight together, so a union costs the longer walk's
// round trips, not the sum of both.
__device__ __forceinline__ void uf_find2(int32_t* parent_g, int& a, int& b) {
  volatile lds_i32* parent = (volatile lds_i32*)(parent_g);
  int pa = parent[a], pb = parent[b];
  while (pa != a || pb != b) {
    const int ga = parent[pa], gb = parent[pb];
    if (pa != a) {
      if (ga != pa) parent[a] = ga;
      a = ga;
    }
    if (pb != b) {
      if (gb != pb) parent[b] = gb;
      b = gb;
    }
    pa = parent[a];
    pb = parent[b];
  }
}

__device__ __forceinline__ void uf_union(int32_t* parent, int a, int b) {
  while (true) {
    uf_find2(parent, a, b);
    if (a == b) return;
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(&parent[a], a, b) == a) return;
  }
}

// The union of a listed pair: its larger index is hooked under the smaller
// one at once while it is still a root -- one CAS, no walks.  parent[x] <= x
// holds everywhere (uf_union hooks the larger root, path halving only
// shortens), so a root may hang under any smaller node without closing a
// cycle; the component's root stays its smallest index.
__device__ __forceinline__ void uf_union_pair(int32_t* parent, int a, int b) {
  const int lo = min(a, b), hi = max(a, b);
  if (atomicCAS(&parent[hi], hi, lo) == hi) return;
  uf_union(parent, lo, hi);
}

// A class counter increment aggregated over the wave: one LDS atomic per
// wave for its lanes with pred set; returns the lane's rank (the counter's
// old value + the lanes below it).  The packing's singleton and pair classes
// otherwise take hundreds (E = 1) to thousands (C5) of same-address atomics,
// which the LDS executes one after another.
__device__ __forceinline__ int wave_class_add(int32_t* ctr, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return 0;
  const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(ctr, __builtin_popcountll(m));
  base = __shfl(base, leader);
  return base + below;
}

// LDS words of k_cluster_build: 168 fixed + per-wave pair counters +
// parent[N] + 3 N (cluster sizes, bases, slots) + the env's pair list.
__host__ __device__ inline size_t build_lds_words(int n, int pair_cap) {
  const int wmax = slots_per_env(n, true) / 64;  // either packing
  return 16 + 16 + 3 * 68 + (size_t)((wmax + 3) & ~3) + 4 * (size_t)n + (size_t)pair_cap;
}

// Build step 1, one workgroup per env: counting sort into cells of side
// >= rc_max + skin (global arrays for the chip-wide pair search).
// The body runs in the workgroup of env e (k_build_sort, or a workgroup of a
// fused launch that carries the build along: k_vgrid_sort).
// CH: particles per thread kept in registers across the scan (4, or 16
// above 4096).  publish > 0 (l1_pairs launches, whose pair search runs
// beside this sort): the pair counters were reset by the last k_check, and
// the finished sort is announced in sort_done[e] = publish (release, agent
// scope) for pair blocks that have to wait for it.
__device__ __forceinline__ void publish_sort(const Scratch& sc, int e, uint64_t publish) {
  // (usable candidate lists: no pair block waits for this sort)
  if (publish == 0 || sc.cand_ok[e]) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(&sc.sort_done[e], publish, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int CH>
__device__ __forceinline__ void build_sort_body(const DevState& st, const Scratch& sc, int lx,
                                                int ly, int e, unsigned char* smem,
                                                uint64_t publish = 0) {
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  // cell of particle i at (qx, qy): folded positions in a periodic box; in a
  // non-periodic one a particle outside the box takes the edge cell on its
  // side (cell_coord, as the global path and the oracle)
  const bool per = sc.periodic != 0;
  auto cell_of = [&](int i, uint32_t qx, uint32_t qy) {
    if (per) return cell_index(qx, qy, lx, ly);
    return (cell_coord(qy, st.img[M + base + i], ly, false) << lx) |
           cell_coord(qx, st.img[base + i], lx, false);
  };
  SWARM_STAMP(0);
  // all loads of the cached particles first (one memory latency, not CH)
  uint32_t cqx[CH], cqy[CH];
  int32_t cid[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int i = tid + k * T;
    const bool ok = i < N;
    cqx[k] = ok ? st.q[base + i] : 0u;
    cqy[k] = ok ? st.q[M + base + i] : 0u;
    cid[k] = ok ? (i | (sc.multi_species ? (int32_t)st.species[i] << 24 : 0)) : -1;
  }
  for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
  if (tid == 0) {
    if (publish == 0) {  // (else k_check reset them: the pair search runs already)
      sc.gnpairs[e] = 0;
      sc.gnx[e] = 0;
    }
    sc.fallback[e] = 0;  // the neighbour-list build sets it on overflow
  }
  __syncthreads();
  SWARM_STAMP(1);
#pragma unroll
  for (int k = 0; k < CH; ++k)
    if (cid[k] >= 0) atomicAdd(&cnt[cell_of(tid + k * T, cqx[k], cqy[k])], 1);
  for (int i = tid + CH * T; i < N; i += T)
    atomicAdd(&cnt[cell_of(i, st.q[base + i], st.q[M + base + i])], 1);
  __syncthreads();
  SWARM_STAMP(2);
  block_exclusive_scan(cnt, ncell, wave_sums);
  __syncthreads();
  SWARM_STAMP(3);
  int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  for (int c = tid; c <= ncell; c += T) cs[c] = cnt[c];
  __syncthreads();  // cnt is read above and incremented below
  SWARM_STAMP(4);
  if (sc.sort_stage_k > 0 && N <= CH * T) {
    // claim every cached particle's sorted position, then per pass of K
    // sorted entries scatter the ones that fall in it into LDS (x | y | id
    // rows after the counts) and write the pass out in order: coalesced
    // 16-byte stores instead of 3 N scattered 4-byte ones, which one CU
    // issues at about one lane per cycle (43 k of the 63 k cycles of a
    // 16384-colloid sort)
    const int K = sc.sort_stage_k;
    int spos[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k)
      spos[k] = cid[k] >= 0 ? atomicAdd(&cnt[cell_of(tid + k * T, cqx[k], cqy[k])], 1) : -1;
    // rows start 16-byte aligned (read as uint4 below): the counts round up
    // to a multiple of four words (sort_lds_bytes)
    uint32_t* lx_ = reinterpret_cast<uint32_t*>(cnt + ((ncell + 4) & ~3));
    uint32_t* ly_ = lx_ + K;
    int32_t* lid = reinterpret_cast<int32_t*>(ly_ + K);
    const bool vec = (N & 3) == 0 && (M & 3) == 0 && (K & 3) == 0;
    for (int p0 = 0; p0 < N; p0 += K) {
      const int kn = min(K, N - p0);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int r = spos[k] - p0;
        if (r >= 0 && r < kn) {
          lx_[r] = cqx[k];
          ly_[r] = cqy[k];
          lid[r] = cid[k];
        }
      }
      __syncthreads();
      if (vec) {
        uint4* gx = reinterpret_cast<uint4*>(sc.bsq + base + p0);
        uint4* gy = reinterpret_cast<uint4*>(sc.bsq + M + base + p0);
        int4* gi = reinterpret_cast<int4*>(sc.bsid + base + p0);
        for (int v = tid; v < (kn >> 2); v += T) {
          gx[v] = reinterpret_cast<const uint4*>(lx_)[v];
          gy[v] = reinterpret_cast<const uint4*>(ly_)[v];
          gi[v] = reinterpret_cast<const int4*>(lid)[v];
        }
      } else {
        for (int v = tid; v < kn; v += T) {
          sc.bsq[base + p0 + v] = lx_[v];
          sc.bsq[M + base + p0 + v] = ly_[v];
          sc.bsid[base + p0 + v] = lid[v];
        }
      }
      __syncthreads();  // the rows are refilled by the next pass
    }
    for (int k = tid; k < sc.S; k += T) sc.perm[(size_t)e * sc.S + k] = -1;
    SWARM_STAMP(5);
    publish_sort(sc, e, publish);
    return;
  }
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    if (cid[k] < 0) continue;
    const size_t pos = base + atomicAdd(&cnt[cell_of(tid + k * T, cqx[k], cqy[k])], 1);
    sc.bsq[pos] = cqx[k];
    sc.bsq[M + pos] = cqy[k];
    sc.bsid[pos] = cid[k];
  }
  for (int i = tid + CH * T; i < N; i += T) {
    const uint32_t qx = st.q[base + i], qy = st.q[M + base + i];
    const size_t pos = base + atomicAdd(&cnt[cell_of(i, qx, qy)], 1);
    sc.bsq[pos] = qx;
    sc.bsq[M + pos] = qy;
    sc.bsid[pos] = i | (sc.multi_species ? (int32_t)st.species[i] << 24 : 0);
  }
  // idle wave slots of the next run (k_cluster_build writes the used ones);
  // last, so the stores drain in the shadow of the scatter
  for (int k = tid; k < sc.S; k += T) sc.perm[(size_t)e * sc.S + k] = -1;
  SWARM_STAMP(5);
  publish_sort(sc, e, publish);
}

// Chip-wide 2-D build sort of large envs (N > 4096 outside the ride-along
// launches): the one-workgroup counting sort keeps 16 particles per thread
// going through every phase on one CU (21 us at 16384 colloids).  Here
// k_sort_count ranks every particle in its cell with a global atomic (one
// thread per particle), k_sort_scan (one workgroup per env) turns the
// counts into the cell starts and clears them for the next build, and
// k_sort_scatter writes every particle to its sorted entry.  Same output as
// k_build_sort (bsq, bsid, bcstart, the reset counters and slots); the
// entries of one cell come in atomic order, which nothing depends on (the
// decomposition never changes the integrated bits).
__device__ __forceinline__ int build_cell_of(const DevState& st, const Scratch& sc, size_t M,
                                             size_t gi, uint32_t qx, uint32_t qy, int lx, int ly) {
  if (sc.periodic) return cell_index(qx, qy, lx, ly);
  return (cell_coord(qy, st.img[M + gi], ly, false) << lx) | cell_coord(qx, st.img[gi], lx, false);
}

__global__ __launch_bounds__(256) void k_sort_count(DevState st, Scratch sc, int lx, int ly) {
  const int e = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x, N = st.n;
  if (i >= N) return;
  const size_t M = (size_t)st.m, gi = (size_t)e * N + i;
  const int c = build_cell_of(st, sc, M, gi, st.q[gi], st.q[M + gi], lx, ly);
  sc.gcell[gi] = c;
  sc.grank[gi] = atomicAdd(&sc.gcnt[((size_t)e << (lx + ly)) + c], 1);
}

__global__ __launch_bounds__(1024) void k_sort_scan(Scratch sc, int lx, int ly) {
  extern __shared__ __align__(16) unsigned char smem[];
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = wave_sums + 16;
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x;
  const int ncell = 1 << (lx + ly);
  int32_t* g = sc.gcnt + ((size_t)e << (lx + ly));
  // the counts into LDS, kB loads in flight per thread (one memory latency
  // per kB cells, not per cell), then the next build's counters zeroed
  // (the counters are zeroed again by k_sort_scatter, the slots reset here
  // or -- multi-workgroup builds -- by k_mwb_size: this one workgroup only
  // moves the counts)
  if (tid == 0) {
    sc.gnpairs[e] = 0;
    sc.gnx[e] = 0;
    sc.fallback[e] = 0;  // the neighbour-list build sets it on overflow
  }
  if (!sc.bmisc)
    for (int k = tid; k < sc.S; k += T) sc.perm[(size_t)e * sc.S + k] = -1;
  int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  if (ncell >= 4 * T && ncell <= 16 * T) {
    // 4-16 cells per thread (C5: 16): each thread's run of consecutive
    // counts straight from global memory as int4 loads (a wave reads one
    // contiguous 1-4 KB span), summed in registers, one block scan of the
    // thread totals, the exclusive starts written back through LDS and copied
    // out coalesced.  The 64-cell-per-step wave scan below chains 16 dependent
    // steps per wave here (~7 us at 16384 cells).
    const int nq = ncell / (4 * T);  // int4 per thread: 1, 2 or 4
    int4 v[4];
    int32_t local = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = q < nq ? reinterpret_cast<const int4*>(g)[tid * nq + q] : make_int4(0, 0, 0, 0);
      local += v[q].x + v[q].y + v[q].z + v[q].w;
    }
    const int lane = tid & 63, wave = tid >> 6;
    const int32_t incl = wave_incl_scan(local);
    if (lane == 63) wave_sums[wave] = incl;
    __syncthreads();
    if (wave == 0) {
      const int nw = T >> 6;
      int32_t w = lane < nw ? wave_sums[lane] : 0;
      w = wave_incl_scan(w);
      if (lane < nw) wave_sums[lane] = w;
    }
    __syncthreads();
    int32_t run = incl - local + (wave > 0 ? wave_sums[wave - 1] : 0);
    int4* c4 = reinterpret_cast<int4*>(cnt);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq) {
        int4 y;
        y.x = run;
        y.y = y.x + v[q].x;
        y.z = y.y + v[q].y;
        y.w = y.z + v[q].z;
        run = y.w + v[q].w;
        c4[tid * nq + q] = y;
      }
    }
    if (tid == T - 1) cnt[ncell] = run;
    __syncthreads();
    for (int c = tid; c <= ncell; c += T) cs[c] = cnt[c];
    return;
  }
  constexpr int kB = 16;
  for (int c0 = tid; c0 < ncell; c0 += kB * T) {
    int32_t v[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) v[u] = c0 + u * T < ncell ? g[c0 + u * T] : 0;
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (c0 + u * T < ncell) cnt[c0 + u * T] = v[u];
  }
  __syncthreads();
  block_exclusive_scan(cnt, ncell, wave_sums);
  __syncthreads();
  for (int c = tid; c <= ncell; c += T) cs[c] = cnt[c];
}

__global__ __launch_bounds__(256) void k_sort_scatter(DevState st, Scratch sc, int lx, int ly) {
  const int e = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x, N = st.n;
  if (i >= N) return;
  const size_t M = (size_t)st.m, base = (size_t)e * N, gi = base + i;
  const int ncell = 1 << (lx + ly);
  const int c = sc.gcell[gi];
  const size_t pos = base + sc.bcstart[(size_t)e * (ncell + 1) + c] + sc.grank[gi];
  sc.gcnt[((size_t)e << (lx + ly)) + c] = 0;  // the next build's counter (k_sort_scan read it)
  sc.bsq[pos] = st.q[gi];
  sc.bsq[M + pos] = st.q[M + gi];
  sc.bsid[pos] = i | (sc.multi_species ? (int32_t)st.species[i] << 24 : 0);
}

template <int CH>
__global__ __launch_bounds__(1024) void k_build_sort(DevState st, Scratch sc, int lx, int ly) {
  extern __shared__ __align__(16) unsigned char smem[];
  build_sort_body<CH>(st, sc, lx, ly, blockIdx.x, smem);
}

// Build step 2, chip-wide (grid.y = env, one thread per sorted entry): every
// pair within r_i + r_j + skin once (i < j).  A stencil row (cells x-1..x+1)
// is one contiguous sorted range, plus a wrap range at the grid edge.  The
// six range bounds are loaded together and candidates four at a time (a few
// memory latencies per thread, not one per candidate); up to kKeep pairs per
// thread stay in registers, one atomic per wave reserves the output, and a
// wave with a denser thread rescans to write.
// Body for block bx of env e (k_build_pairs: grid (ceil(N / blockDim), E);
// fused launches pass their own block index); nb2: a block-shared table.
// kLocal (= sc.local_uf, a compile-time variant so that the plain pair
// search carries none of the local union-find's code or registers).
template <bool kLocal = false>
__device__ __forceinline__ void build_pairs_body(const Derived* __restrict__ d, const DevState& st,
                                                 const Scratch& sc, int lx, int ly, int bx, int e,
                                                 float* nb2, int32_t* uf) {
  constexpr int kKeep = 8;
  for (int k = threadIdx.x; k < kMaxSpecies * kMaxSpecies; k += blockDim.x) nb2[k] = d->nb2[k];
  const int N = st.n;
  const int T = blockDim.x, t = threadIdx.x;
  const int lo = bx * T;  // this block's sorted entries [lo, lo + T)
  const int ps = lo + t;
  const bool valid = ps < N;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  const int32_t* gcs = sc.bcstart + (size_t)e * (ncell + 1);
  // the sorted records (x, y, id) and cell starts
  auto QX = [&](int j) -> uint32_t { return sc.bsq[base + j]; };
  auto QY = [&](int j) -> uint32_t { return sc.bsq[M + base + j]; };
  auto SID = [&](int j) -> int32_t { return sc.bsid[base + j]; };
  auto CS = [&](int c) -> int32_t { return gcs[c]; };
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  // non-periodic box (d->periodic == 0): edge cells, no wrap of the stencil,
  // unwrapped pair distances (pair_disp) -- a pair near across the box edge
  // only in the folded sense must not be listed
  const bool per = d->periodic != 0;
  int pk = 0, i = 0;
  uint32_t qx = 0, qy = 0;
  int32_t ix = 0, iy = 0;
  if (valid) {
    pk = SID(ps);
    i = pk & 0xffffff;
    qx = QX(ps);
    qy = QY(ps);
    if (!per) {
      ix = st.img[base + i];
      iy = st.img[M + base + i];
    }
  }
  const int c0 = per ? cell_index(qx, qy, lx, ly)
                     : (cell_coord(qy, iy, ly, false) << lx) | cell_coord(qx, ix, lx, false);
  const int cx = c0 & (ncx - 1), cy = c0 >> lx;
  const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
  const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
  const int xw = ncx >= 3 && per ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
  int rb[6], re[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int oy = loy + (r >> 1), part = r & 1;
    const bool use = valid && oy <= hiy && (part == 0 || xw >= 0) &&
                     (per || (cy + oy >= 0 && cy + oy < ncy));
    const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
    const int c_lo = row | (part == 0 ? xa : xw), c_hi = row | (part == 0 ? xb : xw);
    rb[r] = use ? CS(c_lo) : 0;
    re[r] = use ? CS(c_hi + 1) : 0;
  }
  __syncthreads();  // nb2
  const float* nb2_row = nb2 + (pk >> 24) * kMaxSpecies;
  int found = 0;
  uint32_t keep[kKeep];
#pragma unroll
  for (int v = 0; v < kKeep; ++v) keep[v] = 0u;
  // the six ranges as one flat candidate index f in [0, total), record
  // jj = f + off[r] of the range r holding f: kFly candidates in flight per
  // iteration whatever the split over the ranges (about 11 candidates at
  // area fraction 0.1: two rounds of loads, not one per range; 16 in
  // flight measured slower, 4096 colloids)
  constexpr int kFly = 8;
  int off[6], pre[7];
  pre[0] = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    off[r] = rb[r] - pre[r];
    pre[r + 1] = pre[r] + (re[r] - rb[r]);
  }
  const int total = pre[6];
  for (int f0 = 0; f0 < total; f0 += kFly) {
    int pk4[kFly], jj4[kFly];
    uint32_t x4[kFly], y4[kFly];
#pragma unroll
    for (int u = 0; u < kFly; ++u) {
      const int f = f0 + u;
      int o = off[0];
#pragma unroll
      for (int r = 1; r < 6; ++r) o = f >= pre[r] ? off[r] : o;
      const int jj = f + o;
      const bool ok = f < total;
      jj4[u] = jj;
      pk4[u] = ok ? SID(jj) : -1;
      x4[u] = ok ? QX(jj) : 0u;
      y4[u] = ok ? QY(jj) : 0u;
    }
#pragma unroll
    for (int u = 0; u < kFly; ++u) {
      if (pk4[u] < 0) continue;
      const int j = pk4[u] & 0xffffff;
      const float rx = per ? (float)(int32_t)(x4[u] - qx) * sx0
                           : pair_disp(x4[u], st.img[base + j], qx, ix, sx0, false);
      const float ry = per ? (float)(int32_t)(y4[u] - qy) * sx1
                           : pair_disp(y4[u], st.img[M + base + j], qy, iy, sx1, false);
      if (i < j && rx * rx + ry * ry < nb2_row[pk4[u] >> 24]) {
        // j, and (kLocal) for a partner inside this block's sorted range its
        // block slot + 1 (a pair the block unions itself)
        const int ls = jj4[u] - lo;
        const uint32_t kv =
            (uint32_t)j | (kLocal && ls >= 0 && ls < T ? (uint32_t)(ls + 1) << 16 : 0u);
#pragma unroll
        for (int v = 0; v < kKeep; ++v) keep[v] = found == v ? kv : keep[v];
        ++found;
      }
    }
  }
  const int lane = threadIdx.x & 63;
  const bool dense = __any(found > kKeep);  // a lane kept only kKeep: the wave rescans
  if constexpr (!kLocal) {  // the pair list only (every pair unioned by the build)
    int v = found;
    v = wave_incl_scan(v);
    int wbase = 0;
    uint32_t* out = sc.gplist + (size_t)e * sc.pair_cap;
    const int cap = sc.pair_cap;
    if (lane == 63) wbase = atomicAdd(&sc.gnpairs[e], v);
    wbase = __builtin_amdgcn_readlane(wbase, 63);
    const int my_off = wbase + v - found;
    if (!dense) {
#pragma unroll
      for (int u = 0; u < kKeep; ++u) {
        const int k = my_off + u;
        if (u < found && k < cap) out[k] = (uint32_t)i | ((keep[u] & 0xffffu) << 16);
      }
      return;
    }
    int w = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      for (int jj = rb[r]; jj < re[r]; ++jj) {
        const int packed = SID(jj);
        const int j = packed & 0xffffff;
        const float rx = per ? (float)(int32_t)(QX(jj) - qx) * sx0
                             : pair_disp(QX(jj), st.img[base + j], qx, ix, sx0, false);
        const float ry = per ? (float)(int32_t)(QY(jj) - qy) * sx1
                             : pair_disp(QY(jj), st.img[M + base + j], qy, iy, sx1, false);
        if (i < j && rx * rx + ry * ry < nb2_row[packed >> 24]) {
          const int k = my_off + w;
          if (k < cap) out[k] = (uint32_t)i | ((uint32_t)j << 16);
          ++w;
        }
      }
    }
    return;
  }
  // Block-local union-find of the pairs whose both ends are in this block
  // (LDS only; done before any global store is issued, so the block
  // barriers below wait for LDS operations and not for store write-backs).
  int32_t* lpar = uf;       // [T] block-local union-find over the block's entries
  int32_t* lid = uf + T;    // [T] particle of a block slot
  lpar[t] = t;
  lid[t] = valid ? i : -1;
  __syncthreads();
  if (!dense) {
#pragma unroll
    for (int u = 0; u < kKeep; ++u)
      if (u < found && (keep[u] >> 16) != 0u) uf_union(lpar, t, (int)(keep[u] >> 16) - 1);
  }
  __syncthreads();
  // the local root, and in the upper half the pairs this particle found
  // (as the lower id: each pair once) -- the cluster build's pair count per
  // cluster without another pass over the pair list
  if (valid) {
    const int32_t lr = lid[uf_find(lpar, t)];
    sc.lroot[base + i] = lr | (min(found, 0xffff) << 16);
    if (sc.bmisc) {  // the multi-workgroup build's forest and zeroed cluster words
      sc.gclus[base + i] = lr;
      sc.gclus[M + base + i] = 0;
    }
  }
  if (sc.bmisc && bx == 0) {  // its counters and the wave pair counts
    for (int k = t; k < kBmWords; k += T) sc.bmisc[(size_t)e * kBmWords + k] = 0;
    for (int k = t; k < sc.wmax; k += T) sc.wave_npairs[(size_t)e * sc.wmax + k] = 0;
  }
  // wave prefix sums, one atomic per wave: every pair to the pair list, the
  // pairs whose partner lies outside the block (all of a dense wave's) also
  // to the cross list
  int nx = 0;
  if (!dense) {
#pragma unroll
    for (int u = 0; u < kKeep; ++u) nx += u < found && (keep[u] >> 16) == 0u ? 1 : 0;
  } else {
    nx = found;
  }
  int v = found, vx = nx;
  v = wave_incl_scan(v);
  vx = wave_incl_scan(vx);
  int wbase = 0, xbase = 0;
  if (lane == 63) {
    wbase = atomicAdd(&sc.gnpairs[e], v);
    xbase = atomicAdd(&sc.gnx[e], vx);
  }
  wbase = __builtin_amdgcn_readlane(wbase, 63);
  xbase = __builtin_amdgcn_readlane(xbase, 63);
  const int my_off = wbase + v - found;
  const int my_xoff = xbase + vx - nx;
  // the multi-workgroup build reads a particle's pairs from here
  if (sc.bmisc && valid) sc.gclus[3 * M + base + i] = my_off;
  uint32_t* out = sc.gplist + (size_t)e * sc.pair_cap;
  uint32_t* xout = sc.xpairs + (size_t)e * sc.pair_cap;
  if (!dense) {
    int w = 0;
#pragma unroll
    for (int u = 0; u < kKeep; ++u) {
      const int k = my_off + u;
      const uint32_t j = keep[u] & 0xffffu;
      if (u < found && k < sc.pair_cap) out[k] = (uint32_t)i | (j << 16);
      if (u < found && (keep[u] >> 16) == 0u) {
        if (my_xoff + w < sc.pair_cap) xout[my_xoff + w] = (uint32_t)i | (j << 16);
        ++w;
      }
    }
    return;
  }
  // a lane found more than kKeep pairs: rescan and write in order
  int w = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    for (int jj = rb[r]; jj < re[r]; ++jj) {
      const int packed = SID(jj);
      const int j = packed & 0xffffff;
      const float rx = per ? (float)(int32_t)(QX(jj) - qx) * sx0
                           : pair_disp(QX(jj), st.img[base + j], qx, ix, sx0, false);
      const float ry = per ? (float)(int32_t)(QY(jj) - qy) * sx1
                           : pair_disp(QY(jj), st.img[M + base + j], qy, iy, sx1, false);
      if (i < j && rx * rx + ry * ry < nb2_row[packed >> 24]) {
        const int k = my_off + w;
        if (k < sc.pair_cap) out[k] = (uint32_t)i | ((uint32_t)j << 16);
        if (my_xoff + w < sc.pair_cap) xout[my_xoff + w] = (uint32_t)i | ((uint32_t)j << 16);
        ++w;
      }
    }
  }
}

template <bool kLocal>
__global__ __launch_bounds__(256) void k_build_pairs(const Derived* __restrict__ d, DevState st,
                                                     Scratch sc, int lx, int ly) {
  __shared__ float nb2[kMaxSpecies * kMaxSpecies];
  __shared__ int32_t uf[2 * 256];
  build_pairs_body<kLocal>(d, st, sc, lx, ly, blockIdx.x, blockIdx.y, nb2, uf);
}

// ----------------------------------------- candidate lists (l1_pairs)
// The next window's pair search, prepared a window ahead.  A pair within
// r_i + r_j + skin at the next window's start positions P' was within
// r_i + r_j + skin + D_i + D_j at this window's start P (D: a particle's
// displacement over the window), so while every D <= cand_disp the pairs of
// P' are among the candidates listed here from P with the radius widened by
// 2 cand_disp (nbc2).  k_check knows every particle that moved >= skin / 2
// (the movers; cand_disp >= skin / 2) and marks the lists usable (cand_ok).
// Built by the wide run kernel's extra workgroups during the run (from the
// window's cell-sorted snapshot, which nothing rewrites before the next
// window's build), so none of this is on the slice's critical path.

// Sorted entry t of env e: its partners j > i among the (2 kc + 1)^2 cells
// around its cell (kc = 2 covers the widened radius: cand_disp <= half a cell
// side; the host requires >= 5 cells a side, so no cell is visited twice).
__device__ __forceinline__ void cand_build_body(const Derived* __restrict__ d, const DevState& st,
                                                const Scratch& sc, int lx, int ly, int e, int t) {
  constexpr int kc = 2;
  const int N = st.n;
  if (t >= N) return;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int32_t* cs = sc.bcstart + (size_t)e * ((size_t)ncx * ncy + 1);
  const int pk = sc.bsid[base + t];
  const int i = pk & 0xffffff;
  const uint32_t qx = sc.bsq[base + t], qy = sc.bsq[M + base + t];
  const int cx = (int)(qx >> (32 - lx)), cy = (int)(qy >> (32 - ly));
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float* lim2 = d->nbc2 + (pk >> 24) * kMaxSpecies;
  // the stencil rows as up to two contiguous sorted ranges each (a periodic
  // row wraps at most once), flattened into one candidate index
  int rb[2 * (2 * kc + 1)], rl[2 * (2 * kc + 1)], nr = 0;
#pragma unroll
  for (int oy = -kc; oy <= kc; ++oy) {
    const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
    int x0 = cx - kc, x1 = cx + kc;
    if (x0 < 0) {
      rb[nr] = cs[row | (ncx + x0)];
      rl[nr] = cs[(row | (ncx - 1)) + 1] - rb[nr];
      ++nr;
      x0 = 0;
    } else if (x1 > ncx - 1) {
      rb[nr] = cs[row];
      rl[nr] = cs[(row | (x1 - ncx)) + 1] - rb[nr];
      ++nr;
      x1 = ncx - 1;
    }
    rb[nr] = cs[row | x0];
    rl[nr] = cs[(row | x1) + 1] - rb[nr];
    ++nr;
  }
  const size_t gi = base + i;
  int n = 0, r = 0, rem = nr > 0 ? rl[0] : 0, jj = nr > 0 ? rb[0] : 0;
  while (true) {
    // four candidates in flight per round
    int pj[4];
    uint32_t xj[4], yj[4];
    int got = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      while (rem == 0 && r + 1 < nr) {
        ++r;
        rem = rl[r];
        jj = rb[r];
      }
      pj[u] = -1;
      if (rem > 0) {
        pj[u] = sc.bsid[base + jj];
        xj[u] = sc.bsq[base + jj];
        yj[u] = sc.bsq[M + base + jj];
        ++jj;
        --rem;
        ++got;
      }
    }
    if (got == 0) break;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (pj[u] < 0) continue;
      const int j = pj[u] & 0xffffff;
      if (j <= i) continue;
      const float rx = (float)(int32_t)(xj[u] - qx) * sx0;
      const float ry = (float)(int32_t)(yj[u] - qy) * sx1;
      if (rx * rx + ry * ry < lim2[pj[u] >> 24]) {
        if (n < kCandMax) sc.cand[(size_t)n * M + gi] = (int32_t)((uint32_t)j | ((uint32_t)pj[u] & 0xff000000u));
        ++n;
      }
    }
  }
  sc.ncand[gi] = min(n, kCandMax);
  if (n > kCandMax) sc.cand_ovf[e] = 1;
}

// The pair search of the slice's first launch (l1_pairs): block bx of env e,
// one thread per particle i (blockDim threads a block).  With usable lists
// (cand_ok) every listed j is tested at the current positions -- the same
// test and pair word as build_pairs_body, so the same pairs -- and kept in
// registers, one atomic per wave reserves the output.  Otherwise the block
// waits for this launch's build sort (sort_done == win1, published with a
// release by its workgroup, which has the lowest block index of the launch
// and so is dispatched before any waiting block) and searches its cells.
__device__ __forceinline__ void pair_filter_body(const Derived* __restrict__ d, const DevState& st,
                                                 const Scratch& sc, int lx, int ly, int bx, int e,
                                                 uint64_t win1, float* nb2, int32_t* uf) {
  const bool ok = sc.cand_ok[e] != 0;  // block-uniform
  if (bx == 0 && threadIdx.x == 0) atomicAdd(&sc.stats[ok ? 0 : 1], 1ull);
  if (!ok) {
    if (threadIdx.x == 0)
      while (__hip_atomic_load(&sc.sort_done[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != win1)
        __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    build_pairs_body<false>(d, st, sc, lx, ly, bx, e, nb2, uf);
    return;
  }
  constexpr int kKeep = 8;
  const int N = st.n, T = blockDim.x;
  const int i = bx * T + (int)threadIdx.x;
  const bool valid = i < N;
  const size_t M = (size_t)st.m, base = (size_t)e * N, gi = base + (valid ? i : 0);
  const int nc = valid ? sc.ncand[gi] : 0;
  const uint32_t qx = st.q[gi], qy = st.q[M + gi];
  // the first eight list entries load with the count (one memory latency,
  // not two; entries past the count are never used); sixteen in flight
  // measured no different
  constexpr int kFly = 8;
  int c0[kFly];
#pragma unroll
  for (int u = 0; u < kFly; ++u) c0[u] = sc.cand[(size_t)u * M + gi];
  const bool multi = sc.multi_species != 0;
  const int si = multi && valid ? (int)st.species[i] : 0;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float* nb2_row = d->nb2 + si * kMaxSpecies;
  int found = 0;
  uint32_t keep[kKeep];
#pragma unroll
  for (int v = 0; v < kKeep; ++v) keep[v] = 0u;
  auto test = [&](int c, uint32_t xj, uint32_t yj) {
    const float rx = (float)(int32_t)(xj - qx) * sx0;
    const float ry = (float)(int32_t)(yj - qy) * sx1;
    return rx * rx + ry * ry < nb2_row[multi ? ((uint32_t)c >> 24) : 0];
  };
  for (int k0 = 0; k0 < nc; k0 += kFly) {  // eight candidates in flight per round
    int cj[kFly];
    uint32_t xj[kFly], yj[kFly];
#pragma unroll
    for (int u = 0; u < kFly; ++u)
      cj[u] = k0 + u < nc ? (k0 == 0 ? c0[u] : sc.cand[(size_t)(k0 + u) * M + gi]) : -1;
#pragma unroll
    for (int u = 0; u < kFly; ++u) {
      const size_t gj = base + (cj[u] < 0 ? 0 : (cj[u] & 0xffffff));
      xj[u] = st.q[gj];
      yj[u] = st.q[M + gj];
    }
#pragma unroll
    for (int u = 0; u < kFly; ++u) {
      if (cj[u] >= 0 && test(cj[u], xj[u], yj[u])) {
        const uint32_t kv = (uint32_t)(cj[u] & 0xffffff);
#pragma unroll
        for (int v = 0; v < kKeep; ++v) keep[v] = found == v ? kv : keep[v];
        ++found;
      }
    }
  }
  const int lane = threadIdx.x & 63;
  role_mark(sc, kMarkFilterLoaded);
  const bool dense = __any(found > kKeep);
  int v = wave_incl_scan(found);
  int wbase = 0;
  if (lane == 63) wbase = atomicAdd(&sc.gnpairs[e], v);
  wbase = __builtin_amdgcn_readlane(wbase, 63);
  role_mark(sc, kMarkFilterReserved);
  const int my_off = wbase + v - found;
  uint32_t* out = sc.gplist + (size_t)e * sc.pair_cap;
  const int cap = sc.pair_cap;
  if (!dense) {
#pragma unroll
    for (int u = 0; u < kKeep; ++u) {
      const int k = my_off + u;
      if (u < found && k < cap) out[k] = (uint32_t)i | (keep[u] << 16);
    }
    return;
  }
  int w = 0;  // a lane kept only kKeep: the wave rescans its lists in order
  for (int k = 0; k < nc; ++k) {
    const int c = sc.cand[(size_t)k * M + gi];
    const size_t gj = base + (c & 0xffffff);
    if (test(c, st.q[gj], st.q[M + gj])) {
      if (my_off + w < cap) out[my_off + w] = (uint32_t)i | ((uint32_t)(c & 0xffffff) << 16);
      ++w;
    }
  }
}

// The packing class v whose free-lane range holds singleton rank r < nfree:
// the largest v >= 2 with freebase[v] <= r (its range is non-empty).
// freebase[2..65] is non-decreasing and freebase[65] = nfree > r, so v - 1 =
// #{u in [2, 65]: freebase[u] <= r}: counted in two rounds of eight
// independent LDS reads (every 8th entry, then the eight from the last of
// those <= r) -- two LDS latencies where a binary search waits for six.
__device__ __forceinline__ int free_class(const int32_t* freebase, int r) {
  int k8 = -1;
#pragma unroll
  for (int q = 0; q < 8; ++q) k8 += freebase[2 + 8 * q] <= r ? 1 : 0;
  int v = 1 + 8 * k8;
#pragma unroll
  for (int q = 0; q < 8; ++q) v += freebase[2 + 8 * k8 + q] <= r ? 1 : 0;
  return v;
}

// LDS words of the large-N variant: the union-find forest only.
__host__ __device__ inline size_t build_lds_words_big(int n) {
  const int wmax = slots_per_env(n, true) / 64;  // either packing
  return 16 + 16 + 3 * 68 + (size_t)((wmax + 3) & ~3) + (size_t)n;
}

// Build step 3, one workgroup per env: union-find over the pair list
// (connected components = clusters), packing of the clusters into 64-lane
// wave slots that never straddle a wave, per-wave pair lists.  kBig: the
// cluster sizes, bases, slots and the pair list stay in global memory (N
// too large for them in LDS); the forest is always in LDS.
// kCopy: the pair list (found pairs) is copied from sc.gplist into LDS;
// otherwise (!kBig) it is in LDS already (k_build_env).
template <bool kBig, bool kCopy, bool kLocal = false>
__device__ __forceinline__ void cluster_build_env(const DevState& st, const Scratch& sc, int e,
                                                  unsigned char* smem, int found) {
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t base = (size_t)e * N;
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);  // 16
  int32_t* misc = wave_sums + 16;                          // 16: 0 flag, 1 waves
  int32_t* classcnt = misc + 16;                           // 68
  int32_t* wavebase = classcnt + 68;                       // 68
  int32_t* freebase = wavebase + 68;                       // 68
  const int wmax = sc.wmax;
  int32_t* wave_np = freebase + 68;                        // wmax (padded)
  int32_t* parent = wave_np + ((wmax + 3) & ~3);           // N
  const size_t M = (size_t)st.m;
  int32_t* csz = kBig ? sc.gclus + base : parent + N;              // N
  int32_t* cbase = kBig ? sc.gclus + M + base : parent + 2 * N;    // N
  int32_t* lslot = kBig ? sc.gclus + 2 * M + base : parent + 3 * N;  // N
  uint32_t* plist = kBig ? sc.gplist + (size_t)e * sc.pair_cap
                         : reinterpret_cast<uint32_t*>(parent + 4 * N);  // pair_cap
  const int S = sc.S;
  // kFused (LDS forest): the root walks also count the cluster sizes;
  // kCount: the union sweep counts each particle's pairs (as the lower index)
  // in lslot, and the root walks add them to their cluster -- no separate
  // sweep over the pair list for the one-pass pair counts
  constexpr bool kFused = !kBig;
  constexpr bool kCount = kFused && !kLocal;
  SWARM_STAMP(6);
  const int npairs = min(found, sc.pair_cap);
  // kLocal: the pair search's blocks unioned their own pairs already
  // (sc.lroot: a forest of depth one), only the cross-block pairs remain
  const int nx = kLocal ? sc.gnx[e] : 0;
  const uint32_t* xl = sc.xpairs + (size_t)e * sc.pair_cap;
  for (int k = tid; k < 68; k += T) classcnt[k] = 0;
  for (int k = tid; k < wmax; k += T) wave_np[k] = 0;
  // overflow of the pair or cross list -> global path
  if (tid < 16) misc[tid] = tid == 0 && (found > sc.pair_cap || nx > sc.pair_cap) ? 1 : 0;
  for (int i = tid; i < N; i += T) {
    if (kLocal) {
      const uint32_t l = (uint32_t)sc.lroot[base + i];
      parent[i] = (int32_t)(l & 0xffffu);
      lslot[i] = (int32_t)(l >> 16);  // the member's pair count, until its rank replaces it
    } else {
      parent[i] = i;
      if (kCount) lslot[i] = 0;
    }
    csz[i] = 0;
    cbase[i] = 0;  // pair count of a cluster (one-pass packing), then its base
  }
  if (!kBig && kCopy) {  // pair list into LDS, four loads in flight per thread
    const uint32_t* gp = sc.gplist + (size_t)e * sc.pair_cap;
    for (int k0 = tid; k0 < npairs; k0 += 4 * T) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = k0 + u * T < npairs ? gp[k0 + u * T] : 0u;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k0 + u * T < npairs) plist[k0 + u * T] = v[u];
    }
  }
  __syncthreads();
  SWARM_STAMP(11);
  // kBig: the arrays below live in global memory, so every loop issues its
  // loads / atomics kU at a time before using them -- one memory latency per
  // kU iterations, not one per iteration.  (In LDS, kU = 4 measured no
  // better than 1 at E = 1: the union phase 1 k cycles shorter, the
  // others longer.)
  constexpr int kU = kBig ? 8 : 1;
  // The pair sweeps visit the LDS pair list in a spread order: neighbouring
  // pairs of the cell-sorted list usually share a cluster, so lanes of one
  // wave taking consecutive pairs contend on the same root / wave counter
  // (LDS atomics to one address serialise, union-find CAS retries).  Sweep
  // index k maps to pair (k mod 64) R + k / 64, R = ceil(npairs / 64): the
  // lanes of a wave take pairs R apart (phase stamps: the union phase was
  // 16 k cycles of k_cluster_build's 46 k at E = 1).  kBig keeps the
  // identity (its list is in global memory, read kU at a time).
  const int spread_r = (npairs + 63) >> 6;
  const int nsweep = kBig ? npairs : 64 * spread_r;
  auto sweep_pair = [&](int k) { return kBig ? k : (k & 63) * spread_r + (k >> 6); };
  // (the union sweep reads its pairs four at a time even in LDS: the
  // unions are serial per thread, the list reads need not be)
  constexpr int kUU = kU > 4 ? kU : 4;
  if (kLocal) {  // the cross-block pairs only (global memory, few)
    const int nxc = min(nx, sc.pair_cap);
    for (int k0 = tid; k0 < nxc; k0 += kUU * T) {
      uint32_t pr[kUU];
#pragma unroll
      for (int u = 0; u < kUU; ++u) pr[u] = k0 + u * T < nxc ? xl[k0 + u * T] : 0u;
#pragma unroll
      for (int u = 0; u < kUU; ++u)
        if (k0 + u * T < nxc) uf_union(parent, (int)(pr[u] & 0xffffu), (int)(pr[u] >> 16));
    }
  } else {
    for (int k0 = tid; k0 < nsweep; k0 += kUU * T) {
      uint32_t pr[kUU];
      bool ok[kUU];
#pragma unroll
      for (int u = 0; u < kUU; ++u) {
        const int pk = sweep_pair(k0 + u * T);
        ok[u] = k0 + u * T < nsweep && pk < npairs;
        pr[u] = ok[u] ? plist[pk] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kUU; ++u)
        if (ok[u]) {
          if (kCount && sc.one_pass) atomicAdd(&lslot[pr[u] & 0xffffu], 1);
          uf_union_pair(parent, (int)(pr[u] & 0xffffu), (int)(pr[u] >> 16));
        }
    }
  }
  __syncthreads();
  SWARM_STAMP(7);
  // every particle points at its root (two walks in lockstep per thread);
  // in LDS each walk's end counts its member at once (cluster sizes, the
  // member's rank in lslot): the roots are final after the union sweep, and
  // a walk that passes a member pointed at its root by another thread still
  // ends at the same root -- one barrier and one pass over parent[] fewer
  for (int i = tid; i < N; i += 2 * T) {
    const bool two = i + T < N;
    int a = i, b = two ? i + T : i;
    const int npa = kFused && (kLocal || kCount) ? lslot[i] : 0;
    const int npb = kFused && (kLocal || kCount) && two ? lslot[i + T] : 0;
    uf_find2(parent, a, b);
    parent[i] = a;
    if (two) parent[i + T] = b;
    if (kFused) {
      const int ra = atomicAdd(&csz[a], 1);
      const int rb = two ? atomicAdd(&csz[b], 1) : 0;
      lslot[i] = ra;
      if (two) lslot[i + T] = rb;
      if ((kLocal || kCount) && sc.one_pass) {
        if (npa > 0) atomicAdd(&cbase[a], npa);
        if (npb > 0) atomicAdd(&cbase[b], npb);
      }
    }
  }
  __syncthreads();
  if (!kFused)
  for (int i0 = tid; i0 < N; i0 += kU * T) {
    int32_t r[kU], np_u[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) np_u[u] = kLocal && i0 + u * T < N ? lslot[i0 + u * T] : 0;
#pragma unroll
    for (int u = 0; u < kU; ++u) r[u] = i0 + u * T < N ? atomicAdd(&csz[parent[i0 + u * T]], 1) : 0;
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (i0 + u * T < N) lslot[i0 + u * T] = r[u];
    if (kLocal && sc.one_pass) {  // the cluster's pairs: the members' counts of the pair search
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (np_u[u] > 0) atomicAdd(&cbase[parent[i0 + u * T]], np_u[u]);
    }
  }
  if (!kLocal && !kCount && sc.one_pass)
    for (int k0 = tid; k0 < nsweep; k0 += kU * T) {
      uint32_t pr[kU];
      bool ok[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int pk = sweep_pair(k0 + u * T);
        ok[u] = k0 + u * T < nsweep && pk < npairs;
        pr[u] = ok[u] ? plist[pk] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (ok[u]) atomicAdd(&cbase[parent[pr[u] & 0xffffu]], 1);
    }
  __syncthreads();
  // Lanes reserved per cluster (its packing class w): its size s, or with
  // one-pass packing max(s, min(pairs, 64, 2 s)), so that the clusters of a
  // wave have at most 64 pairs (one pair pass per sub-step) unless a cluster
  // is denser than 2 pairs per particle.  Results do not depend on it.
  for (int i0 = tid; i0 < N; i0 += kU * T) {
    int32_t sz[kU], pc[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * T;
      const bool root = i < N && parent[i] == i;
      sz[u] = root ? csz[i] : 0;
      pc[u] = root ? cbase[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * T;
      const bool root = i < N && parent[i] == i;
      const int s = sz[u];
      const int w = sc.one_pass ? max(s, min(min(pc[u], 64), 2 * s)) : s;
      // one LDS atomic per root (measured, 4096 colloids: the wave-aggregated
      // counters of the packed build cost this one-workgroup build ~0.9 us,
      // cluster build 16.7 -> 15.8 us without them)
      if (!root) continue;
      if (s > 64) {  // wider than a wave: a big cluster, run by k_check's workgroup
        atomicAdd(&misc[4], s);
        cbase[i] = kBigMark;
      } else {
        csz[i] = w;
        cbase[i] = atomicAdd(&classcnt[w], 1);
      }
    }
  }
  __syncthreads();
  SWARM_STAMP(8);
  // -> global path (3-D: any big cluster; its run is 2-D only).  misc[0]
  // (list overflow) and misc[4] are final here, so every thread decides
  // alike, with no barrier for a flag
  if (misc[0] || misc[4] > min(kBigMax, (int)blockDim.x) || (st.dims == 3 && misc[4] > 0)) {
    if (tid == 0) {
      sc.fallback[e] = 1;
      sc.env_waves[e] = 0;
      sc.big_n[e] = 0;
      sc.big_np[e] = 0;
    }
    return;
  }
  // Waves per class.  The tail lanes a class leaves free in its waves
  // (64 - per * w in a full wave, more in its last one) take the singletons
  // first; only the rest of them get waves of their own (fewer, fuller
  // waves: the run kernel's cost is per wave).
  if (tid < 64) {
    const int w = tid + 1;
    const int per = udiv_small(64, w);
    const int cnt = classcnt[w];
    int32_t nw = udiv_small(cnt + per - 1, per);
    int32_t fl = 0;
    if (w >= 2 && nw > 0) fl = (nw - 1) * (64 - per * w) + (64 - (cnt - (nw - 1) * per) * w);
    int32_t f = fl;
    f = wave_incl_scan(f);
    freebase[w] = f - fl;
    const int32_t F = sc.fill_singletons ? __builtin_amdgcn_readlane(f, 63) : 0;
    if (w == 1) nw = (max(cnt - F, 0) + 63) / 64;
    int32_t v = nw;
    v = wave_incl_scan(v);
    wavebase[w] = v - nw;
    if (tid == 63) {
      misc[1] = v;
      misc[3] = F;
      freebase[65] = F;
    }
  }
  __syncthreads();
  // Every particle's slot in one pass: its cluster's base (from the root's
  // class and class rank, worked out by each member for itself -- no pass
  // that stores the bases and no barrier before the members read them) plus
  // its rank in the cluster.
  const int nfree = misc[3];
  for (int i0 = tid; i0 < N; i0 += kU * T) {
    int32_t rt[kU], ls[kU], sz[kU], rk[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * T;
      rt[u] = i < N ? parent[i] : 0;
      ls[u] = i < N ? lslot[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * T;
      sz[u] = i < N ? csz[rt[u]] : 0;
      rk[u] = i < N ? cbase[rt[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * T;
      if (i >= N) continue;
      const int root = rt[u], s = sz[u], r = rk[u];
      int slot;
      if (r == kBigMark) {  // big-cluster member m: slot -1 - m
        const int m = atomicAdd(&misc[5], 1);
        sc.big_list[(size_t)e * kBigMax + m] = i;
        slot = -1 - m;
      } else {
        int cb;
        if (s == 1 && r < nfree) {
          // the class v whose free-lane range holds r, then wave j and lane
          const int v = free_class(freebase, r);
          const int per = udiv_small(64, v);
          const int nw = udiv_small(classcnt[v] + per - 1, per);
          const int ffull = 64 - per * v;
          const int t = r - freebase[v];
          int j, lane;
          if (t < (nw - 1) * ffull) {
            j = udiv_small(t, ffull);
            lane = per * v + (t - j * ffull);
          } else {
            j = nw - 1;
            lane = (classcnt[v] - (nw - 1) * per) * v + (t - (nw - 1) * ffull);
          }
          cb = (wavebase[v] + j) * 64 + lane;
        } else if (s == 1) {
          const int r2 = r - nfree;
          cb = (wavebase[1] + r2 / 64) * 64 + r2 % 64;
        } else {
          const int per = udiv_small(64, s), rq = udiv_small(r, per);
          cb = (wavebase[s] + rq) * 64 + (r - rq * per) * s;
        }
        slot = cb + ls[u];
        sc.perm[(size_t)e * S + slot] = i;
      }
      lslot[i] = slot;
      sc.slot_of[base + i] = slot;
      sc.root[base + i] = root;
    }
  }
  __syncthreads();
  SWARM_STAMP(9);
  // per-wave pair lists (both particles of a pair share a cluster, so a wave)
  for (int k0 = tid; k0 < nsweep; k0 += kU * T) {
   uint32_t prs[kU];
   bool okp[kU];
#pragma unroll
   for (int u = 0; u < kU; ++u) {
     const int pk = sweep_pair(k0 + u * T);
     okp[u] = k0 + u * T < nsweep && pk < npairs;
     prs[u] = okp[u] ? plist[pk] : 0u;
   }
   int32_t sis[kU], sjs[kU];
#pragma unroll
   for (int u = 0; u < kU; ++u) {
     sis[u] = lslot[prs[u] & 0xffffu];
     sjs[u] = lslot[prs[u] >> 16];
   }
#pragma unroll
   for (int u = 0; u < kU; ++u) {
    if (!okp[u]) continue;
    const uint32_t pr = prs[u];
    const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
    const int si = sis[u], sj = sjs[u];
    const uint32_t spp =
        sc.multi_species ? (uint32_t)(st.species[i] * kMaxSpecies + st.species[j]) : 0u;
    if (si < 0) {  // a big cluster's pair (both members of it)
      const int idx = atomicAdd(&misc[6], 1);
      if (idx < kBigPairs)
        sc.big_pairs[(size_t)e * kBigPairs + idx] =
            (uint32_t)(-1 - si) | ((uint32_t)(-1 - sj) << 10) | (spp << 20);
      else
        misc[2] = 1;  // -> global path
      continue;
    }
    const int wv = si >> 6;
    const int idx = atomicAdd(&wave_np[wv], 1);
    if (idx < kPairsPerWave)
      sc.pairs[((size_t)e * wmax + wv) * kPairsPerWave + idx] =
          (uint32_t)(si & 63) | ((uint32_t)(sj & 63) << 6) | (spp << 12);
    else
      misc[2] = 1;  // a wave with more than kPairsPerWave pairs
   }
  }
  __syncthreads();
  SWARM_STAMP(10);
  for (int w = tid; w < misc[1]; w += T)
    sc.wave_npairs[(size_t)e * wmax + w] = min(wave_np[w], kPairsPerWave);
  if (tid == 0) {
    sc.env_waves[e] = misc[2] ? 0 : misc[1];
    sc.fallback[e] = misc[2] ? 1 : 0;
    sc.big_n[e] = misc[5];
    sc.big_np[e] = min(misc[6], kBigPairs);
  }
}

// LDS words of the packed large-N build: two words per particle (N < 65536).
__host__ __device__ inline size_t build_lds_words_packed(int n) {
  const int wmax = slots_per_env(n, true) / 64;
  return 16 + 16 + 3 * 68 + (size_t)((wmax + 3) & ~3) + 2 * (size_t)n;
}

// The large-N build (same result as cluster_build_env<true, false>) with
// its per-particle and per-cluster arrays packed into two LDS words per
// particle instead of global memory (whose returning atomics and dependent
// loads cost ~3x LDS per element from one CU):
//   A[i]: union-find parent; then root | rank << 16 (rank = i's lane within
//         its cluster); then i's wave slot;
//   B[r]: for a root r, size | pairs << 16 (atomic counters, no carry:
//         size < 2^16); then class rank | w << 24; then the cluster's first
//         slot (or kBigMark).
// The pair list stays in global memory (read kU at a time).  Used by the
// large-N builds that union the whole pair list (3-D; 2-D envs with the
// block-local pair search take the multi-workgroup build, k_mwb_*).
__device__ void cluster_build_env_packed(const DevState& st, const Scratch& sc, int e,
                                         unsigned char* smem, int found) {
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t base = (size_t)e * N;
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);  // 16
  int32_t* misc = wave_sums + 16;                          // 16: 0 flag, 1 waves
  int32_t* classcnt = misc + 16;                           // 68
  int32_t* wavebase = classcnt + 68;                       // 68
  int32_t* freebase = wavebase + 68;                       // 68
  const int wmax = sc.wmax;
  int32_t* wave_np = freebase + 68;                        // wmax (padded)
  int32_t* A = wave_np + ((wmax + 3) & ~3);                // N
  int32_t* B = A + N;                                      // N
  const uint32_t* plist = sc.gplist + (size_t)e * sc.pair_cap;
  const int S = sc.S;
  constexpr int kU = 8;
  SWARM_STAMP(6);
  const int npairs = min(found, sc.pair_cap);
  for (int k = tid; k < 68; k += T) classcnt[k] = 0;
  for (int k = tid; k < wmax; k += T) wave_np[k] = 0;
  // overflow of the pair list -> global path
  if (tid < 16) misc[tid] = tid == 0 && found > sc.pair_cap ? 1 : 0;
  for (int i = tid; i < N; i += T) {
    A[i] = i;
    B[i] = 0;
  }
  __syncthreads();
  for (int k0 = tid; k0 < npairs; k0 += kU * T) {
    uint32_t pr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) pr[u] = k0 + u * T < npairs ? plist[k0 + u * T] : 0u;
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (k0 + u * T < npairs) uf_union(A, (int)(pr[u] & 0xffffu), (int)(pr[u] >> 16));
  }
  __syncthreads();
  SWARM_STAMP(7);
  for (int i = tid; i < N; i += T) A[i] = uf_find(A, i);
  __syncthreads();
  for (int i = tid; i < N; i += T) {  // size, the member's rank
    const int root = A[i];
    const uint32_t r = (uint32_t)atomicAdd(&B[root], 1) & 0xffffu;
    A[i] = root | (int32_t)(r << 16);
  }
  if (sc.one_pass)
    for (int k0 = tid; k0 < npairs; k0 += kU * T) {
      uint32_t pr[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) pr[u] = k0 + u * T < npairs ? plist[k0 + u * T] : 0u;
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (k0 + u * T < npairs) {
          // the root of the pair's first particle: A holds root | rank << 16
          // of particles whose rank is already stored, root otherwise
          const int a = (int)(pr[u] & 0xffffu);
          atomicAdd(&B[A[a] & 0xffff], 1 << 16);
        }
    }
  __syncthreads();
  // lanes reserved per cluster (cluster_build_env): class w, class rank
  for (int i = tid; i < N; i += T) {
    const bool root = (A[i] & 0xffff) == i;  // roots only
    const uint32_t b = root ? (uint32_t)B[i] : 0u;
    const int s = (int)(b & 0xffffu), pairs = (int)(b >> 16);
    const int w = sc.one_pass ? max(s, min(min(pairs, 64), 2 * s)) : s;
    // the two most frequent classes by one atomic per wave
    const int r1 = wave_class_add(&classcnt[1], root && s <= 64 && w == 1);
    const int r2 = wave_class_add(&classcnt[2], root && s <= 64 && w == 2);
    if (!root) continue;
    if (s > 64) {  // wider than a wave: a big cluster, run by k_check's workgroup
      atomicAdd(&misc[4], s);
      B[i] = kBigMark;
    } else {
      B[i] = (w == 1 ? r1 : (w == 2 ? r2 : atomicAdd(&classcnt[w], 1))) | (w << 24);
    }
  }
  __syncthreads();
  SWARM_STAMP(8);
  // -> global path (3-D: any big cluster; its run is 2-D only)
  if (tid == 0 && (misc[4] > min(kBigMax, (int)blockDim.x) || (st.dims == 3 && misc[4] > 0)))
    misc[0] = 1;
  __syncthreads();
  if (misc[0]) {
    if (tid == 0) {
      sc.fallback[e] = 1;
      sc.env_waves[e] = 0;
      sc.big_n[e] = 0;
      sc.big_np[e] = 0;
    }
    return;
  }
  if (tid < 64) {  // waves per class (cluster_build_env)
    const int w = tid + 1;
    const int per = udiv_small(64, w);
    const int cnt = classcnt[w];
    int32_t nw = udiv_small(cnt + per - 1, per);
    int32_t fl = 0;
    if (w >= 2 && nw > 0) fl = (nw - 1) * (64 - per * w) + (64 - (cnt - (nw - 1) * per) * w);
    int32_t f = fl;
    f = wave_incl_scan(f);
    freebase[w] = f - fl;
    const int32_t F = sc.fill_singletons ? __builtin_amdgcn_readlane(f, 63) : 0;
    if (w == 1) nw = (max(cnt - F, 0) + 63) / 64;
    int32_t v = nw;
    v = wave_incl_scan(v);
    wavebase[w] = v - nw;
    if (tid == 63) {
      misc[1] = v;
      misc[3] = F;
      freebase[65] = F;
    }
  }
  __syncthreads();
  const int nfree = misc[3];
  for (int i = tid; i < N; i += T) {
    if ((A[i] & 0xffff) != i) continue;
    const int32_t b = B[i];
    if (b == kBigMark) continue;
    const int s = (b >> 24) & 0x7f;
    const int r = b & 0xffffff;
    int cb;
    if (s == 1 && r < nfree) {
      const int v = free_class(freebase, r), per = udiv_small(64, v);
      const int nw = udiv_small(classcnt[v] + per - 1, per);
      const int ffull = 64 - per * v;
      const int t = r - freebase[v];
      int j, lane;
      if (t < (nw - 1) * ffull) {
        j = udiv_small(t, ffull);
        lane = per * v + (t - j * ffull);
      } else {
        j = nw - 1;
        lane = (classcnt[v] - (nw - 1) * per) * v + (t - (nw - 1) * ffull);
      }
      cb = (wavebase[v] + j) * 64 + lane;
    } else if (s == 1) {
      const int r2 = r - nfree;
      cb = (wavebase[1] + r2 / 64) * 64 + r2 % 64;
    } else {
      const int per = udiv_small(64, s), rq = udiv_small(r, per);
      cb = (wavebase[s] + rq) * 64 + (r - rq * per) * s;
    }
    B[i] = cb;
  }
  __syncthreads();
  for (int i = tid; i < N; i += T) {
    const int32_t a = A[i];
    const int root = a & 0xffff;
    const int rank = (int)((uint32_t)a >> 16);
    const int32_t cb = B[root];
    int slot;
    if (cb == kBigMark) {  // big-cluster member m: slot -1 - m
      const int m = atomicAdd(&misc[5], 1);
      sc.big_list[(size_t)e * kBigMax + m] = i;
      slot = -1 - m;
    } else {
      slot = cb + rank;
      sc.perm[(size_t)e * S + slot] = i;
    }
    sc.slot_of[base + i] = slot;
    sc.root[base + i] = root;
    A[i] = slot;  // only this thread reads A[i] in this loop
  }
  __syncthreads();
  SWARM_STAMP(9);
  for (int k0 = tid; k0 < npairs; k0 += kU * T) {
    uint32_t prs[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) prs[u] = k0 + u * T < npairs ? plist[k0 + u * T] : 0u;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (k0 + u * T >= npairs) continue;
      const uint32_t pr = prs[u];
      const int i = (int)(pr & 0xffffu), j = (int)(pr >> 16);
      const int si = A[i], sj = A[j];
      const uint32_t spp =
        sc.multi_species ? (uint32_t)(st.species[i] * kMaxSpecies + st.species[j]) : 0u;
      if (si < 0) {  // a big cluster's pair (both members of it)
        const int idx = atomicAdd(&misc[6], 1);
        if (idx < kBigPairs)
          sc.big_pairs[(size_t)e * kBigPairs + idx] =
              (uint32_t)(-1 - si) | ((uint32_t)(-1 - sj) << 10) | (spp << 20);
        else
          misc[2] = 1;  // -> global path
        continue;
      }
      const int wv = si >> 6;
      const int idx = atomicAdd(&wave_np[wv], 1);
      if (idx < kPairsPerWave)
        sc.pairs[((size_t)e * wmax + wv) * kPairsPerWave + idx] =
            (uint32_t)(si & 63) | ((uint32_t)(sj & 63) << 6) | (spp << 12);
      else
        misc[2] = 1;  // a wave with more than kPairsPerWave pairs
    }
  }
  __syncthreads();
  SWARM_STAMP(10);
  for (int w = tid; w < misc[1]; w += T)
    sc.wave_npairs[(size_t)e * wmax + w] = min(wave_np[w], kPairsPerWave);
  if (tid == 0) {
    sc.env_waves[e] = misc[2] ? 0 : misc[1];
    sc.fallback[e] = misc[2] ? 1 : 0;
    sc.big_n[e] = misc[5];
    sc.big_np[e] = min(misc[6], kBigPairs);
  }
}

__global__ __launch_bounds__(1024) void k_cluster_build_packed(DevState st, Scratch sc) {
  extern __shared__ __align__(16) unsigned char smem[];
  cluster_build_env_packed(st, sc, blockIdx.x, smem, sc.gnpairs[blockIdx.x]);
}

// ------------------------------------- multi-workgroup build (large N, 2-D)
// The cluster build of cluster_build_env_packed<true> spread over the chip
// in four launches of 256-thread workgroups (one env per grid row), for envs
// whose one-workgroup build is the slice's longest serial stage (C5, 16384
// colloids: 47.5 us on one CU).  Same decomposition rules -- connected
// components of the rc + skin graph, lanes per cluster by packing class,
// singletons into the classes' tail lanes -- with the per-particle and
// per-cluster words in global memory (sc.gclus) and the class counters in
// sc.bmisc; the slot order differs from the one-workgroup build, which
// results do not depend on (fixed-point sums).
//   gclus[0 .. M):  P, the union-find forest; the pair search writes each
//                   particle's block-local root (a forest of depth one)
//   gclus[M .. 2M): B, per root: size | pairs << 16 (k_mwb_size), then
//                   class rank | class << 24, or kMwbBig | first member
//                   (k_mwb_class); zeroed by the pair search
//   gclus[2M .. 3M): A, root | rank in the cluster << 16 (k_mwb_size)
// Every launch boundary orders the phases; inside a launch the workgroups
// meet only through agent-scope atomics, and the last workgroup of a launch
// (a ticket) does the launch's serial remainder.

__device__ __forceinline__ int32_t agent_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Root of x in the global forest while other workgroups link roots
// (agent-scope loads: a link made on another XCD is seen).
__device__ __forceinline__ int mwb_find(const int32_t* P, int x) {
  int p = agent_load(P + x);
  while (p != x) {
    x = p;
    p = agent_load(P + x);
  }
  return x;
}

// The last workgroup of a launch to finish (ticket).  No fences: what the
// last workgroup reads are counters the others changed by atomics whose
// results they waited for before their ticket (an agent-scope fence would
// write back and invalidate the L2: ~0.4 us per workgroup, measured 24 us
// for a 64-workgroup launch).
__device__ __forceinline__ bool mwb_last_block(int32_t* ticket, int nblocks, int32_t* flag_lds) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = atomicAdd(ticket, 1);
    *flag_lds = t == nblocks - 1;
    if (t == nblocks - 1) *ticket = 0;  // ready for the next build
  }
  __syncthreads();
  return *flag_lds != 0;
}

// k_mwb_union: the cross-block pairs of the pair search, unioned in the
// global forest (the larger root is hooked under the smaller by CAS; a
// failed CAS -- the root was hooked meanwhile -- walks again).
__global__ __launch_bounds__(256) void k_mwb_union(DevState st, Scratch sc) {
  const int e = blockIdx.y;
  const size_t base = (size_t)e * st.n;
  int32_t* P = sc.gclus + base;
  const int nx = min(sc.gnx[e], sc.pair_cap);
  const uint32_t* xl = sc.xpairs + (size_t)e * sc.pair_cap;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nx; k += gridDim.x * blockDim.x) {
    const uint32_t pr = xl[k];
    int a = (int)(pr & 0xffffu), b = (int)(pr >> 16);
    while (true) {
      a = mwb_find(P, a);
      b = mwb_find(P, b);
      if (a == b) break;
      if (a > b) {
        const int t = a;
        a = b;
        b = t;
      }
      int expect = b;
      if (__hip_atomic_compare_exchange_strong(P + b, &expect, a, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        break;
    }
  }
}

// k_mwb_size: every particle's root (the forest is final), its rank in the
// cluster and the cluster's size and pair count (one atomic per particle on
// its root's B word; the pair count is the pair search's per-particle count).
__global__ __launch_bounds__(256) void k_mwb_size(DevState st, Scratch sc) {
  const int e = blockIdx.y, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int32_t* P = sc.gclus + base;
  int32_t* B = sc.gclus + M + base;
  int r = i, p = P[i];
  while (p != r) {
    r = p;
    p = P[r];
  }
  const int np_i = sc.one_pass ? (int)((uint32_t)sc.lroot[base + i] >> 16) : 0;
  const uint32_t rank = (uint32_t)atomicAdd(&B[r], 1 + (np_i << 16)) & 0xffffu;
  sc.gclus[2 * M + base + i] = r | (int32_t)(rank << 16);
  // the env's slots, idle until k_mwb_slots places the colloids (spread over
  // this launch instead of k_sort_scan's one workgroup)
  for (int k = i; k < sc.S; k += N) sc.perm[(size_t)e * sc.S + k] = -1;
}

// k_mwb_class: every root's packing class and rank in it, counted per
// workgroup in LDS (wave-aggregated for the singleton and pair classes) and
// reserved with one global atomic per class and workgroup; a big cluster
// (wider than a wave) reserves its members' range of the big list.  The
// last workgroup lays the classes out in waves (cluster_build_env) and
// publishes the env's waves and flags, or sends the env to the global path
// (a list overflowed or too many big-cluster members).
__global__ __launch_bounds__(1024) void k_mwb_class(DevState st, Scratch sc) {
  __shared__ int32_t lcnt[68], lbase[68];
  __shared__ int32_t last_flag;
  const int e = blockIdx.y, N = st.n, tid = threadIdx.x;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  int32_t* bm = sc.bmisc + (size_t)e * kBmWords;
  int32_t* B = sc.gclus + M + base;
  const int32_t* A = sc.gclus + 2 * M + base;
  if (tid < 68) lcnt[tid] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + tid;
  const bool root = i < N && (A[i] & 0xffff) == i;
  const uint32_t b = root ? (uint32_t)B[i] : 0u;
  const int s = (int)(b & 0xffffu), pairs = (int)(b >> 16);
  const int w = sc.one_pass ? max(s, min(min(pairs, 64), 2 * s)) : s;
  const int r1 = wave_class_add(lcnt + 1, root && s <= 64 && w == 1);
  const int r2 = wave_class_add(lcnt + 2, root && s <= 64 && w == 2);
  int lr = w == 1 ? r1 : r2;
  if (root && s <= 64 && w > 2) lr = atomicAdd(&lcnt[w], 1);
  __syncthreads();
  if (tid < 68 && lcnt[tid] > 0) lbase[tid] = atomicAdd(bm + kBmClass + tid, lcnt[tid]);
  __syncthreads();
  if (root) {
    if (s > 64)  // a big cluster, run by k_check's workgroup
      B[i] = (int32_t)(kMwbBig | (uint32_t)atomicAdd(bm + kBmMisc + 4, s));
    else
      B[i] = (lbase[w] + lr) | (w << 24);
  }
  if (!mwb_last_block(bm + kBmMisc + 8, gridDim.x, &last_flag)) return;
  const int nbig = agent_load(bm + kBmMisc + 4);
  const bool over = agent_load(sc.gnpairs + e) > sc.pair_cap ||
                    agent_load(sc.gnx + e) > sc.pair_cap || nbig > min(kBigMax, 1024);
  if (over) {
    if (tid == 0) {
      bm[kBmMisc + 0] = 1;
      sc.fallback[e] = 1;
      sc.env_waves[e] = 0;
      sc.big_n[e] = 0;
      sc.big_np[e] = 0;
    }
    return;
  }
  if (tid < 64) {  // waves per class (cluster_build_env)
    const int w = tid + 1;
    const int per = udiv_small(64, w);
    const int cnt = agent_load(bm + kBmClass + w);
    int32_t nw = udiv_small(cnt + per - 1, per);
    int32_t fl = 0;
    if (w >= 2 && nw > 0) fl = (nw - 1) * (64 - per * w) + (64 - (cnt - (nw - 1) * per) * w);
    int32_t f = fl;
    f = wave_incl_scan(f);
    bm[kBmFree + w] = f - fl;
    const int32_t F = sc.fill_singletons ? __builtin_amdgcn_readlane(f, 63) : 0;
    if (w == 1) nw = (max(cnt - F, 0) + 63) / 64;
    int32_t v = nw;
    v = wave_incl_scan(v);
    bm[kBmWave + w] = v - nw;
    if (tid == 63) {
      bm[kBmMisc + 1] = v;
      bm[kBmMisc + 3] = F;
      bm[kBmFree + 65] = F;
      sc.env_waves[e] = v;
      sc.fallback[e] = 0;  // set by k_mwb_pairs when a list overflows
      sc.big_n[e] = nbig;
      sc.big_np[e] = 0;
    }
  }
}

// A particle's wave slot from its root's class word and the class layout
// (tables in LDS: counts, first waves, free-lane bases; misc[3] = free lanes).
__device__ __forceinline__ int mwb_slot(int32_t a, int32_t broot, const int32_t* cls,
                                        const int32_t* wbase, const int32_t* fbase, int nfree) {
  const int rank = (int)((uint32_t)a >> 16);
  if ((uint32_t)broot & kMwbBig) return -1 - (int)(((uint32_t)broot & ~kMwbBig) + rank);
  const int s = (broot >> 24) & 0x7f;
  const int r = broot & 0xffffff;
  int cb;
  if (s == 1 && r < nfree) {
    const int v = free_class(fbase, r), per = udiv_small(64, v);
    const int nw = udiv_small(cls[v] + per - 1, per);
    const int ffull = 64 - per * v;
    const int t = r - fbase[v];
    int j, lane;
    if (t < (nw - 1) * ffull) {
      j = udiv_small(t, ffull);
      lane = per * v + (t - j * ffull);
    } else {
      j = nw - 1;
      lane = (cls[v] - (nw - 1) * per) * v + (t - (nw - 1) * ffull);
    }
    cb = (wbase[v] + j) * 64 + lane;
  } else if (s == 1) {
    const int r2 = r - nfree;
    cb = (wbase[1] + r2 / 64) * 64 + r2 % 64;
  } else {
    const int per = udiv_small(64, s), rq = udiv_small(r, per);
    cb = (wbase[s] + rq) * 64 + (r - rq * per) * s;
  }
  return cb + rank;
}

// k_mwb_slots: every particle's wave slot (perm, slot_of, root); a
// big-cluster member lists its pairs (as the lower index) for k_check's
// big-cluster run, its partner's member index worked out the same way.
__global__ __launch_bounds__(256) void k_mwb_slots(DevState st, Scratch sc) {
  __shared__ int32_t tab[3 * 68];
  const int e = blockIdx.y, N = st.n, tid = threadIdx.x;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int32_t* bm = sc.bmisc + (size_t)e * kBmWords;
  if (bm[kBmMisc + 0]) return;  // the env runs on the global path (k_mwb_class)
  for (int k = tid; k < 3 * 68; k += blockDim.x) tab[k] = bm[kBmClass + k];
  __syncthreads();
  const int32_t *cls = tab, *wbase = tab + 68, *fbase = tab + 136;
  const int nfree = bm[kBmMisc + 3];
  const int32_t* B = sc.gclus + M + base;
  const int32_t* A = sc.gclus + 2 * M + base;
  const int i = blockIdx.x * blockDim.x + tid;
  if (i >= N) return;
  const int32_t a = A[i];
  const int root = a & 0xffff;
  const int slot = mwb_slot(a, B[root], cls, wbase, fbase, nfree);
  sc.slot_of[base + i] = slot;
  sc.root[base + i] = root;
  if (slot >= 0) {
    sc.perm[(size_t)e * sc.S + slot] = i;
    return;
  }
  sc.big_list[(size_t)e * kBigMax + (-1 - slot)] = i;
  // the member's pairs (i the lower index): contiguous in the pair list
  const int n_i = (int)((uint32_t)sc.lroot[base + i] >> 16);
  const int off = sc.gclus[3 * M + base + i];
  const uint32_t* plist = sc.gplist + (size_t)e * sc.pair_cap;
  for (int k = 0; k < n_i && off + k < sc.pair_cap; ++k) {
    const int j = (int)(plist[off + k] >> 16);
    const int32_t aj = A[j];
    const int sj = mwb_slot(aj, B[aj & 0xffff], cls, wbase, fbase, nfree);
    const uint32_t spp =
        sc.multi_species ? (uint32_t)(st.species[i] * kMaxSpecies + st.species[j]) : 0u;
    const int idx = atomicAdd(&sc.big_np[e], 1);
    if (idx < kBigPairs)
      sc.big_pairs[(size_t)e * kBigPairs + idx] =
          (uint32_t)(-1 - slot) | ((uint32_t)(-1 - sj) << 10) | (spp << 20);
    else
      sc.fallback[e] = 1;  // -> global path
  }
}

// k_mwb_pairs: one wave per run wave: each lane's particle lists its pairs
// (as the lower index, contiguous in the pair list from the pair search) at
// its offset of the wave's exclusive scan -- the wave's pair list without
// atomics; a wave with more than kPairsPerWave pairs sends the env to the
// global path.
__global__ __launch_bounds__(256) void k_mwb_pairs(DevState st, Scratch sc) {
  const int e = blockIdx.y, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int32_t* bm = sc.bmisc + (size_t)e * kBmWords;
  if (bm[kBmMisc + 0]) return;
  const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (w >= bm[kBmMisc + 1]) return;
  const int i = sc.perm[(size_t)e * sc.S + w * 64 + lane];
  const int n_i = i >= 0 ? (int)((uint32_t)sc.lroot[base + i] >> 16) : 0;
  const int off = i >= 0 ? sc.gclus[3 * M + base + i] : 0;
  int v = n_i;
  v = wave_incl_scan(v);
  const int total = __builtin_amdgcn_readlane(v, 63);
  const size_t wi = (size_t)e * sc.wmax + w;
  if (lane == 0) sc.wave_npairs[wi] = min(total, kPairsPerWave);
  if (total > kPairsPerWave) {
    if (lane == 0) sc.fallback[e] = 1;  // a wave with more than kPairsPerWave pairs
    return;
  }
  const uint32_t* plist = sc.gplist + (size_t)e * sc.pair_cap;
  uint32_t* out = sc.pairs + wi * kPairsPerWave + (v - n_i);
  for (int k = 0; k < n_i; ++k) {
    const int j = (int)(plist[off + k] >> 16);
    const int sj = sc.slot_of[base + j];
    const uint32_t spp =
        sc.multi_species ? (uint32_t)(st.species[i] * kMaxSpecies + st.species[j]) : 0u;
    out[k] = (uint32_t)lane | ((uint32_t)(sj & 63) << 6) | (spp << 12);
  }
}

template <bool kBig, bool kLocal>
__global__ __launch_bounds__(1024) void k_cluster_build(DevState st, Scratch sc) {
  extern __shared__ __align__(16) unsigned char smem[];
  cluster_build_env<kBig, !kBig, kLocal>(st, sc, blockIdx.x, smem, sc.gnpairs[blockIdx.x]);
}

// Words of k_build_env's sort/search region (wave sums, cell ends, sorted
// x, y, id), which must fit below the pair list of the build's LDS layout.
__host__ __device__ inline size_t build_env_sort_words(int n, int ncell) {
  return 16 + (size_t)((ncell + 2) & ~1) + 3 * (size_t)n;
}

// The whole build of one env in one workgroup, LDS-resident (no global
// intermediates, one launch): counting sort of the positions into cells of
// side >= rc_max + skin, the pair search over the sorted LDS copy (every pair
// within r_i + r_j + skin once, straight into the LDS pair list), then
// union-find and packing (cluster_build_env).  Same pair set as
// k_build_sort -> k_build_pairs -> k_cluster_build, in one launch and without
// their global round trips.
__global__ __launch_bounds__(1024) void k_build_env(const Derived* __restrict__ d, DevState st,
                                                    Scratch sc, int lx, int ly) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ float nb2[kMaxSpecies * kMaxSpecies];
  __shared__ int32_t npair;
  constexpr int CH = 4;   // particles per thread kept in registers across the scan
  constexpr int kKeep = 8;
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  const int ncx = 1 << lx, ncy = 1 << ly;
  int32_t* ws = reinterpret_cast<int32_t*>(smem);
  int32_t* cnt = ws + 16;  // counts, then exclusive starts, then cell ends
  // sorted positions as (x, y) pairs (one 8-byte LDS read per candidate),
  // then the ids; cnt padded to 8-byte alignment
  uint2* lq = reinterpret_cast<uint2*>(cnt + ((ncell + 2) & ~1));
  int32_t* lid = reinterpret_cast<int32_t*>(lq + N);
  const int wmax = sc.wmax;
  uint32_t* plist = reinterpret_cast<uint32_t*>(smem) +
                    (16 + 16 + 3 * 68 + ((wmax + 3) & ~3) + 4 * (size_t)N);
  SWARM_STAMP(0);
  uint32_t cqx[CH], cqy[CH];
  int32_t cid[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int i = tid + k * T;
    const bool ok = i < N;
    cqx[k] = ok ? st.q[base + i] : 0u;
    cqy[k] = ok ? st.q[M + base + i] : 0u;
    cid[k] = ok ? (i | ((int32_t)st.species[i] << 24)) : -1;
  }
  for (int k = tid; k < kMaxSpecies * kMaxSpecies; k += T) nb2[k] = d->nb2[k];
  for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
  if (tid == 0) npair = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CH; ++k)
    if (cid[k] >= 0) atomicAdd(&cnt[cell_index(cqx[k], cqy[k], lx, ly)], 1);
  for (int i = tid + CH * T; i < N; i += T)
    atomicAdd(&cnt[cell_index(st.q[base + i], st.q[M + base + i], lx, ly)], 1);
  __syncthreads();
  block_exclusive_scan(cnt, ncell, ws);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    if (cid[k] < 0) continue;
    const int pos = atomicAdd(&cnt[cell_index(cqx[k], cqy[k], lx, ly)], 1);
    lq[pos] = make_uint2(cqx[k], cqy[k]);
    lid[pos] = cid[k];
  }
  for (int i = tid + CH * T; i < N; i += T) {
    const uint32_t qx = st.q[base + i], qy = st.q[M + base + i];
    const int pos = atomicAdd(&cnt[cell_index(qx, qy, lx, ly)], 1);
    lq[pos] = make_uint2(qx, qy);
    lid[pos] = i | ((int32_t)st.species[i] << 24);
  }
  // idle wave slots of the next run (the packing writes the used ones)
  for (int k = tid; k < sc.S; k += T) sc.perm[(size_t)e * sc.S + k] = -1;
  __syncthreads();  // cnt[c] = end of cell c = start of cell c + 1
  // the window-start cell-sorted snapshot in global memory too, for
  // k_check's cell-based exact test (without it the check tested every mover
  // against every colloid: 23.6 us per launch at E = 64)
  for (int t = tid; t < N; t += T) {
    const uint2 v = lq[t];
    sc.bsq[base + t] = v.x;
    sc.bsq[M + base + t] = v.y;
    sc.bsid[base + t] = lid[t];
  }
  {
    int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
    for (int c = tid; c <= ncell; c += T) cs[c] = c == 0 ? 0 : cnt[c - 1];
  }
  SWARM_STAMP(1);
  // pair search: a stencil row (cells x-1..x+1) is one contiguous sorted
  // range, plus a wrap range at the grid edge
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const int lane = tid & 63;
  for (int ps0 = 0; ps0 < N; ps0 += T) {  // uniform trip count: whole waves
    const int ps = ps0 + tid;
    const bool valid = ps < N;
    int pk = 0, i = 0;
    uint32_t qx = 0, qy = 0;
    if (valid) {
      pk = lid[ps];
      i = pk & 0xffffff;
      const uint2 q = lq[ps];
      qx = q.x;
      qy = q.y;
    }
    const int c0 = cell_index(qx, qy, lx, ly);
    const int cx = c0 & (ncx - 1), cy = c0 >> lx;
    const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
    const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
    const int xw = ncx >= 3 ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
    int rb[6], re[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int oy = loy + (r >> 1), part = r & 1;
      const bool use = valid && oy <= hiy && (part == 0 || xw >= 0);
      const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
      const int c_lo = row | (part == 0 ? xa : xw), c_hi = row | (part == 0 ? xb : xw);
      rb[r] = use ? (c_lo > 0 ? cnt[c_lo - 1] : 0) : 0;
      re[r] = use ? cnt[c_hi] : 0;
    }
    const float* nb2_row = nb2 + (pk >> 24) * kMaxSpecies;
    int found = 0;
    uint32_t keep[kKeep];
#pragma unroll
    for (int v = 0; v < kKeep; ++v) keep[v] = 0u;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      for (int jj0 = rb[r]; jj0 < re[r]; jj0 += 4) {  // four candidates' loads in flight
        int pk4[4];
        uint32_t x4[4], y4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int jj = min(jj0 + u, N - 1);
          pk4[u] = jj0 + u < re[r] ? lid[jj] : -1;
          const uint2 q = lq[jj];
          x4[u] = q.x;
          y4[u] = q.y;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (pk4[u] < 0) continue;
          const int j = pk4[u] & 0xffffff;
          const float rx = (float)(int32_t)(x4[u] - qx) * sx0;
          const float ry = (float)(int32_t)(y4[u] - qy) * sx1;
          if (i < j && rx * rx + ry * ry < nb2_row[pk4[u] >> 24]) {
#pragma unroll
            for (int v = 0; v < kKeep; ++v) keep[v] = found == v ? (uint32_t)j : keep[v];
            ++found;
          }
        }
      }
    }
    // wave prefix sum, one LDS atomic per wave
    int v = found;
    v = wave_incl_scan(v);
    int wbase = 0;
    if (lane == 63) wbase = atomicAdd(&npair, v);
    wbase = __builtin_amdgcn_readlane(wbase, 63);
    const int my_off = wbase + v - found;
    if (!__any(found > kKeep)) {
#pragma unroll
      for (int u = 0; u < kKeep; ++u) {
        const int k = my_off + u;
        if (u < found && k < sc.pair_cap) plist[k] = (uint32_t)i | (keep[u] << 16);
      }
    } else {  // a lane found more than kKeep pairs: rescan and write in order
      int w = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        for (int jj = rb[r]; jj < re[r]; ++jj) {
          const int pkj = lid[jj];
          const int j = pkj & 0xffffff;
          const uint2 q = lq[jj];
          const float rx = (float)(int32_t)(q.x - qx) * sx0;
          const float ry = (float)(int32_t)(q.y - qy) * sx1;
          if (i < j && rx * rx + ry * ry < nb2_row[pkj >> 24]) {
            const int k = my_off + w;
            if (k < sc.pair_cap) plist[k] = (uint32_t)i | ((uint32_t)j << 16);
            ++w;
          }
        }
      }
    }
  }
  __syncthreads();
  SWARM_STAMP(2);
  const int found = npair;
  __syncthreads();  // the sort region is reused by the union-find arrays
  cluster_build_env<false, false>(st, sc, e, smem, found);
}

// -------------------------------------------------------- cluster run
// Orders one wave's LDS accesses (DS operations of a wave execute in order;
// this keeps the compiler from moving them across).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Noise table for latency-bound windows (few waves per SIMD): the normals of
// every (sub-step, particle) computed ahead of the run.  Indexed by particle,
// not wave slot, so it does not wait for the cluster build.
// Particle-major: particle gi's sub-steps
// are one contiguous run of 12-B records, table[(gi * kMaxWindow + s) * 3 +
// c], so a lane reads its sub-step's three normals with one 12-B load and a
// 128-B line (~10 sub-steps of one particle) is fetched by the one XCD that
// runs the particle.  The step-major layout, table[(s * 3 + c) * M + gi],
// shares each line among 32 particles spread over every XCD, so each XCD's
// L2 fetched its own copy (rocprof FETCH ~ 7-8 x the table).
// Two tables, by window parity: the wide run kernel fills the next window's
// on otherwise idle CUs while it reads this one's.  The control block
// records each table's first step and length; a run whose window does not
// match its table draws the normals itself.
__host__ __device__ inline size_t noise_table_words(size_t M) { return (size_t)kMaxWindow * 3 * M; }
// word of normal c of sub-step s of particle gi; the step and component strides
__host__ __device__ inline size_t noise_index(size_t M, size_t gi, int s, int c) {
  (void)M;
  return (gi * kMaxWindow + (size_t)s) * 3 + (size_t)c;
}
__host__ __device__ inline size_t noise_step_stride(size_t) { return 3; }
__host__ __device__ inline size_t noise_comp_stride(size_t) { return 1; }

// Item (k, b) of a table starting at step_start: Philox block b (0..2) of
// group g = g0 + k (g0 = step_start / 4), i.e. normals n[4b..4b+3] of
// sub-steps t = 4 g .. 4 g + 3 (StepNoise's numbers), stored where they
// fall in particle gi's records: element u of the block is word
// f + u = 12 k + 4 b - 3 (step_start mod 4) + u of the particle's run of
// 12-B records, kept when it lies within [0, 3 len).  One block per lane and
// consecutive items at consecutive 16-B words: with an aligned start a wave's
// stores are one float4 per lane over 1 KiB of whole lines (three scalar
// stores per normal at a 48-B lane stride left lines partially written, and
// WRITE_SIZE at 2-3.5x the table).
__device__ __forceinline__ void noise_block(const Derived* __restrict__ d, const DevState& st,
                                            uint64_t step_start, int len,
                                            float* __restrict__ table, long gi, int k, int b) {
  const int e = (int)(gi / st.n);
  const int i = (int)(gi - (long)e * st.n);
  float n[4];
  group_block(d->key0, d->key1 ^ (uint32_t)e, (uint32_t)i, (step_start >> 2) + (uint64_t)k,
              (uint32_t)b, n);
  const int f = 12 * k + 4 * b - 3 * (int)(step_start & 3u);
  float* o = table + noise_index((size_t)st.m, (size_t)gi, 0, 0);
  // streaming stores: the table is read by the next window's run only
  // (same-box A/B, E = 1: the launch ends ~1.1 us sooner, the next
  // window's gathers cost ~0.6 us; head line 51.8 -> 52.5 M)
  if ((f & 3) == 0 && f >= 0 && f + 4 <= 3 * len) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const f32x4 v = {n[0], n[1], n[2], n[3]};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(o + f));
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (f + u >= 0 && f + u < 3 * len) __builtin_nontemporal_store(n[u], o + f + u);
  }
}

// Work item k of a table fill over M particles: noise_items(len) per
// particle, (group, block) in order, so consecutive lanes store consecutive
// 16-B words of one particle's records.
__host__ __device__ inline int noise_groups(int len) { return len / 4 + 2; }  // any alignment
__host__ __device__ inline int noise_items(int len) { return 3 * noise_groups(len); }
__device__ __forceinline__ void noise_item(long k, int per, long* gi, int* grp, int* blk) {
  *gi = k / per;
  const int r = (int)(k - *gi * per);
  *grp = r / 3;
  *blk = r - 3 * *grp;
}

// This window's table of len sub-steps (grid.y = noise_groups(len)) from the
// current step counter.
__global__ __launch_bounds__(256) void k_noise(const Derived* __restrict__ d, DevState st,
                                               uint64_t* __restrict__ ctl,
                                               float* __restrict__ tables, int len) {
  const long M = st.m;
  const int par = window_parity(ctl);
  const uint64_t step0 = ctl[kCtlStep];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl[kCtlTStep + par] = step0;
    ctl[kCtlTLen + par] = (uint64_t)len;
  }
  const int per = noise_items(len);
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= M * per) return;
  long gi;
  int grp, blk;
  noise_item(k, per, &gi, &grp, &blk);
  noise_block(d, st, step0, len, tables + par * noise_table_words(M), gi, grp, blk);
}

// Rotation helper (round 6, latency-bound runs).  A particle's orientation
// never depends on positions or forces: sub-step s turns it by
// f2i32_sat((tz tau + sig_r g2_s) 2^32 / 2 pi), so the whole window's directors
// can be computed apart from the force chain.  In k_cluster_run_wide a
// second wave of the block (another SIMD of the CU: waves are dealt to the
// SIMDs in turn) runs the rotation of a run wave's 64 slots and writes each
// sub-step's director (sin, cos) to LDS ahead of it; the run wave reads them
// in its force round trip's latency window instead of issuing the ~35
// rotation and sin/cos instructions itself (a lone wave's sub-step is
// bounded by its own issue and dependency chain).  Same operation sequence
// as the run wave's own rotation, so the same bits.  The run wave never
// waits: a director the helper has not published yet is computed from the
// window start (helper_director_at), so no wave depends on another's
// progress.
constexpr int32_t kHelpDone = 0x40000000;
struct HelperLds {
  float2* dir;       // [kMaxWindow][64] director of sub-step s (s >= 1)
  uint32_t* an_end;  // [64] orientation after the window
  int32_t* prog;     // directors [0, prog) published; kHelpDone: an_end too
};
__host__ __device__ constexpr size_t helper_lds_bytes() {
  return (size_t)kMaxWindow * 64 * 8 + 64 * 4 + 64;
}
__device__ __forceinline__ HelperLds helper_lds(unsigned char* base, int slot) {
  unsigned char* b = base + (size_t)slot * helper_lds_bytes();
  HelperLds h;
  h.dir = reinterpret_cast<float2*>(b);
  h.an_end = reinterpret_cast<uint32_t*>(b + (size_t)kMaxWindow * 64 * 8);
  h.prog = reinterpret_cast<int32_t*>(b + (size_t)kMaxWindow * 64 * 8 + 256);
  return h;
}

// the orientation increment of sub-step s (bd_step's rotation sequence)
__device__ __forceinline__ uint32_t rot_increment(const PConst& pc, float tzs, float g2) {
  float dth = tzs * pc.rot_dt;
  dth = dth + pc.sigr * g2;  // (+0 without noise: the same increment)
  return (uint32_t)f2i32_sat(dth * kAngInvScale);
}

// The helper wave of run wave gw: publishes the directors of sub-steps
// 1 .. n_steps - 1 and the final orientation.  Table normals only (the
// latency-bound path); g2 loaded eight sub-steps ahead.
template <bool kMulti>
__device__ __forceinline__ void rot_helper(const Derived* __restrict__ d, const DevState& st,
                                           const Scratch& sc, int n_envs, int n_steps,
                                           const float* __restrict__ table, int gw, int lane,
                                           const HelperLds& h, int par) {
  const int e = gw / sc.wmax;
  const int w = gw - e * sc.wmax;
  if (e >= n_envs) return;
  if (sc.fallback[e] != 0 || w >= sc.env_waves[e]) return;
  const int N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int i = sc.perm[(size_t)e * sc.S + w * 64 + lane];
  const bool active = i >= 0;
  const size_t gi = base + (active ? i : 0);
  uint32_t an = 0u;
  float tz0 = 0.0f, tzc = 0.0f;
  int si = 0;
  if (active) {
    an = st.ang[gi];
    si = st.species[i];
    const PrevSlot prv = prev_slot(st, par);
    tzc = st.torque_z[gi];
    tz0 = st.reuse ? prv.tz[gi] : tzc;
  }
  const PConst pc = load_pconst(d, kMulti ? si : 0);
  const float* tg = table + noise_index(M, gi, 0, 2);  // g2 of sub-step 0; stride 3
  float gb[8], gx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) gb[k] = k < n_steps ? tg[3 * k] : 0.0f;
  for (int s0 = 0; s0 < n_steps; s0 += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) gx[k] = s0 + 8 + k < n_steps ? tg[3 * (s0 + 8 + k)] : 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int s = s0 + k;
      if (s < n_steps) {
        an = an + rot_increment(pc, s == 0 ? tz0 : tzc, gb[k]);
        if (s + 1 < n_steps) {
          float sn, cs;
          sincos_turn(an, &sn, &cs);
          h.dir[(size_t)(s + 1) * 64 + lane] = make_float2(sn, cs);
          // publish (a wave's LDS writes complete in order: a reader that
          // sees the count sees the directors)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0)
            __hip_atomic_store(h.prog, s + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) gb[k] = gx[k];
  }
  h.an_end[lane] = an;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_store(h.prog, kHelpDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// One wave of the cluster run: all n_steps sub-steps of the particles in
// its 64 slots.  kTable: the normals come from this window's noise table
// (prefetched one sub-step ahead), else they are drawn here.
// kMulti = false: one species, so the pair constants are wave-uniform scalars.
// kTwoPass: waves with 65-128 pairs get their own unrolled two-pass variant
// (else the general up-to-four-pass loop).
// *p -= v on LDS words, no return (ds_sub_u64).  Ordering: a wave's LDS
// instructions execute in issue order (one instruction for all 64 lanes), so
// the force sums' read-back issued after it sees it; the memory clobber keeps
// the compiler from moving LDS accesses across it.
// px[0] -= vx and px[64] -= vy: the x and y force sums of one slot (the
// run kernels' lacc[wave][2][64] rows, y 512 bytes after x).
__device__ __forceinline__ void lds_sub_u64_xy(unsigned long long* px, unsigned long long vx,
                                               unsigned long long vy) {
  const uint32_t addr = (uint32_t)(uintptr_t)px;  // the LDS offset (low word of the flat address)
  __asm__ volatile("ds_sub_u64 %0, %1\n\tds_sub_u64 %0, %2 offset:512"
                   :
                   : "v"(addr), "v"(vx), "v"(vy)
                   : "memory");
}

template <bool kMulti, bool kTable, bool kWalls, bool kTwoPass = false, bool kHelper = false>
__device__ __forceinline__ void run_wave(const Derived* __restrict__ d, const DevState& st,
                                         const Scratch& sc, int n_envs, int n_steps,
                                         uint64_t step0, const float* __restrict__ table,
                                         int gw, int lane,
                                         unsigned long long* lacc_x, unsigned long long* lacc_y,
                                         const PairTables& pt, int par,
                                         HelperLds hl = HelperLds{},
                                         const float2* ntab = ntab_global()) {
  // the sub-step schedule for latency-bound waves (the wide kernel, which
  // also takes the two-pass variant); the throughput kernel, bound by VALU
  // issue over many waves, keeps the plain one (fewer registers, no spill)
  constexpr int kSched = kTwoPass ? SWARM_RUN_SCHED : 0;
  const int e = gw / sc.wmax;
  const int w = gw - e * sc.wmax;
  if (e >= n_envs) return;
  if (sc.fallback[e] != 0 || w >= sc.env_waves[e]) return;
#ifdef SWARM_PHASE_TIMING
  const uint64_t t_wave0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int slot = w * 64 + lane;
  const int i = sc.perm[(size_t)e * sc.S + slot];
  const bool active = i >= 0;
  PState p = {0u, 0u, 0u, 0, 0};
  int si = 0;
  // fs, tz: this sub-step's swim force and torque -- for sub-step 0 with
  // reuse_forces the previous run's (the current ones are loaded after it)
  float fs = 0.0f, tz = 0.0f, fex = 0.0f, fey = 0.0f;
  uint32_t an0 = 0u;  // orientation of sub-step 0's swim force
  const size_t gi = base + (active ? i : 0);
  if (active) {
    p.qx = st.q[gi];
    p.qy = st.q[M + gi];
    p.ix = st.img[gi];
    p.iy = st.img[M + gi];
    p.an = st.ang[gi];
    si = st.species[i];
    const PrevSlot prv = prev_slot(st, par);  // reuse_forces: this window's slot
    fs = st.reuse ? prv.f[gi] : st.f_swim[gi];
    tz = st.reuse ? prv.tz[gi] : st.torque_z[gi];
    an0 = st.reuse ? prv.ang[gi] : p.an;
    fex = st.f_ext[gi];
    fey = st.f_ext[M + gi];
    // window-start snapshot for k_check's exact test and re-run (taken here,
    // not by the build, so a build may run ahead of the slice's actions)
    sc.bq[gi] = p.qx;
    sc.bq[M + gi] = p.qy;
    sc.bimg[gi] = p.ix;
    sc.bimg[M + gi] = p.iy;
    sc.bang[gi] = p.an;
  }
  // this wave's neighbour pairs: one per lane and pass (wave-uniform count)
  const int np = sc.wave_npairs[(size_t)e * sc.wmax + w];
  const int npass = (np + 63) >> 6;
  const uint32_t* pw = sc.pairs + ((size_t)e * sc.wmax + w) * kPairsPerWave;
  // the first pass's pair stays in a register; a wave with more passes
  // (rare: a cluster denser than 2 pairs per particle) reloads the others
  // from L2 each sub-step, so they do not hold registers for the run
  const uint32_t pr0 = lane < np ? pw[lane] : 0xffffffffu;
  // two passes (a cluster with more than 64 pairs: 65-128 in the wave): the
  // second pass's pair in a register too, and both passes unrolled so their
  // LDS reads and force arithmetic interleave (C5: such a wave set the
  // launch's duration in a third of the windows, 1.7x a one-pass wave)
  const uint32_t pr1 = npass == 2 && 64 + lane < np ? pw[64 + lane] : 0xffffffffu;
  lacc_x[lane] = 0ull;
  lacc_y[lane] = 0ull;
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float eps24 = d->eps24;
  // one species: its constants are wave-uniform (scalar registers)
  const PConst pc = load_pconst(d, kMulti ? si : 0);
  // helper mode: the window-start orientation and torques, for a director
  // the helper has not published yet (helper_director_at)
  const uint32_t an_start = p.an;
  const float tz0 = tz, tzc = (kHelper && active) ? st.torque_z[gi] : 0.0f;
  Carry carry = {0u, 0u, 0, 0};  // the previous sub-step's image carries, pending
  const float cut2_0 = d->cut2[0], sig6_0 = d->sig6[0];
  const uint32_t q0x = p.qx, q0y = p.qy;
  float dmax2 = 0.0f;
  float vx = 0.0f, vy = 0.0f, om = 0.0f;
  const size_t tstep = noise_step_stride(M), ts = noise_comp_stride(M);
  const float* tcol = kTable ? table + noise_index(M, gi, 0, 0) : nullptr;
  float gn[3] = {0.0f, 0.0f, 0.0f};
  StepNoise noise;  // !kTable: the window's normals drawn here, group by group
  noise.tab = ntab;
  if (kTable) {  // idle lanes read particle 0's (never stored)
    gn[0] = tcol[0];
    gn[1] = tcol[ts];
    gn[2] = tcol[2 * ts];
  }
#ifdef SWARM_PHASE_TIMING
  const bool stamp = e == 0 && w == sc.env_waves[e] - 1 && lane == 0;
  uint64_t t_pairs = 0, t_read = 0, t_bd = 0, t0s = 0, t1s = 0;
#endif
  // The rotation and the director do not depend on the forces: each
  // sub-step turns the angle and computes the next sub-step's director while
  // its force sums are in flight in LDS (software-pipelined director).
  // A lone wave pays for every taken branch, so the sub-step is branch-lean:
  // the pass count (0, 1 or up to 4) and the last sub-step (velocities) are
  // compile-time variants, and idle lanes compute along (never stored).
  // the orientation after j sub-steps, from the window start (helper mode:
  // what the helper has not published yet)
  auto helper_angle_at = [&](int j) __attribute__((always_inline)) {
    uint32_t a = an_start;
    for (int k = 0; k < j; ++k) a = a + rot_increment(pc, k == 0 ? tz0 : tzc, tcol[3 * k + 2]);
    return a;
  };
  float dir[2];
  sincos_turn(an0, &dir[0], &dir[1]);
  auto substep = [&](const int s, auto last_t, auto pass_t) __attribute__((always_inline)) {
    constexpr bool kLast = decltype(last_t)::value;
    constexpr int kPass = decltype(pass_t)::value;  // 0, 1, 2 or 4: up to npass
#ifdef SWARM_PHASE_TIMING
    if (stamp) t0s = t1s = __builtin_amdgcn_s_memtime();
#endif
    float gt[3] = {gn[0], gn[1], gn[2]};
    if (kTable && !kLast) {  // the next sub-step's normals, one sub-step ahead
      const float* nx = tcol + (size_t)(s + 1) * tstep;
      gn[0] = nx[0];
      gn[1] = nx[ts];
      gn[2] = nx[2 * ts];
    }
    if (!kTable && pc.noisy) noise.next(k0, k1, (uint32_t)i, step0 + (uint64_t)s, s == 0, gt);
    int64_t ax = 0, ay = 0;
    float dnext[2] = {dir[0], dir[1]};
    uint32_t an_next;
    // rotation (bd_step's sequence): off the force chain
    auto rotate = [&]() __attribute__((always_inline)) {
      if (kHelper) {
        an_next = p.an;  // the helper wave turns the directors
        return;
      }
      // (without noise gt is zero and sigr 0: dth + 0 is the same increment,
      // and no select)
      float dth = tz * pc.rot_dt;
      dth = dth + pc.sigr * gt[2];
      an_next = p.an + (uint32_t)f2i32_sat(dth * kAngInvScale);
    };
    // the previous sub-step's displacement (max is order-free)
    auto prev_disp = [&]() __attribute__((always_inline)) {
      if (kSched && s > 0) {
        const float ddx = (float)(int32_t)(p.qx - q0x) * sx0;
        const float ddy = (float)(int32_t)(p.qy - q0y) * sx1;
        dmax2 = __uint_as_float(max(__float_as_uint(dmax2), __float_as_uint(ddx * ddx + ddy * ddy)));
      }
    };
    // the next sub-step's director, pinned where it is computed: without a
    // use there the compiler sinks it past the read-back's vote branch into
    // the next sub-step's translation, onto the force chain
    int hprog = 0;  // helper mode: the published count read with the director
    auto director = [&]() __attribute__((always_inline)) {
      if constexpr (kHelper) {
        if (!kLast) {  // the count first, then the director (LDS order)
          hprog = __hip_atomic_load(hl.prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const float2 dv = hl.dir[(size_t)(s + 1) * 64 + lane];
          dnext[0] = dv.x;
          dnext[1] = dv.y;
        }
        return;
      }
      if (!kLast) sincos_turn(an_next, &dnext[0], &dnext[1]);
      if (kSched) __asm__ volatile("" : "+v"(dnext[0]), "+v"(dnext[1]));
    };
    if (kPass == 0 || kSched < 2) {
      if (kSched) prev_disp();
    }
    // one-pass waves convert speculatively (see below); sa, sb, sv_*: the
    // lane's pair for the rare fix-up
    constexpr bool kSpec = kSched >= 3 && (kPass == 1 || kPass == 2);
    // speculative read-back conversion, image carries deferred (any pass count)
    constexpr bool kDefer = kSched >= 3 && kPass > 0 && !kWalls;
    float sv_x[2] = {0.0f, 0.0f}, sv_y[2] = {0.0f, 0.0f};
    int sa[2] = {lane, lane}, sb[2] = {lane, lane};
    bool spec_ok = true;
    if (kPass > 0) {
      for (int q = 0; q < (kPass == 1 ? 1 : (kPass == 2 ? 2 : npass)); ++q) {
        {  // wave-uniform; an empty slot names the lane twice
          const uint32_t e_ = q == 0 ? pr0
                                     : (kPass == 2 ? pr1
                                                   : (q * 64 + lane < np ? pw[q * 64 + lane]
                                                                         : 0xffffffffu));
          const int a = e_ == 0xffffffffu ? lane : (int)(e_ & 63u);
          const int b = e_ == 0xffffffffu ? lane : (int)((e_ >> 6) & 63u);
          // both ends' positions straight from their lanes' registers
          // (ds_bpermute: no LDS row written and waited for first; same-box
          // A/B: E = 1 run 50.9 -> 50.3 us, E = 64 247.7 -> 244.5 us)
          const uint2 pa = make_uint2((uint32_t)__builtin_amdgcn_ds_bpermute(a << 2, (int)p.qx),
                                      (uint32_t)__builtin_amdgcn_ds_bpermute(a << 2, (int)p.qy));
          const uint2 pb = make_uint2((uint32_t)__builtin_amdgcn_ds_bpermute(b << 2, (int)p.qx),
                                      (uint32_t)__builtin_amdgcn_ds_bpermute(b << 2, (int)p.qy));
          if (kSched >= 2 && q == 0) {
            // the exchange's latency window: rotation and displacement
            __builtin_amdgcn_sched_barrier(0);
            rotate();
            if (!kHelper || !SWARM_HELPER_WIN2) {  // (helper: the round trip's window)
              prev_disp();
              if (kDefer) apply_carry(p, carry);
            }
            // pinned here (the compiler would sink them behind the vote branch)
            __asm__ volatile("" : "+v"(an_next), "+v"(dmax2), "+v"(p.ix), "+v"(p.iy));
            __builtin_amdgcn_sched_barrier(0);
          }
          const float rx = (float)(int32_t)(pb.x - pa.x) * sx0;
          const float ry = (float)(int32_t)(pb.y - pa.y) * sx1;
          int64_t fx, fy;  // on a; b receives exactly the negation
          if (kSpec) {
            // speculative int32 conversion: the atomics do not wait for the
            // wave vote; a wave whose vote fails adds the exact remainder
            // after them (spec_fix below), so the sums are the same integers
            const int qq = q & 1;  // (kSpec: q < 2, unrolled)
            if (kMulti) {
              const int sp = (int)((e_ >> 12) & 255u);
              pair_vals(pt.cut2[sp], pt.sig6[sp], eps24, rx, ry, sv_x[qq], sv_y[qq]);
            } else {
              pair_vals(cut2_0, sig6_0, eps24, rx, ry, sv_x[qq], sv_y[qq]);
            }
            spec_ok = spec_ok && wave_all2(fabsf(sv_x[qq]) < 2147483520.0f,
                                           fabsf(sv_y[qq]) < 2147483520.0f);
            fx = (int64_t)__float2int_rn(sv_x[qq]);
            fy = (int64_t)__float2int_rn(sv_y[qq]);
            sa[qq] = a;
            sb[qq] = b;
          } else if (kMulti) {
            const int sp = (int)((e_ >> 12) & 255u);
            pair_fix_sel(pt.cut2[sp], pt.sig6[sp], eps24, rx, ry, fx, fy);
          } else {
            pair_fix_sel(cut2_0, sig6_0, eps24, rx, ry, fx, fy);
          }
          atomicAdd(&lacc_x[a], (unsigned long long)fx);
          atomicAdd(&lacc_y[a], (unsigned long long)fy);
          // b: the exact negation.  The throughput kernel issues ds_sub_u64
          // itself (lds_sub_u64); atomicSub compiles to ds_add_u64 of the
          // negated value, a 64-bit negation (two VALU operations and a
          // hazard wait) per component and pass
          if (kSched == 0) {
            lds_sub_u64_xy(&lacc_x[b], (unsigned long long)fx, (unsigned long long)fy);
          } else {
            atomicSub(&lacc_x[b], (unsigned long long)fx);
            atomicSub(&lacc_y[b], (unsigned long long)fy);
          }
        }
      }
    }
    if (kSched >= 2 && kPass > 0) {
      // the read-back issued right behind the atomics (a wave's DS operations
      // execute in order), the director computed in its latency window
      wave_lds_sync();
      ax = (int64_t)lacc_x[lane];
      ay = (int64_t)lacc_y[lane];
      lacc_x[lane] = 0ull;
      lacc_y[lane] = 0ull;
      if (kSpec && __builtin_expect(!spec_ok, 0)) {
        // a pair force beyond 2^31 fixed-point units on some lane: the
        // exact int64 values' remainders over the speculative int32 ones go
        // through the (zeroed) sums once more
        auto wide = [](float v) __attribute__((always_inline)) {
          return __float2ll_rn(
              fminf(fmaxf(v, -4.611686018427387904e18f), 4.611686018427387904e18f));
        };
#pragma unroll
        for (int qq = 0; qq < kPass; ++qq) {
          const int64_t rx_ = wide(sv_x[qq]) - (int64_t)__float2int_rn(sv_x[qq]);
          const int64_t ry_ = wide(sv_y[qq]) - (int64_t)__float2int_rn(sv_y[qq]);
          atomicAdd(&lacc_x[sa[qq]], (unsigned long long)rx_);
          atomicAdd(&lacc_y[sa[qq]], (unsigned long long)ry_);
          atomicSub(&lacc_x[sb[qq]], (unsigned long long)rx_);
          atomicSub(&lacc_y[sb[qq]], (unsigned long long)ry_);
        }
        wave_lds_sync();
        ax += (int64_t)lacc_x[lane];
        ay += (int64_t)lacc_y[lane];
        lacc_x[lane] = 0ull;
        lacc_y[lane] = 0ull;
      }
      __builtin_amdgcn_sched_barrier(0);
      director();
      if (kHelper && SWARM_HELPER_WIN2) {
        // the round trip's latency window holds no rotation in helper mode:
        // the previous sub-step's displacement and image carries go here
        prev_disp();
        if (kDefer) apply_carry(p, carry);
        __asm__ volatile("" : "+v"(dmax2), "+v"(p.ix), "+v"(p.iy));
      }
      __builtin_amdgcn_sched_barrier(0);
    } else {
      // rotation (bd_step's sequence) and the next director, between the
      // force-sum atomics and their read-back
      __builtin_amdgcn_sched_barrier(0);
      rotate();
      director();
      __builtin_amdgcn_sched_barrier(0);
      __asm__ volatile("" ::: "memory");  // keep the read-back after the director
      if (kPass > 0) {
        wave_lds_sync();
#ifdef SWARM_PHASE_TIMING
        if (stamp) {
          t1s = __builtin_amdgcn_s_memtime();
          t_pairs += t1s - t0s;
        }
#endif
        ax = (int64_t)lacc_x[lane];
        ay = (int64_t)lacc_y[lane];
        lacc_x[lane] = 0ull;
        lacc_y[lane] = 0ull;
#ifdef SWARM_PHASE_TIMING
        if (stamp) {
          const uint64_t t2 = __builtin_amdgcn_s_memtime();
          t_read += t2 - t1s;
          t1s = t2;
        }
#endif
      }
    }
    if (kWalls && active) {  // contacts of real particles only
      int64_t az = 0;
      wall_forces<2>(d, si, (float)p.qx * sx0, (float)p.qy * sx1, 0.0f, ax, ay, az,
                     st.wall_viol);
    }
    if (kDefer) {
      // speculative read-back conversion: the translation runs from the
      // int32 view of the sums while the wave vote resolves; the rare wave
      // with a sum beyond int32 redoes it from the exact conversion
      // the image carries are applied in the next sub-step's exchange window
      // (the last sub-step applies its own)
      const PState p0 = p;
      const bool fits = wave_all2(fits_i32(ax), fits_i32(ay));
      bd_translate_f(pc, p, (float)(int32_t)ax, (float)(int32_t)ay, fs, tz, fex, fey, k0,
                           k1, (uint32_t)i, step0 + (uint64_t)s, kLast, &vx, &vy, &om, gt, dir[0],
                           dir[1], kLast ? nullptr : &carry);
      // computed before the vote's branch (else the compiler moves the
      // translation behind it, back onto the chain)
      __asm__ volatile("" : "+v"(p.qx), "+v"(p.qy));
      if (__builtin_expect(!fits, 0)) {
        p = p0;
        bd_translate_f(pc, p, i64_to_f32_wide(ax), i64_to_f32_wide(ay), fs, tz, fex, fey,
                             k0, k1, (uint32_t)i, step0 + (uint64_t)s, kLast, &vx, &vy, &om, gt,
                             dir[0], dir[1], kLast ? nullptr : &carry);
      }
    } else {
      // (the throughput kernel: the three-operation carry, advance_adc)
      bd_translate(pc, p, ax, ay, fs, tz, fex, fey, k0, k1, (uint32_t)i, step0 + (uint64_t)s,
                   kLast, &vx, &vy, &om, gt, dir[0], dir[1], kSched == 0);
    }
    if (!kSched || kLast) {  // (else the next sub-step's prev_disp)
      const float ddx = (float)(int32_t)(p.qx - q0x) * sx0;
      const float ddy = (float)(int32_t)(p.qy - q0y) * sx1;
      // non-negative floats order like their bit patterns: one v_max_u32
      // (fmaxf adds a canonicalising max)
      dmax2 = __uint_as_float(max(__float_as_uint(dmax2), __float_as_uint(ddx * ddx + ddy * ddy)));
    }
    p.an = an_next;
    if (kHelper && !kLast && __builtin_amdgcn_readfirstlane(hprog) <= s + 1) {
      // not published yet (the window's first sub-steps): from the start
      const uint32_t a = helper_angle_at(s + 1);
      sincos_turn(a, &dnext[0], &dnext[1]);
    }
    if (!kLast) {
      dir[0] = dnext[0];
      dir[1] = dnext[1];
    }
#ifdef SWARM_PHASE_TIMING
    if (stamp) t_bd += __builtin_amdgcn_s_memtime() - t1s;
#endif
  };
  auto run_steps = [&](auto pass_t) __attribute__((always_inline)) {
    int s = 0;
    if (n_steps > 1) {
      // sub-step 0 peeled: with reuse_forces it swims with the previous run's
      // actions, and the current ones are loaded once after it (no register
      // holds them across the loop)
      substep(0, std::false_type{}, pass_t);
      if (st.reuse && active) {
        fs = st.f_swim[gi];
        tz = st.torque_z[gi];
      }
      if constexpr (kTable) {
        // two sub-steps per iteration: the next normals load into alternating
        // registers (no copies) and the scheduler sees across the boundary
        // (E=1 run 53.9 -> 53.4 us).  Not in the in-kernel-noise variant: at
        // its 96-VGPR bound the unrolled loop spills 80 B/lane, not 24.
        for (s = 1; s + 1 < n_steps - 1; s += 2) {
          substep(s, std::false_type{}, pass_t);
          substep(s + 1, std::false_type{}, pass_t);
        }
        if (s < n_steps - 1) substep(s++, std::false_type{}, pass_t);
      } else {
        for (s = 1; s < n_steps - 1; ++s) substep(s, std::false_type{}, pass_t);
      }
    }
    substep(s, std::true_type{}, pass_t);  // velocities of the last sub-step
  };
  if (npass == 0)
    run_steps(std::integral_constant<int, 0>{});
  else if (npass == 1)
    run_steps(std::integral_constant<int, 1>{});
  else if (kTwoPass && npass == 2)
    run_steps(std::integral_constant<int, 2>{});
  else
    run_steps(std::integral_constant<int, 4>{});
  if constexpr (kHelper) {  // the window's final orientation
    const int pg = __hip_atomic_load(hl.prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t ae = hl.an_end[lane];
    p.an = __builtin_amdgcn_readfirstlane(pg) == kHelpDone ? ae : helper_angle_at(n_steps);
  }
#ifdef SWARM_PHASE_TIMING
  if (stamp) {
    sc.phase[16] = t_pairs;
    sc.phase[17] = t_read;
    sc.phase[18] = t_bd;
    sc.phase[19] = (uint64_t)n_steps;
    sc.phase[20] = (uint64_t)npass;
  }
  if (lane == 0) {  // per-wave realtime stamps (100 MHz): entry, end, passes, pairs
    // (passes | XCC_ID << 16 | HW_ID << 32: which XCD, CU and SIMD ran the wave)
    uint64_t* ws = sc.phase + 32 + 4 * (size_t)gw;
    const uint32_t hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc_id = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    ws[0] = t_wave0;
    ws[1] = __builtin_amdgcn_s_memrealtime();
    ws[2] = (uint64_t)npass | ((uint64_t)(xcc_id & 0xffu) << 16) | ((uint64_t)hw_id << 32);
    ws[3] = (uint64_t)np;
  }
#endif
  if (active) {
    st.q[gi] = p.qx;
    st.q[M + gi] = p.qy;
    st.img[gi] = p.ix;
    st.img[M + gi] = p.iy;
    st.ang[gi] = p.an;
    st.vel[gi] = vx;
    st.vel[M + gi] = vy;
    st.vel[2 * M + gi] = 0.0f;
    st.omega[gi] = om;
    const float disp = sqrt_rn(dmax2);
    sc.disp[gi] = disp;
    if (!(disp < 0.5f * d->skin)) {  // a mover (k_check's exact test)
      const int k = atomicAdd(&sc.nmov[e], 1);
      if (k < kMaxMovers) sc.movers[(size_t)e * kMaxMovers + k] = i;
    }
    if (st.reuse) {  // the next window's sub-step 0 (the other slot)
      // (fs, tz hold this run's actions unless the window was one sub-step)
      const PrevSlot w = prev_slot(st, par ^ 1);
      w.f[gi] = n_steps > 1 ? fs : st.f_swim[gi];
      w.tz[gi] = n_steps > 1 ? tz : st.torque_z[gi];
      w.ang[gi] = p.an;
    }
  }
}

// Uniform dispatch to the compile-time variants: normals from a table
// (table != null) or drawn here; walls or none.
template <bool kMulti, bool kWalls, bool kTwoPass = false>
__device__ __forceinline__ void run_wave_dispatch(const Derived* __restrict__ d, const DevState& st,
                                                  const Scratch& sc, int n_envs, int n_steps,
                                                  uint64_t step0, const float* __restrict__ table,
                                                  int gw, int lane,
                                                  unsigned long long* lacc_x,
                                                  unsigned long long* lacc_y,
                                                  const PairTables& pt, int par,
                                                  bool help = false, HelperLds hl = HelperLds{},
                                                  const float2* ntab = ntab_global()) {
  if (table && help)
    run_wave<kMulti, true, kWalls, kTwoPass, true>(d, st, sc, n_envs, n_steps, step0, table, gw,
                                                   lane, lacc_x, lacc_y, pt, par, hl);
  else if (table)
    run_wave<kMulti, true, kWalls, kTwoPass>(d, st, sc, n_envs, n_steps, step0, table, gw, lane,
                                             lacc_x, lacc_y, pt, par, HelperLds{}, ntab);
  else
    run_wave<kMulti, false, kWalls, kTwoPass>(d, st, sc, n_envs, n_steps, step0, nullptr, gw, lane,
                                              lacc_x, lacc_y, pt, par, HelperLds{}, ntab);
}

// Launch-duration stamps for measurement (bench.py, swarm_engine_profile
// under graph capture): tstamp[0] = the earliest block start, tstamp[1] = the
// latest wave end, realtime clock (100 MHz); null otherwise (one uniform
// branch per block / wave).
__device__ __forceinline__ void stamp_start(unsigned long long* tstamp) {
  if (tstamp && threadIdx.x == 0)
    atomicMin(&tstamp[2 * (blockIdx.x & (kStampSub - 1))], (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void stamp_end(unsigned long long* tstamp) {
  if (tstamp && (threadIdx.x & 63) == 0)
    atomicMax(&tstamp[2 * (blockIdx.x & (kStampSub - 1)) + 1], (unsigned long long)wall_clock64());
}

// XCD-aware placement of per-env work (envs_per_xcd_map: blocks of one env):
// workgroup b is dispatched to XCD b mod 8 (MI355X_MICROARCH.md: for speed
// only, nothing depends on it), so the env's blocks are the b with
// b mod 8 == e mod 8.  All waves of an env then share one XCD's L2: the
// particle-indexed state lines an env's scattered lanes load and store are
// fetched and written back by one L2 instead of partial copies in eight.
// Returns false for a block beyond the last env.
__device__ __forceinline__ bool xcd_env_block(int b, int blocks_per_env, int n_envs, int* e,
                                              int* lb) {
  const int x = b & 7, k = b >> 3;
  *e = x + 8 * (k / blocks_per_env);
  *lb = k - (k / blocks_per_env) * blocks_per_env;
  return *e < n_envs;
}

// Throughput launch: 256-thread blocks, 4 waves each.  kWalls (host-chosen)
// keeps the wall-force variant's registers out of the wall-free kernel.
// xcd_bpe > 0: blocks placed by xcd_env_block with xcd_bpe blocks per env
// (ceil(wmax / 4)); else block b runs waves 4 b .. 4 b + 3 of the env-major
// wave list.
template <bool kMulti, bool kTable, bool kWalls>
__global__ __launch_bounds__(256, kRunMinBlocks) void k_cluster_run(const Derived* __restrict__ d, DevState st,
                                                     Scratch sc, int n_envs, int n_steps,
                                                     const uint64_t* __restrict__ ctl,
                                                     const float* __restrict__ tables,
                                                     int xcd_bpe,
                                                     unsigned long long* __restrict__ tstamp) {
  __shared__ PairTables pt;
  __shared__ unsigned long long lacc[4][2][64];  // int64 force sums (x, y)
  // the normal table in LDS (16.9 KB): the in-kernel normals' lookups are
  // scattered 8-byte reads, one per normal (ordered by stage_pair_tables'
  // barrier)
  __shared__ float2 ntab_lds[SWARM_NTAB_BINS];
  stamp_start(tstamp);
  for (int k = threadIdx.x; k < SWARM_NTAB_BINS; k += blockDim.x) ntab_lds[k] = ntab_global()[k];
  stage_pair_tables(d, &pt);
  const int par = window_parity(ctl);
  const uint64_t step0 = ctl[kCtlStep];
  const bool table_ok = kTable && ctl[kCtlTStep + par] == step0 &&
                        (uint64_t)n_steps <= ctl[kCtlTLen + par];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (xcd_bpe > 0) {
    int e, lb;
    if (!xcd_env_block((int)blockIdx.x, xcd_bpe, n_envs, &e, &lb)) return;
    const int w = lb * 4 + wv;
    if (w >= sc.wmax) return;
    gw = e * sc.wmax + w;
  }
  // a table that does not cover this window (the device check; the host
  // normally guarantees it) -> the normals are drawn in the kernel
  run_wave_dispatch<kMulti, kWalls>(d, st, sc, n_envs, n_steps, step0,
                                    table_ok ? tables + par * noise_table_words(st.m) : nullptr,
                                    gw, lane, lacc[wv][0], lacc[wv][1], pt, par, false,
                                    HelperLds{}, ntab_lds);
  stamp_end(tstamp);
}

// Latency-bound launch (few envs x particles: the run's waves fill few
// SIMDs): 1024-thread blocks whose dynamic LDS (set by the host) keeps one
// block per CU.  Blocks [0, nnb) fill the NEXT window's noise table
// (kMaxWindow sub-steps from this window's end) on CUs the run leaves idle,
// so no noise kernel sits between the policy and the run; the other blocks
// run with waves [0, run_wpb) only: one run wave per CU at E = 1 (its
// scattered noise-table gathers then have the CU's texture path to themselves),
// up to one per SIMD for more envs.
template <bool kMulti, bool kWalls>
__global__ __launch_bounds__(1024) void k_cluster_run_wide(const Derived* __restrict__ d,
                                                           DevState st, Scratch sc, int n_envs,
                                                           int n_steps, uint64_t* __restrict__ ctl,
                                                           float* __restrict__ tables,
                                                           int n_noise_blocks, int run_wpb,
                                                           int n_cand_blocks, int lxb, int lyb,
                                                           unsigned long long* __restrict__ tstamp,
                                                           int helpers) {
  __shared__ PairTables pt;
  __shared__ unsigned long long lacc[4][2][64];
  extern __shared__ __align__(16) unsigned char dyn_lds[];  // rotation helpers' tables
  stamp_start(tstamp);
  // helpers != 0 (host: run_wpb <= 2 and the dynamic LDS holds run_wpb
  // helper tables): the published counts start at zero before any wave of
  // the block reads them (ordered by stage_pair_tables' barrier)
  if (helpers && threadIdx.x < (unsigned)run_wpb)
    *helper_lds(dyn_lds, (int)threadIdx.x).prog = 0;
  stage_pair_tables(d, &pt);
  const int par = window_parity(ctl);
  const uint64_t step0 = ctl[kCtlStep];
  const size_t M = (size_t)st.m;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b < n_noise_blocks) {
    const uint64_t start = step0 + (uint64_t)n_steps;
    if (b == 0 && tid == 0) {
      ctl[kCtlTStep + (par ^ 1)] = start;
      ctl[kCtlTLen + (par ^ 1)] = (uint64_t)kMaxWindow;
    }
    float* t = tables + (par ^ 1) * noise_table_words(M);
    const int per = noise_items(kMaxWindow);
    const long total = (long)per * (long)M;
    for (long k = (long)b * blockDim.x + tid; k < total; k += (long)n_noise_blocks * blockDim.x) {
      long gi;
      int grp, blk;
      noise_item(k, per, &gi, &grp, &blk);
      noise_block(d, st, start, kMaxWindow, t, gi, grp, blk);
    }
    stamp_end(tstamp);
    return;
  }
  if (b < n_noise_blocks + n_cand_blocks) {  // the next window's candidate lists
    const int cb = b - n_noise_blocks, bpe = n_cand_blocks / n_envs;
    cand_build_body(d, st, sc, lxb, lyb, cb / bpe, (cb % bpe) * (int)blockDim.x + tid);
    stamp_end(tstamp);
    return;
  }
  const int lane = tid & 63, wv = tid >> 6;
  // wave-major over the envs (slot t: wave t / E of env t % E): every env's
  // low waves -- the ones that exist -- come in the first blocks, the slots
  // past an env's wave count (they exit at once) last, so no live wave waits
  // for a CU behind them (C4, 8 x 1024: start skew up to 19 us env-major)
  const int t0 = (b - n_noise_blocks - n_cand_blocks) * run_wpb;
  const bool table_ok = ctl[kCtlTStep + par] == step0 && (uint64_t)n_steps <= ctl[kCtlTLen + par];
  const float* table = table_ok ? tables + par * noise_table_words(M) : nullptr;
  // waves [run_wpb, 2 run_wpb): the rotation helpers of waves [0, run_wpb)
  // (on other SIMDs of the CU), with the table normals only
  const bool help = helpers && table != nullptr;
  const int slot = wv >= run_wpb ? wv - run_wpb : wv;
  if (wv >= (help ? 2 * run_wpb : run_wpb)) return;
  const int t = t0 + slot;
  if (t >= n_envs * sc.wmax) return;  // the last block's padding
  const int gw = (t % n_envs) * sc.wmax + t / n_envs;
  if (wv >= run_wpb) {
    rot_helper<kMulti>(d, st, sc, n_envs, n_steps, table, gw, lane, helper_lds(dyn_lds, slot), par);
    return;
  }
  const HelperLds hl = helper_lds(dyn_lds, slot);
  // latency-bound launches last as long as their slowest wave: one with
  // 65-128 pairs (a cluster denser than two pairs per particle) runs its own
  // unrolled two-pass sub-step instead of the general pass loop
  run_wave_dispatch<kMulti, kWalls, true>(d, st, sc, n_envs, n_steps, step0, table, gw, lane,
                                          lacc[wv][0], lacc[wv][1], pt, par, help, hl);
  stamp_end(tstamp);
}

// The env's big clusters (wider than a wave) for the window, by k_check's
// workgroup: one member per thread, the clusters' pairs spread over the
// threads; per sub-step the members publish their positions, every pair's
// force goes to both members' int64 sums (LDS atomics, as in the run
// kernel), then the members take the Brownian step (bd_step, normals drawn
// here: the same numbers as the noise table).  Writes the window-start
// snapshot, the final state, velocities and displacements like the run
// kernel, so k_check's exact test covers the members too.
// lds: 6 * kBigMax + 2 words (uint2 positions, two u64 force sums).
__device__ void run_big_clusters(const Derived* __restrict__ d, const DevState& st,
                                 const Scratch& sc, int e, int n_steps, uint64_t step0,
                                 int32_t* lds, const PairTables* pt, int par) {
  const int T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int nm = sc.big_n[e], np = min(sc.big_np[e], kBigPairs);
  uint2* lp = reinterpret_cast<uint2*>(lds + ((reinterpret_cast<uintptr_t>(lds) >> 2) & 1));
  unsigned long long* ax = reinterpret_cast<unsigned long long*>(lp + kBigMax);
  unsigned long long* ay = ax + kBigMax;
  const bool mem = tid < nm;
  const int i = mem ? sc.big_list[(size_t)e * kBigMax + tid] : 0;
  const size_t gi = base + i;
  PState p = {st.q[gi], st.q[M + gi], st.ang[gi], st.img[gi], st.img[M + gi]};
  const int si = st.species[i];
  const float fs = st.f_swim[gi], tz = st.torque_z[gi];
  // reuse_forces: sub-step 0 takes the previous run's actions and director
  const PrevSlot prv = prev_slot(st, par);
  const float fs0 = st.reuse ? prv.f[gi] : fs, tz0 = st.reuse ? prv.tz[gi] : tz;
  const uint32_t an0 = st.reuse ? prv.ang[gi] : p.an;
  const float fex = st.f_ext[gi], fey = st.f_ext[M + gi];
  const PConst pc = load_pconst(d, si);
  if (mem) {
    sc.bq[gi] = p.qx;
    sc.bq[M + gi] = p.qy;
    sc.bimg[gi] = p.ix;
    sc.bimg[M + gi] = p.iy;
    sc.bang[gi] = p.an;
  }
  const uint32_t q0x = p.qx, q0y = p.qy;
  constexpr int kPer = kBigPairs / 1024;  // pairs per thread (blockDim 1024)
  uint32_t pr[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int k = tid + u * T;
    pr[u] = k < np ? sc.big_pairs[(size_t)e * kBigPairs + k] : 0u;  // 0: member 0 twice
  }
  const uint32_t k0 = d->key0, k1 = d->key1 ^ (uint32_t)e;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const float eps24 = d->eps24;
  float dmax2 = 0.0f, vx = 0.0f, vy = 0.0f, om = 0.0f;
  StepNoise noise;
  if (mem) {
    ax[tid] = 0ull;
    ay[tid] = 0ull;
  }
  for (int s = 0; s < n_steps; ++s) {
    if (mem) lp[tid] = make_uint2(p.qx, p.qy);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      // (wave-uniform: a wave whose slots all lie past the list skips them)
      if (u * T + (tid & ~63) >= np) break;
      const int a = (int)(pr[u] & 1023u), b = (int)((pr[u] >> 10) & 1023u);
      const int sp = (int)(pr[u] >> 20);
      const uint2 pa = lp[a], pb = lp[b];
      const float rx = (float)(int32_t)(pb.x - pa.x) * sx0;
      const float ry = (float)(int32_t)(pb.y - pa.y) * sx1;
      int64_t fx, fy;  // zero for an empty slot (a == b: r = 0)
      pair_fix_sel(pt->cut2[sp], pt->sig6[sp], eps24, rx, ry, fx, fy);
      if (a != b) {
        atomicAdd(&ax[a], (unsigned long long)fx);
        atomicAdd(&ay[a], (unsigned long long)fy);
        atomicAdd(&ax[b], (unsigned long long)(-fx));
        atomicAdd(&ay[b], (unsigned long long)(-fy));
      }
    }
    __syncthreads();
    if (mem) {
      int64_t fxs = (int64_t)ax[tid], fys = (int64_t)ay[tid];
      ax[tid] = 0ull;
      ay[tid] = 0ull;
      if (d->n_walls) {
        int64_t az = 0;
        wall_forces<2>(d, si, (float)p.qx * sx0, (float)p.qy * sx1, 0.0f, fxs, fys, az,
                       st.wall_viol);
      }
      bd_step(pc, p, fxs, fys, s == 0 ? fs0 : fs, s == 0 ? tz0 : tz, fex, fey, k0, k1,
              (uint32_t)i, step0 + (uint64_t)s, s == n_steps - 1, &vx, &vy, &om,
              s == 0 ? an0 : p.an, nullptr, &noise, s == 0);
      const float ddx = (float)(int32_t)(p.qx - q0x) * sx0;
      const float ddy = (float)(int32_t)(p.qy - q0y) * sx1;
      dmax2 = fmaxf(dmax2, ddx * ddx + ddy * ddy);
    }
  }
  if (mem) {
    st.q[gi] = p.qx;
    st.q[M + gi] = p.qy;
    st.img[gi] = p.ix;
    st.img[M + gi] = p.iy;
    st.ang[gi] = p.an;
    st.vel[gi] = vx;
    st.vel[M + gi] = vy;
    st.vel[2 * M + gi] = 0.0f;
    st.omega[gi] = om;
    const float disp = sqrt_rn(dmax2);
    sc.disp[gi] = disp;
    if (!(disp < 0.5f * d->skin)) {  // a mover
      const int k = atomicAdd(&sc.nmov[e], 1);
      if (k < kMaxMovers) sc.movers[(size_t)e * kMaxMovers + k] = i;
    }
    if (st.reuse) {
      const PrevSlot w = prev_slot(st, par ^ 1);
      w.f[gi] = fs;
      w.tz[gi] = tz;
      w.ang[gi] = p.an;
    }
  }
  // the rest of k_check (this workgroup) reads the members' state, movers
  // and displacements: the barrier's workgroup-scope fences suffice
  __syncthreads();
}

// ------------------------------------------- neighbour-list window (2-D)
// Dense boxes: the rc + skin graph percolates, so clusters exceed a wave
// (and k_check's big-cluster workgroup).  The window keeps the build grid,
// the exact check and the exact re-run, but its sub-steps run chip-wide: a
// Verlet list per colloid (every j within r_i + r_j + skin), then one launch
// per sub-step with one thread per colloid, positions read from one buffer
// and written to the other (st.q, sc.qalt alternate; k_check copies back
// after an odd window).  Forces, noise and update are block_global_run's
// (pair_force, bd_step with the step's normals drawn fresh), so the bits are
// the same.  The 3-D twin is k_build_nlist3 / k_nl_step3.
constexpr int kNlMax = 48;  // neighbours per colloid (more: the env re-runs)

// Build step 2 (neighbour-list path), grid (ceil(N / 256), E), one thread
// per cell-sorted entry of k_build_sort: its neighbours into nl[k][gi]
// (neighbour-major, so the sub-step's reads coalesce).
__global__ __launch_bounds__(256) void k_build_nlist2(const Derived* __restrict__ d, DevState st,
                                                      Scratch sc, int lx, int ly) {
  __shared__ float nb2[kMaxSpecies * kMaxSpecies];
  for (int k = threadIdx.x; k < kMaxSpecies * kMaxSpecies; k += blockDim.x) nb2[k] = d->nb2[k];
  __syncthreads();
  const int e = blockIdx.y, N = st.n;
  const int ps = blockIdx.x * blockDim.x + threadIdx.x;
  if (ps >= N) return;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  const int ncell = 1 << (lx + ly);
  const int32_t* cs = sc.bcstart + (size_t)e * (ncell + 1);
  const int ncx = 1 << lx, ncy = 1 << ly;
  const int loy = ncy >= 3 ? -1 : 0, hiy = ncy >= 3 ? 1 : ncy - 1;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const int pk = sc.bsid[base + ps];
  const int i = pk & 0xffffff;
  const uint32_t qx = sc.bsq[base + ps], qy = sc.bsq[M + base + ps];
  const int c0 = cell_index(qx, qy, lx, ly);
  const int cx = c0 & (ncx - 1), cy = c0 >> lx;
  const int xa = ncx >= 3 ? max(cx - 1, 0) : 0;
  const int xb = ncx >= 3 ? min(cx + 1, ncx - 1) : ncx - 1;
  const int xw = ncx >= 3 ? (cx == 0 ? ncx - 1 : (cx == ncx - 1 ? 0 : -1)) : -1;
  int rb[6], re[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const int oy = loy + (r >> 1), part = r & 1;
    const bool use = oy <= hiy && (part == 0 || xw >= 0);
    const int row = ((cy + oy + ncy) & (ncy - 1)) << lx;
    const int c_lo = row | (part == 0 ? xa : xw), c_hi = row | (part == 0 ? xb : xw);
    rb[r] = use ? cs[c_lo] : 0;
    re[r] = use ? cs[c_hi + 1] : 0;
  }
  const float* nb2_row = nb2 + (pk >> 24) * kMaxSpecies;
  int cnt = 0;
  int32_t* out = sc.nl + base + i;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    for (int jj0 = rb[r]; jj0 < re[r]; jj0 += 4) {
      int pk4[4];
      uint32_t x4[4], y4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int jj = jj0 + u;
        const bool ok = jj < re[r];
        pk4[u] = ok ? sc.bsid[base + jj] : -1;
        x4[u] = ok ? sc.bsq[base + jj] : 0u;
        y4[u] = ok ? sc.bsq[M + base + jj] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (pk4[u] < 0 || (pk4[u] & 0xffffff) == i) continue;
        const float rx = (float)(int32_t)(x4[u] - qx) * sx0;
        const float ry = (float)(int32_t)(y4[u] - qy) * sx1;
        if (rx * rx + ry * ry < nb2_row[pk4[u] >> 24]) {
          if (cnt < kNlMax) out[(size_t)cnt * M] = pk4[u];
          ++cnt;
        }
      }
    }
  }
  sc.nn[base + i] = min(cnt, kNlMax);
  reinterpret_cast<uint2*>(sc.qa)[base + i] = make_uint2(qx, qy);  // sub-step 0's read buffer
  if (cnt > kNlMax) sc.fallback[e] = 1;  // -> the env re-runs on the global path
}

// Sub-step s of the 2-D neighbour-list window, one thread per colloid of
// every env (XCD-aware workgroup order: one env's colloids share an L2).
// Positions ping-pong between two AoS uint2 buffers in sc.qa (sub-step s
// reads buffer s & 1, the build filled buffer 0); the last sub-step writes
// st.q.
// sc.disp holds the squared maximum displacement until the last sub-step.
template <bool kMulti, bool kWalls>
__global__ __launch_bounds__(256) void k_nl_step2(const Derived* __restrict__ d, DevState st,
                                                  Scratch sc, int n_steps, int s,
                                                  const uint64_t* __restrict__ ctl) {
  __shared__ PairTables pt;
  if (kMulti) stage_pair_tables(d, &pt);
  const size_t M = (size_t)st.m;
  const unsigned per_xcd = gridDim.x >> 3;  // grid: a multiple of 8 workgroups
  const unsigned lb = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
  const size_t gi = (size_t)lb * blockDim.x + threadIdx.x;
  if (gi >= M) return;
  const int N = st.n;
  const int e = (int)(gi / N), i = (int)(gi - (size_t)e * N);
  if (sc.fallback[e] != 0) return;
  const size_t base = (size_t)e * N;
  const bool first = s == 0, last = s == n_steps - 1;
  const uint2* R = reinterpret_cast<const uint2*>(sc.qa) + (s & 1) * M;
  uint2* W = reinterpret_cast<uint2*>(sc.qa) + ((s & 1) ^ 1) * M;
  const int par = window_parity(ctl);
  const uint64_t step = ctl[kCtlStep] + (uint64_t)s;
  const int si = kMulti ? st.species[i] : 0;
  const float sx0 = d->sx[0], sx1 = d->sx[1];
  const int nn = sc.nn[gi];
  PState p;
  const uint2 qo = R[gi];
  p.qx = qo.x;
  p.qy = qo.y;
  p.ix = st.img[gi];
  p.iy = st.img[M + gi];
  p.an = st.ang[gi];
  uint32_t q0x, q0y;
  float dmax2 = 0.0f;
  if (first) {
    q0x = p.qx;
    q0y = p.qy;
    sc.bq[gi] = p.qx;
    sc.bq[M + gi] = p.qy;
    sc.bimg[gi] = p.ix;
    sc.bimg[M + gi] = p.iy;
    sc.bang[gi] = p.an;
  } else {
    q0x = sc.bq[gi];
    q0y = sc.bq[M + gi];
    dmax2 = sc.disp[gi];
  }
  const float eps24 = d->eps24;
  int64_t ax = 0, ay = 0;
  const int32_t* nlp = sc.nl + gi;
  for (int k0 = 0; k0 < nn; k0 += 8) {
    // eight neighbours per round: indices, then positions, in flight together
    int32_t pk[8];
    uint32_t xj[8], yj[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) pk[u] = k0 + u < nn ? nlp[(size_t)(k0 + u) * M] : -1;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint2 qj = R[base + (pk[u] < 0 ? i : (pk[u] & 0xffffff))];
      xj[u] = qj.x;
      yj[u] = qj.y;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (pk[u] < 0) continue;
      const float rx = (float)(int32_t)(xj[u] - p.qx) * sx0;
      const float ry = (float)(int32_t)(yj[u] - p.qy) * sx1;
      if (kMulti) {
        const int sp = si * kMaxSpecies + (pk[u] >> 24);
        pair_force(pt.cut2[sp], pt.sig6[sp], eps24, rx, ry, ax, ay);
      } else {
        pair_force(d->cut2[0], d->sig6[0], eps24, rx, ry, ax, ay);
      }
    }
  }
  if (kWalls) {
    int64_t az = 0;
    wall_forces<2>(d, si, (float)p.qx * sx0, (float)p.qy * sx1, 0.0f, ax, ay, az, st.wall_viol);
  }
  const bool reuse0 = st.reuse && first;  // sub-step 0 reuses the previous run's actions
  const PrevSlot prv = prev_slot(st, par);
  const float fs = reuse0 ? prv.f[gi] : st.f_swim[gi];
  const float tz = reuse0 ? prv.tz[gi] : st.torque_z[gi];
  const uint32_t an_swim = reuse0 ? prv.ang[gi] : p.an;
  const PConst pc = load_pconst(d, si);
  float vx = 0.0f, vy = 0.0f, om = 0.0f;
  bd_step(pc, p, ax, ay, fs, tz, st.f_ext[gi], st.f_ext[M + gi], d->key0, d->key1 ^ (uint32_t)e,
          (uint32_t)i, step, last, &vx, &vy, &om, an_swim);
  if (last) {  // nobody reads st.q during the window
    st.q[gi] = p.qx;
    st.q[M + gi] = p.qy;
  } else {
    W[gi] = make_uint2(p.qx, p.qy);
  }
  st.img[gi] = p.ix;
  st.img[M + gi] = p.iy;
  st.ang[gi] = p.an;
  const float ddx = (float)(int32_t)(p.qx - q0x) * sx0;
  const float ddy = (float)(int32_t)(p.qy - q0y) * sx1;
  dmax2 = fmaxf(dmax2, ddx * ddx + ddy * ddy);
  if (!last) {
    sc.disp[gi] = dmax2;
    return;
  }
  st.vel[gi] = vx;
  st.vel[M + gi] = vy;
  st.vel[2 * M + gi] = 0.0f;
  st.omega[gi] = om;
  const float disp = sqrt_rn(dmax2);
  sc.disp[gi] = disp;
  if (!(disp < 0.5f * d->skin)) {  // a mover (k_check's exact test)
    const int k = atomicAdd(&sc.nmov[e], 1);
    if (k < kMaxMovers) sc.movers[(size_t)e * kMaxMovers + k] = i;
  }
  if (st.reuse) save_forces(st, gi, par ^ 1);  // this run's actions, the final angle
}

// ---------------------------------------------------------------- check
// Whether the first n entries of a pair list (16-byte aligned, readable in
// whole 16-entry rounds) hold k1 or k2 under mask: 16 entries per round of
// loads.
__device__ __forceinline__ bool list_holds(const uint4* __restrict__ l, int n, uint32_t mask,
                                           uint32_t k1, uint32_t k2) {
  bool hit = false;
  for (int k = 0; k < n && !hit; k += 16) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = l[(k >> 2) + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t x = w[c] & mask;
        hit |= k + 4 * u + c < n && (x == k1 || x == k2);
      }
    }
  }
  return hit;
}

// cell_lx, cell_ly: the window's build grid, whose counting sort left the
// cell-sorted snapshot in global memory (sc.bsq / bsid / bcstart: every 2-D
// build, k_build_env included); -1: scan every colloid per mover.
__global__ __launch_bounds__(1024) void k_check(const Derived* __restrict__ d, DevState st,
                                                Scratch sc, int n_steps,
                                                uint64_t* __restrict__ step_ctr,
                                                uint32_t* __restrict__ arrive, int lx, int ly,
                                                int nlist, int cell_lx, int cell_ly) {
  extern __shared__ __align__(16) unsigned char smem[];
  int32_t* wave_sums = reinterpret_cast<int32_t*>(smem);  // 16
  int32_t* misc = wave_sums + 16;                          // 16
  int32_t* movers = misc + 16;                             // kMaxMovers
  int32_t* cnt = movers + kMaxMovers;                      // global-path cell counts
  __shared__ PairTables pt;
  const int e = blockIdx.x, T = blockDim.x, tid = threadIdx.x, N = st.n;
  const size_t M = (size_t)st.m, base = (size_t)e * N;
  role_begin(sc, kRoleCheck);
#ifdef SWARM_CHECK_TIMING
  uint64_t ct0 = __builtin_amdgcn_s_memrealtime(), ct1 = 0, ct2 = 0;
  int ckc = -1;
#endif
  // every load the test starts from is issued here together -- the window
  // counters, the build's flags, the mover count and list (written by the
  // run kernel) and the pair tables: one memory latency, not a chain
  const uint64_t step0 = step_ctr[kCtlStep];
  const int par = window_parity(step_ctr);  // reuse_forces slot of this window
  const int fb = sc.fallback[e];
  const int bign = nlist ? 0 : sc.big_n[e];
  const int nm_run = sc.nmov[e];
  const int mv_run = tid < kMaxMovers ? sc.movers[(size_t)e * kMaxMovers + tid] : 0;
  const int ovf = sc.l1_pairs ? sc.cand_ovf[e] : 0;
  for (int k = tid; k < kMaxSpecies * kMaxSpecies; k += T) {
    pt.cut2[k] = d->cut2[k];
    pt.sig6[k] = d->sig6[k];
  }
  if (tid < 16) misc[tid] = 0;
  __syncthreads();
  // flagged by the build: the env did not run (its state is the window start)
  const bool flagged_build = fb == 1;
  if (!flagged_build && bign > 0)
    run_big_clusters(d, st, sc, e, n_steps, step0, cnt, &pt, par);
#ifdef SWARM_CHECK_TIMING
  ct1 = __builtin_amdgcn_s_memrealtime();
#endif
  int nm = 0;  // movers of the window (listed in LDS below)
  bool kc_dmax = false;  // misc[7] holds the movers' largest displacement
  if (!flagged_build) {
    // the movers (displacement >= skin / 2) were listed by the run kernel
    // and the big-cluster run: no scan over all colloids here
    nm = nm_run;
    if (bign > 0) {
      // the big-cluster run of this workgroup appended entries a moment
      // ago: agent-scope loads
      if (tid == 0) misc[0] = __hip_atomic_load(&sc.nmov[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      nm = misc[0];
      for (int k = tid; k < min(nm, kMaxMovers); k += T)
        movers[k] = __hip_atomic_load(&sc.movers[(size_t)e * kMaxMovers + k], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (int k = tid; k < min(nm, kMaxMovers); k += T)
        movers[k] = k < kMaxMovers && k == tid ? mv_run : sc.movers[(size_t)e * kMaxMovers + k];
    }
    __syncthreads();
    if (nm > kMaxMovers) {
      if (tid == 0) misc[1] = 1;
    } else if (nm > 0) {
      // exact test of every (mover, non-neighbour) pair at the window-start
      // positions: d0 < rc + D_i + D_j could have interacted without its
      // force being computed.  Same-cluster pairs count too: a cluster links
      // particles through chains, so two of its members need not be listed
      // neighbours of each other.
      const bool multi = d->n_species > 1;  // else every pair's cutoff is cut2[0]
      const float rc0 = sqrtf(pt.cut2[0]);
      const float sx0 = d->sx[0], sx1 = d->sx[1];
      const bool per = d->periodic != 0;
      // Each global load of the test is a round trip to another XCD's
      // writes (~1 us): the mover's own state and the first 16 entries of its
      // wave's pair list are loaded once per mover, the candidate's four
      // words together, so a mover costs four rounds (its state; cell
      // ranges and list; candidate ids; candidate state), not seven.
      struct MoverCtx {
        uint32_t qx, qy;
        int32_t ix, iy;
        float disp;
        int sm, root, np;
        uint4 l[4];  // the first 16 entries of the mover's wave pair list
      };
      auto mover_ctx = [&](int m) {
        MoverCtx c;
        c.qx = sc.bq[base + m];
        c.qy = sc.bq[M + base + m];
        c.ix = per ? 0 : sc.bimg[base + m];
        c.iy = per ? 0 : sc.bimg[M + base + m];
        c.disp = sc.disp[base + m];
        c.sm = nlist ? 0 : sc.slot_of[base + m];
        c.root = nlist ? 0 : sc.root[base + m];
        c.np = 0;
        if (!nlist && c.sm >= 0) {
          const size_t wl = (size_t)e * sc.wmax + (c.sm >> 6);
          const uint4* pw = reinterpret_cast<const uint4*>(sc.pairs + wl * kPairsPerWave);
          c.np = sc.wave_npairs[wl];
#pragma unroll
          for (int u = 0; u < 4; ++u) c.l[u] = pw[u];
        }
        return c;
      };
      auto test_pair = [&](int m, int j, const MoverCtx& c) {
        const uint32_t jqx = sc.bq[base + j], jqy = sc.bq[M + base + j];
        const int32_t jix = per ? 0 : sc.bimg[base + j], jiy = per ? 0 : sc.bimg[M + base + j];
        const float jd = sc.disp[base + j];
        const int sj = nlist ? 0 : sc.slot_of[base + j];
        const int rj = nlist ? 0 : sc.root[base + j];
        // (non-periodic box: the unwrapped separation; the folded one would
        // only make the test stricter)
        const float rx = per ? (float)(int32_t)(jqx - c.qx) * sx0
                             : pair_disp(jqx, jix, c.qx, c.ix, sx0, false);
        const float ry = per ? (float)(int32_t)(jqy - c.qy) * sx1
                             : pair_disp(jqy, jiy, c.qy, c.iy, sx1, false);
        // the pair's own WCA cutoff r_m + r_j (not the largest one: a dense
        // mixture would fail the test for pairs that cannot interact)
        const float rc = multi ? sqrtf(pt.cut2[st.species[m] * kMaxSpecies + st.species[j]]) : rc0;
        const float lim = rc + c.disp + jd + 1e-3f;
        if (rx * rx + ry * ry < lim * lim) {
          // the lists are scanned 16 entries per round of loads (an
          // entry-by-entry loop waited one round trip per entry)
          bool listed = false;
          const int sm = c.sm;
          if (nlist) {  // j among m's listed neighbours
            const int nn = sc.nn[base + m];
            for (int k = 0; k < nn && !listed; k += 8) {
              int32_t v[8];
#pragma unroll
              for (int u = 0; u < 8; ++u)
                v[u] = k + u < nn ? sc.nl[(size_t)(k + u) * M + base + m] : -1;
#pragma unroll
              for (int u = 0; u < 8; ++u) listed |= (v[u] & 0xffffff) == j;
            }
          } else if (rj == c.root && sm < 0) {  // same big cluster
            const uint32_t bm = (uint32_t)(-1 - sm), bj = (uint32_t)(-1 - sj);
            const uint32_t k1 = bm | bj << 10, k2 = bj | bm << 10;
            const uint4* bp = reinterpret_cast<const uint4*>(sc.big_pairs + (size_t)e * kBigPairs);
            const int np = min(sc.big_np[e], kBigPairs);
            listed = list_holds(bp, np, 0xfffffu, k1, k2);
          } else if (rj == c.root) {  // same wave: its pairs
            const uint32_t lm = (uint32_t)(sm & 63), lj = (uint32_t)(sj & 63);
            const uint32_t k1 = lm | lj << 6, k2 = lj | lm << 6;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const uint32_t w[4] = {c.l[u].x, c.l[u].y, c.l[u].z, c.l[u].w};
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const uint32_t x = w[q] & 0xfffu;
                listed |= 4 * u + q < c.np && (x == k1 || x == k2);
              }
            }
            if (!listed && c.np > 16) {
              const uint4* pw = reinterpret_cast<const uint4*>(
                  sc.pairs + ((size_t)e * sc.wmax + (sm >> 6)) * kPairsPerWave);
              listed = list_holds(pw + 4, c.np - 16, 0xfffu, k1, k2);
            }
          }
          if (!listed) misc[1] = 1;
        }
      };
      // Candidates of a mover from the window's cell-sorted snapshot: every
      // j with d0 < rc + D_m + D_j lies within lim_max = rc_max + 2 D_max of
      // m (D_max: the largest displacement; non-movers moved less than
      // skin / 2), so within kc = ceil(lim_max / cell side) cells.  One wave
      // per mover, its lanes over the (2 kc + 1) rows' ranges.  Grids too
      // coarse for that (kc > 2, or fewer than 2 kc + 1 cells a side) scan
      // every colloid.
      int kc = 99;
      const int ncx = cell_lx >= 1 ? 1 << cell_lx : 0, ncy = cell_ly >= 1 ? 1 << cell_ly : 0;
      if (cell_lx >= 1 && cell_ly >= 1) {
        if (tid == 0) misc[7] = __float_as_int(0.5f * d->skin);
        __syncthreads();
        for (int k = tid; k < nm; k += T)
          atomicMax(&misc[7], __float_as_int(sc.disp[base + movers[k]]));  // >= 0: int order
        __syncthreads();
        const float dmax = __int_as_float(misc[7]);
        kc_dmax = true;
        const float lim_max = d->rc_max_f + 2.0f * dmax + 1e-3f;
        const float side = fminf(sx0 * (float)(1u << (32 - cell_lx)),
                                 sx1 * (float)(1u << (32 - cell_ly)));
        kc = (int)ceilf(lim_max / side);
        if (kc > 2 || ncx < 2 * kc + 1 || ncy < 2 * kc + 1) kc = 99;
      }
#ifdef SWARM_CHECK_TIMING
      ckc = kc;
#endif
      if (kc <= 2) {
        const int32_t* cs = sc.bcstart + (size_t)e * ((size_t)ncx * ncy + 1);
        // G lanes per mover, G = 64 / 2^k with every mover in flight at once
        // when they fit in the workgroup (a wave per mover took one chain of
        // memory latencies per 16 movers: the 9-16 us checks of the windows
        // with many movers)
        int G = 64;
        while (G > 4 && nm * G > T) G >>= 1;
        const int lane = tid & (G - 1), ng = T / G;
        for (int k = tid / G; k < nm; k += ng) {
          const int m = movers[k];
          const MoverCtx c = mover_ctx(m);
          const int cx = per ? (int)(c.qx >> (32 - cell_lx)) : cell_coord(c.qx, c.ix, cell_lx, false);
          const int cy = per ? (int)(c.qy >> (32 - cell_ly)) : cell_coord(c.qy, c.iy, cell_ly, false);
          for (int oy = -kc; oy <= kc; ++oy) {
            int y = cy + oy;
            if (!per && (y < 0 || y >= ncy)) continue;
            y = (y + ncy) & (ncy - 1);
            const int row = y << cell_lx;
            int x0 = cx - kc, x1 = cx + kc;
            if (!per) {
              x0 = max(x0, 0);
              x1 = min(x1, ncx - 1);
            }
            // the row's cells as up to two sorted ranges (a periodic row
            // wraps at one end at most: ncx >= 2 kc + 1)
            int b1 = 0, l1 = 0;
            if (x0 < 0) {
              b1 = cs[row | (ncx + x0)];
              l1 = cs[(row | (ncx - 1)) + 1] - b1;
              x0 = 0;
            } else if (x1 > ncx - 1) {
              b1 = cs[row];
              l1 = cs[(row | (x1 - ncx)) + 1] - b1;
              x1 = ncx - 1;
            }
            const int b0 = cs[row | x0], l0 = cs[(row | x1) + 1] - b0;
            for (int f = lane; f < l0 + l1; f += G) {
              const int j = sc.bsid[base + (f < l0 ? b0 + f : b1 + f - l0)] & 0xffffff;
              if (j != m) test_pair(m, j, c);
            }
          }
        }
      } else {
        for (int k = 0; k < nm; ++k) {  // every colloid against each mover
          const int m = movers[k];
          const MoverCtx c = mover_ctx(m);
          for (int j = tid; j < N; j += T)
            if (j != m) test_pair(m, j, c);
        }
      }
    }
    __syncthreads();
  }
  const bool rerun = flagged_build || misc[1] != 0;
#ifdef SWARM_CHECK_TIMING
  ct2 = __builtin_amdgcn_s_memrealtime();
#endif
  if (sc.l1_pairs) {
    // the candidate lists the run's extra workgroups built from this
    // window's start positions hold every pair of the next window's start
    // when the window ran on its decomposition (no re-run), no list
    // overflowed, and no particle moved more than cand_disp -- only movers
    // (>= skin / 2 <= cand_disp) can have: their largest displacement is
    // misc[7] when the cell test ran (kc_dmax), else it is taken here
    bool far = false;
    if (!rerun && nm > 0 && !kc_dmax) {
      if (tid == 0) misc[8] = 0;
      __syncthreads();
      for (int k = tid; k < nm; k += T) far |= !(sc.disp[base + movers[k]] <= d->cand_disp);
      if (far) misc[8] = 1;
      __syncthreads();
      far = misc[8] != 0;
    } else if (!rerun && nm > 0) {
      far = !(__int_as_float(misc[7]) <= d->cand_disp);
    }
    if (tid == 0) {
      sc.cand_ok[e] = !rerun && !far && ovf == 0 ? 1 : 0;
      sc.cand_ovf[e] = 0;
    }
  }
  if (tid == 0) {
    if (rerun) atomicAdd(&sc.stats[2], 1ull);
    atomicAdd(&sc.stats[3], 1ull);
  }
  if (rerun) {
    // a flagged env was skipped by k_cluster_run: its state is the window
    // start already; otherwise restore the snapshot k_cluster_run took
    for (int i = tid; i < N && !flagged_build; i += T) {
      const size_t gi = base + i;
      st.q[gi] = sc.bq[gi];
      st.q[M + gi] = sc.bq[M + gi];
      st.img[gi] = sc.bimg[gi];
      st.img[M + gi] = sc.bimg[M + gi];
      st.ang[gi] = sc.bang[gi];
    }
    if (tid == 0) sc.fallback[e] = 2;  // diagnostics: env re-run on the global path
    __syncthreads();
    if (global_lds_extra_words(N, st.dims, 1 << (lx + ly)) && d->periodic)  // LDS variant: periodic
      block_global_run_lds(d, st, e, n_steps, step0, lx, ly, false, 0.0f, 0.0f, cnt, wave_sums,
                           cnt + (1 << (lx + ly)) + 1, &pt, par);
    else
      block_global_run(d, st, sc, e, n_steps, step0, lx, ly, false, 0.0f, 0.0f, cnt, wave_sums,
                       &pt, par);
    save_forces_env(st, e, par ^ 1);  // the re-run replaced the run kernel's final state
  }
  __syncthreads();  // every read of nmov above is done
  if (tid == 0) {
    sc.nmov[e] = 0;
    // the next build's pair counters (an l1_pairs pair search starts before
    // its sort, so the sort cannot reset them)
    sc.gnpairs[e] = 0;
    sc.gnx[e] = 0;
  }
  advance_counter(step_ctr, arrive, step0, n_steps);
#ifdef SWARM_CHECK_TIMING
  if (tid == 0) {
    uint64_t* cw = sc.phase + 32 + 8 * (size_t)e;
    cw[0] = ct0; cw[1] = ct1; cw[2] = ct2; cw[3] = __builtin_amdgcn_s_memrealtime();
    cw[4] = (uint64_t)nm; cw[5] = (uint64_t)bign; cw[6] = (uint64_t)(int64_t)ckc; cw[7] = rerun;
  }
#endif
  role_end(sc, kRoleCheck);
}

}  // namespace swarm
