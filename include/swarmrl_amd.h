/*
 * swarmrl_amd.h -- C ABI of the MI355X active-Brownian swarm engine.
 *
 * This is the drop-in boundary that replaces the ESPResSo calls made by
 * SwarmRL's engine adapter (reference: swarmrl/engine/espresso.py).  Every
 * entry point below names the reference call site it stands in for.  The
 * ABI uses only plain C types and pointers: no torch, no HIP types (a HIP
 * stream is passed as `void*`).  All functions return SWARM_OK (0) or an
 * error code; the message of the last error on the calling thread is
 * returned by swarm_last_error().  No C++ exception crosses this boundary.
 *
 * Error codes map onto the Python exceptions the reference raises:
 *   SWARM_EINVAL    -> ValueError   (bad configuration, espresso.py:180-182, 252-288)
 *   SWARM_ESTATE    -> RuntimeError (mutation after first integrate, espresso.py:300-305)
 *   SWARM_EDEVICE   -> RuntimeError (HIP runtime failure)
 *   SWARM_ECAPACITY -> ValueError   (size beyond what this build supports)
 *
 * Units: simulation units of the reference (espresso.py:211-234):
 * length 1 um, time 1 s, energy 293 K * k_B.
 *
 * State representation (identical in the CPU oracle and on the GPU):
 *   position  : per axis a uint32 fraction of the box (q * L / 2^32) plus an
 *               int32 image counter; unwrapped x = (img + q / 2^32) * L.
 *   orientation (2-D): uint32 angle, theta = a * 2 pi / 2^32.
 *   orientation (3-D): fp32 unit director [3], rotated each sub-step by
 *               the rotation vector (Rodrigues) and renormalised.
 * Index g = env * n_particles + i.  Device arrays are axis-major [3][E*N].
 */
#ifndef SWARMRL_AMD_H
#define SWARMRL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_MAX_SPECIES 16
#define SWARM_MAX_CONES 16
#define SWARM_MAX_DETECTED_TYPES 8

#define SWARM_OK 0
#define SWARM_EINVAL 1
#define SWARM_ESTATE 2
#define SWARM_EDEVICE 3
#define SWARM_ECAPACITY 4

/* Physical parameters of one engine (all envs share them).
 * Mirrors MDParams (espresso.py:30-88) after unit conversion, plus the
 * per-particle friction/mass registered by add_colloid_on_point
 * (espresso.py:376-413).  A "species" is one distinct
 * (radius, gamma_t, gamma_r, mass, rinertia) combination. */
typedef struct swarm_params {
  int32_t n_dims;   /* 2 or 3 (espresso.py:143-152, n_dims) */
  int32_t periodic; /* MDParams.periodic (espresso.py:270) */
  double box[3];    /* box_l (espresso.py:267) */
  double time_step; /* system.time_step (espresso.py:268) */
  double kT;        /* Brownian thermostat kT (espresso.py:1171, 1179-1184) */
  double wca_epsilon; /* WCA epsilon (espresso.py:814-819) */
  uint64_t seed;    /* thermostat seed (espresso.py:1183) */
  int32_t n_species;
  /* ESPResSo's integrator.run(k, reuse_forces=True) (espresso.py:1304-1306):
   * the Brownian propagator takes each step's forces from the force
   * calculation that ended the previous step, and a run with reuse_forces
   * does not recompute them first -- so sub-step 0 of every run uses the
   * swim force, torque and director of the previous run's last force
   * calculation (the actions set since then act from sub-step 1).
   * 1: that semantics (SwarmEngine's default, as the reference);
   * 0: every sub-step uses the current actions. */
  int32_t reuse_forces;
  double radius[SWARM_MAX_SPECIES];
  double gamma_t[SWARM_MAX_SPECIES];  /* 6 pi eta r  (espresso.py:108-113) */
  double gamma_r[SWARM_MAX_SPECIES];  /* 8 pi eta r^3 */
  double mass[SWARM_MAX_SPECIES];     /* used for the BD thermal velocity */
  double rinertia[SWARM_MAX_SPECIES]; /* used for the BD thermal omega */
} swarm_params_t;

/* Raw device pointers of the SoA state, for zero-copy consumers. */
typedef struct swarm_device_views {
  uint32_t *q;        /* [3][E*N] */
  int32_t *img;       /* [3][E*N] */
  uint32_t *ang;      /* [E*N]    */
  float *f_swim;      /* [E*N]    */
  float *torque_z;    /* [E*N]    */
  float *f_ext;       /* [3][E*N] */
  float *vel;         /* [3][E*N] (written by the last sub-step of a run) */
  float *omega_z;     /* [E*N]    */
  uint8_t *species;   /* [N]      */
  int32_t n_envs;
  int32_t n_particles;
  int32_t n_dims;
  int32_t reserved0;
  float *dir3;        /* [3][E*N] 3-D directors */
  float *torque_xy;   /* [2][E*N] 3-D torque x, y */
  float *omega_xy;    /* [2][E*N] 3-D angular velocity x, y */
} swarm_device_views_t;

/* A confining or user wall (espresso.py:667-800): a WCA constraint with
 * sigma = r_particle * 2^(-1/6), cutoff = r_particle (the wall type has
 * radius 0) and the engine's epsilon, acting on every particle.
 *   kind 0 = espressomd.shapes.Wall: dist = n . x_folded - offset
 *            (add_confining_walls, espresso.py:683-697);
 *   kind 1 = the vertical Rhomboid of add_walls (espresso.py:765-784):
 *            corner + s a + t b (s, t in [0, 1]), a and b in the xy plane,
 *            spanning the whole box in z; distance in the xy plane.
 * A particle on or inside a wall (dist <= 0) is a constraint violation:
 * it is counted (swarm_engine_wall_violations) and gets no wall force. */
typedef struct swarm_wall {
  int32_t kind;
  int32_t reserved;
  double normal[3]; /* kind 0 */
  double offset;    /* kind 0 */
  double corner[3]; /* kind 1 */
  double a[3];      /* kind 1 */
  double b[3];      /* kind 1 */
} swarm_wall_t;

#define SWARM_MAX_WALLS 16

/* Vision-cone parameters (SubdividedVisionCones,
 * swarmrl/observables/subdivided_vision_cones.py:25-60). */
typedef struct swarm_vision_params {
  float vision_range;
  float vision_half_angle;
  int32_t n_cones;
  int32_t n_types;                       /* len(detected_types) */
  int32_t detected_types[SWARM_MAX_DETECTED_TYPES];
  float rims[SWARM_MAX_CONES + 1];       /* -a + k*2a/n, computed in fp32 */
} swarm_vision_params_t;

typedef struct swarm_engine swarm_engine_t;

/* Thread-local message of the last failing call. */
const char *swarm_last_error(void);

/* Build provenance (no reference counterpart): the 12-hex-digit hash of the
 * HIP sources and this header the library was compiled from
 * (__graft_entry__.build, swarmrl_amd._capi.source_hash); swarmrl_amd._capi
 * warns when it differs from the checkout it runs in. */
const char *swarm_build_id(void);

/* Engine construction: replaces espressomd.System(...) + _init_system +
 * part.add for all particles (espresso.py:192-196, 236-288, 415-441).
 * `species` is [n_particles]: index into the per-species arrays of params. */
int swarm_engine_create(const swarm_params_t *params, int32_t n_envs,
                        int32_t n_particles, const int32_t *species,
                        swarm_engine_t **out);
void swarm_engine_destroy(swarm_engine_t *e);

/* Bind all later launches to a HIP stream (hipStream_t as void*). */
int swarm_engine_set_stream(swarm_engine_t *e, void *hip_stream);

/* Initial state from host fp64 arrays pos[E][N][3] (unwrapped) and
 * dir[E][N][3]; replaces part.add(pos=...) + _rotate_colloid_to_2d
 * (espresso.py:428-449). */
int swarm_engine_upload_state(swarm_engine_t *e, const double *pos,
                              const double *director);

/* Exact state transfer in the engine's own number format (host arrays):
 * q/img [3][E*N], ang [E*N].  Used for checkpoints and bit-exact parity. */
int swarm_engine_upload_raw(swarm_engine_t *e, const uint32_t *q,
                            const int32_t *img, const uint32_t *ang);
int swarm_engine_download_raw(swarm_engine_t *e, uint32_t *q, int32_t *img,
                              uint32_t *ang);

/* Synchronous copy of the state to host fp64 arrays [E][N][3]; replaces
 * the particle property getters used by get_particle_data and the Colloid
 * snapshot (espresso.py:1216-1225, 1320-1336).  Any pointer may be NULL. */
int swarm_engine_download_state(swarm_engine_t *e, double *pos_unwrapped,
                                double *director, double *velocity);

/* Per-particle swim force and z-torque [E*N]; replaces
 * coll.swimming = {"f_swim": ...} and coll.ext_torque = ...
 * (espresso.py:1228-1235).  on_device = 0: host arrays (copied);
 * 1: device arrays copied on the engine stream; 2: device arrays BOUND
 * (zero copy): later launches read them directly, so the caller keeps them
 * alive and unchanged until the next set_actions call. */
int swarm_engine_set_actions(swarm_engine_t *e, const float *f_swim,
                             const float *torque_z, int32_t on_device);

/* Per-particle external force [E*N][3] (host); replaces p.ext_force. */
int swarm_engine_set_external_force(swarm_engine_t *e, const double *f_ext);

/* new_direction handling of manage_forces (espresso.py:1236-1249): in 2-D
 * rotate about +-z so the director equals dir; in 3-D set the director to
 * dir (normalised).  dir [E*N][3], mask [E*N]. */
int swarm_engine_set_directors(swarm_engine_t *e, const double *dir,
                               const uint8_t *mask);

/* 3-D only: the x and y components of the lab-frame torque [2][E*N]
 * (the z component is set_actions' torque_z); replaces coll.ext_torque =
 * action.torque (espresso.py:1230-1235).  on_device as in set_actions
 * (0 host, 1 device copy; binding is not offered). */
int swarm_engine_set_torque_xy(swarm_engine_t *e, const float *torque_xy,
                               int32_t on_device);

/* 3-D directors in the engine's own format (host fp32 [3][E*N]), for
 * checkpoints and bit-exact parity. */
int swarm_engine_upload_directors(swarm_engine_t *e, const float *dir3);
int swarm_engine_download_directors(swarm_engine_t *e, float *dir3);

/* Walls (see swarm_wall_t); replaces add_confining_walls / add_walls
 * (espresso.py:667-800).  Replaces any previous set; n_walls <= 16. */
int swarm_engine_set_walls(swarm_engine_t *e, const swarm_wall_t *walls,
                           int32_t n_walls);

/* Number of (particle, sub-step) wall contacts with dist <= 0 since the
 * engine was created (ESPResSo raises for those; synchronous). */
int swarm_engine_wall_violations(swarm_engine_t *e, uint64_t *count);

/* Steepest-descent overlap removal (espresso.py:1161-1168): n_steps of
 * dp = clamp(gamma * F, -max_disp, max_disp) per free coordinate. */
int swarm_engine_remove_overlap(swarm_engine_t *e, int32_t n_steps,
                                double gamma, double max_displacement);

/* n_steps Brownian-dynamics sub-steps with WCA pair forces; replaces
 * system.integrator.run(k, reuse_forces=True, recalc_forces=False)
 * (espresso.py:1304-1306).  Asynchronous on the engine stream. */
int swarm_engine_integrate(swarm_engine_t *e, int32_t n_steps);

/* Launch the next integration window's position-only preparation (cluster
 * decomposition) on `stream` (a hipStream_t; NULL = engine stream), so it
 * can overlap the observable and policy work that produces the slice's
 * actions (espresso.py:1253-1306: manage_forces precedes integrator.run and
 * cannot change positions).  The caller orders `stream` after the last
 * position change and the engine stream after `stream` (events); the next
 * swarm_engine_integrate consumes the preparation.  Any position change in
 * between (upload, remove_overlap) discards it.  No-op for engines on the
 * global path.  n_steps_hint is unused (kept for the noise variant below). */
int swarm_engine_prebuild(swarm_engine_t *e, void *stream, int32_t n_steps_hint);

/* Defer the next window's cluster decomposition instead (latency-bound 2-D
 * engines with the three-launch build): its three stages -- counting sort,
 * pair search, cluster build -- then ride along as extra workgroups in the
 * slice's next engine-bound launches, swarm_vision_cone (stages 1 and 2)
 * and swarm_engine_policy_mlp_sample (stage 3), on the engine stream with
 * no second stream, fork or join (espresso.py:1253-1306: the positions do
 * not change between manage_forces and integrator.run).  Stages no launch
 * carried run at the next swarm_engine_integrate.  *deferred = 0 when the
 * engine cannot defer (use swarm_engine_prebuild). */
int swarm_engine_defer_build(swarm_engine_t *e, int32_t *deferred);

/* Same contract for the noise table of latency-bound engines: the normals
 * of the next min(n_steps_hint, 128) sub-steps, computed on `stream` (it
 * depends on the step counter only, so it may run beside the build).  No-op
 * for engines without a noise table. */
int swarm_engine_prebuild_noise(swarm_engine_t *e, void *stream, int32_t n_steps_hint);

/* Counters of the cluster windows since the engine was created (or the
 * last reset), summed over the envs: out4[0] windows whose pair search
 * filtered the candidate lists prepared during the previous run, out4[1]
 * windows whose pair search waited for the fresh build sort instead (the
 * lists could not be used), out4[2] windows re-run exactly on the global
 * path, out4[3] windows checked.  Measurement only (bench.py); reset != 0
 * zeroes them after reading. */
int swarm_engine_build_stats(swarm_engine_t *e, uint64_t *out4, int32_t reset);

/* Diagnostics of the last integration window, per env (host arrays [E],
 * either may be NULL): fallback 0 = cluster path, 1 = flagged by the build
 * (cluster > 64 lanes or neighbour overflow), 2 = re-run on the global path;
 * waves = 64-lane waves the env's clusters were packed into. */
int swarm_engine_window_stats(swarm_engine_t *e, int32_t *fallback,
                              int32_t *waves);

/* Kernel timing for measurement (bench.py roofline): returns the summed
 * duration (ms) and count of the eager k_cluster_run launches recorded since
 * the previous call (HIP events on the engine stream; waits for them), then
 * enables (1) or disables (0) recording.  While recording, a window captured
 * into a HIP graph gets event-record nodes (hipEventRecordExternal) around
 * its run-kernel node instead: see swarm_engine_profile_graph. */
int swarm_engine_profile(swarm_engine_t *e, int32_t enable, double *run_ms,
                         int32_t *launches);

/* Run-kernel durations inside captured graphs (bench.py roofline: the kernel
 * timed as it runs in the replayed episode): after a replay of a
 * graph captured with recording enabled has been launched, waits for the
 * device and writes the time (ms) between the event nodes around every
 * captured run node, in capture order, to ms_out[0..cap), and (cal_out, may
 * be NULL) the time between the two event nodes of an empty pair recorded
 * right after each run node -- what a pair of event nodes adds by itself --
 * and their count to *launches (each value is the latest replay's).
 * release = 1 then destroys the events (only once no graph holding them
 * replays again). */
int swarm_engine_profile_graph(swarm_engine_t *e, int32_t release, float *ms_out,
                               float *cal_out, int32_t cap, int32_t *launches);

/* The same captured run nodes timed by the kernel itself: each records the
 * earliest start of its blocks and the latest end of its waves on the
 * device's constant-rate wall clock.  reset = 1: clears the stamps on
 * `stream` (before a replay); reset = 0: waits for the device and writes the
 * durations (ms, end - start) of the captured run nodes, in capture order,
 * to ms_out[0..cap) (each the latest replay's).  *launches = the number of
 * stamped nodes (at most 512; swarm_engine_profile_graph's release resets
 * the count). */
int swarm_engine_profile_stamps(swarm_engine_t *e, int32_t reset, void *stream, float *ms_out,
                                int32_t cap, int32_t *launches);

/* The workgroup roles of the launches between the captured run nodes,
 * stamped the same way while profiling (stamp slot k: the k_check after the
 * k-th run node and the next window's build / observable / policy launches
 * up to the next run).  Writes, for slot k and role q (k_check, build sort,
 * vision grid, field, pair search, vision cone, cluster build, policy MLP,
 * then three progress marks: pair filter lists tested, pair filter output
 * reserved, vision-cone bins summed; *n_roles = 11, swarm::kRoles),
 * us_out[2 (k n_roles + q) + 0 / 1] = the role's earliest
 * start / latest end in microseconds after the k-th run node's end (NaN
 * where the role did not run), for entries below cap.  Waits for the
 * device; reset with swarm_engine_profile_stamps. */
int swarm_engine_profile_roles(swarm_engine_t *e, double *us_out, int32_t cap, int32_t *n_roles);

/* Kernel timing for measurement (bench.py roofline): builds the next 2-D
 * cluster window from the current positions, then launches its run kernel
 * `reps` times back to back between two HIP events on the engine stream and
 * returns the mean duration (ms) per launch; the exact check follows
 * (untimed).  The repeats integrate the same window again and again on one
 * decomposition, so the state afterwards is for measurement only (re-upload
 * it to continue a simulation).  SWARM_ESTATE unless the engine runs 2-D
 * cluster windows. */
int swarm_engine_time_run(swarm_engine_t *e, int32_t n_steps, int32_t reps,
                          double *run_ms);

/* Diagnostics: 32 shader-clock stamps of the last cluster build's phases
 * (env 0), filled only by builds compiled with -DSWARM_PHASE_TIMING. */
int swarm_engine_debug_phases(swarm_engine_t *e, uint64_t *out32);
/* Diagnostics (SWARM_PHASE_TIMING builds fill it; zeros otherwise): per run
 * wave w of the last cluster window, out[4w..4w+3] = realtime stamps (100 MHz)
 * at the wave's entry and end, its pair passes and pair count. */
int swarm_engine_debug_wave_stamps(swarm_engine_t *e, uint64_t *out, int32_t n_words);

/* Trajectory recording (espresso.py:1110-1159: _update_traj_holder at every
 * write interval, chunks written to HDF5) without a host synchronisation, so
 * it can sit inside a captured HIP graph.  swarm_engine_traj_ring allocates
 * a ring of `capacity` entries for env `env` in host-pinned, device-mapped,
 * coherent memory and returns its host address: bytes [0, 8) hold the count
 * of entries recorded so far (uint64), entry k % capacity starts at byte
 * 64 + (k % capacity) * entry_bytes.  swarm_engine_traj_record launches, on
 * the engine stream, the copy of the env's state into the next slot (the
 * slot index is a device counter, so graph replays fill successive slots)
 * and then publishes the new count.  The caller drains entries
 * [drained, count) with swarm_traj_entry_to_host, and must do so before
 * `capacity` newer ones overwrite them.  Entry layout: uint64 step counter,
 * uint32 q[D][N], int32 img[D][N], then uint32 ang[N] (2-D) or float
 * dir[3][N] (3-D), then float vel[D][N]. */
int swarm_engine_traj_ring(swarm_engine_t *e, int32_t capacity, int32_t env,
                           void **host_ring, int64_t *entry_bytes);
int swarm_engine_traj_record(swarm_engine_t *e);
/* One ring entry -> fp64 [N][3] arrays exactly as swarm_engine_download_state
 * converts the live state (unwrapped positions, directors, velocities) and
 * its step counter; any output may be NULL.  Host only (no device access). */
int swarm_traj_entry_to_host(const swarm_engine_t *e, const void *entry, double *pos,
                             double *director, double *velocity, uint64_t *step);

/* Total number of BD sub-steps integrated so far (the noise counter). */
int64_t swarm_engine_step_count(const swarm_engine_t *e);

int swarm_engine_device_views(swarm_engine_t *e, swarm_device_views_t *v);

/* Vision cones for n_agents agents (distinct indices into [0,N), device int32),
 * radii[N] device fp32 (radius of the SEEN colloid by list position,
 * subdivided_vision_cones.py:199-203); out device fp32
 * [E][n_agents][n_cones][n_types].  Replaces
 * SubdividedVisionCones.compute_observable (subdivided_vision_cones.py:241-258).
 * types[N] device int32: particle type of every colloid. */
int swarm_vision_cone(swarm_engine_t *e, const swarm_vision_params_t *vp,
                      const int32_t *agent_idx, int32_t n_agents,
                      const float *radii, const int32_t *types, float *out);

/* swarm_vision_cone with the caller's promise that agent_idx, radii and
 * types stay allocated and unchanged while the engine lives (the
 * SubdividedVisionCones observable keeps them).  The engine remembers the
 * arguments: when the next build is deferred (swarm_engine_defer_build),
 * the slice's reward launch (swarm_field_transform / swarm_field_distance)
 * also builds the vision grid of the positions it sees, and the next call
 * with the same arguments -- the next slice's observable, nothing having
 * moved the colloids in between -- runs the cone without a grid launch. */
int swarm_vision_cone_persistent(swarm_engine_t *e, const swarm_vision_params_t *vp,
                                 const int32_t *agent_idx, int32_t n_agents,
                                 const float *radii, const int32_t *types, float *out);

/* The observable and the rollout policy of an actor-critic agent in one
 * launch: swarm_vision_cone_persistent's cones into `features` ([E][n_agents]
 * [n_cones][n_types], n_cones * n_types <= 4) and, from them, the actor MLP +
 * Gumbel sampling of swarm_policy_mlp_sample (features as its observation,
 * d_in = n_cones * n_types, k <= 4 actions, hidden <= 256; weights read in
 * place) into out_idx / out_logp / out_f / out_t[E * n_agents] (agent
 * e * n_agents + a, the flattened observable's order; out_logits optional).
 * Replaces SubdividedVisionCones.compute_observable + FlaxModel.compute_action
 * + the sampling and action-table lookup of ActorCriticAgent.calc_action
 * (subdivided_vision_cones.py:241-258, actor_critic.py:159-184,
 * flax_network.py:153-195, gumbel_distribution.py:37-40).  agent_state:
 * device call counters, one per agent (n_state >= E * n_agents; each call
 * draws agent a's uniforms with counter agent_state[a] and advances it).
 * Runs on the engine's stream; a deferred build rides along as in the two
 * calls it replaces.  Sampling parity is statistical, as for
 * swarm_policy_mlp_sample; the logits may differ from that kernel's in the
 * last bits (the hidden units are summed in another split). */
int swarm_engine_vision_policy(swarm_engine_t *e, const swarm_vision_params_t *vp,
                               const int32_t *agent_idx, int32_t n_agents, const float *radii,
                               const int32_t *types, float *features, const float *w1,
                               const float *b1, int32_t hidden, const float *w2, const float *b2,
                               int32_t k, uint64_t seed, uint64_t *agent_state, int32_t n_state,
                               float explore_p, const float *f_table, const float *t_table,
                               int64_t *out_idx, float *out_logp, float *out_f, float *out_t,
                               float *out_logits);

/* Distances to a source for the concentration-field observable and the
 * gradient-sensing task (concentration_field.py:84-108,
 * gradient_sensing.py:92-126): for agent a of env e,
 *   p      = unwrapped_pos / box_scale (fp64),
 *   d_cur  = || fp32(source/box_scale - p) ||,
 *   d_prev = same for the history position,
 * then (if update_history) history <- current.  History is kept as raw
 * engine coordinates hist_q/hist_img [3][E*n_agents] (device).
 * init_only != 0: only copy the current positions into the history. */
int swarm_field_distance(swarm_engine_t *e, const int32_t *agent_idx,
                         int32_t n_agents, const double source[3],
                         const double box_scale[3], uint32_t *hist_q,
                         int32_t *hist_img, float *d_cur, float *d_prev,
                         int32_t update_history, int32_t init_only);

/* Fused field observable / reward for an affine decay f(d) = a + b d:
 * out[e][a] = scale * (f(d_cur) - f(d_prev)) (concentration_field.py:
 * 102-104), clipped at 0 when clip_at_zero (gradient_sensing.py:117-118);
 * the history is updated.  Distances as in swarm_field_distance. */
int swarm_field_transform(swarm_engine_t *e, const int32_t *agent_idx,
                          int32_t n_agents, const double source[3],
                          const double box_scale[3], uint32_t *hist_q,
                          int32_t *hist_img, float decay_a, float decay_b,
                          float scale, int32_t clip_at_zero, float *out);

/* Parity helper: all pairs (i<j) of env `env` closer than `cutoff`
 * (minimum image if periodic) as int32 [max_pairs][2] (host), count in
 * *n_pairs; returns SWARM_ECAPACITY if more than max_pairs. */
int swarm_engine_neighbor_pairs(swarm_engine_t *e, int32_t env, double cutoff,
                                int32_t *pairs, int32_t max_pairs,
                                int32_t *n_pairs);

/* Pairwise scaled distances for ParticleSensing / SpeciesSearch
 * (particle_sensing.py:95-121, species_search.py:97-130): for every env e,
 * agent a < n_agents and sensed column m in [m0, m0 + mc),
 *   out[e][m - m0][a] = || (fp32(x_sensed[m]) - fp32(x_agent[a])) / box_scale ||
 * with unwrapped positions (no minimum image, as the reference).  Indices
 * are device int32 into [0, N); out is device fp32 [E][mc][n_agents]. */
int swarm_pair_distances(swarm_engine_t *e, const int32_t *agent_idx, int32_t n_agents,
                         const int32_t *sensed_idx, int32_t m0, int32_t mc,
                         const double box_scale[3], float *out);

/* Fused action sampling for the device rollout path (all pointers device):
 * per agent a < n, over logits [n][k] fp32 (k <= 64):
 *   idx  = argmax_j(logits_j - log(-log u_j))     gumbel_distribution.py:37-40
 *   idx  = RandomExploration(idx) when explore_p > 0 (random_exploration.py:54-71)
 *   logp = log(softmax(logits)_idx + 1e-8)         flax_network.py:185-192
 *   out_f = f_table[idx], out_t = t_table[idx]     actor_critic.py:159-184
 * u from Philox4x32-10 keyed by seed; state = n_state >= ceil(n / 64) uint64
 * call counters of device memory (one per group of 64 agents; zero-initialise
 * once), advanced on every call so graph replays draw fresh numbers.
 * Asynchronous on `stream` (hipStream_t, NULL = default stream).
 * Replaces the jnp sampling chain of FlaxModel.compute_action. */
int swarm_sample_actions(const float *logits, int32_t n, int32_t k, uint64_t seed,
                         uint64_t *state, int32_t n_state, float explore_p,
                         const float *f_table, const float *t_table, int64_t *out_idx,
                         float *out_logp, float *out_f, float *out_t, void *stream);

/* The whole rollout policy of FlaxModel.compute_action
 * (networks/flax_network.py:153-195) for the reference's actor-critic MLP
 * (Dense(hidden) -> ReLU -> Dense(k), CI/espresso_tests/integration_tests/
 * test_rl_trainers.py:17-26) in one launch:
 *   logits = W2 relu(W1 obs_a + b1) + b2        (fp32; torch Linear layouts
 *            W1 [hidden][d_in], W2 [k][hidden], read in place)
 * followed by exactly the sampling of swarm_sample_actions (same counters,
 * same bits for the same logits).  obs [n][d_in]; d_in <= 16, hidden <= 256,
 * k <= 16.  out_logits [n][k] is optional (NULL: not written).  The critic
 * head is not evaluated (the rollout does not read it). */
int swarm_policy_mlp_sample(const float *obs, int32_t n, int32_t d_in, const float *w1,
                            const float *b1, int32_t hidden, const float *w2, const float *b2,
                            int32_t k, uint64_t seed, uint64_t *state, int32_t n_state,
                            float explore_p, const float *f_table, const float *t_table,
                            int64_t *out_idx, float *out_logp, float *out_f, float *out_t,
                            float *out_logits, void *stream);

/* swarm_policy_mlp_sample, also carrying the last stage of engine e's
 * deferred build (swarm_engine_defer_build) as extra workgroups of the same
 * launch when it is pending; same arguments and results otherwise. */
int swarm_engine_policy_mlp_sample(swarm_engine_t *e, const float *obs, int32_t n,
                                   int32_t d_in, const float *w1, const float *b1,
                                   int32_t hidden, const float *w2, const float *b2,
                                   int32_t k, uint64_t seed, uint64_t *state,
                                   int32_t n_state, float explore_p, const float *f_table,
                                   const float *t_table, int64_t *out_idx, float *out_logp,
                                   float *out_f, float *out_t, float *out_logits,
                                   void *stream);

/* Kernel timing for measurement (bench.py's roofline of the PPO update):
 * the summed duration (ms) and count of the k_ppo_grads launches this
 * thread made through swarm_ppo_epoch_grad since the previous call (HIP
 * events on the caller's stream around each epoch's launches; waits for
 * them), then enables recording with `enable` back-to-back launches of the
 * (deterministic) gradient kernel per epoch, or disables it (0).  Not for
 * use under graph capture. */
int swarm_ppo_profile(int32_t enable, double *grads_ms, int32_t *launches);

/* The gradient of one PPO epoch -- ProximalPolicyLoss._calculate_loss
 * differentiated by jax.value_and_grad (swarmrl/losses/
 * proximal_policy_loss.py:62-138, :160-168) with its GAE value function
 * (value_functions/generalized_advantage_estimate.py:42-72) -- for the
 * actor-critic MLP Dense(hidden) -> ReLU -> {Dense(k) logits, Dense(1)
 * value}.  Samples are T time slices x S agent columns, sample t * S + col:
 * x [T*S][d_in], actions [T*S] (int64), old_logp [T*S], rewards [T][S].
 * Parameters in torch Linear layouts: w1 [hidden][d_in], b1 [hidden],
 * wa [k][hidden], ba [k], wc [1][hidden], bc [1].  Writes grad =
 * d loss / d params, concatenated as w1 | b1 | wa | ba | wc | bc
 * (hidden*d_in + hidden + k*hidden + k + hidden + 1 floats).  The loss:
 *   sum -min(r A, clip(r, 1 - clip_eps, 1 + clip_eps) A)
 *   - entropy_coef * sum -(p + 1e-8) log(p + 1e-8)
 *   + 0.5 * sum huber(V, R)
 * with r = exp(log(p_a + 1e-8) - old_logp), A the GAE advantages
 * normalised by mean and population std (+ fp32 eps) and held constant,
 * R = A_raw + V differentiated through V as in the reference.
 * d_in <= 32, hidden <= 256, k <= 16, T*S < 2^31.  workspace: device
 * memory of at least swarm_ppo_workspace_bytes(T, S, d_in, hidden, k)
 * bytes.  Deterministic (fixed reduction order).  Asynchronous on
 * `stream`. */
int64_t swarm_ppo_workspace_bytes(int32_t T, int32_t S, int32_t d_in, int32_t hidden,
                                  int32_t k);
int swarm_ppo_epoch_grad(const float *x, int32_t T, int32_t S, int32_t d_in,
                         const int64_t *actions, const float *old_logp, const float *rewards,
                         const float *w1, const float *b1, int32_t hidden, const float *wa,
                         const float *ba, int32_t k, const float *wc, const float *bc,
                         float gamma, float lambda, float clip_eps, float entropy_coef,
                         void *workspace, int64_t workspace_bytes, float *grad, void *stream);

/* The optimizer of the PPO update (torch.optim.Adam as TorchModel builds it
 * for the optax optimizer of swarmrl/networks/flax_network.py:42-79): the six tensors
 * w1 | b1 | wa | ba | wc | bc of swarm_ppo_epoch_grad, updated in place with
 * their first / second moments and per-tensor step counts (device fp32, as
 * torch's capturable Adam keeps them).  weight_decay 0, no amsgrad. */
typedef struct {
  float lr, beta1, beta2, eps;
  float *param[6];
  float *exp_avg[6];
  float *exp_avg_sq[6];
  float *step[6];
} swarm_adam_t;

/* One PPO epoch with the optimizer step fused into its last launch: the
 * gradient of swarm_ppo_epoch_grad (written to grad, the parameters read
 * from adam->param) followed by the Adam step of torch's fused Adam
 * (step += 1; m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
 * p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps), fp32).
 * Replaces swarm_ppo_epoch_grad + optimizer.step() (three launches fewer per
 * epoch).  The workspace must be zero-filled before its first use (the
 * kernel leaves its ticket at zero after each call). */
int swarm_ppo_epoch_step(const float *x, int32_t T, int32_t S, int32_t d_in,
                         const int64_t *actions, const float *old_logp, const float *rewards,
                         int32_t hidden, int32_t k, float gamma, float lambda, float clip_eps,
                         float entropy_coef, const swarm_adam_t *adam, void *workspace,
                         int64_t workspace_bytes, float *grad, void *stream);

/* Random Network Distillation distance (the intrinsic reward of
 * swarmrl/intrinsic_reward/random_network_distillation.py:126-143 with the
 * networks of rnd_configs.py:17-38): for every observation a < n of x
 * [n][d_in] (device fp32), target and predictor networks Dense(width) ->
 * ReLU -> Dense(width) -> ReLU -> Dense(width), and
 *   out[a] = (sum_k |t_k - p_k|^order)^(1/order)      (ZnNL OrderNDifference).
 * target / predictor: host arrays of the six device parameter pointers
 * w1 [width][d_in], b1, w2 [width][width], b2, w3 [width][width], b3 (torch
 * Linear layouts, read in place).  width = 32, d_in <= 16.  Asynchronous on
 * `stream`. */
int swarm_rnd_distance(const float *x, int32_t n, int32_t d_in, int32_t width,
                       const float *const *target, const float *const *predictor,
                       int32_t order, float *out, void *stream);

/* The per-env RND intrinsic reward added to the task reward (the device
 * path of random_network_distillation.py:126-143 followed by the
 * `task + intrinsic` of actor_critic.py calc_reward): x [n_envs * per_env]
 * [d_in] observations (env-major), the metric of every observation into
 * metric[n_envs * per_env] (as swarm_rnd_distance), r_e = mean of env e's
 * metrics (fp64 sum in a fixed order), clipped to [clip_lo, clip_hi] when
 * clip != 0, into env_reward[n_envs], and
 *   rewards[e][a] = base[e][a] + r_e   (base NULL: r_e).
 * workspace: device memory of swarm_rnd_env_workspace_bytes(n_envs, per_env)
 * bytes, zeroed before its first use (the call leaves it ready for the
 * next one; one workspace per concurrent caller).  One launch, asynchronous
 * on `stream`; no host synchronisation. */
int swarm_rnd_env_reward(const float *x, int32_t n_envs, int32_t per_env, int32_t d_in,
                         int32_t width, const float *const *target,
                         const float *const *predictor, int32_t order, int32_t clip,
                         float clip_lo, float clip_hi, const float *base, float *metric,
                         float *env_reward, float *rewards, void *workspace,
                         int64_t workspace_bytes, void *stream);
int64_t swarm_rnd_env_workspace_bytes(int32_t n_envs, int32_t per_env);

/* Neighbour reductions for the classical agents (all pointers device):
 * get_colloids_in_vision of bechinger_models.py:156-171 (range + cone) and
 * lymburn_model.py:113-125 (range only, half_angle < 0), fused with the
 * sums those agents take over the neighbours it returns.  pos, dir and vel
 * [E][N][3] fp64 (pos unwrapped; vel may be NULL), types [N];
 * candidates: j != agent with bit types[j] set in cand_type_mask.  Per env
 * e and agent a, out[e][a][12] (fp64) = {count, sum 1/(2 pi |d|), sum d (3),
 * sum |d|^2, sum dir_j (3), sum v_j (3)} with d = x_j - x_agent.
 * Asynchronous on `stream`. */
int swarm_neighbor_reduce(const double *pos, const double *dir, const double *vel,
                          const int32_t *types, int32_t n_envs, int32_t n,
                          const int32_t *agent_idx, int32_t n_agents,
                          uint32_t cand_type_mask, double vision_range,
                          double half_angle, double *out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* SWARMRL_AMD_H */
