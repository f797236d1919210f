/*
 * phd_capi.h — the C-ABI boundary of the MI355X-native RB-PHD-SLAM filter
 * (libphdslam.so, built from cuda-phdslam_amd/csrc).
 *
 * Plain pointers, sizes and int status codes; no C++ or torch types.  Each
 * entry point names the reference interface it replaces (file:line in the
 * reference tree).  The reference's own API is C++ (src/phdfilter.h:10-34,
 * guarded by #ifdef __cplusplus); include/phdfilter.h re-exports that exact
 * C++ surface on top of this layer (cuda-phdslam_amd/csrc/phdfilter_shim.cpp),
 * and INTEGRATION.md shows the ctypes / C++ bindings a maintainer adds.
 *
 * Ownership: a phd_ctx owns a device-resident particle store (poses,
 * log-weights, per-particle GM map slabs) for n_particles particles on one GPU.
 * Unlike the reference (which mallocs/copies/frees device memory inside every
 * call, phdfilter.cu:3403-3409, 3778), state stays in HBM between calls and is
 * mirrored to the host only on request (phd_export_*).
 *
 * Streams: every call is enqueued on the context's stream (phd_set_stream) and
 * is asynchronous unless its comment says "synchronises".
 *
 * Errors: functions return PHD_OK (0) or a negative PHD_E* code; the reference
 * aborts inside checkCudaErrors instead (phdfilter.cu, passim).
 * phd_last_error() returns a human-readable message for the calling thread.
 */
#ifndef PHD_CAPI_H
#define PHD_CAPI_H

#include "phd_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PHD_OK 0
#define PHD_E_ARG -1        /* bad argument / shape */
#define PHD_E_HIP -2        /* HIP runtime error */
#define PHD_E_CAPACITY -3   /* a per-particle capacity (map slab, candidates) was exceeded */
#define PHD_E_UNSUPPORTED -4 /* configuration outside the implemented path */
#define PHD_E_NODEVICE -5   /* no GPU visible */

typedef struct phd_ctx phd_ctx;

/* Sizing of the device store. Zero fields take defaults. */
typedef struct phd_capacity {
    int map_capacity;        /* max GM components per particle map (slab width) */
    int max_measurements;    /* max |Z| per update (reference clamps to 256, phdfilter.cu:3390) */
    int candidate_capacity;  /* max merge candidates per particle (LDS) */
    int survivor_capacity;   /* max detection terms surviving the prune precheck per particle */
    int max_particles;       /* live particles the context can hold (0: n_particles).  With
                                n_predict_particles > 1 every predict multiplies the live count
                                (phdfilter.cu:1185-1238) until a resample draws n_particles
                                again (main.cpp:1286-1289: nEff, or more than 5 x n_particles) */
} phd_capacity;

/* Library identity and error text. */
const char* phd_version(void);
const char* phd_last_error(void);
int phd_device_count(int* count);

/* Context lifecycle.  Replaces the per-call cudaMalloc/cudaFree pattern of
 * phdPredict (phdfilter.cu:1080-1257) and phdUpdateSynth (:3336-3761). */
int phd_ctx_create(phd_ctx** out, int device, int n_particles, const phd_capacity* cap);
int phd_ctx_destroy(phd_ctx* ctx);
int phd_ctx_info(const phd_ctx* ctx, int* n_particles, phd_capacity* cap);

/* setDeviceConfig (phdfilter.cu:3885-3890, declared phdfilter.h:33). Copies the
 * 324-B SlamConfig; derived clutterDensity is taken as given (main.cpp:1065). */
int phd_set_config(phd_ctx* ctx, const phd_slam_config* cfg);

/* Stream the context enqueues on (hipStream_t, NULL = a private non-blocking
 * stream).  PHD_STREAM_NULL selects the HIP null stream itself (what a caller
 * whose own work runs on stream 0, e.g. torch's default stream, must pass to
 * order the context's kernels with its own). */
#define PHD_STREAM_NULL ((void*)-1)
int phd_set_stream(phd_ctx* ctx, void* hip_stream);
void* phd_get_stream(phd_ctx* ctx);
int phd_synchronize(phd_ctx* ctx);

/* Seed of the counter-based RNG contract (include/phd_rng.h); replaces the
 * time-seeded boost generators (rng.cpp:10-13) and initRandomNumberGenerators
 * (phdfilter.cu:142-157). */
int phd_set_seed(phd_ctx* ctx, uint64_t seed);

/* Host <-> device particle store.  maps are CSR: Gaussian2D AoS + offsets[n+1]
 * (the reference's concat + offsets, phdfilter.cu:2947-2960).  Synchronises. */
int phd_load_particles(phd_ctx* ctx, int n, const phd_pose* poses, const float* log_weights,
                       const phd_gaussian2d* maps, const int* offsets);
int phd_export_particles(phd_ctx* ctx, int n, phd_pose* poses, float* log_weights, int* map_sizes);
/* Poses only (the predict of the phdfilter.h shim).  Synchronises. */
int phd_set_poses(phd_ctx* ctx, int n, const phd_pose* poses);
/* Raw component counts of the n slabs of the current slab set (the sizes the
 * last update wrote, before any resample remap).  Synchronises. */
int phd_slab_sizes(phd_ctx* ctx, int* sizes);
/* offsets[n+1] must come from map_sizes (exclusive scan) of the same state. */
int phd_export_maps(phd_ctx* ctx, int n, const int* offsets, phd_gaussian2d* maps);

/* Mixed static + dynamic feature model (feature_model 2; SynthSLAM::maps_dynamic,
 * slamtypes.h:291).  phd_enable_dynamic allocates the dynamic slab sets
 * (dyn_capacity Gaussian4D per particle) and the update scratch.  With
 * feature_model 2, every predict (phd_predict_*, phd_step) also runs
 * predictMapMixed (phdfilter.cu:966-1035, :1241-1242) and phd_update /
 * phd_step run the mixed update (phdUpdateKernelMixed, :2323-2635, with
 * mergeAndCopyMaps of both maps, :3703-3726).  Dynamic maps follow the static
 * maps' slab references, so resampling and n_predict_particles carry them.
 * phd_load_dynamic_maps needs particle i to own slab i (after
 * phd_load_particles or an update).  Not supported with feature_model 2: CPHD,
 * replay mode, sharded steps.  Synchronise (except phd_predict_dynamic). */
int phd_enable_dynamic(phd_ctx* ctx, int dyn_capacity);
int phd_load_dynamic_maps(phd_ctx* ctx, int n, const phd_gaussian4d* maps, const int* offsets);
int phd_dynamic_sizes(phd_ctx* ctx, int* sizes);
int phd_export_dynamic_maps(phd_ctx* ctx, int n, const int* offsets, phd_gaussian4d* maps);
/* one predictMapMixed of every dynamic map (what each phdPredict does) */
int phd_predict_dynamic(phd_ctx* ctx);

/* phdPredict, Ackerman branch (phdfilter.cu:1140-1167 + kernel :785-825).
 * noise: host array of n AckermanNoise, or NULL to draw it on the device from
 * the RNG contract (stream PREDICT, counter = particle index, step). */
int phd_predict_ackerman(phd_ctx* ctx, phd_ackerman_control u, const phd_ackerman_noise* noise, uint64_t step);
/* phdPredict, constant-velocity branch (phdfilter.cu:1107-1134 + kernel :827-859). */
int phd_predict_cv(phd_ctx* ctx, const phd_cv_noise* noise, uint64_t step);

/* Measurements for the next update (host array, |Z| <= max_measurements; the
 * reference clamps at 256 and keeps them in __constant__ Z[256]). */
int phd_set_measurements(phd_ctx* ctx, const phd_measurement* z, int n_measure);

/* Static GM-PHD update of every particle (phdUpdateSynth static branch,
 * phdfilter.cu:3336-3761): in-range split, births, EKF, weights, prune, merge,
 * append out-of-range.  Adds Δlog w to the log-weights (no normalisation). */
int phd_update(phd_ctx* ctx);

/* logSumExp normalisation of the log-weights (phdfilter.cu:3748-3755).  If
 * lse_override is non-NULL the host-provided value (e.g. a global LSE from an
 * RCCL all-gather) is subtracted instead of the local one. */
int phd_normalize(phd_ctx* ctx, const float* lse_override);

/* nEff = 1/Σexp(2w)/N (main.cpp:1281-1284).  Synchronises; result to *neff. */
int phd_neff(phd_ctx* ctx, float* neff);

/* Stratified resample (main.cpp:453-501) with the fixed-point CDF of
 * phd_detmath.h; uniforms from the RNG contract (stream RESAMPLE, step), or
 * from u_host (n doubles, one per stratum) when non-NULL.  Copies parent
 * particles (SynthSLAM::copy_particles, slamtypes.h:313-333), sets
 * w = -log N.  idx_host (optional, n ints) receives the parent indices. */
int phd_resample(phd_ctx* ctx, const double* u_host, uint64_t step, int* idx_host);

/* One full filter step (run_synth loop body, main.cpp:1233-1297):
 * predict (if do_predict) -> update (if |Z|>0) -> normalize -> nEff ->
 * resample when nEff <= resample_threshold.  *resampled (optional) reports it. */
int phd_step(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step, float* neff_out,
             int* resampled);
/* CPHD (filter_type 1): log cardinality distribution of every particle after
 * the last update, cn_host[n * (max_cardinality+1) + k] = log p_n(k)
 * (particles.cardinalities, phdfilter.cu.bak:2700-2706).  Synchronises. */
int phd_cardinality_distribution(phd_ctx* ctx, float* cn_host);
/* Number of normalisations so far (phd_step, phd_normalize, sharded resample)
 * whose nEff decision triggered a resample (a device counter; the bench
 * reports the resample rate without a per-step read-back).  Synchronises. */
int phd_resample_count(phd_ctx* ctx, int* count);
/* The part of phd_step before normalisation: predict (if do_predict) and
 * update, then (optional) a device copy of the n unnormalised log-weights to
 * dev_logw_out — a shard's input to the all-gather of a sharded step. */
int phd_predict_update(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step,
                       float* dev_logw_out);

/* CPHD births through the prediction (addBirths / birthsKernel,
 * phdfilter.cu.bak:738-870 — the CPHD update array has no birth terms): append
 * to every particle's map one component per measurement of z (the previous
 * scan; static-labelled ones when labels are on): the inverse measurement from
 * the particle's pose, weight birth_weight.  Replaces the context's
 * measurements (call phd_set_measurements for the update afterwards).  Not in
 * replay mode.  A context whose step births follow the filter type (the
 * default, phd_set_step_births(ctx, -1)) switches them off at the first call —
 * the caller's loop places the births, as before step births existed; with
 * phd_set_step_births(ctx, 1) the call fails (births are never placed twice). */
int phd_add_births(phd_ctx* ctx, const phd_measurement* z, int n_measure);

/* The step's births (replaces addBirths in the driver loop, phdfilter.cu.bak:
 * 738-870 / main.cpp's CPHD step: predict -> births of the previous scan ->
 * update): phd_step, phd_predict_update and the sharded re-update place one
 * birth per valid measurement of the PREVIOUS measurement set (the one before
 * the last phd_set_measurements; replay mode: the replayed set itself) at each
 * particle's predicted pose, weight birth_weight, after its map — read by the
 * update in place (no copy of the maps; with no measurements this step they
 * are appended to the maps).  on: 1 on, 0 off, -1 with the filter type (the
 * default: on for CPHD, whose update array has no birth terms; the PHD update
 * has its own).  phd_step_births reports the effective setting. */
int phd_set_step_births(phd_ctx* ctx, int on);
int phd_step_births(phd_ctx* ctx, int* on);

/* ---- device-pointer hooks for multi-GPU sharding (RCCL all-gather lives in
 * the caller: bench.py / phdslam.dist).  All pointers are device pointers. ---- */
int phd_copy_log_weights(phd_ctx* ctx, float* dev_dst);            /* n floats */
int phd_set_log_weights(phd_ctx* ctx, const float* dev_src);       /* n floats */
/* Resample with a caller-computed parent index list whose parents are all
 * local (dev_idx: n ints in [0,n)). */
int phd_apply_resample(phd_ctx* ctx, const int* dev_idx, float new_log_weight);
/* Global normalise + nEff + resample decision + parent list over the
 * all-gathered log-weights of every rank (dev_w_all: n_total floats, normalised
 * in place).  Every rank runs the same deterministic kernels on identical input
 * and gets identical results; seed is the shared resample seed (stratum j uses
 * counter j of stream RESAMPLE).  The local slice [offset, offset+n) of the
 * normalised weights is copied into the context.  dev_parents (n_total ints)
 * is written only when *resampled = 1.  Synchronises. */
int phd_global_resample(phd_ctx* ctx, float* dev_w_all, int n_total, int offset, uint64_t seed, uint64_t step,
                        int* dev_parents, float* neff, int* resampled);
/* Everything of a sharded resample before its all-to-all (phdslam/dist.py),
 * with one host read-back.  dev_w_all holds the world*n gathered log-weights
 * (rank r's shard at r*n).  On the device: global normalise + nEff + decision +
 * parents (as phd_global_resample, identical on every rank), the migration plan
 * (k_migration_plan: children of local parents stay, surplus fills deficits in
 * rank order, one record per distinct parent and destination), the records this
 * rank sends packed into dev_send_records (room for send_capacity records, log-
 * weight new_log_weight) and the local remap (keep_src) with new_log_weight.
 * Device scratch: dev_parents (world*n ints), dev_keep_src (n), dev_send_src
 * (send_capacity), dev_recv_rec (n).  Host outputs (world ints each): demand
 * (children per rank), send_records (per destination), recv_records (per
 * source) — the all-to-all sizes in records.  The migrants are placed by
 * phd_shard_receive.  PHD_E_CAPACITY if the records exceed send_capacity (the
 * remap is applied already: abandon the step).  world*n <= 2^20 (the global
 * part runs one 1024-thread workgroup per chunk of 1024 log-weights).
 * Synchronises. */
int phd_shard_resample(phd_ctx* ctx, float* dev_w_all, int world, int rank, uint64_t seed, uint64_t step,
                       int* dev_parents, int* dev_keep_src, int* dev_send_src, int* dev_recv_rec,
                       void* dev_send_records, int send_capacity, float new_log_weight, int* demand,
                       int* send_records, int* recv_records, float* neff, int* resampled);
/* Place received records (source-rank order) into slots first_slot .. +n_slots
 * (first_slot = demand[rank]): slot first_slot+i takes record dev_recv_rec[i]. */
int phd_shard_receive(phd_ctx* ctx, const void* dev_records, const int* dev_recv_rec, int n_slots, int first_slot);

/* ---- sync-free sharded step (phdslam/dist.py ShardedFilter.step) ----
 * The plan of phd_shard_resample without its host read-back: every rank
 * exchanges FIXED blocks of block_records records per peer (one equal-split
 * all-to-all of world * block_records * phd_record_bytes bytes, block d for
 * rank d), so nothing on the host waits for the counts.  Records beyond a
 * peer's block go to dev_overflow (room for overflow_capacity records) and are
 * exchanged later, after phd_shard_poll, only when some were written; the slots
 * they feed stay "pending" until then.  Enqueues: global normalise + nEff +
 * decision + parents, this rank's plan, the remap of the kept particles (the
 * identity without a resample, swapped in unconditionally), the packing of
 * dev_send_blocks (world blocks) and an asynchronous read-back of the counts.
 * Scratch as phd_shard_resample. */
int phd_shard_resample_async(phd_ctx* ctx, float* dev_w_all, int world, int rank, uint64_t seed, uint64_t step,
                             int* dev_parents, int* dev_keep_src, int* dev_send_src, int* dev_recv_rec,
                             void* dev_send_blocks, int block_records, void* dev_overflow, int overflow_capacity,
                             float new_log_weight);
/* The sharded step's plan beside part C.  phd_wait_logw makes `stream` wait
 * until the log-weights of every update enqueued so far on the context's
 * stream are final, with their mirror (dev_logw_out) written: after the CPHD
 * terms launch or the split PHD update's part A, else after the update — so an
 * all-gather enqueued on `stream` runs beside part C.  phd_set_plan_stream
 * (NULL: off) makes phd_shard_resample_async launch the plan on that stream
 * (after the caller's all-gather there) and order the pack of the outgoing
 * records, which reads the posterior maps, after it on the context stream. */
int phd_wait_logw(phd_ctx* ctx, void* stream);
int phd_set_plan_stream(phd_ctx* ctx, void* stream);
/* Place the records of the received blocks (block s from rank s) into this
 * rank's deficit slots (the deficit is read on the device). */
int phd_shard_receive_blocks(phd_ctx* ctx, const void* dev_recv_blocks, int block_records, const int* dev_recv_rec);
/* Wait for the last plan's counts (call it once the next step's update is
 * enqueued, so the device never idles on it): demand, records sent to / received
 * from each rank (world ints each), pending slots, nEff, decision.  Records
 * beyond block_records per peer (send_records[d] > block_records) must then be
 * exchanged from the overflow buffers, sender position Σ_{d'<d} max(sent_d' - K,
 * 0) onward, and placed with phd_shard_receive_overflow; the pending slots are
 * then re-updated by phd_update_pending.  PHD_E_CAPACITY if the overflow buffer
 * was too small. */
int phd_shard_poll(phd_ctx* ctx, int* demand, int* send_records, int* recv_records, int* pending, float* neff,
                   int* resampled);
int phd_shard_receive_overflow(phd_ctx* ctx, const void* dev_recv_overflow, int block_records,
                               const int* dev_recv_rec);
/* Predict + update of the pending slots of the last poll with the sets of the
 * last update (same input and output slabs): the slots whose record arrived
 * after the update ran on them.  dev_logw_out as phd_predict_update. */
int phd_update_pending(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step,
                       float* dev_logw_out);
/* Global particle index of local particle 0 (predict-noise counter offset). */
int phd_set_index_offset(phd_ctx* ctx, int offset);
/* Set every log-weight to `value` (e.g. -log N after a sharded resample). */
int phd_fill_log_weights(phd_ctx* ctx, float value);
/* Fixed-size particle records for migration between ranks. */
int phd_record_bytes(const phd_ctx* ctx, size_t* bytes);
int phd_pack_particles(phd_ctx* ctx, const int* dev_src_idx, int count, void* dev_records);
int phd_unpack_particles(phd_ctx* ctx, const void* dev_records, const int* dev_dst_idx, int count);

/* Outputs of recoverSlamState (main.cpp:318-388): expected pose
 * (Σ exp(w)·state), arg-max particle, and per-particle cardinality Σ_j w_j.
 * Synchronises. */
int phd_expected_pose(phd_ctx* ctx, phd_pose* pose, int* map_particle);
int phd_cardinalities(phd_ctx* ctx, float* cn_host);
/* EAP expected map (computeExpectedMap main.cpp:290-316 +
 * reduceGaussianMixture gm_reduce.cpp:59-132) of the current store, computed
 * on the device: the components of every map weighted by exp(log w_n), reduced
 * by the greedy merge in the reference's emission order.  Writes *n_out; if
 * out is NULL or out_cap < *n_out nothing is copied and PHD_E_CAPACITY is
 * returned (out_cap >= the total component count always suffices). */
int phd_expected_map(phd_ctx* ctx, phd_gaussian2d* out, long out_cap, long* n_out);
/* EAP map of the dynamic (Gaussian4D) maps, feature_model 2: recoverSlamState's
 * exp_map_dynamic (main.cpp:369-371 -> gm_reduce.cpp:59-132, 4-D LLT distance).
 * Same conventions as phd_expected_map. */
int phd_expected_map_dynamic(phd_ctx* ctx, phd_gaussian4d* out, long out_cap, long* n_out);
/* Synchronous decision rounds of the last phd_expected_map (diagnostic; 1 for
 * the single-workgroup fallback of non-finite inputs). */
int phd_expected_map_groups(phd_ctx* ctx, int* groups);

/* Per-update timing of the fused kernel with HIP events recorded on the
 * context stream around each launch (ring of max_records pairs).
 * phd_update_timing synchronises, returns the summed ms over the recorded
 * launches and clears the ring; phd_last_update_ms reads the latest one. */
int phd_enable_timing(phd_ctx* ctx, int max_records);
/* Record the events around every stride-th update only (default 1: every
 * update).  Each event record costs the stream a few microseconds, so a long
 * timed run samples its updates instead of timing all of them. */
int phd_set_timing_stride(phd_ctx* ctx, int stride);
int phd_update_timing(phd_ctx* ctx, float* total_ms, int* count);
int phd_last_update_ms(phd_ctx* ctx, float* ms);

/* Replay mode (the reference's profile_run, main.cpp:1314-1321): the state
 * loaded by the preceding phd_load_particles becomes a fixed prior; every
 * subsequent predict restores poses/log-weights from it and every update reads
 * it again (writing the posterior to the other slab set).  Each phd_step then
 * does identical work, as the bench requires.  on=0 leaves replay mode. */
int phd_set_replay(phd_ctx* ctx, int on);

/* Local pieces of a cross-rank log-sum-exp: out[0] = max w, out[1] = Σ exp(w - max).
 * Synchronises. */
int phd_lse_parts(phd_ctx* ctx, float* out_host);

/* Per-update capacity check (a 4-B read-back + sync) on/off, and an explicit
 * check of the sticky error word. */
int phd_set_check_each_update(phd_ctx* ctx, int on);
int phd_check_errors(phd_ctx* ctx);

/* Merge implementation: 0 = parallel exact greedy (default; falls back to the
 * serial greedy per particle on degenerate input), 1 = serial greedy only.
 * phd_merge_fallbacks returns (and clears) how many particle-updates took the
 * serial fallback since the last call.  Synchronises. */
int phd_set_merge_mode(phd_ctx* ctx, int mode);
/* Threads per particle of the fused update (one workgroup per particle):
 * 0 = automatic (fewest rounds of resident workgroups, weighted by the
 * per-workgroup latency of each size), or 256 / 512 / 1024.
 * phd_update_threads reports the choice, its LDS and the resident workgroups. */
int phd_set_update_threads(phd_ctx* ctx, int threads);
int phd_update_threads(phd_ctx* ctx, int* threads, size_t* lds_bytes, int* resident_workgroups);
/* Form of the PHD update: 0 = automatic (the occupancy cost model), 1 = one
 * fused launch, 2 = split into part A (classify, pair walk) and part C
 * (candidates, merge) through a per-particle handoff in HBM — the form whose
 * halves fit more workgroups per CU when the maps are large (config 5).  The
 * CPHD update is always split (its terms launch sits between the parts).
 * phd_update_form reports whether the configured update runs split. */
int phd_set_update_form(phd_ctx* ctx, int form);
/* Undirected-edge pool of the parallel merge (0 = automatic: the occupancy
 * model's, grown while the workgroups per CU stay the same).  A particle whose
 * merge graph has more edges takes the serial greedy; its culled-pair list
 * shares the pool's LDS (a longer list walks again with the exact distances).
 * For tests of those paths and capacity studies. */
int phd_set_edge_pool(phd_ctx* ctx, int pool);
/* Culled-pair list of the parallel merge held to at most `pairs` entries per
 * particle (0 = the layout's, par | off | pool): a longer list walks again with
 * the exact distances in place.  A test hook for that path. */
int phd_set_pair_list_cap(phd_ctx* ctx, int pairs);
int phd_update_form(phd_ctx* ctx, int* split);
/* Diagnostics (-DPHD_STAMPS builds): enable / fetch n*32 per-workgroup phase
 * clock stamps of the fused update.  Synchronises when host != NULL. */
int phd_debug_stamps(phd_ctx* ctx, unsigned long long* host, int enable);
int phd_merge_fallbacks(phd_ctx* ctx, int* count);
/* Returns (and clears) how many particle-updates overflowed the merge's culled
 * pair list and ran the neighbourhood walk a second time with the exact
 * distances in place (still the parallel merge).  Synchronises. */
int phd_merge_pair_overflows(phd_ctx* ctx, int* count);
/* Returns (and clears) how many particle-updates set a capacity / range error
 * status bit (survivor, candidate or map capacity, likelihood range) since the
 * last call — the count behind phd_check_errors' sticky bits.  Synchronises. */
int phd_status_errors(phd_ctx* ctx, int* count);
/* Per-particle status word of the last update (n ints, PHD_ST_* bits of
 * phd_kernels.h: 1 survivor / 2 candidate / 4 map capacity, 8 serial merge,
 * 16 likelihood range, 32 pair-list overflow walk).  Synchronises. */
int phd_particle_status(phd_ctx* ctx, int* host_status);

/* Config file loader for the reference's cfg/config.cfg surface
 * (loadConfig, main.cpp:956-1073): "key = value" lines, '#' comments.  Fills
 * defaults first, then computes clutterDensity (main.cpp:1065-1066).
 * data_dir (optional, cap bytes) receives data_directory. */
int phd_config_defaults(phd_slam_config* cfg);
int phd_config_load(const char* path, phd_slam_config* cfg, char* data_dir, int data_dir_cap);

/* Synthetic replay scenarios for BASELINE.json configs; host-only.
 * phd_synth_preset fills the config and shape of config `id` (1..5);
 * phd_synth_scenario writes n poses / log-weights, n*G prior components (CSR
 * offsets n+1) and M measurements. */
int phd_synth_preset(int id, phd_slam_config* cfg, int* n, int* G, int* M, float* detect_frac);
int phd_synth_scenario(const phd_slam_config* cfg, int n, int G, int M, float detect_frac, uint64_t seed,
                       phd_pose* poses, float* log_weights, phd_gaussian2d* maps, int* offsets, phd_measurement* z);

#ifdef __cplusplus
}
#endif

#endif /* PHD_CAPI_H */
