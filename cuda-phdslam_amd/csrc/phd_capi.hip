/*
 * phd_capi.hip — implementation of the C-ABI (include/phd_capi.h): context,
 * device-resident particle store, launches, host mirroring.
 *
 * The reference allocates, uploads, launches, downloads and frees inside every
 * phdPredict / phdUpdateSynth call (phdfilter.cu:1080-1257, :3336-3761) and
 * interleaves ~4 small memcpys per particle (:3227-3257).  Here the store lives
 * in HBM for the lifetime of the context; a filter step is a handful of
 * asynchronous launches on one stream with no host round trip.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "phd_capi.h"
#include "phd_kernels.h"
#include "phd_mixed_k.h"

using namespace phd;

static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIPCHK(expr)                                                                         \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return fail(PHD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
    } while (0)

struct phd_ctx {
    int device = 0;
    int n = 0;        // live particles (grows by n_predict_particles per predict until a resample)
    int n_base = 0;   // the filter's particle count (phd_ctx_create): a resample draws this many
    int nmax = 0;     // allocated particles: max(n_base, capacity.max_particles)
    phd_capacity cap{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    phd_slam_config cfg{};
    bool cfg_set = false;
    uint64_t seed = 0x5eed5eedULL;
    /* Device store.  Two slab sets (ping-pong between updates) plus a migration
     * set X; particle n's map is slab d_src[n] of set `cur` (bit 30 -> set X).
     * Resampling rewrites d_src (copy-on-write), never the slabs. */
    int cur = 0;
    float* d_map[2] = {nullptr, nullptr};
    int* d_size[2] = {nullptr, nullptr};
    float* d_map_x = nullptr;
    int* d_size_x = nullptr;
    int* d_src = nullptr;
    phd_pose* d_pose = nullptr;
    float* d_logw = nullptr;
    phd_pose* d_tmp_pose = nullptr;
    int* d_tmp_src = nullptr;
    float* d_tmp_logw = nullptr;
    // replay mode (bench): fixed prior in set 0 + saved poses / log-weights
    bool replay = false;
    phd_pose* d_pose_prior = nullptr;
    float* d_logw_prior = nullptr;
    // scratch
    float* d_delta = nullptr;
    int* d_status = nullptr;
    int* d_err = nullptr;
    float* d_zr = nullptr;
    float* d_zb = nullptr;
    int* d_zok = nullptr;
    float4* d_zs = nullptr;  // valid measurements sorted by wrapped bearing
    unsigned short* d_zbin = nullptr;  // bearing-bin index into d_zs
    int Mv = 0;
    int M = 0;
    int zwide = 0;  // some |measurement bearing| >= 3 (see UpdateArgs::zwide)
    phd_ackerman_noise* d_noise_a = nullptr;
    phd_cv_noise* d_noise_cv = nullptr;
    unsigned long long* d_cdf = nullptr;
    int* d_idx = nullptr;
    double* d_u = nullptr;
    float* d_out = nullptr;  // [0]=lse [1]=neff [2]=resample flag ...
    float* d_cn = nullptr;
    size_t upd_lds = 0;
    int upd_threads = 256;   // threads per particle of the fused update
    int upd_threads_req = 0; // 0 = automatic (choose_update_threads)
    int upd_resident = 0;    // update workgroups resident at once on the device
    int upd_resident_a = 0;  // the same for part A of the three-launch CPHD update
    int upd_resident_p = 0;  // the same for the launch that carries a fused predict (its own registers)
    int epool = 0;
    int upd_cphd = 0;            // launch configured for the CPHD kernels
    int upd_split = 0;           // the update runs as part A + part C (CPHD: always, with the terms between)
    int upd_form_req = 0;        // PHD form requested: 0 automatic, 1 fused, 2 split (phd_set_update_form)
    int epool_req = 0;           // merge edge pool requested (phd_set_edge_pool; 0: the occupancy model's)
    int plreq = 0;               // culled-pair list cap (phd_set_pair_list_cap; 0: the layout's)
    size_t upd_lds_a = 0;        // CPHD: LDS of part A (upd_lds: part C)
    unsigned char* d_hand = nullptr;  // CPHD: per-particle handoff between the three launches
    double* d_cn_coef = nullptr; // CPHD cardinality coefficients, n x cn_stride (row = slab of the current set)
    double* d_cn_x = nullptr;    // their rows for migration set X
    int cn_stride = 0;
    double* d_lfact = nullptr;   // log n!, n = 0..lfact_n-1
    int lfact_n = 0;
    bool cn_valid = false;       // a CPHD update has produced coefficients
    unsigned long long* d_stamps = nullptr;  // diagnostic builds (PHD_STAMPS)
    int merge_mode = 0;
    bool check_each_update = true;
    int index_offset = 0;                       // global id of local particle 0 (noise counter)
    unsigned long long* d_cdf_g = nullptr;      // CDF scratch for the global resample
    int cdf_g_cap = 0;
    int* d_mig = nullptr;  // per-rank demand of a sharded resample
    int* h_mig = nullptr;      // host-mapped copy of d_mig, written by the plan's tail itself
    int* h_mig_dev = nullptr;  // its device address
    int h_mig_cap = 0;
    int h_mig_world = 0;  // world of the plans h_mig holds (its sequence word's slot depends on it)
    int mig_cap = 0;
    // sync-free sharded step: pending slots (records beyond the fixed blocks),
    // the plan's read-back event, and its state
    int* d_pend = nullptr;
    bool plan_open = false;   // a plan's counts not yet polled
    unsigned plan_seq = 0;    // sequence number of the last plan launched (h_mig[3 world + MIG_SEQ] when done)
    int plan_ovf_cap = 0;     // overflow capacity of the open plan (records)
    int plan_world = 0;
    int plan_rank = 0;
    int pend_count = 0;       // pending slots of the last polled plan
    // chunk partials + chunk-relative CDF of the multi-block sharded plan (k_rs_*)
    unsigned char* d_rsx = nullptr;
    size_t rsx_bytes = 0;
    unsigned* d_plan_sync = nullptr;  // k_shard_plan's hand-off words (PLAN_*), zero between launches
    float* logw_mirror = nullptr;     // the next full update also writes its log-weights here (phd_predict_update)
    // PHD_RS_OVERLAP: the resample k_rs_step of this phd_step, launched by the
    // CPHD chain on `aux` after the terms (its arguments; `launched` once done)
    struct {
        bool armed = false, launched = false;
        bool lead = false;  // (PHD_RS_LEAD) it ran in part C's lead workgroup: no event to wait on
        RsStepArgs a;
        int B = 0;
    } rs_ov;
    hipStream_t aux = nullptr;
    hipEvent_t ev_terms = nullptr, ev_rs = nullptr;
    // the sharded step beside part C (phd_wait_logw / phd_set_plan_stream):
    // ev_logw marks the last update's log-weights final (after the CPHD terms /
    // the split part A, else after the update); the plan runs on plan_stream
    // and ev_plan orders the pack after it
    hipEvent_t ev_logw = nullptr, ev_plan = nullptr;
    hipStream_t plan_stream = nullptr;
    bool logw_marked = false;  // ev_logw recorded since the last phd_wait_logw-relevant update
    bool src_fresh = false;    // every slab reference is the identity (a full update since the last remap)
    int plan_max_blocks = 0;          // workgroups of k_shard_plan resident at once (0: not queried)
    // per-update kernel timing (HIP events on the context stream)
    std::vector<hipEvent_t> ev_a, ev_b;
    int ev_next = 0, ev_used = 0;
    int timing_stride = 1, timing_tick = 0;  // events around every timing_stride-th update
    EapScratch* eap = nullptr;  // expected-map scratch (phd_eap.hip), allocated on first use
    int eap_groups = 0;
    // mixed feature model (feature_model 2, phd_enable_dynamic): dynamic slab
    // sets (same slab ids as the static sets, own ping-pong index) + scratch
    int* d_zlab = nullptr;         // measurement labels
    // measurements: one device block (d_zr .. d_zbin point into it, zblk_layout)
    // filled by ONE copy from a pinned host ring, so phd_set_measurements never
    // waits for the device (a slot is reused PHD_ZRING calls later, after its event)
    unsigned char* d_zblk = nullptr;
    // the previous scan's raw rows (zr | zb | zok, zblk_layout) for the step's
    // births (CPHD: births through the prediction from the previous scan)
    unsigned char* d_zprev = nullptr;
    int M_prev = 0, Mv_prev = 0;
    bool have_prev = false;
    int z_sets = 0;               // phd_set_measurements calls so far
    int step_births_req = -1;     // -1: with the filter type (CPHD on), 0 off, 1 on (phd_set_step_births)
    float* d_births = nullptr;    // the step's birth slabs, nmax x 7 x map_capacity (written by the classify)
    int births_now = 0;           // the next launch_update places this many births per particle (0: none)
    const float *births_zr = nullptr, *births_zb = nullptr;  // ... from these rows
    const int* births_zvi = nullptr;
    unsigned char* h_zring = nullptr;
    hipEvent_t ev_zring[4] = {};
    bool zring_used[4] = {};
    int zring_next = 0;
    bool dyn = false;
    int dcap = 0;
    int dcur = 0;
    float* d_dmap[2] = {nullptr, nullptr};
    int* d_dsize[2] = {nullptr, nullptr};
    float* d_mx_ekf = nullptr;
    float* d_mx_cand = nullptr;
    size_t mx_lds = 0;
};

static int set_device(phd_ctx* c) {
    HIPCHK(hipSetDevice(c->device));
    return PHD_OK;
}

static int launch_predict_dynamic(phd_ctx* ctx);

/* Normalise + nEff + decision + stratified parents of n log-weights (in place)
 * on ceil(n/1024) workgroups: k_rs_max, k_rs_sum, k_rs_cdf, k_rs_search (the
 * multi-block form of k_normalize_resample, same results bit for bit).  out:
 * [0] lse, [1] nEff, [2] decision, [4] decisions counter; parents written only
 * when the decision is 1.  With `remap`, k_rs_search also writes the remapped
 * poses / slab references of its strata into the spare arrays (the identity
 * without a resample) and the new log-weight.  Stream-ordered, no host
 * synchronisation. */
/* CPHD cardinality coefficients (allocated with the first CPHD use): one row
 * per slab, written by the update of the particle whose posterior slab it is. */
static int ensure_cn(phd_ctx* c) {
    if (!(c->cfg_set && c->cfg.filterType == PHD_FILTER_CPHD) || c->d_cn_coef) return PHD_OK;
    HIPCHK(hipMalloc((void**)&c->d_cn_coef, (size_t)c->nmax * c->cn_stride * sizeof(double)));
    return PHD_OK;
}

/* cardinality doubles carried by a migration record (0 unless CPHD) */
static int rec_cn_stride(const phd_ctx* c) {
    return (c->cfg_set && c->cfg.filterType == PHD_FILTER_CPHD) ? c->cn_stride : 0;
}

/* migration slab set X (+ its cardinality rows), allocated on first receive */
static int ensure_x(phd_ctx* c) {
    if (!c->d_map_x) {
        HIPCHK(hipMalloc((void**)&c->d_map_x, (size_t)c->n * 7 * c->cap.map_capacity * sizeof(float)));
        HIPCHK(hipMalloc((void**)&c->d_size_x, c->n * sizeof(int)));
        HIPCHK(hipMemsetAsync(c->d_size_x, 0, c->n * sizeof(int), c->stream));
    }
    if (rec_cn_stride(c) && !c->d_cn_x)
        HIPCHK(hipMalloc((void**)&c->d_cn_x, (size_t)c->n * c->cn_stride * sizeof(double)));
    return ensure_cn(c);
}

/* chunk partials + chunk-relative CDF of a chunked resample over n entries */
struct RsParts {
    unsigned long long* cdf_rel;
    double *part_sum, *part_s2;
    unsigned long long *part_tot, *part_key;
    float* part_max;
};
static int rs_parts(phd_ctx* ctx, int n, RsParts& P) {
    const int B = (n + RS_THREADS - 1) / RS_THREADS;
    if (B > RS_MAX_CHUNKS) return fail(PHD_E_ARG, "more than 2^20 log-weights in a chunked resample");
    const size_t need = (size_t)B * (sizeof(float) + 2 * sizeof(double) + 2 * sizeof(unsigned long long)) + 64 +
                        (size_t)n * sizeof(unsigned long long);
    if (ctx->rsx_bytes < need) {
        if (ctx->d_rsx) hipFree(ctx->d_rsx);
        ctx->d_rsx = nullptr;
        ctx->rsx_bytes = 0;
        HIPCHK(hipMalloc((void**)&ctx->d_rsx, need));
        ctx->rsx_bytes = need;
    }
    P.cdf_rel = (unsigned long long*)ctx->d_rsx;
    P.part_sum = (double*)(P.cdf_rel + n);
    P.part_s2 = P.part_sum + B;
    P.part_tot = (unsigned long long*)(P.part_s2 + B);
    P.part_key = P.part_tot + B;
    P.part_max = (float*)(P.part_key + B);
    return PHD_OK;
}

/* the in-launch hand-off words of k_shard_plan / k_rs_step: zeroed once, every
 * launch leaves them zero */
static int ensure_sync(phd_ctx* ctx) {
    if (!ctx->d_plan_sync) {
        HIPCHK(hipMalloc((void**)&ctx->d_plan_sync, 64));
        HIPCHK(hipMemsetAsync(ctx->d_plan_sync, 0, 64, ctx->stream));
    }
    return PHD_OK;
}

static int launch_rs_chunks(phd_ctx* ctx, float* w, int n, float* out, uint64_t seed, uint64_t step, int* parents,
                            bool remap = false, float new_logw = 0.f, bool fused_max = false,
                            unsigned* beyond = nullptr) {
    const int B = (n + RS_THREADS - 1) / RS_THREADS;
    RsParts P;
    int rc = rs_parts(ctx, n, P);
    if (rc) return rc;
    unsigned long long* cdf_rel = P.cdf_rel;
    double* part_sum = P.part_sum;
    double* part_s2 = P.part_s2;
    unsigned long long* part_tot = P.part_tot;
    unsigned long long* part_key = P.part_key;
    float* part_max = P.part_max;
    const int has_meas = ctx->M > 0 ? 1 : 0;
    // fused (phd_step, up to 16 chunks): one k_rs_sumcdf launch (every block
    // takes the max and all chunk sums itself), the normalised weights out of
    // place in d_tmp_logw until k_rs_search moves them
    const bool fused = fused_max && remap && B <= 16;
    if (fused) {  // one launch: k_rs_step (<= 16 workgroups, always resident at once)
        if (ensure_sync(ctx)) return PHD_E_HIP;
        RsStepArgs a{};
        a.w = w;
        a.w_out = ctx->d_tmp_logw;
        a.N = n;
        a.B = B;
        a.has_meas = has_meas;
        a.resample_thresh = ctx->cfg.resampleThresh;
        a.new_logw = new_logw;
        a.seed = seed;
        a.step = step;
        a.part_s2 = part_s2;
        a.cdf_rel = cdf_rel;
        a.part_tot = part_tot;
        a.part_key = part_key;
        a.sync = ctx->d_plan_sync;
        a.out = out;
        a.parents = parents;
        a.pose = ctx->d_pose;
        a.src = ctx->d_src;
        a.new_pose = ctx->d_tmp_pose;
        a.new_src = ctx->d_tmp_src;
        a.logw = w;
        a.err = ctx->d_err;
        if (ctx->rs_ov.armed) {  // (PHD_RS_OVERLAP) the update chain launches it beside part C
            a.src = nullptr;      // the update resets the slab references to the identity
            ctx->rs_ov.a = a;
            ctx->rs_ov.B = B;
            return PHD_OK;
        }
        hipLaunchKernelGGL(k_rs_step, dim3(B), dim3(RS_THREADS), 0, ctx->stream, a);
        HIPCHK(hipGetLastError());
        return PHD_OK;
    } else {
        hipLaunchKernelGGL(k_rs_max, dim3(B), dim3(RS_THREADS), 0, ctx->stream, (const float*)w, n, part_max);
        hipLaunchKernelGGL(k_rs_sum, dim3(B), dim3(RS_THREADS), 0, ctx->stream, (const float*)w, n,
                           (const float*)part_max, B, part_sum, 0);
        hipLaunchKernelGGL(k_rs_cdf, dim3(B), dim3(RS_THREADS), 0, ctx->stream, w, n, (const float*)part_max,
                           (const double*)part_sum, B, part_s2, cdf_rel, part_tot, part_key, out);
    }
    hipLaunchKernelGGL(k_rs_search, dim3(B), dim3(RS_THREADS), 0, ctx->stream, n, B, (const double*)part_s2,
                       (const unsigned long long*)part_tot, (const unsigned long long*)part_key,
                       (const unsigned long long*)cdf_rel, ctx->cfg.resampleThresh, has_meas, seed, step, parents,
                       out, remap ? (const phd_pose*)ctx->d_pose : nullptr, (const int*)ctx->d_src, ctx->d_tmp_pose,
                       ctx->d_tmp_src, w, new_logw, fused ? (const float*)ctx->d_tmp_logw : nullptr, beyond);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

extern "C" {

const char* phd_version(void) { return "phdslam-mi355x 0.1 (gfx950)"; }
const char* phd_last_error(void) { return g_last_error.c_str(); }

int phd_device_count(int* count) {
    if (!count) return fail(PHD_E_ARG, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    return PHD_OK;
}

/* the measurement block: zr | zb | zok | zvi (the valid measurements' indices
 * in order) | zlab (256 each) | zs (256 float4) | zbin; [zr, zlab) is what the
 * step's births read (kept for the previous scan) */
#define PHD_ZRING 4

/* Events that only order work on this device (the overlap's cross-stream
 * hand-offs) or only time it: recorded without the system-scope fence, which
 * writes back and invalidates the caches at every record and costs the stream
 * a gap of several microseconds.  (The host reads the sharded plan's counts
 * after polling the sequence word the plan stores last with a system-scope
 * release: no event there either.) */
#ifndef PHD_EV_DEVICE_SCOPE
#define PHD_EV_DEVICE_SCOPE 1
#endif
static constexpr unsigned kEvOrder = hipEventDisableTiming | (PHD_EV_DEVICE_SCOPE ? hipEventDisableSystemFence : 0u);
#ifndef PHD_FUSE_PREDICT_ALL
#define PHD_FUSE_PREDICT_ALL 0 /* 1: CPHD part A runs the predict at any number of workgroup rounds */
#endif
#ifndef PHD_TIMING_EVENTS
#define PHD_TIMING_EVENTS 1 /* 0: a diagnostic build that never records the update timing events */
#endif
static constexpr unsigned kEvTime = PHD_EV_DEVICE_SCOPE ? hipEventDisableSystemFence : hipEventDefault;
struct ZBlk {
    size_t zr, zb, zok, zvi, zlab, zs, zbin, bytes;
};
static ZBlk zblk_layout() {
    ZBlk L;
    L.zr = 0;
    L.zb = L.zr + 256 * sizeof(float);
    L.zok = L.zb + 256 * sizeof(float);
    L.zvi = L.zok + 256 * sizeof(int);
    L.zlab = L.zvi + 256 * sizeof(int);
    L.zs = L.zlab + 256 * sizeof(int);
    L.zbin = L.zs + 256 * sizeof(float4);
    L.bytes = L.zbin + PHD_ZBINS * sizeof(unsigned short);
    return L;
}

static int ctx_free(phd_ctx* c) {
    if (!c) return PHD_OK;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->d_zprev) hipFree(c->d_zprev);
    if (c->d_births) hipFree(c->d_births);
    void* ptrs[] = {c->d_map[0], c->d_map[1], c->d_size[0], c->d_size[1], c->d_map_x, c->d_size_x, c->d_src,
                    c->d_pose, c->d_logw, c->d_tmp_pose, c->d_tmp_src, c->d_tmp_logw, c->d_pose_prior, c->d_logw_prior,
                    c->d_delta, c->d_status, c->d_err, c->d_zblk, c->d_noise_a, c->d_noise_cv,
                    c->d_cdf, c->d_idx, c->d_u, c->d_out, c->d_cn, c->d_cdf_g, c->d_mig, c->d_stamps, c->d_cn_coef, c->d_cn_x, c->d_hand, c->d_lfact,
                    c->d_rsx, c->d_plan_sync, c->d_dmap[0], c->d_dmap[1], c->d_dsize[0], c->d_dsize[1], c->d_mx_ekf,
                    c->d_mx_cand};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (c->eap) eap_free(c->eap);
    if (c->h_mig) hipHostFree(c->h_mig);
    if (c->h_zring) hipHostFree(c->h_zring);
    for (auto e : c->ev_zring)
        if (e) hipEventDestroy(e);
    if (c->d_pend) hipFree(c->d_pend);
    if (c->ev_terms) hipEventDestroy(c->ev_terms);
    if (c->ev_logw) hipEventDestroy(c->ev_logw);
    if (c->ev_plan) hipEventDestroy(c->ev_plan);
    if (c->ev_rs) hipEventDestroy(c->ev_rs);
    if (c->aux) hipStreamDestroy(c->aux);
    for (auto e : c->ev_a) hipEventDestroy(e);
    for (auto e : c->ev_b) hipEventDestroy(e);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return PHD_OK;
}

__global__ void k_iota(int* a, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = i;
}

/* The workgroup update kernel of nt threads: part 0 the fused PHD update,
 * 1 / 2 part A / part C of the split update (CPHD: always split, with
 * k_cphd_terms between the parts; PHD: split when it pays, update_form). */
static const void* update_kernel(int nt, int cphd, int part) {
    const void* k[2][3][3] = {
        {{(const void*)k_update_fused_256, (const void*)k_update_fused_512, (const void*)k_update_fused_1024},
         {(const void*)k_update_phd_a_256, (const void*)k_update_phd_a_512, (const void*)k_update_phd_a_1024},
         {(const void*)k_update_phd_c_256, (const void*)k_update_phd_c_512, (const void*)k_update_phd_c_1024}},
        {{nullptr, nullptr, nullptr},
         {(const void*)k_update_cphd_a_256, (const void*)k_update_cphd_a_512, (const void*)k_update_cphd_a_1024},
         {(const void*)k_update_cphd_c_256, (const void*)k_update_cphd_c_512, (const void*)k_update_cphd_c_1024}}};
    return k[cphd ? 1 : 0][part][nt == 256 ? 0 : nt == 512 ? 1 : 2];
}

/* Threads per particle for the fused update.  The kernel is latency-bound, so
 * the step time is about (rounds of resident workgroups) x (per-workgroup
 * latency): residency from hipOccupancyMaxActiveBlocksPerMultiprocessor (LDS
 * layout, VGPRs, allocation granularity), relative latency measured at
 * config 3 (256 threads 1.25, 512 threads 1.0, 1024 threads ~0.85). */
/* workgroups per CU of `kernel` with `lds` bytes: the LDS bound (160 KiB /
 * the layout) within the VGPR bound; hipOccupancyMaxActiveBlocksPerMultiprocessor
 * under-reports the LDS bound here (it gave 5 where 6 workgroups of 27 KB run) */
/* LDS allocation granularity per workgroup (bytes) of the occupancy model:
 * measured on gfx950 (part C's residency timeline, stamps builds, 256 CUs): a
 * 27 120 B workgroup holds a CU to 5 (1 280 resident), a 26 864 B one to 6
 * (1 536) — consistent with 1 280-byte granules of the 160 KiB, not with the
 * 128 B this model assumed before round 5 (which had grown config 3's and 4's
 * edge pools to 27 248 B: 5 per CU, not the 6 the bench line reported) */
#ifndef PHD_LDS_GRAN
#define PHD_LDS_GRAN 1280
#endif
static int blocks_per_cu(const void* kernel, int nt, size_t lds) {
    int vblocks = 0;  // the VGPR / wave bound alone: the runtime's answer without LDS
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&vblocks, kernel, nt, 0) != hipSuccess || vblocks <= 0)
        vblocks = 32 / (nt / 64);
    const size_t g = PHD_LDS_GRAN;
    return (int)std::min<long>((160 * 1024) / (long)((lds + g - 1) / g * g), vblocks);
}

static int configure_update_launch(phd_ctx* c, int req) {
    const phd_capacity& cap = c->cap;
    const int cphd = c->cfg_set && c->cfg.filterType == PHD_FILTER_CPHD ? 1 : 0;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    if (ncu <= 0) ncu = 1;
    int best = 0, best_blocks = 0, best_split = 0;
    double best_cost = 1e300;
    size_t best_lds = 0;
    int best_ep = c->epool;
    // forms: the fused PHD update (one launch), or split into part A and part C
    // (CPHD always: its terms sit between the parts)
    for (int split = cphd ? 1 : 0; split <= 1; split++) {
        if (!cphd && c->upd_form_req && split != c->upd_form_req - 1) continue;
        for (int nt = UPD_THREADS_MIN; nt <= UPD_THREADS_MAX; nt *= 2) {
            const int pc = split ? 2 : 0;  // the launch whose layout holds the merge
            // edge pool: the minimal one, grown while the workgroups per CU stay the same
            auto lds_of = [&](int e) {
                return upd_lds_layout(cap.map_capacity, cap.max_measurements, cap.candidate_capacity,
                                      cap.survivor_capacity, e, nt, cphd, pc)
                    .total;
            };
            const void* kc = update_kernel(nt, cphd, pc);
            // minimal edge pool: one edge per candidate (+16 for CPHD): the births
            // join the detected landmarks' clusters — config 4's shard overflowed a
            // pool of K / 2 + 32 in 48 % of its particle-updates (serial greedy), and
            // config 3 with the step's births has up to 795 edges of 807 candidates
            // (K = 832: a pool of 800 fell back to the serial greedy in 3 of 1.2 M
            // particle-updates, 848 in none)
            int ep = c->epool_req > 0 ? c->epool_req : cap.candidate_capacity + (cphd ? 16 : 0);
            const size_t l0 = lds_of(ep);
            if (l0 > 160 * 1024) continue;
            const int b0 = blocks_per_cu(kc, nt, l0);
            while (!c->epool_req && ep + 16 <= upd_epool(cap.candidate_capacity) &&
                   blocks_per_cu(kc, nt, lds_of(ep + 16)) >= b0)
                ep += 16;
            const size_t lds = lds_of(ep);
            const int blocks = blocks_per_cu(kc, nt, lds);
            if (blocks < 1) continue;
            // per-workgroup latency relative to 512 threads (config 3 measurements:
            // 256 threads 1.25, 512 1.0, 1024 ~0.85); part A ~0.4 and part C ~0.6
            // of the whole update (config 3: A 66 us, C 160 us minus the CPHD-only work)
            const double lat = nt == 256 ? 1.25 : nt == 512 ? 1.0 : 0.85;
            const long resident = (long)blocks * ncu;
            double cost = (double)((c->n + resident - 1) / resident) * lat;
            if (split) {
                const size_t la = upd_lds_layout(cap.map_capacity, cap.max_measurements, cap.candidate_capacity,
                                                 cap.survivor_capacity, ep, nt, cphd, 1)
                                      .total;
                const int ba = blocks_per_cu(update_kernel(nt, cphd, 1), nt, la);
                if (ba < 1) continue;
                const long ra = (long)ba * ncu;
                cost = 0.6 * cost + 0.4 * (double)((c->n + ra - 1) / ra) * lat;
            }
            if (req ? (nt == req && (best == 0 || cost < best_cost)) : cost < best_cost) {
                best = nt;
                best_cost = cost;
                best_blocks = blocks;
                best_lds = lds;
                best_ep = ep;
                best_split = split;
            }
        }
    }
    if (!best) {
        const size_t need = upd_lds_layout(cap.map_capacity, cap.max_measurements, cap.candidate_capacity,
                                           cap.survivor_capacity, c->epool, UPD_THREADS_MIN, cphd, cphd ? 2 : 0)
                                .total;
        return fail(PHD_E_CAPACITY, "capacities need " + std::to_string(need) + " B of LDS (> 160 KiB)");
    }
    c->upd_threads = best;
    c->upd_cphd = cphd;
    c->upd_split = best_split;
    c->upd_threads_req = req;
    c->upd_lds = best_lds;
    c->upd_lds_a = best_split ? upd_lds_layout(cap.map_capacity, cap.max_measurements, cap.candidate_capacity,
                                               cap.survivor_capacity, best_ep, best, cphd, 1)
                                    .total
                              : 0;
    c->epool = best_ep;
    c->upd_resident = best_blocks * ncu;
    c->upd_resident_a =
        best_split ? blocks_per_cu(update_kernel(best, cphd, 1), best, c->upd_lds_a) * ncu : 0;
    // the fused-predict forms (CPHD: part A; PHD: the fused update) carry the
    // predict's registers: phd_step fuses the predict only when every particle's
    // workgroup of THAT launch is resident at once
    {
        const void* kp = nullptr;
        size_t lp = 0;
        if (cphd && best <= 512) {
            kp = best == 256 ? (const void*)k_update_cphd_a_p256 : (const void*)k_update_cphd_a_p512;
            lp = c->upd_lds_a;
        } else if (!cphd && !best_split && best <= 512) {
            kp = best == 256 ? (const void*)k_update_fused_p256 : (const void*)k_update_fused_p512;
            lp = c->upd_lds;
        }
        c->upd_resident_p = kp ? blocks_per_cu(kp, best, lp) * ncu : 0;
    }
    return PHD_OK;
}

int phd_ctx_create(phd_ctx** out, int device, int n_particles, const phd_capacity* capin) {
    if (!out || n_particles <= 0) return fail(PHD_E_ARG, "bad arguments to phd_ctx_create");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PHD_E_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(PHD_E_ARG, "device index out of range");
    phd_ctx* c = new phd_ctx();
    c->device = device;
    c->n = n_particles;
    c->n_base = n_particles;
    phd_capacity cap = capin ? *capin : phd_capacity{};
    if (cap.max_particles < n_particles) cap.max_particles = n_particles;
    c->nmax = cap.max_particles;
    if (cap.map_capacity <= 0) cap.map_capacity = 1024;
    if (cap.max_measurements <= 0) cap.max_measurements = 256;
    if (cap.max_measurements > 256) cap.max_measurements = 256;
    if (cap.candidate_capacity <= 0) cap.candidate_capacity = cap.map_capacity + 4 * cap.max_measurements;
    if (cap.survivor_capacity <= 0) cap.survivor_capacity = 4 * cap.max_measurements;
    if (cap.map_capacity > 32767 || cap.candidate_capacity > 16383) {
        delete c;
        return fail(PHD_E_ARG, "map_capacity must be <= 32767 and candidate_capacity <= 16383");
    }
    cap.survivor_capacity = (cap.survivor_capacity + 3) & ~3;  // rank sort reads keys 4 at a time
    c->cap = cap;
    c->epool = upd_epool(cap.candidate_capacity);
    c->cn_stride = cap.max_measurements + 8;
    int rc = set_device(c);
    if (rc) {
        delete c;
        return rc;
    }
#define ALLOC(ptr, bytes)                                                              \
    do {                                                                               \
        hipError_t _e = hipMalloc((void**)&(ptr), (bytes));                           \
        if (_e != hipSuccess) {                                                        \
            ctx_free(c);                                                               \
            return fail(PHD_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(_e)); \
        }                                                                              \
    } while (0)
    const size_t N = (size_t)c->nmax;
    const size_t slab = N * 7 * (size_t)cap.map_capacity * sizeof(float);
    for (int b = 0; b < 2; b++) {
        ALLOC(c->d_map[b], slab);
        ALLOC(c->d_size[b], N * sizeof(int));
    }
    ALLOC(c->d_src, N * sizeof(int));
    ALLOC(c->d_pose, N * sizeof(phd_pose));
    ALLOC(c->d_logw, N * sizeof(float));
    ALLOC(c->d_tmp_pose, N * sizeof(phd_pose));
    ALLOC(c->d_tmp_src, N * sizeof(int));
    ALLOC(c->d_tmp_logw, N * sizeof(float));
    ALLOC(c->d_delta, N * sizeof(float));
    ALLOC(c->d_status, N * sizeof(int));
    ALLOC(c->d_err, 4 * sizeof(int));  // error bits, serial-merge fallbacks, pair-list overflow walks, error statuses
    {
        const ZBlk Z = zblk_layout();
        ALLOC(c->d_zblk, Z.bytes);
        c->d_zr = (float*)(c->d_zblk + Z.zr);
        c->d_zb = (float*)(c->d_zblk + Z.zb);
        c->d_zok = (int*)(c->d_zblk + Z.zok);
        c->d_zlab = (int*)(c->d_zblk + Z.zlab);
        c->d_zs = (float4*)(c->d_zblk + Z.zs);
        c->d_zbin = (unsigned short*)(c->d_zblk + Z.zbin);
    }
    ALLOC(c->d_noise_a, N * sizeof(phd_ackerman_noise));
    ALLOC(c->d_noise_cv, N * sizeof(phd_cv_noise));
    ALLOC(c->d_cdf, N * sizeof(unsigned long long));
    ALLOC(c->d_idx, N * sizeof(int));
    ALLOC(c->d_u, N * sizeof(double));
    ALLOC(c->d_out, 64 * sizeof(float));
    ALLOC(c->d_cn, N * sizeof(float));
#undef ALLOC
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        ctx_free(c);
        return fail(PHD_E_HIP, "hipStreamCreate failed");
    }
    c->own_stream = true;
    hipMemsetAsync(c->d_size[0], 0, N * sizeof(int), c->stream);
    hipMemsetAsync(c->d_size[1], 0, N * sizeof(int), c->stream);
    hipMemsetAsync(c->d_err, 0, 4 * sizeof(int), c->stream);
    hipMemsetAsync(c->d_out, 0, 64 * sizeof(float), c->stream);
    hipMemsetAsync(c->d_logw, 0, N * sizeof(float), c->stream);
    hipMemsetAsync(c->d_pose, 0, N * sizeof(phd_pose), c->stream);
    hipLaunchKernelGGL(k_iota, dim3((c->nmax + 255) / 256), dim3(256), 0, c->stream, c->d_src, c->nmax);
    for (int nt = UPD_THREADS_MIN; nt <= UPD_THREADS_MAX; nt *= 2)
        for (int cp = 0; cp < 2; cp++)
            for (int part = cp; part < 3; part++)
                hipFuncSetAttribute(update_kernel(nt, cp, part), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024);
    hipFuncSetAttribute((const void*)k_update_cphd_a_p256, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_update_cphd_a_p512, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_update_fused_p256, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_update_fused_p512, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_resample, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * RS_LDS_MAX);
    hipFuncSetAttribute((const void*)k_normalize_resample, hipFuncAttributeMaxDynamicSharedMemorySize,
                        8 * RS_LDS_MAX);
    // a limit a kernel cannot take only caps its launches (checked at launch):
    // do not leave it as the runtime's last error for the next launch check
    (void)hipGetLastError();
    if (configure_update_launch(c, 0) != PHD_OK) {
        const std::string msg = g_last_error;
        ctx_free(c);
        return fail(PHD_E_CAPACITY, msg);
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
        ctx_free(c);
        return fail(PHD_E_HIP, "initialisation failed");
    }
    *out = c;
    return PHD_OK;
}

int phd_ctx_destroy(phd_ctx* ctx) { return ctx_free(ctx); }

int phd_ctx_info(const phd_ctx* ctx, int* n_particles, phd_capacity* cap) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (n_particles) *n_particles = ctx->n;
    if (cap) *cap = ctx->cap;
    return PHD_OK;
}

int phd_set_config(phd_ctx* ctx, const phd_slam_config* cfg) {
    if (!ctx || !cfg) return fail(PHD_E_ARG, "null argument");
    ctx->cfg = *cfg;
    ctx->cfg_set = true;
    const int cphd = cfg->filterType == PHD_FILTER_CPHD ? 1 : 0;
    if (cphd != ctx->upd_cphd) {
        // the CPHD kernels have their own LDS layout and occupancy
        if (set_device(ctx)) return PHD_E_HIP;
        int rc = configure_update_launch(ctx, ctx->upd_threads_req);
        if (rc) return rc;
    }
    return PHD_OK;
}

int phd_set_stream(phd_ctx* ctx, void* s) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (s) {
        if (ctx->own_stream && ctx->stream) {
            hipStreamSynchronize(ctx->stream);
            hipStreamDestroy(ctx->stream);
        }
        ctx->stream = s == PHD_STREAM_NULL ? (hipStream_t)0 : (hipStream_t)s;
        ctx->own_stream = false;
    }
    return PHD_OK;
}

void* phd_get_stream(phd_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int phd_synchronize(phd_ctx* ctx) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_set_seed(phd_ctx* ctx, uint64_t seed) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    ctx->seed = seed;
    return PHD_OK;
}

int phd_load_particles(phd_ctx* ctx, int n, const phd_pose* poses, const float* logw, const phd_gaussian2d* maps,
                       const int* offsets) {
    if (!ctx || n <= 0 || n > ctx->nmax || !poses || !logw || !offsets)
        return fail(PHD_E_ARG, "bad arguments to phd_load_particles");
    if (set_device(ctx)) return PHD_E_HIP;
    ctx->n = n;  // the live count (n_particles, or up to capacity.max_particles)
    const int cap = ctx->cap.map_capacity;
    std::vector<float> slab((size_t)n * 7 * cap, 0.f);
    std::vector<int> sizes(n);
    for (int p = 0; p < n; p++) {
        const int sz = offsets[p + 1] - offsets[p];
        if (sz < 0 || sz > cap) return fail(PHD_E_CAPACITY, "particle map exceeds map_capacity");
        sizes[p] = sz;
        float* s = slab.data() + (size_t)p * 7 * cap;
        for (int k = 0; k < sz; k++) {
            const phd_gaussian2d& g = maps[offsets[p] + k];
            s[k] = g.weight;
            s[1 * cap + k] = g.mean[0];
            s[2 * cap + k] = g.mean[1];
            s[3 * cap + k] = g.cov[0];
            s[4 * cap + k] = g.cov[1];
            s[5 * cap + k] = g.cov[2];
            s[6 * cap + k] = g.cov[3];
        }
    }
    ctx->cur = 0;
    ctx->replay = false;
    HIPCHK(hipMemcpyAsync(ctx->d_map[0], slab.data(), slab.size() * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_size[0], sizes.data(), n * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_pose, poses, n * sizeof(phd_pose), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_logw, logw, n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_iota, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_src, n);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_set_poses(phd_ctx* ctx, int n, const phd_pose* poses) {
    if (!ctx || n != ctx->n || !poses) return fail(PHD_E_ARG, "bad arguments to phd_set_poses");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipMemcpyAsync(ctx->d_pose, poses, n * sizeof(phd_pose), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

/* Host image of the current state: slab reference table + the sets it references. */
struct HostState {
    std::vector<int> src, size_cur, size_x;
    std::vector<float> map_cur, map_x;
};

static int fetch_state(phd_ctx* ctx, HostState& h, bool with_maps) {
    // slabs of the current set: a resample after n_predict_particles > 1 may
    // leave live particles referencing slabs beyond the live count
    const int n = ctx->n, ns = ctx->nmax, cap = ctx->cap.map_capacity;
    h.src.resize(n);
    h.size_cur.resize(ns);
    HIPCHK(hipMemcpyAsync(h.src.data(), ctx->d_src, n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(h.size_cur.data(), ctx->d_size[ctx->cur], ns * sizeof(int), hipMemcpyDeviceToHost,
                          ctx->stream));
    if (ctx->d_size_x) {
        h.size_x.resize(n);
        HIPCHK(hipMemcpyAsync(h.size_x.data(), ctx->d_size_x, n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    }
    if (with_maps) {
        h.map_cur.resize((size_t)ns * 7 * cap);
        HIPCHK(hipMemcpyAsync(h.map_cur.data(), ctx->d_map[ctx->cur], h.map_cur.size() * sizeof(float),
                              hipMemcpyDeviceToHost, ctx->stream));
        if (ctx->d_map_x) {
            h.map_x.resize((size_t)n * 7 * cap);
            HIPCHK(hipMemcpyAsync(h.map_x.data(), ctx->d_map_x, h.map_x.size() * sizeof(float), hipMemcpyDeviceToHost,
                                  ctx->stream));
        }
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

static inline int host_size(const HostState& h, int p) {
    const int r = h.src[p];
    return (r & PHD_SLAB_X) ? h.size_x[r & PHD_SLAB_MASK] : h.size_cur[r];
}

int phd_export_particles(phd_ctx* ctx, int n, phd_pose* poses, float* logw, int* sizes) {
    if (!ctx || n != ctx->n) return fail(PHD_E_ARG, "bad arguments to phd_export_particles");
    if (set_device(ctx)) return PHD_E_HIP;
    if (poses) HIPCHK(hipMemcpyAsync(poses, ctx->d_pose, n * sizeof(phd_pose), hipMemcpyDeviceToHost, ctx->stream));
    if (logw) HIPCHK(hipMemcpyAsync(logw, ctx->d_logw, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HostState h;
    int rc = fetch_state(ctx, h, false);
    if (rc) return rc;
    if (sizes)
        for (int p = 0; p < n; p++) sizes[p] = host_size(h, p);
    return PHD_OK;
}

int phd_export_maps(phd_ctx* ctx, int n, const int* offsets, phd_gaussian2d* maps) {
    if (!ctx || n != ctx->n || !offsets || !maps) return fail(PHD_E_ARG, "bad arguments to phd_export_maps");
    if (set_device(ctx)) return PHD_E_HIP;
    const int cap = ctx->cap.map_capacity;
    HostState h;
    int rc = fetch_state(ctx, h, true);
    if (rc) return rc;
    for (int p = 0; p < n; p++) {
        const int r = h.src[p];
        const bool in_x = (r & PHD_SLAB_X) != 0;
        const float* s = (in_x ? h.map_x.data() : h.map_cur.data()) + (size_t)(r & PHD_SLAB_MASK) * 7 * cap;
        const int sz = offsets[p + 1] - offsets[p];
        if (sz != host_size(h, p)) return fail(PHD_E_ARG, "offsets do not match the current map sizes");
        for (int k = 0; k < sz; k++) {
            phd_gaussian2d& g = maps[offsets[p] + k];
            g.weight = s[k];
            g.mean[0] = s[1 * cap + k];
            g.mean[1] = s[2 * cap + k];
            g.cov[0] = s[3 * cap + k];
            g.cov[1] = s[4 * cap + k];
            g.cov[2] = s[5 * cap + k];
            g.cov[3] = s[6 * cap + k];
        }
    }
    return PHD_OK;
}

/* ---- mixed static + dynamic feature model (feature_model 2) ---- */
int phd_enable_dynamic(phd_ctx* ctx, int dyn_capacity) {
    if (!ctx || dyn_capacity <= 0) return fail(PHD_E_ARG, "bad arguments to phd_enable_dynamic");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ctx->dyn && ctx->dcap == dyn_capacity) return PHD_OK;
    for (int k = 0; k < 2; k++) {
        if (ctx->d_dmap[k]) hipFree(ctx->d_dmap[k]);
        if (ctx->d_dsize[k]) hipFree(ctx->d_dsize[k]);
        ctx->d_dmap[k] = nullptr;
        ctx->d_dsize[k] = nullptr;
    }
    if (ctx->d_mx_ekf) hipFree(ctx->d_mx_ekf);
    if (ctx->d_mx_cand) hipFree(ctx->d_mx_cand);
    ctx->d_mx_ekf = ctx->d_mx_cand = nullptr;
    const size_t ns = (size_t)ctx->nmax;
    for (int k = 0; k < 2; k++) {
        HIPCHK(hipMalloc((void**)&ctx->d_dmap[k], ns * PHD_DYN_FIELDS * dyn_capacity * sizeof(float)));
        HIPCHK(hipMalloc((void**)&ctx->d_dsize[k], ns * sizeof(int)));
        HIPCHK(hipMemsetAsync(ctx->d_dsize[k], 0, ns * sizeof(int), ctx->stream));
    }
    HIPCHK(hipMalloc((void**)&ctx->d_mx_ekf, ns * mixed_ekf_floats(ctx->cap.map_capacity, dyn_capacity) * sizeof(float)));
    HIPCHK(hipMalloc((void**)&ctx->d_mx_cand, ns * mixed_cand_floats(ctx->cap.candidate_capacity) * sizeof(float)));
    HIPCHK(mixed_set_lds_limit());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->dyn = true;
    ctx->dcap = dyn_capacity;
    ctx->dcur = 0;
    return PHD_OK;
}

int phd_load_dynamic_maps(phd_ctx* ctx, int n, const phd_gaussian4d* maps, const int* offsets) {
    if (!ctx || n != ctx->n || !offsets || (offsets[n] > 0 && !maps))
        return fail(PHD_E_ARG, "bad arguments to phd_load_dynamic_maps");
    if (!ctx->dyn) return fail(PHD_E_ARG, "phd_enable_dynamic not called");
    if (set_device(ctx)) return PHD_E_HIP;
    // particle i must own slab i (as after phd_load_particles or an update)
    std::vector<int> src(n);
    HIPCHK(hipMemcpyAsync(src.data(), ctx->d_src, n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int p = 0; p < n; p++)
        if (src[p] != p)
            return fail(PHD_E_ARG, "phd_load_dynamic_maps: particles share slabs (load after phd_load_particles or an update)");
    const int dcap = ctx->dcap;
    std::vector<float> slab((size_t)n * PHD_DYN_FIELDS * dcap, 0.f);
    std::vector<int> sizes(n);
    for (int p = 0; p < n; p++) {
        const int sz = offsets[p + 1] - offsets[p];
        if (sz < 0 || sz > dcap) return fail(PHD_E_CAPACITY, "dynamic map exceeds the dynamic capacity");
        sizes[p] = sz;
        float* sl = slab.data() + (size_t)p * PHD_DYN_FIELDS * dcap;
        for (int k = 0; k < sz; k++) {
            const phd_gaussian4d& g = maps[offsets[p] + k];
            sl[k] = g.weight;
            for (int i = 0; i < 4; i++) sl[(1 + i) * dcap + k] = g.mean[i];
            for (int i = 0; i < 16; i++) sl[(5 + i) * dcap + k] = g.cov[i];
        }
    }
    HIPCHK(hipMemcpyAsync(ctx->d_dmap[ctx->dcur], slab.data(), slab.size() * sizeof(float), hipMemcpyHostToDevice,
                          ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_dsize[ctx->dcur], sizes.data(), n * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_dynamic_sizes(phd_ctx* ctx, int* sizes) {
    if (!ctx || !sizes) return fail(PHD_E_ARG, "null argument");
    if (!ctx->dyn) return fail(PHD_E_ARG, "phd_enable_dynamic not called");
    if (set_device(ctx)) return PHD_E_HIP;
    const int n = ctx->n;
    std::vector<int> src(n), dsz(ctx->nmax);
    HIPCHK(hipMemcpyAsync(src.data(), ctx->d_src, n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(dsz.data(), ctx->d_dsize[ctx->dcur], ctx->nmax * sizeof(int), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int p = 0; p < n; p++) sizes[p] = dsz[src[p] & PHD_SLAB_MASK];
    return PHD_OK;
}

int phd_export_dynamic_maps(phd_ctx* ctx, int n, const int* offsets, phd_gaussian4d* maps) {
    if (!ctx || n != ctx->n || !offsets || (offsets[n] > 0 && !maps))
        return fail(PHD_E_ARG, "bad arguments to phd_export_dynamic_maps");
    if (!ctx->dyn) return fail(PHD_E_ARG, "phd_enable_dynamic not called");
    if (set_device(ctx)) return PHD_E_HIP;
    const int dcap = ctx->dcap;
    std::vector<int> src(n), dsz(ctx->nmax);
    std::vector<float> all((size_t)ctx->nmax * PHD_DYN_FIELDS * dcap);
    HIPCHK(hipMemcpyAsync(src.data(), ctx->d_src, n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(dsz.data(), ctx->d_dsize[ctx->dcur], ctx->nmax * sizeof(int), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipMemcpyAsync(all.data(), ctx->d_dmap[ctx->dcur], all.size() * sizeof(float), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int p = 0; p < n; p++) {
        const int r = src[p] & PHD_SLAB_MASK;
        const int sz = offsets[p + 1] - offsets[p];
        if (sz != dsz[r]) return fail(PHD_E_ARG, "offsets do not match the current dynamic map sizes");
        const float* sl = all.data() + (size_t)r * PHD_DYN_FIELDS * dcap;
        for (int k = 0; k < sz; k++) {
            phd_gaussian4d& g = maps[offsets[p] + k];
            g.weight = sl[k];
            for (int i = 0; i < 4; i++) g.mean[i] = sl[(1 + i) * dcap + k];
            for (int i = 0; i < 16; i++) g.cov[i] = sl[(5 + i) * dcap + k];
        }
    }
    return PHD_OK;
}

int phd_predict_dynamic(phd_ctx* ctx) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (set_device(ctx)) return PHD_E_HIP;
    return launch_predict_dynamic(ctx);
}

int phd_slab_sizes(phd_ctx* ctx, int* sizes) {
    if (!ctx || !sizes) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipMemcpyAsync(sizes, ctx->d_size[ctx->cur], ctx->n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_set_replay(phd_ctx* ctx, int on) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    if (on) {
        if (ctx->cur != 0) return fail(PHD_E_ARG, "phd_set_replay must follow phd_load_particles");
        if (ctx->n != ctx->n_base) return fail(PHD_E_UNSUPPORTED, "replay mode needs n_particles live particles");
        if (!ctx->d_pose_prior) HIPCHK(hipMalloc((void**)&ctx->d_pose_prior, ctx->n * sizeof(phd_pose)));
        if (!ctx->d_logw_prior) HIPCHK(hipMalloc((void**)&ctx->d_logw_prior, ctx->n * sizeof(float)));
        HIPCHK(hipMemcpyAsync(ctx->d_pose_prior, ctx->d_pose, ctx->n * sizeof(phd_pose), hipMemcpyDeviceToDevice,
                              ctx->stream));
        HIPCHK(hipMemcpyAsync(ctx->d_logw_prior, ctx->d_logw, ctx->n * sizeof(float), hipMemcpyDeviceToDevice,
                              ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    ctx->replay = on != 0;
    return PHD_OK;
}

static PredictCfg predict_cfg(const phd_slam_config& c, int index_offset) {
    PredictCfg p;
    p.index_offset = index_offset;
    p.dt = c.dt;
    p.subdivide = c.subdividePredict > 0 ? c.subdividePredict : 1;
    p.l = c.l;
    p.h = c.h;
    p.a = c.a;
    p.b = c.b;
    p.stdAlpha = c.stdAlpha;
    p.stdEncoder = c.stdEncoder;
    p.ax = c.ax;
    p.ay = c.ay;
    p.ayaw = c.ayaw;
    return p;
}

static int check_predict(phd_ctx* ctx) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (ctx->cfg.nPredictParticles > 1 && ctx->replay)
        return fail(PHD_E_UNSUPPORTED, "n_predict_particles > 1 in replay mode");
    return set_device(ctx);
}

/* n_predict_particles > 1 (phdPredict, phdfilter.cu:1185-1238): every live
 * particle spawns npp children (pose, slab reference, weight - log npp) before
 * the predict kernel moves each child with its own noise draw.  The live count
 * grows by npp per predict, within capacity.max_particles. */
static int expand_particles(phd_ctx* ctx) {
    const int npp = ctx->cfg.nPredictParticles;
    if (npp <= 1) return PHD_OK;
    if ((long)ctx->n * npp > ctx->nmax)
        return fail(PHD_E_CAPACITY, "n_predict_particles: " + std::to_string((long)ctx->n * npp) +
                                        " live particles exceed capacity.max_particles (" +
                                        std::to_string(ctx->nmax) + ")");
    const int m = ctx->n * npp;
    const float log_npp = std::log((float)npp);  // safeLog(nPredictParticles) in float (phdfilter.cu:1214)
    hipLaunchKernelGGL(k_expand, dim3((m + 255) / 256), dim3(256), 0, ctx->stream, ctx->n, npp,
                       (const phd_pose*)ctx->d_pose, (const int*)ctx->d_src, (const float*)ctx->d_logw,
                       ctx->d_tmp_pose, ctx->d_tmp_src, ctx->d_tmp_logw, log_npp);
    HIPCHK(hipGetLastError());
    std::swap(ctx->d_pose, ctx->d_tmp_pose);
    std::swap(ctx->d_src, ctx->d_tmp_src);
    std::swap(ctx->d_logw, ctx->d_tmp_logw);
    ctx->src_fresh = false;  // (children reference their parent's slab)
    ctx->n = m;
    return PHD_OK;
}

/* the resample decision's mode argument: 0 no measurements, 1 measurements,
 * 2 forced — more than 5 x n_particles live particles (main.cpp:1286) */
static int rs_mode(const phd_ctx* ctx) {
    if ((long)ctx->n > 5L * ctx->n_base) return 2;
    return ctx->M > 0 ? 1 : 0;
}

/* predict of all particles, or of `count` slots listed on the device */
static int launch_predict(phd_ctx* ctx, phd_ackerman_control u, const void* noise, uint64_t step,
                          const int* slots, int count) {
    if (count <= 0) return PHD_OK;
    if (ctx->cfg.featureModel == PHD_FEATURE_MIXED) {  // predictMapMixed with every phdPredict (phdfilter.cu:1241-1242)
        if (slots) return fail(PHD_E_UNSUPPORTED, "feature_model 2: slot predicts (sharded step) are not supported");
        int rc = launch_predict_dynamic(ctx);
        if (rc) return rc;
    }
    const PredictCfg pc = predict_cfg(ctx->cfg, ctx->index_offset);
    const phd_pose* pp = ctx->replay ? ctx->d_pose_prior : nullptr;
    const float* lp = ctx->replay ? ctx->d_logw_prior : nullptr;
    if (ctx->cfg.motionType == PHD_MOTION_ACKERMAN)
        hipLaunchKernelGGL(k_predict_ackerman, dim3((count + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_pose,
                           count, u, (const phd_ackerman_noise*)noise, pc, ctx->seed, step, pp, lp, ctx->d_logw, slots);
    else
        hipLaunchKernelGGL(k_predict_cv, dim3((count + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_pose, count,
                           (const phd_cv_noise*)noise, pc, ctx->seed, step, pp, lp, ctx->d_logw, slots);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_predict_ackerman(phd_ctx* ctx, phd_ackerman_control u, const phd_ackerman_noise* noise, uint64_t step) {
    int rc = check_predict(ctx);
    if (rc) return rc;
    if (ctx->cfg.motionType != PHD_MOTION_ACKERMAN) return fail(PHD_E_ARG, "motion_type is not Ackerman");
    rc = expand_particles(ctx);
    if (rc) return rc;
    const int n = ctx->n;  // (noise: one entry per live particle after the expansion)
    const phd_ackerman_noise* dn = nullptr;
    if (noise) {
        HIPCHK(hipMemcpyAsync(ctx->d_noise_a, noise, n * sizeof(phd_ackerman_noise), hipMemcpyHostToDevice,
                              ctx->stream));
        dn = ctx->d_noise_a;
    }
    return launch_predict(ctx, u, dn, step, nullptr, n);
}

int phd_predict_cv(phd_ctx* ctx, const phd_cv_noise* noise, uint64_t step) {
    int rc = check_predict(ctx);
    if (rc) return rc;
    if (ctx->cfg.motionType == PHD_MOTION_ACKERMAN) return fail(PHD_E_ARG, "motion_type is Ackerman, not CV");
    rc = expand_particles(ctx);
    if (rc) return rc;
    const int n = ctx->n;  // (noise: one entry per live particle after the expansion)
    const phd_cv_noise* dn = nullptr;
    if (noise) {
        HIPCHK(hipMemcpyAsync(ctx->d_noise_cv, noise, n * sizeof(phd_cv_noise), hipMemcpyHostToDevice, ctx->stream));
        dn = ctx->d_noise_cv;
    }
    return launch_predict(ctx, phd_ackerman_control{0.f, 0.f}, dn, step, nullptr, n);
}

/* phdUpdateSynth's measurement upload (phdfilter.cu:3389-3400: clamp to 256,
 * cudaMemcpyToSymbol(Z)): the measurements, labels, and the bearing-sorted
 * valid ones with their 256-bin table for the banded pair walk, staged in a
 * pinned ring slot and sent as ONE stream-ordered copy.  No host wait: the slot
 * is reused PHD_ZRING calls later, after the event of its copy (long
 * complete); the device block is overwritten in stream order, after every
 * earlier launch that reads it. */
int phd_set_measurements(phd_ctx* ctx, const phd_measurement* z, int n_measure) {
    if (!ctx || n_measure < 0 || (n_measure > 0 && !z)) return fail(PHD_E_ARG, "bad arguments to phd_set_measurements");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (set_device(ctx)) return PHD_E_HIP;
    int M = std::min(n_measure, 256);  // phdfilter.cu:3390-3394
    if (M > ctx->cap.max_measurements) return fail(PHD_E_CAPACITY, "more measurements than max_measurements");
    const ZBlk Z = zblk_layout();
    if (!ctx->h_zring) {
        HIPCHK(hipHostMalloc((void**)&ctx->h_zring, PHD_ZRING * Z.bytes, hipHostMallocDefault));
        for (auto& e : ctx->ev_zring) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (ctx->z_sets > 0) {
        // the current scan becomes the previous one (the step's births, CPHD):
        // its raw rows, copied in stream order ahead of the new upload
        if (!ctx->d_zprev) HIPCHK(hipMalloc((void**)&ctx->d_zprev, Z.zlab));
        if (ctx->M > 0) HIPCHK(hipMemcpyAsync(ctx->d_zprev, ctx->d_zblk, Z.zlab, hipMemcpyDeviceToDevice, ctx->stream));
        ctx->M_prev = ctx->M;
        ctx->Mv_prev = ctx->Mv;
        ctx->have_prev = true;
    }
    ctx->z_sets++;
    const int slot = ctx->zring_next;
    ctx->zring_next = (slot + 1) % PHD_ZRING;
    if (ctx->zring_used[slot]) HIPCHK(hipEventSynchronize(ctx->ev_zring[slot]));  // the copy PHD_ZRING calls ago (done long since)
    unsigned char* h = ctx->h_zring + (size_t)slot * Z.bytes;
    float* zr = (float*)(h + Z.zr);
    float* zb = (float*)(h + Z.zb);
    int* zok = (int*)(h + Z.zok);
    int* zlab = (int*)(h + Z.zlab);
    int* zvi = (int*)(h + Z.zvi);
    float4* zs = (float4*)(h + Z.zs);
    unsigned short* zbin = (unsigned short*)(h + Z.zbin);
    int Mv = 0, zwide = 0;
    for (int m = 0; m < M; m++) {
        zr[m] = z[m].range;
        zb[m] = z[m].bearing;
        zok[m] = (z[m].label == PHD_MEAS_STATIC || !ctx->cfg.labeledMeasurements) ? 1 : 0;
        zlab[m] = z[m].label;
        if (!(std::fabs(zb[m]) < 3.f)) zwide = 1;
        if (!zok[m]) continue;
        zvi[Mv] = m;
        // bearing-sorted valid measurements for the banded pair loop (key = bearing wrapped to [-pi, pi))
        double key = std::fmod((double)zb[m] + M_PI, 2 * M_PI);
        if (key < 0) key += 2 * M_PI;
        key -= M_PI;
        float kf = (float)key;
        if (kf >= (float)M_PI) kf = -(float)M_PI;
        float idx;
        std::memcpy(&idx, &m, sizeof(int));
        zs[Mv++] = make_float4(zr[m], zb[m], idx, kf);
    }
    std::stable_sort(zs, zs + Mv, [](const float4& x, const float4& y) { return x.w < y.w; });
    for (int b = 0, k = 0; b < PHD_ZBINS; b++) {
        const float edge = (float)(-M_PI + b * (2 * M_PI / PHD_ZBINS));
        while (k < Mv && zs[k].w < edge) k++;
        zbin[b] = (unsigned short)k;
    }
    if (M > 0) {
        HIPCHK(hipMemcpyAsync(ctx->d_zblk, h, Z.bytes, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipEventRecord(ctx->ev_zring[slot], ctx->stream));
        ctx->zring_used[slot] = true;
    }
    ctx->M = M;
    ctx->Mv = Mv;
    ctx->zwide = zwide;
    return PHD_OK;
}

static DevCfg dev_cfg(const phd_slam_config& c) {
    DevCfg d;
    d.minRange = c.minRange;
    d.maxRange = c.maxRange;
    d.maxBearing = c.maxBearing;
    d.stdRange = c.stdRange;
    d.stdBearing = c.stdBearing;
    d.pd = c.pd;
    d.kappa = c.clutterDensity;
    d.birthWeight = c.birthWeight;
    d.birthNoiseFactor = c.birthNoiseFactor;
    d.minFeatureWeight = c.minFeatureWeight;
    d.minSeparation = c.minSeparation;
    d.log_birth = c.birthWeight <= 0 ? -FLT_MAX : phd_det_logf(c.birthWeight);  // (D17: the oracle's bits)
    d.log_2pi = (double)std::log((float)(2 * M_PI));
    const double kb = (double)c.clutterDensity + (double)c.birthWeight;
    if (c.minFeatureWeight > 0 && kb > 0)
        d.lq_keep_thresh = (float)(std::log((double)c.minFeatureWeight) + std::log(kb) - 0.5);
    else
        d.lq_keep_thresh = -INFINITY;
    d.labeled = c.labeledMeasurements ? 1 : 0;
    d.cphd_rate = (double)c.clutterRate;
    d.cphd_lrate = c.clutterRate > 0 ? std::log((double)c.clutterRate) : -INFINITY;
    d.cphd_lck = d.cphd_lrate - std::log((double)c.clutterDensity);
    d.cphd_log1mpd = 1 - c.pd <= 0 ? -FLT_MAX : std::log(1 - c.pd);
    d.log_minfw = c.minFeatureWeight > 0 ? std::log(c.minFeatureWeight) : -INFINITY;
    d.cphd_thr0 = (float)((std::log((double)c.minFeatureWeight) + std::log((double)c.clutterDensity) - 2.5) *
                          1.4426950408889634);
    d.cphd_leta_min = (float)(std::log((double)c.clutterDensity) - 2.0);
    {
        // PHD: η_m >= κ + β, so a term below (κ + β) 2^-40 moves it by < 2^-40
        // relative.  CPHD: Λ_m = rate Σ q / κ enters as (1 + Λ_m x): terms below
        // κ / rate 2^-48 move it by < 2^-48 absolute each.  The two-level fixed
        // point resolves 2^-70: the floor never goes below -72.
        const bool cphd = c.filterType == PHD_FILTER_CPHD;
        const double kb = cphd ? (double)c.clutterDensity / std::max((double)c.clutterRate, 1.0)
                               : (double)c.clutterDensity + (double)c.birthWeight;
        double fl = kb > 0 ? std::log2(kb) - (cphd ? 48.0 : 40.0) : -72.0;
        fl = std::max(fl, -72.0);
        const double thr0 = cphd ? (double)d.cphd_thr0 : (double)d.lq_keep_thresh * 1.4426950408889634;
        d.walk_floor = (float)std::min(fl, thr0 - 1.0);  // every listable pair is walked
    }
    return d;
}

struct FusedPredict {
    int predict;  // 1 Ackerman, 2 CV
    phd_ackerman_control u;
    uint64_t step;
};

/* Mixed static + dynamic update (feature_model 2; phd_mixed.hip). */
static int launch_update_mixed(phd_ctx* ctx) {
    const phd_slam_config& cfg = ctx->cfg;
    if (!ctx->dyn) return fail(PHD_E_ARG, "feature_model 2 needs phd_enable_dynamic");
    if (cfg.filterType != PHD_FILTER_PHD) return fail(PHD_E_UNSUPPORTED, "feature_model 2 with the CPHD filter");
    if (cfg.particleWeighting != 0) return fail(PHD_E_UNSUPPORTED, "particle_weighting != 0 is not implemented");
    if (cfg.distanceMetric != 0) return fail(PHD_E_UNSUPPORTED, "distance_metric != 0 (Hellinger) is not implemented");
    if (ctx->replay) return fail(PHD_E_UNSUPPORTED, "feature_model 2 in replay mode");
    if (ctx->d_map_x) return fail(PHD_E_UNSUPPORTED, "feature_model 2 with migrated (sharded) particles");
    if (ctx->n <= 0) return PHD_OK;
    const int in_set = ctx->cur, out_set = in_set ^ 1;
    const int din = ctx->dcur, dout = din ^ 1;
    MixedArgs a;
    a.n = ctx->n;
    a.cap = ctx->cap.map_capacity;
    a.dcap = ctx->dcap;
    a.M = ctx->M;
    a.Kcap = ctx->cap.candidate_capacity;
    a.src = ctx->d_src;
    a.src_reset = ctx->d_src;
    a.map_in = ctx->d_map[in_set];
    a.map_out = ctx->d_map[out_set];
    a.size_in = ctx->d_size[in_set];
    a.size_out = ctx->d_size[out_set];
    a.dmap_in = ctx->d_dmap[din];
    a.dmap_out = ctx->d_dmap[dout];
    a.dsize_in = ctx->d_dsize[din];
    a.dsize_out = ctx->d_dsize[dout];
    a.poses = ctx->d_pose;
    a.logw = ctx->d_logw;
    a.delta = ctx->d_delta;
    a.status = ctx->d_status;
    a.err = ctx->d_err;
    a.zr = ctx->d_zr;
    a.zb = ctx->d_zb;
    a.zlab = ctx->d_zlab;
    a.c = phd_mx_config(&cfg);
    a.ekf = ctx->d_mx_ekf;
    a.cand = ctx->d_mx_cand;
    const size_t lds = mixed_lds_bytes(a.cap, a.dcap, ctx->cap.max_measurements, a.Kcap);
    if (lds > 150 * 1024) return fail(PHD_E_CAPACITY, "feature_model 2: capacities exceed the 150 KB LDS budget");
    const bool timed = PHD_TIMING_EVENTS && !ctx->ev_a.empty() && ctx->timing_tick++ % ctx->timing_stride == 0;
    const int ei = ctx->ev_next;
    if (timed) HIPCHK(hipEventRecord(ctx->ev_a[ei], ctx->stream));
    HIPCHK(mixed_launch_update(a, lds, ctx->stream));
    if (timed) {
        HIPCHK(hipEventRecord(ctx->ev_b[ei], ctx->stream));
        ctx->ev_next = (ei + 1) % (int)ctx->ev_a.size();
        if (ctx->ev_used < (int)ctx->ev_a.size()) ctx->ev_used++;
    }
    ctx->cur = out_set;
    ctx->dcur = dout;
    return PHD_OK;
}

/* predictMapMixed (one phdPredict): every slab of the dynamic set, in -> out. */
static int launch_predict_dynamic(phd_ctx* ctx) {
    if (!ctx->dyn) return fail(PHD_E_ARG, "feature_model 2 needs phd_enable_dynamic");
    const int din = ctx->dcur, dout = din ^ 1;
    HIPCHK(mixed_launch_predict(ctx->nmax, ctx->dcap, ctx->d_dmap[din], ctx->d_dsize[din], ctx->d_dmap[dout],
                                ctx->d_dsize[dout], phd_mx_config(&ctx->cfg), ctx->stream));
    ctx->dcur = dout;
    return PHD_OK;
}

/* The fused update of every particle, or (slots != NULL) a re-update of
 * `nslots` listed slots with the sets of the last launch (a sharded step's
 * overflow recovery: same input slabs, same output slabs, cur unchanged). */
/* Trailing workgroups of an update launch that run at the highest wave
 * priority (UpdateArgs.prio): the ones dispatched last finish the launch, and
 * while they share SIMDs with earlier workgroups (which have slack) their
 * instructions issue first, so the launch drains sooner.  Default: the last
 * 20 % of the grid (measured at config 3: +1.3 % for 40 %; with the
 * last-written-first part C order 25 % is +0.2 % over 40 %, 55 % -1.5 %,
 * 20 % +1.0 % over 25 %, 15 % -0.5 %; four graded levels were no better;
 * round 4 close: 20 % = 35 %, none -1.3 %, profiles/r04fin_c3_prio_tail.txt). */
#ifndef UPD_PRIO_TAIL_PCT
#define UPD_PRIO_TAIL_PCT 20
#endif
static int prio_tail(int grid, int resident) {
    if (grid <= resident) return 0;
    return (int)((long)grid * UPD_PRIO_TAIL_PCT / 100);
}

static int launch_update(phd_ctx* ctx, const FusedPredict* fused = nullptr, const int* slots = nullptr,
                         int nslots = 0) {
    const phd_slam_config& cfg = ctx->cfg;
    if (cfg.featureModel == PHD_FEATURE_MIXED) {
        if (slots) return fail(PHD_E_UNSUPPORTED, "feature_model 2: slot updates (sharded step) are not supported");
        return launch_update_mixed(ctx);
    }
    if (cfg.featureModel != PHD_FEATURE_STATIC)
        return fail(PHD_E_UNSUPPORTED,
                    "feature_model 1 (dynamic only): the reference's update is a stub (phdfilter.cu:3663-3671)");
    if (cfg.distanceMetric != 0) return fail(PHD_E_UNSUPPORTED, "distance_metric != 0 (Hellinger) is not implemented");
    const bool cphd = cfg.filterType == PHD_FILTER_CPHD;
    if (cfg.filterType != PHD_FILTER_PHD && !cphd) return fail(PHD_E_UNSUPPORTED, "unknown filter_type");
    if (cphd) {
        if (ctx->M > PHD_CPHD_MAX_M)
            return fail(PHD_E_UNSUPPORTED, "CPHD update supports at most " + std::to_string(PHD_CPHD_MAX_M) +
                                               " measurements per step");
        if (cfg.maxCardinality < 0) return fail(PHD_E_ARG, "CPHD needs max_cardinality >= 0");
        if (fused && ctx->upd_threads > 512) return fail(PHD_E_ARG, "internal: no fused predict at 1024 threads");
        const int nl = std::max(cfg.maxCardinality, ctx->cap.max_measurements) + 2;
        if (ctx->lfact_n < nl) {
            std::vector<double> lf(nl);
            lf[0] = 0;
            for (int i = 1; i < nl; i++) lf[i] = lf[i - 1] + std::log((double)i);  // as the oracle
            if (ctx->d_lfact) hipFree(ctx->d_lfact);
            HIPCHK(hipMalloc((void**)&ctx->d_lfact, nl * sizeof(double)));
            HIPCHK(hipMemcpyAsync(ctx->d_lfact, lf.data(), nl * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
            HIPCHK(hipStreamSynchronize(ctx->stream));
            ctx->lfact_n = nl;
        }
        if (ensure_cn(ctx)) return PHD_E_HIP;
        if (!ctx->upd_cphd) {
            int rc = configure_update_launch(ctx, ctx->upd_threads_req);
            if (rc) return rc;
        }
    }
    if (cfg.particleWeighting != 0)
        return fail(PHD_E_UNSUPPORTED, "particle_weighting != 0 is not implemented on the device path");
    const int in_set = ctx->replay ? 0 : (slots ? ctx->cur ^ 1 : ctx->cur);
    const int out_set = in_set ^ 1;
    const int grid = slots ? nslots : ctx->n;
    if (grid <= 0) return PHD_OK;
    UpdateArgs a{};
    a.n = ctx->n;
    a.slots = slots;
    a.first = 0;
    a.prio = 0;  // set per launch (prio_tail)
    a.order = 0;
    a.cap = ctx->cap.map_capacity;
    a.M = ctx->M;
    a.Mcap = ctx->cap.max_measurements;
    a.Kcap = ctx->cap.candidate_capacity;
    a.Scap = ctx->cap.survivor_capacity;
    a.Epool = ctx->epool;
    a.plreq = ctx->plreq;
    a.Bbuckets = ctx->upd_split
                     ? upd_lds_layout(a.cap, a.Mcap, a.Kcap, a.Scap, a.Epool, ctx->upd_threads, cphd, 2).B
                     : upd_buckets(a.Kcap, 0);
    a.merge_mode = ctx->merge_mode;
    a.src = ctx->replay ? nullptr : ctx->d_src;
    a.src_reset = ctx->d_src;
    a.map_x = ctx->d_map_x;
    a.size_x = ctx->d_size_x;
    a.map_in = ctx->d_map[in_set];
    a.map_out = ctx->d_map[out_set];
    a.size_in = ctx->d_size[in_set];
    a.size_out = ctx->d_size[out_set];
    a.poses = ctx->d_pose;
    a.logw = ctx->d_logw;
    a.logw_out = slots ? nullptr : ctx->logw_mirror;  // (a partial update leaves the rest of the mirror stale)
    a.delta = ctx->d_delta;
    a.zr = ctx->d_zr;
    a.zb = ctx->d_zb;
    a.zok = ctx->d_zok;
    a.zs = ctx->d_zs;
    a.zbin = ctx->d_zbin;
    a.Mv = ctx->Mv;
    a.zwide = ctx->zwide;
    a.status = ctx->d_status;
    a.err = ctx->d_err;
    a.stamps = ctx->d_stamps;
    a.predict = 0;
    a.pu = phd_ackerman_control{0.f, 0.f};
    a.pc = predict_cfg(cfg, ctx->index_offset);
    a.pseed = ctx->seed;
    a.pstep = 0;
    a.pose_prior = nullptr;
    a.logw_prior = nullptr;
    if (fused) {
        a.predict = fused->predict;
        a.pu = fused->u;
        a.pstep = fused->step;
        a.pose_prior = ctx->replay ? ctx->d_pose_prior : nullptr;
        a.logw_prior = ctx->replay ? ctx->d_logw_prior : nullptr;
    }
    a.births = ctx->births_now > 0 ? ctx->d_births : nullptr;
    a.Mb = ctx->births_now;
    a.bzr = ctx->births_zr;
    a.bzb = ctx->births_zb;
    a.bzvi = ctx->births_zvi;
    ctx->births_now = 0;  // (consumed by this update)
    a.cn_coef = cphd ? ctx->d_cn_coef : nullptr;
    a.hand = nullptr;
    if (ctx->upd_split) {
        const size_t hb = (size_t)ctx->nmax * cphd_hand_layout(ctx->cap.map_capacity, ctx->cap.max_measurements,
                                                             ctx->cap.survivor_capacity)
                                               .stride;
        if (!ctx->d_hand) HIPCHK(hipMalloc((void**)&ctx->d_hand, hb));
        a.hand = ctx->d_hand;
    }
    a.cn_stride = ctx->cn_stride;
    a.lfact = ctx->d_lfact;
    a.Nmax = cfg.maxCardinality;
    a.c = dev_cfg(cfg);
    const bool timed =
        PHD_TIMING_EVENTS && !ctx->ev_a.empty() && !slots && ctx->timing_tick++ % ctx->timing_stride == 0;
    const int ei = ctx->ev_next;
    if (timed) HIPCHK(hipEventRecord(ctx->ev_a[ei], ctx->stream));
    // the launches of one chunk of particles [a.first, a.first + grid) on stream st
    // PHD_RS_OVERLAP: once the log-weights are final (after the CPHD terms
    // launch, or after the split PHD update's part A) the step's resample runs
    // on the auxiliary stream beside part C; part C reads neither the
    // log-weights nor the arrays the resample writes
    // PHD_RS_LEAD: instead, part C's lead workgroup runs it (rs_step_block): the
    // launch gets RS_LEAD_WGS workgroups in front (the others return at once,
    // so every particle keeps its XCD) and no event crosses streams.  Returns
    // the lead workgroups of the part C launch.  (The diagnostic stamps build
    // indexes its records by workgroup: it keeps the second stream.)
    auto rs_lead = [&](UpdateArgs& x) -> int {
        if (!PHD_RS_LEAD || !ctx->rs_ov.armed || slots || x.stamps) return 0;
        x.rs_lead = RS_LEAD_WGS;
        x.rs = ctx->rs_ov.a;
        ctx->rs_ov.launched = true;
        ctx->rs_ov.lead = true;
        return RS_LEAD_WGS;
    };
    auto rs_beside = [&](hipStream_t st) {
        if (!ctx->rs_ov.armed || slots || ctx->rs_ov.launched) return;
        hipEventRecord(ctx->ev_terms, st);
        hipStreamWaitEvent(ctx->aux, ctx->ev_terms, 0);
        hipLaunchKernelGGL(k_rs_step, dim3(ctx->rs_ov.B), dim3(RS_THREADS), 0, ctx->aux, ctx->rs_ov.a);
        hipEventRecord(ctx->ev_rs, ctx->aux);
        ctx->rs_ov.launched = true;
    };
    auto chain = [&](UpdateArgs a, int grid, hipStream_t st) {
        if (grid <= 0) return;
        a.prio = prio_tail(grid, ctx->upd_resident);
        if (cphd) {
            // part A -> CPHD terms (one wave per particle) -> part C (the diagnostic
            // phase stamps record part C)
            UpdateArgs aa = a;
            aa.stamps = nullptr;
#ifdef PHD_STAMP_PART_A
            aa.stamps = a.stamps;  // diagnostic stamps build: record part A instead
            a.stamps = nullptr;
#endif
            // part A runs the particle's predict when fused (the CPHD update is three
            // launches: the predict's registers cost part A nothing that matters)
            const void* ka = fused ? (ctx->upd_threads == 256 ? (const void*)k_update_cphd_a_p256
                                                                : (const void*)k_update_cphd_a_p512)
                                   : update_kernel(ctx->upd_threads, 1, 1);
            aa.prio = prio_tail(grid, ctx->upd_resident_a);
            hipLaunchKernelGGL((void (*)(UpdateArgs))ka, dim3(grid), dim3(ctx->upd_threads), ctx->upd_lds_a, st,
                               aa);
            // the fused predict is done: parts B and C read the predicted poses
            a.predict = 0;
            a.pose_prior = nullptr;
            a.logw_prior = nullptr;
            // the terms and part C read part A's handoff and prior slab: last-written first
            a.order = 1;
            hipLaunchKernelGGL(k_cphd_terms, dim3(grid), dim3(64), cphd_terms_lds(ctx->cap.max_measurements), st,
                               a);
            if (ctx->ev_logw) {  // the log-weights are final (phd_wait_logw)
                hipEventRecord(ctx->ev_logw, st);
                ctx->logw_marked = true;
            }
            const int lead = rs_lead(a);
            rs_beside(st);
            hipLaunchKernelGGL((void (*)(UpdateArgs))update_kernel(ctx->upd_threads, 1, 2), dim3(grid + lead),
                               dim3(ctx->upd_threads), ctx->upd_lds, st, a);
            ctx->cn_valid = true;
        } else if (ctx->upd_split) {
            // split PHD update: part A -> part C through the handoff (the predict ran
            // as its own launch: enqueue_predict_update does not fuse it here)
            UpdateArgs aa = a;
            aa.stamps = nullptr;
#ifdef PHD_STAMP_PART_A
            aa.stamps = a.stamps;
            a.stamps = nullptr;
#endif
            aa.prio = prio_tail(grid, ctx->upd_resident_a);
            hipLaunchKernelGGL((void (*)(UpdateArgs))update_kernel(ctx->upd_threads, 0, 1), dim3(grid),
                               dim3(ctx->upd_threads), ctx->upd_lds_a, st, aa);
            if (ctx->ev_logw) {  // part A wrote the log-weights (phd_wait_logw)
                hipEventRecord(ctx->ev_logw, st);
                ctx->logw_marked = true;
            }
            const int lead = rs_lead(a);
            rs_beside(st);
            a.predict = 0;
            a.pose_prior = nullptr;
            a.logw_prior = nullptr;
            a.order = 1;  // last-written first, XCD-preserving (upd_particle)
            hipLaunchKernelGGL((void (*)(UpdateArgs))update_kernel(ctx->upd_threads, 0, 2), dim3(grid + lead),
                               dim3(ctx->upd_threads), ctx->upd_lds, st, a);
        } else if (fused && ctx->upd_threads == 256) {
            hipLaunchKernelGGL(k_update_fused_p256, dim3(grid), dim3(256), ctx->upd_lds, st, a);
        } else if (fused && ctx->upd_threads == 512) {
            hipLaunchKernelGGL(k_update_fused_p512, dim3(grid), dim3(512), ctx->upd_lds, st, a);
        } else {
            switch (ctx->upd_threads) {
                case 256: hipLaunchKernelGGL(k_update_fused_256, dim3(grid), dim3(256), ctx->upd_lds, st, a); break;
                case 512: hipLaunchKernelGGL(k_update_fused_512, dim3(grid), dim3(512), ctx->upd_lds, st, a); break;
                default: hipLaunchKernelGGL(k_update_fused_1024, dim3(grid), dim3(1024), ctx->upd_lds, st, a); break;
            }
        }
    };
    ctx->logw_marked = false;
    chain(a, grid, ctx->stream);
    HIPCHK(hipGetLastError());
    if (ctx->ev_logw && !ctx->logw_marked) {  // (the fused update: its log-weights at its end)
        HIPCHK(hipEventRecord(ctx->ev_logw, ctx->stream));
        ctx->logw_marked = true;
    }
    if (!slots) ctx->src_fresh = true;  // part C reset every slab reference to the identity
    if (timed) {
        HIPCHK(hipEventRecord(ctx->ev_b[ei], ctx->stream));
        ctx->ev_next = (ei + 1) % (int)ctx->ev_a.size();
        if (ctx->ev_used < (int)ctx->ev_a.size()) ctx->ev_used++;
    }
    if (!slots) ctx->cur = out_set;
    return PHD_OK;
}

static int check_err(phd_ctx* ctx);

/* the step adds births (phd_set_step_births; by default with CPHD, whose
 * update array has no birth terms: phdfilter.cu.bak:738-870) */
static bool step_births_on(const phd_ctx* ctx) {
    return ctx->step_births_req < 0 ? ctx->cfg.filterType == PHD_FILTER_CPHD : ctx->step_births_req != 0;
}

int phd_set_step_births(phd_ctx* ctx, int on) {
    if (!ctx || on < -1 || on > 1) return fail(PHD_E_ARG, "bad arguments to phd_set_step_births");
    ctx->step_births_req = on;
    return PHD_OK;
}

int phd_step_births(phd_ctx* ctx, int* on) {
    if (!ctx || !on) return fail(PHD_E_ARG, "null argument");
    *on = step_births_on(ctx) ? 1 : 0;
    return PHD_OK;
}

/* the scan the step's births come from: its raw rows, measurement count and
 * valid count (false: no births this step) */
static bool birth_rows(const phd_ctx* ctx, const float** zr, const float** zb, const int** zok, int* Mr, int* Mv) {
    if (!step_births_on(ctx) || ctx->cfg.featureModel != PHD_FEATURE_STATIC) return false;  // (mixed: update terms)
    const bool own = ctx->replay;  // replay: the fixed scan is also the previous one
    if (!own && !ctx->have_prev) return false;
    *Mr = own ? ctx->M : ctx->M_prev;
    *Mv = own ? ctx->Mv : ctx->Mv_prev;
    if (*Mr <= 0 || *Mv <= 0) return false;
    const ZBlk Z = zblk_layout();
    const unsigned char* rows = own ? ctx->d_zblk : ctx->d_zprev;
    *zr = (const float*)(rows + Z.zr);
    *zb = (const float*)(rows + Z.zb);
    *zok = (const int*)(rows + Z.zok);
    return true;
}

/* The step's births, after its predict: the previous scan's valid measurements
 * (replay: the replayed scan's own).  With an update this step the update's
 * classify places them itself after each particle's map (UpdateArgs::births:
 * this only arms it); with no measurements they are appended to the maps by
 * k_add_births, as the reference does without an update. */
static int launch_step_births(phd_ctx* ctx, const int* slots, int count) {
    ctx->births_now = 0;
    if (count <= 0) return PHD_OK;
    const float *zr = nullptr, *zb = nullptr;
    const int* zok = nullptr;
    int Mr = 0, Mv = 0;
    if (!birth_rows(ctx, &zr, &zb, &zok, &Mr, &Mv)) return PHD_OK;
    if (ctx->M <= 0) {
        // no update this step: the births join the maps themselves.  Pending
        // slots (a sharded settle on an empty scan) take the sets a slot update
        // takes (launch_update): their records (set X) -> their slabs of the
        // current set, which the step's own births launch wrote
        const int in_set = slots ? ctx->cur ^ 1 : ctx->cur, out_set = slots ? ctx->cur : ctx->cur ^ 1;
        hipLaunchKernelGGL(k_add_births, dim3(count), dim3(256), 0, ctx->stream, ctx->d_src, slots, count,
                           ctx->cap.map_capacity, (const float*)ctx->d_map[in_set], (const int*)ctx->d_size[in_set],
                           (const float*)ctx->d_map_x, (const int*)ctx->d_size_x, ctx->d_map[out_set],
                           ctx->d_size[out_set], (const phd_pose*)ctx->d_pose, zr, zb, zok, Mr, dev_cfg(ctx->cfg),
                           ctx->d_status, ctx->d_err);
        HIPCHK(hipGetLastError());
        if (!slots) {
            hipLaunchKernelGGL(k_iota, dim3((ctx->n + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_src, ctx->n);
            HIPCHK(hipGetLastError());
            ctx->cur = out_set;
        }
        return PHD_OK;
    }
    if (!ctx->d_births)
        HIPCHK(hipMalloc((void**)&ctx->d_births, (size_t)ctx->nmax * 7 * ctx->cap.map_capacity * sizeof(float)));
    const ZBlk Z = zblk_layout();
    const unsigned char* rows = (const unsigned char*)zr - Z.zr;
    ctx->births_zr = zr;
    ctx->births_zb = zb;
    ctx->births_zvi = (const int*)(rows + Z.zvi);
    ctx->births_now = Mv;
    return PHD_OK;
}

/* CPHD births through the prediction (phd_capi.h). */
int phd_add_births(phd_ctx* ctx, const phd_measurement* z, int n_measure) {
    if (!ctx || n_measure < 0 || (n_measure > 0 && !z)) return fail(PHD_E_ARG, "bad arguments to phd_add_births");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (ctx->replay) return fail(PHD_E_ARG, "phd_add_births: not in replay mode");
    if (ctx->step_births_req < 0)
        ctx->step_births_req = 0;  // the caller's loop places the births (the pre-step-births API): from now on
    if (step_births_on(ctx))
        return fail(PHD_E_ARG, "phd_add_births: phd_set_step_births(ctx, 1) asked the step to add the births of "
                               "the previous scan itself");
    if (n_measure == 0) return PHD_OK;
    if (set_device(ctx)) return PHD_E_HIP;
    // the previous scan's measurements through phd_set_measurements' device rows
    // (they replace the context's measurements: set the update's afterwards)
    int rc = phd_set_measurements(ctx, z, n_measure);
    if (rc) return rc;
    const int M = ctx->M;
    const int in_set = ctx->cur, out_set = in_set ^ 1;
    hipLaunchKernelGGL(k_add_births, dim3(ctx->n), dim3(256), 0, ctx->stream, ctx->d_src, (const int*)nullptr, ctx->n,
                       ctx->cap.map_capacity, (const float*)ctx->d_map[in_set], (const int*)ctx->d_size[in_set],
                       (const float*)ctx->d_map_x, (const int*)ctx->d_size_x, ctx->d_map[out_set],
                       ctx->d_size[out_set], (const phd_pose*)ctx->d_pose, (const float*)ctx->d_zr,
                       (const float*)ctx->d_zb, (const int*)ctx->d_zok, M, dev_cfg(ctx->cfg), ctx->d_status,
                       ctx->d_err);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_iota, dim3((ctx->n + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_src, ctx->n);
    HIPCHK(hipGetLastError());
    ctx->cur = out_set;
    if (ctx->check_each_update) return check_err(ctx);
    return PHD_OK;
}

int phd_enable_timing(phd_ctx* ctx, int max_records) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (auto e : ctx->ev_a) hipEventDestroy(e);
    for (auto e : ctx->ev_b) hipEventDestroy(e);
    ctx->ev_a.clear();
    ctx->ev_b.clear();
    ctx->ev_next = ctx->ev_used = 0;
    ctx->timing_tick = 0;
    for (int i = 0; i < max_records; i++) {
        hipEvent_t a, b;
        HIPCHK(hipEventCreateWithFlags(&a, kEvTime));
        HIPCHK(hipEventCreateWithFlags(&b, kEvTime));
        ctx->ev_a.push_back(a);
        ctx->ev_b.push_back(b);
    }
    return PHD_OK;
}

int phd_set_timing_stride(phd_ctx* ctx, int stride) {
    if (!ctx || stride < 1) return fail(PHD_E_ARG, "bad arguments to phd_set_timing_stride");
    ctx->timing_stride = stride;
    ctx->timing_tick = 0;
    return PHD_OK;
}

int phd_update_timing(phd_ctx* ctx, float* total_ms, int* count) {
    if (!ctx || !total_ms) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float tot = 0.f;
    for (int i = 0; i < ctx->ev_used; i++) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev_a[i], ctx->ev_b[i]));
        tot += ms;
    }
    *total_ms = tot;
    if (count) *count = ctx->ev_used;
    ctx->ev_used = 0;
    ctx->ev_next = 0;
    return PHD_OK;
}

static int check_err(phd_ctx* ctx) {
    int err = 0;
    HIPCHK(hipMemcpyAsync(&err, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (err) {
        hipMemsetAsync(ctx->d_err, 0, sizeof(int), ctx->stream);
        std::string m = "update capacity exceeded:";
        if (err & PHD_ST_SURVIVOR_OVERFLOW) m += " survivor_capacity";
        if (err & PHD_ST_CANDIDATE_OVERFLOW) m += " candidate_capacity";
        if (err & PHD_ST_MAP_OVERFLOW) m += " map_capacity";
        if (err & PHD_ST_ETA_RANGE) m += " likelihood range (a term >= 2^20)";
        if (err & PHD_ST_WAIT_TIMEOUT) m += " (a one-launch resample wait timed out: not every workgroup was resident)";
        return fail(PHD_E_CAPACITY, m);
    }
    return PHD_OK;
}

int phd_update(phd_ctx* ctx) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ctx->M == 0) return PHD_OK;  // run_synth skips the update when |Z| == 0 (main.cpp:1260)
    int rc = launch_update(ctx);
    if (rc) return rc;
    if (ctx->check_each_update) return check_err(ctx);
    return PHD_OK;
}

int phd_last_update_ms(phd_ctx* ctx, float* ms) {
    if (!ctx || !ms) return fail(PHD_E_ARG, "null argument");
    if (ctx->ev_used == 0) return fail(PHD_E_ARG, "timing not enabled (phd_enable_timing) or no update recorded");
    const int i = (ctx->ev_next + (int)ctx->ev_a.size() - 1) % (int)ctx->ev_a.size();
    HIPCHK(hipEventSynchronize(ctx->ev_b[i]));
    HIPCHK(hipEventElapsedTime(ms, ctx->ev_a[i], ctx->ev_b[i]));
    return PHD_OK;
}

int phd_normalize(phd_ctx* ctx, const float* lse_override) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    const float* d_ov = nullptr;
    if (lse_override) {
        HIPCHK(hipMemcpyAsync(ctx->d_out + 8, lse_override, sizeof(float), hipMemcpyHostToDevice, ctx->stream));
        d_ov = ctx->d_out + 8;
    }
    hipLaunchKernelGGL(k_normalize, dim3(1), dim3(1024), 0, ctx->stream, ctx->d_logw, ctx->n, d_ov, ctx->d_out,
                       ctx->cfg.resampleThresh, rs_mode(ctx));
    HIPCHK(hipGetLastError());
    if (lse_override) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_neff(phd_ctx* ctx, float* neff) {
    if (!ctx || !neff) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    float out[2];
    HIPCHK(hipMemcpyAsync(out, ctx->d_out, 2 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *neff = out[1];
    return PHD_OK;
}

/* dynamic LDS of the resample kernels: the CDF when it fits (RS_LDS_MAX) */
static size_t rs_lds(int n) { return n <= RS_LDS_MAX ? (size_t)n * sizeof(unsigned long long) : 0; }

/* resample the live particles into n_particles (main.cpp:1289, resampleParticles(particles, n_particles)) */
static int launch_resample(phd_ctx* ctx, const int* d_flag, const double* du, uint64_t step) {
    const float neglogn = (float)(-std::log((double)ctx->n_base));  // slamtypes.h:328
    ctx->src_fresh = false;  // (the resample remaps the slab references)
    hipLaunchKernelGGL(k_resample, dim3(1), dim3(1024), rs_lds(ctx->n), ctx->stream, d_flag, ctx->d_logw, ctx->d_logw,
                       ctx->n, ctx->n_base, du, ctx->seed, step, ctx->d_cdf, ctx->d_idx, ctx->d_pose, ctx->d_src,
                       ctx->d_tmp_pose, ctx->d_tmp_src, neglogn);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_resample(phd_ctx* ctx, const double* u_host, uint64_t step, int* idx_host) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    const double* du = nullptr;
    if (u_host) {
        HIPCHK(hipMemcpyAsync(ctx->d_u, u_host, ctx->n_base * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
        du = ctx->d_u;
    }
    int rc = launch_resample(ctx, nullptr, du, step);
    if (rc) return rc;
    ctx->n = ctx->n_base;
    if (idx_host) {
        HIPCHK(hipMemcpyAsync(idx_host, ctx->d_idx, ctx->n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    }
    if (u_host || idx_host) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_apply_resample(phd_ctx* ctx, const int* dev_idx, float new_log_weight) {
    if (!ctx || !dev_idx) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    ctx->src_fresh = false;
    hipLaunchKernelGGL(k_apply_parents, dim3(1), dim3(1024), 0, ctx->stream, (const int*)nullptr, dev_idx, ctx->n,
                       ctx->d_pose, ctx->d_src,
                       ctx->d_logw, ctx->d_tmp_pose, ctx->d_tmp_src, new_log_weight);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

/* predict (fused into the update when it pays) + update: the part of a step
 * before the cross-particle normalisation. */
static int enqueue_predict_update(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step,
                                  const int* slots = nullptr, int nslots = 0) {
    const phd_slam_config& cfg = ctx->cfg;
    int rc;
    const int count = slots ? nslots : ctx->n;
    // the step's births are placed by the update's classify from the predicted
    // pose (also when the predict is fused into the update)
    const bool births = step_births_on(ctx) && cfg.featureModel == PHD_FEATURE_STATIC;
    if (do_predict && ctx->M > 0 && cfg.nPredictParticles == 1 && cfg.featureModel == PHD_FEATURE_STATIC &&
        (ctx->n <= ctx->upd_resident_p || (PHD_FUSE_PREDICT_ALL && cfg.filterType == PHD_FILTER_CPHD)) &&
        ctx->upd_threads <= 512 && (cfg.filterType == PHD_FILTER_CPHD || !ctx->upd_split)) {
        // predict fused into the update launch when every particle's workgroup is
        // resident at once (saves a launch); with several rounds of workgroups the
        // serial per-particle predict would sit on each round's critical path
        FusedPredict fp;
        fp.predict = cfg.motionType == PHD_MOTION_ACKERMAN ? 1 : 2;
        if (fp.predict == 1 && !u) return fail(PHD_E_ARG, "Ackerman predict needs a control");
        fp.u = u ? *u : phd_ackerman_control{0.f, 0.f};
        fp.step = step;
        if (births) {
            rc = launch_step_births(ctx, slots, slots ? count : ctx->n);
            if (rc) return rc;
        }
        rc = launch_update(ctx, &fp, slots, nslots);
        if (rc) return rc;
    } else if (do_predict) {
        rc = check_predict(ctx);
        if (rc) return rc;
        const int sub = cfg.subdividePredict > 0 ? cfg.subdividePredict : 1;
        if (cfg.motionType == PHD_MOTION_ACKERMAN && !u) return fail(PHD_E_ARG, "Ackerman predict needs a control");
        if (cfg.nPredictParticles > 1 && slots) return fail(PHD_E_UNSUPPORTED, "n_predict_particles > 1 on slots");
        for (int k = 0; k < sub; k++) {  // (main.cpp:1248-1254: subdividePredict calls of phdPredict)
            const uint64_t s = step * (uint64_t)sub + (uint64_t)k;
            rc = expand_particles(ctx);
            if (rc) return rc;
            rc = launch_predict(ctx, u ? *u : phd_ackerman_control{0.f, 0.f}, nullptr, s, slots,
                                slots ? count : ctx->n);
            if (rc) return rc;
        }
        if (births) {
            rc = launch_step_births(ctx, slots, slots ? count : ctx->n);
            if (rc) return rc;
        }
        if (ctx->M > 0) {
            rc = launch_update(ctx, nullptr, slots, nslots);
            if (rc) return rc;
        }
    } else {
        if (births) {
            rc = launch_step_births(ctx, slots, slots ? count : ctx->n);
            if (rc) return rc;
        }
        if (ctx->M > 0) {
            rc = launch_update(ctx, nullptr, slots, nslots);
            if (rc) return rc;
        }
    }
    return PHD_OK;
}

int phd_predict_update(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step,
                       float* dev_logw_out) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (set_device(ctx)) return PHD_E_HIP;
    // the update writes each new log-weight to dev_logw_out as well (no copy
    // launch), when every particle is updated by the static-model kernels
    const bool mirror = dev_logw_out && ctx->M > 0 && ctx->cfg.featureModel == PHD_FEATURE_STATIC &&
                        ctx->cfg.nPredictParticles <= 1 && ctx->n == ctx->n_base;
    ctx->logw_mirror = mirror ? dev_logw_out : nullptr;
    ctx->logw_marked = false;
    int rc = enqueue_predict_update(ctx, u, do_predict, step);
    ctx->logw_mirror = nullptr;
    if (rc) return rc;
    if (dev_logw_out && !mirror)
        HIPCHK(hipMemcpyAsync(dev_logw_out, ctx->d_logw, ctx->n * sizeof(float), hipMemcpyDeviceToDevice,
                              ctx->stream));
    // phd_wait_logw promises the mirror complete: when no update marked the
    // log-weights final this call (an empty scan: no update at all) or the
    // mirror is a copy, mark them after it
    if (ctx->ev_logw && (!ctx->logw_marked || (dev_logw_out && !mirror)))
        HIPCHK(hipEventRecord(ctx->ev_logw, ctx->stream));
    return PHD_OK;
}

int phd_step(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step, float* neff_out,
             int* resampled) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config not called");
    if (set_device(ctx)) return PHD_E_HIP;
    const phd_slam_config& cfg = ctx->cfg;
    // chunked normalise up to 16 chunks: each block takes the max of all
    // entries itself instead of a k_rs_max launch (same max, same bits)
    const bool fuse_max = ctx->n <= 16 * RS_THREADS;
    // normalise + nEff + device-side resample decision + resample (main.cpp:1281-1297)
    const float neglogn = (float)(-std::log((double)ctx->n));
    // PHD_RS_OVERLAP: the one-launch resample beside part C of a CPHD step (its
    // log-weights are final after the terms launch) or of a split PHD step
    // (final after part A); armed only records its arguments, and a chain that
    // does not launch it (the fused PHD update) leaves it to the main stream
    // below.  Its workgroups wait out part C on their CUs, so only while part C
    // is a few rounds of resident workgroups (config 4's per-GPU shard, 2.7
    // rounds: 3 409 -> 3 504 steps/s; config 5's, 16 rounds: 674 -> 645)
    const bool overlap = (cfg.filterType == PHD_FILTER_CPHD ? (PHD_RS_OVERLAP & 1) : ctx->upd_split && (PHD_RS_OVERLAP & 2)) &&
                         ctx->n <= 4 * ctx->upd_resident && cfg.nPredictParticles <= 1 &&
                         ctx->n == ctx->n_base && ctx->n > 2 * RS_THREADS && fuse_max && ctx->M > 0 &&
                         cfg.featureModel == PHD_FEATURE_STATIC;
    if (overlap) {
        if (!ctx->aux) {
            int lo = 0, hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking, hi));
            HIPCHK(hipEventCreateWithFlags(&ctx->ev_terms, kEvOrder));
            HIPCHK(hipEventCreateWithFlags(&ctx->ev_rs, kEvOrder));
        }
        ctx->rs_ov.armed = true;
        ctx->rs_ov.launched = false;
        ctx->rs_ov.lead = false;
        int rc0 = launch_rs_chunks(ctx, ctx->d_logw, ctx->n, ctx->d_out, ctx->seed, step, ctx->d_idx, true, neglogn,
                                   fuse_max);  // (armed: only records the launch's arguments)
        if (rc0) {
            ctx->rs_ov.armed = false;
            return rc0;
        }
    }
    int rc = enqueue_predict_update(ctx, u, do_predict, step);
    // (in the lead workgroup: ordered by the stream itself, no event to wait on)
    const bool ov_launched = ctx->rs_ov.launched && !ctx->rs_ov.lead;
    const bool ov_done = ctx->rs_ov.launched;
    ctx->rs_ov.armed = false;
    ctx->rs_ov.launched = false;
    ctx->rs_ov.lead = false;
    if (rc) {
        // the resample may already run on the auxiliary stream (it writes the
        // log-weights, the parents and the spare pose / slab arrays): order
        // everything the caller enqueues next after it
        if (ov_launched) hipStreamWaitEvent(ctx->stream, ctx->ev_rs, 0);
        return rc;
    }
    if (cfg.nPredictParticles > 1 || ctx->n != ctx->n_base) {
        // live count above n_particles: the resample draws n_particles children
        // and the next step's launches depend on the decision, so it is read
        // back here (one host synchronisation per step in this mode)
        hipLaunchKernelGGL(k_normalize, dim3(1), dim3(1024), 0, ctx->stream, ctx->d_logw, ctx->n,
                           (const float*)nullptr, ctx->d_out, cfg.resampleThresh, rs_mode(ctx));
        HIPCHK(hipGetLastError());
        rc = launch_resample(ctx, (const int*)(ctx->d_out + 2), nullptr, step);
        if (rc) return rc;
        if (ctx->M > 0 && ctx->check_each_update) {
            rc = check_err(ctx);
            if (rc) return rc;
        }
        float out[3];
        HIPCHK(hipMemcpyAsync(out, ctx->d_out, 3 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        int f;
        memcpy(&f, &out[2], sizeof(int));
        if (f) ctx->n = ctx->n_base;
        if (neff_out) *neff_out = out[1];
        if (resampled) *resampled = f;
        return PHD_OK;
    }
    if (ctx->n <= 2 * RS_THREADS) {  // one launch: a single block is fastest here
        hipLaunchKernelGGL(k_normalize_resample, dim3(1), dim3(1024), rs_lds(ctx->n), ctx->stream, ctx->d_logw,
                           ctx->n, ctx->d_out, cfg.resampleThresh, ctx->M > 0 ? 1 : 0, ctx->seed, step, ctx->d_cdf,
                           ctx->d_idx, ctx->d_pose, ctx->d_src, ctx->d_tmp_pose, ctx->d_tmp_src, neglogn);
        HIPCHK(hipGetLastError());
    } else {  // chunked over n/1024 workgroups; the search writes the remap into the spare arrays
        if (ov_done) {
            if (ov_launched) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_rs, 0));  // (ran beside part C)
        } else {
            rc = launch_rs_chunks(ctx, ctx->d_logw, ctx->n, ctx->d_out, ctx->seed, step, ctx->d_idx, true, neglogn,
                                  fuse_max);
            if (rc) return rc;
        }
        std::swap(ctx->d_pose, ctx->d_tmp_pose);  // identity copy when no resample was decided
        std::swap(ctx->d_src, ctx->d_tmp_src);
        ctx->src_fresh = false;  // (a remap, when the device decided to resample)
    }
    if (ctx->M > 0 && ctx->check_each_update) {
        rc = check_err(ctx);
        if (rc) return rc;
    }
    if (neff_out || resampled) {
        float out[3];
        HIPCHK(hipMemcpyAsync(out, ctx->d_out, 3 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        if (neff_out) *neff_out = out[1];
        if (resampled) {
            int f;
            memcpy(&f, &out[2], sizeof(int));
            *resampled = f;
        }
    }
    return PHD_OK;
}

__global__ void k_fill(float* a, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = v;
}

int phd_set_index_offset(phd_ctx* ctx, int offset) {
    if (!ctx || offset < 0) return fail(PHD_E_ARG, "bad arguments");
    ctx->index_offset = offset;
    return PHD_OK;
}

int phd_fill_log_weights(phd_ctx* ctx, float value) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_fill, dim3((ctx->n + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_logw, ctx->n, value);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_global_resample(phd_ctx* ctx, float* dev_w_all, int n_total, int offset, uint64_t seed, uint64_t step,
                        int* dev_parents, float* neff, int* resampled) {
    if (!ctx || !dev_w_all || !dev_parents || n_total < ctx->n || offset < 0 || offset + ctx->n > n_total)
        return fail(PHD_E_ARG, "bad arguments to phd_global_resample");
    if (ctx->cfg.nPredictParticles > 1 || ctx->n != ctx->n_base)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with n_predict_particles > 1 (shards hold n_particles each)");
    if (ctx->cfg.featureModel != PHD_FEATURE_STATIC)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with feature_model != 0");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ctx->cdf_g_cap < n_total) {
        if (ctx->d_cdf_g) hipFree(ctx->d_cdf_g);
        HIPCHK(hipMalloc((void**)&ctx->d_cdf_g, (size_t)n_total * sizeof(unsigned long long)));
        ctx->cdf_g_cap = n_total;
    }
    float* out = ctx->d_out + 40;
    hipLaunchKernelGGL(k_normalize, dim3(1), dim3(1024), 0, ctx->stream, dev_w_all, n_total, (const float*)nullptr, out,
                       ctx->cfg.resampleThresh, ctx->M > 0 ? 1 : 0);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ctx->d_logw, dev_w_all + offset, ctx->n * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    const float neglogn = (float)(-std::log((double)n_total));
    hipLaunchKernelGGL(k_resample, dim3(1), dim3(1024), rs_lds(n_total), ctx->stream, (const int*)(out + 2), dev_w_all, dev_w_all,
                       n_total, n_total, (const double*)nullptr, seed, step, ctx->d_cdf_g, dev_parents, (phd_pose*)nullptr,
                       (int*)nullptr, (phd_pose*)nullptr, (int*)nullptr, neglogn);
    HIPCHK(hipGetLastError());
    float h[3];
    HIPCHK(hipMemcpyAsync(h, out, 3 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (neff) *neff = h[1];
    if (resampled) memcpy(resampled, &h[2], sizeof(int));
    return PHD_OK;
}

/* plan buffers of a sharded step for `world` ranks (device + pinned read-back) */
static int ensure_mig(phd_ctx* ctx, int world) {
    if (ctx->mig_cap < world) {
        if (ctx->d_mig) hipFree(ctx->d_mig);
        ctx->d_mig = nullptr;
        HIPCHK(hipMalloc((void**)&ctx->d_mig, (size_t)(3 * world + MIG_TAIL) * sizeof(int)));
        ctx->mig_cap = world;
    }
    if (ctx->h_mig_cap < world) {  // host-mapped, coherent: the tail writes the plan's counts into it (no copy launch)
        if (ctx->h_mig) hipHostFree(ctx->h_mig);
        ctx->h_mig = nullptr;
        ctx->h_mig_dev = nullptr;
        HIPCHK(hipHostMalloc((void**)&ctx->h_mig, (size_t)(3 * world + MIG_TAIL) * sizeof(int),
                             hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&ctx->h_mig_dev, ctx->h_mig, 0));
        memset(ctx->h_mig, 0, (size_t)(3 * world + MIG_TAIL) * sizeof(int));
        ctx->plan_seq = 0;
        ctx->h_mig_cap = world;
        ctx->h_mig_world = world;
    }
    if (ctx->h_mig_world != world) {
        // the poll's sequence word sits at 3 world + MIG_SEQ: under another world
        // that slot held a count of an earlier plan, which could equal the next
        // sequence number — clear the buffer once the earlier plans are done
        HIPCHK(hipStreamSynchronize(ctx->stream));
        memset(ctx->h_mig, 0, (size_t)(3 * ctx->h_mig_cap + MIG_TAIL) * sizeof(int));
        ctx->h_mig_world = world;
    }
    if (!ctx->d_pend) HIPCHK(hipMalloc((void**)&ctx->d_pend, (size_t)ctx->n * sizeof(int)));
    if (ensure_sync(ctx)) return PHD_E_HIP;
    if (!ctx->plan_max_blocks) {
        int per_cu = 0, ncu = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_shard_plan, RS_THREADS, 0));
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        // one workgroup per CU whatever the query says beyond that: the query can
        // be one high, and a grid that is not resident at once would stall its waits
        ctx->plan_max_blocks = per_cu > 0 ? std::max(ncu, 1) : -1;
    }
    return PHD_OK;
}

/* The sharded plan (global normalise / nEff / decision / parents, then this
 * rank's migration plan and remap): one k_shard_plan launch when its
 * ceil(N/1024) workgroups can all be resident (every config here: <= 256), else
 * the k_rs_* chain + k_shard_tail. */
static int launch_shard_plan(phd_ctx* ctx, float* dev_w_all, int world, int rank, uint64_t seed, uint64_t step,
                             int* dev_parents, int* dev_keep_src, int* dev_send_src, int* dev_recv_rec,
                             float new_log_weight, int block_records, bool chain = false, bool with_src = true) {
    const int n_total = world * ctx->n;
    const int B = (n_total + RS_THREADS - 1) / RS_THREADS;
    float* out = ctx->d_out + 40;
    const int* src = with_src ? (const int*)ctx->d_src : nullptr;  // (NULL: the identity)
    if (!chain && B <= ctx->plan_max_blocks) {
        RsParts P;
        int rc = rs_parts(ctx, n_total, P);
        if (rc) return rc;
        ShardPlanArgs a;
        a.w = dev_w_all;
        a.N = n_total;
        a.B = B;
        a.n = ctx->n;
        a.world = world;
        a.rank = rank;
        a.has_meas = ctx->M > 0 ? 1 : 0;
        a.block_records = block_records;
        a.resample_thresh = ctx->cfg.resampleThresh;
        a.new_logw = new_log_weight;
        a.seed = seed;
        a.step = step;
        a.part_sum = P.part_sum;
        a.part_s2 = P.part_s2;
        a.cdf_rel = P.cdf_rel;
        a.part_tot = P.part_tot;
        a.part_key = P.part_key;
        a.sync = ctx->d_plan_sync;
        a.out = out;
        a.parents = dev_parents;
        a.mig = ctx->d_mig;
        a.mig_host = ctx->h_mig_dev;
        a.stamps = ctx->d_stamps;  // (allocated by phd_debug_stamps only)
        a.seq = ++ctx->plan_seq;
        a.keep_src = dev_keep_src;
        a.send_src = dev_send_src;
        a.recv_rec = dev_recv_rec;
        a.pending = ctx->d_pend;
        a.pose = ctx->d_pose;
        a.src = src;
        a.new_pose = ctx->d_tmp_pose;
        a.new_src = ctx->d_tmp_src;
        a.logw_local = ctx->d_logw;
        hipLaunchKernelGGL(k_shard_plan, dim3(B), dim3(RS_THREADS), 0, ctx->stream, a);
        HIPCHK(hipGetLastError());
        return PHD_OK;
    }
    int rc = launch_rs_chunks(ctx, dev_w_all, n_total, out, seed, step, dev_parents, false, 0.f, false,
                              ctx->d_plan_sync + PLAN_BEYOND);
    if (rc) return rc;
    hipLaunchKernelGGL(k_shard_tail, dim3(1), dim3(RS_THREADS), 0, ctx->stream, (const float*)dev_w_all, ctx->n,
                       world, rank, (const float*)out, (const int*)dev_parents, ctx->d_plan_sync, ctx->d_mig,
                       ctx->h_mig_dev, dev_keep_src, dev_send_src, dev_recv_rec, (const phd_pose*)ctx->d_pose, src,
                       ctx->d_tmp_pose, ctx->d_tmp_src, ctx->d_logw, new_log_weight, block_records, ctx->d_pend,
                       ++ctx->plan_seq);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_shard_resample(phd_ctx* ctx, float* dev_w_all, int world, int rank, uint64_t seed, uint64_t step,
                       int* dev_parents, int* dev_keep_src, int* dev_send_src, int* dev_recv_rec,
                       void* dev_send_records, int send_capacity, float new_log_weight, int* demand,
                       int* send_records, int* recv_records, float* neff, int* resampled) {
    if (!ctx || !dev_w_all || !dev_parents || !dev_keep_src || !dev_send_src || !dev_recv_rec || !demand ||
        !send_records || !recv_records || world < 1 || world > 1024 || rank < 0 || rank >= world ||
        (long long)world * ctx->n > (long long)RS_MAX_CHUNKS * RS_THREADS || send_capacity < 0 || (send_capacity > 0 && !dev_send_records))
        return fail(PHD_E_ARG, "bad arguments to phd_shard_resample");
    if (ctx->cfg.nPredictParticles > 1 || ctx->n != ctx->n_base)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with n_predict_particles > 1 (shards hold n_particles each)");
    if (ctx->cfg.featureModel != PHD_FEATURE_STATIC)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with feature_model != 0");
    if (set_device(ctx)) return PHD_E_HIP;
    const int n_total = world * ctx->n;
    if (ensure_mig(ctx, world)) return PHD_E_HIP;
    // the global part and this rank's plan (k_shard_plan, or the k_rs_* chain + k_shard_tail)
    int rc = launch_shard_plan(ctx, dev_w_all, world, rank, seed, step, dev_parents, dev_keep_src, dev_send_src,
                               dev_recv_rec, new_log_weight, ctx->n);
    if (rc) return rc;
    if (send_capacity > 0) {
        if (ensure_cn(ctx)) return PHD_E_HIP;
        // records this rank sends (count on the device) from the pre-resample
        // store; they carry the new log-weight
        hipLaunchKernelGGL(k_pack, dim3(std::min(send_capacity, 256)), dim3(256), 0, ctx->stream,
                           (const int*)(ctx->d_mig + 3 * world), (const int*)dev_send_src, send_capacity,
                           ctx->cap.map_capacity, ctx->d_src, ctx->d_map[ctx->cur], ctx->d_size[ctx->cur],
                           ctx->d_map_x, ctx->d_size_x, ctx->d_pose, ctx->d_logw, 1, new_log_weight,
                           ctx->d_cn_coef, ctx->d_cn_x, rec_cn_stride(ctx), (float*)dev_send_records);
        HIPCHK(hipGetLastError());
    }
    int* h = ctx->h_mig;  // (written by the plan's tail)
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (h[3 * world + MIG_TIMEOUT])
        return fail(PHD_E_HIP, "phd_shard_resample: the one-launch plan lost residency (a wait timed out)");
    float o[2];
    memcpy(o, h + 3 * world + MIG_LSE, sizeof(o));
    const int flag = h[3 * world + MIG_FLAG];
    if (flag) {  // the remapped poses / slab references become the store
        std::swap(ctx->d_pose, ctx->d_tmp_pose);
        std::swap(ctx->d_src, ctx->d_tmp_src);
        ctx->src_fresh = false;
    }
    if (neff) *neff = o[1];
    if (resampled) *resampled = flag;
    memcpy(demand, h, world * sizeof(int));
    memcpy(send_records, h + world, world * sizeof(int));
    memcpy(recv_records, h + 2 * world, world * sizeof(int));
    if (h[3 * world] > send_capacity)
        return fail(PHD_E_CAPACITY, "phd_shard_resample: send buffer smaller than this rank's surplus records");
    return PHD_OK;
}

/* Sync-free sharded plan (see phd_capi.h). */
int phd_shard_resample_async(phd_ctx* ctx, float* dev_w_all, int world, int rank, uint64_t seed, uint64_t step,
                             int* dev_parents, int* dev_keep_src, int* dev_send_src, int* dev_recv_rec,
                             void* dev_send_blocks, int block_records, void* dev_overflow, int overflow_capacity,
                             float new_log_weight) {
    if (!ctx || !dev_w_all || !dev_parents || !dev_keep_src || !dev_send_src || !dev_recv_rec || world < 1 ||
        world > 1024 || rank < 0 || rank >= world || block_records < 0 || overflow_capacity < 0 ||
        (long long)world * ctx->n > (long long)RS_MAX_CHUNKS * RS_THREADS ||
        (world > 1 && block_records > 0 && !dev_send_blocks) || (overflow_capacity > 0 && !dev_overflow))
        return fail(PHD_E_ARG, "bad arguments to phd_shard_resample_async");
    if (ctx->plan_open) return fail(PHD_E_ARG, "phd_shard_poll the previous plan first");
    if (ctx->cfg.nPredictParticles > 1 || ctx->n != ctx->n_base)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with n_predict_particles > 1 (shards hold n_particles each)");
    if (ctx->cfg.featureModel != PHD_FEATURE_STATIC)
        return fail(PHD_E_UNSUPPORTED, "sharded resample with feature_model != 0");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ensure_mig(ctx, world)) return PHD_E_HIP;
    if (ensure_cn(ctx)) return PHD_E_HIP;
    int rc;
    if (ctx->plan_stream) {
        // the plan beside part C (phd_set_plan_stream): on the plan stream, after
        // the caller's all-gather there (which waited for phd_wait_logw); with
        // every slab reference the identity (the step's update resets them) it
        // reads none (src NULL), so part C may still be writing them.  The launch
        // chain, not the one-launch plan: its workgroups need not be resident at
        // once beside part C's, and its latency is hidden.  The pack, which reads
        // the posterior maps, waits for it on the context stream.
        if (!ctx->ev_plan) HIPCHK(hipEventCreateWithFlags(&ctx->ev_plan, kEvOrder));
        if (!ctx->src_fresh) {  // (no update since the last remap: after the whole stream)
            HIPCHK(hipEventRecord(ctx->ev_plan, ctx->stream));
            HIPCHK(hipStreamWaitEvent(ctx->plan_stream, ctx->ev_plan, 0));
        }
        hipStream_t main = ctx->stream;
        ctx->stream = ctx->plan_stream;
        rc = launch_shard_plan(ctx, dev_w_all, world, rank, seed, step, dev_parents, dev_keep_src, dev_send_src,
                               dev_recv_rec, new_log_weight, block_records, true, !ctx->src_fresh);
        ctx->stream = main;
        if (rc) return rc;
        if (PHD_PLAN_WAIT_KERNEL) {
            // the pack / the next step wait for the plan inside the context
            // stream (k_wait_plan polls the tail's sequence word), not through
            // a cross-stream event (its barrier packet: ~15 us of idle stream)
            hipLaunchKernelGGL(k_wait_plan, dim3(1), dim3(64), 0, ctx->stream,
                               (const int*)(ctx->h_mig_dev + 3 * world + MIG_SEQ), ctx->plan_seq,
                               ctx->d_plan_sync + PLAN_TIMEOUT);
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipEventRecord(ctx->ev_plan, ctx->plan_stream));
            HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_plan, 0));
        }
    } else {
        rc = launch_shard_plan(ctx, dev_w_all, world, rank, seed, step, dev_parents, dev_keep_src, dev_send_src,
                               dev_recv_rec, new_log_weight, block_records);
        if (rc) return rc;
    }
    if (world > 1) {  // records from the pre-resample store (the pointers are swapped below)
        hipLaunchKernelGGL(k_pack_blocks, dim3(std::min(ctx->n, 256)), dim3(256), 0, ctx->stream,
                           (const int*)ctx->d_mig, world, (const int*)dev_send_src, block_records, overflow_capacity,
                           ctx->cap.map_capacity, (const int*)ctx->d_src, (const float*)ctx->d_map[ctx->cur],
                           (const int*)ctx->d_size[ctx->cur], (const float*)ctx->d_map_x, (const int*)ctx->d_size_x,
                           (const phd_pose*)ctx->d_pose, new_log_weight, (const double*)ctx->d_cn_coef,
                           (const double*)ctx->d_cn_x, rec_cn_stride(ctx), (float*)dev_send_blocks,
                           (float*)dev_overflow, ctx->h_mig_dev + 3 * world + MIG_OVF_CAP);
        HIPCHK(hipGetLastError());
    }
    // the tail wrote the remapped store (the identity without a resample): swap it in
    std::swap(ctx->d_pose, ctx->d_tmp_pose);
    std::swap(ctx->d_src, ctx->d_tmp_src);
    ctx->src_fresh = false;
    // (the counts reach h_mig from the tail directly; the host polls the plan's
    // sequence number there: no event record, whose system-scope release would
    // cost the stream a gap)
    ctx->plan_ovf_cap = overflow_capacity;
    ctx->plan_open = true;
    ctx->plan_world = world;
    ctx->plan_rank = rank;
    return PHD_OK;
}

int phd_wait_logw(phd_ctx* ctx, void* stream) {
    if (!ctx || !stream) return fail(PHD_E_ARG, "bad arguments to phd_wait_logw");
    if (set_device(ctx)) return PHD_E_HIP;
    if (!ctx->ev_logw) {
        // first call: from here on every update marks its log-weights final;
        // until one has, the whole stream
        HIPCHK(hipEventCreateWithFlags(&ctx->ev_logw, kEvOrder));
        HIPCHK(hipEventRecord(ctx->ev_logw, ctx->stream));
    }
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, ctx->ev_logw, 0));
    return PHD_OK;
}

int phd_set_plan_stream(phd_ctx* ctx, void* stream) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    if (stream && !ctx->ev_logw) {
        HIPCHK(hipEventCreateWithFlags(&ctx->ev_logw, kEvOrder));
        HIPCHK(hipEventRecord(ctx->ev_logw, ctx->stream));
    }
    ctx->plan_stream = (hipStream_t)stream;
    return PHD_OK;
}

int phd_shard_receive_blocks(phd_ctx* ctx, const void* dev_recv_blocks, int block_records, const int* dev_recv_rec) {
    if (!ctx || !dev_recv_rec || block_records < 0 || (block_records > 0 && !dev_recv_blocks) || !ctx->plan_world)
        return fail(PHD_E_ARG, "bad arguments to phd_shard_receive_blocks");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ensure_x(ctx)) return PHD_E_HIP;
    ctx->src_fresh = false;
    hipLaunchKernelGGL(k_unpack_blocks, dim3(std::min(ctx->n, 256)), dim3(256), 0, ctx->stream, (const float*)dev_recv_blocks,
                       (const float*)nullptr, block_records, 0, (const int*)ctx->d_mig, ctx->plan_world,
                       ctx->plan_rank, dev_recv_rec, ctx->n, ctx->cap.map_capacity, ctx->d_map_x,
                       ctx->d_size_x, ctx->d_src, ctx->d_pose, ctx->d_logw, ctx->d_cn_x, rec_cn_stride(ctx));
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_shard_poll(phd_ctx* ctx, int* demand, int* send_records, int* recv_records, int* pending, float* neff,
                   int* resampled) {
    if (!ctx || !ctx->plan_open) return fail(PHD_E_ARG, "no sharded plan to poll");
    if (set_device(ctx)) return PHD_E_HIP;
    const int w = ctx->plan_world;
    const int* h = ctx->h_mig;
    {
        // the plan's tail stores its sequence number last (system-scope release)
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned spin = 0;; spin++) {
            if ((unsigned)__atomic_load_n(h + 3 * w + MIG_SEQ, __ATOMIC_ACQUIRE) == ctx->plan_seq) break;
            if ((spin & 1023u) == 1023u) {
                const hipError_t q = hipStreamQuery(ctx->stream);
                if (q != hipSuccess && q != hipErrorNotReady) {
                    ctx->plan_open = false;
                    return fail(PHD_E_HIP, std::string("phd_shard_poll: ") + hipGetErrorString(q));
                }
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                    ctx->plan_open = false;
                    return fail(PHD_E_HIP, "phd_shard_poll: the plan did not complete within 60 s");
                }
            }
        }
    }
    ctx->plan_open = false;
    if (demand) memcpy(demand, h, w * sizeof(int));
    if (send_records) memcpy(send_records, h + w, w * sizeof(int));
    if (recv_records) memcpy(recv_records, h + 2 * w, w * sizeof(int));
    ctx->pend_count = h[3 * w + MIG_PENDING];
    if (pending) *pending = ctx->pend_count;
    if (neff) memcpy(neff, h + 3 * w + MIG_NEFF, sizeof(float));
    if (resampled) *resampled = h[3 * w + MIG_FLAG];
    if (h[3 * w + MIG_TIMEOUT])
        return fail(PHD_E_HIP, "phd_shard_resample_async: the one-launch plan lost residency (a wait timed out)");
    if (h[3 * w + MIG_OVF_SEND] > ctx->plan_ovf_cap)  // (what k_pack_blocks flags, from the counts)
        return fail(PHD_E_CAPACITY, "phd_shard_resample_async: overflow buffer smaller than the records beyond the blocks");
    return PHD_OK;
}

int phd_shard_receive_overflow(phd_ctx* ctx, const void* dev_recv_overflow, int block_records,
                               const int* dev_recv_rec) {
    if (!ctx || !dev_recv_rec || !ctx->plan_world || ctx->plan_open)
        return fail(PHD_E_ARG, "bad arguments to phd_shard_receive_overflow (poll the plan first)");
    if (ctx->pend_count == 0) return PHD_OK;
    if (!dev_recv_overflow) return fail(PHD_E_ARG, "phd_shard_receive_overflow: pending slots need the records");
    if (set_device(ctx)) return PHD_E_HIP;
    ctx->src_fresh = false;
    hipLaunchKernelGGL(k_unpack_blocks, dim3(std::min(ctx->n, 256)), dim3(256), 0, ctx->stream, (const float*)nullptr,
                       (const float*)dev_recv_overflow, block_records, 1, (const int*)ctx->d_mig, ctx->plan_world,
                       ctx->plan_rank, dev_recv_rec, ctx->n, ctx->cap.map_capacity, ctx->d_map_x,
                       ctx->d_size_x, ctx->d_src, ctx->d_pose, ctx->d_logw, ctx->d_cn_x, rec_cn_stride(ctx));
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_update_pending(phd_ctx* ctx, const phd_ackerman_control* u, int do_predict, uint64_t step,
                       float* dev_logw_out) {
    if (!ctx || !ctx->cfg_set) return fail(PHD_E_ARG, "bad arguments to phd_update_pending");
    if (ctx->pend_count == 0) return PHD_OK;
    if (set_device(ctx)) return PHD_E_HIP;
    int rc = enqueue_predict_update(ctx, u, do_predict, step, ctx->d_pend, ctx->pend_count);
    if (rc) return rc;
    if (dev_logw_out)
        HIPCHK(hipMemcpyAsync(dev_logw_out, ctx->d_logw, ctx->n * sizeof(float), hipMemcpyDeviceToDevice,
                              ctx->stream));
    if (ctx->ev_logw) HIPCHK(hipEventRecord(ctx->ev_logw, ctx->stream));  // (the mirror is complete here)
    ctx->src_fresh = true;  // the pending slots (the only references off the identity) were re-updated
    return PHD_OK;
}

int phd_shard_receive(phd_ctx* ctx, const void* dev_records, const int* dev_recv_rec, int n_slots, int first_slot) {
    if (!ctx || n_slots < 0 || first_slot < 0 || first_slot + n_slots > ctx->n ||
        (n_slots > 0 && (!dev_records || !dev_recv_rec)))
        return fail(PHD_E_ARG, "bad arguments to phd_shard_receive");
    if (n_slots == 0) return PHD_OK;
    if (set_device(ctx)) return PHD_E_HIP;
    if (ensure_x(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_unpack_slots, dim3(n_slots), dim3(256), 0, ctx->stream, (const float*)dev_records,
                       dev_recv_rec, n_slots, first_slot, ctx->cap.map_capacity, ctx->d_map_x, ctx->d_size_x,
                       ctx->d_src, ctx->d_pose, ctx->d_logw, ctx->d_cn_x, rec_cn_stride(ctx));
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_cardinality_distribution(phd_ctx* ctx, float* cn_host) {
    if (!ctx || !cn_host) return fail(PHD_E_ARG, "null argument");
    if (!ctx->cn_valid) return fail(PHD_E_ARG, "no CPHD update has run on this context");
    if (set_device(ctx)) return PHD_E_HIP;
    const int Nmax = ctx->cfg.maxCardinality;
    const size_t bytes = (size_t)ctx->n * (Nmax + 1) * sizeof(float);
    float* d = nullptr;
    HIPCHK(hipMalloc((void**)&d, bytes));
    hipLaunchKernelGGL(k_cphd_cardinality, dim3(ctx->n), dim3(256), 0, ctx->stream, (const int*)ctx->d_src,
                       (const double*)ctx->d_cn_coef, (const double*)ctx->d_cn_x, ctx->cn_stride,
                       ctx->d_lfact, Nmax, ctx->n, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(cn_host, d, bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    hipFree(d);
    if (e != hipSuccess) return fail(PHD_E_HIP, std::string("phd_cardinality_distribution: ") + hipGetErrorString(e));
    return PHD_OK;
}

int phd_resample_count(phd_ctx* ctx, int* count) {
    if (!ctx || !count) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    unsigned c[2];
    HIPCHK(hipMemcpyAsync(&c[0], ctx->d_out + 4, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(&c[1], ctx->d_out + 44, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *count = (int)(c[0] + c[1]);
    return PHD_OK;
}

int phd_copy_log_weights(phd_ctx* ctx, float* dev_dst) {
    if (!ctx || !dev_dst) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipMemcpyAsync(dev_dst, ctx->d_logw, ctx->n * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    return PHD_OK;
}

int phd_set_log_weights(phd_ctx* ctx, const float* dev_src) {
    if (!ctx || !dev_src) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipMemcpyAsync(ctx->d_logw, dev_src, ctx->n * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    return PHD_OK;
}

int phd_record_bytes(const phd_ctx* ctx, size_t* bytes) {
    if (!ctx || !bytes) return fail(PHD_E_ARG, "null argument");
    *bytes = record_words(ctx->cap.map_capacity, rec_cn_stride(ctx)) * sizeof(float);
    return PHD_OK;
}

int phd_pack_particles(phd_ctx* ctx, const int* dev_src_idx, int count, void* dev_records) {
    if (!ctx || (count > 0 && (!dev_src_idx || !dev_records))) return fail(PHD_E_ARG, "bad arguments");
    if (count <= 0) return PHD_OK;
    if (set_device(ctx)) return PHD_E_HIP;
    if (ensure_cn(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_pack, dim3(count), dim3(256), 0, ctx->stream, (const int*)nullptr, dev_src_idx, count,
                       ctx->cap.map_capacity, ctx->d_src, ctx->d_map[ctx->cur], ctx->d_size[ctx->cur], ctx->d_map_x,
                       ctx->d_size_x, ctx->d_pose, ctx->d_logw, 0, 0.f, ctx->d_cn_coef, ctx->d_cn_x,
                       rec_cn_stride(ctx), (float*)dev_records);
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_unpack_particles(phd_ctx* ctx, const void* dev_records, const int* dev_dst_idx, int count) {
    if (!ctx || (count > 0 && (!dev_dst_idx || !dev_records))) return fail(PHD_E_ARG, "bad arguments");
    if (count <= 0) return PHD_OK;
    if (count > ctx->n) return fail(PHD_E_ARG, "more migrants than particles");
    if (set_device(ctx)) return PHD_E_HIP;
    if (ensure_x(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_unpack, dim3(count), dim3(256), 0, ctx->stream, (const float*)dev_records, dev_dst_idx,
                       (const int*)nullptr, count, ctx->cap.map_capacity, ctx->d_map_x, ctx->d_size_x, ctx->d_src,
                       ctx->d_pose, ctx->d_logw, ctx->d_cn_x, rec_cn_stride(ctx));
    HIPCHK(hipGetLastError());
    return PHD_OK;
}

int phd_expected_pose(phd_ctx* ctx, phd_pose* pose, int* map_particle) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_expected_pose, dim3(1), dim3(1024), 0, ctx->stream, ctx->d_logw, ctx->d_pose, ctx->n,
                       ctx->d_out + 16);
    HIPCHK(hipGetLastError());
    float out[7];
    HIPCHK(hipMemcpyAsync(out, ctx->d_out + 16, 7 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (pose) memcpy(pose, out, sizeof(phd_pose));
    if (map_particle) memcpy(map_particle, &out[6], sizeof(int));
    return PHD_OK;
}

int phd_cardinalities(phd_ctx* ctx, float* cn_host) {
    if (!ctx || !cn_host) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_cardinality, dim3((ctx->n + 3) / 4), dim3(256), 0, ctx->stream, ctx->d_src,
                       ctx->d_map[ctx->cur], ctx->d_size[ctx->cur], ctx->d_map_x, ctx->d_size_x, ctx->n,
                       ctx->cap.map_capacity, ctx->d_cn);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(cn_host, ctx->d_cn, ctx->n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

/* EAP expected map (computeExpectedMap main.cpp:290-316 + reduceGaussianMixture
 * gm_reduce.cpp:59-132) of the current store, on the device (phd_eap.hip). */
int phd_expected_map(phd_ctx* ctx, phd_gaussian2d* out, long out_cap, long* n_out) {
    if (!ctx || !n_out) return fail(PHD_E_ARG, "null argument");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config first");
    if (set_device(ctx)) return PHD_E_HIP;
    std::string err;
    const long nout = eap_run(&ctx->eap, ctx->stream, ctx->d_src, ctx->d_map[ctx->cur], ctx->d_size[ctx->cur],
                              ctx->d_map_x, ctx->d_size_x, ctx->d_logw, ctx->n, ctx->cap.map_capacity,
                              ctx->cfg.minSeparation, out, out ? out_cap : 0, &ctx->eap_groups, err);
    if (nout < 0) return fail(PHD_E_HIP, "expected map: " + err);
    *n_out = nout;
    if (nout > 0 && (!out || nout > out_cap))
        return fail(PHD_E_CAPACITY, "expected map has " + std::to_string(nout) + " components; out_cap too small");
    return PHD_OK;
}

/* EAP map of the dynamic maps (feature_model 2): recoverSlamState's
 * exp_map_dynamic (main.cpp:369-371) on the device (phd_mixed.hip). */
int phd_expected_map_dynamic(phd_ctx* ctx, phd_gaussian4d* out, long out_cap, long* n_out) {
    if (!ctx || !n_out) return fail(PHD_E_ARG, "null argument");
    if (!ctx->cfg_set) return fail(PHD_E_ARG, "phd_set_config first");
    if (!ctx->dyn) return fail(PHD_E_ARG, "phd_enable_dynamic not called");
    if (set_device(ctx)) return PHD_E_HIP;
    std::string err;
    const long nout = mixed_expected_map_dynamic(ctx->stream, ctx->d_src, ctx->d_dmap[ctx->dcur],
                                                 ctx->d_dsize[ctx->dcur], ctx->n, ctx->dcap, ctx->d_logw,
                                                 ctx->cfg.minSeparation, out, out ? out_cap : 0, err);
    if (nout < 0) return fail(PHD_E_HIP, "dynamic expected map: " + err);
    *n_out = nout;
    if (nout > 0 && (!out || nout > out_cap))
        return fail(PHD_E_CAPACITY, "dynamic expected map has " + std::to_string(nout) + " components; out_cap too small");
    return PHD_OK;
}

int phd_expected_map_groups(phd_ctx* ctx, int* groups) {
    if (!ctx || !groups) return fail(PHD_E_ARG, "null argument");
    *groups = ctx->eap_groups;
    return PHD_OK;
}

/* Local LSE parts for a cross-rank log-sum-exp: out_host[0] = max, out_host[1] = Σexp(w - max). */
int phd_lse_parts(phd_ctx* ctx, float* out_host) {
    if (!ctx || !out_host) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    hipLaunchKernelGGL(k_lse_parts, dim3(1), dim3(1024), 0, ctx->stream, ctx->d_logw, ctx->n, ctx->d_out + 32);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out_host, ctx->d_out + 32, 2 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

/* Turn the per-update capacity check (one 4-B D2H + sync) on/off; the bench
 * turns it off inside the timed loop and checks once at the end. */
int phd_set_check_each_update(phd_ctx* ctx, int on) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    ctx->check_each_update = on != 0;
    return PHD_OK;
}

/* Diagnostic: copy the per-workgroup phase stamps of the last update (PHD_STAMPS builds). */
int phd_debug_stamps(phd_ctx* ctx, unsigned long long* host, int enable) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    if (enable && !ctx->d_stamps) {
        HIPCHK(hipMalloc((void**)&ctx->d_stamps, (size_t)ctx->nmax * PHD_STAMP_SLOTS * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(ctx->d_stamps, 0, (size_t)ctx->nmax * PHD_STAMP_SLOTS * sizeof(unsigned long long), ctx->stream));
    }
    if (host && ctx->d_stamps) {
        HIPCHK(hipMemcpyAsync(host, ctx->d_stamps, (size_t)ctx->n * PHD_STAMP_SLOTS * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    return PHD_OK;
}

int phd_set_update_threads(phd_ctx* ctx, int threads) {
    if (!ctx || !(threads == 0 || threads == 256 || threads == 512 || threads == 1024))
        return fail(PHD_E_ARG, "threads must be 0 (automatic), 256, 512 or 1024");
    if (set_device(ctx)) return PHD_E_HIP;
    return configure_update_launch(ctx, threads);
}

int phd_set_edge_pool(phd_ctx* ctx, int pool) {
    if (!ctx || pool < 0 || pool > 32768) return fail(PHD_E_ARG, "edge pool must be 0 (automatic) .. 32768");
    if (set_device(ctx)) return PHD_E_HIP;
    const int old = ctx->epool_req;
    ctx->epool_req = pool;
    const int rc = configure_update_launch(ctx, ctx->upd_threads_req);
    if (rc) ctx->epool_req = old;
    return rc;
}

int phd_set_pair_list_cap(phd_ctx* ctx, int pairs) {
    if (!ctx || pairs < 0) return fail(PHD_E_ARG, "pair-list cap must be >= 0 (0: the layout's)");
    ctx->plreq = pairs;
    return PHD_OK;
}

int phd_set_update_form(phd_ctx* ctx, int form) {
    if (!ctx || form < 0 || form > 2) return fail(PHD_E_ARG, "form must be 0 (automatic), 1 (fused) or 2 (split)");
    if (set_device(ctx)) return PHD_E_HIP;
    const int old = ctx->upd_form_req;
    ctx->upd_form_req = form;
    const int rc = configure_update_launch(ctx, ctx->upd_threads_req);
    if (rc) ctx->upd_form_req = old;
    return rc;
}

int phd_update_form(phd_ctx* ctx, int* split) {
    if (!ctx || !split) return fail(PHD_E_ARG, "null argument");
    *split = ctx->upd_split;
    return PHD_OK;
}

int phd_update_threads(phd_ctx* ctx, int* threads, size_t* lds_bytes, int* resident) {
    if (!ctx) return fail(PHD_E_ARG, "null context");
    if (threads) *threads = ctx->upd_threads;
    if (lds_bytes) *lds_bytes = ctx->upd_lds;
    if (resident) *resident = ctx->upd_resident;
    return PHD_OK;
}

int phd_set_merge_mode(phd_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 1) return fail(PHD_E_ARG, "bad arguments");
    ctx->merge_mode = mode;
    return PHD_OK;
}

int phd_merge_fallbacks(phd_ctx* ctx, int* count) {
    if (!ctx || !count) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    int v[2];
    HIPCHK(hipMemcpyAsync(v, ctx->d_err, 2 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *count = v[1];
    HIPCHK(hipMemsetAsync(ctx->d_err + 1, 0, sizeof(int), ctx->stream));
    return PHD_OK;
}

/* read and clear one of the counters after the sticky error word */
static int take_counter(phd_ctx* ctx, int k, int* count) {
    if (!ctx || !count) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    int v = 0;
    HIPCHK(hipMemcpyAsync(&v, ctx->d_err + k, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *count = v;
    HIPCHK(hipMemsetAsync(ctx->d_err + k, 0, sizeof(int), ctx->stream));
    return PHD_OK;
}

int phd_status_errors(phd_ctx* ctx, int* count) { return take_counter(ctx, 3, count); }

int phd_particle_status(phd_ctx* ctx, int* host_status) {
    if (!ctx || !host_status) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    HIPCHK(hipMemcpyAsync(host_status, ctx->d_status, ctx->n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PHD_OK;
}

int phd_merge_pair_overflows(phd_ctx* ctx, int* count) {
    if (!ctx || !count) return fail(PHD_E_ARG, "null argument");
    if (set_device(ctx)) return PHD_E_HIP;
    int v = 0;
    HIPCHK(hipMemcpyAsync(&v, ctx->d_err + 2, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *count = v;
    HIPCHK(hipMemsetAsync(ctx->d_err + 2, 0, sizeof(int), ctx->stream));
    return PHD_OK;
}

int phd_check_errors(phd_ctx* ctx) {
    if (!ctx) return fail(PHD_E_ARG, "null ctx");
    if (set_device(ctx)) return PHD_E_HIP;
    return check_err(ctx);
}

}  // extern "C"
