/*
 * phd_kernels.h — kernel argument structs, LDS layout and launch declarations
 * shared by phd_kernels.hip and phd_capi.hip.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "phd_device.h"
#include "phd_types.h"

/* threads per particle of the fused update (one workgroup per particle) */
/* bearing bins of the banded pair loop's measurement index */
#define PHD_ZBINS 256
/* per-workgroup clock stamps of the diagnostic build */
#define PHD_STAMP_SLOTS 52
#define UPD_THREADS_MIN 256
#define UPD_THREADS_MAX 1024
#define PHD_CPHD_MAX_M 127  /* CPHD: measurements per step (two ESF coefficients per lane) */
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 4
#define PHD_CPHD_SEG 2
#elif defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 5
#define PHD_CPHD_SEG 1
#else
#define PHD_CPHD_SEG 4 /* CPHD: measurements per wave segment of the ESF sweep */
#endif

/* per-particle status bits of the fused update */
#define PHD_ST_SURVIVOR_OVERFLOW 1
#define PHD_ST_CANDIDATE_OVERFLOW 2
#define PHD_ST_MAP_OVERFLOW 4
#define PHD_ST_SERIAL_MERGE 8 /* informational: the particle used the serial merge fallback */
#define PHD_ST_ETA_RANGE 16     /* a likelihood term >= 2^20: the fixed-point eta sum may overflow */
#define PHD_ST_PAIR_OVERFLOW 32 /* informational: the merge walked twice (culled pair list overflow) */
#define PHD_ST_WAIT_TIMEOUT 64  /* an in-launch wait of the one-launch resample gave up: results invalid */
#define PHD_ST_INFO (PHD_ST_SERIAL_MERGE | PHD_ST_PAIR_OVERFLOW) /* bits that are not errors */

/* slab reference encoding in the index table: bit 30 selects the migration set X */
#define PHD_SLAB_X 0x40000000
#define PHD_SLAB_MASK 0x3fffffff

#include <string>

namespace phd {

struct PredictCfg {
    int index_offset; /* global id of local particle 0: RNG counter = index_offset + i */
    float dt;
    int subdivide;
    float l, h, a, b;
    float stdAlpha, stdEncoder;
    float ax, ay, ayaw;
};

struct RsStepArgs {
    const float* w;
    float* w_out;
    int N, B, has_meas;
    float resample_thresh, new_logw;
    uint64_t seed, step;
    double* part_s2;
    unsigned long long *cdf_rel, *part_tot, *part_key;
    unsigned* sync;
    float* out;
    int* parents;
    const phd_pose* pose;
    const int* src;
    phd_pose* new_pose;
    int* new_src;
    float* logw;
    int* err;
};

/* part C's lead workgroups (PHD_RS_LEAD of them, RS_LEAD_WGS): the first runs
 * phd_step's normalise / nEff / decision / resample (rs_step_block: k_rs_step's
 * arithmetic, the same bits), the rest return at once — so the particles keep
 * their XCD (upd_particle) and no second stream or cross-stream event sits on
 * the step's critical path */
#define RS_LEAD_WGS 8

struct UpdateArgs {
    int n, cap, M, Mcap, Kcap, Scap;
    int Epool;      /* undirected-edge pool of the parallel merge */
    int plreq;      /* culled-pair list cap (phd_set_pair_list_cap; 0 = the layout's) */
    int Bbuckets;   /* merge lattice buckets (upd_buckets) */
    int merge_mode; /* 0 = parallel exact merge (serial fallback), 1 = serial only */
    const int* slots;     /* particle of workgroup b = slots[b] (NULL = first + b): a re-update of some slots */
    int first;            /* first particle of this launch (a chunk of the update on its own stream) */
    int prio;             /* trailing workgroups at the highest wave priority (prio_tail, 0 = none) */
    int order;            /* 0: particle first + b; 1: groups of 8 in reverse (upd_particle) */
    unsigned char* hand;  /* three-launch CPHD update: per-particle handoff (cphd_hand_layout) */
    const int* src;       /* slab reference per particle (NULL = identity) */
    int* src_reset;       /* if non-NULL, set to identity after the update */
    const float* map_x;   /* migration slab set X */
    const int* size_x;
    const float* map_in;
    float* map_out;
    const int* size_in;
    int* size_out;
    phd_pose* poses; /* written by the fused predict */
    float* logw;
    float* logw_out; /* optional mirror of every updated log-weight (the sharded step's all-gather input) */
    float* delta;
    const float* zr;
    const float* zb;
    const int* zok;
    const float4* zs; /* valid measurements sorted by wrapped bearing: (range, bearing, index bits, key) */
    const unsigned short* zbin; /* PHD_ZBINS entries: first sorted measurement with key >= -pi + b * 2pi / PHD_ZBINS */
    int Mv;
    int zwide;        /* some |bearing| >= 3 (wave walk: general wrapAngle instead of the branch-free one) */
    int* status;
    int* err;
    unsigned long long* stamps; /* diagnostic build only (PHD_STAMPS) */
    /* fused predict (phd_step): 0 none, 1 Ackerman, 2 CV; device Philox noise */
    int predict;
    phd_ackerman_control pu;
    PredictCfg pc;
    uint64_t pseed, pstep;
    const phd_pose* pose_prior; /* replay: fixed prior poses / log-weights restored first */
    const float* logw_prior;
    /* births of the step (CPHD: the previous scan's inverse measurements,
     * phdfilter.cu.bak:738-870): prior components G .. G + Mb - 1 of the update
     * after the slab's G; the classify (part A / the fused update) places birth
     * j from the pose and valid measurement bzvi[j] of the rows bzr / bzb and
     * writes it to row j of the particle's birth slab (births + n 7 cap), where
     * the later phases (part C) read it (NULL: none) */
    float* births;
    int Mb;
    const float* bzr;
    const float* bzb;
    const int* bzvi;
    /* CPHD (filter_type 1): per-particle cardinality coefficients out, log n! table */
    double* cn_coef;
    int cn_stride;
    const double* lfact;
    int Nmax;
    DevCfg c;
    int rs_lead;   /* part C: RS_LEAD_WGS lead workgroups before the particles' (0: none) */
    RsStepArgs rs; /* their resample (rs_lead) */
};

/* Particle of workgroup b.  order 1 walks the launch's full groups of 8
 * particles last-written-first, keeping each particle's position in its group:
 * workgroups are dealt round-robin to the 8 XCDs, so particle n still runs on
 * XCD n mod 8 — the one whose L2 holds what the previous launch wrote for it —
 * and the particles that launch wrote last (still in that L2) are read first. */
__host__ __device__ inline int upd_particle(const UpdateArgs& a, int b, int grid) {
    if (a.slots) return a.slots[b];
    const int g8 = grid & ~7;
    if (a.order == 1 && b < g8) b = g8 - 8 - (b & ~7) + (b & 7);
    return a.first + b;
}

/* Byte offsets into the fused update's dynamic LDS.
 *   A (whole kernel): measurements, normalisers, eta partials, out-of-range list, scratch
 *   C (union): component pair table (phases 2-3) |
 *              candidates (phase 4 on) + merge adjacency (phase 5)
 *   D (union): in/near lists + detection-term keys (phases 1-4) | merge cell index (phase 5) */
struct UpdLds {
    size_t zr, zb, zok, leta, zs, etafx, etalo, zbin, out, cnt, scr, red, redf, pose, uni, thr;
    size_t u;                                // region C: candidate records P
    size_t detv;                             // region C: detection covariances (the tags ride in the records)
    size_t mpar, moff, mcur, medge, mpool;   // region C, merge adjacency (after the candidates; moff = mcur)
    size_t in, near, skey, skey2;            // region D, phases 1-4
    size_t skeyidx, gstart;                  // region D, merge (part C: gstart over cur | edges when they hold it)
    size_t total;
    int B;                                   // merge lattice buckets of this layout
};

__host__ __device__ inline size_t upd_align16(size_t x) { return (x + 15) & ~(size_t)15; }

/* PHD_RS_OVERLAP: phd_step's one-launch resample runs on a second
 * (high-priority) stream beside part C, whose tail leaves CUs idle, as soon as
 * the log-weights are final — after the terms launch of a CPHD step (bit 1),
 * after part A of a split PHD step (bit 2).  3 = shipped; a cleared bit is the
 * diagnostic variant that runs that form's resample after part C. */
#ifndef PHD_RS_OVERLAP
#define PHD_RS_OVERLAP 3
#endif
#ifndef PHD_RS_LEAD
/* 1: the overlapped resample runs in part C's lead workgroup (UpdateArgs::
 * rs_lead) instead of on a second stream beside part C (0) */
#define PHD_RS_LEAD 1
#endif


/* Part C's merge lattice: the largest of 32x32 .. PHD_PARTC_BMAX buckets (64x32
 * = 2048, 64x64 = 4096) whose starts fit over the dead degree / edge memory
 * (no LDS of their own; a variant value is defined for every source of a
 * build).  Fewer aliased neighbour tests with more buckets. */
#ifndef PHD_PARTC_BMAX
#define PHD_PARTC_BMAX 1024
#endif
static_assert(PHD_PARTC_BMAX == 1024 || PHD_PARTC_BMAX == 2048 || PHD_PARTC_BMAX == 4096,
              "PHD_PARTC_BMAX: 1024, 2048 or 4096 buckets");

/* merge lattice buckets: 32x32 (Kcap <= 1024), 64x32 (<= 2048), 64x64 (<= 8192), 128x128.
 * Part C's bucket starts live over the dead degree / edge memory whenever that
 * region holds them (upd_lds_layout; then 32x32 also at Kcap <= 768, whose
 * starts of its own would be a 32x16 lattice). */
__host__ __device__ inline int upd_buckets(int Kcap, int part = 0) {
    return Kcap <= 768 && part == 2 ? 512 : Kcap <= 1024 ? 1024 : Kcap <= 2048 ? 2048 : Kcap <= 8192 ? 4096 : 16384;
}

/* default undirected-edge pool of the parallel merge */
__host__ __device__ inline int upd_epool(int Kcap) { return (3 * Kcap) / 2 + 16; }

/* part: 0 the whole update in one kernel; CPHD in three launches: 1 = part A
 * (classify, pair table, walk; ends at the handoff), 2 = part C (from the
 * handoff: survivors, candidates, merge) — part A needs no merge scratch, part C
 * no CPHD scratch (the CPHD terms run in between, k_cphd_terms). */
__host__ __device__ inline UpdLds upd_lds_layout(int cap, int Mcap, int Kcap, int Scap, int Epool, int NT,
                                                  int cphd = 0, int part = 0) {
    UpdLds L;
    const int B = upd_buckets(Kcap, part);
    size_t o = 0;
    // (the split CPHD parts read the raw measurements, the normalisers and the
    // listing bounds from global memory (part C) or not at all (part A): sized 0)
    const bool pz = part != 0;
    L.zr = o;
    o = upd_align16(o + (pz ? 0 : 4 * (size_t)Mcap));
    L.zb = o;
    o = upd_align16(o + (pz ? 0 : 4 * (size_t)Mcap));
    L.zok = o;
    o = upd_align16(o + (pz ? 0 : 4 * (size_t)Mcap));
    L.leta = o;  // (the PHD part C computes its normalisers here; the CPHD one reads the terms' from the handoff)
    o = upd_align16(o + (pz && !(part == 2 && !cphd) ? 0 : 4 * (size_t)Mcap));
    // part C reads the sorted measurements, their bins and the out-of-range list
    // from global memory (pass 1 only / the handoff) and has no eta sums
    const bool pc = part == 2;
    const bool pa = part == 1;  // part A writes its in / near / out lists straight into the handoff
    L.zs = o;
    o = upd_align16(o + (pc ? 0 : 16 * (size_t)Mcap));
    L.etafx = o;
    o = upd_align16(o + (pc ? 0 : 8 * (size_t)Mcap));
    L.etalo = o;
    o = upd_align16(o + (pc ? 0 : 8 * (size_t)Mcap));
    L.zbin = o;
    o = upd_align16(o + (pc ? 0 : 2 * (size_t)PHD_ZBINS));
    L.out = o;
    o = upd_align16(o + (pc || pa ? 0 : 2 * (size_t)cap));
    L.cnt = o;
    o = upd_align16(o + 4 * 16);
    // part C: block-helper scratch (two buffers), block_sum<4> and merge_serial's
    // reductions only; the other forms keep room for classification / CPHD
    L.scr = o;
    o = upd_align16(o + (pc ? 4 * 2 * (size_t)(NT / 64) : 4 * 64));
    L.red = o;
    o = upd_align16(o + (pc ? 8 * 4 * (size_t)(NT / 64) : 8 * 64));
    L.redf = o;
    o = upd_align16(o + (pc ? 4 * (32 + (size_t)(NT / 64)) : 4 * 64));
    L.pose = o;
    o = upd_align16(o + sizeof(phd_pose));
    L.uni = o;  // workgroup-uniform values kept in LDS across phases (not in VGPRs)
    o = upd_align16(o + 8 * 8);
    L.thr = o;
    o = upd_align16(o + (cphd && !pz ? 4 * (size_t)Mcap : 0));
    // region C
    const size_t c0 = o;
    L.u = o;
    size_t m = c0 + 16 * (size_t)Kcap;  // candidate records P (with their tags) | detection / birth covariances
    L.detv = m;
    // detection (+ birth: PHD only) covariances; part C keeps them in its handoff
    m = upd_align16(m + (pc ? 0 : 16 * ((size_t)Scap + (cphd ? 0 : (size_t)Mcap))));
    L.mcur = m;
    m = upd_align16(m + 2 * ((size_t)Kcap + 2));
    L.medge = m;
    m = upd_align16(m + 4 * (size_t)Epool);
    // par | off | pool contiguous: the culled-pair list aliases them before the CSR exists
    L.mpar = m;
    m = upd_align16(m + 2 * (size_t)Kcap);
    // the CSR offsets are the degree cursors after the scatter (each ends at its
    // row's start; cur[K] holds the total): no array of their own (round 5:
    // 1.7 KB at config 3, part C's sixth workgroup per CU)
    L.moff = L.mcur;
    L.mpool = m;
    m = upd_align16(m + 4 * (size_t)Epool);
    size_t table = c0 + (size_t)cap * (8 * 4) + 16 + 2 * (size_t)NT;
    // (part C keeps the pair table of its rare pass-1 rebuild in the handoff)
    o = upd_align16(part == 1 || (part != 2 && table > m) ? table : m);
    // region D
    const size_t d0 = o;
    // in / near lists: part C reads them from its handoff
    L.in = o;
    o = upd_align16(o + (pc || pa ? 0 : 2 * (size_t)cap));
    L.near = o;
    o = upd_align16(o + (pc || pa ? 0 : 2 * (size_t)cap));
    const size_t skb = upd_align16(4 * ((size_t)Scap + 4));
    if (pc && L.mpool + 4 * (size_t)Epool >= L.mcur + 2 * skb) {
        // part C: the survivor keys and their order live over the merge
        // adjacency (cur .. pool), dead until the merge — region D then holds
        // only the merge's cell-order index
        L.skey = L.mcur;
        L.skey2 = L.mcur + skb;
    } else {
        L.skey = o;  // (part A lists into its handoff)
        o = upd_align16(o + (pa ? 0 : skb));
        L.skey2 = o;  // (the survivor order: not in part A)
        o = upd_align16(o + (pa ? 0 : skb));
    }
    const size_t d_a = o;
    o = d0;
    L.skeyidx = o;
    o = upd_align16(o + 2 * (size_t)Kcap);
    L.B = B;
    // part C: the degree counters and the edge list are dead until the exact
    // distances, so the bucket starts live there during the bucket sort and the
    // cull walk: the largest lattice up to PHD_PARTC_BMAX buckets (at least
    // 32 x 32, at least upd_buckets' for the candidate capacity) that fits
    int Bp = 0;
    if (part == 2) {
        const int bmin = B > 1024 ? B : 1024;
        for (int b = PHD_PARTC_BMAX > bmin ? PHD_PARTC_BMAX : bmin; b >= bmin && !Bp; b >>= 1)
            if (L.mpar - L.mcur >= 2 * ((size_t)b + 2)) Bp = b;
    }
    if (Bp) {
        L.B = Bp;
        L.gstart = L.mcur;
    } else {
        L.gstart = o;
        o = upd_align16(o + 2 * ((size_t)L.B + 2));
    }
    L.total = (part == 1 || o <= d_a) ? d_a : o;
    return L;
}

/* Per-particle handoff of the three-launch CPHD update (global scratch,
 * hand_stride bytes per particle): part A's counts, sums, eta fixed point,
 * index lists and listed detection terms; k_cphd_terms' per-measurement
 * factors / listing bounds, non-detection factor and wide flag. */
struct CphdHand {
    size_t cnt, sums, ehi, elo, in, near, out, skey, leta, thr, misc, detv, table, rb, stride;
};
#define HAND_GIN 0
#define HAND_GNEAR 1
#define HAND_GOUT 2
#define HAND_NSURV 3
#define HAND_FLAGS 4
__host__ __device__ inline CphdHand cphd_hand_layout(int cap, int Mcap, int Scap) {
    CphdHand H;
    size_t o = 0;
    H.cnt = o;
    o += 64;  // 16 ints
    H.sums = o;
    o += 32;  // card, win, qd, wall (double)
    H.ehi = o;
    o = upd_align16(o + 8 * (size_t)Mcap);
    H.elo = o;
    o = upd_align16(o + 8 * (size_t)Mcap);
    H.in = o;
    o = upd_align16(o + 2 * (size_t)cap);
    H.near = o;
    o = upd_align16(o + 2 * (size_t)cap);
    H.out = o;
    o = upd_align16(o + 2 * (size_t)cap);
    H.skey = o;
    o = upd_align16(o + 4 * (size_t)Scap);
    H.leta = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    H.thr = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    H.misc = o;  // float non-detection log factor, int wide
    o = upd_align16(o + 16);
    H.detv = o;  // part C: covariances of its detection (and, PHD, birth) candidates (out of LDS)
    o = upd_align16(o + 16 * ((size_t)Scap + (size_t)Mcap));
    H.table = o;  // part C: the pair table of its rare pass-1 rebuild (out of LDS)
    o = upd_align16(o + 32 * (size_t)cap + 16 + 2 * 1024);
    H.rb = o;  // part A -> part C: (range, bearing) of each in-range component (its in-list index)
    o = upd_align16(o + 8 * (size_t)cap);
    H.stride = (o + 255) & ~(size_t)255;
    return H;
}

__global__ void k_predict_ackerman(phd_pose* poses, int n, phd_ackerman_control u, const phd_ackerman_noise* noise_in,
                                   PredictCfg c, uint64_t seed, uint64_t step, const phd_pose* pose_prior,
                                   const float* logw_prior, float* logw, const int* slots);
__global__ void k_expand(int n, int npp, const phd_pose* pose, const int* src, const float* logw, phd_pose* new_pose,
                         int* new_src, float* new_logw, float log_npp);
__global__ void k_predict_cv(phd_pose* poses, int n, const phd_cv_noise* noise_in, PredictCfg c, uint64_t seed,
                             uint64_t step, const phd_pose* pose_prior, const float* logw_prior, float* logw,
                             const int* slots);
__global__ void k_update_fused_256(UpdateArgs a);
__global__ void k_update_fused_512(UpdateArgs a);
__global__ void k_update_fused_1024(UpdateArgs a);
/* three-launch CPHD update: part A (k_update_cphd_a_*), the CPHD terms
 * (k_cphd_terms, one wave per particle, phd_terms.hip), part C (k_update_cphd_c_*) */
__global__ void k_update_cphd_a_256(UpdateArgs a);
__global__ void k_update_cphd_a_512(UpdateArgs a);
__global__ void k_update_cphd_a_1024(UpdateArgs a);
__global__ void k_update_cphd_a_p256(UpdateArgs a);  /* part A with the particle's fused predict */
__global__ void k_update_cphd_a_p512(UpdateArgs a);
__global__ void k_update_cphd_c_256(UpdateArgs a);
__global__ void k_update_cphd_c_512(UpdateArgs a);
__global__ void k_update_cphd_c_1024(UpdateArgs a);
/* split PHD update: part A -> part C through the same handoff (no terms launch) */
__global__ void k_update_phd_a_256(UpdateArgs a);
__global__ void k_update_phd_a_512(UpdateArgs a);
__global__ void k_update_phd_a_1024(UpdateArgs a);
__global__ void k_update_phd_c_256(UpdateArgs a);
__global__ void k_update_phd_c_512(UpdateArgs a);
__global__ void k_update_phd_c_1024(UpdateArgs a);
/* the CPHD weight terms of the three-launch update: one wave per particle from
 * part A's handoff (eta fixed point, sums) to part C's (factors, listing
 * bounds, non-detection factor, wide flag); Δ log w, cardinality coefficients
 * (phd_terms.hip).  Dynamic LDS: cphd_terms_lds(Mcap). */
__global__ void k_cphd_terms(UpdateArgs a);
inline size_t cphd_terms_lds(int Mcap) { return (size_t)7 * 8 * ((size_t)Mcap + 4); }
__global__ void k_cphd_cardinality(const int* src, const double* cn_coef, const double* cn_x, int stride,
                                   const double* lfact, int Nmax, int n, float* out);
__global__ void k_update_fused_p256(UpdateArgs a);
__global__ void k_update_fused_p512(UpdateArgs a);
__global__ void k_normalize(float* logw, int n, const float* lse_override, float* out, float resample_thresh,
                            int has_meas);
__global__ void k_lse_parts(const float* logw, int n, float* out);
__global__ void k_resample(const int* flag, const float* logw_in, float* logw_out, int n, int n_out,
                           const double* u_in,
                           uint64_t seed, uint64_t step, unsigned long long* cdf, int* idx, phd_pose* pose, int* src,
                           phd_pose* tmp_pose, int* tmp_src, float new_logw);
/* resample CDF kept in LDS up to this many particles (8 B each) */
#define RS_LDS_MAX 8192
__global__ void k_normalize_resample(float* logw, int n, float* out, float resample_thresh, int has_meas, uint64_t seed,
                                     uint64_t step, unsigned long long* cdf, int* idx, phd_pose* pose, int* src,
                                     phd_pose* tmp_pose, int* tmp_src, float new_logw);
__global__ void k_apply_parents(const int* flag, const int* idx, int n, phd_pose* pose, int* src, float* logw,
                                phd_pose* tmp_pose, int* tmp_src, float new_logw);
__global__ void k_add_births(int* src, const int* slots, int n, int cap, const float* map_in, const int* size_in,
                             const float* map_x, const int* size_x, float* map_out, int* size_out,
                             const phd_pose* pose, const float* zr, const float* zb, const int* zok, int M, DevCfg c,
                             int* status, int* err);
#define RS_THREADS 1024    /* threads of the resample / normalisation blocks */
#define RS_STAGE_CHUNKS 4  /* k_rs_search stages the CDF in LDS up to this many chunks (32 KB) */
#define RS_MAX_CHUNKS 1024 /* sharded plan: at most 1024 chunks of RS_THREADS (1M particles job-wide) */
__global__ void k_rs_max(const float* w, int N, float* part_max);
/* max_of_w: every block takes the max of all N entries itself and stores it as
 * its chunk's partial for k_rs_cdf (no k_rs_max launch; small N) */
__global__ void k_rs_sum(const float* w, int N, const float* part_max, int B, double* part_sum, int max_of_w);
__global__ void k_rs_cdf(float* w, int N, const float* part_max, const double* part_sum, int B, double* part_s2,
                         unsigned long long* cdf_rel, unsigned long long* part_tot, unsigned long long* part_key,
                         float* out);
__global__ void k_rs_search(int N, int B, const double* part_s2, const unsigned long long* part_tot,
                            const unsigned long long* part_key, const unsigned long long* cdf_rel,
                            float resample_thresh, int has_meas, uint64_t seed, uint64_t step, int* parents,
                            float* out, const phd_pose* pose, const int* src, phd_pose* new_pose, int* new_src,
                            float* logw, float new_logw, const float* w_norm, unsigned* beyond);
__global__ void k_rs_sumcdf(const float* w, float* w_out, int N, int B, double* part_s2, unsigned long long* cdf_rel,
                            unsigned long long* part_tot, unsigned long long* part_key, float* out);
/* mig[] of a sharded plan: [0, w) demand, [w, 2w) records sent to each rank,
 * [2w, 3w) records received from each rank, then MIG_SENT (records sent),
 * MIG_LSE, MIG_NEFF, MIG_FLAG (resample decided), MIG_PENDING (slots whose
 * record is beyond the fixed blocks), MIG_OVF_SEND / MIG_OVF_RECV (records
 * beyond the fixed blocks), MIG_OVF_CAP (the overflow buffer was too small),
 * MIG_TIMEOUT (an in-launch wait of k_shard_plan gave up: not every workgroup
 * was resident), MIG_SEQ (the plan's sequence number, stored last into the
 * host's copy: the host polls it instead of an event) */
#define MIG_SENT 0
#define MIG_LSE 1
#define MIG_NEFF 2
#define MIG_FLAG 3
#define MIG_PENDING 4
#define MIG_OVF_SEND 5
#define MIG_OVF_RECV 6
#define MIG_OVF_CAP 7
#define MIG_TIMEOUT 8
#define MIG_SEQ 9
#define MIG_TAIL 10
/* words of the plan's in-launch hand-offs (zeroed once at allocation; the
 * launch's last workgroup zeroes them for the next launch) */
#define PLAN_ARRIVE0 0
#define PLAN_ARRIVE1 1
#define PLAN_TICKET 2
#define PLAN_BEYOND 3 /* strata past the CDF's end: max of N - j */
#define PLAN_TIMEOUT 4
#define PLAN_SYNC_WORDS 5
#define STEP_ARRIVE 8 /* k_rs_step's wait, ticket and timeout words (same block) */
#define STEP_TICKET 9
#define STEP_TIMEOUT 10
__global__ void k_shard_tail(const float* w_all, int n, int world, int rank, const float* out, const int* parents,
                             unsigned* sync, int* mig, int* mig_host, int* keep_src, int* send_src, int* recv_rec,
                             const phd_pose* pose, const int* src, phd_pose* new_pose, int* new_src,
                             float* logw_local, float new_logw, int block_records, int* pending, unsigned seq);
/* The context stream's wait for a plan launched on the plan stream: one lane
 * polls the plan tail's sequence word (host-mapped, stored last with a
 * system-scope release), bounded (a timeout goes to sync_timeout, which the
 * next plan's tail reports) */
__global__ void k_wait_plan(const int* seqw, unsigned seq, unsigned* sync_timeout);
/* PHD_PLAN_WAIT_KERNEL: that kernel in place of a cross-stream event wait */
#ifndef PHD_PLAN_WAIT_KERNEL
#define PHD_PLAN_WAIT_KERNEL 1
#endif
/* k_shard_plan's arguments: the gathered log-weights (normalised in place), the
 * chunk partials, the hand-off words, and the tail's outputs (as k_shard_tail) */
struct ShardPlanArgs {
    float* w;
    int N, B, n, world, rank, has_meas, block_records;
    float resample_thresh, new_logw;
    uint64_t seed, step;
    double *part_sum, *part_s2;
    unsigned long long *cdf_rel, *part_tot, *part_key;
    unsigned* sync;
    float* out;
    int *parents, *mig, *keep_src, *send_src, *recv_rec, *pending;
    int* mig_host; /* host-mapped copy of mig (the host's read of the plan) */
    unsigned seq;  /* stored into mig_host[3 world + MIG_SEQ] after everything else */
    unsigned long long* stamps; /* diagnostic builds (PHD_PLAN_STAMPS): phase clocks, else unused */
    const phd_pose* pose;
    const int* src;
    phd_pose* new_pose;
    int* new_src;
    float* logw_local;
};
__global__ void k_shard_plan(ShardPlanArgs a);
/* k_rs_step's arguments: k_rs_sumcdf's and k_rs_search's (remap form) */
__global__ void k_rs_step(RsStepArgs a);
__global__ void k_pack_blocks(const int* mig, int world, const int* send_src, int block_records, int ovf_capacity,
                              int cap, const int* src, const float* map_in, const int* size_in, const float* map_x,
                              const int* size_x, const phd_pose* pose, float logw_value, const double* cn,
                              const double* cn_x, int cn_stride, float* blocks, float* ovf, int* ovf_flag);
__global__ void k_unpack_blocks(const float* blocks, const float* ovf, int block_records, int overflow, const int* mig,
                                int world, int rank, const int* recv_rec, int n, int cap, float* map_x, int* size_x,
                                int* src, phd_pose* pose, float* logw, double* cn_x, int cn_stride);
/* Particle record (cross-rank migration): [pose 6 | logw | size | map 7*cap]
 * 32-bit words, then (CPHD contexts) cn_stride doubles of cardinality
 * coefficients. */
__host__ __device__ inline size_t record_words(int cap, int cn_stride) {
    return 8 + (size_t)7 * cap + 2 * (size_t)cn_stride;
}
__global__ void k_unpack_slots(const float* rec, const int* slot_rec, int nslots, int first_slot, int cap, float* map_x,
                               int* size_x, int* src, phd_pose* pose, float* logw, double* cn_x, int cn_stride);
__global__ void k_pack(const int* dcount, const int* src_idx, int count, int cap, const int* src, const float* map_in,
                       const int* size_in, const float* map_x, const int* size_x, const phd_pose* pose,
                       const float* logw, int logw_set, float logw_value, const double* cn, const double* cn_x,
                       int cn_stride, float* rec);
__global__ void k_unpack(const float* rec, const int* dst_idx, const int* x_slot, int count, int cap, float* map_x,
                         int* size_x, int* src, phd_pose* pose, float* logw, double* cn_x, int cn_stride);
__global__ void k_expected_pose(const float* logw, const phd_pose* pose, int n, float* out);
__global__ void k_cardinality(const int* src, const float* map_in, const int* size_in, const float* map_x,
                              const int* size_x, int n, int cap, float* cn);

/* EAP expected map (phd_eap.hip) */
struct EapScratch;
void eap_free(EapScratch* s);
long eap_run(EapScratch** sp, hipStream_t st, const int* d_src, const float* d_map, const int* d_size,
             const float* d_map_x, const int* d_size_x, const float* d_logw, int n, int cap, float T,
             phd_gaussian2d* out, long out_cap, int* n_groups, std::string& err);

}  // namespace phd
