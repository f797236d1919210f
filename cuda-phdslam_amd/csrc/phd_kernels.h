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

#define UPD_THREADS 256

/* per-particle status bits of the fused update */
#define PHD_ST_SURVIVOR_OVERFLOW 1
#define PHD_ST_CANDIDATE_OVERFLOW 2
#define PHD_ST_MAP_OVERFLOW 4
#define PHD_ST_SERIAL_MERGE 8 /* informational: the particle used the serial merge fallback */

/* slab reference encoding in the index table: bit 30 selects the migration set X */
#define PHD_SLAB_X 0x40000000
#define PHD_SLAB_MASK 0x3fffffff

namespace phd {

struct PredictCfg {
    int index_offset; /* global id of local particle 0: RNG counter = index_offset + i */
    float dt;
    int subdivide;
    float l, h, a, b;
    float stdAlpha, stdEncoder;
    float ax, ay, ayaw;
};

struct UpdateArgs {
    int n, cap, M, Mcap, Kcap, Scap;
    int Epool;      /* neighbour-pool entries of the parallel merge */
    int Bbuckets;   /* spatial-hash buckets (power of two >= Kcap, >= UPD_THREADS) */
    int merge_mode; /* 0 = parallel exact merge (serial fallback), 1 = serial only */
    const int* src;       /* slab reference per particle (NULL = identity) */
    int* src_reset;       /* if non-NULL, set to identity after the update */
    const float* map_x;   /* migration slab set X */
    const int* size_x;
    const float* map_in;
    float* map_out;
    const int* size_in;
    int* size_out;
    const phd_pose* poses;
    float* logw;
    float* delta;
    const float* zr;
    const float* zb;
    const int* zok;
    int* status;
    int* err;
    unsigned long long* stamps; /* diagnostic build only (PHD_STAMPS) */
    DevCfg c;
};

/* Byte offsets into the fused update's dynamic LDS.
 *   A (whole kernel): measurements, normalisers, eta partials, out-of-range list, scratch
 *   C (union): component pair table (phases 2-3) | merge candidates (phases 4-6)
 *   D (union): in/near lists + detection-term list (phases 1-4) | merge scratch (phase 5) */
struct UpdLds {
    size_t zr, zb, zok, leta, part, out, cnt, red, redf;
    size_t u;                        // region C
    size_t in, near, skey;           // region D, phases 1-4
    size_t mlam, mpar, mdeg, moff, mgids, mgstart, mpool;  // region D, phase 5
    size_t total;
};

__host__ __device__ inline size_t upd_align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline int upd_buckets(int Kcap) {
    int b = UPD_THREADS;
    while (b < Kcap) b <<= 1;
    return b;
}

__host__ __device__ inline UpdLds upd_lds_layout(int cap, int Mcap, int Kcap, int Scap, int Epool) {
    UpdLds L;
    const int B = upd_buckets(Kcap);
    size_t o = 0;
    L.zr = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    L.zb = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    L.zok = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    L.leta = o;
    o = upd_align16(o + 4 * (size_t)Mcap);
    L.part = o;
    o = upd_align16(o + 4 * (size_t)UPD_THREADS);
    L.out = o;
    o = upd_align16(o + 2 * (size_t)cap);
    L.cnt = o;
    o = upd_align16(o + 4 * 16);
    L.red = o;
    o = upd_align16(o + 8 * 16);
    L.redf = o;
    o = upd_align16(o + 4 * 16);
    // region C
    L.u = o;
    const size_t table = (size_t)cap * (6 * 4);
    const size_t cand = (size_t)Kcap * (7 * 4);
    o = upd_align16(o + (table > cand ? table : cand));
    // region D
    const size_t d0 = o;
    L.in = o;
    o = upd_align16(o + 2 * (size_t)cap);
    L.near = o;
    o = upd_align16(o + 2 * (size_t)cap);
    L.skey = o;
    o = upd_align16(o + 4 * (size_t)Scap);
    const size_t d_a = o;
    o = d0;
    L.mlam = o;
    o = upd_align16(o + 4 * (size_t)Kcap);
    L.mpar = o;
    o = upd_align16(o + 4 * (size_t)Kcap);
    L.mdeg = o;
    o = upd_align16(o + 2 * (size_t)B);
    L.moff = o;
    o = upd_align16(o + 2 * (size_t)B);
    L.mgids = o;
    o = upd_align16(o + 2 * (size_t)Kcap);
    L.mgstart = o;
    o = upd_align16(o + 2 * (size_t)(B + 2));
    L.mpool = o;
    o = upd_align16(o + 2 * (size_t)Epool);
    L.total = (o > d_a) ? o : d_a;
    return L;
}

__global__ void k_predict_ackerman(phd_pose* poses, int n, phd_ackerman_control u, const phd_ackerman_noise* noise_in,
                                   PredictCfg c, uint64_t seed, uint64_t step, const phd_pose* pose_prior,
                                   const float* logw_prior, float* logw);
__global__ void k_predict_cv(phd_pose* poses, int n, const phd_cv_noise* noise_in, PredictCfg c, uint64_t seed,
                             uint64_t step, const phd_pose* pose_prior, const float* logw_prior, float* logw);
__global__ void k_update_fused(UpdateArgs a);
__global__ void k_normalize(float* logw, int n, const float* lse_override, float* out, float resample_thresh,
                            int has_meas);
__global__ void k_lse_parts(const float* logw, int n, float* out);
__global__ void k_resample(const int* flag, const float* logw_in, float* logw_out, int n, const double* u_in,
                           uint64_t seed, uint64_t step, unsigned long long* cdf, int* idx, phd_pose* pose, int* src,
                           phd_pose* tmp_pose, int* tmp_src, float new_logw);
__global__ void k_apply_parents(const int* idx, int n, phd_pose* pose, int* src, float* logw, phd_pose* tmp_pose,
                                int* tmp_src, float new_logw);
__global__ void k_materialize(const int* src, int n, int cap, const float* map_in, const int* size_in,
                              const float* map_x, const int* size_x, float* map_dst, int* size_dst);
__global__ void k_pack(const int* src_idx, int count, int cap, const int* src, const float* map_in, const int* size_in,
                       const float* map_x, const int* size_x, const phd_pose* pose, const float* logw, float* rec);
__global__ void k_unpack(const float* rec, const int* dst_idx, const int* x_slot, int count, int cap, float* map_x,
                         int* size_x, int* src, phd_pose* pose, float* logw);
__global__ void k_expected_pose(const float* logw, const phd_pose* pose, int n, float* out);
__global__ void k_cardinality(const int* src, const float* map_in, const int* size_in, const float* map_x,
                              const int* size_x, int n, int cap, float* cn);

}  // namespace phd
