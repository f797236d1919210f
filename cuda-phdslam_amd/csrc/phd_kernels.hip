/*
 * phd_kernels.hip — gfx950 kernels of the RB-PHD-SLAM filter step.
 *
 * Device-resident particle store: for particle n the map
 * slab is 7 SoA rows of `cap` floats: [w | mx | my | P00 | P10 | P01 | P11],
 * base n*7*cap.  Lanes read consecutive components -> coalesced 256-B rows.
 *
 * Kernels:
 *   k_predict_ackerman / k_predict_cv  — phdfilter.cu:785-859 (one lane/particle)
 *   k_update_fused                     — phdfilter.cu:1279-3333 fused: in-range
 *       split, EKF, pair loop (η_m, Δlog w), births, prune, candidate
 *       build, greedy merge, out-of-range append.  One 256-thread workgroup
 *       per particle; the F×M pair space never touches HBM.
 *   k_normalize                        — phdfilter.cu:3748-3755 + main.cpp:1281-1284
 *   k_resample / k_apply_parents       — main.cpp:453-501 + slamtypes.h:313-333 (index remap)
 *   k_pack / k_unpack                  — particle records for cross-rank migration
 *   k_migration_plan / k_unpack_slots  — keep / send / receive slots of a sharded resample
 *   k_expected_pose / k_cardinality    — main.cpp:331-361
 */
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "phd_detmath.h"
#include "phd_device.h"
#include "phd_kernels.h"
#include "phd_rng.h"
#include "phd_devutil.h"
#include "phd_cphd_terms.h"

#define NF 7 /* fields per component */

/* Diagnostic build only (-DPHD_STAMPS): thread 0 of each workgroup records the
 * shader clock at phase boundaries into a.stamps[block][16]. */
#ifdef PHD_STAMPS
#define STAMP(k)                                                                                  \
    do {                                                                                          \
        if (threadIdx.x == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif
/* Diagnostic build only (-DPHD_PLAN_STAMPS): the sharded plan's phase
 * boundaries, real-time clock (100 MHz), thread 0 of each workgroup into
 * stamps[block * 8 + k]; the tail's into stamps[B * 8 + k]. */
#ifdef PHD_PLAN_STAMPS
#define PSTAMP(p, k)                                                                              \
    do {                                                                                          \
        if (threadIdx.x == 0 && (p)) (p)[k] = __builtin_amdgcn_s_memrealtime();                  \
    } while (0)
#else
#define PSTAMP(p, k) \
    do {             \
    } while (0)
#endif
/* Timing ablations of the workgroup update (diagnostic builds only, results
 * wrong by design): PHD_XK 1 no pair walk, 2 no CPHD terms, 3 no merge (no
 * output), 4 no candidates and no merge, 7 no LFMIS
 * (every candidate a seed), 8 no merge cull (no edges), 9 no clustered emission,
 * 10 the cull walk but no exact distances (no edges); part A: 11 eta summed by
 * plain (racing) LDS adds instead of atomics, 12 no eta sums, 13 the classify's
 * bearing by the platform atan2f instead of phd_atan2f.  (No survivor-ordering
 * ablation: unordered survivor keys index global memory out of bounds.) */
#ifndef PHD_XK
#define PHD_XK 0
#endif

namespace phd {

/* ------------------------------------------------------------------ predict */


__global__ void k_predict_ackerman(phd_pose* __restrict__ poses, int n, phd_ackerman_control u,
                                   const phd_ackerman_noise* __restrict__ noise_in, PredictCfg c, uint64_t seed,
                                   uint64_t step, const phd_pose* __restrict__ pose_prior,
                                   const float* __restrict__ logw_prior, float* __restrict__ logw,
                                   const int* __restrict__ slots) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int i = slots ? slots[t] : t;  // n counts the slots when given
    if (logw_prior) logw[i] = logw_prior[i];  // replay: restore the fixed prior
    float n_alpha, n_enc;
    if (noise_in) {
        n_alpha = noise_in[i].n_alpha;
        n_enc = noise_in[i].n_encoder;
    } else {
        ackerman_noise(seed, c.index_offset + i, step, c, &n_alpha, &n_enc);
    }
    poses[i] = predict_ackerman_one(pose_prior ? pose_prior[i] : poses[i], u, n_alpha, n_enc, c);
}

__global__ void k_predict_cv(phd_pose* __restrict__ poses, int n, const phd_cv_noise* __restrict__ noise_in,
                             PredictCfg c, uint64_t seed, uint64_t step, const phd_pose* __restrict__ pose_prior,
                             const float* __restrict__ logw_prior, float* __restrict__ logw,
                             const int* __restrict__ slots) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int i = slots ? slots[t] : t;
    if (logw_prior) logw[i] = logw_prior[i];  // replay: restore the fixed prior
    const phd_cv_noise w = noise_in ? noise_in[i] : cv_noise(seed, c.index_offset + i, step, c);
    poses[i] = predict_cv_one(pose_prior ? pose_prior[i] : poses[i], w, c);
}

/* n_predict_particles > 1 (phdPredict, phdfilter.cu:1185-1238): particle i
 * spawns children i*npp .. i*npp+npp-1, each with i's pose (predicted next,
 * one noise draw per child, phdfilter.cu:795), i's map by slab reference (an
 * index remap, like the resample: no map copy) and weight w_i - log(npp). */
__global__ void k_expand(int n, int npp, const phd_pose* __restrict__ pose, const int* __restrict__ src,
                         const float* __restrict__ logw, phd_pose* __restrict__ new_pose, int* __restrict__ new_src,
                         float* __restrict__ new_logw, float log_npp) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n * npp) return;
    const int i = j / npp;
    new_pose[j] = pose[i];
    new_src[j] = src[i];
    new_logw[j] = logw[i] - log_npp;
}

/* ------------------------------------------------------------ block helpers */

/* Order-preserving compaction rank of `pred` within a 256-thread block.
 * Returns this thread's exclusive rank; *total gets the block count. */
/* TAIL = false drops the trailing barrier: the caller alternates between two
 * scratch buffers (sb_at), so a buffer is rewritten only after the next
 * call's barrier, by which every thread has read it. */
template <int NT, bool TAIL = true>
__device__ __forceinline__ int block_rank(bool pred, int* s_wcnt, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long m = __ballot(pred);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wcnt[wid] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const int c = s_wcnt[w];
        off += (w < wid) ? c : 0;
        tot += c;
    }
    if (TAIL) __syncthreads();
    *total = tot;
    return off + rank;
}

/* the scratch buffer of the k-th call of a barrier-light (TAIL = false) sequence */
template <int NT>
__device__ __forceinline__ int* sb_at(int* s_w, int& k) {
    return s_w + ((k++ & 1) ? NT / 64 : 0);
}


/* ------------------------------------------------------- fused PHD update */

/* Block-wide exclusive scan of one int per thread; returns the exclusive
 * prefix, *total gets the block sum.  s_w holds >= NT/64 ints. */
template <int NT, bool TAIL = true>
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int x = wave_incl_scan(v);
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const int c = s_w[w];
        off += (w < wid) ? c : 0;
        tot += c;
    }
    if (TAIL) __syncthreads();
    *total = tot;
    return off + x - v;
}

template <int NT, bool TAIL = true>
__device__ __forceinline__ float block_max_f(float v, float* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_incl_max(v);
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    float r = -INFINITY;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) r = fmaxf(r, s_w[w]);
    if (TAIL) __syncthreads();
    return r;
}

/* Exclusive prefix sums, in index order, of A quantities over one batch of up
 * to 1024 consecutive items (item i = base + r NT + tid, r < 1024 / NT) with
 * ONE barrier: a wave scan per (r, quantity), the wave totals through LDS, each
 * thread adds up what precedes it; tot[a] = the batch totals.  s holds
 * 2 (1024 / 64) A ints: the two halves alternate with the call counter k, so a
 * call's half is rewritten only after the next call's barrier. */
template <int NT, int A>
__device__ __forceinline__ void block_scan_batch(const int (&v)[1024 / NT][A], int (&pre)[1024 / NT][A],
                                                 int (&tot)[A], int* s, int& k) {
    constexpr int R = 1024 / NT, NW = NT / 64;
    int* buf = s + ((k++ & 1) ? R * A * NW : 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x[R][A];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < A; q++) {
            x[r][q] = wave_incl_scan(v[r][q]);
            if (lane == 63) buf[(r * A + q) * NW + wid] = x[r][q];
        }
    __syncthreads();
    int run[A];
#pragma unroll
    for (int q = 0; q < A; q++) run[q] = 0;
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < A; q++) {
            int off = 0, t = 0;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                const int c = buf[(r * A + q) * NW + w];
                off += (w < wid) ? c : 0;
                t += c;
            }
            pre[r][q] = run[q] + off + x[r][q] - v[r][q];
            run[q] += t;
        }
#pragma unroll
    for (int q = 0; q < A; q++) tot[q] = run[q];
}

template <int NT, bool TAIL = true>
__device__ __forceinline__ int block_or(int v, int* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long b = __ballot(v != 0);
    if (lane == 0) s_w[wid] = b ? 1 : 0;
    __syncthreads();
    int r = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) r |= s_w[w];
    if (TAIL) __syncthreads();
    return r;
}


/* Posterior stores (PHD_NT_OUT: non-temporal, so the output lines do not
 * displace the candidates' covariances the merge re-reads from L2). */
#ifndef PHD_NT_OUT
#define PHD_NT_OUT 0
#endif
__device__ __forceinline__ void st_out(G1 float* p, float v) {
#if PHD_NT_OUT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

/* A merge set of one member is emitted as that member (its covariance
 * symmetrised) instead of the one-member form of the merged moments
 * ((w x) / w, (w (P + d d')) / w), which differs from it by at most an ulp
 * (oracle deviation D15): no divisions for the isolated seeds. */
__device__ __forceinline__ void emit_single(G1 float* dst, int cap, int slot, const float4& p, const float4& v) {
    if (slot >= cap) return;
    const float s = (v.y + v.z) / 2;  // force_symmetric_covariance (device_math.cuh:710-725)
    st_out(dst + slot, p.z);
    st_out(dst + 1 * cap + slot, p.x);
    st_out(dst + 2 * cap + slot, p.y);
    st_out(dst + 3 * cap + slot, v.x);
    st_out(dst + 4 * cap + slot, s);
    st_out(dst + 5 * cap + slot, s);
    st_out(dst + 6 * cap + slot, v.w);
}

/* Write one merged component (moments summed in double, oracle D3). */
__device__ __forceinline__ void emit_merged(G1 float* dst, int cap, int slot, float W, float gx, float gy,
                                            const double* cv) {
    if (slot >= cap) return;
    const float rW = 1.0f / W;  // (D18: one reciprocal, as the oracle)
    float p0 = (float)cv[0] * rW, p1 = (float)cv[1] * rW, p2 = (float)cv[2] * rW, p3 = (float)cv[3] * rW;
    p1 = (p1 + p2) / 2;  // force_symmetric_covariance (device_math.cuh:710-725)
    p2 = p1;
    st_out(dst + slot, W);
    st_out(dst + 1 * cap + slot, gx);
    st_out(dst + 2 * cap + slot, gy);
    st_out(dst + 3 * cap + slot, p0);
    st_out(dst + 4 * cap + slot, p1);
    st_out(dst + 5 * cap + slot, p2);
    st_out(dst + 6 * cap + slot, p3);
}

/* v1 greedy merge (phdUpdateMergeKernel :2739-2890): one selection per
 * iteration with block-parallel scans.  Exact fallback for particles the
 * parallel merge declines (non-finite candidates, edge-pool overflow).
 * key[i] is the candidate index of record i (NULL = identity) for the
 * lowest-index tie-break.  Outputs in selection order.  Returns nout. */
template <int NT>
__device__ int merge_serial(const Cand& C, const unsigned short* key, int ncand, short* cflag, float T, G1 float* dst,
                            int cap, double* s_red, float* s_redf) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int i = tid; i < ncand; i += NT) cflag[i] = 0;
    __syncthreads();
    int nout = 0;
    while (true) {
        float bw = -INFINITY;
        int bk = INT_MAX, bi = -1;
        for (int i = tid; i < ncand; i += NT) {
            const float w = C.P[i].z;
            const int k = key ? key[i] : i;
            if (cflag[i] == 0 && (bi < 0 || earlier(w, k, bw, bk))) {
                bw = w;
                bk = k;
                bi = i;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ow = __shfl_xor(bw, o, 64);
            const int ok = __shfl_xor(bk, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oi >= 0 && (bi < 0 || earlier(ow, ok, bw, bk))) {
                bw = ow;
                bk = ok;
                bi = oi;
            }
        }
        if (lane == 0) {
            s_redf[wid] = bw;
            ((int*)s_redf)[16 + wid] = bk;
            ((int*)s_redf)[32 + wid] = bi;
        }
        __syncthreads();
        bw = -INFINITY;
        bk = INT_MAX;
        bi = -1;
#pragma unroll
        for (int w2 = 0; w2 < NT / 64; w2++) {
            const float ow = s_redf[w2];
            const int ok = ((int*)s_redf)[16 + w2];
            const int oi = ((int*)s_redf)[32 + w2];
            if (oi >= 0 && (bi < 0 || earlier(ow, ok, bw, bk))) {
                bw = ow;
                bk = ok;
                bi = oi;
            }
        }
        __syncthreads();
        if (bi < 0) break;
        const float4 bp = C.P[bi], bv = C.V(bi);
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = tid; i < ncand; i += NT) {
            if (cflag[i] != 0) continue;
            const float4 p = C.P[i];
            if (cand_mahal(bp, bv, p, C.V(i)) < T) {
                cflag[i] = 2;
                acc[0] += (double)p.z;
                acc[1] += (double)(p.z * p.x);
                acc[2] += (double)(p.z * p.y);
                acc[3] += 1.0;
            }
        }
        block_sum<4, NT>(acc, s_red);
        if (acc[3] == 1.0 && acc[0] != 0.0 && cflag[bi] == 2) {  // the seed alone (D15)
            for (int i = tid; i < ncand; i += NT)
                if (cflag[i] == 2) cflag[i] = 1;
            if (tid == 0) emit_single(dst, cap, nout, bp, bv);
            nout++;
            __syncthreads();
            continue;
        }
        const float W = (float)acc[0];
        if (W == 0.f) break;
        const float rW = 1.0f / W;
        const float gx = (float)acc[1] * rW, gy = (float)acc[2] * rW;
        double cv[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = tid; i < ncand; i += NT) {
            if (cflag[i] != 2) continue;
            const float4 p = C.P[i], v = C.V(i);
            const float d0 = gx - p.x, d1 = gy - p.y;
            cv[0] += (double)(p.z * (v.x + d0 * d0));
            cv[1] += (double)(p.z * (v.y + d0 * d1));
            cv[2] += (double)(p.z * (v.z + d1 * d0));
            cv[3] += (double)(p.z * (v.w + d1 * d1));
            cflag[i] = 1;
        }
        block_sum<4, NT>(cv, s_red);
        if (tid == 0) emit_merged(dst, cap, nout, W, gx, gy, cv);
        nout++;
    }
    return nout;
}

/* neighbour lists up to this length are handled in registers */
#ifndef MERGE_DEG_REG
#define MERGE_DEG_REG 8
#endif
#ifndef MERGE_DEG_REG2
#define MERGE_DEG_REG2 12
#endif
/* records per thread of the merge walk's in-register cell-order permutation */
#ifndef PHD_WALK_SEG4
#define PHD_WALK_SEG4 1
#endif
#ifndef PHD_M3B_H
#define PHD_M3B_H 2
#endif
#ifndef PHD_LFMIS_ASYNC
#define PHD_LFMIS_ASYNC 1
#endif
#ifndef PHD_LFMIS_B
#define PHD_LFMIS_B 3
#endif
#ifndef PHD_EMIT_PF
#define PHD_EMIT_PF 4
#endif
#ifndef MERGE_PERM_REC
#define MERGE_PERM_REC 4
#endif
#ifndef PHD_MERGE_CELLWALK
#define PHD_MERGE_CELLWALK 1
#endif

/* Scratch of the parallel merge. */
struct MergeScratch {
    Cand K;                  // candidates in candidate-index order (region C)
    short* par;              // region C, after the records: -2 seed, -1 undecided, >= 0 absorbed by
    unsigned short* off;     // K + 1 CSR offsets
    unsigned short* cur;     // K degrees / scatter cursors (16-bit halves of 32-bit atomics)
    unsigned int* edges;     // Epool undirected edges (i << 16 | j)
    unsigned short* pool;    // 2 * Epool adjacency entries
    unsigned int* plist;     // culled candidate pairs (aliases par | off | pool)
    int plcap;
    unsigned short* key;     // cell-order position -> candidate index (region D)
    unsigned short* gstart;  // B + 2 bucket starts (region D)
    int* st_tests;           // diagnostic builds: neighbour tests of the cull walk
};


/* Neighbourhood walk of the parallel merge over the cell-order index `key`: a
 * bucket row is a contiguous run of cell-order positions, and position q visits
 * its forward half-neighbourhood — the rest of its own bucket and the next
 * bucket of its row (one run, two at the lattice wrap), the three buckets of
 * the next row (one run, two at the wrap) — plus the ill-conditioned tail.
 * Each unordered pair of adjacent buckets is forward of exactly one of the two
 * (Px, Py >= 3), so every pair is tested once; culls with the isotropic bound
 * and hands each surviving pair (i, j) of candidate indices to `on_pair`. */
template <int NT, bool CELL = false, class F>
__device__ __forceinline__ void merge_walk(const MergeScratch& X, int K, int Knw, int B, int Px, int Py, int lgPx,
                                           float invR, float thr, F&& on_pair) {
    const int tid = threadIdx.x;
    for (int q = tid; q < K; q += NT) {
        // CELL: the records themselves are in cell order (merge_parallel permutes
        // them for the walk), so a neighbour is one record load, not index ->
        // record, and the pair handed on is the two cell-order positions
        const int i = CELL ? q : X.key[q];
        const float4 p = X.K.P[i];
        int lo1 = q + 1, hi1 = K, lo2 = 0, hi2 = 0, lo3 = 0, hi3 = 0, lo4 = 0, hi4 = 0, lo0 = 0, hi0 = 0;
        const bool wild = q >= Knw;
        if (!wild) {
            const int cx = (int)floorf(fminf(fmaxf(p.x * invR, -8192.f), 8192.f));
            const int cy = (int)floorf(fminf(fmaxf(p.y * invR, -8192.f), 8192.f));
            const int cxm = cx & (Px - 1), cym = cy & (Py - 1);
            const int rb = cym << lgPx, rn = ((cym + 1) & (Py - 1)) << lgPx;
            // this row: the rest of bucket cxm and bucket cxm + 1 (bucket 0 at the wrap)
            hi1 = X.gstart[rb + cxm + (cxm + 1 < Px ? 2 : 1)];
            if (cxm == Px - 1) {
                lo2 = X.gstart[rb];
                hi2 = X.gstart[rb + 1];
            }
            // next row: buckets cxm - 1 .. cxm + 1, split at the wrap
            lo3 = X.gstart[rn + (cxm == 0 ? 0 : cxm - 1)];
            hi3 = X.gstart[rn + (cxm == Px - 1 ? Px : cxm + 2)];
            if (cxm == 0 || cxm == Px - 1) {
                const int cw = cxm == 0 ? Px - 1 : 0;
                lo4 = X.gstart[rn + cw];
                hi4 = X.gstart[rn + cw + 1];
            }
            lo0 = Knw;  // the wild tail
            hi0 = K;
        }
        const int n1 = max(hi1 - lo1, 0), n2 = max(hi2 - lo2, 0), n3 = max(hi3 - lo3, 0), n4 = max(hi4 - lo4, 0),
                  n0 = max(hi0 - lo0, 0);
        const int e1 = n1, e2 = e1 + n2, e3 = e2 + n3, e4 = e3 + n4, e0 = e4 + n0;
#ifdef PHD_STAMPS
        if (X.st_tests) {
            atomicAdd(X.st_tests, e0);
            // divergence: the wave runs ceil(max e0 / 4) steps of this batch
            // (the active lanes are a prefix of the wave: read the last one)
            const int last = 63 - __builtin_clzll(__ballot(1));
            const int wm = __builtin_amdgcn_readlane(wave_incl_max_i(e0), last);
            if ((threadIdx.x & 63) == 0) atomicAdd(X.st_tests + 2, (wm + 3) / 4);
        }
#endif
        // flattened walk over the segments, position = t + offset of its segment
        const int g1 = (lo2 - e1) - lo1, g2 = (lo3 - e2) - (lo2 - e1), g3 = (lo4 - e3) - (lo3 - e2),
                  g4 = (lo0 - e4) - (lo4 - e3);
        auto at = [&](int t) {
            return t + lo1 + (t >= e1 ? g1 : 0) + (t >= e2 ? g2 : 0) + (t >= e3 ? g3 : 0) + (t >= e4 ? g4 : 0);
        };
        // four entries per step: their index and record loads issue together
        for (int t = 0; t < e0; t += 4) {
            int jj[4];
            float4 pp[4];
#pragma unroll
            for (int k = 0; k < 4; k++) jj[k] = (t + k < e0) ? (CELL ? at(t + k) : (int)X.key[at(t + k)]) : i;
#pragma unroll
            for (int k = 0; k < 4; k++) pp[k] = X.K.P[jj[k]];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                bool test = t + k < e0;
                if (!wild && pp[k].w >= 0.f) {
                    const float dx = pp[k].x - p.x, dy = pp[k].y - p.y;
                    test = test && !(dx * dx + dy * dy > thr * (p.w + pp[k].w));
                }
                if (test) on_pair(i, jj[k]);
            }
        }
    }
}

/* merge_walk over records in cell order (merge_parallel permutes them for the
 * walk), wave by wave over 64 positions at a time.  A position's forward
 * neighbourhood (merge_walk) is cut into chunks of WU consecutive entries and
 * the wave's chunks are dealt 64 per step: a lane finds its chunk's owner by a
 * binary search over the chunk prefix (ds_bpermute) and reads the owner's
 * record and segments the same way, so a step tests 64 chunks however unevenly
 * the neighbourhoods are spread over the positions (a dense cluster no longer
 * holds the wave for its longest list).  Two dealt passes: the four segments
 * (rest of the bucket row + the next row's three buckets, and their lattice
 * wraps) in one, and the pairs with an ill-conditioned position, whose exact
 * distance decides the listing.  A neighbour is one record load, the tests of a chunk
 * are branch-free, and the step's surviving pairs (two cell-order positions,
 * q << 16 | pos) are listed with one LDS atomic per wave (ranks from ballots of
 * the per-lane count). */
#ifndef PHD_WALK_UNROLL
#define PHD_WALK_UNROLL 4
#endif
template <int WU, bool EXACT = false, bool SEG4 = false>
__device__ __forceinline__ void walk_dealt(const MergeScratch& X, int qb, float px, float py, float tpw, int la, int na,
                                           int lb, int nb, float thr, int* npair, int plcap, int lc = 0, int nc = 0,
                                           int ld = 0, int nd = 0) {
    // (SEG4: four segments a, b, c, d per lane — the common ones and the lattice
    // wraps in one pass)
    // (EXACT: a pair is listed when its exact distance is below thr = T; tpw
    // then carries the owner record's w word, whose low half is the covariance tag)
    const int lane = threadIdx.x & 63;
    const int c = (na + nb + (SEG4 ? nc + nd : 0) + WU - 1) / WU;  // chunks of this lane
    const int inc = wave_incl_scan(c);
    const int tot = __builtin_amdgcn_readlane(inc, 63);
    if (tot == 0) return;  // (wave-uniform)
#ifdef PHD_STAMPS
    if (X.st_tests && lane == 0) atomicAdd(X.st_tests + 2, (tot + 63) / 64);  // dealt steps
#endif
    const int P = inc - c;  // first chunk of this lane
    const int pk1 = la | (lb << 16), pk2 = na | ((na + nb) << 16);
    const int pk3 = lc | (ld << 16), pk4 = (na + nb + nc) | ((na + nb + nc + nd) << 16);
    for (int base = 0; base < tot; base += 64) {
        const int w = base + lane;
        // owner: the last lane whose first chunk is <= w (a lane without chunks
        // shares its P with the next lane, so the last such lane has chunks)
        int o = 0;
#pragma unroll
        for (int st = 32; st; st >>= 1) o += __shfl(P, o + st) <= w ? st : 0;
        const int t0 = (w - __shfl(P, o)) * WU;
        const float ox = __shfl(px, o), oy = __shfl(py, o), otpw = __shfl(tpw, o);
        const int o1 = __shfl(pk1, o), o2 = __shfl(pk2, o);
        const int ola = o1 & 0xffff, olb = (int)((unsigned)o1 >> 16), ona = o2 & 0xffff;
        int on = w < tot ? (int)((unsigned)o2 >> 16) : 0;
        int olc = 0, old = 0, onab = on, onabc = on;
        if constexpr (SEG4) {
            const int o3 = __shfl(pk3, o), o4 = __shfl(pk4, o);
            olc = o3 & 0xffff;
            old = (int)((unsigned)o3 >> 16);
            onabc = o4 & 0xffff;
            on = w < tot ? (int)((unsigned)o4 >> 16) : 0;
        }
        int jj[WU];
        float4 pp[WU];
#pragma unroll
        for (int k = 0; k < WU; k++) {
            const int t = t0 + k;
            int pos = t < ona ? ola + t : olb + (t - ona);
            if constexpr (SEG4) pos = t < onab ? pos : t < onabc ? olc + (t - onab) : old + (t - onabc);
            jj[k] = t < on ? pos : 0;
        }
#pragma unroll
        for (int k = 0; k < WU; k++) pp[k] = X.K.P[jj[k]];
        int m = 0;
        if constexpr (EXACT) {
            const float4 po = make_float4(ox, oy, 0.f, otpw);
            const float4 vo = X.K.Vp(po);
#pragma unroll
            for (int k = 0; k < WU; k++) {
                const float4 vk = X.K.Vp(pp[k]);
                const int ok = (int)(t0 + k < on) & (int)(cand_mahal(po, vo, pp[k], vk) < thr);
                m |= ok << k;
            }
        } else {
#pragma unroll
            for (int k = 0; k < WU; k++) {
                const float dx = pp[k].x - ox, dy = pp[k].y - oy;
                const float d2 = dx * dx + dy * dy;
                const int ok = (int)(t0 + k < on) & (int)!(d2 > fmaf(thr, pp[k].w, otpw));
                m |= ok << k;
            }
        }
        static_assert(WU >= 1 && WU <= 15, "the listing ranks count up to 15 pairs per lane and step");
        const int cnt = __builtin_popcount(m);
        const unsigned long long b0 = __ballot(cnt & 1), b1 = WU > 1 ? __ballot(cnt & 2) : 0ull,
                                 b2 = WU > 3 ? __ballot(cnt & 4) : 0ull, b3 = WU > 7 ? __ballot(cnt & 8) : 0ull;
        const int ntot = __builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2) +
                         8 * __builtin_popcountll(b3);
        if (ntot) {  // (wave-uniform)
            int sbase = 0;
            if (lane == 0) sbase = atomicAdd(npair, ntot);
            sbase = __builtin_amdgcn_readlane(sbase, 0);
            int sl = sbase + (int)(__builtin_amdgcn_mbcnt_hi((unsigned)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b0, 0)) +
                                   2 * __builtin_amdgcn_mbcnt_hi((unsigned)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b1, 0)) +
                                   4 * __builtin_amdgcn_mbcnt_hi((unsigned)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b2, 0)) +
                                   8 * __builtin_amdgcn_mbcnt_hi((unsigned)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b3, 0)));
            const unsigned int qhi = (unsigned int)(qb + o) << 16;
#pragma unroll
            for (int k = 0; k < WU; k++) {
                if ((m >> k) & 1) {
                    if (sl < plcap) X.plist[sl] = qhi | (unsigned int)jj[k];
                    sl++;
                }
            }
        }
    }
}

template <int NT, int WU = PHD_WALK_UNROLL>
__device__ __forceinline__ void merge_walk_cell(const MergeScratch& X, int K, int Knw, int Px, int Py, int lgPx,
                                                float invR, float thr, float T, int* npair, int plcap) {
    const int tid = threadIdx.x, lane = tid & 63;
    for (int qb0 = 0; qb0 < K; qb0 += NT) {
        const int qb = qb0 + (tid & ~63);  // this wave's first position
        if (qb >= K) break;                // (wave-uniform)
        const int q = qb + lane;
        const bool live = q < K;
        const float4 p = X.K.P[live ? q : 0];
        const bool wild = q >= Knw;
        // segments: [q+1, hi1) the rest of the bucket and the next bucket of its
        // row, [lo2, hi2) the row wrap, [lo3, hi3) + [lo4, hi4) the next row's
        // three buckets and their wrap; a wild position: [q+1, K)
        int lo1 = q + 1, hi1 = K, lo2 = 0, hi2 = 0, lo3 = 0, hi3 = 0, lo4 = 0, hi4 = 0;
        if (live && !wild) {
            const int cx = (int)floorf(fminf(fmaxf(p.x * invR, -8192.f), 8192.f));
            const int cy = (int)floorf(fminf(fmaxf(p.y * invR, -8192.f), 8192.f));
            const int cxm = cx & (Px - 1), cym = cy & (Py - 1);
            const int rb = cym << lgPx, rn = ((cym + 1) & (Py - 1)) << lgPx;
            hi1 = X.gstart[rb + cxm + (cxm + 1 < Px ? 2 : 1)];
            if (cxm == Px - 1) {
                lo2 = X.gstart[rb];
                hi2 = X.gstart[rb + 1];
            }
            lo3 = X.gstart[rn + (cxm == 0 ? 0 : cxm - 1)];
            hi3 = X.gstart[rn + (cxm == Px - 1 ? Px : cxm + 2)];
            if (cxm == 0 || cxm == Px - 1) {
                const int cw = cxm == 0 ? Px - 1 : 0;
                lo4 = X.gstart[rn + cw];
                hi4 = X.gstart[rn + cw + 1];
            }
        }
        const int n1 = live ? max(hi1 - lo1, 0) : 0, n2 = max(hi2 - lo2, 0), n3 = max(hi3 - lo3, 0),
                  n4 = max(hi4 - lo4, 0);
        // (a wild position or neighbour is never culled: its bound is +inf / its w < 0 only in the tail pass)
        const float tpw = wild ? INFINITY : thr * p.w;
#ifdef PHD_STAMPS
        if (X.st_tests) {
            const int e0 = n1 + n2 + n3 + n4 + (live && !wild ? K - Knw : 0);
            atomicAdd(X.st_tests, e0);
        }
#endif
#if PHD_WALK_SEG4
        walk_dealt<WU, false, true>(X, qb, p.x, p.y, tpw, lo1, wild ? 0 : n1, lo3, n3, thr, npair, plcap, lo2, n2, lo4,
                                    n4);
#else
        walk_dealt<WU>(X, qb, p.x, p.y, tpw, lo1, wild ? 0 : n1, lo3, n3, thr, npair, plcap);
        walk_dealt<WU>(X, qb, p.x, p.y, tpw, lo2, n2, lo4, n4, thr, npair, plcap);
#endif
        // pairs with an ill-conditioned candidate (the wild tail after every
        // binned position; everything after a wild one): the isotropic bound
        // does not cover their float distance, so the exact distance decides
        // the listing here — one entry per lane and step — instead of listing
        // every such pair (a few wild births at close range would overflow the
        // pair list: 7 % of the particle-updates of bench.py --mode sequence)
        if (Knw < K)
            walk_dealt<1, true>(X, qb, p.x, p.y, p.w, wild ? q + 1 : Knw, !live ? 0 : wild ? K - q - 1 : K - Knw, 0, 0,
                                T, npair, plcap);
    }
}

/* Merged moments of clustered seed i whose adjacency row pool[o, o + nd) has
 * nd <= R entries: the set's members (neighbours absorbed by i, and i) sorted
 * by candidate index in registers (odd-even transposition network; the rest
 * INT_MAX), so both passes are straight loads in that order.  False when every
 * neighbour went to another seed (D15: emitted as a single member). */
template <int R, int PF = PHD_EMIT_PF>
__device__ __forceinline__ bool cluster_moments(const MergeScratch& X, int i, int o, int nd, float& Wf, float& gx,
                                                float& gy, double* cv) {
    double W = 0.0, sx = 0.0, sy = 0.0;
    int mb[R + 1];
#pragma unroll
    for (int k = 0; k < R; k++) mb[k] = k < nd ? X.pool[o + k] : i;
#pragma unroll
    for (int k = 0; k < R; k++) mb[k] = (mb[k] != i && X.par[mb[k]] == i) ? mb[k] : INT_MAX;
    mb[R] = i;
    constexpr int NM = R + 1;
#pragma unroll
    for (int r = 0; r < NM; r++) {
#pragma unroll
        for (int k = r & 1; k + 1 < NM; k += 2) {
            const int lo = min(mb[k], mb[k + 1]), hi = max(mb[k], mb[k + 1]);
            mb[k] = lo;
            mb[k + 1] = hi;
        }
    }
    if (mb[1] == INT_MAX) return false;  // every neighbour went to another seed (D15)
    // every member's covariance load issued before the sums (a prior's
    // or a birth's lives in its slab): one memory latency, not one per member
    constexpr int NPF = PF < 1 ? 1 : PF < NM ? PF : NM;  // prefetched members
    float4 vv[NPF];
#pragma unroll
    for (int k = 0; k < NPF; k++) vv[k] = X.K.Vp(X.K.P[mb[k] == INT_MAX ? i : mb[k]]);
#pragma unroll
    for (int k = 0; k < NM; k++) {
        if (mb[k] == INT_MAX) break;
        const float4 pj = X.K.P[mb[k]];
        W += (double)pj.z;
        sx += (double)(pj.z * pj.x);
        sy += (double)(pj.z * pj.y);
    }
    Wf = (float)W;
    const float rW = 1.0f / Wf;
    gx = (float)sx * rW;
    gy = (float)sy * rW;
#pragma unroll
    for (int k = 0; k < NM; k++) {
        if (mb[k] == INT_MAX) break;
        const float4 pj = X.K.P[mb[k]], vj = k < NPF ? vv[k < NPF ? k : 0] : X.K.V(mb[k]);
        const float d0 = gx - pj.x, d1 = gy - pj.y, w = pj.z;
        cv[0] += (double)(w * (vj.x + d0 * d0));
        cv[1] += (double)(w * (vj.y + d0 * d1));
        cv[2] += (double)(w * (vj.z + d1 * d0));
        cv[3] += (double)(w * (vj.w + d1 * d1));
    }
    return true;
}

/*
 * Parallel exact greedy merge.  The greedy of phdUpdateMergeKernel takes the
 * heaviest unmerged candidate c*, absorbs every unmerged i with
 * d(c*, i) < minSeparation, and repeats.  When every candidate absorbs itself
 * (d(i,i) < T, i.e. a non-singular covariance), this is, with candidates
 * ordered by priority (weight desc, index asc) and E = {(a,b): d(a,b) < T}
 * (d is bitwise symmetric): i is absorbed by the first seed among its
 * higher-priority neighbours, and is a seed if it has none — a
 * lexicographically-first maximal independent set on E, solved in rounds.
 *
 * E is found exactly.  Well-conditioned candidates (lambda_min > 1e-4
 * lambda_max) are binned on a P x P lattice-hashed grid of cell size
 * R = sqrt(1.05 T max lambda_max) (d >= 2|dmu|^2/(lambda_a+lambda_b), the 5 %
 * covering float rounding up to cond 1e4), so every edge joins two candidates
 * in adjacent cells; P >= 32 keeps the 9 cells of a neighbourhood in 9
 * distinct buckets.  The cell-order index `key` makes a neighbourhood 3 rows
 * of at most 2 contiguous segments each, and every pair is tested once (by the
 * lower cell-order position).  Ill-conditioned ("wild") candidates sit after
 * the binned ones and are tested against everything exactly.
 * Returns nout (outputs in candidate-index order of their seeds), or -1 when
 * the particle needs the serial greedy (non-finite candidate, d(i,i) >= T,
 * edge-pool overflow).
 */
template <int NT>
__device__ int merge_parallel(const MergeScratch& X, int K, float T, G1 float* dst, int cap, int Epool, int B, int* s_w,
                              float* s_wf, int* s_misc, int screen_bad, float screen_lmax, const UpdateArgs& a) {
    const int tid = threadIdx.x;
    int lgPx, lgPy;
    lattice_dims(B, &lgPx, &lgPy);
    const int Px = 1 << lgPx, Py = 1 << lgPy;
    // M1: the screen ran when the candidates were written (cand_record): one
    // reduction gives max lambda_max, and +inf when a candidate needs the serial greedy
#ifdef PHD_STAMPS
    if (threadIdx.x == 0) {
        s_misc[4] = 0;
        s_misc[10] = 0;
    }
#endif
    // (the bucket counters are cleared under the reduction's barrier)
    for (int b = tid; b < B + 2; b += NT) X.gstart[b] = 0;
    if (tid == 0) s_misc[1] = 0;  // wild count
    int sbk = 0;                  // barrier-light helper sequence (sb_at)
    // (no trailing barrier: s_wf is next written after the far check's barrier)
    const float lsc = block_max_f<NT, false>(screen_bad ? INFINITY : screen_lmax, s_wf);
    if (!(lsc < INFINITY)) return -1;
    const float lmax = lsc;
#ifdef PHD_STAMPS
    MergeScratch& Xw = const_cast<MergeScratch&>(X);
    Xw.st_tests = s_misc + 10;  // s_cnt[13], s_cnt[7], s_cnt[15]: unused by the update
    if (threadIdx.x == 0) s_misc[12] = 0;
    {
        float ls = 0.f;
        for (int i = threadIdx.x; i < K; i += NT) ls += X.K.P[i].w;
        atomicAdd((float*)(s_misc + 4), ls);
    }
#endif
    STAMP(11);
    const float R = sqrtf(1.05f * T * lmax);
    const float invR = (lmax > 0.f) ? 1.0f / (R * 1.001f) : 0.f;
    // M2: bucket counting sort of the binned candidates; wild ones go last.
    // Up to four candidates per thread (K <= 4 NT) each keeps its rank in its
    // bucket from the counting atomic, so the fill is plain stores at start +
    // rank; beyond that the fill takes a second atomic per candidate.
    const bool rk1 = K <= 4 * NT;
    unsigned int rk[4] = {~0u, ~0u, ~0u, ~0u};  // bucket << 16 | rank (~0: none / wild)
    int far = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        for (int i = tid + r * NT; i < K; i += (rk1 ? 4 * NT : NT)) {
            const float4 p = X.K.P[i];
            if (p.w < 0.f) {
                X.key[K - 1 - atomicAdd(s_misc + 1, 1)] = (unsigned short)i;
                continue;
            }
            far |= !(fabsf(p.x * invR) < 8192.f && fabsf(p.y * invR) < 8192.f);
            const unsigned int bkt = lattice_bucket(p.x, p.y, invR, Px, Py, lgPx);
            if (rk1) {
                const unsigned int old = atomicAdd((unsigned int*)(X.gstart + (bkt & ~1u)), (bkt & 1u) ? 0x10000u : 1u);
                rk[r] = (bkt << 16) | ((bkt & 1u) ? (old >> 16) : (old & 0xffffu));
            } else {
                atomicAdd((unsigned int*)(X.gstart + (bkt & ~1u)), (bkt & 1u) ? 0x10000u : 1u);
            }
        }
        if (!rk1) break;  // (the strided loop above covered every candidate)
    }
    if (block_or<NT, false>(far, sb_at<NT>(s_w, sbk))) return -1;
    STAMP(16);
    const int Knw = K - s_misc[1];
    {  // scan over B counters: gstart[b] = start of bucket b (rk1), else its end
        const int per = (B + NT - 1) / NT;
        const int base = tid * per;
        int sum = 0;
        for (int q = 0; q < per; q++) sum += base + q < B ? X.gstart[base + q] : 0;
        int tot;
        int pre = block_excl_scan<NT, false>(sum, sb_at<NT>(s_w, sbk), &tot);
        for (int q = 0; q < per && base + q < B; q++) {
            const int cnt = X.gstart[base + q];
            X.gstart[base + q] = (unsigned short)(rk1 ? pre : pre + cnt);
            pre += cnt;
        }
    }
    __syncthreads();
    STAMP(17);
    if (rk1) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int i = tid + r * NT;
            if (rk[r] != ~0u) X.key[X.gstart[rk[r] >> 16] + (rk[r] & 0xffffu)] = (unsigned short)i;
        }
    } else {
        for (int i = tid; i < K; i += NT) {
            const float4 p = X.K.P[i];
            if (p.w < 0.f) continue;
            const unsigned int bkt = lattice_bucket(p.x, p.y, invR, Px, Py, lgPx);
            const unsigned int old = atomicSub((unsigned int*)(X.gstart + (bkt & ~1u)), (bkt & 1u) ? 0x10000u : 1u);
            X.key[((bkt & 1u) ? (int)(old >> 16) : (int)(old & 0xffffu)) - 1] = (unsigned short)i;
        }
    }
    // (the bucket starts may live over cur | edges: then cur is cleared after the walk)
    const bool gs_alias = (const void*)X.gstart == (const void*)X.cur;
    if (!gs_alias)
        for (int i = tid; i < K; i += NT) X.cur[i] = 0;
    if (tid == 0) {
        X.gstart[B] = (unsigned short)Knw;
        s_misc[0] = 0;  // edge count
        s_misc[2] = 0;  // candidate-pair count
    }
    __syncthreads();
    // The walk reads the records in cell order: permuted in place through
    // registers (up to MERGE_PERM_REC per thread) and restored right after it,
    // so everything else keeps candidate-index order (a pair-list overflow
    // walks again by index, below).
    const bool cellw = K <= MERGE_PERM_REC * NT && PHD_MERGE_CELLWALK;
    auto permute = [&](bool to_cell) {
        // (named records: an array here is left in scratch)
        const int q0 = tid, q1 = tid + NT, q2 = tid + 2 * NT, q3 = tid + 3 * NT;
        const bool h3 = MERGE_PERM_REC > 3 && q3 < K;
        const int i0 = q0 < K ? X.key[q0] : 0, i1 = q1 < K ? X.key[q1] : 0, i2 = q2 < K ? X.key[q2] : 0,
                  i3 = h3 ? X.key[q3] : 0;
        float4 r0, r1, r2, r3;
        if (q0 < K) r0 = X.K.P[to_cell ? i0 : q0];
        if (q1 < K) r1 = X.K.P[to_cell ? i1 : q1];
        if (q2 < K) r2 = X.K.P[to_cell ? i2 : q2];
        if (h3) r3 = X.K.P[to_cell ? i3 : q3];
        __syncthreads();
        if (q0 < K) X.K.P[to_cell ? q0 : i0] = r0;
        if (q1 < K) X.K.P[to_cell ? q1 : i1] = r1;
        if (q2 < K) X.K.P[to_cell ? q2 : i2] = r2;
        if (h3) X.K.P[to_cell ? q3 : i3] = r3;
        __syncthreads();
    };
    static_assert(MERGE_PERM_REC == 3 || MERGE_PERM_REC == 4, "permute() holds three or four records per thread");
    if (cellw) permute(true);
    STAMP(12);
    // M3a: candidate pairs (merge_walk), listed so the exact distance runs
    // densely in M3b instead of under a divergent mask.
    const float thr = 1.05f * T * 0.5f;
    const int plcap = a.plreq > 0 ? min(X.plcap, a.plreq) : X.plcap;
    auto list_pair = [&](int i, int j) {
        const int sl = atomicAdd(s_misc + 2, 1);
        if (sl < plcap) X.plist[sl] = ((unsigned int)i << 16) | (unsigned int)j;
    };
    if (PHD_XK != 8) {
        if (cellw)
            merge_walk_cell<NT>(X, K, Knw, Px, Py, lgPx, invR, thr, T, s_misc + 2, plcap);  // pairs of positions
        else
            merge_walk<NT>(X, K, Knw, B, Px, Py, lgPx, invR, thr, list_pair);
    }
    __syncthreads();
    if (cellw) permute(false);  // (its barriers also publish the pair count)
    STAMP(23);
    const int npairs = s_misc[2];
    // the bucket starts of an overflow walk (below)
    MergeScratch Xo = X;
    if (gs_alias) {
        // the walk is done with the bucket starts: cur holds the degrees from here.
        // On a pair-list overflow the walk runs again with the exact distances in
        // place, writing cur and edges: its bucket starts move first into the
        // abandoned pair list (par | off | pool, dead until the CSR).
        if (npairs > plcap) {
            if (2 * X.plcap < B + 2) return -1;  // (no room: the serial greedy)
            if (tid == 0) {
                atomicAdd(a.err + 2, 1);
                s_misc[11] |= PHD_ST_PAIR_OVERFLOW;  // (s_cnt[14]: read after the merge's barriers)
            }
            unsigned short* gs2 = (unsigned short*)X.plist;
            for (int b = tid; b < B + 2; b += NT) gs2[b] = X.gstart[b];
            __syncthreads();
            Xo.gstart = gs2;
        }
        for (int i = tid; i < K; i += NT) X.cur[i] = 0;
        __syncthreads();
    }
    if (npairs <= plcap) {
        // M3b: exact distances of the listed pairs -> edges and degrees,
        // PHD_M3B_H pairs per thread and step with all their covariance loads
        // in flight together (a prior's or a birth's covariance is read from its slab)
        constexpr int H = PHD_M3B_H;
        for (int e0 = tid; e0 < (PHD_XK == 10 ? 0 : npairs); e0 += H * NT) {
            unsigned int pr[H];
            bool ok[H];
#pragma unroll
            for (int h = 0; h < H; h++) {
                ok[h] = e0 + h * NT < npairs;
                pr[h] = X.plist[ok[h] ? e0 + h * NT : e0];
                if (cellw) pr[h] = ((unsigned int)X.key[pr[h] >> 16] << 16) | (unsigned int)X.key[pr[h] & 0xffffu];
            }
            float4 vi[H], vj[H];
#pragma unroll
            for (int h = 0; h < H; h++) {
                vi[h] = X.K.Vp(X.K.P[pr[h] >> 16]);
                vj[h] = X.K.Vp(X.K.P[pr[h] & 0xffffu]);
            }
#pragma unroll
            for (int h = 0; h < H; h++) {
                const int i = (int)(pr[h] >> 16), j = (int)(pr[h] & 0xffffu);
                if (ok[h] && cand_mahal(X.K.P[i], vi[h], X.K.P[j], vj[h]) < T) {
                    const int sl = atomicAdd(s_misc, 1);
                    if (sl < Epool) X.edges[sl] = pr[h];
                    cnt16_inc(X.cur, i);
                    cnt16_inc(X.cur, j);
                }
            }
        }
    } else {
        // pair list overflow: walk again with the exact distance in place
        if (!gs_alias && tid == 0) {
            atomicAdd(a.err + 2, 1);
            s_misc[11] |= PHD_ST_PAIR_OVERFLOW;
        }
        merge_walk<NT>(Xo, K, Knw, B, Px, Py, lgPx, invR, thr, [&](int i, int j) {
            if (cand_mahal(X.K.P[i], X.K.V(i), X.K.P[j], X.K.V(j)) < T) {
                const int sl = atomicAdd(s_misc, 1);
                if (sl < Epool) X.edges[sl] = ((unsigned int)i << 16) | (unsigned int)j;
                cnt16_inc(X.cur, i);
                cnt16_inc(X.cur, j);
            }
        });
    }
    __syncthreads();
    STAMP(13);
    const int E = s_misc[0];
#ifdef PHD_STAMPS
    if (tid == 0 && a.stamps) {
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 24] = ((unsigned long long)npairs << 32) | (unsigned)E;
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 43] =
            ((unsigned long long)(unsigned)s_misc[10] << 32) | (unsigned)__float_as_uint(lmax);
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 44] =
            ((unsigned long long)(unsigned)K << 32) | (unsigned)s_misc[4];
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 45] =
            ((unsigned long long)(unsigned)s_misc[12] << 32) | (unsigned)(K - Knw);
    }
#endif
    if (E > Epool) return -1;
    // M4: adjacency lists (CSR over candidate index): off = exclusive scan of the
    // degrees, and the active (non-isolated) candidates listed in index order
    // (into the cell-order index, dead after the walk) — one barrier per 1024
    // candidates.  s_scan: the merge's scan scratch (block_scan_batch).
    constexpr int RB = 1024 / NT;
    int* s_scan = s_w;
    int sbb = 0;
    unsigned short* alist = X.key;
    int nact = 0;
    {
        int running = 0;
        for (int base = 0; base < K; base += 1024) {
            // degree | active << 16 in one scan (the degrees of a batch sum to at
            // most 2E < 2^16: the CSR offsets are 16-bit)
            int v[RB][1], pre[RB][1], tot[1];
#pragma unroll
            for (int r = 0; r < RB; r++) {
                const int i = base + r * NT + tid;
                const int c = (i < K) ? X.cur[i] : 0;
                v[r][0] = c | (c > 0 ? 0x10000 : 0);
            }
            block_scan_batch<NT, 1>(v, pre, tot, s_scan, sbb);
#pragma unroll
            for (int r = 0; r < RB; r++) {
                const int i = base + r * NT + tid;
                if (i >= K) continue;
                const int c = v[r][0] & 0xffff, o = running + (pre[r][0] & 0xffff);
                // end cursor, decremented by the scatter down to the row start o:
                // the cursors then are the CSR offsets (X.off aliases X.cur)
                X.cur[i] = (unsigned short)(o + c);
                X.par[i] = (short)(c == 0 ? -2 : -1);  // isolated candidates are seeds of their own
                if (c > 0) alist[nact + (pre[r][0] >> 16)] = (unsigned short)i;
            }
            running += tot[0] & 0xffff;
            nact += tot[0] >> 16;
        }
        if (tid == 0) {
            X.off[K] = (unsigned short)running;  // (cur[K]: no cursor of its own; untouched by the scatter)
            s_misc[3] = 0;  // LFMIS failsafe flag
        }
    }
    __syncthreads();
    STAMP(18);
    for (int e = tid; e < E; e += NT) {
        const unsigned int ed = X.edges[e];
        const int i = (int)(ed >> 16), j = (int)(ed & 0xffffu);
        X.pool[cnt16_dec(X.cur, i)] = (unsigned short)j;
        X.pool[cnt16_dec(X.cur, j)] = (unsigned short)i;
    }
    __syncthreads();
    STAMP(19);
    STAMP(14);
    // M5: lexicographically-first MIS (-2 seed, >= 0 absorbed by that seed).
    // Among i's higher-priority neighbours let s* be the first seed and u* the
    // first undecided one (priority order): i decides once no higher-priority
    // neighbour is undecided — it joins s*, or becomes a seed when there is none
    // (the decision of a scan of the priority-sorted list, without sorting it).
    // i may also decide while a later-priority neighbour than s* is undecided.
    // Synchronous rounds: every round decides at least the highest-priority
    // undecided candidate, a decision is final, and reading a neighbour decided
    // in the same round only decides earlier — so the result does not depend on
    // timing.  The rounds end when no active candidate is undecided.
#define PHD_CONSIDER(E, WE, ST)                                                             \
    {                                                                                       \
        const int e_ = (E);                                                                 \
        const float we_ = (WE);                                                             \
        const int st_ = (ST);                                                               \
        if (earlier(we_, e_, wi, i)) {                                                      \
            const bool s_better = st_ == -2 && (bs < 0 || earlier(we_, e_, ws, bs));         \
            const bool u_better = st_ == -1 && (bu < 0 || earlier(we_, e_, wu, bu));         \
            ws = s_better ? we_ : ws;                                                       \
            bs = s_better ? e_ : bs;                                                        \
            wu = u_better ? we_ : wu;                                                       \
            bu = u_better ? e_ : bu;                                                        \
        }                                                                                   \
    }
    int nrounds = 0;
    // one LFMIS decision of active candidate i: true when it is still pending
    auto lfmis_try = [&](int i) -> bool {
        const int o = X.off[i], nd = X.off[i + 1] - o;
        const float wi = X.K.P[i].z;
        float ws = 0.f, wu = 0.f;
        int bs = -1, bu = -1;
        // PHD_LFMIS_B neighbours per batch with their loads in flight together
        // (a padding entry is i itself: never earlier than i)
        for (int r0 = 0; r0 < nd; r0 += PHD_LFMIS_B) {
            int e[PHD_LFMIS_B];
            float we[PHD_LFMIS_B];
            int st[PHD_LFMIS_B];
#pragma unroll
            for (int k = 0; k < PHD_LFMIS_B; k++) e[k] = r0 + k < nd ? (int)X.pool[o + r0 + k] : i;
#pragma unroll
            for (int k = 0; k < PHD_LFMIS_B; k++) {
                we[k] = X.K.P[e[k]].z;
                st[k] = __hip_atomic_load(X.par + e[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int k = 0; k < PHD_LFMIS_B; k++) PHD_CONSIDER(e[k], we[k], st[k])
        }
        if (bu >= 0 && (bs < 0 || earlier(wu, bu, ws, bs))) return true;  // an undecided one precedes the first seed
        __hip_atomic_store(X.par + i, (short)(bs >= 0 ? bs : -2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return false;
    };
    if (PHD_XK == 7) {
        for (int i = tid; i < K; i += NT) X.par[i] = -2;
    } else {
        // Each wave owns the active-list slots wid*64 + k*NT + lane (k = 0, 1, ..)
        // and keeps its still-pending candidates compacted in place at the front
        // of its own slots (ballot + mbcnt; a write never passes an unread slot
        // of the wave, and no other wave touches them), so after round 1 a wave
        // iterates over its pending candidates only — no decided-check loads,
        // no empty batches.
        const int lane = tid & 63, wid = tid >> 6;
        auto wslot = [&](int j) { return wid * 64 + (j >> 6) * NT + (j & 63); };
        const int w_first = wid * 64;
        // this wave's slots below nact: full batches of 64 plus the partial one
        int cnt_w = nact > w_first ? ((nact - w_first) / NT) * 64 + min(64, (nact - w_first) % NT) : 0;
        for (int round = 0;; round++) {
            nrounds = round + 1;
            int kept = 0;  // wave-uniform
            for (int j0 = 0; j0 < cnt_w; j0 += 64) {
                const int j = j0 + lane;
                const bool live = j < cnt_w;
                const int i = live ? alist[wslot(j)] : 0;
                const bool pend = live && lfmis_try(i);
                const unsigned long long b = __ballot(pend);
                if (pend) {
                    const int r = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned)b, 0));
                    alist[wslot(kept + r)] = (unsigned short)i;
                }
                kept += __builtin_popcountll(b);
            }
            cnt_w = kept;
#if PHD_LFMIS_ASYNC
            // each wave re-scans its own pending candidates until none is left,
            // reading the other waves' decisions as they land (a decision is
            // final, and one read early only decides earlier): no workgroup
            // barrier per round.  The workgroup's highest-priority undecided
            // candidate can always decide, so some wave always progresses.
            if (kept == 0) break;  // (wave-uniform)
            if (round > 64 * K + 64) {  // failsafe: never hang; the serial greedy takes over
                if (lane == 0) s_misc[3] = 1;
                break;
            }
#else
            if (!block_or<NT, false>(kept, sb_at<NT>(s_w, sbk))) break;  // (its barrier publishes this round's decisions)
            if (round > K) {  // failsafe: never hang; the serial greedy takes over
                if (tid == 0) s_misc[3] = 1;
                break;
            }
#endif
        }
    }
#undef PHD_CONSIDER
    __syncthreads();
    if (s_misc[3]) return -1;
    STAMP(20);
    // M6: seeds emit their merge sets, in candidate-index order of the seeds.
    // Members are summed in candidate-index order (seed included), the order of
    // the greedy's own sums, so the moments are the greedy's bit for bit.
    // Isolated seeds take the one-member form of the same arithmetic; seeds with
    // neighbours are listed and emitted densely afterwards.
    unsigned int* slist = (unsigned int*)X.edges;  // (seed << 16 | slot), the edge list is dead
    int nout = 0, nclu = 0;
    for (int base = 0; base < K; base += 1024) {
        // seed slots (their rank in candidate-index order) and the clustered
        // seeds' list positions: one barrier per 1024 candidates
        int v[RB][1], pre[RB][1], tot[1];  // seed | clustered seed << 16
#pragma unroll
        for (int r = 0; r < RB; r++) {
            const int i = base + r * NT + tid;
            const bool seed = (i < K) && X.par[i] == -2;
            v[r][0] = seed ? ((X.off[i + 1] > X.off[i]) ? 0x10001 : 1) : 0;
        }
        block_scan_batch<NT, 1>(v, pre, tot, s_scan, sbb);
#pragma unroll
        for (int r = 0; r < RB; r++) {
            const int i = base + r * NT + tid;
            if (!v[r][0]) continue;
            const int slot = nout + (pre[r][0] & 0xffff);
            if (v[r][0] >> 16) {
                slist[nclu + (pre[r][0] >> 16)] = ((unsigned int)i << 16) | (unsigned int)min(slot, 65535);
            } else {
                emit_single(dst, cap, slot, X.K.P[i], X.K.V(i));  // an isolated seed (D15)
            }
        }
        nout += tot[0] & 0xffff;
        nclu += tot[0] >> 16;
    }
#ifdef PHD_STAMPS
    if (tid == 0 && a.stamps) {
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 46] = ((unsigned long long)nrounds << 32) | (unsigned)nact;
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 47] = ((unsigned long long)nclu << 32) | (unsigned)nout;
    }
#endif
    (void)nrounds;
    __syncthreads();  // slist complete
    for (int c2 = tid; c2 < (PHD_XK == 9 ? 0 : nclu); c2 += NT) {
        const int i = (int)(slist[c2] >> 16), slot = (int)(slist[c2] & 0xffffu);
        if (slot >= cap) continue;
        const int o = X.off[i], nd = X.off[i + 1] - o;
        double cv[4] = {0.0, 0.0, 0.0, 0.0};
        float Wf, gx, gy;
        if (nd <= MERGE_DEG_REG2) {
            // (the longer rows, 8 < nd <= 12: three in ten particles at config 3
            // with births hold one, the rest of their wave masked off meanwhile)
            if (!(nd <= MERGE_DEG_REG ? cluster_moments<MERGE_DEG_REG>(X, i, o, nd, Wf, gx, gy, cv)
                                      : cluster_moments<MERGE_DEG_REG2, 2>(X, i, o, nd, Wf, gx, gy, cv))) {
                emit_single(dst, cap, slot, X.K.P[i], X.K.V(i));
                continue;
            }
        } else {
            // a long adjacency list: members enumerated in candidate-index order by scans
            double W = 0.0, sx = 0.0, sy = 0.0;
            auto next_member = [&](int last) {
                int nx = i > last ? i : INT_MAX;
                for (int r = 0; r < nd; r++) {
                    const int j = X.pool[o + r];
                    if (j > last && j < nx && X.par[j] == i) nx = j;
                }
                return nx;
            };
            {
                const int j0 = next_member(-1);
                if (j0 == i && next_member(i) == INT_MAX) {  // every neighbour went to another seed (D15)
                    emit_single(dst, cap, slot, X.K.P[i], X.K.V(i));
                    continue;
                }
            }
            for (int j = next_member(-1); j != INT_MAX; j = next_member(j)) {
                const float4 pj = X.K.P[j];
                W += (double)pj.z;
                sx += (double)(pj.z * pj.x);
                sy += (double)(pj.z * pj.y);
            }
            Wf = (float)W;
            const float rW = 1.0f / Wf;
            gx = (float)sx * rW;
            gy = (float)sy * rW;
            for (int j = next_member(-1); j != INT_MAX; j = next_member(j)) {
                const float4 pj = X.K.P[j], vj = X.K.V(j);
                const float d0 = gx - pj.x, d1 = gy - pj.y, w = pj.z;
                cv[0] += (double)(w * (vj.x + d0 * d0));
                cv[1] += (double)(w * (vj.y + d0 * d1));
                cv[2] += (double)(w * (vj.z + d1 * d0));
                cv[3] += (double)(w * (vj.w + d1 * d1));
            }
        }
        emit_merged(dst, cap, slot, Wf, gx, gy, cv);
    }
    return nout;
}

/* Replay restore + fused predict of particle n (thread 0 of its workgroup). */
template <bool PRED>
__device__ __forceinline__ phd_pose fused_predict(const UpdateArgs& a, int n) {
    phd_pose ps = a.pose_prior ? a.pose_prior[n] : a.poses[n];
    if (a.logw_prior) a.logw[n] = a.logw_prior[n];  // replay: restore the fixed prior
    if (PRED && a.predict) {
        for (int k = 0; k < a.pc.subdivide; k++) {
            const uint64_t st = a.pstep * (uint64_t)a.pc.subdivide + (uint64_t)k;
            if (a.predict == 1) {
                float n_alpha, n_enc;
                ackerman_noise(a.pseed, a.pc.index_offset + n, st, a.pc, &n_alpha, &n_enc);
                ps = predict_ackerman_one(ps, a.pu, n_alpha, n_enc, a.pc);
            } else {
                ps = predict_cv_one(ps, cv_noise(a.pseed, a.pc.index_offset + n, st, a.pc), a.pc);
            }
        }
        a.poses[n] = ps;
    }
    return ps;
}

/* Log cardinality distribution of each particle after a CPHD update:
 * cn[n] = log p(n) + Ψ0(n) - <Ψ0,p> from the coefficients k_cphd_terms stored
 * (one block per particle, threads over n). */
__global__ void __launch_bounds__(256)
    k_cphd_cardinality(const int* __restrict__ src, const double* __restrict__ cn_coef,
                       const double* __restrict__ cn_x, int stride, const double* __restrict__ lfact, int Nmax,
                       int n, float* __restrict__ out) {
    const int p = blockIdx.x;
    if (p >= n) return;
    // coefficients live with the slab (row n = the posterior slab the update of
    // particle n wrote), so a resample's index remap carries them like the map
    const int sref = src ? src[p] : p;
    const double* co = ((sref & PHD_SLAB_X) ? cn_x : cn_coef) + (size_t)(sref & PHD_SLAB_MASK) * stride;
    const double ip0 = co[0], lq = co[1], lw = co[2], logW = co[3], W = co[4];
    const int M = (int)co[5];
    for (int k = threadIdx.x; k <= Nmax; k += blockDim.x) {
        double mx = -INFINITY;
        if (k > 0 && !(W > 0)) {  // an empty map predicts n = 0 only: p(k) = 0, no ∞ - ∞
            out[(size_t)p * (Nmax + 1) + k] = PHD_LOG0;
            continue;
        }
        for (int j = 0; j <= min(k, M); j++) {
            const double b = co[6 + j];
            if (b == -INFINITY) continue;
            const double t = b + (k > 0 ? (double)k * logW : 0.0) - W - lfact[k - j] +
                             (k - j > 0 ? (double)(k - j) * lq : 0.0) - (k > 0 ? (double)k * lw : 0.0);
            mx = fmax(mx, t);
        }
        double sum = 0.0;
        if (mx != -INFINITY)
            for (int j = 0; j <= min(k, M); j++) {
                const double b = co[6 + j];
                if (b == -INFINITY) continue;
                const double t = b + (k > 0 ? (double)k * logW : 0.0) - W - lfact[k - j] +
                                 (k - j > 0 ? (double)(k - j) * lq : 0.0) - (k > 0 ? (double)k * lw : 0.0);
                sum += exp(t - mx);
            }
        out[(size_t)p * (Nmax + 1) + k] = mx == -INFINITY ? PHD_LOG0 : (float)(log(sum) + mx - ip0);
    }
}

/* Bearing window of an in-range component (phase 2): since d >= kappa db^2
 * (kappa = S3 - S12^2 / 4 S0, the minimum of the quadratic form over the range
 * innovation), a measurement further than hw = sqrt(2 (C2 - floor) / (k2 kappa))
 * in bearing has log2 q < floor (factor 2 on d for float rounding): it is not
 * walked (oracle deviation D7; the walk floor is DevCfg::walk_floor).  Returns
 * lo | count << 16, a circular range of the bearing-sorted valid measurements. */
__device__ __forceinline__ unsigned int bearing_window(float C2, float S0, float S12, float S3, float bearing,
                                                       float floor2, int Mv, const unsigned short* s_zbin) {
    const float k2 = 0.72134752044448170f;  // log2(e)/2
    unsigned int win = (unsigned int)Mv << 16;  // lo 0, count Mv: every valid measurement
    if (!(C2 > floor2) && C2 == C2) return 0;   // every pair below the floor
    // (approximate reciprocals: the window is a bound with margins — hw x 1.001
    // + 1e-4 and a bin either side — and an S0 too small for its reciprocal
    // gives kap <= 0, the whole ring; part A -1.9 us at config 3 against IEEE
    // divisions)
    const float kap = S3 - S12 * S12 * __builtin_amdgcn_rcpf(4.f * S0);
    if (S0 > 0.f && kap > 0.f && kap < INFINITY && C2 < 1e30f) {
        const float hw = sqrtf(2.f * (C2 - floor2) * __builtin_amdgcn_rcpf(k2 * kap)) * 1.001f + 1e-4f;
        // conservative bins of the host-built table (bin width 2pi/PHD_ZBINS)
        const float ibinw = PHD_ZBINS / 6.28318530717958648f;
        const int ba = (int)floorf((bearing - hw + 3.14159265358979f) * ibinw) - 1;
        const int bc = (int)floorf((bearing + hw + 3.14159265358979f) * ibinw) + 2;
        if (bc - ba < PHD_ZBINS) {
            const int fa = ba >= 0 ? ba / PHD_ZBINS : -((PHD_ZBINS - 1 - ba) / PHD_ZBINS);
            const int fc = bc >= 0 ? bc / PHD_ZBINS : -((PHD_ZBINS - 1 - bc) / PHD_ZBINS);
            const int ia = s_zbin[ba - fa * PHD_ZBINS] + fa * Mv;
            const int ic = s_zbin[bc - fc * PHD_ZBINS] + fc * Mv;
            const int lo = ia - fa * Mv;
            win = (unsigned int)lo | ((unsigned int)min(ic - ia, Mv) << 16);
        }
    }
    return win;
}

/* one walked term into the two-level fixed point of its measurement: terms
 * q >= 2^-17 as q 2^40 (hi, exact: their ulp is >= 2^-40), smaller ones as
 * q lo_scale (lo: 2^70, or 2^60 for maps above 2047 components — headroom for
 * the term count); order independent, so deterministic.  q >= 2^20 would
 * exhaust hi's headroom: PHD_ST_ETA_RANGE. */
__device__ __forceinline__ void eta_term(unsigned long long* ehi, unsigned long long* elo, int m, float q,
                                         float lo_scale, int& flags) {
    flags |= q >= 1048576.f ? PHD_ST_ETA_RANGE : 0;
    const bool hi = q >= 7.62939453125e-06f;  // 2^-17
    const unsigned long long y = (unsigned long long)(fminf(q, 4194304.f) * (hi ? 1099511627776.f : lo_scale));
#if PHD_XK == 11
    if (y) (hi ? ehi : elo)[m] += y;
#else
    if (y) atomicAdd((hi ? ehi : elo) + m, y);
#endif
}

template <int NT>
__device__ void rs_step_block(const RsStepArgs& a, unsigned char* smem);

template <int NT, bool PRED, bool CPHD = false, int PART = 0>
__device__ __forceinline__ void update_body(const UpdateArgs& a) {
    static_assert(!CPHD || PART != 0, "the CPHD update runs as three launches (part A, k_cphd_terms, part C)");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // part C's lead workgroups (UpdateArgs::rs_lead): the first runs the step's
    // resample, the others return; the particles follow, each on its XCD
    const int lead = PART == 2 ? a.rs_lead : 0;
    if (PART == 2 && (int)blockIdx.x < lead) {
        if (blockIdx.x == 0) rs_step_block<NT>(a.rs, smem);
        return;
    }
    const int b_ = (int)blockIdx.x - lead, grid_ = (int)gridDim.x - lead;
    const UpdLds L = upd_lds_layout(a.cap, a.Mcap, a.Kcap, a.Scap, a.Epool, NT, CPHD ? 1 : 0, PART);
    float* s_zr = (float*)(smem + L.zr);
    float* s_zb = (float*)(smem + L.zb);
    int* s_zok = (int*)(smem + L.zok);
    float* s_leta = (float*)(smem + L.leta);
    float* s_thr = (float*)(smem + L.thr);  // CPHD: per-measurement listing bound
    // bearing-sorted valid measurements (range, bearing, index, key); part C: global (pass 1 only)
    const float4* s_zs = PART == 2 ? a.zs : (const float4*)(smem + L.zs);
    unsigned long long* s_etafx = (unsigned long long*)(smem + L.etafx);  // η / Σq fixed point, terms >= 2^-17 (2^40)
    unsigned long long* s_etalo = (unsigned long long*)(smem + L.etalo);  // smaller terms (lo scale)
    // first sorted measurement of each bearing bin; part C: global
    const unsigned short* s_zbin = PART == 2 ? a.zbin : (const unsigned short*)(smem + L.zbin);
    unsigned short* s_out = (unsigned short*)(smem + L.out);  // part C: the handoff's list (set below)
    int* s_cnt = (int*)(smem + L.cnt);  // [0]=n_in [1]=n_near [2]=n_out [3]=n_surv
    int* s_scr = (int*)(smem + L.scr);  // [0..15] block-helper scratch, [16..63] classification
    double* s_red = (double*)(smem + L.red);
    float* s_redf = (float*)(smem + L.redf);
    // region D, phases 1-4: in / near lists, detection-term keys
    unsigned short* s_in = (unsigned short*)(smem + L.in);
    unsigned short* s_near = (unsigned short*)(smem + L.near);
    unsigned int* s_skey = (unsigned int*)(smem + L.skey);
    unsigned int* s_skey2 = (unsigned int*)(smem + L.skey2);
    // region C: comp table (phases 2-3) / candidates (phase 4) / merge lists (phase 5)
    float4* t_a = (float4*)(smem + L.u);             // (r, bearing, S0, S1+S2)
    float2* t_b = (float2*)(smem + L.u + 16 * (size_t)a.cap);  // (S3, C2)
    unsigned int* t_w = (unsigned int*)(smem + L.u + 24 * (size_t)a.cap);  // bearing window lo | count << 16
    int* t_pre = (int*)(smem + L.u + 28 * (size_t)a.cap);                  // prefix of window counts (cap + 1)
    unsigned short* t_start = (unsigned short*)(smem + L.u + 32 * (size_t)a.cap + 16);  // walk chunk starts (NT)
    MergeScratch X;
    X.K.P = (float4*)(smem + L.u);
    X.K.detv = (float4*)(smem + L.detv);
    X.K.cap = a.cap;
    X.par = (short*)(smem + L.mpar);
    X.off = (unsigned short*)(smem + L.moff);
    X.cur = (unsigned short*)(smem + L.mcur);
    X.edges = (unsigned int*)(smem + L.medge);
    X.pool = (unsigned short*)(smem + L.mpool);
    X.plist = (unsigned int*)(smem + L.mpar);
    X.plcap = (int)((L.mpool + 4 * (size_t)a.Epool - L.mpar) / 4);
    X.key = (unsigned short*)(smem + L.skeyidx);
    X.gstart = (unsigned short*)(smem + L.gstart);
    X.st_tests = nullptr;

    const int n = upd_particle(a, b_, grid_);
    const int tid = threadIdx.x;
#ifdef PHD_STAMPS
    // the workgroup's residency on the device-wide real-time clock (100 MHz):
    // the launch's timeline of resident workgroups (slots 48 / 49)
    if (tid == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 48] = __builtin_amdgcn_s_memrealtime();
#endif
    const DevCfg& c = a.c;
    const int M = a.M;
    // slab of particle n: set `in` (or the migration set X) via the index table
    const int sref = a.src ? a.src[n] : n;
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int slab = sref & PHD_SLAB_MASK;
    const int G = in_x ? a.size_x[slab] : a.size_in[slab];
    const G1 float* __restrict__ src = g1(uni_p((in_x ? a.map_x : a.map_in) + (size_t)slab * NF * a.cap));
    // the step's births (CPHD: the previous scan's inverse measurements through
    // the prediction, phdfilter.cu.bak:738-870): prior components G .. Gp - 1
    // after the slab's G, placed by the classify below from the predicted pose
    // and kept in this particle's birth slab for part C (appended to the map as
    // addBirths does, without copying the slab)
    const int Mb = a.births ? max(0, min(a.Mb, a.cap - G)) : 0;
    const int Gp = G + Mb;
    G1 float* __restrict__ bdst = a.births ? g1(uni_p(a.births + (size_t)n * NF * a.cap)) : nullptr;
    const G1 float* __restrict__ bsrc = a.births ? bdst - G : src;  // (indexed by prior component k >= G)
    // prior component k's field row: slab or birth slab
    auto prior = [&](int k) -> const G1 float* { return (k < G ? src : bsrc) + k; };
    X.K.src = src;
    X.K.bsrc = bsrc;
    X.K.G = G;
    G1 float* __restrict__ dst = g1(uni_p(a.map_out + (size_t)n * NF * a.cap));
    // fused predict (phd_step): thread 0 advances this particle's pose through
    // the sub-steps (a call, so its registers do not count against the body's)
    phd_pose& s_pose = *(phd_pose*)(smem + L.pose);
    // workgroup-uniform doubles needed phases later: [0] Σ pd w in range,
    // [1..3] CPHD Σw in range, Σ(1-pd)w, Σw; [4] (float) CPHD non-detection factor
    double* s_uni = (double*)(smem + L.uni);
    // the launch's last a.prio workgroups at the highest wave priority
    // (prio_tail in phd_capi.hip): they finish the launch, and their
    // instructions issue ahead of the earlier workgroups' on a shared SIMD
    if (b_ >= grid_ - a.prio) __builtin_amdgcn_s_setprio(3);
    // three-launch CPHD: this particle's handoff (part A writes it, part C reads it)
    const CphdHand H = cphd_hand_layout(a.cap, a.Mcap, a.Scap);
    unsigned char* hand = PART ? a.hand + (size_t)n * H.stride : nullptr;
    if (PART == 1) {  // part A: classification and listing write straight into the handoff
        s_out = (unsigned short*)(hand + H.out);
        s_in = (unsigned short*)(hand + H.in);
        s_near = (unsigned short*)(hand + H.near);
        s_skey = (unsigned int*)(hand + H.skey);
    }
    if (PART == 2) {  // part C: the lists and the detection covariances stay in its handoff (LDS for occupancy)
        s_out = (unsigned short*)(hand + H.out);
        s_in = (unsigned short*)(hand + H.in);
        s_near = (unsigned short*)(hand + H.near);
        X.K.detv = (float4*)(hand + H.detv);
        s_zr = const_cast<float*>(a.zr);
        s_zb = const_cast<float*>(a.zb);
        s_zok = const_cast<int*>(a.zok);
        if (CPHD) {  // (the PHD part C computes its normalisers into LDS)
            s_leta = (float*)(hand + H.leta);
            s_thr = (float*)(hand + H.thr);
        }
        unsigned char* tb = hand + H.table;
        t_a = (float4*)tb;
        t_b = (float2*)(tb + 16 * (size_t)a.cap);
        t_w = (unsigned int*)(tb + 24 * (size_t)a.cap);
        t_pre = (int*)(tb + 28 * (size_t)a.cap);
        t_start = (unsigned short*)(tb + 32 * (size_t)a.cap + 16);
    }
    // the first PF rows of NT components of the prior slab, all 7 fields, issued
    // first thing: one HBM round trip, overlapped with the staging of
    // the measurements below, instead of two per row inside the classify loop
    // (part C: the rows its non-detection candidates read, and the handoff's
    // counts and first list entries, all issued here: one round trip instead of
    // a chain of dependent ones after the measurement staging)
    constexpr int PF = 2;
    float pf[PF][NF];
#pragma unroll
    for (int it = 0; it < PF; it++) {
        const int k = it * NT + tid;
#pragma unroll
        for (int f = 0; f < NF; f++) pf[it][f] = (k < G) ? src[f * a.cap + k] : 0.f;  // (births: placed below)
    }
    int hp_cnt[5] = {0, 0, 0, 0, 0};
    unsigned int hp_skey = 0;
    float hp_leta = 0.f, hp_thr = 0.f, hp_nd = 0.f;
    int hp_wide = 0;
    unsigned long long hp_eta[2] = {0ull, 0ull};
    if constexpr (PART == 2) {
        const int* hc = (const int*)(hand + H.cnt);
#pragma unroll
        for (int i = 0; i < 5; i++) hp_cnt[i] = hc[i];
        if (tid < a.Scap) hp_skey = ((const unsigned int*)(hand + H.skey))[tid];
        if (CPHD) {
            if (tid < M) {
                hp_leta = ((const float*)(hand + H.leta))[tid];
                hp_thr = ((const float*)(hand + H.thr))[tid];
            }
            hp_nd = ((const float*)(hand + H.misc))[0];
            hp_wide = ((const int*)(hand + H.misc))[1];
        } else if (tid < M) {  // the PHD part C: its measurement's eta fixed point
            hp_eta[0] = ((const unsigned long long*)(hand + H.ehi))[tid];
            hp_eta[1] = ((const unsigned long long*)(hand + H.elo))[tid];
        }
    }
    // the predict after the prefetch loads have issued: its pose load and
    // arithmetic overlap their round trip (the pose is read after the barrier below)
    if (tid == 0) s_pose = fused_predict<PRED && PART != 2>(a, n);

    const int Mv = a.Mv;
    for (int m = tid; m < M; m += NT) {
        if (PART == 0) {
            s_zr[m] = a.zr[m];
            s_zb[m] = a.zb[m];
            s_zok[m] = a.zok[m];
        }
        if (PART != 2) {
            s_etafx[m] = 0ull;
            s_etalo[m] = 0ull;
        }
    }
    if (PART != 2) {
        for (int m = tid; m < Mv; m += NT) ((float4*)(smem + L.zs))[m] = a.zs[m];
        for (int b = tid; b < PHD_ZBINS; b += NT) ((unsigned short*)(smem + L.zbin))[b] = a.zbin[b];
    }
    if (tid < 16) s_cnt[tid] = 0;
    __syncthreads();
    const phd_pose pose = s_pose;
    STAMP(0);

    /* Phases 1+2 in one pass over the prior: 3-way range classification
     * (computeInRangeKernel :1328-1346), order-preserving split into in / near
     * / out index lists, and for in-range components the EKF terms
     * (preUpdateSynthKernel :1824-1925) -> LDS pair table at their compacted
     * index, in the log2 domain: log2 q_jm = C2_j - (log2(e)/2) d_jm.
     * Bearing window: d_jm >= kappa_j * db^2 (kappa_j = S3 - S12^2 / 4 S0, the
     * minimum of the quadratic form over the range innovation), so a
     * measurement whose bearing is further than hw_j = sqrt(2 (C2_j + 160) /
     * (k2 kappa_j)) from the component's has l2q < -160 (with a factor 2 on d
     * for float rounding): exp2 underflows to +0 and the pair is not evaluated
     * (oracle deviation D7; the sums are unchanged).  The window is a circular
     * range of the bearing-sorted valid measurements. */
    const float k2 = 0.72134752044448170f;  // log2(e)/2
    double card_d = 0.0;
    double win_d = 0.0, qd_d = 0.0, wall_d = 0.0;  // CPHD: Σw in range, Σ(1-pd)w in range, Σw whole map
    // running in / near / out counts (every thread holds them); the per-wave
    // counts of a batch go to one of two scratch buffers by batch parity, so
    // one barrier per batch suffices (a wave writing buffer b again has passed
    // the next batch's barrier, which every wave reaches after reading b)
    int n1r = 0, n2r = 0, n0r = 0;
    constexpr int NW = NT / 64;
    // safeLog(pd) once: a component's detection probability is pd or 0, so its
    // log is this or PHD_LOG0 (the same bits as d_safe_log(e.pd))
    const float lpd = d_safe_log(c.pd);
    for (int base = 0; base < (PART == 2 ? 0 : Gp); base += NT) {
        const int k = base + tid;
        int cls = -1;
        float4 ta = make_float4(0.f, 0.f, 0.f, 0.f);
        float2 tb = make_float2(0.f, 0.f);
        unsigned int win = 0;
        if (k < Gp) {
            float v[NF];  // this component's fields: prefetched rows, else loaded here
            if (k >= G) {
                // the step's birth k - G, placed here from the predicted pose
                // (birthsKernel, phdfilter.cu.bak:757-784) and kept in the birth slab
                // for the later phases / part C
                const int m = a.bzvi[k - G];
                float mean[2], cov[4];
                d_birth(c, pose.px, pose.py, pose.ptheta, a.bzr[m], a.bzb[m], mean, cov);
                v[0] = c.birthWeight;
                v[1] = mean[0];
                v[2] = mean[1];
                v[3] = cov[0];
                v[4] = cov[1];
                v[5] = cov[2];
                v[6] = cov[3];
#pragma unroll
                for (int f = 0; f < NF; f++) bdst[f * a.cap + (k - G)] = v[f];
            } else if (base == 0) {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = pf[0][f];
            } else if (base == NT) {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = pf[1][f];
            } else {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = src[f * a.cap + k];
            }
            const float dx = v[1] - pose.px;
            const float dy = v[2] - pose.py;
            const float r2 = dx * dx + dy * dy;
            const float r = sqrtf(r2);
            const float bearing = d_wrap((PHD_XK == 13 ? atan2f(dy, dx) : phd_atan2f(dy, dx)) - pose.ptheta);
            const float ab = fabsf(bearing);
            if (CPHD) wall_d += (double)v[0];
            if (r >= c.minRange && r <= c.maxRange && ab <= c.maxBearing)
                cls = 1;
            else if ((double)r >= 0.8 * (double)c.minRange && (double)r <= 1.2 * (double)c.maxRange &&
                     (double)ab <= 1.2 * (double)c.maxBearing)
                cls = 2;
            else
                cls = 0;
            if (cls == 1) {
                const float w = v[0];
                DevEkf e;
                d_ekf_from_geometry(c, dx, dy, r2, r, bearing, v[3], v[4], v[5], v[6], e);
                // C2 = log2(e) * (log pd + log w - log 2pi - 0.5 log det)
                const double lc =
                    (double)((e.pd > 0.f ? lpd : PHD_LOG0) + d_safe_log(w)) - c.log_2pi - 0.5 * (double)d_safe_log(e.det);
                const float C2 = (float)(1.4426950408889634 * lc);
                const float S12 = e.S1 + e.S2;
                ta = make_float4(e.r, e.bearing, e.S0, S12);
                tb = make_float2(e.S3, C2);
                card_d += (double)(e.pd * w);
                if (CPHD) {
                    win_d += (double)w;
                    qd_d += (double)(1 - e.pd) * (double)w;
                }
                win = bearing_window(C2, e.S0, S12, e.S3, e.bearing, c.walk_floor, Mv, s_zbin);
            }
        }
        const int lane = tid & 63, wid = tid >> 6;
        const unsigned long long b1 = __ballot(cls == 1), b2 = __ballot(cls == 2), b0 = __ballot(cls == 0);
        const unsigned long long lt = (1ull << lane) - 1ull;
        int* sb = s_scr + 16 + ((base / NT) & 1) * 3 * NW;
        if (lane == 0) {
            sb[wid] = __popcll(b1);
            sb[NW + wid] = __popcll(b2);
            sb[2 * NW + wid] = __popcll(b0);
        }
        __syncthreads();
        int o1 = n1r, o2 = n2r, o0 = n0r, t1 = 0, t2 = 0, t0 = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const int c1 = sb[w], c2 = sb[NW + w], c0 = sb[2 * NW + w];
            if (w < wid) {
                o1 += c1;
                o2 += c2;
                o0 += c0;
            }
            t1 += c1;
            t2 += c2;
            t0 += c0;
        }
        if (cls == 1) {
            const int j = o1 + __popcll(b1 & lt);
            s_in[j] = (unsigned short)k;
            t_a[j] = ta;
            t_b[j] = tb;
            t_w[j] = win;
            // (part C's detection terms take the range and bearing from here
            // instead of a square root and phd_atan2f each: the same bits)
            if (PART == 1) {
                G1 float* rbp = (G1 float*)(hand + H.rb) + 2 * j;
                rbp[0] = ta.x;
                rbp[1] = ta.y;
            }
        }
        if (cls == 2) s_near[o2 + __popcll(b2 & lt)] = (unsigned short)k;
        if (cls == 0) s_out[o0 + __popcll(b0 & lt)] = (unsigned short)k;
        n1r += t1;
        n2r += t2;
        n0r += t0;
    }
    if (PART != 2 && tid == 0) {  // (published by the barrier of the sums below)
        s_cnt[0] = n1r;
        s_cnt[1] = n2r;
        s_cnt[2] = n0r;
    }
    int Gin = PART == 2 ? s_cnt[0] : n1r;  // (near / out counts are re-read from LDS where used)
    STAMP(1);
    if constexpr (PART == 2) {
        // (part C classifies nothing: its sums come with the handoff)
    } else if (CPHD) {
        double v[4] = {card_d, win_d, qd_d, wall_d};
        block_sum<4, NT>(v, s_red);  // also orders phase-2 LDS writes before phase 3
        if (tid == 0) {
            s_uni[0] = v[0];
            s_uni[1] = v[1];
            s_uni[2] = v[2];
            s_uni[3] = v[3];
        }
    } else {
        double v[1] = {card_d};
        block_sum<1, NT>(v, s_red);  // also orders phase-2 LDS writes before phase 3
        if (tid == 0) s_uni[0] = v[0];
    }
    STAMP(2);
    /* Phase 3: banded pair loop.  The window counts are prefix-summed and
     * every thread walks an equal contiguous chunk of the (component, window
     * entry) sequence, four entries per step: the four terms are evaluated
     * together, go to the two-level fixed point of their measurements (order
     * independent, so deterministic), and the ones that may survive the prune
     * are listed with one LDS atomic per wave and step (ballots). */
    {
        const float thr2 = c.lq_keep_thresh * 1.4426950408889634f;
        const float lo_scale = a.cap <= 2047 ? 1.1805916207174113e21f : 1.152921504606846976e18f;
        const int lane = tid & 63;
        const unsigned long long lt = (1ull << lane) - 1ull;
        int eflags = 0;
        int W = 0, chunk = 0;
        // work units (up to 4 consecutive window entries of one component), their
        // prefix, and each thread's first component
        auto plan_walk = [&]() {
            W = 0;
            for (int base = 0; base < Gin; base += NT) {
                const int j = base + tid;
                const int units = j < Gin ? (int)((t_w[j] >> 16) + 3) >> 2 : 0;
                int tot;
                const int pre = block_excl_scan<NT>(units, s_scr, &tot);
                if (j < Gin) t_pre[j] = W + pre;
                W += tot;
            }
            if (tid == 0) t_pre[Gin] = W;
            __syncthreads();
            chunk = (W + NT - 1) / NT;
            // chunk starts: component j owns the threads whose first unit lies in its range
            for (int j = tid; j < Gin && chunk > 0; j += NT) {
                const int t0 = (t_pre[j] + chunk - 1) / chunk, t1 = min((t_pre[j + 1] + chunk - 1) / chunk, NT);
                for (int t = t0; t < t1; t++) t_start[t] = (unsigned short)j;
            }
            __syncthreads();
        };
        auto walk = [&](const int pass) {
        const bool do_sum = pass == 0;
        const float thr_u = CPHD ? c.cphd_thr0 : thr2;  // pass 0 bound (CPHD: covers factors <= e^2/κ)
        const int w0 = tid * chunk, w1 = min(w0 + chunk, W);
#ifdef PHD_STAMPS
        int st_pairs = 0, st_qpos = 0;  // per-thread counts, one atomic each after the walk
#endif
        int j = w0 < w1 ? t_start[tid] : 0;
        STAMP(25);
        int jbeg = t_pre[j], jend = t_pre[j + 1];
        // every lane runs `chunk` steps (lanes past their range idle): wave-uniform
        // control flow, so the listing can aggregate with ballots
        for (int it = 0; it < (PHD_XK == 1 ? 0 : chunk); it++) {
            const int w = w0 + it;
            const bool act = w < w1;
            if (act && w == jend) {
                j++;
                while (t_pre[j + 1] <= w) j++;
                jbeg = t_pre[j];
                jend = t_pre[j + 1];
            }
            const float4 ta = t_a[j];
            const float2 tb = t_b[j];
            const unsigned int win = t_w[j];
            const int cnt = act ? (int)(win >> 16) : 0;
            const int e0 = 4 * (w - jbeg);
            int ms = (int)(win & 0xffffu) + (act ? e0 : 0);
            while (ms >= Mv) ms -= Mv;
            float4 z[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                z[k] = s_zs[ms];
                ms = (ms + 1 == Mv) ? 0 : ms + 1;
            }
            float l2q[4];
            int mm[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float i0 = z[k].x - ta.x;
                float i1 = z[k].y - ta.y;
                if (fabsf(i1) > 3.14159250f) i1 = d_wrap(i1);  // rare: wrapAngle's ±2pi branch
                const float u = __builtin_fmaf(i0, ta.z, i1 * ta.w);
                const float dist = __builtin_fmaf(i0, u, i1 * i1 * tb.x);
                l2q[k] = e0 + k < cnt ? __builtin_fmaf(-k2, dist, tb.y) : -INFINITY;
                mm[k] = __float_as_int(z[k].z);
            }
            if (do_sum) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float q = __builtin_amdgcn_exp2f(l2q[k]);
                    if (PHD_XK != 12 && q > 0.f) eta_term(s_etafx, s_etalo, mm[k], q, lo_scale, eflags);
#ifdef PHD_STAMPS
                    st_pairs += e0 + k < cnt;
                    st_qpos += q > 0.f;
#endif
                }
            }
            bool lst[4];
#pragma unroll
            for (int k = 0; k < 4; k++) lst[k] = l2q[k] >= (pass == 0 ? thr_u : s_thr[e0 + k < cnt ? mm[k] : 0]);
            unsigned long long bl[4];
#pragma unroll
            for (int k = 0; k < 4; k++) bl[k] = __ballot(lst[k]);
            const int c0 = __popcll(bl[0]), c1 = __popcll(bl[1]), c2 = __popcll(bl[2]), c3 = __popcll(bl[3]);
            const int ntot = c0 + c1 + c2 + c3;
            if (ntot) {  // wave-uniform
                int base = 0;
                if (lane == 0) base = atomicAdd(&s_cnt[3], ntot);
                base = __shfl(base, 0, 64);
                const int off[4] = {base, base + c0, base + c0 + c1, base + c0 + c1 + c2};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int sl = off[k] + __popcll(bl[k] & lt);
                    if (lst[k] && sl < a.Scap) s_skey[sl] = ((unsigned int)mm[k] << 16) | (unsigned int)j;
                }
            }
        }
#ifdef PHD_STAMPS
        atomicAdd(&s_cnt[8 + pass], st_pairs);
        atomicAdd(&s_cnt[10 + pass], st_qpos);
#endif
        if (eflags) atomicOr(&s_cnt[14], eflags);
        __syncthreads();
        };
        if constexpr (PART != 2) {
        plan_walk();
#ifdef PHD_STAMPS
        if (tid == 0) s_cnt[12] = W;
#endif
        STAMP(21);
        walk(0);
        if constexpr (PART == 1) {
            // three-launch CPHD: hand the particle over to k_cphd_terms and part C
            int* hc = (int*)(hand + H.cnt);
            if (tid == 0) {
                hc[HAND_GIN] = Gin;
                hc[HAND_GNEAR] = s_cnt[1];
                hc[HAND_GOUT] = s_cnt[2];
                hc[HAND_NSURV] = s_cnt[3];
                hc[HAND_FLAGS] = s_cnt[14];
            }
            if (tid < 4) ((double*)(hand + H.sums))[tid] = s_uni[tid];
            for (int m = tid; m < M; m += NT) {
                ((unsigned long long*)(hand + H.ehi))[m] = s_etafx[m];
                ((unsigned long long*)(hand + H.elo))[m] = s_etalo[m];
            }
            if constexpr (!CPHD) {
                // the split PHD update: Δ log w here, where the normalisers are
                // complete (the same expressions and summation order as the fused
                // form below) — the log-weight is final after part A, so a sharded
                // step's all-gather and plan can run beside part C
                static_assert(NT >= 256, "one measurement per thread (M <= 256)");
                float lt = 0.f;
                if (tid < M) {
                    float sum;
                    if (Gin > 0) {
                        double sd = (double)s_etafx[tid] * 9.094947017729282e-13 +  // 2^-40
                                    (double)s_etalo[tid] * (a.cap <= 2047 ? 8.470329472543003e-22 : 8.673617379884035e-19);
                        sd += (double)c.kappa;
                        sd += (double)c.birthWeight;
                        sum = (float)sd;
                    } else {
                        sum = c.kappa + c.birthWeight;
                    }
                    lt = d_det_safe_log(sum);  // (D17)
                }
                __syncthreads();  // (every eta read: the terms go over the fixed point)
                if (tid < M) ((float*)s_etafx)[tid] = lt;
                __syncthreads();
                if (tid == 0) {
                    float pw = 0.f;
                    for (int m = 0; m < M; m++) pw += ((const float*)s_etafx)[m];
                    const float cardp = (float)(s_uni[0] + (double)M * (double)c.birthWeight);
                    const float delta = pw - cardp;
                    a.delta[n] = delta;
                    const float nw = a.logw[n] + delta;
                    a.logw[n] = nw;
                    if (a.logw_out) a.logw_out[n] = nw;
                }
            }
            STAMP(9);
            return;
        }
        } else {
            // split update, part C: the particle from its handoff (and, CPHD, the
            // terms; counts and first entries prefetched at the kernel start)
            if (tid == 0) {
                s_cnt[0] = hp_cnt[HAND_GIN];
                s_cnt[1] = hp_cnt[HAND_GNEAR];
                s_cnt[2] = hp_cnt[HAND_GOUT];
                s_cnt[3] = hp_cnt[HAND_NSURV];
                s_cnt[14] = hp_cnt[HAND_FLAGS];
                ((float*)(s_uni + 4))[0] = hp_nd;  // non-detection log factor
                ((float*)(s_uni + 4))[1] = phd_det_expf(hp_nd);  // its exp (D18: as the oracle)
                s_uni[5] = (double)hp_wide;       // wide
                if (!CPHD) s_uni[0] = ((const double*)(hand + H.sums))[0];  // Σ pd w in range
            }
            // (s_leta / s_thr point at the handoff's rows in part C)
            Gin = hp_cnt[HAND_GIN];
            const int nsk = min(hp_cnt[HAND_NSURV], a.Scap);
            for (int q = tid; q < nsk; q += NT) s_skey[q] = q == tid ? hp_skey : ((const unsigned int*)(hand + H.skey))[q];
            __syncthreads();
            if (CPHD && (s_uni[5] != 0.0 || s_cnt[3] > a.Scap)) {
                // pass 1 (rare): the pair table again, windows down to the lowest
                // per-measurement bound, and the listing walk
                float tm = INFINITY;
                for (int m = tid; m < M; m += NT) tm = fminf(tm, s_thr[m]);
                const float fl = fminf(c.walk_floor, -block_max_f<NT>(-tm, s_redf) - 1.f);
                for (int q = tid; q < Gin; q += NT) {
                    const int k = s_in[q];
                    const G1 float* sk = prior(k);
                    const float dx = sk[1 * a.cap] - pose.px;
                    const float dy = sk[2 * a.cap] - pose.py;
                    const float r2 = dx * dx + dy * dy;
                    const float r = sqrtf(r2);
                    const float bearing = d_wrap(phd_atan2f(dy, dx) - pose.ptheta);
                    DevEkf e;
                    d_ekf_from_geometry(c, dx, dy, r2, r, bearing, sk[3 * a.cap], sk[4 * a.cap], sk[5 * a.cap],
                                        sk[6 * a.cap], e);
                    const double lc = (double)(d_safe_log(e.pd) + d_safe_log(sk[0])) - c.log_2pi -
                                      0.5 * (double)d_safe_log(e.det);
                    const float C2 = (float)(1.4426950408889634 * lc);
                    const float S12 = e.S1 + e.S2;
                    t_a[q] = make_float4(e.r, e.bearing, e.S0, S12);
                    t_b[q] = make_float2(e.S3, C2);
                    t_w[q] = bearing_window(C2, e.S0, S12, e.S3, e.bearing, fl, Mv, s_zbin);
                }
                __syncthreads();
                plan_walk();
                if (tid == 0) s_cnt[3] = 0;
                __syncthreads();
                walk(1);
            }
        }
        STAMP(22);
        if (!CPHD && tid < M) {
            float sum;
            if (Gin > 0) {
                const unsigned long long ehi = PART == 2 ? hp_eta[0] : s_etafx[tid];
                const unsigned long long elo = PART == 2 ? hp_eta[1] : s_etalo[tid];
                double sd = (double)ehi * 9.094947017729282e-13 +  // 2^-40
                            (double)elo * (a.cap <= 2047 ? 8.470329472543003e-22 : 8.673617379884035e-19);
                sd += (double)c.kappa;
                sd += (double)c.birthWeight;
                sum = (float)sd;
            } else {
                sum = c.kappa + c.birthWeight;
            }
            s_leta[tid] = d_det_safe_log(sum);  // (D17)
        }
        __syncthreads();
    }
    if (!CPHD && PART != 2 && tid == 0) {  // (the split form: in part A)
        float pw = 0.f;
        for (int m = 0; m < M; m++) pw += s_leta[m];
        const float cardp = (float)(s_uni[0] + (double)M * (double)c.birthWeight);
        const float delta = pw - cardp;
        a.delta[n] = delta;
        const float nw = a.logw[n] + delta;
        a.logw[n] = nw;
        if (a.logw_out) a.logw_out[n] = nw;
    }
    STAMP(3);
    int nsurv = s_cnt[3];
    int flags = s_cnt[14];  // PHD_ST_ETA_RANGE from the walk
    if (Mb < (a.births ? a.Mb : 0)) flags |= PHD_ST_MAP_OVERFLOW;  // births beyond the map capacity dropped
    if (nsurv > a.Scap) {
        flags |= PHD_ST_SURVIVOR_OVERFLOW;
        nsurv = a.Scap;
    }

    /* Listed detection terms into update-array order (m-major, j): a counting
     * sort by measurement (one LDS atomic per key), then each key's rank inside
     * its measurement's bucket (keys are unique; buckets hold a few entries).
     * Scratch: the start of region C (the pair table / candidates are dead / not
     * yet written here). */
    {
        int* b_cnt = (int*)(smem + L.u);         // M + 1 counters, then bucket starts
        int* b_base = b_cnt + 264;
        unsigned short* b_pos = (unsigned short*)(b_base + 264);
        unsigned int* b_tmp = (unsigned int*)(smem + L.u + 2 * 264 * 4 + upd_align16(2 * (size_t)a.Scap));
        for (int m = tid; m <= M; m += NT) b_cnt[m] = 0;
        __syncthreads();
        for (int s = tid; s < nsurv; s += NT)
            b_pos[s] = (unsigned short)atomicAdd(&b_cnt[s_skey[s] >> 16], 1);
        __syncthreads();
        {
            int run = 0;
            for (int base = 0; base < M; base += NT) {
                const int m = base + tid;
                int tot;
                const int pre = block_excl_scan<NT>(m < M ? b_cnt[m] : 0, s_scr, &tot);
                if (m < M) b_base[m] = run + pre;
                run += tot;
            }
        }
        __syncthreads();
        for (int s = tid; s < nsurv; s += NT) {
            const unsigned int key = s_skey[s];
            b_tmp[b_base[key >> 16] + b_pos[s]] = key;
        }
        __syncthreads();
        for (int s = tid; s < nsurv; s += NT) {
            const unsigned int key = s_skey[s];
            const int m = (int)(key >> 16), b0 = b_base[m], nb = b_cnt[m];
            int r = 0;
            for (int q = 0; q < nb; q++) r += b_tmp[b0 + q] < key;
            s_skey2[b0 + r] = key;
        }
        __syncthreads();
    }

    STAMP(4);
    /* Phase 4: merge candidates in update-array order
     * [non-detect | detect (m-major) | births | near-range]; prune w < minW.
     * Detection terms are re-evaluated exactly like the oracle (double g, expf). */
    int ncand = 0;
    int sbc = 0;           // barrier-light helper sequence of phases 4a-4c (sb_at)
    int sc_bad = 0;        // merge screen (cand_record), reduced once in the merge
    float sc_lmax = 0.f;
    // 4a non-detection terms
    for (int base = 0; base < (PHD_XK == 4 ? 0 : Gin); base += NT) {
        const int j = base + tid;
        float w = 0.f;
        bool keep = false;
        int k = 0;
        float v[NF];
        if (j < Gin) {
            k = s_in[j];
            // part C: the row prefetched at the start when the in-range list is
            // the identity there (all of the map in range), else loaded here
            if (PART == 2 && base == 0 && k == j && k < G) {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = pf[0][f];
            } else if (PART == 2 && base == NT && k == j && k < G) {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = pf[1][f];
            } else {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = prior(k)[f * a.cap];
            }
            // cphdUpdateKernel's exp(log w + lnd) as w e^lnd (D18)
            w = CPHD ? (v[0] > 0.f ? v[0] * ((const float*)(s_uni + 4))[1] : 0.f) : v[0] * (1 - c.pd);
            keep = !(w < c.minFeatureWeight);
        }
        int tot;
        const int r = block_rank<NT, false>(keep, sb_at<NT>(s_scr, sbc), &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                const float4 vc = make_float4(v[3], v[4], v[5], v[6]);
                X.K.P[p] = cand_record(v[1], v[2], w, vc, c.minSeparation, sc_bad, sc_lmax, (unsigned)k);
            }
        }
        ncand += tot;
    }
    STAMP(5);
    const int nd0 = min(ncand, a.Kcap);  // first detection / birth candidate (covariance slot 0)
    // 4b detection terms
    for (int base = 0; base < (PHD_XK == 4 ? 0 : nsurv); base += NT) {
        const int s = base + tid;
        bool keep = false;
        float w = 0.f, mx = 0.f, my = 0.f;
        DevEkf e;
        if (s < nsurv) {
            const unsigned int key = s_skey2[s];
            const int m = (int)(key >> 16);
            const int j = (int)(key & 0xffffu);
            const int k = s_in[j];
            const G1 float* sk = prior(k);
            mx = sk[1 * a.cap];
            my = sk[2 * a.cap];
            if constexpr (PART == 2) {  // range and bearing as part A computed them (H.rb)
                const G1 float* rbp = (const G1 float*)(hand + H.rb) + 2 * j;
                const float dx = mx - s_pose.px, dy = my - s_pose.py;
                d_ekf_from_geometry(c, dx, dy, dx * dx + dy * dy, rbp[0], rbp[1], sk[3 * a.cap], sk[4 * a.cap],
                                    sk[5 * a.cap], sk[6 * a.cap], e);
            } else {
                d_compute_ekf(c, s_pose.px, s_pose.py, s_pose.ptheta, mx, my, sk[3 * a.cap], sk[4 * a.cap],
                              sk[5 * a.cap], sk[6 * a.cap], e);
            }
            const float i0 = s_zr[m] - e.r;
            const float i1 = d_wrap(s_zb[m] - e.bearing);
            const float dist = i0 * i0 * e.S0 + i0 * i1 * (e.S1 + e.S2) + i1 * i1 * e.S3;
            const float g = (float)(-0.5 * (double)dist - c.log_2pi - 0.5 * (double)d_safe_log(e.det));
            const float lq = d_safe_log(e.pd) + d_safe_log(sk[0]) + g;
            w = expf(lq - s_leta[m]);
            keep = !(w < c.minFeatureWeight);
            mx = mx + e.K0 * i0 + e.K2 * i1;
            my = my + e.K1 * i0 + e.K3 * i1;
        }
        int tot;
        const int r = block_rank<NT, false>(keep, sb_at<NT>(s_scr, sbc), &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                const float4 v = make_float4(e.cu0, e.cu1, e.cu2, e.cu3);
                X.K.P[p] = cand_record(mx, my, w, v, c.minSeparation, sc_bad, sc_lmax, 0x8000u | (unsigned)(p - nd0));
                X.K.detv[p - nd0] = v;
            }
        }
        ncand += tot;
    }
    STAMP(6);
    // 4c births (none in the CPHD update array)
    for (int base = 0; base < (CPHD ? 0 : M); base += NT) {
        const int m = base + tid;
        bool keep = false;
        float w = 0.f;
        if (m < M) {
            const float lb = s_zok[m] ? c.log_birth : PHD_LOG0;
            w = expf(lb - s_leta[m]);
            keep = !(w < c.minFeatureWeight);
        }
        int tot;
        const int r = block_rank<NT, false>(keep, sb_at<NT>(s_scr, sbc), &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                float mean[2], cov[4];
                d_birth(c, s_pose.px, s_pose.py, s_pose.ptheta, s_zr[m], s_zb[m], mean, cov);
                const float4 v = make_float4(cov[0], cov[1], cov[2], cov[3]);
                X.K.P[p] = cand_record(mean[0], mean[1], w, v, c.minSeparation, sc_bad, sc_lmax,
                                       0x8000u | (unsigned)(p - nd0));
                X.K.detv[p - nd0] = v;
            }
        }
        ncand += tot;
    }
    // 4d near-range components join the merge unpruned (mergeAndCopyMaps :3227-3257)
    const int Gnear = s_cnt[1];
    for (int q = tid; q < Gnear; q += NT) {
        const int p = ncand + q;
        if (p < a.Kcap) {
            const int k = s_near[q];
            const G1 float* sk = prior(k);
            const float4 v = make_float4(sk[3 * a.cap], sk[4 * a.cap], sk[5 * a.cap], sk[6 * a.cap]);
            X.K.P[p] = cand_record(sk[1 * a.cap], sk[2 * a.cap], sk[0], v, c.minSeparation, sc_bad, sc_lmax,
                                   (unsigned)k);
        }
    }
    ncand += Gnear;
    if (ncand > a.Kcap) {
        flags |= PHD_ST_CANDIDATE_OVERFLOW;
        ncand = a.Kcap;
    }
    __syncthreads();

    STAMP(7);
    /* Phase 5: greedy merge — parallel exact form, serial fallback. */
    int nout = (PHD_XK == 3 || PHD_XK == 4) ? 0
               : a.merge_mode != 0         ? -1
                                           : merge_parallel<NT>(X, ncand, c.minSeparation, dst, a.cap, a.Epool,
                                                                a.Bbuckets, s_scr, s_redf, s_cnt + 3, sc_bad, sc_lmax, a);
    if (nout < 0) {
        __syncthreads();
        nout = merge_serial<NT>(X.K, nullptr, ncand, X.par, c.minSeparation, dst, a.cap, s_red, s_redf);
        flags |= PHD_ST_SERIAL_MERGE;
    }

    STAMP(8);
    flags |= s_cnt[14] & PHD_ST_PAIR_OVERFLOW;
    /* Phase 6: out-of-range components appended unchanged (mergeAndCopyMaps :3304-3323). */
    const int Gout = s_cnt[2];
    for (int q = tid; q < Gout; q += NT) {
        const int p = nout + q;
        if (p < a.cap) {
            const int k = s_out[q];
#pragma unroll
            for (int f = 0; f < NF; f++) st_out(dst + f * a.cap + p, prior(k)[f * a.cap]);
        }
    }
    int total = nout + Gout;
    if (total > a.cap) {
        flags |= PHD_ST_MAP_OVERFLOW;
        total = a.cap;
    }
    if (tid == 0) {
        a.size_out[n] = total;
        a.status[n] = flags;
        if (flags & ~PHD_ST_INFO) {
            atomicOr(a.err, flags & ~PHD_ST_INFO);
            atomicAdd(a.err + 3, 1);
        }
        if (flags & PHD_ST_SERIAL_MERGE) atomicAdd(a.err + 1, 1);
        if (a.src_reset) a.src_reset[n] = n;  // posterior of particle n now lives in out slab n
    }
    STAMP(9);
#ifdef PHD_STAMPS
    if (tid == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 49] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 10] = ((unsigned long long)ncand << 32) | (unsigned)nsurv;
    if (tid == 0 && a.stamps) {
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 40] = ((unsigned long long)s_cnt[8] << 32) | (unsigned)s_cnt[10];
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 41] = ((unsigned long long)s_cnt[9] << 32) | (unsigned)s_cnt[11];
        a.stamps[(size_t)blockIdx.x * PHD_STAMP_SLOTS + 42] = ((unsigned long long)Gin << 32) | (unsigned)s_cnt[12];
    }
#endif
}

/* The update kernels read their UpdateArgs through the kernel argument segment
 * pointer instead of the by-value parameter, so the compiler loads each field
 * where it is used (s_load, scalar cache) instead of keeping much of the struct
 * live in SGPRs across the kernel (spilled to VGPR lanes: v_writelane /
 * v_readlane, VALU instructions; 489 -> 230 reloads in part C's code). */
typedef const __attribute__((address_space(4))) UpdateArgs KArgs;  // the kernel argument segment
__device__ __forceinline__ const UpdateArgs& kargs(const UpdateArgs& a) {
    (void)a;
    unsigned long long v = (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(v));  // (the compiler cannot tie the loads to the parameter)
    return *(const UpdateArgs*)(KArgs*)v;
}

/* One kernel per workgroup size; the _p forms also run the particle's predict
 * (phd_step when every workgroup is resident at once: the predict's registers
 * then cost no occupancy that matters). */
__global__ void __launch_bounds__(256) k_update_fused_256(UpdateArgs a) { update_body<256, false>(kargs(a)); }
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(6, 8))) k_update_fused_512(UpdateArgs a) {
    update_body<512, false>(kargs(a));  // <= 80 VGPRs: three 512-thread workgroups per CU
}
__global__ void __launch_bounds__(1024) k_update_fused_1024(UpdateArgs a) { update_body<1024, false>(kargs(a)); }
__global__ void __launch_bounds__(256) k_update_fused_p256(UpdateArgs a) { update_body<256, true>(kargs(a)); }
// <= 168 VGPRs: the CPHD layout's LDS already holds a CU to 3 workgroups of 256
// (12 waves), so 128 would only add scratch spills
#define PHD_CPHD_WPE __attribute__((amdgpu_waves_per_eu(4, 8)))
__global__ void __launch_bounds__(512) k_update_fused_p512(UpdateArgs a) { update_body<512, true>(kargs(a)); }
/* three-launch CPHD update: part A (classify, pair table, walk -> handoff) and
 * part C (handoff + CPHD terms -> survivors, candidates, merge, out slab); the
 * CPHD terms in between are k_cphd_terms (phd_terms.hip). */
// part A: <= 80 VGPRs (6 waves per SIMD): its LDS (26.7 KB at config 3) fits 6 workgroups per CU
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_update_cphd_a_256(UpdateArgs a) {
    update_body<256, false, true, 1>(kargs(a));
}
__global__ void __launch_bounds__(512) k_update_cphd_a_512(UpdateArgs a) { update_body<512, false, true, 1>(kargs(a)); }
__global__ void __launch_bounds__(1024) k_update_cphd_a_1024(UpdateArgs a) { update_body<1024, false, true, 1>(kargs(a)); }
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_update_cphd_a_p256(UpdateArgs a) {
    update_body<256, true, true, 1>(kargs(a));
}
__global__ void __launch_bounds__(512) k_update_cphd_a_p512(UpdateArgs a) { update_body<512, true, true, 1>(kargs(a)); }
/* split PHD update (configs with large maps: one fused workgroup per CU at
 * config 5): part A (classify, pair table, walk -> handoff) and part C
 * (handoff -> normalisers, Δ log w, survivors, candidates with births,
 * merge), no CPHD terms in between */
__global__ void __launch_bounds__(256) k_update_phd_a_256(UpdateArgs a) { update_body<256, false, false, 1>(kargs(a)); }
__global__ void __launch_bounds__(512) k_update_phd_a_512(UpdateArgs a) { update_body<512, false, false, 1>(kargs(a)); }
__global__ void __launch_bounds__(1024) k_update_phd_a_1024(UpdateArgs a) { update_body<1024, false, false, 1>(kargs(a)); }
// <= 80 VGPRs (6 waves per SIMD): config 4's part C LDS (25.8 KB) fits 6 workgroups per CU
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_update_phd_c_256(UpdateArgs a) {
    update_body<256, false, false, 2>(kargs(a));
}
__global__ void __launch_bounds__(512) k_update_phd_c_512(UpdateArgs a) { update_body<512, false, false, 2>(kargs(a)); }
__global__ void __launch_bounds__(1024) k_update_phd_c_1024(UpdateArgs a) { update_body<1024, false, false, 2>(kargs(a)); }
// part C: <= 80 VGPRs (6 waves per SIMD) — its LDS layout (pair table, in / near
// lists, detection covariances, measurements and normalisers in the handoff /
// global memory; 24.0 KB at config 3 with the step's births: candidates 832)
// fits 6 workgroups per CU; at 72 VGPRs (7) the births' prior reads spilled
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_update_cphd_c_256(UpdateArgs a) {
    update_body<256, false, true, 2>(kargs(a));
}
__global__ void __launch_bounds__(512) PHD_CPHD_WPE k_update_cphd_c_512(UpdateArgs a) { update_body<512, false, true, 2>(kargs(a)); }
__global__ void __launch_bounds__(1024) k_update_cphd_c_1024(UpdateArgs a) { update_body<1024, false, true, 2>(kargs(a)); }

/* -------------------------------------------------------- normalise, nEff */

template <typename T>
__device__ __forceinline__ T block_reduce_1024(T v, T* s, bool is_max) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const T u = __shfl_xor(v, o, 64);
        v = is_max ? (u > v ? u : v) : v + u;
    }
    if (lane == 0) s[wid] = v;
    __syncthreads();
    T r = is_max ? (T)-INFINITY : (T)0;
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; w++) r = is_max ? (s[w] > r ? s[w] : r) : r + s[w];
    __syncthreads();
    return r;
}


/* logSumExp normalisation and nEff (standalone; the same block function as
 * k_normalize_resample, so both paths produce identical weights). */
__device__ int normalize_block(float* __restrict__ logw, int n, const float* lse_override, float* __restrict__ out,
                               float resample_thresh, int has_meas, double* s_d, float* s_f);

__global__ void __launch_bounds__(1024) k_normalize(float* __restrict__ logw, int n, const float* lse_override,
                                                    float* __restrict__ out /* [0]=lse [1]=neff [2]=resample? */,
                                                    float resample_thresh, int has_meas) {
    __shared__ double s_d[32];
    __shared__ float s_f[32];
    normalize_block(logw, n, lse_override, out, resample_thresh, has_meas, s_d, s_f);
}

/* Local log-sum-exp only (for the multi-GPU global LSE). out[0]=max, out[1]=Σexp(w-max). */
__global__ void __launch_bounds__(1024) k_lse_parts(const float* __restrict__ logw, int n, float* __restrict__ out) {
    __shared__ float sf[32];
    __shared__ double sd[32];
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, logw[i]);
    mx = block_reduce_1024<float>(mx, sf, true);
    double sum = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) sum += (double)expf(logw[i] - mx);
    sum = block_reduce_1024<double>(sum, sd, false);
    if (threadIdx.x == 0) {
        out[0] = mx;
        out[1] = (float)sum;
    }
}


/* --------------------------------------------------------------- resample */

/* 64-bit DPP helpers for the single-block resample (1024 threads). */
template <int CTRL, int ROWMASK>
__device__ __forceinline__ unsigned long long dpp_or_zero_u64(unsigned long long v) {
    const unsigned int lo = (unsigned int)v, hi = (unsigned int)(v >> 32);
    const unsigned int lo2 = (unsigned int)dpp_or_zero<CTRL, ROWMASK>((int)lo);
    const unsigned int hi2 = (unsigned int)dpp_or_zero<CTRL, ROWMASK>((int)hi);
    return ((unsigned long long)hi2 << 32) | lo2;
}

__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long x) {
    x += dpp_or_zero_u64<0x111, 0xf>(x);
    x += dpp_or_zero_u64<0x112, 0xf>(x);
    x += dpp_or_zero_u64<0x114, 0xf>(x);
    x += dpp_or_zero_u64<0x118, 0xf>(x);
    x += dpp_or_zero_u64<0x142, 0xa>(x);
    x += dpp_or_zero_u64<0x143, 0xc>(x);
    return x;
}

__device__ __forceinline__ unsigned long long wave_incl_max_u64(unsigned long long x) {
    unsigned long long y;
    y = dpp_or_zero_u64<0x111, 0xf>(x); x = y > x ? y : x;
    y = dpp_or_zero_u64<0x112, 0xf>(x); x = y > x ? y : x;
    y = dpp_or_zero_u64<0x114, 0xf>(x); x = y > x ? y : x;
    y = dpp_or_zero_u64<0x118, 0xf>(x); x = y > x ? y : x;
    y = dpp_or_zero_u64<0x142, 0xa>(x); x = y > x ? y : x;
    y = dpp_or_zero_u64<0x143, 0xc>(x); x = y > x ? y : x;
    return x;
}

/* Stratified resample (main.cpp:453-501) by one 1024-thread block: fixed-point
 * CDF of det_expf terms (phd_detmath.h) in LDS (global `cdf_g` when n exceeds
 * RS_LDS_MAX), chunked scan, per-stratum binary search, and the
 * copy_particles remap (slamtypes.h:313-333) as an index remap: children take
 * the parent's pose and slab reference; maps are never copied.  The general
 * form (any n; the CDF in global memory past RS_LDS_MAX); callers with
 * n <= RS_LDS_MAX use norm_resample_regs.  logw_in must be visible to the
 * whole block (normalize_block's writes precede a barrier). */
__device__ void resample_block(const float* __restrict__ logw_in, int n, int n_out, const double* __restrict__ u_in,
                               uint64_t seed, uint64_t step, unsigned long long* __restrict__ cdf_g,
                               unsigned long long* __restrict__ s_cdf, unsigned long long* s_w64, int* __restrict__ idx,
                               phd_pose* __restrict__ pose, int* __restrict__ src, phd_pose* __restrict__ tmp_pose,
                               int* __restrict__ tmp_src, float* __restrict__ logw_out, float new_logw) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    unsigned long long* cdf = s_cdf ? s_cdf : cdf_g;
    // terms and arg-max (first maximum: key = term bits << 32 | ~index)
    unsigned long long best = 0ull;
    for (int i = t; i < n; i += RS_THREADS) {
        const float tv = phd_det_expf(logw_in[i]);
        cdf[i] = (unsigned long long)phd_fix_term(tv);
        const unsigned long long key = ((unsigned long long)__float_as_uint(tv) << 32) | (0xffffffffu - (unsigned)i);
        best = key > best ? key : best;
    }
    best = wave_incl_max_u64(best);
    if (lane == 63) s_w64[32 + wid] = best;
    if (!s_cdf) __threadfence_block();
    __syncthreads();
    // chunked inclusive scan: thread t owns [t*per, (t+1)*per)
    const int per = (n + RS_THREADS - 1) / RS_THREADS;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    unsigned long long acc = 0;
    for (int i = lo; i < hi; i++) {
        acc += s_cdf ? cdf[i] : __hip_atomic_load(cdf + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cdf[i] = acc;
    }
    const unsigned long long wsc = wave_incl_scan_u64(acc);
    if (lane == 63) s_w64[wid] = wsc;
    __syncthreads();
    unsigned long long off = wsc - acc;
    unsigned long long amaxk = 0ull;
#pragma unroll
    for (int w = 0; w < RS_THREADS / 64; w++) {
        off += (w < wid) ? s_w64[w] : 0ull;
        const unsigned long long k = s_w64[32 + w];
        amaxk = k > amaxk ? k : amaxk;
    }
    for (int i = lo; i < hi; i++) cdf[i] += off;
    const int amax = (int)(0xffffffffu - (unsigned)(amaxk & 0xffffffffull));
    if (!s_cdf) __threadfence_block();
    __syncthreads();
    // a global CDF was written by other waves of this block: read it past the L1
    auto cdf_at = [&](int i) -> unsigned long long {
        return s_cdf ? cdf[i] : __hip_atomic_load(cdf + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // Thread t takes the contiguous strata [t*per_o, (t+1)*per_o): one binary
    // search for the first, then a galloping search forward from the previous
    // parent (strata and the CDF both increase, so parents do) — the same lower
    // bound as a search per stratum, without per-stratum chains of dependent
    // reads.  n_out strata over the n entries (n_out < n after a predict that
    // spawned n_predict_particles children, main.cpp:1289).
    const int per_o = (n_out + RS_THREADS - 1) / RS_THREADS;
    const int lo_o = min(n_out, t * per_o), hi_o = min(n_out, lo_o + per_o);
    int pos = 0;
    for (int j = lo_o; j < hi_o; j++) {
        double u;
        if (u_in) {
            u = u_in[j];
        } else {
            const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
            u = phd_u01(x.v[0]);
        }
        const unsigned long long r = phd_fix_stratum(j, u, n_out);
        int a0 = pos, b0 = n;  // invariant: cdf[a0 - 1] < r (or a0 == 0), answer in [a0, b0]
        if (j > lo_o) {
            int step_g = 1;
            while (a0 + step_g - 1 < n && cdf_at(a0 + step_g - 1) < r) {
                a0 += step_g;
                step_g <<= 1;
            }
            b0 = min(n, a0 + step_g - 1);
        }
        while (a0 < b0) {
            const int mid = (a0 + b0) >> 1;
            if (cdf_at(mid) >= r)
                b0 = mid;
            else
                a0 = mid + 1;
        }
        pos = a0;
        const int p = (a0 < n) ? a0 : amax;
        idx[j] = p;
        if (pose) {
            tmp_pose[j] = pose[p];
            tmp_src[j] = src ? src[p] : p;
        }
    }
    if (pose) {
        __threadfence_block();
        __syncthreads();
        for (int j = t; j < n_out; j += RS_THREADS) {
            pose[j] = tmp_pose[j];
            if (src) src[j] = tmp_src[j];
            logw_out[j] = new_logw;
        }
    }
}

/* Standalone resample.  If `flag` is non-NULL and *flag == 0 the kernel does
 * nothing (device-side decision).  Dynamic LDS: 8*n bytes when n <= RS_LDS_MAX. */
__global__ void __launch_bounds__(RS_THREADS)
    k_resample(const int* __restrict__ flag, const float* __restrict__ logw_in, float* __restrict__ logw_out, int n,
               int n_out, const double* __restrict__ u_in, uint64_t seed, uint64_t step, unsigned long long* __restrict__ cdf,
               int* __restrict__ idx, phd_pose* __restrict__ pose, int* __restrict__ src, phd_pose* __restrict__ tmp_pose,
               int* __restrict__ tmp_src, float new_logw) {
    if (flag && *flag == 0) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_smem[];
    __shared__ unsigned long long s_w64[64];
    unsigned long long* s_cdf = n <= RS_LDS_MAX ? (unsigned long long*)rs_smem : nullptr;
    resample_block(logw_in, n, n_out, u_in, seed, step, cdf, s_cdf, s_w64, idx, pose, src, tmp_pose, tmp_src,
                   logw_out, new_logw);
}

/* The canonical order of the double sums of the normalisation (oracle D3: the
 * intended exact sum, up to one fixed reduction tree shared by every path).
 * The entries are cut into chunks of RS_THREADS; chunk c holds entries
 * c*1024 + t.  A chunk's sum is the wave_incl_scan_d total of each of its 16
 * waves, added in wave order; the chunk sums are added in chunk order.  The
 * single-block kernels (one thread per entry of every chunk) and the
 * multi-block sharded plan (one workgroup per chunk, k_rs_*) all evaluate
 * exactly this, so their weights agree bit for bit. */
template <class F>
__device__ double chunk_sum_block(int n, F&& f, double* s /* 32 doubles */) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    double total = 0.0;
    for (int c = 0; c * RS_THREADS < n; c++) {
        const int i = c * RS_THREADS + t;
        double x = i < n ? f(i) : 0.0;
        x = wave_incl_scan_d(x);
        double* sb = s + (c & 1) * 16;  // double-buffered: one barrier per chunk
        if (lane == 63) sb[wid] = x;
        __syncthreads();
        double cs = 0.0;
#pragma unroll
        for (int w = 0; w < RS_THREADS / 64; w++) cs += sb[w];
        total += cs;
    }
    return total;
}

/* logSumExp normalisation (phdfilter.cu:3748-3755), nEff (main.cpp:1281-1284)
 * and the resample decision (main.cpp:1286-1289) by one 1024-thread block;
 * thread t owns entries t, t+1024, ...; sums in the canonical chunk order.
 * The writes of the normalised entries precede a barrier.  s_d: 64 doubles.
 * Returns the decision. */
__device__ int normalize_block(float* __restrict__ logw, int n, const float* lse_override, float* __restrict__ out,
                               float resample_thresh, int has_meas, double* s_d, float* s_f) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    float mx = -INFINITY;
    for (int i = t; i < n; i += RS_THREADS) mx = fmaxf(mx, logw[i]);
    mx = wave_incl_max(mx);
    if (lane == 63) s_f[wid] = mx;
    __syncthreads();
    mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < RS_THREADS / 64; w++) mx = fmaxf(mx, s_f[w]);
    float lse;
    if (lse_override) {
        lse = *lse_override;
    } else {
        const double sum = chunk_sum_block(n, [&](int i) { return (double)expf(logw[i] - mx); }, s_d);
        lse = d_safe_log((float)sum) + mx;
    }
    const double s2 = chunk_sum_block(
        n,
        [&](int i) {
            const float w = logw[i] - lse;
            logw[i] = w;
            return (double)expf(2 * w);
        },
        s_d + 32);
    const float neff = (float)(1.0 / (double)(float)s2 / (double)n);
    const int resample = (has_meas == 2 || (has_meas && neff <= resample_thresh)) ? 1 : 0;  // 2: forced (n > 5N)
    if (t == 0) {
        out[0] = lse;
        out[1] = neff;
        ((int*)out)[2] = resample;
        if (resample) atomicAdd((unsigned*)out + 4, 1u);  // decisions counter (phd_resample_count); result unused
    }
    return resample;
}

/* Register-resident form of normalize_block + resample_block for
 * n <= 1024*PER: thread t holds entries t + 1024 k (k < PER) in registers from
 * one coalesced read through the log-sum-exp, nEff (canonical chunk order,
 * chunk_sum_block), the fixed-point terms and the chunked block scan; the CDF
 * is written to LDS once.  Strata are then taken in contiguous runs
 * [t*PER, t*PER + PER) with a galloping search from the previous parent.  Same
 * arithmetic as the two block functions (phdfilter.cu:3748-3755,
 * main.cpp:1281-1297, 453-501).  `local` (optional) receives the normalised
 * entries [local_lo, local_lo + local_n) when there is no resample.  Returns
 * the decision; when it is 1, idx[j] (LDS or global) holds the parent of every
 * stratum and the block has synced.  s_w64: 16*PER + 16; s_d: 32*PER. */
template <int PER>
__device__ int norm_resample_regs(float* __restrict__ logw, int n, float* __restrict__ out, float resample_thresh,
                                  int has_meas, uint64_t seed, uint64_t step, unsigned long long* __restrict__ s_cdf,
                                  int* __restrict__ idx, float* __restrict__ local, int local_lo, int local_n,
                                  unsigned long long* s_w64, double* s_d, float* s_f) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    constexpr int W = RS_THREADS / 64;
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) v[k] = k * RS_THREADS + t < n ? logw[k * RS_THREADS + t] : -INFINITY;
    float mx = v[0];
#pragma unroll
    for (int k = 1; k < PER; k++) mx = fmaxf(mx, v[k]);
    mx = wave_incl_max(mx);
    if (lane == 63) s_f[wid] = mx;
    __syncthreads();
    mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; w++) mx = fmaxf(mx, s_f[w]);
    // chunk sums: wave totals of every chunk at once, then chunk by chunk in order
    auto chunk_total = [&](double (&x)[PER], double* sb) {
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const double y = wave_incl_scan_d(x[k]);
            if (lane == 63) sb[k * W + wid] = y;
        }
        __syncthreads();
        double total = 0.0;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            if (k * RS_THREADS >= n) break;
            double cs = 0.0;
#pragma unroll
            for (int w = 0; w < W; w++) cs += sb[k * W + w];
            total += cs;
        }
        return total;
    };
    double x[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) x[k] = k * RS_THREADS + t < n ? (double)expf(v[k] - mx) : 0.0;
    const float lse = d_safe_log((float)chunk_total(x, s_d)) + mx;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = k * RS_THREADS + t;
        x[k] = 0.0;
        if (i < n) {
            const float w = v[k] - lse;
            v[k] = w;
            logw[i] = w;
            x[k] = (double)expf(2 * w);
        }
    }
    const double s2 = chunk_total(x, s_d + 16 * PER);
    const float neff = (float)(1.0 / (double)(float)s2 / (double)n);
    const int resample = (has_meas == 2 || (has_meas && neff <= resample_thresh)) ? 1 : 0;  // 2: forced (n > 5N)
    if (t == 0) {
        out[0] = lse;
        out[1] = neff;
        ((int*)out)[2] = resample;
        if (resample) atomicAdd((unsigned*)out + 4, 1u);  // decisions counter (phd_resample_count); result unused
    }
    if (!resample) {  // (with a resample the caller writes the new log-weight instead)
        if (local) {
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int i = k * RS_THREADS + t;
                if (i < n && i >= local_lo && i < local_lo + local_n) local[i - local_lo] = v[k];
            }
        }
        return 0;
    }
    // fixed-point terms, first arg-max key, chunked block scan
    unsigned long long c[PER];
    unsigned long long best = 0ull;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int i = k * RS_THREADS + t;
        unsigned long long term = 0ull;
        if (i < n) {
            const float tv = phd_det_expf(v[k]);
            term = (unsigned long long)phd_fix_term(tv);
            const unsigned long long key = ((unsigned long long)__float_as_uint(tv) << 32) | (0xffffffffu - (unsigned)i);
            best = key > best ? key : best;
        }
        c[k] = wave_incl_scan_u64(term);  // inclusive within the wave
        if (lane == 63) s_w64[k * W + wid] = c[k];
    }
    best = wave_incl_max_u64(best);
    if (lane == 63) s_w64[PER * W + wid] = best;
    __syncthreads();
    unsigned long long amaxk = 0ull;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const unsigned long long kk = s_w64[PER * W + w];
        amaxk = kk > amaxk ? kk : amaxk;
    }
    const int amax = (int)(0xffffffffu - (unsigned)(amaxk & 0xffffffffull));
    unsigned long long run = 0ull;  // CDF before chunk k
#pragma unroll
    for (int k = 0; k < PER; k++) {
        unsigned long long off = run, ctot = 0ull;
#pragma unroll
        for (int w = 0; w < W; w++) {
            const unsigned long long sw = s_w64[k * W + w];
            off += (w < wid) ? sw : 0ull;
            ctot += sw;
        }
        const int i = k * RS_THREADS + t;
        if (i < n) s_cdf[i] = c[k] + off;
        run += ctot;
    }
    __syncthreads();
    // strata [t*PER, t*PER + PER): lower bound of r_j in the CDF, galloping
    // forward from the previous parent (strata and the CDF both increase)
    const int base = t * PER;
    int pos = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int j = base + k;
        if (j >= n) break;
        const phd_u32x4 xr = phd_rng_draw(seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
        const unsigned long long r = phd_fix_stratum(j, phd_u01(xr.v[0]), n);
        int a0 = pos, b0 = n;  // invariant: cdf[a0 - 1] < r (or a0 == 0), answer in [a0, b0]
        if (k > 0) {
            int step_g = 1;
            while (a0 + step_g - 1 < n && s_cdf[a0 + step_g - 1] < r) {
                a0 += step_g;
                step_g <<= 1;
            }
            b0 = min(n, a0 + step_g - 1);
        }
        while (a0 < b0) {
            const int mid = (a0 + b0) >> 1;
            if (s_cdf[mid] >= r)
                b0 = mid;
            else
                a0 = mid + 1;
        }
        pos = a0;
        idx[j] = (a0 < n) ? a0 : amax;
    }
    __syncthreads();
    return 1;
}

/* normalise + nEff + decision + (conditional) resample in one launch (phd_step):
 * phdfilter.cu:3748-3755, main.cpp:1281-1297. */
template <int PER>
__device__ void normalize_resample_regs_body(float* __restrict__ logw, int n, float* __restrict__ out,
                                             float resample_thresh, int has_meas, uint64_t seed, uint64_t step,
                                             int* __restrict__ idx, phd_pose* __restrict__ pose, int* __restrict__ src,
                                             phd_pose* __restrict__ tmp_pose, int* __restrict__ tmp_src, float new_logw,
                                             unsigned char* smem, unsigned long long* s_w64, double* s_d, float* s_f) {
    unsigned long long* s_cdf = (unsigned long long*)smem;
    if (!norm_resample_regs<PER>(logw, n, out, resample_thresh, has_meas, seed, step, s_cdf, idx, nullptr, 0, 0, s_w64,
                                 s_d, s_f))
        return;
    // copy_particles as an index remap; the strata of thread t are its own
    // entries, so only the parent reads cross threads (barrier before the writes)
    const int base = threadIdx.x * PER;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int j = base + k;
        if (j < n) {
            const int p = idx[j];
            tmp_pose[j] = pose[p];
            tmp_src[j] = src ? src[p] : p;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int j = base + k;
        if (j < n) {
            pose[j] = tmp_pose[j];
            if (src) src[j] = tmp_src[j];
            logw[j] = new_logw;
        }
    }
}

__global__ void __launch_bounds__(RS_THREADS)
    k_normalize_resample(float* __restrict__ logw, int n, float* __restrict__ out, float resample_thresh,
                         int has_meas, uint64_t seed, uint64_t step, unsigned long long* __restrict__ cdf,
                         int* __restrict__ idx, phd_pose* __restrict__ pose, int* __restrict__ src,
                         phd_pose* __restrict__ tmp_pose, int* __restrict__ tmp_src, float new_logw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_smem[];
    __shared__ unsigned long long s_w64[16 * 8 + 16];
    __shared__ double s_d[32 * 8];
    __shared__ float s_f[32];
    // register-resident form when the CDF fits the dynamic LDS (host: rs_lds)
    if (n <= RS_THREADS * 8 && n <= RS_LDS_MAX) {
#define NR_CASE(P)                                                                                                  \
    normalize_resample_regs_body<P>(logw, n, out, resample_thresh, has_meas, seed, step, idx, pose, src, tmp_pose, \
                                    tmp_src, new_logw, rs_smem, s_w64, s_d, s_f)
        if (n <= RS_THREADS) NR_CASE(1);
        else if (n <= 2 * RS_THREADS) NR_CASE(2);
        else if (n <= 4 * RS_THREADS) NR_CASE(4);
        else NR_CASE(8);
#undef NR_CASE
        return;
    }
    const int resample = normalize_block(logw, n, nullptr, out, resample_thresh, has_meas, s_d, s_f);
    if (!resample) return;
    unsigned long long* s_cdf = n <= RS_LDS_MAX ? (unsigned long long*)rs_smem : nullptr;
    resample_block(logw, n, n, nullptr, seed, step, cdf, s_cdf, s_w64, idx, pose, src, tmp_pose, tmp_src, logw,
                   new_logw);
}

/* Apply a caller-computed parent list (local parents): same remap as k_resample.
 * With `flag` (device-side decision) it does nothing when *flag == 0. */
__global__ void __launch_bounds__(1024)
    k_apply_parents(const int* __restrict__ flag, const int* __restrict__ idx, int n, phd_pose* __restrict__ pose,
                    int* __restrict__ src, float* __restrict__ logw, phd_pose* __restrict__ tmp_pose,
                    int* __restrict__ tmp_src, float new_logw) {
    if (flag && *flag == 0) return;
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const int p = idx[j];
        tmp_pose[j] = pose[p];
        tmp_src[j] = src[p];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        pose[j] = tmp_pose[j];
        src[j] = tmp_src[j];
        logw[j] = new_logw;
    }
}

/* r with a[r] <= e < a[r+1] over the nondecreasing prefix array a[0..m] */
__device__ __forceinline__ int range_of(const int* a, int m, int e) {
    int lo = 0, hi = m + 1;  // upper_bound(a, e) - 1
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] <= e) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;
}

/* exclusive count of set flags before this thread and the block total (1024 threads) */
__device__ __forceinline__ int block_flag_scan(int flag, int* s_wc, int& total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const unsigned long long m = __ballot(flag);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wc[w] = __popcll(m);
    __syncthreads();
    int off = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int c = s_wc[k];
        off += k < w ? c : 0;
        total += c;
    }
    __syncthreads();
    return off + before;
}

/* Words another workgroup of the same launch wrote (the one-launch plan's
 * hand-offs): vector loads at agent scope, past this CU's L1 and never through
 * the scalar cache, whatever the compiler proves about the address. */
__device__ __forceinline__ int ld_par(const int* a, int i) {
    return __hip_atomic_load(a + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_u64(const unsigned long long* a, int i) {
    return __hip_atomic_load(a + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_f64(const double* a, int i) {
    return __longlong_as_double((long long)ld_u64((const unsigned long long*)a, i));
}
__device__ __forceinline__ float ld_f32(const float* a, int i) {
    return __int_as_float(ld_par((const int*)a, i));
}
/* Stores of words handed to other workgroups of the same launch (WT: the
 * one-launch kernels): write-through agent-scope stores, so the hand-off needs
 * no release fence (its arrive drains them, plan_arrive); plain stores else. */
template <bool WT>
__device__ __forceinline__ void st_u32(void* p, unsigned v) {
    if constexpr (WT) __hip_atomic_store((unsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(unsigned*)p = v;
}
template <bool WT>
__device__ __forceinline__ void st_u64(void* p, unsigned long long v) {
    if constexpr (WT) __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(unsigned long long*)p = v;
}

/* The parent list as the plan reads it.  Strata past the CDF's end (weights
 * summing to a little under one) take the first maximum, as the reference's
 * resampler does (main.cpp:470-488), so the otherwise nondecreasing list can
 * drop at its end: a suffix of k strata, all with parent pm.  The plan needs
 * the list grouped by owning rank in stratum order (dist.py plan_migration),
 * so the view moves that suffix to the end of pm's rank (position ins of the
 * prefix).  k = 0: the list itself. */
struct ParentView {
    const int* p;
    int k, ins, pm;
    __device__ int at(int i) const {
        if (k == 0 || i < ins) return ld_par(p, i);
        if (i < ins + k) return pm;
        return ld_par(p, i - k);
    }
};

/* the view of the N-entry list whose last `beyond` strata fell past the end
 * (block-uniform; s_tmp: one LDS int) */
__device__ __forceinline__ ParentView parent_view(const int* parents, int N, int n, int beyond, int* s_tmp) {
    ParentView v{parents, 0, 0, 0};
    if (beyond <= 0 || beyond >= N) return v;  // none, or every stratum: still sorted
    const int jstar = N - beyond;
    const int pm = ld_par(parents, N - 1);
    if (threadIdx.x == 0) {  // first prefix stratum owned past pm's rank (rare path: one thread)
        const int key = (pm / n + 1) * n;
        int a0 = 0, b0 = jstar;
        while (a0 < b0) {
            const int mid = (a0 + b0) >> 1;
            if (ld_par(parents, mid) < key) a0 = mid + 1;
            else b0 = mid;
        }
        s_tmp[0] = a0;
    }
    __syncthreads();
    const int ins = s_tmp[0];
    if (ins < jstar) {  // else the suffix already sits at the end of its rank
        v.k = beyond;
        v.ins = ins;
        v.pm = pm;
    }
    return v;
}

/* Migration plan of a sharded resample (phdslam/dist.py plan_migration, on the
 * device, with duplicate records folded).  `parents` is the global parent list
 * (identical on every rank), read through its rank-grouped view; rank s owns
 * global ids [s*n, (s+1)*n), so its children are the contiguous run of the view
 * in that range and demand[s] is its length.  The first min(demand, n)
 * children of a rank stay (keep_src: local parents); its remaining children, in
 * stratum order, form its part of the job-wide surplus sequence, which fills
 * the deficit slots of the ranks short of n children, in rank order.  Children
 * of one parent are identical until the next predict, so a sender ships one
 * record per distinct (parent, destination) and the receiver points every slot
 * of that parent at the one migration slab.  Every rank derives the same
 * sequence, so the sender packs, and the receiver maps slots to records,
 * without talking to each other.
 * Outputs: mig = [demand (world) | send records per destination (world) |
 * receive records per source (world) | records sent], send_src (local parent of
 * each record sent, destinations ascending), recv_rec (record index of each
 * receiving slot demand[rank] + i).  Without a resample (flag 0): demand n,
 * identity keep, nothing moves. */
#define MIG_MAX_WORLD 1024
#define MIG_SAMPLES 2048 /* rank boundaries: a sample of the view staged in LDS */

struct MigLds {
    int lo[MIG_MAX_WORLD + 1], s0[MIG_MAX_WORLD + 1], f0[MIG_MAX_WORLD + 1];
    int send[MIG_MAX_WORLD], recv[MIG_MAX_WORLD];
    int samp[MIG_SAMPLES];
    int wc[16];
};

/* The remap the keep pass writes next to keep_src: slot q takes local parent
 * k's pose and slab reference and a log-weight (keep_load(q, k) reads them,
 * keep_store(q, rec) writes them). */
struct KeepRec {
    phd_pose p;
    int s;
    float w;
};

/* The plan of one rank by one 1024-thread block (see above).  keep_src[q] and
 * the remap of slot q: two slots per thread per pass, each pass's parent
 * loads and then its gathers issued together (two round trips per pass). */
template <class FL, class FS>
__device__ __forceinline__ void migration_plan_block(int resampled, const ParentView& par, int n, int world,
                                                     int rank, int* __restrict__ mig, int* __restrict__ keep_src,
                                                     int* __restrict__ send_src, int* __restrict__ recv_rec, MigLds& L,
                                                     FL&& keep_load, FS&& keep_store,
                                     unsigned long long* st = nullptr) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int N = n * world;
    (void)st;
    // slots q < d keep local parent par[lo + q] - rank n (identity: q), the
    // rest (deficit slots) the placeholder 0
    auto keep_pass = [&](bool identity, int lo, int d) {
        const int bd = (int)blockDim.x, base_rank = rank * n;
        auto parent_of = [&](int q) { return identity ? q : (q < n && q < d) ? par.at(lo + q) - base_rank : 0; };
        for (int q0 = t; q0 < n; q0 += 2 * bd) {
            const int q1 = q0 + bd;
            const bool v1 = q1 < n;
            const int k0 = parent_of(q0), k1 = v1 ? parent_of(q1) : 0;
            const KeepRec r0 = keep_load(q0, k0);
            KeepRec r1{};
            if (v1) r1 = keep_load(q1, k1);
            keep_src[q0] = k0;
            keep_store(q0, r0);
            if (v1) {
                keep_src[q1] = k1;
                keep_store(q1, r1);
            }
        }
    };
    if (!resampled) {
        for (int s = t; s < world; s += blockDim.x) {
            mig[s] = n;
            mig[world + s] = 0;
            mig[2 * world + s] = 0;
        }
        keep_pass(true, 0, n);
        if (t == 0) mig[3 * world] = 0;
        return;
    }
    // rank boundaries lo[s] = first view position owned by rank >= s: a
    // search of every S-th entry (staged in LDS, one load round) narrows s to
    // S entries, which one wave tests 64 at a time (a ballot), instead of a
    // chain of dependent global loads per rank
    int S = 64;
    while ((N + S - 1) / S > MIG_SAMPLES) S += 64;
    const int ns = (N + S - 1) / S;
    for (int i = t; i < ns; i += blockDim.x) L.samp[i] = par.at(i * S);
    __syncthreads();
    for (int s = wid; s <= world; s += (int)(blockDim.x >> 6)) {
        int lb = 0;
        if (s == world) {
            lb = N;
        } else if (s > 0) {
            const int key = s * n;
            int a0 = 0, b0 = ns;  // first sample at or past key
            while (a0 < b0) {
                const int mid = (a0 + b0) >> 1;
                if (L.samp[mid] >= key) b0 = mid;
                else a0 = mid + 1;
            }
            const int lo_i = a0 == 0 ? 0 : (a0 - 1) * S + 1;
            const int hi_i = a0 == ns ? N : a0 * S;
            lb = hi_i;
            for (int base = lo_i; base < hi_i; base += 64) {
                const int idx = base + lane;
                const unsigned long long m = __ballot(idx < hi_i && par.at(idx) >= key);
                if (m) {
                    lb = base + __ffsll((long long)m) - 1;
                    break;
                }
            }
        }
        if (lane == 0) {
            L.lo[s] = lb;
            if (s < world) L.send[s] = L.recv[s] = 0;
        }
    }
    __syncthreads();
    if (t == 0) {
        L.s0[0] = L.f0[0] = 0;
        for (int s = 0; s < world; s++) {
            const int d = L.lo[s + 1] - L.lo[s];
            L.s0[s + 1] = L.s0[s] + (d > n ? d - n : 0);
            L.f0[s + 1] = L.f0[s] + (d < n ? n - d : 0);
        }
    }
    for (int s = t; s < world; s += blockDim.x) mig[s] = L.lo[s + 1] - L.lo[s];
    __syncthreads();
    PSTAMP(st, 2);
    const int lo = L.lo[rank];
    const int d = L.lo[rank + 1] - lo;
    const int base_rank = rank * n;
    keep_pass(false, lo, d);
    PSTAMP(st, 3);

    // sender: my children q in [n, d) are surplus elements e = s0[rank] + q - n
    int sent = 0;
    for (int b = n; b < d; b += blockDim.x) {
        const int q = b + t;
        int fresh = 0, dst = 0, pp = 0;
        if (q < d) {
            const int e = L.s0[rank] + q - n;
            pp = par.at(lo + q);
            dst = range_of(L.f0, world, e);
            fresh = q == n || pp != par.at(lo + q - 1) || dst != range_of(L.f0, world, e - 1);
        }
        int total;
        const int pos = block_flag_scan(fresh, L.wc, total);
        if (fresh) {
            send_src[sent + pos] = pp - base_rank;
            atomicAdd(&L.send[dst], 1);
        }
        sent += total;
    }
    // receiver: my deficit slots d + i, i in [0, n - d), take surplus elements e = f0[rank] + i
    int recs = 0;
    for (int b = 0; b < n - d; b += blockDim.x) {
        const int i = b + t;
        int fresh = 0, src = 0;
        if (i < n - d) {
            const int e = L.f0[rank] + i;
            src = range_of(L.s0, world, e);
            const int pp = par.at(L.lo[src] + n + (e - L.s0[src]));
            if (i == 0) {
                fresh = 1;
            } else {
                const int sp = range_of(L.s0, world, e - 1);
                fresh = sp != src || pp != par.at(L.lo[sp] + n + (e - 1 - L.s0[sp]));
            }
        }
        int total;
        const int pos = block_flag_scan(fresh, L.wc, total);
        if (i < n - d) {
            recv_rec[i] = recs + pos + fresh - 1;
            if (fresh) atomicAdd(&L.recv[src], 1);
        }
        recs += total;
    }
    __syncthreads();
    PSTAMP(st, 4);
    for (int s = t; s < world; s += blockDim.x) {
        mig[world + s] = L.send[s];
        mig[2 * world + s] = L.recv[s];
    }
    if (t == 0) mig[3 * world] = sent;
}

/* ---- sharded plan (phd_shard_resample[_async]): every rank runs it on the
 * identical gathered log-weights.  The global part — logSumExp normalisation,
 * nEff and decision (phdfilter.cu:3748-3755, main.cpp:1281-1289) and the
 * stratified resample into the global parent list (main.cpp:453-501) — runs
 * one workgroup per chunk of RS_THREADS entries, so the N = world*n entries
 * are spread over N/1024 CUs instead of one; the double sums follow the
 * canonical chunk order (chunk_sum_block), so the weights equal the
 * single-block paths' bit for bit.  Then one block derives this rank's
 * migration plan and the local remap (shard_tail_block).  k_shard_plan does
 * all of it in ONE launch (two in-launch waits and a last-arriver ticket in
 * place of four kernel boundaries); the k_rs_* kernels are the multi-launch
 * form phd_step uses above 16 chunks and the plan uses when its grid cannot
 * be resident at once. */

/* block-wide max of the B chunk maxima (every thread gets it) */
__device__ float rs_global_max(const float* __restrict__ part_max, int B, float* s_f,
                              const float* __restrict__ w_all = nullptr, int N = 0) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    float m = -INFINITY;
    if (w_all) {  // every block takes the max of all N entries itself (no k_rs_max launch)
        // 16-byte loads, four in flight per thread (the max is order-free: the
        // same value whatever the grouping)
        const float4* w4 = (const float4*)w_all;
        const int N4 = ((uintptr_t)w_all & 15u) ? 0 : N >> 2;
        float m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
        int i = t;
        for (; i + 3 * RS_THREADS < N4; i += 4 * RS_THREADS) {
            const float4 a0 = w4[i], a1 = w4[i + RS_THREADS], a2 = w4[i + 2 * RS_THREADS], a3 = w4[i + 3 * RS_THREADS];
            m = fmaxf(m, fmaxf(fmaxf(a0.x, a0.y), fmaxf(a0.z, a0.w)));
            m1 = fmaxf(m1, fmaxf(fmaxf(a1.x, a1.y), fmaxf(a1.z, a1.w)));
            m2 = fmaxf(m2, fmaxf(fmaxf(a2.x, a2.y), fmaxf(a2.z, a2.w)));
            m3 = fmaxf(m3, fmaxf(fmaxf(a3.x, a3.y), fmaxf(a3.z, a3.w)));
        }
        for (; i < N4; i += RS_THREADS) {
            const float4 a0 = w4[i];
            m = fmaxf(m, fmaxf(fmaxf(a0.x, a0.y), fmaxf(a0.z, a0.w)));
        }
        for (int k = 4 * N4 + t; k < N; k += RS_THREADS) m1 = fmaxf(m1, w_all[k]);
        m = fmaxf(fmaxf(m, m1), fmaxf(m2, m3));
    } else {
        for (int b = t; b < B; b += RS_THREADS) m = fmaxf(m, part_max[b]);
    }
    m = wave_incl_max(m);
    if (lane == 63) s_f[wid] = m;
    __syncthreads();
    m = -INFINITY;
#pragma unroll
    for (int w = 0; w < RS_THREADS / 64; w++) m = fmaxf(m, s_f[w]);
    return m;
}

/* chunk b's sum of exp(w - mx) in the canonical wave tree (valid on thread 0) */
__device__ __forceinline__ double rs_chunk_expsum(const float* w, int N, float mx, int b, double* s_d) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int i = b * RS_THREADS + t;
    const double x = wave_incl_scan_d(i < N ? (double)expf(w[i] - mx) : 0.0);
    if (lane == 63) s_d[wid] = x;
    __syncthreads();
    double cs = 0.0;
    if (t == 0)
        for (int k = 0; k < RS_THREADS / 64; k++) cs += s_d[k];
    return cs;
}

/* chunk b normalised by lse (w_out may be w_in); its s2 partial, fixed-point
 * terms and their chunk-relative inclusive scan, chunk total and first arg-max
 * key */
template <bool WT = false>
__device__ __forceinline__ void rs_chunk_cdf(const float* w_in, float* w_out, int N, float lse, int b, double* part_s2,
                             unsigned long long* cdf_rel, unsigned long long* part_tot,
                             unsigned long long* part_key, double* s_d, unsigned long long* s_w64) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int i = b * RS_THREADS + t;
    double x2 = 0.0;
    unsigned long long term = 0ull, key = 0ull;
    if (i < N) {
        const float wv = w_in[i] - lse;
        st_u32<WT>(w_out + i, __float_as_uint(wv));
        x2 = (double)expf(2 * wv);
        const float tv = phd_det_expf(wv);
        term = (unsigned long long)phd_fix_term(tv);
        key = ((unsigned long long)__float_as_uint(tv) << 32) | (0xffffffffu - (unsigned)i);
    }
    x2 = wave_incl_scan_d(x2);
    const unsigned long long inc = wave_incl_scan_u64(term);
    key = wave_incl_max_u64(key);
    if (lane == 63) {
        s_d[wid] = x2;
        s_w64[wid] = inc;
        s_w64[16 + wid] = key;
    }
    __syncthreads();
    unsigned long long off = 0ull;
#pragma unroll
    for (int k = 0; k < RS_THREADS / 64; k++) off += k < wid ? s_w64[k] : 0ull;
    if (i < N) st_u64<WT>(cdf_rel + i, inc + off);
    if (t == 0) {
        double cs = 0.0;
        unsigned long long tot = 0ull, kmax = 0ull;
        for (int k = 0; k < RS_THREADS / 64; k++) {
            cs += s_d[k];
            tot += s_w64[k];
            kmax = s_w64[16 + k] > kmax ? s_w64[16 + k] : kmax;
        }
        st_u64<WT>(part_s2 + b, (unsigned long long)__double_as_longlong(cs));
        st_u64<WT>(part_tot + b, tot);
        st_u64<WT>(part_key + b, kmax);
    }
}

__global__ void __launch_bounds__(RS_THREADS) k_rs_max(const float* __restrict__ w, int N, float* __restrict__ part_max) {
    __shared__ float s_f[16];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int i = blockIdx.x * RS_THREADS + t;
    float m = wave_incl_max(i < N ? w[i] : -INFINITY);
    if (lane == 63) s_f[wid] = m;
    __syncthreads();
    if (t == 0) {
        m = -INFINITY;
        for (int k = 0; k < RS_THREADS / 64; k++) m = fmaxf(m, s_f[k]);
        part_max[blockIdx.x] = m;
    }
}

__global__ void __launch_bounds__(RS_THREADS)
    k_rs_sum(const float* __restrict__ w, int N, const float* __restrict__ part_max, int B,
             double* __restrict__ part_sum, int max_of_w) {
    __shared__ float s_f[16];
    __shared__ double s_d[16];
    const float mx = rs_global_max(part_max, B, s_f, max_of_w ? w : nullptr, N);
    // (k_rs_cdf normalises w in place, so it reads the max from here, not from w)
    if (max_of_w && threadIdx.x == 0) const_cast<float*>(part_max)[blockIdx.x] = mx;
    const double cs = rs_chunk_expsum(w, N, mx, blockIdx.x, s_d);
    if (threadIdx.x == 0) part_sum[blockIdx.x] = cs;
}

__global__ void __launch_bounds__(RS_THREADS)
    k_rs_cdf(float* __restrict__ w, int N, const float* __restrict__ part_max, const double* __restrict__ part_sum,
             int B, double* __restrict__ part_s2, unsigned long long* __restrict__ cdf_rel,
             unsigned long long* __restrict__ part_tot, unsigned long long* __restrict__ part_key,
             float* __restrict__ out) {
    __shared__ float s_f[16];
    __shared__ double s_d[16];
    __shared__ unsigned long long s_w64[32];
    __shared__ float s_lse;
    const int t = threadIdx.x;
    const float mx = rs_global_max(part_max, B, s_f);
    if (t == 0) {
        double total = 0.0;  // chunk sums in chunk order (chunk_sum_block)
        for (int b = 0; b < B; b++) total += part_sum[b];
        s_lse = d_safe_log((float)total) + mx;
    }
    __syncthreads();
    const float lse = s_lse;
    if (blockIdx.x == 0 && t == 0) out[0] = lse;
    rs_chunk_cdf(w, w, N, lse, blockIdx.x, part_s2, cdf_rel, part_tot, part_key, s_d, s_w64);
}

/* k_rs_sum + k_rs_cdf in one launch, up to 16 chunks (phd_step): every block
 * takes the max and the chunk sums of ALL entries itself — the same per-chunk
 * wave trees, added in chunk order, so the same bits as the two launches — and
 * then normalises its own chunk into w_out (w is left alone: the other blocks
 * are still reading it; the search moves w_out into place). */
template <bool WT = false>
__device__ __forceinline__ void rs_sumcdf_block(const float* __restrict__ w, float* __restrict__ w_out, int N, int B,
                                                double* part_s2, unsigned long long* cdf_rel,
                                                unsigned long long* part_tot, unsigned long long* part_key,
                                                float* __restrict__ out, float* s_f, double* s_d, double* s_dc,
                                                unsigned long long* s_w64, float* s_lse) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const float mx = rs_global_max(nullptr, B, s_f, w, N);
    for (int c = 0; c < B; c++) {
        const int i = c * RS_THREADS + t;
        const double x = wave_incl_scan_d(i < N ? (double)expf(w[i] - mx) : 0.0);
        if (lane == 63) s_dc[c * 16 + wid] = x;
    }
    __syncthreads();
    if (t == 0) {
        double total = 0.0;  // chunk sums in chunk order (chunk_sum_block)
        for (int c = 0; c < B; c++) {
            double cs = 0.0;
            for (int k = 0; k < RS_THREADS / 64; k++) cs += s_dc[c * 16 + k];
            total += cs;
        }
        *s_lse = d_safe_log((float)total) + mx;
    }
    __syncthreads();
    const float lse = *s_lse;
    if (blockIdx.x == 0 && t == 0) out[0] = lse;
    rs_chunk_cdf<WT>(w, w_out, N, lse, blockIdx.x, part_s2, cdf_rel, part_tot, part_key, s_d, s_w64);
}

__global__ void __launch_bounds__(RS_THREADS)
    k_rs_sumcdf(const float* __restrict__ w, float* __restrict__ w_out, int N, int B, double* __restrict__ part_s2,
                unsigned long long* __restrict__ cdf_rel, unsigned long long* __restrict__ part_tot,
                unsigned long long* __restrict__ part_key, float* __restrict__ out) {
    __shared__ float s_f[16];
    __shared__ double s_d[16];
    __shared__ double s_dc[16 * 16];
    __shared__ unsigned long long s_w64[32];
    __shared__ float s_lse;
    rs_sumcdf_block(w, w_out, N, B, part_s2, cdf_rel, part_tot, part_key, out, s_f, s_d, s_dc, s_w64, &s_lse);
}

struct RsSearchLds {
    unsigned long long end[RS_MAX_CHUNKS];
    unsigned long long w64[32];
    unsigned long long cdf[RS_STAGE_CHUNKS * RS_THREADS];
    int flag, cmin, cmax;
};

/* nEff and the decision (every block, identically); then stratum j = this
 * block's chunk entry: chunk by a search over the chunk ends, parent by a
 * search of that chunk's CDF.  The lower bound of r_j in the global CDF, as
 * resample_block; beyond the end it takes the first maximum (and `beyond`, when
 * given, records how many strata did: max of N - j).  The chunk results are
 * read with agent-scope vector loads (another workgroup of the one-launch plan
 * may have written them). */
template <bool WT = false>
__device__ __forceinline__ void rs_search_block(int N, int B, const double* part_s2, const unsigned long long* part_tot,
                                const unsigned long long* part_key, const unsigned long long* cdf_rel,
                                float resample_thresh, int has_meas, uint64_t seed, uint64_t step,
                                int* __restrict__ parents, float* out, const phd_pose* __restrict__ pose,
                                const int* __restrict__ src, phd_pose* __restrict__ new_pose, int* __restrict__ new_src,
                                float* __restrict__ logw, float new_logw, const float* __restrict__ w_norm,
                                unsigned* beyond, RsSearchLds& S, int blk) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    // up to RS_STAGE_CHUNKS chunks the whole CDF is staged in LDS, so the
    // stratum search costs LDS latencies instead of ten dependent global
    // loads; the loads issue here, under the decision's own loads
    const bool stage = B <= RS_STAGE_CHUNKS;
    unsigned long long cpre[RS_STAGE_CHUNKS];
#pragma unroll
    for (int k = 0; k < RS_STAGE_CHUNKS; k++) {
        const int e = k * RS_THREADS + t;
        cpre[k] = (stage && e < N) ? cdf_rel[e] : 0ull;
    }
    // the B chunk partials: one load per thread in parallel (S.end is free until
    // the chunk ends below), then summed in chunk order by one thread
    if (t < B) S.end[t] = ld_u64((const unsigned long long*)part_s2, t);
    __syncthreads();
    if (t == 0) {
        double s2 = 0.0;
        for (int b = 0; b < B; b++) s2 += __longlong_as_double((long long)S.end[b]);
        const float neff = (float)(1.0 / (double)(float)s2 / (double)N);
        const int resample = (has_meas == 2 || (has_meas && neff <= resample_thresh)) ? 1 : 0;  // 2: forced
        S.flag = resample;
        S.cmin = INT_MAX;  // (the chunks this workgroup's strata fall in, below)
        S.cmax = -1;
        if (blk == 0) {
            st_u32<WT>(out + 1, __float_as_uint(neff));
            st_u32<WT>(out + 2, (unsigned)resample);
            if (resample) atomicAdd((unsigned*)out + 4, 1u);  // decisions counter (phd_resample_count)
        }
    }
    // chunk ends (inclusive prefix of the chunk totals) and the first arg-max
    const unsigned long long tot = t < B ? ld_u64(part_tot, t) : 0ull;
    const unsigned long long kk = wave_incl_max_u64(t < B ? ld_u64(part_key, t) : 0ull);
    const unsigned long long inc = wave_incl_scan_u64(tot);
    if (lane == 63) {
        S.w64[wid] = inc;
        S.w64[16 + wid] = kk;
    }
    __syncthreads();
    const int j = blk * RS_THREADS + t;
    if (!S.flag) {
        if (pose && j < N) {  // remap form: the identity into the spare arrays
            new_pose[j] = pose[j];
            new_src[j] = src ? src[j] : j;
            if (w_norm) logw[j] = w_norm[j];  // (k_rs_sumcdf normalised out of place)
        }
        return;
    }
    unsigned long long off = 0ull, amaxk = 0ull;
#pragma unroll
    for (int k = 0; k < RS_THREADS / 64; k++) {
        off += k < wid ? S.w64[k] : 0ull;
        amaxk = S.w64[16 + k] > amaxk ? S.w64[16 + k] : amaxk;
    }
    if (t < B) S.end[t] = inc + off;
    if (stage) {
#pragma unroll
        for (int k = 0; k < RS_STAGE_CHUNKS; k++) S.cdf[k * RS_THREADS + t] = cpre[k];
    }
    __syncthreads();
    const bool live = j < N;
    unsigned long long r = 0ull;
    int a0 = B;  // first chunk whose end reaches r
    if (live) {
        const phd_u32x4 xr = phd_rng_draw(seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
        r = phd_fix_stratum(j, phd_u01(xr.v[0]), N);
        int b0 = B;
        a0 = 0;
        while (a0 < b0) {
            const int mid = (a0 + b0) >> 1;
            if (S.end[mid] >= r)
                b0 = mid;
            else
                a0 = mid + 1;
        }
    }
    // more chunks than are staged up front: the strata of one workgroup fall in
    // a few neighbouring chunks (consecutive strata, nondecreasing parents), so
    // those are staged now when they fit — one load round instead of a chain of
    // dependent global loads per stratum
    int c_lo = 0;
    bool staged = stage;
    if (!stage) {
        const bool in = live && a0 < B;
        const int lmax = __builtin_amdgcn_readlane(wave_incl_max_i(in ? a0 : -1), 63);
        const int lmin = -__builtin_amdgcn_readlane(wave_incl_max_i(in ? -a0 : -INT_MAX), 63);
        if (lane == 0 && lmax >= 0) {
            atomicMin(&S.cmin, lmin);
            atomicMax(&S.cmax, lmax);
        }
        __syncthreads();
        const int cmin = S.cmin, cmax = S.cmax;  // (workgroup-uniform)
        if (cmax >= cmin && cmax - cmin < RS_STAGE_CHUNKS) {
            for (int k = 0; k <= cmax - cmin; k++) {
                const int e = (cmin + k) * RS_THREADS + t;
                S.cdf[k * RS_THREADS + t] = e < N ? cdf_rel[e] : 0ull;
            }
            __syncthreads();
            staged = true;
            c_lo = cmin;
        }
    }
    if (!live) return;
    int p;
    if (a0 == B) {
        p = (int)(0xffffffffu - (unsigned)(amaxk & 0xffffffffull));
        if (beyond) __hip_atomic_fetch_max(beyond, (unsigned)(N - j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        const int c = a0;
        const unsigned long long base = c > 0 ? S.end[c - 1] : 0ull;
        const unsigned long long rr = r - base;  // r > base
        int lo = 0, hi = min(RS_THREADS, N - c * RS_THREADS) - 1;  // cc[hi] >= rr
        const unsigned long long* cc =
            staged ? S.cdf + (c - c_lo) * RS_THREADS : cdf_rel + (size_t)c * RS_THREADS;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cc[mid] >= rr)
                hi = mid;
            else
                lo = mid + 1;
        }
        p = c * RS_THREADS + lo;
    }
    st_u32<WT>(parents + j, (unsigned)p);
    if (pose) {  // copy_particles as an index remap (slamtypes.h:313-333): stratum j is this thread's
        new_pose[j] = pose[p];
        new_src[j] = src ? src[p] : p;  // (src NULL: the update just reset it to the identity)
        logw[j] = new_logw;
    }
}

__global__ void __launch_bounds__(RS_THREADS)
    k_rs_search(int N, int B, const double* __restrict__ part_s2, const unsigned long long* __restrict__ part_tot,
                const unsigned long long* __restrict__ part_key, const unsigned long long* __restrict__ cdf_rel,
                float resample_thresh, int has_meas, uint64_t seed, uint64_t step, int* __restrict__ parents,
                float* __restrict__ out, const phd_pose* __restrict__ pose, const int* __restrict__ src,
                phd_pose* __restrict__ new_pose, int* __restrict__ new_src, float* __restrict__ logw,
                float new_logw, const float* __restrict__ w_norm, unsigned* __restrict__ beyond) {
    __shared__ RsSearchLds S;
    rs_search_block(N, B, part_s2, part_tot, part_key, cdf_rel, resample_thresh, has_meas, seed, step, parents, out,
                    pose, src, new_pose, new_src, logw, new_logw, w_norm, beyond, S, blockIdx.x);
}

/* phd_step's normalise + nEff + decision + stratified resample by ONE
 * workgroup of NT threads — part C's lead workgroup (UpdateArgs::rs_lead),
 * whose log-weights are final (after the CPHD terms / the split PHD part A).
 * k_rs_step's arithmetic in its canonical order, so the same bits: chunk c's
 * virtual wave v (entries c 1024 + 64 v + lane) is scanned by real wave
 * v mod NW, its totals added in wave order per chunk and the chunks in chunk
 * order; the fixed-point CDF is exact.  The strata are searched in contiguous
 * runs per thread, each continuing from the previous parent (galloping).
 * LDS: ~9 KB of the part C allocation. */
template <int NT>
__device__ void rs_step_block(const RsStepArgs& a, unsigned char* smem) {
    constexpr int NW = NT / 64, VW = RS_THREADS / 64;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int N = a.N, B = a.B;  // B <= 16
    double* s_xs = (double*)smem;                                          // [16][VW] exp-sum wave totals
    double* s_x2 = s_xs + 16 * VW;                                         // [16][VW] s2 wave totals
    unsigned long long* s_tt = (unsigned long long*)(s_x2 + 16 * VW);      // [16][VW] fixed-point wave totals
    unsigned long long* s_tk = s_tt + 16 * VW;                             // [16][VW] arg-max keys
    unsigned long long* s_end = s_tk + 16 * VW;                            // [16] chunk ends
    float* s_f = (float*)(s_end + 16);                                     // NW maxima, lse
    int* s_i = (int*)(s_f + NW + 1);                                       // flag, arg-max
    // the max of every entry (order-free)
    float m = -INFINITY;
    for (int i = t; i < N; i += NT) m = fmaxf(m, a.w[i]);
    m = wave_incl_max(m);
    if (lane == 63) s_f[wid] = m;
    __syncthreads();
    float mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; w++) mx = fmaxf(mx, s_f[w]);
    // chunk sums of exp(w - mx) in the canonical wave tree (rs_sumcdf_block)
    for (int c = 0; c < B; c++)
        for (int v = wid; v < VW; v += NW) {
            const int i = c * RS_THREADS + v * 64 + lane;
            const double x = wave_incl_scan_d(i < N ? (double)expf(a.w[i] - mx) : 0.0);
            if (lane == 63) s_xs[c * VW + v] = x;
        }
    __syncthreads();
    if (t == 0) {
        double total = 0.0;
        for (int c = 0; c < B; c++) {
            double cs = 0.0;
            for (int k = 0; k < VW; k++) cs += s_xs[c * VW + k];
            total += cs;
        }
        s_f[NW] = d_safe_log((float)total) + mx;
    }
    __syncthreads();
    const float lse = s_f[NW];
    if (t == 0) a.out[0] = lse;
    // normalised entries (out of place), s2 terms, fixed-point terms -> each
    // virtual wave's inclusive scan into cdf_rel (chunk offsets added below)
    for (int c = 0; c < B; c++)
        for (int v = wid; v < VW; v += NW) {
            const int i = c * RS_THREADS + v * 64 + lane;
            double x2 = 0.0;
            unsigned long long term = 0ull, key = 0ull;
            if (i < N) {
                const float wv = a.w[i] - lse;
                a.w_out[i] = wv;
                x2 = (double)expf(2 * wv);
                const float tv = phd_det_expf(wv);
                term = (unsigned long long)phd_fix_term(tv);
                key = ((unsigned long long)__float_as_uint(tv) << 32) | (0xffffffffu - (unsigned)i);
            }
            x2 = wave_incl_scan_d(x2);
            const unsigned long long inc = wave_incl_scan_u64(term);
            key = wave_incl_max_u64(key);
            if (i < N) a.cdf_rel[i] = inc;
            if (lane == 63) {
                s_x2[c * VW + v] = x2;
                s_tt[c * VW + v] = inc;
                s_tk[c * VW + v] = key;
            }
        }
    __syncthreads();
    // chunk-relative offsets of the virtual waves (this thread's own entries)
    for (int c = 0; c < B; c++)
        for (int v = wid; v < VW; v += NW) {
            const int i = c * RS_THREADS + v * 64 + lane;
            unsigned long long off = 0ull;
            for (int k = 0; k < v; k++) off += s_tt[c * VW + k];
            if (i < N && off) a.cdf_rel[i] += off;
        }
    if (t == 0) {  // nEff, the decision, the chunk ends and the first arg-max (rs_search_block)
        double s2 = 0.0;
        unsigned long long e = 0ull, km = 0ull;
        for (int c = 0; c < B; c++) {
            double cs = 0.0;
            unsigned long long tot = 0ull;
            for (int k = 0; k < VW; k++) {
                cs += s_x2[c * VW + k];
                tot += s_tt[c * VW + k];
                km = s_tk[c * VW + k] > km ? s_tk[c * VW + k] : km;
            }
            s2 += cs;
            e += tot;
            s_end[c] = e;
        }
        const float neff = (float)(1.0 / (double)(float)s2 / (double)N);
        const int resample = (a.has_meas == 2 || (a.has_meas && neff <= a.resample_thresh)) ? 1 : 0;
        s_i[0] = resample;
        s_i[1] = (int)(0xffffffffu - (unsigned)(km & 0xffffffffull));
        a.out[1] = neff;
        ((unsigned*)a.out)[2] = (unsigned)resample;
        if (resample) atomicAdd((unsigned*)a.out + 4, 1u);  // decisions counter (phd_resample_count)
    }
    __syncthreads();
    if (!s_i[0]) {  // the identity into the spare arrays, the normalised weights into place
        for (int j = t; j < N; j += NT) {
            a.new_pose[j] = a.pose[j];
            a.new_src[j] = a.src ? a.src[j] : j;
            a.logw[j] = a.w_out[j];
        }
        return;
    }
    const int amax = s_i[1];
    const int per = (N + NT - 1) / NT, j0 = t * per, j1 = min(j0 + per, N);
    int c = 0, lo = 0;
    for (int j = j0; j < j1; j++) {
        const phd_u32x4 xr = phd_rng_draw(a.seed, (uint32_t)j, a.step, PHD_STREAM_RESAMPLE);
        const unsigned long long r = phd_fix_stratum(j, phd_u01(xr.v[0]), N);
        while (c < B && s_end[c] < r) {
            c++;
            lo = 0;
        }
        int p;
        if (c == B) {
            p = amax;  // past the CDF's end: the first maximum (main.cpp:470-488)
        } else {
            const unsigned long long rr = r - (c > 0 ? s_end[c - 1] : 0ull);
            const unsigned long long* cc = a.cdf_rel + (size_t)c * RS_THREADS;
            const int len = min(RS_THREADS, N - c * RS_THREADS);
            int h = lo, st = 1;
            while (cc[h] < rr) {  // (cc[len - 1] >= rr: the chunk's end reaches r)
                lo = h + 1;
                h = min(h + st, len - 1);
                st <<= 1;
            }
            while (lo < h) {
                const int mid = (lo + h) >> 1;
                if (cc[mid] >= rr)
                    h = mid;
                else
                    lo = mid + 1;
            }
            p = c * RS_THREADS + lo;
        }
        a.parents[j] = p;
        a.new_pose[j] = a.pose[p];  // copy_particles as an index remap (slamtypes.h:313-333)
        a.new_src[j] = a.src ? a.src[p] : p;
        a.logw[j] = a.new_logw;
    }
}

/* this rank's migration plan and local remap (one block), after the search:
 * the remapped poses / slab references go to the spare arrays (the identity
 * when no resample was decided), so the caller swaps them in without looking
 * at the decision, and the packing of outgoing records (next in the stream)
 * still reads the pre-resample store.  Without a resample the local
 * log-weights are the normalised slice.  mig[3 world + MIG_*] gets the
 * decision, nEff, and — with fixed blocks of `block_records` records per peer —
 * the slots whose record lies beyond its block (`pending`, in slot order) and the
 * overflow record counts, so one read-back (which may come a step later)
 * returns everything.  `out` / `w_all` / `parents` may have been written by
 * other workgroups of the same launch: read on the vector path. */
struct TailLds {
    MigLds L;
    int pre[MIG_MAX_WORLD + 1];
    int tmp;
};

__device__ __forceinline__ void shard_tail_block(const float* w_all, int n, int world, int rank, const float* out,
                                 const int* parents, int beyond, int* __restrict__ mig, int* __restrict__ keep_src,
                                 int* __restrict__ send_src, int* __restrict__ recv_rec,
                                 const phd_pose* __restrict__ pose, const int* __restrict__ src,
                                 phd_pose* __restrict__ new_pose, int* __restrict__ new_src,
                                 float* __restrict__ logw_local, float new_logw, int block_records,
                                 int* __restrict__ pending, unsigned timeout, int* mig_host, unsigned seq,
                                 TailLds& T, unsigned long long* st = nullptr) {
    const int t = threadIdx.x;
    PSTAMP(st, 0);
    const int resample = ld_par((const int*)out, 2);
    int* tail = mig + 3 * world;
    auto keep_store = [&](int q, const KeepRec& r) {
        new_pose[q] = r.p;
        new_src[q] = r.s;
        logw_local[q] = r.w;
    };
    if (!resample) {  // the identity; the local log-weights are the normalised slice
        migration_plan_block(
            0, ParentView{parents, 0, 0, 0}, n, world, rank, mig, keep_src, send_src, recv_rec, T.L,
            [&](int q, int k) { return KeepRec{pose[k], src ? src[k] : k, ld_f32(w_all, rank * n + q)}; }, keep_store, st);
    } else {
        const ParentView par = parent_view(parents, n * world, n, beyond, &T.tmp);
        PSTAMP(st, 1);
        migration_plan_block(
            1, par, n, world, rank, mig, keep_src, send_src, recv_rec, T.L,
            [&](int q, int k) { return KeepRec{pose[k], src ? src[k] : k, new_logw}; }, keep_store, st);
    }
    __syncthreads();
    // records beyond the fixed blocks: sent, received, and the slots they feed
    // (the per-rank counts from the plan's LDS: nothing moves without a resample)
    const int K = block_records;
    if (t == 0) {
        int os = 0, orc = 0;
        T.pre[0] = 0;
        for (int s = 0; s < world; s++) {
            const int sn = resample ? T.L.send[s] : 0, rc = resample ? T.L.recv[s] : 0;
            os += max(sn - K, 0);
            orc += max(rc - K, 0);
            T.pre[s + 1] = T.pre[s] + rc;  // first record of source s
        }
        tail[MIG_OVF_SEND] = os;
        tail[MIG_OVF_RECV] = orc;
    }
    __syncthreads();
    const int d = resample ? min(T.L.lo[rank + 1] - T.L.lo[rank], n) : n;
    int npend = 0;
    for (int b = 0; b < n - d; b += RS_THREADS) {
        const int i = b + t;
        int late = 0;
        if (i < n - d) {
            const int rho = recv_rec[i];
            int a0 = 0, b0 = world;  // source of record rho: last s with pre[s] <= rho
            while (b0 - a0 > 1) {
                const int mid = (a0 + b0) >> 1;
                if (T.pre[mid] <= rho) a0 = mid;
                else b0 = mid;
            }
            late = rho - T.pre[a0] >= K;
        }
        int total;
        const int pos = block_flag_scan(late, T.L.wc, total);
        if (late) pending[npend + pos] = d + i;
        npend += total;
    }
    if (t == 0) {
        tail[MIG_LSE] = ld_par((const int*)out, 0);
        tail[MIG_NEFF] = ld_par((const int*)out, 1);
        tail[MIG_FLAG] = resample;
        tail[MIG_PENDING] = npend;
        tail[MIG_OVF_CAP] = 0;
        tail[MIG_TIMEOUT] = (int)timeout;
    }
    PSTAMP(st, 5);
    if (mig_host) {  // the host's copy of the plan (host-mapped memory: no read-back launch)
        __syncthreads();
        for (int i = t; i < 3 * world + MIG_SEQ; i += RS_THREADS) mig_host[i] = mig[i];
        // then the sequence number the host polls: every wave's stores to the
        // host have completed, one system-scope release store after them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(mig_host + 3 * world + MIG_SEQ, (int)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    PSTAMP(st, 6);
}

/* the tail as its own launch (after k_rs_search, when the one-launch plan's
 * grid would not be resident at once): reads and clears the beyond count */
__global__ void __launch_bounds__(RS_THREADS)
    k_shard_tail(const float* __restrict__ w_all, int n, int world, int rank, const float* __restrict__ out,
                 const int* __restrict__ parents, unsigned* __restrict__ sync, int* __restrict__ mig,
                 int* __restrict__ mig_host, int* __restrict__ keep_src, int* __restrict__ send_src, int* __restrict__ recv_rec,
                 const phd_pose* __restrict__ pose, const int* __restrict__ src, phd_pose* __restrict__ new_pose,
                 int* __restrict__ new_src, float* __restrict__ logw_local, float new_logw, int block_records,
                 int* __restrict__ pending, unsigned seq) {
    __shared__ TailLds T;
    const int beyond = (int)__hip_atomic_load(sync + PLAN_BEYOND, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(sync + PLAN_BEYOND, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    shard_tail_block(w_all, n, world, rank, out, parents, beyond, mig, keep_src, send_src, recv_rec, pose, src,
                     new_pose, new_src, logw_local, new_logw, block_records, pending, 0u, mig_host, seq, T);
}

/* The context stream's wait for the plan on the plan stream (phd_kernels.h):
 * a cross-stream event's barrier packet had held the context stream ~15 us
 * after part C although the plan had finished before it
 * (profiles/r06_shard_w1_trace_summary.txt); one poll of the word, normally
 * already written, and the next launch's acquire at its start. */
__global__ void __launch_bounds__(64) k_wait_plan(const int* seqw, unsigned seq, unsigned* sync_timeout) {
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while ((int)((unsigned)__hip_atomic_load(seqw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins == (1u << 26)) {  // (~4 s: a plan takes ~50 us)
                __hip_atomic_fetch_or(sync_timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
}

/* In-launch hand-off of k_shard_plan / k_rs_step (every workgroup resident:
 * the host keeps the grid within one workgroup per CU).  The handed-off words
 * are stored write-through (st_u32 / st_u64 <true>), so no release fence is
 * needed.  Arrive: every storing wave drains its stores (vmcnt(0)), the
 * workgroup barrier orders them before one lane's agent-scope counter add.
 * Wait: one lane polls the counter relaxed, with a sleep, then one agent-scope
 * acquire (this CU's L1 invalidated) before the workgroup barrier; the spin is
 * bounded, a timeout is recorded and the kernel goes on, so the grid always
 * drains. */
__device__ __forceinline__ void plan_arrive(unsigned* ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void plan_wait(unsigned* ctr, unsigned target, unsigned* timeout) {
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins == (1u << 22)) {
                __hip_atomic_fetch_or(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

/* The whole sharded plan in one launch of B = ceil(N / RS_THREADS) workgroups:
 *   1. every workgroup takes the max of all N entries itself and its chunk's
 *      sum of exp(w - max) (k_rs_sum's tree) -> part_sum; wait for all B;
 *   2. lse from the B chunk sums in chunk order, its chunk normalised in place,
 *      CDF terms (k_rs_cdf) -> part_s2 / part_tot / part_key / cdf_rel; wait;
 *   3. nEff, decision, the parents of its strata (k_rs_search); a ticket;
 *   4. the last workgroup to take a ticket runs this rank's tail
 *      (shard_tail_block) and resets the launch's counters for the next one.
 * Same arithmetic in the same order as the four-launch chain, so the same
 * bits. */
__global__ void __launch_bounds__(RS_THREADS) k_shard_plan(ShardPlanArgs a) {
    __shared__ float s_f[16];
    __shared__ double s_d[16];
    __shared__ float s_lse;
    __shared__ int s_last;
    __shared__ union PlanLds {
        RsSearchLds rs;
        TailLds tail;
    } U;
    const int t = threadIdx.x, b = blockIdx.x;
    unsigned* sync = a.sync;
    const unsigned B = (unsigned)a.B;
    unsigned long long* st = a.stamps ? a.stamps + (size_t)b * 8 : nullptr;
    (void)st;
    PSTAMP(st, 0);
    // 1. the max of all N, this chunk's exp sum
    const float mx = rs_global_max(nullptr, a.B, s_f, a.w, a.N);
    const double cs = rs_chunk_expsum(a.w, a.N, mx, b, s_d);
    if (t == 0) st_u64<true>(a.part_sum + b, (unsigned long long)__double_as_longlong(cs));
    PSTAMP(st, 1);
    plan_arrive(sync + PLAN_ARRIVE0);
    plan_wait(sync + PLAN_ARRIVE0, B, sync + PLAN_TIMEOUT);
    PSTAMP(st, 2);
    // 2. lse, this chunk normalised, its CDF terms (the chunk sums: one load per
    // thread in parallel, added in chunk order by one thread)
    if (t < a.B) U.rs.end[t] = ld_u64((const unsigned long long*)a.part_sum, t);
    __syncthreads();
    if (t == 0) {
        double total = 0.0;  // chunk sums in chunk order (chunk_sum_block)
        for (int c = 0; c < a.B; c++) total += __longlong_as_double((long long)U.rs.end[c]);
        s_lse = d_safe_log((float)total) + mx;
    }
    __syncthreads();
    const float lse = s_lse;
    if (b == 0 && t == 0) st_u32<true>(a.out, __float_as_uint(lse));
    rs_chunk_cdf<true>(a.w, a.w, a.N, lse, b, a.part_s2, a.cdf_rel, a.part_tot, a.part_key, s_d, U.rs.w64);
    PSTAMP(st, 3);
    plan_arrive(sync + PLAN_ARRIVE1);
    plan_wait(sync + PLAN_ARRIVE1, B, sync + PLAN_TIMEOUT);
    PSTAMP(st, 4);
    // 3. decision and parents
    rs_search_block<true>(a.N, a.B, a.part_s2, a.part_tot, a.part_key, a.cdf_rel, a.resample_thresh, a.has_meas,
                          a.seed, a.step, a.parents, a.out, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, nullptr,
                          sync + PLAN_BEYOND, U.rs, b);
    PSTAMP(st, 5);
    // 4. ticket: the last workgroup runs the tail (parents and the decision
    // were stored write-through: drained, then the ticket)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const unsigned old = __hip_atomic_fetch_add(sync + PLAN_TICKET, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == B - 1u;
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    PSTAMP(st, 6);
    if (!s_last) return;
    const int beyond = (int)__hip_atomic_load(sync + PLAN_BEYOND, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned timeout = __hip_atomic_load(sync + PLAN_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    // every workgroup has passed both waits and taken its ticket: reset for the next launch
    if (t < PLAN_SYNC_WORDS) __hip_atomic_store(sync + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    shard_tail_block(a.w, a.n, a.world, a.rank, a.out, a.parents, beyond, a.mig, a.keep_src, a.send_src, a.recv_rec,
                     a.pose, a.src, a.new_pose, a.new_src, a.logw_local, a.new_logw, a.block_records, a.pending,
                     timeout, a.mig_host, a.seq, U.tail, a.stamps ? a.stamps + (size_t)a.B * 8 : nullptr);
}

/* phd_step's normalise + nEff + decision + resample + remap up to 16 chunks in
 * ONE launch: k_rs_sumcdf's work (every workgroup the max and all chunk sums
 * itself), one in-launch wait for the chunk results, then k_rs_search's
 * (decision, parents, the remapped store into the spare arrays).  Same
 * arithmetic, so the same bits as the two launches.  The last workgroup to
 * take a ticket resets the wait's words; a wait that gave up (not every
 * workgroup resident: the host keeps the grid <= 16) sets PHD_ST_WAIT_TIMEOUT. */
/* phd_step's normalise / nEff / resample in one launch: every workgroup
 * searches its own strata after an in-launch wait for all chunk partials.
 * Beside part C (the CPHD step) a workgroup may wait until part C's tail
 * frees a CU for the last one: part C never waits on this launch, so the
 * wait always ends (the bounded spin and PHD_ST_WAIT_TIMEOUT are a safety
 * net).  A ticket form without any wait — the last workgroup to arrive
 * searching every chunk — cost 1.6 % steps/s at config 3 (its serial
 * searches start in part C's tail; round 5, profiles/r05_c3_partC_ab.txt). */
__global__ void __launch_bounds__(RS_THREADS) k_rs_step(RsStepArgs a) {
    __shared__ float s_f[16];
    __shared__ double s_d[16];
    __shared__ double s_dc[16 * 16];
    __shared__ float s_lse;
    __shared__ int s_last;
    __shared__ RsSearchLds S;
    const int t = threadIdx.x;
    unsigned* sync = a.sync;
    rs_sumcdf_block<true>(a.w, a.w_out, a.N, a.B, a.part_s2, a.cdf_rel, a.part_tot, a.part_key, a.out, s_f, s_d, s_dc,
                          S.w64, &s_lse);
    plan_arrive(sync + STEP_ARRIVE);
    plan_wait(sync + STEP_ARRIVE, (unsigned)a.B, sync + STEP_TIMEOUT);
    rs_search_block(a.N, a.B, a.part_s2, a.part_tot, a.part_key, a.cdf_rel, a.resample_thresh, a.has_meas, a.seed,
                    a.step, a.parents, a.out, a.pose, a.src, a.new_pose, a.new_src, a.logw, a.new_logw, a.w_out,
                    nullptr, S, blockIdx.x);
    __syncthreads();
    if (t == 0) {
        const unsigned old = __hip_atomic_fetch_add(sync + STEP_TICKET, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)a.B - 1u;
    }
    __syncthreads();
    if (s_last && t == 0) {  // every workgroup is past its wait
        if (__hip_atomic_load(sync + STEP_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicOr(a.err, PHD_ST_WAIT_TIMEOUT);
        __hip_atomic_store(sync + STEP_ARRIVE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sync + STEP_TICKET, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sync + STEP_TIMEOUT, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

/* CPHD births through the prediction (addBirths + birthsKernel,
 * phdfilter.cu.bak:738-870): every particle's map gets one component per
 * measurement of the previous scan (static-labelled ones when labels are on):
 * the inverse measurement from the particle's pose (d_birth), weight
 * birthWeight.  The CPHD update array has no birth terms, so this is how its
 * maps grow.  One workgroup per particle: its slab (via the index table) is
 * copied into its slab of the other set with the births appended.  With
 * `slots` (a sharded step's pending slots re-stepped on an empty scan) block b
 * takes particle slots[b] and resets its slab reference to the identity itself
 * (the other particles' references are not touched: no k_iota follows). */
__global__ void __launch_bounds__(256)
    k_add_births(int* __restrict__ src, const int* __restrict__ slots, int n, int cap,
                 const float* __restrict__ map_in, const int* __restrict__ size_in, const float* __restrict__ map_x,
                 const int* __restrict__ size_x, float* __restrict__ map_out, int* __restrict__ size_out,
                 const phd_pose* __restrict__ pose, const float* __restrict__ zr, const float* __restrict__ zb,
                 const int* __restrict__ zok, int M, DevCfg c, int* __restrict__ status, int* __restrict__ err) {
    if ((int)blockIdx.x >= n) return;
    const int j = slots ? slots[blockIdx.x] : (int)blockIdx.x;
    __shared__ int s_rank[257];
    const int sref = src[j];
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int sl = sref & PHD_SLAB_MASK;
    const int G = in_x ? size_x[sl] : size_in[sl];
    const float* s = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
    float* d = map_out + (size_t)j * NF * cap;
    for (int f = 0; f < NF; f++)
        for (int k = threadIdx.x; k < G; k += blockDim.x) d[f * cap + k] = s[f * cap + k];
    if (threadIdx.x == 0) {  // order-preserving ranks of the birth measurements
        int r = 0;
        for (int m = 0; m < M; m++) {
            s_rank[m] = r;
            r += zok[m] != 0;
        }
        s_rank[M] = r;
    }
    __syncthreads();
    const phd_pose ps = pose[j];
    for (int m = threadIdx.x; m < M; m += blockDim.x) {
        if (!zok[m]) continue;
        const int k = G + s_rank[m];
        if (k >= cap) continue;
        float mean[2], cov[4];
        d_birth(c, ps.px, ps.py, ps.ptheta, zr[m], zb[m], mean, cov);
        d[k] = c.birthWeight;
        d[cap + k] = mean[0];
        d[2 * cap + k] = mean[1];
        d[3 * cap + k] = cov[0];
        d[4 * cap + k] = cov[1];
        d[5 * cap + k] = cov[2];
        d[6 * cap + k] = cov[3];
    }
    if (threadIdx.x == 0) {
        const int tot = G + s_rank[M];
        size_out[j] = min(tot, cap);
        if (slots) src[j] = j;  // (every lane read sref before the barrier above)
        if (tot > cap) {
            status[j] |= PHD_ST_MAP_OVERFLOW;
            atomicOr(err, PHD_ST_MAP_OVERFLOW);
            atomicAdd(err + 3, 1);
        }
    }
}

/* Particle record: [pose(6f) | logw | size | map 7*cap] as 32-bit words.
 * `dcount` (device) overrides `count` when given (records beyond it are not
 * written); the grid strides over records.  `logw_set` != 0 writes `logw_value`
 * as the record's log-weight (a sharded resample's -log N). */
__global__ void __launch_bounds__(256)
    k_pack(const int* __restrict__ dcount, const int* __restrict__ src_idx, int count, int cap,
           const int* __restrict__ src, const float* __restrict__ map_in, const int* __restrict__ size_in,
           const float* __restrict__ map_x, const int* __restrict__ size_x, const phd_pose* __restrict__ pose,
           const float* __restrict__ logw, int logw_set, float logw_value, const double* __restrict__ cn,
           const double* __restrict__ cn_x, int cn_stride, float* __restrict__ rec) {
    if (dcount) count = min(*dcount, count);
    const size_t rw = record_words(cap, cn_stride);
    for (int r = blockIdx.x; r < count; r += gridDim.x) {
        const int p = src_idx[r];
        const int sref = src[p];
        const bool in_x = (sref & PHD_SLAB_X) != 0;
        const int sl = sref & PHD_SLAB_MASK;
        float* o = rec + (size_t)r * rw;
        const int sz = in_x ? size_x[sl] : size_in[sl];
        if (threadIdx.x == 0) {
            const float* ps = (const float*)&pose[p];
            for (int k = 0; k < 6; k++) o[k] = ps[k];
            o[6] = logw_set ? logw_value : logw[p];
            ((int*)o)[7] = sz;
        }
        const float* s = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
        for (int f = 0; f < NF; f++)
            for (int k = threadIdx.x; k < sz; k += blockDim.x) o[8 + f * cap + k] = s[f * cap + k];
        if (cn_stride) {  // CPHD cardinality coefficients travel with the particle
            const double* cs = (in_x ? cn_x : cn) + (size_t)sl * cn_stride;
            double* co = (double*)(o + 8 + (size_t)NF * cap);
            for (int k = threadIdx.x; k < cn_stride; k += blockDim.x) co[k] = cs[k];
        }
    }
}

/* Unpack record r into migration slab x_slot[r] of set X and point particle dst_idx[r] at it. */
__global__ void __launch_bounds__(256)
    k_unpack(const float* __restrict__ rec, const int* __restrict__ dst_idx, const int* __restrict__ x_slot, int count,
             int cap, float* __restrict__ map_x, int* __restrict__ size_x, int* __restrict__ src,
             phd_pose* __restrict__ pose, float* __restrict__ logw, double* __restrict__ cn_x, int cn_stride) {
    const int r = blockIdx.x;
    if (r >= count) return;
    const int p = dst_idx[r];
    const int xs = x_slot ? x_slot[r] : r;
    const size_t rw = record_words(cap, cn_stride);
    const float* o = rec + (size_t)r * rw;
    const int sz = min(max(((const int*)o)[7], 0), cap);  // a record never carries more than cap
    if (threadIdx.x == 0) {
        float* pd = (float*)&pose[p];
        for (int k = 0; k < 6; k++) pd[k] = o[k];
        logw[p] = o[6];
        size_x[xs] = sz;
        src[p] = xs | PHD_SLAB_X;
    }
    float* d = map_x + (size_t)xs * NF * cap;
    for (int f = 0; f < NF; f++)
        for (int k = threadIdx.x; k < sz; k += blockDim.x) d[f * cap + k] = o[8 + f * cap + k];
    if (cn_stride) {
        const double* ci = (const double*)(o + 8 + (size_t)NF * cap);
        for (int k = threadIdx.x; k < cn_stride; k += blockDim.x) cn_x[(size_t)xs * cn_stride + k] = ci[k];
    }
}

/* Receive side of a sharded resample: slot first_slot + i takes record
 * slot_rec[i]; the first slot of each record copies its map into migration slab
 * slot_rec[i] of set X, and every slot of the record points at that slab. */
__global__ void __launch_bounds__(256)
    k_unpack_slots(const float* __restrict__ rec, const int* __restrict__ slot_rec, int nslots, int first_slot, int cap,
                   float* __restrict__ map_x, int* __restrict__ size_x, int* __restrict__ src,
                   phd_pose* __restrict__ pose, float* __restrict__ logw, double* __restrict__ cn_x, int cn_stride) {
    const int i = blockIdx.x;
    if (i >= nslots) return;
    const int r = slot_rec[i];
    const int p = first_slot + i;
    const size_t rw = record_words(cap, cn_stride);
    const float* o = rec + (size_t)r * rw;
    const int sz = min(max(((const int*)o)[7], 0), cap);
    if (threadIdx.x == 0) {
        float* pd = (float*)&pose[p];
        for (int k = 0; k < 6; k++) pd[k] = o[k];
        logw[p] = o[6];
        src[p] = r | PHD_SLAB_X;
    }
    if (i > 0 && slot_rec[i - 1] == r) return;
    if (threadIdx.x == 0) size_x[r] = sz;
    float* dd = map_x + (size_t)r * NF * cap;
    for (int f = 0; f < NF; f++)
        for (int k = threadIdx.x; k < sz; k += blockDim.x) dd[f * cap + k] = o[8 + f * cap + k];
    if (cn_stride) {
        const double* ci = (const double*)(o + 8 + (size_t)NF * cap);
        for (int k = threadIdx.x; k < cn_stride; k += blockDim.x) cn_x[(size_t)r * cn_stride + k] = ci[k];
    }
}

/* The sender's records in fixed blocks: record t of send_src goes to rank d
 * (records are grouped by destination, mig[world + d] each) as its r-th record:
 * block slot d * block_records + r, or — beyond the block — position
 * Σ_{d' < d} max(sent_d' - K, 0) + r - K of the overflow buffer (exchanged
 * only when a read-back shows it used).  Records carry the new log-weight. */
__global__ void __launch_bounds__(256)
    k_pack_blocks(const int* __restrict__ mig, int world, const int* __restrict__ send_src, int block_records,
                  int ovf_capacity, int cap, const int* __restrict__ src, const float* __restrict__ map_in,
                  const int* __restrict__ size_in, const float* __restrict__ map_x, const int* __restrict__ size_x,
                  const phd_pose* __restrict__ pose, float logw_value, const double* __restrict__ cn,
                  const double* __restrict__ cn_x, int cn_stride, float* __restrict__ blocks,
                  float* __restrict__ ovf, int* __restrict__ ovf_flag) {
    const int count = mig[3 * world + MIG_SENT];
    const size_t rw = record_words(cap, cn_stride);
    const int K = block_records;
    for (int t = blockIdx.x; t < count; t += gridDim.x) {
        int d = 0, first = 0, ofirst = 0;
        while (d < world - 1 && t >= first + mig[world + d]) {
            first += mig[world + d];
            ofirst += max(mig[world + d] - K, 0);
            d++;
        }
        const int r = t - first;
        float* o;
        if (r < K) {
            o = blocks + ((size_t)d * K + r) * rw;
        } else {
            const int oi = ofirst + r - K;
            if (oi >= ovf_capacity) {
                if (threadIdx.x == 0) ovf_flag[0] = 1;
                continue;
            }
            o = ovf + (size_t)oi * rw;
        }
        const int p = send_src[t];
        const int sref = src[p];
        const bool in_x = (sref & PHD_SLAB_X) != 0;
        const int sl = sref & PHD_SLAB_MASK;
        const int sz = in_x ? size_x[sl] : size_in[sl];
        if (threadIdx.x == 0) {
            const float* ps = (const float*)&pose[p];
            for (int k = 0; k < 6; k++) o[k] = ps[k];
            o[6] = logw_value;
            ((int*)o)[7] = sz;
        }
        const float* sp = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
        for (int f = 0; f < NF; f++)
            for (int k = threadIdx.x; k < sz; k += blockDim.x) o[8 + f * cap + k] = sp[f * cap + k];
        if (cn_stride) {
            const double* cs = (in_x ? cn_x : cn) + (size_t)sl * cn_stride;
            double* co = (double*)(o + 8 + (size_t)NF * cap);
            for (int k = threadIdx.x; k < cn_stride; k += blockDim.x) co[k] = cs[k];
        }
    }
}

/* Receive side: deficit slot d + i takes record recv_rec[i] (records numbered
 * in source-rank order, mig[2 world + s] from source s); record r of source s
 * is slot s * K + r of the fixed blocks, or (overflow != 0) position
 * Σ_{s' < s} max(recv_s' - K, 0) + r - K of the received overflow buffer.  The
 * first slot of each record copies its map into migration slab recv_rec[i] of
 * set X; every slot of the record points at it.  One workgroup per slot at a
 * time, strided over a grid of min(n, 256) (the deficit is read on the device). */
__global__ void __launch_bounds__(256)
    k_unpack_blocks(const float* __restrict__ blocks, const float* __restrict__ ovf, int block_records, int overflow,
                    const int* __restrict__ mig, int world, int rank, const int* __restrict__ recv_rec, int n,
                    int cap, float* __restrict__ map_x, int* __restrict__ size_x, int* __restrict__ src,
                    phd_pose* __restrict__ pose, float* __restrict__ logw, double* __restrict__ cn_x,
                    int cn_stride) {
    const int d = min(mig[rank], n);
    const int K = block_records;
    const size_t rw = record_words(cap, cn_stride);
    // receiving slots d + i, i in [0, n - d), strided over the grid (a grid of
    // min(n, 256) workgroups: a step that moves nothing costs one short wave each)
    for (int i = blockIdx.x; d + i < n; i += gridDim.x) {
        const int rho = recv_rec[i];
        int s = 0, first = 0, ofirst = 0;
        while (s < world - 1 && rho >= first + mig[2 * world + s]) {
            first += mig[2 * world + s];
            ofirst += max(mig[2 * world + s] - K, 0);
            s++;
        }
        const int r = rho - first;
        if ((r >= K) != (overflow != 0)) continue;  // the other pass's record
        const float* o = r < K ? blocks + ((size_t)s * K + r) * rw : ovf + (size_t)(ofirst + r - K) * rw;
        const int p = d + i;
        const int sz = min(max(((const int*)o)[7], 0), cap);
        if (threadIdx.x == 0) {
            float* pd = (float*)&pose[p];
            for (int k = 0; k < 6; k++) pd[k] = o[k];
            logw[p] = o[6];
            src[p] = rho | PHD_SLAB_X;
        }
        if (i > 0 && recv_rec[i - 1] == rho) continue;
        if (threadIdx.x == 0) size_x[rho] = sz;
        float* dd = map_x + (size_t)rho * NF * cap;
        for (int f = 0; f < NF; f++)
            for (int k = threadIdx.x; k < sz; k += blockDim.x) dd[f * cap + k] = o[8 + f * cap + k];
        if (cn_stride) {
            const double* ci = (const double*)(o + 8 + (size_t)NF * cap);
            for (int k = threadIdx.x; k < cn_stride; k += blockDim.x) cn_x[(size_t)rho * cn_stride + k] = ci[k];
        }
    }
}

/* ------------------------------------------------------------ state outputs */

__global__ void __launch_bounds__(1024)
    k_expected_pose(const float* __restrict__ logw, const phd_pose* __restrict__ pose, int n, float* __restrict__ out) {
    __shared__ double s[32];
    double acc[6] = {0, 0, 0, 0, 0, 0};
    float bw = -FLT_MAX;
    int bi = INT_MAX;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float w = logw[i];
        const float ew = expf(w);
        const float* ps = (const float*)&pose[i];
        for (int k = 0; k < 6; k++) acc[k] += (double)(ew * ps[k]);
        if (w > bw) {
            bw = w;
            bi = i;
        }
    }
    for (int k = 0; k < 6; k++) {
        const double v = block_reduce_1024<double>(acc[k], s, false);
        if (threadIdx.x == 0) out[k] = (float)v;
    }
    // first arg-max (strict >, main.cpp:348-353)
    __shared__ float sv[1024];
    __shared__ int si[1024];
    sv[threadIdx.x] = bw;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const float ov = sv[threadIdx.x + o];
            const int oi = si[threadIdx.x + o];
            if (ov > sv[threadIdx.x] || (ov == sv[threadIdx.x] && oi < si[threadIdx.x])) {
                sv[threadIdx.x] = ov;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) ((int*)out)[6] = si[0];
}

/* Per-particle PHD cardinality Σ_j w_j (double sum); one wave per particle. */
__global__ void __launch_bounds__(256)
    k_cardinality(const int* __restrict__ src, const float* __restrict__ map_in, const int* __restrict__ size_in,
                  const float* __restrict__ map_x, const int* __restrict__ size_x, int n, int cap, float* __restrict__ cn) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= n) return;
    const int lane = threadIdx.x & 63;
    const int sref = src[p];
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int sl = sref & PHD_SLAB_MASK;
    const float* w = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
    const int sz = in_x ? size_x[sl] : size_in[sl];
    double s = 0.0;
    for (int k = lane; k < sz; k += 64) s += (double)w[k];
    s = wave_sum_d(s);
    if (lane == 0) cn[p] = (float)s;
}

}  // namespace phd
