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
 *   k_expected_pose / k_cardinality    — main.cpp:331-361
 */
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "phd_detmath.h"
#include "phd_device.h"
#include "phd_kernels.h"
#include "phd_rng.h"

#define NF 7 /* fields per component */

namespace phd {

/* ------------------------------------------------------------------ predict */

__global__ void k_predict_ackerman(phd_pose* __restrict__ poses, int n, phd_ackerman_control u,
                                   const phd_ackerman_noise* __restrict__ noise_in, PredictCfg c, uint64_t seed,
                                   uint64_t step, const phd_pose* __restrict__ pose_prior,
                                   const float* __restrict__ logw_prior, float* __restrict__ logw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (logw_prior) logw[i] = logw_prior[i];  // replay: restore the fixed prior
    float n_alpha, n_enc;
    if (noise_in) {
        n_alpha = noise_in[i].n_alpha;
        n_enc = noise_in[i].n_encoder;
    } else {
        const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)i, step, PHD_STREAM_PREDICT);
        double g0, g1;
        phd_box_muller(x.v[0], x.v[1], &g0, &g1);
        n_alpha = (float)((double)c.stdAlpha * g0);
        n_enc = (float)((double)c.stdEncoder * g1);
    }
    const phd_pose s = pose_prior ? pose_prior[i] : poses[i];
    phd_pose ns;
    const float ve = u.v_encoder + n_enc;
    const float al = u.alpha + n_alpha;
    const float ta = tanf(al);
    const float vc = ve / (1 - ta * c.h / c.l);
    float st, ct;
    sincosf(s.ptheta, &st, &ct);
    const float xc_dot = vc * ct;
    const float yc_dot = vc * st;
    const float thetac_dot = vc * ta / c.l;
    const float dt = c.dt / c.subdivide;
    ns.px = s.px + dt * (xc_dot - thetac_dot * (c.a * st + c.b * ct));
    ns.py = s.py + dt * (yc_dot + thetac_dot * (c.a * ct - c.b * st));
    ns.ptheta = d_wrap(s.ptheta + dt * thetac_dot);
    ns.vx = 0;
    ns.vy = 0;
    ns.vtheta = 0;
    poses[i] = ns;
}

__global__ void k_predict_cv(phd_pose* __restrict__ poses, int n, const phd_cv_noise* __restrict__ noise_in,
                             PredictCfg c, uint64_t seed, uint64_t step, const phd_pose* __restrict__ pose_prior,
                             const float* __restrict__ logw_prior, float* __restrict__ logw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (logw_prior) logw[i] = logw_prior[i];  // replay: restore the fixed prior
    phd_cv_noise w;
    if (noise_in) {
        w = noise_in[i];
    } else {
        const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)i, step, PHD_STREAM_PREDICT);
        double g0, g1, g2, g3;
        phd_box_muller(x.v[0], x.v[1], &g0, &g1);
        phd_box_muller(x.v[2], x.v[3], &g2, &g3);
        w.ax = (float)((double)(3 * c.ax) * g0);
        w.ay = (float)((double)(3 * c.ay) * g1);
        w.atheta = (float)((double)(3 * c.ayaw) * g2);
    }
    const phd_pose s = pose_prior ? pose_prior[i] : poses[i];
    phd_pose ns;
    const float dt = c.dt / c.subdivide;
    float st, ct;
    sincosf(s.ptheta, &st, &ct);
    ns.px = (float)((double)(s.px + dt * (s.vx * ct - s.vy * st)) + (double)(dt * dt) * 0.5 * (double)(w.ax * ct - w.ay * st));
    ns.py = (float)((double)(s.py + dt * (s.vx * st + s.vy * ct)) + (double)(dt * dt) * 0.5 * (double)(w.ax * st + w.ay * ct));
    ns.ptheta = d_wrap((float)((double)(s.ptheta + dt * s.vtheta) + 0.5 * dt * dt * (double)w.atheta));
    ns.vx = s.vx + dt * w.ax;
    ns.vy = s.vy + dt * w.ay;
    ns.vtheta = s.vtheta + dt * w.atheta;
    poses[i] = ns;
}

/* ------------------------------------------------------------ block helpers */

/* Order-preserving compaction rank of `pred` within a 256-thread block.
 * Returns this thread's exclusive rank; *total gets the block count. */
__device__ __forceinline__ int block_rank(bool pred, int* s_wcnt, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long m = __ballot(pred);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wcnt[wid] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < UPD_THREADS / 64; w++) {
        const int c = s_wcnt[w];
        off += (w < wid) ? c : 0;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return off + rank;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* Sum of up to 4 doubles over the block (the "intended exact sum", oracle D3);
 * every thread gets the totals. s_red holds >= 16 doubles. */
template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* s_red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = wave_sum_d(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; k++) s_red[wid * 4 + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < UPD_THREADS / 64; w++) t += s_red[w * 4 + k];
        v[k] = t;
    }
    __syncthreads();
}

/* ------------------------------------------------------- fused PHD update */

__global__ void __launch_bounds__(UPD_THREADS)
    k_update_fused(UpdateArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const UpdLds L = upd_lds_layout(a.cap, a.Mcap, a.Kcap, a.Scap);
    float* s_zr = (float*)(smem + L.zr);
    float* s_zb = (float*)(smem + L.zb);
    int* s_zok = (int*)(smem + L.zok);
    float* s_leta = (float*)(smem + L.leta);
    double* s_part = (double*)(smem + L.part);
    unsigned short* s_in = (unsigned short*)(smem + L.in);
    unsigned short* s_near = (unsigned short*)(smem + L.near);
    unsigned short* s_out = (unsigned short*)(smem + L.out);
    unsigned int* s_skey = (unsigned int*)(smem + L.skey);
    float* s_slq = (float*)(smem + L.slq);
    int* s_cnt = (int*)(smem + L.cnt);  // [0]=n_in [1]=n_near [2]=n_out [3]=n_surv [4]=flags [8..11]=wave counts
    double* s_red = (double*)(smem + L.red);
    float* s_redf = (float*)(smem + L.redf);
    // union region: comp table (phases 2-3) / candidates (phases 4-5)
    float* t_r = (float*)(smem + L.u);
    float* t_b = t_r + a.cap;
    float* t_S0 = t_b + a.cap;
    float* t_S12 = t_S0 + a.cap;
    float* t_S3 = t_S12 + a.cap;
    float* t_c = t_S3 + a.cap;
    double* t_hk = (double*)(t_c + a.cap);
    float* cw = (float*)(smem + L.u);
    float* cx = cw + a.Kcap;
    float* cy = cx + a.Kcap;
    float* cc0 = cy + a.Kcap;
    float* cc1 = cc0 + a.Kcap;
    float* cc2 = cc1 + a.Kcap;
    float* cc3 = cc2 + a.Kcap;
    int* cflag = (int*)(cc3 + a.Kcap);

    const int n = blockIdx.x;
    const int tid = threadIdx.x;
    const DevCfg& c = a.c;
    const int M = a.M;
    // slab of particle n: set `in` (or the migration set X) via the index table
    const int sref = a.src ? a.src[n] : n;
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int slab = sref & PHD_SLAB_MASK;
    const int G = in_x ? a.size_x[slab] : a.size_in[slab];
    const float* __restrict__ src = (in_x ? a.map_x : a.map_in) + (size_t)slab * NF * a.cap;
    float* __restrict__ dst = a.map_out + (size_t)n * NF * a.cap;
    const phd_pose pose = a.poses[n];

    for (int m = tid; m < M; m += UPD_THREADS) {
        s_zr[m] = a.zr[m];
        s_zb[m] = a.zb[m];
        s_zok[m] = a.zok[m];
    }
    if (tid < 8) s_cnt[tid] = 0;
    __syncthreads();

    /* Phase 1: 3-way range classification (computeInRangeKernel :1328-1346),
     * order-preserving split into in / near / out index lists. */
    for (int base = 0; base < G; base += UPD_THREADS) {
        const int k = base + tid;
        int cls = -1;
        if (k < G) {
            const float dx = src[1 * a.cap + k] - pose.px;
            const float dy = src[2 * a.cap + k] - pose.py;
            const float r = sqrtf(dx * dx + dy * dy);
            const float ab = fabsf(d_wrap(phd_atan2f(dy, dx) - pose.ptheta));
            if (r >= c.minRange && r <= c.maxRange && ab <= c.maxBearing)
                cls = 1;
            else if ((double)r >= 0.8 * (double)c.minRange && (double)r <= 1.2 * (double)c.maxRange &&
                     (double)ab <= 1.2 * (double)c.maxBearing)
                cls = 2;
            else
                cls = 0;
        }
        int tot;
        int r1 = block_rank(cls == 1, s_cnt + 8, &tot);
        if (cls == 1) s_in[s_cnt[0] + r1] = (unsigned short)k;
        const int t1 = tot;
        int r2 = block_rank(cls == 2, s_cnt + 8, &tot);
        if (cls == 2) s_near[s_cnt[1] + r2] = (unsigned short)k;
        const int t2 = tot;
        int r0 = block_rank(cls == 0, s_cnt + 8, &tot);
        if (cls == 0) s_out[s_cnt[2] + r0] = (unsigned short)k;
        const int t0 = tot;
        __syncthreads();
        if (tid == 0) {
            s_cnt[0] += t1;
            s_cnt[1] += t2;
            s_cnt[2] += t0;
        }
        __syncthreads();
    }
    const int Gin = s_cnt[0], Gnear = s_cnt[1], Gout = s_cnt[2];

    /* Phase 2: per in-range component EKF terms into the LDS pair table. */
    double card_d = 0.0;
    for (int j = tid; j < Gin; j += UPD_THREADS) {
        const int k = s_in[j];
        const float w = src[k];
        DevEkf e;
        d_compute_ekf(c, pose.px, pose.py, pose.ptheta, src[1 * a.cap + k], src[2 * a.cap + k], src[3 * a.cap + k],
                      src[4 * a.cap + k], src[5 * a.cap + k], src[6 * a.cap + k], e);
        t_r[j] = e.r;
        t_b[j] = e.bearing;
        t_S0[j] = e.S0;
        t_S12[j] = e.S1 + e.S2;
        t_S3[j] = e.S3;
        t_c[j] = d_safe_log(e.pd) + d_safe_log(w);
        t_hk[j] = c.log_2pi + 0.5 * (double)d_safe_log(e.det);
        card_d += (double)(e.pd * w);
    }
    {
        double v[1] = {card_d};
        block_sum<1>(v, s_red);  // also orders phase-2 LDS writes before phase 3
        card_d = v[0];
    }

    /* Phase 3: pair loop — lanes over measurements, groups over components.
     * η_m partials stay in registers; surviving-candidate terms are listed. */
    {
        const int ngrp = UPD_THREADS / M;
        const int m = tid % M;
        const int grp = tid / M;
        double eta = 0.0;
        if (grp < ngrp) {
            const float zr = s_zr[m], zb = s_zb[m];
            const bool zok = s_zok[m] != 0;
            for (int j = grp; j < Gin; j += ngrp) {
                const float i0 = zr - t_r[j];
                const float i1 = d_wrap(zb - t_b[j]);
                const float dist = i0 * i0 * t_S0[j] + i0 * i1 * t_S12[j] + i1 * i1 * t_S3[j];
                const float g = (float)(-0.5 * (double)dist - t_hk[j]);
                const float lq = zok ? t_c[j] + g : PHD_LOG0;
                eta += (double)expf(lq);
                if (lq >= c.lq_keep_thresh) {
                    const int s = atomicAdd(&s_cnt[3], 1);
                    if (s < a.Scap) {
                        s_skey[s] = ((unsigned int)m << 16) | (unsigned int)j;
                        s_slq[s] = lq;
                    }
                }
            }
        }
        s_part[tid] = eta;
        __syncthreads();
        if (tid < M) {
            float sum = 0.f;
            if (Gin > 0) {
                double sd = 0.0;
                for (int g2 = 0; g2 < ngrp; g2++) sd += s_part[g2 * M + tid];
                sd += (double)c.kappa;
                sd += (double)c.birthWeight;
                sum = (float)sd;
            } else {
                sum = c.kappa + c.birthWeight;
            }
            s_leta[tid] = d_safe_log(sum);
        }
        __syncthreads();
    }
    if (tid == 0) {
        float pw = 0.f;
        for (int m = 0; m < M; m++) pw += s_leta[m];
        const float cardp = (float)(card_d + (double)M * (double)c.birthWeight);
        const float delta = pw - cardp;
        a.delta[n] = delta;
        a.logw[n] += delta;
    }
    int nsurv = s_cnt[3];
    int flags = 0;
    if (nsurv > a.Scap) {
        flags |= PHD_ST_SURVIVOR_OVERFLOW;
        nsurv = a.Scap;
    }

    /* Sort surviving detection terms by their update-array position (m-major, j). */
    {
        int P = 1;
        while (P < nsurv) P <<= 1;
        for (int i = nsurv + tid; i < P; i += UPD_THREADS) s_skey[i] = 0xffffffffu;
        __syncthreads();
        for (int k2 = 2; k2 <= P; k2 <<= 1) {
            for (int jj = k2 >> 1; jj > 0; jj >>= 1) {
                for (int i = tid; i < P; i += UPD_THREADS) {
                    const int ixj = i ^ jj;
                    if (ixj > i) {
                        const bool asc = (i & k2) == 0;
                        const unsigned int ki = s_skey[i], kj = s_skey[ixj];
                        if ((ki > kj) == asc) {
                            s_skey[i] = kj;
                            s_skey[ixj] = ki;
                            const float t = s_slq[i];
                            s_slq[i] = s_slq[ixj];
                            s_slq[ixj] = t;
                        }
                    }
                }
                __syncthreads();
            }
        }
    }

    /* Phase 4: merge candidates in update-array order
     * [non-detect | detect (m-major) | births | near-range]; prune w < minW. */
    int ncand = 0;
    // 4a non-detection terms
    for (int base = 0; base < Gin; base += UPD_THREADS) {
        const int j = base + tid;
        float w = 0.f;
        bool keep = false;
        int k = 0;
        if (j < Gin) {
            k = s_in[j];
            w = src[k] * (1 - c.pd);
            keep = !(w < c.minFeatureWeight);
        }
        int tot;
        const int r = block_rank(keep, s_cnt + 8, &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                cw[p] = w;
                cx[p] = src[1 * a.cap + k];
                cy[p] = src[2 * a.cap + k];
                cc0[p] = src[3 * a.cap + k];
                cc1[p] = src[4 * a.cap + k];
                cc2[p] = src[5 * a.cap + k];
                cc3[p] = src[6 * a.cap + k];
            }
        }
        ncand += tot;
    }
    // 4b detection terms (recompute EKF for the component; correction μ + Kν)
    for (int base = 0; base < nsurv; base += UPD_THREADS) {
        const int s = base + tid;
        bool keep = false;
        float w = 0.f;
        int j = 0, m = 0;
        if (s < nsurv) {
            const unsigned int key = s_skey[s];
            m = (int)(key >> 16);
            j = (int)(key & 0xffffu);
            w = expf(s_slq[s] - s_leta[m]);
            keep = !(w < c.minFeatureWeight);
        }
        int tot;
        const int r = block_rank(keep, s_cnt + 8, &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                const int k = s_in[j];
                const float mx = src[1 * a.cap + k], my = src[2 * a.cap + k];
                DevEkf e;
                d_compute_ekf(c, pose.px, pose.py, pose.ptheta, mx, my, src[3 * a.cap + k], src[4 * a.cap + k],
                              src[5 * a.cap + k], src[6 * a.cap + k], e);
                const float i0 = s_zr[m] - e.r;
                const float i1 = d_wrap(s_zb[m] - e.bearing);
                cw[p] = w;
                cx[p] = mx + e.K0 * i0 + e.K2 * i1;
                cy[p] = my + e.K1 * i0 + e.K3 * i1;
                cc0[p] = e.cu0;
                cc1[p] = e.cu1;
                cc2[p] = e.cu2;
                cc3[p] = e.cu3;
            }
        }
        ncand += tot;
    }
    // 4c births
    for (int base = 0; base < M; base += UPD_THREADS) {
        const int m = base + tid;
        bool keep = false;
        float w = 0.f;
        if (m < M) {
            const float lb = s_zok[m] ? c.log_birth : PHD_LOG0;
            w = expf(lb - s_leta[m]);
            keep = !(w < c.minFeatureWeight);
        }
        int tot;
        const int r = block_rank(keep, s_cnt + 8, &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < a.Kcap) {
                float mean[2], cov[4];
                d_birth(c, pose.px, pose.py, pose.ptheta, s_zr[m], s_zb[m], mean, cov);
                cw[p] = w;
                cx[p] = mean[0];
                cy[p] = mean[1];
                cc0[p] = cov[0];
                cc1[p] = cov[1];
                cc2[p] = cov[2];
                cc3[p] = cov[3];
            }
        }
        ncand += tot;
    }
    // 4d near-range components join the merge unpruned (mergeAndCopyMaps :3227-3257)
    for (int q = tid; q < Gnear; q += UPD_THREADS) {
        const int p = ncand + q;
        if (p < a.Kcap) {
            const int k = s_near[q];
            cw[p] = src[k];
            cx[p] = src[1 * a.cap + k];
            cy[p] = src[2 * a.cap + k];
            cc0[p] = src[3 * a.cap + k];
            cc1[p] = src[4 * a.cap + k];
            cc2[p] = src[5 * a.cap + k];
            cc3[p] = src[6 * a.cap + k];
        }
    }
    ncand += Gnear;
    if (ncand > a.Kcap) {
        flags |= PHD_ST_CANDIDATE_OVERFLOW;
        ncand = a.Kcap;
    }
    for (int i = tid; i < ncand; i += UPD_THREADS) cflag[i] = 0;
    __syncthreads();

    /* Phase 5: greedy merge (phdUpdateMergeKernel :2739-2890).  Ties in the
     * max-weight search resolve to the lowest candidate index (oracle D1). */
    int nout = 0;
    const int lane = tid & 63, wid = tid >> 6;
    const float T = c.minSeparation;
    while (true) {
        float bw = -INFINITY;
        int bi = INT_MAX;
        for (int i = tid; i < ncand; i += UPD_THREADS) {
            if (cflag[i] == 0 && (bi == INT_MAX || cw[i] > bw)) {
                bw = cw[i];
                bi = i;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ow = __shfl_xor(bw, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oi != INT_MAX && (bi == INT_MAX || ow > bw || (ow == bw && oi < bi))) {
                bw = ow;
                bi = oi;
            }
        }
        if (lane == 0) {
            s_redf[wid] = bw;
            ((int*)s_redf)[8 + wid] = bi;
        }
        __syncthreads();
        bw = -INFINITY;
        bi = INT_MAX;
#pragma unroll
        for (int w2 = 0; w2 < UPD_THREADS / 64; w2++) {
            const float ow = s_redf[w2];
            const int oi = ((int*)s_redf)[8 + w2];
            if (oi != INT_MAX && (bi == INT_MAX || ow > bw || (ow == bw && oi < bi))) {
                bw = ow;
                bi = oi;
            }
        }
        __syncthreads();
        if (bi == INT_MAX) break;
        const float mx = cx[bi], my = cy[bi], m0 = cc0[bi], m1 = cc1[bi], m2 = cc2[bi], m3 = cc3[bi];
        double acc[3] = {0.0, 0.0, 0.0};
        for (int i = tid; i < ncand; i += UPD_THREADS) {
            if (cflag[i] != 0) continue;
            const float d = d_mahal(mx, my, m0, m1, m2, m3, cx[i], cy[i], cc0[i], cc1[i], cc2[i], cc3[i]);
            if (d < T) {
                cflag[i] = 2;
                const float w = cw[i];
                acc[0] += (double)w;
                acc[1] += (double)(w * cx[i]);
                acc[2] += (double)(w * cy[i]);
            }
        }
        block_sum<3>(acc, s_red);
        const float W = (float)acc[0];
        if (W == 0.f) break;
        const float gx = (float)acc[1] / W, gy = (float)acc[2] / W;
        double cv[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = tid; i < ncand; i += UPD_THREADS) {
            if (cflag[i] != 2) continue;
            const float d0 = gx - cx[i], d1 = gy - cy[i];
            const float w = cw[i];
            cv[0] += (double)(w * (cc0[i] + d0 * d0));
            cv[1] += (double)(w * (cc1[i] + d0 * d1));
            cv[2] += (double)(w * (cc2[i] + d1 * d0));
            cv[3] += (double)(w * (cc3[i] + d1 * d1));
            cflag[i] = 1;
        }
        block_sum<4>(cv, s_red);
        if (tid == 0) {
            if (nout < a.cap) {
                float p0 = (float)cv[0] / W, p1 = (float)cv[1] / W, p2 = (float)cv[2] / W, p3 = (float)cv[3] / W;
                p1 = (p1 + p2) / 2;
                p2 = p1;
                dst[nout] = W;
                dst[1 * a.cap + nout] = gx;
                dst[2 * a.cap + nout] = gy;
                dst[3 * a.cap + nout] = p0;
                dst[4 * a.cap + nout] = p1;
                dst[5 * a.cap + nout] = p2;
                dst[6 * a.cap + nout] = p3;
            }
        }
        nout++;
    }

    /* Phase 6: out-of-range components appended unchanged (mergeAndCopyMaps :3304-3323). */
    for (int q = tid; q < Gout; q += UPD_THREADS) {
        const int p = nout + q;
        if (p < a.cap) {
            const int k = s_out[q];
#pragma unroll
            for (int f = 0; f < NF; f++) dst[f * a.cap + p] = src[f * a.cap + k];
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
        if (flags) atomicOr(a.err, flags);
        if (a.src_reset) a.src_reset[n] = n;  // posterior of particle n now lives in out slab n
    }
}

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

/* logSumExp normalisation (phdfilter.cu:3748-3755) and nEff (main.cpp:1281-1284);
 * sums in double (oracle D3). */
__global__ void __launch_bounds__(1024) k_normalize(float* __restrict__ logw, int n, const float* lse_override,
                                                    float* __restrict__ out /* [0]=lse [1]=neff [2]=resample? */,
                                                    float resample_thresh, int has_meas) {
    __shared__ float sf[32];
    __shared__ double sd[32];
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, logw[i]);
    mx = block_reduce_1024<float>(mx, sf, true);
    float lse;
    if (lse_override) {
        lse = *lse_override;
    } else {
        double sum = 0.0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) sum += (double)expf(logw[i] - mx);
        sum = block_reduce_1024<double>(sum, sd, false);
        lse = d_safe_log((float)sum) + mx;
    }
    double s2 = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float w = logw[i] - lse;
        logw[i] = w;
        s2 += (double)expf(2 * w);
    }
    s2 = block_reduce_1024<double>(s2, sd, false);
    if (threadIdx.x == 0) {
        const float neff = (float)(1.0 / (double)(float)s2 / (double)n);
        out[0] = lse;
        out[1] = neff;
        // main.cpp:1286-1289 (the n_particles > 5*N clause never fires: n is fixed here)
        ((int*)out)[2] = (has_meas && neff <= resample_thresh) ? 1 : 0;
    }
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

/* Stratified resample (main.cpp:453-501), single 1024-thread block:
 * fixed-point CDF of det_expf terms (phd_detmath.h) -> per-stratum binary
 * search -> parent indices.  copy_particles (slamtypes.h:313-333) becomes an
 * index remap: children take the parent's pose and slab reference; maps are
 * never copied (copy-on-write through the slab index table).  If `flag` is
 * non-NULL and *flag == 0 the kernel does nothing (device-side decision). */
__global__ void __launch_bounds__(1024)
    k_resample(const int* __restrict__ flag, const float* __restrict__ logw_in, float* __restrict__ logw_out, int n,
               const double* __restrict__ u_in, uint64_t seed, uint64_t step, unsigned long long* __restrict__ cdf,
               int* __restrict__ idx, phd_pose* __restrict__ pose, int* __restrict__ src, phd_pose* __restrict__ tmp_pose,
               int* __restrict__ tmp_src, float new_logw) {
    if (flag && *flag == 0) return;
    __shared__ unsigned long long s_tot[1024];
    __shared__ float s_tv[1024];
    __shared__ int s_ti[1024];
    const int t = threadIdx.x;
    const int per = (n + blockDim.x - 1) / blockDim.x;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    unsigned long long acc = 0;
    float tmax = -1.f;
    int imax = INT_MAX;
    for (int i = lo; i < hi; i++) {
        const float tv = phd_det_expf(logw_in[i]);
        acc += (unsigned long long)phd_fix_term(tv);
        cdf[i] = acc;
        if (tv > tmax) {
            tmax = tv;
            imax = i;
        }
    }
    s_tot[t] = acc;
    s_tv[t] = tmax;
    s_ti[t] = imax;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {
        const unsigned long long add = (t >= o) ? s_tot[t - o] : 0ull;
        __syncthreads();
        s_tot[t] += add;
        __syncthreads();
    }
    const unsigned long long off = (t > 0) ? s_tot[t - 1] : 0ull;
    for (int i = lo; i < hi; i++) cdf[i] += off;
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (t < o) {
            const float ov = s_tv[t + o];
            const int oi = s_ti[t + o];
            if (ov > s_tv[t] || (ov == s_tv[t] && oi < s_ti[t])) {
                s_tv[t] = ov;
                s_ti[t] = oi;
            }
        }
        __syncthreads();
    }
    const int amax = s_ti[0];
    __syncthreads();
    for (int j = t; j < n; j += blockDim.x) {
        double u;
        if (u_in) {
            u = u_in[j];
        } else {
            const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
            u = phd_u01(x.v[0]);
        }
        const unsigned long long r = phd_fix_stratum(j, u, n);
        int a0 = 0, b0 = n;
        while (a0 < b0) {
            const int mid = (a0 + b0) >> 1;
            if (cdf[mid] >= r)
                b0 = mid;
            else
                a0 = mid + 1;
        }
        const int p = (a0 < n) ? a0 : amax;
        idx[j] = p;
        if (pose) {
            tmp_pose[j] = pose[p];
            tmp_src[j] = src ? src[p] : p;
        }
    }
    __syncthreads();
    if (pose) {
        for (int j = t; j < n; j += blockDim.x) {
            pose[j] = tmp_pose[j];
            if (src) src[j] = tmp_src[j];
            logw_out[j] = new_logw;
        }
    }
}

/* Apply a caller-computed parent list (local parents): same remap as k_resample. */
__global__ void __launch_bounds__(1024)
    k_apply_parents(const int* __restrict__ idx, int n, phd_pose* __restrict__ pose, int* __restrict__ src,
                    float* __restrict__ logw, phd_pose* __restrict__ tmp_pose, int* __restrict__ tmp_src, float new_logw) {
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

/* Materialise slab references into dense slabs (export helper): dst slab j = slab src[j]. */
__global__ void __launch_bounds__(256)
    k_materialize(const int* __restrict__ src, int n, int cap, const float* __restrict__ map_in,
                  const int* __restrict__ size_in, const float* __restrict__ map_x, const int* __restrict__ size_x,
                  float* __restrict__ map_dst, int* __restrict__ size_dst) {
    const int j = blockIdx.x;
    const int sref = src[j];
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int sl = sref & PHD_SLAB_MASK;
    const int sz = in_x ? size_x[sl] : size_in[sl];
    const float* s = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
    float* d = map_dst + (size_t)j * NF * cap;
    for (int f = 0; f < NF; f++)
        for (int k = threadIdx.x; k < sz; k += blockDim.x) d[f * cap + k] = s[f * cap + k];
    if (threadIdx.x == 0) size_dst[j] = sz;
}

/* Particle record: [pose(6f) | logw | size | map 7*cap] as 32-bit words. */
__global__ void __launch_bounds__(256)
    k_pack(const int* __restrict__ src_idx, int count, int cap, const int* __restrict__ src, const float* __restrict__ map_in,
           const int* __restrict__ size_in, const float* __restrict__ map_x, const int* __restrict__ size_x,
           const phd_pose* __restrict__ pose, const float* __restrict__ logw, float* __restrict__ rec) {
    const int r = blockIdx.x;
    if (r >= count) return;
    const int p = src_idx[r];
    const int sref = src[p];
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int sl = sref & PHD_SLAB_MASK;
    const size_t rw = 8 + (size_t)NF * cap;
    float* o = rec + (size_t)r * rw;
    const int sz = in_x ? size_x[sl] : size_in[sl];
    if (threadIdx.x == 0) {
        const float* ps = (const float*)&pose[p];
        for (int k = 0; k < 6; k++) o[k] = ps[k];
        o[6] = logw[p];
        ((int*)o)[7] = sz;
    }
    const float* s = (in_x ? map_x : map_in) + (size_t)sl * NF * cap;
    for (int f = 0; f < NF; f++)
        for (int k = threadIdx.x; k < sz; k += blockDim.x) o[8 + f * cap + k] = s[f * cap + k];
}

/* Unpack record r into migration slab x_slot[r] of set X and point particle dst_idx[r] at it. */
__global__ void __launch_bounds__(256)
    k_unpack(const float* __restrict__ rec, const int* __restrict__ dst_idx, const int* __restrict__ x_slot, int count,
             int cap, float* __restrict__ map_x, int* __restrict__ size_x, int* __restrict__ src,
             phd_pose* __restrict__ pose, float* __restrict__ logw) {
    const int r = blockIdx.x;
    if (r >= count) return;
    const int p = dst_idx[r];
    const int xs = x_slot ? x_slot[r] : r;
    const size_t rw = 8 + (size_t)NF * cap;
    const float* o = rec + (size_t)r * rw;
    const int sz = ((const int*)o)[7];
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
