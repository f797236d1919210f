/*
 * phd_wave.hip — the fused RB-PHD / CPHD update with ONE WAVEFRONT PER PARTICLE
 * (the north-star layout): a 64-thread workgroup owns particle blockIdx.x for
 * the whole update.  Every "block" operation of the workgroup-per-particle
 * kernel (phd_kernels.hip) becomes a wave operation — DPP scans, ballot/mbcnt
 * compaction, readlane broadcasts — so the update has no s_barrier on its
 * path and its LDS footprint (phd_wave.h) admits several particles per CU.
 *
 * Reference semantics (same arithmetic as the workgroup kernel and the oracle):
 *   classification      phdfilter.cu:1328-1346 (computeInRangeKernel)
 *   EKF / pair terms    phdfilter.cu:1824-1925 (preUpdateSynthKernel)
 *   weights, eta        phdfilter.cu:2083-2321 (phdUpdateKernel)
 *   births              phdfilter.cu:3466-3518
 *   prune               phdfilter.cu:3105-3174
 *   merge, copy maps    phdfilter.cu:2707-2898, :3176-3333
 *   CPHD terms          phdfilter.cu.bak:990-1504, Poisson prior .bak:2473-2497
 *
 * Phases of one particle:
 *   1+3  chunks of 64 prior components, lane = component: classify, EKF terms
 *        in registers, then the lane walks its own bearing window of the
 *        bearing-sorted measurements (oracle D7); eta_m accumulates as an exact
 *        two-word fixed point (2^-40 integer part | 2^-72 fraction) with 64-bit
 *        LDS atomics (order independent, so deterministic); listable
 *        detection terms are appended to a key list.
 *   2    CPHD terms (one wave) or the PHD normaliser and delta log w.
 *   4    merge candidates [non-detect | detect (m-major) | births | near] in
 *        LDS; covariances of prior-derived candidates stay in the prior slab
 *        (read from L2 when needed), detection / birth covariances in LDS.
 *   5    exact parallel greedy merge (lattice cull, CSR, asynchronous LFMIS)
 *        with the serial greedy as fallback; emission straight to the slab.
 *   6    out-of-range components appended.
 */
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "phd_detmath.h"
#include "phd_device.h"
#include "phd_devutil.h"
#include "phd_kernels.h"
#include "phd_rng.h"
#include "phd_wave.h"
#include "phd_cphd_terms.h"

#define NF 7
#ifndef MERGE_DEG_REG
#define MERGE_DEG_REG 8 /* merge neighbour lists up to this length are handled in registers */
#endif


namespace phd {





__device__ __forceinline__ float uni_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ int uni_i(int x) { return __builtin_amdgcn_readfirstlane(x); }

/* exclusive rank of `pred` among the lanes below, and the wave count */
__device__ __forceinline__ int wrank(bool pred, int* total) {
    const unsigned long long b = __ballot(pred);
    *total = __popcll(b);
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u));
}

__device__ __forceinline__ int wave_max_i(int x) {
    x = max(x, dpp_or_zero<0x111, 0xf>(x));
    x = max(x, dpp_or_zero<0x112, 0xf>(x));
    x = max(x, dpp_or_zero<0x114, 0xf>(x));
    x = max(x, dpp_or_zero<0x118, 0xf>(x));
    x = max(x, dpp_or_zero<0x142, 0xa>(x));
    x = max(x, dpp_or_zero<0x143, 0xc>(x));
    return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ int wave_sum_i(int x) { return __builtin_amdgcn_readlane(wave_incl_scan(x), 63); }
__device__ __forceinline__ int wave_or_i(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
    return uni_i(x);
}
__device__ __forceinline__ float wave_max_fu(float x) { return uni_f(__shfl(wave_incl_max(x), 63, 64)); }

/* eta_m (and the CPHD Lambda_m) as an order-independent fixed point with ONE
 * 64-bit LDS atomic per term: terms q >= 2^-17 go to hi as q 2^40 (exact: their
 * ulp is >= 2^-40), smaller ones to lo as q 2^70 (exact for q >= 2^-47,
 * truncated below 2^-70).  lo has headroom for 2^11 terms of < 2^53 per
 * measurement (lo_shift 70 for maps up to 2047 components, 60 above); q >= 2^20
 * sets PHD_ST_ETA_RANGE (hi's headroom).  Terms below 2^-lo_shift add nothing,
 * which is what bounds the bearing windows (WALK_LOG2_FLOOR). */
#define WALK_LOG2_FLOOR (-72.f)
__device__ __forceinline__ void eta_add(u64* ehi, u64* elo, int m, float q, float lo_scale, int& flags) {
#if defined(PHD_EXPERIMENT) && (PHD_EXPERIMENT == 11 || PHD_EXPERIMENT == 23)
    if (q > 1e30f) flags |= 32;  // timing ablation: no atomics
    return;
#endif
    // branch-free: one scale, one conversion, one (non-returning) atomic
    if (q >= 1048576.f) flags |= PHD_ST_ETA_RANGE;
    const bool hi = q >= 7.62939453125e-06f;  // 2^-17
    const u64 y = (u64)(fminf(q, 4194304.f) * (hi ? 1099511627776.f : lo_scale));  // 2^40 | lo scale
    if (y) atomicAdd((hi ? ehi : elo) + m, y);
}

/* wrapAngle (d_wrap) for |x| < 4 pi_f without branches: fmodf by 2 pi_f is the
 * exact subtraction there (Sterbenz), then the same +-2 pi step in double. */
__device__ __forceinline__ float wrap_small(float x) {
    const float two_pi_f = (float)(2 * M_PI);
    const float r = fabsf(x) < two_pi_f ? x : x - copysignf(two_pi_f, x);
    const double d = r;
    return d > M_PI ? (float)(d - 2 * M_PI) : d < -M_PI ? (float)(d + 2 * M_PI) : r;
}

/* Per-lane EKF terms of one prior component (phase 1). */
struct WComp {
    float r, b, S0, S12, S3, C2;
    int lo, cnt;  // bearing window into the sorted measurements
};

/* classification + EKF + bearing window of component fields v (phases 1-2 of
 * the workgroup kernel; same expressions).  Returns the class (0 out, 1 in, 2 near). */
__device__ __forceinline__ int classify_comp(const DevCfg& c, const phd_pose& pose, const float* v, int Mv,
                                             const unsigned short* s_zbin, float lb, WComp& t, float& pdw) {
    const float k2 = 0.72134752044448170f;
    const float dx = v[1] - pose.px;
    const float dy = v[2] - pose.py;
    const float r2 = dx * dx + dy * dy;
    const float r = sqrtf(r2);
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 21
    const float bearing = d_wrap(atan2f(dy, dx) - pose.ptheta);  // timing ablation
#else
    const float bearing = d_wrap(phd_atan2f(dy, dx) - pose.ptheta);
#endif
    const float ab = fabsf(bearing);
    int cls;
    if (r >= c.minRange && r <= c.maxRange && ab <= c.maxBearing)
        cls = 1;
    else if ((double)r >= 0.8 * (double)c.minRange && (double)r <= 1.2 * (double)c.maxRange &&
             (double)ab <= 1.2 * (double)c.maxBearing)
        cls = 2;
    else
        cls = 0;
    t.cnt = 0;
    t.lo = 0;
    pdw = 0.f;
    if (cls == 1) {
        const float w = v[0];
        DevEkf e;
        d_ekf_from_geometry(c, dx, dy, r2, r, bearing, v[3], v[4], v[5], v[6], e);
        const double lc = (double)(d_safe_log(e.pd) + d_safe_log(w)) - c.log_2pi - 0.5 * (double)d_safe_log(e.det);
        const float C2 = (float)(1.4426950408889634 * lc);
        const float S12 = e.S1 + e.S2;
        t.r = e.r;
        t.b = e.bearing;
        t.S0 = e.S0;
        t.S12 = S12;
        t.S3 = e.S3;
        t.C2 = C2;
        pdw = e.pd;
        t.cnt = Mv;  // every valid measurement
        if (!(C2 > lb) && C2 == C2) {
            t.cnt = 0;  // every pair underflows
        } else {
            const float kap = e.S3 - S12 * S12 / (4.f * e.S0);
            if (e.S0 > 0.f && kap > 0.f && kap < INFINITY && C2 < 1e30f) {
                const float hw = sqrtf(2.f * (C2 - lb) / (k2 * kap)) * 1.001f + 1e-4f;
                const float binw = 6.28318530717958648f / PHD_ZBINS;
                const int ba = (int)floorf((e.bearing - hw + 3.14159265358979f) / binw) - 1;
                const int bc = (int)floorf((e.bearing + hw + 3.14159265358979f) / binw) + 2;
                if (bc - ba < PHD_ZBINS) {
                    const int fa = ba >= 0 ? ba / PHD_ZBINS : -((PHD_ZBINS - 1 - ba) / PHD_ZBINS);
                    const int fc = bc >= 0 ? bc / PHD_ZBINS : -((PHD_ZBINS - 1 - bc) / PHD_ZBINS);
                    const int ia = s_zbin[ba - fa * PHD_ZBINS] + fa * Mv;
                    const int ic = s_zbin[bc - fc * PHD_ZBINS] + fc * Mv;
                    t.lo = ia - fa * Mv;
                    t.cnt = min(ic - ia, Mv);
                }
            }
        }
    }
    return cls;
}

/* One chunk's balanced pair walk (the (component, window entry) pairs,
 * component-major, cut into 64 equal contiguous ranges; lane L walks range L
 * with the component terms read from the compact chunk table).  SUM: the
 * eta pass (fixed-point atomics; listing against thr0), else the listing pass
 * against the exact per-measurement bounds.  The steps are branch-free
 * (selects, atomics that may add 0, a dummy key slot) and both passes are
 * compile-time, so a batch of eight steps is one scheduling region and their
 * LDS round trips overlap. */
struct WalkArgs {
    float4* s_wta;
    float4* s_wtb;
    unsigned char* s_wst;
    const float4* s_zs;
    const float* s_thr;
    u64* s_ehi;
    u64* s_elo;
    unsigned int* s_skey;
    int Mv, Scap, base, P;
    float k2, thr0, lo_scale;
};

template <bool SUM, bool ZW>
__device__ __forceinline__ void walk_chunk(const WalkArgs& w, const WComp& t, int cnt, int incl, int& nlist,
                                           int& flags, unsigned long long* dbg) {
#ifdef PHD_STAMPS
    unsigned long long tq0 = __builtin_amdgcn_s_memtime();
#endif
    const int lane = threadIdx.x;
    const int P = w.P, Mv = w.Mv;
    const int pre = incl - cnt;
    const int per = (P + 63) >> 6;
    // compact table of the components with pairs, in component order
    int nnz;
    const int ci = wrank(cnt > 0, &nnz);
    if (cnt > 0) {
        w.s_wta[ci] = make_float4(t.r, t.b, t.S0, t.S12);
        w.s_wtb[ci] = make_float4(t.S3, t.C2, __int_as_float(t.lo | (cnt << 8) | (lane << 17)), __int_as_float(pre));
        const int t0 = (pre + per - 1) / per, t1 = min((pre + cnt + per - 1) / per, 64);
        for (int tt = t0; tt < t1; tt++) w.s_wst[tt] = (unsigned char)ci;
    }
    wsync();
    const int p0 = lane * per, p1 = max(min(p0 + per, P), p0);  // empty past P
    // the lane's range spans components j0, j0+1, j0+2 (else: the generic tail below)
    const int j0 = p0 < P ? w.s_wst[lane] : 0;
    auto end_of = [&](int j) {
        if (j >= nnz) return P;
        const float4 b = w.s_wtb[j];
        return __float_as_int(b.w) + ((__float_as_int(b.z) >> 8) & 511);
    };
    // the terms of j0, j0+1, j0+2 in registers: a step selects among them
    const float4 TA0 = w.s_wta[j0], TB0 = w.s_wtb[j0];
    const float4 TA1 = w.s_wta[min(j0 + 1, 63)], TB1 = w.s_wtb[min(j0 + 1, 63)];
    const float4 TA2 = w.s_wta[min(j0 + 2, 63)], TB2 = w.s_wtb[min(j0 + 2, 63)];
    auto tend = [&](int i, const float4& tb) {
        return j0 + i < nnz ? __float_as_int(tb.w) + ((__float_as_int(tb.z) >> 8) & 511) : P;
    };
    auto sel3 = [](int k, const float4& x0, const float4& x1, const float4& x2) {
        return make_float4(k == 0 ? x0.x : k == 1 ? x1.x : x2.x, k == 0 ? x0.y : k == 1 ? x1.y : x2.y,
                           k == 0 ? x0.z : k == 1 ? x1.z : x2.z, k == 0 ? x0.w : k == 1 ? x1.w : x2.w);
    };
    const int e0 = tend(0, TB0), e1 = tend(1, TB1), e2 = tend(2, TB2);
#ifdef PHD_STAMPS
    {
        const unsigned long long tq1 = __builtin_amdgcn_s_memtime();
        dbg[0] += tq1 - tq0;
        tq0 = tq1;
    }
#endif
    const int pend = max(min(p1, e2), p0);
    struct Step {
        u64 y;
        int a;  // eta word (hi / lo array offset, measurement)
        bool lst;
        unsigned key;
    };
    // the arithmetic of a step from its terms and measurement
    auto math = [&](bool act, const float4& ta, const float4& tb, const float4& z) -> Step {
        const int zi = __float_as_int(tb.z);
        const float i0 = z.x - ta.x;
        float i1 = z.y - ta.y;
        i1 = ZW ? d_wrap(i1) : wrap_small(i1);
        const float u = __builtin_fmaf(i0, ta.z, i1 * ta.w);
        const float dist = __builtin_fmaf(i0, u, i1 * i1 * tb.x);
        const float l2q = __builtin_fmaf(-w.k2, dist, tb.y);
        const int m = __float_as_int(z.z);
        Step st;
        st.key = ((unsigned int)m << 16) | (unsigned int)(w.base + (zi >> 17));
        if (SUM) {
            const float q = act ? __builtin_amdgcn_exp2f(l2q) : 0.f;
            flags |= q >= 1048576.f ? PHD_ST_ETA_RANGE : 0;
            const bool hi = q >= 7.62939453125e-06f;  // 2^-17 (eta_add, without its branch)
            st.y = (u64)(fminf(q, 4194304.f) * (hi ? 1099511627776.f : w.lo_scale));
            st.a = hi ? m : m + 256;
            st.lst = act && l2q >= w.thr0;
        } else {
            st.y = 0;
            st.a = 0;
            st.lst = act && l2q >= w.s_thr[m];
        }
#if defined(PHD_EXPERIMENT) && (PHD_EXPERIMENT == 22 || PHD_EXPERIMENT == 23)
        st.lst = false;
#endif
        return st;
    };
    auto commit = [&](const Step& st) {
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 17
        if (SUM && st.y == 0xffffffffffffffffull) atomicAdd(w.s_ehi + st.a, st.y);
#else
        if (SUM) atomicAdd(w.s_ehi + st.a, st.y);  // may add 0; s_elo = s_ehi + 256
#endif
        int tot;
        const int r = wrank(st.lst, &tot);
        const int slot = (st.lst && nlist + r < w.Scap) ? nlist + r : w.Scap;  // Scap: dummy slot
        w.s_skey[slot] = st.key;
        nlist += tot;
    };
    auto msof = [&](int pp, const float4& tb) {
        const int ms = (__float_as_int(tb.z) & 255) + (pp - __float_as_int(tb.w));
        return ms >= Mv ? ms - Mv : ms;
    };
    /* batches of eight steps: the measurement reads of all eight are issued
     * before the arithmetic, the atomics and key writes after it (a wave's
     * LDS operations complete in order) */
    const int nmain = wave_max_i(pend - p0);
    for (int s0 = 0; s0 < nmain; s0 += 8) {
        int sel[8], zi[8];
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const int pp = p0 + s0 + h;
            sel[h] = (pp >= e0) + (pp >= e1);
            zi[h] = pp < pend ? msof(pp, sel3(sel[h], TB0, TB1, TB2)) : 0;
        }
        float4 zv[8];
#pragma unroll
        for (int h = 0; h < 8; h++) zv[h] = w.s_zs[zi[h]];
        Step st[8];
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const int pp = p0 + s0 + h;
            st[h] = math(pp < pend, sel3(sel[h], TA0, TA1, TA2), sel3(sel[h], TB0, TB1, TB2), zv[h]);
        }
#pragma unroll
        for (int h = 0; h < 8; h++) commit(st[h]);
    }
#ifdef PHD_STAMPS
    {
        wsync();
        const unsigned long long tq1 = __builtin_amdgcn_s_memtime();
        dbg[1] += tq1 - tq0;
        tq0 = tq1;
    }
#endif
    if (__ballot(p1 > pend) != 0ull) {  // ranges over more than three components
        int j = j0 + 2;
        const int ntail = wave_max_i(max(p1 - pend, 0));
        for (int s1 = 0; s1 < ntail; s1++) {
            const int pp = pend + s1;
            const bool act = pp < p1;
            while (act && pp >= end_of(j)) j++;
            const int jj = act ? min(j, 63) : 0;
            const float4 ta = w.s_wta[jj], tb = w.s_wtb[jj];
            const float4 z = w.s_zs[act ? msof(pp, tb) : 0];
            commit(math(act, ta, tb, z));
        }
    }
    wsync();  // the chunk table is rewritten by the next chunk
#ifdef PHD_STAMPS
    dbg[2] += __builtin_amdgcn_s_memtime() - tq0;
#endif
}

/* Three-launch workgroup CPHD update, middle launch: the CPHD terms of one
 * particle by one wave (cphd_terms_one) from part A's handoff. */
__global__ void __launch_bounds__(64) k_cphd_terms(UpdateArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cphd_terms_one(a, upd_particle(a, (int)blockIdx.x, (int)gridDim.x), (double*)smem);
}

/* ------------------------------------------------------------- merge, one wave */

/* candidate covariance: detection / birth candidates keep theirs in LDS
 * (tag bit 15), prior-derived ones (non-detect, near) read the prior slab */
struct WCand {
    float4* P;
    unsigned short* tag;
    float4* detv;
    const G1 float* src;
    int cap;
    __device__ __forceinline__ float4 V(int i) const {
        const unsigned t = tag[i];
        if (t & 0x8000u) return detv[t & 0x7fffu];
        return make_float4(src[3 * cap + t], src[4 * cap + t], src[5 * cap + t], src[6 * cap + t]);
    }
};

__device__ __forceinline__ void w_emit(G1 float* dst, int cap, int slot, float W, float gx, float gy, const double* cv) {
    if (slot >= cap) return;
    float p0 = (float)cv[0] / W, p1 = (float)cv[1] / W, p2 = (float)cv[2] / W, p3 = (float)cv[3] / W;
    p1 = (p1 + p2) / 2;  // force_symmetric_covariance (device_math.cuh:710-725)
    p2 = p1;
    dst[slot] = W;
    dst[1 * cap + slot] = gx;
    dst[2 * cap + slot] = gy;
    dst[3 * cap + slot] = p0;
    dst[4 * cap + slot] = p1;
    dst[5 * cap + slot] = p2;
    dst[6 * cap + slot] = p3;
}

/* serial greedy (phdUpdateMergeKernel :2739-2890), one selection per round;
 * the exact fallback of the parallel form.  flag: 2 B per candidate. */
__device__ __noinline__ int w_merge_serial(WCand C, int K, short* flag, float T, G1 float* dst, int cap) {
    const int lane = threadIdx.x;
    for (int i = lane; i < K; i += 64) flag[i] = 0;
    wsync();
    int nout = 0;
    while (true) {
        float bw = -INFINITY;
        int bi = -1;
        for (int i = lane; i < K; i += 64) {
            const float w = C.P[i].z;
            if (flag[i] == 0 && (bi < 0 || earlier(w, i, bw, bi))) {
                bw = w;
                bi = i;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ow = __shfl_xor(bw, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oi >= 0 && (bi < 0 || earlier(ow, oi, bw, bi))) {
                bw = ow;
                bi = oi;
            }
        }
        bi = uni_i(bi);
        if (bi < 0) break;
        const float4 bp = C.P[bi], bv = C.V(bi);
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
        for (int i = lane; i < K; i += 64) {
            if (flag[i] != 0) continue;
            const float4 p = C.P[i];
            if (cand_mahal(bp, bv, p, C.V(i)) < T) {
                flag[i] = 2;
                acc0 += (double)p.z;
                acc1 += (double)(p.z * p.x);
                acc2 += (double)(p.z * p.y);
            }
        }
        acc0 = wave_sum_dx(acc0);
        acc1 = wave_sum_dx(acc1);
        acc2 = wave_sum_dx(acc2);
        const float W = (float)acc0;
        if (W == 0.f) break;
        const float gx = (float)acc1 / W, gy = (float)acc2 / W;
        double cv[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = lane; i < K; i += 64) {
            if (flag[i] != 2) continue;
            const float4 p = C.P[i], v = C.V(i);
            const float d0 = gx - p.x, d1 = gy - p.y;
            cv[0] += (double)(p.z * (v.x + d0 * d0));
            cv[1] += (double)(p.z * (v.y + d0 * d1));
            cv[2] += (double)(p.z * (v.z + d1 * d0));
            cv[3] += (double)(p.z * (v.w + d1 * d1));
            flag[i] = 1;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) cv[k] = wave_sum_dx(cv[k]);
        if (lane == 0) w_emit(dst, cap, nout, W, gx, gy, cv);
        nout++;
        wsync();
    }
    return nout;
}

struct WMerge {
    WCand C;
    unsigned short* key;     // cell-order position -> candidate
    unsigned short* gstart;  // B + 2 bucket ends / starts
    unsigned int* plist;     // culled pairs
    int plcap;
    unsigned int* edges;     // Epool undirected edges (i << 16 | j)
    unsigned short* cur;     // degrees / scatter cursors (16-bit halves of 32-bit atomics)
    unsigned short* off;     // CSR offsets (K + 1)
    unsigned short* pool;    // 2 Epool adjacency entries
    short* par;              // -2 seed, -1 undecided, >= 0 absorbed by
};

/* Neighbourhood walk (as merge_walk of phd_kernels.hip, for one wave). */
template <class F>
__device__ __forceinline__ void w_merge_walk(const WMerge& X, int K, int Knw, int B, int Px, int Py, int lgPx,
                                             float invR, float thr, F&& on_pair) {
    const int lane = threadIdx.x;
    for (int q0 = 0; q0 < K; q0 += 64) {  // wave-uniform trip counts: on_pair may use ballots
        const int q = q0 + lane;
        const bool vq = q < K;
        const int i = vq ? X.key[q] : 0;
        const float4 p = X.C.P[i];
        int lo0 = q + 1, hi0 = vq ? K : 0, lo1 = 0, hi1 = 0, lo2 = 0, hi2 = 0, lo3 = 0, hi3 = 0, lo4 = 0, hi4 = 0,
            lo5 = 0, hi5 = 0, lo6 = 0, hi6 = 0;
        const bool wild = q >= Knw;
        if (vq && !wild) {
            const int cx = (int)floorf(fminf(fmaxf(p.x * invR, -8192.f), 8192.f));
            const int cy = (int)floorf(fminf(fmaxf(p.y * invR, -8192.f), 8192.f));
            const int cxm = cx & (Px - 1);
            lo0 = max(Knw, q + 1);
#define PHD_ROW(DY, LOA, HIA, LOB, HIB)                                           \
    {                                                                             \
        const int rb = ((cy + (DY)) & (Py - 1)) << lgPx;                         \
        const int ca = cxm == 0 ? 0 : cxm - 1, cb = cxm == Px - 1 ? Px : cxm + 2; \
        LOA = X.gstart[rb + ca];                                                  \
        HIA = (rb + cb < B) ? X.gstart[rb + cb] : Knw;                            \
        if (cxm == 0 || cxm == Px - 1) {                                          \
            const int cw = cxm == 0 ? Px - 1 : 0;                                 \
            LOB = X.gstart[rb + cw];                                              \
            HIB = (rb + cw + 1 < B) ? X.gstart[rb + cw + 1] : Knw;                \
        }                                                                         \
        LOA = max(LOA, q + 1);                                                    \
        LOB = max(LOB, q + 1);                                                    \
    }
            PHD_ROW(-1, lo1, hi1, lo2, hi2)
            PHD_ROW(0, lo3, hi3, lo4, hi4)
            PHD_ROW(1, lo5, hi5, lo6, hi6)
#undef PHD_ROW
        }
        const int n0 = max(hi0 - lo0, 0), n1 = max(hi1 - lo1, 0), n2 = max(hi2 - lo2, 0), n3 = max(hi3 - lo3, 0),
                  n4 = max(hi4 - lo4, 0), n5 = max(hi5 - lo5, 0), n6 = max(hi6 - lo6, 0);
        const int e1 = n1, e2 = e1 + n2, e3 = e2 + n3, e4 = e3 + n4, e5 = e4 + n5, e6 = e5 + n6, e0 = e6 + n0;
        const int g1 = (lo2 - e1) - lo1, g2 = (lo3 - e2) - (lo2 - e1), g3 = (lo4 - e3) - (lo3 - e2),
                  g4 = (lo5 - e4) - (lo4 - e3), g5 = (lo6 - e5) - (lo5 - e4), g6 = (lo0 - e6) - (lo6 - e5);
        auto at = [&](int t) {
            return t + lo1 + (t >= e1 ? g1 : 0) + (t >= e2 ? g2 : 0) + (t >= e3 ? g3 : 0) + (t >= e4 ? g4 : 0) +
                   (t >= e5 ? g5 : 0) + (t >= e6 ? g6 : 0);
        };
        const int emax = wave_max_i(e0);
        for (int t = 0; t < emax; t += 4) {
            int jj[4];
            float4 pp[4];
#pragma unroll
            for (int k = 0; k < 4; k++) jj[k] = (t + k < e0) ? X.key[at(t + k)] : i;
#pragma unroll
            for (int k = 0; k < 4; k++) pp[k] = X.C.P[jj[k]];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                bool test = t + k < e0;
                if (!wild && pp[k].w >= 0.f) {
                    const float dx = pp[k].x - p.x, dy = pp[k].y - p.y;
                    test = test && !(dx * dx + dy * dy > thr * (p.w + pp[k].w));
                }
                on_pair(test, i, jj[k]);
            }
        }
    }
}

/* Parallel exact greedy merge for one wave (merge_parallel of phd_kernels.hip:
 * lattice-culled candidate pairs, exact distances, CSR, lexicographically-first
 * MIS by priority, emission in candidate-index order of the seeds with the
 * members summed in candidate-index order).  Returns nout, or -1 when the
 * particle needs the serial greedy. */
#ifdef PHD_STAMPS
#define MSTAMP(k)                                                        \
    do {                                                                 \
        if (lane == 0 && stp) stp[(k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define MSTAMP(k) \
    do {          \
    } while (0)
#endif
__device__ __forceinline__ int w_merge_parallel(const WMerge& X, int K, float T, G1 float* dst, int cap, int Epool, int B, int* s_misc,
                                int screen_bad, float screen_lmax, unsigned long long* stp) {
    const int lane = threadIdx.x;
    const int lgPx = B >= 4096 ? 6 : 5, lgPy = (B >= 4096 ? 12 : B >= 1024 ? 10 : 9) - lgPx;
    const int Px = 1 << lgPx, Py = 1 << lgPy;
    const bool bad = __ballot(screen_bad != 0) != 0ull;
    if (bad) return -1;
    const float lmax = wave_max_fu(screen_lmax);
    if (!(lmax < INFINITY)) return -1;
    const float R = sqrtf(1.05f * T * lmax);
    const float invR = (lmax > 0.f) ? 1.0f / (R * 1.001f) : 0.f;
    // M2: counting sort of the binned candidates by bucket; wild ones last
    for (int b = lane; b < B + 2; b += 64) X.gstart[b] = 0;
    wsync();
    int far = 0, nwild = 0;
    for (int i0 = 0; i0 < K; i0 += 64) {
        const int i = i0 + lane;
        const float4 p = X.C.P[i < K ? i : 0];
        const bool wildc = i < K && p.w < 0.f;
        int tot;
        const int r = wrank(wildc, &tot);
        if (wildc) X.key[K - 1 - (nwild + r)] = (unsigned short)i;
        nwild += tot;
        if (i < K && !wildc) {
            far |= !(fabsf(p.x * invR) < 8192.f && fabsf(p.y * invR) < 8192.f);
            const unsigned int bkt = lattice_bucket(p.x, p.y, invR, Px, Py, lgPx);
            atomicAdd((unsigned int*)(X.gstart + (bkt & ~1u)), (bkt & 1u) ? 0x10000u : 1u);
        }
    }
    if (__ballot(far != 0) != 0ull) return -1;
    wsync();
    MSTAMP(11);
    const int Knw = K - nwild;
    {  // inclusive scan over B counters: gstart[b] = end of bucket b
        const int per = B / 64;
        const int base = lane * per;
        int sum = 0;
        for (int q = 0; q < per; q++) sum += X.gstart[base + q];
        int pre = wave_incl_scan(sum) - sum;
        for (int q = 0; q < per; q++) {
            pre += X.gstart[base + q];
            X.gstart[base + q] = (unsigned short)pre;
        }
    }
    wsync();
    for (int i = lane; i < K; i += 64) {
        const float4 p = X.C.P[i];
        if (p.w < 0.f) continue;
        const unsigned int bkt = lattice_bucket(p.x, p.y, invR, Px, Py, lgPx);
        const unsigned int old = atomicSub((unsigned int*)(X.gstart + (bkt & ~1u)), (bkt & 1u) ? 0x10000u : 1u);
        X.key[((bkt & 1u) ? (int)(old >> 16) : (int)(old & 0xffffu)) - 1] = (unsigned short)i;
    }
    for (int i = lane; i < K + 2; i += 64) X.cur[i] = 0;
    if (lane == 0) X.gstart[B] = (unsigned short)Knw;
    wsync();
    MSTAMP(12);
    // M3: culled pairs, then exact distances -> edges + degrees
    const float thr = 1.05f * T * 0.5f;
    const int plcap = X.plcap;
    int npairs = 0, E = 0;  // wave-uniform counters (ballot compaction)
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 26
    if (K > 100000)
#endif
    if (plcap > 0)  // culled pairs listed, exact distances densely after; else tested in place
    w_merge_walk(X, K, Knw, B, Px, Py, lgPx, invR, thr, [&](bool test, int i, int j) {
        int tot;
        const int r = wrank(test, &tot);
        if (test && npairs + r < plcap) X.plist[npairs + r] = ((unsigned int)i << 16) | (unsigned int)j;
        npairs += tot;
    });
    wsync();
    MSTAMP(23);
    if (plcap > 0 && npairs <= plcap) {
        for (int e0 = 0; e0 < npairs; e0 += 64) {
            const int e = e0 + lane;
            const unsigned int pr = X.plist[e < npairs ? e : 0];
            const int i = (int)(pr >> 16), j = (int)(pr & 0xffffu);
            const bool ok = e < npairs && cand_mahal(X.C.P[i], X.C.V(i), X.C.P[j], X.C.V(j)) < T;
            int tot;
            const int r = wrank(ok, &tot);
            if (ok) {
                if (E + r < Epool) X.edges[E + r] = pr;
                cnt16_inc(X.cur, i);
                cnt16_inc(X.cur, j);
            }
            E += tot;
        }
    } else {
        w_merge_walk(X, K, Knw, B, Px, Py, lgPx, invR, thr, [&](bool test, int i, int j) {
            const bool ok = test && cand_mahal(X.C.P[i], X.C.V(i), X.C.P[j], X.C.V(j)) < T;
            int tot;
            const int r = wrank(ok, &tot);
            if (ok) {
                if (E + r < Epool) X.edges[E + r] = ((unsigned int)i << 16) | (unsigned int)j;
                cnt16_inc(X.cur, i);
                cnt16_inc(X.cur, j);
            }
            E += tot;
        });
    }
    wsync();
    MSTAMP(13);
#ifdef PHD_STAMPS
    if (lane == 0 && stp) stp[24] = ((unsigned long long)npairs << 32) | (unsigned)E;
#endif
    if (E > Epool) return -1;
    // M4: CSR over candidate index (off = exclusive scan of degrees); R1's early
    // form (keys, buckets, pairs) is dead from here on
    {
        int running = 0;
        for (int base = 0; base < K; base += 64) {
            const int i = base + lane;
            const int cdeg = (i < K) ? X.cur[i] : 0;
            const int incl = wave_incl_scan(cdeg);
            const int pre = incl - cdeg;
            if (i < K) {
                X.off[i] = (unsigned short)(running + pre);
                X.cur[i] = (unsigned short)(running + pre + cdeg);
                X.par[i] = (short)(cdeg == 0 ? -2 : -1);
            }
            running += __builtin_amdgcn_readlane(incl, 63);
        }
        if (lane == 0) X.off[K] = (unsigned short)running;
    }
    wsync();
    for (int e = lane; e < E; e += 64) {
        const unsigned int ed = X.edges[e];
        const int i = (int)(ed >> 16), j = (int)(ed & 0xffffu);
        X.pool[cnt16_dec(X.cur, i)] = (unsigned short)j;
        X.pool[cnt16_dec(X.cur, j)] = (unsigned short)i;
    }
    wsync();
    // active (non-isolated) candidates, in index order, into the dead edge list
    unsigned short* alist = (unsigned short*)X.edges;
    int nact = 0;
    for (int base = 0; base < K; base += 64) {
        const int i = base + lane;
        const bool act = i < K && X.off[i + 1] > X.off[i];
        int tot;
        const int r = wrank(act, &tot);
        if (act) alist[nact + r] = (unsigned short)i;
        nact += tot;
    }
    wsync();
    MSTAMP(19);
    // M5: lexicographically-first MIS by priority, asynchronous polling rounds
    int failed = 0;
#define PHD_CONSIDER(E_, WE, ST)                                                    \
    {                                                                               \
        const int e_ = (E_);                                                        \
        const float we_ = (WE);                                                     \
        const int st_ = (ST);                                                       \
        if (earlier(we_, e_, wi, i)) {                                              \
            const bool s_better = st_ == -2 && (bs < 0 || earlier(we_, e_, ws, bs)); \
            const bool u_better = st_ == -1 && (bu < 0 || earlier(we_, e_, wu, bu)); \
            ws = s_better ? we_ : ws;                                               \
            bs = s_better ? e_ : bs;                                                \
            wu = u_better ? we_ : wu;                                               \
            bu = u_better ? e_ : bu;                                                \
        }                                                                           \
    }
    {
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 27
        bool pending = false;
#else
        bool pending = true;
#endif
        int sweeps = 0;
        while (__ballot(pending) != 0ull) {
            if (++sweeps > (1 << 16)) {
                failed = 1;
                break;
            }
            pending = false;
            for (int a0 = lane; a0 < nact; a0 += 64) {
                const int i = alist[a0];
                if (__hip_atomic_load(X.par + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != -1) continue;
                const int o = X.off[i], nd = X.off[i + 1] - o;
                const float wi = X.C.P[i].z;
                float ws = 0.f, wu = 0.f;
                int bs = -1, bu = -1;
                for (int r = 0; r < nd; r++) {
                    const int e = X.pool[o + r];
                    PHD_CONSIDER(e, X.C.P[e].z,
                                 __hip_atomic_load(X.par + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                }
                const bool wait = bu >= 0 && (bs < 0 || earlier(wu, bu, ws, bs));
                if (!wait)
                    __hip_atomic_store(X.par + i, (short)(bs >= 0 ? bs : -2), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                pending |= wait;
            }
            wsync();  // this sweep's decisions before the next sweep's polls (one wave: LDS in order)
        }
    }
#undef PHD_CONSIDER
    wsync();
    MSTAMP(20);
    if (failed) return -1;
    // M6: seeds emit in candidate-index order; isolated seeds directly, seeds
    // with neighbours listed and emitted densely (members in index order)
    unsigned int* slist = (unsigned int*)X.edges;  // (seed << 16 | slot); alist is dead
    int nout = 0, nclu = 0;
    for (int base = 0; base < K; base += 64) {
        const int i = base + lane;
        const bool seed = (i < K) && X.par[i] == -2;
        int tot;
        const int slot = nout + wrank(seed, &tot);
        const bool clustered = seed && X.off[i + 1] > X.off[i];
        int ctot;
        const int cr = wrank(clustered, &ctot);
        if (clustered) {
            slist[nclu + cr] = ((unsigned int)i << 16) | (unsigned int)min(slot, 65535);
        } else if (seed && slot < cap) {
            const float4 ps = X.C.P[i], vs = X.C.V(i);
            const float W = ps.z;
            const float gx = (W * ps.x) / W, gy = (W * ps.y) / W;
            const float d0 = gx - ps.x, d1 = gy - ps.y;
            float p0 = (W * (vs.x + d0 * d0)) / W, p1 = (W * (vs.y + d0 * d1)) / W;
            float p2 = (W * (vs.z + d1 * d0)) / W, p3 = (W * (vs.w + d1 * d1)) / W;
            p1 = (p1 + p2) / 2;  // force_symmetric_covariance
            dst[slot] = W;
            dst[1 * cap + slot] = gx;
            dst[2 * cap + slot] = gy;
            dst[3 * cap + slot] = p0;
            dst[4 * cap + slot] = p1;
            dst[5 * cap + slot] = p1;
            dst[6 * cap + slot] = p3;
        }
        nout += tot;
        nclu += ctot;
    }
    wsync();
    for (int c2 = lane; c2 < nclu; c2 += 64) {
        const int i = (int)(slist[c2] >> 16), slot = (int)(slist[c2] & 0xffffu);
        if (slot >= cap) continue;
        const int o = X.off[i], nd = X.off[i + 1] - o;
        const bool reg = nd <= MERGE_DEG_REG;
        int mb[MERGE_DEG_REG];
#pragma unroll
        for (int k = 0; k < MERGE_DEG_REG; k++) mb[k] = (reg && k < nd) ? X.pool[o + k] : i;
#pragma unroll
        for (int k = 0; k < MERGE_DEG_REG; k++) mb[k] = (mb[k] != i && X.par[mb[k]] == i) ? mb[k] : INT_MAX;
        auto next_member = [&](int last) {
            int nx = i > last ? i : INT_MAX;
            if (reg) {
#pragma unroll
                for (int k = 0; k < MERGE_DEG_REG; k++) nx = (mb[k] > last && mb[k] < nx) ? mb[k] : nx;
            } else {
                for (int r = 0; r < nd; r++) {
                    const int j = X.pool[o + r];
                    if (j > last && j < nx && X.par[j] == i) nx = j;
                }
            }
            return nx;
        };
        double W = 0.0, sx = 0.0, sy = 0.0;
        for (int j = next_member(-1); j != INT_MAX; j = next_member(j)) {
            const float4 pj = X.C.P[j];
            W += (double)pj.z;
            sx += (double)(pj.z * pj.x);
            sy += (double)(pj.z * pj.y);
        }
        const float Wf = (float)W;
        const float gx = (float)sx / Wf, gy = (float)sy / Wf;
        double cv[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = next_member(-1); j != INT_MAX; j = next_member(j)) {
            const float4 pj = X.C.P[j], vj = X.C.V(j);
            const float d0 = gx - pj.x, d1 = gy - pj.y, w = pj.z;
            cv[0] += (double)(w * (vj.x + d0 * d0));
            cv[1] += (double)(w * (vj.y + d0 * d1));
            cv[2] += (double)(w * (vj.z + d1 * d0));
            cv[3] += (double)(w * (vj.w + d1 * d1));
        }
        w_emit(dst, cap, slot, Wf, gx, gy, cv);
    }
    return nout;
}

/* ------------------------------------------------------------ the update */

template <bool CPHD>
__device__ __forceinline__ void wave_update(const UpdateArgs& a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const WaveLds L = wave_lds_layout(a.cap, a.Mcap, a.Kcap, a.Scap, a.Epool, CPHD ? 1 : 0);
    float* s_zr = (float*)(smem + L.zr);
    float* s_zb = (float*)(smem + L.zb);
    int* s_zok = (int*)(smem + L.zok);
    float* s_leta = (float*)(smem + L.leta);
    float* s_thr = (float*)(smem + L.thr);
    unsigned char* s_cls = smem + L.cls;
    int* s_misc = (int*)(smem + L.misc);  // [0..7] merge, [8] survivors, [9] flags
    float4* s_zs = (float4*)(smem + L.zs);
    unsigned short* s_zbin = (unsigned short*)(smem + L.zbin);
    u64* s_ehi = (u64*)(smem + L.ehi);
    u64* s_elo = (u64*)(smem + L.elo);
    unsigned int* s_skey = (unsigned int*)(smem + L.skey);
    unsigned int* s_skey2 = (unsigned int*)(smem + L.skey2);

    const int lane = threadIdx.x;
    const int n = a.slots ? a.slots[blockIdx.x] : a.first + (int)blockIdx.x;
    const DevCfg& c = a.c;
    const int M = a.M, Mv = a.Mv, cap = a.cap;
    const bool zwide = a.zwide != 0;  // some |measurement bearing| >= 3: the general wrapAngle
    const int sref = uni_i(a.src ? g1(a.src)[n] : n);
    const bool in_x = (sref & PHD_SLAB_X) != 0;
    const int slab = sref & PHD_SLAB_MASK;
    const int G = uni_i(in_x ? g1(a.size_x)[slab] : g1(a.size_in)[slab]);
    const G1 float* __restrict__ src = g1(uni_p((in_x ? a.map_x : a.map_in) + (size_t)slab * NF * cap));
    G1 float* __restrict__ dst = g1(uni_p(a.map_out + (size_t)n * NF * cap));
    // first chunk of the prior, issued before anything waits
    float pv[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) pv[f] = lane < G ? src[f * cap + lane] : 0.f;
    // replay restore + fused predict (every lane computes the same pose)
    phd_pose pose;
    {  // fields through a global float view (a struct copy would need a generic pointer)
        const G1 float* pp = g1((const float*)(a.pose_prior ? a.pose_prior : a.poses) + (size_t)n * 6);
        pose.px = pp[0];
        pose.py = pp[1];
        pose.ptheta = pp[2];
        pose.vx = pp[3];
        pose.vy = pp[4];
        pose.vtheta = pp[5];
    }
    const float logw0 = a.logw_prior ? g1(a.logw_prior)[n] : g1(a.logw)[n];
    if (a.predict) {
        for (int k = 0; k < a.pc.subdivide; k++) {
            const uint64_t st = a.pstep * (uint64_t)a.pc.subdivide + (uint64_t)k;
            if (a.predict == 1) {
                float n_alpha, n_enc;
                ackerman_noise(a.pseed, a.pc.index_offset + n, st, a.pc, &n_alpha, &n_enc);
                pose = predict_ackerman_one(pose, a.pu, n_alpha, n_enc, a.pc);
            } else {
                pose = predict_cv_one(pose, cv_noise(a.pseed, a.pc.index_offset + n, st, a.pc), a.pc);
            }
        }
    }
    pose.px = uni_f(pose.px);
    pose.py = uni_f(pose.py);
    pose.ptheta = uni_f(pose.ptheta);
    if (a.predict && lane == 0) {
        G1 float* pp = g1((float*)a.poses + (size_t)n * 6);
        pp[0] = pose.px;
        pp[1] = pose.py;
        pp[2] = pose.ptheta;
        pp[3] = pose.vx;
        pp[4] = pose.vy;
        pp[5] = pose.vtheta;
    }
    for (int m = lane; m < M; m += 64) {
        s_zr[m] = g1(a.zr)[m];
        s_zb[m] = g1(a.zb)[m];
        s_zok[m] = g1(a.zok)[m];
        s_ehi[m] = 0ull;
        s_elo[m] = 0ull;
    }
    for (int m = lane; m < Mv; m += 64) {
        const G1 float* zf = g1((const float*)a.zs + 4 * (size_t)m);
        s_zs[m] = make_float4(zf[0], zf[1], zf[2], zf[3]);
    }
    for (int b = lane; b < PHD_ZBINS; b += 64) s_zbin[b] = g1(a.zbin)[b];
    if (lane < 16) s_misc[8 + lane] = 0;
    wsync();
    WSTAMP(0);

    /* Phases 1+3: chunks of 64 prior components; lane = component. */
    const float k2 = 0.72134752044448170f;
    int flags = 0;
    double card_d = 0.0, win_d = 0.0, qd_d = 0.0, wall_d = 0.0;
    int gin = 0;  // in-range components (per lane, reduced after the pass)
#ifdef PHD_STAMPS
    unsigned long long dbg_cls = 0, dbg_walk = 0, dbg_iter = 0, dbg_pairs = 0;
#endif
    unsigned long long dbgw[3] = {0, 0, 0};  // walk: table+terms, main batches, tail (diagnostic build)
    const float thr0 = CPHD ? c.cphd_thr0 : c.lq_keep_thresh * 1.4426950408889634f;
    // eta fixed point: lo scale 2^70 up to 2047 components per map (headroom), 2^60 above
    const float lo_scale = cap <= 2047 ? 1.1805916207174113e21f : 1.152921504606846976e18f;
    const double lo_unscale = cap <= 2047 ? 8.470329472543003e-22 : 8.673617379884035e-19;
    float4* s_wta = (float4*)(smem + L.wtab);          // chunk table: r, b, S0, S12
    float4* s_wtb = s_wta + 64;                         // S3, C2, lo | cnt << 16, first pair
    unsigned char* s_wst = (unsigned char*)(s_wtb + 64);  // first component of each lane's pair range
    int npass = 1;
    int nlist = 0;  // listed detection terms (wave-uniform)
    float lb = c.walk_floor;  // log2 bound of the bearing windows (<= WALK_LOG2_FLOOR, thr0 - 1)
    for (int pass = 0; pass < npass; pass++) {
        const bool sum_pass = pass == 0;
        nlist = 0;
        if (pass == 1) {  // exact per-measurement bounds: the windows must reach the lowest
            float tm = INFINITY;
            for (int m = lane; m < M; m += 64) tm = fminf(tm, s_thr[m]);
            lb = fminf(lb, -wave_max_fu(-tm) - 1.f);
        }
        for (int base = 0; base < G; base += 64) {
            const int k = base + lane;
            float v[NF];
            if (sum_pass) {  // this chunk was loaded one iteration ago; issue the next
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = pv[f];
                if (base + 64 < G) {
#pragma unroll
                    for (int f = 0; f < NF; f++) pv[f] = k + 64 < G ? src[f * cap + k + 64] : 0.f;
                }
            } else {
#pragma unroll
                for (int f = 0; f < NF; f++) v[f] = k < G ? src[f * cap + k] : 0.f;
            }
#ifdef PHD_STAMPS
            const unsigned long long tA = __builtin_amdgcn_s_memtime();
#endif
            WComp t;
            int cls = 0;
            t.cnt = 0;
            t.lo = 0;
            if (k < G) {
                float pdw;
                cls = classify_comp(c, pose, v, Mv, s_zbin, lb, t, pdw);
                if (sum_pass) {
                    s_cls[k] = (unsigned char)cls;
                    gin += cls == 1;
                    if (CPHD) wall_d += (double)v[0];
                    if (cls == 1) {
                        card_d += (double)(pdw * v[0]);
                        if (CPHD) {
                            win_d += (double)v[0];
                            qd_d += (double)(1 - pdw) * (double)v[0];
                        }
                    }
                }
            }
            /* Balanced pair walk of this chunk: the (component, window entry)
             * pairs, component-major, are cut into 64 equal contiguous ranges;
             * lane L walks range L with the component terms read from the chunk
             * table.  Eight entries per batch: their LDS reads issue together,
             * the atomics follow the arithmetic. */
            const int cnt = cls == 1 ? t.cnt : 0;
            const int incl = wave_incl_scan(cnt);
            const int P = __builtin_amdgcn_readlane(incl, 63);
#ifdef PHD_STAMPS
            const unsigned long long tB = __builtin_amdgcn_s_memtime();
            dbg_cls += tB - tA;
            dbg_pairs += P;
#endif
            if (P > 0) {
                WalkArgs wa{s_wta, s_wtb, s_wst, s_zs, s_thr, s_ehi, s_elo, s_skey, Mv, a.Scap, base, P, k2, thr0,
                            lo_scale};
                if (sum_pass) {
                    if (zwide) walk_chunk<true, true>(wa, t, cnt, incl, nlist, flags, dbgw);
                    else walk_chunk<true, false>(wa, t, cnt, incl, nlist, flags, dbgw);
                } else {
                    if (zwide) walk_chunk<false, true>(wa, t, cnt, incl, nlist, flags, dbgw);
                    else walk_chunk<false, false>(wa, t, cnt, incl, nlist, flags, dbgw);
                }
#ifdef PHD_STAMPS
                dbg_iter += (P + 63) >> 6;
#endif
            }
#ifdef PHD_STAMPS
            wsync();
            dbg_walk += __builtin_amdgcn_s_memtime() - tB;
#endif
        }
        wsync();
        if (pass == 0) {
            card_d = wave_sum_dx(card_d);
            gin = wave_sum_i(gin);
            if (CPHD) {
                win_d = wave_sum_dx(win_d);
                qd_d = wave_sum_dx(qd_d);
                wall_d = wave_sum_dx(wall_d);
            }
        }
        WSTAMP(1 + pass);
#if defined(PHD_EXPERIMENT) && (PHD_EXPERIMENT == 16 || PHD_EXPERIMENT == 17)
        return;  // timing ablation: pass 0 only (17: without the eta atomics)
#endif
        if (CPHD && pass == 0) {
            CphdOut co;
            cphd_wave(a, n, M, s_ehi, s_elo, lo_unscale, win_d, qd_d, wall_d, (double*)(smem + L.cphd), s_leta, s_thr,
                      co);
            if (lane == 0) {
                s_misc[12] = __float_as_int((float)(co.ip1 - co.ip0 + (double)c.cphd_log1mpd));  // non-detection log factor
                const float delta = (float)co.ip0;  // particle weight *= <Psi0,p> (.bak:2697)
                g1(a.delta)[n] = delta;
                g1(a.logw)[n] = logw0 + delta;
            }
            if (co.wide || nlist > a.Scap) npass = 2;  // exact per-measurement listing bounds: re-walk
        }
    }
    if (!CPHD) {
        for (int m = lane; m < M; m += 64) {
            float sum;
            if (gin > 0) {
                double sd = eta_value(s_ehi, s_elo, m, lo_unscale);
                sd += (double)c.kappa;
                sd += (double)c.birthWeight;
                sum = (float)sd;
            } else {
                sum = c.kappa + c.birthWeight;
            }
            s_leta[m] = d_safe_log(sum);
        }
        wsync();
        if (lane == 0) {
            float pw = 0.f;
            for (int m = 0; m < M; m++) pw += s_leta[m];
            const float cardp = (float)(card_d + (double)M * (double)c.birthWeight);
            const float delta = pw - cardp;
            g1(a.delta)[n] = delta;
            g1(a.logw)[n] = logw0 + delta;
        }
    }
    WSTAMP(3);
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 12
    return;  // timing ablation: pass 0 + weights only
#endif
    int nsurv = nlist;
    if (nsurv > a.Scap) {
        flags |= PHD_ST_SURVIVOR_OVERFLOW;
        nsurv = a.Scap;
    }
    // survivor keys into update-array order (m-major, then prior index): rank = count of smaller keys
    {
        const int n4 = (nsurv + 3) & ~3;
        for (int s = nsurv + lane; s < n4; s += 64) s_skey[s] = 0xffffffffu;
        wsync();
        const uint4* k4 = (const uint4*)s_skey;
        for (int s = lane; s < nsurv; s += 64) {
            const unsigned int key = s_skey[s];
            int r = 0;
            for (int q = 0; q < n4 / 4; q++) {
                const uint4 kk = k4[q];
                r += (kk.x < key) + (kk.y < key) + (kk.z < key) + (kk.w < key);
            }
            s_skey2[r] = key;
        }
        wsync();
    }
    WSTAMP(4);

    /* Phase 4: candidates [non-detect | detect | births | near]; prune. */
    WCand C;
    C.P = (float4*)(smem + L.cp);
    C.tag = (unsigned short*)(smem + L.ctag);
    C.detv = (float4*)(smem + L.detv);
    C.src = src;
    C.cap = cap;
    const float ndf = CPHD ? __int_as_float(s_misc[12]) : 0.f;
    int ncand = 0, sc_bad = 0;
    float sc_lmax = 0.f;
    const int Kcap = a.Kcap;
    // 4a non-detection terms, prior order
    for (int base = 0; base < G; base += 64) {
        const int k = base + lane;
        const bool in = k < G && s_cls[k] == 1;
        float w = 0.f;
        if (in) {
            const float w0 = src[k];
            w = CPHD ? expf(d_safe_log(w0) + ndf) : w0 * (1 - c.pd);
        }
        const bool keep = in && !(w < c.minFeatureWeight);
        int tot;
        const int r = wrank(keep, &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < Kcap) {
                const float4 v = make_float4(src[3 * cap + k], src[4 * cap + k], src[5 * cap + k], src[6 * cap + k]);
                C.P[p] = cand_record(src[1 * cap + k], src[2 * cap + k], w, v, c.minSeparation, sc_bad, sc_lmax);
                C.tag[p] = (unsigned short)k;
            }
        }
        ncand += tot;
    }
    const int nd0 = min(ncand, Kcap);  // first detection / birth candidate
    WSTAMP(5);
    // 4b detection terms (sorted keys)
    for (int base = 0; base < nsurv; base += 64) {
        const int s = base + lane;
        bool keep = false;
        float w = 0.f, mx = 0.f, my = 0.f;
        DevEkf e;
        if (s < nsurv) {
            const unsigned int key = s_skey2[s];
            const int m = (int)(key >> 16);
            const int k = (int)(key & 0xffffu);
            mx = src[1 * cap + k];
            my = src[2 * cap + k];
            const float w0 = src[k];
            d_compute_ekf(c, pose.px, pose.py, pose.ptheta, mx, my, src[3 * cap + k], src[4 * cap + k],
                          src[5 * cap + k], src[6 * cap + k], e);
            const float i0 = s_zr[m] - e.r;
            const float i1 = d_wrap(s_zb[m] - e.bearing);
            const float dist = i0 * i0 * e.S0 + i0 * i1 * (e.S1 + e.S2) + i1 * i1 * e.S3;
            const float g = (float)(-0.5 * (double)dist - c.log_2pi - 0.5 * (double)d_safe_log(e.det));
            const float lq = d_safe_log(e.pd) + d_safe_log(w0) + g;
            w = expf(lq - s_leta[m]);
            keep = !(w < c.minFeatureWeight);
            mx = mx + e.K0 * i0 + e.K2 * i1;
            my = my + e.K1 * i0 + e.K3 * i1;
        }
        int tot;
        const int r = wrank(keep, &tot);
        if (keep) {
            const int p = ncand + r;
            if (p < Kcap) {
                const float4 v = make_float4(e.cu0, e.cu1, e.cu2, e.cu3);
                C.P[p] = cand_record(mx, my, w, v, c.minSeparation, sc_bad, sc_lmax);
                C.tag[p] = (unsigned short)(0x8000u | (unsigned)(p - nd0));
                C.detv[p - nd0] = v;
            }
        }
        ncand += tot;
    }
    WSTAMP(6);
    // 4c births (none in the CPHD update array)
    if (!CPHD) {
        for (int base = 0; base < M; base += 64) {
            const int m = base + lane;
            bool keep = false;
            float w = 0.f;
            if (m < M) {
                const float lb = s_zok[m] ? c.log_birth : PHD_LOG0;
                w = expf(lb - s_leta[m]);
                keep = !(w < c.minFeatureWeight);
            }
            int tot;
            const int r = wrank(keep, &tot);
            if (keep) {
                const int p = ncand + r;
                if (p < Kcap) {
                    float mean[2], cov[4];
                    d_birth(c, pose.px, pose.py, pose.ptheta, s_zr[m], s_zb[m], mean, cov);
                    const float4 v = make_float4(cov[0], cov[1], cov[2], cov[3]);
                    C.P[p] = cand_record(mean[0], mean[1], w, v, c.minSeparation, sc_bad, sc_lmax);
                    C.tag[p] = (unsigned short)(0x8000u | (unsigned)(p - nd0));
                    C.detv[p - nd0] = v;
                }
            }
            ncand += tot;
        }
    }
    // 4d near-range components join the merge unpruned (mergeAndCopyMaps :3227-3257)
    for (int base = 0; base < G; base += 64) {
        const int k = base + lane;
        const bool near = k < G && s_cls[k] == 2;
        int tot;
        const int r = wrank(near, &tot);
        if (near) {
            const int p = ncand + r;
            if (p < Kcap) {
                const float4 v = make_float4(src[3 * cap + k], src[4 * cap + k], src[5 * cap + k], src[6 * cap + k]);
                C.P[p] = cand_record(src[1 * cap + k], src[2 * cap + k], src[k], v, c.minSeparation, sc_bad, sc_lmax);
                C.tag[p] = (unsigned short)k;
            }
        }
        ncand += tot;
    }
    if (ncand > Kcap) {
        flags |= PHD_ST_CANDIDATE_OVERFLOW;
        ncand = Kcap;
    }
    wsync();
    WSTAMP(7);
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 13
    return;  // timing ablation: up to the candidates
#endif

    /* Phase 5: greedy merge — parallel exact form, serial fallback. */
    WMerge X;
    X.C = C;
    X.key = (unsigned short*)(smem + L.mkey);
    X.gstart = (unsigned short*)(smem + L.mgst);
    X.plist = (unsigned int*)(smem + L.mplist);
    X.plcap = L.plcap;
    X.edges = (unsigned int*)(smem + L.medge);
    X.cur = (unsigned short*)(smem + L.mcur);
    X.off = (unsigned short*)(smem + L.moff);
    X.pool = (unsigned short*)(smem + L.mpool);
    X.par = (short*)(smem + L.mpar);
    int nout = a.merge_mode == 0
                   ? w_merge_parallel(X, ncand, c.minSeparation, dst, cap, a.Epool, L.B, s_misc, sc_bad, sc_lmax,
#ifdef PHD_STAMPS
                                      a.stamps ? a.stamps + (size_t)n * PHD_STAMP_SLOTS : nullptr
#else
                                      nullptr
#endif
                                      )
                   : -1;
    if (nout < 0) {
        wsync();
        nout = w_merge_serial(C, ncand, X.par, c.minSeparation, dst, cap);
        flags |= PHD_ST_SERIAL_MERGE;
    }
    WSTAMP(8);
#if defined(PHD_EXPERIMENT) && PHD_EXPERIMENT == 14
    return;  // timing ablation: up to the merge
#endif

    /* Phase 6: out-of-range components appended unchanged (mergeAndCopyMaps :3304-3323). */
    int nouts = 0;
    for (int base = 0; base < G; base += 64) {
        const int k = base + lane;
        const bool out = k < G && s_cls[k] == 0;
        int tot;
        const int r = wrank(out, &tot);
        if (out) {
            const int p = nout + nouts + r;
            if (p < cap) {
#pragma unroll
                for (int f = 0; f < NF; f++) dst[f * cap + p] = src[f * cap + k];
            }
        }
        nouts += tot;
    }
    int total = nout + nouts;
    if (total > cap) {
        flags |= PHD_ST_MAP_OVERFLOW;
        total = cap;
    }
    flags = wave_or_i(flags);
    if (lane == 0) {
        g1(a.size_out)[n] = total;
        g1(a.status)[n] = flags;
        if (flags & ~PHD_ST_SERIAL_MERGE) atomicOr(a.err, flags & ~PHD_ST_SERIAL_MERGE);
        if (flags & PHD_ST_SERIAL_MERGE) atomicAdd(a.err + 1, 1);
        if (a.src_reset) g1(a.src_reset)[n] = n;
    }
    WSTAMP(9);
#ifdef PHD_STAMPS
    if (lane == 0 && a.stamps) {
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 10] = ((unsigned long long)ncand << 32) | (unsigned)nsurv;
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 40] = dbg_cls;
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 41] = dbg_walk;
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 42] = dbg_iter;
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 43] = dbg_pairs;
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 44] = dbgw[0];
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 45] = dbgw[1];
        a.stamps[(size_t)n * PHD_STAMP_SLOTS + 46] = dbgw[2];
    }
#endif
}

__global__ void __launch_bounds__(64) k_update_wave(UpdateArgs a) { wave_update<false>(a); }
__global__ void __launch_bounds__(64) k_update_wave_cphd(UpdateArgs a) { wave_update<true>(a); }

}  // namespace phd
