/*
 * phd_devutil.h — device helpers shared by the fused update kernels
 * (phd_kernels.hip, workgroup per particle) and the CPHD terms (phd_terms.hip):
 * predict steps, wave64 DPP scans and reductions, the Q40 eta encoding, merge
 * candidate records and the merge lattice.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "phd_detmath.h"
#include "phd_device.h"
#include "phd_kernels.h"
#include "phd_rng.h"

namespace phd {

/* Global (address space 1) views of device pointers: loads and stores through
 * them are global_* instructions.  Through generic pointers (e.g. after a
 * readfirstlane of the address, uni_p) the compiler emits flat_* ones, which
 * also count in lgkmcnt — every LDS wait would then also wait for the slab
 * loads in flight. */
#define G1 __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ G1 T* g1(T* p) {
    return (G1 T*)p;
}

/* One Ackerman step (phdfilter.cu:802-820) with this particle's noise. */
__device__ __forceinline__ phd_pose predict_ackerman_one(const phd_pose& s, const phd_ackerman_control& u,
                                                         float n_alpha, float n_enc, const PredictCfg& c) {
    phd_pose ns;
    const float ve = u.v_encoder + n_enc;
    const float al = u.alpha + n_alpha;
    const float ta = phd_det_tanf(al);  // D16
    const float vc = ve / (1 - ta * c.h / c.l);
    float st, ct;
    phd_det_sincosf(s.ptheta, &st, &ct);
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
    return ns;
}

/* Philox Ackerman noise of global particle id (host-noise semantics: phdfilter.cu:1148-1152). */
__device__ __forceinline__ void ackerman_noise(uint64_t seed, int id, uint64_t step, const PredictCfg& c,
                                               float* n_alpha, float* n_enc) {
    const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)id, step, PHD_STREAM_PREDICT);
    double g0, g1;
    phd_box_muller(x.v[0], x.v[1], &g0, &g1);
    *n_alpha = (float)((double)c.stdAlpha * g0);
    *n_enc = (float)((double)c.stdEncoder * g1);
}

/* One constant-velocity step (phdfilter.cu:841-856). */
__device__ __forceinline__ phd_pose predict_cv_one(const phd_pose& s, const phd_cv_noise& w, const PredictCfg& c) {
    phd_pose ns;
    const float dt = c.dt / c.subdivide;
    float st, ct;
    phd_det_sincosf(s.ptheta, &st, &ct);
    ns.px = (float)((double)(s.px + dt * (s.vx * ct - s.vy * st)) + (double)(dt * dt) * 0.5 * (double)(w.ax * ct - w.ay * st));
    ns.py = (float)((double)(s.py + dt * (s.vx * st + s.vy * ct)) + (double)(dt * dt) * 0.5 * (double)(w.ax * st + w.ay * ct));
    ns.ptheta = d_wrap((float)((double)(s.ptheta + dt * s.vtheta) + 0.5 * dt * dt * (double)w.atheta));
    ns.vx = s.vx + dt * w.ax;
    ns.vy = s.vy + dt * w.ay;
    ns.vtheta = s.vtheta + dt * w.atheta;
    return ns;
}

__device__ __forceinline__ phd_cv_noise cv_noise(uint64_t seed, int id, uint64_t step, const PredictCfg& c) {
    const phd_u32x4 x = phd_rng_draw(seed, (uint32_t)id, step, PHD_STREAM_PREDICT);
    double g0, g1, g2, g3;
    phd_box_muller(x.v[0], x.v[1], &g0, &g1);
    phd_box_muller(x.v[2], x.v[3], &g2, &g3);
    phd_cv_noise w;
    w.ax = (float)((double)(3 * c.ax) * g0);
    w.ay = (float)((double)(3 * c.ay) * g1);
    w.atheta = (float)((double)(3 * c.ayaw) * g2);
    return w;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

/* Wave-wide inclusive scans on DPP (row_shr 1/2/4/8 within 16-lane rows,
 * then row_bcast15 / row_bcast31 across rows): VALU only, no LDS crossbar.
 * Lanes whose DPP source is out of range read the identity. */
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_or_zero(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWMASK, 0xf, false);
}

__device__ __forceinline__ int wave_incl_scan(int x) {
    x += dpp_or_zero<0x111, 0xf>(x);
    x += dpp_or_zero<0x112, 0xf>(x);
    x += dpp_or_zero<0x114, 0xf>(x);
    x += dpp_or_zero<0x118, 0xf>(x);
    x += dpp_or_zero<0x142, 0xa>(x);
    x += dpp_or_zero<0x143, 0xc>(x);
    return x;
}

/* running max of non-negative ints; lane 63 holds the wave maximum */
__device__ __forceinline__ int wave_incl_max_i(int x) {
    x = max(x, dpp_or_zero<0x111, 0xf>(x));
    x = max(x, dpp_or_zero<0x112, 0xf>(x));
    x = max(x, dpp_or_zero<0x114, 0xf>(x));
    x = max(x, dpp_or_zero<0x118, 0xf>(x));
    x = max(x, dpp_or_zero<0x142, 0xa>(x));
    x = max(x, dpp_or_zero<0x143, 0xc>(x));
    return x;
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_or_zero_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(dpp_or_zero<CTRL, ROWMASK>(hi), dpp_or_zero<CTRL, ROWMASK>(lo));
}

/* inclusive scan in double; lane 63 holds the wave total */
__device__ __forceinline__ double wave_incl_scan_d(double x) {
    x += dpp_or_zero_d<0x111, 0xf>(x);
    x += dpp_or_zero_d<0x112, 0xf>(x);
    x += dpp_or_zero_d<0x114, 0xf>(x);
    x += dpp_or_zero_d<0x118, 0xf>(x);
    x += dpp_or_zero_d<0x142, 0xa>(x);
    x += dpp_or_zero_d<0x143, 0xc>(x);
    return x;
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_or_ninf(float x) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(x), CTRL, ROWMASK, 0xf, false));
}

/* running max; lane 63 holds the wave maximum */
__device__ __forceinline__ float wave_incl_max(float x) {
    x = fmaxf(x, dpp_or_ninf<0x111, 0xf>(x));
    x = fmaxf(x, dpp_or_ninf<0x112, 0xf>(x));
    x = fmaxf(x, dpp_or_ninf<0x114, 0xf>(x));
    x = fmaxf(x, dpp_or_ninf<0x118, 0xf>(x));
    x = fmaxf(x, dpp_or_ninf<0x142, 0xa>(x));
    x = fmaxf(x, dpp_or_ninf<0x143, 0xc>(x));
    return x;
}

/* Sum of up to 4 doubles over the block (the "intended exact sum", oracle D3);
 * every thread gets the totals. s_red holds >= 4 * NT/64 doubles. */
template <int K, int NT>
__device__ __forceinline__ void block_sum(double (&v)[K], double* s_red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = wave_incl_scan_d(v[k]);
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < K; k++) s_red[wid * 4 + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) t += s_red[w * 4 + k];
        v[k] = t;
    }
    __syncthreads();
}

/* floor(q * 2^40) for 0 <= q < 2^22 (clamped), from exact float steps. */
__device__ __forceinline__ unsigned long long to_q40(float q) {
    q = fminf(q, 4194304.f);
    const float h = q * 256.f;                 // exact
    const unsigned int hi = (unsigned int)h;   // trunc
    const float rem = h - (float)hi;           // exact fraction
    const unsigned int lo = (unsigned int)(rem * 4294967296.f);
    return ((unsigned long long)hi << 32) | lo;
}

/* merge priority: heavier first, then lower candidate index (oracle D1) */
__device__ __forceinline__ bool earlier(float wa, int ka, float wb, int kb) {
    return wa > wb || (wa == wb && ka < kb);
}

/* Merge candidates in LDS: P = (x, y, weight, lambda_max or -1).  The
 * covariance of a prior-derived candidate (non-detection, near range) stays in
 * the prior slab (tag = its component index); detection / birth candidates keep
 * theirs in LDS (tag bit 15 | slot in detv). */
/* A candidate's covariance tag rides in the low 16 bits of its record's
 * lambda slot (cand_record): < 0x8000 the prior component it copies, else
 * 0x8000 | its row of detv. */
__device__ __forceinline__ unsigned cand_tag(const float4& p) { return __float_as_uint(p.w) & 0xffffu; }

struct Cand {
    float4* P;
    float4* detv;
    const G1 float* src;
    const G1 float* bsrc;  // the step's birth slab shifted by -G: prior component t >= G is bsrc[f cap + t]
    int G;                 // slab components (prior components from G on are the step's births)
    int cap;
    __device__ __forceinline__ float4 V(int i) const {
        const unsigned t = cand_tag(P[i]);
        if (t & 0x8000u) return detv[t & 0x7fffu];
        const G1 float* s = ((int)t < G ? src : bsrc) + t;
        return make_float4(s[3 * cap], s[4 * cap], s[5 * cap], s[6 * cap]);
    }
    /* V(i) of a candidate whose record p = P[i] is already loaded, without a
     * branch: both the LDS and the slab loads are issued (the slab address of a
     * detection record is the slab's first component), so the loads of several
     * candidates can be in flight together. */
    __device__ __forceinline__ float4 Vp(const float4& p) const {
        const unsigned t = cand_tag(p);
        const bool det = (t & 0x8000u) != 0;
        const float4 d = detv[det ? (t & 0x7fffu) : 0u];
        const G1 float* s = det ? src : ((int)t < G ? src : bsrc) + t;
        const float4 g = make_float4(s[3 * cap], s[4 * cap], s[5 * cap], s[6 * cap]);
        return det ? d : g;
    }
};

__device__ __forceinline__ float cand_mahal(const float4& pa, const float4& va, const float4& pb, const float4& vb) {
    return d_mahal(pa.x, pa.y, va.x, va.y, va.z, va.w, pb.x, pb.y, vb.x, vb.y, vb.z, vb.w);
}

/* cand_mahal(p, v, p, v) < T, bit for bit, for a finite mean: the differences
 * are exact zeros, so the distance is (0 i0 + 0 (i1 + i2)) + 0 i3 — zero when the
 * three inverse terms are finite, NaN otherwise.  They are certainly finite
 * when every |v| <= 1e18 (the halved sums are then v itself and the products
 * finite) and |det| >= 1e-19 (1 / det <= 1e19, every inverse term <= 1e37);
 * only the rest evaluates the distance. */
__device__ __forceinline__ bool own_distance_below(const float4& p, const float4& v, float T) {
    const float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    const float det = v.x * v.w - v.z * v.y;
    if (m <= 1e18f && fabsf(det) >= 1e-19f) return 0.f < T;
    return cand_mahal(p, v, p, v) < T;
}

/* Candidate record with the merge's screen folded in: P.w = an upper bound of
 * lambda_max of the covariance when well conditioned (lambda_min > 1e-4
 * lambda_max), else -1 ("wild"), with the covariance tag in its low 16 bits
 * (cand_tag): max(lambda_max, 1e-30) (1 + 2^-6) with its low 16 mantissa bits
 * replaced stays above lambda_max (they weigh < 2^-7), so the walk's isotropic
 * cull stays conservative; the lattice is sized by the exact maximum.  `bad`
 * flags what only the serial greedy reproduces: non-finite values or a failed
 * own-distance test d(i,i) < T; lmax tracks the largest well-conditioned
 * lambda_max. */
__device__ __forceinline__ float4 cand_record(float x, float y, float w, const float4& v, float T, int& bad,
                                              float& lmax, unsigned tag) {
    float4 p = make_float4(x, y, w, 0.f);
    const float aa = v.x, d = v.w, b = 0.5f * (v.y + v.z);
    const float h = 0.5f * (aa - d);
    const float rt = sqrtf(h * h + b * b);
    const float l1 = 0.5f * (aa + d) + rt, l2 = 0.5f * (aa + d) - rt;
    const bool finite = (w > 0.f) && (w < INFINITY) && (fabsf(x) < INFINITY) && (fabsf(y) < INFINITY);
    const bool ok = finite && (l1 < INFINITY) && l2 > 1e-4f * l1;
    bad |= !finite || !own_distance_below(p, v, T);  // the greedy's own-distance test
    if (ok) lmax = fmaxf(lmax, l1);
    const unsigned lb = __float_as_uint(ok ? fmaxf(l1, 1e-30f) * 1.015625f : -1.f);
    p.w = __uint_as_float((lb & 0xffff0000u) | tag);
    return p;
}

/* lattice of B = 2^lgPx x 2^lgPy buckets (upd_buckets) */
__device__ __forceinline__ void lattice_dims(int B, int* lgPx, int* lgPy) {
    *lgPx = B >= 16384 ? 7 : B >= 2048 ? 6 : 5;
    *lgPy = B >= 16384 ? 7 : B >= 4096 ? 6 : B >= 1024 ? 5 : 4;
}

__device__ __forceinline__ unsigned int lattice_bucket(float x, float y, float invR, int Px, int Py, int lgPx) {
    const int cx = (int)floorf(fminf(fmaxf(x * invR, -8192.f), 8192.f));
    const int cy = (int)floorf(fminf(fmaxf(y * invR, -8192.f), 8192.f));
    return (unsigned int)(cx & (Px - 1)) | ((unsigned int)(cy & (Py - 1)) << lgPx);
}

/* 16-bit counters updated through 32-bit LDS atomics on their containing word */
__device__ __forceinline__ void cnt16_inc(unsigned short* c, int i) {
    atomicAdd((unsigned int*)(c + (i & ~1)), (i & 1) ? 0x10000u : 1u);
}
__device__ __forceinline__ int cnt16_dec(unsigned short* c, int i) {  // returns the new value
    const unsigned int old = atomicSub((unsigned int*)(c + (i & ~1)), (i & 1) ? 0x10000u : 1u);
    return (int)((i & 1) ? (old >> 16) : (old & 0xffffu)) - 1;
}

/* k * log x with 0 * log 0 = 0 (all detection ratios zero: an empty map) */
__device__ __forceinline__ double kpow_d(int k, double lx) { return k == 0 ? 0.0 : (double)k * lx; }

__device__ __forceinline__ double readlane_d(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_or_ninf_d(double v) {
    const double ninf = -INFINITY;
    return __hiloint2double(
        __builtin_amdgcn_update_dpp(__double2hiint(ninf), __double2hiint(v), CTRL, ROWMASK, 0xf, false),
        __builtin_amdgcn_update_dpp(__double2loint(ninf), __double2loint(v), CTRL, ROWMASK, 0xf, false));
}
/* wave-uniform max / sum of doubles: DPP prefix (row shifts, row broadcasts), lane 63 read back */
__device__ __forceinline__ double wave_max_dx(double x) {
    x = fmax(x, dpp_or_ninf_d<0x111, 0xf>(x));
    x = fmax(x, dpp_or_ninf_d<0x112, 0xf>(x));
    x = fmax(x, dpp_or_ninf_d<0x114, 0xf>(x));
    x = fmax(x, dpp_or_ninf_d<0x118, 0xf>(x));
    x = fmax(x, dpp_or_ninf_d<0x142, 0xa>(x));
    x = fmax(x, dpp_or_ninf_d<0x143, 0xc>(x));
    return readlane_d(x, 63);
}
__device__ __forceinline__ double wave_sum_dx(double x) { return readlane_d(wave_incl_scan_d(x), 63); }
/* log-sum-exp over the wave of two terms per lane (-inf terms allowed) */
__device__ __forceinline__ double wave_lse2(double t0, double t1) {
    const double mx = wave_max_dx(fmax(t0, t1));
    if (mx == -INFINITY) return -INFINITY;
    const double s = wave_sum_dx(exp(t0 - mx) + exp(t1 - mx));
    return log(s) + mx;
}

/* cross-lane shifts of a two-slot (k = lane, lane + 64) coefficient vector:
 * DPP wave_shr:1 / wave_shl:1 (GFX9 wave-wide shifts) plus one readlane for
 * the slot carry — no LDS round trip on the recursion's critical path */
/* c <- c + x * (c shifted up one coefficient): multiply by (1 + x z) */
__device__ __forceinline__ void poly_mul_lin(double& c0, double& c1, double x) {
    const double carry = readlane_d(c0, 63);
    const double u0 = dpp_or_zero_d<0x138, 0xf>(c0);  // wave_shr:1, lane 0 <- 0
    double u1 = dpp_or_zero_d<0x138, 0xf>(c1);
    if ((threadIdx.x & 63) == 0) u1 = carry;
    c0 = fma(x, u0, c0);
    c1 = fma(x, u1, c1);
}
/* t <- t + x * (t shifted down one coefficient) */
__device__ __forceinline__ void suffix_step(double& t0, double& t1, double x) {
    const double carry = readlane_d(t1, 0);
    double d0 = dpp_or_zero_d<0x130, 0xf>(t0);  // wave_shl:1, lane 63 <- 0
    const double d1 = dpp_or_zero_d<0x130, 0xf>(t1);
    if ((threadIdx.x & 63) == 63) d0 = carry;
    t0 = fma(x, d0, t0);
    t1 = fma(x, d1, t1);
}

/* a workgroup-uniform double / pointer moved to scalar registers
 * (readfirstlane of both halves): it then costs no VGPRs while it stays live */
template <class T>
__device__ __forceinline__ T* uni_p(T* p) {
    const unsigned long long v = (unsigned long long)p;
    return (T*)(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v));
}
__device__ __forceinline__ double uni_d(double x) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                            __builtin_amdgcn_readfirstlane(__double2loint(x)));
}

}  // namespace phd
