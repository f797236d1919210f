/*
 * phd_device.h — gfx950 device helpers for the PHD update path.
 *
 * Scalar semantics follow the reference's device helpers so that the GPU and
 * the CPU oracle round the same way wherever IEEE operations are involved:
 *   safeLog            device_math.cuh:9-16
 *   wrapAngle          device_math.cuh:242-251 (fmodf, then ±2π in double)
 *   computeMahalDist   device_math.cuh:309-325
 *   EKF terms          phdfilter.cu:1836-1895
 *   birth terms        phdfilter.cu:3474-3506 (host loop; device twin :205-242)
 * The translation unit is compiled with -ffp-contract=off so that a*b+c is not
 * fused where the reference rounds twice.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "phd_detmath.h"
#include "phd_types.h"

#define PHD_LOG0 (-FLT_MAX)

__device__ __forceinline__ float d_safe_log(float x) { return x <= 0.f ? PHD_LOG0 : logf(x); }
/* safeLog of a PHD normaliser / the birth weight with the deterministic log of
 * phd_detmath.h (oracle deviation D17): the oracle takes the same bits, so
 * normalisers one float ulp apart that one logf maps to one value and another
 * to two (libm's and ocml's logf each within an ulp, not of each other) give the
 * same exact ties among the birth weights beta / eta on both sides — the greedy
 * merge breaks those ties by candidate index (D1). */
__device__ __forceinline__ float d_det_safe_log(float x) { return x <= 0.f ? PHD_LOG0 : phd_det_logf(x); }

/* wrapAngle: fmodf is exact; |a| < 2π (the common case) is the identity. */
__device__ __forceinline__ float d_wrap(float a) {
    const float two_pi_f = (float)(2 * M_PI);
    float rem = (fabsf(a) < two_pi_f) ? a : fmodf(a, two_pi_f);
    const double r = rem;
    if (r > M_PI)
        rem = (float)(r - 2 * M_PI);
    else if (r < -M_PI)
        rem = (float)(r + 2 * M_PI);
    return rem;
}

/* The per-component quantities the pair loop and the correction need. */
struct DevEkf {
    float r, bearing, pd, det;
    float S0, S1, S2, S3;
    float K0, K1, K2, K3;
    float cu0, cu1, cu2, cu3;
};

struct DevCfg {
    float minRange, maxRange, maxBearing;
    float stdRange, stdBearing, pd;
    float kappa, birthWeight, birthNoiseFactor;
    float minFeatureWeight, minSeparation;
    float log_birth;       /* safeLog(birthWeight) */
    float lq_keep_thresh;  /* log q below which a detection term can never survive the prune */
    double log_2pi;        /* (double)safeLog((float)(2π)) */
    int labeled;
    /* CPHD (filter_type 1) */
    double cphd_rate;      /* clutterRate */
    double cphd_lrate;     /* log clutterRate */
    double cphd_lck;       /* log clutterRate - log clutterDensity */
    float cphd_log1mpd;    /* safeLog(1 - pd) */
    float log_minfw;       /* log minFeatureWeight */
    float cphd_thr0;       /* log2 listing bound of the single-pass CPHD walk: log(minFW κ) - 2.5, x log2 e */
    float cphd_leta_min;   /* log κ - 2: detection factors up to e^2/κ are covered by cphd_thr0 */
    /* log2 floor of the pair walk: a term q < 2^walk_floor neither moves a
     * normaliser (its share of the smallest possible η / Λ is below 2^-40) nor can
     * be listed, so the bearing windows only reach pairs with log2 q >= walk_floor */
    float walk_floor;
};

/* EKF terms from the predicted range/bearing geometry (dx, dy, r^2, r, bearing).
 * The Jacobian and the innovation inverse from reciprocals 1 / r, (1 / r)^2
 * and 1 / det (oracle deviation D18, the oracle computes the same products):
 * an ulp or two from the reference's quotients, six IEEE divisions fewer. */
__device__ __forceinline__ void d_ekf_from_geometry(const DevCfg& c, float dx, float dy, float r2, float r,
                                                    float bearing, float P0, float P1, float P2, float P3, DevEkf& e) {
    float pd = 0.f;
    if (r <= c.maxRange && fabsf(bearing) <= c.maxBearing) pd = c.pd;
    const float ir = 1.0f / r, ir2 = ir * ir;
    const float J0 = dx * ir, J2 = dy * ir, J1 = -dy * ir2, J3 = dx * ir2;
    const float sR2 = c.stdRange * c.stdRange, sB2 = c.stdBearing * c.stdBearing;
    float s0 = (P0 * J0 + J2 * P1) * J0 + (J0 * P2 + P3 * J2) * J2 + sR2;
    float s1 = (P0 * J1 + J3 * P1) * J0 + (J1 * P2 + P3 * J3) * J2;
    float s2 = (P0 * J0 + J2 * P1) * J1 + (J0 * P2 + P3 * J2) * J3;
    float s3 = (P0 * J1 + J3 * P1) * J1 + (J1 * P2 + P3 * J3) * J3 + sB2;
    s1 = (s1 + s2) / 2;
    s2 = s1;
    const float det = s0 * s3 - s1 * s2;
    const float id = 1.0f / det;
    const float S0 = s3 * id, S1 = -s1 * id, S2 = -s2 * id, S3 = s0 * id;
    const float K0 = S0 * (P0 * J0 + P2 * J2) + S1 * (P0 * J1 + P2 * J3);
    const float K1 = S0 * (P1 * J0 + P3 * J2) + S1 * (P1 * J1 + P3 * J3);
    const float K2 = S2 * (P0 * J0 + P2 * J2) + S3 * (P0 * J1 + P2 * J3);
    const float K3 = S2 * (P1 * J0 + P3 * J2) + S3 * (P1 * J1 + P3 * J3);
    const float sR = c.stdRange, sB = c.stdBearing;
    const float a00 = 1 - K0 * J0 - K2 * J1;
    const float a01 = -K0 * J2 - K2 * J3;
    const float a10 = -K1 * J0 - K3 * J1;
    const float a11 = 1 - K1 * J2 - K3 * J3;
    e.cu0 = (a00 * P0 + a01 * P1) * a00 + (a00 * P2 + a01 * P3) * a01 + K0 * K0 * sR * sR + K2 * K2 * sB * sB;
    e.cu2 = (a00 * P0 + a01 * P1) * a10 + (a00 * P2 + a01 * P3) * a11 + K0 * sR * sR * K1 + K2 * sB * sB * K3;
    e.cu1 = (a10 * P0 + a11 * P1) * a00 + (a10 * P2 + a11 * P3) * a01 + K0 * sR * sR * K1 + K2 * sB * sB * K3;
    e.cu3 = (a10 * P0 + a11 * P1) * a10 + (a10 * P2 + a11 * P3) * a11 + K1 * K1 * sR * sR + K3 * K3 * sB * sB;
    e.r = r;
    e.bearing = bearing;
    e.pd = pd;
    e.det = det;
    e.S0 = S0;
    e.S1 = S1;
    e.S2 = S2;
    e.S3 = S3;
    e.K0 = K0;
    e.K1 = K1;
    e.K2 = K2;
    e.K3 = K3;
}

__device__ __forceinline__ void d_compute_ekf(const DevCfg& c, float px, float py, float pth, float mx, float my,
                                              float P0, float P1, float P2, float P3, DevEkf& e) {
    const float dx = mx - px;
    const float dy = my - py;
    const float r2 = dx * dx + dy * dy;
    const float r = sqrtf(r2);
    const float bearing = d_wrap(phd_atan2f(dy, dx) - pth);
    d_ekf_from_geometry(c, dx, dy, r2, r, bearing, P0, P1, P2, P3, e);
}

/* Birth component of measurement (range, bearing); host-loop semantics incl. its double pow. */
__device__ __forceinline__ void d_birth(const DevCfg& c, float px, float py, float pth, float zr, float zb,
                                       float* mean, float* cov) {
    const float theta = pth + zb;
    float sn, cs;
    phd_det_sincosf(theta, &sn, &cs);  // D16: the oracle's bits
    const float dx = zr * cs;
    const float dy = zr * sn;
    mean[0] = px + dx;
    mean[1] = py + dy;
    const float izr = 1.0f / zr;  // (D18, as the oracle)
    const float J0 = dx * izr, J1 = dy * izr, J2 = -dy, J3 = dx;
    const double vr_d = (double)(c.stdRange * c.birthNoiseFactor);
    const double vb_d = (double)(c.stdBearing * c.birthNoiseFactor);
    const float var_range = (float)(vr_d * vr_d);
    const float var_bearing = (float)(vb_d * vb_d);
    cov[0] = (float)((double)J0 * (double)J0 * (double)var_range + (double)J2 * (double)J2 * (double)var_bearing);
    cov[1] = J0 * J1 * var_range + J2 * J3 * var_bearing;
    cov[2] = cov[1];
    cov[3] = (float)((double)J1 * (double)J1 * (double)var_range + (double)J3 * (double)J3 * (double)var_bearing);
}

/* computeMahalDist for 2-D Gaussians given as (mean, cov[4]).  The inverse
 * from one reciprocal of the determinant (oracle deviation D18, as the
 * oracle).  Symmetric in its two arguments bit for bit (the summed covariance
 * and the squared differences do not depend on the order). */
__device__ __forceinline__ float d_mahal(float ax, float ay, float a0, float a1, float a2, float a3, float bx, float by,
                                         float b0, float b1, float b2, float b3) {
    const float s0 = (a0 + b0) / 2, s1 = (a1 + b1) / 2, s2 = (a2 + b2) / 2, s3 = (a3 + b3) / 2;
    const float det = s0 * s3 - s2 * s1;
    const float r = 1.0f / det;
    const float i0 = s3 * r, i1 = -s1 * r, i2 = -s2 * r, i3 = s0 * r;
    const float d0 = ax - bx, d1 = ay - by;
    return d0 * d0 * i0 + d0 * d1 * (i1 + i2) + d1 * d1 * i3;
}

/* Wave64 helpers. */
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
