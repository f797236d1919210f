/*
 * phd_mixed.h — arithmetic of the mixed static + dynamic feature model
 * (feature_model = 2), host + device, header-only.
 *
 * Shared by the GPU kernels (csrc/phd_mixed.hip) and the CPU oracle
 * (oracle/scphd_cpu.cpp orc_update_mixed / orc_predict_dynamic): parity of the
 * mixed path checks the orchestration (classification, weights, normalisers,
 * prune, merge order); the expressions below are pinned by closed-form tests
 * (tests/test_oracle_closed_form.py: 4x4 inverse, Kalman update and the
 * constant-velocity prediction against float64 numpy).
 *
 * Every function restates one reference routine with its float / double
 * promotions (cited per function).  Device-side pow(x, 2) of the reference is
 * the float square x * x; powf(dt, 3|4) is the correctly rounded power.
 * Exponentials and logarithms go through phd_det_expf / phd_det_logf (exact
 * double primitives, rounded once) so the CPU and gfx950 agree bit for bit
 * (DESIGN.md deviation D14).
 */
#ifndef PHD_MIXED_H
#define PHD_MIXED_H

#include <float.h>

#include "phd_detmath.h"
#include "phd_types.h"

#ifdef __clang__
#define PHD_MX_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define PHD_MX_NOCONTRACT
#endif

/* safeLog (device_math.cuh:9-16) on the deterministic log. */
PHD_DHD float phd_mx_safe_log(float x) { return x <= 0.0f ? -FLT_MAX : phd_det_logf(x); }

/* wrapAngle (device_math.cuh:242-251): fmod in float, comparisons and the
 * +-2 pi shift in double, stored float. */
PHD_DHD float phd_mx_wrap(float a) {
    PHD_MX_NOCONTRACT
    float rem = PHD_DNS fmod(a, (float)(2 * 3.14159265358979323846));
    const double r = rem;
    if (r > 3.14159265358979323846)
        rem = (float)(r - 2 * 3.14159265358979323846);
    else if (r < -3.14159265358979323846)
        rem = (float)(r + 2 * 3.14159265358979323846);
    return rem;
}

/* invert_matrix4 (device_math.cuh:87-106): cofactors over the explicit
 * determinant, with the reference's term order; the last entry multiplies the
 * double reciprocal of the determinant. */
PHD_DHD void phd_inv4(const float* A, float* R) {
    PHD_MX_NOCONTRACT
    const float a0 = A[0], a1 = A[1], a2 = A[2], a3 = A[3], a4 = A[4], a5 = A[5], a6 = A[6], a7 = A[7];
    const float a8 = A[8], a9 = A[9], a10 = A[10], a11 = A[11], a12 = A[12], a13 = A[13], a14 = A[14], a15 = A[15];
    const float D = a0 * a5 * a15 * a10 - a0 * a5 * a11 * a14 - a0 * a7 * a13 * a10 + a0 * a11 * a6 * a13 -
                    a0 * a15 * a6 * a9 + a0 * a7 * a9 * a14 + a5 * a3 * a8 * a14 - a5 * a15 * a2 * a8 +
                    a5 * a11 * a2 * a12 - a5 * a3 * a12 * a10 - a15 * a10 * a1 * a4 + a15 * a6 * a1 * a8 +
                    a15 * a2 * a4 * a9 + a3 * a12 * a6 * a9 + a7 * a13 * a2 * a8 + a7 * a1 * a12 * a10 +
                    a3 * a4 * a13 * a10 + a11 * a14 * a1 * a4 - a11 * a6 * a1 * a12 - a11 * a2 * a4 * a13 -
                    a3 * a8 * a6 * a13 - a7 * a9 * a2 * a12 - a7 * a1 * a8 * a14 - a3 * a4 * a9 * a14;
    R[0] = (a5 * a15 * a10 - a5 * a11 * a14 - a7 * a13 * a10 + a11 * a6 * a13 - a15 * a6 * a9 + a7 * a9 * a14) / D;
    R[1] = -(a15 * a10 * a1 - a11 * a14 * a1 + a3 * a9 * a14 - a15 * a2 * a9 - a3 * a13 * a10 + a11 * a2 * a13) / D;
    R[2] = (a5 * a3 * a14 - a5 * a15 * a2 + a15 * a6 * a1 + a7 * a13 * a2 - a3 * a6 * a13 - a7 * a1 * a14) / D;
    R[3] = -(a5 * a3 * a10 - a5 * a11 * a2 - a3 * a6 * a9 - a7 * a1 * a10 + a11 * a6 * a1 + a7 * a9 * a2) / D;
    R[4] = -(a15 * a10 * a4 - a15 * a6 * a8 - a7 * a12 * a10 - a11 * a14 * a4 + a11 * a6 * a12 + a7 * a8 * a14) / D;
    R[5] = (a0 * a15 * a10 - a0 * a11 * a14 + a3 * a8 * a14 - a15 * a2 * a8 + a11 * a2 * a12 - a3 * a12 * a10) / D;
    R[6] = -(a0 * a15 * a6 - a0 * a7 * a14 - a15 * a2 * a4 - a3 * a12 * a6 + a3 * a4 * a14 + a7 * a2 * a12) / D;
    R[7] = (-a0 * a7 * a10 + a0 * a11 * a6 + a7 * a2 * a8 + a3 * a4 * a10 - a11 * a2 * a4 - a3 * a8 * a6) / D;
    R[8] = (-a5 * a15 * a8 + a5 * a11 * a12 + a15 * a4 * a9 + a7 * a13 * a8 - a11 * a4 * a13 - a7 * a9 * a12) / D;
    R[9] = -(a0 * a15 * a9 - a0 * a11 * a13 - a15 * a1 * a8 - a3 * a12 * a9 + a11 * a1 * a12 + a3 * a8 * a13) / D;
    R[10] = (a15 * a0 * a5 - a15 * a1 * a4 - a3 * a12 * a5 - a7 * a0 * a13 + a7 * a1 * a12 + a3 * a4 * a13) / D;
    R[11] = -(a11 * a0 * a5 - a11 * a1 * a4 - a3 * a8 * a5 - a7 * a0 * a9 + a7 * a1 * a8 + a3 * a4 * a9) / D;
    R[12] = -(-a5 * a8 * a14 + a5 * a12 * a10 - a12 * a6 * a9 - a4 * a13 * a10 + a8 * a6 * a13 + a4 * a9 * a14) / D;
    R[13] = (-a0 * a13 * a10 + a0 * a9 * a14 + a13 * a2 * a8 + a1 * a12 * a10 - a9 * a2 * a12 - a1 * a8 * a14) / D;
    R[14] = -(a14 * a0 * a5 - a14 * a1 * a4 - a2 * a12 * a5 - a6 * a0 * a13 + a6 * a1 * a12 + a2 * a4 * a13) / D;
    R[15] = (float)(1.0 / (double)D *
                    (double)(a10 * a0 * a5 - a10 * a1 * a4 - a2 * a8 * a5 - a6 * a0 * a9 + a6 * a1 * a8 + a2 * a4 * a9));
}

/* computeMahalDist(Gaussian4D, Gaussian4D) (device_math.cuh:346-363). */
PHD_DHD float phd_mahal4(const float* ca, const float* ma, const float* cb, const float* mb) {
    PHD_MX_NOCONTRACT
    float s[16], si[16];
    for (int i = 0; i < 16; i++) s[i] = (ca[i] + cb[i]) / 2;
    phd_inv4(s, si);
    const float i0 = ma[0] - mb[0], i1 = ma[1] - mb[1], i2 = ma[2] - mb[2], i3 = ma[3] - mb[3];
    return i0 * (si[0] * i0 + si[4] * i1 + si[8] * i2 + si[12] * i3) +
           i1 * (si[1] * i0 + si[5] * i1 + si[9] * i2 + si[13] * i3) +
           i2 * (si[2] * i0 + si[6] * i1 + si[10] * i2 + si[14] * i3) +
           i3 * (si[3] * i0 + si[7] * i1 + si[11] * i2 + si[15] * i3);
}

/* computeMahalDist(Gaussian2D, Gaussian2D) with invert_matrix2 (device_math.cuh:57-69, 308-325). */
PHD_DHD float phd_mahal2(const float* ca, const float* ma, const float* cb, const float* mb) {
    PHD_MX_NOCONTRACT
    float s[4];
    for (int i = 0; i < 4; i++) s[i] = (ca[i] + cb[i]) / 2;
    const float det = s[0] * s[3] - s[2] * s[1];
    const float si0 = s[3] / det, si1 = -s[1] / det, si2 = -s[2] / det, si3 = s[0] / det;
    const float i0 = ma[0] - mb[0], i1 = ma[1] - mb[1];
    return i0 * i0 * si0 + i0 * i1 * (si1 + si2) + i1 * i1 * si3;
}

/* Model parameters of the mixed update, from SlamConfig. */
typedef struct {
    float maxRange, minRange, maxBearing, stdRange, stdBearing, pd;
    float clutterDensity, birthWeight, birthNoiseFactor, minFeatureWeight, minSeparation;
    float covVxBirth, covVyBirth;
    float dt, stdAxMap, stdAyMap, ps, tau, beta;
    int labeled;
} phd_mx_cfg;

PHD_DHD phd_mx_cfg phd_mx_config(const phd_slam_config* c) {
    phd_mx_cfg m;
    m.maxRange = c->maxRange;
    m.minRange = c->minRange;
    m.maxBearing = c->maxBearing;
    m.stdRange = c->stdRange;
    m.stdBearing = c->stdBearing;
    m.pd = c->pd;
    m.clutterDensity = c->clutterDensity;
    m.birthWeight = c->birthWeight;
    m.birthNoiseFactor = c->birthNoiseFactor;
    m.minFeatureWeight = c->minFeatureWeight;
    m.minSeparation = c->minSeparation;
    m.covVxBirth = c->covVxBirth;
    m.covVyBirth = c->covVyBirth;
    m.dt = c->dt;
    m.stdAxMap = c->stdAxMap;
    m.stdAyMap = c->stdAyMap;
    m.ps = c->ps;
    m.tau = c->tau;
    m.beta = c->beta;
    m.labeled = c->labeledMeasurements ? 1 : 0;
    return m;
}

/* Range class of a component against a pose (computeInRangeKernel,
 * phdfilter.cu:1327-1346): 1 in range, 2 nearly in range, 0 out of range. */
PHD_DHD int phd_mx_range_class(const phd_mx_cfg& c, const phd_pose& pose, float mx, float my) {
    PHD_MX_NOCONTRACT
    const float dx = mx - pose.px, dy = my - pose.py;
    const float r = PHD_DNS sqrt(dx * dx + dy * dy);
    const float b = phd_mx_wrap(phd_atan2f(dy, dx) - pose.ptheta);
    const float ab = PHD_DNS fabs(b);
    if (r >= c.minRange && r <= c.maxRange && ab <= c.maxBearing) return 1;
    if ((double)r >= 0.8 * c.minRange && (double)r <= 1.2 * c.maxRange && (double)ab <= 1.2 * c.maxBearing) return 2;
    return 0;
}

/* Pre-update terms of one in-range component (computePreUpdate,
 * phdfilter.cu:302-395 for Gaussian2D, :397-521 for Gaussian4D). */
typedef struct {
    float r, bearing, pd, det;
    float S[4];
    float K[8];     /* 2-D: K[0..3] */
    float cu[16];   /* 2-D: cu[0..3] */
} phd_mx_ekf;

PHD_DHD void phd_mx_ekf2(const phd_mx_cfg& c, const phd_pose& pose, const float* mean, const float* P,
                         phd_mx_ekf& e) {
    PHD_MX_NOCONTRACT
    const float dx = mean[0] - pose.px, dy = mean[1] - pose.py;
    const float r2 = dx * dx + dy * dy;
    const float r = PHD_DNS sqrt(r2);
    const float bearing = phd_mx_wrap(phd_atan2f(dy, dx) - pose.ptheta);
    e.pd = (r <= c.maxRange && PHD_DNS fabs(bearing) <= c.maxBearing) ? c.pd : 0.0f;
    const float J0 = dx / r, J2 = dy / r, J1 = -dy / r2, J3 = dx / r2;
    const float sR2 = c.stdRange * c.stdRange, sB2 = c.stdBearing * c.stdBearing;
    float sg0 = (P[0] * J0 + J2 * P[1]) * J0 + (J0 * P[2] + P[3] * J2) * J2 + sR2;
    float sg1 = (P[0] * J1 + J3 * P[1]) * J0 + (J1 * P[2] + P[3] * J3) * J2;
    float sg2 = (P[0] * J0 + J2 * P[1]) * J1 + (J0 * P[2] + P[3] * J2) * J3;
    const float sg3 = (P[0] * J1 + J3 * P[1]) * J1 + (J1 * P[2] + P[3] * J3) * J3 + sB2;
    sg1 = (sg1 + sg2) / 2;
    sg2 = sg1;
    const float det = sg0 * sg3 - sg1 * sg2;
    float* S = e.S;
    S[0] = sg3 / det;
    S[1] = -sg1 / det;
    S[2] = -sg2 / det;
    S[3] = sg0 / det;
    float* K = e.K;
    K[0] = S[0] * (P[0] * J0 + P[2] * J2) + S[1] * (P[0] * J1 + P[2] * J3);
    K[1] = S[0] * (P[1] * J0 + P[3] * J2) + S[1] * (P[1] * J1 + P[3] * J3);
    K[2] = S[2] * (P[0] * J0 + P[2] * J2) + S[3] * (P[0] * J1 + P[2] * J3);
    K[3] = S[2] * (P[1] * J0 + P[3] * J2) + S[3] * (P[1] * J1 + P[3] * J3);
    const float sR = c.stdRange, sB = c.stdBearing;
    const float a00 = 1 - K[0] * J0 - K[2] * J1, a01 = -K[0] * J2 - K[2] * J3;
    const float a10 = -K[1] * J0 - K[3] * J1, a11 = 1 - K[1] * J2 - K[3] * J3;
    float* cu = e.cu;
    cu[0] = (a00 * P[0] + a01 * P[1]) * a00 + (a00 * P[2] + a01 * P[3]) * a01 + K[0] * K[0] * sR * sR +
            K[2] * K[2] * sB * sB;
    cu[2] = (a00 * P[0] + a01 * P[1]) * a10 + (a00 * P[2] + a01 * P[3]) * a11 + K[0] * sR * sR * K[1] +
            K[2] * sB * sB * K[3];
    cu[1] = (a10 * P[0] + a11 * P[1]) * a00 + (a10 * P[2] + a11 * P[3]) * a01 + K[0] * sR * sR * K[1] +
            K[2] * sB * sB * K[3];
    cu[3] = (a10 * P[0] + a11 * P[1]) * a10 + (a10 * P[2] + a11 * P[3]) * a11 + K[1] * K[1] * sR * sR +
            K[3] * K[3] * sB * sB;
    e.r = r;
    e.bearing = bearing;
    e.det = det;
}

PHD_DHD void phd_mx_ekf4(const phd_mx_cfg& c, const phd_pose& pose, const float* mean, const float* P,
                         phd_mx_ekf& e) {
    PHD_MX_NOCONTRACT
    const float dx = mean[0] - pose.px, dy = mean[1] - pose.py;
    const float r2 = dx * dx + dy * dy;
    const float r = PHD_DNS sqrt(r2);
    const float bearing = phd_mx_wrap(phd_atan2f(dy, dx) - pose.ptheta);
    e.pd = (r <= c.maxRange && PHD_DNS fabs(bearing) <= c.maxBearing) ? c.pd : 0.0f;
    const float J0 = dx / r, J2 = dy / r, J1 = -dy / r2, J3 = dx / r2;
    const float vr = c.stdRange * c.stdRange, vb = c.stdBearing * c.stdBearing;
    float sg0 = J0 * (P[0] * J0 + P[4] * J2) + J2 * (P[1] * J0 + P[5] * J2) + vr;
    float sg1 = J1 * (P[0] * J0 + P[4] * J2) + J3 * (P[1] * J0 + P[5] * J2);
    float sg2 = J0 * (P[0] * J1 + P[4] * J3) + J2 * (P[1] * J1 + P[5] * J3);
    const float sg3 = J1 * (P[0] * J1 + P[4] * J3) + J3 * (P[1] * J1 + P[5] * J3) + vb;
    sg1 = (sg1 + sg2) / 2;
    sg2 = sg1;
    const float det = sg0 * sg3 - sg1 * sg2;
    float* S = e.S;
    S[0] = sg3 / det;
    S[1] = -sg1 / det;
    S[2] = -sg2 / det;
    S[3] = sg0 / det;
    const float u0 = J0 * S[0] + J1 * S[1], v0 = J2 * S[0] + J3 * S[1];
    const float u1 = J0 * S[2] + J1 * S[3], v1 = J2 * S[2] + J3 * S[3];
    float* K = e.K;
    K[0] = P[0] * u0 + P[4] * v0;
    K[1] = P[1] * u0 + P[5] * v0;
    K[2] = P[2] * u0 + P[6] * v0;
    K[3] = P[3] * u0 + P[7] * v0;
    K[4] = P[0] * u1 + P[4] * v1;
    K[5] = P[1] * u1 + P[5] * v1;
    K[6] = P[2] * u1 + P[6] * v1;
    K[7] = P[3] * u1 + P[7] * v1;
    // Joseph form (phdfilter.cu:472-487): rows of (I - K J) applied to P
    const float A0 = 1 - K[0] * J0 - K[4] * J1, A1 = -K[0] * J2 - K[4] * J3;
    const float B0 = -K[1] * J0 - K[5] * J1, B1 = 1 - K[1] * J2 - K[5] * J3;
    const float C0 = -K[2] * J0 - K[6] * J1, C1 = -K[2] * J2 - K[6] * J3;
    const float D0 = -K[3] * J0 - K[7] * J1, D1 = -K[3] * J2 - K[7] * J3;
    const float pa0 = P[0] * A0 + P[4] * A1, pa1 = P[1] * A0 + P[5] * A1;
    const float pb0 = P[0] * B0 + P[4] * B1, pb1 = P[1] * B0 + P[5] * B1;
    const float pc0 = P[0] * C0 + P[4] * C1 + P[8], pc1 = P[1] * C0 + P[5] * C1 + P[9];
    const float pd0 = P[0] * D0 + P[4] * D1 + P[12], pd1 = P[1] * D0 + P[5] * D1 + P[13];
    float* cu = e.cu;
    cu[0] = A0 * pa0 + A1 * pa1 + vr * (K[0] * K[0]) + vb * (K[4] * K[4]);
    cu[1] = B0 * pa0 + B1 * pa1 + K[0] * vr * K[1] + K[4] * vb * K[5];
    cu[2] = C0 * pa0 + C1 * pa1 + P[2] * A0 + P[6] * A1 + K[0] * vr * K[2] + K[4] * vb * K[6];
    cu[3] = D0 * pa0 + D1 * pa1 + P[3] * A0 + P[7] * A1 + K[0] * vr * K[3] + K[4] * vb * K[7];
    cu[4] = A0 * pb0 + A1 * pb1 + K[0] * vr * K[1] + K[4] * vb * K[5];
    cu[5] = B0 * pb0 + B1 * pb1 + vr * (K[1] * K[1]) + vb * (K[5] * K[5]);
    cu[6] = C0 * pb0 + C1 * pb1 + P[2] * B0 + P[6] * B1 + K[1] * vr * K[2] + K[5] * vb * K[6];
    cu[7] = D0 * pb0 + D1 * pb1 + P[3] * B0 + P[7] * B1 + K[1] * vr * K[3] + K[5] * vb * K[7];
    cu[8] = A0 * pc0 + A1 * pc1 + K[0] * vr * K[2] + K[4] * vb * K[6];
    cu[9] = B0 * pc0 + B1 * pc1 + K[1] * vr * K[2] + K[5] * vb * K[6];
    cu[10] = C0 * pc0 + C1 * pc1 + P[2] * C0 + P[6] * C1 + P[10] + vr * (K[2] * K[2]) + vb * (K[6] * K[6]);
    cu[11] = D0 * pc0 + D1 * pc1 + P[3] * C0 + P[7] * C1 + P[11] + K[2] * vr * K[3] + K[6] * vb * K[7];
    cu[12] = A0 * pd0 + A1 * pd1 + K[0] * vr * K[3] + K[4] * vb * K[7];
    cu[13] = B0 * pd0 + B1 * pd1 + K[1] * vr * K[3] + K[5] * vb * K[7];
    cu[14] = C0 * pd0 + C1 * pd1 + P[2] * D0 + P[6] * D1 + P[14] + K[2] * vr * K[3] + K[6] * vb * K[7];
    cu[15] = D0 * pd0 + D1 * pd1 + P[3] * D0 + P[7] * D1 + P[15] + vr * (K[3] * K[3]) + vb * (K[7] * K[7]);
    e.r = r;
    e.bearing = bearing;
    e.det = det;
}

/* Innovation, Mahalanobis distance and the partially updated log-weight of a
 * detection term (phdfilter.cu:371-393 / :495-519): the float sum of the two
 * logs, then the rest in double, stored float; LOG0 for a measurement of the
 * other label when labels are on.  i0 / i1 receive the innovation. */
PHD_DHD float phd_mx_logq(const phd_mx_ekf& e, float w, float zr, float zb, int label_ok, float* i0, float* i1) {
    PHD_MX_NOCONTRACT
    const float a = zr - e.r;
    const float b = phd_mx_wrap(zb - e.bearing);
    *i0 = a;
    *i1 = b;
    if (!label_ok) return -FLT_MAX;
    const float dist = a * a * e.S[0] + a * b * (e.S[1] + e.S[2]) + b * b * e.S[3];
    const float l2 = phd_mx_safe_log(e.pd) + phd_mx_safe_log(w);
    return (float)((double)l2 - 0.5 * (double)dist - (double)phd_mx_safe_log((float)(2 * 3.14159265358979323846)) -
                   0.5 * (double)phd_mx_safe_log(e.det));
}

/* computeBirth (phdfilter.cu:205-242 Gaussian2D, :244-299 Gaussian4D), device
 * form.  dims = 2 writes cov[4] / mean[2]; dims = 4 cov[16] / mean[4]. */
PHD_DHD float phd_mx_birth(const phd_mx_cfg& c, const phd_pose& pose, float zr, float zb, int label_ok, int dims,
                           float* mean, float* cov) {
    PHD_MX_NOCONTRACT
    const float theta = pose.ptheta + zb;
    float sn_, cs_;
    phd_det_sincosf(theta, &sn_, &cs_);  // D16
    const float dx = zr * cs_, dy = zr * sn_;
    mean[0] = pose.px + dx;
    mean[1] = pose.py + dy;
    const float J0 = dx / zr, J1 = dy / zr, J2 = -dy, J3 = dx;
    const float sr = c.stdRange * c.birthNoiseFactor, sb = c.stdBearing * c.birthNoiseFactor;
    const float vr = sr * sr, vb = sb * sb;
    const float c00 = (J0 * J0) * vr + (J2 * J2) * vb;
    const float c01 = J0 * J1 * vr + J2 * J3 * vb;
    const float c11 = (J1 * J1) * vr + (J3 * J3) * vb;
    if (dims == 2) {
        cov[0] = c00;
        cov[1] = c01;
        cov[2] = c01;
        cov[3] = c11;
    } else {
        mean[2] = 0.0f;
        mean[3] = 0.0f;
        for (int i = 0; i < 16; i++) cov[i] = 0.0f;
        cov[0] = c00;
        cov[1] = c01;
        cov[4] = c01;
        cov[5] = c11;
        cov[10] = c.covVxBirth;
        cov[15] = c.covVyBirth;
    }
    return label_ok ? phd_mx_safe_log(c.birthWeight) : -FLT_MAX;
}

/* Correctly rounded dt^k (powf(dt, k) of the reference, k = 3, 4). */
PHD_DHD float phd_mx_powi(float x, int k) {
    double r = 1.0;
    for (int i = 0; i < k; i++) r *= (double)x;
    return (float)r;
}

/* predictMapKernelMixed, MIXED_MODEL branch (phdfilter.cu:910-963), with
 * ConstantVelocityMotionModel::compute_prediction (device_math.cuh:608-657)
 * at scale 1: survival p_jmm * ps with the jump probability p_jmm =
 * 1 / (1 + exp(beta (tau - |v|))).  The jump component the reference forms is
 * never used (phdfilter.cu:1016-1019) and is not produced. */
PHD_DHD void phd_mx_predict4(const phd_mx_cfg& c, const float* m, const float* p, float w, float* mo, float* po,
                             float* wo) {
    PHD_MX_NOCONTRACT
    const float vx = m[2], vy = m[3];
    const float vmag = PHD_DNS sqrt(vx * vx + vy * vy);
    const float sig = 1 / (1 + phd_det_expf(c.beta * (c.tau - vmag)));
    const float dt = c.dt;
    const float var_x = c.stdAxMap * c.stdAxMap * 1.0f, var_y = c.stdAyMap * c.stdAyMap * 1.0f;
    const float d3 = phd_mx_powi(dt, 3), d4 = phd_mx_powi(dt, 4);
    mo[0] = m[0] + dt * m[2];
    mo[1] = m[1] + dt * m[3];
    mo[2] = m[2];
    mo[3] = m[3];
    po[0] = (float)((double)(p[0] + p[8] * dt + dt * (p[2] + p[10] * dt)) + (double)(d4 * var_x) / 4.0);
    po[1] = p[1] + p[9] * dt + dt * (p[3] + p[11] * dt);
    po[2] = (float)((double)(p[2] + p[10] * dt) + (double)(d3 * var_x) / 2.0);
    po[3] = p[3] + p[11] * dt;
    po[4] = p[4] + p[12] * dt + dt * (p[6] + p[14] * dt);
    po[5] = (float)((double)(p[5] + p[13] * dt + dt * (p[7] + p[15] * dt)) + (double)(d4 * var_y) / 4.0);
    po[6] = p[6] + p[14] * dt;
    po[7] = (float)((double)(p[7] + p[15] * dt) + (double)(d3 * var_y) / 2.0);
    po[8] = (float)((double)(p[8] + p[10] * dt) + (double)(d3 * var_x) / 2.0);
    po[9] = p[9] + p[11] * dt;
    po[10] = p[10] + var_x * dt * dt;
    po[11] = p[11];
    po[12] = p[12] + p[14] * dt;
    po[13] = (float)((double)(p[13] + p[15] * dt) + (double)(d3 * var_y) / 2.0);
    po[14] = p[14];
    po[15] = p[15] + var_y * dt * dt;
    *wo = sig * c.ps * w;
}

/* force_symmetric_covariance (device_math.cuh:710-725), column-major dims x dims. */
PHD_DHD void phd_mx_symmetrize(float* cov, int dims) {
    PHD_MX_NOCONTRACT
    for (int i = 0; i < dims; i++)
        for (int j = 0; j < i; j++) {
            const int lo = i + j * dims, up = j + i * dims;
            cov[lo] = (cov[lo] + cov[up]) / 2;
            cov[up] = cov[lo];
        }
}

/* EAP expected map of the dynamic (Gaussian4D) maps, exp_map_dynamic
 * (main.cpp:369-371 -> reduceGaussianMixture<Gaussian4D>, gm_reduce.cpp:59-132):
 * the Mahalanobis distance of the generic GaussianX path (gm_reduce.cpp:30-37):
 * sigma = (a.cov + b.cov) / 2, L = chol(sigma) (the lower triangle, Eigen LLT),
 * x = L^-1 (a.mean - b.mean) by forward substitution, |x|^2.  Covariances are
 * column-major (cov[i + 4 j]); parity unpinned (Eigen is not in the image). */
PHD_DHD float phd_eap_mahal4(const float* ma, const float* ca, const float* mb, const float* cb) {
    PHD_MX_NOCONTRACT
    float s[4][4];  // lower triangle of the averaged covariance, s[i][j] = sigma(i, j), i >= j
    for (int j = 0; j < 4; j++)
        for (int i = j; i < 4; i++) s[i][j] = 0.5f * (ca[i + 4 * j] + cb[i + 4 * j]);
    float L[4][4];
    for (int j = 0; j < 4; j++) {
        float d = s[j][j];
        for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k];
        L[j][j] = sqrtf(d);
        for (int i = j + 1; i < 4; i++) {
            float v = s[i][j];
            for (int k = 0; k < j; k++) v -= L[i][k] * L[j][k];
            L[i][j] = v / L[j][j];
        }
    }
    float x[4], r = 0.0f;
    for (int i = 0; i < 4; i++) {
        float v = ma[i] - mb[i];
        for (int k = 0; k < i; k++) v -= L[i][k] * x[k];
        x[i] = v / L[i][i];
        r += x[i] * x[i];
    }
    return r;
}

/* Moment match of one EAP merge set (gm_reduce.cpp:103-123): the seed first,
 * then the absorbed members in priority order; float, the reference's order. */
struct phd_eap4_acc {
    float W, m[4], c[16];
};
PHD_DHD void phd_eap4_mean_begin(phd_eap4_acc& a, float w, const float* m) {
    PHD_MX_NOCONTRACT
    a.W = w;
    for (int i = 0; i < 4; i++) a.m[i] = m[i] * w;
}
PHD_DHD void phd_eap4_mean_add(phd_eap4_acc& a, float w, const float* m) {
    PHD_MX_NOCONTRACT
    for (int i = 0; i < 4; i++) a.m[i] += w * m[i];
    a.W += w;
}
PHD_DHD void phd_eap4_cov_begin(phd_eap4_acc& a, float w, const float* m, const float* c) {
    PHD_MX_NOCONTRACT
    for (int i = 0; i < 4; i++) a.m[i] /= a.W;
    float d[4];
    for (int i = 0; i < 4; i++) d[i] = a.m[i] - m[i];
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 4; i++) a.c[i + 4 * j] = w * (c[i + 4 * j] + d[i] * d[j]);
}
PHD_DHD void phd_eap4_cov_add(phd_eap4_acc& a, float w, const float* m, const float* c) {
    PHD_MX_NOCONTRACT
    float d[4];
    for (int i = 0; i < 4; i++) d[i] = a.m[i] - m[i];
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 4; i++) a.c[i + 4 * j] += w * (c[i + 4 * j] + d[i] * d[j]);
}
PHD_DHD void phd_eap4_finish(const phd_eap4_acc& a, phd_gaussian4d* out) {
    PHD_MX_NOCONTRACT
    out->weight = a.W;
    for (int i = 0; i < 4; i++) out->mean[i] = a.m[i];
    for (int k = 0; k < 16; k++) out->cov[k] = a.c[k] / a.W;
}

#endif /* PHD_MIXED_H */
