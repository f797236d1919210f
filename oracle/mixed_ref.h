/*
 * mixed_ref.h — the oracle's OWN restatement of the mixed static + dynamic
 * feature-model arithmetic (feature_model 2), TEST INFRASTRUCTURE ONLY.
 *
 * Written from the reference sources, independently of the product header
 * include/phd_mixed.h, so the GPU-vs-oracle tests of the mixed path compare
 * two separate statements of the same reference expressions:
 *   invert_matrix4            device_math.cuh:87-106
 *   computeMahalDist (4-D)    device_math.cuh:346-363; (2-D) :57-69, :308-325
 *   wrapAngle / safeLog       device_math.cuh:242-251 / :9-16
 *   computePreUpdate 2-D      phdfilter.cu:302-395 (Maple expressions, Joseph form)
 *   computePreUpdate 4-D      phdfilter.cu:397-521
 *   computeBirth              phdfilter.cu:205-299 (device form)
 *   compute_prediction (CV)   device_math.cuh:608-657, predictMapKernelMixed phdfilter.cu:910-963
 *   force_symmetric_covariance device_math.cuh:710-725
 *   reduceGaussianMixture<4>  gm_reduce.cpp:30-37 (LLT distance), :103-123 (moments)
 * Every float / double promotion of the reference is kept: `x / 0.4e1` and
 * `- 0.5*dist` are double operations, pow(x, 2) of a float is the exact float
 * square, powf(dt, 3|4) the correctly rounded power.  Only exp / log go through
 * the deterministic primitives of the phd_detmath.h contract (D14; shared like
 * det_expf, D8) so both sides round them alike.
 */
#ifndef ORACLE_MIXED_REF_H
#define ORACLE_MIXED_REF_H

#include <cfloat>
#include <cmath>

#include "phd_detmath.h"
#include "phd_types.h"

namespace orx {

constexpr double PI = 3.14159265358979323846;

/* safeLog on the deterministic log (device_math.cuh:9-16, D14) */
inline float safe_log(float x) { return x <= 0.0f ? -FLT_MAX : phd_det_logf(x); }

/* wrapAngle: float fmod, then the comparisons and the 2 pi shift in double */
inline float wrap(float a) {
    float rem = std::fmod(a, (float)(2 * PI));
    const double r = rem;
    if (r > PI) rem = (float)(r - 2 * PI);
    else if (r < -PI) rem = (float)(r + 2 * PI);
    return rem;
}

/* invert_matrix4: every entry is its cofactor sum divided by the same
 * determinant expression (evaluated once: identical bits), the last one as
 * 0.1e1 / det (double) times its cofactor sum (float promoted). */
inline void inverse4(const float* A, float* Ainv) {
    const float det =
        A[0] * A[5] * A[15] * A[10] - A[0] * A[5] * A[11] * A[14] - A[0] * A[7] * A[13] * A[10] +
        A[0] * A[11] * A[6] * A[13] - A[0] * A[15] * A[6] * A[9] + A[0] * A[7] * A[9] * A[14] +
        A[5] * A[3] * A[8] * A[14] - A[5] * A[15] * A[2] * A[8] + A[5] * A[11] * A[2] * A[12] -
        A[5] * A[3] * A[12] * A[10] - A[15] * A[10] * A[1] * A[4] + A[15] * A[6] * A[1] * A[8] +
        A[15] * A[2] * A[4] * A[9] + A[3] * A[12] * A[6] * A[9] + A[7] * A[13] * A[2] * A[8] +
        A[7] * A[1] * A[12] * A[10] + A[3] * A[4] * A[13] * A[10] + A[11] * A[14] * A[1] * A[4] -
        A[11] * A[6] * A[1] * A[12] - A[11] * A[2] * A[4] * A[13] - A[3] * A[8] * A[6] * A[13] -
        A[7] * A[9] * A[2] * A[12] - A[7] * A[1] * A[8] * A[14] - A[3] * A[4] * A[9] * A[14];
    float c[16];
    c[0] = A[5] * A[15] * A[10] - A[5] * A[11] * A[14] - A[7] * A[13] * A[10] + A[11] * A[6] * A[13] -
           A[15] * A[6] * A[9] + A[7] * A[9] * A[14];
    c[1] = -(A[15] * A[10] * A[1] - A[11] * A[14] * A[1] + A[3] * A[9] * A[14] - A[15] * A[2] * A[9] -
             A[3] * A[13] * A[10] + A[11] * A[2] * A[13]);
    c[2] = A[5] * A[3] * A[14] - A[5] * A[15] * A[2] + A[15] * A[6] * A[1] + A[7] * A[13] * A[2] -
           A[3] * A[6] * A[13] - A[7] * A[1] * A[14];
    c[3] = -(A[5] * A[3] * A[10] - A[5] * A[11] * A[2] - A[3] * A[6] * A[9] - A[7] * A[1] * A[10] +
             A[11] * A[6] * A[1] + A[7] * A[9] * A[2]);
    c[4] = -(A[15] * A[10] * A[4] - A[15] * A[6] * A[8] - A[7] * A[12] * A[10] - A[11] * A[14] * A[4] +
             A[11] * A[6] * A[12] + A[7] * A[8] * A[14]);
    c[5] = A[0] * A[15] * A[10] - A[0] * A[11] * A[14] + A[3] * A[8] * A[14] - A[15] * A[2] * A[8] +
           A[11] * A[2] * A[12] - A[3] * A[12] * A[10];
    c[6] = -(A[0] * A[15] * A[6] - A[0] * A[7] * A[14] - A[15] * A[2] * A[4] - A[3] * A[12] * A[6] +
             A[3] * A[4] * A[14] + A[7] * A[2] * A[12]);
    c[7] = -A[0] * A[7] * A[10] + A[0] * A[11] * A[6] + A[7] * A[2] * A[8] + A[3] * A[4] * A[10] -
           A[11] * A[2] * A[4] - A[3] * A[8] * A[6];
    c[8] = -A[5] * A[15] * A[8] + A[5] * A[11] * A[12] + A[15] * A[4] * A[9] + A[7] * A[13] * A[8] -
           A[11] * A[4] * A[13] - A[7] * A[9] * A[12];
    c[9] = -(A[0] * A[15] * A[9] - A[0] * A[11] * A[13] - A[15] * A[1] * A[8] - A[3] * A[12] * A[9] +
             A[11] * A[1] * A[12] + A[3] * A[8] * A[13]);
    c[10] = A[15] * A[0] * A[5] - A[15] * A[1] * A[4] - A[3] * A[12] * A[5] - A[7] * A[0] * A[13] +
            A[7] * A[1] * A[12] + A[3] * A[4] * A[13];
    c[11] = -(A[11] * A[0] * A[5] - A[11] * A[1] * A[4] - A[3] * A[8] * A[5] - A[7] * A[0] * A[9] +
              A[7] * A[1] * A[8] + A[3] * A[4] * A[9]);
    c[12] = -(-A[5] * A[8] * A[14] + A[5] * A[12] * A[10] - A[12] * A[6] * A[9] - A[4] * A[13] * A[10] +
              A[8] * A[6] * A[13] + A[4] * A[9] * A[14]);
    c[13] = -A[0] * A[13] * A[10] + A[0] * A[9] * A[14] + A[13] * A[2] * A[8] + A[1] * A[12] * A[10] -
            A[9] * A[2] * A[12] - A[1] * A[8] * A[14];
    c[14] = -(A[14] * A[0] * A[5] - A[14] * A[1] * A[4] - A[2] * A[12] * A[5] - A[6] * A[0] * A[13] +
              A[6] * A[1] * A[12] + A[2] * A[4] * A[13]);
    const float c15 = A[10] * A[0] * A[5] - A[10] * A[1] * A[4] - A[2] * A[8] * A[5] - A[6] * A[0] * A[9] +
                      A[6] * A[1] * A[8] + A[2] * A[4] * A[9];
    for (int k = 0; k < 15; k++) Ainv[k] = c[k] / det;
    Ainv[15] = (float)(0.1e1 / (double)det * (double)c15);
}

/* computeMahalDist(Gaussian4D) — innov' (sigma_avg)^-1 innov, row by row */
inline float mahal4(const float* ma, const float* ca, const float* mb, const float* cb) {
    float sig[16], si[16], v[4];
    for (int i = 0; i < 16; i++) sig[i] = (ca[i] + cb[i]) / 2;
    inverse4(sig, si);
    for (int i = 0; i < 4; i++) v[i] = ma[i] - mb[i];
    float d = 0.0f;
    for (int i = 0; i < 4; i++) {
        const float row = si[i] * v[0] + si[4 + i] * v[1] + si[8 + i] * v[2] + si[12 + i] * v[3];
        d = i == 0 ? v[0] * row : d + v[i] * row;
    }
    return d;
}

/* computeMahalDist(Gaussian2D) with invert_matrix2 */
inline float mahal2(const float* ma, const float* ca, const float* mb, const float* cb) {
    float sig[4];
    for (int i = 0; i < 4; i++) sig[i] = (ca[i] + cb[i]) / 2;
    const float det = sig[0] * sig[3] - sig[2] * sig[1];
    const float i00 = sig[3] / det, i01 = -sig[1] / det, i10 = -sig[2] / det, i11 = sig[0] / det;
    const float a = ma[0] - mb[0], b = ma[1] - mb[1];
    return a * a * i00 + a * b * (i01 + i10) + b * b * i11;
}

/* range class of computeInRangeKernel (phdfilter.cu:1327-1346) */
inline int range_class(const phd_slam_config& c, const phd_pose& pose, float mx, float my) {
    const float dx = mx - pose.px, dy = my - pose.py;
    const float r = std::sqrt(dx * dx + dy * dy);
    const float ab = std::fabs(wrap(phd_atan2f(dy, dx) - pose.ptheta));
    if (r >= c.minRange && r <= c.maxRange && ab <= c.maxBearing) return 1;
    if ((double)r >= 0.8 * c.minRange && (double)r <= 1.2 * c.maxRange && (double)ab <= 1.2 * c.maxBearing) return 2;
    return 0;
}

/* computePreUpdate products: predicted range / bearing, pd, det(sigma), sigma^-1,
 * gain (2 x dims, column pairs: K[i] range column, K[dims + i] bearing column)
 * and the Joseph-form updated covariance (column-major dims x dims). */
struct PreUpdate {
    float r, bearing, pd, det;
    float S[4];
    float K[8];
    float cov[16];
};

/* the common front: geometry, pd, Jacobian J = [J0 J1; J2 J3] (reference
 * layout: J[0] = dr/dx, J[2] = dr/dy, J[1] = db/dx, J[3] = db/dy) */
inline void front(const phd_slam_config& c, const phd_pose& pose, const float* mean, PreUpdate& u, float J[4],
                  float& r2) {
    const float dx = mean[0] - pose.px, dy = mean[1] - pose.py;
    r2 = dx * dx + dy * dy;
    u.r = std::sqrt(r2);
    u.bearing = wrap(phd_atan2f(dy, dx) - pose.ptheta);
    u.pd = (u.r <= c.maxRange && std::fabs(u.bearing) <= c.maxBearing) ? c.pd : 0.0f;
    J[0] = dx / u.r;
    J[2] = dy / u.r;
    J[1] = -dy / r2;
    J[3] = dx / r2;
}

inline void invert_sigma(float s0, float s1, float s2, float s3, PreUpdate& u) {
    s1 = (s1 + s2) / 2;  // enforce symmetry
    s2 = s1;
    u.det = s0 * s3 - s1 * s2;
    u.S[0] = s3 / u.det;
    u.S[1] = -s1 / u.det;
    u.S[2] = -s2 / u.det;
    u.S[3] = s0 / u.det;
}

/* phdfilter.cu:302-395: P is the 2x2 column-major covariance */
inline void preupdate2(const phd_slam_config& c, const phd_pose& pose, const float* mean, const float* P,
                       PreUpdate& u) {
    float J[4], r2;
    front(c, pose, mean, u, J, r2);
    const float vr = c.stdRange * c.stdRange, vb = c.stdBearing * c.stdBearing;  // pow(float, 2)
    invert_sigma((P[0] * J[0] + J[2] * P[1]) * J[0] + (J[0] * P[2] + P[3] * J[2]) * J[2] + vr,
                 (P[0] * J[1] + J[3] * P[1]) * J[0] + (J[1] * P[2] + P[3] * J[3]) * J[2],
                 (P[0] * J[0] + J[2] * P[1]) * J[1] + (J[0] * P[2] + P[3] * J[2]) * J[3],
                 (P[0] * J[1] + J[3] * P[1]) * J[1] + (J[1] * P[2] + P[3] * J[3]) * J[3] + vb, u);
    const float* S = u.S;
    float* K = u.K;
    const float pj0 = P[0] * J[0] + P[2] * J[2], pj1 = P[0] * J[1] + P[2] * J[3];
    const float qj0 = P[1] * J[0] + P[3] * J[2], qj1 = P[1] * J[1] + P[3] * J[3];
    K[0] = S[0] * pj0 + S[1] * pj1;
    K[1] = S[0] * qj0 + S[1] * qj1;
    K[2] = S[2] * pj0 + S[3] * pj1;
    K[3] = S[2] * qj0 + S[3] * qj1;
    // (I - K J) rows: e = row 0, f = row 1
    const float e0 = 1 - K[0] * J[0] - K[2] * J[1], e1 = -K[0] * J[2] - K[2] * J[3];
    const float f0 = -K[1] * J[0] - K[3] * J[1], f1 = 1 - K[1] * J[2] - K[3] * J[3];
    const float sR = c.stdRange, sB = c.stdBearing;
    float* cu = u.cov;
    cu[0] = (e0 * P[0] + e1 * P[1]) * e0 + (e0 * P[2] + e1 * P[3]) * e1 + K[0] * K[0] * sR * sR + K[2] * K[2] * sB * sB;
    cu[2] = (e0 * P[0] + e1 * P[1]) * f0 + (e0 * P[2] + e1 * P[3]) * f1 + K[0] * sR * sR * K[1] + K[2] * sB * sB * K[3];
    cu[1] = (f0 * P[0] + f1 * P[1]) * e0 + (f0 * P[2] + f1 * P[3]) * e1 + K[0] * sR * sR * K[1] + K[2] * sB * sB * K[3];
    cu[3] = (f0 * P[0] + f1 * P[1]) * f0 + (f0 * P[2] + f1 * P[3]) * f1 + K[1] * K[1] * sR * sR + K[3] * K[3] * sB * sB;
}

/* phdfilter.cu:397-521: P is the 4x4 column-major covariance */
inline void preupdate4(const phd_slam_config& c, const phd_pose& pose, const float* mean, const float* P,
                       PreUpdate& u) {
    float J[4], r2;
    front(c, pose, mean, u, J, r2);
    const float vr = c.stdRange * c.stdRange, vb = c.stdBearing * c.stdBearing;
    const float h0 = P[0] * J[0] + P[4] * J[2], h1 = P[1] * J[0] + P[5] * J[2];
    const float g0 = P[0] * J[1] + P[4] * J[3], g1 = P[1] * J[1] + P[5] * J[3];
    invert_sigma(J[0] * h0 + J[2] * h1 + vr, J[1] * h0 + J[3] * h1, J[0] * g0 + J[2] * g1, J[1] * g0 + J[3] * g1 + vb,
                 u);
    const float* S = u.S;
    float* K = u.K;
    const float a = J[0] * S[0] + J[1] * S[1], b = J[2] * S[0] + J[3] * S[1];
    const float a2 = J[0] * S[2] + J[1] * S[3], b2 = J[2] * S[2] + J[3] * S[3];
    for (int i = 0; i < 4; i++) {
        K[i] = P[i] * a + P[4 + i] * b;
        K[4 + i] = P[i] * a2 + P[4 + i] * b2;
    }
    // rows of (I - K J) restricted to the position columns: L[i][0..1]
    float L[4][2];
    for (int i = 0; i < 4; i++) {
        L[i][0] = (i == 0 ? 1 - K[i] * J[0] : -K[i] * J[0]) - K[4 + i] * J[1];
        L[i][1] = (i == 1 ? 1 - K[i] * J[2] : -K[i] * J[2]) - K[4 + i] * J[3];
    }
    // column j of P (I - K J)' : the two position rows, plus P's own entry for the velocity columns
    for (int j = 0; j < 4; j++) {
        float t0 = P[0] * L[j][0] + P[4] * L[j][1];
        float t1 = P[1] * L[j][0] + P[5] * L[j][1];
        if (j >= 2) {  // the velocity columns carry P's own entry
            t0 = t0 + P[4 * j];
            t1 = t1 + P[4 * j + 1];
        }
        for (int i = 0; i < 4; i++) {
            float v = L[i][0] * t0 + L[i][1] * t1;
            if (i >= 2) {
                v = v + P[i] * L[j][0] + P[4 + i] * L[j][1];
                if (j >= 2) v = v + P[4 * j + i];
            }
            if (i == j) v = v + vr * (K[i] * K[i]) + vb * (K[4 + i] * K[4 + i]);
            else {
                const int lo = i < j ? i : j, hi = i < j ? j : i;
                v = v + K[lo] * vr * K[hi] + K[4 + lo] * vb * K[4 + hi];
            }
            u.cov[4 * j + i] = v;
        }
    }
}

/* partially updated log-weight of a detection term (float sum of the two logs,
 * the rest in double, stored float); -FLT_MAX for the other label */
inline float log_q(const PreUpdate& u, float w, float zr, float zb, bool label_ok, float& i0, float& i1) {
    i0 = zr - u.r;
    i1 = wrap(zb - u.bearing);
    if (!label_ok) return -FLT_MAX;
    const float dist = i0 * i0 * u.S[0] + i0 * i1 * (u.S[1] + u.S[2]) + i1 * i1 * u.S[3];
    const float lw = safe_log(u.pd) + safe_log(w);
    return (float)((double)lw - 0.5 * (double)dist - (double)safe_log((float)(2 * PI)) - 0.5 * (double)safe_log(u.det));
}

/* computeBirth, device form: the inverse measurement, J R J' in float; the 4-D
 * form adds the velocity birth variances */
inline float birth(const phd_slam_config& c, const phd_pose& pose, float zr, float zb, bool label_ok, int dims,
                   float* mean, float* cov) {
    const float th = pose.ptheta + zb;
    float sn_, cs_;
    phd_det_sincosf(th, &sn_, &cs_);  // D16
    const float dx = zr * cs_, dy = zr * sn_;
    mean[0] = pose.px + dx;
    mean[1] = pose.py + dy;
    const float J0 = dx / zr, J1 = dy / zr, J2 = -dy, J3 = dx;
    const float s_r = c.stdRange * c.birthNoiseFactor, s_b = c.stdBearing * c.birthNoiseFactor;
    const float vr = s_r * s_r, vb = s_b * s_b;
    const float xx = (J0 * J0) * vr + (J2 * J2) * vb, xy = J0 * J1 * vr + J2 * J3 * vb,
                yy = (J1 * J1) * vr + (J3 * J3) * vb;
    for (int k = 0; k < dims * dims; k++) cov[k] = 0.0f;
    cov[0] = xx;
    cov[1] = xy;
    cov[dims] = xy;
    cov[dims + 1] = yy;
    if (dims == 4) {
        mean[2] = 0.0f;
        mean[3] = 0.0f;
        cov[10] = c.covVxBirth;
        cov[15] = c.covVyBirth;
    }
    return label_ok ? safe_log(c.birthWeight) : -FLT_MAX;
}

/* predictMapKernelMixed (MIXED_MODEL) with the CV compute_prediction at scale 1 */
inline void predict_cv4(const phd_slam_config& c, const float* m, const float* p, float w, float* mo, float* po,
                        float* wo) {
    const float vmag = std::sqrt(m[2] * m[2] + m[3] * m[3]);
    const float p_jmm = 1 / (1 + phd_det_expf(c.beta * (c.tau - vmag)));
    const float dt = c.dt;
    const float vx = c.stdAxMap * c.stdAxMap * 1.0f, vy = c.stdAyMap * c.stdAyMap * 1.0f;
    const float dt3 = (float)((double)dt * dt * dt), dt4 = (float)((double)dt * dt * dt * dt);  // powf(dt, 3|4)
    mo[0] = m[0] + dt * m[2];
    mo[1] = m[1] + dt * m[3];
    mo[2] = m[2];
    mo[3] = m[3];
    // the entries with a powf term add it in double: powf(dt, k) * var / 0.Ne1
    auto plus = [](float f, float q, double div) { return (float)((double)f + (double)q / div); };
    po[0] = plus(p[0] + p[8] * dt + dt * (p[2] + p[10] * dt), dt4 * vx, 4.0);
    po[1] = p[1] + p[9] * dt + dt * (p[3] + p[11] * dt);
    po[2] = plus(p[2] + p[10] * dt, dt3 * vx, 2.0);
    po[3] = p[3] + p[11] * dt;
    po[4] = p[4] + p[12] * dt + dt * (p[6] + p[14] * dt);
    po[5] = plus(p[5] + p[13] * dt + dt * (p[7] + p[15] * dt), dt4 * vy, 4.0);
    po[6] = p[6] + p[14] * dt;
    po[7] = plus(p[7] + p[15] * dt, dt3 * vy, 2.0);
    po[8] = plus(p[8] + p[10] * dt, dt3 * vx, 2.0);
    po[9] = p[9] + p[11] * dt;
    po[10] = p[10] + vx * dt * dt;
    po[11] = p[11];
    po[12] = p[12] + p[14] * dt;
    po[13] = plus(p[13] + p[15] * dt, dt3 * vy, 2.0);
    po[14] = p[14];
    po[15] = p[15] + vy * dt * dt;
    *wo = p_jmm * c.ps * w;
}

/* force_symmetric_covariance: the lower entry (i, j), i > j, is the average,
 * copied to the upper one */
inline void symmetrize(float* cov, int dims) {
    for (int i = 1; i < dims; i++)
        for (int j = 0; j < i; j++) {
            float& lo = cov[i + j * dims];
            float& up = cov[j + i * dims];
            lo = (lo + up) / 2;
            up = lo;
        }
}

/* gm_reduce.cpp:30-37: sigma = (a + b) / 2 (the LLT reads its lower triangle),
 * L = chol(sigma) column by column, x = L^-1 (ma - mb), |x|^2 — float */
inline float llt_dist4(const float* ma, const float* ca, const float* mb, const float* cb) {
    float L[4][4];
    for (int j = 0; j < 4; j++) {
        float d = 0.5f * (ca[j + 4 * j] + cb[j + 4 * j]);
        for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k];
        L[j][j] = std::sqrt(d);
        for (int i = j + 1; i < 4; i++) {
            float v = 0.5f * (ca[i + 4 * j] + cb[i + 4 * j]);
            for (int k = 0; k < j; k++) v -= L[i][k] * L[j][k];
            L[i][j] = v / L[j][j];
        }
    }
    float x[4], s = 0.0f;
    for (int i = 0; i < 4; i++) {
        float v = ma[i] - mb[i];
        for (int k = 0; k < i; k++) v -= L[i][k] * x[k];
        x[i] = v / L[i][i];
        s += x[i] * x[i];
    }
    return s;
}

}  // namespace orx

#endif
