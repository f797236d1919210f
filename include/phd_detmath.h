/*
 * phd_detmath.h — bit-reproducible helpers shared by the GPU resampler and the
 * CPU oracle (host + device, header-only).
 *
 * The reference resampler (src/main.cpp:453-501) walks a double-precision CDF
 * of expf(log-weight) terms.  expf differs by an ulp between libm and the GPU,
 * and a parallel prefix sum in double reorders the additions, so neither gives
 * resample indices that match a CPU run bit for bit.  This build therefore
 * (SURVEY.md §7 hard part 4):
 *   1. evaluates every CDF term with phd_det_expf(): exp in double using only
 *      IEEE-exact operations (+ - * /, floor, ldexp) with FP contraction off,
 *      then rounds to float — the same bits on the CPU and on gfx950;
 *   2. converts each term to unsigned 64-bit fixed point (scale 2^40) so the
 *      CDF is an exact, order-independent integer prefix sum.
 * The faithful double-CDF walk is kept in the oracle and the two are compared
 * in tests (tests/test_oracle_resample.py).
 */
#ifndef PHD_DETMATH_H
#define PHD_DETMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define PHD_DHD __host__ __device__ inline
#else
#define PHD_DHD inline
#endif

#ifdef __cplusplus
#include <cmath>
#define PHD_DNS std::
#else
#include <math.h>
#define PHD_DNS
#endif

#define PHD_FIX_BITS 40
#define PHD_FIX_SCALE 1099511627776.0 /* 2^40 */

/* exp(x) for float x, evaluated in double with exact primitives, rounded to float. */
PHD_DHD float phd_det_expf(float xf) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double x = (double)xf;
    if (!(x == x)) return xf;          /* NaN */
    if (x < -110.0) return 0.0f;       /* below float's smallest subnormal */
    if (x > 89.0) return (float)INFINITY;
    const double inv_ln2 = 1.4426950408889634;
    const double ln2_hi = 0.693147180369123816490;   /* 32 significant bits: k*ln2_hi exact */
    const double ln2_lo = 1.90821492927058770002e-10;
    const double k = PHD_DNS floor(x * inv_ln2 + 0.5);
    const double r = (x - k * ln2_hi) - k * ln2_lo;  /* |r| <= ~0.35 */
    /* Horner Taylor series, degree 13: truncation < 1e-17 relative. */
    double p = 1.0 / 6227020800.0;                   /* 1/13! */
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    return (float)PHD_DNS ldexp(p, (int)k);
}

/*
 * atan2 for float arguments, evaluated in double with IEEE-exact operations
 * only (+ - * /, contraction off) and rounded once to float: the same bits on
 * the CPU and on gfx950, within 0.5 ulp of the true value.  Used for the
 * predicted bearing of every component (phdfilter.cu:1845, :1333), whose
 * ulp-level differences are amplified by 1/sigma_b^2 in the likelihood; the
 * reference evaluated it with CUDA's atan2f (<= 2 ulp), which neither libm nor
 * ocml reproduces bit for bit.
 * Range reduction by a table: with a = min/max of |y|, |x| in [0, 1] and
 * c = k/8 the nearest eighth, atan(a) = atan(c) + atan((a - c) / (1 + a c)),
 * |reduced| <= 1/16, so a degree-15 odd series leaves < 1e-20 relative
 * (one float and one double IEEE division, no square roots: the part A
 * classify evaluates it for every prior component).  phd_atan_eighth(k) =
 * atan(k/8), correctly rounded.
 */
PHD_DHD double phd_atan_eighth(int k) {  /* a table in memory: one load, no constants held in registers */
    static const double T[9] = {0.0,
                                0.12435499454676144,
                                0.24497866312686414,
                                0.35877067027057225,
                                0.4636476090008061,
                                0.5585993153435624,
                                0.6435011087932844,
                                0.7188299996216245,
                                0.7853981633974483};
    return T[k];
}

PHD_DHD float phd_atan2f(float yf, float xf) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double y = (double)yf, x = (double)xf;
    if (!(x == x) || !(y == y)) return xf + yf;
    const double PI = 3.141592653589793238462643383279502884;
    const double ax = PHD_DNS fabs(x), ay = PHD_DNS fabs(y);
    double r;
    if (ax == 0.0 && ay == 0.0) {
        r = (PHD_DNS signbit(x)) ? PI : 0.0;
    } else if (ax == INFINITY || ay == INFINITY) {
        if (ax == INFINITY && ay == INFINITY)
            r = (PHD_DNS signbit(x)) ? 0.75 * PI : 0.25 * PI;
        else if (ay == INFINITY)
            r = 0.5 * PI;
        else
            r = (PHD_DNS signbit(x)) ? PI : 0.0;
    } else {
        const bool swap = ay > ax;
        const double num = swap ? ax : ay, den = swap ? ay : ax;  // a = num / den in [0, 1]
        // k: the nearest eighth of a from the float quotient (IEEE on both
        // sides); k may be one off round(8 a) when 8 a lies within a float ulp
        // of a half, which leaves |u| <= 1/16 + 2^-20, inside the series' range
        const int k = (int)((float)num / (float)den * 8.0f + 0.5f);
        const double tk = phd_atan_eighth(k);  // (issued before the division)
        const double c = (double)k * 0.125;
        // u = (a - c) / (1 + a c) as ONE quotient of exact terms: c den and
        // c num are exact (k / 8 has 4 significant bits, num / den 24), and so
        // are the difference and the sum (28-bit operands within 2^7 of each
        // other when k > 0; k = 0 leaves num / den)
        const double u = (num - c * den) / (den + c * num);  // |u| <= 1/16
        const double u2 = u * u;
        double p = -1.0 / 15.0;
        p = 1.0 / 13.0 + u2 * p;
        p = -1.0 / 11.0 + u2 * p;
        p = 1.0 / 9.0 + u2 * p;
        p = -1.0 / 7.0 + u2 * p;
        p = 1.0 / 5.0 + u2 * p;
        p = -1.0 / 3.0 + u2 * p;
        double t = tk + (u + u * u2 * p);  // atan(a)
        if (swap) t = 0.5 * PI - t;
        r = PHD_DNS signbit(x) ? PI - t : t;
    }
    return (float)(PHD_DNS signbit(y) ? -r : r);
}

/*
 * sin and cos of a float, evaluated in double with IEEE-exact operations only
 * (+ - * floor, contraction off) and each rounded once to float: the same bits
 * on the CPU and on gfx950 (oracle deviation D16).  libm's cosf / sinf and
 * ocml's sincosf are each within an ulp of the true value but not of each
 * other: a birth mean px + r cos(theta + b) one ulp apart moved a merged mean
 * by an ulp and, through the d d' term, its covariance by 1.4e-5 of the
 * matrix scale (config 5, particle 1025).  Used for the birth means
 * (phdfilter.cu:3474-3506) and the predict steps (phdfilter.cu:802-856).
 * Reduction by pi/2 in two parts (Cody-Waite, fdlibm's pio2_1 / pio2_1t: the
 * first part has 33 significant bits, so k pio2_1 is exact for |k| < 2^20,
 * i.e. |x| < 1.6e6); Taylor series on |r| <= pi/4 to r^17 / r^18 (truncation
 * < 1e-19 relative).  Larger |x| (never a pose angle) take libm / ocml.
 */
PHD_DHD double phd_det_sin_kernel(double r, double r2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    double p = 1.0 / 355687428096000.0;  /* 1/17! */
    p = p * r2 - 1.0 / 1307674368000.0;  /* 1/15! */
    p = p * r2 + 1.0 / 6227020800.0;     /* 1/13! */
    p = p * r2 - 1.0 / 39916800.0;       /* 1/11! */
    p = p * r2 + 1.0 / 362880.0;
    p = p * r2 - 1.0 / 5040.0;
    p = p * r2 + 1.0 / 120.0;
    p = p * r2 - 1.0 / 6.0;
    return r + (r * r2) * p;
}

PHD_DHD double phd_det_cos_kernel(double r2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    double p = 1.0 / 6402373705728000.0;  /* 1/18! */
    p = p * r2 - 1.0 / 20922789888000.0;  /* 1/16! */
    p = p * r2 + 1.0 / 87178291200.0;     /* 1/14! */
    p = p * r2 - 1.0 / 479001600.0;       /* 1/12! */
    p = p * r2 + 1.0 / 3628800.0;
    p = p * r2 - 1.0 / 40320.0;
    p = p * r2 + 1.0 / 720.0;
    p = p * r2 - 1.0 / 24.0;
    p = p * r2 + 0.5;
    return 1.0 - r2 * p;
}

/* sin(x), cos(x) of float x in double (see above); returns 0 when the reduction
 * applied, 1 when |x| was too large (the caller's platform fallback). */
PHD_DHD int phd_det_sincos_d(float xf, double* s, double* c) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double x = (double)xf;
    if (!(PHD_DNS fabs(x) < 1.5e6)) return 1;
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
    const double pio2_1t = 6.07710050650619224932e-11; /* pi/2 - pio2_1 */
    const double k = PHD_DNS floor(x * two_over_pi + 0.5);
    const double r = (x - k * pio2_1) - k * pio2_1t;
    const double r2 = r * r;
    const double sr = phd_det_sin_kernel(r, r2), cr = phd_det_cos_kernel(r2);
    const int q = ((int)(k - 4.0 * PHD_DNS floor(k * 0.25)));  /* k mod 4 */
    switch (q) {
        case 0: *s = sr; *c = cr; break;
        case 1: *s = cr; *c = -sr; break;
        case 2: *s = -sr; *c = -cr; break;
        default: *s = -cr; *c = sr; break;
    }
    return 0;
}

PHD_DHD void phd_det_sincosf(float x, float* s, float* c) {
    double sd, cd;
    if (phd_det_sincos_d(x, &sd, &cd)) {
        *s = PHD_DNS sin(x);
        *c = PHD_DNS cos(x);
        return;
    }
    *s = (float)sd;
    *c = (float)cd;
}

PHD_DHD float phd_det_tanf(float x) {
    double sd, cd;
    if (phd_det_sincos_d(x, &sd, &cd)) return PHD_DNS tan(x);
    return (float)(sd / cd);
}

/* Fixed-point CDF term of a float in [0, 2^23). Truncation is exact on both sides. */
PHD_DHD uint64_t phd_fix_term(float t) {
    return (uint64_t)((double)t * PHD_FIX_SCALE);
}

/* Fixed-point stratum position r_j = (j + u_j) / n. */
PHD_DHD uint64_t phd_fix_stratum(int j, double u, int n) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double r = ((double)j + u) / (double)n;
    return (uint64_t)(r * PHD_FIX_SCALE);
}

/* log(x) for float x > 0 in double with exact primitives, rounded once
 * (oracle deviation D14: the mixed model's logarithms, CPU and GPU alike). */
PHD_DHD float phd_det_logf(float xf) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (!(xf > 0.0f)) return xf == 0.0f ? -INFINITY : NAN;
    if (xf == INFINITY) return xf;
    int e = 0;
    double m = PHD_DNS frexp((double)xf, &e);  // m in [0.5, 1)
    if (m < 0.70710678118654752440) {
        m *= 2.0;
        e -= 1;
    }
    const double s = (m - 1.0) / (m + 1.0);  // |s| < 0.1716
    const double s2 = s * s;
    double p = 1.0 / 25.0;  // atanh series: s^27/27 < 3e-21
    p = p * s2 + 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    p = p * s2 + 1.0;
    const double ln2_hi = 0.693147180369123816490, ln2_lo = 1.90821492927058770002e-10;
    const double r = (double)e * ln2_hi + ((double)e * ln2_lo + 2.0 * s * p);
    return (float)r;
}


#endif /* PHD_DETMATH_H */
