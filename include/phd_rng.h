/*
 * phd_rng.h — the build's deterministic random-number contract (host + device).
 *
 * The reference draws its noise with a time-seeded boost::mt19937 behind
 * randn()/randu01() (src/rng.cpp:10-13), so its streams cannot be reproduced
 * (SURVEY.md §0.7).  This build replaces them with a counter-based generator so
 * the CPU oracle and the GPU kernels see bit-identical uniforms:
 *
 *   Philox4x32-10 (Salmon et al., SC'11; "Random123"), key = 64-bit seed,
 *   counter = (index, step_lo, step_hi, stream).
 *
 * Uniforms are exact: u = x * 2^-32 in double (boost uniform_01 semantics).
 * Normals use Box-Muller in double; the transcendental calls (log, sqrt, sin,
 * cos) are libm on the host and ocml on the device, so normals agree to an ulp
 * or two of double, which vanishes after the float conversion the filter does.
 *
 * Header-only; compiles as plain C++ (gcc) and as HIP device code.
 */
#ifndef PHD_RNG_H
#define PHD_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define PHD_HD __host__ __device__ inline
#else
#define PHD_HD inline
#endif

#ifdef __cplusplus
#include <cmath>
#define PHD_MATH_NS std::
#else
#include <math.h>
#define PHD_MATH_NS
#endif

/* Stream ids (4th counter word). */
#define PHD_STREAM_PREDICT 0x50524544u  /* 'PRED' */
#define PHD_STREAM_RESAMPLE 0x52534d50u /* 'RSMP' */
#define PHD_STREAM_SYNTH 0x53594e54u    /* 'SYNT' */

typedef struct phd_u32x4 {
    uint32_t v[4];
} phd_u32x4;

PHD_HD void phd_mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

/* Philox4x32 with 10 rounds. */
PHD_HD phd_u32x4 phd_philox4x32_10(phd_u32x4 ctr, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += W0;
            k1 += W1;
        }
        uint32_t hi0, lo0, hi1, lo1;
        phd_mulhilo32(M0, ctr.v[0], &hi0, &lo0);
        phd_mulhilo32(M1, ctr.v[2], &hi1, &lo1);
        phd_u32x4 n;
        n.v[0] = hi1 ^ ctr.v[1] ^ k0;
        n.v[1] = lo1;
        n.v[2] = hi0 ^ ctr.v[3] ^ k1;
        n.v[3] = lo0;
        ctr = n;
    }
    return ctr;
}

PHD_HD phd_u32x4 phd_rng_draw(uint64_t seed, uint32_t index, uint64_t step, uint32_t stream) {
    phd_u32x4 c;
    c.v[0] = index;
    c.v[1] = (uint32_t)step;
    c.v[2] = (uint32_t)(step >> 32);
    c.v[3] = stream;
    return phd_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

/* Uniform on [0,1): exact in double. */
PHD_HD double phd_u01(uint32_t x) { return (double)x * 2.3283064365386963e-10; /* 2^-32 */ }

/* Two standard normals from two 32-bit words (Box-Muller, double). */
PHD_HD void phd_box_muller(uint32_t a, uint32_t b, double* n0, double* n1) {
    const double u1 = ((double)a + 1.0) * 2.3283064365386963e-10; /* (0,1] */
    const double u2 = (double)b * 2.3283064365386963e-10;         /* [0,1) */
    const double rad = PHD_MATH_NS sqrt(-2.0 * PHD_MATH_NS log(u1));
    const double ang = 6.283185307179586476925286766559 * u2;
    *n0 = rad * PHD_MATH_NS cos(ang);
    *n1 = rad * PHD_MATH_NS sin(ang);
}

#endif /* PHD_RNG_H */
