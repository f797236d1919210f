/*
 * phd_synth.cpp — deterministic synthetic replay scenarios for BASELINE.json
 * configs 2-5.  Host-only code; regenerated identically on
 * any machine (std::mt19937_64 + Box-Muller in double, libm sqrt/log/sin/cos).
 *
 * Scenario (one filter step's worth of state, replayed K times by bench.py):
 *   landmarks L_j, j<G, uniform in a disc of radius 0.95*max_range;
 *   particle prior component j: mean L_j + N(0, 0.3^2 I),
 *       cov = [s1^2, r s1 s2; r s1 s2, s2^2], s ~ U(0.2,0.6), r ~ U(-0.3,0.3),
 *       weight ~ U(0.5, 1.0);
 *   particle pose ~ N(0, diag(0.5^2, 0.5^2, 0.02^2)), log-weight -log N;
 *   measurements from the true pose 0: D = round(detect_frac*M) detections of
 *       distinct landmarks (range/bearing noise std_range/std_bearing) then
 *       M-D clutter returns r ~ U(0, max_range), b ~ U(-pi, pi).
 */
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "phd_capi.h"

namespace {

struct Rng {
    std::mt19937_64 g;
    explicit Rng(uint64_t s) : g(s) {}
    double u01() { return (double)(g() >> 11) * (1.0 / 9007199254740992.0); }
    double uni(double a, double b) { return a + (b - a) * u01(); }
    double normal() {
        double u1 = 1.0 - u01();  // (0,1]
        double u2 = u01();
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
    }
};

inline float wrap_pi(double a) {
    while (a > M_PI) a -= 2 * M_PI;
    while (a < -M_PI) a += 2 * M_PI;
    return (float)a;
}

}  // namespace

extern "C" {

/* Preset of BASELINE.json config `id` (2..5): fills cfg and the shape. */
int phd_synth_preset(int id, phd_slam_config* cfg, int* n, int* G, int* M, float* detect_frac) {
    if (!cfg || id < 1 || id > 5) return PHD_E_ARG;
    phd_config_defaults(cfg);
    // cfg/config.cfg of the reference (sensor, Ackerman, filter keys) ...
    cfg->motionType = PHD_MOTION_ACKERMAN;
    cfg->maxBearing = 3.141593f;
    cfg->stdRange = 0.25f;
    cfg->stdBearing = 0.008727f;
    cfg->clutterRate = 20.f;
    cfg->pd = 0.95f;
    cfg->l = 1.415f;
    cfg->h = 0.38f;
    cfg->a = 1.89f;
    cfg->b = 0.5f;
    cfg->stdEncoder = 1.0f;
    cfg->stdAlpha = 0.034907f;
    cfg->dt = 0.1f;
    cfg->filterType = PHD_FILTER_PHD;
    cfg->featureModel = PHD_FEATURE_STATIC;
    cfg->particleWeighting = 0;
    cfg->distanceMetric = 0;
    cfg->subdividePredict = 1;
    cfg->resampleThresh = 0.5f;
    cfg->birthWeight = 0.0001f;
    cfg->birthNoiseFactor = 1.f;
    cfg->gateBirths = false;
    cfg->gateMeasurements = false;
    cfg->minExpectedFeatureWeight = 0.f;
    cfg->minSeparation = 10.f;
    cfg->minFeatureWeight = 0.000001f;
    cfg->nPredictParticles = 1;
    cfg->maxCardinality = 255;
    cfg->mapEstimate = 0;
    // ... with max_range = 50 for the synthetic scenarios
    cfg->maxRange = 50.f;
    int nn = 64, gg = 64, mm = 96;
    float df = 0.75f;
    switch (id) {
        case 1:
            cfg->maxRange = 50.f;
            nn = 64;
            gg = 64;
            mm = 96;
            break;
        case 2:
            nn = 1024;
            gg = 256;
            mm = 32;
            break;
        case 3:
            nn = 4096;
            gg = 512;
            mm = 64;
            cfg->motionType = PHD_MOTION_CV;
            cfg->ax = 0.5f;
            cfg->ay = 0.f;
            cfg->ayaw = 0.0087f;
            cfg->filterType = PHD_FILTER_CPHD;  // config 3 runs the CPHD update
            cfg->maxCardinality = 1023;
            break;
        case 4:
            nn = 32768;
            gg = 512;
            mm = 64;
            break;
        case 5:
            nn = 65536;
            gg = 1024;
            mm = 128;
            cfg->pd = 0.7f;
            df = 0.5f;
            break;
    }
    cfg->n_particles = nn;
    cfg->clutterDensity = cfg->clutterRate / (2 * cfg->maxBearing * cfg->maxRange);
    if (n) *n = nn;
    if (G) *G = gg;
    if (M) *M = mm;
    if (detect_frac) *detect_frac = df;
    return PHD_OK;
}

/* Generate a replay scenario.  maps must hold n*G components; offsets n+1; Z M. */
int phd_synth_scenario(const phd_slam_config* cfg, int n, int G, int M, float detect_frac, uint64_t seed,
                       phd_pose* poses, float* logw, phd_gaussian2d* maps, int* offsets, phd_measurement* Z) {
    if (!cfg || n <= 0 || G < 0 || M < 0 || !poses || !logw || !offsets || (G > 0 && !maps) || (M > 0 && !Z))
        return PHD_E_ARG;
    Rng rng(seed);
    const double R = 0.95 * cfg->maxRange;
    std::vector<double> lx(G), ly(G);
    for (int j = 0; j < G; j++) {
        const double rr = R * std::sqrt(rng.u01());
        const double th = 2 * M_PI * rng.u01();
        lx[j] = rr * std::cos(th);
        ly[j] = rr * std::sin(th);
    }
    const float neglogn = (float)(-std::log((double)n));
    offsets[0] = 0;
    for (int p = 0; p < n; p++) {
        phd_pose s;
        s.px = (float)(0.5 * rng.normal());
        s.py = (float)(0.5 * rng.normal());
        s.ptheta = (float)(0.02 * rng.normal());
        s.vx = s.vy = s.vtheta = 0.f;
        poses[p] = s;
        logw[p] = neglogn;
        for (int j = 0; j < G; j++) {
            phd_gaussian2d& g = maps[(size_t)p * G + j];
            g.mean[0] = (float)(lx[j] + 0.3 * rng.normal());
            g.mean[1] = (float)(ly[j] + 0.3 * rng.normal());
            const double s1 = rng.uni(0.2, 0.6), s2 = rng.uni(0.2, 0.6), rho = rng.uni(-0.3, 0.3);
            g.cov[0] = (float)(s1 * s1);
            g.cov[1] = (float)(rho * s1 * s2);
            g.cov[2] = g.cov[1];
            g.cov[3] = (float)(s2 * s2);
            g.weight = (float)rng.uni(0.5, 1.0);
        }
        offsets[p + 1] = (p + 1) * G;
    }
    const int D = std::min(G, (int)std::lround(detect_frac * M));
    std::vector<int> perm(G);
    std::iota(perm.begin(), perm.end(), 0);
    for (int i = 0; i < D; i++) {  // partial Fisher-Yates
        const int k = i + (int)(rng.u01() * (G - i));
        std::swap(perm[i], perm[std::min(k, G - 1)]);
    }
    for (int m = 0; m < M; m++) {
        phd_measurement& z = Z[m];
        z.label = 0;
        if (m < D) {
            const int j = perm[m];
            const double r = std::sqrt(lx[j] * lx[j] + ly[j] * ly[j]);
            const double b = std::atan2(ly[j], lx[j]);
            z.range = (float)(r + cfg->stdRange * rng.normal());
            z.bearing = wrap_pi(b + cfg->stdBearing * rng.normal());
        } else {
            z.range = (float)rng.uni(0.0, cfg->maxRange);
            z.bearing = (float)rng.uni(-M_PI, M_PI);
        }
    }
    return PHD_OK;
}

}  // extern "C"
