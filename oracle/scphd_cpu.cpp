/*
 * scphd_cpu.cpp — CPU ORACLE for the RB-PHD-SLAM static update path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker /
 * the timed CPU baseline — never as part of the shipped product path.
 *
 * What this is: a plain C++ restatement of the reference's algorithm for the
 * hot path, written so that every float/double promotion the reference makes
 * is made here too.  The reference's own CPU entry
 * points (SynthSLAM::predict_cpu / update_cpu, slamtypes.h:335-336, with
 * src/scphd_cpu.cpp empty) were never written, and the CUDA path cannot be
 * built here, so this file follows the CUDA kernels and the
 * host code in the reference line by line (citations per function).
 *
 * Parity pinning: the measurement/motion models are pinned against golden
 * vectors produced by the reference's own Python models
 * (tests/golden/make_golden.py -> tests/golden/models_golden.json).  The
 * reference ships no golden vectors for the update/merge/resample path, so
 * those stages are "parity unpinned" against the reference itself; they are
 * pinned against hand-derived closed forms in tests/test_oracle_*.py.
 *
 * Deliberate, documented deviations:
 *   D1 merge ties: the max-weight search picks the lowest candidate index on
 *      equal weights (the reference's pick depends on its 256-thread layout,
 *      phdfilter.cu:2747-2776);
 *   D2 merge indices are ints (reference stores them in float sdata,
 *      phdfilter.cu:2747-2787, inexact above 2^24);
 *   D3 sums: every reduction (predicted cardinality, normalisers η_m, merge
 *      moments, logSumExp, nEff, expected pose) accumulates float terms in
 *      double and rounds once — the intended exact sum.  The reference's
 *      float tree reductions (sumByReduction, device_math.cuh:452-472) race on
 *      sdata[0] (phdfilter.cu:2201-2210) and are order dependent; a double
 *      accumulation is order independent to ~1e-16, so the GPU's parallel
 *      reduction and this sequential loop round to the same float;
 *   D4 CV noise buffer sized n*nPredict (reference sizes it n, :1123-1127);
 *   D5 resample: fixed-point CDF over det_expf terms (phd_detmath.h); the
 *      faithful double walk (main.cpp:453-501) is orc_resample_faithful();
 *   D6 bearings: atan2 via phd_atan2f (phd_detmath.h), a shared correctly
 *      rounded routine, where the reference used CUDA atan2f (<= 2 ulp);
 *   D15 a merge set of one member (the seed alone) is emitted as that member,
 *      its covariance symmetrised, instead of the one-member moments
 *      ((w x) / w, (w (P + d d')) / w: within an ulp of it; the reference's own
 *      float tree sums are order dependent at that level, D3);
 *   D17 the PHD normalisers' logs log(eta_m) and log(birthWeight) by
 *      phd_det_logf (phd_detmath.h), as the GPU: every clutter-only
 *      measurement of a scan gives its birth the same weight beta / eta_m, an
 *      exact tie the merge breaks by candidate index (D1), and libm's and
 *      ocml's logf (each within an ulp, not of each other) map normalisers an
 *      ulp apart to one log on one side and two on the other — the tie groups,
 *      hence the merge sets, then differ (config 1, scan 36).
 *   D18 the EKF's Jacobian (dx / r, dy / r, dy / r^2, dx / r^2) and the
 *      2x2 inverses of the innovation covariance and of computeMahalDist's
 *      summed covariance (four quotients s_k / det each) from reciprocals:
 *      x * (1 / r), s_k * (1 / det) — and the merged moments Σ w x / W,
 *      Σ w (P + d d') / W as products with 1 / W, the CPHD non-detection
 *      weight exp(log w + lnd) as w * phd_det_expf(lnd) — within an ulp or two of the quotients,
 *      as the GPU computes them (its IEEE divisions cost ~10 instructions
 *      each; the reference's own nvcc build contracts a*b+c into FMAs, so it
 *      is reproducible only to that level anyway).
 *
 * Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fno-fast-math).
 */
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <vector>

#include <omp.h>

#include "phd_detmath.h"
#include "mixed_ref.h"  // the oracle's own restatement of the mixed-model arithmetic
#include "phd_rng.h"
#include "phd_types.h"

namespace {

typedef phd_gaussian2d G2;

const float LOG0 = -FLT_MAX;  // slamtypes.h:26

/* device_math.cuh:9-16 */
inline float safeLog(float x) { return x <= 0 ? LOG0 : std::log(x); }
/* safeLog of the PHD normalisers and of the birth weight by phd_det_logf
 * (deviation D17, as the GPU): normalisers one float ulp apart must map to one
 * log or two on both sides alike, or the exact ties among the birth weights
 * beta / eta_m (every clutter-only measurement of a scan) — broken by candidate
 * index in the merge (D1) — differ between the two. */
inline float detSafeLog(float x) { return x <= 0 ? LOG0 : phd_det_logf(x); }

/* device_math.cuh:242-251: fmod in float, comparisons/±2pi in double, back to float. */
inline float wrapAngle(float a) {
    float remainder = std::fmod(a, (float)(2 * M_PI));
    double r = remainder;
    if (r > M_PI)
        remainder = (float)(r - 2 * M_PI);
    else if (r < -M_PI)
        remainder = (float)(r + 2 * M_PI);
    return remainder;
}

/* Per-particle bookkeeping of how close each threshold decision came to flipping. */
/* Margin of one particle's threshold decisions: m = the closest relative
 * distance of any decision to its threshold; `cls` / `pm` count the decisions
 * within NEAR of their threshold — range classification (which also moves the
 * log-weight) and prune / merge (which only move the map components they touch). */
struct Margin {
    static constexpr double NEAR = 1e-4;
    float m = FLT_MAX;
    int cls = 0, pm = 0;
    inline void rel(double v, double thr, bool classification = false) {
        double s = std::fabs(thr) > 0 ? std::fabs(v - thr) / std::fabs(thr) : std::fabs(v - thr);
        if (s < m) m = (float)s;
        if (s < NEAR) (classification ? cls : pm)++;
    }
};
std::vector<int> g_near_counts;  // per particle of the last orc_update_cn: cls | pm << 16

/* EKF terms of one in-range component (phdfilter.cu:1836-1895). */
struct Ekf {
    float r, bearing, pd, det;
    float S[4], K[4], cov_update[4];
};

inline void compute_ekf(const phd_slam_config& cfg, const phd_pose& pose, const G2& f, Ekf& e) {
    float dx = f.mean[0] - pose.px;
    float dy = f.mean[1] - pose.py;
    float r2 = dx * dx + dy * dy;
    float r = std::sqrt(r2);
    float bearing = wrapAngle(phd_atan2f(dy, dx) - pose.ptheta);
    float pd = 0;
    if (r <= cfg.maxRange && std::fabs(bearing) <= cfg.maxBearing) pd = cfg.pd;
    float J[4];
    const float ir = 1.0f / r, ir2 = ir * ir;  // (D18: reciprocals, as the GPU)
    J[0] = dx * ir;
    J[2] = dy * ir;
    J[1] = -dy * ir2;
    J[3] = dx * ir2;
    const float* P = f.cov;
    const float sR2 = cfg.stdRange * cfg.stdRange;   // pow(stdRange,2), float overload
    const float sB2 = cfg.stdBearing * cfg.stdBearing;
    float sigma[4];
    sigma[0] = (P[0] * J[0] + J[2] * P[1]) * J[0] + (J[0] * P[2] + P[3] * J[2]) * J[2] + sR2;
    sigma[1] = (P[0] * J[1] + J[3] * P[1]) * J[0] + (J[1] * P[2] + P[3] * J[3]) * J[2];
    sigma[2] = (P[0] * J[0] + J[2] * P[1]) * J[1] + (J[0] * P[2] + P[3] * J[2]) * J[3];
    sigma[3] = (P[0] * J[1] + J[3] * P[1]) * J[1] + (J[1] * P[2] + P[3] * J[3]) * J[3] + sB2;
    sigma[1] = (sigma[1] + sigma[2]) / 2;
    sigma[2] = sigma[1];
    float det = sigma[0] * sigma[3] - sigma[1] * sigma[2];
    float* S = e.S;
    const float id = 1.0f / det;  // (D18)
    S[0] = sigma[3] * id;
    S[1] = -sigma[1] * id;
    S[2] = -sigma[2] * id;
    S[3] = sigma[0] * id;
    float* K = e.K;
    K[0] = S[0] * (P[0] * J[0] + P[2] * J[2]) + S[1] * (P[0] * J[1] + P[2] * J[3]);
    K[1] = S[0] * (P[1] * J[0] + P[3] * J[2]) + S[1] * (P[1] * J[1] + P[3] * J[3]);
    K[2] = S[2] * (P[0] * J[0] + P[2] * J[2]) + S[3] * (P[0] * J[1] + P[2] * J[3]);
    K[3] = S[2] * (P[1] * J[0] + P[3] * J[2]) + S[3] * (P[1] * J[1] + P[3] * J[3]);
    // Joseph-form covariance, same association as phdfilter.cu:1891-1894.
    const float sR = cfg.stdRange, sB = cfg.stdBearing;
    float a00 = 1 - K[0] * J[0] - K[2] * J[1];
    float a01 = -K[0] * J[2] - K[2] * J[3];
    float a10 = -K[1] * J[0] - K[3] * J[1];
    float a11 = 1 - K[1] * J[2] - K[3] * J[3];
    float* cu = e.cov_update;
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
    e.pd = pd;
    e.det = det;
}

/* Single-object log-likelihood term g (phdfilter.cu:1907-1911): evaluated in double, stored float. */
inline float log_g(float dist, float det) {
    return (float)(-0.5 * (double)dist - (double)safeLog((float)(2 * M_PI)) - 0.5 * (double)safeLog(det));
}

/* computeMahalDist (device_math.cuh:309-325) with invert_matrix2 (:57-65). */
inline float mahal(const G2& a, const G2& b) {
    float sigma[4], si[4];
    for (int i = 0; i < 4; i++) sigma[i] = (a.cov[i] + b.cov[i]) / 2;
    float det = sigma[0] * sigma[3] - sigma[2] * sigma[1];
    const float rd = 1.0f / det;  // (D18)
    si[0] = sigma[3] * rd;
    si[1] = -sigma[1] * rd;
    si[2] = -sigma[2] * rd;
    si[3] = sigma[0] * rd;
    float i0 = a.mean[0] - b.mean[0];
    float i1 = a.mean[1] - b.mean[1];
    return i0 * i0 * si[0] + i0 * i1 * (si[1] + si[2]) + i1 * i1 * si[3];
}

/* Births from measurements (host loop phdfilter.cu:3466-3510). */
inline G2 compute_birth(const phd_slam_config& cfg, const phd_pose& pose, const phd_measurement& z) {
    G2 b;
    float theta = pose.ptheta + z.bearing;
    float sn, cs;
    phd_det_sincosf(theta, &sn, &cs);  // D16: sin / cos in double, rounded once (GPU: the same bits)
    float dx = z.range * cs;
    float dy = z.range * sn;
    b.mean[0] = pose.px + dx;
    b.mean[1] = pose.py + dy;
    float J[4];
    const float izr = 1.0f / z.range;  // (D18)
    J[0] = dx * izr;
    J[1] = dy * izr;
    J[2] = -dy;
    J[3] = dx;
    // std::pow(float,int) promotes to double (C++11); pow(x,2) is restated as the
    // correctly rounded double square x*x.
    const double vr = (double)(cfg.stdRange * cfg.birthNoiseFactor);
    const double vb = (double)(cfg.stdBearing * cfg.birthNoiseFactor);
    float var_range = (float)(vr * vr);
    float var_bearing = (float)(vb * vb);
    b.cov[0] = (float)((double)J[0] * (double)J[0] * (double)var_range +
                       (double)J[2] * (double)J[2] * (double)var_bearing);
    b.cov[1] = J[0] * J[1] * var_range + J[2] * J[3] * var_bearing;
    b.cov[2] = b.cov[1];
    b.cov[3] = (float)((double)J[1] * (double)J[1] * (double)var_range +
                       (double)J[3] * (double)J[3] * (double)var_bearing);
    if (z.label == PHD_MEAS_STATIC || !cfg.labeledMeasurements)
        b.weight = detSafeLog(cfg.birthWeight);  // (D17)
    else
        b.weight = safeLog(0);
    return b;
}

/*
 * Greedy GM merge of one particle's candidates (phdUpdateMergeKernel,
 * phdfilter.cu:2739-2890).  Appends merged components to `out` in selection
 * order.  Sums are sequential in candidate order.
 */
void merge_candidates(const phd_slam_config& cfg, const std::vector<G2>& cand, std::vector<G2>& out,
                      Margin& mg) {
    const size_t n = cand.size();
    std::vector<char> merged(n, 0);
    std::vector<float> dist(n);
    const float T = cfg.minSeparation;
    while (true) {
        long best = -1;
        for (size_t i = 0; i < n; i++) {
            if (merged[i]) continue;
            if (best < 0 || cand[best].weight < cand[i].weight) best = (long)i;  // D1: first max
        }
        if (best < 0) break;
        const G2 mx = cand[best];
        double Wd = 0, m0 = 0, m1 = 0;
        int members = 0;
        for (size_t i = 0; i < n; i++) {
            if (merged[i]) continue;
            float d = mahal(mx, cand[i]);
            dist[i] = d;
            if ((long)i != best) mg.rel(d, T);
            if (d < T) {
                Wd += (double)cand[i].weight;
                m0 += (double)(cand[i].weight * cand[i].mean[0]);
                m1 += (double)(cand[i].weight * cand[i].mean[1]);
                members++;
            }
        }
        const float W = (float)Wd;
        if (W == 0) break;
        if (members == 1 && dist[best] < T) {  // D15: the seed alone
            G2 g = mx;
            g.cov[1] = (g.cov[1] + g.cov[2]) / 2;
            g.cov[2] = g.cov[1];
            merged[best] = 1;
            out.push_back(g);
            continue;
        }
        G2 g;
        g.weight = W;
        const float rW = 1.0f / W;  // (D18)
        g.mean[0] = (float)m0 * rW;
        g.mean[1] = (float)m1 * rW;
        double c[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < n; i++) {
            if (merged[i]) continue;
            if (dist[i] < T) {
                float d0 = g.mean[0] - cand[i].mean[0];
                float d1 = g.mean[1] - cand[i].mean[1];
                const float w = cand[i].weight;
                c[0] += (double)(w * (cand[i].cov[0] + d0 * d0));
                c[1] += (double)(w * (cand[i].cov[1] + d0 * d1));
                c[2] += (double)(w * (cand[i].cov[2] + d1 * d0));
                c[3] += (double)(w * (cand[i].cov[3] + d1 * d1));
                merged[i] = 1;
            }
        }
        for (int k = 0; k < 4; k++) g.cov[k] = (float)c[k] * rW;
        // force_symmetric_covariance (device_math.cuh:710-725)
        g.cov[1] = (g.cov[1] + g.cov[2]) / 2;
        g.cov[2] = g.cov[1];
        out.push_back(g);
    }
}

std::vector<G2> g_debug_cand;
int g_debug_particle = -1;
long g_max_cand = 0;  // largest merge candidate list of the last orc_update (capacity sizing)

/* ---- A12: CPHD (Vo, Vo & Cantoni analytic GM-CPHD) as the reference states it
 * in its commented-out kernels (phdfilter.cu:1360-1820; older copy
 * phdfilter.cu.bak:369-545, 990-1504) with the Poisson predicted cardinality of
 * the host code (.bak:2473-2497).  Direct formulas, all in double:
 *   W = Σ w over the whole predicted map, cn_pred[n] = n log W - W - log n!
 *   <1,w>, <q_D,w> over the in-range components
 *   Λ_m = Σ_j pd w_j N(z_m) · clutterRate / clutterDensity      (computeEsfKernel)
 *   e_k(Λ), e_k(Λ \ z_m)                                         (ESF, ESFd)
 *   Ψ0, Ψ1, Ψ1d_m(n) and their inner products with cn_pred      (computePsiKernel)
 *   cn_update[n] = cn_pred[n] + Ψ0(n) - <Ψ0,p>;  Δ log w = <Ψ0,p>
 * Deviations (D9): the ESFs are computed as the exact positive
 * recursion in log space (the reference's commented kernels subtract in the
 * linear domain, which overflows fp32 at M=64, and the .bak variant takes |a-b|
 * of log terms); Ψ1d's log-sum-exp uses its own maximum (.bak:1476 uses Ψ0's).
 * Births are not part of the CPHD update array (as in .bak, where births enter
 * through the prediction). */
double lse_add(double a, double b) {
    if (a == -INFINITY) return b;
    if (b == -INFINITY) return a;
    const double m = a > b ? a : b;
    return m + std::log(std::exp(a - m) + std::exp(b - m));
}

void esf_log(const std::vector<double>& lam, int skip, std::vector<double>& e) {
    const int M = (int)lam.size();
    e.assign(M + 1, -INFINITY);
    e[0] = 0.0;
    int k = 0;
    for (int m = 0; m < M; m++) {
        if (m == skip) continue;
        k++;
        for (int q = k; q >= 1; q--) e[q] = lse_add(e[q], lam[m] + e[q - 1]);
    }
}

struct CphdOut {
    double ip0, ip1;
    std::vector<double> ip1d, cn_update;
};

/* logq: G x M (float, as the PHD path), w_in: in-range weights, pd_in: their pd,
 * W: Σ w over the whole map.  Nmax = maxCardinality. */
void cphd_terms(const phd_slam_config& cfg, int G, int M, const std::vector<float>& logq, const std::vector<G2>& in,
                const std::vector<float>& pd_in, double W, CphdOut& o) {
    const int Nmax = cfg.maxCardinality;
    std::vector<double> lf(std::max(Nmax, M) + 2);
    lf[0] = 0;
    for (size_t i = 1; i < lf.size(); i++) lf[i] = lf[i - 1] + std::log((double)i);
    const double lrate = std::log((double)cfg.clutterRate), lck = lrate - std::log((double)cfg.clutterDensity);
    double win = 0, qd = 0;
    for (int j = 0; j < G; j++) {
        win += (double)in[j].weight;
        qd += (double)(1 - pd_in[j]) * (double)in[j].weight;
    }
    const double lw = win > 0 ? std::log(win) : -INFINITY;
    const double lq = qd > 0 ? std::log(qd) : -INFINITY;
    const double logW = W > 0 ? std::log(W) : -INFINITY;
    std::vector<double> lam(M);
    for (int m = 0; m < M; m++) {
        double sm = 0;
        for (int j = 0; j < G; j++) sm += (double)std::exp(logq[(size_t)j * M + m]);
        lam[m] = sm > 0 ? std::log(sm) + lck : -INFINITY;
    }
    std::vector<double> e, ed;
    esf_log(lam, -1, e);
    auto cn_pred = [&](int n) { return (n == 0 ? 0.0 : n * logW) - W - lf[n]; };
    auto clut = [&](int k) { return (k == 0 ? 0.0 : k * lrate) - cfg.clutterRate - lf[k]; };  // log Poisson
    // n-th power terms: (n - j) lq - n lw with 0 * (-inf) = 0
    auto pw = [&](int n, int jj) {
        double t = 0;
        if (n - jj > 0) t += (n - jj) * lq;
        if (n > 0) t -= n * lw;
        return t;
    };
    std::vector<double> psi0(Nmax + 1), psi1(Nmax + 1);
    for (int n = 0; n <= Nmax; n++) {
        double a0 = -INFINITY, a1 = -INFINITY;
        if (cn_pred(n) == -INFINITY) {  // p(n) = 0 (an empty map predicts n = 0 only): no term, no ∞ - ∞
            psi0[n] = psi1[n] = -INFINITY;
            continue;
        }
        for (int j = 0; j <= std::min(n, M); j++) {
            if (e[j] == -INFINITY) continue;
            const double aux = lf[M - j] + clut(M - j) + e[j];
            a0 = lse_add(a0, aux + (lf[n] - lf[n - j]) + pw(n, j));
            if (j + 1 <= n) a1 = lse_add(a1, aux + (lf[n] - lf[n - j - 1]) + pw(n, j + 1));
        }
        psi0[n] = a0;
        psi1[n] = a1;
    }
    o.ip0 = -INFINITY;
    o.ip1 = -INFINITY;
    for (int n = 0; n <= Nmax; n++) {
        o.ip0 = lse_add(o.ip0, psi0[n] + cn_pred(n));
        o.ip1 = lse_add(o.ip1, psi1[n] + cn_pred(n));
    }
    o.cn_update.resize(Nmax + 1);
    for (int n = 0; n <= Nmax; n++) o.cn_update[n] = cn_pred(n) == -INFINITY ? -INFINITY : cn_pred(n) + psi0[n] - o.ip0;
    o.ip1d.assign(M, -INFINITY);
    for (int t = 0; t < M; t++) {
        esf_log(lam, t, ed);
        double acc = -INFINITY;
        for (int n = 0; n <= Nmax; n++) {
            if (cn_pred(n) == -INFINITY) continue;
            double a = -INFINITY;
            for (int j = 0; j <= std::min(n, M - 1); j++) {
                if (ed[j] == -INFINITY || j + 1 > n) continue;
                a = lse_add(a, lf[M - 1 - j] + clut(M - 1 - j) + ed[j] + (lf[n] - lf[n - j - 1]) + pw(n, j + 1));
            }
            acc = lse_add(acc, a + cn_pred(n));
        }
        o.ip1d[t] = acc;
    }
}

}  // namespace

extern "C" {

/* Debug: remember the merge candidates of particle p during the next orc_update. */
void orc_debug_select(int p) { g_debug_particle = p; }
long orc_max_candidates(int reset) {
    const long v = g_max_cand;
    if (reset) g_max_cand = 0;
    return v;
}
long orc_debug_candidates(phd_gaussian2d* out, long cap) {
    long n = (long)g_debug_cand.size();
    for (long i = 0; i < n && i < cap; i++) out[i] = g_debug_cand[i];
    return n;
}

/* OpenMP threads of the per-particle update loop (0 = the runtime default). */
int orc_set_threads(int t) {
    if (t > 0) omp_set_num_threads(t);
    return omp_get_max_threads();
}

/* ---- scalar helpers exported for the golden tests ---- */
float orc_wrap_angle(float a) { return wrapAngle(a); }
float orc_safe_log(float x) { return safeLog(x); }
float orc_det_expf(float x) { return phd_det_expf(x); }
float orc_atan2f(float y, float x) { return phd_atan2f(y, x); }
void orc_sincosf(float x, float* s, float* c) { phd_det_sincosf(x, s, c); }
float orc_tanf(float x) { return phd_det_tanf(x); }

void orc_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out) {
    phd_u32x4 c = {{c0, c1, c2, c3}};
    phd_u32x4 r = phd_philox4x32_10(c, k0, k1);
    for (int i = 0; i < 4; i++) out[i] = r.v[i];
}

/* Range-bearing h(x) (phdfilter.cu:1841-1845). out = (range, bearing). */
void orc_measure(const phd_pose* pose, float fx, float fy, float* out) {
    float dx = fx - pose->px, dy = fy - pose->py;
    float r = std::sqrt(dx * dx + dy * dy);
    out[0] = r;
    out[1] = wrapAngle(phd_atan2f(dy, dx) - pose->ptheta);
}

/* Inverse measurement (birth mean + covariance + log-weight) for one measurement. */
void orc_birth(const phd_slam_config* cfg, const phd_pose* pose, const phd_measurement* z, phd_gaussian2d* out) {
    *out = compute_birth(*cfg, *pose, *z);
}

/* ---- noise generation with the build's RNG contract ---- */
void orc_noise_ackerman(const phd_slam_config* cfg, int n, uint64_t seed, uint64_t step, phd_ackerman_noise* out) {
    for (int i = 0; i < n; i++) {
        phd_u32x4 x = phd_rng_draw(seed, (uint32_t)i, step, PHD_STREAM_PREDICT);
        double g0, g1;
        phd_box_muller(x.v[0], x.v[1], &g0, &g1);
        out[i].n_alpha = (float)(cfg->stdAlpha * g0);      // phdfilter.cu:1148-1152
        out[i].n_encoder = (float)(cfg->stdEncoder * g1);
    }
}

void orc_noise_cv(const phd_slam_config* cfg, int n, uint64_t seed, uint64_t step, phd_cv_noise* out) {
    for (int i = 0; i < n; i++) {
        phd_u32x4 x = phd_rng_draw(seed, (uint32_t)i, step, PHD_STREAM_PREDICT);
        double g0, g1, g2, g3;
        phd_box_muller(x.v[0], x.v[1], &g0, &g1);
        phd_box_muller(x.v[2], x.v[3], &g2, &g3);
        (void)g3;
        out[i].ax = (float)(3 * cfg->ax * g0);               // phdfilter.cu:1112-1118
        out[i].ay = (float)(3 * cfg->ay * g1);
        out[i].atheta = (float)(3 * cfg->ayaw * g2);
    }
}

void orc_resample_uniforms(int n, uint64_t seed, uint64_t step, double* out) {
    for (int j = 0; j < n; j++) {
        phd_u32x4 x = phd_rng_draw(seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
        out[j] = phd_u01(x.v[0]);
    }
}

/* ---- A1: Ackerman predict (phdPredictKernelAckerman, phdfilter.cu:785-825) ---- */
void orc_predict_ackerman(const phd_slam_config* cfg, int n_predict, const phd_pose* prior,
                          phd_ackerman_control control, const phd_ackerman_noise* noise, phd_pose* out) {
    const phd_slam_config& c = *cfg;
    for (int idx = 0; idx < n_predict; idx++) {
        int prior_idx = (int)std::floor((float)idx / c.nPredictParticles);
        phd_pose s = prior[prior_idx], ns;
        float ve = control.v_encoder + noise[idx].n_encoder;
        float al = control.alpha + noise[idx].n_alpha;
        // D16: tan / sin / cos in double with exact primitives, rounded once (phd_detmath.h)
        const float ta = phd_det_tanf(al);
        float st, ct;
        phd_det_sincosf(s.ptheta, &st, &ct);
        float vc = ve / (1 - ta * c.h / c.l);
        float xc_dot = vc * ct;
        float yc_dot = vc * st;
        float thetac_dot = vc * ta / c.l;
        float dt = c.dt / c.subdividePredict;
        ns.px = s.px + dt * (xc_dot - thetac_dot * (c.a * st + c.b * ct));
        ns.py = s.py + dt * (yc_dot + thetac_dot * (c.a * ct - c.b * st));
        ns.ptheta = wrapAngle(s.ptheta + dt * thetac_dot);
        ns.vx = 0;
        ns.vy = 0;
        ns.vtheta = 0;
        out[idx] = ns;
    }
}

/* ---- A2: constant-velocity predict (phdPredictKernel, phdfilter.cu:827-859) ---- */
void orc_predict_cv(const phd_slam_config* cfg, int n_predict, const phd_pose* prior, const phd_cv_noise* noise,
                    phd_pose* out) {
    const phd_slam_config& c = *cfg;
    for (int idx = 0; idx < n_predict; idx++) {
        int prior_idx = (int)std::floor((float)idx / c.nPredictParticles);
        phd_pose s = prior[prior_idx], ns;
        float dt = c.dt / c.subdividePredict;
        const phd_cv_noise& w = noise[idx];
        float ct, st;
        phd_det_sincosf(s.ptheta, &st, &ct);  // D16
        ns.px = (float)((double)(s.px + dt * (s.vx * ct - s.vy * st)) +
                        (double)(dt * dt) * 0.5 * (double)(w.ax * ct - w.ay * st));
        ns.py = (float)((double)(s.py + dt * (s.vx * st + s.vy * ct)) +
                        (double)(dt * dt) * 0.5 * (double)(w.ax * st + w.ay * ct));
        ns.ptheta = wrapAngle((float)((double)(s.ptheta + dt * s.vtheta) + 0.5 * dt * dt * (double)w.atheta));
        ns.vx = s.vx + dt * w.ax;
        ns.vy = s.vy + dt * w.ay;
        ns.vtheta = s.vtheta + dt * w.atheta;
        out[idx] = ns;
    }
}

/*
 * ---- A3..A8: static PHD update for n particles (phdUpdateSynth, phdfilter.cu:3336-3761) ----
 *
 * maps_in:  CSR (Gaussian2D AoS) with offsets_in[n+1].
 * maps_out: caller-allocated AoS of capacity out_cap; offsets_out[n+1] filled.
 * delta:    per-particle Δlog w (particle_weighting = 0, phdfilter.cu:2264-2268).
 * margin:   per-particle minimum relative distance of any threshold decision to its threshold.
 * Returns the total number of output components, or -1 on overflow / unsupported config.
 * Does NOT touch the particle weights (see orc_normalize).
 */
}  // extern "C"

namespace {

/* One particle of the update (the body of phdUpdateSynth's per-particle work);
 * particles are independent, so orc_update_cn runs them in parallel (OpenMP)
 * and concatenates the results in particle order. */
struct ParticleOut {
    std::vector<G2> maps;  // merged candidates, then the out-of-range components
    float delta = 0, margin = FLT_MAX;
    int near = 0;
};

void update_particle(const phd_slam_config& cfg, int p, const phd_pose& pose, const G2* comps, int ncomp,
                     const phd_measurement* Zin, int M, double* cn_row, ParticleOut& po) {
    const bool cphd = cfg.filterType == PHD_FILTER_CPHD;
    const float kappa = cfg.clutterDensity, beta = cfg.birthWeight;
    std::vector<G2> in, out1, out2, cand;
    std::vector<Ekf> ekf;
    std::vector<float> logq;
    Margin mg;
    // A3: classification (computeInRangeKernel :1328-1346)
    for (int k = 0; k < ncomp; k++) {
        const G2& f = comps[k];
        float dx = f.mean[0] - pose.px, dy = f.mean[1] - pose.py;
        float r = std::sqrt(dx * dx + dy * dy);
        float bearing = wrapAngle(phd_atan2f(dy, dx) - pose.ptheta);
        float ab = std::fabs(bearing);
        mg.rel(r, cfg.maxRange, true);
        if (cfg.minRange > 0) mg.rel(r, cfg.minRange, true);
        if (cfg.maxBearing < (float)M_PI) mg.rel(ab, cfg.maxBearing, true);
        if (r >= cfg.minRange && r <= cfg.maxRange && ab <= cfg.maxBearing) {
            in.push_back(f);
        } else if ((double)r >= 0.8 * cfg.minRange && (double)r <= 1.2 * cfg.maxRange &&
                   (double)ab <= 1.2 * cfg.maxBearing) {
            mg.rel(r, 1.2 * cfg.maxRange, true);
            out2.push_back(f);
        } else {
            mg.rel(r, 1.2 * cfg.maxRange, true);
            out1.push_back(f);
        }
    }
    const int G = (int)in.size();
    // A5: pre-update (preUpdateSynthKernel)
    ekf.resize(G);
    logq.assign((size_t)G * M, 0.f);
    double card_d = 0;  // Σ pd·w + M·β  (phdfilter.cu:2148-2186)
    for (int j = 0; j < G; j++) {
        compute_ekf(cfg, pose, in[j], ekf[j]);
        const Ekf& e = ekf[j];
        for (int m = 0; m < M; m++) {
            float i0 = Zin[m].range - e.r;
            float i1 = wrapAngle(Zin[m].bearing - e.bearing);
            float dist = i0 * i0 * e.S[0] + i0 * i1 * (e.S[1] + e.S[2]) + i1 * i1 * e.S[3];
            float g = log_g(dist, e.det);
            if (Zin[m].label == PHD_MEAS_STATIC || !cfg.labeledMeasurements)
                logq[(size_t)j * M + m] = safeLog(e.pd) + safeLog(in[j].weight) + g;
            else
                logq[(size_t)j * M + m] = safeLog(0);
        }
        card_d += (double)(e.pd * in[j].weight);
    }
    for (int m = 0; m < M; m++) card_d += (double)beta;
    const float card = (float)card_d;
    CphdOut co;
    if (cphd) {
        double W = 0;  // whole predicted map (.bak:2486-2488)
        for (int k = 0; k < ncomp; k++) W += (double)comps[k].weight;
        std::vector<float> pd_in(G);
        for (int j = 0; j < G; j++) pd_in[j] = ekf[j].pd;
        cphd_terms(cfg, G, M, logq, in, pd_in, W, co);
        if (cn_row)
            for (int k = 0; k <= cfg.maxCardinality; k++) cn_row[k] = co.cn_update[k];
    }
    const double lck = std::log((double)cfg.clutterRate) - std::log((double)cfg.clutterDensity);
    // A6: weights (phdUpdateKernel :2190-2253)
    float pw = 0;
    std::vector<float> logeta(M);
    for (int m = 0; m < M; m++) {
        float sum = 0;
        if (G > 0) {
            double sd = 0;
            for (int j = 0; j < G; j++) sd += (double)std::exp(logq[(size_t)j * M + m]);
            sd += (double)kappa;
            sd += (double)beta;
            sum = (float)sd;
        } else {
            sum = kappa + beta;
        }
        logeta[m] = detSafeLog(sum);  // (D17)
        pw += logeta[m];
        if (cphd) logeta[m] = (float)((co.ip0 - co.ip1d[m]) - lck);  // detection factor (cphdUpdateKernel)
    }
    // candidates in the reference's update-array order: [nondetect | detect (m-major) | births]
    const float minw = cfg.minFeatureWeight;
    const float lnd = cphd ? (float)(co.ip1 - co.ip0 + (double)safeLog(1 - cfg.pd)) : 0.f;
    const float e_nd = phd_det_expf(lnd);  // (D18: exp(log w + lnd) as w e^lnd, e^lnd once)
    for (int j = 0; j < G; j++) {
        G2 g = in[j];
        if (cphd)
            g.weight = g.weight > 0 ? g.weight * e_nd : 0.f;  // non-detection (cphdUpdateKernel; D18)
        else
            g.weight *= (1 - ekf[j].pd);
        mg.rel(g.weight, minw);
        if (!(g.weight < minw)) cand.push_back(g);
    }
    for (int m = 0; m < M; m++) {
        for (int j = 0; j < G; j++) {
            const Ekf& e = ekf[j];
            float i0 = Zin[m].range - e.r;
            float i1 = wrapAngle(Zin[m].bearing - e.bearing);
            G2 g;
            g.mean[0] = in[j].mean[0] + e.K[0] * i0 + e.K[2] * i1;
            g.mean[1] = in[j].mean[1] + e.K[1] * i0 + e.K[3] * i1;
            for (int k = 0; k < 4; k++) g.cov[k] = e.cov_update[k];
            g.weight = std::exp(logq[(size_t)j * M + m] - logeta[m]);
            if (g.weight > 1e-12f) mg.rel(g.weight, minw);
            if (!(g.weight < minw)) cand.push_back(g);
        }
    }
    for (int m = 0; m < M && !cphd; m++) {
        G2 b = compute_birth(cfg, pose, Zin[m]);
        b.weight = std::exp(b.weight - logeta[m]);
        mg.rel(b.weight, minw);
        if (!(b.weight < minw)) cand.push_back(b);
    }
    for (const G2& g : out2) cand.push_back(g);  // interleave (mergeAndCopyMaps :3227-3257)
#pragma omp critical(orc_maxcand)
    g_max_cand = std::max(g_max_cand, (long)cand.size());
    if (p == g_debug_particle) {
#pragma omp critical(orc_debug)
        g_debug_cand = cand;
    }
    // A8: merge + append out1
    po.maps.clear();
    merge_candidates(cfg, cand, po.maps, mg);
    for (const G2& g : out1) po.maps.push_back(g);
    po.delta = cphd ? (float)co.ip0 : pw - card;
    po.margin = mg.m;
    po.near = std::min(mg.cls, 0xffff) | (std::min(mg.pm, 0x7fff) << 16);
}

}  // namespace

extern "C" {

long orc_update_cn(const phd_slam_config* cfgp, int n, const phd_pose* poses, const phd_gaussian2d* maps_in,
                   const int* offsets_in, const phd_measurement* Zin, int n_measure, phd_gaussian2d* maps_out,
                   long out_cap, int* offsets_out, float* delta, float* margin, double* cn_out) {
    const phd_slam_config& cfg = *cfgp;
    if (cfg.distanceMetric != 0 || cfg.particleWeighting != 0 || cfg.featureModel != PHD_FEATURE_STATIC) return -1;
    const bool cphd = cfg.filterType == PHD_FILTER_CPHD;
    if (cphd && cfg.maxCardinality < 0) return -1;
    const int M = std::min(n_measure, 256);  // phdfilter.cu:3390-3394
    g_near_counts.assign((size_t)n, 0);
    std::vector<ParticleOut> res((size_t)n);
    // particles are independent (one block per particle in the reference, phdfilter.cu:2119)
#pragma omp parallel for schedule(dynamic, 1)
    for (int p = 0; p < n; p++)
        update_particle(cfg, p, poses[p], maps_in + offsets_in[p], offsets_in[p + 1] - offsets_in[p], Zin, M,
                        cn_out ? cn_out + (size_t)p * (cfg.maxCardinality + 1) : nullptr, res[(size_t)p]);
    long total = 0;
    offsets_out[0] = 0;
    for (int p = 0; p < n; p++) {
        const ParticleOut& po = res[(size_t)p];
        if (total + (long)po.maps.size() > out_cap) return -1;
        for (const G2& g : po.maps) maps_out[total++] = g;
        offsets_out[p + 1] = (int)total;
        delta[p] = po.delta;
        if (margin) margin[p] = po.margin;
        g_near_counts[(size_t)p] = po.near;
    }
    return total;
}

long orc_update(const phd_slam_config* cfgp, int n, const phd_pose* poses, const phd_gaussian2d* maps_in,
                const int* offsets_in, const phd_measurement* Zin, int n_measure, phd_gaussian2d* maps_out,
                long out_cap, int* offsets_out, float* delta, float* margin) {
    return orc_update_cn(cfgp, n, poses, maps_in, offsets_in, Zin, n_measure, maps_out, out_cap, offsets_out, delta,
                         margin, nullptr);
}

/* CPHD births through the prediction (addBirths / birthsKernel,
 * phdfilter.cu.bak:738-870): append to every particle's map one component per
 * measurement (static-labelled ones when labels are on), the inverse
 * measurement from the particle's pose, weight birthWeight (linear).  CSR in ->
 * CSR out (caller-allocated, out_cap components).  Returns the total or -1. */
long orc_add_births(const phd_slam_config* cfgp, int n, const phd_pose* poses, const phd_gaussian2d* maps_in,
                    const int* offsets_in, const phd_measurement* Z, int n_measure, phd_gaussian2d* maps_out,
                    long out_cap, int* offsets_out) {
    const phd_slam_config& cfg = *cfgp;
    const int M = std::min(n_measure, 256);
    long t = 0;
    offsets_out[0] = 0;
    for (int p = 0; p < n; p++) {
        for (int k = offsets_in[p]; k < offsets_in[p + 1]; k++) {
            if (t >= out_cap) return -1;
            maps_out[t++] = maps_in[k];
        }
        for (int m = 0; m < M; m++) {
            if (!(Z[m].label == PHD_MEAS_STATIC || !cfg.labeledMeasurements)) continue;
            if (t >= out_cap) return -1;
            G2 b = compute_birth(cfg, poses[p], Z[m]);
            b.weight = cfg.birthWeight;
            maps_out[t++] = b;
        }
        offsets_out[p + 1] = (int)t;
    }
    return t;
}

}  // extern "C"

namespace {
/* ---- §8(f) rank 4: the mixed static + dynamic feature model (feature_model = 2) ----
 *
 * phdPredict -> predictMapMixed (phdfilter.cu:966-1035, kernel :910-963) and
 * phdUpdateSynth's MIXED_MODEL branch (:3412-3462 -> phdUpdateKernelMixed
 * :2323-2635, then mergeAndCopyMaps :3703-3726).  The per-component
 * arithmetic is the oracle's own restatement (mixed_ref.h, written from the
 * reference independently of the product's include/phd_mixed.h); this is the
 * orchestration, restated with these documented deviations:
 *   D12 the predicted cardinality sums this particle's predicted weights (the
 *       reference indexes features_predict_static[feature_idx] without the
 *       particle's offset, :2411 / :2437, i.e. particle 0's features);
 *   D13 threads past the last feature write nothing (the reference's
 *       `~is_static` (:2515) sends them to ptr_dynamic[-1], a racy write);
 *   D3 the normaliser and cardinality sums accumulate in double (order free);
 *   D14 exponentials / logarithms through phd_det_expf / phd_det_logf.
 * Everything else follows the reference: measurement labels select the map a
 * measurement updates, both maps' detection terms share one normaliser per
 * measurement (+ clutter + one birth weight, two when unlabeled), nearly
 * in-range static components join the static merge and out-of-range ones are
 * appended; dynamic components outside the range are dropped (:3715-3719).
 */
template <int D>
struct CompD {
    float w;
    float m[D];
    float c[D * D];
};

template <int D>
void merge_generic(const phd_slam_config& cfg, const std::vector<CompD<D>>& cand, std::vector<CompD<D>>& out,
                   Margin& mg) {
    const size_t n = cand.size();
    std::vector<char> merged(n, 0);
    std::vector<float> dist(n);
    const float T = cfg.minSeparation;
    while (true) {
        long best = -1;
        for (size_t i = 0; i < n; i++) {
            if (merged[i]) continue;
            if (best < 0 || cand[best].w < cand[i].w) best = (long)i;  // D1: first max
        }
        if (best < 0) break;
        const CompD<D> mx = cand[best];
        double Wd = 0, md[D] = {};
        for (size_t i = 0; i < n; i++) {
            if (merged[i]) continue;
            const float d = D == 2 ? orx::mahal2(mx.m, mx.c, cand[i].m, cand[i].c)
                                   : orx::mahal4(mx.m, mx.c, cand[i].m, cand[i].c);
            dist[i] = d;
            if ((long)i != best) mg.rel(d, T);
            if (d < T) {
                Wd += (double)cand[i].w;
                for (int k = 0; k < D; k++) md[k] += (double)(cand[i].w * cand[i].m[k]);
            }
        }
        const float W = (float)Wd;
        if (W == 0) break;
        CompD<D> g;
        g.w = W;
        for (int k = 0; k < D; k++) g.m[k] = (float)md[k] / W;
        double cd[D * D] = {};
        for (size_t i = 0; i < n; i++) {
            if (merged[i] || !(dist[i] < T)) continue;
            float dm[D];
            for (int k = 0; k < D; k++) dm[k] = g.m[k] - cand[i].m[k];
            const float w = cand[i].w;
            for (int j = 0; j < D; j++)
                for (int k = 0; k < D; k++) cd[j * D + k] += (double)(w * (cand[i].c[j * D + k] + dm[j] * dm[k]));
            merged[i] = 1;
        }
        for (int k = 0; k < D * D; k++) g.c[k] = (float)cd[k] / W;
        orx::symmetrize(g.c, D);
        out.push_back(g);
    }
}

}  // namespace

extern "C" {

/* Scalar / per-component helpers of the oracle's mixed-model restatement
 * (mixed_ref.h), exported for the closed-form tests (tests/test_oracle_mixed.py). */
float orc_det_logf(float x) { return phd_det_logf(x); }
void orc_mx_inv4(const float* A, float* R) { orx::inverse4(A, R); }
float orc_mx_mahal4(const phd_gaussian4d* a, const phd_gaussian4d* b) {
    return orx::mahal4(a->mean, a->cov, b->mean, b->cov);
}
/* out: r, bearing, pd, det, S[4], K[8], cu[16] (32 floats) */
void orc_mx_ekf(const phd_slam_config* cfg, const phd_pose* pose, const phd_gaussian4d* g, int dims, float* out) {
    orx::PreUpdate e;
    if (dims == 2) {
        const float P[4] = {g->cov[0], g->cov[1], g->cov[4], g->cov[5]};
        orx::preupdate2(*cfg, *pose, g->mean, P, e);
    } else {
        orx::preupdate4(*cfg, *pose, g->mean, g->cov, e);
    }
    out[0] = e.r;
    out[1] = e.bearing;
    out[2] = e.pd;
    out[3] = e.det;
    for (int i = 0; i < 4; i++) out[4 + i] = e.S[i];
    for (int i = 0; i < 8; i++) out[8 + i] = e.K[i];
    for (int i = 0; i < 16; i++) out[16 + i] = e.cov[i];
}

/* predictMapMixed on a flat array of dynamic components (one call of phdPredict). */
void orc_predict_dynamic(const phd_slam_config* cfgp, long count, const phd_gaussian4d* in, phd_gaussian4d* out) {
    for (long i = 0; i < count; i++) {
        phd_gaussian4d g;
        orx::predict_cv4(*cfgp, in[i].mean, in[i].cov, in[i].weight, g.mean, g.cov, &g.weight);
        out[i] = g;
    }
}

/* Mixed update of n particles: static maps (CSR of Gaussian2D) and dynamic maps
 * (CSR of Gaussian4D) in, both posteriors out (caller-allocated, capacities
 * s_cap / d_cap components), delta = Δ log w.  Returns 0, or -1 on overflow /
 * unsupported configuration. */
long orc_update_mixed(const phd_slam_config* cfgp, int n, const phd_pose* poses, const phd_gaussian2d* s_in,
                      const int* s_off_in, const phd_gaussian4d* d_in, const int* d_off_in, const phd_measurement* Z,
                      int n_measure, phd_gaussian2d* s_out, long s_cap, int* s_off_out, phd_gaussian4d* d_out,
                      long d_cap, int* d_off_out, float* delta, float* margin) {
    const phd_slam_config& cfg = *cfgp;
    if (cfg.featureModel != PHD_FEATURE_MIXED || cfg.filterType != PHD_FILTER_PHD || cfg.particleWeighting != 0 ||
        cfg.distanceMetric != 0)
        return -1;
    const phd_slam_config& c = cfg;
    const bool labeled = cfg.labeledMeasurements != 0;
    const int M = std::min(n_measure, 256);  // phdfilter.cu:3390-3394
    const float minw = cfg.minFeatureWeight;
    long ts = 0, td = 0;
    s_off_out[0] = 0;
    d_off_out[0] = 0;
    g_near_counts.assign((size_t)n, 0);
    for (int p = 0; p < n; p++) {
        Margin mg;
        const phd_pose& pose = poses[p];
        std::vector<CompD<2>> sin, sout1, sout2, scand, smerged;
        std::vector<CompD<4>> din, dcand, dmerged;
        for (int k = s_off_in[p]; k < s_off_in[p + 1]; k++) {
            CompD<2> g;
            g.w = s_in[k].weight;
            for (int i = 0; i < 2; i++) g.m[i] = s_in[k].mean[i];
            for (int i = 0; i < 4; i++) g.c[i] = s_in[k].cov[i];
            const int cls = orx::range_class(c, pose, g.m[0], g.m[1]);
            const float dx = g.m[0] - pose.px, dy = g.m[1] - pose.py;
            mg.rel(std::sqrt(dx * dx + dy * dy), cfg.maxRange, true);
            (cls == 1 ? sin : cls == 2 ? sout2 : sout1).push_back(g);
        }
        for (int k = d_off_in[p]; k < d_off_in[p + 1]; k++) {
            CompD<4> g;
            g.w = d_in[k].weight;
            for (int i = 0; i < 4; i++) g.m[i] = d_in[k].mean[i];
            for (int i = 0; i < 16; i++) g.c[i] = d_in[k].cov[i];
            const float dx = g.m[0] - pose.px, dy = g.m[1] - pose.py;
            mg.rel(std::sqrt(dx * dx + dy * dy), cfg.maxRange, true);
            if (orx::range_class(c, pose, g.m[0], g.m[1]) == 1) din.push_back(g);
        }
        const int Gs = (int)sin.size(), Gd = (int)din.size();
        std::vector<orx::PreUpdate> es(Gs), ed(Gd);
        double card_d = 0;
        for (int j = 0; j < Gs; j++) {
            orx::preupdate2(c, pose, sin[j].m, sin[j].c, es[j]);
            card_d += (double)(es[j].pd * sin[j].w);
        }
        for (int j = 0; j < Gd; j++) {
            orx::preupdate4(c, pose, din[j].m, din[j].c, ed[j]);
            card_d += (double)(ed[j].pd * din[j].w);
        }
        const float card = (float)card_d;
        std::vector<float> lqs((size_t)Gs * M), lqd((size_t)Gd * M), leta(M);
        float pw = 0;
        for (int m = 0; m < M; m++) {
            const bool ok_s = Z[m].label == PHD_MEAS_STATIC || !labeled;
            const bool ok_d = Z[m].label == PHD_MEAS_DYNAMIC || !labeled;
            double sd = 0;
            float i0, i1;
            for (int j = 0; j < Gs; j++) {
                lqs[(size_t)j * M + m] = orx::log_q(es[j], sin[j].w, Z[m].range, Z[m].bearing, ok_s, i0, i1);
                sd += (double)phd_det_expf(lqs[(size_t)j * M + m]);
            }
            for (int j = 0; j < Gd; j++) {
                lqd[(size_t)j * M + m] = orx::log_q(ed[j], din[j].w, Z[m].range, Z[m].bearing, ok_d, i0, i1);
                sd += (double)phd_det_expf(lqd[(size_t)j * M + m]);
            }
            sd += (double)cfg.clutterDensity;
            sd += (double)cfg.birthWeight;
            if (!labeled) sd += (double)cfg.birthWeight;  // two birth terms (:2501-2503)
            leta[m] = orx::safe_log((float)sd);
            pw += leta[m];
        }
        // static candidates in update-array order [non-detect | detect (m-major) | births], then nearly in range
        for (int j = 0; j < Gs; j++) {
            CompD<2> g = sin[j];
            g.w = sin[j].w * (1 - es[j].pd);
            mg.rel(g.w, minw);
            if (!(g.w < minw)) scand.push_back(g);
        }
        for (int m = 0; m < M; m++)
            for (int j = 0; j < Gs; j++) {
                const orx::PreUpdate& e = es[j];
                float i0, i1;
                orx::log_q(e, sin[j].w, Z[m].range, Z[m].bearing, true, i0, i1);
                CompD<2> g;
                g.m[0] = sin[j].m[0] + e.K[0] * i0 + e.K[2] * i1;
                g.m[1] = sin[j].m[1] + e.K[1] * i0 + e.K[3] * i1;
                for (int k = 0; k < 4; k++) g.c[k] = e.cov[k];
                g.w = phd_det_expf(lqs[(size_t)j * M + m] - leta[m]);
                if (g.w > 1e-12f) mg.rel(g.w, minw);
                if (!(g.w < minw)) scand.push_back(g);
            }
        for (int m = 0; m < M; m++) {
            CompD<2> b;
            const float lw = orx::birth(c, pose, Z[m].range, Z[m].bearing,
                                        Z[m].label == PHD_MEAS_STATIC || !labeled, 2, b.m, b.c);
            b.w = phd_det_expf(lw - leta[m]);
            if (b.w > 1e-12f) mg.rel(b.w, minw);
            if (!(b.w < minw)) scand.push_back(b);
        }
        for (const CompD<2>& g : sout2) scand.push_back(g);
        merge_generic<2>(cfg, scand, smerged, mg);
        // dynamic candidates [non-detect | detect (m-major) | births]; nothing out of range survives
        for (int j = 0; j < Gd; j++) {
            CompD<4> g = din[j];
            g.w = din[j].w * (1 - ed[j].pd);
            mg.rel(g.w, minw);
            if (!(g.w < minw)) dcand.push_back(g);
        }
        for (int m = 0; m < M; m++)
            for (int j = 0; j < Gd; j++) {
                const orx::PreUpdate& e = ed[j];
                float i0, i1;
                orx::log_q(e, din[j].w, Z[m].range, Z[m].bearing, true, i0, i1);
                CompD<4> g;
                for (int k = 0; k < 4; k++) g.m[k] = din[j].m[k] + e.K[k] * i0 + e.K[4 + k] * i1;
                for (int k = 0; k < 16; k++) g.c[k] = e.cov[k];
                g.w = phd_det_expf(lqd[(size_t)j * M + m] - leta[m]);
                if (g.w > 1e-12f) mg.rel(g.w, minw);
                if (!(g.w < minw)) dcand.push_back(g);
            }
        for (int m = 0; m < M; m++) {
            CompD<4> b;
            const float lw = orx::birth(c, pose, Z[m].range, Z[m].bearing,
                                        Z[m].label == PHD_MEAS_DYNAMIC || !labeled, 4, b.m, b.c);
            b.w = phd_det_expf(lw - leta[m]);
            if (b.w > 1e-12f) mg.rel(b.w, minw);
            if (!(b.w < minw)) dcand.push_back(b);
        }
        merge_generic<4>(cfg, dcand, dmerged, mg);
        if (ts + (long)smerged.size() + (long)sout1.size() > s_cap || td + (long)dmerged.size() > d_cap) return -1;
        auto put2 = [&](const CompD<2>& g) {
            phd_gaussian2d& o = s_out[ts++];
            o.weight = g.w;
            for (int k = 0; k < 2; k++) o.mean[k] = g.m[k];
            for (int k = 0; k < 4; k++) o.cov[k] = g.c[k];
        };
        for (const CompD<2>& g : smerged) put2(g);
        for (const CompD<2>& g : sout1) put2(g);
        for (const CompD<4>& g : dmerged) {
            phd_gaussian4d& o = d_out[td++];
            o.weight = g.w;
            for (int k = 0; k < 4; k++) o.mean[k] = g.m[k];
            for (int k = 0; k < 16; k++) o.cov[k] = g.c[k];
        }
        s_off_out[p + 1] = (int)ts;
        d_off_out[p + 1] = (int)td;
        delta[p] = pw - card;
        if (margin) margin[p] = mg.m;
        g_near_counts[p] = std::min(mg.cls, 0xffff) | (std::min(mg.pm, 0x7fff) << 16);
    }
    return 0;
}

/* EAP expected map of the dynamic maps, exp_map_dynamic (main.cpp:369-371,
 * computeExpectedMap main.cpp:290-316 over maps_dynamic, reduceGaussianMixture
 * gm_reduce.cpp:59-132 with the 4-D LLT distance): components weighted by
 * exp(log w_n) (D8: det_expf), stable priority order (weight descending), the
 * greedy, sums in the reference's float order (gm_reduce.cpp:103-123: the seed
 * first, then the absorbed members in priority order). */
long orc_expected_map_dynamic(const phd_slam_config* cfg, int n, const float* w, const phd_gaussian4d* maps,
                              const int* offsets, phd_gaussian4d* out, long out_cap) {
    std::vector<phd_gaussian4d> all;
    for (int p = 0; p < n; p++) {
        const float ew = phd_det_expf(w[p]);
        for (int k = offsets[p]; k < offsets[p + 1]; k++) {
            phd_gaussian4d g = maps[k];
            g.weight *= ew;
            all.push_back(g);
        }
    }
    std::vector<size_t> order(all.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return all[a].weight > all[b].weight; });
    std::vector<char> used(all.size(), 0);
    const float T = cfg->minSeparation;
    long nout = 0;
    std::vector<size_t> grp;
    for (size_t oi = 0; oi < order.size(); oi++) {
        const size_t a = order[oi];
        if (used[a]) continue;
        used[a] = 1;
        const phd_gaussian4d& mx = all[a];
        grp.clear();
        for (size_t oj = oi + 1; oj < order.size(); oj++) {
            const size_t b = order[oj];
            if (used[b]) continue;
            if (orx::llt_dist4(mx.mean, mx.cov, all[b].mean, all[b].cov) < T) {
                grp.push_back(b);
                used[b] = 1;
            }
        }
        // merge_element.mean = w_max mean_max; += w_i mean_i; weight += w_i; mean /= weight
        float W = mx.weight, m[4], cv[16];
        for (int i = 0; i < 4; i++) m[i] = mx.mean[i] * mx.weight;
        for (size_t b : grp) {
            for (int i = 0; i < 4; i++) m[i] += all[b].weight * all[b].mean[i];
            W += all[b].weight;
        }
        for (int i = 0; i < 4; i++) m[i] /= W;
        // cov = w_max (cov_max + d d'); += w_i (cov_i + d d'); cov /= weight
        auto outer = [&](const phd_gaussian4d& g, bool first) {
            float d[4];
            for (int i = 0; i < 4; i++) d[i] = m[i] - g.mean[i];
            for (int j = 0; j < 4; j++)
                for (int i = 0; i < 4; i++) {
                    const float t = g.weight * (g.cov[i + 4 * j] + d[i] * d[j]);
                    cv[i + 4 * j] = first ? t : cv[i + 4 * j] + t;
                }
        };
        outer(mx, true);
        for (size_t b : grp) outer(all[b], false);
        if (nout >= out_cap) return -1;
        phd_gaussian4d& o = out[nout++];
        o.weight = W;
        for (int i = 0; i < 4; i++) o.mean[i] = m[i];
        for (int k = 0; k < 16; k++) o.cov[k] = cv[k] / W;
    }
    return nout;
}

/* Near-threshold decision counts of the last orc_update / orc_update_cn call,
 * per particle: out_cls = range classifications, out_pm = prune / merge
 * decisions within Margin::NEAR (1e-4 relative) of their threshold. */
int orc_near_counts(int n, int* out_cls, int* out_pm) {
    if (n > (int)g_near_counts.size()) return -1;
    for (int p = 0; p < n; p++) {
        out_cls[p] = g_near_counts[p] & 0xffff;
        out_pm[p] = g_near_counts[p] >> 16;
    }
    return 0;
}

/* A9: logSumExp normalisation on the host (device_math.cuh:549-558, phdfilter.cu:3748-3755). */
float orc_normalize(int n, float* w) {
    float maxval = *std::max_element(w, w + n);
    double sum = 0;
    for (int i = 0; i < n; i++) sum += (double)std::exp(w[i] - maxval);
    float lse = safeLog((float)sum) + maxval;
    for (int i = 0; i < n; i++) w[i] -= lse;
    return lse;
}

/* A11: nEff (main.cpp:1281-1284). */
float orc_neff(int n, const float* w) {
    double s = 0;
    for (int i = 0; i < n; i++) s += (double)std::exp(2 * w[i]);
    return (float)(1.0 / (double)(float)s / n);
}

/*
 * A11: faithful stratified resample (main.cpp:453-501).  u has n+1 uniforms:
 * u[0] is the reference's discarded leading draw, stratum j uses u[j+1].
 */
void orc_resample_faithful(int n, const float* w, const double* u, int* idx) {
    double interval = 1.0 / n;
    double c = std::exp(w[0]);
    int i = 0;
    for (int j = 0; j < n; j++) {
        double r = j * interval + u[j + 1] * interval;
        while (r > c) {
            i++;
            if (i >= n) {
                double mw = -1;
                int mi = -1;
                for (int k = 0; k < n; k++)
                    if (std::exp(w[k]) > mw) {
                        mw = std::exp(w[k]);
                        mi = k;
                    }
                i = mi;
                c = 2;
                break;
            }
            c += std::exp(w[i]);
        }
        idx[j] = i;
    }
}

/* D5: the build's resample (what the GPU computes): fixed-point CDF of det_expf terms. u[j] per stratum. */
void orc_resample_fixed_to(int n, const float* w, int n_out, const double* u, int* idx);
void orc_resample_fixed(int n, const float* w, const double* u, int* idx) { orc_resample_fixed_to(n, w, n, u, idx); }

/* n_out strata over n weights: resampleParticles(particles, n_particles) after
 * n_predict_particles > 1 grew the live set (main.cpp:1286-1289, 453-501). */
void orc_resample_fixed_to(int n, const float* w, int n_out, const double* u, int* idx) {
    std::vector<uint64_t> cdf(n);
    uint64_t acc = 0;
    int amax = 0;
    float tmax = -1;
    for (int i = 0; i < n; i++) {
        float t = phd_det_expf(w[i]);
        acc += phd_fix_term(t);
        cdf[i] = acc;
        if (t > tmax) {
            tmax = t;
            amax = i;
        }
    }
    for (int j = 0; j < n_out; j++) {
        uint64_t r = phd_fix_stratum(j, u[j], n_out);
        // smallest i with cdf[i] >= r
        int lo = 0, hi = n;
        while (lo < hi) {
            int mid = (lo + hi) / 2;
            if (cdf[mid] >= r)
                hi = mid;
            else
                lo = mid + 1;
        }
        idx[j] = lo < n ? lo : amax;
    }
}

/* A10: expected pose (main.cpp:331-340) and MAP particle index (main.cpp:344-361). */
int orc_expected_pose(int n, const float* w, const phd_pose* s, phd_pose* out) {
    double e[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        float ew = std::exp(w[i]);
        const float* ps = &s[i].px;
        for (int k = 0; k < 6; k++) e[k] += (double)(ew * ps[k]);
    }
    out->px = (float)e[0];
    out->py = (float)e[1];
    out->ptheta = (float)e[2];
    out->vx = (float)e[3];
    out->vy = (float)e[4];
    out->vtheta = (float)e[5];
    float mw = -FLT_MAX;
    int mi = -1;
    for (int i = 0; i < n; i++)
        if (w[i] > mw) {
            mi = i;
            mw = w[i];
        }
    return mi;
}

/*
 * A10: EAP expected map — computeExpectedMap (main.cpp:290-316) +
 * reduceGaussianMixture (gm_reduce.cpp:59-132).  Eigen's LLT Mahalanobis is
 * restated for 2x2 with forward substitution (Eigen version unpinned: parity
 * unpinned at this third-party boundary).  The descending-weight sort is made
 * stable (the reference's std::sort is unstable).  The particle-weight factor
 * exp(w_n) is phd_det_expf (D8), the exp the GPU evaluates too, so both sides
 * see bit-identical component weights and hence the same priority order.
 */
long orc_expected_map(const phd_slam_config* cfg, int n, const float* w, const phd_gaussian2d* maps,
                      const int* offsets, phd_gaussian2d* out, long out_cap) {
    std::vector<G2> all;
    for (int p = 0; p < n; p++) {
        float ew = phd_det_expf(w[p]);  // exp(weights[n]) (main.cpp:302); D8: the shared deterministic exp
        for (int k = offsets[p]; k < offsets[p + 1]; k++) {
            G2 g = maps[k];
            g.weight *= ew;
            all.push_back(g);
        }
    }
    std::vector<size_t> order(all.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return all[a].weight > all[b].weight; });
    std::vector<char> used(all.size(), 0);
    long nout = 0;
    const float T = cfg->minSeparation;
    for (size_t oi = 0; oi < order.size(); oi++) {
        size_t a = order[oi];
        if (used[a]) continue;
        used[a] = 1;
        const G2& mx = all[a];
        std::vector<size_t> grp;
        for (size_t oj = oi + 1; oj < order.size(); oj++) {
            size_t b = order[oj];
            if (used[b]) continue;
            const G2& o = all[b];
            float s00 = 0.5f * (mx.cov[0] + o.cov[0]);
            float s10 = 0.5f * (mx.cov[1] + o.cov[1]);
            float s11 = 0.5f * (mx.cov[3] + o.cov[3]);
            float l00 = std::sqrt(s00);
            float l10 = s10 / l00;
            float l11 = std::sqrt(s11 - l10 * l10);
            float d0 = mx.mean[0] - o.mean[0], d1 = mx.mean[1] - o.mean[1];
            float x0 = d0 / l00;
            float x1 = (d1 - l10 * x0) / l11;
            float d = x0 * x0 + x1 * x1;
            if (d < T) {
                grp.push_back(b);
                used[b] = 1;
            }
        }
        float W = mx.weight;
        float m0 = mx.mean[0] * mx.weight, m1 = mx.mean[1] * mx.weight;
        for (size_t b : grp) {
            m0 += all[b].weight * all[b].mean[0];
            m1 += all[b].weight * all[b].mean[1];
            W += all[b].weight;
        }
        m0 /= W;
        m1 /= W;
        float e0 = m0 - mx.mean[0], e1 = m1 - mx.mean[1];
        float c[4];
        c[0] = mx.weight * (mx.cov[0] + e0 * e0);
        c[1] = mx.weight * (mx.cov[1] + e1 * e0);
        c[2] = mx.weight * (mx.cov[2] + e0 * e1);
        c[3] = mx.weight * (mx.cov[3] + e1 * e1);
        for (size_t b : grp) {
            float f0 = m0 - all[b].mean[0], f1 = m1 - all[b].mean[1];
            c[0] += all[b].weight * (all[b].cov[0] + f0 * f0);
            c[1] += all[b].weight * (all[b].cov[1] + f1 * f0);
            c[2] += all[b].weight * (all[b].cov[2] + f0 * f1);
            c[3] += all[b].weight * (all[b].cov[3] + f1 * f1);
        }
        if (nout >= out_cap) return -1;
        G2 g;
        g.weight = W;
        g.mean[0] = m0;
        g.mean[1] = m1;
        for (int k = 0; k < 4; k++) g.cov[k] = c[k] / W;
        out[nout++] = g;
    }
    return nout;
}

/* The same greedy (orc_expected_map, gm_reduce.cpp:59-132) with the distance
 * tests restricted to the touching lattice cells of each seed — exact for the
 * FLOAT distance, whatever the conditioning: the LLT's float d = x0^2 + x1^2
 * with x0 = d0 / l00 and d1 = l10 x0 + l11 x1 (l10^2 + l11^2 = s11 up to
 * rounding relative to s11, not to the determinant) gives d0^2 <= d s00 and
 * d1^2 <= d s11, so a pair with d < T has |Δμ|^2 < T tr(Σ) = T (tr P_a + tr P_b) / 2
 * <= T max tr: it lies in touching cells of side sqrt(1.1 T max tr) (10 % for
 * the rounding).  (An eigenvalue bound |Δμ|^2 < T λmax(Σ) holds for the exact
 * distance only: a nearly singular Σ's float l11 can come out far too large.)
 * Seeds, absorbed sets, their priority order and every float expression are
 * those of orc_expected_map, so the outputs are identical; it only makes the
 * oracle feasible at config 3's 2.1 M components (test infrastructure for the
 * GPU EAP map at scale).  Non-finite input falls back to the plain loop. */
long orc_expected_map_cells(const phd_slam_config* cfg, int n, const float* w, const phd_gaussian2d* maps,
                            const int* offsets, phd_gaussian2d* out, long out_cap) {
    std::vector<G2> all;
    for (int p = 0; p < n; p++) {
        float ew = phd_det_expf(w[p]);
        for (int k = offsets[p]; k < offsets[p + 1]; k++) {
            G2 g = maps[k];
            g.weight *= ew;
            all.push_back(g);
        }
    }
    const float T = cfg->minSeparation;
    double trmax = 0;
    bool finite = T > 0 && T < INFINITY;
    for (const G2& g : all) {
        const double tr = (double)g.cov[0] + (double)g.cov[3];
        if (!(std::fabs(g.mean[0]) < INFINITY && std::fabs(g.mean[1]) < INFINITY && std::fabs(tr) < INFINITY))
            finite = false;
        else
            trmax = std::max(trmax, tr);
    }
    if (!finite || !(trmax > 0)) return orc_expected_map(cfg, n, w, maps, offsets, out, out_cap);
    const double R = std::sqrt(1.1 * (double)T * trmax) * 1.0001;
    const size_t K = all.size();
    std::vector<size_t> order(K);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return all[a].weight > all[b].weight; });
    auto cell_of = [&](const G2& g, long long* cx, long long* cy) {
        *cx = (long long)std::floor((double)g.mean[0] / R);
        *cy = (long long)std::floor((double)g.mean[1] / R);
    };
    auto ckey = [](long long cx, long long cy) {
        return ((unsigned long long)(cx + (1LL << 31)) << 32) | (unsigned long long)((cy + (1LL << 31)) & 0xffffffffLL);
    };
    // cell -> priority positions (ascending: inserted in priority order)
    std::unordered_map<unsigned long long, std::vector<size_t>> cells;
    cells.reserve(K / 4 + 16);
    for (size_t oi = 0; oi < K; oi++) {
        long long cx, cy;
        cell_of(all[order[oi]], &cx, &cy);
        cells[ckey(cx, cy)].push_back(oi);
    }
    std::vector<char> used(K, 0);  // by priority position
    long nout = 0;
    std::vector<size_t> grp;
    for (size_t oi = 0; oi < K; oi++) {
        if (used[oi]) continue;
        used[oi] = 1;
        const G2& mx = all[order[oi]];
        long long cx, cy;
        cell_of(mx, &cx, &cy);
        grp.clear();
        for (int dx = -1; dx <= 1; dx++)
            for (int dy = -1; dy <= 1; dy++) {
                auto it = cells.find(ckey(cx + dx, cy + dy));
                if (it == cells.end()) continue;
                std::vector<size_t>& lst = it->second;
                size_t keep = 0;  // drop merged entries as the list is walked
                for (size_t e = 0; e < lst.size(); e++) {
                    const size_t oj = lst[e];
                    if (used[oj]) continue;
                    lst[keep++] = oj;
                    if (oj <= oi) continue;
                    const G2& o = all[order[oj]];
                    float s00 = 0.5f * (mx.cov[0] + o.cov[0]);
                    float s10 = 0.5f * (mx.cov[1] + o.cov[1]);
                    float s11 = 0.5f * (mx.cov[3] + o.cov[3]);
                    float l00 = std::sqrt(s00);
                    float l10 = s10 / l00;
                    float l11 = std::sqrt(s11 - l10 * l10);
                    float d0 = mx.mean[0] - o.mean[0], d1 = mx.mean[1] - o.mean[1];
                    float x0 = d0 / l00;
                    float x1 = (d1 - l10 * x0) / l11;
                    float d = x0 * x0 + x1 * x1;
                    if (d < T) grp.push_back(oj);
                }
                lst.resize(keep);
            }
        std::sort(grp.begin(), grp.end());  // priority order, as the plain loop visits them
        for (size_t oj : grp) used[oj] = 1;
        float W = mx.weight;
        float m0 = mx.mean[0] * mx.weight, m1 = mx.mean[1] * mx.weight;
        for (size_t oj : grp) {
            const G2& b = all[order[oj]];
            m0 += b.weight * b.mean[0];
            m1 += b.weight * b.mean[1];
            W += b.weight;
        }
        m0 /= W;
        m1 /= W;
        float e0 = m0 - mx.mean[0], e1 = m1 - mx.mean[1];
        float c[4];
        c[0] = mx.weight * (mx.cov[0] + e0 * e0);
        c[1] = mx.weight * (mx.cov[1] + e1 * e0);
        c[2] = mx.weight * (mx.cov[2] + e0 * e1);
        c[3] = mx.weight * (mx.cov[3] + e1 * e1);
        for (size_t oj : grp) {
            const G2& b = all[order[oj]];
            float f0 = m0 - b.mean[0], f1 = m1 - b.mean[1];
            c[0] += b.weight * (b.cov[0] + f0 * f0);
            c[1] += b.weight * (b.cov[1] + f1 * f0);
            c[2] += b.weight * (b.cov[2] + f0 * f1);
            c[3] += b.weight * (b.cov[3] + f1 * f1);
        }
        if (nout >= out_cap) return -1;
        G2 g;
        g.weight = W;
        g.mean[0] = m0;
        g.mean[1] = m1;
        for (int k = 0; k < 4; k++) g.cov[k] = c[k] / W;
        out[nout++] = g;
    }
    return nout;
}

/* Map copy of a resample (SynthSLAM::copy_particles, slamtypes.h:313-333). */
long orc_copy_particles(int n, const int* idx, const phd_pose* poses, const phd_gaussian2d* maps,
                        const int* offsets, phd_pose* poses_out, float* w_out, phd_gaussian2d* maps_out,
                        int* offsets_out) {
    long total = 0;
    offsets_out[0] = 0;
    const float neg_log_n = (float)(-std::log((double)n));
    for (int j = 0; j < n; j++) {
        int i = idx[j];
        poses_out[j] = poses[i];
        w_out[j] = neg_log_n;
        for (int k = offsets[i]; k < offsets[i + 1]; k++) maps_out[total++] = maps[k];
        offsets_out[j + 1] = (int)total;
    }
    return total;
}

}  // extern "C"
