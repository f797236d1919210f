/*
 * phd_cphd_terms.h — the GM-CPHD weight terms of one particle evaluated by one
 * wavefront (A12: the reference's commented kernels phdfilter.cu:1360-1820 /
 * phdfilter.cu.bak:990-1504, Poisson predicted cardinality .bak:2473-2497; the
 * oracle states them directly, oracle/scphd_cpu.cpp cphd_terms).  The middle
 * launch of the three-launch CPHD update, k_cphd_terms (instantiated in
 * phd_terms.hip): one wave per particle between part A and part C.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "phd_devutil.h"
#include "phd_kernels.h"

#ifdef PHD_STAMPS
#define WSTAMP(k)                                                                                         \
    do {                                                                                                  \
        if (lane == 0 && a.stamps) a.stamps[(size_t)n * PHD_STAMP_SLOTS + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define WSTAMP(k) \
    do {          \
    } while (0)
#endif

namespace phd {

typedef unsigned long long u64;

/* The LDS of this wave is written and read by other lanes of the same wave.
 * A wave's LDS operations complete in issue order, so ordering them needs no
 * barrier: wait for the outstanding LDS operations (lgkmcnt only — never the
 * vector-memory counter, which would drain prefetches and slab stores) and keep
 * the compiler from moving memory accesses across. */
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double eta_value(const u64* ehi, const u64* elo, int m, double lo_unscale) {
    return (double)ehi[m] * 9.094947017729282e-13 + (double)elo[m] * lo_unscale;  // 2^-40
}

/* ------------------------------------------------------------- CPHD, one wave
 * The CPHD weight terms of cphd_block (phd_kernels.hip, same quantities and
 * expressions) evaluated by one wavefront; lane m owns measurement m and
 * hypothesis size j = m (slot 0: lane, slot 1: lane + 64). */
struct CphdOut {
    double ip0, ip1, bmax;
    int wide;
};

__device__ __forceinline__ void cphd_wave(const UpdateArgs& a, int n, int M, const u64* ehi, const u64* elo,
                                          double lo_unscale, double win, double qd, double W, double* sc,
                                          float* s_leta, float* s_thr, CphdOut& out) {
    const DevCfg& c = a.c;
    const int lane = threadIdx.x & 63;
    const int Q = a.Mcap + 4;
    double* lS = sc;            // log S(T0 + t)
    double* lB0 = sc + Q;       // log B0_j
    double* lB1 = sc + 2 * Q;   // log B1_j
    double* beta = sc + 3 * Q;  // beta'_j
    double* le = sc + 4 * Q;    // log e_k(Lambda)
    double* ip1d = sc + 5 * Q;  // raw <Psi1d_m, p> e^-bmax
    double* lampa = sc + 6 * Q; // lambda'_m
    const int Nmax = a.Nmax;
    win = uni_d(win);
    qd = uni_d(qd);
    W = uni_d(W);
    const double lw = uni_d(win > 0 ? log(win) : -INFINITY);
    const double lq = uni_d(qd > 0 ? log(qd) : -INFINITY);
    const double logW = uni_d(W > 0 ? log(W) : -INFINITY);
    const double lr = win > 0 ? lq - lw : (double)c.cphd_log1mpd;
    const double aexp = uni_d(logW + lr);
    const double dd = uni_d((win > 0 && W > 0) ? logW - lw : 0.0);
    // log Lambda_m, two slots
    auto lam_of = [&](int m) -> double {
        if (m >= M) return -INFINITY;
        const double S = eta_value(ehi, elo, m, lo_unscale);
        return S > 0 ? log(S) + c.cphd_lck : -INFINITY;
    };
    const double lam0 = lam_of(lane), lam1 = lam_of(lane + 64);  // (eta_value: lo_unscale passed in)
    const G1 double* lf = g1(a.lfact);
    double um = -INFINITY;
    for (int i = lane; i <= Nmax; i += 64) um = fmax(um, i == 0 ? 0.0 : (double)i * aexp - lf[i]);
    um = wave_max_dx(um);
    const double lmax = wave_max_dx(fmax(lam0, lam1));
    const double lsum = wave_sum_dx((lane < M ? lam0 : 0.0) + (lane + 64 < M ? lam1 : 0.0));
    const int T0 = max(0, Nmax - M - 1);
    double part = 0.0;
    for (int i = lane; i < T0; i += 64) part += exp((i == 0 ? 0.0 : (double)i * aexp - lf[i]) - um);
    part = wave_sum_dx(part);
    if (lane < M) lampa[lane] = lam0 == -INFINITY ? 0.0 : exp(lam0 - lmax);
    if (lane + 64 < M) lampa[lane + 64] = lam1 == -INFINITY ? 0.0 : exp(lam1 - lmax);
    {  // S(T0 + t) = part + prefix of the tail: t <= nt = min(Nmax, M + 1) <= 128, so
       // up to 129 terms — two wave slots and the single t = 128 of a third (M = 127)
        const int nt = Nmax - T0;
        auto term = [&](int t) -> double {
            if (t > nt) return 0.0;
            const int i = T0 + t;
            return exp((i == 0 ? 0.0 : (double)i * aexp - lf[i]) - um);
        };
        const double s0 = wave_incl_scan_d(term(lane));
        const double s1 = wave_incl_scan_d(term(lane + 64)) + readlane_d(s0, 63);
        if (lane <= nt) lS[lane] = log(part + s0) + um;
        if (lane + 64 <= nt) lS[lane + 64] = log(part + s1) + um;
        if (nt >= 128 && lane == 0) lS[128] = log(part + (readlane_d(s1, 63) + term(128))) + um;
    }
    wsync();
    // B_j per hypothesis size j, beta'_j
    double bv0 = -INFINITY, bv1 = -INFINITY;
    for (int sl = 0; sl < 2; sl++) {
        const int j = lane + 64 * sl;
        if (j > M) continue;
        lB0[j] = Nmax - j >= 0 ? (j == 0 ? 0.0 : (double)j * dd) - W + lS[Nmax - j - T0] : -INFINITY;
        const double b1 = Nmax - j - 1 >= 0 ? (double)(j + 1) * dd - W + lS[Nmax - j - 1 - T0] : -INFINITY;
        lB1[j] = b1;
        double bv = -INFINITY;
        if (j < M && b1 != -INFINITY) bv = (double)(M - 1 - j) * c.cphd_lrate - c.cphd_rate + b1 + kpow_d(j, lmax);
        if (sl == 0) bv0 = bv; else bv1 = bv;
    }
    const double bmax = wave_max_dx(fmax(bv0, bv1));
    if (lane < M) beta[lane] = (bv0 == -INFINITY || bmax == -INFINITY) ? 0.0 : exp(bv0 - bmax);
    if (lane + 64 < M) beta[lane + 64] = (bv1 == -INFINITY || bmax == -INFINITY) ? 0.0 : exp(bv1 - bmax);
    if (M == 0 && lane == 0) le[0] = 0.0;
    wsync();
    WSTAMP(30);
    /* <Psi1d_m, p> = log sum_a P_m[a] T_m[a] (prefix products P, suffix sums T;
     * positive recursions), by segments of L measurements: the T chain runs
     * down from M-1 and the P chain up from 0 side by side (independent). */
    if (M <= 64) {
        constexpr int L = 16;
        const double lp = lane < M ? lampa[lane] : 0.0;
        for (int m0 = 0; m0 < M; m0 += L) {
            const int m1 = min(m0 + L, M);
            double T = lane < M ? beta[lane] : 0.0;
            double P = lane == 0 ? 1.0 : 0.0;
            const int nT = M - m1, nP = m0;
            for (int s = 0; s < max(nT, nP); s++) {
                if (s < nT) {
                    const int m = M - 1 - s;
                    T = fma(readlane_d(lp, m), dpp_or_zero_d<0x130, 0xf>(T), T);
                }
                if (s < nP) P = fma(readlane_d(lp, s), dpp_or_zero_d<0x138, 0xf>(P), P);
            }
            double tr[L];
#pragma unroll
            for (int q = L - 1; q >= 0; q--) {
                const int m = m0 + q;
                tr[q] = T;
                if (m < m1 && m > m0) T = fma(readlane_d(lp, m), dpp_or_zero_d<0x130, 0xf>(T), T);
            }
#pragma unroll
            for (int q = 0; q < L; q++) {
                const int m = m0 + q;
                tr[q] *= P;
                if (m < m1) P = fma(readlane_d(lp, m), dpp_or_zero_d<0x138, 0xf>(P), P);
            }
#pragma unroll
            for (int q = 0; q < L; q++) tr[q] = wave_sum_dx(tr[q]);
            if (lane < L && m0 + lane < m1) {
                double v = tr[0];
#pragma unroll
                for (int q = 1; q < L; q++) v = lane == q ? tr[q] : v;
                ip1d[m0 + lane] = v;
            }
            if (m1 == M) {  // P_M below degree M; e_M = prod Lambda
                if (lane < M) le[lane] = P > 0 ? log(P) + kpow_d(lane, lmax) : -INFINITY;
                if (lane == 0) le[M] = lsum;
            }
        }
    } else {
        constexpr int L = PHD_CPHD_SEG;
        const double lp0 = lane < M ? lampa[lane] : 0.0, lp1 = lane + 64 < M ? lampa[lane + 64] : 0.0;
#define PHD_LAMP(m) readlane_d((m) < 64 ? lp0 : lp1, (m) & 63)
        for (int m0 = 0; m0 < M; m0 += L) {
            const int m1 = min(m0 + L, M);
            double T0 = lane < M ? beta[lane] : 0.0, T1 = lane + 64 < M ? beta[lane + 64] : 0.0;
            for (int m = M - 1; m >= m1; m--) suffix_step(T0, T1, PHD_LAMP(m));
            double tr0[L], tr1[L];
#pragma unroll
            for (int q = L - 1; q >= 0; q--) {
                const int m = m0 + q;
                tr0[q] = T0;
                tr1[q] = T1;
                if (m < m1 && m > m0) suffix_step(T0, T1, PHD_LAMP(m));
            }
            double P0 = lane == 0 ? 1.0 : 0.0, P1 = 0.0;
            for (int m = 0; m < m0; m++) poly_mul_lin(P0, P1, PHD_LAMP(m));
            double fs[L];
#pragma unroll
            for (int q = 0; q < L; q++) {
                const int m = m0 + q;
                fs[q] = P0 * tr0[q] + P1 * tr1[q];
                if (m < m1) poly_mul_lin(P0, P1, PHD_LAMP(m));
            }
#pragma unroll
            for (int q = 0; q < L; q++) fs[q] = wave_sum_dx(fs[q]);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < L; q++)
                    if (m0 + q < m1) ip1d[m0 + q] = fs[q];
            }
            if (m1 == M) {
                const int k0 = lane, k1 = lane + 64;
                if (k0 <= M) le[k0] = P0 > 0 ? log(P0) + kpow_d(k0, lmax) : -INFINITY;
                if (k1 <= M) le[k1] = P1 > 0 ? log(P1) + kpow_d(k1, lmax) : -INFINITY;
            }
        }
#undef PHD_LAMP
    }
    wsync();
    WSTAMP(31);
    double b0 = -INFINITY, b1 = -INFINITY, p0 = -INFINITY, p1 = -INFINITY, q0 = -INFINITY, q1 = -INFINITY;
    const int k0 = lane, k1 = lane + 64;
    if (k0 <= M && le[k0] != -INFINITY) {
        b0 = (double)(M - k0) * c.cphd_lrate - c.cphd_rate + le[k0];
        p0 = b0 + lB0[k0];
        q0 = b0 + lB1[k0];
    }
    if (k1 <= M && le[k1] != -INFINITY) {
        b1 = (double)(M - k1) * c.cphd_lrate - c.cphd_rate + le[k1];
        p1 = b1 + lB0[k1];
        q1 = b1 + lB1[k1];
    }
    const double ip0 = uni_d(wave_lse2(p0, p1));
    const double ip1 = uni_d(wave_lse2(q0, q1));
    G1 double* co = a.cn_coef ? g1(uni_p(a.cn_coef + (size_t)n * a.cn_stride)) : nullptr;
    if (co) {
        if (k0 <= M) co[6 + k0] = b0;
        if (k1 <= M) co[6 + k1] = b1;
        if (lane == 0) {
            co[0] = ip0;
            co[1] = lq;
            co[2] = lw;
            co[3] = logW;
            co[4] = W;
            co[5] = (double)M;
        }
    }
    int wide = 0;
    for (int m = lane; m < M; m += 64) {
        const double sm = ip1d[m];
        const float le_m = (float)((ip0 - (sm > 0 ? log(sm) + bmax : -INFINITY)) - c.cphd_lck);
        s_leta[m] = le_m;
        s_thr[m] = (c.log_minfw + le_m - 0.5f) * 1.4426950408889634f;
        wide |= !(le_m >= c.cphd_leta_min);
    }
    out.ip0 = ip0;
    out.ip1 = ip1;
    out.bmax = bmax;
    out.wide = __ballot(wide != 0) != 0ull;
    wsync();
}

/* CDNA4 half exchanges of two doubles: lanes 32-63 of a <-> lanes 0-31 of b
 * (v_permlane32_swap), odd 16-lane rows of a <-> even rows of b
 * (v_permlane16_swap) — register moves, no LDS round trip. */
__device__ __forceinline__ void swap32_d(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16_d(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
/* the value of lane L ^ 8 (a rotation by 8 inside each 16-lane row, DPP row_ror:8) */
__device__ __forceinline__ double xor8_d(double v) {
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x128, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x128, 0xf, 0xf, false));
}

/* Sum over the 64 lanes of x[0..7] at once (a transposed butterfly: 10
 * exchanges instead of 8 x 6): lane L returns the total of x[(L >> 3) & 7].
 * The first two levels are half swaps: after swap32(x[i], x[i + 4]) the low
 * half holds (x[i], its partner's x[i]) and the high half (x[i + 4]'s partner
 * value, x[i + 4]), so one add gives each half its pair sum — the additions of
 * the shuffle form with the operands of the high half commuted, the same bits. */
__device__ __forceinline__ double wave_sum8_d(double (&x)[8]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double a = x[i], b = x[i + 4];
        swap32_d(a, b);
        x[i] = a + b;  // lanes 0-31: x[i] + x[i]^32; lanes 32-63: x[i+4]^32 + x[i+4]
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
        double a = x[i], b = x[i + 2];
        swap16_d(a, b);
        x[i] = a + b;
    }
    {
        const bool hi = lane & 8;
        const double keep = hi ? x[1] : x[0], give = hi ? x[0] : x[1];
        x[0] = keep + xor8_d(give);
    }
    double v = x[0];
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
    return v;
}

/* The CPHD terms of cphd_wave for M <= 64 when the cardinality series is
 * complete: S(K) = Σ_{i<=K} λ^i / i! with λ = W r equals e^λ to double
 * precision for every K >= T0 = Nmax - M - 1 once the Poisson tail beyond T0 is
 * below e^-45 (Chernoff: e^-λ (e λ / K)^K), so log S(K) = λ with no series.
 * The elementary-symmetric inner products Σ_a P_m[a] T_m[a] run as ONE forward
 * chain of the prefix products P_m (kept in registers, half the measurements at
 * a time) and ONE backward chain of the suffix sums T_m, the 64 per-measurement
 * wave sums batched eight at a time (wave_sum8_d) — instead of the segmented,
 * partly redundant chains of cphd_wave.  Same quantities, same positive
 * recursions.  Returns false (nothing written) when the series condition fails. */
/* pst: NULL keeps the stored prefix products in registers (32 doubles per
 * lane: the one-wave launch, k_cphd_terms); else an LDS buffer of 32 x 64
 * doubles for them (PST_LDS, 16 KB: inside a larger workgroup whose register
 * budget is shared with the rest of the update). */
template <bool PST_LDS = false>
__device__ bool cphd_fast64(const UpdateArgs& a, int n, int M, const u64* ehi, const u64* elo, double lo_unscale,
                            double win, double qd, double W, float* leta, float* thr, CphdOut& out,
                            double* pst = nullptr) {
    const DevCfg& c = a.c;
    const int lane = threadIdx.x & 63;
    const int Nmax = a.Nmax;
    if (M > 64 || M < 1) return false;
    win = uni_d(win);
    qd = uni_d(qd);
    W = uni_d(W);
    const double lw = win > 0 ? log(win) : -INFINITY;
    const double lq = qd > 0 ? log(qd) : -INFINITY;
    const double logW = W > 0 ? log(W) : -INFINITY;
    const double lr = win > 0 ? lq - lw : (double)c.cphd_log1mpd;
    const double aexp = logW + lr;
    const double dd = (win > 0 && W > 0) ? logW - lw : 0.0;
    const int T0 = Nmax - M - 1;
    if (T0 < 1) return false;
    const double lam = aexp > -INFINITY ? exp(aexp) : 0.0;  // Poisson mean of the series
    if (lam > 0.0) {
        const double K = (double)T0;
        if (!(K > lam) || !(-lam + K * (1.0 + aexp - log(K)) < -45.0)) return false;
    }
    const double lSc = lam;  // log S(K), every K in [T0, Nmax]
    const double S = lane < M ? (double)ehi[lane] * 9.094947017729282e-13 + (double)elo[lane] * lo_unscale : 0.0;
    const double lam0 = (lane < M && S > 0) ? log(S) + c.cphd_lck : -INFINITY;
    const double lmax = wave_max_dx(lam0);
    const double lsum = wave_sum_dx(lane < M ? lam0 : 0.0);
    const double lp = lam0 == -INFINITY ? 0.0 : exp(lam0 - lmax);  // λ'_m, lane m
    // λ' of every measurement in LDS: the chains below read λ'_m as a broadcast
    // LDS load (issued ahead of the chain) instead of two v_readlane each
    __shared__ double s_lp[64];
    s_lp[lane] = lp;
    wsync();  // (one wave: no workgroup barrier, so a larger workgroup's wave 0 can run it alone)
    auto lB0f = [&](int j) { return Nmax - j >= 0 ? (j == 0 ? 0.0 : (double)j * dd) - W + lSc : -INFINITY; };
    auto lB1f = [&](int j) { return Nmax - j - 1 >= 0 ? (double)(j + 1) * dd - W + lSc : -INFINITY; };
    double bv = -INFINITY;
    if (lane < M) {
        const double b1 = lB1f(lane);
        if (b1 != -INFINITY) bv = (double)(M - 1 - lane) * c.cphd_lrate - c.cphd_rate + b1 + kpow_d(lane, lmax);
    }
    const double bmax = wave_max_dx(bv);
    double T = (bv == -INFINITY || bmax == -INFINITY) ? 0.0 : exp(bv - bmax);  // T_{M-1} = β'
    double ipm = 0.0;   // lane m: Σ_a P_m[a] T_m[a] (scaled by e^-bmax)
    double Pfull = 0.0; // P_M: the ESF of all Λ' (lane k: coefficient k)
#pragma unroll
    for (int h = 1; h >= 0; h--) {  // measurements [32h, 32h + 32): P_m stored for this half
        double Pst_r[PST_LDS ? 1 : 32];
        auto Pst = [&](int i) -> double& {
            if constexpr (PST_LDS) return pst[i * 64 + lane];
            else return Pst_r[i];
        };
        double P = lane == 0 ? 1.0 : 0.0;
#pragma unroll
        for (int m = 0; m < 32 * h + 32; m++) {
            if (m >= 32 * h) Pst(m - 32 * h) = P;
            if (m < M) P = fma(s_lp[m], dpp_or_zero_d<0x138, 0xf>(P), P);
        }
        if (h == 1) Pfull = P;
#pragma unroll
        for (int b = 3; b >= 0; b--) {  // batches of 8 measurements, descending
            double x[8];
#pragma unroll
            for (int q = 7; q >= 0; q--) {
                const int m = 32 * h + 8 * b + q;
                x[q] = m < M ? Pst(m - 32 * h) * T : 0.0;
                if (m < M) T = fma(s_lp[m], dpp_or_zero_d<0x130, 0xf>(T), T);
            }
            const double sum = wave_sum8_d(x);  // lane L: measurement 32h + 8b + (L >> 3)
            const int m0 = 32 * h + 8 * b;
            const double mine = __shfl(sum, ((lane - m0) & 7) << 3, 64);
            if (lane >= m0 && lane < m0 + 8) ipm = mine;
        }
    }
    // b_k = log of the hypothesis terms (k <= M; k = 64 is a scalar when M = 64)
    double bk = -INFINITY, p0 = -INFINITY, q0 = -INFINITY;
    if (lane <= M) {
        const double le = lane == M ? lsum : (Pfull > 0 ? log(Pfull) + kpow_d(lane, lmax) : -INFINITY);
        if (le != -INFINITY) {
            bk = (double)(M - lane) * c.cphd_lrate - c.cphd_rate + le;
            p0 = bk + lB0f(lane);
            q0 = bk + lB1f(lane);
        }
    }
    double b64 = -INFINITY, p1 = -INFINITY, q1 = -INFINITY;  // k = 64 (M = 64 only), on lane 0
    if (M == 64 && lane == 0) {
        b64 = -c.cphd_rate + lsum;
        p1 = b64 + lB0f(64);
        q1 = b64 + lB1f(64);
    }
    const double ip0 = uni_d(wave_lse2(p0, p1));
    const double ip1 = uni_d(wave_lse2(q0, q1));
    G1 double* co = a.cn_coef ? g1(uni_p(a.cn_coef + (size_t)n * a.cn_stride)) : nullptr;
    if (co) {
        if (lane <= M) co[6 + lane] = bk;
        if (M == 64 && lane == 0) co[6 + 64] = b64;
        if (lane == 0) {
            co[0] = ip0;
            co[1] = lq;
            co[2] = lw;
            co[3] = logW;
            co[4] = W;
            co[5] = (double)M;
        }
    }
    int wide = 0;
    if (lane < M) {
        const float le_m = (float)((ip0 - (ipm > 0 ? log(ipm) + bmax : -INFINITY)) - c.cphd_lck);
        leta[lane] = le_m;
        thr[lane] = (c.log_minfw + le_m - 0.5f) * 1.4426950408889634f;
        wide = !(le_m >= c.cphd_leta_min);
    }
    out.ip0 = ip0;
    out.ip1 = ip1;
    out.bmax = bmax;
    out.wide = __ballot(wide != 0) != 0ull;
    return true;
}

/* Outputs of the CPHD terms into particle n's handoff and weight: the
 * non-detection log factor and the wide flag (handoff misc; the detection
 * factors and listing bounds are already there), Δ log w = <Ψ0,p>. */
__device__ __forceinline__ void cphd_terms_store(const UpdateArgs& a, unsigned char* hand, const CphdHand& H, int n,
                                                 double ip0, double ip1, int wide) {
    ((float*)(hand + H.misc))[0] = (float)(ip1 - ip0 + (double)a.c.cphd_log1mpd);  // non-detection
    ((int*)(hand + H.misc))[1] = wide;
    const float delta = (float)ip0;  // particle weight *= <Ψ0,p> (.bak:2697)
    a.delta[n] = delta;
    const float nw = a.logw[n] + delta;
    a.logw[n] = nw;
    if (a.logw_out) a.logw_out[n] = nw;
}

/* The fast form of the CPHD terms of particle n by ONE wave (lanes
 * threadIdx.x & 63) from part A's handoff, when it applies (M <= 64 and a
 * complete cardinality series, cphd_fast64): the per-measurement detection
 * factors and listing bounds, then cphd_terms_store.  Returns false (nothing
 * written) when the general form is needed.  PST_LDS: pst = 16 KB of LDS for
 * the stored prefix products. */
template <bool PST_LDS = false>
__device__ __forceinline__ bool cphd_terms_fast(const UpdateArgs& a, int n, double* pst = nullptr) {
    const CphdHand H = cphd_hand_layout(a.cap, a.Mcap, a.Scap);
    unsigned char* hand = a.hand + (size_t)n * H.stride;
    const double* sums = (const double*)(hand + H.sums);
    const double lo_unscale = a.cap <= 2047 ? 8.470329472543003e-22 : 8.673617379884035e-19;
    CphdOut co;
    if (!cphd_fast64<PST_LDS>(a, n, a.M, (const u64*)(hand + H.ehi), (const u64*)(hand + H.elo), lo_unscale, sums[1],
                              sums[2], sums[3], (float*)(hand + H.leta), (float*)(hand + H.thr), co, pst))
        return false;
    if ((threadIdx.x & 63) == 0) cphd_terms_store(a, hand, H, n, co.ip0, co.ip1, co.wide);
    return true;
}

/* The CPHD terms of particle n by ONE wave: the fast form, else the general
 * one (cphd_wave, any M <= 127, the truncated series summed).  sc: 7 (Mcap + 4)
 * doubles of LDS scratch. */
__device__ __forceinline__ void cphd_terms_one(const UpdateArgs& a, int n, double* sc) {
    if (cphd_terms_fast<false>(a, n)) return;
    const CphdHand H = cphd_hand_layout(a.cap, a.Mcap, a.Scap);
    unsigned char* hand = a.hand + (size_t)n * H.stride;
    const double* sums = (const double*)(hand + H.sums);
    const double lo_unscale = a.cap <= 2047 ? 8.470329472543003e-22 : 8.673617379884035e-19;
    CphdOut co;
    cphd_wave(a, n, a.M, (const u64*)(hand + H.ehi), (const u64*)(hand + H.elo), lo_unscale, sums[1], sums[2], sums[3],
              sc, (float*)(hand + H.leta), (float*)(hand + H.thr), co);
    if ((threadIdx.x & 63) == 0) cphd_terms_store(a, hand, H, n, co.ip0, co.ip1, co.wide);
}

}  // namespace phd
