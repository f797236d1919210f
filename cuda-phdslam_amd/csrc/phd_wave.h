/*
 * phd_wave.h — LDS layout and launch declarations of the wave-per-particle
 * fused update (phd_wave.hip): one 64-lane wavefront owns one particle for the
 * whole update, so every reduction, scan and compaction is a wave operation
 * (DPP / ballot / mbcnt) and the kernel has no workgroup barrier on its path.
 */
#pragma once
#include <cstddef>

#include "phd_kernels.h"

namespace phd {

/* Byte offsets into the dynamic LDS of one wave (= one workgroup).
 *   persistent : measurements by index, detection factors, listing bounds,
 *                class byte per prior component, counters
 *   region C   : walk phase — bearing-sorted measurements, bearing bins, eta
 *                fixed-point sums, CPHD scratch;
 *                candidate phase on — candidate records P, their V source tag,
 *                the covariances of detection / birth candidates
 *   region R   : walk + candidate phase — survivor keys (unsorted, sorted);
 *                merge — R1 [cell key | bucket starts | culled pairs], later
 *                [CSR offsets | adjacency pool | state]; R2 [edges | degrees] */
struct WaveLds {
    size_t zr, zb, zok, leta, thr, cls, misc;
    size_t zs, zbin, ehi, elo, wtab, cphd;
    size_t cp, ctag, detv;
    size_t skey, skey2;
    size_t mkey, mgst, mplist, moff, mpool, mpar, medge, mcur;
    int plcap, B;
    size_t total;
};

__host__ __device__ inline size_t wv_al(size_t x) { return (x + 15) & ~(size_t)15; }

/* merge lattice buckets of the wave kernel (32 x 32 up to 2048 candidates, 64 x 64 above) */
__host__ __device__ inline int wave_buckets(int Kcap) { return Kcap <= 1024 ? 512 : Kcap <= 2048 ? 1024 : 4096; }

/* edge pool of the wave kernel's parallel merge (overflow -> exact serial greedy) */
__host__ __device__ inline int wave_epool(int Kcap) { return Kcap / 2 + 128; }

__host__ __device__ inline WaveLds wave_lds_layout(int cap, int Mcap, int Kcap, int Scap, int Epool, int cphd) {
    WaveLds L;
    size_t o = 0;
    L.zr = o;
    o = wv_al(o + 4 * (size_t)Mcap);
    L.zb = o;
    o = wv_al(o + 4 * (size_t)Mcap);
    L.zok = o;
    o = wv_al(o + 4 * (size_t)Mcap);
    L.leta = o;
    o = wv_al(o + 4 * (size_t)Mcap);
    L.thr = o;
    o = wv_al(o + 4 * (size_t)Mcap);
    L.cls = o;
    o = wv_al(o + (size_t)cap);
    L.misc = o;
    o = wv_al(o + 64 * 4);
    // region C
    const size_t c0 = o;
    size_t w = c0;
    L.zs = w;
    w = wv_al(w + 16 * (size_t)Mcap);
    L.zbin = w;
    w = wv_al(w + 2 * (size_t)PHD_ZBINS);
    L.ehi = w;  // eta words: hi[256] | lo[256] (the walk addresses lo as hi + 256)
    w = wv_al(w + 8 * 256);
    L.elo = w;
    w = wv_al(w + 8 * 256);
    L.wtab = w;  // balanced walk: 64 x 32 B component table + 64 start bytes
    w = wv_al(w + 32 * 64 + 64);
    L.cphd = w;
    if (cphd) w = wv_al(w + 8 * 8 * ((size_t)Mcap + 4));
    size_t k = c0;
    L.cp = k;
    k = wv_al(k + 16 * (size_t)Kcap);
    L.ctag = k;
    k = wv_al(k + 2 * (size_t)Kcap);
    L.detv = k;
    k = wv_al(k + 16 * ((size_t)Scap + (cphd ? 0 : (size_t)Mcap)));  // CPHD: no births
    o = w > k ? w : k;
    // region R
    const size_t r0 = o;
    const size_t rs = wv_al(r0 + 4 * ((size_t)Scap + 1));  // + the walk's dummy key slot
    const size_t rs2 = wv_al(rs + 4 * (size_t)Scap);
    L.skey = r0;
    L.skey2 = rs;
    L.B = wave_buckets(Kcap);
    // R2 (edges | degrees) first, R1 after it
    L.medge = r0;
    size_t m = wv_al(r0 + 4 * (size_t)Epool);
    L.mcur = m;
    m = wv_al(m + 2 * ((size_t)Kcap + 2));
    const size_t r1 = m;
    // R1, late form: CSR offsets | pool | state
    L.moff = r1;
    size_t q = wv_al(r1 + 2 * ((size_t)Kcap + 2));
    L.mpool = q;
    q = wv_al(q + 4 * (size_t)Epool);
    L.mpar = q;
    q = wv_al(q + 2 * (size_t)Kcap);
    // R1, early form: cell keys | bucket starts | culled pairs (at least Kcap of them)
    L.mkey = r1;
    size_t e = wv_al(r1 + 2 * (size_t)Kcap);
    L.mgst = e;
    e = wv_al(e + 2 * ((size_t)L.B + 2));
    L.mplist = e;
    size_t eend = q > e + 4 * (size_t)Kcap ? q : e + 4 * (size_t)Kcap;
    L.plcap = (int)((eend - e) / 4);
    size_t rend = wv_al(eend);
    if (rend < rs2) rend = rs2;
    L.total = rend;
    return L;
}

/* The edge pool actually used: the largest (up to 1.5 Kcap + 16) that keeps the
 * occupancy of the minimal layout — spare LDS per wave goes to the merge. */
inline int wave_epool_fit(int cap, int Mcap, int Kcap, int Scap, int cphd, size_t lds_per_cu = 160 * 1024) {
    int e = wave_epool(Kcap);
    if (Kcap <= 1024) return e;  // small maps: the minimal pool (occupancy first)
    const size_t t0 = wave_lds_layout(cap, Mcap, Kcap, Scap, e, cphd).total;
    if (t0 > lds_per_cu) return e;
    const size_t budget = (lds_per_cu / (lds_per_cu / t0)) & ~(size_t)15;
    const int emax = (3 * Kcap) / 2 + 16;
    while (e + 16 <= emax && wave_lds_layout(cap, Mcap, Kcap, Scap, e + 16, cphd).total <= budget) e += 16;
    return e;
}

__global__ void k_update_wave(UpdateArgs a);
__global__ void k_update_wave_cphd(UpdateArgs a);
/* the CPHD weight terms of the three-launch workgroup update: one wave per
 * particle from part A's handoff (eta fixed point, sums) to part C's (factors,
 * listing bounds, non-detection factor, wide flag); Δ log w, cardinality
 * coefficients.  Dynamic LDS: cphd_terms_lds(Mcap). */
__global__ void k_cphd_terms(UpdateArgs a);
inline size_t cphd_terms_lds(int Mcap) { return (size_t)7 * 8 * ((size_t)Mcap + 4); }

}  // namespace phd
