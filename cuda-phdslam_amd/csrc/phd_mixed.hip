/*
 * phd_mixed.hip — the mixed static + dynamic feature model on gfx950
 * (feature_model = 2).
 *
 * k_predict_dynamic: predictMapMixed (phdfilter.cu:966-1035, kernel :910-963),
 *   one thread per dynamic component of every slab: constant-velocity
 *   prediction, weight x p_jmm x ps.  Static maps are not predicted (:1241).
 * k_update_mixed: phdUpdateSynth's MIXED_MODEL branch (:3412-3462,
 *   phdUpdateKernelMixed :2323-2635, mergeAndCopyMaps :3703-3726), one
 *   256-thread workgroup per particle:
 *     1. range classes of both maps (computeInRangeKernel :1327-1346),
 *        order-preserving ballot compaction (static: in / near / out; dynamic:
 *        in — the rest is dropped, :3715-3719);
 *     2. pre-update terms of every in-range component (computePreUpdate
 *        :302-521) into per-particle global scratch;
 *     3. one normaliser per measurement over BOTH maps' detection terms +
 *        clutter + birth weight(s) (:2463-2550), a thread per measurement
 *        summing in component order (double); Δ log w = Σ log η_m − Σ pd w
 *        (:2553);
 *     4. per map: candidates in the reference's update-array order
 *        [non-detect | detect (m-major) | births] (+ nearly in-range static
 *        components), pruned below minFeatureWeight (:2611-2633), compacted in
 *        order into global scratch;
 *     5. per map: the greedy merge of phdUpdateMergeKernel (:2739-2890): seed =
 *        heaviest unmerged (lowest index on ties, D1), members = unmerged with
 *        d(seed, i) < minSeparation (2-D / 4-D Mahalanobis), listed in index
 *        order; one lane sums them in that order in double, so the moments
 *        equal the oracle's bit for bit; static out-of-range components are
 *        appended.
 * The arithmetic is include/phd_mixed.h (shared with the oracle).  This is a
 * correctness-first form: no benchmark config of the reference uses the mixed
 * model, so it is not tuned like the static update.
 */
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include <hipcub/hipcub.hpp>

#include <vector>

#include "phd_detmath.h"
#include "phd_mixed_k.h"

namespace phd {

#define MX_NT 256
#define MX_W (MX_NT / 64)
#define MX_EKF 32 /* floats of one phd_mx_ekf */

static_assert(sizeof(phd_mx_ekf) == MX_EKF * sizeof(float), "phd_mx_ekf layout");

/* rank of this thread among the block's threads with pred set (thread order) */
__device__ __forceinline__ int mx_rank(bool pred, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long b = __ballot(pred);
    const int within = __popcll(b & ((1ull << lane) - 1ull));
    __syncthreads();  // s_w of a previous call has been read
    if (lane == 0) s_w[wid] = __popcll(b);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < MX_W; w++) {
        const int c = s_w[w];
        off += (w < wid) ? c : 0;
        tot += c;
    }
    *total = tot;
    return off + within;
}

__device__ __forceinline__ bool mx_better(float aw, int ai, float bw, int bi) {
    return ai >= 0 && (bi < 0 || aw > bw || (aw == bw && ai < bi));
}

template <int D>
struct MxComp {
    static constexpr int F = 1 + D + D * D;  // w | mean | cov
};

/* prior component j of a slab (static SoA: w mx my P00 P10 P01 P11; dynamic:
 * w m0..m3 c0..c15) */
template <int D>
__device__ __forceinline__ void mx_read_prior(const float* slab, int scap, int j, float& w, float* m, float* c) {
    w = slab[j];
#pragma unroll
    for (int k = 0; k < D; k++) m[k] = slab[(1 + k) * scap + j];
#pragma unroll
    for (int k = 0; k < D * D; k++) c[k] = slab[(1 + D + k) * scap + j];
}

/* Candidates of one map in the reference's update-array order, pruned and
 * compacted into cand (AoS, F floats each).  Returns the count (> Kcap: overflow). */
template <int D>
__device__ int mx_candidates(const MixedArgs& a, const phd_pose& pose, const float* slab, int scap, const int* s_list,
                             int G, const phd_mx_ekf* ekf, const float* s_leta, const int* s_near, int Gnear,
                             int label, float* cand, int* s_w) {
    constexpr int F = MxComp<D>::F;
    const int M = a.M;
    const long R = (long)G + (long)M * G + M + Gnear;
    const float minw = a.c.minFeatureWeight;
    int K = 0;
    for (long base = 0; base < R; base += MX_NT) {
        const long r = base + threadIdx.x;
        float w = 0.f, m[D], c[D * D];
        bool keep = false;
        if (r < G) {  // non-detection
            const int j = s_list[r];
            float w0;
            mx_read_prior<D>(slab, scap, j, w0, m, c);
            w = w0 * (1 - ekf[r].pd);
            keep = !(w < minw);
        } else if (r < (long)G + (long)M * G) {  // detection of measurement mm by component t
            const long q = r - G;
            const int mm = (int)(q / G), t = (int)(q % G);
            const phd_mx_ekf& e = ekf[t];
            float w0;
            mx_read_prior<D>(slab, scap, s_list[t], w0, m, c);
            const int ok = a.zlab[mm] == label || !a.c.labeled;
            float i0, i1;
            const float lq = phd_mx_logq(e, w0, a.zr[mm], a.zb[mm], ok, &i0, &i1);
#pragma unroll
            for (int k = 0; k < D; k++) m[k] = m[k] + e.K[k] * i0 + e.K[(D == 2 ? 2 : 4) + k] * i1;
#pragma unroll
            for (int k = 0; k < D * D; k++) c[k] = e.cu[k];
            w = phd_det_expf(lq - s_leta[mm]);
            keep = !(w < minw);
        } else if (r < (long)G + (long)M * G + M) {  // birth of measurement mm
            const int mm = (int)(r - G - (long)M * G);
            const int ok = a.zlab[mm] == label || !a.c.labeled;
            const float lw = phd_mx_birth(a.c, pose, a.zr[mm], a.zb[mm], ok, D, m, c);
            w = phd_det_expf(lw - s_leta[mm]);
            keep = !(w < minw);
        } else if (r < R) {  // nearly in range (static): joins the merge unpruned
            mx_read_prior<D>(slab, scap, s_near[r - G - (long)M * G - M], w, m, c);
            keep = true;
        }
        int tot;
        const int slot = K + mx_rank(keep, s_w, &tot);
        if (keep && slot < a.Kcap) {
            float* o = cand + (size_t)slot * F;
            o[0] = w;
#pragma unroll
            for (int k = 0; k < D; k++) o[1 + k] = m[k];
#pragma unroll
            for (int k = 0; k < D * D; k++) o[1 + D + k] = c[k];
        }
        K += tot;
    }
    __syncthreads();  // candidates visible to the block
    return K;
}

/* Greedy merge (phdUpdateMergeKernel) of K candidates into dst (SoA slab,
 * capacity scap).  Returns the number of merged components (may exceed scap:
 * overflow, only the first scap written). */
template <int D>
__device__ int mx_merge(const MixedArgs& a, const float* cand, int K, float* dst, int scap, unsigned char* s_merged,
                        int* s_list, int* s_w, float* s_wf, int* s_wi, int* s_misc) {
    constexpr int F = MxComp<D>::F;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float T = a.c.minSeparation;
    for (int i = tid; i < K; i += MX_NT) s_merged[i] = 0;
    __syncthreads();
    int nout = 0;
    while (true) {
        // seed: heaviest unmerged candidate, lowest index on ties (D1)
        float bw = 0.f;
        int bi = -1;
        for (int i = tid; i < K; i += MX_NT) {
            if (s_merged[i]) continue;
            const float w = cand[(size_t)i * F];
            if (mx_better(w, i, bw, bi)) {
                bw = w;
                bi = i;
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float ow = __shfl_xor(bw, off);
            const int oi = __shfl_xor(bi, off);
            if (mx_better(ow, oi, bw, bi)) {
                bw = ow;
                bi = oi;
            }
        }
        if (lane == 0) {
            s_wf[wid] = bw;
            s_wi[wid] = bi;
        }
        __syncthreads();
        if (tid == 0) {
            float w0 = s_wf[0];
            int i0 = s_wi[0];
            for (int w = 1; w < MX_W; w++)
                if (mx_better(s_wf[w], s_wi[w], w0, i0)) {
                    w0 = s_wf[w];
                    i0 = s_wi[w];
                }
            s_misc[0] = i0;
        }
        __syncthreads();
        const int seed = s_misc[0];
        if (seed < 0) break;
        const float* sd = cand + (size_t)seed * F;
        float sm[D], sc[D * D];
#pragma unroll
        for (int k = 0; k < D; k++) sm[k] = sd[1 + k];
#pragma unroll
        for (int k = 0; k < D * D; k++) sc[k] = sd[1 + D + k];
        // members in index order
        int cnt = 0;
        for (int base = 0; base < K; base += MX_NT) {
            const int i = base + tid;
            bool mem = false;
            if (i < K && !s_merged[i]) {
                const float* ci = cand + (size_t)i * F;
                const float d = D == 2 ? phd_mahal2(sc, sm, ci + 1 + D, ci + 1) : phd_mahal4(sc, sm, ci + 1 + D, ci + 1);
                mem = d < T;
            }
            int tot;
            const int r = mx_rank(mem, s_w, &tot);
            if (mem) s_list[cnt + r] = i;
            cnt += tot;
        }
        __syncthreads();
        if (tid == 0) {
            double W = 0.0, md[D];
#pragma unroll
            for (int k = 0; k < D; k++) md[k] = 0.0;
            for (int q = 0; q < cnt; q++) {
                const float* ci = cand + (size_t)s_list[q] * F;
                W += (double)ci[0];
#pragma unroll
                for (int k = 0; k < D; k++) md[k] += (double)(ci[0] * ci[1 + k]);
            }
            const float Wf = (float)W;
            int stop = 0;
            if (Wf == 0.f) {
                stop = 1;
            } else {
                float g[D], gc[D * D];
                double cd[D * D];
#pragma unroll
                for (int k = 0; k < D; k++) g[k] = (float)md[k] / Wf;
#pragma unroll
                for (int k = 0; k < D * D; k++) cd[k] = 0.0;
                for (int q = 0; q < cnt; q++) {
                    const float* ci = cand + (size_t)s_list[q] * F;
                    float dm[D];
#pragma unroll
                    for (int k = 0; k < D; k++) dm[k] = g[k] - ci[1 + k];
                    const float w = ci[0];
#pragma unroll
                    for (int j = 0; j < D; j++)
#pragma unroll
                        for (int k = 0; k < D; k++)
                            cd[j * D + k] += (double)(w * (ci[1 + D + j * D + k] + dm[j] * dm[k]));
                    s_merged[s_list[q]] = 1;
                }
#pragma unroll
                for (int k = 0; k < D * D; k++) gc[k] = (float)cd[k] / Wf;
                phd_mx_symmetrize(gc, D);
                if (nout < scap) {
                    dst[nout] = Wf;
#pragma unroll
                    for (int k = 0; k < D; k++) dst[(1 + k) * scap + nout] = g[k];
#pragma unroll
                    for (int k = 0; k < D * D; k++) dst[(1 + D + k) * scap + nout] = gc[k];
                }
            }
            s_misc[1] = stop;
        }
        __syncthreads();
        if (s_misc[1]) break;
        nout++;
    }
    return nout;
}

__global__ void __launch_bounds__(MX_NT) k_update_mixed(MixedArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char mx_smem[];
    const int n = blockIdx.x, tid = threadIdx.x;
    const int cap = a.cap, dcap = a.dcap, M = a.M;
    int* s_in = (int*)mx_smem;
    int* s_near = s_in + cap;
    int* s_out = s_near + cap;
    int* d_in = s_out + cap;
    float* s_leta = (float*)(d_in + dcap);
    int* s_list = (int*)(s_leta + (M > 0 ? M : 1));
    unsigned char* s_merged = (unsigned char*)(s_list + a.Kcap);
    __shared__ int s_w[MX_W];
    __shared__ float s_wf[MX_W];
    __shared__ int s_wi[MX_W];
    __shared__ int s_misc[4];
    __shared__ float s_delta;

    const phd_pose pose = a.poses[n];
    const int slab = a.src[n];
    const float* S = a.map_in + (size_t)slab * 7 * cap;
    const float* DY = a.dmap_in + (size_t)slab * PHD_DYN_FIELDS * dcap;
    const int ns = min(a.size_in[slab], cap), nd = min(a.dsize_in[slab], dcap);
    int flags = 0;

    // 1. range classes, order-preserving compaction
    int Gs = 0, Gn = 0, Go = 0, Gd = 0;
    for (int base = 0; base < ns; base += MX_NT) {
        const int j = base + tid;
        const int cls = j < ns ? phd_mx_range_class(a.c, pose, S[cap + j], S[2 * cap + j]) : -1;
        int t1, t2, t0;
        const int r1 = mx_rank(cls == 1, s_w, &t1);
        if (cls == 1) s_in[Gs + r1] = j;
        const int r2 = mx_rank(cls == 2, s_w, &t2);
        if (cls == 2) s_near[Gn + r2] = j;
        const int r0 = mx_rank(cls == 0, s_w, &t0);
        if (cls == 0) s_out[Go + r0] = j;
        Gs += t1;
        Gn += t2;
        Go += t0;
    }
    for (int base = 0; base < nd; base += MX_NT) {
        const int j = base + tid;
        const int cls = j < nd ? phd_mx_range_class(a.c, pose, DY[dcap + j], DY[2 * dcap + j]) : -1;
        int t1;
        const int r1 = mx_rank(cls == 1, s_w, &t1);
        if (cls == 1) d_in[Gd + r1] = j;
        Gd += t1;
    }
    __syncthreads();

    // 2. pre-update terms of the in-range components
    phd_mx_ekf* es = (phd_mx_ekf*)(a.ekf + (size_t)n * (cap + dcap) * MX_EKF);
    phd_mx_ekf* ed = es + cap;
    for (int t = tid; t < Gs + Gd; t += MX_NT) {
        phd_mx_ekf e;
        if (t < Gs) {
            float w, m[2], c[4];
            mx_read_prior<2>(S, cap, s_in[t], w, m, c);
            phd_mx_ekf2(a.c, pose, m, c, e);
            es[t] = e;
        } else {
            float w, m[4], c[16];
            mx_read_prior<4>(DY, dcap, d_in[t - Gs], w, m, c);
            phd_mx_ekf4(a.c, pose, m, c, e);
            ed[t - Gs] = e;
        }
    }
    __syncthreads();

    // 3. normalisers (both maps) and the particle weight
    for (int m = tid; m < M; m += MX_NT) {
        const int ok_s = a.zlab[m] == PHD_MEAS_STATIC || !a.c.labeled;
        const int ok_d = a.zlab[m] == PHD_MEAS_DYNAMIC || !a.c.labeled;
        double sd = 0.0;
        float i0, i1;
        for (int t = 0; t < Gs; t++)
            sd += (double)phd_det_expf(phd_mx_logq(es[t], S[s_in[t]], a.zr[m], a.zb[m], ok_s, &i0, &i1));
        for (int t = 0; t < Gd; t++)
            sd += (double)phd_det_expf(phd_mx_logq(ed[t], DY[d_in[t]], a.zr[m], a.zb[m], ok_d, &i0, &i1));
        sd += (double)a.c.clutterDensity;
        sd += (double)a.c.birthWeight;
        if (!a.c.labeled) sd += (double)a.c.birthWeight;
        s_leta[m] = phd_mx_safe_log((float)sd);
    }
    __syncthreads();
    if (tid == 0) {
        double card = 0.0;
        for (int t = 0; t < Gs; t++) card += (double)(es[t].pd * S[s_in[t]]);
        for (int t = 0; t < Gd; t++) card += (double)(ed[t].pd * DY[d_in[t]]);
        float pw = 0.f;
        for (int m = 0; m < M; m++) pw += s_leta[m];
        s_delta = pw - (float)card;
    }

    // 4-5. static map: candidates, merge, out-of-range appended
    float* cs = a.cand + (size_t)n * a.Kcap * (MxComp<2>::F + MxComp<4>::F);
    float* cd = cs + (size_t)a.Kcap * MxComp<2>::F;
    float* so = a.map_out + (size_t)n * 7 * cap;
    int Ks = mx_candidates<2>(a, pose, S, cap, s_in, Gs, es, s_leta, s_near, Gn, PHD_MEAS_STATIC, cs, s_w);
    if (Ks > a.Kcap) {
        flags |= PHD_ST_CANDIDATE_OVERFLOW_MX;
        Ks = a.Kcap;
    }
    const int nos = mx_merge<2>(a, cs, Ks, so, cap, s_merged, s_list, s_w, s_wf, s_wi, s_misc);
    for (int t = tid; t < Go; t += MX_NT) {
        const int slot = nos + t;
        if (slot < cap)
            for (int f = 0; f < 7; f++) so[f * cap + slot] = S[f * cap + s_out[t]];
    }
    // dynamic map
    float* dout = a.dmap_out + (size_t)n * PHD_DYN_FIELDS * dcap;
    int Kd = mx_candidates<4>(a, pose, DY, dcap, d_in, Gd, ed, s_leta, nullptr, 0, PHD_MEAS_DYNAMIC, cd, s_w);
    if (Kd > a.Kcap) {
        flags |= PHD_ST_CANDIDATE_OVERFLOW_MX;
        Kd = a.Kcap;
    }
    const int nod = mx_merge<4>(a, cd, Kd, dout, dcap, s_merged, s_list, s_w, s_wf, s_wi, s_misc);
    if (tid == 0) {
        int ts = nos + Go;
        if (ts > cap || nod > dcap) flags |= PHD_ST_MAP_OVERFLOW_MX;
        a.size_out[n] = min(ts, cap);
        a.dsize_out[n] = min(nod, dcap);
        a.status[n] = flags;
        if (flags) {
            atomicOr(a.err, flags);
            atomicAdd(a.err + 3, 1);
        }
        a.delta[n] = s_delta;
        a.logw[n] += s_delta;
        a.src_reset[n] = n;
    }
}

__global__ void __launch_bounds__(256) k_predict_dynamic(int nslabs, int dcap, const float* __restrict__ din,
                                                         const int* __restrict__ dsize_in, float* __restrict__ dout,
                                                         int* __restrict__ dsize_out, phd_mx_cfg c) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(gid / dcap), k = (int)(gid % dcap);
    if (s >= nslabs) return;
    const int sz = min(max(dsize_in[s], 0), dcap);
    if (k == 0) dsize_out[s] = sz;
    if (k >= sz) return;
    const float* src = din + (size_t)s * PHD_DYN_FIELDS * dcap;
    float* dst = dout + (size_t)s * PHD_DYN_FIELDS * dcap;
    float w, m[4], p[16], mo[4], po[16], wo;
    mx_read_prior<4>(src, dcap, k, w, m, p);
    phd_mx_predict4(c, m, p, w, mo, po, &wo);
    dst[k] = wo;
    for (int i = 0; i < 4; i++) dst[(1 + i) * dcap + k] = mo[i];
    for (int i = 0; i < 16; i++) dst[(5 + i) * dcap + k] = po[i];
}

size_t mixed_lds_bytes(int cap, int dcap, int Mcap, int Kcap) {
    return (size_t)4 * (3 * (size_t)cap + dcap) + 4 * (size_t)(Mcap > 0 ? Mcap : 1) + 4 * (size_t)Kcap +
           (size_t)Kcap + 16;
}

size_t mixed_ekf_floats(int cap, int dcap) { return (size_t)(cap + dcap) * MX_EKF; }

size_t mixed_cand_floats(int Kcap) { return (size_t)Kcap * (MxComp<2>::F + MxComp<4>::F); }

hipError_t mixed_set_lds_limit() {
    // (the static __shared__ words come out of the same 160 KB)
    return hipFuncSetAttribute((const void*)k_update_mixed, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
}

hipError_t mixed_launch_update(const MixedArgs& a, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_update_mixed, dim3(a.n), dim3(MX_NT), lds, s, a);
    return hipGetLastError();
}

hipError_t mixed_launch_predict(int nslabs, int dcap, const float* din, const int* dsize_in, float* dout,
                                int* dsize_out, const phd_mx_cfg& c, hipStream_t s) {
    const long total = (long)nslabs * dcap;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_predict_dynamic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, nslabs, dcap, din,
                       dsize_in, dout, dsize_out, c);
    return hipGetLastError();
}

/* ---- EAP map of the dynamic maps (exp_map_dynamic, main.cpp:369-371) ----
 * computeExpectedMap over maps_dynamic (main.cpp:290-316): every particle's
 * Gaussian4D components with weight x exp(log w_n) (D8: det_expf), then
 * reduceGaussianMixture<Gaussian4D> (gm_reduce.cpp:59-132): stable priority
 * order (weight descending, concatenation index ascending; a stable radix
 * sort), seeds in that order absorb every unmerged later component at LLT
 * Mahalanobis distance < minSeparation (phd_eap_mahal4), the moments summed
 * serially in priority order by one lane (phd_eap4_*, the oracle's
 * expressions: orc_expected_map_dynamic) — one workgroup over the whole set
 * (dynamic maps are small: no benchmark config uses the mixed model). */
__global__ void __launch_bounds__(256) k_eap4_gather(const int* __restrict__ src, const float* __restrict__ dmap,
                                                     const int* __restrict__ off, const float* __restrict__ logw,
                                                     int dcap, long K, float* __restrict__ comp) {
    const int p = blockIdx.x;
    const int r = src[p] & 0x3fffffff;
    const float* s = dmap + (size_t)r * PHD_DYN_FIELDS * dcap;
    const int o = off[p], sz = off[p + 1] - o;
    const float ew = phd_det_expf(logw[p]);
    for (int k = threadIdx.x; k < sz; k += blockDim.x) {
        comp[o + k] = s[k] * ew;  // map[i].weight *= exp(weights[n]) (main.cpp:302-303)
        for (int f = 1; f < PHD_DYN_FIELDS; f++) comp[(size_t)f * K + o + k] = s[(size_t)f * dcap + k];
    }
}

__global__ void k_eap4_iota(unsigned int* a, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (unsigned int)i;
}

#define EAP4_NT 1024
__global__ void __launch_bounds__(EAP4_NT) k_eap4_merge(const float* __restrict__ comp, long K,
                                                        const unsigned int* __restrict__ ord, float T,
                                                        unsigned char* __restrict__ flag, unsigned int* __restrict__ mem,
                                                        phd_gaussian4d* __restrict__ out, int* __restrict__ nout) {
    __shared__ int s_w[EAP4_NT / 64];
    __shared__ float s_seed[PHD_DYN_FIELDS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (long j = tid; j < K; j += EAP4_NT) flag[j] = 0;
    __syncthreads();
    auto fld = [&](unsigned int c, int f) { return comp[(size_t)f * K + c]; };
    int count = 0;
    long p = 0;
    while (p < K) {
        // the seed: the first unmerged priority position >= p
        long s = K;
        for (long base = p; base < K && s == K; base += EAP4_NT) {
            const long j = base + tid;
            int v = (j < K && flag[j] == 0) ? (int)(j - base) : EAP4_NT;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
            if (lane == 0) s_w[wid] = v;
            __syncthreads();
            int m = EAP4_NT;
            for (int w = 0; w < EAP4_NT / 64; w++) m = min(m, s_w[w]);
            __syncthreads();
            if (m < EAP4_NT) s = base + m;
        }
        if (s >= K) break;
        const unsigned int si = ord[s];
        if (tid < PHD_DYN_FIELDS) s_seed[tid] = fld(si, tid);
        __syncthreads();
        float sm[4], sc[16];
        for (int i = 0; i < 4; i++) sm[i] = s_seed[1 + i];
        for (int i = 0; i < 16; i++) sc[i] = s_seed[5 + i];
        // absorb the unmerged later components within T, listed in priority order
        int nm = 0;
        for (long base = s + 1; base < K; base += EAP4_NT) {
            const long j = base + tid;
            bool in = false;
            if (j < K && flag[j] == 0) {
                const unsigned int bi = ord[j];
                float bm[4], bc[16];
                for (int i = 0; i < 4; i++) bm[i] = fld(bi, 1 + i);
                for (int i = 0; i < 16; i++) bc[i] = fld(bi, 5 + i);
                in = phd_eap_mahal4(sm, sc, bm, bc) < T;
            }
            const unsigned long long b = __ballot(in);
            if (lane == 0) s_w[wid] = __popcll(b);
            __syncthreads();
            int pre = nm, tot = 0;
            for (int w = 0; w < EAP4_NT / 64; w++) {
                if (w < wid) pre += s_w[w];
                tot += s_w[w];
            }
            if (in) {
                flag[j] = 1;
                mem[pre + __popcll(b & ((1ull << lane) - 1ull))] = (unsigned int)j;
            }
            nm += tot;
            __syncthreads();
        }
        if (tid == 0) {
            phd_eap4_acc acc;
            const float sw = s_seed[0];
            phd_eap4_mean_begin(acc, sw, sm);
            for (int k = 0; k < nm; k++) {
                const unsigned int bi = ord[mem[k]];
                float bm[4];
                for (int i = 0; i < 4; i++) bm[i] = fld(bi, 1 + i);
                phd_eap4_mean_add(acc, fld(bi, 0), bm);
            }
            phd_eap4_cov_begin(acc, sw, sm, sc);
            for (int k = 0; k < nm; k++) {
                const unsigned int bi = ord[mem[k]];
                float bm[4], bc[16];
                for (int i = 0; i < 4; i++) bm[i] = fld(bi, 1 + i);
                for (int i = 0; i < 16; i++) bc[i] = fld(bi, 5 + i);
                phd_eap4_cov_add(acc, fld(bi, 0), bm, bc);
            }
            phd_eap4_finish(acc, out + count);
            flag[s] = 1;
        }
        count++;
        __syncthreads();
        p = s + 1;
    }
    if (tid == 0) *nout = count;
}

long mixed_expected_map_dynamic(hipStream_t st, const int* d_src, const float* d_dmap, const int* d_dsize, int n,
                                int dcap, const float* d_logw, float T, phd_gaussian4d* out, long out_cap,
                                std::string& err) {
#define E4CHK(expr)                      \
    do {                                 \
        hipError_t _e = (expr);          \
        if (_e != hipSuccess) {          \
            err = hipGetErrorString(_e); \
            return -1;                   \
        }                                \
    } while (0)
    std::vector<int> src(n), sz((size_t)n), off(n + 1, 0);
    E4CHK(hipMemcpyAsync(src.data(), d_src, n * sizeof(int), hipMemcpyDeviceToHost, st));
    E4CHK(hipStreamSynchronize(st));
    int maxs = 0;
    for (int p = 0; p < n; p++) maxs = std::max(maxs, src[p] & 0x3fffffff);
    std::vector<int> dsz(maxs + 1);
    E4CHK(hipMemcpyAsync(dsz.data(), d_dsize, (maxs + 1) * sizeof(int), hipMemcpyDeviceToHost, st));
    E4CHK(hipStreamSynchronize(st));
    for (int p = 0; p < n; p++) off[p + 1] = off[p] + std::min(std::max(dsz[src[p] & 0x3fffffff], 0), dcap);
    const long K = off[n];
    if (K == 0) return 0;
    size_t tmp = 0;
    hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, (float*)nullptr, (float*)nullptr,
                                                 (unsigned int*)nullptr, (unsigned int*)nullptr, (int)K, 0, 32, st);
    const size_t bytes = (size_t)(n + 1) * 4 + (size_t)K * (PHD_DYN_FIELDS * 4 + 4 + 4 + 4 + 4 + 1) +
                         (size_t)K * sizeof(phd_gaussian4d) + tmp + 8 * 256;
    char* buf = nullptr;
    E4CHK(hipMalloc((void**)&buf, bytes));
    size_t o = 0;
    auto take = [&](size_t b) {
        char* q = buf + o;
        o = (o + b + 255) & ~(size_t)255;
        return q;
    };
    int* d_off = (int*)take((n + 1) * 4);
    float* comp = (float*)take((size_t)K * PHD_DYN_FIELDS * 4);
    float* wsorted = (float*)take((size_t)K * 4);
    unsigned int* i0 = (unsigned int*)take((size_t)K * 4);
    unsigned int* ord = (unsigned int*)take((size_t)K * 4);
    unsigned int* mem = (unsigned int*)take((size_t)K * 4);
    unsigned char* flag = (unsigned char*)take((size_t)K);
    phd_gaussian4d* d_out = (phd_gaussian4d*)take((size_t)K * sizeof(phd_gaussian4d));
    int* d_n = (int*)take(4);
    void* d_tmp = take(tmp);
    long nout = -1;
    do {
        if (hipMemcpyAsync(d_off, off.data(), (n + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess) break;
        hipLaunchKernelGGL(k_eap4_gather, dim3(n), dim3(256), 0, st, d_src, d_dmap, d_off, d_logw, dcap, K, comp);
        hipLaunchKernelGGL(k_eap4_iota, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st, i0, K);
        size_t tb = tmp;
        if (hipcub::DeviceRadixSort::SortPairsDescending(d_tmp, tb, comp, wsorted, i0, ord, (int)K, 0, 32, st) !=
            hipSuccess)
            break;
        hipLaunchKernelGGL(k_eap4_merge, dim3(1), dim3(EAP4_NT), 0, st, comp, K, ord, T, flag, mem, d_out, d_n);
        if (hipGetLastError() != hipSuccess) break;
        int cnt = 0;
        if (hipMemcpyAsync(&cnt, d_n, 4, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        nout = cnt;
        if (out && cnt <= out_cap)
            if (hipMemcpyAsync(out, d_out, (size_t)cnt * sizeof(phd_gaussian4d), hipMemcpyDeviceToHost, st) !=
                    hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                nout = -1;
    } while (0);
    if (nout < 0 && err.empty()) err = hipGetErrorString(hipGetLastError());
    hipFree(buf);
    return nout;
#undef E4CHK
}

}  // namespace phd
