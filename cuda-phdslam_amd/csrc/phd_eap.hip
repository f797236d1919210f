/*
 * phd_eap.hip — A10 / SURVEY.md §8(f) rank 1: the EAP expected map on the GPU.
 *
 * Reference: computeExpectedMap (src/main.cpp:290-316) concatenates every
 * particle's map with the component weights scaled by exp(log w_n), then
 * reduceGaussianMixture (src/gm_reduce.cpp:59-132): sort by weight
 * (descending), repeatedly take the heaviest unmerged component, absorb every
 * unmerged component whose Mahalanobis distance (LLT of the averaged
 * covariance, gm_reduce.cpp:30-37) is below minSeparation, emit the
 * moment-matched merge.  The CPU form is O(K^2) over K = N*G components
 * (c3: 2.1 M) — infeasible beyond config 1.
 *
 * Exact parallel form (same outputs, same order as the oracle's
 * orc_expected_map, which fixes the sort to be stable):
 *   1. gather the weighted components (SoA) and the largest covariance
 *      eigenvalue Λ of the set;
 *   2. lattice cells of side R = sqrt(1.05 T Λ): d < T implies |Δμ|² < T Λ,
 *      so merge edges only join cells that touch (8-neighbourhood);
 *   3. order by the global priority (weight descending, concatenation index
 *      ascending: a stable radix sort of the identity), then group the
 *      priority positions by cell (stable radix sort by cell key: ascending
 *      positions within a cell) and run-length-encode the occupied cells;
 *   4. the greedy's decisions as a lexicographically-first maximal independent
 *      set, in synchronous rounds over all positions at once: position j is
 *      absorbed by the first (in priority order) higher-priority position k of
 *      its 3 x 3 cells with d(k, j) < T that is not absorbed elsewhere, if that
 *      k is a seed; it waits while that k is undecided; it is a seed when there
 *      is no such k.  Decisions are final and a same-round read only decides
 *      earlier, so the result is the serial greedy's whatever the timing;
 *   5. members grouped by seed (stable sort: priority order within a group),
 *      one thread per seed sums the moments serially in that order with the
 *      reference's float expression order (bit-identical to the oracle);
 *   6. outputs in their seed's priority order = the reference's emission
 *      order.
 * Non-finite means or a non-finite Λ fall back to one workgroup running the
 * greedy over everything (k_eap_merge; still exact).  Ill-conditioned
 * covariances do not (k_eap_gather: the bound holds for the float distance at
 * any conditioning).
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <vector>

#include "phd_detmath.h"
#include "phd_kernels.h"

#define NF 7 /* fields per component of a map slab (phd_kernels.hip) */

namespace phd {

/* per-particle component counts of the current store (slab references) */
__global__ void k_eap_sizes(const int* __restrict__ src, const int* __restrict__ size_in,
                            const int* __restrict__ size_x, int n, int* __restrict__ sz) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int r = src[p];
    sz[p] = (r & PHD_SLAB_X) ? size_x[r & PHD_SLAB_MASK] : size_in[r & PHD_SLAB_MASK];
}

/* Weighted components (SoA: w x y c00 c10 c01 c11), one block per particle;
 * Λ = max eigenvalue of the symmetric [[c00 c10][c10 c11]] over the set
 * (positive floats order as their bit patterns; a non-finite value sets bad:
 * the exhaustive greedy).
 * The lattice bound holds for the FLOAT LLT distance at any conditioning
 * (DESIGN.md §4.5): the float d satisfies |Δμ|^2 <= (1 + 10 eps) d tr(Σ) (the
 * forward substitution's rounding is relative to s00 and s11, never to the
 * determinant), and tr(Σ) <= 1.01 λmax(Σ) once λmin < λmax / 100; below that
 * condition the float d is within 1e-4 of the exact one, which is >= |Δμ|^2 /
 * λmax(Σ).  Either way d < T puts |Δμ|^2 under 1.05 T λmax(Σ) <= 1.05 T Λ, so
 * ill-conditioned (nearly rank-1) covariances keep the culled decision rounds. */
__global__ void __launch_bounds__(256)
    k_eap_gather(const int* __restrict__ src, const float* __restrict__ map_in, const float* __restrict__ map_x,
                 const int* __restrict__ off, const float* __restrict__ logw, int cap, long K,
                 float* __restrict__ comp, unsigned int* __restrict__ lam_bits, int* __restrict__ bad) {
    const int p = blockIdx.x;
    const int r = src[p];
    const float* s = ((r & PHD_SLAB_X) ? map_x : map_in) + (size_t)(r & PHD_SLAB_MASK) * NF * cap;
    const int o = off[p], sz = off[p + 1] - o;
    // map[i].weight *= exp(weights[n]) (main.cpp:302-303); D8: the deterministic exp shared with the oracle
    const float ew = phd_det_expf(logw[p]);
    float lmax = 0.f;
    int nonfinite = 0;
    for (int k = threadIdx.x; k < sz; k += blockDim.x) {
        const long i = o + k;
        const float w = s[k] * ew;
        const float x = s[1 * cap + k], y = s[2 * cap + k];
        const float a = s[3 * cap + k], b = s[4 * cap + k], c = s[5 * cap + k], d = s[6 * cap + k];
        comp[0 * K + i] = w;
        comp[1 * K + i] = x;
        comp[2 * K + i] = y;
        comp[3 * K + i] = a;
        comp[4 * K + i] = b;
        comp[5 * K + i] = c;
        comp[6 * K + i] = d;
        // λmax of [[a b][b d]] (the LLT reads the lower triangle only)
        const double h = 0.5 * ((double)a + (double)d), q = 0.5 * ((double)a - (double)d);
        const double rt = sqrt(q * q + (double)b * (double)b);
        const double lm = h + rt;
        if (!(fabs(x) < INFINITY && fabs(y) < INFINITY && fabs(lm) < INFINITY)) nonfinite = 1;
        else lmax = fmaxf(lmax, (float)lm * 1.0000002f);
    }
    if (nonfinite) atomicOr(bad, 1);
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o2, 64));
    if ((threadIdx.x & 63) == 0 && lmax > 0.f) atomicMax(lam_bits, __float_as_uint(lmax));
}

__global__ void k_iota_u32(unsigned int* a, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (unsigned int)i;
}

/* rank[i] = priority position of component i; gkey[j] = group of the j-th by priority */
__global__ void k_eap_rank(const unsigned int* __restrict__ by_prio, const unsigned int* __restrict__ gid, long K,
                           unsigned int* __restrict__ rank, unsigned int* __restrict__ gkey) {
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const unsigned int i = by_prio[j];
    rank[i] = (unsigned int)j;
    gkey[j] = gid[i];
}

/* Mahalanobis distance of gm_reduce.cpp:30-37 for 2x2 (Eigen LLT restated,
 * oracle/scphd_cpu.cpp orc_expected_map): seed a, other b. */
__device__ __forceinline__ float eap_dist(float ax, float ay, float a0, float a1, float a3, float bx, float by, float b0,
                                          float b1, float b3) {
    const float s00 = 0.5f * (a0 + b0), s10 = 0.5f * (a1 + b1), s11 = 0.5f * (a3 + b3);
    const float l00 = sqrtf(s00);
    const float l10 = s10 / l00;
    const float l11 = sqrtf(s11 - l10 * l10);
    const float d0 = ax - bx, d1 = ay - by;
    const float x0 = d0 / l00;
    const float x1 = (d1 - l10 * x0) / l11;
    return x0 * x0 + x1 * x1;
}

#define EAP_NT 256
#define EAP_CHUNK 1024  /* members staged in LDS per serial-sum chunk */

/* block-wide min of one int per thread (two barriers; uniform result) */
__device__ __forceinline__ int eap_block_min(int v, int* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    if (lane == 0) s_w[wid] = v;
    __syncthreads();
    int r = s_w[0];
#pragma unroll
    for (int w = 1; w < EAP_NT / 64; w++) r = min(r, s_w[w]);
    __syncthreads();
    return r;
}

/* Greedy reduce of one group (block): members ord[gs .. ge) in priority order.
 * flag[j]: 0 unmerged, 1 merged (per position, private to the block); the
 * seed's members are listed in priority order (mem), staged through LDS and
 * summed by one thread in that order — gm_reduce.cpp:105-121's float
 * expression order, so equal inputs give the oracle's bits. */
__global__ void __launch_bounds__(EAP_NT)
    k_eap_merge(const float* __restrict__ comp, long K, const unsigned int* __restrict__ ord,
                const int* __restrict__ gstart, const unsigned int* __restrict__ rank, float T,
                unsigned char* __restrict__ flag, unsigned int* __restrict__ mem, float* __restrict__ out,
                unsigned int* __restrict__ out_rank, int* __restrict__ nout) {
    __shared__ int s_w[EAP_NT / 64];
    __shared__ float s_m[7][EAP_CHUNK];
    __shared__ float s_acc[8];
    const int g = blockIdx.x;
    const int gs = gstart[g], ge = gstart[g + 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int j = gs + tid; j < ge; j += EAP_NT) flag[j] = 0;
    __syncthreads();
    unsigned int* mlist = mem + gs;  // member positions of the current seed (group-private scratch)
    int p = gs;
    while (p < ge) {
        // the seed: first unmerged position >= p
        int s = ge;
        for (int base = p; base < ge && s == ge; base += EAP_NT) {
            const int j = base + tid;
            s = eap_block_min((j < ge && flag[j] == 0) ? j : ge, s_w);
        }
        if (s >= ge) break;
        const unsigned int si = ord[s];
        const float sw = comp[0 * K + si], sx = comp[1 * K + si], sy = comp[2 * K + si];
        const float sa = comp[3 * K + si], sb = comp[4 * K + si], sc = comp[5 * K + si], sd = comp[6 * K + si];
        // absorb every unmerged later member within T, listed in priority order
        int nm = 0;
        for (int base = s + 1; base < ge; base += EAP_NT) {
            const int j = base + tid;
            bool in = false;
            if (j < ge && flag[j] == 0) {
                const unsigned int bi = ord[j];
                const float d = eap_dist(sx, sy, sa, sb, sd, comp[1 * K + bi], comp[2 * K + bi], comp[3 * K + bi],
                                         comp[4 * K + bi], comp[6 * K + bi]);
                in = d < T;
            }
            const unsigned long long b = __ballot(in);
            if (lane == 0) s_w[wid] = __popcll(b);
            __syncthreads();
            int pre = nm, tot = 0;
#pragma unroll
            for (int w = 0; w < EAP_NT / 64; w++) {
                if (w < wid) pre += s_w[w];
                tot += s_w[w];
            }
            if (in) {
                flag[j] = 1;
                mlist[pre + __popcll(b & ((1ull << lane) - 1ull))] = (unsigned int)j;
            }
            nm += tot;
            __syncthreads();
        }
        // merged moments: pass 0 weight and mean sums, pass 1 covariance sums
        if (tid == 0) {
            s_acc[0] = sw;
            s_acc[1] = sx * sw;
            s_acc[2] = sy * sw;
        }
        for (int pass = 0; pass < 2; pass++) {
            if (pass == 1 && tid == 0) {
                const float W = s_acc[0];
                const float m0 = s_acc[1] / W, m1 = s_acc[2] / W;
                const float e0 = m0 - sx, e1 = m1 - sy;
                s_acc[1] = m0;
                s_acc[2] = m1;
                s_acc[3] = sw * (sa + e0 * e0);
                s_acc[4] = sw * (sb + e1 * e0);
                s_acc[5] = sw * (sc + e0 * e1);
                s_acc[6] = sw * (sd + e1 * e1);
            }
            for (int c0 = 0; c0 < nm; c0 += EAP_CHUNK) {
                const int cn = min(EAP_CHUNK, nm - c0);
                __syncthreads();
                for (int k = tid; k < cn; k += EAP_NT) {
                    const unsigned int bi = ord[mlist[c0 + k]];
#pragma unroll
                    for (int f = 0; f < 7; f++) s_m[f][k] = comp[(size_t)f * K + bi];
                }
                __syncthreads();
                if (tid == 0) {
                    if (pass == 0) {
                        float W = s_acc[0], m0 = s_acc[1], m1 = s_acc[2];
                        for (int k = 0; k < cn; k++) {
                            const float bw = s_m[0][k];
                            m0 += bw * s_m[1][k];
                            m1 += bw * s_m[2][k];
                            W += bw;
                        }
                        s_acc[0] = W;
                        s_acc[1] = m0;
                        s_acc[2] = m1;
                    } else {
                        const float m0 = s_acc[1], m1 = s_acc[2];
                        float c0v = s_acc[3], c1v = s_acc[4], c2v = s_acc[5], c3v = s_acc[6];
                        for (int k = 0; k < cn; k++) {
                            const float bw = s_m[0][k];
                            const float f0 = m0 - s_m[1][k], f1 = m1 - s_m[2][k];
                            c0v += bw * (s_m[3][k] + f0 * f0);
                            c1v += bw * (s_m[4][k] + f1 * f0);
                            c2v += bw * (s_m[5][k] + f0 * f1);
                            c3v += bw * (s_m[6][k] + f1 * f1);
                        }
                        s_acc[3] = c0v;
                        s_acc[4] = c1v;
                        s_acc[5] = c2v;
                        s_acc[6] = c3v;
                    }
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            // (pass 1's prologue ran for every seed: s_acc holds W, mean, Σ w (P + d dᵀ))
            const float W = s_acc[0], m0 = s_acc[1], m1 = s_acc[2];
            const int slot = atomicAdd(nout, 1);
            float* o = out + (size_t)slot * 7;
            o[0] = W;
            o[1] = m0;
            o[2] = m1;
            o[3] = s_acc[3] / W;
            o[4] = s_acc[4] / W;
            o[5] = s_acc[5] / W;
            o[6] = s_acc[6] / W;
            out_rank[slot] = rank[si];
            flag[s] = 1;
        }
        __syncthreads();
        p = s + 1;
    }
}

/* cell key of the component at priority position j (k_eap_cellkey's key) */
__global__ void k_eap_poskey(const float* __restrict__ comp, long K, const unsigned int* __restrict__ ord, float invR,
                             unsigned long long* __restrict__ key, unsigned int* __restrict__ pos) {
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const unsigned int i = ord[j];
    const float x = comp[1 * K + i], y = comp[2 * K + i];
    const double fx = floor((double)x * invR), fy = floor((double)y * invR);
    const long long cx = (long long)fmin(fmax(fx, -2147483000.0), 2147483000.0);
    const long long cy = (long long)fmin(fmax(fy, -2147483000.0), 2147483000.0);
    key[j] = ((unsigned long long)(cx + 2147483648LL) << 32) | (unsigned long long)(cy + 2147483648LL);
    pos[j] = (unsigned int)j;
}

/* nb9[9 c + r] = the occupied cell at offset (r / 3 - 1, r % 3 - 1) of
 * occupied cell c (binary search of the sorted unique keys), or -1 */
__global__ void k_eap_nb9(const unsigned long long* __restrict__ cells, int ncell, int* __restrict__ nb9) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncell) return;
    const unsigned long long k0 = cells[c];
    const long long cx = (long long)(k0 >> 32), cy = (long long)(k0 & 0xffffffffull);
    for (int r = 0; r < 9; r++) {
        const long long x = cx + (r / 3 - 1), y = cy + (r % 3 - 1);
        const unsigned long long k = ((unsigned long long)x << 32) | (unsigned long long)y;
        int lo = 0, hi = ncell;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cells[mid] < k) lo = mid + 1;
            else hi = mid;
        }
        nb9[(size_t)c * 9 + r] = (lo < ncell && cells[lo] == k) ? lo : -1;
    }
}

/* Records in cell order t (pos_by_cell order): rec0 = (x, y, λmax, position
 * bits), rec1 = (c00, c10, c11, 0) — what the decision rounds read. */
__global__ void k_eap_cellrec(const float* __restrict__ comp, long K, const unsigned int* __restrict__ ord,
                              const unsigned int* __restrict__ pos_by_cell, float4* __restrict__ rec0,
                              float4* __restrict__ rec1) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= K) return;
    const unsigned int p = pos_by_cell[t];
    const unsigned int i = ord[p];
    const float a = comp[3 * K + i], b = comp[4 * K + i], d = comp[6 * K + i];
    const double h = 0.5 * ((double)a + (double)d), q = 0.5 * ((double)a - (double)d);
    const float lm = (float)(h + sqrt(q * q + (double)b * (double)b)) * 1.0000002f;
    rec0[t] = make_float4(comp[1 * K + i], comp[2 * K + i], lm, __uint_as_float(p));
    rec1[t] = make_float4(a, b, d, 0.f);
}

#define EAP3_NT 256

/* One synchronous decision round (step 4) for one chunk of one occupied cell
 * (work item = cell, first cell-order index, count).  state[t] (cell order):
 * -1 undecided, -2 seed, else the absorbing seed's position.  Every thread
 * owns one position j of the chunk and looks for its decider among the
 * higher-priority positions of the 3 x 3 cells (own cell first), which the
 * workgroup streams through LDS in tiles of ascending position — a tile is
 * read by all lanes at once (broadcast), and the stream stops at the first
 * tile no undecided thread still needs.  A pair passes the isotropic bound
 * |Δμ|² <= 1.05 T (λk + λj) / 2 (d >= 2|Δμ|²/(λk + λj), the lattice's
 * margin) before the exact distance.  Counts the positions still waiting. */
__global__ void __launch_bounds__(EAP3_NT)
    k_eap_lfmis(const int4* __restrict__ work, const float4* __restrict__ rec0, const float4* __restrict__ rec1,
                const int* __restrict__ nb9, const int* __restrict__ run, float T, int* state,
                int* __restrict__ pending) {
    __shared__ float4 s_r0[EAP3_NT], s_r1[EAP3_NT];
    __shared__ int s_st[EAP3_NT];
    __shared__ int s_w[EAP3_NT / 64], s_c[EAP3_NT / 64];
    const int4 wk = work[blockIdx.x];
    const int c = wk.x, t = wk.y + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const bool own = (int)threadIdx.x < wk.z;
    const bool undecided = own && __hip_atomic_load(state + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1;
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
    if (undecided) {
        r0 = rec0[t];
        r1 = rec1[t];
    }
    const int pj = __float_as_int(r0.w);
    int best = undecided ? pj : -1;  // the deciding position so far (pj: none); -1: nothing to find
    int bst = 0;
    const float thr = 1.05f * T * 0.5f;
    for (int rr = 0; rr < 9; rr++) {
        const int r = rr == 0 ? 4 : (rr <= 4 ? rr - 1 : rr);  // own cell first: its decider is usually there
        const int cc = nb9[(size_t)c * 9 + r];
        if (cc < 0) continue;
        const int e1 = run[cc + 1];
        for (int base = run[cc]; base < e1; base += EAP3_NT) {
            // the largest position any thread still accepts (block max; its barrier
            // also retires the previous tile)
            int v = best;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
            if (lane == 0) s_w[wid] = v;
            __syncthreads();
            int need = s_w[0];
#pragma unroll
            for (int w = 1; w < EAP3_NT / 64; w++) need = max(need, s_w[w]);
            const int tn = min(EAP3_NT, e1 - base);
            const int lead = __float_as_int(rec0[base].w);
            if (lead >= need) break;  // ascending positions: no later tile of this cell is needed either
            // the tile's entries that can decide anyone: not absorbed, below `need`
            // (compacted in position order, so the scans skip the absorbed mass)
            float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f);
            int sq = 0;
            bool keep = false;
            if ((int)threadIdx.x < tn) {
                q0 = rec0[base + threadIdx.x];
                sq = __hip_atomic_load(state + base + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                keep = sq < 0 && __float_as_int(q0.w) < need;
            }
            const unsigned long long kb = __ballot(keep);
            if (lane == 0) s_c[wid] = (int)__popcll(kb);
            __syncthreads();
            int off = 0, nk = 0;
#pragma unroll
            for (int w = 0; w < EAP3_NT / 64; w++) {
                off += w < wid ? s_c[w] : 0;
                nk += s_c[w];
            }
            if (keep) {
                off += (int)__popcll(kb & ((1ull << lane) - 1ull));
                s_r0[off] = q0;
                s_r1[off] = rec1[base + threadIdx.x];
                s_st[off] = sq;
            }
            __syncthreads();
            for (int e = 0; e < nk && best >= 0; e++) {
                const float4 e0 = s_r0[e];
                const int k = __float_as_int(e0.w);
                if (k >= best) break;
                const float dx = e0.x - r0.x, dy = e0.y - r0.y;
                if (dx * dx + dy * dy > thr * (e0.z + r0.z)) continue;
                const float4 e1v = s_r1[e];
                if (eap_dist(e0.x, e0.y, e1v.x, e1v.y, e1v.z, r0.x, r0.y, r1.x, r1.y, r1.z) < T) {
                    best = k;
                    bst = s_st[e];
                    break;
                }
            }
        }
        __syncthreads();  // (the tile arrays and s_w are rewritten next)
    }
    bool wait = false;
    if (undecided) {
        if (best == pj || bst == -2) {
            __hip_atomic_store(state + t, best == pj ? -2 : best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            wait = true;  // the first candidate seed is still undecided
        }
    }
    const unsigned long long b = __ballot(wait);
    if (lane == 0 && b != 0ull) atomicAdd(pending, (int)__popcll(b));
}

/* state by position (from cell order) */
__global__ void k_eap_state_pos(const int* __restrict__ state_t, const unsigned int* __restrict__ pos_by_cell, long K,
                                int* __restrict__ state) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < K) state[pos_by_cell[t]] = state_t[t];
}

/* seed flag and the sort key of every position (its seed's position) */
__global__ void k_eap_seedkey(const int* __restrict__ state, long K, int* __restrict__ flag,
                              unsigned int* __restrict__ key) {
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    const int st = state[j];
    flag[j] = st == -2 ? 1 : 0;
    key[j] = (unsigned int)(st == -2 ? j : st);
}

/* gstart[slot of seed] = first index of its group in the seed-sorted positions */
__global__ void k_eap_gstart(const unsigned int* __restrict__ key_sorted, const int* __restrict__ slot, long K,
                             int nseed, int* __restrict__ gstart) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) gstart[nseed] = (int)K;
    if (t >= K) return;
    if (t == 0 || key_sorted[t] != key_sorted[t - 1]) gstart[slot[key_sorted[t]]] = (int)t;
}

/* Merged moments of seed g (one wave per seed): members mem[gstart[g] ..
 * gstart[g+1]) in priority order, the seed first; the wave stages 64 members
 * at a time in LDS and lane 0 sums them serially in gm_reduce.cpp:103-123's
 * expression order (the same arithmetic as k_eap_merge). */
#define EAP_SUM_NT 256
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__global__ void __launch_bounds__(EAP_SUM_NT)
    k_eap_sum(const float* __restrict__ comp, long K, const unsigned int* __restrict__ ord,
              const unsigned int* __restrict__ mem, const int* __restrict__ gstart, int nseed,
              float* __restrict__ out, unsigned int* __restrict__ out_rank) {
    __shared__ float s_m[EAP_SUM_NT / 64][7][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * (EAP_SUM_NT / 64) + wid;
    if (g >= nseed) return;  // (wave-private LDS: no workgroup barrier below)
    float(*sm)[64] = s_m[wid];
    const int a = gstart[g], b = gstart[g + 1];
    const unsigned int s = mem[a];
    const unsigned int si = ord[s];
    const float sw = comp[0 * K + si], sx = comp[1 * K + si], sy = comp[2 * K + si];
    const float sa = comp[3 * K + si], sb = comp[4 * K + si], sc = comp[5 * K + si], sd = comp[6 * K + si];
    float W = sw, m0 = sx * sw, m1 = sy * sw;
    float c0v = 0.f, c1v = 0.f, c2v = 0.f, c3v = 0.f;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            m0 = m0 / W;
            m1 = m1 / W;
            const float e0 = m0 - sx, e1 = m1 - sy;
            c0v = sw * (sa + e0 * e0);
            c1v = sw * (sb + e1 * e0);
            c2v = sw * (sc + e0 * e1);
            c3v = sw * (sd + e1 * e1);
        }
        for (int c0 = a + 1; c0 < b; c0 += 64) {
            const int cn = min(64, b - c0);
            if (lane < cn) {
                const unsigned int bi = ord[mem[c0 + lane]];
                sm[0][lane] = comp[0 * K + bi];
                sm[1][lane] = comp[1 * K + bi];
                sm[2][lane] = comp[2 * K + bi];
                if (pass == 1) {
                    sm[3][lane] = comp[3 * K + bi];
                    sm[4][lane] = comp[4 * K + bi];
                    sm[5][lane] = comp[5 * K + bi];
                    sm[6][lane] = comp[6 * K + bi];
                }
            }
            wave_lds_sync();
            if (lane == 0) {
                if (pass == 0) {
                    for (int k = 0; k < cn; k++) {
                        const float bw = sm[0][k];
                        m0 += bw * sm[1][k];
                        m1 += bw * sm[2][k];
                        W += bw;
                    }
                } else {
                    for (int k = 0; k < cn; k++) {
                        const float bw = sm[0][k];
                        const float f0 = m0 - sm[1][k], f1 = m1 - sm[2][k];
                        c0v += bw * (sm[3][k] + f0 * f0);
                        c1v += bw * (sm[4][k] + f1 * f0);
                        c2v += bw * (sm[5][k] + f0 * f1);
                        c3v += bw * (sm[6][k] + f1 * f1);
                    }
                }
            }
            wave_lds_sync();  // (the chunk is rewritten next)
        }
    }
    if (lane == 0) {
        float* o = out + (size_t)g * 7;
        o[0] = W;
        o[1] = m0;
        o[2] = m1;
        o[3] = c0v / W;
        o[4] = c1v / W;
        o[5] = c2v / W;
        o[6] = c3v / W;
        out_rank[g] = s;
    }
}

/* final gather into the emission order */
__global__ void k_eap_emit(const float* __restrict__ out, const unsigned int* __restrict__ slot_by_rank, int nout,
                           phd_gaussian2d* __restrict__ dst) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nout) return;
    const float* o = out + (size_t)slot_by_rank[k] * 7;
    phd_gaussian2d g;
    g.weight = o[0];
    g.mean[0] = o[1];
    g.mean[1] = o[2];
    g.cov[0] = o[3];
    g.cov[1] = o[4];
    g.cov[2] = o[5];
    g.cov[3] = o[6];
    dst[k] = g;
}

/* ------------------------------------------------------------------ host */

struct EapScratch {
    void* buf = nullptr;
    size_t bytes = 0;
    int* pinned = nullptr;  // read-back slots of the decision rounds
    ~EapScratch() {
        if (buf) hipFree(buf);
        if (pinned) hipHostFree(pinned);
    }
};

void eap_free(EapScratch* s) { delete s; }

#define EAPCHK(expr)                                \
    do {                                            \
        hipError_t _e = (expr);                     \
        if (_e != hipSuccess) {                     \
            err = hipGetErrorString(_e);            \
            return -1;                              \
        }                                           \
    } while (0)

namespace {
struct Carve {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T* p = (T*)(base ? base + off : nullptr);
        off += count * sizeof(T);
        return p;
    }
};

}  // namespace

struct EapBufs {
    float* comp;                 // 7 x K SoA weighted components
    unsigned int* misc;          // [0] Λ bits [1] non-finite [2] run count [3] output count
    unsigned long long *key, *key2;
    unsigned int *i0, *i1, *gid, *rank, *gkey, *gkey2, *mem, *orank, *orank2, *oslot, *oslot2;
    unsigned char* flag;
    int *runs, *off;
    int* nb9;                    // 9 x K neighbour cells of every occupied cell
    float4 *rec0, *rec1;         // records in cell order (decision rounds)
    int4* work;                  // decision rounds' work items
    float* out;                  // 7 x K merged components (slot order)
    phd_gaussian2d* g;           // emission order
    void* tmp;                   // hipcub temporary storage
};

static size_t eap_carve(char* base, long K, int n, size_t tmp, EapBufs* b) {
    Carve c{base};
    EapBufs t;
    t.off = c.take<int>(n + 1);
    t.comp = c.take<float>(7 * (size_t)K);
    t.misc = c.take<unsigned int>(8);
    t.key = c.take<unsigned long long>(K);
    t.key2 = c.take<unsigned long long>(K);
    t.i0 = c.take<unsigned int>(K);
    t.i1 = c.take<unsigned int>(K);
    t.gid = c.take<unsigned int>(K);
    t.rank = c.take<unsigned int>(K);
    t.gkey = c.take<unsigned int>(K);
    t.gkey2 = c.take<unsigned int>(K + 1);
    t.mem = c.take<unsigned int>(K);
    t.orank = c.take<unsigned int>(K);
    t.orank2 = c.take<unsigned int>(K);
    t.oslot = c.take<unsigned int>(K);
    t.oslot2 = c.take<unsigned int>(K);
    t.flag = c.take<unsigned char>(K);
    t.runs = c.take<int>(K + 1);
    t.nb9 = c.take<int>(9 * (size_t)K);
    t.rec0 = c.take<float4>(K);
    t.rec1 = c.take<float4>(K);
    t.work = c.take<int4>((size_t)K + (size_t)K / EAP3_NT + 2);
    t.out = c.take<float>(7 * (size_t)K);
    t.g = c.take<phd_gaussian2d>(K);
    t.tmp = (void*)c.take<char>(tmp);
    if (b) *b = t;
    return c.off + 256;
}

static int bits_for(unsigned int v) {  // radix bits covering 0..v
    int b = 1;
    while (b < 32 && (v >> b) != 0) b++;
    return b;
}

/* Expected map of the current store into host `out` (out_cap entries).
 * Returns the component count (also when it exceeds out_cap: nothing is then
 * copied), or -1 on a HIP error (err).  *n_groups = independent groups. */
long eap_run(EapScratch** sp, hipStream_t st, const int* d_src, const float* d_map, const int* d_size,
             const float* d_map_x, const int* d_size_x, const float* d_logw, int n, int cap, float T,
             phd_gaussian2d* out, long out_cap, int* n_groups, std::string& err) {
    if (!*sp) *sp = new EapScratch();
    EapScratch& S = **sp;
    auto ensure = [&](size_t need) -> int {
        if (S.bytes >= need) return 0;
        if (S.buf) hipFree(S.buf);
        S.buf = nullptr;
        S.bytes = 0;
        if (hipMalloc(&S.buf, need) != hipSuccess) return -1;
        S.bytes = need;
        return 0;
    };
    if (n_groups) *n_groups = 0;
    // component counts -> offsets (one read-back of n ints)
    if (ensure((size_t)(n + 1) * sizeof(int))) {
        err = "expected map: out of device memory";
        return -1;
    }
    hipLaunchKernelGGL(k_eap_sizes, dim3((n + 255) / 256), dim3(256), 0, st, d_src, d_size, d_size_x, n, (int*)S.buf);
    std::vector<int> off(n + 1, 0);
    EAPCHK(hipMemcpyAsync(off.data() + 1, S.buf, n * sizeof(int), hipMemcpyDeviceToHost, st));
    EAPCHK(hipStreamSynchronize(st));
    long Kl = 0;
    for (int p = 0; p < n; p++) {
        Kl += off[p + 1];
        off[p + 1] = (int)Kl;
    }
    if (Kl == 0) return 0;
    if (Kl >= (1L << 31) - 1) {
        err = "expected map: more than 2^31 components";
        return -1;
    }
    const long K = Kl;
    const int Ki = (int)K;
    size_t tmp = 0, t2 = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, t2, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                       (unsigned int*)nullptr, (unsigned int*)nullptr, Ki, 0, 64, st);
    tmp = std::max(tmp, t2);
    hipcub::DeviceRadixSort::SortPairsDescending(nullptr, t2, (float*)nullptr, (float*)nullptr, (unsigned int*)nullptr,
                                                 (unsigned int*)nullptr, Ki, 0, 32, st);
    tmp = std::max(tmp, t2);
    hipcub::DeviceRadixSort::SortPairs(nullptr, t2, (unsigned int*)nullptr, (unsigned int*)nullptr,
                                       (unsigned int*)nullptr, (unsigned int*)nullptr, Ki, 0, 32, st);
    tmp = std::max(tmp, t2);
    hipcub::DeviceRunLengthEncode::Encode(nullptr, t2, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                          (int*)nullptr, (int*)nullptr, Ki, st);
    tmp = std::max(tmp, t2);
    hipcub::DeviceScan::InclusiveSum(nullptr, t2, (int*)nullptr, (int*)nullptr, Ki, st);
    tmp = std::max(tmp, t2);
    hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (int*)nullptr, (int*)nullptr, Ki, st);
    tmp = std::max(tmp, t2);
    if (ensure(eap_carve(nullptr, K, n, tmp, nullptr))) {
        err = "expected map: out of device memory";
        return -1;
    }
    EapBufs B;
    eap_carve((char*)S.buf, K, n, tmp, &B);
    size_t tb;
    EAPCHK(hipMemcpyAsync(B.off, off.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice, st));
    EAPCHK(hipMemsetAsync(B.misc, 0, 8 * sizeof(unsigned int), st));
    hipLaunchKernelGGL(k_eap_gather, dim3(n), dim3(256), 0, st, d_src, d_map, d_map_x, B.off, d_logw, cap, K, B.comp,
                       B.misc, (int*)B.misc + 1);
    unsigned int misc[2];
    EAPCHK(hipMemcpyAsync(misc, B.misc, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost, st));
    EAPCHK(hipStreamSynchronize(st));
    float lam;
    memcpy(&lam, &misc[0], 4);
    const bool one_group = misc[1] != 0 || !(lam > 0.f) || !(lam < INFINITY) || !(T > 0.f) || !(T < INFINITY);
    const unsigned int nb = (unsigned int)((K + 255) / 256);
    // priority: weight descending, concatenation index ascending (stable sort of the identity)
    hipLaunchKernelGGL(k_iota_u32, dim3(nb), dim3(256), 0, st, B.i0, K);
    tb = tmp;
    EAPCHK(hipcub::DeviceRadixSort::SortPairsDescending(B.tmp, tb, B.comp, (float*)B.key2, B.i0, B.i1, Ki, 0, 32, st));
    const unsigned int* ord = B.i1;  // component at priority position j
    int nout = 0, rounds = 1;
    if (one_group) {
        const int gs[2] = {0, Ki};
        EAPCHK(hipMemsetAsync(B.gid, 0, K * sizeof(unsigned int), st));
        hipLaunchKernelGGL(k_eap_rank, dim3(nb), dim3(256), 0, st, ord, B.gid, K, B.rank, B.gkey);
        EAPCHK(hipMemcpyAsync(B.runs, gs, 2 * sizeof(int), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_eap_merge, dim3(1), dim3(EAP_NT), 0, st, B.comp, K, ord, B.runs, B.rank, T, B.flag,
                           B.mem, B.out, B.orank, (int*)B.misc + 3);
        EAPCHK(hipGetLastError());
        EAPCHK(hipMemcpyAsync(&nout, (int*)B.misc + 3, sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
    } else {
        // lattice cells of side R; d < T  =>  |Δμ|² < T Λ (5 % margin for float rounding)
        const double R = std::sqrt(1.05 * (double)T * (double)lam) * 1.0001;
        const float invR = (float)(1.0 / R);
        unsigned long long* keyp = B.key;   // cell key by position, then the unique occupied cells
        unsigned long long* keys = B.key2;  // cell keys sorted
        unsigned int* pos_by_cell = B.mem;  // positions grouped by cell, ascending within a cell
        int* counts = (int*)B.gkey;
        int* run = (int*)B.gkey2;            // run[c] .. run[c + 1]: cell c's slice of pos_by_cell
        int* state = (int*)B.gid;    // by position
        int* state_t = (int*)B.rank;  // by cell order (the rounds)
        hipLaunchKernelGGL(k_eap_poskey, dim3(nb), dim3(256), 0, st, B.comp, K, ord, invR, keyp, B.i0);
        tb = tmp;
        EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, keyp, keys, B.i0, pos_by_cell, Ki, 0, 64, st));
        tb = tmp;
        EAPCHK(hipcub::DeviceRunLengthEncode::Encode(B.tmp, tb, keys, keyp, counts, (int*)B.misc + 4, Ki, st));
        int ncell = 0;
        EAPCHK(hipMemcpyAsync(&ncell, (int*)B.misc + 4, sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
        // cell runs and the rounds' work items (cell, first index, count): chunks of EAP3_NT
        std::vector<int> cnt(ncell), runh(ncell + 1, 0);
        EAPCHK(hipMemcpyAsync(cnt.data(), counts, ncell * sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
        std::vector<int4> work;
        work.reserve((size_t)ncell + (size_t)(K / EAP3_NT) + 1);
        for (int c = 0; c < ncell; c++) {
            runh[c + 1] = runh[c] + cnt[c];
            for (int q = 0; q < cnt[c]; q += EAP3_NT) work.push_back(make_int4(c, runh[c] + q, std::min(EAP3_NT, cnt[c] - q), 0));
        }
        EAPCHK(hipMemcpyAsync(run, runh.data(), (ncell + 1) * sizeof(int), hipMemcpyHostToDevice, st));
        EAPCHK(hipMemcpyAsync(B.work, work.data(), work.size() * sizeof(int4), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_eap_nb9, dim3((ncell + 255) / 256), dim3(256), 0, st, keyp, ncell, B.nb9);
        hipLaunchKernelGGL(k_eap_cellrec, dim3(nb), dim3(256), 0, st, B.comp, K, ord, pos_by_cell, B.rec0, B.rec1);
        EAPCHK(hipMemsetAsync(state_t, 0xff, K * sizeof(int), st));  // -1: undecided
        // step 4: decision rounds until no position waits (each round decides at
        // least the highest-priority undecided position)
#ifdef PHD_EAP_DEBUG
        constexpr bool dbg = true;  // diagnostic build: per-round timing on stderr
#else
        constexpr bool dbg = false;
#endif
        std::chrono::steady_clock::time_point t_r0 = std::chrono::steady_clock::now();
        if (dbg) fprintf(stderr, "[eap] K %ld ncell %d R %g work %zu\n", K, ncell, R, work.size());
        if (!S.pinned) EAPCHK(hipHostMalloc((void**)&S.pinned, 64, hipHostMallocDefault));
        hipEvent_t ev0 = nullptr, ev1 = nullptr;
        if (dbg) {
            EAPCHK(hipEventCreate(&ev0));
            EAPCHK(hipEventCreate(&ev1));
        }
        for (rounds = 1;; rounds++) {
            EAPCHK(hipMemsetAsync((int*)B.misc + 5, 0, sizeof(int), st));
            if (dbg) EAPCHK(hipEventRecord(ev0, st));
            hipLaunchKernelGGL(k_eap_lfmis, dim3((unsigned)work.size()), dim3(EAP3_NT), 0, st, B.work, B.rec0, B.rec1,
                               B.nb9, run, T, state_t, (int*)B.misc + 5);
            if (dbg) EAPCHK(hipEventRecord(ev1, st));
            EAPCHK(hipMemcpyAsync(S.pinned, (int*)B.misc + 5, sizeof(int), hipMemcpyDeviceToHost, st));
            EAPCHK(hipStreamSynchronize(st));
            const int waiting = S.pinned[0];
            if (dbg) {
                const auto t_r1 = std::chrono::steady_clock::now();
                float kms = 0.f;
                EAPCHK(hipEventElapsedTime(&kms, ev0, ev1));
                fprintf(stderr, "[eap] round %d: %d waiting, %.2f ms (kernel %.2f ms)\n", rounds, waiting,
                        std::chrono::duration<double, std::milli>(t_r1 - t_r0).count(), kms);
                t_r0 = t_r1;
            }
            if (waiting == 0) break;
            if (rounds > Ki) {
                err = "decision rounds did not converge";
                return -1;
            }
        }
        if (ev0) hipEventDestroy(ev0);
        if (ev1) hipEventDestroy(ev1);
        hipLaunchKernelGGL(k_eap_state_pos, dim3(nb), dim3(256), 0, st, state_t, pos_by_cell, K, state);
        // step 5: seeds' slots (priority order), members grouped by seed
        int* flag = counts;                          // (the cell counts are dead)
        unsigned int* skey = (unsigned int*)B.key;   // seed position of every position (the cells are dead)
        int* slot = (int*)B.key + K;                 // seed slot = seeds before it
        unsigned int* skey2 = (unsigned int*)B.key2;
        unsigned int* mem = pos_by_cell;             // positions grouped by seed, ascending within a group
        hipLaunchKernelGGL(k_eap_seedkey, dim3(nb), dim3(256), 0, st, state, K, flag, skey);
        tb = tmp;
        EAPCHK(hipcub::DeviceScan::ExclusiveSum(B.tmp, tb, flag, slot, Ki, st));
        int last[2] = {0, 0};
        EAPCHK(hipMemcpyAsync(&last[0], slot + (K - 1), sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipMemcpyAsync(&last[1], flag + (K - 1), sizeof(int), hipMemcpyDeviceToHost, st));
        hipLaunchKernelGGL(k_iota_u32, dim3(nb), dim3(256), 0, st, B.i0, K);
        tb = tmp;
        EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, skey, skey2, B.i0, mem, Ki, 0,
                                                  bits_for((unsigned int)(K - 1)), st));
        EAPCHK(hipStreamSynchronize(st));
        nout = last[0] + last[1];
        hipLaunchKernelGGL(k_eap_gstart, dim3(nb), dim3(256), 0, st, skey2, slot, K, nout, B.runs);
        hipLaunchKernelGGL(k_eap_sum, dim3((nout + EAP_SUM_NT / 64 - 1) / (EAP_SUM_NT / 64)), dim3(EAP_SUM_NT), 0, st,
                           B.comp, K, ord, mem, B.runs, nout, B.out, B.orank);
        EAPCHK(hipGetLastError());
        if (dbg) {
            EAPCHK(hipStreamSynchronize(st));
            fprintf(stderr, "[eap] %d seeds, grouping + sums %.2f ms\n", nout,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_r0).count());
        }
    }
    if (n_groups) *n_groups = rounds;
    if (nout > out_cap || !out) return nout;
    // emission order = seed priority (the reference's selection order)
    hipLaunchKernelGGL(k_iota_u32, dim3((nout + 255) / 256), dim3(256), 0, st, B.oslot, (long)nout);
    tb = tmp;
    EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, B.orank, B.orank2, B.oslot, B.oslot2, nout, 0,
                                              bits_for((unsigned int)(K - 1)), st));
    hipLaunchKernelGGL(k_eap_emit, dim3((nout + 255) / 256), dim3(256), 0, st, B.out, B.oslot2, nout, B.g);
    EAPCHK(hipMemcpyAsync(out, B.g, (size_t)nout * sizeof(phd_gaussian2d), hipMemcpyDeviceToHost, st));
    EAPCHK(hipStreamSynchronize(st));
    return nout;
}

}  // namespace phd
