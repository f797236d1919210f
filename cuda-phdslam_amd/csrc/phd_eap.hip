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
 *   3. radix-sort by cell, run-length-encode the occupied cells, and split
 *      them into groups = connected components of touching occupied cells
 *      (host union-find over the cell list: a few thousand entries);
 *   4. within each group, order by the global priority (weight descending,
 *      concatenation index ascending: two stable radix sorts);
 *   5. one workgroup per group runs the greedy on its members — the greedy
 *      over a disjoint union of independent sets is the union of the
 *      per-set greedies — seeds in priority order, distance tests in
 *      parallel, the merged moments summed serially in priority order with
 *      the reference's float expression order (bit-identical to the oracle
 *      for identical weights);
 *   6. outputs sorted by their seed's global priority = the reference's
 *      emission order.
 * Non-finite means or a non-finite Λ fall back to one group (still exact).
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <unordered_map>
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
 * (positive floats order as their bit patterns; a non-finite value sets bad). */
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
        const double lm = h + sqrt(q * q + (double)b * (double)b);
        if (!(fabs(x) < INFINITY && fabs(y) < INFINITY && fabs(lm) < INFINITY)) nonfinite = 1;
        else lmax = fmaxf(lmax, (float)lm * 1.0000002f);
    }
    if (nonfinite) atomicOr(bad, 1);
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o2, 64));
    if ((threadIdx.x & 63) == 0 && lmax > 0.f) atomicMax(lam_bits, __float_as_uint(lmax));
}

/* lattice cell key of every component (64 bit: cx | cy, biased) */
__global__ void k_eap_cellkey(const float* __restrict__ comp, long K, float invR, unsigned long long* __restrict__ key,
                              unsigned int* __restrict__ idx) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K) return;
    const float x = comp[1 * K + i], y = comp[2 * K + i];
    const double fx = floor((double)x * invR), fy = floor((double)y * invR);
    const long long cx = (long long)fmin(fmax(fx, -2147483000.0), 2147483000.0);
    const long long cy = (long long)fmin(fmax(fy, -2147483000.0), 2147483000.0);
    key[i] = ((unsigned long long)(cx + 2147483648LL) << 32) | (unsigned long long)(cy + 2147483648LL);
    idx[i] = (unsigned int)i;
}

__global__ void k_iota_u32(unsigned int* a, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (unsigned int)i;
}

/* group id of every component from its cell run (one block per run) */
__global__ void k_eap_run_gid(const unsigned int* __restrict__ idx_by_cell, const int* __restrict__ run_start,
                              const int* __restrict__ run_gid, unsigned int* __restrict__ gid) {
    const int r = blockIdx.x;
    const int a = run_start[r], b = run_start[r + 1], g = run_gid[r];
    for (int j = a + threadIdx.x; j < b; j += blockDim.x) gid[idx_by_cell[j]] = (unsigned int)g;
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

#define EAP2_NT 1024
#define EAP2_LIST 8192  /* absorbed members sorted in LDS up to this many per seed */

/* Greedy reduce of one group (block) with the distance tests restricted to the
 * seed's 3 x 3 lattice cells (a pair at distance < T lies in touching cells,
 * eap_run step 2): the occupied cells are the sorted unique keys `cells`
 * (nruns), the priority positions of cell r are pos_by_cell[run[r] .. run[r+1])
 * in ascending order.  For each seed (first unmerged position), the unmerged
 * later positions of its 9 cells are tested in parallel, the absorbed ones
 * marked (mark[j] = seed id) and listed; the list is sorted by position
 * (bitonic, in LDS) and one thread sums the moments in that order — the
 * reference's order, so the outputs equal k_eap_merge's (and the oracle's)
 * bit for bit.  More than EAP2_LIST absorbed members: thread 0 merges the 9
 * cell runs in position order instead. */
__global__ void __launch_bounds__(EAP2_NT)
    k_eap_merge_cells(const float* __restrict__ comp, long K, const unsigned int* __restrict__ ord,
                      const int* __restrict__ gstart, const unsigned int* __restrict__ rank,
                      const unsigned long long* __restrict__ cells, int nruns, const int* __restrict__ run,
                      const unsigned int* __restrict__ pos_by_cell, float invR, float T,
                      unsigned int* __restrict__ mark, float* __restrict__ out, unsigned int* __restrict__ out_rank,
                      int* __restrict__ nout) {
    __shared__ int s_w[EAP2_NT / 64];
    __shared__ unsigned int s_list[EAP2_LIST];
    __shared__ float s_m[7][EAP_CHUNK];
    __shared__ float s_acc[8];
    __shared__ int s_seg[10][2];  // the 9 cell runs of the seed: [start, end) in pos_by_cell
    __shared__ int s_nm;
    const int g = blockIdx.x;
    const int gs = gstart[g], ge = gstart[g + 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int j = gs + tid; j < ge; j += EAP2_NT) mark[j] = 0u;
    __syncthreads();
    int p = gs;
    unsigned int sid = 0;  // seed counter of this group (marks)
    while (p < ge) {
        // the seed: first unmarked position >= p
        int s = ge;
        for (int base = p; base < ge && s == ge; base += EAP2_NT) {
            const int j = base + tid;
            int v = (j < ge && mark[j] == 0u) ? j : ge;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
            if (lane == 0) s_w[wid] = v;
            __syncthreads();
            int r = s_w[0];
#pragma unroll
            for (int w = 1; w < EAP2_NT / 64; w++) r = min(r, s_w[w]);
            __syncthreads();
            s = r;
        }
        if (s >= ge) break;
        sid++;
        const unsigned int si = ord[s];
        const float sw = comp[0 * K + si], sx = comp[1 * K + si], sy = comp[2 * K + si];
        const float sa = comp[3 * K + si], sb = comp[4 * K + si], sc = comp[5 * K + si], sd = comp[6 * K + si];
        // the seed's 9 cells -> runs (binary search of the sorted occupied cells)
        if (tid < 9) {
            const double fx = floor((double)sx * invR), fy = floor((double)sy * invR);
            const long long cx = (long long)fmin(fmax(fx, -2147483000.0), 2147483000.0) + (tid / 3 - 1);
            const long long cy = (long long)fmin(fmax(fy, -2147483000.0), 2147483000.0) + (tid % 3 - 1);
            const unsigned long long k =
                ((unsigned long long)(cx + 2147483648LL) << 32) | (unsigned long long)(cy + 2147483648LL);
            int lo = 0, hi = nruns;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (cells[mid] < k) lo = mid + 1;
                else hi = mid;
            }
            const bool hit = lo < nruns && cells[lo] == k;
            s_seg[tid][0] = hit ? run[lo] : 0;
            s_seg[tid][1] = hit ? run[lo + 1] : 0;
        }
        if (tid == 0) {
            s_nm = 0;
            mark[s] = sid;
        }
        __syncthreads();
        int e[10];
        e[0] = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) e[k + 1] = e[k] + (s_seg[k][1] - s_seg[k][0]);
        // absorb the unmarked later positions of those cells within T
        for (int t = tid; t < e[9]; t += EAP2_NT) {
            int k = 0;
#pragma unroll
            for (int q = 1; q < 9; q++) k += t >= e[q] ? 1 : 0;
            const int j = (int)pos_by_cell[s_seg[k][0] + (t - e[k])];
            if (j <= s || mark[j] != 0u) continue;
            const unsigned int bi = ord[j];
            const float d = eap_dist(sx, sy, sa, sb, sd, comp[1 * K + bi], comp[2 * K + bi], comp[3 * K + bi],
                                     comp[4 * K + bi], comp[6 * K + bi]);
            if (d < T) {
                mark[j] = sid;
                const int q = atomicAdd(&s_nm, 1);
                if (q < EAP2_LIST) s_list[q] = (unsigned int)j;
            }
        }
        __syncthreads();
        const int nm = s_nm;
        const bool listed = nm <= EAP2_LIST;
        if (listed && nm > 1) {  // bitonic sort of the listed positions
            int n2 = 1;
            while (n2 < nm) n2 <<= 1;
            for (int q = nm + tid; q < n2; q += EAP2_NT) s_list[q] = 0xffffffffu;
            __syncthreads();
            for (int k = 2; k <= n2; k <<= 1)
                for (int jj = k >> 1; jj > 0; jj >>= 1) {
                    for (int i = tid; i < n2; i += EAP2_NT) {
                        const int ixj = i ^ jj;
                        if (ixj > i) {
                            const unsigned int x = s_list[i], y = s_list[ixj];
                            if ((x > y) == ((i & k) == 0)) {
                                s_list[i] = y;
                                s_list[ixj] = x;
                            }
                        }
                    }
                    __syncthreads();
                }
        }
        // merged moments (gm_reduce.cpp:103-123 order): pass 0 weight and mean,
        // pass 1 covariance; members staged through LDS in position order
        if (tid == 0) {
            s_acc[0] = sw;
            s_acc[1] = sx * sw;
            s_acc[2] = sy * sw;
        }
        if (!listed) {
            // more members than the list holds: thread 0 merges the 9 runs in position order
            if (tid == 0) {
                for (int pass = 0; pass < 2; pass++) {
                    float W = s_acc[0], m0 = s_acc[1], m1 = s_acc[2];
                    if (pass == 1) {
                        m0 /= W;
                        m1 /= W;
                        const float e0 = m0 - sx, e1 = m1 - sy;
                        s_acc[1] = m0;
                        s_acc[2] = m1;
                        s_acc[3] = sw * (sa + e0 * e0);
                        s_acc[4] = sw * (sb + e1 * e0);
                        s_acc[5] = sw * (sc + e0 * e1);
                        s_acc[6] = sw * (sd + e1 * e1);
                    }
                    float c0v = s_acc[3], c1v = s_acc[4], c2v = s_acc[5], c3v = s_acc[6];
                    int cur[9];
                    for (int k = 0; k < 9; k++) cur[k] = s_seg[k][0];
                    while (true) {
                        int best = -1;
                        unsigned int bj = 0xffffffffu;
                        for (int k = 0; k < 9; k++) {
                            while (cur[k] < s_seg[k][1] && mark[pos_by_cell[cur[k]]] != sid) cur[k]++;
                            if (cur[k] < s_seg[k][1] && pos_by_cell[cur[k]] < bj) {
                                bj = pos_by_cell[cur[k]];
                                best = k;
                            }
                        }
                        if (best < 0) break;
                        cur[best]++;
                        if ((int)bj == s) continue;
                        const unsigned int bi = ord[bj];
                        const float bw = comp[0 * K + bi], bx = comp[1 * K + bi], by = comp[2 * K + bi];
                        if (pass == 0) {
                            m0 += bw * bx;
                            m1 += bw * by;
                            W += bw;
                        } else {
                            const float f0 = s_acc[1] - bx, f1 = s_acc[2] - by;
                            c0v += bw * (comp[3 * K + bi] + f0 * f0);
                            c1v += bw * (comp[4 * K + bi] + f1 * f0);
                            c2v += bw * (comp[5 * K + bi] + f0 * f1);
                            c3v += bw * (comp[6 * K + bi] + f1 * f1);
                        }
                    }
                    if (pass == 0) {
                        s_acc[0] = W;
                        s_acc[1] = m0;
                        s_acc[2] = m1;
                    } else {
                        s_acc[3] = c0v;
                        s_acc[4] = c1v;
                        s_acc[5] = c2v;
                        s_acc[6] = c3v;
                    }
                }
            }
        } else {
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
                    for (int k = tid; k < cn; k += EAP2_NT) {
                        const unsigned int bi = ord[s_list[c0 + k]];
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
                if (pass == 0 && nm == 0) __syncthreads();
            }
        }
        __syncthreads();
        if (tid == 0) {
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
        }
        __syncthreads();
        p = s + 1;
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
    ~EapScratch() {
        if (buf) hipFree(buf);
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

int uf_find(std::vector<int>& par, int x) {
    while (par[x] != x) {
        par[x] = par[par[x]];
        x = par[x];
    }
    return x;
}
}  // namespace

struct EapBufs {
    float* comp;                 // 7 x K SoA weighted components
    unsigned int* misc;          // [0] Λ bits [1] non-finite [2] run count [3] output count
    unsigned long long *key, *key2;
    unsigned int *i0, *i1, *gid, *rank, *gkey, *gkey2, *mem, *orank, *orank2, *oslot, *oslot2;
    unsigned char* flag;
    int *runs, *off;
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
    std::vector<int> gsize;
    int G = 0;
    if (!one_group) {
        // lattice cells; d < T  =>  |Δμ|² < T Λ (5 % margin for float rounding)
        const double R = std::sqrt(1.05 * (double)T * (double)lam) * 1.0001;
        hipLaunchKernelGGL(k_eap_cellkey, dim3(nb), dim3(256), 0, st, B.comp, K, (float)(1.0 / R), B.key, B.i0);
        tb = tmp;
        EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, B.key, B.key2, B.i0, B.i1, Ki, 0, 64, st));
        tb = tmp;
        EAPCHK(hipcub::DeviceRunLengthEncode::Encode(B.tmp, tb, B.key2, B.key, B.runs, (int*)B.misc + 2, Ki, st));
        int nruns = 0;
        EAPCHK(hipMemcpyAsync(&nruns, (int*)B.misc + 2, sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
        std::vector<unsigned long long> cells(nruns);
        std::vector<int> cnt(nruns);
        EAPCHK(hipMemcpyAsync(cells.data(), B.key, nruns * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        EAPCHK(hipMemcpyAsync(cnt.data(), B.runs, nruns * sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
        // groups: connected components of touching occupied cells (union-find)
        std::unordered_map<unsigned long long, int> at;
        at.reserve((size_t)nruns * 2);
        for (int r = 0; r < nruns; r++) at.emplace(cells[r], r);
        std::vector<int> par(nruns);
        for (int r = 0; r < nruns; r++) par[r] = r;
        static const int fwd[4][2] = {{0, 1}, {1, -1}, {1, 0}, {1, 1}};  // each touching pair once
        for (int r = 0; r < nruns; r++) {
            const unsigned long long cx = cells[r] >> 32, cy = cells[r] & 0xffffffffull;
            for (const auto& d : fwd) {
                const unsigned long long nk = ((cx + (unsigned long long)(long long)d[0]) << 32) |
                                              ((cy + (unsigned long long)(long long)d[1]) & 0xffffffffull);
                auto it = at.find(nk);
                if (it == at.end()) continue;
                const int a = uf_find(par, r), b = uf_find(par, it->second);
                if (a != b) par[std::max(a, b)] = std::min(a, b);
            }
        }
        std::vector<int> run_gid(nruns), root_gid(nruns, -1), run_start(nruns + 1, 0);
        for (int r = 0; r < nruns; r++) {
            const int root = uf_find(par, r);
            if (root_gid[root] < 0) {
                root_gid[root] = G++;
                gsize.push_back(0);
            }
            run_gid[r] = root_gid[root];
            gsize[run_gid[r]] += cnt[r];
            run_start[r + 1] = run_start[r] + cnt[r];
        }
        EAPCHK(hipMemcpyAsync(B.runs, run_start.data(), (nruns + 1) * sizeof(int), hipMemcpyHostToDevice, st));
        EAPCHK(hipMemcpyAsync(B.gkey2, run_gid.data(), nruns * sizeof(int), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_eap_run_gid, dim3(nruns), dim3(256), 0, st, B.i1, B.runs, (const int*)B.gkey2, B.gid);
        EAPCHK(hipStreamSynchronize(st));  // host vectors above are released at scope exit
    } else {
        G = 1;
        gsize.assign(1, Ki);
        EAPCHK(hipMemsetAsync(B.gid, 0, K * sizeof(unsigned int), st));
    }
    // priority: weight descending, concatenation index ascending (stable sort of the identity)
    hipLaunchKernelGGL(k_iota_u32, dim3(nb), dim3(256), 0, st, B.i0, K);
    tb = tmp;
    EAPCHK(hipcub::DeviceRadixSort::SortPairsDescending(B.tmp, tb, B.comp, (float*)B.key2, B.i0, B.i1, Ki, 0, 32, st));
    hipLaunchKernelGGL(k_eap_rank, dim3(nb), dim3(256), 0, st, B.i1, B.gid, K, B.rank, B.gkey);
    tb = tmp;
    EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, B.gkey, B.gkey2, B.i1, B.i0, Ki, 0,
                                              bits_for((unsigned int)std::max(G - 1, 0)), st));
    std::vector<int> gstart(G + 1, 0);
    for (int g = 0; g < G; g++) gstart[g + 1] = gstart[g] + gsize[g];
    EAPCHK(hipMemcpyAsync(B.runs, gstart.data(), (G + 1) * sizeof(int), hipMemcpyHostToDevice, st));
    if (one_group) {
        hipLaunchKernelGGL(k_eap_merge, dim3(G), dim3(EAP_NT), 0, st, B.comp, K, B.i0, B.runs, B.rank, T, B.flag,
                           B.mem, B.out, B.orank, (int*)B.misc + 3);
    } else {
        // the distance tests of a seed only reach its 3 x 3 lattice cells: the
        // priority positions grouped by cell (ascending within a cell), the
        // occupied cells sorted, their run starts
        const double R = std::sqrt(1.05 * (double)T * (double)lam) * 1.0001;
        const float invR = (float)(1.0 / R);
        unsigned long long* keyp = B.key;
        unsigned long long* keys = B.key2;
        unsigned int* pos_by_cell = B.mem;
        int* counts = (int*)B.gkey;
        int* run = (int*)B.gkey2;
        unsigned int* mark = B.gid;
        hipLaunchKernelGGL(k_eap_poskey, dim3(nb), dim3(256), 0, st, B.comp, K, B.i0, invR, keyp, B.i1);
        tb = tmp;
        EAPCHK(hipcub::DeviceRadixSort::SortPairs(B.tmp, tb, keyp, keys, B.i1, pos_by_cell, Ki, 0, 64, st));
        tb = tmp;
        EAPCHK(hipcub::DeviceRunLengthEncode::Encode(B.tmp, tb, keys, keyp, counts, (int*)B.misc + 4, Ki, st));
        int ncell = 0;
        EAPCHK(hipMemcpyAsync(&ncell, (int*)B.misc + 4, sizeof(int), hipMemcpyDeviceToHost, st));
        EAPCHK(hipStreamSynchronize(st));
        EAPCHK(hipMemsetAsync(run, 0, sizeof(int), st));
        tb = tmp;
        EAPCHK(hipcub::DeviceScan::InclusiveSum(B.tmp, tb, counts, run + 1, ncell, st));
        hipLaunchKernelGGL(k_eap_merge_cells, dim3(G), dim3(EAP2_NT), 0, st, B.comp, K, B.i0, B.runs, B.rank, keyp,
                           ncell, run, pos_by_cell, invR, T, mark, B.out, B.orank, (int*)B.misc + 3);
    }
    EAPCHK(hipGetLastError());
    int nout = 0;
    EAPCHK(hipMemcpyAsync(&nout, (int*)B.misc + 3, sizeof(int), hipMemcpyDeviceToHost, st));
    EAPCHK(hipStreamSynchronize(st));
    if (n_groups) *n_groups = G;
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
