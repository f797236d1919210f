/*
 * phd_terms.hip — middle launch of the three-launch CPHD update (config 3):
 * the GM-CPHD weight terms of one particle by ONE WAVEFRONT (64 lanes), from
 * part A's handoff (η fixed point, map sums) to part C's (per-measurement
 * detection factors and listing bounds, non-detection factor, Δ log w, the
 * particle's cardinality coefficients).  Arithmetic: phd_cphd_terms.h
 * (phdfilter.cu.bak:990-1504, Poisson prior .bak:2473-2497).
 */
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "phd_detmath.h"
#include "phd_device.h"
#include "phd_devutil.h"
#include "phd_kernels.h"
#include "phd_cphd_terms.h"

namespace phd {

__global__ void __launch_bounds__(64) k_cphd_terms(UpdateArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cphd_terms_one(a, upd_particle(a, (int)blockIdx.x, (int)gridDim.x), (double*)smem);
}

}  // namespace phd
