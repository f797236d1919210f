/*
 * phd_mixed_k.h — launch interface of the mixed static + dynamic feature model
 * kernels (phd_mixed.hip; SURVEY.md §8(f) rank 4, feature_model = 2).
 *
 * Dynamic maps live in their own ping-pong slab sets, indexed by the same slab
 * id as the static maps (particle n's maps are slab d_src[n] of each set), so
 * resampling and the n_predict_particles spawn (index remaps of d_src) carry
 * them with no copy.  Dynamic slab: SoA [w | m0..m3 | c0..c15] x dcap floats.
 */
#ifndef PHD_MIXED_K_H
#define PHD_MIXED_K_H

#include <hip/hip_runtime.h>

#include <string>

#include "phd_mixed.h"
#include "phd_types.h"

namespace phd {

#define PHD_DYN_FIELDS 21
/* status bits (phd_kernels.h PHD_ST_CANDIDATE_OVERFLOW / PHD_ST_MAP_OVERFLOW) */
#define PHD_ST_CANDIDATE_OVERFLOW_MX 2
#define PHD_ST_MAP_OVERFLOW_MX 4

struct MixedArgs {
    int n;            // particles (one workgroup each)
    int cap, dcap;    // static / dynamic slab capacities
    int M, Kcap;      // measurements, candidate capacity per map
    const int* src;   // slab of particle n in the input sets
    int* src_reset;   // posterior of particle n -> output slab n
    const float* map_in;
    float* map_out;
    const int* size_in;
    int* size_out;
    const float* dmap_in;
    float* dmap_out;
    const int* dsize_in;
    int* dsize_out;
    const phd_pose* poses;
    float* logw;
    float* delta;
    int* status;
    int* err;
    const float* zr;
    const float* zb;
    const int* zlab;
    phd_mx_cfg c;
    float* ekf;       // per particle (cap + dcap) x 32 floats
    float* cand;      // per particle Kcap x (7 + 21) floats
};

/* dynamic LDS bytes of k_update_mixed */
size_t mixed_lds_bytes(int cap, int dcap, int Mcap, int Kcap);
/* per-particle global scratch (floats) */
size_t mixed_ekf_floats(int cap, int dcap);
size_t mixed_cand_floats(int Kcap);

hipError_t mixed_launch_update(const MixedArgs& a, size_t lds, hipStream_t s);
/* one predictMapMixed over `nslabs` slabs: set in -> set out */
hipError_t mixed_launch_predict(int nslabs, int dcap, const float* din, const int* dsize_in, float* dout,
                                int* dsize_out, const phd_mx_cfg& c, hipStream_t s);
hipError_t mixed_set_lds_limit();
/* EAP map of the dynamic maps of n particles (exp_map_dynamic): the component
 * count (nothing copied when out is NULL or too small), -1 on a HIP error */
long mixed_expected_map_dynamic(hipStream_t st, const int* d_src, const float* d_dmap, const int* d_dsize, int n,
                                int dcap, const float* d_logw, float T, phd_gaussian4d* out, long out_cap,
                                std::string& err);

}  // namespace phd

#endif /* PHD_MIXED_K_H */
