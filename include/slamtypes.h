/*
 * slamtypes.h — drop-in C++ types of the reference (src/slamtypes.h) for code
 * written against phdfilter.h (e.g. the reference's main.cpp driver).
 *
 * The POD types are the plain-C layouts of phd_types.h under the reference's
 * names; byte layouts are identical (static asserts in phd_types.h).  The
 * particle containers (ParticleSLAM, SynthSLAM) keep the reference's members
 * and copy_particles semantics (slamtypes.h:272-337) so host code compiles
 * unchanged.  Not carried over: the disparity/camera types (out of scope,
 * SURVEY.md §2.1) and the never-defined SynthSLAM::predict_cpu/update_cpu
 * (slamtypes.h:335-336; the CPU restatement of the path is the test oracle,
 * oracle/scphd_cpu.cpp).
 */
#ifndef SLAMTYPES_H_
#define SLAMTYPES_H_

#include <float.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "phd_types.h"

#define REAL float
#define PHD_TYPE PHD_FILTER_PHD
#define CPHD_TYPE PHD_FILTER_CPHD
#define CV_MOTION PHD_MOTION_CV
#define ACKERMAN_MOTION PHD_MOTION_ACKERMAN
#define LOG0 -FLT_MAX
#define STATIC_MODEL PHD_FEATURE_STATIC
#define DYNAMIC_MODEL PHD_FEATURE_DYNAMIC
#define MIXED_MODEL PHD_FEATURE_MIXED
#define STATIC_MEASUREMENT PHD_MEAS_STATIC
#define DYNAMIC_MEASUREMENT PHD_MEAS_DYNAMIC

// The reference header exports the std namespace; host code relies on it.
using namespace std;

// ConstantVelocityState, ConstantVelocityNoise, AckermanControl, AckermanNoise,
// RangeBearingMeasurement, Gaussian2D, Gaussian4D and SlamConfig are the struct tags of
// phd_types.h (identical layouts, identical C++ names).

typedef struct {
    REAL px, py, ptheta;
} AckermanState;

typedef struct {
    REAL cov[9];
    REAL mean[3];
    REAL weight;
} Gaussian3D;

typedef vector<Gaussian2D> GaussianMixture;
typedef vector<RangeBearingMeasurement> measurementSet;

class ParticleSLAM {
public:
    int n_particles;
    vector<REAL> weights;
    vector<ConstantVelocityState> states;
    vector<int> resample_idx;

    ParticleSLAM(unsigned int n = 100) : n_particles(n), weights(n), states(n), resample_idx(n) {}
};

class SynthSLAM : public ParticleSLAM {
public:
    vector<vector<Gaussian2D> > maps_static;
    vector<vector<Gaussian4D> > maps_dynamic;
    vector<Gaussian2D> max_map_static;
    vector<Gaussian4D> max_map_dynamic;
    vector<Gaussian2D> exp_map_static;
    vector<Gaussian4D> exp_map_dynamic;
    vector<vector<REAL> > cardinalities;
    vector<REAL> cardinality_birth;
    vector<REAL> variances;

    SynthSLAM(unsigned int n)
        : ParticleSLAM(n), maps_static(n), maps_dynamic(n), cardinalities(n), variances(n) {}

    /* Children take the parent's state and maps; weights become -log N. */
    SynthSLAM copy_particles(const vector<int>& indices) const {
        SynthSLAM out((unsigned int)indices.size());
        const REAL w = -log((double)indices.size());
        for (size_t j = 0; j < indices.size(); j++) {
            const int i = indices[j];
            out.maps_static[j] = maps_static[i];
            out.maps_dynamic[j] = maps_dynamic[i];
            out.cardinalities[j] = cardinalities[i];
            out.weights[j] = w;
            out.states[j] = states[i];
            out.variances[j] = variances[i];
        }
        out.resample_idx = indices;
        return out;
    }
};

#endif /* SLAMTYPES_H_ */
