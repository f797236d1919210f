/*
 * phd_types.h — plain-C layouts shared by the C-ABI, the HIP kernels, the CPU
 * oracle and the C++ drop-in headers.
 *
 * Every struct here is byte-identical to the reference type it stands in for
 * (reference: src/slamtypes.h).  Sizes/offsets are pinned with static asserts
 * below and re-checked from Python in tests/test_capi_symbols.py:
 *   Gaussian2D               28 B   (slamtypes.h:123-127)
 *   Gaussian4D               84 B   (slamtypes.h:135-139)
 *   ConstantVelocityState    24 B   (slamtypes.h:44-51)
 *   AckermanControl           8 B   (slamtypes.h:83-87)
 *   AckermanNoise             8 B   (slamtypes.h:90-93)
 *   ConstantVelocityNoise    12 B   (slamtypes.h:70-74)
 *   RangeBearingMeasurement  12 B   (slamtypes.h:96-101)
 *   SlamConfig              324 B   (slamtypes.h:142-250)
 *
 * The C typedef names carry a phd_ prefix; the struct tags are the reference's
 * type names, so C++ code sees the same types (and the same mangled symbol
 * names, e.g. phdUpdateSynth(SynthSLAM&, std::vector<RangeBearingMeasurement>))
 * as a build against the reference's slamtypes.h.
 */
#ifndef PHD_TYPES_H
#define PHD_TYPES_H

#ifndef __cplusplus
#include <stdbool.h>
#endif
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Filter / model selectors (slamtypes.h:21-35). */
#define PHD_FILTER_PHD 0
#define PHD_FILTER_CPHD 1
#define PHD_MOTION_CV 0
#define PHD_MOTION_ACKERMAN 1
#define PHD_FEATURE_STATIC 0
#define PHD_FEATURE_DYNAMIC 1
#define PHD_FEATURE_MIXED 2
#define PHD_MEAS_STATIC 0
#define PHD_MEAS_DYNAMIC 1

/* One 2-D Gaussian-mixture component: column-major 2x2 covariance, mean, weight. */
typedef struct Gaussian2D {
    float cov[4];
    float mean[2];
    float weight;
} phd_gaussian2d;

/* One 4-D (position + velocity) component of a dynamic map: column-major 4x4
 * covariance, mean (x, y, vx, vy), weight (slamtypes.h:135-139). */
typedef struct Gaussian4D {
    float cov[16];
    float mean[4];
    float weight;
} phd_gaussian4d;

/* Vehicle pose particle state (position, heading, and their rates). */
typedef struct ConstantVelocityState {
    float px, py, ptheta;
    float vx, vy, vtheta;
} phd_pose;

typedef struct AckermanControl {
    float alpha;      /* steering angle */
    float v_encoder;  /* encoder velocity */
} phd_ackerman_control;

typedef struct AckermanNoise {
    float n_alpha;
    float n_encoder;
} phd_ackerman_noise;

typedef struct ConstantVelocityNoise {
    float ax, ay, atheta;
} phd_cv_noise;

typedef struct RangeBearingMeasurement {
    float range;
    float bearing;
    int label;
} phd_measurement;

/* Run configuration; field order/size is the ABI of the reference's SlamConfig. */
typedef struct SlamConfig {
    bool debug;
    float x0, y0, z0, roll0, pitch0, yaw0;
    float vx0, vy0, vz0, vroll0, vpitch0, vyaw0;
    bool followTrajectory;
    float ax, ay, az, aroll, apitch, ayaw;
    float dt;
    float minRange, maxRange, maxBearing;
    float stdRange, stdBearing;
    float clutterRate, clutterDensity, pd;
    float stdVxMap, stdVyMap, stdAxMap, stdAyMap;
    float covVxBirth, covVyBirth;
    float ps, tau, beta;
    int particlesPerFeature, imageWidth, imageHeight;
    float stdU, stdV, disparityBirth, stdDBirth, fx, fy, u0, v0;
    int n_particles, nPredictParticles, subdividePredict;
    float resampleThresh, birthWeight, birthNoiseFactor;
    bool gateBirths, gateMeasurements;
    float gateThreshold, minExpectedFeatureWeight, minSeparation;
    int maxFeatures;
    float minFeatureWeight;
    int particleWeighting, daughterMixtureType, nSamples, maxCardinality;
    int filterType, distanceMetric, maxSteps, featureModel, motionType;
    int mapEstimate, cphdDistType;
    float nu;
    bool labeledMeasurements;
    float l, h, a, b, stdAlpha, stdEncoder;
    bool saveAllMaps, savePrediction;
} phd_slam_config;

#ifdef __cplusplus
}  /* extern "C" */
#define PHD_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define PHD_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

PHD_STATIC_ASSERT(sizeof(phd_gaussian2d) == 28, "Gaussian2D must be 28 B");
PHD_STATIC_ASSERT(sizeof(phd_gaussian4d) == 84, "Gaussian4D must be 84 B");
PHD_STATIC_ASSERT(sizeof(phd_pose) == 24, "ConstantVelocityState must be 24 B");
PHD_STATIC_ASSERT(sizeof(phd_ackerman_control) == 8, "AckermanControl must be 8 B");
PHD_STATIC_ASSERT(sizeof(phd_measurement) == 12, "RangeBearingMeasurement must be 12 B");
PHD_STATIC_ASSERT(sizeof(phd_slam_config) == 324, "SlamConfig must be 324 B");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, clutterDensity) == 108, "clutterDensity@108");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, pd) == 112, "pd@112");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, n_particles) == 196, "n_particles@196");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, labeledMeasurements) == 292, "labeled@292");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, l) == 296, "l@296");
PHD_STATIC_ASSERT(offsetof(phd_slam_config, saveAllMaps) == 320, "saveAllMaps@320");

#endif /* PHD_TYPES_H */
