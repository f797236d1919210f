/*
 * phdfilter.h — the reference's filter API (src/phdfilter.h:10-34), exported
 * by libphdslam.so (cuda-phdslam_amd/csrc/phdfilter_shim.cpp) on top of the
 * C-ABI in phd_capi.h.  Same names, argument meaning and in-place semantics:
 *
 *   setDeviceConfig(config)          copy of the run configuration (phdfilter.cu:3885)
 *   initRandomNumberGenerators()     (re)seed the RNG contract (phd_rng.h)
 *   phdPredict(particles, ...)       in place; Ackerman reads one AckermanControl
 *                                    by value from the variadic list (phdfilter.cu:1140)
 *   phdUpdateSynth(particles, Z)     in place on maps_static / weights (normalised);
 *                                    returns the pre-update particles (phdfilter.cu:3351)
 *   recoverSlamState(...)            expected pose, MAP / EAP map (main.cpp:318-388)
 *
 * Host state is authoritative through this surface (like the reference), so
 * each call moves the particle store over PCIe; the device-resident fast path
 * is the C-ABI (phd_step, phd_capi.h).
 */
#ifndef PHDFILTER_H
#define PHDFILTER_H

#ifdef __cplusplus

#include "slamtypes.h"

void initRandomNumberGenerators();

void predictMap(SynthSLAM& p);

void phdPredict(SynthSLAM& particles, ...);

SynthSLAM phdUpdateSynth(SynthSLAM& particles, measurementSet measurements);

void recoverSlamState(SynthSLAM& particles, ConstantVelocityState& expectedPose, vector<REAL>& cn_estimate);

void setDeviceConfig(const SlamConfig& config);

/* CPHD births through the prediction (addBirths, phdfilter.cu.bak:794-870):
 * in place, one birth component per measurement of the previous scan appended
 * to every particle's map (phd_add_births on the device). */
void addBirths(SynthSLAM& particles, measurementSet measurements);

/* Host-side stratified resample of the run_synth driver (main.cpp:453-501)
 * with the build's RNG contract: returns the resampled particle set. */
SynthSLAM resampleParticles(const SynthSLAM& particles, int n_new_particles, uint64_t step);

#endif

#endif  // PHDFILTER_H
