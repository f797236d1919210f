/*
 * phd_io.h — host-only data loaders and the per-step log writer of the
 * reference driver (src/main.cpp), as C-ABI functions of libphdslam.so.
 * No GPU is touched; they run on any host.  Return PHD_OK or a PHD_E* code
 * (PHD_E_CAPACITY: the output buffer is too small — the count is still
 * written so the caller can size it and call again).
 */
#ifndef PHD_IO_H
#define PHD_IO_H

#include "phd_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Format flags of the loaders. */
#define PHD_IO_HEADER 1 /* first line is a header and is skipped (the reference's loaders, main.cpp:176,230) */
#define PHD_IO_COMMAS 2 /* ',' separates values (python/controls_synth.txt: "v, alpha") */
#define PHD_IO_PAIRS 4  /* measurements are (range, bearing) pairs, label 0 (python/measurements_synth.txt) */
#define PHD_IO_COMMENTS 8 /* lines starting with '%' or '#' are skipped (MATLAB-style headers) */

/* loadTimestamps (main.cpp:147-167): one value per line. */
int phd_load_timestamps(const char* path, double* out, int cap, int* n);

/* loadControls (main.cpp:169-190): one "v_encoder alpha" per line. */
int phd_load_controls(const char* path, int flags, phd_ackerman_control* out, int cap, int* n);

/* loadMeasurements + parseMeasurements (main.cpp:192-245): one time step per
 * line; measurements of step s are out[offsets[s] .. offsets[s+1]).
 * offsets holds max_steps + 1 entries; *n_steps receives the step count. */
int phd_load_measurements(const char* path, int flags, phd_measurement* out, long cap, int* offsets, int max_steps,
                          int* n_steps);

/* writeLog (main.cpp:848-954): appends dir/state_estimateNNNNN.log (t = NNNNN)
 * with the reference's seven lines.  resample_idx NULL = identity; cn holds
 * max_cardinality + 1 values and is read only when filter_type == 1 (CPHD). */
int phd_write_state_log(const char* dir, int t, const phd_pose* expected_pose, const phd_gaussian2d* map,
                        long n_map, const float* log_weights, const phd_pose* poses, int n, const int* resample_idx,
                        const float* cn, int max_cardinality, int filter_type, int n_predict_particles);

#ifdef __cplusplus
}
#endif

#endif /* PHD_IO_H */
