"""Reference data formats (include/phd_io.h, host-only; no GPU).

Loaders of the reference driver (src/main.cpp:147-245) and its per-step log
writer writeLog (src/main.cpp:848-954), backed by libphdslam.so.  Format flags:

  HEADER    skip the first line (the reference's loadControls / loadMeasurements)
  COMMAS    ',' separates values (python/controls_synth.txt)
  PAIRS     (range, bearing) pairs per measurement, label 0 (python/measurements_synth.txt);
            default is the reference's (range, bearing, label) triples
  COMMENTS  skip lines starting with '%' or '#'
"""
import ctypes
import os

import numpy as np

from . import _lib
from .types import ACKERMAN_CONTROL, GAUSSIAN2D, MEASUREMENT, POSE

HEADER, COMMAS, PAIRS, COMMENTS = 1, 2, 4, 8


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


def _path(path):
    return os.fsencode(os.fspath(path))


def load_timestamps(path):
    """loadTimestamps (main.cpp:147-167) -> float64 array."""
    n = ctypes.c_int()
    rc = _lib.lib().phd_load_timestamps(_path(path), None, 0, ctypes.byref(n))
    if rc not in (_lib.PHD_OK, _lib.PHD_E_CAPACITY):
        _lib.check(rc, "phd_load_timestamps")
    out = np.zeros(n.value, np.float64)
    _lib.check(_lib.lib().phd_load_timestamps(_path(path), _p(out), n.value, ctypes.byref(n)), "phd_load_timestamps")
    return out


def load_controls(path, flags=HEADER):
    """loadControls (main.cpp:169-190) -> ACKERMAN_CONTROL array (fields v_encoder, alpha)."""
    n = ctypes.c_int()
    rc = _lib.lib().phd_load_controls(_path(path), int(flags), None, 0, ctypes.byref(n))
    if rc not in (_lib.PHD_OK, _lib.PHD_E_CAPACITY):
        _lib.check(rc, "phd_load_controls")
    out = np.zeros(n.value, ACKERMAN_CONTROL)
    _lib.check(_lib.lib().phd_load_controls(_path(path), int(flags), _p(out), n.value, ctypes.byref(n)),
               "phd_load_controls")
    return out


def load_measurements(path, flags=HEADER):
    """loadMeasurements (main.cpp:221-245) -> (MEASUREMENT array, offsets[n_steps + 1])."""
    ns = ctypes.c_int()
    off1 = np.zeros(1, np.int32)
    rc = _lib.lib().phd_load_measurements(_path(path), int(flags), None, 0, _p(off1), 0, ctypes.byref(ns))
    if rc not in (_lib.PHD_OK, _lib.PHD_E_CAPACITY):
        _lib.check(rc, "phd_load_measurements")
    steps = ns.value
    offs = np.zeros(steps + 1, np.int32)
    # the count pass sizes the offsets; the measurement count comes from a pass with offsets
    rc = _lib.lib().phd_load_measurements(_path(path), int(flags), None, 0, _p(offs), steps, ctypes.byref(ns))
    if rc not in (_lib.PHD_OK, _lib.PHD_E_CAPACITY):
        _lib.check(rc, "phd_load_measurements")
    total = int(offs[steps])
    z = np.zeros(total, MEASUREMENT)
    _lib.check(_lib.lib().phd_load_measurements(_path(path), int(flags), _p(z), total, _p(offs), steps,
                                                ctypes.byref(ns)), "phd_load_measurements")
    return z, offs


def write_state_log(directory, t, expected_pose, exp_map, log_weights, poses, resample_idx=None, cn=None,
                    max_cardinality=0, filter_type=0, n_predict_particles=1):
    """writeLog (main.cpp:848-954): append directory/state_estimate{t:05d}.log."""
    ep = np.ascontiguousarray(np.asarray(expected_pose, POSE).reshape(1))
    m = np.ascontiguousarray(np.asarray(exp_map, GAUSSIAN2D).reshape(-1))
    w = np.ascontiguousarray(np.asarray(log_weights, np.float32).reshape(-1))
    ps = np.ascontiguousarray(np.asarray(poses, POSE).reshape(-1))
    ri = None if resample_idx is None else np.ascontiguousarray(np.asarray(resample_idx, np.int32).reshape(-1))
    c = None if cn is None else np.ascontiguousarray(np.asarray(cn, np.float32).reshape(-1))
    if len(w) != len(ps) or (ri is not None and len(ri) != len(w)):
        raise ValueError("log_weights, poses and resample_idx must have one entry per particle")
    if filter_type == 1 and (c is None or len(c) < max_cardinality + 1):
        raise ValueError("a CPHD log needs max_cardinality + 1 cardinality values")
    _lib.check(_lib.lib().phd_write_state_log(_path(directory), int(t), _p(ep), _p(m), len(m), _p(w), _p(ps), len(w),
                                              _p(ri), _p(c), int(max_cardinality), int(filter_type),
                                              int(n_predict_particles)), "phd_write_state_log")
    return os.path.join(os.fspath(directory), f"state_estimate{int(t):05d}.log")


def read_state_log(path):
    """Parse a state_estimate log back (the line layout of writeLog; python/batch_analyze.py
    compute_error_k reads the first lines the same way with numpy.fromstring(sep=' '))."""
    with open(path) as f:
        lines = f.read().split("\n")

    def vals(i):
        return np.array(lines[i].split(), np.float64) if i < len(lines) else np.zeros(0)

    pose = vals(0)
    m = vals(1).reshape(-1, 7)
    return {"pose": pose, "map_weight": m[:, 0], "map_mean": m[:, 1:3], "map_cov": m[:, 3:7], "dynamic": vals(2),
            "log_weights": vals(3), "poses": vals(4).reshape(-1, 6), "resample_idx": vals(5).astype(np.int64),
            "cardinality": vals(6)}
