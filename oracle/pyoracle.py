"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product path.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
from phdslam.types import (ACKERMAN_NOISE, CV_NOISE, GAUSSIAN2D, GAUSSIAN4D, MEASUREMENT, POSE,  # noqa: E402
                           AckermanControl, SlamConfig)

_L = None
_LF = None


def lib(fast=False):
    """The checker build (liboracle.so), or fast=True: the optimised build of
    the same source (liboracle_fast.so, bench.py's cpu_baseline leg only)."""
    global _L, _LF
    if fast:
        if _LF is None:
            path = os.path.join(HERE, "liboracle_fast.so")
            if not os.path.exists(path):
                subprocess.run(["make", "-s", "-C", HERE, "liboracle_fast.so"], check=True)
            _LF = _bind(ctypes.CDLL(path))
        return _LF
    if _L is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        _L = _bind(ctypes.CDLL(path))
    return _L


def _bind(L):
    vp = ctypes.c_void_p
    L.orc_set_threads.restype = ctypes.c_int
    L.orc_set_threads.argtypes = [ctypes.c_int]
    L.orc_wrap_angle.restype = ctypes.c_float
    L.orc_wrap_angle.argtypes = [ctypes.c_float]
    L.orc_safe_log.restype = ctypes.c_float
    L.orc_safe_log.argtypes = [ctypes.c_float]
    L.orc_det_expf.restype = ctypes.c_float
    L.orc_det_expf.argtypes = [ctypes.c_float]
    L.orc_atan2f.restype = ctypes.c_float
    L.orc_atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    L.orc_sincosf.argtypes = [ctypes.c_float, vp, vp]
    L.orc_tanf.restype = ctypes.c_float
    L.orc_tanf.argtypes = [ctypes.c_float]
    L.orc_philox.argtypes = [ctypes.c_uint32] * 6 + [vp]
    L.orc_measure.argtypes = [vp, ctypes.c_float, ctypes.c_float, vp]
    L.orc_birth.argtypes = [vp, vp, vp, vp]
    L.orc_noise_ackerman.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.orc_noise_cv.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.orc_resample_uniforms.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.orc_predict_ackerman.argtypes = [vp, ctypes.c_int, vp, AckermanControl, vp, vp]
    L.orc_predict_cv.argtypes = [vp, ctypes.c_int, vp, vp, vp]
    L.orc_update.restype = ctypes.c_long
    L.orc_update.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_long, vp, vp, vp]
    L.orc_update_cn.restype = ctypes.c_long
    L.orc_update_cn.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_long, vp, vp, vp, vp]
    L.orc_normalize.restype = ctypes.c_float
    L.orc_normalize.argtypes = [ctypes.c_int, vp]
    L.orc_neff.restype = ctypes.c_float
    L.orc_neff.argtypes = [ctypes.c_int, vp]
    L.orc_resample_faithful.argtypes = [ctypes.c_int, vp, vp, vp]
    L.orc_resample_fixed.argtypes = [ctypes.c_int, vp, vp, vp]
    L.orc_resample_fixed_to.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, vp]
    L.orc_expected_pose.restype = ctypes.c_int
    L.orc_expected_pose.argtypes = [ctypes.c_int, vp, vp, vp]
    L.orc_expected_map.restype = ctypes.c_long
    L.orc_expected_map.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_long]
    L.orc_expected_map_cells.restype = ctypes.c_long
    L.orc_expected_map_cells.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_long]
    L.orc_copy_particles.restype = ctypes.c_long
    L.orc_copy_particles.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    return L


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _cfgp(cfg):
    return ctypes.cast(ctypes.pointer(cfg), ctypes.c_void_p)


def wrap_angle(a):
    return lib().orc_wrap_angle(float(a))


def det_expf(x):
    return lib().orc_det_expf(float(x))


def atan2f(y, x):
    return lib().orc_atan2f(float(y), float(x))


def sincosf(x):
    """(sin x, cos x) of the shared deterministic helper (phd_detmath.h, D16)."""
    s, c = ctypes.c_float(), ctypes.c_float()
    lib().orc_sincosf(float(x), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def tanf(x):
    return lib().orc_tanf(float(x))


def philox(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().orc_philox(*[int(c) & 0xffffffff for c in ctr], *[int(k) & 0xffffffff for k in key], _p(out))
    return out


def measure(pose, fx, fy):
    p = np.zeros(1, POSE)
    p[0] = pose
    out = np.zeros(2, np.float32)
    lib().orc_measure(_p(p), float(fx), float(fy), _p(out))
    return out


def birth(cfg, pose, z):
    p = np.zeros(1, POSE)
    p[0] = pose
    zz = np.zeros(1, MEASUREMENT)
    zz[0] = z
    out = np.zeros(1, GAUSSIAN2D)
    lib().orc_birth(_cfgp(cfg), _p(p), _p(zz), _p(out))
    return out[0]


def set_threads(t, fast=False):
    """OpenMP threads of the oracle's per-particle loop; returns the effective count."""
    return lib(fast).orc_set_threads(int(t))


def noise_ackerman(cfg, n, seed, step):
    out = np.zeros(n, ACKERMAN_NOISE)
    lib().orc_noise_ackerman(_cfgp(cfg), n, seed, step, _p(out))
    return out


def noise_cv(cfg, n, seed, step):
    out = np.zeros(n, CV_NOISE)
    lib().orc_noise_cv(_cfgp(cfg), n, seed, step, _p(out))
    return out


def resample_uniforms(n, seed, step):
    out = np.zeros(n, np.float64)
    lib().orc_resample_uniforms(n, seed, step, _p(out))
    return out


def predict_ackerman(cfg, poses, v_encoder, alpha, noise, fast=False):
    poses = np.ascontiguousarray(poses, POSE)
    noise = np.ascontiguousarray(noise, ACKERMAN_NOISE)
    out = np.zeros(len(noise), POSE)
    lib(fast).orc_predict_ackerman(_cfgp(cfg), len(noise), _p(poses), AckermanControl(alpha, v_encoder),
                                   _p(noise), _p(out))
    return out


def predict_cv(cfg, poses, noise, fast=False):
    poses = np.ascontiguousarray(poses, POSE)
    noise = np.ascontiguousarray(noise, CV_NOISE)
    out = np.zeros(len(noise), POSE)
    lib(fast).orc_predict_cv(_cfgp(cfg), len(noise), _p(poses), _p(noise), _p(out))
    return out


def add_births(cfg, poses, maps, offsets, z, fast=False):
    """CPHD births of the measurements z appended to every map (orc_add_births;
    fast=True: the optimised build, bench.py's cpu_baseline)."""
    poses = np.ascontiguousarray(poses, POSE)
    maps = np.ascontiguousarray(maps, GAUSSIAN2D)
    offsets = np.ascontiguousarray(offsets, np.int32)
    z = np.ascontiguousarray(z, MEASUREMENT)
    n = len(poses)
    cap = len(maps) + n * len(z) + 1
    out = np.zeros(cap, GAUSSIAN2D)
    offs = np.zeros(n + 1, np.int32)
    L = lib(fast)
    L.orc_add_births.restype = ctypes.c_long
    tot = L.orc_add_births(_cfgp(cfg), n, _p(poses), _p(maps), _p(offsets), _p(z), len(z), _p(out), cap, _p(offs))
    if tot < 0:
        raise RuntimeError("orc_add_births failed")
    return out[:tot].copy(), offs


_last_near = [0]


def near_counts():
    """Per particle of the last update(): (classification, prune/merge) counts of
    decisions within 1e-4 (relative) of their threshold.  A near classification
    can move the log-weight and any component; a near prune / merge decision only
    the components built from the candidates it touches."""
    n = _last_near[0]
    cls = np.zeros(n, np.int32)
    pm = np.zeros(n, np.int32)
    if lib().orc_near_counts(n, _p(cls), _p(pm)) != 0:
        raise RuntimeError("no oracle update to report")
    return cls, pm


def update(cfg, poses, maps, offsets, z, cardinality=False, fast=False):
    """Static PHD (filterType 0) or CPHD (filterType 1) update of every particle
    (particles on the oracle's OpenMP threads).  Returns (maps_out, offsets_out,
    delta, margin), plus the per-particle log cardinality distribution
    (n, maxCardinality+1) when cardinality=True (CPHD).  fast=True: the
    optimised build (bench.py's cpu_baseline leg)."""
    poses = np.ascontiguousarray(poses, POSE)
    maps = np.ascontiguousarray(maps, GAUSSIAN2D)
    offsets = np.ascontiguousarray(offsets, np.int32)
    z = np.ascontiguousarray(z, MEASUREMENT)
    n = len(poses)
    M = min(len(z), 256)
    sizes = np.diff(offsets)
    cap = int(np.sum(sizes * (M + 1) + M) + 16)
    out = np.zeros(cap, GAUSSIAN2D)
    offs = np.zeros(n + 1, np.int32)
    delta = np.zeros(n, np.float32)
    margin = np.zeros(n, np.float32)
    cn = np.zeros((n, max(cfg.maxCardinality, 0) + 1), np.float64) if cardinality else None
    tot = lib(fast).orc_update_cn(_cfgp(cfg), n, _p(poses), _p(maps), _p(offsets), _p(z), len(z), _p(out), cap,
                              _p(offs), _p(delta), _p(margin), _p(cn) if cn is not None else None)
    if tot < 0:
        raise RuntimeError("oracle update failed (unsupported config or overflow)")
    if not fast:
        _last_near[0] = n
    if cardinality:
        return out[:tot].copy(), offs, delta, margin, cn
    return out[:tot].copy(), offs, delta, margin


def predict_dynamic(cfg, comps):
    """predictMapMixed of a flat array of Gaussian4D components (orc_predict_dynamic)."""
    comps = np.ascontiguousarray(comps, GAUSSIAN4D)
    out = np.zeros(len(comps), GAUSSIAN4D)
    L = lib()
    L.orc_predict_dynamic.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    L.orc_predict_dynamic(_cfgp(cfg), len(comps), _p(comps), _p(out))
    return out


def update_mixed(cfg, poses, smaps, soffs, dmaps, doffs, z):
    """Mixed static + dynamic update (feature_model 2) of every particle.
    Returns (static maps, offsets, dynamic maps, offsets, delta, margin)."""
    poses = np.ascontiguousarray(poses, POSE)
    smaps = np.ascontiguousarray(smaps, GAUSSIAN2D)
    soffs = np.ascontiguousarray(soffs, np.int32)
    dmaps = np.ascontiguousarray(dmaps, GAUSSIAN4D)
    doffs = np.ascontiguousarray(doffs, np.int32)
    z = np.ascontiguousarray(z, MEASUREMENT)
    n = len(poses)
    M = min(len(z), 256)
    scap = int(np.sum(np.diff(soffs) * (M + 1) + M) + 16)
    dcap = int(np.sum(np.diff(doffs) * (M + 1) + M) + 16)
    sout = np.zeros(scap, GAUSSIAN2D)
    dout = np.zeros(dcap, GAUSSIAN4D)
    so = np.zeros(n + 1, np.int32)
    do = np.zeros(n + 1, np.int32)
    delta = np.zeros(n, np.float32)
    margin = np.zeros(n, np.float32)
    L = lib()
    L.orc_update_mixed.restype = ctypes.c_long
    vp = ctypes.c_void_p
    L.orc_update_mixed.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_long, vp,
                                   vp, ctypes.c_long, vp, vp, vp]
    rc = L.orc_update_mixed(_cfgp(cfg), n, _p(poses), _p(smaps), _p(soffs), _p(dmaps), _p(doffs), _p(z), len(z),
                            _p(sout), scap, _p(so), _p(dout), dcap, _p(do), _p(delta), _p(margin))
    if rc < 0:
        raise RuntimeError("oracle mixed update failed (unsupported config or overflow)")
    _last_near[0] = n
    return sout[:so[-1]].copy(), so, dout[:do[-1]].copy(), do, delta, margin


def normalize(w, fast=False):
    w = np.array(w, dtype=np.float32)
    lse = lib(fast).orc_normalize(len(w), _p(w))
    return w, lse


def neff(w):
    w = np.ascontiguousarray(w, np.float32)
    return lib().orc_neff(len(w), _p(w))


def resample_faithful(w, u_with_leading):
    w = np.ascontiguousarray(w, np.float32)
    u = np.ascontiguousarray(u_with_leading, np.float64)
    assert len(u) == len(w) + 1
    idx = np.zeros(len(w), np.int32)
    lib().orc_resample_faithful(len(w), _p(w), _p(u), _p(idx))
    return idx


def resample_fixed(w, u):
    """len(u) strata over the weights w (len(u) < len(w) after n_predict_particles spawned children)."""
    w = np.ascontiguousarray(w, np.float32)
    u = np.ascontiguousarray(u, np.float64)
    idx = np.zeros(len(u), np.int32)
    lib().orc_resample_fixed_to(len(w), _p(w), len(u), _p(u), _p(idx))
    return idx


def expected_pose(w, poses):
    w = np.ascontiguousarray(w, np.float32)
    poses = np.ascontiguousarray(poses, POSE)
    out = np.zeros(1, POSE)
    mi = lib().orc_expected_pose(len(w), _p(w), _p(poses), _p(out))
    return out[0], mi


def expected_map(cfg, w, maps, offsets, cells=False):
    """EAP expected map (computeExpectedMap + reduceGaussianMixture).  cells=True:
    the same greedy with the distance tests restricted to touching lattice cells
    (orc_expected_map_cells: identical outputs, feasible at millions of components)."""
    w = np.ascontiguousarray(w, np.float32)
    maps = np.ascontiguousarray(maps, GAUSSIAN2D)
    offsets = np.ascontiguousarray(offsets, np.int32)
    out = np.zeros(max(1, len(maps)), GAUSSIAN2D)
    fn = lib().orc_expected_map_cells if cells else lib().orc_expected_map
    n = fn(_cfgp(cfg), len(w), _p(w), _p(maps), _p(offsets), _p(out), len(out))
    return out[:n].copy()


def expected_map_dynamic(cfg, w, maps, offsets):
    """EAP map of the dynamic (Gaussian4D) maps (exp_map_dynamic, main.cpp:369-371)."""
    w = np.ascontiguousarray(w, np.float32)
    maps = np.ascontiguousarray(maps, GAUSSIAN4D)
    offsets = np.ascontiguousarray(offsets, np.int32)
    out = np.zeros(max(1, len(maps)), GAUSSIAN4D)
    L = lib()
    L.orc_expected_map_dynamic.restype = ctypes.c_long
    L.orc_expected_map_dynamic.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_long]
    k = L.orc_expected_map_dynamic(_cfgp(cfg), len(w), _p(w), _p(maps), _p(offsets), _p(out), len(out))
    return out[:k].copy()


def copy_particles(idx, poses, maps, offsets):
    idx = np.ascontiguousarray(idx, np.int32)
    poses = np.ascontiguousarray(poses, POSE)
    maps = np.ascontiguousarray(maps, GAUSSIAN2D)
    offsets = np.ascontiguousarray(offsets, np.int32)
    n = len(idx)
    sizes = np.diff(offsets)
    total = int(np.sum(sizes[idx]))
    po = np.zeros(n, POSE)
    wo = np.zeros(n, np.float32)
    mo = np.zeros(max(total, 1), GAUSSIAN2D)
    oo = np.zeros(n + 1, np.int32)
    lib().orc_copy_particles(n, _p(idx), _p(poses), _p(maps), _p(offsets), _p(po), _p(wo), _p(mo), _p(oo))
    return po, wo, mo[:total], oo


__all__ = ["SlamConfig"]
