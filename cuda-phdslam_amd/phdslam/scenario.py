"""Synthetic replay scenarios for BASELINE.json configs (host-side, via libphdslam.so).

`preset(id)` returns the SlamConfig and shape of config `id` (1..5, numbering
as in SURVEY.md §8(d)); `scenario(...)` generates the deterministic prior /
measurement set the bench replays (cuda-phdslam_amd/csrc/phd_synth.cpp).
"""
import ctypes

import numpy as np

from . import _lib
from .types import GAUSSIAN2D, MEASUREMENT, POSE, SlamConfig

SEED_BASE = 20261015


def preset(config_id):
    cfg = SlamConfig()
    n, G, M = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    df = ctypes.c_float()
    _lib.check(_lib.lib().phd_synth_preset(int(config_id), ctypes.byref(cfg), ctypes.byref(n), ctypes.byref(G),
                                           ctypes.byref(M), ctypes.byref(df)), "phd_synth_preset")
    return cfg, n.value, G.value, M.value, df.value


def scenario(cfg, n, G, M, detect_frac=0.75, seed=SEED_BASE):
    poses = np.zeros(n, POSE)
    lw = np.zeros(n, np.float32)
    maps = np.zeros(n * G, GAUSSIAN2D)
    offsets = np.zeros(n + 1, np.int32)
    z = np.zeros(M, MEASUREMENT)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    _lib.check(_lib.lib().phd_synth_scenario(ctypes.byref(cfg), n, G, M, float(detect_frac), int(seed), p(poses),
                                             p(lw), p(maps), p(offsets), p(z)), "phd_synth_scenario")
    return poses, lw, maps, offsets, z


def config_scenario(config_id, n=None, G=None, M=None, seed=None):
    """Preset + scenario of config `id`, optionally with a smaller shape (parity tests)."""
    cfg, n0, G0, M0, df = preset(config_id)
    n = n0 if n is None else n
    G = G0 if G is None else G
    M = M0 if M is None else M
    seed = SEED_BASE + config_id if seed is None else seed
    return (cfg,) + scenario(cfg, n, G, M, df, seed)


def bench_capacities(config_id, G, M, wide=False):
    """Per-particle capacities bench.py runs config `config_id` with (and the
    parity test of the benched configuration, tests/test_gpu_parity.py):
    map G + 2M + 64 (64-aligned); candidates G + 5M = 832 at config 3 (its step
    places M births after the G prior components: the oracle's largest list on
    every 8th particle of the replay scenario is 805, 675 without births) or
    G + 3M + 16 (config 2; config 4, whose PHD update adds M births: G + 4M +
    16), 1800 at config 5; survivors 3M + 32 (config 3: 4M + 32, its births'
    own detections; 640 at config 5).
    wide=True: the roomier fallback bench.py switches to when the tight set
    overflows on a scenario (status bits after the warm-up)."""
    cap = (G + 2 * M + 64 + 63) // 64 * 64
    if wide:
        return dict(map_capacity=cap + 128, max_measurements=M, candidate_capacity=G + 4 * M + 128,
                    survivor_capacity=max(256, 4 * M) + 128)
    # (config 4 is the PHD update of config 3's shape: its M births join the
    # candidates, so G + 4M + 16)
    kcap = 1800 if config_id == 5 else G + 4 * M + 16 if config_id == 4 else G + 5 * M if config_id == 3 else \
        G + 3 * M + 16
    return dict(map_capacity=cap, max_measurements=M, candidate_capacity=kcap,
                survivor_capacity=640 if config_id == 5 else 4 * M + 32 if config_id == 3 else 3 * M + 32)


def load_config(path):
    """cfg/config.cfg loader (loadConfig, main.cpp:956-1073). Returns (SlamConfig, data_directory)."""
    cfg = SlamConfig()
    buf = ctypes.create_string_buffer(4096)
    rc = _lib.lib().phd_config_load(str(path).encode(), ctypes.byref(cfg), buf, 4096)
    _lib.check(rc, f"phd_config_load({path})")
    return cfg, buf.value.decode()


def default_config():
    cfg = SlamConfig()
    _lib.check(_lib.lib().phd_config_defaults(ctypes.byref(cfg)), "phd_config_defaults")
    return cfg


def mixed_config(**kw):
    """Defaults (phd_config_defaults) set up for the mixed static + dynamic
    feature model (feature_model 2, PHD, labelled measurements)."""
    import math
    c = default_config()
    c.featureModel = 2
    c.filterType = 0
    c.particleWeighting = 0
    c.distanceMetric = 0
    c.maxRange = 20.0
    c.minRange = 0.0
    c.maxBearing = math.pi
    c.stdRange = 0.3
    c.stdBearing = 0.02
    c.pd = 0.9
    c.clutterRate = 5.0
    c.birthWeight = 0.05
    c.birthNoiseFactor = 1.5
    c.minFeatureWeight = 1e-5
    c.minSeparation = 4.0
    c.covVxBirth = 1.0
    c.covVyBirth = 1.0
    c.stdAxMap = 0.5
    c.stdAyMap = 0.5
    c.ps = 0.98
    c.tau = 1.5
    c.beta = 4.0
    c.dt = 0.1
    c.labeledMeasurements = True
    for k, v in kw.items():
        setattr(c, k, v)
    c.update_clutter_density()
    return c


def mixed_scenario(cfg, n, Gs, Gd, M, seed=SEED_BASE + 100, pose_jitter=0.3):
    """Deterministic mixed-model input: n poses near the origin, per particle Gs
    static (Gaussian2D) and Gd dynamic (Gaussian4D) components spread over the
    sensor range (a few nearly in range / out of range), and M labelled
    measurements: noisy detections of particle 0's features plus clutter."""
    from .types import GAUSSIAN4D
    rng = np.random.default_rng(seed)
    R = float(cfg.maxRange)
    poses = np.zeros(n, POSE)
    poses["px"] = rng.normal(0, pose_jitter, n)
    poses["py"] = rng.normal(0, pose_jitter, n)
    poses["ptheta"] = rng.normal(0, 0.02, n)
    base_s = rng.uniform(-1.15 * R, 1.15 * R, (Gs, 2))
    base_d = rng.uniform(-1.0 * R, 1.0 * R, (Gd, 2))
    vel_d = rng.normal(0, 1.5, (Gd, 2))
    smaps = np.zeros(n * Gs, GAUSSIAN2D)
    dmaps = np.zeros(n * Gd, GAUSSIAN4D)
    for p in range(n):
        s = smaps[p * Gs:(p + 1) * Gs]
        s["mean"] = base_s + rng.normal(0, 0.2, (Gs, 2))
        a = rng.uniform(0.05, 0.3, Gs)
        b = rng.uniform(0.05, 0.3, Gs)
        cxy = rng.uniform(-0.02, 0.02, Gs)
        s["cov"] = np.stack([a, cxy, cxy, b], axis=1)
        s["weight"] = rng.uniform(0.2, 1.0, Gs)
        d = dmaps[p * Gd:(p + 1) * Gd]
        d["mean"] = np.concatenate([base_d + rng.normal(0, 0.2, (Gd, 2)), vel_d + rng.normal(0, 0.1, (Gd, 2))], 1)
        cov = np.zeros((Gd, 4, 4))
        cov[:, 0, 0] = rng.uniform(0.05, 0.3, Gd)
        cov[:, 1, 1] = rng.uniform(0.05, 0.3, Gd)
        cov[:, 2, 2] = rng.uniform(0.2, 1.0, Gd)
        cov[:, 3, 3] = rng.uniform(0.2, 1.0, Gd)
        cov[:, 0, 2] = cov[:, 2, 0] = rng.uniform(-0.02, 0.02, Gd)
        cov[:, 1, 3] = cov[:, 3, 1] = rng.uniform(-0.02, 0.02, Gd)
        d["cov"] = cov.transpose(0, 2, 1).reshape(Gd, 16)
        d["weight"] = rng.uniform(0.2, 1.0, Gd)
    soffs = np.arange(n + 1, dtype=np.int32) * Gs
    doffs = np.arange(n + 1, dtype=np.int32) * Gd
    z = np.zeros(M, MEASUREMENT)
    k = 0
    feats = [(m, 0) for m in base_s] + [(m, 1) for m in base_d]
    order = rng.permutation(len(feats))
    for i in order:
        if k >= int(0.7 * M):
            break
        (fx, fy), lab = feats[i]
        r = float(np.hypot(fx, fy))
        if r > R or r < 0.5:
            continue
        z[k]["range"] = r + rng.normal(0, cfg.stdRange)
        z[k]["bearing"] = np.arctan2(fy, fx) + rng.normal(0, cfg.stdBearing)
        z[k]["label"] = lab
        k += 1
    while k < M:
        z[k]["range"] = rng.uniform(1.0, R)
        z[k]["bearing"] = rng.uniform(-np.pi, np.pi)
        z[k]["label"] = int(rng.integers(0, 2))
        k += 1
    return poses, smaps, soffs, dmaps, doffs, z
