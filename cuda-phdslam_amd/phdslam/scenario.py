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
