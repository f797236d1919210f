"""Config 1's loop on the CPU oracle (oracle/config1_loop.py): the G-cap policy
and the first scans of the reference's own data."""
import numpy as np

import config1_loop as L
from phdslam.types import GAUSSIAN2D


def test_cap_keeps_heaviest_in_map_order():
    m = np.zeros(7, GAUSSIAN2D)
    m["weight"] = [0.1, 0.5, 0.2, 0.5, 0.05, 0.3, 0.9]
    m["mean"][:, 0] = np.arange(7)
    offs = np.array([0, 5, 7], np.int32)
    cm, co = L.cap_maps(m, offs, g_cap=3)
    np.testing.assert_array_equal(co, [0, 3, 5])
    # particle 0: the three heaviest of [.1 .5 .2 .5 .05] are indices 1, 3 (tie kept by index) and 2, in map order
    np.testing.assert_array_equal(cm["mean"][:3, 0], [1, 2, 3])
    np.testing.assert_array_equal(cm["mean"][3:, 0], [5, 6])


def test_cap_is_identity_below_the_cap():
    m = np.zeros(4, GAUSSIAN2D)
    offs = np.array([0, 2, 4], np.int32)
    cm, co = L.cap_maps(m, offs, g_cap=64)
    assert cm is m and co is offs


def test_config1_first_scans():
    import phdslam
    cfg = phdslam.preset(1)[0]
    assert cfg.maxRange == 50.0 and cfg.motionType == 1 and cfg.filterType == 0
    controls, scans = L.load_scans()
    assert len(scans) == 1135 and len(controls) == 1134
    state, dt, S, rs = L.run(cfg, n=64, seed=5, scans_limit=12, fast=False)
    sizes = np.diff(state[3])
    assert S == 12 and rs > 0
    assert sizes.max() <= L.G_CAP and sizes.min() > 0
    assert np.isfinite(state[1]).all()
