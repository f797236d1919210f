"""phdslam — MI355X-native RB-PHD-SLAM filter (host side of libphdslam.so).

The compute path is the HIP library; this package is the Python mirror of the
reference's operator surface (src/phdfilter.h) used by tests and bench.py.
"""
from . import types  # noqa: F401
from ._lib import PHDError, device_count, lib  # noqa: F401
from .filter import PHDFilter  # noqa: F401
from .scenario import config_scenario, default_config, load_config, preset, scenario  # noqa: F401
from .types import GAUSSIAN2D, MEASUREMENT, POSE, SlamConfig  # noqa: F401
