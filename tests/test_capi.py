"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol
include/*.h declares, struct layouts match the reference, and the host-only
entry points (config loader, scenario generator) behave.  No GPU compute."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(phd_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(built):
    import phdslam
    L = phdslam.lib()
    names = sorted(set(_declared("phd_capi.h")) | set(_declared("phd_io.h")))
    assert len(names) >= 34
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the ctypes binding covers them all
    from phdslam._lib import SIGNATURES
    assert set(names) <= set(SIGNATURES), set(names) - set(SIGNATURES)


def test_cxx_dropin_symbols_exported(built):
    """include/phdfilter.h re-exports the reference's C++ API (phdfilter.h:10-34)."""
    import subprocess
    so = os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "libphdslam.so")
    out = subprocess.run(["nm", "-DC", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    for sym in ["phdPredict(SynthSLAM&, ...)",
                "phdUpdateSynth(SynthSLAM&, std::vector<RangeBearingMeasurement, std::allocator<RangeBearingMeasurement> >)",
                "setDeviceConfig(SlamConfig const&)", "initRandomNumberGenerators()",
                "recoverSlamState(SynthSLAM&, ConstantVelocityState&, std::vector<float, std::allocator<float> >&)"]:
        assert sym in out, sym


def test_struct_layouts(built):
    from phdslam import types as T
    assert T.GAUSSIAN2D.itemsize == 28
    assert T.POSE.itemsize == 24
    assert T.MEASUREMENT.itemsize == 12
    assert T.ACKERMAN_CONTROL.itemsize == 8
    assert ctypes.sizeof(T.SlamConfig) == 324
    off = {f: getattr(T.SlamConfig, f).offset for f, _ in T.SlamConfig._fields_}
    assert off["clutterDensity"] == 108 and off["pd"] == 112 and off["n_particles"] == 196
    assert off["labeledMeasurements"] == 292 and off["l"] == 296 and off["saveAllMaps"] == 320


def test_version_and_device_count(built):
    import phdslam
    assert b"gfx950" in phdslam.lib().phd_version()
    assert phdslam.device_count() >= 0


def test_error_codes_without_context(built):
    import phdslam
    L = phdslam.lib()
    assert L.phd_update(None) == phdslam._lib.PHD_E_ARG
    assert b"null" in L.phd_last_error()


def test_config_defaults_match_loadconfig(built):
    import phdslam
    c = phdslam.default_config()
    # main.cpp:961-1048 defaults
    assert c.motionType == 1 and abs(c.maxRange - 20) < 1e-6 and abs(c.pd - 0.98) < 1e-7
    assert c.n_particles == 512 and c.filterType == 1 and c.particleWeighting == 1
    np.testing.assert_allclose(c.clutterDensity, np.float32(15) / (np.float32(2) * np.float32(np.pi) * 20), rtol=1e-6)


SYNTH_CFG = """
# synthetic-scenario configuration (same key surface as cfg/config.cfg)
motion_type = 1
max_range = 50.000000
max_bearing = 3.141593
std_range = 0.250000
std_bearing = 0.008727
clutter_rate = 20.000000
pd = 0.950000
l = 1.415000
h = 0.380000
a = 1.890000
b = 0.500000
std_encoder = 1.000000
std_alpha = 0.034907
filter_type = 0
feature_model = 0 # 0-static ; 1-dynamic ; 2-mixed
particle_weighting = 0
n_particles = 200
birth_weight = 0.0001
min_separation = 10
min_feature_weight=0.000001
labeled_measurements = 0
initial_vz = 3
data_directory = /tmp/synth/
"""


def test_config_loader(built, tmp_path):
    import phdslam
    p = tmp_path / "c.cfg"
    p.write_text(SYNTH_CFG)
    c, d = phdslam.load_config(p)
    assert d == "/tmp/synth/"
    assert c.motionType == 1 and c.n_particles == 200 and c.featureModel == 0 and c.filterType == 0
    assert abs(c.maxRange - 50) < 1e-6 and abs(c.minFeatureWeight - 1e-6) < 1e-12
    assert abs(c.vz0 - 3) < 1e-6  # bound to vz0 (reference binds vy0, main.cpp:970)
    np.testing.assert_allclose(c.clutterDensity, np.float32(20) / (np.float32(2) * np.float32(3.141593) * 50),
                               rtol=1e-6)
    # unknown keys are rejected like boost::program_options does
    q = tmp_path / "bad.cfg"
    q.write_text("no_such_key = 1\n")
    with pytest.raises(phdslam.PHDError):
        phdslam.load_config(q)


def test_reference_config_file_parses(built):
    path = "/root/reference/cfg/config.cfg"
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box)")
    import phdslam
    c, d = phdslam.load_config(path)
    assert c.motionType == 1 and c.n_particles == 200 and abs(c.maxRange - 15) < 1e-6
    assert abs(c.minSeparation - 10) < 1e-6 and c.filterType == 0


def test_synth_scenario_deterministic(built):
    import phdslam
    a = phdslam.config_scenario(2, n=8, G=16, M=12)
    b = phdslam.config_scenario(2, n=8, G=16, M=12)
    for x, y in zip(a[1:], b[1:]):
        assert x.tobytes() == y.tobytes()
    cfg, poses, lw, maps, offs, z = a
    assert len(maps) == 8 * 16 and offs[-1] == 128 and len(z) == 12
    r = np.hypot(maps["mean"][:, 0], maps["mean"][:, 1])
    assert r.max() < 50.0
    np.testing.assert_allclose(lw, -np.log(8), rtol=1e-6)


@pytest.mark.parametrize("src,defines", [
    ("phd_kernels.hip", ["-DPHD_STAMPS"]),
    ("phd_kernels.hip", ["-DPHD_XK=3"]),
    ("phd_kernels.hip", ["-DPHD_XK=10", "-DPHD_STAMPS"]),
    ("phd_capi.hip", ["-DPHD_STAMPS", "-DPHD_STAMP_PART_A"]),
    ("phd_eap.hip", ["-DPHD_EAP_DEBUG"]),
])
def test_diagnostic_builds_compile(src, defines):
    """The diagnostic variants (stamps, ablations, EAP round timing: compile-time
    -D flags of build.py's build_stamps_lib / build_ablation, never the shipped
    library) still compile — host and gfx950 device, syntax and semantics."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not present")
    csrc = os.path.join(REPO, "cuda-phdslam_amd", "csrc")
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", *defines,
                        "-I" + os.path.join(REPO, "include"), "-I" + csrc, "-fsyntax-only", os.path.join(csrc, src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
