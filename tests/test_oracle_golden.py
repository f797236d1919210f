"""Pin the CPU oracle against the reference's own Python models (golden vectors).

tests/golden/models_golden.json was produced by tests/golden/make_golden.py from
/root/reference/python/{RangeBearingMeasurementModel,AckermanMotionModel}.py.
The oracle computes in float (like the reference's CUDA path) and the Python
models in double, so agreement is to float precision.
"""
import json
import math
import os

import numpy as np
import pytest

import pyoracle
from phdslam.types import POSE, MEASUREMENT

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "models_golden.json")


@pytest.fixture(scope="module")
def golden(built):
    with open(GOLDEN) as f:
        return json.load(f)


def _cfg(**kw):
    import phdslam
    c = phdslam.default_config()
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_wrap_angle(golden):
    g = golden["wrap_angle"]
    for a, expect in zip(g["in"], g["out"]):
        got = pyoracle.wrap_angle(a)
        # float input rounding: compare against wrap of the float-rounded input
        assert abs(got - expect) <= 2e-6 * max(1.0, abs(a)), (a, got, expect)


def test_measurement_h(golden):
    for c in golden["measurement_h"]["cases"]:
        pose = np.zeros(1, POSE)[0]
        pose["px"], pose["py"], pose["ptheta"] = c["pose"]
        got = pyoracle.measure(pose, *c["feature"])
        r, b = c["z"]
        assert abs(got[0] - r) <= 1e-5 * max(1.0, r)
        assert abs(got[1] - b) <= 2e-5


def test_inverse_measurement_birth_mean(golden):
    cfg = _cfg(stdRange=0.25, stdBearing=0.008727, birthNoiseFactor=1.0, birthWeight=1e-4)
    for c in golden["measurement_hinv"]["cases"]:
        pose = np.zeros(1, POSE)[0]
        pose["px"], pose["py"], pose["ptheta"] = c["pose"]
        z = np.zeros(1, MEASUREMENT)[0]
        z["range"], z["bearing"] = c["z"]
        g = pyoracle.birth(cfg, pose, z)
        fx, fy = c["feature"]
        assert abs(g["mean"][0] - fx) <= 1e-5 * max(1.0, abs(fx)) + 2e-5
        assert abs(g["mean"][1] - fy) <= 1e-5 * max(1.0, abs(fy)) + 2e-5
        # birth covariance = J R J^T with J = d(x,y)/d(r,b) (phdfilter.cu:3480-3500)
        r, b = c["z"]
        th = c["pose"][2] + b
        J = np.array([[math.cos(th), -r * math.sin(th)], [math.sin(th), r * math.cos(th)]])
        R = np.diag([0.25 ** 2, 0.008727 ** 2])
        P = J @ R @ J.T
        np.testing.assert_allclose(np.array(g["cov"]).reshape(2, 2, order="F"), P, rtol=2e-4, atol=1e-7)
        assert abs(g["weight"] - math.log(1e-4)) < 1e-6


def test_ackerman_predict(golden):
    p = golden["ackerman"]["params"]
    for c in golden["ackerman"]["cases"]:
        cfg = _cfg(l=p["l"], h=p["h"], a=p["a"], b=p["b"], dt=c["dt"], subdividePredict=1, nPredictParticles=1)
        pose = np.zeros(1, POSE)
        pose[0]["px"], pose[0]["py"], pose[0]["ptheta"] = c["pose"]
        noise = np.zeros(1, pyoracle.ACKERMAN_NOISE)
        out = pyoracle.predict_ackerman(cfg, pose, c["v_encoder"], c["alpha"], noise)[0]
        ex, ey, et = c["out"]
        assert abs(out["px"] - ex) <= 1e-5 * max(1.0, abs(ex)) + 1e-5, (c, out)
        assert abs(out["py"] - ey) <= 1e-5 * max(1.0, abs(ey)) + 1e-5, (c, out)
        dth = (out["ptheta"] - et + math.pi) % (2 * math.pi) - math.pi
        assert abs(dth) <= 2e-5, (c, out)
        assert out["vx"] == 0 and out["vy"] == 0 and out["vtheta"] == 0


def test_ackerman_survey_example(golden):
    """SURVEY.md §8(c) worked example: pose 0, v=2.77796, alpha=-0.186915, dt=.1."""
    c = golden["ackerman"]["cases"][0]
    np.testing.assert_allclose(c["out"], [0.28203613, -0.06678198, -0.03533438], rtol=1e-6)


def test_config1_fixture_shape():
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1_data.npz"))
    assert d["controls"].shape == (1134, 2)
    assert len(d["meas_offsets"]) == 1136
    steps = np.diff(d["meas_offsets"])
    assert 70 <= steps.mean() <= 120  # ≈96 measurements per step
    assert d["meas"][:, 0].max() < 51.0


def test_cv_predict(golden):
    """A2 pinned by the reference's python/ConstantVelocityMotionModel.py:13-29
    (noise-free step; the oracle's noise terms are zero): planar pose + velocities."""
    for c in golden["cv"]["cases"]:
        cfg = _cfg(dt=c["dt"], subdividePredict=1, nPredictParticles=1)
        pose = np.zeros(1, POSE)
        for k, v in zip(POSE.names, c["pose"]):
            pose[0][k] = v
        noise = np.zeros(1, pyoracle.CV_NOISE)
        out = pyoracle.predict_cv(cfg, pose, noise)[0]
        for k, e in zip(POSE.names, c["out"]):
            if k == "ptheta":
                d = (out[k] - e + math.pi) % (2 * math.pi) - math.pi
                assert abs(d) <= 2e-5, (c, out)
            else:
                assert abs(out[k] - e) <= 1e-5 * max(1.0, abs(e)) + 1e-5, (k, c, out)


def test_cv_dataset_fixture_shape():
    """The first 40 steps of the reference's CV dataset (matlab/measurements_synth_cv.txt)."""
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "config3_cv_data.npz"))
    assert len(d["meas_offsets"]) == 41
    assert d["meas"].shape == (d["meas_offsets"][-1], 2) and np.isfinite(d["meas"]).all()
    # noisy simulated data: ranges up to ~11 (a few slightly negative), bearings up to ~pi + 0.03
    assert d["meas"][:, 0].max() < 12.0 and (np.abs(d["meas"][:, 1]) < np.pi + 0.1).all()
