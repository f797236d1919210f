"""Reference data formats: the loaders of src/main.cpp:147-245
and the writeLog writer of src/main.cpp:848-954, host-only entry points of
libphdslam.so (include/phd_io.h).  No GPU.

Golden anchors: the reference's shipped data files (python/controls_synth.txt,
python/measurements_synth.txt) as committed in tests/golden/config1_data.npz,
and the writer's byte format = std::ostream default float formatting, which
Python's "%g" reproduces (6 significant digits)."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "config1_data.npz")
REF_PY = "/root/reference/python"


def _g(x):
    """std::ostream << float (default flags, precision 6) == printf %g."""
    return "%g" % x


def test_controls_reference_format(built, tmp_path):
    """loadControls: header line skipped, 'v_encoder alpha' per line (main.cpp:176-185)."""
    from phdslam import io
    p = tmp_path / "controls.txt"
    p.write_text("v alpha\n1.5 0.25\n-2 -0.125\n3e-1 7\n")
    u = io.load_controls(p)
    assert len(u) == 3
    np.testing.assert_array_equal(u["v_encoder"], np.float32([1.5, -2, 0.3]))
    np.testing.assert_array_equal(u["alpha"], np.float32([0.25, -0.125, 7]))
    # no trailing garbage element for the read at EOF (the reference pushes one)
    p.write_text("v alpha\n1 2\n\n\n")
    assert len(io.load_controls(p)) == 1


def test_measurements_reference_format(built, tmp_path):
    """loadMeasurements + parseMeasurements: header skipped, one step per line of
    (range bearing label) triples; empty lines are empty steps (main.cpp:192-245)."""
    from phdslam import io
    p = tmp_path / "meas.txt"
    p.write_text("header\n1 0.5 0 2 -0.5 1\n\n3 0.25 0 \n")
    z, offs = io.load_measurements(p)
    assert list(offs) == [0, 2, 2, 3]
    np.testing.assert_array_equal(z["range"], np.float32([1, 2, 3]))
    np.testing.assert_array_equal(z["bearing"], np.float32([0.5, -0.5, 0.25]))
    assert list(z["label"]) == [0, 1, 0]


def test_shipped_synth_data_matches_golden(built, tmp_path):
    """The reference's own data files (comma-separated controls, range/bearing pairs,
    no header) load to the committed config-1 fixture."""
    from phdslam import io
    d = np.load(GOLDEN)
    if os.path.isdir(REF_PY):
        cpath, mpath = os.path.join(REF_PY, "controls_synth.txt"), os.path.join(REF_PY, "measurements_synth.txt")
    else:  # rewrite the fixture in the shipped formats
        cpath, mpath = tmp_path / "c.txt", tmp_path / "m.txt"
        with open(cpath, "w") as f:
            for v, a in d["controls"].astype(np.float64):
                f.write(f"{float(v)!r}, {float(a)!r}\n")
        with open(mpath, "w") as f:
            mo = d["meas_offsets"]
            for s in range(len(mo) - 1):
                f.write(" ".join(repr(float(x)) for x in d["meas"][mo[s]:mo[s + 1]].ravel()) + "\n")
    u = io.load_controls(cpath, flags=io.COMMAS)
    np.testing.assert_array_equal(np.stack([u["v_encoder"], u["alpha"]], 1), d["controls"])
    z, offs = io.load_measurements(mpath, flags=io.PAIRS)
    mo = d["meas_offsets"]
    steps = len(offs) - 1
    assert steps >= 1134
    np.testing.assert_array_equal(offs, mo[:steps + 1].astype(np.int32))
    np.testing.assert_array_equal(np.stack([z["range"], z["bearing"]], 1), d["meas"][:offs[-1]])
    assert (z["label"] == 0).all()


def test_timestamps(built, tmp_path):
    from phdslam import io
    p = tmp_path / "t.txt"
    p.write_text("0.0\n0.1\n0.25\n")
    np.testing.assert_array_equal(io.load_timestamps(p), [0.0, 0.1, 0.25])


def test_comment_lines(built, tmp_path):
    from phdslam import io
    p = tmp_path / "c.txt"
    p.write_text("% matlab header\n1, 2\n# another\n3, 4\n")
    u = io.load_controls(p, flags=io.COMMAS | io.COMMENTS)
    np.testing.assert_array_equal(u["v_encoder"], [1, 3])


def _state(n, K, rng):
    from phdslam.types import GAUSSIAN2D, POSE
    poses = np.zeros(n, POSE)
    for f in POSE.names:
        poses[f] = rng.normal(size=n).astype(np.float32)
    m = np.zeros(K, GAUSSIAN2D)
    m["weight"] = rng.uniform(0.1, 2, K)
    m["mean"] = rng.normal(0, 30, (K, 2))
    m["cov"] = rng.uniform(0.01, 1, (K, 4))
    lw = np.log(rng.dirichlet(np.ones(n))).astype(np.float32)
    return poses, m, lw


def test_state_log_format(built, tmp_path):
    """writeLog's seven lines, byte for byte (main.cpp:860-952)."""
    from phdslam import io
    rng = np.random.default_rng(3)
    n, K = 5, 4
    poses, m, lw = _state(n, K, rng)
    ep = poses[2]
    idx = np.array([0, 0, 2, 3, 3], np.int32)
    path = io.write_state_log(tmp_path, 7, ep, m, lw, poses, idx, max_cardinality=3)
    assert os.path.basename(path) == "state_estimate00007.log"
    lines = open(path).read().split("\n")
    want = [
        "".join(_g(float(ep[f])) + " " for f in ("px", "py", "ptheta", "vx", "vy", "vtheta")),
        "".join(_g(float(g["weight"])) + " " + "".join(_g(float(x)) + " " for x in g["mean"]) +
                "".join(_g(float(x)) + " " for x in g["cov"]) for g in m),
        "",
        "".join(_g(float(x)) + " " for x in lw),
        "".join("".join(_g(float(p[f])) + " " for f in ("px", "py", "ptheta", "vx", "vy", "vtheta")) for p in poses),
        "".join(f"{i} " for i in idx),
        "0 0 0 0 ",
        "",
    ]
    assert lines == want
    # appended, like the reference's fstream::app
    io.write_state_log(tmp_path, 7, ep, m, lw, poses, idx, max_cardinality=3)
    assert len(open(path).read().split("\n")) == 2 * 7 + 1


def test_state_log_roundtrip_and_shotgun(built, tmp_path):
    """read_state_log parses what writeLog wrote; at t = 0 the particle lines repeat
    n_predict_particles times (main.cpp:906-935); CPHD writes the cardinality line."""
    from phdslam import io
    rng = np.random.default_rng(4)
    n, K = 6, 9
    poses, m, lw = _state(n, K, rng)
    cn = np.log(rng.dirichlet(np.ones(11))).astype(np.float32)
    path = io.write_state_log(tmp_path, 0, poses[0], m, lw, poses, None, cn=cn, max_cardinality=10, filter_type=1,
                              n_predict_particles=3)
    r = io.read_state_log(path)
    assert len(r["log_weights"]) == 3 * n and len(r["poses"]) == 3 * n
    np.testing.assert_allclose(r["log_weights"][:n], lw, rtol=1e-5)
    np.testing.assert_allclose(r["map_mean"], m["mean"], rtol=1e-5)
    np.testing.assert_allclose(r["map_cov"], m["cov"], rtol=1e-5)
    np.testing.assert_allclose(r["cardinality"], cn, rtol=1e-5)
    assert list(r["resample_idx"]) == list(range(n))


def test_io_errors(built, tmp_path):
    from phdslam import PHDError, io
    with pytest.raises(PHDError):
        io.load_controls(tmp_path / "missing.txt")
    with pytest.raises(ValueError):
        io.write_state_log(tmp_path, 0, np.zeros(1, io.POSE), [], [0.0], np.zeros(2, io.POSE))
