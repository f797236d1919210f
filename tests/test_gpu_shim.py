"""The C++ drop-in surface (include/phdfilter.h, phdfilter_shim.cpp) against the oracle.

tests/shim_harness (built by cuda-phdslam_amd/build.py from tests/shim_harness.cpp)
calls setDeviceConfig / initRandomNumberGenerators / phdPredict / addBirths /
phdUpdateSynth on a SynthSLAM exactly as the reference's run_synth does
(main.cpp:1178-1312); the particle set it returns is compared with the oracle's
statement of the same calls: maps as multisets (1e-5), log-weights after the
normalisation phdUpdateSynth applies (phdfilter.cu:3735-3755), CPHD
cardinalities (phdfilter.cu.bak:2700-2706), n_predict_particles duplication
(phdfilter.cu:1185-1238).
"""
import os
import subprocess

import numpy as np
import pytest

import parity
import pyoracle
from phdslam.types import GAUSSIAN2D, GAUSSIAN4D, MEASUREMENT, POSE

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "tests", "shim_harness")
SEED = 0x1234ABCD


def _run(tmp_path, ops, cfg, poses, lw, maps, offs, z=None, zb=None, control=(0.0, 0.0), dyn=None):
    if not os.path.exists(HARNESS):
        pytest.fail("tests/shim_harness is not built (python cuda-phdslam_amd/build.py)")
    n = len(poses)
    z = np.zeros(0, MEASUREMENT) if z is None else z
    zb = np.zeros(0, MEASUREMENT) if zb is None else zb
    sizes = np.diff(np.asarray(offs)).astype(np.int32)
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(np.array([ops, n, len(z), len(zb)], np.int32).tobytes())
        f.write(np.uint64(SEED).tobytes())
        f.write(bytes(cfg))
        f.write(np.array([control[1], control[0]], np.float32).tobytes())  # AckermanControl {alpha, v_encoder}
        f.write(np.ascontiguousarray(poses, POSE).tobytes())
        f.write(np.ascontiguousarray(lw, np.float32).tobytes())
        f.write(sizes.tobytes())
        f.write(np.ascontiguousarray(maps, GAUSSIAN2D).tobytes())
        f.write(np.ascontiguousarray(z, MEASUREMENT).tobytes())
        f.write(np.ascontiguousarray(zb, MEASUREMENT).tobytes())
        if dyn is not None:  # feature_model 2: dynamic maps
            f.write(np.diff(np.asarray(dyn[1])).astype(np.int32).tobytes())
            f.write(np.ascontiguousarray(dyn[0], GAUSSIAN4D).tobytes())
    out = tmp_path / "out.bin"
    r = subprocess.run([HARNESS, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    b = out.read_bytes()
    nn, K = np.frombuffer(b, np.int32, 2)
    o = 8
    gp = np.frombuffer(b, POSE, nn, o).copy(); o += nn * POSE.itemsize
    gw = np.frombuffer(b, np.float32, nn, o).copy(); o += 4 * nn
    gs = np.frombuffer(b, np.int32, nn, o).copy(); o += 4 * nn
    gm = np.frombuffer(b, GAUSSIAN2D, int(gs.sum()), o).copy(); o += GAUSSIAN2D.itemsize * int(gs.sum())
    gc = np.frombuffer(b, np.float32, nn * K, o).reshape(nn, K).copy(); o += 4 * nn * K
    go = np.concatenate([[0], np.cumsum(gs)]).astype(np.int64)
    if dyn is not None:
        ds = np.frombuffer(b, np.int32, nn, o).copy(); o += 4 * nn
        dm = np.frombuffer(b, GAUSSIAN4D, int(ds.sum()), o).copy()
        do = np.concatenate([[0], np.cumsum(ds)]).astype(np.int64)
        return gp, gw, gm, go, gc, dm, do
    return gp, gw, gm, go, gc


def _compare_update(label, cfg, poses, lw, maps, offs, z, gw, gm, go):
    om, ooffs, odelta, _ = pyoracle.update(cfg, poses, maps, offs, z)
    ncls, npm = pyoracle.near_counts()
    compared = 0
    for p in range(len(poses)):
        if ncls[p] or npm[p]:
            continue
        A, B = om[ooffs[p]:ooffs[p + 1]], gm[go[p]:go[p + 1]]
        assert len(A) == len(B), (label, p, len(A), len(B))
        ok, worst = parity.compare_maps(A, B)
        assert ok, (label, p, worst)
        compared += 1
    assert compared >= 0.9 * len(poses), f"{label}: only {compared} particles compared"
    if ncls.sum() == 0:  # normalised log-weights (a near range class moves η of one particle)
        ow, _ = pyoracle.normalize((lw + odelta).astype(np.float32))
        assert parity.close(gw, ow, 1e-5, floor=1e-5).all(), f"{label}: {np.max(np.abs(gw - ow))}"
    return compared


def test_shim_update_synth_phd(gpu, tmp_path):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=48, G=128, M=24)
    gp, gw, gm, go, gc = _run(tmp_path, 4, c, poses, lw, maps, offs, z)
    assert gp.tobytes() == np.ascontiguousarray(poses, POSE).tobytes()
    assert gc.shape[1] == 0  # PHD: cardinalities untouched (empty)
    _compare_update("shim phd", c, poses, lw, maps, offs, z, gw, gm, go)


def test_shim_update_synth_cphd_cardinalities(gpu, tmp_path):
    """filter_type 1: phdUpdateSynth fills particles.cardinalities with the
    posterior log cardinality distribution (maxCardinality + 1 entries)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=16, G=200, M=40)
    c.maxCardinality = 300
    gp, gw, gm, go, gc = _run(tmp_path, 4, c, poses, lw, maps, offs, z)
    _compare_update("shim cphd", c, poses, lw, maps, offs, z, gw, gm, go)
    _, _, _, _, cn = pyoracle.update(c, poses, maps, offs, z, cardinality=True)
    assert gc.shape == cn.shape == (16, 301)
    sig = cn > -60.0
    assert parity.close(gc[sig], cn[sig], 1e-5, floor=1e-4).all()


def test_shim_births_then_update_cphd(gpu, tmp_path):
    """addBirths(particles, ZPrev) before phdUpdateSynth (the CPHD birth
    model, phdfilter.cu.bak:738-870) equals the oracle's add_births + update."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=16, G=128, M=32)
    zb = z[::3].copy()
    gp, gw, gm, go, gc = _run(tmp_path, 2 | 4, c, poses, lw, maps, offs, z, zb)
    bm, boffs = pyoracle.add_births(c, poses, maps, offs, zb)
    _compare_update("shim births+cphd", c, poses, lw, bm, boffs, z, gw, gm, go)


@pytest.mark.parametrize("cid", [2, 3])
def test_shim_predict_n_predict_particles(gpu, tmp_path, cid):
    """nPredictParticles = 3: every particle spawns 3 children that share its map
    (and cardinalities) with weight w - log 3, each predicted with its own noise
    draw (Philox stream PREDICT, counter = child index, step 0)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=20, G=16, M=4)
    c.nPredictParticles = 3
    poses["vx"] = 1.0
    poses["vtheta"] = 0.1
    u = (2.0, 0.05)
    gp, gw, gm, go, gc = _run(tmp_path, 1, c, poses, lw, maps, offs, control=u)
    assert len(gp) == 60
    parent = np.repeat(np.arange(20), 3)
    c1 = c.copy()
    c1.nPredictParticles = 1
    if cid == 3:
        op = pyoracle.predict_cv(c1, poses[parent], pyoracle.noise_cv(c1, 60, SEED, 0))
    else:
        op = pyoracle.predict_ackerman(c1, poses[parent], u[0], u[1], pyoracle.noise_ackerman(c1, 60, SEED, 0))
    for k in POSE.names:
        assert parity.close(gp[k], op[k], 1e-5, scale=1.0).all(), k
    assert parity.close(gw, lw[parent].astype(np.float64) - np.log(3.0), 1e-6, floor=1e-6).all()
    for j in range(60):
        i = parent[j]
        assert gm[go[j]:go[j + 1]].tobytes() == maps[offs[i]:offs[i + 1]].tobytes()


def test_shim_mixed_predict_and_update(gpu, tmp_path):
    """feature_model 2 through the drop-in surface: phdPredict predicts the
    dynamic maps (predictMapMixed, phdfilter.cu:1241-1242) and phdUpdateSynth
    runs the mixed update on maps_static + maps_dynamic (phdfilter.cu:3449-3462,
    3703-3726); both against the oracle."""
    from phdslam.scenario import mixed_config, mixed_scenario
    cfg = mixed_config()
    cfg.motionType = 0
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, 16, 30, 12, 10, seed=31)
    lw = np.full(16, -np.log(16), np.float32)
    # predict only: dynamic maps predicted, static maps untouched
    gp, gw, gm, go, gc, gdm, gdo = _run(tmp_path, 1, cfg, poses, lw, sm, sof, dyn=(dm, dof))
    od = pyoracle.predict_dynamic(cfg, dm)
    assert np.array_equal(gdo, dof)
    for fld in ("weight", "mean", "cov"):
        assert np.array_equal(gdm[fld], od[fld]), fld
    assert gm.tobytes() == np.ascontiguousarray(sm, GAUSSIAN2D).tobytes()
    # update only
    gp, gw, gm, go, gc, gdm, gdo = _run(tmp_path, 4, cfg, poses, lw, sm, sof, z, dyn=(dm, dof))
    os_, oso, odm, odo, odelta, _ = pyoracle.update_mixed(cfg, poses, sm, sof, dm, dof, z)
    ncls, npm = pyoracle.near_counts()
    assert ncls.sum() == 0 and npm.sum() == 0
    assert np.array_equal(go, oso) and np.array_equal(gdo, odo)
    for p in range(16):
        ok, w = parity.compare_maps(os_[oso[p]:oso[p + 1]], gm[go[p]:go[p + 1]])
        assert ok, (p, w)
    for fld, tol in (("weight", 1e-5), ("mean", 1e-5), ("cov", 5e-5)):
        assert parity.close(gdm[fld], odm[fld], tol, floor=1e-6).all(), fld
    ow, _ = pyoracle.normalize((lw + odelta).astype(np.float32))
    assert parity.close(gw, ow, 1e-5, floor=1e-5).all()
