"""Pin the oracle's update / merge / resample / RNG against closed forms.

The reference ships no golden vectors for these stages, so they
are checked here against hand-derived double-precision formulas of the same
equations (phdfilter.cu:1836-1923 EKF, :2083-2321 weights, :2739-2890 merge,
main.cpp:453-501 resample).
"""
import math

import numpy as np
import pytest

import parity
import pyoracle
from phdslam.types import GAUSSIAN2D, MEASUREMENT, POSE


def _cfg(**kw):
    import phdslam
    c = phdslam.default_config()
    c.maxRange = 50.0
    c.maxBearing = math.pi
    c.stdRange = 0.25
    c.stdBearing = 0.008727
    c.clutterRate = 20.0
    c.pd = 0.95
    c.birthWeight = 1e-4
    c.birthNoiseFactor = 1.0
    c.minFeatureWeight = 1e-6
    c.minSeparation = 10.0
    c.particleWeighting = 0
    c.featureModel = 0
    c.distanceMetric = 0
    c.filterType = 0  # PHD (the reference's default_value is CPHD, main.cpp:1009)
    for k, v in kw.items():
        setattr(c, k, v)
    c.update_clutter_density()
    return c


def _one_particle(comp_mean, comp_cov, w, z_rb):
    poses = np.zeros(1, POSE)
    maps = np.zeros(1, GAUSSIAN2D)
    maps[0]["mean"] = comp_mean
    maps[0]["cov"] = np.array(comp_cov, np.float64).reshape(2, 2).ravel(order="F")
    maps[0]["weight"] = w
    offsets = np.array([0, 1], np.int32)
    z = np.zeros(len(z_rb), MEASUREMENT)
    for i, (r, b) in enumerate(z_rb):
        z[i]["range"], z[i]["bearing"] = r, b
    return poses, maps, offsets, z


def _closed_form(cfg, mean, P, w, zr, zb):
    mx, my = mean
    r = math.hypot(mx, my)
    b = math.atan2(my, mx)
    H = np.array([[mx / r, my / r], [-my / r ** 2, mx / r ** 2]])
    R = np.diag([cfg.stdRange ** 2, cfg.stdBearing ** 2])
    S = H @ P @ H.T + R
    K = P @ H.T @ np.linalg.inv(S)
    A = np.eye(2) - K @ H
    Pp = A @ P @ A.T + K @ R @ K.T
    nu = np.array([zr - r, zb - b])
    d = nu @ np.linalg.solve(S, nu)
    q = cfg.pd * w * math.exp(-0.5 * d) / (2 * math.pi * math.sqrt(np.linalg.det(S)))
    eta = q + cfg.clutterDensity + cfg.birthWeight
    return dict(mu=np.array(mean) + K @ nu, P=Pp, q=q, eta=eta, delta=math.log(eta) - (cfg.pd * w + cfg.birthWeight))


def test_single_component_update_no_merge():
    cfg = _cfg(minSeparation=1e-12)
    P = np.array([[0.1, 0.02], [0.02, 0.15]])
    poses, maps, offs, z = _one_particle([10.0, 1.0], P, 0.8, [(10.2, 0.11)])
    out, oo, delta, margin = pyoracle.update(cfg, poses, maps, offs, z)
    cf = _closed_form(cfg, [10.0, 1.0], P, 0.8, 10.2, 0.11)
    assert oo[1] == 3  # non-detection, detection, birth — nothing merges at T ~ 0
    np.testing.assert_allclose(delta[0], cf["delta"], rtol=1e-5)
    by_w = sorted(out, key=lambda g: -g["weight"])
    wts = sorted([0.8 * (1 - cfg.pd), cf["q"] / cf["eta"], cfg.birthWeight / cf["eta"]], reverse=True)
    np.testing.assert_allclose([g["weight"] for g in by_w], wts, rtol=1e-5)
    det = [g for g in out if abs(g["weight"] - cf["q"] / cf["eta"]) < 1e-6 * cf["q"] / cf["eta"] + 1e-12][0]
    np.testing.assert_allclose(det["mean"], cf["mu"], rtol=1e-5)
    np.testing.assert_allclose(np.array(det["cov"]).reshape(2, 2, order="F"), cf["P"], rtol=2e-4, atol=1e-7)


def test_single_component_update_full_merge():
    cfg = _cfg(minSeparation=1e9)
    P = np.array([[0.1, 0.0], [0.0, 0.1]])
    poses, maps, offs, z = _one_particle([10.0, 0.0], P, 0.8, [(10.1, 0.005)])
    out, oo, delta, _ = pyoracle.update(cfg, poses, maps, offs, z)
    assert oo[1] == 1
    cf = _closed_form(cfg, [10.0, 0.0], P, 0.8, 10.1, 0.005)
    # merged weight = w(1-pd) + q/eta + beta/eta
    W = 0.8 * (1 - cfg.pd) + cf["q"] / cf["eta"] + cfg.birthWeight / cf["eta"]
    np.testing.assert_allclose(out[0]["weight"], W, rtol=1e-5)
    assert out[0]["cov"][1] == out[0]["cov"][2]  # force_symmetric_covariance


def test_out_of_range_passthrough_and_near_range_merge():
    cfg = _cfg(maxRange=20.0)
    poses = np.zeros(1, POSE)
    maps = np.zeros(3, GAUSSIAN2D)
    for i, (x, y) in enumerate([(10.0, 0.0), (22.0, 0.0), (60.0, 0.0)]):  # in, near (<=1.2*maxR), out
        maps[i]["mean"] = (x, y)
        maps[i]["cov"] = (0.1, 0.0, 0.0, 0.1)
        maps[i]["weight"] = 0.7
    offs = np.array([0, 3], np.int32)
    z = np.zeros(1, MEASUREMENT)
    z[0]["range"], z[0]["bearing"] = 5.0, 1.0
    out, oo, _, _ = pyoracle.update(cfg, poses, maps, offs, z)
    # the class-0 component is appended last, bit-identical (mergeAndCopyMaps :3304-3323)
    assert out[-1]["mean"][0] == 60.0 and out[-1]["weight"] == np.float32(0.7)
    # the near-range component survives the merge unchanged in weight
    assert any(abs(g["mean"][0] - 22.0) < 1e-5 and abs(g["weight"] - 0.7) < 1e-6 for g in out[:-1])


def test_labeled_dynamic_measurement_gets_no_detection_or_birth():
    cfg = _cfg(labeledMeasurements=True, minSeparation=1e-12)
    P = np.eye(2) * 0.1
    poses, maps, offs, z = _one_particle([10.0, 0.0], P, 0.8, [(10.0, 0.0)])
    z[0]["label"] = 1
    out, oo, delta, _ = pyoracle.update(cfg, poses, maps, offs, z)
    assert oo[1] == 1  # only the non-detection term survives the prune
    np.testing.assert_allclose(out[0]["weight"], 0.8 * (1 - cfg.pd), rtol=1e-6)


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 with 10 rounds
    np.testing.assert_array_equal(pyoracle.philox([0, 0, 0, 0], [0, 0]),
                                  np.array([0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8], np.uint32))
    np.testing.assert_array_equal(pyoracle.philox([0xffffffff] * 4, [0xffffffff] * 2),
                                  np.array([0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd], np.uint32))
    np.testing.assert_array_equal(
        pyoracle.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]),
        np.array([0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1], np.uint32))


def test_det_expf_accuracy():
    xs = np.concatenate([np.linspace(-100, 5, 20001), -np.logspace(-8, 2, 500)]).astype(np.float32)
    got = np.array([pyoracle.det_expf(x) for x in xs], np.float64)
    ref = np.exp(xs.astype(np.float64))
    rel = np.abs(got - ref) / np.maximum(ref, 1e-38)
    assert np.all(rel[ref > 1e-37] < 1.2e-7)  # correctly rounded to <= 1 float ulp


def test_shared_atan2f_correctly_rounded():
    rng = np.random.default_rng(7)
    ys = np.concatenate([rng.normal(0, 30, 3000), [0.0, -0.0, 1.0, -1.0, 1e-30]]).astype(np.float32)
    xs = np.concatenate([rng.normal(0, 30, 3000), [-1.0, -1.0, 0.0, 0.0, -5.0]]).astype(np.float32)
    got = np.array([pyoracle.atan2f(y, x) for y, x in zip(ys, xs)], np.float32)
    ref = np.arctan2(ys.astype(np.float64), xs.astype(np.float64))
    # correctly rounded: equal to the float nearest to the double result
    assert np.mean(got == ref.astype(np.float32)) > 0.9999
    assert np.all(np.abs(got.astype(np.float64) - ref) <= np.spacing(np.abs(ref).astype(np.float32)))
    assert pyoracle.atan2f(0.0, -1.0) == np.float32(np.pi) and pyoracle.atan2f(-0.0, -1.0) == -np.float32(np.pi)


def test_shared_sincosf_tanf_correctly_rounded():
    """D16: the birth means and the predict steps take sin / cos / tan from one
    double evaluation shared by the oracle and the GPU (phd_detmath.h)."""
    rng = np.random.default_rng(11)
    xs = np.concatenate([rng.uniform(-7, 7, 4000), rng.uniform(-300, 300, 500), rng.normal(0, 0.2, 500),
                         [0.0, -0.0, np.pi / 2, -np.pi / 2, np.pi, 3 * np.pi / 4, 1e-30]]).astype(np.float32)
    got = np.array([pyoracle.sincosf(x) for x in xs], np.float32)
    x64 = xs.astype(np.float64)
    for k, ref in ((0, np.sin(x64)), (1, np.cos(x64))):
        assert np.mean(got[:, k] == ref.astype(np.float32)) > 0.9999
        assert np.all(np.abs(got[:, k].astype(np.float64) - ref) <= np.spacing(np.abs(ref).astype(np.float32)))
    ts = xs[np.abs(xs) < 1.4]
    tg = np.array([pyoracle.tanf(x) for x in ts], np.float32)
    tr = np.tan(ts.astype(np.float64))
    assert np.mean(tg == tr.astype(np.float32)) > 0.9999
    assert pyoracle.sincosf(0.0) == (0.0, 1.0)


@pytest.mark.parametrize("n,seed", [(16, 1), (257, 2), (4096, 3)])
def test_resample_fixed_point_matches_faithful(n, seed):
    rng = np.random.default_rng(seed)
    w = rng.normal(0, 2, n).astype(np.float32)
    w, _ = pyoracle.normalize(w)
    u = pyoracle.resample_uniforms(n + 1, 99, seed)
    a = pyoracle.resample_faithful(w, u)
    b = pyoracle.resample_fixed(w, u[1:])
    # identical except where a stratum lands within 2^-40 of a CDF knot (det_expf vs libm expf)
    assert np.mean(a == b) >= 0.999
    assert np.all(np.diff(b) >= 0)


def test_resample_overrun_fills_argmax():
    n = 64
    w = np.full(n, math.log(0.5 / n), np.float32)  # weights sum to 0.5
    w[7] = math.log(0.9 / n)
    u = np.full(n + 1, 0.5)
    a = pyoracle.resample_faithful(w, u)
    b = pyoracle.resample_fixed(w, u[1:])
    np.testing.assert_array_equal(a, b)
    assert np.all(a[n // 2 + 1:] == 7)


def test_normalize_and_neff():
    w = np.log(np.array([0.1, 0.2, 0.3, 0.4], np.float32)) + 5
    wn, lse = pyoracle.normalize(w)
    np.testing.assert_allclose(np.exp(wn.astype(np.float64)).sum(), 1.0, rtol=1e-6)
    neff = pyoracle.neff(wn)
    np.testing.assert_allclose(neff, 1 / np.sum(np.array([0.1, 0.2, 0.3, 0.4]) ** 2) / 4, rtol=1e-5)


def test_expected_pose_and_map_estimate():
    w = np.log(np.array([0.25, 0.75], np.float32))
    poses = np.zeros(2, POSE)
    poses["px"] = [1.0, 3.0]
    poses["ptheta"] = [0.1, 0.2]
    p, mi = pyoracle.expected_pose(w, poses)
    assert mi == 1
    np.testing.assert_allclose(p["px"], 2.5, rtol=1e-6)
    np.testing.assert_allclose(p["ptheta"], 0.175, rtol=1e-6)


def test_expected_map_merges_identical_components():
    cfg = _cfg(minSeparation=5.0)
    maps = np.zeros(4, GAUSSIAN2D)
    maps["mean"] = [(0, 0), (0, 0), (10, 10), (10, 10)]
    maps["cov"] = (1, 0, 0, 1)
    maps["weight"] = 1.0
    offs = np.array([0, 2, 4], np.int32)
    w = np.log(np.array([0.5, 0.5], np.float32))
    em = pyoracle.expected_map(cfg, w, maps, offs)
    assert len(em) == 2
    np.testing.assert_allclose(sorted(em["weight"]), [1.0, 1.0], rtol=1e-6)


def _cphd_case(G=24, M=8, nmax=200, n=4, seed=7):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=G, M=M, seed=seed)
    c.maxRange = 1000.0  # every component in range: W = <1,w>
    c.birthWeight = 1e-30  # the PHD normaliser is then kappa + sum_j q
    c.maxCardinality = nmax
    return c, poses, lw, maps, offs, z


def test_cphd_poisson_equivalence():
    """With a Poisson predicted cardinality whose mean equals the in-range mass,
    the GM-CPHD update reduces to the GM-PHD update (Vo, Vo & Cantoni 2007):
    the same posterior components, and <Ψ0,p> = Σ_m log(κ + Σ_j q_jm) - pd W
    - λc + M log(λc/κ).  Pins the oracle's CPHD algebra (A12) on a closed form."""
    c, poses, lw, maps, offs, z = _cphd_case()
    c.filterType = 0
    pm, po, pd_, _ = pyoracle.update(c, poses, maps, offs, z)
    c.filterType = 1
    cm, co, cd, _, cn = pyoracle.update(c, poses, maps, offs, z, cardinality=True)
    assert np.array_equal(po, co)
    for p in range(len(poses)):
        A, B = pm[po[p]:po[p + 1]], cm[co[p]:co[p + 1]]
        ok, worst = parity.compare_maps(A, B, rtol=1e-4)
        assert ok, (p, worst)
    W = np.array([maps[offs[p]:offs[p + 1]]["weight"].astype(np.float64).sum() for p in range(len(poses))])
    lam = float(c.clutterRate)
    expect = pd_.astype(np.float64) - lam + len(z) * math.log(lam / c.clutterDensity)
    # PHD delta = Σ log η - card_pred, card_pred = pd W (+ M β ≈ 0)
    np.testing.assert_allclose(cd, expect, rtol=0, atol=2e-3 * np.maximum(1, np.abs(expect)).max())
    # posterior cardinality: a normalised distribution
    lse = np.log(np.exp(cn - cn.max(1, keepdims=True)).sum(1)) + cn.max(1)
    np.testing.assert_allclose(lse, 0.0, atol=1e-9)


def test_cphd_cardinality_shifts_with_detections():
    """Posterior cardinality mean grows when measurements match components and
    shrinks under pure clutter (missed detections), relative to the prior."""
    c, poses, lw, maps, offs, z = _cphd_case(G=16, M=6, nmax=100, n=2, seed=3)
    c.filterType = 1
    _, _, _, _, cn_det = pyoracle.update(c, poses, maps, offs, z, cardinality=True)
    zc = z.copy()
    zc["bearing"] = zc["bearing"] + 2.5  # far from every component: clutter only
    _, _, _, _, cn_clut = pyoracle.update(c, poses, maps, offs, zc, cardinality=True)
    k = np.arange(cn_det.shape[1])
    mean_det = (np.exp(cn_det) * k).sum(1)
    mean_clut = (np.exp(cn_clut) * k).sum(1)
    W = np.array([maps[offs[p]:offs[p + 1]]["weight"].astype(np.float64).sum() for p in range(len(poses))])
    assert np.all(mean_clut < mean_det)
    assert np.all(np.abs(mean_clut - W * (1 - c.pd)) < 0.05 * W)  # thinned prior when nothing is detected


@pytest.mark.parametrize("cid,n,G", [(2, 32, 256), (3, 16, 512), (5, 8, 1024)])
def test_expected_map_cells_equals_plain_greedy(cid, n, G):
    """orc_expected_map_cells (the EAP greedy with distance tests restricted to
    touching lattice cells, the oracle used at config 3's 2.1 M components)
    returns exactly the plain O(K^2) greedy's map (gm_reduce.cpp:59-132): same
    components, same emission order, same bits."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n, G=G, M=16)
    w = np.log(np.random.default_rng(cid).dirichlet(np.ones(n))).astype(np.float32)
    a = pyoracle.expected_map(c, w, maps, offs)
    b = pyoracle.expected_map(c, w, maps, offs, cells=True)
    assert len(a) > 0 and a.tobytes() == b.tobytes()


def test_expected_map_cells_exact_for_nearly_singular_covariances():
    """The cell-restricted EAP oracle stays exact when covariances are nearly
    rank-1 (condition 1e5 .. 1e8), whose float LLT distance is least accurate:
    partners along the thick axis at the merge distance, along the thin axis at
    a few thin-axis sigmas, and both."""
    import phdslam
    rng = np.random.default_rng(5)
    c = phdslam.default_config()
    c.minSeparation = 10.0
    T = c.minSeparation
    n, per = 16, 64
    K = n * per
    maps = np.zeros(K, GAUSSIAN2D)
    maps["weight"] = rng.uniform(0.2, 1.0, K).astype(np.float32)
    for s in range(0, K, 4):
        th = rng.uniform(0, np.pi)
        u = np.array([np.cos(th), np.sin(th)])
        v = np.array([-np.sin(th), np.cos(th)])
        l1 = rng.uniform(0.05, 0.2)
        l2 = l1 * 10.0 ** rng.uniform(-8, -5)
        P = l1 * np.outer(u, u) + l2 * np.outer(v, v)
        mu = rng.uniform(-15, 15, 2)
        offs4 = [0.0 * u, np.sqrt(T * l1) * rng.uniform(0.95, 1.05) * u,
                 np.sqrt(T * l2) * rng.uniform(0.3, 30.0) * v,
                 np.sqrt(T * l1) * rng.uniform(0.9, 1.1) * u + np.sqrt(T * l2) * rng.uniform(0.3, 3.0) * v]
        for q in range(4):
            maps["mean"][s + q] = (mu + offs4[q]).astype(np.float32)
            maps["cov"][s + q] = np.array([P[0, 0], P[1, 0], P[0, 1], P[1, 1]], np.float32)
    offs = (np.arange(n + 1) * per).astype(np.int32)
    w = np.log(rng.dirichlet(np.ones(n))).astype(np.float32)
    a = pyoracle.expected_map(c, w, maps, offs)
    b = pyoracle.expected_map(c, w, maps, offs, cells=True)
    assert K // 4 < len(a) < K and a.tobytes() == b.tobytes()
