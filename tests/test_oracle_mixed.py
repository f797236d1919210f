"""Pin the mixed static + dynamic feature model's arithmetic (include/phd_mixed.h,
shared by the oracle and the GPU) and the oracle's orchestration against closed
forms (phdfilter.cu:205-521 pre-update / births,
:910-963 map prediction, :2323-2635 the mixed kernel, device_math.cuh:87-106,
346-363, 608-657).  The reference ships no vectors for this path: these are
float64 numpy restatements of the same equations.
"""
import ctypes
import math

import numpy as np

import pyoracle
from phdslam.scenario import mixed_config, mixed_scenario
from phdslam.types import GAUSSIAN2D, GAUSSIAN4D, MEASUREMENT, POSE


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _cfgp(c):
    return ctypes.cast(ctypes.pointer(c), ctypes.c_void_p)


def _L():
    L = pyoracle.lib()
    L.orc_det_logf.restype = ctypes.c_float
    L.orc_det_logf.argtypes = [ctypes.c_float]
    L.orc_mx_inv4.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.orc_mx_mahal4.restype = ctypes.c_float
    L.orc_mx_mahal4.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.orc_mx_ekf.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    return L


def _spd(rng, d, scale=1.0):
    a = rng.normal(0, scale, (d, d))
    return a @ a.T + np.eye(d) * 0.3 * scale


def test_det_logf_within_one_ulp():
    L = _L()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(1e-30, 1e-20, 200), rng.uniform(1e-6, 10, 2000), rng.uniform(10, 1e30, 200),
                         np.array([1.0, 2.0, 0.5, 1e-38, 3.4e38], np.float64)]).astype(np.float32)
    for x in xs:
        got = np.float32(L.orc_det_logf(float(x)))
        ref = math.log(float(x))
        ulp = np.spacing(np.float32(abs(ref))) if ref != 0 else np.float32(1e-45)
        assert abs(float(got) - ref) <= 1.0 * float(ulp), (x, got, ref)
    assert L.orc_det_logf(0.0) == -math.inf


def test_inv4_and_mahal4():
    L = _L()
    rng = np.random.default_rng(2)
    for _ in range(50):
        A = _spd(rng, 4).astype(np.float32)
        a = np.ascontiguousarray(A.ravel(order="F"))
        r = np.zeros(16, np.float32)
        L.orc_mx_inv4(_p(a), _p(r))
        Ri = r.reshape(4, 4, order="F").astype(np.float64)
        np.testing.assert_allclose(Ri @ A.astype(np.float64), np.eye(4), atol=2e-4)
        ga = np.zeros(1, GAUSSIAN4D)
        gb = np.zeros(1, GAUSSIAN4D)
        B = _spd(rng, 4).astype(np.float32)
        ga[0]["cov"] = A.ravel(order="F")
        gb[0]["cov"] = B.ravel(order="F")
        ga[0]["mean"] = rng.normal(0, 1, 4)
        gb[0]["mean"] = rng.normal(0, 1, 4)
        d = L.orc_mx_mahal4(_p(ga), _p(gb))
        S = (A.astype(np.float64) + B.astype(np.float64)) / 2
        dm = ga[0]["mean"].astype(np.float64) - gb[0]["mean"].astype(np.float64)
        ref = dm @ np.linalg.solve(S, dm)
        assert abs(d - ref) <= 1e-3 * max(1.0, ref), (d, ref)


def _ekf_ref(cfg, pose, mean, P, dims):
    dx, dy = mean[0] - pose["px"], mean[1] - pose["py"]
    r2 = dx * dx + dy * dy
    r = math.sqrt(r2)
    H = np.zeros((2, dims))
    H[0, 0], H[0, 1] = dx / r, dy / r
    H[1, 0], H[1, 1] = -dy / r2, dx / r2
    Rm = np.diag([cfg.stdRange ** 2, cfg.stdBearing ** 2])
    S = H @ P @ H.T + Rm
    K = P @ H.T @ np.linalg.inv(S)
    IKH = np.eye(dims) - K @ H
    Pu = IKH @ P @ IKH.T + K @ Rm @ K.T
    return r, math.atan2(dy, dx) - pose["ptheta"], S, K, Pu


def test_preupdate_2d_and_4d_against_kalman():
    L = _L()
    cfg = mixed_config()
    rng = np.random.default_rng(3)
    for dims in (2, 4):
        for _ in range(30):
            pose = np.zeros(1, POSE)
            pose[0]["px"], pose[0]["py"], pose[0]["ptheta"] = rng.normal(0, 1, 3)
            g = np.zeros(1, GAUSSIAN4D)
            P = _spd(rng, dims, 0.3)
            mean = rng.uniform(-10, 10, 4)
            g[0]["mean"] = mean
            if dims == 2:
                P4 = np.zeros((4, 4))
                P4[:2, :2] = P
                g[0]["cov"] = P4.ravel(order="F")
            else:
                g[0]["cov"] = P.ravel(order="F")
            out = np.zeros(32, np.float32)
            L.orc_mx_ekf(_cfgp(cfg), _p(pose), _p(g), dims, _p(out))
            Pf = (g[0]["cov"].reshape(4, 4, order="F")[:dims, :dims]).astype(np.float64)
            r, b, S, K, Pu = _ekf_ref(cfg, pose[0], g[0]["mean"].astype(np.float64), Pf, dims)
            assert abs(out[0] - r) <= 1e-5 * r
            assert abs(out[3] - np.linalg.det(S)) <= 2e-3 * abs(np.linalg.det(S))
            Sinv = np.linalg.inv(S)
            np.testing.assert_allclose(out[4:8].reshape(2, 2, order="F"), Sinv, rtol=3e-3, atol=1e-6 * np.abs(Sinv).max())
            Kg = out[8:8 + 2 * dims] if dims == 4 else out[8:12]
            Kg = Kg.reshape(dims, 2, order="F")
            np.testing.assert_allclose(Kg, K, rtol=3e-3, atol=1e-5 * np.abs(K).max())
            cu = out[16:16 + dims * dims].reshape(dims, dims, order="F")
            np.testing.assert_allclose(cu, Pu, rtol=5e-3, atol=1e-5 * np.abs(Pu).max())


def test_predict_dynamic_against_cv_model():
    cfg = mixed_config(dt=0.25, stdAxMap=0.7, stdAyMap=0.4, ps=0.95, tau=1.2, beta=3.0)
    rng = np.random.default_rng(4)
    g = np.zeros(40, GAUSSIAN4D)
    for i in range(len(g)):
        g[i]["cov"] = _spd(rng, 4, 0.5).ravel(order="F")
        g[i]["mean"] = rng.normal(0, 2, 4)
        g[i]["weight"] = rng.uniform(0.1, 1)
    out = pyoracle.predict_dynamic(cfg, g)
    dt = cfg.dt
    F = np.eye(4)
    F[0, 2] = F[1, 3] = dt
    for i in range(len(g)):
        P = g[i]["cov"].reshape(4, 4, order="F").astype(np.float64)
        Q = np.zeros((4, 4))
        for (a, v, var) in ((0, 2, cfg.stdAxMap ** 2), (1, 3, cfg.stdAyMap ** 2)):
            Q[a, a] = dt ** 4 / 4 * var
            Q[a, v] = Q[v, a] = dt ** 3 / 2 * var
            Q[v, v] = dt ** 2 * var
        Pp = F @ P @ F.T + Q
        np.testing.assert_allclose(out[i]["cov"].reshape(4, 4, order="F"), Pp, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(out[i]["mean"], F @ g[i]["mean"].astype(np.float64), rtol=1e-6, atol=1e-6)
        vm = math.hypot(g[i]["mean"][2], g[i]["mean"][3])
        pj = 1 / (1 + math.exp(cfg.beta * (cfg.tau - vm)))
        assert abs(out[i]["weight"] - pj * cfg.ps * g[i]["weight"]) <= 1e-6


def test_mixed_update_single_static_feature_closed_form():
    """One static feature observed at its predicted position (zero innovation),
    one static-labelled measurement: normaliser, weights, merge and Δ log w in
    closed form (phdfilter.cu:2387-2553)."""
    cfg = mixed_config(minSeparation=1.0)
    pose = np.zeros(1, POSE)
    sm = np.zeros(1, GAUSSIAN2D)
    sm[0]["mean"] = (6.0, 2.0)
    P = np.array([[0.2, 0.01], [0.01, 0.15]])
    sm[0]["cov"] = P.ravel(order="F")
    w = 0.8
    sm[0]["weight"] = w
    z = np.zeros(1, MEASUREMENT)
    z[0]["range"] = math.hypot(6.0, 2.0)
    z[0]["bearing"] = math.atan2(2.0, 6.0)
    z[0]["label"] = 0
    dm = np.zeros(0, GAUSSIAN4D)
    so, sof, do, dof, delta, _ = pyoracle.update_mixed(cfg, pose, sm, np.array([0, 1], np.int32), dm,
                                                        np.array([0, 0], np.int32), z)
    r, b, S, K, Pu = _ekf_ref(cfg, pose[0], np.array([6.0, 2.0]), P, 2)
    q = cfg.pd * w * math.exp(-0.0) / (2 * math.pi * math.sqrt(np.linalg.det(S)))
    eta = q + cfg.clutterDensity + cfg.birthWeight
    det_w = q / eta
    nd_w = w * (1 - cfg.pd)
    birth_w = cfg.birthWeight / eta
    assert abs(delta[0] - (math.log(eta) - cfg.pd * w)) < 2e-5
    # non-detection and detection share the mean: one merged component (+ the
    # birth, far from it in Mahalanobis terms only if its covariance is small;
    # here it merges too when within minSeparation)
    tot = sum(c["weight"] for c in so)
    assert abs(tot - (nd_w + det_w + birth_w)) < 2e-5 * max(1.0, tot)
    assert len(do) == 0 or abs(sum(c["weight"] for c in do) - cfg.birthWeight / eta * 0) < 1e-6


def test_mixed_update_scenario_properties():
    """A mixed scenario: label routing (no dynamic births from static-labelled
    measurements), map mass bounded by prior + births, out-of-range dynamic
    components dropped and out-of-range static ones kept."""
    cfg = mixed_config()
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, 4, 24, 12, 10)
    so, so_off, do, do_off, delta, margin = pyoracle.update_mixed(cfg, poses, sm, sof, dm, dof, z)
    assert np.all(np.isfinite(delta))
    for p in range(4):
        s_post = so[so_off[p]:so_off[p + 1]]
        d_post = do[do_off[p]:do_off[p + 1]]
        assert np.all(np.isfinite(s_post["weight"])) and np.all(s_post["weight"] > 0)
        assert np.all(np.isfinite(d_post["mean"]))
        n_dyn_labels = int(np.sum(z["label"] == 1))
        prior_d = dm[dof[p]:dof[p + 1]]["weight"].sum()
        assert d_post["weight"].sum() <= prior_d + n_dyn_labels + 1e-4
        # out-of-range static components are appended unchanged
        far = sm[sof[p]:sof[p + 1]]
        dx = far["mean"][:, 0] - poses[p]["px"]
        dy = far["mean"][:, 1] - poses[p]["py"]
        out1 = far[np.hypot(dx, dy) > 1.2 * cfg.maxRange]
        for g in out1:
            assert np.any(np.all(s_post["mean"] == g["mean"], axis=1))
    # labels off: both maps see every measurement, two birth terms in each normaliser
    cfg2 = mixed_config(labeledMeasurements=False)
    _, _, _, _, delta2, _ = pyoracle.update_mixed(cfg2, poses, sm, sof, dm, dof, z)
    assert np.all(np.isfinite(delta2)) and not np.allclose(delta, delta2)


def _np_eap4(T, w, comps, offs):
    """float64 restatement of exp_map_dynamic (main.cpp:369-371 ->
    gm_reduce.cpp:59-132 over Gaussian4D, LLT Mahalanobis of the averaged
    covariance): the closed-form check of orc_expected_map_dynamic."""
    allc = []
    for p in range(len(w)):
        for k in range(offs[p], offs[p + 1]):
            g = comps[k]
            allc.append((float(g["weight"]) * math.exp(float(w[p])), g["mean"].astype(np.float64),
                         g["cov"].astype(np.float64).reshape(4, 4).T))  # column-major storage
    order = sorted(range(len(allc)), key=lambda i: -allc[i][0])  # stable
    used = [False] * len(allc)
    out = []
    for oi, a in enumerate(order):
        if used[a]:
            continue
        used[a] = True
        wa, ma, ca = allc[a]
        grp = []
        for b in order[oi + 1:]:
            if used[b]:
                continue
            wb, mb, cb = allc[b]
            S = 0.5 * (ca + cb)
            x = np.linalg.solve(np.linalg.cholesky(S), ma - mb)
            if x @ x < T:
                grp.append(b)
                used[b] = True
        W = wa + sum(allc[b][0] for b in grp)
        m = (wa * ma + sum(allc[b][0] * allc[b][1] for b in grp)) / W
        C = wa * (ca + np.outer(m - ma, m - ma))
        for b in grp:
            wb, mb, cb = allc[b]
            C = C + wb * (cb + np.outer(m - mb, m - mb))
        out.append((W, m, C / W))
    return out


def test_expected_map_dynamic_closed_form():
    """orc_expected_map_dynamic (the oracle of the GPU dynamic EAP map) against
    a float64 restatement: three particles whose near-origin components merge
    into one (ties in priority broken by index) and far components that stay."""
    from phdslam.scenario import default_config
    cfg = default_config()
    cfg.minSeparation = 4.0
    rng = np.random.default_rng(3)
    n = 3
    comps = np.zeros(3 * n, GAUSSIAN4D)
    offs = np.arange(n + 1, dtype=np.int32) * 3
    for p in range(n):
        for k in range(3):
            g = comps[3 * p + k]
            base = np.array([0.0, 0.0, 1.0, -1.0]) if k == 0 else np.array([10.0 * k + p, -5.0 * k, 0.0, 0.5])
            A = rng.normal(0, 0.1, (4, 4))
            C = np.diag([0.2, 0.3, 0.5, 0.4]) + A @ A.T * 0.1
            g["mean"] = base + (rng.normal(0, 0.05, 4) if k == 0 else 0.0)
            g["cov"] = C.T.reshape(16)
            g["weight"] = rng.uniform(0.3, 1.0)
    w = np.log(np.array([0.2, 0.3, 0.5])).astype(np.float32)
    got = pyoracle.expected_map_dynamic(cfg, w, comps, offs)
    ref = _np_eap4(cfg.minSeparation, w, comps, offs)
    assert len(got) == len(ref) == 1 + 2 * n
    for g, (W, m, C) in zip(got, ref):
        assert abs(float(g["weight"]) - W) <= 1e-5 * W
        assert np.allclose(g["mean"], m, rtol=1e-5, atol=1e-5)
        assert np.allclose(g["cov"].reshape(4, 4).T, C, rtol=1e-4, atol=1e-5)
