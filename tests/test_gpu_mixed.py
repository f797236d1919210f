"""GPU parity of the mixed static + dynamic feature model (feature_model 2,
SURVEY.md §8(f) rank 4): the HIP path (phd_mixed.hip, through the C-ABI)
against the CPU oracle (orc_update_mixed / orc_predict_dynamic).

Tolerances as tests/test_gpu_parity.py: fp32 fields within 1e-5 relative;
maps compared in order (both sides emit merged components in the greedy's
selection order, then the static out-of-range components); particles whose
oracle decided a prune / merge / range class within 1e-4 of its threshold may
differ only in the components those decisions touch (compared as multisets);
birth means use the platform cosf / sinf (≤ 1 ulp apart), everything else is
shared arithmetic (include/phd_mixed.h).
"""
import numpy as np
import pytest

import parity
import pyoracle
from phdslam.scenario import mixed_config, mixed_scenario
from phdslam.types import GAUSSIAN4D

pytestmark = pytest.mark.gpu


def _filter(cfg, n, cap=128, dcap=64, M=32, K=4096, **kw):
    import phdslam
    f = phdslam.PHDFilter(n, cfg, map_capacity=cap, max_measurements=M, candidate_capacity=K,
                          survivor_capacity=256, **kw)
    f.set_seed(77)
    f.enable_dynamic(dcap)
    return f


def _cmp4(A, B, rtol=parity.RTOL):
    """Dynamic maps in order: weight, mean (scaled), covariance (scaled by the matrix)."""
    if len(A) != len(B):
        return False, float("inf")
    if len(A) == 0:
        return True, 0.0
    ok_w = parity.close(A["weight"], B["weight"], rtol, floor=1e-12)
    ms = np.maximum(np.abs(A["mean"]).max(1, keepdims=True), 1.0)
    ok_m = parity.close(A["mean"], B["mean"], rtol, scale=ms)
    cs = np.abs(A["cov"]).max(1, keepdims=True)
    ok_c = parity.close(A["cov"], B["cov"], 5 * rtol, scale=cs)
    worst = max(parity._rel(A["weight"], B["weight"]), parity._rel(A["mean"], B["mean"], ms),
                parity._rel(A["cov"], B["cov"], cs))
    return bool(ok_w.all() and ok_m.all() and ok_c.all()), worst


def _check_mixed(cfg, poses, sm, sof, dm, dof, z, label, **cap):
    n = len(poses)
    f = _filter(cfg, n, **cap)
    f.load(poses, np.zeros(n, np.float32), sm, sof)
    f.load_dynamic(dm, dof)
    f.update(z)
    f.check_errors()
    _, glw, gs, gso = f.export()
    gd, gdo = f.export_dynamic()
    f.close()
    os_, oso, od, odo, odelta, margin = pyoracle.update_mixed(cfg, poses, sm, sof, dm, dof, z)
    ncls, npm = pyoracle.near_counts()
    bad = []
    worst = 0.0
    compared = 0
    for p in range(n):
        if ncls[p]:
            continue
        compared += 1
        A, B = os_[oso[p]:oso[p + 1]], gs[gso[p]:gso[p + 1]]
        C, D = od[odo[p]:odo[p + 1]], gd[gdo[p]:gdo[p + 1]]
        if not parity.close([glw[p]], [odelta[p]], 1e-5, floor=1e-5).all():
            bad.append((p, "delta", float(glw[p]), float(odelta[p])))
        if npm[p] == 0:
            ok, w = parity.compare_maps(A, B) if len(A) == len(B) else (False, float("inf"))
            ok4, w4 = _cmp4(C, D)
            worst = max(worst, w, w4)
            if not ok:
                bad.append((p, "static", len(A), len(B), w))
            if not ok4:
                bad.append((p, "dynamic", len(C), len(D), w4))
        else:
            ua, ub = parity.unmatched(A, B)
            if max(ua, ub) > 3 * npm[p]:
                bad.append((p, "near static", ua, ub, int(npm[p])))
    assert compared >= max(1, n - max(2, n // 10)), f"{label}: only {compared}/{n} particles compared"
    assert not bad, f"{label}: {bad[:6]}"
    return worst, compared


@pytest.mark.parametrize("labeled", [True, False])
def test_mixed_update_matches_oracle(gpu, labeled):
    cfg = mixed_config(labeledMeasurements=labeled)
    data = mixed_scenario(cfg, 24, 40, 16, 12)
    worst, compared = _check_mixed(cfg, *data, f"mixed labeled={labeled}")
    assert worst < 1e-5


def test_mixed_update_larger_maps(gpu):
    """More components than threads per workgroup (multi-chunk classification,
    candidate and merge passes) and a candidate list of several thousand."""
    cfg = mixed_config()
    data = mixed_scenario(cfg, 6, 300, 90, 24, seed=991)
    _check_mixed(cfg, *data, "mixed large", cap=512, dcap=192, K=1536)


def test_mixed_empty_maps_and_no_dynamic(gpu):
    """Empty dynamic maps: only births enter the dynamic map; empty static maps too."""
    cfg = mixed_config()
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, 8, 12, 6, 10, seed=5)
    dof0 = np.zeros_like(dof)
    _check_mixed(cfg, poses, sm, sof, dm[:0], dof0, z, "no dynamic")
    sof0 = np.zeros_like(sof)
    _check_mixed(cfg, poses, sm[:0], sof0, dm, dof, z, "no static")


def test_predict_dynamic_matches_oracle(gpu):
    cfg = mixed_config(dt=0.2)
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, 10, 8, 20, 6, seed=8)
    f = _filter(cfg, 10)
    f.load(poses, np.zeros(10, np.float32), sm, sof)
    f.load_dynamic(dm, dof)
    f.predict_dynamic()
    f.predict_dynamic()
    g, go = f.export_dynamic()
    f.close()
    o = pyoracle.predict_dynamic(cfg, pyoracle.predict_dynamic(cfg, dm))
    assert np.array_equal(go, dof)
    for fld in ("weight", "mean", "cov"):
        assert np.array_equal(g[fld], o[fld]), fld  # shared arithmetic: bit for bit


def test_mixed_sequence_with_resample(gpu):
    """Three filter steps (CV predict with host noise + predictMapMixed, mixed
    update, normalise, resample with given parents) against the oracle run on
    the same inputs; dynamic maps follow their particles through the resample."""
    import phdslam
    cfg = mixed_config()
    cfg.motionType = 0
    n = 12
    poses, sm, sof, dm, dof, z0 = mixed_scenario(cfg, n, 30, 10, 10, seed=21)
    f = _filter(cfg, n)
    lw = np.full(n, -np.log(n), np.float32)
    f.load(poses, lw, sm, sof)
    f.load_dynamic(dm, dof)
    o_poses, o_lw, o_sm, o_sof, o_dm, o_dof = poses.copy(), lw.copy(), sm, sof, dm, dof
    rng = np.random.default_rng(3)
    for step in range(3):
        noise = pyoracle.noise_cv(cfg, n, 11, step)
        f.predict_cv(noise, step)
        o_poses = pyoracle.predict_cv(cfg, o_poses, noise)
        o_dm = pyoracle.predict_dynamic(cfg, o_dm)
        z = z0.copy()
        z["range"] += rng.normal(0, 0.05, len(z)).astype(np.float32)
        f.update(z)
        f.check_errors()
        o_sm, o_sof, o_dm, o_dof, odelta, _ = pyoracle.update_mixed(cfg, o_poses, o_sm, o_sof, o_dm, o_dof, z)
        ncls, npm = pyoracle.near_counts()
        assert ncls.sum() == 0 and npm.sum() == 0, "scenario has near-threshold decisions: pick another seed"
        o_lw = o_lw + odelta
        gp, glw, gs, gso = f.export()
        gd, gdo = f.export_dynamic()
        assert parity.close(glw, o_lw, 1e-5, floor=1e-5).all()
        assert np.array_equal(gso, o_sof) and np.array_equal(gdo, o_dof)
        ok, _ = _cmp4(gd, o_dm)
        assert ok
        for p in range(n):
            ok2, _ = parity.compare_maps(o_sm[o_sof[p]:o_sof[p + 1]], gs[gso[p]:gso[p + 1]])
            assert ok2, (step, p)
        # resample (device draws): maps of both kinds follow their parents
        f.normalize()
        parents = f.resample(step=step)
        o_poses = gp[parents]
        o_lw = np.full(n, -np.log(n), np.float32)
        o_sm, o_sof = _remap(gs, gso, parents)
        o_dm, o_dof = _remap(gd, gdo, parents)
        gp2, glw2, gs2, gso2 = f.export()
        gd2, gdo2 = f.export_dynamic()
        assert np.array_equal(gso2, o_sof) and np.array_equal(gdo2, o_dof)
        for fld in ("weight", "mean", "cov"):
            assert np.array_equal(gd2[fld], o_dm[fld]) and np.array_equal(gs2[fld], o_sm[fld])
    f.close()


def _remap(maps, offs, parents):
    parts = [maps[offs[p]:offs[p + 1]] for p in parents]
    out = np.concatenate(parts) if parts else maps[:0]
    o = np.zeros(len(parents) + 1, np.int32)
    o[1:] = np.cumsum([len(x) for x in parts])
    return out, o


@pytest.mark.parametrize("steps", [0, 2])
def test_expected_map_dynamic_matches_oracle(gpu, steps):
    """exp_map_dynamic (main.cpp:369-371): the GPU EAP map of the dynamic maps
    (phd_expected_map_dynamic, 4-D LLT distance, greedy in priority order) equals
    the oracle's (orc_expected_map_dynamic) on the exported store, in emission
    order — on the loaded maps and after mixed updates with normalised weights."""
    cfg = mixed_config()
    n = 48
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, n, 40, 24, 24)
    f = _filter(cfg, n)
    lw = np.log(np.random.default_rng(5).dirichlet(np.ones(n))).astype(np.float32)
    f.load(poses, lw, sm, sof)
    f.load_dynamic(dm, dof)
    for k in range(steps):
        f.update(z)
        f.normalize()
    _, gw, _, _ = f.export(with_maps=False)
    gd, gdo = f.export_dynamic()
    eap = f.expected_map_dynamic()
    f.close()
    ref = pyoracle.expected_map_dynamic(cfg, gw, gd, gdo)
    assert len(eap) > 0
    ok, worst = _cmp4(eap, ref)
    assert ok, f"dynamic EAP differs (worst {worst}); {len(eap)} vs {len(ref)} components"
    tot = float(np.sum(np.exp(gw.astype(np.float64)) * np.array(
        [gd["weight"][gdo[p]:gdo[p + 1]].astype(np.float64).sum() for p in range(n)])))
    assert abs(eap["weight"].astype(np.float64).sum() - tot) <= 1e-4 * tot


def test_mixed_rejects_unsupported(gpu):
    import phdslam
    cfg = mixed_config(filterType=1)
    poses, sm, sof, dm, dof, z = mixed_scenario(cfg, 4, 6, 4, 5, seed=2)
    f = _filter(cfg, 4)
    f.load(poses, np.zeros(4, np.float32), sm, sof)
    f.load_dynamic(dm, dof)
    with pytest.raises(phdslam.PHDError):
        f.update(z)
    f.close()
    cfg = mixed_config(featureModel=1)
    f = _filter(cfg, 4)
    f.load(poses, np.zeros(4, np.float32), sm, sof)
    with pytest.raises(phdslam.PHDError):
        f.update(z)
    f.close()
