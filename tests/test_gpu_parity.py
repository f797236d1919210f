"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Tolerances: fp32 fields |a-b| <= 1e-5 * max(|a|,|b|) (with a
matrix/mean scale floor for near-zero entries); maps compared as multisets;
prune/merge/classification decisions must agree exactly except where the oracle
itself decided within MARGIN (1e-4 relative) of a threshold: such prune / merge
decisions may change only the components they touch (the rest of the particle
is still compared), a near range classification skips the particle (counted,
bounded).  Resample indices are bit-exact.
"""
import os

import numpy as np
import pytest

import parity
import pyoracle
from phdslam.types import GAUSSIAN2D, MEASUREMENT, POSE

pytestmark = pytest.mark.gpu
MARGIN = 1e-4


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _filter(cfg, n, **cap):
    import phdslam
    f = phdslam.PHDFilter(n, cfg, **cap)
    f.set_seed(1234)
    return f


def _check_update(cfg, poses, lw, maps, offs, z, label, max_skip_frac=0.02, threads=0, sample=None, form=0,
                  with_form=False, rtol=parity.RTOL, births=False, elementwise=False, **cap):
    """Update through the C-ABI vs the oracle.  Particles without near-threshold
    decisions are compared whole (map multiset, log-weight).  Particles whose
    oracle has prune / merge decisions within MARGIN of their threshold are still
    compared component by component: every component those decisions do not
    touch must match (at most 3 per near decision may differ), and their
    log-weights must match (prune / merge never moves Δ log w).  Only a near
    range classification (which moves η, hence every weight) skips a particle;
    those are counted and bounded by max_skip_frac.  threads: the update's
    workgroup size (0 = the context's automatic choice).  sample: compare only
    these particles (the GPU updates all of them).  Returns (worst relative
    deviation, particles compared, filter's update_threads()).  births: the
    step's births (CPHD: the scan's inverse measurements placed after the map
    before the update, phd_set_step_births) — run as the bench runs them (replay,
    phd_predict_update without a predict) against the oracle's add_births ->
    update.  elementwise: assert SURVEY §8(d)'s per-element measure on every
    entry that is not a cancellation entry (_compare_with_oracle)."""
    n = len(poses)
    f = _filter(cfg, n, **cap)
    if form:
        f.set_update_form(form)
    if threads:
        f.set_update_threads(threads)
    f.load(poses, lw, maps, offs)
    if births:
        f.set_step_births(1)
        f.set_replay(True)
        f.set_measurements(z)
        f.predict_update(None, 0, do_predict=False)
    else:
        f.set_step_births(0)
        f.update(z)
    f.check_errors()
    gp, glw, gmaps, goffs = f.export()
    ut = f.update_threads()
    split = f.update_form()
    f.close()
    if births:
        maps, offs = pyoracle.add_births(cfg, poses, maps, offs, z)
    worst, compared = _compare_with_oracle(cfg, poses, lw, maps, offs, z, (glw, gmaps, goffs), label, max_skip_frac,
                                           sample, rtol, elementwise)
    # poses untouched by the update
    assert gp.tobytes() == np.ascontiguousarray(poses, POSE).tobytes()
    if with_form:
        return worst, compared, ut, split
    return worst, compared, ut


def _subset(poses, lw, maps, offs, sample):
    """The particles `sample` of a CSR particle set (the oracle's input)."""
    sample = np.asarray(sample)
    sizes = np.diff(offs)[sample]
    so = np.zeros(len(sample) + 1, np.int32)
    so[1:] = np.cumsum(sizes)
    sm = np.concatenate([maps[offs[p]:offs[p + 1]] for p in sample]) if len(sample) else maps[:0]
    return poses[sample], lw[sample], sm, so


def _record_elementwise(entry):
    """Append one comparison's per-element figures to the parity record (JSON
    lines; PHD_PARITY_RECORD, default gpurun_out/parity_elementwise.jsonl —
    scripts/parity_record.py folds it into profiles/)."""
    import json
    path = os.environ.get("PHD_PARITY_RECORD", os.path.join(REPO, "gpurun_out", "parity_elementwise.jsonl"))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as fh:
            fh.write(json.dumps(entry) + "\n")
    except OSError:
        pass  # (a read-only tree: the figures are still printed)


def _compare_with_oracle(cfg, poses, lw, maps, offs, z, gpu, label, max_skip_frac=0.02, sample=None,
                         rtol=parity.RTOL, elementwise=False):
    """elementwise: besides the scaled contract (parity.compare_maps), every
    entry that is not a cancellation entry (weights, covariance diagonals, mean
    coordinates with |x| >= 1; parity.noncancellation_mask) must meet SURVEY
    §8(d)'s per-element |a - b| <= 1e-5 max(|a|, |b|) itself.  The figures of
    every call are appended to the parity record (_record_elementwise)."""
    glw, gmaps, goffs = gpu
    n = len(poses)
    sample = np.arange(n) if sample is None else np.asarray(sample)
    sp, slw, sm, so = _subset(poses, lw, maps, offs, sample)
    om, ooffs, odelta, margin = pyoracle.update(cfg, sp, sm, so, z)
    ncls, npm = pyoracle.near_counts()
    ns = len(sample)
    skip = ncls > 0
    assert skip.sum() <= max(2, max_skip_frac * ns), \
        f"{label}: too many near-threshold classifications ({skip.sum()}/{ns})"
    worst = 0.0
    # SURVEY §8(d)'s per-element measure, reported beside the contract's (parity.elementwise):
    # [worst, beyond, elements, beyond among non-cancellation entries, worst among them]
    strict = [0.0, 0, 0, 0, 0.0]
    bad = []
    compared = 0
    for i, p in enumerate(sample):
        if skip[i]:
            continue
        A = om[ooffs[i]:ooffs[i + 1]]
        B = gmaps[goffs[p]:goffs[p + 1]]
        compared += 1
        if npm[i] == 0:
            if len(A) != len(B):
                bad.append((int(p), "size", len(A), len(B)))
                continue
            ok, w = parity.compare_maps(A, B, rtol, strict)
            worst = max(worst, w)
            if not ok:
                bad.append((int(p), "values", w))
        else:
            ua, ub = parity.unmatched(A, B, rtol)
            if max(ua, ub) > 3 * npm[i]:
                bad.append((int(p), "near-threshold components", ua, ub, int(npm[i])))
    print(f"{label}: worst scaled deviation {worst:.3g} (contract rtol {rtol:g}); per-element worst "
          f"{strict[0]:.3g}, {strict[1]} of {strict[2]} elements beyond 1e-5 max(|a|,|b|), "
          f"{strict[3]} of them not cancellation entries (worst {strict[4]:.3g})")
    ow = (slw + odelta).astype(np.float32)
    g = glw[sample]
    lref = np.maximum(np.abs(g[~skip]).astype(np.float64), np.abs(ow[~skip]).astype(np.float64))
    ldev = np.abs(g[~skip].astype(np.float64) - ow[~skip].astype(np.float64))
    _record_elementwise(dict(label=label, particles=int(ns), compared=int(compared), skipped=int(skip.sum()),
                             near_prune_merge=int(np.sum(npm > 0)), contract_worst=float(worst), rtol=float(rtol),
                             elem_worst=float(strict[0]), elem_beyond=int(strict[1]), elements=int(strict[2]),
                             noncancel_beyond=int(strict[3]), noncancel_worst=float(strict[4]),
                             logw_elem_worst=float(np.max(ldev / np.maximum(lref, 1e-30))) if ldev.size else 0.0,
                             logw_elem_beyond=int(np.sum(ldev > 1e-5 * lref + 1e-30)), elementwise_asserted=elementwise))
    assert not bad, f"{label}: {bad[:5]}"
    if elementwise:
        assert strict[3] == 0, (f"{label}: {strict[3]} weights / covariance diagonals / means with |x| >= 1 beyond "
                                f"1e-5 of themselves (worst {strict[4]:.3g})")
    # log-weights: lw + delta (no normalisation yet); the tolerance scales with
    # the addends (delta is rounded to float before the float sum, so when
    # delta ~ -lw the sum carries an absolute error of an ulp of |delta|)
    mag = np.maximum(np.abs(slw), np.abs(odelta))
    ok = parity.close(g[~skip], ow[~skip], 1e-5, floor=1e-5, scale=mag[~skip])
    assert ok.all(), f"{label}: log-weight mismatch max {np.max(np.abs(g - ow))}"
    return worst, compared


def test_update_tiny_closed_form_case(gpu):
    cfg = pyoracle  # noqa: F841 (keep import order)
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=4, G=3, M=2)
    _, compared, _ = _check_update(c, poses, lw, maps, offs, z, "tiny")
    assert compared >= 3, f"only {compared} of 4 particles compared"


@pytest.mark.parametrize("form", [1, 2])
@pytest.mark.parametrize("threads", [256, 512, 1024])
@pytest.mark.parametrize("n,G,M", [(64, 64, 32), (128, 256, 32), (32, 512, 64), (16, 300, 100)])
def test_update_matches_oracle(gpu, n, G, M, threads, form):
    """Every compiled instance of the PHD update — one fused launch (form 1) and
    split into part A + part C (form 2), at 256 / 512 / 1024 threads — is
    compared, not only the one the occupancy model picks."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=G, M=M)
    nt = threads
    worst, _, ut = _check_update(c, poses, lw, maps, offs, z, f"n{n}G{G}M{M}t{threads}f{form}", threads=nt,
                                 form=form, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024)
    if nt:
        assert ut[0] == nt
    print(f"worst relative deviation {worst:.3g}")


def _check_cardinality(c, n, poses, lw, maps, offs, z, threads=0, sample=None, **cap):
    f = _filter(c, n, **cap)
    if threads:
        f.set_update_threads(threads)
    f.load(poses, lw, maps, offs)
    f.update(z)
    cn_gpu = f.cardinality_distribution().astype(np.float64)
    f.close()
    sample = np.arange(n) if sample is None else np.asarray(sample)
    sp, _, sm, so = _subset(poses, lw, maps, offs, sample)
    _, _, _, _, cn = pyoracle.update(c, sp, sm, so, z, cardinality=True)
    cn_gpu = cn_gpu[sample]
    sig = cn > -60.0  # probabilities above ~1e-26
    ok = parity.close(cn_gpu[sig], cn[sig], 1e-5, floor=1e-4)
    assert ok.all(), f"cardinality mismatch max {np.max(np.abs(cn_gpu[sig] - cn[sig]))}"
    assert np.all(cn_gpu[~sig] < -50.0)


@pytest.mark.parametrize("threads", [256, 512, 1024])
@pytest.mark.parametrize("n,G,M,nmax", [(8, 64, 16, 127), (16, 200, 40, 300), (64, 512, 64, 1023),
                                        (8, 300, 100, 400), (4, 256, 127, 300)])
def test_cphd_update_matches_oracle(gpu, n, G, M, nmax, threads):
    """A12: CPHD update (config 3 semantics) against the oracle's direct
    formulas: posterior maps, Δ log w = <Ψ0,p>, and the log cardinality
    distribution.  M = 100 and 127 take the two-coefficients-per-lane branch of
    the CPHD terms (M > 64); every compiled workgroup size is compared."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=n, G=G, M=M)
    assert c.filterType == 1
    c.maxCardinality = nmax
    nt = threads
    cap = dict(map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024, max_measurements=M)
    _, _, ut = _check_update(c, poses, lw, maps, offs, z, f"cphd n{n}G{G}M{M}t{threads}", threads=nt, **cap)
    if nt:
        assert ut[0] == nt
    _check_cardinality(c, n, poses, lw, maps, offs, z, threads=nt, **cap)


@pytest.mark.parametrize("nmax_over", [0, 2, 12])
def test_cphd_cardinality_series_near_lambda(gpu, nmax_over):
    """max_cardinality close to the predicted mean cardinality λ = Σ w: the
    Poisson series' tail is not negligible, the Chernoff check of the closed
    form log S(K) = λ fails and the terms sum the truncated series (DESIGN D9)
    — against the oracle's direct sums (scphd_cpu.cpp cphd_terms)."""
    import phdslam
    n, G, M = 8, 96, 24
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=n, G=G, M=M)
    lam = float(np.max([maps[offs[p]:offs[p + 1]]["weight"].sum() for p in range(n)]))
    c.maxCardinality = int(np.ceil(lam)) + nmax_over
    cap = dict(map_capacity=256, candidate_capacity=512, survivor_capacity=256, max_measurements=M)
    _check_update(c, poses, lw, maps, offs, z, f"cphd series nmax {c.maxCardinality} lambda {lam:.1f}", **cap)
    _check_cardinality(c, n, poses, lw, maps, offs, z, **cap)


@pytest.mark.parametrize("threads,births", [(0, True), (256, True), (0, False)])
def test_cphd_update_bench_configuration(gpu, threads, births):
    """The configuration behind the bench number: config 3 at its full shape
    (4096 particles x 512 x 64, CV + CPHD) with bench.py's capacities
    (phdslam.scenario.bench_capacities: map 704, candidates 832, survivors 288,
    M 64) and, as the bench's step runs it, the step's 64 births after each
    particle's 512 prior components (births=False: the update alone) — the
    256-thread part A / part C code objects, several rounds of resident
    workgroups with the high-priority tail and the last-written-first XCD order
    active.  threads 0: the automatic choice must be that instance.  256
    particles (every 16th) are compared with the oracle (maps, log-weights,
    cardinality distributions)."""
    import phdslam
    from phdslam.scenario import bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
    n, G, M = len(poses), 512, 64
    assert n == 4096 and len(z) == M and c.filterType == 1
    cap = bench_capacities(3, G, M)
    assert cap == dict(map_capacity=704, max_measurements=64, candidate_capacity=832, survivor_capacity=288)
    sample = np.arange(0, n, 16)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    _, compared, ut = _check_update(c, poses, lw, maps, offs, z, "bench config 3", threads=threads, sample=sample,
                                    births=births, elementwise=True, **cap)
    assert ut[0] == 256, f"update instance {ut}"
    assert ut[2] < n, "all workgroups resident: the multi-round path is not exercised"
    assert compared >= 250
    if births:
        maps, offs = pyoracle.add_births(c, poses, maps, offs, z)
    _check_cardinality(c, n, poses, lw, maps, offs, z, threads=threads, sample=sample, **cap)


def test_cphd_update_bench_configuration_every_particle(gpu):
    """The bench configuration (config 3, 4096 x 512 x 64 with the step's 64
    births, bench capacities, the automatic 256-thread instance) with EVERY
    particle compared with the oracle (maps and log-weights; the oracle runs on
    OpenMP), not a sample: no particle of the benched update escapes the check."""
    import phdslam
    from phdslam.scenario import bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
    n, G, M = len(poses), 512, 64
    cap = bench_capacities(3, G, M)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    _, compared, ut = _check_update(c, poses, lw, maps, offs, z, "bench config 3 (every particle)", births=True,
                                    elementwise=True, **cap)
    assert ut[0] == 256, f"update instance {ut}"
    assert compared >= n - max(2, int(0.02 * n)), f"{compared} of {n} compared"


@pytest.mark.parametrize("cid,n,nt,split,every,rtol", [(2, 1024, None, None, 1, 1e-5), (4, 4096, None, None, 1, 1e-5),
                                                       (5, 8192, 512, True, 1, 1e-5)])
def test_phd_update_bench_configuration(gpu, cid, n, nt, split, every, rtol):
    """The PHD configurations behind the bench lines, at their benched per-GPU
    shapes with bench.py's capacities (phdslam.scenario.bench_capacities) and
    the automatic workgroup size: config 2 (1024 x 256 x 32, candidates
    G+3M+16 = 368, survivors 128; the fused or the split form, whichever the
    occupancy model picks — both at six 256-thread workgroups per CU when the
    fused kernel fits 80 VGPRs), config 4's per-GPU shard as SURVEY §8(d)
    defines config 4 (Ackerman + static PHD, 4096 x 512 x 64) and config 5's
    per-GPU shard (8192 x 1024 x 128 at Pd 0.7, candidates 1800, survivors 640:
    the split update, part A + part C at 512 threads).  Every `every`-th particle
    is compared with the oracle (every = 1: all of them; maps and log-weights),
    at 1e-5.  (Config 5's sweep over all 8192 particles, ~7.3 M components, once
    needed 2e-5: particle 1025 merged a birth whose mean came from libm's cosf
    on the CPU and ocml's on the GPU, an ulp apart; both now take sin / cos from
    phd_detmath.h, D16.)"""
    import phdslam
    from phdslam.scenario import bench_capacities
    cfg, n0, G, M, _ = phdslam.preset(cid)
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n)
    assert c.filterType == 0 and c.motionType == 1 and len(z) == M
    cap = bench_capacities(cid, G, M)
    sample = np.arange(0, n, every)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    _, compared, ut, form = _check_update(c, poses, lw, maps, offs, z, f"bench config {cid}", sample=sample,
                                          with_form=True, rtol=rtol, elementwise=True, **cap)
    if nt is not None:  # (configs 2 / 4: whichever the occupancy model picks — bench.py runs the same choice)
        assert ut[0] == nt and form == split, f"update instance {ut}, split {form}"
    assert compared >= 0.98 * len(sample) and len(sample) >= 32


def test_cphd_bench_configuration_pair_list_overflow(gpu):
    """bench.py --mode sequence's second measurement set (fresh range / bearing
    noise, 25 % clutter) at config 3's full shape and bench capacities: some
    particles overflow part C's culled pair list, whose bucket starts share the
    degree / edge memory (32 x 32 lattice); they must walk again with the exact
    distances in place (still the parallel merge, no serial fallback) and match
    the oracle.  Every 8th particle is compared."""
    import phdslam
    from phdslam.scenario import SEED_BASE, bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
    n, G, M = len(poses), 512, 64
    rng = np.random.default_rng(SEED_BASE + 3 + 1)  # bench.py's sequence sets
    for _ in range(2):
        zk = z.copy()
        zk["range"] = np.abs(zk["range"] + rng.normal(0, c.stdRange, len(zk))).astype(np.float32)
        zk["bearing"] = (zk["bearing"] + rng.normal(0, c.stdBearing, len(zk))).astype(np.float32)
        clut = rng.random(len(zk)) < 0.25
        zk["range"][clut] = rng.uniform(0, c.maxRange, int(clut.sum()))
        zk["bearing"][clut] = rng.uniform(-np.pi, np.pi, int(clut.sum()))
    # the update alone, at the tight capacities of the update without births
    # (candidates 704, survivors 224), an edge pool of K / 2 + 32 and the pair
    # list held to 400 entries (the walk lists the pairs of an ill-conditioned
    # candidate only when their exact distance makes them edges, so this set's
    # natural lists, ~450 at most, fit the par | off | pool space)
    cap = dict(map_capacity=704, max_measurements=64, candidate_capacity=704, survivor_capacity=224)
    f = _filter(c, n, **cap)
    f.set_edge_pool(704 // 2 + 32)
    f.set_pair_list_cap(400)
    f.load(poses, lw, maps, offs)
    f.merge_fallbacks()
    f.merge_pair_overflows()
    f.update(zk)
    f.check_errors()
    ovf, fb = f.merge_pair_overflows(), f.merge_fallbacks()
    st = f.particle_status()
    _, glw, gmaps, goffs = f.export()
    f.close()
    assert ovf > 0, "the set no longer overflows the pair list: the overflow walk is not exercised"
    assert fb == 0, f"{fb} particle-updates took the serial greedy ({ovf} pair-list overflows)"
    walked_twice = np.nonzero(st & 32)[0]  # PHD_ST_PAIR_OVERFLOW
    assert len(walked_twice) == ovf, (len(walked_twice), ovf)
    # every particle that took the overflow walk, plus every 8th
    sample = np.union1d(np.arange(0, n, 8), walked_twice)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    _compare_with_oracle(c, poses, lw, maps, offs, zk, (glw, gmaps, goffs), f"pair-list overflow ({ovf})", 0.05,
                         sample)
    ncls, _ = pyoracle.near_counts()
    idx = np.searchsorted(sample, walked_twice)
    assert np.sum(ncls[idx] == 0) >= 1, "no overflowing particle was compared with the oracle"


def test_update_config5_shape_pd07(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(5, n=16, G=1024, M=128)
    _check_update(c, poses, lw, maps, offs, z, "c5", map_capacity=1536, max_measurements=128,
                  candidate_capacity=1800, survivor_capacity=1024)


@pytest.mark.parametrize("phi,unwrapped", [(3.0, False), (-2.9, True), (3.14159, False)])
def test_update_bearing_window_across_the_cut(gpu, phi, unwrapped):
    """Banded pair loop (D7): components and measurements straddle the +-pi cut, and with
    `unwrapped` half of the measurement bearings are given 2*pi off (wrapAngle semantics)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=32, G=128, M=48)
    poses["ptheta"] = poses["ptheta"] + np.float32(phi)
    zb = z["bearing"].astype(np.float64) - phi
    zb = (zb + np.pi) % (2 * np.pi) - np.pi
    if unwrapped:
        zb[::2] += 2 * np.pi
    z["bearing"] = zb.astype(np.float32)
    _check_update(c, poses, lw, maps, offs, z, f"cut{phi}")


def test_update_wide_bearing_windows(gpu):
    """Large map covariances make every window wider than pi (all pairs evaluated)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=16, G=64, M=24)
    maps["cov"] = maps["cov"] * np.float32(400.0)
    _check_update(c, poses, lw, maps, offs, z, "wide")


def test_update_ragged_and_empty_maps(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=32, G=64, M=16)
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 65, 32)
    sizes[0] = 0
    sizes[1] = 64
    parts = [maps[offs[p]:offs[p] + sizes[p]] for p in range(32)]
    from phdslam.types import csr_from_maps
    m2, o2 = csr_from_maps(parts)
    _check_update(c, poses, lw, m2, o2, z, "ragged")


def test_update_out_of_range_components(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=32, G=128, M=16)
    c.maxRange = 30.0  # many components now near-range (class 2) or out of range (class 0)
    c.update_clutter_density()
    _check_update(c, poses, lw, maps, offs, z, "range-split", max_skip_frac=0.15)


def test_update_single_measurement_and_labels(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=16, G=64, M=8)
    c.labeledMeasurements = True
    z["label"][::2] = 1
    _check_update(c, poses, lw, maps, offs, z, "labels")
    c2, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=16, G=64, M=1)
    _check_update(c2, poses, lw, maps, offs, z, "M1")


@pytest.mark.parametrize("cid,clutter,birth", [(2, 0.0, 1e-6), (2, 0.0, 1e-12), (3, 0.05, 1e-6)])
def test_update_low_clutter_small_birth_weight(gpu, cid, clutter, birth):
    """η edge: with κ = 0 and a tiny birth weight, η_m is a sum of small
    likelihood terms (two-level fixed point, D3), so the lo level's resolution
    sets the error: log-weights and detection weights must still match to 1e-5."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=64, G=256, M=32)
    c.clutterRate = clutter
    c.update_clutter_density()
    c.birthWeight = birth
    # measurements 3 range sigmas off their feature: the likelihood terms are
    # ~e^-4.5 of their peak, η sits far below the hi level's 2^-40 resolution
    z["range"] = z["range"] + np.float32(3 * c.stdRange)
    _, compared, _ = _check_update(c, poses, lw, maps, offs, z, f"low-clutter c{cid} b{birth}", max_measurements=32)
    assert compared >= 60


def test_update_sharp_likelihood_flags_eta_range(gpu):
    """A likelihood term >= 2^20 would exhaust the fixed-point η's headroom:
    the update reports PHD_ST_ETA_RANGE (through phd_check_errors) rather than
    returning a clamped sum."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=4, G=8, M=4)
    c.stdRange, c.stdBearing = 1e-4, 1e-5
    maps["cov"] = maps["cov"] * np.float32(1e-8)
    maps["weight"] = 1.0
    for p in range(4):  # noise-free measurements of particle p's first four features
        for m in range(4):
            r, b = pyoracle.measure(poses[p], *maps[offs[p] + m]["mean"])
            if p == 0:
                z[m]["range"], z[m]["bearing"] = r, b
    f = _filter(c, 4)
    f.load(poses, lw, maps, offs)
    with pytest.raises(Exception, match="likelihood range"):
        f.update(z)
    f.close()


def test_update_moderate_likelihood_no_eta_flag(gpu):
    """Just below the 2^20 bound the same construction updates without a flag
    and matches the oracle."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=4, G=8, M=4)
    c.stdRange, c.stdBearing = 0.05, 0.01
    for m in range(4):
        r, b = pyoracle.measure(poses[0], *maps[offs[0] + m]["mean"])
        z[m]["range"], z[m]["bearing"] = r, b
    _check_update(c, poses, lw, maps, offs, z, "moderate")


@pytest.mark.parametrize("cid,n,G,M", [(2, 64, 256, 32), (5, 8, 1024, 128)])
def test_parallel_merge_equals_serial_greedy(gpu, cid, n, G, M):
    """The LFMIS formulation makes exactly the greedy's decisions (only the output order differs)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n, G=G, M=M)
    outs = []
    for mode in (0, 1):
        f = _filter(c, n, map_capacity=max(1024, G + 2 * M), max_measurements=M,
                    candidate_capacity=min(2 * G + 4 * M + 64, 1800), survivor_capacity=1024)
        f.set_merge_mode(mode)
        f.load(poses, lw, maps, offs)
        f.update(z)
        if mode == 0:
            assert f.merge_fallbacks() == 0
        outs.append(f.export())
        f.close()
    (_, w0, m0, o0), (_, w1, m1, o1) = outs
    np.testing.assert_array_equal(o0, o1)
    np.testing.assert_array_equal(w0, w1)
    for p in range(n):
        ok, worst = parity.compare_maps(m0[o0[p]:o0[p + 1]], m1[o1[p]:o1[p + 1]], rtol=1e-6)
        assert ok, (p, worst)


def _parity_all(c, poses, maps, offs, z, gm, go, n):
    om, oo, od, margin = pyoracle.update(c, poses, maps, offs, z)
    ncls, npm = pyoracle.near_counts()
    for p in range(n):
        A, B = om[oo[p]:oo[p + 1]], gm[go[p]:go[p + 1]]
        if ncls[p]:
            continue
        if npm[p]:
            ua, ub = parity.unmatched(A, B)
            assert max(ua, ub) <= 3 * npm[p], (p, ua, ub, int(npm[p]))
            continue
        ok, worst = parity.compare_maps(A, B)
        assert ok, (p, worst)


def test_degenerate_covariance_stays_on_parallel_merge(gpu):
    """Ill-conditioned candidates are tested exactly against all others inside the parallel merge."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=8, G=32, M=8)
    maps["cov"][offs[3] + 5] = (1e-9, 0.0, 0.0, 0.5)  # near-singular prior components
    maps["cov"][offs[5] + 2] = (0.3, 0.0, 0.0, 1e-8)
    f = _filter(c, 8)
    f.load(poses, lw, maps, offs)
    f.update(z)
    assert f.merge_fallbacks() == 0
    gp, glw, gm, go = f.export()
    f.close()
    _parity_all(c, poses, maps, offs, z, gm, go, 8)


@pytest.mark.parametrize("births", [True, False])
def test_wild_candidates_listed_by_exact_distance(gpu, births):
    """Ill-conditioned ("wild") candidates among config 3's dense maps, at its
    bench capacities: every 16th prior component nearly rank 1 (condition
    ~2e6), the step's births on or off.  The merge walk lists a pair with a wild
    candidate only when its exact distance makes it an edge: no
    pair-list overflow, no serial greedy, maps and log-weights as the oracle's
    on every particle."""
    import phdslam
    from phdslam.scenario import bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=256)
    G, M = 512, 64
    for p in range(len(poses)):
        for j in range(p % 16, G, 16):
            maps["cov"][offs[p] + j] = (0.4, 0.0, 0.0, 2e-7) if j % 32 else (3e-7, 0.0, 0.0, 0.3)
    cap = bench_capacities(3, G, M)
    f = _filter(c, len(poses), **cap)
    f.load(poses, lw, maps, offs)
    f.set_step_births(1 if births else 0)
    if births:  # as the bench runs the step (replay, phd_predict_update without a predict)
        f.set_replay(True)
        f.set_measurements(z)
        f.predict_update(None, 0, do_predict=False)
    else:
        f.update(z)
    f.check_errors()
    ovf, fb = f.merge_pair_overflows(), f.merge_fallbacks()
    _, glw, gmaps, goffs = f.export()
    f.close()
    assert ovf == 0 and fb == 0, (ovf, fb)
    if births:
        maps, offs = pyoracle.add_births(c, poses, maps, offs, z)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    _, compared = _compare_with_oracle(c, poses, lw, maps, offs, z, (glw, gmaps, goffs),
                                       f"wild candidates (births {births})", 0.02, None, parity.RTOL)
    assert compared >= 0.98 * len(poses)


def test_singular_covariance_takes_serial_fallback(gpu):
    """A zero covariance fails the greedy's own-distance test d(i,i) < T (NaN): the greedy then stops
    early (oracle semantics), which only the serial merge reproduces."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=8, G=32, M=8)
    maps["cov"][offs[6] + 1] = (0.0, 0.0, 0.0, 0.0)
    f = _filter(c, 8)
    f.load(poses, lw, maps, offs)
    f.update(z)
    assert f.merge_fallbacks() >= 1
    gp, glw, gm, go = f.export()
    f.close()
    _parity_all(c, poses, maps, offs, z, gm, go, 8)


def test_zero_separation_takes_serial_fallback(gpu):
    """minSeparation <= 0: nothing merges, the greedy stops at its first zero-weight set (oracle semantics)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=8, G=32, M=8)
    c.minSeparation = 0.0
    f = _filter(c, 8)
    f.load(poses, lw, maps, offs)
    f.update(z)
    assert f.merge_fallbacks() == 8
    gp, glw, gm, go = f.export()
    f.close()
    _parity_all(c, poses, maps, offs, z, gm, go, 8)


def test_dense_cluster_edge_overflow_takes_serial_fallback(gpu):
    """A map whose components all coincide has ~K^2/2 merge edges: the edge pool overflows and the
    particle falls back to the serial greedy on the cell-ordered records."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=4, G=96, M=8)
    p1 = slice(offs[1], offs[2])
    maps["mean"][p1] = maps["mean"][offs[1]] + 0.01 * np.arange(offs[2] - offs[1])[:, None].astype(np.float32)
    f = _filter(c, 4)
    f.load(poses, lw, maps, offs)
    f.update(z)
    assert f.merge_fallbacks() >= 1
    gp, glw, gm, go = f.export()
    f.close()
    _parity_all(c, poses, maps, offs, z, gm, go, 4)


def test_capacity_overflow_is_reported(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=8, G=64, M=32)
    f = _filter(c, 8, map_capacity=64, candidate_capacity=70, survivor_capacity=64)
    f.load(poses, lw, maps, offs)
    with pytest.raises(phdslam.PHDError) as e:
        f.update(z)
    assert e.value.code == phdslam._lib.PHD_E_CAPACITY
    f.close()


def test_predict_ackerman_host_noise_and_device_rng(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=1000, G=4, M=4)
    f = _filter(c, 1000)
    f.load(poses, lw, maps, offs)
    noise = pyoracle.noise_ackerman(c, 1000, 77, 5)
    f.predict_ackerman(2.5, 0.1, noise=noise)
    gp = f.export(with_maps=False)[0]
    op = pyoracle.predict_ackerman(c, poses, 2.5, 0.1, noise)
    for k in ("px", "py", "ptheta"):
        assert parity.close(gp[k], op[k], 1e-5, scale=1.0).all(), k
    # device-side Philox noise == the RNG contract evaluated on the host
    f.load(poses, lw, maps, offs)
    f.set_seed(77)
    f.predict_ackerman(2.5, 0.1, noise=None, step=5)
    gp2 = f.export(with_maps=False)[0]
    for k in ("px", "py", "ptheta"):
        assert parity.close(gp2[k], op[k], 1e-5, scale=1.0).all(), k
    f.close()


def test_predict_cv(gpu):
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=512, G=4, M=4)
    poses["vx"] = 1.5
    poses["vtheta"] = 0.2
    f = _filter(c, 512)
    f.load(poses, lw, maps, offs)
    noise = pyoracle.noise_cv(c, 512, 11, 3)
    f.predict_cv(noise=noise)
    gp = f.export(with_maps=False)[0]
    op = pyoracle.predict_cv(c, poses, noise)
    for k in POSE.names:
        assert parity.close(gp[k], op[k], 1e-5, scale=1.0).all(), k
    f.close()


@pytest.mark.parametrize("n", [4096, 1000, 9000])
def test_normalize_neff_resample_bit_exact(gpu, n):
    """n=9000 exceeds RS_LDS_MAX: the CDF lives in global memory."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=8, M=4)
    rng = np.random.default_rng(0)
    w = rng.normal(-8, 3, n).astype(np.float32)
    f = _filter(c, n)
    f.load(poses, w, maps, offs)
    f.normalize()
    neff = f.neff()
    gw = f.export(with_maps=False)[1]
    ow, _ = pyoracle.normalize(w)
    assert parity.close(gw, ow, 1e-5, floor=1e-5).all()
    np.testing.assert_allclose(neff, pyoracle.neff(ow), rtol=1e-5)
    # resample from identical weights: indices must be bit-exact
    u = pyoracle.resample_uniforms(n, 99, 7)
    f.load(poses, ow, maps, offs)
    idx = f.resample(uniforms=u)
    np.testing.assert_array_equal(idx, pyoracle.resample_fixed(ow, u))
    # the device RNG path draws the same uniforms
    f.load(poses, ow, maps, offs)
    f.set_seed(99)
    idx2 = f.resample(uniforms=None, step=7)
    np.testing.assert_array_equal(idx2, idx)
    # copy_particles semantics
    gp, gw2, gm, go = f.export()
    op, owc, om, oo = pyoracle.copy_particles(idx, poses, maps, offs)
    assert gp.tobytes() == op.tobytes() and gm.tobytes() == om.tobytes()
    np.testing.assert_array_equal(gw2, owc)
    f.close()


@pytest.mark.parametrize("n", [2048, 4096, 9000])
def test_step_fused_normalize_resample(gpu, n):
    """phd_step's normalise + nEff + decision + resample (Philox uniforms on the
    device; one block up to 2048 particles, chunked over n/1024 workgroups
    above) equals the oracle's update -> normalise -> nEff -> stratified
    resample.  Empty maps keep the update to births and a common
    weight shift; parents are read back through the pose remap."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=8, M=4)
    c.resampleThresh = 1.0  # always resample
    poses["px"] = np.arange(n, dtype=np.float32)  # distinct poses identify parents
    w = np.random.default_rng(3).normal(-8, 3, n).astype(np.float32)
    empty = np.zeros(0, maps.dtype)
    offs0 = np.zeros(n + 1, np.int32)
    f = _filter(c, n)
    f.load(poses, w, empty, offs0)
    f.set_measurements(z)
    f.set_seed(4242)
    neff, resampled = f.step(do_predict=False, step=11)
    gp, gw, _, _ = f.export()
    f.close()
    # the same update + normalise through the separate entry points gives the
    # weights the fused launch resampled (same device reductions)
    g = _filter(c, n)
    g.load(poses, w, empty, offs0)
    g.set_measurements(z)
    g.update()
    g.normalize()
    gw_norm = g.export(with_maps=False)[1]
    g.close()
    _, _, delta, _ = pyoracle.update(c, poses, empty, offs0, z)
    ow, _ = pyoracle.normalize((w + delta).astype(np.float32))
    assert parity.close(gw_norm, ow, 1e-5, floor=1e-5).all()
    np.testing.assert_allclose(neff, pyoracle.neff(ow), rtol=1e-5)
    assert resampled
    idx = pyoracle.resample_fixed(gw_norm, pyoracle.resample_uniforms(n, 4242, 11))
    np.testing.assert_array_equal(gp["px"], poses["px"][idx])
    np.testing.assert_allclose(gw, np.float32(-np.log(n)), rtol=1e-6)


@pytest.mark.parametrize("replay", [False, True])
@pytest.mark.parametrize("thresh", [1.0, 0.0])
def test_step_cphd_overlapped_resample_matches_separate_calls(gpu, thresh, replay):
    """Config 3 at its full shape through phd_step (CV predict, the three CPHD
    launches, and the one-launch resample on the second stream beside part C,
    PHD_RS_OVERLAP) against a second context running the separate entry points
    predict -> update -> normalize -> resample with the same seed and step:
    poses, log-weights, every map and the cardinality distributions equal bit
    for bit, with (threshold 1) and without (threshold 0) a resample, over two
    steps; in replay mode the second step (re-predicted from the fixed prior)
    equals one fresh step of the separate calls.  The step places the births of
    the previous scan (replay: of the replayed scan) after the predict; the
    separate calls add them with phd_add_births."""
    import phdslam
    from phdslam.scenario import bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
    n = len(poses)
    c.resampleThresh = thresh
    cap = bench_capacities(3, 512, 64)
    zs = [z, z.copy()]
    zs[1]["range"] = (zs[1]["range"] + 0.05).astype(np.float32)  # a second scan
    f = _filter(c, n, **cap)
    f.load(poses, lw, maps, offs)
    f_births = f.step_births()
    if replay:
        f.set_measurements(z)
        f.set_replay(True)
    g = _filter(c, n, **cap)
    g.set_step_births(0)
    g.load(poses, lw, maps, offs)
    for k in range(2):
        if not replay:
            f.set_measurements(zs[k])
        f.step(do_predict=True, step=k)
        if replay and k == 0:
            continue
        g.predict_cv(step=k)
        if replay:
            g.add_births(z)
        elif k > 0:
            g.add_births(zs[k - 1])
        g.set_measurements(z if replay else zs[k])
        g.update()
        g.normalize()
        if thresh > 0:
            g.resample(step=k, return_indices=False)
    f.check_errors()
    g.check_errors()
    a, b = f.export(), g.export()
    ca, cb = f.cardinality_distribution(), g.cardinality_distribution()
    f.close()
    g.close()
    for x, y, name in zip(a, b, ("poses", "log-weights", "maps", "offsets")):
        assert x.tobytes() == y.tobytes(), f"{name} differ"
    assert ca.tobytes() == cb.tobytes(), "cardinality distributions differ"
    assert f_births


@pytest.mark.parametrize("replay", [False, True])
@pytest.mark.parametrize("thresh", [1.0, 0.0])
def test_step_phd_split_overlapped_resample_matches_separate_calls(gpu, thresh, replay):
    """Config 4's per-GPU shard (Ackerman + static PHD, 4096 x 512 x 64, bench
    capacities: the split update) through phd_step — the Ackerman predict, part A,
    and the one-launch resample on the second stream beside part C
    (PHD_RS_OVERLAP: the log-weights are final after part A) — against a second
    context running predict -> update -> normalize -> resample through the
    separate entry points with the same seed and step: poses, log-weights and
    every map equal bit for bit, with and without a resample, over two steps
    (replay: the second step re-predicted from the fixed prior)."""
    import phdslam
    from phdslam.scenario import bench_capacities
    cfg, n0, G, M, _ = phdslam.preset(4)
    n = 4096
    c, poses, lw, maps, offs, z = phdslam.config_scenario(4, n=n)
    c.resampleThresh = thresh
    cap = bench_capacities(4, G, M)
    if not replay:  # (the second update's prior is the first one's posterior: more survivors than the bench's)
        cap["survivor_capacity"] = 2 * cap["survivor_capacity"]
    zs = [z, z]
    u = (2.0, 0.05)  # (v_encoder, alpha): bench.py's control
    f = _filter(c, n, **cap)
    f.load(poses, lw, maps, offs)
    assert f.update_form(), "config 4's per-GPU shard takes the split update"
    if replay:
        f.set_measurements(z)
        f.set_replay(True)
    g = _filter(c, n, **cap)
    g.load(poses, lw, maps, offs)
    for k in range(2):
        if not replay:
            f.set_measurements(zs[k])
        f.step(control=u, do_predict=True, step=k)
        if replay and k == 0:
            continue
        g.predict_ackerman(u[0], u[1], step=k)
        g.set_measurements(z if replay else zs[k])
        g.update()
        g.normalize()
        if thresh > 0:
            g.resample(step=k, return_indices=False)
    f.check_errors()
    g.check_errors()
    a, b = f.export(), g.export()
    f.close()
    g.close()
    for x, y, name in zip(a, b, ("poses", "log-weights", "maps", "offsets")):
        assert x.tobytes() == y.tobytes(), f"{name} differ"


@pytest.mark.parametrize("n,thresh", [(4096, 1.0), (9000, 1.0), (4096, 0.0), (9000, 0.0)])
def test_step_chunked_remap_with_maps(gpu, n, thresh):
    """phd_step above 2048 particles (chunked normalise / resample, the search
    kernel writing pose, slab reference and log-weight of each stratum) with
    non-empty maps: after a resample the exported store equals the oracle's
    copy_particles of the parents; without one (threshold 0) the identity copy
    and pointer swap leave poses and maps as the update left them."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=4, M=4)
    c.resampleThresh = thresh
    poses["px"] = np.arange(n, dtype=np.float32)
    w = np.random.default_rng(5).normal(-8, 3, n).astype(np.float32)
    f = _filter(c, n, map_capacity=64)
    f.load(poses, w, maps, offs)
    f.set_measurements(z)
    f.set_seed(99)
    neff, resampled = f.step(do_predict=False, step=3)
    gp, gw, gm, go = f.export()
    f.close()
    g = _filter(c, n, map_capacity=64)  # the same update + normalise without the resample
    g.load(poses, w, maps, offs)
    g.set_measurements(z)
    g.update()
    g.normalize()
    up, uw, um, uo = g.export()
    g.close()
    assert resampled == (thresh > 0)
    if resampled:
        idx = pyoracle.resample_fixed(uw, pyoracle.resample_uniforms(n, 99, 3))
        np.testing.assert_array_equal(gp["px"], poses["px"][idx])
        op, ow, om, oo = pyoracle.copy_particles(idx, up, um, uo)
        assert gp.tobytes() == op.tobytes() and gm.tobytes() == om.tobytes()
        np.testing.assert_array_equal(go, oo)
    else:
        assert gp.tobytes() == up.tobytes() and gm.tobytes() == um.tobytes()
        np.testing.assert_array_equal(gw, uw)


def _spawn(lw, maps, offs, npp):
    """Oracle statement of the n_predict_particles duplication (phdfilter.cu:1185-1238)."""
    n = len(lw)
    parent = np.repeat(np.arange(n), npp).astype(np.int32)
    _, _, m2, o2 = pyoracle.copy_particles(parent, np.zeros(n, POSE), maps, offs)
    return parent, (lw[parent] - np.float32(np.log(np.float32(npp)))).astype(np.float32), m2, o2


@pytest.mark.parametrize("cid,host_noise", [(2, False), (3, False), (3, True)])
def test_predict_n_predict_particles_device(gpu, cid, host_noise):
    """n_predict_particles = 3 on the device: the live count triples, every child
    takes its parent's map by slab reference and weight w - log 3, and is moved
    with its own noise draw (device Philox keyed by the child index, or the
    caller's n*3 noise entries — D4)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=40, G=16, M=4)
    c.nPredictParticles = 3
    poses["vx"] = 1.0
    poses["vtheta"] = 0.1
    f = _filter(c, 40, max_particles=120)
    f.load(poses, lw, maps, offs)
    c1 = c.copy()
    c1.nPredictParticles = 1
    if cid == 3:
        noise = pyoracle.noise_cv(c1, 120, 77 if host_noise else 1234, 5)
        f.predict_cv(noise=noise if host_noise else None, step=5)
        parent = np.repeat(np.arange(40), 3)
        op = pyoracle.predict_cv(c1, poses[parent], noise)
    else:
        noise = pyoracle.noise_ackerman(c1, 120, 1234, 5)
        f.predict_ackerman(2.0, 0.05, step=5)
        parent = np.repeat(np.arange(40), 3)
        op = pyoracle.predict_ackerman(c1, poses[parent], 2.0, 0.05, noise)
    assert f.n == 120
    gp, gw, gm, go = f.export()
    for k in POSE.names:
        assert parity.close(gp[k], op[k], 1e-5, scale=1.0).all(), k
    _, ow, om, oo = _spawn(lw, maps, offs, 3)
    np.testing.assert_array_equal(gw, ow)
    assert gm.tobytes() == om.tobytes()
    np.testing.assert_array_equal(go, oo)
    with pytest.raises(Exception, match="max_particles"):
        f.predict_cv() if cid == 3 else f.predict_ackerman(2.0, 0.05)  # 360 > 120
    f.close()


@pytest.mark.parametrize("n_live", [256, 9000])
def test_resample_live_particles_to_n_particles(gpu, n_live):
    """After spawned children grew the live set, the resample draws n_particles
    strata over all live weights (resampleParticles(particles, n_particles),
    main.cpp:1289): indices bit-exact against the oracle from identical weights;
    children take the parent's pose and map, weight -log n_particles."""
    import phdslam
    nb = 64 if n_live == 256 else 2000
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n_live, G=4, M=4)
    poses["px"] = np.arange(n_live, dtype=np.float32)
    w = np.random.default_rng(3).normal(-8, 3, n_live).astype(np.float32)
    f = _filter(c, nb, max_particles=n_live)
    f.load(poses, w, maps, offs)
    assert f.n == n_live
    f.normalize()
    wn = f.export(with_maps=False)[1]
    idx = f.resample(step=7)
    assert f.n == nb and len(idx) == nb
    oi = pyoracle.resample_fixed(wn, pyoracle.resample_uniforms(nb, 1234, 7))
    np.testing.assert_array_equal(idx, oi)
    gp, gw, gm, go = f.export()
    np.testing.assert_array_equal(gp["px"], poses["px"][oi])
    _, _, om, oo = pyoracle.copy_particles(oi, poses, maps, offs)
    assert gm.tobytes() == om.tobytes()
    np.testing.assert_array_equal(gw, np.float32(-np.log(nb)))
    f.close()


def test_step_n_predict_particles_sequence(gpu):
    """phd_step with n_predict_particles = 2 and no nEff resample (threshold 0):
    the live set grows 64 -> 128 -> 256 -> 512, which exceeds 5 x 64, so that
    step resamples back to 64 (main.cpp:1286) and the next grows again.  Each
    step is checked against the oracle started from the GPU's state before it:
    spawn + predict (poses, weights), update + normalise (maps, weights)."""
    import phdslam
    nb = 64
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=nb, G=64, M=16)
    c.nPredictParticles = 2
    c.resampleThresh = 0.0
    c1 = c.copy()
    c1.nPredictParticles = 1
    f = _filter(c, nb, max_particles=512, map_capacity=256, candidate_capacity=512)
    f.load(poses, lw, maps, offs)
    f.set_measurements(z)
    u = (1.0, 0.02)
    live = []
    for s in range(4):
        p0, w0, m0, o0 = f.export()
        neff, rs = f.step(control=u, step=s)
        live.append(f.n)
        parent, ow, om, oo = _spawn(w0, m0, o0, 2)
        n2 = len(parent)
        op = pyoracle.predict_ackerman(c1, p0[parent], u[0], u[1], pyoracle.noise_ackerman(c1, n2, 1234, s))
        um, uo, delta, _ = pyoracle.update(c, op, om, oo, z)
        ncls, npm = pyoracle.near_counts()
        wn, _ = pyoracle.normalize((ow + delta).astype(np.float32))
        gp, gw, gm, go = f.export()
        if not rs:
            assert f.n == n2
            for k in POSE.names:
                assert parity.close(gp[k], op[k], 1e-5, scale=1.0).all(), (s, k)
            if ncls.sum() == 0:
                assert parity.close(gw, wn, 1e-5, floor=1e-5).all(), s
            bad = 0
            for p in range(n2):
                if ncls[p] or npm[p]:
                    continue
                ok, _ = parity.compare_maps(um[uo[p]:uo[p + 1]], gm[go[p]:go[p + 1]]) \
                    if uo[p + 1] - uo[p] == go[p + 1] - go[p] else (False, 0)
                bad += not ok
            assert bad == 0, (s, bad)
        else:
            # forced: n_particles strata over the n2 live weights; parents ascend
            assert n2 > 5 * nb and f.n == nb
            np.testing.assert_array_equal(gw, np.float32(-np.log(nb)))
            oi = pyoracle.resample_fixed(wn, pyoracle.resample_uniforms(nb, 1234, s))
            # weights agree to 1e-5, not bit for bit: a stratum may rarely fall on the other side of a CDF step
            same = int(parity.close(gp["px"], op["px"][oi], 1e-5, scale=1.0).sum())
            assert same >= 0.95 * nb, (s, same)
    assert live == [128, 256, 64, 128]


@pytest.mark.parametrize("cid", [2, 3])
def test_step_fused_predict_equals_separate_kernels(gpu, cid):
    """phd_step fuses predict into the update launch; the result equals the
    separate predict -> update -> normalise calls bit for bit."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=64, G=64, M=16)
    c.resampleThresh = 0.0  # compare without a resample
    outs = []
    for fused in (True, False):
        f = _filter(c, 64)
        f.set_seed(77)
        f.load(poses, lw, maps, offs)
        f.set_measurements(z)
        if fused:
            f.step(control=(2.0, 0.05) if c.motionType == 1 else None, step=5)
        else:
            if c.motionType == 1:
                f.predict_ackerman(2.0, 0.05, noise=None, step=5)
            else:
                f.predict_cv(noise=None, step=5)
            f.update()
            f.normalize()
        outs.append(f.export())
        f.close()
    for a, b in zip(outs[0], outs[1]):
        assert a.tobytes() == b.tobytes()


def _slice_particles(poses, lw, maps, offs, lo, hi):
    o = offs[lo:hi + 1]
    return poses[lo:hi].copy(), lw[lo:hi].copy(), maps[o[0]:o[-1]].copy(), (o - o[0]).astype(np.int32)


def _emulated_step(shards, ctrl, k, dev):
    """One sync-free sharded step (ShardedFilter.step) of every emulated rank,
    the collectives emulated by device copies between the shards' buffers."""
    import torch
    for sf in shards:
        sf.local_update(ctrl, k)
    _emulated_settle(shards, ctrl, k)
    for sf in shards:
        if sf.aux is None:
            sf.w_all.copy_(torch.cat([o.w_local for o in shards]))
        else:  # the all-gather beside part C, as ShardedFilter.gather: after every rank's log-weights are final
            for o in shards:
                o.f.wait_logw(sf.aux.cuda_stream)
            with torch.cuda.stream(sf.aux):
                sf.w_all.copy_(torch.cat([o.w_local for o in shards]))
        sf.plan(k)
    blk = shards[0].K * shards[0].record_bytes
    for d, sf in enumerate(shards):  # equal-split all_to_all: block d of every rank -> rank d
        sf.recv_blocks.copy_(torch.cat([src.send_blocks[d * blk:(d + 1) * blk] for src in shards]))
        sf.receive()


def _emulated_settle(shards, ctrl, k):
    for sf in shards:
        sf.poll()
    for r, sf in enumerate(shards):  # point-to-point overflow transfers
        for s_, buf in sf._ovf[1]:
            src = [t for d, t in shards[s_]._ovf[0] if d == r]
            assert len(src) == 1 and src[0].numel() == buf.numel()
            buf.copy_(src[0])
    for sf in shards:
        sf.settle_finish(ctrl, k)


def _sharded_vs_single(cid, world, n, K, G=32, M=16, steps=3, caps=None, S=0x5eed, births=False, empty_steps=()):
    """`world` emulated ranks of ShardedFilter (sync-free: global normalise /
    resample on the gathered log-weights, fixed blocks of K records per peer, the
    rest exchanged after the next update is enqueued and its slots re-updated)
    on one device against a single context of world * n particles stepped from
    the gathered shards of the previous step.  After each step the particles
    held across the shards must equal the single context's exactly, up to order:
    poses, log-weights, every map, and (CPHD) every cardinality distribution —
    the cardinality coefficient rows travel in the migration records.
    births: the shards' steps place the births of the previous scan (the scan
    is set again before every step, so from step 2 on; the pending slots'
    re-updates place them too) and the single context adds them explicitly.
    empty_steps: steps whose scan is empty (no update, no resample:
    main.cpp:1260; the births of the previous scan still join the maps, and on
    the shards also the pending slots' records re-stepped on that empty scan).
    Returns (pending slots, migrated particles) over the run."""
    import torch
    import phdslam
    from phdslam.dist import ShardedFilter
    caps = caps or {}
    N = world * n
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=N, G=G, M=M)
    c.resampleThresh = 1.0  # resample every step
    cphd = c.filterType == 1
    ack = c.motionType == 1
    ctrl = (2.0, 0.05) if ack else None
    dev = torch.device("cuda", 0)
    single = _filter(c, N, **caps)
    single.set_seed(S)
    single.set_step_births(0)
    single.load(poses, lw, maps, offs)
    single.set_measurements(z)
    shards = []
    for r in range(world):
        f = _filter(c, n, **caps)
        f.set_seed(S)
        f.set_step_births(1 if births else 0)
        f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        f.load(*_slice_particles(poses, lw, maps, offs, r * n, (r + 1) * n))
        if not births:  # (with births the scan is set before every step: its previous one from step 2 on)
            f.set_measurements(z)
        shards.append(ShardedFilter(f, None, dev, world=world, rank=r, seed=S, block_records=K))

    def gathered():
        got = [sf.f.export() for sf in shards]
        gmaps, goffs = [], [0]
        for g in got:
            gmaps.append(g[2])
            goffs.extend((np.asarray(g[3][1:]) + goffs[-1]).tolist())
        return (np.concatenate([g[0] for g in got]), np.concatenate([g[1] for g in got]),
                np.concatenate(gmaps), np.asarray(goffs, dtype=np.int32))

    pending = 0
    z_empty = z[:0]
    for k in range(1, steps + 1):
        zk = z_empty if k in empty_steps else z
        prev_empty = (k - 1) in empty_steps
        # the single context steps from the gathered shards of step k-1 (migration
        # keeps survivors in place, so the global order differs; predict noise is
        # keyed by global particle index)
        if k > 1:
            single.load(*gathered_prev)  # (CPHD rows: the update recomputes them from the map)
        if ack:
            single.predict_ackerman(*ctrl, noise=None, step=k)
        else:
            single.predict_cv(noise=None, step=k)
        if births and k > 1 and not prev_empty:
            single.add_births(z)
        if births or empty_steps:
            single.set_measurements(zk)
        single.update()
        single.normalize()
        if len(zk):
            single.resample(uniforms=None, step=k)
        if births or empty_steps:
            for sf in shards:
                sf.f.set_measurements(zk)
        _emulated_step(shards, ctrl, k, dev)
        # the shards' state after step k: settle the open plan as flush() does
        # (no update follows) — on copies of the contexts' store via export
        _emulated_settle(shards, None, None)
        torch.cuda.synchronize()
        pending += sum(sf.stats["pending_slots"] for sf in shards)
        if k in empty_steps:  # (no update: no resample, main.cpp:1281-1297)
            assert not any(sf.last[1] for sf in shards)
        else:
            assert all(sf.last[1] for sf in shards)
        moved = sum(sf.stats["migrated"] for sf in shards)
        records = sum(sf.stats["records"] for sf in shards)
        assert records <= moved
        gathered_prev = gathered()
        sp, sw, sm, so = single.export()
        gp, gw, gm, goffs = gathered_prev
        assert len(gp) == N
        key = lambda P: np.lexsort((P["ptheta"], P["py"], P["px"]))
        ks, kg = key(sp), key(gp)
        assert sp[ks].tobytes() == gp[kg].tobytes(), f"step {k}: particle poses differ"
        np.testing.assert_array_equal(sw, gw)
        # maps of matched particles
        for a_, b_ in zip(ks, kg):
            ms = sm[so[a_]:so[a_ + 1]]
            mg = gm[goffs[b_]:goffs[b_ + 1]]
            assert ms.tobytes() == mg.tobytes(), f"step {k}: map of particle {a_} differs"
        if cphd and k not in empty_steps:  # (cardinality rows come from an update)
            cs = single.cardinality_distribution()
            cg = np.concatenate([sf.f.cardinality_distribution() for sf in shards])
            assert cs[ks].tobytes() == cg[kg].tobytes(), f"step {k}: cardinality distributions differ"
    moved = sum(sf.stats["migrated"] for sf in shards)
    single.close()
    for sf in shards:
        sf.f.close()
    return pending, moved


@pytest.mark.parametrize("cid", [2, 3])
@pytest.mark.parametrize("world,n,K", [(2, 48, 4), (3, 48, 1), (5, 48, 0), (2, 1000, 4), (3, 700, 2), (3, 700, 0)])
def test_sharded_step_matches_single_context(gpu, cid, world, n, K):
    """Multi-GPU step emulated with `world` contexts on one device (see
    _sharded_vs_single), PHD (config 2's model) and CPHD (config 3's: CV
    predict, cardinality rows in the records).  K = 0 and 1 force the overflow
    path (every or most records beyond the blocks).  (2, 1000): the shards'
    chunked plan (2 chunks of 1024) against the single context's one-block
    k_normalize_resample (2000 <= 2048) — the canonical sum order makes them
    agree bit for bit; (3, 700): 3 chunks, the last one partial, on both sides.
    CPHD runs with the step's births (from step 2 on)."""
    pending, moved = _sharded_vs_single(cid, world, n, K, births=cid == 3)
    if K == 0:
        assert pending > 0  # the overflow path ran
    assert moved > 0


@pytest.mark.parametrize("cid", [2, 3])
@pytest.mark.parametrize("K", [0, 2])
def test_sharded_step_with_empty_scan(gpu, cid, K):
    """A sharded run whose second scan is empty: no update, no resample, the
    all-gather fed by the log-weight copy (its ready event recorded after the
    copy, phd_predict_update), and with K = 0 the previous step's records all
    beyond the blocks — pending slots re-stepped on the empty scan, CPHD placing
    their births of the previous scan (a slot-indexed k_add_births).  Equal bit
    for bit to one context of world * n particles after every step."""
    pending, moved = _sharded_vs_single(cid, 3, 64, K, steps=4, births=cid == 3, empty_steps=(2,))
    if K == 0:
        assert pending > 0
    assert moved > 0


def test_sharded_step_config4_survey_model(gpu):
    """Config 4 as SURVEY §8(d) / BASELINE configs[3] define it (phdslam.preset(4):
    Ackerman predict + static PHD, 8 x 4096 = 32768 particles x 512 GM x 64
    measurements), emulated on one device with bench.py's capacities, fixed
    blocks of 4 records per peer and a resample every step, against one
    32768-particle context — equal bit for bit after every step (poses,
    log-weights, maps), with particles migrating between the ranks."""
    from phdslam.scenario import bench_capacities
    pending, moved = _sharded_vs_single(4, 8, 4096, 4, G=512, M=64, steps=2, caps=bench_capacities(4, 512, 64))
    assert moved > 0


def test_sharded_step_config4_full_shape(gpu):
    """Config 4's job as bench.py --gpus 8 runs it by default (config-3 shards,
    the north-star shape per GPU), emulated on one device:
    8 ranks x 4096 particles (32768) at 512 GM x 64 measurements, CV + CPHD,
    bench.py's capacities, fixed blocks of 4 records per peer, a resample every
    step, against one 32768-particle context — equal bit for bit after every
    step (poses, log-weights, maps, cardinality distributions), with particles
    migrating between the ranks.  (The RCCL leg itself needs the 8-GPU node.)"""
    from phdslam.scenario import bench_capacities
    pending, moved = _sharded_vs_single(3, 8, 4096, 4, G=512, M=64, steps=2, caps=bench_capacities(3, 512, 64),
                                        births=True)
    assert moved > 0


def test_sharded_step_config5_whole_job(gpu):
    """Config 5's whole job (BASELINE configs[4]: 8 x 8192 = 65536 particles x
    1024 GM x 128 measurements at Pd 0.7, min_separation 10 — the merge-stress
    configuration, Ackerman + PHD) emulated on one device: 8 ranks with bench.py's
    per-GPU capacities (candidates 1800, survivors 640), fixed blocks of 4 records
    per peer, a resample every step, against one 65536-particle context — equal
    bit for bit after every step (poses, log-weights, maps), with particles
    migrating between the ranks (records of up to 1536 components)."""
    from phdslam.scenario import bench_capacities
    pending, moved = _sharded_vs_single(5, 8, 8192, 4, G=1024, M=128, steps=2, caps=bench_capacities(5, 1024, 128))
    assert moved > 0


class _LocalComm:
    """The transport of a world-1 ShardedFilter: every collective is a copy."""

    def all_gather(self, out, inp):
        out.copy_(inp)

    def all_to_all_equal(self, out, inp):
        out.copy_(inp)

    def exchange(self, sends, recvs):
        for (_, t), (_, b) in zip(sends, recvs):
            b.copy_(t)


@pytest.mark.parametrize("cid,n,steps", [(2, 256, 3), (3, 300, 2)])
def test_group_driver_matches_sharded_filter(gpu, tmp_path, cid, n, steps):
    """The multi-GPU C++ host (phdslam_run --synth --gpus N over
    libphdslam_group.so: RCCL called directly, ncclCommInitAll + grouped calls,
    no PyTorch) at world 1 on this GPU against phdslam.dist.ShardedFilter at
    world 1 on the same scenario, seeds, capacities and steps (a resample every
    step): every particle's pose, log-weight and map equal bit for bit."""
    import subprocess
    import torch
    import phdslam
    from phdslam.dist import ShardedFilter
    from phdslam.scenario import SEED_BASE, bench_capacities
    exe = os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "phdslam_run")
    dump = tmp_path / "group.bin"
    r = subprocess.run([exe, "--synth", str(cid), "--gpus", "1", "--particles", str(n), "--steps", str(steps),
                        "--resample-every", "--dump", str(dump)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    cfg, _, G, M, _ = phdslam.preset(cid)
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n)
    c.resampleThresh = 1.0
    dev = torch.device("cuda", 0)
    f = phdslam.PHDFilter(n, c, **bench_capacities(cid, G, M))
    f.set_seed(SEED_BASE + cid)
    f.load(poses, lw, maps, offs)
    f.set_measurements(z)
    f.set_check_each_update(False)
    sf = ShardedFilter(f, None, dev, world=1, rank=0, block_records=4, comm=_LocalComm())
    ctrl = (2.0, 0.05) if c.motionType == 1 else None
    for k in range(1, steps + 1):
        sf.step(ctrl, k)
    sf.flush()
    torch.cuda.synchronize()
    f.check_errors()
    gp, gw, gm, go = f.export()
    f.close()
    raw = dump.read_bytes()
    o = 0
    cnt = int(np.frombuffer(raw, np.int32, 1, o)[0])
    o += 4
    assert cnt == n
    dp = np.frombuffer(raw, POSE, n, o)
    o += POSE.itemsize * n
    dw = np.frombuffer(raw, np.float32, n, o)
    o += 4 * n
    dsz = np.frombuffer(raw, np.int32, n, o)
    o += 4 * n
    dm = np.frombuffer(raw, GAUSSIAN2D, int(dsz.sum()), o)
    assert dp.tobytes() == gp.tobytes(), "poses differ"
    assert dw.tobytes() == gw.tobytes(), "log-weights differ"
    assert np.array_equal(dsz, np.diff(go)), "map sizes differ"
    assert dm.tobytes() == gm.tobytes(), "maps differ"
    assert '"resamples": ' in r.stdout


@pytest.mark.parametrize("cid,n,steps", [(2, 256, 3), (3, 300, 3)])
def test_group_rank_matches_sharded_filter(gpu, cid, n, steps):
    """bench.py's sharded transport (phdslam.dist.GroupRank: the C++ host's
    per-process rank, phd_group_create_rank over ncclCommInitRank, one C call
    per step) at world 1 on this GPU against phdslam.dist.ShardedFilter at
    world 1 on the same scenario, seeds, capacities and steps (a resample every
    step): every particle's pose, log-weight and map equal bit for bit, and the
    step counters agree."""
    import torch
    import phdslam
    from phdslam.dist import GroupRank, ShardedFilter
    from phdslam.scenario import SEED_BASE, bench_capacities
    cfg, _, G, M, _ = phdslam.preset(cid)
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n)
    c.resampleThresh = 1.0
    dev = torch.device("cuda", 0)
    ctrl = (2.0, 0.05) if c.motionType == 1 else None
    out = []
    for kind in ("torch", "cxx"):
        f = phdslam.PHDFilter(n, c, **bench_capacities(cid, G, M))
        f.set_seed(SEED_BASE + cid)
        f.load(poses, lw, maps, offs)
        f.set_measurements(z)
        f.set_check_each_update(False)
        if kind == "torch":
            sf = ShardedFilter(f, None, dev, world=1, rank=0, block_records=4, comm=_LocalComm())
        else:
            sf = GroupRank(f, None, dev, world=1, rank=0, block_records=4)
        for k in range(1, steps + 1):
            sf.step(ctrl, k)
        sf.flush()
        torch.cuda.synchronize()
        f.check_errors()
        out.append((f.export(), dict(sf.stats)))
        if kind == "cxx":
            sf.close()
        f.close()
    (a, sa), (b, sb) = out
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()
    assert sa["resamples"] == sb["resamples"] == steps
    assert sa["migrated"] == sb["migrated"] and sa["records"] == sb["records"]


def _plan_reference(parents, n, world):
    """dist.plan_migration per rank, with the device's record folding: per
    rank (demand, keep, local parent of each record sent in destination order)."""
    from phdslam.dist import plan_migration
    out = []
    for r, p in enumerate(plan_migration(parents, n, world)):
        recs = []
        for d in sorted(p["send"]):
            prev = None
            for q in p["send"][d].tolist():
                if q != prev:
                    recs.append(q)
                prev = q
        out.append((int(np.sum(np.asarray(parents) // n == r)), p["keep"], np.asarray(recs, np.int32)))
    return out


@pytest.mark.parametrize("world,n", [(4, 1024), (8, 4096)])
def test_shard_plan_strata_past_cdf_end(gpu, world, n):
    """Strata past the CDF's end.  Gathered log-weights near 30000 put lse on a
    coarse float grid (ulp 2e-3), so for about half the draws the normalised
    weights sum to a few 1/N under one and the last strata fall past the
    fixed-point CDF's end: they take the first maximum, as the reference's
    resampler does (main.cpp:470-488), and the parent list drops at its end.
    The one-launch plan (k_shard_plan: (8, 4096) is config 4's 32 workgroups)
    must give the parents of the single-block resample (phd_global_resample)
    bit for bit, and on every rank the demand, kept children and records of
    dist.plan_migration on that list — the suffix read as children of its
    parent's rank, never as children of the last rank."""
    import torch
    import phdslam
    N = world * n
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=4, M=4)
    c.resampleThresh = 1.0
    dev = torch.device("cuda", 0)
    f = _filter(c, n, map_capacity=64, max_measurements=4)
    f.load(poses, lw, maps, offs)
    f.set_measurements(z)
    seed, step = 0x5eed, 3
    par_ref = torch.empty(N, dtype=torch.int32, device=dev)
    found = None
    for k in range(64):
        base = (np.float32(30000.0) + np.random.default_rng(100 + k).normal(0.0, 1.0, N)).astype(np.float32)
        w = torch.from_numpy(base.copy()).to(dev)
        f.global_resample(w.data_ptr(), N, 0, seed, step, par_ref.data_ptr())
        torch.cuda.synchronize()
        pr = par_ref.cpu().numpy()
        if np.any(np.diff(pr) < 0):
            found = (base, pr)
            break
    assert found is not None, "no draw put strata past the CDF's end"
    base, pr = found
    ref = _plan_reference(pr, n, world)
    rec_bytes = f.record_bytes()
    parents = torch.empty(N, dtype=torch.int32, device=dev)
    keep = torch.empty(n, dtype=torch.int32, device=dev)
    send = torch.empty(n * (world - 1), dtype=torch.int32, device=dev)
    recv = torch.empty(n, dtype=torch.int32, device=dev)
    records = torch.empty(n * rec_bytes, dtype=torch.uint8, device=dev)
    for r in range(world):
        f.load(poses, lw, maps, offs)
        w = torch.from_numpy(base.copy()).to(dev)
        neff, rs, demand, snd, rcv = f.shard_resample(w.data_ptr(), world, r, seed, step, parents.data_ptr(),
                                                      keep.data_ptr(), send.data_ptr(), recv.data_ptr(),
                                                      records.data_ptr(), n, -np.log(N))
        torch.cuda.synchronize()
        assert rs
        np.testing.assert_array_equal(parents.cpu().numpy(), pr)
        d_ref, keep_ref, recs_ref = ref[r]
        assert demand[r] == d_ref and demand == [x[0] for x in ref]
        np.testing.assert_array_equal(keep.cpu().numpy()[:min(d_ref, n)], keep_ref)
        np.testing.assert_array_equal(send.cpu().numpy()[:len(recs_ref)], recs_ref)
        assert sum(snd) == len(recs_ref)
    f.close()


@pytest.mark.parametrize("K", [4, 0])
def test_sharded_step_overflow_recovery_reupdates_slots(gpu, K):
    """The overflow path inside a running sequence: step k's records beyond the
    blocks arrive after step k+1's update was enqueued; their slots are
    re-updated (phd_update_pending).  Three chained sharded steps with and
    without the blocks equal each other exactly."""
    import torch
    import phdslam
    from phdslam.dist import ShardedFilter
    world, n = 3, 64
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=world * n, G=32, M=16)
    c.resampleThresh = 1.0
    dev = torch.device("cuda", 0)
    runs = []
    for kk in (K, 64):
        shards = []
        for r in range(world):
            f = _filter(c, n)
            f.set_seed(7)
            f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            f.load(*_slice_particles(poses, lw, maps, offs, r * n, (r + 1) * n))
            f.set_measurements(z)
            shards.append(ShardedFilter(f, None, dev, world=world, rank=r, seed=7, block_records=kk))
        for k in range(1, 4):
            _emulated_step(shards, (2.0, 0.05), k, dev)
        _emulated_settle(shards, None, None)
        torch.cuda.synchronize()
        runs.append([sf.f.export() for sf in shards])
        if kk == 0:
            assert sum(sf.stats["pending_slots"] for sf in shards) > 0
        for sf in shards:
            sf.f.close()
    for a, b in zip(*runs):
        for x, y in zip(a, b):
            assert x.tobytes() == y.tobytes()


@pytest.mark.parametrize("cid", [2, 3])
def test_sharded_step_two_processes(gpu, tmp_path, cid):
    """Config 4's leg under a real process group: two ranks, each its own process
    on cuda:0 running the product's ShardedFilter.step over torch.distributed
    (gloo: RCCL refuses two ranks on one GPU), at config 4's per-particle shape
    (G = 512, M = 64) with 1024 particles per rank and a resample every step —
    PHD with Ackerman predict (cid 2) and CPHD with CV predict (cid 3, the
    bench's N>1 workload).  After every step the particles held across the two
    shards equal a single context of 2048 particles stepped from the previous
    gathered state, bit for bit (poses, log-weights, every map, CPHD
    cardinality distributions), up to order."""
    import socket
    import torch
    import torch.multiprocessing as mp
    import phdslam
    import shard_worker
    world, n, G, M, steps, S = 2, 1024, 512, 64, 3, 0x5eed
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=shard_worker.run, args=(r, world, port, n, G, M, steps, S, str(tmp_path), 4, cid))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=world * n, G=G, M=M)
    c.resampleThresh = 1.0
    single = _filter(c, world * n, map_capacity=1024, max_measurements=M, candidate_capacity=2048,
                     survivor_capacity=1024)
    single.set_seed(S)
    single.set_measurements(z)
    prev = (poses, lw, maps, offs)
    migrated = 0
    for k in range(1, steps + 1):
        single.load(*prev)
        if c.motionType == 1:
            single.predict_ackerman(2.0, 0.05, noise=None, step=k)
        else:
            single.predict_cv(noise=None, step=k)
        single.update()
        single.normalize()
        single.resample(uniforms=None, step=k)
        sp, sw, sm, so = single.export()
        parts = [np.load(tmp_path / f"r{r}_k{k}.npz") for r in range(world)]
        assert all(int(p_["resampled"]) == 1 for p_ in parts)
        migrated = sum(int(p_["migrated"]) for p_ in parts)
        gp = np.concatenate([p_["poses"] for p_ in parts])
        gw = np.concatenate([p_["w"] for p_ in parts])
        gm = np.concatenate([p_["maps"] for p_ in parts])
        go = [0]
        for p_ in parts:
            go.extend((p_["offs"][1:] + go[-1]).tolist())
        go = np.asarray(go, np.int32)
        key = lambda P: np.lexsort((P["ptheta"], P["py"], P["px"]))
        ks, kg = key(sp), key(gp)
        assert sp[ks].tobytes() == gp[kg].tobytes(), f"step {k}: particle poses differ"
        np.testing.assert_array_equal(sw, gw)
        for a_, b_ in zip(ks, kg):
            assert sm[so[a_]:so[a_ + 1]].tobytes() == gm[go[b_]:go[b_ + 1]].tobytes(), f"step {k}: map {a_}"
        if c.filterType == 1:
            cs = single.cardinality_distribution()
            cg = np.concatenate([p_["cn"] for p_ in parts])
            assert cs[ks].tobytes() == cg[kg].tobytes(), f"step {k}: cardinality distributions differ"
        prev = (gp, gw, gm, go)
    single.close()
    assert migrated > 0  # particles changed rank: the all-to-all carried records
    torch.cuda.synchronize()


def test_expected_pose_and_cardinality(gpu):
    import phdslam
    n = 300
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=32, M=8)
    w, _ = pyoracle.normalize(np.random.default_rng(1).normal(0, 1, n).astype(np.float32))
    f = _filter(c, n)
    f.load(poses, w, maps, offs)
    gpose, gmi = f.expected_pose()
    opose, omi = pyoracle.expected_pose(w, poses)
    assert gmi == omi
    for k in POSE.names:
        assert parity.close(gpose[k], opose[k], 1e-5, scale=1e-3).all(), k
    cn = f.cardinalities()
    ref = np.array([maps["weight"][offs[p]:offs[p + 1]].astype(np.float64).sum() for p in range(n)])
    np.testing.assert_allclose(cn, ref, rtol=1e-5)
    f.close()


@pytest.mark.parametrize("scans", [1135])
def test_multistep_sequence_config1_data(gpu, scans):
    """Config 1 (BASELINE configs[0]) as the reference's loop runs it
    (main.cpp:1178-1312) over its own data (python/*_synth.txt: 64 particles,
    Ackerman, ≈96 measurements per scan) with the G-cap-64 policy
    (oracle/config1_loop.py), over every scan of the data (1 135): each scan the GPU
    predicts (device Philox, seed 5), updates, and — when the oracle's nEff
    decides to resample — resamples from the oracle's weights, all from the
    oracle's capped state of the previous scan (re-synchronised each scan).
    Predicted poses, posterior maps and log-weights are held to the oracle
    (_compare_with_oracle), resample parents bit for bit.  (Before D17 the
    clutter births' exact weight ties split differently on the two sides from
    scan 36 on: 8 of 7 680 particle-updates in 120 scans differed.)"""
    import time
    import phdslam
    import config1_loop as L
    c = phdslam.preset(1)[0]
    n, seed = 64, 5
    controls, zs = L.load_scans()
    cap = dict(map_capacity=1024, max_measurements=256, candidate_capacity=1600, survivor_capacity=1024)
    f = _filter(c, n, **cap)
    f.set_seed(seed)
    state = L.initial_state(n)
    resamples = compared = 0
    t0 = time.perf_counter()
    for s_ in range(min(scans, len(zs))):
        poses, lw, maps, offs = state
        z = zs[s_]
        f.load(poses, lw, maps, offs)
        if s_ > 0:
            v, alpha = controls[s_ - 1]
            f.predict_ackerman(float(v), float(alpha), noise=None, step=s_)
        nxt, rec = L.step(c, state, controls, zs, s_, seed)
        gp = f.export(with_maps=False)[0]
        for k_ in ("px", "py", "ptheta"):
            assert parity.close(gp[k_], rec["pred"][k_], 1e-5, scale=1.0).all(), (s_, k_)
        if len(z):
            f.set_measurements(z)
            f.update()
            f.check_errors()
            _, glw, gmaps, goffs = f.export()
            _, n_cmp = _compare_with_oracle(c, rec["pred"], lw, maps, offs, z, (glw, gmaps, goffs), f"c1 scan {s_}",
                                            0.1)
            compared += n_cmp
        if rec["parents"] is not None:
            # the device's stratified resample from the oracle's capped, normalised state
            f.load(rec["pred"], rec["lw"], rec["maps"], rec["offs"])
            idx = f.resample(uniforms=None, step=s_)
            np.testing.assert_array_equal(idx, rec["parents"], err_msg=f"scan {s_}: resample parents")
            resamples += 1
        state = nxt
    f.close()
    print(f"config 1: {min(scans, len(zs))} scans, {compared} particle-updates compared, {resamples} resamples, "
          f"{time.perf_counter() - t0:.1f} s")
    assert resamples > 0 and compared >= 0.9 * n * (min(scans, len(zs)) - 1)


def test_multistep_cv_cphd_reference_cv_data(gpu):
    """Config 3's path (CV predict + CPHD update) over the first steps of the
    reference's own CV dataset (matlab/measurements_synth_cv.txt, generated by
    matlab/SynthSetup2.m: range 10 m, dt .02, clutter rate 20, Pd .95), GPU vs
    oracle on identical noise, re-synchronised each step; the log cardinality
    distributions are compared too.  The CPHD update array has no birth terms
    (phdfilter.cu.bak:1437-1504), so step 0 builds the prior map with the PHD
    update's births and the CPHD update runs from step 1 on."""
    import phdslam
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "config3_cv_data.npz"))
    c, _, _, _, _ = phdslam.preset(3)
    assert c.motionType == 0 and c.filterType == 1
    c.maxRange = 10.0
    c.dt = 0.02
    c.maxCardinality = 255
    c.update_clutter_density()
    n = 64
    poses = np.zeros(n, POSE)
    lw = np.full(n, -np.log(n), np.float32)
    maps = np.zeros(0, GAUSSIAN2D)
    offs = np.zeros(n + 1, np.int32)
    cap = dict(map_capacity=1024, max_measurements=64, candidate_capacity=1600, survivor_capacity=512)
    c0 = c.copy()
    c0.filterType = 0
    for step in range(7):
        zz = d["meas"][d["meas_offsets"][step]:d["meas_offsets"][step + 1]]
        z = np.zeros(len(zz), MEASUREMENT)
        z["range"], z["bearing"] = zz[:, 0], zz[:, 1]
        if step > 0:
            poses = pyoracle.predict_cv(c, poses, pyoracle.noise_cv(c, n, 9, step))
        if step == 0:
            _check_update(c0, poses, lw, maps, offs, z, "cv0 (PHD births)", **cap)
            maps, offs, delta, _ = pyoracle.update(c0, poses, maps, offs, z)
            lw, _ = pyoracle.normalize(lw + delta)
            continue
        _check_update(c, poses, lw, maps, offs, z, f"cv{step}", max_skip_frac=0.1, **cap)
        f = _filter(c, n, **cap)
        f.load(poses, lw, maps, offs)
        f.update(z)
        cn_gpu = f.cardinality_distribution().astype(np.float64)
        f.close()
        maps, offs, delta, _, cn = pyoracle.update(c, poses, maps, offs, z, cardinality=True)
        ncls, _ = pyoracle.near_counts()
        sig = (cn > -60.0) & (ncls == 0)[:, None]
        assert parity.close(cn_gpu[sig], cn[sig], 1e-5, floor=1e-4).all(), f"step {step}: cardinality"
        lw, _ = pyoracle.normalize(lw + delta)


def _eap_compare(g, o, label):
    assert len(g) == len(o), f"{label}: {len(g)} GPU vs {len(o)} oracle components"
    for k in ("weight", "mean", "cov"):
        a, b = g[k].astype(np.float64), o[k].astype(np.float64)
        scale = 1e-30 if k == "weight" else 1e-4
        # a merged component whose weights all underflowed to 0 has mean/cov 0/0 = NaN in the
        # reference too (gm_reduce.cpp:113,122 divide by the summed weight): NaN must match NaN
        ok = parity.close(a, b, 1e-5, scale=scale) | (np.isnan(a) & np.isnan(b))
        assert ok.all(), f"{label}: {k} differs (worst {np.nanmax(np.abs(a - b))})"


@pytest.mark.parametrize("n,G,M,resample", [(64, 64, 16, False), (64, 64, 16, True), (1024, 256, 32, False)])
def test_expected_map_matches_oracle(gpu, n, G, M, resample):
    """§8(f) rank 1: the GPU EAP expected map (computeExpectedMap main.cpp:290-316 +
    reduceGaussianMixture gm_reduce.cpp:59-132) equals the oracle's greedy
    reduce of the same exported state, in emission order.  The resampled case
    holds duplicated children: exact weight ties, broken by index on both sides.
    n=1024, G=256 is the config-2 scale (262k components)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(2, n=n, G=G, M=M)
    f = _filter(c, n, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024)
    f.load(poses, lw, maps, offs)
    f.update(z)
    f.normalize()
    if resample:
        f.resample(step=3)
    gp, gw, gm, go = f.export()
    eap = f.expected_map()
    groups = f.expected_map_groups()
    f.close()
    ref = pyoracle.expected_map(c, gw, gm, go)
    _eap_compare(eap, ref, f"eap n{n}G{G}M{M}")
    assert groups >= 1
    # the reduction conserves the weighted mass
    tot = sum(float(np.exp(np.float64(gw[p]))) * gm["weight"][go[p]:go[p + 1]].astype(np.float64).sum()
              for p in range(n))
    assert abs(eap["weight"].astype(np.float64).sum() - tot) <= 1e-4 * tot


@pytest.mark.parametrize("case", ["dense", "chains", "single", "nonfinite", "zero_weights", "near_singular",
                                  "rank1_pairs"])
def test_expected_map_edge_cases(gpu, case):
    """The GPU EAP map against the oracle's greedy on shapes the scenario
    tests do not reach: `dense` — 512 particles x 96 components piled on 12
    landmarks (every cell holds thousands of positions: the decision rounds
    stream many LDS tiles and compact the absorbed ones); `chains` — components
    spaced just inside the merge distance along lines, so decisions wait on
    long chains of undecided predecessors (many rounds); `single` — one
    component; `nonfinite` — a NaN mean (the single-workgroup fallback);
    `zero_weights` — particles of log-weight -inf (components of weight 0);
    `near_singular` — covariances of condition ~1e6 among well-conditioned ones;
    `rank1_pairs` — nearly rank-1 covariances (condition 1e5 .. 1e8, random
    orientations) with partners along the thick axis right at the merge
    distance and along the thin axis at a few thin-axis sigmas (where the float
    LLT distance is least accurate).  Both keep the culled decision rounds
    (rounds > 1): the lattice bound holds for the float distance at any
    conditioning (phd_eap.hip k_eap_gather)."""
    import phdslam
    rng = np.random.default_rng(7)
    c = phdslam.default_config()
    c.minSeparation = 10.0
    if case == "single":
        n, per = 1, 1
    elif case == "dense":
        n, per = 512, 96
    else:
        n, per = 64, 40
    K = n * per
    maps = np.zeros(K, GAUSSIAN2D)
    if case == "dense":
        lm = rng.uniform(-20, 20, (12, 2))
        idx = rng.integers(0, 12, K)
        maps["mean"] = (lm[idx] + rng.normal(0, 0.05, (K, 2))).astype(np.float32)
    elif case == "chains":
        # minSeparation 10 (Mahalanobis) with covariance 0.1 I: merge distance
        # sqrt(10 * 0.1) = 1; consecutive components 0.9 apart along 8 lines
        t = np.arange(K) % (K // 8)
        line = np.arange(K) // (K // 8)
        maps["mean"][:, 0] = (0.9 * t - 100).astype(np.float32)
        maps["mean"][:, 1] = (5.0 * line).astype(np.float32)
    else:
        maps["mean"] = rng.uniform(-30, 30, (K, 2)).astype(np.float32)
    maps["weight"] = rng.uniform(0.2, 1.0, K).astype(np.float32)
    a = rng.uniform(0.05, 0.15, K).astype(np.float32)
    maps["cov"][:, 0] = a
    maps["cov"][:, 3] = a
    b = (0.2 * a * rng.uniform(-1, 1, K)).astype(np.float32)
    maps["cov"][:, 1] = b
    maps["cov"][:, 2] = b
    if case == "nonfinite":
        maps["mean"][K // 3, 0] = np.nan
    if case == "near_singular":
        # a few nearly rank-1 covariances (cond ~1e6, beyond the lattice margin's
        # 1e4) placed where the isotropic bound alone would cull their merges:
        # the map must take the exhaustive greedy and still equal the oracle
        k = rng.choice(K, 6, replace=False)
        maps["cov"][k, 0] = 1.0
        maps["cov"][k, 3] = 1.0
        maps["cov"][k, 1] = np.float32(1.0 - 2e-6)
        maps["cov"][k, 2] = np.float32(1.0 - 2e-6)
    if case == "rank1_pairs":
        T = c.minSeparation
        for s in range(0, K - 3, 4):
            th = rng.uniform(0, np.pi)
            u = np.array([np.cos(th), np.sin(th)])
            v = np.array([-np.sin(th), np.cos(th)])
            l1 = rng.uniform(0.05, 0.2)
            l2 = l1 * 10.0 ** rng.uniform(-8, -5)
            P = l1 * np.outer(u, u) + l2 * np.outer(v, v)
            mu = maps["mean"][s].astype(np.float64)
            offs4 = [0.0 * u, np.sqrt(T * l1) * rng.uniform(0.95, 1.05) * u,
                     np.sqrt(T * l2) * rng.uniform(0.3, 30.0) * v, np.sqrt(T * l1) * rng.uniform(0.9, 1.1) * u
                     + np.sqrt(T * l2) * rng.uniform(0.3, 3.0) * v]
            for q in range(4):
                maps["mean"][s + q] = (mu + offs4[q]).astype(np.float32)
                maps["cov"][s + q] = np.array([P[0, 0], P[1, 0], P[0, 1], P[1, 1]], np.float32)
    offs = (np.arange(n + 1) * per).astype(np.int32)
    lw = rng.normal(-np.log(n), 0.3, n).astype(np.float32)
    if case == "zero_weights":
        lw[::5] = -np.inf
    poses = np.zeros(n, POSE)
    f = _filter(c, n, map_capacity=max(per, 64), max_measurements=16, candidate_capacity=256,
                survivor_capacity=128)
    f.load(poses, lw, maps, offs)
    eap = f.expected_map()
    rounds = f.expected_map_groups()
    f.close()
    ref = pyoracle.expected_map(c, lw, maps, offs)
    _eap_compare(eap, ref, f"eap {case}")
    if case == "chains":
        assert rounds > 3, rounds
    if case in ("near_singular", "rank1_pairs"):
        assert rounds > 1, rounds  # the decision rounds, not the one-workgroup greedy
    if case == "dense":
        assert len(eap) < K // 50


def test_expected_map_config3_scale(gpu, capsys):
    """§8(f) rank 1 at the north-star scale: after a config-3 update of 4096
    particles x 512 components (CV + CPHD, bench capacities) the GPU EAP map of
    all ~2.1 M weighted components equals the oracle's greedy
    (orc_expected_map_cells: gm_reduce.cpp:59-132 with cell-restricted distance
    tests, identical outputs — tests/test_oracle_closed_form.py) in emission
    order, conserves the weighted mass, and is reproducible bit for bit.
    It takes the parallel decision rounds (the config-3 posterior holds nearly
    rank-1 covariances near the sensor, which once sent the whole map to the
    one-workgroup greedy: 15.7 s) and finishes in well under 200 ms."""
    import time
    import phdslam
    from phdslam.scenario import bench_capacities
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
    n = len(poses)
    f = _filter(c, n, **bench_capacities(3, 512, 64))
    f.load(poses, lw, maps, offs)
    f.update(z)
    f.normalize()
    f.synchronize()
    gp, gw, gm, go = f.export()
    t0 = time.perf_counter()
    eap = f.expected_map()
    t1 = time.perf_counter()
    eap2 = f.expected_map()
    groups = f.expected_map_groups()
    f.close()
    assert eap.tobytes() == eap2.tobytes()
    t2 = time.perf_counter()
    ref = pyoracle.expected_map(c, gw, gm, go, cells=True)
    t3 = time.perf_counter()
    with capsys.disabled():
        print(f"\n[eap config 3] {int(go[-1])} components -> {len(eap)} (rounds {groups}); GPU {1e3 * (t1 - t0):.1f} ms, "
              f"oracle (cells) {1e3 * (t3 - t2):.0f} ms")
    _eap_compare(eap, ref, "eap config 3")
    assert groups > 1, "the config-3 map took the one-workgroup exhaustive greedy"
    assert t1 - t0 < 0.2, f"config-3 EAP map took {1e3 * (t1 - t0):.0f} ms"
    tot = float(np.sum(np.exp(gw.astype(np.float64)) * np.add.reduceat(gm["weight"].astype(np.float64), go[:-1])))
    assert abs(eap["weight"].astype(np.float64).sum() - tot) <= 1e-4 * tot


def test_step_cphd_births_multistep_matches_oracle(gpu):
    """Config 3's CPHD step through phd_step with the step's births over four
    scans of fresh measurements (noise + 25 % clutter, as bench.py --mode
    sequence): each step predicts on the device (Philox noise, seed 1234), places
    the PREVIOUS scan's births after every map in the update's classify, updates
    and normalises (resample threshold 0: no resample).  Against the oracle's
    predict -> add_births(previous scan) -> update -> normalize from the same
    state, re-synchronised each step (maps of every particle, log-weights)."""
    import phdslam
    c, poses, lw, maps, offs, z0 = phdslam.config_scenario(3, n=64, G=96, M=24)
    c.resampleThresh = 0.0
    n = len(poses)
    cap = dict(map_capacity=384, max_measurements=24, candidate_capacity=640, survivor_capacity=192)
    rng = np.random.default_rng(11)
    scans = []
    for _ in range(4):
        zk = z0.copy()
        zk["range"] = np.abs(zk["range"] + rng.normal(0, c.stdRange, len(zk))).astype(np.float32)
        zk["bearing"] = (zk["bearing"] + rng.normal(0, c.stdBearing, len(zk))).astype(np.float32)
        clut = rng.random(len(zk)) < 0.25
        zk["range"][clut] = rng.uniform(0.5, c.maxRange, int(clut.sum()))
        zk["bearing"][clut] = rng.uniform(-np.pi, np.pi, int(clut.sum()))
        scans.append(zk)
    pyoracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    prev = None
    for k, z in enumerate(scans):
        f = _filter(c, n, **cap)
        assert f.step_births()  # (CPHD: on by default)
        f.load(poses, lw, maps, offs)
        if prev is not None:
            f.set_measurements(prev)  # the previous scan: the step's births come from it
        f.set_measurements(z)
        f.step(None, True, k)
        f.check_errors()
        gp, glw, gmaps, goffs = f.export()
        f.close()
        op = pyoracle.predict_cv(c, poses, pyoracle.noise_cv(c, n, 1234, k))
        for name in POSE.names:
            assert parity.close(gp[name], op[name], 1e-5, scale=1.0).all(), (k, name)
        bm, bo = pyoracle.add_births(c, op, maps, offs, prev) if prev is not None else (maps, offs)
        # phd_step normalised the log-weights: put the oracle's normaliser back
        _, _, odelta, _ = pyoracle.update(c, op, bm, bo, z)
        ou = (lw + odelta).astype(np.float32)
        on, _ = pyoracle.normalize(ou)
        norm = float(np.float64(ou[0]) - np.float64(on[0]))
        _compare_with_oracle(c, op, lw, bm, bo, z, ((glw + norm).astype(np.float32), gmaps, goffs),
                             f"step {k} (births of the {'previous' if prev is not None else 'no'} scan)", 0.05)
        # re-synchronise on the oracle's state
        poses = op
        maps, offs, odelta, _ = pyoracle.update(c, op, bm, bo, z)
        lw, _ = pyoracle.normalize((lw + odelta).astype(np.float32))
        prev = z


@pytest.mark.parametrize("mode", ["explicit_off", "default"])
def test_add_births_matches_oracle(gpu, mode):
    """CPHD births through the prediction (phd_add_births; addBirths /
    birthsKernel, phdfilter.cu.bak:738-870) against the oracle, with labelled
    measurements and ragged maps.  On a context left at the default step-births
    setting the call switches the step's own births off (the pre-step-births
    loop keeps working); after phd_set_step_births(1) it is refused."""
    import phdslam
    from phdslam._lib import PHDError
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=32, G=48, M=20)
    c.labeledMeasurements = True
    z["label"][::3] = 1
    f = _filter(c, 32, map_capacity=256, max_measurements=64)
    if mode == "explicit_off":
        f.set_step_births(0)  # (explicit births: the step's own are off)
    else:
        f.set_step_births(1)
        with pytest.raises(PHDError):
            f.add_births(z)
        f.set_step_births(-1)
        assert f.step_births()
    f.load(poses, lw, maps, offs)
    f.add_births(z)
    assert not f.step_births()
    gp, gw, gm, go = f.export()
    f.close()
    om, oo = pyoracle.add_births(c, poses, maps, offs, z)
    np.testing.assert_array_equal(go, oo)
    for p_ in range(32):
        ok, worst = parity.compare_maps(om[oo[p_]:oo[p_ + 1]], gm[go[p_]:go[p_ + 1]])
        assert ok, (p_, worst)


def test_cphd_update_of_empty_maps(gpu):
    """An empty map predicts cardinality 0 with certainty: every measurement is
    clutter, Δ log w = M log λc - λc, the posterior cardinality is δ_0 (no ∞ - ∞)."""
    import phdslam
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=8, G=8, M=16)
    c.maxCardinality = 63
    empty = np.zeros(0, GAUSSIAN2D)
    offs0 = np.zeros(9, np.int32)
    f = _filter(c, 8, max_measurements=64)
    f.load(poses, lw, empty, offs0)
    f.update(z)
    gw = f.export(with_maps=False)[1]
    cn = f.cardinality_distribution()
    f.close()
    _, _, delta, _, ocn = pyoracle.update(c, poses, empty, offs0, z, cardinality=True)
    assert np.isfinite(delta).all()
    assert parity.close(gw, lw + delta, 1e-5, floor=1e-5).all()
    assert np.all(np.abs(cn[:, 0]) < 1e-6) and np.all(cn[:, 1:] < -1e30)


def _run_driver(tmp_path, tag, steps, n, device_loop, filter_type=0, map_estimate=2, extra=""):
    """The run_synth driver (csrc/phdslam_run.cpp) on the reference's shipped data
    formats (tests/golden/config1_data.npz rewritten as comma-separated controls
    and range/bearing pair lines), as a child process (started, not exec'd)."""
    import subprocess
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1_data.npz"))
    data = tmp_path / f"data_{tag}"
    data.mkdir()
    with open(data / "controls.txt", "w") as f:
        for v, a in d["controls"][:steps].astype(np.float64):
            f.write(f"{float(v)!r}, {float(a)!r}\n")
    mo = d["meas_offsets"]
    with open(data / "measurements.txt", "w") as f:
        for s_ in range(steps):
            f.write(" ".join(repr(float(x)) for x in d["meas"][mo[s_]:mo[s_ + 1]].ravel()) + "\n")
    cfg = tmp_path / f"run_{tag}.cfg"
    cfg.write_text("motion_type = 1\nmax_range = 50\nmax_bearing = 3.141593\nstd_range = 0.25\n"
                   "std_bearing = 0.008727\nclutter_rate = 20\npd = 0.95\nl = 1.415\nh = 0.38\na = 1.89\n"
                   "b = 0.5\nstd_encoder = 1\nstd_alpha = 0.034907\n"
                   f"filter_type = {filter_type}\nfeature_model = 0\nparticle_weighting = 0\n"
                   f"n_particles = {n}\nbirth_weight = 0.0001\nmin_separation = 10\n"
                   f"min_feature_weight = 0.000001\nmap_estimate = {map_estimate}\nmax_cardinality = 63\n"
                   f"{extra}data_directory = {data}/\n")
    logs = tmp_path / f"logs_{tag}"
    logs.mkdir()
    exe = os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "phdslam_run")
    cmd = [exe, str(cfg), "--log", str(logs)] + (["--device-loop"] if device_loop else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    files = sorted(os.listdir(logs))
    assert files == [f"state_estimate{t:05d}.log" for t in range(steps)]
    return logs, files, d


@pytest.mark.parametrize("device_loop", [False, True])
def test_dropin_driver_writes_state_logs(gpu, tmp_path, device_loop):
    """The run_synth driver through the C++ drop-in surface (phdPredict /
    phdUpdateSynth / recoverSlamState with the GPU EAP map) or the device loop,
    with --log: one state_estimateNNNNN.log per step in writeLog's layout
    (main.cpp:848-954)."""
    from phdslam import io
    steps, n = 12, 32
    logs, files, _ = _run_driver(tmp_path, "phd", steps, n, device_loop)
    for t in (0, steps - 1):
        st = io.read_state_log(logs / files[t])
        assert len(st["pose"]) == 6 and np.isfinite(st["pose"]).all()
        assert len(st["log_weights"]) == n and len(st["poses"]) == n
        lw = st["log_weights"]
        assert abs(np.log(np.exp(lw - lw.max()).sum()) + lw.max()) < 1e-3  # normalised
        assert (st["map_weight"] > 0).all() and len(st["map_weight"]) >= 1
        # the EAP map is a reduction of the weighted particle maps: its mass is the
        # expected feature count, finite and below the total map size
        assert 0 < st["map_weight"].sum() < 10 * len(st["map_weight"])
        assert len(st["cardinality"]) >= 1 and (st["cardinality"] == 0).all()


def test_dropin_driver_cphd_cardinality_and_modes_agree(gpu, tmp_path):
    """filter_type = 1 through both driver modes: CPHD births from the previous
    scan (addBirths), the CPHD update, the MAP estimate (map_estimate = 1).  Every
    step's cardinality line is the MAP particle's posterior log cardinality
    distribution (phd_cardinality_distribution, recomputed here in-process by the
    same C-ABI sequence), the resample indices are the real parents, and the
    drop-in (shim) mode writes the same logs as the device loop."""
    import phdslam
    from phdslam import io
    steps, n = 8, 16
    logs_d, files, d = _run_driver(tmp_path, "cphd_dev", steps, n, True, filter_type=1, map_estimate=1)
    logs_s, _, _ = _run_driver(tmp_path, "cphd_shim", steps, n, False, filter_type=1, map_estimate=1)
    # in-process replay of the device loop through the Python C-ABI binding, same cfg file
    c = phdslam.load_config(tmp_path / "run_cphd_dev.cfg")[0]
    assert c.filterType == 1 and c.maxCardinality == 63
    f = _filter(c, n, map_capacity=1024, candidate_capacity=2048)
    f.set_seed(0x5eed5eed)
    f.set_step_births(0)  # (the separate calls with explicit births: the shim's order)
    f.load(np.zeros(n, POSE), np.full(n, -np.log(np.float32(n)), np.float32), np.zeros(0, GAUSSIAN2D),
           np.zeros(n + 1, np.int32))
    mo = d["meas_offsets"]

    def Z(k):
        zz = d["meas"][mo[k]:mo[k + 1]]
        z = np.zeros(len(zz), MEASUREMENT)
        z["range"], z["bearing"] = zz[:, 0], zz[:, 1]
        return z

    for t in range(steps):
        if t > 0:
            v, a = d["controls"][t - 1]
            f.predict_ackerman(float(v), float(a), noise=None, step=t - 1)
            f.add_births(Z(t - 1))
        f.set_measurements(Z(t))
        f.update()
        f.normalize()
        w = f.export(with_maps=False)[1]
        cn = f.cardinality_distribution()
        mi = int(np.argmax(w))
        stv = io.read_state_log(logs_d / files[t])
        sts = io.read_state_log(logs_s / files[t])
        assert len(stv["cardinality"]) == 64
        fin = cn[mi] > -60
        assert parity.close(stv["cardinality"][fin], cn[mi][fin], 1e-5, floor=1e-4).all(), f"step {t}: cardinality"
        assert np.all(stv["cardinality"][~fin] < -50)
        ps = np.exp(stv["cardinality"] - stv["cardinality"].max())
        assert np.isfinite(ps).all() and ps.sum() > 0
        # both driver modes: same weights, poses, cardinality, parents
        for k in ("log_weights", "poses", "cardinality", "pose"):
            a_, b_ = stv[k], sts[k]
            ok = np.isclose(a_, b_, rtol=1e-4, atol=1e-4) | ((a_ < -50) & (b_ < -50))
            assert ok.all(), f"step {t}: {k} differs between driver modes"
        np.testing.assert_array_equal(stv["resample_idx"], sts["resample_idx"])
        nEff = 1.0 / np.sum(np.exp(2 * w.astype(np.float64))) / n
        if nEff <= c.resampleThresh:
            idx = f.resample(uniforms=None, step=t)
            np.testing.assert_array_equal(stv["resample_idx"], idx)
        else:
            assert (stv["resample_idx"] == np.arange(n)).all()
    f.close()


def test_dropin_driver_n_predict_particles_modes_agree(gpu, tmp_path):
    """n_predict_particles = 2 through both driver modes: the shim duplicates the
    host SynthSLAM (phdfilter.cu:1185-1238), the device loop spawns children by
    slab reference; the live set doubles per step until it exceeds 5 x
    n_particles, when the resample draws n_particles again (main.cpp:1286).
    Both modes log the same live counts, weights, poses and parents."""
    from phdslam import io
    steps, n = 7, 16
    extra = "n_predict_particles = 2\nresample_threshold = 0.0\n"
    logs_d, files, _ = _run_driver(tmp_path, "npp_dev", steps, n, True, extra=extra)
    logs_s, _, _ = _run_driver(tmp_path, "npp_shim", steps, n, False, extra=extra)
    sizes = []
    for t in range(steps):
        stv = io.read_state_log(logs_d / files[t])
        sts = io.read_state_log(logs_s / files[t])
        sizes.append(len(stv["log_weights"]))
        for k in ("log_weights", "poses", "pose"):
            assert stv[k].shape == sts[k].shape, (t, k)
            assert np.isclose(stv[k], sts[k], rtol=1e-4, atol=1e-4).all(), f"step {t}: {k} differs"
        np.testing.assert_array_equal(stv["resample_idx"], sts["resample_idx"])
    # step 0 has no predict; 16 -> 32 -> 64 -> 128 (> 80: resampled to 16 after logging) -> 32 ...
    assert sizes == [16, 32, 64, 128, 32, 64, 128], sizes
