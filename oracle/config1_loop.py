"""Config 1 (BASELINE.json configs[0]): the reference's run_synth loop
(/root/reference/src/main.cpp:1178-1312) over its own data files
(python/controls_synth.txt + python/measurements_synth.txt, converted to
tests/golden/config1_data.npz by tests/golden/make_golden.py), on the CPU
oracle.  TEST INFRASTRUCTURE ONLY: imported by tests/ and by bench.py's
CPU-only `--config 1` line, never by the product.

Per scan n (main.cpp:1178-1297):
  * n > 0: Ackerman predict with control n-1 (main.cpp:1232, 1244-1254;
    noise: Philox stream PREDICT, (seed, step n) — the device RNG's draws);
  * |Z| > 0: PHD update (phdUpdateSynth, main.cpp:1260-1271) and the
    normalisation it ends with (phdfilter.cu:3735-3755);
  * the G cap (below);
  * nEff = 1 / Σ exp(2 w) / N (main.cpp:1281-1284); resample when
    nEff <= resample_threshold and |Z| > 0 (main.cpp:1286-1289): stratified,
    Philox stream RESAMPLE (seed, step n), fixed-point CDF (DESIGN D5), maps
    copied by copy_particles (slamtypes.h:313-333).

The G cap (a build-documented policy: the reference
has no cap — `max_features` is parsed but unused): after the update, a map with
more than G_CAP = 64 components keeps its 64 heaviest (ties: the lower index),
in their map order.  Without it the maps of the 1 135-scan run grow with every
scan's ≈96 births."""
import os

import numpy as np

import pyoracle

G_CAP = 64
HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), "tests", "golden", "config1_data.npz")


def load_scans(path=DATA):
    """(controls (S-1, 2) float32 [v_encoder, alpha], list of S measurement sets)."""
    from phdslam.types import MEASUREMENT
    d = np.load(path)
    mo = d["meas_offsets"]
    scans = []
    for s in range(len(mo) - 1):
        zz = d["meas"][mo[s]:mo[s + 1]]
        z = np.zeros(len(zz), MEASUREMENT)
        z["range"], z["bearing"] = zz[:, 0], zz[:, 1]
        scans.append(z)
    return d["controls"], scans


def cap_maps(maps, offs, g_cap=G_CAP):
    """The G cap: each map's g_cap heaviest components (stable: ties keep the
    lower index), in map order."""
    sizes = np.diff(offs)
    if sizes.max(initial=0) <= g_cap:
        return maps, offs
    keep = []
    for p in range(len(sizes)):
        lo, hi = int(offs[p]), int(offs[p + 1])
        if hi - lo <= g_cap:
            keep.append(np.arange(lo, hi))
            continue
        w = maps["weight"][lo:hi]
        top = np.argsort(-w.astype(np.float64), kind="stable")[:g_cap]
        keep.append(lo + np.sort(top))
    idx = np.concatenate(keep) if keep else np.zeros(0, np.int64)
    out_offs = np.zeros(len(sizes) + 1, np.int32)
    out_offs[1:] = np.cumsum(np.minimum(sizes, g_cap))
    return maps[idx].copy(), out_offs


def initial_state(n):
    from phdslam.types import GAUSSIAN2D, POSE
    return (np.zeros(n, POSE), np.full(n, -np.log(n), np.float32), np.zeros(0, GAUSSIAN2D),
            np.zeros(n + 1, np.int32))


def step(cfg, state, controls, scans, s, seed, fast=False):
    """One scan of the loop from `state` = (poses, lw, maps, offs).  Returns
    (state after the scan, record) where record holds the predicted poses, the
    capped posterior before the resample, the normalised log-weights, nEff and
    the resample parents (None when no resample)."""
    poses, lw, maps, offs = state
    z = scans[s]
    n = len(poses)
    if s > 0:
        v, alpha = controls[s - 1]
        poses = pyoracle.predict_ackerman(cfg, poses, float(v), float(alpha),
                                          pyoracle.noise_ackerman(cfg, n, seed, s), fast=fast)
    pred = poses
    if len(z):
        maps, offs, delta, _ = pyoracle.update(cfg, poses, maps, offs, z, fast=fast)
        lw, _ = pyoracle.normalize((lw + delta).astype(np.float32), fast=fast)
    maps, offs = cap_maps(maps, offs)
    neff = float(pyoracle.neff(lw))
    lw_post = lw
    parents = None
    maps_post, offs_post = maps, offs
    if len(z) and neff <= cfg.resampleThresh:
        parents = pyoracle.resample_fixed(lw, pyoracle.resample_uniforms(n, seed, s))
        poses, lw, maps, offs = pyoracle.copy_particles(parents, poses, maps, offs)
    rec = dict(pred=pred, maps=maps_post, offs=offs_post, lw=lw_post, neff=neff, parents=parents)
    return (poses, lw, maps, offs), rec


def run(cfg, n=64, seed=1, scans_limit=None, fast=True, threads=1):
    """The whole loop; returns (final state, seconds, scans run, resamples)."""
    import time
    controls, scans = load_scans()
    S = len(scans) if scans_limit is None else min(scans_limit, len(scans))
    pyoracle.set_threads(threads, fast=fast)
    state = initial_state(n)
    resamples = 0
    t0 = time.perf_counter()
    for s in range(S):
        state, rec = step(cfg, state, controls, scans, s, seed, fast=fast)
        resamples += rec["parents"] is not None
    return state, time.perf_counter() - t0, S, resamples
