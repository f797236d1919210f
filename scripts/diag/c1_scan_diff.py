"""Diagnostic: config 1's loop (oracle/config1_loop.py) up to scan S, then one
particle's merge candidates on the oracle: the merge decisions closest to the
threshold measured in the units that matter — how far each pair's distance is
from T relative to the change one float ulp of the candidate means moves it.
    python scripts/diag/c1_scan_diff.py S particle [particle ...]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-phdslam_amd"), os.path.join(REPO, "oracle")]
import phdslam  # noqa: E402
import pyoracle  # noqa: E402
import config1_loop as L  # noqa: E402
from phdslam.types import GAUSSIAN2D  # noqa: E402

S = int(sys.argv[1])
parts = [int(x) for x in sys.argv[2:]]
c = phdslam.preset(1)[0]
controls, zs = L.load_scans()
st = L.initial_state(64)
for s in range(S):
    st, _ = L.step(c, st, controls, zs, s, 5)
poses, lw, maps, offs = st
v, al = controls[S - 1]
pred = pyoracle.predict_ackerman(c, poses, float(v), float(al), pyoracle.noise_ackerman(c, 64, 5, S))
lib = pyoracle.lib()
T = c.minSeparation
for p in parts:
    sm = maps[offs[p]:offs[p + 1]]
    so = np.array([0, len(sm)], np.int32)
    lib.orc_debug_select(0)
    om, oo, od, mg = pyoracle.update(c, pred[p:p + 1], sm, so, zs[S])
    cand = np.zeros(20000, GAUSSIAN2D)
    lib.orc_debug_candidates.restype = ctypes.c_long
    k = lib.orc_debug_candidates(ctypes.c_void_p(cand.ctypes.data), 20000)
    cand = cand[:k]
    mu = cand["mean"].astype(np.float64)
    P = cand["cov"].astype(np.float64)
    near = []
    for i in range(k):
        d_mu = mu - mu[i]
        Sg = (P + P[i]) / 2
        det = Sg[:, 0] * Sg[:, 3] - Sg[:, 1] * Sg[:, 2]
        inv0, inv3, inv12 = Sg[:, 3] / det, Sg[:, 0] / det, -(Sg[:, 1] + Sg[:, 2]) / det
        d = d_mu[:, 0] ** 2 * inv0 + d_mu[:, 0] * d_mu[:, 1] * inv12 + d_mu[:, 1] ** 2 * inv3
        # one ulp of each mean coordinate (float at |mu|) moves d by about
        ulp = np.spacing(np.maximum(np.abs(mu), np.abs(mu[i])).astype(np.float32)).astype(np.float64)
        grad = 2 * np.sqrt(np.maximum(d, 0)) * np.sqrt(np.maximum(np.abs(inv0), np.abs(inv3)))
        dd = grad * np.hypot(ulp[:, 0], ulp[:, 1]) * 2
        for j in range(i + 1, k):
            if abs(d[j] - T) < 50 * dd[j] or abs(d[j] - T) < 1e-3 * T:
                near.append((abs(d[j] - T) / max(dd[j], 1e-30), i, j, d[j], dd[j], float(np.sqrt(np.abs(P[i, 0])))))
    near.sort()
    print(f"particle {p}: {k} candidates, map {len(sm)} -> {oo[1]}, oracle margin {float(mg[0]):.3g}")
    for r in near[:8]:
        print(f"   |d-T| = {r[0]:.2f} ulp-moves  pair ({r[1]}, {r[2]})  d = {r[3]:.7f}  1-ulp move {r[4]:.3g}  sigma_i {r[5]:.3g}")
