"""Diagnostic: config 5 per-GPU bench configuration, one particle's GPU map
against the oracle's, field by field (which field and how far).
    python scripts/diag/c5_particle_diff.py [particle ...]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import phdslam  # noqa: E402
from phdslam.scenario import bench_capacities  # noqa: E402
from oracle import pyoracle  # noqa: E402
import parity  # noqa: E402

parts = [int(x) for x in sys.argv[1:]] or [1025]
cfg, n0, G, M, _ = phdslam.preset(5)
n = 8192
c, poses, lw, maps, offs, z = phdslam.config_scenario(5, n=n)
cap = bench_capacities(5, G, M)
f = phdslam.PHDFilter(n, c, **cap)
f.load(poses, lw, maps, offs)
f.set_measurements(z)
f.update()
gp, glw, gmaps, goffs = f.export()
pyoracle.set_threads(16)
out = {}
for p in parts:
    sp = poses[p:p + 1]
    sm = maps[offs[p]:offs[p + 1]]
    so = np.array([0, len(sm)], offs.dtype)
    om, ooffs, odelta, margin = pyoracle.update(c, sp, sm, so, z)
    ncls, npm = pyoracle.near_counts()
    A = om[ooffs[0]:ooffs[1]]
    B = gmaps[goffs[p]:goffs[p + 1]]
    ia, ib = parity.match_maps(A, B)
    a, b = A[ia], B[ib]
    rows = []
    for k in range(len(a)):
        dw = abs(float(a["weight"][k]) - float(b["weight"][k])) / max(abs(float(a["weight"][k])), 1e-30)
        dm = np.abs(a["mean"][k].astype(np.float64) - b["mean"][k]) / max(np.abs(a["mean"][k]).max(), 1.0)
        sa = np.sqrt(abs(float(a["cov"][k][0]) * float(a["cov"][k][3])))
        dc = np.abs(a["cov"][k].astype(np.float64) - b["cov"][k]) / max(sa, 1e-30)
        worst = max(dw, dm.max(), dc.max())
        if worst > 2e-6:
            rows.append({"k": int(k), "worst": worst, "dw": dw, "dm": dm.tolist(), "dc": dc.tolist(),
                         "oracle": {"w": float(a["weight"][k]), "mean": a["mean"][k].tolist(), "cov": a["cov"][k].tolist()},
                         "gpu": {"w": float(b["weight"][k]), "mean": b["mean"][k].tolist(), "cov": b["cov"][k].tolist()}})
    out[p] = {"sizes": [len(A), len(B)], "near": [int(ncls[0]), int(npm[0])], "margin": float(margin[0]) if np.ndim(margin) else float(margin),
              "rows": sorted(rows, key=lambda r: -r["worst"])[:8]}
print(json.dumps(out, indent=1))
