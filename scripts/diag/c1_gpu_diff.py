"""Diagnostic (GPU box): config 1's loop (oracle/config1_loop.py) for S scans,
the GPU update of each scan from the oracle's state against the oracle's,
listing every particle whose map differs (size, or components without a
partner within the tolerance) with the components that differ.
    python scripts/diag/c1_gpu_diff.py S [out.json]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-phdslam_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import phdslam  # noqa: E402
import pyoracle  # noqa: E402
import parity  # noqa: E402
import config1_loop as L  # noqa: E402

S = int(sys.argv[1])
c = phdslam.preset(1)[0]
controls, zs = L.load_scans()
n = 64
f = phdslam.PHDFilter(n, c, map_capacity=1024, max_measurements=256, candidate_capacity=1600, survivor_capacity=1024)
f.set_seed(5)
st = L.initial_state(n)
bad = []
for s in range(S):
    poses, lw, maps, offs = st
    nxt, rec = L.step(c, st, controls, zs, s, 5)
    if len(zs[s]):
        f.load(rec["pred"], lw, maps, offs)
        f.set_measurements(zs[s])
        f.update()
        status = f.status() if hasattr(f, "status") else None
        _, glw, gm, go = f.export()
        om, oo, od, mg = pyoracle.update(c, rec["pred"], maps, offs, zs[s])
        ncls, npm = pyoracle.near_counts()
        for p in range(n):
            A = om[oo[p]:oo[p + 1]]
            B = gm[go[p]:go[p + 1]]
            if len(A) == len(B) and parity.compare_maps(A, B)[0]:
                continue
            ua = []
            ub = []
            used = np.zeros(len(B), bool)
            for i in range(len(A)):
                hit = -1
                for j in range(len(B)):
                    if used[j]:
                        continue
                    a, b = A[i], B[j]
                    if (abs(float(a["weight"]) - float(b["weight"])) <= 1e-5 * max(abs(float(a["weight"])), 1e-12)
                            and np.all(np.abs(a["mean"] - b["mean"]) <= 1e-5 * max(np.abs(a["mean"]).max(), 1))):
                        hit = j
                        break
                if hit < 0:
                    ua.append(i)
                else:
                    used[hit] = True
            ub = np.flatnonzero(~used).tolist()
            row = lambda X, k: {"w": float(X["weight"][k]), "mean": X["mean"][k].tolist(), "cov": X["cov"][k].tolist()}
            bad.append({"scan": s, "particle": p, "sizes": [len(A), len(B)], "near": [int(ncls[p]), int(npm[p])],
                        "margin": float(mg[p]), "oracle_only": [row(A, k) for k in ua[:6]],
                        "gpu_only": [row(B, k) for k in ub[:6]]})
    st = nxt
    if s % 50 == 0:
        print(f"scan {s}: {len(bad)} differing particle-updates so far", flush=True)
f.close()
print(json.dumps({"scans": S, "differing": len(bad)}))
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out", "c1_gpu_diff.json")
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(bad, open(out, "w"), indent=1)
