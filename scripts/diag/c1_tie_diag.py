"""Diagnostic (GPU box): config 1 scan S, particle p — the GPU's merge
candidates against the oracle's (minSeparation ~ 0: no merge, so the output is
the candidate list), weights compared bit for bit, and the GPU's serial greedy
(phd_set_merge_mode 1) against its parallel merge and the oracle.
    python scripts/diag/c1_tie_diag.py S p [p ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-phdslam_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import phdslam  # noqa: E402
import pyoracle  # noqa: E402
import config1_loop as L  # noqa: E402

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
z = zs[S]
cap = dict(map_capacity=2048, max_measurements=256, candidate_capacity=1600, survivor_capacity=1024)


def gpu(cfg, mode=0):
    f = phdslam.PHDFilter(64, cfg, **cap)
    f.set_merge_mode(mode)
    f.load(pred, lw, maps, offs)
    f.set_measurements(z)
    f.update()
    out = f.export()
    f.close()
    return out


c0 = c.copy()
c0.minSeparation = 1e-12
g_nm = gpu(c0)
o_nm = pyoracle.update(c0, pred, maps, offs, z)
g_par = gpu(c)
g_ser = gpu(c, 1)
o = pyoracle.update(c, pred, maps, offs, z)
for p in parts:
    A = o_nm[0][o_nm[1][p]:o_nm[1][p + 1]]
    B = g_nm[2][g_nm[3][p]:g_nm[3][p + 1]]
    wa, wb = np.sort(A["weight"]), np.sort(B["weight"])
    print(f"particle {p}: candidates oracle {len(A)} gpu {len(B)}")
    if len(wa) == len(wb):
        d = np.flatnonzero(wa != wb)
        print(f"   weights differing bitwise (sorted): {len(d)}", [(float(wa[i]), float(wb[i])) for i in d[:10]])
    for name, arr in (("oracle", wa), ("gpu", wb)):
        u, cnt = np.unique(arr, return_counts=True)
        print(f"   {name} tie groups:", [(float(x), int(k)) for x, k in zip(u, cnt) if k > 1][:8])
    # order of the tied births in candidate order: the weights as the candidates come (no merge: output order =
    # seed order = candidate index order among unmerged)
    print("   oracle cand weights (first 12 births-ish):", [float(x) for x in A["weight"][-20:]])
    print("   gpu    cand weights (first 12 births-ish):", [float(x) for x in B["weight"][-20:]])
    sizes = (o[1][p + 1] - o[1][p], g_par[3][p + 1] - g_par[3][p], g_ser[3][p + 1] - g_ser[3][p])
    print(f"   merged sizes: oracle {sizes[0]} gpu parallel {sizes[1]} gpu serial {sizes[2]}")
