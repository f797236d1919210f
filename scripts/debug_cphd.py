"""Diagnostic: CPHD update vs the oracle, repeated — map-size mismatches per
run for the library PHDSLAM_LIB selects (race hunting)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-phdslam_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import phdslam  # noqa: E402
import pyoracle  # noqa: E402

for (n, G, M, nmax) in [(8, 64, 16, 127), (16, 200, 40, 300), (4, 512, 64, 1023)]:
    c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=n, G=G, M=M)
    c.maxCardinality = nmax
    om, oo, od, margin, ocn = pyoracle.update(c, poses, maps, offs, z, cardinality=True)
    res = []
    for rep in range(4):
        f = phdslam.PHDFilter(n, c, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024,
                              max_measurements=M)
        f.load(poses, lw, maps, offs)
        f.update(z)
        gp, glw, gm, go = f.export()
        f.close()
        res.append(int(np.sum(np.diff(go) != np.diff(oo))))
    print(f"n{n} G{G} M{M}: size mismatches per run {res}", flush=True)
