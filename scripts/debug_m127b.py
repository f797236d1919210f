"""Debug: CPHD M=127 — repeated fresh contexts of one configuration (uninitialised-memory check)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
import phdslam  # noqa: E402

n, G, M, nmax = 4, 256, 127, 300
c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=n, G=G, M=M)
c.maxCardinality = nmax
threads = int(sys.argv[1]) if len(sys.argv) > 1 else 256
keep = []
for rep in range(6):
    f = phdslam.PHDFilter(n, c, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024,
                          max_measurements=M)
    f.set_update_threads(threads)
    f.load(poses, lw, maps, offs)
    f.update(z)
    f.synchronize()
    gp, gw, gm, go = f.export()
    cn = f.cardinality_distribution()
    print(f"rep {rep} threads {threads}: delta {gw - lw} sizes {np.diff(go)} cn[:,0] {cn[:, 0]}", flush=True)
    if os.environ.get("KEEP"):
        keep.append(f)
    else:
        f.close()
