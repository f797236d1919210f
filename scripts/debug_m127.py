"""Debug: CPHD M=127 at 1024 threads (split path) vs 512 threads — deltas and map sizes."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import phdslam  # noqa: E402
import pyoracle  # noqa: E402

n, G, M, nmax = 4, 256, 127, 300
c, poses, lw, maps, offs, z = phdslam.config_scenario(3, n=n, G=G, M=M)
c.maxCardinality = nmax
om, oo, od, _ = pyoracle.update(c, poses, maps, offs, z)
print("oracle delta", od, "sizes", np.diff(oo))
for threads in (256, 512, 1024):
    for cell in ("0", "1"):
        os.environ["PHD_MERGE_CELL"] = cell
        f = phdslam.PHDFilter(n, c, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024,
                              max_measurements=M)
        f.set_update_threads(threads)
        f.load(poses, lw, maps, offs)
        f.update(z)
        st = None
        try:
            f.check_errors()
        except Exception as e:  # noqa: BLE001
            st = str(e)
        gp, gw, gm, go = f.export()
        print(f"threads {threads} cell {cell}: delta {gw - lw} sizes {np.diff(go)} merge fallbacks "
              f"{f.merge_fallbacks()} err {st}")
        f.close()
