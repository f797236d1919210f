"""Run the GPU update on parity scenarios and dump raw outputs (for offline diagnosis vs the oracle)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
import phdslam  # noqa: E402

out = os.path.join(REPO, "gpurun_out")
os.makedirs(out, exist_ok=True)
for tag, cid, n, G, M in [("a", 2, 64, 64, 32), ("b", 2, 32, 512, 64)]:
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n, G=G, M=M)
    f = phdslam.PHDFilter(n, c, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024)
    f.load(poses, lw, maps, offs)
    f.update(z)
    gp, glw, gmaps, goffs = f.export()
    f.close()
    np.savez(os.path.join(out, f"dump_{tag}.npz"), lw=glw, maps=gmaps.view(np.uint8), offs=goffs)
    print(tag, "ok", len(gmaps))
