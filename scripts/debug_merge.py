"""Compare the parallel merge against the serial greedy per particle (GPU debugging aid)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
import phdslam  # noqa: E402

cid, n, G, M = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (2, 128, 256, 32)))
threads = int(sys.argv[5]) if len(sys.argv) > 5 else 0
c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=n, G=G, M=M)
outs = []
for mode in (0, 1):
    f = phdslam.PHDFilter(n, c, map_capacity=1024, candidate_capacity=2048, survivor_capacity=1024,
                          max_measurements=max(M, 1))
    f.set_update_threads(threads)
    f.set_merge_mode(mode)
    f.load(poses, lw, maps, offs)
    f.update(z)
    print("mode", mode, "threads/lds", f.update_threads(), "fallbacks", f.merge_fallbacks())
    outs.append(f.export())
    f.close()
(_, w0, m0, o0), (_, w1, m1, o1) = outs
bad = 0
for p in range(n):
    a = m0[o0[p]:o0[p + 1]]
    b = m1[o1[p]:o1[p + 1]]
    ka = np.lexsort((a["mean"][:, 1], a["mean"][:, 0]))
    kb = np.lexsort((b["mean"][:, 1], b["mean"][:, 0]))
    same = len(a) == len(b) and np.allclose(a["mean"][ka], b["mean"][kb], rtol=1e-5, atol=1e-6) and np.allclose(
        a["weight"][ka], b["weight"][kb], rtol=1e-5, atol=1e-12)
    if not same:
        bad += 1
        if bad <= 2:
            print(f"particle {p}: sizes {len(a)} vs {len(b)}")
            A = {tuple(np.round(x, 3)) for x in a["mean"]}
            B = {tuple(np.round(x, 3)) for x in b["mean"]}
            print("  only parallel:", sorted(A - B)[:8])
            print("  only serial:  ", sorted(B - A)[:8])
print("differing particles:", bad, "of", n)
