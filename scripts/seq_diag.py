"""Sequence-mode diagnostic: merge fallbacks and update time per step at config 3
with fresh measurement sets (bench.py --mode sequence's sets)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
import phdslam  # noqa: E402
from phdslam.scenario import SEED_BASE, bench_capacities  # noqa: E402

cfgn = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg, n, G, M, _ = phdslam.preset(cfgn)
seed = SEED_BASE + cfgn
_, poses, lw, maps, offs, z = phdslam.config_scenario(cfgn, n=n, G=G, M=M, seed=seed)
f = phdslam.PHDFilter(n, cfg, **bench_capacities(cfgn, G, M))
f.set_seed(seed)
f.load(poses, lw, maps, offs)
f.set_replay(True)
rng = np.random.default_rng(seed + 1)
for k in range(8):
    zk = z.copy()
    if k:
        zk["range"] = np.abs(zk["range"] + rng.normal(0, cfg.stdRange, len(zk))).astype(np.float32)
        zk["bearing"] = (zk["bearing"] + rng.normal(0, cfg.stdBearing, len(zk))).astype(np.float32)
        clut = rng.random(len(zk)) < 0.25
        zk["range"][clut] = rng.uniform(0, cfg.maxRange, int(clut.sum()))
        zk["bearing"][clut] = rng.uniform(-np.pi, np.pi, int(clut.sum()))
    f.set_measurements(zk)
    fb0 = f.merge_fallbacks()
    f.enable_timing(1)
    f.update()
    ms, cnt = f.update_timing()
    st = f.status() if hasattr(f, "status") else None
    print(f"set {k} ({'replay' if k == 0 else 'perturbed'}): update {ms:.3f} ms, serial-merge fallbacks {f.merge_fallbacks() - fb0}",
          flush=True)
