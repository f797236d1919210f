"""Per-phase cycle breakdown of the fused update (diagnostic PHD_STAMPS build).

    PHDSLAM_LIB=cuda-phdslam_amd/phdslam/libphdslam_stamps.so python scripts/phase_stamps.py --config 2
Read the SHARES, not the absolute time (stamps perturb the schedule).
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
os.environ.setdefault("PHDSLAM_LIB", os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "libphdslam_stamps.so"))
import ctypes  # noqa: E402

import phdslam  # noqa: E402
from phdslam import _lib  # noqa: E402

NAMES = ["classify", "ekf+table", "pairs+eta", "sort-surv", "cand-nondet", "cand-detect", "cand-births+near",
         "merge", "append+write"]
MNAMES = {11: "m:lambda", 12: "m:bucket+permute", 13: "m:edges", 14: "m:csr+sort"}

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--particles", type=int, default=0)
ap.add_argument("--threads", type=int, default=0)
a = ap.parse_args()
cfg, n, G, M, df = phdslam.preset(a.config)
if a.particles:
    n = a.particles
c, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
f = phdslam.PHDFilter(n, c, map_capacity=max(1024, 2 * G), max_measurements=M, candidate_capacity=G + 4 * M + 64,
                      survivor_capacity=max(256, 8 * M))
f.load(poses, lw, maps, offs)
f.set_measurements(z)
f.set_replay(True)
f.set_update_threads(a.threads)
f.enable_timing(16)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, None, 1), "stamps")
for k in range(5):
    f.update()
buf = np.zeros(n * 16, np.uint64)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, ctypes.c_void_p(buf.ctypes.data), 0), "stamps")
ms, cnt = f.update_timing()
st = buf.reshape(n, 16).astype(np.int64)
tot = st[:, 9] - st[:, 0]
print(f"threads/LDS {f.update_threads()}")
print(f"config {a.config}: N={n} G={G} M={M}; avg update kernel {ms / cnt:.3f} ms; per-WG cycles "
      f"mean {tot.mean():.0f} max {tot.max():.0f}")
prev = 0
for k, name in enumerate(NAMES):
    d = st[:, k + 1] - st[:, k]
    print(f"  {name:18s} mean {d.mean():9.0f} cyc  ({100 * d.mean() / tot.mean():5.1f} %)  max {d.max():9.0f}")
for k in (11, 12, 13, 14):
    base = st[:, 7] if k == 11 else st[:, k - 1]
    d = st[:, k] - base
    print(f"    {MNAMES[k]:16s} mean {d.mean():9.0f} cyc")
d = st[:, 8] - st[:, 14]
print(f"    {'m:lfmis+emit':16s} mean {d.mean():9.0f} cyc")
info = st[:, 10]
print(f"  candidates per particle: mean {np.mean(info >> 32):.1f} max {np.max(info >> 32)}; "
      f"listed detection terms mean {np.mean(info & 0xffffffff):.1f} max {np.max(info & 0xffffffff)}")
print(f"  serial-merge fallbacks: {f.merge_fallbacks()}")
