"""Per-phase cycle breakdown of the wave-per-particle update (PHD_STAMPS build).

    python scripts/wave_stamps.py --config 3
Stamps are s_memtime ticks taken by lane 0 of each particle's wave; read the
shares (stamps perturb the schedule by ~10 %).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
os.environ.setdefault("PHDSLAM_LIB", os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "libphdslam_stamps.so"))

import phdslam  # noqa: E402
from phdslam import _lib  # noqa: E402

SLOTS = 48
LABELS = {0: "start (pose, measurements staged)", 1: "pass 0: classify+EKF+walk", 30: "cphd: series, beta",
          31: "cphd: ESF sweep", 2: "cphd: pass 1 re-walk", 3: "weights / factors", 4: "survivor sort",
          5: "cand: non-detect", 6: "cand: detect", 7: "cand: births+near", 11: "merge: screen+bucket count",
          12: "merge: bucket scan+fill", 23: "merge: cull walk", 13: "merge: exact distances",
          19: "merge: csr", 20: "merge: lfmis", 8: "merge: emit", 9: "out-of-range + status"}

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--particles", type=int, default=0)
ap.add_argument("--kcap", type=int, default=0)
ap.add_argument("--scap", type=int, default=0)
a = ap.parse_args()
cfg, n, G, M, df = phdslam.preset(a.config)
if a.particles:
    n = a.particles
c, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
kcap = a.kcap or (1800 if a.config == 5 else G + 4 * M + 64)
scap = a.scap or (640 if a.config == 5 else max(256, 4 * M))
f = phdslam.PHDFilter(n, c, map_capacity=(G + 2 * M + 64 + 63) // 64 * 64, max_measurements=M,
                      candidate_capacity=kcap, survivor_capacity=scap)
f.set_update_threads(64)
f.load(poses, lw, maps, offs)
f.set_measurements(z)
f.set_replay(True)
f.enable_timing(16)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, None, 1), "stamps")
for k in range(6):
    f.update()
buf = np.zeros(n * SLOTS, np.uint64)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, ctypes.c_void_p(buf.ctypes.data), 0), "stamps")
ms, cnt = f.update_timing()
st = buf.reshape(n, SLOTS).astype(np.int64)
t0 = st[:, 0]
tot = st[:, 9] - t0
print(f"threads/LDS/resident {f.update_threads()}")
print(f"config {a.config}: N={n} G={G} M={M}; avg update kernel {ms / cnt:.3f} ms; per-wave cycles "
      f"mean {tot.mean():.0f} max {tot.max():.0f}")
present = [k for k in LABELS if np.mean(st[:, k] != 0) > 0.99]
keep = np.all(st[:, present] != 0, axis=1)
st, t0, tot = st[keep], t0[keep], tot[keep]
rel = {k: (st[:, k] - t0) for k in present}
order = sorted(present, key=lambda k: rel[k].mean())
prev = None
for k in order:
    if prev is None:
        prev = k
        continue
    d = st[:, k] - st[:, prev]
    print(f"  {LABELS[k]:32s} mean {d.mean():9.0f} cyc ({100 * d.mean() / tot.mean():5.1f} %)  max {d.max():9.0f}")
    prev = k
info = st[:, 10]
print(f"  candidates per particle: mean {np.mean(info >> 32):.1f} max {np.max(info >> 32)}; "
      f"listed detection terms mean {np.mean(info & 0xffffffff):.1f} max {np.max(info & 0xffffffff)}")
info = st[:, 24]
print(f"  merge: culled pairs mean {np.mean(info >> 32):.0f} max {np.max(info >> 32)}; edges mean "
      f"{np.mean(info & 0xffffffff):.0f} max {np.max(info & 0xffffffff)}")
print(f"  serial-merge fallbacks: {f.merge_fallbacks()}")
print(f"  pass loops: load+classify+EKF {st[:, 40].mean():.0f} cyc, walk {st[:, 41].mean():.0f} cyc; walk iterations "
      f"{st[:, 42].mean():.1f}, pairs {st[:, 43].mean():.0f}")
print(f"  walk split: table+terms {st[:, 44].mean():.0f}, batches {st[:, 45].mean():.0f}, tail {st[:, 46].mean():.0f} cyc")
