"""Per-phase cycle breakdown of the fused update (diagnostic PHD_STAMPS build).

    python scripts/phase_stamps.py --config 3 [--threads 512]
Prints every stamp in chronological order with the mean cycles since the
previous one.  Read the SHARES, not the absolute time (stamps perturb the
schedule, ~+10 %).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
_PART_A = "--part" in sys.argv and sys.argv[sys.argv.index("--part") + 1:sys.argv.index("--part") + 2] == ["A"]
# the stamps build that records CPHD part A is its own library (-DPHD_STAMP_PART_A)
os.environ.setdefault("PHDSLAM_LIB", os.path.join(REPO, "cuda-phdslam_amd", "phdslam",
                                                  "libphdslam_stampsA.so" if _PART_A else "libphdslam_stamps.so"))

import phdslam  # noqa: E402
from phdslam import _lib  # noqa: E402

SLOTS = 52
LABELS = {0: "start (measurements staged)", 1: "classify", 2: "ekf+window table", 21: "pairs: window prefix", 25: "pairs: walk start search",
          22: "pairs: banded walk", 3: "eta + particle weight", 4: "survivor order", 5: "cand: non-detect",
          6: "cand: detect", 7: "cand: births+near", 11: "merge: lambda screen", 16: "merge: bucket count",
          17: "merge: bucket scan", 12: "merge: bucket fill", 23: "merge: cull + pair list", 13: "merge: exact distances", 18: "merge: csr scan",
          19: "merge: csr scatter", 14: "merge: list sort", 20: "merge: lfmis rounds", 8: "merge: emit",
          9: "append out-of-range + status", 28: "cphd: pass-0 walk (sums)", 26: "cphd: lambda + series S(K)",
          27: "cphd: ESF sweep", 29: "cphd: inner products, factors", 30: "cphd: beta prep",
          31: "cphd: esf T chain", 32: "cphd: esf P chain", 33: "cphd: esf wave sums", 34: "cphd: esf logs"}

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--particles", type=int, default=0)
ap.add_argument("--threads", type=int, default=0)
ap.add_argument("--part", choices=["A", "C"], default="C", help="CPHD: the launch to record (part A or part C)")
ap.add_argument("--births", type=int, default=-1, help="the step's births (-1: with the filter type, as the bench)")
a = ap.parse_args()
if a.part == "A":
    LABELS[9] = "pairs: banded walk + handoff"
cfg, n, G, M, df = phdslam.preset(a.config)
if a.particles:
    n = a.particles
c, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
from phdslam.scenario import bench_capacities  # noqa: E402
f = phdslam.PHDFilter(n, c, **bench_capacities(a.config, G, M))  # the bench's capacities (and merge lattice)
f.load(poses, lw, maps, offs)
f.set_measurements(z)
f.set_replay(True)
f.set_update_threads(a.threads)
f.set_step_births(a.births)
f.enable_timing(16)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, None, 1), "stamps")
for k in range(6):
    if f.step_births():  # (replay: the births of the replayed scan, then the update — the bench's update)
        f.predict_update(None, 0, do_predict=False)
    else:
        f.update()
buf = np.zeros(n * SLOTS, np.uint64)
_lib.check(_lib.lib().phd_debug_stamps(f.handle, ctypes.c_void_p(buf.ctypes.data), 0), "stamps")
ms, cnt = f.update_timing()
st = buf.reshape(n, SLOTS).astype(np.int64)
rt0, rt1 = st[:, 48], st[:, 49]  # the workgroups' residency, real-time clock (100 MHz)
t0 = st[:, 0]
tot = st[:, 9] - t0
print(f"threads/LDS {f.update_threads()}")
print(f"config {a.config}: N={n} G={G} M={M}; avg update kernel {ms / cnt:.3f} ms; per-WG cycles "
      f"mean {tot.mean():.0f} max {tot.max():.0f}")
present = [k for k in LABELS if k not in (10, 24, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49) and np.mean(st[:, k] != 0) > 0.99]
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
cyc = tot.astype(np.float64)
print(f"  per-WG cycles p10/p50/p90/max {np.percentile(cyc, 10):.0f} / {np.percentile(cyc, 50):.0f} / "
      f"{np.percentile(cyc, 90):.0f} / {cyc.max():.0f}; corr with candidates "
      f"{np.corrcoef(cyc, (info >> 32).astype(np.float64))[0, 1]:.2f}, with listed terms "
      f"{np.corrcoef(cyc, (info & 0xffffffff).astype(np.float64))[0, 1]:.2f}")
print(f"  candidates per particle: mean {np.mean(info >> 32):.1f} max {np.max(info >> 32)}; "
      f"listed detection terms mean {np.mean(info & 0xffffffff):.1f} max {np.max(info & 0xffffffff)}")
info = st[:, 24]
print(f"  merge: culled pairs mean {np.mean(info >> 32):.0f} max {np.max(info >> 32)}; edges mean "
      f"{np.mean(info & 0xffffffff):.0f} max {np.max(info & 0xffffffff)}")
print(f"  serial-merge fallbacks: {f.merge_fallbacks()}")
i43 = st[:, 43].astype(np.uint64)
i44 = st[:, 44].astype(np.uint64)
tests = (i43 >> np.uint64(32)).astype(np.int64)
lmx = (i43 & np.uint64(0xffffffff)).astype(np.uint32).view(np.float32)
kk = (i44 >> np.uint64(32)).astype(np.int64)
lsum = (i44 & np.uint64(0xffffffff)).astype(np.uint32).view(np.float32)
if tests.any():
    print(f"  merge cull: neighbour tests mean {tests.mean():.0f} max {tests.max()}; lambda max mean {lmx.mean():.4g}, "
          f"lambda mean {np.mean(lsum / np.maximum(kk, 1)):.4g}")
    i45 = st[:, 45].astype(np.uint64)
    steps = (i45 >> np.uint64(32)).astype(np.int64)
    wild = (i45 & np.uint64(0xffffffff)).astype(np.int64)
    # a wave step tests up to 4 entries per lane: 256 lane-tests per wave step
    print(f"  merge cull: wave steps mean {steps.mean():.1f} max {steps.max()} (balanced: {tests.mean() / 256:.1f}); "
          f"wild candidates mean {wild.mean():.1f} max {wild.max()}")
i40, i41, i42 = st[:, 40], st[:, 41], st[:, 42]
print(f"  walk: Gin mean {np.mean(i42 >> 32):.0f}; units mean {np.mean(i42 & 0xffffffff):.0f}; pass-0 pairs mean "
      f"{np.mean(i40 >> 32):.0f} (q>0 {np.mean(i40 & 0xffffffff):.0f}); pass-1 pairs mean {np.mean(i41 >> 32):.0f} "
      f"in {np.mean((i41 >> 32) > 0) * 100:.1f} % of particles")
i46, i47 = st[:, 46].astype(np.uint64), st[:, 47].astype(np.uint64)
if i46.any():
    rounds = (i46 >> np.uint64(32)).astype(np.int64)
    nact = (i46 & np.uint64(0xffffffff)).astype(np.int64)
    nclu = (i47 >> np.uint64(32)).astype(np.int64)
    nout = (i47 & np.uint64(0xffffffff)).astype(np.int64)
    print(f"  lfmis: rounds mean {rounds.mean():.2f} p90 {np.percentile(rounds, 90):.0f} max {rounds.max()}; active "
          f"candidates mean {nact.mean():.0f} max {nact.max()}")
    print(f"  emission: outputs mean {nout.mean():.0f}; clustered seeds mean {nclu.mean():.0f} max {nclu.max()}")
if (rt0 > 0).all() and (rt1 > 0).all():
    # resident workgroups over the launch (real-time clock: 10 ns ticks)
    lo, hi = rt0.min(), rt1.max()
    span = (hi - lo) * 0.01
    nb = 20
    edges = np.linspace(lo, hi, nb + 1)
    mid = 0.5 * (edges[:-1] + edges[1:])
    act = [int(np.sum((rt0 <= m) & (rt1 > m))) for m in mid]
    life = (rt1 - rt0) * 0.01
    print(f"  timeline: launch span {span:.1f} us (first start -> last end); workgroup lifetime mean {life.mean():.1f} "
          f"p90 {np.percentile(life, 90):.1f} max {life.max():.1f} us; resident workgroups per 1/{nb} of the span: {act}")
    last = np.sort(rt0)
    print(f"  timeline: last workgroup starts at {(last[-1] - lo) * 0.01:.1f} us; the launch's last 10 % of "
          f"workgroups start after {(last[int(0.9 * len(last))] - lo) * 0.01:.1f} us")
    if os.environ.get("PHD_STAMPS_NPZ"):  # the raw residency (launch order = workgroup index) for offline analysis
        np.savez(os.environ["PHD_STAMPS_NPZ"], rt0=rt0, rt1=rt1, cyc=tot)
