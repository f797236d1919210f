"""Host submission cost of phd_step at config 3 (bench.py's replay step): the
time the host spends inside K phd_step calls (no synchronisation) against the
wall time of the K steps including the GPU's completion."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-phdslam_amd"))
import phdslam  # noqa: E402
from phdslam import _lib  # noqa: E402
from phdslam.scenario import bench_capacities  # noqa: E402

c, poses, lw, maps, offs, z = phdslam.config_scenario(3)
n = len(poses)
f = phdslam.PHDFilter(n, c, **bench_capacities(3, 512, 64))
f.load(poses, lw, maps, offs)
f.set_measurements(z)
f.set_replay(True)
f.set_check_each_update(False)
lib = _lib.lib()
for k in range(20):
    lib.phd_step(f.handle, None, 1, k, None, None)
f.synchronize()
for K in (50, 300):
    calls = []
    t0 = time.perf_counter()
    for k in range(K):
        a = time.perf_counter()
        lib.phd_step(f.handle, None, 1, k, None, None)
        calls.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    f.synchronize()
    t2 = time.perf_counter()
    calls.sort()
    print(f"K={K}: host in phd_step {1e6 * (t1 - t0) / K:.1f} us/step (median call {1e6 * calls[K // 2]:.1f}, "
          f"p90 {1e6 * calls[int(0.9 * K)]:.1f}, max {1e6 * calls[-1]:.1f}); wall incl. GPU {1e6 * (t2 - t0) / K:.1f} us/step")
