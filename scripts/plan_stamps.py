"""Phase times of the one-launch sharded plan (k_shard_plan) at an emulated
world (diagnostic PHD_PLAN_STAMPS build: libphdslam_vpst.so).

    python scripts/plan_stamps.py [--config 3] [--world 8] [--plans 50]

Runs ShardedFilter over the in-process transport of scripts/shard_overhead.py
and reads the real-time clock stamps (100 MHz) of every plan: per workgroup
the phase-1 sums, the first wait, the CDF, the second wait, the search and the
ticket; then the last workgroup's tail (parent view, rank boundaries, keep /
remap, sender + receiver plans, pending slots, the host copy).  Prints the
mean microseconds of each phase from the launch's first stamp.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, os.path.join(REPO, "scripts"))
os.environ.setdefault("PHDSLAM_LIB", os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "libphdslam_vpst.so"))

SLOTS = 48


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--plans", type=int, default=50)
    a = ap.parse_args()
    import torch
    import phdslam
    from phdslam import _lib
    from phdslam.dist import ShardedFilter
    from phdslam.scenario import bench_capacities
    from shard_overhead import LocalComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg, n, G, M, df = phdslam.preset(a.config)
    if a.config == 4:
        n //= 8
    _, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
    f = phdslam.PHDFilter(n, cfg, device=0, **bench_capacities(a.config, G, M))
    f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    f.load(poses, lw, maps, offs)
    f.set_measurements(z)
    f.set_replay(True)
    f.set_check_each_update(False)
    sh = ShardedFilter(f, None, dev, world=a.world, rank=0, comm=LocalComm(a.world))
    motion_ack = cfg.motionType == 1
    control = (2.0, 0.05) if motion_ack else None
    _lib.check(_lib.lib().phd_debug_stamps(f.handle, None, 1), "stamps")
    B = (a.world * n + 1023) // 1024
    buf = np.zeros(n * SLOTS, np.uint64)
    blk, tail = [], []
    for k in range(a.plans + 5):
        sh.step(control, k)
        sh.flush()
        torch.cuda.synchronize()
        _lib.check(_lib.lib().phd_debug_stamps(f.handle, ctypes.c_void_p(buf.ctypes.data), 0), "stamps")
        if k < 5:
            continue
        s = buf[:B * 8 + 8].astype(np.int64)
        b = s[:B * 8].reshape(B, 8)[:, :7]
        t = s[B * 8:B * 8 + 7]
        t0 = b[:, 0].min()
        blk.append((b - t0) / 100.0)  # 100 MHz -> us
        tail.append((t - t0) / 100.0)
    blk = np.array(blk)
    tail = np.array(tail)
    names = ["start", "phase-1 sums", "wait 1", "normalise + CDF", "wait 2", "search", "ticket"]
    print(f"config {a.config}, world {a.world}: N = {a.world * n}, {B} workgroups, {len(blk)} plans (us from the first stamp)")
    for k in range(7):
        print(f"  {names[k]:18s} mean over WGs {blk[:, :, k].mean():7.2f}   first {blk[:, :, k].min(axis=1).mean():7.2f}"
              f"   last {blk[:, :, k].max(axis=1).mean():7.2f}")
    tn = ["tail start", "parent view", "rank boundaries", "keep / remap", "send + recv plans", "pending slots",
          "host copy (end)"]
    for k in range(7):
        print(f"  tail: {tn[k]:18s} {tail[:, k].mean():7.2f}")


if __name__ == "__main__":
    main()
