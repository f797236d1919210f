"""Per-step cost of the sharded step's host-synchronised structure on ONE GPU.

    python scripts/shard_overhead.py [--config 2] [--world 8] [--steps 200]

Runs the fused single-GPU step (phd_step, no host read-back) and the sharded
step (ShardedFilter.step) with an in-process stand-in for torch.distributed:
all_gather copies this rank's log-weights into every rank slot (so every rank
looks identical and nothing migrates) and all_to_all copies locally.  The
difference is the sharded step's own overhead (plan kernel, read-back, host
logic), i.e. what the collectives add to on top on a real node.  Diagnostic.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, REPO)


class LocalDist:
    def __init__(self, world, rank=0):
        self.world, self.rank = world, rank

    def get_world_size(self):
        return self.world

    def get_rank(self):
        return self.rank

    def all_gather_into_tensor(self, out, inp):
        out.view(self.world, -1).copy_(inp.view(1, -1).expand(self.world, -1))

    def all_to_all_single(self, out, inp, out_splits, in_splits):
        n = min(out.numel(), inp.numel())
        if n:
            out[:n].copy_(inp[:n])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import torch
    import phdslam
    from phdslam.dist import ShardedFilter
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg, n, G, M, df = phdslam.preset(a.config)
    _, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
    cap = (G + 2 * M + 64 + 63) // 64 * 64

    def make():
        f = phdslam.PHDFilter(n, cfg, device=0, map_capacity=cap, max_measurements=M,
                              candidate_capacity=G + 4 * M + 64, survivor_capacity=max(256, 4 * M))
        f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        f.load(poses, lw, maps, offs)
        f.set_measurements(z)
        f.set_replay(True)
        f.set_check_each_update(False)
        return f

    control = (2.0, 0.05)
    motion_ack = cfg.motionType == 1
    res = {}
    f = make()
    for k in range(20):
        bench._step_async(f, control, motion_ack, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        bench._step_async(f, control, motion_ack, 20 + k)
    torch.cuda.synchronize()
    res["fused_step_us"] = 1e6 * (time.perf_counter() - t0) / a.steps
    f.close()
    f = make()
    sh = ShardedFilter(f, LocalDist(a.world), dev)
    for k in range(20):
        sh.step(control if motion_ack else None, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    phases = {"update": 0.0, "gather": 0.0, "plan": 0.0, "migrate": 0.0}
    for k in range(a.steps):
        sh.step(control if motion_ack else None, 20 + k)
    torch.cuda.synchronize()
    res["sharded_step_us"] = 1e6 * (time.perf_counter() - t0) / a.steps
    # host-side split of one sharded step (synchronising after each phase)
    for k in range(a.steps // 4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        sh.local_update(control if motion_ack else None, 300 + k)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sh.dist.all_gather_into_tensor(sh.w_all, sh.w_local)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        neff, rs = sh.resample_plan(300 + k)
        t3 = time.perf_counter()
        if rs:
            sendbuf, sc, rc = sh.migrate_out()
            torch.cuda.synchronize()
        t4 = time.perf_counter()
        phases["update"] += t1 - t
        phases["gather"] += t2 - t1
        phases["plan"] += t3 - t2
        phases["migrate"] += t4 - t3
    res.update({f"{k}_us": round(1e6 * v / (a.steps // 4), 1) for k, v in phases.items()})
    res["world"] = a.world
    res["config"] = a.config
    f.close()
    print(res)


if __name__ == "__main__":
    main()
