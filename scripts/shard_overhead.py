"""Per-step cost of the sharded step's own structure on ONE GPU.

    python scripts/shard_overhead.py [--config 2] [--world 8] [--steps 200]

Runs the fused single-GPU step (phd_step, no host read-back) and the sync-free
sharded step (ShardedFilter.step) with an in-process stand-in for the
transport: all_gather copies this rank's log-weights into every rank slot (so
every rank looks identical and nothing migrates) and the block all-to-all
copies locally.  The difference is the sharded step's own overhead (plan
kernels, block exchange copies), i.e. what the collectives add to on top on a
real node.  `--skew s` offsets rank r's gathered log-weights by r * s, so the
plan migrates particles (this rank, the lightest, receives: records arrive in
the blocks and, beyond them, through the overflow exchange and a re-update of
the pending slots).  `host_wait_us` is the time step() spends waiting for the device per
step: the only wait is phd_shard_poll on the PREVIOUS step's plan while the
current update runs, so the device queue never drains (`gpu_idle_us`: sharded
step time minus the device time of its kernels ≈ 0).  Diagnostic.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, REPO)


class LocalComm:
    """Transport stand-in: every rank is this one.  With `skew`, rank r's slot of
    the gathered log-weights is this rank's plus r * skew, so the ranks'
    weight totals differ and the plan migrates particles (rank 0, this one,
    is the lightest: it receives)."""

    def __init__(self, world, skew=0.0):
        self.world = world
        self.skew = skew

    def all_gather(self, out, inp):
        v = out.view(self.world, -1)
        v.copy_(inp.view(1, -1).expand(self.world, -1))
        if self.skew:
            import torch
            v += self.skew * torch.arange(self.world, device=v.device, dtype=v.dtype).view(-1, 1)

    def all_to_all_equal(self, out, inp):
        if out.numel():
            out.copy_(inp)

    def exchange(self, sends, recvs):
        for (_, t), (_, u) in zip(sends, recvs):
            u.copy_(t[:u.numel()])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--particles", type=int, default=0, help="particles per rank (default: the config's per GPU)")
    ap.add_argument("--skew", type=float, default=0.0,
                    help="log-weight offset per rank slot: > 0 makes the plan migrate particles")
    a = ap.parse_args()
    import torch
    import phdslam
    from phdslam.dist import ShardedFilter
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg, n, G, M, df = phdslam.preset(a.config)
    if a.particles:
        n = a.particles
    elif a.config == 4:  # preset(4) is the 8-GPU job: per rank its 4096-particle shard
        n //= 8
    _, poses, lw, maps, offs, z = phdslam.config_scenario(a.config, n=n, G=G, M=M)
    from phdslam.scenario import bench_capacities

    def make():
        f = phdslam.PHDFilter(n, cfg, device=0, **bench_capacities(a.config, G, M))
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
    sh = ShardedFilter(f, None, dev, world=a.world, rank=0, comm=LocalComm(a.world, a.skew))
    for k in range(20):
        sh.step(control if motion_ack else None, k)
    sh.flush()
    torch.cuda.synchronize()
    wait = 0.0
    import phdslam.filter as pf
    poll = pf.PHDFilter.shard_poll

    def timed_poll(self, world):  # host time spent waiting on the previous plan's counts
        nonlocal wait
        t = time.perf_counter()
        r = poll(self, world)
        wait += time.perf_counter() - t
        return r

    pf.PHDFilter.shard_poll = timed_poll
    f.enable_timing(a.steps, stride=8)  # (sampled: the event records would add to the sharded leg only)
    t0 = time.perf_counter()
    for k in range(a.steps):
        sh.step(control if motion_ack else None, 20 + k)
    sh.flush()
    torch.cuda.synchronize()
    res["sharded_step_us"] = 1e6 * (time.perf_counter() - t0) / a.steps
    upd_ms, cnt = f.update_timing()
    pf.PHDFilter.shard_poll = poll
    res["update_kernel_us"] = round(1e3 * upd_ms / max(cnt, 1), 1)
    res["host_wait_us"] = round(1e6 * wait / a.steps, 1)
    res["sharded_minus_fused_us"] = round(res["sharded_step_us"] - res["fused_step_us"], 1)
    res["world"] = a.world
    res["config"] = a.config
    res["skew"] = a.skew
    for k in ("migrated", "records", "overflow_records", "pending_slots"):
        if k in sh.stats:
            res[k + "_per_step"] = round(sh.stats[k] / (a.steps + 20), 1)
    f.close()
    print(res)


if __name__ == "__main__":
    main()
