"""Worker of tests/test_gpu_parity.py::test_sharded_step_two_processes: one rank
of a sharded filter (phdslam.dist.ShardedFilter.step, the product's step) in
its own process on cuda:0, torch.distributed over gloo (RCCL refuses two ranks
on one GPU).  Started with torch.multiprocessing spawn (never exec).  Writes the
shard's exported state after every step to <out>/r<rank>_k<step>.npz."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(rank, world, port, n, G, M, steps, seed, out_dir, block_records, cid=2):
    sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import phdslam
    from phdslam.dist import ShardedFilter
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    c, poses, lw, maps, offs, z = phdslam.config_scenario(cid, n=world * n, G=G, M=M)
    c.resampleThresh = 1.0
    o = offs[rank * n:(rank + 1) * n + 1]
    f = phdslam.PHDFilter(n, c, device=0, map_capacity=1024, max_measurements=M, candidate_capacity=2048,
                          survivor_capacity=1024)
    f.set_seed(seed)
    f.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    f.load(poses[rank * n:(rank + 1) * n].copy(), lw[rank * n:(rank + 1) * n].copy(), maps[o[0]:o[-1]].copy(),
           (o - o[0]).astype(np.int32))
    f.set_measurements(z)
    sf = ShardedFilter(f, dist, dev, seed=seed, block_records=block_records)
    ctrl = (2.0, 0.05) if c.motionType == 1 else None  # config 3: CV predict
    for k in range(1, steps + 1):
        sf.step(ctrl, k)
        sf.flush()
        torch.cuda.synchronize()
        gp, gw, gm, go = f.export()
        cn = f.cardinality_distribution() if c.filterType == 1 else np.zeros((0, 0), np.float32)
        np.savez(os.path.join(out_dir, f"r{rank}_k{k}.npz"), poses=gp, w=gw, maps=gm, offs=go, cn=cn,
                 resampled=np.int32(sf.last[1]), migrated=np.int32(sf.stats["migrated"]))
    dist.barrier()
    f.close()
    dist.destroy_process_group()
