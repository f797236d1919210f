"""Multi-rank sharding logic on CPU (gloo, world_size 2 and 3).

The GPU path (bench.py --gpus N under torchrun) uses the same plan_migration /
exchange code with RCCL and device tensors; here the particle store is a numpy
mock whose records carry the parent's global id, so the test can check that
after the exchange every rank holds exactly the children the global parent
list assigns (as a multiset), with only the imbalance moving.
"""
import os
import socket

import numpy as np
import pytest

from phdslam.dist import exchange, migration_counts, plan_migration


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,n,seed", [(2, 8, 0), (3, 5, 1), (4, 64, 2), (8, 16, 3)])
def test_plan_migration_multiset_and_minimal(world, n, seed):
    rng = np.random.default_rng(seed)
    N = world * n
    w = rng.exponential(1.0, N) ** 3
    parents = np.searchsorted(np.cumsum(w / w.sum()), (np.arange(N) + rng.random(N)) / N)
    parents = np.minimum(parents, N - 1)
    plans = plan_migration(parents, n, world)
    held = []
    moved = 0
    for r, p in enumerate(plans):
        recv = sum(p["recv"].values())
        assert len(p["keep"]) + recv == n
        held.extend((p["keep"] + r * n).tolist())
        for d, idx in p["send"].items():
            assert d != r
            held.extend((idx + r * n).tolist())
            moved += len(idx)
    assert sorted(held) == sorted(parents.tolist())
    # only the imbalance moves
    owner_counts = np.bincount(parents // n, minlength=world)
    assert moved == int(np.maximum(owner_counts - n, 0).sum())


@pytest.mark.parametrize("world,n,seed", [(1, 8, 0), (2, 8, 0), (3, 5, 1), (4, 64, 2), (8, 16, 3), (8, 4, 9)])
def test_migration_counts_match_plan(world, n, seed):
    """The all-to-all sizes each rank derives from the demand vector (the device
    plan's only read-back) equal plan_migration's."""
    rng = np.random.default_rng(seed)
    N = world * n
    w = rng.exponential(1.0, N) ** 4
    parents = np.minimum(np.searchsorted(np.cumsum(w / w.sum()), (np.arange(N) + rng.random(N)) / N), N - 1)
    demand = np.bincount(parents // n, minlength=world)
    for r, p in enumerate(plan_migration(parents, n, world)):
        keep, send, recv = migration_counts(demand, n, world, r)
        assert keep == len(p["keep"])
        assert send == [len(p["send"].get(d, ())) for d in range(world)]
        assert recv == [p["recv"].get(s, 0) for s in range(world)]


def _worker(rank, world, port, n, parents, out):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    RB = 16  # record bytes: int64 global id + padding
    # local store: slot -> global particle id
    store = np.arange(rank * n, rank * n + n, dtype=np.int64)
    plan = plan_migration(parents, n, world)[rank]

    def pack(idx):
        rec = np.zeros((len(idx), 2), np.int64)
        rec[:, 0] = store[idx]
        return torch.from_numpy(rec.view(np.uint8).ravel().copy())

    new_store = np.empty(n, np.int64)
    new_store[:len(plan["keep"])] = store[plan["keep"]]

    def unpack(buf, cnt):
        rec = buf.numpy().view(np.int64).reshape(cnt, 2)
        new_store[len(plan["keep"]):len(plan["keep"]) + cnt] = rec[:, 0]

    got = exchange(dist, plan, world, rank, RB, pack, unpack, "cpu")
    assert got == sum(plan["recv"].values())
    gathered = [torch.zeros(n, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(new_store))
    if rank == 0:
        out.put(torch.cat(gathered).numpy().tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_over_gloo(world):
    import torch.multiprocessing as mp
    n = 12
    rng = np.random.default_rng(world)
    N = world * n
    w = rng.exponential(1.0, N) ** 4
    parents = np.minimum(np.searchsorted(np.cumsum(w / w.sum()), (np.arange(N) + rng.random(N)) / N), N - 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, parents, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(res) == sorted(parents.tolist())
