"""Multi-rank sharding logic on CPU (gloo, world_size 2 and 3).

The GPU path (bench.py --gpus N under torchrun) runs phdslam.dist.ShardedFilter,
whose transport (TorchComm: the fixed-block all-to-all and the point-to-point
overflow exchange at overflow_slices' positions) is exercised here on a real
gloo group with a numpy mock of the particle store whose records carry the
parent's global id: after the exchange every rank holds exactly the children
the global parent list assigns (as a multiset), with only the imbalance moving.
plan_migration is the host statement of the device plan (k_shard_tail).
"""
import os
import socket

import numpy as np
import pytest

from phdslam.dist import TorchComm, migration_counts, overflow_slices, plan_migration


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


def _worker(rank, world, port, n, parents, K, out):
    """One rank of the sharded step's transport: the fixed blocks of K records per
    peer go through TorchComm.all_to_all_equal, the records beyond them through
    TorchComm.exchange at the positions overflow_slices gives (the layout of
    k_pack_blocks / k_unpack_blocks); the particle store is a numpy mock whose
    records carry the parent's global id."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = TorchComm(dist, torch.device("cpu"))
    RB = 16  # record bytes: int64 global id + padding
    store = np.arange(rank * n, rank * n + n, dtype=np.int64)
    plans = plan_migration(parents, n, world)
    plan = plans[rank]
    snd = [len(plan["send"].get(d, ())) for d in range(world)]
    rcv = [plan["recv"].get(s, 0) for s in range(world)]
    # sender: record r for rank d -> block d slot r, or the overflow buffer
    blocks = np.zeros((world, K, 2), np.int64)
    ovf = []
    for d in range(world):
        ids = store[plan["send"].get(d, np.zeros(0, np.int32))]
        blocks[d, :min(K, len(ids)), 0] = ids[:K]
        ovf.extend(ids[K:].tolist())
    ovf_send = torch.zeros(max(len(ovf), 1) * RB, dtype=torch.uint8)
    if ovf:
        o = np.zeros((len(ovf), 2), np.int64)
        o[:, 0] = ovf
        ovf_send[:len(ovf) * RB] = torch.from_numpy(o.view(np.uint8).ravel().copy())
    send_blocks = torch.from_numpy(blocks.view(np.uint8).ravel().copy())
    recv_blocks = torch.zeros_like(send_blocks)
    comm.all_to_all_equal(recv_blocks, send_blocks)
    sends, recvs = overflow_slices(snd, rcv, K, RB)
    ovf_recv = torch.zeros(max(sum(max(c - K, 0) for c in rcv), 1) * RB, dtype=torch.uint8)
    comm.exchange([(d, ovf_send[lo:hi]) for d, lo, hi in sends], [(s_, ovf_recv[lo:hi]) for s_, lo, hi in recvs])
    rb = recv_blocks.numpy().view(np.int64).reshape(world, K, 2)
    ro = ovf_recv.numpy().view(np.int64).reshape(-1, 2)
    new_store = np.empty(n, np.int64)
    nk = len(plan["keep"])
    new_store[:nk] = store[plan["keep"]]
    pos, op = nk, 0
    for s_ in range(world):  # records in source-rank order, block first, then overflow
        c = rcv[s_]
        new_store[pos:pos + min(c, K)] = rb[s_, :min(c, K), 0]
        pos += min(c, K)
        x = max(c - K, 0)
        new_store[pos:pos + x] = ro[op:op + x, 0]
        pos += x
        op += x
    assert pos == n
    gathered = [torch.zeros(n, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(new_store))
    if rank == 0:
        out.put(torch.cat(gathered).numpy().tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,K", [(2, 2), (3, 1), (3, 0), (4, 64)])
def test_sharded_transport_over_gloo(world, K):
    """The transport ShardedFilter.step uses (TorchComm + overflow_slices) on a
    real gloo process group: after the fixed-block all-to-all and the overflow
    exchange every rank holds exactly the children the global parent list
    assigns (as a multiset).  K = 0 sends everything by overflow; K = 64 nothing."""
    import torch.multiprocessing as mp
    n = 12
    rng = np.random.default_rng(world + K)
    N = world * n
    w = rng.exponential(1.0, N) ** 4
    parents = np.minimum(np.searchsorted(np.cumsum(w / w.sum()), (np.arange(N) + rng.random(N)) / N), N - 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, parents, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(res) == sorted(parents.tolist())


def test_overflow_slices_pair_up():
    """Sender and receiver derive the same overflow pairs and byte sizes."""
    rng = np.random.default_rng(3)
    world, K, RB = 5, 2, 24
    counts = rng.integers(0, 7, (world, world))  # counts[s, d] records s -> d
    np.fill_diagonal(counts, 0)
    per = [overflow_slices(counts[r], counts[:, r], K, RB) for r in range(world)]
    for s_ in range(world):
        for d, lo, hi in per[s_][0]:
            match = [(lo2, hi2) for src, lo2, hi2 in per[d][1] if src == s_]
            assert len(match) == 1 and match[0][1] - match[0][0] == hi - lo == (counts[s_, d] - K) * RB


def test_group_overflow_slices_match_dist(built):
    """The C++ multi-GPU host (include/phd_group.h, libphdslam_group.so: one
    process driving N GPUs over RCCL) places the records beyond the fixed blocks
    exactly where phdslam.dist.overflow_slices does (the layout of k_pack_blocks /
    k_unpack_blocks), for random per-peer record counts at world 1..8.  Run in a
    child process: the group library links RCCL, which this (torch) process must
    not load twice."""
    import json
    import subprocess
    import sys
    REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(REPO, "cuda-phdslam_amd", "phdslam", "libphdslam_group.so")
    if not os.path.exists(lib):
        pytest.skip("libphdslam_group.so not built")
    rng = np.random.default_rng(5)
    cases = []
    for world in (1, 2, 3, 8):
        for _ in range(6):
            cases.append((world, rng.integers(0, 9, world).tolist(), rng.integers(0, 9, world).tolist(),
                          int(rng.integers(0, 5)), int(rng.integers(1, 4000))))
    prog = r'''
import ctypes, json, sys
L = ctypes.CDLL(sys.argv[1])
out = []
for world, snd, rcv, K, rb in json.loads(sys.argv[2]):
    S = (ctypes.c_longlong * (3 * world))(); R = (ctypes.c_longlong * (3 * world))()
    ns, nr = ctypes.c_int(), ctypes.c_int()
    rc = L.phd_group_overflow_slices(world, (ctypes.c_int * world)(*snd), (ctypes.c_int * world)(*rcv), K,
                                     ctypes.c_size_t(rb), S, ctypes.byref(ns), R, ctypes.byref(nr))
    out.append([rc, [list(S[3 * i:3 * i + 3]) for i in range(ns.value)], [list(R[3 * i:3 * i + 3]) for i in range(nr.value)]])
print(json.dumps(out))
'''
    r = subprocess.run([sys.executable, "-c", prog, lib, json.dumps(cases)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout)
    for (world, snd, rcv, K, rb), (rc, S, R) in zip(cases, got):
        assert rc == 0
        es, er = overflow_slices(snd, rcv, K, rb)
        assert [tuple(x) for x in S] == [(d, lo, hi - lo) for d, lo, hi in es]
        assert [tuple(x) for x in R] == [(s, lo, hi - lo) for s, lo, hi in er]
