"""Multi-GPU particle sharding: one process per GPU, RCCL over xGMI.

Rank r owns a contiguous shard of n particles (global ids r*n .. r*n+n-1).
Predict and update are per-particle independent and run locally with no
communication.  The cross-particle steps (phdfilter.cu:3748-3755 normalise,
main.cpp:1281-1297 nEff + resample) need every log-weight:

  1. all_gather of the n unnormalised log-weights per rank (RCCL);
  2. every rank runs the same deterministic kernels on the identical gathered
     vector: global logSumExp, nEff, resample decision and the parent index of
     every one of the N = world*n strata (fixed-point CDF, phd_detmath.h), so
     no broadcast is needed and all ranks agree bit for bit;
  3. migration plan (k_migration_plan on the device; plan_migration is its host
     statement, migration_counts the all-to-all sizes every rank derives from
     the per-rank demand): children of a local parent stay local; only the
     imbalance moves.  Surplus children are
     packed as fixed-size particle records and exchanged with one
     all_to_all_single; receivers unpack them into their migration slab set.

The particle order after a resample is a permutation of the single-GPU order;
the resampled multiset of particles is the same.
"""
import numpy as np


def plan_migration(parents, n_local, world):
    """Deterministic migration plan from the global parent list.

    parents: int array (world*n_local,), parent global id of every stratum.
    Returns per-rank dicts with
      keep:  local parent indices of the children that stay (new slots 0..len-1)
      send:  {dst_rank: local parent indices to send}, in stratum order
      recv:  {src_rank: count}, received into slots len(keep).. in src-rank order
    """
    parents = np.asarray(parents, np.int64)
    owner = parents // n_local
    plans = []
    surplus = []  # per rank: parent global ids beyond the local quota
    deficit = np.zeros(world, np.int64)
    for r in range(world):
        mine = parents[owner == r]  # stratum order
        keep = mine[:n_local] - r * n_local
        surplus.append(mine[n_local:])
        deficit[r] = n_local - len(keep)
        plans.append({"keep": keep.astype(np.int32), "send": {}, "recv": {}})
    # match surplus (rank order) to deficits (rank order)
    d = 0
    for s in range(world):
        todo = surplus[s]
        pos = 0
        while pos < len(todo):
            while deficit[d] == 0:
                d += 1
            take = int(min(deficit[d], len(todo) - pos))
            chunk = todo[pos:pos + take] - s * n_local
            plans[s]["send"].setdefault(d, []).extend(chunk.tolist())
            plans[d]["recv"][s] = plans[d]["recv"].get(s, 0) + take
            deficit[d] -= take
            pos += take
    for p in plans:
        p["send"] = {k: np.array(v, np.int32) for k, v in p["send"].items()}
    assert int(deficit.sum()) == 0
    return plans


def migration_counts(demand, n_local, world, rank):
    """All-to-all counts of plan_migration from the per-rank demand alone.

    demand[s] = number of children of rank s's particles (phd_shard_resample
    returns it; identical on every rank).  Surplus children beyond n_local, in rank
    order, fill the deficits, in rank order.  Returns (keep, send_counts,
    recv_counts) for `rank`, the same as plan_migration's keep/send/recv sizes.
    """
    demand = [int(d) for d in demand]
    s0, f0 = [0], [0]  # surplus / deficit ranges of rank s: [s0[s], s0[s+1])
    for d in demand:
        s0.append(s0[-1] + max(d - n_local, 0))
        f0.append(f0[-1] + max(n_local - d, 0))
    assert s0[-1] == f0[-1], "demand does not sum to world * n_local"

    def overlap(a0, a1, b0, b1):
        return max(0, min(a1, b1) - max(a0, b0))

    send = [overlap(s0[rank], s0[rank + 1], f0[d], f0[d + 1]) for d in range(world)]
    recv = [overlap(s0[s], s0[s + 1], f0[rank], f0[rank + 1]) for s in range(world)]
    return min(demand[rank], n_local), send, recv


def exchange(dist, plan, world, rank, record_bytes, pack, unpack, device):
    """Move surplus particles: pack -> all_to_all_single -> unpack.

    pack(local_idx_array) -> uint8 tensor of len(idx)*record_bytes (on `device`)
    unpack(records_uint8, n_records) places them in slots len(keep)...
    Returns the number of received records.
    """
    import torch
    send_counts = [len(plan["send"].get(d, ())) for d in range(world)]
    recv_counts = [plan["recv"].get(s, 0) for s in range(world)]
    # no per-rank early exit: a rank with nothing to move still joins the collective
    idx = np.concatenate([plan["send"][d] for d in range(world) if send_counts[d]] or [np.zeros(0, np.int32)])
    sendbuf = pack(idx) if len(idx) else torch.empty(0, dtype=torch.uint8, device=device)
    recvbuf = torch.empty(sum(recv_counts) * record_bytes, dtype=torch.uint8, device=device)
    dist.all_to_all_single(recvbuf, sendbuf, [c * record_bytes for c in recv_counts],
                           [c * record_bytes for c in send_counts])
    n_recv = sum(recv_counts)
    if n_recv:
        unpack(recvbuf, n_recv)
    return n_recv


class ShardedFilter:
    """Weak-scaling sharded filter step over a local PHDFilter (one per GPU)."""

    def __init__(self, f, dist, device, world=None, rank=None, seed=0x9e3779b97f4a7c15):
        import torch
        self.f = f
        self.dist = dist
        self.device = device
        self.world = dist.get_world_size() if world is None else world
        self.rank = dist.get_rank() if rank is None else rank
        self.n = f.n
        self.N = self.n * self.world
        self.w_local = torch.empty(self.n, dtype=torch.float32, device=device)
        self.w_all = torch.empty(self.N, dtype=torch.float32, device=device)
        self.parents = torch.empty(self.N, dtype=torch.int32, device=device)
        self.keep_src = torch.empty(self.n, dtype=torch.int32, device=device)
        self.send_src = torch.empty(self.n * max(self.world - 1, 1), dtype=torch.int32, device=device)
        self.recv_rec = torch.empty(self.n, dtype=torch.int32, device=device)
        # record staging: a rank sends at most n*(world-1) particles (all weight
        # on its shard) and receives at most n
        self.record_bytes = f.record_bytes()
        self.send_capacity = self.n * (self.world - 1)
        self.sendbuf = torch.empty(max(self.send_capacity, 1) * self.record_bytes, dtype=torch.uint8, device=device)
        self.recvbuf = torch.empty(self.n * self.record_bytes, dtype=torch.uint8, device=device)
        self.stats = {"resamples": 0, "migrated": 0, "records": 0}
        self.seed = seed  # shared by all ranks: identical resample uniforms
        self.new_logw = float(np.float32(-np.log(self.N)))
        self._counts = None
        self._moved = 0
        # the collectives and the staging buffers are ordered on torch's current
        # stream: enqueue the context's kernels there too
        f.set_stream(torch.cuda.current_stream(device).cuda_stream)
        f.set_index_offset(self.rank * self.n)

    # The step is split into phases around its two collectives so the same code
    # runs under torch.distributed (step) and under a single-process emulation of
    # several ranks (tests/test_gpu_parity.py::test_sharded_step_matches_single_context).
    def local_update(self, control, k):
        """predict + update of the local shard (the predict fused into the update
        launch when it pays, as phd_step); log-weights into w_local (device)."""
        self.f.predict_update(control, k, self.w_local.data_ptr())

    def resample_plan(self, k):
        """After the all-gather into w_all: global normalise / nEff / parents, the
        migration plan, the packing of outgoing records and the local remap, all
        on the device (identical decisions on every rank; one read-back of nEff,
        the decision and the record counts).  Returns (neff, resampled)."""
        neff, resample, demand, snd, rcv = self.f.shard_resample(
            self.w_all.data_ptr(), self.world, self.rank, self.seed, k, self.parents.data_ptr(),
            self.keep_src.data_ptr(), self.send_src.data_ptr(), self.recv_rec.data_ptr(), self.sendbuf.data_ptr(),
            self.send_capacity, self.new_logw)
        self._counts = (demand, snd, rcv) if resample else None
        # particles moved job-wide: the same on every rank, so all ranks take or
        # skip the all-to-all together
        self._moved = sum(max(d - self.n, 0) for d in demand) if resample else 0
        return neff, resample

    def migrate_out(self):
        """Outgoing records (packed by resample_plan).  Returns (sendbuf,
        send_counts, recv_counts), counts in records, for all_to_all_single."""
        demand, send_counts, recv_counts = self._counts
        n_send = sum(send_counts)
        self.stats["migrated"] += max(demand[self.rank] - self.n, 0)
        self.stats["records"] += n_send
        self.stats["resamples"] += 1
        return self.sendbuf[:n_send * self.record_bytes], send_counts, recv_counts

    def recv_buffer(self, n_recv):
        return self.recvbuf[:n_recv * self.record_bytes]

    def migrate_in(self, recvbuf, n_recv):
        """Point the slots after the kept ones at the received records (log-weight
        already -log N)."""
        d = self._counts[0][self.rank]
        if d < self.n:
            self.f.shard_receive(recvbuf.data_ptr(), self.recv_rec.data_ptr(), self.n - d, d)

    def step(self, control, k):
        import torch
        self.local_update(control, k)
        self.dist.all_gather_into_tensor(self.w_all, self.w_local)
        neff, resample = self.resample_plan(k)
        if not resample:
            return neff, False
        sendbuf, send_counts, recv_counts = self.migrate_out()
        if self._moved:
            recvbuf = self.recv_buffer(sum(recv_counts))
            self.dist.all_to_all_single(recvbuf, sendbuf, [c * self.record_bytes for c in recv_counts],
                                        [c * self.record_bytes for c in send_counts])
            self.migrate_in(recvbuf, sum(recv_counts))
        return neff, True
