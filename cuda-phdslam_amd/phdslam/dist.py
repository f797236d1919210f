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
  3. migration plan (plan_migration, identical on every rank): children of a
     local parent stay local; only the imbalance moves.  Surplus children are
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


def exchange(dist, plan, world, rank, record_bytes, pack, unpack, device):
    """Move surplus particles: pack -> all_to_all_single -> unpack.

    pack(local_idx_array) -> uint8 tensor of len(idx)*record_bytes (on `device`)
    unpack(records_uint8, n_records) places them in slots len(keep)...
    Returns the number of received records.
    """
    import torch
    send_counts = [len(plan["send"].get(d, ())) for d in range(world)]
    recv_counts = [plan["recv"].get(s, 0) for s in range(world)]
    if sum(send_counts) == 0 and sum(recv_counts) == 0:
        # every rank computes the same plan, so all ranks skip together
        return 0
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
        self.record_bytes = f.record_bytes()
        self.stats = {"resamples": 0, "migrated": 0}
        self.seed = seed  # shared by all ranks: identical resample uniforms
        self.new_logw = float(np.float32(-np.log(self.N)))
        self._plan = None
        f.set_index_offset(self.rank * self.n)

    # The step is split into phases around its two collectives so the same code
    # runs under torch.distributed (step) and under a single-process emulation of
    # several ranks (tests/test_gpu_parity.py::test_sharded_step_matches_single_context).
    def local_update(self, control, k):
        """predict + update of the local shard; log-weights into w_local (device)."""
        f = self.f
        if control is not None:
            f.predict_ackerman(control[0], control[1], noise=None, step=k)
        else:
            f.predict_cv(noise=None, step=k)
        f.update()
        f.copy_log_weights_to(self.w_local.data_ptr())

    def resample_plan(self, k):
        """After the all-gather into w_all: global normalise / nEff / parents (identical on
        every rank) and this rank's migration plan.  Returns (neff, resampled)."""
        neff, resample = self.f.global_resample(self.w_all.data_ptr(), self.N, self.rank * self.n, self.seed, k,
                                                self.parents.data_ptr())
        self._plan = None
        if resample:
            parents = self.parents.cpu().numpy()
            self._plan = plan_migration(parents, self.n, self.world)[self.rank]
        return neff, resample

    def migrate_out(self):
        """Pack outgoing particles, remap the kept ones locally.  Returns
        (sendbuf, send_counts, recv_counts) in records for all_to_all_single."""
        import torch
        plan = self._plan
        keep = plan["keep"]
        send_counts = [len(plan["send"].get(d, ())) for d in range(self.world)]
        recv_counts = [plan["recv"].get(s, 0) for s in range(self.world)]
        sendbuf = None
        if sum(send_counts):
            idx = np.concatenate([plan["send"][d] for d in range(self.world) if send_counts[d]])
            sendbuf = self._pack(idx)  # before the local remap changes the store
        if sendbuf is None:
            sendbuf = torch.empty(0, dtype=torch.uint8, device=self.device)
        full = np.empty(self.n, np.int32)
        full[:len(keep)] = keep
        full[len(keep):] = 0  # placeholders, overwritten by the unpacked migrants
        idx_dev = torch.from_numpy(full).to(self.device)
        self.f.apply_resample(idx_dev.data_ptr(), self.new_logw)
        self.stats["migrated"] += int(sum(send_counts))
        self.stats["resamples"] += 1
        return sendbuf, send_counts, recv_counts

    def migrate_in(self, recvbuf, n_recv):
        """Unpack received particles into the slots after the kept ones."""
        import torch
        if n_recv:
            keep = len(self._plan["keep"])
            dst = torch.arange(keep, keep + n_recv, dtype=torch.int32, device=self.device)
            self.f.unpack(recvbuf.data_ptr(), dst.data_ptr(), n_recv)
            self.f.fill_log_weights(self.new_logw)
            torch.cuda.current_stream(self.device).synchronize()

    def step(self, control, k):
        import torch
        self.local_update(control, k)
        self.dist.all_gather_into_tensor(self.w_all, self.w_local)
        neff, resample = self.resample_plan(k)
        if not resample:
            return neff, False
        sendbuf, send_counts, recv_counts = self.migrate_out()
        if sum(send_counts) or sum(recv_counts):
            recvbuf = torch.empty(sum(recv_counts) * self.record_bytes, dtype=torch.uint8, device=self.device)
            self.dist.all_to_all_single(recvbuf, sendbuf, [c * self.record_bytes for c in recv_counts],
                                        [c * self.record_bytes for c in send_counts])
            self.migrate_in(recvbuf, sum(recv_counts))
        return neff, True

    def _pack(self, local_idx):
        import torch
        idx = torch.from_numpy(np.ascontiguousarray(local_idx, np.int32)).to(self.device)
        buf = torch.empty(len(local_idx) * self.record_bytes, dtype=torch.uint8, device=self.device)
        self.f.pack(idx.data_ptr(), len(local_idx), buf.data_ptr())
        torch.cuda.current_stream(self.device).synchronize()
        return buf
