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
  3. migration plan (k_shard_tail on the device; plan_migration is its host
     statement, migration_counts the per-rank record counts every rank derives
     from the per-rank demand): children of a local parent stay local; only the
     imbalance moves.  Surplus children are packed as particle records into
     fixed blocks per peer and exchanged with one equal-split all_to_all_single
     per step — no host read-back sits on the step (ShardedFilter below).

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


def overflow_slices(send_records, recv_records, block_records, record_bytes):
    """Byte ranges of the records beyond the fixed blocks of a sharded step.

    The sender's overflow buffer holds, per destination d in rank order, its
    records block_records .. send_records[d]-1; the receiver's holds, per source
    s in rank order, records block_records .. recv_records[s]-1 (the layout of
    k_pack_blocks / k_unpack_blocks).  Returns ([(d, lo, hi)], [(s, lo, hi)]) in
    bytes; both sides derive the same pairs from the same global plan.
    """
    K = block_records
    sends, recvs = [], []
    o = 0
    for d, c in enumerate(send_records):
        x = max(int(c) - K, 0)
        if x:
            sends.append((d, o * record_bytes, (o + x) * record_bytes))
        o += x
    o = 0
    for s_, c in enumerate(recv_records):
        x = max(int(c) - K, 0)
        if x:
            recvs.append((s_, o * record_bytes, (o + x) * record_bytes))
        o += x
    return sends, recvs


class TorchComm:
    """The step's transport over torch.distributed (RCCL over xGMI for "nccl").

    gloo moves CPU tensors only for some collectives: with CUDA buffers under
    gloo (a functional rehearsal of N ranks on one GPU) every transfer is staged
    through host memory."""

    def __init__(self, dist, device):
        self.dist = dist
        self.stage = str(dist.get_backend()) == "gloo" and getattr(device, "type", "cpu") == "cuda"

    def _host(self, t):
        return t.cpu() if self.stage else t

    def all_gather(self, out, inp):
        if self.stage:
            o = out.cpu()
            self.dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)
        else:
            self.dist.all_gather_into_tensor(out, inp)

    def all_to_all_equal(self, out, inp):
        if out.numel() == 0:
            return
        if self.stage:
            o = out.cpu()
            self.dist.all_to_all_single(o, inp.cpu())
            out.copy_(o)
        else:
            self.dist.all_to_all_single(out, inp)

    def exchange(self, sends, recvs):
        """Point-to-point transfers of [(peer, tensor)] (only the ranks a pair
        involves take part; both sides know the pair from the global plan)."""
        if not sends and not recvs:
            return
        dist = self.dist
        sb = [(p, self._host(t)) for p, t in sends]
        rb = [(p, torch_empty_like_host(t) if self.stage else t) for p, t in recvs]
        ops = [dist.P2POp(dist.isend, t, p) for p, t in sb] + [dist.P2POp(dist.irecv, t, p) for p, t in rb]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        if self.stage:
            for (p, t), (_, h) in zip(recvs, rb):
                t.copy_(h)


def torch_empty_like_host(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype, device="cpu")


class ShardedFilter:
    """Sync-free sharded filter step over a local PHDFilter (one per GPU).

    Per step k, all on torch's current stream (collectives and kernels are
    ordered without host waits):
      1. predict + update of the local shard, log-weights into w_local;
      2. settle step k-1's plan: its counts were read back asynchronously and are
         long complete (the update of step k is running); only when a peer had
         more than `block_records` records for this rank are the rest exchanged
         point to point and their slots re-updated — else nothing happens;
      3. all_gather of the log-weights; the plan (global normalise, nEff,
         decision, parents, migration, remap; one record per distinct parent and
         destination) packs FIXED blocks of `block_records` records per peer;
      4. one equal-split all_to_all of the blocks (every step: the host never
         learns the decision before it), and the receive into the deficit slots.
    flush() settles the last plan (before reading the store on the host).
    Fix the local filter's update form (set_update_form / set_update_threads)
    before constructing: the plan stream beside part C is set up only for the
    split form found here (a later change stays correct — the all-gather waits
    on phd_wait_logw, which every form records — without the overlap).
    """

    def __init__(self, f, dist, device, world=None, rank=None, seed=0x9e3779b97f4a7c15, block_records=4, comm=None,
                 overlap=True):
        import torch
        self.f = f
        self.dist = dist
        self.device = device
        self.world = dist.get_world_size() if world is None else world
        self.rank = dist.get_rank() if rank is None else rank
        self.n = f.n
        self.N = self.n * self.world
        self.K = int(block_records)
        self.w_local = torch.empty(self.n, dtype=torch.float32, device=device)
        self.w_all = torch.empty(self.N, dtype=torch.float32, device=device)
        self.parents = torch.empty(self.N, dtype=torch.int32, device=device)
        self.keep_src = torch.empty(self.n, dtype=torch.int32, device=device)
        self.send_src = torch.empty(self.n * max(self.world - 1, 1), dtype=torch.int32, device=device)
        self.recv_rec = torch.empty(self.n, dtype=torch.int32, device=device)
        self.record_bytes = f.record_bytes()
        blk = self.world * self.K * self.record_bytes  # may be 0: every record then goes by overflow
        self.send_blocks = torch.empty(blk, dtype=torch.uint8, device=device)
        self.recv_blocks = torch.empty(blk, dtype=torch.uint8, device=device)
        # beyond the blocks: a rank sends at most n (world - 1) records, receives at most n
        self.ovf_capacity = self.n * max(self.world - 1, 1)
        self.ovf_send = torch.empty(self.ovf_capacity * self.record_bytes, dtype=torch.uint8, device=device)
        self.ovf_recv = torch.empty(self.n * self.record_bytes, dtype=torch.uint8, device=device)
        self.stats = {"resamples": 0, "migrated": 0, "records": 0, "overflow_records": 0, "pending_slots": 0}
        self.seed = seed  # shared by all ranks: identical resample uniforms
        self.new_logw = float(np.float32(-np.log(self.N)))
        self.comm = comm if comm is not None else (TorchComm(dist, device) if dist is not None else None)
        self._open = False
        self._ovf = ([], [])
        self.last = (None, None)
        f.set_stream(torch.cuda.current_stream(device).cuda_stream)
        f.set_index_offset(self.rank * self.n)
        # the all-gather and the plan on a second, high-priority stream beside the
        # update's part C (its log-weights are final after the CPHD terms / the
        # split PHD part A: phd_wait_logw); the pack waits for the plan
        self.aux = None
        if overlap and f.update_form():
            self.aux = torch.cuda.Stream(device=device, priority=-1)
            f.set_plan_stream(self.aux.cuda_stream)

    # The phases are separate methods so the same code runs under
    # torch.distributed (step) and under a single-process emulation of several
    # ranks (tests/test_gpu_parity.py::test_sharded_step_matches_single_context).
    def local_update(self, control, k):
        """predict + update of the local shard (the predict fused into the update
        launch when it pays, as phd_step); log-weights into w_local (device)."""
        self.f.predict_update(control, k, self.w_local.data_ptr())

    def poll(self):
        """Counts of the open plan (waits only for that plan's read-back).
        Returns (neff, resampled); sets the overflow transfers of settle()."""
        if not self._open:
            return self.last
        # the C side closes the plan whichever way the poll ends (a capacity error
        # included): close it here first, so both sides agree and a later settle
        # does not poll again and mask the real error
        self._open = False
        neff, rs, demand, snd, rcv, pend = self.f.shard_poll(self.world)
        if rs:
            self.stats["resamples"] += 1
            self.stats["migrated"] += max(demand[self.rank] - self.n, 0)
            self.stats["records"] += sum(snd)
        self.stats["overflow_records"] += sum(max(c - self.K, 0) for c in snd)
        self.stats["pending_slots"] += pend
        sends, recvs = overflow_slices(snd, rcv, self.K, self.record_bytes)
        self._ovf = ([(d, self.ovf_send[lo:hi]) for d, lo, hi in sends],
                     [(s_, self.ovf_recv[lo:hi]) for s_, lo, hi in recvs])
        self.last = (neff, rs)
        return self.last

    def settle_finish(self, control=None, k=None):
        """After the overflow transfers: place those records, re-update their
        slots when an update (step k) already ran on them."""
        if self._ovf[1]:
            self.f.shard_receive_overflow(self.ovf_recv.data_ptr(), self.K, self.recv_rec.data_ptr())
            if k is not None:
                self.f.update_pending(control, k, self.w_local.data_ptr())
        self._ovf = ([], [])

    def settle(self, control=None, k=None):
        out = self.poll()
        if self._ovf[0] or self._ovf[1]:
            self.comm.exchange(*self._ovf)
        self.settle_finish(control, k)
        return out

    def gather(self):
        """All-gather of the log-weights (beside part C on the plan stream)."""
        import torch
        if self.aux is None:
            self.comm.all_gather(self.w_all, self.w_local)
            return
        self.f.wait_logw(self.aux.cuda_stream)
        with torch.cuda.stream(self.aux):
            self.comm.all_gather(self.w_all, self.w_local)

    def plan(self, k):
        """After the all-gather into w_all: the global plan, the fixed send blocks,
        the local remap — enqueued, nothing read back."""
        self.f.shard_resample_async(
            self.w_all.data_ptr(), self.world, self.rank, self.seed, k, self.parents.data_ptr(),
            self.keep_src.data_ptr(), self.send_src.data_ptr(), self.recv_rec.data_ptr(), self.send_blocks.data_ptr(),
            self.K, self.ovf_send.data_ptr(), self.ovf_capacity, self.new_logw)
        self._open = True

    def receive(self):
        """After the all-to-all of the blocks into recv_blocks."""
        self.f.shard_receive_blocks(self.recv_blocks.data_ptr(), self.K, self.recv_rec.data_ptr())

    def step(self, control, k):
        """One sharded filter step.  Returns (neff, resampled) of the PREVIOUS
        step's plan — its decision is only known once that plan is polled here
        (the current step's plan is polled by the next step, or by flush()); the
        first step returns (None, None).  The device store is final only after
        flush()."""
        self.local_update(control, k)
        prev = self.settle(control, k)
        self.gather()
        self.plan(k)
        self.comm.all_to_all_equal(self.recv_blocks, self.send_blocks)
        self.receive()
        return prev

    def flush(self):
        """Settle the last plan (no update follows): the store is then final."""
        return self.settle(None, None)


class GroupRank:
    """The sharded step of ShardedFilter as ONE C call per step: this process's
    rank of an RCCL group driven by the C++ host (libphdslam_group.so,
    include/phd_group.h: phd_group_create_rank + phd_group_step).  The
    communicator is RCCL's own (ncclCommInitRank); its unique id is made on rank
    0 and broadcast over the torch.distributed group `dist`.  Same step, same
    plans, same results bit for bit as ShardedFilter (tests/test_gpu_parity.py::
    test_group_rank_matches_sharded_filter); the Python dispatch of the step's
    phases (poll, all-gather on the plan stream, plan, all-to-all, unpack) is
    gone from the step.  The local filter's update form is fixed before
    construction (phd_group.h)."""

    def __init__(self, f, dist, device, world=None, rank=None, seed=0x9e3779b97f4a7c15, block_records=4,
                 unique_id=None):
        import ctypes
        from . import _lib
        self.f = f
        self.world = dist.get_world_size() if world is None else world
        self.rank = dist.get_rank() if rank is None else rank
        self.n = f.n
        self.K = int(block_records)
        self.L = group_lib()
        if unique_id is None:
            uid = bytearray(128)
            if self.rank == 0:
                buf = (ctypes.c_char * 128).from_buffer(uid)
                _group_check(self.L, self.L.phd_group_unique_id(buf, 128), "phd_group_unique_id")
            if self.world > 1:
                obj = [bytes(uid)]
                dist.broadcast_object_list(obj, src=0)
                uid = bytearray(obj[0])
            unique_id = bytes(uid)
        self._uid = ctypes.create_string_buffer(bytes(unique_id), 128)
        f.set_stream(__import__("torch").cuda.current_stream(device).cuda_stream)
        h = ctypes.c_void_p()
        _group_check(self.L, self.L.phd_group_create_rank(ctypes.byref(h), f.handle, int(device.index or 0),
                                                         self.world, self.rank, self._uid, self.K,
                                                         ctypes.c_uint64(seed)), "phd_group_create_rank")
        self._g = h
        self.last = (None, None)
        _lib.lib()  # (the product library is loaded first: the group library resolves against it)

    def step(self, control, k):
        """One sharded step; returns the PREVIOUS step's (neff, resampled)."""
        import ctypes
        from .types import AckermanControl
        u = ctypes.byref(AckermanControl(float(control[1]), float(control[0]))) if control is not None else None
        ne, rs = ctypes.c_float(), ctypes.c_int()
        _group_check(self.L, self.L.phd_group_step(self._g, u, ctypes.c_uint64(int(k)), ctypes.byref(ne),
                                                   ctypes.byref(rs)), "phd_group_step")
        self.last = (ne.value, rs.value) if rs.value >= 0 else (None, None)
        return self.last

    def flush(self):
        _group_check(self.L, self.L.phd_group_flush(self._g), "phd_group_flush")

    @property
    def stats(self):
        import ctypes
        out = (ctypes.c_longlong * 5)()
        _group_check(self.L, self.L.phd_group_stats(self._g, out), "phd_group_stats")
        return {"resamples": out[0], "migrated": out[1], "records": out[2], "overflow_records": out[3],
                "pending_slots": out[4]}

    def close(self):
        if self._g:
            self.L.phd_group_destroy(self._g)
            self._g = None


_GROUP = None


def group_lib():
    """libphdslam_group.so (built in-tree by build.py next to libphdslam.so)."""
    global _GROUP
    if _GROUP is None:
        import ctypes
        import os
        from . import _lib
        _lib.lib()
        path = os.path.join(os.path.dirname(os.path.abspath(_lib.LIB_PATH)), "libphdslam_group.so")
        if not os.path.exists(path):
            raise OSError(f"{path} not found: build it with `python cuda-phdslam_amd/build.py`")
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        L.phd_group_unique_id.argtypes = [vp, ctypes.c_size_t]
        L.phd_group_create_rank.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                                            ctypes.c_int, ctypes.c_uint64]
        L.phd_group_step.argtypes = [vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float),
                                     ctypes.POINTER(ctypes.c_int)]
        L.phd_group_flush.argtypes = [vp]
        L.phd_group_stats.argtypes = [vp, vp]
        L.phd_group_destroy.argtypes = [vp]
        L.phd_group_last_error.restype = ctypes.c_char_p
        _GROUP = L
    return _GROUP


def _group_check(L, rc, where):
    if rc != 0:
        from ._lib import PHDError
        raise PHDError(rc, where, (L.phd_group_last_error() or b"").decode())
