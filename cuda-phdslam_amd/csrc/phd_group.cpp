/*
 * phd_group.cpp — include/phd_group.h: one host process drives a
 * particle-sharded filter over N GPUs through RCCL (xGMI).  The step is
 * phdslam/dist.py's ShardedFilter.step with the torch.distributed transport
 * replaced by RCCL called directly: communicators from ncclCommInitAll (one per
 * device, this process owns them all), every collective issued for all ranks
 * inside one ncclGroupStart / ncclGroupEnd, each rank's part on that rank's
 * context stream, so kernels and transfers are ordered without host waits.
 * The host waits only in phd_shard_poll (the previous plan's counts, read back
 * asynchronously while the current update runs), as ShardedFilter does.
 * phd_group_create_rank: the same step for one process per GPU (torchrun /
 * bench.py --gpus N) — the process's rank of a world-wide communicator
 * (ncclCommInitRank from a unique id the caller distributes), so a step is one
 * C call instead of ShardedFilter's Python-issued phases.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "phd_capi.h"
#include "phd_group.h"

namespace {

thread_local std::string g_err;

int gfail(int code, const std::string& m) {
    g_err = m;
    return code;
}

struct Rank {
    phd_ctx* ctx = nullptr;
    int device = 0;
    int rank = 0;  // this shard's rank in the world-wide group
    hipStream_t st = nullptr;
    hipStream_t aux = nullptr;  // the all-gather and the plan beside part C (split updates; NULL: serial)
    ncclComm_t comm = nullptr;
    float* w_local = nullptr;  // n
    float* w_all = nullptr;    // world * n
    int* parents = nullptr;    // world * n
    int* keep_src = nullptr;   // n
    int* send_src = nullptr;   // n * max(world - 1, 1)
    int* recv_rec = nullptr;   // n
    unsigned char* send_blocks = nullptr;  // world * K * record_bytes
    unsigned char* recv_blocks = nullptr;
    unsigned char* ovf_send = nullptr;     // ovf_capacity * record_bytes
    unsigned char* ovf_recv = nullptr;     // n * record_bytes
    std::vector<long long> sends, recvs;   // overflow (peer, offset, bytes) triples of the open plan
};

}  // namespace

struct phd_group {
    int world = 0, n = 0, K = 0;  // world: ranks of the whole group (r.size(): the ranks this process drives)
    size_t rec = 0;
    int ovf_capacity = 0;
    uint64_t seed = 0;
    float new_logw = 0.f;
    bool open = false;
    bool have_ovf = false;
    std::vector<Rank> r;
    long long stats[5] = {0, 0, 0, 0, 0};
};

#define NCCLCHK(expr)                                                                      \
    do {                                                                                   \
        ncclResult_t _e = (expr);                                                          \
        if (_e != ncclSuccess) return gfail(PHD_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(_e)); \
    } while (0)
#define HIPCHKG(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) return gfail(PHD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)
#define PHDCHK(expr)                                                                       \
    do {                                                                                   \
        int _rc = (expr);                                                                  \
        if (_rc != PHD_OK) return gfail(_rc, std::string(#expr) + ": " + phd_last_error()); \
    } while (0)

extern "C" {

int phd_group_overflow_slices(int world, const int* send_records, const int* recv_records, int block_records,
                              size_t record_bytes, long long* send_slices, int* n_send, long long* recv_slices,
                              int* n_recv) {
    if (world <= 0 || !send_records || !recv_records || block_records < 0 || !send_slices || !n_send ||
        !recv_slices || !n_recv)
        return gfail(PHD_E_ARG, "bad arguments to phd_group_overflow_slices");
    int ns = 0, nr = 0;
    long long o = 0;
    for (int d = 0; d < world; d++) {
        const long long x = send_records[d] > block_records ? send_records[d] - block_records : 0;
        if (x) {
            send_slices[3 * ns] = d;
            send_slices[3 * ns + 1] = o * (long long)record_bytes;
            send_slices[3 * ns + 2] = x * (long long)record_bytes;
            ns++;
        }
        o += x;
    }
    o = 0;
    for (int s = 0; s < world; s++) {
        const long long x = recv_records[s] > block_records ? recv_records[s] - block_records : 0;
        if (x) {
            recv_slices[3 * nr] = s;
            recv_slices[3 * nr + 1] = o * (long long)record_bytes;
            recv_slices[3 * nr + 2] = x * (long long)record_bytes;
            nr++;
        }
        o += x;
    }
    *n_send = ns;
    *n_recv = nr;
    return PHD_OK;
}

static void free_rank(Rank& k) {
    (void)hipSetDevice(k.device);
    void* p[] = {k.w_local, k.w_all, k.parents, k.keep_src, k.send_src, k.recv_rec,
                 k.send_blocks, k.recv_blocks, k.ovf_send, k.ovf_recv};
    for (void* q : p)
        if (q) (void)hipFree(q);
    if (k.comm) ncclCommDestroy(k.comm);
    if (k.aux) {
        (void)hipStreamSynchronize(k.aux);
        if (k.ctx) phd_set_plan_stream(k.ctx, nullptr);
        (void)hipStreamDestroy(k.aux);
    }
}

int phd_group_destroy(phd_group* g) {
    if (!g) return PHD_OK;
    for (Rank& k : g->r) {
        (void)hipSetDevice(k.device);
        if (k.st) (void)hipStreamSynchronize(k.st);
        free_rank(k);
    }
    delete g;
    return PHD_OK;
}

/* The rank's staging buffers, its predict index offset and (split updates)
 * its plan stream. */
static int setup_rank(phd_group* g, Rank& k) {
    if (phd_set_index_offset(k.ctx, k.rank * g->n) != PHD_OK)
        return gfail(PHD_E_ARG, std::string("phd_set_index_offset: ") + phd_last_error());
    (void)hipSetDevice(k.device);
    const size_t n = (size_t)g->n, N = n * g->world, blk = (size_t)g->world * g->K * g->rec;
    auto A = [&](void** p, size_t bytes) { return hipMalloc(p, bytes ? bytes : 16) == hipSuccess; };
    const bool ok = A((void**)&k.w_local, n * 4) && A((void**)&k.w_all, N * 4) && A((void**)&k.parents, N * 4) &&
                    A((void**)&k.keep_src, n * 4) && A((void**)&k.send_src, (size_t)g->ovf_capacity * 4) &&
                    A((void**)&k.recv_rec, n * 4) && A((void**)&k.send_blocks, blk) && A((void**)&k.recv_blocks, blk) &&
                    A((void**)&k.ovf_send, (size_t)g->ovf_capacity * g->rec) && A((void**)&k.ovf_recv, n * g->rec);
    if (!ok) return gfail(PHD_E_HIP, "phd_group: hipMalloc failed");
    // a split update (CPHD, or the split PHD form) has its log-weights final
    // before part C: the all-gather and the plan run beside it on a second,
    // high-priority stream (phd_wait_logw / phd_set_plan_stream)
    int split = 0;
    if (phd_update_form(k.ctx, &split) == PHD_OK && split) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
            hipStreamCreateWithPriority(&k.aux, hipStreamNonBlocking, hi) != hipSuccess ||
            phd_set_plan_stream(k.ctx, k.aux) != PHD_OK)
            return gfail(PHD_E_HIP, "phd_group: the plan stream");
    }
    return PHD_OK;
}

int phd_group_create(phd_group** out, int world, phd_ctx* const* ctxs, const int* devices, int block_records,
                     uint64_t seed) {
    if (!out || world <= 0 || !ctxs || !devices || block_records < 0)
        return gfail(PHD_E_ARG, "bad arguments to phd_group_create");
    *out = nullptr;
    phd_group* g = new phd_group();
    g->world = world;
    g->K = block_records;
    g->seed = seed;
    g->r.resize(world);
    int n0 = -1;
    size_t rb0 = 0;
    for (int r = 0; r < world; r++) {
        int n = 0;
        size_t rb = 0;
        if (phd_ctx_info(ctxs[r], &n, nullptr) != PHD_OK || phd_record_bytes(ctxs[r], &rb) != PHD_OK) {
            delete g;
            return gfail(PHD_E_ARG, std::string("phd_group_create: ") + phd_last_error());
        }
        if (r == 0) {
            n0 = n;
            rb0 = rb;
        } else if (n != n0 || rb != rb0) {
            delete g;
            return gfail(PHD_E_ARG, "phd_group_create: shards differ in particle count or record size");
        }
        g->r[r].ctx = ctxs[r];
        g->r[r].device = devices[r];
        g->r[r].st = (hipStream_t)phd_get_stream(ctxs[r]);
    }
    g->n = n0;
    g->rec = rb0;
    g->ovf_capacity = n0 * (world > 1 ? world - 1 : 1);
    g->new_logw = (float)(-std::log((double)n0 * world));
    std::vector<ncclComm_t> comms(world);
    std::vector<int> devs(devices, devices + world);
    {
        ncclResult_t e = ncclCommInitAll(comms.data(), world, devs.data());
        if (e != ncclSuccess) {
            delete g;
            return gfail(PHD_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(e));
        }
    }
    for (int r = 0; r < world; r++) {
        g->r[r].comm = comms[r];
        g->r[r].rank = r;
        const int rc = setup_rank(g, g->r[r]);
        if (rc) {
            phd_group_destroy(g);
            return rc;
        }
    }
    *out = g;
    return PHD_OK;
}

int phd_group_unique_id(void* out, size_t bytes) {
    if (!out || bytes < sizeof(ncclUniqueId)) return gfail(PHD_E_ARG, "phd_group_unique_id: a buffer of 128 bytes");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return PHD_OK;
}

int phd_group_create_rank(phd_group** out, phd_ctx* ctx, int device, int world, int rank, const void* unique_id,
                          int block_records, uint64_t seed) {
    if (!out || !ctx || world <= 0 || rank < 0 || rank >= world || !unique_id || block_records < 0)
        return gfail(PHD_E_ARG, "bad arguments to phd_group_create_rank");
    *out = nullptr;
    int n = 0;
    size_t rb = 0;
    if (phd_ctx_info(ctx, &n, nullptr) != PHD_OK || phd_record_bytes(ctx, &rb) != PHD_OK)
        return gfail(PHD_E_ARG, std::string("phd_group_create_rank: ") + phd_last_error());
    phd_group* g = new phd_group();
    g->world = world;
    g->K = block_records;
    g->seed = seed;
    g->n = n;
    g->rec = rb;
    g->ovf_capacity = n * (world > 1 ? world - 1 : 1);
    g->new_logw = (float)(-std::log((double)n * world));
    g->r.resize(1);
    Rank& k = g->r[0];
    k.ctx = ctx;
    k.device = device;
    k.rank = rank;
    k.st = (hipStream_t)phd_get_stream(ctx);
    (void)hipSetDevice(device);
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    {
        const ncclResult_t e = ncclCommInitRank(&k.comm, world, id, rank);
        if (e != ncclSuccess) {
            delete g;
            return gfail(PHD_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
        }
    }
    const int rc = setup_rank(g, k);
    if (rc) {
        phd_group_destroy(g);
        return rc;
    }
    *out = g;
    return PHD_OK;
}

/* Poll the open plan of every rank and move the records beyond the fixed
 * blocks point to point (ShardedFilter.poll / comm.exchange). */
static int settle_poll(phd_group* g, float* neff, int* resampled) {
    g->have_ovf = false;
    if (!g->open) return PHD_OK;
    g->open = false;
    const int W = g->world;
    std::vector<int> demand(W), snd(W), rcv(W);
    for (size_t r = 0; r < g->r.size(); r++) {
        Rank& k = g->r[r];
        int pend = 0, rs = 0;
        float ne = 0.f;
        PHDCHK(phd_shard_poll(k.ctx, demand.data(), snd.data(), rcv.data(), &pend, &ne, &rs));
        if (r == 0) {
            if (neff) *neff = ne;
            if (resampled) *resampled = rs;
            if (rs) g->stats[0]++;
        }
        if (rs) {
            g->stats[1] += demand[k.rank] > g->n ? demand[k.rank] - g->n : 0;
            for (int d = 0; d < W; d++) g->stats[2] += snd[d];
        }
        for (int d = 0; d < W; d++) g->stats[3] += snd[d] > g->K ? snd[d] - g->K : 0;
        g->stats[4] += pend;
        k.sends.assign(3 * W, 0);
        k.recvs.assign(3 * W, 0);
        int ns = 0, nr = 0;
        PHDCHK(phd_group_overflow_slices(W, snd.data(), rcv.data(), g->K, g->rec, k.sends.data(), &ns, k.recvs.data(),
                                         &nr));
        k.sends.resize(3 * ns);
        k.recvs.resize(3 * nr);
        if (ns || nr) g->have_ovf = true;
    }
    if (g->have_ovf) {
        NCCLCHK(ncclGroupStart());
        for (Rank& k : g->r) {
            for (size_t i = 0; i < k.sends.size(); i += 3)
                NCCLCHK(ncclSend(k.ovf_send + k.sends[i + 1], (size_t)k.sends[i + 2], ncclUint8, (int)k.sends[i],
                                 k.comm, k.st));
            for (size_t i = 0; i < k.recvs.size(); i += 3)
                NCCLCHK(ncclRecv(k.ovf_recv + k.recvs[i + 1], (size_t)k.recvs[i + 2], ncclUint8, (int)k.recvs[i],
                                 k.comm, k.st));
        }
        NCCLCHK(ncclGroupEnd());
    }
    return PHD_OK;
}

/* After the overflow transfers: place the records, re-update their slots when
 * an update (step k) already ran on them (ShardedFilter.settle_finish). */
static int settle_finish(phd_group* g, const phd_ackerman_control* u, const uint64_t* step) {
    if (!g->have_ovf) return PHD_OK;
    for (Rank& k : g->r) {
        if (k.recvs.empty()) continue;
        PHDCHK(phd_shard_receive_overflow(k.ctx, k.ovf_recv, g->K, k.recv_rec));
        if (step) PHDCHK(phd_update_pending(k.ctx, u, 1, *step, k.w_local));
    }
    g->have_ovf = false;
    return PHD_OK;
}

int phd_group_step(phd_group* g, const phd_ackerman_control* u, uint64_t step, float* neff, int* resampled) {
    if (!g) return gfail(PHD_E_ARG, "null group");
    if (neff) *neff = 0.f;
    if (resampled) *resampled = -1;
    const int W = g->world;
    // 1. predict + update of every shard, log-weights into w_local
    for (Rank& k : g->r) PHDCHK(phd_predict_update(k.ctx, u, 1, step, k.w_local));
    // 2. settle the previous step's plan
    int rc = settle_poll(g, neff, resampled);
    if (rc) return rc;
    rc = settle_finish(g, u, &step);
    if (rc) return rc;
    // 3. all-gather of the log-weights (beside part C: on the plan stream, once
    // the log-weights are final)
    for (Rank& k : g->r)
        if (k.aux) PHDCHK(phd_wait_logw(k.ctx, k.aux));
    NCCLCHK(ncclGroupStart());
    for (Rank& k : g->r)
        NCCLCHK(ncclAllGather(k.w_local, k.w_all, (size_t)g->n, ncclFloat32, k.comm, k.aux ? k.aux : k.st));
    NCCLCHK(ncclGroupEnd());
    // 4. the global plan, identical on every rank; the fixed blocks packed
    for (Rank& k : g->r)
        PHDCHK(phd_shard_resample_async(k.ctx, k.w_all, W, k.rank, g->seed, step, k.parents, k.keep_src, k.send_src,
                                        k.recv_rec, k.send_blocks, g->K, k.ovf_send, g->ovf_capacity, g->new_logw));
    g->open = true;
    // 5. equal-split all-to-all of the blocks: block d of rank r -> rank d.  A
    // rank never sends records to itself (its own parents' children stay in
    // place: k_shard_tail), so the diagonal pair is not issued — and at world 1,
    // with no peer, neither the exchange nor the unpack (nothing can arrive)
    const size_t blk = (size_t)g->K * g->rec;
    if (blk && W > 1) {
        NCCLCHK(ncclGroupStart());
        for (Rank& k : g->r)
            for (int d = 0; d < W; d++) {
                if (d == k.rank) continue;
                NCCLCHK(ncclSend(k.send_blocks + d * blk, blk, ncclUint8, d, k.comm, k.st));
                NCCLCHK(ncclRecv(k.recv_blocks + d * blk, blk, ncclUint8, d, k.comm, k.st));
            }
        NCCLCHK(ncclGroupEnd());
    }
    // 6. received records into the deficit slots
    if (W > 1)
        for (Rank& k : g->r) PHDCHK(phd_shard_receive_blocks(k.ctx, k.recv_blocks, g->K, k.recv_rec));
    return PHD_OK;
}

int phd_group_flush(phd_group* g) {
    if (!g) return gfail(PHD_E_ARG, "null group");
    int rc = settle_poll(g, nullptr, nullptr);
    if (rc) return rc;
    rc = settle_finish(g, nullptr, nullptr);
    if (rc) return rc;
    return phd_group_synchronize(g);
}

int phd_group_synchronize(phd_group* g) {
    if (!g) return gfail(PHD_E_ARG, "null group");
    for (Rank& k : g->r) {
        HIPCHKG(hipSetDevice(k.device));
        HIPCHKG(hipStreamSynchronize(k.st));
    }
    return PHD_OK;
}

int phd_group_stats(const phd_group* g, long long* out5) {
    if (!g || !out5) return gfail(PHD_E_ARG, "null argument");
    for (int i = 0; i < 5; i++) out5[i] = g->stats[i];
    return PHD_OK;
}

const char* phd_group_last_error(void) { return g_err.c_str(); }

}  // extern "C"
