/*
 * phd_group.h — one host process driving a particle-sharded filter over N
 * GPUs of one node through RCCL (ncclCommInitAll + grouped calls over xGMI),
 * C ABI.  The same sync-free step as phdslam/dist.py (ShardedFilter.step),
 * for C / C++ callers of phdfilter.h / phd_capi.h that have no PyTorch:
 *
 *   per step k, every rank r (each call on rank r's context stream):
 *     1. phd_predict_update(ctx_r, u, 1, k, w_local_r)
 *     2. settle step k-1's plan: phd_shard_poll; records beyond the fixed
 *        blocks go point to point (grouped ncclSend / ncclRecv), then
 *        phd_shard_receive_overflow + phd_update_pending on the slots they feed
 *     3. ncclAllGather of the n log-weights (grouped over the ranks)
 *     4. phd_shard_resample_async (global normalise / nEff / decision /
 *        parents, identical on every rank; plan; fixed blocks packed)
 *     5. equal-split all-to-all of the blocks (grouped ncclSend / ncclRecv)
 *     6. phd_shard_receive_blocks
 *
 * The reference has no multi-GPU path (main.cpp:1446 prints the device count
 * only); this is SURVEY.md §8(e).  Built as libphdslam_group.so (it links
 * RCCL; libphdslam.so itself does not, so a PyTorch process never loads two
 * RCCL copies).
 */
#ifndef PHD_GROUP_H
#define PHD_GROUP_H
#include <stddef.h>
#include <stdint.h>

#include "phd_capi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct phd_group phd_group;

/* world contexts, ctxs[r] created on device devices[r] with the same particle
 * count n, configuration and capacities, each loaded with its shard.  The
 * group sets each context's predict index offset (r * n) and creates one RCCL
 * communicator per device (ncclCommInitAll).  seed: the resample seed shared
 * by every rank (phdslam.dist.ShardedFilter's default 0x9e3779b97f4a7c15);
 * block_records: particle records per peer in the fixed all-to-all blocks.
 * The update form (phd_set_update_form / phd_set_update_threads) must be fixed
 * before this call: the plan stream beside part C is set up only for a split
 * update found here.  A later change of form stays correct (the all-gather
 * waits on phd_wait_logw, which every form records) but loses or gains no
 * overlap until the group is re-created. */
int phd_group_create(phd_group** out, int world, phd_ctx* const* ctxs, const int* devices, int block_records,
                     uint64_t seed);
/* One process per GPU: this process's shard `ctx` (on `device`) as rank `rank`
 * of a `world`-rank group whose RCCL communicator comes from ncclCommInitRank
 * with `unique_id` — the 128 bytes phd_group_unique_id wrote on one rank, handed
 * to every rank by the caller (e.g. a torch.distributed broadcast).  Every rank
 * calls this, then phd_group_step once per step: the whole sharded step of
 * ShardedFilter (phdslam/dist.py) in one C call.  Same seed / block_records on
 * every rank; the update form is fixed before the call (as phd_group_create). */
int phd_group_unique_id(void* out, size_t bytes);
int phd_group_create_rank(phd_group** out, phd_ctx* ctx, int device, int world, int rank, const void* unique_id,
                          int block_records, uint64_t seed);
int phd_group_destroy(phd_group* g);
/* One sharded filter step (predict with control u — NULL for CV — update,
 * global normalise / nEff / resample, migration).  Returns with every rank's
 * work enqueued; *neff / *resampled (optional) receive the PREVIOUS step's plan
 * (its counts are polled here), 0 / -1 on the first step. */
int phd_group_step(phd_group* g, const phd_ackerman_control* u, uint64_t step, float* neff, int* resampled);
/* Settle the last plan (no update follows): the contexts' stores are final. */
int phd_group_flush(phd_group* g);
/* Counters over the steps so far: [0] resamples, [1] migrated particles,
 * [2] records sent, [3] records beyond the fixed blocks, [4] pending slots. */
int phd_group_stats(const phd_group* g, long long* out5);
/* Wait for every rank's stream. */
int phd_group_synchronize(phd_group* g);
/* Text of the last phd_group_* failure of this thread. */
const char* phd_group_last_error(void);

/* Host-side transport plan of the records beyond the fixed blocks (the layout
 * of k_pack_blocks / k_unpack_blocks): the sender's overflow buffer holds, per
 * destination d in rank order, its records block_records .. send_records[d]-1;
 * the receiver's, per source s in rank order, records block_records ..
 * recv_records[s]-1.  Writes (peer, byte offset, byte count) triples — at most
 * world each — and their numbers.  Pure host arithmetic (no device). */
int phd_group_overflow_slices(int world, const int* send_records, const int* recv_records, int block_records,
                              size_t record_bytes, long long* send_slices, int* n_send, long long* recv_slices,
                              int* n_recv);

#ifdef __cplusplus
}
#endif
#endif
