/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odpg_group.h — one batch classified by several MI355X devices of one node,
 * in one process.
 *
 * Packets are independent (the reference classifies each inside its
 * driver's recv(), pktio/loop.c:276-331, with no state shared between
 * packets but the rule tables and the counters), so a batch shards by
 * packet range: member i of a group of N device contexts classifies its
 * contiguous, tile-aligned range of the batch on its own device and stream.
 * The rule table is compiled once on the host (odpg_rules_compile) and the
 * image imported on every member (odpg_table_import), which the reference's
 * shared cos_t / pmr_t tables (odp_classification_datamodel.h:66-174) stand
 * for. The counters each member keeps (odpg.h "sharded counters") are summed
 * on the host when read, as odp_cls_cos_stats / odp_pktio_stats read the
 * reference's atomics at query time. There is no data-path exchange between
 * devices: verdict words of member i's range are written by member i.
 *
 * The torch.distributed path (one process per GPU, bench.py / odp_amd/shard.py)
 * is the same sharding across processes with RCCL for the image broadcast and
 * the counter all-reduce; this header is the in-process form a C integrator
 * or the ODP runtime (ODPG_DEVICES) uses.
 */
#ifndef ODPG_GROUP_H_
#define ODPG_GROUP_H_

#include <stdint.h>

#include "odpg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct odpg_group_s odpg_group_t;

/* Threads: odpg_group_load must not overlap a classify call on the same
 * group (it replaces the members' tables). Classify calls may come from
 * several threads; odpg_group_counters_fold may run beside them and then
 * sees the launches each member's stream had completed (as the reference's
 * counters read at query time). */

/* A group of n (1..64) device contexts, member i on devices[i] (a device may
 * repeat: its members then share the GPU, each with its own stream). */
int  odpg_group_create(const int *devices, uint32_t n, odpg_group_t **grp);
void odpg_group_destroy(odpg_group_t *grp);
uint32_t odpg_group_size(const odpg_group_t *grp);
/* member i's context (device buffers for odpg_group_classify are allocated
 * on it: odpg_dev_alloc) and, after odpg_group_load, its table */
odpg_ctx_t   *odpg_group_ctx(odpg_group_t *grp, uint32_t member);
odpg_table_t *odpg_group_table(odpg_group_t *grp, uint32_t member);

/* Compile `rules` once and import the image on every member, with a counters
 * object per member; a new generation replaces the previous one (its counts
 * are kept for odpg_group_counters_fold when the CoS count is unchanged). */
int  odpg_group_load(odpg_group_t *grp, const odpg_rules_t *rules);

/* Member i's packet range [lo, hi) of a num-packet batch over n members:
 * contiguous, starting on a 64-packet tile boundary, the last member taking
 * the remainder (empty ranges when num < 64 n). Pure host arithmetic. */
void odpg_group_range(uint32_t num, uint32_t n, uint32_t member, uint32_t *lo, uint32_t *hi);

/* A host batch (odpg_classify_host semantics: pointers in batch / res are
 * host pointers, desc offsets relative to batch->frames) split by packet
 * range, the members running concurrently; synchronous. res->stats and
 * res->counters must be NULL; counted != 0 adds the launch's counts to the
 * members' counters. */
int  odpg_group_classify_host(odpg_group_t *grp, const odpg_batch_t *batch,
			      const odpg_result_t *res, int counted, uint32_t chunk_pkts);

/* Device-resident shards: batches[i] / results[i] are in member i's HBM (one
 * per member; a member with num == 0 launches nothing). Asynchronous on each
 * member's stream; odpg_group_sync waits for all. */
int  odpg_group_classify(odpg_group_t *grp, const odpg_batch_t *batches,
			 const odpg_result_t *results, int counted);
int  odpg_group_sync(odpg_group_t *grp);

/* The members' counters summed (ODPG_COUNTER_WORDS(num_cos) words of the
 * loaded table, odpg.h layout), added to words, then cleared. */
int  odpg_group_counters_fold(odpg_group_t *grp, uint64_t *words);

#ifdef __cplusplus
}
#endif

#endif /* ODPG_GROUP_H_ */
