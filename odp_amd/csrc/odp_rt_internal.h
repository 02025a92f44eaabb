/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Private seam between the classifier object model (odp_cls.c) and the ODP
 * runtime subset (odp_rt.c), both inside libodpg.so.
 *
 * Lock order: odp_rt.c's poll lock (held across a receive burst) may be
 * held while odp_cls.c's lock is taken, never the other way round; odp_cls.c
 * calls back into odp_rt.c only for queue creation / destruction (the
 * runtime's queue registry lock) and, with its lock released, to close a
 * pktio's receive state.
 */
#ifndef ODP_RT_INTERNAL_H_
#define ODP_RT_INTERNAL_H_

#include "../../include/odp_cls.h"

/* odp_rt.c: a pktio was opened / is closing (its receive state) */
int  odpg_rt_pktio_open(odp_pktio_t pktio, const char *name, odp_pool_t pool,
			const odp_pktio_param_t *param);
void odpg_rt_pktio_close(odp_pktio_t pktio);
/* odp_rt.c: odp_pktio_stop delivers the receive bursts still in flight */
void odpg_rt_pktio_drain(odp_pktio_t pktio);
/* odp_rt.c: odp_pktin_queue_config's input queues (the event queues of
 * SCHED / QUEUE mode) and their hash protocols (odp_pktin_hash_proto_t bits,
 * 0 without hash_enable); 0 or -1 (too many queues) */
int  odpg_rt_pktin_config(odp_pktio_t pktio, uint32_t num_queues, uint32_t hash_bits);

/* odp_cls.c: odpg_pktio_recv_batch's host path, also writing the parse
 * result of every packet (meta may be NULL) */
int odpg_cls_pktio_recv_meta(odp_pktio_t pktio, odpg_ctx_t *ctx, const uint8_t *frames,
			     const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
			     odpg_meta_t *meta);
/* the same on pinned host buffers read and written in place by the kernel
 * (zero-copy), complete on return */
int odpg_cls_pktio_recv_meta_zc(odp_pktio_t pktio, odpg_ctx_t *ctx, const uint8_t *frames,
			     const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
			     odpg_meta_t *meta);
/* its asynchronous form: launches, records `fence` behind the launch and
 * returns a token holding the pktio's binding; the results are valid once
 * the fence has completed, and odpg_cls_pktio_recv_end(token) then lets the
 * binding go (every started receive must be ended) */
int odpg_cls_pktio_recv_start_zc(odp_pktio_t pktio, odpg_ctx_t *ctx, const uint8_t *frames,
				 const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
				 odpg_meta_t *meta, odpg_fence_t *fence, void **token);
void odpg_cls_pktio_recv_end(void *token);
/* the pktio is started (with the classifier enabled) */
int odpg_cls_pktio_started(odp_pktio_t pktio);
int odpg_cls_pktio_classifies(odp_pktio_t pktio);
/* host-side counter changes the kernel does not see: a packet it counted
 * that the runtime then discarded (CoS pool copy failed, loop.c's
 * _odp_pktio_packet_to_pool branch), and transmits */
void odpg_cls_pktio_count(odp_pktio_t pktio, int64_t in_packets, int64_t in_octets,
			  uint64_t in_discards, uint64_t out_packets, uint64_t out_octets);
/* per-queue counters of a CoS the kernel cannot know: packets it counted as
 * delivered to `queue` that the runtime could not enqueue (_odp_cos_enq's
 * failed odp_queue_enq_multi -> _odp_cos_queue_stats_add(cos, dst, ret,
 * num - ret), odp_classification_internal.h:139-156) or did not hand to the
 * queue at all (pool copy failure) */
void odpg_cls_queue_count(odp_cos_t cos, odp_queue_t queue, int64_t packets,
			  uint64_t discards);

#endif
