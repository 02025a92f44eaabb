/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odpg.h — C-ABI of the MI355X-native ODP receive-path classifier.
 *
 * One call classifies a whole batch of received frames on the GPU: the
 * L2/L3/L4 header parse, the RX IPv4/UDP/TCP/SCTP checksum verdict and the
 * Pattern-Matching-Rule (PMR) -> Class-of-Service (CoS) walk that ODP's
 * platform/linux-generic runs per packet inside a pktio driver's recv():
 *
 *   reference (per packet, host)                       replaced by
 *   ------------------------------------------------   ---------------------------
 *   packet_parse_reset()                                odpg_classify() (batch)
 *     platform/linux-generic/include/odp_packet_internal.h:433-444
 *   _odp_packet_parse_common()
 *     platform/linux-generic/include/odp_parse_internal.h:80-112
 *   _odp_packet_l4_chksum()
 *     platform/linux-generic/odp_packet.c:1906-1984
 *   _odp_cls_classify_packet()
 *     platform/linux-generic/odp_classification.c:1719-1749
 *     (prototype include/odp_classification_internal.h:238-239)
 *   the per-packet loop that calls them
 *     platform/linux-generic/pktio/loop.c:276-331
 *
 * Everything here is plain C: pointers, sizes and integers, no HIP or torch
 * types. Pointers documented as "device" must point to HBM of the context's
 * device (hipMalloc / odpg_dev_alloc). Functions return 0 on success or a
 * negative errno value.
 *
 * Per-packet verdict word (odpg_out_t, 4 bytes), written for every packet:
 *   bits  0..15  CoS index the packet was classified to (odp_packet_hdr_t.cos,
 *                odp_classification.c:1739), or
 *                ODPG_COS_NONE  (0xFFFF): no CoS, _odp_cls_classify_packet() == -1
 *                               (loop.c:317-318 counts it in in_discards)
 *                ODPG_COS_PDROP (0xFFFE): parser returned < 0, packet dropped
 *                               before classification (loop.c:304-310)
 *                ODPG_COS_LOOP  (0xFFFD): the CoS graph has a cycle that this
 *                               packet keeps matching; the reference loops
 *                               forever (match_pmr_cos, :1603-1631)
 *                ODPG_COS_NOCLS (0xFFFC): classification disabled
 *   bits 16..17  L3 checksum status  (odp_packet_l3_chksum_status(),
 *                include/odp/api/plat/packet_inlines.h:385-399)
 *   bits 18..19  L4 checksum status  (packet_inlines.h:401-417)
 *                0 = ODP_PACKET_CHKSUM_UNKNOWN, 1 = OK, 2 = BAD
 *   bit  20      packet has an error (any of the 7 parser error flags,
 *                packet_inline_types.h:150-164)
 *   bit  21      classified to a CoS with ODP_COS_ACTION_DROP (return 1)
 *   bit  22      cls mark valid (input_flags.cls_mark, odp_classification.c:1633-1639)
 *   bit  23      parser returned non-zero (counted in pktio in_errors, loop.c:304-305)
 *   bits 24..28  hash queue index within the CoS when its num_queue > 1
 *                (get_dest_queue(), odp_classification.c:372-382)
 *   bits 29..31  zero
 */
#ifndef ODPG_H_
#define ODPG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ODPG_ABI_VERSION 2

/* ---- limits ------------------------------------------------------------ */
/* Reference limits (odp_classification_datamodel.h:31-46) are enforced by the
 * odp_cls_* object model by default; the compiled device table itself accepts
 * up to these sizes (raised-limit configs, e.g. the 1024-PMR bench config). */
#define ODPG_MAX_COS           4096
#define ODPG_MAX_PMR           16384
#define ODPG_MAX_TERMS         8     /* CLS_PMRTERM_MAX */
#define ODPG_MAX_TERM_SIZE     16    /* MAX_PMR_TERM_SIZE */
#define ODPG_MAX_RULES_PER_COS 1024
#define ODPG_COS_QUEUE_MAX     32    /* CLS_COS_QUEUE_MAX */

/* ---- verdict word ------------------------------------------------------ */
typedef uint32_t odpg_out_t;

#define ODPG_COS_NONE   0xFFFFu
#define ODPG_COS_PDROP  0xFFFEu
#define ODPG_COS_LOOP   0xFFFDu
#define ODPG_COS_NOCLS  0xFFFCu

#define ODPG_OUT_COS(w)        ((uint32_t)(w) & 0xFFFFu)
#define ODPG_OUT_L3_STATUS(w)  (((uint32_t)(w) >> 16) & 3u)
#define ODPG_OUT_L4_STATUS(w)  (((uint32_t)(w) >> 18) & 3u)
#define ODPG_OUT_ERROR         (1u << 20)
#define ODPG_OUT_CLS_DROP      (1u << 21)
#define ODPG_OUT_MARK_VALID    (1u << 22)
#define ODPG_OUT_PARSE_ERR     (1u << 23)
#define ODPG_OUT_HASHQ(w)      (((uint32_t)(w) >> 24) & 31u)

#define ODPG_CHKSUM_UNKNOWN 0u
#define ODPG_CHKSUM_OK      1u
#define ODPG_CHKSUM_BAD     2u

/* ---- optional per-packet parser metadata (parity / debug) -------------- */
/* Bit-identical to packet_parser_t (odp_packet_internal.h:55-70):
 * input_flags uses the _odp_packet_input_flags_t layout and flags the
 * _odp_packet_flags_t layout (packet_inline_types.h:60-166). */
typedef struct odpg_meta_s {
	uint64_t input_flags;
	uint32_t flags;
	uint16_t l2_offset;
	uint16_t l3_offset;
	uint16_t l4_offset;
	uint16_t cls_mark;   /* odp_packet_hdr_t.cls_mark (valid if input_flags.cls_mark) */
	uint32_t reserved;
} odpg_meta_t;

/* ---- rule snapshot (input of the table compiler) ----------------------- */
/* One PMR term exactly as pmr_create_term() stores it
 * (odp_classification.c:645-738): value already AND-ed with mask, bytes in
 * the caller's order (network order except ODP_PMR_LEN, CPU endian). */
typedef struct odpg_term_s {
	uint32_t term;        /* odp_cls_pmr_term_t value */
	uint32_t val_sz;      /* 1..16 */
	uint32_t offset;      /* custom terms only */
	uint8_t  value[ODPG_MAX_TERM_SIZE];
	uint8_t  mask[ODPG_MAX_TERM_SIZE];
} odpg_term_t;

/* pmr_t (odp_classification_datamodel.h:149-157) */
typedef struct odpg_pmr_s {
	uint32_t    num_terms;
	uint32_t    mark;      /* 0..65535 */
	odpg_term_t terms[ODPG_MAX_TERMS];
} odpg_pmr_t;

/* cos_t (odp_classification_datamodel.h:124-146), the part the fast path reads */
typedef struct odpg_cos_s {
	uint32_t valid;
	uint32_t action;        /* 0 = ODP_COS_ACTION_ENQUEUE, 1 = ODP_COS_ACTION_DROP */
	uint32_t num_queue;     /* 1..32, > 1 enables hash queues */
	uint32_t hash_proto;    /* odp_cls_hash_proto_t: bit0 ipv4, bit1 ipv6, bit2 udp, bit3 tcp */
	uint32_t stats_enable;
	uint32_t num_rule;      /* rules attached, in cos->pmr[] order */
	uint32_t rule_start;    /* first slot in odpg_rules_t.rule_pmr / rule_dst */
} odpg_cos_t;

typedef struct odpg_rules_s {
	uint32_t          num_cos;
	const odpg_cos_t *cos;
	uint32_t          num_pmr;
	const odpg_pmr_t *pmr;
	uint32_t          num_slots;
	const uint32_t   *rule_pmr;   /* slot -> pmr index   (cos->pmr[i])        */
	const uint32_t   *rule_dst;   /* slot -> CoS index   (cos->linked_cos[i]) */
	int32_t           default_cos;/* classifier_t.default_cos, -1 = NULL     */
	int32_t           error_cos;  /* classifier_t.error_cos,   -1 = NULL     */
} odpg_rules_t;

/* ---- batch description ------------------------------------------------- */
/* Variable-length frames: frame i starts at frames + desc[i].offset and is
 * desc[i].len bytes long. offset must be a multiple of 16. */
typedef struct odpg_desc_s {
	uint32_t offset;
	uint32_t len;
} odpg_desc_t;

typedef struct odpg_batch_s {
	const uint8_t     *frames;    /* device */
	const odpg_desc_t *desc;      /* device, or NULL: fixed stride, len = stride */
	uint32_t           stride;    /* bytes between frames when desc == NULL (multiple of 16) */
	uint32_t           num;       /* number of frames */
	uint64_t           pktin_opt; /* odp_pktin_config_opt_t.all_bits (packet_io_types.h:390-434) */
	uint32_t           layer;     /* odp_proto_layer_t: 0 NONE, 1 L2, 2 L3, 3 L4, 4 ALL */
	uint32_t           classify;  /* non-zero: classifier enabled (pktio_cls_enabled) */
} odpg_batch_t;

/* pktin_opt bits (odp_pktin_config_opt_t) */
#define ODPG_PKTIN_TS_ALL        (1ull << 0)
#define ODPG_PKTIN_TS_PTP        (1ull << 1)
#define ODPG_PKTIN_IPV4_CHKSUM   (1ull << 2)
#define ODPG_PKTIN_UDP_CHKSUM    (1ull << 3)
#define ODPG_PKTIN_TCP_CHKSUM    (1ull << 4)
#define ODPG_PKTIN_SCTP_CHKSUM   (1ull << 5)
#define ODPG_PKTIN_DROP_IPV4_ERR (1ull << 6)
#define ODPG_PKTIN_DROP_IPV6_ERR (1ull << 7)
#define ODPG_PKTIN_DROP_UDP_ERR  (1ull << 8)
#define ODPG_PKTIN_DROP_TCP_ERR  (1ull << 9)
#define ODPG_PKTIN_DROP_SCTP_ERR (1ull << 10)

/* Batch counters, accumulated (added to) by odpg_classify when
 * odpg_result_t.stats != NULL. Layout (uint64_t words):
 *   [0] in_packets  [1] in_octets  [2] in_errors  [3] in_discards
 *       (pktio stats as loopback_recv() counts them, loop.c:304-374)
 *   [4 + c]  cos c stats.packets (odp_cls_cos_stats(), odp_classification.c:1621-1622,1697-1698)
 */
#define ODPG_STATS_WORDS(num_cos) (4u + (num_cos))

/* ---- opaque objects ---------------------------------------------------- */
typedef struct odpg_ctx_s      odpg_ctx_t;
typedef struct odpg_table_s    odpg_table_t;
typedef struct odpg_counters_s odpg_counters_t;

typedef struct odpg_result_s {
	odpg_out_t  *out;    /* device, num words (required)             */
	uint16_t    *mark;   /* device, num entries, or NULL             */
	odpg_meta_t *meta;   /* device, num entries, or NULL             */
	uint64_t    *stats;  /* device, ODPG_STATS_WORDS(num_cos), or NULL */
	odpg_counters_t *counters;  /* sharded counters (below), or NULL; not
				     * together with stats */
} odpg_result_t;

/* ---- sharded counters ----------------------------------------------------
 * The counts a launch makes (the pktio, CoS and per-queue counters the
 * reference keeps as atomics: loop.c:304-374, odp_classification.c:1621-1622,
 * 1697-1698, odp_classification_internal.h:64-78) accumulate in a device
 * block with one row per workgroup of the resident grid: each workgroup adds
 * its counts into its own row at its end (no atomics between workgroups, no
 * extra kernel per launch). odpg_counters_fold() sums the rows, adds the
 * totals to the caller's words and clears the rows, ordered on the context
 * stream after every launch enqueued before it; the reference reads its
 * counters the same way, at query time (odp_cls_cos_stats, odp_pktio_stats).
 * A counters object belongs to one table (its CoS and queue layout) and one
 * context. Folded layout (uint64_t words, added to):
 *   [0..3]                    in_packets, in_octets, in_errors, in_discards
 *   [4 + c]                   CoS c stats.packets (CoS with stats_enable)
 *   [4 + num_cos + 32 c + q]  packets delivered to queue q of CoS c (the
 *                             classifier returned 0: _odp_cls_enq input)  */
#define ODPG_COUNTER_WORDS(num_cos) (4u + (num_cos) + (num_cos) * ODPG_COS_QUEUE_MAX)

/* Library / device */
int         odpg_abi_version(void);
const char *odpg_build_info(void);
int         odpg_device_count(void);

/* Context: one per (device, stream). stream is a hipStream_t, or NULL to let
 * the context create its own non-blocking stream.
 *
 * Object lifetimes: tables, counters, forwarders (odpg_fwd.h) and fences
 * may be destroyed in any order relative to each other and to their
 * context. odpg_ctx_destroy() releases the caller's handle and the odp_cls
 * bindings made on the context; counters, forwarders and fences created on
 * it hold a reference, and the context's stream and device memory are freed
 * when the last of them is destroyed (the context handle itself may not be
 * used after odpg_ctx_destroy). A table refers to its device only. */
int  odpg_ctx_create(int device, void *stream, odpg_ctx_t **ctx);
void odpg_ctx_destroy(odpg_ctx_t *ctx);
void *odpg_ctx_stream(odpg_ctx_t *ctx);
/* Kernel strategy: 0 = auto (hash walk for tables of single-word compares
 * with at most 8 distinct (field, mask) groups; evaluate-all for other such
 * tables up to 1024 PMRs; the hybrid hash walk for tables where at most half
 * the PMRs need the generic compare; the wave-cooperative walk otherwise),
 * 1 = walk, 2 = evaluate-all, 3 = hash walk (single-word and hybrid tables;
 * walk otherwise). All strategies produce identical results; this only
 * selects the code path. */
int  odpg_ctx_set_kernel_mode(odpg_ctx_t *ctx, int mode);
/* Which kernel the last odpg_classify launch in this process used (a
 * diagnostic for tests and benches): 0 the general kernel, 1 the lean
 * 64-byte kernel that auto mode picks for fixed 64-byte strides, tables of
 * at most 64 single-word PMRs and verdict-only results. -1 before any. */
int  odpg_last_kernel(void);
int  odpg_ctx_sync(odpg_ctx_t *ctx);

/* Rule table: compiled, immutable snapshot of the CoS/PMR graph. The
 * reference reads rule tables unlocked ("in-flight packets during a PMR change
 * is indeterminate", odp_classification.c:1348-1349); here each snapshot is
 * immutable and rebuilt per generation. */
int  odpg_table_create(odpg_ctx_t *ctx, const odpg_rules_t *rules, odpg_table_t **tbl);
/* Compiled-table image, host only (no device): the bytes a multi-GPU job
 * compiles once and broadcasts; each rank imports them on its
 * own device. With blob NULL or *size too small: -ENOSPC and *size = the
 * bytes needed. */
int  odpg_rules_compile(const odpg_rules_t *rules, void *blob, size_t *size);
int  odpg_table_import(odpg_ctx_t *ctx, const void *blob, size_t size, odpg_table_t **tbl);
/* Recompile `tbl` in place from new rules (a new generation): the upload is
 * ordered on the context stream after the launches already enqueued with the
 * old contents, so it needs no wait and no reallocation unless the table
 * grew. Not concurrently with other threads' launches on the table. */
int  odpg_table_update(odpg_ctx_t *ctx, odpg_table_t *tbl, const odpg_rules_t *rules);
void odpg_table_destroy(odpg_table_t *tbl);
uint32_t odpg_table_num_cos(const odpg_table_t *tbl);
int  odpg_table_has_cycle(const odpg_table_t *tbl);

int  odpg_counters_create(odpg_ctx_t *ctx, const odpg_table_t *tbl, odpg_counters_t **cnt);
void odpg_counters_destroy(odpg_counters_t *cnt);
/* 1 if `cnt` can count launches on `tbl` (its layout: CoS count, queues and
 * stats flags), else 0 */
int  odpg_counters_match(const odpg_counters_t *cnt, const odpg_table_t *tbl);
/* Synchronous: words has ODPG_COUNTER_WORDS(odpg_table_num_cos(tbl)) entries. */
int  odpg_counters_fold(odpg_counters_t *cnt, uint64_t *words);

/* Device-resident batch: frames/desc/results all in HBM. Asynchronous on the
 * context stream. */
int odpg_classify(odpg_ctx_t *ctx, const odpg_table_t *tbl,
		  const odpg_batch_t *batch, const odpg_result_t *res);

/* Host batch (pinned or pageable host memory): chunked H2D copy, classify and
 * D2H of the verdict words with double buffering across two streams. The
 * pointers in batch/res are host pointers; desc offsets are relative to
 * batch->frames. Synchronous. */
int odpg_classify_host(odpg_ctx_t *ctx, const odpg_table_t *tbl,
		       const odpg_batch_t *batch, const odpg_result_t *res,
		       uint32_t chunk_pkts);

/* Thin memory helpers so hosts without a GPU framework can drive the ABI. */
int odpg_dev_alloc(odpg_ctx_t *ctx, size_t bytes, void **ptr);
int odpg_dev_free(odpg_ctx_t *ctx, void *ptr);
int odpg_host_alloc_pinned(size_t bytes, void **ptr);
int odpg_host_free_pinned(void *ptr);
/* The device address of pinned host memory (odpg_host_alloc_pinned): kernels
 * read and write it in place over PCIe (zero-copy; small batches) */
int odpg_host_device_ptr(void *host_ptr, void **dev_ptr);
int odpg_memcpy_h2d(odpg_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int odpg_memcpy_d2h(odpg_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int odpg_memset_dev(odpg_ctx_t *ctx, void *dst, int value, size_t bytes);

/* Timing on the context stream (HIP events), for benchmarks. */
int odpg_event_record(odpg_ctx_t *ctx, int slot);
int odpg_event_elapsed_ms(odpg_ctx_t *ctx, int slot_a, int slot_b, float *ms);

/* Completion fences on the context stream (a HIP event without timing):
 * record after an asynchronous launch, then poll (1 done, 0 pending, < 0
 * error) or wait. The runtime's receive path keeps several bursts in
 * flight with them (odp_rt.c "receive pipeline"). */
typedef struct odpg_fence_s odpg_fence_t;
int  odpg_fence_create(odpg_ctx_t *ctx, odpg_fence_t **fence);
int  odpg_fence_record(odpg_ctx_t *ctx, odpg_fence_t *fence);
int  odpg_fence_query(odpg_fence_t *fence);
int  odpg_fence_wait(odpg_fence_t *fence);
void odpg_fence_destroy(odpg_fence_t *fence);

/* Diagnostic streaming floor (not a classification entry point): read npkt
 * 64-byte frames at src, write one u32 per frame to out, with access pattern
 * 0 coalesced / 1 lane-per-frame / 2 coalesced-via-LDS (| 0x10 nontemporal),
 * over `grid` workgroups (0 = one per 256 frames). Used by tools/ and
 * DESIGN.md to state the achievable HBM floor of the launch shape. */
int odpg_diag_stream(odpg_ctx_t *ctx, const void *src, uint32_t npkt, uint32_t *out,
		     int pattern, uint32_t grid);

#ifdef __cplusplus
}
#endif

#endif /* ODPG_H_ */
