/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp_cls.h — ODP classification API (odp_cls_* / odp_cos_* / pktio
 * classifier setters) served by the MI355X classifier library.
 *
 * Names, argument meaning, handle encoding (index + 1, 0 = invalid) and
 * error behaviour follow the reference:
 *   API spec      include/odp/api/spec/classification.h:697-1073
 *   pktio setters include/odp/api/spec/packet_io.h:677-724
 *   semantics     platform/linux-generic/odp_classification.c:137-1877
 * The loop-pktio subset (open/config/start/recv) is the minimum needed to
 * drive the classifier the way pktio/loop.c does; it is not the full
 * odp_pktio API.
 *
 * Every struct the API passes has the reference's x86-64 layout (field
 * order, types, sizes), checked against the reference header text by
 * tests/test_abi_layout.py.
 */
#ifndef ODP_CLS_H_
#define ODP_CLS_H_

#include <stdbool.h>
#include <stdint.h>
#include <stddef.h>

#include "odpg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- base and handle types ----------------------------------------------
 * Layouts are those of the reference's x86-64 linux-generic ABI (a caller
 * compiled against the reference headers passes the same bytes):
 * odp_bool_t is C bool (abi-default/std_types.h), handles are pointers
 * (ODP_HANDLE_T, include-abi), scheduler ids are int (abi-default/
 * schedule_types.h). tests/test_abi_layout.py checks every struct below
 * field by field against a layout computed from the reference header text. */
typedef bool odp_bool_t;
typedef uint32_t odp_percent_t;

typedef struct _odp_cos_hdl    *odp_cos_t;
typedef struct _odp_pmr_hdl    *odp_pmr_t;
typedef struct _odp_queue_hdl  *odp_queue_t;
typedef struct _odp_pool_hdl   *odp_pool_t;
typedef struct _odp_pktio_hdl  *odp_pktio_t;
typedef struct _odp_packet_hdl *odp_packet_t;

#define ODP_COS_INVALID    ((odp_cos_t)0)
#define ODP_PMR_INVALID    ((odp_pmr_t)0)
#define ODP_QUEUE_INVALID  ((odp_queue_t)0)
#define ODP_POOL_INVALID   ((odp_pool_t)0)
#define ODP_PKTIO_INVALID  ((odp_pktio_t)0)
#define ODP_PACKET_INVALID ((odp_packet_t)0)

#define ODP_COS_NAME_LEN     32
#define ODP_PKTIN_MAX_QUEUES 64

typedef enum odp_support_t {
	ODP_SUPPORT_NO = 0,
	ODP_SUPPORT_YES,
	ODP_SUPPORT_PREFERRED
} odp_support_t;

/* ---- threshold.h ---------------------------------------------------------- */
typedef enum odp_threshold_type_t {
	ODP_THRESHOLD_PERCENT,
	ODP_THRESHOLD_PACKET,
	ODP_THRESHOLD_BYTE
} odp_threshold_type_t;

typedef union odp_threshold_types_t {
	struct {
		uint8_t percent : 1;
		uint8_t packet  : 1;
		uint8_t bytes   : 1;
	};
	uint8_t all_bits;
} odp_threshold_types_t;

typedef struct odp_threshold_t {
	odp_threshold_type_t type;
	union {
		struct {
			odp_percent_t max;
			odp_percent_t min;
		} percent;
		struct {
			uint64_t max;
			uint64_t min;
		} packet;
		struct {
			uint64_t max;
			uint64_t min;
		} byte;
	};
} odp_threshold_t;

/* ---- queue / schedule parameters (queue_types.h, schedule_types.h) -------- */
typedef int odp_schedule_prio_t;
typedef int odp_schedule_sync_t;
typedef int odp_schedule_group_t;

#define ODP_SCHED_SYNC_PARALLEL 0
#define ODP_SCHED_SYNC_ATOMIC   1
#define ODP_SCHED_SYNC_ORDERED  2
#define ODP_SCHED_GROUP_ALL     0
#define ODP_SCHED_GROUP_WORKER  1
#define ODP_SCHED_GROUP_CONTROL 2

typedef enum odp_queue_type_t {
	ODP_QUEUE_TYPE_PLAIN = 0,
	ODP_QUEUE_TYPE_SCHED
} odp_queue_type_t;

typedef enum odp_queue_op_mode_t {
	ODP_QUEUE_OP_MT = 0,
	ODP_QUEUE_OP_MT_UNSAFE,
	ODP_QUEUE_OP_DISABLED
} odp_queue_op_mode_t;

typedef enum odp_queue_order_t {
	ODP_QUEUE_ORDER_KEEP = 0,
	ODP_QUEUE_ORDER_IGNORE
} odp_queue_order_t;

typedef enum odp_nonblocking_t {
	ODP_BLOCKING = 0,
	ODP_NONBLOCKING_LF,
	ODP_NONBLOCKING_WF
} odp_nonblocking_t;

typedef struct odp_schedule_param_t {
	odp_schedule_prio_t  prio;
	odp_schedule_sync_t  sync;
	odp_schedule_group_t group;
	uint32_t lock_count;
} odp_schedule_param_t;

typedef struct odp_queue_param_t {
	odp_queue_type_t type;
	odp_queue_op_mode_t enq_mode;
	odp_queue_op_mode_t deq_mode;
	odp_schedule_param_t sched;
	odp_queue_order_t order;
	odp_nonblocking_t nonblocking;
	void *context;
	uint32_t context_len;
	uint32_t size;
} odp_queue_param_t;

/* ---- classification types (classification.h) ----------------------------- */
typedef enum {
	ODP_PMR_LEN = 0,
	ODP_PMR_ETHTYPE_0,
	ODP_PMR_ETHTYPE_X,
	ODP_PMR_VLAN_ID_0,
	ODP_PMR_VLAN_ID_X,
	ODP_PMR_VLAN_PCP_0,
	ODP_PMR_DMAC,
	ODP_PMR_IPPROTO,
	ODP_PMR_IP_DSCP,
	ODP_PMR_UDP_DPORT,
	ODP_PMR_TCP_DPORT,
	ODP_PMR_UDP_SPORT,
	ODP_PMR_TCP_SPORT,
	ODP_PMR_SIP_ADDR,
	ODP_PMR_DIP_ADDR,
	ODP_PMR_SIP6_ADDR,
	ODP_PMR_DIP6_ADDR,
	ODP_PMR_IPSEC_SPI,
	ODP_PMR_LD_VNI,
	ODP_PMR_CUSTOM_FRAME,
	ODP_PMR_CUSTOM_L3,
	ODP_PMR_IGMP_GRP_ADDR,
	ODP_PMR_ICMP_ID,
	ODP_PMR_ICMP_TYPE,
	ODP_PMR_ICMP_CODE,
	ODP_PMR_SCTP_SPORT,
	ODP_PMR_SCTP_DPORT,
	ODP_PMR_GTPV1_TEID,
	ODP_PMR_INNER_HDR_OFF = 32
} odp_cls_pmr_term_t;

typedef struct odp_pmr_param_t {
	odp_cls_pmr_term_t term;
	odp_bool_t range_term;
	union {
		struct {
			const void *value;
			const void *mask;
		} match;
		struct {
			const void *val_start;
			const void *val_end;
		} range;
	};
	uint32_t val_sz;
	uint32_t offset;
} odp_pmr_param_t;

typedef struct odp_pmr_create_opt_t {
	odp_pmr_param_t *terms;
	int num_terms;
	uint64_t mark;
} odp_pmr_create_opt_t;

typedef enum {
	ODP_COS_ACTION_ENQUEUE,
	ODP_COS_ACTION_DROP
} odp_cos_action_t;

typedef union odp_pktin_hash_proto_t {
	struct {
		uint32_t ipv4_udp : 1;
		uint32_t ipv4_tcp : 1;
		uint32_t ipv4     : 1;
		uint32_t ipv6_udp : 1;
		uint32_t ipv6_tcp : 1;
		uint32_t ipv6     : 1;
	} proto;
	uint32_t all_bits;
} odp_pktin_hash_proto_t;

typedef struct odp_red_param_t {
	odp_bool_t enable;
	odp_threshold_t threshold;
} odp_red_param_t;

typedef struct odp_bp_param_t {
	odp_bool_t enable;
	odp_threshold_t threshold;
	uint8_t pfc_level;
} odp_bp_param_t;

typedef struct odp_pktin_vector_config_t {
	odp_bool_t enable;
	odp_pool_t pool;
	uint64_t max_tmo_ns;
	uint32_t max_size;
} odp_pktin_vector_config_t;

typedef struct odp_cls_cos_param {
	odp_cos_action_t action;
	odp_bool_t stats_enable;
	uint32_t num_queue;
	union {
		odp_queue_t queue;
		struct {
			odp_queue_param_t queue_param;
			odp_pktin_hash_proto_t hash_proto;
		};
	};
	odp_pool_t pool;
	odp_red_param_t red;
	odp_bp_param_t bp;
	odp_pktin_vector_config_t vector;
} odp_cls_cos_param_t;

typedef union odp_cls_pmr_terms_t {
	struct {
		uint64_t len : 1;
		uint64_t ethtype_0 : 1;
		uint64_t ethtype_x : 1;
		uint64_t vlan_id_0 : 1;
		uint64_t vlan_id_x : 1;
		uint64_t vlan_pcp_0 : 1;
		uint64_t dmac : 1;
		uint64_t ip_proto : 1;
		uint64_t ip_dscp : 1;
		uint64_t udp_dport : 1;
		uint64_t tcp_dport : 1;
		uint64_t udp_sport : 1;
		uint64_t tcp_sport : 1;
		uint64_t sip_addr : 1;
		uint64_t dip_addr : 1;
		uint64_t sip6_addr : 1;
		uint64_t dip6_addr : 1;
		uint64_t ipsec_spi : 1;
		uint64_t ld_vni : 1;
		uint64_t custom_frame : 1;
		uint64_t custom_l3 : 1;
		uint64_t igmp_grp_addr : 1;
		uint64_t icmp_id : 1;
		uint64_t icmp_type : 1;
		uint64_t icmp_code : 1;
		uint64_t sctp_sport : 1;
		uint64_t sctp_dport : 1;
		uint64_t gtpv1_teid : 1;
	} bit;
	uint64_t all_bits;
} odp_cls_pmr_terms_t;

/* counters a CoS / a CoS queue supports (one layout for both) */
typedef struct odp_cls_stats_capability_t {
	struct {
		union {
			struct {
				uint64_t octets   : 1;
				uint64_t packets  : 1;
				uint64_t discards : 1;
				uint64_t errors   : 1;
			} counter;
			uint64_t all_counters;
		};
	} cos;
	struct {
		union {
			struct {
				uint64_t octets   : 1;
				uint64_t packets  : 1;
				uint64_t discards : 1;
				uint64_t errors   : 1;
			} counter;
			uint64_t all_counters;
		};
	} queue;
} odp_cls_stats_capability_t;

typedef struct odp_cls_capability_t {
	odp_cls_pmr_terms_t supported_terms;
	uint32_t max_pmr;
	uint32_t max_pmr_per_cos;
	uint32_t max_terms_per_pmr;
	uint32_t max_cos;
	uint32_t max_cos_stats;
	uint32_t max_hash_queues;
	odp_pktin_hash_proto_t hash_protocols;
	odp_bool_t pmr_range_supported;
	odp_support_t random_early_detection;
	odp_threshold_types_t threshold_red;
	odp_support_t back_pressure;
	odp_threshold_types_t threshold_bp;
	uint64_t max_mark;
	odp_cls_stats_capability_t stats;
} odp_cls_capability_t;

typedef struct odp_cls_cos_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_cls_cos_stats_t;

typedef struct odp_cls_queue_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_cls_queue_stats_t;

/* ---- classification API (classification.h:697-1073) -------------------- */
int  odp_cls_capability(odp_cls_capability_t *capability);
void odp_cls_cos_param_init(odp_cls_cos_param_t *param);
void odp_cls_pmr_param_init(odp_pmr_param_t *param);
void odp_cls_pmr_create_opt_init(odp_pmr_create_opt_t *opt);
odp_cos_t odp_cls_cos_create(const char *name, const odp_cls_cos_param_t *param);
int  odp_cls_cos_create_multi(const char *name[], const odp_cls_cos_param_t param[],
			      odp_cos_t cos[], int num);
int  odp_cos_destroy(odp_cos_t cos);
int  odp_cos_destroy_multi(odp_cos_t cos[], int num);
int  odp_cos_queue_set(odp_cos_t cos, odp_queue_t queue);
odp_queue_t odp_cos_queue(odp_cos_t cos);
uint32_t odp_cls_cos_num_queue(odp_cos_t cos);
uint32_t odp_cls_cos_queues(odp_cos_t cos, odp_queue_t queue[], uint32_t num);
odp_pmr_t odp_cls_pmr_create(const odp_pmr_param_t *terms, int num_terms,
			     odp_cos_t src_cos, odp_cos_t dst_cos);
odp_pmr_t odp_cls_pmr_create_opt(const odp_pmr_create_opt_t *opt,
				 odp_cos_t src_cos, odp_cos_t dst_cos);
int  odp_cls_pmr_create_multi(const odp_pmr_create_opt_t opt[], odp_cos_t src_cos[],
			      odp_cos_t dst_cos[], odp_pmr_t pmr[], int num);
int  odp_cls_pmr_destroy(odp_pmr_t pmr);
int  odp_cls_pmr_destroy_multi(odp_pmr_t pmr[], int num);
int  odp_cls_cos_pool_set(odp_cos_t cos, odp_pool_t pool);
odp_pool_t odp_cls_cos_pool(odp_cos_t cos);
int  odp_cls_cos_stats(odp_cos_t cos, odp_cls_cos_stats_t *stats);
int  odp_cls_queue_stats(odp_cos_t cos, odp_queue_t queue, odp_cls_queue_stats_t *stats);
void odp_cls_print_all(void);
/* The queue of `cos` a packet is enqueued to (classification.h:769;
 * odp_classification.c:384-414): the CoS queue, or for a hash-queue CoS the
 * queue get_dest_queue() picks from the packet's parse result.
 * odp_cls_hash_result() takes the runtime's packets (odp/rt.h: what
 * odp_schedule / odp_queue_deq / odp_pktin_recv hand out, or
 * odp_packet_alloc + odp_packet_parse). odpg_cls_hash_result() is the same
 * for a frame of a device batch described by an odpg_packet_t (frame bytes +
 * the odpg_meta_t a classify launch wrote for it). ODP_QUEUE_INVALID on a
 * bad CoS or packet. */
typedef struct odpg_packet_s {
	const uint8_t *data;
	uint32_t len;
	uint32_t reserved;
	odpg_meta_t meta;
} odpg_packet_t;
odp_queue_t odp_cls_hash_result(odp_cos_t cos, odp_packet_t packet);
odp_queue_t odpg_cls_hash_result(odp_cos_t cos, const odpg_packet_t *packet);
uint64_t odp_cos_to_u64(odp_cos_t hdl);
uint64_t odp_pmr_to_u64(odp_pmr_t hdl);

/* ---- loop pktio subset (packet_io.h, packet_io_types.h) ------------------ */
typedef union odp_pktin_config_opt_t {
	struct {
		uint64_t ts_all        : 1;
		uint64_t ts_ptp        : 1;
		uint64_t ipv4_chksum   : 1;
		uint64_t udp_chksum    : 1;
		uint64_t tcp_chksum    : 1;
		uint64_t sctp_chksum   : 1;
		uint64_t drop_ipv4_err : 1;
		uint64_t drop_ipv6_err : 1;
		uint64_t drop_udp_err  : 1;
		uint64_t drop_tcp_err  : 1;
		uint64_t drop_sctp_err : 1;
	} bit;
	uint64_t all_bits;
} odp_pktin_config_opt_t;

typedef union odp_pktout_config_opt_t {
	struct {
		uint64_t ts_ena          : 1;
		uint64_t ipv4_chksum_ena : 1;
		uint64_t udp_chksum_ena  : 1;
		uint64_t tcp_chksum_ena  : 1;
		uint64_t sctp_chksum_ena : 1;
		uint64_t ipv4_chksum     : 1;
		uint64_t udp_chksum      : 1;
		uint64_t tcp_chksum      : 1;
		uint64_t sctp_chksum     : 1;
		uint64_t no_packet_refs  : 1;
		uint64_t aging_ena       : 1;
		uint64_t deprecated_tx_compl_ena : 1;   /* ODP_DEPRECATE(tx_compl_ena) */
		uint64_t proto_stats_ena : 1;
	} bit;
	uint64_t all_bits;
} odp_pktout_config_opt_t;

typedef enum odp_proto_layer_t {
	ODP_PROTO_LAYER_NONE = 0,
	ODP_PROTO_LAYER_L2,
	ODP_PROTO_LAYER_L3,
	ODP_PROTO_LAYER_L4,
	ODP_PROTO_LAYER_ALL
} odp_proto_layer_t;

typedef struct odp_pktio_parser_config_t {
	odp_proto_layer_t layer;
} odp_pktio_parser_config_t;

typedef struct odp_reass_config_t {
	odp_bool_t en_ipv4;
	odp_bool_t en_ipv6;
	uint64_t max_wait_time;
	uint16_t max_num_frags;
} odp_reass_config_t;

typedef enum odp_pktio_link_pause_t {
	ODP_PKTIO_LINK_PAUSE_UNKNOWN = -1,
	ODP_PKTIO_LINK_PAUSE_OFF = 0,
	ODP_PKTIO_LINK_PAUSE_ON = 1,
	ODP_PKTIO_LINK_PFC_ON = 2
} odp_pktio_link_pause_t;

typedef struct odp_pktio_config_t {
	odp_pktin_config_opt_t pktin;
	odp_pktout_config_opt_t pktout;
	odp_pktio_parser_config_t parser;
	odp_bool_t enable_loop;
	odp_bool_t inbound_ipsec;
	odp_bool_t outbound_ipsec;
	odp_bool_t enable_lso;
	odp_reass_config_t reassembly;
	struct {
		odp_pktio_link_pause_t pause_rx;
		odp_pktio_link_pause_t pause_tx;
	} flow_control;
	struct {
		uint32_t mode_event : 1;
		uint32_t mode_poll  : 1;
		uint32_t max_compl_id;
	} tx_compl;
} odp_pktio_config_t;

typedef enum odp_pktin_mode_t {
	ODP_PKTIN_MODE_DIRECT = 0,
	ODP_PKTIN_MODE_SCHED,
	ODP_PKTIN_MODE_QUEUE,
	ODP_PKTIN_MODE_DISABLED
} odp_pktin_mode_t;

typedef enum odp_pktout_mode_t {
	ODP_PKTOUT_MODE_DIRECT = 0,
	ODP_PKTOUT_MODE_QUEUE,
	ODP_PKTOUT_MODE_TM,
	ODP_PKTOUT_MODE_DISABLED
} odp_pktout_mode_t;

typedef struct odp_pktio_param_t {
	odp_pktin_mode_t in_mode;
	odp_pktout_mode_t out_mode;
} odp_pktio_param_t;

typedef enum odp_pktio_op_mode_t {
	ODP_PKTIO_OP_MT = 0,
	ODP_PKTIO_OP_MT_UNSAFE
} odp_pktio_op_mode_t;

typedef struct odp_pktin_queue_param_ovr_t {
	odp_schedule_group_t group;
} odp_pktin_queue_param_ovr_t;

typedef struct odp_pktin_queue_param_t {
	odp_pktio_op_mode_t op_mode;
	odp_bool_t classifier_enable;
	odp_bool_t hash_enable;
	odp_pktin_hash_proto_t hash_proto;
	uint32_t num_queues;
	uint32_t queue_size[ODP_PKTIN_MAX_QUEUES];
	odp_queue_param_t queue_param;
	odp_pktin_queue_param_ovr_t *queue_param_ovr;
	odp_pktin_vector_config_t vector;
} odp_pktin_queue_param_t;

typedef struct odp_pktio_stats_t {
	uint64_t in_octets;
	uint64_t in_packets;
	uint64_t in_ucast_pkts;
	uint64_t in_mcast_pkts;
	uint64_t in_bcast_pkts;
	uint64_t in_discards;
	uint64_t in_errors;
	uint64_t out_octets;
	uint64_t out_packets;
	uint64_t out_ucast_pkts;
	uint64_t out_mcast_pkts;
	uint64_t out_bcast_pkts;
	uint64_t out_discards;
	uint64_t out_errors;
} odp_pktio_stats_t;

void odp_queue_param_init(odp_queue_param_t *param);
void odp_pktio_param_init(odp_pktio_param_t *param);
odp_pktio_t odp_pktio_open(const char *name, odp_pool_t pool, const odp_pktio_param_t *param);
int  odp_pktio_close(odp_pktio_t pktio);
void odp_pktio_config_init(odp_pktio_config_t *config);
int  odp_pktio_config(odp_pktio_t pktio, const odp_pktio_config_t *config);
void odp_pktin_queue_param_init(odp_pktin_queue_param_t *param);
int  odp_pktin_queue_config(odp_pktio_t pktio, const odp_pktin_queue_param_t *param);
int  odp_pktio_start(odp_pktio_t pktio);
int  odp_pktio_stop(odp_pktio_t pktio);
int  odp_pktio_stats(odp_pktio_t pktio, odp_pktio_stats_t *stats);
int  odp_pktio_stats_reset(odp_pktio_t pktio);
uint64_t odp_pktio_to_u64(odp_pktio_t pktio);

/* classifier setters (odp_classification.c:580-643) */
int odp_pktio_default_cos_set(odp_pktio_t pktio, odp_cos_t default_cos);
int odp_pktio_error_cos_set(odp_pktio_t pktio, odp_cos_t error_cos);
int odp_pktio_skip_set(odp_pktio_t pktio, uint32_t offset);
int odp_pktio_headroom_set(odp_pktio_t pktio, uint32_t headroom);

/* ---- MI355X extensions ------------------------------------------------- */
/* Raise the CoS / PMR table limits above the reference's
 * (odp_classification_datamodel.h:31-46). Only before the first create. */
int odpg_cls_set_limits(uint32_t max_cos, uint32_t max_pmr, uint32_t max_pmr_per_cos);
/* Reset the whole classifier state (all CoS, PMR, pktio). Test helper. */
void odpg_cls_reset(void);
/* Monotonic generation, bumped by every rule/pktio-classifier change. */
uint64_t odpg_cls_generation(void);

/* Snapshot the classifier view of a pktio into `rules`. The arrays stay valid
 * until the next snapshot call or reset. */
int odpg_pktio_rules(odp_pktio_t pktio, odpg_rules_t *rules);

/* The receive path of a started loop pktio (body of loopback_recv(),
 * pktio/loop.c:276-374) for a whole batch on the GPU: parse layer ALL when
 * the classifier is enabled (odp_packet_io.c:709-711), the pktio's pktin
 * checksum options, the current rule table (compiled and cached per
 * generation and context), then the pktio (in_*) and CoS / queue counters are
 * updated: the launch adds them into device-resident sharded counters
 * (odpg.h), folded when odp_pktio_stats / odp_cls_cos_stats /
 * odp_cls_queue_stats / odp_pktio_stats_reset read them.
 * device_ptrs != 0: frames/desc/out/mark are device pointers and the call is
 * asynchronous on the context stream like odpg_classify() (odpg_ctx_sync()
 * before reading out/mark); otherwise host pointers (pinned preferred)
 * streamed through odpg_classify_host(), synchronous. The classifier lock is
 * not held across the GPU work: receives on different contexts or threads run
 * concurrently. odp_pktio_close() fails while a receive is in flight. */
int odpg_pktio_recv_batch(odp_pktio_t pktio, odpg_ctx_t *ctx,
			  const uint8_t *frames, const odpg_desc_t *desc, uint32_t stride,
			  uint32_t num, int device_ptrs, odpg_out_t *out, uint16_t *mark);

#ifdef __cplusplus
}
#endif

#endif /* ODP_CLS_H_ */
