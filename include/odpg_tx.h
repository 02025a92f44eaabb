/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odpg_tx.h — the loop pktio transmit side on the GPU (SURVEY.md §8(f)
 * rank 3): per packet, loopback_send()'s checksum insertion and loop queue
 * pick (platform/linux-generic/pktio/loop.c:415-523), over a device-resident
 * batch, frames rewritten in place.
 *
 * Replaces, per packet of a loopback_send() burst (pktio/loop.c:525-575):
 *   loopback_fix_checksums(pkt, &config.pktout, &capa.config.pktout)
 *     (loop.c:415-466, check_proto loop.c:382-411)
 *     _odp_packet_ipv4_chksum_insert   odp_packet.c:1729-1787
 *     _odp_packet_tcp_chksum_insert    odp_packet.c:1789-1862, 1864-1872
 *     _odp_packet_udp_chksum_insert    odp_packet.c:1789-1862, 1874-1882
 *     _odp_packet_sctp_chksum_insert   odp_packet.c:1884-1898
 *   get_dest_queue(pkt_loop, pkt, index)          loop.c:468-523
 *     odp_hash_crc32c                  arch/default/odp_hash_crc32.c
 * The MTU check, queue enqueue and out_packets / out_octets counters stay on
 * the host (they need the whole burst / the queues).
 *
 * Reference behaviour reproduced bit for bit, including:
 *  - the TCP checksum is written at l4 + 6 (_ODP_UDP_CSUM_OFFSET, odp_packet.c
 *    :1838-1840), over the segment with those two bytes zeroed; the TCP
 *    header's checksum field (l4 + 16) is summed as it stands;
 *  - the UDP checksum sums the UDP length field a second time
 *    (odp_packet.c:1841-1846) and maps 0 to 0xffff;
 *  - ranges that run past frame_len contribute 0 (packet_sum_partial
 *    odp_packet.c:1669-1692) and writes past frame_len are skipped.
 */
#ifndef ODPG_TX_H_
#define ODPG_TX_H_

#include <stdint.h>

#include "odpg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* odp_pktout_config_opt_t bits (include/odp/api/spec/packet_io_types.h:
 * 480-545): the per-packet default insert bits loopback_fix_checksums reads
 * from the pktio config and from its capability */
#define ODPG_PKTOUT_IPV4_CHKSUM (1ull << 5)
#define ODPG_PKTOUT_UDP_CHKSUM  (1ull << 6)
#define ODPG_PKTOUT_TCP_CHKSUM  (1ull << 7)
#define ODPG_PKTOUT_SCTP_CHKSUM (1ull << 8)
/* the loop pktio capability (loop.c:671-674) */
#define ODPG_PKTOUT_LOOP_CAPA   (ODPG_PKTOUT_IPV4_CHKSUM | ODPG_PKTOUT_UDP_CHKSUM | \
				 ODPG_PKTOUT_TCP_CHKSUM | ODPG_PKTOUT_SCTP_CHKSUM)

/* odp_pktin_hash_proto_t bits (packet_io_types.h:125-147) */
#define ODPG_HASH_IPV4_UDP (1u << 0)
#define ODPG_HASH_IPV4_TCP (1u << 1)
#define ODPG_HASH_IPV4     (1u << 2)
#define ODPG_HASH_IPV6_UDP (1u << 3)
#define ODPG_HASH_IPV6_TCP (1u << 4)
#define ODPG_HASH_IPV6     (1u << 5)

/* per-packet TX metadata: the odp_packet_hdr_t fields the send path reads */
#define ODPG_TX_L3_CHKSUM_SET (1u << 0)   /* p.flags.l3_chksum_set (packet_inline_types.h:136) */
#define ODPG_TX_L3_CHKSUM     (1u << 1)   /* p.flags.l3_chksum override */
#define ODPG_TX_L4_CHKSUM_SET (1u << 2)   /* p.flags.l4_chksum_set */
#define ODPG_TX_L4_CHKSUM     (1u << 3)   /* p.flags.l4_chksum override */
#define ODPG_TX_HAS_IPV4      (1u << 8)   /* odp_packet_has_ipv4() etc. (input flags) */
#define ODPG_TX_HAS_IPV6      (1u << 9)
#define ODPG_TX_HAS_UDP       (1u << 10)
#define ODPG_TX_HAS_TCP       (1u << 11)
#define ODPG_OFFSET_INVALID   0xFFFFu     /* ODP_PACKET_OFFSET_INVALID */

typedef struct odpg_tx_meta_s {
	uint16_t l3_offset;
	uint16_t l4_offset;
	uint32_t flags;       /* ODPG_TX_* */
} odpg_tx_meta_t;         /* 8 bytes */

typedef struct odpg_tx_batch_s {
	uint8_t              *frames;  /* device; rewritten in place */
	const odpg_desc_t    *desc;    /* device, or NULL: fixed stride */
	uint32_t              stride;  /* bytes per frame when desc == NULL */
	uint32_t              num;
	const odpg_tx_meta_t *meta;    /* device, or NULL: each frame is parsed
					* (_odp_packet_parse_common, all layers,
					* no checksum checks) and has no overrides */
} odpg_tx_batch_t;

typedef struct odpg_tx_cfg_s {
	uint64_t pktout_cfg;   /* odp_pktout_config_opt_t.all_bits (pktio config) */
	uint64_t pktout_capa;  /* capability bits; ODPG_PKTOUT_LOOP_CAPA for loop */
	uint32_t hash_proto;   /* pkt_loop->hash: param->hash_enable ? hash_proto : 0 */
	uint32_t num_qs;       /* loop queues, >= 1 */
	uint32_t index;        /* pktout queue index (the queue when hash_proto == 0) */
	uint32_t reserved;
} odpg_tx_cfg_t;

/* out[i] (device, one word per packet):
 *   bits 0..15  destination loop queue index (get_dest_queue)
 *   bit  16     IPv4 header checksum inserted
 *   bit  17     UDP checksum inserted
 *   bit  18     TCP checksum inserted (at l4 + 6, see above)
 *   bit  19     SCTP CRC32c inserted
 * ("inserted": the insert function ran and returned 0.) */
#define ODPG_TX_OUT_QUEUE_MASK 0xFFFFu
#define ODPG_TX_OUT_IPV4       (1u << 16)
#define ODPG_TX_OUT_UDP        (1u << 17)
#define ODPG_TX_OUT_TCP        (1u << 18)
#define ODPG_TX_OUT_SCTP       (1u << 19)

/* Asynchronous on the context's stream. 0, or -EINVAL (bad arguments,
 * num_qs == 0) / -EIO. */
int odpg_tx_prepare(odpg_ctx_t *ctx, const odpg_tx_batch_t *batch, const odpg_tx_cfg_t *cfg,
		    uint32_t *out);

#ifdef __cplusplus
}
#endif

#endif /* ODPG_TX_H_ */
