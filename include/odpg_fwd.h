/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odpg_fwd.h — batch IPv4 forwarding decision of ODP's example/l3fwd on
 * MI355X (BASELINE config C5).
 *
 * Per packet the reference l3fwd worker (example/l3fwd/odp_l3fwd.c) does:
 *   drop_err_pkts()            odp_l3fwd.c:269-292   has_error (with -e) or !ipv4 -> drop
 *   l3fwd_pkt_hash()           odp_l3fwd.c:194-234   find_fwd_db_entry(): dst-IP key,
 *                                                     first match in the LIFO route list
 *                                                     (odp_l3fwd_db.c:474-508)
 *   l3fwd_pkt_lpm()            odp_l3fwd.c:236-256   fib_tbl_lookup() on the 16-4-4-4-4
 *                                                     trie (odp_l3fwd_lpm.c:210-230)
 *   ipv4_dec_ttl_csum_update() odp_l3fwd.c:183-192   TTL - 1, incremental checksum
 *   MAC rewrite + output port
 * on packets parsed by the pktio at layer L4 (ALL with -e), with no RX
 * checksum options (odp_l3fwd.c:132-135). odpg_l3fwd() does all of it for a
 * device-resident batch: one lane per packet, frames rewritten in place.
 *
 * Flow cache: the reference's hash mode keeps a flow cache
 * (odp_l3fwd_db.c:37-63 Jenkins hash, :178-335) in front of the route scan.
 * init_fwd_hash_cache() warms it deterministically: newest route first, the
 * addresses addr + i for i < 2^(32 - depth) (wrapping at 2^32), stopping at
 * the first address already cached or when the FWD_MAX_FLOW_COUNT (2^22)
 * flows are used up. A lookup then returns a warmed address's cached route,
 * else the first list match of the masked compare (as x86-64 computes it:
 * a /32 route's mask is 0, so it only matches as 0.0.0.0/32; a route with
 * host bits set never matches), which it caches without changing any later
 * answer. So the decision is a function of the destination alone:
 * odpg_fwd_create() folds the warmed ranges and the scan into one interval
 * table that the kernel searches. Every route set of 1..32 routes, depth
 * 1..32, is accepted in both modes.
 */
#ifndef ODPG_FWD_H_
#define ODPG_FWD_H_

#include <stdint.h>

#include "odpg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ODPG_FWD_MAX_ROUTES 32     /* MAX_DB (odp_l3fwd_db.h:18) */
#define ODPG_FWD_MAX_PORTS  32     /* MAX_NB_PKTIO */

/* fwd_db_entry_t (odp_l3fwd_db.h:63-70) after resolve_fwd_db() / setup_fwd_db() */
typedef struct odpg_route_s {
	uint32_t addr;       /* subnet.addr, host byte order */
	uint32_t depth;      /* subnet.depth, 1..32 */
	int32_t  oif_id;     /* output port */
	uint8_t  src_mac[6]; /* entry->src_mac (hash mode) */
	uint8_t  dst_mac[6]; /* entry->dst_mac (hash mode) */
} odpg_route_t;          /* 24 bytes */

#define ODPG_FWD_HASH 0      /* -h / default: find_fwd_db_entry() */
#define ODPG_FWD_LPM  1      /* fib_tbl_insert / fib_tbl_lookup */

typedef struct odpg_fwd_param_s {
	uint32_t mode;                       /* ODPG_FWD_HASH or ODPG_FWD_LPM */
	uint32_t num_ports;
	uint8_t  port_mac[ODPG_FWD_MAX_PORTS][6];  /* LPM: l3fwd_pktios[i].mac_addr */
	uint8_t  dest_mac[ODPG_FWD_MAX_PORTS][6];  /* LPM: eth_dest_mac[i]           */
} odpg_fwd_param_t;

typedef struct odpg_fwd_s odpg_fwd_t;

/* routes[] in the order the application added them (create_fwd_db_entry();
 * the reference prepends each, so lookups see the last one first). */
int  odpg_fwd_create(odpg_ctx_t *ctx, const odpg_route_t *routes, uint32_t num_routes,
		     const odpg_fwd_param_t *param, odpg_fwd_t **fwd);
void odpg_fwd_destroy(odpg_fwd_t *fwd);

typedef struct odpg_fwd_batch_s {
	uint8_t  *frames;       /* device; rewritten in place (MACs, TTL, IPv4 checksum) */
	uint32_t  stride;       /* bytes between frames, frame length = stride (multiple of 16) */
	uint32_t  num;
	int32_t   src_port;     /* sif: port the batch arrived on */
	uint32_t  error_check;  /* -e: drop packets with parse errors; parse layer ALL */
} odpg_fwd_batch_t;

/* out_port[i] (device) = output port, or -1 when the packet is dropped
 * (parse drop, error with error_check, not IPv4). Asynchronous on the
 * context stream. */
int odpg_l3fwd(odpg_ctx_t *ctx, const odpg_fwd_t *fwd, const odpg_fwd_batch_t *batch,
	       int32_t *out_port);

#ifdef __cplusplus
}
#endif

#endif /* ODPG_FWD_H_ */
