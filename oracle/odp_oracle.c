/* SPDX-License-Identifier: BSD-3-Clause
 *
 * ============================================================================
 *  TEST INFRASTRUCTURE ONLY — NOT PART OF THE PRODUCT.
 *  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 *  load this library, and only as the checker / the timed CPU baseline.
 * ============================================================================
 *
 * CPU restatement of ODP linux-generic's receive-path parse + RX checksum
 * verdict + PMR -> CoS classification, written from the reference's
 * behaviour (not copied). Every function names the reference lines it follows.
 *
 * Parity pinning: the reference cannot be compiled here without
 * configure-generated headers and a link shim (see DESIGN.md "Oracle"), so
 * this restatement is pinned against the reference's own fixtures and
 * known-answer tests (tests/golden/, tests/test_oracle_*.py).
 *
 * Documented deviation (reference behaviour undefined): bytes the reference
 * would read past the end of a frame (only for malformed/truncated frames)
 * read as zero here and on the GPU.
 */
#include <sched.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>
#include <time.h>

#include "../include/odpg.h"

/* ---- _odp_packet_input_flags_t bit positions (packet_inline_types.h:60-113) */
enum {
	IF_DST_QUEUE = 0, IF_CLS_MARK, IF_FLOW_HASH, IF_TIMESTAMP,
	IF_L2, IF_L3, IF_L4,
	IF_ETH, IF_ETH_BCAST, IF_ETH_MCAST, IF_JUMBO, IF_VLAN, IF_VLAN_QINQ,
	IF_SNAP, IF_ARP,
	IF_IPV4, IF_IPV6, IF_IP_BCAST, IF_IP_MCAST, IF_IPFRAG, IF_IPOPT,
	IF_IPSEC, IF_IPSEC_AH, IF_IPSEC_ESP,
	IF_UDP, IF_TCP, IF_SCTP, IF_ICMP, IF_NO_NEXT_HDR,
	IF_COLOR0, IF_COLOR1, IF_NODROP,
	IF_L3_CHKSUM_DONE, IF_L4_CHKSUM_DONE, IF_IPSEC_UDP, IF_UDP_CHKSUM_ZERO
};
#define IFB(x) (1ull << (x))

/* ---- _odp_packet_flags_t error bits (packet_inline_types.h:150-164) */
enum {
	F_SNAP_LEN_ERR = 25, F_IP_ERR, F_L3_CHKSUM_ERR, F_TCP_ERR, F_UDP_ERR,
	F_SCTP_ERR, F_L4_CHKSUM_ERR
};
#define FB(x) (1u << (x))
#define F_ERROR_MASK 0xFE000000u   /* flags.all.error: bits 25..31 */

/* ---- odp_cls_pmr_term_t (include/odp/api/spec/classification.h:68-195) */
enum {
	T_LEN = 0, T_ETHTYPE_0, T_ETHTYPE_X, T_VLAN_ID_0, T_VLAN_ID_X,
	T_VLAN_PCP_0, T_DMAC, T_IPPROTO, T_IP_DSCP, T_UDP_DPORT, T_TCP_DPORT,
	T_UDP_SPORT, T_TCP_SPORT, T_SIP_ADDR, T_DIP_ADDR, T_SIP6_ADDR,
	T_DIP6_ADDR, T_IPSEC_SPI, T_LD_VNI, T_CUSTOM_FRAME, T_CUSTOM_L3,
	T_INNER_HDR_OFF = 32
};

/* protocol constants (protocols/eth.h:95-100, ip.h:159-174, udp.h:41) */
#define ETH_LEN_MAX        1514
#define ETHTYPE_IPV4       0x0800
#define ETHTYPE_ARP        0x0806
#define ETHTYPE_VLAN       0x8100
#define ETHTYPE_VLAN_OUTER 0x88A8
#define ETHTYPE_IPV6       0x86dd
#define PROTO_HOPOPTS 0x00
#define PROTO_ICMPV4  0x01
#define PROTO_IPIP    0x04
#define PROTO_TCP     0x06
#define PROTO_UDP     0x11
#define PROTO_ROUTE   0x2B
#define PROTO_FRAG    0x2C
#define PROTO_ESP     0x32
#define PROTO_AH      0x33
#define PROTO_ICMPV6  0x3A
#define PROTO_NO_NEXT 0x3B
#define PROTO_SCTP    0x84
#define UDP_IPSEC_PORT 4500

/* odp_proto_layer_t */
enum { LAYER_NONE = 0, LAYER_L2, LAYER_L3, LAYER_L4, LAYER_ALL };

#define OFFSET_INVALID 0xFFFF  /* ODP_PACKET_OFFSET_INVALID */

typedef struct {
	uint64_t input_flags;
	uint32_t flags;
	uint16_t l2_offset, l3_offset, l4_offset;
	uint16_t cls_mark;
	uint16_t cos;
	uint8_t  hashq;
} hdr_t;

/* packet view: reads past frame_len return 0 (documented deviation) */
typedef struct {
	const uint8_t *d;
	uint32_t len;
} pv_t;

static inline uint8_t B(const pv_t *v, uint32_t off)
{
	return off < v->len ? v->d[off] : 0;
}

static inline uint16_t be16(const pv_t *v, uint32_t off)
{
	return (uint16_t)((B(v, off) << 8) | B(v, off + 1));
}

/* raw little-endian load of n bytes, what the x86 reference gets from a
 * plain `*(uintNN_t *)ptr` of network-order bytes */
static inline uint64_t raw(const pv_t *v, uint32_t off, int n)
{
	uint64_t x = 0;

	if (off + (uint32_t)n <= v->len) {
		memcpy(&x, v->d + off, (size_t)n);
		return x;
	}
	for (int i = 0; i < n; i++)
		x |= (uint64_t)B(v, off + i) << (8 * i);
	return x;
}

/* ---- chksum_finalize / chksum_partial (odp_chksum_internal.h:22-196) --- */
static inline uint16_t chksum_finalize(uint64_t sum)
{
	sum = (sum >> 32) + (sum & 0xffffffff);
	sum = (sum >> 16) + (sum & 0xffff);
	return (uint16_t)((sum >> 16) + sum);
}

/* x86 path (_ODP_UNALIGNED): 32-bit LE words from addr, tail word, tail
 * byte, odd-offset byte swap. */
static uint64_t chksum_partial_mem(const uint8_t *b, uint32_t len, uint32_t offset)
{
	uint64_t sum = 0;
	uint32_t w32;
	uint16_t w16;

	offset &= 1;
	while (len >= 4) {
		memcpy(&w32, b, 4);
		sum += w32;
		b += 4;
		len -= 4;
	}
	if (len > 1) {
		memcpy(&w16, b, 2);
		sum += w16;
		b += 2;
		len -= 2;
	}
	if (len) {
		/* odp_cpu_to_be_16((uint16_t)*b << 8) on LE == *b */
		sum += *b;
	}
	if (offset)
		sum = ((sum & 0xff00ff00ff00ffull) << 8) |
		      ((sum & 0xff00ff00ff00ff00ull) >> 8);
	return sum;
}

static uint64_t chksum_partial(const pv_t *v, uint32_t off, uint32_t len, uint32_t offset)
{
	if (off + len <= v->len)
		return chksum_partial_mem(v->d + off, len, offset);

	/* range runs past the frame: zero-extended copy */
	uint8_t tmp[4096 + 64];
	uint8_t *buf = len <= sizeof(tmp) ? tmp : malloc(len);
	uint64_t s;

	for (uint32_t i = 0; i < len; i++)
		buf[i] = B(v, off + i);
	s = chksum_partial_mem(buf, len, offset);
	if (buf != tmp)
		free(buf);
	return s;
}

/* ---- CRC32C, reflected Castagnoli, no final xor
 * (arch/default/odp_hash_crc32.c:437-463 semantics) */
static uint32_t crc32c_tbl[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;

static void crc_init(void)
{
	for (uint32_t i = 0; i < 256; i++) {
		uint32_t c = i;

		for (int k = 0; k < 8; k++)
			c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
		crc32c_tbl[i] = c;
	}
}

static uint32_t crc32c(const pv_t *v, uint32_t off, uint32_t len, uint32_t crc)
{
	for (uint32_t i = 0; i < len; i++)
		crc = crc32c_tbl[(crc ^ B(v, off + i)) & 0xff] ^ (crc >> 8);
	return crc;
}

/* ---- _odp_parse_eth (odp_parse.c:23-106) ------------------------------- */
static uint16_t parse_eth(hdr_t *prs, const pv_t *v, uint32_t *offset, uint32_t frame_len)
{
	uint64_t inf = IFB(IF_L2) | IFB(IF_ETH);
	uint16_t ethtype;
	const uint32_t s = *offset;        /* 0 on receive; odp_packet_parse's offset */
	uint16_t mac0 = be16(v, s);

	if (frame_len - *offset > ETH_LEN_MAX)
		inf |= IFB(IF_JUMBO);
	if ((mac0 & 0x0100) == 0x0100)
		inf |= IFB(IF_ETH_MCAST);
	if (mac0 == 0xffff && be16(v, s + 2) == 0xffff && be16(v, s + 4) == 0xffff)
		inf |= IFB(IF_ETH_BCAST);

	ethtype = be16(v, s + 12);
	*offset += 14;

	if (ethtype < ETH_LEN_MAX) {                       /* SNAP, :61-71 */
		inf |= IFB(IF_SNAP);
		if (ethtype > frame_len - *offset) {
			prs->flags |= FB(F_SNAP_LEN_ERR);
			ethtype = 0;
			goto error;
		}
		ethtype = be16(v, *offset + 6);
		*offset += 8;
	}
	if (ethtype == ETHTYPE_VLAN_OUTER) {               /* :74-82 */
		inf |= IFB(IF_VLAN_QINQ) | IFB(IF_VLAN);
		ethtype = be16(v, *offset + 2);
		*offset += 4;
	}
	if (ethtype == ETHTYPE_VLAN) {                     /* :84-90 */
		inf |= IFB(IF_VLAN);
		ethtype = be16(v, *offset + 2);
		*offset += 4;
	}
	if (*offset > frame_len) {                         /* :96-100 */
		inf = IFB(IF_L2);
		ethtype = 0;
	}
error:
	prs->input_flags |= inf;
	return ethtype;
}

/* ---- parse_ipv4 (odp_parse.c:113-169) ---------------------------------- */
static uint8_t parse_ipv4(hdr_t *prs, const pv_t *v, uint32_t *offset, uint32_t frame_len,
			  uint64_t opt, uint64_t *l4_part_sum)
{
	uint32_t o = *offset;
	uint8_t ver_ihl = B(v, o);
	uint32_t dstaddr = ((uint32_t)be16(v, o + 16) << 16) | be16(v, o + 18);
	uint32_t l3_len = be16(v, o + 2);
	uint16_t frag_offset = be16(v, o + 6);
	uint8_t ver = (ver_ihl & 0xf0) >> 4;
	uint8_t ihl = ver_ihl & 0x0f;

	if ((prs->flags & FB(F_L3_CHKSUM_ERR)) || ihl < 5 || ver != 4 ||
	    20 > frame_len - o || l3_len > frame_len - o) {
		prs->flags |= FB(F_IP_ERR);
		return 0;
	}
	if (opt & ODPG_PKTIN_IPV4_CHKSUM) {
		prs->input_flags |= IFB(IF_L3_CHKSUM_DONE);
		if (chksum_finalize(chksum_partial(v, o, ihl * 4u, 0)) != 0xffff) {
			prs->flags |= FB(F_IP_ERR) | FB(F_L3_CHKSUM_ERR);
			return 0;
		}
	}
	*offset += ihl * 4u;
	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM))
		*l4_part_sum = chksum_partial(v, o + 12, 8, 0);
	if (ihl > 5)
		prs->input_flags |= IFB(IF_IPOPT);
	if (frag_offset & 0x3fff)
		prs->input_flags |= IFB(IF_IPFRAG);
	if (dstaddr == 0xffffffff)
		prs->input_flags |= IFB(IF_IP_BCAST);
	if ((dstaddr >> 28) == 0xe)
		prs->input_flags |= IFB(IF_IP_MCAST);
	return B(v, o + 9);
}

/* ---- parse_ipv6 (odp_parse.c:179-245) ---------------------------------- */
static uint8_t parse_ipv6(hdr_t *prs, const pv_t *v, uint32_t *offset, uint32_t frame_len,
			  uint32_t seg_end, uint64_t opt, uint64_t *l4_part_sum)
{
	uint32_t o = *offset;
	uint32_t ver_tc_flow = ((uint32_t)be16(v, o) << 16) | be16(v, o + 2);
	uint32_t payload_len = be16(v, o + 4);
	uint32_t l3_len = payload_len + 40;
	uint8_t next_hdr = B(v, o + 6);
	uint8_t dst0 = B(v, o + 24);

	if ((prs->flags & FB(F_L3_CHKSUM_ERR)) || (ver_tc_flow >> 28) != 6 ||
	    40 > frame_len - o || l3_len > frame_len - o) {
		prs->flags |= FB(F_IP_ERR);
		return 0;
	}
	if (dst0 == 0xff)
		prs->input_flags |= IFB(IF_IP_MCAST);
	else
		prs->input_flags &= ~IFB(IF_IP_MCAST);
	prs->input_flags &= ~IFB(IF_IP_BCAST);

	*offset += 40;
	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM))
		*l4_part_sum = chksum_partial(v, o + 8, 32, 0);

	if (next_hdr == PROTO_HOPOPTS || next_hdr == PROTO_ROUTE) {
		uint32_t ext;
		uint8_t ext_next;

		prs->input_flags |= IFB(IF_IPOPT);
		do {
			ext = *offset;
			ext_next = B(v, ext);
			*offset += 8u + B(v, ext + 1) * 8u;
		} while ((ext_next == PROTO_HOPOPTS || ext_next == PROTO_ROUTE) &&
			 *offset < seg_end);

		if (*offset >= (uint32_t)prs->l3_offset + payload_len) {
			prs->flags |= FB(F_IP_ERR);
			return 0;
		}
		if (ext_next == PROTO_FRAG)
			prs->input_flags |= IFB(IF_IPFRAG);
		return ext_next;
	}
	if (next_hdr == PROTO_FRAG)
		prs->input_flags |= IFB(IF_IPOPT) | IFB(IF_IPFRAG);
	return next_hdr;
}

/* ---- parse_tcp / parse_udp / parse_sctp (odp_parse.c:252-352) ---------- */
static void parse_tcp(hdr_t *prs, const pv_t *v, uint32_t o, uint16_t tcp_len,
		      uint64_t opt, uint64_t *l4_part_sum)
{
	uint8_t hl = B(v, o + 12) >> 4;

	if (hl < 5)
		prs->flags |= FB(F_TCP_ERR);
	if ((opt & ODPG_PKTIN_TCP_CHKSUM) && !(prs->input_flags & IFB(IF_IPFRAG))) {
		*l4_part_sum += (uint16_t)((tcp_len >> 8) | (tcp_len << 8)); /* cpu_to_be_16 */
		*l4_part_sum += PROTO_TCP << 8;
	}
}

static void parse_udp(hdr_t *prs, const pv_t *v, uint32_t o, uint64_t opt,
		      uint64_t *l4_part_sum)
{
	uint32_t udplen = be16(v, o + 4);
	uint16_t chksum_raw = (uint16_t)raw(v, o + 6, 2);

	if (udplen < 8) {
		prs->flags |= FB(F_UDP_ERR);
		return;
	}
	if ((opt & ODPG_PKTIN_UDP_CHKSUM) && !(prs->input_flags & IFB(IF_IPFRAG))) {
		if (chksum_raw == 0) {
			prs->input_flags |= IFB(IF_L4_CHKSUM_DONE);
			if (!(prs->input_flags & IFB(IF_IPV4)))
				prs->flags |= FB(F_L4_CHKSUM_ERR);
			else
				prs->flags &= ~FB(F_L4_CHKSUM_ERR);
		} else {
			*l4_part_sum += (uint16_t)raw(v, o + 4, 2);
			*l4_part_sum += PROTO_UDP << 8;
		}
		if (chksum_raw == 0)
			prs->input_flags |= IFB(IF_UDP_CHKSUM_ZERO);
		else
			prs->input_flags &= ~IFB(IF_UDP_CHKSUM_ZERO);
	}
	if (be16(v, o + 2) == UDP_IPSEC_PORT && udplen > 4) {
		if (raw(v, o + 8, 4) != 0)
			prs->input_flags |= IFB(IF_IPSEC) | IFB(IF_IPSEC_UDP);
	}
}

static void parse_sctp(hdr_t *prs, const pv_t *v, uint32_t o, uint16_t sctp_len,
		       uint64_t opt, uint64_t *l4_part_sum)
{
	if (sctp_len < 12) {
		prs->flags |= FB(F_SCTP_ERR);
		return;
	}
	if ((opt & ODPG_PKTIN_SCTP_CHKSUM) && !(prs->input_flags & IFB(IF_IPFRAG))) {
		uint32_t crc = ~0u;

		crc = crc32c(v, o, 8, crc);
		crc = crc32c_tbl[crc & 0xff] ^ (crc >> 8);   /* 4 zero bytes */
		crc = crc32c_tbl[crc & 0xff] ^ (crc >> 8);
		crc = crc32c_tbl[crc & 0xff] ^ (crc >> 8);
		crc = crc32c_tbl[crc & 0xff] ^ (crc >> 8);
		*l4_part_sum = crc;
	}
}

/* ---- _odp_packet_parse_common_l3_l4 (odp_parse.c:360-475) -------------- */
static int parse_l3_l4(hdr_t *prs, const pv_t *v, uint32_t offset, uint32_t frame_len,
		       uint32_t seg_end, int layer, uint16_t ethtype,
		       uint64_t *l4_part_sum, uint64_t opt)
{
	uint8_t ip_proto;

	prs->l3_offset = (uint16_t)offset;
	if (layer <= LAYER_L2)
		return (prs->flags & F_ERROR_MASK) != 0;

	prs->input_flags |= IFB(IF_L3);
	switch (ethtype) {
	case ETHTYPE_IPV4:
		prs->input_flags |= IFB(IF_IPV4);
		ip_proto = parse_ipv4(prs, v, &offset, frame_len, opt, l4_part_sum);
		if (!(prs->flags & FB(F_IP_ERR)))
			prs->l4_offset = (uint16_t)offset;
		else if (opt & ODPG_PKTIN_DROP_IPV4_ERR)
			return -1;
		break;
	case ETHTYPE_IPV6:
		prs->input_flags |= IFB(IF_IPV6);
		ip_proto = parse_ipv6(prs, v, &offset, frame_len, seg_end, opt, l4_part_sum);
		if (!(prs->flags & FB(F_IP_ERR)))
			prs->l4_offset = (uint16_t)offset;
		else if (opt & ODPG_PKTIN_DROP_IPV6_ERR)
			return -1;
		break;
	case ETHTYPE_ARP:
		prs->input_flags |= IFB(IF_ARP);
		ip_proto = 255;
		break;
	default:
		prs->input_flags &= ~IFB(IF_L3);
		ip_proto = 255;
	}

	if (layer == LAYER_L3)
		return (prs->flags & F_ERROR_MASK) != 0;

	prs->input_flags |= IFB(IF_L4);
	switch (ip_proto) {
	case PROTO_ICMPV4:
	case PROTO_ICMPV6:
		prs->input_flags |= IFB(IF_ICMP);
		break;
	case PROTO_IPIP:
		break;
	case PROTO_TCP:
		if (offset + 20 > seg_end)
			return -1;
		prs->input_flags |= IFB(IF_TCP);
		parse_tcp(prs, v, offset, (uint16_t)(frame_len - prs->l4_offset), opt, l4_part_sum);
		if ((prs->flags & FB(F_TCP_ERR)) && (opt & ODPG_PKTIN_DROP_TCP_ERR))
			return -1;
		break;
	case PROTO_UDP:
		if (offset + 8 > seg_end)
			return -1;
		prs->input_flags |= IFB(IF_UDP);
		parse_udp(prs, v, offset, opt, l4_part_sum);
		if ((prs->flags & FB(F_UDP_ERR)) && (opt & ODPG_PKTIN_DROP_UDP_ERR))
			return -1;
		break;
	case PROTO_AH:
		prs->input_flags |= IFB(IF_IPSEC) | IFB(IF_IPSEC_AH);
		break;
	case PROTO_ESP:
		prs->input_flags |= IFB(IF_IPSEC) | IFB(IF_IPSEC_ESP);
		break;
	case PROTO_SCTP:
		prs->input_flags |= IFB(IF_SCTP);
		parse_sctp(prs, v, offset, (uint16_t)(frame_len - prs->l4_offset), opt, l4_part_sum);
		if ((prs->flags & FB(F_SCTP_ERR)) && (opt & ODPG_PKTIN_DROP_SCTP_ERR))
			return -1;
		break;
	case PROTO_NO_NEXT:
		prs->input_flags |= IFB(IF_NO_NEXT_HDR);
		break;
	default:
		prs->input_flags &= ~IFB(IF_L4);
		break;
	}
	return (prs->flags & F_ERROR_MASK) != 0;
}

/* ---- _odp_packet_l4_chksum (odp_packet.c:1906-1984) -------------------- */
static uint16_t packet_sum(const pv_t *v, uint32_t l3, uint32_t off, uint32_t len, uint64_t sum)
{
	/* packet_sum_partial (odp_packet.c:1669-1692): 0 if out of frame */
	if (off + len <= v->len)
		sum += chksum_partial(v, off, len, off - l3);
	return chksum_finalize(sum);
}

static int l4_chksum(hdr_t *h, const pv_t *v, uint64_t opt, uint64_t l4_part_sum)
{
	uint64_t inf = h->input_flags;
	uint32_t frame_len = v->len;

	if ((opt & ODPG_PKTIN_UDP_CHKSUM) && (inf & IFB(IF_UDP)) &&
	    !(inf & IFB(IF_IPFRAG)) && !(inf & IFB(IF_UDP_CHKSUM_ZERO))) {
		uint16_t sum = (uint16_t)~packet_sum(v, h->l3_offset, h->l4_offset,
						     frame_len - h->l4_offset, l4_part_sum);

		h->input_flags |= IFB(IF_L4_CHKSUM_DONE);
		if (sum != 0) {
			h->flags |= FB(F_L4_CHKSUM_ERR) | FB(F_UDP_ERR);
			if (opt & ODPG_PKTIN_DROP_UDP_ERR)
				return -1;
		}
	}
	if ((opt & ODPG_PKTIN_TCP_CHKSUM) && (inf & IFB(IF_TCP)) && !(inf & IFB(IF_IPFRAG))) {
		uint16_t sum = (uint16_t)~packet_sum(v, h->l3_offset, h->l4_offset,
						     frame_len - h->l4_offset, l4_part_sum);

		h->input_flags |= IFB(IF_L4_CHKSUM_DONE);
		if (sum != 0) {
			h->flags |= FB(F_L4_CHKSUM_ERR) | FB(F_TCP_ERR);
			if (opt & ODPG_PKTIN_DROP_TCP_ERR)
				return -1;
		}
	}
	if ((opt & ODPG_PKTIN_SCTP_CHKSUM) && (inf & IFB(IF_SCTP)) && !(inf & IFB(IF_IPFRAG))) {
		uint32_t l4 = h->l4_offset;
		uint32_t len = frame_len - l4 - 12;
		uint32_t sum = (uint32_t)l4_part_sum;

		/* packet_sum_crc32c (odp_packet.c:1704-1727): init returned if out of frame */
		if (l4 + 12 + len <= frame_len)
			sum = crc32c(v, l4 + 12, len, sum);
		sum = ~sum;
		h->input_flags |= IFB(IF_L4_CHKSUM_DONE);
		if (sum != (uint32_t)raw(v, l4 + 8, 4)) {
			h->flags |= FB(F_L4_CHKSUM_ERR) | FB(F_SCTP_ERR);
			if (opt & ODPG_PKTIN_DROP_SCTP_ERR)
				return -1;
		}
	}
	return (h->flags & F_ERROR_MASK) != 0;
}

/* ---- _odp_packet_parse_common (odp_parse_internal.h:80-112) ------------ */
static int parse_common(hdr_t *h, const pv_t *v, uint32_t seg_len, int layer, uint64_t opt)
{
	uint32_t offset = 0;
	uint64_t l4_part_sum = 0;
	uint16_t ethtype;
	int r;

	if (layer == LAYER_NONE)
		return 0;
	h->l2_offset = 0;
	ethtype = parse_eth(h, v, &offset, v->len);
	r = parse_l3_l4(h, v, offset, v->len, seg_len, layer, ethtype, &l4_part_sum, opt);
	if (!r && layer >= LAYER_L4)
		r = l4_chksum(h, v, opt, l4_part_sum);
	return r;
}

/* ---- odp_packet_parse (odp_packet.c:1986-2052) -------------------------
 * One single-segment packet parsed from `offset`, starting with protocol
 * `proto` (odp_proto_t: 1 ETH, 2 IPV4, 3 IPV6, else none known) up to
 * `layer`, with the odp_proto_chksums_t bits `chksums` (ipv4, udp, tcp,
 * sctp) as the checksum options. *meta is updated in place as the packet
 * header is: packet_parse_reset(pkt_hdr, 0) keeps the non-error flags.
 * Returns 0, or -1 as odp_packet_parse does. */
static int packet_parse(const pv_t *v, uint32_t offset, int proto, int layer, uint32_t chksums,
			odpg_meta_t *meta)
{
	hdr_t h;
	uint64_t opt = 0, l4_part_sum = 0;
	uint16_t ethtype;
	int ret;

	if (proto == 0 || layer == LAYER_NONE)
		return -1;
	if (offset >= v->len)                      /* packet_map: no data there */
		return -1;
	memset(&h, 0, sizeof(h));
	h.l2_offset = h.l3_offset = h.l4_offset = OFFSET_INVALID;
	h.flags = meta->flags & ~F_ERROR_MASK;
	if (chksums & 1u)
		opt |= ODPG_PKTIN_IPV4_CHKSUM;
	if (chksums & 2u)
		opt |= ODPG_PKTIN_UDP_CHKSUM;
	if (chksums & 4u)
		opt |= ODPG_PKTIN_TCP_CHKSUM;
	if (chksums & 8u)
		opt |= ODPG_PKTIN_SCTP_CHKSUM;
	if (proto == 1) {
		h.l2_offset = (uint16_t)offset;
		ethtype = parse_eth(&h, v, &offset, v->len);
	} else if (proto == 2) {
		ethtype = ETHTYPE_IPV4;
	} else if (proto == 3) {
		ethtype = ETHTYPE_IPV6;
	} else {
		ethtype = 0;
	}
	ret = parse_l3_l4(&h, v, offset, v->len, v->len, layer, ethtype, &l4_part_sum, opt);
	if (!ret && layer >= LAYER_L4)
		ret = l4_chksum(&h, v, opt, l4_part_sum);
	meta->input_flags = h.input_flags;
	meta->flags = h.flags;
	meta->l2_offset = h.l2_offset;
	meta->l3_offset = h.l3_offset;
	meta->l4_offset = h.l4_offset;
	meta->cls_mark = 0;
	meta->reserved = 0;
	return ret ? -1 : 0;
}

/* ---- verify_pmr and the per-term matchers (odp_classification.c:906-1490) */
static inline uint64_t tval(const odpg_term_t *t, int word)
{
	uint64_t x;

	memcpy(&x, t->value + 8 * word, 8);
	return x;
}

static inline uint64_t tmask(const odpg_term_t *t, int word)
{
	uint64_t x;

	memcpy(&x, t->mask + 8 * word, 8);
	return x;
}

static int verify_term(const odpg_term_t *t, const pv_t *v, const hdr_t *h)
{
	uint64_t inf = h->input_flags;
	uint64_t value = tval(t, 0), mask = tmask(t, 0);
	uint32_t l2 = h->l2_offset, l3 = h->l3_offset, l4 = h->l4_offset;
	int ipv4 = !!(inf & IFB(IF_IPV4)), ipv6 = !!(inf & IFB(IF_IPV6));

	switch (t->term) {
	case T_LEN:                                          /* :906-914 */
		return value == ((uint64_t)v->len & mask);
	case T_ETHTYPE_0:                                    /* :1290-1307 */
		if (!(inf & IFB(IF_ETH)))
			return 0;
		return value == (raw(v, l2 + 12, 2) & mask);
	case T_ETHTYPE_X: {                                  /* :1309-1332 */
		uint32_t vo = l2 + 14;

		if (!(inf & IFB(IF_VLAN)) && !(inf & IFB(IF_VLAN_QINQ)))
			return 0;
		if (inf & IFB(IF_VLAN_QINQ))
			vo += 4;
		return value == (raw(v, vo + 2, 2) & mask);
	}
	case T_VLAN_ID_0:                                    /* :1132-1153 */
		if (!(inf & IFB(IF_ETH)) || !(inf & IFB(IF_VLAN)))
			return 0;
		return value == ((raw(v, l2 + 14, 2) & 0xff0f) & mask);
	case T_VLAN_ID_X: {                                  /* :1155-1180 */
		uint32_t vo = l2 + 14;

		if (!(inf & IFB(IF_VLAN)) && !(inf & IFB(IF_VLAN_QINQ)))
			return 0;
		if (inf & IFB(IF_VLAN_QINQ))
			vo += 4;
		return value == ((raw(v, vo, 2) & 0xff0f) & mask);
	}
	case T_VLAN_PCP_0: {                                 /* :1182-1202 */
		uint8_t pcp;

		if (!(inf & IFB(IF_ETH)) || !(inf & IFB(IF_VLAN)))
			return 0;
		pcp = (uint8_t)(be16(v, l2 + 14) >> 13);
		return value == (pcp & mask);
	}
	case T_DMAC: {                                       /* :1062-1084 */
		uint64_t d;

		if (!(inf & IFB(IF_ETH)))
			return 0;
		d = raw(v, l2, 6);
		return (d & mask & 0xffffffffffffull) == (value & 0xffffffffffffull);
	}
	case T_IPPROTO:                                      /* :1397-1407 */
		if (ipv4)
			return value == (B(v, l3 + 9) & mask);
		if (ipv6)
			return value == (B(v, l3 + 6) & mask);
		return 0;
	case T_IP_DSCP:                                      /* :1408-1418 */
		if (ipv4)
			return value == ((uint8_t)((B(v, l3 + 1) & 0xfc) >> 2) & mask);
		if (ipv6) {
			uint32_t vtf = ((uint32_t)be16(v, l3) << 16) | be16(v, l3 + 2);

			return value == ((uint8_t)(((vtf & 0x0fc00000) >> 22) & 0xff) & mask);
		}
		return 0;
	case T_UDP_DPORT:                                    /* :1028-1043 */
		if (!(inf & IFB(IF_UDP)))
			return 0;
		return value == (raw(v, l4 + 2, 2) & mask);
	case T_TCP_DPORT:                                    /* :1011-1026 */
		if (!(inf & IFB(IF_TCP)))
			return 0;
		return value == (raw(v, l4 + 2, 2) & mask);
	case T_UDP_SPORT:                                    /* :1045-1060 */
		if (!(inf & IFB(IF_UDP)))
			return 0;
		return value == (raw(v, l4, 2) & mask);
	case T_TCP_SPORT:                                    /* :994-1009 */
		if (!(inf & IFB(IF_TCP)))
			return 0;
		return value == (raw(v, l4, 2) & mask);
	case T_SIP_ADDR:                                     /* :960-975 */
		if (!ipv4)
			return 0;
		return value == (raw(v, l3 + 12, 4) & mask);
	case T_DIP_ADDR:                                     /* :977-992 */
		if (!ipv4)
			return 0;
		return value == (raw(v, l3 + 16, 4) & mask);
	case T_SIP6_ADDR:                                    /* :1086-1107 */
	case T_DIP6_ADDR: {                                  /* :1109-1130 */
		uint32_t a = l3 + (t->term == T_SIP6_ADDR ? 8 : 24);

		if (!ipv6)
			return 0;
		return (raw(v, a, 8) & tmask(t, 0)) == tval(t, 0) &&
		       (raw(v, a + 8, 8) & tmask(t, 1)) == tval(t, 1);
	}
	case T_IPSEC_SPI: {                                  /* :1204-1223 */
		uint64_t spi;

		if (inf & IFB(IF_IPSEC_AH))
			spi = raw(v, l4 + 4, 4);
		else if (inf & IFB(IF_IPSEC_ESP))
			spi = raw(v, l4, 4);
		else
			return 0;
		return value == (spi & mask);
	}
	case T_LD_VNI:                                       /* :1225-1231 */
		return 0;
	case T_CUSTOM_FRAME: {                               /* :1233-1257 */
		uint32_t off = t->offset;

		if (v->len <= off + t->val_sz)
			return 0;
		for (uint32_t i = 0; i < t->val_sz; i++)
			if ((B(v, off + i) & t->mask[i]) != t->value[i])
				return 0;
		return 1;
	}
	case T_CUSTOM_L3: {                                  /* :1259-1288 */
		uint32_t off = l3 + t->offset;

		if (!(inf & IFB(IF_L2)) || l3 == OFFSET_INVALID)
			return 0;
		if (v->len <= off + t->val_sz)
			return 0;
		for (uint32_t i = 0; i < t->val_sz; i++)
			if ((B(v, off + i) & t->mask[i]) != t->value[i])
				return 0;
		return 1;
	}
	case T_INNER_HDR_OFF:
		return 1;
	default:
		return 0;
	}
}

static int verify_pmr(const odpg_pmr_t *pmr, const pv_t *v, const hdr_t *h)
{
	for (uint32_t i = 0; i < pmr->num_terms; i++)
		if (!verify_term(&pmr->terms[i], v, h))
			return 0;
	return 1;
}

/* ---- thash_softrss / packet_rss_hash (protocols/thash.h:81-99,
 *      odp_classification.c:1751-1817) */
static const uint8_t default_rss[40] = {
	0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2,
	0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0,
	0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4,
	0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30, 0xf2, 0x0c,
	0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa,
};

static uint32_t key_be(int j)
{
	return ((uint32_t)default_rss[4 * j] << 24) | ((uint32_t)default_rss[4 * j + 1] << 16) |
	       ((uint32_t)default_rss[4 * j + 2] << 8) | default_rss[4 * j + 3];
}

static uint32_t thash_softrss(const uint32_t *tuple, uint32_t len)
{
	uint32_t ret = 0;

	for (uint32_t j = 0; j < len; j++)
		for (uint32_t i = 0; i < 32; i++)
			if (tuple[j] & (1u << (31 - i)))
				ret ^= (key_be(j) << i) |
				       (uint32_t)((uint64_t)key_be(j + 1) >> (32 - i));
	return ret;
}

static uint32_t packet_rss_hash(const hdr_t *h, const pv_t *v, uint32_t hp)
{
	/* tuple zero-initialised: the reference leaves unused words
	 * uninitialised (documented deviation for odd hash_proto mixes) */
	uint32_t tuple[11] = {0};
	uint32_t len = 0;
	uint64_t inf = h->input_flags;
	int hipv4 = hp & 1, hipv6 = hp & 2, hudp = hp & 4, htcp = hp & 8;

	if (inf & IFB(IF_IPV4)) {
		if (hipv4) {
			tuple[0] = (uint32_t)raw(v, h->l3_offset + 12, 4);
			tuple[1] = (uint32_t)raw(v, h->l3_offset + 16, 4);
			len += 2;
		}
		if ((inf & IFB(IF_TCP)) && htcp) {
			tuple[2] = (uint32_t)raw(v, h->l4_offset, 4);
			len += 1;
		} else if ((inf & IFB(IF_UDP)) && hudp) {
			tuple[2] = (uint32_t)raw(v, h->l4_offset, 4);
			len += 1;
		}
	} else if (inf & IFB(IF_IPV6)) {
		if (hipv6) {
			for (int i = 0; i < 4; i++) {
				tuple[i] = ((uint32_t)be16(v, h->l3_offset + 8 + 4 * i) << 16) |
					   be16(v, h->l3_offset + 10 + 4 * i);
				tuple[4 + i] = ((uint32_t)be16(v, h->l3_offset + 24 + 4 * i) << 16) |
					       be16(v, h->l3_offset + 26 + 4 * i);
			}
			len += 8;
		}
		if ((inf & IFB(IF_TCP)) && htcp) {
			tuple[8] = (uint32_t)raw(v, h->l4_offset, 4);
			len += 1;
		} else if ((inf & IFB(IF_UDP)) && hudp) {
			tuple[8] = (uint32_t)raw(v, h->l4_offset, 4);
			len += 1;
		}
	}
	return len ? thash_softrss(tuple, len) : 0;
}

/* ---- match_pmr_cos / cls_select_cos / _odp_cls_classify_packet
 *      (odp_classification.c:1599-1642, :1669-1701, :1719-1749) ---------- */
typedef struct {
	const odpg_rules_t *r;
	uint64_t *cos_pkts;   /* per-CoS stats.packets */
} cls_t;

#define COS_LOOP (-2)

static int match_pmr_cos(const cls_t *c, int cos, const pv_t *v, hdr_t *h)
{
	const odpg_rules_t *r = c->r;
	const odpg_pmr_t *pmr_match = NULL;
	uint32_t steps = 0;

	while (1) {
		const odpg_cos_t *ce = &r->cos[cos];
		uint32_t i, num_rule = ce->num_rule;

		for (i = 0; i < num_rule; i++) {
			uint32_t slot = ce->rule_start + i;
			const odpg_pmr_t *pmr = &r->pmr[r->rule_pmr[slot]];
			int linked = (int)r->rule_dst[slot];

			if (!r->cos[linked].valid)
				continue;
			if (verify_pmr(pmr, v, h)) {
				pmr_match = pmr;
				cos = linked;
				if (r->cos[cos].stats_enable && c->cos_pkts)
					c->cos_pkts[cos]++;
				break;
			}
		}
		if (i == num_rule)
			break;
		/* the reference never terminates on a matching cycle */
		if (++steps >= r->num_cos)
			return COS_LOOP;
	}
	if (pmr_match) {
		h->input_flags &= ~IFB(IF_CLS_MARK);
		if (pmr_match->mark) {
			h->input_flags |= IFB(IF_CLS_MARK);
			h->cls_mark = (uint16_t)pmr_match->mark;
		}
	}
	return cos;
}

static int cls_select_cos(const cls_t *c, const pv_t *v, hdr_t *h)
{
	const odpg_rules_t *r = c->r;
	int def = r->default_cos;
	int cos;

	if (h->flags & F_ERROR_MASK) {
		cos = r->error_cos;
		goto done;
	}
	if (def >= 0 && r->cos[def].valid) {
		cos = match_pmr_cos(c, def, v, h);
		if (cos == COS_LOOP)
			return COS_LOOP;
		if (cos >= 0 && cos != def)
			return cos;
	}
	cos = def;
done:
	if (cos >= 0 && r->cos[cos].stats_enable && c->cos_pkts)
		c->cos_pkts[cos]++;
	return cos;
}

/* returns -1 (no CoS), 1 (drop action), 0 ok; -2 cycle */
static int classify_packet(const cls_t *c, const pv_t *v, hdr_t *h)
{
	const odpg_rules_t *r = c->r;
	int cos = cls_select_cos(c, v, h);

	if (cos == COS_LOOP) {
		h->cos = ODPG_COS_LOOP;
		return -2;
	}
	if (cos < 0) {
		h->cos = ODPG_COS_NONE;
		return -1;
	}
	h->cos = (uint16_t)cos;
	if (r->cos[cos].action == 1)   /* ODP_COS_ACTION_DROP */
		return 1;
	h->input_flags |= IFB(IF_DST_QUEUE);
	if (r->cos[cos].num_queue > 1) {
		uint32_t hash = packet_rss_hash(h, v, r->cos[cos].hash_proto);

		h->hashq = (uint8_t)((hash & 31) % r->cos[cos].num_queue);
	}
	return 0;
}

/* ---- the loopback_recv() per-packet body (pktio/loop.c:276-348) -------- */
typedef struct {
	const uint8_t *frames;
	const odpg_desc_t *desc;
	uint32_t stride;
	uint64_t opt;
	int layer;
	int classify;
} batch_t;

static void process_one(const batch_t *b, const cls_t *c, uint32_t i,
			odpg_out_t *out, uint16_t *mark, odpg_meta_t *meta, uint64_t *pk)
{
	pv_t v;
	hdr_t h;
	int ret, cret = 0;
	uint32_t w;

	if (b->desc) {
		v.d = b->frames + b->desc[i].offset;
		v.len = b->desc[i].len;
	} else {
		v.d = b->frames + (size_t)i * b->stride;
		v.len = b->stride;
	}
	/* packet_parse_reset(hdr, 1) (odp_packet_internal.h:433-444) */
	memset(&h, 0, sizeof(h));
	h.l2_offset = h.l3_offset = h.l4_offset = OFFSET_INVALID;

	ret = 0;
	if (b->layer) {
		ret = parse_common(&h, &v, v.len, b->layer, b->opt);
		if (ret)
			pk[2]++;                       /* in_errors */
	}
	w = 0;
	if (ret < 0) {
		w = ODPG_COS_PDROP;
	} else if (b->layer && b->classify) {
		cret = classify_packet(c, &v, &h);
		if (cret == -1 || cret == -2)
			pk[3]++;                       /* in_discards */
		w = h.cos;
		if (cret == 1)
			w |= ODPG_OUT_CLS_DROP;
		if (cret == 0)
			w |= (uint32_t)h.hashq << 24;
	} else {
		w = ODPG_COS_NOCLS;
	}
	if (ret >= 0 && cret == 0 && !(h.flags & F_ERROR_MASK)) {
		pk[0]++;                               /* in_packets */
		pk[1] += v.len;                        /* in_octets  */
	}
	if (h.input_flags & IFB(IF_L3_CHKSUM_DONE))
		w |= (h.flags & FB(F_L3_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 16;
	if (h.input_flags & IFB(IF_L4_CHKSUM_DONE))
		w |= (h.flags & FB(F_L4_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 18;
	if (h.flags & F_ERROR_MASK)
		w |= ODPG_OUT_ERROR;
	if (h.input_flags & IFB(IF_CLS_MARK))
		w |= ODPG_OUT_MARK_VALID;
	if (ret)
		w |= ODPG_OUT_PARSE_ERR;
	out[i] = w;
	if (mark)
		mark[i] = (h.input_flags & IFB(IF_CLS_MARK)) ? h.cls_mark : 0;
	if (meta) {
		meta[i].input_flags = h.input_flags;
		meta[i].flags = h.flags;
		meta[i].l2_offset = h.l2_offset;
		meta[i].l3_offset = h.l3_offset;
		meta[i].l4_offset = h.l4_offset;
		meta[i].cls_mark = (h.input_flags & IFB(IF_CLS_MARK)) ? h.cls_mark : 0;
		meta[i].reserved = 0;
	}
}

/* ---- exported entry points -------------------------------------------- */
/* Single-threaded batch. stats (optional) has ODPG_STATS_WORDS(num_cos)
 * words and is added to. Returns 0. */
int oracle_classify(const odpg_rules_t *rules, const uint8_t *frames,
		    const odpg_desc_t *desc, uint32_t stride, uint32_t num,
		    uint64_t opt, int layer, int classify,
		    odpg_out_t *out, uint16_t *mark, odpg_meta_t *meta, uint64_t *stats)
{
	batch_t b = { frames, desc, stride, opt, layer, classify };
	cls_t c = { rules, stats ? stats + 4 : NULL };
	uint64_t pk[4] = {0, 0, 0, 0};

	pthread_once(&crc_once, crc_init);
	for (uint32_t i = 0; i < num; i++)
		process_one(&b, &c, i, out, mark, meta, pk);
	if (stats)
		for (int k = 0; k < 4; k++)
			stats[k] += pk[k];
	return 0;
}

/* one cache line (or more) per thread: the workers share no written line */
typedef struct {
	const odpg_rules_t *rules;
	batch_t b;
	uint32_t lo, hi;
	uint32_t reps;
	odpg_out_t *out;
	uint64_t pk[4];
	int cpu;             /* pin to this CPU, or -1 */
} __attribute__((aligned(128))) mt_arg_t;

static void *mt_worker(void *p)
{
	mt_arg_t *a = p;
	cls_t c = { a->rules, NULL };
	/* the pktio counters in the thread's own registers / stack, added to
	 * the shared block once at the end (loopback_recv likewise adds its
	 * burst's packet and octet counts once per burst, loop.c:370-371) */
	uint64_t pk[4] = {0, 0, 0, 0};

	if (a->cpu >= 0) {
		cpu_set_t set;

		CPU_ZERO(&set);
		CPU_SET(a->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}

	for (uint32_t r = 0; r < a->reps; r++)
		for (uint32_t i = a->lo; i < a->hi; i++)
			process_one(&a->b, &c, i, a->out, NULL, NULL, pk);
	memcpy(a->pk, pk, sizeof(pk));
	return NULL;
}

/* Multi-threaded batch for the CPU baseline: contiguous slices per thread,
 * `reps` passes over the batch, per-CoS stats not collected; thread t is
 * pinned to cpus[t] when cpus is given. Returns the number of threads used. */
int oracle_classify_mt(const odpg_rules_t *rules, const uint8_t *frames,
		       const odpg_desc_t *desc, uint32_t stride, uint32_t num,
		       uint64_t opt, int layer, int classify, odpg_out_t *out,
		       int nthreads, uint32_t reps, const int *cpus)
{
	pthread_t th[256];
	static mt_arg_t args[256];   /* 32 KiB: off the caller's stack */

	pthread_once(&crc_once, crc_init);
	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	for (int t = 0; t < nthreads; t++) {
		args[t].rules = rules;
		args[t].b = (batch_t){ frames, desc, stride, opt, layer, classify };
		args[t].lo = (uint32_t)((uint64_t)num * t / nthreads);
		args[t].hi = (uint32_t)((uint64_t)num * (t + 1) / nthreads);
		args[t].reps = reps;
		args[t].out = out;
		memset(args[t].pk, 0, sizeof(args[t].pk));
		args[t].cpu = cpus ? cpus[t] : -1;
		pthread_create(&th[t], NULL, mt_worker, &args[t]);
	}
	for (int t = 0; t < nthreads; t++)
		pthread_join(th[t], NULL);
	return nthreads;
}

/* Exposed for the checksum known-answer tests (test/validation/api/chksum):
 * odp_chksum_ones_comp16() == chksum_finalize(chksum_partial(p, len, 0))
 * (odp_chksum.c:11). */
/* odp_packet_parse_multi (odp_packet.c:2064-2075) over a batch: returns
 * the index of the first packet that fails (num if none); packets after it
 * are not touched. ret[i] gets each parsed packet's return value. */
int oracle_packet_parse_multi(const uint8_t *frames, const odpg_desc_t *desc, uint32_t num,
			      const uint32_t *offset, int proto, int layer, uint32_t chksums,
			      odpg_meta_t *meta, int32_t *ret)
{
	pthread_once(&crc_once, crc_init);
	for (uint32_t i = 0; i < num; i++) {
		pv_t v = { frames + desc[i].offset, desc[i].len };

		ret[i] = packet_parse(&v, offset[i], proto, layer, chksums, &meta[i]);
		if (ret[i])
			return (int)i;
	}
	return (int)num;
}

uint16_t oracle_chksum_ones_comp16(const uint8_t *p, uint32_t len)
{
	return chksum_finalize(chksum_partial_mem(p, len, 0));
}

uint32_t oracle_crc32c(const uint8_t *p, uint32_t len, uint32_t init)
{
	pv_t v = { p, len };

	pthread_once(&crc_once, crc_init);
	return crc32c(&v, 0, len, init);
}

uint32_t oracle_thash(const uint32_t *tuple, uint32_t len)
{
	return thash_softrss(tuple, len);
}

/* ---- odph_udp_tcp_chksum() (helper/chksum.c:265-353) over one contiguous
 * frame: the application-side checksum of the helper library, which BASELINE
 * config C3 is also checked against. It differs from the platform verify
 * (_odp_packet_l4_chksum, odp_packet.c:1906-1984) in its length: UDP sums
 * udp.length bytes (:127-130), TCP sums l3_len - (l4 - l3) from the IP
 * header (:232), where the platform sums frame_len - l4_offset.
 * op: 0 GENERATE (writes the field), 1 VERIFY, 2 RETURN (as odph_chksum_op_t).
 * Returns <0 error (length leaves the frame, not UDP/TCP), 0 ok / generated,
 * 1 VERIFY of a UDP packet with checksum field 0, 2 VERIFY mismatch. */
static uint32_t helper_seg_sum(const uint8_t *p, uint32_t len)
{
	/* data_seg_sum (:32-90) for a single, last segment: host-order (LE)
	 * 16-bit words, a trailing odd byte as the low byte of a word */
	uint32_t sum = 0, i;

	for (i = 0; i + 1 < len; i += 2)
		sum += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
	if (len & 1)
		sum += p[len - 1];
	return sum;
}

int oracle_helper_udp_tcp_chksum(uint8_t *frame, uint32_t frame_len, uint32_t l3_off,
				 uint32_t l4_off, int is_ipv6, int is_tcp, int op,
				 uint16_t *chksum_out)
{
	uint32_t ck_off = l4_off + (is_tcp ? 16u : 6u);
	uint32_t l3_len, l4_len, sum, ones;
	uint16_t stored, chksum;
	const uint8_t *addrs;
	uint32_t addrs_len, proto;

	if (ck_off + 2 > frame_len || l4_off < l3_off)
		return -1;
	stored = (uint16_t)(frame[ck_off] | (frame[ck_off + 1] << 8));
	/* VERIFY of a UDP packet without checksum (:152-154) */
	if (op == 1 && stored == 0 && !is_tcp && chksum_out == NULL)
		return 1;
	if (op == 0 && stored != 0) {                    /* :158-164 */
		frame[ck_off] = 0;
		frame[ck_off + 1] = 0;
	}
	if (!is_ipv6) {                                  /* odph_process_l3_hdr :198-210 */
		if (l3_off + 20 > frame_len)
			return -1;
		addrs = frame + l3_off + 12;
		addrs_len = 8;
		proto = frame[l3_off + 9];
		l3_len = ((uint32_t)frame[l3_off + 2] << 8) | frame[l3_off + 3];
	} else {                                         /* :211-224 */
		if (l3_off + 40 > frame_len)
			return -1;
		addrs = frame + l3_off + 8;
		addrs_len = 32;
		proto = frame[l3_off + 6];
		l3_len = (((uint32_t)frame[l3_off + 4] << 8) | frame[l3_off + 5]) + 40;
	}
	l4_len = is_tcp ? l3_len - (l4_off - l3_off)
			: (((uint32_t)frame[l4_off + 4] << 8) | frame[l4_off + 5]);
	if (l4_len > frame_len - l4_off)   /* would walk past the last segment */
		return -1;
	sum = helper_seg_sum(addrs, addrs_len);
	/* swap_buf {len_hi, len_lo, 0, proto} as two host-order words (:241-246) */
	sum += ((l4_len >> 8) & 0xFF) | ((l4_len & 0xFF) << 8);
	sum += (uint32_t)proto << 8;
	sum += helper_seg_sum(frame + l4_off, l4_len);
	ones = (sum & 0xFFFF) + (sum >> 16);             /* :329-331 */
	ones = (ones & 0xFFFF) + (ones >> 16);
	chksum = (uint16_t)(~ones & 0xFFFF);
	if (chksum_out)
		*chksum_out = chksum;
	if (op == 0) {
		frame[ck_off] = (uint8_t)chksum;
		frame[ck_off + 1] = (uint8_t)(chksum >> 8);
		return 0;
	}
	if (op == 1) {                                   /* :342-347 */
		if (stored == 0 && !is_tcp)
			return 1;
		return chksum == 0 ? 0 : 2;
	}
	return 0;
}

/* ======================================================================
 * example/l3fwd forwarding decision.
 * Restated from example/l3fwd/odp_l3fwd.c, odp_l3fwd_db.c, odp_l3fwd_lpm.c.
 * ==================================================================== */
#include "../include/odpg_fwd.h"

/* ---- 16-4-4-4-4 trie of odp_l3fwd_lpm.c, node-array form ---------------
 * fib_node_t (:31-38) keeps {next_hop | next, valid:1, end:1, depth:6}; a
 * node's children are 16 consecutive nodes of the sub-table pool. Every
 * quirk of the reference builder is kept: fib_alloc_sub (:57-74) hands out
 * the nodes at (k + 1) * 16; a split (:107-122) copies next_hop / depth to
 * the children but leaves them invalid; a depth <= 16 route touches one
 * first-level node (:184-201); a route ending inside a stride updates the
 * single child at `ip >> ip_width` (:124-130); fib_update_node (:76-99)
 * recurses only into children that are leaves. */
#define FIB_L1    65536u
#define FIB_POOL  16384u

typedef struct {
	uint32_t nh;        /* next hop, or first child index in the pool */
	uint8_t valid, end, depth;
} fnode_t;

typedef struct {
	fnode_t l1[FIB_L1];
	fnode_t pool[FIB_POOL];
	uint32_t nsub;
	int overflow;
} fib_t;

static fnode_t *fib_child(fib_t *f, const fnode_t *fe, uint32_t i)
{
	return &f->pool[fe->nh + i];
}

static int fib_new_sub(fib_t *f, uint32_t *base)
{
	uint32_t b = (f->nsub + 1u) * 16u;

	/* the reference resets b entries from its new table on (:52-57) */
	if (2u * b > FIB_POOL) {
		f->overflow = 1;
		return -1;
	}
	for (uint32_t i = 0; i < b; i++) {
		f->pool[b + i].valid = 0;
		f->pool[b + i].end = 1;
	}
	f->nsub++;
	*base = b;
	return 0;
}

static void fib_update(fib_t *f, fnode_t *fe, uint32_t port, uint32_t depth)
{
	if (fe->end) {
		if (!fe->valid) {
			fe->depth = (uint8_t)depth;
			fe->nh = port;
			fe->valid = 1;
		} else if (fe->depth <= depth) {
			fe->nh = port;
			fe->depth = (uint8_t)depth;
		}
		return;
	}
	for (uint32_t i = 0; i < 16u; i++) {
		fnode_t *c = fib_child(f, fe, i);

		if (c->end)
			fib_update(f, c, port, depth);
	}
}

static void fib_insert_sub(fib_t *f, fnode_t *fe, uint32_t ip, uint32_t port,
			   uint32_t width, uint32_t eaten, uint32_t depth)
{
	for (;;) {
		if (fe->end) {
			uint32_t base, old = fe->nh;

			if (fib_new_sub(f, &base))
				return;
			fe->nh = base;
			fe->end = 0;
			if (fe->valid)
				for (uint32_t i = 0; i < 16u; i++) {
					f->pool[base + i].nh = old;
					f->pool[base + i].depth = fe->depth;
				}
		}
		if (depth - eaten <= 4u) {
			width -= depth - eaten;
			fib_update(f, fib_child(f, fe, ip >> width), port, depth);
			return;
		}
		width -= 4u;
		fnode_t *c = fib_child(f, fe, ip >> width);

		ip &= (1u << width) - 1u;
		eaten += 4u;
		fe = c;
	}
}

static void fib_insert(fib_t *f, uint32_t ip, uint32_t port, uint32_t depth)
{
	fnode_t *fe = &f->l1[ip >> 16];

	if (depth <= 16u) {
		if (fe->end) {
			fe->nh = port;
			fe->depth = (uint8_t)depth;
			fe->valid = 1;
			return;
		}
		for (uint32_t i = 0; i < 16u; i++) {
			fnode_t *c = fib_child(f, fe, i);

			if (c->end)
				fib_update(f, c, port, depth);
			else
				for (uint32_t j = 0; j < 16u; j++)
					fib_update(f, fib_child(f, c, j), port, depth);
		}
		return;
	}
	fib_insert_sub(f, fe, ip & 0xffffu, port, 16u, 16u, depth);
}

static int fib_lookup(const fib_t *f, uint32_t ip, int32_t *port)
{
	const fnode_t *fe = &f->l1[ip >> 16];
	uint32_t bits = 16u;

	ip &= 0xffffu;
	while (!fe->end) {
		bits -= 4u;
		fe = &f->pool[fe->nh + (ip >> bits)];
		ip &= (1u << bits) - 1u;
	}
	*port = (int32_t)fe->nh;
	return fe->valid ? 0 : -1;
}

/* ---- find_fwd_db_entry (odp_l3fwd_db.c:474-508): first match in the list,
 * which create_fwd_db_entry() prepends to (:427-428), i.e. newest first. The
 * mask is computed as the reference computes it on x86-64: for depth 32,
 * "1u << 32" shifts by 32 mod 32, so the mask is 0 and only address 0.0.0.0
 * matches; a route with host bits set never matches here. */
static int route_first_match(const odpg_route_t *r, uint32_t n, uint32_t ip)
{
	for (int k = (int)n - 1; k >= 0; k--) {
		uint32_t d = r[k].depth;
		uint32_t mask = ((1u << (d & 31u)) - 1u) << ((32u - d) & 31u);

		if (r[k].addr == (ip & mask))
			return k;
	}
	return -1;
}

/* ---- the hash-mode flow cache (odp_l3fwd_db.c:178-335, 474-508) --------
 * FWD_MAX_FLOW_COUNT flows; keys carry the destination address only. The
 * bucket layout (Jenkins hash, :37-63) decides where a flow sits, never
 * whether it is found, so an exact-match table stands in for the buckets;
 * what is restated literally is the content: init_fwd_hash_cache()'s
 * warm-up walks the route list (newest first), inserting addr + i for
 * i < 2^(32 - depth) (u32 wrap), and stops at the first address already
 * cached or when the flow store is full; find_fwd_db_entry() returns a
 * cached flow's route, else the first list match, which it then caches. */
#define FWD_MAX_FLOW_COUNT (1u << 22)
#define FC_SLOTS (1u << 23)                 /* open addressing, load <= 1/2 */

typedef struct {
	uint32_t *key;       /* dst + 1 (0 = empty) */
	int32_t *route;
	uint32_t used;
} fcache_t;

static uint32_t fc_slot(uint32_t dst)
{
	uint32_t h = dst * 0x9e3779b1u;

	return (h ^ (h >> 15)) & (FC_SLOTS - 1u);
}

static int fc_find(const fcache_t *c, uint32_t dst, int32_t *route)
{
	for (uint32_t s = fc_slot(dst);; s = (s + 1u) & (FC_SLOTS - 1u)) {
		if (c->key[s] == 0u)
			return 0;
		if (c->key[s] == dst + 1u) {
			*route = c->route[s];
			return 1;
		}
	}
}

/* insert_fwd_cache + get_new_flow: 0 when the flow store is exhausted */
static int fc_insert(fcache_t *c, uint32_t dst, int32_t route)
{
	uint32_t s;

	if (c->used >= FWD_MAX_FLOW_COUNT)
		return 0;
	for (s = fc_slot(dst); c->key[s] != 0u; s = (s + 1u) & (FC_SLOTS - 1u))
		;
	c->key[s] = dst + 1u;
	c->route[s] = route;
	c->used++;
	return 1;
}

static int fc_warm(fcache_t *c, const odpg_route_t *r, uint32_t n)
{
	int32_t dummy;

	c->key = calloc(FC_SLOTS, sizeof(uint32_t));
	c->route = calloc(FC_SLOTS, sizeof(int32_t));
	c->used = 0;
	if (!c->key || !c->route)
		return -1;
	for (int k = (int)n - 1; k >= 0; k--) {
		uint64_t nb = 1ull << (32u - r[k].depth);

		for (uint64_t i = 0; i < nb; i++) {
			uint32_t dst = r[k].addr + (uint32_t)i;

			if (fc_find(c, dst, &dummy))
				return 0;              /* "if (flow) return;" */
			if (!fc_insert(c, dst, k))
				return 0;              /* flow store exhausted: goto out */
		}
	}
	return 0;
}

static int fwd_hash_lookup(fcache_t *c, const odpg_route_t *r, uint32_t n, uint32_t dst)
{
	int32_t k;

	if (fc_find(c, dst, &k))
		return k;
	k = route_first_match(r, n, dst);
	if (k >= 0)
		fc_insert(c, dst, k);
	return k;
}

static uint32_t rd_be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* One batch through drop_err_pkts + l3fwd_pkt_hash / l3fwd_pkt_lpm
 * (odp_l3fwd.c:183-292), `reps` times over the same frames (the CPU
 * baseline's passes; tests use 1). The LPM trie or the warmed flow cache is
 * built once, as l3fwd's init does before its workers start (setup_fwd_db,
 * init_fwd_hash_cache); *pass_ns (optional) gets the time of the passes
 * alone. frames are rewritten in place; out_port[i] = port or -1
 * (dropped). Returns 0, or -1 for a route set outside the supported domain
 * (see include/odpg_fwd.h). */
int oracle_l3fwd_reps(const odpg_route_t *routes, uint32_t nroutes, const odpg_fwd_param_t *prm,
		      uint8_t *frames, uint32_t stride, uint32_t num, int32_t sif, int error_check,
		      int32_t *out_port, uint32_t reps, uint64_t *pass_ns)
{
	fib_t *fib = NULL;
	fcache_t fc = { NULL, NULL, 0 };
	struct timespec t0, t1;

	pthread_once(&crc_once, crc_init);
	if (nroutes > ODPG_FWD_MAX_ROUTES)
		return -1;
	if (prm->mode == ODPG_FWD_LPM) {
		fib = calloc(1, sizeof(*fib));
		if (!fib)
			return -1;
		for (uint32_t i = 0; i < FIB_L1; i++)
			fib->l1[i].end = 1;               /* fib_tbl_init (:140-172) */
		/* setup_fwd_db walks the list newest first (odp_l3fwd.c:154-176) */
		for (int k = (int)nroutes - 1; k >= 0; k--)
			fib_insert(fib, routes[k].addr, (uint32_t)routes[k].oif_id, routes[k].depth);
		if (fib->overflow) {
			free(fib);
			return -1;
		}
	} else {
		for (uint32_t k = 0; k < nroutes; k++)
			if (routes[k].depth < 1 || routes[k].depth > 32)
				return -1;
		if (fc_warm(&fc, routes, nroutes)) {
			free(fc.key);
			free(fc.route);
			return -1;
		}
	}
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (uint32_t rep = 0; rep < reps; rep++)
	for (uint32_t i = 0; i < num; i++) {
		uint8_t *fr = frames + (size_t)i * stride;
		pv_t v = { fr, stride };
		hdr_t h;
		int ret;

		memset(&h, 0, sizeof(h));
		h.l2_offset = h.l3_offset = h.l4_offset = OFFSET_INVALID;
		ret = parse_common(&h, &v, stride, error_check ? LAYER_ALL : LAYER_L4, 0);
		if (ret < 0 || (error_check && (h.flags & F_ERROR_MASK)) ||
		    !(h.input_flags & IFB(IF_IPV4))) {
			out_port[i] = -1;
			continue;
		}
		uint8_t *ip = fr + h.l3_offset;
		uint32_t dst = rd_be32(ip + 16);
		int32_t dif;
		/* ipv4_dec_ttl_csum_update (odp_l3fwd.c:183-192): raw LE u16 of the
		 * checksum field, a = ~cpu_to_be_16(0x100) = 0xfffe */
		uint16_t cs = (uint16_t)(ip[10] | (ip[11] << 8));

		ip[8]--;
		cs = cs >= 0xfffeu ? (uint16_t)(cs - 0xfffeu) : (uint16_t)(cs + 1u);
		ip[10] = (uint8_t)cs;
		ip[11] = (uint8_t)(cs >> 8);
		if (prm->mode == ODPG_FWD_LPM) {
			int32_t p;

			dif = fib_lookup(fib, dst, &p) ? sif : p;
			memcpy(fr, prm->dest_mac[dif], 6);
			memcpy(fr + 6, prm->port_mac[dif], 6);
		} else {
			int k = fwd_hash_lookup(&fc, routes, nroutes, dst);

			if (k >= 0) {
				memcpy(fr + 6, routes[k].src_mac, 6);
				memcpy(fr, routes[k].dst_mac, 6);
				dif = routes[k].oif_id;
			} else {
				memcpy(fr, fr + 6, 6);          /* eth->dst = eth->src */
				dif = sif;
			}
		}
		out_port[i] = dif;
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	if (pass_ns)
		*pass_ns = (uint64_t)(t1.tv_sec - t0.tv_sec) * 1000000000ull +
			   (uint64_t)(t1.tv_nsec - t0.tv_nsec);
	free(fib);
	free(fc.key);
	free(fc.route);
	return 0;
}

int oracle_l3fwd(const odpg_route_t *routes, uint32_t nroutes, const odpg_fwd_param_t *prm,
		 uint8_t *frames, uint32_t stride, uint32_t num, int32_t sif, int error_check,
		 int32_t *out_port)
{
	return oracle_l3fwd_reps(routes, nroutes, prm, frames, stride, num, sif, error_check,
				 out_port, 1u, NULL);
}

/* test hook: trie lookup of one address after building from routes[] */
int oracle_fib_lookup(const odpg_route_t *routes, uint32_t nroutes, const uint32_t *ips,
		      uint32_t n, int32_t *port, int32_t *valid)
{
	fib_t *fib = calloc(1, sizeof(*fib));

	if (!fib)
		return -1;
	for (uint32_t i = 0; i < FIB_L1; i++)
		fib->l1[i].end = 1;
	for (int k = (int)nroutes - 1; k >= 0; k--)
		fib_insert(fib, routes[k].addr, (uint32_t)routes[k].oif_id, routes[k].depth);
	for (uint32_t i = 0; i < n; i++)
		valid[i] = fib_lookup(fib, ips[i], &port[i]) == 0;
	int ovf = fib->overflow;

	free(fib);
	return ovf ? -1 : 0;
}

/* ==========================================================================
 * Loop pktio transmit side (include/odpg_tx.h):
 * loopback_fix_checksums + get_dest_queue, per packet of loopback_send()
 * (pktio/loop.c:525-575). Frames are rewritten in place.
 * ========================================================================== */
#include "../include/odpg_tx.h"

typedef struct {
	uint8_t *d;        /* writable frame */
	uint32_t len;      /* frame_len */
} wv_t;

/* odp_packet_copy_from_mem (fails when the range leaves the frame) */
static int tx_write(wv_t *w, uint32_t off, const void *src, uint32_t n)
{
	if (off + n > w->len)
		return -1;
	memcpy(w->d + off, src, n);
	return 0;
}

/* packet_sum_partial (odp_packet.c:1669-1692): 0 when the range leaves the
 * frame; `offset - l3` selects the odd-byte swap */
static uint64_t tx_sum_partial(const wv_t *w, uint32_t l3, uint32_t off, uint32_t len)
{
	pv_t v = { w->d, w->len };

	/* (a range whose end wraps past 2^32, only for metadata offsets beyond
	 * the frame, is treated as leaving the frame) */
	if (off > w->len || len > w->len - off)
		return 0;
	return chksum_partial(&v, off, len, off - l3);
}

/* check_proto (loop.c:382-411) */
static int tx_check_proto(const wv_t *w, uint32_t l3, int *v4, uint8_t *l4p)
{
	pv_t v = { w->d, w->len };
	uint32_t l3_len = w->len - l3;
	uint8_t ver = (uint8_t)(B(&v, l3) >> 4);

	if (ver == 4 && l3_len >= 20) {
		*v4 = 1;
		*l4p = (be16(&v, l3 + 6) & 0x3fff) ? 255 : B(&v, l3 + 9);
		return 0;
	}
	if (ver == 6 && l3_len >= 40) {
		*v4 = 0;
		*l4p = B(&v, l3 + 6);
		return 0;
	}
	return -1;
}

/* _odp_packet_ipv4_chksum_insert + packet_ipv4_chksum (odp_packet.c:1729-1787) */
static int tx_ipv4_insert(wv_t *w, uint32_t l3)
{
	uint8_t buf[60];
	uint32_t nleft;
	uint16_t c;

	if (l3 == OFFSET_INVALID || l3 + 20 > w->len)
		return -1;
	nleft = (uint32_t)(w->d[l3] & 0x0f) * 4;
	if (nleft < 20 || l3 + nleft > w->len)
		return -1;
	memcpy(buf, w->d + l3, nleft);
	buf[10] = buf[11] = 0;
	c = (uint16_t)~chksum_finalize(chksum_partial_mem(buf, nleft, 0));
	return tx_write(w, l3 + 10, &c, 2);
}

/* _odp_packet_tcp_udp_chksum_insert (odp_packet.c:1789-1862) */
static int tx_tcp_udp_insert(wv_t *w, uint32_t l3, uint32_t l4, uint16_t proto)
{
	uint64_t sum;
	uint32_t zero = 0, csum_off = l4 + 6;   /* _ODP_UDP_CSUM_OFFSET for both */
	uint16_t c;

	if (l3 == OFFSET_INVALID || l4 == OFFSET_INVALID)
		return -1;
	if ((w->d[l3] >> 4) == 4)
		sum = tx_sum_partial(w, l3, l3 + 12, 8);
	else
		sum = tx_sum_partial(w, l3, l3 + 8, 32);
	sum += (uint64_t)proto << 8;
	if (proto == 6) {
		uint16_t tl = (uint16_t)(w->len - l4);

		sum += (uint16_t)((tl >> 8) | (tl << 8));      /* odp_cpu_to_be_16 */
	} else {
		sum += tx_sum_partial(w, l3, l4 + 4, 2);
	}
	tx_write(w, csum_off, &zero, 2);
	sum += tx_sum_partial(w, l3, l4, w->len - l4);
	c = (uint16_t)~chksum_finalize(sum);
	if (proto == 17 && c == 0)
		c = 0xffff;
	return tx_write(w, csum_off, &c, 2);
}

/* _odp_packet_sctp_chksum_insert (odp_packet.c:1884-1898) */
static int tx_sctp_insert(wv_t *w, uint32_t l4)
{
	uint32_t sum = 0;
	pv_t v;

	if (l4 == OFFSET_INVALID)
		return -1;
	tx_write(w, l4 + 8, &sum, 4);
	v.d = w->d;
	v.len = w->len;
	sum = ~0u;
	if (l4 <= w->len)      /* packet_sum_crc32c: init returned if out of frame */
		sum = crc32c(&v, l4, w->len - l4, sum);
	sum = ~sum;
	return tx_write(w, l4 + 8, &sum, 4);
}

/* get_dest_queue (loop.c:468-523) */
static uint32_t tx_dest_queue(const wv_t *w, uint32_t l3, uint32_t l4, uint32_t fl,
			      const odpg_tx_cfg_t *cfg)
{
	const uint32_t hp = cfg->hash_proto;
	uint8_t data[36];
	uint32_t n = 0;
	pv_t v = { w->d, w->len };

	if (hp == 0)
		return cfg->index % cfg->num_qs;
	memset(data, 0, sizeof(data));
	if (l4 != OFFSET_INVALID) {
		if ((hp & (ODPG_HASH_IPV4_UDP | ODPG_HASH_IPV6_UDP)) && (fl & ODPG_TX_HAS_UDP)) {
			if (l4 + 8 <= w->len) {
				memcpy(data + n, w->d + l4, 4);       /* src_port, dst_port */
				n += 4;
			}
		} else if ((hp & (ODPG_HASH_IPV4_TCP | ODPG_HASH_IPV6_TCP)) &&
			   (fl & ODPG_TX_HAS_TCP)) {
			if (l4 + 20 <= w->len) {
				memcpy(data + n, w->d + l4, 4);
				n += 4;
			}
		}
	}
	if (l3 != OFFSET_INVALID) {
		if ((hp & ODPG_HASH_IPV4) && (fl & ODPG_TX_HAS_IPV4)) {
			if (l3 + 20 <= w->len) {
				memcpy(data + n, w->d + l3 + 12, 8);  /* src_addr, dst_addr */
				n += 8;
			}
		} else if ((hp & ODPG_HASH_IPV6) && (fl & ODPG_TX_HAS_IPV6)) {
			if (l3 + 40 <= w->len) {
				memcpy(data + n, w->d + l3 + 8, 32);
				n += 32;
			}
		}
	}
	v.d = data;
	v.len = n;
	return crc32c(&v, 0, n, 0) % cfg->num_qs;
}

#define OL_TX_CHKSUM_PKT(cfg, capa, proto, ovr_set, ovr) \
	((capa) && (proto) && ((ovr_set) ? (ovr) : (cfg)))   /* loop.c:379-380 */

/* loopback_fix_checksums (loop.c:415-466) + get_dest_queue for packet i */
static uint32_t tx_one(wv_t *w, uint32_t l3, uint32_t l4, uint32_t fl, const odpg_tx_cfg_t *cfg)
{
	uint32_t res = 0;
	int v4 = 0;
	uint8_t l4p = 0;

	if (l3 != OFFSET_INVALID && l3 < w->len && tx_check_proto(w, l3, &v4, &l4p) == 0) {
		const uint64_t c = cfg->pktout_cfg, k = cfg->pktout_capa;
		const int l3s = !!(fl & ODPG_TX_L3_CHKSUM_SET), l3o = !!(fl & ODPG_TX_L3_CHKSUM);
		const int l4s = !!(fl & ODPG_TX_L4_CHKSUM_SET), l4o = !!(fl & ODPG_TX_L4_CHKSUM);
		const int ip4 = OL_TX_CHKSUM_PKT(!!(c & ODPG_PKTOUT_IPV4_CHKSUM),
						 !!(k & ODPG_PKTOUT_IPV4_CHKSUM), v4, l3s, l3o);
		const int udp = OL_TX_CHKSUM_PKT(!!(c & ODPG_PKTOUT_UDP_CHKSUM),
						 !!(k & ODPG_PKTOUT_UDP_CHKSUM), l4p == 17, l4s, l4o);
		const int tcp = OL_TX_CHKSUM_PKT(!!(c & ODPG_PKTOUT_TCP_CHKSUM),
						 !!(k & ODPG_PKTOUT_TCP_CHKSUM), l4p == 6, l4s, l4o);
		const int sctp = OL_TX_CHKSUM_PKT(!!(c & ODPG_PKTOUT_SCTP_CHKSUM),
						  !!(k & ODPG_PKTOUT_SCTP_CHKSUM), l4p == 132, l4s, l4o);

		if (ip4 && tx_ipv4_insert(w, l3) == 0)
			res |= ODPG_TX_OUT_IPV4;
		if (tcp && tx_tcp_udp_insert(w, l3, l4, 6) == 0)
			res |= ODPG_TX_OUT_TCP;
		if (udp && tx_tcp_udp_insert(w, l3, l4, 17) == 0)
			res |= ODPG_TX_OUT_UDP;
		if (sctp && tx_sctp_insert(w, l4) == 0)
			res |= ODPG_TX_OUT_SCTP;
	}
	return res | (tx_dest_queue(w, l3, l4, fl, cfg) & ODPG_TX_OUT_QUEUE_MASK);
}

/* Batch entry (host buffers). meta == NULL: each frame is parsed first
 * (_odp_packet_parse_common, all layers, no checksum options). Returns 0, or
 * -1 for num_qs == 0. */
int oracle_tx_prepare(uint8_t *frames, const odpg_desc_t *desc, uint32_t stride, uint32_t num,
		      const odpg_tx_meta_t *meta, const odpg_tx_cfg_t *cfg, uint32_t *out)
{
	if (!cfg || cfg->num_qs == 0)
		return -1;
	pthread_once(&crc_once, crc_init);
	for (uint32_t i = 0; i < num; i++) {
		wv_t w;
		uint32_t l3, l4, fl;

		if (desc) {
			w.d = frames + desc[i].offset;
			w.len = desc[i].len;
		} else {
			w.d = frames + (size_t)i * stride;
			w.len = stride;
		}
		if (meta) {
			l3 = meta[i].l3_offset;
			l4 = meta[i].l4_offset;
			fl = meta[i].flags;
		} else {
			hdr_t h;
			pv_t v = { w.d, w.len };

			memset(&h, 0, sizeof(h));
			h.l2_offset = h.l3_offset = h.l4_offset = OFFSET_INVALID;
			parse_common(&h, &v, v.len, LAYER_ALL, 0);
			l3 = h.l3_offset;
			l4 = h.l4_offset;
			fl = ((h.input_flags & IFB(IF_IPV4)) ? ODPG_TX_HAS_IPV4 : 0u) |
			     ((h.input_flags & IFB(IF_IPV6)) ? ODPG_TX_HAS_IPV6 : 0u) |
			     ((h.input_flags & IFB(IF_UDP)) ? ODPG_TX_HAS_UDP : 0u) |
			     ((h.input_flags & IFB(IF_TCP)) ? ODPG_TX_HAS_TCP : 0u);
		}
		out[i] = tx_one(&w, l3, l4, fl, cfg);
	}
	return 0;
}
