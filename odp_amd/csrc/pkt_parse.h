/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Device-side packet parse shared by the gfx950 kernels (classify.hip,
 * fwd.hip): frame byte access over an LDS window with an optional global
 * tail, the restated _odp_packet_parse_common (odp_parse_internal.h:80-112,
 * odp_parse.c:23-475) with the RX checksum verdicts (odp_packet.c:1906-1984),
 * the wave-cooperative long-frame checksum tails, and the register fast
 * path for plain 64-byte Eth/IPv4/UDP|TCP frames.
 */
#ifndef ODPG_PKT_PARSE_H_
#define ODPG_PKT_PARSE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/odpg.h"
#include "odpg_internal.h"

#define BLOCK 256

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

/* 16-byte load of once-read frame data. Lane-per-frame loads (lanes 64 B
 * apart) use the default cache policy: with the nontemporal hint the same
 * pattern streams at 3.7 TB/s instead of 5.5 (tools/diag_stream.py,
 * patterns 1 vs 17). */
__device__ __forceinline__ uint4 ld_stream(const uint4 *p)
{
	return *p;
}

/* nontemporal 16-byte load: for coalesced streaming only (a lane-per-frame
 * pattern with this hint runs at 2/3 of the plain load's rate,
 * profiles/r01/diag_stream_floor.jsonl) */
__device__ __forceinline__ uint4 ld_nt16(const uint4 *p)
{
	typedef unsigned int nt_u32x4 __attribute__((ext_vector_type(4)));
	const nt_u32x4 v = __builtin_nontemporal_load((const nt_u32x4 *)p);

	return make_uint4(v.x, v.y, v.z, v.w);
}

#define IF(x)  (1ull << (x))
#define FB(x)  (1u << (x))

/* ----------------------------------------------------------------------- */
/* packet byte access: LDS window, optional global tail, zero past frame    */
template <int W, bool GF>
struct Pkt {
	const uint32_t *row;   /* LDS, W/4 dwords of the frame start */
	const uint8_t  *g;     /* global frame start (16-byte aligned) */
	uint32_t        len;

	__device__ __forceinline__ uint32_t word(uint32_t w) const
	{
		if (w < (uint32_t)(W / 4))
			return row[w];
		if (GF) {
			uint32_t nw = (len + 3u) >> 2;

			if (w < nw) {
				uint32_t x = *(const uint32_t *)(g + 4u * w);
				uint32_t rem = len - 4u * w;

				if (rem < 4u)
					x &= (1u << (8u * rem)) - 1u;
				return x;
			}
		}
		return 0u;
	}

	/* little-endian u32 of bytes [pos, pos + 4) */
	__device__ __forceinline__ uint32_t rd32(uint32_t pos) const
	{
		uint32_t w = pos >> 2;
		uint32_t lo = word(w);

		if ((pos & 3u) == 0u)
			return lo;
		uint32_t hi = word(w + 1u);

		return __builtin_amdgcn_alignbyte(hi, lo, pos & 3u);
	}

	__device__ __forceinline__ uint32_t u8(uint32_t pos) const
	{
		return (word(pos >> 2) >> (8u * (pos & 3u))) & 0xffu;
	}

	/* network-order 16-bit field */
	__device__ __forceinline__ uint32_t be16(uint32_t pos) const
	{
		uint32_t x = rd32(pos);

		return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
	}

	/* raw little-endian 16-bit load (what the reference's u16 reads see) */
	__device__ __forceinline__ uint32_t raw16(uint32_t pos) const
	{
		return rd32(pos) & 0xffffu;
	}
};

/* one's-complement accumulate (end-around carry): keeps the residue mod
 * 0xffff of the reference's 64-bit sum of little-endian words
 * (chksum_partial, odp_chksum_internal.h:60-196) and is zero only when every
 * added word is zero, so the folded verdict is identical. */
__device__ __forceinline__ uint32_t oc_add(uint32_t s, uint32_t x)
{
	uint32_t r = s + x;

	return r + (r < x ? 1u : 0u);
}

/* chksum_finalize (odp_chksum_internal.h:22-31) of a one's-complement sum */
__device__ __forceinline__ uint32_t oc_fold(uint32_t s)
{
	s = (s >> 16) + (s & 0xffffu);
	s = (s >> 16) + (s & 0xffffu);
	return s;
}

/* sum of bytes [a, b) of the frame, a even, bytes past the frame zero */
template <int W, bool GF>
__device__ uint32_t sum_range(const Pkt<W, GF> &v, uint32_t a, uint32_t b)
{
	if (b > v.len)
		b = v.len;
	if (b <= a)
		return 0u;
	uint32_t w0 = a >> 2, w1 = (b - 1u) >> 2;
	uint32_t s = 0;
	uint32_t lim = w1 < (uint32_t)(W / 4 - 1) ? w1 : (uint32_t)(W / 4 - 1);
	uint32_t w = w0;

	/* part inside the LDS window */
	for (; w <= lim; ++w) {
		uint32_t x = v.row[w];

		if (w == w0 && (a & 3u))
			x &= 0xffff0000u;
		if (w == w1 && (b & 3u))
			x &= (1u << (8u * (b & 3u))) - 1u;
		s = oc_add(s, x);
	}
	if (GF && w <= w1) {
		/* tail beyond the window, straight from HBM: 16 B per load once
		 * the word index is 16-byte aligned */
		for (; w <= w1 && (w & 3u); ++w) {
			uint32_t x = v.word(w);

			if (w == w0 && (a & 3u))
				x &= 0xffff0000u;
			if (w == w1 && (b & 3u))
				x &= (1u << (8u * (b & 3u))) - 1u;
			s = oc_add(s, x);
		}
		/* whole 16-byte chunks: 64-bit accumulation (one add per word),
		 * four loads in flight per step; folded end-around below, which
		 * keeps the residue mod 0xffff (0xffffffff = 0xffff * 0x10001) */
		uint64_t acc = 0ull;

		if (w == w0 && (a & 3u) && w + 4u <= w1) {
			uint4 q = *(const uint4 *)(v.g + 4u * w);

			acc += (uint64_t)(q.x & 0xffff0000u) + q.y + q.z + q.w;
			w += 4u;
		}
		while (w + 16u <= w1) {
			const uint4 *gp = (const uint4 *)(v.g + 4u * w);
			const uint4 q0 = gp[0], q1 = gp[1], q2 = gp[2], q3 = gp[3];

			acc += (uint64_t)q0.x + q0.y + q0.z + q0.w;
			acc += (uint64_t)q1.x + q1.y + q1.z + q1.w;
			acc += (uint64_t)q2.x + q2.y + q2.z + q2.w;
			acc += (uint64_t)q3.x + q3.y + q3.z + q3.w;
			w += 16u;
		}
		while (w + 4u <= w1) {
			const uint4 q = *(const uint4 *)(v.g + 4u * w);

			acc += (uint64_t)q.x + q.y + q.z + q.w;
			w += 4u;
		}
		acc = (acc & 0xffffffffull) + (acc >> 32);
		s = oc_add(oc_add(s, (uint32_t)acc), (uint32_t)(acc >> 32));
		for (; w <= w1; ++w) {
			uint32_t x = v.word(w);

			if (w == w0 && (a & 3u))
				x &= 0xffff0000u;
			if (w == w1 && (b & 3u))
				x &= (1u << (8u * (b & 3u))) - 1u;
			s = oc_add(s, x);
		}
	}
	return s;
}

/* CRC32C (reflected Castagnoli, no final xor: arch/default/odp_hash_crc32.c) */
__device__ __forceinline__ uint32_t crc32c_byte(uint32_t crc, uint32_t b)
{
	crc ^= b;
#pragma unroll
	for (int k = 0; k < 8; ++k)
		crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
	return crc;
}

template <int W, bool GF>
__device__ uint32_t crc32c_range(const Pkt<W, GF> &v, uint32_t off, uint32_t len, uint32_t crc)
{
	for (uint32_t i = 0; i < len; ++i)
		crc = crc32c_byte(crc, v.u8(off + i));
	return crc;
}

/* ----------------------------------------------------------------------- */
struct Prs {
	uint64_t inf;
	uint32_t fl;
	uint32_t l2, l3, l4;
};

enum { LAYER_NONE = 0, LAYER_L2, LAYER_L3, LAYER_L4, LAYER_ALL };

/* _odp_parse_eth (odp_parse.c:23-106) */
template <int W, bool GF>
__device__ __forceinline__ uint32_t parse_eth(Prs &p, const Pkt<W, GF> &v, uint32_t &off)
{
	uint64_t inf = IF(IFL_L2) | IF(IFL_ETH);
	uint32_t len = v.len;
	uint32_t w0 = v.word(0), w1 = v.word(1), w3 = v.word(3);
	uint32_t mac0 = ((w0 & 0xffu) << 8) | ((w0 >> 8) & 0xffu);
	uint32_t ethtype = ((w3 & 0xffu) << 8) | ((w3 >> 8) & 0xffu);

	if (len - off > 1514u)
		inf |= IF(IFL_JUMBO);
	if (mac0 & 0x0100u)
		inf |= IF(IFL_ETH_MCAST);
	if (mac0 == 0xffffu && (w0 >> 16) == 0xffffu && (w1 & 0xffffu) == 0xffffu)
		inf |= IF(IFL_ETH_BCAST);
	off += 14u;

	if (ethtype < 1514u) {
		inf |= IF(IFL_SNAP);
		if (ethtype > len - off) {
			p.fl |= FB(FL_SNAP_LEN_ERR);
			p.inf |= inf;
			return 0u;
		}
		ethtype = v.be16(off + 6u);
		off += 8u;
	}
	if (ethtype == 0x88A8u) {
		inf |= IF(IFL_VLAN_QINQ) | IF(IFL_VLAN);
		ethtype = v.be16(off + 2u);
		off += 4u;
	}
	if (ethtype == 0x8100u) {
		inf |= IF(IFL_VLAN);
		ethtype = v.be16(off + 2u);
		off += 4u;
	}
	if (off > len) {
		inf = IF(IFL_L2);
		ethtype = 0u;
	}
	p.inf |= inf;
	return ethtype;
}

/* parse_ipv4 (odp_parse.c:113-169); returns proto, accumulates pseudo header */
template <int W, bool GF>
__device__ __forceinline__ uint32_t parse_ipv4(Prs &p, const Pkt<W, GF> &v, uint32_t &off,
					       uint64_t opt, uint32_t &l4sum)
{
	uint32_t o = off;
	uint32_t len = v.len;
	uint32_t h0 = v.rd32(o);            /* ver_ihl tos tot_len */
	uint32_t h1 = v.rd32(o + 4u);       /* id frag_offset */
	uint32_t h2 = v.rd32(o + 8u);       /* ttl proto chksum */
	uint32_t dst = v.rd32(o + 16u);     /* raw */
	uint32_t ver = (h0 & 0xf0u) >> 4, ihl = h0 & 0x0fu;
	uint32_t l3_len = ((h0 >> 8) & 0xff00u) | (h0 >> 24);
	uint32_t frag = ((h1 >> 8) & 0xff00u) | (h1 >> 24);
	uint32_t dst_be = __builtin_bswap32(dst);

	if ((p.fl & FB(FL_L3_CHKSUM_ERR)) || ihl < 5u || ver != 4u || 20u > len - o ||
	    l3_len > len - o) {
		p.fl |= FB(FL_IP_ERR);
		return 0u;
	}
	if (opt & ODPG_PKTIN_IPV4_CHKSUM) {
		p.inf |= IF(IFL_L3_CHKSUM_DONE);
		if (oc_fold(sum_range(v, o, o + ihl * 4u)) != 0xffffu) {
			p.fl |= FB(FL_IP_ERR) | FB(FL_L3_CHKSUM_ERR);
			return 0u;
		}
	}
	off += ihl * 4u;
	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM))
		l4sum = sum_range(v, o + 12u, o + 20u);
	if (ihl > 5u)
		p.inf |= IF(IFL_IPOPT);
	if (frag & 0x3fffu)
		p.inf |= IF(IFL_IPFRAG);
	if (dst_be == 0xffffffffu)
		p.inf |= IF(IFL_IP_BCAST);
	if ((dst_be >> 28) == 0xeu)
		p.inf |= IF(IFL_IP_MCAST);
	return (h2 >> 8) & 0xffu;
}

/* parse_ipv6 (odp_parse.c:179-245) */
template <int W, bool GF>
__device__ __forceinline__ uint32_t parse_ipv6(Prs &p, const Pkt<W, GF> &v, uint32_t &off,
					       uint32_t seg_end, uint64_t opt, uint32_t &l4sum)
{
	uint32_t o = off;
	uint32_t len = v.len;
	uint32_t h0 = v.rd32(o);            /* ver_tc_flow */
	uint32_t h1 = v.rd32(o + 4u);       /* payload_len next_hdr hop_limit */
	uint32_t vtf = __builtin_bswap32(h0);
	uint32_t payload_len = ((h1 & 0xffu) << 8) | ((h1 >> 8) & 0xffu);
	uint32_t next_hdr = (h1 >> 16) & 0xffu;
	uint32_t dst0 = v.u8(o + 24u);

	if ((p.fl & FB(FL_L3_CHKSUM_ERR)) || (vtf >> 28) != 6u || 40u > len - o ||
	    payload_len + 40u > len - o) {
		p.fl |= FB(FL_IP_ERR);
		return 0u;
	}
	if (dst0 == 0xffu)
		p.inf |= IF(IFL_IP_MCAST);
	else
		p.inf &= ~IF(IFL_IP_MCAST);
	p.inf &= ~IF(IFL_IP_BCAST);
	off += 40u;
	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM))
		l4sum = sum_range(v, o + 8u, o + 40u);

	if (next_hdr == 0x00u || next_hdr == 0x2Bu) {
		uint32_t ext_next;

		p.inf |= IF(IFL_IPOPT);
		do {
			uint32_t e = off;

			ext_next = v.u8(e);
			off += 8u + v.u8(e + 1u) * 8u;
		} while ((ext_next == 0x00u || ext_next == 0x2Bu) && off < seg_end);

		if (off >= p.l3 + payload_len) {
			p.fl |= FB(FL_IP_ERR);
			return 0u;
		}
		if (ext_next == 0x2Cu)
			p.inf |= IF(IFL_IPFRAG);
		return ext_next;
	}
	if (next_hdr == 0x2Cu)
		p.inf |= IF(IFL_IPOPT) | IF(IFL_IPFRAG);
	return next_hdr;
}

/* UDP / TCP checksum of a frame longer than the LDS window, left for the
 * wave-cooperative tail pass (coop_tail_sums): the partial sum of the
 * pseudo header + window bytes and the byte range [a, b) still to add */
struct L4Pend {
	uint32_t kind;      /* 0 none, 1 UDP, 2 TCP */
	uint32_t sum;
	uint32_t a, b;
};

#define PARSE_PEND 2

/* _odp_packet_parse_common (odp_parse_internal.h:80-112) incl. the L3/L4
 * switch (odp_parse.c:360-475) and _odp_packet_l4_chksum (odp_packet.c:1906-1984).
 * With a non-null `pend` (global-tail kernels) the UDP/TCP checksum of a frame
 * longer than the window returns PARSE_PEND instead; finish_l4() applies the
 * verdict once the tail sum is known. */
template <int W, bool GF>
__device__ int parse_common(Prs &p, const Pkt<W, GF> &v, uint32_t layer, uint64_t opt,
			    L4Pend *pend = nullptr)
{
	uint32_t off = 0, len = v.len, seg_end = v.len;
	uint32_t l4sum = 0;
	uint32_t sctp_crc = 0;
	uint32_t ip_proto;

	if (layer == LAYER_NONE)
		return 0;
	p.l2 = 0;
	uint32_t ethtype = parse_eth(p, v, off);

	/* _odp_packet_parse_common_l3_l4 */
	p.l3 = off;
	if (layer <= LAYER_L2)
		return (p.fl & FL_ERROR_MASK) != 0u;
	p.inf |= IF(IFL_L3);
	if (ethtype == 0x0800u) {
		p.inf |= IF(IFL_IPV4);
		ip_proto = parse_ipv4(p, v, off, opt, l4sum);
		if (!(p.fl & FB(FL_IP_ERR)))
			p.l4 = off;
		else if (opt & ODPG_PKTIN_DROP_IPV4_ERR)
			return -1;
	} else if (ethtype == 0x86ddu) {
		p.inf |= IF(IFL_IPV6);
		ip_proto = parse_ipv6(p, v, off, seg_end, opt, l4sum);
		if (!(p.fl & FB(FL_IP_ERR)))
			p.l4 = off;
		else if (opt & ODPG_PKTIN_DROP_IPV6_ERR)
			return -1;
	} else if (ethtype == 0x0806u) {
		p.inf |= IF(IFL_ARP);
		ip_proto = 255u;
	} else {
		p.inf &= ~IF(IFL_L3);
		ip_proto = 255u;
	}
	if (layer == LAYER_L3)
		return (p.fl & FL_ERROR_MASK) != 0u;

	p.inf |= IF(IFL_L4);
	bool frag = (p.inf & IF(IFL_IPFRAG)) != 0;

	switch (ip_proto) {
	case 0x01u:
	case 0x3Au:
		p.inf |= IF(IFL_ICMP);
		break;
	case 0x04u:
		break;
	case 0x06u: {                                       /* parse_tcp :252-274 */
		if (off + 20u > seg_end)
			return -1;
		p.inf |= IF(IFL_TCP);
		if ((v.u8(off + 12u) >> 4) < 5u)
			p.fl |= FB(FL_TCP_ERR);
		if ((opt & ODPG_PKTIN_TCP_CHKSUM) && !frag) {
			uint32_t tl = (len - p.l4) & 0xffffu;

			l4sum = oc_add(l4sum, ((tl >> 8) | (tl << 8)) & 0xffffu);
			l4sum = oc_add(l4sum, 0x06u << 8);
		}
		if ((p.fl & FB(FL_TCP_ERR)) && (opt & ODPG_PKTIN_DROP_TCP_ERR))
			return -1;
		break;
	}
	case 0x11u: {                                       /* parse_udp :281-322 */
		if (off + 8u > seg_end)
			return -1;
		p.inf |= IF(IFL_UDP);
		uint32_t u1 = v.rd32(off + 4u);            /* length chksum */
		uint32_t ulen_raw = u1 & 0xffffu, csum_raw = u1 >> 16;
		uint32_t udplen = ((ulen_raw & 0xffu) << 8) | (ulen_raw >> 8);

		if (udplen < 8u) {
			p.fl |= FB(FL_UDP_ERR);
		} else {
			if ((opt & ODPG_PKTIN_UDP_CHKSUM) && !frag) {
				if (csum_raw == 0u) {
					p.inf |= IF(IFL_L4_CHKSUM_DONE) | IF(IFL_UDP_CHKSUM_ZERO);
					if (!(p.inf & IF(IFL_IPV4)))
						p.fl |= FB(FL_L4_CHKSUM_ERR);
				} else {
					l4sum = oc_add(l4sum, ulen_raw);
					l4sum = oc_add(l4sum, 0x11u << 8);
				}
			}
			if (v.be16(off + 2u) == 4500u && udplen > 4u && v.rd32(off + 8u) != 0u)
				p.inf |= IF(IFL_IPSEC) | IF(IFL_IPSEC_UDP);
		}
		if ((p.fl & FB(FL_UDP_ERR)) && (opt & ODPG_PKTIN_DROP_UDP_ERR))
			return -1;
		break;
	}
	case 0x33u:
		p.inf |= IF(IFL_IPSEC) | IF(IFL_IPSEC_AH);
		break;
	case 0x32u:
		p.inf |= IF(IFL_IPSEC) | IF(IFL_IPSEC_ESP);
		break;
	case 0x84u: {                                       /* parse_sctp :329-352 */
		p.inf |= IF(IFL_SCTP);
		if (((len - p.l4) & 0xffffu) < 12u) {
			p.fl |= FB(FL_SCTP_ERR);
		} else if ((opt & ODPG_PKTIN_SCTP_CHKSUM) && !frag) {
			uint32_t crc = crc32c_range(v, off, 8u, 0xffffffffu);

			for (int k = 0; k < 4; ++k)
				crc = crc32c_byte(crc, 0u);
			sctp_crc = crc;
		}
		if ((p.fl & FB(FL_SCTP_ERR)) && (opt & ODPG_PKTIN_DROP_SCTP_ERR))
			return -1;
		break;
	}
	case 0x3Bu:
		p.inf |= IF(IFL_NO_NEXT_HDR);
		break;
	default:
		p.inf &= ~IF(IFL_L4);
		break;
	}
	if (p.fl & FL_ERROR_MASK)
		return 1;
	if (layer < LAYER_L4)
		return 0;

	/* _odp_packet_l4_chksum (odp_packet.c:1906-1984) */
	uint64_t inf = p.inf;

	if (GF && pend && len > (uint32_t)W &&
	    (((opt & ODPG_PKTIN_UDP_CHKSUM) && (inf & IF(IFL_UDP)) && !(inf & IF(IFL_IPFRAG)) &&
	      !(inf & IF(IFL_UDP_CHKSUM_ZERO))) ||
	     ((opt & ODPG_PKTIN_TCP_CHKSUM) && (inf & IF(IFL_TCP)) && !(inf & IF(IFL_IPFRAG))))) {
		pend->kind = (inf & IF(IFL_UDP)) ? 1u : 2u;
		pend->sum = oc_add(l4sum, sum_range(v, p.l4, (uint32_t)W));
		pend->a = p.l4 > (uint32_t)W ? p.l4 : (uint32_t)W;
		pend->b = len;
		return PARSE_PEND;
	}
	if ((opt & ODPG_PKTIN_UDP_CHKSUM) && (inf & IF(IFL_UDP)) && !(inf & IF(IFL_IPFRAG)) &&
	    !(inf & IF(IFL_UDP_CHKSUM_ZERO))) {
		uint32_t s = oc_add(l4sum, sum_range(v, p.l4, len));

		p.inf |= IF(IFL_L4_CHKSUM_DONE);
		if (oc_fold(s) != 0xffffu) {
			p.fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_UDP_ERR);
			if (opt & ODPG_PKTIN_DROP_UDP_ERR)
				return -1;
		}
	}
	if ((opt & ODPG_PKTIN_TCP_CHKSUM) && (inf & IF(IFL_TCP)) && !(inf & IF(IFL_IPFRAG))) {
		uint32_t s = oc_add(l4sum, sum_range(v, p.l4, len));

		p.inf |= IF(IFL_L4_CHKSUM_DONE);
		if (oc_fold(s) != 0xffffu) {
			p.fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_TCP_ERR);
			if (opt & ODPG_PKTIN_DROP_TCP_ERR)
				return -1;
		}
	}
	if ((opt & ODPG_PKTIN_SCTP_CHKSUM) && (inf & IF(IFL_SCTP)) && !(inf & IF(IFL_IPFRAG))) {
		uint32_t crc = crc32c_range(v, p.l4 + 12u, len - p.l4 - 12u, sctp_crc);

		p.inf |= IF(IFL_L4_CHKSUM_DONE);
		if (~crc != v.rd32(p.l4 + 8u)) {
			p.fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_SCTP_ERR);
			if (opt & ODPG_PKTIN_DROP_SCTP_ERR)
				return -1;
		}
	}
	return (p.fl & FL_ERROR_MASK) != 0u;
}

/* verdict of a PARSE_PEND checksum (the UDP / TCP steps of
 * _odp_packet_l4_chksum, odp_packet.c:1927-1964) given the tail sum */
__device__ __forceinline__ int finish_l4(Prs &p, const L4Pend &pd, uint32_t tail, uint64_t opt)
{
	const uint32_t s = oc_add(pd.sum, tail);

	p.inf |= IF(IFL_L4_CHKSUM_DONE);
	if (oc_fold(s) != 0xffffu) {
		if (pd.kind == 1u) {
			p.fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_UDP_ERR);
			if (opt & ODPG_PKTIN_DROP_UDP_ERR)
				return -1;
		} else {
			p.fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_TCP_ERR);
			if (opt & ODPG_PKTIN_DROP_TCP_ERR)
				return -1;
		}
	}
	return (p.fl & FL_ERROR_MASK) != 0u;
}

/* plain u32 sum over the 64 lanes: DPP row prefix sums, then the four row
 * totals; every lane must be active */
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x)
{
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
	return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) +
	       (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
	       (uint32_t)__builtin_amdgcn_readlane((int)x, 47) +
	       (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

/* this lane's share of frame j's tail [a, b): 16-byte chunks c0 + 16 * idx,
 * idx = lane, lane + 64, ...; only the chunk holding byte b - 1 (and the
 * first one when a is not 16-aligned) is masked, with wave-uniform masks.
 * Returns the share folded to 16 bits (residue mod 0xffff). */
typedef unsigned short tail_us2 __attribute__((ext_vector_type(2)));

/* acc + w.lo16 + w.hi16 (one v_dot2_u32_u16 against {1, 1}) */
__device__ __forceinline__ uint32_t tail_dot2(uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(tail_us2, w),
				      __builtin_bit_cast(tail_us2, 0x00010001u), acc, false);
}

/* inclusive prefix sum over the 64 lanes (DPP row scans, then the row
 * carries by row_bcast:15 / row_bcast:31); every lane must be active */
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t x)
{
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
	return x;
}

/* inclusive prefix max over the 64 lanes (wave_scan_u32's DPP steps with
 * max); every lane must be active */
__device__ __forceinline__ uint32_t wave_max_scan_u32(uint32_t x)
{
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true));
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true));
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true));
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true));
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
	x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
	return x;
}

/* lane `src`'s value of v (ds_bpermute; every lane active) */
__device__ __forceinline__ uint32_t lane_pull(uint32_t v, uint32_t src)
{
	return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

/* bytes [0, n) of a little-endian word, n clamped to [0, 4] */
__device__ __forceinline__ uint32_t keep_below(int n)
{
	const int c = n < 0 ? 0 : n > 4 ? 4 : n;

	return c >= 4 ? ~0u : ~(~0u << (8 * c));
}

/* 16-byte load through a global (address space 1) pointer: an address
 * rebuilt from integers would otherwise become a flat load, which also counts
 * on lgkmcnt, so every LDS / bpermute wait after it would wait for the load */
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

__device__ __forceinline__ uint4 ld_g16(uint64_t addr)
{
	const u32x4 v = *(g_u32x4 *)(uintptr_t)addr;

	return make_uint4(v.x, v.y, v.z, v.w);
}

/* sum of bytes [lead, re) of the 64-byte unit at addr (16-byte aligned), as
 * 16-bit halves (v_dot2), 0 <= lead < re <= 64. Only the 16-byte chunks
 * holding bytes below re are read, so nothing past the aligned 16 bytes
 * holding the frame's last byte is touched. */
__device__ __forceinline__ uint32_t unit_sum_masked(uint64_t addr, int lead, int re)
{
	uint32_t acc = 0u;

#pragma unroll
	for (int k = 0; k < 4; ++k) {
		uint4 q = make_uint4(0u, 0u, 0u, 0u);

		if (16 * k < re)
			q = ld_g16(addr + 16u * k);
		const uint32_t w[4] = { q.x, q.y, q.z, q.w };

#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const int o = 16 * k + 4 * j;

			acc = tail_dot2(w[j] & keep_below(re - o) & ~keep_below(lead - o), acc);
		}
	}
	return acc;
}

/* Bytes [0, re) of the 64-byte unit at addr, 1 <= re <= 64, as 16-bit
 * halves: the words below re / 4 kept by a compare each, the one holding
 * the last byte masked, its dword loaded first, beside the chunk loads (a
 * cache hit: its chunk is loaded too), not behind their sums. A third of
 * unit_sum_masked's instructions. */
__device__ __forceinline__ uint32_t unit_sum_end(uint64_t addr, uint32_t re)
{
	const uint32_t nw = re >> 2, pb = re & 3u;
	/* the partial word (at a loaded word of the unit when there is none) */
	const uint32_t pwv = *(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)
			     (addr + 4u * (pb ? nw : 0u));
	uint4 q[4];

#pragma unroll
	for (int k = 0; k < 4; ++k) {
		q[k] = make_uint4(0u, 0u, 0u, 0u);
		if (16u * k < re)
			q[k] = ld_g16(addr + 16u * k);
	}
	uint32_t acc = tail_dot2(pb ? pwv & ((1u << (8u * pb)) - 1u) : 0u, 0u);

#pragma unroll
	for (int k = 0; k < 4; ++k) {
		acc = tail_dot2(4 * k + 0 < (int)nw ? q[k].x : 0u, acc);
		acc = tail_dot2(4 * k + 1 < (int)nw ? q[k].y : 0u, acc);
		acc = tail_dot2(4 * k + 2 < (int)nw ? q[k].z : 0u, acc);
		acc = tail_dot2(4 * k + 3 < (int)nw ? q[k].w : 0u, acc);
	}
	return acc;
}

template <bool XP = true>
__device__ __forceinline__ uint32_t seg_tail_sums4(uint64_t m, const uint8_t *g, const L4Pend &pd,
						uint32_t *marks = nullptr)
{
	const uint32_t lane = __lane_id();
	const bool mine = ((m >> lane) & 1ull) && pd.b > pd.a;
	const uint32_t c0 = pd.a & ~15u;
	const uint32_t lead = pd.a & 15u;
	const uint32_t nu = mine ? ((pd.b - 1u - c0) >> 6) + 1u : 0u;   /* 64-byte units */
	const bool own_first = mine && lead != 0u && nu >= 2u;
	const uint32_t f0 = own_first ? 1u : 0u;                        /* first shared unit */
	const uint32_t ni = mine ? nu - 1u - f0 : 0u;                   /* shared units */
	const uint64_t gb = (uint64_t)(uintptr_t)g + c0;
	uint32_t own = 0u;

	/* the lane's own units: last (masked to b, and to a when it is the
	 * first), then the first when it carries a lead. XP with no lead in
	 * the wave (C3: a = 64): the last units in the line shape as well, 16
	 * a load instruction, four lanes a unit (the units ranked by lane
	 * through the wave's LDS scratch) */
	const bool xp_own = XP && marks && !__ballot(mine && lead != 0u);   /* uniform */

	if (xp_own) {
		const uint64_t mm = __ballot(mine);
		const uint32_t nown = (uint32_t)__builtin_popcountll(mm);
		const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
								__builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
		const uint32_t lu = mine ? nu - 1u : 0u;
		const uint64_t ua = gb + 64ull * lu;
		const uint32_t re = mine ? pd.b - c0 - 64u * lu : 0u;   /* 1..64 */
		const uint32_t ua_lo = (uint32_t)ua, ua_hi = (uint32_t)(ua >> 32);
		volatile __attribute__((address_space(3))) uint32_t *mk =
			(volatile __attribute__((address_space(3))) uint32_t *)marks;
		uint32_t t = 0u;

		if (mine)
			mk[rank] = lane;
		__builtin_amdgcn_wave_barrier();
		for (uint32_t k = 0; 16u * k < nown; ++k) {                 /* uniform, <= 4 */
			const uint32_t idx = 16u * k + (lane >> 2);
			const uint32_t src = idx < nown ? mk[idx] : 0u;
			/* pulls with every lane active: a lane outside the ranks
			 * may hold a unit another lane reads */
			const uint32_t rp = lane_pull(re, src);
			const uint32_t rs = idx < nown ? rp : 0u;
			const uint64_t as = ((uint64_t)lane_pull(ua_hi, src) << 32) | lane_pull(ua_lo, src);
			const uint32_t o = 16u * (lane & 3u);
			uint4 x = make_uint4(0u, 0u, 0u, 0u);

			if (o < rs)
				x = ld_g16(as + o);
			uint32_t c = tail_dot2(x.x & keep_below((int)rs - (int)o), 0u);

			c = tail_dot2(x.y & keep_below((int)rs - (int)o - 4), c);
			c = tail_dot2(x.z & keep_below((int)rs - (int)o - 8), c);
			c = tail_dot2(x.w & keep_below((int)rs - (int)o - 12), c);
			c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xf, 0xf, false);
			c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xf, 0xf, false);
			t = (lane & 3u) == k ? c : t;
		}
		own = lane_pull(t, 4u * (rank & 15u) + (rank >> 4));
		own = mine ? own : 0u;
	} else if (mine) {
		const uint32_t lu = nu - 1u;

		if (!__ballot(mine && lead != 0u && lu == 0u))
			/* every last unit starting at its first byte (C3's early
			 * tails: a = 64, always) */
			own = unit_sum_end(gb + 64ull * lu, pd.b - c0 - 64u * lu);
		else
			own = unit_sum_masked(gb + 64ull * lu, lu ? 0 : (int)lead,
					      (int)(pd.b - c0 - 64u * lu));
		if (own_first)
			own = oc_add(own, unit_sum_masked(gb, (int)lead, 64));
	}

	const uint32_t incl = wave_scan_u32(ni);
	const uint32_t first = incl - ni;                               /* first shared slot */
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
	/* shared slot s of this lane's frame starts at cb + 64 s */
	const uint64_t cb = gb + 64ull * f0 - 64ull * first;
	const uint32_t cb_lo = (uint32_t)cb, cb_hi = (uint32_t)(cb >> 32);
	uint32_t acc = 0u;

	/* base address of the owner of slot min(base + lane, total - 1): binary
	 * search of incl over the lanes that can own a slot of the pass */
	auto owner = [&](uint32_t base) __attribute__((always_inline)) -> uint64_t {
		const uint32_t slot = min(base + lane, total - 1u);
		if (marks) {
			/* with a wave's 64-dword LDS scratch: every frame with a
			 * slot in the pass marks the lane of its first one (the
			 * frame running into the pass marks lane 0) with its own
			 * lane + 1, and a prefix max spreads the marks over the
			 * frame's lanes (one LDS round trip instead of the
			 * search's dependent bpermutes; LDS operations of a wave
			 * complete in order) */
			const bool in = ni && incl > base && first < base + 64u;
			/* volatile: lanes read what other lanes wrote, which the
			 * compiler's per-thread view would forward or drop */
			volatile __attribute__((address_space(3))) uint32_t *mk =
				(volatile __attribute__((address_space(3))) uint32_t *)marks;

			mk[lane] = 0u;
			__builtin_amdgcn_wave_barrier();
			if (in)
				mk[first > base ? first - base : 0u] = lane + 1u;
			__builtin_amdgcn_wave_barrier();
			const uint32_t o = wave_max_scan_u32(mk[lane]) - 1u;

			return (((uint64_t)lane_pull(cb_hi, o) << 32) | lane_pull(cb_lo, o)) +
			       64ull * slot;
		}
		const uint64_t past = __ballot(incl > base);
		const uint64_t beyond = __ballot(incl > base + 63u);
		const uint32_t lo = past ? (uint32_t)__builtin_ctzll(past) : 63u;
		const uint32_t hi = beyond ? (uint32_t)__builtin_ctzll(beyond) : 63u;
		const uint32_t span = hi > lo ? hi - lo : 0u;
		int p = -1;

		for (uint32_t step = span ? 1u << (31 - __builtin_clz(span)) : 0u; step;
		     step >>= 1) {                                         /* uniform */
			const uint32_t cand = (uint32_t)(p + (int)step);
			const uint32_t src = lo + cand < 64u ? lo + cand : 63u;
			const uint32_t v = lane_pull(incl, src);

			if (cand <= span && v <= slot)
				p = (int)cand;
		}
		const uint32_t o = lo + (uint32_t)(p + 1);

		return (((uint64_t)lane_pull(cb_hi, o) << 32) | lane_pull(cb_lo, o)) + 64ull * slot;
	};
	/* a pass's sum: each lane's unit, then every frame's share of the pass
	 * from the pass prefix sum (its slots of the pass are lanes [fl, ll]) */
	auto consume = [&](const uint4 (&q)[4], uint32_t base) __attribute__((always_inline)) {
		uint32_t s = 0u;

		if constexpr (XP) {
			/* each instruction's chunk sums, added over the unit's quad
			 * of lanes; lane 4j + m keeps unit 16m + j's, which lane
			 * 16m + j then takes */
			uint32_t t = 0u;

#pragma unroll
			for (int k = 0; k < 4; ++k) {
				uint32_t c = tail_dot2(q[k].x, 0u);

				c = tail_dot2(q[k].y, c);
				c = tail_dot2(q[k].z, c);
				c = tail_dot2(q[k].w, c);
				c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0xB1, 0xf, 0xf, false);
				c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x4E, 0xf, 0xf, false);
				t = (lane & 3u) == (uint32_t)k ? c : t;
			}
			s = lane_pull(t, 4u * (lane & 15u) + (lane >> 4));
		} else {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				s = tail_dot2(q[k].x, s);
				s = tail_dot2(q[k].y, s);
				s = tail_dot2(q[k].z, s);
				s = tail_dot2(q[k].w, s);
			}
		}
		const uint32_t ps = wave_scan_u32(base + lane < total ? oc_fold(s) : 0u);
		const bool in = ni && incl > base && first < base + 64u;
		const uint32_t fl = in && first > base ? first - base : 0u;
		const uint32_t ll = in ? (incl - 1u < base + 63u ? incl - 1u - base : 63u) : 0u;
		const uint32_t hv = lane_pull(ps, ll);
		const uint32_t lv = lane_pull(ps, fl ? fl - 1u : 0u);

		acc += in ? hv - (fl ? lv : 0u) : 0u;
	};
	/* line-shaped loads: instruction k reads the 16 units 16k .. 16k + 15 of
	 * the pass, four lanes a unit (16 bytes each), so that its 1 KiB covers
	 * whole 128-byte lines of a frame instead of a quarter of 32 lines, with
	 * the nontemporal hint: the tail bytes are read once, and the L2 then
	 * keeps the lines that are read twice (a window's line, a frame's last
	 * line shared with the next frame's window; C3 92.7 -> 87.6 us). XP;
	 * otherwise a lane reads its own unit: fewer registers */
	auto load = [&](uint4 (&q)[4], uint64_t a) __attribute__((always_inline)) {
		if constexpr (XP) {
			const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);

#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const uint32_t src = 16u * k + (lane >> 2);

				typedef unsigned int nt_v4 __attribute__((ext_vector_type(4)));
				const uint64_t ak = (((uint64_t)lane_pull(ahi, src) << 32) | lane_pull(alo, src)) +
						    16u * (lane & 3u);
				const nt_v4 v = __builtin_nontemporal_load(
					(const __attribute__((address_space(1))) nt_v4 *)(uintptr_t)ak);

				q[k] = make_uint4(v.x, v.y, v.z, v.w);
			}
		} else {
#pragma unroll
			for (int k = 0; k < 4; ++k)
				q[k] = ld_g16(a + 16u * k);
		}
	};
	uint64_t addr = total ? owner(0u) : 0ull;
	uint4 qa[4], qb[4];

	/* two passes in flight (8 KiB per wave): pass p + 2's loads are issued
	 * as soon as pass p is summed, and each pass's owners are found while
	 * the loads before it are in flight */
	if (total) {                                                   /* uniform */
		load(qa, addr);
		if (64u < total) {
			addr = owner(64u);
			load(qb, addr);
			if (128u < total)
				addr = owner(128u);
		}
	}
	for (uint32_t base = 0; base < total; base += 128u) {           /* uniform */
		consume(qa, base);
		if (base + 128u < total) {
			load(qa, addr);
			if (base + 192u < total)
				addr = owner(base + 192u);
		}
		if (base + 64u < total) {
			consume(qb, base + 64u);
			if (base + 192u < total) {
				load(qb, addr);
				if (base + 256u < total)
					addr = owner(base + 256u);
			}
		}
	}
	return mine ? oc_fold(oc_add(oc_fold(acc), oc_fold(own))) : 0u;
}

/* ---- register fast path: plain 64-byte Eth/IPv4/UDP|TCP frames ----------
 * Frames whose generic parse takes the straight path (no SNAP / VLAN, IPv4
 * IHL 5, UDP length >= 8 or TCP header >= 20 B) are parsed from the 16
 * registers holding the frame with compile-time offsets (l3 = 14, l4 = 34).
 * A wave takes it only when all its live lanes qualify (ballot); results are
 * bit-identical to parse_common() for those frames. */
template <int K>
__device__ __forceinline__ uint32_t fw(const uint32_t (&f)[16])
{
	/* little-endian u32 of frame bytes [K, K + 4), K constant */
	if constexpr ((K & 3) == 0)
		return f[K >> 2];
	else
		return __builtin_amdgcn_alignbyte(f[(K >> 2) + 1], f[K >> 2], K & 3);
}

__device__ __forceinline__ uint32_t swap16(uint32_t x)
{
	return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

__device__ __forceinline__ bool plain_v4(const uint32_t (&f)[16])
{
	const uint32_t w3 = f[3];
	const uint32_t tot_len = swap16(f[4] & 0xffffu);
	const uint32_t proto = f[5] >> 24;

	if ((w3 & 0x00ffffffu) != 0x00450008u)      /* ethtype 0x0800, ver_ihl 0x45 */
		return false;
	if (tot_len > 64u - 14u)
		return false;
	if (proto == 0x11u)
		return swap16(f[9] >> 16) >= 8u;         /* udp length */
	if (proto == 0x06u)
		return ((f[11] >> 20) & 0xfu) >= 5u;     /* tcp data offset */
	return false;
}

__device__ __forceinline__ int parse_fast(Prs &p, const uint32_t (&f)[16], uint64_t opt)
{
	const uint32_t len = 64u;
	uint64_t inf = IF(IFL_L2) | IF(IFL_ETH) | IF(IFL_L3) | IF(IFL_IPV4) | IF(IFL_L4);
	uint32_t fl = 0u;

	p.l2 = 0u;
	p.l3 = 14u;
	if (f[0] & 0x1u)
		inf |= IF(IFL_ETH_MCAST);
	if (f[0] == 0xffffffffu && (f[1] & 0xffffu) == 0xffffu)
		inf |= IF(IFL_ETH_BCAST);
	if (opt & ODPG_PKTIN_IPV4_CHKSUM) {
		uint32_t s = oc_add(f[3] & 0xffff0000u, f[4]);

		s = oc_add(s, f[5]);
		s = oc_add(s, f[6]);
		s = oc_add(s, f[7]);
		s = oc_add(s, f[8] & 0xffffu);
		inf |= IF(IFL_L3_CHKSUM_DONE);
		if (oc_fold(s) != 0xffffu) {
			/* ip_err: no l4 offset, ip_proto 0 -> l4 flag cleared */
			p.inf = inf & ~IF(IFL_L4);
			p.fl = FB(FL_IP_ERR) | FB(FL_L3_CHKSUM_ERR);
			p.l4 = 0xffffu;
			return 1;
		}
	}
	const bool frag = (swap16(f[5] & 0xffffu) & 0x3fffu) != 0u;
	const uint32_t dst_be = __builtin_bswap32(fw<30>(f));

	if (frag)
		inf |= IF(IFL_IPFRAG);
	if (dst_be == 0xffffffffu)
		inf |= IF(IFL_IP_BCAST);
	if ((dst_be >> 28) == 0xeu)
		inf |= IF(IFL_IP_MCAST);
	p.l4 = 34u;
	uint32_t l4sum = 0u;

	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM))
		l4sum = oc_add(oc_add(f[6] & 0xffff0000u, f[7]), f[8] & 0xffffu);
	bool do_sum = false;

	if ((f[5] >> 24) == 0x11u) {                 /* parse_udp */
		const uint32_t u1 = fw<38>(f);
		const uint32_t ulen_raw = u1 & 0xffffu, csum_raw = u1 >> 16;
		const uint32_t udplen = swap16(ulen_raw);

		inf |= IF(IFL_UDP);
		if ((opt & ODPG_PKTIN_UDP_CHKSUM) && !frag) {
			if (csum_raw == 0u) {
				inf |= IF(IFL_L4_CHKSUM_DONE) | IF(IFL_UDP_CHKSUM_ZERO);
			} else {
				l4sum = oc_add(oc_add(l4sum, ulen_raw), 0x11u << 8);
				do_sum = true;
			}
		}
		if (swap16(f[9] & 0xffffu) == 4500u && udplen > 4u && fw<42>(f) != 0u)
			inf |= IF(IFL_IPSEC) | IF(IFL_IPSEC_UDP);
		if (do_sum) {
			uint32_t s = oc_add(l4sum, f[8] & 0xffff0000u);

#pragma unroll
			for (int k = 9; k < 16; ++k)
				s = oc_add(s, f[k]);
			inf |= IF(IFL_L4_CHKSUM_DONE);
			if (oc_fold(s) != 0xffffu)
				fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_UDP_ERR);
		}
	} else {                                     /* parse_tcp */
		inf |= IF(IFL_TCP);
		if ((opt & ODPG_PKTIN_TCP_CHKSUM) && !frag) {
			uint32_t tl = (len - 34u) & 0xffffu;
			uint32_t s = oc_add(oc_add(l4sum, swap16(tl)), 0x06u << 8);

			s = oc_add(s, f[8] & 0xffff0000u);
#pragma unroll
			for (int k = 9; k < 16; ++k)
				s = oc_add(s, f[k]);
			inf |= IF(IFL_L4_CHKSUM_DONE);
			if (oc_fold(s) != 0xffffu)
				fl |= FB(FL_L4_CHKSUM_ERR) | FB(FL_TCP_ERR);
		}
	}
	p.inf = inf;
	p.fl = fl;
	return fl ? 1 : 0;
}

#endif /* ODPG_PKT_PARSE_H_ */
