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

/* mask of the first `n` bytes (0..4) of a little-endian word */
__device__ __forceinline__ uint32_t byte_mask(int n)
{
	n = n < 0 ? 0 : n > 4 ? 4 : n;
	return (uint32_t)((1ull << (8 * n)) - 1ull);
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

__device__ __forceinline__ uint32_t tail_share(const uint8_t *gp, uint32_t a, uint32_t b,
					       uint32_t lane)
{
	const uint32_t c0 = a & ~15u;
	const uint32_t last = (b - 1u - c0) >> 4;          /* uniform */
	const int rem = (int)(((b - 1u) & 15u) + 1u);       /* bytes of the last chunk */
	const uint32_t e0 = byte_mask(rem), e1 = byte_mask(rem - 4), e2 = byte_mask(rem - 8),
		       e3 = byte_mask(rem - 12);
	const int lead = (int)(a & 15u);                    /* bytes to drop at the start */
	const uint32_t s0 = ~byte_mask(lead), s1 = ~byte_mask(lead - 4),
		       s2 = ~byte_mask(lead - 8), s3 = ~byte_mask(lead - 12);
	uint32_t acc = 0u;

	for (uint32_t base = 0; base <= last; base += 64u) {   /* uniform: 1-2 passes for IMIX */
		const uint32_t idx = base + lane;

		if (idx <= last) {
			const uint4 q = *(const uint4 *)(gp + c0 + 16u * idx);
			const bool end = idx == last, start = idx == 0u;
			const uint32_t w0 = q.x & (end ? e0 : ~0u) & (start ? s0 : ~0u);
			const uint32_t w1 = q.y & (end ? e1 : ~0u) & (start ? s1 : ~0u);
			const uint32_t w2 = q.z & (end ? e2 : ~0u) & (start ? s2 : ~0u);
			const uint32_t w3 = q.w & (end ? e3 : ~0u) & (start ? s3 : ~0u);

			/* sums of the 16-bit halves (v_dot2_u32_u16): the same value
			 * mod 0xffff as the 32-bit word sum; at most 8 x 0xffff per
			 * pass, so no carry out below 8 MiB tails */
			acc = tail_dot2(w0, acc);
			acc = tail_dot2(w1, acc);
			acc = tail_dot2(w2, acc);
			acc = tail_dot2(w3, acc);
		}
	}
	return oc_fold(acc);
}

#ifndef COOP_BATCH
#define COOP_BATCH 4
#endif
/* Wave-cooperative sums of the frame tails [a, b) of the lanes in `m`: the
 * whole wave reads one frame's tail with coalesced 16-byte loads (1 KiB per
 * wave instruction), COOP_BATCH pairs of frames at a time so their loads
 * overlap. Each lane folds its share to 16 bits; two frames travel packed in
 * one lane reduction (64 x 0xffff < 2^22 per half). Lane j receives its own
 * tail sum. */
__device__ __forceinline__ uint32_t coop_tail_sums(uint64_t m, const uint8_t *g, const L4Pend &pd)
{
	const uint32_t lane = __lane_id();
	const uint64_t gv = (uint64_t)(uintptr_t)g;
	uint32_t mine = 0u;

#ifdef ODPG_EXP_NOTAIL      /* experiment builds only: cost without the tail reads */
	return 0u;
#endif
	while (m) {
		int jj[2 * COOP_BATCH];
		uint32_t sh[2 * COOP_BATCH];

#pragma unroll
		for (int k = 0; k < 2 * COOP_BATCH; ++k) {
			jj[k] = m ? __builtin_ctzll(m) : -1;
			m &= m - 1ull;
		}
#pragma unroll
		for (int k = 0; k < 2 * COOP_BATCH; ++k) {
			sh[k] = 0u;
			if (jj[k] >= 0) {
				const uint32_t glo = __builtin_amdgcn_readlane((int)(uint32_t)gv, jj[k]);
				const uint32_t ghi = __builtin_amdgcn_readlane((int)(uint32_t)(gv >> 32), jj[k]);
				const uint8_t *gp = (const uint8_t *)(uintptr_t)(((uint64_t)ghi << 32) | glo);
				const uint32_t a = __builtin_amdgcn_readlane((int)pd.a, jj[k]);
				const uint32_t b = __builtin_amdgcn_readlane((int)pd.b, jj[k]);

				sh[k] = tail_share(gp, a, b, lane);
			}
		}
#pragma unroll
		for (int k = 0; k < COOP_BATCH; ++k) {
			if (jj[2 * k] >= 0) {
				const uint32_t t0 = wave_sum_u32(sh[2 * k]);
				const uint32_t t1 = jj[2 * k + 1] >= 0 ? wave_sum_u32(sh[2 * k + 1]) : 0u;

				if (lane == (uint32_t)jj[2 * k])
					mine = oc_fold(t0);
				if (lane == (uint32_t)jj[2 * k + 1])
					mine = oc_fold(t1);
			}
		}
	}
	return mine;
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

/* Tail sums of the lanes in `m` as one balanced segmented reduction: the
 * 16-byte chunks of every pending tail [a, b) (chunk-aligned at a & ~15 of
 * the lane's frame g) are numbered across the wave in lane order (prefix sum
 * of the per-frame chunk counts) and spread over the 64 lanes, 64 chunks per
 * pass: a pass loads 1 KiB of tails with every lane busy, whatever the mix
 * of frame lengths. Each lane masks its chunk to [a, b), sums its 16-bit
 * halves (v_dot2) and folds; one wave prefix sum per pass then gives every
 * frame's share of the pass as a difference of two lanes. Lane j receives
 * its own tail sum (the same value coop_tail_sums returns: the one's-
 * complement residue and zero-ness of the exact sum are kept). */
#ifndef SEG_BATCH
#define SEG_BATCH 4
#endif
__device__ __forceinline__ uint32_t seg_tail_sums(uint64_t m, const uint8_t *g, const L4Pend &pd)
{
#ifdef ODPG_EXP_NOTAIL      /* experiment builds only: cost without the tail reads */
	return 0u;
#endif
	const uint32_t lane = __lane_id();
	const uint64_t gv = (uint64_t)(uintptr_t)g;
	const bool mine = ((m >> lane) & 1ull) && pd.b > pd.a;
	const uint32_t c0 = pd.a & ~15u;
	const uint32_t n = mine ? ((pd.b - 1u - c0) >> 4) + 1u : 0u;   /* chunks */
	const uint32_t incl = wave_scan_u32(n);
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
	uint32_t acc = 0u;

	/* SEG_BATCH passes at a time: their loads are all issued before the
	 * first is summed, so a wave keeps several KiB of tails in flight */
	for (uint32_t b0 = 0; b0 < total; b0 += 64u * SEG_BATCH) {   /* uniform */
		uint4 q[SEG_BATCH];
		uint32_t lead[SEG_BATCH], rem[SEG_BATCH];
		uint64_t pass_frames[SEG_BATCH];

#pragma unroll
		for (int k = 0; k < SEG_BATCH; ++k) {
			const uint32_t base = b0 + 64u * (uint32_t)k;
			const uint32_t slot = base + lane;
			const uint64_t in_pass = base < total ?
				__ballot(n && incl > base && incl - n < base + 64u) : 0ull;
			uint32_t own = 64u, first = 0u, glo = 0u, ghi = 0u, oa = 0u, ob = 0u, on = 0u;

			pass_frames[k] = in_pass;
			/* the frame owning this lane's chunk, and its fields */
			for (uint64_t f = in_pass; f; f &= f - 1ull) {
				const int j = __builtin_ctzll(f);
				const uint32_t ij = (uint32_t)__builtin_amdgcn_readlane((int)incl, j);
				const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)n, j);
				const bool hit = slot >= ij - nj && slot < ij;

				own = hit ? (uint32_t)j : own;
				first = hit ? ij - nj : first;
				on = hit ? nj : on;
				glo = hit ? (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gv, j) : glo;
				ghi = hit ? (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(gv >> 32), j) : ghi;
				oa = hit ? (uint32_t)__builtin_amdgcn_readlane((int)pd.a, j) : oa;
				ob = hit ? (uint32_t)__builtin_amdgcn_readlane((int)pd.b, j) : ob;
			}
			const uint32_t idx = slot - first;

			q[k] = make_uint4(0u, 0u, 0u, 0u);
			lead[k] = idx == 0u ? (oa & 15u) : 0u;
			rem[k] = own < 64u ? (idx + 1u == on ? ((ob - 1u) & 15u) + 1u : 16u) : 0u;
			if (own < 64u) {
				const uint8_t *gp = (const uint8_t *)(uintptr_t)(((uint64_t)ghi << 32) | glo);

				q[k] = *(const uint4 *)(gp + (oa & ~15u) + 16u * idx);
			}
		}
#pragma unroll
		for (int k = 0; k < SEG_BATCH; ++k) {
			if (!pass_frames[k])
				continue;
			const uint32_t base = b0 + 64u * (uint32_t)k;
			const int le = (int)lead[k], re = (int)rem[k];
			uint32_t acc4 = 0u;

			acc4 = tail_dot2(q[k].x & byte_mask(re) & ~byte_mask(le), acc4);
			acc4 = tail_dot2(q[k].y & byte_mask(re - 4) & ~byte_mask(le - 4), acc4);
			acc4 = tail_dot2(q[k].z & byte_mask(re - 8) & ~byte_mask(le - 8), acc4);
			acc4 = tail_dot2(q[k].w & byte_mask(re - 12) & ~byte_mask(le - 12), acc4);
			/* frames own contiguous lanes: a frame's share of the pass is
			 * the prefix sum at its last lane minus the one before its first */
			const uint32_t ps = wave_scan_u32(oc_fold(acc4));

			for (uint64_t f = pass_frames[k]; f; f &= f - 1ull) {
				const int j = __builtin_ctzll(f);
				const uint32_t ij = (uint32_t)__builtin_amdgcn_readlane((int)incl, j);
				const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)n, j);
				const uint32_t lo = ij - nj > base ? ij - nj - base : 0u;
				const uint32_t hi = (ij < base + 64u ? ij : base + 64u) - base - 1u;
				const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)ps, (int)hi) -
						    (lo ? (uint32_t)__builtin_amdgcn_readlane((int)ps, (int)lo - 1) : 0u);

				acc += lane == (uint32_t)j ? sh : 0u;
			}
		}
	}
	return mine ? oc_fold(acc) : 0u;
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

/* seg_tail_sums with the per-pass bookkeeping done lane-parallel (round 2,
 * second form): the owner of a lane's chunk is found by a binary search of
 * the inclusive chunk counts over the lanes that can own a chunk of this
 * pass (ds_bpermute per step: log2 of that lane range, 2-4 steps for IMIX),
 * the owner's chunk base address and bounds are pulled in four more
 * bpermutes, and each frame pulls its share of the pass from two lanes of
 * the pass's prefix sum. No per-frame loops: the pass costs the same
 * whatever number of frames it touches. Same result as seg_tail_sums. */
__device__ __forceinline__ uint32_t seg_tail_sums2(uint64_t m, const uint8_t *g, const L4Pend &pd)
{
#ifdef ODPG_EXP_NOTAIL
	return 0u;
#endif
	const uint32_t lane = __lane_id();
	const bool mine = ((m >> lane) & 1ull) && pd.b > pd.a;
	const uint32_t c0 = pd.a & ~15u;
	const uint32_t n = mine ? ((pd.b - 1u - c0) >> 4) + 1u : 0u;   /* chunks */
	const uint32_t incl = wave_scan_u32(n);
	const uint32_t first = incl - n;                                /* first slot */
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
	/* the address of slot s of this lane's frame is cb + 16 s */
	const uint64_t cb = (uint64_t)(uintptr_t)g + c0 - 16ull * first;
	const uint32_t cb_lo = (uint32_t)cb, cb_hi = (uint32_t)(cb >> 32);
	const uint32_t pk = (incl & 0xffffffu) | ((pd.a & 15u) << 24) | (((pd.b - 1u) & 15u) << 28);
	uint32_t acc = 0u;

	for (uint32_t b0 = 0; b0 < total; b0 += 64u * SEG_BATCH) {   /* uniform */
		uint4 q[SEG_BATCH];
		uint32_t lead[SEG_BATCH], rem[SEG_BATCH];

#pragma unroll
		for (int k = 0; k < SEG_BATCH; ++k) {
			const uint32_t base = b0 + 64u * (uint32_t)k;
			const uint32_t slot = base + lane;
			const bool valid = slot < total;
			/* owners of this pass's chunks lie in lanes [lo, hi] (uniform) */
			const uint64_t past = __ballot(incl > base);
			const uint64_t beyond = __ballot(incl > base + 63u);
			const uint32_t lo = past ? (uint32_t)__builtin_ctzll(past) : 63u;
			const uint32_t hi = beyond ? (uint32_t)__builtin_ctzll(beyond) : 63u;
			const uint32_t span = hi > lo ? hi - lo : 0u;
			int p = -1;        /* lanes lo .. lo + p hold incl <= slot */

			for (uint32_t step = span ? 1u << (31 - __builtin_clz(span)) : 0u; step;
			     step >>= 1) {                                  /* uniform */
				const uint32_t cand = (uint32_t)(p + (int)step);
				const uint32_t src = lo + cand < 64u ? lo + cand : 63u;
				const uint32_t v = lane_pull(incl, src);

				if (cand <= span && v <= slot)
					p = (int)cand;
			}
			const uint32_t own = lo + (uint32_t)(p + 1);
			const uint32_t olo = lane_pull(cb_lo, own), ohi = lane_pull(cb_hi, own);
			const uint32_t opk = lane_pull(pk, own), ofirst = lane_pull(first, own);

			q[k] = make_uint4(0u, 0u, 0u, 0u);
			lead[k] = slot == ofirst ? (opk >> 24) & 15u : 0u;
			rem[k] = !valid ? 0u : slot + 1u == (opk & 0xffffffu) ? (opk >> 28) + 1u : 16u;
			if (valid)
				q[k] = *(const uint4 *)(uintptr_t)((((uint64_t)ohi << 32) | olo) +
								   16ull * slot);
		}
#pragma unroll
		for (int k = 0; k < SEG_BATCH; ++k) {
			const uint32_t base = b0 + 64u * (uint32_t)k;

			if (base >= total)                                  /* uniform */
				break;
			const int le = (int)lead[k], re = (int)rem[k];
			uint32_t acc4 = 0u;

			acc4 = tail_dot2(q[k].x & byte_mask(re) & ~byte_mask(le), acc4);
			acc4 = tail_dot2(q[k].y & byte_mask(re - 4) & ~byte_mask(le - 4), acc4);
			acc4 = tail_dot2(q[k].z & byte_mask(re - 8) & ~byte_mask(le - 8), acc4);
			acc4 = tail_dot2(q[k].w & byte_mask(re - 12) & ~byte_mask(le - 12), acc4);
			const uint32_t ps = wave_scan_u32(oc_fold(acc4));
			/* this lane's frame: its chunks of the pass are lanes [fl, ll] */
			const bool in = n && incl > base && first < base + 64u;
			const uint32_t fl = in && first > base ? first - base : 0u;
			const uint32_t ll = in ? (incl - 1u < base + 63u ? incl - 1u - base : 63u) : 0u;
			const uint32_t hv = lane_pull(ps, ll);
			const uint32_t lv = lane_pull(ps, fl ? fl - 1u : 0u);

			acc += in ? hv - (fl ? lv : 0u) : 0u;
		}
	}
	return mine ? oc_fold(acc) : 0u;
}

/* bytes [0, n) of a little-endian word, n clamped to [0, 4] */
__device__ __forceinline__ uint32_t keep_below(int n)
{
	const int c = n < 0 ? 0 : n > 4 ? 4 : n;

	return c >= 4 ? ~0u : ~(~0u << (8 * c));
}

/* seg_tail_sums2 over 64-byte units (third form, the default): a lane
 * loads and sums 64 contiguous bytes of one tail per pass (4 x 16 B), so the
 * per-pass bookkeeping — owner search, owner fields, the pass prefix sum
 * and the per-frame shares — is paid once per 64 bytes instead of once per
 * 16, and the next pass's owners are found while this pass's loads are in
 * flight. A unit's bytes outside [a, b) are masked per word. Same result as
 * seg_tail_sums. */
__device__ __forceinline__ uint32_t seg_tail_sums3(uint64_t m, const uint8_t *g, const L4Pend &pd)
{
#ifdef ODPG_EXP_NOTAIL
	return 0u;
#endif
	const uint32_t lane = __lane_id();
	const bool mine = ((m >> lane) & 1ull) && pd.b > pd.a;
	const uint32_t c0 = pd.a & ~15u;
	const uint32_t n = mine ? ((pd.b - 1u - c0) >> 6) + 1u : 0u;   /* 64-byte units */
	const uint32_t incl = wave_scan_u32(n);
	const uint32_t first = incl - n;                                /* first unit slot */
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
	/* unit slot s of this lane's frame starts at cb + 64 s */
	const uint64_t cb = (uint64_t)(uintptr_t)g + c0 - 64ull * first;
	const uint32_t cb_lo = (uint32_t)cb, cb_hi = (uint32_t)(cb >> 32);
	/* inclusive end slot | bytes to drop at the start | bytes of the last unit - 1 */
	const uint32_t pk = (incl & 0xfffffu) | ((pd.a & 15u) << 20) | (((pd.b - 1u - c0) & 63u) << 24);
	uint32_t acc = 0u;

	/* the owner of slot base + lane: a binary search of incl over the lanes
	 * that can own a unit of the pass, then its fields */
	auto owner = [&](uint32_t base, uint32_t &olo, uint32_t &ohi, uint32_t &opk,
			 uint32_t &ofirst) __attribute__((always_inline)) {
		const uint32_t slot = base + lane;
		const uint64_t past = __ballot(incl > base);
		const uint64_t beyond = __ballot(incl > base + 63u);
		const uint32_t lo = past ? (uint32_t)__builtin_ctzll(past) : 63u;
		const uint32_t hi = beyond ? (uint32_t)__builtin_ctzll(beyond) : 63u;
		const uint32_t span = hi > lo ? hi - lo : 0u;
		int p = -1;

		for (uint32_t step = span ? 1u << (31 - __builtin_clz(span)) : 0u; step;
		     step >>= 1) {                                     /* uniform */
			const uint32_t cand = (uint32_t)(p + (int)step);
			const uint32_t src = lo + cand < 64u ? lo + cand : 63u;
			const uint32_t v = lane_pull(incl, src);

			if (cand <= span && v <= slot)
				p = (int)cand;
		}
		const uint32_t own = lo + (uint32_t)(p + 1);

		olo = lane_pull(cb_lo, own);
		ohi = lane_pull(cb_hi, own);
		opk = lane_pull(pk, own);
		ofirst = lane_pull(first, own);
	};
	uint32_t olo, ohi, opk, ofirst;

	if (total)                                                     /* uniform */
		owner(0u, olo, ohi, opk, ofirst);
	for (uint32_t base = 0; base < total; base += 64u) {            /* uniform */
		const uint32_t slot = base + lane;
		const bool valid = slot < total;
		const int le = slot == ofirst ? (int)((opk >> 20) & 15u) : 0;
		const int re = !valid ? 0 : slot + 1u == (opk & 0xfffffu) ? (int)(opk >> 24) + 1 : 64;
		uint4 q[4];

#pragma unroll
		for (int k = 0; k < 4; ++k)
			q[k] = make_uint4(0u, 0u, 0u, 0u);
		if (valid) {
			const uint4 *src = (const uint4 *)(uintptr_t)((((uint64_t)ohi << 32) | olo) +
								     64ull * slot);
#pragma unroll
			for (int k = 0; k < 4; ++k)
				q[k] = src[k];
		}
		/* the next pass's owners while the loads are in flight */
		if (base + 64u < total)                                 /* uniform */
			owner(base + 64u, olo, ohi, opk, ofirst);
		uint32_t acc4 = 0u;

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint32_t w[4] = { q[k].x, q[k].y, q[k].z, q[k].w };

#pragma unroll
			for (int j = 0; j < 4; ++j) {
				const int o = 16 * k + 4 * j;
				uint32_t msk = keep_below(re - o);

				if (k == 0)
					msk &= ~keep_below(le - o);
				acc4 = tail_dot2(w[j] & msk, acc4);
			}
		}
		const uint32_t ps = wave_scan_u32(oc_fold(acc4));
		/* this lane's frame: its units of the pass are lanes [fl, ll] */
		const bool in = n && incl > base && first < base + 64u;
		const uint32_t fl = in && first > base ? first - base : 0u;
		const uint32_t ll = in ? (incl - 1u < base + 63u ? incl - 1u - base : 63u) : 0u;
		const uint32_t hv = lane_pull(ps, ll);
		const uint32_t lv = lane_pull(ps, fl ? fl - 1u : 0u);

		acc += in ? hv - (fl ? lv : 0u) : 0u;
	}
	return mine ? oc_fold(acc) : 0u;
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

/* unit_sum_masked over a unit already loaded (16-byte chunks at or past re
 * zero) */
__device__ __forceinline__ uint32_t unit_sum_regs(const uint4 (&q)[4], int lead, int re)
{
	uint32_t acc = 0u;

#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t w[4] = { q[k].x, q[k].y, q[k].z, q[k].w };

#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const int o = 16 * k + 4 * j;

			acc = tail_dot2(w[j] & keep_below(re - o) & ~keep_below(lead - o), acc);
		}
	}
	return acc;
}

/* Tail sums, fourth form (the default): each tail [a, b) is cut into 64-byte
 * units from c0 = a & ~15. The units that need byte masks — the frame's last
 * one, and its first one when a is not 16-aligned — are summed by the lane
 * itself, once per frame; every other unit is a whole 64 bytes inside the
 * tail, and those are spread over the wave as in seg_tail_sums3 but need no
 * masks, no per-unit bounds and only the owner's base address (two
 * bpermutes). All loads go through global pointers. Same result as
 * seg_tail_sums. */
/* One coalesced sweep over every byte of a wave's 64 frames (descriptor
 * batches, 64-byte window): frame f's 64-byte units [0, len) are numbered
 * across the wave frame after frame (a DPP prefix sum of the per-frame unit
 * counts) and spread over the lanes, 64 units per pass, so a frame's window,
 * its tail and the neighbouring frames' bytes are requested by neighbouring
 * lanes of the same or the next load instruction: each 128-byte line is
 * fetched once. A lane holding a frame's unit 0 writes it (zero past the
 * frame) into that frame's LDS row, the window the parse reads; every other
 * unit is masked to the frame and summed (v_dot2). Returns the lane's own
 * frame's sum of bytes [64, len) as a one's-complement partial (residue and
 * zero-ness kept). `rows` is the wave's first row, `rw` the row stride in
 * dwords. All lanes must be active. */
__device__ __forceinline__ uint32_t sweep_frames(const uint8_t *g, uint32_t len, uint32_t *rows,
						 uint32_t rw)
{
	const uint32_t lane = __lane_id();
	const uint32_t nu = len ? ((len - 1u) >> 6) + 1u : 0u;
	const uint32_t incl = wave_scan_u32(nu);
	const uint32_t first = incl - nu;
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
	/* unit slot s of this lane's frame starts at cb + 64 s */
	const uint64_t cb = (uint64_t)(uintptr_t)g - 64ull * first;
	const uint32_t cb_lo = (uint32_t)cb, cb_hi = (uint32_t)(cb >> 32);
	uint32_t acc = 0u;

	if (len == 0u) {                                  /* empty frame: zero window */
#pragma unroll
		for (int w = 0; w < 16; ++w)
			rows[lane * rw + w] = 0u;
	}
	for (uint32_t base = 0; base < total; base += 64u) {            /* uniform */
		const uint32_t slot = min(base + lane, total - 1u);
		const bool valid = base + lane < total;
		const uint64_t past = __ballot(incl > base);
		const uint64_t beyond = __ballot(incl > base + 63u);
		const uint32_t lo = past ? (uint32_t)__builtin_ctzll(past) : 63u;
		const uint32_t hi = beyond ? (uint32_t)__builtin_ctzll(beyond) : 63u;
		const uint32_t span = hi > lo ? hi - lo : 0u;
		int p = -1;

		for (uint32_t st = span ? 1u << (31 - __builtin_clz(span)) : 0u; st;
		     st >>= 1) {                                       /* uniform */
			const uint32_t cand = (uint32_t)(p + (int)st);
			const uint32_t src = lo + cand < 64u ? lo + cand : 63u;
			const uint32_t v = lane_pull(incl, src);

			if (cand <= span && v <= slot)
				p = (int)cand;
		}
		const uint32_t o = lo + (uint32_t)(p + 1);
		const uint64_t a = (((uint64_t)lane_pull(cb_hi, o) << 32) | lane_pull(cb_lo, o)) +
				   64ull * slot;
		/* pulled with every lane active: a bpermute under a partial exec
		 * mask reads inactive source lanes as 0 */
		const uint32_t ofirst = lane_pull(first, o), olen = lane_pull(len, o);
		const uint32_t u = slot - ofirst;
		const int rem = valid ? (int)(olen - 64u * u) : 0;     /* >= 1 */
		/* whole words below rem kept by a compare each; the one partial
		 * word (rem not a multiple of 4) is read again as a dword (a cache
		 * hit: its 16 bytes were just loaded) and masked */
		const uint32_t nw = rem > 0 ? (uint32_t)rem >> 2 : 0u;
		const uint32_t pb = (uint32_t)rem & 3u;
		uint32_t pv = 0u;
		uint32_t w[16];

		if (rem > 0 && pb && nw < 16u)
			pv = *(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)(a + 4u * nw) &
			     ((1u << (8u * pb)) - 1u);
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			uint4 q = make_uint4(0u, 0u, 0u, 0u);

			if (16 * j < rem)
				q = ld_g16(a + 16u * j);
			w[4 * j + 0] = 4 * j + 0 < (int)nw ? q.x : 0u;
			w[4 * j + 1] = 4 * j + 1 < (int)nw ? q.y : 0u;
			w[4 * j + 2] = 4 * j + 2 < (int)nw ? q.z : 0u;
			w[4 * j + 3] = 4 * j + 3 < (int)nw ? q.w : 0u;
		}
		uint32_t sum = 0u;

		if (valid && u == 0u) {
			uint32_t *r = rows + o * rw;

#pragma unroll
			for (int k = 0; k < 16; ++k)
				r[k] = w[k];
			if (pb && nw < 16u)
				r[nw] = pv;
		} else {
#pragma unroll
			for (int k = 0; k < 16; ++k)
				sum = tail_dot2(w[k], sum);
			sum = tail_dot2(pv, sum);
		}
		/* this lane's frame: its units of the pass are lanes [fl, ll] */
		const uint32_t ps = wave_scan_u32(oc_fold(sum));
		const bool in = nu && incl > base && first < base + 64u;
		const uint32_t fl = in && first > base ? first - base : 0u;
		const uint32_t ll = in ? (incl - 1u < base + 63u ? incl - 1u - base : 63u) : 0u;
		const uint32_t hv = lane_pull(ps, ll);
		const uint32_t lv = lane_pull(ps, fl ? fl - 1u : 0u);

		acc += in ? hv - (fl ? lv : 0u) : 0u;
	}
	/* the rows written by other lanes are read next by their own lanes */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	return oc_fold(acc);
}

#ifndef SEG4_PIPE
#define SEG4_PIPE 1
#endif
#ifndef SEG4_OWNEARLY       /* last units' loads issued before the passes' */
#define SEG4_OWNEARLY 0
#endif
#ifndef SEG4_TAILW          /* last units by whole-word compares (unit_sum_head): */
#define SEG4_TAILW 0        /* fewer VALU but a dependent reload; C3 +1.5 us */
#endif

/* sum of bytes [0, re) of the 64-byte unit at addr (16-byte aligned),
 * 1 <= re <= 64, as 16-bit halves: words below re / 4 by a compare each,
 * the word holding the last byte read again as a dword and masked (its 16
 * bytes were just loaded). unit_sum_masked's result for lead 0 at a third
 * of its instructions. */
__device__ __forceinline__ uint32_t unit_sum_head(uint64_t addr, uint32_t re)
{
	const uint32_t nw = re >> 2, pb = re & 3u;
	uint32_t acc = 0u;

#pragma unroll
	for (int k = 0; k < 4; ++k) {
		uint4 q = make_uint4(0u, 0u, 0u, 0u);

		if (16u * k < re)
			q = ld_g16(addr + 16u * k);
		acc = tail_dot2(4 * k + 0 < (int)nw ? q.x : 0u, acc);
		acc = tail_dot2(4 * k + 1 < (int)nw ? q.y : 0u, acc);
		acc = tail_dot2(4 * k + 2 < (int)nw ? q.z : 0u, acc);
		acc = tail_dot2(4 * k + 3 < (int)nw ? q.w : 0u, acc);
	}
	if (pb) {
		const uint32_t w = *(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)(addr + 4u * nw);

		acc = tail_dot2(w & ((1u << (8u * pb)) - 1u), acc);
	}
	return acc;
}
/* unit_sum_head with the partial word's dword load issued first, beside the
 * chunk loads (not behind their sums): bytes [0, re) of the 64-byte unit at
 * addr, 1 <= re <= 64; the words below re / 4 kept by a compare each, the
 * one holding the last byte (a cache hit: its chunk is loaded too) masked.
 * A third of unit_sum_masked's instructions. */
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

__device__ __forceinline__ uint32_t seg_tail_sums4(uint64_t m, const uint8_t *g, const L4Pend &pd,
						uint32_t *marks = nullptr)
{
#ifdef ODPG_EXP_NOTAIL
	return 0u;
#endif
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
	const bool own_late = SEG4_OWNEARLY && !__ballot(own_first);     /* uniform */
	uint4 oq[4] = {};
	int own_re = 0, own_lead = 0;

	/* the lane's own units: last (masked to b, and to a when it is the
	 * first), then the first when it carries a lead */
#ifdef SEG4_EXP_NOOWN       /* experiment builds only: cost of the own units */
	if (mine && pd.b == 12345u) {
#else
	if (mine) {
#endif
		const uint32_t lu = nu - 1u;

		/* SEG4_OWNEARLY without a first own unit anywhere: the last unit's
		 * loads now, its sum once the first passes' loads are issued */
		if (own_late) {
			own_re = (int)(pd.b - c0 - 64u * lu);
			own_lead = lu ? 0 : (int)lead;
#pragma unroll
			for (int k = 0; k < 4; ++k)
				if (16 * k < own_re)
					oq[k] = ld_g16(gb + 64ull * lu + 16u * k);
		} else
		/* every last unit starting at its first byte (C3's early tails
		 * always): whole words by a compare each, the partial one read
		 * again as a dword (a cache hit) */
		if (SEG4_TAILW && !__ballot(mine && lead != 0u && lu == 0u))
			own = unit_sum_head(gb + 64ull * lu, pd.b - c0 - 64u * lu);
		else if (!__ballot(mine && lead != 0u && lu == 0u))
			/* every last unit starts at its first byte (C3's early
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
#ifdef SEG4_EXP_NOOWNER     /* experiment builds only: cost of the owner search */
		return (((uint64_t)cb_hi << 32) | cb_lo) + 64ull * slot;
#endif
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

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			s = tail_dot2(q[k].x, s);
			s = tail_dot2(q[k].y, s);
			s = tail_dot2(q[k].z, s);
			s = tail_dot2(q[k].w, s);
		}
#ifdef SEG4_EXP_NOSCAN      /* experiment builds only: cost of the pass attribution */
		acc += s;
		return;
#endif
		const uint32_t ps = wave_scan_u32(base + lane < total ? oc_fold(s) : 0u);
		const bool in = ni && incl > base && first < base + 64u;
		const uint32_t fl = in && first > base ? first - base : 0u;
		const uint32_t ll = in ? (incl - 1u < base + 63u ? incl - 1u - base : 63u) : 0u;
		const uint32_t hv = lane_pull(ps, ll);
		const uint32_t lv = lane_pull(ps, fl ? fl - 1u : 0u);

		acc += in ? hv - (fl ? lv : 0u) : 0u;
	};
	auto load = [&](uint4 (&q)[4], uint64_t a) __attribute__((always_inline)) {
#pragma unroll
		for (int k = 0; k < 4; ++k)
			q[k] = ld_g16(a + 16u * k);
	};
	uint64_t addr = total ? owner(0u) : 0ull;
	uint4 qa[4], qb[4];

#if SEG4_PIPE
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
	if (own_late && mine)
		own = unit_sum_regs(oq, own_lead, own_re);
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
#else
	if (own_late && mine)
		own = unit_sum_regs(oq, own_lead, own_re);
	for (uint32_t base = 0; base < total; base += 64u) {            /* uniform */
		load(qa, addr);
		/* the next pass's owners while the loads are in flight */
		if (base + 64u < total)                                 /* uniform */
			addr = owner(base + 64u);
		consume(qa, base);
	}
	(void)qb;
#endif
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
