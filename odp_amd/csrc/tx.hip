/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Loop pktio transmit side on gfx950 (include/odpg_tx.h, SURVEY.md §8(f)
 * rank 3): per packet, loopback_fix_checksums() and get_dest_queue() of
 * loopback_send() (platform/linux-generic/pktio/loop.c:415-523), frames
 * rewritten in place.
 *
 * One lane per packet. The frame's first 64 bytes are staged in the lane's
 * LDS row for the optional parse; checksum ranges are summed from global
 * memory as frame-aligned little-endian dwords (end-around carry), which
 * keeps the reference's 64-bit chksum_partial residue mod 0xffff; the
 * reference pairs bytes relative to the L3 offset (chksum_partial's odd
 * offset swap, odp_chksum_internal.h:60-196), so an odd L3 offset swaps the
 * folded sum. CRC32c (SCTP insert, queue hash) is table driven from LDS.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>

#include "../../include/odpg_tx.h"
#include "odpg_internal.h"
#include "pkt_parse.h"

namespace {

constexpr uint32_t TX_BLOCK = 256;
constexpr uint32_t TX_W = 64;               /* LDS window per lane */
constexpr uint32_t TX_RW = TX_W / 4 + 1;    /* odd dword row stride */

struct TxArgs {
	uint8_t *frames;
	const odpg_desc_t *desc;
	uint32_t stride, num;
	const odpg_tx_meta_t *meta;
	uint64_t cfg, capa;
	uint32_t hash_proto, num_qs, index;
	uint32_t *out;
};

/* one dword of the frame at byte 4 * w (bytes past len read as zero) */
__device__ __forceinline__ uint32_t tx_word(const uint8_t *g, uint32_t len, uint32_t w)
{
	if (4u * w >= len)
		return 0u;
	uint32_t x;

	__builtin_memcpy(&x, g + 4u * w, 4);
	const uint32_t rem = len - 4u * w;

	return rem < 4u ? x & ((1u << (8u * rem)) - 1u) : x;
}

__device__ __forceinline__ uint32_t tx_u8(const uint8_t *g, uint32_t len, uint32_t p)
{
	return p < len ? g[p] : 0u;
}

/* mask of bytes [lo, hi) within dword w (frame positions) */
__device__ __forceinline__ uint32_t tx_bmask(uint32_t w, uint32_t lo, uint32_t hi)
{
	uint32_t m = 0u;

#pragma unroll
	for (uint32_t j = 0; j < 4; ++j) {
		const uint32_t p = 4u * w + j;

		m |= (p >= lo && p < hi) ? 0xffu << (8u * j) : 0u;
	}
	return m;
}

/* packet_sum_partial (odp_packet.c:1669-1692) of [off, off + n) with the
 * bytes of [z0, z1) taken as zero: 0 when the range leaves the frame;
 * otherwise the one's-complement residue, folded to 16 bits, of the bytes
 * paired relative to l3 */
__device__ uint32_t tx_sum(const uint8_t *g, uint32_t len, uint32_t l3, uint32_t off, uint32_t n,
			   uint32_t z0 = 0u, uint32_t z1 = 0u)
{
	if (n == 0u || off + n > len || off + n < off)
		return 0u;
	const uint32_t end = off + n, w0 = off >> 2, w1 = (end - 1u) >> 2;
	uint32_t s = 0u;

	for (uint32_t w = w0; w <= w1; ++w) {
		uint32_t x = tx_word(g, len, w);

		if (w == w0 || w == w1 || (z1 > z0 && 4u * w + 4u > z0 && 4u * w < z1))
			x &= tx_bmask(w, off, end) & ~tx_bmask(w, z0, z1);
		s = oc_add(s, x);
	}
	s = oc_fold(s);
	return (l3 & 1u) ? ((s & 0xffu) << 8) | (s >> 8) : s;
}

__device__ __forceinline__ uint32_t crc_tab(const uint32_t *tab, uint32_t crc, uint32_t b)
{
	return tab[(crc ^ b) & 0xffu] ^ (crc >> 8);
}

/* byte stores (frames may sit at any alignment); false when the range
 * leaves the frame (odp_packet_copy_from_mem fails) */
__device__ __forceinline__ bool tx_store(uint8_t *g, uint32_t len, uint32_t off, uint32_t v,
					 uint32_t n)
{
	if (off + n > len)
		return false;
	for (uint32_t j = 0; j < n; ++j)
		g[off + j] = (uint8_t)(v >> (8u * j));
	return true;
}

/* acc + w.lo * x.lo16 + w.hi * x.hi16 (one v_dot2_u32_u16) */
typedef unsigned short tx_us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t d2(uint32_t x, uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(tx_us2, x), __builtin_bit_cast(tx_us2, w),
				      acc, false);
}

/* end-around fold of a sum of < 2^15 16-bit words */
__device__ __forceinline__ uint32_t d2fold(uint32_t s)
{
	s = d2(s, 0x00010001u, 0u);
	return d2(s, 0x00010001u, 0u);
}

/* the generic path's result for a plain 64-byte frame (plain_v4(f)):
 * l3 = 14, l4 = 34, no overrides; dwords 6 (bytes 24..27, the IPv4 checksum)
 * and 10 (bytes 40..43, the UDP checksum / the TCP write at l4 + 6) are
 * stored back when changed */
__device__ __forceinline__ uint32_t tx_fast64(const TxArgs &A, const uint32_t *tab,
					      uint32_t (&f)[16], uint32_t *g)
{
	constexpr uint32_t W11 = 0x00010001u, W10 = 0x00000001u, W01 = 0x00010000u;
	const uint32_t proto = f[5] >> 24;
	const bool frag = (f[5] & 0xff3fu) != 0u;   /* be16(frag) & 0x3fff */
	const uint32_t l4p = frag ? 255u : proto;
	uint32_t res = 0u;
	bool w6 = false, w10 = false;

	if ((A.capa & ODPG_PKTOUT_IPV4_CHKSUM) && (A.cfg & ODPG_PKTOUT_IPV4_CHKSUM)) {
		/* bytes 14..33, the checksum field (24..25) as zero */
		uint32_t s = d2(f[3], W01, 0u);

		s = d2(f[4], W11, s);
		s = d2(f[5], W11, s);
		s = d2(f[6], W01, s);
		s = d2(f[7], W11, s);
		s = d2(f[8], W10, s);
		f[6] = (f[6] & 0xffff0000u) | (~d2fold(s) & 0xffffu);
		w6 = true;
		res |= ODPG_TX_OUT_IPV4;
	}
	const bool udp = l4p == 17u && (A.capa & ODPG_PKTOUT_UDP_CHKSUM) &&
			 (A.cfg & ODPG_PKTOUT_UDP_CHKSUM);
	const bool tcp = l4p == 6u && (A.capa & ODPG_PKTOUT_TCP_CHKSUM) &&
			 (A.cfg & ODPG_PKTOUT_TCP_CHKSUM);

	if (udp || tcp) {
		/* addresses (26..33) + proto << 8 + (UDP: the length field again;
		 * TCP: be16(30)) + bytes 34..63 with 40..41 as zero */
		uint32_t s = udp ? 0x1100u : 0x0600u + 0x1e00u;

		s = d2(f[6], W01, s);
		s = d2(f[7], W11, s);
		s = d2(f[8], W11, s);
		s = d2(f[9], udp ? 0x00020001u : W11, s);
		s = d2(f[10], W01, s);
#pragma unroll
		for (int k = 11; k < 16; ++k)
			s = d2(f[k], W11, s);
		uint32_t c = ~d2fold(s) & 0xffffu;

		if (udp && c == 0u)
			c = 0xffffu;
		f[10] = (f[10] & 0xffff0000u) | c;
		w10 = true;
		res |= udp ? ODPG_TX_OUT_UDP : ODPG_TX_OUT_TCP;
	}
	if (g && w6)
		g[6] = f[6];
	if (g && w10)
		g[10] = f[10];

	/* get_dest_queue: ports (34..37), then the IPv4 addresses (26..33) */
	uint32_t q;

	if (A.hash_proto == 0u) {
		q = A.index % A.num_qs;
	} else {
		const uint32_t hp = A.hash_proto;
		/* plain frames are UDP or TCP: the parser's has_udp / has_tcp */
		const bool ports = proto == 17u ? (hp & (ODPG_HASH_IPV4_UDP | ODPG_HASH_IPV6_UDP)) != 0u
				   : (hp & (ODPG_HASH_IPV4_TCP | ODPG_HASH_IPV6_TCP)) != 0u;
		uint32_t crc = 0u;

		if (ports) {
			const uint32_t pw = __builtin_amdgcn_alignbyte(f[9], f[8], 2);

#pragma unroll
			for (int j = 0; j < 4; ++j)
				crc = crc_tab(tab, crc, (pw >> (8 * j)) & 0xffu);
		}
		if (hp & ODPG_HASH_IPV4) {
			const uint32_t a0 = __builtin_amdgcn_alignbyte(f[7], f[6], 2);
			const uint32_t a1 = __builtin_amdgcn_alignbyte(f[8], f[7], 2);

#pragma unroll
			for (int j = 0; j < 4; ++j)
				crc = crc_tab(tab, crc, (a0 >> (8 * j)) & 0xffu);
#pragma unroll
			for (int j = 0; j < 4; ++j)
				crc = crc_tab(tab, crc, (a1 >> (8 * j)) & 0xffu);
		}
		q = crc % A.num_qs;
	}
	return res | (q & ODPG_TX_OUT_QUEUE_MASK);
}

/* one packet through loopback_fix_checksums + get_dest_queue, general
 * form (any layout, metadata or the parse; byte-range sums and stores);
 * row: the lane's LDS row for the parse */
__device__ void tx_generic(const TxArgs &A, const uint32_t *tab, uint32_t *row, uint32_t i)
{
	uint8_t *g;
	uint32_t len;

	if (A.desc) {
		const odpg_desc_t d = A.desc[i];

		g = A.frames + d.offset;
		len = d.len;
	} else {
		g = A.frames + (size_t)i * A.stride;
		len = A.stride;
	}
	uint32_t l3, l4, fl;

	if (A.meta) {
		const odpg_tx_meta_t m = A.meta[i];

		l3 = m.l3_offset;
		l4 = m.l4_offset;
		fl = m.flags;
	} else {
		/* _odp_packet_parse_common, all layers, no checksum options */
		for (uint32_t w = 0; w < TX_W / 4; ++w)
			row[w] = tx_word(g, len, w);
		Pkt<TX_W, true> v;
		Prs p;

		v.row = row;
		v.g = g;
		v.len = len;
		p.inf = 0ull;
		p.fl = 0u;
		p.l2 = p.l3 = p.l4 = 0xffffu;
		parse_common(p, v, LAYER_ALL, 0ull);
		l3 = p.l3;
		l4 = p.l4;
		fl = ((p.inf & IF(IFL_IPV4)) ? ODPG_TX_HAS_IPV4 : 0u) |
		     ((p.inf & IF(IFL_IPV6)) ? ODPG_TX_HAS_IPV6 : 0u) |
		     ((p.inf & IF(IFL_UDP)) ? ODPG_TX_HAS_UDP : 0u) |
		     ((p.inf & IF(IFL_TCP)) ? ODPG_TX_HAS_TCP : 0u);
	}
	uint32_t res = 0u;

	/* ---- loopback_fix_checksums (loop.c:415-466) ---------------------- */
	if (l3 != ODPG_OFFSET_INVALID && l3 < len) {
		/* check_proto (loop.c:382-411) */
		const uint32_t ver = tx_u8(g, len, l3) >> 4, l3_len = len - l3;
		bool ok = false, v4 = false;
		uint32_t l4p = 0u;

		if (ver == 4u && l3_len >= 20u) {
			const uint32_t frag = (tx_u8(g, len, l3 + 6u) << 8) | tx_u8(g, len, l3 + 7u);

			ok = true;
			v4 = true;
			l4p = (frag & 0x3fffu) ? 255u : tx_u8(g, len, l3 + 9u);
		} else if (ver == 6u && l3_len >= 40u) {
			ok = true;
			l4p = tx_u8(g, len, l3 + 6u);
		}
		if (ok) {
			/* OL_TX_CHKSUM_PKT (loop.c:379-380) */
			auto want = [&](uint64_t bit, bool proto, uint32_t set, uint32_t ovr) {
				return (A.capa & bit) && proto && ((fl & set) ? (fl & ovr) != 0u
									: (A.cfg & bit) != 0u);
			};
			const bool ip4 = want(ODPG_PKTOUT_IPV4_CHKSUM, v4, ODPG_TX_L3_CHKSUM_SET,
					      ODPG_TX_L3_CHKSUM);
			const bool udp = want(ODPG_PKTOUT_UDP_CHKSUM, l4p == 17u, ODPG_TX_L4_CHKSUM_SET,
					      ODPG_TX_L4_CHKSUM);
			const bool tcp = want(ODPG_PKTOUT_TCP_CHKSUM, l4p == 6u, ODPG_TX_L4_CHKSUM_SET,
					      ODPG_TX_L4_CHKSUM);
			const bool sctp = want(ODPG_PKTOUT_SCTP_CHKSUM, l4p == 132u,
					       ODPG_TX_L4_CHKSUM_SET, ODPG_TX_L4_CHKSUM);

			/* _odp_packet_ipv4_chksum_insert (odp_packet.c:1729-1787) */
			if (ip4 && l3 + 20u <= len) {
				const uint32_t nleft = (tx_u8(g, len, l3) & 0x0fu) * 4u;

				if (nleft >= 20u && l3 + nleft <= len) {
					const uint32_t s = tx_sum(g, len, l3, l3, nleft, l3 + 10u, l3 + 12u);

					if (tx_store(g, len, l3 + 10u, ~s & 0xffffu, 2u))
						res |= ODPG_TX_OUT_IPV4;
				}
			}
			/* _odp_packet_tcp_udp_chksum_insert (odp_packet.c:1789-1862):
			 * both write at l4 + _ODP_UDP_CSUM_OFFSET */
			for (int pass = 0; pass < 2; ++pass) {
				const bool is_tcp = pass == 0;

				if (!(is_tcp ? tcp : udp) || l4 == ODPG_OFFSET_INVALID)
					continue;
				const uint32_t cs = l4 + 6u;
				uint32_t s = (tx_u8(g, len, l3) >> 4) == 4u
					     ? tx_sum(g, len, l3, l3 + 12u, 8u)
					     : tx_sum(g, len, l3, l3 + 8u, 32u);

				s = oc_add(s, (is_tcp ? 6u : 17u) << 8);
				if (is_tcp) {
					const uint32_t tl = (len - l4) & 0xffffu;

					s = oc_add(s, ((tl >> 8) | (tl << 8)) & 0xffffu);
				} else {
					s = oc_add(s, tx_sum(g, len, l3, l4 + 4u, 2u));
				}
				const bool zeroed = cs + 2u <= len;   /* the zero write */

				s = oc_add(s, tx_sum(g, len, l3, l4, len - l4,
						      zeroed ? cs : 0u, zeroed ? cs + 2u : 0u));
				uint32_t c = ~oc_fold(s) & 0xffffu;

				if (!is_tcp && c == 0u)
					c = 0xffffu;
				if (tx_store(g, len, cs, c, 2u))
					res |= is_tcp ? ODPG_TX_OUT_TCP : ODPG_TX_OUT_UDP;
			}
			/* _odp_packet_sctp_chksum_insert (odp_packet.c:1884-1898) */
			if (sctp && l4 != ODPG_OFFSET_INVALID) {
				const bool zeroed = l4 + 12u <= len;
				uint32_t crc = 0xffffffffu;

				if (l4 <= len)
					for (uint32_t p = l4; p < len; ++p) {
						const uint32_t b = (zeroed && p >= l4 + 8u && p < l4 + 12u)
								   ? 0u : g[p];

						crc = crc_tab(tab, crc, b);
					}
				if (tx_store(g, len, l4 + 8u, ~crc, 4u))
					res |= ODPG_TX_OUT_SCTP;
			}
		}
	}

	/* ---- get_dest_queue (loop.c:468-523) ------------------------------- */
	uint32_t q;

	if (A.hash_proto == 0u) {
		q = A.index % A.num_qs;
	} else {
		const uint32_t hp = A.hash_proto;
		uint32_t crc = 0u;

		if (l4 != ODPG_OFFSET_INVALID) {
			bool ports = false;

			if ((hp & (ODPG_HASH_IPV4_UDP | ODPG_HASH_IPV6_UDP)) && (fl & ODPG_TX_HAS_UDP))
				ports = l4 + 8u <= len;
			else if ((hp & (ODPG_HASH_IPV4_TCP | ODPG_HASH_IPV6_TCP)) &&
				 (fl & ODPG_TX_HAS_TCP))
				ports = l4 + 20u <= len;
			if (ports)
				for (uint32_t j = 0; j < 4u; ++j)
					crc = crc_tab(tab, crc, g[l4 + j]);
		}
		if (l3 != ODPG_OFFSET_INVALID) {
			uint32_t a = 0u, n = 0u;

			if ((hp & ODPG_HASH_IPV4) && (fl & ODPG_TX_HAS_IPV4)) {
				if (l3 + 20u <= len) {
					a = l3 + 12u;
					n = 8u;
				}
			} else if ((hp & ODPG_HASH_IPV6) && (fl & ODPG_TX_HAS_IPV6)) {
				if (l3 + 40u <= len) {
					a = l3 + 8u;
					n = 32u;
				}
			}
			for (uint32_t j = 0; j < n; ++j)
				crc = crc_tab(tab, crc, g[a + j]);
		}
		q = crc % A.num_qs;
	}
	A.out[i] = res | (q & ODPG_TX_OUT_QUEUE_MASK);
}

__global__ __launch_bounds__(TX_BLOCK) void odpg_tx_kernel(const TxArgs A)
{
	__shared__ uint32_t tab[256];
	__shared__ uint32_t rows[TX_BLOCK * TX_RW];
	const uint32_t tid = threadIdx.x;

	{
		/* reflected Castagnoli table (arch/default/odp_hash_crc32.c) */
		uint32_t c = tid;

		for (int k = 0; k < 8; ++k)
			c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
		tab[tid] = c;
	}
	__syncthreads();
	const uint32_t i = blockIdx.x * TX_BLOCK + tid;
	const bool live = i < A.num;

	if (A.stride == 64u && !A.desc && !A.meta) {
		/* register fast path: a wave whose frames are all plain
		 * Eth/IPv4 (IHL 5)/UDP|TCP 64-byte frames (the parse gives l3 14,
		 * l4 34, IPv4 + UDP|TCP) works on the 16 frame registers and
		 * stores back only the dwords holding the checksum fields */
		uint32_t f[16];
		uint4 *src = (uint4 *)(A.frames + (size_t)(live ? i : A.num - 1u) * 64u);

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint4 x = src[k];

			f[4 * k + 0] = x.x;
			f[4 * k + 1] = x.y;
			f[4 * k + 2] = x.z;
			f[4 * k + 3] = x.w;
		}
		if (__ballot(live && !plain_v4(f)) == 0ull) {
			if (live)
				A.out[i] = tx_fast64(A, tab, f, (uint32_t *)src);
			return;
		}
	}
	if (live)
		tx_generic(A, tab, rows + tid * TX_RW, i);
}

/* Stride-64 batches without metadata (the bench's and the loop device's
 * shape): waves persistent over 64-frame tiles; a tile's 4 KiB loaded
 * coalesced one tile ahead and transposed to a frame per lane through the
 * wave's LDS rows, and, on waves of plain frames, the frames written back
 * whole the same way (1 KiB of whole lines per store instruction; a
 * partial-sector write costs more than a whole one, fwd.hip). Same swizzle
 * as classify64.hip's L64_COAL staging. Waves with any other frame take
 * tx_generic per lane. */
#ifndef TX_PWAVES           /* waves per SIMD: 160 VGPRs, the generic path inlined without spills */
#define TX_PWAVES 3
#endif
__global__ __launch_bounds__(TX_BLOCK, TX_PWAVES * 256 / TX_BLOCK) void odpg_tx64_kernel(const TxArgs A)
{
	__shared__ uint32_t tab[256];
	__shared__ __attribute__((aligned(16))) uint32_t rows[TX_BLOCK * TX_RW];
	const uint32_t tid = threadIdx.x;
	const uint32_t lane = __lane_id();
	const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (TX_BLOCK / 64) + (tid >> 6));
	const uint32_t nwaves = gridDim.x * (TX_BLOCK / 64);
	const uint32_t num = A.num;
	const uint32_t ntiles = (num + 63u) >> 6;
	uint4 *frames = (uint4 *)A.frames;
	uint32_t *stg = rows + (tid & ~63u) * TX_RW;
	const uint32_t sw_fr = lane >> 2;
	const uint32_t sw_w = 16u * sw_fr + 4u * (((lane & 3u) + sw_fr + (sw_fr >> 2)) & 3u);
	const uint32_t sw_c = lane + (lane >> 2);
	/* checksum inserts the configuration asks for: plain waves write back */
	const bool wb = ((A.capa & A.cfg) & (ODPG_PKTOUT_IPV4_CHKSUM | ODPG_PKTOUT_UDP_CHKSUM |
					     ODPG_PKTOUT_TCP_CHKSUM)) != 0u;

	auto load_raw = [&](uint32_t (&dst)[16], uint32_t t) {
		if (t >= ntiles)
			return;
		const uint32_t lim = num * 4u - 1u;       /* < 2^30 packets (launcher) */
		const uint32_t c0 = t * 256u + lane;

#pragma unroll
		for (int q = 0; q < 4; ++q) {
			const uint4 x = frames[min(c0 + 64u * q, lim)];

			dst[4 * q + 0] = x.x;
			dst[4 * q + 1] = x.y;
			dst[4 * q + 2] = x.z;
			dst[4 * q + 3] = x.w;
		}
	};
	uint32_t fn[16] = {};

	load_raw(fn, gw);
	{
		uint32_t c = tid;

		for (int k = 0; k < 8; ++k)
			c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
		tab[tid] = c;
	}
	__syncthreads();

	for (uint32_t t = gw; t < ntiles; t += nwaves) {
		uint32_t f[16];

#pragma unroll
		for (int q = 0; q < 4; ++q)
			*(uint4 *)(stg + sw_w + 256u * q) =
				make_uint4(fn[4 * q], fn[4 * q + 1], fn[4 * q + 2], fn[4 * q + 3]);
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const uint4 x = *(const uint4 *)(stg + 16u * lane + 4u * ((j + sw_c) & 3u));

			f[4 * j + 0] = x.x;
			f[4 * j + 1] = x.y;
			f[4 * j + 2] = x.z;
			f[4 * j + 3] = x.w;
		}
		const uint32_t i = t * 64u + lane;
		const bool live = i < num;

		if (__ballot(live && !plain_v4(f)) == 0ull) {
			/* the next tile's loads only here: none are in flight (no
			 * registers held) across the generic path below */
			load_raw(fn, t + nwaves);
			const uint32_t r = tx_fast64(A, tab, f, nullptr);

			if (live)
				A.out[i] = r;
			if (wb) {
				/* the frame back through its LDS slots (dwords 6 and
				 * 10 may have changed), then the tile's chunks in
				 * load order */
#pragma unroll
				for (int j = 1; j < 3; ++j)
					*(uint4 *)(stg + 16u * lane + 4u * ((j + sw_c) & 3u)) =
						make_uint4(f[4 * j], f[4 * j + 1], f[4 * j + 2], f[4 * j + 3]);
				const uint32_t cb = t * 256u + lane, nc = num * 4u;

#pragma unroll
				for (int q = 0; q < 4; ++q)
					if (cb + 64u * q < nc)
						frames[cb + 64u * q] = *(const uint4 *)(stg + sw_w + 256u * q);
			}
			continue;
		}
		/* the generic path reads the frame from global memory; its LDS
		 * row is this lane's slice of the wave's staging area */
		if (live)
			tx_generic(A, tab, rows + tid * TX_RW, i);
		load_raw(fn, t + nwaves);
	}
}

} /* namespace */

extern "C" uint32_t odpg_resident_grid(const void *kernel, uint32_t block, size_t lds);

extern "C" int odpg_tx_prepare(odpg_ctx_t *ctx, const odpg_tx_batch_t *b,
			       const odpg_tx_cfg_t *cfg, uint32_t *out)
{
	if (!ctx || !b || !cfg || cfg->num_qs == 0u || (b->num && (!b->frames || !out)) ||
	    (!b->desc && b->num && b->stride == 0u))
		return -EINVAL;
	if (b->num == 0)
		return 0;
	TxArgs A;

	A.frames = b->frames;
	A.desc = b->desc;
	A.stride = b->stride;
	A.num = b->num;
	A.meta = b->meta;
	A.cfg = cfg->pktout_cfg;
	A.capa = cfg->pktout_capa;
	A.hash_proto = cfg->hash_proto;
	A.num_qs = cfg->num_qs;
	A.index = cfg->index;
	A.out = out;
	hipStream_t s = (hipStream_t)odpg_ctx_stream(ctx);

	if (b->stride == 64u && !b->desc && !b->meta && b->num < (1u << 30)) {
		const uint32_t want = ((b->num + 63u) / 64u + TX_BLOCK / 64u - 1u) / (TX_BLOCK / 64u);
		uint32_t grid = odpg_resident_grid((const void *)odpg_tx64_kernel, TX_BLOCK, 0);

		grid = grid < want ? grid : want;
		hipLaunchKernelGGL(odpg_tx64_kernel, dim3(grid ? grid : 1u), dim3(TX_BLOCK), 0, s, A);
		return hipGetLastError() == hipSuccess ? 0 : -EIO;
	}
	hipLaunchKernelGGL(odpg_tx_kernel, dim3((b->num + TX_BLOCK - 1) / TX_BLOCK), dim3(TX_BLOCK),
			   0, s, A);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
