/* SPDX-License-Identifier: BSD-3-Clause
 *
 * gfx950 batch forwarding decision of ODP's example/l3fwd (include/odpg_fwd.h,
 * SURVEY.md §8(f) rank 2, BASELINE config C5).
 *
 * One lane per packet, 256-lane workgroups. Per packet:
 *   1. parse like the pktio does for l3fwd (layer L4, or ALL with -e; no RX
 *      checksum options, odp_l3fwd.c:132-135): waves whose frames are all
 *      plain 64-byte Eth/IPv4/UDP|TCP take the register parse of
 *      pkt_parse.h; other waves stage the frame in LDS and run the restated
 *      _odp_packet_parse_common;
 *   2. drop_err_pkts (odp_l3fwd.c:269-292): parse drop, error with -e, or
 *      not IPv4 -> out_port = -1, frame untouched;
 *   3. route: hash mode = first match of the newest-first route list
 *      (find_fwd_db_entry, odp_l3fwd_db.c:474-508; routes are wave-uniform
 *      scalar loads); LPM mode = the reference's 16-4-4-4-4 trie
 *      (fib_tbl_lookup, odp_l3fwd_lpm.c:210-230), one dependent L2-resident
 *      load per level;
 *   4. ipv4_dec_ttl_csum_update (odp_l3fwd.c:183-192) and the MAC rewrite of
 *      l3fwd_pkt_hash / l3fwd_pkt_lpm, written back in place (fast waves:
 *      two 16-byte stores of bytes 0..31).
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/odpg_fwd.h"
#include "pkt_parse.h"

#define FBLOCK 256

/* trie node word: bit 31 leaf (end), bit 30 valid, bits 0..23 next hop
 * (leaf) or first child index in the sub-table pool (inner node) */
#define FN_END   0x80000000u
#define FN_VALID 0x40000000u
#define FN_VAL   0x00ffffffu
/* hash-mode interval table: 0, two points per route's scan range, up to
 * four per route's warmed ranges (two when a range wraps past 2^32) */
#define FWD_MAX_IV (6 * ODPG_FWD_MAX_ROUTES + 1)

struct odpg_fwd_s {
	odpg_ctx_t *ctx;
	uint32_t mode;
	uint32_t nroutes;
	uint4 *d_routes;      /* newest first: {addr, mask, oif, 0} */
	uint4 *d_rmac;        /* per route: frame bytes 0..11 after rewrite, oif */
	uint4 *d_pmac;        /* per port (LPM): frame bytes 0..11, 3 words */
	uint32_t *d_l1;       /* LPM: 65536 first-level nodes; hash: route intervals */
	uint32_t *d_pool;     /* sub-table pool */
	uint32_t num_ports;
};

/* ---- host: the reference trie builder, restated (odp_l3fwd_lpm.c) -------
 * Kept exactly, quirks included (see oracle/odp_oracle.c for the list):
 * first-level nodes for depth <= 16 are set one node at a time, a split
 * leaves the children invalid, a route ending inside a stride updates the
 * single child at `ip >> width`, updates recurse only into leaf children,
 * sub table k lives at pool index (k + 1) * 16. */
namespace {

struct TrieNode {
	uint32_t val = 0;     /* next hop, or pool index of the children */
	bool valid = false, leaf = true;
	uint8_t depth = 0;
};

class FibTrie {
public:
	static constexpr uint32_t kL1 = 65536, kPool = 16384;
	std::vector<TrieNode> top, pool;
	uint32_t used = 0;
	bool overflow = false;

	FibTrie() : top(kL1), pool(kPool) {}

	void add(uint32_t ip, uint32_t port, uint32_t depth)
	{
		TrieNode &n = top[ip >> 16];

		if (depth <= 16) {
			if (n.leaf) {
				n.val = port;
				n.depth = (uint8_t)depth;
				n.valid = true;
				return;
			}
			for (uint32_t i = 0; i < 16; i++) {
				TrieNode &c = pool[n.val + i];

				if (c.leaf) {
					refresh(c, port, depth);
				} else {
					for (uint32_t j = 0; j < 16; j++)
						refresh(pool[c.val + j], port, depth);
				}
			}
			return;
		}
		descend(n, ip & 0xffffu, port, 16, 16, depth);
	}

private:
	bool grow(uint32_t &base)
	{
		const uint32_t b = (used + 1) * 16;

		if (2 * b > kPool) {
			overflow = true;
			return false;
		}
		for (uint32_t i = 0; i < b; i++) {
			pool[b + i].valid = false;
			pool[b + i].leaf = true;
		}
		used++;
		base = b;
		return true;
	}

	void refresh(TrieNode &n, uint32_t port, uint32_t depth)
	{
		if (!n.leaf) {
			for (uint32_t i = 0; i < 16; i++)
				if (pool[n.val + i].leaf)
					refresh(pool[n.val + i], port, depth);
			return;
		}
		if (!n.valid || n.depth <= depth) {
			n.val = port;
			n.depth = (uint8_t)depth;
			n.valid = true;
		}
	}

	void descend(TrieNode &start, uint32_t ip, uint32_t port, uint32_t width, uint32_t eaten,
		     uint32_t depth)
	{
		TrieNode *n = &start;

		while (true) {
			if (n->leaf) {
				uint32_t base;
				const uint32_t keep = n->val;

				if (!grow(base))
					return;
				if (n->valid)
					for (uint32_t i = 0; i < 16; i++) {
						pool[base + i].val = keep;
						pool[base + i].depth = n->depth;
					}
				n->val = base;
				n->leaf = false;
			}
			if (depth - eaten <= 4) {
				width -= depth - eaten;
				refresh(pool[n->val + (ip >> width)], port, depth);
				return;
			}
			width -= 4;
			n = &pool[n->val + (ip >> width)];
			ip &= (1u << width) - 1u;
			eaten += 4;
		}
	}
};

uint32_t node_word(const TrieNode &n)
{
	return (n.leaf ? FN_END : 0u) | (n.valid ? FN_VALID : 0u) | (n.val & FN_VAL);
}

/* frame bytes 0..11 = dst MAC | src MAC as three little-endian words */
uint4 mac_words(const uint8_t dst[6], const uint8_t src[6])
{
	uint8_t b[12];
	uint4 w;

	memcpy(b, dst, 6);
	memcpy(b + 6, src, 6);
	memcpy(&w.x, b, 4);
	memcpy(&w.y, b + 4, 4);
	memcpy(&w.z, b + 8, 4);
	w.w = 0;
	return w;
}

template <typename T>
int upload(odpg_ctx_t *ctx, const std::vector<T> &h, T **d)
{
	void *p = nullptr;
	const size_t bytes = h.size() * sizeof(T);

	if (odpg_dev_alloc(ctx, bytes ? bytes : 16, &p))
		return -ENOMEM;
	if (bytes && odpg_memcpy_h2d(ctx, p, h.data(), bytes)) {
		odpg_dev_free(ctx, p);
		return -EIO;
	}
	*d = (T *)p;
	return 0;
}

} /* namespace */

/* ---- device ------------------------------------------------------------ */
__device__ __forceinline__ uint32_t ttl_csum_word5(uint32_t w5)
{
	/* byte 22 (TTL) of a plain frame is bits 16..23 of word 5 */
	return (w5 & 0xff00ffffu) | ((((w5 >> 16) - 1u) & 0xffu) << 16);
}

__device__ __forceinline__ uint32_t csum_update(uint32_t cs)
{
	/* raw little-endian u16 of the checksum field, a = ~be16(0x100) = 0xfffe */
	return cs >= 0xfffeu ? cs - 0xfffeu : cs + 1u;
}

/* W: bytes of the frame staged per lane in LDS for the generic parse (the
 * frame itself at stride 64; 128 otherwise, the rest from global when GF).
 * The row array is the kernel's whole LDS: 64-byte rows (17 KiB per
 * workgroup) leave 8 workgroups per CU resident where 128-byte rows (34 KiB)
 * allowed 4 (C5 10 M packets: hash 291 -> 281 us, LPM 311 -> 265 us) */
template <int W, bool GF>
__global__ __launch_bounds__(FBLOCK) void odpg_l3fwd_kernel(
	uint8_t *__restrict__ frames, uint32_t stride, uint32_t num, int32_t sif, uint32_t layer,
	uint32_t mode, const uint4 *__restrict__ routes, const uint4 *__restrict__ rmac,
	uint32_t nroutes, const uint32_t *__restrict__ l1, const uint32_t *__restrict__ pool,
	const uint4 *__restrict__ pmac, int32_t *__restrict__ out_port)
{
	constexpr uint32_t RW = W / 4 + 1;
	__shared__ uint32_t rows[FBLOCK * RW];
	__shared__ uint4 s_rmac[ODPG_FWD_MAX_ROUTES];
	__shared__ uint4 s_pmac[ODPG_FWD_MAX_PORTS];
	/* hash mode: the route list as address intervals (fwd_intervals) */
	__shared__ uint32_t s_ivb[FWD_MAX_IV], s_iva[FWD_MAX_IV];

	const uint32_t tid = threadIdx.x;
	const uint32_t i = blockIdx.x * FBLOCK + tid;
	const bool live = i < num;

	if (tid < ODPG_FWD_MAX_ROUTES && tid < nroutes)
		s_rmac[tid] = rmac[tid];
	if (tid < ODPG_FWD_MAX_PORTS)
		s_pmac[tid] = pmac[tid];
	const uint32_t niv = mode != ODPG_FWD_LPM ? l1[0] : 0u;   /* uniform */

	if (tid < niv) {
		s_ivb[tid] = l1[1u + 2u * tid];
		s_iva[tid] = l1[2u + 2u * tid];
	}

	uint8_t *fr = frames + (size_t)(live ? i : 0u) * stride;
	uint32_t f[16];
	bool plain = false;

	if (stride == 64u) {
		const uint4 *src = (const uint4 *)fr;

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint4 x = live ? src[k] : make_uint4(0u, 0u, 0u, 0u);

			f[4 * k + 0] = x.x;
			f[4 * k + 1] = x.y;
			f[4 * k + 2] = x.z;
			f[4 * k + 3] = x.w;
		}
		plain = layer >= LAYER_L4 && plain_v4(f);
	}
	const bool wave_fast = __ballot(live && !plain) == 0ull;
	uint32_t *row = rows + tid * RW;

	if (!wave_fast) {
		/* stage the first W bytes in this lane's LDS row, zero past the end */
#pragma unroll
		for (uint32_t part = 0; part < W / 16; ++part) {
			const uint32_t b0 = part * 16u;
			uint4 x = make_uint4(0u, 0u, 0u, 0u);

			if (live && b0 < stride)
				x = *(const uint4 *)(fr + b0);
			row[part * 4u + 0u] = x.x;
			row[part * 4u + 1u] = x.y;
			row[part * 4u + 2u] = x.z;
			row[part * 4u + 3u] = x.w;
		}
	}
	__syncthreads();

	Prs p;

	p.inf = 0ull;
	p.fl = 0u;
	p.l2 = p.l3 = p.l4 = 0xffffu;
	int ret = 0;
	Pkt<W, GF> v;

	v.row = row;
	v.g = fr;
	v.len = live ? stride : 0u;
	if (wave_fast) {
		if (live)
			ret = parse_fast(p, f, 0ull);
	} else if (live) {
		ret = parse_common(p, v, layer, 0ull);
	}
	const bool drop = !live || ret < 0 || (layer == LAYER_ALL && (p.fl & FL_ERROR_MASK)) ||
			  !(p.inf & IF(IFL_IPV4));
	const uint32_t l3 = p.l3;
	const uint32_t dst = wave_fast ? __builtin_bswap32(fw<30>(f))
				       : (drop ? 0u : __builtin_bswap32(v.rd32(l3 + 16u)));
	int32_t dif = sif;
	uint4 mac;

	if (mode == ODPG_FWD_LPM) {
		uint32_t n = l1[dst >> 16], rest = dst & 0xffffu, bits = 16u;

		while (!(n & FN_END)) {          /* at most four sub levels */
			bits -= 4u;
			n = pool[(n & FN_VAL) + (rest >> bits)];
			rest &= (1u << bits) - 1u;
		}
		if (n & FN_VALID)
			dif = (int32_t)(n & FN_VAL);
		mac = s_pmac[(uint32_t)dif & (ODPG_FWD_MAX_PORTS - 1u)];
	} else {
		/* first match of the newest-first route list
		 * (find_fwd_db_entry): the interval holding dst carries it.
		 * Branch-free binary search for the last start <= dst (the
		 * first start is 0). */
		uint32_t pos = 0u;

#pragma unroll
		for (uint32_t step = 128u; step; step >>= 1) {   /* reaches index 255 >= FWD_MAX_IV - 1 */
			const uint32_t q = pos + step;

			if (q < niv && s_ivb[q] <= dst)
				pos = q;
		}
		const int32_t k = niv ? (int32_t)s_iva[pos] : -1;
		if (k >= 0) {
			mac = s_rmac[k];
			dif = (int32_t)mac.w;
		} else {
			/* no route: eth->dst = eth->src, src unchanged */
			const uint32_t w1 = wave_fast ? f[1] : row[1], w2 = wave_fast ? f[2] : row[2];

			mac.x = __builtin_amdgcn_alignbyte(w2, w1, 2);
			mac.y = (w2 >> 16) | (w1 & 0xffff0000u);
			mac.z = w2;
		}
	}

	if (!drop) {
		if (wave_fast) {
			f[0] = mac.x;
			f[1] = mac.y;
			f[2] = mac.z;
			f[5] = ttl_csum_word5(f[5]);
			f[6] = (f[6] & 0xffff0000u) | csum_update(f[6] & 0xffffu);
			uint4 *dp = (uint4 *)fr;

			dp[0] = make_uint4(f[0], f[1], f[2], f[3]);
			dp[1] = make_uint4(f[4], f[5], f[6], f[7]);
		} else {
			uint32_t *w = (uint32_t *)fr;
			const uint32_t ttl = v.u8(l3 + 8u);
			const uint32_t cs = v.rd32(l3 + 10u) & 0xffffu;

			w[0] = mac.x;
			w[1] = mac.y;
			w[2] = mac.z;
			fr[l3 + 8u] = (uint8_t)(ttl - 1u);
			*(uint16_t *)(fr + l3 + 10u) = (uint16_t)csum_update(cs);
		}
	}
	if (live)
		out_port[i] = drop ? -1 : dif;
}

/* ---- persistent kernel for 64-byte frames ---------------------------------
 * The same per-packet work as odpg_l3fwd_kernel<64, false>, for stride 64:
 * one wave per 64-packet tile, waves persistent over tiles. A tile's 4 KiB
 * arrive as coalesced 16-byte loads (lane l: chunks l, l + 64, l + 128,
 * l + 192), issued one tile ahead, and are transposed to one frame per lane
 * through the wave's own LDS rows, chunk (frame r, part p) at slot
 * (p + r + r / 4) % 4 of row r: conflict-free for the ds_write_b128 and
 * ds_read_b128 lane groups (as classify64.hip's L64_COAL staging). Hash mode
 * issues the next tile's loads before this tile's route search (LDS only);
 * LPM mode after its trie walk, whose dependent global loads would otherwise
 * wait for them (vector-memory loads retire in issue order). */
#ifndef FWD_PBLOCK
#define FWD_PBLOCK 256
#endif
#ifndef FWD_WAVES           /* waves per SIMD the launch bounds ask for */
#define FWD_WAVES 8
#endif

template <bool LPM>
__global__ __launch_bounds__(FWD_PBLOCK, FWD_WAVES * 256 / FWD_PBLOCK) void odpg_l3fwd64_kernel(
	uint4 *__restrict__ frames, uint32_t num, int32_t sif, uint32_t layer,
	const uint4 *__restrict__ rmac, uint32_t nroutes, const uint32_t *__restrict__ l1,
	const uint32_t *__restrict__ pool, const uint4 *__restrict__ pmac,
	int32_t *__restrict__ out_port)
{
	constexpr uint32_t RW = 17;                 /* odd dword row stride */
	__shared__ __attribute__((aligned(16))) uint32_t rows[FWD_PBLOCK * RW];
	__shared__ uint4 s_rmac[ODPG_FWD_MAX_ROUTES];
	__shared__ uint4 s_pmac[ODPG_FWD_MAX_PORTS];
	__shared__ uint32_t s_ivb[FWD_MAX_IV], s_iva[FWD_MAX_IV];

	const uint32_t tid = threadIdx.x;
	const uint32_t lane = __lane_id();
	const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (FWD_PBLOCK / 64) + (tid >> 6));
	const uint32_t nwaves = gridDim.x * (FWD_PBLOCK / 64);
	const uint32_t ntiles = (num + 63u) >> 6;
	uint32_t *row = rows + tid * RW;
	uint32_t *stg = rows + (tid & ~63u) * RW;
	const uint32_t sw_fr = lane >> 2;
	const uint32_t sw_w = 16u * sw_fr + 4u * (((lane & 3u) + sw_fr + (sw_fr >> 2)) & 3u);
	const uint32_t sw_c = lane + (lane >> 2);

	auto load_raw = [&](uint32_t (&dst)[16], uint32_t t) {
		if (t >= ntiles)
			return;
		const size_t lim = (size_t)num * 4u - 1u;
		const size_t c0 = (size_t)t * 256u + lane;

#pragma unroll
		for (int q = 0; q < 4; ++q) {
			const size_t c = c0 + 64u * q;
			const uint4 x = frames[c < lim ? c : lim];

			dst[4 * q + 0] = x.x;
			dst[4 * q + 1] = x.y;
			dst[4 * q + 2] = x.z;
			dst[4 * q + 3] = x.w;
		}
	};
	auto stage = [&](const uint32_t (&raw)[16], uint32_t (&f)[16]) {
#pragma unroll
		for (int q = 0; q < 4; ++q)
			*(uint4 *)(stg + sw_w + 256u * q) =
				make_uint4(raw[4 * q], raw[4 * q + 1], raw[4 * q + 2], raw[4 * q + 3]);
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const uint4 x = *(const uint4 *)(stg + 16u * lane + 4u * ((j + sw_c) & 3u));

			f[4 * j + 0] = x.x;
			f[4 * j + 1] = x.y;
			f[4 * j + 2] = x.z;
			f[4 * j + 3] = x.w;
		}
	};
	uint32_t fn[16] = {};

	load_raw(fn, gw);
	for (uint32_t k = tid; k < nroutes && k < ODPG_FWD_MAX_ROUTES; k += FWD_PBLOCK)
		s_rmac[k] = rmac[k];
	for (uint32_t k = tid; k < ODPG_FWD_MAX_PORTS; k += FWD_PBLOCK)
		s_pmac[k] = pmac[k];
	const uint32_t niv = LPM ? 0u : l1[0];     /* uniform */

	for (uint32_t k = tid; k < niv; k += FWD_PBLOCK) {
		s_ivb[k] = l1[1u + 2u * k];
		s_iva[k] = l1[2u + 2u * k];
	}
	__syncthreads();

	/* the route of dst: out port and the frame's new bytes 0..11 (w1, w2:
	 * the frame's words 1, 2, for the no-route MAC swap) */
	auto route = [&](uint32_t dst, uint32_t w1, uint32_t w2, uint4 &mac) -> int32_t {
		int32_t dif = sif;

		if constexpr (LPM) {
			uint32_t n = l1[dst >> 16], rest = dst & 0xffffu, bits = 16u;

			while (!(n & FN_END)) {          /* at most four sub levels */
				bits -= 4u;
				n = pool[(n & FN_VAL) + (rest >> bits)];
				rest &= (1u << bits) - 1u;
			}
			if (n & FN_VALID)
				dif = (int32_t)(n & FN_VAL);
			mac = s_pmac[(uint32_t)dif & (ODPG_FWD_MAX_PORTS - 1u)];
		} else {
			uint32_t pos = 0u;

#pragma unroll
			for (uint32_t step = 128u; step; step >>= 1) {   /* reaches index 255 >= FWD_MAX_IV - 1 */
				const uint32_t q = pos + step;

				if (q < niv && s_ivb[q] <= dst)
					pos = q;
			}
			const int32_t k = niv ? (int32_t)s_iva[pos] : -1;

			if (k >= 0) {
				mac = s_rmac[k];
				dif = (int32_t)mac.w;
			} else {
				mac.x = __builtin_amdgcn_alignbyte(w2, w1, 2);
				mac.y = (w2 >> 16) | (w1 & 0xffff0000u);
				mac.z = w2;
			}
		}
		return dif;
	};

	for (uint32_t t = gw; t < ntiles; t += nwaves) {
		uint32_t f[16];

		stage(fn, f);
		if (!LPM)
			load_raw(fn, t + nwaves);
		const uint32_t i = t * 64u + lane;
		const bool live = i < num;
		uint4 *fr = frames + (size_t)(live ? i : 0u) * 4u;
		const bool fast = __ballot(live && !(layer >= LAYER_L4 && plain_v4(f))) == 0ull;

		if (fast) {
			/* plain frames, no RX checksum options: parse_fast cannot flag
			 * an error, every frame is IPv4 (drop_err_pkts keeps it) */
			uint4 mac;
			const int32_t dif = route(__builtin_bswap32(fw<30>(f)), f[1], f[2], mac);

			if (LPM)
				load_raw(fn, t + nwaves);
			/* the rewritten frame back through the same LDS slots, then each
			 * lane stores the chunks it loaded (1 KiB contiguous per store
			 * instruction; whole frames: a partial-sector write costs more
			 * than the whole sector) */
			const uint4 c0 = make_uint4(mac.x, mac.y, mac.z, f[3]);
			const uint4 c1 = make_uint4(f[4], ttl_csum_word5(f[5]),
						    (f[6] & 0xffff0000u) | csum_update(f[6] & 0xffffu), f[7]);

			*(uint4 *)(stg + 16u * lane + 4u * ((0u + sw_c) & 3u)) = c0;
			*(uint4 *)(stg + 16u * lane + 4u * ((1u + sw_c) & 3u)) = c1;
			if (live)
				out_port[i] = dif;
			const size_t cb = (size_t)t * 256u + lane;
			const size_t nc = (size_t)num * 4u;

#pragma unroll
			for (int q = 0; q < 4; ++q) {
				const size_t c = cb + 64u * q;

				if (c < nc)
					frames[c] = *(const uint4 *)(stg + sw_w + 256u * q);
			}
			continue;
		}
		/* any other wave: the generic parse over the frame in its LDS row */
#pragma unroll
		for (int q = 0; q < 16; ++q)
			row[q] = f[q];
		Prs p;

		p.inf = 0ull;
		p.fl = 0u;
		p.l2 = p.l3 = p.l4 = 0xffffu;
		int ret = 0;
		Pkt<64, false> v;

		v.row = row;
		v.g = (const uint8_t *)fr;
		v.len = live ? 64u : 0u;
		if (live)
			ret = parse_common(p, v, layer, 0ull);
		const bool drop = !live || ret < 0 || (layer == LAYER_ALL && (p.fl & FL_ERROR_MASK)) ||
				  !(p.inf & IF(IFL_IPV4));
		const uint32_t l3 = p.l3;
		const uint32_t dst = drop ? 0u : __builtin_bswap32(v.rd32(l3 + 16u));
		uint4 mac;
		const int32_t dif = route(dst, row[1], row[2], mac);

		if (LPM)
			load_raw(fn, t + nwaves);
		if (!drop) {
			uint8_t *fb = (uint8_t *)fr;
			uint32_t *w = (uint32_t *)fr;
			const uint32_t ttl = v.u8(l3 + 8u);
			const uint32_t cs = v.rd32(l3 + 10u) & 0xffffu;

			w[0] = mac.x;
			w[1] = mac.y;
			w[2] = mac.z;
			fb[l3 + 8u] = (uint8_t)(ttl - 1u);
			*(uint16_t *)(fb + l3 + 10u) = (uint16_t)csum_update(cs);
		}
		if (live)
			out_port[i] = drop ? -1 : dif;
	}
}

extern "C" uint32_t odpg_resident_grid(const void *kernel, uint32_t block, size_t lds);

/* ---- host API ------------------------------------------------------------ */
extern "C" int odpg_fwd_create(odpg_ctx_t *ctx, const odpg_route_t *routes, uint32_t num_routes,
			       const odpg_fwd_param_t *param, odpg_fwd_t **out)
{
	if (!ctx || !param || !out || (num_routes && !routes) || num_routes > ODPG_FWD_MAX_ROUTES ||
	    param->num_ports > ODPG_FWD_MAX_PORTS ||
	    (param->mode != ODPG_FWD_HASH && param->mode != ODPG_FWD_LPM))
		return -EINVAL;
	for (uint32_t k = 0; k < num_routes; k++) {
		const uint32_t d = routes[k].depth;

		if (d < 1 || d > 32 || routes[k].oif_id < 0 ||
		    (uint32_t)routes[k].oif_id >= ODPG_FWD_MAX_PORTS)
			return -EINVAL;
	}
	std::vector<uint4> rt, rm, pm(ODPG_FWD_MAX_PORTS);

	for (int k = (int)num_routes - 1; k >= 0; k--) {      /* newest first */
		const uint32_t d = routes[k].depth;

		/* find_fwd_db_entry's mask as x86-64 computes it: depth 32
		 * shifts "1u << 32" by 0, giving mask 0 (odp_l3fwd_db.c:496-497) */
		rt.push_back(make_uint4(routes[k].addr, ((1u << (d & 31u)) - 1u) << ((32u - d) & 31u),
					(uint32_t)routes[k].oif_id, 0u));
		uint4 m = mac_words(routes[k].dst_mac, routes[k].src_mac);

		m.w = (uint32_t)routes[k].oif_id;
		rm.push_back(m);
	}
	for (uint32_t p = 0; p < ODPG_FWD_MAX_PORTS; p++)
		pm[p] = mac_words(param->dest_mac[p], param->port_mac[p]);
	std::vector<uint32_t> l1(FibTrie::kL1, FN_END), pool(16, FN_END);

	if (param->mode == ODPG_FWD_HASH) {
		/* find_fwd_db_entry (odp_l3fwd_db.c:474-508) is a function of the
		 * destination alone once init_fwd_hash_cache (:304-335) has warmed
		 * the flow cache: a warmed address returns its cached route, any
		 * other the first list match (which is then cached, without
		 * changing later answers). The warm-up walks the list newest
		 * first, caching addr + i for i < 2^(32 - depth) (u32 wrap), and
		 * stops at the first address already cached or when the
		 * FWD_MAX_FLOW_COUNT flows are used up; so the warmed set is a few
		 * ranges. Both are folded into one interval table:
		 * l1 = {count, {start, route | -1}...} over [0, 2^32). */
		struct Iv {
			uint64_t lo, hi;    /* [lo, hi) */
			uint32_t route;
		};
		std::vector<Iv> warm;
		const uint64_t cap = 1ull << 22, space = 1ull << 32;
		uint64_t used = 0;

		for (size_t k = 0; k < rt.size(); k++) {
			const uint32_t d = routes[num_routes - 1 - k].depth;
			const uint64_t n = 1ull << (32u - d), a = rt[k].x;
			/* the key sequence a, a + 1, ... as at most two segments */
			const uint64_t seg[2][3] = {{a, std::min(a + n, space), 0},
						    {0, a + n > space ? a + n - space : 0, space - a}};
			uint64_t dup = n;

			for (const Iv &w : warm)
				for (const auto &g : seg) {
					const uint64_t lo = std::max(g[0], w.lo), hi = std::min(g[1], w.hi);

					if (lo < hi)
						dup = std::min(dup, g[2] + (lo - g[0]));
				}
			const uint64_t take = std::min(dup, cap - used);

			for (const auto &g : seg) {
				const uint64_t lo = g[0], hi = std::min(g[1], g[0] + (take > g[2] ? take - g[2] : 0));

				if (lo < hi)
					warm.push_back({lo, hi, (uint32_t)k});
			}
			used += take;
			if (take < n)
				break;
		}
		/* first list match of the route scan: the newest route whose
		 * masked compare holds (a route with host bits set never does) */
		auto scan = [&](uint32_t ip) -> uint32_t {
			for (size_t k = 0; k < rt.size(); k++)
				if ((ip & rt[k].y) == rt[k].x)
					return (uint32_t)k;
			return 0xffffffffu;
		};
		std::vector<uint64_t> pts{0u};

		for (const uint4 &r : rt) {
			pts.push_back(r.x & r.y);
			pts.push_back((uint64_t)(r.x & r.y) + (uint64_t)(~r.y) + 1u);
		}
		for (const Iv &w : warm) {
			pts.push_back(w.lo);
			pts.push_back(w.hi);
		}
		std::sort(pts.begin(), pts.end());
		pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
		while (!pts.empty() && pts.back() >= space)
			pts.pop_back();
		if (pts.size() > FWD_MAX_IV)
			return -ENOSPC;
		l1.assign(1u + 2u * pts.size(), 0u);
		l1[0] = (uint32_t)pts.size();
		for (size_t i = 0; i < pts.size(); i++) {
			uint32_t a = 0xffffffffu;
			bool hit = false;

			for (const Iv &w : warm)
				if (pts[i] >= w.lo && pts[i] < w.hi) {
					a = w.route;
					hit = true;
					break;
				}
			if (!hit)
				a = scan((uint32_t)pts[i]);
			l1[1 + 2 * i] = (uint32_t)pts[i];
			l1[2 + 2 * i] = a;
		}
	}

	if (param->mode == ODPG_FWD_LPM) {
		FibTrie t;

		/* setup_fwd_db inserts newest first (odp_l3fwd.c:154-176) */
		for (int k = (int)num_routes - 1; k >= 0; k--)
			t.add(routes[k].addr, (uint32_t)routes[k].oif_id, routes[k].depth);
		if (t.overflow)
			return -ENOSPC;
		for (uint32_t k = 0; k < FibTrie::kL1; k++)
			l1[k] = node_word(t.top[k]);
		pool.assign(FibTrie::kPool, FN_END);
		for (uint32_t k = 0; k < FibTrie::kPool; k++)
			pool[k] = node_word(t.pool[k]);
	}
	odpg_fwd_t *f = (odpg_fwd_t *)calloc(1, sizeof(*f));

	if (!f)
		return -ENOMEM;
	f->ctx = ctx;
	odpg_ctx_ref(ctx);
	f->mode = param->mode;
	f->nroutes = num_routes;
	f->num_ports = param->num_ports;
	if (rt.empty()) {
		rt.push_back(make_uint4(0u, 0u, 0u, 0u));
		rm.push_back(make_uint4(0u, 0u, 0u, 0u));
	}
	int rc = upload(ctx, rt, &f->d_routes);

	if (!rc)
		rc = upload(ctx, rm, &f->d_rmac);
	if (!rc)
		rc = upload(ctx, pm, &f->d_pmac);
	if (!rc)
		rc = upload(ctx, l1, &f->d_l1);
	if (!rc)
		rc = upload(ctx, pool, &f->d_pool);
	if (rc) {
		odpg_fwd_destroy(f);
		return rc;
	}
	*out = f;
	return 0;
}

extern "C" void odpg_fwd_destroy(odpg_fwd_t *f)
{
	if (!f)
		return;
	void *bufs[] = {f->d_routes, f->d_rmac, f->d_pmac, f->d_l1, f->d_pool};

	for (void *b : bufs)
		if (b)
			odpg_dev_free(f->ctx, b);
	odpg_ctx_unref(f->ctx);
	free(f);
}

extern "C" int odpg_l3fwd(odpg_ctx_t *ctx, const odpg_fwd_t *f, const odpg_fwd_batch_t *b,
			  int32_t *out_port)
{
	if (!ctx || !f || !b || !out_port || (b->num && !b->frames) || (b->stride & 15u) ||
	    b->stride < 16u || b->src_port < 0 || (uint32_t)b->src_port >= ODPG_FWD_MAX_PORTS)
		return -EINVAL;
	if (b->num == 0)
		return 0;
	hipStream_t s = (hipStream_t)odpg_ctx_stream(ctx);
	const uint32_t grid = (b->num + FBLOCK - 1) / FBLOCK;
	const uint32_t layer = b->error_check ? LAYER_ALL : LAYER_L4;

	if (b->stride == 64u) {
		const uint32_t ntiles = (b->num + 63u) / 64u;
		const uint32_t want = (ntiles + FWD_PBLOCK / 64u - 1u) / (FWD_PBLOCK / 64u);
		auto go = [&](const void *k) {
			const uint32_t g = odpg_resident_grid(k, FWD_PBLOCK, 0);

			return g < want ? g : want;
		};
		if (f->mode == ODPG_FWD_LPM)
			hipLaunchKernelGGL((odpg_l3fwd64_kernel<true>),
					   dim3(go((const void *)odpg_l3fwd64_kernel<true>)), dim3(FWD_PBLOCK), 0,
					   s, (uint4 *)b->frames, b->num, b->src_port, layer, f->d_rmac,
					   f->nroutes, f->d_l1, f->d_pool, f->d_pmac, out_port);
		else
			hipLaunchKernelGGL((odpg_l3fwd64_kernel<false>),
					   dim3(go((const void *)odpg_l3fwd64_kernel<false>)), dim3(FWD_PBLOCK), 0,
					   s, (uint4 *)b->frames, b->num, b->src_port, layer, f->d_rmac,
					   f->nroutes, f->d_l1, f->d_pool, f->d_pmac, out_port);
	} else
	if (b->stride == 64u)
		hipLaunchKernelGGL((odpg_l3fwd_kernel<64, false>), dim3(grid), dim3(FBLOCK), 0, s,
				   b->frames, b->stride, b->num, b->src_port, layer, f->mode,
				   f->d_routes, f->d_rmac, f->nroutes, f->d_l1, f->d_pool, f->d_pmac,
				   out_port);
	else if (b->stride <= 128u)
		hipLaunchKernelGGL((odpg_l3fwd_kernel<128, false>), dim3(grid), dim3(FBLOCK), 0, s,
				   b->frames, b->stride, b->num, b->src_port, layer, f->mode,
				   f->d_routes, f->d_rmac, f->nroutes, f->d_l1, f->d_pool, f->d_pmac,
				   out_port);
	else
		hipLaunchKernelGGL((odpg_l3fwd_kernel<128, true>), dim3(grid), dim3(FBLOCK), 0, s,
				   b->frames, b->stride, b->num, b->src_port, layer, f->mode,
				   f->d_routes, f->d_rmac, f->nroutes, f->d_l1, f->d_pool, f->d_pmac,
				   out_port);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
