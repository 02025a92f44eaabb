/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Lean gfx950 classify kernel for descriptor (IMIX) batches: frames of any
 * length at (offset, len) descriptors (or a fixed stride, the descriptor
 * computed: the C2x launches), a hybrid hash-walk table in its
 * hit-map form (TBL_XMASK, cls_compile.cpp), verdict words only. The C3
 * shape: IMIX 64/570/1518-byte IPv4 / IPv6 UDP / TCP traffic with the RX
 * checksum checks and a 256-PMR DAG. Same per-packet semantics as
 * odpg_classify_kernel (classify.hip), bit-identical results
 * (tests/test_gf_kernel.py, tests/test_gpu_parity.py).
 *
 * Per packet: parse + RX checksum verdicts (_odp_packet_parse_common,
 * odp_parse_internal.h:80-112, odp_packet.c:1906-1984), error-CoS selection
 * and the match_pmr_cos first-match walk (odp_classification.c:1599-1701).
 *
 * Layout: one lane per packet, one wave per 64-packet tile, waves persistent
 * over tiles, no workgroup barrier in the loop. A lane's first 64 frame bytes
 * arrive as 4 x 16-byte loads straight into registers (plus the dword at
 * byte 64), the next tile's issued while the current tile walks. A wave whose
 * frames are all plain Eth / IPv4 (no options) or IPv6 (no extension header)
 * UDP / TCP frames of >= 64 bytes parses them from the registers at
 * per-lane L4 offsets 34 / 54 (v_dot2 sums for the header and pseudo-header
 * checksums); any other wave runs the generic parse over an LDS copy of the
 * windows. The UDP / TCP checksum bytes past the window are summed by the
 * whole wave in balanced 64-byte units (seg_tail_sums4, pkt_parse.h).
 *
 * The walk: the packet's hit map (<= 256 PMRs, 8 registers) holds every
 * PMR that matches it. Each walk group (single-word PMRs sharing slot, gate
 * and mask) is read once per packet: its masked key word hashes
 * collision-free to the group's entry for that value, whose map of the PMRs
 * (of every CoS) comparing equal to it is ORed in. A level of
 * match_pmr_cos is then the lowest set bit of the current CoS's rule range
 * [rule_start, rule_start + nrule), the CoS's complex PMRs below that one
 * evaluated in rule order from their LDS term records, and one LDS read of
 * the winner's destination, mark and the destination's ranges.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>

#include "../../include/odpg.h"
#include "odpg_internal.h"
#include "pkt_parse.h"
#include "cls_match.h"

/* the register parse combines its compares with bitwise & / | on purpose
 * (branch-free: plain_gf, parse_fast_gf) */
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"

#ifndef GF_BLOCK            /* threads per workgroup */
#define GF_BLOCK 256
#endif
#ifndef GF_WAVES            /* waves per SIMD the launch bounds ask for: */
#define GF_WAVES 5          /* verdict-only launches with 2-word hit maps */
#endif
#ifndef GF_WAVES_WIDE       /* wider hit maps, counted launches (C3: 100.7 vs */
#define GF_WAVES_WIDE 4     /* 106.0 us at 5, whose VGPR budget spills) */
#endif
#ifndef GF_WAVES_CNT        /* counted launches with 2-word hit maps */
#define GF_WAVES_CNT 5
#endif
/* counted launches: the counter row read at the start is held in registers
 * until the flush (C3 counted 99.4-99.6 vs 99.9-100.4 us) where the VGPR
 * budget allows; at 5 waves (2-word maps) it spills (C2x 49.7 vs 48.8 us)
 * and the row goes through LDS at the start */
#define GF_ROW_REGS(nw) ((nw) > 2)
#define GF_WAVES_OF(cm, nw) ((nw) == 2 ? ((cm) == 0 ? GF_WAVES : GF_WAVES_CNT) : GF_WAVES_WIDE)
#ifndef GF_WAVES_S64W       /* fixed 64-byte stride launches (S64) */
#define GF_WAVES_S64W 6
#endif
#ifndef GF_WAVES_S64C       /* ... counted */
#define GF_WAVES_S64C 6
#endif
#define GF_WAVES_S64(cm, nw) ((nw) == 2 ? ((cm) == 0 ? GF_WAVES_S64W : GF_WAVES_S64C) : GF_WAVES_WIDE)
#ifndef GF_RW               /* LDS row stride per lane, dwords (16-byte multiple) */
#define GF_RW 20
#endif

struct GFArgs {
	const uint8_t *frames;
	uint32_t num;
	uint32_t stride;            /* fixed-stride batch (descs unused), or 0 */
	uint32_t opt;               /* ODPG_PKTIN_* (all defined bits are < 32) */
	uint32_t ngroups;           /* hit-map groups (descriptors in xmg) */
	uint32_t num_cos;
	int32_t default_cos, error_cos;
	const dcos_t *coses;
	const uint32_t *xlds;       /* the table's LDS part (xm_layout_t) */
	xm_layout_t L;
	const uint32_t *xfc;        /* lazy form: per CoS first complex record | count << 16 */
	uint32_t num_xflat;         /* lazy form: complex records */
	odpg_cnt_dev cnt;           /* CM 2: the sharded counters' layout, by value */
	uint32_t cnt_words;         /* CM 2: words of a counter row */
};

/* sharded-counter histogram bins before the CoS bins (CM 2) */
#define GF_BIN_ERR    0u
#define GF_BIN_PDROP  1u
#define GF_BIN_NOCOS  2u
#define GF_BIN_DROP   3u
#define GF_BIN_EXTRA  4u

typedef unsigned short gf_us2 __attribute__((ext_vector_type(2)));
/* key slots 0..15 of a packet, indexed by a wave-uniform slot (v_movrels) */
typedef uint32_t gf_kv_t __attribute__((ext_vector_type(16)));

/* acc + w.lo * x.lo16 + w.hi * x.hi16 (one v_dot2_u32_u16) */
__device__ __forceinline__ uint32_t gd2(uint32_t x, uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(gf_us2, x), __builtin_bit_cast(gf_us2, w),
				      acc, false);
}

#define GW11 0x00010001u   /* both halves */
#define GW10 0x00000001u   /* low half (first byte pair) */
#define GW01 0x00010000u   /* high half */

/* 0xffff iff the one's-complement sum of the 16-bit halves is all-ones,
 * as chksum_finalize folds the reference's 64-bit word sum
 * (odp_chksum_internal.h:22-31) */
__device__ __forceinline__ uint32_t gfold(uint32_t s)
{
	return oc_fold(s);
}

/* frame bytes [K, K + 4) of the window registers, K constant */
template <int K>
__device__ __forceinline__ uint32_t wb(const uint32_t (&f)[16])
{
	return fw<K>(f);
}

/* Tag dwords of a frame (0 untagged; 1 one VLAN tag, or a QinQ outer tag
 * alone; 2 a QinQ outer tag and a VLAN tag) and whether the outer one is a
 * QinQ tag, as _odp_parse_eth walks them (odp_parse.c:23-106: an 0x88A8 tag,
 * then an 0x8100 tag). */
__device__ __forceinline__ uint32_t tag_dwords(const uint32_t (&f)[16], bool &qinq)
{
	const uint32_t e0 = f[3] & 0xffffu;

	qinq = e0 == 0xa888u;
	if (qinq)
		return (f[4] & 0xffffu) == 0x0081u ? 2u : 1u;
	return e0 == 0x0081u ? 1u : 0u;
}

/* The frames the register parse takes, on the tag-shifted window (g[k] =
 * frame dword k + sh for k >= 3, so the L3 header sits at byte 14 as in an
 * untagged frame; x16 stands in for the dword past the window): Eth (no
 * SNAP) with up to two tags, then IPv4 with IHL 5 and tot_len within the
 * frame, or IPv6 (at most one tag) without extension headers and payload
 * within the frame; then UDP with length >= 8 (IPv6: not port 4500, whose
 * IPsec marker lies past the window) or TCP with data offset >= 5 and its
 * 20 header bytes inside the frame (IPv6: untagged); frame length >= 64.
 * x16 is the frame's dword at byte 64 (the IPv6 TCP data-offset byte). */
__device__ __forceinline__ bool plain_gf(const uint32_t (&f)[16], uint32_t x16, uint32_t len,
					 uint32_t sh)
{
	/* branch-free: compares combined with & / | (a wave mixes IPv4 / IPv6
	 * and UDP / TCP frames; divergent ifs ran both sides with exec-mask
	 * bookkeeping around each) */
	const uint32_t et = f[3] & 0xffffu;
	const uint32_t vb = (f[3] >> 16) & 0xffu;
	const uint32_t l3 = 14u + 4u * sh;
	const uint32_t room = len - l3;             /* bytes from the L3 header on */
	const bool v4 = (et == 0x0008u) & (vb == 0x45u) & (swap16(f[4] & 0xffffu) <= room);
	const bool v6 = (et == 0xdd86u) & ((vb & 0xf0u) == 0x60u) & (sh <= 1u) &
			(swap16(f[4] >> 16) + 40u <= room);
	/* IPv4 with IHL 5: protocol byte 23, UDP length at 38, TCP data offset
	 * at 46; IPv6: next header byte 20, UDP length at 58, port at 56, TCP
	 * data offset past the window (x16) */
	/* both versions' fields computed, then selected (a ?: with a call in
	 * an arm is emitted as a branch, which stays one in divergent code) */
	const uint32_t proto4 = f[5] >> 24, proto6 = f[5] & 0xffu;
	const uint32_t proto = v6 ? proto6 : proto4;
	const uint32_t uw = v6 ? f[14] : f[9];
	const uint32_t ulen = swap16(uw >> 16), uport = swap16(uw & 0xffffu);
	const bool udp_ok = (proto == 0x11u) & (ulen >= 8u) & !(v6 & (uport == 4500u));
	const uint32_t doff4 = (f[11] >> 20) & 0xfu, doff6 = (x16 >> 20) & 0xfu;
	const uint32_t doff = v6 ? doff6 : doff4;
	const bool tcp_ok = (proto == 0x06u) & (doff >= 5u) & !(v6 & ((sh != 0u) | (len < 74u)));

	return (len >= 64u) & (v4 | v6) & (udp_ok | tcp_ok);
}

/* parse_common() of a plain_gf() frame from its tag-shifted window
 * registers: returns 0 / 1 (error flagged) or PARSE_PEND with the UDP / TCP
 * checksum left for the tail bytes [64, len) (pd: the pseudo header + window
 * part). s14 / s15: g[14] / g[15] as the window sums take them (zero where
 * they hold bytes past the frame's byte 64, which the tail pass sums).
 * Branch-free over IPv4 / IPv6 and UDP / TCP: the pseudo-header addresses
 * and the segment are one contiguous byte range of the window ([26, 64) for
 * IPv4, [22, 64) for IPv6), so the L4 sum is one v_dot2 chain whose first two
 * weights depend on the version. The ip_err / pending / IPsec results stay
 * behind (uniform-heavy) ifs: computing every arm and selecting made the
 * 8-word-map instantiation (C3, 128 VGPRs) spill one register, 6 for the
 * counted one, whose scratch traffic took C3 from 404 to 410 MB per launch;
 * the fixed-stride instantiation compiles the same either way. */
__device__ __forceinline__ int parse_fast_gf(Prs &p, L4Pend &pd, const uint32_t (&f)[16],
					     uint32_t s14, uint32_t s15, uint32_t len, uint32_t opt,
					     uint32_t sh, bool qinq)
{
	const bool v6 = (f[3] & 0xffffu) == 0xdd86u;
	const uint32_t l3 = 14u + 4u * sh;
	/* input flags, low and high words (the checksum-done / zero bits are
	 * >= 32) */
	uint32_t lo = (uint32_t)(IF(IFL_L2) | IF(IFL_ETH) | IF(IFL_L3) | IF(IFL_L4)) |
		      (v6 ? (uint32_t)IF(IFL_IPV6) : (uint32_t)IF(IFL_IPV4)) |
		      (sh ? (uint32_t)IF(IFL_VLAN) : 0u) | (qinq ? (uint32_t)IF(IFL_VLAN_QINQ) : 0u) |
		      (len > 1514u ? (uint32_t)IF(IFL_JUMBO) : 0u) |
		      ((f[0] & 0x1u) ? (uint32_t)IF(IFL_ETH_MCAST) : 0u) |
		      (((f[0] == 0xffffffffu) & ((f[1] & 0xffffu) == 0xffffu)) ? (uint32_t)IF(IFL_ETH_BCAST) : 0u);
	uint32_t hi = 0u;

	/* parse_ipv4 (odp_parse.c:113-169): the header checksum over bytes
	 * 14..33; a bad one is ip_err (no L4 parse, no L4 flag) */
	const bool ck3 = !v6 & ((opt & ODPG_PKTIN_IPV4_CHKSUM) != 0u);
	uint32_t hs = gd2(f[3], GW01, 0u);

	hs = gd2(f[4], GW11, hs);
	hs = gd2(f[5], GW11, hs);
	hs = gd2(f[6], GW11, hs);
	hs = gd2(f[7], GW11, hs);
	hs = gd2(f[8], GW10, hs);
	const bool l3bad = ck3 & (gfold(hs) != 0xffffu);

	hi |= ck3 ? (uint32_t)(IF(IFL_L3_CHKSUM_DONE) >> 32) : 0u;
	const uint32_t lo3 = lo, hi3 = hi;          /* what an ip_err frame keeps */

	const bool frag = !v6 & ((swap16(f[5] & 0xffffu) & 0x3fffu) != 0u);
	const uint32_t dst_be = __builtin_bswap32(wb<30>(f));
	const bool mc = v6 ? ((f[9] >> 16) & 0xffu) == 0xffu : (dst_be >> 28) == 0xeu;

	lo |= (frag ? (uint32_t)IF(IFL_IPFRAG) : 0u) |
	      ((!v6 & (dst_be == 0xffffffffu)) ? (uint32_t)IF(IFL_IP_BCAST) : 0u) |
	      (mc ? (uint32_t)IF(IFL_IP_MCAST) : 0u);
	const uint32_t proto = v6 ? (f[5] & 0xffu) : (f[5] >> 24);
	/* bytes [26, 64) (IPv4: addresses 26..33, segment 34..) or [22, 64)
	 * (IPv6: addresses 22..53, segment 54..) */
	uint32_t sum = gd2(f[5], v6 ? GW01 : 0u, 0u);

	sum = gd2(f[6], v6 ? GW11 : GW01, sum);
#pragma unroll
	for (int k = 7; k < 14; ++k)
		sum = gd2(f[k], GW11, sum);
	sum = gd2(s15, GW11, gd2(s14, GW11, sum));
	const uint32_t uw = v6 ? f[14] : f[9];              /* UDP ports + length */
	const uint32_t ulen_raw = uw >> 16;
	const uint32_t csum_raw = (v6 ? f[15] : f[10]) & 0xffffu;
	const uint32_t l4 = l3 + (v6 ? 40u : 20u);
	const bool udp = proto == 0x11u;

	lo |= udp ? (uint32_t)IF(IFL_UDP) : (uint32_t)IF(IFL_TCP);
	/* parse_udp / parse_tcp (odp_parse.c:252-322) */
	const bool udpck = udp & ((opt & ODPG_PKTIN_UDP_CHKSUM) != 0u) & !frag;
	const bool tcpck = !udp & ((opt & ODPG_PKTIN_TCP_CHKSUM) != 0u) & !frag;
	const bool zero = udpck & (csum_raw == 0u);
	uint32_t fl = (zero & v6) ? FB(FL_L4_CHKSUM_ERR) : 0u;

	hi |= zero ? (uint32_t)((IF(IFL_L4_CHKSUM_DONE) | IF(IFL_UDP_CHKSUM_ZERO)) >> 32) : 0u;
	/* the IPsec-over-UDP marker (port 4500, a non-zero SPI at byte 42) */
	if (!v6 & udp & (swap16(uw & 0xffffu) == 4500u) & (swap16(ulen_raw) > 4u) & (wb<42>(f) != 0u)) {
		lo |= (uint32_t)IF(IFL_IPSEC);
		hi |= (uint32_t)(IF(IFL_IPSEC_UDP) >> 32);
	}
	const bool need = (udpck & !zero) | tcpck;

	sum += udp ? ulen_raw + (0x11u << 8) : swap16((len - l4) & 0xffffu) + (0x06u << 8);
	const bool pend = need & (len > 64u);
	/* _odp_packet_l4_chksum (odp_packet.c:1906-1984) within the window */
	const bool done = need & !pend;
	const bool bad = done & (gfold(sum) != 0xffffu);

	hi |= done ? (uint32_t)(IF(IFL_L4_CHKSUM_DONE) >> 32) : 0u;
	fl |= bad ? FB(FL_L4_CHKSUM_ERR) | (udp ? FB(FL_UDP_ERR) : FB(FL_TCP_ERR)) : 0u;
	/* the results by select (an early return for ip_err compiled to a
	 * divergent branch with the rest sunk into it) */
	p.l2 = 0u;
	p.l3 = l3;
	if (l3bad) {
		p.inf = ((uint64_t)hi3 << 32) | (lo3 & ~(uint32_t)IF(IFL_L4));
		p.fl = FB(FL_IP_ERR) | FB(FL_L3_CHKSUM_ERR);
		p.l4 = 0xffffu;
		return 1;
	}
	p.inf = ((uint64_t)hi << 32) | lo;
	p.fl = fl;
	p.l4 = l4;
	if (pend) {
		pd.kind = udp ? 1u : 2u;
		pd.sum = sum;
		pd.a = 64u;
		pd.b = len;
		return PARSE_PEND;
	}
	return (fl & FL_ERROR_MASK) != 0u;
}

#ifndef GF_PROBES           /* chain-free groups probed together (2-word maps) */
#define GF_PROBES 2
#endif

/* a packet's key words 16, 17 (L4 + 0, 4) and 18 (frame length) */
typedef uint32_t gf_kx_t __attribute__((ext_vector_type(4)));

/* U hit-map groups' probes for this lane's packet, branch-free: each masked
 * key word hashed to its group's direct entry (cls_compile.cpp
 * "TBL_XMASK"), whose value and bit map are read together; m[u] = the
 * entry's map and hk[u] all-ones when the value, the group's gate and (G)
 * its CUSTOM_L3 / CUSTOM_FRAME length guard (len >= (l3 & l3mask) +
 * threshold) hold, else 0 (an empty slot's map is 0 too). All U
 * descriptors are loaded first and all LDS reads issued together: scalar
 * and LDS loads share one counter, so a descriptor load issued behind a
 * probe's reads would wait for them. Key words by value, read with a
 * wave-uniform index (v_movrels): the group's word of the 16-word key
 * vector, or (KX: the table reads more than 16 slots) its slot, 16..18
 * selected from kx. The hit test is one compare of (gate & ~inf) |
 * (value ^ key) with zero, in vector registers (ninf = ~input flags).
 * 2-word maps: the entry {map0, map1, value, 0} is one ds_read_b128. */
template <int NW, int U, bool KX, bool G>
__device__ __forceinline__ void gf_probes(const uint4 *__restrict__ xmg, uint32_t gi, gf_kv_t kv,
					  gf_kx_t kx, uint32_t ninf, uint32_t l3, uint32_t len,
					  const uint32_t *tb, const xm_layout_t &L, uint32_t (&m)[U][NW],
					  uint32_t (&hk)[U])
{
	uint4 q0[U], q1[U];
	uint32_t e[U], kvm[U], v[U];

#pragma unroll
	for (int u = 0; u < U; ++u) {
		q0[u] = xmg[4u * (gi + u)];        /* mul, shift, key index, entry base */
		q1[u] = xmg[4u * (gi + u) + 1u];   /* guard, gate, mask, L3 mask */
	}
#pragma unroll
	for (int u = 0; u < U; ++u) {
		uint32_t key;

		if constexpr (KX) {
			const uint32_t sl = q0[u].z & 0xffu;

			key = sl < 16u ? kv[sl & 15u] : kx[sl & 3u];
		} else {
			key = kv[q0[u].z & 15u];
		}
		kvm[u] = key & q1[u].z;
		const uint32_t h = (kvm[u] * q0[u].x) >> q0[u].y;

		/* 2-word maps: the entry's byte offset as one shift-add of the
		 * hash onto the base scaled on the scalar unit (written as asm:
		 * the compiler otherwise adds first and shifts the sum, one more
		 * vector instruction per probe; s_mul_i32, unlike s_lshl_b32,
		 * leaves SCC alone, which the compiler may hold across it) */
		if constexpr (NW == 2) {
			uint32_t wb;

			asm("s_mul_i32 %0, %1, 16" : "=s"(wb) : "s"(q0[u].w));
			e[u] = (h << 4) + wb;
		} else {
			e[u] = q0[u].w + h;
		}
	}
#pragma unroll
	for (int u = 0; u < U; ++u) {
		if constexpr (NW == 2) {
			/* whole ds_read_b128 (the unused fourth word kept: narrowed
			 * to ds_read_b96 it takes twice the LDS cycles) */
			const uint4 x = *(const uint4 *)((const uint8_t *)tb + e[u]);

			asm volatile("" ::"v"(x.w));

			m[u][0] = x.x;
			m[u][1] = x.y;
			v[u] = x.z;
		} else {
			v[u] = tb[L.values + e[u]];
#pragma unroll
			for (int q = 0; q < NW; q += 4) {
				const uint4 x = *(const uint4 *)(tb + L.masks + NW * e[u] + q);

				m[u][q] = x.x;
				m[u][q + 1] = x.y;
				m[u][q + 2] = x.z;
				m[u][q + 3] = x.w;
			}
		}
	}
#pragma unroll
	for (int u = 0; u < U; ++u) {
		bool hit = ((q1[u].y & ninf) | (v[u] ^ kvm[u])) == 0u;

		if constexpr (G)
			hit = hit & (len >= (l3 & q1[u].w) + q1[u].x);
		/* all-ones on a hit: the callers fold it into their OR / AND
		 * (v_and_or_b32) instead of a select per word */
		hk[u] = 0u - (uint32_t)hit;
	}
}

/* CM: counters of the launch, 0 none, 2 sharded counter rows (odpg.h);
 * NW: hit-map words per packet (the table's rule bits, 2 / 4 / 8 x 32);
 * S64: a fixed 64-byte stride (the C2x launches): every frame is its 64-byte
 * window, loaded as the lean 64-byte kernel does (coalesced nontemporal
 * 16-byte loads, 1 KiB of contiguous lines per instruction, transposed to
 * one frame per lane through the wave's LDS rows), no descriptors and no
 * checksum tail pass; KX: the table's groups read more than 16 key slots
 * (slots 16..18 selected per probe, gf_probes) */
template <int CM, int NW, bool S64, bool KX>
__global__ __launch_bounds__(GF_BLOCK) __attribute__((amdgpu_waves_per_eu(S64 ? GF_WAVES_S64(CM, NW) : GF_WAVES_OF(CM, NW)))) void
odpg_clsgf_kernel(const GFArgs A, const uint4 *__restrict__ xmg, const uint32_t *__restrict__ xhdr,
		  const odpg_desc_t *__restrict__ descs, odpg_out_t *__restrict__ out)
{
	/* read-only tables as restrict kernel arguments: their wave-uniform
	 * reads compile to scalar loads */
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	/* generic-parse LDS row (dwords): GF_RW 16 packs the rows; 20 (80 B,
	 * still 16-byte aligned) spreads a wave's reads of one row offset over
	 * 8 banks instead of 2 */
	constexpr uint32_t RW = GF_RW;
	uint32_t *row = smem + threadIdx.x * RW;
	/* CM 2: the workgroup's histogram after the rows (odpg.h "sharded
	 * counters"): four bins, then one per CoS */
	uint32_t *dlv = smem + GF_BLOCK * RW;
	const uint32_t nbins = CM == 2 ? ((A.num_cos + GF_BIN_EXTRA + 3u) & ~3u) : 0u;
	/* the table's LDS part (odpg_internal.h xm_layout_t): entry bit maps,
	 * their values, the groups' slot bytes, per CoS {bit range, action},
	 * per rule bit {dst | mark << 16, the destination's bit range, the
	 * destination's complex records (lazy form): first | count << 16, 0},
	 * the lazy form's complex records {gate, mask, value, slot | guard end <<
	 * 8 | absolute << 30 | guarded << 31}, {pmr bit, last record of its
	 * chain, that record's index, 0} */
	uint32_t *tb = dlv + nbins;
	const uint2 *xci = (const uint2 *)(tb + A.L.xci);
	const uint4 *pdst = (const uint4 *)(tb + A.L.xpd);
	const uint4 *xfl = (const uint4 *)(tb + A.L.xflat);
	/* CM 2: the workgroup's counter row as it stood before this launch
	 * (read at the start; the flush stores row + histogram) */
	unsigned long long *base = (unsigned long long *)(tb + ((A.L.lds_words + 1u) & ~1u));
	/* the wave's 64-dword scratch of the tail pass's owner map
	 * (seg_tail_sums4) */
	uint32_t *marks = tb + ((A.L.lds_words + 1u) & ~1u) + (CM == 2 ? 2u * A.cnt_words : 0u) +
			  (threadIdx.x >> 6) * 64u;

	const uint32_t lane = __lane_id();
	/* line-shaped window loads of descriptor batches (load_win) */
	constexpr bool XW = NW > 2 && !S64;
	/* the window chunks go through the frames' LDS rows at the tile start */
	constexpr bool STG = XW || S64;
	const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (GF_BLOCK / 64) +
							   (threadIdx.x >> 6));
	const uint32_t nwaves = gridDim.x * (GF_BLOCK / 64);
	const uint32_t ntiles = (A.num + 63u) >> 6;
	const uint32_t num = A.num;

	/* the first tile's descriptors and windows are issued before the table
	 * copy below */
	auto load_desc = [&](uint32_t t) __attribute__((always_inline)) -> uint2 {
		const uint32_t i = t * 64u + lane;

		if constexpr (S64)
			return make_uint2(0u, 0u);   /* unused: (64 i, 64) */
		if (t < ntiles && i < num)
			return A.stride ? make_uint2(i * A.stride, A.stride) : *(const uint2 *)(descs + i);
		return make_uint2(0u, 0u);
	};
	/* S64: tile t's 4 KiB as 4 coalesced nontemporal loads (lane l: chunks
	 * l, l + 64, l + 128, l + 192 of the tile, i.e. frame 16 q + l / 4, part
	 * l % 4), clamped to the batch's last chunk (the lean 64-byte kernel's
	 * load_raw, classify64.hip) */
	auto load_tile = [&](uint32_t (&f)[16], uint32_t t) __attribute__((always_inline)) {
		if (t >= ntiles)
			return;
		const uint32_t lim = num * 4u - 1u;
		const uint32_t c0 = t * 256u + lane;

#pragma unroll
		for (int q = 0; q < 4; ++q) {
			const uint4 x = ld_nt16((const uint4 *)A.frames + min(c0 + 64u * q, lim));

			f[4 * q + 0] = x.x;
			f[4 * q + 1] = x.y;
			f[4 * q + 2] = x.z;
			f[4 * q + 3] = x.w;
		}
	};
	/* a frame's first 64 bytes (16-byte chunks holding frame bytes only: the
	 * chunk with the last byte is masked), and its dword at byte 64. Wide
	 * hit maps (NW > 2, the C3 launches): line-shaped, instruction k loads
	 * frames 16k .. 16k + 15 of the tile, four lanes a frame (its 16-byte
	 * chunk lane & 3), so that one instruction touches 16 lines instead of
	 * 64 (TA / L1 request slots, not bytes, bound the C3 loads: 98.6 ->
	 * 92.9 us with the tail passes' line-shaped loads); the tile loop puts
	 * the chunks through the frames' LDS rows. The 2-word instantiation
	 * (C2x) keeps lane-per-frame loads: it has no registers for the
	 * transposition (45.0 vs 39.7 us, spilled) */
	auto load_win = [&](uint32_t (&f)[16], uint32_t &x16, uint2 d) __attribute__((always_inline)) {
		if constexpr (XW) {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				const uint32_t src = 16u * k + (lane >> 2), c = lane & 3u;
				const uint32_t off = lane_pull(d.x, src), ln = lane_pull(d.y, src);
				uint4 x = make_uint4(0u, 0u, 0u, 0u);

				if (16u * c < ln)
					x = *(const uint4 *)(A.frames + off + 16u * c);
				f[4 * k + 0] = x.x;
				f[4 * k + 1] = x.y;
				f[4 * k + 2] = x.z;
				f[4 * k + 3] = x.w;
			}
		} else {
#pragma unroll
			for (int q = 0; q < 4; ++q) {
				uint4 x = make_uint4(0u, 0u, 0u, 0u);

				if (16u * q < d.y)
					x = *(const uint4 *)(A.frames + d.x + 16u * q);
				f[4 * q + 0] = x.x;
				f[4 * q + 1] = x.y;
				f[4 * q + 2] = x.z;
				f[4 * q + 3] = x.w;
			}
		}
		x16 = d.y > 64u ? *(const uint32_t *)(A.frames + d.x + 64u) : 0u;
	};
	uint32_t fn[16] = {}, xn = 0u;
	uint2 dn = load_desc(gw), dnn;
	/* The tails of a tile's frames, bytes [64, len), as each lane's
	 * one's-complement partial (seg_tail_sums4; the whole wave), summed one
	 * tile ahead (every frame's, whether or not its parse will want them),
	 * right after the tile's windows are issued: a 128-byte line shared by
	 * a window and a tail unit is then requested twice within a short time
	 * instead of a tile apart, when the L2 has let it go (tails summed in
	 * their own tile read 1.24x the algorithmic bytes) */
	const bool l4ck = (A.opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM)) != 0u;
	auto early_tails = [&](uint2 d, uint32_t t) __attribute__((always_inline)) -> uint32_t {
		const uint32_t len = t < ntiles && t * 64u + lane < num ? d.y : 0u;
		const uint64_t m = __ballot(len > 64u);

		if (!m)
			return 0u;
		const L4Pend q = {0u, 0u, 64u, len};

		return seg_tail_sums4<XW>(m, A.frames + d.x, q, marks);
	};
	uint32_t tn = 0u;

	if constexpr (S64) {
		load_tile(fn, gw);
	} else {
		load_win(fn, xn, dn);
		if (l4ck)
			tn = early_tails(dn, gw);
		dnn = load_desc(gw + nwaves);
	}

	for (uint32_t k = threadIdx.x; k < A.L.lds_words; k += GF_BLOCK)
		tb[k] = A.xlds[k];
	/* CM 2: the counter layout is read now, not behind the tile loop's
	 * last wait; the workgroup's last wave to finish flushes the histogram */
	__shared__ uint32_t waves_done;
	__shared__ odpg_cnt_dev cnt_lds;
	unsigned long long rowv = 0ull;   /* CM 2: this thread's word of the row */
	__shared__ unsigned long long octets;
	if constexpr (CM == 2) {
		/* the layout (a kernel argument) is kept in LDS for the flush:
		 * nothing of it is held through the tile loop (scalar registers) */
		const odpg_cnt_dev C = A.cnt;

		if (threadIdx.x == 0u)
			cnt_lds = C;
		const __attribute__((address_space(1))) unsigned long long *r0 =
			(const __attribute__((address_space(1))) unsigned long long *)(uintptr_t)(C.rows + (size_t)blockIdx.x * C.words);

		if (GF_ROW_REGS(NW) && C.words <= GF_BLOCK) {
			/* one word per thread, held in registers until the flush:
			 * nothing waits for the row before the tile loop */
			if (threadIdx.x < C.words)
				rowv = r0[threadIdx.x];
		} else {
			for (uint32_t k = threadIdx.x; k < C.words; k += GF_BLOCK)
				base[k] = r0[k];
		}
		for (uint32_t k = threadIdx.x; k < nbins; k += GF_BLOCK)
			dlv[k] = 0u;
		if (threadIdx.x == 0u) {
			waves_done = 0u;
			octets = 0ull;
		}
	}

	__syncthreads();

	const uint32_t ngroups = A.ngroups;
	const uint32_t opt = A.opt;
	const bool def_valid = A.default_cos >= 0 && A.coses[A.default_cos].valid;
	const bool def_rules = def_valid && A.coses[A.default_cos].nrule != 0u;
	/* the chain bits (they start set, groups clear them), uniform */
	uint32_t chain[NW];
	/* the key slots the groups read; the key-vector words of slots 16..18
	 * (0xff: none); the group order (odpg_internal.h XM_HDR_WORDS) */
	const uint32_t kslots = xhdr[6];
	const uint32_t kpos = xhdr[4];
	const uint32_t gcut = xhdr[7];

#pragma unroll
	for (int w = 0; w < NW; ++w)
		chain[w] = xhdr[8 + w];

	for (uint32_t t = gw; t < ntiles; t += nwaves) {
		const uint32_t i = t * 64u + lane;
		const bool live = i < num;
		const uint2 d = S64 ? make_uint2(i * 64u, 64u) : dn;
		const uint32_t tsum = tn;       /* this tile's tails [64, len) */
		const uint8_t *g = A.frames + d.x;
		const uint32_t len = live ? d.y : 0u;
		uint32_t f[16];
		uint32_t x16 = S64 ? 0u : xn;
		uint32_t tile_oct = 0u;  /* CM 2: octets this lane hands over */
		if constexpr (STG) {
			/* the staged chunks into the frames' rows, then each lane's
			 * own row back (a wave's LDS operations complete in order) */
			uint32_t *wrow = smem + (threadIdx.x - lane) * RW;

#pragma unroll
			for (int k = 0; k < 4; ++k)
				*(uint4 *)(wrow + (16u * k + (lane >> 2)) * RW + 4u * (lane & 3u)) =
					make_uint4(fn[4 * k], fn[4 * k + 1], fn[4 * k + 2], fn[4 * k + 3]);
			__asm__ volatile("" ::: "memory");
#pragma unroll
			for (int q = 0; q < 16; q += 4) {
				const uint4 x = *(const uint4 *)(row + q);

				fn[q] = x.x;
				fn[q + 1] = x.y;
				fn[q + 2] = x.z;
				fn[q + 3] = x.w;
			}
		}

		if (!S64 && __ballot(live && len < 64u)) {
#pragma unroll
			for (int q = 0; q < 16; ++q) {
				/* bytes past the frame read as zero (the reference's
				 * undefined reads past the end: DESIGN.md deviation 1) */
				const int nb = (int)len - 4 * q;

				f[q] = nb >= 4 ? fn[q] : nb <= 0 ? 0u : fn[q] & ((1u << (8 * nb)) - 1u);
			}
		} else {
			/* no live frame shorter than the window (dead lanes' bytes
			 * are never used) */
#pragma unroll
			for (int q = 0; q < 16; ++q)
				f[q] = fn[q];
		}
		if constexpr (!S64)
			dn = dnn;

		/* ---- parse + checksum verdicts -------------------------------- */
		Prs p;
		L4Pend pd = {0u, 0u, 0u, 0u};
		int ret = 0;
		Bases b;
		uint32_t hm[NW];

		p.inf = 0ull;
		p.fl = 0u;
		p.l2 = p.l3 = p.l4 = 0xffffu;
		/* the LDS row: the generic parse's window, and the key reads of
		 * the generic waves (unshifted frame bytes; S64: the staged row
		 * already holds them) */
		if constexpr (!S64) {
#pragma unroll
			for (int q = 0; q < 16; q += 4)
				*(uint4 *)(row + q) = make_uint4(f[q], f[q + 1], f[q + 2], f[q + 3]);
		}
		/* VLAN / QinQ frames: the window shifted by the tag dwords, so that
		 * the register parse reads their L3 / L4 headers at the untagged
		 * offsets; the L2 words and the VLAN tag are read from u3..u5 */
		const uint32_t u3 = f[3], u4 = f[4], u5 = f[5];
		bool qinq = false;
		const uint32_t sh = live ? tag_dwords(f, qinq) : 0u;
		uint32_t s14 = f[14], s15 = f[15];

		if (__ballot(sh != 0u)) {
#pragma unroll
			for (int k = 3; k < 16; ++k) {
				const uint32_t n1 = k + 1 < 16 ? f[k + 1] : x16;
				const uint32_t n2 = k + 2 < 16 ? f[k + 2] : k + 2 == 16 ? x16 : 0u;

				f[k] = sh == 0u ? f[k] : sh == 1u ? n1 : n2;
			}
			/* the bytes past the frame's byte 64 are the tail pass's */
			s14 = sh == 2u ? 0u : f[14];
			s15 = sh != 0u ? 0u : f[15];
		}
		const bool fastw = __ballot(live && !plain_gf(f, x16, len, sh)) == 0ull;

		auto bases = [&]() __attribute__((always_inline)) {
			b.l2 = p.l2;
			b.l3 = p.l3;
			b.l4 = p.l4;
			b.vlanx = 14u + ((p.inf & IF(IFL_VLAN_QINQ)) ? 4u : 0u);
			b.len = len;
			b.inf_lo = (uint32_t)p.inf;
		};
		/* the packet's key slots (odpg_internal.h "key slots"), extracted
		 * once: slots 0..15 in a register vector the groups index by their
		 * uniform slot, 16 / 17 (L4) and 18 (length) beside it */
		gf_kv_t kv = {};
		uint32_t k16 = 0u, k17 = 0u;

		if (fastw) {
			/* dead lanes too (no branch): their results are unused */
			ret = parse_fast_gf(p, pd, f, s14, s15, len, opt, sh, qinq);
			bases();
			const bool v6 = (b.inf_lo & (uint32_t)IF(IFL_IPV6)) != 0u;
			const bool l4ok = b.l4 != 0xffffu;

			/* the innermost VLAN tag */
			const uint32_t vq = __builtin_amdgcn_alignbyte(u5, u4, 2);
			const uint32_t vt = __builtin_amdgcn_alignbyte(u4, u3, 2);
			const uint32_t w34 = wb<34>(f), w38 = wb<38>(f);
			const uint32_t w54 = wb<54>(f), w58 = wb<58>(f);

			/* one vector literal: built in place (element stores into a
			 * zero vector compiled to a copy of the whole tuple) */
			kv = gf_kv_t{f[0], f[1], f[2], u3, u4, qinq ? vq : vt, wb<14>(f), wb<18>(f),
				     wb<22>(f), wb<26>(f), wb<30>(f), w34, w38, wb<42>(f), wb<46>(f),
				     wb<50>(f)};
			k16 = !l4ok ? 0u : v6 ? w54 : w34;
			k17 = !l4ok ? 0u : v6 ? w58 : w38;
		} else {
			Pkt<64, true> v;

			v.row = row;
			v.g = g;
			v.len = len;
			if (live)
				ret = parse_common(p, v, LAYER_ALL, (uint64_t)opt, S64 ? nullptr : &pd);
			bases();
			KeySrc<64, true> key;

			key.f = nullptr;
			key.v = &v;
			key.b = &b;
			key.fast = false;
			/* the slots the groups read (uniform mask) */
#pragma unroll
			for (uint32_t sl = 0; sl < 16u; ++sl)
				if ((kslots >> sl) & 1u)
					kv[sl] = key(sl);
			if ((kslots >> 16) & 1u)
				k16 = key(16u);
			if ((kslots >> 17) & 1u)
				k17 = key(17u);
		}
		if constexpr (!KX) {
			/* slots 16..18 into their key-vector words (uniform; three
			 * distinct words no group's slot < 16 uses, cls_compile.cpp) */
			kv[kpos & 15u] = k16;
			kv[(kpos >> 8) & 15u] = k17;
			kv[(kpos >> 16) & 15u] = len;
		}
		/* the hit map: each group's masked key word, once per packet.
		 * Single-word rules OR their bits in; a complex rule's chain bit
		 * (set to start with) stays set only while every group holding one
		 * of its records has it in the entry for the packet's key. The
		 * groups without chain records come first (xhdr[7] of them), each
		 * kind in a loop of its own */
		{
			const bool on = live && (p.fl & FL_ERROR_MASK) == 0u;

#pragma unroll
			for (int w = 0; w < NW; ++w)
				hm[w] = on ? chain[w] : 0u;
			const gf_kv_t kvv = kv;
			const gf_kx_t kxv = {k16, k17, (uint32_t)len, 0u};
			const uint32_t ninf = ~b.inf_lo, l3 = b.l3, flen = len;

			/* the AND-chain groups: a chain bit stays set only where
			 * every group holding one of its records has it */
			auto chain_upd = [&](uint32_t g, const uint32_t (&mm)[NW], uint32_t h) __attribute__((always_inline)) {
				const uint4 a0 = xmg[4u * g + 2u];
				const uint4 a1 = xmg[4u * g + 3u];
				const uint32_t na[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};

#pragma unroll
				for (int w = 0; w < NW; ++w) {
					const uint32_t x = mm[w] & h;

					hm[w] = (hm[w] & (x | na[w])) | (x & ~chain[w]);
				}
			};
			/* groups [lo, hi) of one kind (G: length-guarded; CH: with
			 * chain members), U probes in flight together */
			auto probe_range = [&](auto gc, auto chc, uint32_t lo, uint32_t hi) __attribute__((always_inline)) {
				constexpr bool G = decltype(gc)::value;
				constexpr bool CH = decltype(chc)::value;
				constexpr uint32_t U = CH || NW != 2 ? 2u : GF_PROBES;
				uint32_t gi = lo;

#pragma unroll 1
				for (; gi + U <= hi; gi += U) {
					uint32_t m[U][NW], hk[U];

					gf_probes<NW, U, KX, G>(xmg, gi, kvv, kxv, ninf, l3, flen, tb, A.L, m, hk);
#pragma unroll
					for (uint32_t u = 0; u < U; ++u) {
						if constexpr (CH) {
							chain_upd(gi + u, m[u], hk[u]);
						} else {
#pragma unroll
							for (int w = 0; w < NW; ++w)
								hm[w] |= m[u][w] & hk[u];
						}
					}
				}
#pragma unroll 1
				for (; gi < hi; ++gi) {
					uint32_t m[1][NW], hk[1];

					gf_probes<NW, 1, KX, G>(xmg, gi, kvv, kxv, ninf, l3, flen, tb, A.L, m, hk);
					if constexpr (CH) {
						chain_upd(gi, m[0], hk[0]);
					} else {
#pragma unroll
						for (int w = 0; w < NW; ++w)
							hm[w] |= m[0][w] & hk[0];
					}
				}
			};
			if (__ballot(on)) {
				typedef std::integral_constant<bool, false> F_;
				typedef std::integral_constant<bool, true> T_;
				const uint32_t n0 = gcut & 0xffu, n1 = (gcut >> 8) & 0xffu;
				const uint32_t n2 = (gcut >> 16) & 0xffu;

				probe_range(F_(), F_(), 0u, n0);
				probe_range(T_(), F_(), n0, n1);
				probe_range(F_(), T_(), n1, n2);
				probe_range(T_(), T_(), n2, ngroups);
			}
		}

		/* ---- checksum bytes past the window: the whole wave. Even waves
		 * sum them before the walk, odd waves after it (a pending lane walks
		 * as if its L4 checksum were good; one that fails then takes the
		 * error CoS, which error packets get without a walk): persistent
		 * waves that start together would otherwise stream and walk in
		 * step, leaving the memory idle while they all walk */
		/* ---- the UDP / TCP checksum bytes past the window: the partial
		 * of [64, len) summed a tile ahead, less the bytes [64, a) when the
		 * L4 header starts past the window (generic frames: the residue mod
		 * 0xffff is the tail's, and the pending sum holds the nonzero
		 * protocol term, so the verdict is the same) */
		if (!S64 && ret == PARSE_PEND) {
			uint32_t tail = tsum;

			if (pd.a > 64u) {
				Pkt<64, true> v;

				v.row = row;
				v.g = g;
				v.len = len;
				tail = oc_add(tail, 0xffffu - oc_fold(sum_range(v, 64u, pd.a)));
			}
			ret = finish_l4(p, pd, tail, (uint64_t)opt);
		}

		/* the next tile's windows, in flight during the walk, and its
		 * tails right behind them */
		if constexpr (S64) {
			load_tile(fn, t + nwaves);
		} else {
			load_win(fn, xn, dn);
			if (l4ck)
				tn = early_tails(dn, t + nwaves);
			dnn = load_desc(t + 2u * nwaves);
		}

		/* ---- CoS walk (cls_select_cos + match_pmr_cos) ------------------ */
		bool err = (p.fl & FL_ERROR_MASK) != 0u;
		const bool want_cls = live && ret >= 0;
		uint32_t cos = ODPG_COS_NOCLS;
		bool active = false, any_match = false;
		uint32_t mark = 0u, steps = 0u;

		if (want_cls) {
			if (err) {
				cos = A.error_cos < 0 ? ODPG_COS_NONE : (uint32_t)A.error_cos;
			} else if (def_valid) {
				cos = (uint32_t)A.default_cos;
				active = def_rules;
			} else {
				cos = A.default_cos < 0 ? ODPG_COS_NONE : (uint32_t)A.default_cos;
			}
		}
		{
			/* a level: the lowest set bit of the CoS's bit range [start,
			 * start + n) in the hit map; (lazy form) the CoS's complex PMRs
			 * below it, in rule order, from their term records (gate,
			 * CUSTOM_L3 length guard, masked slot word); then the bit's PMR
			 * destination, mark and the destination's bit range */
			uint32_t crs = 0u, cxf = 0u;

			if (active) {
				crs = xci[cos].x;
				cxf = A.num_xflat ? A.xfc[cos] : 0u;
			}
			while (__ballot(active)) {
				if (active) {
					uint32_t best = 0xffffffffu;

					if constexpr (NW == 2) {
						/* 2-word maps: the CoS's bit range of the 64-bit
						 * map, branch-free (a CoS with rules has 1..64
						 * bits starting below 64) */
						const uint32_t st = crs & 0x3fu, n = crs >> 16;
						uint64_t x = (((uint64_t)hm[1] << 32) | hm[0]) >> st;

						x &= n < 64u ? (1ull << n) - 1ull : ~0ull;
						best = x ? st + (uint32_t)__builtin_ctzll(x) : best;
					} else {
						uint32_t bi = crs & 0xffffu;
						const uint32_t end = bi + (crs >> 16);

						while (bi < end) {
							const uint32_t w = bi >> 5;
							uint32_t x = hm[0];

#pragma unroll
							for (uint32_t k = 1; k < NW; ++k)
								x = w == k ? hm[k] : x;
							x >>= bi & 31u;
							if (end - bi < 32u)
								x &= (1u << (end - bi)) - 1u;
							if (x) {
								best = bi + (uint32_t)__builtin_ctz(x);
								break;
							}
							bi = (w + 1u) << 5;
						}
					}
					uint32_t j = cxf & 0xffffu;
					const uint32_t jend = j + (cxf >> 16);
					bool acc = true;

					for (; j < jend; ++j) {
						/* both halves of the record issued together */
						const uint4 q = xfl[2u * j + 1u];
						const uint4 r = xfl[2u * j];

						if (q.x >= best)
							break;
						Pkt<64, true> v;

						v.row = row;
						v.g = g;
						v.len = len;
						KeySrc<64, true> key;

						key.f = nullptr;
						key.v = &v;
						key.b = &b;
						key.fast = false;
						acc = acc && (b.inf_lo & r.x) == r.x &&
						      (!(r.w >> 31) ||
						       b.len > ((r.w >> 30) & 1u ? 0u : b.l3) + ((r.w >> 8) & 0xffffu)) &&
						      (key(r.w & 0xffu) & r.y) == r.z;
						if (q.y) {              /* the chain's last record */
							if (acc) {
								best = q.x;
								break;
							}
							acc = true;
						} else if (!acc) {      /* failed: on to the next chain */
							j = q.z;
							acc = true;
						}
					}
					if (best == 0xffffffffu) {
						active = false;
					} else {
						const uint4 pd2 = pdst[best];

						cos = pd2.x & 0xffffu;
						mark = pd2.x >> 16;
						crs = pd2.y;
						cxf = pd2.z;
						any_match = true;
						if (++steps >= A.num_cos) {
							cos = ODPG_COS_LOOP;
							active = false;
						} else {
							active = (crs >> 16) != 0u;   /* no rules below: done */
						}
					}
				}
			}
		}

		/* ---- verdict word (odpg.h) ------------------------------------- */
		if (live) {
			int cret = 0;
			bool markv = false;

			if (want_cls) {
				if (cos == ODPG_COS_LOOP)
					cret = -2;
				else if (cos == ODPG_COS_NONE)
					cret = -1;
				else if (cos < A.num_cos && (xci[cos].y & 0xffu) == 1u)
					cret = 1;
				markv = any_match && !err && cos != ODPG_COS_LOOP && mark != 0u;
			} else if (ret < 0) {
				cos = ODPG_COS_PDROP;
			}
			uint32_t w = cos & 0xffffu;

			if (cret == 1)
				w |= ODPG_OUT_CLS_DROP;
			if (p.inf & IF(IFL_L3_CHKSUM_DONE))
				w |= (p.fl & FB(FL_L3_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 16;
			if (p.inf & IF(IFL_L4_CHKSUM_DONE))
				w |= (p.fl & FB(FL_L4_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 18;
			if (err)
				w |= ODPG_OUT_ERROR;
			if (markv)
				w |= ODPG_OUT_MARK_VALID;
			if (ret)
				w |= ODPG_OUT_PARSE_ERR;
			out[i] = w;
			if constexpr (CM == 2) {
				/* one histogram add per packet carries every counter: the
				 * CoS it is handed to error-free (_odp_cls_enq; in_packets,
				 * in_octets), an error packet (to the error CoS; in_errors),
				 * a parse drop (in_errors), no CoS or a CoS loop
				 * (in_discards), a drop CoS (no counter) */
				const uint32_t bn = ret < 0 ? GF_BIN_PDROP : err ? GF_BIN_ERR :
						    cos >= A.num_cos ? GF_BIN_NOCOS :
						    cret == 1 ? GF_BIN_DROP : GF_BIN_EXTRA + cos;

				atomicAdd(&dlv[bn], 1u);
				tile_oct = bn >= GF_BIN_EXTRA ? len : 0u;
			}
		}
		if constexpr (CM == 2) {
			/* the tile's octets (< 2^32: 64 frames) summed across the wave
			 * and added to the workgroup's total: no register carried
			 * through the loop (the counted kernel's VGPR budget) */
			const uint32_t to = wave_sum_u32(tile_oct);

			if (lane == 0u && to)
				atomicAdd(&octets, (unsigned long long)to);
		}
	}
	if constexpr (CM == 2) {
		/* loopback_recv accounting (loop.c:304-374) and the per-queue
		 * delivery counts into this workgroup's counter row: no barrier,
		 * each wave counts itself done after its adds, the last one of the
		 * workgroup flushes while the others have exited */
		if (GF_ROW_REGS(NW) && A.cnt.words <= GF_BLOCK && threadIdx.x < A.cnt.words)
			base[threadIdx.x] = rowv;
		__threadfence_block();
		uint32_t prev = 0u;

		if (lane == 0u)
			prev = atomicAdd(&waves_done, 1u);
		if ((uint32_t)__builtin_amdgcn_readfirstlane((int)prev) != GF_BLOCK / 64u - 1u)
			return;
		__threadfence_block();
		const odpg_cnt_dev C = cnt_lds;
		/* global (not flat) pointers: a flat store counts on the LDS counter
		 * too, so every histogram read would wait for the stores before it */
		__attribute__((address_space(1))) unsigned long long *r =
			(__attribute__((address_space(1))) unsigned long long *)(uintptr_t)(C.rows + (size_t)blockIdx.x * C.words);
		const __attribute__((address_space(1))) uint32_t *qc =
			(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)C.qcol;
		const uint32_t nc = A.num_cos < C.ncos ? A.num_cos : C.ncos;
		/* without hash queues each CoS owns one column */
		auto col = [&](uint32_t c) __attribute__((always_inline)) { return 4u + C.ncos + qc[c]; };
		const uint32_t ne = dlv[GF_BIN_ERR], np = dlv[GF_BIN_PDROP];
		const uint32_t ec = A.error_cos < 0 ? 0xffffffffu : (uint32_t)A.error_cos;
		/* error packets: delivered to the error CoS unless it drops;
		 * without an error CoS they are discards too */
		const bool edeliv = ne && ec < nc && (xci[ec].y & 0xffu) != 1u;
		uint32_t tot = 0u;

		/* plain stores of the row read at the start + the histogram (the
		 * workgroup owns its row; launches on the stream are ordered) */
		/* the identity case (no hash queues) in a loop of its own without
		 * loads: a load there would wait for every store before it */
		auto flush_cols = [&](auto cf) __attribute__((always_inline)) {
			for (uint32_t k0 = 0; k0 < nc; k0 += 64u) {
				const uint32_t k = k0 + lane;
				const uint32_t x = k < nc ? dlv[GF_BIN_EXTRA + k] : 0u;
				const uint32_t xe = x + (edeliv && k == ec ? ne : 0u);

				if (xe) {
					const uint32_t cc = cf(k);

					r[cc] = base[cc] + xe;
				}
				tot += x;
			}
		};

		if (C.ident)
			flush_cols([&](uint32_t k) { return 4u + C.ncos + k; });
		else
			flush_cols(col);
		const uint32_t tp = wave_sum_u32(tot);                  /* in_packets */

		if (lane == 0u) {
			const uint32_t nd = dlv[GF_BIN_NOCOS] + (ec >= nc ? ne : 0u);

			if (tp) {
				r[0] = base[0] + tp;
				r[1] = base[1] + octets;
			}
			if (ne + np)
				r[2] = base[2] + (ne + np);
			if (nd)
				r[3] = base[3] + nd;
		}
	}
}

/* ---- launch ----------------------------------------------------------------- */
extern "C" uint32_t odpg_resident_grid(const void *kernel, uint32_t block, size_t lds);
extern "C" uint32_t odpg_lds_limit(void);

static void gf_layout(const odpg_launch_args *a, xm_layout_t *L)
{
	xm_layout_of(a->xm_nw, a->num_xment, a->xm_slot_bytes, a->num_cos, a->xm_nbits, a->num_xflat, L);
}

/* dynamic LDS of a launch: generic-parse rows + the table's LDS part */
extern "C" size_t odpg_clsgf_lds(const odpg_launch_args *a)
{
	xm_layout_t L;

	gf_layout(a, &L);
	const size_t bins = a->cnt.row ? (((size_t)a->num_cos + GF_BIN_EXTRA + 3u) & ~(size_t)3u) * 4u : 0u;

	return (size_t)GF_BLOCK * GF_RW * 4u + bins + (size_t)((L.lds_words + 1u) & ~1u) * 4u +
	       (a->cnt.row ? (size_t)a->cnt.words * 8u : 0u) +
	       (size_t)GF_BLOCK * 4u;
}

extern "C" int odpg_launch_clsgf(const odpg_launch_args *a, hipStream_t s)
{
	if (a->num == 0)
		return 0;
	if (a->xm_nw != 2u && a->xm_nw != 4u && a->xm_nw != 8u)
		return -EINVAL;
	GFArgs A;

	A.frames = a->frames;
	A.num = a->num;
	A.stride = a->desc ? 0u : a->stride;   /* gf_ok: num * stride < 2^32 */
	A.opt = (uint32_t)a->opt;
	A.ngroups = a->xm_ngroups;
	A.num_cos = a->num_cos;
	A.default_cos = a->default_cos;
	A.error_cos = a->error_cos;
	A.coses = a->coses;
	A.num_xflat = a->num_xflat;
	gf_layout(a, &A.L);
	const uint32_t *xhdr = a->xm;
	const uint4 *xmg = (const uint4 *)(a->xm + XM_HDR_WORDS);

	A.xlds = a->xm + XM_HDR_WORDS + XM_GROUP_WORDS * a->xm_ngroups;
	A.xfc = A.xlds + A.L.lds_words;
	A.cnt = odpg_cnt_layout(&a->cnt);
	A.cnt_words = a->cnt.row ? a->cnt.words : 0u;

	const size_t lds = odpg_clsgf_lds(a);
	const uint32_t ntiles = (a->num + 63u) / 64u;
	const uint32_t want = (ntiles + GF_BLOCK / 64u - 1u) / (GF_BLOCK / 64u);
	const uint32_t rows = a->cnt.row ? a->cnt.rows : 0xffffffffu;

	/* resident grid of the instantiation launched, at most one workgroup per
	 * counter row */
	auto go = [&](auto kern) {
		uint32_t grid = odpg_resident_grid((const void *)kern, GF_BLOCK, lds);

		grid = grid < want ? grid : want;
		grid = grid < rows ? grid : rows;
		hipLaunchKernelGGL(kern, dim3(grid ? grid : 1u), dim3(GF_BLOCK), lds, s, A, xmg, xhdr,
				   a->desc, a->out);
	};
	const bool cm = a->cnt.row != nullptr;
	/* fixed 64-byte stride, 16-byte aligned frames: the S64 instantiation
	 * (its chunk indices are 32-bit) */
	const bool s64 = !a->desc && a->stride == 64u && !((uintptr_t)a->frames & 15u) &&
			 a->num < (1u << 30);

	/* KX tables (more than 16 key slots read) take the descriptor
	 * instantiation, whose probes select slots 16..18 */
	const bool kx = a->xm_kx != 0u;

#define GF_GO(nw)                                                                              \
	(kx ? (cm ? go(odpg_clsgf_kernel<2, nw, false, true>) : go(odpg_clsgf_kernel<0, nw, false, true>)) \
	    : s64 ? (cm ? go(odpg_clsgf_kernel<2, nw, true, false>) : go(odpg_clsgf_kernel<0, nw, true, false>)) \
	    : (cm ? go(odpg_clsgf_kernel<2, nw, false, false>) : go(odpg_clsgf_kernel<0, nw, false, false>)))
	switch (a->xm_nw) {
	case 2: GF_GO(2); break;
	case 4: GF_GO(4); break;
	default: GF_GO(8); break;
	}
#undef GF_GO
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
