/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Lean gfx950 classify kernel for the production receive shape: fixed
 * 64-byte frame stride, a TBL_SIMPLE rule table of <= 64 PMRs (mask groups,
 * odpg_internal.h), verdict words plus the loopback_recv pktio counters (no
 * marks, metadata or per-CoS counters).
 * Same per-packet semantics as odpg_classify_kernel (classify.hip), which
 * handles every other layout / table / output; results are bit-identical
 * (tests/test_gpu_parity.py runs both on the same inputs).
 *
 * Two table forms: HW = false, mask groups (<= 64 PMRs, u64 hit map, one
 * LDS read per walk level); HW = true, CoS-keyed cuckoo groups (TBL_LEAN64HW
 * simple tables of any size, e.g. the 1024-PMR C4 table): per level of the
 * walk both candidates of each group holding rules of the current CoS are
 * read at once with key (masked key word, CoS), and the lowest PMR index
 * found is the first match (odpg_internal.h "CoS-keyed cuckoo groups").
 *
 * Per packet: parse + RX checksum verdicts (_odp_packet_parse_common,
 * odp_parse_internal.h:80-112, odp_packet.c:1906-1984), error-CoS selection
 * and the match_pmr_cos first-match walk (odp_classification.c:1599-1701)
 * over the table's PMR hit bits.
 *
 * Layout: one lane per packet, one wave per 64-packet tile, waves persistent
 * over tiles (no workgroup barrier in the loop). A lane's 64 bytes arrive as
 * 4 x 16 B loads straight into registers, issued one tile ahead. A wave
 * whose frames are all plain Eth/IPv4/UDP|TCP takes the register parse
 * (checksums as v_dot2_u32_u16 sums of 16-bit halves); any other wave copies
 * its frames to LDS rows and runs the generic parse. The mask-group entries
 * and the resolve table live in LDS.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/odpg.h"
#include "odpg_internal.h"
#include "pkt_parse.h"
#include "cls_match.h"
#include "stats_commit.h"

/* waves per SIMD the launch bounds ask for: verdict-only and pktio-block
 * launches at 8 (64 VGPRs, no spills), sharded-counter launches at 6 (their
 * histogram flush spills more scalar registers at 8: 15.9 vs 15.3 us) */
#ifndef L64_WAVES
#define L64_WAVES 8
#endif
#ifndef L64_WAVES_CNT
#define L64_WAVES_CNT 6
#endif
#ifndef L64_WAVES_HW     /* CoS-keyed cuckoo (walk-group) tables, e.g. C4 */
#define L64_WAVES_HW 6
#endif
#ifndef L64_BLOCK        /* threads per workgroup */
#define L64_BLOCK 256
#endif
#ifndef L64_BLOCK_HW      /* threads per workgroup of the CoS-keyed cuckoo kernels */
#define L64_BLOCK_HW 1024
#endif
#define LB L64_BLOCK
/* a kernel's workgroup size: the cuckoo tables are one LDS copy per
 * workgroup, so larger workgroups share it among more waves */
#ifndef L64_BLOCK_CNT     /* threads per workgroup of the sharded-counter kernels */
#define L64_BLOCK_CNT L64_BLOCK
#endif
#define LBH(hw, cm) ((hw) ? L64_BLOCK_HW : (cm) == 2 ? L64_BLOCK_CNT : L64_BLOCK)

struct L64Args {
	const uint4 *frames;
	uint32_t num;
	uint32_t opt;          /* ODPG_PKTIN_* (all defined bits are < 32) */
	uint32_t layer;        /* >= LAYER_L4 */
	uint32_t num_mgroups;
	const dmgroup_t *mgroups;
	const uint4 *ments;
	uint32_t num_ment, num_pmr, num_cos;
	/* HW kernels: cuckoo groups, their entries, pinfo3 */
	const dmgroup_t *cgroups;
	const uint2 *cents;
	uint32_t num_cent;
	const uint2 *pinfo3;
	const uint4 *pinfo4;   /* mask groups: {dst | mark << 16, action, rule mask lo, hi} */
	uint32_t def_mlo, def_mhi;   /* the default CoS's rule mask */
	uint32_t def_cgmask;
	uint32_t err_cos;      /* error CoS, or ODPG_COS_NONE */
	uint32_t err_act;      /* its action */
	uint32_t def_cos;      /* CoS of error-free packets before the walk */
	uint32_t def_act;
	uint32_t def_rules;    /* the default CoS is valid and has rules: walk */
	uint32_t depth;        /* longest rule chain (1..4: unrolled walk), 0 = loop */
	odpg_out_t *out;
	uint64_t *stats;       /* pktio counters (odpg.h), or NULL */
	uint64_t *sred;        /* stats_commit scratch */
	/* sharded counters (odpg.h): their layout, by value (a kernel
	 * argument: the row read at the start depends on no other load) */
	odpg_cnt_dev cnt;
};

/* ---- register parse of plain 64-byte frames ------------------------------ */
typedef unsigned short l64_us2 __attribute__((ext_vector_type(2)));

/* acc + w.lo * x.lo16 + w.hi * x.hi16 (one v_dot2_u32_u16) */
__device__ __forceinline__ uint32_t d2(uint32_t x, uint32_t w, uint32_t acc)
{
	return __builtin_amdgcn_udot2(__builtin_bit_cast(l64_us2, x),
				      __builtin_bit_cast(l64_us2, w), acc, false);
}

/* end-around fold of a sum of < 2^15 16-bit words (chksum_finalize,
 * odp_chksum_internal.h:22-31): 0xffff iff the one's-complement sum is
 * all-ones, as the reference's 64-bit word sum folds */
__device__ __forceinline__ uint32_t d2fold(uint32_t s)
{
	s = d2(s, 0x00010001u, 0u);
	return d2(s, 0x00010001u, 0u);
}

#define W11 0x00010001u   /* both halves */
#define W10 0x00000001u   /* low half (first byte pair) */
#define W01 0x00010000u   /* high half */

/* Verdict of a plain frame (plain_v4() true): parse_fast() semantics.
 * Returns the output word's checksum / error / parse-error bits and the
 * low input flags the rule gates read. */
struct FastV {
	uint32_t wbits;   /* ODPG_OUT_* status bits */
	uint32_t inf_lo;
	bool err;
};

__device__ __forceinline__ FastV parse_fast64(const uint32_t (&f)[16], uint32_t opt)
{
	FastV r;
	const bool udp = (f[5] >> 24) == 0x11u;
	uint32_t inf = (uint32_t)(IF(IFL_L2) | IF(IFL_ETH) | IF(IFL_L3) | IF(IFL_IPV4) | IF(IFL_L4));

	inf |= udp ? (uint32_t)IF(IFL_UDP) : (uint32_t)IF(IFL_TCP);
	r.inf_lo = inf;
	uint32_t wb = 0u;
	bool l3bad = false;

	/* IPv4 header checksum over bytes 14..33 (parse_ipv4, odp_parse.c:134-141);
	 * a bad one is ip_err: no L4 parse, no L4 verdict */
	if (opt & ODPG_PKTIN_IPV4_CHKSUM) {
		uint32_t s = d2(f[3], W01, 0u);

		s = d2(f[4], W11, s);
		s = d2(f[5], W11, s);
		s = d2(f[6], W11, s);
		s = d2(f[7], W11, s);
		s = d2(f[8], W10, s);
		l3bad = d2fold(s) != 0xffffu;
		wb = (l3bad ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 16;
	}
	/* L4 checksum over the pseudo header and bytes 34..63
	 * (_odp_packet_l4_chksum, odp_packet.c:1906-1984; length frame_len - 34):
	 * src + dst, proto << 8, the length field (UDP: its own raw bytes 38..39,
	 * counted again; TCP: be16(30)), then the segment. Branch-free per lane:
	 * the sum is formed whenever either protocol's check is on. */
	bool l4bad = false;

	if (opt & (ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM)) {
		const bool frag = (f[5] & 0xff3fu) != 0u;          /* be16(frag) & 0x3fff */
		const uint32_t need = udp ? ODPG_PKTIN_UDP_CHKSUM : ODPG_PKTIN_TCP_CHKSUM;
		const bool zero_csum = udp && (f[10] & 0xffffu) == 0u;
		uint32_t s = udp ? 0x1100u : 0x1e00u + 0x0600u;

		s = d2(f[6], W01, s);
		s = d2(f[7], W11, s);
		s = d2(f[8], W11, s);
		s = d2(f[9], udp ? 0x00020001u : W11, s);
#pragma unroll
		for (int k = 10; k < 16; ++k)
			s = d2(f[k], W11, s);
		const bool done = ((opt & need) != 0u) & !frag & !l3bad;   /* zero: udp_chksum_zero, ok */

		l4bad = done & !zero_csum & (d2fold(s) != 0xffffu);
		wb |= done ? (l4bad ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 18 : 0u;
	}
	r.err = l3bad | l4bad;
	r.wbits = wb | (r.err ? ODPG_OUT_ERROR | ODPG_OUT_PARSE_ERR : 0u);
	return r;
}

/* plain_v4() (pkt_parse.h) without branches: Eth/IPv4 IHL 5 within the 64
 * bytes, UDP with length >= 8 or TCP with data offset >= 5 */
__device__ __forceinline__ bool plain64(const uint32_t (&f)[16])
{
	const uint32_t tot_len = swap16(f[4] & 0xffffu);
	const uint32_t proto = f[5] >> 24;
	const bool eth_ip = (f[3] & 0x00ffffffu) == 0x00450008u;   /* ethtype 0x0800, ver_ihl 0x45 */
	const bool udp_ok = (proto == 0x11u) & (swap16(f[9] >> 16) >= 8u);
	const bool tcp_ok = (proto == 0x06u) & (((f[11] >> 20) & 0xfu) >= 5u);

	return eth_ip & (tot_len <= 64u - 14u) & (udp_ok | tcp_ok);
}

/* one mask group's descriptor, wave-uniform (SGPRs): sh == 0 marks a
 * single-value group ({value, lo, hi} in {m1, m2, off}, dmgroup_t.count 1) */
struct MGd {
	uint32_t slot, o, req, mask, sh, off, m1, m2;
	/* o: frame byte offset of the slot word in a plain Eth/IPv4 frame */
};

typedef uint32_t u32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

/* single: mask groups (count 1 = one inline value); cuckoo groups keep sh */
__device__ __forceinline__ MGd load_mg(const dmgroup_t *g, bool single = true)
{
	const uint4 g0 = *(const uint4 *)g;
	const uint4 g1 = *((const uint4 *)g + 1);
	MGd d;

	d.slot = __builtin_amdgcn_readfirstlane(g0.x);
	d.req = __builtin_amdgcn_readfirstlane(g0.y);
	d.mask = __builtin_amdgcn_readfirstlane(g0.z);
	d.sh = single && __builtin_amdgcn_readfirstlane(g1.w) == 1u ? 0u
								 : __builtin_amdgcn_readfirstlane(g0.w);
	d.off = __builtin_amdgcn_readfirstlane(g1.x);
	d.m1 = __builtin_amdgcn_readfirstlane(g1.y);
	d.m2 = __builtin_amdgcn_readfirstlane(g1.z);
	/* frame offset of the slot word in a plain Eth/IPv4 frame (l3 14, l4 34;
	 * the VLANX slot reads l3's word, its VLAN gate fails there) */
	d.o = d.slot < SLOT_VLANX ? 4u * d.slot :
	      d.slot < SLOT_L3 ? 14u :
	      d.slot < SLOT_L4 ? 14u + 4u * (d.slot - SLOT_L3) :
	      d.slot < SLOT_LEN ? 34u + 4u * (d.slot - SLOT_L4) : 0u;
	return d;
}

/* a 16-byte LDS table entry read as one ds_read_b128 even when a field is
 * unused (the compiler would narrow it to ds_read_b96: 8 lane groups and
 * 32-bank mapping, twice the LDS cycles, MI355X_MICROARCH.md "LDS") */
__device__ __forceinline__ uint4 lds_ent(const uint4 *p)
{
	const uint4 e = *p;

	asm volatile("" ::"v"(e.w));
	return e;
}

/* sharded-counter histogram bins after the CoS bins (CM 2) */
#define BIN_ERR    0u
#define BIN_PDROP  1u
#define BIN_NOCOS  2u
#define BIN_DROP   3u
#define BIN_EXTRA  4u


/* ---- the kernel ------------------------------------------------------------
 * NG > 0: the table has exactly NG mask groups (HW: walk groups); their
 * descriptors are read once into scalar registers before the tile loop.
 * NG = 0 (mask groups only): any count, read per tile. */
/* CM: counters of the launch: 0 none, 1 the caller's pktio block
 * (stats_commit.h), 2 sharded counter rows (odpg.h). CK: every hoisted
 * group is a cuckoo group over a frame word (TBL_MG_CUCKOO): no per-group
 * kind tests in the tile loop. */
template <int NG, bool HW, int CM, bool CK>
__global__ __launch_bounds__(LBH(HW, CM), (CM == 2 ? L64_WAVES_CNT : HW ? L64_WAVES_HW : L64_WAVES) * 256 / LBH(HW, CM)) void
odpg_cls64_kernel(const L64Args A)
{
	static_assert(!HW || NG > 0, "walk groups are hoisted");
	constexpr uint32_t LBK = LBH(HW, CM);
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	constexpr uint32_t RW = 17;                     /* odd dword row stride */
	uint32_t *row = smem + threadIdx.x * RW;        /* generic-parse LDS row */
	/* sharded counters (CM 2): the histogram right after the rows, at a
	 * fixed offset (its adds need no base register); the table after it */
	uint32_t *dlv = smem + LBK * RW;
	const uint32_t nbins = CM == 2 ? ((A.num_cos + BIN_EXTRA + 3u) & ~3u) : 0u;
	uint4 *ments = (uint4 *)(dlv + nbins);
	uint4 *pinfo4 = ments + A.num_ment;
	/* HW: cuckoo entries, pinfo3 */
	uint2 *cents = (uint2 *)(dlv + nbins);
	uint2 *pinfo3 = cents + A.num_cent;
	/* CM 2: the workgroup's counter row as it stood before this launch,
	 * read at the start (behind the first tile's loads), so that the
	 * flush is plain stores of row + histogram, not atomics at the
	 * kernel's common tail (the workgroup owns its row) */
	unsigned long long *base = HW ? (unsigned long long *)(pinfo3 + A.num_pmr)
				      : (unsigned long long *)(pinfo4 + A.num_pmr);

	const uint32_t lane = __lane_id();
	/* wave-uniform (readfirstlane): buffer resources are built from it */
	const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (LBK / 64) + (threadIdx.x >> 6));
	const uint32_t nwaves = gridDim.x * (LBK / 64);
	const uint32_t ntiles = (A.num + 63u) >> 6;
	const uint32_t num = A.num;
	uint32_t fn[16];
	/* This wave's tiles: tw0 + k * tws, k < twn, round robin over the waves */
	const uint32_t tw0 = gw, tws = nwaves;
	const uint32_t twn = gw < ntiles ? (ntiles - gw + nwaves - 1u) / nwaves : 0u;

	MGd mg[NG > 0 ? NG : 1];
	/* A tile's 4 KiB arrive as coalesced nontemporal 16-byte loads, lane l
	 * holding chunks l, l + 64, l + 128, l + 192 of the tile (each load
	 * instruction reads 1 KiB of contiguous lines, not 64 frames' first 16
	 * bytes), and are transposed to one frame per lane through the wave's own
	 * 4 KiB of LDS (its generic-parse rows). Chunk c (frame c / 4, part
	 * c % 4) of frame r sits at row r, slot (part + r + r / 4) % 4: the
	 * ds_write_b128 lane groups (8 contiguous lanes, banks mod 32) and the
	 * ds_read_b128 groups ({0-3, 12-15, 20-27}, ... banks mod 64) then both
	 * touch distinct banks (MI355X_MICROARCH.md "LDS"). */
	uint32_t *stg = smem + (threadIdx.x & ~63u) * RW;
	const uint32_t sw_fr = lane >> 2;
	const uint32_t sw_w = 16u * sw_fr + 4u * (((lane & 3u) + sw_fr + (sw_fr >> 2)) & 3u);
	const uint32_t sw_c = lane + (lane >> 2);
	auto load_raw = [&](uint32_t (&dst)[16], uint32_t t) {
		if (t >= ntiles)
			return;
		/* chunk indices in 32 bits (launches of < 2^30 packets,
		 * lean64_ok), clamped to the batch's last chunk */
		const uint32_t lim = num * 4u - 1u;
		const uint32_t c0 = t * 256u + lane;

#pragma unroll
		for (int q = 0; q < 4; ++q) {
			const uint32_t c = min(c0 + 64u * q, lim);
			const uint4 x = ld_nt16(A.frames + c);

			dst[4 * q + 0] = x.x;
			dst[4 * q + 1] = x.y;
			dst[4 * q + 2] = x.z;
			dst[4 * q + 3] = x.w;
		}
	};

	/* raw chunks -> LDS -> this lane's frame (the wave's LDS ops run in
	 * order: the next stage's writes follow this stage's reads) */
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
	/* the first tile's frames are issued before the table copy below */
	load_raw(fn, twn ? tw0 : ntiles);

	if constexpr (HW) {
		for (uint32_t k = threadIdx.x; k < A.num_cent; k += LBK)
			cents[k] = A.cents[k];
		for (uint32_t k = threadIdx.x; k < A.num_pmr; k += LBK)
			pinfo3[k] = A.pinfo3[k];
#pragma unroll
		for (int g = 0; g < NG; ++g)
			mg[g] = load_mg(A.cgroups + g, false);
	} else {
		for (uint32_t k = threadIdx.x; k < A.num_ment; k += LBK)
			ments[k] = A.ments[k];
		for (uint32_t k = threadIdx.x; k < A.num_pmr; k += LBK)
			pinfo4[k] = A.pinfo4[k];
		if constexpr (NG > 0) {
#pragma unroll
			for (int g = 0; g < NG; ++g)
				mg[g] = load_mg(A.mgroups + g);
		}
	}
	/* CM 2: the counter layout is read now, not behind the tile loop's
	 * last wait; the workgroup's last wave to finish flushes the histogram */
	__shared__ uint32_t waves_done;
	__shared__ odpg_cnt_dev cnt_lds;
	__shared__ uint32_t flush_tot;
	unsigned long long rowv = 0ull;   /* CM 2: this thread's word of the row */
	bool row_out = false;             /* CM 2: rowv written to LDS */

	if constexpr (CM == 2) {
		/* the layout (a kernel argument) is kept in LDS for the flush:
		 * nothing of it is held through the tile loop (scalar registers) */
		const odpg_cnt_dev C = A.cnt;

		if (threadIdx.x == 0u)
			cnt_lds = C;
		const __attribute__((address_space(1))) unsigned long long *r0 =
			(const __attribute__((address_space(1))) unsigned long long *)(uintptr_t)(C.rows + (size_t)blockIdx.x * C.words);

		if (C.words <= LBK) {
			/* one word per thread, held in registers until the flush:
			 * nothing waits for the row before the tile loop (C1
			 * counted 13.5-13.9 vs 14.3-14.4 us through LDS here) */
			if (threadIdx.x < C.words)
				rowv = r0[threadIdx.x];
		} else {
			for (uint32_t k = threadIdx.x; k < C.words; k += LBK)
				base[k] = r0[k];
		}
		for (uint32_t k = threadIdx.x; k < A.num_cos + BIN_EXTRA; k += LBK)
			dlv[k] = 0u;
		if (threadIdx.x == 0u) {
			waves_done = 0u;
			flush_tot = 0u;
		}
	}
	__syncthreads();

	/* loopback_recv accounting (loop.c:304-374), wave-uniform counts */
	uint32_t n_pkt = 0u, n_err = 0u, n_disc = 0u;
	const bool walk = A.def_rules != 0u;

	/* Hit bits of one mask group: both cuckoo candidates are read and the
	 * entry whose value equals the packet's masked key word ORs its PMR bits
	 * (odpg_internal.h "Mask groups"). */
	auto probe = [&](const MGd &d, uint32_t key, uint32_t inf_lo, uint32_t &lo, uint32_t &hi) {
		const uint32_t kvm = key & d.mask;
		const bool rq = (inf_lo & d.req) == d.req;

		if (!CK && d.sh == 0u) {
			const bool h = rq & (kvm == d.m1);

			lo |= h ? d.m2 : 0u;
			hi |= h ? d.off : 0u;
		} else if (d.m1 == d.m2) {
			/* collision-free group (cls_compile.cpp build_mgroup): one read */
			const uint4 e1 = lds_ent(ments + d.off + ((kvm * d.m1) >> d.sh));
			const bool h1 = rq & (e1.x == kvm);

			lo |= h1 ? e1.y : 0u;
			hi |= h1 ? e1.z : 0u;
		} else {
			const uint4 e1 = ments[d.off + ((kvm * d.m1) >> d.sh)];
			const uint4 e2 = ments[d.off + ((kvm * d.m2) >> d.sh)];
			const bool h1 = rq & (e1.x == kvm), h2 = rq & (e2.x == kvm);

			lo |= (h1 ? e1.y : 0u) | (h2 ? e2.y : 0u);
			hi |= (h1 ? e1.z : 0u) | (h2 ? e2.z : 0u);
		}
	};

	/* cls_select_cos + match_pmr_cos (odp_classification.c:1599-1701) on the
	 * packet's hit bits (mask groups) or masked group keys (HW), then the
	 * verdict word (odpg.h) and the wave's pktio counts */
	auto finish = [&](bool live, bool pdrop, bool err, uint32_t wbits, uint32_t lo, uint32_t hi,
			  const uint32_t *kv, const bool *krq) -> uint32_t {
		uint32_t cos = err ? A.err_cos : A.def_cos;
		uint32_t act = err ? A.err_act : A.def_act;
		uint32_t mark = 0u;
		bool any_match = false;

		if constexpr (HW) {
			/* one level per iteration: at CoS c both candidates of each
			 * group holding a rule of c are read with key (c, masked key
			 * word); the lowest PMR index found is c's first matching rule */
			bool active = live && !pdrop && !err && walk;
			uint32_t steps = 0u, gm = A.def_cgmask;

			if (A.depth - 1u < 4u) {
				/* acyclic table, longest chain A.depth rules: exactly
				 * that many levels without divergent branches. A group
				 * is skipped (a uniform branch) when no lane of the wave
				 * is at a CoS with rules in it; otherwise every lane
				 * reads its candidates and a lane without the group in
				 * its CoS's mask ignores them. A lane whose level finds
				 * no rule keeps its state and is inactive from then on. */
#pragma unroll
				for (uint32_t l = 0; l < 4u; ++l) {
					if (l >= A.depth || !__ballot(active))
						break;
					uint32_t best = 0xffffffffu;

#pragma unroll
					for (int g = 0; g < NG; ++g) {
						const bool v = active & krq[g] & (((gm >> g) & 1u) != 0u);

						if (!__ballot(v))
							continue;
						const uint32_t x = cgroup_key(kv[g], cos);
						const uint2 e1 = cents[mg[g].off + ((x * mg[g].m1) >> mg[g].sh)];
						const uint2 e2 = cents[mg[g].off + ((x * mg[g].m2) >> mg[g].sh)];
						const bool h1 = v & (e1.x == kv[g]) & ((e1.y & 0xffffu) == cos);
						const bool h2 = v & (e2.x == kv[g]) & ((e2.y & 0xffffu) == cos);

						best = min(best, min(h1 ? e1.y >> 16 : 0xffffffffu,
								     h2 ? e2.y >> 16 : 0xffffffffu));
					}
					const bool hit = best != 0xffffffffu;
					const uint2 pi = pinfo3[hit ? best : 0u];

					cos = hit ? (pi.x & 0xffffu) : cos;
					mark = hit ? (pi.x >> 16) : mark;
					act = hit ? (pi.y & 0xffu) : act;
					any_match |= hit;
					active = hit & (((pi.y >> 8) & 1u) != 0u);   /* rules below */
					gm = pi.y >> 12;
				}
				active = false;
			}
			while (active) {
				uint32_t best = 0xffffffffu;

#pragma unroll
				for (int g = 0; g < NG; ++g) {
					if (!krq[g] || !((gm >> g) & 1u))
						continue;
					const uint32_t x = cgroup_key(kv[g], cos);
					const uint2 e1 = cents[mg[g].off + ((x * mg[g].m1) >> mg[g].sh)];
					const uint2 e2 = cents[mg[g].off + ((x * mg[g].m2) >> mg[g].sh)];

					if (e1.x == kv[g] && (e1.y & 0xffffu) == cos)
						best = min(best, e1.y >> 16);
					if (e2.x == kv[g] && (e2.y & 0xffffu) == cos)
						best = min(best, e2.y >> 16);
				}
				if (best == 0xffffffffu)
					break;
				const uint2 pi = pinfo3[best];

				cos = pi.x & 0xffffu;
				mark = pi.x >> 16;
				act = pi.y & 0xffu;
				any_match = true;
				if (++steps >= A.num_cos) {
					cos = ODPG_COS_LOOP;
					break;
				}
				active = (pi.y >> 8) & 1u;   /* rules below */
				gm = pi.y >> 12;
			}
		} else {
			/* first hit among the current CoS's rules: the hit bits AND
			 * the CoS's rule mask, lowest set bit; one LDS read per level
			 * (pinfo4 carries the next CoS's mask) */
			uint32_t mlo = err ? 0u : A.def_mlo, mhi = err ? 0u : A.def_mhi;

			if (A.depth - 1u < 4u) {
				/* acyclic table, longest chain A.depth rules: exactly that
				 * many levels, branch-free (a level without a hit keeps
				 * the state: its mask becomes 0) */
#pragma unroll
				for (uint32_t l = 0; l < 4u; ++l) {
					if (l >= A.depth)
						break;
					const uint32_t xl = lo & mlo, xh = hi & mhi;
					const bool hit = !pdrop & ((xl | xh) != 0u);
					const uint32_t k = xl ? (uint32_t)__builtin_ctz(xl)
							      : xh ? 32u + (uint32_t)__builtin_ctz(xh) : 0u;
					const uint4 pi = pinfo4[k];

					cos = hit ? (pi.x & 0xffffu) : cos;
					mark = hit ? (pi.x >> 16) : mark;
					act = hit ? pi.y : act;
					mlo = hit ? pi.z : 0u;
					mhi = hit ? pi.w : 0u;
					any_match |= hit;
				}
			} else if (live && !pdrop) {
				uint32_t steps = 0u;

				for (;;) {
					const uint32_t xl = lo & mlo, xh = hi & mhi;

					if ((xl | xh) == 0u)
						break;
					const uint32_t k = xl ? (uint32_t)__builtin_ctz(xl)
							      : 32u + (uint32_t)__builtin_ctz(xh);
					const uint4 pi = pinfo4[k];

					cos = pi.x & 0xffffu;
					mark = pi.x >> 16;
					act = pi.y;
					mlo = pi.z;
					mhi = pi.w;
					any_match = true;
					if (++steps >= A.num_cos) {
						cos = ODPG_COS_LOOP;
						break;
					}
				}
			}
		}
		uint32_t w;

		if (pdrop) {
			w = ODPG_COS_PDROP | wbits;
		} else {
			w = (cos & 0xffffu) | wbits;
			if (cos < ODPG_COS_NOCLS && act == 1u)
				w |= ODPG_OUT_CLS_DROP;
			if (any_match && !err && cos != ODPG_COS_LOOP && mark)
				w |= ODPG_OUT_MARK_VALID;
		}
		if constexpr (CM == 2) {
			/* one histogram add per packet carries every counter (four
			 * bins, then one per CoS): the CoS it is handed to
			 * error-free (_odp_cls_enq; in_packets), an error packet (goes
			 * to the error CoS; in_errors), a parse drop (in_errors), no
			 * CoS or a CoS loop (in_discards), a drop CoS (no counter) */
			const uint32_t b = pdrop ? BIN_PDROP : err ? BIN_ERR :
					   cos >= A.num_cos ? BIN_NOCOS : act == 1u ? BIN_DROP : BIN_EXTRA + cos;

			if (live)
				atomicAdd(&dlv[b], 1u);
		} else if constexpr (CM == 1) {
			/* in_packets: delivered error-free (cls ret 0); in_errors:
			 * parse ret != 0; in_discards: cls ret -1 (no CoS; a CoS loop
			 * counts the same) */
			const bool nocos = cos == ODPG_COS_NONE || cos == ODPG_COS_LOOP;
			const bool ok = live && !pdrop && !err && !nocos && act != 1u;

			n_pkt += (uint32_t)__builtin_popcountll(__ballot(ok));
			n_err += (uint32_t)__builtin_popcountll(__ballot(live && (wbits & ODPG_OUT_PARSE_ERR)));
			n_disc += (uint32_t)__builtin_popcountll(__ballot(live && !pdrop && nocos));
		}
		return w;
	};

	/* Tiles in chunks of up to 64 per wave. Inside a chunk only plain waves
	 * are classified, each tile's frames prefetched one tile ahead; a tile
	 * with any other frame is marked in `defer` and classified after the
	 * chunk by the generic parse, with its frames re-read. The hot loop thus
	 * stays small (instruction cache) and no prefetch registers are live
	 * across the generic parse (register pressure); the last tile of a chunk
	 * issues no prefetch (a wave never re-reads past its last tile). */
	constexpr uint32_t NO_TILE = 0xffffffffu;
	auto tile_n = [&](uint32_t t) -> uint32_t {    /* frames of tile t in the batch */
		return t < ntiles ? min(num - t * 64u, 64u) : 0u;
	};
	uint32_t pend_t = NO_TILE, pend_w = 0u;
	auto store_pending = [&]() {
		if (lane < tile_n(pend_t))
			A.out[pend_t * 64u + lane] = pend_w;
		pend_t = NO_TILE;
	};

	/* One tile from a frame buffer whose loads were issued earlier: the
	 * previous tile's verdict is stored, then this tile is classified if
	 * every live frame is plain (otherwise it is deferred). Returns true if
	 * the tile was deferred. */
	auto tile = [&](const uint32_t (&f)[16], uint32_t t) -> bool {
		const bool live = lane < tile_n(t);

		store_pending();
		if (__ballot(live && !plain64(f)) != 0ull)
			return true;
		/* register parse of plain frames + the table's key words at fixed
		 * frame offsets (uniform register index, no per-slot branches) */
		uint32_t lo = 0u, hi = 0u;
		uint32_t kv[HW ? NG : 1];
		bool krq[HW ? NG : 1];
		const FastV r = parse_fast64(f, A.opt);

		if (walk) {
			const u32x16_t fv = {f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7],
					     f[8], f[9], f[10], f[11], f[12], f[13], f[14], f[15]};
			auto fast_key = [&](const MGd &d) -> uint32_t {
				if (!CK && d.slot == SLOT_LEN)
					return 64u;
				return __builtin_amdgcn_alignbyte(fv[(d.o >> 2) + 1u], fv[d.o >> 2], d.o & 3u);
			};
			if constexpr (HW) {
#pragma unroll
				for (int g = 0; g < NG; ++g) {
					kv[g] = fast_key(mg[g]) & mg[g].mask;
					krq[g] = (r.inf_lo & mg[g].req) == mg[g].req;
				}
			} else if constexpr (NG > 0) {
#pragma unroll
				for (int g = 0; g < NG; ++g)
					probe(mg[g], fast_key(mg[g]), r.inf_lo, lo, hi);
			} else {
				for (uint32_t gi = 0; gi < A.num_mgroups; ++gi) {
					const MGd d = load_mg(A.mgroups + gi);

					probe(d, fast_key(d), r.inf_lo, lo, hi);
				}
			}
		}
		const uint32_t w = finish(live, false, r.err, r.wbits, lo, hi, kv, krq);
		pend_t = t;
		pend_w = w;
		return false;
	};

	/* Tiles in chunks of up to 64 per wave. Inside a chunk only plain waves
	 * are classified; a tile's raw chunks (fn, loaded one tile ahead) are
	 * transposed into the frame buffer fb through the wave's LDS rows, and
	 * the next tile's loads are issued before this one is classified.
	 * A tile with any other frame is marked in `defer` and classified after
	 * the chunk by the generic parse, with its frames re-read: the hot loop
	 * stays small (instruction cache) and no prefetch registers are live
	 * across the generic parse (register pressure). */
	uint32_t fb[16];   /* this tile's frames, one per lane (fn: the raw chunks) */
	bool first = true;

	for (uint32_t t0 = tw0, rem = twn; rem;) {
		const uint32_t nk = rem < 64u ? rem : 64u;
		uint64_t defer = 0ull;

		if (!first) {
			load_raw(fn, t0);
		}
		first = false;
		for (uint32_t k = 0; k < nk; ++k) {
			const uint32_t t = t0 + k * tws;

			stage(fn, fb);
			load_raw(fn, k + 1u < nk ? t + tws : NO_TILE);
			if (tile(fb, t))
				defer |= 1ull << k;
			if (CM == 2 && !row_out) {
				/* the counter row's word into LDS behind the first
				 * tile: its wait (the compiler's vmcnt(0), the load
				 * long landed) then only covers the next tile's loads,
				 * which the next stage waits for anyway; at the flush
				 * it would wait for every verdict store first */
				if (A.cnt.words <= LBK && threadIdx.x < A.cnt.words)
					base[threadIdx.x] = rowv;
				row_out = true;
			}
		}
		store_pending();

		/* ---- the chunk's deferred tiles: generic parse ------------------- */
		while (defer) {
			const uint32_t k = (uint32_t)__builtin_ctzll(defer);

			defer &= defer - 1ull;
			const uint32_t t = t0 + k * tws;
			const uint32_t i = t * 64u + lane;
			const bool live = i < num;
			const uint4 *src = A.frames + (size_t)min(i, num - 1u) * 4u;
			uint32_t f[16];

#pragma unroll
			for (int q = 0; q < 4; ++q) {
				const uint4 x = ld_stream(src + q);

				f[4 * q + 0] = x.x;
				f[4 * q + 1] = x.y;
				f[4 * q + 2] = x.z;
				f[4 * q + 3] = x.w;
			}
			Bases b;
			Pkt<64, false> v;

			v.row = row;
			v.g = (const uint8_t *)src;
			v.len = 64u;
#pragma unroll
			for (int q = 0; q < 16; ++q)
				row[q] = f[q];
			Prs p;

			p.inf = 0ull;
			p.fl = 0u;
			p.l2 = p.l3 = p.l4 = 0xffffu;
			const int ret = live ? parse_common(p, v, A.layer, (uint64_t)A.opt) : 0;
			uint32_t wbits = 0u;

			if (p.inf & IF(IFL_L3_CHKSUM_DONE))
				wbits |= (p.fl & FB(FL_L3_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 16;
			if (p.inf & IF(IFL_L4_CHKSUM_DONE))
				wbits |= (p.fl & FB(FL_L4_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 18;
			const bool err = (p.fl & FL_ERROR_MASK) != 0u;

			if (err)
				wbits |= ODPG_OUT_ERROR;
			if (ret)
				wbits |= ODPG_OUT_PARSE_ERR;
			const uint32_t inf_lo = (uint32_t)p.inf;

			b.l2 = p.l2;
			b.l3 = p.l3;
			b.l4 = p.l4;
			b.vlanx = 14u + ((p.inf & IF(IFL_VLAN_QINQ)) ? 4u : 0u);
			b.len = 64u;
			b.inf_lo = inf_lo;
			uint32_t lo = 0u, hi = 0u;
			uint32_t kv[HW ? NG : 1];
			bool krq[HW ? NG : 1];

			if (walk) {
				KeySrc<64, false> key;

				key.f = f;
				key.v = &v;
				key.b = &b;
				key.fast = false;
				if constexpr (HW) {
#pragma unroll
					for (int g = 0; g < NG; ++g) {
						kv[g] = key(mg[g].slot) & mg[g].mask;
						krq[g] = (inf_lo & mg[g].req) == mg[g].req;
					}
				} else if constexpr (NG > 0) {
#pragma unroll
					for (int g = 0; g < NG; ++g)
						probe(mg[g], key(mg[g].slot), inf_lo, lo, hi);
				} else {
					for (uint32_t gi = 0; gi < A.num_mgroups; ++gi) {
						const MGd d = load_mg(A.mgroups + gi);

						probe(d, key(d.slot), inf_lo, lo, hi);
					}
				}
			}
			const uint32_t w = finish(live, ret < 0, err, wbits, lo, hi, kv, krq);

			if (live)
				A.out[i] = w;
		}
		t0 += nk * tws;
		rem -= nk;
	}
	if constexpr (CM == 2) {
		/* the workgroup's histogram into its own counter row (odpg.h
		 * "sharded counters"): plain stores of the row read at the start
		 * plus the histogram (the workgroup owns the row; the launches
		 * on the stream are ordered). No-return atomics here, ~70 per
		 * workgroup, all reached L2 together at the kernel's common tail
		 * (+1 us of 13.3 on C2) */
		/* Mask-group tables (<= 64 PMRs, a few dozen bins): no barrier,
		 * each wave counts itself done after its histogram adds (LDS
		 * operations of a wave complete in order; the fence makes that
		 * explicit) and the last of the workgroup's waves flushes while the
		 * others have already exited. CoS-keyed tables (HW, up to 1024+
		 * CoS, 1024-thread workgroups): a barrier, then every wave flushes a
		 * slice of the bins (one wave alone would issue ~17 passes of 64
		 * at the kernel's tail: C4 counted 22.6 vs 16.4 us with atomics). */
		uint32_t k_first = lane, k_step = 64u;
		bool lead = lane == 0u;

		if (!row_out && A.cnt.words <= LBK && threadIdx.x < A.cnt.words)
			base[threadIdx.x] = rowv;      /* a wave without tiles */

		if constexpr (HW) {
			__syncthreads();
			k_first = threadIdx.x;
			k_step = LBK;
			lead = threadIdx.x == 0u;
		} else {
			__threadfence_block();
			uint32_t prev = 0u;

			if (lane == 0u)
				prev = atomicAdd(&waves_done, 1u);
			if ((uint32_t)__builtin_amdgcn_readfirstlane((int)prev) != LBK / 64u - 1u)
				return;
			__threadfence_block();
		}
		const odpg_cnt_dev C = cnt_lds;
		/* global (not flat) pointers: a flat store counts on the LDS counter
		 * too, so every histogram read would wait for the stores before it */
		__attribute__((address_space(1))) unsigned long long *r =
			(__attribute__((address_space(1))) unsigned long long *)(uintptr_t)(C.rows + (size_t)blockIdx.x * C.words);
		const __attribute__((address_space(1))) uint32_t *qc =
			(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)C.qcol;
		const uint32_t nc = A.num_cos < C.ncos ? A.num_cos : C.ncos;
		/* without hash queues each CoS owns one column; else its first */
		auto col = [&](uint32_t c) { return 4u + C.ncos + qc[c]; };
		const uint32_t ne = dlv[BIN_ERR], np = dlv[BIN_PDROP];
		/* error packets are delivered to the error CoS unless it drops;
		 * without an error CoS they are discards too */
		const bool edeliv = ne && A.err_cos < nc && A.err_act != 1u;
		uint32_t tot = 0u;

		/* the identity case (no hash queues) in a loop of its own without
		 * loads: a load there would wait for every store before it */
		auto flush_cols = [&](auto cf) {
			for (uint32_t k = k_first; k < (nc + 63u) / 64u * 64u; k += k_step) {
				const uint32_t x = k < nc ? dlv[BIN_EXTRA + k] : 0u;
				const uint32_t xe = x + (edeliv && k == A.err_cos ? ne : 0u);

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
		uint32_t t = wave_sum_u32(tot);            /* in_packets, in_octets */

		if constexpr (HW) {
			/* every wave flushed a slice: the in_packets total over them */
			if (lane == 0u && t)
				atomicAdd(&flush_tot, t);
			__syncthreads();
			t = flush_tot;
		}
		if (lead) {
			const uint32_t nd = dlv[BIN_NOCOS] + (A.err_cos >= nc ? ne : 0u);

			if (t) {
				r[0] = base[0] + t;
				r[1] = base[1] + (unsigned long long)t * 64ull;
			}
			if (ne + np)
				r[2] = base[2] + (ne + np);
			if (nd)
				r[3] = base[3] + nd;
		}
	} else if constexpr (CM == 1) {
		const uint64_t v[4] = {n_pkt, (uint64_t)n_pkt * 64u, n_err, n_disc};

		stats_commit_wave(v, A.sred);
	}
}

/* ---- launch ----------------------------------------------------------------- */
extern "C" uint32_t odpg_resident_grid(const void *kernel, uint32_t block, size_t lds);

/* dynamic LDS of a lean launch: generic-parse rows + the table copy */
size_t odpg_cls64_lds(const odpg_launch_args &a)
{
	const bool hw = (a.tbl_flags & TBL_LEAN64HW) && !(a.tbl_flags & TBL_LEAN64);

	return (size_t)LBH(hw, a.cnt.row ? 2 : 0) * 17u * 4u +
	       (hw ? (size_t)a.num_cent * 8u + (size_t)a.num_pmr * 8u
		   : (size_t)a.num_ment * 16u + (size_t)a.num_pmr * 16u) +
	       (a.cnt.row ? (((size_t)a.num_cos + BIN_EXTRA + 3u) & ~(size_t)3u) * 4u +
				    (size_t)a.cnt.words * 8u : 0u);
}

extern "C" int odpg_launch_cls64(const odpg_launch_args *a, hipStream_t s)
{
	if (a->num == 0)
		return 0;
	L64Args A;

	A.frames = (const uint4 *)a->frames;
	A.num = a->num;
	A.opt = (uint32_t)a->opt;
	A.layer = a->layer;
	A.num_mgroups = a->num_mgroups;
	A.mgroups = a->mgroups;
	A.ments = (const uint4 *)a->ments;
	A.num_ment = a->num_ment;
	A.num_pmr = a->num_pmr;
	A.num_cos = a->num_cos;
	A.err_cos = a->l64_err_cos;
	A.err_act = a->l64_err_act;
	A.def_cos = a->l64_def_cos;
	A.def_act = a->l64_def_act;
	A.def_rules = a->l64_def_rules;
	A.depth = a->l64_depth;
	A.cgroups = a->cgroups;
	A.cents = (const uint2 *)a->cents;
	A.num_cent = a->num_cent;
	A.pinfo3 = (const uint2 *)a->pinfo3;
	A.pinfo4 = (const uint4 *)a->pinfo4;
	A.def_mlo = a->l64_def_mlo;
	A.def_mhi = a->l64_def_mhi;
	A.def_cgmask = a->def_cgmask;
	A.out = a->out;
	A.stats = a->stats;
	A.sred = a->sred;
	A.cnt = odpg_cnt_layout(&a->cnt);

	const bool hw = (a->tbl_flags & TBL_LEAN64HW) && !(a->tbl_flags & TBL_LEAN64);
	size_t lds = odpg_cls64_lds(*a);
	const uint32_t ntiles = (a->num + 63u) / 64u;
	const uint32_t lb = LBH(hw, a->cnt.row ? 2 : 0);
	const uint32_t want = (ntiles + lb / 64u - 1u) / (lb / 64u);
	const uint32_t rows = a->cnt.row ? a->cnt.rows : 0xffffffffu;
	const int cm = a->cnt.row ? 2 : a->stats ? 1 : 0;
	const bool ck = !hw && (a->tbl_flags & TBL_MG_CUCKOO);

	/* resident grid of the instantiation launched, at most one workgroup
	 * per counter row */
	auto go = [&](const void *k, auto launch) {
		uint32_t grid = odpg_resident_grid(k, lb, lds);

		/* verdict-only mask-group launches with a walk of two or more
		 * levels leave an eighth of the resident slots empty: C2 13.2-13.6
		 * vs 13.7-13.9 us at 7 vs 8 workgroups per CU, while the one-level
		 * C1 runs better at 8 (12.5-12.7 vs 12.8-13.1 us) */
		if (!hw && cm == 0 && a->l64_depth != 1u)
			grid -= grid / 8u;
		grid = grid < want ? grid : want;
		grid = grid < rows ? grid : rows;
		launch(grid);
	};
#define L64_LAUNCH_CM(ng, h, c, k)                                                           \
	go((const void *)odpg_cls64_kernel<ng, h, c, k>, [&](uint32_t grid) {                 \
		hipLaunchKernelGGL((odpg_cls64_kernel<ng, h, c, k>), dim3(grid), dim3(lb), lds, s, A); \
	})
#define L64_LAUNCH_K(ng, h, k)                                                                 \
	(cm == 2 ? L64_LAUNCH_CM(ng, h, 2, k) : cm == 1 ? L64_LAUNCH_CM(ng, h, 1, k) : L64_LAUNCH_CM(ng, h, 0, k))
#define L64_LAUNCH(ng, h) (ck ? L64_LAUNCH_K(ng, h, true) : L64_LAUNCH_K(ng, h, false))
	if (hw) {
		switch (a->num_cgroups) {
		case 1: L64_LAUNCH_K(1, true, false); break;
		case 2: L64_LAUNCH_K(2, true, false); break;
		case 3: L64_LAUNCH_K(3, true, false); break;
		default: L64_LAUNCH_K(4, true, false); break;   /* TBL_LEAN64HW: <= 4 groups */
		}
	} else {
		switch (a->num_mgroups) {
		case 1: L64_LAUNCH(1, false); break;
		case 2: L64_LAUNCH(2, false); break;
		case 3: L64_LAUNCH(3, false); break;
		case 4: L64_LAUNCH(4, false); break;
		default: L64_LAUNCH_K(0, false, false); break;
		}
	}
#undef L64_LAUNCH
#undef L64_LAUNCH_K
#undef L64_LAUNCH_CM
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
