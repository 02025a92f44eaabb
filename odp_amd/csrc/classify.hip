/* SPDX-License-Identifier: BSD-3-Clause
 *
 * gfx950 (MI355X, CDNA4) kernels for ODP's receive-path classifier.
 *
 * One lane = one packet, 256-lane workgroups (4 wave64s). Per packet:
 *   1. stage the first W bytes of the frame in LDS (bytes past the frame end
 *      are zero). For the fixed 64-byte stride layout the workgroup loads its
 *      256 x 64 B = 16 KiB slice with fully coalesced 16-byte-per-lane loads
 *      and transposes it into per-packet LDS rows (row stride W+4 bytes = an
 *      odd number of dwords, so same-offset reads by 32 lanes hit 32 banks);
 *   2. parse L2/L3/L4 exactly like _odp_packet_parse_common()
 *      (odp_parse_internal.h:80-112, odp_parse.c:23-475) and verify the IPv4
 *      header / UDP / TCP / SCTP checksums (odp_packet.c:1906-1984);
 *   3. walk the CoS graph like match_pmr_cos() (odp_classification.c:1599-1642).
 *      The walk is wave-cooperative: the wave repeatedly takes the CoS of its
 *      first unfinished lane (readfirstlane), and every lane sitting on that
 *      CoS evaluates its rules together, so rule and term descriptors are
 *      wave-uniform scalar loads and only the packet bytes are per lane.
 *      First-match order, invalid-destination skipping, marks and per-CoS
 *      counters follow the reference;
 *   4. write one 4-byte verdict word (odpg.h) and optional mark / metadata.
 * Packets are independent: no inter-workgroup communication. Per-workgroup
 * counter partials are summed by a second small kernel (no same-address
 * global atomics).
 */
#include <hip/hip_runtime.h>
#include <mutex>
#include <vector>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/odpg.h"
#include "odpg_internal.h"

#include "pkt_parse.h"
#include "cls_match.h"
#include "stats_commit.h"

/* ----------------------------------------------------------------------- */
/* compiled term evaluation (odp_classification.c:1338-1490 via cls_compile) */

/* byte fields of the term / slot descriptors read as one dword: the
 * wave-uniform reads then compile to scalar loads (a byte field would be a
 * vector load, ordered behind every outstanding frame load) */
__device__ __forceinline__ uint32_t term_hdr(const dterm_t *t)
{
	uint32_t x;

	__builtin_memcpy(&x, t, 4);     /* kind | base << 8 | nwords << 16 | tflags << 24 */
	return x;
}

__device__ __forceinline__ uint32_t slot_hdr(const dslot_t *sl)
{
	uint32_t x;

	__builtin_memcpy(&x, sl, 4);    /* slot | nw << 8 */
	return x;
}

template <int W, bool GF>
__device__ __forceinline__ bool term_cmp(const dterm_t *__restrict__ t, const Pkt<W, GF> &v,
					 const Bases &b)
{
	const uint32_t th = term_hdr(t);
	uint32_t kind = th & 0xffu;

	if (kind == DK_LEN)
		return (b.len & t->mask[0]) == t->value[0];
	if (kind != DK_CMP)
		return false;
	uint32_t base_k = (th >> 8) & 0xffu;
	uint32_t base = base_k == DB_L3 ? b.l3 : base_k == DB_L4 ? b.l4 :
			base_k == DB_L2 ? b.l2 : base_k == DB_VLANX ? b.vlanx : 0u;
	uint32_t pos = base + (uint32_t)t->off;

	if (((th >> 24) & DT_GUARD) && !(b.len > pos + t->size))
		return false;
	bool ok = true;
	uint32_t nw = (th >> 16) & 0xffu;

	for (uint32_t k = 0; k < nw; ++k)
		ok = ok & ((v.rd32(pos + 4u * k) & t->mask[k]) == t->value[k]);
	return ok;
}

template <int W, bool GF>
__device__ __forceinline__ bool pmr_match(const dterm_t *__restrict__ terms, uint32_t start,
					  uint32_t n, const Pkt<W, GF> &v, const Bases &b)
{
	bool ok = true;
	uint32_t end = start + n;

	/* term indices stay wave-uniform (scalar loads of the term table): an
	 * IPv4/IPv6 alternative pair is evaluated on both sides and selected
	 * per lane, never by a per-lane pointer */
	for (uint32_t ti = __builtin_amdgcn_readfirstlane(start); ti < end;) {
		const dterm_t *t = terms + ti;
		bool r;

		if ((term_hdr(t) >> 24) & DT_ALT_NEXT) {
			const dterm_t *t2 = t + 1;
			const bool first = (b.inf_lo & t->req) == t->req;
			const bool r1 = term_cmp(t, v, b);
			const bool r2 = ((b.inf_lo & t2->req) == t2->req) & term_cmp(t2, v, b);

			r = first ? r1 : r2;
			ti += 2;
		} else {
			r = ((b.inf_lo & t->req) == t->req) & term_cmp(t, v, b);
			ti += 1;
		}
		ok = ok & r;
	}
	return ok;
}

/* thash_softrss (protocols/thash.h:81-99) with the default key
 * (odp_classification.c:50-58) */
__constant__ uint32_t c_rss_key_be[11] = {
	0x6d5a56dau, 0x255b0ec2u, 0x4167253du, 0x43a38fb0u, 0xd0ca2bcbu,
	0xae7b30b4u, 0x77cb2da3u, 0x8030f20cu, 0x6a42b73bu, 0xbeac01fau, 0u
};

__device__ uint32_t thash(const uint32_t *tuple, uint32_t n)
{
	uint32_t ret = 0;

	for (uint32_t j = 0; j < n; ++j) {
		uint32_t k0 = c_rss_key_be[j], k1 = c_rss_key_be[j + 1];

		for (uint32_t i = 0; i < 32; ++i)
			if (tuple[j] & (1u << (31 - i)))
				ret ^= (k0 << i) | (i ? (k1 >> (32 - i)) : 0u);
	}
	return ret;
}

/* packet_rss_hash (odp_classification.c:1751-1817) */
template <int W, bool GF>
__device__ uint32_t rss_hash(const Prs &p, const Pkt<W, GF> &v, uint32_t hp)
{
	uint32_t tuple[9];
	uint32_t n = 0;

#pragma unroll
	for (int k = 0; k < 9; ++k)
		tuple[k] = 0u;
	if (p.inf & IF(IFL_IPV4)) {
		if (hp & 1u) {
			tuple[0] = v.rd32(p.l3 + 12u);
			tuple[1] = v.rd32(p.l3 + 16u);
			n += 2;
		}
		if (((p.inf & IF(IFL_TCP)) && (hp & 8u)) || (!(p.inf & IF(IFL_TCP)) &&
		    (p.inf & IF(IFL_UDP)) && (hp & 4u))) {
			tuple[2] = v.rd32(p.l4);
			n += 1;
		}
	} else if (p.inf & IF(IFL_IPV6)) {
		if (hp & 2u) {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				tuple[k] = __builtin_bswap32(v.rd32(p.l3 + 8u + 4u * k));
				tuple[4 + k] = __builtin_bswap32(v.rd32(p.l3 + 24u + 4u * k));
			}
			n += 8;
		}
		if (((p.inf & IF(IFL_TCP)) && (hp & 8u)) || (!(p.inf & IF(IFL_TCP)) &&
		    (p.inf & IF(IFL_UDP)) && (hp & 4u))) {
			tuple[8] = v.rd32(p.l4);
			n += 1;
		}
	}
	return n ? thash(tuple, n) : 0u;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		x += __shfl_xor(x, o, 64);
	return x;
}




__device__ __forceinline__ void extract_key_fast(uint32_t (&key)[KEY_SLOTS], const uint32_t (&f)[16],
						 const Prs &p, uint32_t slot_mask)
{
#pragma unroll
	for (int s = 0; s < 5; ++s)
		key[SLOT_L2 + s] = f[s];
	key[SLOT_VLANX] = fw<14>(f);
	key[SLOT_L3 + 0] = fw<14>(f);
	key[SLOT_L3 + 1] = fw<18>(f);
	key[SLOT_L3 + 2] = fw<22>(f);
	key[SLOT_L3 + 3] = fw<26>(f);
	key[SLOT_L3 + 4] = fw<30>(f);
	key[SLOT_L3 + 5] = fw<34>(f);
	key[SLOT_L3 + 6] = fw<38>(f);
	key[SLOT_L3 + 7] = fw<42>(f);
	key[SLOT_L3 + 8] = fw<46>(f);
	key[SLOT_L3 + 9] = fw<50>(f);
	const bool l4ok = p.l4 != 0xffffu;

	key[SLOT_L4 + 0] = l4ok ? fw<34>(f) : 0u;
	key[SLOT_L4 + 1] = l4ok ? fw<38>(f) : 0u;
	key[SLOT_LEN] = 64u;
	(void)slot_mask;
}



/* ---- evaluate-all helpers ---------------------------------------------- */
/* extract the key slots the table reads (odpg_internal.h "key slots") */
template <int W, bool GF>
__device__ __forceinline__ void extract_key(uint32_t (&key)[KEY_SLOTS], const Pkt<W, GF> &v,
					    const Bases &b, uint32_t slot_mask)
{
#pragma unroll
	for (int s = 0; s < KEY_SLOTS; ++s)
		key[s] = 0u;
#pragma unroll
	for (int s = 0; s < 5; ++s)
		if (slot_mask & (1u << (SLOT_L2 + s)))
			key[SLOT_L2 + s] = v.rd32(b.l2 + 4u * s);
	if (slot_mask & (1u << SLOT_VLANX))
		key[SLOT_VLANX] = v.rd32(b.vlanx);
	if (slot_mask & (0x3ffu << SLOT_L3)) {
		/* L3 words: read the covering aligned words once, then funnel */
		uint32_t base = b.l3, w0 = base >> 2, sh = base & 3u;
		uint32_t prev = v.word(w0);
#pragma unroll
		for (int s = 0; s < 10; ++s) {
			if ((slot_mask >> (SLOT_L3 + s)) & (0x3ffu >> s)) {   /* slot s or later used */
				uint32_t nxt = v.word(w0 + s + 1);

				key[SLOT_L3 + s] = sh ? __builtin_amdgcn_alignbyte(nxt, prev, sh) : prev;
				prev = nxt;
			}
		}
	}
#pragma unroll
	for (int s = 0; s < 2; ++s)
		if (slot_mask & (1u << (SLOT_L4 + s)))
			key[SLOT_L4 + s] = v.rd32(b.l4 + 4u * s);
	key[SLOT_LEN] = b.len;
}

template <int W, bool GF>
__device__ __forceinline__ bool term_eval(const dterm_t *__restrict__ t, const dslot_t *__restrict__ sl,
					  const KeySrc<W, GF> &key, const Pkt<W, GF> &v,
					  const Bases &b)
{
	const bool req_ok = (b.inf_lo & t->req) == t->req;

	const uint32_t sh = slot_hdr(sl);

	if ((sh & 0xffu) == SLOT_NONE)
		return req_ok & term_cmp(t, v, b);
	bool ok = req_ok;
	const uint32_t s0 = sh & 0xffu, nw = (sh >> 8) & 0xffu;

	for (uint32_t k = 0; k < nw; ++k)
		ok = ok & ((key(s0 + k) & sl->mask[k]) == sl->value[k]);
	return ok;
}

/* verify_pmr (odp_classification.c:1338-1490) for one compiled PMR */
template <int W, bool GF>
__device__ __forceinline__ bool pmr_eval(const dterm_t *__restrict__ terms,
					 const dslot_t *__restrict__ slots, uint32_t start,
					 uint32_t n, const KeySrc<W, GF> &key,
					 const Pkt<W, GF> &v, const Bases &b)
{
	bool ok = true;
	const uint32_t end = start + n;

	/* wave-uniform term index (see pmr_match) */
	for (uint32_t ti = __builtin_amdgcn_readfirstlane(start); ti < end;) {
		const dterm_t *t = terms + ti;
		bool r;

		if ((term_hdr(t) >> 24) & DT_ALT_NEXT) {
			const bool first = (b.inf_lo & t->req) == t->req;
			const bool r1 = term_eval(t, slots + ti, key, v, b);
			const bool r2 = term_eval(t + 1, slots + ti + 1, key, v, b);

			r = first ? r1 : r2;
			ti += 2;
		} else {
			r = term_eval(t, slots + ti, key, v, b);
			ti += 1;
		}
		ok = ok & r;
	}
	return ok;
}


__device__ __forceinline__ int first_hit_lds(const uint32_t *hrow, uint32_t rs, uint32_t nr)
{
	const uint32_t end = rs + nr;

	for (uint32_t bpos = rs; bpos < end;) {
		uint32_t sh = bpos & 31u, take = 32u - sh;

		if (take > end - bpos)
			take = end - bpos;
		uint32_t x = hrow[bpos >> 5] >> sh;

		if (take < 32u)
			x &= (1u << take) - 1u;
		if (x)
			return (int)(bpos - rs + (uint32_t)__builtin_ctz(x));
		bpos += take;
	}
	return -1;
}

/* ----------------------------------------------------------------------- */
/* LEAN: launch-time specialisation for the common production shape, a
 * TBL_SIMPLE table without hash-queue CoS, verdict words only (no marks,
 * metadata or counters): the unused paths compile out, which frees the
 * scalar registers the general kernel spills. Results are identical. */
template <int W, bool COOP, bool GF, bool DESC, int MODE, bool FAST, bool LEAN>
#ifndef LEAN_WAVES
#define LEAN_WAVES 5
#endif
#ifndef GEN_WAVES
#define GEN_WAVES 6
#endif
#ifndef ODPG_DEFER_MOD          /* waves w with w % MOD < K sum tails after the walk */
#define ODPG_DEFER_MOD 3
#define ODPG_DEFER_K 1
#endif
__global__ __launch_bounds__(BLOCK, LEAN ? LEAN_WAVES : FAST ? 5 : GEN_WAVES) void odpg_classify_kernel(
	const uint8_t *__restrict__ frames, const odpg_desc_t *__restrict__ desc,
	uint32_t stride, uint32_t num, uint64_t opt, uint32_t layer, uint32_t classify,
	const dterm_t *__restrict__ terms, const dpmr_t *__restrict__ pmrs,
	const dcos_t *__restrict__ coses, uint32_t num_cos, int32_t default_cos,
	int32_t error_cos, uint32_t tbl_flags, uint32_t num_pmr, uint32_t slot_mask,
	const dslot_t *__restrict__ slots, const dsimple_t *__restrict__ simple,
	const drun_t *__restrict__ runs, uint32_t num_runs,
	const dhgroup_t *__restrict__ hgroups, uint32_t num_hgroups,
	const dhent_t *__restrict__ hents_g, uint32_t num_hent,
	const uint2 *__restrict__ cinfo_g, const uint32_t *__restrict__ pinfo_g,
	const dmgroup_t *__restrict__ mgroups, uint32_t num_mgroups,
	const uint4 *__restrict__ ments_g, uint32_t num_ment, const uint2 *__restrict__ pinfo2_g,
	odpg_out_t *__restrict__ out, uint16_t *__restrict__ mark_out,
	odpg_meta_t *__restrict__ meta_out, uint64_t *__restrict__ pk_partial,
	uint32_t *__restrict__ cos_partial, uint64_t *__restrict__ sred,
	const uint2 *__restrict__ xcos_g, const uint32_t *__restrict__ xlist_g, uint32_t num_xent,
	uint32_t num_xwords, const odpg_cnt_args cnt)
{
	constexpr uint32_t RW = W / 4 + 1;       /* odd dword row stride */
	extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
	/* u64 hit-map kernel: mask-group entries (16 B aligned, after the rows)
	 * and the one-read-per-level resolve table */
	const bool use_mg = MODE == 1 && (tbl_flags & TBL_MGROUPS);
	uint4 *ments_l = (uint4 *)(smem + BLOCK * RW);
	uint32_t *cos_cnt = (uint32_t *)(ments_l + (use_mg ? num_ment : 0u));
	/* sharded counters: per-queue delivered counts after the CoS counters */
	const bool cos_words = cos_partial || (cnt.row && cnt.cos);
	uint32_t *dlv = cos_cnt + (cos_words ? ((num_cos + 3u) & ~3u) : 0u);
	/* MODE 2: per-lane PMR hit bitmap after the counters */
	const uint32_t hrw = ((num_pmr + 31u) >> 5) | 1u;
	uint32_t *hitmap = dlv + (cnt.row ? ((cnt.ncols + 3u) & ~3u) : 0u);
	/* exact-match hash tables, copied to LDS when small */
	uint2 *hents_l = (uint2 *)(hitmap + (MODE == 2 ? BLOCK * hrw : 0u));
	const bool hent_in_lds = !use_mg && num_hent <= HENT_LDS_MAX;
	/* per-lane CoS / PMR lookups of the first-match resolve, in LDS */
	uint2 *cinfo = hents_l + (hent_in_lds ? num_hent : 0u);
	uint32_t *pinfo = (uint32_t *)(cinfo + num_cos);
	uint2 *pinfo2 = (uint2 *)(pinfo + ((num_pmr + 1u) & ~1u));
	/* hybrid hash walk (TBL_XWALK): per-CoS complex-rule lists in LDS, in
	 * the place MODE 1 keeps pinfo2 */
	const bool use_x = MODE == 3 && (tbl_flags & TBL_XWALK);
	uint2 *xcos_l = pinfo2;
	uint2 *xlist_l = (uint2 *)(xcos_l + (use_x ? ((num_cos + 1u) & ~1u) : 0u));
	/* xterm records: read as uint2 pairs (the LDS carve-up is 8-byte aligned) */
	const uint2 *xterm_l = xlist_l + ((num_xent + 1u) & ~1u);
	__shared__ unsigned long long blk_pk[4];

	const uint32_t tid = threadIdx.x;
	if constexpr (LEAN) {
		mark_out = nullptr;
		meta_out = nullptr;
		pk_partial = nullptr;
		cos_partial = nullptr;
		tbl_flags = (tbl_flags | TBL_SIMPLE) & ~(TBL_GENERIC | TBL_ANY_HASHQ);
	}
	const bool do_stats = pk_partial != nullptr || cnt.row != nullptr;
	const bool do_cos_stats = cos_partial != nullptr || (cnt.row && cnt.cos);
	uint32_t *row = smem + tid * RW;
	/* loopback_recv counts: packets / errors / discards as wave-uniform
	 * ballot counts (scalar registers), octets per lane */
	uint32_t w_pkt = 0u, w_err = 0u, w_disc = 0u;
	uint64_t lane_oct = 0;

	/* persistent workgroups: tiles of BLOCK packets */
	const uint32_t ntiles = (num + BLOCK - 1) / BLOCK;
	uint32_t fn[16];   /* FAST: next tile's frame, prefetched one tile ahead */

	if constexpr (FAST) {
		/* first tile's frames are issued before the table copy below, so
		 * the frame stream starts at once instead of behind the table
		 * reads' round trip; unconditional (index clamped into the batch)
		 * so the loads always issue and the wait counts stay exact */
		const uint32_t i0 = min(blockIdx.x * BLOCK + tid, num - 1u);
		const uint4 *src = (const uint4 *)(frames + (size_t)i0 * 64u);

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint4 x = ld_stream(src + k);

			fn[4 * k + 0] = x.x;
			fn[4 * k + 1] = x.y;
			fn[4 * k + 2] = x.z;
			fn[4 * k + 3] = x.w;
		}
	}
	if (tid < 4)
		blk_pk[tid] = 0ull;
	if (do_cos_stats)
		for (uint32_t c = tid; c < num_cos; c += BLOCK)
			cos_cnt[c] = 0u;
	if (cnt.row)
		for (uint32_t c = tid; c < cnt.ncols; c += BLOCK)
			dlv[c] = 0u;
	if (MODE != 0 && hent_in_lds)
		for (uint32_t k = tid; k < num_hent; k += BLOCK)
			hents_l[k] = *(const uint2 *)(hents_g + k);
	if (MODE != 0) {
		for (uint32_t k = tid; k < num_cos; k += BLOCK)
			cinfo[k] = cinfo_g[k];
		for (uint32_t k = tid; k < num_pmr; k += BLOCK)
			pinfo[k] = pinfo_g[k];
	}
	if (use_mg)
		for (uint32_t k = tid; k < num_ment; k += BLOCK)
			ments_l[k] = ments_g[k];
	if (MODE == 1)
		for (uint32_t k = tid; k < num_pmr; k += BLOCK)
			pinfo2[k] = pinfo2_g[k];
	if (use_x) {
		for (uint32_t k = tid; k < num_cos; k += BLOCK)
			xcos_l[k] = xcos_g[k];
		for (uint32_t k = tid; k < num_xwords; k += BLOCK)
			((uint32_t *)xlist_l)[k] = xlist_g[k];
	}
	__syncthreads();
	/* default CoS entry: read once, outside the tile loop */
	const bool def_valid = default_cos >= 0 && coses[default_cos].valid;
	const bool def_rules = def_valid && coses[default_cos].nrule != 0u;
	/* per-lane CoS info: LDS copy in the evaluate-all kernels, global otherwise */
	auto cinfo_at = [&](uint32_t c) -> uint2 {
		if constexpr (MODE != 0)
			return cinfo[c];
		else
			return cinfo_g[c];
	};

	/* result stores of a tile are issued at the top of the next one, before
	 * that tile's prefetch: vector-memory counters retire in issue order, so
	 * a store issued after the prefetch would make the next wait on the
	 * prefetched frame wait on the store too */
	bool pend = false;
	uint32_t pend_i = 0u, pend_w = 0u, pend_mk = 0u;

	for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
	const uint32_t blk0 = tile * BLOCK;
	const uint32_t i = blk0 + tid;
	const bool live = i < num;

	if (pend) {
		out[pend_i] = pend_w;
		if (mark_out)
			mark_out[pend_i] = (uint16_t)pend_mk;
	}

	/* ---- 1. stage the frame window in LDS ---------------------------- */
	const uint8_t *g;
	uint32_t len;

	if (DESC) {
		odpg_desc_t d = live ? desc[i] : odpg_desc_t{0u, 0u};

		g = frames + d.offset;
		len = d.len;
	} else {
		g = frames + (size_t)i * stride;
		len = live ? stride : 0u;
	}

	uint32_t f[16];
	bool wave_fast = false;

	if constexpr (FAST) {
		/* 64-byte frames straight into 16 registers, 4 x 16 B per lane;
		 * this tile's were prefetched, issue the next tile's now */
#pragma unroll
		for (int k = 0; k < 16; ++k)
			f[k] = fn[k];
		const uint32_t nt = tile + gridDim.x;
		const uint32_t inx = min(nt < ntiles ? nt * BLOCK + tid : i, num - 1u);
		const uint4 *src = (const uint4 *)(frames + (size_t)inx * 64u);

#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint4 x = ld_stream(src + k);

			fn[4 * k + 0] = x.x;
			fn[4 * k + 1] = x.y;
			fn[4 * k + 2] = x.z;
			fn[4 * k + 3] = x.w;
		}
		const bool plain = live && layer >= LAYER_L4 &&
				   !(opt & (ODPG_PKTIN_DROP_IPV4_ERR | ODPG_PKTIN_DROP_IPV6_ERR |
					    ODPG_PKTIN_DROP_UDP_ERR | ODPG_PKTIN_DROP_TCP_ERR |
					    ODPG_PKTIN_DROP_SCTP_ERR)) && plain_v4(f);

		wave_fast = __ballot(live && !plain) == 0ull;
		if (!wave_fast || (tbl_flags & (TBL_GENERIC | TBL_ANY_HASHQ))) {
#pragma unroll
			for (int k = 0; k < 16; ++k)
				row[k] = f[k];
		}
	} else if (COOP) {
		/* stride == W: the block's frames are one contiguous span */
		constexpr uint32_t CPP = W / 16;
		const uint4 *src = (const uint4 *)(frames + (size_t)blk0 * W);
		uint32_t nvalid = num - blk0 < BLOCK ? num - blk0 : BLOCK;

#pragma unroll
		for (uint32_t k = 0; k < CPP; ++k) {
			uint32_t c = k * BLOCK + tid;
			uint32_t pk = c / CPP, part = c % CPP;
			uint4 x = make_uint4(0u, 0u, 0u, 0u);

			if (pk < nvalid)
				x = src[c];
			uint32_t *dst = smem + pk * RW + part * 4u;

			dst[0] = x.x;
			dst[1] = x.y;
			dst[2] = x.z;
			dst[3] = x.w;
		}
	} else {
#pragma unroll
		for (uint32_t part = 0; part < W / 16; ++part) {
			uint32_t b0 = part * 16u;
			uint4 x = make_uint4(0u, 0u, 0u, 0u);

			if (b0 < len) {
				x = *(const uint4 *)(g + b0);
				uint32_t rem = len - b0;

				if (rem < 16u) {
					uint32_t m[4];

#pragma unroll
					for (int q = 0; q < 4; ++q) {
						int nb = (int)rem - 4 * q;

						m[q] = nb >= 4 ? 0xffffffffu : nb <= 0 ? 0u :
						       (1u << (8 * nb)) - 1u;
					}
					x.x &= m[0];
					x.y &= m[1];
					x.z &= m[2];
					x.w &= m[3];
				}
			}
			row[part * 4u + 0u] = x.x;
			row[part * 4u + 1u] = x.y;
			row[part * 4u + 2u] = x.z;
			row[part * 4u + 3u] = x.w;
		}
	}
	if (COOP)
		__syncthreads();

	Pkt<W, GF> v;

	v.row = row;
	v.g = g;
	v.len = len;

	/* ---- 2. parse + checksum verdicts --------------------------------- */
	Prs p;

	p.inf = 0ull;
	p.fl = 0u;
	p.l2 = p.l3 = p.l4 = 0xffffu;
	int ret = 0;
	L4Pend pd = {0u, 0u, 0u, 0u};

	if (FAST && wave_fast) {
		if (live)
			ret = parse_fast(p, f, opt);
	} else if (live && layer) {
		if constexpr (GF)
			ret = parse_common(p, v, layer, opt, &pd);
		else
			ret = parse_common(p, v, layer, opt);
	}
	/* long UDP / TCP frames: tails summed by the whole wave (all 64 lanes
	 * active, as the cooperative loads and DPP need). Odd waves sum them
	 * after the CoS walk instead of before it: the walk does not depend on
	 * the L4 checksum (a frame it fails is re-pointed to the error CoS
	 * afterwards, as cls_select_cos would have done), and with half the
	 * waves in each order the memory-bound tail passes of some waves run
	 * while others issue their walks. Launches that count per-CoS packets
	 * keep the original order (the walk counts the CoSes it visits). */
	const bool defer = GF && !do_cos_stats &&
			   (((blockIdx.x * (BLOCK / 64u)) + (tid >> 6)) % ODPG_DEFER_MOD) <
				   ODPG_DEFER_K;
	auto run_tails = [&]() {
		const uint64_t pm = __ballot(ret == PARSE_PEND);

		if (pm) {
			const uint32_t tail = seg_tail_sums4<false>(pm, g, pd);

			if (ret == PARSE_PEND)
				ret = finish_l4(p, pd, tail, opt);
		}
	};

	if constexpr (GF) {
		if (!defer)
			run_tails();
	}

	/* ---- 3. CoS walk ------------------------------------------------- */
	uint32_t cos = ODPG_COS_NOCLS;
	int cret = 0;
	bool any_match = false;
	uint32_t mark = 0u;
	bool want_cls = live && layer && classify && ret >= 0;
	bool active = false;
	uint32_t steps = 0;

	if (want_cls) {
		if (p.fl & FL_ERROR_MASK) {
			cos = error_cos < 0 ? ODPG_COS_NONE : (uint32_t)error_cos;
		} else if (def_valid) {
			cos = (uint32_t)default_cos;
			active = def_rules;
		} else {
			cos = default_cos < 0 ? ODPG_COS_NONE : (uint32_t)default_cos;
		}
	}

	Bases b;

	b.l2 = p.l2;
	b.l3 = p.l3;
	b.l4 = p.l4;
	b.vlanx = 14u + ((p.inf & IF(IFL_VLAN_QINQ)) ? 4u : 0u);
	b.len = len;
	b.inf_lo = (uint32_t)p.inf;

	if constexpr (MODE == 3) {
		/* hash walk: match_pmr_cos (odp_classification.c:1599-1642) one
		 * level at a time; at CoS c a packet probes each CoS-keyed walk
		 * group once with (c, masked key word) and the lowest PMR index
		 * found is the first match of c's rule list (odpg_internal.h).
		 * hgroups / hents carry the walk groups in this mode. */
		KeySrc<W, GF> key;

		key.f = f;
		key.v = &v;
		key.b = &b;
		key.fast = FAST && wave_fast;
		auto probe = [&](const uint2 *ents, uint32_t off, uint32_t h, uint32_t szm,
				 uint32_t kv, uint32_t c) -> uint32_t {
			for (uint32_t pr = 0; pr <= szm; ++pr) {
				const uint2 e = ents[off + h];

				if (e.y == HENT_EMPTY)
					break;
				if (e.x == kv && (e.y & 0xffffu) == c)
					return e.y >> 16;
				h = (h + 1u) & szm;
			}
			return 0xffffffffu;
		};
		/* hybrid walk with at most XWALK_KEYS groups: the masked key
		 * words do not depend on the CoS, so each group's key is read
		 * once per packet (gok: groups whose gate holds), not per level */
		constexpr uint32_t XK = XWALK_KEYS;
		const bool xkeys = use_x && num_hgroups <= XK;
		uint32_t kvx[XK];
		uint32_t gok = 0u;

		if (xkeys) {
#pragma unroll
			for (uint32_t gi = 0; gi < XK; ++gi) {
				kvx[gi] = 0u;
				if (gi < num_hgroups) {
					const uint4 g0 = *(const uint4 *)(hgroups + gi);
					const uint32_t gslot = __builtin_amdgcn_readfirstlane(g0.x);
					const uint32_t greq = __builtin_amdgcn_readfirstlane(g0.y);
					const uint32_t gmask = __builtin_amdgcn_readfirstlane(g0.z);

					if (active && (b.inf_lo & greq) == greq) {
						kvx[gi] = key(gslot) & gmask;
						gok |= 1u << gi;
					}
				}
			}
		}
		while (__ballot(active)) {
			uint32_t best = 0xffffffffu;
			uint32_t xs = 0u, xn = 0u;

			if (xkeys) {
				/* every key group, wave-uniform control flow: a group's
				 * table is probed at exactly its longest displacement
				 * (maxp, cls_compile) with no early exit, and the result
				 * kept when the CoS has a rule in the group (gm). A key
				 * that is in the table sits within maxp slots of its
				 * home, so the result is the probe loop's. */
				const uint2 xe = active ? xcos_l[cos] : make_uint2(0u, 0u);
				const uint32_t gm = xe.y & gok;
				const uint32_t ck = cos * 0x85EBCA6Bu;

				xs = xe.x & 0xffffu;
				xn = xe.x >> 16;
#pragma unroll
				for (uint32_t gi = 0; gi < XK; ++gi) {
					if (gi >= num_hgroups)
						break;
					/* deep levels: few lanes still walking, most
					 * groups hold no rule of their CoSes */
					if (!__ballot((gm >> gi) & 1u))
						continue;
					const uint4 g0 = *(const uint4 *)(hgroups + gi);
					const uint4 g1 = *((const uint4 *)(hgroups + gi) + 1);
					const uint32_t lg = __builtin_amdgcn_readfirstlane(g0.w);
					const uint32_t goff = __builtin_amdgcn_readfirstlane(g1.x);
					const uint32_t maxp = __builtin_amdgcn_readfirstlane(g1.z);
					const uint32_t szm = (1u << lg) - 1u;
					const uint32_t kv = kvx[gi];
					const uint32_t h = ((kv ^ ck) * 0x9E3779B1u) >> (32u - lg);

					if (hent_in_lds && maxp - 1u < XWALK_MAXP) {
						uint32_t r = 0xffffffffu;

#pragma unroll
						for (uint32_t pr = 0; pr < XWALK_MAXP; ++pr) {
							if (pr >= maxp)
								break;
							const uint2 e = hents_l[goff + ((h + pr) & szm)];

							r = (e.x == kv && (e.y & 0xffffu) == cos) ? e.y >> 16 : r;
						}
						best = ((gm >> gi) & 1u) && r < best ? r : best;
					} else if (active && ((gm >> gi) & 1u)) {
						const uint32_t r = hent_in_lds
							? probe(hents_l, goff, h, szm, kv, cos)
							: probe((const uint2 *)hents_g, goff, h, szm, kv, cos);

						best = r < best ? r : best;
					}
				}
			} else if (active) {
				uint32_t gm = 0xffffffffu;

				if (use_x) {
					/* complex rules of this CoS, and the walk
					 * groups holding one of its single-word rules */
					const uint2 xe = xcos_l[cos];

					xs = xe.x & 0xffffu;
					xn = xe.x >> 16;
					gm = xe.y;
				}
				for (uint32_t gi = 0; gi < num_hgroups; ++gi) {
					const uint4 g0 = *(const uint4 *)(hgroups + gi);
					const uint2 g1 = *(const uint2 *)((const uint32_t *)(hgroups + gi) + 4);
					const uint32_t gslot = __builtin_amdgcn_readfirstlane(g0.x);
					const uint32_t greq = __builtin_amdgcn_readfirstlane(g0.y);
					const uint32_t gmask = __builtin_amdgcn_readfirstlane(g0.z);
					const uint32_t lg = __builtin_amdgcn_readfirstlane(g0.w);
					const uint32_t goff = __builtin_amdgcn_readfirstlane(g1.x);

					if (((gm >> gi) & 1u) && (b.inf_lo & greq) == greq) {
						const uint32_t kv = key(gslot) & gmask;
						const uint32_t h = walk_hash(kv, cos, lg);
						const uint32_t r = hent_in_lds
							? probe(hents_l, goff, h, (1u << lg) - 1u, kv, cos)
							: probe((const uint2 *)hents_g, goff, h, (1u << lg) - 1u, kv, cos);

						best = r < best ? r : best;
					}
				}
			}
			if (use_x) {
				/* the CoS's complex rules below the best group hit, in
				 * rule order. Rules of single-word slot compares are
				 * evaluated per lane from their xterm records; the others
				 * one PMR at a time across the wave (uniform index:
				 * scalar term loads, as MODE 0) */
				uint32_t xk = 0u;
				bool xp = active && xn != 0u && xlist_l[xs].x < best;

				while (__ballot(xp)) {
					if (xp) {
						const uint2 xe = xlist_l[xs + xk];
						const uint32_t nt = xe.y >> 24;
						bool hit = false, done = false;

						if (nt) {
							const uint2 *tr = xterm_l + 2u * (xe.y & 0xffffffu);

							hit = true;
							for (uint32_t t = 0; t < nt && hit; ++t) {
								const uint2 r0 = tr[2u * t], r1 = tr[2u * t + 1u];
								const uint4 r = make_uint4(r0.x, r0.y, r1.x, r1.y);
								const uint32_t sl = r.w & 0xffu;

								/* gate, then the CUSTOM_L3 length guard,
								 * before the slot is read */
								/* bit 30: CUSTOM_FRAME, guard and
								 * word from the frame start (the L2
								 * slots whenever the parse set l2 = 0) */
								const bool ab = (r.w >> 30) & 1u;
								const uint32_t kw = ab && b.l2 != 0u ? v.rd32(4u * sl) : key(sl);

								hit = (b.inf_lo & r.x) == r.x &&
								      (!(r.w >> 31) ||
								       b.len > (ab ? 0u : b.l3) + ((r.w >> 8) & 0xffffu)) &&
								      (kw & r.y) == r.z;
							}
							done = true;
						} else {
							const uint32_t u = __builtin_amdgcn_readfirstlane(xe.x);

							if (xe.x == u) {
								const dpmr_t pm = pmrs[u];

								hit = pmr_match(terms, pm.term_start, pm.nterms, v, b);
								done = true;
							}
						}
						if (done) {
							if (hit) {
								best = xe.x;
								xp = false;
							} else {
								++xk;
								xp = xk < xn && xlist_l[xs + xk].x < best;
							}
						}
					}
				}
			}
			if (active) {
				if (best == 0xffffffffu) {
					active = false;
				} else {
					const uint32_t pi = pinfo[best];

					cos = pi & 0xffffu;
					mark = pi >> 16;
					any_match = true;
					if (do_cos_stats && ((cinfo[cos].y >> 16) & 0xffu))
						atomicAdd(&cos_cnt[cos], 1u);
					if (++steps >= num_cos) {
						cos = ODPG_COS_LOOP;
						active = false;
					} else if ((cinfo[cos].x >> 16) == 0u) {
						active = false;       /* no rules below: done */
					}
				}
			}
		}
	} else if constexpr (MODE != 0) {
		/* evaluate every PMR of the table (branch-free, wave-uniform
		 * descriptors), then resolve match_pmr_cos's depth-first
		 * first-match walk (odp_classification.c:1599-1642) on the hit
		 * bits. Same verdict as evaluating rules only at visited CoS:
		 * rule evaluation has no side effects. */
		uint64_t hits = 0ull;
		uint32_t *hrow = hitmap + tid * hrw;

		if (__ballot(active)) {
			KeySrc<W, GF> key;

			key.f = f;
			key.v = &v;
			key.b = &b;
			key.fast = FAST && wave_fast;
			if (use_mg) {
				/* mask groups: both cuckoo candidates of every group
				 * are read (independent LDS reads, no probe chain) and
				 * the entry whose value matches ORs its PMR bits */
				uint32_t lo = 0u, hi = 0u;

				for (uint32_t gi = 0; gi < num_mgroups; ++gi) {
					const uint4 g0 = *(const uint4 *)(mgroups + gi);
					const uint4 g1 = *((const uint4 *)(mgroups + gi) + 1);
					const uint32_t gslot = __builtin_amdgcn_readfirstlane(g0.x);
					const uint32_t greq = __builtin_amdgcn_readfirstlane(g0.y);
					const uint32_t gmask = __builtin_amdgcn_readfirstlane(g0.z);
					const uint32_t gsh = __builtin_amdgcn_readfirstlane(g0.w);
					const uint32_t goff = __builtin_amdgcn_readfirstlane(g1.x);
					const uint32_t gm1 = __builtin_amdgcn_readfirstlane(g1.y);
					const uint32_t gm2 = __builtin_amdgcn_readfirstlane(g1.z);
					const uint32_t gcnt = __builtin_amdgcn_readfirstlane(g1.w);
					const uint32_t kvm = key(gslot) & gmask;
					const bool rq = (b.inf_lo & greq) == greq;

					if (gcnt == 1u) {
						/* one value: inline {value, lo, hi} = {m1, m2, off} */
						const bool h = rq & (kvm == gm1);

						lo |= h ? gm2 : 0u;
						hi |= h ? goff : 0u;
						continue;
					}
					const uint4 e1 = ments_l[goff + ((kvm * gm1) >> gsh)];
					const uint4 e2 = ments_l[goff + ((kvm * gm2) >> gsh)];
					const bool h1 = rq & (e1.x == kvm), h2 = rq & (e2.x == kvm);

					lo |= (h1 ? e1.y : 0u) | (h2 ? e2.y : 0u);
					hi |= (h1 ? e1.z : 0u) | (h2 ? e2.z : 0u);
				}
				hits = ((uint64_t)hi << 32) | lo;
			} else if (tbl_flags & TBL_SIMPLE) {
				uint32_t lo = 0u, hi = 0u;

				if (MODE == 2)
					for (uint32_t w = 0; w < hrw; ++w)
						hrow[w] = 0u;
				/* exact-match groups: one probe sequence each; the
				 * entry table is read through an LDS-typed pointer when
				 * resident (a generic pointer would make each probe wait
				 * on the outstanding frame prefetch) */
				auto probe = [&](const uint2 *hents, uint32_t hoff, uint32_t h,
						 uint32_t szm, uint32_t kvm) {
					for (uint32_t pr = 0; pr <= szm; ++pr) {
						const uint2 e = hents[hoff + h];

						if (e.y == HENT_EMPTY)
							break;
						if (e.x == kvm) {
							if (MODE == 1) {
								const uint64_t bit = 1ull << e.y;

								lo |= (uint32_t)bit;
								hi |= (uint32_t)(bit >> 32);
							} else {
								hrow[e.y >> 5] |= 1u << (e.y & 31u);
							}
						}
						h = (h + 1u) & szm;
					}
				};
				for (uint32_t gi = 0; gi < num_hgroups; ++gi) {
					const uint4 g0 = *(const uint4 *)(hgroups + gi);
					const uint2 g1 = *(const uint2 *)((const uint32_t *)(hgroups + gi) + 4);
					const uint32_t hslot = __builtin_amdgcn_readfirstlane(g0.x);
					const uint32_t hreq = __builtin_amdgcn_readfirstlane(g0.y);
					const uint32_t hmask = __builtin_amdgcn_readfirstlane(g0.z);
					const uint32_t lg = __builtin_amdgcn_readfirstlane(g0.w);
					const uint32_t hoff = __builtin_amdgcn_readfirstlane(g1.x);
					const uint32_t kvm = key(hslot) & hmask;

					if ((b.inf_lo & hreq) == hreq) {
						const uint32_t szm = (1u << lg) - 1u;
						const uint32_t h = (kvm * HASH_MUL) >> (32u - lg);

						if (hent_in_lds)
							probe(hents_l, hoff, h, szm, kvm);
						else
							probe((const uint2 *)hents_g, hoff, h, szm, kvm);
					}
				}
				for (uint32_t r = 0; r < num_runs; ++r) {
					const uint4 run = *(const uint4 *)(runs + r);
					const uint32_t slot = __builtin_amdgcn_readfirstlane(run.x);
					const uint32_t word = __builtin_amdgcn_readfirstlane(run.y);
					const uint32_t start = __builtin_amdgcn_readfirstlane(run.z);
					const uint32_t count = __builtin_amdgcn_readfirstlane(run.w);
					const uint32_t kv = key(slot);
					const uint4 *e = (const uint4 *)(simple + start);
					uint32_t acc = 0u;

#pragma unroll 8
					for (uint32_t q = 0; q < count; ++q) {
						const uint4 x = e[q];   /* req, mask, value, idx */
						const bool ok = ((b.inf_lo & x.x) == x.x) & ((kv & x.y) == x.z);

						acc |= ok ? (1u << (x.w & 31u)) : 0u;
					}
					const drun_t run_s = {slot, word, start, count};
					if (MODE == 1) {
						if (run_s.word == 0)
							lo |= acc;
						else
							hi |= acc;
					} else {
						hrow[run_s.word] |= acc;
					}
				}
				hits = ((uint64_t)hi << 32) | lo;
			} else {
				uint32_t acc = 0u;

				for (uint32_t pi = 0; pi < num_pmr; ++pi) {
					const dpmr_t pm = pmrs[pi];
					const bool ok = pmr_eval(terms, slots, pm.term_start, pm.nterms,
								 key, v, b);

					if (MODE == 1) {
						hits |= (uint64_t)ok << pi;
					} else {
						acc |= (uint32_t)ok << (pi & 31u);
						if ((pi & 31u) == 31u || pi + 1u == num_pmr) {
							hrow[pi >> 5] = acc;
							acc = 0u;
						}
					}
				}
			}
		}
		/* MODE 1: pinfo2 carries the destination's rule range, so each
		 * level costs one LDS read */
		uint32_t rs = 0u, nr = 0u;

		if (MODE == 1 && active) {
			const uint32_t ci = cinfo[cos].x;

			rs = ci & 0xffffu;
			nr = ci >> 16;
		}
		while (MODE == 1 && active) {
			const int k = first_hit64(hits, rs, nr);

			if (k < 0)
				break;
			const uint2 pi = pinfo2[rs + (uint32_t)k];

			cos = pi.x & 0xffffu;
			mark = pi.x >> 16;
			rs = pi.y & 0xffu;
			nr = (pi.y >> 8) & 0xffu;
			any_match = true;
			if (do_cos_stats && ((cinfo[cos].y >> 16) & 0xffu))
				atomicAdd(&cos_cnt[cos], 1u);
			if (++steps >= num_cos) {
				cos = ODPG_COS_LOOP;
				break;
			}
		}
		while (MODE == 2 && active) {
			const uint32_t ci = cinfo[cos].x;
			const uint32_t rs = ci & 0xffffu, nr = ci >> 16;
			const int k = first_hit_lds(hrow, rs, nr);

			if (k < 0)
				break;
			const uint32_t pi = pinfo[rs + (uint32_t)k];

			cos = pi & 0xffffu;
			mark = pi >> 16;
			any_match = true;
			if (do_cos_stats && ((cinfo[cos].y >> 16) & 0xffu))
				atomicAdd(&cos_cnt[cos], 1u);
			if (++steps >= num_cos) {
				cos = ODPG_COS_LOOP;
				break;
			}
		}
		active = false;
	}

	while (MODE == 0 && __ballot(active)) {
		if (active) {
			const uint32_t c = __builtin_amdgcn_readfirstlane(cos);

			if (cos == c) {
				const uint32_t cx = cinfo_g[c].x;   /* uniform: scalar load */
				const uint32_t rs = cx & 0xffffu, nr = cx >> 16;
				bool hit = false;
				uint32_t nd = 0u, nmark = 0u;

				for (uint32_t r = 0; r < nr; ++r) {
					const dpmr_t pm = pmrs[rs + r];
					bool ok = false;

					if (!hit)
						ok = pmr_match(terms, pm.term_start, pm.nterms, v, b);
					if (ok) {
						hit = true;
						nd = pm.dst;
						nmark = pm.mark;
					}
					if (do_cos_stats && ((cinfo_g[pm.dst].y >> 16) & 0xffu)) {
						uint64_t bm = __ballot(ok);

						if (bm && (__lane_id() == (uint32_t)__builtin_ctzll(__ballot(true))))
							atomicAdd(&cos_cnt[pm.dst], (uint32_t)__popcll(bm));
					}
					if (__ballot(!hit) == 0ull)
						break;
				}
				if (hit) {
					cos = nd;
					mark = nmark;
					any_match = true;
					if (++steps >= num_cos) {
						cos = ODPG_COS_LOOP;
						active = false;
					} else if ((cinfo_g[nd].x >> 16) == 0u) {
						active = false;
					}
				} else {
					active = false;
				}
			}
		}
	}

	if constexpr (GF) {
		if (defer) {
			run_tails();
			if (ret < 0) {
				want_cls = false;           /* pktin drop option */
			} else if (want_cls && (p.fl & FL_ERROR_MASK)) {
				/* cls_select_cos's error branch (no PMR walk) */
				cos = error_cos < 0 ? ODPG_COS_NONE : (uint32_t)error_cos;
				any_match = false;
				mark = 0u;
			}
		}
	}

	if (want_cls) {
		/* cls_select_cos() "done" path counts default / error CoS once
		 * (odp_classification.c:1696-1698): error packets, and packets
		 * that matched nothing below the default CoS */
		bool err = (p.fl & FL_ERROR_MASK) != 0u;
		bool at_done = err || !any_match;

		if (do_cos_stats && at_done && cos < num_cos &&
		    ((cinfo_at(cos).y >> 16) & 0xffu))
			atomicAdd(&cos_cnt[cos], 1u);

		if (cos == ODPG_COS_LOOP) {
			cret = -2;
		} else if (cos == ODPG_COS_NONE) {
			cret = -1;
		} else if ((cinfo_at(cos).y & 0xffu) == 1u) {
			cret = 1;
		} else {
			cret = 0;
			p.inf |= IF(IFL_DST_QUEUE);
		}
		if (any_match && !err && cos != ODPG_COS_LOOP) {
			p.inf &= ~IF(IFL_CLS_MARK);
			if (mark)
				p.inf |= IF(IFL_CLS_MARK);
		}
	} else if (live && ret < 0) {
		cos = ODPG_COS_PDROP;
	}

	/* ---- 4. outputs --------------------------------------------------- */
	if (live) {
		uint32_t w = cos & 0xffffu;

		if (cret == 1)
			w |= ODPG_OUT_CLS_DROP;
		if (cret == 0 && want_cls && (tbl_flags & TBL_ANY_HASHQ) &&
		    ((cinfo_at(cos).y >> 8) & 0xffu) > 1u) {
			/* rare path (hash-queue CoS): table read from global */
			const uint32_t cy = cinfo_at(cos).y;
			uint32_t h = rss_hash(p, v, cy >> 24);

			w |= ((h & 31u) % ((cy >> 8) & 0xffu)) << 24;
		}
		if (p.inf & IF(IFL_L3_CHKSUM_DONE))
			w |= (p.fl & FB(FL_L3_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 16;
		if (p.inf & IF(IFL_L4_CHKSUM_DONE))
			w |= (p.fl & FB(FL_L4_CHKSUM_ERR) ? ODPG_CHKSUM_BAD : ODPG_CHKSUM_OK) << 18;
		if (p.fl & FL_ERROR_MASK)
			w |= ODPG_OUT_ERROR;
		if (p.inf & IF(IFL_CLS_MARK))
			w |= ODPG_OUT_MARK_VALID;
		if (ret)
			w |= ODPG_OUT_PARSE_ERR;
		uint32_t mk = (p.inf & IF(IFL_CLS_MARK)) ? mark : 0u;

		/* packets handed to a CoS queue (_odp_cls_enq input; per-queue
		 * counters, odp_classification_internal.h:64-78) */
		if (cnt.row && cret == 0 && want_cls && cos < num_cos)
			atomicAdd(&dlv[cnt.qcol[cos] + ((w >> 24) & 31u)], 1u);
		if constexpr (FAST) {
			pend_i = i;
			pend_w = w;
			pend_mk = mk;
		} else {
			/* no frame prefetch to keep ahead of: store now, and no
			 * deferred-store registers live across the next tile */
			out[i] = w;
			if (mark_out)
				mark_out[i] = (uint16_t)mk;
		}
		if (meta_out) {
			odpg_meta_t m;

			m.input_flags = p.inf;
			m.flags = p.fl;
			m.l2_offset = (uint16_t)p.l2;
			m.l3_offset = (uint16_t)p.l3;
			m.l4_offset = (uint16_t)p.l4;
			m.cls_mark = (uint16_t)mk;
			m.reserved = 0u;
			meta_out[i] = m;
		}
	}

	/* ---- 5. loopback_recv accounting (loop.c:304-374), per lane ------- */
	if (do_stats) {
		const bool is_pkt = live && ret >= 0 && cret == 0 && !(p.fl & FL_ERROR_MASK);

		w_err += (uint32_t)__popcll(__ballot(live && layer && ret != 0));
		w_disc += (uint32_t)__popcll(__ballot(live && (cret == -1 || cret == -2)));
		w_pkt += (uint32_t)__popcll(__ballot(is_pkt));
		lane_oct += is_pkt ? (uint64_t)len : 0u;
	}
	pend = FAST && live;
	if (COOP)
		__syncthreads();          /* LDS rows are reused by the next tile */
	}   /* tile loop */
	if (pend) {
		out[pend_i] = pend_w;
		if (mark_out)
			mark_out[pend_i] = (uint16_t)pend_mk;
	}

	/* ---- 6. per-workgroup counter partials ---------------------------- */
	if (do_stats) {
		uint64_t a = w_pkt, o = wave_sum_u64(lane_oct);
		uint64_t e = w_err, d = w_disc;

		if (sred && !cnt.row) {
			/* pktio counters only: committed in-kernel (stats_commit.h) */
			const uint64_t v[4] = {a, o, e, d};

			stats_commit_wave(v, sred);
		} else if (__lane_id() == 0) {
			atomicAdd(&blk_pk[0], (unsigned long long)a);
			atomicAdd(&blk_pk[1], (unsigned long long)o);
			atomicAdd(&blk_pk[2], (unsigned long long)e);
			atomicAdd(&blk_pk[3], (unsigned long long)d);
		}
	}
	if ((do_stats && (!sred || cnt.row)) || do_cos_stats)
		__syncthreads();
	if (cnt.row) {
		/* this workgroup's row of the sharded counters (odpg.h) */
		uint64_t *r = cnt.row + (size_t)blockIdx.x * cnt.words;

		if (tid < 4 && blk_pk[tid])
			r[tid] += blk_pk[tid];
		if (do_cos_stats)
			for (uint32_t c = tid; c < num_cos && c < cnt.ncos; c += BLOCK)
				if (cos_cnt[c])
					r[4u + c] += cos_cnt[c];
		for (uint32_t c = tid; c < cnt.ncols; c += BLOCK)
			if (dlv[c])
				r[4u + cnt.ncos + c] += dlv[c];
		return;
	}
	if (do_stats && !sred && tid < 4)
		pk_partial[(size_t)blockIdx.x * 4u + tid] = blk_pk[tid];
	if (do_cos_stats)
		for (uint32_t c = tid; c < num_cos; c += BLOCK)
			cos_partial[(size_t)blockIdx.x * num_cos + c] = cos_cnt[c];
}

/* sum per-workgroup partials into the caller's 64-bit counters */
__global__ __launch_bounds__(BLOCK) void odpg_stats_reduce_kernel(
	const uint64_t *__restrict__ pk_partial, const uint32_t *__restrict__ cos_partial,
	uint32_t nblocks, uint32_t num_cos, uint64_t *__restrict__ stats)
{
	const uint32_t tid = threadIdx.x;
	const uint32_t nwords = 4u + (cos_partial ? num_cos : 0u);

	for (uint32_t wd = blockIdx.x; wd < nwords; wd += gridDim.x) {
		uint64_t s = 0;

		if (wd < 4u) {
			for (uint32_t bl = tid; bl < nblocks; bl += BLOCK)
				s += pk_partial[(size_t)bl * 4u + wd];
		} else {
			uint32_t c = wd - 4u;

			for (uint32_t bl = tid; bl < nblocks; bl += BLOCK)
				s += cos_partial[(size_t)bl * num_cos + c];
		}
		s = wave_sum_u64(s);
		__shared__ unsigned long long red[BLOCK / 64];

		if (__lane_id() == 0)
			red[tid / 64] = s;
		__syncthreads();
		if (tid == 0) {
			uint64_t t = 0;

			for (int k = 0; k < BLOCK / 64; ++k)
				t += red[k];
			stats[wd] += t;
		}
		__syncthreads();
	}
}

/* sharded counters (odpg.h): sum the rows into `sum` (zeroed by the caller)
 * and clear them. Block (64 columns x 4 row lanes), blockIdx.y a band of
 * FOLD_ROWS rows: coalesced 512-byte row segments, one atomic per column per
 * band. Stream-ordered after the launches that wrote the rows. */
#define FOLD_ROWS 32u

__global__ __launch_bounds__(BLOCK) void odpg_counters_fold_kernel(
	uint64_t *__restrict__ rows, uint32_t nrows, uint32_t words, uint64_t *__restrict__ sum)
{
	const uint32_t col = blockIdx.x * 64u + (threadIdx.x & 63u);
	const uint32_t ty = threadIdx.x >> 6;
	const uint32_t r0 = blockIdx.y * FOLD_ROWS;
	__shared__ unsigned long long part[BLOCK / 64][64];
	uint64_t s = 0;

	if (col < words)
		for (uint32_t r = r0 + ty; r < r0 + FOLD_ROWS && r < nrows; r += BLOCK / 64) {
			uint64_t *p = rows + (size_t)r * words + col;
			const uint64_t x = *p;

			if (x) {
				s += x;
				*p = 0ull;
			}
		}
	part[ty][threadIdx.x & 63u] = s;
	__syncthreads();
	if (ty == 0 && col < words) {
		for (uint32_t k = 1; k < BLOCK / 64; ++k)
			s += part[k][threadIdx.x];
		if (s)
			atomicAdd((unsigned long long *)&sum[col], (unsigned long long)s);
	}
}

extern "C" int odpg_launch_counters_fold(uint64_t *rows, uint32_t nrows, uint32_t words,
					 uint64_t *sum, hipStream_t s)
{
	const dim3 grid((words + 63u) / 64u, (nrows + FOLD_ROWS - 1u) / FOLD_ROWS);

	hipLaunchKernelGGL(odpg_counters_fold_kernel, grid, dim3(BLOCK), 0, s, rows, nrows, words, sum);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

/* ----------------------------------------------------------------------- */
/* host-side launch helper (called from runtime.cpp)                        */

extern "C" uint32_t odpg_launch_grid(uint32_t num);

/* dynamic LDS of one odpg_classify_kernel launch (its carve-up, kernel
 * prologue); mode 3 reads the walk groups through the hgroup / hent fields */
static size_t lds_need(const odpg_launch_args &a, int mode, int w)
{
	size_t lds = (size_t)BLOCK * (w / 4 + 1) * 4u;

	if (a.cos_partial || (a.cnt.row && a.cnt.cos))
		lds += (size_t)((a.num_cos + 3u) & ~3u) * 4u;
	if (a.cnt.row)
		lds += (size_t)((a.cnt.ncols + 3u) & ~3u) * 4u;
	if (mode == 2)
		lds += (size_t)BLOCK * (((a.num_pmr + 31u) >> 5) | 1u) * 4u;
	const bool use_mg = mode == 1 && (a.tbl_flags & TBL_MGROUPS);

	if (mode != 0 && !use_mg && a.num_hent <= HENT_LDS_MAX)
		lds += (size_t)a.num_hent * 8u;
	if (use_mg)
		lds += (size_t)a.num_ment * 16u;
	if (mode == 1)
		lds += (size_t)a.num_pmr * 8u + 4u;
	if (mode != 0)
		lds += (size_t)a.num_cos * 8u + (size_t)a.num_pmr * 4u;
	if (mode == 3 && (a.tbl_flags & TBL_XWALK))
		lds += (size_t)((a.num_cos + 1u) & ~1u) * 8u + (size_t)a.num_xwords * 4u + 16u;
	return lds;
}

/* Resident grid of a kernel at a dynamic LDS size: occupancy x CUs of the
 * current device, from hipOccupancyMaxActiveBlocksPerMultiprocessor; cached
 * per (kernel, LDS bytes, device) under a lock (contexts on several threads
 * and devices launch concurrently). */
extern "C" uint32_t odpg_resident_grid(const void *kernel, uint32_t block, size_t lds)
{
	struct Occ {
		const void *k;
		size_t lds;
		int dev;
		uint32_t block, grid;
	};
	static std::mutex m;
	static std::vector<Occ> cache;
	int dev = 0;

	hipGetDevice(&dev);
	{
		std::lock_guard<std::mutex> g(m);

		for (const Occ &o : cache)
			if (o.k == kernel && o.lds == lds && o.dev == dev && o.block == block)
				return o.grid;
	}
	int nb = 0, cus = 0;

	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, (int)block, lds) != hipSuccess ||
	    nb <= 0)
		nb = 1;
	const uint32_t grid = (uint32_t)(nb * (cus > 0 ? cus : 256));
	std::lock_guard<std::mutex> g(m);

	cache.push_back({kernel, lds, dev, block, grid});
	return grid;
}

/* the device's LDS per workgroup (160 KiB on gfx950), per device */
extern "C" size_t odpg_lds_limit(void)
{
	static size_t lim[64];
	int dev = 0;

	hipGetDevice(&dev);
	if (dev < 0 || dev >= 64)
		return 65536u;
	size_t v = __atomic_load_n(&lim[dev], __ATOMIC_RELAXED);

	if (!v) {
		hipDeviceProp_t pr;

		v = hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.sharedMemPerBlock ?
		    (size_t)pr.sharedMemPerBlock : 65536u;
		__atomic_store_n(&lim[dev], v, __ATOMIC_RELAXED);
	}
	return v;
}

/* frame row width a launch of this layout uses (launch_layout below) */
static int layout_w(const odpg_launch_args &a)
{
	if (a.desc)
		return 64;   /* GF_W */
	if (a.stride == 64 || a.stride == 128)
		return a.stride;
	return a.stride < 128 ? 128 : 96;
}

template <int W, bool COOP, bool GF, bool DESC, int MODE, bool FAST = false, bool LEAN = false>
static hipError_t launch_one(const odpg_launch_args &a, uint32_t &grid, hipStream_t s)
{
	const size_t lds = lds_need(a, MODE, W);
	/* persistent grid: exactly the workgroups that are resident at once
	 * (occupancy x CUs), each looping over tiles */
	const uint32_t occ_grid = odpg_resident_grid(
		(const void *)odpg_classify_kernel<W, COOP, GF, DESC, MODE, FAST, LEAN>, BLOCK, lds);

	if (!odpg_debug_env("ODPG_GRID_CAP") && grid > occ_grid)
		grid = occ_grid;
	if (a.cnt.row && grid > a.cnt.rows)
		grid = a.cnt.rows;   /* one counter row per workgroup */
	hipLaunchKernelGGL((odpg_classify_kernel<W, COOP, GF, DESC, MODE, FAST, LEAN>), dim3(grid),
			   dim3(BLOCK), lds, s, a.frames, a.desc, a.stride, a.num, a.opt, a.layer,
			   a.classify, a.terms, a.pmrs, a.coses, a.num_cos, a.default_cos,
			   a.error_cos, a.tbl_flags, a.num_pmr, a.slot_mask, a.slots, a.simple,
			   a.runs, a.num_runs, a.hgroups, a.num_hgroups, a.hents, a.num_hent,
			   (const uint2 *)a.cinfo, a.pinfo, a.mgroups, a.num_mgroups,
			   (const uint4 *)a.ments, a.num_ment, (const uint2 *)a.pinfo2, a.out, a.mark, a.meta, a.pk_partial,
			   a.cos_partial, a.pk_atomic ? a.sred : nullptr, (const uint2 *)a.xcos, a.xlist,
			   a.num_xlist, a.num_xwords, a.cnt);
	return hipGetLastError();
}

/* LDS window of the descriptor (IMIX) layout; the rest of a frame is read
 * from global memory. 64 B: the global tail then starts on a fresh 64-byte
 * line instead of re-fetching the window's second line (C3 305.7 -> 300.2 us
 * against a 96-byte window) */
#ifndef GF_W
#define GF_W 64
#endif

template <int MODE>
static hipError_t launch_layout(const odpg_launch_args &a, uint32_t &grid, hipStream_t s)
{
	if (a.desc)
		return launch_one<GF_W, false, true, true, MODE>(a, grid, s);
	if (a.stride == 64) {
		const bool lean = (a.tbl_flags & TBL_SIMPLE) &&
				  !(a.tbl_flags & (TBL_GENERIC | TBL_ANY_HASHQ)) && !a.mark &&
				  !a.meta && !a.stats;

		if ((MODE == 1 || MODE == 3) && lean)
			return launch_one<64, false, false, false, MODE, true, true>(a, grid, s);
		if (MODE != 0)   /* register fast path for plain frames */
			return launch_one<64, false, false, false, MODE, true>(a, grid, s);
		return launch_one<64, true, false, false, MODE>(a, grid, s);
	}
	if (a.stride == 128)
		return launch_one<128, true, false, false, MODE>(a, grid, s);
	if (a.stride < 128)
		return launch_one<128, false, false, false, MODE>(a, grid, s);
	return launch_one<96, false, true, false, MODE>(a, grid, s);
}

extern "C" int odpg_launch_cls64(const odpg_launch_args *a, hipStream_t s);

/* the lean 64-byte kernel (classify64.hip) covers this launch: fixed 64-byte
 * stride, a <= 64-PMR simple table whose gates its register parse computes,
 * verdict words and pktio counters only (no marks, metadata, CoS counters),
 * full parse with classification and no drop options */
static bool lean64_ok(const odpg_launch_args &a)
{
	static const bool off = odpg_debug_env("ODPG_NO_LEAN64") != nullptr;
	const uint64_t drops = ODPG_PKTIN_DROP_IPV4_ERR | ODPG_PKTIN_DROP_IPV6_ERR |
			       ODPG_PKTIN_DROP_UDP_ERR | ODPG_PKTIN_DROP_TCP_ERR |
			       ODPG_PKTIN_DROP_SCTP_ERR;

	const bool mg = (a.tbl_flags & TBL_LEAN64) && a.num_pmr <= MGROUP_MAX_PMR;
	const bool hw = (a.tbl_flags & TBL_LEAN64HW) && a.num_cgroups >= 1u && a.num_cgroups <= 4u &&
			a.num_cos < ODPG_COS_NOCLS;

	extern size_t odpg_cls64_lds(const odpg_launch_args &a);

	/* (its tile loads index the batch's 16-byte chunks in 32 bits) */
	return !off && a.mode == 0 && !a.desc && a.stride == 64 && (mg || hw) &&
	       a.num < (1u << 30) &&
	       odpg_cls64_lds(a) <= odpg_lds_limit() &&
	       !(a.tbl_flags & (TBL_GENERIC | TBL_ANY_HASHQ)) &&
	       !a.mark && !a.meta && !(a.stats && (a.tbl_flags & TBL_ANY_STATS)) &&
	       !(a.cnt.row && a.cnt.cos) &&
	       a.layer >= LAYER_L4 && a.classify &&
	       !(a.opt & drops) && !(a.opt >> 32);
}

extern "C" int odpg_launch_clsgf(const odpg_launch_args *a, hipStream_t s);
extern "C" size_t odpg_clsgf_lds(const odpg_launch_args *a);

/* the lean descriptor kernel (classify_gf.hip) covers this launch: a
 * descriptor batch, a hybrid hash-walk table in its hit-map form
 * (TBL_XMASK) without hash-queue CoS, verdict words and the sharded pktio /
 * per-queue counters (no CoS counters), full parse with classification and
 * no drop options */
static bool gf_ok(const odpg_launch_args &a)
{
	static const bool off = odpg_debug_env("ODPG_NO_GF") != nullptr;
	const uint64_t drops = ODPG_PKTIN_DROP_IPV4_ERR | ODPG_PKTIN_DROP_IPV6_ERR |
			       ODPG_PKTIN_DROP_UDP_ERR | ODPG_PKTIN_DROP_TCP_ERR |
			       ODPG_PKTIN_DROP_SCTP_ERR;

	/* descriptors, or a fixed stride whose offsets fit the kernel's 32 bits */
	const bool layout = a.desc || (a.stride && (uint64_t)a.num * a.stride <= 0xffffffffull);

	return !off && a.mode == 0 && layout && (a.tbl_flags & TBL_XMASK) &&
	       !(a.tbl_flags & TBL_ANY_HASHQ) && a.num_cos < ODPG_COS_NOCLS &&
	       odpg_clsgf_lds(&a) <= odpg_lds_limit() &&
	       !a.mark && !a.meta && !a.stats && !(a.cnt.row && a.cnt.cos) &&
	       a.layer >= LAYER_L4 && a.classify && !(a.opt & drops) && !(a.opt >> 32);
}

static int g_last_kernel = -1;

extern "C" int odpg_last_kernel(void)
{
	return __atomic_load_n(&g_last_kernel, __ATOMIC_RELAXED);
}

/* stats_commit.h: the slot sums of one classify launch into the caller's
 * counters (stream-ordered after it, so plain read-modify-writes), slots
 * re-zeroed for the next launch */
__global__ __launch_bounds__(64) void odpg_stats_fold_kernel(uint64_t *__restrict__ sred,
							      uint64_t *__restrict__ stats)
{
	const uint32_t g = threadIdx.x;
	uint64_t x[4];

#pragma unroll
	for (int w = 0; w < 4; ++w) {
		x[w] = sred[g * 8u + w];
		sred[g * 8u + w] = 0ull;
	}
#pragma unroll
	for (int w = 0; w < 4; ++w) {
		const uint64_t t = wave_sum_u64(x[w]);

		if (g == 0u && t)
			stats[w] += t;
	}
}

static int fold_stats(const odpg_launch_args *a, hipStream_t s)
{
	static_assert(SRED_GROUPS == 64u, "one fold lane per slot group");
	hipLaunchKernelGGL(odpg_stats_fold_kernel, dim3(1), dim3(64), 0, s, a->sred, a->pk_partial);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int odpg_launch_classify(const odpg_launch_args *a, hipStream_t s)
{
	if (a->num == 0)
		return 0;
	const bool lean = lean64_ok(*a);
	const bool gf = !lean && gf_ok(*a);

	__atomic_store_n(&g_last_kernel, lean ? 1 : gf ? 2 : 0, __ATOMIC_RELAXED);
	if (gf)
		return odpg_launch_clsgf(a, s);   /* counters folded at read time */
	if (lean) {
		int rc = odpg_launch_cls64(a, s);

		return rc ? rc : a->pk_atomic && !a->cnt.row ? fold_stats(a, s) : 0;
	}
	uint32_t grid = odpg_launch_grid(a->num);
	int mode = a->mode;
	hipError_t e;

	/* auto: single-word tables take evaluate-all (one probe per exact-match
	 * group, C2 23 vs 32 us for the hash walk) unless their groups repeat
	 * values across CoS (C4: every probe would walk ~15 equal keys; hash
	 * walk 38 vs 72 us); other tables take the walk, which only evaluates
	 * the rules of the CoS a packet visits (C3: 4x faster than evaluating
	 * all 256 generic PMRs per packet) */
	const bool simple = (a->tbl_flags & TBL_SIMPLE) != 0;

	if (mode == 0)
		mode = !simple && (a->tbl_flags & TBL_XWALK) ? 3
		       : simple && (a->tbl_flags & TBL_HASHWALK) && a->num_wgroups <= WALK_MAX_GROUPS ? 3
		       : simple && a->num_pmr <= EVAL_ALL_MAX_PMR ? 2
		       : simple && a->num_wgroups <= WALK_MAX_GROUPS ? 3 : 1;
	if (mode == 2 && a->num_pmr > EVAL_ALL_MAX_PMR)
		mode = 1;
	if (mode == 3 && !simple && !(a->tbl_flags & TBL_XWALK))
		mode = 1;
	{
		/* a table too large for a strategy's LDS carve-up (a hash-walk or
		 * hybrid-walk table near the raised limits) takes the walk, whose
		 * rule tables stay in global memory */
		odpg_launch_args w = *a;

		if (mode == 3) {
			w.num_hent = a->num_went;
			w.hgroups = a->wgroups;
		}
		const int kmode = mode == 1 ? 0 : mode == 2 ? (a->num_pmr <= 64 ? 1 : 2) : 3;

		if (kmode != 0 && lds_need(w, kmode, layout_w(*a)) > odpg_lds_limit())
			mode = 1;
	}
	if (mode == 3) {
		/* the hash walk reads its CoS-keyed groups through the
		 * exact-match group arguments */
		odpg_launch_args w = *a;

		w.hgroups = a->wgroups;
		w.num_hgroups = a->num_wgroups;
		w.hents = (const dhent_t *)a->wents;
		w.num_hent = a->num_went;
		e = launch_layout<3>(w, grid, s);
	} else if (mode == 1)
		e = launch_layout<0>(*a, grid, s);
	else if (a->num_pmr <= 64)
		e = launch_layout<1>(*a, grid, s);
	else
		e = launch_layout<2>(*a, grid, s);
	if (e != hipSuccess)
		return -EIO;
	if (a->cnt.row)
		return 0;   /* folded at read time (odpg_counters_fold) */
	if (a->pk_atomic)
		return fold_stats(a, s);
	if (a->stats && (a->pk_partial || a->cos_partial)) {
		uint32_t nwords = 4u + (a->cos_partial ? a->num_cos : 0u);
		uint32_t rgrid = nwords < 1024u ? nwords : 1024u;

		hipLaunchKernelGGL(odpg_stats_reduce_kernel, dim3(rgrid), dim3(BLOCK), 0, s,
				   a->pk_partial, a->cos_partial, grid, a->num_cos, a->stats);
		if (hipGetLastError() != hipSuccess)
			return -EIO;
	}
	return 0;
}

/* Workgroups loop over tiles. The launch uses the resident grid (occupancy x
 * CUs, launch_one) unless ODPG_GRID_CAP is set; this is the upper bound that
 * sizes the per-workgroup counter partials. */
#define DEFAULT_GRID_CAP 65536u

extern "C" uint32_t odpg_launch_grid(uint32_t num)
{
	static uint32_t cap = 0;

	if (cap == 0) {
		const char *e = odpg_debug_env("ODPG_GRID_CAP");
		long v = e ? strtol(e, nullptr, 0) : 0;

		cap = v > 0 ? (uint32_t)v : DEFAULT_GRID_CAP;
	}
	uint32_t tiles = (num + BLOCK - 1) / BLOCK;

	return tiles < cap ? tiles : cap;
}
