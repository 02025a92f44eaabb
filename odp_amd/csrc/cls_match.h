/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Classifier match helpers shared by the gfx950 classify kernels
 * (classify.hip: every layout and strategy; classify64.hip: the lean
 * 64-byte-stride kernel): parser bases, on-demand key slots and the
 * first-match scan of a u64 hit map (match_pmr_cos, odp_classification.c:
 * 1599-1642).
 */
#ifndef ODPG_CLS_MATCH_H_
#define ODPG_CLS_MATCH_H_

#include "pkt_parse.h"

/* compiled term evaluation (odp_classification.c:1338-1490 via cls_compile) */
struct Bases {
	uint32_t l2, l3, l4, vlanx, len, inf_lo;
};

/* ---- key slots on demand ------------------------------------------------
 * The word a compiled term compares (odpg_internal.h "key slots"), fetched
 * when a rule group needs it: from the frame registers on fast waves
 * (uniform switch), from the LDS window otherwise. No per-packet key array
 * is materialised (keeps register pressure and scratch at zero). */
template <int W, bool GF>
struct KeySrc {
	const uint32_t *f;     /* 16 frame registers (fast waves) or nullptr */
	const Pkt<W, GF> *v;
	const Bases *b;
	bool fast;

	__device__ __forceinline__ uint32_t operator()(uint32_t slot) const
	{
		if (fast) {
			const uint32_t (&r)[16] = *reinterpret_cast<const uint32_t (*)[16]>(f);
			const bool l4ok = b->l4 != 0xffffu;

			switch (slot) {
			case 0: return r[0];
			case 1: return r[1];
			case 2: return r[2];
			case 3: return r[3];
			case 4: return r[4];
			case 5: return fw<14>(r);
			case 6: return fw<14>(r);
			case 7: return fw<18>(r);
			case 8: return fw<22>(r);
			case 9: return fw<26>(r);
			case 10: return fw<30>(r);
			case 11: return fw<34>(r);
			case 12: return fw<38>(r);
			case 13: return fw<42>(r);
			case 14: return fw<46>(r);
			case 15: return fw<50>(r);
			case 16: return l4ok ? fw<34>(r) : 0u;
			case 17: return l4ok ? fw<38>(r) : 0u;
			default: return b->len;
			}
		}
		uint32_t pos;

		if (slot < SLOT_VLANX)
			pos = b->l2 + 4u * slot;
		else if (slot == SLOT_VLANX)
			pos = b->vlanx;
		else if (slot < SLOT_L4)
			pos = b->l3 + 4u * (slot - SLOT_L3);
		else if (slot < SLOT_LEN)
			pos = b->l4 + 4u * (slot - SLOT_L4);
		else
			return b->len;
		return v->rd32(pos);
	}
};

/* first set bit of the rule range [rs, rs + nr) in a per-lane hit map */
__device__ __forceinline__ int first_hit64(uint64_t hits, uint32_t rs, uint32_t nr)
{
	if (nr == 0u || rs >= 64u)
		return -1;
	uint64_t x = hits >> rs;

	if (nr < 64u)
		x &= (1ull << nr) - 1ull;
	return x ? (int)__builtin_ctzll(x) : -1;
}

#endif /* ODPG_CLS_MATCH_H_ */
