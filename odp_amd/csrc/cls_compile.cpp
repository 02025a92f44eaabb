/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Rule-table compiler: odpg_rules_t (a snapshot of the reference's CoS/PMR
 * data model, odp_classification_datamodel.h:66-174) -> flat immutable device
 * table (odpg_internal.h). Runs on the host once per table generation.
 *
 * Each reference term matcher (odp_classification.c:906-1332) is lowered to
 * a byte-wise masked compare at a parser-relative offset. The lowering keeps
 * the reference's raw-memory compare semantics: values and masks are the
 * caller's bytes (network order, except ODP_PMR_LEN which is CPU endian).
 */
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <algorithm>
#include <map>
#include <tuple>
#include <vector>

#include "../../include/odpg.h"
#include "odpg_internal.h"
#include "cls_compile.h"

namespace {

dterm_t make_cmp(uint32_t req, uint8_t base, int32_t off, const uint8_t *mask,
		 const uint8_t *value, uint32_t nbytes, uint8_t tflags = 0)
{
	dterm_t t;

	memset(&t, 0, sizeof(t));
	t.kind = DK_CMP;
	t.base = base;
	t.req = req;
	t.off = off;
	t.size = nbytes;
	t.nwords = (uint8_t)((nbytes + 3) / 4);
	t.tflags = tflags;
	uint8_t m[16] = {0}, v[16] = {0};

	memcpy(m, mask, nbytes);
	memcpy(v, value, nbytes);
	memcpy(t.mask, m, 16);
	memcpy(t.value, v, 16);
	return t;
}

dterm_t make_never()
{
	dterm_t t;

	memset(&t, 0, sizeof(t));
	t.kind = DK_NEVER;
	return t;
}

#define RQ(bit) (1u << (bit))

/* Lower one reference term; appends 0, 1 or 2 compiled entries. */
int lower_term(const odpg_term_t *src, std::vector<dterm_t> &out)
{
	const uint8_t *m = src->mask, *v = src->value;
	uint32_t sz = src->val_sz;

	if (sz > 16)
		return -EINVAL;

	switch (src->term) {
	case PMR_LEN: {                           /* verify_pmr_packet_len :906-914 */
		dterm_t t;

		memset(&t, 0, sizeof(t));
		t.kind = DK_LEN;
		memcpy(t.mask, m, sz < 4 ? sz : 4);
		memcpy(t.value, v, sz < 4 ? sz : 4);
		out.push_back(t);
		return 0;
	}
	case PMR_ETHTYPE_0:                       /* :1290-1307 eth->type */
		out.push_back(make_cmp(RQ(IFL_ETH), DB_L2, 12, m, v, sz));
		return 0;
	case PMR_ETHTYPE_X:                       /* :1309-1332 innermost vlan->type */
		/* vlan_qinq is only ever set together with vlan (odp_parse.c:74-82),
		 * so "vlan || vlan_qinq" == vlan */
		out.push_back(make_cmp(RQ(IFL_VLAN), DB_VLANX, 2, m, v, sz));
		return 0;
	case PMR_VLAN_ID_0:                       /* :1132-1153 tci & be16(0x0fff) */
	case PMR_VLAN_ID_X: {                     /* :1155-1180 */
		uint8_t mm[2] = { (uint8_t)(m[0] & 0x0f), m[1] };

		if (src->term == PMR_VLAN_ID_0)
			out.push_back(make_cmp(RQ(IFL_ETH) | RQ(IFL_VLAN), DB_L2, 14, mm, v, sz));
		else
			out.push_back(make_cmp(RQ(IFL_VLAN), DB_VLANX, 0, mm, v, sz));
		return 0;
	}
	case PMR_VLAN_PCP_0: {                    /* :1182-1202 pcp = be16(tci) >> 13 */
		if (v[0] & ~0x07) {               /* pcp & mask can never equal value */
			out.push_back(make_never());
			return 0;
		}
		uint8_t mm = (uint8_t)((m[0] & 0x07) << 5), vv = (uint8_t)(v[0] << 5);

		out.push_back(make_cmp(RQ(IFL_ETH) | RQ(IFL_VLAN), DB_L2, 14, &mm, &vv, 1));
		return 0;
	}
	case PMR_DMAC:                            /* :1062-1084 */
		out.push_back(make_cmp(RQ(IFL_ETH), DB_L2, 0, m, v, sz));
		return 0;
	case PMR_IPPROTO:                         /* :1397-1407 ipv4->proto / ipv6->next_hdr */
		out.push_back(make_cmp(RQ(IFL_IPV4), DB_L3, 9, m, v, sz, DT_ALT_NEXT));
		out.push_back(make_cmp(RQ(IFL_IPV6), DB_L3, 6, m, v, sz));
		return 0;
	case PMR_IP_DSCP: {                       /* :1408-1418, :938-958 */
		if (v[0] & ~0x3f) {
			out.push_back(make_never());
			return 0;
		}
		uint8_t m6 = m[0] & 0x3f, v6 = v[0];
		/* v4: dscp = (tos & 0xfc) >> 2 */
		uint8_t m4 = (uint8_t)(m6 << 2), v4 = (uint8_t)(v6 << 2);
		/* v6: dscp = (be32(ver_tc_flow) >> 22) & 0x3f = bits of bytes 0..1 */
		uint8_t mv6[2] = { (uint8_t)(m6 >> 2), (uint8_t)((m6 & 3) << 6) };
		uint8_t vv6[2] = { (uint8_t)(v6 >> 2), (uint8_t)((v6 & 3) << 6) };

		out.push_back(make_cmp(RQ(IFL_IPV4), DB_L3, 1, &m4, &v4, 1, DT_ALT_NEXT));
		out.push_back(make_cmp(RQ(IFL_IPV6), DB_L3, 0, mv6, vv6, 2));
		return 0;
	}
	case PMR_UDP_DPORT:                       /* :1028-1043 */
		out.push_back(make_cmp(RQ(IFL_UDP), DB_L4, 2, m, v, sz));
		return 0;
	case PMR_TCP_DPORT:                       /* :1011-1026 */
		out.push_back(make_cmp(RQ(IFL_TCP), DB_L4, 2, m, v, sz));
		return 0;
	case PMR_UDP_SPORT:                       /* :1045-1060 */
		out.push_back(make_cmp(RQ(IFL_UDP), DB_L4, 0, m, v, sz));
		return 0;
	case PMR_TCP_SPORT:                       /* :994-1009 */
		out.push_back(make_cmp(RQ(IFL_TCP), DB_L4, 0, m, v, sz));
		return 0;
	case PMR_SIP_ADDR:                        /* :960-975 */
		out.push_back(make_cmp(RQ(IFL_IPV4), DB_L3, 12, m, v, sz));
		return 0;
	case PMR_DIP_ADDR:                        /* :977-992 */
		out.push_back(make_cmp(RQ(IFL_IPV4), DB_L3, 16, m, v, sz));
		return 0;
	case PMR_SIP6_ADDR:                       /* :1086-1107 */
		out.push_back(make_cmp(RQ(IFL_IPV6), DB_L3, 8, m, v, sz));
		return 0;
	case PMR_DIP6_ADDR:                       /* :1109-1130 */
		out.push_back(make_cmp(RQ(IFL_IPV6), DB_L3, 24, m, v, sz));
		return 0;
	case PMR_IPSEC_SPI:                       /* :1204-1223 AH spi @4, ESP spi @0 */
		out.push_back(make_cmp(RQ(IFL_IPSEC_AH), DB_L4, 4, m, v, sz, DT_ALT_NEXT));
		out.push_back(make_cmp(RQ(IFL_IPSEC_ESP), DB_L4, 0, m, v, sz));
		return 0;
	case PMR_CUSTOM_FRAME:                    /* :1233-1257 */
		out.push_back(make_cmp(0, DB_ABS, (int32_t)src->offset, m, v, sz, DT_GUARD));
		return 0;
	case PMR_CUSTOM_L3:                       /* :1259-1288 (l2 flag, l3 valid) */
		out.push_back(make_cmp(RQ(IFL_L2), DB_L3, (int32_t)src->offset, m, v, sz, DT_GUARD));
		return 0;
	case PMR_INNER_HDR_OFF:                   /* :1479-1480 always passes */
		return 0;
	case PMR_LD_VNI:                          /* :1225-1231 unimplemented -> 0 */
	default:                                  /* :1481-1483 */
		out.push_back(make_never());
		return 0;
	}
}

/* Re-express a compiled term as a compare of consecutive key slots
 * (odpg_internal.h), or SLOT_NONE when it must use the generic compare. */
dslot_t slotify(const dterm_t &t)
{
	dslot_t s;

	memset(&s, 0, sizeof(s));
	s.slot = SLOT_NONE;
	if (t.kind == DK_LEN) {
		s.slot = SLOT_LEN;
		s.nw = 1;
		s.mask[0] = t.mask[0];
		s.value[0] = t.value[0];
		return s;
	}
	if (t.kind == DK_NEVER) {
		s.slot = 0;
		s.nw = 1;
		s.mask[0] = 0;
		s.value[0] = 1;    /* (x & 0) == 1 never holds */
		return s;
	}
	if (t.kind != DK_CMP || (t.tflags & DT_GUARD) || t.size == 0 || t.off < 0)
		return s;

	int first, count;

	switch (t.base) {
	case DB_L2:
		first = SLOT_L2;
		count = SLOT_VLANX - SLOT_L2;
		break;
	case DB_VLANX:
		first = SLOT_VLANX;
		count = 1;
		break;
	case DB_L3:
		first = SLOT_L3;
		count = SLOT_L4 - SLOT_L3;
		break;
	case DB_L4:
		first = SLOT_L4;
		count = SLOT_LEN - SLOT_L4;
		break;
	default:
		return s;
	}
	uint32_t w0 = (uint32_t)t.off / 4, w1 = ((uint32_t)t.off + t.size - 1) / 4;

	if (w1 >= (uint32_t)count || w1 - w0 + 1 > 4)
		return s;
	for (uint32_t j = 0; j < t.size; j++) {
		uint32_t mb = (t.mask[j / 4] >> (8 * (j % 4))) & 0xff;
		uint32_t vb = (t.value[j / 4] >> (8 * (j % 4))) & 0xff;
		uint32_t pos = (uint32_t)t.off + j;
		uint32_t w = pos / 4 - w0, lane = pos % 4;

		s.mask[w] |= mb << (8 * lane);
		s.value[w] |= vb << (8 * lane);
	}
	s.slot = (uint8_t)(first + w0);
	s.nw = (uint8_t)(w1 - w0 + 1);
	/* words with zero mask and value compare equal for every packet: drop
	 * them from both ends (a SIP6 /124 suffix becomes one word) */
	while (s.nw > 1 && s.mask[s.nw - 1] == 0 && s.value[s.nw - 1] == 0)
		s.nw--;
	while (s.nw > 1 && s.mask[0] == 0 && s.value[0] == 0) {
		for (uint32_t w = 0; w + 1 < s.nw; w++) {
			s.mask[w] = s.mask[w + 1];
			s.value[w] = s.value[w + 1];
		}
		s.mask[s.nw - 1] = s.value[s.nw - 1] = 0;
		s.nw--;
		s.slot++;
	}
	return s;
}

} /* namespace */

/* Two-choice cuckoo placement of one mask group's distinct values
 * (odpg_internal.h "Mask groups"). Deterministic: multipliers come from a
 * fixed sequence; the table doubles when no pair places every value. */
/* two-choice cuckoo table of (value, cos | pmr << 16) keyed by
 * cgroup_key(value, cos); g.shift / m1 / m2 / off / count as dmgroup_t.
 * Free entries are {0, HENT_EMPTY}: their CoS field (0xffff) is never a
 * packet's CoS. Returns -1 if no placement is found. */
static int build_cgroup(const std::vector<std::pair<uint32_t, uint32_t>> &keys, dmgroup_t &g,
			std::vector<dwent_t> &ents)
{
	const size_t n = keys.size();
	uint32_t lg = 1;

	while ((1u << lg) < 2 * n)
		lg++;
	uint64_t seed = 0xC2B2AE3D27D4EB4Full;
	auto next_mul = [&]() {
		seed ^= seed << 13;
		seed ^= seed >> 7;
		seed ^= seed << 17;
		return (uint32_t)(seed >> 32) | 1u;
	};
	std::vector<uint32_t> x(n);

	for (size_t k = 0; k < n; k++)
		x[k] = cgroup_key(keys[k].first, keys[k].second & 0xffffu);
	for (; lg <= 20; lg++) {
		const uint32_t sz = 1u << lg, sh = 32u - lg;

		for (int attempt = 0; attempt < 64; attempt++) {
			const uint32_t m1 = next_mul(), m2 = next_mul();
			std::vector<int> slot(sz, -1);
			bool ok = true;

			for (size_t k = 0; k < n && ok; k++) {
				int cur = (int)k;
				uint32_t pos = (x[k] * m1) >> sh;

				for (int kick = 0;; kick++) {
					if (kick > 4 * (int)sz + 16) {
						ok = false;
						break;
					}
					std::swap(cur, slot[pos]);
					if (cur < 0)
						break;
					uint32_t p1 = (x[cur] * m1) >> sh, p2 = (x[cur] * m2) >> sh;

					pos = pos == p1 ? p2 : p1;
				}
			}
			if (!ok)
				continue;
			g.shift = sh;
			g.m1 = m1;
			g.m2 = m2;
			g.off = (uint32_t)ents.size();
			g.count = (uint32_t)n;
			ents.resize(ents.size() + sz, dwent_t{0u, HENT_EMPTY});
			for (uint32_t s2 = 0; s2 < sz; s2++)
				if (slot[s2] >= 0)
					ents[g.off + s2] = dwent_t{keys[slot[s2]].first, keys[slot[s2]].second};
			return 0;
		}
	}
	return -1;
}

static void build_mgroup(const std::map<uint32_t, uint64_t> &vals, dmgroup_t &g,
			 std::vector<dment_t> &ents)
{
	const size_t n = vals.size();
	uint32_t lg = 1;

	if (n == 1) {
		/* inline single value: {value, lo, hi} in {m1, m2, off}, no entries */
		g.count = 1;
		g.shift = 31;
		g.m1 = vals.begin()->first;
		g.m2 = (uint32_t)vals.begin()->second;
		g.off = (uint32_t)(vals.begin()->second >> 32);
		return;
	}

	while ((1u << lg) < 2 * n)
		lg++;
	uint64_t seed = 0x9E3779B97F4A7C15ull;
	auto next_mul = [&]() {
		seed ^= seed << 13;
		seed ^= seed >> 7;
		seed ^= seed << 17;
		return (uint32_t)(seed >> 32) | 1u;
	};
	/* A collision-free single-probe hash, when one exists within the cuckoo
	 * table's size: m1 == m2, so a lookup reads one entry (the lean kernel
	 * tests m1 == m2 wave-uniformly; the other kernels read the same entry
	 * twice, harmlessly). Power-of-two multipliers first: they extract a bit
	 * field of the key, which separates structured values such as a port
	 * range or the prefix bits of a subnet list; then random multipliers. */
#ifndef ODPG_NO_PERFECT      /* experiment builds only: cuckoo groups */
	{
		uint32_t plg = 1;

		while ((1u << plg) < n)
			plg++;
		for (; plg <= lg; plg++) {
			const uint32_t sz = 1u << plg, sh = 32u - plg;

			for (int attempt = 0; attempt < 32 + 64; attempt++) {
				const uint32_t m = attempt < 32 ? 1u << attempt : next_mul();
				std::vector<int> slot(sz, -1);
				bool ok = true;
				int k = 0;

				for (auto it = vals.begin(); it != vals.end() && ok; ++it, ++k) {
					const uint32_t pos = (it->first * m) >> sh;

					if (slot[pos] >= 0)
						ok = false;
					else
						slot[pos] = k;
				}
				if (!ok)
					continue;
				g.shift = sh;
				g.m1 = m;
				g.m2 = m;
				g.off = (uint32_t)ents.size();
				g.count = (uint32_t)n;
				ents.resize(ents.size() + sz, dment_t{0u, 0u, 0u, 0u});
				for (auto &v : vals) {
					dment_t &e = ents[g.off + ((v.first * m) >> sh)];

					e.value = v.first;
					e.lo = (uint32_t)v.second;
					e.hi = (uint32_t)(v.second >> 32);
				}
				return;
			}
		}
	}
#endif
	for (;; lg++) {
		const uint32_t sz = 1u << lg, sh = 32u - lg;

		for (int attempt = 0; attempt < 64; attempt++) {
			const uint32_t m1 = next_mul(), m2 = next_mul();
			std::vector<int> slot(sz, -1);
			std::vector<uint32_t> key;
			bool ok = true;

			for (auto &v : vals)
				key.push_back(v.first);
			for (size_t k = 0; k < n && ok; k++) {
				int cur = (int)k;
				uint32_t pos = (key[k] * m1) >> sh;

				for (int kick = 0;; kick++) {
					if (kick > 4 * (int)sz + 16) {
						ok = false;
						break;
					}
					std::swap(cur, slot[pos]);
					if (cur < 0)
						break;
					/* move the evicted value to its other slot */
					uint32_t p1 = (key[cur] * m1) >> sh, p2 = (key[cur] * m2) >> sh;

					pos = pos == p1 ? p2 : p1;
				}
			}
			if (!ok)
				continue;
			g.shift = sh;
			g.m1 = m1;
			g.m2 = m2;
			g.off = (uint32_t)ents.size();
			g.count = (uint32_t)n;
			ents.resize(ents.size() + sz, dment_t{0u, 0u, 0u, 0u});
			std::vector<uint64_t> bits;

			for (auto &v : vals)
				bits.push_back(v.second);
			for (uint32_t s = 0; s < sz; s++) {
				if (slot[s] < 0)
					continue;
				dment_t &e = ents[g.off + s];

				e.value = key[slot[s]];
				e.lo = (uint32_t)bits[slot[s]];
				e.hi = (uint32_t)(bits[slot[s]] >> 32);
			}
			return;
		}
	}
}

int odpg_compile_rules(const odpg_rules_t *r, std::vector<uint8_t> &blob, dtable_hdr_t *hdr_out)
{
	std::vector<dcos_t> cos;
	std::vector<dpmr_t> pmr;
	std::vector<dterm_t> terms;

	if (!r || r->num_cos > ODPG_MAX_COS || (r->num_cos && !r->cos))
		return -EINVAL;
	if (r->default_cos >= (int32_t)r->num_cos || r->error_cos >= (int32_t)r->num_cos)
		return -EINVAL;

	/* CoS slots past the last valid or referenced one can never be reached */
	uint32_t ncos = 0;

	for (uint32_t c = 0; c < r->num_cos; c++) {
		if (r->cos[c].valid)
			ncos = c + 1;
		for (uint32_t i = 0; i < r->cos[c].num_rule && r->cos[c].valid; i++) {
			uint32_t slot = r->cos[c].rule_start + i;

			if (slot < r->num_slots && r->rule_dst[slot] + 1 > ncos &&
			    r->rule_dst[slot] < r->num_cos)
				ncos = r->rule_dst[slot] + 1;
		}
	}
	if (r->default_cos >= 0 && (uint32_t)r->default_cos + 1 > ncos)
		ncos = (uint32_t)r->default_cos + 1;
	if (r->error_cos >= 0 && (uint32_t)r->error_cos + 1 > ncos)
		ncos = (uint32_t)r->error_cos + 1;

	cos.resize(ncos);
	for (uint32_t c = 0; c < ncos; c++) {
		const odpg_cos_t *ce = &r->cos[c];
		dcos_t &d = cos[c];

		memset(&d, 0, sizeof(d));
		d.valid = ce->valid ? 1 : 0;
		d.action = (uint8_t)ce->action;
		d.num_queue = (uint8_t)(ce->num_queue ? ce->num_queue : 1);
		d.hash_proto = (uint8_t)ce->hash_proto;
		d.stats = ce->stats_enable ? 1 : 0;
		d.rule_start = (uint32_t)pmr.size();
		if (ce->num_queue > ODPG_COS_QUEUE_MAX || ce->num_rule > ODPG_MAX_RULES_PER_COS)
			return -EINVAL;

		for (uint32_t i = 0; i < ce->num_rule; i++) {
			uint32_t slot = ce->rule_start + i;

			if (slot >= r->num_slots)
				return -EINVAL;
			uint32_t pi = r->rule_pmr[slot], dst = r->rule_dst[slot];

			if (pi >= r->num_pmr || dst >= r->num_cos)
				return -EINVAL;
			/* match_pmr_cos skips rules whose linked CoS is invalid
			 * (odp_classification.c:1610-1611); the snapshot is
			 * immutable, so drop them here. */
			if (!r->cos[dst].valid)
				continue;
			const odpg_pmr_t *p = &r->pmr[pi];
			dpmr_t dp;

			if (p->num_terms > ODPG_MAX_TERMS)
				return -EINVAL;
			dp.term_start = (uint32_t)terms.size();
			for (uint32_t t = 0; t < p->num_terms; t++) {
				int rc = lower_term(&p->terms[t], terms);

				if (rc)
					return rc;
			}
			if (terms.size() > 65535)
				return -E2BIG;
			dp.nterms = (uint32_t)(terms.size() - dp.term_start);
			dp.mark = p->mark & 0xffffu;
			dp.dst = dst;
			pmr.push_back(dp);
			if (pmr.size() > ODPG_MAX_PMR * 4)
				return -E2BIG;
		}
		d.nrule = (uint16_t)(pmr.size() - d.rule_start);
	}

	/* key-slot forms and the compact single-compare table */
	std::vector<dslot_t> slots(terms.size());
	std::vector<dsimple_t> simple;
	uint32_t slot_mask = 0;
	bool is_simple = true;

	for (size_t k = 0; k < terms.size(); k++) {
		slots[k] = slotify(terms[k]);
		if (slots[k].slot != SLOT_NONE)
			for (uint32_t w = 0; w < slots[k].nw; w++)
				slot_mask |= 1u << (slots[k].slot + w);
	}
	std::vector<uint32_t> simple_slot;
	bool generic = false;

	for (size_t k = 0; k < terms.size(); k++)
		if (slots[k].slot == SLOT_NONE && terms[k].kind == DK_CMP)
			generic = true;
	/* every PMR's single-word form for the walk groups, or "complex" (the
	 * hybrid hash walk evaluates those rules with the generic compare) */
	std::vector<dsimple_t> wsimple;
	std::vector<uint32_t> wsimple_slot;
	std::vector<bool> complex_pmr(pmr.size(), false);

	for (size_t pi = 0; pi < pmr.size(); pi++) {
		const dpmr_t &p = pmr[pi];
		dsimple_t e;

		memset(&e, 0, sizeof(e));
		e.idx = (uint32_t)pi;
		if (p.nterms == 0) {
			wsimple.push_back(e);
			wsimple_slot.push_back(0);
			continue;
		}
		const dterm_t &t = terms[p.term_start];
		const dslot_t &sl = slots[p.term_start];

		if (p.nterms == 2 && (t.tflags & DT_ALT_NEXT)) {
			/* IPv4 / IPv6 (or AH / ESP) alternative pair: the gates
			 * are exclusive parse results, so "first gate ? cmp1 :
			 * gate2 && cmp2" is the disjunction of two gated compares
			 * and the PMR goes into both of their groups */
			const dterm_t &t2 = terms[p.term_start + 1];
			const dslot_t &s2 = slots[p.term_start + 1];
			const bool excl = ((t.req & RQ(IFL_IPV4)) && (t2.req & RQ(IFL_IPV6))) ||
					  ((t.req & RQ(IFL_IPSEC_AH)) && (t2.req & RQ(IFL_IPSEC_ESP)));

			if (excl && sl.slot != SLOT_NONE && sl.nw == 1 && s2.slot != SLOT_NONE &&
			    s2.nw == 1 && !(t2.tflags & DT_ALT_NEXT)) {
				e.req = t.req;
				e.mask = sl.mask[0];
				e.value = sl.value[0];
				wsimple.push_back(e);
				wsimple_slot.push_back(sl.slot);
				e.req = t2.req;
				e.mask = s2.mask[0];
				e.value = s2.value[0];
				wsimple.push_back(e);
				wsimple_slot.push_back(s2.slot);
				continue;
			}
		}
		if (p.nterms != 1 || sl.slot == SLOT_NONE || sl.nw != 1 || (t.tflags & DT_ALT_NEXT)) {
			complex_pmr[pi] = true;
			continue;
		}
		e.req = t.req;
		e.mask = sl.mask[0];
		e.value = sl.value[0];
		wsimple.push_back(e);
		wsimple_slot.push_back(sl.slot);
	}
	size_t num_complex = 0;

	for (size_t pi = 0; pi < pmr.size(); pi++)
		num_complex += complex_pmr[pi] ? 1 : 0;

	for (size_t pi = 0; pi < pmr.size(); pi++) {
		const dpmr_t &p = pmr[pi];
		dsimple_t e;

		memset(&e, 0, sizeof(e));
		e.idx = (uint32_t)pi;
		if (p.nterms == 0) {
			simple.push_back(e);            /* no terms: always matches */
			simple_slot.push_back(0);
			continue;
		}
		const dterm_t &t = terms[p.term_start];
		const dslot_t &sl = slots[p.term_start];

		if (p.nterms != 1 || sl.slot == SLOT_NONE || sl.nw != 1 || (t.tflags & DT_ALT_NEXT)) {
			is_simple = false;
			break;
		}
		e.req = t.req;
		e.mask = sl.mask[0];
		e.value = sl.value[0];
		simple.push_back(e);
		simple_slot.push_back(sl.slot);
	}
	std::vector<drun_t> runs;
	std::vector<dhgroup_t> hgroups;
	std::vector<dhent_t> hents;
	std::vector<dhgroup_t> wgroups;
	std::vector<dwent_t> wents;

	/* hybrid hash walk (TBL_XWALK): walk groups over the single-word PMRs
	 * of a table that also holds a few complex ones */
	const bool xwalk = !is_simple && num_complex * 2 <= pmr.size() && pmr.size() < 65536 &&
			   ncos < 65536;
	std::vector<uint32_t> src_cos(pmr.size(), 0);

	for (uint32_t c = 0; c < ncos; c++)
		for (uint32_t k = 0; k < cos[c].nrule; k++)
			src_cos[cos[c].rule_start + k] = c;
	if (is_simple || xwalk) {
		/* CoS-keyed walk groups over every single-word PMR (odpg_internal.h) */
		std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::vector<size_t>> by_key;

		for (size_t k = 0; k < wsimple.size(); k++)
			by_key[std::make_tuple(wsimple_slot[k], wsimple[k].req, wsimple[k].mask)].push_back(k);
		for (auto &kv : by_key) {
			/* lowest PMR index per (cos, value); values with bits outside
			 * the mask never match and are left out */
			std::map<std::pair<uint32_t, uint32_t>, uint32_t> first;

			for (size_t k : kv.second) {
				const dsimple_t &e = wsimple[k];

				if (e.value & ~e.mask)
					continue;
				auto key = std::make_pair(src_cos[e.idx], e.value);
				auto it = first.find(key);

				if (it == first.end() || e.idx < it->second)
					first[key] = e.idx;
			}
			uint32_t lg = 1;

			while ((1u << lg) < 2 * first.size())
				lg++;
			dhgroup_t g;

			memset(&g, 0, sizeof(g));
			g.slot = std::get<0>(kv.first);
			g.req = std::get<1>(kv.first);
			g.mask = std::get<2>(kv.first);
			g.log2sz = lg;
			g.off = (uint32_t)wents.size();
			g.count = (uint32_t)first.size();
			wents.resize(wents.size() + (1u << lg), dwent_t{0u, HENT_EMPTY});
			/* Robin Hood insertion (an entry displaced less than the one
			 * being placed gives up its slot): the same probe-until-empty
			 * lookup finds every key, and the longest displacement, which
			 * the hybrid walk probes branch-free, stays short */
			const uint32_t szm = (1u << lg) - 1u;

			for (auto &f : first) {
				dwent_t cur = {f.first.second, f.first.first | (f.second << 16)};
				uint32_t hsh = walk_hash(cur.value, cur.cos_pmr & 0xffffu, lg);
				uint32_t d = 0;

				while (wents[g.off + hsh].cos_pmr != HENT_EMPTY) {
					dwent_t &o = wents[g.off + hsh];
					const uint32_t od = (hsh - walk_hash(o.value, o.cos_pmr & 0xffffu, lg)) & szm;

					if (od < d) {
						std::swap(cur, o);
						d = od;
					}
					hsh = (hsh + 1) & szm;
					d++;
				}
				wents[g.off + hsh] = cur;
			}
			for (uint32_t e = 0; e <= szm; e++) {
				const dwent_t &o = wents[g.off + e];

				if (o.cos_pmr != HENT_EMPTY) {
					const uint32_t np = ((e - walk_hash(o.value, o.cos_pmr & 0xffffu, lg)) & szm) + 1;

					g.maxp = np > g.maxp ? np : g.maxp;
				}
			}
			wgroups.push_back(g);
		}
	}

	/* CoS-keyed cuckoo groups for the lean kernel's walk form: the same
	 * (cos, value) -> lowest PMR index maps as the walk groups above, as
	 * two-choice cuckoo tables (both candidates read at once, no probe
	 * chain) */
	std::vector<dmgroup_t> cgroups;
	std::vector<dwent_t> cents;

	for (size_t gi = 0; gi < wgroups.size() && wgroups.size() <= 4 && is_simple; gi++) {
		const dhgroup_t &wg = wgroups[gi];
		std::vector<std::pair<uint32_t, uint32_t>> keys;   /* (value, cos_pmr) */

		for (uint32_t e = 0; e < (1u << wg.log2sz); e++)
			if (wents[wg.off + e].cos_pmr != HENT_EMPTY)
				keys.push_back({wents[wg.off + e].value, wents[wg.off + e].cos_pmr});
		dmgroup_t g;

		memset(&g, 0, sizeof(g));
		g.slot = wg.slot;
		g.req = wg.req;
		g.mask = wg.mask;
		if (build_cgroup(keys, g, cents) != 0) {
			cgroups.clear();
			cents.clear();
			break;
		}
		cgroups.push_back(g);
	}

	/* TBL_XWALK: per CoS {xlist start | count << 16, walk-group mask}; per
	 * CoS its complex PMRs in rule order as {pmr, xterm start | n << 24},
	 * then the xterm records {req, mask, value, slot | guard end << 8 |
	 * guarded << 31} of the complex PMRs whose terms are all single-word
	 * slot compares (n > 0; n == 0: the generic compare) */
	std::vector<uint32_t> xcos, xlist, xterm;
	uint32_t num_xent = 0;
	/* one AND-chain of a PMR's terms as records: `pick` chooses, for each
	 * alternative pair (a term with DT_ALT_NEXT and the one after it: the
	 * IPv4 / IPv6 or AH / ESP forms of one reference term, whose gates
	 * exclude each other), which of the two is in the chain (bit j for the
	 * j-th pair) */
	auto slotted_terms = [&](const dpmr_t &p, std::vector<uint32_t> &rec, uint32_t pick) -> bool {
		uint32_t pair = 0;

		for (uint32_t k = 0; k < p.nterms; k++) {
			dterm_t t = terms[p.term_start + k];
			uint32_t gend = 0, guarded = 0;

			if (t.tflags & DT_ALT_NEXT) {
				if (k + 1 >= p.nterms)
					return false;
				if ((pick >> pair++) & 1u)
					t = terms[p.term_start + k + 1];
				k++;
			}
			uint32_t absolute = 0;

			if (t.tflags & DT_GUARD) {
				/* CUSTOM_L3: frame_len > l3 + off + size (the kernel's
				 * term_cmp guard) checked before the slot read;
				 * CUSTOM_FRAME: frame_len > off + size, the slot an
				 * absolute frame word (the L2 slots at l2 == 0) */
				if (t.kind != DK_CMP || (t.base != DB_L3 && t.base != DB_ABS) || t.off < 0)
					return false;
				gend = (uint32_t)t.off + t.size;
				guarded = 1;
				if (t.base == DB_ABS) {
					absolute = 1;
					t.base = DB_L2;
				}
				t.tflags &= (uint8_t)~DT_GUARD;
			}
			const dslot_t sl = slotify(t);

			if (sl.slot == SLOT_NONE || sl.nw < 1 || sl.nw > 4 || gend > 0xffffu ||
			    (guarded && sl.nw != 1))
				return false;
			/* a term over nw consecutive key slots (SIP6 / DIP6, DMAC) is the
			 * AND of nw single-word compares: one record per word, words
			 * whose mask and value are both zero dropped (always equal) */
			uint32_t nrec = 0;

			for (uint32_t w = 0; w < sl.nw; w++) {
				if (sl.mask[w] == 0u && sl.value[w] == 0u && !(w == 0u && sl.nw == 1u))
					continue;
				rec.push_back(t.req);
				rec.push_back(sl.mask[w]);
				rec.push_back(sl.value[w]);
				rec.push_back((sl.slot + w) | (gend << 8) | (absolute << 30) | (guarded << 31));
				nrec++;
			}
			if (nrec == 0u) {            /* every word always equal: gate only */
				rec.push_back(t.req);
				rec.push_back(0u);
				rec.push_back(0u);
				rec.push_back(sl.slot | (gend << 8) | (absolute << 30) | (guarded << 31));
			}
		}
		return p.nterms > 0;
	};

	if (xwalk && wgroups.size() <= XWALK_MAX_GROUPS) {
		std::vector<uint32_t> gm(ncos, 0u);

		for (size_t g = 0; g < wgroups.size(); g++)
			for (uint32_t e = 0; e < (1u << wgroups[g].log2sz); e++) {
				const dwent_t &w = wents[wgroups[g].off + e];

				if (w.cos_pmr != HENT_EMPTY)
					gm[w.cos_pmr & 0xffffu] |= 1u << g;
			}
		xcos.resize(2 * ncos);
		for (uint32_t c = 0; c < ncos; c++) {
			uint32_t st = (uint32_t)(xlist.size() / 2);

			for (uint32_t k = 0; k < cos[c].nrule; k++) {
				const uint32_t pi = cos[c].rule_start + k;

				if (!complex_pmr[pi])
					continue;
				/* a PMR with alternative pairs is the OR of its chains,
				 * one xlist entry each (same PMR index, consecutive:
				 * both kernels take the first entry that matches); up to
				 * two pairs, else the generic compare */
				uint32_t npair = 0;

				for (uint32_t k = 0; k < pmr[pi].nterms; k++)
					if (terms[pmr[pi].term_start + k].tflags & DT_ALT_NEXT)
						npair++;
				std::vector<std::vector<uint32_t>> chains;
				bool ok = npair <= 2;

				/* gates that no packet carries together: a chain needing
				 * both never matches and is left out */
				const uint32_t excl[][2] = {{RQ(IFL_IPV4), RQ(IFL_IPV6)},
							    {RQ(IFL_IPSEC_AH), RQ(IFL_IPSEC_ESP)}};

				for (uint32_t pick = 0; ok && pick < (1u << npair); pick++) {
					std::vector<uint32_t> r;

					ok = slotted_terms(pmr[pi], r, pick) && r.size() / 4 < 256u;
					uint32_t req = 0;

					for (size_t q = 0; q < r.size(); q += 4)
						req |= r[q];
					bool never = false;

					for (const auto &e : excl)
						never |= (req & e[0]) && (req & e[1]);
					if (ok && !never)
						chains.push_back(r);
				}
				if (ok && chains.empty())        /* no chain can match */
					chains.push_back({0u, 0u, 1u, 0u});   /* (x & 0) == 1: never */
				if (ok && xterm.size() / 4 + 64u < (1u << 24)) {
					for (const auto &r : chains) {
						xlist.push_back(pi);
						xlist.push_back((uint32_t)(xterm.size() / 4) |
								((uint32_t)(r.size() / 4) << 24));
						xterm.insert(xterm.end(), r.begin(), r.end());
					}
				} else {
					xlist.push_back(pi);
					xlist.push_back(0u);
				}
			}
			xcos[2 * c] = st | (((uint32_t)(xlist.size() / 2) - st) << 16);
			xcos[2 * c + 1] = gm[c];
		}
		num_xent = (uint32_t)(xlist.size() / 2);
		if (num_xent & 1u) {            /* xterm records start 16-byte aligned */
			xlist.push_back(0u);
			xlist.push_back(0u);
		}
		xlist.insert(xlist.end(), xterm.begin(), xterm.end());
		if (num_xent > 65535 || xlist.size() > (1u << 20)) {
			xcos.clear();
			xlist.clear();
			num_xent = 0;
		}
	}

	std::vector<dmgroup_t> mgroups;
	std::vector<dment_t> ments;

	if (is_simple && pmr.size() <= MGROUP_MAX_PMR) {
		/* mask groups over every PMR, in (slot, req, mask) order */
		std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::map<uint32_t, uint64_t>> by_key;

		for (size_t k = 0; k < simple.size(); k++) {
			const dsimple_t &e = simple[k];
			auto &vals = by_key[std::make_tuple(simple_slot[k], e.req, e.mask)];

			if (e.value & ~e.mask)
				continue;   /* can never match: no bit anywhere */
			vals[e.value] |= 1ull << e.idx;
		}
		for (auto &kv : by_key) {
			if (kv.second.empty())
				continue;
			dmgroup_t g;

			memset(&g, 0, sizeof(g));
			g.slot = std::get<0>(kv.first);
			g.req = std::get<1>(kv.first);
			g.mask = std::get<2>(kv.first);
			build_mgroup(kv.second, g, ments);
			mgroups.push_back(g);
		}
	}

	size_t dup_entries = 0, dup_distinct = 0;

	if (is_simple) {
		/* exact-match groups -> hash tables; the rest stays linear */
		std::vector<size_t> order(simple.size());

		for (size_t k = 0; k < order.size(); k++)
			order[k] = k;
		auto gkey = [&](size_t k) {
			return std::make_tuple(simple_slot[k], simple[k].req, simple[k].mask);
		};
		std::stable_sort(order.begin(), order.end(),
				 [&](size_t a, size_t b) { return gkey(a) < gkey(b); });
		std::vector<bool> hashed(simple.size(), false);

		for (size_t g0 = 0; g0 < order.size();) {
			size_t g1 = g0;

			while (g1 < order.size() && gkey(order[g1]) == gkey(order[g0]))
				g1++;
			size_t cnt = g1 - g0;
			bool ok = cnt >= HASH_MIN;

			for (size_t k = g0; k < g1 && ok; k++)
				if (simple[order[k]].value & ~simple[order[k]].mask)
					ok = false;   /* can never match: keep it linear */
			if (ok) {
				std::vector<uint32_t> vals;

				for (size_t k = g0; k < g1; k++)
					vals.push_back(simple[order[k]].value);
				std::sort(vals.begin(), vals.end());
				dup_entries += cnt;
				dup_distinct += (size_t)(std::unique(vals.begin(), vals.end()) - vals.begin());
				uint32_t lg = 3;

				while ((1u << lg) < 2 * cnt)
					lg++;
				dhgroup_t hg;

				memset(&hg, 0, sizeof(hg));
				hg.slot = simple_slot[order[g0]];
				hg.req = simple[order[g0]].req;
				hg.mask = simple[order[g0]].mask;
				hg.log2sz = lg;
				hg.off = (uint32_t)hents.size();
				hg.count = (uint32_t)cnt;
				hents.resize(hents.size() + (1u << lg), dhent_t{0u, HENT_EMPTY});
				for (size_t k = g0; k < g1; k++) {
					const dsimple_t &e = simple[order[k]];
					uint32_t h = (e.value * HASH_MUL) >> (32 - lg);

					while (hents[hg.off + h].idx != HENT_EMPTY)
						h = (h + 1) & ((1u << lg) - 1);
					hents[hg.off + h].value = e.value;
					hents[hg.off + h].idx = e.idx;
					hashed[order[k]] = true;
				}
				hgroups.push_back(hg);
			}
			g0 = g1;
		}
		std::vector<dsimple_t> lin;
		std::vector<uint32_t> lin_slot;

		for (size_t k = 0; k < simple.size(); k++)
			if (!hashed[k]) {
				lin.push_back(simple[k]);
				lin_slot.push_back(simple_slot[k]);
			}
		simple.swap(lin);
		simple_slot.swap(lin_slot);
	}

	if (is_simple) {
		/* order by (slot, hit word, index): one key-slot read and one
		 * hit-word update per run */
		std::vector<size_t> ord(simple.size());

		for (size_t k = 0; k < ord.size(); k++)
			ord[k] = k;
		std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
			uint64_t ka = ((uint64_t)simple_slot[a] << 40) | ((uint64_t)(simple[a].idx >> 5) << 20) | simple[a].idx;
			uint64_t kb = ((uint64_t)simple_slot[b] << 40) | ((uint64_t)(simple[b].idx >> 5) << 20) | simple[b].idx;
			return ka < kb;
		});
		std::vector<dsimple_t> sorted;

		for (size_t k = 0; k < ord.size(); k++) {
			const dsimple_t &e = simple[ord[k]];
			uint32_t sl = simple_slot[ord[k]], wd = e.idx >> 5;

			if (runs.empty() || runs.back().slot != sl || runs.back().word != wd ||
			    runs.back().count == 0xffffu) {
				drun_t r;

				memset(&r, 0, sizeof(r));
				r.slot = sl;
				r.word = wd;
				r.start = (uint32_t)k;
				runs.push_back(r);
			}
			runs.back().count++;
			sorted.push_back(e);
		}
		simple.swap(sorted);
		if (simple.size() > 65535)
			is_simple = false;
	}

	dtable_hdr_t h;

	memset(&h, 0, sizeof(h));
	h.slot_mask = slot_mask;
	if (is_simple)
		h.flags |= TBL_SIMPLE;
	if (is_simple && dup_distinct && dup_entries >= 3 * dup_distinct)
		h.flags |= TBL_HASHWALK;
	if (generic)
		h.flags |= TBL_GENERIC;
	h.num_runs = is_simple ? (uint32_t)runs.size() : 0;
	h.num_hgroups = is_simple ? (uint32_t)hgroups.size() : 0;
	h.num_hent = is_simple ? (uint32_t)hents.size() : 0;
	const bool keep_w = is_simple || !xcos.empty();

	h.num_wgroups = keep_w ? (uint32_t)wgroups.size() : 0;
	h.num_went = keep_w ? (uint32_t)wents.size() : 0;
	if (!xcos.empty()) {
		h.flags |= TBL_XWALK;
		h.num_xlist = num_xent;
		h.num_xwords = (uint32_t)xlist.size();
		/* the descriptor-layout lean kernel (classify_gf.hip) evaluates
		 * every complex rule from its xterm records */
		bool gf = ncos < 65536;

		for (uint32_t k = 0; gf && k < num_xent; k++)
			gf = (xlist[2 * k + 1] >> 24) != 0u;
		if (gf)
			h.flags |= TBL_XGF;
	}

	/* TBL_XMASK (classify_gf.hip's hit-map form). A packet's hit map holds
	 * one bit per "rule bit": the rule bits of a CoS are contiguous and in
	 * rule order, so a level of match_pmr_cos is the lowest set bit of the
	 * CoS's bit range. A single-word PMR (or an IPv4 / IPv6 alternative pair
	 * of them) has one bit, set when any of its groups' entries for the
	 * packet's key holds it (OR). A complex PMR has one bit per AND-chain of
	 * its terms (the chains of one PMR consecutive, so the lowest set one is
	 * the PMR's first match); a chain's bit starts set and is cleared by
	 * every group holding one of its records whose entry for the packet's
	 * key does not hold it (AND): hm = (hm & (h | ~A)) | (h & ~CH), A the
	 * group's chain members, CH every chain bit. Groups are keyed by (slot
	 * and guard, gate, mask); each has a collision-free multiplicative hash
	 * of its distinct masked values (slot = (value * mul) >> shift) into a
	 * table of 2^lg direct entries {value, bit map} (empty slots: map 0). Only the
	 * lowest PMR per (CoS, value) of a single-word group is entered: a
	 * higher one of the same key matches exactly when that one does.
	 * When the chain bits do not fit XM_MAX_PMR, the bits are the PMR
	 * indices and the complex PMRs are evaluated per level from their
	 * records (xflat, in rule order per CoS) instead. */
	bool xm = (h.flags & TBL_XGF) != 0;
	std::vector<uint32_t> bit_of(pmr.size(), 0u), chain_bit(num_xent, 0u);
	std::vector<uint32_t> cbit_start(ncos, 0u), cbit_n(ncos, 0u);
	uint32_t nbits = 0;
	bool and_form = xm;

	for (uint32_t c = 0; xm && c < ncos; c++) {
		const uint32_t st = xcos[2 * c] & 0xffffu, n = xcos[2 * c] >> 16;
		uint32_t k2 = st;

		cbit_start[c] = nbits;
		for (uint32_t k = 0; k < cos[c].nrule; k++) {
			const uint32_t pi = cos[c].rule_start + k;

			bit_of[pi] = nbits;
			if (!complex_pmr[pi]) {
				nbits++;
				continue;
			}
			while (k2 < st + n && xlist[2 * k2] == pi)
				chain_bit[k2++] = nbits++;
		}
		cbit_n[c] = nbits - cbit_start[c];
	}
	/* ODPG_XM_LAZY=1 forces the lazy form (experiment builds only,
	 * ODPG_DEBUG_KNOBS: A/B runs) */
	static const bool force_lazy = odpg_debug_env("ODPG_XM_LAZY") && atoi(odpg_debug_env("ODPG_XM_LAZY"));

	if (xm && (nbits > XM_MAX_PMR || force_lazy)) {
		/* lazy form: bit = PMR index, complex PMRs from their records */
		and_form = false;
		nbits = (uint32_t)pmr.size();
		for (uint32_t c = 0; c < ncos; c++) {
			cbit_start[c] = cos[c].rule_start;
			cbit_n[c] = cos[c].nrule;
		}
		for (size_t pi = 0; pi < pmr.size(); pi++)
			bit_of[pi] = (uint32_t)pi;
	}
	if (nbits > XM_MAX_PMR)
		xm = false;
	typedef std::tuple<uint32_t, uint32_t, uint32_t> gkey_t;   /* slot | guard, gate, mask */
	typedef std::vector<uint32_t> bm_t;                          /* XM_WORDS */
	std::map<gkey_t, std::map<uint32_t, bm_t>> gv;
	std::map<gkey_t, bm_t> gand;
	bm_t chain_all(XM_WORDS, 0u);
	auto setb = [](bm_t &m, uint32_t b) {
		m.resize(XM_WORDS, 0u);
		m[b >> 5] |= 1u << (b & 31u);
	};

	for (size_t gi = 0; xm && gi < wgroups.size(); gi++) {
		const dhgroup_t &g = wgroups[gi];
		auto &vm = gv[std::make_tuple(g.slot, g.req, g.mask)];

		for (uint32_t e = 0; e < (1u << g.log2sz); e++) {
			const dwent_t &w = wents[g.off + e];

			if (w.cos_pmr != HENT_EMPTY)
				setb(vm[w.value], bit_of[w.cos_pmr >> 16]);
		}
	}
	for (uint32_t k = 0; xm && and_form && k < num_xent; k++) {
		const uint32_t nt = xlist[2 * k + 1] >> 24, ts = xlist[2 * k + 1] & 0xffffffu;
		std::map<gkey_t, uint32_t> recs;
		bool dead = false;

		for (uint32_t tt = 0; tt < nt; tt++) {
			const uint32_t *r = &xterm[4 * (ts + tt)];
			const gkey_t key = std::make_tuple(r[3], r[0], r[1]);
			auto it = recs.find(key);

			/* bits outside the mask, or two values for one masked word:
			 * the chain never matches */
			if ((r[2] & ~r[1]) || (it != recs.end() && it->second != r[2]))
				dead = true;
			recs[key] = r[2];
		}
		if (dead)
			continue;
		for (auto &kv : recs) {
			setb(gv[kv.first][kv.second], chain_bit[k]);
			setb(gand[kv.first], chain_bit[k]);
		}
		setb(chain_all, chain_bit[k]);
	}
	if (gv.empty() || gv.size() > XM_MAX_GROUPS)
		xm = false;
	const uint32_t nw = nbits <= 64u ? 2u : nbits <= 128u ? 4u : 8u;
	std::vector<uint32_t> xmg, xmmask, xmval;
	uint64_t rs = 0x9E3779B97F4A7C15ull;

	/* the groups without chain records first (their entries only OR bits
	 * in), then the AND-chain groups, each kind's groups without a length
	 * guard first: the kernel runs each of the four in a loop of its own
	 * (the hit map's result does not depend on group order) */
	std::vector<decltype(gv.begin())> gorder;
	uint32_t gcut[3] = {0, 0, 0};
	auto guarded_key = [](const gkey_t &k) { return (std::get<0>(k) >> 31) != 0; };

	for (int kind = 0; kind < 4; kind++) {
		for (auto git = gv.begin(); git != gv.end(); ++git)
			if ((gand.count(git->first) != 0) == (kind >= 2) &&
			    guarded_key(git->first) == ((kind & 1) != 0))
				gorder.push_back(git);
		if (kind < 3)
			gcut[kind] = (uint32_t)gorder.size();
	}
	/* the kernel's 16-word key vector: slot s < 16 at word s; slots 16..18
	 * (L4 + 0, L4 + 4, frame length) in three words no group's slot < 16
	 * uses (the kernel writes all three unconditionally: a conditional
	 * indexed write compiled to a copy and a select of the whole vector),
	 * when at least three are free (else xm_kx: the kernel selects them per
	 * probe) */
	uint32_t kused = 0, kpos[3] = {0xffu, 0xffu, 0xffu};
	bool kx = false;

	for (auto &kv : gv)
		kused |= 1u << (std::get<0>(kv.first) & 0x1fu);
	{
		uint32_t freew = ~kused & 0xffffu;

		if (__builtin_popcount(freew) < 3) {
			kx = true;
		} else {
			for (uint32_t s = 16; s < 19; s++) {
				kpos[s - 16] = (uint32_t)__builtin_ctz(freew);
				freew &= freew - 1u;
			}
		}
	}
	for (size_t go = 0; xm && go < gorder.size(); ++go) {
		const auto git = gorder[go];
		const auto &vm = git->second;

		if (vm.size() > 255) {
			xm = false;
			break;
		}
		uint32_t lg = 1, mul = 0;
		bool found = false;

		while ((1u << lg) < 2 * vm.size())
			lg++;
		for (; lg <= XM_MAX_LG && !found; lg += found ? 0 : 1) {
			std::vector<uint8_t> used(1u << lg);

			for (int t = 0; t < 4096 && !found; t++) {
				rs ^= rs << 13;
				rs ^= rs >> 7;
				rs ^= rs << 17;
				mul = (uint32_t)(rs >> 16) | 1u;
				std::fill(used.begin(), used.end(), 0);
				found = true;
				for (auto &v : vm) {
					uint8_t &u = used[(v.first * mul) >> (32u - lg)];

					if (u) {
						found = false;
						break;
					}
					u = 1;
				}
			}
			if (found)
				break;
		}
		if (!found) {
			xm = false;
			break;
		}
		/* direct entries: slot (value * mul) >> shift of the group's
		 * 2^lg holds that value and its bit map; an empty slot's map is
		 * zero (a probe landing there changes nothing, as a miss) */
		const uint32_t ebase = (uint32_t)xmval.size();

		if (ebase + (1u << lg) > XM_MAX_ENTS) {
			xm = false;
			break;
		}
		xmval.resize(ebase + (1u << lg), 0u);
		xmmask.resize((size_t)(ebase + (1u << lg)) * nw, 0u);
		for (auto &v : vm) {
			const uint32_t e = ebase + ((v.first * mul) >> (32u - lg));
			bm_t m = v.second;

			m.resize(XM_WORDS, 0u);
			xmval[e] = v.first;
			std::copy(m.begin(), m.begin() + nw, xmmask.begin() + (size_t)e * nw);
		}
		auto ait = gand.find(git->first);
		bm_t a = ait == gand.end() ? bm_t(XM_WORDS, 0u) : ait->second;
		/* the group's key slot and its CUSTOM_L3 / CUSTOM_FRAME length
		 * guard (term_cmp: frame_len > base + off + size) as
		 * len >= (l3 & l3mask) + gthr */
		const uint32_t sg = std::get<0>(git->first);
		const uint32_t slot = sg & 0xffu;
		const uint32_t kidx = kx || slot < 16u ? slot : kpos[slot - 16u];
		const bool guarded = (sg >> 31) != 0;
		const uint32_t l3mask = guarded && !((sg >> 30) & 1u) ? ~0u : 0u;
		const uint32_t gthr = guarded ? ((sg >> 8) & 0xffffu) + 1u : 0u;

		a.resize(XM_WORDS, 0u);
		xmg.insert(xmg.end(), {mul, 32u - lg, kidx | (slot << 8), ebase, gthr,
				       std::get<1>(git->first), std::get<2>(git->first), l3mask});
		for (uint32_t w = 0; w < XM_WORDS; w++)
			xmg.push_back(~a[w]);
	}
	/* lazy form: the complex PMRs' terms flat, per CoS in rule order:
	 * {gate, mask, value, slot | guard end << 8 | absolute << 30 | guarded <<
	 * 31}, {pmr, last record of its chain, flat index of that record, 0}; per
	 * CoS its first flat record | count << 16 */
	std::vector<uint32_t> xflat, xfc(ncos, 0u), xfstart(num_xent + 1, 0u);

	for (uint32_t k = 0; xm && !and_form && k < num_xent; k++) {
		const uint32_t nt = xlist[2 * k + 1] >> 24, ts = xlist[2 * k + 1] & 0xffffffu;

		xfstart[k] = (uint32_t)(xflat.size() / 8);
		for (uint32_t tt = 0; tt < nt; tt++) {
			xflat.insert(xflat.end(), xterm.begin() + 4 * (ts + tt), xterm.begin() + 4 * (ts + tt + 1));
			xflat.insert(xflat.end(), {xlist[2 * k], tt + 1 == nt ? 1u : 0u,
						   xfstart[k] + nt - 1u, 0u});
		}
	}
	xfstart[num_xent] = (uint32_t)(xflat.size() / 8);
	for (uint32_t c = 0; xm && !and_form && c < ncos; c++) {
		const uint32_t st = xcos[2 * c] & 0xffffu, n = xcos[2 * c] >> 16;

		xfc[c] = xfstart[st] | ((xfstart[st + n] - xfstart[st]) << 16);
	}
	if (xflat.size() / 8 > XM_MAX_XTERMS)
		xm = false;
	std::vector<uint32_t> xmlds, xmhdr;

	if (xm) {
		xm_layout_t L;

		xm_layout_of(nw, (uint32_t)xmval.size(), 0u, ncos, nbits,
			     (uint32_t)(xflat.size() / 8), &L);
		xmlds.assign(L.lds_words, 0u);
		for (size_t e = 0; e < xmval.size(); e++) {
			for (uint32_t w = 0; w < nw; w++)
				xmlds[L.masks + e * L.estride + w] = xmmask[e * nw + w];
			xmlds[L.values + e * L.vstride] = xmval[e];
		}
		for (uint32_t c = 0; c < ncos; c++) {
			xmlds[L.xci + 2 * c] = cbit_start[c] | (cbit_n[c] << 16);
			xmlds[L.xci + 2 * c + 1] = cos[c].action | ((uint32_t)cos[c].num_queue << 8) |
						   ((uint32_t)cos[c].stats << 16) |
						   ((uint32_t)cos[c].hash_proto << 24);
		}
		/* per rule bit: its PMR's destination and mark, the destination's
		 * bit range and (lazy form) complex records */
		for (size_t pi = 0; pi < pmr.size(); pi++) {
			const uint32_t d = pmr[pi].dst;
			const uint32_t c = src_cos[pi];
			const uint32_t b0 = bit_of[pi];
			uint32_t b1 = b0 + 1u;

			/* the PMR's bits: up to the next PMR's first bit (or its
			 * CoS's end) */
			if (pi + 1 < pmr.size() && src_cos[pi + 1] == c)
				b1 = bit_of[pi + 1];
			else
				b1 = cbit_start[c] + cbit_n[c];
			for (uint32_t b = b0; b < b1; b++) {
				xmlds[L.xpd + 4 * b] = (d & 0xffffu) | ((pmr[pi].mark & 0xffffu) << 16);
				xmlds[L.xpd + 4 * b + 1] = cbit_start[d] | (cbit_n[d] << 16);
				xmlds[L.xpd + 4 * b + 2] = xfc[d];
			}
		}
		std::copy(xflat.begin(), xflat.end(), xmlds.begin() + L.xflat);
		xmhdr.assign(XM_HDR_WORDS, 0u);
		xmhdr[0] = nw;
		xmhdr[1] = nbits;
		xmhdr[2] = (uint32_t)gv.size();
		xmhdr[3] = (uint32_t)xmval.size();
		xmhdr[4] = kpos[0] | (kpos[1] << 8) | (kpos[2] << 16) | ((kx ? 1u : 0u) << 24);
		xmhdr[5] = (uint32_t)(xflat.size() / 8);
		/* the key slots the groups read (the kernel extracts them once per
		 * packet) */
		for (auto &kv : gv)
			xmhdr[6] |= 1u << (std::get<0>(kv.first) & 0x1fu);
		xmhdr[7] = gcut[0] | (gcut[1] << 8) | (gcut[2] << 16);
		for (uint32_t w = 0; w < XM_WORDS; w++)
			xmhdr[8 + w] = chain_all[w];
		h.flags |= TBL_XMASK;
		h.num_xment = (uint32_t)xmval.size();
		h.xm_slot_bytes = 0u;
		h.num_xflat = (uint32_t)(xflat.size() / 8);
		h.xm_nw = nw;
		h.xm_nbits = nbits;
		h.xm_ngroups = (uint32_t)gv.size();
		h.xm_kx = kx ? 1u : 0u;
	}
	const uint32_t lean_req = (1u << IFL_L2) | (1u << IFL_L3) | (1u << IFL_L4) |
				  (1u << IFL_ETH) | (1u << IFL_VLAN) | (1u << IFL_IPV4) |
				  (1u << IFL_IPV6) | (1u << IFL_UDP) | (1u << IFL_TCP) |
				  (1u << IFL_IPSEC_AH) | (1u << IFL_IPSEC_ESP);

	if ((h.flags & TBL_HASHWALK) && !cgroups.empty() && cgroups.size() == wgroups.size() &&
	    pmr.size() < 65536 && ncos < 4096) {
		bool lean = true;

		for (const dhgroup_t &g : wgroups)
			if (g.req & ~lean_req)
				lean = false;
		if (lean) {
			h.flags |= TBL_LEAN64HW;
			h.num_cgroups = (uint32_t)cgroups.size();
			h.num_cent = (uint32_t)cents.size();
		}
	}
	if (is_simple && pmr.size() <= MGROUP_MAX_PMR) {
		bool lean = true;

		for (const dmgroup_t &g : mgroups)
			if (g.req & ~lean_req)
				lean = false;
		bool cuckoo = true;

		for (const dmgroup_t &g : mgroups)
			if (g.count <= 1u || g.slot == SLOT_LEN)
				cuckoo = false;
		h.flags |= TBL_MGROUPS | (lean ? TBL_LEAN64 : 0u) | (cuckoo ? TBL_MG_CUCKOO : 0u);
		h.num_mgroups = (uint32_t)mgroups.size();
		h.num_ment = (uint32_t)ments.size();
	}
	h.num_cos = ncos;
	h.default_cos = r->default_cos;
	h.error_cos = r->error_cos;
	h.num_pmr = (uint32_t)pmr.size();
	h.num_terms = (uint32_t)terms.size();
	for (const dpmr_t &p : pmr)
		if (p.mark)
			h.flags |= TBL_ANY_MARK;
	for (const dcos_t &c : cos) {
		if (c.num_queue > 1)
			h.flags |= TBL_ANY_HASHQ;
		if (c.stats)
			h.flags |= TBL_ANY_STATS;
	}

	std::vector<uint32_t> cinfo(2 * cos.size()), pinfo(pmr.size());

	for (size_t c = 0; c < cos.size(); c++) {
		cinfo[2 * c] = (cos[c].rule_start & 0xffffu) | ((uint32_t)cos[c].nrule << 16);
		cinfo[2 * c + 1] = cos[c].action | ((uint32_t)cos[c].num_queue << 8) |
				   ((uint32_t)cos[c].stats << 16) | ((uint32_t)cos[c].hash_proto << 24);
	}
	for (size_t k = 0; k < pmr.size(); k++)
		pinfo[k] = (pmr[k].dst & 0xffffu) | ((pmr[k].mark & 0xffffu) << 16);
	std::vector<uint32_t> pinfo2;

	if (pmr.size() <= MGROUP_MAX_PMR) {
		/* rule_start < 64 and nrule <= 64 fit 8 bits each */
		pinfo2.resize(2 * pmr.size());
		for (size_t k = 0; k < pmr.size(); k++) {
			const dcos_t &d = cos[pmr[k].dst];

			pinfo2[2 * k] = pinfo[k];
			pinfo2[2 * k + 1] = (d.rule_start & 0xffu) | ((uint32_t)(d.nrule & 0xffu) << 8) |
					    ((uint32_t)d.action << 16);
		}
	}

	std::vector<uint32_t> pinfo4;

	if (pmr.size() <= MGROUP_MAX_PMR) {
		pinfo4.resize(4 * pmr.size());
		for (size_t k = 0; k < pmr.size(); k++) {
			const dcos_t &d = cos[pmr[k].dst];
			const uint64_t m = d.nrule ? ((d.nrule >= 64 ? ~0ull : ((1ull << d.nrule) - 1ull))
						      << d.rule_start) : 0ull;

			pinfo4[4 * k] = pinfo[k];
			pinfo4[4 * k + 1] = d.action;
			pinfo4[4 * k + 2] = (uint32_t)m;
			pinfo4[4 * k + 3] = (uint32_t)(m >> 32);
		}
	}
	std::vector<uint32_t> pinfo3;

	if (h.num_cgroups) {
		/* per PMR {dst | mark << 16, dst action | has rules << 8 | the dst's
		 * cuckoo-group mask << 12}; cgmask[c]: groups holding a rule of c */
		std::vector<uint32_t> cgmask(ncos, 0u);

		for (size_t g = 0; g < cgroups.size(); g++)
			for (uint32_t e = 0; e < (1u << (32u - cgroups[g].shift)); e++) {
				const dwent_t &w = cents[cgroups[g].off + e];

				if (w.cos_pmr != HENT_EMPTY)
					cgmask[w.cos_pmr & 0xffffu] |= 1u << g;
			}
		pinfo3.resize(2 * pmr.size());
		for (size_t k = 0; k < pmr.size(); k++) {
			const uint32_t d = pmr[k].dst;

			pinfo3[2 * k] = pinfo[k];
			pinfo3[2 * k + 1] = cos[d].action | ((cos[d].nrule ? 1u : 0u) << 8) |
					    (cgmask[d] << 12);
		}
		h.def_cgmask = r->default_cos >= 0 && (uint32_t)r->default_cos < ncos ?
			       cgmask[r->default_cos] : 0u;
	}

	auto align = [](uint32_t x) { return (x + 63u) & ~63u; };
	h.term_off = 0;
	h.slot_off = align(h.term_off + (uint32_t)(terms.size() * sizeof(dterm_t)));
	h.simple_off = align(h.slot_off + (uint32_t)(slots.size() * sizeof(dslot_t)));
	h.run_off = align(h.simple_off + (uint32_t)(is_simple ? simple.size() * sizeof(dsimple_t) : 0));
	h.hgroup_off = align(h.run_off + (uint32_t)(is_simple ? runs.size() * sizeof(drun_t) : 0));
	h.hent_off = align(h.hgroup_off + h.num_hgroups * (uint32_t)sizeof(dhgroup_t));
	h.pmr_off = align(h.hent_off + h.num_hent * (uint32_t)sizeof(dhent_t));
	h.cos_off = align(h.pmr_off + (uint32_t)(pmr.size() * sizeof(dpmr_t)));
	h.cinfo_off = align(h.cos_off + (uint32_t)(cos.size() * sizeof(dcos_t)));
	h.pinfo_off = align(h.cinfo_off + (uint32_t)(cinfo.size() * 4u));
	h.wgroup_off = align(h.pinfo_off + (uint32_t)(pinfo.size() * 4u));
	h.went_off = align(h.wgroup_off + h.num_wgroups * (uint32_t)sizeof(dhgroup_t));
	h.mgroup_off = align(h.went_off + h.num_went * (uint32_t)sizeof(dwent_t));
	h.ment_off = align(h.mgroup_off + h.num_mgroups * (uint32_t)sizeof(dmgroup_t));
	h.pinfo2_off = align(h.ment_off + h.num_ment * (uint32_t)sizeof(dment_t));
	h.cgroup_off = align(h.pinfo2_off + (uint32_t)(pinfo2.size() * 4u));
	h.cent_off = align(h.cgroup_off + h.num_cgroups * (uint32_t)sizeof(dmgroup_t));
	h.pinfo3_off = align(h.cent_off + h.num_cent * (uint32_t)sizeof(dwent_t));
	h.pinfo4_off = align(h.pinfo3_off + (uint32_t)(pinfo3.size() * 4u));
	h.xcos_off = align(h.pinfo4_off + (uint32_t)(pinfo4.size() * 4u));
	h.xlist_off = align(h.xcos_off + (uint32_t)(xcos.size() * 4u));
	h.xm_off = align(h.xlist_off + (uint32_t)(xlist.size() * 4u));
	/* TBL_XMASK region: header (XM_HDR_WORDS), group descriptors
	 * (XM_GROUP_WORDS each), the LDS part (xm_layout_t), xfc[num_cos] */
	const uint32_t xm_bytes = (h.flags & TBL_XMASK) ?
		(uint32_t)((xmhdr.size() + xmg.size() + xmlds.size() + xfc.size()) * 4u) : 0u;
	h.blob_bytes = align(h.xm_off + xm_bytes);
	if (h.blob_bytes == 0)
		h.blob_bytes = 64;
	blob.assign(h.blob_bytes, 0);
	if (!terms.empty())
		memcpy(blob.data() + h.term_off, terms.data(), terms.size() * sizeof(dterm_t));
	if (!slots.empty())
		memcpy(blob.data() + h.slot_off, slots.data(), slots.size() * sizeof(dslot_t));
	if (is_simple) {
		if (!simple.empty())
			memcpy(blob.data() + h.simple_off, simple.data(),
			       simple.size() * sizeof(dsimple_t));
		if (!runs.empty())
			memcpy(blob.data() + h.run_off, runs.data(), runs.size() * sizeof(drun_t));
		if (!hgroups.empty())
			memcpy(blob.data() + h.hgroup_off, hgroups.data(), hgroups.size() * sizeof(dhgroup_t));
		if (!hents.empty())
			memcpy(blob.data() + h.hent_off, hents.data(), hents.size() * sizeof(dhent_t));
	}
	if (!pmr.empty())
		memcpy(blob.data() + h.pmr_off, pmr.data(), pmr.size() * sizeof(dpmr_t));
	if (!cos.empty())
		memcpy(blob.data() + h.cos_off, cos.data(), cos.size() * sizeof(dcos_t));
	if (!cinfo.empty())
		memcpy(blob.data() + h.cinfo_off, cinfo.data(), cinfo.size() * 4u);
	if (!pinfo.empty())
		memcpy(blob.data() + h.pinfo_off, pinfo.data(), pinfo.size() * 4u);
	if (h.num_wgroups)
		memcpy(blob.data() + h.wgroup_off, wgroups.data(), wgroups.size() * sizeof(dhgroup_t));
	if (h.num_went)
		memcpy(blob.data() + h.went_off, wents.data(), wents.size() * sizeof(dwent_t));
	if (h.num_mgroups)
		memcpy(blob.data() + h.mgroup_off, mgroups.data(), mgroups.size() * sizeof(dmgroup_t));
	if (h.num_ment)
		memcpy(blob.data() + h.ment_off, ments.data(), ments.size() * sizeof(dment_t));
	if (!pinfo2.empty())
		memcpy(blob.data() + h.pinfo2_off, pinfo2.data(), pinfo2.size() * 4u);
	if (!pinfo4.empty())
		memcpy(blob.data() + h.pinfo4_off, pinfo4.data(), pinfo4.size() * 4u);
	if (h.num_cgroups) {
		memcpy(blob.data() + h.cgroup_off, cgroups.data(), cgroups.size() * sizeof(dmgroup_t));
		memcpy(blob.data() + h.cent_off, cents.data(), cents.size() * sizeof(dwent_t));
		memcpy(blob.data() + h.pinfo3_off, pinfo3.data(), pinfo3.size() * 4u);
	}
	if (!xcos.empty())
		memcpy(blob.data() + h.xcos_off, xcos.data(), xcos.size() * 4u);
	if (!xlist.empty())
		memcpy(blob.data() + h.xlist_off, xlist.data(), xlist.size() * 4u);
	if (h.flags & TBL_XMASK) {
		uint8_t *o = blob.data() + h.xm_off;

		for (const std::vector<uint32_t> *v : {&xmhdr, &xmg, &xmlds, &xfc}) {
			if (!v->empty())
				memcpy(o, v->data(), v->size() * 4u);
			o += v->size() * 4u;
		}
	}
	*hdr_out = h;
	return 0;
}

/* Does any packet path revisit a CoS? (reference loops forever on a matching
 * cycle, odp_classification.c:1603-1631) */
int odpg_rules_has_cycle(const std::vector<uint8_t> &blob, const dtable_hdr_t &h)
{
	const dcos_t *cos = (const dcos_t *)(blob.data() + h.cos_off);
	const dpmr_t *pmr = (const dpmr_t *)(blob.data() + h.pmr_off);
	std::vector<int> state(h.num_cos, 0);
	std::vector<std::pair<uint32_t, uint32_t>> stack;

	for (uint32_t s = 0; s < h.num_cos; s++) {
		if (state[s])
			continue;
		stack.push_back({s, 0});
		state[s] = 1;
		while (!stack.empty()) {
			auto &top = stack.back();
			uint32_t c = top.first;

			if (top.second < cos[c].nrule) {
				uint32_t d = pmr[cos[c].rule_start + top.second].dst;

				top.second++;
				if (state[d] == 1)
					return 1;
				if (state[d] == 0) {
					state[d] = 1;
					stack.push_back({d, 0});
				}
			} else {
				state[c] = 2;
				stack.pop_back();
			}
		}
	}
	return 0;
}
