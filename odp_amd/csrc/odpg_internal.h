/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Internal layout shared by the host table compiler (cls_compile.cpp) and
 * the gfx950 kernels (classify.hip). Not part of the public ABI.
 */
#ifndef ODPG_INTERNAL_H_
#define ODPG_INTERNAL_H_

#include <stdint.h>
#include <stdlib.h>

/* Strategy switches for A/B experiment builds (ODPG_NO_LEAN64, ODPG_NO_GF,
 * ODPG_GRID_CAP, ODPG_XM_LAZY): read from the environment only in a build
 * made with -DODPG_DEBUG_KNOBS (make EXTRA=-DODPG_DEBUG_KNOBS); the shipped
 * library ignores them */
static inline const char *odpg_debug_env(const char *name)
{
#ifdef ODPG_DEBUG_KNOBS
	return getenv(name);
#else
	(void)name;
	return (const char *)0;
#endif
}

/* _odp_packet_input_flags_t bit positions (packet_inline_types.h:60-113) */
enum {
	IFL_DST_QUEUE = 0, IFL_CLS_MARK, IFL_FLOW_HASH, IFL_TIMESTAMP,
	IFL_L2, IFL_L3, IFL_L4,
	IFL_ETH, IFL_ETH_BCAST, IFL_ETH_MCAST, IFL_JUMBO, IFL_VLAN, IFL_VLAN_QINQ,
	IFL_SNAP, IFL_ARP,
	IFL_IPV4, IFL_IPV6, IFL_IP_BCAST, IFL_IP_MCAST, IFL_IPFRAG, IFL_IPOPT,
	IFL_IPSEC, IFL_IPSEC_AH, IFL_IPSEC_ESP,
	IFL_UDP, IFL_TCP, IFL_SCTP, IFL_ICMP, IFL_NO_NEXT_HDR,
	IFL_COLOR0, IFL_COLOR1, IFL_NODROP,
	IFL_L3_CHKSUM_DONE, IFL_L4_CHKSUM_DONE, IFL_IPSEC_UDP, IFL_UDP_CHKSUM_ZERO
};

/* _odp_packet_flags_t error bits (packet_inline_types.h:150-164) */
enum {
	FL_SNAP_LEN_ERR = 25, FL_IP_ERR, FL_L3_CHKSUM_ERR, FL_TCP_ERR, FL_UDP_ERR,
	FL_SCTP_ERR, FL_L4_CHKSUM_ERR
};
#define FL_ERROR_MASK 0xFE000000u

/* odp_cls_pmr_term_t (include/odp/api/spec/classification.h:68-195) */
enum {
	PMR_LEN = 0, PMR_ETHTYPE_0, PMR_ETHTYPE_X, PMR_VLAN_ID_0, PMR_VLAN_ID_X,
	PMR_VLAN_PCP_0, PMR_DMAC, PMR_IPPROTO, PMR_IP_DSCP, PMR_UDP_DPORT,
	PMR_TCP_DPORT, PMR_UDP_SPORT, PMR_TCP_SPORT, PMR_SIP_ADDR, PMR_DIP_ADDR,
	PMR_SIP6_ADDR, PMR_DIP6_ADDR, PMR_IPSEC_SPI, PMR_LD_VNI, PMR_CUSTOM_FRAME,
	PMR_CUSTOM_L3, PMR_IGMP_GRP_ADDR, PMR_ICMP_ID, PMR_ICMP_TYPE, PMR_ICMP_CODE,
	PMR_SCTP_SPORT, PMR_SCTP_DPORT, PMR_GTPV1_TEID, PMR_INNER_HDR_OFF = 32
};

/* ---- compiled device table ---------------------------------------------
 * Every reference term matcher (odp_classification.c:906-1332) reduces to a
 * byte-wise masked compare of up to 16 bytes at (base + off), gated by a set
 * of parser input flags that must all be present. Terms whose matcher
 * depends on the IP version / IPsec header kind (IPPROTO, IP_DSCP,
 * IPSEC_SPI) compile to two alternatives: the first applies when its flags
 * are present, otherwise the second is evaluated. */
enum { DK_CMP = 0, DK_LEN = 1, DK_NEVER = 2 };
enum { DB_ABS = 0, DB_L2 = 1, DB_L3 = 2, DB_L4 = 3, DB_VLANX = 4 };
#define DT_GUARD    0x1   /* require frame_len > pos + size (custom terms)    */
#define DT_ALT_NEXT 0x2   /* if req flags absent, result = next term's result */

typedef struct dterm_s {
	uint8_t  kind;
	uint8_t  base;
	uint8_t  nwords;    /* 0..4 compared 32-bit little-endian words */
	uint8_t  tflags;
	uint32_t req;       /* low 32 input flags that must all be set */
	int32_t  off;
	uint32_t size;      /* bytes compared (guard length) */
	uint32_t mask[4];
	uint32_t value[4];
} dterm_t;              /* 48 bytes */

/* 32-bit fields throughout: wave-uniform reads of these tables become
 * scalar (s_load) loads only when every field is dword aligned */
typedef struct dpmr_s {
	uint32_t term_start;
	uint32_t nterms;    /* compiled entries, including ALT_NEXT partners */
	uint32_t mark;
	uint32_t dst;
} dpmr_t;               /* 16 bytes */

typedef struct dcos_s {
	uint32_t rule_start;
	uint16_t nrule;
	uint8_t  action;
	uint8_t  num_queue;
	uint8_t  hash_proto;
	uint8_t  stats;
	uint8_t  valid;
	uint8_t  pad;
} dcos_t;               /* 12 bytes */

#define TBL_ANY_MARK   0x1
#define TBL_ANY_HASHQ  0x2
#define TBL_ANY_STATS  0x4
#define TBL_SIMPLE     0x8   /* every PMR is one single-word slotted compare */
#define TBL_GENERIC    0x10  /* some term needs the generic (base + off) compare */
#define TBL_HASHWALK   0x20  /* exact-match groups repeat values across CoS (mean
			      * >= 3 entries per distinct value): per-level
			      * CoS-keyed probes beat evaluating every entry */
#define TBL_MGROUPS    0x40  /* mask groups + pinfo2 built (simple, <= 64 PMRs) */
#define TBL_LEAN64     0x80  /* TBL_MGROUPS and every group gates only on flags
			      * the lean kernel's register parse computes
			      * (L2, L3, L4, ETH, VLAN, IPV4, IPV6, UDP, TCP,
			      * IPSEC_AH, IPSEC_ESP) */
#define TBL_MG_CUCKOO  0x400 /* every mask group is a cuckoo group (> 1 value)
			      * over a frame word (no frame-length slot) */
#define TBL_XWALK      0x200 /* hybrid hash walk: walk groups over the single-word
                              * PMRs, xcos / xlist name the complex ones per CoS */
#define TBL_XGF        0x800 /* TBL_XWALK with every complex PMR in xterm
			      * records (the form classify_gf.hip evaluates) */
#define TBL_XMASK      0x1000 /* TBL_XGF with <= XM_MAX_PMR PMRs and a collision-free
			       * value hash per walk group: the hit-map form
			       * (cls_compile.cpp "TBL_XMASK") */
#define XM_MAX_PMR     256
#define XM_WORDS       8     /* hit-map words per packet (XM_MAX_PMR / 32) */
#define XM_MAX_LG      9     /* largest per-group entry table: 512 entries */
#define XM_MAX_ENTS    4096  /* direct entries of all groups (LDS: (nw + 1) words each) */
#define XM_MAX_XTERMS  512   /* complex-PMR terms the kernel evaluates per packet */
#define XM_MAX_GROUPS  64    /* groups read per packet */
#define XM_GROUP_WORDS 16    /* xmg descriptor: {mul, shift, key index | slot << 8,
			      * entry base}, {guard threshold, gate, mask, L3
			      * mask of the length guard}, not-member words[8].
			      * The key index is the group's word in the kernel's
			      * 16-word key vector: the slot itself for slots < 16,
			      * slots 16..18 (L4 + 0, L4 + 4, frame length) folded
			      * into a word no group's slot uses (xhdr[4]); with
			      * xm_kx (more than 16 slots read) the slot itself */
#define XM_HDR_WORDS   16    /* region header: nw, nbits, ngroups, num_xment,
			      * the key-vector words of slots 16 / 17 / 18 (bytes
			      * 0..2, 0xff: not read; byte 3: xm_kx), num_xflat,
			      * key slots the groups read (bit mask), the group
			      * order (n0 | n1 << 8 | n2 << 16: groups [0, n0)
			      * without chain members or length guard, [n0, n1)
			      * without chain members, guarded, [n1, n2) with
			      * chain members, unguarded, [n2, ngroups) the rest),
			      * chain bits[8] */

/* TBL_XMASK region, after the header and the group descriptors: the part
 * every workgroup copies to LDS (word offsets, each part 16-byte aligned),
 * then xfc[num_cos]. Shared by cls_compile.cpp and classify_gf.hip. */
typedef struct xm_layout_s {
	uint32_t masks;     /* [num_xment + 1..4] entry bit maps (nw words at a
			     * stride of estride words): each group's 2^lg
			     * direct entries (slot = value * mul >> shift), an
			     * empty slot's map zero */
	uint32_t values;    /* [num_xment] masked key values (stride vstride).
			     * 2-word maps: entries interleaved {map0, map1,
			     * value, 0}, one ds_read_b128 per probe */
	uint32_t estride, vstride;
	uint32_t slots;     /* unused (slot_bytes 0) */
	uint32_t xci;       /* uint2 [num_cos]: {bit start | bits << 16, cinfo.y} */
	uint32_t xpd;       /* uint4 [nbits]: {dst | mark << 16, dst's xci.x, dst's
			     * xfc, 0} */
	uint32_t xflat;     /* 2 x uint4 [num_xflat]: per-level complex records */
	uint32_t lds_words; /* end of the LDS part */
} xm_layout_t;

static inline
#if defined(__HIPCC__)
__host__ __device__
#endif
void xm_layout_of(uint32_t nw, uint32_t num_xment, uint32_t slot_bytes, uint32_t num_cos,
		  uint32_t nbits, uint32_t num_xflat, xm_layout_t *L)
{
	/* at least one zero entry past the last (index num_xment: a probe's
	 * bit map on a miss) */
	const uint32_t nx = (num_xment + 4u) & ~3u;

	L->masks = 0u;
	if (nw == 2u) {
		L->estride = 4u;
		L->values = 2u;
		L->vstride = 4u;
		L->slots = 4u * nx;
	} else {
		L->estride = nw;
		L->values = L->masks + nx * nw;
		L->vstride = 1u;
		L->slots = L->values + nx;
	}
	L->xci = L->slots + ((slot_bytes + 15u) & ~15u) / 4u;
	L->xpd = L->xci + 2u * ((num_cos + 1u) & ~1u);
	L->xflat = L->xpd + 4u * nbits;
	L->lds_words = L->xflat + 8u * num_xflat;
}
#define TBL_LEAN64HW   0x100 /* TBL_HASHWALK with <= 4 walk groups whose gates
			      * the lean kernel's register parse computes: the
			      * lean kernel's walk-group form */

/* ---- per-packet key slots (evaluate-all kernels) -------------------------
 * The parser-relative 32-bit words the terms can compare, extracted once per
 * packet into registers:
 *   0..4   L2 + 0, 4, 8, 12, 16   (DMAC, ETHTYPE_0, VLAN_ID_0 / PCP)
 *   5      VLANX + 0              (innermost VLAN tci + ethertype)
 *   6..15  L3 + 0 .. 36           (IPv4 / IPv6 header fields and addresses)
 *   16..17 L4 + 0, 4              (ports, AH / ESP SPI)
 *   18     frame length           (ODP_PMR_LEN)
 * A term compares up to four consecutive slots, masks re-aligned to the slot
 * words by the compiler. Terms outside these windows (custom terms) keep the
 * generic (base + off) compare. */
#define KEY_SLOTS     19
#define SLOT_L2       0
#define SLOT_VLANX    5
#define SLOT_L3       6
#define SLOT_L4       16
#define SLOT_LEN      18
#define SLOT_NONE     0xFF

typedef struct dslot_s {
	uint8_t  slot;      /* first slot, SLOT_NONE = generic compare */
	uint8_t  nw;        /* consecutive slots compared */
	uint16_t pad;
	uint32_t mask[4];
	uint32_t value[4];
} dslot_t;              /* 36 bytes, parallel to dterm_t */

/* TBL_SIMPLE tables: one entry per PMR, sorted by (key slot, hit word), and
 * grouped in runs that share the slot word and the 32-bit hit-map word */
typedef struct dsimple_s {
	uint32_t req;
	uint32_t mask;
	uint32_t value;
	uint32_t idx;       /* PMR index in table order (hit-map bit) */
} dsimple_t;            /* 16 bytes */

typedef struct drun_s {
	uint32_t slot;
	uint32_t word;      /* hit-map word = idx >> 5 */
	uint32_t start;     /* first dsimple_t */
	uint32_t count;
} drun_t;               /* 16 bytes */

/* Exact-match groups: TBL_SIMPLE entries sharing (slot, req, mask) compile to
 * an open-addressing hash table of (value, pmr index); one probe sequence per
 * packet replaces `count` compares. Load factor <= 1/2, linear probing,
 * h = (key * 0x9E3779B1) >> (32 - log2sz). */
typedef struct dhgroup_s {
	uint32_t slot;
	uint32_t req;
	uint32_t mask;
	uint32_t log2sz;
	uint32_t off;       /* first dhent_t of this group */
	uint32_t count;     /* real entries */
	uint32_t maxp;      /* CoS-keyed walk groups: longest probe sequence of
			     * any entry (1 = every entry in its home slot) */
	uint32_t pad;
} dhgroup_t;            /* 32 bytes */

typedef struct dhent_s {
	uint32_t value;
	uint32_t idx;       /* PMR index, HENT_EMPTY = free slot */
} dhent_t;

/* CoS-keyed walk groups (TBL_SIMPLE tables): every single-word PMR is in the
 * group of its (slot, req, mask); the group's open-addressing table is keyed
 * by (source CoS, masked value) and holds the lowest PMR index for that key.
 * A packet at CoS c probes each group once per level of the match_pmr_cos
 * walk; the smallest PMR index found is the first match of c's rule list. */
typedef struct dwent_s {
	uint32_t value;
	uint32_t cos_pmr;   /* cos | pmr << 16, HENT_EMPTY = free slot */
} dwent_t;

#define WALK_MAX_GROUPS 8    /* more groups: evaluate-all is cheaper */
#define XWALK_MAX_GROUPS 32  /* hybrid walk: per-CoS group mask is one word */
#ifndef XWALK_KEYS
#define XWALK_KEYS 12        /* hybrid walk: group keys held in registers */
#endif
#ifndef XWALK_MAXP
#define XWALK_MAXP 4         /* hybrid walk: groups probed branch-free up to this */
#endif

/* Mask groups (TBL_SIMPLE tables of <= 64 PMRs, the u64 hit-map kernel):
 * every (slot, req, mask) group is a two-choice cuckoo table keyed by the
 * masked value; an entry holds the OR of the hit bits of every PMR of the
 * group that compares equal to that value. A packet reads both candidate
 * entries of each group (two independent LDS reads, no probe sequence) and
 * ORs the mask of the one whose value matches. Free entries have zero masks,
 * so a false value match on a free entry adds nothing. */
typedef struct dmgroup_s {
	uint32_t slot;
	uint32_t req;
	uint32_t mask;
	uint32_t shift;     /* 32 - log2(entries) */
	uint32_t off;       /* first dment_t of this group */
	uint32_t m1, m2;    /* odd multipliers: h = (key * m) >> shift */
	uint32_t count;     /* distinct values; 1: {value, lo, hi} inline in
			     * {m1, m2, off} and no entries */
} dmgroup_t;            /* 32 bytes */

typedef struct dment_s {
	uint32_t value;
	uint32_t lo, hi;    /* hit bits of the PMRs equal to value */
	uint32_t pad;
} dment_t;              /* 16 bytes */

#define MGROUP_MAX_PMR 64

/* pinfo2[num_pmr] (u64 hit-map kernel): the first-match resolve follows one
 * LDS read per level, {dst | mark << 16, dst rule_start | dst nrule << 8 |
 * dst action << 16}. pinfo4[num_pmr] (lean kernel): {dst | mark << 16, dst
 * action, dst rule mask lo, hi}, the mask holding the hit-map bits of the
 * destination's rules, so a level is one AND + find-first-set. */

#if defined(__HIPCC__)
#define ODPG_HD __host__ __device__
#else
#define ODPG_HD
#endif
/* CoS-keyed cuckoo groups (TBL_LEAN64HW): the walk groups' (cos, value)
 * -> lowest PMR maps as two-choice cuckoo tables in dmgroup_t form (shift,
 * m1, m2, off, count) over dwent_t entries; a key's candidates are
 * (cgroup_key(value, cos) * m) >> shift for m = m1, m2. pinfo3[k] =
 * {dst | mark << 16, dst action | dst has rules << 8 | dst group mask << 12}. */
static inline ODPG_HD uint32_t cgroup_key(uint32_t value, uint32_t cos)
{
	return value ^ (cos * 0x85EBCA6Bu);
}

/* slot of (value, cos) in a walk group of 2^lg entries (lg >= 1) */
static inline ODPG_HD uint32_t walk_hash(uint32_t value, uint32_t cos, uint32_t lg)
{
	return ((value ^ (cos * 0x85EBCA6Bu)) * 0x9E3779B1u) >> (32u - lg);
}

#define HENT_EMPTY    0xFFFFFFFFu
#define HASH_MIN      6      /* smaller groups stay linear */
#define HASH_MUL      0x9E3779B1u
#ifndef HENT_LDS_MAX
#define HENT_LDS_MAX  4096   /* entries copied to LDS per workgroup */
#endif

#define EVAL_ALL_MAX_PMR 1024

typedef struct dtable_hdr_s {
	uint32_t num_cos;
	int32_t  default_cos;
	int32_t  error_cos;
	uint32_t flags;
	uint32_t num_pmr;
	uint32_t num_terms;
	uint32_t cos_off;    /* byte offsets inside the device blob */
	uint32_t pmr_off;
	uint32_t term_off;
	uint32_t slot_off;   /* dslot_t[num_terms] */
	uint32_t simple_off; /* dsimple_t[num_pmr] when TBL_SIMPLE */
	uint32_t run_off;    /* drun_t[num_runs] when TBL_SIMPLE */
	uint32_t num_runs;
	uint32_t hgroup_off; /* dhgroup_t[num_hgroups] */
	uint32_t num_hgroups;
	uint32_t hent_off;   /* dhent_t[num_hent] */
	uint32_t num_hent;
	uint32_t cinfo_off;  /* uint2[num_cos]: {rule_start | nrule << 16,
	                      *  action | num_queue << 8 | stats << 16 | hash_proto << 24} */
	uint32_t pinfo_off;  /* uint32[num_pmr]: dst | mark << 16 */
	uint32_t slot_mask;  /* key slots any slotted term reads */
	uint32_t wgroup_off; /* dhgroup_t[num_wgroups], CoS-keyed (dwent_t tables) */
	uint32_t num_wgroups;
	uint32_t went_off;   /* dwent_t[num_went] */
	uint32_t num_went;
	uint32_t mgroup_off; /* dmgroup_t[num_mgroups] (num_pmr <= 64, TBL_SIMPLE) */
	uint32_t num_mgroups;
	uint32_t ment_off;   /* dment_t[num_ment] */
	uint32_t num_ment;
	uint32_t pinfo2_off; /* uint2[num_pmr] when num_pmr <= 64 */
	uint32_t cgroup_off; /* dmgroup_t[num_cgroups]: CoS-keyed cuckoo groups (TBL_LEAN64HW) */
	uint32_t num_cgroups;
	uint32_t cent_off;   /* dwent_t[num_cent] */
	uint32_t num_cent;
	uint32_t pinfo3_off; /* uint2[num_pmr] (TBL_LEAN64HW) */
	uint32_t pinfo4_off; /* uint4[num_pmr] when num_pmr <= 64 (lean kernel) */
	uint32_t def_cgmask; /* cuckoo groups holding a rule of the default CoS */
	uint32_t xcos_off;   /* uint2[num_cos] (TBL_XWALK): {xlist start | count << 16,
	                      *  walk groups holding a single-word rule of the CoS} */
	uint32_t xlist_off;  /* uint32[num_xwords]: uint2[num_xlist] {pmr, xterm start |
	                      *  n << 24} per CoS in rule order (padded to even), then
	                      *  uint4 xterm records (cls_compile.cpp) */
	uint32_t num_xlist;
	uint32_t num_xwords;
	uint32_t xm_off;     /* TBL_XMASK region (cls_compile.cpp) */
	uint32_t num_xment;
	uint32_t xm_slot_bytes;
	uint32_t num_xflat;
	uint32_t blob_bytes;
	uint32_t xm_nw;      /* TBL_XMASK hit-map words per packet (2, 4 or 8) */
	uint32_t xm_nbits;   /* rule bits (chains of the complex PMRs have their own) */
	uint32_t xm_ngroups; /* groups read per packet */
	uint32_t xm_kx;      /* TBL_XMASK: the groups read more than 16 key slots, so
			      * slots 16..18 are not folded into the 16-word key
			      * vector (classify_gf.hip KX) */
} dtable_hdr_t;

typedef struct uint2_s { uint32_t x, y; } uint2_t;

/* sharded counters of one launch (odpg.h "sharded counters"): row r of
 * `words` u64 belongs to workgroup r: [4 pktio][ncos CoS stats][ncols
 * delivered per queue column, qcol[c] + hash queue] */
typedef struct odpg_cnt_dev {
	uint64_t *rows;
	const uint32_t *qcol;   /* queue column of each CoS (num_cos + 1) */
	uint32_t words, ncos, ncols;
	uint32_t ident;         /* ncols == ncos: qcol[c] == c */
} odpg_cnt_dev;

typedef struct odpg_cnt_args {
	uint64_t *row;          /* rows base, NULL = no sharded counters */
	const uint32_t *qcol;   /* device, queue column of each CoS (num_cos + 1) */
	uint32_t words, rows, ncos, ncols;
	uint32_t cos;           /* the table has CoS with stats_enable */
	uint32_t pad;
} odpg_cnt_args;

/* the layout the lean kernels take by value as a kernel argument */
static inline odpg_cnt_dev odpg_cnt_layout(const odpg_cnt_args *c)
{
	odpg_cnt_dev d;

	d.rows = c->row;
	d.qcol = c->qcol;
	d.words = c->words;
	d.ncos = c->ncos;
	d.ncols = c->ncols;
	d.ident = c->ncols == c->ncos;
	return d;
}

/* odp_cls.c: drop the classifier's tables / counters bound to a context
 * (called by odpg_ctx_destroy before the context's stream goes away) */
#ifdef __cplusplus
extern "C"
#endif
void odpg_cls_ctx_release(struct odpg_ctx_s *ctx);
/* context references held by objects created on it (runtime.hip; odpg.h
 * "object lifetimes") */
#ifdef __cplusplus
extern "C" {
#endif
void odpg_ctx_ref(struct odpg_ctx_s *ctx);
void odpg_ctx_unref(struct odpg_ctx_s *ctx);
#ifdef __cplusplus
}
#endif

/* kernel launch arguments (runtime.hip -> classify.hip) */
#include "../../include/odpg.h"
typedef struct odpg_launch_args {
	const uint8_t *frames;
	const odpg_desc_t *desc;
	uint32_t stride, num;
	uint64_t opt;
	uint32_t layer, classify;
	const dterm_t *terms;
	const dpmr_t *pmrs;
	const dcos_t *coses;
	uint32_t num_cos;
	int32_t default_cos, error_cos;
	uint32_t tbl_flags;
	uint32_t num_pmr;
	uint32_t slot_mask;
	const dslot_t *slots;
	const dsimple_t *simple;
	const drun_t *runs;
	uint32_t num_runs;
	const dhgroup_t *hgroups;
	uint32_t num_hgroups;
	const dhent_t *hents;
	uint32_t num_hent;
	const uint2_t *cinfo;
	const uint32_t *pinfo;
	const dhgroup_t *wgroups;
	uint32_t num_wgroups;
	const dwent_t *wents;
	uint32_t num_went;
	const dmgroup_t *mgroups;
	uint32_t num_mgroups;
	const dment_t *ments;
	uint32_t num_ment;
	const uint2_t *pinfo2;
	const dmgroup_t *cgroups;   /* TBL_LEAN64HW cuckoo groups */
	uint32_t num_cgroups;
	const dwent_t *cents;
	uint32_t num_cent;
	const uint2_t *pinfo3;
	const uint32_t *pinfo4;     /* uint4 entries */
	uint32_t def_cgmask;
	const uint2_t *xcos;        /* TBL_XWALK */
	const uint32_t *xlist;
	uint32_t num_xlist, num_xwords;
	const uint32_t *xm;         /* TBL_XMASK region */
	uint32_t num_xment, xm_slot_bytes, num_xflat;
	uint32_t xm_nw, xm_nbits, xm_ngroups, xm_kx;
	/* lean 64-byte kernel (classify64.hip): CoS start state, from the host
	 * copy of the table */
	uint32_t l64_err_cos, l64_err_act, l64_def_cos, l64_def_act, l64_def_ci, l64_def_rules;
	uint32_t l64_def_mlo, l64_def_mhi;   /* the default CoS's rule mask (pinfo4 form) */
	uint32_t l64_depth;    /* longest rule chain from the default CoS, 0 = cyclic */
	int mode;          /* 0 auto, 1 walk, 2 evaluate-all, 3 hash walk */
	odpg_out_t *out;
	uint16_t *mark;
	odpg_meta_t *meta;
	uint64_t *pk_partial;
	uint32_t *cos_partial;
	uint32_t pk_atomic;    /* pk_partial is the caller's counters (stats_commit.h) */
	uint64_t *sred;        /* the context's stats_commit scratch (zeroed) */
	uint64_t *stats;
	odpg_cnt_args cnt;
} odpg_launch_args;

#endif
