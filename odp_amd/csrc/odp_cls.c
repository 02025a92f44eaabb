/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Host control plane: the ODP CoS / PMR object model (odp_cls_* API) and the
 * loop-pktio classifier glue, re-implemented for the MI355X classifier.
 *
 * Semantics follow platform/linux-generic/odp_classification.c exactly where
 * an application can observe them: handles are index + 1 (:60-78), slots are
 * taken first-free (:276-343, :419-437), a CoS holds at most
 * max_pmr_per_cos rules (:807-808), rule creation appends in cos->pmr[] order
 * (:826-829), rule destruction swaps the last rule into the freed slot
 * (:757-761), destroyed CoS keep their slot contents until reuse (:464-478).
 * The data plane never reads these structures: every change bumps a
 * generation and odpg_pktio_recv_batch() compiles an immutable snapshot
 * (odpg_rules_t -> device table) the first time a generation is used on a
 * context. The launches add their pktio / CoS / queue counts into the
 * binding's device-resident sharded counters (odpg.h); the statistics calls
 * fold them into the host totals when they are read, as the reference reads
 * its atomics at query time. The global lock covers the object model and the
 * binding lookup, never a receive's launch. It is held, though, while a
 * binding is recompiled for a new rule generation (odpg_table_update, which
 * orders its upload on the context stream and may wait for that stream when
 * the table grows) and while statistics are folded (odpg_counters_fold
 * waits for the launches before it): a rule change or a statistics read
 * can therefore wait for GPU work already queued.
 *
 * A CoS with num_queue > 1 owns its hash queues: they are created with the
 * CoS's queue_param as "_odp_cos_hq_<cos>_<i>" by odp_queue_create (the
 * runtime's queues, odp/rt.h) and destroyed with the CoS
 * (odp_classification.c:283-307, 464-478).
 */
#include <errno.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/odp_api.h"
#include "odp_rt_internal.h"

#define REF_MAX_COS          64      /* CLS_COS_MAX_ENTRY   */
#define REF_MAX_PMR          256     /* CLS_PMR_MAX_ENTRY   */
#define REF_MAX_PMR_PER_COS  8       /* CLS_PMR_PER_COS_MAX */
#define MAX_TERMS            8       /* CLS_PMRTERM_MAX     */
#define MAX_TERM_SIZE        16
#define COS_QUEUE_MAX        32
#define MAX_MARK             UINT16_MAX
#define MAX_PKTIO            64

#define ERR(...) fprintf(stderr, "odp_cls: " __VA_ARGS__)

typedef struct {
	int valid;
	char name[ODP_COS_NAME_LEN];
	uint32_t *pmr;          /* [max_pmr_per_cos] pmr index    */
	uint32_t *linked;       /* [max_pmr_per_cos] cos index    */
	uint32_t num_rule;
	int stats_enable;
	int action;
	odp_queue_t queue;
	uint32_t num_queue;
	odp_pool_t pool;
	uint32_t index;
	int queue_group;
	uint32_t hash_proto;    /* odp_cls_hash_proto_t bits */
	odp_pktin_vector_config_t vector;
	odp_queue_param_t queue_param;
	uint64_t st_packets, st_discards;
	uint64_t q_packets[COS_QUEUE_MAX], q_discards[COS_QUEUE_MAX];
	odp_queue_t hq[COS_QUEUE_MAX];   /* implementation-created hash queues */
	uint64_t uid;           /* creation serial: counts of an earlier CoS in
				 * the slot are not folded into this one */
} cos_e;

typedef struct {
	int valid;
	uint32_t num_pmr;
	uint16_t mark;
	odpg_term_t terms[MAX_TERMS];
	int src_cos;            /* -1 = none */
} pmr_e;

typedef struct {
	int valid;
	int started;
	int closing;                 /* odp_pktio_close in progress: no start, no second close */
	char name[64];
	odp_pool_t pool;
	odp_pktio_config_t config;
	int cls_enabled;
	int parse_layer;
	int default_cos;        /* -1 = NULL */
	int error_cos;          /* -1 = NULL */
	uint32_t headroom;
	odp_pktio_stats_t stats;
	/* the runtime's host-side counts (odpg_cls_pktio_count): added with
	 * atomics outside the lock (the transmitting threads count every
	 * send), read into stats by odp_pktio_stats: in_packets, in_octets,
	 * in_discards, out_packets, out_octets */
	uint64_t hc[5];
	struct bind_s *binds;   /* compiled tables, one per context in use */
} pktio_e;

/* A pktio's compiled table on one context and the sharded counters its
 * launches add into. A binding whose generation is old is stale: it is
 * folded and freed once no receive holds it. */
typedef struct bind_s {
	struct bind_s *next;
	odpg_ctx_t *ctx;
	odpg_table_t *tbl;
	odpg_counters_t *cnt;
	uint64_t gen;
	uint32_t ncos;
	uint64_t *cos_uid;      /* [ncos] CoS serials the table was compiled from */
	uint64_t *words;        /* [ODPG_COUNTER_WORDS(ncos)] fold buffer */
	uint64_t pktin_opt;
	uint32_t layer, classify;
	int refs;               /* receives in flight */
	int dirty;              /* launched since the last fold */
	int stale;
} bind_t;

static struct {
	int init;
	pthread_mutex_t lock;
	uint32_t max_cos, max_pmr, max_per_cos;
	cos_e *cos;
	pmr_e *pmr;
	pktio_e pktio[MAX_PKTIO];
	uint64_t generation;
	uint64_t next_uid;
	/* snapshot buffers */
	odpg_cos_t *s_cos;
	odpg_pmr_t *s_pmr;
	uint32_t *s_rule_pmr, *s_rule_dst;
} g = { 0, PTHREAD_MUTEX_INITIALIZER, REF_MAX_COS, REF_MAX_PMR, REF_MAX_PMR_PER_COS,
	NULL, NULL, {{0}}, 1, 1, NULL, NULL, NULL, NULL };

static void free_tables(void)
{
	if (g.cos) {
		for (uint32_t i = 0; i < g.max_cos; i++) {
			free(g.cos[i].pmr);
			free(g.cos[i].linked);
		}
	}
	free(g.cos);
	free(g.pmr);
	free(g.s_cos);
	free(g.s_pmr);
	free(g.s_rule_pmr);
	free(g.s_rule_dst);
	g.cos = NULL;
	g.pmr = NULL;
	g.s_cos = NULL;
	g.s_pmr = NULL;
	g.s_rule_pmr = NULL;
	g.s_rule_dst = NULL;
}

/* _odp_classification_init_global (odp_classification.c:92-125) */
static int ensure_init(void)
{
	if (g.init)
		return 0;
	g.cos = calloc(g.max_cos, sizeof(cos_e));
	g.pmr = calloc(g.max_pmr, sizeof(pmr_e));
	if (!g.cos || !g.pmr)
		goto fail;
	for (uint32_t i = 0; i < g.max_cos; i++) {
		g.cos[i].pmr = calloc(g.max_per_cos, sizeof(uint32_t));
		g.cos[i].linked = calloc(g.max_per_cos, sizeof(uint32_t));
		if (!g.cos[i].pmr || !g.cos[i].linked)
			goto fail;
	}
	for (uint32_t i = 0; i < g.max_pmr; i++)
		g.pmr[i].src_cos = -1;
	g.init = 1;
	return 0;
fail:
	free_tables();
	return -ENOMEM;
}

#define LOCK()   pthread_mutex_lock(&g.lock)
#define UNLOCK() pthread_mutex_unlock(&g.lock)

static inline uint32_t cos_to_ndx(odp_cos_t c)
{
	return (uint32_t)((uintptr_t)c - 1u);
}

static inline odp_cos_t cos_from_ndx(uint32_t n)
{
	return (odp_cos_t)(uintptr_t)(n + 1u);
}

static inline uint32_t pmr_to_ndx(odp_pmr_t p)
{
	return (uint32_t)((uintptr_t)p - 1u);
}

static inline odp_pmr_t pmr_from_ndx(uint32_t n)
{
	return (odp_pmr_t)(uintptr_t)(n + 1u);
}

/* get_cos_entry (odp_classification.c:439-449) */
static cos_e *get_cos(odp_cos_t c)
{
	uint32_t n = cos_to_ndx(c);

	if (!g.init || c == ODP_COS_INVALID || n >= g.max_cos || !g.cos[n].valid)
		return NULL;
	return &g.cos[n];
}

static pmr_e *get_pmr(odp_pmr_t p)
{
	uint32_t n = pmr_to_ndx(p);

	if (!g.init || p == ODP_PMR_INVALID || n >= g.max_pmr || !g.pmr[n].valid)
		return NULL;
	return &g.pmr[n];
}

static pktio_e *get_pktio(odp_pktio_t p)
{
	uintptr_t n = (uintptr_t)p;

	if (n == 0 || n > MAX_PKTIO || !g.pktio[n - 1].valid)
		return NULL;
	return &g.pktio[n - 1];
}

static void bump(void)
{
	g.generation++;
}

/* ---- bindings and their counters --------------------------------------- */
/* Sum a binding's device counters into the pktio's and the CoS's totals
 * (loop.c:304-374 pktio counters, odp_classification.c:1621-1622,1697-1698
 * CoS packets, odp_classification_internal.h:64-78 queue packets). */
static void bind_fold_locked(pktio_e *p, bind_t *b)
{
	if (!b->dirty || !b->cnt)
		return;
	const uint32_t nw = ODPG_COUNTER_WORDS(b->ncos);

	memset(b->words, 0, (size_t)nw * sizeof(uint64_t));
	if (odpg_counters_fold(b->cnt, b->words)) {
		ERR("counter fold failed\n");
		return;
	}
	b->dirty = 0;
	p->stats.in_packets += b->words[0];
	p->stats.in_octets += b->words[1];
	p->stats.in_errors += b->words[2];
	p->stats.in_discards += b->words[3];
	for (uint32_t c = 0; c < b->ncos && c < g.max_cos; c++) {
		cos_e *ce = &g.cos[c];
		const uint64_t *q = b->words + 4u + b->ncos + (size_t)c * ODPG_COS_QUEUE_MAX;

		if (ce->uid != b->cos_uid[c])
			continue;       /* the CoS was destroyed since the compile */
		ce->st_packets += b->words[4u + c];
		for (uint32_t k = 0; k < COS_QUEUE_MAX; k++)
			ce->q_packets[k] += q[k];
	}
}

static void bind_free(bind_t *b)
{
	odpg_counters_destroy(b->cnt);
	odpg_table_destroy(b->tbl);
	free(b->cos_uid);
	free(b->words);
	free(b);
}

/* unlink and free the pktio's bindings that match (ctx NULL = all), folding
 * their counts first unless `drop` */
static void binds_release_locked(pktio_e *p, const odpg_ctx_t *ctx, int drop)
{
	bind_t **pp = &p->binds;

	while (*pp) {
		bind_t *b = *pp;

		if (ctx && b->ctx != ctx) {
			pp = &b->next;
			continue;
		}
		if (!drop)
			bind_fold_locked(p, b);
		*pp = b->next;
		bind_free(b);
	}
}

static void fold_pktio_locked(pktio_e *p)
{
	for (bind_t *b = p->binds; b; b = b->next)
		bind_fold_locked(p, b);
}

static void fold_all_locked(void)
{
	for (int i = 0; i < MAX_PKTIO; i++)
		if (g.pktio[i].valid)
			fold_pktio_locked(&g.pktio[i]);
}

/* odpg_ctx_destroy() hook: nothing may keep a table or counters of a context
 * past its end (a later context at the same address must not find them) */
void odpg_cls_ctx_release(odpg_ctx_t *ctx)
{
	LOCK();
	for (int i = 0; i < MAX_PKTIO; i++)
		if (g.pktio[i].valid)
			binds_release_locked(&g.pktio[i], ctx, 0);
	UNLOCK();
}

int odpg_cls_set_limits(uint32_t max_cos, uint32_t max_pmr, uint32_t max_pmr_per_cos)
{
	int rc = 0;

	LOCK();
	if (g.init) {
		rc = -EBUSY;
	} else if (max_cos == 0 || max_cos > ODPG_MAX_COS || max_pmr == 0 ||
		   max_pmr > ODPG_MAX_PMR || max_pmr_per_cos == 0 ||
		   max_pmr_per_cos > ODPG_MAX_RULES_PER_COS) {
		rc = -EINVAL;
	} else {
		g.max_cos = max_cos;
		g.max_pmr = max_pmr;
		g.max_per_cos = max_pmr_per_cos;
	}
	UNLOCK();
	return rc;
}

void odpg_cls_reset(void)
{
	LOCK();
	for (int i = 0; i < MAX_PKTIO; i++)
		binds_release_locked(&g.pktio[i], NULL, 1);
	memset(g.pktio, 0, sizeof(g.pktio));
	free_tables();
	g.init = 0;
	g.max_cos = REF_MAX_COS;
	g.max_pmr = REF_MAX_PMR;
	g.max_per_cos = REF_MAX_PMR_PER_COS;
	g.generation++;
	UNLOCK();
}

uint64_t odpg_cls_generation(void)
{
	return g.generation;
}

/* odp_cls_capability (odp_classification.c:153-201) */
int odp_cls_capability(odp_cls_capability_t *capa)
{
	memset(capa, 0, sizeof(*capa));
	capa->max_pmr = g.max_pmr;
	capa->max_pmr_per_cos = g.max_per_cos;
	capa->max_terms_per_pmr = MAX_TERMS;
	capa->max_cos = g.max_cos;
	capa->max_cos_stats = capa->max_cos;
	capa->pmr_range_supported = 0;
	capa->supported_terms.bit.len = 1;
	capa->supported_terms.bit.ethtype_0 = 1;
	capa->supported_terms.bit.ethtype_x = 1;
	capa->supported_terms.bit.vlan_id_0 = 1;
	capa->supported_terms.bit.vlan_id_x = 1;
	capa->supported_terms.bit.vlan_pcp_0 = 1;
	capa->supported_terms.bit.dmac = 1;
	capa->supported_terms.bit.ip_proto = 1;
	capa->supported_terms.bit.ip_dscp = 1;
	capa->supported_terms.bit.udp_dport = 1;
	capa->supported_terms.bit.udp_sport = 1;
	capa->supported_terms.bit.tcp_dport = 1;
	capa->supported_terms.bit.tcp_sport = 1;
	capa->supported_terms.bit.sip_addr = 1;
	capa->supported_terms.bit.dip_addr = 1;
	capa->supported_terms.bit.sip6_addr = 1;
	capa->supported_terms.bit.dip6_addr = 1;
	capa->supported_terms.bit.ipsec_spi = 1;
	capa->supported_terms.bit.custom_frame = 1;
	capa->supported_terms.bit.custom_l3 = 1;
	capa->max_hash_queues = COS_QUEUE_MAX;
	capa->hash_protocols.proto.ipv4_udp = 1;
	capa->hash_protocols.proto.ipv4_tcp = 1;
	capa->hash_protocols.proto.ipv4 = 1;
	capa->hash_protocols.proto.ipv6_udp = 1;
	capa->hash_protocols.proto.ipv6_tcp = 1;
	capa->hash_protocols.proto.ipv6 = 1;
	capa->max_mark = MAX_MARK;
	capa->stats.cos.all_counters = 0x2 | 0x4;     /* packets, discards */
	capa->stats.queue.all_counters = 0x2 | 0x4;
	return 0;
}

void odp_cls_cos_param_init(odp_cls_cos_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->queue = ODP_QUEUE_INVALID;
	param->pool = ODP_POOL_INVALID;
	param->num_queue = 1;
	param->vector.enable = false;
	odp_queue_param_init(&param->queue_param);   /* as the reference (:137-146) */
}

void odp_cls_pmr_param_init(odp_pmr_param_t *param)
{
	memset(param, 0, sizeof(*param));
}

void odp_cls_pmr_create_opt_init(odp_pmr_create_opt_t *opt)
{
	opt->terms = NULL;
	opt->num_terms = 0;
	opt->mark = 0;
}

/* _odp_cls_update_hash_proto (odp_classification.c:210-223) */
static uint32_t hash_proto_bits(odp_pktin_hash_proto_t hp)
{
	uint32_t b = 0;

	if (hp.proto.ipv4 || hp.proto.ipv4_tcp || hp.proto.ipv4_udp)
		b |= 1;
	if (hp.proto.ipv6 || hp.proto.ipv6_tcp || hp.proto.ipv6_udp)
		b |= 2;
	if (hp.proto.ipv4_udp || hp.proto.ipv6_udp)
		b |= 4;
	if (hp.proto.ipv4_tcp || hp.proto.ipv6_tcp)
		b |= 8;
	return b;
}

/* the hash queues of CoS slot i (odp_classification.c:283-307): -1, with
 * the ones made so far destroyed again, if one cannot be created */
static int hash_queues_create(cos_e *c, uint32_t i, uint32_t num)
{
	for (uint32_t j = 0; j < num; j++) {
		char hq_name[ODP_QUEUE_NAME_LEN];

		snprintf(hq_name, sizeof(hq_name), "_odp_cos_hq_%u_%u", i, j);
		c->hq[j] = odp_queue_create(hq_name, &c->queue_param);
		if (c->hq[j] == ODP_QUEUE_INVALID) {
			while (j > 0)                  /* _cls_queue_unwind */
				odp_queue_destroy(c->hq[--j]);
			return -1;
		}
	}
	return 0;
}

/* odp_cls_cos_create (odp_classification.c:231-347) */
odp_cos_t odp_cls_cos_create(const char *name, const odp_cls_cos_param_t *param_in)
{
	odp_cls_cos_param_t param = *param_in;
	odp_cos_t ret = ODP_COS_INVALID;

	if (param.action == ODP_COS_ACTION_DROP) {
		param.num_queue = 1;
		param.queue = ODP_QUEUE_INVALID;
		param.pool = ODP_POOL_INVALID;
		param.vector.enable = 0;
	} else if (param.num_queue == 1 && param.queue == ODP_QUEUE_INVALID) {
		return ODP_COS_INVALID;
	}
	if (param.num_queue > COS_QUEUE_MAX || param.num_queue < 1)
		return ODP_COS_INVALID;
	if (param.vector.enable) {
		if (param.vector.pool == ODP_POOL_INVALID) {
			ERR("invalid packet vector pool\n");
			return ODP_COS_INVALID;
		}
		if (param.vector.max_size == 0) {
			ERR("vector.max_size is zero\n");
			return ODP_COS_INVALID;
		}
	}

	LOCK();
	if (ensure_init()) {
		UNLOCK();
		return ODP_COS_INVALID;
	}
	for (uint32_t i = 0; i < g.max_cos; i++) {
		cos_e *c = &g.cos[i];

		if (c->valid)
			continue;
		if (name == NULL)
			c->name[0] = 0;
		else
			snprintf(c->name, ODP_COS_NAME_LEN, "%s", name);
		for (uint32_t j = 0; j < g.max_per_cos; j++) {
			c->pmr[j] = 0;
			c->linked[j] = 0;
		}
		c->num_queue = param.num_queue;
		c->hash_proto = 0;
		if (param.num_queue > 1) {
			c->queue_param = param.queue_param;
			c->queue_group = 1;
			c->queue = ODP_QUEUE_INVALID;
			c->hash_proto = hash_proto_bits(param.hash_proto);
			if (hash_queues_create(c, i, param.num_queue))
				break;
		} else {
			c->queue_group = 0;
			c->queue = param.queue;
		}
		c->st_packets = 0;
		c->st_discards = 0;
		memset(c->q_packets, 0, sizeof(c->q_packets));
		memset(c->q_discards, 0, sizeof(c->q_discards));
		c->action = param.action;
		c->pool = param.pool;
		c->valid = 1;
		c->num_rule = 0;
		c->index = i;
		c->vector = param.vector;
		c->stats_enable = param.stats_enable;
		c->uid = g.next_uid++;
		ret = cos_from_ndx(i);
		bump();
		break;
	}
	if (ret == ODP_COS_INVALID)
		ERR("CLS_COS_MAX_ENTRY reached\n");
	UNLOCK();
	return ret;
}

int odp_cls_cos_create_multi(const char *name[], const odp_cls_cos_param_t param[],
			     odp_cos_t cos[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		odp_cos_t c = odp_cls_cos_create(name ? name[i] : NULL, &param[i]);

		if (c == ODP_COS_INVALID)
			return i == 0 ? -1 : i;
		cos[i] = c;
	}
	return i;
}

/* odp_cos_destroy (odp_classification.c:464-478) */
int odp_cos_destroy(odp_cos_t cos_id)
{
	int rc = 0;

	LOCK();
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		rc = -1;
	} else {
		if (c->queue_group)           /* _cls_queue_unwind */
			for (uint32_t j = 0; j < c->num_queue; j++)
				odp_queue_destroy(c->hq[j]);
		c->valid = 0;
		bump();
	}
	UNLOCK();
	return rc;
}

int odp_cos_destroy_multi(odp_cos_t cos[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		int r = odp_cos_destroy(cos[i]);

		if (r)
			return i == 0 ? r : i;
	}
	return i;
}

int odp_cos_queue_set(odp_cos_t cos_id, odp_queue_t queue)
{
	int rc = -1;

	LOCK();
	cos_e *c = get_cos(cos_id);

	if (!c)
		ERR("Invalid odp_cos_t handle\n");
	else if (queue == ODP_QUEUE_INVALID)
		ERR("Invalid queue\n");
	else if (c->num_queue != 1)
		ERR("Hashing enabled, cannot set queue\n");
	else {
		c->queue = queue;
		rc = 0;
		bump();
	}
	UNLOCK();
	return rc;
}

odp_queue_t odp_cos_queue(odp_cos_t cos_id)
{
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return ODP_QUEUE_INVALID;
	}
	return c->queue;
}

uint32_t odp_cls_cos_num_queue(odp_cos_t cos_id)
{
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return 0;
	}
	return c->num_queue;
}

/* odp_cls_cos_queues (odp_classification.c:546-578) */
uint32_t odp_cls_cos_queues(odp_cos_t cos_id, odp_queue_t queue[], uint32_t num)
{
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return 0;
	}
	if (c->num_queue == 1) {
		if (num == 0)
			return 1;
		queue[0] = c->queue;
		return 1;
	}
	uint32_t n = num < c->num_queue ? num : c->num_queue;

	for (uint32_t i = 0; i < n; i++)
		queue[i] = c->hq[i];
	return c->num_queue;
}

/* pmr_create_term (odp_classification.c:645-738) */
static int pmr_create_term(odpg_term_t *v, const odp_pmr_param_t *param)
{
	uint32_t size;
	int custom = 0;

	if (param->range_term) {
		ERR("PMR value range not supported\n");
		return -1;
	}
	switch (param->term) {
	case ODP_PMR_VLAN_PCP_0:
	case ODP_PMR_IPPROTO:
	case ODP_PMR_IP_DSCP:
		size = 1;
		break;
	case ODP_PMR_ETHTYPE_0:
	case ODP_PMR_ETHTYPE_X:
	case ODP_PMR_VLAN_ID_0:
	case ODP_PMR_VLAN_ID_X:
	case ODP_PMR_UDP_DPORT:
	case ODP_PMR_TCP_DPORT:
	case ODP_PMR_UDP_SPORT:
	case ODP_PMR_TCP_SPORT:
		size = 2;
		break;
	case ODP_PMR_LEN:
	case ODP_PMR_SIP_ADDR:
	case ODP_PMR_DIP_ADDR:
	case ODP_PMR_IPSEC_SPI:
	case ODP_PMR_LD_VNI:
		size = 4;
		break;
	case ODP_PMR_DMAC:
		size = 6;
		break;
	case ODP_PMR_SIP6_ADDR:
	case ODP_PMR_DIP6_ADDR:
		size = 16;
		break;
	case ODP_PMR_CUSTOM_FRAME:
	case ODP_PMR_CUSTOM_L3:
		custom = 1;
		size = MAX_TERM_SIZE;
		break;
	default:
		ERR("Bad PMR term\n");
		return -1;
	}
	if ((!custom && param->val_sz != size) || (custom && param->val_sz > size)) {
		ERR("Bad PMR value size: %u\n", param->val_sz);
		return -1;
	}
	memset(v, 0, sizeof(*v));
	v->term = (uint32_t)param->term;
	if (param->val_sz) {
		memcpy(v->value, param->match.value, param->val_sz);
		memcpy(v->mask, param->match.mask, param->val_sz);
	}
	for (uint32_t i = 0; i < param->val_sz; i++)
		v->value[i] &= v->mask[i];
	v->offset = param->offset;
	v->val_sz = param->val_sz;
	return 0;
}

/* cls_pmr_create (odp_classification.c:787-833) */
static odp_pmr_t cls_pmr_create(const odp_pmr_param_t *terms, int num_terms, uint16_t mark,
				odp_cos_t src_cos, odp_cos_t dst_cos)
{
	odp_pmr_t id = ODP_PMR_INVALID;

	LOCK();
	cos_e *src = get_cos(src_cos);
	cos_e *dst = get_cos(dst_cos);

	if (!src || !dst) {
		ERR("Invalid odp_cos_t handle\n");
		goto out;
	}
	if (num_terms > MAX_TERMS) {
		ERR("no of terms greater than supported CLS_PMRTERM_MAX\n");
		goto out;
	}
	if (src->num_rule == g.max_per_cos)
		goto out;
	for (uint32_t i = 0; i < g.max_pmr; i++) {
		pmr_e *p = &g.pmr[i];

		if (p->valid)
			continue;
		/* alloc_pmr (:419-437) marks the slot valid before the terms
		 * are checked; a bad term releases it again */
		p->valid = 1;
		p->num_pmr = num_terms > 0 ? (uint32_t)num_terms : 0;
		for (int t = 0; t < num_terms; t++) {
			if (pmr_create_term(&p->terms[t], &terms[t])) {
				p->valid = 0;
				goto out;
			}
		}
		p->mark = mark;
		src->pmr[src->num_rule] = i;
		src->linked[src->num_rule] = (uint32_t)(dst - g.cos);
		src->num_rule++;
		p->src_cos = (int)(src - g.cos);
		id = pmr_from_ndx(i);
		bump();
		goto out;
	}
	ERR("CLS_PMR_MAX_ENTRY reached\n");
out:
	UNLOCK();
	return id;
}

odp_pmr_t odp_cls_pmr_create(const odp_pmr_param_t *terms, int num_terms,
			     odp_cos_t src_cos, odp_cos_t dst_cos)
{
	return cls_pmr_create(terms, num_terms, 0, src_cos, dst_cos);
}

odp_pmr_t odp_cls_pmr_create_opt(const odp_pmr_create_opt_t *opt,
				 odp_cos_t src_cos, odp_cos_t dst_cos)
{
	if (opt == NULL) {
		ERR("Bad parameter\n");
		return ODP_PMR_INVALID;
	}
	if (opt->mark > MAX_MARK) {
		ERR("Too large mark value: %" PRIu64 "\n", opt->mark);
		return ODP_PMR_INVALID;
	}
	return cls_pmr_create(opt->terms, opt->num_terms, (uint16_t)opt->mark, src_cos, dst_cos);
}

int odp_cls_pmr_create_multi(const odp_pmr_create_opt_t opt[], odp_cos_t src_cos[],
			     odp_cos_t dst_cos[], odp_pmr_t pmr[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		odp_pmr_t p = odp_cls_pmr_create_opt(&opt[i], src_cos[i], dst_cos[i]);

		if (p == ODP_PMR_INVALID)
			return i == 0 ? -1 : i;
		pmr[i] = p;
	}
	return i;
}

/* odp_cls_pmr_destroy (odp_classification.c:740-768), including its
 * unconditional num_rule decrement */
int odp_cls_pmr_destroy(odp_pmr_t pmr_id)
{
	int rc = 0;

	LOCK();
	pmr_e *p = get_pmr(pmr_id);

	if (!p || p->src_cos < 0) {
		rc = -1;
	} else {
		cos_e *src = &g.cos[p->src_cos];
		uint32_t idx = pmr_to_ndx(pmr_id);
		uint32_t loc = src->num_rule;

		if (loc != 0) {
			loc -= 1;
			for (uint32_t i = 0; i <= loc; i++)
				if (src->pmr[i] == idx) {
					src->pmr[i] = src->pmr[loc];
					src->linked[i] = src->linked[loc];
				}
			src->num_rule--;
		}
		p->valid = 0;
		bump();
	}
	UNLOCK();
	return rc;
}

int odp_cls_pmr_destroy_multi(odp_pmr_t pmr[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		int r = odp_cls_pmr_destroy(pmr[i]);

		if (r)
			return i == 0 ? r : i;
	}
	return i;
}

int odp_cls_cos_pool_set(odp_cos_t cos_id, odp_pool_t pool)
{
	int rc = -1;

	LOCK();
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
	} else {
		c->pool = pool;
		rc = 0;
	}
	UNLOCK();
	return rc;
}

odp_pool_t odp_cls_cos_pool(odp_cos_t cos_id)
{
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return ODP_POOL_INVALID;
	}
	return c->pool;
}

/* odp_cls_cos_stats (odp_classification.c:1829-1847) */
int odp_cls_cos_stats(odp_cos_t cos_id, odp_cls_cos_stats_t *stats)
{
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return -1;
	}
	if (!stats) {
		ERR("Output structure NULL\n");
		return -1;
	}
	memset(stats, 0, sizeof(*stats));
	LOCK();
	fold_all_locked();
	stats->discards = c->st_discards;
	stats->packets = c->st_packets;
	UNLOCK();
	return 0;
}

/* _odp_cos_queue_idx (odp_classification_internal.h:43-60) */
static int cos_queue_idx(const cos_e *c, odp_queue_t q)
{
	if (c->num_queue == 1)
		return c->queue == q ? 0 : -1;
	for (uint32_t i = 0; i < c->num_queue; i++)
		if (c->hq[i] == q)
			return (int)i;
	return -1;
}

/* odp_cls_queue_stats (odp_classification.c:1849-1877) */
int odp_cls_queue_stats(odp_cos_t cos_id, odp_queue_t queue, odp_cls_queue_stats_t *stats)
{
	cos_e *c = get_cos(cos_id);
	int qi;

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		return -1;
	}
	if (!stats) {
		ERR("Output structure NULL\n");
		return -1;
	}
	qi = cos_queue_idx(c, queue);
	if (qi < 0) {
		ERR("Invalid odp_queue_t handle\n");
		return -1;
	}
	memset(stats, 0, sizeof(*stats));
	LOCK();
	fold_all_locked();
	stats->discards = c->q_discards[qi];
	stats->packets = c->q_packets[qi];
	UNLOCK();
	return 0;
}

/* thash_softrss (protocols/thash.h:81-99) with the default RSS key
 * (odp_classification.c:50-58), as the classify kernels compute it */
static uint32_t thash_words(const uint32_t *tuple, uint32_t n)
{
	static const uint32_t key[11] = {
		0x6d5a56dau, 0x255b0ec2u, 0x4167253du, 0x43a38fb0u, 0xd0ca2bcbu,
		0xae7b30b4u, 0x77cb2da3u, 0x8030f20cu, 0x6a42b73bu, 0xbeac01fau, 0u
	};
	uint32_t ret = 0;

	for (uint32_t j = 0; j < n; j++)
		for (uint32_t i = 0; i < 32; i++)
			if (tuple[j] & (1u << (31 - i)))
				ret ^= (key[j] << i) | (i ? (key[j + 1] >> (32 - i)) : 0u);
	return ret;
}

static int rd32_le(const odpg_packet_t *pk, uint32_t off, uint32_t *v)
{
	if ((uint64_t)off + 4u > pk->len)
		return -1;
	memcpy(v, pk->data + off, 4);
	return 0;
}

/* packet_rss_hash (odp_classification.c:1751-1817) on a parse result; hp is
 * the CoS's hash protocol bits (hash_proto_bits): 1 IPv4, 2 IPv6, 4 UDP,
 * 8 TCP */
static int packet_rss_hash(const odpg_packet_t *pk, uint32_t hp, uint32_t *hash)
{
	const uint64_t inf = pk->meta.input_flags;
	const uint32_t l3 = pk->meta.l3_offset, l4 = pk->meta.l4_offset;
	const int tcp = (inf >> 25) & 1, udp = (inf >> 24) & 1;
	const int ports = (tcp && (hp & 8u)) || (!tcp && udp && (hp & 4u));
	uint32_t tuple[9] = {0}, n = 0, x;

	if ((inf >> 15) & 1) {                         /* IPv4 */
		if (hp & 1u) {
			if (rd32_le(pk, l3 + 12u, &tuple[0]) || rd32_le(pk, l3 + 16u, &tuple[1]))
				return -1;
			n += 2;
		}
		if (ports) {
			if (rd32_le(pk, l4, &tuple[2]))
				return -1;
			n += 1;
		}
	} else if ((inf >> 16) & 1) {                  /* IPv6 */
		if (hp & 2u) {
			for (uint32_t k = 0; k < 4; k++) {
				if (rd32_le(pk, l3 + 8u + 4u * k, &x))
					return -1;
				tuple[k] = __builtin_bswap32(x);
				if (rd32_le(pk, l3 + 24u + 4u * k, &x))
					return -1;
				tuple[4 + k] = __builtin_bswap32(x);
			}
			n += 8;
		}
		if (ports) {
			if (rd32_le(pk, l4, &tuple[8]))
				return -1;
			n += 1;
		}
	}
	*hash = n ? thash_words(tuple, n) : 0u;
	return 0;
}

/* odp_cls_hash_result (odp_classification.c:384-414): get_dest_queue's
 * queue, hash & (CLS_COS_QUEUE_MAX - 1) modulo the CoS's queue count */
odp_queue_t odpg_cls_hash_result(odp_cos_t cos_id, const odpg_packet_t *pk)
{
	odp_queue_t q = ODP_QUEUE_INVALID;
	uint32_t h;

	LOCK();
	cos_e *c = get_cos(cos_id);

	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
	} else if (c->num_queue == 1) {
		q = c->queue;
	} else if (pk && pk->data && !packet_rss_hash(pk, c->hash_proto, &h)) {
		q = c->hq[(h & (COS_QUEUE_MAX - 1u)) % c->num_queue];
	}
	UNLOCK();
	return q;
}

/* the same on the runtime's packets (the frame and the parse result a
 * receive or odp_packet_parse left on it) */
odp_queue_t odp_cls_hash_result(odp_cos_t cos_id, odp_packet_t packet)
{
	odpg_packet_t view;

	if (packet == ODP_PACKET_INVALID || odpg_packet_view(packet, &view)) {
		ERR("Invalid odp_packet_t handle\n");
		return ODP_QUEUE_INVALID;
	}
	return odpg_cls_hash_result(cos_id, &view);
}

void odpg_cls_queue_count(odp_cos_t cos_id, odp_queue_t queue, int64_t packets,
			  uint64_t discards)
{
	LOCK();
	cos_e *c = get_cos(cos_id);
	const int qi = c ? cos_queue_idx(c, queue) : -1;

	if (qi >= 0) {
		c->q_packets[qi] += (uint64_t)packets;
		c->q_discards[qi] += discards;
	}
	UNLOCK();
}

/* odp_cls_print_all (odp_classification.c:1879-1981), reduced */
void odp_cls_print_all(void)
{
	LOCK();
	printf("\nClassifier info\n---------------\n");
	if (g.init) {
		for (uint32_t i = 0; i < g.max_cos; i++) {
			cos_e *c = &g.cos[i];

			if (!c->valid)
				continue;
			printf("  %s(%u): %u rule(s)%s\n", c->name, i + 1, c->num_rule,
			       c->action == ODP_COS_ACTION_DROP ? " [drop]" : "");
			for (uint32_t r = 0; r < c->num_rule; r++) {
				pmr_e *p = &g.pmr[c->pmr[r]];

				printf("    pmr(%u) terms=%u mark=%u -> %s(%u)\n", c->pmr[r] + 1,
				       p->num_pmr, p->mark, g.cos[c->linked[r]].name,
				       c->linked[r] + 1);
			}
		}
	}
	printf("\n");
	UNLOCK();
}

uint64_t odp_cos_to_u64(odp_cos_t hdl)
{
	return (uint64_t)(uintptr_t)hdl;
}

uint64_t odp_pmr_to_u64(odp_pmr_t hdl)
{
	return (uint64_t)(uintptr_t)hdl;
}

/* ---- loop pktio subset -------------------------------------------------- */
odp_pktio_t odp_pktio_open(const char *name, odp_pool_t pool, const odp_pktio_param_t *param)
{
	odp_pktio_t ret = ODP_PKTIO_INVALID;

	if (!name || (strncmp(name, "loop", 4) != 0 && strncmp(name, "pcap:", 5) != 0)) {
		ERR("only loop and pcap pktio are supported: %s\n", name ? name : "(null)");
		return ODP_PKTIO_INVALID;
	}
	LOCK();
	for (int i = 0; i < MAX_PKTIO; i++)
		if (g.pktio[i].valid && !strncmp(g.pktio[i].name, name, sizeof(g.pktio[i].name))) {
			UNLOCK();
			ERR("pktio device %s already opened\n", name);   /* odp_packet_io.c:406-410 */
			return ODP_PKTIO_INVALID;
		}
	for (int i = 0; i < MAX_PKTIO; i++) {
		pktio_e *p = &g.pktio[i];

		if (p->valid)
			continue;
		memset(p, 0, sizeof(*p));
		p->valid = 1;
		snprintf(p->name, sizeof(p->name), "%s", name);
		p->pool = pool;
		odp_pktio_config_init(&p->config);
		p->default_cos = -1;
		p->error_cos = -1;
		ret = (odp_pktio_t)(uintptr_t)(i + 1);
		bump();
		break;
	}
	UNLOCK();
	if (ret != ODP_PKTIO_INVALID && odpg_rt_pktio_open(ret, name, pool, param)) {
		odp_pktio_close(ret);
		return ODP_PKTIO_INVALID;
	}
	return ret;
}

/* odp_pktio_lookup (odp_packet_io.c:798-829): an open pktio by name */
odp_pktio_t odp_pktio_lookup(const char *name)
{
	odp_pktio_t ret = ODP_PKTIO_INVALID;

	if (!name)
		return ret;
	LOCK();
	for (int i = 0; i < MAX_PKTIO; i++)
		if (g.pktio[i].valid && !strncmp(g.pktio[i].name, name, sizeof(g.pktio[i].name))) {
			ret = (odp_pktio_t)(uintptr_t)(i + 1);
			break;
		}
	UNLOCK();
	return ret;
}

/* odp_pktio_close (odp_packet_io.c:497-545): refused while started
 * ("Missing odp_pktio_stop() before close", :507-510) or while a receive
 * holds one of its tables; only then is the receive state (capture, loop
 * ring, pktin / pktout queues) torn down and the slot freed */
int odp_pktio_close(odp_pktio_t hdl)
{
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || p->closing) {
		UNLOCK();
		return -1;
	}
	if (p->started) {
		UNLOCK();
		ERR("Missing odp_pktio_stop() before close.\n");
		return -1;
	}
	for (bind_t *b = p->binds; b; b = b->next)
		if (b->refs) {
			UNLOCK();
			ERR("pktio close during a receive\n");
			return -1;
		}
	/* marked closing before the lock is dropped for the runtime side: a
	 * start in that window is refused, and a stopped pktio takes no new
	 * receive (recv_impl, rx_burst), so nothing re-binds */
	p->closing = 1;
	UNLOCK();
	odpg_rt_pktio_close(hdl);
	LOCK();
	p = get_pktio(hdl);
	if (p) {
		binds_release_locked(p, NULL, 0);   /* CoS counts outlive the pktio */
		memset(p, 0, sizeof(*p));
		bump();
	}
	UNLOCK();
	return 0;
}

/* odp_queue_param_init (queue_basic.c:653-667): plain, MT, blocking;
 * scheduled queues get the parallel sync in the all-threads group */
void odp_queue_param_init(odp_queue_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->type = ODP_QUEUE_TYPE_PLAIN;
	param->enq_mode = ODP_QUEUE_OP_MT;
	param->deq_mode = ODP_QUEUE_OP_MT;
	param->sched.sync = ODP_SCHED_SYNC_PARALLEL;
	param->sched.group = ODP_SCHED_GROUP_ALL;
	param->nonblocking = ODP_BLOCKING;
	param->order = ODP_QUEUE_ORDER_KEEP;
}

/* odp_pktio_param_init (odp_packet_io.c:1304-1309) */
void odp_pktio_param_init(odp_pktio_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->in_mode = ODP_PKTIN_MODE_DIRECT;
	param->out_mode = ODP_PKTOUT_MODE_DIRECT;
}

/* odp_pktio_config_init (odp_packet_io.c:1327-1335) */
void odp_pktio_config_init(odp_pktio_config_t *config)
{
	memset(config, 0, sizeof(*config));
	config->parser.layer = ODP_PROTO_LAYER_ALL;
	config->reassembly.max_num_frags = 2;
	config->flow_control.pause_rx = ODP_PKTIO_LINK_PAUSE_OFF;
	config->flow_control.pause_tx = ODP_PKTIO_LINK_PAUSE_OFF;
}

/* odp_pktio_config (odp_packet_io.c:602-682) with the loop capability
 * (pktio/loop.c:650-670): timestamps + ipv4/udp/tcp/sctp checksum checks */
int odp_pktio_config(odp_pktio_t hdl, const odp_pktio_config_t *config)
{
	odp_pktio_config_t def;
	const uint64_t capa = ODPG_PKTIN_TS_ALL | ODPG_PKTIN_TS_PTP | ODPG_PKTIN_IPV4_CHKSUM |
			      ODPG_PKTIN_UDP_CHKSUM | ODPG_PKTIN_TCP_CHKSUM |
			      ODPG_PKTIN_SCTP_CHKSUM;
	int rc = 0;

	if (!config) {
		odp_pktio_config_init(&def);
		config = &def;
	}
	if (config->pktin.all_bits & ~capa) {
		ERR("Unsupported input configuration option\n");
		return -1;
	}
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p) {
		rc = -1;
	} else if (p->started) {
		rc = -1;
	} else {
		p->config = *config;
		bump();
	}
	UNLOCK();
	return rc;
}

/* odp_pktin_queue_param_init (odp_packet_io.c:1311-1318) */
void odp_pktin_queue_param_init(odp_pktin_queue_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->op_mode = ODP_PKTIO_OP_MT;
	param->num_queues = 1;
	odp_queue_param_init(&param->queue_param);
}

/* odp_pktin_queue_config (odp_packet_io.c): with the classifier enabled one
 * input queue; otherwise num_queues (at least 1, at most the capability).
 * The runtime creates the pktin event queue of SCHED / QUEUE mode. */
int odp_pktin_queue_config(odp_pktio_t hdl, const odp_pktin_queue_param_t *param)
{
	odp_pktin_queue_param_t def;
	int rc = 0;

	if (!param) {
		odp_pktin_queue_param_init(&def);
		param = &def;
	}
	if (!param->classifier_enable && param->num_queues == 0) {
		ERR("invalid num_queues for operation mode\n");
		return -1;
	}
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || p->started) {
		rc = -1;
	} else {
		p->cls_enabled = !!param->classifier_enable;
		bump();
	}
	UNLOCK();
	if (rc == 0)
		rc = odpg_rt_pktin_config(hdl, param->classifier_enable ? 1u : param->num_queues,
					  param->classifier_enable || !param->hash_enable ? 0u :
					  param->hash_proto.all_bits);
	return rc;
}

/* odp_pktio_start (odp_packet_io.c:684-720): parse_layer = ALL with cls */
int odp_pktio_start(odp_pktio_t hdl)
{
	int rc = 0;

	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || p->started || p->closing) {
		rc = -1;
	} else {
		p->parse_layer = p->cls_enabled ? ODP_PROTO_LAYER_ALL : (int)p->config.parser.layer;
		__atomic_store_n(&p->started, 1, __ATOMIC_RELEASE);
		bump();
	}
	UNLOCK();
	return rc;
}

int odp_pktio_stop(odp_pktio_t hdl)
{
	int rc = 0;

	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || !p->started)
		rc = -1;
	else
		__atomic_store_n(&p->started, 0, __ATOMIC_RELEASE);
	UNLOCK();
	if (!rc)
		odpg_rt_pktio_drain(hdl);
	return rc;
}

int odp_pktio_stats(odp_pktio_t hdl, odp_pktio_stats_t *stats)
{
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || !stats) {
		UNLOCK();
		return -1;
	}
	fold_pktio_locked(p);
	*stats = p->stats;
	stats->in_packets += __atomic_load_n(&p->hc[0], __ATOMIC_RELAXED);
	stats->in_octets += __atomic_load_n(&p->hc[1], __ATOMIC_RELAXED);
	stats->in_discards += __atomic_load_n(&p->hc[2], __ATOMIC_RELAXED);
	stats->out_packets += __atomic_load_n(&p->hc[3], __ATOMIC_RELAXED);
	stats->out_octets += __atomic_load_n(&p->hc[4], __ATOMIC_RELAXED);
	UNLOCK();
	return 0;
}

int odp_pktio_stats_reset(odp_pktio_t hdl)
{
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p) {
		UNLOCK();
		return -1;
	}
	fold_pktio_locked(p);
	memset(&p->stats, 0, sizeof(p->stats));
	for (int i = 0; i < 5; i++)
		__atomic_store_n(&p->hc[i], 0, __ATOMIC_RELAXED);
	UNLOCK();
	return 0;
}

uint64_t odp_pktio_to_u64(odp_pktio_t hdl)
{
	return (uint64_t)(uintptr_t)hdl;
}

/* odp_pktio_default_cos_set (odp_classification.c:580-601) */
int odp_pktio_default_cos_set(odp_pktio_t hdl, odp_cos_t default_cos)
{
	int rc = 0;

	LOCK();
	pktio_e *p = get_pktio(hdl);
	cos_e *c = NULL;

	if (!p) {
		ERR("Invalid odp_pktio_t handle\n");
		rc = -1;
		goto out;
	}
	if (default_cos != ODP_COS_INVALID) {
		c = get_cos(default_cos);
		if (!c) {
			ERR("Invalid odp_cos_t handle\n");
			rc = -1;
			goto out;
		}
	}
	p->default_cos = c ? (int)(c - g.cos) : -1;
	bump();
out:
	UNLOCK();
	return rc;
}

/* odp_pktio_error_cos_set (odp_classification.c:603-622) */
int odp_pktio_error_cos_set(odp_pktio_t hdl, odp_cos_t error_cos)
{
	int rc = 0;

	LOCK();
	pktio_e *p = get_pktio(hdl);
	cos_e *c;

	if (!p) {
		ERR("Invalid odp_pktio_t handle\n");
		rc = -1;
		goto out;
	}
	c = get_cos(error_cos);
	if (!c) {
		ERR("Invalid odp_cos_t handle\n");
		rc = -1;
		goto out;
	}
	p->error_cos = (int)(c - g.cos);
	bump();
out:
	UNLOCK();
	return rc;
}

int odp_pktio_skip_set(odp_pktio_t hdl, uint32_t offset)
{
	(void)hdl;
	(void)offset;
	return -ENOTSUP;
}

int odp_pktio_headroom_set(odp_pktio_t hdl, uint32_t headroom)
{
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p) {
		UNLOCK();
		ERR("Invalid odp_pktio_t handle\n");
		return -1;
	}
	p->headroom = headroom;
	UNLOCK();
	return 0;
}

/* ---- snapshot + GPU receive path ---------------------------------------- */
static int snapshot_locked(const pktio_e *p, odpg_rules_t *r)
{
	uint32_t slots = 0;

	if (ensure_init())
		return -ENOMEM;
	if (!g.s_cos) {
		g.s_cos = calloc(g.max_cos, sizeof(odpg_cos_t));
		g.s_pmr = calloc(g.max_pmr, sizeof(odpg_pmr_t));
		g.s_rule_pmr = calloc((size_t)g.max_cos * g.max_per_cos, sizeof(uint32_t));
		g.s_rule_dst = calloc((size_t)g.max_cos * g.max_per_cos, sizeof(uint32_t));
		if (!g.s_cos || !g.s_pmr || !g.s_rule_pmr || !g.s_rule_dst)
			return -ENOMEM;
	}
	for (uint32_t i = 0; i < g.max_cos; i++) {
		const cos_e *c = &g.cos[i];
		odpg_cos_t *s = &g.s_cos[i];

		s->valid = (uint32_t)c->valid;
		s->action = (uint32_t)c->action;
		s->num_queue = c->num_queue ? c->num_queue : 1;
		s->hash_proto = c->hash_proto;
		s->stats_enable = (uint32_t)c->stats_enable;
		s->num_rule = c->num_rule;
		s->rule_start = slots;
		for (uint32_t k = 0; k < c->num_rule; k++) {
			g.s_rule_pmr[slots] = c->pmr[k];
			g.s_rule_dst[slots] = c->linked[k];
			slots++;
		}
	}
	for (uint32_t i = 0; i < g.max_pmr; i++) {
		const pmr_e *pe = &g.pmr[i];
		odpg_pmr_t *s = &g.s_pmr[i];

		s->num_terms = pe->num_pmr;
		s->mark = pe->mark;
		memcpy(s->terms, pe->terms, sizeof(s->terms));
	}
	r->num_cos = g.max_cos;
	r->cos = g.s_cos;
	r->num_pmr = g.max_pmr;
	r->pmr = g.s_pmr;
	r->num_slots = slots;
	r->rule_pmr = g.s_rule_pmr;
	r->rule_dst = g.s_rule_dst;
	r->default_cos = p ? p->default_cos : -1;
	r->error_cos = p ? p->error_cos : -1;
	return 0;
}

int odpg_pktio_rules(odp_pktio_t hdl, odpg_rules_t *r)
{
	int rc;

	LOCK();
	pktio_e *p = get_pktio(hdl);

	rc = p ? snapshot_locked(p, r) : -EINVAL;
	UNLOCK();
	return rc;
}

/* recompile an idle binding for the current generation; nonzero = build a
 * new binding instead */
static int bind_update_locked(pktio_e *p, bind_t *b)
{
	odpg_rules_t r;

	if (snapshot_locked(p, &r) || odpg_table_update(b->ctx, b->tbl, &r))
		return -1;
	const uint32_t ncos = odpg_table_num_cos(b->tbl);
	int same = odpg_counters_match(b->cnt, b->tbl) && ncos == b->ncos;

	for (uint32_t c = 0; same && c < ncos && c < g.max_cos; c++)
		same = b->cos_uid[c] == (g.cos[c].valid ? g.cos[c].uid : 0);
	if (!same) {
		/* counts so far belong to the CoS the old table named */
		uint64_t *uid = calloc(ncos ? ncos : 1, sizeof(uint64_t));
		uint64_t *words = calloc(ODPG_COUNTER_WORDS(ncos), sizeof(uint64_t));

		if (!uid || !words) {
			free(uid);
			free(words);
			return -1;
		}
		bind_fold_locked(p, b);
		if (!odpg_counters_match(b->cnt, b->tbl)) {
			odpg_counters_destroy(b->cnt);
			b->cnt = NULL;
			if (odpg_counters_create(b->ctx, b->tbl, &b->cnt)) {
				free(uid);
				free(words);
				return -1;     /* the caller retires b */
			}
		}
		free(b->cos_uid);
		free(b->words);
		b->cos_uid = uid;
		b->words = words;
		b->ncos = ncos;
		for (uint32_t c = 0; c < ncos && c < g.max_cos; c++)
			b->cos_uid[c] = g.cos[c].valid ? g.cos[c].uid : 0;
	}
	b->gen = g.generation;
	b->pktin_opt = p->config.pktin.all_bits;
	b->layer = (uint32_t)p->parse_layer;
	b->classify = (uint32_t)p->cls_enabled;
	return 0;
}

/* the pktio's current binding on `ctx`, compiled now if the rules changed
 * since (stale bindings of the context are retired); NULL + *rc on error */
static bind_t *bind_get_locked(pktio_e *p, odpg_ctx_t *ctx, int *rc)
{
	bind_t *b, **pp = &p->binds;
	odpg_rules_t r;

	for (b = p->binds; b; b = b->next)
		if (b->ctx == ctx && !b->stale && b->gen == g.generation)
			return b;
	/* an idle binding of the context is recompiled in place: no device
	 * allocation, and its counters carry on when the CoS layout is kept */
	for (b = p->binds; b; b = b->next)
		if (b->ctx == ctx && !b->stale && !b->refs)
			break;
	if (b && !bind_update_locked(p, b))
		return b;
	while ((b = *pp)) {
		if (b->ctx == ctx && !b->stale)
			b->stale = 1;
		if (b->stale && !b->refs) {
			bind_fold_locked(p, b);
			*pp = b->next;
			bind_free(b);
		} else {
			pp = &b->next;
		}
	}
	if ((*rc = snapshot_locked(p, &r)))
		return NULL;
	b = calloc(1, sizeof(*b));
	if (!b) {
		*rc = -ENOMEM;
		return NULL;
	}
	if ((*rc = odpg_table_create(ctx, &r, &b->tbl))) {
		free(b);
		return NULL;
	}
	b->ncos = odpg_table_num_cos(b->tbl);
	b->cos_uid = calloc(b->ncos ? b->ncos : 1, sizeof(uint64_t));
	b->words = calloc(ODPG_COUNTER_WORDS(b->ncos), sizeof(uint64_t));
	if (!b->cos_uid || !b->words) {
		*rc = -ENOMEM;
		bind_free(b);
		return NULL;
	}
	if ((*rc = odpg_counters_create(ctx, b->tbl, &b->cnt))) {
		bind_free(b);
		return NULL;
	}
	for (uint32_t c = 0; c < b->ncos && c < g.max_cos; c++)
		b->cos_uid[c] = g.cos[c].valid ? g.cos[c].uid : 0;
	b->ctx = ctx;
	b->gen = g.generation;
	b->pktin_opt = p->config.pktin.all_bits;
	b->layer = (uint32_t)p->parse_layer;
	b->classify = (uint32_t)p->cls_enabled;
	b->next = p->binds;
	p->binds = b;
	return b;
}

/* a receive's hold on its binding (the launch's table and counters) */
typedef struct recv_tok {
	pktio_e *p;
	bind_t *bd;
} recv_tok_t;

static void recv_release(pktio_e *p, bind_t *bd)
{
	LOCK();
	if (--bd->refs == 0 && bd->stale) {
		bind_t **pp = &p->binds;

		while (*pp != bd)
			pp = &(*pp)->next;
		bind_fold_locked(p, bd);
		*pp = bd->next;
		bind_free(bd);
	}
	UNLOCK();
}

/* device_ptrs: 0 host buffers (staged copies), 1 device buffers, 2 pinned
 * host buffers the kernel reads and writes in place (zero-copy). With a
 * fence (zero-copy only) the launch is left running: the fence is recorded
 * behind it and *tok holds the binding until odpg_cls_pktio_recv_end */
static int recv_impl(odp_pktio_t hdl, odpg_ctx_t *ctx, const uint8_t *frames,
		     const odpg_desc_t *desc, uint32_t stride, uint32_t num,
		     int device_ptrs, odpg_out_t *out, uint16_t *mark, odpg_meta_t *meta,
		     odpg_fence_t *fence, recv_tok_t **tok)
{
	int rc = 0;
	odpg_batch_t b;
	odpg_result_t res;
	bind_t *bd;
	recv_tok_t *t = NULL;

	if (!ctx || !out || (fence && (device_ptrs != 2 || !tok)))
		return -EINVAL;
	if (fence && !(t = malloc(sizeof(*t))))
		return -ENOMEM;
	LOCK();
	pktio_e *p = get_pktio(hdl);

	if (!p || !p->started) {
		UNLOCK();
		free(t);
		return -EINVAL;
	}
	if (!(bd = bind_get_locked(p, ctx, &rc))) {
		UNLOCK();
		free(t);
		return rc;
	}
	bd->refs++;
	bd->dirty = 1;
	UNLOCK();

	/* the launch: verdicts, marks and the binding's counters (no host
	 * counting, no lock held) */
	memset(&b, 0, sizeof(b));
	b.frames = frames;
	b.desc = desc;
	b.stride = stride;
	b.num = num;
	b.pktin_opt = bd->pktin_opt;
	b.layer = bd->layer;
	b.classify = bd->classify;
	memset(&res, 0, sizeof(res));
	res.out = out;
	res.mark = mark;
	res.meta = meta;
	res.counters = bd->cnt;
	rc = device_ptrs ? odpg_classify(ctx, bd->tbl, &b, &res)
			 : odpg_classify_host(ctx, bd->tbl, &b, &res, 0);
	if (!rc && fence)
		rc = odpg_fence_record(ctx, fence);
	if (!rc && fence) {
		t->p = p;
		t->bd = bd;
		*tok = t;
		return 0;
	}
	/* zero-copy: complete before the results are read and the binding
	 * can go */
	if (fence)
		odpg_ctx_sync(ctx);
	else if (!rc && device_ptrs == 2)
		rc = odpg_ctx_sync(ctx);
	free(t);
	recv_release(p, bd);
	return rc;
}

int odpg_cls_pktio_recv_start_zc(odp_pktio_t hdl, odpg_ctx_t *ctx, const uint8_t *frames,
				 const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
				 odpg_meta_t *meta, odpg_fence_t *fence, void **token)
{
	if (!fence || !token)
		return -EINVAL;
	return recv_impl(hdl, ctx, frames, desc, 0, num, 2, out, NULL, meta, fence,
			 (recv_tok_t **)token);
}

void odpg_cls_pktio_recv_end(void *token)
{
	recv_tok_t *t = token;

	if (!t)
		return;
	recv_release(t->p, t->bd);
	free(t);
}

int odpg_pktio_recv_batch(odp_pktio_t hdl, odpg_ctx_t *ctx, const uint8_t *frames,
			  const odpg_desc_t *desc, uint32_t stride, uint32_t num,
			  int device_ptrs, odpg_out_t *out, uint16_t *mark)
{
	return recv_impl(hdl, ctx, frames, desc, stride, num, device_ptrs, out, mark, NULL, NULL,
			 NULL);
}

int odpg_cls_pktio_recv_meta(odp_pktio_t hdl, odpg_ctx_t *ctx, const uint8_t *frames,
			     const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
			     odpg_meta_t *meta)
{
	return recv_impl(hdl, ctx, frames, desc, 0, num, 0, out, NULL, meta, NULL, NULL);
}

int odpg_cls_pktio_recv_meta_zc(odp_pktio_t hdl, odpg_ctx_t *ctx, const uint8_t *frames,
				const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
				odpg_meta_t *meta)
{
	return recv_impl(hdl, ctx, frames, desc, 0, num, 2, out, NULL, meta, NULL, NULL);
}

void odpg_cls_pktio_count(odp_pktio_t hdl, int64_t in_packets, int64_t in_octets,
			  uint64_t in_discards, uint64_t out_packets, uint64_t out_octets)
{
	/* no lock: the pktio slots are a static table (an entry being closed
	 * counts into a slot nobody reads until it is opened again, and the
	 * open clears the counts) */
	pktio_e *p = get_pktio(hdl);
	const uint64_t v[5] = { (uint64_t)in_packets, (uint64_t)in_octets, in_discards,
				out_packets, out_octets };

	if (p)
		for (int i = 0; i < 5; i++)
			if (v[i])
				__atomic_fetch_add(&p->hc[i], v[i], __ATOMIC_RELAXED);
}

/* read without the lock: asked on every send and receive burst */
int odpg_cls_pktio_started(odp_pktio_t hdl)
{
	pktio_e *p = get_pktio(hdl);

	return p && __atomic_load_n(&p->started, __ATOMIC_ACQUIRE);
}

int odpg_cls_pktio_classifies(odp_pktio_t hdl)
{
	LOCK();
	pktio_e *p = get_pktio(hdl);
	const int r = p && p->started && p->cls_enabled;

	UNLOCK();
	return r;
}
