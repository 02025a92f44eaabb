/* SPDX-License-Identifier: BSD-3-Clause
 *
 * The ODP runtime subset around the GPU classifier (include/odp_api.h,
 * include/odp/rt.h, include/odp/helper/odph_api.h): what an ODP application
 * such as the reference's example/classifier needs to receive classified
 * packets — init, shared memory, packet pools, queues and the scheduler,
 * pcap / loop pktio input, packet accessors, time, CPU masks, helper
 * threads.
 *
 * Receive path: the scheduler polls every started pktio opened in
 * ODP_PKTIN_MODE_SCHED. A poll takes a burst of frames from the pktio's
 * capture (pktio/pcap.c's pcapif_recv_pkt role: "pcap:in=<file>", with
 * ":loops=<n>"), classifies the burst on the GPU through the classifier's
 * own receive entry point (odpg_pktio_recv_batch's path: parse, checksum
 * verdicts, PMR -> CoS, the pktio / CoS / queue counters), and enqueues
 * every packet on its CoS's queue, as loopback_recv() ->
 * _odp_cls_enq() does (pktio/loop.c:304-374, odp_classification_internal.h:
 * 139-225). The parse result each packet carries is the odpg_meta_t the
 * kernel wrote. Packets that get no CoS, a drop CoS or a parse drop are
 * freed there, as the reference's receive loop frees them.
 *
 * This is a functional runtime, not a fast path: the device-resident batch
 * API (odpg.h) is the throughput path.
 */
#include <errno.h>
#include <inttypes.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/odp_api.h"
#include "../../include/odp/helper/odph_api.h"
#include "../../include/odpg_pcap.h"
#include "odp_rt_internal.h"

#define ERR(...) fprintf(stderr, "odp_rt: " __VA_ARGS__)

#define RT_MAX_PKTIO 64
#define RT_MAX_POOL  64
#define RT_BURST     1024

/* ---- objects -------------------------------------------------------------- */
typedef struct rt_pkt {
	odp_pool_t pool;
	uint32_t len;
	uint32_t cap;
	odp_cos_t cos;
	odpg_meta_t meta;
	uint8_t *data;
	struct rt_pkt *next;       /* queue link */
} rt_pkt_t;

typedef struct rt_pool {
	int valid;
	char name[ODP_POOL_NAME_LEN];
	odp_pool_param_t param;
	uint32_t in_use;
	pthread_mutex_t lock;
} rt_pool_t;

typedef struct rt_queue {
	uint32_t magic;
	char name[ODP_QUEUE_NAME_LEN];
	odp_queue_param_t param;
	pthread_mutex_t lock;
	rt_pkt_t *head, *tail;
	struct rt_queue *next_sched;
	int dead;
} rt_queue_t;
#define QUEUE_MAGIC 0x51554555u

typedef struct rt_pktio {
	int valid;
	int sched_in;              /* ODP_PKTIN_MODE_SCHED */
	odpg_capture_t cap;
	int have_cap;
	uint32_t pos;              /* next frame of the capture */
	uint32_t loops, loop;      /* passes over the capture, done */
	int promisc;
} rt_pktio_t;

static struct {
	pthread_mutex_t lock;      /* object tables */
	pthread_mutex_t poll_lock; /* one poller at a time */
	int init;
	odpg_ctx_t *ctx;
	rt_pool_t pool[RT_MAX_POOL];
	rt_pktio_t pktio[RT_MAX_PKTIO];
	rt_queue_t *sched;         /* scheduled queues */
	uint32_t rr;
	int next_thread;
	/* poll buffers */
	odpg_out_t out[RT_BURST];
	odpg_meta_t meta[RT_BURST];
	odpg_desc_t desc[RT_BURST];
} rt = { PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, 0, NULL, {{0}}, {{0}},
	 NULL, 0, 0, {0}, {{0}}, {{0}} };

static __thread int thr_id = -1;

/* ---- init / threads ------------------------------------------------------- */
void odp_init_param_init(odp_init_t *param)
{
	memset(param, 0, sizeof(*param));
	param->mem_model = ODP_MEM_MODEL_THREAD;
}

int odp_init_global(odp_instance_t *instance, const odp_init_t *param, const void *platform)
{
	(void)param;
	(void)platform;
	pthread_mutex_lock(&rt.lock);
	if (!rt.init) {
		int rc = odpg_ctx_create(0, NULL, &rt.ctx);

		if (rc) {
			pthread_mutex_unlock(&rt.lock);
			ERR("no MI355X context (odpg_ctx_create: %d): the classifier runs only on "
			    "the GPU\n", rc);
			return -1;
		}
		rt.init = 1;
	}
	pthread_mutex_unlock(&rt.lock);
	if (instance)
		*instance = (odp_instance_t)(uintptr_t)&rt;
	return 0;
}

int odp_term_global(odp_instance_t instance)
{
	(void)instance;
	pthread_mutex_lock(&rt.lock);
	if (rt.init) {
		odpg_ctx_destroy(rt.ctx);
		rt.ctx = NULL;
		rt.init = 0;
	}
	pthread_mutex_unlock(&rt.lock);
	return 0;
}

int odp_init_local(odp_instance_t instance, odp_thread_type_t thr_type)
{
	(void)instance;
	(void)thr_type;
	if (thr_id < 0)
		thr_id = __atomic_fetch_add(&rt.next_thread, 1, __ATOMIC_RELAXED);
	return 0;
}

int odp_term_local(void)
{
	return 0;
}

int odp_thread_id(void)
{
	return thr_id < 0 ? 0 : thr_id;
}

int odp_cpu_count(void)
{
	long n = sysconf(_SC_NPROCESSORS_ONLN);

	return n > 0 ? (int)n : 1;
}

void odp_sys_info_print(void)
{
	printf("\nODP system info\n---------------\n");
	printf("ODP API version: odp_amd classifier runtime (libodpg ABI %d)\n",
	       odpg_abi_version());
	printf("CPU count:       %i\n", odp_cpu_count());
	printf("GPU devices:     %i\n\n", odpg_device_count());
}

/* ---- CPU masks ------------------------------------------------------------ */
void odp_cpumask_zero(odp_cpumask_t *mask)
{
	memset(mask, 0, sizeof(*mask));
}

void odp_cpumask_set(odp_cpumask_t *mask, int cpu)
{
	if (cpu >= 0 && cpu < ODP_CPUMASK_SIZE)
		mask->bits[cpu / 64] |= 1ull << (cpu % 64);
}

int odp_cpumask_isset(const odp_cpumask_t *mask, int cpu)
{
	return cpu >= 0 && cpu < ODP_CPUMASK_SIZE && ((mask->bits[cpu / 64] >> (cpu % 64)) & 1);
}

int odp_cpumask_count(const odp_cpumask_t *mask)
{
	int n = 0;

	for (int k = 0; k < ODP_CPUMASK_SIZE / 64; k++)
		n += __builtin_popcountll(mask->bits[k]);
	return n;
}

int odp_cpumask_next(const odp_cpumask_t *mask, int cpu)
{
	for (int c = cpu + 1; c < ODP_CPUMASK_SIZE; c++)
		if (odp_cpumask_isset(mask, c))
			return c;
	return -1;
}

int odp_cpumask_first(const odp_cpumask_t *mask)
{
	return odp_cpumask_next(mask, -1);
}

/* hex string, most significant nibble first, "0x" prefix (cpumask.h) */
int32_t odp_cpumask_to_str(const odp_cpumask_t *mask, char *str, int32_t size)
{
	int top = -1;

	for (int c = ODP_CPUMASK_SIZE - 1; c >= 0 && top < 0; c--)
		if (odp_cpumask_isset(mask, c))
			top = c;
	const int nib = top < 0 ? 1 : top / 4 + 1;

	if (!str || size < nib + 3)
		return -1;
	str[0] = '0';
	str[1] = 'x';
	for (int k = 0; k < nib; k++) {
		const int n = nib - 1 - k;
		unsigned v = 0;

		for (int b = 0; b < 4; b++)
			v |= (unsigned)odp_cpumask_isset(mask, 4 * n + b) << b;
		str[2 + k] = "0123456789abcdef"[v];
	}
	str[2 + nib] = 0;
	return nib + 3;
}

/* workers on the CPUs of the affinity mask after the first (the control
 * thread's), as many as asked (0 = all) */
static int default_mask(odp_cpumask_t *mask, int num, int worker)
{
	cpu_set_t set;
	int n = 0, first = -1;

	odp_cpumask_zero(mask);
	if (sched_getaffinity(0, sizeof(set), &set))
		return 0;
	for (int c = 0; c < CPU_SETSIZE && c < ODP_CPUMASK_SIZE; c++) {
		if (!CPU_ISSET(c, &set))
			continue;
		if (first < 0) {
			first = c;
			if (worker && CPU_COUNT(&set) > 1)
				continue;
		}
		if (num && n >= num)
			break;
		odp_cpumask_set(mask, c);
		n++;
		if (!worker)
			break;
	}
	return n;
}

int odp_cpumask_default_worker(odp_cpumask_t *mask, int num)
{
	return default_mask(mask, num, 1);
}

int odp_cpumask_default_control(odp_cpumask_t *mask, int num)
{
	(void)num;
	return default_mask(mask, 1, 0);
}

/* ---- time ----------------------------------------------------------------- */
odp_time_t odp_time_local(void)
{
	struct timespec ts;
	odp_time_t t;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	t.nsec = (uint64_t)ts.tv_sec * ODP_TIME_SEC_IN_NS + (uint64_t)ts.tv_nsec;
	return t;
}

odp_time_t odp_time_global(void)
{
	return odp_time_local();
}

uint64_t odp_time_diff_ns(odp_time_t t2, odp_time_t t1)
{
	return t2.nsec - t1.nsec;
}

uint64_t odp_time_to_ns(odp_time_t time)
{
	return time.nsec;
}

void odp_time_wait_ns(uint64_t ns)
{
	struct timespec ts = { (time_t)(ns / ODP_TIME_SEC_IN_NS), (long)(ns % ODP_TIME_SEC_IN_NS) };

	nanosleep(&ts, NULL);
}

/* ---- shared memory -------------------------------------------------------- */
odp_shm_t odp_shm_reserve(const char *name, uint64_t size, uint64_t align, uint32_t flags)
{
	void *p = NULL;

	(void)name;
	(void)flags;
	if (align < sizeof(void *))
		align = sizeof(void *);
	if (posix_memalign(&p, align, size ? size : 1))
		return ODP_SHM_INVALID;
	memset(p, 0, size);
	return (odp_shm_t)p;
}

void *odp_shm_addr(odp_shm_t shm)
{
	return (void *)shm;
}

int odp_shm_free(odp_shm_t shm)
{
	if (shm == ODP_SHM_INVALID)
		return -1;
	free(shm);
	return 0;
}

/* ---- pools ---------------------------------------------------------------- */
static rt_pool_t *get_pool(odp_pool_t hdl)
{
	const uintptr_t n = (uintptr_t)hdl;

	return n && n <= RT_MAX_POOL && rt.pool[n - 1].valid ? &rt.pool[n - 1] : NULL;
}

void odp_pool_param_init(odp_pool_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->type = ODP_POOL_PACKET;
	param->pkt.seg_len = 1856;
	param->pkt.len = 1856;
	param->pkt.num = 1024;
}

odp_pool_t odp_pool_create(const char *name, const odp_pool_param_t *param)
{
	odp_pool_t ret = ODP_POOL_INVALID;

	if (!param || param->type != ODP_POOL_PACKET || !param->pkt.num) {
		ERR("only packet pools are supported\n");
		return ODP_POOL_INVALID;
	}
	pthread_mutex_lock(&rt.lock);
	for (int i = 0; i < RT_MAX_POOL; i++) {
		rt_pool_t *p = &rt.pool[i];

		if (p->valid)
			continue;
		memset(p, 0, sizeof(*p));
		p->valid = 1;
		snprintf(p->name, sizeof(p->name), "%s", name ? name : "");
		p->param = *param;
		pthread_mutex_init(&p->lock, NULL);
		ret = (odp_pool_t)(uintptr_t)(i + 1);
		break;
	}
	pthread_mutex_unlock(&rt.lock);
	return ret;
}

int odp_pool_destroy(odp_pool_t hdl)
{
	pthread_mutex_lock(&rt.lock);
	rt_pool_t *p = get_pool(hdl);
	int rc = p ? 0 : -1;

	if (p)
		p->valid = 0;
	pthread_mutex_unlock(&rt.lock);
	return rc;
}

void odp_pool_print(odp_pool_t hdl)
{
	rt_pool_t *p = get_pool(hdl);

	if (p)
		printf("pool %" PRIu64 " '%s': packets %u x %u B, in use %u\n",
		       (uint64_t)(uintptr_t)hdl, p->name, p->param.pkt.num, p->param.pkt.len,
		       p->in_use);
}

void odp_pool_print_all(void)
{
	printf("\nPools\n-----\n");
	for (int i = 0; i < RT_MAX_POOL; i++)
		if (rt.pool[i].valid)
			odp_pool_print((odp_pool_t)(uintptr_t)(i + 1));
	printf("\n");
}

odp_packet_t odp_packet_alloc(odp_pool_t pool, uint32_t len)
{
	rt_pool_t *p = get_pool(pool);
	rt_pkt_t *k;

	if (!p)
		return ODP_PACKET_INVALID;
	pthread_mutex_lock(&p->lock);
	if (p->in_use >= p->param.pkt.num) {
		pthread_mutex_unlock(&p->lock);
		return ODP_PACKET_INVALID;
	}
	p->in_use++;
	pthread_mutex_unlock(&p->lock);
	k = calloc(1, sizeof(*k));
	if (k)
		k->data = malloc(len ? len : 1);
	if (!k || !k->data) {
		if (k)
			free(k);
		pthread_mutex_lock(&p->lock);
		p->in_use--;
		pthread_mutex_unlock(&p->lock);
		return ODP_PACKET_INVALID;
	}
	k->pool = pool;
	k->len = len;
	k->cap = len;
	k->meta.l2_offset = k->meta.l3_offset = k->meta.l4_offset = 0xffff;
	return (odp_packet_t)k;
}

void odp_packet_free(odp_packet_t pkt)
{
	rt_pkt_t *k = (rt_pkt_t *)pkt;
	rt_pool_t *p;

	if (!k)
		return;
	p = get_pool(k->pool);
	if (p) {
		pthread_mutex_lock(&p->lock);
		p->in_use--;
		pthread_mutex_unlock(&p->lock);
	}
	free(k->data);
	free(k);
}

void odp_packet_free_multi(const odp_packet_t pkt[], int num)
{
	for (int i = 0; i < num; i++)
		odp_packet_free(pkt[i]);
}

/* ---- packet accessors ------------------------------------------------------ */
#define PK(p) ((rt_pkt_t *)(p))
#define IFLAG(p, bit) ((int)((PK(p)->meta.input_flags >> (bit)) & 1u))

odp_event_t odp_packet_to_event(odp_packet_t pkt)
{
	return (odp_event_t)pkt;
}

odp_packet_t odp_packet_from_event(odp_event_t ev)
{
	return (odp_packet_t)ev;
}

void odp_packet_from_event_multi(odp_packet_t pkt[], const odp_event_t ev[], int num)
{
	for (int i = 0; i < num; i++)
		pkt[i] = (odp_packet_t)ev[i];
}

uint32_t odp_packet_len(odp_packet_t pkt)
{
	return PK(pkt)->len;
}

void *odp_packet_data(odp_packet_t pkt)
{
	return PK(pkt)->data;
}

odp_pool_t odp_packet_pool(odp_packet_t pkt)
{
	return PK(pkt)->pool;
}

/* packet_flags.h over packet_parser_t (input_flags bits as
 * packet_inline_types.h:60-113, error flags as odpg_meta_t.flags) */
int odp_packet_has_error(odp_packet_t pkt)
{
	return (PK(pkt)->meta.flags & 0xFE000000u) != 0u;   /* error_flags (FL_ERROR_MASK) */
}

int odp_packet_has_eth(odp_packet_t pkt)  { return IFLAG(pkt, 7); }
int odp_packet_has_ipv4(odp_packet_t pkt) { return IFLAG(pkt, 15); }
int odp_packet_has_ipv6(odp_packet_t pkt) { return IFLAG(pkt, 16); }
int odp_packet_has_udp(odp_packet_t pkt)  { return IFLAG(pkt, 24); }
int odp_packet_has_tcp(odp_packet_t pkt)  { return IFLAG(pkt, 25); }
int odp_packet_has_flow_hash(odp_packet_t pkt) { return IFLAG(pkt, 2); }

static void *layer_ptr(odp_packet_t pkt, uint32_t off, uint32_t *len)
{
	if (off == 0xffffu || off >= PK(pkt)->len)
		return NULL;
	if (len)
		*len = PK(pkt)->len - off;
	return PK(pkt)->data + off;
}

void *odp_packet_l2_ptr(odp_packet_t pkt, uint32_t *len)
{
	return layer_ptr(pkt, PK(pkt)->meta.l2_offset, len);
}

void *odp_packet_l3_ptr(odp_packet_t pkt, uint32_t *len)
{
	return layer_ptr(pkt, PK(pkt)->meta.l3_offset, len);
}

void *odp_packet_l4_ptr(odp_packet_t pkt, uint32_t *len)
{
	return layer_ptr(pkt, PK(pkt)->meta.l4_offset, len);
}

uint32_t odp_packet_l2_offset(odp_packet_t pkt) { return PK(pkt)->meta.l2_offset; }
uint32_t odp_packet_l3_offset(odp_packet_t pkt) { return PK(pkt)->meta.l3_offset; }
uint32_t odp_packet_l4_offset(odp_packet_t pkt) { return PK(pkt)->meta.l4_offset; }

odp_cos_t odp_packet_cos(odp_packet_t pkt)
{
	return PK(pkt)->cos;
}

void odp_packet_print_data(odp_packet_t pkt, uint32_t offset, uint32_t len)
{
	const rt_pkt_t *k = PK(pkt);

	printf("Packet data (offset %u, len %u of %u):\n", offset, len, k->len);
	for (uint32_t i = 0; i < len && offset + i < k->len; i++)
		printf("%02x%s", k->data[offset + i], (i % 16 == 15) ? "\n" : " ");
	printf("\n");
}

/* ---- queues ---------------------------------------------------------------- */
static rt_queue_t *get_queue(odp_queue_t q)
{
	rt_queue_t *x = (rt_queue_t *)q;

	/* the classifier's own hash-queue handles are small integers */
	if (!x || (uintptr_t)x < 0x100000000ull || x->magic != QUEUE_MAGIC || x->dead)
		return NULL;
	return x;
}

odp_queue_t odp_queue_create(const char *name, const odp_queue_param_t *param)
{
	rt_queue_t *q = calloc(1, sizeof(*q));

	if (!q)
		return ODP_QUEUE_INVALID;
	q->magic = QUEUE_MAGIC;
	snprintf(q->name, sizeof(q->name), "%s", name ? name : "");
	if (param)
		q->param = *param;
	else
		odp_queue_param_init(&q->param);
	pthread_mutex_init(&q->lock, NULL);
	if (q->param.type == ODP_QUEUE_TYPE_SCHED) {
		pthread_mutex_lock(&rt.lock);
		q->next_sched = rt.sched;
		rt.sched = q;
		pthread_mutex_unlock(&rt.lock);
	}
	return (odp_queue_t)q;
}

int odp_queue_destroy(odp_queue_t queue)
{
	rt_queue_t *q = get_queue(queue);

	if (!q)
		return -1;
	pthread_mutex_lock(&q->lock);
	if (q->head) {
		pthread_mutex_unlock(&q->lock);
		ERR("queue '%s' not empty\n", q->name);
		return -1;
	}
	q->dead = 1;      /* stays linked: schedulers may still hold it */
	pthread_mutex_unlock(&q->lock);
	return 0;
}

int odp_queue_info(odp_queue_t queue, odp_queue_info_t *info)
{
	rt_queue_t *q = get_queue(queue);

	if (!q || !info)
		return -1;
	info->name = q->name;
	info->param = q->param;
	return 0;
}

int odp_queue_enq(odp_queue_t queue, odp_event_t ev)
{
	rt_queue_t *q = get_queue(queue);
	rt_pkt_t *k = (rt_pkt_t *)ev;

	if (!q || !k)
		return -1;
	k->next = NULL;
	pthread_mutex_lock(&q->lock);
	if (q->tail)
		q->tail->next = k;
	else
		q->head = k;
	q->tail = k;
	pthread_mutex_unlock(&q->lock);
	return 0;
}

odp_event_t odp_queue_deq(odp_queue_t queue)
{
	rt_queue_t *q = get_queue(queue);
	rt_pkt_t *k;

	if (!q)
		return ODP_EVENT_INVALID;
	pthread_mutex_lock(&q->lock);
	k = q->head;
	if (k) {
		q->head = k->next;
		if (!q->head)
			q->tail = NULL;
	}
	pthread_mutex_unlock(&q->lock);
	return (odp_event_t)k;
}

/* up to num events of one queue */
static int deq_multi(rt_queue_t *q, odp_event_t ev[], int num)
{
	int n = 0;

	pthread_mutex_lock(&q->lock);
	while (n < num && q->head) {
		rt_pkt_t *k = q->head;

		q->head = k->next;
		ev[n++] = (odp_event_t)k;
	}
	if (!q->head)
		q->tail = NULL;
	pthread_mutex_unlock(&q->lock);
	return n;
}

/* ---- pktio input ----------------------------------------------------------- */
static rt_pktio_t *get_rt_pktio(odp_pktio_t hdl)
{
	const uintptr_t n = (uintptr_t)hdl;

	return n && n <= RT_MAX_PKTIO && rt.pktio[n - 1].valid ? &rt.pktio[n - 1] : NULL;
}

/* "pcap:in=<file>[:loops=<n>]" (pktio/pcap.c's device string) */
int odpg_rt_pktio_open(odp_pktio_t hdl, const char *name, const odp_pktio_param_t *param)
{
	const uintptr_t n = (uintptr_t)hdl;
	rt_pktio_t *p;

	if (!n || n > RT_MAX_PKTIO)
		return -1;
	p = &rt.pktio[n - 1];
	memset(p, 0, sizeof(*p));
	p->valid = 1;
	p->loops = 1;
	p->sched_in = param && param->in_mode == ODP_PKTIN_MODE_SCHED;
	if (!strncmp(name, "pcap:", 5)) {
		char buf[1024], *save = NULL, *tok;

		snprintf(buf, sizeof(buf), "%s", name + 5);
		for (tok = strtok_r(buf, ":", &save); tok; tok = strtok_r(NULL, ":", &save)) {
			if (!strncmp(tok, "in=", 3)) {
				int rc = odpg_pcap_read(tok + 3, 64, &p->cap);

				if (rc) {
					ERR("cannot read capture %s: %d\n", tok + 3, rc);
					p->valid = 0;
					return -1;
				}
				p->have_cap = 1;
			} else if (!strncmp(tok, "loops=", 6)) {
				p->loops = (uint32_t)strtoul(tok + 6, NULL, 0);
			}
		}
		if (!p->have_cap) {
			ERR("pcap pktio without in=<file>: %s\n", name);
			p->valid = 0;
			return -1;
		}
	}
	return 0;
}

void odpg_rt_pktio_close(odp_pktio_t hdl)
{
	pthread_mutex_lock(&rt.poll_lock);
	rt_pktio_t *p = get_rt_pktio(hdl);

	if (p) {
		if (p->have_cap)
			odpg_pcap_free(&p->cap);
		memset(p, 0, sizeof(*p));
	}
	pthread_mutex_unlock(&rt.poll_lock);
}

/* the CoS queue a verdict names (get_dest_queue's pick for hash CoS) */
static odp_queue_t dest_queue(uint32_t w, odp_cos_t *cos)
{
	const uint32_t c = ODPG_OUT_COS(w);
	odp_queue_t qs[ODPG_COS_QUEUE_MAX];
	uint32_t n;

	if (c >= ODPG_COS_NOCLS || (w & ODPG_OUT_CLS_DROP))
		return ODP_QUEUE_INVALID;
	*cos = (odp_cos_t)(uintptr_t)(c + 1u);
	n = odp_cls_cos_queues(*cos, qs, ODPG_COS_QUEUE_MAX);
	if (n == 0)
		return ODP_QUEUE_INVALID;
	return n == 1 ? qs[0] : qs[ODPG_OUT_HASHQ(w) % n];
}

/* one burst of every polled pktio: classify on the GPU, enqueue by CoS.
 * Returns the packets enqueued (0: nothing left to read). */
static int poll_input(void)
{
	int got = 0;

	if (pthread_mutex_trylock(&rt.poll_lock))
		return 0;
	for (int i = 0; i < RT_MAX_PKTIO && rt.init; i++) {
		rt_pktio_t *p = &rt.pktio[i];
		const odp_pktio_t hdl = (odp_pktio_t)(uintptr_t)(i + 1);

		if (!p->valid || !p->sched_in || !p->have_cap || !odpg_cls_pktio_classifies(hdl))
			continue;
		if (p->pos >= p->cap.num) {
			if (p->loop + 1 >= p->loops && p->loops != 0)
				continue;
			p->loop++;
			p->pos = 0;
		}
		const uint32_t first = p->pos;
		const uint32_t num = p->cap.num - first < RT_BURST ? p->cap.num - first : RT_BURST;

		memcpy(rt.desc, p->cap.desc + first, num * sizeof(odpg_desc_t));
		if (odpg_cls_pktio_recv_meta(hdl, rt.ctx, p->cap.frames, rt.desc, num, rt.out,
					     rt.meta)) {
			ERR("classify failed\n");
			continue;
		}
		p->pos += num;
		for (uint32_t k = 0; k < num; k++) {
			odp_cos_t cos = ODP_COS_INVALID;
			const odp_queue_t q = dest_queue(rt.out[k], &cos);
			odp_pool_t pool = cos != ODP_COS_INVALID ? odp_cls_cos_pool(cos)
								 : ODP_POOL_INVALID;
			const odpg_desc_t *d = &p->cap.desc[first + k];
			odp_packet_t pkt;

			if (q == ODP_QUEUE_INVALID || !get_queue(q))
				continue;         /* no CoS / drop / parse drop: freed */
			if (pool == ODP_POOL_INVALID)
				continue;
			pkt = odp_packet_alloc(pool, d->len);
			if (pkt == ODP_PACKET_INVALID)
				continue;         /* pool empty: dropped, as the reference */
			memcpy(PK(pkt)->data, p->cap.frames + d->offset, d->len);
			PK(pkt)->meta = rt.meta[k];
			PK(pkt)->cos = cos;
			if (odp_queue_enq(q, (odp_event_t)pkt))
				odp_packet_free(pkt);
			else
				got++;
		}
	}
	pthread_mutex_unlock(&rt.poll_lock);
	return got;
}

/* ---- scheduler -------------------------------------------------------------- */
void odp_schedule_config_init(odp_schedule_config_t *config)
{
	memset(config, 0, sizeof(*config));
}

int odp_schedule_config(const odp_schedule_config_t *config)
{
	(void)config;
	return 0;
}

uint64_t odp_schedule_wait_time(uint64_t ns)
{
	return ns;
}

int odp_schedule_default_prio(void)
{
	return 0;
}

static int sched_once(odp_queue_t *from, odp_event_t ev[], int num)
{
	pthread_mutex_lock(&rt.lock);
	rt_queue_t *list = rt.sched;
	uint32_t skip = rt.rr++;
	pthread_mutex_unlock(&rt.lock);

	int nq = 0;

	for (rt_queue_t *q = list; q; q = q->next_sched)
		nq++;
	for (int pass = 0; pass < nq; pass++) {
		rt_queue_t *q = list;

		for (uint32_t s = (skip + (uint32_t)pass) % (uint32_t)nq; s; s--)
			q = q->next_sched;
		if (q->dead)
			continue;
		const int n = deq_multi(q, ev, num);

		if (n) {
			if (from)
				*from = (odp_queue_t)q;
			return n;
		}
	}
	return 0;
}

int odp_schedule_multi(odp_queue_t *from, uint64_t wait, odp_event_t events[], int num)
{
	const odp_time_t t0 = odp_time_local();

	for (;;) {
		int n = sched_once(from, events, num);

		if (n)
			return n;
		if (poll_input())
			continue;
		if (wait == ODP_SCHED_NO_WAIT)
			return 0;
		if (wait != ODP_SCHED_WAIT && odp_time_diff_ns(odp_time_local(), t0) >= wait)
			return 0;
		odp_time_wait_ns(50 * ODP_TIME_USEC_IN_NS);
	}
}

odp_event_t odp_schedule(odp_queue_t *from, uint64_t wait)
{
	odp_event_t ev = ODP_EVENT_INVALID;

	odp_schedule_multi(from, wait, &ev, 1);
	return ev;
}

/* ---- pktio output and capabilities ----------------------------------------- */
int odp_pktio_capability(odp_pktio_t pktio, odp_pktio_capability_t *capa)
{
	if (!get_rt_pktio(pktio) || !capa)
		return -1;
	memset(capa, 0, sizeof(*capa));
	capa->max_input_queues = 1;
	capa->max_output_queues = ODP_PKTIN_MAX_QUEUES;
	odp_pktio_config_init(&capa->config);
	capa->config.pktin.bit.ipv4_chksum = 1;
	capa->config.pktin.bit.udp_chksum = 1;
	capa->config.pktin.bit.tcp_chksum = 1;
	capa->config.pktin.bit.sctp_chksum = 1;
	capa->set_op.op.promisc_mode = 1;
	return 0;
}

void odp_pktout_queue_param_init(odp_pktout_queue_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->op_mode = ODP_PKTIO_OP_MT;
	param->num_queues = 1;
}

int odp_pktout_queue_config(odp_pktio_t pktio, const odp_pktout_queue_param_t *param)
{
	if (!get_rt_pktio(pktio) || !param || param->num_queues > ODP_PKTIN_MAX_QUEUES)
		return -1;
	return 0;
}

int odp_pktout_queue(odp_pktio_t pktio, odp_pktout_queue_t queues[], int num)
{
	if (!get_rt_pktio(pktio))
		return -1;
	for (int i = 0; i < num; i++) {
		queues[i].pktio = pktio;
		queues[i].index = i;
	}
	return num;
}

/* transmit: the pcap / loop pktio here has no wire; packets are consumed */
int odp_pktout_send(odp_pktout_queue_t queue, const odp_packet_t packets[], int num)
{
	if (!get_rt_pktio(queue.pktio))
		return -1;
	odp_packet_free_multi(packets, num);
	return num;
}

int odp_pktio_promisc_mode(odp_pktio_t pktio)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	return p ? p->promisc : -1;
}

int odp_pktio_promisc_mode_set(odp_pktio_t pktio, odp_bool_t enable)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p)
		return -1;
	p->promisc = enable ? 1 : 0;
	return 0;
}

/* the pcap pktio's fixed address (pktio/pcap.c:pcapif_mac_addr_get) */
int odp_pktio_mac_addr(odp_pktio_t pktio, void *mac_addr, int size)
{
	static const uint8_t mac[6] = { 0x02, 0xe9, 0x34, 0x80, 0x73, 0x04 };

	if (!get_rt_pktio(pktio) || size < 6)
		return -1;
	memcpy(mac_addr, mac, 6);
	return 6;
}

/* ---- helper: options, threads, parsers ------------------------------------- */
int odph_parse_options(int argc, char *argv[])
{
	int out = 1;

	for (int i = 1; i < argc; i++) {
		if (!strncmp(argv[i], "--odph_", 7))
			continue;         /* helper options: thread model only */
		argv[out++] = argv[i];
	}
	if (out < argc)
		argv[out] = NULL;
	return out;
}

int odph_options(odph_helper_options_t *options)
{
	memset(options, 0, sizeof(*options));
	options->mem_model = ODP_MEM_MODEL_THREAD;
	return 0;
}

void odph_thread_common_param_init(odph_thread_common_param_t *param)
{
	memset(param, 0, sizeof(*param));
}

void odph_thread_param_init(odph_thread_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->thr_type = ODP_THREAD_WORKER;
}

static void *thread_main(void *arg)
{
	odph_thread_t *t = arg;

	odp_init_local(t->instance, t->param.thr_type);
	t->status = t->param.start ? t->param.start(t->param.arg) : 0;
	odp_term_local();
	return NULL;
}

int odph_thread_create(odph_thread_t thread[], const odph_thread_common_param_t *param,
		       const odph_thread_param_t thr_param[], int num)
{
	int cpu = param->cpumask ? odp_cpumask_first(param->cpumask) : -1;
	int n = 0;

	for (int i = 0; i < num; i++) {
		odph_thread_t *t = &thread[i];
		pthread_t tid;
		pthread_attr_t attr;

		memset(t, 0, sizeof(*t));
		t->param = thr_param[param->share_param ? 0 : i];
		t->instance = param->instance;
		t->cpu = cpu;
		pthread_attr_init(&attr);
		if (cpu >= 0 && cpu < CPU_SETSIZE) {
			cpu_set_t set;

			CPU_ZERO(&set);
			CPU_SET(cpu, &set);
			pthread_attr_setaffinity_np(&attr, sizeof(set), &set);
		}
		if (pthread_create(&tid, &attr, thread_main, t)) {
			pthread_attr_destroy(&attr);
			break;
		}
		pthread_attr_destroy(&attr);
		t->thread = (uint64_t)tid;
		t->started = 1;
		n++;
		if (param->cpumask) {
			const int nx = odp_cpumask_next(param->cpumask, cpu);

			cpu = nx >= 0 ? nx : odp_cpumask_first(param->cpumask);
		}
	}
	return n;
}

int odph_thread_join(odph_thread_t thread[], int num)
{
	int n = 0;

	for (int i = 0; i < num; i++) {
		if (!thread[i].started)
			continue;
		pthread_join((pthread_t)thread[i].thread, NULL);
		thread[i].started = 0;
		n++;
	}
	return n;
}

/* "aa:bb:cc:dd:ee:ff" (helper/eth.c odph_eth_addr_parse) */
int odph_eth_addr_parse(odph_ethaddr_t *mac, const char *str)
{
	unsigned b[6];
	char tail;

	if (!str || sscanf(str, "%x:%x:%x:%x:%x:%x%c", &b[0], &b[1], &b[2], &b[3], &b[4], &b[5],
			   &tail) != 6)
		return -1;
	for (int i = 0; i < 6; i++) {
		if (b[i] > 255)
			return -1;
		mac->addr[i] = (uint8_t)b[i];
	}
	return 0;
}

/* "a.b.c.d" in host byte order (helper/ip.c odph_ipv4_addr_parse) */
int odph_ipv4_addr_parse(uint32_t *ip_addr, const char *str)
{
	unsigned b[4];
	char tail;

	if (!str || sscanf(str, "%u.%u.%u.%u%c", &b[0], &b[1], &b[2], &b[3], &tail) != 4)
		return -1;
	for (int i = 0; i < 4; i++)
		if (b[i] > 255)
			return -1;
	*ip_addr = (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3];
	return 0;
}

char *odph_strcpy(char *dst, const char *src, size_t sz)
{
	if (sz == 0)
		return dst;
	strncpy(dst, src, sz - 1);
	dst[sz - 1] = 0;
	return dst;
}
