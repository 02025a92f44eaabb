/* SPDX-License-Identifier: BSD-3-Clause
 *
 * The ODP runtime subset around the GPU classifier (include/odp_api.h,
 * include/odp/rt.h, include/odp/helper/odph_api.h): what an ODP application
 * such as the reference's example/classifier needs to receive classified
 * packets — init, shared memory, packet pools, queues and the scheduler,
 * pcap / loop pktio input, packet accessors, time, CPU masks, helper
 * threads.
 *
 * Receive path: one burst of a pktio's input — the next frames of its
 * capture (pktio/pcap.c's pcapif_recv_pkt role: "pcap:in=<file>", with
 * ":loops=<n>"), or the packets sent on a loop device (pktio/loop.c: what
 * odp_pktout_send() put on the device comes back) — is classified on the
 * GPU through the classifier's own receive entry point
 * (odpg_pktio_recv_batch's path: parse, checksum verdicts, PMR -> CoS, the
 * pktio / CoS / queue counters). Every packet with a CoS goes to its CoS
 * queue, as loopback_recv() -> _odp_cls_enq() does (pktio/loop.c:304-374,
 * odp_classification_internal.h:139-225), in the CoS's pool (the pktio's
 * when the CoS names none, odp_classification.c:1734-1736); with the
 * classifier disabled the packet is the receive call's (DIRECT mode,
 * odp_pktin_recv) or goes to the pktin event queue (QUEUE / SCHED mode).
 * Bursts are taken by odp_pktin_recv(), by a dequeue from an empty QUEUE-mode
 * pktin queue, and by the scheduler for SCHED-mode pktios. The parse result
 * each packet carries is the odpg_meta_t the kernel wrote. Packets that get
 * no CoS, a drop CoS or a parse drop are freed there, as the reference's
 * receive loop frees them.
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
	odp_pktio_t pktin;         /* a QUEUE-mode pktin queue: dequeue polls it */
	odp_pktio_t pktout;        /* a pktout event queue: enqueue transmits */
} rt_queue_t;
#define QUEUE_MAGIC 0x51554555u

typedef struct rt_pktio {
	int valid;
	int in_mode;               /* odp_pktin_mode_t */
	int out_mode;              /* odp_pktout_mode_t */
	int loopdev;               /* "loop...": transmitted packets come back */
	odp_pool_t pool;           /* the pktio's packet pool */
	odpg_capture_t cap;
	int have_cap;
	uint32_t pos;              /* next frame of the capture */
	uint32_t loops, loop;      /* passes over the capture, done */
	int promisc;
	uint32_t mtu;
	uint32_t num_in, num_out;  /* configured input / output queues */
	rt_queue_t *inq;           /* pktin event queue (QUEUE / SCHED mode) */
	rt_queue_t *outq;          /* pktout event queue (QUEUE mode) */
	pthread_mutex_t ring_lock; /* the loop device's packets in flight */
	rt_pkt_t *ring_head, *ring_tail;
	uint8_t *stage;            /* loop packets gathered for one launch */
	size_t stage_cap;
} rt_pktio_t;

#define LOOP_MTU 65535u            /* LOOP_MTU_MAX (pktio/loop.c:45) */

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

odp_time_t odp_time_local_strict(void)
{
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
	return odp_time_local();
}

odp_time_t odp_time_global_strict(void)
{
	return odp_time_local_strict();
}

uint64_t odp_time_local_ns(void)
{
	return odp_time_local().nsec;
}

uint64_t odp_time_global_ns(void)
{
	return odp_time_local().nsec;
}

uint64_t odp_time_local_strict_ns(void)
{
	return odp_time_local_strict().nsec;
}

odp_time_t odp_time_local_from_ns(uint64_t ns)
{
	odp_time_t t = { ns };

	return t;
}

odp_time_t odp_time_global_from_ns(uint64_t ns)
{
	return odp_time_local_from_ns(ns);
}

odp_time_t odp_time_diff(odp_time_t t2, odp_time_t t1)
{
	odp_time_t t = { t2.nsec - t1.nsec };

	return t;
}

odp_time_t odp_time_sum(odp_time_t t1, odp_time_t t2)
{
	odp_time_t t = { t1.nsec + t2.nsec };

	return t;
}

odp_time_t odp_time_add_ns(odp_time_t time, uint64_t ns)
{
	time.nsec += ns;
	return time;
}

int odp_time_cmp(odp_time_t t2, odp_time_t t1)
{
	return t2.nsec < t1.nsec ? -1 : t2.nsec > t1.nsec;
}

uint64_t odp_time_local_res(void)
{
	return ODP_TIME_SEC_IN_NS;
}

void odp_time_wait_ns(uint64_t ns)
{
	struct timespec ts = { (time_t)(ns / ODP_TIME_SEC_IN_NS), (long)(ns % ODP_TIME_SEC_IN_NS) };

	nanosleep(&ts, NULL);
}

void odp_time_wait_until(odp_time_t time)
{
	const odp_time_t now = odp_time_local();

	if (time.nsec > now.nsec)
		odp_time_wait_ns(time.nsec - now.nsec);
}

/* ---- CPU cycle counter (the TSC on x86-64, else the nanosecond clock) ----- */
uint64_t odp_cpu_cycles(void)
{
#if defined(__x86_64__)
	return __builtin_ia32_rdtsc();
#else
	return odp_time_local().nsec;
#endif
}

uint64_t odp_cpu_cycles_diff(uint64_t c2, uint64_t c1)
{
	return c2 - c1;
}

uint64_t odp_cpu_cycles_max(void)
{
	return UINT64_MAX;
}

uint64_t odp_cpu_cycles_resolution(void)
{
	return 1;
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

/* packet pools of malloc'd packets, one segment each */
int odp_pool_capability(odp_pool_capability_t *capa)
{
	if (!capa)
		return -1;
	memset(capa, 0, sizeof(*capa));
	capa->max_pools = RT_MAX_POOL;
	capa->pkt.max_pools = RT_MAX_POOL;
	capa->pkt.max_len = LOOP_MTU;
	capa->pkt.max_num = 0;                 /* no limit but memory */
	capa->pkt.max_align = 64;
	capa->pkt.max_segs_per_pkt = 1;
	capa->pkt.min_seg_len = 1;
	capa->pkt.max_seg_len = LOOP_MTU;
	capa->pkt.max_num_subparam = 0;
	return 0;
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
static int pktout_send_impl(odp_pktio_t pktio, const odp_packet_t packets[], int num);
static void pktin_queue_fill(odp_pktio_t pktio);

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
	if (q->pktout) {                    /* pktout event queue: transmit */
		const odp_packet_t pkt = (odp_packet_t)k;

		return pktout_send_impl(q->pktout, &pkt, 1) == 1 ? 0 : -1;
	}
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
	if (q->pktin && !__atomic_load_n(&q->head, __ATOMIC_RELAXED))
		pktin_queue_fill(q->pktin);     /* QUEUE mode: receive a burst */
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

int odp_queue_enq_multi(odp_queue_t queue, const odp_event_t ev[], int num)
{
	int n = 0;

	while (n < num && odp_queue_enq(queue, ev[n]) == 0)
		n++;
	return n ? n : (num > 0 ? -1 : 0);
}

static int deq_multi(rt_queue_t *q, odp_event_t ev[], int num);

int odp_queue_deq_multi(odp_queue_t queue, odp_event_t ev[], int num)
{
	rt_queue_t *q = get_queue(queue);

	if (!q)
		return -1;
	if (q->pktin && !__atomic_load_n(&q->head, __ATOMIC_RELAXED))
		pktin_queue_fill(q->pktin);
	return deq_multi(q, ev, num);
}

/* every event here is a packet */
void odp_event_free(odp_event_t event)
{
	odp_packet_free((odp_packet_t)event);
}

void odp_event_free_multi(const odp_event_t event[], int num)
{
	for (int i = 0; i < num; i++)
		odp_packet_free((odp_packet_t)event[i]);
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

/* a queue the pktio owns: unlinked from use, its packets freed; the memory
 * stays (schedulers may still walk it) */
static void pktio_queue_kill(rt_queue_t *q)
{
	if (!q)
		return;
	pthread_mutex_lock(&q->lock);
	rt_pkt_t *k = q->head;

	q->head = q->tail = NULL;
	q->dead = 1;
	q->pktin = q->pktout = ODP_PKTIO_INVALID;
	pthread_mutex_unlock(&q->lock);
	while (k) {
		rt_pkt_t *nx = k->next;

		odp_packet_free((odp_packet_t)k);
		k = nx;
	}
}

/* "loop[...]" (pktio/loop.c) or "pcap:in=<file>[:loops=<n>]" (pktio/pcap.c's
 * device string) */
int odpg_rt_pktio_open(odp_pktio_t hdl, const char *name, odp_pool_t pool,
		       const odp_pktio_param_t *param)
{
	const uintptr_t n = (uintptr_t)hdl;
	rt_pktio_t *p;
	odp_pktio_param_t def;

	if (!n || n > RT_MAX_PKTIO)
		return -1;
	if (!param) {
		odp_pktio_param_init(&def);
		param = &def;
	}
	if (rt.pktio[n - 1].valid)          /* left over by odpg_cls_reset() */
		odpg_rt_pktio_close(hdl);
	p = &rt.pktio[n - 1];
	memset(p, 0, sizeof(*p));
	p->valid = 1;
	p->loops = 1;
	p->in_mode = param->in_mode;
	p->out_mode = param->out_mode;
	p->pool = pool;
	p->mtu = LOOP_MTU;
	p->loopdev = !strncmp(name, "loop", 4);
	pthread_mutex_init(&p->ring_lock, NULL);
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
		rt_pkt_t *k = p->ring_head;

		if (p->have_cap)
			odpg_pcap_free(&p->cap);
		pktio_queue_kill(p->inq);
		pktio_queue_kill(p->outq);
		while (k) {
			rt_pkt_t *nx = k->next;

			odp_packet_free((odp_packet_t)k);
			k = nx;
		}
		free(p->stage);
		pthread_mutex_destroy(&p->ring_lock);
		memset(p, 0, sizeof(*p));
	}
	pthread_mutex_unlock(&rt.poll_lock);
}

/* the input queues odp_pktin_queue_config() asked for; QUEUE / SCHED mode
 * get their event queue ("odp-pktin-<i>-<q>", odp_packet_io.c) */
int odpg_rt_pktin_config(odp_pktio_t hdl, uint32_t num_queues)
{
	rt_pktio_t *p = get_rt_pktio(hdl);
	odp_queue_param_t qp;
	char name[ODP_QUEUE_NAME_LEN];

	if (!p)
		return -1;
	if (p->in_mode == ODP_PKTIN_MODE_DISABLED)
		return 0;
	if (num_queues > 1) {
		ERR("pktio %" PRIu64 ": too many input queues\n", (uint64_t)(uintptr_t)hdl);
		return -1;
	}
	p->num_in = num_queues;
	if (p->in_mode != ODP_PKTIN_MODE_QUEUE && p->in_mode != ODP_PKTIN_MODE_SCHED)
		return 0;
	pktio_queue_kill(p->inq);
	odp_queue_param_init(&qp);
	qp.type = p->in_mode == ODP_PKTIN_MODE_SCHED ? ODP_QUEUE_TYPE_SCHED : ODP_QUEUE_TYPE_PLAIN;
	snprintf(name, sizeof(name), "odp-pktin-%u-0", (unsigned)(uintptr_t)hdl);
	p->inq = (rt_queue_t *)odp_queue_create(name, &qp);
	if (!p->inq)
		return -1;
	if (p->in_mode == ODP_PKTIN_MODE_QUEUE)
		p->inq->pktin = hdl;
	return 0;
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

#define ALIGN64(x) (((x) + 63u) & ~(size_t)63u)

/* One burst of the pktio's input through the GPU classifier (loopback_recv,
 * pktio/loop.c:304-374; pcapif_recv_pkt + the same classify step). Packets
 * with a CoS are enqueued on its queue; with the classifier disabled
 * (ODPG_COS_NOCLS) they are returned in pkts[]. *nret = packets returned.
 * Returns the frames taken from the input (0: none waiting), or -1.
 * Caller holds rt.poll_lock (the launch buffers are shared). */
static int rx_burst(rt_pktio_t *p, odp_pktio_t hdl, odp_packet_t pkts[], int num, int *nret)
{
	rt_pkt_t *src[RT_BURST];
	const uint8_t *frames;
	uint32_t n = 0, first = 0;

	*nret = 0;
	if (num > RT_BURST)
		num = RT_BURST;
	if (num <= 0 || !rt.init || !odpg_cls_pktio_started(hdl))
		return 0;
	if (p->loopdev) {
		size_t need = 0, off = 0;

		pthread_mutex_lock(&p->ring_lock);
		while (n < (uint32_t)num && p->ring_head) {
			src[n] = p->ring_head;
			p->ring_head = p->ring_head->next;
			need += ALIGN64(src[n]->len);
			n++;
		}
		if (!p->ring_head)
			p->ring_tail = NULL;
		pthread_mutex_unlock(&p->ring_lock);
		if (!n)
			return 0;
		if (need > p->stage_cap) {
			uint8_t *b = NULL;

			if (posix_memalign((void **)&b, 64, need)) {
				for (uint32_t k = 0; k < n; k++)
					odp_packet_free((odp_packet_t)src[k]);
				return -1;
			}
			free(p->stage);
			p->stage = b;
			p->stage_cap = need;
		}
		for (uint32_t k = 0; k < n; k++) {
			memcpy(p->stage + off, src[k]->data, src[k]->len);
			rt.desc[k].offset = (uint32_t)off;
			rt.desc[k].len = src[k]->len;
			off += ALIGN64(src[k]->len);
		}
		frames = p->stage;
	} else if (p->have_cap) {
		if (p->pos >= p->cap.num) {
			if (p->loops != 0 && p->loop + 1 >= p->loops)
				return 0;
			p->loop++;
			p->pos = 0;
		}
		first = p->pos;
		n = p->cap.num - first < (uint32_t)num ? p->cap.num - first : (uint32_t)num;
		if (!n)
			return 0;
		memcpy(rt.desc, p->cap.desc + first, n * sizeof(odpg_desc_t));
		frames = p->cap.frames;
	} else {
		return 0;
	}
	if (odpg_cls_pktio_recv_meta(hdl, rt.ctx, frames, rt.desc, n, rt.out, rt.meta)) {
		ERR("classify failed\n");
		if (p->loopdev)
			for (uint32_t k = 0; k < n; k++)
				odp_packet_free((odp_packet_t)src[k]);
		return -1;
	}
	if (!p->loopdev)
		p->pos += n;
	for (uint32_t k = 0; k < n; k++) {
		const uint32_t w = rt.out[k];
		const uint32_t len = rt.desc[k].len;
		rt_pkt_t *have = p->loopdev ? src[k] : NULL;
		odp_cos_t cos = ODP_COS_INVALID;
		odp_queue_t q = ODP_QUEUE_INVALID;
		odp_pool_t pool = p->pool;
		odp_packet_t pkt;

		if (ODPG_OUT_COS(w) != ODPG_COS_NOCLS) {
			q = dest_queue(w, &cos);
			if (q == ODP_QUEUE_INVALID || !get_queue(q)) {
				if (have)                 /* no CoS / drop / parse drop */
					odp_packet_free((odp_packet_t)have);
				continue;
			}
			if (odp_cls_cos_pool(cos) != ODP_POOL_INVALID)
				pool = odp_cls_cos_pool(cos);
		}
		if (have && have->pool == pool) {
			pkt = (odp_packet_t)have;
		} else {
			/* into the CoS's pool (_odp_pktio_packet_to_pool) */
			pkt = odp_packet_alloc(pool, len);
			if (pkt != ODP_PACKET_INVALID)
				memcpy(PK(pkt)->data, frames + rt.desc[k].offset, len);
			if (have)
				odp_packet_free((odp_packet_t)have);
			if (pkt == ODP_PACKET_INVALID) {
				const int counted = !(w & ODPG_OUT_ERROR);

				odpg_cls_pktio_count(hdl, counted ? -1 : 0,
						     counted ? -(int64_t)len : 0, 1, 0, 0);
				continue;
			}
		}
		PK(pkt)->meta = rt.meta[k];
		PK(pkt)->cos = cos;
		if (q == ODP_QUEUE_INVALID) {
			pkts[(*nret)++] = pkt;
		} else if (odp_queue_enq(q, (odp_event_t)pkt)) {
			odp_packet_free(pkt);
		}
	}
	return (int)n;
}

/* a burst of a QUEUE / SCHED mode pktio onto its pktin event queue */
static int rx_to_inq(rt_pktio_t *p, odp_pktio_t hdl)
{
	odp_packet_t pkts[RT_BURST];
	int nret;
	const int took = rx_burst(p, hdl, pkts, RT_BURST, &nret);

	for (int k = 0; k < nret; k++)
		if (!p->inq || odp_queue_enq((odp_queue_t)p->inq, (odp_event_t)pkts[k]))
			odp_packet_free(pkts[k]);
	return took;
}

static void pktin_queue_fill(odp_pktio_t hdl)
{
	pthread_mutex_lock(&rt.poll_lock);
	rt_pktio_t *p = get_rt_pktio(hdl);

	if (p && p->in_mode == ODP_PKTIN_MODE_QUEUE)
		rx_to_inq(p, hdl);
	pthread_mutex_unlock(&rt.poll_lock);
}

/* one burst of every SCHED-mode pktio (the scheduler's pktin poll).
 * Returns the frames taken (0: nothing waiting). */
static int poll_input(void)
{
	int got = 0;

	if (pthread_mutex_trylock(&rt.poll_lock))
		return 0;
	for (int i = 0; i < RT_MAX_PKTIO && rt.init; i++) {
		rt_pktio_t *p = &rt.pktio[i];

		if (!p->valid || p->in_mode != ODP_PKTIN_MODE_SCHED)
			continue;
		const int took = rx_to_inq(p, (odp_pktio_t)(uintptr_t)(i + 1));

		if (took > 0)
			got += took;
	}
	pthread_mutex_unlock(&rt.poll_lock);
	return got;
}

/* odp_pktin_queue (odp_packet_io.c:2404-2441) */
int odp_pktin_queue(odp_pktio_t pktio, odp_pktin_queue_t queues[], int num)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p || num < 0)
		return -1;
	if (p->in_mode == ODP_PKTIN_MODE_DISABLED)
		return 0;
	if (p->in_mode != ODP_PKTIN_MODE_DIRECT)
		return -1;
	for (int i = 0; queues && i < num && i < (int)p->num_in; i++) {
		queues[i].pktio = pktio;
		queues[i].index = i;
	}
	return (int)p->num_in;
}

/* odp_pktin_event_queue (odp_packet_io.c:2364-2402) */
int odp_pktin_event_queue(odp_pktio_t pktio, odp_queue_t queues[], int num)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p || num < 0)
		return -1;
	if (p->in_mode == ODP_PKTIN_MODE_DISABLED)
		return 0;
	if (p->in_mode != ODP_PKTIN_MODE_QUEUE && p->in_mode != ODP_PKTIN_MODE_SCHED)
		return -1;
	if (queues && num > 0 && p->inq)
		queues[0] = (odp_queue_t)p->inq;
	return p->inq ? 1 : 0;
}

/* DIRECT-mode receive: one burst through the GPU classifier */
int odp_pktin_recv(odp_pktin_queue_t queue, odp_packet_t packets[], int num)
{
	int nret = 0;

	pthread_mutex_lock(&rt.poll_lock);
	rt_pktio_t *p = get_rt_pktio(queue.pktio);

	if (!p || p->in_mode != ODP_PKTIN_MODE_DIRECT || queue.index < 0 ||
	    (uint32_t)queue.index >= p->num_in) {
		pthread_mutex_unlock(&rt.poll_lock);
		return -1;
	}
	const int rc = rx_burst(p, queue.pktio, packets, num, &nret);

	pthread_mutex_unlock(&rt.poll_lock);
	return rc < 0 ? -1 : nret;
}

/* per-queue counters: one input / output queue per pktio here, so queue 0
 * carries the interface's counters (loopback_pktin_stats /
 * loopback_pktout_stats, pktio/loop.c:762-786) */
static int in_queue_stats(odp_pktio_t pktio, uint32_t index, odp_pktin_queue_stats_t *st)
{
	odp_pktio_stats_t s;

	if (!st || index != 0 || odp_pktio_stats(pktio, &s))
		return -1;
	memset(st, 0, sizeof(*st));
	st->octets = s.in_octets;
	st->packets = s.in_packets;
	st->discards = s.in_discards;
	st->errors = s.in_errors;
	return 0;
}

static int out_queue_stats(odp_pktio_t pktio, uint32_t index, odp_pktout_queue_stats_t *st)
{
	odp_pktio_stats_t s;

	if (!st || index != 0 || odp_pktio_stats(pktio, &s))
		return -1;
	memset(st, 0, sizeof(*st));
	st->octets = s.out_octets;
	st->packets = s.out_packets;
	return 0;
}

/* odp_pktin_queue_stats (odp_packet_io.c:1696-1730): DIRECT mode only */
int odp_pktin_queue_stats(odp_pktin_queue_t queue, odp_pktin_queue_stats_t *stats)
{
	rt_pktio_t *p = get_rt_pktio(queue.pktio);

	if (!p || p->in_mode != ODP_PKTIN_MODE_DIRECT || queue.index < 0 ||
	    (uint32_t)queue.index >= p->num_in)
		return -1;
	return in_queue_stats(queue.pktio, (uint32_t)queue.index, stats);
}

/* odp_pktin_event_queue_stats (odp_packet_io.c:1732-1769): QUEUE / SCHED */
int odp_pktin_event_queue_stats(odp_pktio_t pktio, odp_queue_t queue,
				odp_pktin_queue_stats_t *stats)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p || (p->in_mode != ODP_PKTIN_MODE_SCHED && p->in_mode != ODP_PKTIN_MODE_QUEUE) ||
	    !p->inq || queue != (odp_queue_t)p->inq)
		return -1;
	return in_queue_stats(pktio, 0, stats);
}

/* ---- scheduler -------------------------------------------------------------- */
/* one scheduling priority and group; queues are limited by memory only */
int odp_schedule_capability(odp_schedule_capability_t *capa)
{
	if (!capa)
		return -1;
	memset(capa, 0, sizeof(*capa));
	capa->max_prios = 1;
	capa->max_groups = 1;
	capa->max_queues = 1u << 20;
	capa->max_queue_size = 0;          /* no limit */
	capa->lockfree_queues = ODP_SUPPORT_NO;
	capa->waitfree_queues = ODP_SUPPORT_NO;
	capa->order_wait = ODP_SUPPORT_NO;
	return 0;
}

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
	capa->max_output_queues = 1;
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

/* odp_pktout_queue_config (odp_packet_io.c): QUEUE mode gets its event
 * queue, whose enqueue transmits */
int odp_pktout_queue_config(odp_pktio_t pktio, const odp_pktout_queue_param_t *param)
{
	rt_pktio_t *p = get_rt_pktio(pktio);
	odp_pktout_queue_param_t def;
	odp_queue_param_t qp;
	char name[ODP_QUEUE_NAME_LEN];

	if (!param) {
		odp_pktout_queue_param_init(&def);
		param = &def;
	}
	if (!p || odpg_cls_pktio_started(pktio))
		return -1;
	if (p->out_mode == ODP_PKTOUT_MODE_DISABLED)
		return 0;
	if (param->num_queues == 0 || param->num_queues > 1) {
		ERR("pktio %" PRIu64 ": invalid number of output queues\n",
		    (uint64_t)(uintptr_t)pktio);
		return -1;
	}
	p->num_out = param->num_queues;
	if (p->out_mode != ODP_PKTOUT_MODE_QUEUE)
		return 0;
	pktio_queue_kill(p->outq);
	odp_queue_param_init(&qp);
	snprintf(name, sizeof(name), "odp-pktout-%u-0", (unsigned)(uintptr_t)pktio);
	p->outq = (rt_queue_t *)odp_queue_create(name, &qp);
	if (!p->outq)
		return -1;
	p->outq->pktout = pktio;
	return 0;
}

/* odp_pktout_queue (odp_packet_io.c:2474-2503): DIRECT mode */
int odp_pktout_queue(odp_pktio_t pktio, odp_pktout_queue_t queues[], int num)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p)
		return -1;
	if (p->out_mode == ODP_PKTOUT_MODE_DISABLED)
		return 0;
	if (p->out_mode != ODP_PKTOUT_MODE_DIRECT)
		return -1;
	for (int i = 0; queues && i < num && i < (int)p->num_out; i++) {
		queues[i].pktio = pktio;
		queues[i].index = i;
	}
	return (int)p->num_out;
}

/* odp_pktout_event_queue (odp_packet_io.c:2443-2472): QUEUE mode */
int odp_pktout_event_queue(odp_pktio_t pktio, odp_queue_t queues[], int num)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p)
		return -1;
	if (p->out_mode == ODP_PKTOUT_MODE_DISABLED)
		return 0;
	if (p->out_mode != ODP_PKTOUT_MODE_QUEUE)
		return -1;
	if (queues && num > 0 && p->outq)
		queues[0] = (odp_queue_t)p->outq;
	return p->outq ? 1 : 0;
}

/* transmit (loopback_send, pktio/loop.c:525-580): on a loop device the
 * packets go back to its input, up to the first one over the MTU (-1 if
 * that is the first); the pcap device here has no output file, so its
 * packets are consumed. Counted as out_packets / out_octets. */
static int pktout_send_impl(odp_pktio_t pktio, const odp_packet_t packets[], int num)
{
	rt_pktio_t *p = get_rt_pktio(pktio);
	uint64_t octets = 0;
	int n = 0;

	if (!p || num < 0)
		return -1;
	if (!odpg_cls_pktio_started(pktio))
		return 0;
	for (; n < num; n++) {
		rt_pkt_t *k = PK(packets[n]);

		if (k->len > p->mtu) {
			if (n == 0)
				return -1;
			break;
		}
		octets += k->len;
	}
	if (p->loopdev) {
		pthread_mutex_lock(&p->ring_lock);
		for (int i = 0; i < n; i++) {
			rt_pkt_t *k = PK(packets[i]);

			k->next = NULL;
			if (p->ring_tail)
				p->ring_tail->next = k;
			else
				p->ring_head = k;
			p->ring_tail = k;
		}
		pthread_mutex_unlock(&p->ring_lock);
	} else {
		odp_packet_free_multi(packets, n);
	}
	odpg_cls_pktio_count(pktio, 0, 0, 0, (uint64_t)n, octets);
	return n;
}

int odp_pktout_send(odp_pktout_queue_t queue, const odp_packet_t packets[], int num)
{
	rt_pktio_t *p = get_rt_pktio(queue.pktio);

	if (!p || p->out_mode != ODP_PKTOUT_MODE_DIRECT || queue.index < 0 ||
	    (uint32_t)queue.index >= p->num_out)
		return -1;
	return pktout_send_impl(queue.pktio, packets, num);
}

/* odp_pktout_queue_stats (odp_packet_io.c:1771-1805): DIRECT mode */
int odp_pktout_queue_stats(odp_pktout_queue_t queue, odp_pktout_queue_stats_t *stats)
{
	rt_pktio_t *p = get_rt_pktio(queue.pktio);

	if (!p || p->out_mode != ODP_PKTOUT_MODE_DIRECT || queue.index < 0 ||
	    (uint32_t)queue.index >= p->num_out)
		return -1;
	return out_queue_stats(queue.pktio, (uint32_t)queue.index, stats);
}

/* odp_pktout_event_queue_stats (odp_packet_io.c:1807-1843): QUEUE mode */
int odp_pktout_event_queue_stats(odp_pktio_t pktio, odp_queue_t queue,
				 odp_pktout_queue_stats_t *stats)
{
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (!p || p->out_mode != ODP_PKTOUT_MODE_QUEUE || !p->outq ||
	    queue != (odp_queue_t)p->outq)
		return -1;
	return out_queue_stats(pktio, 0, stats);
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
