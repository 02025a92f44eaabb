/* SPDX-License-Identifier: BSD-3-Clause
 *
 * The ODP runtime subset around the GPU classifier (include/odp_api.h,
 * include/odp/rt.h, include/odp/helper/odph_api.h): what an ODP application
 * such as the reference's example/classifier or test/performance's
 * odp_pktio_perf needs to receive classified packets — init, thread ids,
 * named shared memory, barriers, packet pools, queues and the scheduler,
 * pcap / loop pktio input, packet accessors and odp_packet_parse, time, CPU
 * masks, helper threads.
 *
 * Receive path: one burst of a pktio's input — the next frames of its
 * capture (pktio/pcap.c's pcapif_recv_pkt role: "pcap:in=<file>", with
 * ":loops=<n>"), or the packets sent on a loop device (pktio/loop.c: what
 * odp_pktout_send() put on the device comes back) — is classified on the
 * GPU through the classifier's own receive entry point
 * (odpg_pktio_recv_batch's path: parse, checksum verdicts, PMR -> CoS, the
 * pktio / CoS / queue counters). Every packet with a CoS goes to its CoS
 * queue (the hash queue get_dest_queue picks for a hash-queue CoS), in the
 * CoS's pool (the pktio's when the CoS names none, odp_classification.c:
 * 1734-1736), and consecutive packets for the same (CoS, queue) are
 * enqueued with one odp_queue_enq_multi, as loopback_recv() ->
 * _odp_cls_enq() batches them (pktio/loop.c:304-374,
 * odp_classification_internal.h:139-225); a failed enqueue frees the rest
 * of the run and counts it as the queue's discards. With the classifier
 * disabled the packet is the receive call's (DIRECT mode, odp_pktin_recv)
 * or goes to the pktin event queue (QUEUE / SCHED mode). Bursts are taken
 * by odp_pktin_recv(), by a dequeue from an empty QUEUE-mode pktin queue,
 * and by the scheduler for SCHED-mode pktios. The parse result each packet
 * carries is the odpg_meta_t the kernel wrote (the packet_parser_t layout,
 * cls_mark included), which the odp_packet_has_* / chksum status / cls_mark
 * accessors decode. Packets that get no CoS, a drop CoS or a parse drop are
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
#define RX_PF        8         /* packets prefetched ahead in staging / delivery */
#ifndef RX_CHUNK
#define RX_CHUNK     64        /* packets a delivering thread takes at a time */
#endif
#define RT_INFLIGHT  4              /* receive bursts in flight per pktio */
#define RT_MAX_DEV   16             /* device contexts (ODPG_DEVICES) */
#define RT_MAXQ      16             /* input / output queues of a loop device */

/* ---- objects -------------------------------------------------------------- */
#define PKT_MAGIC 0x504b5452u

/* the first 64 bytes hold what receive touches (staging reads len and
 * data, delivery writes pool .. input): one line per packet there */
typedef struct rt_pkt {
	uint32_t magic;
	uint32_t len;
	odp_pool_t pool;
	uint8_t *data;
	odpg_meta_t meta;          /* parse result: packet_parser_t + cls_mark */
	odp_cos_t cos;
	odp_pktio_t input;         /* the pktio it was received on */
	uint32_t cap;
	uint32_t ext;              /* data malloc'd on its own (longer than the pool's buffers) */
	uint32_t pgen;             /* its pool's generation (rt_pool_t.gen) */
	struct rt_pkt *next;       /* queue link */
} rt_pkt_t;
_Static_assert(__builtin_offsetof(rt_pkt_t, cap) == 64, "rt_pkt_t receive line");
#define PK(p) ((rt_pkt_t *)(p))

#define TC_N     512       /* largest per-thread cache of one pool */

typedef struct rt_pool {
	int valid;
	char name[ODP_POOL_NAME_LEN];
	odp_pool_param_t param;
	uint32_t in_use;           /* buffers out of the pool (made - free, caches count as out) */
	pthread_mutex_t lock;
	/* packet buffers (pool.c's buffer stack + per-thread caches): made in
	 * chunks on demand up to param.pkt.num, a header and `buf` data bytes
	 * each, never returned to the system before odp_pool_destroy */
	uint32_t gen;              /* create count of this slot: thread caches check it */
	uint32_t tc_max;           /* buffers a thread's cache may hold (0: no caching) */
	uint32_t buf;              /* data bytes of a pooled buffer */
	uint32_t made;             /* buffers made (pooled) or allocated (ext) */
	rt_pkt_t **stack;          /* free pooled buffers */
	uint32_t nfree;
	void **chunks;
	uint32_t nchunks;
} rt_pool_t;

/* the runtime's short critical sections (pool stacks, queue rings, the loop
 * ring): an adaptive mutex spins a while before it sleeps, so workers
 * meeting on one of them do not pay a futex round trip each */
static void rt_mutex_init(pthread_mutex_t *m)
{
	pthread_mutexattr_t a;

	pthread_mutexattr_init(&a);
	pthread_mutexattr_settype(&a, PTHREAD_MUTEX_ADAPTIVE_NP);
	pthread_mutex_init(m, &a);
	pthread_mutexattr_destroy(&a);
}

/* a FIFO of handles: v[rd..rd+n) modulo cap (a power of two), grown by
 * doubling; its owner's lock held. n is also read without the lock (an empty
 * ring is seen without taking it), so it is stored atomically. */
typedef struct ptr_ring {
	void **v;
	uint32_t cap, rd, n;
} ptr_ring_t;

/* num handles at the tail, all or none (-1: no memory) */
static int pring_push(ptr_ring_t *r, void *const h[], uint32_t num)
{
	const uint32_t n = r->n;

	if (n + num > r->cap) {
		uint32_t cap = r->cap ? r->cap : 256u;

		while (cap < n + num)
			cap *= 2u;
		void **x = malloc((size_t)cap * sizeof(*x));

		if (!x)
			return -1;
		for (uint32_t i = 0; i < n; i++)
			x[i] = r->v[(r->rd + i) & (r->cap - 1u)];
		free(r->v);
		r->v = x;
		r->cap = cap;
		r->rd = 0;
	}
	const uint32_t w = (r->rd + n) & (r->cap - 1u);
	const uint32_t k = num < r->cap - w ? num : r->cap - w;

	memcpy(r->v + w, h, (size_t)k * sizeof(*h));
	memcpy(r->v, h + k, (size_t)(num - k) * sizeof(*h));
	__atomic_store_n(&r->n, n + num, __ATOMIC_RELEASE);
	return 0;
}

/* up to num handles from the head; returns how many */
static uint32_t pring_pop(ptr_ring_t *r, void *h[], uint32_t num)
{
	const uint32_t n = r->n < num ? r->n : num;
	const uint32_t k = n < r->cap - r->rd ? n : r->cap - r->rd;

	memcpy(h, r->v + r->rd, (size_t)k * sizeof(*h));
	memcpy(h + k, r->v, (size_t)(n - k) * sizeof(*h));
	if (n) {
		r->rd = (r->rd + n) & (r->cap - 1u);
		__atomic_store_n(&r->n, r->n - n, __ATOMIC_RELAXED);
	}
	return n;
}

/* every handle freed as a packet, the ring emptied and its memory given back */
static void pring_free_packets(ptr_ring_t *r)
{
	for (uint32_t i = 0; i < r->n; i++)
		odp_packet_free((odp_packet_t)r->v[(r->rd + i) & (r->cap - 1u)]);
	free(r->v);
	memset(r, 0, sizeof(*r));
}

typedef struct rt_queue {
	uint32_t magic;
	odp_queue_t hdl;           /* registry handle */
	char name[ODP_QUEUE_NAME_LEN];
	odp_queue_param_t param;
	pthread_mutex_t lock;
	ptr_ring_t ev;             /* the events (kept when the slot is reused) */
	int sched;                 /* ODP_QUEUE_TYPE_SCHED: counted in rt.sched_n */
	struct rt_queue *next_sched;
	int dead;
	uint32_t gen;              /* registry slot generation (in the handle) */
	odp_pktio_t pktin;         /* a QUEUE-mode pktin queue: dequeue polls it */
	odp_pktio_t pktout;        /* a pktout event queue: enqueue transmits */
	uint32_t pindex;           /* its pktin / pktout queue index */
} rt_queue_t;
#define QUEUE_MAGIC 0x51554555u

/* a receive burst's buffers (odp_rt.c "receive pipeline") */
typedef struct rx_slot {
	uint32_t n;                /* frames in the burst */
	rt_pkt_t *src[RT_BURST];   /* loop device: the transmitted packets */
	uint8_t qi[RT_BURST];      /* the input queue each came in on */
	uint8_t *stage, *dstage;   /* frames (pinned host, and its device address) */
	size_t stage_cap;
	odpg_desc_t *desc, *ddesc;
	odpg_out_t *out, *dout;
	odpg_meta_t *meta, *dmeta;
	odpg_fence_t *fence;       /* behind the burst's launch */
	odpg_ctx_t *ctx;           /* the device context its bursts launch on */
	void *token;               /* the launch's binding (odpg_cls_pktio_recv_end) */
	/* delivery in chunks (receive pipeline): the burst's launch count
	 * (seq) and next unclaimed chunk packed in one word, so that a thread
	 * holding an old count cannot claim from a reused slot; chunks hand
	 * their packets to the queues in order (commit); busy counts the
	 * threads inside, which a launch into the slot waits out */
	uint32_t open;             /* 1 while its chunks are being delivered */
	uint32_t nchunks;
	uint64_t claimw;           /* seq << 32 | next chunk */
	uint32_t commit;           /* chunks handed over */
	uint32_t busy;
} rx_slot_t;

typedef struct rt_pktio {
	int valid;
	int in_mode;               /* odp_pktin_mode_t */
	int out_mode;              /* odp_pktout_mode_t */
	int loopdev;               /* "loop...": transmitted packets come back */
	odp_pool_t pool;           /* the pktio's packet pool */
	odpg_capture_t cap;
	int have_cap;
	uint32_t pos;              /* next frame of the capture */
	uint32_t loops, loop_cnt;  /* pcap.c's loops / loop_cnt (starts at 1) */
	int promisc;
	uint32_t mtu;
	uint32_t num_in, num_out;  /* configured input / output queues */
	uint32_t hash_bits;        /* odp_pktin_hash_proto_t of the input queues
				    * (hash_enable), 0: no hashing */
	rt_queue_t *inq[RT_MAXQ];  /* pktin event queues (QUEUE / SCHED mode) */
	rt_queue_t *outq[RT_MAXQ]; /* pktout event queues (QUEUE mode) */
	pthread_mutex_t ring_lock; /* the loop device's packets in flight */
	/* the transmitted packets per input queue, in order (loop.c's loopqs[],
	 * one queue per input queue: get_dest_queue picks it); ring_n: all
	 * of them (read unlocked) */
	ptr_ring_t ring[RT_MAXQ];
	uint32_t ring_n;
	uint32_t rr;               /* event modes: the ring a burst starts at */
	/* DIRECT mode, per input queue: received (classified) packets beyond
	 * what the last odp_pktin_recv asked for */
	rt_pkt_t *ahead[RT_MAXQ], *ahead_tail[RT_MAXQ];
	/* per-queue counters of a device with more than one input / output
	 * queue (loop.c loopqs[].stats); one queue reports the interface's */
	struct {
		uint64_t in_octets, in_packets, in_discards, in_errors;
		uint64_t out_octets, out_packets;
	} qst[RT_MAXQ];
	struct rx_slot *slot[RT_INFLIGHT];  /* receive bursts ("receive pipeline") */
	/* bursts launched / delivered (wrapping counts): the ones in flight
	 * sit in slots delivered .. launched - 1 (mod RT_INFLIGHT). launched
	 * moves under rt.poll_lock, delivered under rx_dlock[] (receive
	 * pipeline: one thread launches while another delivers) */
	uint32_t launched, delivered;
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
	uint32_t sched_n;          /* events in them (read without a lock) */
	int polling;               /* a thread is in poll_input */
	/* the device contexts receive bursts launch on (ODPG_DEVICES; ctx is
	 * the first; slot_get) */
	odpg_ctx_t *ctxs[RT_MAX_DEV];
	uint32_t nctx;
} rt = { PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, 0, NULL, {{0}}, {{0}},
	 NULL, 0, 0, {NULL}, 0 };

/* a pktio's delivery side (receive pipeline), outside the pktio object so
 * that close can hold it across the object's reset; lock order: poll_lock,
 * then rx_dlock */
static pthread_mutex_t rx_dlock[RT_MAX_PKTIO] = { [0 ... RT_MAX_PKTIO - 1] =
							   PTHREAD_MUTEX_INITIALIZER };
static int rx_dbusy[RT_MAX_PKTIO];
static uint32_t rx_helpers[RT_MAX_PKTIO];   /* threads in a pktio's delivery side */

/* a spin-wait's step: a pause, and after 2^15 of them (~0.5 ms) a yield of
 * the CPU at every step (the thread waited for may have been preempted:
 * more workers than CPUs, or two pinned to one). The waits of a running
 * pipeline end well before that: with a yield from the 1024th pause on, the
 * record's odp_pktio_perf -c 8 ran at 48 Mpps against 64 in the session
 * before (other boxes; not an A/B) */
static inline void spin_wait(uint32_t *steps)
{
	if (*steps < (1u << 15)) {
		++*steps;
		__builtin_ia32_pause();
	} else {
		sched_yield();
	}
}

/* pinned host memory and its device address (zero-copy launch buffers) */
static int pinned_alloc(size_t bytes, void **host, void **dev)
{
	if (odpg_host_alloc_pinned(bytes, host))
		return -1;
	if (odpg_host_device_ptr(*host, dev)) {
		odpg_host_free_pinned(*host);
		*host = NULL;
		return -1;
	}
	return 0;
}


/* ---- init / threads ------------------------------------------------------- */
/* thread ids: the lowest free id, given back at odp_term_local (odp_thread.c
 * alloc_id / free_id), so ids stay below ODP_THREAD_COUNT_MAX however many
 * threads come and go (odp_pktio_perf indexes its stats by them) */
static pthread_mutex_t thr_lock = PTHREAD_MUTEX_INITIALIZER;
static uint64_t thr_used[ODP_THREAD_COUNT_MAX / 64];
static int thr_count;
static __thread int thr_id = -1;
static __thread odp_thread_type_t thr_type = ODP_THREAD_WORKER;

void odp_init_param_init(odp_init_t *param)
{
	memset(param, 0, sizeof(*param));
	param->mem_model = ODP_MEM_MODEL_THREAD;
}

/* ODP_RT_PROF=1: receive-burst counts and times, printed by odp_term_global */
static struct {
	int on;
	uint64_t bursts, pkts, stage_ns, gpu_ns, post_ns;
	uint64_t end_ns, enq_ns;   /* of post_ns: the binding's release, the queue appends */
} rxprof = { -1, 0, 0, 0, 0, 0, 0, 0 };

static uint64_t prof_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int odp_init_global(odp_instance_t *instance, const odp_init_t *param, const void *platform)
{
	(void)param;
	(void)platform;
	if (rxprof.on < 0)
		rxprof.on = getenv("ODP_RT_PROF") && atoi(getenv("ODP_RT_PROF"));
	pthread_mutex_lock(&rt.lock);
	if (!rt.init) {
		/* ODPG_DEVICES="0,1,..." (default "0"): one context per entry
		 * (a device may repeat: its contexts share the GPU); receive
		 * bursts spread over them (odpg_group.h is the same sharding for
		 * a single batch) */
		const char *dl = getenv("ODPG_DEVICES");
		char buf[256];
		int rc = 0;

		snprintf(buf, sizeof(buf), "%s", dl && *dl ? dl : "0");
		rt.nctx = 0;
		for (char *save = NULL, *tok = strtok_r(buf, ", ", &save);
		     tok && rt.nctx < RT_MAX_DEV && !rc; tok = strtok_r(NULL, ", ", &save)) {
			rc = odpg_ctx_create((int)strtol(tok, NULL, 0), NULL, &rt.ctxs[rt.nctx]);
			if (!rc)
				rt.nctx++;
		}
		if (rc || !rt.nctx) {
			for (uint32_t k = 0; k < rt.nctx; k++)
				odpg_ctx_destroy(rt.ctxs[k]);
			rt.nctx = 0;
			pthread_mutex_unlock(&rt.lock);
			ERR("no MI355X context (odpg_ctx_create: %d, ODPG_DEVICES=%s): the "
			    "classifier runs only on the GPU\n", rc, dl ? dl : "0");
			return -1;
		}
		rt.ctx = rt.ctxs[0];
		rt.init = 1;
	}
	pthread_mutex_unlock(&rt.lock);
	if (instance)
		*instance = (odp_instance_t)(uintptr_t)&rt;
	return 0;
}

static void parse_release(void);

static void rx_release(rt_pktio_t *p);

static void grave_release(void);

int odp_term_global(odp_instance_t instance)
{
	(void)instance;
	parse_release();
	if (rxprof.on > 0 && rxprof.bursts)
		fprintf(stderr, "odp_rt: %llu receive bursts, %.1f packets each; per burst: "
			"staging %.2f us, launch (+ GPU wait in DIRECT mode) %.2f us, delivery %.2f us "
			"(binding release %.2f us, queue appends %.2f us)\n",
			(unsigned long long)rxprof.bursts, (double)rxprof.pkts / rxprof.bursts,
			rxprof.stage_ns / 1e3 / rxprof.bursts, rxprof.gpu_ns / 1e3 / rxprof.bursts,
			rxprof.post_ns / 1e3 / rxprof.bursts, rxprof.end_ns / 1e3 / rxprof.bursts,
			rxprof.enq_ns / 1e3 / rxprof.bursts);
	pthread_mutex_lock(&rt.poll_lock);
	for (int i = 0; i < RT_MAX_PKTIO; i++) {
		pthread_mutex_lock(&rx_dlock[i]);
		rx_release(&rt.pktio[i]);
		pthread_mutex_unlock(&rx_dlock[i]);
	}
	pthread_mutex_unlock(&rt.poll_lock);
	pthread_mutex_lock(&rt.lock);
	if (rt.init) {
		for (uint32_t k = 0; k < rt.nctx; k++)
			odpg_ctx_destroy(rt.ctxs[k]);
		rt.nctx = 0;
		rt.ctx = NULL;
		rt.init = 0;
	}
	pthread_mutex_unlock(&rt.lock);
	grave_release();
	return 0;
}

int odp_init_local(odp_instance_t instance, odp_thread_type_t type)
{
	(void)instance;
	if (thr_id >= 0)
		return 0;
	pthread_mutex_lock(&thr_lock);
	for (int i = 0; i < ODP_THREAD_COUNT_MAX; i++) {
		if (thr_used[i / 64] & (1ull << (i % 64)))
			continue;
		thr_used[i / 64] |= 1ull << (i % 64);
		/* read unlocked by odp_thread_count */
		__atomic_fetch_add(&thr_count, 1, __ATOMIC_RELAXED);
		thr_id = i;
		break;
	}
	pthread_mutex_unlock(&thr_lock);
	if (thr_id < 0) {
		ERR("all %d thread ids in use\n", ODP_THREAD_COUNT_MAX);
		return -1;
	}
	thr_type = type;
	return 0;
}

static void tcache_flush(void);

int odp_term_local(void)
{
	tcache_flush();
	if (thr_id < 0)
		return 0;
	pthread_mutex_lock(&thr_lock);
	thr_used[thr_id / 64] &= ~(1ull << (thr_id % 64));
	__atomic_fetch_sub(&thr_count, 1, __ATOMIC_RELAXED);
	pthread_mutex_unlock(&thr_lock);
	thr_id = -1;
	return 0;
}

int odp_thread_id(void)
{
	return thr_id < 0 ? 0 : thr_id;
}

int odp_thread_count(void)
{
	return __atomic_load_n(&thr_count, __ATOMIC_RELAXED);
}

int odp_thread_count_max(void)
{
	return ODP_THREAD_COUNT_MAX;
}

odp_thread_type_t odp_thread_type(void)
{
	return thr_type;
}

int odp_cpu_id(void)
{
	const int c = sched_getcpu();

	return c < 0 ? 0 : c;
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

/* ---- barrier: two-phase arrival count, spin then yield -------------------- */
void odp_barrier_init(odp_barrier_t *barr, int count)
{
	barr->count = (uint32_t)count;
	odp_atomic_init_u32(&barr->bar, 0);
}

/* arrivals count 0 .. 2 * count - 1: the first count arrivals meet in phase
 * 0, the next count in phase 1, so a fast thread re-entering the barrier
 * cannot overtake a slow one still leaving it */
void odp_barrier_wait(odp_barrier_t *barr)
{
	const uint32_t count = barr->count;
	const uint32_t n = __atomic_fetch_add(&barr->bar.v, 1, __ATOMIC_ACQ_REL);
	const int phase = n >= count;
	uint32_t spins = 0;

	if (n + 1 == count)
		return;                    /* the last of phase 0 releases it */
	if (n + 1 == 2 * count) {
		/* the last of phase 1 releases it by wrapping to 0 */
		__atomic_store_n(&barr->bar.v, 0, __ATOMIC_RELEASE);
		return;
	}
	for (;;) {
		const uint32_t v = __atomic_load_n(&barr->bar.v, __ATOMIC_ACQUIRE);

		/* phase 0 is released once every thread arrived (v >= count);
		 * phase 1 once the count wrapped to zero */
		if (phase == 0 ? v >= count : v < count)
			return;
		if (++spins > 1000)
			sched_yield();
	}
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

/* the first CPU of a sysfs CPU list file (the L3's or the core's sharers);
 * -1 when absent */
static int cpu_list_first(int cpu, const char *what)
{
	char path[128];
	int first = -1;

	snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/%s", cpu, what);
	FILE *f = fopen(path, "r");

	if (f) {
		if (fscanf(f, "%d", &first) != 1)
			first = -1;
		fclose(f);
	}
	return first;
}

/* num workers (num > 0) inside one L3 cache: the packets, queues and locks
 * the workers share then move between cores of one CCD instead of across
 * the IO die (on a 2 x 64-core EPYC host, 8 workers on CPUs 1-8 span two
 * CCDs and odp_pktio_perf -c 8 fell to a third of -c 6's rate). One core's
 * first hardware thread each; the control CPU's own L3 first, else the
 * first L3 with num free cores; else the same with second hardware threads
 * added. Returns 0 when no L3 holds them (or the topology is not in sysfs):
 * the caller takes CPUs in order. */
static int l3_mask(const cpu_set_t *set, int control, int num, odp_cpumask_t *mask)
{
	enum { NC = CPU_SETSIZE < ODP_CPUMASK_SIZE ? CPU_SETSIZE : ODP_CPUMASK_SIZE };
	/* per CPU of the set, read once: its L3 (the first CPU of the L3's
	 * sharers, which need not be in the set: a cpuset slice may start
	 * inside an L3) and whether it is its core's first hardware thread */
	int l3of[NC], first[NC], ids[NC], nid = 0;

	for (int c = 0; c < NC; c++) {
		l3of[c] = -1;
		if (!CPU_ISSET(c, set))
			continue;
		l3of[c] = cpu_list_first(c, "cache/index3/shared_cpu_list");
		if (l3of[c] < 0)
			return 0;
		first[c] = cpu_list_first(c, "topology/thread_siblings_list") == c;
		int k = 0;

		while (k < nid && ids[k] != l3of[c])
			k++;
		if (k == nid)
			ids[nid++] = l3of[c];
	}
	if (control < 0 || control >= NC || l3of[control] < 0)
		return 0;
	const int ctl_l3 = l3of[control];

	/* passes: the control's L3, then the others, first hardware threads
	 * only; then the same with the second hardware threads of its cores
	 * after the first ones (sharing a core beats crossing the IO die) */
	for (int pass = 0; pass < 4; pass++) {
		const int smt = pass >= 2;

		for (int k = 0; k < nid; k++) {
			const int l3 = ids[k];

			if (((pass & 1) == 0) != (l3 == ctl_l3))
				continue;
			int n = 0;

			odp_cpumask_zero(mask);
			for (int sib = 0; sib <= smt; sib++)
				for (int c = 0; c < NC && n < num; c++)
					if (c != control && l3of[c] == l3 && first[c] == !sib) {
						odp_cpumask_set(mask, c);
						n++;
					}
			if (n == num)
				return n;
		}
	}
	odp_cpumask_zero(mask);
	return 0;
}

/* workers on the CPUs of the affinity mask after the first (the control
 * thread's), as many as asked (0 = all): a given number inside one L3 where
 * one holds them (l3_mask) */
static int default_mask(odp_cpumask_t *mask, int num, int worker)
{
	cpu_set_t set;
	int n = 0, first = -1;

	odp_cpumask_zero(mask);
	if (sched_getaffinity(0, sizeof(set), &set))
		return 0;
	if (worker && num > 0 && CPU_COUNT(&set) > num) {
		int control = 0;

		while (!CPU_ISSET(control, &set))
			control++;
		const int n = l3_mask(&set, control, num, mask);

		if (n)
			return n;
	}
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

/* ---- shared memory: named blocks ------------------------------------------ */
#define SHM_MAGIC 0x53484d42u

typedef struct rt_shm {
	uint32_t magic;
	char name[64];
	void *addr;
	struct rt_shm *next;
} rt_shm_t;

static pthread_mutex_t shm_lock = PTHREAD_MUTEX_INITIALIZER;
static rt_shm_t *shm_list;     /* newest first */

odp_shm_t odp_shm_reserve(const char *name, uint64_t size, uint64_t align, uint32_t flags)
{
	rt_shm_t *s = calloc(1, sizeof(*s));
	void *p = NULL;

	(void)flags;
	if (!s)
		return ODP_SHM_INVALID;
	if (align < sizeof(void *))
		align = sizeof(void *);
	if (posix_memalign(&p, align, size ? size : 1)) {
		free(s);
		return ODP_SHM_INVALID;
	}
	memset(p, 0, size);
	s->magic = SHM_MAGIC;
	snprintf(s->name, sizeof(s->name), "%s", name ? name : "");
	s->addr = p;
	pthread_mutex_lock(&shm_lock);
	s->next = shm_list;
	shm_list = s;
	pthread_mutex_unlock(&shm_lock);
	return (odp_shm_t)s;
}

odp_shm_t odp_shm_lookup(const char *name)
{
	rt_shm_t *s;

	if (!name)
		return ODP_SHM_INVALID;
	pthread_mutex_lock(&shm_lock);
	for (s = shm_list; s; s = s->next)
		if (!strcmp(s->name, name))
			break;
	pthread_mutex_unlock(&shm_lock);
	return (odp_shm_t)s;
}

void *odp_shm_addr(odp_shm_t shm)
{
	rt_shm_t *s = (rt_shm_t *)shm;

	return s && s->magic == SHM_MAGIC ? s->addr : NULL;
}

int odp_shm_free(odp_shm_t shm)
{
	rt_shm_t *s = (rt_shm_t *)shm, **pp;

	if (!s)
		return -1;
	pthread_mutex_lock(&shm_lock);
	for (pp = &shm_list; *pp && *pp != s; pp = &(*pp)->next)
		;
	/* not a live block (freed before, or never reserved): nothing of it
	 * is read */
	if (!*pp || s->magic != SHM_MAGIC) {
		pthread_mutex_unlock(&shm_lock);
		return -1;
	}
	*pp = s->next;
	s->magic = 0;
	pthread_mutex_unlock(&shm_lock);
	free(s->addr);
	free(s);
	return 0;
}

uint64_t odp_shm_to_u64(odp_shm_t shm)
{
	return (uint64_t)(uintptr_t)shm;
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
	capa->pkt.min_cache_size = 0;
	capa->pkt.max_cache_size = TC_N;
	return 0;
}

void odp_pool_param_init(odp_pool_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->type = ODP_POOL_PACKET;
	param->pkt.seg_len = 1856;
	param->pkt.len = 1856;
	param->pkt.num = 1024;
	param->pkt.cache_size = 256;        /* the reference's default local cache */
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
		const uint32_t gen = p->gen;

		memset(p, 0, sizeof(*p));
		p->gen = gen + 1u;
		snprintf(p->name, sizeof(p->name), "%s", name ? name : "");
		p->param = *param;
		/* a pooled buffer holds the pool's packet length (seg_len at
		 * least); longer packets get their own allocation */
		p->buf = param->pkt.len > param->pkt.seg_len ? param->pkt.len : param->pkt.seg_len;
		if (p->buf < 64u)
			p->buf = 64u;
		/* per-thread caches hold the pool's cache_size (0: no
		 * caching), at most 1/32 of the pool each, so that buffers
		 * freed by other threads cannot strand a small pool's
		 * allocations (pools of < 64 buffers: no caching) */
		p->tc_max = param->pkt.num / 32u < TC_N ? param->pkt.num / 32u : TC_N;
		if (param->pkt.cache_size < p->tc_max)
			p->tc_max = param->pkt.cache_size;
		if (p->tc_max < 2u)
			p->tc_max = 0u;
		p->stack = malloc((size_t)param->pkt.num * sizeof(rt_pkt_t *));
		if (!p->stack)
			break;
		rt_mutex_init(&p->lock);
		p->valid = 1;
		ret = (odp_pool_t)(uintptr_t)(i + 1);
		break;
	}
	pthread_mutex_unlock(&rt.lock);
	return ret;
}

/* Chunks of pools destroyed while buffers were still out (held by the
 * application or another thread's cache): a later odp_packet_free of such a
 * buffer reads its header to find the pool gone (generation check), so the
 * memory stays mapped until odp_term_global (the reference frees it and
 * leaves that free undefined; found by the AddressSanitizer build,
 * tests/c/Makefile "san") */
static struct {
	pthread_mutex_t lock;
	void **chunks;
	uint32_t n, cap;
} grave = {PTHREAD_MUTEX_INITIALIZER, NULL, 0, 0};

static void grave_release(void)
{
	pthread_mutex_lock(&grave.lock);
	for (uint32_t c = 0; c < grave.n; c++)
		free(grave.chunks[c]);
	free(grave.chunks);
	grave.chunks = NULL;
	grave.n = grave.cap = 0;
	pthread_mutex_unlock(&grave.lock);
}

/* a destroyed pool's chunks: freed now when every buffer is back on its
 * stack, else kept until odp_term_global */
static void pool_chunks_release(rt_pool_t *p)
{
	const int out = p->nfree != p->made;

	pthread_mutex_lock(&grave.lock);
	for (uint32_t c = 0; c < p->nchunks; c++) {
		if (out && grave.n == grave.cap) {
			const uint32_t cap = grave.cap ? 2u * grave.cap : 64u;
			void **nc = realloc(grave.chunks, cap * sizeof(void *));

			if (nc) {
				grave.chunks = nc;
				grave.cap = cap;
			}
		}
		if (out && grave.n < grave.cap)
			grave.chunks[grave.n++] = p->chunks[c];
		else
			free(p->chunks[c]);
	}
	pthread_mutex_unlock(&grave.lock);
}

int odp_pool_destroy(odp_pool_t hdl)
{
	pthread_mutex_lock(&rt.lock);
	rt_pool_t *p = get_pool(hdl);
	int rc = p ? 0 : -1;

	if (p) {
		/* under the pool's lock: a free or alloc that looked the pool up
		 * before this re-checks valid there (pool.c destroys under
		 * pool->lock too) */
		pthread_mutex_lock(&p->lock);
		p->valid = 0;
		pool_chunks_release(p);
		free(p->chunks);
		free(p->stack);
		p->chunks = NULL;
		p->stack = NULL;
		p->nchunks = p->nfree = p->made = 0;
		pthread_mutex_unlock(&p->lock);
	}
	pthread_mutex_unlock(&rt.lock);
	return rc;
}

/* odp_pool_lookup (odp_pool.c): a pool by the name it was created with */
odp_pool_t odp_pool_lookup(const char *name)
{
	odp_pool_t ret = ODP_POOL_INVALID;

	if (!name)
		return ret;
	pthread_mutex_lock(&rt.lock);
	for (int i = 0; i < RT_MAX_POOL; i++)
		if (rt.pool[i].valid && !strcmp(rt.pool[i].name, name)) {
			ret = (odp_pool_t)(uintptr_t)(i + 1);
			break;
		}
	pthread_mutex_unlock(&rt.lock);
	return ret;
}

uint64_t odp_pool_to_u64(odp_pool_t pool)
{
	return (uint64_t)(uintptr_t)pool;
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

#define PKT_HDR ((sizeof(rt_pkt_t) + 63u) & ~(size_t)63u)   /* data offset in a pooled buffer */

/* per-thread buffer caches (pool.c's local cache): a few pools per thread */
#define TC_POOLS 8
static __thread struct {
	uint32_t pool, gen, n;
	rt_pkt_t *b[TC_N];
} tcache[TC_POOLS];

/* a chunk of pooled buffers onto the pool's stack (pool lock held) */
static int pool_grow_locked(rt_pool_t *p)
{
	const uint32_t num = p->param.pkt.num;
	uint32_t n = num - p->made < 256u ? num - p->made : 256u;
	const size_t one = PKT_HDR + ((p->buf + 63u) & ~63u);

	if (!n)
		return -1;
	uint8_t *c = NULL;
	void **nc = realloc(p->chunks, (p->nchunks + 1u) * sizeof(void *));

	if (!nc)
		return -1;
	p->chunks = nc;
	if (posix_memalign((void **)&c, 64, one * n))
		return -1;
	p->chunks[p->nchunks++] = c;
	for (uint32_t i = 0; i < n; i++) {
		rt_pkt_t *k = (rt_pkt_t *)(c + one * i);

		memset(k, 0, sizeof(*k));
		k->data = (uint8_t *)k + PKT_HDR;
		k->cap = p->buf;
		p->stack[p->nfree++] = k;
	}
	p->made += n;
	return 0;
}

static int tc_slot(odp_pool_t pool, const rt_pool_t *p)
{
	const uint32_t id = (uint32_t)(uintptr_t)pool;
	int freeslot = -1;

	if (!p->tc_max)
		return -1;
	for (int i = 0; i < TC_POOLS; i++) {
		if (tcache[i].pool == id) {
			if (tcache[i].gen == p->gen)
				return i;
			tcache[i].n = 0;           /* a destroyed pool's buffers */
			tcache[i].gen = p->gen;
			return i;
		}
		if (!tcache[i].pool && freeslot < 0)
			freeslot = i;
	}
	if (freeslot >= 0) {
		tcache[freeslot].pool = id;
		tcache[freeslot].gen = p->gen;
		tcache[freeslot].n = 0;
	}
	return freeslot;
}

static void pkt_init(rt_pkt_t *k, odp_pool_t pool, uint32_t len)
{
	k->magic = PKT_MAGIC;
	k->pgen = get_pool(pool)->gen;
	k->pool = pool;
	k->len = len;
	k->cos = ODP_COS_INVALID;
	k->input = ODP_PKTIO_INVALID;
	memset(&k->meta, 0, sizeof(k->meta));
	k->meta.l2_offset = k->meta.l3_offset = k->meta.l4_offset = 0xffff;
	k->next = NULL;
}

odp_packet_t odp_packet_alloc(odp_pool_t pool, uint32_t len)
{
	rt_pool_t *p = get_pool(pool);
	rt_pkt_t *k = NULL;

	if (!p)
		return ODP_PACKET_INVALID;
	const int ts = tc_slot(pool, p);

	if (ts >= 0 && tcache[ts].n) {
		k = tcache[ts].b[--tcache[ts].n];
	} else {
		pthread_mutex_lock(&p->lock);
		if (!p->valid) {                  /* destroyed meanwhile */
			pthread_mutex_unlock(&p->lock);
			return ODP_PACKET_INVALID;
		}
		if (!p->nfree)
			pool_grow_locked(p);
		if (p->nfree) {
			k = p->stack[--p->nfree];
			/* refill the thread's cache with up to half of it */
			while (ts >= 0 && p->nfree && tcache[ts].n < p->tc_max / 2)
				tcache[ts].b[tcache[ts].n++] = p->stack[--p->nfree];
		}
		p->in_use = p->made - p->nfree;
		pthread_mutex_unlock(&p->lock);
		if (!k)
			return ODP_PACKET_INVALID;
	}
	if (len > p->buf) {
		/* longer than the pool's buffers: one of the pool's buffers with
		 * data of its own */
		uint8_t *d = malloc(len);

		if (!d) {
			k->pgen = p->gen;
			odp_packet_free((odp_packet_t)k);
			return ODP_PACKET_INVALID;
		}
		k->data = d;
		k->cap = len;
		k->ext = 1;
	}
	pkt_init(k, pool, len);
	return (odp_packet_t)k;
}

void odp_packet_free(odp_packet_t pkt)
{
	rt_pkt_t *k = (rt_pkt_t *)pkt;
	rt_pool_t *p;

	if (!k)
		return;
	k->magic = 0;
	if (k->ext) {
		free(k->data);
		k->data = (uint8_t *)k + PKT_HDR;
		k->ext = 0;
	}
	p = get_pool(k->pool);
	if (!p || p->gen != k->pgen)    /* its pool was destroyed: the memory went with it */
		return;
	k->cap = p->buf;
	const int ts = tc_slot(k->pool, p);

	if (ts >= 0 && tcache[ts].n < p->tc_max) {
		tcache[ts].b[tcache[ts].n++] = k;
		return;
	}
	pthread_mutex_lock(&p->lock);
	if (!p->valid || p->gen != k->pgen) {   /* destroyed meanwhile */
		pthread_mutex_unlock(&p->lock);
		return;
	}
	p->stack[p->nfree++] = k;
	/* and half of the thread's cache back */
	while (ts >= 0 && tcache[ts].n > p->tc_max / 2)
		p->stack[p->nfree++] = tcache[ts].b[--tcache[ts].n];
	p->in_use = p->made - p->nfree;
	pthread_mutex_unlock(&p->lock);
}

/* a thread's cached buffers back to their pools (odp_term_local) */
static void tcache_flush(void)
{
	for (int i = 0; i < TC_POOLS; i++) {
		rt_pool_t *p = tcache[i].pool ? get_pool((odp_pool_t)(uintptr_t)tcache[i].pool) : NULL;

		if (p && p->gen == tcache[i].gen && tcache[i].n) {
			pthread_mutex_lock(&p->lock);
			while (p->valid && p->gen == tcache[i].gen && tcache[i].n)
				p->stack[p->nfree++] = tcache[i].b[--tcache[i].n];
			p->in_use = p->made - p->nfree;
			pthread_mutex_unlock(&p->lock);
		}
		tcache[i].n = 0;
		tcache[i].pool = 0;
	}
}

/* runs of one pool's packets in one pass: the thread's cache filled, the
 * rest onto the pool's stack under one lock (with the cache trimmed to half,
 * as odp_packet_free does) */
void odp_packet_free_multi(const odp_packet_t pkt[], int num)
{
	for (int i = 0; i < num;) {
		rt_pkt_t *k0 = PK(pkt[i]);

		if (!k0) {
			i++;
			continue;
		}
		const odp_pool_t pool = k0->pool;
		const uint32_t pgen = k0->pgen;
		rt_pool_t *p = get_pool(pool);
		int j = i;

		while (j < num && pkt[j] && PK(pkt[j])->pool == pool && PK(pkt[j])->pgen == pgen)
			j++;
		if (!p || p->gen != pgen) {      /* its pool was destroyed */
			for (; i < j; i++)
				odp_packet_free(pkt[i]);
			continue;
		}
		const int ts = tc_slot(pool, p);
		int over = j;                    /* the first not cached */

		for (int m = i; m < j; m++) {
			rt_pkt_t *k = PK(pkt[m]);

			k->magic = 0;
			if (k->ext) {
				free(k->data);
				k->data = (uint8_t *)k + PKT_HDR;
				k->ext = 0;
			}
			k->cap = p->buf;
			if (over == j && ts >= 0 && tcache[ts].n < p->tc_max)
				tcache[ts].b[tcache[ts].n++] = k;
			else if (over == j)
				over = m;
		}
		if (over < j) {
			pthread_mutex_lock(&p->lock);
			if (p->valid && p->gen == pgen) {
				for (int m = over; m < j; m++)
					p->stack[p->nfree++] = PK(pkt[m]);
				while (ts >= 0 && tcache[ts].n > p->tc_max / 2)
					p->stack[p->nfree++] = tcache[ts].b[--tcache[ts].n];
				p->in_use = p->made - p->nfree;
			}
			pthread_mutex_unlock(&p->lock);
		}
		i = j;
	}
}

/* up to n of a pool's buffers for packets of at most its buffer length (the
 * caller initialises them: pkt_init): the thread's cache first, then the
 * stack under one lock, the cache refilled to half. Returns how many. */
static uint32_t pool_take(odp_pool_t pool, rt_pkt_t *out[], uint32_t n)
{
	rt_pool_t *p = get_pool(pool);
	uint32_t got = 0;

	if (!p)
		return 0;
	const int ts = tc_slot(pool, p);

	while (ts >= 0 && got < n && tcache[ts].n)
		out[got++] = tcache[ts].b[--tcache[ts].n];
	if (got == n)
		return got;
	pthread_mutex_lock(&p->lock);
	if (p->valid) {
		while (got < n && (p->nfree || !pool_grow_locked(p)))
			out[got++] = p->stack[--p->nfree];
		while (ts >= 0 && p->nfree && tcache[ts].n < p->tc_max / 2)
			tcache[ts].b[tcache[ts].n++] = p->stack[--p->nfree];
		p->in_use = p->made - p->nfree;
	}
	pthread_mutex_unlock(&p->lock);
	return got;
}

/* ---- packet accessors ------------------------------------------------------ */

/* _odp_packet_input_flags_t bits (packet_inline_types.h:60-113) */
enum {
	IF_DST_QUEUE = 0, IF_CLS_MARK, IF_FLOW_HASH, IF_TIMESTAMP, IF_L2, IF_L3, IF_L4,
	IF_ETH, IF_ETH_BCAST, IF_ETH_MCAST, IF_JUMBO, IF_VLAN, IF_VLAN_QINQ, IF_SNAP, IF_ARP,
	IF_IPV4, IF_IPV6, IF_IP_BCAST, IF_IP_MCAST, IF_IPFRAG, IF_IPOPT, IF_IPSEC,
	IF_IPSEC_AH, IF_IPSEC_ESP, IF_UDP, IF_TCP, IF_SCTP, IF_ICMP, IF_NO_NEXT_HDR,
	IF_L3_CHKSUM_DONE = 32, IF_L4_CHKSUM_DONE
};
/* _odp_packet_flags_t error bits (packet_inline_types.h:150-164) */
enum {
	F_SNAP_LEN_ERR = 25, F_IP_ERR, F_L3_CHKSUM_ERR, F_TCP_ERR, F_UDP_ERR, F_SCTP_ERR,
	F_L4_CHKSUM_ERR
};
#define F_ERROR_MASK 0xFE000000u

#define IFLAG(p, bit) ((int)((PK(p)->meta.input_flags >> (bit)) & 1u))
#define EFLAG(p, bit) ((int)((PK(p)->meta.flags >> (bit)) & 1u))

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

odp_event_type_t odp_event_type(odp_event_t event)
{
	(void)event;
	return ODP_EVENT_PACKET;
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

odp_pktio_t odp_packet_input(odp_packet_t pkt)
{
	return PK(pkt)->input;
}

int odp_packet_input_index(odp_packet_t pkt)
{
	return PK(pkt)->input == ODP_PKTIO_INVALID ? -1 : 0;
}

int odpg_packet_view(odp_packet_t pkt, odpg_packet_t *view)
{
	const rt_pkt_t *k = PK(pkt);

	if (!k || k->magic != PKT_MAGIC || !view)
		return -1;
	memset(view, 0, sizeof(*view));
	view->data = k->data;
	view->len = k->len;
	view->meta = k->meta;
	return 0;
}

/* packet_flag_inlines.h:62-288 over the kernel's packet_parser_t */
int odp_packet_has_error(odp_packet_t pkt)
{
	return (PK(pkt)->meta.flags & F_ERROR_MASK) != 0u;   /* flags.all.error */
}

int odp_packet_has_l2_error(odp_packet_t pkt) { return EFLAG(pkt, F_SNAP_LEN_ERR); }
int odp_packet_has_l3_error(odp_packet_t pkt) { return EFLAG(pkt, F_IP_ERR); }

int odp_packet_has_l4_error(odp_packet_t pkt)
{
	return EFLAG(pkt, F_TCP_ERR) | EFLAG(pkt, F_UDP_ERR);
}

int odp_packet_has_l2(odp_packet_t pkt)         { return IFLAG(pkt, IF_L2); }
int odp_packet_has_l3(odp_packet_t pkt)         { return IFLAG(pkt, IF_L3); }
int odp_packet_has_l4(odp_packet_t pkt)         { return IFLAG(pkt, IF_L4); }
int odp_packet_has_eth(odp_packet_t pkt)        { return IFLAG(pkt, IF_ETH); }
int odp_packet_has_eth_bcast(odp_packet_t pkt)  { return IFLAG(pkt, IF_ETH_BCAST); }
int odp_packet_has_eth_mcast(odp_packet_t pkt)  { return IFLAG(pkt, IF_ETH_MCAST); }
int odp_packet_has_jumbo(odp_packet_t pkt)      { return IFLAG(pkt, IF_JUMBO); }
int odp_packet_has_vlan(odp_packet_t pkt)       { return IFLAG(pkt, IF_VLAN); }
int odp_packet_has_vlan_qinq(odp_packet_t pkt)  { return IFLAG(pkt, IF_VLAN_QINQ); }
int odp_packet_has_arp(odp_packet_t pkt)        { return IFLAG(pkt, IF_ARP); }
int odp_packet_has_ipv4(odp_packet_t pkt)       { return IFLAG(pkt, IF_IPV4); }
int odp_packet_has_ipv6(odp_packet_t pkt)       { return IFLAG(pkt, IF_IPV6); }
int odp_packet_has_ip_bcast(odp_packet_t pkt)   { return IFLAG(pkt, IF_IP_BCAST); }
int odp_packet_has_ip_mcast(odp_packet_t pkt)   { return IFLAG(pkt, IF_IP_MCAST); }
int odp_packet_has_ipfrag(odp_packet_t pkt)     { return IFLAG(pkt, IF_IPFRAG); }
int odp_packet_has_ipopt(odp_packet_t pkt)      { return IFLAG(pkt, IF_IPOPT); }
int odp_packet_has_ipsec(odp_packet_t pkt)      { return IFLAG(pkt, IF_IPSEC); }
int odp_packet_has_udp(odp_packet_t pkt)        { return IFLAG(pkt, IF_UDP); }
int odp_packet_has_tcp(odp_packet_t pkt)        { return IFLAG(pkt, IF_TCP); }
int odp_packet_has_sctp(odp_packet_t pkt)       { return IFLAG(pkt, IF_SCTP); }
int odp_packet_has_icmp(odp_packet_t pkt)       { return IFLAG(pkt, IF_ICMP); }
int odp_packet_has_flow_hash(odp_packet_t pkt)  { return IFLAG(pkt, IF_FLOW_HASH); }
int odp_packet_has_ts(odp_packet_t pkt)         { return IFLAG(pkt, IF_TIMESTAMP); }

/* packet_inlines.h:385-417 */
static odp_packet_chksum_status_t chksum_status(odp_packet_t pkt, int done_bit, int err_bit)
{
	if (!IFLAG(pkt, done_bit))
		return ODP_PACKET_CHKSUM_UNKNOWN;
	return EFLAG(pkt, err_bit) ? ODP_PACKET_CHKSUM_BAD : ODP_PACKET_CHKSUM_OK;
}

odp_packet_chksum_status_t odp_packet_l3_chksum_status(odp_packet_t pkt)
{
	return chksum_status(pkt, IF_L3_CHKSUM_DONE, F_L3_CHKSUM_ERR);
}

odp_packet_chksum_status_t odp_packet_l4_chksum_status(odp_packet_t pkt)
{
	return chksum_status(pkt, IF_L4_CHKSUM_DONE, F_L4_CHKSUM_ERR);
}

/* packet_inlines.h:617: the mark of the last PMR matched, if one was */
uint64_t odp_packet_cls_mark(odp_packet_t pkt)
{
	return IFLAG(pkt, IF_CLS_MARK) ? PK(pkt)->meta.cls_mark : 0;
}

/* packet_inlines.h:334-383 */
odp_proto_l2_type_t odp_packet_l2_type(odp_packet_t pkt)
{
	return IFLAG(pkt, IF_ETH) ? ODP_PROTO_L2_TYPE_ETH : ODP_PROTO_L2_TYPE_NONE;
}

odp_proto_l3_type_t odp_packet_l3_type(odp_packet_t pkt)
{
	if (IFLAG(pkt, IF_IPV4))
		return ODP_PROTO_L3_TYPE_IPV4;
	if (IFLAG(pkt, IF_IPV6))
		return ODP_PROTO_L3_TYPE_IPV6;
	if (IFLAG(pkt, IF_ARP))
		return ODP_PROTO_L3_TYPE_ARP;
	return ODP_PROTO_L3_TYPE_NONE;
}

odp_proto_l4_type_t odp_packet_l4_type(odp_packet_t pkt)
{
	if (IFLAG(pkt, IF_TCP))
		return ODP_PROTO_L4_TYPE_TCP;
	if (IFLAG(pkt, IF_UDP))
		return ODP_PROTO_L4_TYPE_UDP;
	if (IFLAG(pkt, IF_SCTP))
		return ODP_PROTO_L4_TYPE_SCTP;
	if (IFLAG(pkt, IF_IPSEC_AH))
		return ODP_PROTO_L4_TYPE_AH;
	if (IFLAG(pkt, IF_IPSEC_ESP))
		return ODP_PROTO_L4_TYPE_ESP;
	if (IFLAG(pkt, IF_ICMP) && IFLAG(pkt, IF_IPV4))
		return ODP_PROTO_L4_TYPE_ICMPV4;
	if (IFLAG(pkt, IF_ICMP) && IFLAG(pkt, IF_IPV6))
		return ODP_PROTO_L4_TYPE_ICMPV6;
	if (IFLAG(pkt, IF_NO_NEXT_HDR))
		return ODP_PROTO_L4_TYPE_NO_NEXT;
	return ODP_PROTO_L4_TYPE_NONE;
}

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

/* odp_packet_lN_offset_set (odp_packet.c): offsets inside the packet; the
 * L2 setter also marks the packet as having L2 (packet_hdr_has_l2_set) */
static int offset_set(odp_packet_t pkt, uint16_t *field, uint32_t off)
{
	if (off >= PK(pkt)->len)
		return -1;
	*field = (uint16_t)off;
	return 0;
}

int odp_packet_l2_offset_set(odp_packet_t pkt, uint32_t offset)
{
	if (offset_set(pkt, &PK(pkt)->meta.l2_offset, offset))
		return -1;
	PK(pkt)->meta.input_flags |= 1ull << IF_L2;
	return 0;
}

int odp_packet_l3_offset_set(odp_packet_t pkt, uint32_t offset)
{
	return offset_set(pkt, &PK(pkt)->meta.l3_offset, offset);
}

int odp_packet_l4_offset_set(odp_packet_t pkt, uint32_t offset)
{
	return offset_set(pkt, &PK(pkt)->meta.l4_offset, offset);
}

int odp_packet_copy_to_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, void *dst)
{
	const rt_pkt_t *k = PK(pkt);

	if ((uint64_t)offset + len > k->len)
		return -1;
	memcpy(dst, k->data + offset, len);
	return 0;
}

int odp_packet_copy_from_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, const void *src)
{
	rt_pkt_t *k = PK(pkt);

	if ((uint64_t)offset + len > k->len)
		return -1;
	memcpy(k->data + offset, src, len);
	return 0;
}

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

/* odp_chksum.c: chksum_finalize(chksum_partial(p, len, 0)) — 32-bit
 * little-endian words into a 64-bit sum, a 16-bit and a byte tail, folded */
uint16_t odp_chksum_ones_comp16(const void *data, uint32_t len)
{
	const uint8_t *b = data;
	uint64_t sum = 0;
	uint32_t w;
	uint16_t h;

	for (; len >= 4; b += 4, len -= 4) {
		memcpy(&w, b, 4);
		sum += w;
	}
	if (len >= 2) {
		memcpy(&h, b, 2);
		sum += h;
		b += 2;
		len -= 2;
	}
	if (len)
		sum += *b;
	sum = (sum >> 32) + (sum & 0xffffffffu);
	sum = (sum >> 16) + (sum & 0xffffu);
	return (uint16_t)((sum >> 16) + sum);
}

/* ---- odp_packet_parse on the GPU parser ------------------------------------
 * odp_packet.c:1986-2075. The packets' bytes from `offset` are staged into
 * one 64-byte aligned buffer and parsed by the classifier kernel with
 * classification off, the batch's parse layer and the parameter's checksum
 * options. A parse that starts at L3 (ODP_PROTO_IPV4 / IPV6) is staged
 * behind a 14-byte Ethernet header carrying that ethertype; the L2 result
 * of that header is then removed again (l2 / eth / jumbo flags, L2 offset),
 * which is exactly the reference's state after _odp_packet_parse_common_l3_l4
 * was called with that ethtype: every L3 / L4 check is relative to the
 * parse offset and the frame's end, so the header in front changes none of
 * them. Offsets are rebased to the packet. A packet fails (-1) when the
 * parser returned non-zero, i.e. any error flag (or a drop) — as
 * odp_packet_parse returns -1 on a non-zero _odp_packet_parse_common_l3_l4
 * or _odp_packet_l4_chksum. Flags outside the error group are kept
 * (packet_parse_reset(pkt_hdr, 0)). */
static struct {
	pthread_mutex_t lock;
	odpg_table_t *tbl;         /* an empty rule table: parse only */
	uint8_t *buf;
	size_t cap;
	odpg_desc_t *desc;
	odpg_out_t *out;
	odpg_meta_t *meta;
	uint32_t n_cap;
} prs = { PTHREAD_MUTEX_INITIALIZER, NULL, NULL, 0, NULL, NULL, NULL, 0 };

static void parse_release(void)
{
	pthread_mutex_lock(&prs.lock);
	if (prs.tbl)
		odpg_table_destroy(prs.tbl);
	prs.tbl = NULL;
	free(prs.buf);
	free(prs.desc);
	free(prs.out);
	free(prs.meta);
	prs.buf = NULL;
	prs.desc = NULL;
	prs.out = NULL;
	prs.meta = NULL;
	prs.cap = 0;
	prs.n_cap = 0;
	pthread_mutex_unlock(&prs.lock);
}

#define ALIGN64(x) (((x) + 63u) & ~(size_t)63u)
#define PARSE_FAKE_L2 14u

static int parse_batch(const odp_packet_t pkt[], const uint32_t offset[], int num,
		       const odp_packet_parse_param_t *param)
{
	const int l3start = param->proto != ODP_PROTO_ETH;
	const uint32_t pre = l3start ? PARSE_FAKE_L2 : 0u;
	uint16_t ethtype = 0xffffu;        /* unknown: not IPv4 / IPv6 / ARP / VLAN / SNAP */
	uint64_t opt = 0;
	size_t need = 0, off = 0;
	int ok = 0;

	if (num <= 0)
		return 0;
	if (param->proto == ODP_PROTO_NONE || param->last_layer == ODP_PROTO_LAYER_NONE)
		return 0;                  /* the first packet fails */
	if (param->proto == ODP_PROTO_IPV4)
		ethtype = 0x0800;
	else if (param->proto == ODP_PROTO_IPV6)
		ethtype = 0x86dd;
	if (param->chksums.chksum.ipv4)
		opt |= ODPG_PKTIN_IPV4_CHKSUM;
	if (param->chksums.chksum.udp)
		opt |= ODPG_PKTIN_UDP_CHKSUM;
	if (param->chksums.chksum.tcp)
		opt |= ODPG_PKTIN_TCP_CHKSUM;
	if (param->chksums.chksum.sctp)
		opt |= ODPG_PKTIN_SCTP_CHKSUM;

	/* stage up to the first packet whose offset is past its end (packet_map
	 * fails: -1 before anything is parsed) */
	int n = 0;

	for (; n < num; n++) {
		const rt_pkt_t *k = PK(pkt[n]);

		if (offset[n] >= k->len)
			break;
		need += ALIGN64(pre + k->len - offset[n]);
	}
	if (n == 0)
		return 0;
	if (!rt.init && odp_init_global(NULL, NULL, NULL))
		return -1;
	pthread_mutex_lock(&prs.lock);
	if (!prs.tbl) {
		odpg_rules_t none;

		memset(&none, 0, sizeof(none));
		none.default_cos = -1;
		none.error_cos = -1;
		if (odpg_table_create(rt.ctx, &none, &prs.tbl)) {
			pthread_mutex_unlock(&prs.lock);
			return -1;
		}
	}
	need += 128;
	if (need > prs.cap) {
		uint8_t *b = NULL;

		if (posix_memalign((void **)&b, 64, need)) {
			pthread_mutex_unlock(&prs.lock);
			return -1;
		}
		free(prs.buf);
		prs.buf = b;
		prs.cap = need;
	}
	if ((uint32_t)n > prs.n_cap) {
		free(prs.desc);
		free(prs.out);
		free(prs.meta);
		prs.desc = malloc((size_t)n * sizeof(*prs.desc));
		prs.out = malloc((size_t)n * sizeof(*prs.out));
		prs.meta = malloc((size_t)n * sizeof(*prs.meta));
		prs.n_cap = prs.desc && prs.out && prs.meta ? (uint32_t)n : 0;
		if (!prs.n_cap) {
			pthread_mutex_unlock(&prs.lock);
			return -1;
		}
	}
	for (int i = 0; i < n; i++) {
		const rt_pkt_t *k = PK(pkt[i]);
		uint8_t *d = prs.buf + off;
		const uint32_t len = k->len - offset[i];

		if (pre) {
			memset(d, 0, 12);
			d[0] = 0x02;               /* locally administered unicast */
			d[12] = (uint8_t)(ethtype >> 8);
			d[13] = (uint8_t)ethtype;
		}
		memcpy(d + pre, k->data + offset[i], len);
		prs.desc[i].offset = (uint32_t)off;
		prs.desc[i].len = pre + len;
		off += ALIGN64(pre + len);
	}
	memset(prs.buf + off, 0, 128);

	odpg_batch_t b;
	odpg_result_t r;

	memset(&b, 0, sizeof(b));
	memset(&r, 0, sizeof(r));
	b.frames = prs.buf;
	b.desc = prs.desc;
	b.num = (uint32_t)n;
	b.pktin_opt = opt;
	b.layer = (uint32_t)param->last_layer;
	b.classify = 0;
	r.out = prs.out;
	r.meta = prs.meta;
	if (odpg_classify_host(rt.ctx, prs.tbl, &b, &r, 0)) {
		pthread_mutex_unlock(&prs.lock);
		return -1;
	}
	for (int i = 0; i < n; i++) {
		rt_pkt_t *k = PK(pkt[i]);
		odpg_meta_t m = prs.meta[i];
		const uint32_t base = offset[i];

		if (l3start) {
			m.input_flags &= ~((1ull << IF_L2) | (1ull << IF_ETH) | (1ull << IF_JUMBO) |
					   (1ull << IF_ETH_BCAST) | (1ull << IF_ETH_MCAST));
			m.l2_offset = 0xffff;
		} else if (m.l2_offset != 0xffff) {
			m.l2_offset = (uint16_t)(m.l2_offset + base);
		}
		if (m.l3_offset != 0xffff)
			m.l3_offset = (uint16_t)(m.l3_offset - pre + base);
		if (m.l4_offset != 0xffff)
			m.l4_offset = (uint16_t)(m.l4_offset - pre + base);
		m.flags = (k->meta.flags & ~F_ERROR_MASK) | (m.flags & F_ERROR_MASK);
		m.cls_mark = 0;
		m.reserved = 0;
		k->meta = m;
		if (prs.out[i] & ODPG_OUT_PARSE_ERR)
			break;                     /* odp_packet_parse returned -1 */
		ok++;
	}
	pthread_mutex_unlock(&prs.lock);
	return ok;
}

int odp_packet_parse(odp_packet_t pkt, uint32_t offset, const odp_packet_parse_param_t *param)
{
	const int r = parse_batch(&pkt, &offset, 1, param);

	return r == 1 ? 0 : -1;
}

int odp_packet_parse_multi(const odp_packet_t pkt[], const uint32_t offset[], int num,
			   const odp_packet_parse_param_t *param)
{
	const int r = parse_batch(pkt, offset, num, param);

	return r < 0 ? -1 : r;
}

/* odp_packet.c:2077-2126 */
void odp_packet_parse_result(odp_packet_t pkt, odp_packet_parse_result_t *res)
{
	res->flag.all = 0;
	res->flag.has_error = odp_packet_has_error(pkt);
	res->flag.has_l2_error = odp_packet_has_l2_error(pkt);
	res->flag.has_l3_error = odp_packet_has_l3_error(pkt);
	res->flag.has_l4_error = odp_packet_has_l4_error(pkt);
	res->flag.has_l2 = odp_packet_has_l2(pkt);
	res->flag.has_l3 = odp_packet_has_l3(pkt);
	res->flag.has_l4 = odp_packet_has_l4(pkt);
	res->flag.has_eth = odp_packet_has_eth(pkt);
	res->flag.has_eth_bcast = odp_packet_has_eth_bcast(pkt);
	res->flag.has_eth_mcast = odp_packet_has_eth_mcast(pkt);
	res->flag.has_jumbo = odp_packet_has_jumbo(pkt);
	res->flag.has_vlan = odp_packet_has_vlan(pkt);
	res->flag.has_vlan_qinq = odp_packet_has_vlan_qinq(pkt);
	res->flag.has_arp = odp_packet_has_arp(pkt);
	res->flag.has_ipv4 = odp_packet_has_ipv4(pkt);
	res->flag.has_ipv6 = odp_packet_has_ipv6(pkt);
	res->flag.has_ip_bcast = odp_packet_has_ip_bcast(pkt);
	res->flag.has_ip_mcast = odp_packet_has_ip_mcast(pkt);
	res->flag.has_ipfrag = odp_packet_has_ipfrag(pkt);
	res->flag.has_ipopt = odp_packet_has_ipopt(pkt);
	res->flag.has_ipsec = odp_packet_has_ipsec(pkt);
	res->flag.has_udp = odp_packet_has_udp(pkt);
	res->flag.has_tcp = odp_packet_has_tcp(pkt);
	res->flag.has_sctp = odp_packet_has_sctp(pkt);
	res->flag.has_icmp = odp_packet_has_icmp(pkt);
	res->packet_len = odp_packet_len(pkt);
	res->l2_offset = odp_packet_l2_offset(pkt);
	res->l3_offset = odp_packet_l3_offset(pkt);
	res->l4_offset = odp_packet_l4_offset(pkt);
	res->l3_chksum_status = odp_packet_l3_chksum_status(pkt);
	res->l4_chksum_status = odp_packet_l4_chksum_status(pkt);
	res->l2_type = odp_packet_l2_type(pkt);
	res->l3_type = odp_packet_l3_type(pkt);
	res->l4_type = odp_packet_l4_type(pkt);
}

void odp_packet_parse_result_multi(const odp_packet_t pkt[], odp_packet_parse_result_t *result[],
				   int num)
{
	for (int i = 0; i < num; i++)
		odp_packet_parse_result(pkt[i], result[i]);
}

/* ---- queues: a registry of tagged handles ---------------------------------- */
static int pktout_send_impl(odp_pktio_t pktio, uint32_t index, const odp_packet_t packets[],
			    int num);
static void pktin_queue_fill(odp_pktio_t pktio);

#define QH_TAG      0x0DD0000000000000ull  /* no user-space pointer has these bits */
#define QH_TAG_MASK 0xFFFF000000000000ull
#define QH_IDX_BITS 21                     /* slot index + 1 */
#define QH_GEN_MASK 0x7FFFFFFull           /* the 27 bits above it */
#define QCHUNK      4096u
#define QCHUNKS     256u                   /* up to 1 M live queues */

/* Queue registry: a handle is tag | generation | slot + 1. A destroyed
 * queue's slot goes on a free list and its object is reused by the next
 * create with the generation advanced, so create / destroy cycles do not
 * use the registry up and a stale handle stops resolving (queue_basic.c's
 * queue table frees and reuses its entries the same way). Objects are never
 * freed: a lookup racing a destroy reads valid memory and fails on the
 * handle. Scheduled queues are unlinked from the scheduler's list under the
 * write side of sched_rw, which every scheduler walk holds for reading, so
 * no walk is inside an object when it is reused. */
static struct {
	pthread_mutex_t lock;
	rt_queue_t **chunk[QCHUNKS];
	uint32_t num;              /* slots handed out (published with release) */
	uint32_t *free;            /* destroyed slots */
	uint32_t nfree, cap;
} qreg = { PTHREAD_MUTEX_INITIALIZER, {0}, 0, NULL, 0, 0 };
static pthread_rwlock_t sched_rw = PTHREAD_RWLOCK_INITIALIZER;

static rt_queue_t *queue_slot(odp_queue_t q)
{
	const uint64_t v = (uint64_t)(uintptr_t)q;

	if ((v & QH_TAG_MASK) != QH_TAG)
		return NULL;
	const uint64_t idx = (v & ((1ull << QH_IDX_BITS) - 1u)) - 1u;

	if (idx >= __atomic_load_n(&qreg.num, __ATOMIC_ACQUIRE))
		return NULL;
	return qreg.chunk[idx / QCHUNK][idx % QCHUNK];
}

static rt_queue_t *get_queue(odp_queue_t q)
{
	rt_queue_t *x = queue_slot(q);

	if (!x || x->magic != QUEUE_MAGIC ||
	    __atomic_load_n(&x->hdl, __ATOMIC_ACQUIRE) != q || x->dead)
		return NULL;
	return x;
}

static rt_queue_t *queue_new(const char *name, const odp_queue_param_t *param)
{
	rt_queue_t *q = NULL;
	uint32_t idx;

	pthread_mutex_lock(&qreg.lock);
	if (qreg.nfree) {
		idx = qreg.free[--qreg.nfree];
		q = qreg.chunk[idx / QCHUNK][idx % QCHUNK];
	} else {
		idx = qreg.num;
		if (idx >= QCHUNK * QCHUNKS ||
		    (!qreg.chunk[idx / QCHUNK] &&
		     !(qreg.chunk[idx / QCHUNK] = calloc(QCHUNK, sizeof(rt_queue_t *)))) ||
		    !(q = calloc(1, sizeof(*q)))) {
			pthread_mutex_unlock(&qreg.lock);
			ERR("queue registry full\n");
			return NULL;
		}
		rt_mutex_init(&q->lock);
		q->magic = QUEUE_MAGIC;
	}
	/* a reused object: the destroyed queue's fields reset (its lock and
	 * magic stay), generation advanced */
	q->gen = (q->gen + 1u) & (uint32_t)QH_GEN_MASK;
	snprintf(q->name, sizeof(q->name), "%s", name ? name : "");
	if (param)
		q->param = *param;
	else
		odp_queue_param_init(&q->param);
	q->ev.rd = 0;
	__atomic_store_n(&q->ev.n, 0u, __ATOMIC_RELAXED);
	q->sched = q->param.type == ODP_QUEUE_TYPE_SCHED;
	q->next_sched = NULL;
	q->pktin = q->pktout = ODP_PKTIO_INVALID;
	q->dead = 0;
	__atomic_store_n(&q->hdl, (odp_queue_t)(uintptr_t)(QH_TAG | ((uint64_t)q->gen << QH_IDX_BITS) |
							     (uint64_t)(idx + 1u)), __ATOMIC_RELEASE);
	if (idx == qreg.num) {
		qreg.chunk[idx / QCHUNK][idx % QCHUNK] = q;
		__atomic_store_n(&qreg.num, idx + 1u, __ATOMIC_RELEASE);
	}
	pthread_mutex_unlock(&qreg.lock);
	if (q->param.type == ODP_QUEUE_TYPE_SCHED) {
		pthread_rwlock_wrlock(&sched_rw);
		q->next_sched = rt.sched;
		rt.sched = q;
		pthread_rwlock_unlock(&sched_rw);
	}
	return q;
}

/* a dead queue out of the scheduler's list and its slot onto the free list */
static void queue_release(rt_queue_t *q)
{
	if (q->param.type == ODP_QUEUE_TYPE_SCHED) {
		pthread_rwlock_wrlock(&sched_rw);
		for (rt_queue_t **pp = &rt.sched; *pp; pp = &(*pp)->next_sched)
			if (*pp == q) {
				*pp = q->next_sched;
				break;
			}
		pthread_rwlock_unlock(&sched_rw);
	}
	const uint64_t v = (uint64_t)(uintptr_t)q->hdl;
	const uint32_t idx = (uint32_t)((v & ((1ull << QH_IDX_BITS) - 1u)) - 1u);

	pthread_mutex_lock(&qreg.lock);
	if (qreg.nfree == qreg.cap) {
		const uint32_t nc = qreg.cap ? 2u * qreg.cap : 256u;
		uint32_t *nf = realloc(qreg.free, nc * sizeof(uint32_t));

		if (!nf) {                      /* the slot stays used */
			pthread_mutex_unlock(&qreg.lock);
			return;
		}
		qreg.free = nf;
		qreg.cap = nc;
	}
	qreg.free[qreg.nfree++] = idx;
	pthread_mutex_unlock(&qreg.lock);
}

odp_queue_t odp_queue_create(const char *name, const odp_queue_param_t *param)
{
	rt_queue_t *q = queue_new(name, param);

	return q ? q->hdl : ODP_QUEUE_INVALID;
}

/* queue_basic.c queue_destroy: an empty queue only; its slot is reused */
int odp_queue_destroy(odp_queue_t queue)
{
	rt_queue_t *q = get_queue(queue);

	if (!q)
		return -1;
	pthread_mutex_lock(&q->lock);
	if (q->ev.n || q->dead) {
		const int busy = q->ev.n != 0;

		pthread_mutex_unlock(&q->lock);
		if (busy)
			ERR("queue '%s' not empty\n", q->name);
		return -1;
	}
	q->dead = 1;
	pthread_mutex_unlock(&q->lock);
	queue_release(q);
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

odp_queue_type_t odp_queue_type(odp_queue_t queue)
{
	rt_queue_t *q = get_queue(queue);

	return q ? q->param.type : ODP_QUEUE_TYPE_PLAIN;
}

uint64_t odp_queue_to_u64(odp_queue_t queue)
{
	return (uint64_t)(uintptr_t)queue;
}

/* num events at the queue's tail, all or none (-1: no memory) */
static int queue_push(rt_queue_t *q, const odp_event_t ev[], uint32_t num)
{
	pthread_mutex_lock(&q->lock);
	const int ret = pring_push(&q->ev, (void *const *)ev, num);

	if (!ret && q->sched)
		__atomic_fetch_add(&rt.sched_n, num, __ATOMIC_RELEASE);
	pthread_mutex_unlock(&q->lock);
	return ret;
}

int odp_queue_enq(odp_queue_t queue, odp_event_t ev)
{
	return odp_queue_enq_multi(queue, &ev, 1) == 1 ? 0 : -1;
}

/* all num events in one append (queue_basic.c enq_multi), or -1 */
int odp_queue_enq_multi(odp_queue_t queue, const odp_event_t ev[], int num)
{
	rt_queue_t *q = get_queue(queue);

	if (!q || num < 0)
		return -1;
	if (num == 0)
		return 0;
	for (int i = 0; i < num; i++)
		if (!ev[i])
			return -1;
	if (q->pktout)                  /* pktout event queue: transmit */
		return pktout_send_impl(q->pktout, q->pindex, (const odp_packet_t *)ev, num);
	return queue_push(q, ev, (uint32_t)num) ? -1 : num;
}

static int deq_multi(rt_queue_t *q, odp_event_t ev[], int num);

odp_event_t odp_queue_deq(odp_queue_t queue)
{
	odp_event_t ev = ODP_EVENT_INVALID;

	return odp_queue_deq_multi(queue, &ev, 1) == 1 ? ev : ODP_EVENT_INVALID;
}

int odp_queue_deq_multi(odp_queue_t queue, odp_event_t ev[], int num)
{
	rt_queue_t *q = get_queue(queue);

	if (!q)
		return -1;
	if (q->pktin && !__atomic_load_n(&q->ev.n, __ATOMIC_RELAXED))
		pktin_queue_fill(q->pktin);     /* QUEUE mode: receive a burst */
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
	/* an empty queue without its lock: pollers spinning on empty queues
	 * keep off the line the producer locks */
	if (num <= 0 || !__atomic_load_n(&q->ev.n, __ATOMIC_ACQUIRE))
		return 0;
	pthread_mutex_lock(&q->lock);
	const uint32_t n = pring_pop(&q->ev, (void **)ev, (uint32_t)num);

	if (n && q->sched)
		__atomic_fetch_sub(&rt.sched_n, n, __ATOMIC_RELAXED);
	pthread_mutex_unlock(&q->lock);
	return (int)n;
}

/* ---- pktio input ----------------------------------------------------------- */
static rt_pktio_t *get_rt_pktio(odp_pktio_t hdl)
{
	const uintptr_t n = (uintptr_t)hdl;

	return n && n <= RT_MAX_PKTIO && rt.pktio[n - 1].valid ? &rt.pktio[n - 1] : NULL;
}

/* a queue the pktio owns: unlinked from use, its packets freed, its slot
 * reused */
static void pktio_queue_kill(rt_queue_t **qp)
{
	rt_queue_t *q = *qp;

	*qp = NULL;
	if (!q)
		return;
	pthread_mutex_lock(&q->lock);
	ptr_ring_t ev = q->ev;
	const int was_dead = q->dead;

	memset(&q->ev, 0, sizeof(q->ev));
	if (q->sched && ev.n)
		__atomic_fetch_sub(&rt.sched_n, ev.n, __ATOMIC_RELAXED);
	q->dead = 1;
	q->pktin = q->pktout = ODP_PKTIO_INVALID;
	pthread_mutex_unlock(&q->lock);
	pring_free_packets(&ev);
	if (!was_dead)
		queue_release(q);
}

/* "loop[...]" (pktio/loop.c) or "pcap:in=<file>[:loops=<n>]" (pktio/pcap.c's
 * device string, _pcapif_parse_devname) */
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
	p->loops = 1;                       /* pcapif_init: loops = 1, loop_cnt = 1 */
	p->loop_cnt = 1;
	p->in_mode = param->in_mode;
	p->out_mode = param->out_mode;
	p->pool = pool;
	p->mtu = LOOP_MTU;
	p->loopdev = !strncmp(name, "loop", 4);
	rt_mutex_init(&p->ring_lock);
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
		pthread_mutex_lock(&rx_dlock[p - rt.pktio]);
		/* no new delivering thread looks at the pktio; those inside
		 * finish their chunks (the bursts in flight are dropped or, when
		 * opened, delivered by rx_release) */
		__atomic_store_n(&p->valid, 0, __ATOMIC_SEQ_CST);
		for (uint32_t sp = 0; __atomic_load_n(&rx_helpers[p - rt.pktio], __ATOMIC_SEQ_CST);)
			spin_wait(&sp);
		if (p->have_cap)
			odpg_pcap_free(&p->cap);
		for (uint32_t q = 0; q < RT_MAXQ; q++) {
			pktio_queue_kill(&p->inq[q]);
			pktio_queue_kill(&p->outq[q]);
			for (rt_pkt_t *x = p->ahead[q]; x;) {
				rt_pkt_t *nx = x->next;

				odp_packet_free((odp_packet_t)x);
				x = nx;
			}
			p->ahead[q] = p->ahead_tail[q] = NULL;
			pring_free_packets(&p->ring[q]);
		}
		rx_release(p);
		pthread_mutex_destroy(&p->ring_lock);
		memset(p, 0, sizeof(*p));
		pthread_mutex_unlock(&rx_dlock[p - rt.pktio]);
	}
	pthread_mutex_unlock(&rt.poll_lock);
}

/* the input queues odp_pktin_queue_config() asked for (a loop device up to
 * RT_MAXQ, loop.c:206-235; a capture one) and their hash protocols; QUEUE /
 * SCHED mode get their event queues ("odp-pktin-<i>-<q>", odp_packet_io.c) */
int odpg_rt_pktin_config(odp_pktio_t hdl, uint32_t num_queues, uint32_t hash_bits)
{
	rt_pktio_t *p = get_rt_pktio(hdl);
	odp_queue_param_t qp;
	char name[ODP_QUEUE_NAME_LEN];

	if (!p)
		return -1;
	if (p->in_mode == ODP_PKTIN_MODE_DISABLED)
		return 0;
	if (num_queues > (p->loopdev ? RT_MAXQ : 1u)) {
		ERR("pktio %" PRIu64 ": too many input queues\n", (uint64_t)(uintptr_t)hdl);
		return -1;
	}
	p->num_in = num_queues;
	p->hash_bits = hash_bits;
	for (uint32_t q = 0; q < RT_MAXQ; q++)
		pktio_queue_kill(&p->inq[q]);
	if (p->in_mode != ODP_PKTIN_MODE_QUEUE && p->in_mode != ODP_PKTIN_MODE_SCHED)
		return 0;
	odp_queue_param_init(&qp);
	qp.type = p->in_mode == ODP_PKTIN_MODE_SCHED ? ODP_QUEUE_TYPE_SCHED : ODP_QUEUE_TYPE_PLAIN;
	for (uint32_t q = 0; q < num_queues; q++) {
		snprintf(name, sizeof(name), "odp-pktin-%u-%u", (unsigned)(uintptr_t)hdl, q);
		p->inq[q] = queue_new(name, &qp);
		if (!p->inq[q])
			return -1;
		p->inq[q]->pindex = q;
		if (p->in_mode == ODP_PKTIN_MODE_QUEUE)
			p->inq[q]->pktin = hdl;
	}
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

/* _odp_cos_enq (odp_classification_internal.h:139-156): a run of packets
 * for one (CoS, queue) in one odp_queue_enq_multi; what is not enqueued is
 * freed and counted as the queue's discards (the kernel counted the run as
 * delivered) */
static void cos_enq(odp_cos_t cos, odp_queue_t q, odp_packet_t run[], int num)
{
	int ret;

	if (num <= 0)
		return;
	ret = odp_queue_enq_multi(q, (const odp_event_t *)run, num);
	if (ret < 0)
		ret = 0;
	if (ret != num) {
		odp_packet_free_multi(&run[ret], num - ret);
		odpg_cls_queue_count(cos, q, -(int64_t)(num - ret), (uint64_t)(num - ret));
	}
}

/* ---- receive pipeline ----------------------------------------------------------
 * A receive burst: the frames waiting on the loop device (or the next ones of
 * the capture) gathered into a slot's pinned staging buffer, classified by one
 * zero-copy launch (the kernel reads the frames and descriptors and writes the
 * verdicts and parse metadata in place over PCIe: a burst is a few KiB), then
 * delivered (loopback_recv's post-classification steps: CoS queues, pools,
 * discards). The event-queue modes keep up to RT_INFLIGHT bursts in flight per
 * pktio: a poll delivers the bursts whose fence has completed, oldest first,
 * and launches the frames that have arrived meanwhile, without waiting for
 * the GPU. DIRECT mode (odp_pktin_recv) launches and waits. */
static rx_slot_t *slot_get(rt_pktio_t *p, uint32_t i)
{
	rx_slot_t *s = p->slot[i];

	if (s)
		return s;
	if (!(s = calloc(1, sizeof(*s))))
		return NULL;
	/* bursts of pktio k in slot i launch on device context (k RT_INFLIGHT +
	 * i) mod nctx: a pktio's bursts in flight spread over the devices,
	 * and several pktios over all of them */
	s->ctx = rt.ctxs[((uint32_t)(p - rt.pktio) * RT_INFLIGHT + i) % (rt.nctx ? rt.nctx : 1u)];
	if (pinned_alloc(RT_BURST * sizeof(odpg_desc_t), (void **)&s->desc, (void **)&s->ddesc) ||
	    pinned_alloc(RT_BURST * sizeof(odpg_out_t), (void **)&s->out, (void **)&s->dout) ||
	    pinned_alloc(RT_BURST * sizeof(odpg_meta_t), (void **)&s->meta, (void **)&s->dmeta) ||
	    odpg_fence_create(s->ctx, &s->fence)) {
		odpg_host_free_pinned(s->desc);
		odpg_host_free_pinned(s->out);
		odpg_host_free_pinned(s->meta);
		free(s);
		ERR("no pinned host memory for a receive burst\n");
		return NULL;
	}
	p->slot[i] = s;
	return s;
}

static void slots_free(rt_pktio_t *p)
{
	for (uint32_t i = 0; i < RT_INFLIGHT; i++) {
		rx_slot_t *s = p->slot[i];

		if (!s)
			continue;
		odpg_fence_destroy(s->fence);
		odpg_host_free_pinned(s->desc);
		odpg_host_free_pinned(s->out);
		odpg_host_free_pinned(s->meta);
		odpg_host_free_pinned(s->stage);
		free(s);
		p->slot[i] = NULL;
	}
	p->launched = p->delivered = 0;
}

static void rx_drop(struct rx_slot *s);

/* the bursts in flight waited for and dropped, the slots freed (close,
 * termination) */
static int rx_help(rt_pktio_t *p, odp_pktio_t hdl);

static void rx_release(rt_pktio_t *p)
{
	while (p->delivered != p->launched) {
		const uint32_t d = p->delivered;
		rx_slot_t *s = p->slot[d % RT_INFLIGHT];

		if (__atomic_load_n(&s->open, __ATOMIC_ACQUIRE)) {
			if ((uint32_t)(__atomic_load_n(&s->claimw, __ATOMIC_ACQUIRE) >> 32) == d) {
				/* partly delivered: the rest goes out too */
				rx_help(p, (odp_pktio_t)(uintptr_t)(p - rt.pktio + 1));
				for (uint32_t sp = 0; __atomic_load_n(&p->delivered, __ATOMIC_ACQUIRE) == d;)
					spin_wait(&sp);
			} else {
				/* the slot's previous burst still closing */
				for (uint32_t sp = 0; __atomic_load_n(&s->open, __ATOMIC_ACQUIRE);)
					spin_wait(&sp);
			}
			continue;
		}
		odpg_fence_wait(s->fence);
		odpg_cls_pktio_recv_end(s->token);
		s->token = NULL;
		rx_drop(s);
		__atomic_store_n(&p->delivered, d + 1u, __ATOMIC_RELEASE);
	}
	for (uint32_t i = 0; i < RT_INFLIGHT; i++)
		for (uint32_t sp = 0; p->slot[i] && __atomic_load_n(&p->slot[i]->busy, __ATOMIC_ACQUIRE);)
			spin_wait(&sp);
	slots_free(p);
}

/* the slot's pinned staging buffer, at least `need` bytes */
static int stage_reserve(rx_slot_t *s, size_t need)
{
	uint8_t *b = NULL, *db = NULL;

	if (need <= s->stage_cap)
		return 0;
	need = need < (64u << 10) ? (64u << 10) : need;
	if (pinned_alloc(need, (void **)&b, (void **)&db))
		return -1;
	odpg_host_free_pinned(s->stage);
	s->stage = b;
	s->dstage = db;
	s->stage_cap = need;
	return 0;
}

/* up to `num` waiting frames into the slot; returns how many (0: none, or
 * no staging memory: the loop device's frames are then dropped) */
static uint32_t rx_stage(rt_pktio_t *p, rx_slot_t *s, uint32_t num, int queue)
{
	uint32_t n = 0;
	size_t need = 0, off = 0;

	if (p->loopdev) {
		/* the handles only under the lock (the transmitters wait on
		 * it); the packets are read after. DIRECT mode takes its queue's
		 * ring (loopback_recv(index)); the event modes take every ring,
		 * starting at a rotating one, and remember each packet's queue */
		if (!__atomic_load_n(&p->ring_n, __ATOMIC_ACQUIRE))
			return 0;
		pthread_mutex_lock(&p->ring_lock);
		if (queue >= 0) {
			n = pring_pop(&p->ring[queue], (void **)s->src, num);
			memset(s->qi, queue, n);
		} else {
			const uint32_t nq = p->num_in ? p->num_in : 1u;

			for (uint32_t j = 0; j < nq && n < num; j++) {
				const uint32_t q = (p->rr + j) % nq;
				const uint32_t m = pring_pop(&p->ring[q], (void **)s->src + n, num - n);

				memset(s->qi + n, (int)q, m);
				n += m;
			}
			p->rr = (p->rr + 1u) % nq;
		}
		__atomic_store_n(&p->ring_n, p->ring_n - n, __ATOMIC_RELEASE);
		pthread_mutex_unlock(&p->ring_lock);
		if (!n)
			return 0;
		for (uint32_t k = 0; k < n; k++) {
			if (k + RX_PF < n)
				__builtin_prefetch(s->src[k + RX_PF], 0, 3);
			need += ALIGN64(s->src[k]->len);
		}
		if (stage_reserve(s, need)) {
			for (uint32_t k = 0; k < n; k++)
				odp_packet_free((odp_packet_t)s->src[k]);
			return 0;
		}
		for (uint32_t k = 0; k < n; k++) {
			if (k + RX_PF < n)
				__builtin_prefetch(s->src[k + RX_PF]->data, 0, 3);
			memcpy(s->stage + off, s->src[k]->data, s->src[k]->len);
			s->desc[k].offset = (uint32_t)off;
			s->desc[k].len = s->src[k]->len;
			off += ALIGN64(s->src[k]->len);
		}
	} else if (p->have_cap) {
		if (p->pos >= p->cap.num) {
			/* _pcapif_reopen: loops = 0 repeats forever, else the
			 * capture is read again while ++loop_cnt < loops */
			if (p->loops != 0 && ++p->loop_cnt >= p->loops)
				return 0;
			p->pos = 0;
		}
		const uint32_t first = p->pos;

		n = p->cap.num - first < num ? p->cap.num - first : num;
		if (!n)
			return 0;
		for (uint32_t k = 0; k < n; k++)
			need += ALIGN64(p->cap.desc[first + k].len);
		if (stage_reserve(s, need))
			return 0;
		for (uint32_t k = 0; k < n; k++) {
			const odpg_desc_t d = p->cap.desc[first + k];

			memcpy(s->stage + off, p->cap.frames + d.offset, d.len);
			s->desc[k].offset = (uint32_t)off;
			s->desc[k].len = d.len;
			s->src[k] = NULL;
			s->qi[k] = 0;
			off += ALIGN64(d.len);
		}
		p->pos += n;
	}
	s->n = n;
	return n;
}

static void rx_drop(rx_slot_t *s)
{
	for (uint32_t k = 0; k < s->n; k++)
		if (s->src[k])
			odp_packet_free((odp_packet_t)s->src[k]);
	s->n = 0;
}

static int rx_launch(odp_pktio_t hdl, rx_slot_t *s)
{
	if (odpg_cls_pktio_recv_start_zc(hdl, s->ctx, s->dstage, s->ddesc, s->n, s->dout, s->dmeta,
					 s->fence, &s->token)) {
		ERR("classify failed\n");
		rx_drop(s);
		return -1;
	}
	return 0;
}

/* what a range's delivery hands to the queues, in packet order */
typedef struct rx_out {
	int ninq, nq;
	odp_packet_t inq[RX_CHUNK];        /* no CoS queue: the pktin queue / caller */
	uint8_t inqi[RX_CHUNK];            /* ... of the input queue they came in on */
	odp_packet_t qp[RX_CHUNK];         /* to a CoS queue */
	odp_cos_t qcos[RX_CHUNK];
	odp_queue_t qq[RX_CHUNK];
} rx_out_t;

/* a multi-queue device's per-queue input counters for one packet's verdict,
 * as loopback_recv counts them per queue (loop.c:304-374): a parse drop or
 * an error packet in_errors, no CoS (or a CoS loop) in_discards, a drop CoS
 * nothing, otherwise in_packets / in_octets; d = -1 takes a delivered
 * packet back as a discard (no buffer for it) */
static void qcount(rt_pktio_t *p, uint32_t qi, uint32_t w, uint32_t len, int d)
{
	const uint32_t c = ODPG_OUT_COS(w);

	if (qi >= RT_MAXQ)
		return;
	if (d < 0) {
		__atomic_fetch_sub(&p->qst[qi].in_packets, 1u, __ATOMIC_RELAXED);
		__atomic_fetch_sub(&p->qst[qi].in_octets, len, __ATOMIC_RELAXED);
		__atomic_fetch_add(&p->qst[qi].in_discards, 1u, __ATOMIC_RELAXED);
	} else if (c == ODPG_COS_PDROP || (w & ODPG_OUT_ERROR)) {
		__atomic_fetch_add(&p->qst[qi].in_errors, 1u, __ATOMIC_RELAXED);
	} else if (c == ODPG_COS_NONE || c == ODPG_COS_LOOP) {
		__atomic_fetch_add(&p->qst[qi].in_discards, 1u, __ATOMIC_RELAXED);
	} else if (!(w & ODPG_OUT_CLS_DROP)) {
		__atomic_fetch_add(&p->qst[qi].in_packets, 1u, __ATOMIC_RELAXED);
		__atomic_fetch_add(&p->qst[qi].in_octets, len, __ATOMIC_RELAXED);
	}
}

/* packets [k0, k1) of a completed burst (k1 - k0 <= RX_CHUNK): verdicts to
 * pools, the packets for the queues into *o (handed over by rx_commit, in
 * chunk order); what is dropped is freed here */
static void rx_deliver_range(rt_pktio_t *p, odp_pktio_t hdl, rx_slot_t *s, uint32_t k0,
			     uint32_t k1, rx_out_t *o)
{
	odp_packet_t dead[RX_CHUNK];
	rt_pkt_t *fresh[RX_CHUNK];
	int ndead = 0;
	uint32_t want = 0, nfresh = 0, used = 0;
	const rt_pool_t *own = get_pool(p->pool);

	o->ninq = o->nq = 0;
	/* the packets without a CoS that land in the pktio's pool from
	 * elsewhere (a capture's frames; the loop device's packets from a
	 * separate transmit pool, loop.c's _odp_pktio_packet_to_pool): their
	 * buffers in one take, the originals freed in one pass at the end */
	for (uint32_t k = k0; k < k1; k++)
		if (ODPG_OUT_COS(s->out[k]) == ODPG_COS_NOCLS &&
		    (!s->src[k] || s->src[k]->pool != p->pool))
			want++;
	if (want && own)
		nfresh = pool_take(p->pool, fresh, want);
	for (uint32_t k = k0; k < k1; k++) {
		const uint32_t w = s->out[k];
		const uint32_t len = s->desc[k].len;
		rt_pkt_t *have = s->src[k];

		/* the lines this touches were last written on other cores (the
		 * transmitting threads' headers, the receiving threads' freed
		 * buffers): their ownership requested ahead, not one at a time */
		if (k + RX_PF < k1 && s->src[k + RX_PF]) {
			__builtin_prefetch(s->src[k + RX_PF], 1, 3);
			__builtin_prefetch((uint8_t *)s->src[k + RX_PF] + 64, 1, 3);
		}
		if (used + RX_PF < nfresh) {
			__builtin_prefetch(fresh[used + RX_PF], 1, 3);
			__builtin_prefetch((uint8_t *)fresh[used + RX_PF] + 64, 1, 3);
			__builtin_prefetch(fresh[used + RX_PF]->data, 1, 3);
		}
		odp_cos_t cos = ODP_COS_INVALID;
		odp_queue_t q = ODP_QUEUE_INVALID;
		odp_pool_t pool = p->pool;
		odp_packet_t pkt;

		if (p->num_in > 1u)
			qcount(p, s->qi[k], w, len, 0);

		if (ODPG_OUT_COS(w) != ODPG_COS_NOCLS) {
			q = dest_queue(w, &cos);
			if (q == ODP_QUEUE_INVALID) {
				if (have)                 /* no CoS / drop / parse drop */
					dead[ndead++] = (odp_packet_t)have;
				continue;
			}
			if (odp_cls_cos_pool(cos) != ODP_POOL_INVALID)
				pool = odp_cls_cos_pool(cos);
		}
		if (have && have->pool == pool) {
			pkt = (odp_packet_t)have;
		} else {
			/* into the CoS's pool (_odp_pktio_packet_to_pool) */
			if (pool == p->pool && used < nfresh && len <= own->buf) {
				pkt = (odp_packet_t)fresh[used++];
				pkt_init(PK(pkt), pool, len);
			} else {
				pkt = odp_packet_alloc(pool, len);
			}
			if (pkt != ODP_PACKET_INVALID)
				memcpy(PK(pkt)->data, s->stage + s->desc[k].offset, len);
			if (have)
				dead[ndead++] = (odp_packet_t)have;
			if (pkt == ODP_PACKET_INVALID) {
				/* loop.c:320-326: in_discards, and never counted
				 * as received nor handed to the CoS queue */
				const int counted = !(w & ODPG_OUT_ERROR);

				odpg_cls_pktio_count(hdl, counted ? -1 : 0,
						     counted ? -(int64_t)len : 0, 1, 0, 0);
				if (p->num_in > 1u && counted)
					qcount(p, s->qi[k], w, len, -1);
				if (q != ODP_QUEUE_INVALID)
					odpg_cls_queue_count(cos, q, -1, 0);
				continue;
			}
		}
		PK(pkt)->meta = s->meta[k];
		PK(pkt)->cos = cos;
		PK(pkt)->input = hdl;
		if (q == ODP_QUEUE_INVALID) {
			o->inqi[o->ninq] = s->qi[k];
			o->inq[o->ninq++] = pkt;
		} else {
			o->qp[o->nq] = pkt;
			o->qcos[o->nq] = cos;
			o->qq[o->nq++] = q;
		}
	}
	if (ndead)
		odp_packet_free_multi(dead, ndead);
	/* buffers taken and not used (longer packets, errors) go back */
	for (uint32_t k = used; k < nfresh; k++)
		pkt_init(fresh[k], p->pool, 0);
	odp_packet_free_multi((const odp_packet_t *)fresh + used, (int)(nfresh - used));
}

static void to_inq(rt_pktio_t *p, odp_packet_t pkts[], const uint8_t qi[], int nret);

/* a range's packets to their queues: runs of the same (CoS, queue) in one
 * enqueue each (_odp_cls_enq), the rest to the pktin queue, or to out[]
 * (DIRECT mode, *nret advanced) */
static void rx_commit(rt_pktio_t *p, rx_out_t *o, odp_packet_t out[], int *nret)
{
	for (int i = 0; i < o->nq;) {
		int j = i + 1;

		while (j < o->nq && o->qq[j] == o->qq[i] && o->qcos[j] == o->qcos[i])
			j++;
		cos_enq(o->qcos[i], o->qq[i], &o->qp[i], j - i);
		i = j;
	}
	if (out) {
		memcpy(out + *nret, o->inq, (size_t)o->ninq * sizeof(*out));
		*nret += o->ninq;
	} else {
		to_inq(p, o->inq, o->inqi, o->ninq);
	}
}

/* a completed burst delivered by this thread alone (DIRECT mode): the
 * binding released, the ranges handed over in order */
static void rx_deliver(rt_pktio_t *p, odp_pktio_t hdl, rx_slot_t *s, odp_packet_t pkts[],
		       int *nret)
{
	rx_out_t o;

	odpg_cls_pktio_recv_end(s->token);
	s->token = NULL;
	for (uint32_t k0 = 0; k0 < s->n; k0 += RX_CHUNK) {
		rx_deliver_range(p, hdl, s, k0, k0 + RX_CHUNK < s->n ? k0 + RX_CHUNK : s->n, &o);
		rx_commit(p, &o, pkts, nret);
	}
	s->n = 0;
}

static void prof_add(uint64_t bursts, uint64_t pkts, uint64_t t0, uint64_t t1, uint64_t t2,
		     uint64_t t3)
{
	/* the launch and delivery sides count from different threads */
	__atomic_fetch_add(&rxprof.bursts, bursts, __ATOMIC_RELAXED);
	__atomic_fetch_add(&rxprof.pkts, pkts, __ATOMIC_RELAXED);
	__atomic_fetch_add(&rxprof.stage_ns, t1 - t0, __ATOMIC_RELAXED);
	__atomic_fetch_add(&rxprof.gpu_ns, t2 - t1, __ATOMIC_RELAXED);
	__atomic_fetch_add(&rxprof.post_ns, t3 - t2, __ATOMIC_RELAXED);
}

/* DIRECT mode: one burst, launched and waited for. Returns the frames taken
 * (< 0 on a failed launch); *nret packets without a CoS queue in pkts[] */
static int rx_burst(rt_pktio_t *p, odp_pktio_t hdl, int queue, odp_packet_t pkts[], int num,
		    int *nret)
{
	rx_slot_t *s;

	*nret = 0;
	if (num > RT_BURST)
		num = RT_BURST;
	if (num <= 0 || !rt.init || !odpg_cls_pktio_started(hdl) || !(s = slot_get(p, 0)))
		return 0;
	const uint64_t t0 = rxprof.on > 0 ? prof_ns() : 0;
	const uint32_t n = rx_stage(p, s, (uint32_t)num, queue);

	if (!n)
		return 0;
	const uint64_t t1 = rxprof.on > 0 ? prof_ns() : 0;

	if (rx_launch(hdl, s))
		return -1;
	if (odpg_fence_wait(s->fence)) {
		ERR("receive burst failed on the GPU: dropped\n");
		odpg_cls_pktio_recv_end(s->token);
		s->token = NULL;
		rx_drop(s);
		return -1;
	}
	const uint64_t t2 = rxprof.on > 0 ? prof_ns() : 0;

	rx_deliver(p, hdl, s, pkts, nret);
	if (rxprof.on > 0)
		prof_add(1, n, t0, t1, t2, prof_ns());
	return (int)n;
}

/* a delivered burst's packets without a CoS queue onto the pktin event
 * queue of the input queue each came in on (runs of one queue in one
 * enqueue) */
static void to_inq(rt_pktio_t *p, odp_packet_t pkts[], const uint8_t qi[], int nret)
{
	const uint64_t t0 = rxprof.on > 0 ? prof_ns() : 0;

	for (int i = 0; i < nret;) {
		int j = i + 1;

		while (j < nret && qi[j] == qi[i])
			j++;
		rt_queue_t *q = qi[i] < RT_MAXQ ? p->inq[qi[i]] : NULL;

		int r = q ? odp_queue_enq_multi(q->hdl, (const odp_event_t *)&pkts[i], j - i) : 0;

		if (r < 0)
			r = 0;
		if (r < j - i)
			odp_packet_free_multi(&pkts[i + r], j - i - r);
		i = j;
	}
	if (rxprof.on > 0)
		__atomic_fetch_add(&rxprof.enq_ns, prof_ns() - t0, __ATOMIC_RELAXED);
}

/* QUEUE / SCHED mode, the delivery side. A burst whose fence has completed
 * is opened (rx_open, under rx_dlock: one thread) and then delivered in
 * chunks of RX_CHUNK packets by every thread that polls (rx_help, no lock):
 * a thread claims the next chunk, classifies its packets into pools
 * (rx_deliver_range), waits for the chunks before it to reach their queues
 * and hands its own over (rx_commit), so queue order is packet order. The
 * thread handing over the last chunk moves `delivered` on. */

/* the oldest burst in flight opened for delivery, if its fence has
 * completed (waited for with `drain`); a failed launch's burst is dropped.
 * Returns 1 when the oldest burst is open (now or before), else 0 */
static int rx_open(rt_pktio_t *p, int drain)
{
	for (;;) {
		const uint32_t d = p->delivered;

		if (d == __atomic_load_n(&p->launched, __ATOMIC_ACQUIRE))
			return 0;
		rx_slot_t *s = p->slot[d % RT_INFLIGHT];

		if (__atomic_load_n(&s->open, __ATOMIC_ACQUIRE)) {
			if ((uint32_t)(__atomic_load_n(&s->claimw, __ATOMIC_ACQUIRE) >> 32) == d)
				return 1;
			/* the slot's previous burst is still being closed (its
			 * last chunk's thread clears `open` after moving
			 * `delivered` on) */
			if (!drain)
				return 0;
			for (uint32_t sp = 0; __atomic_load_n(&s->open, __ATOMIC_ACQUIRE);)
				spin_wait(&sp);
			continue;
		}
		const int fs = drain ? (odpg_fence_wait(s->fence) ? -1 : 1) : odpg_fence_query(s->fence);

		if (fs == 0)
			return 0;
		const uint64_t t0 = rxprof.on > 0 ? prof_ns() : 0;

		odpg_cls_pktio_recv_end(s->token);
		s->token = NULL;
		if (rxprof.on > 0)
			__atomic_fetch_add(&rxprof.end_ns, prof_ns() - t0, __ATOMIC_RELAXED);
		if (fs < 0) {
			/* the launch failed: its verdicts were never written */
			ERR("receive burst failed on the GPU: dropped\n");
			rx_drop(s);
			__atomic_store_n(&p->delivered, d + 1u, __ATOMIC_RELEASE);
			continue;
		}
		s->nchunks = (s->n + RX_CHUNK - 1u) / RX_CHUNK;
		s->commit = 0;
		__atomic_store_n(&s->claimw, (uint64_t)d << 32, __ATOMIC_RELEASE);
		__atomic_store_n(&s->open, 1u, __ATOMIC_RELEASE);
		return 1;
	}
}

/* chunks of the oldest open burst, claimed one at a time until none is
 * left. Returns the frames this thread delivered */
static int rx_help(rt_pktio_t *p, odp_pktio_t hdl)
{
	const uint32_t d = __atomic_load_n(&p->delivered, __ATOMIC_ACQUIRE);
	int got = 0;

	if (d == __atomic_load_n(&p->launched, __ATOMIC_ACQUIRE))
		return 0;
	rx_slot_t *s = p->slot[d % RT_INFLIGHT];

	if (!s)
		return 0;
	__atomic_fetch_add(&s->busy, 1u, __ATOMIC_SEQ_CST);
	for (;;) {
		uint64_t cw = __atomic_load_n(&s->claimw, __ATOMIC_ACQUIRE);

		/* a slot reused for a later burst carries that burst's count */
		if (!__atomic_load_n(&s->open, __ATOMIC_ACQUIRE) || (uint32_t)(cw >> 32) != d ||
		    (uint32_t)cw >= s->nchunks)
			break;
		if (!__atomic_compare_exchange_n(&s->claimw, &cw, cw + 1u, false, __ATOMIC_ACQ_REL,
						 __ATOMIC_ACQUIRE))
			continue;
		const uint32_t c = (uint32_t)cw;
		const uint32_t k0 = c * RX_CHUNK, k1 = k0 + RX_CHUNK < s->n ? k0 + RX_CHUNK : s->n;
		const uint64_t t2 = rxprof.on > 0 ? prof_ns() : 0;
		rx_out_t o;

		rx_deliver_range(p, hdl, s, k0, k1, &o);
		for (uint32_t sp = 0; __atomic_load_n(&s->commit, __ATOMIC_ACQUIRE) != c;)
			spin_wait(&sp);
		rx_commit(p, &o, NULL, NULL);
		got += (int)(k1 - k0);
		if (c + 1u == s->nchunks) {
			/* `delivered` first: while `open` is still set nobody
			 * can open the burst a second time */
			s->n = 0;
			__atomic_store_n(&s->commit, c + 1u, __ATOMIC_RELEASE);
			__atomic_store_n(&p->delivered, d + 1u, __ATOMIC_RELEASE);
			__atomic_store_n(&s->open, 0u, __ATOMIC_RELEASE);
		} else {
			__atomic_store_n(&s->commit, c + 1u, __ATOMIC_RELEASE);
		}
		if (rxprof.on > 0)
			prof_add(0, 0, t2, t2, t2, prof_ns());
	}
	__atomic_fetch_sub(&s->busy, 1u, __ATOMIC_RELEASE);
	return got;
}

/* every completed burst (all of them with `drain`, waiting) delivered by
 * this thread, with whatever help others give (rx_dlock held) */
static int rx_deliver_done(rt_pktio_t *p, odp_pktio_t hdl, int drain)
{
	int got = 0;

	while (rx_open(p, drain)) {
		const uint32_t d = p->delivered;

		got += rx_help(p, hdl);
		/* the last chunks may still be with other threads */
		for (uint32_t sp = 0; __atomic_load_n(&p->delivered, __ATOMIC_ACQUIRE) == d;)
			spin_wait(&sp);
	}
	return got;
}

/* the launch side (rt.poll_lock held): stage and launch while slots are
 * free and frames wait */
static int rx_launch_more(rt_pktio_t *p, odp_pktio_t hdl)
{
	int got = 0;

	while (odpg_cls_pktio_started(hdl)) {
		const uint32_t l = p->launched;
		const uint32_t inflight = l - __atomic_load_n(&p->delivered, __ATOMIC_ACQUIRE);

		if (inflight >= RT_INFLIGHT ||
		    (p->loopdev && inflight && __atomic_load_n(&p->ring_n, __ATOMIC_RELAXED) < RT_BURST / 4u))
			break;
		rx_slot_t *s = slot_get(p, l % RT_INFLIGHT);

		if (!s)
			break;
		/* a thread that looked at the slot's previous burst late is out */
		for (uint32_t sp = 0; __atomic_load_n(&s->busy, __ATOMIC_ACQUIRE);)
			spin_wait(&sp);
		const uint64_t t0 = rxprof.on > 0 ? prof_ns() : 0;
		const uint32_t n = rx_stage(p, s, RT_BURST, -1);

		if (!n)
			break;
		const uint64_t t1 = rxprof.on > 0 ? prof_ns() : 0;

		if (rx_launch(hdl, s))
			break;
		if (rxprof.on > 0) {
			const uint64_t t2 = prof_ns();

			prof_add(1, n, t0, t1, t2, t2);
		}
		__atomic_store_n(&p->launched, l + 1u, __ATOMIC_RELEASE);
		got += (int)n;
	}
	return got;
}

/* both sides in one thread (rt.poll_lock held): QUEUE-mode fill, drain */
static int rx_to_inq(rt_pktio_t *p, odp_pktio_t hdl, int drain)
{
	const uint32_t i = (uint32_t)(p - rt.pktio);
	int got;

	if (!rt.init)
		return 0;
	pthread_mutex_lock(&rx_dlock[i]);
	got = rx_deliver_done(p, hdl, drain);
	pthread_mutex_unlock(&rx_dlock[i]);
	if (!drain)
		got += rx_launch_more(p, hdl);
	return got;
}

/* odp_pktio_stop: the bursts in flight are delivered (they were received
 * before the stop) */
void odpg_rt_pktio_drain(odp_pktio_t hdl)
{
	pthread_mutex_lock(&rt.poll_lock);
	rt_pktio_t *p = get_rt_pktio(hdl);

	if (p)
		rx_to_inq(p, hdl, 1);
	pthread_mutex_unlock(&rt.poll_lock);
}

static void pktin_queue_fill(odp_pktio_t hdl)
{
	pthread_mutex_lock(&rt.poll_lock);
	rt_pktio_t *p = get_rt_pktio(hdl);

	if (p && p->in_mode == ODP_PKTIN_MODE_QUEUE)
		rx_to_inq(p, hdl, 0);
	pthread_mutex_unlock(&rt.poll_lock);
}

/* one burst of every SCHED-mode pktio (the scheduler's pktin poll).
 * Returns the frames taken (0: nothing waiting). */
static int poll_input(void)
{
	int got = 0;

	if (!rt.init)
		return 0;
	/* the delivery side: a completed burst is opened by one thread
	 * (rx_dlock) and its chunks delivered by every polling thread; a
	 * thread counts itself in rx_helpers before it looks at the pktio,
	 * which close waits out (the counts and busy flag are read first, not
	 * the locks' lines written) */
	for (int i = 0; i < RT_MAX_PKTIO; i++) {
		rt_pktio_t *p = &rt.pktio[i];
		const odp_pktio_t hdl = (odp_pktio_t)(uintptr_t)(i + 1);

		if (!p->valid || p->in_mode != ODP_PKTIN_MODE_SCHED ||
		    __atomic_load_n(&p->launched, __ATOMIC_RELAXED) ==
			    __atomic_load_n(&p->delivered, __ATOMIC_RELAXED))
			continue;
		__atomic_fetch_add(&rx_helpers[i], 1u, __ATOMIC_SEQ_CST);
		for (int it = 0; it < RT_INFLIGHT && __atomic_load_n(&p->valid, __ATOMIC_SEQ_CST) &&
				 p->in_mode == ODP_PKTIN_MODE_SCHED; it++) {
			const uint32_t d = __atomic_load_n(&p->delivered, __ATOMIC_ACQUIRE);

			if (d == __atomic_load_n(&p->launched, __ATOMIC_ACQUIRE))
				break;
			if (!__atomic_load_n(&p->slot[d % RT_INFLIGHT]->open, __ATOMIC_ACQUIRE)) {
				int opened = 0;

				if (__atomic_load_n(&rx_dbusy[i], __ATOMIC_RELAXED) ||
				    pthread_mutex_trylock(&rx_dlock[i]))
					break;
				__atomic_store_n(&rx_dbusy[i], 1, __ATOMIC_RELAXED);
				opened = rx_open(p, 0);
				__atomic_store_n(&rx_dbusy[i], 0, __ATOMIC_RELAXED);
				pthread_mutex_unlock(&rx_dlock[i]);
				if (!opened)
					break;
			}
			const int n = rx_help(p, hdl);

			got += n;
			if (!n)
				break;
		}
		__atomic_fetch_sub(&rx_helpers[i], 1u, __ATOMIC_RELEASE);
	}
	/* the launch side: another thread at the same time */
	if (__atomic_load_n(&rt.polling, __ATOMIC_RELAXED) || pthread_mutex_trylock(&rt.poll_lock))
		return got;
	__atomic_store_n(&rt.polling, 1, __ATOMIC_RELAXED);
	for (int i = 0; i < RT_MAX_PKTIO; i++) {
		rt_pktio_t *p = &rt.pktio[i];

		if (p->valid && p->in_mode == ODP_PKTIN_MODE_SCHED)
			got += rx_launch_more(p, (odp_pktio_t)(uintptr_t)(i + 1));
	}
	__atomic_store_n(&rt.polling, 0, __ATOMIC_RELAXED);
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
	int n = 0;

	for (uint32_t q = 0; q < p->num_in && p->inq[q]; q++, n++)
		if (queues && n < num)
			queues[n] = p->inq[q]->hdl;
	return n;
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
	/* a loop device: one launch classifies everything waiting (up to
	 * RT_BURST), as a NIC fills its receive ring; what the caller did not
	 * ask for is handed out by the next calls, in order, without a launch
	 * of their own (its frames already sit in packets). A capture is read
	 * `num` frames at a time, as pcap_recv does: each of its frames needs
	 * a packet from the pool, and frames read ahead would be dropped when
	 * the pool is short */
	const int qi = queue.index;

	if (num > 0 && !p->ahead[qi]) {
		odp_packet_t got[RT_BURST];
		const int rc = rx_burst(p, queue.pktio, p->loopdev ? qi : -1, got,
					p->loopdev ? RT_BURST : num, &nret);

		if (rc < 0) {
			pthread_mutex_unlock(&rt.poll_lock);
			return -1;
		}
		for (int k = nret - 1; k >= 0; k--) {
			rt_pkt_t *x = (rt_pkt_t *)got[k];

			x->next = p->ahead[qi];
			p->ahead[qi] = x;
			if (!x->next)
				p->ahead_tail[qi] = x;
		}
	}
	nret = 0;
	while (nret < num && p->ahead[qi]) {
		rt_pkt_t *x = p->ahead[qi];

		p->ahead[qi] = x->next;
		x->next = NULL;
		packets[nret++] = (odp_packet_t)x;
	}
	if (!p->ahead[qi])
		p->ahead_tail[qi] = NULL;
	pthread_mutex_unlock(&rt.poll_lock);
	return nret;
}

/* per-queue counters (loopback_pktin_stats / loopback_pktout_stats,
 * pktio/loop.c:761-785): with one input (output) queue it carries the
 * interface's counters; a device with several keeps per-queue counts
 * (qcount at delivery, the send path) */
static int in_queue_stats(odp_pktio_t pktio, uint32_t index, odp_pktin_queue_stats_t *st)
{
	odp_pktio_stats_t s;
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (p && st && p->num_in > 1u && index < p->num_in) {
		memset(st, 0, sizeof(*st));
		st->octets = __atomic_load_n(&p->qst[index].in_octets, __ATOMIC_RELAXED);
		st->packets = __atomic_load_n(&p->qst[index].in_packets, __ATOMIC_RELAXED);
		st->discards = __atomic_load_n(&p->qst[index].in_discards, __ATOMIC_RELAXED);
		st->errors = __atomic_load_n(&p->qst[index].in_errors, __ATOMIC_RELAXED);
		return 0;
	}
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
	rt_pktio_t *p = get_rt_pktio(pktio);

	if (p && st && p->num_out > 1u && index < p->num_out) {
		memset(st, 0, sizeof(*st));
		st->octets = __atomic_load_n(&p->qst[index].out_octets, __ATOMIC_RELAXED);
		st->packets = __atomic_load_n(&p->qst[index].out_packets, __ATOMIC_RELAXED);
		return 0;
	}
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

	if (!p || (p->in_mode != ODP_PKTIN_MODE_SCHED && p->in_mode != ODP_PKTIN_MODE_QUEUE))
		return -1;
	for (uint32_t q = 0; q < p->num_in; q++)
		if (p->inq[q] && queue == p->inq[q]->hdl)
			return in_queue_stats(pktio, q, stats);
	return -1;
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
	capa->max_queues = QCHUNK * QCHUNKS;
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
	/* the list is walked under the read side of sched_rw: a destroy
	 * unlinks under the write side before the object is reused */
	static __thread uint32_t rr;   /* this thread's round-robin start */

	/* nothing queued: the walk (and the lock's shared line) skipped */
	if (!__atomic_load_n(&rt.sched_n, __ATOMIC_ACQUIRE))
		return 0;
	pthread_rwlock_rdlock(&sched_rw);
	rt_queue_t *list = rt.sched;
	const uint32_t skip = rr++;
	int nq = 0, n = 0;

	for (rt_queue_t *q = list; q; q = q->next_sched)
		nq++;
	for (int pass = 0; pass < nq && !n; pass++) {
		rt_queue_t *q = list;

		for (uint32_t s = (skip + (uint32_t)pass) % (uint32_t)nq; s; s--)
			q = q->next_sched;
		if (q->dead)
			continue;
		n = deq_multi(q, ev, num);
		if (n && from)
			*from = q->hdl;
	}
	pthread_rwlock_unlock(&sched_rw);
	return n;
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
	capa->max_input_queues = get_rt_pktio(pktio)->loopdev ? RT_MAXQ : 1u;
	capa->max_output_queues = RT_MAXQ;
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
	if (param->num_queues == 0 || param->num_queues > RT_MAXQ) {
		ERR("pktio %" PRIu64 ": invalid number of output queues\n",
		    (uint64_t)(uintptr_t)pktio);
		return -1;
	}
	p->num_out = param->num_queues;
	for (uint32_t q = 0; q < RT_MAXQ; q++)
		pktio_queue_kill(&p->outq[q]);
	if (p->out_mode != ODP_PKTOUT_MODE_QUEUE)
		return 0;
	odp_queue_param_init(&qp);
	for (uint32_t q = 0; q < p->num_out; q++) {
		snprintf(name, sizeof(name), "odp-pktout-%u-%u", (unsigned)(uintptr_t)pktio, q);
		p->outq[q] = queue_new(name, &qp);
		if (!p->outq[q])
			return -1;
		p->outq[q]->pktout = pktio;
		p->outq[q]->pindex = q;
	}
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
	int n = 0;

	for (uint32_t q = 0; q < p->num_out && p->outq[q]; q++, n++)
		if (queues && n < num)
			queues[n] = p->outq[q]->hdl;
	return n;
}

/* odp_hash_crc32c (Castagnoli, reflected, no final inversion; the table
 * built once) */
static uint32_t crc32c_tbl[256];
static pthread_once_t crc32c_once = PTHREAD_ONCE_INIT;

static void crc32c_init(void)
{
	for (uint32_t i = 0; i < 256; i++) {
		uint32_t c = i;

		for (int k = 0; k < 8; k++)
			c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
		crc32c_tbl[i] = c;
	}
}

static uint32_t crc32c(const uint8_t *d, uint32_t len, uint32_t crc)
{
	pthread_once(&crc32c_once, crc32c_init);
	for (uint32_t i = 0; i < len; i++)
		crc = crc32c_tbl[(crc ^ d[i]) & 0xffu] ^ (crc >> 8);
	return crc;
}

/* get_dest_queue (pktio/loop.c:472-523): the input queue a transmitted
 * packet goes to. Without hashing the queue of the pktout index; with it
 * the crc32c of the UDP / TCP ports and the IPv4 / IPv6 addresses the
 * packet's parse result names (those whose header lies inside the packet),
 * modulo the input queues. The GPU batch form is odpg_tx_prepare
 * (include/odpg_tx.h); one send burst is too small for a launch. */
static uint32_t loop_dest_queue(const rt_pktio_t *p, const rt_pkt_t *k, uint32_t index)
{
	const uint32_t nq = p->num_in ? p->num_in : 1u, h = p->hash_bits;
	const uint64_t inf = k->meta.input_flags;
	uint8_t data[2 * 2 + 2 * 16];
	uint32_t n = 0, off;

	if (h == 0u)
		return index % nq;
	off = k->meta.l4_offset;
	if (off != ODP_PACKET_OFFSET_INVALID) {
		if ((h & 0x9u) && ((inf >> IF_UDP) & 1u)) {          /* ipv4_udp | ipv6_udp */
			if (off + 8u <= k->len) {
				memcpy(data, k->data + off, 4);     /* source, destination port */
				n = 4;
			}
		} else if ((h & 0x12u) && ((inf >> IF_TCP) & 1u)) {  /* ipv4_tcp | ipv6_tcp */
			if (off + 20u <= k->len) {
				memcpy(data, k->data + off, 4);
				n = 4;
			}
		}
	}
	off = k->meta.l3_offset;
	if (off != ODP_PACKET_OFFSET_INVALID) {
		if ((h & 0x4u) && ((inf >> IF_IPV4) & 1u)) {
			if (off + 20u <= k->len) {
				memcpy(data + n, k->data + off + 12u, 8);   /* source, destination */
				n += 8;
			}
		} else if ((h & 0x20u) && ((inf >> IF_IPV6) & 1u)) {
			if (off + 40u <= k->len) {
				memcpy(data + n, k->data + off + 8u, 32);
				n += 32;
			}
		}
	}
	return crc32c(data, n, 0u) % nq;
}

/* transmit (loopback_send, pktio/loop.c:525-580): on a loop device the
 * packets go back to its input, each to the input queue get_dest_queue
 * picks, up to the first one over the MTU (-1 if that is the first); the
 * pcap device here has no output file, so its packets are consumed.
 * Counted as out_packets / out_octets (per output queue `index` on a device
 * with several). */
static int pktout_send_impl(odp_pktio_t pktio, uint32_t index, const odp_packet_t packets[],
			    int num)
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
		uint8_t qd[RT_BURST];
		int full = 0;

		/* the picks read the packets' headers: before the lock */
		if (p->num_in > 1u) {
			if (n > RT_BURST)
				n = RT_BURST;
			octets = 0;
			for (int i = 0; i < n; i++) {
				qd[i] = (uint8_t)loop_dest_queue(p, PK(packets[i]), index);
				octets += PK(packets[i])->len;
			}
		}
		pthread_mutex_lock(&p->ring_lock);
		if (p->num_in > 1u) {
			/* runs of one queue in one push; the packets of a run go
			 * in whole or not at all (no memory for the ring) */
			int i = 0;

			while (i < n && !full) {
				int j = i + 1;

				while (j < n && qd[j] == qd[i])
					j++;
				full = pring_push(&p->ring[qd[i]], (void *const *)&packets[i],
						  (uint32_t)(j - i));
				if (!full)
					i = j;
			}
			if (full) {             /* sent: the packets before the run */
				octets = 0;
				for (int k = 0; k < i; k++)
					octets += PK(packets[k])->len;
				n = i;
			}
		} else {
			full = pring_push(&p->ring[0], (void *const *)packets, (uint32_t)n);
			if (full)
				n = 0;
		}
		__atomic_store_n(&p->ring_n, p->ring_n + (uint32_t)n, __ATOMIC_RELEASE);
		pthread_mutex_unlock(&p->ring_lock);
		if (!n)
			return 0;       /* no memory for the ring: nothing sent */
	} else {
		odp_packet_free_multi(packets, n);
	}
	odpg_cls_pktio_count(pktio, 0, 0, 0, (uint64_t)n, octets);
	if (p->num_out > 1u && index < RT_MAXQ) {
		__atomic_fetch_add(&p->qst[index].out_packets, (uint64_t)n, __ATOMIC_RELAXED);
		__atomic_fetch_add(&p->qst[index].out_octets, octets, __ATOMIC_RELAXED);
	}
	return n;
}

int odp_pktout_send(odp_pktout_queue_t queue, const odp_packet_t packets[], int num)
{
	rt_pktio_t *p = get_rt_pktio(queue.pktio);

	if (!p || p->out_mode != ODP_PKTOUT_MODE_DIRECT || queue.index < 0 ||
	    (uint32_t)queue.index >= p->num_out)
		return -1;
	return pktout_send_impl(queue.pktio, (uint32_t)queue.index, packets, num);
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

	if (!p || p->out_mode != ODP_PKTOUT_MODE_QUEUE)
		return -1;
	for (uint32_t q = 0; q < p->num_out; q++)
		if (p->outq[q] && queue == p->outq[q]->hdl)
			return out_queue_stats(pktio, q, stats);
	return -1;
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

/* "aa:bb:cc:dd:ee:ff" (helper/eth.c odph_eth_addr_parse: sscanf, trailing
 * characters ignored) */
int odph_eth_addr_parse(odph_ethaddr_t *mac, const char *str)
{
	unsigned b[6];

	if (!str || sscanf(str, "%x:%x:%x:%x:%x:%x", &b[0], &b[1], &b[2], &b[3], &b[4],
			   &b[5]) != 6)
		return -1;
	for (int i = 0; i < 6; i++) {
		if (b[i] > 255)
			return -1;
		mac->addr[i] = (uint8_t)b[i];
	}
	return 0;
}

/* "a.b.c.d" in host byte order (helper/ip.c odph_ipv4_addr_parse: sscanf,
 * trailing characters ignored) */
int odph_ipv4_addr_parse(uint32_t *ip_addr, const char *str)
{
	unsigned b[4];

	if (!str || sscanf(str, "%u.%u.%u.%u", &b[0], &b[1], &b[2], &b[3]) != 4)
		return -1;
	for (int i = 0; i < 4; i++)
		if (b[i] > 255)
			return -1;
	*ip_addr = (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3];
	return 0;
}

/* odph_ipv4_csum (helper ip.h:98-131): the header's ihl * 4 bytes with the
 * checksum field zeroed; < 0 when ihl < 5 or the header leaves the packet */
static int ipv4_csum(odp_packet_t pkt, uint32_t l3, uint16_t *sum)
{
	uint8_t hdr[60];
	uint32_t hl;

	if (l3 == ODP_PACKET_OFFSET_INVALID ||
	    odp_packet_copy_to_mem(pkt, l3, ODPH_IPV4HDR_LEN, hdr))
		return -1;
	hl = (uint32_t)ODPH_IPV4HDR_IHL(hdr[0]) * 4u;
	if (hl < ODPH_IPV4HDR_LEN)
		return -1;
	if (hl > ODPH_IPV4HDR_LEN &&
	    odp_packet_copy_to_mem(pkt, l3 + ODPH_IPV4HDR_LEN, hl - ODPH_IPV4HDR_LEN,
				   hdr + ODPH_IPV4HDR_LEN))
		return -1;
	hdr[ODPH_IPV4HDR_CSUM_OFFSET] = hdr[ODPH_IPV4HDR_CSUM_OFFSET + 1] = 0;
	*sum = (uint16_t)~odp_chksum_ones_comp16(hdr, hl);
	return 0;
}

int odph_ipv4_csum_update(odp_packet_t pkt)
{
	const uint32_t l3 = odp_packet_l3_offset(pkt);
	uint16_t sum;

	if (ipv4_csum(pkt, l3, &sum))
		return -1;
	return odp_packet_copy_from_mem(pkt, l3 + ODPH_IPV4HDR_CSUM_OFFSET, 2, &sum);
}

int odph_ipv4_csum_valid(odp_packet_t pkt)
{
	const uint32_t l3 = odp_packet_l3_offset(pkt);
	uint16_t sum, cur;

	if (ipv4_csum(pkt, l3, &sum) ||
	    odp_packet_copy_to_mem(pkt, l3 + ODPH_IPV4HDR_CSUM_OFFSET, 2, &cur))
		return 0;
	return sum == cur;
}

char *odph_strcpy(char *dst, const char *src, size_t sz)
{
	if (sz == 0)
		return dst;
	strncpy(dst, src, sz - 1);
	dst[sz - 1] = 0;
	return dst;
}
