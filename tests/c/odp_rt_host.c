/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Host-only checks of the ODP runtime subset (odp_amd/csrc/odp_rt.c) under
 * thread contention, no GPU: the two-phase barrier re-entered many times
 * with a shared counter checked between phases (test/validation/api/barrier
 * does the same), thread ids handed out and given back by concurrent
 * odp_init_local / odp_term_local (unique, below ODP_THREAD_COUNT_MAX), named
 * shm reserve / lookup / free (a second free fails cleanly), the packet
 * pool (buffers through per-thread caches, the num limit, long packets,
 * destroy / re-create with a packet outstanding), the queue registry:
 * create / destroy cycles beyond its slot count, stale handles refused, the
 * queues' event rings (growth, wrap, FIFO order per producer with several
 * producers and consumers, through dequeue and the scheduler), and scheduled queues created and destroyed while other threads
 * schedule. Prints PASS or the first failure. Run by tests/test_odp_rt.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <odp_api.h>

#define NT 8
static int fails;

#define CHECK(c, ...)                                                            \
	do {                                                                     \
		if (!(c)) {                                                      \
			printf("FAIL %s:%d: ", __FILE__, __LINE__);              \
			printf(__VA_ARGS__);                                     \
			printf("\n");                                            \
			__atomic_fetch_add(&fails, 1, __ATOMIC_RELAXED);         \
		}                                                                \
	} while (0)

/* ---- barrier ---------------------------------------------------------------- */
static odp_barrier_t barr;
static uint32_t shared_count;
#define BAR_ITERS 20000

static void *bar_thread(void *arg)
{
	(void)arg;
	for (uint32_t it = 0; it < BAR_ITERS && !fails; it++) {
		__atomic_fetch_add(&shared_count, 1, __ATOMIC_RELAXED);
		odp_barrier_wait(&barr);
		const uint32_t v = __atomic_load_n(&shared_count, __ATOMIC_RELAXED);

		CHECK(v == (it + 1) * NT, "barrier iteration %u: count %u, want %u", it, v,
		      (it + 1) * NT);
		odp_barrier_wait(&barr);
	}
	return NULL;
}

/* ---- thread ids --------------------------------------------------------------- */
static int owner[ODP_THREAD_COUNT_MAX];

static void *id_thread(void *arg)
{
	const int me = (int)(intptr_t)arg + 1;

	for (int it = 0; it < 3000 && !fails; it++) {
		CHECK(odp_init_local((odp_instance_t)0, ODP_THREAD_WORKER) == 0, "init_local");
		const int id = odp_thread_id();

		CHECK(id >= 0 && id < ODP_THREAD_COUNT_MAX, "thread id %d out of range", id);
		if (id < 0 || id >= ODP_THREAD_COUNT_MAX)
			break;
		int z = 0;

		CHECK(__atomic_compare_exchange_n(&owner[id], &z, me, 0, __ATOMIC_ACQ_REL,
						  __ATOMIC_ACQUIRE),
		      "thread id %d handed to two live threads", id);
		CHECK(odp_thread_count() <= NT, "thread count %d", odp_thread_count());
		__atomic_store_n(&owner[id], 0, __ATOMIC_RELEASE);
		CHECK(odp_term_local() == 0, "term_local");
	}
	return NULL;
}

/* ---- packet pool: buffers through the per-thread caches ------------------------- */
static odp_pool_t churn_pool;

static void *pool_thread(void *arg)
{
	(void)arg;
	odp_packet_t held[48];

	for (int it = 0; it < 20000 && !fails; it++) {
		int n = 0;

		for (; n < 48; n++) {
			held[n] = odp_packet_alloc(churn_pool, 60 + (n & 7));
			if (held[n] == ODP_PACKET_INVALID)
				break;
			((uint8_t *)odp_packet_data(held[n]))[0] = (uint8_t)n;
		}
		for (int k = 0; k < n; k++) {
			CHECK(((uint8_t *)odp_packet_data(held[k]))[0] == (uint8_t)k &&
			      odp_packet_len(held[k]) == 60u + (k & 7), "packet %d overwritten", k);
			odp_packet_free(held[k]);
		}
	}
	return NULL;
}

/* ---- a small pool: allocated by one thread, freed by another ------------------- */
static odp_packet_t xfer[32];

static void *free_thread(void *arg)
{
	(void)arg;
	for (int k = 0; k < 32; k++)
		odp_packet_free(xfer[k]);
	return NULL;
}

/* ---- scheduled queues created / destroyed under schedulers -------------------- */
static int sched_stop;

static void *sched_thread(void *arg)
{
	(void)arg;
	while (!__atomic_load_n(&sched_stop, __ATOMIC_ACQUIRE)) {
		odp_event_t ev[4];
		odp_queue_t from;

		CHECK(odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 4) == 0,
		      "events from empty queues");
	}
	return NULL;
}

static void *churn_thread(void *arg)
{
	(void)arg;
	odp_queue_param_t qp;

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	for (int it = 0; it < 20000 && !fails; it++) {
		odp_queue_t q = odp_queue_create("sq", &qp);

		CHECK(q != ODP_QUEUE_INVALID, "sched queue create %d", it);
		CHECK(odp_queue_destroy(q) == 0, "sched queue destroy %d", it);
	}
	return NULL;
}

/* ---- queue rings: producers and consumers of tagged handles ---------------- */
#define QP 4                       /* producers (and consumers) */
#define QN 200000                  /* events per producer */
static odp_queue_t fifo;
static int fifo_sched;             /* consumers call the scheduler */
static uint32_t fifo_got;
static uint8_t *fifo_seen;

static odp_event_t tag_ev(uint32_t p, uint32_t i)
{
	return (odp_event_t)(uintptr_t)(((uint64_t)(p + 1u) << 32) | i);
}

static void *fifo_prod(void *arg)
{
	const uint32_t p = (uint32_t)(intptr_t)arg;
	odp_event_t ev[37];

	for (uint32_t i = 0; i < QN && !fails;) {
		const uint32_t b = 1u + (i * 7u + p) % 37u, k = b < QN - i ? b : QN - i;

		for (uint32_t j = 0; j < k; j++)
			ev[j] = tag_ev(p, i + j);
		CHECK(odp_queue_enq_multi(fifo, ev, (int)k) == (int)k, "enq %u", i);
		i += k;
	}
	return NULL;
}

static void *fifo_cons(void *arg)
{
	uint32_t last[QP];
	odp_event_t ev[29];

	(void)arg;
	memset(last, 0xff, sizeof(last));
	while (__atomic_load_n(&fifo_got, __ATOMIC_RELAXED) < QP * QN && !fails) {
		odp_queue_t from = ODP_QUEUE_INVALID;
		const int n = fifo_sched ? odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 29)
					 : odp_queue_deq_multi(fifo, ev, 29);

		CHECK(n >= 0 && (!n || !fifo_sched || from == fifo), "dequeue");
		for (int j = 0; j < n; j++) {
			const uint64_t v = (uint64_t)(uintptr_t)ev[j];
			const uint32_t p = (uint32_t)(v >> 32) - 1u, i = (uint32_t)v;

			CHECK(p < QP && i < QN, "a handle never enqueued: %llx", (unsigned long long)v);
			if (p >= QP || i >= QN)
				break;
			CHECK(last[p] == 0xffffffffu || i > last[p],
			      "producer %u: %u after %u (FIFO order)", p, i, last[p]);
			CHECK(!__atomic_exchange_n(&fifo_seen[p * QN + i], 1, __ATOMIC_RELAXED),
			      "event %u.%u twice", p, i);
			last[p] = i;
		}
		if (n > 0)
			__atomic_fetch_add(&fifo_got, (uint32_t)n, __ATOMIC_RELAXED);
	}
	return NULL;
}

/* QP producers and QP consumers through one queue (plain: dequeue; SCHED:
 * the scheduler), every event exactly once and each producer's in order */
static void fifo_run(int sched)
{
	odp_queue_param_t qp;
	pthread_t t[2 * QP];

	odp_queue_param_init(&qp);
	qp.type = sched ? ODP_QUEUE_TYPE_SCHED : ODP_QUEUE_TYPE_PLAIN;
	fifo = odp_queue_create("fifo", &qp);
	fifo_sched = sched;
	fifo_got = 0;
	fifo_seen = calloc((size_t)QP * QN, 1);
	CHECK(fifo != ODP_QUEUE_INVALID && fifo_seen, "fifo queue");
	for (int i = 0; i < QP; i++) {
		pthread_create(&t[i], NULL, fifo_prod, (void *)(intptr_t)i);
		pthread_create(&t[QP + i], NULL, fifo_cons, NULL);
	}
	for (int i = 0; i < 2 * QP; i++)
		pthread_join(t[i], NULL);
	CHECK(fifo_got == QP * QN, "%u of %u events", fifo_got, QP * QN);
	CHECK(odp_queue_deq(fifo) == ODP_EVENT_INVALID, "events left");
	CHECK(odp_queue_destroy(fifo) == 0, "fifo destroy");
	free(fifo_seen);
}

static void run(void *(*fn)(void *), int n)
{
	pthread_t t[NT];

	for (int i = 0; i < n; i++)
		pthread_create(&t[i], NULL, fn, (void *)(intptr_t)i);
	for (int i = 0; i < n; i++)
		pthread_join(t[i], NULL);
}

int main(void)
{
	/* barrier */
	odp_barrier_init(&barr, NT);
	run(bar_thread, NT);
	printf("barrier: %d x %d waits\n", NT, 2 * BAR_ITERS);

	/* thread ids */
	run(id_thread, NT);
	CHECK(odp_thread_count() == 0, "thread count after every term_local: %d",
	      odp_thread_count());
	printf("thread ids: %d threads x 3000 init/term\n", NT);

	/* shm */
	odp_shm_t a = odp_shm_reserve("blk_a", 100, 64, 0);
	odp_shm_t b = odp_shm_reserve("blk_b", 4096, 4096, 0);

	CHECK(a != ODP_SHM_INVALID && b != ODP_SHM_INVALID, "shm reserve");
	CHECK(odp_shm_lookup("blk_a") == a && odp_shm_lookup("blk_b") == b, "shm lookup");
	CHECK(odp_shm_addr(a) && ((uintptr_t)odp_shm_addr(b) & 4095u) == 0, "shm addr / align");
	memset(odp_shm_addr(a), 0x5a, 100);
	CHECK(odp_shm_free(a) == 0, "shm free");
	CHECK(odp_shm_lookup("blk_a") == ODP_SHM_INVALID, "lookup after free");
	CHECK(odp_shm_free(b) == 0 && odp_shm_free(b) == -1, "second free of a block");
	printf("shm: reserve / lookup / free\n");

	/* packet pool: the num limit, buffers shared by threads, long packets,
	 * destroy / re-create with a packet outstanding */
	odp_pool_param_t pp;

	odp_pool_param_init(&pp);
	pp.type = ODP_POOL_PACKET;
	pp.pkt.num = 1024;
	pp.pkt.len = 128;
	pp.pkt.seg_len = 128;
	churn_pool = odp_pool_create("churn", &pp);
	CHECK(churn_pool != ODP_POOL_INVALID, "pool create");
	run(pool_thread, NT);
	{
		static odp_packet_t all[1100];
		int n = 0;

		/* the pool's num, less what the other threads' caches hold */
		while (n < 1100 && (all[n] = odp_packet_alloc(churn_pool, 64)) != ODP_PACKET_INVALID)
			n++;
		CHECK(n <= 1024 && n >= 1024 - NT * 64, "num limit: %d packets", n);
		odp_packet_free(all[--n]);
		odp_packet_t big = odp_packet_alloc(churn_pool, 4000);   /* its own data */

		CHECK(big != ODP_PACKET_INVALID && odp_packet_len(big) == 4000u, "long packet");
		memset(odp_packet_data(big), 1, 4000);
		CHECK(odp_packet_alloc(churn_pool, 64) == ODP_PACKET_INVALID, "num limit with a long packet");
		odp_packet_free(big);
		/* freed in one pass (the cache filled, the rest onto the stack),
		 * every one allocatable again */
		odp_packet_free_multi(all, n);
		int m = 0;

		while (m < n && (all[m] = odp_packet_alloc(churn_pool, 64)) != ODP_PACKET_INVALID)
			m++;
		CHECK(m == n, "after odp_packet_free_multi: %d of %d packets", m, n);
		odp_packet_free_multi(all, m);
		odp_packet_t stale = odp_packet_alloc(churn_pool, 64);

		CHECK(odp_pool_destroy(churn_pool) == 0, "pool destroy");
		churn_pool = odp_pool_create("churn2", &pp);
		odp_packet_free(stale);                 /* its pool is gone: ignored */
		odp_packet_t fresh = odp_packet_alloc(churn_pool, 64);

		CHECK(fresh != ODP_PACKET_INVALID && fresh != stale, "re-created pool hands out its own");
		odp_packet_free(fresh);
		CHECK(odp_pool_destroy(churn_pool) == 0, "pool destroy 2");
	}
	printf("pool: %d threads x 20000 x 48 alloc/free, limits, re-create\n", NT);

	/* a 32-buffer pool whose buffers one thread allocates and another frees
	 * (a producer and a worker): the freeing thread's cache must not strand
	 * them, every buffer is allocatable again */
	{
		odp_pool_param_init(&pp);
		pp.type = ODP_POOL_PACKET;
		pp.pkt.num = 32;
		pp.pkt.len = 128;
		odp_pool_t small = odp_pool_create("small", &pp);

		CHECK(small != ODP_POOL_INVALID, "small pool");
		for (int round = 0; round < 3; round++) {
			int n = 0;

			for (; n < 32; n++)
				if ((xfer[n] = odp_packet_alloc(small, 64)) == ODP_PACKET_INVALID)
					break;
			CHECK(n == 32, "round %d: %d of 32 buffers", round, n);
			if (n < 32)
				break;
			run(free_thread, 1);
		}
		CHECK(odp_pool_destroy(small) == 0, "small pool destroy");
		printf("pool: 32 buffers, allocated here and freed by another thread, 3 rounds\n");
	}

	/* pkt.cache_size 0: no per-thread caches, so after the churn threads
	 * every buffer is allocatable here (the reference's set_pool_cache_size
	 * honours 0 the same way) */
	{
		odp_pool_capability_t capa;
		static odp_packet_t all2[1100];
		int n = 0;

		CHECK(odp_pool_capability(&capa) == 0 && capa.pkt.min_cache_size == 0 &&
		      capa.pkt.max_cache_size >= 256, "pool capability cache sizes");
		odp_pool_param_init(&pp);
		CHECK(pp.pkt.cache_size == 256, "default cache_size %u", pp.pkt.cache_size);
		pp.type = ODP_POOL_PACKET;
		pp.pkt.num = 1024;
		pp.pkt.len = 128;
		pp.pkt.seg_len = 128;
		pp.pkt.cache_size = 0;
		churn_pool = odp_pool_create("nocache", &pp);
		CHECK(churn_pool != ODP_POOL_INVALID, "pool without caches");
		run(pool_thread, NT);
		while (n < 1100 && (all2[n] = odp_packet_alloc(churn_pool, 64)) != ODP_PACKET_INVALID)
			n++;
		CHECK(n == 1024, "cache_size 0: %d of 1024 packets after the churn", n);
		odp_packet_free_multi(all2, n);
		CHECK(odp_pool_destroy(churn_pool) == 0, "nocache pool destroy");
		printf("pool: cache_size 0, all 1024 buffers allocatable after %d threads' churn\n", NT);
	}

	/* queue registry: more create / destroy cycles than slots */
	odp_queue_t first = odp_queue_create("q", NULL), q = first;

	CHECK(odp_queue_destroy(first) == 0, "destroy");
	CHECK(odp_queue_destroy(first) == -1, "second destroy of a queue");
	for (uint32_t it = 0; it < (1u << 21) && !fails; it++) {
		q = odp_queue_create("q", NULL);
		CHECK(q != ODP_QUEUE_INVALID, "create %u", it);
		CHECK(odp_queue_destroy(q) == 0, "destroy %u", it);
	}
	CHECK(odp_queue_enq(first, ODP_EVENT_INVALID) == -1 &&
	      odp_queue_deq(first) == ODP_EVENT_INVALID, "a stale handle still resolves");
	odp_queue_t live = odp_queue_create("live", NULL);

	CHECK(live != ODP_QUEUE_INVALID && live != first && live != q, "handle reuse");
	CHECK(odp_queue_destroy(live) == 0, "destroy live");
	printf("queues: 2^21 create/destroy cycles\n");

	/* a queue's ring: growth and wrap in FIFO order, one thread */
	{
		odp_queue_t f = odp_queue_create("ring", NULL);
		uint32_t wr = 0, rd = 0;

		for (uint32_t it = 0; it < 20000 && !fails; it++) {
			odp_event_t ev[300];
			const uint32_t k = 1u + (it * 131u) % 300u, d = 1u + (it * 97u) % 290u;

			for (uint32_t j = 0; j < k; j++)
				ev[j] = tag_ev(0, wr++);
			CHECK(odp_queue_enq_multi(f, ev, (int)k) == (int)k, "ring enq");
			const int n = odp_queue_deq_multi(f, ev, (int)d);

			for (int j = 0; j < n; j++)
				CHECK(ev[j] == tag_ev(0, rd + (uint32_t)j), "ring order at %u", rd);
			rd += (uint32_t)n;
		}
		CHECK(odp_queue_destroy(f) == -1, "a non-empty queue destroyed");
		for (int n; (n = odp_queue_deq_multi(f, (odp_event_t[64]){0}, 64)) > 0;)
			rd += (uint32_t)n;
		CHECK(rd == wr && odp_queue_destroy(f) == 0, "ring drained: %u of %u", rd, wr);
	}
	fifo_run(0);
	fifo_run(1);
	printf("queue rings: growth / wrap, %d producers x %d consumers (plain and scheduled)\n",
	       QP, QP);

	/* scheduled queues under concurrent schedulers */
	pthread_t s[4], c[2];

	for (int i = 0; i < 4; i++)
		pthread_create(&s[i], NULL, sched_thread, NULL);
	for (int i = 0; i < 2; i++)
		pthread_create(&c[i], NULL, churn_thread, NULL);
	for (int i = 0; i < 2; i++)
		pthread_join(c[i], NULL);
	__atomic_store_n(&sched_stop, 1, __ATOMIC_RELEASE);
	for (int i = 0; i < 4; i++)
		pthread_join(s[i], NULL);
	printf("sched queues: 2 x 20000 create/destroy under 4 schedulers\n");

	printf(fails ? "FAILED (%d)\n" : "PASS\n", fails);
	return fails ? 1 : 0;
}
