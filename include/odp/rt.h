/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp/rt.h — the ODP runtime subset around the GPU classifier (odp_api.h).
 *
 * Receive model: a pktio opened as "pcap:in=<file>[:loops=<n>]" (the pcap
 * pktio, platform/linux-generic/pktio/pcap.c) or "loop" in
 * ODP_PKTIN_MODE_SCHED mode with the classifier enabled is polled by the
 * scheduler. Each poll takes a burst of frames, classifies it on the GPU
 * (odpg_pktio_recv_batch's path: parse, checksums, PMR -> CoS, the pktio /
 * CoS / queue counters) and enqueues the packets on their CoS's queue
 * (_odp_cls_enq, odp_classification_internal.h:139-225); odp_schedule*()
 * then returns them from the scheduled queues. Packets carry the parse
 * result the kernel wrote (odpg_meta_t), which the odp_packet_has_* /
 * l2 / l3 accessors read.
 *
 * Spec references: init.h, shared_memory.h, pool.h / pool_types.h,
 * queue.h / queue_types.h, schedule.h, packet.h / packet_flags.h,
 * packet_io.h, packet_io_stats.h, time.h, cpu.h, cpumask.h, thread.h,
 * atomic.h, byteorder.h, hints.h, debug.h.
 */
#ifndef ODP_RT_H_
#define ODP_RT_H_

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hints, alignment, byte order ------------------------------------ */
#define odp_likely(x)   __builtin_expect(!!(x), 1)
#define odp_unlikely(x) __builtin_expect(!!(x), 0)
#define ODP_UNUSED      __attribute__((__unused__))
#define ODP_PRINTF_FORMAT(x, y) __attribute__((format(printf, (x), (y))))
#define ODP_STATIC_ASSERT(cond, msg) _Static_assert(cond, msg)
#define ODP_CACHE_LINE_SIZE 64
#define ODP_ALIGNED(x)    __attribute__((__aligned__(x)))
#define ODP_ALIGNED_CACHE ODP_ALIGNED(ODP_CACHE_LINE_SIZE)
#define ODP_PACKED        __attribute__((__packed__))
#define ODP_PAGE_SIZE     4096

typedef uint16_t odp_u16be_t;
typedef uint32_t odp_u32be_t;
typedef uint64_t odp_u64be_t;
typedef uint16_t odp_u16sum_t;

static inline uint16_t odp_cpu_to_be_16(uint16_t x) { return __builtin_bswap16(x); }
static inline uint32_t odp_cpu_to_be_32(uint32_t x) { return __builtin_bswap32(x); }
static inline uint64_t odp_cpu_to_be_64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint16_t odp_be_to_cpu_16(uint16_t x) { return __builtin_bswap16(x); }
static inline uint32_t odp_be_to_cpu_32(uint32_t x) { return __builtin_bswap32(x); }
static inline uint64_t odp_be_to_cpu_64(uint64_t x) { return __builtin_bswap64(x); }

/* ---- atomics (atomic.h), relaxed unless named otherwise --------------- */
typedef struct { uint64_t v; } odp_atomic_u64_t;
typedef struct { uint32_t v; } odp_atomic_u32_t;

static inline void odp_atomic_init_u64(odp_atomic_u64_t *a, uint64_t v)
{ __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_load_u64(odp_atomic_u64_t *a)
{ return __atomic_load_n(&a->v, __ATOMIC_RELAXED); }
static inline void odp_atomic_store_u64(odp_atomic_u64_t *a, uint64_t v)
{ __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_add_u64(odp_atomic_u64_t *a, uint64_t v)
{ __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_inc_u64(odp_atomic_u64_t *a)
{ __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_fetch_inc_u64(odp_atomic_u64_t *a)
{ return __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_init_u32(odp_atomic_u32_t *a, uint32_t v)
{ __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_load_u32(odp_atomic_u32_t *a)
{ return __atomic_load_n(&a->v, __ATOMIC_RELAXED); }
static inline void odp_atomic_store_u32(odp_atomic_u32_t *a, uint32_t v)
{ __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_inc_u32(odp_atomic_u32_t *a)
{ __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_add_u32(odp_atomic_u32_t *a, uint32_t v)
{ __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_inc_u32(odp_atomic_u32_t *a)
{ return __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_add_u32(odp_atomic_u32_t *a, uint32_t v)
{ return __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_sub_u32(odp_atomic_u32_t *a, uint32_t v)
{ return __atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_sub_u32(odp_atomic_u32_t *a, uint32_t v)
{ __atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_dec_u32(odp_atomic_u32_t *a)
{ __atomic_fetch_sub(&a->v, 1, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_dec_u32(odp_atomic_u32_t *a)
{ return __atomic_fetch_sub(&a->v, 1, __ATOMIC_RELAXED); }
static inline int odp_atomic_cas_u32(odp_atomic_u32_t *a, uint32_t *old, uint32_t nv)
{ return __atomic_compare_exchange_n(&a->v, old, nv, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_load_acq_u32(odp_atomic_u32_t *a)
{ return __atomic_load_n(&a->v, __ATOMIC_ACQUIRE); }
static inline void odp_atomic_store_rel_u32(odp_atomic_u32_t *a, uint32_t v)
{ __atomic_store_n(&a->v, v, __ATOMIC_RELEASE); }
static inline uint64_t odp_atomic_fetch_add_u64(odp_atomic_u64_t *a, uint64_t v)
{ return __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_fetch_sub_u64(odp_atomic_u64_t *a, uint64_t v)
{ return __atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_sub_u64(odp_atomic_u64_t *a, uint64_t v)
{ __atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_dec_u64(odp_atomic_u64_t *a)
{ __atomic_fetch_sub(&a->v, 1, __ATOMIC_RELAXED); }
static inline int odp_atomic_cas_u64(odp_atomic_u64_t *a, uint64_t *old, uint64_t nv)
{ return __atomic_compare_exchange_n(&a->v, old, nv, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED); }

/* ---- barrier (barrier.h): count threads meet, reusable ------------------- */
typedef struct odp_barrier_t {
	uint32_t count;
	odp_atomic_u32_t bar;      /* arrivals, 0 .. 2 * count - 1 (two phases) */
} odp_barrier_t;

void odp_barrier_init(odp_barrier_t *barr, int count);
void odp_barrier_wait(odp_barrier_t *barr);

/* ---- init (init.h) ------------------------------------------------------ */
typedef uint64_t odp_instance_t;

typedef enum odp_mem_model_t {
	ODP_MEM_MODEL_THREAD = 0,
	ODP_MEM_MODEL_PROCESS
} odp_mem_model_t;

typedef enum odp_thread_type_t {
	ODP_THREAD_WORKER = 0,
	ODP_THREAD_CONTROL
} odp_thread_type_t;

#define ODP_THREAD_COUNT_MAX 256

typedef struct odp_init_t {
	int num_worker;
	int num_control;
	const void *worker_cpus;
	const void *control_cpus;
	int (*log_fn)(int level, const char *fmt, ...);
	void (*abort_fn)(void);
	odp_mem_model_t mem_model;
	uint64_t reserved[8];
} odp_init_t;

void odp_init_param_init(odp_init_t *param);
int  odp_init_global(odp_instance_t *instance, const odp_init_t *param, const void *platform);
int  odp_init_local(odp_instance_t instance, odp_thread_type_t thr_type);
int  odp_term_local(void);
int  odp_term_global(odp_instance_t instance);
void odp_sys_info_print(void);
/* thread ids (thread.h): the lowest free id in [0, ODP_THREAD_COUNT_MAX) is
 * taken by odp_init_local() and given back by odp_term_local(), as the
 * reference's thread table does (odp_thread.c:alloc_id / free_id) */
int  odp_thread_id(void);
int  odp_thread_count(void);
int  odp_thread_count_max(void);
odp_thread_type_t odp_thread_type(void);
int  odp_cpu_id(void);
int  odp_cpu_count(void);

/* ---- CPU cycle counter (cpu.h) ------------------------------------------ */
uint64_t odp_cpu_cycles(void);
uint64_t odp_cpu_cycles_diff(uint64_t c2, uint64_t c1);
uint64_t odp_cpu_cycles_max(void);
uint64_t odp_cpu_cycles_resolution(void);

/* ---- CPU masks (cpumask.h) --------------------------------------------- */
#define ODP_CPUMASK_SIZE     1024
#define ODP_CPUMASK_STR_SIZE ((ODP_CPUMASK_SIZE + 3) / 4 + 3)

typedef struct odp_cpumask_t {
	uint64_t bits[ODP_CPUMASK_SIZE / 64];
} odp_cpumask_t;

void    odp_cpumask_zero(odp_cpumask_t *mask);
void    odp_cpumask_set(odp_cpumask_t *mask, int cpu);
int     odp_cpumask_isset(const odp_cpumask_t *mask, int cpu);
int     odp_cpumask_count(const odp_cpumask_t *mask);
int     odp_cpumask_first(const odp_cpumask_t *mask);
int     odp_cpumask_next(const odp_cpumask_t *mask, int cpu);
int32_t odp_cpumask_to_str(const odp_cpumask_t *mask, char *str, int32_t size);
int     odp_cpumask_default_worker(odp_cpumask_t *mask, int num);
int     odp_cpumask_default_control(odp_cpumask_t *mask, int num);

/* ---- time (time.h) ------------------------------------------------------ */
#define ODP_TIME_USEC_IN_NS 1000ULL
#define ODP_TIME_MSEC_IN_NS 1000000ULL
#define ODP_TIME_SEC_IN_NS  1000000000ULL
#define ODP_TIME_MIN_IN_NS  60000000000ULL
#define ODP_TIME_HOUR_IN_NS 3600000000000ULL

typedef struct odp_time_t {
	uint64_t nsec;
} odp_time_t;

#define ODP_TIME_NULL ((odp_time_t){ 0 })

/* one monotonic nanosecond clock serves local and global time; the
 * _strict variants order the read against earlier loads and stores */
odp_time_t odp_time_local(void);
odp_time_t odp_time_global(void);
odp_time_t odp_time_local_strict(void);
odp_time_t odp_time_global_strict(void);
uint64_t   odp_time_local_ns(void);
uint64_t   odp_time_global_ns(void);
uint64_t   odp_time_local_strict_ns(void);
odp_time_t odp_time_local_from_ns(uint64_t ns);
odp_time_t odp_time_global_from_ns(uint64_t ns);
odp_time_t odp_time_diff(odp_time_t t2, odp_time_t t1);
uint64_t   odp_time_diff_ns(odp_time_t t2, odp_time_t t1);
odp_time_t odp_time_sum(odp_time_t t1, odp_time_t t2);
odp_time_t odp_time_add_ns(odp_time_t time, uint64_t ns);
int        odp_time_cmp(odp_time_t t2, odp_time_t t1);
uint64_t   odp_time_to_ns(odp_time_t time);
uint64_t   odp_time_local_res(void);
void       odp_time_wait_ns(uint64_t ns);
void       odp_time_wait_until(odp_time_t time);

/* ---- shared memory (shared_memory.h) ------------------------------------ */
typedef struct _odp_shm_hdl *odp_shm_t;
#define ODP_SHM_INVALID ((odp_shm_t)0)

/* named blocks: odp_shm_lookup() finds a block by the name it was reserved
 * under (the newest, if names repeat) */
odp_shm_t odp_shm_reserve(const char *name, uint64_t size, uint64_t align, uint32_t flags);
odp_shm_t odp_shm_lookup(const char *name);
void     *odp_shm_addr(odp_shm_t shm);
int       odp_shm_free(odp_shm_t shm);
uint64_t  odp_shm_to_u64(odp_shm_t shm);

/* ---- packet pools (pool.h, pool_types.h) -------------------------------- */
#define ODP_POOL_NAME_LEN 32

typedef enum odp_pool_type_t {
	ODP_POOL_BUFFER = 1,
	ODP_POOL_PACKET,
	ODP_POOL_TIMEOUT,
	ODP_POOL_VECTOR
} odp_pool_type_t;

typedef struct odp_pool_param_t {
	odp_pool_type_t type;
	struct {
		uint32_t num;
		uint32_t size;
		uint32_t align;
	} buf;
	struct {
		uint32_t num;
		uint32_t max_num;
		uint32_t len;
		uint32_t max_len;
		uint32_t seg_len;
		uint32_t uarea_size;
		uint32_t headroom;
		/* buffers a thread may keep in its local cache (0: none; the
		 * runtime caps it at 1/32 of num and max_cache_size) */
		uint32_t cache_size;
	} pkt;
	uint64_t reserved[8];
} odp_pool_param_t;

/* odp_pool_capability_t (pool_types.h), field for field */
typedef union odp_pool_stats_opt_t {
	struct {
		uint64_t available          : 1;
		uint64_t alloc_ops          : 1;
		uint64_t alloc_fails        : 1;
		uint64_t free_ops           : 1;
		uint64_t total_ops          : 1;
		uint64_t cache_available    : 1;
		uint64_t cache_alloc_ops    : 1;
		uint64_t cache_free_ops     : 1;
		uint64_t thread_cache_available : 1;
	} bit;
	uint64_t all;
} odp_pool_stats_opt_t;

typedef struct odp_pool_capability_t {
	uint32_t max_pools;
	struct {
		uint32_t max_pools;
		uint32_t max_align;
		uint32_t max_size;
		uint32_t max_num;
		uint32_t max_uarea_size;
		odp_bool_t uarea_persistence;
		uint32_t min_cache_size;
		uint32_t max_cache_size;
		odp_pool_stats_opt_t stats;
	} buf;
	struct {
		uint32_t max_pools;
		uint32_t max_len;
		uint32_t max_num;
		uint32_t max_align;
		uint32_t min_headroom;
		uint32_t max_headroom;
		uint32_t min_tailroom;
		uint32_t max_segs_per_pkt;
		uint32_t min_seg_len;
		uint32_t max_seg_len;
		uint32_t max_uarea_size;
		odp_bool_t uarea_persistence;
		uint8_t max_num_subparam;
		uint32_t min_cache_size;
		uint32_t max_cache_size;
		odp_pool_stats_opt_t stats;
	} pkt;
	struct {
		uint32_t max_pools;
		uint32_t max_num;
		uint32_t max_uarea_size;
		odp_bool_t uarea_persistence;
		uint32_t min_cache_size;
		uint32_t max_cache_size;
		odp_pool_stats_opt_t stats;
	} tmo;
	struct {
		uint32_t max_pools;
		uint32_t max_num;
		uint32_t max_size;
		uint32_t max_uarea_size;
		odp_bool_t uarea_persistence;
		uint32_t min_cache_size;
		uint32_t max_cache_size;
		odp_pool_stats_opt_t stats;
	} vector;
} odp_pool_capability_t;

/* packet pools only; buffer / timeout / vector pools report max_pools 0 */
int        odp_pool_capability(odp_pool_capability_t *capa);
void       odp_pool_param_init(odp_pool_param_t *param);
odp_pool_t odp_pool_create(const char *name, const odp_pool_param_t *param);
int        odp_pool_destroy(odp_pool_t pool);
odp_pool_t odp_pool_lookup(const char *name);
uint64_t   odp_pool_to_u64(odp_pool_t pool);
void       odp_pool_print(odp_pool_t pool);
void       odp_pool_print_all(void);

/* ---- events, queues, scheduler (queue.h, schedule.h) -------------------- */
typedef struct _odp_event_hdl *odp_event_t;
#define ODP_EVENT_INVALID ((odp_event_t)0)

/* odp_event_type_t (include-abi/odp/api/abi/event_types.h): every event of
 * this runtime is a packet */
typedef enum odp_event_type_t {
	ODP_EVENT_BUFFER = 1,
	ODP_EVENT_PACKET = 2,
	ODP_EVENT_TIMEOUT = 3,
	ODP_EVENT_IPSEC_STATUS = 5,
	ODP_EVENT_PACKET_VECTOR = 6,
	ODP_EVENT_PACKET_TX_COMPL = 7,
	ODP_EVENT_DMA_COMPL = 8,
	ODP_EVENT_ML_COMPL = 9
} odp_event_type_t;

odp_event_type_t odp_event_type(odp_event_t event);

/* Queue handles come from a registry (odp_queue_create): a tag in the top
 * bits that no user-space pointer has, and the queue's slot. Any other value
 * (e.g. an integer an application hands the classifier as a queue) is not a
 * queue here: operations on it fail. */
#define ODP_QUEUE_NAME_LEN 32

typedef struct odp_queue_info_t {
	const char *name;
	odp_queue_param_t param;
} odp_queue_info_t;

odp_queue_t odp_queue_create(const char *name, const odp_queue_param_t *param);
int         odp_queue_destroy(odp_queue_t queue);
int         odp_queue_info(odp_queue_t queue, odp_queue_info_t *info);
odp_queue_type_t odp_queue_type(odp_queue_t queue);
uint64_t    odp_queue_to_u64(odp_queue_t queue);
int         odp_queue_enq(odp_queue_t queue, odp_event_t ev);
odp_event_t odp_queue_deq(odp_queue_t queue);
int         odp_queue_enq_multi(odp_queue_t queue, const odp_event_t ev[], int num);
int         odp_queue_deq_multi(odp_queue_t queue, odp_event_t ev[], int num);
void        odp_event_free(odp_event_t event);
void        odp_event_free_multi(const odp_event_t event[], int num);

#define ODP_SCHED_WAIT    UINT64_MAX
#define ODP_SCHED_NO_WAIT 0

typedef struct odp_schedule_config_t {
	uint32_t num_queues;
	uint32_t queue_size;
	uint64_t reserved[4];
} odp_schedule_config_t;

/* odp_schedule_capability_t (schedule_types.h), field for field */
typedef struct odp_schedule_capability_t {
	uint32_t max_ordered_locks;
	uint32_t max_groups;
	uint32_t max_prios;
	uint32_t max_queues;
	uint32_t max_queue_size;
	uint32_t max_flow_id;
	odp_support_t lockfree_queues;
	odp_support_t waitfree_queues;
	odp_support_t order_wait;
} odp_schedule_capability_t;

int      odp_schedule_capability(odp_schedule_capability_t *capa);
void     odp_schedule_config_init(odp_schedule_config_t *config);
int      odp_schedule_config(const odp_schedule_config_t *config);
uint64_t odp_schedule_wait_time(uint64_t ns);
odp_event_t odp_schedule(odp_queue_t *from, uint64_t wait);
int      odp_schedule_multi(odp_queue_t *from, uint64_t wait, odp_event_t events[], int num);
int      odp_schedule_default_prio(void);

/* ---- packets (packet.h, packet_flags.h) --------------------------------- */
odp_event_t  odp_packet_to_event(odp_packet_t pkt);
odp_packet_t odp_packet_from_event(odp_event_t ev);
void     odp_packet_from_event_multi(odp_packet_t pkt[], const odp_event_t ev[], int num);
odp_packet_t odp_packet_alloc(odp_pool_t pool, uint32_t len);
void     odp_packet_free(odp_packet_t pkt);
void     odp_packet_free_multi(const odp_packet_t pkt[], int num);
uint32_t odp_packet_len(odp_packet_t pkt);
void    *odp_packet_data(odp_packet_t pkt);
odp_pool_t odp_packet_pool(odp_packet_t pkt);
/* the pktio a packet was received on (ODP_PKTIO_INVALID if none) */
odp_pktio_t odp_packet_input(odp_packet_t pkt);
int      odp_packet_input_index(odp_packet_t pkt);
void    *odp_packet_l2_ptr(odp_packet_t pkt, uint32_t *len);
void    *odp_packet_l3_ptr(odp_packet_t pkt, uint32_t *len);
void    *odp_packet_l4_ptr(odp_packet_t pkt, uint32_t *len);
uint32_t odp_packet_l2_offset(odp_packet_t pkt);
uint32_t odp_packet_l3_offset(odp_packet_t pkt);
uint32_t odp_packet_l4_offset(odp_packet_t pkt);
/* 0, or -1 for an offset past the packet (packet.h) */
int      odp_packet_l2_offset_set(odp_packet_t pkt, uint32_t offset);
int      odp_packet_l3_offset_set(odp_packet_t pkt, uint32_t offset);
int      odp_packet_l4_offset_set(odp_packet_t pkt, uint32_t offset);
/* 0, or -1 when [offset, offset + len) leaves the packet */
int      odp_packet_copy_to_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, void *dst);
int      odp_packet_copy_from_mem(odp_packet_t pkt, uint32_t offset, uint32_t len,
				  const void *src);
odp_cos_t odp_packet_cos(odp_packet_t pkt);
void     odp_packet_print_data(odp_packet_t pkt, uint32_t offset, uint32_t len);

/* The receive verdict a packet carries: the parse result the GPU kernel
 * wrote for it (odpg_meta_t = packet_parser_t) and its classifier mark. The
 * accessors decode it exactly as the reference's inline accessors decode
 * packet_parser_t (include/odp/api/plat/packet_inlines.h:334-417,617,
 * packet_flag_inlines.h:62-288). */
typedef enum odp_packet_chksum_status_t {
	ODP_PACKET_CHKSUM_UNKNOWN = 0,
	ODP_PACKET_CHKSUM_BAD,
	ODP_PACKET_CHKSUM_OK
} odp_packet_chksum_status_t;

odp_packet_chksum_status_t odp_packet_l3_chksum_status(odp_packet_t pkt);
odp_packet_chksum_status_t odp_packet_l4_chksum_status(odp_packet_t pkt);
uint64_t odp_packet_cls_mark(odp_packet_t pkt);

int odp_packet_has_error(odp_packet_t pkt);
int odp_packet_has_l2_error(odp_packet_t pkt);
int odp_packet_has_l3_error(odp_packet_t pkt);
int odp_packet_has_l4_error(odp_packet_t pkt);
int odp_packet_has_l2(odp_packet_t pkt);
int odp_packet_has_l3(odp_packet_t pkt);
int odp_packet_has_l4(odp_packet_t pkt);
int odp_packet_has_eth(odp_packet_t pkt);
int odp_packet_has_eth_bcast(odp_packet_t pkt);
int odp_packet_has_eth_mcast(odp_packet_t pkt);
int odp_packet_has_jumbo(odp_packet_t pkt);
int odp_packet_has_vlan(odp_packet_t pkt);
int odp_packet_has_vlan_qinq(odp_packet_t pkt);
int odp_packet_has_arp(odp_packet_t pkt);
int odp_packet_has_ipv4(odp_packet_t pkt);
int odp_packet_has_ipv6(odp_packet_t pkt);
int odp_packet_has_ip_bcast(odp_packet_t pkt);
int odp_packet_has_ip_mcast(odp_packet_t pkt);
int odp_packet_has_ipfrag(odp_packet_t pkt);
int odp_packet_has_ipopt(odp_packet_t pkt);
int odp_packet_has_ipsec(odp_packet_t pkt);
int odp_packet_has_udp(odp_packet_t pkt);
int odp_packet_has_tcp(odp_packet_t pkt);
int odp_packet_has_sctp(odp_packet_t pkt);
int odp_packet_has_icmp(odp_packet_t pkt);
int odp_packet_has_flow_hash(odp_packet_t pkt);
int odp_packet_has_ts(odp_packet_t pkt);

/* protocol types (packet_types.h:60-175) */
typedef uint8_t  odp_proto_l2_type_t;
typedef uint16_t odp_proto_l3_type_t;
typedef uint8_t  odp_proto_l4_type_t;
#define ODP_PROTO_L2_TYPE_NONE    0
#define ODP_PROTO_L2_TYPE_ETH     1
#define ODP_PROTO_L3_TYPE_NONE    0xFFFF
#define ODP_PROTO_L3_TYPE_ARP     0x0806
#define ODP_PROTO_L3_TYPE_IPV4    0x0800
#define ODP_PROTO_L3_TYPE_IPV6    0x86DD
#define ODP_PROTO_L4_TYPE_NONE    255
#define ODP_PROTO_L4_TYPE_ICMPV4  1
#define ODP_PROTO_L4_TYPE_TCP     6
#define ODP_PROTO_L4_TYPE_UDP     17
#define ODP_PROTO_L4_TYPE_ESP     50
#define ODP_PROTO_L4_TYPE_AH      51
#define ODP_PROTO_L4_TYPE_ICMPV6  58
#define ODP_PROTO_L4_TYPE_NO_NEXT 59
#define ODP_PROTO_L4_TYPE_SCTP    132

odp_proto_l2_type_t odp_packet_l2_type(odp_packet_t pkt);
odp_proto_l3_type_t odp_packet_l3_type(odp_packet_t pkt);
odp_proto_l4_type_t odp_packet_l4_type(odp_packet_t pkt);

/* Parsing packets the application holds (packet.h, odp_packet_parse):
 * the batch goes through the same GPU parser as a receive, starting at
 * `offset` with the given protocol. odp_packet_parse_multi() parses up to
 * the first packet that fails and returns its index (num when none does),
 * as odp_packet.c:2064-2075; packets after it keep their metadata. */
typedef enum odp_proto_t {
	ODP_PROTO_NONE = 0,
	ODP_PROTO_ETH,
	ODP_PROTO_IPV4,
	ODP_PROTO_IPV6
} odp_proto_t;

typedef union odp_proto_chksums_t {
	struct {
		uint32_t ipv4 : 1;
		uint32_t udp  : 1;
		uint32_t tcp  : 1;
		uint32_t sctp : 1;
	} chksum;
	uint32_t all_chksum;
} odp_proto_chksums_t;

typedef struct odp_packet_parse_param_t {
	odp_proto_t proto;
	odp_proto_layer_t last_layer;
	odp_proto_chksums_t chksums;
} odp_packet_parse_param_t;

typedef union odp_packet_parse_result_flag_t {
	uint64_t all;
	struct {
		uint64_t has_error     : 1;
		uint64_t has_l2_error  : 1;
		uint64_t has_l3_error  : 1;
		uint64_t has_l4_error  : 1;
		uint64_t has_l2        : 1;
		uint64_t has_l3        : 1;
		uint64_t has_l4        : 1;
		uint64_t has_eth       : 1;
		uint64_t has_eth_bcast : 1;
		uint64_t has_eth_mcast : 1;
		uint64_t has_jumbo     : 1;
		uint64_t has_vlan      : 1;
		uint64_t has_vlan_qinq : 1;
		uint64_t has_arp       : 1;
		uint64_t has_ipv4      : 1;
		uint64_t has_ipv6      : 1;
		uint64_t has_ip_bcast  : 1;
		uint64_t has_ip_mcast  : 1;
		uint64_t has_ipfrag    : 1;
		uint64_t has_ipopt     : 1;
		uint64_t has_ipsec     : 1;
		uint64_t has_udp       : 1;
		uint64_t has_tcp       : 1;
		uint64_t has_sctp      : 1;
		uint64_t has_icmp      : 1;
	};
} odp_packet_parse_result_flag_t;

typedef struct odp_packet_parse_result_t {
	odp_packet_parse_result_flag_t flag;
	uint32_t packet_len;
	uint32_t l2_offset;
	uint32_t l3_offset;
	uint32_t l4_offset;
	odp_packet_chksum_status_t l3_chksum_status;
	odp_packet_chksum_status_t l4_chksum_status;
	odp_proto_l2_type_t l2_type;
	odp_proto_l3_type_t l3_type;
	odp_proto_l4_type_t l4_type;
} odp_packet_parse_result_t;

int  odp_packet_parse(odp_packet_t pkt, uint32_t offset, const odp_packet_parse_param_t *param);
int  odp_packet_parse_multi(const odp_packet_t pkt[], const uint32_t offset[], int num,
			    const odp_packet_parse_param_t *param);
void odp_packet_parse_result(odp_packet_t pkt, odp_packet_parse_result_t *result);
void odp_packet_parse_result_multi(const odp_packet_t pkt[], odp_packet_parse_result_t *result[],
				   int num);

/* A runtime packet as the batch API sees a frame (odp_cls.h odpg_packet_t):
 * its bytes and the parse result it carries (odpg_meta_t, the
 * packet_parser_t layout plus cls_mark). 0, or -1 if `pkt` is not a packet
 * of this runtime. */
int odpg_packet_view(odp_packet_t pkt, odpg_packet_t *view);

/* checksum (chksum.h:26-40): the 16-bit ones' complement sum (not inverted)
 * of the data's 16-bit words in memory byte order, an odd tail byte padded
 * with zero (odp_chksum.c: chksum_finalize(chksum_partial(p, len, 0))) */
uint16_t odp_chksum_ones_comp16(const void *data, uint32_t len);

#define ODP_PACKET_OFFSET_INVALID 0xFFFFu

/* ---- pktio beyond the classifier setters (packet_io.h) ------------------ */
typedef struct odp_pktin_queue_t {
	odp_pktio_t pktio;
	int index;
} odp_pktin_queue_t;

typedef struct odp_pktout_queue_t {
	odp_pktio_t pktio;
	int index;
} odp_pktout_queue_t;

/* packet_io_stats.h */
typedef struct odp_pktin_queue_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_pktin_queue_stats_t;

typedef struct odp_pktout_queue_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_pktout_queue_stats_t;

#ifndef ODP_PKTOUT_MAX_QUEUES
#define ODP_PKTOUT_MAX_QUEUES 64
#endif

/* packet_io_types.h:325-339 */
typedef struct odp_pktout_queue_param_t {
	odp_pktio_op_mode_t op_mode;
	uint32_t num_queues;
	uint32_t queue_size[ODP_PKTOUT_MAX_QUEUES];
} odp_pktout_queue_param_t;

typedef union odp_pktio_set_op_t {
	struct {
		uint32_t promisc_mode : 1;
		uint32_t mac_addr     : 1;
		uint32_t maxlen       : 1;
	} op;
	uint32_t all_bits;
} odp_pktio_set_op_t;

typedef struct odp_pktio_capability_t {
	uint32_t max_input_queues;
	uint32_t max_output_queues;
	odp_pktio_config_t config;
	odp_pktio_set_op_t set_op;
	odp_bool_t loop_supported;
	uint64_t reserved[8];
} odp_pktio_capability_t;

int  odp_pktio_capability(odp_pktio_t pktio, odp_pktio_capability_t *capa);
odp_pktio_t odp_pktio_lookup(const char *name);

/* input: the loop device (frames sent on it come back, pktio/loop.c) and
 * the pcap device are received through the GPU classifier, in bursts:
 * ODP_PKTIN_MODE_DIRECT by odp_pktin_recv(), ODP_PKTIN_MODE_QUEUE by a
 * dequeue from the pktin event queue, ODP_PKTIN_MODE_SCHED by the
 * scheduler. Packets the classifier places go to their CoS queue; with the
 * classifier disabled they are returned / enqueued on the pktin queue. */
int  odp_pktin_queue(odp_pktio_t pktio, odp_pktin_queue_t queues[], int num);
int  odp_pktin_event_queue(odp_pktio_t pktio, odp_queue_t queues[], int num);
int  odp_pktin_recv(odp_pktin_queue_t queue, odp_packet_t packets[], int num);
int  odp_pktin_queue_stats(odp_pktin_queue_t queue, odp_pktin_queue_stats_t *stats);
int  odp_pktin_event_queue_stats(odp_pktio_t pktio, odp_queue_t queue,
				 odp_pktin_queue_stats_t *stats);
int  odp_pktout_event_queue(odp_pktio_t pktio, odp_queue_t queues[], int num);
int  odp_pktout_queue_stats(odp_pktout_queue_t queue, odp_pktout_queue_stats_t *stats);
int  odp_pktout_event_queue_stats(odp_pktio_t pktio, odp_queue_t queue,
				  odp_pktout_queue_stats_t *stats);
void odp_pktout_queue_param_init(odp_pktout_queue_param_t *param);
int  odp_pktout_queue_config(odp_pktio_t pktio, const odp_pktout_queue_param_t *param);
int  odp_pktout_queue(odp_pktio_t pktio, odp_pktout_queue_t queues[], int num);
int  odp_pktout_send(odp_pktout_queue_t queue, const odp_packet_t packets[], int num);
int  odp_pktio_promisc_mode(odp_pktio_t pktio);
int  odp_pktio_promisc_mode_set(odp_pktio_t pktio, odp_bool_t enable);
int  odp_pktio_mac_addr(odp_pktio_t pktio, void *mac_addr, int size);

#ifdef __cplusplus
}
#endif

#endif
