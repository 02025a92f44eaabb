/* SPDX-License-Identifier: BSD-3-Clause
 *
 * TEST INFRASTRUCTURE ONLY: the libodpg.so device entry points the host
 * runtime calls (odp_amd/csrc/odp_rt.c, odp_cls.c), restated on the CPU so
 * that the runtime can be built and run under ThreadSanitizer and
 * AddressSanitizer + UBSan without a GPU (tests/c/Makefile "san" targets,
 * tests/test_sanitizers.py). GPU AddressSanitizer is not available on the
 * MI355X pool; this is how the host code gets the sanitizer coverage the
 * reference's CI gives its own (.github/workflows/ci-pipeline.yml:399-412).
 *
 * Classification runs synchronously through the CPU oracle
 * (oracle/odp_oracle.c, oracle_classify), so verdicts, marks and metadata
 * are the ones the GPU produces (the parity tests pin that); fences are
 * complete as soon as they are recorded; "pinned" host memory is plain
 * aligned memory and its device address is itself. Counters fold the
 * oracle's pktio / CoS counts and per-queue deliveries in the layout of
 * ODPG_COUNTER_WORDS. Nothing here is part of the product library.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/odpg.h"

int oracle_classify(const odpg_rules_t *rules, const uint8_t *frames, const odpg_desc_t *desc,
		    uint32_t stride, uint32_t num, uint64_t opt, int layer, int classify,
		    odpg_out_t *out, uint16_t *mark, odpg_meta_t *meta, uint64_t *stats);

struct odpg_ctx_s {
	int device;
	int refs;
	pthread_mutex_t lock;
};

struct odpg_table_s {
	odpg_rules_t r;
	odpg_cos_t *cos;
	odpg_pmr_t *pmr;
	uint32_t *rule_pmr, *rule_dst;
};

struct odpg_counters_s {
	odpg_ctx_t *ctx;
	uint32_t num_cos;
	uint64_t *words;
	pthread_mutex_t lock;
};

struct odpg_fence_s {
	odpg_ctx_t *ctx;
};

int odpg_abi_version(void)
{
	return ODPG_ABI_VERSION;
}

const char *odpg_build_info(void)
{
	return "gpu_stub (CPU oracle, sanitizer builds)";
}

int odpg_device_count(void)
{
	return 1;
}

static void ctx_unref(odpg_ctx_t *c)
{
	pthread_mutex_lock(&c->lock);
	const int left = --c->refs;

	pthread_mutex_unlock(&c->lock);
	if (!left) {
		pthread_mutex_destroy(&c->lock);
		free(c);
	}
}

static void ctx_ref(odpg_ctx_t *c)
{
	pthread_mutex_lock(&c->lock);
	c->refs++;
	pthread_mutex_unlock(&c->lock);
}

int odpg_ctx_create(int device, void *stream, odpg_ctx_t **ctx)
{
	(void)stream;
	if (!ctx || device != 0)
		return -EINVAL;
	odpg_ctx_t *c = calloc(1, sizeof(*c));

	if (!c)
		return -ENOMEM;
	c->device = device;
	c->refs = 1;
	pthread_mutex_init(&c->lock, NULL);
	*ctx = c;
	return 0;
}

void odpg_ctx_destroy(odpg_ctx_t *ctx)
{
	if (ctx)
		ctx_unref(ctx);
}

int odpg_ctx_sync(odpg_ctx_t *ctx)
{
	return ctx ? 0 : -EINVAL;
}

static void table_free(odpg_table_t *t)
{
	free(t->cos);
	free(t->pmr);
	free(t->rule_pmr);
	free(t->rule_dst);
}

/* a deep copy of the rule snapshot (the caller's arrays are not kept) */
static int table_fill(odpg_table_t *t, const odpg_rules_t *r)
{
	memset(t, 0, sizeof(*t));
	t->r = *r;
	t->cos = calloc(r->num_cos ? r->num_cos : 1, sizeof(odpg_cos_t));
	t->pmr = calloc(r->num_pmr ? r->num_pmr : 1, sizeof(odpg_pmr_t));
	t->rule_pmr = calloc(r->num_slots ? r->num_slots : 1, sizeof(uint32_t));
	t->rule_dst = calloc(r->num_slots ? r->num_slots : 1, sizeof(uint32_t));
	if (!t->cos || !t->pmr || !t->rule_pmr || !t->rule_dst) {
		table_free(t);
		return -ENOMEM;
	}
	if (r->num_cos)
		memcpy(t->cos, r->cos, r->num_cos * sizeof(odpg_cos_t));
	if (r->num_pmr)
		memcpy(t->pmr, r->pmr, r->num_pmr * sizeof(odpg_pmr_t));
	if (r->num_slots) {
		memcpy(t->rule_pmr, r->rule_pmr, r->num_slots * sizeof(uint32_t));
		memcpy(t->rule_dst, r->rule_dst, r->num_slots * sizeof(uint32_t));
	}
	t->r.cos = t->cos;
	t->r.pmr = t->pmr;
	t->r.rule_pmr = t->rule_pmr;
	t->r.rule_dst = t->rule_dst;
	return 0;
}

int odpg_table_create(odpg_ctx_t *ctx, const odpg_rules_t *rules, odpg_table_t **tbl)
{
	if (!ctx || !rules || !tbl)
		return -EINVAL;
	odpg_table_t *t = malloc(sizeof(*t));

	if (!t)
		return -ENOMEM;
	if (table_fill(t, rules)) {
		free(t);
		return -ENOMEM;
	}
	*tbl = t;
	return 0;
}

/* the compiled image (odpg_rules_compile / odpg_table_import) of the stub:
 * a tag and the caller's rule snapshot pointer, imported in the same process
 * while the snapshot lives (the device groups' load, group.cpp) */
#define STUB_IMAGE_TAG 0x53545542u

struct stub_image {
	uint32_t tag;
	const odpg_rules_t *rules;
};

int odpg_rules_compile(const odpg_rules_t *rules, void *buf, size_t *size)
{
	if (!rules || !size)
		return -EINVAL;
	if (!buf || *size < sizeof(struct stub_image)) {
		*size = sizeof(struct stub_image);
		return -ENOSPC;
	}
	struct stub_image im = { STUB_IMAGE_TAG, rules };

	memcpy(buf, &im, sizeof(im));
	*size = sizeof(im);
	return 0;
}

int odpg_table_import(odpg_ctx_t *ctx, const void *image, size_t size, odpg_table_t **tbl)
{
	struct stub_image im;

	if (!image || size != sizeof(im))
		return -EINVAL;
	memcpy(&im, image, sizeof(im));
	if (im.tag != STUB_IMAGE_TAG)
		return -EINVAL;
	return odpg_table_create(ctx, im.rules, tbl);
}

int odpg_table_update(odpg_ctx_t *ctx, odpg_table_t *tbl, const odpg_rules_t *rules)
{
	odpg_table_t n;

	if (!ctx || !tbl || !rules)
		return -EINVAL;
	if (table_fill(&n, rules))
		return -ENOMEM;
	table_free(tbl);
	*tbl = n;
	return 0;
}

void odpg_table_destroy(odpg_table_t *tbl)
{
	if (!tbl)
		return;
	table_free(tbl);
	free(tbl);
}

uint32_t odpg_table_num_cos(const odpg_table_t *tbl)
{
	return tbl ? tbl->r.num_cos : 0u;
}

int odpg_table_has_cycle(const odpg_table_t *tbl)
{
	(void)tbl;
	return 0;
}

int odpg_counters_create(odpg_ctx_t *ctx, const odpg_table_t *tbl, odpg_counters_t **cnt)
{
	if (!ctx || !tbl || !cnt)
		return -EINVAL;
	odpg_counters_t *c = calloc(1, sizeof(*c));

	if (!c)
		return -ENOMEM;
	c->num_cos = tbl->r.num_cos;
	c->words = calloc(ODPG_COUNTER_WORDS(c->num_cos), sizeof(uint64_t));
	if (!c->words) {
		free(c);
		return -ENOMEM;
	}
	pthread_mutex_init(&c->lock, NULL);
	c->ctx = ctx;
	ctx_ref(ctx);
	*cnt = c;
	return 0;
}

void odpg_counters_destroy(odpg_counters_t *cnt)
{
	if (!cnt)
		return;
	ctx_unref(cnt->ctx);
	pthread_mutex_destroy(&cnt->lock);
	free(cnt->words);
	free(cnt);
}

int odpg_counters_match(const odpg_counters_t *cnt, const odpg_table_t *tbl)
{
	return cnt && tbl && cnt->num_cos == tbl->r.num_cos;
}

int odpg_counters_fold(odpg_counters_t *cnt, uint64_t *words)
{
	if (!cnt || !words)
		return -EINVAL;
	pthread_mutex_lock(&cnt->lock);
	for (uint32_t k = 0; k < ODPG_COUNTER_WORDS(cnt->num_cos); k++) {
		words[k] += cnt->words[k];
		cnt->words[k] = 0;
	}
	pthread_mutex_unlock(&cnt->lock);
	return 0;
}

/* the launch's counts into a counters object: the oracle's pktio and CoS
 * counts, and per (CoS, hash queue) the packets the classifier handed over
 * (an error packet to the error CoS unless it drops) */
static void count(odpg_counters_t *c, const odpg_table_t *t, const odpg_out_t *out, uint32_t num,
		  const uint64_t *st)
{
	const uint32_t nc = c->num_cos;

	pthread_mutex_lock(&c->lock);
	for (uint32_t k = 0; k < 4u + nc; k++)
		c->words[k] += st[k];
	for (uint32_t i = 0; i < num; i++) {
		const uint32_t w = out[i], cos = ODPG_OUT_COS(w);

		if (cos >= nc || (w & ODPG_OUT_CLS_DROP))
			continue;
		if ((w & ODPG_OUT_ERROR) && (int32_t)cos != t->r.error_cos)
			continue;
		c->words[4u + nc + ODPG_COS_QUEUE_MAX * cos + ODPG_OUT_HASHQ(w)]++;
	}
	pthread_mutex_unlock(&c->lock);
}

int odpg_classify(odpg_ctx_t *ctx, const odpg_table_t *tbl, const odpg_batch_t *b,
		  const odpg_result_t *res)
{
	if (!ctx || !tbl || !b || !res || !res->out || (res->stats && res->counters))
		return -EINVAL;
	if (!b->num)
		return 0;
	uint64_t *st = calloc(4u + tbl->r.num_cos, sizeof(uint64_t));

	if (!st)
		return -ENOMEM;
	oracle_classify(&tbl->r, b->frames, b->desc, b->stride, b->num, b->pktin_opt,
			(int)b->layer, (int)b->classify, res->out, res->mark, res->meta, st);
	if (res->stats)
		for (uint32_t k = 0; k < 4u + tbl->r.num_cos; k++)
			res->stats[k] += st[k];
	if (res->counters)
		count(res->counters, tbl, res->out, b->num, st);
	free(st);
	return 0;
}

int odpg_classify_host(odpg_ctx_t *ctx, const odpg_table_t *tbl, const odpg_batch_t *batch,
		       const odpg_result_t *res, uint32_t chunk_pkts)
{
	(void)chunk_pkts;
	return odpg_classify(ctx, tbl, batch, res);
}

int odpg_host_alloc_pinned(size_t bytes, void **ptr)
{
	if (!ptr)
		return -EINVAL;
	return posix_memalign(ptr, 4096, bytes ? bytes : 16) ? -ENOMEM : 0;
}

int odpg_host_free_pinned(void *ptr)
{
	free(ptr);
	return 0;
}

int odpg_host_device_ptr(void *host_ptr, void **dev_ptr)
{
	if (!dev_ptr)
		return -EINVAL;
	*dev_ptr = host_ptr;
	return 0;
}

int odpg_fence_create(odpg_ctx_t *ctx, odpg_fence_t **fence)
{
	if (!ctx || !fence)
		return -EINVAL;
	odpg_fence_t *f = calloc(1, sizeof(*f));

	if (!f)
		return -ENOMEM;
	f->ctx = ctx;
	ctx_ref(ctx);
	*fence = f;
	return 0;
}

int odpg_fence_record(odpg_ctx_t *ctx, odpg_fence_t *fence)
{
	return ctx && fence ? 0 : -EINVAL;
}

int odpg_fence_query(odpg_fence_t *fence)
{
	return fence ? 1 : -EINVAL;
}

int odpg_fence_wait(odpg_fence_t *fence)
{
	return fence ? 0 : -EINVAL;
}

void odpg_fence_destroy(odpg_fence_t *fence)
{
	if (!fence)
		return;
	ctx_unref(fence->ctx);
	free(fence);
}
