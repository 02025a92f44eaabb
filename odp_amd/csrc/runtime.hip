/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Host runtime behind the odpg.h C-ABI: contexts (device + stream + scratch),
 * compiled rule tables in HBM, device-resident and host-buffer batch
 * classification, and thin memory / timing helpers.
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/odpg.h"
#include "odpg_internal.h"
#include "stats_commit.h"
#include "cls_compile.h"


extern "C" int odpg_launch_classify(const odpg_launch_args *a, hipStream_t s);
extern "C" uint32_t odpg_launch_grid(uint32_t num);

#define NUM_EVENTS 16

/* host-path staging (odpg_classify_host): NSTAGE buffer sets cycle
 * through H2D (copy stream) -> classify + D2H (context stream); kept in the
 * context and grown on demand, so repeated calls allocate nothing */
#define NSTAGE 3

struct Stage {
	uint8_t *frames;
	odpg_desc_t *desc;
	odpg_out_t *out;
	uint16_t *mark;
	odpg_meta_t *meta;
	odpg_desc_t *hdesc;    /* pinned host, chunk-relative descriptors */
	hipEvent_t h2d_done, compute_done;
};

struct odpg_ctx_s {
	int device;
	hipStream_t stream;
	bool own_stream;
	hipStream_t copy_stream;
	void *ws;          /* per-workgroup counter partials */
	uint64_t *sred;    /* stats_commit scratch (SRED_BYTES, kept zeroed) */
	Stage stage[NSTAGE];
	size_t stage_span;     /* bytes of frames per stage */
	uint32_t stage_chunk;  /* packets per stage (out / desc / mark / meta) */
	uint32_t stage_flags;  /* 1 desc, 2 mark, 4 meta allocated */
	uint64_t *stage_stats;
	uint32_t stage_nstats;
	size_t ws_bytes;
	hipEvent_t ev[NUM_EVENTS];
	int kernel_mode;   /* 0 auto, 1 walk, 2 evaluate-all, 3 hash walk */
	std::mutex lock;
	/* the caller's handle + one per counters / forwarder / fence created on
	 * the context (odpg.h "object lifetimes"): the stream and device memory
	 * are freed when the last of them is released */
	std::atomic<int> refs;
};

static void free_stage(odpg_ctx_t *c);

struct odpg_table_s {
	dtable_hdr_t hdr;
	std::vector<uint8_t> blob;
	void *dblob;
	int device;
	int cycle;
	uint32_t depth;    /* longest rule chain from the default CoS (0: a cycle) */
	uint64_t qsig;     /* counter layout: CoS count, queues and stats flags */
	size_t cap;        /* bytes allocated at dblob */
	hipEvent_t uploaded;   /* the last upload of `blob` has been consumed */
};

/* odpg.h "sharded counters" */
struct odpg_counters_s {
	odpg_ctx_t *ctx;
	uint64_t qsig;
	uint32_t ncos, ncols, words, rows;
	uint32_t any_cos;              /* some CoS has stats_enable */
	uint64_t *drows;               /* device, rows x words */
	uint32_t *dqcol;               /* device, queue column of each CoS */
	uint64_t *dsum;                /* device, words (fold target) */
	uint64_t *hsum;                /* pinned host, words */
	hipEvent_t done;
	std::vector<uint32_t> qcol;    /* host: ncos + 1 prefix of num_queue */
	std::vector<uint8_t> nq;
	std::mutex lock;               /* one fold at a time */
};

/* The longest chain of rules cls_select_cos can follow from the default CoS
 * (odp_classification.c:1599-1631: at CoS c every rule of c may lead to its
 * destination, whose rules are tried next), or 0 when a cycle is reachable.
 * The lean kernel walks exactly that many levels, without a loop. */
static uint32_t table_walk_depth(const odpg_table_t *t)
{
	const dtable_hdr_t &h = t->hdr;
	const dcos_t *hc = (const dcos_t *)(t->blob.data() + h.cos_off);
	const uint32_t *pinfo = (const uint32_t *)(t->blob.data() + h.pinfo_off);
	const int32_t dc = h.default_cos;

	if (dc < 0 || (uint32_t)dc >= h.num_cos || !hc[dc].valid)
		return 1;
	std::vector<uint8_t> state(h.num_cos, 0);     /* 0 new, 1 on path, 2 done */
	std::vector<uint32_t> len(h.num_cos, 0);
	bool cyclic = false;
	/* iterative DFS: longest number of rules from c */
	std::vector<std::pair<uint32_t, uint32_t>> st{{(uint32_t)dc, 0u}};

	state[dc] = 1;
	while (!st.empty() && !cyclic) {
		auto &[c, i] = st.back();

		if (i < hc[c].nrule) {
			const uint32_t k = hc[c].rule_start + i++;
			const uint32_t d = k < h.num_pmr ? (pinfo[k] & 0xffffu) : 0xffffu;

			if (d >= h.num_cos)
				continue;
			if (state[d] == 1) {
				cyclic = true;
			} else if (state[d] == 0) {
				state[d] = 1;
				st.push_back({d, 0u});
			}
		} else {
			uint32_t best = 0;

			for (uint32_t r = 0; r < hc[c].nrule; r++) {
				const uint32_t k = hc[c].rule_start + r;
				const uint32_t d = k < h.num_pmr ? (pinfo[k] & 0xffffu) : 0xffffu;

				if (d < h.num_cos)
					best = std::max(best, 1u + len[d]);
			}
			len[c] = best;
			state[c] = 2;
			st.pop_back();
		}
	}
	return cyclic ? 0u : std::max(len[dc], 1u);
}

/* layout signature of a table's counters: a counters object serves every
 * table with the same CoS count, queue counts and stats flags */
static uint64_t table_qsig(const odpg_table_t *t)
{
	const dcos_t *hc = (const dcos_t *)(t->blob.data() + t->hdr.cos_off);
	uint64_t h = 1469598103934665603ull ^ t->hdr.num_cos;

	for (uint32_t c = 0; c < t->hdr.num_cos; c++) {
		const uint32_t nq = hc[c].num_queue ? hc[c].num_queue : 1u;

		h = (h ^ (nq | ((uint32_t)(hc[c].stats != 0) << 8))) * 1099511628211ull;
	}
	return h;
}

#define HIPCHK(x)                                                              \
	do {                                                                   \
		hipError_t e_ = (x);                                           \
		if (e_ != hipSuccess) {                                        \
			fprintf(stderr, "odpg: %s failed: %s (%s:%d)\n", #x,    \
				hipGetErrorString(e_), __FILE__, __LINE__);    \
			return -EIO;                                           \
		}                                                              \
	} while (0)

extern "C" {

int odpg_abi_version(void)
{
	return ODPG_ABI_VERSION;
}

const char *odpg_build_info(void)
{
	return "odpg gfx950 classifier, ABI 2";
}

int odpg_device_count(void)
{
	int n = 0;

	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

int odpg_ctx_create(int device, void *stream, odpg_ctx_t **out)
{
	if (!out)
		return -EINVAL;
	int n = odpg_device_count();

	if (device < 0 || device >= n)
		return -ENODEV;
	odpg_ctx_t *c = new odpg_ctx_t();

	c->device = device;
	c->ws = nullptr;
	c->ws_bytes = 0;
	c->kernel_mode = 0;
	c->refs.store(1);
	if (hipSetDevice(device) != hipSuccess) {
		delete c;
		return -EIO;
	}
	if (stream) {
		c->stream = (hipStream_t)stream;
		c->own_stream = false;
	} else {
		if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
			delete c;
			return -EIO;
		}
		c->own_stream = true;
	}
	if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) {
		delete c;
		return -EIO;
	}
	for (int k = 0; k < NUM_EVENTS; k++)
		if (hipEventCreate(&c->ev[k]) != hipSuccess) {
			delete c;
			return -EIO;
		}
	if (hipMalloc(&c->sred, SRED_BYTES) != hipSuccess ||
	    hipMemset(c->sred, 0, SRED_BYTES) != hipSuccess) {
		delete c;
		return -EIO;
	}
	for (int k = 0; k < NSTAGE; k++)
		if (hipEventCreateWithFlags(&c->stage[k].h2d_done, hipEventDisableTiming) != hipSuccess ||
		    hipEventCreateWithFlags(&c->stage[k].compute_done, hipEventDisableTiming) != hipSuccess) {
			delete c;
			return -EIO;
		}
	*out = c;
	return 0;
}

/* the context's resources, once nothing refers to it any more */
static void ctx_free(odpg_ctx_t *c)
{
	hipSetDevice(c->device);
	hipStreamSynchronize(c->stream);
	hipStreamSynchronize(c->copy_stream);
	if (c->ws)
		hipFree(c->ws);
	hipFree(c->sred);
	free_stage(c);
	hipFree(c->stage_stats);
	for (int k = 0; k < NSTAGE; k++) {
		hipEventDestroy(c->stage[k].h2d_done);
		hipEventDestroy(c->stage[k].compute_done);
	}
	for (int k = 0; k < NUM_EVENTS; k++)
		hipEventDestroy(c->ev[k]);
	hipStreamDestroy(c->copy_stream);
	if (c->own_stream)
		hipStreamDestroy(c->stream);
	delete c;
}

void odpg_ctx_ref(odpg_ctx_t *c)
{
	c->refs.fetch_add(1);
}

void odpg_ctx_unref(odpg_ctx_t *c)
{
	if (c->refs.fetch_sub(1) == 1)
		ctx_free(c);
}

void odpg_ctx_destroy(odpg_ctx_t *c)
{
	if (!c)
		return;
	/* the odp_cls bindings on this context go now (their counters and
	 * tables); objects the caller still holds keep the context alive */
	odpg_cls_ctx_release(c);
	odpg_ctx_unref(c);
}

int odpg_ctx_set_kernel_mode(odpg_ctx_t *c, int mode)
{
	if (!c || mode < 0 || mode > 3)
		return -EINVAL;
	c->kernel_mode = mode;
	return 0;
}

void *odpg_ctx_stream(odpg_ctx_t *c)
{
	return c ? (void *)c->stream : nullptr;
}

int odpg_ctx_sync(odpg_ctx_t *c)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

/* compiled-table image: this header, dtable_hdr_t, then the blob */
struct table_image_hdr {
	uint32_t magic;        /* IMAGE_MAGIC */
	uint32_t abi;          /* ODPG_ABI_VERSION */
	uint32_t hdr_bytes;    /* sizeof(dtable_hdr_t) */
	uint32_t blob_bytes;
};
#define IMAGE_MAGIC 0x5450444fu   /* "ODPT" in memory order */

int odpg_rules_compile(const odpg_rules_t *rules, void *image, size_t *size)
{
	if (!rules || !size)
		return -EINVAL;
	std::vector<uint8_t> blob;
	dtable_hdr_t hdr;
	int rc = odpg_compile_rules(rules, blob, &hdr);

	if (rc)
		return rc;
	const size_t need = sizeof(table_image_hdr) + sizeof(dtable_hdr_t) + hdr.blob_bytes;

	if (!image || *size < need) {
		*size = need;
		return -ENOSPC;
	}
	table_image_hdr ih = {IMAGE_MAGIC, ODPG_ABI_VERSION, (uint32_t)sizeof(dtable_hdr_t),
			      hdr.blob_bytes};
	uint8_t *o = (uint8_t *)image;

	memcpy(o, &ih, sizeof(ih));
	memcpy(o + sizeof(ih), &hdr, sizeof(hdr));
	memcpy(o + sizeof(ih) + sizeof(hdr), blob.data(), hdr.blob_bytes);
	*size = need;
	return 0;
}

/* a compiled table (host blob + header) onto the context's device */
static int table_upload(odpg_ctx_t *c, odpg_table_t *t, odpg_table_t **out)
{
	t->cycle = odpg_rules_has_cycle(t->blob, t->hdr);
	t->depth = table_walk_depth(t);
	t->device = c->device;
	t->qsig = table_qsig(t);
	t->uploaded = nullptr;
	hipSetDevice(c->device);
	if (hipMalloc(&t->dblob, t->hdr.blob_bytes) != hipSuccess) {
		delete t;
		return -ENOMEM;
	}
	t->cap = t->hdr.blob_bytes;
	if (hipMemcpyAsync(t->dblob, t->blob.data(), t->hdr.blob_bytes, hipMemcpyHostToDevice,
			   c->stream) != hipSuccess ||
	    hipStreamSynchronize(c->stream) != hipSuccess) {
		hipFree(t->dblob);
		delete t;
		return -EIO;
	}
	*out = t;
	return 0;
}

int odpg_table_import(odpg_ctx_t *c, const void *image, size_t size, odpg_table_t **out)
{
	if (!c || !image || !out || size < sizeof(table_image_hdr))
		return -EINVAL;
	table_image_hdr ih;

	memcpy(&ih, image, sizeof(ih));
	if (ih.magic != IMAGE_MAGIC || ih.abi != ODPG_ABI_VERSION ||
	    ih.hdr_bytes != sizeof(dtable_hdr_t) ||
	    size != sizeof(ih) + sizeof(dtable_hdr_t) + (size_t)ih.blob_bytes)
		return -EINVAL;
	odpg_table_t *t = new odpg_table_t();

	memcpy(&t->hdr, (const uint8_t *)image + sizeof(ih), sizeof(dtable_hdr_t));
	if (t->hdr.blob_bytes != ih.blob_bytes) {
		delete t;
		return -EINVAL;
	}
	t->blob.assign((const uint8_t *)image + sizeof(ih) + sizeof(dtable_hdr_t),
		       (const uint8_t *)image + size);
	return table_upload(c, t, out);
}

int odpg_table_create(odpg_ctx_t *c, const odpg_rules_t *rules, odpg_table_t **out)
{
	if (!c || !rules || !out)
		return -EINVAL;
	odpg_table_t *t = new odpg_table_t();
	int rc = odpg_compile_rules(rules, t->blob, &t->hdr);

	if (rc) {
		delete t;
		return rc;
	}
	return table_upload(c, t, out);
}

int odpg_table_update(odpg_ctx_t *c, odpg_table_t *t, const odpg_rules_t *rules)
{
	if (!c || !t || !rules)
		return -EINVAL;
	if (t->device != c->device)
		return -EXDEV;
	std::vector<uint8_t> blob;
	dtable_hdr_t hdr;
	int rc = odpg_compile_rules(rules, blob, &hdr);

	if (rc)
		return rc;
	std::lock_guard<std::mutex> g(c->lock);

	hipSetDevice(c->device);
	/* the previous upload read t->blob asynchronously */
	if (t->uploaded && hipEventSynchronize(t->uploaded) != hipSuccess)
		return -EIO;
	if (!t->uploaded && hipEventCreateWithFlags(&t->uploaded, hipEventDisableTiming) != hipSuccess)
		return -EIO;
	if (hdr.blob_bytes > t->cap) {
		void *nb = nullptr;

		/* launches still reading the old allocation end first */
		if (hipStreamSynchronize(c->stream) != hipSuccess ||
		    hipMalloc(&nb, hdr.blob_bytes) != hipSuccess)
			return -ENOMEM;
		hipFree(t->dblob);
		t->dblob = nb;
		t->cap = hdr.blob_bytes;
	}
	t->blob.swap(blob);
	t->hdr = hdr;
	t->cycle = odpg_rules_has_cycle(t->blob, t->hdr);
	t->depth = table_walk_depth(t);
	t->qsig = table_qsig(t);
	if (hipMemcpyAsync(t->dblob, t->blob.data(), t->hdr.blob_bytes, hipMemcpyHostToDevice,
			   c->stream) != hipSuccess ||
	    hipEventRecord(t->uploaded, c->stream) != hipSuccess)
		return -EIO;
	return 0;
}

void odpg_table_destroy(odpg_table_t *t)
{
	if (!t)
		return;
	hipSetDevice(t->device);
	if (t->uploaded) {
		hipEventSynchronize(t->uploaded);
		hipEventDestroy(t->uploaded);
	}
	hipFree(t->dblob);
	delete t;
}

uint32_t odpg_table_num_cos(const odpg_table_t *t)
{
	return t ? t->hdr.num_cos : 0;
}

int odpg_table_has_cycle(const odpg_table_t *t)
{
	return t ? t->cycle : 0;
}

/* ---- sharded counters ---------------------------------------------------- */
#define CNT_ROWS_PER_CU 8u
#define CNT_MAX_BYTES   (512ull << 20)
#define CNT_MAX_LDS     (48u << 10)   /* LDS histograms of one workgroup */

extern "C" int odpg_launch_counters_fold(uint64_t *rows, uint32_t nrows, uint32_t words,
					 uint64_t *sum, hipStream_t s);

static void counters_free(odpg_counters_t *k)
{
	odpg_ctx_t *c = k->ctx;

	hipFree(k->drows);
	hipFree(k->dqcol);
	hipFree(k->dsum);
	if (k->hsum)
		hipHostFree(k->hsum);
	if (k->done)
		hipEventDestroy(k->done);
	delete k;
	odpg_ctx_unref(c);
}

int odpg_counters_create(odpg_ctx_t *c, const odpg_table_t *t, odpg_counters_t **out)
{
	if (!c || !t || !out)
		return -EINVAL;
	if (t->device != c->device)
		return -EXDEV;
	const dtable_hdr_t &h = t->hdr;
	const dcos_t *hc = (const dcos_t *)(t->blob.data() + h.cos_off);
	odpg_counters_t *k = new odpg_counters_t();

	k->ctx = c;
	odpg_ctx_ref(c);
	k->qsig = t->qsig;
	k->ncos = h.num_cos;
	k->qcol.resize(h.num_cos + 1u);
	k->nq.resize(h.num_cos);
	uint32_t col = 0;

	for (uint32_t i = 0; i < h.num_cos; i++) {
		k->qcol[i] = col;
		k->nq[i] = (uint8_t)(hc[i].num_queue ? hc[i].num_queue : 1u);
		col += k->nq[i];
		k->any_cos |= hc[i].stats ? 1u : 0u;
	}
	k->qcol[h.num_cos] = col;
	k->ncols = col;
	k->words = 4u + k->ncos + k->ncols;
	if (((size_t)k->ncos + k->ncols) * 4u > CNT_MAX_LDS) {
		counters_free(k);
		return -E2BIG;
	}
	int cus = 0;

	hipSetDevice(c->device);
	if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
	    cus <= 0)
		cus = 256;
	k->rows = (uint32_t)cus * CNT_ROWS_PER_CU;
	while (k->rows > (uint32_t)cus && (size_t)k->rows * k->words * 8u > CNT_MAX_BYTES)
		k->rows >>= 1;
	if ((size_t)k->rows * k->words * 8u > CNT_MAX_BYTES) {
		counters_free(k);
		return -E2BIG;
	}
	const size_t rb = (size_t)k->rows * k->words * 8u;

	if (hipMalloc(&k->drows, rb) != hipSuccess ||
	    hipMalloc(&k->dqcol, (size_t)(k->ncos + 1u) * 4u) != hipSuccess ||
	    hipMalloc(&k->dsum, (size_t)k->words * 8u) != hipSuccess ||
	    hipHostMalloc(&k->hsum, (size_t)k->words * 8u, hipHostMallocDefault) != hipSuccess ||
	    hipEventCreateWithFlags(&k->done, hipEventDisableTiming) != hipSuccess) {
		counters_free(k);
		return -ENOMEM;
	}
	{
		std::lock_guard<std::mutex> g(c->lock);

		if (hipMemsetAsync(k->drows, 0, rb, c->stream) != hipSuccess ||
		    hipMemsetAsync(k->dsum, 0, (size_t)k->words * 8u, c->stream) != hipSuccess ||
		    hipMemcpyAsync(k->dqcol, k->qcol.data(), (size_t)(k->ncos + 1u) * 4u,
				   hipMemcpyHostToDevice, c->stream) != hipSuccess ||
		    hipEventRecord(k->done, c->stream) != hipSuccess) {
			counters_free(k);
			return -EIO;
		}
	}
	if (hipEventSynchronize(k->done) != hipSuccess) {
		counters_free(k);
		return -EIO;
	}
	*out = k;
	return 0;
}

int odpg_counters_match(const odpg_counters_t *k, const odpg_table_t *t)
{
	return k && t && k->qsig == t->qsig && k->ncos == t->hdr.num_cos;
}

void odpg_counters_destroy(odpg_counters_t *k)
{
	if (!k)
		return;
	hipSetDevice(k->ctx->device);
	hipStreamSynchronize(k->ctx->stream);   /* launches still adding into the rows */
	counters_free(k);
}

int odpg_counters_fold(odpg_counters_t *k, uint64_t *words)
{
	if (!k || !words)
		return -EINVAL;
	odpg_ctx_t *c = k->ctx;
	std::lock_guard<std::mutex> fl(k->lock);

	hipSetDevice(c->device);
	{
		/* enqueue behind every launch already on the context stream */
		std::lock_guard<std::mutex> g(c->lock);

		if (odpg_launch_counters_fold(k->drows, k->rows, k->words, k->dsum, c->stream) ||
		    hipMemcpyAsync(k->hsum, k->dsum, (size_t)k->words * 8u, hipMemcpyDeviceToHost,
				   c->stream) != hipSuccess ||
		    hipMemsetAsync(k->dsum, 0, (size_t)k->words * 8u, c->stream) != hipSuccess ||
		    hipEventRecord(k->done, c->stream) != hipSuccess)
			return -EIO;
	}
	HIPCHK(hipEventSynchronize(k->done));
	for (uint32_t w = 0; w < 4u + k->ncos; w++)
		words[w] += k->hsum[w];
	const uint64_t *dl = k->hsum + 4u + k->ncos;
	uint64_t *uq = words + 4u + k->ncos;

	for (uint32_t i = 0; i < k->ncos; i++)
		for (uint32_t q = 0; q < k->nq[i]; q++)
			uq[(size_t)i * ODPG_COS_QUEUE_MAX + q] += dl[k->qcol[i] + q];
	return 0;
}

static int ensure_ws(odpg_ctx_t *c, size_t bytes)
{
	if (c->ws_bytes >= bytes)
		return 0;
	if (c->ws) {
		HIPCHK(hipStreamSynchronize(c->stream));
		HIPCHK(hipFree(c->ws));
		c->ws = nullptr;
		c->ws_bytes = 0;
	}
	HIPCHK(hipMalloc(&c->ws, bytes));
	c->ws_bytes = bytes;
	return 0;
}

static int validate_batch(const odpg_batch_t *b)
{
	if (!b)
		return -EINVAL;
	if (b->num && !b->frames)
		return -EINVAL;
	if (!b->desc && (b->stride == 0 || (b->stride & 15u)))
		return -EINVAL;
	if (b->layer > 4)
		return -EINVAL;
	return 0;
}

static int classify_on(odpg_ctx_t *c, hipStream_t s, const odpg_table_t *t,
		       const odpg_batch_t *b, const odpg_result_t *r, void *ws)
{
	odpg_launch_args a;
	const dtable_hdr_t &h = t->hdr;
	uint32_t grid = odpg_launch_grid(b->num);
	bool cos_stats = r->stats && (h.flags & TBL_ANY_STATS);

	memset(&a, 0, sizeof(a));
	a.frames = b->frames;
	a.desc = b->desc;
	a.stride = b->stride;
	a.num = b->num;
	a.opt = b->pktin_opt;
	a.layer = b->layer;
	a.classify = b->classify;
	a.terms = (const dterm_t *)((const uint8_t *)t->dblob + h.term_off);
	a.pmrs = (const dpmr_t *)((const uint8_t *)t->dblob + h.pmr_off);
	a.coses = (const dcos_t *)((const uint8_t *)t->dblob + h.cos_off);
	a.num_cos = h.num_cos;
	a.default_cos = h.default_cos;
	a.error_cos = h.error_cos;
	a.tbl_flags = h.flags;
	a.num_pmr = h.num_pmr;
	a.slot_mask = h.slot_mask;
	a.slots = (const dslot_t *)((const uint8_t *)t->dblob + h.slot_off);
	a.simple = (const dsimple_t *)((const uint8_t *)t->dblob + h.simple_off);
	a.runs = (const drun_t *)((const uint8_t *)t->dblob + h.run_off);
	a.num_runs = h.num_runs;
	a.hgroups = (const dhgroup_t *)((const uint8_t *)t->dblob + h.hgroup_off);
	a.num_hgroups = h.num_hgroups;
	a.hents = (const dhent_t *)((const uint8_t *)t->dblob + h.hent_off);
	a.num_hent = h.num_hent;
	a.cinfo = (const uint2_t *)((const uint8_t *)t->dblob + h.cinfo_off);
	a.pinfo = (const uint32_t *)((const uint8_t *)t->dblob + h.pinfo_off);
	a.wgroups = (const dhgroup_t *)((const uint8_t *)t->dblob + h.wgroup_off);
	a.num_wgroups = h.num_wgroups;
	a.wents = (const dwent_t *)((const uint8_t *)t->dblob + h.went_off);
	a.num_went = h.num_went;
	a.mgroups = (const dmgroup_t *)((const uint8_t *)t->dblob + h.mgroup_off);
	a.num_mgroups = h.num_mgroups;
	a.ments = (const dment_t *)((const uint8_t *)t->dblob + h.ment_off);
	a.num_ment = h.num_ment;
	a.pinfo2 = (const uint2_t *)((const uint8_t *)t->dblob + h.pinfo2_off);
	a.cgroups = (const dmgroup_t *)((const uint8_t *)t->dblob + h.cgroup_off);
	a.num_cgroups = h.num_cgroups;
	a.cents = (const dwent_t *)((const uint8_t *)t->dblob + h.cent_off);
	a.num_cent = h.num_cent;
	a.pinfo3 = (const uint2_t *)((const uint8_t *)t->dblob + h.pinfo3_off);
	a.pinfo4 = (const uint32_t *)((const uint8_t *)t->dblob + h.pinfo4_off);
	a.def_cgmask = h.def_cgmask;
	a.xcos = (const uint2_t *)((const uint8_t *)t->dblob + h.xcos_off);
	a.xlist = (const uint32_t *)((const uint8_t *)t->dblob + h.xlist_off);
	a.num_xlist = h.num_xlist;
	a.num_xwords = h.num_xwords;
	a.xm = (const uint32_t *)((const uint8_t *)t->dblob + h.xm_off);
	a.num_xment = h.num_xment;
	a.xm_slot_bytes = h.xm_slot_bytes;
	a.num_xflat = h.num_xflat;
	a.xm_nw = h.xm_nw;
	a.xm_nbits = h.xm_nbits;
	a.xm_ngroups = h.xm_ngroups;
	a.xm_kx = h.xm_kx;
	{
		/* start state of cls_select_cos (odp_classification.c:1669-1701)
		 * for the lean kernel, as classify.hip derives it per packet */
		const dcos_t *hc = (const dcos_t *)(t->blob.data() + h.cos_off);
		const int32_t dc = h.default_cos, ec = h.error_cos;
		const bool dvalid = dc >= 0 && (uint32_t)dc < h.num_cos && hc[dc].valid;

		a.l64_err_cos = ec < 0 ? ODPG_COS_NONE : (uint32_t)ec;
		a.l64_err_act = ec >= 0 && (uint32_t)ec < h.num_cos ? hc[ec].action : 0u;
		a.l64_def_cos = dc < 0 ? ODPG_COS_NONE : (uint32_t)dc;
		a.l64_def_act = dc >= 0 && (uint32_t)dc < h.num_cos ? hc[dc].action : 0u;
		a.l64_def_rules = dvalid && hc[dc].nrule;
		a.l64_def_ci = dvalid && hc[dc].nrule ?
			       (hc[dc].rule_start & 0xffu) | ((uint32_t)(hc[dc].nrule & 0xffu) << 8) : 0u;
		const uint64_t dm = dvalid && hc[dc].nrule && hc[dc].rule_start < 64u ?
				    (hc[dc].nrule >= 64u ? ~0ull : ((1ull << hc[dc].nrule) - 1ull))
				    << hc[dc].rule_start : 0ull;

		a.l64_depth = t->depth;
		a.l64_def_mlo = (uint32_t)dm;
		a.l64_def_mhi = (uint32_t)(dm >> 32);
	}
	a.mode = c->kernel_mode;
	a.out = r->out;
	a.mark = r->mark;
	a.meta = r->meta;
	a.stats = r->stats;
	if (r->counters) {
		odpg_counters_t *k = r->counters;

		a.cnt.row = k->drows;
		a.cnt.qcol = k->dqcol;
		a.cnt.words = k->words;
		a.cnt.rows = k->rows;
		a.cnt.ncos = k->ncos;
		a.cnt.ncols = k->ncols;
		a.cnt.cos = k->any_cos;
	} else if (r->stats && !cos_stats) {
		/* pktio counters only: workgroups add straight into them */
		a.pk_partial = r->stats;
		a.pk_atomic = 1u;
		a.sred = c->sred;
	} else if (r->stats) {
		a.pk_partial = (uint64_t *)ws;
		a.cos_partial = (uint32_t *)((uint8_t *)ws + (size_t)grid * 32u);
	}
	return odpg_launch_classify(&a, s);
}

static void free_stage(odpg_ctx_t *c)
{
	for (int k = 0; k < NSTAGE; k++) {
		Stage &B = c->stage[k];

		hipFree(B.frames);
		hipFree(B.desc);
		hipFree(B.out);
		hipFree(B.mark);
		hipFree(B.meta);
		if (B.hdesc)
			hipHostFree(B.hdesc);
		B.frames = nullptr;
		B.desc = nullptr;
		B.out = nullptr;
		B.mark = nullptr;
		B.meta = nullptr;
		B.hdesc = nullptr;
	}
	c->stage_span = 0;
	c->stage_chunk = 0;
	c->stage_flags = 0;
}

/* grow-only staging for odpg_classify_host */
static int ensure_stage(odpg_ctx_t *c, size_t span, uint32_t chunk, bool desc, bool mark,
			bool meta, uint32_t nstats)
{
	const uint32_t want = (desc ? 1u : 0u) | (mark ? 2u : 0u) | (meta ? 4u : 0u);

	if (c->stage_span < span + 16 || c->stage_chunk < chunk ||
	    (c->stage_flags & want) != want) {
		HIPCHK(hipStreamSynchronize(c->stream));
		HIPCHK(hipStreamSynchronize(c->copy_stream));
		const size_t nspan = span + 16 > c->stage_span ? span + 16 : c->stage_span;
		const uint32_t nchunk = chunk > c->stage_chunk ? chunk : c->stage_chunk;
		const uint32_t flags = want | c->stage_flags;

		free_stage(c);
		for (int k = 0; k < NSTAGE; k++) {
			Stage &B = c->stage[k];

			if (hipMalloc(&B.frames, nspan) != hipSuccess ||
			    hipMalloc(&B.out, (size_t)nchunk * sizeof(odpg_out_t)) != hipSuccess ||
			    ((flags & 1u) && (hipMalloc(&B.desc, (size_t)nchunk * sizeof(odpg_desc_t)) != hipSuccess ||
					      hipHostMalloc(&B.hdesc, (size_t)nchunk * sizeof(odpg_desc_t),
							    hipHostMallocDefault) != hipSuccess)) ||
			    ((flags & 2u) && hipMalloc(&B.mark, (size_t)nchunk * 2u) != hipSuccess) ||
			    ((flags & 4u) && hipMalloc(&B.meta, (size_t)nchunk * sizeof(odpg_meta_t)) != hipSuccess)) {
				free_stage(c);
				return -ENOMEM;
			}
		}
		c->stage_span = nspan;
		c->stage_chunk = nchunk;
		c->stage_flags = flags;
	}
	if (nstats > c->stage_nstats) {
		HIPCHK(hipStreamSynchronize(c->stream));
		hipFree(c->stage_stats);
		c->stage_stats = nullptr;
		c->stage_nstats = 0;
		if (hipMalloc(&c->stage_stats, nstats * 8u) != hipSuccess)
			return -ENOMEM;
		c->stage_nstats = nstats;
	}
	return 0;
}

static size_t ws_need(const odpg_table_t *t, uint32_t num, bool stats)
{
	if (!stats)
		return 0;
	if (!(t->hdr.flags & TBL_ANY_STATS))
		return 0;   /* pktio counters only: added in place */
	uint32_t grid = odpg_launch_grid(num);

	return (size_t)grid * 32u + (size_t)grid * t->hdr.num_cos * 4u;
}

/* a counters object serves launches on its own context (its rows are
 * updated with plain read-modify-writes, stream-ordered) and tables of its
 * layout; not together with the caller's stats block */
static int check_counters(const odpg_ctx_t *c, const odpg_table_t *t, const odpg_result_t *r)
{
	const odpg_counters_t *k = r->counters;

	if (!k)
		return 0;
	if (r->stats || k->ctx != c || k->qsig != t->qsig || k->ncos != t->hdr.num_cos)
		return -EINVAL;
	return 0;
}

int odpg_classify(odpg_ctx_t *c, const odpg_table_t *t, const odpg_batch_t *b,
		  const odpg_result_t *r)
{
	int rc;

	if (!c || !t || !r || (b && b->num && !r->out))
		return -EINVAL;
	if ((rc = validate_batch(b)))
		return rc;
	if (t->device != c->device)
		return -EXDEV;
	if ((rc = check_counters(c, t, r)))
		return rc;
	if (b->num == 0)
		return 0;
	std::lock_guard<std::mutex> g(c->lock);

	hipSetDevice(c->device);
	if ((rc = ensure_ws(c, ws_need(t, b->num, r->stats != nullptr))))
		return rc;
	return classify_on(c, c->stream, t, b, r, c->ws);
}

/* Host-buffer path: frames/desc/results in host memory (pinned is fastest).
 * Two device buffer sets alternate between the copy stream (H2D) and the
 * compute stream (kernel + D2H). */
int odpg_classify_host(odpg_ctx_t *c, const odpg_table_t *t, const odpg_batch_t *b,
		       const odpg_result_t *r, uint32_t chunk)
{
	int rc;

	if (!c || !t || !r || (b && b->num && !r->out))
		return -EINVAL;
	if ((rc = validate_batch(b)))
		return rc;
	if (t->device != c->device)
		return -EXDEV;
	if ((rc = check_counters(c, t, r)))
		return rc;
	if (b->num == 0)
		return 0;
	if (chunk == 0)
		chunk = 1u << 18;
	if (chunk > b->num)
		chunk = b->num;
	std::lock_guard<std::mutex> g(c->lock);

	hipSetDevice(c->device);

	/* size the frame staging buffers */
	size_t max_span = 0;
	uint32_t nchunks = (b->num + chunk - 1) / chunk;
	std::vector<size_t> span_lo(nchunks), span_hi(nchunks);

	for (uint32_t k = 0; k < nchunks; k++) {
		uint32_t first = k * chunk, n = b->num - first < chunk ? b->num - first : chunk;
		size_t lo, hi;

		if (b->desc) {
			lo = (size_t)-1;
			hi = 0;
			for (uint32_t j = first; j < first + n; j++) {
				size_t o = b->desc[j].offset, e = o + b->desc[j].len;

				if (o & 15u)
					return -EINVAL;
				lo = o < lo ? o : lo;
				e = (e + 15u) & ~(size_t)15u;
				hi = e > hi ? e : hi;
			}
		} else {
			lo = (size_t)first * b->stride;
			hi = lo + (size_t)n * b->stride;
		}
		span_lo[k] = lo;
		span_hi[k] = hi;
		if (hi - lo > max_span)
			max_span = hi - lo;
	}

	uint32_t nstats = ODPG_STATS_WORDS(t->hdr.num_cos);
	int err = 0;

	if ((err = ensure_stage(c, max_span, chunk, b->desc != nullptr, r->mark != nullptr,
				r->meta != nullptr, r->stats ? nstats : 0u)))
		return err;
	if (r->stats && hipMemsetAsync(c->stage_stats, 0, nstats * 8u, c->stream) != hipSuccess)
		return -EIO;
	err = ensure_ws(c, ws_need(t, chunk, r->stats != nullptr));

	for (uint32_t k = 0; k < nchunks && !err; k++) {
		Stage &B = c->stage[k % NSTAGE];
		uint32_t first = k * chunk, n = b->num - first < chunk ? b->num - first : chunk;
		size_t lo = span_lo[k], bytes = span_hi[k] - span_lo[k];

		/* buffer reuse: the copy stream waits until the chunk that used this
		 * stage has been classified and its results copied back */
		if (k >= NSTAGE && hipStreamWaitEvent(c->copy_stream, B.compute_done, 0) != hipSuccess) {
			err = -EIO;
			break;
		}
		if (hipMemcpyAsync(B.frames, b->frames + lo, bytes, hipMemcpyHostToDevice,
				   c->copy_stream) != hipSuccess) {
			err = -EIO;
			break;
		}
		if (b->desc) {
			/* chunk-relative descriptors, staged through a pinned buffer
			 * the host rewrites once the stage's previous chunk is done */
			if (k >= NSTAGE)
				hipEventSynchronize(B.compute_done);
			for (uint32_t j = 0; j < n; j++) {
				B.hdesc[j].offset = (uint32_t)(b->desc[first + j].offset - lo);
				B.hdesc[j].len = b->desc[first + j].len;
			}
			if (hipMemcpyAsync(B.desc, B.hdesc, (size_t)n * sizeof(odpg_desc_t),
					   hipMemcpyHostToDevice, c->copy_stream) != hipSuccess) {
				err = -EIO;
				break;
			}
		}
		hipEventRecord(B.h2d_done, c->copy_stream);
		hipStreamWaitEvent(c->stream, B.h2d_done, 0);

		odpg_batch_t cb = *b;
		odpg_result_t cr;

		cb.frames = B.frames;
		cb.desc = b->desc ? B.desc : nullptr;
		cb.num = n;
		cr.out = B.out;
		cr.mark = r->mark ? B.mark : nullptr;
		cr.meta = r->meta ? B.meta : nullptr;
		cr.stats = r->stats ? c->stage_stats : nullptr;
		cr.counters = r->counters;
		if (classify_on(c, c->stream, t, &cb, &cr, c->ws)) {
			err = -EIO;
			break;
		}
		hipMemcpyAsync(r->out + first, B.out, (size_t)n * sizeof(odpg_out_t),
			       hipMemcpyDeviceToHost, c->stream);
		if (r->mark)
			hipMemcpyAsync(r->mark + first, B.mark, (size_t)n * 2u, hipMemcpyDeviceToHost,
				       c->stream);
		if (r->meta)
			hipMemcpyAsync(r->meta + first, B.meta, (size_t)n * sizeof(odpg_meta_t),
				       hipMemcpyDeviceToHost, c->stream);
		hipEventRecord(B.compute_done, c->stream);
	}
	if (!err && r->stats) {
		std::vector<uint64_t> hs(nstats);

		if (hipMemcpyAsync(hs.data(), c->stage_stats, nstats * 8u, hipMemcpyDeviceToHost,
				   c->stream) != hipSuccess ||
		    hipStreamSynchronize(c->stream) != hipSuccess)
			err = -EIO;
		else
			for (uint32_t k = 0; k < nstats; k++)
				r->stats[k] += hs[k];
	}
	if (hipStreamSynchronize(c->stream) != hipSuccess ||
	    hipStreamSynchronize(c->copy_stream) != hipSuccess)
		err = err ? err : -EIO;
	return err;
}

int odpg_dev_alloc(odpg_ctx_t *c, size_t bytes, void **ptr)
{
	if (!c || !ptr)
		return -EINVAL;
	hipSetDevice(c->device);
	if (hipMalloc(ptr, bytes ? bytes : 16) != hipSuccess)
		return -ENOMEM;
	return 0;
}

int odpg_dev_free(odpg_ctx_t *c, void *ptr)
{
	if (!c)
		return -EINVAL;
	hipSetDevice(c->device);
	HIPCHK(hipFree(ptr));
	return 0;
}

int odpg_host_alloc_pinned(size_t bytes, void **ptr)
{
	if (!ptr)
		return -EINVAL;
	if (hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess)
		return -ENOMEM;
	return 0;
}

int odpg_host_device_ptr(void *host_ptr, void **dev_ptr)
{
	if (!host_ptr || !dev_ptr)
		return -EINVAL;
	if (hipHostGetDevicePointer(dev_ptr, host_ptr, 0) != hipSuccess)
		return -EINVAL;
	return 0;
}

int odpg_host_free_pinned(void *ptr)
{
	if (!ptr)
		return 0;
	HIPCHK(hipHostFree(ptr));
	return 0;
}

int odpg_memcpy_h2d(odpg_ctx_t *c, void *dst, const void *src, size_t bytes)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

int odpg_memcpy_d2h(odpg_ctx_t *c, void *dst, const void *src, size_t bytes)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

int odpg_memset_dev(odpg_ctx_t *c, void *dst, int value, size_t bytes)
{
	if (!c)
		return -EINVAL;
	HIPCHK(hipMemsetAsync(dst, value, bytes, c->stream));
	return 0;
}

int odpg_event_record(odpg_ctx_t *c, int slot)
{
	if (!c || slot < 0 || slot >= NUM_EVENTS)
		return -EINVAL;
	HIPCHK(hipEventRecord(c->ev[slot], c->stream));
	return 0;
}

struct odpg_fence_s {
	hipEvent_t ev;
	int device;
	odpg_ctx_t *ctx;   /* referenced: any destroy order (odpg.h) */
};

int odpg_fence_create(odpg_ctx_t *c, odpg_fence_t **fence)
{
	if (!c || !fence)
		return -EINVAL;
	odpg_fence_t *f = new (std::nothrow) odpg_fence_t;

	if (!f)
		return -ENOMEM;
	f->device = c->device;
	f->ctx = c;
	hipSetDevice(c->device);
	if (hipEventCreateWithFlags(&f->ev, hipEventDisableTiming) != hipSuccess) {
		delete f;
		return -EIO;
	}
	odpg_ctx_ref(c);
	*fence = f;
	return 0;
}

int odpg_fence_record(odpg_ctx_t *c, odpg_fence_t *f)
{
	if (!c || !f || f->device != c->device)
		return -EINVAL;
	HIPCHK(hipEventRecord(f->ev, c->stream));
	return 0;
}

int odpg_fence_query(odpg_fence_t *f)
{
	if (!f)
		return -EINVAL;
	const hipError_t e = hipEventQuery(f->ev);

	return e == hipSuccess ? 1 : e == hipErrorNotReady ? 0 : -EIO;
}

int odpg_fence_wait(odpg_fence_t *f)
{
	if (!f)
		return -EINVAL;
	HIPCHK(hipEventSynchronize(f->ev));
	return 0;
}

void odpg_fence_destroy(odpg_fence_t *f)
{
	if (!f)
		return;
	hipSetDevice(f->device);
	hipEventDestroy(f->ev);
	odpg_ctx_unref(f->ctx);
	delete f;
}

int odpg_event_elapsed_ms(odpg_ctx_t *c, int a, int b, float *ms)
{
	if (!c || !ms || a < 0 || b < 0 || a >= NUM_EVENTS || b >= NUM_EVENTS)
		return -EINVAL;
	HIPCHK(hipEventSynchronize(c->ev[b]));
	HIPCHK(hipEventElapsedTime(ms, c->ev[a], c->ev[b]));
	return 0;
}

} /* extern "C" */
