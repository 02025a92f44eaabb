/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Device groups (include/odpg_group.h): one batch classified by several
 * device contexts of one process, sharded by packet range. Host code only:
 * every device operation goes through the single-context C-ABI (odpg.h),
 * one context per member, so each member's launches run on its own device
 * and stream. The table image is compiled once and imported per member; the
 * per-member counters are folded and summed on the host when read.
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <thread>
#include <vector>

#include "../../include/odpg.h"
#include "../../include/odpg_group.h"

#define GROUP_MAX 64u

struct odpg_group_s {
	std::vector<odpg_ctx_t *> ctx;
	std::vector<odpg_table_t *> tbl;
	std::vector<odpg_counters_t *> cnt;
	/* counts folded from earlier generations (same CoS count) */
	std::vector<uint64_t> acc;
	uint32_t num_cos = 0;
	std::mutex lock;
};

static void drop_tables(odpg_group_t *g)
{
	for (odpg_counters_t *&c : g->cnt) {
		odpg_counters_destroy(c);
		c = nullptr;
	}
	for (odpg_table_t *&t : g->tbl) {
		odpg_table_destroy(t);
		t = nullptr;
	}
}

extern "C" int odpg_group_create(const int *devices, uint32_t n, odpg_group_t **grp)
{
	if (!devices || !grp || n == 0 || n > GROUP_MAX)
		return -EINVAL;
	odpg_group_t *g = new (std::nothrow) odpg_group_t;

	if (!g)
		return -ENOMEM;
	for (uint32_t i = 0; i < n; i++) {
		odpg_ctx_t *c = nullptr;
		const int rc = odpg_ctx_create(devices[i], nullptr, &c);

		if (rc) {
			odpg_group_destroy(g);
			return rc;
		}
		g->ctx.push_back(c);
	}
	g->tbl.assign(n, nullptr);
	g->cnt.assign(n, nullptr);
	*grp = g;
	return 0;
}

extern "C" void odpg_group_destroy(odpg_group_t *g)
{
	if (!g)
		return;
	drop_tables(g);
	for (odpg_ctx_t *c : g->ctx)
		odpg_ctx_destroy(c);
	delete g;
}

extern "C" uint32_t odpg_group_size(const odpg_group_t *g)
{
	return g ? (uint32_t)g->ctx.size() : 0u;
}

extern "C" odpg_ctx_t *odpg_group_ctx(odpg_group_t *g, uint32_t i)
{
	return g && i < g->ctx.size() ? g->ctx[i] : nullptr;
}

extern "C" odpg_table_t *odpg_group_table(odpg_group_t *g, uint32_t i)
{
	return g && i < g->tbl.size() ? g->tbl[i] : nullptr;
}

/* the members' counters into g->acc (under g->lock) */
static int fold_members(odpg_group_t *g)
{
	if (g->acc.size() != ODPG_COUNTER_WORDS(g->num_cos))
		g->acc.assign(ODPG_COUNTER_WORDS(g->num_cos), 0ull);
	for (odpg_counters_t *c : g->cnt) {
		if (!c)
			continue;
		const int rc = odpg_counters_fold(c, g->acc.data());

		if (rc)
			return rc;
	}
	return 0;
}

extern "C" int odpg_group_load(odpg_group_t *g, const odpg_rules_t *rules)
{
	if (!g || !rules)
		return -EINVAL;
	size_t size = 0;
	int rc = odpg_rules_compile(rules, nullptr, &size);

	if (rc && rc != -ENOSPC)
		return rc;
	std::vector<uint8_t> img(size);

	if ((rc = odpg_rules_compile(rules, img.data(), &size)))
		return rc;
	const uint32_t n = (uint32_t)g->ctx.size();
	std::vector<odpg_table_t *> nt(n, nullptr);
	std::vector<odpg_counters_t *> nc(n, nullptr);

	for (uint32_t i = 0; i < n && !rc; i++) {
		rc = odpg_table_import(g->ctx[i], img.data(), size, &nt[i]);
		if (!rc)
			rc = odpg_counters_create(g->ctx[i], nt[i], &nc[i]);
	}
	if (rc) {
		for (uint32_t i = 0; i < n; i++) {
			odpg_counters_destroy(nc[i]);
			odpg_table_destroy(nt[i]);
		}
		return rc;
	}
	std::lock_guard<std::mutex> lk(g->lock);
	const uint32_t ncos = odpg_table_num_cos(nt[0]);

	/* the previous generation's counts stay with the group when the
	 * counter layout is unchanged */
	if (g->tbl[0] && ncos == g->num_cos)
		fold_members(g);
	else
		g->acc.assign(ODPG_COUNTER_WORDS(ncos), 0ull);
	drop_tables(g);
	g->tbl = nt;
	g->cnt = nc;
	g->num_cos = ncos;
	return 0;
}

extern "C" void odpg_group_range(uint32_t num, uint32_t n, uint32_t i, uint32_t *lo, uint32_t *hi)
{
	uint32_t l = 0, h = 0;

	if (n && i < n) {
		const uint64_t tiles = ((uint64_t)num + 63u) / 64u;
		const uint64_t per = (tiles + n - 1u) / n * 64u;   /* packets per member */
		const uint64_t a = per * i, b = a + per;

		l = (uint32_t)(a < num ? a : num);
		h = (uint32_t)(i + 1u == n ? num : b < num ? b : num);
		if (h < l)
			h = l;
	}
	if (lo)
		*lo = l;
	if (hi)
		*hi = h;
}

/* member i's part of a batch / result: the range [lo, hi) */
static void sub_range(const odpg_batch_t *b, const odpg_result_t *r, uint32_t lo, uint32_t hi,
		      odpg_batch_t *sb, odpg_result_t *sr)
{
	*sb = *b;
	*sr = *r;
	sb->num = hi - lo;
	if (b->desc)
		sb->desc = b->desc + lo;             /* offsets stay relative to frames */
	else
		sb->frames = b->frames + (size_t)lo * b->stride;
	sr->out = r->out + lo;
	if (r->mark)
		sr->mark = r->mark + lo;
	if (r->meta)
		sr->meta = r->meta + lo;
}

extern "C" int odpg_group_classify_host(odpg_group_t *g, const odpg_batch_t *b,
					const odpg_result_t *r, int counted, uint32_t chunk)
{
	if (!g || !b || !r || r->stats || r->counters || (b->num && !r->out))
		return -EINVAL;
	const uint32_t n = (uint32_t)g->ctx.size();

	if (!g->tbl[0])
		return -ENOENT;
	std::vector<int> rc(n, 0);
	std::vector<std::thread> th;
	auto run = [&](uint32_t i) {
		uint32_t lo, hi;

		odpg_group_range(b->num, n, i, &lo, &hi);
		if (lo == hi)
			return;
		odpg_batch_t sb;
		odpg_result_t sr;

		sub_range(b, r, lo, hi, &sb, &sr);
		if (counted)
			sr.counters = g->cnt[i];
		rc[i] = odpg_classify_host(g->ctx[i], g->tbl[i], &sb, &sr, chunk);
	};
	try {
		for (uint32_t i = 1; i < n; i++)
			th.emplace_back(run, i);
	} catch (...) {
		for (std::thread &t : th)
			t.join();
		return -EAGAIN;
	}
	run(0);
	for (std::thread &t : th)
		t.join();
	for (uint32_t i = 0; i < n; i++)
		if (rc[i])
			return rc[i];
	return 0;
}

extern "C" int odpg_group_classify(odpg_group_t *g, const odpg_batch_t *batches,
				   const odpg_result_t *results, int counted)
{
	if (!g || !batches || !results)
		return -EINVAL;
	if (!g->tbl[0])
		return -ENOENT;
	for (uint32_t i = 0; i < g->ctx.size(); i++) {
		if (!batches[i].num)
			continue;
		if (results[i].stats || results[i].counters)
			return -EINVAL;
		odpg_result_t sr = results[i];

		if (counted)
			sr.counters = g->cnt[i];
		const int rc = odpg_classify(g->ctx[i], g->tbl[i], &batches[i], &sr);

		if (rc)
			return rc;
	}
	return 0;
}

extern "C" int odpg_group_sync(odpg_group_t *g)
{
	if (!g)
		return -EINVAL;
	int rc = 0;

	for (odpg_ctx_t *c : g->ctx) {
		const int e = odpg_ctx_sync(c);

		rc = rc ? rc : e;
	}
	return rc;
}

extern "C" int odpg_group_counters_fold(odpg_group_t *g, uint64_t *words)
{
	if (!g || !words)
		return -EINVAL;
	std::lock_guard<std::mutex> lk(g->lock);

	if (!g->tbl[0])
		return -ENOENT;
	const int rc = fold_members(g);

	if (rc)
		return rc;
	for (size_t k = 0; k < g->acc.size(); k++) {
		words[k] += g->acc[k];
		g->acc[k] = 0;
	}
	return 0;
}
