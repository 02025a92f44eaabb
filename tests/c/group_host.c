/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Device groups (include/odpg_group.h, odp_amd/csrc/group.cpp) under
 * ThreadSanitizer and AddressSanitizer + UBSan, built only with the
 * test-only device stub (tests/c/gpu_stub.c, tests/c/Makefile "san"): the
 * members' host threads, the per-member counters and their fold. A loop
 * pktio with a default CoS and one SIP_ADDR rule (the ODP API, as
 * odp_rt_loop.c case B) gives the rule snapshot; a batch of 64-byte
 * IPv4/UDP frames, half of them from 10.10.10.0/24, is classified by one
 * context and by groups of 1, 3 and 5 members, as a host batch and as
 * per-member shards: the verdicts and the folded counters must be equal.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <odp_api.h>
#include <odp_cls.h>
#include <odpg.h>
#include <odpg_group.h>

static int fails;

#define CHECK(c, ...)                                                      \
	do {                                                               \
		if (!(c)) {                                                \
			fails++;                                           \
			printf("FAIL %s:%d: ", __FILE__, __LINE__);       \
			printf(__VA_ARGS__);                               \
			printf("\n");                                      \
		}                                                          \
	} while (0)

#define NUM 5003u

/* frame i: Ethernet / IPv4 (IHL 5) / UDP, source 10.10.10.i or 10.20.0.i */
static void make_frames(uint8_t *f)
{
	memset(f, 0, (size_t)NUM * 64u);
	for (uint32_t i = 0; i < NUM; i++) {
		uint8_t *p = f + (size_t)i * 64u;

		memset(p, 0x02, 12);
		p[12] = 0x08;                      /* IPv4 */
		p[14] = 0x45;
		p[16] = 0;
		p[17] = 46;                        /* total length: 64 - 14 - 4 */
		p[22] = 64;                        /* TTL */
		p[23] = 17;                        /* UDP */
		p[26] = 10;
		p[27] = (i & 1u) ? 20 : 10;
		p[28] = (i & 1u) ? 0 : 10;
		p[29] = (uint8_t)i;
		p[30] = 10;
		p[33] = 1;
		p[34] = 0x13;                      /* source port 5000 */
		p[35] = 0x88;
		p[36] = 0x13;                      /* destination port 5001 */
		p[37] = 0x89;
		p[38] = 0;
		p[39] = 26;                        /* UDP length */
	}
}

static int same_words(const uint64_t *a, const uint64_t *b, size_t n)
{
	return !memcmp(a, b, n * sizeof(uint64_t));
}

int main(void)
{
	odp_instance_t inst;

	if (odp_init_global(&inst, NULL, NULL) || odp_init_local(inst, ODP_THREAD_CONTROL)) {
		printf("FAIL: init\n");
		return 1;
	}
	odp_pool_param_t pl;

	odp_pool_param_init(&pl);
	pl.type = ODP_POOL_PACKET;
	pl.pkt.num = 256;
	pl.pkt.len = 128;
	pl.pkt.seg_len = 128;
	odp_pool_t pool = odp_pool_create("grp", &pl);
	odp_pktio_param_t pp;
	odp_pktin_queue_param_t ip;
	odp_pktout_queue_param_t op;

	odp_pktio_param_init(&pp);
	pp.in_mode = ODP_PKTIN_MODE_SCHED;
	odp_pktio_t pktio = odp_pktio_open("loop", pool, &pp);

	CHECK(pool != ODP_POOL_INVALID && pktio != ODP_PKTIO_INVALID, "pool / pktio");
	odp_pktin_queue_param_init(&ip);
	ip.classifier_enable = 1;
	odp_pktout_queue_param_init(&op);
	CHECK(!odp_pktin_queue_config(pktio, &ip) && !odp_pktout_queue_config(pktio, &op),
	      "queue config");
	odp_queue_param_t qp;
	odp_cls_cos_param_t cp;
	odp_pmr_param_t pmr;
	uint32_t val = odp_cpu_to_be_32(0x0a0a0a00), mask = odp_cpu_to_be_32(0xffffff00);

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	odp_cls_cos_param_init(&cp);
	cp.queue = odp_queue_create("dflt", &qp);
	cp.pool = pool;
	odp_cos_t cd = odp_cls_cos_create("dflt", &cp);

	cp.queue = odp_queue_create("net10", &qp);
	odp_cos_t cn = odp_cls_cos_create("net10", &cp);

	CHECK(cd != ODP_COS_INVALID && cn != ODP_COS_INVALID, "cos create");
	CHECK(odp_pktio_default_cos_set(pktio, cd) == 0, "default cos");
	odp_cls_pmr_param_init(&pmr);
	pmr.term = ODP_PMR_SIP_ADDR;
	pmr.match.value = &val;
	pmr.match.mask = &mask;
	pmr.val_sz = 4;
	CHECK(odp_cls_pmr_create(&pmr, 1, cd, cn) != ODP_PMR_INVALID, "pmr create");
	CHECK(odp_pktio_start(pktio) == 0, "start");
	odpg_rules_t rules;

	CHECK(odpg_pktio_rules(pktio, &rules) == 0 && rules.num_cos >= 2, "rule snapshot");

	uint8_t *frames = malloc((size_t)NUM * 64u);
	odpg_out_t *one = calloc(NUM, sizeof(odpg_out_t)), *out = calloc(NUM, sizeof(odpg_out_t));
	const size_t nw = ODPG_COUNTER_WORDS(rules.num_cos);
	uint64_t *w1 = calloc(nw, sizeof(uint64_t)), *wg = calloc(nw, sizeof(uint64_t));

	make_frames(frames);
	odpg_batch_t b = { frames, NULL, 64u, NUM, 0u, 4u, 1u };

	/* one context, counted */
	odpg_ctx_t *ctx = NULL;
	odpg_table_t *tbl = NULL;
	odpg_counters_t *cnt = NULL;

	CHECK(odpg_ctx_create(0, NULL, &ctx) == 0 && odpg_table_create(ctx, &rules, &tbl) == 0 &&
	      odpg_counters_create(ctx, tbl, &cnt) == 0, "single context");
	odpg_result_t r1 = { one, NULL, NULL, NULL, cnt };

	CHECK(odpg_classify_host(ctx, tbl, &b, &r1, 512) == 0, "single classify");
	CHECK(odpg_counters_fold(cnt, w1) == 0, "single fold");
	uint32_t net = 0;

	for (uint32_t i = 0; i < NUM; i++)
		net += (one[i] & 0xffffu) != (one[0] & 0xffffu);
	CHECK(net == NUM / 2u, "%u of %u packets to the other CoS", net, NUM);

	const int devs[5] = { 0, 0, 0, 0, 0 };

	for (uint32_t n = 1; n <= 5; n += 2) {
		odpg_group_t *g = NULL;

		CHECK(odpg_group_create(devs, n, &g) == 0 && odpg_group_size(g) == n, "group of %u", n);
		CHECK(odpg_group_load(g, &rules) == 0, "load");
		/* a host batch, twice (the members' threads run concurrently) */
		for (int pass = 0; pass < 2; pass++) {
			odpg_result_t rg = { out, NULL, NULL, NULL, NULL };

			memset(out, 0xff, (size_t)NUM * sizeof(odpg_out_t));
			CHECK(odpg_group_classify_host(g, &b, &rg, 1, 256) == 0, "classify_host");
			CHECK(!memcmp(out, one, (size_t)NUM * sizeof(odpg_out_t)),
			      "group of %u: verdicts", n);
		}
		memset(wg, 0, nw * sizeof(uint64_t));
		CHECK(odpg_group_counters_fold(g, wg) == 0, "group fold");
		for (size_t k = 0; k < nw; k++)
			w1[k] *= 2u;
		CHECK(same_words(w1, wg, nw), "group of %u: counters of two passes", n);
		for (size_t k = 0; k < nw; k++)
			w1[k] /= 2u;
		/* per-member shards (stub: host memory is device memory) */
		odpg_batch_t bs[5];
		odpg_result_t rs[5];

		memset(out, 0xff, (size_t)NUM * sizeof(odpg_out_t));
		for (uint32_t i = 0; i < n; i++) {
			uint32_t lo, hi;

			odpg_group_range(NUM, n, i, &lo, &hi);
			bs[i] = b;
			bs[i].frames = frames + (size_t)lo * 64u;
			bs[i].num = hi - lo;
			memset(&rs[i], 0, sizeof(rs[i]));
			rs[i].out = out + lo;
		}
		CHECK(odpg_group_classify(g, bs, rs, 1) == 0 && odpg_group_sync(g) == 0, "shards");
		CHECK(!memcmp(out, one, (size_t)NUM * sizeof(odpg_out_t)), "group of %u: shards", n);
		memset(wg, 0, nw * sizeof(uint64_t));
		CHECK(odpg_group_counters_fold(g, wg) == 0 && same_words(w1, wg, nw),
		      "group of %u: shard counters", n);
		/* a reload of the same layout keeps nothing pending: the next fold is zero */
		CHECK(odpg_group_load(g, &rules) == 0, "reload");
		memset(wg, 0, nw * sizeof(uint64_t));
		CHECK(odpg_group_counters_fold(g, wg) == 0 && wg[0] == 0, "fold after reload");
		odpg_group_destroy(g);
	}
	printf("groups of 1, 3, 5 contexts: %u packets, verdicts and counters equal one context's\n",
	       NUM);

	odpg_counters_destroy(cnt);
	odpg_table_destroy(tbl);
	odpg_ctx_destroy(ctx);
	free(frames);
	free(one);
	free(out);
	free(w1);
	free(wg);
	CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "close");
	odp_cos_destroy(cn);
	odp_cos_destroy(cd);
	odp_pool_destroy(pool);
	odp_term_local();
	odp_term_global(inst);
	printf(fails ? "FAILED (%d)\n" : "PASS\n", fails);
	return fails ? 1 : 0;
}
