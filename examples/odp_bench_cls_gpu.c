/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp_bench_cls_gpu — the classifier cases of test/performance on the
 * MI355X library.
 *
 * 1. cls_pmr_create: test/performance/odp_bench_pktio_sp.c's case of that
 *    name (cls_pmr_create :681-789, check_cls_capa :633-672,
 *    find_first_supported_l3_pmr :615-631): num_pmr + 1 CoS, the first one
 *    the pktio's default CoS; per round, num_pmr single-term PMRs
 *    (value 1024, 1025, ..., mask 0xffff) from the default CoS to the others
 *    are created and then destroyed, each call timed. Output: per function
 *    the number of calls and the average / min / max ns, as bench_tm prints.
 * 2. rule-table rebuild: the device path keeps one compiled table per rule
 *    generation, so the first odpg_pktio_recv_batch after a PMR change pays
 *    the compile + upload. Timed on a one-packet batch, against the same
 *    call with an unchanged generation.
 * 3. recv_batch: device-resident batches of 64-byte Eth/IPv4/UDP frames whose
 *    source ports hit the PMRs round-robin, through odpg_pktio_recv_batch
 *    (classify + pktio / CoS counter updates), in Mpps. The batches rotate
 *    over copies in HBM that together exceed the 256 MiB Infinity Cache (at
 *    least five), so every launch streams its frames from HBM.
 *
 * Usage: odp_bench_cls_gpu [-n num_pmr] [-r rounds] [-b batch] [-s steps]
 * -n is the reference's PMR count option (default 64 here, the headline rule
 * count; above 8 the per-CoS limit is raised with odpg_cls_set_limits).
 */
#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <odp_cls.h>
#include <odpg.h>

#define NBUF_MAX 64

typedef struct {
	const char *name;
	uint64_t num, sum, min, max;
} tm_rec_t;

static uint64_t now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static void tm_record(tm_rec_t *r, uint64_t t1, uint64_t t2)
{
	uint64_t d = t2 - t1;

	if (r->num == 0 || d < r->min)
		r->min = d;
	if (d > r->max)
		r->max = d;
	r->sum += d;
	r->num++;
}

static void tm_print(const tm_rec_t *r)
{
	printf("  %-26s %10" PRIu64 " calls  avg %10.1f ns  min %8" PRIu64 " ns  max %10" PRIu64
	       " ns\n", r->name, r->num, r->num ? (double)r->sum / (double)r->num : 0.0, r->min,
	       r->max);
}

/* find_first_supported_l3_pmr (odp_bench_pktio_sp.c:615-631) */
static int first_supported_l4_pmr(const odp_cls_capability_t *capa, odp_cls_pmr_term_t *term)
{
	if (capa->supported_terms.bit.udp_sport)
		*term = ODP_PMR_UDP_SPORT;
	else if (capa->supported_terms.bit.udp_dport)
		*term = ODP_PMR_UDP_DPORT;
	else if (capa->supported_terms.bit.tcp_sport)
		*term = ODP_PMR_TCP_SPORT;
	else if (capa->supported_terms.bit.tcp_dport)
		*term = ODP_PMR_TCP_DPORT;
	else
		return 0;
	return 1;
}

/* 64-byte Eth/IPv4 (IHL 5, valid header checksum)/UDP frames, source port
 * 1024 + i % nport (network order), destination port 9 */
static void make_frames(uint8_t *buf, uint32_t n, uint32_t nport)
{
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *f = buf + (size_t)i * 64u;
		uint32_t s = 0;
		uint16_t sp = (uint16_t)(1024u + i % nport);

		memset(f, 0, 64);
		memcpy(f, "\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02", 12);
		f[12] = 0x08;
		f[13] = 0x00;
		f[14] = 0x45;
		f[16] = 0;
		f[17] = 50;                      /* tot_len */
		f[22] = 64;                      /* ttl */
		f[23] = 17;                      /* udp */
		f[26] = 10; f[27] = 0; f[28] = (uint8_t)(i >> 8); f[29] = (uint8_t)i;
		f[30] = 10; f[31] = 1; f[32] = 0; f[33] = 1;
		for (int k = 14; k < 34; k += 2)
			s += (uint32_t)(f[k] << 8 | f[k + 1]);
		while (s >> 16)
			s = (s & 0xffffu) + (s >> 16);
		f[24] = (uint8_t)(~s >> 8);
		f[25] = (uint8_t)~s;
		f[34] = (uint8_t)(sp >> 8);
		f[35] = (uint8_t)sp;
		f[37] = 9;
		f[39] = 30;                      /* udp length; checksum 0 */
	}
}

int main(int argc, char *argv[])
{
	uint32_t num_pmr = 64, rounds = 1000, batch = 1u << 20, steps = 100;
	int opt;

	while ((opt = getopt(argc, argv, "n:r:b:s:h")) != -1) {
		switch (opt) {
		case 'n': num_pmr = (uint32_t)strtoul(optarg, NULL, 0); break;
		case 'r': rounds = (uint32_t)strtoul(optarg, NULL, 0); break;
		case 'b': batch = (uint32_t)strtoul(optarg, NULL, 0); break;
		case 's': steps = (uint32_t)strtoul(optarg, NULL, 0); break;
		default:
			fprintf(stderr, "usage: %s [-n num_pmr] [-r rounds] [-b batch] [-s steps]\n",
				argv[0]);
			return opt == 'h' ? EXIT_SUCCESS : EXIT_FAILURE;
		}
	}
	if (num_pmr == 0 || batch == 0 || rounds == 0 || steps == 0) {
		fprintf(stderr, "Error: sizes must be > 0\n");
		return EXIT_FAILURE;
	}

	/* check_cls_capa (odp_bench_pktio_sp.c:633-672) */
	odp_cls_capability_t capa;
	odp_cls_pmr_term_t term;

	if (odp_cls_capability(&capa)) {
		fprintf(stderr, "Error: reading classifier capa failed\n");
		return EXIT_FAILURE;
	}
	if (!first_supported_l4_pmr(&capa, &term)) {
		fprintf(stderr, "Error: no TCP/UDP PMR supported\n");
		return EXIT_FAILURE;
	}
	if (num_pmr > capa.max_pmr_per_cos) {
		/* every PMR leaves the default CoS: raise the reference's 8 per CoS
		 * (odp_classification_datamodel.h:31-46), MI355X extension */
		if (odpg_cls_set_limits(num_pmr + 1 > capa.max_cos ? num_pmr + 1 : capa.max_cos,
					num_pmr > capa.max_pmr ? num_pmr : capa.max_pmr, num_pmr) ||
		    odp_cls_capability(&capa)) {
			fprintf(stderr, "Error: raising classifier limits failed\n");
			return EXIT_FAILURE;
		}
	}
	if (num_pmr + 1 > capa.max_cos || num_pmr > capa.max_pmr) {
		fprintf(stderr, "Error: not enough CoS / PMRs supported: %u/%u\n", num_pmr + 1,
			capa.max_cos);
		return EXIT_FAILURE;
	}

	odp_pktio_t pktio = odp_pktio_open("loop", ODP_POOL_INVALID, NULL);
	odp_pktio_config_t cfg;
	odp_pktin_queue_param_t qp;

	if (pktio == ODP_PKTIO_INVALID) {
		fprintf(stderr, "Error: pktio open failed\n");
		return EXIT_FAILURE;
	}
	odp_pktio_config_init(&cfg);
	cfg.parser.layer = ODP_PROTO_LAYER_ALL;
	odp_pktin_queue_param_init(&qp);
	qp.classifier_enable = 1;
	if (odp_pktio_config(pktio, &cfg) || odp_pktin_queue_config(pktio, &qp) ||
	    odp_pktio_start(pktio)) {
		fprintf(stderr, "Error: pktio config / start failed\n");
		return EXIT_FAILURE;
	}

	const uint32_t num_cos = num_pmr + 1;
	odp_cos_t *cos = calloc(num_cos, sizeof(*cos));
	odp_pmr_t *pmr = calloc(num_pmr, sizeof(*pmr));
	odp_cls_cos_param_t cp;
	int ret = EXIT_FAILURE;

	if (!cos || !pmr)
		return EXIT_FAILURE;
	odp_cls_cos_param_init(&cp);
	for (uint32_t i = 0; i < num_cos; i++) {
		cp.queue = (odp_queue_t)(uintptr_t)(0x1000u + i);
		cos[i] = odp_cls_cos_create(NULL, &cp);
		if (cos[i] == ODP_COS_INVALID) {
			fprintf(stderr, "Error: odp_cls_cos_create() failed %u / %u\n", i + 1, num_cos);
			return EXIT_FAILURE;
		}
	}
	if (odp_pktio_default_cos_set(pktio, cos[0])) {
		fprintf(stderr, "Error: setting default CoS failed\n");
		return EXIT_FAILURE;
	}

	/* 1. cls_pmr_create (odp_bench_pktio_sp.c:681-789) */
	odp_pmr_param_t pp;
	uint16_t val = 1024, mask = 0xffff;
	tm_rec_t rc_create = { "odp_cls_pmr_create()", 0, 0, 0, 0 };
	tm_rec_t rc_destroy = { "odp_cls_pmr_destroy()", 0, 0, 0, 0 };

	odp_cls_pmr_param_init(&pp);
	pp.term = term;
	pp.match.value = &val;
	pp.match.mask = &mask;
	pp.val_sz = sizeof(val);
	for (uint32_t r = 0; r < rounds; r++) {
		uint32_t created = 0;

		for (uint32_t j = 0; j < num_pmr; j++) {
			uint64_t t1 = now_ns();

			pmr[j] = odp_cls_pmr_create(&pp, 1, cos[0], cos[j + 1]);
			uint64_t t2 = now_ns();

			val++;
			if (pmr[j] == ODP_PMR_INVALID)
				break;
			tm_record(&rc_create, t1, t2);
			created++;
		}
		for (uint32_t j = 0; j < created; j++) {
			uint64_t t1 = now_ns();
			int rc = odp_cls_pmr_destroy(pmr[j]);
			uint64_t t2 = now_ns();

			if (rc) {
				fprintf(stderr, "Error: destroying PMR failed: %d\n", rc);
				return EXIT_FAILURE;
			}
			tm_record(&rc_destroy, t1, t2);
		}
	}
	printf("cls_pmr_create (%u PMRs x %u rounds, term %d)\n", num_pmr, rounds, (int)term);
	tm_print(&rc_create);
	tm_print(&rc_destroy);

	/* the rule set the device runs: source port 1024 + j (network order)
	 * to CoS j + 1, left in place */
	for (uint32_t j = 0; j < num_pmr; j++) {
		uint16_t be = (uint16_t)((uint16_t)(1024u + j) >> 8 | (uint16_t)(1024u + j) << 8);

		pp.match.value = &be;
		pmr[j] = odp_cls_pmr_create(&pp, 1, cos[0], cos[j + 1]);
		if (pmr[j] == ODP_PMR_INVALID) {
			fprintf(stderr, "Error: odp_cls_pmr_create() failed %u\n", j);
			return EXIT_FAILURE;
		}
	}

	/* 2 + 3: device side */
	odpg_ctx_t *ctx = NULL;
	uint8_t *hframes = NULL, *dframes = NULL;
	uint8_t *dbuf[NBUF_MAX] = { NULL };
	uint32_t nbuf = 0;
	odpg_out_t *dout = NULL;
	odpg_out_t *hout = NULL;
	int rc;

	if ((rc = odpg_ctx_create(0, NULL, &ctx))) {
		fprintf(stderr, "Error: odpg_ctx_create: %d\n", rc);
		goto out;
	}
	hframes = malloc((size_t)batch * 64u);
	hout = malloc((size_t)batch * sizeof(*hout));
	if (!hframes || !hout || odpg_dev_alloc(ctx, (size_t)batch * 64u, (void **)&dframes) ||
	    odpg_dev_alloc(ctx, (size_t)batch * sizeof(*dout), (void **)&dout)) {
		fprintf(stderr, "Error: allocation failed\n");
		goto out;
	}
	make_frames(hframes, batch, num_pmr);
	if (odpg_memcpy_h2d(ctx, dframes, hframes, (size_t)batch * 64u))
		goto out;
	/* rotating HBM copies: >= 5 and > 320 MiB in all */
	nbuf = (uint32_t)((320ull << 20) / ((uint64_t)batch * 64u) + 1u);
	nbuf = nbuf < 5u ? 5u : nbuf > NBUF_MAX ? NBUF_MAX : nbuf;
	dbuf[0] = dframes;
	for (uint32_t k = 1; k < nbuf; k++)
		if (odpg_dev_alloc(ctx, (size_t)batch * 64u, (void **)&dbuf[k]) ||
		    odpg_memcpy_h2d(ctx, dbuf[k], hframes, (size_t)batch * 64u)) {
			fprintf(stderr, "Error: allocation failed\n");
			goto out;
		}

	tm_rec_t rc_rebuild = { "recv_batch, new rules", 0, 0, 0, 0 };
	tm_rec_t rc_same = { "recv_batch, same rules", 0, 0, 0, 0 };
	uint16_t spare = 0x60ea;                  /* port 60000, network order */

	pp.match.value = &spare;
	for (uint32_t r = 0; r < 20; r++) {
		/* a PMR change bumps the generation: the next batch recompiles */
		odp_pmr_t x = odp_cls_pmr_create(&pp, 1, cos[1], cos[2]);
		uint64_t t1, t2;

		if (x == ODP_PMR_INVALID || odp_cls_pmr_destroy(x))
			goto out;
		t1 = now_ns();
		rc = odpg_pktio_recv_batch(pktio, ctx, dframes, NULL, 64, 1, 1, dout, NULL);
		odpg_ctx_sync(ctx);
		t2 = now_ns();
		if (rc < 0)
			goto out;
		tm_record(&rc_rebuild, t1, t2);
		t1 = now_ns();
		rc = odpg_pktio_recv_batch(pktio, ctx, dframes, NULL, 64, 1, 1, dout, NULL);
		odpg_ctx_sync(ctx);
		t2 = now_ns();
		if (rc < 0)
			goto out;
		tm_record(&rc_same, t1, t2);
	}
	printf("rule-table rebuild (one-packet batch, %u PMRs)\n", num_pmr);
	tm_print(&rc_rebuild);
	tm_print(&rc_same);

	for (uint32_t w = 0; w < 5; w++)
		if (odpg_pktio_recv_batch(pktio, ctx, dframes, NULL, 64, batch, 1, dout, NULL) < 0)
			goto out;
	odpg_ctx_sync(ctx);
	uint64_t t1 = now_ns();

	for (uint32_t s = 0; s < steps; s++)
		if (odpg_pktio_recv_batch(pktio, ctx, dbuf[s % nbuf], NULL, 64, batch, 1, dout,
					  NULL) < 0)
			goto out;
	odpg_ctx_sync(ctx);
	uint64_t t2 = now_ns();
	double sec = (double)(t2 - t1) * 1e-9;

	if (odpg_memcpy_d2h(ctx, hout, dout, (size_t)batch * sizeof(*hout)))
		goto out;
	/* every packet's verdict: the CoS of the PMR its source port hits */
	uint32_t bad = 0;
	uint32_t cos_of_port1 = hout[0] & 0xffffu;

	for (uint32_t i = 0; i < batch; i++)
		if ((hout[i] & 0xffffu) != cos_of_port1 + i % num_pmr)
			bad++;
	printf("recv_batch: %u x %u packets (64 B, device-resident, %u rotating HBM buffers): "
	       "%.1f Mpps, %u verdicts off\n",
	       steps, batch, nbuf, (double)steps * batch / sec * 1e-6, bad);

	/* the same batches through the raw batch entry point on the same rules,
	 * verdicts only: what recv_batch's bookkeeping costs on top */
	{
		odpg_rules_t rules;
		odpg_table_t *tbl = NULL;
		odpg_batch_t bt;
		odpg_result_t res;

		if (odpg_pktio_rules(pktio, &rules) || odpg_table_create(ctx, &rules, &tbl))
			goto out;
		memset(&bt, 0, sizeof(bt));
		bt.frames = dframes;
		bt.stride = 64;
		bt.num = batch;
		bt.layer = ODP_PROTO_LAYER_ALL;
		bt.classify = 1;
		memset(&res, 0, sizeof(res));
		res.out = dout;
		for (uint32_t w = 0; w < 5; w++)
			odpg_classify(ctx, tbl, &bt, &res);
		odpg_ctx_sync(ctx);
		uint64_t r1 = now_ns();

		for (uint32_t s = 0; s < steps; s++) {
			bt.frames = dbuf[s % nbuf];
			if (odpg_classify(ctx, tbl, &bt, &res) < 0)
				break;
		}
		odpg_ctx_sync(ctx);
		uint64_t r2 = now_ns();
		double rsec = (double)(r2 - r1) * 1e-9;

		printf("odpg_classify (raw, verdicts only): %.1f Mpps; recv_batch / raw = %.3f\n",
		       (double)steps * batch / rsec * 1e-6, rsec / sec);
		odpg_table_destroy(tbl);
	}

	odp_pktio_stats_t st;

	if (odp_pktio_stats(pktio, &st) == 0)
		printf("pktio in_packets %" PRIu64 ", in_octets %" PRIu64 ", in_discards %" PRIu64
		       ", in_errors %" PRIu64 "\n", st.in_packets, st.in_octets, st.in_discards,
		       st.in_errors);
	ret = bad ? EXIT_FAILURE : EXIT_SUCCESS;
out:
	if (ret != EXIT_SUCCESS)
		fprintf(stderr, "Error: device part failed\n");
	for (uint32_t k = 0; k < NBUF_MAX; k++)
		if (dbuf[k])
			odpg_dev_free(ctx, dbuf[k]);
	if (dframes && !dbuf[0])
		odpg_dev_free(ctx, dframes);
	if (dout)
		odpg_dev_free(ctx, dout);
	if (ctx)
		odpg_ctx_destroy(ctx);
	free(hframes);
	free(hout);
	for (uint32_t j = 0; j < num_pmr; j++)
		odp_cls_pmr_destroy(pmr[j]);
	odp_pktio_default_cos_set(pktio, ODP_COS_INVALID);
	for (uint32_t i = 0; i < num_cos; i++)
		odp_cos_destroy(cos[i]);
	odp_pktio_stop(pktio);
	odp_pktio_close(pktio);
	free(cos);
	free(pmr);
	return ret;
}
