/* SPDX-License-Identifier: BSD-3-Clause
 *
 * The receive verdict on the runtime's own packets, end to end on the GPU
 * (tests/test_rt_verdict.py drives it and checks every line against the
 * oracle): frames from an input file are sent on a loop pktio whose pktin
 * configuration enables the IPv4 / UDP / TCP / SCTP checksum checks, come
 * back through the GPU classifier (pktio/loop.c: loopback_send ->
 * loopback_recv), and land on their CoS queues. Then every packet of every
 * queue is read back through the ODP accessors an application would use:
 *   odp_packet_l3_chksum_status / odp_packet_l4_chksum_status
 *     (packet_inlines.h:385-417), odp_packet_cls_mark (:617),
 *   odp_packet_parse_result -> every odp_packet_has_* flag, has_l2/l3/l4_error,
 *     the offsets and l2/l3/l4 types (odp_packet.c:2077-2118),
 *   odp_packet_cos, odp_packet_input,
 *   odp_cls_hash_result(cos, pkt) (odp_classification.c:384-414), which must
 *     name the queue the packet was found on,
 * plus the raw parse result (odpg_packet_view) for a bit-exact comparison.
 *
 * Rules (created in this order; the test builds the same set for the
 * oracle): CoS 0 "dflt" with 4 hash queues over every hash protocol
 * (default CoS); CoS 1 "err" (error CoS, plain queue); CoS 2 "udp" (plain
 * queue, PMR IPPROTO == 17 from dflt, mark 0x77); CoS 3 "tcp" with 3 hash
 * queues over TCP (PMR IPPROTO == 6 from dflt, mark 0x1234); CoS 4 "drop"
 * (ODP_COS_ACTION_DROP, PMR ETHTYPE_0 == ARP from dflt); CoS 5 "v6udp"
 * (plain, PMR UDP_DPORT == 63 from udp, mark 9).
 *
 * Usage: odp_rt_verdict <in.bin> <out.txt>
 *   in.bin: u32 magic 0x56524454, u32 n, u64 pktin option bits, then n x
 *           (u32 len, len bytes)
 * Output lines:
 *   Q <qid> <cos> <index in cos>                 every CoS queue
 *   P <frame> <qid> <l3st> <l4st> <mark> <flag.all> <l2> <l3> <l4> <l2type>
 *     <l3type> <l4type> <cos> <hashq qid> <input ok> <input_flags> <flags>
 *   S <in_packets> <in_octets> <in_errors> <in_discards>
 *   C <cos> <packets>           QS <qid> <packets> <discards>
 * Exit status 0 when the run completed (the checks are the test's).
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <odp_api.h>
#include <odp/helper/odph_api.h>

#define MAXQ 64

static uint8_t **frame;
static uint32_t *flen;
static uint8_t *taken;
static uint32_t nframe;

static odp_cos_t coses[6];
static odp_queue_t qs[MAXQ];
static int q_cos[MAXQ], q_idx[MAXQ], nq;

static int qid_of(odp_queue_t q)
{
	for (int i = 0; i < nq; i++)
		if (qs[i] == q)
			return i;
	return -1;
}

static int cos_index(odp_cos_t c)
{
	for (int i = 0; i < 6; i++)
		if (coses[i] == c)
			return i;
	return -1;
}

/* the first not yet matched sent frame with these bytes */
static int which_frame(odp_packet_t pkt)
{
	const uint32_t len = odp_packet_len(pkt);
	const uint8_t *d = odp_packet_data(pkt);

	for (uint32_t k = 0; k < nframe; k++)
		if (!taken[k] && flen[k] == len && !memcmp(frame[k], d, len)) {
			taken[k] = 1;
			return (int)k;
		}
	return -1;
}

static int read_input(const char *path, uint64_t *opt)
{
	FILE *f = fopen(path, "rb");
	uint32_t hdr[2];

	if (!f || fread(hdr, 4, 2, f) != 2 || hdr[0] != 0x56524454u || fread(opt, 8, 1, f) != 1)
		return -1;
	nframe = hdr[1];
	frame = calloc(nframe, sizeof(*frame));
	flen = calloc(nframe, sizeof(*flen));
	taken = calloc(nframe ? nframe : 1, 1);
	for (uint32_t k = 0; k < nframe; k++) {
		if (fread(&flen[k], 4, 1, f) != 1)
			return -1;
		frame[k] = malloc(flen[k] ? flen[k] : 1);
		if (flen[k] && fread(frame[k], 1, flen[k], f) != flen[k])
			return -1;
	}
	fclose(f);
	return 0;
}

static odp_cos_t mk_cos(const char *name, odp_pool_t pool, int action, uint32_t num_queue,
			uint32_t hash_bits)
{
	odp_cls_cos_param_t cp;
	odp_queue_param_t qp;

	odp_queue_param_init(&qp);
	odp_cls_cos_param_init(&cp);
	cp.action = action;
	cp.pool = pool;
	cp.stats_enable = 1;
	cp.num_queue = num_queue;
	if (num_queue > 1) {
		cp.queue_param = qp;
		cp.hash_proto.all_bits = hash_bits;
	} else if (action != ODP_COS_ACTION_DROP) {
		cp.queue = odp_queue_create(name, &qp);
	}
	return odp_cls_cos_create(name, &cp);
}

static int mk_pmr(odp_cos_t src, odp_cos_t dst, odp_cls_pmr_term_t term, const void *val,
		  const void *mask, uint32_t sz, uint64_t mark)
{
	odp_pmr_param_t pp;
	odp_pmr_create_opt_t opt;

	odp_cls_pmr_param_init(&pp);
	pp.term = term;
	pp.match.value = val;
	pp.match.mask = mask;
	pp.val_sz = sz;
	odp_cls_pmr_create_opt_init(&opt);
	opt.terms = &pp;
	opt.num_terms = 1;
	opt.mark = mark;
	return odp_cls_pmr_create_opt(&opt, src, dst) == ODP_PMR_INVALID ? -1 : 0;
}

int main(int argc, char *argv[])
{
	odp_instance_t inst;
	odp_pool_param_t pp;
	odp_pktio_param_t pip;
	odp_pktin_queue_param_t iqp;
	odp_pktio_config_t cfg;
	odp_pktin_queue_t inq;
	odp_pktout_queue_t outq;
	odp_pool_t pool;
	odp_pktio_t pktio;
	uint64_t opt;
	FILE *out;

	if (argc != 3 || read_input(argv[1], &opt)) {
		fprintf(stderr, "usage: odp_rt_verdict <in.bin> <out.txt>\n");
		return 2;
	}
	out = fopen(argv[2], "w");
	if (!out || odp_init_global(&inst, NULL, NULL) || odp_init_local(inst, ODP_THREAD_CONTROL))
		return 2;
	odp_pool_param_init(&pp);
	pp.type = ODP_POOL_PACKET;
	pp.pkt.num = nframe + 16;
	pp.pkt.len = 2048;
	pool = odp_pool_create("verdict", &pp);
	odp_pktio_param_init(&pip);
	pip.in_mode = ODP_PKTIN_MODE_DIRECT;
	pip.out_mode = ODP_PKTOUT_MODE_DIRECT;
	pktio = odp_pktio_open("loop", pool, &pip);
	if (pool == ODP_POOL_INVALID || pktio == ODP_PKTIO_INVALID)
		return 2;
	odp_pktio_config_init(&cfg);
	cfg.pktin.all_bits = opt;
	odp_pktin_queue_param_init(&iqp);
	iqp.classifier_enable = 1;
	if (odp_pktio_config(pktio, &cfg) || odp_pktin_queue_config(pktio, &iqp) ||
	    odp_pktout_queue_config(pktio, NULL))
		return 2;

	/* hash protocol bits (odp_pktin_hash_proto_t): ipv4_udp 1, ipv4_tcp 2,
	 * ipv4 4, ipv6_udp 8, ipv6_tcp 16, ipv6 32 */
	coses[0] = mk_cos("dflt", ODP_POOL_INVALID, ODP_COS_ACTION_ENQUEUE, 4, 0x3f);
	coses[1] = mk_cos("err", ODP_POOL_INVALID, ODP_COS_ACTION_ENQUEUE, 1, 0);
	coses[2] = mk_cos("udp", ODP_POOL_INVALID, ODP_COS_ACTION_ENQUEUE, 1, 0);
	coses[3] = mk_cos("tcp", ODP_POOL_INVALID, ODP_COS_ACTION_ENQUEUE, 3, 2 | 16);
	coses[4] = mk_cos("drop", ODP_POOL_INVALID, ODP_COS_ACTION_DROP, 1, 0);
	coses[5] = mk_cos("v6udp", ODP_POOL_INVALID, ODP_COS_ACTION_ENQUEUE, 1, 0);
	for (int c = 0; c < 6; c++)
		if (coses[c] == ODP_COS_INVALID)
			return 2;
	{
		const uint8_t udp = 17, tcp = 6, ff = 0xff;
		const uint16_t arp = odp_cpu_to_be_16(0x0806), port = odp_cpu_to_be_16(63);
		const uint16_t m16 = 0xffff;

		if (mk_pmr(coses[0], coses[2], ODP_PMR_IPPROTO, &udp, &ff, 1, 0x77) ||
		    mk_pmr(coses[0], coses[3], ODP_PMR_IPPROTO, &tcp, &ff, 1, 0x1234) ||
		    mk_pmr(coses[0], coses[4], ODP_PMR_ETHTYPE_0, &arp, &m16, 2, 0) ||
		    mk_pmr(coses[2], coses[5], ODP_PMR_UDP_DPORT, &port, &m16, 2, 9))
			return 2;
	}
	if (odp_pktio_default_cos_set(pktio, coses[0]) || odp_pktio_error_cos_set(pktio, coses[1]))
		return 2;
	for (int c = 0; c < 6; c++) {
		odp_queue_t cq[32];
		const uint32_t n = odp_cls_cos_queues(coses[c], cq, 32);

		for (uint32_t i = 0; i < n && c != 4; i++) {
			qs[nq] = cq[i];
			q_cos[nq] = c;
			q_idx[nq] = (int)i;
			fprintf(out, "Q %d %d %u\n", nq, c, i);
			nq++;
		}
	}
	if (odp_pktio_start(pktio) || odp_pktin_queue(pktio, &inq, 1) != 1 ||
	    odp_pktout_queue(pktio, &outq, 1) != 1)
		return 2;

	/* send everything, then receive the loop ring in bursts */
	for (uint32_t k = 0; k < nframe; k++) {
		odp_packet_t pkt = odp_packet_alloc(pool, flen[k]);

		if (pkt == ODP_PACKET_INVALID)
			return 2;
		memcpy(odp_packet_data(pkt), frame[k], flen[k]);
		if (odp_pktout_send(outq, &pkt, 1) != 1)
			return 2;
	}
	for (uint32_t r = 0; r < nframe / 64 + 4; r++) {
		odp_packet_t got[1024];

		if (odp_pktin_recv(inq, got, 1024) != 0)   /* all go to CoS queues */
			return 3;
	}

	/* read every queue back through the accessors */
	uint32_t received = 0;

	for (int q = 0; q < nq; q++) {
		odp_event_t ev;

		while ((ev = odp_queue_deq(qs[q])) != ODP_EVENT_INVALID) {
			odp_packet_t pkt = odp_packet_from_event(ev);
			odp_packet_parse_result_t pr;
			odpg_packet_t view;
			const odp_cos_t cos = odp_packet_cos(pkt);

			odp_packet_parse_result(pkt, &pr);
			if (odpg_packet_view(pkt, &view))
				return 4;
			fprintf(out, "P %d %d %d %d %" PRIu64 " %" PRIu64 " %u %u %u %u %u %u %d %d %d "
				"%" PRIu64 " %u\n",
				which_frame(pkt), q, (int)odp_packet_l3_chksum_status(pkt),
				(int)odp_packet_l4_chksum_status(pkt), odp_packet_cls_mark(pkt),
				pr.flag.all, pr.l2_offset, pr.l3_offset, pr.l4_offset, pr.l2_type,
				pr.l3_type, pr.l4_type, cos_index(cos),
				qid_of(odp_cls_hash_result(cos, pkt)), odp_packet_input(pkt) == pktio,
				view.meta.input_flags, view.meta.flags);
			odp_packet_free(pkt);
			received++;
		}
	}

	odp_pktio_stats_t st;

	if (odp_pktio_stats(pktio, &st))
		return 5;
	fprintf(out, "S %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 "\n", st.in_packets,
		st.in_octets, st.in_errors, st.in_discards);
	for (int c = 0; c < 6; c++) {
		odp_cls_cos_stats_t cs;

		if (odp_cls_cos_stats(coses[c], &cs))
			return 5;
		fprintf(out, "C %d %" PRIu64 "\n", c, cs.packets);
	}
	for (int q = 0; q < nq; q++) {
		odp_cls_queue_stats_t s;

		if (odp_cls_queue_stats(coses[q_cos[q]], qs[q], &s))
			return 5;
		fprintf(out, "QS %d %" PRIu64 " %" PRIu64 "\n", q, s.packets, s.discards);
	}
	fclose(out);
	if (odp_pktio_stop(pktio) || odp_pktio_close(pktio))
		return 6;
	printf("received %u of %u frames\n", received, nframe);
	odp_term_local();
	odp_term_global(inst);
	return 0;
}
