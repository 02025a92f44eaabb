/* SPDX-License-Identifier: BSD-3-Clause
 *
 * The loop pktio of the ODP runtime subset end to end on the GPU
 * (tests/test_odp_rt.py runs it): packets sent on a loop device come back
 * through the GPU classifier (pktio/loop.c: loopback_send -> loopback_recv),
 * in the three input modes:
 *   A  DIRECT in / DIRECT out, classifier off: odp_pktin_recv() returns the
 *      frames unchanged, in order, with the kernel's parse result; interface
 *      and per-queue counters.
 *   B  SCHED in, classifier on (default CoS + an ODP_PMR_SIP_ADDR /24 rule):
 *      odp_schedule() hands every packet out from its CoS queue; CoS and
 *      queue counters.
 *   C  QUEUE in / QUEUE out, classifier off: enqueue on the pktout event
 *      queue transmits, dequeue from the pktin event queue receives.
 *   D  pcap input "pcap:in=<file>:loops=<n>": the capture is read
 *      max(1, n - 1) times for n >= 1 (pcapif_init sets loop_cnt = 1 and
 *      _pcapif_reopen stops when ++loop_cnt >= loops, pktio/pcap.c:215,266).
 *   F  SCHED in, classifier off, 4 receiving threads and a sender, the
 *      transmit packets from a pool of their own (so that delivery copies
 *      them into the pktio's pool, as loop.c does): every packet is handed
 *      out exactly once, and each thread sees one sender's packets in
 *      sending order (the receive pipeline's chunked delivery keeps queue
 *      order).
 *   G  4 input queues (DIRECT and SCHED), 2 output queues: with hashing
 *      (ipv4_udp + ipv4) every packet arrives once, on the input queue the
 *      oracle's crc32c pick names (loop.c get_dest_queue over the parse
 *      result the sender's odp_packet_parse gave it), in sending order per
 *      queue, with per-queue counters; without hashing on the input queue
 *      of its output queue index (index % queues).
 * Plus the pktio lookup / duplicate-open rule and the mode checks of the
 * queue accessors (odp_packet_io.c:406-410, 798-829, 1696-1843, 2364-2503),
 * and close refused while started (odp_packet_io.c:507-510).
 * Prints one line per check; exit status 0 when all pass.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <odp_api.h>
#include <odp/helper/odph_api.h>

#define NPKT 300

/* oracle/odp_oracle.c (test infrastructure): odp_hash_crc32c */
uint32_t oracle_crc32c(const uint8_t *p, uint32_t len, uint32_t init);

static int fails;

#define CHECK(cond, ...) do { \
	if (!(cond)) { \
		fails++; \
		printf("FAIL %s:%d: ", __FILE__, __LINE__); \
		printf(__VA_ARGS__); \
		printf("\n"); \
	} \
} while (0)

static uint8_t frame[NPKT][1600];
static uint32_t flen[NPKT];

/* frame k: IPv4/UDP from 10.10.10.k (even k) or 192.168.1.k (odd k), every
 * 10th an ARP frame; lengths 60..1499 */
static void make_frames(void)
{
	for (int k = 0; k < NPKT; k++) {
		uint8_t *f = frame[k];
		const uint32_t len = 60 + (uint32_t)(k * 37) % 1440;

		memset(f, 0, sizeof(frame[k]));
		for (uint32_t i = 0; i < len; i++)
			f[i] = (uint8_t)(k * 7 + i);
		memcpy(f, "\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02", 12);
		flen[k] = len;
		if (k % 10 == 9) {
			f[12] = 0x08;
			f[13] = 0x06;               /* ARP */
			continue;
		}
		f[12] = 0x08;
		f[13] = 0x00;
		uint8_t *ip = f + 14;

		ip[0] = 0x45;
		ip[1] = 0;
		ip[2] = (uint8_t)((len - 14) >> 8);
		ip[3] = (uint8_t)(len - 14);
		ip[6] = 0x40;                       /* DF, no fragment */
		ip[7] = 0;
		ip[8] = 64;
		ip[9] = 17;
		if (k % 2 == 0) {
			ip[12] = 10; ip[13] = 10; ip[14] = 10; ip[15] = (uint8_t)k;
		} else {
			ip[12] = 192; ip[13] = 168; ip[14] = 1; ip[15] = (uint8_t)k;
		}
		ip[16] = 10; ip[17] = 0; ip[18] = 0; ip[19] = 1;
		ip[10] = ip[11] = 0;
		uint32_t sum = 0;

		for (int i = 0; i < 20; i += 2)
			sum += (uint32_t)ip[i] << 8 | ip[i + 1];
		while (sum >> 16)
			sum = (sum & 0xffff) + (sum >> 16);
		ip[10] = (uint8_t)(~sum >> 8);
		ip[11] = (uint8_t)~sum;
		uint8_t *udp = ip + 20;

		udp[0] = 0x30; udp[1] = 0x39;
		udp[2] = 0x00; udp[3] = 0x35;
		udp[4] = (uint8_t)((len - 34) >> 8);
		udp[5] = (uint8_t)(len - 34);
		udp[6] = udp[7] = 0;                /* no UDP checksum */
	}
}

static uint64_t total_octets(void)
{
	uint64_t s = 0;

	for (int k = 0; k < NPKT; k++)
		s += flen[k];
	return s;
}

static int send_all_direct(odp_pktio_t pktio, odp_pool_t pool)
{
	odp_pktout_queue_t out;
	int sent = 0;

	if (odp_pktout_queue(pktio, &out, 1) != 1)
		return -1;
	for (int k = 0; k < NPKT; k++) {
		odp_packet_t pkt = odp_packet_alloc(pool, flen[k]);

		if (pkt == ODP_PACKET_INVALID)
			return -1;
		memcpy(odp_packet_data(pkt), frame[k], flen[k]);
		if (odp_pktout_send(out, &pkt, 1) != 1) {
			odp_packet_free(pkt);
			return -1;
		}
		sent++;
	}
	return sent;
}

/* the frame a received packet carries (by content) */
static int which_frame(odp_packet_t pkt)
{
	const uint8_t *d = odp_packet_data(pkt);

	for (int k = 0; k < NPKT; k++)
		if (odp_packet_len(pkt) == flen[k] && !memcmp(d, frame[k], flen[k]))
			return k;
	return -1;
}

static odp_pktio_t open_loop(const char *name, odp_pool_t pool, odp_pktin_mode_t in,
			     odp_pktout_mode_t out, int cls)
{
	odp_pktio_param_t pp;
	odp_pktin_queue_param_t ip;
	odp_pktout_queue_param_t op;
	odp_pktio_t pktio;

	odp_pktio_param_init(&pp);
	pp.in_mode = in;
	pp.out_mode = out;
	pktio = odp_pktio_open(name, pool, &pp);
	if (pktio == ODP_PKTIO_INVALID)
		return pktio;
	odp_pktin_queue_param_init(&ip);
	ip.classifier_enable = cls;
	odp_pktout_queue_param_init(&op);
	if (odp_pktin_queue_config(pktio, &ip) || odp_pktout_queue_config(pktio, &op)) {
		odp_pktio_close(pktio);
		return ODP_PKTIO_INVALID;
	}
	return pktio;
}

static void case_direct(odp_pool_t pool)
{
	odp_pktio_t pktio = open_loop("loop", pool, ODP_PKTIN_MODE_DIRECT,
				      ODP_PKTOUT_MODE_DIRECT, 0);
	odp_pktio_param_t pp;
	odp_pktin_queue_t inq;
	odp_queue_t evq;
	odp_packet_t pkts[64];
	odp_pktio_stats_t st;
	odp_pktin_queue_stats_t is;
	odp_pktout_queue_stats_t os;
	odp_pktout_queue_t oq;
	int got = 0, order_ok = 1, meta_ok = 1;

	CHECK(pktio != ODP_PKTIO_INVALID, "open loop");
	if (pktio == ODP_PKTIO_INVALID)
		return;
	odp_pktio_param_init(&pp);
	CHECK(odp_pktio_open("loop", pool, &pp) == ODP_PKTIO_INVALID, "second open of loop");
	CHECK(odp_pktio_lookup("loop") == pktio, "lookup");
	CHECK(odp_pktio_lookup("loop9") == ODP_PKTIO_INVALID, "lookup of a closed name");
	CHECK(odp_pktin_queue(pktio, &inq, 1) == 1, "odp_pktin_queue");
	CHECK(odp_pktin_event_queue(pktio, &evq, 1) == -1, "event queue in DIRECT mode");
	CHECK(odp_pktout_event_queue(pktio, &evq, 1) == -1, "pktout event queue in DIRECT");
	CHECK(odp_pktio_start(pktio) == 0, "start");
	CHECK(send_all_direct(pktio, pool) == NPKT, "send");
	for (int tries = 0; got < NPKT && tries < 1000; tries++) {
		const int n = odp_pktin_recv(inq, pkts, 64);

		CHECK(n >= 0, "odp_pktin_recv %d", n);
		if (n < 0)
			break;
		for (int i = 0; i < n; i++, got++) {
			const int k = got;
			const int arp = k % 10 == 9;

			if (k >= NPKT || odp_packet_len(pkts[i]) != flen[k] ||
			    memcmp(odp_packet_data(pkts[i]), frame[k], flen[k]))
				order_ok = 0;
			else if (odp_packet_has_eth(pkts[i]) != 1 ||
				 odp_packet_has_ipv4(pkts[i]) != !arp ||
				 odp_packet_has_udp(pkts[i]) != !arp ||
				 odp_packet_l2_offset(pkts[i]) != 0 ||
				 odp_packet_l3_offset(pkts[i]) != 14 ||
				 (!arp && odp_packet_l4_offset(pkts[i]) != 34) ||
				 odp_packet_has_error(pkts[i]))
				meta_ok = 0;
			odp_packet_free(pkts[i]);
		}
	}
	CHECK(got == NPKT, "received %d of %d", got, NPKT);
	CHECK(order_ok, "frames back unchanged and in order");
	CHECK(meta_ok, "parse result on the packets");
	CHECK(odp_pktin_recv(inq, pkts, 64) == 0, "nothing more");
	CHECK(odp_pktio_stats(pktio, &st) == 0, "stats");
	CHECK(st.in_packets == NPKT && st.in_octets == total_octets(),
	      "in %lu pkts %lu B", (unsigned long)st.in_packets, (unsigned long)st.in_octets);
	CHECK(st.out_packets == NPKT && st.out_octets == total_octets(),
	      "out %lu pkts %lu B", (unsigned long)st.out_packets, (unsigned long)st.out_octets);
	CHECK(odp_pktin_queue_stats(inq, &is) == 0 && is.packets == NPKT &&
	      is.octets == total_octets(), "pktin queue stats");
	CHECK(odp_pktout_queue(pktio, &oq, 1) == 1 && odp_pktout_queue_stats(oq, &os) == 0 &&
	      os.packets == NPKT, "pktout queue stats");
	CHECK(odp_pktio_stats_reset(pktio) == 0 && odp_pktin_queue_stats(inq, &is) == 0 &&
	      is.packets == 0, "stats reset");
	CHECK(odp_pktio_close(pktio) == -1, "close refused while started");
	CHECK(odp_pktio_lookup("loop") == pktio, "still open after the refused close");
	CHECK(odp_pktio_stop(pktio) == 0, "stop");
	CHECK(odp_pktio_close(pktio) == 0, "close");
	CHECK(odp_pktio_lookup("loop") == ODP_PKTIO_INVALID, "lookup after close");
	printf("A direct: received %d\n", got);
}

static void case_sched_cls(odp_pool_t pool)
{
	odp_pktio_t pktio = open_loop("loop1", pool, ODP_PKTIN_MODE_SCHED,
				      ODP_PKTOUT_MODE_DIRECT, 1);
	odp_queue_param_t qp;
	odp_cls_cos_param_t cp;
	odp_pmr_param_t pmr;
	odp_queue_t qd, qn, evq;
	odp_cos_t cd, cn;
	/* protocol field values in network byte order (classification.h:273-291) */
	uint32_t val = odp_cpu_to_be_32(0x0a0a0a00), mask = odp_cpu_to_be_32(0xffffff00);
	int got = 0, route_ok = 1;
	int n_net = 0, n_def = 0;
	odp_cls_cos_stats_t cs;
	odp_pktin_queue_stats_t is;

	CHECK(pktio != ODP_PKTIO_INVALID, "open loop1");
	if (pktio == ODP_PKTIO_INVALID)
		return;
	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	qd = odp_queue_create("dflt", &qp);
	qn = odp_queue_create("net10", &qp);
	odp_cls_cos_param_init(&cp);
	cp.queue = qd;
	cp.pool = pool;
	cp.stats_enable = 1;
	cd = odp_cls_cos_create("dflt", &cp);
	cp.queue = qn;
	cn = odp_cls_cos_create("net10", &cp);
	CHECK(cd != ODP_COS_INVALID && cn != ODP_COS_INVALID, "cos create");
	CHECK(odp_pktio_default_cos_set(pktio, cd) == 0, "default cos");
	odp_cls_pmr_param_init(&pmr);
	pmr.term = ODP_PMR_SIP_ADDR;
	pmr.match.value = &val;
	pmr.match.mask = &mask;
	pmr.val_sz = 4;
	CHECK(odp_cls_pmr_create(&pmr, 1, cd, cn) != ODP_PMR_INVALID, "pmr create");
	CHECK(odp_pktin_event_queue(pktio, &evq, 1) == 1, "pktin event queue");
	CHECK(odp_pktio_start(pktio) == 0, "start");
	CHECK(send_all_direct(pktio, pool) == NPKT, "send");
	for (;;) {
		odp_queue_t from;
		odp_event_t ev = odp_schedule(&from, odp_schedule_wait_time(200 * ODP_TIME_MSEC_IN_NS));

		if (ev == ODP_EVENT_INVALID)
			break;
		odp_packet_t pkt = odp_packet_from_event(ev);
		const int k = which_frame(pkt);
		const int net = k >= 0 && k % 10 != 9 && k % 2 == 0;

		if (k < 0 || from != (net ? qn : qd) || odp_packet_cos(pkt) != (net ? cn : cd))
			route_ok = 0;
		n_net += net;
		n_def += !net;
		got++;
		odp_event_free(ev);
	}
	CHECK(got == NPKT, "scheduled %d of %d", got, NPKT);
	CHECK(route_ok, "every packet from its CoS queue");
	CHECK(odp_cls_cos_stats(cn, &cs) == 0 && cs.packets == (uint64_t)n_net,
	      "net10 CoS packets %lu vs %d", (unsigned long)cs.packets, n_net);
	CHECK(odp_cls_cos_stats(cd, &cs) == 0 && cs.packets == (uint64_t)n_def,
	      "default CoS packets %lu vs %d", (unsigned long)cs.packets, n_def);
	CHECK(odp_pktin_event_queue_stats(pktio, evq, &is) == 0 && is.packets == NPKT,
	      "pktin event queue stats %lu", (unsigned long)is.packets);
	CHECK(odp_pktio_stop(pktio) == 0, "stop");
	CHECK(odp_pktio_default_cos_set(pktio, ODP_COS_INVALID) == 0, "clear default cos");
	CHECK(odp_pktio_close(pktio) == 0, "close");
	odp_cos_destroy(cn);
	odp_cos_destroy(cd);
	CHECK(odp_queue_destroy(qn) == 0 && odp_queue_destroy(qd) == 0, "queue destroy");
	printf("B sched+cls: %d packets, %d to net10, %d to default\n", got, n_net, n_def);
}

/* G: the input queue loop.c's get_dest_queue picks for frame k with
 * ipv4_udp + ipv4 hashing over nq queues: crc32c of the UDP ports and the
 * IPv4 addresses (none for the ARP frames: queue 0) */
static int expected_queue(int k, int nq)
{
	uint8_t d[12] = {0};

	if (k % 10 == 9)
		return (int)(oracle_crc32c(d, 0, 0) % (uint32_t)nq);
	memcpy(d, frame[k] + 34, 4);
	memcpy(d + 4, frame[k] + 26, 8);
	return (int)(oracle_crc32c(d, 12, 0) % (uint32_t)nq);
}

#define MQ_IN  4
#define MQ_OUT 2

static void case_multiqueue(odp_pool_t pool, odp_pktin_mode_t mode, int hash)
{
	odp_pktio_param_t pp;
	odp_pktin_queue_param_t ip;
	odp_pktout_queue_param_t op;
	odp_pktio_capability_t capa;
	odp_pktin_queue_t inq[MQ_IN];
	odp_queue_t evq[MQ_IN];
	odp_pktout_queue_t outq[MQ_OUT];
	odp_packet_parse_param_t prm;
	int cnt[MQ_IN] = {0}, last[MQ_IN], got = 0, where_ok = 1, order_ok = 1;
	uint64_t oct[MQ_IN] = {0};
	const char *mname = mode == ODP_PKTIN_MODE_DIRECT ? "direct" : "sched";

	odp_pktio_param_init(&pp);
	pp.in_mode = mode;
	pp.out_mode = ODP_PKTOUT_MODE_DIRECT;
	odp_pktio_t pktio = odp_pktio_open("loop3", pool, &pp);

	CHECK(pktio != ODP_PKTIO_INVALID, "open loop3");
	if (pktio == ODP_PKTIO_INVALID)
		return;
	CHECK(odp_pktio_capability(pktio, &capa) == 0 && capa.max_input_queues >= MQ_IN &&
	      capa.max_output_queues >= MQ_OUT, "multi-queue capability");
	odp_pktin_queue_param_init(&ip);
	ip.num_queues = MQ_IN;
	ip.hash_enable = hash;
	ip.hash_proto.proto.ipv4_udp = 1;
	ip.hash_proto.proto.ipv4 = 1;
	odp_pktout_queue_param_init(&op);
	op.num_queues = MQ_OUT;
	CHECK(odp_pktin_queue_config(pktio, &ip) == 0, "%d input queues", MQ_IN);
	CHECK(odp_pktout_queue_config(pktio, &op) == 0, "%d output queues", MQ_OUT);
	if (mode == ODP_PKTIN_MODE_DIRECT)
		CHECK(odp_pktin_queue(pktio, inq, MQ_IN) == MQ_IN, "odp_pktin_queue: %d", MQ_IN);
	else
		CHECK(odp_pktin_event_queue(pktio, evq, MQ_IN) == MQ_IN, "event queues: %d", MQ_IN);
	CHECK(odp_pktout_queue(pktio, outq, MQ_OUT) == MQ_OUT, "odp_pktout_queue: %d", MQ_OUT);
	CHECK(odp_pktio_start(pktio) == 0, "start");
	memset(&prm, 0, sizeof(prm));
	prm.proto = ODP_PROTO_ETH;
	prm.last_layer = ODP_PROTO_LAYER_ALL;
	for (int k = 0; k < NPKT; k++) {
		odp_packet_t pkt = odp_packet_alloc(pool, flen[k]);

		CHECK(pkt != ODP_PACKET_INVALID, "alloc");
		if (pkt == ODP_PACKET_INVALID)
			break;
		memcpy(odp_packet_data(pkt), frame[k], flen[k]);
		CHECK(odp_packet_parse(pkt, 0, &prm) == 0, "parse frame %d", k);
		if (odp_pktout_send(outq[k % MQ_OUT], &pkt, 1) != 1) {
			CHECK(0, "send frame %d", k);
			odp_packet_free(pkt);
		}
	}
	for (int q = 0; q < MQ_IN; q++)
		last[q] = -1;
	/* a received packet: its queue and its place in that queue's order */
	#define MQ_TAKE(pkt, q) do { \
		const int k_ = which_frame(pkt); \
		const int want_ = k_ < 0 ? -1 : hash ? expected_queue(k_, MQ_IN) : (k_ % MQ_OUT) % MQ_IN; \
		if (k_ < 0 || want_ != (q)) \
			where_ok = 0; \
		if (k_ <= last[q]) \
			order_ok = 0; \
		if (k_ >= 0) { \
			last[q] = k_; \
			oct[q] += flen[k_]; \
		} \
		cnt[q]++; \
		got++; \
		odp_packet_free(pkt); \
	} while (0)
	if (mode == ODP_PKTIN_MODE_DIRECT) {
		odp_packet_t pkts[64];

		for (int q = 0; q < MQ_IN; q++) {
			int n;

			while ((n = odp_pktin_recv(inq[q], pkts, 64)) > 0)
				for (int i = 0; i < n; i++)
					MQ_TAKE(pkts[i], q);
			CHECK(n == 0, "odp_pktin_recv on queue %d: %d", q, n);
		}
	} else {
		for (;;) {
			odp_queue_t from;
			odp_event_t ev = odp_schedule(&from,
						      odp_schedule_wait_time(200 * ODP_TIME_MSEC_IN_NS));
			int q = -1;

			if (ev == ODP_EVENT_INVALID)
				break;
			for (int j = 0; j < MQ_IN; j++)
				if (from == evq[j])
					q = j;
			CHECK(q >= 0, "scheduled from a pktin event queue");
			if (q < 0) {
				odp_event_free(ev);
				continue;
			}
			MQ_TAKE(odp_packet_from_event(ev), q);
		}
	}
	#undef MQ_TAKE
	CHECK(got == NPKT, "G %s hash=%d: received %d of %d", mname, hash, got, NPKT);
	CHECK(where_ok, "G %s hash=%d: every packet on the queue the pick names", mname, hash);
	CHECK(order_ok, "G %s hash=%d: sending order per queue", mname, hash);
	int used = 0;

	for (int q = 0; q < MQ_IN; q++) {
		odp_pktin_queue_stats_t is;

		used += cnt[q] > 0;
		if (mode == ODP_PKTIN_MODE_DIRECT)
			CHECK(odp_pktin_queue_stats(inq[q], &is) == 0 && is.packets == (uint64_t)cnt[q] &&
			      is.octets == oct[q], "queue %d stats %lu vs %d", q,
			      (unsigned long)is.packets, cnt[q]);
		else
			CHECK(odp_pktin_event_queue_stats(pktio, evq[q], &is) == 0 &&
			      is.packets == (uint64_t)cnt[q], "event queue %d stats", q);
	}
	CHECK(used == (hash ? MQ_IN : MQ_OUT), "G %s hash=%d: %d queues used", mname, hash, used);
	for (int q = 0; q < MQ_OUT; q++) {
		odp_pktout_queue_stats_t os;

		CHECK(odp_pktout_queue_stats(outq[q], &os) == 0 && os.packets == NPKT / MQ_OUT,
		      "output queue %d stats", q);
	}
	CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "stop / close");
	printf("G %s hash=%d: %d packets over queues %d/%d/%d/%d, in order\n", mname, hash, got,
	       cnt[0], cnt[1], cnt[2], cnt[3]);
}

/* F: multi-threaded scheduled receive (chunked delivery) */
#define MT_RX 4
#define MT_N  200000
static uint8_t *mt_seen;
static uint32_t mt_got, mt_bad;
static int mt_stop;
static odp_instance_t mt_inst;

static void *mt_rx(void *arg)
{
	uint32_t last = 0;
	int have_last = 0;

	(void)arg;
	odp_init_local(mt_inst, ODP_THREAD_WORKER);
	while (!__atomic_load_n(&mt_stop, __ATOMIC_ACQUIRE)) {
		odp_event_t ev[32];
		const int n = odp_schedule_multi(NULL, ODP_SCHED_NO_WAIT, ev, 32);

		for (int i = 0; i < n; i++) {
			odp_packet_t pkt = odp_packet_from_event(ev[i]);
			const uint8_t *d = odp_packet_data(pkt);
			uint32_t seq;

			memcpy(&seq, d + 42, 4);
			if (odp_packet_len(pkt) != 64 || seq >= MT_N ||
			    __atomic_exchange_n(&mt_seen[seq], 1, __ATOMIC_RELAXED) ||
			    (have_last && seq <= last))
				__atomic_fetch_add(&mt_bad, 1u, __ATOMIC_RELAXED);
			last = seq;
			have_last = 1;
			odp_event_free(ev[i]);
		}
		if (n > 0)
			__atomic_fetch_add(&mt_got, (uint32_t)n, __ATOMIC_RELAXED);
	}
	odp_term_local();
	return NULL;
}

static void case_sched_mt(void)
{
	odp_pool_param_t pp;
	odp_pool_t rxp, txp;
	odp_pktout_queue_t out;
	pthread_t t[MT_RX];

	odp_pool_param_init(&pp);
	pp.type = ODP_POOL_PACKET;
	pp.pkt.num = 16384;
	pp.pkt.len = 64;
	rxp = odp_pool_create("mt_rx", &pp);
	txp = odp_pool_create("mt_tx", &pp);
	CHECK(rxp != ODP_POOL_INVALID && txp != ODP_POOL_INVALID, "F pools");
	odp_pktio_t pktio = open_loop("loop_mt", rxp, ODP_PKTIN_MODE_SCHED, ODP_PKTOUT_MODE_DIRECT, 0);

	CHECK(pktio != ODP_PKTIO_INVALID, "F open");
	if (pktio == ODP_PKTIO_INVALID)
		return;
	mt_seen = calloc(MT_N, 1);
	CHECK(odp_pktout_queue(pktio, &out, 1) == 1 && odp_pktio_start(pktio) == 0, "F start");
	for (int i = 0; i < MT_RX; i++)
		pthread_create(&t[i], NULL, mt_rx, NULL);
	for (uint32_t seq = 0; seq < MT_N;) {
		odp_packet_t pk[32];
		int n = 0;

		for (; n < 32 && seq + (uint32_t)n < MT_N; n++) {
			pk[n] = odp_packet_alloc(txp, 64);
			if (pk[n] == ODP_PACKET_INVALID)
				break;
			uint8_t *d = odp_packet_data(pk[n]);
			const uint32_t v = seq + (uint32_t)n;

			memcpy(d, frame[0], 64);
			memcpy(d + 42, &v, 4);
		}
		const int sent = n ? odp_pktout_send(out, pk, n) : 0;

		if (sent > 0)
			seq += (uint32_t)sent;
		if (sent < n)
			odp_packet_free_multi(pk + (sent > 0 ? sent : 0), n - (sent > 0 ? sent : 0));
		if (sent <= 0)
			usleep(50);   /* the transmit pool is in flight: let it drain */
	}
	for (int w = 0; w < 20000 && __atomic_load_n(&mt_got, __ATOMIC_RELAXED) < MT_N; w++)
		usleep(500);
	__atomic_store_n(&mt_stop, 1, __ATOMIC_RELEASE);
	for (int i = 0; i < MT_RX; i++)
		pthread_join(t[i], NULL);
	CHECK(mt_got == MT_N, "F received %u of %u", mt_got, MT_N);
	CHECK(mt_bad == 0, "F %u packets duplicated, corrupt or out of sending order", mt_bad);
	CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "F stop / close");
	CHECK(odp_pool_destroy(rxp) == 0 && odp_pool_destroy(txp) == 0, "F pool destroy");
	free(mt_seen);
	printf("F sched, %d threads: %u packets, each once and in order per thread\n", MT_RX, mt_got);
}

static void case_queue(odp_pool_t pool)
{
	odp_pktio_t pktio = open_loop("loop2", pool, ODP_PKTIN_MODE_QUEUE,
				      ODP_PKTOUT_MODE_QUEUE, 0);
	odp_queue_t inq, outq;
	odp_pktout_queue_t oq;
	odp_pktout_queue_stats_t os;
	int got = 0, seen_ok = 1;

	CHECK(pktio != ODP_PKTIO_INVALID, "open loop2");
	if (pktio == ODP_PKTIO_INVALID)
		return;
	CHECK(odp_pktout_queue(pktio, &oq, 1) == -1, "pktout queue in QUEUE mode");
	CHECK(odp_pktin_event_queue(pktio, &inq, 1) == 1, "pktin event queue");
	CHECK(odp_pktout_event_queue(pktio, &outq, 1) == 1, "pktout event queue");
	CHECK(odp_pktio_start(pktio) == 0, "start");
	for (int k = 0; k < NPKT; k++) {
		odp_packet_t pkt = odp_packet_alloc(pool, flen[k]);

		memcpy(odp_packet_data(pkt), frame[k], flen[k]);
		if (odp_queue_enq(outq, odp_packet_to_event(pkt))) {
			seen_ok = 0;
			odp_packet_free(pkt);
		}
	}
	for (int tries = 0; got < NPKT && tries < 100000; tries++) {
		odp_event_t ev = odp_queue_deq(inq);

		if (ev == ODP_EVENT_INVALID)
			continue;
		if (which_frame(odp_packet_from_event(ev)) != got)
			seen_ok = 0;
		got++;
		odp_event_free(ev);
	}
	CHECK(got == NPKT && seen_ok, "queue mode: %d of %d back in order", got, NPKT);
	CHECK(odp_pktout_event_queue_stats(pktio, outq, &os) == 0 && os.packets == NPKT,
	      "pktout event queue stats");
	CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "stop/close");
	printf("C queue: %d packets\n", got);
}

/* a capture of the first 20 frames */
static int write_pcap(const char *path)
{
	FILE *f = fopen(path, "wb");
	const uint32_t gh[6] = { 0xa1b2c3d4u, 0x00040002u, 0, 0, 65535, 1 };

	if (!f)
		return -1;
	fwrite(gh, 4, 6, f);
	for (int k = 0; k < 20; k++) {
		const uint32_t rh[4] = { (uint32_t)k, 0, flen[k], flen[k] };

		fwrite(rh, 4, 4, f);
		fwrite(frame[k], 1, flen[k], f);
	}
	return fclose(f);
}

static void case_pcap_loops(odp_pool_t pool)
{
	char path[] = "/tmp/odp_rt_loop_XXXXXX";
	const int fd = mkstemp(path);
	const uint32_t loops[4] = { 1, 2, 3, 4 }, passes[4] = { 1, 1, 2, 3 };

	CHECK(fd >= 0 && write_pcap(path) == 0, "write capture");
	if (fd < 0)
		return;
	close(fd);
	for (int t = 0; t < 4; t++) {
		char dev[128];
		odp_pktin_queue_t inq;
		odp_packet_t pkts[64];
		int got = 0;

		snprintf(dev, sizeof(dev), "pcap:in=%s:loops=%u", path, loops[t]);
		odp_pktio_t pktio = open_loop(dev, pool, ODP_PKTIN_MODE_DIRECT,
					      ODP_PKTOUT_MODE_DIRECT, 0);

		CHECK(pktio != ODP_PKTIO_INVALID, "open %s", dev);
		if (pktio == ODP_PKTIO_INVALID)
			continue;
		CHECK(odp_pktin_queue(pktio, &inq, 1) == 1 && odp_pktio_start(pktio) == 0,
		      "start pcap");
		for (int tries = 0; tries < 100; tries++) {
			const int n = odp_pktin_recv(inq, pkts, 64);

			if (n <= 0)
				break;
			got += n;
			odp_packet_free_multi(pkts, n);
		}
		CHECK(got == (int)(20 * passes[t]), "loops=%u: %d packets, want %u", loops[t], got,
		      20 * passes[t]);
		CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "stop/close pcap");
		printf("D pcap loops=%u: %d packets\n", loops[t], got);
	}
	unlink(path);
}

/* E: DIRECT receive of a capture one frame at a time into a 4-packet pool:
 * a capture frame needs a packet from the pool, so the receive reads `num`
 * frames per call (pcap_recv) and loses none, whatever the pool's size */
static void case_pcap_small_pool(void)
{
	char path[] = "/tmp/odp_rt_loop_XXXXXX";
	const int fd = mkstemp(path);
	odp_pool_param_t pp;

	CHECK(fd >= 0 && write_pcap(path) == 0, "write capture");
	if (fd < 0)
		return;
	close(fd);
	odp_pool_param_init(&pp);
	pp.type = ODP_POOL_PACKET;
	pp.pkt.num = 4;
	pp.pkt.len = 1600;
	odp_pool_t small = odp_pool_create("small", &pp);
	char dev[128];
	odp_pktin_queue_t inq;
	int got = 0, tries = 0;

	CHECK(small != ODP_POOL_INVALID, "small pool");
	snprintf(dev, sizeof(dev), "pcap:in=%s", path);
	odp_pktio_t pktio = open_loop(dev, small, ODP_PKTIN_MODE_DIRECT, ODP_PKTOUT_MODE_DIRECT, 0);

	CHECK(pktio != ODP_PKTIO_INVALID, "open %s", dev);
	if (pktio != ODP_PKTIO_INVALID) {
		CHECK(odp_pktin_queue(pktio, &inq, 1) == 1 && odp_pktio_start(pktio) == 0,
		      "start pcap");
		for (; tries < 100; tries++) {
			odp_packet_t pkt;
			const int n = odp_pktin_recv(inq, &pkt, 1);

			if (n <= 0)
				break;
			CHECK(which_frame(pkt) == got, "frame %d out of order", got);
			got++;
			odp_packet_free(pkt);
		}
		CHECK(got == 20, "one at a time into 4 packets: %d of 20 frames", got);
		CHECK(odp_pktio_stop(pktio) == 0 && odp_pktio_close(pktio) == 0, "stop/close pcap");
	}
	CHECK(odp_pool_destroy(small) == 0, "small pool destroy");
	printf("E pcap small pool: %d packets\n", got);
	unlink(path);
}

int main(void)
{
	odp_instance_t inst;
	odp_pool_param_t pp;

	odp_pool_capability_t pc;
	odp_schedule_capability_t sc;
	odp_pool_t pool;

	make_frames();
	if (odp_init_global(&inst, NULL, NULL) || odp_init_local(inst, ODP_THREAD_CONTROL)) {
		printf("FAIL init\n");
		return 2;
	}
	CHECK(odp_schedule_config(NULL) == 0, "schedule config");
	CHECK(odp_pool_capability(&pc) == 0 && pc.pkt.max_pools > 0, "pool capability");
	CHECK(odp_schedule_capability(&sc) == 0 && sc.max_queues > 0, "schedule capability");
	odp_pool_param_init(&pp);
	pp.type = ODP_POOL_PACKET;
	pp.pkt.num = 4 * NPKT;
	pp.pkt.len = 1600;
	pool = odp_pool_create("pkts", &pp);
	CHECK(pool != ODP_POOL_INVALID, "pool");
	case_direct(pool);
	case_sched_cls(pool);
	case_queue(pool);
	case_pcap_loops(pool);
	case_pcap_small_pool();
	case_multiqueue(pool, ODP_PKTIN_MODE_DIRECT, 1);
	case_multiqueue(pool, ODP_PKTIN_MODE_SCHED, 1);
	case_multiqueue(pool, ODP_PKTIN_MODE_DIRECT, 0);
	mt_inst = inst;
	case_sched_mt();
	CHECK(odp_pool_destroy(pool) == 0, "pool destroy");
	odp_term_local();
	odp_term_global(inst);
	printf("%s (%d failed checks)\n", fails ? "FAIL" : "PASS", fails);
	return fails ? 1 : 0;
}
