/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp_classifier_gpu — example/classifier's classification run on the
 * MI355X library.
 *
 * Same rule syntax, CoS naming and CI pass check as the reference example
 * (example/classifier/odp_classifier.c: parse_pmr_policy :918-1111,
 * configure_default_cos :471-540, configure_cos :542-624,
 * check_ci_pass_count :134-164), so its test line
 *   odp_classifier -i $IF0 -m 0 -p "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1"
 *                  -P -C "queue1:100" -C "DefaultCos:100"
 * (example/classifier/odp_classifier_run.sh:17-19, pktio_env:21-22) runs as
 *   odp_classifier_gpu -i udp64.pcap -p "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1"
 *                      -C "queue1:100" -C "DefaultCos:100"
 * The interface is a capture file (the reference's pcap pktio input); the
 * rules go through the odp_cls_* API of libodpg (include/odp_cls.h), the
 * capture through odpg_pcap_read, and the whole capture is classified in one
 * odpg_pktio_recv_batch call on the GPU. As in the reference's worker,
 * packets with parse errors are not counted (drop_err_pkts :812-835), and a
 * CI rule passes when its CoS received at least the given count.
 * Options -m, -t, -c, -P, -v and -e are accepted for command-line
 * compatibility and ignored (there is no packet echo / timer here).
 */
#include <ctype.h>
#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <odp_cls.h>
#include <odpg.h>
#include <odpg_pcap.h>

#define MAX_PMR_COUNT 32
#define MAX_VAL_SIZE  16

typedef struct {
	char name[ODP_COS_NAME_LEN];
	odp_cos_t cos;
	uint64_t count;
} cos_ent_t;

typedef struct {
	odp_cls_pmr_term_t term;
	uint8_t value[MAX_VAL_SIZE], mask[MAX_VAL_SIZE];
	uint32_t val_sz, offset;
	char src[ODP_COS_NAME_LEN], dst[ODP_COS_NAME_LEN];
	int has_src;
} policy_t;

static cos_ent_t coses[MAX_PMR_COUNT + 1];
static int ncos;

static int term_from_str(const char *t, odp_cls_pmr_term_t *term)
{
	static const struct {
		const char *s;
		odp_cls_pmr_term_t t;
	} map[] = {
		{"ODP_PMR_ETHTYPE_0", ODP_PMR_ETHTYPE_0}, {"ODP_PMR_ETHTYPE_X", ODP_PMR_ETHTYPE_X},
		{"ODP_PMR_VLAN_ID_0", ODP_PMR_VLAN_ID_0}, {"ODP_PMR_VLAN_ID_X", ODP_PMR_VLAN_ID_X},
		{"ODP_PMR_UDP_DPORT", ODP_PMR_UDP_DPORT}, {"ODP_PMR_TCP_DPORT", ODP_PMR_TCP_DPORT},
		{"ODP_PMR_UDP_SPORT", ODP_PMR_UDP_SPORT}, {"ODP_PMR_TCP_SPORT", ODP_PMR_TCP_SPORT},
		{"ODP_PMR_DIP_ADDR", ODP_PMR_DIP_ADDR}, {"ODP_PMR_SIP_ADDR", ODP_PMR_SIP_ADDR},
		{"ODP_PMR_DMAC", ODP_PMR_DMAC}, {"ODP_PMR_CUSTOM_FRAME", ODP_PMR_CUSTOM_FRAME},
		{"ODP_PMR_CUSTOM_L3", ODP_PMR_CUSTOM_L3},
	};

	for (size_t i = 0; t && i < sizeof(map) / sizeof(map[0]); i++)
		if (strcasecmp(t, map[i].s) == 0) {
			*term = map[i].t;
			return 0;
		}
	return -1;
}

/* hex string without 0x prefix -> bytes (parse_custom, :242-265) */
static int parse_hex(const char *s, uint8_t *out, int max)
{
	int n = (int)strlen(s);

	if (n == 0 || (n & 1) || n / 2 > max)
		return -1;
	for (int i = 0; i < n / 2; i++) {
		unsigned v;

		if (!isxdigit((unsigned char)s[2 * i]) || !isxdigit((unsigned char)s[2 * i + 1]) ||
		    sscanf(s + 2 * i, "%2x", &v) != 1)
			return -1;
		out[i] = (uint8_t)v;
	}
	return n / 2;
}

static int parse_ipv4(const char *s, uint32_t *ip)
{
	unsigned a, b, c, d;
	char tail;

	if (sscanf(s, "%u.%u.%u.%u%c", &a, &b, &c, &d, &tail) != 4 || a > 255 || b > 255 ||
	    c > 255 || d > 255)
		return -1;
	*ip = (a << 24) | (b << 16) | (c << 8) | d;
	return 0;
}

/* parse_pmr_policy (odp_classifier.c:918-1111): values in network order */
static int parse_policy(char *arg, policy_t *p)
{
	char *tok = strtok(arg, ":"), *c0, *c1;
	unsigned long v;

	memset(p, 0, sizeof(*p));
	if (term_from_str(tok, &p->term))
		return -1;
	switch (p->term) {
	case ODP_PMR_ETHTYPE_0:
	case ODP_PMR_ETHTYPE_X:
	case ODP_PMR_VLAN_ID_0:
	case ODP_PMR_VLAN_ID_X:
	case ODP_PMR_UDP_DPORT:
	case ODP_PMR_TCP_DPORT:
	case ODP_PMR_UDP_SPORT:
	case ODP_PMR_TCP_SPORT:
		if (!(tok = strtok(NULL, ":")))
			return -1;
		v = strtoul(tok, NULL, 0);
		p->value[0] = (uint8_t)(v >> 8);
		p->value[1] = (uint8_t)v;
		if (!(tok = strtok(NULL, ":")))
			return -1;
		v = strtoul(tok, NULL, 0);
		p->mask[0] = (uint8_t)(v >> 8);
		p->mask[1] = (uint8_t)v;
		p->val_sz = 2;
		break;
	case ODP_PMR_DIP_ADDR:
	case ODP_PMR_SIP_ADDR: {
		uint32_t ip;

		if (!(tok = strtok(NULL, ":")) || parse_ipv4(tok, &ip))
			return -1;
		for (int i = 0; i < 4; i++)
			p->value[i] = (uint8_t)(ip >> (24 - 8 * i));
		if (!(tok = strtok(NULL, ":")))
			return -1;
		v = strtoul(tok, NULL, 0);
		for (int i = 0; i < 4; i++)
			p->mask[i] = (uint8_t)(v >> (24 - 8 * i));
		p->val_sz = 4;
		break;
	}
	case ODP_PMR_DMAC: {
		/* :<11-22-33-44-55-66>:<mask hex> */
		unsigned m[6];

		if (!(tok = strtok(NULL, ":")) ||
		    sscanf(tok, "%x-%x-%x-%x-%x-%x", &m[0], &m[1], &m[2], &m[3], &m[4], &m[5]) != 6)
			return -1;
		for (int i = 0; i < 6; i++)
			p->value[i] = (uint8_t)m[i];
		p->val_sz = 6;
		if (!(tok = strtok(NULL, ":")) || parse_hex(tok, p->mask, 6) != 6)
			return -1;
		break;
	}
	case ODP_PMR_CUSTOM_FRAME:
	case ODP_PMR_CUSTOM_L3: {
		/* :<offset>:<value hex>:<mask hex> */
		int vs, ms;

		if (!(tok = strtok(NULL, ":")))
			return -1;
		errno = 0;
		p->offset = (uint32_t)strtoul(tok, NULL, 0);
		if (errno || !(tok = strtok(NULL, ":")))
			return -1;
		vs = parse_hex(tok, p->value, MAX_VAL_SIZE);
		if (vs <= 0 || !(tok = strtok(NULL, ":")))
			return -1;
		ms = parse_hex(tok, p->mask, MAX_VAL_SIZE);
		if (ms != vs)
			return -1;
		p->val_sz = (uint32_t)vs;
		break;
	}
	default:
		return -1;
	}
	c0 = strtok(NULL, ":");
	c1 = strtok(NULL, ":");
	if (!c0)
		return -1;
	if (c1) {
		p->has_src = 1;
		snprintf(p->src, sizeof(p->src), "%s", c0);
		snprintf(p->dst, sizeof(p->dst), "%s", c1);
	} else {
		snprintf(p->dst, sizeof(p->dst), "%s", c0);
	}
	return 0;
}

static cos_ent_t *find_cos(const char *name)
{
	for (int i = 0; i < ncos; i++)
		if (strcmp(coses[i].name, name) == 0)
			return &coses[i];
	return NULL;
}

static void usage(const char *prog)
{
	fprintf(stderr,
		"usage: %s -i <capture.pcap|pcapng> -p <policy> [-p ...] [-C <cos>:<count> ...]\n"
		"  policy: <ODP_PMR_term>:<value>:<mask>[:<src_cos>]:<cos>  (example/classifier syntax)\n",
		prog);
}

int main(int argc, char *argv[])
{
	static const struct option longopts[] = {
		{"interface", required_argument, NULL, 'i'}, {"policy", required_argument, NULL, 'p'},
		{"ci_pass", required_argument, NULL, 'C'}, {"mode", required_argument, NULL, 'm'},
		{"time", required_argument, NULL, 't'}, {"count", required_argument, NULL, 'c'},
		{"help", no_argument, NULL, 'h'}, {NULL, 0, NULL, 0}};
	policy_t pol[MAX_PMR_COUNT];
	struct { char name[ODP_COS_NAME_LEN]; uint64_t count; } ci[MAX_PMR_COUNT];
	int npol = 0, nci = 0, opt;
	const char *input = NULL;

	while ((opt = getopt_long(argc, argv, "+i:p:C:m:t:c:e:Pvh", longopts, NULL)) != -1) {
		switch (opt) {
		case 'i':
			input = optarg;
			break;
		case 'p':
			if (npol >= MAX_PMR_COUNT - 1 || parse_policy(optarg, &pol[npol])) {
				fprintf(stderr, "Error: bad policy '%s'\n", optarg);
				return EXIT_FAILURE;
			}
			npol++;
			break;
		case 'C': {
			char *c = strchr(optarg, ':');

			if (!c || nci >= MAX_PMR_COUNT) {
				fprintf(stderr, "Error: bad ci_pass '%s'\n", optarg);
				return EXIT_FAILURE;
			}
			*c = '\0';
			snprintf(ci[nci].name, sizeof(ci[nci].name), "%s", optarg);
			ci[nci].count = strtoull(c + 1, NULL, 0);
			nci++;
			break;
		}
		case 'h':
			usage(argv[0]);
			return EXIT_SUCCESS;
		default:
			break;                     /* -m -t -c -e -P -v: accepted, ignored */
		}
	}
	if (!input || npol == 0) {
		usage(argv[0]);
		return EXIT_FAILURE;
	}

	/* loop pktio with the classifier enabled, parser layer ALL */
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
	if (odp_pktio_config(pktio, &cfg) || odp_pktin_queue_config(pktio, &qp)) {
		fprintf(stderr, "Error: pktio config failed\n");
		return EXIT_FAILURE;
	}

	/* configure_default_cos + configure_cos: one CoS (own queue) per name */
	odp_cls_cos_param_t cp;

	odp_cls_cos_param_init(&cp);
	cp.queue = (odp_queue_t)(uintptr_t)0x1000;
	snprintf(coses[0].name, sizeof(coses[0].name), "DefaultCos");
	coses[0].cos = odp_cls_cos_create("DefaultCos", &cp);
	ncos = 1;
	if (coses[0].cos == ODP_COS_INVALID || odp_pktio_default_cos_set(pktio, coses[0].cos)) {
		fprintf(stderr, "Error: default CoS failed\n");
		return EXIT_FAILURE;
	}
	for (int i = 0; i < npol; i++) {
		char cname[ODP_COS_NAME_LEN + 4];

		if (find_cos(pol[i].dst))
			continue;
		odp_cls_cos_param_init(&cp);
		cp.queue = (odp_queue_t)(uintptr_t)(0x1000 + ncos);
		snprintf(cname, sizeof(cname), "CoS%s", pol[i].dst);
		snprintf(coses[ncos].name, sizeof(coses[ncos].name), "%s", pol[i].dst);
		coses[ncos].cos = odp_cls_cos_create(cname, &cp);
		if (coses[ncos].cos == ODP_COS_INVALID) {
			fprintf(stderr, "Error: CoS %s failed\n", pol[i].dst);
			return EXIT_FAILURE;
		}
		ncos++;
	}
	for (int i = 0; i < npol; i++) {
		odp_pmr_param_t pp;
		cos_ent_t *src = pol[i].has_src ? find_cos(pol[i].src) : &coses[0];
		cos_ent_t *dst = find_cos(pol[i].dst);

		if (!src || !dst) {
			fprintf(stderr, "Error: unknown CoS in policy %d\n", i);
			return EXIT_FAILURE;
		}
		odp_cls_pmr_param_init(&pp);
		pp.term = pol[i].term;
		pp.match.value = pol[i].value;
		pp.match.mask = pol[i].mask;
		pp.val_sz = pol[i].val_sz;
		pp.offset = pol[i].offset;
		if (odp_cls_pmr_create(&pp, 1, src->cos, dst->cos) == ODP_PMR_INVALID) {
			fprintf(stderr, "Error: PMR %d create failed\n", i);
			return EXIT_FAILURE;
		}
	}
	if (odp_pktio_start(pktio)) {
		fprintf(stderr, "Error: pktio start failed\n");
		return EXIT_FAILURE;
	}

	/* the capture, classified on the GPU in one batch */
	odpg_capture_t capf;
	int rc = odpg_pcap_read(input, 64, &capf);

	if (rc) {
		fprintf(stderr, "Error: cannot read %s (%d)\n", input, rc);
		return EXIT_FAILURE;
	}
	odpg_ctx_t *ctx = NULL;
	odpg_out_t *out = calloc(capf.num ? capf.num : 1, sizeof(*out));

	if (!out || (rc = odpg_ctx_create(0, NULL, &ctx))) {
		fprintf(stderr, "Error: no GPU context (%d)\n", rc);
		return EXIT_FAILURE;
	}
	rc = odpg_pktio_recv_batch(pktio, ctx, capf.frames, capf.desc, 0, capf.num, 0, out, NULL);
	if (rc) {
		fprintf(stderr, "Error: classification failed (%d)\n", rc);
		return EXIT_FAILURE;
	}

	/* per-CoS counts of delivered, error-free packets (drop_err_pkts) */
	uint64_t errs = 0;

	for (uint32_t i = 0; i < capf.num; i++) {
		const uint32_t w = out[i], c = w & 0xFFFFu;   /* bits 0..15: CoS index */

		if (w & (ODPG_OUT_ERROR | ODPG_OUT_CLS_DROP) || c >= ODPG_COS_NOCLS) {
			errs++;
			continue;
		}
		for (int k = 0; k < ncos; k++)
			if (odp_cos_to_u64(coses[k].cos) == (uint64_t)c + 1u)
				coses[k].count++;
	}
	printf("%u packets from %s, %" PRIu64 " not delivered\n", capf.num, input, errs);
	for (int k = 0; k < ncos; k++)
		printf("%-16s %" PRIu64 "\n", coses[k].name, coses[k].count);

	/* check_ci_pass_count (odp_classifier.c:134-164) */
	int fail = 0;

	for (int i = 0; i < nci; i++) {
		cos_ent_t *e = find_cos(ci[i].name);

		if (!e) {
			fprintf(stderr, "Error: Cos %s not found\n", ci[i].name);
			fail = 1;
		} else if (ci[i].count > e->count) {
			fprintf(stderr, "Error: Cos = %s, expected packets = %" PRIu64
				", received packet = %" PRIu64 "\n", e->name, ci[i].count, e->count);
			fail = 1;
		}
	}
	odpg_ctx_destroy(ctx);
	odpg_pcap_free(&capf);
	free(out);
	odp_pktio_stop(pktio);
	odp_pktio_close(pktio);
	if (fail) {
		fprintf(stderr, "Error: Packet count verification failed\n");
		return EXIT_FAILURE;
	}
	return EXIT_SUCCESS;
}
