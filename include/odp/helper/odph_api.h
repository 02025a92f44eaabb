/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp/helper/odph_api.h — the ODP helper subset the library's runtime
 * serves (the headers under helper/include/odp/helper): option parsing, threads
 * (pthreads), Ethernet / IPv4 header types and address parsers.
 */
#ifndef ODPH_API_H_
#define ODPH_API_H_

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../odp_api.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ODPH_ERR(fmt, ...) \
	fprintf(stderr, "%s:%d:%s(): " fmt, __FILE__, __LINE__, __func__, ##__VA_ARGS__)
#define ODPH_DBG(fmt, ...) do { } while (0)
#define ODPH_ABORT(fmt, ...) do { \
	fprintf(stderr, "%s:%d:%s(): " fmt, __FILE__, __LINE__, __func__, ##__VA_ARGS__); \
	abort(); \
} while (0)
#define ODPH_ASSERT(cond) do { \
	if (!(cond)) \
		ODPH_ABORT("%s\n", #cond); \
} while (0)
#define ODPH_ARRAY_SIZE(x) (sizeof(x) / sizeof((x)[0]))

/* ---- protocol headers (eth.h, ip.h, udp.h, tcp.h) ----------------------- */
#define ODPH_ETHADDR_LEN   6
#define ODPH_ETHHDR_LEN    14
#define ODPH_ETHTYPE_IPV4  0x0800
#define ODPH_ETHTYPE_IPV6  0x86dd
#define ODPH_ETHTYPE_ARP   0x0806
#define ODPH_ETHTYPE_VLAN  0x8100
#define ODPH_ETHTYPE_VLAN_OUTER 0x88A8
#define ODPH_IPV4          4
#define ODPH_IPV4HDR_LEN   20
#define ODPH_IPV4HDR_IHL_MIN 5
#define ODPH_IPV4ADDR_LEN  4
#define ODPH_IPV4HDR_VER(ver_ihl) (((ver_ihl) & 0xf0) >> 4)
#define ODPH_IPV4HDR_IHL(ver_ihl) ((ver_ihl) & 0x0f)
#define ODPH_IPV4HDR_CSUM_OFFSET 10
#define ODPH_IPV6          6
#define ODPH_IPV6HDR_LEN   40
#define ODPH_UDPHDR_LEN    8
#define ODPH_TCPHDR_LEN    20
#define ODPH_IPPROTO_UDP   0x11
#define ODPH_IPPROTO_TCP   0x06
#define ODPH_IPPROTO_ICMPV4 0x01
#define ODPH_IPPROTO_SCTP  0x84

typedef struct __attribute__((packed)) odph_ethaddr_t {
	uint8_t addr[ODPH_ETHADDR_LEN];
} odph_ethaddr_t;

typedef struct __attribute__((packed)) odph_ethhdr_t {
	odph_ethaddr_t dst;
	odph_ethaddr_t src;
	odp_u16be_t type;
} odph_ethhdr_t;

typedef struct odph_ipv4hdr_t {
	uint8_t ver_ihl;
	uint8_t tos;
	odp_u16be_t tot_len;
	odp_u16be_t id;
	odp_u16be_t frag_offset;
	uint8_t ttl;
	uint8_t proto;
	odp_u16sum_t chksum;
	odp_u32be_t src_addr;
	odp_u32be_t dst_addr;
} odph_ipv4hdr_t;

typedef struct odph_udphdr_t {
	odp_u16be_t src_port;
	odp_u16be_t dst_port;
	odp_u16be_t length;
	odp_u16sum_t chksum;
} odph_udphdr_t;

int odph_eth_addr_parse(odph_ethaddr_t *mac, const char *str);
int odph_ipv4_addr_parse(uint32_t *ip_addr, const char *str);

/* IPv4 header checksum at the packet's L3 offset (helper ip.h:98-193):
 * _update writes it (0, or < 0 when there is no IPv4 header there), _valid
 * returns 1 when the stored one is right, else 0 */
int odph_ipv4_csum_update(odp_packet_t pkt);
int odph_ipv4_csum_valid(odp_packet_t pkt);

/* odph_strcpy (helper/include/odp/helper/string.h): strncpy that always
 * terminates; returns dst */
char *odph_strcpy(char *dst, const char *src, size_t sz);

/* ---- options and threads (threads.h) ------------------------------------ */
typedef struct odph_helper_options_t {
	odp_mem_model_t mem_model;
	int64_t shm_size;
} odph_helper_options_t;

int odph_parse_options(int argc, char *argv[]);
int odph_options(odph_helper_options_t *options);

typedef struct odph_thread_param_t {
	int (*start)(void *arg);
	void *arg;
	odp_thread_type_t thr_type;
	uint64_t stack_size;
} odph_thread_param_t;

typedef enum odph_thread_sync_t { ODPH_THREAD_SYNC_DEFAULT = 0 } odph_thread_sync_t;

typedef struct odph_thread_common_param_t {
	odp_instance_t instance;
	const odp_cpumask_t *cpumask;
	int thread_model;            /* 0: pthreads (the only model here) */
	int sync;
	int sync_timeout;
	int share_param;
} odph_thread_common_param_t;

typedef struct odph_thread_t {
	uint64_t thread;             /* pthread_t */
	int cpu;
	int status;
	odph_thread_param_t param;
	odp_instance_t instance;
	int started;
} odph_thread_t;

void odph_thread_common_param_init(odph_thread_common_param_t *param);
void odph_thread_param_init(odph_thread_param_t *param);
int  odph_thread_create(odph_thread_t thread[], const odph_thread_common_param_t *param,
			const odph_thread_param_t thr_param[], int num);
int  odph_thread_join(odph_thread_t thread[], int num);

#ifdef __cplusplus
}
#endif

#endif
