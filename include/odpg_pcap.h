/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odpg_pcap.h — capture files into a classifier batch (SURVEY.md §8(f)
 * rank 4). The reference replays its example / performance captures through
 * the pcap pktio (platform/linux-generic/pktio/pcap.c, pcapif_recv_pkt :281-360 on libpcap);
 * here a capture is read straight into one host buffer of frames plus an
 * odpg_desc_t per frame, the layout odpg_classify / odpg_classify_host /
 * odpg_pktio_recv_batch take.
 *
 * Formats: classic pcap (either byte order, microsecond or nanosecond
 * magic) and pcapng (section header, interface description, enhanced and
 * simple packet blocks, either byte order). Link type Ethernet only. Each
 * frame is its captured bytes (caplen), as the pcap pktio delivers them.
 */
#ifndef ODPG_PCAP_H_
#define ODPG_PCAP_H_

#include <stdint.h>

#include "odpg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct odpg_capture_s {
	uint8_t     *frames;   /* host buffer, frames at `align`-aligned offsets */
	odpg_desc_t *desc;     /* num entries {offset, len} into frames */
	uint32_t     num;
	uint64_t     bytes;    /* size of frames (with padding and a 128 B tail) */
} odpg_capture_t;

/* Read a whole capture. align: 1 .. 4096, a power of two (64 matches pool
 * segment alignment). Returns 0, or -ENOENT (cannot open), -EINVAL (bad
 * arguments, not a pcap / pcapng file, unsupported link type, truncated
 * record), -ENOMEM. */
int  odpg_pcap_read(const char *path, uint32_t align, odpg_capture_t *cap);
void odpg_pcap_free(odpg_capture_t *cap);

#ifdef __cplusplus
}
#endif

#endif /* ODPG_PCAP_H_ */
