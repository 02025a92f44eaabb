/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Capture files into a classifier batch (include/odpg_pcap.h). Replaces the
 * frame source of the pcap pktio (platform/linux-generic/pktio/pcap.c,
 * pcapif_recv_pkt :281-360, pkt_len = caplen :323) for replaying the
 * reference's example and performance captures: classic pcap and pcapng,
 * Ethernet link type, one frame per record (its captured bytes).
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/odpg_pcap.h"

#define LINKTYPE_ETHERNET 1u

static uint32_t rd32(const uint8_t *p, int swap)
{
	uint32_t x;

	memcpy(&x, p, 4);
	return swap ? __builtin_bswap32(x) : x;
}

static uint16_t rd16(const uint8_t *p, int swap)
{
	uint16_t x;

	memcpy(&x, p, 2);
	return swap ? __builtin_bswap16(x) : x;
}

/* growable list of (pointer into the file image, length) */
typedef struct {
	const uint8_t **p;
	uint32_t *len;
	uint32_t n, cap;
} recs_t;

static int recs_add(recs_t *r, const uint8_t *p, uint32_t len)
{
	if (r->n == r->cap) {
		uint32_t nc = r->cap ? 2 * r->cap : 256;
		const uint8_t **np = realloc(r->p, nc * sizeof(*np));
		uint32_t *nl;

		if (!np)
			return -ENOMEM;
		r->p = np;
		nl = realloc(r->len, nc * sizeof(*nl));
		if (!nl)
			return -ENOMEM;
		r->len = nl;
		r->cap = nc;
	}
	r->p[r->n] = p;
	r->len[r->n] = len;
	r->n++;
	return 0;
}

/* classic pcap: 24-byte global header, 16-byte record headers */
static int parse_pcap(const uint8_t *d, size_t n, recs_t *r)
{
	const uint32_t magic = rd32(d, 0);
	int swap;

	if (magic == 0xA1B2C3D4u || magic == 0xA1B23C4Du)
		swap = 0;
	else if (magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u)
		swap = 1;
	else
		return -EINVAL;
	if (n < 24 || (rd32(d + 20, swap) & 0x0fffffffu) != LINKTYPE_ETHERNET)
		return -EINVAL;
	for (size_t off = 24; off < n;) {
		if (off + 16 > n)
			return -EINVAL;
		const uint32_t incl = rd32(d + off + 8, swap);

		if (incl > n - off - 16)
			return -EINVAL;
		if (recs_add(r, d + off + 16, incl))
			return -ENOMEM;
		off += 16 + (size_t)incl;
	}
	return 0;
}

/* pcapng: blocks {type, total length, body, total length}; the section
 * header's byte-order magic sets the byte order of its section */
static int parse_pcapng(const uint8_t *d, size_t n, recs_t *r)
{
	int swap = 0;
	uint32_t nif = 0, if_link[64];

	for (size_t off = 0; off < n;) {
		if (off + 12 > n)
			return -EINVAL;
		uint32_t type = rd32(d + off, 0);

		if (type == 0x0A0D0D0Au) {                 /* section header */
			const uint32_t bom = rd32(d + off + 8, 0);

			if (bom == 0x1A2B3C4Du)
				swap = 0;
			else if (bom == 0x4D3C2B1Au)
				swap = 1;
			else
				return -EINVAL;
			nif = 0;
		} else {
			type = rd32(d + off, swap);
		}
		const uint32_t blen = rd32(d + off + 4, swap);

		if (blen < 12 || (blen & 3u) || blen > n - off)
			return -EINVAL;
		const uint8_t *b = d + off + 8;            /* block body */
		const uint32_t body = blen - 12;

		if (type == 1u) {                          /* interface description */
			if (body < 8)
				return -EINVAL;
			if (nif < 64)
				if_link[nif] = rd16(b, swap);
			nif++;
		} else if (type == 6u) {                   /* enhanced packet */
			if (body < 20)
				return -EINVAL;
			const uint32_t ifid = rd32(b, swap), cap = rd32(b + 12, swap);

			if (ifid >= nif || ifid >= 64 || if_link[ifid] != LINKTYPE_ETHERNET)
				return -EINVAL;
			if (cap > body - 20)
				return -EINVAL;
			if (recs_add(r, b + 20, cap))
				return -ENOMEM;
		} else if (type == 3u) {                   /* simple packet: interface 0 */
			if (body < 4 || nif == 0 || if_link[0] != LINKTYPE_ETHERNET)
				return -EINVAL;
			uint32_t plen = rd32(b, swap);

			if (plen > body - 4)
				plen = body - 4;           /* snapped to the block */
			if (recs_add(r, b + 4, plen))
				return -ENOMEM;
		}
		off += blen;
	}
	return 0;
}

int odpg_pcap_read(const char *path, uint32_t align, odpg_capture_t *cap)
{
	FILE *f;
	long sz;
	uint8_t *img = NULL;
	recs_t r = {NULL, NULL, 0, 0};
	int rc;

	if (!path || !cap || align == 0 || align > 4096 || (align & (align - 1)))
		return -EINVAL;
	memset(cap, 0, sizeof(*cap));
	f = fopen(path, "rb");
	if (!f)
		return -ENOENT;
	if (fseek(f, 0, SEEK_END) || (sz = ftell(f)) < 0 || fseek(f, 0, SEEK_SET)) {
		fclose(f);
		return -EINVAL;
	}
	img = malloc(sz > 0 ? (size_t)sz : 1);
	if (!img) {
		fclose(f);
		return -ENOMEM;
	}
	if (fread(img, 1, (size_t)sz, f) != (size_t)sz) {
		fclose(f);
		free(img);
		return -EINVAL;
	}
	fclose(f);
	if (sz < 4)
		rc = -EINVAL;
	else if (rd32(img, 0) == 0x0A0D0D0Au)
		rc = parse_pcapng(img, (size_t)sz, &r);
	else
		rc = parse_pcap(img, (size_t)sz, &r);
	if (rc == 0) {
		uint64_t total = 0;

		for (uint32_t i = 0; i < r.n; i++)
			total += ((uint64_t)r.len[i] + align - 1) & ~(uint64_t)(align - 1);
		cap->bytes = total + 128;
		cap->frames = calloc(1, (size_t)cap->bytes);
		cap->desc = calloc(r.n ? r.n : 1, sizeof(odpg_desc_t));
		if (!cap->frames || !cap->desc || total > 0xFFFFFFFFull) {
			odpg_pcap_free(cap);
			rc = total > 0xFFFFFFFFull ? -EINVAL : -ENOMEM;
		} else {
			uint64_t pos = 0;

			for (uint32_t i = 0; i < r.n; i++) {
				memcpy(cap->frames + pos, r.p[i], r.len[i]);
				cap->desc[i].offset = (uint32_t)pos;
				cap->desc[i].len = r.len[i];
				pos += ((uint64_t)r.len[i] + align - 1) & ~(uint64_t)(align - 1);
			}
			cap->num = r.n;
		}
	}
	free(r.p);
	free(r.len);
	free(img);
	return rc;
}

void odpg_pcap_free(odpg_capture_t *cap)
{
	if (!cap)
		return;
	free(cap->frames);
	free(cap->desc);
	memset(cap, 0, sizeof(*cap));
}
