/* SPDX-License-Identifier: BSD-3-Clause
 *
 * Private seam between the classifier object model (odp_cls.c) and the ODP
 * runtime subset (odp_rt.c), both inside libodpg.so.
 */
#ifndef ODP_RT_INTERNAL_H_
#define ODP_RT_INTERNAL_H_

#include "../../include/odp_cls.h"

/* odp_rt.c: a pktio was opened / is closing (its receive state) */
int  odpg_rt_pktio_open(odp_pktio_t pktio, const char *name, const odp_pktio_param_t *param);
void odpg_rt_pktio_close(odp_pktio_t pktio);

/* odp_cls.c: odpg_pktio_recv_batch's host path, also writing the parse
 * result of every packet (meta may be NULL) */
int odpg_cls_pktio_recv_meta(odp_pktio_t pktio, odpg_ctx_t *ctx, const uint8_t *frames,
			     const odpg_desc_t *desc, uint32_t num, odpg_out_t *out,
			     odpg_meta_t *meta);
/* the pktio is started with the classifier enabled */
int odpg_cls_pktio_classifies(odp_pktio_t pktio);

#endif
