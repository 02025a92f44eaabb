/* SPDX-License-Identifier: BSD-3-Clause
 *
 * odp_api.h — the ODP API subset this library serves: the classifier API
 * (odp_cls.h) and the runtime an ODP application needs around it to receive
 * classified packets (odp/rt.h: init, shared memory, packet pools, queues,
 * the scheduler, pcap / loop pktio, packet accessors, time, CPU masks,
 * threads). Enough for the reference's example/classifier source to build
 * unchanged against these headers and run on the GPU classifier
 * (tests/test_odp_rt.py). Names and argument meaning follow
 * the headers under include/odp/api/spec.
 */
#ifndef ODP_API_H_
#define ODP_API_H_

#include <inttypes.h>
#include <signal.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "odp_cls.h"
#include "odp/rt.h"

#endif
