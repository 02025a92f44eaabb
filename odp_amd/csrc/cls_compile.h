/* SPDX-License-Identifier: BSD-3-Clause */
#ifndef ODPG_CLS_COMPILE_H_
#define ODPG_CLS_COMPILE_H_

#include <stdint.h>
#include <vector>

#include "../../include/odpg.h"
#include "odpg_internal.h"

int odpg_compile_rules(const odpg_rules_t *r, std::vector<uint8_t> &blob, dtable_hdr_t *hdr);
int odpg_rules_has_cycle(const std::vector<uint8_t> &blob, const dtable_hdr_t &h);

#endif
