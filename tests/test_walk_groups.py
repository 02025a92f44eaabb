"""CoS-keyed walk groups of a compiled table (cls_compile.cpp, the hybrid
hash walk of classify.hip): every entry sits within its group's recorded
`maxp` slots of its home slot, which is what lets the kernel probe exactly
`maxp` slots per group with no early exit; Robin Hood insertion keeps that
bound short. Read from the table image's header and blob (odpg_internal.h
layout: dtable_hdr_t, dhgroup_t, dwent_t)."""
import struct

import numpy as np

from helpers import ALL_CHKSUM
from odp_amd import gen, gpu

HDR_FIELDS = ("num_cos default_cos error_cos flags num_pmr num_terms cos_off pmr_off "
              "term_off slot_off simple_off run_off num_runs hgroup_off num_hgroups "
              "hent_off num_hent cinfo_off pinfo_off slot_mask wgroup_off num_wgroups "
              "went_off num_went").split()
EMPTY = 0xFFFFFFFF


def walk_hash(value, cos, lg):
    """odpg_internal.h walk_hash"""
    x = (value ^ ((cos * 0x85EBCA6B) & 0xFFFFFFFF)) & 0xFFFFFFFF
    return ((x * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - lg)


def walk_groups(img):
    hdr_bytes = struct.unpack_from("<4I", img, 0)[2]
    h = dict(zip(HDR_FIELDS, struct.unpack_from("<%di" % len(HDR_FIELDS), img, 16)))
    blob = img[16 + hdr_bytes:]
    groups = []
    for gi in range(h["num_wgroups"]):
        g = struct.unpack_from("<8I", blob, h["wgroup_off"] + 32 * gi)
        ents = np.frombuffer(blob, np.uint32, 2 * (1 << g[3]), h["went_off"] + 8 * g[4])
        groups.append({"log2sz": g[3], "count": g[5], "maxp": g[6],
                       "ents": ents.reshape(-1, 2)})
    return groups


def test_c3_walk_groups_maxp(fresh_cls):
    p = fresh_cls.loop_pktio(pktin=ALL_CHKSUM)
    gen.build_c3_rules(fresh_cls, p)
    assert fresh_cls.pktio_start(p) == 0
    groups = walk_groups(gpu.compile_rules(fresh_cls.pktio_rules(p)))
    assert len(groups) == 11
    for g in groups:
        lg, szm = g["log2sz"], (1 << g["log2sz"]) - 1
        used = [(i, int(v), int(cp)) for i, (v, cp) in enumerate(g["ents"]) if cp != EMPTY]
        assert len(used) == g["count"] and 2 * len(used) <= szm + 1
        disp = [((i - walk_hash(v, cp & 0xFFFF, lg)) & szm) + 1 for i, v, cp in used]
        assert max(disp) == g["maxp"]
        # the kernel's branch-free form covers every C3 group (XWALK_MAXP 4)
        assert 1 <= g["maxp"] <= 4
        # probe-until-empty still finds every key: no empty slot between an
        # entry and its home
        for i, v, cp in used:
            h = walk_hash(v, cp & 0xFFFF, lg)
            k = h
            while k != i:
                assert g["ents"][k][1] != EMPTY
                k = (k + 1) & szm
