"""Mask groups of the lean 64-byte kernel (cls_compile.cpp build_mgroup):
the compiled image's groups either hash every value of the group to its own
slot with one multiplier (m1 == m2, a single-probe lookup) or are two-choice
cuckoo tables; either way every value sits in one of its candidate slots
with its PMR bits. Host only (odpg_rules_compile)."""
import struct

import numpy as np

from odp_amd import gen, gpu

MG_SIZE, ENT_SIZE = 32, 16          # dmgroup_t, dment_t (odpg_internal.h)


def _groups(rules):
    img = gpu.compile_rules(rules)
    hdr_size = struct.unpack_from("<I", img, 8)[0]
    h = struct.unpack_from("<%dI" % (hdr_size // 4), img, 16)
    blob = 16 + hdr_size
    mg_off, n_mg, ment_off, n_ment = h[24], h[25], h[26], h[27]
    groups = [struct.unpack_from("<8I", img, blob + mg_off + MG_SIZE * g) for g in range(n_mg)]
    ents = [struct.unpack_from("<4I", img, blob + ment_off + ENT_SIZE * e) for e in range(n_ment)]
    return groups, ents


def _check(groups, ents):
    perfect = 0
    for slot, req, mask, shift, off, m1, m2, count in groups:
        if count == 1:
            continue                      # one value inline, no entries
        size = 1 << (32 - shift)
        table = ents[off:off + size]
        held = [e for e in table if e[1] or e[2]]
        assert len(held) == count
        for value, lo, hi, _ in held:
            cands = {((value * m) & 0xFFFFFFFF) >> shift for m in (m1, m2)}
            assert any(table[c][0] == value and (table[c][1], table[c][2]) == (lo, hi)
                       for c in cands)
        perfect += m1 == m2
    return perfect


def test_c2_groups_are_collision_free(fresh_cls):
    p = fresh_cls.loop_pktio()
    gen.build_c2_rules(fresh_cls, p)
    groups, ents = _groups(fresh_cls.pktio_rules(p))
    assert len(groups) == 2
    # the SIP /19 and the UDP_DPORT values separate on a bit field of the key
    assert _check(groups, ents) == 2
    for g in groups:
        assert g[5] & (g[5] - 1) == 0     # a power-of-two multiplier


def test_random_groups_keep_every_value(fresh_cls):
    """Values without structure: whichever form the compiler picks, every
    value is found in its candidate slots."""
    rng = np.random.default_rng(11)
    p = fresh_cls.loop_pktio()
    d = fresh_cls.cos_create("d", queue=fresh_cls.queue(0))
    assert fresh_cls.default_cos_set(p, d) == 0
    ports = rng.permutation(1 << 16)[:56]
    for a in range(7):                    # 1 + 7 + 56 CoS: the 64-CoS limit
        c = fresh_cls.cos_create(f"l1_{a}", queue=fresh_cls.queue(1 + a))
        v = int(rng.integers(0, 1 << 32))
        assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_DIP_ADDR, v.to_bytes(4, "big"),
                                                     b"\xff\xff\xff\xff")], d, c)
        for j in range(8):
            leaf = fresh_cls.cos_create(f"leaf_{a}_{j}", queue=fresh_cls.queue(8 + 8 * a + j))
            assert fresh_cls.pmr_create([fresh_cls.Term(fresh_cls.PMR_UDP_DPORT,
                                                         int(ports[8 * a + j]).to_bytes(2, "big"),
                                                         b"\xff\xff")], c, leaf)
    groups, ents = _groups(fresh_cls.pktio_rules(p))
    assert groups
    _check(groups, ents)
